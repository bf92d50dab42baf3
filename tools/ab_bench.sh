# same-box A/B of a bench.py environment toggle: AB_ENV="VAR=a+VAR=b",
# interleaved, AB_REPS times, each a short bench (no CPU leg)
set -e
out=gpurun_out/${AB_NAME:-ab}/bench_ab.txt
IFS='+' read -ra envs <<< "${AB_ENV}"
for rep in $(seq "${AB_REPS:-3}"); do
  for e in "${envs[@]}"; do
    echo "$e" >> "$out"
    env "$e" timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 \
      --no-cpu-baseline ${AB_ARGS} 2>/dev/null | grep '^{' >> "$out"
  done
done
