# same-box A/B of C5 (tools/bench_configs.py --only c5) under an environment
# toggle: AB_ENV="VAR=a+VAR=b", interleaved, AB_REPS times
set -e
out=gpurun_out/${AB_NAME:-ab}/c5_ab.txt
IFS='+' read -ra envs <<< "${AB_ENV}"
for rep in $(seq "${AB_REPS:-2}"); do
  for e in "${envs[@]}"; do
    echo "$e" >> "$out"
    env "$e" timeout -k 10 300 python3 -u tools/bench_configs.py --only c5 \
      2>/dev/null | grep '^{' >> "$out"
  done
done
