#!/bin/bash
# One parametrised runner for every GPU call (run ON the GPU box):
#
#   /usr/local/graft/bin/gpurun --timeout 1200 -- \
#       'bash tools/gpu_job.sh NAME STEP [STEP ...]'
#
# Output goes to gpurun_out/NAME/<k>_<step>.txt.  Every step runs under its
# own time limit; the steps are chained, so the first failure (test failure,
# GPU fault, abort, time limit) ends the call there.  Steps:
#
#   suite                 the whole -m gpu suite (+ the parity json files)
#   tests=EXPR[@FILES]    pytest -m gpu -k EXPR [FILES, comma-separated]
#   smoke                 __graft_entry__.smoke()
#   bench[=ARGS]          bench.py (default --steps 20 --warmup 5)
#   rankslice             bench.py --rank-slice R for R = 1, 2, 4, 8
#   profile=TAG           rocprofv3 kernel stats + PMC passes of the bench
#                         (one counter group per pass) -> prof_TAG/
#   kernels               tools/bench_kernels.py (per-kernel roofline table)
#   configs               tools/bench_configs.py (BASELINE configs end to end)
#   py=SECS:SCRIPT ARGS   python3 -u SCRIPT ARGS under a SECS limit
#   bin=SECS:PROGRAM ARGS  a compiled probe under a SECS limit
#   stats=SECS:SCRIPT ARGS
#                         rocprofv3 kernel trace + stats over python3 SCRIPT
#   pmc=SECS:COUNTERS:SCRIPT ARGS
#                         one rocprofv3 --pmc pass (counters comma-separated)
#                         over python3 SCRIPT ARGS
set -e -o pipefail
NAME=$1
shift
OUT=gpurun_out/$NAME
mkdir -p "$OUT"
export TMPDIR=/tmp
k=0
run() {  # run SECS LOGNAME cmd...
  local secs=$1 log=$2
  shift 2
  echo "[$(date +%T)] $log: $*"
  timeout -k 10 "$secs" "$@" > "$OUT/$log.txt" 2>&1
}
for step in "$@"; do
  k=$((k + 1))
  key=${step%%=*}
  arg=${step#*=}
  if [ "$arg" = "$step" ]; then arg=""; fi
  case $key in
    suite)
      run 1000 "${k}_suite" python -u -m pytest tests -m gpu -x -v -s \
        --timeout 300 --timeout-method thread
      for f in kde_fullsize_parity.json quantile_parity.json; do
        if [ -f gpurun_out/$f ]; then cp gpurun_out/$f "$OUT/"; fi
      done ;;
    tests)
      expr=${arg%%@*}
      files=tests
      if [ "$arg" != "$expr" ]; then files=$(echo "${arg#*@}" | tr , ' '); fi
      # shellcheck disable=SC2086
      run 900 "${k}_tests" python -u -m pytest $files -m gpu -x -v -s \
        -k "$expr" --timeout 300 --timeout-method thread ;;
    smoke)
      run 150 "${k}_smoke" python3 -c \
        "import __graft_entry__ as g; g.smoke()" ;;
    bench)
      # shellcheck disable=SC2086
      run 400 "${k}_bench" python3 -u bench.py ${arg:---steps 20 --warmup 5} ;;
    rankslice)
      for R in 1 2 4 8; do
        run 300 "${k}_rankslice_$R" python3 -u bench.py --rank-slice $R \
          --steps 10 --warmup 3 --no-cpu-baseline
      done ;;
    profile)
      P=$OUT/prof_${arg:-r04}
      B="bench.py --steps 2 --warmup 1 --no-cpu-baseline"
      mkdir -p "$P"
      # shellcheck disable=SC2086
      run 300 "${k}_stats" rocprofv3 --kernel-trace --stats -T -f csv \
        -d "$P/stats" -o run -- python3 $B
      for tg in "fetch:FETCH_SIZE" "write:WRITE_SIZE" \
          "pmcA:SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_TRANS_F32 SQ_WAVES GRBM_GUI_ACTIVE" \
          "pmcB:SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
          "pmcC:SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
        tag=${tg%%:*}
        grp=${tg#*:}
        echo "[$(date +%T)] pmc $grp"
        # shellcheck disable=SC2086
        timeout -s KILL 150 rocprofv3 --pmc $grp -T -f csv -d "$P/$tag" \
          -o run -- python3 $B > "$OUT/${k}_pmc_$tag.txt" 2>&1
      done ;;
    kernels)
      run 400 "${k}_kernels" python3 -u tools/bench_kernels.py ;;
    configs)
      run 500 "${k}_configs" python3 -u tools/bench_configs.py ;;
    py)
      secs=${arg%%:*}
      # shellcheck disable=SC2086
      run "$secs" "${k}_py" python3 -u ${arg#*:} ;;
    bin)
      secs=${arg%%:*}
      # shellcheck disable=SC2086
      run "$secs" "${k}_bin" ${arg#*:} ;;
    stats)
      secs=${arg%%:*}
      # shellcheck disable=SC2086
      run "$secs" "${k}_stats" rocprofv3 --kernel-trace --stats -T -f csv \
        -d "$OUT/stats_$k" -o run -- python3 -u ${arg#*:} ;;
    pmc)
      secs=${arg%%:*}
      rest=${arg#*:}
      ctr=$(echo "${rest%%:*}" | tr , ' ')
      echo "[$(date +%T)] pmc $ctr: ${rest#*:}"
      # shellcheck disable=SC2086
      timeout -s KILL "$secs" rocprofv3 --pmc $ctr -T -f csv \
        -d "$OUT/pmc_$k" -o run -- python3 ${rest#*:} > "$OUT/${k}_pmc.txt" 2>&1 ;;
    *)
      echo "unknown step: $step" >&2
      exit 2 ;;
  esac
done
echo "[$(date +%T)] $NAME done"
