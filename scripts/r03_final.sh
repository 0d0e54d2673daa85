#!/bin/bash
# round-3 evidence runs (each step under its own limit, stop on a crash):
#   1 = default bench (the driver's command) + learner span + Breakout bench
#   2 = rocprofv3 stats/trace + FETCH/WRITE passes + conv counter passes
#   3 = Atari env-mode bench lines + the whole GPU test suite
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 limit=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 3 "gpurun_out/$name.log" | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
for s in "$@"; do
  case "$s" in
    1) step bench_final 600 python bench.py
       RTH_BENCH_SPAN=1 step span 300 python bench.py --steps 300 --warmup 20 --no-cpu-baseline --no-sweep
       step bench_breakout 600 python bench.py --workload breakout --steps 100 --warmup 10 --no-cpu-baseline --no-sweep ;;
    2) step rocprof_stats 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof" -o run \
          -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-sweep
       step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv --kernel-include-regex "rth::" \
          -d "$PWD/gpurun_out/pmc_fetch" -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sweep
       step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv --kernel-include-regex "rth::" \
          -d "$PWD/gpurun_out/pmc_write" -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sweep
       bash scripts/pmc_conv.sh ;;
    3) step bench_atari 600 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-sweep --env atari
       step bench_atari_h2d 600 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-sweep --env atari-h2d
       step gpu_tests 1100 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests ;;
  esac
done
