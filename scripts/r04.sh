#!/bin/bash
# round-4 GPU steps (each under its own limit; stop on a crash / timeout):
#   transient = per-step GPU times of the driver's command shape (--steps 20 --warmup 5)
#               with / without the in-window timers and the conv probe, and after a long warmup
#   tests     = the GPU test suite;  smoke = __graft_entry__.smoke()
#   bench     = the driver's command
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 limit=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 4 "gpurun_out/$name.log" | cut -c1-600
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
for s in "$@"; do
  case "$s" in
    transient)
      RTH_BENCH_STEPTIMES=1 step tr_default 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
      RTH_BENCH_STEPTIMES=1 RTH_BENCH_NOTIMER=1 step tr_notimer 300 python bench.py --steps 20 --warmup 5 \
          --no-cpu-baseline --no-sweep --no-probe
      RTH_BENCH_STEPTIMES=1 step tr_longwarm 300 python bench.py --steps 20 --warmup 300 --no-cpu-baseline --no-sweep
      RTH_BENCH_STEPTIMES=1 RTH_BENCH_NOTIMER=1 step tr_longwarm_notimer 300 python bench.py --steps 20 --warmup 300 \
          --no-cpu-baseline --no-sweep --no-probe ;;
    transient2)
      RTH_BENCH_STEPTIMES=1 RTH_BENCH_NOTIMER=1 step tr2_short 300 python bench.py --steps 40 --warmup 5 \
          --no-cpu-baseline --no-sweep --no-probe
      RTH_BENCH_STEPTIMES=1 RTH_BENCH_NOTIMER=1 step tr2_long 300 python bench.py --steps 40 --warmup 300 \
          --no-cpu-baseline --no-sweep --no-probe ;;
    learnerfull) step learner_full 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
          tests/test_learner_full_gpu.py ;;
    newtests) step new_tests 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
          tests/test_apex_gpu.py tests/test_learner_full_gpu.py tests/test_zmtp_gpu.py tests/test_dropin_gpu.py ;;
    benchdiag) RTH_BENCH_STEPTIMES=1 step bench_diag 600 python bench.py --steps 40 --warmup 5 --no-cpu-baseline ;;
    first)
      RTH_BENCH_STEPTIMES=1 RTH_BENCH_PROFILE0=1 step first_prof 300 python bench.py --steps 20 --warmup 5 \
          --no-cpu-baseline --no-sweep --probe-steps 0
      RTH_BENCH_STEPTIMES=1 RTH_BENCH_SETTLE_SYNC=16 step first_sync16 300 python bench.py --steps 20 --warmup 5 \
          --no-cpu-baseline --no-sweep --probe-steps 0
      RTH_BENCH_STEPTIMES=1 step first_nosettle 300 python bench.py --steps 20 --warmup 5 --settle 0 \
          --no-cpu-baseline --no-sweep --probe-steps 0
      RTH_BENCH_STEPTIMES=1 step first_plain 300 python bench.py --steps 20 --warmup 5 \
          --no-cpu-baseline --no-sweep --probe-steps 0 ;;
    dp8) RTH_SHARE_GPU=1 RTH_DIST_BACKEND=gloo step dp8_gloo_rehearsal 900 python -m torch.distributed.run --nnodes=1 \
          --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 8 --faithful --steps 20 \
          --warmup 5 --no-cpu-baseline --no-sweep ;;
    tests) step gpu_tests 1100 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
  esac
done
