#!/bin/bash
# round-3 GPU check: focused tests, a short bench, conv PMC passes (each step under its own limit)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
(timeout -k 10 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true)
step() {
  local name=$1 limit=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
for s in "$@"; do
  case "$s" in
    t) step tests 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread ${TESTS:-tests/test_learner_full_gpu.py tests/test_fused_learner_gpu.py tests/test_apex_gpu.py tests/test_weights_gpu.py tests/test_replay_gpu.py tests/test_dp_gpu.py} ;;
    b) step bench 600 python bench.py --steps 50 --warmup 10 --cpu-iters 5 ${BENCH_ARGS:-} ;;
    p) bash scripts/pmc_conv.sh ;;
    # evidence: rocprofv3 kernel trace + stats of the bench, then FETCH_SIZE / WRITE_SIZE passes
    # (scripts/summarize_profile.py TAG --steps 200 reads them)
    e) export TMPDIR=/tmp
       step rocprof_stats 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof" -o run \
          -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-sweep
       step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv --kernel-include-regex "rth::" \
          -d "$PWD/gpurun_out/pmc_fetch" -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sweep
       step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv --kernel-include-regex "rth::" \
          -d "$PWD/gpurun_out/pmc_write" -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sweep ;;
    c) step conv_tests 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_conv_gpu.py tests/test_fused_learner_gpu.py
       RTH_CONV2_X9_MAX=512 RTH_CONV3_X9_MIN=600 step conv_tests_hybrid 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_gpu.py
       CONV_NS=1024,512,256 step bench_conv_x9 300 python scripts/bench_conv.py
       RTH_CONV_F32MFMA=1 CONV_NS=1024,512,256 step bench_conv_f32 300 python scripts/bench_conv.py ;;
    q) step bench_quick 600 python bench.py --steps 100 --warmup 20 --no-cpu-baseline ${BENCH_ARGS:-}
       RTH_CONV_F32MFMA=1 step bench_quick_f32 600 python bench.py --steps 100 --warmup 20 --no-cpu-baseline ${BENCH_ARGS:-} ;;
    a) step bench_atari 600 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-sweep --env atari
       step bench_atari_h2d 600 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-sweep --env atari-h2d ;;
  esac
done
