#!/bin/bash
# OOB-zero buffer loads in k_conv_dgrad / k_conv_x9 (no load under a branch, so no vmcnt(0)
# before each group): conv / learner tests, the kernels alone (old vs new library), then an
# interleaved in-loop A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -rf --timeout 120 --timeout-method thread \
  tests/test_conv_gpu.py tests/test_learner_gpu.py tests/test_fused_learner_gpu.py > gpurun_out/bufld_tests.log 2>&1
rc=$?; tail -3 gpurun_out/bufld_tests.log; [ $rc -eq 0 ] || exit $rc
for v in r03_head r03_bufld; do
  echo "== $v alone"
  RTH_LIB_PATH=$PWD/build_ab/$v.so timeout -k 10 200 python scripts/bench_dgrad.py 2>&1 | tail -4 || exit 1
  RTH_LIB_PATH=$PWD/build_ab/$v.so timeout -k 10 200 python scripts/bench_conv.py 2>&1 | tail -6 || exit 1
done
scripts/ab_bench.sh ${ROUNDS:-3} ${STEPS:-400} build_ab/r03_head.so build_ab/r03_bufld.so
