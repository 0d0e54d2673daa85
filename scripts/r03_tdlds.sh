#!/bin/bash
# k_td_heads_backward with B * (A + 1) floats of dynamic LDS instead of a 64 KB static array
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -rf --timeout 120 --timeout-method thread tests/test_fused_learner_gpu.py \
  tests/test_learner_full_gpu.py tests/test_learner_gpu.py > gpurun_out/tdlds_tests.log 2>&1
rc=$?; tail -1 gpurun_out/tdlds_tests.log; [ $rc -eq 0 ] || exit $rc
scripts/ab_bench.sh ${ROUNDS:-4} ${STEPS:-500} build_ab/r03_head.so build_ab/r03_tdlds.so
