#!/bin/bash
# unconditional loads in the heads kernels (k_heads_fc2 staging, k_heads_backward /
# k_td_heads_backward rows, the TD rows in registers): learner tests, then an in-loop A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -rf --timeout 120 --timeout-method thread \
  tests/test_learner_gpu.py tests/test_fused_learner_gpu.py tests/test_actor_gpu.py tests/test_apex_gpu.py > gpurun_out/qnetld_tests.log 2>&1
rc=$?; tail -3 gpurun_out/qnetld_tests.log; [ $rc -eq 0 ] || exit $rc
scripts/ab_bench.sh ${ROUNDS:-3} ${STEPS:-400} build_ab/r03_head.so build_ab/r03_qnetld.so
