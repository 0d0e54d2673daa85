#!/bin/bash
# range-checked buffer loads in k_grad_sqsum / k_adam, 16 loads in flight in k_wgrad_reduce:
# optimizer / conv / learner tests, then an in-loop A/B against the previous commit
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -rf --timeout 120 --timeout-method thread tests/test_optim_gpu.py \
  tests/test_conv_gpu.py tests/test_learner_gpu.py tests/test_fused_learner_gpu.py tests/test_learner_full_gpu.py \
  > gpurun_out/optld_tests.log 2>&1
rc=$?; tail -3 gpurun_out/optld_tests.log; [ $rc -eq 0 ] || exit $rc
scripts/ab_bench.sh ${ROUNDS:-4} ${STEPS:-500} build_ab/r03_head.so build_ab/r03_optld.so
