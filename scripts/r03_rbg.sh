#!/bin/bash
# ReLU-mask + bias-partials kernels with their loads batched (k_relu_bias_grad_nchw: a sample's
# loads all in flight; k_relu_bias_grad: 4 rows per round trip): learner / conv tests, then an
# in-loop A/B against the previous commit
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -rf --timeout 120 --timeout-method thread tests/test_conv_gpu.py \
  tests/test_fused_learner_gpu.py tests/test_learner_full_gpu.py tests/test_learner_gpu.py > gpurun_out/rbg_tests.log 2>&1
rc=$?; tail -3 gpurun_out/rbg_tests.log; [ $rc -eq 0 ] || exit $rc
scripts/r03_abx.sh ${ROUNDS:-4} ${STEPS:-500} build_ab/r03_head.so build_ab/r03_rbg.so
