#!/bin/bash
# GPU check of the device-counted actor heads (rth_linear_relu_rows_upto / rth_heads_fc2_upto):
# the new kernel tests and the actor / apex tests, then an interleaved A/B of the bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -rf --timeout 120 --timeout-method thread \
  tests/test_fused_learner_gpu.py tests/test_actor_gpu.py tests/test_apex_gpu.py > gpurun_out/cfc_tests.log 2>&1
rc=$?; tail -5 gpurun_out/cfc_tests.log; [ $rc -eq 0 ] || exit $rc
scripts/ab_env.sh ${ROUNDS:-3} ${STEPS:-300} "counted RTH_ACTOR_COUNTED_FC=1" "gemm2N RTH_ACTOR_COUNTED_FC=0"
