#!/bin/bash
# the actor tail's heads rows in registers (k_actor_tail<8>) vs the pointer form
# (RTH_ACTOR_TAIL_REG=0): actor / apex tests, then an interleaved in-loop A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -rf --timeout 120 --timeout-method thread tests/test_actor_gpu.py \
  tests/test_apex_gpu.py tests/test_scale_gpu.py > gpurun_out/tail_tests.log 2>&1
rc=$?; tail -3 gpurun_out/tail_tests.log; [ $rc -eq 0 ] || exit $rc
RTH_ACTOR_TAIL_REG=0 timeout -k 10 600 python -u -m pytest -x -q -rf --timeout 120 --timeout-method thread \
  tests/test_actor_gpu.py > gpurun_out/tail_tests0.log 2>&1
rc=$?; tail -1 gpurun_out/tail_tests0.log; [ $rc -eq 0 ] || exit $rc
scripts/ab_env.sh ${ROUNDS:-4} ${STEPS:-500} "reg RTH_ACTOR_TAIL_REG=1" "ptr RTH_ACTOR_TAIL_REG=0"
