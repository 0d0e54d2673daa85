#!/bin/bash
# the actors' second layer over the counted rows with the heads-cache scatter in its launch,
# against the separate scatter (RTH_ACTOR_FC2_CACHE=0); tests first
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -rf --timeout 120 --timeout-method thread \
  tests/test_fused_learner_gpu.py tests/test_actor_gpu.py tests/test_apex_gpu.py > gpurun_out/fc2c_tests.log 2>&1
rc=$?; tail -3 gpurun_out/fc2c_tests.log; [ $rc -eq 0 ] || exit $rc
scripts/ab_env.sh ${ROUNDS:-4} ${STEPS:-400} "fused RTH_ACTOR_FC2_CACHE=1" "separate RTH_ACTOR_FC2_CACHE=0"
