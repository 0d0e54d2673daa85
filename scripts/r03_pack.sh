#!/bin/bash
# weight packing with every load before the bf16 split (k_conv_pack_many): conv / learner
# tests, then an in-loop A/B against the previous commit
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -rf --timeout 120 --timeout-method thread tests/test_conv_gpu.py \
  tests/test_fused_learner_gpu.py tests/test_learner_full_gpu.py tests/test_actor_gpu.py > gpurun_out/pack_tests.log 2>&1
rc=$?; tail -3 gpurun_out/pack_tests.log; [ $rc -eq 0 ] || exit $rc
scripts/ab_bench.sh ${ROUNDS:-4} ${STEPS:-500} build_ab/r03_head.so build_ab/r03_pack.so
