#!/bin/bash
# k_heads_fc2_lean (no LDS, <= 64 VGPRs: fits beside the x9 convs) vs k_heads_fc2: the FC2
# tests under both, then an interleaved in-loop A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in 1 0; do
  RTH_FC2_LEAN=$v timeout -k 10 600 python -u -m pytest -x -q -rf --timeout 120 --timeout-method thread \
    tests/test_fused_learner_gpu.py tests/test_actor_gpu.py tests/test_learner_full_gpu.py > gpurun_out/lean_tests$v.log 2>&1
  rc=$?; tail -1 gpurun_out/lean_tests$v.log; [ $rc -eq 0 ] || exit $rc
done
scripts/ab_env.sh ${ROUNDS:-4} ${STEPS:-500} "lean RTH_FC2_LEAN=1" "lds RTH_FC2_LEAN=0"
