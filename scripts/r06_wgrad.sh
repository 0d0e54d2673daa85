#!/bin/bash
# r06: the register-only fp32 weight gradient: parity tests, then alone-timings over variants
# (GRID lines: conv2-variant conv2-splits conv3-variant conv3-splits; 0 splits = the variant's own)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -k wgrad -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/wgrad_tests.log 2>&1; rc=$?; tail -3 gpurun_out/wgrad_tests.log
[ $rc -ne 0 ] && exit $rc
while read -r v2 s2 v3 s3; do
  [ -z "$v2" ] && continue
  echo "== conv2 variant $v2 splits $s2 / conv3 variant $v3 splits $s3"
  RTH_WGF_V2=$v2 RTH_WGF_SPLITS2=$s2 RTH_WGF_V3=$v3 RTH_WGF_SPLITS3=$s3 WGF_ONLY=1 timeout -k 10 120 \
    python scripts/bench_wgrad_f32.py 2>&1 | grep rth_conv_wgrad_f32 || exit $?
done <<< "${GRID:-0 0 0 0}"
