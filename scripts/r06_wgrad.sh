#!/bin/bash
# r06: the fp32 weight gradient's parity tests, then its alone timing against rth_conv_wgrad_x9 and
# MIOpen (scripts/bench_wgrad_f32.py).  (The split / variant grid of profiles/r06/wgrad_ab.txt ran
# through tuning switches that were removed once the forms were picked.)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -k wgrad -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/wgrad_tests.log 2>&1; rc=$?; tail -3 gpurun_out/wgrad_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python scripts/bench_wgrad_f32.py 2>&1 | grep -v amdgpu.ids
