#!/bin/bash
# r06: selected GPU test files (TESTS), then optional in-loop A/B arms (ARMS, see r06_ab.sh)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/check_tests.log 2>&1; rc=$?; tail -5 gpurun_out/check_tests.log
[ $rc -ne 0 ] && exit $rc
[ -n "${ARMS:-}" ] && exec_ab=1 && bash scripts/r06_ab.sh
exit 0
