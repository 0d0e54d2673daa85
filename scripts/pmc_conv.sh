#!/bin/bash
# SQ / cache counter passes over scripts/conv_pmc.py (one rocprofv3 run per pass, each
# under its own time limit; stop at the first failure).  Output: gpurun_out/pmc_conv_<pass>/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
pass() {
  local name=$1; shift
  echo "== pmc $name ($(date +%T))"
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$PWD/gpurun_out/pmc_conv_$name" \
      -o run -- python scripts/conv_pmc.py > "gpurun_out/pmc_conv_$name.log" 2>&1
  local rc=$?
  echo "pmc $name rc=$rc"; tail -n 3 "gpurun_out/pmc_conv_$name.log"
  [ $rc -eq 0 ] || exit $rc
}
pass sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES \
    SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT
pass inst GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_LDS_IDX_ACTIVE
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass l2 TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
