#!/bin/bash
# r06: kernel times + SQ counters of the fp32 weight gradient alone (scripts/bench_wgrad_f32.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/wgrad_prof" -o run -- \
  python scripts/bench_wgrad_f32.py > gpurun_out/wgrad_prof.log 2>&1 || exit $?
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$PWD/gpurun_out/wgrad_pmc_$name" \
      -o run -- python scripts/bench_wgrad_f32.py > "gpurun_out/wgrad_pmc_$name.log" 2>&1
  local rc=$?; echo "pmc $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
pass sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT
pass inst GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_LDS_IDX_ACTIVE
pass fetch FETCH_SIZE
