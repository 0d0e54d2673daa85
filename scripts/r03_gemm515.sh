#!/bin/bash
# hipBLASLt solution 627515 for the 512-row FC1 forward (actor + target pass) against the
# committed 627513: determinism / fp64 error (gemm_probe.py), then an interleaved in-loop A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/screen
src=reth_amd/tuned/tunableop_results_mi355x.csv
csv=$PWD/gpurun_out/screen/tun_515.csv
sed "s/tn_512_512_3136_ld_3136_3136_512,Gemm_Hipblaslt_627513,/tn_512_512_3136_ld_3136_3136_512,Gemm_Hipblaslt_627515,/" $src > $csv
RTH_TUNABLEOP_IN=$csv timeout -k 10 300 python scripts/gemm_probe.py 2>&1 | grep -v amdgpu | tail -6 || exit 1
scripts/ab_env.sh ${ROUNDS:-4} ${STEPS:-500} "s513 RTH_X=0" "s515 RTH_TUNABLEOP_IN=$csv"
