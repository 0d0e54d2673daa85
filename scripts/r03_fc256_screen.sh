#!/bin/bash
# In-loop screen of the actors' 256-row FC1 GEMM (the counted dedup forward): a few hipBLASLt
# solutions for tn_512_256_3136 appended to the committed TunableOp file, against the 2N-row
# GEMM (RTH_ACTOR_COUNTED_FC=0), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/screen
src=reth_amd/tuned/tunableop_results_mi355x.csv
specs=("base RTH_ACTOR_COUNTED_FC=0" "dflt RTH_ACTOR_COUNTED_FC=1")
for sol in ${SOLS:-627513 627486 627408}; do
  csv=$PWD/gpurun_out/screen/tun256_$sol.csv
  grep -v "tn_512_256_3136" "$src" > "$csv"
  echo "GemmAndBiasTunableOp_float_TN,tn_512_256_3136_ld_3136_3136_512,Gemm_Hipblaslt_$sol,0.02" >> "$csv"
  specs+=("s$sol RTH_TUNABLEOP_IN=$csv")
done
scripts/ab_env.sh ${ROUNDS:-2} ${STEPS:-300} "${specs[@]}"
