#!/bin/bash
# Development aid: screen hipBLASLt solutions for one FC1 GEMM shape inside the Ape-X loop
# (the isolated TunableOp winner is not the fastest beside the learner stream).  One bench
# run per candidate, each with its own time limit; one line per run.
# usage: scripts/gemm_screen.sh KEY DEFAULT_SOLUTION FIRST LAST [STEPS]
#   KEY e.g. tn_512_512_3136_ld_3136_3136_512; solutions FIRST..LAST (Gemm_Hipblaslt_<id>)
# or:    SCREEN_LIST="Gemm_Rocblas_-624952332 ..." scripts/gemm_screen.sh KEY DEFAULT_NAME [STEPS]
#   (DEFAULT_NAME: the full solution name in the committed file)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/screen
src=reth_amd/tuned/tunableop_results_mi355x.csv
key=$1
if [ -n "${SCREEN_LIST:-}" ]; then
  dflt=$2 steps=${3:-200}; list=$SCREEN_LIST
else
  dflt=Gemm_Hipblaslt_$2 steps=${5:-200}; list=$(seq -f "Gemm_Hipblaslt_%.0f" "$3" "$4")
fi
for sol in $list; do
  id=${sol#Gemm_}
  csv=gpurun_out/screen/tun_$id.csv
  sed "s/$key,$dflt,/$key,$sol,/" "$src" > "$csv"
  RTH_TUNABLEOP_IN=$PWD/$csv timeout -k 10 120 python bench.py --steps "$steps" --warmup 20 --no-cpu-baseline ${BENCH_ARGS:-} \
    > "gpurun_out/screen/b_$id.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "$id rc=$rc (stopping)"; tail -3 "gpurun_out/screen/b_$id.log"; exit $rc; fi
  python - "$id" "gpurun_out/screen/b_$id.log" <<'PY'
import json, sys
lines = [l for l in open(sys.argv[2]) if l.startswith("{")]
if not lines:
    print(f"{sys.argv[1]}: no result", flush=True)
else:
    d = json.loads(lines[-1])
    print(f"{sys.argv[1]}: {d['ms_per_step']:.4f} ms/step", flush=True)
PY
done
