#!/bin/bash
# interleaved in-loop A/B of library variants with the live per-kernel times the bench reports
# usage: scripts/r03_abx.sh ROUNDS STEPS a.so b.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rounds=$1 steps=$2; shift 2
for r in $(seq 1 "$rounds"); do
  for v in "$@"; do
    b=$(basename "$v" .so)
    RTH_LIB_PATH=$PWD/$v timeout -k 10 300 python bench.py --steps "$steps" --warmup 30 --no-cpu-baseline --no-sweep \
      > "gpurun_out/abx_${b}_$r.log" 2>&1 || { echo "$b failed"; tail -5 "gpurun_out/abx_${b}_$r.log"; exit 1; }
    python - "$b" "$r" "gpurun_out/abx_${b}_$r.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[3]) if l.startswith("{")][-1])
g, c3, c2 = d["roofline_gather"], d["roofline_conv3"], d["roofline_conv2"]
print(f"{sys.argv[1]:>12} r{sys.argv[2]}: {d['ms_per_step']:.4f} ms  gather loop {g['mean_launch_us']:.1f} alone {g['isolated_launch_us']:.1f} us"
      f"  conv3 {c3['mean_launch_us']:.1f}  conv2 {c2['mean_launch_us']:.1f} us", flush=True)
PY
  done
done
