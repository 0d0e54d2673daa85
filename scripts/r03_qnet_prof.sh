#!/bin/bash
# per-kernel times of two library variants in the loop (rocprofv3 kernel trace + stats)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "$@"; do
  RTH_LIB_PATH=$PWD/build_ab/$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$PWD/gpurun_out/prof_$v" -o run -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline \
    > gpurun_out/prof_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/prof_$v.log; exit 1; }
  f=$(find gpurun_out/prof_$v -name "*kernel_stats.csv" | head -1)
  echo "== $v"; python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    n = r["Name"]
    if any(k in n for k in ("heads", "td_", "conv_dgrad", "k_conv_x9", "k_copy_rows", "k_actor_tail")):
        print(f"{float(r['AverageNs'])/1000:8.2f} us x {r['Calls']:>5}  {n[:90]}")
PY
done
