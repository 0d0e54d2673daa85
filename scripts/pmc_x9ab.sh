#!/bin/bash
# SQ counters of the x9 kernels (scripts/x9_ab.py) for the default library and a variant
# (RTH_LIB_PATH=$1); per-kernel medians printed by scripts/summarize_conv_pmc.py-style inline code
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for lib in default "$1"; do
  tag=$(basename "$lib" .so)
  if [ "$lib" = default ]; then unset RTH_LIB_PATH; else export RTH_LIB_PATH=$lib; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS \
      SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace --output-format csv \
      -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_x9_$tag" -o run -- python "$GRAFT_REPO_ROOT/scripts/x9_ab.py" /tmp/x9_pmc.pt \
      > "$GRAFT_REPO_ROOT/gpurun_out/pmc_x9_$tag.log" 2>&1 || { echo "pmc $tag failed"; exit 1; }
  python - "$GRAFT_REPO_ROOT/gpurun_out/pmc_x9_$tag/run_counter_collection.csv" "$tag" <<'PY'
import collections, csv, statistics as st, sys
v = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")
    if "k_conv_x9" not in k:
        continue
    k = k[:70] + " grid=" + r["Grid_Size"]
    v[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in sorted(v.items()):
    m = {n: st.median(x) for n, x in c.items()}
    conf = m.get("SQ_LDS_BANK_CONFLICT", 0) / max(m.get("SQ_LDS_IDX_ACTIVE", 1), 1)
    print(sys.argv[2], k, f"lds_conflict {conf:.3f}", f"valu/mfma {m.get('SQ_INSTS_VALU',0)/max(m.get('SQ_INSTS_MFMA',1),1):.2f}",
          f"wait_lds/wave_cyc {m.get('SQ_WAIT_INST_LDS',0)/max(m.get('SQ_WAVE_CYCLES',1),1):.3f}",
          {n: int(x) for n, x in m.items()})
PY
done
