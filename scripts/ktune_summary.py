"""Median kernel durations per capacity phase from the ktune rocprof runs (development aid)."""
import csv
import glob
import statistics
import sys

for d in sorted(glob.glob(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ktune_*")):
    f = glob.glob(d + "/run_kernel_trace.csv")
    if not f:
        continue
    rows = list(csv.DictReader(open(f[0])))
    out = {}
    for name in ("k_tree_find", "k_tree_sample", "k_tree_update"):
        v = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in rows if name in r["Kernel_Name"]]
        if name == "k_tree_find":  # alternating find512 / find1 per phase
            ph = [v[i:i + 110] for i in range(0, len(v), 110)]
            out["find512"] = [round(statistics.median(p[0::2][:55]), 1) for p in ph]
            out["find1"] = [round(statistics.median(p[1::2][:55]), 1) for p in ph]
        else:
            out[name] = [round(statistics.median(v[i:i + 55]), 1) for i in range(0, len(v), 55)]
    print(d.split("/")[-1], out)
