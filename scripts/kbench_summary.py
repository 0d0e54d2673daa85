"""Median durations of the library's kernels in rocprof runs of bench.py (development aid)."""
import collections
import csv
import glob
import statistics
import sys

for d in sorted(glob.glob(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/kbench_*")):
    f = glob.glob(d + "/run_kernel_trace.csv")
    if not f:
        continue
    rows = list(csv.DictReader(open(f[0])))[-8000:]
    v = collections.defaultdict(list)
    for r in rows:
        n = r["Kernel_Name"]
        if n.startswith("rth::"):
            v[(n.split("(")[0][5:], r["Grid_Size_X"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
    print(d.split("/")[-1], {f"{k[0]}/{k[1]}": round(statistics.median(x), 1) for k, x in sorted(v.items())})
