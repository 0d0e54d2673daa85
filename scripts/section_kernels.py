"""Per-section kernel breakdown of a rocprofv3 kernel trace of scripts/host_probe.py: the
'alone' sections (each block replayed 20 times by itself) are separated by >20 ms gaps.

    python scripts/section_kernels.py gpurun_out/hp/run_kernel_trace.csv
"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
secs, cur, last = [], [], None
for r in rows:
    s = int(r["Start_Timestamp"])
    if last is not None and s - last > 20e6:
        secs.append(cur)
        cur = []
    cur.append(r)
    last = int(r["End_Timestamp"])
secs.append(cur)
names = ["learner pre", "learner full", "actor graph (dedup)", "actor graph (full)", "target pass", "sample+gather"]
for name, sec in zip(names, secs[-len(names):]):
    agg = collections.defaultdict(lambda: [0, 0])
    for r in sec:
        a = agg[r["Kernel_Name"][:90]]
        a[0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        a[1] += 1
    reps = 20
    tot = sum(v[0] for v in agg.values()) / 1e3 / reps
    span = (int(sec[-1]["End_Timestamp"]) - int(sec[0]["Start_Timestamp"])) / 1e3 / reps
    print(f"== {name}: kernel sum {tot:.1f} us per rep, span {span:.1f} us per rep, {len(sec) / reps:.1f} kernels")
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1][0]):
        print(f"   {v[0] / 1e3 / reps:8.1f} us  x{v[1] / reps:4.1f}  {k}")
