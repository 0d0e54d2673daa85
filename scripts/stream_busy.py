"""Per-stream kernel time of the profiled bench window (rocprofv3 kernel trace): which
stream is the critical path and what it runs."""
import collections
import csv
import sys

f = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_trace.csv"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 100
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-int(len(rows) * 0.3):]
t0 = int(rows[0]["Start_Timestamp"])
t1 = max(int(r["End_Timestamp"]) for r in rows)
span = (t1 - t0) / 1000
busy, names = collections.Counter(), collections.defaultdict(collections.Counter)
for r in rows:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    busy[r["Stream_Id"]] += d
    names[r["Stream_Id"]][r["Kernel_Name"][:70]] += d
n_it = iters * 0.3 * (span / span)  # window = last 30% of rows ~ 30% of iterations
per = span / (busy.total() and 1) if False else None
print(f"window {span:.0f} us")
for s, b in busy.most_common():
    print(f"stream {s}: busy {b:.0f} us = {b / span:.1%} of the window")
    for k, v in names[s].most_common(14):
        print(f"   {v / span * 100:6.2f}%  {k}")
