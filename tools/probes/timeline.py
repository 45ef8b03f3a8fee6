"""Print N dispatches from the middle of a rocprofv3 kernel trace (start/end relative to the first
shown, duration, grid) -- python3 tools/timeline.py gpurun_out/prof_TAG [N]."""
import csv
import glob
import os
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
path = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
rows = rows[len(rows) // 2:len(rows) // 2 + n]  # (the bench's timed region: no timing events)
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("%8.1f %8.1f %7.1f  grid=%-7s %s" % ((s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3,
                                             r["Grid_Size_X"], r["Kernel_Name"].split("(")[0][:50]))
