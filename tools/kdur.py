"""Per-launch durations (µs) of the named kernels in a rocprofv3 kernel trace.

    python tools/kdur.py <kernel_trace.csv> k_complex k_bfs ...
"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
for k in sys.argv[2:]:
    v = [round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000, 1)
         for r in rows if r["Kernel_Name"].replace("kmcd::", "").startswith(k + "(")]
    print(k, v)
