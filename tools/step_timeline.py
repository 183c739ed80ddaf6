"""Print the kernel timeline of one step from a rocprofv3 kernel_trace.csv.

    python tools/step_timeline.py <kernel_trace.csv> [step_index_from_end]

Times are relative to the step's first kernel (k_classify), in µs, so the
critical path and the launch gaps between dependent kernels are visible.
"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 3
idx = [i for i, r in enumerate(rows) if "k_classify" in r["Kernel_Name"].split("(")[0]]
i0, i1 = idx[-k], idx[-k + 1]
t0 = int(rows[i0]["Start_Timestamp"])
prev_end = t0
busy = 0.0
for r in rows[i0:i1 + 1]:
    s = (int(r["Start_Timestamp"]) - t0) / 1000
    e = (int(r["End_Timestamp"]) - t0) / 1000
    name = r["Kernel_Name"].replace("kmcd::", "").replace("void ", "").split("(")[0][:34]
    print(f"{name:34s} q{r['Queue_Id']:>2} {s:8.1f} {e:8.1f} {e - s:7.1f}  grid={r['Grid_Size_X']:>8} "
          f"wg={r['Workgroup_Size_X']:>4} vgpr={r['VGPR_Count']:>3} lds={r['LDS_Block_Size']}")
