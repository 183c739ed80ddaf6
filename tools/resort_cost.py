"""Re-sort cost from a rocprofv3 kernel trace: for each re-sort (k_slot_keys
through the next k_home_place, in launch order) the sum of its kernels'
durations, its wall span and its launch count; means over the re-sorts.
  python tools/resort_cost.py run_kernel_trace.csv [...]"""
import csv
import sys

for path in sys.argv[1:]:
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    groups, cur = [], None
    for r in rows:
        name = r["Kernel_Name"].split("(")[0]
        t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if "k_slot_keys" in name:
            cur = [0.0, t0, t1, 0, {}]
        if cur is not None:
            cur[0] += (t1 - t0) / 1e3
            cur[2] = t1
            cur[3] += 1
            short = "rocprim" if "rocprim" in name else name.replace("void ", "").replace("kmcd::", "")
            cur[4][short] = cur[4].get(short, 0.0) + (t1 - t0) / 1e3
            if "k_home_place" in name:
                groups.append(cur)
                cur = None
    n = len(groups)
    if not n:
        print(path, "no re-sort")
        continue
    busy = sum(g[0] for g in groups) / n
    span = sum((g[2] - g[1]) / 1e3 for g in groups) / n
    launches = sum(g[3] for g in groups) / n
    print(f"{path}: {n} re-sorts, kernels {busy:.1f} us, span {span:.1f} us, {launches:.0f} launches per re-sort")
    per = {}
    for g in groups:
        for k, v in g[4].items():
            per[k] = per.get(k, 0.0) + v / n
    for k, v in sorted(per.items(), key=lambda x: -x[1]):
        print(f"    {k:28s} {v:9.1f} us")
