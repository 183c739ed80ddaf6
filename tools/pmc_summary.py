"""Per-kernel mean of rocprofv3 counter_collection CSVs (one row per dispatch × counter)."""
import re
import csv
import collections
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        k = re.sub(r"^void (k_\w+)<\d+>$", r"\1", r["Kernel_Name"].split("(")[0].replace("kmcd::", ""))
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
want = sys.stdin.read().split() if not sys.stdin.isatty() else None
for k, cs in sorted(acc.items()):
    if want and k not in want:
        continue
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:24s} {sum(v) / len(v):16.1f}")
