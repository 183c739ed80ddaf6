"""Summarise a rocprofv3 kernel-trace CSV: per-kernel mean duration (µs),
skipping the first `skip` launches of each kernel (clock ramp / warm-up)."""
import re
import csv
import collections
import sys

path = sys.argv[1]
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rows = list(csv.DictReader(open(path)))
by = collections.defaultdict(list)
for r in rows:
    name = re.sub(r"^void (k_\w+)<\d+>$", r"\1", r["Kernel_Name"].split("(")[0].replace("kmcd::", ""))
    by[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
tot = 0
out = []
for k, v in by.items():
    v = v[skip:] if len(v) > skip else v
    m = sum(v) / len(v)
    out.append((m, k, len(v)))
for m, k, n in sorted(out, reverse=True):
    print(f"{k:32s} {m:10.2f} us  (n={n})")
print("sum of means (us):", round(sum(m for m, _, _ in out), 1))
