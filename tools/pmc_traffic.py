"""Per-kernel HBM traffic per launch from rocprofv3 FETCH_SIZE / WRITE_SIZE passes.

    python tools/pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv> [out.json]

Corrections (/opt/skills/guides/MI355X_MICROARCH.md, "HBM"): FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half of the bytes of a
wide coalesced streaming read, so it is doubled; WRITE_SIZE is taken as is.
The first `skip` dispatches of every kernel (clock ramp) are dropped.
Output: {kernel: {"fetch_bytes", "write_bytes", "traffic_bytes", "launches"}}.
"""
import re
import collections
import csv
import json
import sys


def per_kernel(path, counter, skip=5):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        k = re.sub(r"^void (k_\w+)<\d+>$", r"\1", r["Kernel_Name"].split("(")[0].replace("kmcd::", ""))
        acc[k].append(float(r["Counter_Value"]))
    return {k: (v[skip:] if len(v) > skip else v) for k, v in acc.items()}


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [0.0])
        w = write.get(k, [0.0])
        fb = 2.0 * 1024.0 * sum(f) / len(f)
        wb = 1024.0 * sum(w) / len(w)
        out[k] = {"fetch_bytes": fb, "write_bytes": wb, "traffic_bytes": fb + wb, "launches": len(f)}
    text = json.dumps(out, indent=1, sort_keys=True)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(text + "\n")
    else:
        print(text)


if __name__ == "__main__":
    main()
