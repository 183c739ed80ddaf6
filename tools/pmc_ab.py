"""A/B of library variants or debug knobs from one saved steady state, with
HIP-event timings and rocprofv3 PMC counters per variant (runs on the GPU box).

  python tools/pmc_ab.py OUT [--workload C3] [--rounds 2] [--pmc GROUP ...] VARIANT ...

VARIANT = label[:lib=PATH][:ENV=VALUE ...]: `lib` selects a diagnostic build
(KMC_DIAG=1 KMC_LIB_PATH=..., tools/build_variants.py), the rest are
environment variables (e.g. KMC_DEBUG_SCAN_STAGE=1).  The workload is evolved
once with the in-tree library and saved (bench.py --save-state); every
variant then runs `rounds` interleaved timing benches (--profile: per-kernel
HIP-event means) and, per PMC group (counters separated by commas; each group
a separate rocprofv3 pass), one counter pass.  Output: OUT/<label>_<round>.json
/.err (bench lines), OUT/<label>_pmc<g>/ (rocprof CSVs), OUT/summary.json and
a table on stdout (ms/step, the pair scan and the selected kernels' counters).
"""
from __future__ import annotations

import re
import argparse
import csv
import glob
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = ("k_propose_free", "k_pair_scan", "k_col_exact", "k_commit_rxn", "k_complex_heavy",
           "k_move_members")


def run(cmd, env, out, err, limit):
    with open(out, "w") as fo, open(err, "w") as fe:
        p = subprocess.Popen(cmd, env=env, stdout=fo, stderr=fe, cwd=REPO)
        try:
            return p.wait(timeout=limit)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
            return 124


def variant_env(spec):
    parts = spec.split(":")
    label, env = parts[0], dict(os.environ)
    for kv in parts[1:]:
        k, v = kv.split("=", 1)
        if k == "lib":
            env["KMC_DIAG"] = "1"
            env["KMC_LIB_PATH"] = os.path.join(REPO, v)
        else:
            env[k] = v
    return label, env


def counters(path_glob):
    acc = {}
    for path in glob.glob(path_glob, recursive=True):
        for r in csv.DictReader(open(path)):
            k = re.sub(r"^void (k_\w+)<\d+>$", r"\1", r["Kernel_Name"].split("(")[0].replace("kmcd::", ""))
            acc.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--workload", default="C3")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--pmc", action="append", default=[])
    a = ap.parse_args()
    out = os.path.abspath(a.out)
    os.makedirs(out, exist_ok=True)
    state = f"/tmp/kmc_pmc_{a.workload}.kmc"
    bench = [sys.executable, os.path.join(REPO, "bench.py"), "--workload", a.workload]
    rc = run(bench + ["--steps", "10", "--warmup", "0", "--no-cpu-baseline", "--no-fresh-window", "--save-state",
                      state], dict(os.environ), f"{out}/evolve.json", f"{out}/evolve.err", 500)
    if rc != 0:
        sys.exit(f"evolution failed ({rc})")
    res = {}
    try:
        for r in range(a.rounds):
            for spec in a.variants:
                label, env = variant_env(spec)
                t0 = time.time()
                rc = run(bench + ["--load-state", state, "--steps", str(a.steps), "--warmup", "30",
                                  "--no-cpu-baseline", "--profile"], env, f"{out}/{label}_{r}.json",
                         f"{out}/{label}_{r}.err", 200)
                if rc != 0:
                    sys.exit(f"{label} round {r} failed ({rc})")
                line = json.loads(open(f"{out}/{label}_{r}.json").read().strip().splitlines()[-1])
                prof = {}
                for x in open(f"{out}/{label}_{r}.err"):
                    if x.startswith("{"):
                        prof = json.loads(x).get("per_launch_ms", prof)
                res.setdefault(label, {"ms_per_step": [], "per_launch_ms": []})
                res[label]["ms_per_step"].append(line["ms_per_step"])
                res[label]["per_launch_ms"].append(prof)
                print(f"{label} round {r}: {line['ms_per_step']:.4f} ms/step ({time.time() - t0:.0f} s)", flush=True)
        for g, grp in enumerate(a.pmc):
            for spec in a.variants:
                label, env = variant_env(spec)
                d = f"{out}/{label}_pmc{g}"
                cmd = ["rocprofv3", "--kernel-trace", "--pmc", *grp.split(","), "--output-format", "csv", "-d", d,
                       "-o", "run", "--", *bench, "--load-state", state, "--steps", "10", "--warmup", "5",
                       "--no-cpu-baseline"]
                env["TMPDIR"] = "/tmp"
                rc = run(cmd, env, f"{d}.log", f"{d}.err", 150)
                if rc != 0:
                    sys.exit(f"{label} pmc group {g} failed ({rc})")
                for k, cs in counters(f"{d}/**/*counter_collection.csv").items():
                    res[label].setdefault("pmc", {}).setdefault(k, {}).update(cs)
                print(f"{label} pmc {grp} done", flush=True)
    finally:
        if os.path.exists(state):
            os.remove(state)
        json.dump(res, open(f"{out}/summary.json", "w"), indent=1)
    for label, v in res.items():
        pl = v["per_launch_ms"][-1] if v["per_launch_ms"] else {}
        print(label, "ms/step", " ".join(f"{x:.4f}" for x in v["ms_per_step"]),
              " ".join(f"{k[2:]}={pl.get(k, 0) * 1e3:.1f}us" for k in KERNELS if k in pl))
        for k in KERNELS:
            if k in v.get("pmc", {}):
                print("   ", k, " ".join(f"{c}={x:.0f}" for c, x in sorted(v["pmc"][k].items())))


if __name__ == "__main__":
    main()
