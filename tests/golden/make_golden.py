"""Generate the golden fixtures in tests/golden/ from the REFERENCE itself.

Runs in the development container only (needs /root/reference/main.cpp): the
unmodified main.cpp is compiled where it lies, linked with
oracle/ref_interpose.cpp (deterministic clock for rand2(), counted glibc
rand(), portable libm, per-step trace hook) by `make -C oracle ref`, and run
in a scratch directory.  What is stored is data only — traces, states the
reference computed, and the files the reference wrote:

  <scenario>.npz        per-step trace rows (hash of the full state, bond
                        counters, cluster stats, draw counts, stream position)
                        + exact state dumps at a few steps
  <scenario>_<s>.cpt.gz position.cpt written by the reference at step s
  <scenario>_bond.dat   bond.dat written by the reference
  scenarios.json        parameters of every scenario

Usage: python tests/golden/make_golden.py [scenario ...]
"""
from __future__ import annotations

import gzip
import json
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle as O  # noqa: E402

NA, NB = 150, 50  # compiled into main.cpp:47-69

DENSE = dict(
    box_x=1000.0,
    box_y=1000.0,
    box_z=250.0,
    mono_cis_ass_rate=0.01,
    cis_ass_rate=0.09,
    diss_rate=0.00002,
    mono_cis_diss_rate=0.0002,
    cis_diss_rate=0.00005,
)

SCENARIOS = {
    # reference defaults (main.cpp:39-99): free diffusion + collisions
    "default": dict(t0=20251015, steps=3000, params={}, dump=[3000], keep="all"),
    # dense, reaction-heavy: every reaction type, lay-down, multi-ligand
    # alignment incl. the goto-lable4 repeat, all dissociations
    "dense": dict(
        t0=4242,
        steps=20000,
        params=DENSE,
        # x999 dumps: the state one step before each output step, from which
        # the cluster.log blocks (main.cpp:2291-2305) are regenerated
        dump=[4999, 8000, 9999, 14999, 15000, 19999, 20000],
        keep=[(0, 2000), (4999, 5000), (8000, 10000), (14999, 16000), (19999, 20000)],
        cpt_at=[5000, 10000, 15000, 20000],
    ),
    # resume from the reference's own position.cpt of "dense" at step 5000
    # (3-decimal text; main.cpp:226-270) — pins the reader and step+1 rule
    "resume": dict(
        t0=99,
        steps=10000,
        params=DENSE,
        dump=[5000, 9999, 10000],
        keep=[(5000, 6500), (9999, 10000)],
        input_cpt=("dense", 5000),
        cpt_at=[10000],
    ),
}


def ref_env(sc, tmp):
    p = O.capi.default_params(**sc["params"])
    sets = [f"simu_step={sc['steps']}"]
    for k, v in sc["params"].items():
        sets.append(f"{O.REF_GLOBALS[k]}={v!r}")
    env = dict(os.environ)
    env.update(
        KMC_REF_T0=str(sc["t0"]),
        KMC_REF_TRACE=os.path.join(tmp, "trace.txt"),
        KMC_REF_SET=",".join(sets),
        KMC_REF_DUMP_STEPS=",".join(str(s) for s in sc.get("dump", [])),
        KMC_REF_DUMP_PREFIX=os.path.join(tmp, "state_"),
    )
    return env, p


def run_scenario(name, sc):
    tmp = tempfile.mkdtemp(prefix=f"golden_{name}_")
    env, _ = ref_env(sc, tmp)
    if "input_cpt" in sc:
        src, s = sc["input_cpt"]
        with gzip.open(os.path.join(HERE, f"{src}_{s}.cpt.gz"), "rb") as f:
            open(os.path.join(tmp, "position.cpt"), "wb").write(f.read())
    cpt_at = sc.get("cpt_at", [])
    # the reference overwrites position.cpt every 5000 steps: run in segments
    # of its own process?  No — one process, and copy the file as it appears.
    proc = subprocess.Popen([O.REF_BIN], cwd=tmp, env=env, stdout=subprocess.DEVNULL)
    import time

    seen = {}
    cpt = os.path.join(tmp, "position.cpt")
    last_m = os.path.getmtime(cpt) if os.path.exists(cpt) else 0
    while proc.poll() is None:
        time.sleep(0.2)
        _grab(cpt, seen, last_m, cpt_at)
    _grab(cpt, seen, last_m, cpt_at)
    if proc.returncode != 0:
        raise SystemExit(f"reference failed: {proc.returncode}")
    rows = O.parse_trace(os.path.join(tmp, "trace.txt"))
    steps = np.array([r["step"] for r in rows], dtype=np.int64)
    keep = sc["keep"]
    if keep == "all":
        mask = np.ones(len(rows), bool)
    else:
        mask = np.zeros(len(rows), bool)
        for lo, hi in keep:
            mask |= (steps >= lo) & (steps <= hi)
        mask |= steps % 50 == 0
    cols = {}
    for key in ("step", "hash", "rl", "mono", "cis", "bond", "cluster_size", "maxc", "tot_prot", "tot_clu",
                "draws", "clock", "rand_calls"):
        dt = np.float64 if key == "cluster_size" else (np.uint64 if key in ("hash", "clock", "rand_calls") else np.int64)
        cols[key] = np.array([r[key] for r in rows], dtype=dt)[mask]
    dumps = {}
    for s in sc.get("dump", []):
        path = os.path.join(tmp, f"state_{s}.bin")
        raw = open(path, "rb").read()
        dumps[f"state_{s}"] = np.frombuffer(raw, dtype=np.uint8)
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **cols, **dumps)
    for s, data in seen.items():
        with gzip.GzipFile(os.path.join(HERE, f"{name}_{s}.cpt.gz"), "wb", mtime=0) as f:
            f.write(data)
    bond = os.path.join(tmp, "bond.dat")
    if os.path.exists(bond) and os.path.getsize(bond):
        shutil.copy(bond, os.path.join(HERE, f"{name}_bond.dat"))
    # the reference's other outputs (main.cpp:178-205, 2258-2305)
    for fn in ("parameter.log", "test.gro", "cluster.log"):
        src = os.path.join(tmp, fn)
        if os.path.exists(src) and os.path.getsize(src):
            with open(src, "rb") as f, gzip.GzipFile(os.path.join(HERE, f"{name}_{fn}.gz"), "wb", mtime=0) as g:
                g.write(f.read())
    shutil.rmtree(tmp)
    print(name, "rows", len(rows), "kept", int(mask.sum()), "cpts", sorted(seen))


def _grab(cpt, seen, last_m, cpt_at):
    if not os.path.exists(cpt):
        return
    try:
        data = open(cpt, "rb").read()
    except OSError:
        return
    lines = data.split(b"\n")
    if len(lines) < 2 or not lines[-1] == b"":
        return
    try:
        step = int(lines[-2])
    except ValueError:
        return
    expect = NA * 17 + NB * 12 + 6
    if len(lines) - 1 != expect:
        return
    if step in cpt_at and step not in seen:
        seen[step] = data


def main():
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "ref"], check=True)
    names = sys.argv[1:] or list(SCENARIOS)
    meta = {}
    for n in names:
        run_scenario(n, SCENARIOS[n])
    for n, sc in SCENARIOS.items():
        meta[n] = dict(t0=sc["t0"], steps=sc["steps"], params=sc["params"], n_a=NA, n_b=NB,
                       dump=sc.get("dump", []), input_cpt=sc.get("input_cpt"), cpt_at=sc.get("cpt_at", []))
    json.dump(meta, open(os.path.join(HERE, "scenarios.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
