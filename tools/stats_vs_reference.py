"""Statistical parity of the keyed engine with the reference's random process.

The reference draws every uniform from a freshly clock-seeded mt19937_64
(main.cpp:2313-2326), so no run of it can be reproduced; the keyed engine
replaces that by Philox draws addressed by (seed, replica, step, site).  Both
are processes of iid uniforms driving the same physics, so their ensembles
must agree in distribution.  This script (development container only: it
needs /root/reference/main.cpp, compiled unmodified by `make -C oracle ref`)
runs

  * K reference runs of the dense scenario, run r with its clock counter
    starting at T0 = 1000003·(r+1) (independent mt19937_64 seeds), and
  * K keyed-oracle replicas (seed 1, replica r) — the oracle is bit-identical
    to the GPU engine (tests/test_gpu_parity.py),

each from its own random placement, samples the bond.dat / cluster observables
every `every` steps, and writes them with per-(observable, time) Welch
t-statistics to tests/golden/stats_dense.json (data only).

    python tools/stats_vs_reference.py [K=32] [steps=3000] [every=250]
"""
from __future__ import annotations

import json
import math
import multiprocessing as mp
import os
import subprocess
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle as O  # noqa: E402

DENSE = dict(box_x=1000.0, box_y=1000.0, box_z=250.0, mono_cis_ass_rate=0.01, cis_ass_rate=0.09,
             diss_rate=0.00002, mono_cis_diss_rate=0.0002, cis_diss_rate=0.00005)
FIELDS = ["rl", "mono", "cis", "bond", "maxc", "tot_prot", "tot_clu"]
OUT = os.path.join(REPO, "tests", "golden", "stats_dense.json")


def ref_run(args):
    r, steps, every = args
    tmp = tempfile.mkdtemp(prefix=f"stat_ref_{r}_")
    sets = [f"simu_step={steps}"] + [f"{O.REF_GLOBALS[k]}={v!r}" for k, v in DENSE.items()]
    env = dict(os.environ, KMC_REF_T0=str(1000003 * (r + 1)), KMC_REF_TRACE=os.path.join(tmp, "trace.txt"),
               KMC_REF_SET=",".join(sets))
    subprocess.run([O.REF_BIN], cwd=tmp, env=env, stdout=subprocess.DEVNULL, check=True)
    rows = {row["step"]: row for row in O.parse_trace(os.path.join(tmp, "trace.txt"))}
    subprocess.run(["rm", "-rf", tmp], check=True)
    return [[int(rows[s][f]) for f in FIELDS] for s in range(every, steps + 1, every)]


def engine_run(r, steps, every):
    p = O.capi.default_params(n_a=150, n_b=50, seed=1, replica=r, **DENSE)
    o = O.Oracle(p)
    o.init_placement()
    obs, _ = o.step(steps, want_hashes=False)
    names = {"rl": "bond_num_rl", "mono": "bond_num_mono_cis", "cis": "bond_num_cis", "bond": "bond_num",
             "maxc": "protein_num_in_max_complex", "tot_prot": "tot_proteins_in_cluster", "tot_clu": "tot_cluster_num"}
    return [[int(obs[s - 1][names[f]]) for f in FIELDS] for s in range(every, steps + 1, every)]


def welch(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    va, vb = a.var(ddof=1) / len(a), b.var(ddof=1) / len(b)
    if va + vb == 0:
        return 0.0
    return float((a.mean() - b.mean()) / math.sqrt(va + vb))


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3000
    every = int(sys.argv[3]) if len(sys.argv) > 3 else 250
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "ref"], check=True)
    with mp.Pool(min(8, os.cpu_count() or 1)) as pool:
        ref = pool.map(ref_run, [(r, steps, every) for r in range(K)])
    eng = [engine_run(r, steps, every) for r in range(K)]
    ref_a, eng_a = np.array(ref), np.array(eng)  # [run][time][field]
    times = list(range(every, steps + 1, every))
    t = [[welch(ref_a[:, i, f], eng_a[:, i, f]) for f in range(len(FIELDS))] for i in range(len(times))]
    doc = {
        "scenario": "dense 150+50 (tests/golden/make_golden.py DENSE), reference defaults otherwise",
        "fields": FIELDS,
        "times": times,
        "reference_runs": ref,
        "engine_runs": eng,
        "engine": "keyed oracle, seed 1, replicas 0..K-1 (bit-identical to the GPU engine)",
        "reference": "unmodified main.cpp + oracle/ref_interpose.cpp, clock counter T0 = 1000003*(r+1)",
        "welch_t": t,
    }
    json.dump(doc, open(OUT, "w"))
    print("max |t| =", max(abs(x) for row in t for x in row))
    for i, s in enumerate(times):
        print(s, " ".join(f"{FIELDS[f]}={ref_a[:, i, f].mean():6.2f}/{eng_a[:, i, f].mean():6.2f}({t[i][f]:+.1f})"
                          for f in range(len(FIELDS))))


if __name__ == "__main__":
    main()
