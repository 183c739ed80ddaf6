"""Parity chain, link 3: the keyed engine's ensemble agrees in
distribution with the reference's own clock-seeded random process.

tests/golden/stats_dense.json holds, for the dense scenario, 32 runs of the
unmodified reference (compiled here with its clock replaced by a counter, one
independent mt19937_64 stream per run) and 32 keyed replicas, the bond.dat /
cluster observables every 250 steps to step 3000 (tools/stats_vs_reference.py
made it).  The keyed side is re-derived here from the current oracle (which is
bit-identical to the GPU engine), so the fixture cannot drift from the code."""
import json
import math
import os

import numpy as np

from _kmc import DENSE, O, REPO, capi

DOC = json.load(open(os.path.join(REPO, "tests", "golden", "stats_dense.json")))
NAMES = {"rl": "bond_num_rl", "mono": "bond_num_mono_cis", "cis": "bond_num_cis", "bond": "bond_num",
         "maxc": "protein_num_in_max_complex", "tot_prot": "tot_proteins_in_cluster", "tot_clu": "tot_cluster_num"}


def test_stored_engine_runs_are_current():
    times = DOC["times"]
    for r in range(4):
        p = capi.default_params(n_a=150, n_b=50, seed=1, replica=r, **DENSE)
        o = O.Oracle(p)
        o.init_placement()
        obs, _ = o.step(times[-1], want_hashes=False)
        rows = [[int(obs[s - 1][NAMES[f]]) for f in DOC["fields"]] for s in times]
        assert rows == DOC["engine_runs"][r], f"replica {r}"


def test_ensembles_agree():
    ref = np.array(DOC["reference_runs"], float)  # [run][time][field]
    eng = np.array(DOC["engine_runs"], float)
    assert ref.shape == eng.shape and ref.shape[0] >= 32
    worst = 0.0
    for i in range(ref.shape[1]):
        for f in range(ref.shape[2]):
            a, b = ref[:, i, f], eng[:, i, f]
            se = math.sqrt(a.var(ddof=1) / len(a) + b.var(ddof=1) / len(b))
            t = 0.0 if se == 0 else (a.mean() - b.mean()) / se
            worst = max(worst, abs(t))
    # 84 Welch statistics; |t| >= 4.5 has p < 1e-4 each under the null
    assert worst < 4.5, worst
    # reactions actually happened in both ensembles
    assert ref[:, -1, DOC["fields"].index("bond")].mean() > 5
    assert eng[:, -1, DOC["fields"].index("bond")].mean() > 5
