"""Step-wise GPU vs keyed-oracle state diff (debug tool, test infrastructure).

usage: python tools/diff_gpu_oracle.py n_a n_b L steps [seed] [box_z]
Writes gpurun_out/diff_<step>.npz with both states at the first mismatch.
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)
from _kmc import DENSE, O, engine, params  # noqa: E402

na, nb, L, steps = int(sys.argv[1]), int(sys.argv[2]), float(sys.argv[3]), int(sys.argv[4])
seed = int(sys.argv[5]) if len(sys.argv) > 5 else 9
bz = float(sys.argv[6]) if len(sys.argv) > 6 else 250.0
RATES = {k: v for k, v in DENSE.items() if not k.startswith("box")}
p = params(n_a=na, n_b=nb, seed=seed, box_x=L, box_y=L, box_z=bz, **RATES)
st = engine.host_init_random(p)
o = O.Oracle(p, nbmode=O.NB_CELLS)
o.set_state(st)
sim = engine.Simulation(p)
sim.set_state(st)
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
for s in range(1, steps + 1):
    g = sim.step(1)
    oo, _ = o.step(1, want_hashes=False)
    gs, os_ = sim.get_state(), o.get_state()
    if not gs.equal(os_) or g[0] != oo[0]:
        print("first mismatch at step", s, "gpu", g[0], "oracle", oo[0], flush=True)
        np.savez(os.path.join(REPO, "gpurun_out", f"diff_{s}.npz"), g_ra=gs.ra, g_rb=gs.rb, g_ai=gs.a_int,
                 g_bi=gs.b_int, o_ra=os_.ra, o_rb=os_.rb, o_ai=os_.a_int, o_bi=os_.b_int, step=s)
        for name in ("ra", "rb", "a_int", "b_int"):
            a, b = getattr(gs, name), getattr(os_, name)
            if name in ("ra", "rb"):
                bad = np.argwhere(a.view(np.uint64) != b.view(np.uint64))
            else:
                bad = np.argwhere(a != b)
            print(name, "mismatching (row, protein):", bad[:20].tolist(), flush=True)
        sys.exit(1)
print("no mismatch in", steps, "steps", flush=True)
