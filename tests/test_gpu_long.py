"""C2 long-horizon bit-exactness (BASELINE.json config 2: "1e5 particles, 1e5
steps, 1×MI355X, fixed seed — bit-exact state counts vs CPU").

tests/golden/c2_long.npz holds the keyed CPU oracle's (cell-list mode) run of
C2 (75 000 + 25 000 proteins, reference physics and density, seed 1) from the
keyed placement: every step's bond.dat record (main.cpp:2251 columns + cluster
sums) and the full-state hash every 100 steps, for 10^5 steps — 6 564 bonds
at the end, 8 639 lay-downs, 3.8·10^5 multi-ligand alignments, 6.2·10^6
collision rejections.  Steps 0–4·10^4 are one continuous oracle run
(make_c2_long.py 40000, 3.5 h of CPU); steps 4·10^4–10^5 are four oracle
segments of 1.5·10^4 steps (make_c2_long.py --start-state / --save-state),
joined by merge_c2_segments.py only because each segment's own final state is
byte-identical to the next segment's start state (and the first start state's
full hash equals the continuous run's at 4·10^4): every step is the oracle's.
The GPU replays the whole window here in about a minute."""
import os

import numpy as np
import pytest

from _kmc import GOLDEN, engine, workloads

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(600)
def test_c2_long_horizon_matches_oracle_fixture():
    g = np.load(os.path.join(GOLDEN, "c2_long.npz"), allow_pickle=False)
    steps, every = int(g["steps"]), int(g["hash_every"])
    p = workloads.params("C2", seed=int(g["seed"]))
    sim = engine.Simulation(p)
    sim.set_state(engine.host_init_random(p))
    for c in range(steps // every):
        obs = sim.step(every)
        ref = g["obs"][c * every:(c + 1) * every]
        if not np.array_equal(obs, ref):
            s = int(np.flatnonzero(obs != ref)[0])
            pytest.fail(f"step {c * every + s + 1}: gpu {obs[s]} oracle {ref[s]}")
        h = engine.state_hash(p, sim.get_state())
        assert h == int(g["hashes"][c]), f"state hash differs at step {(c + 1) * every}"
    assert sim.current_step == steps
    assert steps >= 100000 and g["obs"][-1]["bond_num"] > 6000
