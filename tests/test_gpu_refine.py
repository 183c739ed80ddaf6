"""The record refinement of the exact collision tests (k_col_exact's
col_refine): a candidate pair with a ligand is first tested from
the two 32-byte records (subunit offsets packed in the ligand record) and
gathers fp64 beads only when the records cannot rule the collision out.  It
must never drop a colliding pair, so the trajectory with it equals the one
without it (KMC_COL_REFINE=0) in every bond.dat record and full-state hash —
here in the ligand-rich C5 regime (1:1 mix at C5's area density), from the
placement and from an evolved state with complexes.  The oracle equality of the
refined path is the rest of the GPU suite (it runs with the default, on)."""
import numpy as np
import pytest

from _kmc import engine

pytestmark = pytest.mark.gpu


def _c5_regime(seed):
    import math

    n = 100000
    L = 5773.0 * math.sqrt(n / 1500)
    return engine.capi.default_params(n_a=n, n_b=n, box_x=L, box_y=L, box_z=1000.0, seed=seed)


def _run(monkeypatch, refine, p, st, steps, every):
    monkeypatch.setenv("KMC_COL_REFINE", refine)
    obs, hashes = [], []
    with engine.Simulation(p) as sim:
        sim.set_state(st)
        for _ in range(steps // every):
            obs.append(sim.step(every))
            hashes.append(engine.state_hash(p, sim.get_state()))
    return np.concatenate(obs), hashes


@pytest.mark.timeout(300)
def test_refinement_changes_nothing(monkeypatch):
    p = _c5_regime(seed=11)
    st0 = engine.host_init_random(p)
    # an evolved state: bonds, complexes, the ligand-rich collision mix
    monkeypatch.setenv("KMC_COL_REFINE", "1")
    with engine.Simulation(p) as sim:
        sim.set_state(st0)
        sim.step(4000)
        st1 = sim.get_state()
    assert int(st1.counters[0]) > 0  # bonds formed
    for st, steps in ((st0, 200), (st1, 400)):
        a, ha = _run(monkeypatch, "1", p, st, steps, 20)
        b, hb = _run(monkeypatch, "0", p, st, steps, 20)
        assert np.array_equal(a, b)
        assert ha == hb
