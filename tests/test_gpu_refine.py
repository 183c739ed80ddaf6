"""The record refinements: a collision candidate with a ligand
(k_col_exact's col_refine) and an R–L reaction pair (k_commit_rxn's
rxn_refine) are first tested from the two 32-byte records (subunit offsets
packed in the ligand record, the receptor's axis and [3][3] site) and gather
fp64 beads only when the records cannot rule the collision / the site gate
out.  Neither may drop a pair that passes, so the trajectory with each equals
the one without it (KMC_COL_REFINE=0, KMC_RXN_REFINE=0) in every bond.dat
record and full-state hash — here in the ligand-rich C5 regime (1:1 mix at
C5's area density, the dense association rates so that bonds form), from the
placement and from an evolved state with complexes.  The oracle equality of
the refined path is the rest of the GPU suite (it runs with the default, on)."""
import numpy as np
import pytest

from _kmc import engine

pytestmark = pytest.mark.gpu


def _c5_regime(seed, **rates):
    import math

    n = 100000
    L = 5773.0 * math.sqrt(n / 1500)
    return engine.capi.default_params(n_a=n, n_b=n, box_x=L, box_y=L, box_z=1000.0, seed=seed, **rates)


def _run(monkeypatch, knob, refine, p, st, steps, every):
    monkeypatch.setenv(knob, refine)
    obs, hashes = [], []
    with engine.Simulation(p) as sim:
        sim.set_state(st)
        for _ in range(steps // every):
            obs.append(sim.step(every))
            hashes.append(engine.state_hash(p, sim.get_state()))
    return np.concatenate(obs), hashes


@pytest.mark.timeout(300)
@pytest.mark.parametrize("knob", ["KMC_COL_REFINE", "KMC_RXN_REFINE"])
def test_refinement_changes_nothing(monkeypatch, knob):
    rates = {} if knob == "KMC_COL_REFINE" else dict(mono_cis_ass_rate=0.01, cis_ass_rate=0.09, ass_rate=0.4)
    p = _c5_regime(seed=11, **rates)
    st0 = engine.host_init_random(p)
    # an evolved state: bonds, complexes, the ligand-rich collision mix
    monkeypatch.setenv(knob, "1")
    with engine.Simulation(p) as sim:
        sim.set_state(st0)
        sim.step(4000)
        st1 = sim.get_state()
    assert int(st1.counters[0]) > 0  # bonds formed
    for st, steps in ((st0, 200), (st1, 400)):
        a, ha = _run(monkeypatch, knob, "1", p, st, steps, 20)
        b, hb = _run(monkeypatch, knob, "0", p, st, steps, 20)
        assert np.array_equal(a, b)
        assert ha == hb


@pytest.mark.timeout(120)
def test_rxn_refinement_engages(monkeypatch, capfd):
    # the R–L refinement is on for a state from the placement (the templates'
    # site geometry, sites_ok) and rules out most site tests in the C5 regime
    p = _c5_regime(seed=11)
    monkeypatch.setenv("KMC_DEBUG_CAND", "1")
    monkeypatch.setenv("KMC_DEBUG_COUNTS", "1")
    with engine.Simulation(p) as sim:
        sim.set_state(engine.host_init_random(p))
        sim.step(50)
    line = [x for x in capfd.readouterr().err.splitlines() if "refined-out" in x][-1]
    f = line.split()
    final, gate, out = int(f[f.index("final") + 1]), int(f[f.index("gate") + 1]), int(f[f.index("refined-out") + 1])
    print(line)
    assert out > 0 and final > 0
