"""The complex chain on a second stream (KMC_CX_STREAM): beside
the free units' proposals the complexes' kernels touch disjoint slots, beads
and records and share lists only through atomics, so every arrangement gives
the one-stream trajectory — mode 1 (the whole chain beside the free units),
2 (the BFS and the parameters), 3 (the checks and the heavy path after the
members; the default from 4 M proteins) — in every bond.dat record and
full-state hash.  Here in the C5 regime with the dense scenario's rates
(multi-ligand complexes, lay-down, the goto repeat, every reaction), from an
evolved state.  The one-stream path's oracle equality is the rest of the
suite; full C5 (mode 3 by default) is test_gpu_steady's C5 step."""
import math

import numpy as np
import pytest

from _kmc import DENSE, engine

pytestmark = pytest.mark.gpu

RATES = {k: v for k, v in DENSE.items() if not k.startswith("box")}


def _params():
    n = 100000
    L = 5773.0 * math.sqrt(n / 1500)
    return engine.capi.default_params(n_a=n, n_b=n, box_x=L, box_y=L, box_z=1000.0, seed=6, **RATES)


def _run(monkeypatch, mode, p, st, steps, every):
    monkeypatch.setenv("KMC_CX_STREAM", mode)
    obs, hashes = [], []
    with engine.Simulation(p) as sim:
        sim.set_state(st)
        for _ in range(steps // every):
            obs.append(sim.step(every))
            hashes.append(engine.state_hash(p, sim.get_state()))
    return np.concatenate(obs), hashes


@pytest.fixture(scope="module")
def evolved():
    p = _params()
    with engine.Simulation(p) as sim:  # (KMC_CX_STREAM unset: one stream at this size)
        sim.set_state(engine.host_init_random(p))
        sim.step(20000)
        st = sim.get_state()
    assert int(st.counters[0]) > 1000  # bonds, complexes
    return p, st


@pytest.mark.timeout(300)
@pytest.mark.parametrize("mode", ["1", "2", "3"])
def test_complex_stream_modes_equal_one_stream(monkeypatch, evolved, mode):
    p, st = evolved
    a, ha = _run(monkeypatch, "0", p, st, 1000, 50)
    b, hb = _run(monkeypatch, mode, p, st, 1000, 50)
    assert np.array_equal(a, b)
    assert ha == hb
