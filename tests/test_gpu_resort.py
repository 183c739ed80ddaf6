"""The re-sort's hand-written radix sort and scan (kmc_kernels.hip
k_rs_hist / k_rs_scatter / k_scan_*, kmc_engine.hip radix_sort / dev_scan).

With KMC_DEBUG_SYNC=1 the engine checks every re-sort on the host: the
sorted slot keys non-decreasing, equal keys in input order (a stable sort),
each kind's values a permutation, and the home list's cell starts the
exclusive scan of its counts — a failure is an engine error.  Nothing of the
trajectory depends on the slot order, so a run re-sorted every
7 steps under each grouping mode must equal the default run in every bond.dat
record and full-state hash; sizes are ragged against the sort's 4096-key
tiles and the keys span several 8-bit passes."""
import math

import numpy as np
import pytest

from _kmc import engine

pytestmark = pytest.mark.gpu


def _params(n_a, n_b, seed):
    L = 5773.0 * math.sqrt((n_a + n_b) / 2000)
    return engine.capi.default_params(n_a=n_a, n_b=n_b, box_x=L, box_y=L, box_z=1000.0, seed=seed)


def _run(monkeypatch, p, st, steps, env):
    for k in ("KMC_RESORT", "KMC_GROUP_SORT", "KMC_DEBUG_SYNC"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    obs, hashes = [], []
    with engine.Simulation(p) as sim:
        sim.set_state(st)
        for _ in range(steps // 10):
            obs.append(sim.step(10))
            hashes.append(engine.state_hash(p, sim.get_state()))
    return np.concatenate(obs), hashes


@pytest.mark.timeout(300)
@pytest.mark.parametrize("n_a,n_b", [(9000, 3001), (30001, 10003)])
def test_resort_sort_checked_and_trajectory_unchanged(monkeypatch, n_a, n_b):
    p = _params(n_a, n_b, seed=5)
    st = engine.host_init_random(p)
    # an evolved state: complexes and dimers give the grouped keys equal runs
    with engine.Simulation(p) as sim:
        sim.set_state(st)
        sim.step(2000)
        st = sim.get_state()
    assert int(st.counters[0]) > 0
    want, hw = _run(monkeypatch, p, st, 60, {})
    for group in ("0", "1", "2"):
        got, hg = _run(monkeypatch, p, st, 60, {"KMC_RESORT": "7", "KMC_GROUP_SORT": group, "KMC_DEBUG_SYNC": "1"})
        assert np.array_equal(got, want), group
        assert hg == hw, group
