"""Steady-state parity at the benchmark sizes.

The reference simulates 2e7 steps; a fresh placement has no bonds.  Here the
GPU evolves a benchmark configuration for thousands of steps (untimed, not
checked step by step — too long for the CPU), then the exact state it reached
(kmc_get_state, full precision) is handed to the keyed oracle (cell-list
mode) and a window of steps is compared bit for bit: every bond.dat record
and the full-state hash.  The oracle's event counters show which code paths
the window exercised (complexes, lay-down, alignment, dissociations,
collision rejections)."""
import sys
import time

import numpy as np
import pytest

from _kmc import DENSE, O, engine, workloads

pytestmark = pytest.mark.gpu

RATES = {k: v for k, v in DENSE.items() if not k.startswith("box")}


def _evolved_window(p, evolve, window):
    sim = engine.Simulation(p)
    sim.set_state(engine.host_init_random(p))
    t = time.time()
    done = 0
    while done < evolve:
        k = min(5000, evolve - done)
        ob = sim.step(k)
        done += k
        print(f"  evolved {done}/{evolve}: bond_num {int(ob[-1]['bond_num'])} ({time.time() - t:.0f}s)",
              file=sys.stderr, flush=True)
    st = sim.get_state()
    assert st.step == evolve
    obs = sim.step(window)
    h = engine.state_hash(p, sim.get_state())
    sim.close()
    o = O.Oracle(p, nbmode=O.NB_CELLS)
    o.set_state(st)
    obs_o = []
    for s in range(window):  # one step at a time: a progress line per oracle step
        obs_o.append(o.step(1, want_hashes=False)[0][0])
        print(f"  oracle step {evolve + s + 1} ({time.time() - t:.0f}s)", file=sys.stderr, flush=True)
    for s in range(window):
        assert obs[s] == obs_o[s], f"step {evolve + s + 1}: gpu {obs[s]} oracle {obs_o[s]}"
    assert h == o.hash()
    return o.stats(), obs


@pytest.mark.timeout(600)
def test_c3_steady_state_window():
    # C3: 1e6 particles, reference physics, 20 000 steps evolved, 20-step window
    p = workloads.params("C3", seed=1)
    ev, obs = _evolved_window(p, 20000, 20)
    print("  C3 window events", ev, file=sys.stderr)
    assert obs[-1]["bond_num"] > 1000
    for k in ("complex", "laydown", "reject", "rl", "snap_bond"):
        assert ev[k] > 0, k


@pytest.mark.timeout(600)
def test_c3_reaction_heavy_steady_state_window():
    # C3's box and population with the dense scenario's reaction rates (cis
    # association x200, dissociations 1e7-1e8 x the reference): every reaction
    # and dissociation type inside the window, multi-ligand complexes
    p = workloads.params("C3", seed=2, **RATES)
    ev, obs = _evolved_window(p, 20000, 20)
    print("  C3-heavy window events", ev, file=sys.stderr)
    assert obs[-1]["bond_num_mono_cis"] > 0 and obs[-1]["bond_num_cis"] > 0
    for k in ("complex", "multi", "reject", "rl", "mono", "cis", "rld", "md", "cd", "snap_bond", "snap_cis"):
        assert ev[k] > 0, k



# C5's regime (VERDICT r02 missing 3): the 1:1 mix and C5's density (10x the
# reference's area density, L = 5773·sqrt(n_a / 1500)) at 2e5 particles, so
# that the cell-list oracle can check a bond-rich window in the suite.  C5's
# reference rates form multi-ligand complexes (main.cpp:974-1732); the dense
# scenario's rates also fire every dissociation (main.cpp:2063-2141).
def _c5_regime(seed, **kw):
    import math

    n = 100000
    L = 5773.0 * math.sqrt(n / 1500)
    return engine.capi.default_params(n_a=n, n_b=n, box_x=L, box_y=L, box_z=1000.0, seed=seed, **kw)


@pytest.mark.timeout(600)
def test_c5_regime_steady_state_window():
    p = _c5_regime(seed=5)
    ev, obs = _evolved_window(p, 20000, 20)
    print("  C5-regime window events", ev, file=sys.stderr)
    assert obs[-1]["bond_num"] > 1000
    for k in ("complex", "multi", "laydown", "reject", "rl", "snap_bond"):
        assert ev[k] > 0, k


@pytest.mark.timeout(600)
def test_c5_regime_reaction_heavy_steady_state_window():
    p = _c5_regime(seed=6, **RATES)
    ev, obs = _evolved_window(p, 20000, 20)
    print("  C5-regime-heavy window events", ev, file=sys.stderr)
    for k in ("complex", "multi", "repeat", "reject", "rl", "mono", "cis", "rld", "md", "cd", "snap_bond",
              "snap_cis"):
        assert ev[k] > 0, k


@pytest.mark.timeout(600)
def test_c5_steady_state_step():
    # C5 itself (1e7 particles, 1:1, 10x area density, reference physics) in a
    # bond-rich state: 10 000 steps evolved on the GPU (≈ 750 000 bonds,
    # multi-ligand complexes), then one step against the oracle, every field
    # and the full-state hash (tools/c5_window.py runs the same check over 3
    # steps after 2e4: profiles/r06/c5_window_r6i_final.log)
    p = workloads.params("C5", seed=3)
    ev, obs = _evolved_window(p, 10000, 1)
    print("  C5 step events", ev, file=sys.stderr)
    assert obs[-1]["bond_num"] > 100000
    for k in ("complex", "multi", "reject", "snap_bond"):
        assert ev[k] > 0, k
