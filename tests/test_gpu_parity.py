"""GPU parity: the HIP engine (through the C-ABI) against the keyed CPU oracle.

Bit-exact: every coordinate, status, link and counter after every step
(FNV-1a hash of the full state) and every bond.dat observable.
"""
import numpy as np
import pytest

from _kmc import DENSE, O, capi, engine, params

pytestmark = pytest.mark.gpu

OPS = {"sin": 0, "cos": 1, "atan2": 2, "acos": 3, "sqrt": 4, "div": 5, "round": 6}


@pytest.mark.parametrize("op", list(OPS))
def test_device_math_bitexact(op):
    rng = np.random.default_rng(OPS[op])
    n = 1 << 18
    if op == "acos":
        x = rng.uniform(-1.0, 1.0, n)
    elif op == "sqrt":
        x = np.abs(rng.standard_normal(n)) * 10.0 ** rng.integers(-3, 12, n)
    else:
        x = rng.uniform(-20.0, 20.0, n) * 10.0 ** rng.integers(-6, 4, n)
    y = rng.uniform(-20.0, 20.0, n)
    x[:8] = [0.0, -0.0, 1.0, -1.0, 0.5, -0.5, 2.5, -2.5]
    h = engine.math(OPS[op], x, y, device=False)
    d = engine.math(OPS[op], x, y, device=True)
    bad = np.flatnonzero(h.view(np.uint64) != d.view(np.uint64))
    assert bad.size == 0, f"{op}: {bad.size} mismatches, first x={x[bad[0]]!r} host={h[bad[0]]!r} dev={d[bad[0]]!r}"


def _run_pair(p, steps, nbmode=O.NB_BRUTE, init_state=None):
    o = O.Oracle(p, rng_mode=O.RNG_KEYED, nbmode=nbmode)
    if init_state is None:
        o.init_placement()
        st = o.get_state()
    else:
        st = init_state
        o.set_state(st)
    sim = engine.Simulation(p)
    sim.set_state(st)
    assert sim.get_state().equal(st)
    return o, sim


def _compare_stepwise(p, steps, nbmode=O.NB_BRUTE, init_state=None):
    o, sim = _run_pair(p, steps, nbmode, init_state)
    obs_o, hashes = o.step(steps)
    for s in range(steps):
        rec = sim.step(1)
        hs = sim.get_state()
        h = engine.state_hash(p, hs)
        if h != int(hashes[s]) or rec[0] != obs_o[s]:
            o2, _ = _run_pair(p, 0, nbmode, init_state)
            o2.step(s + 1, want_hashes=False)
            ref = o2.get_state()
            diff = [(name, np.argwhere(getattr(hs, name) != getattr(ref, name))[:5].tolist())
                    for name in ("ra", "rb", "a_int", "b_int") if not np.array_equal(getattr(hs, name), getattr(ref, name))]
            pytest.fail(f"step {s + 1}: hash {h:x} != {int(hashes[s]):x}; obs gpu={rec[0]} oracle={obs_o[s]}; "
                        f"counters {hs.counters} vs {ref.counters}; diff {diff}")
    sim.close()
    return o


def test_default_box_200_steps():
    p = params(seed=11)
    _compare_stepwise(p, 200)


def test_dense_reactions_3000_steps():
    p = params(seed=5, **DENSE)
    o = _compare_stepwise(p, 3000)
    st = o.stats()
    assert st["rl"] > 0 and st["complex"] > 0 and st["laydown"] > 0


def test_poisoned_rnew_dense(monkeypatch):
    # R_new filled with NaN before every step: any bead a proposal kernel
    # forgets to write would surface as a mismatch
    monkeypatch.setenv("KMC_DEBUG_POISON", "1")
    p = params(seed=21, **DENSE)
    o = O.Oracle(p)
    o.init_placement()
    st = o.get_state()
    sim = engine.Simulation(p)
    sim.set_state(st)
    obs = sim.step(1000)
    obs_o, _ = o.step(1000, want_hashes=False)
    assert np.array_equal(obs, obs_o)
    assert engine.state_hash(p, sim.get_state()) == o.hash()


@pytest.mark.parametrize("tcap", [0, 24])
def test_global_tile_path_dense(monkeypatch, tcap):
    # LDS tile capacity lowered: every (tcap=0) or most (24) tiles take the
    # global-memory scan path of the collision and reaction scans
    monkeypatch.setenv("KMC_DEBUG_TCAP", str(tcap))
    p = params(seed=23, **DENSE)
    o = O.Oracle(p)
    o.init_placement()
    sim = engine.Simulation(p)
    sim.set_state(o.get_state())
    obs = sim.step(1500)
    obs_o, _ = o.step(1500, want_hashes=False)
    assert np.array_equal(obs, obs_o)
    assert engine.state_hash(p, sim.get_state()) == o.hash()


@pytest.mark.parametrize("tout_cap", [None, "0"])
def test_global_tile_path_with_outliers(monkeypatch, capfd, tout_cap):
    # every tile on the dense list (KMC_DEBUG_TCAP=0) and no re-sort: the
    # brute force reads each tile's home records and its outlier bucket
    # (dense_records) — or, when the bucket overflowed (capacity 0), the whole
    # outlier list — with their own stride arithmetic and RID_OUT skip
    import re

    monkeypatch.setenv("KMC_DEBUG_TCAP", "0")
    monkeypatch.setenv("KMC_RESORT", "0")
    monkeypatch.setenv("KMC_DEBUG_COUNTS", "1")
    if tout_cap is not None:
        monkeypatch.setenv("KMC_DEBUG_TOUT_CAP", tout_cap)
    p = params(seed=47, **DENSE)
    o = O.Oracle(p)
    o.init_placement()
    sim = engine.Simulation(p)
    sim.set_state(o.get_state())
    obs = np.concatenate([sim.step(500) for _ in range(3)])
    obs_o, _ = o.step(1500, want_hashes=False)
    assert np.array_equal(obs, obs_o)
    assert engine.state_hash(p, sim.get_state()) == o.hash()
    outl = [int(x) for x in re.findall(r"outliers (\d+)", capfd.readouterr().err)]
    assert outl and outl[-1] > 10, f"too few outlier records to reach the dense path's outlier loop: {outl}"


def test_searched_home_lookup(monkeypatch):
    # KMC_DEBUG_HTAG=0: no tile tags its home entries, so every staged home
    # record finds its (segment, column) by the binary searches of tile_elem
    # (the path of a tile with more than HTAG_MAX home entries)
    monkeypatch.setenv("KMC_DEBUG_HTAG", "0")
    p = params(seed=53, **DENSE)
    o = O.Oracle(p)
    o.init_placement()
    sim = engine.Simulation(p)
    sim.set_state(o.get_state())
    obs = sim.step(1500)
    obs_o, _ = o.step(1500, want_hashes=False)
    assert np.array_equal(obs, obs_o)
    assert engine.state_hash(p, sim.get_state()) == o.hash()


def test_record_step_stamps(monkeypatch):
    # KMC_DEBUG_RECS=1: every record is stamped with its step when written and
    # k_rec_check raises ERR_RESOLVE (kmc_step fails) if any of the 2N records
    # was not rewritten by the kernel that moved its protein this step —
    # through free moves, complexes, lay-downs, alignments, rejections and
    # re-sorts
    monkeypatch.setenv("KMC_DEBUG_RECS", "1")
    p = params(seed=59, **DENSE)
    o = O.Oracle(p)
    o.init_placement()
    sim = engine.Simulation(p)
    sim.set_state(o.get_state())
    obs = sim.step(2000)
    obs_o, _ = o.step(2000, want_hashes=False)
    assert np.array_equal(obs, obs_o)
    st = o.stats()
    assert st["complex"] > 0 and st["laydown"] > 0 and st["reject"] > 0


def test_frequent_slot_resort_dense(monkeypatch):
    # slots re-sorted every 7 steps while bonds form and break: bond fields,
    # random-stream keys and unit keys must survive the renumbering
    monkeypatch.setenv("KMC_RESORT", "7")
    p = params(seed=29, **DENSE)
    o = O.Oracle(p)
    o.init_placement()
    sim = engine.Simulation(p)
    sim.set_state(o.get_state())
    obs = sim.step(2000)
    obs_o, _ = o.step(2000, want_hashes=False)
    assert np.array_equal(obs, obs_o)
    assert engine.state_hash(p, sim.get_state()) == o.hash()
    st = o.stats()
    assert st["rl"] > 0 and st["complex"] > 0


def test_exact_state_resume(tmp_path):
    # save after 400 dense steps, continue; a fresh handle loaded from the
    # file must reproduce the continuation bit for bit (and the oracle's)
    p = params(seed=31, **DENSE)
    o = O.Oracle(p)
    o.init_placement()
    sim = engine.Simulation(p)
    sim.set_state(o.get_state())
    sim.step(400)
    path = str(tmp_path / "state.kmc")
    sim.save_state(path)
    obs_a = sim.step(400)
    h_a = engine.state_hash(p, sim.get_state())
    sim.close()
    sim2 = engine.Simulation(p)
    sim2.load_state(path)
    assert sim2.current_step == 400
    obs_b = sim2.step(400)
    assert np.array_equal(obs_a, obs_b)
    assert engine.state_hash(p, sim2.get_state()) == h_a
    o.step(800, want_hashes=False)
    assert o.hash() == h_a


@pytest.mark.parametrize("graph", ["0", "1"])
def test_graph_replay_dense(monkeypatch, graph):
    # KMC_GRAPH=1: plain steps replay captured HIP graphs (one per buffer
    # parity; re-sorts every 7 steps force eager steps and fresh captures in
    # between); KMC_GRAPH=0: every step launched eagerly
    monkeypatch.setenv("KMC_GRAPH", graph)
    monkeypatch.setenv("KMC_RESORT", "7")
    p = params(seed=37, **DENSE)
    o = O.Oracle(p)
    o.init_placement()
    sim = engine.Simulation(p)
    sim.set_state(o.get_state())
    obs = np.concatenate([sim.step(n) for n in (1, 2, 997, 500)])
    obs_o, _ = o.step(1500, want_hashes=False)
    assert np.array_equal(obs, obs_o)
    assert engine.state_hash(p, sim.get_state()) == o.hash()


def test_chunked_steps_equal_single_steps():
    p = params(seed=3, **DENSE)
    o = O.Oracle(p)
    o.init_placement()
    st = o.get_state()
    sim = engine.Simulation(p)
    sim.set_state(st)
    obs = sim.step(1500)
    obs_o, _ = o.step(1500, want_hashes=False)
    assert np.array_equal(obs, obs_o)
    assert engine.state_hash(p, sim.get_state()) == o.hash()


RATES = {k: v for k, v in DENSE.items() if not k.startswith("box")}


@pytest.mark.parametrize("n_a,n_b,L,steps", [(4000, 1500, 6000.0, 300), (20000, 7000, 14000.0, 150)])
def test_larger_box_cell_oracle(n_a, n_b, L, steps):
    # near the dense scenario's area density; the host generator's placement
    # (proven identical to the oracle's, tests/test_host.py) and the oracle's
    # cell list keep the CPU side tractable
    p = params(n_a=n_a, n_b=n_b, seed=9, box_x=L, box_y=L, box_z=250.0, **RATES)
    st = engine.host_init_random(p)
    o = O.Oracle(p, nbmode=O.NB_CELLS)
    o.set_state(st)
    sim = engine.Simulation(p)
    sim.set_state(st)
    obs = sim.step(steps)
    obs_o, _ = o.step(steps, want_hashes=False)
    assert np.array_equal(obs, obs_o)
    assert engine.state_hash(p, sim.get_state()) == o.hash()


@pytest.mark.parametrize("name,steps", [("C2", 100), ("C3", 8), ("C5", 1)])
def test_benchmark_workload_window(name, steps):
    # the benchmark configurations themselves (C2 1e5, C3 1e6
    # dense, C5 1e7 at 1:1) bit-exact against the keyed oracle (cell mode)
    # over a step window from the same keyed placement
    W = __import__("_kmc").workloads
    p = W.params(name, seed=1)
    st = engine.host_init_random(p)
    o = O.Oracle(p, nbmode=O.NB_CELLS)
    o.set_state(st)
    sim = engine.Simulation(p)
    sim.set_state(st)
    obs = sim.step(steps)
    obs_o, _ = o.step(steps, want_hashes=False)
    assert np.array_equal(obs, obs_o)
    assert engine.state_hash(p, sim.get_state()) == o.hash()


def test_list_overflow_grow_and_replay(monkeypatch, capfd):
    # every output list and edge buffer starts 2^10 times too small: chunks
    # overflow, are undone from the device snapshot, the lists doubled and
    # the chunk replayed — the trajectory must not change (kmc_step)
    monkeypatch.setenv("KMC_DEBUG_CAP_SHIFT", "10")
    monkeypatch.setenv("KMC_DEBUG_COUNTS", "1")
    p = params(seed=37, **DENSE)
    o = O.Oracle(p)
    o.init_placement()
    sim = engine.Simulation(p)
    sim.set_state(o.get_state())
    obs = np.concatenate([sim.step(700), sim.step(800)])
    obs_o, _ = o.step(1500, want_hashes=False)
    assert np.array_equal(obs, obs_o)
    assert engine.state_hash(p, sim.get_state()) == o.hash()
    assert sim.current_step == 1500
    import re
    replays = [int(x) for x in re.findall(r"replays (\d+)", capfd.readouterr().err)]
    assert replays and replays[-1] > 0, "the lists never overflowed: the replay path was not exercised"


@pytest.mark.parametrize("span", [None, "0"])
def test_list_overflow_replay_across_calls(monkeypatch, capfd, span):
    # the snapshot is kept across kmc_step calls (KMC_SNAP_SPAN steps, default
    # 4096): with lists 2^10 times too small and 60 short calls, an overflow in
    # a later call restores the snapshot an earlier call took and replays the
    # steps already returned before it runs the failing chunk again.  Span 0:
    # a snapshot per chunk (the round-3 behaviour).  The trajectory must not
    # change.
    import re

    monkeypatch.setenv("KMC_DEBUG_CAP_SHIFT", "10")
    monkeypatch.setenv("KMC_DEBUG_COUNTS", "1")
    if span is not None:
        monkeypatch.setenv("KMC_SNAP_SPAN", span)
    p = params(seed=37, **DENSE)
    o = O.Oracle(p)
    o.init_placement()
    sim = engine.Simulation(p)
    sim.set_state(o.get_state())
    obs = np.concatenate([sim.step(25) for _ in range(60)])
    obs_o, _ = o.step(1500, want_hashes=False)
    assert np.array_equal(obs, obs_o)
    assert engine.state_hash(p, sim.get_state()) == o.hash()
    assert sim.current_step == 1500
    rows = [tuple(int(x) for x in m) for m in
            re.findall(r"kmc step (\d+):.*replays (\d+), snapshots (\d+)", capfd.readouterr().err)]
    assert len(rows) == 60
    if span is None:
        assert rows[-1][2] == 1, "one snapshot for 1500 steps"
        later = [r for k, r in enumerate(rows[1:], 1) if r[1] > rows[k - 1][1]]
        assert later, "no overflow after the first call: the cross-call replay was not exercised"
    else:
        assert rows[-1][2] == 60


@pytest.mark.parametrize("tout_cap", [None, "2", "0"])
def test_outlier_buckets_without_resort(monkeypatch, capfd, tout_cap):
    # KMC_RESORT=0: the home cells are never refreshed, so records drift more
    # than a cell from home and proteins cross the periodic boundary — the
    # outliers every tile must still stage (kmc_kernels.hip put_rec).  With the
    # default bucket capacity each tile reads its own bucket; with 2 most
    # tiles holding outliers overflow it and read the whole outlier list; with
    # 0 every such tile does.  The trajectory must not change.
    monkeypatch.setenv("KMC_RESORT", "0")
    monkeypatch.setenv("KMC_DEBUG_COUNTS", "1")
    if tout_cap is not None:
        monkeypatch.setenv("KMC_DEBUG_TOUT_CAP", tout_cap)
    p = params(seed=43, **DENSE)
    o = O.Oracle(p)
    o.init_placement()
    sim = engine.Simulation(p)
    sim.set_state(o.get_state())
    obs = np.concatenate([sim.step(500) for _ in range(4)])
    obs_o, _ = o.step(2000, want_hashes=False)
    assert np.array_equal(obs, obs_o)
    assert engine.state_hash(p, sim.get_state()) == o.hash()
    import re
    outl = [int(x) for x in re.findall(r"outliers (\d+)", capfd.readouterr().err)]
    assert outl and outl[-1] > 10, f"too few outlier records to exercise the buckets: {outl}"


def test_threshold_rebuild_without_resort(monkeypatch, capfd):
    # KMC_RESORT=0: no periodic re-sort resets the members[] cursor, so the
    # rows of the kept complexes (appended on every re-registration) reach
    # the limit (half of members[]; lowered here to 64 entries so that it
    # fires within the window) and k_finalize latches a full rebuild for the
    # next step (force_full; k_cx_kill only reads the latch).  The rebuilds
    # must fire and leave the trajectory unchanged.
    monkeypatch.setenv("KMC_RESORT", "0")
    monkeypatch.setenv("KMC_DEBUG_CX_LIMIT", "64")
    monkeypatch.setenv("KMC_DEBUG_COUNTS", "1")
    p = params(seed=41, **DENSE)
    o = O.Oracle(p)
    o.init_placement()
    sim = engine.Simulation(p)
    sim.set_state(o.get_state())
    obs = np.concatenate([sim.step(1000) for _ in range(4)])
    obs_o, _ = o.step(4000, want_hashes=False)
    assert np.array_equal(obs, obs_o)
    assert engine.state_hash(p, sim.get_state()) == o.hash()
    import re
    forced = [int(x) for x in re.findall(r"forced rebuilds (\d+)", capfd.readouterr().err)]
    assert forced and forced[-1] > 0, "the members[] threshold never fired"


def tile_census(p, st, tile):
    """Pair-scan tiles of side `tile` cells (kmc_kernels.hip k_pair_scan) by
    what they stage from state `st` (records at the cells of bead [1][1]):
    (no record in the home region — the block + 2 cells —, records but none in
    the block, block records of one kind only, block records of both kinds)."""
    cs = 130.0
    gx0, gy0 = -p.box_x / 2 - 1000.0, -p.box_y / 2 - 1000.0
    ncx, ncy = max(1, int((p.box_x + 2000.0) / cs) + 1), max(1, int((p.box_y + 2000.0) / cs) + 1)
    xs = np.concatenate([st.ra[0], st.rb[0]])
    ys = np.concatenate([st.ra[1], st.rb[1]])
    lig = np.concatenate([np.zeros(st.n_a, bool), np.ones(st.n_b, bool)])
    cx = np.clip(np.floor((xs - gx0) / cs).astype(int), 0, ncx - 1)
    cy = np.clip(np.floor((ys - gy0) / cs).astype(int), 0, ncy - 1)
    out = [0, 0, 0, 0]
    for y0 in range(0, ncy, tile):
        for x0 in range(0, ncx, tile):
            w, h = min(tile, ncx - x0), min(tile, ncy - y0)
            home = (cx >= x0 - 2) & (cx < x0 + w + 2) & (cy >= y0 - 2) & (cy < y0 + h + 2)
            blk = (cx >= x0) & (cx < x0 + w) & (cy >= y0) & (cy < y0 + h)
            if not home.any():
                out[0] += 1
            elif not blk.any():
                out[1] += 1
            elif lig[blk].all() or (~lig[blk]).all():
                out[2] += 1
            else:
                out[3] += 1
    return out


@pytest.mark.parametrize("tile", ["2", "3"])
def test_small_tiles_empty_tiles(monkeypatch, tile):
    # VERDICT r04 "next" 2: the round-4 illegal memory access (r4e,
    # profiles/r04/fault_r4e_empty_tile) came from a build whose pair-scan
    # staging binned ligands by z against the tile's highest receptor top — a
    # tile staging no receptor record had no top to reduce.
    # Small tiles on the dense scenario put every staging case into the suite:
    # tiles that stage nothing (the grid's 1000 Å margin), tiles with halo
    # records but no item, tiles whose items are of one kind only, and full
    # tiles; the kept walk skips a wave without pairs (tile_walk, Z == 0).
    monkeypatch.setenv("KMC_TILE", tile)
    p = params(seed=61, **DENSE)
    o = O.Oracle(p)
    o.init_placement()
    st = o.get_state()
    census = tile_census(p, st, int(tile))
    assert census[0] > 0 and census[1] > 0 and census[2] > 0 and census[3] > 0, census
    sim = engine.Simulation(p)
    sim.set_state(st)
    obs = np.concatenate([sim.step(750) for _ in range(2)])
    obs_o, _ = o.step(1500, want_hashes=False)
    assert np.array_equal(obs, obs_o)
    assert engine.state_hash(p, sim.get_state()) == o.hash()
    fin = tile_census(p, o.get_state(), int(tile))
    assert fin[0] > 0 and fin[1] > 0, fin
    print(f"tile {tile}: census start {census} end {fin} (empty, halo-only, one-kind, both)")
