"""One trajectory split over G slabs (slabs.py, the
kmc_dd_* contract of include/kmc.h) — the decomposition's protocol on CPU.

The same driver that runs G libkmc handles (tests/test_gpu_slabs.py) runs
here over G keyed oracles restricted to their windows (oracle_dd_*: global
stream keys, owned observables, halo export / import, jumpers).  Every
step's bond.dat record and the full-state hash must equal one oracle over
the whole box (main.cpp:461-2308 restated sequentially), while units of
different slabs collide and bond across the cut.
"""
import os
import socket
import time

import numpy as np
import pytest
import torch.multiprocessing as mp

from _kmc import DENSE, PKG, O, engine, params

import importlib

slabs = importlib.import_module(PKG + ".slabs")
capi = importlib.import_module(PKG + ".capi")

RATES = {k: v for k, v in DENSE.items() if not k.startswith("box")}


class OracleWindow(O.Oracle):
    """An oracle over one slab's window (cell-list mode)."""

    def __init__(self, q):
        super().__init__(q, rng_mode=O.RNG_KEYED, nbmode=O.NB_CELLS)

    def step(self, n):
        return super().step(n, want_hashes=False)[0]  # the records, as engine.Simulation.step

    def close(self):
        pass


def scenario(n_a=4000, n_b=1500, L=6000.0, seed=9):
    p = params(n_a=n_a, n_b=n_b, seed=seed, box_x=L, box_y=L, box_z=250.0, **RATES)
    return p, engine.host_init_random(p)


def whole_box(p, st, steps):
    o = O.Oracle(p, nbmode=O.NB_CELLS)
    o.set_state(st)
    return o.step(steps)


def run_and_compare(p, st, G, steps, halo=900.0, lead=None):
    ref, hashes = whole_box(p, st, steps)
    got_h = []
    recs, ranks = slabs.run_local(p, st, G, steps, OracleWindow, halo=halo, gather_every=1, lead=lead,
                                  on_step=lambda me, k, rec: got_h.append(engine.state_hash(p, me.last_global)))
    bad = [k + 1 for k in range(steps) if recs[k] != ref[k] or got_h[k] != int(hashes[k])]
    assert not bad, f"G={G}: steps {bad[:10]} differ from the whole-box oracle"
    return ranks[0].stats


@pytest.mark.parametrize("G", [2, 3])
def test_slabs_equal_whole_box(G):
    p, st = scenario()
    s = run_and_compare(p, st, G, 250)
    # the cut is crossed: owned units collided with halo units, bonds joined
    # units of two slabs (each moved to one owner without a re-partition),
    # halo copies were verified
    print(f"G={G}: {s}")
    assert s["xcol"] > 0 and s["xbond"] > 0 and s["transfers"] > 0 and s["moved"] > 0, s
    assert s["verified"] > 0 and s["exchanged"] > 0, s
    assert s["owned"] < p.n_a + p.n_b and s["held"] < p.n_a + p.n_b, s


def test_slabs_narrow_halo_recovers():
    # a halo too narrow for the step's reach (band 180 Å, S = 20 Å): jumpers
    # fail their checks and halo copies their verification — every failure
    # rolls back to the checkpoint, replays, re-partitions (widening on a
    # repeat) and the trajectory is still the whole box's (lead 0: no
    # re-partition ahead of a failing jumper, so that the rollback is exercised)
    p, st = scenario(2000, 700, 4500.0, seed=17)
    s = run_and_compare(p, st, 2, 120, halo=360.0, lead=0.0)
    assert s["rollbacks"] > 0 and s["replayed"] > 0, s


def test_slabs_jumpers_repartition_ahead():
    # the same narrow halo with the default lead: a jumper within one step's
    # reach of failing its checks re-partitions the trajectory first, so no
    # step has to be rolled back
    p, st = scenario(2000, 700, 4500.0, seed=17)
    s = run_and_compare(p, st, 2, 120, halo=360.0)
    assert s["rebuild_jumpers"] > 0 and s["rollbacks"] == 0, s


def test_units_and_window_state():
    p, st = scenario(2000, 700, 4500.0, seed=17)
    o = O.Oracle(p, nbmode=O.NB_CELLS)
    o.set_state(st)
    o.step(150, want_hashes=False)
    hs = o.get_state()
    lab = slabs.units(hs)
    # every bond joins one unit; ligand-rooted complexes match the BFS rows
    row, mem = o.clusters()
    k = 0
    for b in range(p.n_b):
        m = mem[k:k + row[b]] - 1
        k += row[b]
        if m.size:
            assert np.all(lab[m] == lab[m].min()) and (lab == lab[m[0]]).sum() == m.size
    rl, mono, cis = slabs.derived_counts(hs)
    assert (rl, cis, mono) == tuple(int(x) for x in hs.counters[1:4]) and rl + mono + cis == hs.counters[0]
    plan = slabs.make_plan(p, hs, 3, 900.0)
    assert np.array_equal(np.sort(np.concatenate([w.gids[w.own == 1] for w in plan.windows])),
                          np.arange(p.n_a + p.n_b))  # every protein owned exactly once
    for w in plan.windows:
        ws = slabs.window_state(hs, w)
        assert engine.host_validate(capi.default_params(n_a=w.n_a, n_b=w.n_b, box_x=p.box_x, box_y=p.box_y,
                                                        box_z=p.box_z), ws) == 0
        # owned units are held whole, and so are the band's
        for sel in (w.own == 1, w.band):
            u = np.unique(lab[w.gids[sel]])
            assert np.isin(np.flatnonzero(np.isin(lab, u)), w.gids).all()


def _gloo_worker(rank, world, port, out, steps):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    p, st = scenario(2000, 700, 4500.0, seed=23)
    me = slabs.SlabRank(p, rank, slabs.TorchComm(), OracleWindow, gather_every=steps)
    me.start(st)
    recs = np.concatenate([me.step() for _ in range(steps)])
    if rank == 0:
        np.savez(out, recs=recs, hash=np.uint64(engine.state_hash(p, me.last_global)),
                 xcol=me.stats["xcol"], exchanged=me.stats["exchanged"])
    me.close()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def test_slabs_two_processes_gloo(tmp_path):
    # one rank per process: the halo exchange, verification and re-partition
    # over torch.distributed (gloo), as between GPUs
    steps = 100
    out = str(tmp_path / "slabs.npz")
    mp.spawn(_gloo_worker, args=(2, _free_port(), out, steps), nprocs=2, join=True)
    got = np.load(out)
    p, st = scenario(2000, 700, 4500.0, seed=23)
    ref, hashes = whole_box(p, st, steps)
    assert np.array_equal(got["recs"], ref)
    assert int(got["hash"]) == int(hashes[-1])
    assert int(got["xcol"]) > 0 and int(got["exchanged"]) > 0


def test_slabs_many_rollbacks_complete(monkeypatch):
    # every 7th step fails its checks once (an injected jumper failure): more
    # than 64 separate rollbacks, each replayed from the checkpoint and
    # retried from a new partition — the retries of ONE step are bounded, not
    # the run's total — and the run completes equal to the whole box
    orig = slabs.SlabRank._jumper_check

    def forced(self, ids, xs):
        fail, warn = orig(self, ids, xs)
        k = self.step_no + 1
        done = self.__dict__.setdefault("_forced", set())
        if k % 7 == 0 and k not in done:
            done.add(k)
            fail += 1
        return fail, warn

    monkeypatch.setattr(slabs.SlabRank, "_jumper_check", forced)
    p, st = scenario(2000, 700, 4500.0, seed=17)
    steps = 500
    ref, _ = whole_box(p, st, steps)
    recs, ranks = slabs.run_local(p, st, 2, steps, OracleWindow)
    s = ranks[0].stats
    assert s["rollbacks"] > 64 and s["replayed"] > 0, s
    assert np.array_equal(recs, ref)


def test_dd_window_arguments_checked():
    # kmc_dd_set_state's argument check (kmc_host_dd_check): a bad window is an
    # error code, never a device fault
    gid = np.array([0, 3, 7, 9], dtype=np.int32)
    own = np.array([1, 0, 1, 1], dtype=np.uint8)
    assert engine.host_dd_check(gid, own) == 0
    assert engine.host_dd_check(np.array([0, 3, 3, 9], np.int32), own) == capi.ERR_ARG  # not increasing
    assert engine.host_dd_check(np.array([-1, 3, 7, 9], np.int32), own) == capi.ERR_ARG
    assert engine.host_dd_check(np.array([0, 3, 7, 2 ** 31 - 1], np.int32), own) == capi.ERR_ARG  # link overflow
    assert engine.host_dd_check(gid, np.array([1, 0, 2, 1], np.uint8)) == capi.ERR_ARG  # ownership 0 / 1


def test_slab_fixture_pinned():
    # tests/golden/slabs_20000_7000.npz (make_slab_fixture.py) is what the GPU
    # decomposition is compared with, step for step: its first 40 steps are
    # the brute-force oracle's (brute_20000_7000.npz), and the cell-list
    # oracle run here reproduces its first 30 steps
    from _kmc import golden

    fx, br = golden("slabs_20000_7000"), golden("brute_20000_7000")
    n = len(br["hashes"])
    assert np.array_equal(fx["hashes"][:n], br["hashes"]) and np.array_equal(fx["obs"][:n], br["obs"])
    p = params(n_a=20000, n_b=7000, seed=9, box_x=14000.0, box_y=14000.0, box_z=250.0, **RATES)
    o = O.Oracle(p, nbmode=O.NB_CELLS)
    o.set_state(engine.host_init_random(p))
    obs, hashes = o.step(30)
    assert np.array_equal(obs, fx["obs"][:30]) and np.array_equal(hashes, fx["hashes"][:30])
    assert int(fx["obs"][-1]["bond_num"]) > 0


def _failing_worker(rank, world, port):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    p, st = scenario(2000, 700, 4500.0, seed=23)
    me = slabs.SlabRank(p, rank, slabs.TorchComm(), OracleWindow)
    me.start(st)
    if rank == 1:  # an error only this rank sees, between two collectives
        orig = me._jumper_check

        def boom(ids, xs):
            if me.step_no >= 4:
                raise RuntimeError("injected failure on rank 1")
            return orig(ids, xs)

        me._jumper_check = boom
    try:
        for _ in range(20):
            me.step()
    except RuntimeError:
        if rank == 1:
            # the failing rank stays alive (a driver writing its logs, say):
            # only the torn-down process group can release the other rank
            time.sleep(60)
        raise


def test_slabs_one_rank_failure_ends_every_rank():
    # an error raised on one rank only must not leave the others
    # waiting in their next collective forever — the failing rank tears the
    # process group down, and the other rank's collective fails at once
    ctx = mp.spawn(_failing_worker, args=(2, _free_port()), nprocs=2, join=False)
    ctx.processes[0].join(timeout=40)
    waiting = ctx.processes[0].is_alive()
    for proc in ctx.processes:
        if proc.is_alive():
            proc.kill()
        proc.join()
    assert not waiting, "rank 0 still waits in a collective after rank 1 failed"
    assert ctx.processes[0].exitcode != 0
