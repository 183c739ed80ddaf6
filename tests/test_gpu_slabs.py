"""One trajectory split over G slabs on the GPU: G libkmc
handles, each stepping its slab's window (kmc_dd_*), the device-resident halo
exchange / verification / ownership moves / re-partition of slabs.py between
them (G ranks as threads of this process, each window unpacking its
neighbours' send buffers on the device; or one rank per process over
torch.distributed).  Every step's bond.dat record and full-state hash must
equal the keyed cell-list oracle's (tests/golden/slabs_20000_7000.npz,
make_slab_fixture.py) — over all 500 steps, while units of different slabs
collide, bond across the cuts and move to one owner."""
import importlib
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from _kmc import DENSE, PKG, engine, golden, params, workloads

pytestmark = pytest.mark.gpu

slabs = importlib.import_module(PKG + ".slabs")
capi = importlib.import_module(PKG + ".capi")
RATES = {k: v for k, v in DENSE.items() if not k.startswith("box")}


def window_handle(q):
    return engine.Simulation(q, device=0)


def box_params():
    # the larger-box scenario of test_gpu_parity (20 000 + 7 000, 14 000 Å, the dense reaction rates)
    return params(n_a=20000, n_b=7000, seed=9, box_x=14000.0, box_y=14000.0, box_z=250.0, **RATES)


def single_gpu(p, st, steps):
    obs = np.zeros(steps, dtype=engine.capi.OBS_DTYPE)
    hashes = []
    with engine.Simulation(p, device=0) as sim:
        sim.set_state(st)
        for k in range(steps):
            obs[k] = sim.step(1)[0]
            hashes.append(engine.state_hash(p, sim.get_state()))
    return obs, hashes


def run_slabs(p, st, G, steps, **kw):
    got_h = []
    recs, ranks = slabs.run_local(p, st, G, steps, window_handle, gather_every=1,
                                  on_step=lambda me, k, rec: got_h.append(engine.state_hash(p, me.last_global)),
                                  **kw)
    for r in ranks:
        r.close()
    return recs, got_h, ranks[0].stats


@pytest.mark.timeout(900)
@pytest.mark.parametrize("G", [2, 4])
def test_slabs_equal_oracle(G):
    p = box_params()
    fx = golden("slabs_20000_7000")
    steps = int(fx["steps"])
    recs, got_h, s = run_slabs(p, engine.host_init_random(p), G, steps)
    print(f"G={G}: {s}")
    bad = [k + 1 for k in range(steps) if recs[k] != fx["obs"][k] or got_h[k] != int(fx["hashes"][k])]
    assert not bad, f"G={G}: steps {bad[:10]} differ from the keyed oracle"
    # the cuts were crossed: collisions and bonds between units of two slabs,
    # each joined unit moved to one owner (no re-partition for it)
    assert s["xcol"] > 0 and s["xbond"] > 0 and s["transfers"] > 0, s
    assert s["verified"] > 0 and s["owned"] < p.n_a + p.n_b, s


@pytest.mark.timeout(900)
@pytest.mark.parametrize("G", [2, 4])
def test_slabs_c2_window(G):
    # BASELINE config 2 (1e5 particles at the reference density), 100 steps,
    # against the single handle (itself the oracle's, test_gpu_parity's C2 window)
    p = workloads.params("C2", seed=1)
    st = engine.host_init_random(p)
    ref, ref_h = single_gpu(p, st, 100)
    recs, got_h, s = run_slabs(p, st, G, 100)
    print(f"C2 G={G}: {s}")
    bad = [k + 1 for k in range(100) if recs[k] != ref[k] or got_h[k] != ref_h[k]]
    assert not bad, f"G={G}: steps {bad[:10]} differ from the single-GPU run"
    assert s["verified"] > 0 and s["owned"] < p.n_a + p.n_b, s


@pytest.mark.timeout(900)
def test_slabs_c3_steady_window():
    # BASELINE config 3 (1e6 particles, dense) evolved 2e4 steps on one handle
    # (≈ 85 000 bonds), then 200 steps both as one handle and as two slab
    # windows on the device: every step's record and the final state equal
    p = workloads.params("C3", seed=1)
    with engine.Simulation(p, device=0) as sim:
        sim.init_random()
        sim.step(20000)
        st = sim.get_state()
        ref = sim.step(200).copy()
        ref_h = engine.state_hash(p, sim.get_state())
    assert int(st.counters[0]) > 50000
    recs, ranks = slabs.run_local(p, st, 2, 200, window_handle, halo=2400.0, gather_every=200)
    s = ranks[0].stats
    h = engine.state_hash(p, ranks[0].last_global)
    for r in ranks:
        r.close()
    print(f"C3 steady G=2: {s}")
    bad = [k for k in range(200) if recs[k] != ref[k]]
    assert not bad, f"steps {[int(ref[k]['step']) for k in bad[:10]]} differ from the single handle"
    assert h == ref_h


def test_dd_bad_window_is_an_error():
    # a window whose keys would overflow (a global index whose link + 1 does
    # not fit an int32) or whose ownership is not 0 / 1: an error code from
    # kmc_dd_set_state, nothing launched
    p = box_params()
    q = capi.Params.from_buffer_copy(p)
    q.n_a, q.n_b = 3, 1
    hs = capi.HostState(3, 1)
    gid = np.array([0, 1, 2, 20000], np.int32)
    with engine.Simulation(q, device=0) as sim:
        for g, own in ((np.array([0, 1, 2, 2 ** 31 - 1], np.int32), np.ones(4, np.uint8)),
                       (gid, np.array([1, 1, 2, 1], np.uint8)),
                       (np.array([0, 2, 1, 20000], np.int32), np.ones(4, np.uint8))):
            with pytest.raises(engine.KmcError) as e:
                sim.dd_set_state(hs, g, own, [0] * 5)
            assert e.value.code == capi.ERR_ARG


def _torch_gpu_worker(rank, world, port, out, steps):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    p = box_params()
    st = engine.host_init_random(p)
    me = slabs.SlabRank(p, rank, slabs.TorchComm(), window_handle, gather_every=steps)
    me.start(st)
    recs = np.concatenate([me.step() for _ in range(steps)])
    if rank == 0:
        np.savez(out, recs=recs, hash=np.uint64(engine.state_hash(p, me.last_global)), xcol=me.stats["xcol"],
                 xbond=me.stats["xbond"], verified=me.stats["verified"])
    me.close()
    dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_slabs_two_processes_gpu(tmp_path):
    # one rank per process, each with its own libkmc handle on the device and
    # the exchange through torch.distributed's all_to_all_single (gloo here:
    # the rows staged through host memory; RCCL needs one device per rank)
    steps = 200
    out = str(tmp_path / "slabs.npz")
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    mp.spawn(_torch_gpu_worker, args=(2, port, out, steps), nprocs=2, join=True)
    got = np.load(out)
    fx = golden("slabs_20000_7000")
    assert np.array_equal(got["recs"], fx["obs"][:steps])
    assert int(got["hash"]) == int(fx["hashes"][steps - 1])
    assert int(got["xcol"]) > 0 and int(got["verified"]) > 0
