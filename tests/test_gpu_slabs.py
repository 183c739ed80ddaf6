"""One trajectory split over G slabs on the GPU (VERDICT r04
"next" 1): G libkmc handles on one device, each stepping its slab's window
(kmc_dd_*), the halo exchange / verification / re-partition of slabs.py
between them (G ranks as threads of this process).  Every step's bond.dat
record and the full-state hash must equal the single-handle run of the same
trajectory (itself bit-identical to the keyed oracle, test_gpu_parity.py),
while units of different slabs collide and bond across the cuts."""
import importlib
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from _kmc import DENSE, PKG, engine, params, workloads

pytestmark = pytest.mark.gpu

slabs = importlib.import_module(PKG + ".slabs")
RATES = {k: v for k, v in DENSE.items() if not k.startswith("box")}


def window_handle(q):
    return engine.Simulation(q, device=0)


def single_gpu(p, st, steps):
    obs = np.zeros(steps, dtype=engine.capi.OBS_DTYPE)
    hashes = []
    with engine.Simulation(p, device=0) as sim:
        sim.set_state(st)
        for k in range(steps):
            obs[k] = sim.step(1)[0]
            hashes.append(engine.state_hash(p, sim.get_state()))
    return obs, hashes


def compare(p, st, G, steps, halo=900.0):
    ref, ref_h = single_gpu(p, st, steps)
    got_h = []
    recs, ranks = slabs.run_local(p, st, G, steps, window_handle, halo=halo, gather_every=1,
                                  on_step=lambda me, k, rec: got_h.append(engine.state_hash(p, me.last_global)))
    try:
        bad = [k + 1 for k in range(steps) if recs[k] != ref[k] or got_h[k] != ref_h[k]]
        assert not bad, f"G={G}: steps {bad[:10]} differ from the single-GPU run"
        return ranks[0].stats, ref
    finally:
        for r in ranks:
            r.close()


@pytest.mark.timeout(900)
@pytest.mark.parametrize("G", [2, 4])
def test_slabs_equal_single_gpu(G):
    # the larger-box scenario of test_gpu_parity (20 000 + 7 000, 14 000 Å,
    # the dense reaction rates) over 500 steps
    p = params(n_a=20000, n_b=7000, seed=9, box_x=14000.0, box_y=14000.0, box_z=250.0, **RATES)
    st = engine.host_init_random(p)
    s, ref = compare(p, st, G, 500)
    print(f"G={G}: {s}")
    assert int(ref[-1]["bond_num"]) > 0
    # cross-slab collisions and bonds happened (each such bond re-partitions)
    assert s["xcol"] > 0 and s["xbond"] > 0 and s["rebuild_bond"] > 0, s
    assert s["verified"] > 0 and s["owned"] < p.n_a + p.n_b, s


@pytest.mark.timeout(900)
@pytest.mark.parametrize("G", [2, 4])
def test_slabs_c2_window(G):
    # BASELINE config 2 (1e5 particles at the reference density), 100 steps
    p = workloads.params("C2", seed=1)
    st = engine.host_init_random(p)
    s, _ = compare(p, st, G, 100)
    print(f"C2 G={G}: {s}")
    assert s["verified"] > 0 and s["owned"] < p.n_a + p.n_b, s


def _gloo_gpu_worker(rank, world, port, out, steps):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    p = params(n_a=20000, n_b=7000, seed=9, box_x=14000.0, box_y=14000.0, box_z=250.0, **RATES)
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
    # the exchange over torch.distributed (gloo): the one-process-per-GPU shape
    # of the decomposed mode, here with both ranks on one device
    steps = 200
    out = str(tmp_path / "slabs.npz")
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    mp.spawn(_gloo_gpu_worker, args=(2, port, out, steps), nprocs=2, join=True)
    got = np.load(out)
    p = params(n_a=20000, n_b=7000, seed=9, box_x=14000.0, box_y=14000.0, box_z=250.0, **RATES)
    ref, ref_h = single_gpu(p, engine.host_init_random(p), steps)
    assert np.array_equal(got["recs"], ref)
    assert int(got["hash"]) == int(ref_h[-1])
    assert int(got["xcol"]) > 0 and int(got["verified"]) > 0
