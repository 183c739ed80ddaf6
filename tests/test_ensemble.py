"""Replica ensembles: the only cross-GPU step is the
all-reduce of bond.dat observables.  Covered here with world_size 2 over gloo
on CPU, each rank's observables coming from the keyed oracle (what the GPU
reproduces bit for bit); the reduced series must equal the sum / max of the
independent replicas."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from _kmc import DENSE, PKG, O, params

import importlib

ensemble = importlib.import_module(PKG + ".ensemble")


def _replica_obs(replica, steps=120):
    p = params(seed=99, replica=replica, **DENSE)
    o = O.Oracle(p)
    o.init_placement()
    obs, _ = o.step(steps, want_hashes=False)
    return obs


def _worker(rank, world, port, out):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    obs = _replica_obs(rank)
    s, m, cluster = ensemble.reduce(obs)
    s2, m2, c2 = ensemble.Reducer(len(obs)).reduce(obs)  # preallocated buffers (bench.py's timed window)
    assert np.array_equal(s, s2) and np.array_equal(m, m2) and np.array_equal(cluster, c2)
    if rank == 0:
        np.savez(out, s=s, m=m, cluster=cluster)
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def test_two_replica_allreduce(tmp_path):
    out = str(tmp_path / "ens.npz")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = np.load(out)
    a, b = _replica_obs(0), _replica_obs(1)
    assert not np.array_equal(a, b), "replicas must be independent trajectories"
    sa, ma = ensemble.pack(a)
    sb, mb = ensemble.pack(b)
    assert np.array_equal(got["s"], sa + sb)
    assert np.array_equal(got["m"], np.maximum(ma, mb))
    tp, tc = (sa + sb)[:, 4], (sa + sb)[:, 5]
    assert np.allclose(got["cluster"], np.where(tc > 0, tp / np.maximum(tc, 1), 0.0))


# ---------------------------------------------------------------- bench launcher
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _bench(*args, env=None):
    import subprocess
    import sys

    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env or {})
    return subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True, env=e, timeout=300)


def test_bench_launcher_starts_n_ranks():
    # bench.py --gpus 2 without torchrun: a GPU-free parent starts 2 rank
    # processes that rendezvous (gloo here) with distinct ranks
    import json

    r = _bench("--gpus", "2", "--launcher-check")
    assert r.returncode == 0, r.stderr
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["world"] == 2
    assert sorted(x["rank"] for x in line["ranks"]) == [0, 1]
    assert sorted(x["local_rank"] for x in line["ranks"]) == [0, 1]
    assert len({x["pid"] for x in line["ranks"]}) == 2


def test_bench_refuses_more_gpus_than_visible():
    r = _bench("--gpus", "64")
    assert r.returncode != 0
    assert "refusing" in r.stderr


def test_bench_refuses_world_size_mismatch():
    r = _bench("--gpus", "1", env={"WORLD_SIZE": "2"})
    assert r.returncode != 0
    assert "WORLD_SIZE" in r.stderr


# ---------------------------------------------------------------- replicas on the GPU
def _gpu_worker(rank, world, port, out, steps):
    import torch.distributed as dist

    engine = importlib.import_module(PKG + ".engine")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    p = params(seed=99, replica=rank, **DENSE)
    with engine.Simulation(p, device=0) as sim:
        sim.set_state(engine.host_init_random(p))
        obs = sim.step(steps)
    s, m, cluster = ensemble.reduce(obs)  # CPU tensors over gloo (two ranks share one GPU)
    if rank == 0:
        np.savez(out, s=s, m=m, cluster=cluster)
    dist.destroy_process_group()


@pytest.mark.gpu
def test_two_gpu_replicas_reduced_equal_oracle_sum(tmp_path):
    # two replica trajectories through the HIP engine (one process each, same
    # GPU); the all-reduced series equals the sum / max of two keyed-oracle runs
    engine = importlib.import_module(PKG + ".engine")
    steps = 400
    out = str(tmp_path / "ens_gpu.npz")
    mp.spawn(_gpu_worker, args=(2, _free_port(), out, steps), nprocs=2, join=True)
    got = np.load(out)
    ref = []
    for r in range(2):
        p = params(seed=99, replica=r, **DENSE)
        o = O.Oracle(p)
        o.set_state(engine.host_init_random(p))
        ref.append(o.step(steps, want_hashes=False)[0])
    assert not np.array_equal(ref[0], ref[1])
    sa, ma = ensemble.pack(ref[0])
    sb, mb = ensemble.pack(ref[1])
    assert np.array_equal(got["s"], sa + sb)
    assert np.array_equal(got["m"], np.maximum(ma, mb))
    assert (sa + sb)[-1, 3] > 0, "the window should form bonds"


# ---------------------------------------------------------------- RCCL on the GPU
def _nccl_worker(rank, world, port, out, steps):
    import torch
    import torch.distributed as dist

    engine = importlib.import_module(PKG + ".engine")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                            device_id=dev)
    assert dist.get_backend() == "nccl"
    p = params(seed=99, replica=rank, **DENSE)
    with engine.Simulation(p, device=0) as sim:
        sim.set_state(engine.host_init_random(p))
        obs = sim.step(steps)
    s, m, cluster = ensemble.reduce(obs, device=dev)  # device tensors through RCCL
    if rank == 0:
        np.savez(out, s=s, m=m, cluster=cluster, obs=obs)
    dist.destroy_process_group()


@pytest.mark.gpu
def test_rccl_one_rank_reduce_equals_oracle(tmp_path):
    # the ensemble reduction of bench.py / C4 (main.cpp:2247-2253 observables)
    # through RCCL on device tensors: a 1-rank "nccl" group on the GPU (RCCL
    # refuses two ranks on one device); the reduced series equals the keyed
    # oracle's own series of the same replica
    engine = importlib.import_module(PKG + ".engine")
    steps = 300
    out = str(tmp_path / "ens_nccl.npz")
    mp.spawn(_nccl_worker, args=(1, _free_port(), out, steps), nprocs=1, join=True)
    got = np.load(out)
    p = params(seed=99, replica=0, **DENSE)
    o = O.Oracle(p)
    o.set_state(engine.host_init_random(p))
    ref = o.step(steps, want_hashes=False)[0]
    assert np.array_equal(got["obs"], ref)
    s, m = ensemble.pack(ref)
    assert np.array_equal(got["s"], s)
    assert np.array_equal(got["m"], m)
    assert s[-1, 3] > 0, "the window should form bonds"


def _c3_worker(rank, world, port, out, steps):
    import torch.distributed as dist

    engine = importlib.import_module(PKG + ".engine")
    workloads = importlib.import_module(PKG + ".workloads")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    p = workloads.params("C3", seed=1, replica=rank)
    with engine.Simulation(p, device=0) as sim:
        sim.set_state(engine.host_init_random(p))
        obs = sim.step(steps)
    s, m, cluster = ensemble.reduce(obs)
    np.save(out + f".obs{rank}.npy", obs)
    if rank == 0:
        np.savez(out, s=s, m=m, cluster=cluster)
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_two_c3_replicas_reduced_equal_oracle_sum(tmp_path):
    # C4's workload per GPU: two C3 replicas (1e6 particles each, key = (1,
    # replica)) through the HIP engine, one process each on the one GPU,
    # reduced over gloo; equal to the sum / max of two keyed-oracle windows
    # (cell-list mode) from the same placements
    engine = importlib.import_module(PKG + ".engine")
    workloads = importlib.import_module(PKG + ".workloads")
    steps = 3
    out = str(tmp_path / "ens_c3.npz")
    mp.spawn(_c3_worker, args=(2, _free_port(), out, steps), nprocs=2, join=True)
    got = np.load(out)
    ref = []
    for r in range(2):
        p = workloads.params("C3", seed=1, replica=r)
        o = O.Oracle(p, nbmode=O.NB_CELLS)
        o.set_state(engine.host_init_random(p))
        ref.append(o.step(steps, want_hashes=False)[0])
        assert np.array_equal(np.load(out + f".obs{r}.npy"), ref[r]), f"replica {r}"
    assert not np.array_equal(ref[0], ref[1])
    sa, ma = ensemble.pack(ref[0])
    sb, mb = ensemble.pack(ref[1])
    assert np.array_equal(got["s"], sa + sb)
    assert np.array_equal(got["m"], np.maximum(ma, mb))
