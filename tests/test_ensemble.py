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
