"""Replica ensembles across GPUs ("replicas only").

A single trajectory does not shard: its unit order and greedy reactions are
global.  Independent trajectories (key = (seed, replica)) run one per GPU;
the only cross-GPU traffic is the ensemble observable reduction — one
all-reduce of the per-step bond.dat counters (SUM) and one of the largest
complex (MAX) per batch of K steps, over RCCL (`torch.distributed` backend
"nccl") on MI355X, or gloo on CPU for tests.  The messages are K·7·8 bytes:
latency-bound, so they are batched per kmc_step call, never per step.
"""
from __future__ import annotations

import numpy as np

SUM_FIELDS = ("bond_num_rl", "bond_num_mono_cis", "bond_num_cis", "bond_num", "tot_proteins_in_cluster",
              "tot_cluster_num")
MAX_FIELDS = ("protein_num_in_max_complex",)


def pack(obs: np.ndarray):
    """kmc_obs records → (K×6 int64 sums, K×1 int64 maxima)."""
    s = np.stack([obs[f].astype(np.int64) for f in SUM_FIELDS], axis=1)
    m = np.stack([obs[f].astype(np.int64) for f in MAX_FIELDS], axis=1)
    return s, m


def reduce(obs: np.ndarray, device=None, group=None):
    """All-reduce a rank's K observables into ensemble totals.

    Returns (sums K×6, maxima K×1, mean cluster size per step) as numpy.
    """
    import torch
    import torch.distributed as dist

    s, m = pack(obs)
    ts = torch.from_numpy(s)
    tm = torch.from_numpy(m)
    if device is not None:
        ts, tm = ts.to(device), tm.to(device)
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(ts, op=dist.ReduceOp.SUM, group=group)
        dist.all_reduce(tm, op=dist.ReduceOp.MAX, group=group)
    s, m = ts.cpu().numpy(), tm.cpu().numpy()
    tot_prot, tot_clu = s[:, 4].astype(np.float64), s[:, 5].astype(np.float64)
    cluster = np.divide(tot_prot, tot_clu, out=np.zeros_like(tot_prot), where=tot_clu != 0)
    return s, m, cluster
