"""Cost of the bench's per-window ensemble reduction on one GPU (RCCL, one
rank): the variants of ensemble reduction bench.py could use, each timed as
the bench times it (host wall clock, device synchronised), after a gap in
which the GPU was idle (as after a timed window).  Diagnostic only.

    python tools/reduce_micro.py [K] [gap_ms]
"""
import importlib
import json
import os
import socket
import statistics
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
ensemble = importlib.import_module("kmc-with-a-diffusion-reaction-algorithm_amd.ensemble")
capi = importlib.import_module("kmc-with-a-diffusion-reaction-algorithm_amd.capi")


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    gap = float(sys.argv[2]) if len(sys.argv) > 2 else 5.0
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    obs = np.zeros(k, dtype=capi.OBS_DTYPE)
    obs["bond_num"] = np.arange(k)
    red = ensemble.Reducer(k, device=dev)
    dsum = torch.zeros((k, 6), dtype=torch.int64, device=dev)
    dmax = torch.zeros((k, 1), dtype=torch.int64, device=dev)
    both = torch.zeros((k, 7), dtype=torch.int64, device=dev)
    gath = torch.zeros((1, k, 7), dtype=torch.int64, device=dev)

    def v_reducer():
        red.reduce(obs)

    def v_plain():
        ensemble.reduce(obs, device=dev)

    def v_device_two():
        dist.all_reduce(dsum, op=dist.ReduceOp.SUM)
        dist.all_reduce(dmax, op=dist.ReduceOp.MAX)
        torch.cuda.synchronize(dev)

    def v_device_one():
        dist.all_reduce(both, op=dist.ReduceOp.SUM)
        torch.cuda.synchronize(dev)

    def v_gather():
        dist.all_gather_into_tensor(gath, both)
        torch.cuda.synchronize(dev)

    def v_sync():
        torch.cuda.synchronize(dev)

    res = {}
    for name, f in [("sync", v_sync), ("device_all_reduce_x2", v_device_two), ("device_all_reduce_x1", v_device_one),
                    ("device_all_gather", v_gather), ("reducer", v_reducer), ("reduce", v_plain)]:
        for _ in range(5):
            f()
        ts = []
        for _ in range(40):
            time.sleep(gap / 1e3)
            torch.cuda.synchronize(dev)
            t = time.perf_counter()
            f()
            ts.append((time.perf_counter() - t) * 1e6)
        res[name] = {"median_us": statistics.median(ts), "min_us": min(ts), "max_us": max(ts)}
        print(name, json.dumps(res[name]), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
