"""Step rate of one trajectory split into G slabs (slabs.py) against the
single-handle engine on the same GPU, from the same placement (diagnostic
measurement, not the bench: the slab driver exchanges halos through the host
every step).
  python -u tools/slab_rate.py [workload] [G ...] [--steps K] [--procs]
Prints per G: ms/step, the driver's counters (units exchanged / verified per
step, re-partitions, rollbacks) and the single-handle ms/step.  --procs: the
G ranks as processes (torch.distributed over gloo, TorchComm, every handle on
device 0) instead of threads of this process.
"""
import argparse
import importlib
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
PKG = "kmc-with-a-diffusion-reaction-algorithm_amd"
engine = importlib.import_module(PKG + ".engine")
slabs = importlib.import_module(PKG + ".slabs")
workloads = importlib.import_module(PKG + ".workloads")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("workload", nargs="?", default="C2")
    ap.add_argument("G", nargs="*", type=int, default=[2, 4])
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--procs", action="store_true")
    a = ap.parse_args()
    p = workloads.params(a.workload, seed=1)
    st = engine.host_init_random(p)
    with engine.Simulation(p) as sim:
        sim.set_state(st)
        sim.step(10)
        t = time.time()
        sim.step(a.steps)
        one = (time.time() - t) / a.steps * 1e3
    print(f"{a.workload} single handle: {one:.3f} ms/step", flush=True)
    if a.procs:
        import socket

        import torch.multiprocessing as mp

        for G in a.G:
            with socket.socket() as so:
                so.bind(("127.0.0.1", 0))
                port = so.getsockname()[1]
            mp.spawn(_proc_rank, args=(G, port, a.workload, a.steps), nprocs=G, join=True)
        return
    for G in a.G:
        # the partition and the windows' handles (start) timed apart: two runs
        # from the same state, of 1 and of K steps
        tt = []
        for k in (1, a.steps):
            t0 = time.time()
            recs, ranks = slabs.run_local(p, st, G, k, lambda q: engine.Simulation(q), gather_every=k)
            tt.append(time.time() - t0)
            s = ranks[0].stats
            if k > 1:
                print("  rank 0 host ms/step by phase: " + ", ".join(
                    f"{n} {v / k * 1e3:.3f}" for n, v in s["sec"].items()), flush=True)
            for r in ranks:
                r.close()
        ms = (tt[1] - tt[0]) / (a.steps - 1) * 1e3
        print(f"{a.workload} G={G}: {ms:.3f} ms/step (start {tt[0] * 1e3:.0f} ms), exchanged "
              f"{s['exchanged'] / a.steps:.0f} verified {s['verified'] / a.steps:.0f} units/step, rebuilds "
              f"{s['rebuilds']}, rollbacks {s['rollbacks']}, held {s['held']} of {p.n_a + p.n_b}", flush=True)


def _proc_rank(rank, G, port, workload, steps):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=G)
    p = workloads.params(workload, seed=1)
    st = engine.host_init_random(p)
    me = slabs.SlabRank(p, rank, slabs.TorchComm(), lambda q: engine.Simulation(q, device=0), gather_every=0)
    t0 = time.time()
    me.start(st)
    dist.barrier()
    t1 = time.time()
    for k in range(steps):
        me.step()
    dist.barrier()
    t2 = time.time()
    if rank == 0:
        s = me.stats
        print(f"{workload} G={G} processes: {(t2 - t1) / steps * 1e3:.3f} ms/step (start {(t1 - t0) * 1e3:.0f} ms), "
              f"rebuilds {s['rebuilds']}, rollbacks {s['rollbacks']}; rank 0 host ms/step by phase: " +
              ", ".join(f"{n} {v / steps * 1e3:.3f}" for n, v in s["sec"].items() if n != "rebuild"), flush=True)
    me.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
