"""Benchmark: KMC particle-updates/s of the HIP engine (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload C3]

One process per GPU (launched by torch.distributed.run for N > 1), each
running an independent replica trajectory (key = (seed, rank)) of the
workload — SURVEY.md §8(e) "replicas only" — with one RCCL all-reduce of the
ensemble observables per timed batch.  Prints ONE JSON line (rank 0):

  value       particle-updates/s over all ranks = N_gpus · particles · K / t,
              t = max over ranks of the timed K steps (barrier + device sync
              on both sides; inputs resident in HBM)
  roofline    the dominant kernel's algorithmic HBM bytes per launch ÷ its
              average duration, measured with HIP events on the engine's
              stream over the timed region; peak 8 TB/s (MI355X HBM3E)
  cpu_baseline the keyed CPU oracle (single thread) on a bounded sample of
              the same workload, rank 0 at N = 1 only
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
PKG = "kmc-with-a-diffusion-reaction-algorithm_amd"
engine = importlib.import_module(PKG + ".engine")
workloads = importlib.import_module(PKG + ".workloads")
ensemble = importlib.import_module(PKG + ".ensemble")

TIMING_EVERY = 8
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md


def kernel_bytes(name: str, n_a: int, n_b: int):
    """Algorithmic HBM bytes per launch."""
    n = n_a + n_b
    models = {
        # read R (16 receptor / 8 ligand beads × xyz × 8 B), write R_new, unit
        # kind; the record counts it also takes write one rank pair per protein
        "k_propose": 768 * n_a + 384 * n_b + n + 8 * n,
        # every record once (float4 + id); candidate writes are data-dependent
        "k_col_scan": 2 * n * 24,
        # old + new reference points (x, y, zlo, zhi) + receptor site, record
        # write (pos, id, site), owner, cell cursor
        "k_rec_scatter": 2 * n * 32 + 2 * n_a * 16 + 2 * n * 32 + 4 * n + 2 * n * 8,
        "k_rec_count": 2 * n * 32 + 2 * n * 4 + 48 * n_a + 48 * n_b,
        # every record once (float4 + id + site) + final flags
        "k_rxn_scan": 2 * n * 32 + n,
        "k_commit": 8 * n,
        "k_classify": 20 * n_a + 12 * n_b + 5 * n,
        "k_observe": 16 * n_a + 5 * n_b,
    }
    return models.get(name)


TRAFFIC_JSON = "profiles/traffic_C3.json"


def pmc_traffic(kernel: str, workload: str):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes
    (FETCH_SIZE x2 + WRITE_SIZE, tools/pmc_traffic.py) of this same bench
    command; None when no profile of this workload is committed."""
    path = os.path.join(REPO, TRAFFIC_JSON)
    if workload != "C3" or not os.path.exists(path):
        return None
    rec = json.load(open(path)).get(kernel_trace_name(kernel))
    return rec["traffic_bytes"] if rec else None


def kernel_trace_name(name: str) -> str:
    # engine timing names -> the kernel symbol rocprof reports
    return {"k_rxn_scan": "k_rxn_scan_tile"}.get(name, name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", default="C3")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-baseline-steps", type=int, default=4)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--profile", action="store_true", help="print the per-kernel breakdown to stderr")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    p = workloads.params(args.workload, seed=args.seed, replica=rank)
    n = p.n_a + p.n_b
    sim = engine.Simulation(p, device=local)
    t0 = time.perf_counter()
    sim.init_random()
    t_init = time.perf_counter() - t0

    # warm-up with every kernel bracketed: find the dominant kernel
    names = engine.kernel_names()
    sim.set_timing(names)
    if args.warmup:
        sim.step(args.warmup)
    kt = sim.kernel_times()
    dom = max(kt, key=lambda k: kt[k][0]) if kt else "k_propose"
    breakdown = {k: round(v[0] / max(v[1], 1), 4) for k, v in sorted(kt.items(), key=lambda x: -x[1][0])}
    # timed region: only the dominant kernel is bracketed, in every 8th step
    # (an event pair adds a few microseconds of queue time to its step)
    sim.set_timing([dom], every=TIMING_EVERY)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    barrier()
    t0 = time.perf_counter()
    obs = sim.step(args.steps)
    sums, maxima, cluster = ensemble.reduce(obs, device=dev)
    barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())

    total_ms, launches = sim.kernel_times().get(dom, (0.0, 0))
    avg_s = total_ms / 1e3 / max(launches, 1)
    kb = kernel_bytes(dom, p.n_a, p.n_b)
    achieved = (kb / avg_s / 1e9) if (kb and avg_s > 0) else None
    traffic = pmc_traffic(dom, args.workload)
    step_b = workloads.step_bytes(p.n_a, p.n_b)
    ms_per_step = dt / args.steps * 1e3

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(p, sim, args.cpu_baseline_steps)

    if args.profile and rank == 0:
        print(json.dumps({"init_s": round(t_init, 3), "per_launch_ms": breakdown}), file=sys.stderr)

    if rank == 0:
        w = workloads.WORKLOADS[args.workload]
        line = {
            "metric": "KMC particle-updates/sec (and steps/sec) at 1e6 particles, 1/2/4/8 MI355X",
            "value": world * n * args.steps / dt,
            "unit": "particle-updates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "steps_per_s": args.steps / dt,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (keyed placement with the reference's rules, main.cpp:281-447)",
            "config": {
                "workload": f"{args.workload}: {w['desc']}",
                "particles_per_gpu": n,
                "n_receptors": p.n_a,
                "n_ligands": p.n_b,
                "box_A": [p.box_x, p.box_y, p.box_z],
                "parallelism": f"replicas x{world} (independent trajectories, RCCL all-reduce of observables)",
                "final_bond_num_ensemble": int(sums[-1, 3]),
            },
            "roofline": {
                "bound": "hbm",
                "kernel": dom,
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                "traffic": traffic,
                "traffic_source": TRAFFIC_JSON if traffic is not None else None,
                "bytes_per_launch": kb,
                "avg_launch_ms": avg_s * 1e3,
                "step_bytes": step_b,
                "step_frac": step_b / (ms_per_step / 1e3) / 1e9 / HBM_PEAK_GBS,
            },
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    sim.close()
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(p, sim, steps: int):
    """Keyed CPU oracle, one thread, a bounded sample of the same workload."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O

    st = sim.get_state()
    o = O.Oracle(p, rng_mode=O.RNG_KEYED, nbmode=O.NB_CELLS)
    o.set_state(st)
    t0 = time.perf_counter()
    o.step(steps, want_hashes=False)
    dt = time.perf_counter() - t0
    n = p.n_a + p.n_b
    return {
        "value": n * steps / dt,
        "unit": "particle-updates/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{steps} steps of the same workload and state on the keyed oracle (cell-list mode), 1 thread",
    }


if __name__ == "__main__":
    main()
