"""Benchmark: KMC particle-updates/s of the HIP engine (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload C3] [--evolve E]

Ranks.  One process per GPU, each an independent replica trajectory (key =
(seed, rank)) — SURVEY.md §8(e) "replicas only" — with one RCCL all-reduce of
the ensemble observables per timed batch.  Under torch.distributed.run
(WORLD_SIZE set) this process is one rank and --gpus must equal WORLD_SIZE.
Without it and --gpus N > 1, this process is a GPU-free launcher: it checks
that N devices are visible (in a child process), starts N fresh rank
processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* on 127.0.0.1), and exits
with the first failing rank's code.  Every rank checks the world size and that
its device is distinct from the others'.

Window.  After the keyed placement: W warm-up steps, a timed K-step window
from the fresh placement (ms_per_step_fresh), E untimed evolution steps
toward the bond-rich steady state the reference simulates for 2e7 steps, W
warm-up steps with every kernel bracketed (per-kernel breakdown, dominant
kernel), then THE timed window of exactly K steps (barrier + device sync on
both sides, max over ranks) that `value` and `ms_per_step` report.

Rank 0 prints ONE JSON line:
  value        particle-updates/s over all ranks = N_gpus · particles · K / t
  roofline     the dominant kernel's algorithmic HBM bytes per launch ÷ its
               average duration (HIP events on the engine's stream over the
               timed region); peak 8 TB/s (MI355X HBM3E)
  cpu_baseline the keyed CPU oracle, one pinned core, on a bounded sample of
               the same state (rank 0 at N = 1 only), plus an ensemble of one
               oracle per core and the C1 link to the unmodified reference
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
PKG = "kmc-with-a-diffusion-reaction-algorithm_amd"
workloads = importlib.import_module(PKG + ".workloads")

TIMING_EVERY = 8
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md
METRIC = "KMC particle-updates/sec (and steps/sec) at 1e6 particles, 1/2/4/8 MI355X"
MAX_CPU_WORKERS = 16  # the GPU box's CPU share for one GPU


def kernel_bytes(name: str, n_a: int, n_b: int):
    """Algorithmic HBM bytes per launch."""
    n = n_a + n_b
    models = {
        # the proposal phase (PROPOSE_PHASE): every protein's R read (16
        # receptor / 8 ligand beads × xyz × 8 B) and R_new written, its unit
        # kind and home position read, its two 32-byte records written
        "k_propose": 768 * n_a + 384 * n_b + n + 8 * n + 64 * n,
        # every record once (float4 + id + site)
        "k_pair_scan": 2 * n * 32,
        "k_classify": 20 * n_a + 12 * n_b + 5 * n,
        "k_observe": 16 * n_a + 5 * n_b,
    }
    return models.get(name)


TRAFFIC_JSON = "profiles/traffic_C3.json"
# wave64 VALU instructions per launch (SQ_INSTS_VALU) from the committed SQ
# pass of the same steady-state profile (profiles/r06/final_C3/pmc_summary.txt)
VALU_JSON = "profiles/valu_C3.json"
# VALU issue ceiling: 256 CUs × 4 SIMDs, one wave64 instruction per SIMD every
# 4 cycles (16 lanes wide) at 2.4 GHz (MI355X_MICROARCH.md: max clock)
VALU_ISSUE_PEAK = 256 * 4 * 2.4e9 / 4


# the proposal phase the engine brackets as "k_propose" (kmc_engine.hip
# launch_step): these kernels back to back on the engine's stream
PROPOSE_PHASE = ("k_bfs", "k_propose_free", "k_move_members", "k_cx_check", "k_complex_heavy")
# single kernels reported beside the phase: the largest one of
# the step (HBM-bound, judged by its counter traffic: its algorithmic bytes
# depend on how many proteins are in complexes) and the furthest below the
# roofline (issue-bound, judged by its algorithmic bytes)
DETAIL_KERNELS = ("k_propose_free", "k_pair_scan")


def pmc_traffic(kernel: str, workload: str):
    """HBM bytes per launch of `kernel` (the proposal phase: the sum over its
    kernels) from the committed rocprofv3 PMC passes (FETCH_SIZE + WRITE_SIZE,
    tools/pmc_traffic.py) of this same bench at the steady state
    (tools/gpu_steady_profile.sh); None when no profile of this workload is
    committed."""
    path = os.path.join(REPO, TRAFFIC_JSON)
    if workload != "C3" or not os.path.exists(path):
        return None
    t = json.load(open(path))
    names = PROPOSE_PHASE if kernel == "k_propose" else (kernel_trace_name(kernel),)
    recs = [t.get(n) for n in names]
    return sum(r["traffic_bytes"] for r in recs) if all(recs) else None


def pmc_valu(kernel: str, workload: str):
    """SQ_INSTS_VALU per launch of `kernel` from VALU_JSON (C3 only), or None."""
    path = os.path.join(REPO, VALU_JSON)
    if workload != "C3" or not os.path.exists(path):
        return None
    r = json.load(open(path)).get(kernel_trace_name(kernel))
    return r["SQ_INSTS_VALU"] if r else None


def kernel_trace_name(name: str) -> str:
    # engine timing names -> the kernel symbol rocprof reports
    return name


def parse(argv):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", default="C3", choices=sorted(workloads.WORKLOADS))
    ap.add_argument("--evolve", type=int, default=None,
                    help="untimed steps before the timed window (default: the workload's, C3 20000)")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-baseline-steps", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-fresh-window", action="store_true")
    ap.add_argument("--save-state", default="", help="write the exact state after the evolution (KMCSTAT1)")
    ap.add_argument("--load-state", default="",
                    help="start from an exact state file instead of placement + fresh window + evolution "
                         "(profiling the steady state without tracing the evolution)")
    ap.add_argument("--profile", action="store_true", help="print the per-kernel breakdown to stderr")
    ap.add_argument("--launcher-check", action="store_true",
                    help="ranks rendezvous over gloo and report who they are; no GPU work (launcher test)")
    return ap.parse_args(argv)


# ---------------------------------------------------------------- launcher
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def visible_devices() -> int:
    """GPU count, asked in a child process so this launcher never touches HIP."""
    r = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                       capture_output=True, text=True)
    try:
        return int(r.stdout.strip().splitlines()[-1])
    except (ValueError, IndexError):
        return 0


def shared_device() -> bool:
    """KMC_BENCH_SHARED_DEVICE=1 (tests only): every rank on device 0 and the
    gloo backend, so the N-rank path (launcher, rendezvous, max over ranks,
    ensemble reduction) runs on a one-GPU box (tests/test_gpu_bench_ranks.py).
    Refused outside a pytest run (PYTEST_CURRENT_TEST): N ranks sharing one
    GPU are not an N-GPU measurement.  The line then carries "value": null,
    "shared_device": true and the one-device rate as "value_shared_device"."""
    if os.environ.get("KMC_BENCH_SHARED_DEVICE") != "1":
        return False
    if not os.environ.get("PYTEST_CURRENT_TEST"):
        sys.exit("bench.py: KMC_BENCH_SHARED_DEVICE=1 is a test-only mode (every rank on one GPU); "
                 "refusing to report it as a measurement")
    return True


def launch(args, argv) -> int:
    n = args.gpus
    if not args.launcher_check:
        ndev = visible_devices()
        if ndev < (1 if shared_device() else n):
            print(f"bench.py: --gpus {n} needs {n} visible GPUs, found {ndev}; refusing to measure fewer",
                  file=sys.stderr, flush=True)
            return 2
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__), *argv], env=env))
    rc = 0
    alive = set(range(n))
    while alive:
        for r in sorted(alive):
            c = procs[r].poll()
            if c is None:
                continue
            alive.discard(r)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 1
                print(f"bench.py: rank {r} exited with {c}; stopping the other ranks", file=sys.stderr, flush=True)
                for q in alive:
                    procs[q].terminate()
        time.sleep(0.1)
    return rc


def launcher_check(rank: int, world: int, local: int):
    import torch.distributed as dist

    dist.init_process_group("gloo")
    assert dist.get_world_size() == world
    who = [None] * world
    dist.all_gather_object(who, {"rank": rank, "local_rank": local, "pid": os.getpid()})
    if rank == 0:
        print(json.dumps({"launcher_check": True, "world": world, "ranks": who}), flush=True)
    dist.destroy_process_group()


# ---------------------------------------------------------------- one rank
def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch(args, argv))
    world = int(env_world or "1")
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.launcher_check:
        launcher_check(rank, world, local)
        return
    run_rank(args, rank, world, local)


def run_rank(args, rank: int, world: int, local: int):
    # stdout carries exactly one JSON line: native libraries (RCCL prints its
    # version banner to stdout at communicator init) write to stderr instead
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    import torch
    import torch.distributed as dist

    engine = importlib.import_module(PKG + ".engine")
    ensemble = importlib.import_module(PKG + ".ensemble")
    # a diagnostic library (KMC_DIAG=1 KMC_LIB_PATH=..., capi.py) is named in the line
    library = os.path.relpath(engine.load_library()._name, REPO)

    # RCCL (backend "nccl") at every world size: at N = 1 the ensemble
    # reduction below runs the same device-tensor all-reduce path as on 8 GPUs
    shared = shared_device()
    if shared:
        local = 0
    torch.cuda.set_device(local)
    if shared:
        dist.init_process_group("gloo")
    elif world == 1 and "MASTER_ADDR" not in os.environ:
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                                device_id=torch.device("cuda", local))
    else:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    if dist.get_world_size() != world:
        sys.exit(f"bench.py: process group has {dist.get_world_size()} ranks, expected {world}")
    if world > 1 and not shared:
        props = torch.cuda.get_device_properties(local)
        me = str(getattr(props, "uuid", "")) or f"{props.name}:{local}"
        devs = [None] * world
        dist.all_gather_object(devs, me)
        if len(set(devs)) != world:
            sys.exit(f"bench.py: ranks share a device: {devs}")
    dev = torch.device("cuda", local)

    w = workloads.WORKLOADS[args.workload]
    evolve = w["evolve"] if args.evolve is None else args.evolve
    p = workloads.params(args.workload, seed=args.seed, replica=rank)
    n = p.n_a + p.n_b
    sim = engine.Simulation(p, device=local)
    t0 = time.perf_counter()
    if args.load_state:
        sim.load_state(args.load_state)
        args.no_fresh_window = True
        evolve = 0
    else:
        sim.init_random()
    t_init = time.perf_counter() - t0

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    last_obs = {}

    reducer = ensemble.Reducer(args.steps, device=None if shared else dev)
    obs_dtype = importlib.import_module(PKG + ".capi").OBS_DTYPE

    def timed(k):
        # the communicator and the reduction's buffers were last used before
        # the evolution (seconds ago): one untimed reduction of a dummy window
        # first, so that the timed one costs what it costs between batches
        reducer.reduce(np.zeros(k, dtype=obs_dtype))
        barrier()
        t = time.perf_counter()
        obs = sim.step(k)
        t_steps = time.perf_counter()
        red = reducer.reduce(obs)
        barrier()
        t_end = time.perf_counter()
        last_obs["obs"] = obs
        last_obs["split_ms"] = {"steps": (t_steps - t) * 1e3, "reduce_and_barrier": (t_end - t_steps) * 1e3}
        return t_end - t, red

    def max_over_ranks(x):
        if world == 1:
            return x, [x]
        allx = [None] * world
        dist.all_gather_object(allx, x)
        return max(allx), allx

    # fresh placement window (bonds ~0: the early transient)
    fresh_ms = None
    if not args.no_fresh_window:
        if args.warmup:
            sim.step(args.warmup)
        dt_f, _ = timed(args.steps)
        fresh_ms = max_over_ranks(dt_f)[0] / args.steps * 1e3
    # evolution toward the steady state (untimed)
    t0 = time.perf_counter()
    chunk = 5000
    done = 0
    while done < evolve:
        k = min(chunk, evolve - done)
        ob = sim.step(k)
        done += k
        if rank == 0:
            print(f"bench: evolved {done}/{evolve} steps, bond_num {int(ob[-1]['bond_num'])}", file=sys.stderr,
                  flush=True)
    t_evolve = time.perf_counter() - t0
    if args.save_state:
        sim.save_state(args.save_state)

    # warm-up with every kernel bracketed: find the dominant kernel
    sim.set_timing(engine.kernel_names())
    if args.warmup:
        sim.step(args.warmup)
    kt = sim.kernel_times()
    dom = max(kt, key=lambda k: kt[k][0]) if kt else "k_propose"
    breakdown = {k: round(v[0] / max(v[1], 1), 4) for k, v in sorted(kt.items(), key=lambda x: -x[1][0])}
    # timed region: only the dominant kernel is bracketed, in every 8th step
    # (an event pair adds a few microseconds of queue time to its step)
    sim.set_timing([dom, *[k for k in DETAIL_KERNELS if k != dom]], every=TIMING_EVERY)
    dt_local, (sums, maxima, cluster) = timed(args.steps)
    dt, per_rank = max_over_ranks(dt_local)

    # what the all-reduce did: at N = 1 the reduced series must equal this
    # rank's own observables (the same RCCL call the N-GPU run makes)
    own_s, own_m = ensemble.pack(last_obs["obs"])
    reduce_info = {"backend": dist.get_backend(), "device": "cpu" if shared else str(dev), "world": world,
                   "shared_device": shared,
                   "ops": ["all_reduce SUM int64[K,6]", "all_reduce MAX int64[K,1]"], "steps_reduced": args.steps}
    if world == 1:
        reduce_info["equals_local"] = bool((sums == own_s).all() and (maxima == own_m).all())

    ktimed = sim.kernel_times()
    total_ms, launches = ktimed.get(dom, (0.0, 0))
    avg_s = total_ms / 1e3 / max(launches, 1)
    detail = {}
    for k in DETAIL_KERNELS:
        ms, nl = ktimed.get(k, (0.0, 0))
        if not nl:
            continue
        a_s = ms / 1e3 / nl
        kb_k = kernel_bytes(k, p.n_a, p.n_b)
        tr_k = pmc_traffic(k, args.workload)
        detail[k] = {
            "avg_launch_ms": a_s * 1e3,
            "bytes_per_launch": kb_k,
            "achieved": (kb_k / a_s / 1e9) if kb_k else None,
            "frac": (kb_k / a_s / 1e9 / HBM_PEAK_GBS) if kb_k else None,
            "traffic": tr_k,
            "achieved_by_traffic": (tr_k / a_s / 1e9) if tr_k else None,
            "frac_by_traffic": (tr_k / a_s / 1e9 / HBM_PEAK_GBS) if tr_k else None,
        }
        valu = pmc_valu(k, args.workload)
        if valu:
            # the issue-bound view (the pair walk: VALU-issue-bound, not HBM)
            detail[k]["valu_per_launch"] = valu
            detail[k]["valu_issue_ms"] = valu / VALU_ISSUE_PEAK * 1e3
            detail[k]["frac_of_valu_issue"] = valu / VALU_ISSUE_PEAK / a_s
    kb = kernel_bytes(dom, p.n_a, p.n_b)
    achieved = (kb / avg_s / 1e9) if (kb and avg_s > 0) else None
    traffic = pmc_traffic(dom, args.workload)
    step_b = workloads.step_bytes(p.n_a, p.n_b)
    ms_per_step = dt / args.steps * 1e3

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        steps = args.cpu_baseline_steps or w["cpu_sample_steps"]
        cpu = cpu_baseline(args.workload, args.seed, sim, steps, w.get("cpu_ensemble_max", MAX_CPU_WORKERS))

    if args.profile and rank == 0:
        print(json.dumps({"init_s": round(t_init, 3), "evolve_s": round(t_evolve, 3), "per_launch_ms": breakdown}),
              file=sys.stderr)

    if rank == 0:
        rate = world * n * args.steps / dt
        line = {
            "metric": METRIC,
            "value": None if shared else rate,
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
                "evolve_steps": evolve,
                "start_state": args.load_state or "keyed placement",
                "timed_from_step": sim.current_step - args.steps,
                "ms_per_step_fresh": fresh_ms,
                "per_rank_ms_per_step": [x / args.steps * 1e3 for x in per_rank],
                "window_split_ms": last_obs["split_ms"],
                "efficiency_vs_rank0": per_rank[0] / dt,
                "final_bond_num_ensemble": int(sums[-1, 3]),
                "final_rl_ensemble": int(sums[-1, 0]),
                "max_complex_ensemble": int(maxima[-1, 0]),
                "mean_cluster_size_ensemble": float(cluster[-1]),
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
                "kernels": list(PROPOSE_PHASE) if dom == "k_propose" else [kernel_trace_name(dom)],
                "bytes_per_launch": kb,
                "avg_launch_ms": avg_s * 1e3,
                "step_bytes": step_b,
                "step_frac": step_b / (ms_per_step / 1e3) / 1e9 / HBM_PEAK_GBS,
                "by_kernel": detail,
            },
            "cpu_baseline": cpu,
            "ensemble_reduce": reduce_info,
            "library": library,
        }
        if shared:
            # every rank on one device (test mode): not an N-GPU throughput
            line["shared_device"] = True
            line["value_shared_device"] = rate
        os.write(json_fd, (json.dumps(line) + "\n").encode())
    sim.close()
    dist.destroy_process_group()


# ---------------------------------------------------------------- CPU baseline
def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return ""


def _workers(jobs):
    """Run oracle/cpu_worker.py jobs concurrently (fresh processes, no GPU);
    returns their JSON results."""
    script = os.path.join(REPO, "oracle", "cpu_worker.py")
    procs = [subprocess.Popen([sys.executable, script, *j], stdout=subprocess.PIPE, text=True) for j in jobs]
    out = []
    for pr in procs:
        so, _ = pr.communicate()
        if pr.returncode != 0:
            raise RuntimeError(f"cpu_worker failed ({pr.returncode})")
        out.append(json.loads(so.strip().splitlines()[-1]))
    return out


def cpu_baseline(workload: str, seed: int, sim, steps: int, ens_max: int):
    """Keyed CPU oracle (oracle/cpu_worker.py), each worker pinned to one core,
    on the exact state the GPU run ended in; plus one worker per core
    (ensemble) and the C1 conversion to the unmodified reference."""
    cores = sorted(os.sched_getaffinity(0))
    nens = min(len(cores), MAX_CPU_WORKERS, ens_max)
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "state.kmc")
        sim.save_state(path)
        base = ["--workload", workload, "--seed", str(seed), "--state", path, "--steps", str(steps)]
        single = _workers([base + ["--core", str(cores[0])]])[0]
        ens = _workers([base + ["--core", str(c)] for c in cores[:nens]]) if nens > 1 else [single]
    c1_steps = 2000
    c1 = _workers([["--workload", "C1", "--seed", "1", "--steps", str(c1_steps), "--core", str(cores[0])]])[0]
    link = None
    lpath = os.path.join(REPO, "profiles", "cpu_link_C1.json")
    if os.path.exists(lpath):
        L = json.load(open(lpath))
        ratio = L["ratio_reference_over_oracle_cells"]
        link = {
            "oracle_C1_steps_per_s_here": c1["steps_per_s"],
            "ratio_reference_over_oracle": ratio,
            "ratio_source": "profiles/cpu_link_C1.json (tools/cpu_link.py; reference C1 rate from BASELINE.md)",
            "reference_equiv_C1_steps_per_s": c1["steps_per_s"] * ratio,
            "reference_equiv_C1_particle_updates_per_s": c1["steps_per_s"] * ratio * 2000,
        }
    return {
        "value": single["particle_updates_per_s"],
        "unit": "particle-updates/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{steps} steps of the same workload from the state the GPU run ended in, keyed oracle "
                  f"(cell-list mode), one pinned core",
        "host_cores": os.cpu_count(),
        "host_cores_usable": len(cores),
        "host_cpu": _cpu_model(),
        "ensemble": {"value": sum(e["particle_updates_per_s"] for e in ens), "processes": len(ens),
                     "unit": "particle-updates/s",
                     "sample": f"one oracle process per usable core (at most {nens}), each pinned, same sample"},
        "reference_link": link,
    }


if __name__ == "__main__":
    main()
