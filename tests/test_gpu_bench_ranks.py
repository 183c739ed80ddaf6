"""The N-rank measurement path of bench.py, executed end to end on one GPU
(VERDICT r03 "next" 2): `bench.py --gpus 2` as a GPU-free launcher starting
two rank processes, their rendezvous, the per-rank replicas (key = (seed,
rank)), the max over ranks of the timed windows and the ensemble reduction of
the bond.dat observables (main.cpp:2247-2253) — the code the 8-GPU C4 run
takes, with KMC_BENCH_SHARED_DEVICE=1 putting both ranks on device 0 over gloo
(RCCL refuses two ranks on one device).  The ensemble's final bond count must
equal the sum of two keyed-oracle runs of replicas 0 and 1."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from _kmc import O, REPO, engine, workloads

pytestmark = pytest.mark.gpu

WARMUP, STEPS, EVOLVE = 5, 20, 1000


@pytest.mark.timeout(300)
def test_bench_two_ranks_shared_device_equals_oracle_replicas():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["KMC_BENCH_SHARED_DEVICE"] = "1"
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--workload", "C1",
                        "--steps", str(STEPS), "--warmup", str(WARMUP), "--evolve", str(EVOLVE),
                        "--no-cpu-baseline"], capture_output=True, text=True, env=env, timeout=280)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [x for x in r.stdout.splitlines() if x.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2
    red = d["ensemble_reduce"]
    assert red["world"] == 2 and red["shared_device"] and red["backend"] == "gloo"
    cfg = d["config"]
    assert len(cfg["per_rank_ms_per_step"]) == 2
    assert d["ms_per_step"] == pytest.approx(max(cfg["per_rank_ms_per_step"]))
    # each rank: placement, W warm-up, K fresh, E evolved, W warm-up, K timed
    total = 2 * WARMUP + 2 * STEPS + EVOLVE
    assert cfg["timed_from_step"] + STEPS == total
    bonds, rl, cmax = 0, 0, 0
    for rank in range(2):
        p = workloads.params("C1", seed=1, replica=rank)
        o = O.Oracle(p, rng_mode=O.RNG_KEYED, nbmode=O.NB_CELLS)
        o.set_state(engine.host_init_random(p))
        obs, _ = o.step(total, want_hashes=False)
        bonds += int(obs[-1]["bond_num"])
        rl += int(obs[-1]["bond_num_rl"])
        cmax = max(cmax, int(obs[-1]["protein_num_in_max_complex"]))
    assert bonds > 0
    assert cfg["final_bond_num_ensemble"] == bonds
    assert cfg["final_rl_ensemble"] == rl
    assert cfg["max_complex_ensemble"] == cmax
    n = cfg["particles_per_gpu"]
    # both ranks on one device: the line refuses to call that an N-GPU value
    assert d["value"] is None and d["shared_device"] is True
    assert d["value_shared_device"] == pytest.approx(2 * n * STEPS / (d["ms_per_step"] * STEPS / 1e3), rel=1e-9)
