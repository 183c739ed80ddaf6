"""Link the keyed CPU oracle to the reference's own CPU speed at C1.

BASELINE.md's C1 row is the UNMODIFIED reference main.cpp (1e3 + 1e3
proteins, reference box, time-seeded rand2, 1e4 steps) at 3.861 steps/s on
one core of this container type (g++ 11.4 -O2).  The reference's sizes are
#defines (main.cpp:47-69) and its rand2 cannot be seeded, so it cannot run
the benchmark configurations; bench.py therefore times the keyed oracle on
the GPU box and converts with the ratio measured here:

    ratio = reference steps/s at C1 / oracle (cell-list mode) steps/s at C1

Usage (this container, one pinned core):
    taskset -c 5 python tools/cpu_link.py [steps]   -> profiles/cpu_link_C1.json
"""
from __future__ import annotations

import importlib
import json
import os
import platform
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "oracle")]
import oracle as O  # noqa: E402

W = importlib.import_module("kmc-with-a-diffusion-reaction-algorithm_amd.workloads")
E = importlib.import_module("kmc-with-a-diffusion-reaction-algorithm_amd.engine")

REF_C1_STEPS_PER_S = 3.861  # BASELINE.md, unmodified main.cpp at C1 (2589.9 s for 1e4 steps incl. init)


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def time_oracle(steps: int, nbmode: int) -> dict:
    p = W.params("C1", seed=1)
    o = O.Oracle(p, rng_mode=O.RNG_KEYED, nbmode=nbmode)
    o.set_state(E.host_init_random(p))
    t = time.perf_counter()
    ob, _ = o.step(steps, want_hashes=False)
    dt = time.perf_counter() - t
    return {"steps": steps, "seconds": dt, "steps_per_s": steps / dt, "final_bond_num": int(ob[-1]["bond_num"])}


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    cells = time_oracle(steps, O.NB_CELLS)
    brute = time_oracle(max(steps // 20, 50), O.NB_BRUTE)
    out = {
        "workload": "C1: 1000 receptors + 1000 ligands, reference box 5773x5773x1000 A, seed 1",
        "host": {"cpu": cpu_model(), "cpu_count": os.cpu_count(), "pinned_cores": len(os.sched_getaffinity(0))},
        "reference_unmodified_steps_per_s": REF_C1_STEPS_PER_S,
        "reference_source": "BASELINE.md C1 row (unmodified main.cpp, 1 core, same container type)",
        "oracle_cells": cells,
        "oracle_brute": brute,
        "ratio_reference_over_oracle_cells": REF_C1_STEPS_PER_S / cells["steps_per_s"],
    }
    path = os.path.join(REPO, "profiles", "cpu_link_C1.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
