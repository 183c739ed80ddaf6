"""GPU side of the C2 long-horizon fixture extension (VERDICT r03 "next" 5).

Runs C2 (75 000 + 25 000 proteins, seed 1) on the GPU from the keyed placement,
checks every step's bond.dat record and every 100th full-state hash against the
committed oracle fixture (tests/golden/c2_long.npz) for as long as it reaches,
and writes the exact state (KMCSTAT1, xz-compressed) at the requested steps into
OUTDIR.  These states are only *starting points* for further oracle segments
(tests/golden/make_c2_long.py --start-state): each segment is accepted only if
the oracle's own state at the segment's end is byte-identical to the next
checkpoint (tests/golden/merge_c2_segments.py), so every step of the extended
fixture is computed by the oracle.

Usage: python tools/c2_checkpoints.py OUTDIR STEP [STEP ...]
"""
from __future__ import annotations

import importlib
import lzma
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
engine = importlib.import_module("kmc-with-a-diffusion-reaction-algorithm_amd.engine")
workloads = importlib.import_module("kmc-with-a-diffusion-reaction-algorithm_amd.workloads")


def main():
    out = sys.argv[1]
    marks = sorted(int(s) for s in sys.argv[2:])
    os.makedirs(out, exist_ok=True)
    g = np.load(os.path.join(REPO, "tests", "golden", "c2_long.npz"), allow_pickle=False)
    gsteps, every = int(g["steps"]), int(g["hash_every"])
    p = workloads.params("C2", seed=int(g["seed"]))
    sim = engine.Simulation(p)
    sim.set_state(engine.host_init_random(p))
    t0 = time.time()
    done = 0
    while done < marks[-1]:
        obs = sim.step(every)
        if done + every <= gsteps:
            ref = g["obs"][done:done + every]
            if not np.array_equal(obs, ref):
                raise SystemExit(f"fixture mismatch in steps {done + 1}..{done + every}")
            h = engine.state_hash(p, sim.get_state())
            if h != int(g["hashes"][done // every]):
                raise SystemExit(f"fixture hash mismatch at step {done + every}")
        done += every
        if done in marks:
            path = os.path.join(out, f"c2_{done}.kst")
            sim.save_state(path)
            with open(path, "rb") as f:
                raw = f.read()
            with open(path + ".xz", "wb") as f:
                f.write(lzma.compress(raw, preset=6))
            os.remove(path)
            print(f"step {done}: saved {path}.xz ({os.path.getsize(path + '.xz')} bytes), "
                  f"bonds {int(obs[-1]['bond_num'])}, {time.time() - t0:.0f}s", flush=True)
        elif done % 10000 == 0:
            print(f"step {done} bonds {int(obs[-1]['bond_num'])} {time.time() - t0:.0f}s", flush=True)
    print(f"fixture checked through step {min(gsteps, done)}", flush=True)


if __name__ == "__main__":
    main()
