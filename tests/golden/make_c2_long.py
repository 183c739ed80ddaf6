"""Generate tests/golden/c2_long.npz: a long-horizon C2 trajectory of the
keyed CPU oracle (VERDICT r01 "next" 8; BASELINE.json config 2: "1e5
particles, 1e5 steps, bit-exact state counts vs CPU").

C2 = 75 000 receptors + 25 000 ligands at the reference density
(workloads.py), seed 1, replica 0, reference physics (main.cpp:39-99), keyed
placement (kmc_host_init_random, identical to the oracle's placement).  The
oracle (cell-list mode) is advanced STEPS steps; stored:

  obs      every step's kmc_obs record (bond.dat columns, main.cpp:2251)
  hashes   FNV-1a hash of the full state (kmc_state_hash) every HASH_EVERY steps
  steps, hash_every, seed

The GPU test (tests/test_gpu_long.py) regenerates the same placement on the
host and replays the whole window.  Runs in this container (about an hour
per 10^4 steps, one thread; the committed fixture: `make_c2_long.py 40000` and four segments, below);
the result is data only.  The file is rewritten
(atomically) every SAVE_EVERY steps with the steps done so far, so a long run
(BASELINE.json C2: 10^5 steps) yields a usable, shorter fixture at any time.

Segments (10^5 steps in parallel, VERDICT r03 "next" 5):
  make_c2_long.py STEPS OUT --start-state S.kst --save-state E.kst
starts the oracle from the exact state S (KMCSTAT1, its step is the segment's
first step), advances it STEPS steps and saves its own exact final state E.
tests/golden/merge_c2_segments.py joins segments into one fixture, and accepts
a join only when the earlier segment's own final state is byte-identical to the
state the next segment started from, so every step of the joined fixture is
the oracle's and the joined run is the one continuous oracle run.

Usage: python tests/golden/make_c2_long.py [steps] [out] [--start-state S] [--save-state E]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
for p in (REPO, os.path.join(REPO, "oracle")):
    sys.path.insert(0, p)
import importlib  # noqa: E402

import oracle as O  # noqa: E402

engine = importlib.import_module("kmc-with-a-diffusion-reaction-algorithm_amd.engine")
workloads = importlib.import_module("kmc-with-a-diffusion-reaction-algorithm_amd.workloads")

HASH_EVERY = 100
SAVE_EVERY = 5000
OUT = os.path.join(HERE, "c2_long.npz")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("steps", type=int, nargs="?", default=10000)
    ap.add_argument("out", nargs="?", default=OUT)
    ap.add_argument("--start-state", default="")
    ap.add_argument("--save-state", default="")
    a = ap.parse_args()
    steps, out = a.steps, a.out
    p = workloads.params("C2", seed=1)
    st = engine.host_load_state(p, a.start_state) if a.start_state else engine.host_init_random(p)
    start = int(st.step)
    o = O.Oracle(p, rng_mode=O.RNG_KEYED, nbmode=O.NB_CELLS)
    o.set_state(st)
    obs = np.zeros(steps, dtype=O.capi.OBS_DTYPE)
    hashes = np.zeros(steps // HASH_EVERY, dtype=np.uint64)
    t0 = time.time()

    def save(done):
        tmp = out + ".tmp.npz"
        np.savez_compressed(tmp, obs=obs[:done], hashes=hashes[:done // HASH_EVERY], steps=done,
                            hash_every=HASH_EVERY, seed=1, start=start,
                            events=np.array(list(o.stats().values()), dtype=np.int64))
        os.replace(tmp, out)
        print("wrote", out, done, o.stats(), flush=True)

    for c in range(steps // HASH_EVERY):
        ob, _ = o.step(HASH_EVERY, want_hashes=False)
        obs[c * HASH_EVERY:(c + 1) * HASH_EVERY] = ob
        hashes[c] = o.hash()
        done = (c + 1) * HASH_EVERY
        if c % 10 == 9:
            print(f"step {start + done} bonds {ob[-1]['bond_num']} rl {ob[-1]['bond_num_rl']} "
                  f"{time.time() - t0:.0f}s", flush=True)
        if done % SAVE_EVERY == 0 or done == steps:
            save(done)
    if a.save_state:
        engine.host_save_state(p, o.get_state(), a.save_state)
        print("saved", a.save_state, "step", o.current_step, flush=True)


if __name__ == "__main__":
    main()
