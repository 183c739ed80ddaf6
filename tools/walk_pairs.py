"""Pairs the pair scan's walks visit per step (diagnostic: needs the
-DWALK_STATS=1 build, tools/build_variants.py walk=-DWALK_STATS=1, selected with
KMC_DIAG=1 KMC_LIB_PATH=ab_variants/libkmc_walk.so and KMC_DEBUG_COUNTS=1).
The workload is evolved E steps, then K steps are run in one call; the
library prints the running total after every call ("kmc walk pairs N").
  python -u tools/walk_pairs.py [workload] [E] [K]
"""
import importlib
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
PKG = "kmc-with-a-diffusion-reaction-algorithm_amd"
engine = importlib.import_module(PKG + ".engine")
workloads = importlib.import_module(PKG + ".workloads")

wl = sys.argv[1] if len(sys.argv) > 1 else "C3"
E = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
K = int(sys.argv[3]) if len(sys.argv) > 3 else 20
p = workloads.params(wl, seed=1)
with engine.Simulation(p) as sim:
    sim.init_random()
    sim.step(E)
    print(f"--- {wl}: evolved {E} steps; the next call runs {K} steps", file=sys.stderr, flush=True)
    sim.step(K)
