"""Benchmark / parity configurations (BASELINE.json configs).

Every configuration uses the reference physics (main.cpp:40-99) and a
synthetic initial state from the keyed placement generator (the
reference's placement rules, main.cpp:281-447).  Box sizes scale the
reference default (150 + 50 proteins in 5773² × 1000 Å³) as SURVEY §8(d)
prescribes.
"""
from __future__ import annotations

import math

from . import capi

# algorithmic HBM bytes, SURVEY.md §8(d): every protein's fp64 state read once
# and written once (receptor 16 beads·3·8 B + 5 ints; ligand 8 beads·3·8 B +
# 8 ints) + 16 B of cell list per protein
def step_bytes(n_a: int, n_b: int) -> int:
    return 808 * n_a + 448 * n_b + 16 * (n_a + n_b)


WORKLOADS = {
    "C1": dict(n_a=1000, n_b=1000, L=5773.0, steps=10000, evolve=0, cpu_sample_steps=2000,
               desc="1e3 receptors + 1e3 ligands, reference box 5773x5773x1000 A"),
    "C2": dict(n_a=75000, n_b=25000, L=5773.0 * math.sqrt(100000 / 200), steps=100000, evolve=0, cpu_sample_steps=40,
               desc="1e5 particles (75000 A + 25000 B) at the reference density"),
    "C3": dict(n_a=750000, n_b=250000, L=5773.0 * math.sqrt(1000000 / 2000), steps=None, evolve=20000,
               cpu_sample_steps=4, desc="1e6 particles (750000 A + 250000 B), dense box (10x area density)"),
    "C5": dict(n_a=5000000, n_b=5000000, L=5773.0 * math.sqrt(5000000 / 1500), steps=None, evolve=20000,
               cpu_sample_steps=1, cpu_ensemble_max=4, desc="1e7 particles (5e6 A + 5e6 B), high ligand concentration"),
}


def params(name: str, seed: int = 1, replica: int = 0, **overrides) -> capi.Params:
    w = WORKLOADS[name]
    return capi.default_params(n_a=w["n_a"], n_b=w["n_b"], box_x=w["L"], box_y=w["L"], box_z=1000.0,
                               seed=seed, replica=replica, **overrides)
