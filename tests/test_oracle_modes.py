"""Oracle self-consistency: neighbour modes, keyed placement, numerics KATs."""
import ctypes as C

import numpy as np
import pytest

from _kmc import DENSE, O, capi, engine, params


def test_brute_equals_cells_dense():
    p = params(seed=13, **DENSE)
    a = O.Oracle(p, nbmode=O.NB_BRUTE)
    b = O.Oracle(p, nbmode=O.NB_CELLS)
    a.init_placement()
    b.init_placement()
    oa, ha = a.step(400)
    ob, hb = b.step(400)
    assert np.array_equal(ha, hb) and np.array_equal(oa, ob)


@pytest.mark.parametrize("n_a,n_b,L", [(150, 50, 5773.0), (150, 50, 1000.0), (900, 400, 3000.0)])
def test_keyed_placement_oracle_equals_library(n_a, n_b, L):
    p = params(n_a=n_a, n_b=n_b, seed=77, box_x=L, box_y=L, box_z=300.0)
    o = O.Oracle(p)
    o.init_placement()
    assert engine.host_init_random(p).equal(o.get_state())


def test_philox_known_answers():
    L = O.lib()
    L.oracle_philox.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    kat = [  # Random123 philox4x32_10 known-answer vectors
        ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
        ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
        ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
         (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
    ]
    for ctr, key, want in kat:
        c = np.array(ctr, dtype=np.uint32)
        k = np.array(key, dtype=np.uint32)
        out = np.zeros(4, dtype=np.uint32)
        L.oracle_philox(c.ctypes.data, k.ctypes.data, out.ctypes.data)
        assert tuple(int(x) for x in out) == want


def test_glibc_rand_restatement_equals_libc():
    L = O.lib()
    L.oracle_glibc_rand.argtypes = [C.c_uint32, C.c_int, C.c_void_p]
    libc = C.CDLL(None)
    for seed in (1, 12345):
        out = np.zeros(20000, dtype=np.int32)
        L.oracle_glibc_rand(seed, out.size, out.ctypes.data)
        libc.srand(seed)
        ref = np.array([libc.rand() for _ in range(out.size)], dtype=np.int32)
        assert np.array_equal(out, ref)
    libc.srand(1)


OPS = {"sin": (0, np.sin), "cos": (1, np.cos), "atan2": (2, np.arctan2), "acos": (3, np.arccos)}


@pytest.mark.parametrize("name", list(OPS))
def test_portable_libm_within_one_ulp(name):
    op, ref = OPS[name]
    rng = np.random.default_rng(op)
    n = 200000
    x = rng.uniform(-1, 1, n) if name == "acos" else rng.uniform(-13.0, 13.0, n)
    y = rng.uniform(-13.0, 13.0, n)
    got = engine.math(op, x, y)
    want = ref(x, y) if name == "atan2" else ref(x)
    ulp = np.abs(got.view(np.int64) - want.view(np.int64))
    assert ulp.max() <= 1


def test_portable_libm_exact_points():
    z = np.array([0.0, -0.0])
    assert np.array_equal(engine.math(0, z).view(np.uint64), z.view(np.uint64))  # sin(±0) = ±0
    assert np.all(engine.math(1, z) == 1.0)
    assert engine.math(3, np.array([1.0]))[0] == 0.0
    r = engine.math(6, np.array([2.5, -2.5, 0.49999999999999994, -0.5, 1e17]))
    assert list(r) == [3.0, -3.0, 0.0, -1.0, 1e17]


BRUTE_CASES = [(4000, 1500), (20000, 7000)]


@pytest.mark.parametrize("n_a,n_b", BRUTE_CASES)
def test_cells_equal_brute_fixture_at_scale(n_a, n_b):
    # the cell-list oracle (the only CPU checker of the GPU at C2/C3/C5) equals
    # brute force — every pair tested, like main.cpp — step for step at
    # thousands of proteins; brute force is O(N^2), so its per-step hashes were
    # stored once (tests/golden/make_brute_cells.py)
    import os
    from _kmc import GOLDEN
    path = os.path.join(GOLDEN, f"brute_{n_a}_{n_b}.npz")
    if not os.path.exists(path):
        pytest.skip("fixture not generated")
    g = np.load(path, allow_pickle=False)
    L = float(g["box"])
    p = params(n_a=n_a, n_b=n_b, seed=int(g["seed"]), box_x=L, box_y=L, box_z=250.0,
               **{k: v for k, v in DENSE.items() if not k.startswith("box")})
    o = O.Oracle(p, nbmode=O.NB_CELLS)
    o.set_state(engine.host_init_random(p))
    obs, hashes = o.step(int(g["steps"]))
    assert np.array_equal(hashes, g["hashes"])
    assert np.array_equal(obs, g["obs"])
    assert obs[-1]["bond_num"] > 0


def test_c2_long_fixture_head_and_shape():
    # the committed C2 long-horizon fixture (tests/golden/c2_long.npz, 10^5
    # steps, replayed on the GPU by test_gpu_long.py) starts where the keyed
    # oracle starts today: its first 60 steps from the placement, records and
    # hashes; every step present once and in order
    import os

    import numpy as np

    from _kmc import GOLDEN, engine, workloads

    g = np.load(os.path.join(GOLDEN, "c2_long.npz"), allow_pickle=False)
    steps, every = int(g["steps"]), int(g["hash_every"])
    assert steps >= 100000 and len(g["obs"]) == steps and len(g["hashes"]) == steps // every
    assert np.array_equal(g["obs"]["step"], np.arange(1, steps + 1))
    p = workloads.params("C2", seed=int(g["seed"]))
    o = O.Oracle(p, rng_mode=O.RNG_KEYED, nbmode=O.NB_CELLS)
    o.set_state(engine.host_init_random(p))
    obs, _ = o.step(60, want_hashes=False)
    assert np.array_equal(obs, g["obs"][:60])
