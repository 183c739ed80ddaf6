"""ctypes mirror of include/kmc.h (the C-ABI of libkmc).

Struct layouts here must match include/kmc.h field for field; the
`tests/test_host.py::test_ctypes_layouts_match_header` CPU test checks sizes/offsets against the compiled
library.  Nothing in this module computes anything: it only marshals host
buffers (numpy arrays) across the C boundary.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# KMC_LIB_PATH: diagnostic builds only (e.g. the -DKMC_STAMPS timing build, the
# A/B variants of tools/build_variants.py).  It is honoured only together with
# KMC_DIAG=1, so a stray variable cannot make tests or benchmarks load a
# library other than the in-tree build.
if os.environ.get("KMC_LIB_PATH") and os.environ.get("KMC_DIAG") != "1":
    raise RuntimeError("KMC_LIB_PATH is set without KMC_DIAG=1: refusing to load a non-default libkmc")
LIB_PATH = os.environ.get("KMC_LIB_PATH") or os.path.join(HERE, "lib", "libkmc.so")

KMC_OK = 0
ERRORS = {
    -1: "KMC_ERR_ARG",
    -2: "KMC_ERR_IO",
    -3: "KMC_ERR_FORMAT",
    -4: "KMC_ERR_STATE",
    -5: "KMC_ERR_PLACEMENT",
    -6: "KMC_ERR_CAPACITY",
    -7: "KMC_ERR_HIP",
    -8: "KMC_ERR_GEOMETRY",
    -9: "KMC_ERR_NODEVICE",
}
# KMC_ERR_* as module constants (ERR_ARG = -1, ...)
globals().update({name[4:]: code for code, name in ERRORS.items()})


class Params(C.Structure):
    """kmc_params — reference globals main.cpp:39-99 as a runtime struct."""

    _fields_ = [
        ("n_a", C.c_int32),
        ("n_b", C.c_int32),
        ("time_step", C.c_double),
        ("box_x", C.c_double),
        ("box_y", C.c_double),
        ("box_z", C.c_double),
        ("pai", C.c_double),
        ("ra_radius", C.c_double),
        ("ra_D", C.c_double),
        ("ra_rot_D", C.c_double),
        ("rb_radius", C.c_double),
        ("rb_D", C.c_double),
        ("rb_rot_D", C.c_double),
        ("mono_cis_ass_rate", C.c_double),
        ("mono_cis_diss_rate", C.c_double),
        ("cis_D", C.c_double),
        ("cis_rot_D", C.c_double),
        ("cis_ass_rate", C.c_double),
        ("cis_diss_rate", C.c_double),
        ("bond_D", C.c_double),
        ("bond_rot_D", C.c_double),
        ("ass_rate", C.c_double),
        ("diss_rate", C.c_double),
        ("bond_dist_cutoff", C.c_double),
        ("bond_thetapd_cutoff", C.c_double),
        ("bond_thetaot_cutoff", C.c_double),
        ("cis_thetaot_cutoff", C.c_double),
        ("cis_dist_cutoff", C.c_double),
        ("simu_step", C.c_int64),
        ("out_interval", C.c_int32),
        ("reserved0", C.c_int32),
        ("seed", C.c_uint64),
        ("replica", C.c_uint32),
        ("reserved1", C.c_int32),
    ]


class Obs(C.Structure):
    """kmc_obs — one bond.dat record (main.cpp:2251) + raw cluster sums."""

    _fields_ = [
        ("step", C.c_int64),
        ("t", C.c_double),
        ("bond_num_rl", C.c_int32),
        ("bond_num_mono_cis", C.c_int32),
        ("bond_num_cis", C.c_int32),
        ("bond_num", C.c_int32),
        ("cluster_size", C.c_double),
        ("protein_num_in_max_complex", C.c_int32),
        ("tot_proteins_in_cluster", C.c_int32),
        ("tot_cluster_num", C.c_int32),
        ("reserved", C.c_int32),
    ]


OBS_DTYPE = np.dtype(
    [
        ("step", "<i8"),
        ("t", "<f8"),
        ("bond_num_rl", "<i4"),
        ("bond_num_mono_cis", "<i4"),
        ("bond_num_cis", "<i4"),
        ("bond_num", "<i4"),
        ("cluster_size", "<f8"),
        ("protein_num_in_max_complex", "<i4"),
        ("tot_proteins_in_cluster", "<i4"),
        ("tot_cluster_num", "<i4"),
        ("reserved", "<i4"),
    ]
)
assert OBS_DTYPE.itemsize == C.sizeof(Obs)


class StateView(C.Structure):
    """kmc_state_view — host SoA buffers, reference bead order (kmc.h)."""

    _fields_ = [
        ("ra", C.POINTER(C.c_double)),
        ("rb", C.POINTER(C.c_double)),
        ("a_int", C.POINTER(C.c_int32)),
        ("b_int", C.POINTER(C.c_int32)),
        ("counters", C.c_int32 * 5),
        ("reserved", C.c_int32),
        ("step", C.c_int64),
    ]


DD_ROW = 416     # KMC_DD_ROW: one exchanged protein (48 doubles + 8 int32)
DD_JCAP = 256    # KMC_DD_JCAP
DD_XCAP = 64     # KMC_DD_XCAP


class DDReport(C.Structure):
    """kmc_dd_report — one slab window's checks after a step's halo exchange."""

    _fields_ = [
        ("xcol", C.c_int64),
        ("xbond", C.c_int64),
        ("bad", C.c_int32),
        ("differed", C.c_int32),
        ("links", C.c_int32),
        ("n_jump", C.c_int32),
        ("n_xb", C.c_int32),
        ("reserved", C.c_int32),
        ("jump_id", C.c_int32 * DD_JCAP),
        ("jump_x", C.c_double * DD_JCAP),
        ("xb", (C.c_int32 * 2) * DD_XCAP),
    ]

    def jumpers(self):
        """(local ids, x) of the listed jumpers."""
        n = min(self.n_jump, DD_JCAP)
        return (np.ctypeslib.as_array(self.jump_id)[:n].copy(), np.ctypeslib.as_array(self.jump_x)[:n].copy())

    def cross_bonds(self) -> np.ndarray:
        """[n, 2] local ids of the listed cross-slab bonds."""
        n = min(self.n_xb, DD_XCAP)
        return np.ctypeslib.as_array(self.xb).reshape(DD_XCAP, 2)[:n].copy()


def default_params(**overrides) -> Params:
    """Reference defaults, main.cpp:39-99 (mirrors kmc_params_default)."""
    p = Params()
    p.n_a, p.n_b = 150, 50
    p.time_step = 10.0
    p.box_x, p.box_y, p.box_z = 5773.0, 5773.0, 1000.0
    p.pai = 3.1415926
    p.ra_radius, p.ra_D, p.ra_rot_D = 20.0, 1.0, 0.0174
    p.rb_radius, p.rb_D, p.rb_rot_D = 30.0, 7.2614, 0.0061209
    p.mono_cis_ass_rate, p.mono_cis_diss_rate = 0.000047, 0.000000000000112
    p.cis_D, p.cis_rot_D, p.cis_ass_rate, p.cis_diss_rate = 0.5, 0.005, 0.00096, 0.000000000000112
    p.bond_D, p.bond_rot_D, p.ass_rate, p.diss_rate = 0.5, 0.005, 0.04, 0.000000000000348
    p.bond_dist_cutoff = 18.0
    p.bond_thetapd_cutoff = 45.0
    p.bond_thetaot_cutoff = 90.0
    p.cis_thetaot_cutoff = 10.0
    p.cis_dist_cutoff = 15.0
    p.simu_step = 20000000
    p.out_interval = 5000
    p.seed = 1
    p.replica = 0
    for k, v in overrides.items():
        if not hasattr(p, k):
            raise AttributeError(k)
        setattr(p, k, v)
    return p


class HostState:
    """numpy-backed kmc_state_view for n_a receptors and n_b ligands."""

    def __init__(self, n_a: int, n_b: int):
        self.n_a, self.n_b = n_a, n_b
        self.ra = np.zeros((48, n_a), dtype=np.float64)
        self.rb = np.zeros((24, n_b), dtype=np.float64)
        self.a_int = np.zeros((5, n_a), dtype=np.int32)
        self.b_int = np.zeros((8, n_b), dtype=np.int32)
        self.counters = np.zeros(5, dtype=np.int32)
        self.step = 0

    def view(self) -> StateView:
        v = StateView()
        v.ra = self.ra.ctypes.data_as(C.POINTER(C.c_double))
        v.rb = self.rb.ctypes.data_as(C.POINTER(C.c_double))
        v.a_int = self.a_int.ctypes.data_as(C.POINTER(C.c_int32))
        v.b_int = self.b_int.ctypes.data_as(C.POINTER(C.c_int32))
        for i in range(5):
            v.counters[i] = int(self.counters[i])
        v.step = int(self.step)
        return v

    def pull(self, v: StateView) -> None:
        self.counters[:] = list(v.counters)
        self.step = int(v.step)

    def copy(self) -> "HostState":
        h = HostState(self.n_a, self.n_b)
        h.ra[:] = self.ra
        h.rb[:] = self.rb
        h.a_int[:] = self.a_int
        h.b_int[:] = self.b_int
        h.counters[:] = self.counters
        h.step = self.step
        return h

    def equal(self, other: "HostState") -> bool:
        """Bitwise equality (coordinates compared as IEEE bit patterns)."""
        return (
            np.array_equal(self.ra.view(np.uint64), other.ra.view(np.uint64))
            and np.array_equal(self.rb.view(np.uint64), other.rb.view(np.uint64))
            and np.array_equal(self.a_int, other.a_int)
            and np.array_equal(self.b_int, other.b_int)
            and np.array_equal(self.counters, other.counters)
            and self.step == other.step
        )


def _fnv_bytes(h: int, data: bytes) -> int:
    for c in data:
        h ^= c
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h
