"""Python host mirror of the reference's step-loop contract over libkmc.

The reference is one process that owns its state in globals and talks
through files (main.cpp:169-278, 2206-2305).  `Simulation` is the same
contract as an object: construct with the physics parameters (the
reference's compile-time globals, main.cpp:39-99), obtain an initial state
(random placement, main.cpp:281-447, or position.cpt, main.cpp:226-270),
advance the diffusion–reaction loop (main.cpp:461-2308) on the GPU, read the
bond.dat observables, write position.cpt.

Everything runs in libkmc (HIP kernels on gfx950); this module only
marshals host buffers.  There is no CPU fallback: if the library or a gfx950
device is missing, construction raises.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import numpy as np

from . import capi

_lib = None


class KmcError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{capi.ERRORS.get(code, code)}: {msg}")
        self.code = code


def load_library(path: Optional[str] = None):
    """Load libkmc.so (built in-tree by build.py).  Raises if absent."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or capi.LIB_PATH
    if not os.path.exists(path):
        raise KmcError(-9, f"{path} not built (run __graft_entry__.build())")
    L = C.CDLL(path)
    P = C.POINTER
    L.kmc_params_default.argtypes = [P(capi.Params)]
    L.kmc_create.argtypes = [P(capi.Params), C.c_int, P(C.c_void_p)]
    L.kmc_destroy.argtypes = [C.c_void_p]
    L.kmc_last_error.restype = C.c_char_p
    L.kmc_last_error.argtypes = [C.c_void_p]
    L.kmc_init_random.argtypes = [C.c_void_p]
    L.kmc_load_cpt.argtypes = [C.c_void_p, C.c_char_p]
    L.kmc_write_cpt.argtypes = [C.c_void_p, C.c_char_p]
    L.kmc_set_state.argtypes = [C.c_void_p, P(capi.StateView)]
    L.kmc_get_state.argtypes = [C.c_void_p, P(capi.StateView)]
    L.kmc_step.argtypes = [C.c_void_p, C.c_int64, C.c_void_p]
    L.kmc_current_step.restype = C.c_int64
    L.kmc_current_step.argtypes = [C.c_void_p]
    L.kmc_set_timing.argtypes = [C.c_void_p, C.c_uint64]
    L.kmc_set_timing_period.argtypes = [C.c_void_p, C.c_int32]
    L.kmc_kernel_times.argtypes = [C.c_void_p, P(C.c_double), P(C.c_int64), C.c_int32]
    L.kmc_kernel_name.restype = C.c_char_p
    L.kmc_kernel_name.argtypes = [C.c_int32]
    L.kmc_format_bond_line.argtypes = [P(capi.Params), P(capi.Obs), C.c_char_p, C.c_size_t]
    L.kmc_state_hash.restype = C.c_uint64
    L.kmc_state_hash.argtypes = [P(capi.Params), P(capi.StateView)]
    L.kmc_host_last_error.restype = C.c_char_p
    L.kmc_host_load_cpt.argtypes = [P(capi.Params), C.c_char_p, P(capi.StateView)]
    L.kmc_host_write_cpt.argtypes = [P(capi.Params), P(capi.StateView), C.c_char_p]
    L.kmc_host_init_random.argtypes = [P(capi.Params), P(capi.StateView)]
    L.kmc_host_validate.argtypes = [P(capi.Params), P(capi.StateView)]
    L.kmc_host_dd_check.argtypes = [C.c_int32, C.c_void_p, C.c_void_p]
    L.kmc_host_save_state.argtypes = [P(capi.Params), P(capi.StateView), C.c_char_p]
    L.kmc_host_load_state.argtypes = [P(capi.Params), C.c_char_p, P(capi.StateView)]
    L.kmc_save_state.argtypes = [C.c_void_p, C.c_char_p]
    L.kmc_load_state.argtypes = [C.c_void_p, C.c_char_p]
    L.kmc_get_clusters.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    L.kmc_host_write_parameter_log.argtypes = [P(capi.Params), C.c_char_p]
    L.kmc_host_append_gro.argtypes = [P(capi.Params), P(capi.StateView), C.c_char_p]
    L.kmc_host_append_cluster_log.argtypes = [P(capi.Params), C.c_int64, C.c_void_p, C.c_void_p, C.c_char_p]
    L.kmc_dd_set_state.argtypes = [C.c_void_p, P(capi.StateView), C.c_void_p, C.c_void_p, C.c_void_p]
    L.kmc_dd_export.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p]
    L.kmc_dd_import.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    L.kmc_dd_drift.argtypes = [C.c_void_p, P(C.c_double)]
    L.kmc_dd_counters.argtypes = [C.c_void_p, C.c_void_p]
    L.kmc_dd_jumpers.argtypes = [C.c_void_p, C.c_double, C.c_int32, C.c_void_p, C.c_void_p, P(C.c_int32)]
    L.kmc_dd_plan.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p]
    L.kmc_dd_pack.argtypes = [C.c_void_p, C.c_void_p]
    L.kmc_dd_send_buffer.restype = C.c_void_p
    L.kmc_dd_send_buffer.argtypes = [C.c_void_p]
    L.kmc_dd_unpack.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32]
    L.kmc_dd_finish.argtypes = [C.c_void_p, P(capi.DDReport)]
    L.kmc_dd_step.argtypes = [C.c_void_p, C.c_void_p, C.c_double, C.c_void_p]
    L.kmc_dd_cut_count.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, P(C.c_int32)]
    L.kmc_list_growth.argtypes = [C.c_void_p]
    L.kmc_set_list_growth.argtypes = [C.c_void_p, C.c_int32]
    for f in ("kmc_host_math", "kmc_device_math"):
        getattr(L, f).argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64]
    _lib = L
    return L


def _host_check(rc: int):
    if rc != 0:
        raise KmcError(rc, load_library().kmc_host_last_error().decode())


# ---------------------------------------------------------------- host-only
def host_init_random(params: capi.Params) -> capi.HostState:
    """Random placement (main.cpp:281-447, keyed draws) into host buffers."""
    hs = capi.HostState(params.n_a, params.n_b)
    v = hs.view()
    _host_check(load_library().kmc_host_init_random(C.byref(params), C.byref(v)))
    hs.pull(v)
    return hs


def host_load_cpt(params: capi.Params, path: str) -> capi.HostState:
    """position.cpt → host state (main.cpp:226-270)."""
    hs = capi.HostState(params.n_a, params.n_b)
    v = hs.view()
    _host_check(load_library().kmc_host_load_cpt(C.byref(params), os.fsencode(path), C.byref(v)))
    hs.pull(v)
    return hs


def host_write_cpt(params: capi.Params, hs: capi.HostState, path: str) -> None:
    """host state → position.cpt (main.cpp:2206-2244)."""
    v = hs.view()
    _host_check(load_library().kmc_host_write_cpt(C.byref(params), C.byref(v), os.fsencode(path)))


def host_save_state(params: capi.Params, hs: capi.HostState, path: str) -> None:
    """host state → exact binary checkpoint (KMCSTAT1, include/kmc.h)."""
    v = hs.view()
    _host_check(load_library().kmc_host_save_state(C.byref(params), C.byref(v), os.fsencode(path)))


def host_load_state(params: capi.Params, path: str) -> capi.HostState:
    """exact binary checkpoint → host state (refuses another trajectory's file)."""
    hs = capi.HostState(params.n_a, params.n_b)
    v = hs.view()
    _host_check(load_library().kmc_host_load_state(C.byref(params), os.fsencode(path), C.byref(v)))
    hs.pull(v)
    return hs


def host_validate(params: capi.Params, hs: capi.HostState) -> int:
    v = hs.view()
    return int(load_library().kmc_host_validate(C.byref(params), C.byref(v)))


def host_dd_check(gid: np.ndarray, own: np.ndarray) -> int:
    """kmc_dd_set_state's argument check on the host: 0 or KMC_ERR_ARG."""
    gid = np.ascontiguousarray(gid, dtype=np.int32)
    own = np.ascontiguousarray(own, dtype=np.uint8)
    if gid.size != own.size:
        raise ValueError("gid / own of one window")
    return int(load_library().kmc_host_dd_check(gid.size, gid.ctypes.data, own.ctypes.data))


def state_hash(params: capi.Params, hs: capi.HostState) -> int:
    v = hs.view()
    return int(load_library().kmc_state_hash(C.byref(params), C.byref(v)))


def bond_line(params: capi.Params, rec) -> str:
    """One bond.dat line (main.cpp:2251) from a kmc_obs record."""
    o = capi.Obs()
    for name in capi.OBS_DTYPE.names:
        setattr(o, name, rec[name].item() if hasattr(rec[name], "item") else rec[name])
    buf = C.create_string_buffer(256)
    n = load_library().kmc_format_bond_line(C.byref(params), C.byref(o), buf, 256)
    return buf.value[:n].decode()


def write_parameter_log(params: capi.Params, path: str) -> None:
    """parameter.log (main.cpp:178-205)."""
    _host_check(load_library().kmc_host_write_parameter_log(C.byref(params), os.fsencode(path)))


def append_gro(params: capi.Params, hs: capi.HostState, path: str) -> None:
    """one test.gro frame (main.cpp:2258-2287)."""
    v = hs.view()
    _host_check(load_library().kmc_host_append_gro(C.byref(params), C.byref(v), os.fsencode(path)))


def append_cluster_log(params: capi.Params, step: int, row_len: np.ndarray, members: np.ndarray, path: str) -> None:
    """one cluster.log block (main.cpp:2291-2305)."""
    row_len = np.ascontiguousarray(row_len, dtype=np.int32)
    members = np.ascontiguousarray(members, dtype=np.int32)
    _host_check(load_library().kmc_host_append_cluster_log(C.byref(params), step, row_len.ctypes.data,
                                                           members.ctypes.data, os.fsencode(path)))


def math(op: int, x: np.ndarray, y: Optional[np.ndarray] = None, device: bool = False) -> np.ndarray:
    """Portable libm (kmc_math.h) on host or device — numerics diagnostics."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.ascontiguousarray(np.zeros_like(x) if y is None else y, dtype=np.float64)
    out = np.empty_like(x)
    L = load_library()
    f = L.kmc_device_math if device else L.kmc_host_math
    rc = f(op, x.ctypes.data, y.ctypes.data, out.ctypes.data, x.size)
    if rc != 0:
        raise KmcError(rc, "math diagnostic failed")
    return out


# ---------------------------------------------------------------- device sim
class Simulation:
    """One trajectory on one GPU (handle = kmc_sim*)."""

    def __init__(self, params: capi.Params, device: int = 0):
        self.params = params
        self.device = device  # HIP ordinal: the decomposed mode's exchange buffers live there
        L = load_library()
        h = C.c_void_p()
        rc = L.kmc_create(C.byref(params), device, C.byref(h))
        if rc != 0:
            raise KmcError(rc, "kmc_create failed (needs a gfx950 device)")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            load_library().kmc_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, rc: int):
        if rc != 0:
            raise KmcError(rc, load_library().kmc_last_error(self._h).decode())

    def init_random(self):
        self._check(load_library().kmc_init_random(self._h))

    def load_cpt(self, path: str):
        self._check(load_library().kmc_load_cpt(self._h, os.fsencode(path)))

    def write_cpt(self, path: str):
        self._check(load_library().kmc_write_cpt(self._h, os.fsencode(path)))

    def save_state(self, path: str):
        """Exact checkpoint: a later load_state continues the trajectory bit for bit."""
        self._check(load_library().kmc_save_state(self._h, os.fsencode(path)))

    def load_state(self, path: str):
        self._check(load_library().kmc_load_state(self._h, os.fsencode(path)))

    def set_state(self, hs: capi.HostState):
        v = hs.view()
        self._check(load_library().kmc_set_state(self._h, C.byref(v)))

    def get_state(self) -> capi.HostState:
        hs = capi.HostState(self.params.n_a, self.params.n_b)
        v = hs.view()
        self._check(load_library().kmc_get_state(self._h, C.byref(v)))
        hs.pull(v)
        return hs

    def step(self, n: int, out: Optional[np.ndarray] = None) -> np.ndarray:
        """Advance n steps; returns the n bond.dat records (capi.OBS_DTYPE)."""
        if out is None:
            out = np.zeros(n, dtype=capi.OBS_DTYPE)
        elif out.dtype != capi.OBS_DTYPE or not out.flags.c_contiguous or not out.flags.writeable or len(out) < n:
            # kmc_step writes n records of sizeof(kmc_obs) through the pointer
            raise ValueError(f"out must be a writeable C-contiguous capi.OBS_DTYPE array of length >= {n}")
        self._check(load_library().kmc_step(self._h, n, out.ctypes.data_as(C.c_void_p)))
        return out

    def clusters(self):
        """BFS member rows of the last step: (row_len[n_b], members) — kmc_get_clusters."""
        row = np.zeros(self.params.n_b, dtype=np.int32)
        mem = np.zeros(self.params.n_a + self.params.n_b, dtype=np.int32)
        self._check(load_library().kmc_get_clusters(self._h, row.ctypes.data, mem.ctypes.data))
        return row, mem[: int(row.sum())]

    @property
    def current_step(self) -> int:
        return int(load_library().kmc_current_step(self._h))

    # ---- one slab's window of a decomposed trajectory (kmc_dd_*, slabs.py)
    def dd_set_state(self, hs: capi.HostState, gid: np.ndarray, own: np.ndarray, ctl5) -> None:
        gid = np.ascontiguousarray(gid, dtype=np.int32)
        own = np.ascontiguousarray(own, dtype=np.uint8)
        c5 = np.ascontiguousarray(ctl5, dtype=np.int32)
        n = self.params.n_a + self.params.n_b
        if gid.size != n or own.size != n or c5.size != 5:
            raise ValueError("dd_set_state: gid / own sized n_a + n_b, ctl5 five values")
        v = hs.view()
        self._check(load_library().kmc_dd_set_state(self._h, C.byref(v), gid.ctypes.data, own.ctypes.data,
                                                    c5.ctypes.data))

    def dd_export(self, ids: np.ndarray):
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        beads = np.zeros((ids.size, 48), dtype=np.float64)
        ints = np.zeros((ids.size, 8), dtype=np.int32)
        self._check(load_library().kmc_dd_export(self._h, ids.size, ids.ctypes.data, beads.ctypes.data,
                                                 ints.ctypes.data))
        return beads, ints

    def dd_import(self, ids: np.ndarray, beads: np.ndarray, ints: np.ndarray) -> np.ndarray:
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        beads = np.ascontiguousarray(beads, dtype=np.float64)
        ints = np.ascontiguousarray(ints, dtype=np.int32)
        if beads.shape != (ids.size, 48) or ints.shape != (ids.size, 8):
            raise ValueError("dd_import: beads [n, 48], ints [n, 8]")
        flags = np.zeros(ids.size, dtype=np.uint8)
        self._check(load_library().kmc_dd_import(self._h, ids.size, ids.ctypes.data, beads.ctypes.data,
                                                 ints.ctypes.data, flags.ctypes.data))
        return flags

    def dd_drift(self) -> float:
        x = C.c_double()
        self._check(load_library().kmc_dd_drift(self._h, C.byref(x)))
        return float(x.value)

    def dd_counters(self):
        out = np.zeros(2, dtype=np.int64)
        self._check(load_library().kmc_dd_counters(self._h, out.ctypes.data))
        return int(out[0]), int(out[1])

    def dd_jumpers(self, S: float):
        """(local ids, x) of the owned proteins displaced more than S Å."""
        cap = 256
        while True:
            ids = np.zeros(cap, dtype=np.int32)
            xs = np.zeros(cap, dtype=np.float64)
            n = C.c_int32()
            self._check(load_library().kmc_dd_jumpers(self._h, S, cap, ids.ctypes.data, xs.ctypes.data, C.byref(n)))
            if n.value <= cap:
                return ids[: n.value], xs[: n.value]
            cap = n.value

    # the device-resident exchange (kmc_dd_plan / pack / unpack / finish)
    def dd_plan(self, send_ids: np.ndarray, recv_ids: np.ndarray, own: np.ndarray, band: np.ndarray) -> None:
        send_ids = np.ascontiguousarray(send_ids, dtype=np.int32)
        recv_ids = np.ascontiguousarray(recv_ids, dtype=np.int32)
        own = np.ascontiguousarray(own, dtype=np.uint8)
        band = np.ascontiguousarray(band, dtype=np.uint8)
        n = self.params.n_a + self.params.n_b
        if own.size != n or band.size != n:
            raise ValueError("dd_plan: own / band sized n_a + n_b")
        self._check(load_library().kmc_dd_plan(self._h, send_ids.size, send_ids.ctypes.data, recv_ids.size,
                                               recv_ids.ctypes.data, own.ctypes.data, band.ctypes.data))

    def dd_pack(self, dst: int = 0) -> int:
        """Pack the plan's rows into device address dst (0: the handle's own
        send buffer); returns the address written."""
        L = load_library()
        self._check(L.kmc_dd_pack(self._h, dst or None))
        return dst or int(L.kmc_dd_send_buffer(self._h) or 0)

    def dd_unpack(self, src: int, first: int, n: int) -> None:
        self._check(load_library().kmc_dd_unpack(self._h, src, first, n))

    def dd_step(self, dst: int, S: float) -> np.ndarray:
        """One step of the window, its exchange rows packed into device
        address dst (0: the handle's send buffer) and its jumpers beyond S
        listed, in one wait; returns the step's record."""
        out = np.zeros(1, dtype=capi.OBS_DTYPE)
        self._check(load_library().kmc_dd_step(self._h, dst or None, S, out.ctypes.data_as(C.c_void_p)))
        return out

    def dd_send_address(self) -> int:
        return int(load_library().kmc_dd_send_buffer(self._h) or 0)

    def dd_finish(self) -> capi.DDReport:
        rep = capi.DDReport()
        self._check(load_library().kmc_dd_finish(self._h, C.byref(rep)))
        return rep

    def dd_cut_count(self, ids: np.ndarray) -> int:
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        c = C.c_int32()
        self._check(load_library().kmc_dd_cut_count(self._h, ids.size, ids.ctypes.data, C.byref(c)))
        return int(c.value)

    @property
    def list_growth(self) -> int:
        return int(load_library().kmc_list_growth(self._h))

    def set_list_growth(self, level: int) -> None:
        self._check(load_library().kmc_set_list_growth(self._h, level))

    def set_timing(self, kernels=(), every: int = 1):
        """Bracket the named kernels with HIP events (empty: off), in every
        `every`-th step only."""
        names = kernel_names()
        mask = 0
        for k in kernels:
            mask |= 1 << names.index(k)
        self._check(load_library().kmc_set_timing(self._h, mask))
        self._check(load_library().kmc_set_timing_period(self._h, every))

    def kernel_times(self) -> dict:
        """{kernel: (total_ms, launches)} accumulated since set_timing."""
        ms = (C.c_double * 64)()
        cnt = (C.c_int64 * 64)()
        n = load_library().kmc_kernel_times(self._h, ms, cnt, 64)
        names = kernel_names()
        return {names[i]: (ms[i], cnt[i]) for i in range(n) if cnt[i]}


def kernel_names():
    L = load_library()
    out = []
    i = 0
    while True:
        nm = L.kmc_kernel_name(i).decode()
        if not nm:
            return out
        out.append(nm)
        i += 1
