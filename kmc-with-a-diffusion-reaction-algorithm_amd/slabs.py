"""One KMC trajectory split over G slabs.

The reference's step is one sequential loop over every unit
(main.cpp:577-1872, Gauss–Seidel reads of R_new at 640-664 / 1762-1828)
followed by greedy reactions over all pairs (main.cpp:1877-2058).  Both are
global, yet a unit's outcome depends only on the units near it.  Here the box
is cut into G slabs along x; each slab is simulated by its own engine handle
(libkmc's kmc_dd_* entry points, include/kmc.h) over a *window*: the units it
owns plus halo copies of every protein within `halo` Å (periodic in x) of
them.  Because every random number is keyed by (seed, replica; step, global
index, site) — never by who draws it — a handle computes exactly the
trajectory's values for every protein whose neighbourhood it holds.

Per step, on every rank:
  1. step the window (kmc_step, one step): owned units and halo copies alike;
  2. export the end-of-step state of the owned proteins other windows hold,
     exchange (all-to-all), import the owners' state over the halo copies;
  3. VERIFY: every halo protein close enough to interact with an owned one
     (the *band*, within `halo / 2`) must have come out bit-identical to its
     owner's result.  By induction over the step's decision order (unit keys,
     then reaction edges) an owned protein can only be wrong if some band
     protein's decision was, and that shows as a difference here; the outer
     half of the halo only feeds the band's own computation;
  4. all-reduce the observable shares (bond counts of owned receptors, owned
     complexes; the largest complex by max) into the bond.dat record.
Presence.  With band B = halo / 2 and S = (B − R_INT) / 2, a protein that
stays within S (in x) of where it was at the last partition meets, within
R_INT, only proteins its owner's window holds in the band.  The few that
move further (association snaps and lay-downs jump a receptor by up to
≈ 180 Å) are *jumpers*, checked after every step against the partition:
(J_B) a jumper stays within S of its own slab's proteins, (J_A) a jumper is
at least R_INT + S from the proteins of every slab that does not hold it in
its band.  Only accepted positions need checking: a unit whose proposal met
a protein its window lacks can only have lost a collision, so a rejection is
right and an acceptance puts the proposal under the checks.
Re-partition (a collective *rebuild* from the assembled global state, which
is also the rollback checkpoint) happens when a bond joined units of two
slabs (a unit must be owned whole) and when jumpers accumulate; a failed
verification or jumper check rolls back to the checkpoint, replays to the
step before, re-partitions there and retries (a second failure widens the
halo): the run is exact whenever it completes.

This module is the host side of the decomposed path; the engine under each
rank is anything with the kmc_dd_* contract (engine.Simulation on a gfx950
device; the tests also run the same driver over the CPU oracle).  The
exchange goes through a Comm: LocalComm (G ranks as threads of one process,
e.g. G windows on one GPU) or TorchComm (one rank per process over
torch.distributed).
"""
from __future__ import annotations

import os
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, List, Optional

import numpy as np

from . import capi

# Largest x distance between the [1][1] reference points of two proteins that
# interact within one step: a ligand–ligand collision has subunit centres
# < 60 Å apart, each within 35 Å of its ligand's [1][1] (DESIGN.md §cell
# list) — 130 Å; R–L gates are shorter (< 104 Å), receptor pairs < 56 Å.
R_INT = 140.0
# re-partition when more than this many jumpers (all slabs) have accumulated
JUMPERS_MAX = 64

A_LINKS = (2, 4)  # kmc_state_view a_int rows holding protein links (nei2, nei3)
B_LINKS = (4, 5, 6, 7)


class SlabError(RuntimeError):
    pass


# ---------------------------------------------------------------- comms
class LocalComm:
    """G ranks as threads of one process (one engine handle each)."""

    def __init__(self, world: int):
        self.world = world
        self._slots: list = [None] * world
        self._bar = threading.Barrier(world)

    def allgather(self, rank: int, obj):
        self._slots[rank] = obj
        self._bar.wait()
        out = list(self._slots)
        self._bar.wait()
        return out

    def alltoall(self, rank: int, objs: list) -> list:
        allv = self.allgather(rank, objs)
        return [allv[src][rank] for src in range(self.world)]


class TorchComm:
    """One rank per process over an initialised torch.distributed group."""

    def __init__(self):
        import torch.distributed as dist

        self.dist = dist
        self.world = dist.get_world_size()

    def allgather(self, rank: int, obj):
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def alltoall(self, rank: int, objs: list) -> list:
        """objs[r] to rank r; returns the messages from every rank.  Over gloo
        each message goes only to its destination (sizes all-gathered, then
        point-to-point); other backends all-gather every message."""
        if self.dist.get_backend() != "gloo":
            allv = self.allgather(rank, objs)
            return [allv[src][rank] for src in range(self.world)]
        import pickle

        import torch

        W = self.world
        data = [b"" if r == rank or objs[r] is None else pickle.dumps(objs[r], protocol=5) for r in range(W)]
        sizes = [torch.zeros(W, dtype=torch.int64) for _ in range(W)]
        self.dist.all_gather(sizes, torch.tensor([len(x) for x in data], dtype=torch.int64))
        reqs, bufs = [], {}
        for r in range(W):
            if r == rank:
                continue
            if data[r]:
                reqs.append(self.dist.isend(torch.frombuffer(bytearray(data[r]), dtype=torch.uint8), r))
            n = int(sizes[r][rank])
            if n:
                bufs[r] = torch.empty(n, dtype=torch.uint8)
                reqs.append(self.dist.irecv(bufs[r], r))
        for q in reqs:
            q.wait()
        out = [None] * W
        out[rank] = objs[rank]
        for r, b in bufs.items():
            out[r] = pickle.loads(b.numpy().tobytes())  # (a peer rank's own message)
        return out


def run_threads(world: int, fn: Callable[[int], object]) -> list:
    """fn(rank) on `world` threads; re-raises the first failure."""
    out: list = [None] * world
    err: list = []

    def body(r):
        try:
            out[r] = fn(r)
        except BaseException as e:  # noqa: BLE001
            err.append(e)
            # unblock the others waiting in a collective
            for c in _comms_of(fn):
                c._bar.abort()

    th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if err:
        real = [e for e in err if not isinstance(e, threading.BrokenBarrierError)]
        if len(real) > 1:
            real[0].add_note("other ranks: " + "; ".join(repr(e) for e in real[1:])) if hasattr(real[0], "add_note") \
                else None
            real[0].args = real[0].args + tuple(f"(also: {e!r})" for e in real[1:])
        raise (real or err)[0]
    return out


def _comms_of(fn):
    comms = getattr(fn, "comms", None)
    return comms if comms is not None else []


# ---------------------------------------------------------------- global state
def derived_counts(hs: capi.HostState):
    """rl, mono_cis, cis pair counts of a state (main.cpp:1931-2136 bookkeeping)."""
    st2, st3, nei3 = hs.a_int[0], hs.a_int[1], hs.a_int[4]
    rl = int((st2 == 1).sum())
    i = np.flatnonzero((st3 == 1) & (nei3 - 1 > np.arange(hs.n_a)))
    q = nei3[i] - 1
    mono = int(((st2[i] == 0) & (st2[q] == 0)).sum())
    return rl, mono, int(i.size) - mono


def ref_x(hs: capi.HostState) -> np.ndarray:
    """x of bead [1][1] of every protein, global order."""
    return np.concatenate([hs.ra[0], hs.rb[0]])


def units(hs: capi.HostState) -> np.ndarray:
    """Unit (connected component of the bond graph) of every protein, labelled
    by its lowest global index: a free protein, a cis dimer or a
    ligand-rooted complex (main.cpp:514-562, 584, 682, 905)."""
    n_a, n = hs.n_a, hs.n_a + hs.n_b
    lab = np.arange(n, dtype=np.int64)
    src, dst = [], []
    for r in A_LINKS:
        v = hs.a_int[r]
        k = np.flatnonzero(v > 0)
        src.append(k)
        dst.append(v[k] - 1)
    for r in B_LINKS:
        v = hs.b_int[r]
        k = np.flatnonzero(v > 0)
        src.append(n_a + k)
        dst.append(v[k] - 1)
    src = np.concatenate(src).astype(np.int64)
    dst = np.concatenate(dst).astype(np.int64)
    while True:  # min-label propagation to a fixed point (components are small)
        m = np.minimum(lab[src], lab[dst])
        new = lab.copy()
        np.minimum.at(new, src, m)
        np.minimum.at(new, dst, m)
        new = new[new]
        if np.array_equal(new, lab):
            return lab
        lab = new


def periodic_dist(x: np.ndarray, ref_sorted: np.ndarray, L: float) -> np.ndarray:
    """Distance (periodic in L) of each x to the nearest value of ref_sorted."""
    if ref_sorted.size == 0:
        return np.full(x.shape, np.inf)
    j = np.searchsorted(ref_sorted, x)
    lo = ref_sorted[(j - 1) % ref_sorted.size]
    hi = ref_sorted[j % ref_sorted.size]
    d1 = np.abs(x - lo)
    d2 = np.abs(hi - x)
    d1 = np.minimum(d1, L - d1)
    d2 = np.minimum(d2, L - d2)
    return np.minimum(d1, d2)


@dataclass
class Window:
    gids: np.ndarray          # global indices held, increasing (receptors first)
    own: np.ndarray           # uint8 per held protein
    band: np.ndarray          # bool per held protein: halo within halo / 2 of an owned protein
    n_a: int = 0
    n_b: int = 0
    loc: dict = field(default_factory=dict)  # global index -> local index


@dataclass
class Plan:
    """The partition of one state into G windows (identical on every rank)."""

    owner: np.ndarray         # rank per global protein
    windows: List[Window]
    halo: float
    own_x: List[np.ndarray]   # per rank: sorted wrapped x of its owned proteins
    near: List[np.ndarray]    # per rank: bool per global protein, owned or in its band


def make_plan(p: capi.Params, hs: capi.HostState, G: int, halo: float) -> Plan:
    L = p.box_x
    n_a = hs.n_a
    x = ref_x(hs)
    xw = x - L * np.floor((x + L / 2) / L)  # wrapped into [-L/2, L/2)
    lab = units(hs)
    slab = np.clip(np.floor((xw[lab] + L / 2) / (L / G)).astype(np.int64), 0, G - 1)  # by the unit's lead
    owner = slab
    band_w = halo / 2
    windows, own_x, near = [], [], []
    for r in range(G):
        own = owner == r
        ref = np.sort(xw[own])
        own_x.append(ref)
        d = periodic_dist(xw, ref, L)
        held = own | (d < halo)
        band = ~own & (d < band_w)
        near.append(own | band)
        # a band protein's whole unit is held: its local computation then
        # sees every member (a unit is moved and decided as one)
        held |= np.isin(lab, np.unique(lab[band]))
        gids = np.flatnonzero(held).astype(np.int32)
        w = Window(gids=gids, own=own[gids].astype(np.uint8), band=band[gids],
                   n_a=int((gids < n_a).sum()), n_b=int((gids >= n_a).sum()))
        w.loc = {int(g): i for i, g in enumerate(gids)}
        windows.append(w)
    return Plan(owner=owner, windows=windows, halo=halo, own_x=own_x, near=near)


def window_state(hs: capi.HostState, w: Window) -> capi.HostState:
    """The window's proteins in local numbering; links to proteins outside the
    window are cut (status and link cleared: only outer-halo proteins have
    them — band units are held whole)."""
    n_a = hs.n_a
    ga = w.gids[: w.n_a]
    gb = w.gids[w.n_a:] - n_a
    out = capi.HostState(w.n_a, w.n_b)
    out.ra[:] = hs.ra[:, ga]
    out.rb[:] = hs.rb[:, gb]
    out.a_int[:] = hs.a_int[:, ga]
    out.b_int[:] = hs.b_int[:, gb]
    out.step = hs.step
    g2l = np.full(hs.n_a + hs.n_b + 1, 0, dtype=np.int32)  # global + 1 -> local + 1 (0 = outside)
    g2l[w.gids + 1] = np.arange(1, w.gids.size + 1, dtype=np.int32)
    a, b = out.a_int, out.b_int
    # receptor links: nei2 (row 2; status st2, site nei4) and nei3 (row 4; st3)
    l2 = g2l[a[2]]
    cut = (a[2] > 0) & (l2 == 0)
    a[0][cut] = 0
    a[3][cut] = 0
    a[2] = l2
    l3 = g2l[a[4]]
    cut = (a[4] > 0) & (l3 == 0)
    a[1][cut] = 0
    a[4] = l3
    for j in range(4):  # ligand site j+1: status row j, link row 4+j
        lk = g2l[b[4 + j]]
        cut = (b[4 + j] > 0) & (lk == 0)
        b[j][cut] = 0
        b[4 + j] = lk
    return out


# ---------------------------------------------------------------- one rank
class SlabRank:
    """Rank `rank` of a G-slab trajectory.  make_engine(params) returns a fresh
    handle with the kmc_dd_* methods for a window's proteins."""

    def __init__(self, p: capi.Params, rank: int, comm, make_engine: Callable, halo: float = 900.0,
                 gather_every: int = 0):
        self.p = p
        self.rank = rank
        self.comm = comm
        self.G = comm.world
        self.make_engine = make_engine
        self.halo = float(halo)
        self.gather_every = gather_every  # assemble the global state every k steps (tests: 1)
        self.eng = None
        self.plan: Optional[Plan] = None
        self.win: Optional[Window] = None
        self.step_no = 0
        self.counters = np.zeros(5, dtype=np.int32)
        self.ckpt: Optional[capi.HostState] = None
        self.history: list = []  # global records since the checkpoint (replay check)
        self.stats = dict(steps=0, rebuilds=0, rebuild_bond=0, rebuild_jumpers=0, rollbacks=0, replayed=0, xcol=0,
                          xbond=0,
                          exchanged=0, verified=0, jumpers=0, held=0, owned=0, why=[],
                          sec=dict(step=0.0, export=0.0, comm=0.0, imp=0.0, jumpers=0.0, gather=0.0, rebuild=0.0))
        self.last_global: Optional[capi.HostState] = None
        self._xc = (0, 0)
        self._njump = 0  # jumpers after the last step, all slabs
        # debug (KMC_SLABS_CHECK=1): the window's bond graph and extent bounds
        # validated (kmc_host_validate) after every import
        self.check = os.environ.get("KMC_SLABS_CHECK") == "1"

    @property
    def band(self) -> float:
        return self.halo / 2

    @property
    def S(self) -> float:
        """Displacement since the partition below which a protein is no jumper."""
        return (self.band - R_INT) / 2

    # -- partition -------------------------------------------------------
    def start(self, hs: capi.HostState) -> None:
        """Every rank calls this with the same global state."""
        self.step_no = int(hs.step)
        self.counters = hs.counters.copy()
        self._rebuild_from(hs)

    def _rebuild_from(self, hs: capi.HostState) -> None:
        t0 = time.perf_counter()
        self._rebuild_inner(hs)
        self.stats["sec"]["rebuild"] += time.perf_counter() - t0

    def _rebuild_inner(self, hs: capi.HostState) -> None:
        self.ckpt = hs.copy()
        self.ckpt.counters[:] = self.counters
        self.ckpt.step = self.step_no
        self.history = []
        self.plan = make_plan(self.p, hs, self.G, self.halo)
        w = self.plan.windows[self.rank]
        self.win = w
        ws = window_state(hs, w)
        rl, mono, cis = derived_counts(hs)
        c = self.counters
        ctl5 = [c[0] - (rl + mono + cis), c[1] - rl, c[2] - cis, c[3] - mono, c[4]] if self.rank == 0 else [0] * 5
        if self.eng is not None:
            self.eng.close()
        q = capi.Params.from_buffer_copy(self.p)
        q.n_a, q.n_b = w.n_a, w.n_b
        self.q = q
        self.eng = self.make_engine(q)
        self.eng.dd_set_state(ws, w.gids, w.own, ctl5)
        self._xc = (0, 0)
        self._njump = 0
        # export lists: my owned proteins held by each other window (local
        # indices here, global in transit)
        self.exp = []
        for r in range(self.G):
            if r == self.rank:
                self.exp.append(np.zeros(0, np.int32))
                continue
            g = np.intersect1d(w.gids[w.own == 1], self.plan.windows[r].gids, assume_unique=True)
            self.exp.append(np.array([w.loc[int(x)] for x in g], dtype=np.int32))
        self.g2l = np.zeros(self.p.n_a + self.p.n_b + 1, dtype=np.int32)  # global + 1 -> local + 1
        self.g2l[w.gids + 1] = np.arange(1, w.gids.size + 1, dtype=np.int32)
        self.stats["held"] = int(w.gids.size)
        self.stats["owned"] = int(w.own.sum())
        self.stats["rebuilds"] += 1

    def _links(self, ints: np.ndarray, local_ids: np.ndarray, to_global: bool, win: Window) -> np.ndarray:
        """Translate the link fields of exchanged records (local <-> global + 1)."""
        out = ints.copy()
        rec = local_ids < win.n_a
        for f in range(8):
            col = out[:, f]
            is_link = (rec & ((f == 2) | (f == 4))) | (~rec & (f >= 4))
            m = is_link & (col > 0)
            if to_global:
                col[m] = win.gids[col[m] - 1] + 1
            else:
                col[m] = self.g2l[col[m]]
        return out

    def global_state(self) -> capi.HostState:
        """Collective: the trajectory's state assembled from every slab's owned proteins."""
        w = self.win
        ids = np.flatnonzero(w.own).astype(np.int32)
        beads, ints = self.eng.dd_export(ids)
        ints = self._links(ints, ids, True, w)
        parts = self.comm.allgather(self.rank, (w.gids[ids], beads, ints))
        n_a, n_b = self.p.n_a, self.p.n_b
        hs = capi.HostState(n_a, n_b)
        for g, b, i in parts:
            ra = g < n_a
            hs.ra[:, g[ra]] = b[ra].T
            hs.a_int[:, g[ra]] = i[ra, :5].T
            hs.rb[:, g[~ra] - n_a] = b[~ra, :24].T
            hs.b_int[:, g[~ra] - n_a] = i[~ra].T
        hs.counters[:] = self.counters
        hs.step = self.step_no
        return hs

    # -- one step --------------------------------------------------------
    def step(self) -> np.ndarray:
        """Advance the trajectory one step; returns its bond.dat record (global,
        a one-element capi.OBS_DTYPE array)."""
        rec = self._one()
        tries = 0
        while rec is None:  # a check failed on some slab: back to the step before, re-partition, retry
            tries += 1
            self._recover(widen=tries > 1)
            rec = self._one()
        self._remember(rec)
        self.stats["steps"] += 1
        return rec

    def _remember(self, rec: np.ndarray) -> None:
        # the records since the checkpoint (a re-partition inside the step
        # made its end state the checkpoint: nothing to replay for it)
        if int(rec["step"][0]) > self.ckpt.step:
            self.history.append(rec.copy())

    def _one(self) -> Optional[np.ndarray]:
        if self._njump > JUMPERS_MAX:
            self.stats["rebuild_jumpers"] += 1
            self._rebuild_from(self.global_state())
        return self._step_exchange()

    def _jumper_check(self) -> int:
        """Jumpers of my slab violating J_A / J_B (module docstring): count."""
        ids, xs = self.eng.dd_jumpers(self.S)
        self._my_jumpers = int(ids.size)
        if ids.size == 0:
            return 0
        L = self.p.box_x
        xw = xs - L * np.floor((xs + L / 2) / L)
        g = self.win.gids[ids]
        bad = int((periodic_dist(xw, self.plan.own_x[self.rank], L) > self.S).sum())  # J_B
        for r in range(self.G):
            if r == self.rank:
                continue
            far = ~self.plan.near[r][g]
            if far.any():
                bad += int((periodic_dist(xw[far], self.plan.own_x[r], L) < R_INT + self.S).sum())  # J_A
        return bad

    def _step_exchange(self) -> Optional[np.ndarray]:
        w = self.win
        sec = self.stats["sec"]  # host seconds by phase (tools/slab_rate.py)
        t0 = time.perf_counter()
        part = self.eng.step(1)[0]
        xcol, xbond = self.eng.dd_counters()
        t1 = time.perf_counter()
        sec["step"] += t1 - t0
        dcol, dbond = xcol - self._xc[0], xbond - self._xc[1]
        self._xc = (xcol, xbond)
        # halo exchange: my owned proteins' end state to every window holding them
        out = []
        for r in range(self.G):
            ids = self.exp[r]
            if ids.size == 0:
                out.append(None)
                continue
            beads, ints = self.eng.dd_export(ids)
            out.append((w.gids[ids], beads, self._links(ints, ids, True, w)))
        t2 = time.perf_counter()
        sec["export"] += t2 - t1
        got = self.comm.alltoall(self.rank, out)
        t3 = time.perf_counter()
        sec["comm"] += t3 - t2
        bad = 0
        nver = 0
        for src, msg in enumerate(got):
            if msg is None:
                continue
            g, beads, ints = msg
            loc = self.g2l[g + 1] - 1
            if (loc < 0).any():
                raise SlabError("a halo record of a protein this window does not hold")
            li = self._links(ints, loc, False, w)
            # a link to a protein outside the window (outer halo only): cut it
            lost = (ints > 0) & (li == 0)
            lost_any = lost.any(axis=1)
            if lost_any.any():
                if w.band[loc[lost_any]].any():
                    bad += 1  # a band unit reached outside the window: re-partition
                rec = loc < w.n_a
                for k in np.flatnonzero(lost_any):
                    for f in np.flatnonzero(lost[k]):
                        if rec[k]:
                            li[k, 0 if f == 2 else 1] = 0
                            if f == 2:
                                li[k, 3] = 0
                        else:
                            li[k, f - 4] = 0
            flags = self.eng.dd_import(loc, beads, li)
            vb = w.band[loc]
            nver += int(vb.sum())
            bad += int((flags[vb] != 0).sum())
            self.stats["exchanged"] += int(loc.size)
        self.stats["verified"] += nver
        if self.check:
            from . import engine as _engine

            rc = _engine.host_validate(self.q, self.eng.get_state())
            if rc != 0:
                raise SlabError(f"rank {self.rank}: window state invalid ({rc}) after the import of step "
                                f"{self.step_no + 1}: {_engine.load_library().kmc_host_last_error().decode()}")
        t4 = time.perf_counter()
        sec["imp"] += t4 - t3
        jbad = self._jumper_check()
        t5 = time.perf_counter()
        sec["jumpers"] += t5 - t4
        # the step's record from every slab's share; checks, triggers
        shares = self.comm.allgather(self.rank, (part.copy(), bad, jbad, dbond, dcol, self._my_jumpers))
        sec["gather"] += time.perf_counter() - t5
        if any(s[1] or s[2] for s in shares):
            self.stats["why"].append((self.step_no + 1, "verify" if any(s[1] for s in shares) else "jumper",
                                      sum(s[1] for s in shares), sum(s[2] for s in shares)))
            return None
        self.stats["xbond"] += sum(s[3] for s in shares)
        self.stats["xcol"] += sum(s[4] for s in shares)
        self._njump = sum(s[5] for s in shares)
        self.stats["jumpers"] = max(self.stats["jumpers"], self._njump)
        rec = combine([s[0] for s in shares])
        r0 = rec[0]
        self.step_no = int(r0["step"])
        self.counters[:] = [r0["bond_num"], r0["bond_num_rl"], r0["bond_num_cis"], r0["bond_num_mono_cis"],
                            r0["protein_num_in_max_complex"]]
        need = any(s[3] for s in shares)  # a bond between two slabs' units: one owner for the new unit
        if need or (self.gather_every and self.step_no % self.gather_every == 0):
            gs = self.global_state()
            self.last_global = gs
            if need:
                self.stats["rebuild_bond"] += 1
                self._rebuild_from(gs)
        return rec

    def _recover(self, widen: bool) -> None:
        """Back to the checkpoint, replay to the last good step, re-partition
        there (with a wider halo on a repeated failure)."""
        self.stats["rollbacks"] += 1
        if self.stats["rollbacks"] > 64 or self.halo > 64 * self.p.box_x:
            raise SlabError("decomposed step does not pass its checks even with the whole box as halo")
        hist = self.history
        self.stats["replayed"] += len(hist)
        if widen:
            self.halo *= 1.5
        self.counters = self.ckpt.counters.copy()
        self.step_no = int(self.ckpt.step)
        self._rebuild_from(self.ckpt)
        for want in hist:
            rec = self._step_exchange()
            if rec is None or not np.array_equal(rec, want):
                raise SlabError(f"rank {self.rank}: replaying from the checkpoint (step {self.ckpt.step}) did not "
                                f"reproduce step {int(want['step'][0])}: "
                                f"{'a check failed' if rec is None else f'{rec} != {want}'}; checks: {self.stats['why']}")
            self._remember(rec)
        if hist:
            self._rebuild_from(self.global_state())

    def close(self):
        if self.eng is not None:
            self.eng.close()
            self.eng = None


def combine(parts) -> np.ndarray:
    """bond.dat record of the trajectory from the slabs' shares (sums; the
    largest complex by max; cluster_size as k_finalize computes it)."""
    rec = np.zeros(1, dtype=capi.OBS_DTYPE)
    rec["step"] = parts[0]["step"]
    rec["t"] = parts[0]["t"]
    for f in ("bond_num_rl", "bond_num_mono_cis", "bond_num_cis", "bond_num", "tot_proteins_in_cluster",
              "tot_cluster_num"):
        rec[f] = sum(int(x[f]) for x in parts)
    rec["protein_num_in_max_complex"] = max(int(x["protein_num_in_max_complex"]) for x in parts)
    tp, tc = int(rec["tot_proteins_in_cluster"][0]), int(rec["tot_cluster_num"][0])
    rec["cluster_size"] = tp / tc if tc != 0 else 0.0
    return rec


def run_local(p: capi.Params, hs: capi.HostState, G: int, steps: int, make_engine: Callable,
              halo: float = 900.0, gather_every: int = 0, on_step: Optional[Callable] = None):
    """G slabs as threads of this process (e.g. G handles on one GPU).
    Returns (records[steps], ranks).  on_step(rank0, k, rec) after each step on rank 0."""
    comm = LocalComm(G)
    ranks = [SlabRank(p, r, comm, make_engine, halo=halo, gather_every=gather_every) for r in range(G)]
    recs = np.zeros(steps, dtype=capi.OBS_DTYPE)

    def body(r):
        me = ranks[r]
        me.start(hs)
        for k in range(steps):
            rec = me.step()
            if r == 0:
                recs[k] = rec[0]
                if on_step:
                    on_step(me, k, rec)
        return True

    body.comms = [comm]
    run_threads(G, body)
    return recs, ranks
