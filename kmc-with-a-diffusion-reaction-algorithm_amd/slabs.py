"""One KMC trajectory split over G slabs.

The reference's step is one sequential loop over every unit
(main.cpp:577-1872, Gauss–Seidel reads of R_new at 640-664 / 1762-1828)
followed by greedy reactions over all pairs (main.cpp:1877-2058).  Both are
global, yet a unit's outcome depends only on the units near it.  Here the box
is cut into G slabs along x; each slab is simulated by its own engine handle
(libkmc's kmc_dd_* entry points, include/kmc.h) over a *window*: the units it
owns plus halo copies of every protein within `halo` Å (periodic in x) of
them, and `margin` Å more.  Because every random number is keyed by (seed,
replica; step, global index, site) — never by who draws it — a handle
computes exactly the trajectory's values for every protein whose
neighbourhood it holds.

Per step, on every rank:
  1. step the window (kmc_step, one step): owned units and halo copies alike;
  2. the halo exchange, on device memory: every window packs the end-of-step
     rows of its owned proteins other windows hold (kmc_dd_pack, links as
     global indices), the rows travel (G handles on one device: each window
     reads its neighbours' send buffers directly; one rank per GPU: one
     all_to_all_single of device buffers over RCCL), and every window unpacks
     its owners' rows over its halo copies (kmc_dd_unpack: links found by a
     binary search of the window's global indices, cut where they leave it);
  3. VERIFY, counted on the device (kmc_dd_finish): every halo protein close
     enough to interact with an owned one (the *band*, within `halo / 2`)
     must have come out bit-identical to its owner's result, and none of its
     links may leave the window.  By induction over the step's decision order
     (unit keys, then reaction edges) an owned protein can only be wrong if
     some band protein's decision was, and that shows as a difference here;
     the outer half of the halo only feeds the band's own computation;
  4. all-gather the observable shares (bond counts of owned receptors, owned
     complexes; the largest complex by max) into the bond.dat record, with
     each rank's check results.
Presence.  With band B = halo / 2 and S = (B − R_INT) / 2, a protein that
stays within S (in x) of where it was at the last partition (its *anchor*)
meets, within R_INT, only proteins its owner's window holds in the band.  The
few that move further (association snaps and lay-downs jump a receptor by up
to ≈ 180 Å) are *jumpers*, listed by kmc_dd_finish: (J_B) a jumper stays
within S of its own slab's anchors, (J_A) a jumper is at least R_INT + S from
the anchors of every slab that does not hold it in its band.  Only accepted
positions need checking: a unit whose proposal met a protein its window lacks
can only have lost a collision, so a rejection is right and an acceptance
puts the proposal under the checks.
Cross-slab bonds.  A unit must be owned whole.  When a bond joins units of
two slabs (kmc_dd_finish lists it), the joined unit moves to the owner of its
lowest-index member: the windows are kept, only ownership, band and the
exchange lists change (kmc_dd_plan), provided the new owner holds every
protein within `halo` of the moved anchors (C1) and every new band protein's
unit whole (C2, kmc_dd_cut_count); otherwise the trajectory re-partitions.
Re-partition (a collective *rebuild* from the assembled global state, which
is also the rollback checkpoint) also happens when jumpers accumulate; a
failed verification or jumper check rolls back to the checkpoint, replays to
the step before, re-partitions there and retries (a second failure widens
the halo): the run is exact whenever it completes.

This module is the host side of the decomposed path; the engine under each
rank is anything with the kmc_dd_* contract (engine.Simulation on a gfx950
device; the tests also run the same driver over the CPU oracle, whose
"device" addresses are host addresses).  The exchange goes through a Comm:
LocalComm (G ranks as threads of one process, e.g. G windows on one GPU) or
TorchComm (one rank per process over torch.distributed: device buffers over
RCCL, host staging over gloo).
"""
from __future__ import annotations

import os
import threading
import time
from dataclasses import dataclass
from typing import Callable, List, Optional

import numpy as np

from . import capi

# Largest x distance between the [1][1] reference points of two proteins that
# interact within one step: a ligand–ligand collision has subunit centres
# < 60 Å apart, each within 35 Å of its ligand's [1][1] (DESIGN.md §cell
# list) — 130 Å; R–L gates are shorter (< 104 Å), receptor pairs < 56 Å.
R_INT = 140.0
# re-partition when more jumpers than the exchange report lists (all slabs)
# have accumulated
JUMPERS_MAX = capi.DD_JCAP
# a step that fails its checks this many times in a row (each retry from a
# wider partition) is not recoverable
MAX_TRIES = 8
ROW = capi.DD_ROW

A_LINKS = (2, 4)  # kmc_state_view a_int rows holding protein links (nei2, nei3)
B_LINKS = (4, 5, 6, 7)


class SlabError(RuntimeError):
    pass


def _engine_error(e: BaseException) -> Optional[int]:
    """The KMC_ERR_* code of an engine (libkmc or oracle) error, else None."""
    return getattr(e, "code", None)


# ---------------------------------------------------------------- comms
class LocalComm:
    """G ranks as threads of one process (one engine handle each).  The halo
    exchange reads the neighbours' send buffers in place: G handles on one
    device (or the oracle's host buffers)."""

    def __init__(self, world: int):
        self.world = world
        # two slot arrays used in turn: a rank writes the next call's slots
        # only after the barrier of this call, and the call after that (same
        # slots) only after every rank has passed the next call's barrier —
        # so one barrier per call suffices
        self._slots = [[None] * world, [None] * world]
        self._turn = [0] * world
        self._bar = threading.Barrier(world)

    def allgather(self, rank: int, obj):
        slots = self._slots[self._turn[rank]]
        self._turn[rank] ^= 1
        slots[rank] = obj
        self._bar.wait()
        return list(slots)

    def send_address(self, me: "SlabRank") -> int:
        return 0  # the window's own send buffer, which the others read in place

    def abort(self) -> None:
        """A rank failed outside a collective: release the others' waits."""
        self._bar.abort()

    def exchange(self, rank: int, me: "SlabRank") -> None:
        """The rows were packed by the step (kmc_dd_step)."""
        ptr = me.eng.dd_send_address() if me.eng_ok else None
        peers = self.allgather(rank, (ptr, me.send_first))
        if not me.eng_ok:
            return
        for src in range(self.world):
            n = me.recv_n[src]
            if src == rank or n == 0:
                continue
            sptr, sfirst = peers[src]
            if sptr is None:  # the source's step failed: the step is redone anyway
                continue
            me.eng.dd_unpack(sptr + sfirst[rank] * ROW, me.recv_first[src], n)


class TorchComm:
    """One rank per process over an initialised torch.distributed group.  The
    halo rows go through one all_to_all_single per step: on device buffers
    when the backend is a device one (nccl = RCCL on ROCm, one GPU per rank),
    through host memory over gloo."""

    def __init__(self):
        import torch.distributed as dist

        self.dist = dist
        self.world = dist.get_world_size()
        self.device_backend = dist.get_backend() != "gloo"
        self._bufs = {}

    def allgather(self, rank: int, obj):
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def abort(self) -> None:
        """A rank failed outside a collective: tear the group down, so that
        the other ranks' next collective fails instead of waiting forever."""
        try:
            self.dist.destroy_process_group()
        except Exception:  # noqa: BLE001 — already torn down or never complete
            pass

    def _buf(self, key, nbytes, device):
        import torch

        b = self._bufs.get(key)
        if b is None or b.numel() < nbytes or b.device != device:
            b = torch.empty(max(nbytes, ROW), dtype=torch.uint8, device=device)
            self._bufs[key] = b
        return b

    def _edev(self, me: "SlabRank"):
        import torch

        dev = getattr(me.eng, "device", None)
        if self.device_backend and dev is None:
            raise SlabError("a device backend exchanges device buffers: the ranks' engines must be on GPUs")
        return torch.device("cuda", dev) if dev is not None else torch.device("cpu")

    def send_address(self, me: "SlabRank") -> int:
        """The step packs its rows straight into the collective's send buffer."""
        return self._buf("send", me.n_send * ROW, self._edev(me)).data_ptr()

    def exchange(self, rank: int, me: "SlabRank") -> None:
        """The rows were packed by the step (kmc_dd_step) into send_address()."""
        import torch

        edev = self._edev(me)
        wdev = edev if self.device_backend else torch.device("cpu")  # where the collective's buffers live
        ns, nr = me.n_send * ROW, me.n_recv * ROW
        send = self._buf("send", ns, edev)
        if not me.eng_ok:
            send.zero_()
        if wdev != edev:
            send = send[:ns].to(wdev)
        recv = self._buf("recv", nr, wdev)
        self.dist.all_to_all_single(recv[:nr], send[:ns], [n * ROW for n in me.recv_n],
                                    [n * ROW for n in me.send_n])
        if wdev != edev:
            recv = self._buf("recv_dev", nr, edev)
            recv[:nr].copy_(self._bufs["recv"][:nr])
        if edev.type == "cuda":
            torch.cuda.synchronize(edev)
        if me.eng_ok and me.n_recv:
            me.eng.dd_unpack(recv.data_ptr(), 0, me.n_recv)


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
    if src.size == 0:
        return lab
    # min-label propagation to a fixed point over the bonded proteins only
    # (components are small; most proteins are free)
    nodes = np.unique(np.concatenate([src, dst]))
    s = np.searchsorted(nodes, src)
    t = np.searchsorted(nodes, dst)
    sub = nodes.copy()
    while True:
        m = np.minimum(sub[s], sub[t])
        new = sub.copy()
        np.minimum.at(new, s, m)
        np.minimum.at(new, t, m)
        new = new[np.searchsorted(nodes, new)]
        if np.array_equal(new, sub):
            lab[nodes] = sub
            return lab
        sub = new


def periodic_dist(x: np.ndarray, ref_sorted: np.ndarray, L: float) -> np.ndarray:
    """Distance (periodic in L) of each x to the nearest value of ref_sorted."""
    if ref_sorted.size == 0:
        return np.full(np.shape(x), np.inf)
    j = np.searchsorted(ref_sorted, x)
    lo = ref_sorted[(j - 1) % ref_sorted.size]
    hi = ref_sorted[j % ref_sorted.size]
    d1 = np.abs(x - lo)
    d2 = np.abs(hi - x)
    d1 = np.minimum(d1, L - d1)
    d2 = np.minimum(d2, L - d2)
    return np.minimum(d1, d2)


def wrap(x, L: float):
    """x wrapped into [-L/2, L/2)."""
    return x - L * np.floor((x + L / 2) / L)


@dataclass
class Window:
    gids: np.ndarray          # global indices held, increasing (receptors first)
    own: np.ndarray           # uint8 per held protein
    band: np.ndarray          # bool per held protein: halo within halo / 2 of an owned anchor
    n_a: int = 0
    n_b: int = 0


@dataclass
class Plan:
    """The partition of one state into G windows (identical on every rank)."""

    owner: np.ndarray         # rank per global protein
    windows: List[Window]
    halo: float
    xw: np.ndarray            # anchors: wrapped x of every protein at the partition
    xs: np.ndarray            # the anchors sorted
    xs_order: np.ndarray      # ... and their global indices
    held: List[np.ndarray]    # per rank: bool per global protein, held by its window
    own_x: List[np.ndarray]   # per rank: sorted anchors of its owned proteins
    near: List[np.ndarray]    # per rank: bool per global protein, owned or in its band
    L: float = 0.0

    def within(self, x: float, h: float) -> np.ndarray:
        """Global indices of the proteins whose anchor is within h of x (periodic)."""
        L = self.L
        lo, hi = x - h, x + h
        spans = [(lo, hi)]
        if lo < -L / 2:
            spans = [(lo + L, L / 2), (-L / 2, hi)]
        elif hi >= L / 2:
            spans = [(lo, L / 2), (-L / 2, hi - L)]
        idx = [self.xs_order[np.searchsorted(self.xs, a, "left"):np.searchsorted(self.xs, b, "right")]
               for a, b in spans]
        return np.concatenate(idx) if len(idx) > 1 else idx[0]


def _dist_to_set(xs: np.ndarray, mask: np.ndarray, L: float) -> np.ndarray:
    """Periodic distance of every sorted anchor xs[i] to the nearest xs[j]
    with mask[j] (0 for the members themselves): the nearest member at or
    below and at or above each position by running max / min of the member
    positions — O(N), no search."""
    n = xs.size
    if not mask.any():
        return np.full(n, np.inf)
    idx = np.arange(n)
    prev = np.maximum.accumulate(np.where(mask, idx, -1))
    nxt = np.minimum.accumulate(np.where(mask, idx, n)[::-1])[::-1]
    first, last = int(np.argmax(mask)), n - 1 - int(np.argmax(mask[::-1]))
    xp = np.where(prev >= 0, xs[np.maximum(prev, 0)], xs[last] - L)  # across the seam: the last member − L
    xn = np.where(nxt < n, xs[np.minimum(nxt, n - 1)], xs[first] + L)
    return np.minimum(xs - xp, xn - xs)


def make_plan(p: capi.Params, hs: capi.HostState, G: int, halo: float, margin: float = 0.0) -> Plan:
    L = p.box_x
    n_a, n = hs.n_a, hs.n_a + hs.n_b
    xw = wrap(ref_x(hs), L)
    lab = units(hs)
    # by the unit's lead; the cuts sit half a slab off the periodic seam (x =
    # ±L/2), which lies inside slab G − 1: a complex whose members straddle
    # the seam rotates about a centre of mass far from all of them (no
    # minimum image, main.cpp:1068-1131), so its members sweep hundreds of Å
    # in a few dozen steps — inside a slab they fail no check
    slab = np.floor((xw[lab] + L / 2) / (L / G) + 0.5).astype(np.int64) % G
    owner = slab
    band_w = halo / 2
    order = np.argsort(xw, kind="stable")
    xs = xw[order]
    windows, own_x, near, held_all = [], [], [], []
    for r in range(G):
        own = owner == r
        own_s = own[order]
        own_x.append(xs[own_s])
        d = np.empty(n)
        d[order] = _dist_to_set(xs, own_s, L)
        held = own | (d < halo + margin)
        band = ~own & (d < band_w)
        near.append(own | band)
        # a band protein's whole unit is held: its local computation then
        # sees every member (a unit is moved and decided as one)
        mark = np.zeros(n, dtype=bool)
        mark[lab[band]] = True
        held |= mark[lab]
        held_all.append(held)
        gids = np.flatnonzero(held).astype(np.int32)
        w = Window(gids=gids, own=own[gids].astype(np.uint8), band=band[gids],
                   n_a=int((gids < n_a).sum()), n_b=int((gids >= n_a).sum()))
        windows.append(w)
    return Plan(owner=owner, windows=windows, halo=halo, xw=xw, xs=xs, xs_order=order, held=held_all,
                own_x=own_x, near=near, L=L)


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


def _components(nodes: np.ndarray, edges: np.ndarray) -> List[np.ndarray]:
    """Connected components of a small graph (nodes sorted; edges [m, 2])."""
    lab = np.arange(nodes.size)
    if edges.size:
        s = np.searchsorted(nodes, edges[:, 0])
        t = np.searchsorted(nodes, edges[:, 1])
        while True:
            m = np.minimum(lab[s], lab[t])
            new = lab.copy()
            np.minimum.at(new, s, m)
            np.minimum.at(new, t, m)
            new = new[new]
            if np.array_equal(new, lab):
                break
            lab = new
    return [nodes[lab == v] for v in np.unique(lab)]


# ---------------------------------------------------------------- one rank
class SlabRank:
    """Rank `rank` of a G-slab trajectory.  make_engine(params) returns a fresh
    handle with the kmc_dd_* methods for a window's proteins."""

    def __init__(self, p: capi.Params, rank: int, comm, make_engine: Callable, halo: float = 900.0,
                 gather_every: int = 0, margin: Optional[float] = None, lead: Optional[float] = None):
        self.p = p
        self.rank = rank
        self.comm = comm
        self.G = comm.world
        self.make_engine = make_engine
        self.halo = float(halo)
        # the window holds `margin` Å beyond the halo, so that a unit joined
        # across the cut can move to its new owner without a re-partition (C1)
        self.margin = float(400.0 if margin is None else margin)
        self._lead = lead  # None: min(200, S / 2); 0: no pre-emptive re-partition (tests of the rollback)
        self.gather_every = gather_every  # assemble the global state every k steps (tests: 1)
        self.eng = None
        self.eng_ok = True
        self.grow = 0  # output-list growth carried to the handles of a rebuild (kmc_list_growth)
        self.plan: Optional[Plan] = None
        self.win: Optional[Window] = None
        self.step_no = 0
        self.counters = np.zeros(5, dtype=np.int32)
        self.ckpt: Optional[capi.HostState] = None
        self.history: list = []  # global records since the checkpoint (replay check)
        self.stats = dict(steps=0, rebuilds=0, rebuild_bond=0, rebuild_jumpers=0, transfers=0, moved=0,
                          rollbacks=0, replayed=0, xcol=0, xbond=0, exchanged=0, verified=0, jumpers=0, held=0,
                          owned=0, why=[],
                          sec=dict(step=0.0, exchange=0.0, finish=0.0, jumpers=0.0, gather=0.0, transfer=0.0,
                                   rebuild=0.0))
        self.last_global: Optional[capi.HostState] = None
        self._xc = (0, 0)
        self._njump = 0  # jumpers after the last step, all slabs
        # debug (KMC_SLABS_CHECK=1): the window's bond graph and extent bounds
        # validated (kmc_host_validate) after every exchange
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
        sub = self.stats.setdefault("rebuild_sec", dict(plan=0.0, window=0.0, create=0.0, set_state=0.0,
                                                        lists=0.0))
        t0 = time.perf_counter()
        self.ckpt = hs.copy()
        self.ckpt.counters[:] = self.counters
        self.ckpt.step = self.step_no
        self.history = []
        self.plan = make_plan(self.p, hs, self.G, self.halo, self.margin)
        w = self.plan.windows[self.rank]
        self.win = w
        t1 = time.perf_counter()
        ws = window_state(hs, w)
        rl, mono, cis = derived_counts(hs)
        c = self.counters
        ctl5 = [c[0] - (rl + mono + cis), c[1] - rl, c[2] - cis, c[3] - mono, c[4]] if self.rank == 0 else [0] * 5
        t2 = time.perf_counter()
        if self.eng is not None:
            self.eng.close()
            self.eng = None
        q = capi.Params.from_buffer_copy(self.p)
        q.n_a, q.n_b = w.n_a, w.n_b
        self.q = q
        self.eng = self.make_engine(q)
        if self.grow:
            self.eng.set_list_growth(self.grow)
        t3 = time.perf_counter()
        self.eng.dd_set_state(ws, w.gids, w.own, ctl5)
        t4 = time.perf_counter()
        self.eng_ok = True
        self._xc = (0, 0)
        self._njump = 0
        self._set_lists()
        t5 = time.perf_counter()
        for k, a, b in (("plan", t0, t1), ("window", t1, t2), ("create", t2, t3), ("set_state", t3, t4),
                        ("lists", t4, t5)):
            sub[k] += b - a
        self.stats["rebuilds"] += 1

    def _set_lists(self) -> None:
        """The window's exchange plan from the partition: it sends its owned
        proteins each other window holds (to each in increasing global index)
        and receives every protein it holds but does not own from its owner."""
        w, plan, G = self.win, self.plan, self.G
        own = w.own == 1
        own_g = w.gids[own]
        send, self.send_n = [], [0] * G
        for dst in range(G):
            if dst == self.rank:
                continue
            g = own_g[plan.held[dst][own_g]]
            send.append(np.searchsorted(w.gids, g).astype(np.int32))
            self.send_n[dst] = int(g.size)
        src_of = plan.owner[w.gids]
        recv, self.recv_n = [], [0] * G
        for src in range(G):
            if src == self.rank:
                continue
            loc = np.flatnonzero((src_of == src) & ~own).astype(np.int32)
            recv.append(loc)
            self.recv_n[src] = int(loc.size)
        self.send_first = [int(x) for x in np.concatenate([[0], np.cumsum(self.send_n)[:-1]])]
        self.recv_first = [int(x) for x in np.concatenate([[0], np.cumsum(self.recv_n)[:-1]])]
        send_ids = np.concatenate(send) if send else np.zeros(0, np.int32)
        recv_ids = np.concatenate(recv) if recv else np.zeros(0, np.int32)
        self.n_send, self.n_recv = int(send_ids.size), int(recv_ids.size)
        self.n_verify = int(w.band[recv_ids].sum())
        self.eng.dd_plan(send_ids, recv_ids, w.own, w.band.astype(np.uint8))
        self.stats["held"] = int(w.gids.size)
        self.stats["owned"] = int(own.sum())

    def global_state(self) -> capi.HostState:
        """Collective: the trajectory's state assembled from every slab's owned proteins."""
        w = self.win
        ids = np.flatnonzero(w.own).astype(np.int32)
        beads, ints = self.eng.dd_export(ids)
        rec = ids < w.n_a
        for f in range(8):  # links local + 1 -> global + 1
            col = ints[:, f]
            m = ((rec & ((f == 2) | (f == 4))) | (~rec & (f >= 4))) & (col > 0)
            col[m] = w.gids[col[m] - 1] + 1
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
        a one-element capi.OBS_DTYPE array).  An error on this rank that the
        others cannot see (outside the per-step all-gather) aborts the comm."""
        try:
            return self._step()
        except SlabError:
            raise  # raised on every rank alike (from the all-gathered shares)
        except BaseException:
            self.comm.abort()
            raise

    def _step(self) -> np.ndarray:
        rec = self._one()
        tries = 0
        while rec is None:  # a check failed on some slab: back to the step before, re-partition, retry
            tries += 1
            if tries > MAX_TRIES or self.halo > 64 * self.p.box_x:
                raise SlabError(f"step {self.step_no + 1} does not pass its checks after {tries - 1} retries "
                                f"(halo {self.halo:.0f} Å): {self.stats['why'][-3:]}")
            # a repeated failure, or one right after the partition (nothing to
            # replay: the same partition would fail again), widens the halo
            self._recover(widen=tries > 1 or not self.history)
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

    @property
    def lead(self) -> float:
        """How far ahead of a failure the jumper checks re-partition: a protein
        moves at most this far in one step (association snaps and lay-downs ≈
        180 Å), so a jumper that passes the checks with S − lead
        passes them with S after the next step."""
        return min(200.0, self.S / 2) if self._lead is None else self._lead

    def _jumper_check(self, ids: np.ndarray, xs: np.ndarray):
        """The listed proteins (displaced more than S − lead from their anchors):
        (J_A / J_B failures of the jumpers proper — displaced more than S —,
        warnings: any of them failing the checks with S − lead)."""
        if ids.size == 0:
            return 0, 0
        L, S, lead = self.p.box_x, self.S, self.lead
        xw = wrap(xs, L)
        g = self.win.gids[ids]
        dx = np.abs(xw - self.plan.xw[g])
        jump = np.minimum(dx, L - dx) > S
        dj = periodic_dist(xw, self.plan.own_x[self.rank], L)
        fail, warn = jump & (dj > S), dj > S - lead  # J_B
        for r in range(self.G):
            if r == self.rank:
                continue
            far = ~self.plan.near[r][g]
            if far.any():
                dr = periodic_dist(xw[far], self.plan.own_x[r], L)
                fail[far] |= jump[far] & (dr < R_INT + S)  # J_A
                warn[far] |= dr < R_INT + S + lead
        if fail.any():  # (diagnostics: global index, anchor, x now)
            self._jfail = [(int(a), round(float(self.plan.xw[a]), 1), round(float(b), 1))
                           for a, b in zip(g[fail][:4], xw[fail][:4])]
        return int(fail.sum()), int(warn.sum())

    def _cross_units(self, rep) -> Optional[list]:
        """The units joined by this step's cross-slab bonds, as sorted global
        indices, from this window's links (None: more bonds than listed)."""
        if rep.n_xb == 0:
            return []
        if rep.n_xb > capi.DD_XCAP:
            return None
        w = self.win
        pairs = rep.cross_bonds()
        nodes = np.unique(pairs.ravel()).astype(np.int32)
        edges = [pairs]
        frontier = nodes
        while frontier.size:
            _, ints = self.eng.dd_export(frontier)
            rec = frontier < w.n_a
            nb = []
            for f in range(8):
                m = ((rec & ((f == 2) | (f == 4))) | (~rec & (f >= 4))) & (ints[:, f] > 0)
                if m.any():
                    e = np.stack([frontier[m], ints[m, f] - 1], axis=1)
                    edges.append(e)
                    nb.append(e[:, 1])
            new = np.setdiff1d(np.concatenate(nb) if nb else np.zeros(0, np.int32), nodes).astype(np.int32)
            nodes = np.union1d(nodes, new).astype(np.int32)
            frontier = new
        comps = _components(nodes, np.concatenate(edges).astype(np.int64))
        return [w.gids[c].astype(np.int64) for c in comps]

    def _step_exchange(self) -> Optional[np.ndarray]:
        sec = self.stats["sec"]  # host seconds by phase (tools/slab_rate.py)
        t0 = time.perf_counter()
        part, fail, err = None, False, None
        try:
            part = self.eng.dd_step(self.comm.send_address(self), self.S - self.lead)[0].copy()
        except Exception as e:  # noqa: BLE001 — every rank must learn of it (the shares below)
            self.eng_ok = False
            if _engine_error(e) == capi.ERR_CAPACITY:
                fail = True  # the lists were full: redo the step from the checkpoint with larger ones
                self.grow = max(self.grow, int(getattr(self.eng, "list_growth", 0)))
            else:
                err = f"rank {self.rank}: {e!r}"
        t1 = time.perf_counter()
        sec["step"] += t1 - t0
        # the halo exchange: my owned proteins' end state to every window holding them
        self.comm.exchange(self.rank, self)
        t2 = time.perf_counter()
        sec["exchange"] += t2 - t1
        bad = jbad = jwarn = nj = 0
        dcol = dbond = 0
        xunits: Optional[list] = []
        if self.eng_ok:
            rep = self.eng.dd_finish()
            t3 = time.perf_counter()
            sec["finish"] += t3 - t2
            bad = rep.bad
            dcol, dbond = rep.xcol - self._xc[0], rep.xbond - self._xc[1]
            self._xc = (rep.xcol, rep.xbond)
            self.stats["exchanged"] += self.n_recv
            self.stats["verified"] += self.n_verify
            nj = rep.n_jump
            jbad, jwarn = self._jumper_check(*rep.jumpers())
            xunits = self._cross_units(rep)
            if self.check:
                from . import engine as _engine

                rc = _engine.host_validate(self.q, self.eng.get_state())
                if rc != 0:
                    err = (f"rank {self.rank}: window state invalid ({rc}) after the exchange of step "
                           f"{self.step_no + 1}: {_engine.load_library().kmc_host_last_error().decode()}")
            sec["jumpers"] += time.perf_counter() - t3
        t5 = time.perf_counter()
        # the step's record from every slab's share, the checks and triggers:
        # every rank decides alike
        shares = self.comm.allgather(self.rank, (part, bad, jbad, dbond, dcol, nj, xunits, fail, err, jwarn))
        sec["gather"] += time.perf_counter() - t5
        errs = [s[8] for s in shares if s[8]]
        if errs:
            raise SlabError("; ".join(errs))
        if any(s[7] for s in shares):
            self.stats["why"].append((self.step_no + 1, "capacity", 0, 0))
            return None
        if any(s[1] or s[2] for s in shares):
            self.stats["why"].append((self.step_no + 1, "verify" if any(s[1] for s in shares) else "jumper",
                                      sum(s[1] for s in shares), sum(s[2] for s in shares),
                                      getattr(self, "_jfail", None)))
            self._jfail = None
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
        gs = None
        if any(s[6] is None for s in shares):  # more cross-slab bonds than listed
            gs = self.global_state()
            self.stats["rebuild_bond"] += 1
            self._rebuild_from(gs)
        else:
            joined = [u for s in shares for u in s[6]]
            if joined:
                t6 = time.perf_counter()
                ok = self._transfer(joined)
                sec["transfer"] += time.perf_counter() - t6
                if not ok:
                    gs = self.global_state()
                    self.stats["rebuild_bond"] += 1
                    self._rebuild_from(gs)
        if gs is None and any(s[9] for s in shares):
            # a jumper within one step's reach of failing its checks: re-partition
            # now rather than roll back later
            gs = self.global_state()
            self.stats["rebuild_jumpers"] += 1
            self._rebuild_from(gs)
        if self.gather_every and self.step_no % self.gather_every == 0:
            self.last_global = gs if gs is not None else self.global_state()
        return rec

    # -- a unit joined across the cut moves to one owner ---------------------
    def _transfer(self, joined: list) -> bool:
        """Collective (every rank, the same `joined`): give each joined unit to
        the owner of its lowest-index member, keeping every window.  False if
        the partition cannot take it (C1 / C2): the caller re-partitions."""
        plan, L, G = self.plan, self.p.box_x, self.G
        nodes = np.unique(np.concatenate(joined))
        edges = [np.stack([u[:-1], u[1:]], axis=1) for u in joined if u.size > 1]
        groups = _components(nodes, np.concatenate(edges) if edges else np.zeros((0, 2), np.int64))
        owner2 = plan.owner.copy()
        for u in groups:
            owner2[u] = plan.owner[u.min()]
        moved = np.flatnonzero(owner2 != plan.owner)
        if moved.size == 0:
            return True
        # C1: the new owner holds every protein within the halo of a moved anchor
        for g in moved:
            if not plan.held[owner2[g]][plan.within(plan.xw[g], self.halo + 1.0)].all():
                return False
        # the band can change only within halo / 2 of a moved anchor
        X = np.unique(np.concatenate([plan.within(plan.xw[g], self.band + 1.0) for g in moved]))
        affected = sorted(set(owner2[moved].tolist()) | set(plan.owner[moved].tolist()))
        own_x = list(plan.own_x)
        near = list(plan.near)
        for r in affected:
            own_x[r] = _resorted(plan.own_x[r], plan.xw, moved, plan.owner, owner2, r)
            nr = plan.near[r].copy()
            hx = X[plan.held[r][X]]
            nr[X] = False
            nr[hx] = (owner2[hx] == r) | (periodic_dist(plan.xw[hx], own_x[r], L) < self.band)
            near[r] = nr
        w = self.win
        own_loc = owner2[w.gids] == self.rank
        band_loc = near[self.rank][w.gids] & ~own_loc
        # C2: a protein that joins my band must have its unit held whole here:
        # none of its links was cut at the exchange
        newb = np.flatnonzero(band_loc & ~w.band).astype(np.int32)
        cut = self.eng.dd_cut_count(newb) if newb.size else 0
        if not all(self.comm.allgather(self.rank, cut == 0)):
            return False
        plan.owner = owner2
        plan.own_x = own_x
        plan.near = near
        w.own = own_loc.astype(np.uint8)
        w.band = band_loc
        self._set_lists()
        self.stats["transfers"] += 1
        self.stats["moved"] += int(moved.size)
        return True

    def _recover(self, widen: bool) -> None:
        """Back to the checkpoint, replay to the last good step, re-partition
        there (with a wider halo on a repeated failure)."""
        self.stats["rollbacks"] += 1  # a statistic: the retries of one step are bounded in step()
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


def _resorted(own_x: np.ndarray, xw: np.ndarray, moved: np.ndarray, owner: np.ndarray, owner2: np.ndarray,
              r: int) -> np.ndarray:
    """Rank r's sorted owned anchors after the moves (the others unchanged)."""
    out = own_x
    lose = moved[(owner[moved] == r) & (owner2[moved] != r)]
    gain = moved[(owner[moved] != r) & (owner2[moved] == r)]
    if lose.size:
        keep = np.ones(out.size, bool)
        for x in xw[lose]:
            j = np.searchsorted(out, x)
            while not keep[j]:  # equal anchors: drop the next copy
                j += 1
            keep[j] = False
        out = out[keep]
    if gain.size:
        xg = np.sort(xw[gain])
        out = np.insert(out, np.searchsorted(out, xg), xg)
    return out


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
              halo: float = 900.0, gather_every: int = 0, on_step: Optional[Callable] = None,
              margin: Optional[float] = None, lead: Optional[float] = None):
    """G slabs as threads of this process (e.g. G handles on one GPU).
    Returns (records[steps], ranks).  on_step(rank0, k, rec) after each step on rank 0."""
    comm = LocalComm(G)
    ranks = [SlabRank(p, r, comm, make_engine, halo=halo, gather_every=gather_every, margin=margin, lead=lead)
             for r in range(G)]
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
