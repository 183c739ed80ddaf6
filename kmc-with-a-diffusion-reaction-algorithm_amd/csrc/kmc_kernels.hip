// kmc_kernels.hip — HIP/CDNA4 kernels of one KMC time step
// (reference: /root/reference/main.cpp:461-2308).
//
// Parallel restatement of a sequential, order-dependent loop.  The reference
// visits units (free receptor, cis dimer, free ligand, ligand-rooted complex)
// in index order and tests each trial move against R_new, which already holds
// every earlier unit's accepted move (Gauss–Seidel, main.cpp:640-664).  Here:
//
//   1. classify + BFS      every protein learns the key (trigger index) of the
//                          unit that moves it; complexes get their BFS member
//                          order (main.cpp:514-562)
//   2. propose             every unit computes its trial move from R with its
//                          own keyed Philox draws (independent of order)
//   3. records             old and proposed positions of every protein go into
//                          a 130 Å xy cell list (counting sort)
//   4. resolve             a unit's fate depends only on lower-keyed units near
//                          it: decided units are read, undecided ones block;
//                          rounds until every unit is decided — exactly the
//                          sequential outcome
//   5. commit              rejected units copy R back into R_new
//   6. reactions           candidate pairs from the cell list; the reference's
//                          greedy loop order (main.cpp:1877-2058) is reproduced
//                          as a lexicographic-first greedy matching
//   7. dissociation, observables
//
// Every floating-point expression mirrors the reference's operation order;
// the file is compiled with -ffp-contract=off.
#include "kmc_device.h"

namespace kmcd {

// Output list with NSHARD counter shards: workgroup b appends to shard
// b % NSHARD, which owns data[shard·cap, (shard+1)·cap).  One device-scope
// word sustains only ≈90 atomics/µs (MI355X_MICROARCH.md, dequeue / fan-in),
// so thousands of workgroups appending to one counter would serialise.
#ifndef NSHARD  // counter shards per list, a power of two <= 64 (sl_prefix scans them in one wave)
#define NSHARD 64
#endif
struct SList {
  int2* data;
  uint32_t* cnt;  // [NSHARD]
  uint32_t cap;   // entries per shard
};

struct Dev {
  Beads cur, nxt;
  int32_t* a_int;  // [5][NA]  st2 st3 nei2 nei4 nei3 (nei: reference 1-based)
  int32_t* b_int;  // [8][NB]  st1..4 nei1..4
  int32_t* owner;  // [N] key (reference index of the lead protein) of the unit that moves slot p
  int32_t* id_of;    // [N] slot -> reference protein index (0-based)
  int32_t* slot_of;  // [N] reference protein index -> slot
  uint8_t* ukind;  // [N] unit kind keyed at p
  uint32_t* ustate;  // [N] (step<<2)|S this step; older tag = accepted
  uint32_t* moved;   // [N] step tag (main.cpp:122)
  int32_t* cx_off;   // [NB]
  int32_t* cx_size;  // [NB]
  int32_t* cx_nb;    // [NB] ligands in complex
  uint32_t* cx_ext;  // [NB] by root: a member of the complex broke the extent bound in k_move_members (k_cx_check
                     // reads and clears it)
  int32_t* members;  // [mcap] BFS rows of the registered complexes (kept across steps, BFS order)
  int32_t* shuf;     // [mcap] the rows after this step's multi-ligand shuffles (cluster.log)
  int4* mrec;        // [mcap] member records of rows of <= CXL members (register_complex)
  double* cxp;       // [NB][16] rigid-move parameters of the complex rooted at lb (cx_params)
  uint32_t* shuf_tag;  // [NB] step whose shuffled row of root lb is in shuf
  uint32_t mcap;     // members[] capacity (3N): rows are appended until a full rebuild
  int32_t* croot;    // [N] slot of the root ligand of the protein's registered complex | CROOT_BIG, -1 none
  uint32_t* cx_alive;  // [NB] 1 while ligand lb roots a registered complex
  uint32_t* bfs_cand;  // [NB] step tag: ligand lb runs the BFS this step
  int32_t* dlist;    // [2][N] proteins whose bonds changed during step s (list s & 1)
  uint32_t* pend;    // [N] round tag: unit still waiting (resolution pass C)
  unsigned long long* ccnt;  // [N] round 0 of unit u's conflict entries (k_col_resolve; 0 between steps)
  int32_t* overflow; // [NB]
  int4* cx_list;     // [NB] descriptors of the registered complexes (kept across steps; cx_params, k_cx_check)
  int4* cx_heavy;    // [NB] descriptors for k_complex_heavy: larger complexes, and those k_cx_check
                     //      moved but whose lay-down / alignment changes beads
  // Home list (§records): every protein has a home position hp in an order
  // sorted by its home cell — the cell of its reference point at the last
  // re-sort — and its two records of a step (old and proposed position) live
  // at rec[2 hp], rec[2 hp + 1].  Rebuilt only with the slot order.
  uint2* home;          // [N] slot -> {hp, home cell cx | cy << 16}
  int32_t* hstart;      // [ncell+1] first home position of each (row, kind, column) cell
  struct Rec* rec;      // [2N] records, home order; written by the kernels that move the protein
  int4* outl;           // [outl_cap] records more than one cell from their home cell: {record, cx, cy, -}
  uint32_t outl_cap;
  int2* tout;           // [ntiles][TOUT_CAP] the outliers whose cell lies in a pair-scan tile's block + halo:
                        //   {record, cx | cy << 16}
  uint32_t* tout_n;     // [ntiles] entries of each tile's bucket this step (zeroed by the tile's k_pair_scan)
  uint32_t* rec_step;   // [2N] debug (KMC_DEBUG_RECS): the step each record was last written in
  int4* dense;          // [dense_cap] tiles whose records overflow the pair scan's LDS: {x0 | y0 << 16,
                        // w | h << 16, the tile's outlier bucket or -1 (the whole outlier list), its entries}
  uint32_t dense_cap;
  SList cand;           // collision candidates (proposal record, other record)
  SList conf;           // conflict entries (u, kq | isnew<<31)
  SList plist;          // units with conflict entries (u, 0)
  SList rej;            // units rejected this step (u, 0)
  SList pairs;          // reaction candidates (receptor, partner)
  int32_t* pq_units;    // [N] units still pending after round 0 (k_col_resolve)
  int2* pq_ent;         // [conf capacity] conflict entries left pending by round 0 (k_col_resolve)
  uint32_t* shard_cnt;  // [5][NSHARD] counters of the lists above
  int32_t* obs_part;    // [blocks][8] per-block observable partials
  uint64_t* rl_keys;    // [cap]
  uint64_t* cis_keys;   // [cap]
  uint64_t* ent;        // [2*cap] greedy scratch
  int32_t* gi32;        // [6*cap] greedy scratch
  uint32_t cap_edges;   // power of two
  int32_t* bfs_queue;   // [N]
  uint32_t* vtag;       // [N]
  Ctl* ctl;
  struct kmc_obs_dev* obs;
  // decomposed trajectories (KParams::dd, kmc_dd_set_state), by local reference index: the trajectory's
  // global reference index (the random-stream key), 1 if this slab owns the protein, x of bead [1][1] when
  // the slab's window was set (kmc_dd_drift)
  const int32_t* gid;
  const uint8_t* dd_own;
  const double* dd_x0;
  DDRep* dd_rep;  // the window's per-step exchange report (kmc_dd_finish): cross-slab bonds, jumpers, checks
  uint32_t nkeys;  // unit keys (local reference indices) are < nkeys = N: a key outside latches ERR_RESOLVE
};

// one record (32 B): float reference point, ids, cis site
struct alignas(16) Rec {
  float4 pos;   // x, y of bead [1][1]; z span (receptor: lowest/highest domain; ligand: centre, then
                // the first word of its subunit offsets, lig_pack)
  int2 id;      // {slot | cell code << 25 | st3 << 29 | st2 << 30 | isnew << 31, owner key}
  float2 site;  // receptor [3][3] site xy (reaction prefilter); ligand: the other two words of lig_pack
};
#define RID_PID 0x00ffffff  // the slot (global records) or the home position (the pair scan's LDS copies)
#define RID_LIG (1 << 24)   // a ligand's record
#define RID_CODE_SHIFT 25  // 4-bit cell code: (dy + 1) * 3 + (dx + 1), the record's cell relative to its home
                           // cell; RID_OUT: more than one cell away (the record is on the outlier list)
#define RID_OUT 15
#define RID_ST3 (1 << 29)
#define RID_ST2 (1 << 30)
__device__ __forceinline__ int rec_code(int2 id) { return (id.x >> RID_CODE_SHIFT) & 15; }

struct kmc_obs_dev {  // == kmc_obs
  int64_t step;
  double t;
  int32_t rl, mono, cis, bond;
  double cluster_size;
  int32_t maxc, tot_prot, tot_clu, reserved;
};

// ---------------------------------------------------------------- state access
#define A_ST2(d, i) (d).a_int[0 * (size_t)NA + (i)]
#define A_ST3(d, i) (d).a_int[1 * (size_t)NA + (i)]
#define A_NEI2(d, i) (d).a_int[2 * (size_t)NA + (i)]
#define A_NEI4(d, i) (d).a_int[3 * (size_t)NA + (i)]
#define A_NEI3(d, i) (d).a_int[4 * (size_t)NA + (i)]
#define B_ST(d, b, j) (d).b_int[(size_t)((j)-1) * NB + (b)]
#define B_NEI(d, b, j) (d).b_int[(size_t)(4 + (j)-1) * NB + (b)]

// a unit key outside [0, N): a protein no unit claimed (inconsistent bond
// graph) or a corrupt record — latched as an error, never used as an index
__device__ __forceinline__ bool bad_key(const Dev& d, int key) {
  if ((uint32_t)key < d.nkeys) return false;
  atomicOr(&d.ctl->err, ERR_RESOLVE);
  return true;
}
__device__ __forceinline__ uint32_t state_of(const Dev& d, int key, uint32_t step) {
  if (bad_key(d, key)) return S_REJ;
  uint32_t v = ld_state(&d.ustate[key]);
  return (v >> 2) == (step & 0x3fffffffu) ? (v & 3u) : S_ACC;  // untouched this step: accepted
}
__device__ __forceinline__ void set_state(const Dev& d, int key, uint32_t step, uint32_t s) {
  if (bad_key(d, key)) return;
  st_state(&d.ustate[key], ((step & 0x3fffffffu) << 2) | s);
}

// random-stream key of local reference index r: the global reference index
// when this handle holds one slab's window of a decomposed trajectory (the
// local numbering is monotone in the global one, so every order comparison
// of local indices is the global one; only the keyed draws need the map)
__device__ __forceinline__ uint32_t rkey(const KParams& P, const Dev& d, int r) {
  return P.dd ? (uint32_t)d.gid[r] : (uint32_t)r;
}
// protein of local reference index r is owned by this slab (always, outside
// a decomposed trajectory)
__device__ __forceinline__ bool dd_owned(const KParams& P, const Dev& d, int r) { return !P.dd || d.dd_own[r]; }
// a bond formed between local proteins a and b (reference indices): one this
// slab owns and one it holds as a halo copy joins units of two slabs — counted
// and listed for the driver, which moves the joined unit to one owner
__device__ __forceinline__ void dd_xbond(const Dev& d, int a, int b) {
  if (d.dd_own[a] == d.dd_own[b]) return;
  atomicAdd(&d.ctl->dd_xbond, 1u);
  const uint32_t k = atomicAdd((uint32_t*)&d.dd_rep->n_xb, 1u);
  if (k < DD_XCAP) {
    d.dd_rep->xb[k][0] = a;
    d.dd_rep->xb[k][1] = b;
  }
}

__device__ __forceinline__ int cell_x(const KParams& P, double x) {
  int c = (int)__builtin_floor((x - P.gx0) / P.cs);
  return c < 0 ? 0 : (c >= P.ncx ? P.ncx - 1 : c);
}
__device__ __forceinline__ int cell_y(const KParams& P, double y) {
  int c = (int)__builtin_floor((y - P.gy0) / P.cs);
  return c < 0 ? 0 : (c >= P.ncy ? P.ncy - 1 : c);
}

#define CROOT_BIG (1 << 30)  // croot flag: the complex has more than CXL members (global-memory path)
#define CXL 16  // members of a complex moved by the streamed path and staged in LDS by k_complex_heavy

// slot for each calling lane (call from the lanes that emit)
__device__ __forceinline__ uint32_t wave_slot(uint32_t* ctr) {
  const uint64_t mask = __ballot(1);
  const int lane = __lane_id();
  const int leader = __ffsll((unsigned long long)mask) - 1;
  const uint32_t rank = __popcll(mask & ((1ull << lane) - 1ull));
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(ctr, (uint32_t)__popcll(mask));
  base = __shfl(base, leader, 64);
  return base + rank;
}

// members[] range of qn entries for each calling lane: one atomic per wave
// (the lanes that reach it together), not per complex — a single counter
// word serialises its atomics (MI355X_MICROARCH.md)
__device__ __forceinline__ uint32_t wave_alloc(uint32_t* ctr, uint32_t qn) {
  const uint64_t mask = __ballot(1);
  const int lane = __lane_id(), leader = __ffsll((unsigned long long)mask) - 1;
  uint32_t pre = 0, tot = 0;
  for (uint64_t m = mask; m; m &= m - 1) {
    const int l = __ffsll((unsigned long long)m) - 1;
    const uint32_t v = (uint32_t)__shfl((int)qn, l, 64);
    pre += l < lane ? v : 0u;
    tot += v;
  }
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(ctr, tot);
  return (uint32_t)__shfl((int)base, leader, 64) + pre;
}

// ================================================================ 1. classify
// Unit kinds, main.cpp:584 (free receptor), 682-686 (cis dimer, moved at the
// lower index), 905 (single ligand = BFS component of size 1).
// CLASSIFY_PER slots per thread (their first loads issued together; chosen as
// k_diss_observe's count)
template <int CLASSIFY_PER>
__global__ void k_classify(KParams P, Dev d) {
  const int NA = P.NA, NB = P.NB;
  const int p0 = blockIdx.x * blockDim.x * CLASSIFY_PER + threadIdx.x;
  // the links / statuses and complex root of every slot of this thread first
  int n2[CLASSIFY_PER], n3[CLASSIFY_PER], s2[CLASSIFY_PER], r[CLASSIFY_PER];
#pragma unroll
  for (int k = 0; k < CLASSIFY_PER; ++k) {
    const int p = p0 + k * (int)blockDim.x;
    n2[k] = n3[k] = s2[k] = 0;
    r[k] = -1;
    if (p >= P.N) continue;
    if (p < NA) {
      n2[k] = A_NEI2(d, p);
      n3[k] = A_NEI3(d, p);
      s2[k] = A_ST2(d, p) | A_ST3(d, p);
    } else {
      const int b = p - NA;
      n2[k] = B_NEI(d, b, 2);
      n3[k] = B_NEI(d, b, 3);
      s2[k] = B_NEI(d, b, 4);
    }
    r[k] = d.croot[p];
    if (r[k] >= 0) r[k] &= ~CROOT_BIG;
  }
#pragma unroll
  for (int k = 0; k < CLASSIFY_PER; ++k) {
    const int p = p0 + k * (int)blockDim.x;
    if (p >= P.N) continue;
    uint8_t kind = U_NONE;
    int own = -1;
    if (p < NA) {
      const int i = p;
      if (s2[k] == 0) {
        kind = U_FREE_A;
        own = p;
      } else if (n2[k] == 0 && n3[k] != 0 && A_NEI3(d, n3[k] - 1) == i + 1 && A_NEI2(d, n3[k] - 1) == 0) {
        int q = n3[k] - 1;
        const bool lead = d.id_of[i] < d.id_of[q];  // moved at the lower reference index
        own = lead ? i : q;
        kind = lead ? U_DIMER : U_DIMER_P;
      }
    } else if (n2[k] == 0 && n3[k] == 0 && s2[k] == 0) {
      kind = U_FREE_B;
      own = p;
    }
    // a member of a complex registered in an earlier step and untouched since
    // (dissolved otherwise): its unit is that complex (new ones are registered
    // by k_bfs)
    if (r[k] >= 0) {
      own = r[k];
      if (r[k] == p) kind = U_COMPLEX;
    }
    d.ukind[p] = kind;
    d.owner[p] = own < 0 ? -1 : d.id_of[own];  // -1: member of a complex k_bfs registers this step
  }
}

// Complexes are kept from step to step: a BFS row depends only on the bond
// graph, which changes only where a bond formed or broke (k_match,
// k_diss_observe list those proteins).  At the end of each step (k_finalize,
// cx_dissolve_dirty) every complex containing a listed protein is dissolved
// (its members' croot reset) and its ligands, and the listed ligands, become
// BFS candidates of the next step; the BFS of the candidates (k_bfs)
// registers the new complexes.  A full rebuild — no complex kept — is
// k_cx_kill: launched by the host before the step after a re-sort, a new
// state or an undone chunk (and every step with KMC_FULL_BFS=1), or done by
// k_finalize itself when the appended rows fill half of members[] or a dirty
// list overflowed: every bonded ligand runs the BFS.
__device__ __forceinline__ void cx_reset_all(const KParams& P, const Dev& d, uint32_t tid, uint32_t nt) {
  for (uint32_t p = tid; p < (uint32_t)P.N; p += nt) d.croot[p] = -1;
  for (uint32_t b = tid; b < (uint32_t)P.NB; b += nt) d.cx_alive[b] = 0;
  if (tid == 0) {
    d.ctl->cx_cursor = 0;
    d.ctl->n_cx = 0;
    d.ctl->full_now = 1;
  }
}
__global__ void k_cx_kill(KParams P, Dev d) {
  cx_reset_all(P, d, blockIdx.x * blockDim.x + threadIdx.x, gridDim.x * blockDim.x);
}
// the complexes of the proteins whose bonds changed during `step` (dirty list
// step & 1), dissolved for step + 1 (k_finalize's workgroup)
__device__ __forceinline__ void cx_dissolve_dirty(const KParams& P, const Dev& d, uint32_t step) {
  const int NA = P.NA;
  const uint32_t li = step & 1, n = min(d.ctl->n_dirty[li], (uint32_t)P.N), next = step + 1;
  for (uint32_t t = threadIdx.x; t < n; t += blockDim.x) {
    const int p = d.dlist[(size_t)li * P.N + t];
    if (p >= NA) d.bfs_cand[p - NA] = next;
    const int r = d.croot[p] & ~CROOT_BIG;
    if (r < 0 || atomicExch(&d.cx_alive[r - NA], 0u) != 1u) continue;
    const int b = r - NA, off = d.cx_off[b], sz = d.cx_size[b];
    for (int i = 0; i < sz; ++i) {
      const int m = d.members[off + i];
      d.croot[m] = -1;
      if (m >= NA) d.bfs_cand[m - NA] = next;
    }
  }
}

// a bond of protein p formed or broke this step (dirty list of step & 1).
// Without ligands no complex exists and the list is never read.  A list that
// overflows (a protein can be listed several times) is not an error: the
// next step rebuilds every complex instead (k_finalize resets them all).
__device__ __forceinline__ void mark_bond_change(const KParams& P, const Dev& d, int p, uint32_t step) {
  if (P.NB == 0) return;
  const uint32_t li = step & 1;
  const uint32_t t = atomicAdd(&d.ctl->n_dirty[li], 1u);
  if (t < (uint32_t)P.N) d.dlist[(size_t)li * P.N + t] = p;
}

// ================================================================ BFS
// Complex of ligand root b: BFS over the bond graph exactly as
// main.cpp:525-561 (receptor neighbours res_nei[2], [3]; ligand neighbours
// res_nei[2], [3], [4]; a node is enqueued when first seen).  The root is the
// lowest-indexed ligand of its component; the BFS of any other ligand of the
// component finds a lower one among its members and registers nothing.
#define BFS_QCAP 32
#ifndef BFS_BATCH  // queued nodes whose links are loaded together (A/B builds)
#define BFS_BATCH 4
#endif

// the neighbours in three fixed slots (-1 = none), in BFS order
__device__ __forceinline__ void nbrs3(const KParams& P, const Dev& d, int x, int* y) {
  const int NA = P.NA, NB = P.NB;
  if (x < NA) {
    const int a = A_NEI2(d, x), b = A_NEI3(d, x);
    y[0] = a > 0 ? a - 1 : (b > 0 ? b - 1 : -1);
    y[1] = a > 0 && b > 0 ? b - 1 : -1;
    y[2] = -1;
  } else {
    const int lb = x - NA;
    const int v2 = B_NEI(d, lb, 2), v3 = B_NEI(d, lb, 3), v4 = B_NEI(d, lb, 4);
    y[0] = v2 > 0 ? v2 - 1 : -1;
    y[1] = v3 > 0 ? v3 - 1 : -1;
    y[2] = v4 > 0 ? v4 - 1 : -1;
  }
}

// Complex descriptor (cx_list / cx_heavy): x = root ligand lb | CXD_MOVED
// (rigid move already done by k_move_members), y = members[] offset, z = size |
// ligands << 16, w = the root's reference index (its random-stream key).
#define CXD_MOVED (1 << 30)
#define CXD_LB 0x3fffffff

// Register the component in queue q (q[t * STRIDE], t < qn, BFS order) rooted
// at ligand slot p: member row, owner keys, descriptor on cx_list (complexes
// of at most CXL members take the streamed path, larger ones the
// global-memory path of k_complex_heavy).
template <int STRIDE = 1>
__device__ __forceinline__ void register_complex(const KParams& P, const Dev& d, int p, const int* q, int qn) {
  const int NA = P.NA, NB = P.NB;
  uint32_t off = wave_alloc(&d.ctl->cx_cursor, (uint32_t)qn);
  if (off + qn > d.mcap) {  // cannot happen below mcap / 2 + N (k_cx_kill): the step is undone (kmc_step)
    atomicOr(&d.ctl->err, ERR_MEMBERS);
    qn = 0;
    off = 0;
  }
  int nb = 0;
  const int rootid = d.id_of[p];
#pragma unroll 4
  for (int t = 0; t < qn; ++t) {
    int m = q[t * STRIDE];
    d.members[off + t] = m;
    d.owner[m] = rootid;
    d.croot[m] = p | (qn > CXL ? CROOT_BIG : 0);
    nb += m >= NA;
  }
  d.cx_alive[p - NA] = 1;
  if (qn <= CXL) {
    // member records: slot + links encoded by BFS position (receptor {slot,
    // nei2, nei3, nei4 (site)}, ligand {slot, nei2, nei3, nei4}; a protein
    // link to position t is t + 1 for a receptor, NA + t + 1 for a ligand) —
    // the LDS image the complex kernels load in one coalesced access, every
    // step the complex is kept
    auto enc = [&](int v) -> int {
      if (v <= 0) return 0;
      for (int t = 0; t < qn; ++t)
        if (q[t * STRIDE] == v - 1) return (v - 1 < NA ? t : NA + t) + 1;
      atomicOr(&d.ctl->err, ERR_RESOLVE);  // a link leaving its component
      return 0;
    };
    for (int t0 = 0; t0 < qn; t0 += 4) {  // the links of four members in flight at once
      int4 r[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int t = t0 + i, m = t < qn ? q[t * STRIDE] : p;
        r[i].x = m;
        if (m < NA) {
          r[i].y = A_NEI2(d, m);
          r[i].z = A_NEI3(d, m);
          r[i].w = A_NEI4(d, m);
        } else {
          r[i].y = B_NEI(d, m - NA, 2);
          r[i].z = B_NEI(d, m - NA, 3);
          r[i].w = B_NEI(d, m - NA, 4);
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (t0 + i >= qn) break;
        r[i].y = enc(r[i].y);
        r[i].z = enc(r[i].z);
        if (r[i].x >= NA) r[i].w = enc(r[i].w);
        d.mrec[off + t0 + i] = r[i];
      }
    }
  }
  int b = p - NA;
  d.cx_off[b] = (int)off;
  d.cx_size[b] = qn;
  d.cx_nb[b] = nb;
  d.ukind[p] = U_COMPLEX;
  // the descriptor list is kept across steps too: a descriptor is current
  // while its root is alive with the same row offset (cx_current checks)
  const int4 desc = make_int4(b, (int)off, qn | nb << 16, rootid);
  const uint32_t slot = wave_slot(&d.ctl->n_cx);
  if (slot < d.mcap / 2) d.cx_list[slot] = desc;
  else atomicOr(&d.ctl->err, ERR_MEMBERS);
}

// One thread per bonded ligand; the queue lives in LDS, one column per thread
// (consecutive lanes, consecutive banks): a dynamically indexed private
// array would go to scratch (400 B/lane).  The lower-ligand test is made once
// over the finished queue (independent loads), so each BFS node costs one
// round of link loads.  Components larger than BFS_QCAP go to the overflow
// path.
__global__ void __launch_bounds__(256) k_bfs(KParams P, Dev d) {
  __shared__ int qs[BFS_QCAP * 256];
  const int NA = P.NA, NB = P.NB;
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= NB) return;
  if (!d.ctl->full_now && d.bfs_cand[b] != d.ctl->step) return;  // its complex is kept (k_cx_kill)
  if (B_NEI(d, b, 2) == 0 && B_NEI(d, b, 3) == 0 && B_NEI(d, b, 4) == 0) return;
  int* q = qs + threadIdx.x;  // q[t * 256]
  int p = NA + b;
  const int pid = d.id_of[p];
  auto lower = [&](int qn) {  // a lower ligand among the first qn members roots the component
    bool lw = false;
    for (int t0 = 1; t0 < qn; t0 += 8) {  // eight independent loads in flight
      int id[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int t = t0 + i, v = t < qn ? q[t * 256] : 0;
        id[i] = v >= NA ? d.id_of[v] : pid;
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) lw |= id[i] < pid;
    }
    return lw;
  };
  int qn = 1, head = 0;
  q[0] = p;
  uint64_t bloom = 1ull << (((uint32_t)p * 0x9E3779B1u) >> 26);
  // nodes are expanded in queue order; the links of the next (up to) BFS_BATCH
  // queued nodes are loaded together first (one round of loads per batch
  // instead of per node)
  while (head < qn) {
    const int nb = min(BFS_BATCH, qn - head);
    int y[BFS_BATCH][3];
#pragma unroll
    for (int i = 0; i < BFS_BATCH; ++i)
      if (i < nb) nbrs3(P, d, q[(head + i) * 256], y[i]);
#pragma unroll
    for (int i = 0; i < BFS_BATCH; ++i) {
      if (i >= nb) break;
#pragma unroll
      for (int e = 0; e < 3; ++e) {
        int v = y[i][e];
        if (v < 0) continue;
        // 64-bit filter of the queued slots: only a possible hit scans the queue
        const uint64_t bit = 1ull << (((uint32_t)v * 0x9E3779B1u) >> 26);
        if (bloom & bit) {
          bool seen = false;
          for (int t = 0; t < qn; ++t) seen |= q[t * 256] == v;
          if (seen) continue;
        }
        bloom |= bit;
        if (qn == BFS_QCAP) {
          if (lower(qn) || (v >= NA && d.id_of[v] < pid)) return;
          uint32_t s = atomicAdd(&d.ctl->n_overflow, 1u);
          d.overflow[s] = b;
          return;
        }
        q[(qn++) * 256] = v;
      }
    }
    head += nb;
  }
  if (lower(qn)) return;
  register_complex<256>(P, d, p, q, qn);
}

// Component of overflow entry o (larger than BFS_QCAP): one thread, global
// queue + visit tags.  Returns the root's ligand index if it roots the
// component (registered, unlisted), else -1.  Called by k_complex_heavy.
__device__ __forceinline__ int bfs_overflow_one(const KParams& P, const Dev& d, uint32_t o) {
  const int NA = P.NA;
  int p = NA + d.overflow[o];
  const int pid = d.id_of[p];
  uint32_t tag = (uint32_t)(++d.ctl->vtag);
  int* q = d.bfs_queue;
  int qn = 0, head = 0;
  q[qn++] = p;
  d.vtag[p] = tag;
  while (head < qn) {
    int x = q[head++];
    int y[3];
    nbrs3(P, d, x, y);
#pragma unroll
    for (int e = 0; e < 3; ++e) {
      int v = y[e];
      if (v < 0) continue;
      if (v >= NA && d.id_of[v] < pid) return -1;
      if (d.vtag[v] == tag) continue;
      d.vtag[v] = tag;
      q[qn++] = v;
    }
  }
  register_complex(P, d, p, q, qn);
  return p - NA;
}

// ---------------------------------------------------------------- record keys
// streaming accesses of the proposal kernels: R is read once per step and
// R_new is re-read only at its reference points, so both bypass the caches
// (nontemporal); the MALL keeps the cell records and lists of the later
// kernels instead (measured: 0.539 -> 0.519 ms/step at C3)
typedef double kmc_dbl2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ double2 ld_r(const double2& r) {
  const kmc_dbl2v v = __builtin_nontemporal_load(reinterpret_cast<const kmc_dbl2v*>(&r));
  return make_double2(v.x, v.y);
}
__device__ __forceinline__ void st_n(double2& r, double2 v) {
  kmc_dbl2v w;
  w.x = v.x;
  w.y = v.y;
  __builtin_nontemporal_store(w, reinterpret_cast<kmc_dbl2v*>(&r));
}

__device__ __forceinline__ void ref_point(const Dev& d, const Beads& B, int p, int NA, double& x, double& y,
                                          double& zlo, double& zhi) {
  if (p < NA) {
    const double2 xy = B.Axy(p, 1, 1), z12 = B.A2(p, 16), z34 = B.A2(p, 20);  // z of domains 1,2 / 3,4
    x = xy.x;
    y = xy.y;
    double z1 = z12.x, z2 = z12.y, z3 = z34.x, z4 = z34.y;
    zlo = fmin(fmin(z1, z2), fmin(z3, z4));  // the axis span of the four domains
    zhi = fmax(fmax(z1, z2), fmax(z3, z4));
  } else {
    const double2 xy = B.Bxy(p - NA, 1, 1);
    x = xy.x;
    y = xy.y;
    zlo = B.B(p - NA, 1, 1, 2);
    zhi = zlo;
  }
}

// rigid-body extent bound the 3x3 stencil relies on (DESIGN.md §cell list)
__device__ __forceinline__ bool extent_ok(const Beads& B, int p, int NA) {
  if (p < NA) {
    double x0 = B.A(p, 1, 1, 0), y0 = B.A(p, 1, 1, 1);
    for (int j = 2; j <= 4; ++j) {
      double dx = B.A(p, j, 1, 0) - x0, dy = B.A(p, j, 1, 1) - y0;
      if (!(dx * dx + dy * dy <= 0.09)) return false;
    }
    return true;
  }
  int b = p - NA;
  double x0 = B.B(b, 1, 1, 0), y0 = B.B(b, 1, 1, 1);
  for (int j = 2; j <= 4; ++j) {
    double dx = B.B(b, j, 1, 0) - x0, dy = B.B(b, j, 1, 1) - y0;
    if (!(dx * dx + dy * dy <= 35.0 * 35.0)) return false;
  }
  return true;
}

// cell index of the (row, kind, column) cell order of the home list
__device__ __forceinline__ int cell_index(const KParams& P, int cx, int cy, int kind) {
  return (cy * 2 + kind) * P.ncx + cx;
}

// ---------------------------------------------------------------- records
// The neighbour searches (collisions main.cpp:640-664, 1762-1828; reactions
// 1877-2058) work on records: one per protein and position (old, proposed),
// written by the kernel that moves the protein, straight from the registers
// that hold its beads — no per-step counting sort.  Record w of slot p lives
// at rec[2·hp + w], hp = the protein's home position: the home list orders
// the proteins by the cell of their reference point at the last re-sort (the
// home cell; k_home_*).  A protein moves a few Å per step, so between
// re-sorts a record stays within one cell of its home cell: the record keeps
// that offset (4-bit cell code), and a tile of the pair scan finds every
// record of its cells (+ one-cell halo) among the home cells of the tile +
// two cells.  A record further away goes onto the outlier list and into the
// bucket of every tile whose block + one-cell halo holds its cell (up to
// four).  Outliers are few but not rare: every protein that crossed the
// periodic boundary since the last re-sort is one (thousands at C5 after 100
// steps), so a tile reads only its own bucket — the whole list only when its
// bucket overflowed.
#ifndef TOUT_CAP
#define TOUT_CAP 64
#endif
__device__ __forceinline__ void tile_bucket_push(const KParams& P, const Dev& d, int ri, int cx, int cy) {
  const int t = P.tile, ntx = (P.ncx + t - 1) / t;
  const int tx = cx / t, ty = cy / t, rx = cx - tx * t, ry = cy - ty * t;
  const int x0 = tx - (rx == 0 && tx > 0 ? 1 : 0), x1 = tx + (rx == t - 1 && (tx + 1) * t < P.ncx ? 1 : 0);
  const int y0 = ty - (ry == 0 && ty > 0 ? 1 : 0), y1 = ty + (ry == t - 1 && (ty + 1) * t < P.ncy ? 1 : 0);
  for (int y = y0; y <= y1; ++y)
    for (int x = x0; x <= x1; ++x) {
      const int b = y * ntx + x;
      const uint32_t o = atomicAdd(&d.tout_n[b], 1u);
      if (o < (uint32_t)P.tout_cap) d.tout[(size_t)b * TOUT_CAP + o] = make_int2(ri, cx | cy << 16);
    }
}

__device__ __forceinline__ void put_rec_raw(const KParams& P, const Dev& d, uint2 h, int p, int w, int st, int own,
                                            double x, double y, float4 pos, float2 site) {
  const int cx = cell_x(P, x), cy = cell_y(P, y);
  const int dx = cx - (int)(h.y & 0xffffu), dy = cy - (int)(h.y >> 16);
  const int ri = 2 * (int)h.x + w;
  int code = RID_OUT;
  if (dx >= -1 && dx <= 1 && dy >= -1 && dy <= 1) {
    code = (dy + 1) * 3 + (dx + 1);
  } else {
    const uint32_t o = atomicAdd(&d.ctl->n_outl, 1u);
    if (o < d.outl_cap) d.outl[o] = make_int4(ri, cx, cy, 0);
    else atomicOr(&d.ctl->err, ERR_EDGES);
    tile_bucket_push(P, d, ri, cx, cy);
  }
  Rec r;
  r.pos = pos;
  r.id = make_int2(p | (p >= P.NA ? RID_LIG : 0) | code << RID_CODE_SHIFT | st | (w << 31), own);
  r.site = site;
  d.rec[ri] = r;
  if (P.dbg_recs) d.rec_step[ri] = d.ctl->step;
}
// a receptor's record: reference point [1][1] xy, z span of its domains, [3][3] site
__device__ __forceinline__ void put_rec(const KParams& P, const Dev& d, uint2 h, int p, int w, int st, int own,
                                        double x, double y, double zlo, double zhi, double sx, double sy) {
  put_rec_raw(P, d, h, p, w, st, own, x, y, make_float4((float)x, (float)y, (float)zlo, (float)zhi),
              make_float2((float)sx, (float)sy));
}
// A ligand's record: centre [1][1] and the offsets of its three subunit
// centres [j][1] (j = 2..4) from it, rounded to whole Å (9 signed bytes in the
// words a receptor record uses for its z top and site).  k_col_exact tests a
// candidate pair's subunits from the records first (col_refine) and gathers
// the fp64 beads only when that cannot rule the collision out.  Byte 9 set:
// an offset out of the byte range (no such ligand within the extent bound),
// the pair goes to the exact test.
__device__ __forceinline__ uint32_t q8(double v, uint32_t& big) {
  const double r = rint(v);
  big |= (r > 120.0 || r < -120.0) ? 1u : 0u;
  return (uint32_t)((int)fmin(fmax(r, -120.0), 120.0) & 0xff);
}
__device__ __forceinline__ void put_rec_lig(const KParams& P, const Dev& d, uint2 h, int p, int w, int own, double cx,
                                            double cy, double cz, const double* sx, const double* sy,
                                            const double* sz) {
  uint32_t big = 0, b[9];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    b[3 * j] = q8(sx[j] - cx, big);
    b[3 * j + 1] = q8(sy[j] - cy, big);
    b[3 * j + 2] = q8(sz[j] - cz, big);
  }
  const uint32_t w0 = b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24, w1 = b[4] | b[5] << 8 | b[6] << 16 | b[7] << 24,
                 w2 = b[8] | big << 8;
  put_rec_raw(P, d, h, p, w, 0, own, cx, cy, make_float4((float)cx, (float)cy, (float)cz, __uint_as_float(w0)),
              make_float2(__uint_as_float(w1), __uint_as_float(w2)));
}

// debug (KMC_DEBUG_RECS=1), after the proposal phase: every protein's two
// records must have been written this step by the kernel that moved it (the
// pair scan reads them in place; a record left from an earlier step would
// pair stale positions silently)
__global__ void k_rec_check(KParams P, Dev d) {
  const uint32_t step = d.ctl->step;
  bool bad = false;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < 2 * P.N; i += gridDim.x * blockDim.x)
    bad |= d.rec_step[i] != step;
  if (__ballot(bad) && __lane_id() == 0) atomicOr(&d.ctl->err, ERR_RESOLVE);
}

// status bits of slot p's records
__device__ __forceinline__ int rec_status(const KParams& P, const Dev& d, int p) {
  const int NA = P.NA;
  return p < NA ? (A_ST2(d, p) ? RID_ST2 : 0) | (A_ST3(d, p) ? RID_ST3 : 0) : 0;
}

// record w of slot p from its beads in global memory (old: R, proposal: R_new)
__device__ __forceinline__ void put_rec_glb(const KParams& P, const Dev& d, uint2 h, int p, int w, int st, int own) {
  const Beads& B = w ? d.nxt : d.cur;
  double x, y, zl, zh, sx = 0.0, sy = 0.0;
  ref_point(d, B, p, P.NA, x, y, zl, zh);
  if (p < P.NA) {
    const double2 s33 = B.Axy(p, 3, 3);
    sx = s33.x;
    sy = s33.y;
  } else {
    double ux[3], uy[3], uz[3];
    for (int j = 0; j < 3; ++j) {
      const double2 xy = B.Bxy(p - P.NA, j + 2, 1);
      ux[j] = xy.x;
      uy[j] = xy.y;
      uz[j] = B.B(p - P.NA, j + 2, 1, 2);
    }
    put_rec_lig(P, d, h, p, w, own, x, y, zl, ux, uy, uz);
    return;
  }
  put_rec(P, d, h, p, w, st, own, x, y, zl, zh, sx, sy);
}

// both records of slot p from global memory, and the extent bound of its
// proposal (DESIGN.md §cell list)
__device__ __forceinline__ void put_recs_glb(const KParams& P, const Dev& d, int p) {
  const uint2 h = d.home[p];
  const int st = rec_status(P, d, p), own = d.owner[p];
  put_rec_glb(P, d, h, p, 0, st, own);
  put_rec_glb(P, d, h, p, 1, st, own);
  if (!extent_ok(d.nxt, p, P.NA)) atomicOr(&d.ctl->err, ERR_GEOMETRY);
}

// ================================================================ 2. proposals

// free receptor, main.cpp:584-635.  All 48 coordinates are loaded (24 16-byte
// rows) before the first store (R and R_new are distinct buffers), so a lane
// has every load in flight at once.
__device__ void propose_free_a(const KParams& P, const Dev& d, int i, uint32_t step) {
  double r[4][4][3];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const double2 v = ld_r(d.cur.A2(i, j * 4 + k));
      r[j][k][0] = v.x;
      r[j][k][1] = v.y;
    }
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const double2 v = ld_r(d.cur.A2(i, 16 + h * 4 + k));
      r[2 * h][k][2] = v.x;
      r[2 * h + 1][k][2] = v.y;
    }
  const uint2 h = d.home[i];
  double u0, u1, u2, u3;
  const uint32_t ri = (uint32_t)d.id_of[i], rk = rkey(P, d, (int)ri);
  kmcr::uniform2(P.key, kmcr::DOM_DIFF, rk, 0, step, 0, &u0, &u1);
  kmcr::uniform2(P.key, kmcr::DOM_DIFF, rk, 0, step, 1, &u2, &u3);
  double amp = P.amp_a * u0;
  double phai = u1 * 2 * P.pai;
  double dx = amp * kmcm::cos(phai), dy = amp * kmcm::sin(phai);
  double o11x = r[0][0][0] + dx, o11y = r[0][0][1] + dy;
  double PBx = P.box_x * kmcm::round_(o11x / P.box_x);
  double PBy = P.box_y * kmcm::round_(o11y / P.box_y);
  Rot t = euler(0, 0, (2 * u2 - 1) * P.rot_a);
  double ncx[4], ncy[4], nz[4][4], nsx = 0.0, nsy = 0.0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    double cx = (r[j][0][0] + dx) - PBx;
    double cy = (r[j][0][1] + dy) - PBy;
    double cz = r[j][0][2];
    ncx[j] = cx;
    ncy[j] = cy;
    nz[j][0] = cz;
    st_n(d.nxt.A2(i, j * 4), make_double2(cx, cy));
#pragma unroll
    for (int k = 1; k < 4; ++k) {
      double ox = (r[j][k][0] + dx) - PBx;
      double oy = (r[j][k][1] + dy) - PBy;
      double oz = r[j][k][2];
      const double nx = rx(t, ox, oy, oz, cx, cy, cz), ny = ry(t, ox, oy, oz, cx, cy, cz);
      st_n(d.nxt.A2(i, j * 4 + k), make_double2(nx, ny));
      if (j == 2 && k == 2) {  // the [3][3] cis site (reaction prefilter)
        nsx = nx;
        nsy = ny;
      }
      nz[j][k] = rz(t, ox, oy, oz, cx, cy, cz);
    }
  }
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int k = 0; k < 4; ++k) st_n(d.nxt.A2(i, 16 + h * 4 + k), make_double2(nz[2 * h][k], nz[2 * h + 1][k]));
  bool ext = true;
#pragma unroll
  for (int j = 1; j < 4; ++j) {
    double ex = ncx[j] - ncx[0], ey = ncy[j] - ncy[0];
    ext &= ex * ex + ey * ey <= 0.09;
  }
  if (!ext) atomicOr(&d.ctl->err, ERR_GEOMETRY);
  // records: z span of the four domain centres (ref_point), [3][3] site
  const int own = (int)ri;  // a free receptor is its own unit, status bits 0
  put_rec(P, d, h, i, 0, 0, own, r[0][0][0], r[0][0][1], fmin(fmin(r[0][0][2], r[1][0][2]), fmin(r[2][0][2], r[3][0][2])),
          fmax(fmax(r[0][0][2], r[1][0][2]), fmax(r[2][0][2], r[3][0][2])), r[2][2][0], r[2][2][1]);
  put_rec(P, d, h, i, 1, 0, own, ncx[0], ncy[0], fmin(fmin(nz[0][0], nz[1][0]), fmin(nz[2][0], nz[3][0])),
          fmax(fmax(nz[0][0], nz[1][0]), fmax(nz[2][0], nz[3][0])), nsx, nsy);
}

// snap receptor a2 onto a1's cis site (x,y of all 16 beads), main.cpp:786-798
template <class S>
__device__ __forceinline__ void snap_cis(const KParams& P, const S& N, int a2, int a1, double cis_cut) {
  const double RA = P.ra;
  double x33 = N.A(a1, 3, 3, 0), x31 = N.A(a1, 3, 1, 0);
  double y33 = N.A(a1, 3, 3, 1), y31 = N.A(a1, 3, 1, 1);
  double x1 = (cis_cut / 2 + RA) / RA * (x33 - x31) + x33;
  double y1 = (cis_cut / 2 + RA) / RA * (y33 - y31) + y33;
  double x3 = (cis_cut / 2) / RA * (x33 - x31) + x33;
  double y3 = (cis_cut / 2) / RA * (y33 - y31) + y33;
  double x2 = (cis_cut / 2 + 2 * RA) / RA * (x33 - x31) + x33;
  double y2 = (cis_cut / 2 + 2 * RA) / RA * (y33 - y31) + y33;
  for (int k = 1; k <= 4; ++k) {
    N.A(a2, k, 1, 0) = x1;
    N.A(a2, k, 1, 1) = y1;
    N.A(a2, k, 4, 0) = x1;
    N.A(a2, k, 4, 1) = y1;
    N.A(a2, k, 3, 0) = x3;
    N.A(a2, k, 3, 1) = y3;
    N.A(a2, k, 2, 0) = x2;
    N.A(a2, k, 2, 1) = y2;
  }
}

// snap receptor a onto ligand site (lb = ligand 0-based in B arrays, j),
// main.cpp:1216-1228
template <class S>
__device__ __forceinline__ void snap_bond(const KParams& P, const S& N, int a, int lb, int j, double bond_cut) {
  const double RA = P.ra, RB = P.rb;
  double x2 = N.B(lb, j, 2, 0), x1 = N.B(lb, j, 1, 0);
  double y2 = N.B(lb, j, 2, 1), y1 = N.B(lb, j, 1, 1);
  double ax1 = (bond_cut / 2 + RA) / RB * (x2 - x1) + x2;
  double ay1 = (bond_cut / 2 + RA) / RB * (y2 - y1) + y2;
  double ax3 = (bond_cut / 2 + 2 * RA) / RB * (x2 - x1) + x2;
  double ay3 = (bond_cut / 2 + 2 * RA) / RB * (y2 - y1) + y2;
  double ax2 = (bond_cut / 2) / RB * (x2 - x1) + x2;
  double ay2 = (bond_cut / 2) / RB * (y2 - y1) + y2;
  for (int k = 1; k <= 4; ++k) {
    N.A(a, k, 1, 0) = ax1;
    N.A(a, k, 1, 1) = ay1;
    N.A(a, k, 4, 0) = ax1;
    N.A(a, k, 4, 1) = ay1;
    N.A(a, k, 3, 0) = ax3;
    N.A(a, k, 3, 1) = ay3;
    N.A(a, k, 2, 0) = ax2;
    N.A(a, k, 2, 1) = ay2;
  }
}

template <class S>
__device__ __forceinline__ double dxyA(const S& N, int p, int j, int k, int q, int jj, int kk) {
  double dx = N.A(p, j, k, 0) - N.A(q, jj, kk, 0), dy = N.A(p, j, k, 1) - N.A(q, jj, kk, 1);
  return kmcm::sqrt_(dx * dx + dy * dy);
}
// ligand lb bead (j,k) vs receptor a bead (jj,kk)
template <class S>
__device__ __forceinline__ double dxyBA(const S& N, int lb, int j, int k, int a, int jj, int kk) {
  double dx = N.B(lb, j, k, 0) - N.A(a, jj, kk, 0), dy = N.B(lb, j, k, 1) - N.A(a, jj, kk, 1);
  return kmcm::sqrt_(dx * dx + dy * dy);
}
template <class S>
__device__ __forceinline__ bool cis_misaligned(const KParams& P, const S& N, int a1, int a2) {
  double dd2 = dxyA(N, a1, 3, 3, a2, 3, 3);
  double dd1 = dxyA(N, a1, 3, 1, a2, 3, 1);
  return !AreSame(dd1, P.cis_cut / 2 + P.ra + P.ra) || !AreSame(dd2, P.cis_cut / 2);
}
__device__ __forceinline__ bool bond_mis_d(const KParams& P, double dd1, double dd2) {
  return !AreSame(dd1, P.bond_cut / 2 + P.ra + P.rb) || !AreSame(dd2, P.bond_cut / 2);
}
template <class S>
__device__ __forceinline__ bool bond_misaligned(const KParams& P, const S& N, int lb, int j, int a1) {
  double dd2 = dxyBA(N, lb, j, 2, a1, 3, 2);
  double dd1 = dxyBA(N, lb, j, 1, a1, 3, 1);
  return bond_mis_d(P, dd1, dd2);
}

// cis dimer lead i with partner q, main.cpp:682-865 (proposal part), and
// both receptors' records.  The [j][1] rows of both receptors (shift, centre)
// are loaded together, then each receptor's rows two domains at a time (12
// rows in flight) before their stores: per-bead accessors cost a load round
// trip per bead (R and R_new may alias for the compiler), and a dimer lead
// held its wave ~30 round trips.  Records and the extent bound come from
// registers, as for the free units.
__device__ __forceinline__ void propose_dimer(const KParams& P, const Dev& d, int i, int q, uint32_t step) {
  double u0, u1, u2, u3;
  const uint32_t rk = rkey(P, d, d.id_of[i]);
  kmcr::uniform2(P.key, kmcr::DOM_DIFF, rk, 0, step, 0, &u0, &u1);
  kmcr::uniform2(P.key, kmcr::DOM_DIFF, rk, 0, step, 1, &u2, &u3);
  double amp = P.amp_cis * u0;
  double phai = u1 * 2 * P.pai;
  double dx = amp * kmcm::cos(phai), dy = amp * kmcm::sin(phai);
  double cmx = 0, cmy = 0, cmz = 0, PBx, PBy;
  {
    // [j][1] (x, y), z of [1,2][1] and [3,4][1], [3][3] (x, y): the shift,
    // the centre and both old records
    double2 ci[4], cq[4], zi[2], zq[2], si, sq;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      ci[j] = d.cur.A2(i, j * 4);
      cq[j] = d.cur.A2(q, j * 4);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      zi[h] = d.cur.A2(i, 16 + h * 4);
      zq[h] = d.cur.A2(q, 16 + h * 4);
    }
    si = d.cur.A2(i, 10);
    sq = d.cur.A2(q, 10);
    put_rec(P, d, d.home[i], i, 0, rec_status(P, d, i), d.owner[i], ci[0].x, ci[0].y,
            fmin(fmin(zi[0].x, zi[0].y), fmin(zi[1].x, zi[1].y)), fmax(fmax(zi[0].x, zi[0].y), fmax(zi[1].x, zi[1].y)),
            si.x, si.y);
    put_rec(P, d, d.home[q], q, 0, rec_status(P, d, q), d.owner[q], cq[0].x, cq[0].y,
            fmin(fmin(zq[0].x, zq[0].y), fmin(zq[1].x, zq[1].y)), fmax(fmax(zq[0].x, zq[0].y), fmax(zq[1].x, zq[1].y)),
            sq.x, sq.y);
    PBx = P.box_x * kmcm::round_(((ci[0].x + dx) + (cq[0].x + dx)) / 2 / P.box_x);
    PBy = P.box_y * kmcm::round_(((ci[0].y + dy) + (cq[0].y + dy)) / 2 / P.box_y);
    // rotation centre: R_new before the move (= R), main.cpp:740-753
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      cmx = cmx + ci[j].x + cq[j].x;
      cmy = cmy + ci[j].y + cq[j].y;
      cmz = cmz + (j & 1 ? zi[j >> 1].y : zi[j >> 1].x) + (j & 1 ? zq[j >> 1].y : zq[j >> 1].x);
    }
  }
  cmx = cmx / (4 * 2);
  cmy = cmy / (4 * 2);
  cmz = cmz / (4 * 2);
  Rot t = euler(0, 0, (2 * u2 - 1) * P.rot_cis);
  double2 n31i, n33i;  // the lead's new [3][1] and [3][3] (x, y)
#pragma unroll 1
  for (int w = 0; w < 2; ++w) {
    const int a = w ? q : i;
    double2 n11, ns, n31;
    double zlo, zhi;  // of the new [j][1] z
    bool ext = true;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      double2 v[12];  // (x, y) rows of domains 2h+1, 2h+2, then their z-pair rows
#pragma unroll
      for (int r = 0; r < 8; ++r) v[r] = ld_r(d.cur.A2(a, h * 8 + r));
#pragma unroll
      for (int k = 0; k < 4; ++k) v[8 + k] = ld_r(d.cur.A2(a, 16 + h * 4 + k));
      double nz[2][4];
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const double ox = (v[jj * 4 + k].x + dx) - PBx;
          const double oy = (v[jj * 4 + k].y + dy) - PBy;
          const double oz_ = jj ? v[8 + k].y : v[8 + k].x;
          const double2 nxy = make_double2(rx(t, ox, oy, oz_, cmx, cmy, cmz), ry(t, ox, oy, oz_, cmx, cmy, cmz));
          nz[jj][k] = rz(t, ox, oy, oz_, cmx, cmy, cmz);
          st_n(d.nxt.A2(a, h * 8 + jj * 4 + k), nxy);
          if (k == 0) {  // [j][1]: reference point and extent bound (extent_ok)
            if (h == 0 && jj == 0) {
              n11 = nxy;
            } else {
              const double ex = nxy.x - n11.x, ey = nxy.y - n11.y;
              ext &= ex * ex + ey * ey <= 0.09;
            }
          }
          if (h == 1 && jj == 0 && k == 0) n31 = nxy;
          if (h == 1 && jj == 0 && k == 2) ns = nxy;
        }
      if (h == 0) {
        zlo = fmin(nz[0][0], nz[1][0]);
        zhi = fmax(nz[0][0], nz[1][0]);
      } else {
        zlo = fmin(zlo, fmin(nz[0][0], nz[1][0]));
        zhi = fmax(zhi, fmax(nz[0][0], nz[1][0]));
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) st_n(d.nxt.A2(a, 16 + h * 4 + k), make_double2(nz[0][k], nz[1][k]));
    }
    if (w == 0) {
      n31i = n31;
      n33i = ns;
    } else {
      // relax, main.cpp:770-799: dxyA on the new positions
      double ex = n33i.x - ns.x, ey = n33i.y - ns.y;
      const double dist2 = kmcm::sqrt_(ex * ex + ey * ey);
      ex = n31i.x - n31.x;
      ey = n31i.y - n31.y;
      const double dist1 = kmcm::sqrt_(ex * ex + ey * ey);
      const double dist3 = P.cis_cut / 2 + P.ra + P.ra;
      const double dist4 = P.cis_cut / 2;
      if (!AreSame(dist1, dist3) || !AreSame(dist2, dist4)) {
        // snap the partner onto the lead's cis site (main.cpp:786-798; snap_cis
        // on registers): every domain's beads 1 and 4 at (x1, y1), 3 at (x3,
        // y3), 2 at (x2, y2) — its [j][1] beads coincide (extent bound holds)
        const double RA = P.ra, cc = P.cis_cut;
        const double x1 = (cc / 2 + RA) / RA * (n33i.x - n31i.x) + n33i.x;
        const double y1 = (cc / 2 + RA) / RA * (n33i.y - n31i.y) + n33i.y;
        const double x3 = (cc / 2) / RA * (n33i.x - n31i.x) + n33i.x;
        const double y3 = (cc / 2) / RA * (n33i.y - n31i.y) + n33i.y;
        const double x2 = (cc / 2 + 2 * RA) / RA * (n33i.x - n31i.x) + n33i.x;
        const double y2 = (cc / 2 + 2 * RA) / RA * (n33i.y - n31i.y) + n33i.y;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          st_n(d.nxt.A2(q, j * 4), make_double2(x1, y1));
          st_n(d.nxt.A2(q, j * 4 + 1), make_double2(x2, y2));
          st_n(d.nxt.A2(q, j * 4 + 2), make_double2(x3, y3));
          st_n(d.nxt.A2(q, j * 4 + 3), make_double2(x1, y1));
        }
        n11 = make_double2(x1, y1);
        ns = make_double2(x3, y3);
        ext = true;
      }
    }
    put_rec(P, d, d.home[a], a, 1, rec_status(P, d, a), d.owner[a], n11.x, n11.y, zlo, zhi, ns.x, ns.y);
    if (!ext) atomicOr(&d.ctl->err, ERR_GEOMETRY);
  }
}

// single ligand, main.cpp:905-969 (all 24 coordinates, 12 16-byte rows,
// loaded first)
__device__ void propose_free_b(const KParams& P, const Dev& d, int lb, int p, uint32_t step) {
  double r[4][2][3];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const double2 v = ld_r(d.cur.B2(lb, j * 2 + k));
      r[j][k][0] = v.x;
      r[j][k][1] = v.y;
    }
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const double2 v = ld_r(d.cur.B2(lb, 8 + h * 2 + k));
      r[2 * h][k][2] = v.x;
      r[2 * h + 1][k][2] = v.y;
    }
  const uint2 h = d.home[p];
  double u[6];
  const uint32_t rp = (uint32_t)d.id_of[p], rk = rkey(P, d, (int)rp);  // unit key, random-stream key
  kmcr::uniform2(P.key, kmcr::DOM_DIFF, rk, 0, step, 0, &u[0], &u[1]);
  kmcr::uniform2(P.key, kmcr::DOM_DIFF, rk, 0, step, 1, &u[2], &u[3]);
  kmcr::uniform2(P.key, kmcr::DOM_DIFF, rk, 0, step, 2, &u[4], &u[5]);
  double amp = P.amp_b * u[0];
  double theta = u[1] * P.pai;
  double phai = u[2] * 2 * P.pai;
  double sth = kmcm::sin(theta), cth = kmcm::cos(theta);
  double dx = amp * sth * kmcm::cos(phai);
  double dy = amp * sth * kmcm::sin(phai);
  double dz = amp * cth;
  double o11x = r[0][0][0] + dx, o11y = r[0][0][1] + dy, o11z = r[0][0][2] + dz;
  double PBx = P.box_x * kmcm::round_(o11x / P.box_x);
  double PBy = P.box_y * kmcm::round_(o11y / P.box_y);
  double PBz = P.box_z * kmcm::round_(o11z / P.box_z);
  bool refl = o11z > P.box_z || o11z < 0;
  Rot t = euler((2 * u[3] - 1) * P.rot_b, (2 * u[4] - 1) * P.rot_b, (2 * u[5] - 1) * P.rot_b);
  double ox[4][2], oy[4][2], oz[4][2];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      double z = r[j][k][2] + dz;
      if (refl) z = -z + 2 * PBz;
      oz[j][k] = z;
      ox[j][k] = (r[j][k][0] + dx) - PBx;
      oy[j][k] = (r[j][k][1] + dy) - PBy;
    }
  // R_new[1][1] = R_new0[1][1], then every bead (incl. [1][1] itself, which
  // updates the centre in place) rotates about R_new[1][1], main.cpp:958-968
  double cx = ox[0][0], cy = oy[0][0], cz = oz[0][0];
  double scx[4], scy[4];  // new subunit centres [j][1] (extent bound)
  double nzs[4][2];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      double nx = rx(t, ox[j][k], oy[j][k], oz[j][k], cx, cy, cz);
      if (j == 0 && k == 0) cx = nx;
      double ny = ry(t, ox[j][k], oy[j][k], oz[j][k], cx, cy, cz);
      if (j == 0 && k == 0) cy = ny;
      double nz = rz(t, ox[j][k], oy[j][k], oz[j][k], cx, cy, cz);
      if (j == 0 && k == 0) cz = nz;
      if (k == 0) {
        scx[j] = nx;
        scy[j] = ny;
      }
      st_n(d.nxt.B2(lb, j * 2 + k), make_double2(nx, ny));
      nzs[j][k] = nz;
    }
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int k = 0; k < 2; ++k) st_n(d.nxt.B2(lb, 8 + h * 2 + k), make_double2(nzs[2 * h][k], nzs[2 * h + 1][k]));
  bool ext = true;
#pragma unroll
  for (int j = 1; j < 4; ++j) {
    double ex = scx[j] - scx[0], ey = scy[j] - scy[0];
    ext &= ex * ex + ey * ey <= 35.0 * 35.0;
  }
  if (!ext) atomicOr(&d.ctl->err, ERR_GEOMETRY);
  // records: the centre [1][1] (a free ligand is its own unit)
  {
    const double ox3[3] = {r[1][0][0], r[2][0][0], r[3][0][0]}, oy3[3] = {r[1][0][1], r[2][0][1], r[3][0][1]},
                 oz3[3] = {r[1][0][2], r[2][0][2], r[3][0][2]};
    put_rec_lig(P, d, h, p, 0, (int)rp, r[0][0][0], r[0][0][1], r[0][0][2], ox3, oy3, oz3);
    const double nz3[3] = {nzs[1][0], nzs[2][0], nzs[3][0]};
    put_rec_lig(P, d, h, p, 1, (int)rp, scx[0], scy[0], nzs[0][0], scx + 1, scy + 1, nz3);
  }
}

// ---------------------------------------------------------------- stamps
// Diagnostic build only (-DKMC_STAMPS): thread 0 of each workgroup adds the
// cycles since its previous stamp to ctl->stamps[base + i] (phase shares of
// the tile scans; kmc_step prints them with KMC_DEBUG_COUNTS=1).  In the
// real build a stamp compiles to nothing.
struct Stamper {
#ifdef KMC_STAMPS
  uint64_t t;
  int base;
  __device__ static uint64_t now() {
    uint64_t v;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");
    return v;
  }
  __device__ explicit Stamper(int b) : t(now()), base(b) {}
  __device__ void operator()(const Dev& d, int i) {
    if (threadIdx.x == 0) {
      const uint64_t v = now();
      atomicAdd((unsigned long long*)&d.ctl->stamps[base + i], (unsigned long long)(v - t));
      t = v;
    }
  }
#else
  __device__ explicit Stamper(int) {}
  __device__ void operator()(const Dev&, int) {}
#endif
};

// ---------------------------------------------------------------- complexes
// Ligand-rooted complex of size > 1: rigid move (main.cpp:974-1131), lay-down
// of a single ligand (1138-1193), receptor / cis re-alignment (1196-1274),
// multi-ligand alignment (1284-1732).  The common case is streamed (below:
// cx_params, k_move_members, k_cx_check); the rest runs one wave per complex
// (k_complex_heavy).
//
// A complex of up to CXL members is staged in LDS: the wave loads the member
// slots and links, moves the beads (lanes over (member, bead)) into LDS, lane
// 0 runs the sequential, data-dependent lay-down / alignment code against LDS
// (a dependent chain of LDS accesses instead of HBM round trips — the step's
// critical path at the bond-rich steady state), then the lanes write R_new
// back and count the members' records.  Members are addressed by their
// position t in the BFS row, encoded like protein numbers so that the
// reference's kind tests carry over unchanged: receptor t -> t, ligand t ->
// NA + t.  Larger complexes (rare) run the same code on global memory.
#define CX_SHUF 6  // random_shuffle passes whose draws are precomputed (4 + 2 repeats of lable4)
// Member stride of the LDS image in doubles.  48 (384 B) put the same
// coordinate of every member on one bank — 96 dwords ≡ 0 mod 32 — so the
// steps that take one member per lane (the alignment's member loops, the
// records, the extent bound) were 16-way conflicted (SQ_LDS_BANK_CONFLICT 41 %
// of the kernel's LDS cycles at C3, profiles/r05/final_C3); 49 (392 B, 98
// dwords) spreads a 16-lane group over 16 bank pairs.
#ifndef CX_STRIDE
#define CX_STRIDE 49
#endif
struct CxLds {
  double bead[CXL][CX_STRIDE];  // R_new of member t: receptor bead (j,k) at ((j-1)*4+(k-1))*3+c, ligand ((j-1)*2+(k-1))*3+c
  int lk[CXL][4];        // links (encoded): receptor {nei4 (site), nei2, nei3, -}, ligand {-, nei2, nei3, nei4}
  int slot[CXL];         // slot of member t
  int res[CXL];          // member row (encoded), shuffled in place like results[c][.]
  uint8_t mv[CXL];       // moved flags of this step (main.cpp:122)
  uint8_t pos[CXL];      // position of member t in the shuffled row res (wave-parallel alignment)
  uint32_t rnd[CX_SHUF][CXL];  // the first CX_SHUF shuffles' keyed draws, computed by all lanes at once
};
struct LdsBeads {
  CxLds* L;
  __device__ double& A(int t, int j, int k, int c) const { return L->bead[t][((j - 1) * 4 + (k - 1)) * 3 + c]; }
  __device__ double& B(int t, int j, int k, int c) const { return L->bead[t][((j - 1) * 2 + (k - 1)) * 3 + c]; }
};
// links and moved flags of a staged complex
struct LdsLinks {
  CxLds* L;
  int NA;
  __device__ int a2(int a) const { return L->lk[a][1]; }
  __device__ int a3(int a) const { return L->lk[a][2]; }
  __device__ int a4(int a) const { return L->lk[a][0]; }
  __device__ int b(int lb, int j) const { return L->lk[lb][j - 1]; }
  __device__ bool moved(int m) const { return L->mv[m < NA ? m : m - NA] != 0; }
  __device__ void set_moved(int m) const { L->mv[m < NA ? m : m - NA] = 1; }
};
// the global state rows (slots)
struct GlbLinks {
  const Dev* d;
  int NA, NB;
  uint32_t step;
  __device__ int a2(int a) const { return d->a_int[2 * (size_t)NA + a]; }
  __device__ int a3(int a) const { return d->a_int[4 * (size_t)NA + a]; }
  __device__ int a4(int a) const { return d->a_int[3 * (size_t)NA + a]; }
  __device__ int b(int lb, int j) const { return d->b_int[(size_t)(4 + j - 1) * NB + lb]; }
  __device__ bool moved(int m) const { return d->moved[m] == step + 1; }
  __device__ void set_moved(int m) const { d->moved[m] = step + 1; }
};

template <class S, class L>
struct CxT {
  const KParams& P;
  uint32_t step;
  uint32_t rootid;  // the root ligand's reference index (random stream key)
  int* res;         // member row (BFS order, shuffled in place like results[c][.])
  int size;
  S N;              // R_new
  L lk;
  uint32_t* err;
  const uint32_t (*pre)[CXL] = nullptr;  // precomputed draws of the first CX_SHUF shuffles (LDS), or none
  __device__ int neiA2(int a) const { return lk.a2(a); }
  __device__ int neiA3(int a) const { return lk.a3(a); }
  __device__ int neiA4(int a) const { return lk.a4(a); }
  __device__ int neiB(int lb, int j) const { return lk.b(lb, j); }
  // res_nei_new[x][j] with reference semantics for the alignment code, where
  // x may be a receptor or a ligand (reference index, 0 = the empty row 0)
  __device__ int rnei(int x_ref, int j) const {
    if (x_ref <= 0) return 0;
    int x = x_ref - 1;
    if (x < P.NA) return j == 2 ? neiA2(x) : j == 3 ? neiA3(x) : j == 4 ? neiA4(x) : 0;
    return j >= 1 && j <= 4 ? neiB(x - P.NA, j) : 0;
  }
  __device__ bool is_moved(int m) const { return lk.moved(m); }
  __device__ void set_moved(int m) const { lk.set_moved(m); }
  __device__ uint32_t shuf_rand(uint32_t call, uint32_t pos) const {
    if (pre && call < CX_SHUF) return pre[call][pos];
    return kmcr::rand31(P.key, kmcr::DOM_SHUF, rootid, call, step, pos);
  }
  // libstdc++ random_shuffle over res[0 .. size-2] (main.cpp:1285)
  __device__ void shuffle(uint32_t call) const {
    for (int i = 1; i < size - 1; ++i) {
      int j = (int)(shuf_rand(call, (uint32_t)i) % (uint32_t)(i + 1));
      if (i != j) {
        int tmp = res[i];
        res[i] = res[j];
        res[j] = tmp;
      }
    }
  }
};

__device__ __forceinline__ void ligand_template(double rb, double tx[5][3], double ty[5][3]) {
  for (int j = 0; j < 5; ++j)
    for (int k = 0; k < 3; ++k) tx[j][k] = ty[j][k] = 0;
  const double s3 = kmcm::sqrt_(3.0);
  tx[2][1] = 0; ty[2][1] = rb * 2 / s3;
  tx[2][2] = 0; ty[2][2] = rb * (2 / s3 + 1);
  tx[3][1] = -rb; ty[3][1] = -rb / s3;
  tx[3][2] = -rb * (s3 / 2 + 1); ty[3][2] = -rb / s3 - rb / 2;
  tx[4][1] = rb; ty[4][1] = -rb / s3;
  tx[4][2] = rb * (s3 / 2 + 1); ty[4][2] = -rb / s3 - rb / 2;
}

// lable4's re-laying of ligand B flat at receptor a1's height, its site j
// facing a1 (main.cpp:1441-1520): every new bead is a function of a1's beads
// and the template only.  bead < 0: all eight beads (one lane); else only
// bead (m, n) = (bead / 2 + 1, bead % 2 + 1) (lanes of a wave, one bead each)
template <class CX>
__device__ __forceinline__ void step2_relayout(const CX& X, int B, int j, int a1, int bead) {
  const KParams& P = X.P;
  const auto& N = X.N;
  const int NA = P.NA;
  int lb = B - NA;
  double za = N.A(a1, 3, 1, 2);
  double tx[5][3], ty[5][3];
  ligand_template(P.rb, tx, ty);
  // tx[j][1], ty[j][1] (j = 2..4) without a dynamically indexed array
  double ax1 = j == 2 ? tx[2][1] : j == 3 ? tx[3][1] : tx[4][1];
  double ay1 = j == 2 ? ty[2][1] : j == 3 ? ty[3][1] : ty[4][1];
  double ax2 = N.A(a1, 3, 1, 0) - N.A(a1, 3, 2, 0);
  double ay2 = N.A(a1, 3, 1, 1) - N.A(a1, 3, 2, 1);
  double dot = ax1 * ax2 + ay1 * ay2;
  double det = ax1 * ay2 - ay1 * ax2;
  double angle = kmcm::atan2(-det, -dot) + P.pai;
  const double s3 = kmcm::sqrt_(3.0);
  double cmx = (P.bond_cut / 2 + P.rb * 2 / s3 + P.rb) / P.ra * (N.A(a1, 3, 2, 0) - N.A(a1, 3, 1, 0)) + N.A(a1, 3, 2, 0);
  double cmy = (P.bond_cut / 2 + P.rb * 2 / s3 + P.rb) / P.ra * (N.A(a1, 3, 2, 1) - N.A(a1, 3, 1, 1)) + N.A(a1, 3, 2, 1);
  double ca = kmcm::cos(angle), sa = kmcm::sin(angle);
  for (int m = 1; m <= 4; ++m)
    for (int n = 1; n <= 2; ++n) {
      if (bead >= 0 && bead != (m - 1) * 2 + (n - 1)) continue;
      // z: every bead at za, the normal point [1][2] at za + rb (main.cpp:1441-1452)
      N.B(lb, m, n, 2) = (m == 1 && n == 2) ? N.A(a1, 3, 1, 2) + P.rb : za;
      N.B(lb, m, n, 0) = tx[m][n] * ca - ty[m][n] * sa + cmx;
      N.B(lb, m, n, 1) = tx[m][n] * sa + ty[m][n] * ca + cmy;
    }
}

// the rest of lable4 (main.cpp:1521-1583): B's receptors snapped onto its
// sites, their cis partners onto them; returns protein_B_index (0-based)
template <class CX>
__device__ __forceinline__ int step2_sites(const CX& X, int B) {
  const KParams& P = X.P;
  const auto& N = X.N;
  const int NA = P.NA;
  int Bref = B + 1;  // protein_B_index in reference numbering
  for (int m = 2; m <= 4; ++m) {
    int A1ref = X.rnei(Bref, m);
    if (X.rnei(A1ref, 2) != 0) {
      Bref = X.rnei(A1ref, 2);
      int n = X.rnei(A1ref, 4);
      int A1 = A1ref - 1, lb2 = Bref - 1 - NA;
      if (bond_misaligned(P, N, lb2, n, A1)) {
        X.set_moved(A1);
        snap_bond(P, N, A1, lb2, n, P.bond_cut);
      }
      if (X.rnei(A1ref, 3) != 0) {
        int A2 = X.rnei(A1ref, 3) - 1;
        if (cis_misaligned(P, N, A1, A2)) {
          X.set_moved(A2);
          snap_cis(P, N, A2, A1, P.cis_cut);
        }
      }
    }
  }
  return Bref - 1;
}

// body of lable4, main.cpp:1441-1583 (one lane); returns protein_B_index (0-based)
template <class CX>
__device__ __forceinline__ int step2_body(const CX& X, int B, int j, int a1) {
  X.set_moved(B);
  step2_relayout(X, B, j, a1, -1);
  return step2_sites(X, B);
}

template <class CX>
__device__ __forceinline__ void multi_ligand_align(const CX& X) {
  const KParams& P = X.P;
  const auto& N = X.N;
  const int NA = P.NA;
  const int csize = X.size;
  int* res = X.res;
  uint32_t call = 0;
  // step 0, main.cpp:1284-1332
  X.shuffle(call++);
  for (int csi = 0; csi < csize; ++csi) {
    int m = res[csi];
    if (m < NA && X.neiA2(m) != 0) {
      int lb = X.neiA2(m) - 1 - NA, j = X.neiA4(m);
      if (bond_misaligned(P, N, lb, j, m)) {
        X.set_moved(m);
        snap_bond(P, N, m, lb, j, P.bond_cut);
      }
    }
  }
  // step 1, main.cpp:1341-1406
  X.shuffle(call++);
  for (int csi = 0; csi < csize; ++csi) {
    int pa = res[csi];
    if (pa < NA) {
      if (X.neiA2(pa) != 0 && X.neiA3(pa) != 0 && X.rnei(X.neiA3(pa), 2) != 0 && !X.is_moved(pa)) {
        int a1 = pa, a2 = X.neiA3(a1) - 1;
        X.set_moved(a1);
        X.set_moved(a2);
        double dd1 = dxyA(N, a1, 3, 1, a2, 3, 1);
        double dd2 = dxyA(N, a1, 3, 3, a2, 3, 3);
        if (!AreSame(dd1, P.cis_cut / 2 + P.ra + P.ra) || !AreSame(dd2, P.cis_cut / 2)) snap_cis(P, N, a1, a2, P.cis_cut);
      }
    }
  }
  // step 2 (main.cpp:1411-1590) + repeat (1595-1635): the goto lable4 re-enters
  // the step-2 loop body at the repeat scan's (member, site) position
  X.shuffle(call++);
  int start_csi = 0, start_j = 2;
  bool jump = false;
  int jB = 0, jA1 = 0;
  double jd1 = 0, jd2 = 0;
  for (int guard = 0;; ++guard) {
    if (guard > 4 * csize + 8) {
      atomicOr(X.err, ERR_ALIGN);
      return;
    }
    for (int csi = start_csi; csi < csize; ++csi) {
      int B = res[csi];
      if (jump) B = jB;
      if (B >= NA) {
        for (int j = jump ? start_j : 2; j <= 4; ++j) {
          int a1;
          double dist1, dist2;
          if (jump) {
            jump = false;
            a1 = jA1;
            dist1 = jd1;
            dist2 = jd2;
          } else {
            int Bref = B + 1;
            int A1ref = X.rnei(Bref, j);
            if (!(A1ref != 0 && X.rnei(A1ref, 3) != 0 && X.rnei(X.rnei(A1ref, 3), 2) != 0 && !X.is_moved(B)))
              continue;
            a1 = A1ref - 1;
            dist2 = dxyBA(N, B - NA, j, 2, a1, 3, 2);
            dist1 = dxyBA(N, B - NA, j, 1, a1, 3, 1);
          }
          if (bond_mis_d(P, dist1, dist2)) B = step2_body(X, B, j, a1);
        }
      }
    }
    X.shuffle(call++);
    bool again = false;
    for (int csi = 0; csi < csize && !again; ++csi) {
      int B = res[csi];
      if (B < NA) continue;
      for (int j = 2; j <= 4; ++j) {
        int Bref = B + 1;
        int A1ref = X.rnei(Bref, j);
        if (A1ref != 0 && X.rnei(A1ref, 3) != 0 && X.rnei(X.rnei(A1ref, 3), 2) != 0 && !X.is_moved(B)) {
          int a1 = A1ref - 1;
          double dd2 = dxyBA(N, B - NA, j, 2, a1, 3, 2);
          double dd1 = dxyBA(N, B - NA, j, 1, a1, 3, 1);
          if (bond_mis_d(P, dd1, dd2)) {
            again = true;
            jump = true;
            start_csi = csi;
            start_j = j;
            jB = B;
            jA1 = a1;
            jd1 = dd1;
            jd2 = dd2;
            break;
          }
        }
      }
    }
    if (!again) break;
  }
  // step 3, main.cpp:1645-1687
  for (int csi = 0; csi < csize; ++csi) {
    int m = res[csi];
    if (m < NA && X.neiA2(m) != 0) {
      int lb = X.neiA2(m) - 1 - NA, j = X.neiA4(m);
      if (bond_misaligned(P, N, lb, j, m)) {
        X.set_moved(m);
        snap_bond(P, N, m, lb, j, P.bond_cut);
      }
    }
  }
  // step 4, main.cpp:1691-1732
  for (int csi = 0; csi < csize; ++csi) {
    int m = res[csi];
    if (m < NA && X.neiA2(m) != 0 && X.neiA3(m) != 0 && X.rnei(X.neiA3(m), 2) == 0) {
      int a2 = X.neiA3(m) - 1;
      if (cis_misaligned(P, N, m, a2)) snap_cis(P, N, a2, m, P.cis_cut);
    }
  }
}

// wave-level ordering of LDS / global accesses between the lanes of one wave
// (each wave of the complex kernels works on its own complex: no workgroup
// barrier)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
}

// ---------------------------------------------------------------- wave-parallel alignment
// The lay-down / alignment of a complex staged in LDS (main.cpp:1138-1732)
// with the lanes of one wave.  Lane t stands for member t (BFS position) in
// the steps whose iterations touch disjoint beads, so that their order does
// not matter; the order-dependent parts stay sequential but cheap:
//  * random_shuffle passes (1285, 1345, 1413, 1597): the row is held one
//    member per lane and permuted by shuffles across lanes, swap by swap in
//    the reference's order (the draws are uniform across the wave);
//  * step 0 / step 3 (1284-1332, 1645-1687): each receptor is tested against
//    and snapped onto its own ligand site — ligands are not written;
//  * step 1 (1341-1406): a cis pair of two ligand-bound receptors is handled
//    by the member met first in the shuffled row among those not yet moved
//    (pa moves itself onto its partner); pairs are disjoint;
//  * step 2 + the goto lable4 repeat (1411-1635): the sequential scan over
//    (member, site) in shuffled order only matters at the positions where
//    lable4's body runs (it sets the ligand moved, so at most once per
//    ligand); all (member, site) tests are evaluated at once and a ballot
//    finds the first position that fires; the body re-lays the ligand one
//    bead per lane and lane 0 snaps its receptors and their partners;
//  * step 4 (1691-1732): each ligand-free cis partner is snapped onto its
//    unique ligand-bound partner.
// Every value is computed by the same expressions as the one-lane version
// (complex_align), so the result is bit-identical.  Requires csize <= 64 (CXL).

// one random_shuffle pass over res[0 .. size-2] (libstdc++, main.cpp:1285)
// on the row held one member per lane
template <class CX>
__device__ __forceinline__ int wave_shuffle(const CX& X, int v, uint32_t call, int lane) {
  uint32_t r = 0;
  if (lane >= 1 && lane < X.size - 1) r = X.shuf_rand(call, (uint32_t)lane);
  for (int i = 1; i < X.size - 1; ++i) {
    const int j = (int)((uint32_t)__shfl((int)r, i, 64) % (uint32_t)(i + 1));
    if (i != j) {  // uniform
      const int vi = __shfl(v, i, 64), vj = __shfl(v, j, 64);
      v = lane == i ? vj : (lane == j ? vi : v);
    }
  }
  return v;
}

// the shuffled row into LDS (res, and the inverse map pos)
template <class CX>
__device__ __forceinline__ void wave_publish_row(const CX& X, CxLds* L, int v, int lane) {
  if (lane < X.size) {
    X.res[lane] = v;
    L->pos[v < X.P.NA ? v : v - X.P.NA] = (uint8_t)lane;
  }
  wave_sync();
}

// Lane t stands for member t (BFS position); its encoded protein number
// (CxLds: receptor t -> t, ligand t -> NA + t) is t only for a receptor, so
// the receptor steps take the lanes whose member is a receptor
__device__ __forceinline__ bool lane_receptor(const CxLds* L, int csize, int NA, int lane) {
  return lane < csize && L->slot[lane] < NA;
}

// steps 0 and 3: receptor m onto its ligand site
template <class CX>
__device__ __forceinline__ void wave_snap_bonds(const CX& X, const CxLds* L, int lane) {
  const KParams& P = X.P;
  const int NA = P.NA;
  const int m = lane;
  if (lane_receptor(L, X.size, NA, lane) && X.neiA2(m) != 0) {
    int lb = X.neiA2(m) - 1 - NA, j = X.neiA4(m);
    if (bond_misaligned(P, X.N, lb, j, m)) {
      X.set_moved(m);
      snap_bond(P, X.N, m, lb, j, P.bond_cut);
    }
  }
  wave_sync();
}

// step 2's test at (member position csi, site j): fires lable4's body
template <class CX>
__device__ __forceinline__ bool step2_fires(const CX& X, int B, int j, int& a1) {
  const KParams& P = X.P;
  const int NA = P.NA;
  if (B < NA) return false;
  int Bref = B + 1;
  int A1ref = X.rnei(Bref, j);
  if (!(A1ref != 0 && X.rnei(A1ref, 3) != 0 && X.rnei(X.rnei(A1ref, 3), 2) != 0 && !X.is_moved(B))) return false;
  a1 = A1ref - 1;
  double dist2 = dxyBA(X.N, B - NA, j, 2, a1, 3, 2);
  double dist1 = dxyBA(X.N, B - NA, j, 1, a1, 3, 1);
  return bond_mis_d(P, dist1, dist2);
}

// the first (member position, site) at or after candidate c0 (c = csi * 3 +
// j - 2) whose test fires, or -1; its receptor in a1 (uniform).  64
// candidates per ballot, from the chunk holding c0.
template <class CX>
__device__ __forceinline__ int step2_first(const CX& X, int v, int c0, int lane, int& a1) {
  for (int base = c0 & ~63; base < 3 * X.size; base += 64) {
    const int c = base + lane, csi = c / 3, j = 2 + c % 3;
    const int B = __shfl(v, min(csi, 63), 64);
    int my_a1 = 0;
    const bool f = c >= c0 && c < 3 * X.size && step2_fires(X, B, j, my_a1);
    const uint64_t m = __ballot(f);
    if (!m) continue;
    const int first = __ffsll((unsigned long long)m) - 1;
    a1 = __shfl(my_a1, first, 64);
    return base + first;
  }
  return -1;
}

// lable4's body at candidate c: the ligand re-laid one bead per lane, then
// lane 0 snaps its receptors and their partners (main.cpp:1441-1583)
template <class CX>
__device__ __forceinline__ void wave_step2_body(const CX& X, int v, int c, int a1, int lane) {
  const int B = __shfl(v, min(c / 3, 63), 64), j = 2 + c % 3;
  if (lane < 8) step2_relayout(X, B, j, a1, lane);
  if (lane == 0) X.set_moved(B);
  wave_sync();
  if (lane == 0) step2_sites(X, B);
  wave_sync();
}

template <class CX>
__device__ __forceinline__ void multi_ligand_align_wave(const CX& X, CxLds* L, int lane) {
  const KParams& P = X.P;
  const auto& N = X.N;
  const int NA = P.NA;
  const int csize = X.size;
  uint32_t call = 0;
  int v = lane < csize ? X.res[lane] : 0;  // the row, one member per lane
  // step 0
  v = wave_shuffle(X, v, call++, lane);
  wave_snap_bonds(X, L, lane);
  // step 1: moved flags as left by step 0, read before any is set
  v = wave_shuffle(X, v, call++, lane);
  wave_publish_row(X, L, v, lane);
  {
    const int pa = lane;
    bool go = false;
    int a2 = 0;
    if (lane_receptor(L, csize, NA, lane) && X.neiA2(pa) != 0 && X.neiA3(pa) != 0 && X.rnei(X.neiA3(pa), 2) != 0 &&
        !X.is_moved(pa)) {
      a2 = X.neiA3(pa) - 1;
      go = X.is_moved(a2) || L->pos[pa] < L->pos[a2];  // the partner does not come first
    }
    wave_sync();
    if (go) {
      X.set_moved(pa);
      X.set_moved(a2);
      double dd1 = dxyA(N, pa, 3, 1, a2, 3, 1);
      double dd2 = dxyA(N, pa, 3, 3, a2, 3, 3);
      if (!AreSame(dd1, P.cis_cut / 2 + P.ra + P.ra) || !AreSame(dd2, P.cis_cut / 2)) snap_cis(P, N, pa, a2, P.cis_cut);
    }
    wave_sync();
  }
  // step 2 + repeat
  v = wave_shuffle(X, v, call++, lane);
  int c0 = 0;
  for (int guard = 0;; ++guard) {
    if (guard > 4 * csize + 8) {
      if (lane == 0) atomicOr(X.err, ERR_ALIGN);
      wave_publish_row(X, L, v, lane);
      return;
    }
    for (;;) {  // the pass from c0 to the end
      int a1 = 0;
      const int c = step2_first(X, v, c0, lane, a1);
      if (c < 0) break;
      wave_step2_body(X, v, c, a1, lane);
      c0 = c + 1;
    }
    v = wave_shuffle(X, v, call++, lane);
    int a1 = 0;
    const int c = step2_first(X, v, 0, lane, a1);
    if (c < 0) break;
    wave_step2_body(X, v, c, a1, lane);
    c0 = c + 1;
  }
  wave_publish_row(X, L, v, lane);
  // step 3
  wave_snap_bonds(X, L, lane);
  // step 4
  {
    const int m = lane;
    if (lane_receptor(L, csize, NA, lane) && X.neiA2(m) != 0 && X.neiA3(m) != 0 && X.rnei(X.neiA3(m), 2) == 0) {
      int a2 = X.neiA3(m) - 1;
      if (cis_misaligned(P, N, m, a2)) snap_cis(P, N, a2, m, P.cis_cut);
    }
    wave_sync();
  }
}

// complex_align with the lanes of one wave (staged complex, root = member 0,
// pA = the last receptor in member order); every lane calls
template <class CX>
__device__ __forceinline__ void complex_align_wave(const CX& X, CxLds* L, int nB, int pA, int lane) {
  const KParams& P = X.P;
  const auto& N = X.N;
  if (nB > 1) {
    multi_ligand_align_wave(X, L, lane);
    return;
  }
  if (nB != 1) return;
  const int lbB = 0;
  // lay-down, main.cpp:1140-1193: one bead per lane; the angle and the
  // centre are read by every lane before any bead is written
  if (N.B(lbB, 1, 2, 2) != (N.B(lbB, 1, 1, 2) + P.rb)) {
    double za = N.A(pA, 3, 1, 2);
    double angle = kmcm::atan2((N.B(lbB, 2, 1, 0) - N.B(lbB, 1, 1, 0)), (N.B(lbB, 2, 1, 1) - N.B(lbB, 1, 1, 1))) + P.pai;
    double tx[5][3], ty[5][3];
    ligand_template(P.rb, tx, ty);
    double l0x = N.B(lbB, 1, 1, 0), l0y = N.B(lbB, 1, 1, 1);
    double ca = kmcm::cos(angle), sa = kmcm::sin(angle);
    wave_sync();
    for (int j = 1; j <= 4; ++j)
      for (int k = 1; k <= 2; ++k) {
        if (lane != (j - 1) * 2 + (k - 1)) continue;
        N.B(lbB, j, k, 2) = (j == 1 && k == 2) ? N.A(pA, 3, 1, 2) + P.rb : za;
        N.B(lbB, j, k, 0) = tx[j][k] * ca - ty[j][k] * sa + l0x;
        N.B(lbB, j, k, 1) = tx[j][k] * sa + ty[j][k] * ca + l0y;
      }
    wave_sync();
  }
  // attached receptors (main.cpp:1196-1233): lane j - 2, distinct receptors
  const int j = lane + 2;
  int a1ref = 0;
  if (lane < 3) {
    a1ref = X.neiB(lbB, j);
    if (a1ref != 0 && bond_misaligned(P, N, lbB, j, a1ref - 1)) snap_bond(P, N, a1ref - 1, lbB, j, P.bond_cut);
  }
  wave_sync();
  // their cis partners (1237-1274): in parallel unless a partner is itself
  // one of the ligand's receptors (then the site order decides: one lane)
  int a2ref = 0;
  if (lane < 3 && a1ref != 0) a2ref = X.neiA3(a1ref - 1);
  const int r2 = __shfl(a1ref, 0, 64), r3 = __shfl(a1ref, 1, 64), r4 = __shfl(a1ref, 2, 64);
  const bool clash = a2ref != 0 && (a2ref == r2 || a2ref == r3 || a2ref == r4);
  if (__ballot(clash) == 0) {
    if (a2ref != 0 && cis_misaligned(P, N, a1ref - 1, a2ref - 1)) snap_cis(P, N, a2ref - 1, a1ref - 1, P.cis_cut);
  } else if (lane == 0) {
    for (int jj = 2; jj <= 4; ++jj) {
      int b1 = X.neiB(lbB, jj);
      if (b1 != 0 && X.neiA3(b1 - 1) != 0) {
        int a1 = b1 - 1, a2 = X.neiA3(a1) - 1;
        if (cis_misaligned(P, N, a1, a2)) snap_cis(P, N, a2, a1, P.cis_cut);
      }
    }
  }
  wave_sync();
}

// lay-down + alignment on lane 0, main.cpp:1138-1732 (lbB: store index of the
// root ligand, pA: of the last receptor in member order)
template <class CX>
__device__ __forceinline__ void complex_align(const CX& X, int nB, int lbB, int pA) {
  const KParams& P = X.P;
  const auto& N = X.N;
  if (nB == 1) {
    // lay-down, main.cpp:1140-1193 (exact != test; the receptor is the last
    // one of the rotation loop, 1107 / 1147)
    if (N.B(lbB, 1, 2, 2) != (N.B(lbB, 1, 1, 2) + P.rb)) {
      for (int j = 1; j <= 4; ++j)
        for (int k = 1; k <= 2; ++k) N.B(lbB, j, k, 2) = N.A(pA, 3, 1, 2);
      N.B(lbB, 1, 2, 2) = N.A(pA, 3, 1, 2) + P.rb;
      double angle = kmcm::atan2((N.B(lbB, 2, 1, 0) - N.B(lbB, 1, 1, 0)), (N.B(lbB, 2, 1, 1) - N.B(lbB, 1, 1, 1))) + P.pai;
      double tx[5][3], ty[5][3];
      ligand_template(P.rb, tx, ty);
      double l0x = N.B(lbB, 1, 1, 0), l0y = N.B(lbB, 1, 1, 1);
      double ca = kmcm::cos(angle), sa = kmcm::sin(angle);
      for (int j = 1; j <= 4; ++j)
        for (int k = 1; k <= 2; ++k) {
          N.B(lbB, j, k, 0) = tx[j][k] * ca - ty[j][k] * sa + l0x;
          N.B(lbB, j, k, 1) = tx[j][k] * sa + ty[j][k] * ca + l0y;
        }
    }
    // align attached receptors, main.cpp:1196-1233
    for (int j = 2; j <= 4; ++j) {
      int a1ref = X.neiB(lbB, j);
      if (a1ref != 0 && bond_misaligned(P, N, lbB, j, a1ref - 1)) snap_bond(P, N, a1ref - 1, lbB, j, P.bond_cut);
    }
    // align their cis partners, main.cpp:1237-1274
    for (int j = 2; j <= 4; ++j) {
      int a1ref = X.neiB(lbB, j);
      if (a1ref != 0 && X.neiA3(a1ref - 1) != 0) {
        int a1 = a1ref - 1, a2 = X.neiA3(a1) - 1;
        if (cis_misaligned(P, N, a1, a2)) snap_cis(P, N, a2, a1, P.cis_cut);
      }
    }
  } else if (nB > 1) {
    multi_ligand_align(X);
  }
}


// LDS image of a complex (lanes < csize) from the member records
// register_complex stored: slots and links encoded by BFS position (one
// coalesced 16-byte load per member); returns the lane's member slot or -1
__device__ __forceinline__ int cx_stage_mrec_r(CxLds* L, int4 r, int csize, int NA, int lane) {
  if (lane >= csize) return -1;
  L->slot[lane] = r.x;
  L->res[lane] = r.x < NA ? lane : NA + lane;
  L->mv[lane] = 0;
  if (r.x < NA) {
    L->lk[lane][0] = r.w;
    L->lk[lane][1] = r.y;
    L->lk[lane][2] = r.z;
  } else {
    L->lk[lane][1] = r.y;
    L->lk[lane][2] = r.z;
    L->lk[lane][3] = r.w;
  }
  return r.x;
}
__device__ __forceinline__ int cx_stage_mrec(const Dev& d, CxLds* L, int off, int csize, int NA, int lane) {
  return cx_stage_mrec_r(L, lane < csize ? d.mrec[off + lane] : make_int4(0, 0, 0, 0), csize, NA, lane);
}

// bead (LDS image) of a staged member's R_new row: receptor rows 0..15 are
// (x, y) of bead `row`, 16..23 the z of beads (2h)·4 + kk and (2h+1)·4 + kk;
// ligand rows 0..7 and 8..11 likewise with 2 beads per j (kmc_device.h)
__device__ __forceinline__ void cx_row_beads(bool lig, int row, int& b0, int& b1, bool& xy) {
  const int nk = lig ? 2 : 4, nxy = 4 * nk;
  xy = row < nxy;
  const int h = (row - nxy) / nk, kk = (row - nxy) % nk;
  b0 = xy ? row : (2 * h) * nk + kk;
  b1 = (2 * h + 1) * nk + kk;
}

#ifndef CX_ROWMAJOR  // staged complexes' (member, row) loads and stores ordered row-major (A/B,
#define CX_ROWMAJOR 0    // profiles/r05/complex/r6u_*: k_complex_heavy at C5 428 -> 447 us, C3 52.0 -> 53.7)
#endif
#ifndef CXB_IT  // (A/B: 3 -> 6, every row of a 16-member complex in one round: C5 437 -> 426 us, profiles/r05/complex/r6d_*)
#define CXB_IT 6
#endif
// R_new rows of every staged member into the LDS image: each lane takes
// (member, row) pairs of all members at once, every load in flight before
// the LDS stores
__device__ __forceinline__ void cx_load_beads(const Dev& d, CxLds* L, int csize, int NA, int lane) {
  constexpr int IT = CXB_IT;  // loads in flight per lane (CXL · ROWS_A = 384 rows: two rounds of 3, one of 6)
  for (int e0 = 0; e0 < csize * ROWS_A; e0 += IT * 64) {
  double2 v[IT];
  int qi[IT];  // member | row << 8 | ligand << 16, or -1
#pragma unroll
  for (int it = 0; it < IT; ++it) {
#if CX_ROWMAJOR
    const int e = e0 + lane + it * 64, row = e / csize, q = e - row * csize;
#else
    const int e = e0 + lane + it * 64, q = e / ROWS_A, row = e - q * ROWS_A;
#endif
    qi[it] = -1;
    if (q < csize && row < ROWS_A) {
      const int m = L->slot[q];
      if (m < NA) {
        v[it] = d.nxt.A2(m, row);
        qi[it] = q | row << 8;
      } else if (row < ROWS_B) {
        v[it] = d.nxt.B2(m - NA, row);
        qi[it] = q | row << 8 | 1 << 16;
      }
    }
  }
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    if (qi[it] < 0) continue;
    int b0, b1;
    bool xy;
    cx_row_beads(qi[it] >> 16, (qi[it] >> 8) & 0xff, b0, b1, xy);
    double* b = L->bead[qi[it] & 0xff];
    if (xy) {
      b[b0 * 3] = v[it].x;
      b[b0 * 3 + 1] = v[it].y;
    } else {
      b[b0 * 3 + 2] = v[it].x;
      b[b1 * 3 + 2] = v[it].y;
    }
  }
  }
}

// R_new rows of every staged member (paired layout, kmc_device.h), (member,
// row) pairs of all members at once, and the member row in its shuffled
// order (cluster.log, main.cpp:2291-2305)
__device__ __forceinline__ void cx_write_back(const Dev& d, CxLds* L, int* grow, int csize, int nB, int NA, int lane) {
  for (int e = lane; e < csize * ROWS_A; e += 64) {
#if CX_ROWMAJOR
    const int row = e / csize, q = e - row * csize, m = L->slot[q];
#else
    const int q = e / ROWS_A, row = e - q * ROWS_A, m = L->slot[q];
#endif
    const bool lig = m >= NA;
    if (lig && row >= ROWS_B) continue;
    int b0, b1;
    bool xy;
    cx_row_beads(lig, row, b0, b1, xy);
    const double* b = L->bead[q];
    const double2 v = xy ? make_double2(b[b0 * 3], b[b0 * 3 + 1]) : make_double2(b[b0 * 3 + 2], b[b1 * 3 + 2]);
    if (lig) d.nxt.B2(m - NA, row) = v;
    else d.nxt.A2(m, row) = v;
  }
  if (nB > 1 && lane < csize) {
    const int e = L->res[lane];
    grow[lane] = L->slot[e < NA ? e : e - NA];
  }
}

// the staged members' new records (reference point from LDS; the old ones
// were written by k_move_members), and the extent bound of the proposals
__device__ __forceinline__ void cx_put_new(const KParams& P, const Dev& d, CxLds* L, int csize, int lane, int own,
                                           uint2 home, int st) {
  if (lane >= csize) return;
  const int m = L->slot[lane];
  const double* b = L->bead[lane];
  const int kind = m >= P.NA;
  bool ext = true;
  for (int j = 2; j <= 4; ++j) {
    const int o = (kind ? (j - 1) * 2 : (j - 1) * 4) * 3;
    const double ex = b[o] - b[0], ey = b[o + 1] - b[1];
    ext &= kind ? ex * ex + ey * ey <= 35.0 * 35.0 : ex * ex + ey * ey <= 0.09;
  }
  if (!ext) atomicOr(&d.ctl->err, ERR_GEOMETRY);
  // reference point (ref_point): [1][1] xy; z span of the domain centres
  // [j][1] (receptor) or the centre's z (ligand); receptor [3][3] site
  double zl = b[2], zh = b[2], sx = 0.0, sy = 0.0;
  if (kind) {
    const double ux[3] = {b[2 * 3], b[4 * 3], b[6 * 3]}, uy[3] = {b[2 * 3 + 1], b[4 * 3 + 1], b[6 * 3 + 1]},
                 uz[3] = {b[2 * 3 + 2], b[4 * 3 + 2], b[6 * 3 + 2]};
    put_rec_lig(P, d, home, m, 1, own, b[0], b[1], b[2], ux, uy, uz);
    return;
  }
  {
    const double z1 = b[2], z2 = b[(4) * 3 + 2], z3 = b[(8) * 3 + 2], z4 = b[(12) * 3 + 2];
    zl = fmin(fmin(z1, z2), fmin(z3, z4));
    zh = fmax(fmax(z1, z2), fmax(z3, z4));
    sx = b[(2 * 4 + 2) * 3];
    sy = b[(2 * 4 + 2) * 3 + 1];
  }
  put_rec(P, d, home, m, 1, st, own, b[0], b[1], zl, zh, sx, sy);
}

// Rigid move of one complex, main.cpp:974-1131.  Lane = (member ql of a pass
// of four, bead slot (j-1)*4 + (k-1)); the order-dependent sums (periodic
// shift, centre of mass: BFS member order, 994-1067) are accumulated in member
// order by every lane from shuffled per-member values.  New coordinates go to
// the LDS image (LDS) or straight to R_new.
// pass-0 bead of this lane: member ql = lane / 16, bead (lane/4 % 4 + 1, lane % 4 + 1)
struct Bead0 {
  double x, y, z;
  bool ok;
};
template <bool LDS>
__device__ __forceinline__ Bead0 cx_bead0(const KParams& P, const Dev& d, CxLds* L, const int* grow, int csize, int lane) {
  const int ql = lane >> 4, bj = ((lane >> 2) & 3) + 1, bk = (lane & 3) + 1;
  Bead0 b{0.0, 0.0, 0.0, false};
  if (ql < csize) {
    const int m = LDS ? L->slot[ql] : grow[ql];
    if (bk <= (m < P.NA ? 4 : 2)) {
      b.x = d.cur.P(m, bj, bk, 0);
      b.y = d.cur.P(m, bj, bk, 1);
      b.z = d.cur.P(m, bj, bk, 2);
      b.ok = true;
    }
  }
  return b;
}
template <bool LDS>
__device__ __forceinline__ void cx_rigid(const KParams& P, const Dev& d, CxLds* L, const int* grow, int csize, int nB,
                                         uint32_t rootid, uint32_t step, int lane, Bead0 b0) {
  const int NA = P.NA;
  const int nA = csize - nB;
  auto mslot = [&](int q) { return LDS ? L->slot[q] : grow[q]; };
  double u0, u1, u2, u3;
  kmcr::uniform2(P.key, kmcr::DOM_DIFF, rootid, 0, step, 0, &u0, &u1);
  kmcr::uniform2(P.key, kmcr::DOM_DIFF, rootid, 0, step, 1, &u2, &u3);
  double amp = (nB == 1 ? P.amp_bond : 0.0) * u0;
  double phai = u1 * 2 * P.pai;
  double dx = amp * kmcm::cos(phai), dy = amp * kmcm::sin(phai);
  const int ql = lane >> 4, bj = ((lane >> 2) & 3) + 1, bk = (lane & 3) + 1;
  const int npass = (csize + 3) >> 2;
  auto load = [&](int q, double& x, double& y, double& z) -> bool {
    if (q >= csize) return false;
    const int m = mslot(q);
    if (bk > (m < NA ? 4 : 2)) return false;
    x = d.cur.P(m, bj, bk, 0);
    y = d.cur.P(m, bj, bk, 1);
    z = d.cur.P(m, bj, bk, 2);
    return true;
  };
  const double c0x = b0.x, c0y = b0.y, c0z = b0.z;
  const bool c0 = b0.ok;
  // bead of this lane in pass ps: valid?, R coordinates
  auto bead = [&](int ps, double& x, double& y, double& z) -> bool {
    if (ps == 0) {
      x = c0x;
      y = c0y;
      z = c0z;
      return c0;
    }
    return load(ps * 4 + ql, x, y, z);
  };
  // periodic shift from the members' [1][1] in member order (main.cpp:994-1004)
  double PBx = 0, PBy = 0;
  for (int ps = 0; ps < npass; ++ps) {
    double x = 0, y = 0, z = 0;
    bead(ps, x, y, z);
    const double vx = x + dx, vy = y + dy;
    const int cnt = min(4, csize - ps * 4);
    for (int s = 0; s < cnt; ++s) {
      PBx = PBx + __shfl(vx, s * 16, 64);
      PBy = PBy + __shfl(vy, s * 16, 64);
    }
  }
  PBx = P.box_x * kmcm::round_(PBx / (nA + nB) / P.box_x);
  PBy = P.box_y * kmcm::round_(PBy / (nA + nB) / P.box_y);
  // centre of the members' [j][1] beads, member order then j (main.cpp:1007-1021)
  double cmx = 0, cmy = 0, cmz = 0;
  for (int ps = 0; ps < npass; ++ps) {
    double x = 0, y = 0, z = 0;
    bead(ps, x, y, z);
    const double ax = (x + dx) - PBx, ay = (y + dy) - PBy;
    const int cnt = min(4, csize - ps * 4);
    for (int s = 0; s < cnt; ++s)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        cmx = cmx + __shfl(ax, s * 16 + j * 4, 64);
        cmy = cmy + __shfl(ay, s * 16 + j * 4, 64);
        cmz = cmz + __shfl(z, s * 16 + j * 4, 64);
      }
  }
  cmx = cmx / (4 * nA + 4 * nB);
  cmy = cmy / (4 * nA + 4 * nB);
  cmz = cmz / (4 * nA + 4 * nB);
  Rot t = euler(0, 0, (2 * u2 - 1) * (nB == 1 ? P.rot_bond : 0.0));
  for (int ps = 0; ps < npass; ++ps) {
    double x = 0, y = 0, z = 0;
    if (!bead(ps, x, y, z)) continue;
    const int q = ps * 4 + ql, m = mslot(q);
    double ox = (x + dx) - PBx;
    double oy = (y + dy) - PBy;
    double oz = z;
    const double nx = rx(t, ox, oy, oz, cmx, cmy, cmz), ny = ry(t, ox, oy, oz, cmx, cmy, cmz),
                 nz = rz(t, ox, oy, oz, cmx, cmy, cmz);
    if (LDS) {
      double* b = &L->bead[q][((bj - 1) * (m < NA ? 4 : 2) + (bk - 1)) * 3];
      b[0] = nx;
      b[1] = ny;
      b[2] = nz;
    } else {
      d.nxt.P(m, bj, bk, 0) = nx;
      d.nxt.P(m, bj, bk, 1) = ny;
      d.nxt.P(m, bj, bk, 2) = nz;
    }
  }
}

// ---------------------------------------------------------------- complexes, streamed
// The rigid move of a complex of at most CXL members (main.cpp:974-1131) in
// three steps, so that its members' beads are moved by the same coalesced,
// one-thread-per-slot stream as the free units:
//   cx_params      one thread per complex (the first workgroups of k_propose_free):
//                  the keyed draws, the periodic shift
//                  and the centre of mass (sums over the members' [1][1] and
//                  [j][1] beads in BFS member order, 994-1067), the rotation
//                  matrix -> cxp[root] (16 doubles)
//   k_move_members (a member's thread) every bead moved with its complex's
//                  parameters — the same expressions as the heavy path's
//   k_cx_check     one thread per complex: the lay-down / alignment tests
//                  (1141, 1215, 1255) on R_new; a complex that passes has its
//                  members' new records counted, any other (a test fails, or
//                  several ligands) goes to k_complex_heavy as moved.
#define CXP 16  // doubles per complex: dx dy PBx PBy cmx cmy cmz t[3][3]

// descriptor c of cx_list: current (root alive with this row) and small
__device__ __forceinline__ bool cx_current(const Dev& d, int4 desc) {
  return d.cx_alive[desc.x] == 1u && d.cx_off[desc.x] == desc.y;
}

// complexes c = first, first + stride, ... of the descriptor list
#ifndef CXP_BATCH  // members whose beads cx_params holds in registers at once (its VGPRs bound k_propose_free's)
#define CXP_BATCH 4
#endif
__device__ __forceinline__ void cx_params(const KParams& P, const Dev& d, uint32_t first, uint32_t stride) {
  const uint32_t n = d.ctl->n_cx, step = d.ctl->step;
  for (uint32_t c = first; c < n; c += stride) {
    const int4 desc = d.cx_list[c];
    if (!cx_current(d, desc)) continue;
    const int csize = desc.z & 0xffff, nB = desc.z >> 16, nA = csize - nB;
    if (csize > CXL) {  // the global-memory path: rigid move and alignment in k_complex_heavy
      d.cx_heavy[atomicAdd(&d.ctl->n_heavy, 1u)] = desc;
      continue;
    }
    double u0, u1, u2, u3;
    const uint32_t rk = rkey(P, d, desc.w);
    kmcr::uniform2(P.key, kmcr::DOM_DIFF, rk, 0, step, 0, &u0, &u1);
    kmcr::uniform2(P.key, kmcr::DOM_DIFF, rk, 0, step, 1, &u2, &u3);
    double amp = (nB == 1 ? P.amp_bond : 0.0) * u0;
    double phai = u1 * 2 * P.pai;
    double dx = amp * kmcm::cos(phai), dy = amp * kmcm::sin(phai);
    const int* row = d.members + desc.y;
    // [j][1] beads of CXP_BATCH members at a time in registers, summed in member order
    double PBx = 0, PBy = 0, cmx = 0, cmy = 0, cmz = 0;
    for (int pass = 0; pass < 2; ++pass) {
      for (int t0 = 0; t0 < csize; t0 += CXP_BATCH) {
        double2 xy[CXP_BATCH][4];
        double z[CXP_BATCH][4];
#pragma unroll
        for (int i = 0; i < CXP_BATCH; ++i) {
          const int t = t0 + i;
          if (t >= csize) break;
          const int m = row[t];
          if (pass == 0) {
            xy[i][0] = m < P.NA ? d.cur.Axy(m, 1, 1) : d.cur.Bxy(m - P.NA, 1, 1);
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              xy[i][j] = m < P.NA ? d.cur.Axy(m, j + 1, 1) : d.cur.Bxy(m - P.NA, j + 1, 1);
              z[i][j] = d.cur.P(m, j + 1, 1, 2);
            }
          }
        }
#pragma unroll
        for (int i = 0; i < CXP_BATCH; ++i) {
          if (t0 + i >= csize) break;
          if (pass == 0) {
            PBx = PBx + (xy[i][0].x + dx);
            PBy = PBy + (xy[i][0].y + dy);
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              cmx = cmx + ((xy[i][j].x + dx) - PBx);
              cmy = cmy + ((xy[i][j].y + dy) - PBy);
              cmz = cmz + z[i][j];
            }
          }
        }
      }
      if (pass == 0) {
        PBx = P.box_x * kmcm::round_(PBx / (nA + nB) / P.box_x);
        PBy = P.box_y * kmcm::round_(PBy / (nA + nB) / P.box_y);
      }
    }
    cmx = cmx / (4 * nA + 4 * nB);
    cmy = cmy / (4 * nA + 4 * nB);
    cmz = cmz / (4 * nA + 4 * nB);
    const Rot t = euler(0, 0, (2 * u2 - 1) * (nB == 1 ? P.rot_bond : 0.0));
    double* o = d.cxp + (size_t)desc.x * CXP;
    o[0] = dx;
    o[1] = dy;
    o[2] = PBx;
    o[3] = PBy;
    o[4] = cmx;
    o[5] = cmy;
    o[6] = cmz;
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int b = 0; b < 3; ++b) o[7 + a * 3 + b] = t.t[a][b];
  }
}

// member i (receptor: IS_A, or ligand) of a streamed complex: all beads moved
// with the complex's parameters (every coordinate loaded first, as the free
// units; compile-time row indices keep them in registers); the old record is
// counted here, the new one by k_cx_check / k_complex_heavy
template <bool IS_A>
__device__ __forceinline__ void move_member(const KParams& P, const Dev& d, int i, const double* cp, int root) {
  constexpr int NK = IS_A ? 4 : 2, ROWS = IS_A ? ROWS_A : ROWS_B;
  const int n = IS_A ? P.NA : P.NB, p = IS_A ? i : P.NA + i;
  const double2* src = reinterpret_cast<const double2*>(IS_A ? d.cur.a : d.cur.b);
  double2* dst = reinterpret_cast<double2*>(IS_A ? d.nxt.a : d.nxt.b);
  double2 r[ROWS];
#pragma unroll
  for (int w = 0; w < ROWS; ++w) r[w] = ld_r(src[bead_elem(i, w, n, ROWS)]);
  const double dx = cp[0], dy = cp[1], PBx = cp[2], PBy = cp[3], cmx = cp[4], cmy = cp[5], cmz = cp[6];
  Rot t;
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int b = 0; b < 3; ++b) t.t[a][b] = cp[7 + a * 3 + b];
  // both records (the new one is rewritten by k_complex_heavy when the
  // complex's lay-down / alignment changes beads): reference point [1][1]
  // (row 0), z span of the domain centres (rows 16, 20: z of [1..4][1]) or the
  // ligand centre's z (row 8), receptor [3][3] site (row 10)
  const uint2 h = d.home[p];
  const int st = rec_status(P, d, p), own = d.owner[p];
  auto recs = [&](int w) {
    if constexpr (IS_A)
      put_rec(P, d, h, p, w, st, own, r[0].x, r[0].y, fmin(fmin(r[16].x, r[16].y), fmin(r[20].x, r[20].y)),
              fmax(fmax(r[16].x, r[16].y), fmax(r[20].x, r[20].y)), r[10].x, r[10].y);
    else {
      // subunit centres [j][1]: xy rows 2, 4, 6; z of [2][1] in row 8 (.y), of [3][1], [4][1] in row 10
      const double ux[3] = {r[2].x, r[4].x, r[6].x}, uy[3] = {r[2].y, r[4].y, r[6].y},
                   uz[3] = {r[8].y, r[10].x, r[10].y};
      put_rec_lig(P, d, h, p, w, own, r[0].x, r[0].y, r[8].x, ux, uy, uz);
    }
  };
  recs(0);
  // beads (j, k) and (j+1, k), j odd: xy rows (j-1)·NK + (k-1) and j·NK + (k-1),
  // their z pair in row 4·NK + ((j-1)>>1)·NK + (k-1); moved in place
#pragma unroll
  for (int jp = 0; jp < 2; ++jp)
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int r1 = 2 * jp * NK + k, r2 = (2 * jp + 1) * NK + k, rzr = 4 * NK + jp * NK + k;
      const double z1 = r[rzr].x, z2 = r[rzr].y;
      const double ox1 = (r[r1].x + dx) - PBx, oy1 = (r[r1].y + dy) - PBy;
      const double ox2 = (r[r2].x + dx) - PBx, oy2 = (r[r2].y + dy) - PBy;
      r[r1] = make_double2(rx(t, ox1, oy1, z1, cmx, cmy, cmz), ry(t, ox1, oy1, z1, cmx, cmy, cmz));
      r[r2] = make_double2(rx(t, ox2, oy2, z2, cmx, cmy, cmz), ry(t, ox2, oy2, z2, cmx, cmy, cmz));
      r[rzr] = make_double2(rz(t, ox1, oy1, z1, cmx, cmy, cmz), rz(t, ox2, oy2, z2, cmx, cmy, cmz));
    }
#pragma unroll
  for (int w = 0; w < ROWS; ++w) st_n(dst[bead_elem(i, w, n, ROWS)], r[w]);
  recs(1);
  // the extent bound of the proposal (DESIGN.md §cell list) from registers:
  // [j][1] xy (rows (j-1)·NK) within 0.3 Å (receptor) / 35 Å (ligand) of
  // [1][1]; k_cx_check raises it for the complexes whose tests pass (the
  // others are realigned by k_complex_heavy, which checks its own result)
  bool ext = true;
#pragma unroll
  for (int j = 1; j < 4; ++j) {
    const double ex = r[j * NK].x - r[0].x, ey = r[j * NK].y - r[0].y;
    ext &= IS_A ? ex * ex + ey * ey <= 0.09 : ex * ex + ey * ey <= 35.0 * 35.0;
  }
  if (!ext) atomicOr(&d.cx_ext[root - P.NA], 1u);
}

#ifndef CXCHECK_BATCH  // (A/B builds: 0 = one chain of loads per bond site)
#define CXCHECK_BATCH 1
#endif
__global__ void __launch_bounds__(256) k_cx_check(KParams P, Dev d) {
  const int NA = P.NA, NB = P.NB;
  const uint32_t n = d.ctl->n_cx;
  const Beads& N = d.nxt;
  for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < n; c += gridDim.x * blockDim.x) {
    const int4 desc = d.cx_list[c];
    if (!cx_current(d, desc)) continue;
    const int csize = desc.z & 0xffff, nB = desc.z >> 16;
    if (csize > CXL) continue;
    const uint32_t xb = d.cx_ext[desc.x & CXD_LB];  // (set by k_move_members, cleared here)
    if (xb) d.cx_ext[desc.x & CXD_LB] = 0u;
    bool heavy = nB != 1;
#if CXCHECK_BATCH
    if (!heavy) {
      // lay-down and every bond's alignment tests (pure: evaluated for all
      // three sites at once, whatever the others gave), in three rounds of
      // loads instead of one chain per site: the links, then the partners and
      // the bond beads, then the cis beads (clamped indices: a site without a
      // bond reads slot 0 and discards it)
      const int lb = desc.x;  // the root: the complex's only ligand
      int a1r[3], a2r[3];
#pragma unroll
      for (int j = 0; j < 3; ++j) a1r[j] = B_NEI(d, lb, j + 2);
      heavy = N.B(lb, 1, 2, 2) != (N.B(lb, 1, 1, 2) + P.rb);
#pragma unroll
      for (int j = 0; j < 3; ++j) a2r[j] = A_NEI3(d, a1r[j] > 0 ? a1r[j] - 1 : 0);
      bool mis[3];
#pragma unroll
      for (int j = 0; j < 3; ++j) mis[j] = bond_misaligned(P, N, lb, j + 2, a1r[j] > 0 ? a1r[j] - 1 : 0);
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const bool cm = cis_misaligned(P, N, a1r[j] > 0 ? a1r[j] - 1 : 0, a2r[j] > 0 ? a2r[j] - 1 : 0);
        heavy |= a1r[j] > 0 && (mis[j] || (a2r[j] != 0 && cm));
      }
    }
#else
    if (!heavy) {
      const int lb = desc.x;
      heavy = N.B(lb, 1, 2, 2) != (N.B(lb, 1, 1, 2) + P.rb);
#pragma unroll
      for (int j = 2; j <= 4; ++j) {
        const int a1ref = B_NEI(d, lb, j);
        if (a1ref == 0) continue;
        const int a1 = a1ref - 1, a2ref = A_NEI3(d, a1);
        heavy |= bond_misaligned(P, N, lb, j, a1) || (a2ref != 0 && cis_misaligned(P, N, a1, a2ref - 1));
      }
    }
#endif
    if (heavy) {
      d.cx_heavy[atomicAdd(&d.ctl->n_heavy, 1u)] = make_int4(desc.x | CXD_MOVED, desc.y, desc.z, desc.w);
      continue;
    }
    if (xb) atomicOr(&d.ctl->err, ERR_GEOMETRY);  // a member's proposal broke the extent bound
  }
}

// k_complex_heavy: the complexes the streamed path did not finish.  Staged ones (<=
// CXL members, already moved) are reloaded from R_new into LDS and lane 0
// runs the lay-down / alignment code against LDS; larger ones run the rigid
// move and the alignment on global memory.  Block 0's first wave first runs
// the BFS of the components that overflowed k_bfs's LDS queue (> BFS_QCAP
// members) and moves those it roots.  Launched after k_cx_check on its stream.
#ifndef HEAVY_WAVES  // minimum waves per SIMD of k_complex_heavy (the register budget: 2 = 256, 3 = 168 VGPRs)
#define HEAVY_WAVES 2
#endif
__global__ void __launch_bounds__(256, HEAVY_WAVES) k_complex_heavy(KParams P, Dev d) {
  __shared__ CxLds lds[4];
  const int lane = __lane_id(), NA = P.NA, NB = P.NB;
  CxLds* L = &lds[threadIdx.x >> 6];
  const uint32_t step = d.ctl->step;
  auto global_path = [&](int lb) {
    const int csize = d.cx_size[lb], nB = d.cx_nb[lb];
    const int* brow = d.members + d.cx_off[lb];  // BFS order (kept across steps)
    int* grow = d.shuf + d.cx_off[lb];           // the working row the shuffles permute
    for (int q = lane; q < csize; q += 64) grow[q] = brow[q];
    if (lane == 0) d.shuf_tag[lb] = step;
    wave_sync();
    cx_rigid<false>(P, d, L, grow, csize, nB, rkey(P, d, d.id_of[NA + lb]), step, lane,
                    cx_bead0<false>(P, d, L, grow, csize, lane));
    wave_sync();
    if (lane == 0) {
      int pA = -1;  // last receptor in member order (main.cpp:1107, 1147)
      for (int q = csize - 1; q >= 0 && pA < 0; --q)
        if (grow[q] < NA) pA = grow[q];
      CxT<Beads, GlbLinks> X{P, step, rkey(P, d, d.id_of[NA + lb]), grow, csize, d.nxt, GlbLinks{&d, NA, NB, step},
                             &d.ctl->err};
      complex_align(X, nB, lb, pA);
    }
    wave_sync();
    for (int q = lane; q < csize; q += 64) put_recs_glb(P, d, grow[q]);
  };
  if (blockIdx.x == 0 && threadIdx.x < 64) {
    const uint32_t no = d.ctl->n_overflow;
    for (uint32_t o = 0; o < no; ++o) {
      int lb = lane == 0 ? bfs_overflow_one(P, d, o) : -1;
      lb = __shfl(lb, 0, 64);
      wave_sync();
      if (lb >= 0) global_path(lb);
    }
  }
  const uint32_t n = d.ctl->n_heavy;
  const uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * blockDim.x) >> 6;
  for (uint32_t c = w; c < n; c += nw) {
#ifdef KMC_STAMPS  // diagnostic build: per-phase cycles of the staged path (lane 0 of each wave)
    uint64_t t0_ = Stamper::now(), t_ = t0_;
#define CXS(i)                                                                                   \
  do {                                                                                           \
    if (lane == 0) {                                                                             \
      const uint64_t v_ = Stamper::now();                                                        \
      atomicAdd((unsigned long long*)&d.ctl->stamps[16 + (i)], (unsigned long long)(v_ - t_)); \
      t_ = v_;                                                                                   \
    }                                                                                            \
  } while (0)
#else
#define CXS(i)
#endif
    const int4 desc = d.cx_heavy[c];
    const int lb = desc.x & CXD_LB;
    if (!(desc.x & CXD_MOVED)) {
      global_path(lb);
      continue;
    }
    const int csize = desc.z & 0xffff, nB = desc.z >> 16;
    const int mslot = cx_stage_mrec(d, L, desc.y, csize, NA, lane);
    // this lane's member's record inputs (cx_put_new), loaded here, long before use
    uint2 mhome = make_uint2(0u, 0u);
    int mst = 0;
    if (mslot >= 0) {
      mhome = d.home[mslot];
      mst = rec_status(P, d, mslot);
    }
    wave_sync();
    cx_load_beads(d, L, csize, NA, lane);  // the moved beads back into LDS
    if (nB > 1)  // the shuffles' keyed draws, all at once (main.cpp:1285, 1345, 1413, 1597)
      for (int e = lane; e < CX_SHUF * CXL; e += 64) {
        const int call = e / CXL, pos = e % CXL;
        if (pos >= 1 && pos < csize - 1)
          L->rnd[call][pos] = kmcr::rand31(P.key, kmcr::DOM_SHUF, rkey(P, d, desc.w), call, step, pos);
      }
    wave_sync();
    CXS(0);
    {
      // the last receptor in member order: the highest lane holding one
      const uint64_t rm = __ballot(lane < csize && L->slot[lane] < NA);
      const int pA = rm ? 63 - __clzll((long long)rm) : -1;
      CxT<LdsBeads, LdsLinks> X{P, step, rkey(P, d, desc.w), L->res, csize, LdsBeads{L}, LdsLinks{L, NA}, &d.ctl->err,
                                L->rnd};
      if (P.cx_serial) {  // debug (KMC_CX_SERIAL=1): the one-lane alignment
        if (lane == 0) complex_align(X, nB, 0, pA);
        wave_sync();
      } else {
        complex_align_wave(X, L, nB, pA, lane);  // the root is member 0
      }
    }
    CXS(1);
    cx_write_back(d, L, d.shuf + desc.y, csize, nB, NA, lane);  // shuffled row: shuf (members keeps BFS order)
    if (nB > 1 && lane == 0) d.shuf_tag[lb] = step;
    CXS(2);
    cx_put_new(P, d, L, csize, lane, desc.w, mhome, mst);
    wave_sync();
    CXS(3);
#ifdef KMC_STAMPS
    if (lane == 0) {
      atomicAdd((unsigned long long*)&d.ctl->stamps[20], 1ull);
      atomicMax((unsigned long long*)&d.ctl->stamps[21], (unsigned long long)(t_ - t0_));
      atomicAdd((unsigned long long*)&d.ctl->stamps[22], (unsigned long long)csize);
    }
#endif
#undef CXS
  }
}

// One thread per slot: free receptors, cis dimers (by default), free ligands.
__device__ __forceinline__ void propose_one(const KParams& P, const Dev& d, int p) {
  if (p >= P.N) return;
  const uint32_t step = d.ctl->step;
  const int NA = P.NA;
  uint8_t k = d.ukind[p];
  if (k == U_FREE_A) {
    propose_free_a(P, d, p, step);
  } else if (k == U_DIMER) {
    const int q = A_NEI3(d, p) - 1;
    propose_dimer(P, d, p, q, step);
  } else if (k == U_FREE_B) {
    propose_free_b(P, d, p - P.NA, p, step);
  }
}

// member p of a complex of at most CXL members (cx_params), one thread per
// slot: a separate launch keeps the free units' kernel at 4 waves/SIMD
#ifndef MEMBER_WAVES  // minimum waves per SIMD of k_move_members
#define MEMBER_WAVES 1
#endif
__global__ void __launch_bounds__(256, MEMBER_WAVES) k_move_members(KParams P, Dev d) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x, NA = P.NA;
  if (p >= P.N) return;
  const int r = d.croot[p];
  if (r < 0 || (r & CROOT_BIG)) return;  // (the flag: no cx_size load on the member's chain)
  const double* cp = d.cxp + (size_t)(r - NA) * CXP;
  if (p < NA) move_member<true>(P, d, p, cp, r);
  else move_member<false>(P, d, p - NA, cp, r);
}

// the free units, one thread per slot
// The complexes' rigid-move parameters (cx_params) run in the first gC
// workgroups, ahead of the free units: their short dependent chains of loads
// overlap the free units' HBM stream instead of taking a launch of their own.
#ifndef FREE_WAVES  // minimum waves per SIMD of k_propose_free
#define FREE_WAVES 1
#endif
__global__ void __launch_bounds__(256, FREE_WAVES) k_propose_free(KParams P, Dev d, int gC) {
  if ((int)blockIdx.x < gC) {
    cx_params(P, d, blockIdx.x * blockDim.x + threadIdx.x, (uint32_t)gC * blockDim.x);
    return;
  }
  propose_one(P, d, (int)((blockIdx.x - gC) * blockDim.x + threadIdx.x));
}

// ================================================================ 4. resolve
// Exact pair tests, main.cpp:640-664 (A vs A [1][1] < 2RA; A domains vs B
// subunits < RA+RB), 1798-1826 (B subunits vs B subunits < 2RB; vs A domains).
// sqrt(s) < c is evaluated as s < T(c) (T precomputed exactly on the host).
struct Own {
  double x[4], y[4], z[4];  // receptor domains [k][1] k=1..4 or ligand subunits [k][1] k=2..4 (idx 1..3)
  bool isA;
};
__device__ __forceinline__ void load_own(const KParams& P, const Beads& B, int m, Own& o) {
  o.isA = m < P.NA;
  // [k][1] beads: (x, y) rows, z of domains / subunits 1,2 and 3,4 in two rows
  double2 z12, z34;
  if (o.isA) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const double2 xy = B.Axy(m, k + 1, 1);
      o.x[k] = xy.x;
      o.y[k] = xy.y;
    }
    z12 = B.A2(m, 16);
    z34 = B.A2(m, 20);
  } else {
    int b = m - P.NA;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const double2 xy = B.Bxy(b, k + 1, 1);
      o.x[k] = xy.x;
      o.y[k] = xy.y;
    }
    z12 = B.B2(b, 8);
    z34 = B.B2(b, 10);
  }
  o.z[0] = z12.x;
  o.z[1] = z12.y;
  o.z[2] = z34.x;
  o.z[3] = z34.y;
}

// Every coordinate of q the test needs is loaded before the first
// comparison (one round of loads per candidate, not one per subunit); the
// outcome is the OR of the same comparisons as the reference's loops.
__device__ bool exact_collide(const KParams& P, const Own& o, const Beads& B, int q) {
  const int NA = P.NA;
  const bool qA = q < NA;
  if (o.isA && qA) {  // domain [1][1] against domain [1][1]
    const double2 xy = B.Axy(q, 1, 1), z12 = B.A2(q, 16);
    const double dx = xy.x - o.x[0], dy = xy.y - o.y[0], dz = z12.x - o.z[0];
    return d2(dx, dy, dz) < P.T_aa;
  }
  // [j][1] beads of q, j = 1..4: (x, y) rows and the two z rows
  double qx[4], qy[4], qz[4];
  double2 z12, z34;
  if (qA) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const double2 xy = B.Axy(q, j + 1, 1);
      qx[j] = xy.x;
      qy[j] = xy.y;
    }
    z12 = B.A2(q, 16);
    z34 = B.A2(q, 20);
  } else {
    const int b = q - NA;
    qx[0] = qy[0] = 0.0;
#pragma unroll
    for (int j = 1; j < 4; ++j) {
      const double2 xy = B.Bxy(b, j + 1, 1);
      qx[j] = xy.x;
      qy[j] = xy.y;
    }
    z12 = B.B2(b, 8);
    z34 = B.B2(b, 10);
  }
  qz[0] = z12.x;
  qz[1] = z12.y;
  qz[2] = z34.x;
  qz[3] = z34.y;
  bool hit = false;
  if (o.isA) {  // receptor domains k = 1..4 against ligand subunits j = 2..4
#pragma unroll
    for (int j = 1; j < 4; ++j)
#pragma unroll
      for (int k = 0; k < 4; ++k) hit |= d2(qx[j] - o.x[k], qy[j] - o.y[k], qz[j] - o.z[k]) < P.T_ab;
  } else if (!qA) {  // ligand subunits against ligand subunits
#pragma unroll
    for (int j = 1; j < 4; ++j)
#pragma unroll
      for (int k = 1; k < 4; ++k) hit |= d2(qx[j] - o.x[k], qy[j] - o.y[k], qz[j] - o.z[k]) < P.T_bb;
  } else {  // ligand subunits against receptor domains j = 1..4
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int k = 1; k < 4; ++k) hit |= d2(qx[j] - o.x[k], qy[j] - o.y[k], qz[j] - o.z[k]) < P.T_ab;
  }
  return hit;
}

// conservative single-precision prefilter on reference points (margins ≥ 1 Å
// cover float rounding and the rigid-body extents)
__device__ __forceinline__ bool prefilter(bool mA, float mx, float my, float mzl, float mzh, bool qA, float4 r) {
  float dx = r.x - mx, dy = r.y - my;
  float dxy2 = dx * dx + dy * dy;
  // same kind: centre distance (receptors: z of the lowest domain)
  float dz = r.z - mzl;
  bool same = dxy2 + dz * dz < (mA ? 42.0f * 42.0f : 131.5f * 131.5f);
  // receptor axis [zlo, zhi] vs ligand centre
  float lz = mA ? r.z : mzl, alo = mA ? mzl : r.z, ahi = mA ? mzh : r.w;
  bool mixed = (dxy2 < 86.5f * 86.5f) & (lz > alo - 86.5f) & (lz < ahi + 86.5f);
  return mA == qA ? same : mixed;  // branch-free: evaluated in the scans' inner loops
}

// The pair walk's filters with the xy differences on packed FP32
// (v_pk_add_f32 / v_pk_mul_f32: two lanes of arithmetic per instruction; no
// contraction, so every value is bit-identical to the scalar form): the
// collision prefilter and the reaction prefilter share one dxy2.
#ifndef PAIR_PK
#define PAIR_PK 1
#endif
typedef float pk2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ bool prefilter_d(bool mA, float mzl, float mzh, bool qA, float4 r, float dxy2) {
  const float dz = r.z - mzl;
  const bool same = dxy2 + dz * dz < (mA ? 42.0f * 42.0f : 131.5f * 131.5f);
  const float lz = mA ? r.z : mzl, alo = mA ? mzl : r.z, ahi = mA ? mzh : r.w;
  const bool mixed = (dxy2 < 86.5f * 86.5f) & (lz > alo - 86.5f) & (lz < ahi + 86.5f);
  return mA == qA ? same : mixed;
}

// ---------------------------------------------------------------- emitters
// Output lists with one global counter: entries are staged in an LDS buffer
// (slots handed out per wave: one LDS atomic per emitting wave-instruction),
// and one global atomicAdd per workgroup reserves the output range.  Entries
// beyond the LDS buffer go straight to global memory.
#define EBUF 128
struct WgList {
  int2 buf[EBUF];
  uint32_t n;
  uint32_t base;
};

__device__ __forceinline__ void wg_list_init(WgList& L) {
  if (threadIdx.x == 0) L.n = 0;
  __syncthreads();
}

__device__ __forceinline__ int my_shard() { return blockIdx.x & (NSHARD - 1); }

// wave-aggregated append of the calling lanes' entries to the workgroup's shard
__device__ __forceinline__ bool sl_push(const SList& s, int2 v, uint32_t* err) {
  const int k = my_shard();
  const uint32_t pos = wave_slot(&s.cnt[k]);
  if (pos < s.cap) {
    s.data[(size_t)k * s.cap + pos] = v;
    return true;
  }
  atomicOr(err, ERR_EDGES);
  return false;
}

__device__ __forceinline__ uint32_t sl_total(const SList& s) {
  uint32_t t = 0;
  for (int k = 0; k < NSHARD; ++k) t += min(s.cnt[k], s.cap);
  return t;
}

// entry t of the concatenated shards (t < sl_total)
__device__ __forceinline__ int2 sl_get(const SList& s, uint32_t t) {
  int k = 0;
  for (; k < NSHARD - 1; ++k) {
    const uint32_t c = min(s.cnt[k], s.cap);
    if (t < c) break;
    t -= c;
  }
  return s.data[(size_t)k * s.cap + t];
}

// Block-level view of a list: pre[k] = entries in shards < k (LDS), total in
// pre[NSHARD]; every thread of the block calls (ends with a barrier).
__device__ __forceinline__ uint32_t sl_prefix(const SList& s, uint32_t* pre) {
  if (threadIdx.x < 64) {
    const int k = threadIdx.x;
    const uint32_t c = k < NSHARD ? min(s.cnt[k], s.cap) : 0u;
    uint32_t inc = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      uint32_t v = __shfl_up(inc, o, 64);
      if (k >= o) inc += v;
    }
    if (k < NSHARD) pre[k] = inc - c;
    if (k == NSHARD - 1) pre[NSHARD] = inc;
  }
  __syncthreads();
  return pre[NSHARD];
}
__device__ __forceinline__ int2 sl_at(const SList& s, const uint32_t* pre, uint32_t t) {
  int k = 0;
#pragma unroll
  for (int st = NSHARD / 2; st; st >>= 1)
    if (pre[k + st] <= t) k += st;
  return s.data[(size_t)k * s.cap + (t - pre[k])];
}

__device__ __forceinline__ void wg_emit(WgList& L, int2 v, const SList& out, uint32_t* err) {
  uint32_t s = wave_slot(&L.n);
  if (s < EBUF) {
    L.buf[s] = v;
    return;
  }
  sl_push(out, v, err);
}

// Two lists of the workgroup at once: both slot reservations (one global
// atomic each, on threads 0 and 64) are in flight together.  All threads.
__device__ __forceinline__ void wg_flush2(WgList& L0, const SList& o0, WgList& L1, const SList& o1, uint32_t* err) {
  __syncthreads();
  const uint32_t m0 = min(L0.n, (uint32_t)EBUF), m1 = min(L1.n, (uint32_t)EBUF);
  const int k = my_shard();
  if (threadIdx.x == 0) L0.base = m0 ? atomicAdd(&o0.cnt[k], m0) : 0;
  if (threadIdx.x == 64) L1.base = m1 ? atomicAdd(&o1.cnt[k], m1) : 0;
  __syncthreads();
  const uint32_t b0 = L0.base, b1 = L1.base;
  for (uint32_t t = threadIdx.x; t < m0 + m1; t += blockDim.x) {
    const bool first = t < m0;
    const uint32_t i = first ? t : t - m0, base = first ? b0 : b1;
    const SList& out = first ? o0 : o1;
    if (base + i < out.cap) out.data[(size_t)k * out.cap + base + i] = first ? L0.buf[i] : L1.buf[i];
    else atomicOr(err, ERR_EDGES);
  }
}

// ---------------------------------------------------------------- LDS tiles
// A workgroup owns a block of cells (tile×tile, the tile side chosen on the
// host from the record density).  It stages into LDS every record whose cell
// lies in the block or its one-cell halo: those are the records of the home
// cells of the block + two cells (home list, §records) whose cell code puts
// them into the halo region, plus the outliers listed this step that fall
// into it.  The home cells of a (row, kind) run of columns are one contiguous
// range of the home list, so the staging reads 2·(rows + 4) contiguous
// ranges, all in flight at once; each home entry's column comes from a tag
// written per home cell (no search).  The staged records are binned by their
// cell in LDS (counting sort: LDS atomics, one block scan, scatter) and tagged
// with (segment = halo row · 2 + kind, column).  Every scanning record of the
// block then takes the LDS indices of the records in its cut stencil — per
// neighbour kind, only the cells within that kind pair's reach of the record
// (its offset inside its cell decides which side columns / rows can hold a
// partner) — as six LDS index ranges, and each wave walks its records' pairs
// with every lane busy (tile_walk).  A tile whose records do not fit in
// TCAP goes onto the dense list: k_col_exact brute-forces it from global
// memory (its home records and its outlier bucket, dense_block).
#ifndef TILE_MAX  // (overridable for tile-size sweeps: tools/build_variants.py)
#define TILE_MAX 13
#endif
#define HALO_MAX (TILE_MAX + 2)
// Staged records are binned by (halo row, kind, column, half column).
// (Measured and rejected, round 4: ligands split further by z — those above
// every receptor's reach in a part of their own, with a second copy of the
// ligands near the split for the ligand-ligand reach: 39 % fewer pairs walked
// at C3, but the second copies and the larger bin table cost the staging 14 %
// and the tile size at C5 (whose ligands sit at the membrane, most of them in
// the overlap) — net +-4 % on the scan and a dense-path cliff when the tile
// choice misjudges the copies.)
#define NPART 2
#define NSEG_MAX (NPART * HALO_MAX)
#define HOME_MAX (TILE_MAX + 4)
#define HSEG_MAX (2 * HOME_MAX)
#ifndef SUBC  // sub-columns per cell in the LDS bins (x extent of the cut stencils: 130 / SUBC Å steps;
#define SUBC 3  // A/B, profiles/r05/ab_walk/r6i_*: 2 -> 3, k_pair_scan 114.1 -> 111.5 us at C3, 1265 -> 1228 at C5)
#endif
#define CFLAT_MAX (NSEG_MAX * (HALO_MAX * SUBC + 1) + 1)
#define SCAN_PER ((CFLAT_MAX + 255) / 256)  // bin counters per thread in the block scans
#ifndef TCAP
#define TCAP 640
#endif
#define HTAG_MAX 640  // home entries tagged for the direct column lookup (more: binary search)

// the staged block: cells [x0, x0 + w) × [y0, y0 + h); halo region origin
// (cx0, cy0) = (x0 - 1, y0 - 1), size hw × hh; home region origin (hx0, hy0)
// = (x0 - 2, y0 - 2), size mw × mh (2·mh home segments)
struct TileGeo {
  int x0, y0, w, h, cx0, cy0, hw, hh, hx0, hy0, mw, mh, nhseg;
};
__device__ __forceinline__ TileGeo tile_geo(int x0, int y0, int w, int h) {
  TileGeo G;
  G.x0 = x0;
  G.y0 = y0;
  G.w = w;
  G.h = h;
  G.cx0 = x0 - 1;
  G.cy0 = y0 - 1;
  G.hw = w + 2;
  G.hh = h + 2;
  G.hx0 = x0 - 2;
  G.hy0 = y0 - 2;
  G.mw = w + 4;
  G.mh = h + 4;
  G.nhseg = 2 * G.mh;
  return G;
}

// the home headers live only through the staging, the output lists only
// through the walk and the flush: they share LDS (one more workgroup per CU)
struct TileHdr {
  int hs[HSEG_MAX][HOME_MAX + 1];  // home segment = home row * 2 + kind: first home position of each column
  int hbase[HSEG_MAX];             // home position − home entry index, per home segment
  int hoff[HSEG_MAX + 1];          // home entries before each home segment; [nhseg] = all
  uint16_t htag[HTAG_MAX];         // home segment | column << 8 of each home entry
};
#define WALK_WIN 32  // words of each wave's start bitmap in the pair walk (a window of 1024 pairs)
struct TileLists {
  WgList Lc, Lr;                   // collision candidates, reaction pairs
  alignas(8) uint32_t wbits[4 * WALK_WIN];  // the pair walk's start bitmaps, one per wave (tile_walk)
};
struct TileLds {
  float4 pos[TCAP];
  int2 id[TCAP];                   // {home position | the record's flags, owner key}
  uint16_t tag[TCAP];              // segment | column << 8 of each staged record's cell
  alignas(16) int cstart[CFLAT_MAX];  // [seg][hw · SUBC + 1] flat, bins = (cell column, sub-column): record
                                   // counts, then the LDS index of each bin's first record; [seg][hw · SUBC]
                                   // = the segment's end
  union {
    TileHdr h;
    TileLists l;
  } u;
  int n, nseq, nhome;
  int obkt;                        // the block's outlier bucket (tile index), or -1: the whole outlier list
  uint32_t nout;                   // entries of that bucket
};
__device__ __forceinline__ int tcs(const TileLds& T, int hw, int seg, int b) { return T.cstart[seg * (hw * SUBC + 1) + b]; }
// Bin of float x in halo column hx: the block-wide sub-column index
// (x − x0)·SUBC/cs (float, truncated: monotone in x) clamped into the
// column's SUBC bins.  Records and cut stencils use the same function, so
// an x interval maps onto a contiguous run of bins holding every record in it.
struct SubCol {
  float x0, k;  // the halo region's left edge, SUBC / cs
};
__device__ __forceinline__ SubCol sub_cols(const KParams& P, const TileGeo& G) {
  return SubCol{(float)(P.gx0 + G.cx0 * P.cs), (float)(SUBC / P.cs)};
}
__device__ __forceinline__ int sub_bin(const SubCol& C, int hx, float x) {
  const int g = (int)((x - C.x0) * C.k);
  return min(max(g, hx * SUBC), hx * SUBC + SUBC - 1);
}

// global record index of staged record l (record w of home position hp at 2·hp + w)
__device__ __forceinline__ int tile_global(const TileLds& T, int l) {
  const int x = T.id[l].x;
  return 2 * (x & RID_PID) + (x < 0 ? 1 : 0);
}

// Thread t's SCAN_PER consecutive bin counters a[SCAN_PER·t ..] (16-byte
// aligned): with SCAN_PER = 4 one ds_read_b128 / ds_write_b128 per thread,
// whose 16-lane groups cover the 64 banks once — element-wise, lanes SCAN_PER
// words apart hit every bank SCAN_PER times (SQ_LDS_BANK_CONFLICT).
__device__ __forceinline__ void scan_ld(const int* a, int t, int m, int* v) {
  if (SCAN_PER == 4 && 4 * t + 3 < m) {
    const int4 x = *reinterpret_cast<const int4*>(a + 4 * t);
    v[0] = x.x;
    v[1] = x.y;
    v[2] = x.z;
    v[3] = x.w;
    return;
  }
  if (SCAN_PER % 2 == 0 && SCAN_PER * t + SCAN_PER - 1 < m) {  // 8-byte accesses
#pragma unroll
    for (int k = 0; k < SCAN_PER; k += 2) {
      const int2 x = *reinterpret_cast<const int2*>(a + SCAN_PER * t + k);
      v[k] = x.x;
      v[k + 1] = x.y;
    }
    return;
  }
#pragma unroll
  for (int k = 0; k < SCAN_PER; ++k) v[k] = SCAN_PER * t + k < m ? a[SCAN_PER * t + k] : 0;
}
__device__ __forceinline__ void scan_st(int* a, int t, int m, const int* v) {
  if (SCAN_PER == 4 && 4 * t + 3 < m) {
    *reinterpret_cast<int4*>(a + 4 * t) = make_int4(v[0], v[1], v[2], v[3]);
    return;
  }
  if (SCAN_PER % 2 == 0 && SCAN_PER * t + SCAN_PER - 1 < m) {
#pragma unroll
    for (int k = 0; k < SCAN_PER; k += 2) *reinterpret_cast<int2*>(a + SCAN_PER * t + k) = make_int2(v[k], v[k + 1]);
    return;
  }
#pragma unroll
  for (int k = 0; k < SCAN_PER; ++k)
    if (SCAN_PER * t + k < m) a[SCAN_PER * t + k] = v[k];
}

// exclusive prefix sum of a[0..m) in LDS by the whole workgroup (m <= SCAN_PER·blockDim)
__device__ __forceinline__ int block_excl_scan(int* a, int m, int* wtot) {
  const int t = threadIdx.x, lane = __lane_id(), w = t >> 6, nw = blockDim.x >> 6;
  int v[SCAN_PER];
  scan_ld(a, t, m, v);
  int sum = 0;
#pragma unroll
  for (int k = 0; k < SCAN_PER; ++k) sum += v[k];
  int inc = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(inc, o, 64);
    if (lane >= o) inc += u;
  }
  if (lane == 63) wtot[w] = inc;
  __syncthreads();
  int base = 0, tot = 0;
  for (int k = 0; k < nw; ++k) {
    base += k < w ? wtot[k] : 0;
    tot += wtot[k];
  }
  int run = base + inc - sum;
#pragma unroll
  for (int k = 0; k < SCAN_PER; ++k) {
    const int x = v[k];
    v[k] = run;
    run += x;
  }
  scan_st(a, t, m, v);
  __syncthreads();
  return tot;
}

// Element q of a block's staging sequence: the home records (2 per home
// entry, segment by segment) then the outlier list.  Returns the global
// record index, with the home cell (home records, kind >= 0) or the record's
// own cell (outliers, kind = -1).
__device__ __forceinline__ int tile_elem(const KParams& P, const Dev& d, const TileLds& T, const TileGeo& G, int q, int& ax, int& ay,
                                         int& kind) {
  const int nhome = T.nhome;
  if (q < 2 * nhome) {
    const int e = q >> 1, w = q & 1;
    int seg, hx;
    if (nhome <= P.htag_max) {
      const int tg = T.u.h.htag[e];
      seg = tg & 0xff;
      hx = tg >> 8;
    } else {  // more home entries than tags: search the segment, then the column
      seg = 0;
#pragma unroll
      for (int st = 32; st; st >>= 1)
        if (seg + st <= G.nhseg - 1 && T.u.h.hoff[seg + st] <= e) seg += st;
      const int hp = T.u.h.hbase[seg] + e;
      hx = 0;
#pragma unroll
      for (int st = 16; st; st >>= 1)
        if (hx + st <= G.mw - 1 && T.u.h.hs[seg][hx + st] <= hp) hx += st;
    }
    ax = G.hx0 + hx;
    ay = G.hy0 + (seg >> 1);
    kind = seg & 1;
    return 2 * (T.u.h.hbase[seg] + e) + w;
  }
  if (T.obkt >= 0) {
    const int2 o = d.tout[(size_t)T.obkt * TOUT_CAP + (q - 2 * nhome)];
    ax = o.y & 0xffff;
    ay = (int)((uint32_t)o.y >> 16);
    kind = -1;
    return o.x;
  }
  const int4 o = d.outl[q - 2 * nhome];
  ax = o.y;
  ay = o.z;
  kind = -1;
  return o.x;
}

// Stage the block's records.  Returns false (uniformly) when more than P.tcap
// records fall into the block + halo (the home headers and tags stay valid
// for the brute-force path).
__device__ bool tile_load(const KParams& P, const Dev& d, const TileGeo& G, TileLds& T, float2* site, Stamper& S) {
  const int hw = G.hw, hh = G.hh, mw = G.mw, nhseg = G.nhseg;
  const int nflat = NPART * hh * (hw * SUBC + 1) + 1;
  const SubCol SC = sub_cols(P, G);
  __shared__ int wtot[16];
#ifndef HDR_WAVE
  {  // home segment heads, every load in flight before the stores; cell counters zeroed
    const int xlo = max(G.hx0, 0), xhi = min(G.hx0 + mw - 1, P.ncx - 1);
    constexpr int NH = (HSEG_MAX * (HOME_MAX + 1) + 255) / 256;
    int v[NH];
#pragma unroll
    for (int k = 0; k < NH; ++k) {
      const int idx = threadIdx.x + k * (int)blockDim.x;
      const int seg = idx / (mw + 1), hx = idx - seg * (mw + 1);
      const int y = G.hy0 + (seg >> 1);
      v[k] = 0;
      if (seg < nhseg && y >= 0 && y < P.ncy && xlo <= xhi)
        v[k] = d.hstart[cell_index(P, min(max(G.hx0 + hx, xlo), xhi + 1), y, seg & 1)];
    }
#pragma unroll
    for (int k = 0; k < NH; ++k) {
      const int idx = threadIdx.x + k * (int)blockDim.x;
      const int seg = idx / (mw + 1), hx = idx - seg * (mw + 1);
      if (seg < nhseg) T.u.h.hs[seg][hx] = v[k];
    }
    for (int idx = threadIdx.x; idx < nflat; idx += blockDim.x) T.cstart[idx] = 0;
  }
#else
  const int lane = __lane_id(), wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
  {  // home segment heads (a wave per segment, a lane per column); cell counters zeroed
    const int xlo = max(G.hx0, 0), xhi = min(G.hx0 + mw - 1, P.ncx - 1);
    for (int seg = wv; seg < nhseg; seg += nwv) {
      const int y = G.hy0 + (seg >> 1);
      if (lane <= mw) {
        int v = 0;
        if (y >= 0 && y < P.ncy && xlo <= xhi)
          v = d.hstart[cell_index(P, min(max(G.hx0 + lane, xlo), xhi + 1), y, seg & 1)];
        T.u.h.hs[seg][lane] = v;
      }
    }
    for (int idx = threadIdx.x; idx < nflat; idx += blockDim.x) T.cstart[idx] = 0;
  }
#endif
  __syncthreads();
  S(d, 0);
  if (threadIdx.x < 64) {  // home segment lengths -> entries before each segment
    const int seg = threadIdx.x;
    const int len = seg < nhseg ? T.u.h.hs[seg][mw] - T.u.h.hs[seg][0] : 0;
    int inc = len;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(inc, o, 64);
      if (seg >= o) inc += t;
    }
    const int total = __shfl(inc, 63, 64);
    if (seg <= nhseg) T.u.h.hoff[seg] = inc - len;
    if (seg < nhseg) T.u.h.hbase[seg] = T.u.h.hs[seg][0] - (inc - len);
    if (seg == 0) {
      T.nhome = total;
      T.nseq = 2 * total + (T.obkt >= 0 ? (int)T.nout : (int)min(d.ctl->n_outl, d.outl_cap));
    }
  }
  __syncthreads();
  if (T.nhome <= P.htag_max)  // home entry -> (segment, column) tags, one thread per home cell
    for (int idx = threadIdx.x; idx < nhseg * mw; idx += blockDim.x) {
      const int seg = idx / mw, hx = idx - seg * mw;
      const int e0 = T.u.h.hoff[seg] + (T.u.h.hs[seg][hx] - T.u.h.hs[seg][0]), e1 = e0 + (T.u.h.hs[seg][hx + 1] - T.u.h.hs[seg][hx]);
      for (int e = e0; e < e1; ++e) T.u.h.htag[e] = (uint16_t)(seg | hx << 8);
    }
  __syncthreads();
  S(d, 1);
  const int nseq = T.nseq;
#ifndef STAGE_NE
#define STAGE_NE 4
#endif
  constexpr int NE = STAGE_NE;  // elements per thread in flight
  const bool one = nseq <= NE * (int)blockDim.x;  // every element held in registers through the binning
  float4 rpos[NE];  // the staged records in registers: position, then {id, site}
  int4 rids[NE];
  int cell[NE], rank[NE], gi[NE], pre[NE];  // pre: sub-bin | column << 8 | halo row << 16, or -1
  // elements base + k·blockDim + tid: record, global index, flat cell index
  // (-1: not in the block + halo)
  auto load = [&](int base) {
    int ax[NE], ay[NE], kd[NE];
#pragma unroll
    for (int k = 0; k < NE; ++k) {
      const int q = base + k * (int)blockDim.x + (int)threadIdx.x;
      gi[k] = q < nseq ? tile_elem(P, d, T, G, q, ax[k], ay[k], kd[k]) : -1;
    }
#pragma unroll
    for (int k = 0; k < NE; ++k)
      if (gi[k] >= 0) {
        const int4* rp = reinterpret_cast<const int4*>(d.rec + gi[k]);
        const int4 a = rp[0], b = rp[1];
        rpos[k] = make_float4(__int_as_float(a.x), __int_as_float(a.y), __int_as_float(a.z), __int_as_float(a.w));
        rids[k] = b;
      }
#pragma unroll
    for (int k = 0; k < NE; ++k) {
      pre[k] = -1;
      if (gi[k] < 0) continue;
      int x = ax[k], y = ay[k];
      if (kd[k] >= 0) {  // home record: its cell from the code; outliers come from the list
        const int c = rec_code(make_int2(rids[k].x, rids[k].y));
        if (c == RID_OUT) continue;
        x += c % 3 - 1;
        y += c / 3 - 1;
      }
      const int hx = x - G.cx0, hy = y - G.cy0;
      if (hx < 0 || hx >= hw || hy < 0 || hy >= hh) continue;
      pre[k] = sub_bin(SC, hx, rpos[k].x) | hx << 8 | hy << 16;
    }
  };
  auto bin = [&]() {
#pragma unroll
    for (int k = 0; k < NE; ++k) {
      cell[k] = -1;
      if (pre[k] < 0) continue;
      const int b = pre[k] & 0xff, hx = (pre[k] >> 8) & 0xff, hy = pre[k] >> 16;
      const int seg = hy * NPART + ((rids[k].x & RID_LIG) ? 1 : 0);
      cell[k] = (seg * (hw * SUBC + 1) + b) | (seg | hx << 8) << 16;  // flat bin | LDS tag << 16
    }
  };
  auto count = [&]() {
#pragma unroll
    for (int k = 0; k < NE; ++k)
      if (cell[k] >= 0) rank[k] = atomicAdd(&T.cstart[cell[k] & 0xffff], 1);
  };
  if (one) {
    load(0);
    bin();
    count();
  } else {
    for (int base = 0; base < nseq; base += NE * blockDim.x) {
      load(base);
      bin();
      count();
    }
  }
  __syncthreads();
  S(d, 2);
  const int n = block_excl_scan(T.cstart, nflat, wtot);
  if (threadIdx.x == 0) T.n = n;
  S(d, 3);
  if (n > P.tcap) return false;
  // LDS record: the home position in place of the slot (tile_global)
  auto place = [&](int k, int l, int cl) {
    T.pos[l] = rpos[k];
    T.id[l] = make_int2((gi[k] >> 1) | (rids[k].x & ~RID_PID), rids[k].y);
    if (site) site[l] = make_float2(__int_as_float(rids[k].z), __int_as_float(rids[k].w));
    T.tag[l] = (uint16_t)(cl >> 16);
  };
  if (one) {
#pragma unroll
    for (int k = 0; k < NE; ++k)
      if (cell[k] >= 0) place(k, T.cstart[cell[k] & 0xffff] + rank[k], cell[k]);
  } else {
    // a second pass with the counters as cursors: each ends at its cell's
    // end (= the next cell's start), shifted back afterwards
    for (int base = 0; base < nseq; base += NE * blockDim.x) {
      load(base);
      bin();
#pragma unroll
      for (int k = 0; k < NE; ++k)
        if (cell[k] >= 0) place(k, atomicAdd(&T.cstart[cell[k] & 0xffff], 1), cell[k]);
    }
    __syncthreads();
    // every counter one bin up: element i takes element i - 1 (the previous
    // thread's last element from its lane, or from LDS for a wave's lane 0)
    int v[SCAN_PER];
    const int t = (int)threadIdx.x;
    scan_ld(T.cstart, t, nflat, v);
    const int prev_lane = __shfl_up(v[SCAN_PER - 1], 1, 64);
    const int prev = t == 0 ? 0 : (__lane_id() == 0 ? (SCAN_PER * t - 1 < nflat ? T.cstart[SCAN_PER * t - 1] : 0) : prev_lane);
#pragma unroll
    for (int k = SCAN_PER - 1; k >= 1; --k) v[k] = v[k - 1];
    v[0] = prev;
    __syncthreads();
    scan_st(T.cstart, t, nflat, v);
  }
  __syncthreads();
  S(d, 4);
  return true;
}

// Record ranges of the staged kind `part` for the record at (seg, hx): the
// bins that can hold a record with x in [xlo, xhi] and y in [ylo, yhi] (an
// interval around the record, less than a cell beyond its cell on each side):
// three row ranges (empty when the row is out of reach).
__device__ __forceinline__ void item_ranges(const KParams& P, const TileLds& T, const TileGeo& G, int seg, int hx,
                                           float xlo, float xhi, float ylo, float yhi, int part, int* r0, int* r1) {
  const int hy = seg / NPART;
  const int cx = G.cx0 + hx, cy = G.cy0 + hy;
  const float xb = (float)(P.gx0 + cx * P.cs), yb = (float)(P.gy0 + cy * P.cs), cs = (float)P.cs;
  const int lo = hx - (xlo < xb ? 1 : 0), hi = hx + (xhi > xb + cs ? 1 : 0);
  // bins from the sub-column of xlo in the first cell to that of xhi in the
  // last (sub_col is monotone: every record with x in the interval lies in
  // between)
  const SubCol SC = sub_cols(P, G);
  const int blo = sub_bin(SC, lo, xlo), bhi = sub_bin(SC, hi, xhi);
  const bool down = ylo < yb, up = yhi > yb + cs;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int s = (hy - 1 + k) * NPART + part;
    const bool on = k == 1 || (k == 0 ? down : up);
    r0[k] = on ? tcs(T, G.hw, s, blo) : 0;
    r1[k] = on ? tcs(T, G.hw, s, bhi + 1) : 0;
  }
}

// Pairs of the block, without a pair list: rng(l, seg, hx, r0, r1) gives the
// six ranges (kind 0 rows, kind 1 rows) of a scanning record l, or false.
// Every lane of a wave holds one record's ranges; the wave walks the
// concatenation of its lanes' ranges 64 pairs at a time — lane L takes pair
// j + L, finds its owner lane and its neighbour record from the owner's packed
// range starts — so every lane checks a pair, the owner's record is a
// broadcast LDS read and the neighbour records of consecutive lanes are mostly
// consecutive.
// Owner lookup (WALK_BITS): the lanes that have pairs are first moved to the
// front in lane order (ds_permute), so every owner's range is non-empty and
// their starts are distinct; each owner sets the bit of its first pair in a
// per-wave bitmap in LDS, and the owner of pair q is (starts <= q) − 1: one
// broadcast read of the chunk's 64 bits and a popcount per lane, in place of
// a six-step binary search of dependent lane shuffles.
// chk(l, r) for every pair; all threads call (no barrier).
#ifndef WALK_STRIDE  // (A/B builds: 0 = each wave takes 64 consecutive records)
#define WALK_STRIDE 1
#endif
#ifndef WALK_BITS  // (A/B builds: 0 = binary search over the lanes' prefix)
#define WALK_BITS 1
#endif
#ifndef WALK_PERM  // (A/B builds: 0 = lane L of wave w takes record base + 4L + w)
#define WALK_PERM 1
#endif
// Item record of lane `lane` of wave `wv` in the 256-record block at `base`
// (4 waves).  The waves sample the whole block (the staged records are in bin
// order; each wave should walk about as many pairs as the others), in runs of
// 16 consecutive records: lane 16g + i takes record 16·((5g + 4wv) mod 16) + i
// — the four waves' runs {5g + 4wv} cover the 16 runs once — so the owner
// reads of the walk (T.pos: ds_read_b128, 16-lane groups, banks (a/4) mod 64;
// T.id, site: ds_read_b64, 32-lane halves) hit distinct banks: a run's 16
// records fill the 64 banks, and runs r, r + 5 of one half differ in parity
// (16 records = 128 B apart mod 256 B).  Records base + 4·lane + wv (the
// round-robin order before) put a group's lanes 64 B apart: 4-way conflicts
// on every owner read (SQ_LDS_BANK_CONFLICT, profiles/r05/ab_walk).
#ifndef WALK_MAXSEL  // the owner's range of a pair chosen by one unsigned max over its packed words (A/B,
#define WALK_MAXSEL 0    // profiles/r05/ab_walk/r7a_*: k_pair_scan 112.3 -> 113.0 us at C3, 1232 -> 1237 at C5)
#endif
#define PAIR_THREADS 256  // threads of a k_pair_scan workgroup (tile_walk's wave count)
// -DWALK_STATS=1 (diagnostic build): the pairs the walks visit, summed over
// the launch (read by KMC_DEBUG_COUNTS)
#ifndef WALK_STATS
#define WALK_STATS 0
#endif
#if WALK_STATS
__device__ unsigned long long kmc_walk_pairs;
__device__ unsigned long long kmc_walk_pairs_old;  // of them, the pairs of old-position (non-proposal) items
#endif
__device__ __forceinline__ int walk_item(int base, int lane, int wv, int nw) {
#if WALK_PERM
  if (nw == 4) return base + 16 * ((5 * (lane >> 4) + 4 * wv) & 15) + (lane & 15);
#endif
  return base + lane * nw + wv;
}
template <class Rng, class Chk>
__device__ __forceinline__ void tile_walk(const TileGeo& G, const TileLds& T, uint32_t* wbits, Rng rng, Chk chk) {
  const int n = T.n, lane = __lane_id();
  // records go to the waves spread over the block (walk_item): the staged
  // records are in bin order, so each wave samples the whole block and the
  // waves of a workgroup walk about the same number of pairs
#if WALK_STRIDE
  constexpr int nw = PAIR_THREADS / 64;  // (the pair scan's only block size)
  const int wv = threadIdx.x >> 6;
#endif
  for (int base = 0; base < n; base += blockDim.x) {
#if WALK_STRIDE
    const int l = walk_item(base, lane, wv, nw);
#else
    const int l = base + threadIdx.x;
#endif
    int r0[6], r1[6];
    bool item = false;
    if (l < n) {
      const int tg = T.tag[l], seg = tg & 0xff, hx = tg >> 8, hy = seg / NPART;
      if (hy >= 1 && hy <= G.h && hx >= 1 && hx <= G.w) item = rng(l, seg, hx, r0, r1);
    }
    // range starts | pairs before the range << 16 (LDS indices < TCAP, counts < 6 TCAP)
    uint32_t pk[6];
    int tot = 0;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const int len = item ? r1[k] - r0[k] : 0;
#if WALK_MAXSEL
      pk[k] = len > 0 ? (uint32_t)r0[k] | (uint32_t)tot << 16 : 0u;  // (an empty range never wins the max)
#else
      pk[k] = (uint32_t)(item ? r0[k] : 0) | (uint32_t)tot << 16;
#endif
      tot += len;
    }
#if WALK_BITS
    const uint64_t Z = __ballot(tot > 0);
    if (Z == 0) continue;  // (uniform)
    {  // owners to the front: lane `dst` receives this lane's ranges and its lane index
      const uint64_t lt = (1ull << lane) - 1ull;
      const int nz = __popcll(Z);
      const int da = (tot > 0 ? __popcll(Z & lt) : nz + __popcll(~Z & lt)) << 2;
      tot = __builtin_amdgcn_ds_permute(da, tot | lane << 24);
#pragma unroll
      for (int k = 0; k < 6; ++k) pk[k] = (uint32_t)__builtin_amdgcn_ds_permute(da, (int)pk[k]);
    }
    const int olane = (int)((uint32_t)tot >> 24);
    tot &= 0xffffff;
#endif
    int inc = tot;  // wave-level inclusive prefix (every lane of the wave is here)
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(inc, o, 64);
      if (lane >= o) inc += t;
    }
    const int excl = inc - tot, wtot = __shfl(inc, 63, 64);
#if WALK_STATS
    if (lane == 0) atomicAdd(&kmc_walk_pairs, (unsigned long long)wtot);
    {
      int old = (item && T.id[l].x >= 0) ? r1[0] - r0[0] + r1[1] - r0[1] + r1[2] - r0[2] + r1[3] - r0[3] +
                                               r1[4] - r0[4] + r1[5] - r0[5]
                                         : 0;
      for (int o = 32; o > 0; o >>= 1) old += __shfl_down(old, o, 64);
      if (lane == 0) atomicAdd(&kmc_walk_pairs_old, (unsigned long long)old);
    }
#endif
#if !WALK_STRIDE
    const int l0 = l - lane;
#endif
#if WALK_BITS
    // excl < 6 TCAP · 64 < 2^24: one word carries the owner's first pair and lane
    const int ew = excl | olane << 24;
    uint32_t* wb = wbits + (threadIdx.x >> 6) * WALK_WIN;
    const uint32_t le_lo = lane < 32 ? (2u << lane) - 1u : ~0u, le_hi = lane < 32 ? 0u : (2u << (lane - 32)) - 1u;
    int before = 0;  // owners whose first pair precedes the chunk
    for (int w0 = 0; w0 < wtot; w0 += 32 * WALK_WIN) {
      // (a wave's LDS operations complete in order: the clear, the bits and
      // the reads below need no barrier)
      if (lane < WALK_WIN) wb[lane] = 0u;
      if (tot > 0 && excl >= w0 && excl < w0 + 32 * WALK_WIN)
        atomicOr(&wb[(excl - w0) >> 5], 1u << ((excl - w0) & 31));
      const int wend = min(wtot, w0 + 32 * WALK_WIN);
      for (int j = w0; j < wend; j += 64) {
        const uint2 m = *reinterpret_cast<const uint2*>(wb + ((j - w0) >> 5));
        const int o = before + __popc(m.x & le_lo) + __popc(m.y & le_hi) - 1;
        before += __popc(m.x) + __popc(m.y);
        const int q = j + lane, oa = o << 2;
        const int eo = __builtin_amdgcn_ds_bpermute(oa, ew);
        const int t = q - (eo & 0xffffff);
#if WALK_MAXSEL
        // the last non-empty range starting at or before pair t: its packed
        // word (start | pairs before << 16) is the largest below (t + 1) << 16,
        // and x - (t + 1) << 16 (mod 2^32) orders those above every other word
        const uint32_t T1 = (uint32_t)(t + 1) << 16;
        uint32_t mx = (uint32_t)__builtin_amdgcn_ds_bpermute(oa, (int)pk[0]) - T1;
#pragma unroll
        for (int k = 1; k < 6; ++k) mx = max(mx, (uint32_t)__builtin_amdgcn_ds_bpermute(oa, (int)pk[k]) - T1);
        const uint32_t sel = mx + T1;
#else
        uint32_t sel = (uint32_t)__builtin_amdgcn_ds_bpermute(oa, (int)pk[0]);
#pragma unroll
        for (int k = 1; k < 6; ++k) {
          const uint32_t v = (uint32_t)__builtin_amdgcn_ds_bpermute(oa, (int)pk[k]);
          if ((int)(v >> 16) <= t) sel = v;
        }
#endif
#if WALK_STRIDE
        if (q < wtot) chk(walk_item(base, (int)((uint32_t)eo >> 24), wv, nw), (int)(sel & 0xffffu) + t - (int)(sel >> 16));
#else
        if (q < wtot) chk(l0 + ((uint32_t)eo >> 24), (int)(sel & 0xffffu) + t - (int)(sel >> 16));
#endif
      }
    }
#else
    for (int j = 0; j < wtot; j += 64) {
      const int q = j + lane;
      int o = 0;  // owner: the number of lanes whose inclusive prefix is <= q
#pragma unroll
      for (int s = 32; s; s >>= 1)
        if (__shfl(inc, o + s - 1, 64) <= q) o += s;
      o = min(o, 63);
      const int t = q - __shfl(excl, o, 64);
      uint32_t sel = __shfl(pk[0], o, 64);
#pragma unroll
      for (int k = 1; k < 6; ++k) {
        const uint32_t v = __shfl(pk[k], o, 64);
        if ((int)(v >> 16) <= t) sel = v;
      }
#if WALK_STRIDE
      if (q < wtot) chk(walk_item(base, o, wv, nw), (int)(sel & 0xffffu) + t - (int)(sel >> 16));
#else
      if (q < wtot) chk(l0 + o, (int)(sel & 0xffffu) + t - (int)(sel >> 16));
#endif
    }
#endif
  }
}

// Up to four (a, b) entries held in registers per lane while pairs are
// checked; the lanes of a wave then reserve their slots with one LDS atomic.
// (LDS indices packed a | b << 16: TCAP < 2^16)
struct PairBuf {
  uint32_t v0, v1, v2, v3;
  int n;
};
__device__ __forceinline__ void pair_push(PairBuf& b, int2 v) {
  const uint32_t x = (uint32_t)v.x | (uint32_t)v.y << 16;
  b.v0 = b.n == 0 ? x : b.v0;
  b.v1 = b.n == 1 ? x : b.v1;
  b.v2 = b.n == 2 ? x : b.v2;
  b.v3 = b.n == 3 ? x : b.v3;
  ++b.n;
}
// active lanes of a wave; entries mapped through f on the way out
template <class F>
__device__ __forceinline__ void pair_flush(const PairBuf& b, WgList& L, const SList& out, uint32_t* err, F f) {
  const int n = min(b.n, 4);
  const uint64_t lt = (1ull << __lane_id()) - 1ull;
  const uint64_t b0 = __ballot(n & 1), b1 = __ballot(n & 2), b2 = __ballot(n & 4);
  const uint32_t pre = __popcll(b0 & lt) + 2 * __popcll(b1 & lt) + 4 * __popcll(b2 & lt);
  const uint32_t tot = __popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2);
  if (tot == 0) return;
  const int leader = __ffsll((unsigned long long)__ballot(1)) - 1;
  uint32_t base = 0;
  if (__lane_id() == leader) base = atomicAdd(&L.n, tot);
  base = __shfl(base, leader, 64);
  for (int k = 0; k < n; ++k) {
    const uint32_t x = k == 0 ? b.v0 : k == 1 ? b.v1 : k == 2 ? b.v2 : b.v3;
    const int2 v = f(make_int2((int)(x & 0xffffu), (int)(x >> 16)));
    const uint32_t s = base + pre + k;
    if (s < EBUF) {
      L.buf[s] = v;
    } else {
      const int sh = my_shard();
      const uint32_t pos = atomicAdd(&out.cnt[sh], 1u);
      if (pos < out.cap) out.data[(size_t)sh * out.cap + pos] = v;
      else atomicOr(err, ERR_EDGES);
    }
  }
}

// reach (xy, Å) of the float prefilters per kind pair, + 1 Å for the float
// cell bounds: receptor-receptor 42, receptor-ligand 86.5, ligand-ligand: any
// collision has centres < 130 Å apart (DESIGN.md §cell list), i.e. all cells
#define REACH_AA 43.0f
#define REACH_AB 87.5f
#define REACH_BB 131.0f
#define REACH_RL 106.0f
#define REACH_CIS 58.0f
// cis search around the item's [3][3] site: the 16 Å site prefilter + 20.3 Å
// from a receptor's site to its record point + 1.2 Å for float rounding
#define REACH_CSITE 37.5f
#ifndef CIS_SITE  // (A/B builds: 0 = the cis search around the record point, REACH_CIS)
#define CIS_SITE 1
#endif

// ---------------------------------------------------------------- 4a. scan
// Pass A: every proposal record (member m of unit u = its owner) is checked
// against the records of its cells.  The filters that do not depend on any
// unit's fate are applied here (main.cpp:640-664 visits R_new, i.e. the
// proposals of earlier units and the old positions of later ones):
//   owner kq == u : only the unit's other proposal records
//   owner kq >  u : only old-position records
//   owner kq <  u : both (which one counts is decided by kq's fate, pass C)
// A record passing them and the conservative prefilter is a candidate.
__device__ __forceinline__ void col_emit(const Dev& d, WgList& L, int rs, int rg) {
  wg_emit(L, make_int2(rs, rg), d.cand, &d.ctl->err);
}

// the fate-independent filters + prefilter for one (proposal, record) pair
// (records identified by slot or by home position: both unique per protein)
__device__ __forceinline__ bool col_pair(int2 me, float4 mp, int2 id, float4 rp) {
  const int m = me.x & RID_PID, u = me.y;
  const int q = id.x & RID_PID, kq = id.y;
  const bool isnew = id.x < 0;
  const bool own_ok = kq == u ? isnew : (kq > u ? !isnew : true);
  return (q != m) & own_ok & prefilter(!(me.x & RID_LIG), mp.x, mp.y, mp.z, mp.w, !(id.x & RID_LIG), rp);
}

// the receptor of record `me` can take part in a reaction (either bond free)
__device__ __forceinline__ bool rxn_item(int2 me) {
  return !(me.x & RID_LIG) & ((me.x & (RID_ST2 | RID_ST3)) != (RID_ST2 | RID_ST3));
}

// prefilter of one (receptor record, record) pair, finality aside
__device__ __forceinline__ bool rxn_pair(int2 me, float4 mp, float2 ms, int2 id, float4 rp, float2 qs) {
  const int i = me.x & RID_PID, q = id.x & RID_PID;
  const bool isB = (id.x & RID_LIG) != 0;
  const float dx = rp.x - mp.x, dy = rp.y - mp.y;
  const float dxy2 = dx * dx + dy * dy;
  const bool rl_ok = isB & !(me.x & RID_ST2) & (dxy2 < 105.0f * 105.0f) & (rp.z > mp.z - 85.0f) &
                     (rp.z < mp.w + 85.0f);
  const float gap = fmaxf(fmaxf(rp.z - mp.w, mp.z - rp.w), 0.0f);
  const float tx = qs.x - ms.x, ty = qs.y - ms.y;
  const bool cis_ok = !isB & !(me.x & RID_ST3) & !(id.x & RID_ST3) & (dxy2 < 57.0f * 57.0f) & (gap < 16.0f) &
                      (tx * tx + ty * ty < 16.0f * 16.0f);
  return (q != i) & (rl_ok | cis_ok);
}

// ---------------------------------------------------------------- 4b. exact
// u rejected; the first to reject it lists it for the commit
__device__ __forceinline__ void mark_rej(const Dev& d, int u, uint32_t tag) {
  if (bad_key(d, u)) return;
  uint32_t old = atomicMax(&d.ustate[u], tag | S_REJ);
  if (old != (tag | S_REJ)) sl_push(d.rej, make_int2(u, 0), &d.ctl->err);  // at most once per unit
}

#ifndef COL_AA_FAST  // receptor-receptor candidates load only the rows their test reads
#define COL_AA_FAST 1  // (A/B, profiles/r04/ab_r4r: k_col_exact 43.4 -> 39.1 us at C3)
#endif
// Pass B: exact fp64 overlap test of each candidate (main.cpp:640-664,
// 1798-1826).  A collision with a record whose relevance is already known
// (own unit, or a later unit's old position) rejects u outright; one with an
// earlier unit's record becomes a conflict entry (u, kq, isnew) for pass C.
// Unit states this step: untouched = accepted, S_PEND, S_REJ (atomicMax).
// Refinement from the two records alone (float, conservative): can the pair
// collide?  A ligand record carries its subunit centres to within 0.87 Å
// (lig_pack); a receptor's domain centres lie within 0.3 Å of the vertical
// segment (record x, y; z from its lowest to its highest domain) — both
// enforced by the extent bound.  Ligand pairs: some subunit pair within 2RB,
// ligand–receptor: some subunit within RA + RB of the segment, each with the
// rounding margins in P.ref_bb / P.ref_ab.  Receptor pairs pass (their
// prefilter is already the exact test's up to 2 Å).  At C5, 93 % of the
// ligand candidates do not collide (KMC_DEBUG_CAND).
__device__ __forceinline__ void lig_subs(const Rec& r, float* x, float* y, float* z, bool& ok) {
  const uint32_t w0 = __float_as_uint(r.pos.w), w1 = __float_as_uint(r.site.x), w2 = __float_as_uint(r.site.y);
  const uint32_t b[9] = {w0, w0 >> 8, w0 >> 16, w0 >> 24, w1, w1 >> 8, w1 >> 16, w1 >> 24, w2};
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    x[j] = r.pos.x + (float)(int8_t)(b[3 * j] & 0xff);
    y[j] = r.pos.y + (float)(int8_t)(b[3 * j + 1] & 0xff);
    z[j] = r.pos.z + (float)(int8_t)(b[3 * j + 2] & 0xff);
  }
  ok = ((w2 >> 8) & 1u) == 0u;
}
__device__ __forceinline__ bool col_refine(const KParams& P, const Rec& a, const Rec& b) {
  const bool la = (a.id.x & RID_LIG) != 0, lb = (b.id.x & RID_LIG) != 0;
  if (!la && !lb) return true;
  float ax[3], ay[3], az[3];
  bool ok;
  lig_subs(la ? a : b, ax, ay, az, ok);
  bool may = !ok;
  if (la && lb) {
    float bx[3], by[3], bz[3];
    bool okb;
    lig_subs(b, bx, by, bz, okb);
    may |= !okb;
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const float dx = ax[j] - bx[k], dy = ay[j] - by[k], dz = az[j] - bz[k];
        may |= dx * dx + dy * dy + dz * dz < P.ref_bb;
      }
    return may;
  }
  const Rec& R = la ? b : a;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const float dx = ax[j] - R.pos.x, dy = ay[j] - R.pos.y;
    const float dz = fmaxf(fmaxf(R.pos.z - az[j], az[j] - R.pos.w), 0.0f);
    may |= dx * dx + dy * dy + dz * dz < P.ref_ab;
  }
  return may;
}

// one candidate (proposal record A, record B)
__device__ __forceinline__ void col_exact_one(const KParams& P, const Dev& d, const Rec& A, const Rec& B, uint32_t tag) {
  const int2 a = A.id, b = B.id;
  int m = a.x & RID_PID, u = a.y, q = b.x & RID_PID, kq = b.y;
  bool isnew = b.x < 0;
  bool hit;
  if (P.col_refine && !col_refine(P, A, B)) {
    hit = false;
  } else if (COL_AA_FAST && m < P.NA && q < P.NA) {
    // receptor against receptor: domain [1][1] against domain [1][1] only
    // (exact_collide's first case), two rows of each instead of load_own's six
    const Beads& Q = isnew ? d.nxt : d.cur;
    const double2 mxy = d.nxt.Axy(m, 1, 1), mz = d.nxt.A2(m, 16), qxy = Q.Axy(q, 1, 1), qz = Q.A2(q, 16);
    const double dx = qxy.x - mxy.x, dy = qxy.y - mxy.y, dz = qz.x - mz.x;
    hit = d2(dx, dy, dz) < P.T_aa;
  } else {
    Own o;
    load_own(P, d.nxt, m, o);
    hit = exact_collide(P, o, isnew ? d.nxt : d.cur, q);
  }
  if (P.dbg_cand) {
    const int kk = (m >= P.NA ? 1 : 0) + (q >= P.NA ? 1 : 0);
    atomicAdd(&d.ctl->cand_kind[2 * kk], 1u);
    if (hit) atomicAdd(&d.ctl->cand_kind[2 * kk + 1], 1u);
  }
  if (!hit) return;
  if (bad_key(d, u) || bad_key(d, kq)) return;
  if (P.dd && d.dd_own[u] != d.dd_own[kq]) atomicAdd(&d.ctl->dd_xcol, 1u);  // an owned unit against a halo unit
  if (kq >= u) {
    mark_rej(d, u, tag);
    return;
  }
  uint32_t old = atomicMax(&d.ustate[u], tag | S_PEND);
  if ((old & ~3u) != tag) {
    sl_push(d.plist, make_int2(u, 0), &d.ctl->err);  // at most one entry per unit (the step's work counts)
  } else if ((old & 3u) == S_REJ) {
    return;
  }
  // each stored entry counted once, taken back by round 0 (k_col_resolve):
  // the count returns to 0 within the step, an overflowed list included
  if (sl_push(d.conf, make_int2(u, kq | (isnew ? (int)0x80000000 : 0)), &d.ctl->err)) atomicAdd(&d.ccnt[u], 1ull);
}

// Records of a dense block's staging sequence (the home records of its home
// region, then its outlier bucket, or the whole outlier list when the bucket
// overflowed: obkt < 0) from global memory: f(record index) for elements
// start, start + stride, ...  A home record coded RID_OUT is skipped (it is an
// outlier).
template <class F>
__device__ __forceinline__ void dense_records(const KParams& P, const Dev& d, const TileGeo& G, int obkt, int nout,
                                              int start, int stride, F f) {
  const int xlo = max(G.hx0, 0), xhi = min(G.hx0 + G.mw - 1, P.ncx - 1);
  int q = 0;  // running element index
  for (int seg = 0; seg < G.nhseg; ++seg) {
    const int y = G.hy0 + (seg >> 1);
    if (y < 0 || y >= P.ncy || xlo > xhi) continue;
    const int lo = d.hstart[cell_index(P, xlo, y, seg & 1)], hi = d.hstart[cell_index(P, xhi + 1, y, seg & 1)];
    const int n = 2 * (hi - lo);
    for (int k = ((start - q) % stride + stride) % stride; k < n; k += stride) {
      const int ri = 2 * lo + k;
      if (rec_code(d.rec[ri].id) != RID_OUT) f(ri);
    }
    q += n;
  }
  if (obkt >= 0) {
    for (int k = ((start - q) % stride + stride) % stride; k < nout; k += stride)
      f(d.tout[(size_t)obkt * TOUT_CAP + k].x);
    return;
  }
  const int no = (int)min(d.ctl->n_outl, d.outl_cap);
  for (int k = ((start - q) % stride + stride) % stride; k < no; k += stride) f(d.outl[k].x);
}

// the exact cell of record ri (from its beads: R for the old position, R_new
// for the proposal)
__device__ __forceinline__ void rec_cell_exact(const KParams& P, const Dev& d, int ri, int& cx, int& cy) {
  const int2 id = d.rec[ri].id;
  const int p = id.x & RID_PID;
  const Beads& B = id.x < 0 ? d.nxt : d.cur;
  cx = cell_x(P, B.P(p, 1, 1, 0));
  cy = cell_y(P, B.P(p, 1, 1, 1));
}

// Brute force over a dense block (k_pair_scan could not stage it): every
// record of the block against every record of the 3x3 cells around it —
// collision candidates tested here at once, reaction candidates emitted.
#ifdef DENSE_NOINLINE  // (A/B builds)
__device__ __noinline__
#else
__device__ __forceinline__
#endif
void dense_block(const KParams& P, const Dev& d, int4 blk, uint32_t tag) {
  const TileGeo G = tile_geo(blk.x & 0xffff, blk.x >> 16, blk.y & 0xffff, blk.y >> 16);
  const int obkt = blk.z, nout = blk.w;
  dense_records(P, d, G, obkt, nout, threadIdx.x, blockDim.x, [&](int ri) {
    int x, y;
    rec_cell_exact(P, d, ri, x, y);
    if (x < G.x0 || x >= G.x0 + G.w || y < G.y0 || y >= G.y0 + G.h) return;
    const Rec mr = d.rec[ri];
    const int2 me = mr.id;
    bool prop = me.x < 0;
    if (prop && me.y < 0) {
      atomicOr(&d.ctl->err, ERR_RESOLVE);
      prop = false;
    }
    const bool rx = rxn_item(me);
    if (!prop && !rx) return;
    dense_records(P, d, G, obkt, nout, 0, 1, [&](int rn) {
      int ox, oy;
      rec_cell_exact(P, d, rn, ox, oy);
      if (abs(ox - x) > 1 || abs(oy - y) > 1) return;
      const Rec o = d.rec[rn];
      if (prop && col_pair(me, mr.pos, o.id, o.pos)) {
        if (o.id.y < 0) atomicOr(&d.ctl->err, ERR_RESOLVE);
        else col_exact_one(P, d, mr, o, tag);
      }
      if (rx && rxn_pair(me, mr.pos, mr.site, o.id, o.pos, o.site)) sl_push(d.pairs, make_int2(ri, rn), &d.ctl->err);
    });
  });
}

// The dense tiles: in k_col_exact's first workgroups (DENSE_KERNEL 0), or in
// a kernel of their own.  The own kernel kept k_col_exact at 58 VGPRs against
// the brute force's 107 (round 2); since the record refinement k_col_exact
// holds ~100 anyway, and the separate launch (4.8 µs, empty at the benchmark
// densities) is the larger cost: C3 34.1 -> 30.1 µs for the pair, C5 equal
// (profiles/r05/tail/r6a_*).
#ifndef DENSE_KERNEL
#define DENSE_KERNEL 0
#endif
__global__ void k_col_dense(KParams P, Dev d) {
  const uint32_t tag = (d.ctl->step & 0x3fffffffu) << 2;
  const uint32_t nd = min(d.ctl->n_dense, d.dense_cap);
  for (uint32_t b = blockIdx.x; b < nd; b += gridDim.x) dense_block(P, d, d.dense[b], tag);
}

#ifndef COLX_WAVES  // minimum waves per SIMD of k_col_exact (4: the 128-VGPR cap an unbounded kernel gets)
#define COLX_WAVES 4
#endif
__global__ void __launch_bounds__(256, COLX_WAVES) k_col_exact(KParams P, Dev d) {
  const uint32_t tag = (d.ctl->step & 0x3fffffffu) << 2;
  __shared__ uint32_t pre[NSHARD + 1];
#if !DENSE_KERNEL
  const uint32_t nd = min(d.ctl->n_dense, d.dense_cap);
  for (uint32_t b = blockIdx.x; b < nd; b += gridDim.x) dense_block(P, d, d.dense[b], tag);
#endif
  const uint32_t n = sl_prefix(d.cand, pre);
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gridDim.x * blockDim.x) {
    const int2 c = sl_at(d.cand, pre, t);
    // the ids first; the rest of the two records (same lines) only for a
    // pair with a ligand, which col_refine reads
    Rec A, B;
    A.id = d.rec[c.x].id;
    B.id = d.rec[c.y].id;
    if ((A.id.x | B.id.x) & RID_LIG) {
      A.pos = d.rec[c.x].pos;
      A.site = d.rec[c.x].site;
      B.pos = d.rec[c.y].pos;
      B.site = d.rec[c.y].site;
    }
    col_exact_one(P, d, A, B, tag);
  }
}

// ---------------------------------------------------------------- 4c. rounds
// Pass C: Gauss–Seidel resolution on the conflict entries.  Entry (u, kq,
// new): once kq is decided, the collision counts iff kq accepted and the
// record is its proposal, or kq was rejected and the record is its old
// position.  A unit is accepted when none of its entries counts or waits.
// Only sound deductions are made, in any order, so the outcome is the
// sequential one; the lowest pending key can always decide, so it ends.
__device__ __forceinline__ uint32_t round_tag(uint32_t step, int round) { return step * 64u + (uint32_t)round; }

// returns true while the entry can still matter: u and kq both pending
__device__ __forceinline__ bool conf_entry(const Dev& d, int2 e, uint32_t step, uint32_t rt) {
  int u = e.x, kq = e.y & 0x7fffffff;
  bool isnew = e.y < 0;
  if (state_of(d, u, step) != S_PEND) return false;
  uint32_t sk = state_of(d, kq, step);
  if (sk == S_PEND) {
    st_state(&d.pend[u], rt);
    return true;
  }
  if ((sk == S_ACC) == isnew) mark_rej(d, u, (step & 0x3fffffffu) << 2);
  return false;
}

// returns 1 if u is still pending after this round
__device__ __forceinline__ int conf_unit(const Dev& d, int u, uint32_t step, uint32_t rt) {
  if (state_of(d, u, step) != S_PEND) return 0;
  if (ld_state(&d.pend[u]) == rt) return 1;
  set_state(d, u, step, S_ACC);
  return 0;
}

// Round 0 over every conflict entry, and of every unit as soon as its last
// entry is evaluated: no grid-wide barrier between the entries and their
// units.  ccnt[u] packs the round in one word that each entry changes with a
// single atomic (so no fence orders an entry's effect before its count): the
// entries not yet evaluated (bits 0-31, counted by k_col_exact), the entries
// left waiting on a pending kq (32-47), the entries that rejected u (48-63).
// The entry that takes the count to 0 decides u and clears the word.  A unit
// decided here may decide a later entry of this round (every deduction is
// sound in any order, so the outcome is still the sequential one).  An entry
// whose kq is still pending is the only kind a later round can change, so
// those, and the units still pending, are compacted for k_col_tail.  The
// counters n_pend / n_pqu / n_pqe were zeroed by the previous step's
// finalisation.
#define CC_WAIT (1ull << 32)
#define CC_REJ (1ull << 48)
__global__ void k_col_resolve(KParams P, Dev d) {
  const uint32_t step = d.ctl->step;
  const uint32_t rt = round_tag(step, 0);
  __shared__ uint32_t pre[NSHARD + 1];
  const uint32_t n = sl_prefix(d.conf, pre);
  int pend = 0;
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gridDim.x * blockDim.x) {
    const int2 e = sl_at(d.conf, pre, t);
    const int u = e.x, kq = e.y & 0x7fffffff;
    unsigned long long inc = 0;
    if (state_of(d, u, step) == S_PEND) {
      const uint32_t sk = state_of(d, kq, step);
      if (sk == S_PEND) {
        inc = CC_WAIT;
        d.pq_ent[wave_slot(&d.ctl->n_pqe)] = e;
      } else if ((sk == S_ACC) == (e.y < 0)) {
        inc = CC_REJ;
        mark_rej(d, u, (step & 0x3fffffffu) << 2);
      }
    }
    const unsigned long long old = atomicAdd(&d.ccnt[u], inc - 1ull);
    if ((uint32_t)old != 1u) continue;
    // u's last entry: every other entry of u has made its change of the word
    const unsigned long long now = old + inc - 1ull;
    d.ccnt[u] = 0ull;
    if ((now >> 48) == 0 && state_of(d, u, step) == S_PEND) {
      if (now >> 32) {  // still pending: the tail's unit list, stamped for its round 1
        ++pend;
        d.pq_units[wave_slot(&d.ctl->n_pqu)] = u;
      } else {
        set_state(d, u, step, S_ACC);
      }
    }
  }
  if (pend) atomicAdd(&d.ctl->n_pend, (uint32_t)pend);
}

// single workgroup: the remaining rounds on the compacted pending entries and
// units (k_col_resolve), until nothing is pending
__global__ void __launch_bounds__(1024) k_col_tail(KParams P, Dev d, int round0) {
  __shared__ uint32_t npend;
  if (d.ctl->n_pend == 0) return;
  const uint32_t step = d.ctl->step;
  const uint32_t n = d.ctl->n_pqe, nu = d.ctl->n_pqu;
  for (int round = round0;; ++round) {
    const uint32_t rt = round_tag(step, round);
    if (threadIdx.x == 0) npend = 0;
    for (uint32_t t = threadIdx.x; t < n; t += blockDim.x) conf_entry(d, d.pq_ent[t], step, rt);
    __syncthreads();
    int pend = 0;
    for (uint32_t t = threadIdx.x; t < nu; t += blockDim.x) pend += conf_unit(d, d.pq_units[t], step, rt);
    if (pend) atomicAdd(&npend, (uint32_t)pend);
    __syncthreads();
    if (npend == 0) break;
    if ((uint32_t)(round - round0) > nu + 2) {
      if (threadIdx.x == 0) atomicOr(&d.ctl->err, ERR_RESOLVE);
      break;
    }
    __syncthreads();
  }
}

// ================================================================ 5. commit
// The members of every rejected unit: their final position is the old one,
// R is copied to R_new (main.cpp:666-674, 851-863, 1831-1860).
// bead row `row` of member m: R_new = R
__device__ __forceinline__ void rej_copy(const KParams& P, const Dev& d, int m, int row) {
  const bool a = m < P.NA;
  const int n = a ? P.NA : P.NB, i = a ? m : m - P.NA;
  if (row >= (a ? ROWS_A : ROWS_B)) return;
  const double2* src = reinterpret_cast<const double2*>(a ? d.cur.a : d.cur.b);
  double2* dst = reinterpret_cast<double2*>(a ? d.nxt.a : d.nxt.b);
  const size_t e = bead_elem(i, row, n, a ? ROWS_A : ROWS_B);
  dst[e] = src[e];
}

// One group of REJ_LANES lanes per rejected unit (two units per wave); its
// lanes take the (member, bead row) copies of all members at once, so a
// complex costs the same few dependent loads as a single protein, and a wave
// carries four units' dependent chains at once (most rejected units are
// single proteins of 12 or 24 rows).
#ifndef REJ_LANES  // (A/B, profiles/r04/ab_r4x: 16 -> 32 lanes, k_rej_commit 21.2 -> 18.4 us at C3)
#define REJ_LANES 32
#endif
#if defined(REJ_SIDE) && REJ_SIDE
// (measured round 4 and removed: the revert beside k_rxn_exact .. k_finalize races with the association snaps
// of k_match, which move receptors in R_new that a revert must restore first — DESIGN.md §8)
#error "REJ_SIDE is wrong by design"
#endif
#ifndef REJ_ROWMAJOR  // the (member, row) copies of a unit's lanes ordered row-major
#define REJ_ROWMAJOR 1
#endif
#ifndef REJ_UNROLL  // rejected units whose lookups a lane group has in flight at once
#define REJ_UNROLL 1
#endif
// (workgroup blk of nblk taking part)
__device__ __forceinline__ void rej_commit(const KParams& P, const Dev& d, uint32_t blk, uint32_t nblk) {
  const int NA = P.NA;
  __shared__ uint32_t pre[NSHARD + 1];
  const uint32_t n = sl_prefix(d.rej, pre);
  const int lane = threadIdx.x % REJ_LANES;
  const uint32_t w0 = (blk * blockDim.x + threadIdx.x) / REJ_LANES, nw = (nblk * blockDim.x) / REJ_LANES;
  constexpr int U = REJ_UNROLL;
  // REJ_UNROLL units per pass: each step of their lookup chains (unit ->
  // slot -> kind -> members) issued for all of them before the next, so a
  // group waits for one chain per pass, not one per unit
  for (uint32_t t0 = w0; t0 < n; t0 += nw * U) {
    int sl[U], off[U], nm[U], q[U];
    uint8_t kind[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t t = t0 + (uint32_t)u * nw;
      sl[u] = t < n ? sl_at(d.rej, pre, t).x : -1;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (sl[u] >= 0) sl[u] = d.slot_of[sl[u]];
#pragma unroll
    for (int u = 0; u < U; ++u) kind[u] = sl[u] >= 0 ? d.ukind[sl[u]] : (uint8_t)U_NONE;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      off[u] = 0;
      nm[u] = sl[u] >= 0 ? 1 : 0;
      q[u] = -1;
      if (kind[u] == U_COMPLEX) {
        off[u] = d.cx_off[sl[u] - NA];
        nm[u] = d.cx_size[sl[u] - NA];
      } else if (kind[u] == U_DIMER) {
        nm[u] = 2;
        q[u] = A_NEI3(d, sl[u]) - 1;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      auto member = [&](int k) { return kind[u] == U_COMPLEX ? d.members[off[u] + k] : (k ? q[u] : sl[u]); };
#if REJ_ROWMAJOR
      // row-major over the members: neighbouring lanes copy one row of
      // neighbouring members, which the grouped slot order puts in consecutive
      // slots — the same cache line of the row's 64-slot block
      for (int e = lane; e < nm[u] * ROWS_A; e += REJ_LANES) rej_copy(P, d, member(e % nm[u]), e / nm[u]);
#else
      for (int e = lane; e < nm[u] * ROWS_A; e += REJ_LANES) rej_copy(P, d, member(e / ROWS_A), e % ROWS_A);
#endif
    }
  }
}

// ================================================================ 6. reactions
// Reaction candidates (main.cpp:1877-2058): a receptor that can still react
// (not both bonds taken) is paired with the receptors (cis) and ligands (R–L)
// near it.  The reference pairs FINAL positions, which are known only after
// the collision resolution; the pair scan below runs before it and pairs
// every record of such a receptor (old and proposed) with every record near
// it, with conservative single-precision prefilters (R–L: ligand centre within
// reach of the [3][2] site; cis: the two [3][3] sites within 16 Å).  Exactly
// one of a protein's two records is final — the proposal if its unit was
// accepted, the old position if it was rejected (rec_final) — so of the up to
// four record combinations of a protein pair at most one is final-final:
// k_rxn_exact keeps that one — the same pairs as a scan of the final records.
// the record holds its protein's final position: the proposal of an accepted
// unit or the old position of a rejected one (owner key = the unit)
__device__ __forceinline__ bool rec_final(const Dev& d, int2 id, uint32_t step) {
  return (state_of(d, id.y, step) == S_REJ) == (id.x >= 0);
}
__device__ __forceinline__ void rxn_emit(const Dev& d, WgList& L, int a, int b) {
  wg_emit(L, make_int2(a, b), d.pairs, &d.ctl->err);
}

// ---------------------------------------------------------------- pair scan
// One staging of each tile for both pair searches of the step: collision
// candidates of the proposal records (pass A, §4a) and reaction candidates of
// the records of receptors that can react (above).  An item's stencil is cut
// to the larger of its two reaches per neighbour kind; each pair is tested
// against both filters.
// Stage block G and walk its pairs (false: more than tcap records, nothing
// emitted; the block then goes onto the dense list, k_col_exact).
__device__ __forceinline__ bool pair_scan_block(const KParams& P, const Dev& d, const TileGeo& G, TileLds& T,
                                                float2* site, WgList& Lc, WgList& Lr, Stamper& S) {
  const int NB = P.NB;
  const bool staged = tile_load(P, d, G, T, site, S);
  wg_list_init(Lc);  // (the lists share LDS with the home headers: after the staging)
  wg_list_init(Lr);
  if (!staged) return false;
  if (P.dbg_stage == 1) return true;
  PairBuf Bc, Br;
  Bc.n = 0;
  Br.n = 0;
  bool bad = false;  // a collision candidate whose record has no owner key
  auto rng = [&](int l, int seg, int hx, int* r0, int* r1) {
    const int2 me = T.id[l];
    bool prop = me.x < 0;  // proposal record: collision candidates
    if (prop && me.y < 0) {
      atomicOr(&d.ctl->err, ERR_RESOLVE);
      prop = false;
    }
    const bool rx = rxn_item(me);
    if (!prop && !rx) return false;
    const bool mA = !(me.x & RID_LIG);
    const float4 mp = T.pos[l];
    // kind 0: the collision reach around the record, and for the cis
    // search a square around its [3][3] site (any cis partner has its
    // site within 16 Å of this one, its record within 20.3 Å of its site)
    const float rc0 = prop ? (mA ? REACH_AA : REACH_AB) : 0.0f;
    float x0lo = mp.x - rc0, x0hi = mp.x + rc0, y0lo = mp.y - rc0, y0hi = mp.y + rc0;
    const bool cis = rx && !(me.x & RID_ST3);
    if (cis) {
#if CIS_SITE
      const float2 ms = site[l];
      const float sxl = ms.x - REACH_CSITE, sxh = ms.x + REACH_CSITE, syl = ms.y - REACH_CSITE,
                  syh = ms.y + REACH_CSITE;
#else
      const float sxl = mp.x - REACH_CIS, sxh = mp.x + REACH_CIS, syl = mp.y - REACH_CIS,
                  syh = mp.y + REACH_CIS;
#endif
      x0lo = rc0 > 0.0f ? fminf(x0lo, sxl) : sxl;
      x0hi = rc0 > 0.0f ? fmaxf(x0hi, sxh) : sxh;
      y0lo = rc0 > 0.0f ? fminf(y0lo, syl) : syl;
      y0hi = rc0 > 0.0f ? fmaxf(y0hi, syh) : syh;
    }
    float reach1 = prop ? (mA ? REACH_AB : REACH_BB) : 0.0f;
    if (rx && !(me.x & RID_ST2) && NB > 0) reach1 = fmaxf(reach1, REACH_RL);
    item_ranges(P, T, G, seg, hx, x0lo, x0hi, y0lo, y0hi, 0, r0, r1);
    item_ranges(P, T, G, seg, hx, mp.x - reach1, mp.x + reach1, mp.y - reach1, mp.y + reach1, 1, r0 + 3,
                r1 + 3);
    if (rc0 == 0.0f && !cis)
      for (int k = 0; k < 3; ++k) r1[k] = r0[k];
    if (reach1 == 0.0f)
      for (int k = 3; k < 6; ++k) r1[k] = r0[k];
    return true;
  };
  // one pair: pushed to the registers' buffers, then to the workgroup's lists
  auto push = [&](bool colp, bool rxp, int il, int nl, int2 id) {
    // (branches: most chunks have no passing pair, and the wave skips the
    // pushes; measured faster than selects on every pair)
    if (colp) {
      if (id.y < 0) bad = true;
      else if (Bc.n < 4) pair_push(Bc, make_int2(il, nl));
      else col_emit(d, Lc, tile_global(T, il), tile_global(T, nl));
    }
    if (rxp) {
      if (Br.n < 4) pair_push(Br, make_int2(il, nl));
      else rxn_emit(d, Lr, tile_global(T, il), tile_global(T, nl));
    }
  };
  tile_walk(
      G, T, T.u.l.wbits, rng,
      [&](int il, int nl) {
        const int2 me = T.id[il], id = T.id[nl];
        const float4 mp = T.pos[il], rp = T.pos[nl];
#if PAIR_PK
        // col_pair and rxn_pair (below), one packed xy difference for both
        const pk2 dd = (pk2){rp.x, rp.y} - (pk2){mp.x, mp.y};
        const pk2 d2v = dd * dd;
        const float dxy2 = d2v.x + d2v.y;
        const int m = me.x & RID_PID, u = me.y, q = id.x & RID_PID, kq = id.y;
        const bool isnew = id.x < 0, mA = !(me.x & RID_LIG), qB = (id.x & RID_LIG) != 0;
        const bool own_ok = kq == u ? isnew : (kq > u ? !isnew : true);
        const bool colp = (me.x < 0) & (u >= 0) & (q != m) & own_ok & prefilter_d(mA, mp.z, mp.w, !qB, rp, dxy2);
        const float2 ms = site[il], qs = site[nl];
        const pk2 tt = (pk2){qs.x, qs.y} - (pk2){ms.x, ms.y};
        const pk2 t2v = tt * tt;
        const bool rl_ok = qB & !(me.x & RID_ST2) & (dxy2 < 105.0f * 105.0f) & (rp.z > mp.z - 85.0f) &
                           (rp.z < mp.w + 85.0f);
        const float gap = fmaxf(fmaxf(rp.z - mp.w, mp.z - rp.w), 0.0f);
        const bool cis_ok = !qB & !(me.x & RID_ST3) & !(id.x & RID_ST3) & (dxy2 < 57.0f * 57.0f) & (gap < 16.0f) &
                            (t2v.x + t2v.y < 16.0f * 16.0f);
        const bool rxp = rxn_item(me) & (q != m) & (rl_ok | cis_ok);
#else
        const bool colp = me.x < 0 && me.y >= 0 && col_pair(me, mp, id, rp);
        const bool rxp = rxn_item(me) && rxn_pair(me, mp, site[il], id, rp, site[nl]);
#endif
        push(colp, rxp, il, nl, id);
      });
  if (bad) atomicOr(&d.ctl->err, ERR_RESOLVE);
  S(d, 5);
  auto glb = [&](int2 v) { return make_int2(tile_global(T, v.x), tile_global(T, v.y)); };
  pair_flush(Bc, Lc, d.cand, &d.ctl->err, glb);
  pair_flush(Br, Lr, d.pairs, &d.ctl->err, glb);
  S(d, 6);
  return true;
}

// One workgroup per tile.  A tile whose records overflow TCAP (never at the
// benchmark densities with the host's tile choice) goes onto the dense list,
// which k_col_exact scans by brute force from global memory: this kernel
// stays free of that path's registers and call frame (measured: a fallback
// inside costs it a third of its speed, through the lost occupancy or the
// scratch frame).
#ifndef PAIR_XCD  // tiles dealt to the XCDs in contiguous runs (A/B, profiles/r04/ab_r4w: the
#define PAIR_XCD 1   // scan's HBM fetch 79 -> 37 MB per launch at C3, its time +1 us)
#endif
#ifndef PAIR_WAVES  // minimum waves per SIMD of the pair scan (A/B builds: tools/build_variants.py)
#define PAIR_WAVES 5
#endif
__global__ void __launch_bounds__(PAIR_THREADS, PAIR_WAVES) k_pair_scan(KParams P, Dev d) {
  __shared__ TileLds T;
  __shared__ float2 site[TCAP];
  WgList& Lc = T.u.l.Lc;
  WgList& Lr = T.u.l.Lr;
  const int ntx = (P.ncx + P.tile - 1) / P.tile;
#if PAIR_XCD
  // XCD-aware tile order: consecutive workgroups go to the 8 XCDs in turn, so
  // workgroup b takes tile k = b / 8 of XCD b % 8's contiguous run of tiles —
  // neighbouring tiles, which stage each other's halo records, share an L2
  const int nt = (int)gridDim.x, q8 = nt / 8, r8 = nt % 8, xcd = (int)blockIdx.x % 8;
  const int tile = xcd * q8 + min(xcd, r8) + (int)blockIdx.x / 8;
#else
  const int tile = (int)blockIdx.x;
#endif
  const int tx = tile % ntx, ty = tile / ntx;
  const int x0 = tx * P.tile, y0 = ty * P.tile, w = min(P.tile, P.ncx - x0), h = min(P.tile, P.ncy - y0);
  if (threadIdx.x == 0) {  // this tile's outlier bucket (read before tile_load's first barrier), then reset
    const uint32_t no = d.tout_n[tile];
    T.nout = no;
    T.obkt = no <= (uint32_t)P.tout_cap ? tile : -1;
    if (no) d.tout_n[tile] = 0;
  }
  Stamper S(0);
  if (!pair_scan_block(P, d, tile_geo(x0, y0, w, h), T, site, Lc, Lr, S) && threadIdx.x == 0) {
    const uint32_t o = atomicAdd(&d.ctl->n_dense, 1u);  // k_col_exact takes it
    if (o < d.dense_cap) d.dense[o] = make_int4(x0 | y0 << 16, w | h << 16, T.obkt, (int)T.nout);
    else atomicOr(&d.ctl->err, ERR_EDGES);
  }
  if (P.dbg_stage == 1 || P.dbg_stage == 3) return;
  wg_flush2(Lc, d.cand, Lr, d.pairs, &d.ctl->err);
  S(d, 7);
}

// Reaction candidates, pass 2: exact R–L association gates (main.cpp:1880-1921)
// and cis gates (1954-1985 / 2009-2039) on each pair; a pair becomes an
// accepting edge when its keyed draw is below the acceptance probability.
// The greedy kernels below replay the reference's loop order on the edges.
// (workgroup blk of nblk taking part)
// Refinement of an R–L reaction pair from the two records (float,
// conservative, before any fp64 gather): bit k − 2 set if the ligand's site
// [k][2] (k = 2..4) may lie within bond_cut of the receptor's site [3][2]
// (main.cpp:1880-1884).  The ligand's sites are (1 + √3/2) times its subunit
// offsets from the centre (main.cpp:392-410), which the record carries to
// 0.87 Å (lig_pack): ≤ 1.62 Å off.  The receptor's [3][2] = 2·[3][1] − [3][3]
// (main.cpp:303-311): its xy from the axis (record x, y; [3][1] within 0.3 Å
// of it) and the [3][3] site xy in the record, ≤ 0.6 Å off; its z within RA
// (+ 0.3) of the domains' z span.  Margin 3 Å (P.ref_rl); sites_ok checks the
// templates' geometry when a state is set.  At C5, 95 % of the final-final R–L
// pairs fail the first gate (profiles/r05/c5_window_r5o_debug_counters.log).
__device__ __forceinline__ uint32_t rxn_refine(const KParams& P, const Rec& R, const Rec& L) {
  const uint32_t w0 = __float_as_uint(L.pos.w), w1 = __float_as_uint(L.site.x), w2 = __float_as_uint(L.site.y);
  if ((w2 >> 8) & 1u) return 7u;  // an offset out of the byte range: no refinement
  const uint32_t b[9] = {w0, w0 >> 8, w0 >> 16, w0 >> 24, w1, w1 >> 8, w1 >> 16, w1 >> 24, w2};
  const float f = 1.8660254f;
  const float sx = 2.0f * R.pos.x - R.site.x, sy = 2.0f * R.pos.y - R.site.y;
  const float zlo = R.pos.z - ((float)P.ra + 0.3f), zhi = R.pos.w + ((float)P.ra + 0.3f);
  uint32_t m = 0;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const float dx = L.pos.x + f * (float)(int8_t)(b[3 * j] & 0xff) - sx;
    const float dy = L.pos.y + f * (float)(int8_t)(b[3 * j + 1] & 0xff) - sy;
    const float z = L.pos.z + f * (float)(int8_t)(b[3 * j + 2] & 0xff);
    const float dz = fmaxf(fmaxf(z - zhi, zlo - z), 0.0f);
    m |= (dx * dx + dy * dy + dz * dz < P.ref_rl ? 1u : 0u) << j;
  }
  return m;
}

__device__ __forceinline__ void rxn_exact(const KParams& P, const Dev& d, uint32_t blk, uint32_t nblk) {
  const int NA = P.NA, NB = P.NB;
  const uint32_t step = d.ctl->step;
  __shared__ uint32_t pre[NSHARD + 1];
  const uint32_t n = sl_prefix(d.pairs, pre);
  for (uint32_t t = blk * blockDim.x + threadIdx.x; t < n; t += nblk * blockDim.x) {
    const int2 pr = sl_at(d.pairs, pre, t);
    const int2 ra = d.rec[pr.x].id, rb = d.rec[pr.y].id;
    if (P.dbg_cand) atomicAdd(&d.ctl->rxn_kind[0], 1u);
    if (!rec_final(d, ra, step) || !rec_final(d, rb, step)) continue;  // not both final positions (see the pair scan)
    if (P.dbg_cand) atomicAdd(&d.ctl->rxn_kind[1], 1u);
    const int i = ra.x & RID_PID, q = rb.x & RID_PID;
    // final positions: the proposal (R_new) of an accepted unit, R of a
    // rejected one — read where they are (the revert has run, but reading R
    // for a rejected unit is the same value)
    const Beads& NI = ra.x < 0 ? d.nxt : d.cur;
    const Beads& NQ = rb.x < 0 ? d.nxt : d.cur;
    if (q >= NA) {
      int lb = q - NA;
      const uint32_t may = P.rxn_refine ? rxn_refine(P, d.rec[pr.x], d.rec[pr.y]) : 7u;
      if (P.dbg_cand && may != 7u) atomicAdd(&d.ctl->rxn_kind[4], 3u - (uint32_t)__popc(may));
      for (int k = 2; k <= 4; ++k) {
        if (!((may >> (k - 2)) & 1u)) continue;
        if (B_ST(d, lb, k) != 0) continue;
        double ddx = NQ.B(lb, k, 2, 0) - NI.A(i, 3, 2, 0), ddy = NQ.B(lb, k, 2, 1) - NI.A(i, 3, 2, 1),
               ddz = NQ.B(lb, k, 2, 2) - NI.A(i, 3, 2, 2);
        if (!(d2(ddx, ddy, ddz) < P.T_bond)) continue;
        if (P.dbg_cand) atomicAdd(&d.ctl->rxn_kind[2], 1u);
        double ot = gettheta(NI.A(i, 3, 1, 0) - NI.A(i, 3, 2, 0), NI.A(i, 3, 1, 1) - NI.A(i, 3, 2, 1),
                             NI.A(i, 3, 1, 2) - NI.A(i, 3, 2, 2), NQ.B(lb, k, 1, 0) - NQ.B(lb, k, 2, 0),
                             NQ.B(lb, k, 1, 1) - NQ.B(lb, k, 2, 1), NQ.B(lb, k, 1, 2) - NQ.B(lb, k, 2, 2));
        double pd = gettheta(NI.A(i, 3, 1, 0) - NI.A(i, 3, 4, 0), NI.A(i, 3, 1, 1) - NI.A(i, 3, 4, 1),
                             NI.A(i, 3, 1, 2) - NI.A(i, 3, 4, 2), NQ.B(lb, 1, 1, 0) - NQ.B(lb, 1, 2, 0),
                             NQ.B(lb, 1, 1, 1) - NQ.B(lb, 1, 2, 1), NQ.B(lb, 1, 1, 2) - NQ.B(lb, 1, 2, 2));
        if (!((kmcm::fabs_(pd) < P.thetapd_cut) && (kmcm::fabs_(ot - 180) < P.thetaot_cut))) continue;
        const uint64_t ri = (uint64_t)d.id_of[i], rq = (uint64_t)d.id_of[q];
        double u = kmcr::uniform(P.key, kmcr::DOM_RL, rkey(P, d, (int)ri), rkey(P, d, (int)rq), step, (uint32_t)k);
        if (!(u < P.p_ass)) continue;
        if (P.dbg_cand) atomicAdd(&d.ctl->rxn_kind[3], 1u);
        uint32_t pos = atomicAdd(&d.ctl->n_rl, 1u);
        if (pos < d.cap_edges)
          d.rl_keys[pos] = (ri << 34) | (rq << 2) | (uint64_t)(k - 2);
        else
          atomicOr(&d.ctl->err, ERR_EDGES);
      }
    } else {
      double ddx = NQ.A(q, 3, 3, 0) - NI.A(i, 3, 3, 0), ddy = NQ.A(q, 3, 3, 1) - NI.A(i, 3, 3, 1),
             ddz = NQ.A(q, 3, 3, 2) - NI.A(i, 3, 3, 2);
      if (!(d2(ddx, ddy, ddz) < P.T_cis)) continue;
      if (P.dbg_cand) atomicAdd(&d.ctl->rxn_kind[2], 1u);
      double ot = gettheta(NI.A(i, 3, 1, 0) - NI.A(i, 3, 3, 0), NI.A(i, 3, 1, 1) - NI.A(i, 3, 3, 1),
                           NI.A(i, 3, 1, 2) - NI.A(i, 3, 3, 2), NQ.A(q, 3, 1, 0) - NQ.A(q, 3, 3, 0),
                           NQ.A(q, 3, 1, 1) - NQ.A(q, 3, 3, 1), NQ.A(q, 3, 1, 2) - NQ.A(q, 3, 3, 2));
      if (!(kmcm::fabs_(ot - 180) < P.cis_theta_cut)) continue;
      const uint64_t ri = (uint64_t)d.id_of[i], rq = (uint64_t)d.id_of[q];
      const uint32_t gi = rkey(P, d, (int)ri), gq = rkey(P, d, (int)rq);
      double um = kmcr::uniform(P.key, kmcr::DOM_MONO, gi, gq, step, 0);
      double uc = kmcr::uniform(P.key, kmcr::DOM_CIS, gi, gq, step, 0);
      uint64_t fl = (um < P.p_mono ? 1u : 0u) | (uc < P.p_cis ? 2u : 0u);
      if (!fl) continue;
      if (P.dbg_cand) atomicAdd(&d.ctl->rxn_kind[3], 1u);
      uint32_t pos = atomicAdd(&d.ctl->n_cisc, 1u);
      if (pos < d.cap_edges)
        d.cis_keys[pos] = (ri << 34) | (rq << 2) | fl;
      else
        atomicOr(&d.ctl->err, ERR_EDGES);
    }
  }
}


// The revert of the rejected units (workgroups [0, nrej)) beside the exact
// reaction tests (the rest) in one launch: the tests read each record's final
// position where it is (R of a rejected unit, which the revert copies into
// R_new), so neither half waits for the other; both are done before k_match
// snaps associated receptors in R_new.
#ifndef COMMIT_MIX  // (A/B builds: 0 = the revert's workgroups first)
#define COMMIT_MIX 1
#endif
__global__ void k_commit_rxn(KParams P, Dev d, int nrej) {
  const uint32_t b = blockIdx.x, nr = (uint32_t)nrej, nx = gridDim.x - nr;
#if COMMIT_MIX
  // the two halves' workgroups alternate while both have some left, so both
  // are resident from the start (the dispatcher goes in workgroup order)
  const uint32_t m = min(nr, nx);
  if (b < 2 * m) {
    if (b & 1) rxn_exact(P, d, b >> 1, nx);
    else rej_commit(P, d, b >> 1, nr);
  } else if (nr > nx) {
    rej_commit(P, d, b - m, nr);
  } else {
    rxn_exact(P, d, b - m, nx);
  }
#else
  if (b < nr) rej_commit(P, d, b, nr);
  else rxn_exact(P, d, b - nr, nx);
#endif
}

// ---------------------------------------------------------------- greedy
// In-place bitonic sort of keys[0..np) (np a power of two) by one workgroup.
__device__ void block_sort(uint64_t* keys, uint32_t np) {
  for (uint32_t k = 2; k <= np; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t i = threadIdx.x; i < np; i += blockDim.x) {
        uint32_t l = i ^ j;
        if (l > i) {
          uint64_t a = keys[i], b = keys[l];
          bool up = (i & k) == 0;
          if ((a > b) == up) {
            keys[i] = b;
            keys[l] = a;
          }
        }
      }
      __syncthreads();
    }
  }
}

__device__ __forceinline__ uint32_t pow2ceil(uint32_t n) {
  uint32_t p = 1;
  while (p < n) p <<= 1;
  return p;
}

// Lexicographic-first greedy matching: edges (sorted keys[0..n)) are taken in
// order; an edge is accepted iff no earlier edge sharing one of its two
// vertices was accepted — the outcome of the reference's nested loops with
// in-place status updates.  Parallel form: per-vertex chains in edge order;
// an edge decides once both chain predecessors have decided.
// vtx(e, w) gives the two vertex ids of edge e.  acc[e] receives the result.
template <typename VF>
__device__ void block_greedy(uint32_t n, const uint64_t* keys, VF vtx, uint64_t* ent, int32_t* g, uint8_t* acc,
                             uint32_t* err) {
  // g layout: pos[2n] | pred[2n] | dec[n]   (ent: 2n vertex entries)
  int32_t* pos = g;
  int32_t* pred = g + 2 * n;
  int32_t* dec = g + 4 * n;
  uint8_t* chain = acc + n;  // 2n flags after acc[n]
  uint32_t np = pow2ceil(2 * n);
  for (uint32_t e = threadIdx.x; e < np; e += blockDim.x) {
    if (e < 2 * n) ent[e] = ((uint64_t)vtx(keys[e >> 1], e & 1) << 32) | e;  // entry = (vertex, 2e+w)
    else ent[e] = ~0ull;
  }
  __syncthreads();
  block_sort(ent, np);
  for (uint32_t x = threadIdx.x; x < 2 * n; x += blockDim.x) {
    uint32_t ew = (uint32_t)ent[x];
    pos[ew] = (int32_t)x;
    pred[x] = (x > 0 && (ent[x - 1] >> 32) == (ent[x] >> 32)) ? (int32_t)(x - 1) : -1;
  }
  for (uint32_t e = threadIdx.x; e < n; e += blockDim.x) dec[e] = 0;
  __syncthreads();
  __shared__ int any_left;
  for (int round = 1;; ++round) {
    if (threadIdx.x == 0) any_left = 0;
    __syncthreads();
    for (uint32_t e = threadIdx.x; e < n; e += blockDim.x) {
      if (dec[e]) continue;
      bool ready = true, blocked = false;
      int px[2];
      for (int w = 0; w < 2; ++w) {
        px[w] = pred[pos[2 * e + w]];
        if (px[w] >= 0) {
          uint32_t pe = ((uint32_t)ent[px[w]]) >> 1;
          int dr = dec[pe];
          if (dr == 0 || dr == round) ready = false;
          else blocked |= chain[px[w]] != 0;
        }
      }
      if (!ready) {
        any_left = 1;
        continue;
      }
      uint8_t a = blocked ? 0 : 1;
      acc[e] = a;
      for (int w = 0; w < 2; ++w) chain[pos[2 * e + w]] = (uint8_t)(a | (px[w] >= 0 ? chain[px[w]] : 0));
      dec[e] = round;
    }
    __syncthreads();
    if (!any_left) break;
    if (round > (int)n + 2) {
      if (threadIdx.x == 0) atomicOr(err, ERR_EDGES);
      break;
    }
    __syncthreads();
  }
  __syncthreads();
}

struct RLV {
  int N;
  __device__ uint32_t operator()(uint64_t key, int w) const {
    if (w == 0) return (uint32_t)(key >> 34);  // receptor
    uint32_t q = (uint32_t)((key >> 2) & 0xffffffffu), k = (uint32_t)(key & 3u);
    return (uint32_t)N + (q - (uint32_t)0) * 4u + k;  // ligand site (distinct id space)
  }
};
struct CisV {
  __device__ uint32_t operator()(uint64_t key, int w) const {
    return w == 0 ? (uint32_t)(key >> 34) : (uint32_t)((key >> 2) & 0xffffffffu);
  }
};

// Few edges (the common case: tens per step at the benchmark sizes): wave 0
// sorts the keys in registers (bitonic network over the 64 lanes, written back
// in order to keys[0..n)); lane l then holds sorted edge l's two vertices, and
// the wave takes the edges in that order — the definition of the
// lexicographic-first matching — each decided by one ballot against the
// edges accepted before it, instead of the sort and dependency rounds of
// block_greedy, whose barriers dominate at this size.
#define SMALL_EDGES 64
// Wave 0 returns its lane's sorted key and acceptance (the callers apply the
// accepted edges from registers, without reading acc / keys back).
template <typename VF>
__device__ bool small_greedy(uint32_t n, uint64_t* keys, VF vtx, uint8_t* acc, uint64_t* key_out) {
  bool mine = false;
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    uint64_t k = lane < (int)n ? keys[lane] : ~0ull;
#pragma unroll
    for (int size = 2; size <= 64; size <<= 1)
#pragma unroll
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        const uint64_t o = (uint64_t)__shfl_xor((long long)k, stride, 64);
        const bool asc = (lane & size) == 0, low = (lane & stride) == 0;
        k = (low == asc) ? (k < o ? k : o) : (k < o ? o : k);
      }
    const bool real = lane < (int)n;
    if (real) keys[lane] = k;
    const uint32_t va = real ? vtx(k, 0) : 0xffffffffu, vb = real ? vtx(k, 1) : 0xffffffffu;
    uint64_t accm = 0;  // accepted edges so far (bits < e)
    for (uint32_t e = 0; e < n; ++e) {
      const uint32_t a = (uint32_t)__shfl((int)va, (int)e, 64), b = (uint32_t)__shfl((int)vb, (int)e, 64);
      const bool shares = (va == a) | (va == b) | (vb == a) | (vb == b);
      if ((__ballot(shares) & accm) == 0) accm |= 1ull << e;
    }
    mine = real && ((accm >> lane) & 1ull);
    if (real) acc[lane] = (uint8_t)mine;
    *key_out = k;
  }
  __syncthreads();
  return mine;
}

// R–L association, main.cpp:1877-1949
__device__ void rl_match(const KParams& P, const Dev& d) {
  const int NA = P.NA, NB = P.NB;
  uint32_t n = d.ctl->n_rl;
  if (n == 0) return;
  if (n > d.cap_edges) n = d.cap_edges;
  uint8_t* acc = (uint8_t*)(d.gi32 + 5 * d.cap_edges);
  auto apply = [&](uint64_t key) {
    int i = d.slot_of[(int)(key >> 34)], q = d.slot_of[(int)((key >> 2) & 0xffffffffu)], k = (int)(key & 3) + 2;
    int lb = q - NA;
    if (P.dd) dd_xbond(d, (int)(key >> 34), (int)((key >> 2) & 0xffffffffu));
    A_ST2(d, i) = 1;
    B_ST(d, lb, k) = 1;
    B_NEI(d, lb, k) = i + 1;
    A_NEI2(d, i) = q + 1;
    A_NEI4(d, i) = k;
    mark_bond_change(P, d, i, d.ctl->step);
    mark_bond_change(P, d, q, d.ctl->step);
  };
  if (n <= SMALL_EDGES) {
    uint64_t key = 0;
    if (small_greedy(n, d.rl_keys, RLV{P.N}, acc, &key)) apply(key);
    return;
  }
  uint32_t np = pow2ceil(n);
  for (uint32_t e = n + threadIdx.x; e < np; e += blockDim.x) d.rl_keys[e] = ~0ull;
  __syncthreads();
  block_sort(d.rl_keys, np);
  block_greedy(n, d.rl_keys, RLV{P.N}, d.ent, d.gi32, acc, &d.ctl->err);
  for (uint32_t e = threadIdx.x; e < n; e += blockDim.x)
    if (acc[e]) apply(d.rl_keys[e]);
}

// cis association: mono (main.cpp:1952-2003) then complex (2007-2058)
__device__ void cis_match(const KParams& P, const Dev& d) {
  const int NA = P.NA;
  uint32_t n0 = d.ctl->n_cisc;
  if (n0 == 0) return;
  if (n0 > d.cap_edges) n0 = d.cap_edges;
  uint64_t* keys = d.cis_keys;
  uint8_t* acc = (uint8_t*)(d.gi32 + 5 * d.cap_edges);
  __shared__ uint32_t m;
  for (int pass = 0; pass < 2; ++pass) {
    // edges of this pass go to the back half of rl_keys as scratch
    uint64_t* e = d.rl_keys;
    if (threadIdx.x == 0) m = 0;
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < n0; t += blockDim.x) {
      uint64_t key = keys[t];
      int i = d.slot_of[(int)(key >> 34)], q = d.slot_of[(int)((key >> 2) & 0xffffffffu)];
      uint32_t fl = (uint32_t)(key & 3);
      bool unb = A_ST2(d, i) == 0 && A_ST2(d, q) == 0;
      bool ok = pass == 0 ? (unb && (fl & 1)) : (!unb && (fl & 2) && A_ST3(d, i) == 0 && A_ST3(d, q) == 0);
      if (ok) e[atomicAdd(&m, 1u)] = key & ~3ull;
    }
    __syncthreads();
    uint32_t n = m;
    auto apply = [&](uint64_t key) {
      int i = d.slot_of[(int)(key >> 34)], q = d.slot_of[(int)((key >> 2) & 0xffffffffu)];
      if (P.dd) dd_xbond(d, (int)(key >> 34), (int)((key >> 2) & 0xffffffffu));
      A_ST3(d, i) = 1;
      A_ST3(d, q) = 1;
      A_NEI3(d, q) = i + 1;
      A_NEI3(d, i) = q + 1;
      mark_bond_change(P, d, i, d.ctl->step);
      mark_bond_change(P, d, q, d.ctl->step);
    };
    if (n > 0 && n <= SMALL_EDGES) {
      uint64_t key = 0;
      if (small_greedy(n, e, CisV{}, acc, &key)) apply(key);
    } else if (n > 0) {
      uint32_t np = pow2ceil(n);
      for (uint32_t t = n + threadIdx.x; t < np; t += blockDim.x) e[t] = ~0ull;
      __syncthreads();
      block_sort(e, np);
      block_greedy(n, e, CisV{}, d.ent, d.gi32, acc, &d.ctl->err);
      for (uint32_t t = threadIdx.x; t < n; t += blockDim.x)
        if (acc[t]) apply(e[t]);
    }
    __syncthreads();
  }
}

// cis dissociation, mono (main.cpp:2097-2117) and complex (2120-2141): both
// members of a pair draw in index order, so a pair breaks iff either draw
// succeeds; handled by the lower index
__device__ __forceinline__ bool cis_diss(const KParams& P, const Dev& d, int i, int q, bool mono, uint32_t step) {
  const int NA = P.NA;
  uint32_t dom = mono ? kmcr::DOM_MD : kmcr::DOM_CD;
  double pd = mono ? P.p_mdiss : P.p_cdiss;
  double ui = kmcr::uniform(P.key, dom, rkey(P, d, d.id_of[i]), 0, step, 0);
  double uq = kmcr::uniform(P.key, dom, rkey(P, d, d.id_of[q]), 0, step, 0);
  if (ui < pd || uq < pd) {
    A_ST3(d, i) = 0;
    A_ST3(d, q) = 0;
    A_NEI3(d, i) = 0;
    A_NEI3(d, q) = 0;
    mark_bond_change(P, d, i, step);
    mark_bond_change(P, d, q, step);
    return true;
  }
  return false;
}

// both association passes in one workgroup (the cis pass reads the R–L outcome)
__global__ void __launch_bounds__(1024) k_match(KParams P, Dev d) {
  rl_match(P, d);
  __syncthreads();
  cis_match(P, d);
}

// R–L dissociation draw of receptor i (bonded), main.cpp:2063-2092
__device__ __forceinline__ bool rl_breaks(const KParams& P, const Dev& d, int i, uint32_t step) {
  return kmcr::uniform(P.key, kmcr::DOM_RLD, rkey(P, d, d.id_of[i]), 0, step, 0) < P.p_diss;
}

// ================================================================ 7. observables
__device__ __forceinline__ int wave_sum(int v) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  return v;
}
__device__ __forceinline__ int wave_max(int v) {
  for (int off = 32; off > 0; off >>= 1) {
    int o = __shfl_down(v, off, 64);
    v = o > v ? o : v;
  }
  return v;
}

// Dissociations and observables, one thread per protein.  Receptor i: R–L
// dissociation (one bond per receptor: independent), then cis dissociation of
// its pair by the lower slot with the R–L outcome (st2 only goes 1 -> 0 and
// its final value is a function of the receptor's own draw, so the partner's
// value read before or after its own update gives the same answer); it then
// counts its final bonds.  Ligand: cluster statistics of this step's BFS.
// DISS_PER proteins per thread (their first loads issued together): 4 for the
// large systems (C5: 101 -> 61 us), 1 below 4M proteins, where fewer
// workgroups than the CUs' slots would cost more than the overlap gains (C3:
// 22 -> 25 us with 4)
template <int DISS_PER>
__global__ void __launch_bounds__(256) k_diss_observe(KParams P, Dev d) {
  const int NA = P.NA, NB = P.NB;
  __shared__ int red[4][6];
  const uint32_t step = d.ctl->step;
  int v[6] = {0, 0, 0, 0, 0, 0};  // rl mono cis tot_prot tot_clu max
  // DISS_PER proteins per thread, blockDim apart (each load coalesced): the
  // status words / unit kinds of all of them in flight before the first branch
  const int p0 = blockIdx.x * blockDim.x * DISS_PER + threadIdx.x;
  int st2[DISS_PER], st3[DISS_PER];
  uint8_t kind[DISS_PER];
#pragma unroll
  for (int k = 0; k < DISS_PER; ++k) {
    const int p = p0 + k * (int)blockDim.x;
    st2[k] = 0;
    st3[k] = 0;
    kind[k] = U_NONE;
    if (p < NA) {
      st2[k] = A_ST2(d, p);
      st3[k] = A_ST3(d, p);
    } else if (p < P.N) {
      kind[k] = d.ukind[p];
    }
  }
#pragma unroll
  for (int k = 0; k < DISS_PER; ++k) {
    const int p = p0 + k * (int)blockDim.x;
    if (p < NA) {
      const int i = p;
      int st2_i = st2[k];
      if (st2_i == 1 && rl_breaks(P, d, i, step)) {
        int q = A_NEI2(d, i) - 1, kk = A_NEI4(d, i);
        int lb = q - NA;
        A_ST2(d, i) = 0;
        B_ST(d, lb, kk) = 0;
        A_NEI2(d, i) = 0;
        A_NEI4(d, i) = 0;
        B_NEI(d, lb, kk) = 0;
        mark_bond_change(P, d, i, step);
        mark_bond_change(P, d, q, step);
        st2_i = 0;
      }
      // a decomposed trajectory counts the bonds of the receptors its slab owns,
      // a cis pair at the owner of its lower reference index (dd_owned)
      v[0] += dd_owned(P, d, d.id_of[i]) ? st2_i : 0;
      if (st3[k] == 1) {
        int q = A_NEI3(d, i) - 1;
        if (i < q) {
          int st2_q = A_ST2(d, q);
          if (st2_q == 1 && rl_breaks(P, d, q, step)) st2_q = 0;
          const bool mono = st2_i == 0 && st2_q == 0;
          if (!cis_diss(P, d, i, q, mono, step)) v[mono ? 1 : 2] += dd_owned(P, d, min(d.id_of[i], d.id_of[q])) ? 1 : 0;
        }
      }
    } else if (p < P.N) {
      uint8_t kd = kind[k];
      if (!dd_owned(P, d, d.id_of[p])) kd = U_NONE;  // a unit (root ligand) of another slab
      if (kd == U_COMPLEX) {
        int sz = d.cx_size[p - NA];
        v[3] += sz;
        v[4] += 1;
        v[5] = max(v[5], sz);
      } else if (kd == U_FREE_B) {
        v[5] = max(v[5], 1);
      }
    }
  }
  for (int f = 0; f < 5; ++f) v[f] = wave_sum(v[f]);
  v[5] = wave_max(v[5]);
  int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0)
    for (int f = 0; f < 6; ++f) red[w][f] = v[f];
  __syncthreads();
  if (threadIdx.x < 6) {  // per-block partials, reduced by k_finalize
    int f = threadIdx.x, a = red[0][f];
    for (int ww = 1; ww < 4; ++ww) a = f == 5 ? max(a, red[ww][f]) : a + red[ww][f];
    d.obs_part[blockIdx.x * 8 + f] = a;
  }
}

// bond.dat record (main.cpp:2195-2202, 2251) and step advance; one
// workgroup of 1024 threads reduces the observable partials of
// k_diss_observe's nblk blocks (39 063 at C5), four partials in flight per
// thread.  The list shard counters are totalled (diagnostics) and zeroed in
// parallel; the control block is read in one batch of loads and written once.
__global__ void __launch_bounds__(1024) k_finalize(KParams P, Dev d, double time_step, int nblk) {
  __shared__ int red[16][6];
  __shared__ uint32_t tot[5];
  if (threadIdx.x < 5) tot[threadIdx.x] = 0;
  int v[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll 4
  for (int b = threadIdx.x; b < nblk; b += blockDim.x) {
    const int4 lo = *(const int4*)&d.obs_part[b * 8];
    const int2 hi = *(const int2*)&d.obs_part[b * 8 + 4];
    v[0] += lo.x;
    v[1] += lo.y;
    v[2] += lo.z;
    v[3] += lo.w;
    v[4] += hi.x;
    v[5] = max(v[5], hi.y);
  }
  for (int f = 0; f < 5; ++f) v[f] = wave_sum(v[f]);
  v[5] = wave_max(v[5]);
  if ((threadIdx.x & 63) == 0)
    for (int f = 0; f < 6; ++f) red[threadIdx.x >> 6][f] = v[f];
  __syncthreads();
  for (int k = threadIdx.x; k < 5 * NSHARD; k += blockDim.x) {  // lists in shard_cnt order: cand conf plist rej pairs
    const int l = k / NSHARD;
    const uint32_t cap = l == 0 ? d.cand.cap : l == 1 ? d.conf.cap : l == 2 ? d.plist.cap : l == 3 ? d.rej.cap : d.pairs.cap;
    atomicAdd(&tot[l], min(d.shard_cnt[k], cap));
    d.shard_cnt[k] = 0;
  }
  // the next step's complexes: dissolve those whose bonds changed, or rebuild
  // every one when the appended rows fill half of members[] or this step's
  // dirty list overflowed (read by every thread before thread 0 writes them)
  const uint32_t fstep = d.ctl->step;
  const uint32_t ff = (d.ctl->cx_cursor > P.cx_limit || d.ctl->n_dirty[fstep & 1] > (uint32_t)P.N) ? 1u : 0u;
  if (P.NB > 0) {
    if (ff) {
      cx_reset_all(P, d, threadIdx.x, blockDim.x);
    } else {
      cx_dissolve_dirty(P, d, fstep);
      if (threadIdx.x == 0) d.ctl->full_now = 0;
    }
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  for (int w = 1; w < (int)(blockDim.x >> 6); ++w)
    for (int f = 0; f < 6; ++f) red[0][f] = f == 5 ? max(red[0][f], red[w][f]) : red[0][f] + red[w][f];
  Ctl* c = d.ctl;
  const uint32_t step = c->step, obs_idx = c->obs_idx, n_rl = c->n_rl, n_cisc = c->n_cisc, n_ovf = c->n_overflow;
  const int32_t off_rl = c->off_rl, off_mono = c->off_mono, off_cis = c->off_cis, off_bond = c->off_bond;
  const int32_t rl = red[0][0], mono = red[0][1], cis = red[0][2], tot_prot = red[0][3], tot_clu = red[0][4];
  const int32_t maxc = max(c->maxc, red[0][5]);
  kmc_obs_dev o;
  o.step = (int64_t)step;
  o.t = (double)(int)step * time_step;
  o.rl = rl + off_rl;
  o.mono = mono + off_mono;
  o.cis = cis + off_cis;
  o.bond = (rl + mono + cis) + off_bond;
  o.cluster_size = tot_clu != 0 ? (double)tot_prot / tot_clu : 0.0;
  o.maxc = maxc;
  o.tot_prot = tot_prot;
  o.tot_clu = tot_clu;
  o.reserved = 0;
  d.obs[obs_idx] = o;
  if (c->err && c->err_step == 0) {  // kmc_step replays up to here
    c->err_step = step;
    c->err_first = c->err;
  }
  c->n_forced += ff;  // (diagnostics: full rebuilds latched here)
  c->maxc = maxc;
  c->obs_idx = obs_idx + 1;
  c->step = step + 1;
  // per-step counters for the next step; the finished step's work counts
  for (int k = 0; k < 5; ++k) c->last[k] = tot[k];
  c->last[5] = n_rl;
  c->last[6] = n_cisc;
  c->last[7] = n_ovf;
  c->last_outl = c->n_outl;
  c->n_overflow = 0;
  c->n_dirty[(step + 1) & 1] = 0;  // consumed above; the next step's reactions fill it
  c->n_heavy = 0;
  c->n_pend = 0;
  c->n_pqu = 0;  // filled by the next step's k_col_resolve
  c->n_pqe = 0;
  c->n_rl = 0;
  c->n_cisc = 0;
  c->n_outl = 0;
  c->n_dense = 0;
}


// ================================================================ slot order
// Proteins live in slots sorted by the tile-major cell of bead [1][1]
// (receptors in [0, NA), ligands in [NA, N)), re-sorted every few hundred
// steps, so that per-protein passes touch spatially coherent cache lines and
// the cell-sorted records are written almost in order.  Nothing of the
// simulation depends on the slot order: random streams, unit keys and the
// reactions' greedy order use reference indices (id_of); bond fields hold
// slot + 1 and are renumbered with the permutation.
// row-major cell order, the order of the home list: the free units' record
// writes (at their home positions) then run along the home list
__device__ __forceinline__ uint32_t slot_key(const KParams& P, double x, double y) {
  return (uint32_t)cell_y(P, y) * (uint32_t)P.ncx + (uint32_t)cell_x(P, x);
}

// Sort key of slot s, packed into the bits the radix sort walks (low to
// high): the unit (ob bits), the cell (kb bits), the complex flag (group 2),
// the kind (receptors before ligands: one sort of all N slots leaves each
// kind in its own range).  With grouping, a protein takes the cell of its
// unit's lead (the last step's owner key: a complex's root ligand, a cis
// dimer's lead receptor, else itself) and the lead's reference index as the
// unit field, so the members of one unit occupy consecutive slots of their
// kind: the complex kernels then touch a few cache lines per bead row instead
// of one per member.
// group 2: members of complexes go after every other protein of their kind,
// so the free units' slots form one dense range: the free proposals then
// write whole cache lines of R_new, and the complexes' rows are contiguous
// runs of their own.
__global__ void k_slot_keys(KParams P, Dev d, uint64_t* keys, int32_t* vals, int group, int ob, int kb) {
  int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= P.N) return;
  int lead = s, own = d.id_of[s];
  if (group) {
    const int o = d.owner[s];
    if (o >= 0 && o < P.N) {
      lead = d.slot_of[o];
      own = o;
    }
  }
  double x = d.cur.P(lead, 1, 1, 0), y = d.cur.P(lead, 1, 1, 1);
  const int tb = group == 2 ? 1 : 0;
  const uint64_t cx = group == 2 && d.croot[s] >= 0 ? 1ull : 0ull;
  const uint64_t kind = s >= P.NA ? 1ull : 0ull;
  keys[s] = kind << (ob + kb + tb) | cx << (ob + kb) | (uint64_t)slot_key(P, x, y) << ob |
            (uint64_t)(group ? (uint32_t)own : 0u);
  vals[s] = s < P.NA ? s : s - P.NA;
}

// ------------------------------------------------------ radix sort and scan
// The re-sort's stable LSD radix sort (8-bit digits, as many passes as the
// packed key has bits) and the exclusive scan of the home list's cell counts.
// A tile of RS_TILE keys per workgroup: its digit histogram (k_rs_hist),
// each digit's row of tile counts scanned (k_rs_rows: the tile's first
// output position within the digit, and the digit's total), then the scatter
// (k_rs_scatter): each wave ranks its 16 chunks of 64 keys in order — the
// lanes with the same digit found by 8 ballots, the running count per digit
// in LDS — the waves' counts are scanned across the workgroup, so equal digits
// keep their input order (the result equals a stable sort of the whole key),
// and the tile, placed in LDS in digit order, is written out run by run.  HBM
// per pass: the keys read twice and the (key, value) pairs written once,
// ≈ 28 B per slot.
#define RS_TILE 4096  // keys per workgroup: 256 threads x 16
#define SCAN_TILE 4096

// lanes of the wave holding the same 8-bit digit as this one (among `live`)
__device__ __forceinline__ uint64_t rs_peers(uint32_t dg, uint64_t live) {
  uint64_t m = live;
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const uint64_t v = __ballot((dg >> b) & 1u);
    m &= (dg >> b) & 1u ? v : ~v;
  }
  return m;
}

__global__ void __launch_bounds__(256) k_rs_hist(const uint64_t* __restrict__ keys, int n, int shift,
                                                 int32_t* __restrict__ cnt, int nblk) {
  __shared__ int h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  const int lane = __lane_id();
  const uint64_t lt = (1ull << lane) - 1ull;
  const size_t base = (size_t)blockIdx.x * RS_TILE;
  for (int j = threadIdx.x; j < RS_TILE; j += 256) {
    const size_t i = base + j;
    const bool ok = i < (size_t)n;
    const uint32_t dg = ok ? (uint32_t)(keys[i] >> shift) & 255u : 0u;
    const uint64_t pe = rs_peers(dg, __ballot(ok));
    // one LDS add per digit present in the wave (its lowest lane)
    if (ok && (pe & lt) == 0) atomicAdd(&h[dg], __popcll(pe));
  }
  __syncthreads();
  cnt[(size_t)threadIdx.x * nblk + blockIdx.x] = h[threadIdx.x];
}

// exclusive scan over a 256-thread workgroup (sh: 4 ints of LDS); total = the sum
__device__ __forceinline__ int block_excl_256(int x, int* sh, int& total) {
  const int lane = __lane_id(), w = threadIdx.x >> 6;
  int inc = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(inc, o, 64);
    if (lane >= o) inc += t;
  }
  if (lane == 63) sh[w] = inc;
  __syncthreads();
  int off = 0;
  total = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = sh[q];
    off += q < w ? c : 0;
    total += c;
  }
  __syncthreads();  // (sh reusable)
  return off + inc - x;
}
// per digit: the exclusive scan of its row of tile counts, and its total
__global__ void __launch_bounds__(256) k_rs_rows(int32_t* __restrict__ cnt, int nblk, int32_t* __restrict__ tot) {
  __shared__ int sh[4];
  int32_t* row = cnt + (size_t)blockIdx.x * nblk;
  int carry = 0;
  for (int b0 = 0; b0 < nblk; b0 += 256) {
    const int i = b0 + (int)threadIdx.x;
    const int x = i < nblk ? row[i] : 0;
    int t;
    const int e = block_excl_256(x, sh, t);
    if (i < nblk) row[i] = carry + e;
    carry += t;
  }
  if (threadIdx.x == 0) tot[blockIdx.x] = carry;
}

// The tile's keys ranked (stable) and placed in LDS in digit order, then
// written out run by run: consecutive threads store consecutive positions of
// a digit's output range.
__global__ void __launch_bounds__(256) k_rs_scatter(const uint64_t* __restrict__ kin, const int32_t* __restrict__ vin,
                                                    uint64_t* __restrict__ kout, int32_t* __restrict__ vout, int n,
                                                    int shift, const int32_t* __restrict__ cnt,
                                                    const int32_t* __restrict__ tot, int nblk) {
  __shared__ int wc[4][256];
  __shared__ int gb[256], ts[256], sh[4];
  __shared__ uint64_t sk[RS_TILE];
  __shared__ int32_t sv[RS_TILE];
  const int lane = __lane_id(), w = threadIdx.x >> 6, t = threadIdx.x;
  for (int i = t; i < 4 * 256; i += 256) (&wc[0][0])[i] = 0;
  {
    int all;
    const int db = block_excl_256(tot[t], sh, all);  // the digit's first output position
    gb[t] = db + cnt[(size_t)t * nblk + blockIdx.x];
  }
  __syncthreads();
  const size_t base = (size_t)blockIdx.x * RS_TILE + (size_t)w * (RS_TILE / 4);
  const uint64_t lt = (1ull << lane) - 1ull;
  constexpr int C = RS_TILE / 256;
  uint64_t k[C];
  int32_t v[C], r[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const size_t i = base + (size_t)c * 64 + lane;
    k[c] = i < (size_t)n ? kin[i] : 0ull;
    v[c] = i < (size_t)n ? vin[i] : 0;
  }
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const bool ok = base + (size_t)c * 64 + lane < (size_t)n;
    const uint32_t dg = (uint32_t)(k[c] >> shift) & 255u;
    const uint64_t pe = rs_peers(dg, __ballot(ok));
    // (a wave's LDS operations complete in order: this chunk's read sees the
    // previous chunk's update)
    const int prior = ok ? wc[w][dg] : 0;
    r[c] = prior + __popcll(pe & lt);
    if (ok && (pe & ~lt & ~(1ull << lane)) == 0) wc[w][dg] = prior + __popcll(pe);  // the group's last lane
  }
  __syncthreads();
  {  // the waves' counts of digit t -> offsets across the waves; the tile's digit starts
    int run = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = wc[q][t];
      wc[q][t] = run;
      run += c;
    }
    int all;
    ts[t] = block_excl_256(run, sh, all);
  }
  __syncthreads();
#pragma unroll
  for (int c = 0; c < C; ++c) {
    if (base + (size_t)c * 64 + lane >= (size_t)n) continue;
    const uint32_t dg = (uint32_t)(k[c] >> shift) & 255u;
    const int lp = ts[dg] + wc[w][dg] + r[c];
    sk[lp] = k[c];
    sv[lp] = v[c];
  }
  __syncthreads();
  const int m = (int)min((size_t)RS_TILE, (size_t)n - (size_t)blockIdx.x * RS_TILE);
  for (int j = t; j < m; j += 256) {
    const uint64_t key = sk[j];
    const uint32_t dg = (uint32_t)(key >> shift) & 255u;
    const int pos = gb[dg] + j - ts[dg];
    kout[pos] = key;
    vout[pos] = sv[j];
  }
}

// exclusive scan, three launches: tile sums, their scan, the tiles' scans
__global__ void __launch_bounds__(256) k_scan_part(const int32_t* __restrict__ in, int n, int32_t* __restrict__ part) {
  __shared__ int sh[4];
  const size_t base = (size_t)blockIdx.x * SCAN_TILE + (size_t)threadIdx.x * (SCAN_TILE / 256);
  int x = 0;
#pragma unroll
  for (int j = 0; j < SCAN_TILE / 256; ++j)
    if (base + j < (size_t)n) x += in[base + j];
  int tot;
  (void)block_excl_256(x, sh, tot);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}
__global__ void __launch_bounds__(256) k_scan_top(int32_t* part, int nb) {
  __shared__ int sh[4];
  int carry = 0;
  for (int b0 = 0; b0 < nb; b0 += 256) {
    const int i = b0 + (int)threadIdx.x;
    const int x = i < nb ? part[i] : 0;
    int tot;
    const int e = block_excl_256(x, sh, tot);
    if (i < nb) part[i] = carry + e;
    carry += tot;
  }
}
__global__ void __launch_bounds__(256) k_scan_down(const int32_t* in, int32_t* out, int n,
                                                   const int32_t* __restrict__ part) {
  __shared__ int sh[4];
  constexpr int J = SCAN_TILE / 256;
  const size_t base = (size_t)blockIdx.x * SCAN_TILE + (size_t)threadIdx.x * J;
  int x[J], s = 0;
#pragma unroll
  for (int j = 0; j < J; ++j) {
    x[j] = base + j < (size_t)n ? in[base + j] : 0;
    s += x[j];
  }
  int tot;
  int run = part[blockIdx.x] + block_excl_256(s, sh, tot);
#pragma unroll
  for (int j = 0; j < J; ++j) {
    if (base + j < (size_t)n) out[base + j] = run;
    run += x[j];
  }
}

// ---------------------------------------------------------------- home list
// Rebuilt with the slot order (and after a state is set or a chunk undone):
// the home cell of slot p is the (row, kind, column) cell of its reference
// point [1][1] in R; home positions are handed out cell by cell (counting
// sort: count with ranks, scan = hstart, place).
__global__ void k_home_count(KParams P, Dev d, int32_t* hcnt) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P.N) return;
  const double2 xy = p < P.NA ? d.cur.Axy(p, 1, 1) : d.cur.Bxy(p - P.NA, 1, 1);
  const int cx = cell_x(P, xy.x), cy = cell_y(P, xy.y);
  const int r = atomicAdd(&hcnt[cell_index(P, cx, cy, p >= P.NA)], 1);
  d.home[p] = make_uint2((uint32_t)r, (uint32_t)cx | (uint32_t)cy << 16);
}
__global__ void k_home_place(KParams P, Dev d) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P.N) return;
  const uint2 h = d.home[p];
  const int cx = (int)(h.y & 0xffffu), cy = (int)(h.y >> 16);
  d.home[p].x = (uint32_t)d.hstart[cell_index(P, cx, cy, p >= P.NA)] + h.x;
}

// perm[s'] = old slot of new slot s' (sorted values, per kind); inverse map
__global__ void k_slot_inverse(KParams P, const int32_t* sorted, int32_t* perm, int32_t* newslot) {
  int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= P.N) return;
  int old = s < P.NA ? sorted[s] : P.NA + sorted[s];
  perm[s] = old;
  newslot[old] = s;
}

// Bead arrays of one kind gathered through perm (offset: the kind's first
// slot).  mode 0: device layout (kmc_device.h §layout) in and out, one double2
// row element per thread; 1: device layout in, host layout out (the
// reference-order SoA [bead·3 + c][n] of kmc_state_view); 2: host in, device out.
__global__ void k_gather_beads(const double* in, double* out, const int32_t* perm, int off, int n, int ligand,
                               int mode) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (mode == 0) {
    if (t >= (size_t)n * (ligand ? ROWS_B : ROWS_A)) return;
    const int r = (int)(t / n), s = (int)(t % n), rows = ligand ? ROWS_B : ROWS_A;
    reinterpret_cast<double2*>(out)[bead_elem(s, r, n, rows)] =
        reinterpret_cast<const double2*>(in)[bead_elem(perm[off + s] - off, r, n, rows)];
    return;
  }
  if (t >= (size_t)n * (ligand ? 24 : 48)) return;
  const int q = (int)(t / n), s = (int)(t % n), src = perm[off + s] - off;
  const int bead = q / 3, c = q % 3, nk = ligand ? 2 : 4, j = bead / nk + 1, k = bead % nk + 1;
  if (mode == 1)
    out[(size_t)q * n + s] = in[ligand ? bead_off_b(src, j, k, c, n) : bead_off_a(src, j, k, c, n)];
  else
    out[ligand ? bead_off_b(s, j, k, c, n) : bead_off_a(s, j, k, c, n)] = in[(size_t)q * n + src];
}

// bond/state rows; rows flagged in link_mask hold protein index + 1 (0 = none)
// and are renumbered through map
__global__ void k_gather_i32(const int32_t* in, int32_t* out, const int32_t* perm, int off, int n, int rows,
                             uint32_t link_mask, const int32_t* map) {
  size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (size_t)n * rows) return;
  int r = (int)(t / n), s = (int)(t % n);
  int v = in[(size_t)r * n + (perm[off + s] - off)];
  if ((link_mask >> r & 1) && v > 0) v = map[v - 1] + 1;
  out[(size_t)r * n + s] = v;
}

__global__ void k_gather_ids(KParams P, const int32_t* id_in, int32_t* id_out, int32_t* slot_of,
                             const int32_t* perm) {
  int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= P.N) return;
  int id = id_in[perm[s]];
  id_out[s] = id;
  slot_of[id] = s;
}

}  // namespace kmcd
