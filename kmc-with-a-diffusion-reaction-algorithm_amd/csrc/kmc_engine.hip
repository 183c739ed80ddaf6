// kmc_engine.hip — C-ABI of libkmc (include/kmc.h): device memory, the
// per-step launch sequence, state transfer.  One handle per GPU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/kmc.h"
#include "kmc_host.h"
#include "kmc_kernels.hip"

using namespace kmcd;

// kernel ids for per-kernel HIP-event timing (kmc_set_timing / kmc_kernel_times)
enum KId {
  KI_CLASSIFY, KI_BFS, KI_PROPOSE, KI_PROPOSE_FREE, KI_MOVE_MEMBERS, KI_CX_CHECK, KI_CX_HEAVY, KI_CX_KILL,
  KI_PAIR_SCAN, KI_COL_EXACT, KI_COL_ROUNDS, KI_COMMIT, KI_MATCH, KI_DISS_OBSERVE,
  KI_RESORT, KI_N
};
static const char* const KNAMES[KI_N] = {
    "k_classify", "k_bfs", "k_propose", "k_propose_free", "k_move_members", "k_cx_check", "k_complex_heavy",
    "k_cx_kill",
    "k_pair_scan", "k_col_exact", "k_col_rounds", "k_commit_rxn",
    "k_match", "k_diss_observe", "slot_resort"};
#define TRING 64  // steps of event pairs kept in flight
#ifndef CX_STREAM_N  // proteins from which the complex chain runs on its own stream (kmc_create)
#define CX_STREAM_N (4 << 20)
#endif

struct kmc_sim {
  kmc_params p;
  KParams K;
  Dev d;
  int device = 0;
  hipStream_t stream = nullptr;
  int64_t step_done = 0;
  std::string err;
  int ncell = 0;
  int ntiles = 0;  // pair-scan tiles (K.tile × K.tile cells each)
  bool have_state = false;
  std::vector<void*> allocs;
  kmc_obs_dev* obs_buf = nullptr;
  int64_t obs_cap = 0;
  Ctl* ctl_host = nullptr;
  bool poison = false;
  // output-list capacities: 2^grow times the initial sizes; kmc_step doubles
  // them and replays the chunk when a list overflows (ERR_EDGES)
  int grow = 0;
  // snapshot for the replay: R, state rows, slot maps, control block.  Taken
  // lazily: a kmc_step chunk reuses the last snapshot while it is at most
  // snap_span steps behind the chunk's end (keyed draws: replaying the steps
  // since the snapshot reproduces them), so short kmc_step calls do not each
  // copy the whole state (KMC_SNAP_SPAN=0: a snapshot per chunk)
  double *snap_a = nullptr, *snap_b = nullptr;
  int32_t *snap_ai = nullptr, *snap_bi = nullptr, *snap_id = nullptr, *snap_slot = nullptr;
  Ctl* snap_ctl = nullptr;
  bool snap_valid = false;
  int64_t snap_step = 0, snap_since = 0, snap_span = 4096;
  int64_t n_replays = 0, n_snapshots = 0;
  // complexes are kept across steps (k_cx_kill); full: register every one anew
  // at the next step (set after a new state, a re-sort is handled per step, an
  // undone chunk); KMC_FULL_BFS=1: every step
  bool need_full = true, always_full = false;
  bool debug_counts = false;  // KMC_DEBUG_COUNTS=1: print the last step's work counts per kmc_step chunk
  bool debug_sync = false;    // KMC_DEBUG_SYNC=1: synchronise after every kernel, name the one that failed
  int64_t launch_base = 0;    // (debug_sync) the step the current launch_step simulates
  // the unit tables (ukind, complex rows) describe the current step: false
  // after a new state and after a chunk undone without a kept step
  bool clusters_valid = false;
  // slot order (kmc_kernels.hip §slot order): scratch of the re-sort
  int64_t resort_every = 100, since_resort = 0;
  int key_bits = 1;
  uint64_t *skeys = nullptr, *skeys2 = nullptr;  // packed slot keys (k_slot_keys), radix sort ping-pong
  int group_sort = 2;  // 1: members of one unit in consecutive slots; 2: and complexes after the free units; 0: cell only
  int32_t *svals = nullptr, *svals2 = nullptr, *perm = nullptr, *newslot = nullptr;
  int32_t *a_tmp = nullptr, *b_tmp = nullptr, *id_tmp = nullptr;
  int32_t* rs_cnt = nullptr;     // [256][tiles] digit counts of the radix sort -> first output positions
  int32_t* rs_tot = nullptr;     // [256] digit totals of a radix pass
  int32_t* scan_part = nullptr;  // tile sums of dev_scan
  int32_t* hcnt = nullptr;   // [ncell+1] home cell counts (home_build)
  // per-kernel timing: a ring of TRING steps of event pairs, read back lazily
  uint64_t tmask = 0;
  int32_t tperiod = 1;    // bracket only every tperiod-th step
  int64_t tcount = 0;     // steps launched since set_timing
  bool tnow = false;      // this step is bracketed
  std::vector<hipEvent_t> tev;  // [TRING][KI_N][2]
  std::vector<uint8_t> tused;   // [TRING][KI_N]
  int tslot = 0;
  double kms[KI_N] = {0};
  int64_t kcount[KI_N] = {0};
  // HIP graphs of one step (KMC_GRAPH=1): a step's launches are fixed by the
  // kernel arguments (KParams, Dev — the R / R_new and counter buffers swap
  // every step) and the host flags; a captured step is replayed whenever the
  // arguments are byte-identical, so the graphs cycle with the buffer parity
  static constexpr int NGRAPH = 4;
  bool use_graphs = false;
  // the complex chain (their rigid-move parameters, k_move_members,
  // k_cx_check, k_complex_heavy) on a second stream beside the free units'
  // proposals (KMC_CX_STREAM; forked after k_bfs, joined before the pair scan)
  int cx_stream = 0;  // 1: the whole chain on the side stream; 2: only k_bfs and the parameters;
                      // 3: k_cx_check and k_complex_heavy beside the free units (after the members)
  hipStream_t side = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  int cx_params_wg = 0;  // mode 3: workgroups of the parameters' launch (KMC_CX_PARAMS_WG; 0: gL)
  struct StepGraph {
    bool valid = false;
    unsigned char key[sizeof(KParams) + sizeof(Dev)];
    hipGraphExec_t exec = nullptr;
  } graphs[NGRAPH];
  int graph_next = 0;
  int64_t graph_launches = 0, graph_captures = 0;
  // one slab's window of a decomposed trajectory (kmc_dd_*): device copies of
  // the local -> global index map, the ownership flags, x at the window's set
  int32_t* dd_gid = nullptr;
  uint8_t* dd_own = nullptr;
  double* dd_x0 = nullptr;
  uint32_t* dd_scratch = nullptr;  // [2]: drift maximum (float bits), differing proteins
  int32_t* dd_ids = nullptr;       // export / import staging: ids, beads, ints, flags
  double* dd_beads = nullptr;
  int32_t* dd_ints = nullptr;
  uint8_t* dd_flags = nullptr;
  int32_t dd_cap = 0;
  // the device-resident exchange (kmc_dd_plan / pack / unpack / finish)
  DDRep* dd_rep = nullptr;          // the step's report, filled by the kernels
  uint8_t* dd_band = nullptr;       // [N] band flags of the plan
  uint8_t* dd_cut = nullptr;        // [N] a link of the protein was cut at the last unpack
  int32_t* dd_send_ids = nullptr;   // [dd_send_cap]
  int32_t* dd_recv_ids = nullptr;   // [dd_recv_cap]
  unsigned char* dd_sendbuf = nullptr;  // [dd_send_cap rows]
  int32_t dd_n_send = 0, dd_n_recv = 0, dd_send_cap = 0, dd_recv_cap = 0;
  bool dd_step_pending = false;     // kmc_dd_step: pack + jumpers after the step's kernels
  unsigned char* dd_step_dst = nullptr;
  double dd_step_S = 0.0;
};

namespace {

int fail(kmc_sim* s, int code, const std::string& m) {
  if (s) s->err = m;
  return code;
}

#define HIPCHK(s, x)                                                                      \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess)                                                                 \
      return fail(s, KMC_ERR_HIP, std::string(#x ": ") + hipGetErrorString(e_));          \
  } while (0)

// Zeroed device buffer.  The zeroing runs on the handle's stream and is
// waited for: a buffer allocated between steps (list growth, the chunk
// snapshot, the decomposition's staging) is written right away by work on
// that non-blocking stream, or by a synchronous copy on the null stream —
// neither is ordered after a null-stream hipMemset, which another thread's
// null-stream work can hold back (measured: G handles in G threads).
template <typename T>
int dalloc(kmc_sim* s, T** p, size_t n) {
  void* v = nullptr;
  size_t bytes = std::max<size_t>(n, 1) * sizeof(T);
  hipError_t e = hipMalloc(&v, bytes);
  if (e != hipSuccess) return fail(s, KMC_ERR_HIP, std::string("hipMalloc: ") + hipGetErrorString(e));
  e = hipMemsetAsync(v, 0, bytes, s->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
  if (e != hipSuccess) return fail(s, KMC_ERR_HIP, std::string("hipMemset: ") + hipGetErrorString(e));
  s->allocs.push_back(v);
  *p = (T*)v;
  return KMC_OK;
}

uint32_t pow2(uint32_t n) {
  uint32_t p = 1;
  while (p < n) p <<= 1;
  return p;
}

template <typename T>
void dfree(kmc_sim* s, T*& p) {
  if (!p) return;
  auto it = std::find(s->allocs.begin(), s->allocs.end(), (void*)p);
  if (it != s->allocs.end()) s->allocs.erase(it);
  (void)hipFree((void*)p);
  p = nullptr;
}

// The sharded output lists and the reaction-edge buffers, sized for 2^grow
// times the defaults (grow < 0 only to test the replay: KMC_DEBUG_CAP_SHIFT).
// Defaults: collision candidates ~1 per proposal at the benchmark densities,
// every pair of records for small dense systems; per-shard capacity is the
// total / NSHARD, but at least 64 Ki entries (a small dense system puts all of
// its entries into the few shards of its few tiles).
int alloc_lists(kmc_sim* s) {
  Dev& d = s->d;
  const uint64_t N = (uint64_t)s->K.N;
  auto scale = [&](uint64_t v) {
    return std::max<uint64_t>(64, s->grow >= 0 ? v << s->grow : v >> -s->grow);
  };
  dfree(s, d.cand.data);
  dfree(s, d.conf.data);
  dfree(s, d.plist.data);
  dfree(s, d.rej.data);
  dfree(s, d.pairs.data);
  dfree(s, d.rl_keys);
  dfree(s, d.cis_keys);
  dfree(s, d.ent);
  dfree(s, d.gi32);
  dfree(s, d.pq_ent);
  dfree(s, d.outl);
  dfree(s, d.dense);
  uint32_t cap = (uint32_t)scale(pow2(std::max<uint32_t>(4096, std::min<uint32_t>(1u << 20, (uint32_t)N / 8 + 1))));
  d.cap_edges = pow2(cap);
  int rc = KMC_OK;
  auto mk = [&](SList& l, uint64_t total, int which) {
    total = scale(total);
    l.cap = (uint32_t)std::max<uint64_t>((total + NSHARD - 1) / NSHARD, std::min<uint64_t>(total, scale(1u << 16)));
    l.cnt = d.shard_cnt + which * NSHARD;
    return dalloc(s, &l.data, (size_t)l.cap * NSHARD);
  };
  const uint64_t cand = std::max<uint64_t>(N, std::min<uint64_t>(4ull * N * N, 1ull << 22));
  rc |= mk(d.cand, cand, 0);
  rc |= mk(d.conf, cand, 1);
  rc |= mk(d.plist, N, 2);
  rc |= mk(d.rej, N, 3);
  rc |= mk(d.pairs, std::max<uint64_t>(N, 1u << 16), 4);
  rc |= dalloc(s, &d.rl_keys, d.cap_edges);
  rc |= dalloc(s, &d.cis_keys, d.cap_edges);
  rc |= dalloc(s, &d.ent, (size_t)2 * d.cap_edges);
  rc |= dalloc(s, &d.gi32, (size_t)6 * d.cap_edges);
  rc |= dalloc(s, &d.pq_ent, (size_t)d.conf.cap * NSHARD);
  // records more than a cell from their home cell: none at the benchmark
  // densities between re-sorts (a protein drifts a few Å per step)
  d.outl_cap = (uint32_t)scale(std::max<uint64_t>(1024, N / 64));
  rc |= dalloc(s, &d.outl, d.outl_cap);
  // pair-scan blocks too dense for LDS (KMC_DEBUG_TCAP; never at the benchmark densities)
  d.dense_cap = (uint32_t)scale(1024);
  rc |= dalloc(s, &d.dense, d.dense_cap);
  return rc;
}

// smallest T with sqrt(T) >= c, so that  sqrt(s) < c  <=>  s < T  (exact)
double sqrt_threshold(double c) {
  double t = c * c;
  while (std::sqrt(t) >= c) t = std::nextafter(t, 0.0);
  while (std::sqrt(t) < c) t = std::nextafter(t, INFINITY);
  return t;
}


}  // namespace

extern "C" {

const char* kmc_last_error(const kmc_sim* s) { return s ? s->err.c_str() : "null handle"; }

// Tile side of the LDS scans for rho proteins per cell: about 200 proposal
// records per 256-thread workgroup, halo records well inside TCAP (a tile
// whose records still overflow goes onto the dense list and is brute-forced
// from global memory: the mean is kept at 0.75 TCAP, > 7 Poisson sigmas below
// TCAP at the benchmark densities).  KMC_TILE overrides (tests, sweeps).
static int choose_tile(double rho) {
  int t = TILE_MAX;
  while (t > 4 && (t * t * rho > 205.0 || (t + 2) * (t + 2) * 2.0 * rho > 0.75 * TCAP)) --t;
  const char* te = getenv("KMC_TILE");
  if (te && *te) t = std::max(2, std::min(TILE_MAX, atoi(te)));
  return t;
}

int kmc_create(const kmc_params* p, int device, kmc_sim** out) {
  if (!p || !out) return KMC_ERR_ARG;
  *out = nullptr;
  if (p->n_a < 0 || p->n_b < 0 || p->n_a + p->n_b <= 0 || (int64_t)p->n_a + p->n_b > (1 << 24))
    return KMC_ERR_ARG;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return KMC_ERR_NODEVICE;
  kmc_sim* s = new kmc_sim();
  s->p = *p;
  if (device >= 0) {
    if (hipSetDevice(device) != hipSuccess) {
      delete s;
      return KMC_ERR_NODEVICE;
    }
    s->device = device;
  } else {
    (void)hipGetDevice(&s->device);
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, s->device) != hipSuccess || std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    delete s;
    return KMC_ERR_NODEVICE;
  }
  if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess) {
    kmc_destroy(s);
    return KMC_ERR_HIP;
  }
  // the neighbour search's cell size and float prefilter radii are derived
  // for the reference's radii and cutoffs (DESIGN.md §cell list); smaller
  // values only shrink every reach
  if (p->ra_radius > 20.0 || p->rb_radius > 30.0 || p->bond_dist_cutoff > 18.0 || p->cis_dist_cutoff > 15.0) {
    kmc_destroy(s);
    return KMC_ERR_ARG;
  }
  KParams& K = s->K;
  const int NA = p->n_a, NB = p->n_b, N = NA + NB;
  K.NA = NA;
  K.NB = NB;
  K.N = N;
  K.cs = 130.0;
  K.gx0 = -p->box_x / 2 - 1000.0;
  K.gy0 = -p->box_y / 2 - 1000.0;
  K.ncx = std::max(1, (int)((p->box_x + 2000.0) / K.cs) + 1);
  K.ncy = std::max(1, (int)((p->box_y + 2000.0) / K.cs) + 1);
  K.box_x = p->box_x;
  K.box_y = p->box_y;
  K.box_z = p->box_z;
  K.pai = p->pai;
  K.ra = p->ra_radius;
  K.rb = p->rb_radius;
  const double ts = p->time_step;
  // expressions as in main.cpp:585, 611, 693, 726, 909, 942, 990, 1089
  K.amp_a = 2 * std::sqrt(p->ra_D * ts / 6);
  K.amp_b = 2 * std::sqrt(p->rb_D * ts / 6);
  K.amp_cis = 2 * std::sqrt(p->cis_D * ts / 6);
  K.amp_bond = 2 * std::sqrt(p->bond_D * ts / 6);
  K.rot_a = std::sqrt(p->ra_rot_D * ts);
  K.rot_b = std::sqrt(p->rb_rot_D * ts);
  K.rot_cis = std::sqrt(p->cis_rot_D * ts);
  K.rot_bond = std::sqrt(p->bond_rot_D * ts);
  K.p_ass = p->ass_rate * ts;
  K.p_mono = p->mono_cis_ass_rate * ts;
  K.p_cis = p->cis_ass_rate * ts;
  K.p_diss = p->diss_rate * ts;
  K.p_mdiss = p->mono_cis_diss_rate * ts;
  K.p_cdiss = p->cis_diss_rate * ts;
  K.bond_cut = p->bond_dist_cutoff;
  K.cis_cut = p->cis_dist_cutoff;
  K.thetapd_cut = p->bond_thetapd_cutoff;
  K.thetaot_cut = p->bond_thetaot_cutoff;
  K.cis_theta_cut = p->cis_thetaot_cutoff;
  K.T_aa = sqrt_threshold(p->ra_radius + p->ra_radius);
  K.T_ab = sqrt_threshold(p->ra_radius + p->rb_radius);
  K.T_bb = sqrt_threshold(p->rb_radius + p->rb_radius);
  K.T_bond = sqrt_threshold(p->bond_dist_cutoff);
  K.T_cis = sqrt_threshold(p->cis_dist_cutoff);
  K.ref_bb = (float)((2 * p->rb_radius + 2.5) * (2 * p->rb_radius + 2.5));
  K.ref_ab = (float)((p->ra_radius + p->rb_radius + 0.3 + 2.5) * (p->ra_radius + p->rb_radius + 0.3 + 2.5));
  K.ref_rl = (float)((p->bond_dist_cutoff + 3.0) * (p->bond_dist_cutoff + 3.0));
  {
    const char* cr = getenv("KMC_COL_REFINE");
    K.col_refine = !(cr && *cr == '0');
  }
  K.key = kmcr::make_key(p->seed, p->replica);

  s->ncell = 2 * K.ncx * K.ncy;  // (row, kind, column) record cells
  Dev& d = s->d;
  d.cur.NA = d.nxt.NA = NA;
  d.cur.NB = d.nxt.NB = NB;
  d.nkeys = (uint32_t)N;
  int rc = KMC_OK;
  rc |= dalloc(s, &d.cur.a, 48 * bead_slots(NA));
  rc |= dalloc(s, &d.nxt.a, 48 * bead_slots(NA));
  rc |= dalloc(s, &d.cur.b, 24 * bead_slots(NB));
  rc |= dalloc(s, &d.nxt.b, 24 * bead_slots(NB));
  rc |= dalloc(s, &d.a_int, (size_t)5 * NA);
  rc |= dalloc(s, &d.b_int, (size_t)8 * NB);
  rc |= dalloc(s, &d.owner, N);
  rc |= dalloc(s, &d.id_of, N);
  rc |= dalloc(s, &d.slot_of, N);
  rc |= dalloc(s, &s->id_tmp, N);
  rc |= dalloc(s, &s->a_tmp, (size_t)5 * NA);
  rc |= dalloc(s, &s->b_tmp, (size_t)8 * NB);
  rc |= dalloc(s, &s->skeys, N);
  rc |= dalloc(s, &s->skeys2, N);
  rc |= dalloc(s, &s->svals, N);
  rc |= dalloc(s, &s->svals2, N);
  rc |= dalloc(s, &s->perm, N);
  rc |= dalloc(s, &s->newslot, N);
  rc |= dalloc(s, &d.ukind, N);
  rc |= dalloc(s, &d.ustate, N);
  rc |= dalloc(s, &d.moved, N);
  rc |= dalloc(s, &d.cx_off, NB);
  rc |= dalloc(s, &d.cx_size, NB);
  rc |= dalloc(s, &d.cx_nb, NB);
  rc |= dalloc(s, &d.cx_ext, NB);
  d.mcap = (uint32_t)(3 * (size_t)N);
  K.cx_limit = d.mcap / 2;
  {
    const char* cl = getenv("KMC_DEBUG_CX_LIMIT");  // debug: rebuild every complex far earlier
    if (cl && *cl) K.cx_limit = (uint32_t)std::max(0, std::min((int)K.cx_limit, atoi(cl)));
  }
  rc |= dalloc(s, &d.members, d.mcap);
  rc |= dalloc(s, &d.shuf, d.mcap);
  rc |= dalloc(s, &d.mrec, d.mcap);
  rc |= dalloc(s, &d.cxp, (size_t)NB * CXP);
  rc |= dalloc(s, &d.shuf_tag, NB);
  rc |= dalloc(s, &d.croot, N);
  rc |= dalloc(s, &d.cx_alive, NB);
  rc |= dalloc(s, &d.bfs_cand, NB);
  rc |= dalloc(s, &d.dlist, 2 * (size_t)N);
  rc |= dalloc(s, &d.pend, N);
  rc |= dalloc(s, &d.ccnt, N);
  rc |= dalloc(s, &d.overflow, NB);
  rc |= dalloc(s, &d.cx_list, (size_t)d.mcap / 2);  // kept across steps: every registration since the last rebuild
  rc |= dalloc(s, &d.cx_heavy, NB);
  rc |= dalloc(s, &s->hcnt, s->ncell + 1);
  {
    const size_t nblk = ((size_t)N + RS_TILE - 1) / RS_TILE;
    rc |= dalloc(s, &s->rs_cnt, 256 * nblk);
    rc |= dalloc(s, &s->rs_tot, 256);
    rc |= dalloc(s, &s->scan_part, ((size_t)s->ncell + 1 + SCAN_TILE - 1) / SCAN_TILE);
  }
  rc |= dalloc(s, &d.hstart, s->ncell + 1);
  rc |= dalloc(s, &d.home, N);
  rc |= dalloc(s, &d.rec, (size_t)2 * N);
  rc |= dalloc(s, &d.shard_cnt, (size_t)5 * NSHARD);
  {
    const char* cs = getenv("KMC_DEBUG_CAP_SHIFT");  // debug: start with lists 2^k times too small
    s->grow = cs && *cs ? -std::max(0, std::min(20, atoi(cs))) : 0;
  }
  rc |= alloc_lists(s);
  rc |= dalloc(s, &d.pq_units, N);
  rc |= dalloc(s, &d.obs_part, (size_t)8 * ((N + 255) / 256));
  rc |= dalloc(s, &d.bfs_queue, N);
  rc |= dalloc(s, &d.vtag, N);
  rc |= dalloc(s, &d.ctl, 1);
  if (rc != KMC_OK) {
    kmc_destroy(s);
    return KMC_ERR_HIP;
  }
  if (hipHostMalloc((void**)&s->ctl_host, sizeof(Ctl)) != hipSuccess) {
    kmc_destroy(s);
    return KMC_ERR_HIP;
  }
  const char* po = getenv("KMC_DEBUG_POISON");
  s->poison = po && *po == '1';
  const char* dc = getenv("KMC_DEBUG_COUNTS");
  s->debug_counts = dc && *dc == '1';
  const char* dsy = getenv("KMC_DEBUG_SYNC");
  s->debug_sync = dsy && *dsy == '1';
  // debug: lower the LDS tile capacity so that tiles take the global path
  const char* tc = getenv("KMC_DEBUG_TCAP");
  K.tcap = TCAP;
  if (tc && *tc) K.tcap = std::max(0, std::min(TCAP, atoi(tc)));
  // debug: smaller per-tile outlier buckets, so that tiles fall back to the whole outlier list
  const char* oc = getenv("KMC_DEBUG_TOUT_CAP");
  K.tout_cap = TOUT_CAP;
  if (oc && *oc) K.tout_cap = std::max(0, std::min(TOUT_CAP, atoi(oc)));
  // tile side of the LDS scans (mean density of the box)
  {
    K.tile = choose_tile((double)N * K.cs * K.cs / std::max(1.0, p->box_x * p->box_y));
    const char* fb = getenv("KMC_FULL_BFS");
    s->always_full = fb && *fb == '1';
    const char* ds = getenv("KMC_DEBUG_SCAN_STAGE");
    K.dbg_stage = ds && *ds ? atoi(ds) : 0;
    const char* cxs = getenv("KMC_CX_SERIAL");
    K.cx_serial = cxs && *cxs == '1';
    const char* gr = getenv("KMC_GRAPH");
    s->use_graphs = gr && *gr == '1';
    // the complexes' checks and heavy path on a second stream beside the free
    // units from CX_STREAM_N proteins (mode 3; C5: 3.90 (none) / 3.85 (the
    // whole chain beside them, mode 1) -> 3.67 ms/step; C3: 0.452 / 0.455 /
    // 0.468, the latency chains slowed by the free units' HBM stream more
    // than they hide: profiles/r06/ab_cx_stream3_*); KMC_CX_STREAM=0..3 forces a mode
    const char* cs = getenv("KMC_CX_STREAM");
    s->cx_stream = (cs && *cs) ? std::max(0, std::min(3, atoi(cs))) : ((int64_t)N >= CX_STREAM_N ? 3 : 0);
    const char* cpw = getenv("KMC_CX_PARAMS_WG");
    s->cx_params_wg = cpw && *cpw ? std::max(0, atoi(cpw)) : 0;
    const char* ht = getenv("KMC_DEBUG_HTAG");  // debug: fewer tagged home entries (the searched lookup)
    K.htag_max = HTAG_MAX;
    if (ht && *ht) K.htag_max = std::max(0, std::min(HTAG_MAX, atoi(ht)));
    const char* dca = getenv("KMC_DEBUG_CAND");
    K.dbg_cand = dca && *dca == '1';
    const char* dr = getenv("KMC_DEBUG_RECS");
    K.dbg_recs = dr && *dr == '1';
    if (K.dbg_recs && dalloc(s, &d.rec_step, 2 * (size_t)N) != KMC_OK) {
      kmc_destroy(s);
      return KMC_ERR_HIP;
    }
    const char* sp = getenv("KMC_SNAP_SPAN");
    if (sp && *sp) s->snap_span = std::max<int64_t>(0, atoll(sp));
  }
  {
    const uint64_t kmax = (uint64_t)K.ncx * K.ncy;  // row-major cell keys (k_slot_keys)
    s->key_bits = 1;
    while ((1ull << s->key_bits) < kmax) ++s->key_bits;
    if (s->key_bits + 33 > 64) {  // the packed slot key: unit (< 2^31), cell, complex flag, kind
      kmc_destroy(s);
      return KMC_ERR_ARG;
    }
    const char* re = getenv("KMC_RESORT");
    if (re && *re) s->resort_every = atoll(re);
    const char* gs = getenv("KMC_GROUP_SORT");
    if (gs && *gs) s->group_sort = std::max(0, std::min(2, atoi(gs)));
    // per-tile outlier buckets of the pair scan (counters zero between steps)
    s->ntiles = ((K.ncx + K.tile - 1) / K.tile) * ((K.ncy + K.tile - 1) / K.tile);
    if (dalloc(s, &s->d.tout, (size_t)s->ntiles * TOUT_CAP) != KMC_OK ||
        dalloc(s, &s->d.tout_n, (size_t)s->ntiles) != KMC_OK) {
      kmc_destroy(s);
      return KMC_ERR_HIP;
    }
  }
  *out = s;
  return KMC_OK;
}

int kmc_destroy(kmc_sim* s) {
  if (!s) return KMC_OK;
  if (s->stream) (void)hipStreamSynchronize(s->stream);
  for (void* v : s->allocs) (void)hipFree(v);
  if (s->obs_buf) (void)hipFree(s->obs_buf);
  if (s->ctl_host) (void)hipHostFree(s->ctl_host);
  for (auto& e : s->tev)
    if (e) (void)hipEventDestroy(e);
  for (auto& g : s->graphs)
    if (g.exec) (void)hipGraphExecDestroy(g.exec);
  if (s->side) (void)hipStreamSynchronize(s->side);
  if (s->ev_fork) (void)hipEventDestroy(s->ev_fork);
  if (s->ev_join) (void)hipEventDestroy(s->ev_join);
  if (s->side) (void)hipStreamDestroy(s->side);
  if (s->stream) (void)hipStreamDestroy(s->stream);
  delete s;
  return KMC_OK;
}

int64_t kmc_current_step(const kmc_sim* s) { return s ? s->step_done : -1; }

// Gather R, the state rows and bond fields through perm (new index -> old
// slot) into R_new / scratch, renumbering bond fields through map, and swap.
// swap_in (re-sort): beads stay in the device layout; otherwise (get_state)
// they come out in the host layout of kmc_state_view.
static void reorder(kmc_sim* s, const int32_t* perm, const int32_t* map, bool swap_in) {
  const KParams& K = s->K;
  Dev& d = s->d;
  hipStream_t st = s->stream;
  const int NA = K.NA, NB = K.NB, T = 256, mode = swap_in ? 0 : 1;
  auto g = [&](size_t n) { return (unsigned)((n + T - 1) / T); };
  if (NA > 0) {
    k_gather_beads<<<g((size_t)(swap_in ? ROWS_A : 48) * NA), T, 0, st>>>(d.cur.a, d.nxt.a, perm, 0, NA, 0, mode);
    // a rows: st2 st3 nei2 nei4 nei3 (nei2, nei3 are protein links)
    k_gather_i32<<<g((size_t)5 * NA), T, 0, st>>>(d.a_int, s->a_tmp, perm, 0, NA, 5, (1u << 2) | (1u << 4), map);
  }
  if (NB > 0) {
    k_gather_beads<<<g((size_t)(swap_in ? ROWS_B : 24) * NB), T, 0, st>>>(d.cur.b, d.nxt.b, perm, NA, NB, 1, mode);
    k_gather_i32<<<g((size_t)8 * NB), T, 0, st>>>(d.b_int, s->b_tmp, perm, NA, NB, 8, 0xf0u, map);
  }
  if (!swap_in) return;
  std::swap(d.cur.a, d.nxt.a);
  std::swap(d.cur.b, d.nxt.b);
  std::swap(d.a_int, s->a_tmp);
  std::swap(d.b_int, s->b_tmp);
}

__global__ void k_iota(int32_t* a, int32_t* b, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) a[i] = b[i] = i;
}

// Exclusive scan of n counts (in may be out): tile sums, their scan, the tiles.
static void dev_scan(kmc_sim* s, const int32_t* in, int32_t* out, int n, hipStream_t st) {
  const int nb = (n + SCAN_TILE - 1) / SCAN_TILE;
  k_scan_part<<<nb, 256, 0, st>>>(in, n, s->scan_part);
  k_scan_top<<<1, 256, 0, st>>>(s->scan_part, nb);
  k_scan_down<<<nb, 256, 0, st>>>(in, out, n, s->scan_part);
}

// Stable LSD radix sort of the N packed slot keys (skeys, svals) over their
// low nbits, 8 bits a pass; returns the buffer holding the sorted values.
static int32_t* radix_sort(kmc_sim* s, int nbits, hipStream_t st, uint64_t** keys_out) {
  const int N = s->K.N, nblk = (N + RS_TILE - 1) / RS_TILE;
  uint64_t *ka = s->skeys, *kb = s->skeys2;
  int32_t *va = s->svals, *vb = s->svals2;
  if (nblk == 0) nbits = 0;  // (no slots: nothing to launch)
  for (int shift = 0; shift < nbits; shift += 8) {
    k_rs_hist<<<nblk, 256, 0, st>>>(ka, N, shift, s->rs_cnt, nblk);
    k_rs_rows<<<256, 256, 0, st>>>(s->rs_cnt, nblk, s->rs_tot);
    k_rs_scatter<<<nblk, 256, 0, st>>>(ka, va, kb, vb, N, shift, s->rs_cnt, s->rs_tot, nblk);
    std::swap(ka, kb);
    std::swap(va, vb);
  }
  *keys_out = ka;
  return va;
}

// debug (KMC_DEBUG_SYNC=1): the sorted keys non-decreasing, equal keys in
// their input order (stability), the values of each kind a permutation
static int check_sort(kmc_sim* s, const uint64_t* dk, const int32_t* dv) {
  const int N = s->K.N, NA = s->K.NA;
  std::vector<uint64_t> k((size_t)N);
  std::vector<int32_t> v((size_t)N);
  HIPCHK(s, hipStreamSynchronize(s->stream));
  HIPCHK(s, hipMemcpy(k.data(), dk, sizeof(uint64_t) * N, hipMemcpyDeviceToHost));
  HIPCHK(s, hipMemcpy(v.data(), dv, sizeof(int32_t) * N, hipMemcpyDeviceToHost));
  std::vector<uint8_t> seen((size_t)N, 0);
  for (int i = 0; i < N; ++i) {
    const int kind = i >= NA, base = kind ? NA : 0, nk = kind ? N - NA : NA;
    if (v[i] < 0 || v[i] >= nk || seen[(size_t)base + v[i]]++)
      return fail(s, KMC_ERR_HIP, "KMC_DEBUG_SYNC: re-sort values not a permutation at " + std::to_string(i));
    if (i > 0 && (k[i] < k[i - 1] || (k[i] == k[i - 1] && v[i] <= v[i - 1])))
      return fail(s, KMC_ERR_HIP, "KMC_DEBUG_SYNC: re-sort keys out of order at " + std::to_string(i));
  }
  return KMC_OK;
}

// Home list (kmc_kernels.hip §records): every slot's home cell and position
// from R, counting sort by cell; hstart = the cells' first home positions.
static int home_build(kmc_sim* s) {
  const KParams& K = s->K;
  Dev& d = s->d;
  hipStream_t st = s->stream;
  const int N = K.N, T = 256;
  HIPCHK(s, hipMemsetAsync(s->hcnt, 0, sizeof(int32_t) * (size_t)(s->ncell + 1), st));
  k_home_count<<<(N + T - 1) / T, T, 0, st>>>(K, d, s->hcnt);
  dev_scan(s, s->hcnt, d.hstart, s->ncell + 1, st);
  if (s->debug_sync) {  // debug: hstart the exclusive scan of the counts
    const size_t n = (size_t)s->ncell + 1;
    std::vector<int32_t> c(n), h(n);
    HIPCHK(s, hipStreamSynchronize(st));
    HIPCHK(s, hipMemcpy(c.data(), s->hcnt, sizeof(int32_t) * n, hipMemcpyDeviceToHost));
    HIPCHK(s, hipMemcpy(h.data(), d.hstart, sizeof(int32_t) * n, hipMemcpyDeviceToHost));
    int64_t run = 0;
    for (size_t i = 0; i < n; ++i) {
      if (h[i] != run) return fail(s, KMC_ERR_HIP, "KMC_DEBUG_SYNC: home scan wrong at " + std::to_string(i));
      run += c[i];
    }
  }
  k_home_place<<<(N + T - 1) / T, T, 0, st>>>(K, d);
  return hipGetLastError() == hipSuccess ? KMC_OK : fail(s, KMC_ERR_HIP, "home_build launch");
}

// Re-sort the slots spatially (between steps; R_new is free scratch then),
// then rebuild the home list in the new slot numbering.
static int resort(kmc_sim* s) {
  const KParams& K = s->K;
  Dev& d = s->d;
  hipStream_t st = s->stream;
  const int N = K.N, T = 256;
  // packed key widths: unit (reference index < N), cell, complex flag, kind
  int ob = 0;
  if (s->group_sort)
    while ((1ll << ob) < N) ++ob;
  const int tb = s->group_sort == 2 ? 1 : 0, nbits = ob + s->key_bits + tb + 1;
  k_slot_keys<<<(N + T - 1) / T, T, 0, st>>>(K, d, s->skeys, s->svals, s->group_sort, ob, s->key_bits);
  uint64_t* skeys = nullptr;
  const int32_t* sorted = radix_sort(s, nbits, st, &skeys);
  if (s->debug_sync) {
    const int rc = check_sort(s, skeys, sorted);
    if (rc != KMC_OK) return rc;
  }
  k_slot_inverse<<<(N + T - 1) / T, T, 0, st>>>(K, sorted, s->perm, s->newslot);
  reorder(s, s->perm, s->newslot, true);
  k_gather_ids<<<(N + T - 1) / T, T, 0, st>>>(K, d.id_of, s->id_tmp, d.slot_of, s->perm);
  std::swap(d.id_of, s->id_tmp);
  if (hipGetLastError() != hipSuccess) return fail(s, KMC_ERR_HIP, "resort launch");
  return home_build(s);
}

// Every array that carries a step / round tag or a per-step count: a state
// (re)loaded at an earlier step must not meet tags of a later one.
static int clear_step_tags(kmc_sim* s) {
  Dev& d = s->d;
  const size_t N = (size_t)s->K.N;
  hipStream_t st = s->stream;
  HIPCHK(s, hipMemsetAsync(d.ustate, 0, sizeof(uint32_t) * N, st));
  HIPCHK(s, hipMemsetAsync(d.moved, 0, sizeof(uint32_t) * N, st));
  HIPCHK(s, hipMemsetAsync(d.pend, 0, sizeof(uint32_t) * N, st));
  HIPCHK(s, hipMemsetAsync(d.ccnt, 0, sizeof(unsigned long long) * N, st));
  HIPCHK(s, hipMemsetAsync(d.vtag, 0, sizeof(uint32_t) * N, st));
  HIPCHK(s, hipMemsetAsync(d.shard_cnt, 0, sizeof(uint32_t) * 5 * NSHARD, st));
  // BFS candidates and shuffled rows are tagged with the step: an undone
  // chunk's tags would match the replayed steps' numbers
  HIPCHK(s, hipMemsetAsync(d.bfs_cand, 0, sizeof(uint32_t) * (size_t)s->K.NB, st));
  HIPCHK(s, hipMemsetAsync(d.shuf_tag, 0, sizeof(uint32_t) * (size_t)s->K.NB, st));
  HIPCHK(s, hipMemsetAsync(d.tout_n, 0, sizeof(uint32_t) * (size_t)s->ntiles, st));
  HIPCHK(s, hipMemsetAsync(d.cx_ext, 0, sizeof(uint32_t) * (size_t)s->K.NB, st));
  return KMC_OK;
}

// Chunk snapshot (kmc_step): everything a step reads from the previous one —
// R (device layout), state rows, slot maps, control block.  Everything else
// is rewritten within a step or is a tag cleared by clear_step_tags.
static int snapshot(kmc_sim* s, bool restore) {
  Dev& d = s->d;
  const size_t NA = (size_t)s->K.NA, NB = (size_t)s->K.NB, N = NA + NB;
  hipStream_t st = s->stream;
  if (!s->snap_ctl) {
    int rc = KMC_OK;
    rc |= dalloc(s, &s->snap_a, 48 * bead_slots((int)NA));
    rc |= dalloc(s, &s->snap_b, 24 * bead_slots((int)NB));
    rc |= dalloc(s, &s->snap_ai, 5 * NA);
    rc |= dalloc(s, &s->snap_bi, 8 * NB);
    rc |= dalloc(s, &s->snap_id, N);
    rc |= dalloc(s, &s->snap_slot, N);
    rc |= dalloc(s, &s->snap_ctl, 1);
    if (rc != KMC_OK) return rc;
  }
  auto cp = [&](void* live, void* snap, size_t bytes) {
    return restore ? hipMemcpyAsync(live, snap, bytes, hipMemcpyDeviceToDevice, st)
                   : hipMemcpyAsync(snap, live, bytes, hipMemcpyDeviceToDevice, st);
  };
  HIPCHK(s, cp(d.cur.a, s->snap_a, sizeof(double) * 48 * bead_slots((int)NA)));
  HIPCHK(s, cp(d.cur.b, s->snap_b, sizeof(double) * 24 * bead_slots((int)NB)));
  HIPCHK(s, cp(d.a_int, s->snap_ai, sizeof(int32_t) * 5 * NA));
  HIPCHK(s, cp(d.b_int, s->snap_bi, sizeof(int32_t) * 8 * NB));
  HIPCHK(s, cp(d.id_of, s->snap_id, sizeof(int32_t) * N));
  HIPCHK(s, cp(d.slot_of, s->snap_slot, sizeof(int32_t) * N));
  HIPCHK(s, cp(d.ctl, s->snap_ctl, sizeof(Ctl)));
  if (!restore) return KMC_OK;
  // the undone chunk may have re-sorted: the home list must describe the
  // restored slot numbering
  const int rc = clear_step_tags(s);
  return rc != KMC_OK ? rc : home_build(s);
}

static int set_state_impl(kmc_sim* s, const kmc_state_view* v);

int kmc_set_state(kmc_sim* s, const kmc_state_view* v) {
  if (!s || !v) return KMC_ERR_ARG;
  s->K.dd = 0;  // the whole trajectory (kmc_dd_set_state: one slab's window)
  return set_state_impl(s, v);
}

// The binding sites where the templates put them (main.cpp:303-311, 392-410,
// 1157-1178; every later move is rigid): a receptor's [3][2] = 2·[3][1] −
// [3][3] at RA from [3][1], a ligand's site [k][2] on the line from its
// centre through subunit [k][1] at (1 + √3/2) times the subunit's offset —
// each within 0.5 Å.  rxn_refine relies on both; a state that breaks them
// (a hand-made position.cpt) runs without it.
static bool sites_ok(const kmc_params* p, const kmc_state_view* v) {
  const int NA = p->n_a, NB = p->n_b;
  auto A = [&](int i, int j, int k, int c) { return v->ra[((size_t)((j - 1) * 4 + (k - 1)) * 3 + c) * NA + i]; };
  auto B = [&](int b, int j, int k, int c) { return v->rb[((size_t)((j - 1) * 2 + (k - 1)) * 3 + c) * NB + b]; };
  const double f = 1.0 + std::sqrt(3.0) / 2.0;
  for (int i = 0; i < NA; ++i) {
    double e = 0, r = 0;
    for (int c = 0; c < 3; ++c) {
      const double d = A(i, 3, 2, c) - (2 * A(i, 3, 1, c) - A(i, 3, 3, c)), q = A(i, 3, 2, c) - A(i, 3, 1, c);
      e += d * d;
      r += q * q;
    }
    if (!(e <= 0.25) || !(std::fabs(std::sqrt(r) - p->ra_radius) <= 0.5)) return false;
  }
  for (int b = 0; b < NB; ++b)
    for (int k = 2; k <= 4; ++k) {
      double e = 0;
      for (int c = 0; c < 3; ++c) {
        const double d = B(b, k, 2, c) - (B(b, 1, 1, c) + f * (B(b, k, 1, c) - B(b, 1, 1, c)));
        e += d * d;
      }
      if (!(e <= 0.25)) return false;
    }
  return true;
}

static int set_state_impl(kmc_sim* s, const kmc_state_view* v) {
  int rc = kmch_host::validate(&s->p, v, &s->err);
  if (rc != KMC_OK) return rc;
  {
    const char* rr = getenv("KMC_RXN_REFINE");
    s->K.rxn_refine = !(rr && *rr == '0') && sites_ok(&s->p, v);
  }
  const int NA = s->p.n_a, NB = s->p.n_b;
  Dev& d = s->d;
  // beads arrive in the host layout: into the scratch buffers, converted to
  // the device layout below
  HIPCHK(s, hipMemcpy(d.nxt.a, v->ra, sizeof(double) * 48 * (size_t)NA, hipMemcpyHostToDevice));
  HIPCHK(s, hipMemcpy(d.nxt.b, v->rb, sizeof(double) * 24 * (size_t)NB, hipMemcpyHostToDevice));
  HIPCHK(s, hipMemcpy(d.a_int, v->a_int, sizeof(int32_t) * 5 * (size_t)NA, hipMemcpyHostToDevice));
  HIPCHK(s, hipMemcpy(d.b_int, v->b_int, sizeof(int32_t) * 8 * (size_t)NB, hipMemcpyHostToDevice));
  int rl, mono, cis;
  kmch_host::derived_counts(&s->p, v, &rl, &mono, &cis);
  Ctl c;
  std::memset(&c, 0, sizeof c);
  c.step = (uint32_t)(v->step + 1);
  // counters keep the reference's incremental bookkeeping (main.cpp:1931-2136):
  // loaded value + change of the derived count
  c.off_bond = v->counters[0] - (rl + mono + cis);
  c.off_rl = v->counters[1] - rl;
  c.off_cis = v->counters[2] - cis;
  c.off_mono = v->counters[3] - mono;
  c.maxc = v->counters[4];
  HIPCHK(s, hipMemcpy(d.ctl, &c, sizeof c, hipMemcpyHostToDevice));
  rc = clear_step_tags(s);
  if (rc != KMC_OK) return rc;
  // no unit keys yet: the first slot sort groups by cell only
  HIPCHK(s, hipMemsetAsync(d.owner, 0xff, sizeof(int32_t) * (size_t)(NA + NB), s->stream));
  HIPCHK(s, hipMemsetAsync(d.croot, 0xff, sizeof(int32_t) * (size_t)(NA + NB), s->stream));
  // reference order = identity slots, then the spatial sort
  k_iota<<<(NA + NB + 255) / 256, 256, 0, s->stream>>>(d.id_of, d.slot_of, NA + NB);
  if (NA > 0)
    k_gather_beads<<<(unsigned)((48 * (size_t)NA + 255) / 256), 256, 0, s->stream>>>(d.nxt.a, d.cur.a, d.id_of, 0,
                                                                                     NA, 0, 2);
  if (NB > 0)
    k_gather_beads<<<(unsigned)((24 * (size_t)NB + 255) / 256), 256, 0, s->stream>>>(d.nxt.b, d.cur.b, d.id_of, NA,
                                                                                     NB, 1, 2);
  rc = resort(s);
  if (rc != KMC_OK) return rc;
  HIPCHK(s, hipStreamSynchronize(s->stream));
  s->step_done = v->step;
  // the sort above had no unit keys (owner, croot are set by the first
  // step): re-sort right before the second step, so that complex members
  // are grouped after the free units from then on, not only after the first
  // periodic re-sort (a loaded state otherwise runs its first resort_every
  // steps in the ungrouped layout)
  s->since_resort = s->resort_every >= 2 ? s->resort_every - 2 : 0;
  s->have_state = true;
  s->need_full = true;
  s->clusters_valid = false;
  s->snap_valid = false;
  return KMC_OK;
}

int kmc_get_state(kmc_sim* s, kmc_state_view* v) {
  if (!s || !v) return KMC_ERR_ARG;
  if (!s->have_state) return fail(s, KMC_ERR_ARG, "no state");
  const int NA = s->p.n_a, NB = s->p.n_b;
  Dev& d = s->d;
  // slots -> reference order (into R_new / scratch; links renumbered to reference indices)
  reorder(s, d.slot_of, d.id_of, false);
  HIPCHK(s, hipStreamSynchronize(s->stream));
  HIPCHK(s, hipMemcpy(v->ra, d.nxt.a, sizeof(double) * 48 * (size_t)NA, hipMemcpyDeviceToHost));
  HIPCHK(s, hipMemcpy(v->rb, d.nxt.b, sizeof(double) * 24 * (size_t)NB, hipMemcpyDeviceToHost));
  HIPCHK(s, hipMemcpy(v->a_int, s->a_tmp, sizeof(int32_t) * 5 * (size_t)NA, hipMemcpyDeviceToHost));
  HIPCHK(s, hipMemcpy(v->b_int, s->b_tmp, sizeof(int32_t) * 8 * (size_t)NB, hipMemcpyDeviceToHost));
  Ctl c;
  HIPCHK(s, hipMemcpy(&c, d.ctl, sizeof c, hipMemcpyDeviceToHost));
  int rl, mono, cis;
  kmch_host::derived_counts(&s->p, v, &rl, &mono, &cis);
  v->counters[0] = (rl + mono + cis) + c.off_bond;
  v->counters[1] = rl + c.off_rl;
  v->counters[2] = cis + c.off_cis;
  v->counters[3] = mono + c.off_mono;
  v->counters[4] = c.maxc;
  v->step = s->step_done;
  return KMC_OK;
}

int kmc_init_random(kmc_sim* s) {
  if (!s) return KMC_ERR_ARG;
  const int NA = s->p.n_a, NB = s->p.n_b;
  std::vector<double> ra((size_t)48 * NA + 1), rb((size_t)24 * NB + 1);
  std::vector<int32_t> ai((size_t)5 * NA + 1), bi((size_t)8 * NB + 1);
  kmc_state_view v{ra.data(), rb.data(), ai.data(), bi.data(), {0, 0, 0, 0, 0}, 0, 0};
  int rc = kmch_host::init_random(&s->p, &v, &s->err);
  if (rc != KMC_OK) return rc;
  return kmc_set_state(s, &v);
}

int kmc_load_cpt(kmc_sim* s, const char* path) {
  if (!s || !path) return KMC_ERR_ARG;
  const int NA = s->p.n_a, NB = s->p.n_b;
  std::vector<double> ra((size_t)48 * NA + 1), rb((size_t)24 * NB + 1);
  std::vector<int32_t> ai((size_t)5 * NA + 1), bi((size_t)8 * NB + 1);
  kmc_state_view v{ra.data(), rb.data(), ai.data(), bi.data(), {0, 0, 0, 0, 0}, 0, 0};
  int rc = kmch_host::load_cpt(&s->p, path, &v, &s->err);
  if (rc != KMC_OK) return rc;
  return kmc_set_state(s, &v);
}

int kmc_write_cpt(kmc_sim* s, const char* path) {
  if (!s || !path) return KMC_ERR_ARG;
  const int NA = s->p.n_a, NB = s->p.n_b;
  std::vector<double> ra((size_t)48 * NA + 1), rb((size_t)24 * NB + 1);
  std::vector<int32_t> ai((size_t)5 * NA + 1), bi((size_t)8 * NB + 1);
  kmc_state_view v{ra.data(), rb.data(), ai.data(), bi.data(), {0, 0, 0, 0, 0}, 0, 0};
  int rc = kmc_get_state(s, &v);
  if (rc != KMC_OK) return rc;
  return kmch_host::write_cpt(&s->p, &v, path, &s->err);
}

int kmc_save_state(kmc_sim* s, const char* path) {
  if (!s || !path) return KMC_ERR_ARG;
  const int NA = s->p.n_a, NB = s->p.n_b;
  std::vector<double> ra((size_t)48 * NA + 1), rb((size_t)24 * NB + 1);
  std::vector<int32_t> ai((size_t)5 * NA + 1), bi((size_t)8 * NB + 1);
  kmc_state_view v{ra.data(), rb.data(), ai.data(), bi.data(), {0, 0, 0, 0, 0}, 0, 0};
  int rc = kmc_get_state(s, &v);
  if (rc != KMC_OK) return rc;
  return kmch_host::save_state(&s->p, &v, path, &s->err);
}

int kmc_load_state(kmc_sim* s, const char* path) {
  if (!s || !path) return KMC_ERR_ARG;
  const int NA = s->p.n_a, NB = s->p.n_b;
  std::vector<double> ra((size_t)48 * NA + 1), rb((size_t)24 * NB + 1);
  std::vector<int32_t> ai((size_t)5 * NA + 1), bi((size_t)8 * NB + 1);
  kmc_state_view v{ra.data(), rb.data(), ai.data(), bi.data(), {0, 0, 0, 0, 0}, 0, 0};
  int rc = kmch_host::load_state(&s->p, path, &v, &s->err);
  if (rc != KMC_OK) return rc;
  return kmc_set_state(s, &v);
}

// accumulate the event pairs of ring slot `slot` (already complete or waited on)
static void harvest(kmc_sim* s, int slot) {
  for (int k = 0; k < KI_N; ++k) {
    size_t i = (size_t)slot * KI_N + k;
    if (!s->tused[i]) continue;
    float ms = 0;
    (void)hipEventSynchronize(s->tev[2 * i + 1]);
    if (hipEventElapsedTime(&ms, s->tev[2 * i], s->tev[2 * i + 1]) == hipSuccess) {
      s->kms[k] += ms;
      s->kcount[k] += 1;
    }
    s->tused[i] = 0;
  }
}

struct Bracket {
  kmc_sim* s;
  int k;
  hipStream_t st;
  Bracket(kmc_sim* s_, int k_, hipStream_t st_) : s(s_), k(k_), st(st_) {
    if (s->tnow && (s->tmask >> k & 1)) (void)hipEventRecord(s->tev[2 * ((size_t)s->tslot * KI_N + k)], st);
  }
  ~Bracket() {
    if (s->tnow && (s->tmask >> k & 1)) {
      size_t i = (size_t)s->tslot * KI_N + k;
      (void)hipEventRecord(s->tev[2 * i + 1], st);
      s->tused[i] = 1;
    }
  }
};
#define TIMED(k, ...) TIMED_ON(k, s->stream, __VA_ARGS__)
#define TIMED_ON(k, STREAM, ...)                                                                        \
  do {                                                                                                  \
    {                                                                                                   \
      Bracket b_(s, k, STREAM);                                                                         \
      __VA_ARGS__;                                                                                      \
    }                                                                                                   \
    if (s->debug_sync) {                                                                                \
      const hipError_t e_ = hipStreamSynchronize(STREAM);                                               \
      if (e_ != hipSuccess)                                                                             \
        return fail(s, KMC_ERR_HIP, std::string("KMC_DEBUG_SYNC: ") + KNAMES[k] + " failed in step " +     \
                                        std::to_string(s->launch_base) + ": " + hipGetErrorString(e_)); \
    }                                                                                                   \
  } while (0)

// debug (KMC_DEBUG_SYNC=1), after the exact tests: the collision lists'
// shard counts within capacity, every candidate a record index, every
// conflict entry / pending unit a unit key of this handle
static int debug_check_lists(kmc_sim* s) {
  Dev& d = s->d;
  const int N = s->K.N;
  HIPCHK(s, hipStreamSynchronize(s->stream));
  std::vector<uint32_t> cnt(5 * NSHARD);
  HIPCHK(s, hipMemcpy(cnt.data(), d.shard_cnt, sizeof(uint32_t) * cnt.size(), hipMemcpyDeviceToHost));
  const SList* L[5] = {&d.cand, &d.conf, &d.plist, &d.rej, &d.pairs};
  const char* names[5] = {"cand", "conf", "plist", "rej", "pairs"};
  char m[300];
  for (int l = 0; l < 5; ++l) {
    std::vector<int2> v((size_t)L[l]->cap * NSHARD);
    HIPCHK(s, hipMemcpy(v.data(), L[l]->data, sizeof(int2) * v.size(), hipMemcpyDeviceToHost));
    for (int k = 0; k < NSHARD; ++k) {
      const uint32_t c = std::min(cnt[l * NSHARD + k], L[l]->cap);
      for (uint32_t t = 0; t < c; ++t) {
        const int2 e = v[(size_t)k * L[l]->cap + t];
        const int x = e.x, y = l == 1 ? (e.y & 0x7fffffff) : e.y;
        bool ok = true;
        if (l == 0 || l == 4) ok = x >= 0 && x < 2 * N && y >= 0 && y < 2 * N;  // record indices
        if (l == 1) ok = x >= 0 && x < N && y >= 0 && y < N;                    // unit keys
        if (l == 2 || l == 3) ok = x >= 0 && x < N;
        if (!ok) {
          snprintf(m, sizeof m, "KMC_DEBUG_SYNC: list %s shard %d entry %u = (%d, %d) out of range (N %d) in step %lld",
                   names[l], k, t, e.x, e.y, N, (long long)s->launch_base);
          return fail(s, KMC_ERR_HIP, m);
        }
      }
    }
  }
  return KMC_OK;
}

#ifndef COARSE_N  // proteins from which the per-slot passes take 4 slots per thread
#define COARSE_N (4 << 20)
#endif
// s->tnow (this step bracketed) is set by the caller
// the complexes' stream and its fork / join events, made on first use
static int side_stream(kmc_sim* s) {
  if (s->side) return KMC_OK;
  // the chain is the longer path (its kernels wait on latency; starved of
  // workgroup slots by the free units' stream they ran 2-5x slower): its
  // stream gets the device's highest priority unless KMC_CX_STREAM_PRIO=0
  int lo = 0, hi = 0;
  const char* pr = getenv("KMC_CX_STREAM_PRIO");
  const bool prio = !(pr && *pr == '0') && hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess;
  if ((prio ? hipStreamCreateWithPriority(&s->side, hipStreamNonBlocking, hi)
            : hipStreamCreateWithFlags(&s->side, hipStreamNonBlocking)) != hipSuccess ||
      hipEventCreateWithFlags(&s->ev_fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&s->ev_join, hipEventDisableTiming) != hipSuccess)
    return fail(s, KMC_ERR_HIP, "the complexes' stream");
  return KMC_OK;
}

static int launch_step(kmc_sim* s, bool re_sort) {
  const KParams& K = s->K;
  Dev& d = s->d;
  hipStream_t st = s->stream;
  const int T = 256;
  const int gN = (K.N + T - 1) / T, gB = (K.NB + T - 1) / T;
  if (s->tnow) harvest(s, s->tslot);  // the slot's previous use is TRING bracketed steps old
  if (re_sort) {
    int rc;
    TIMED(KI_RESORT, rc = resort(s));
    if (rc != KMC_OK) return rc;
  }
  if (s->poison) {
    // debug: every bead of R_new must be rewritten by a proposal or a revert
    (void)hipMemsetAsync(d.nxt.a, 0xff, sizeof(double) * 48 * bead_slots(K.NA), st);
    (void)hipMemsetAsync(d.nxt.b, 0xff, sizeof(double) * 24 * bead_slots(K.NB), st);
  }
  // complexes: the previous step's k_finalize dissolved those whose bonds
  // changed; a full rebuild (after a re-sort, a new state, an undone chunk,
  // KMC_FULL_BFS) resets them all here
  if (K.NB > 0 && (s->need_full || re_sort || s->always_full))
    TIMED(KI_CX_KILL, (k_cx_kill<<<std::min(gN, 1024), T, 0, st>>>(K, d)));
  s->need_full = false;
  // slots per thread of the per-slot passes k_classify / k_diss_observe
  const int per = K.N >= COARSE_N ? 4 : 1, gP = (K.N + T * per - 1) / (T * per);
  if (per == 4) TIMED(KI_CLASSIFY, (k_classify<4><<<gP, T, 0, st>>>(K, d)));
  else TIMED(KI_CLASSIFY, (k_classify<1><<<gP, T, 0, st>>>(K, d)));
  // KI_PROPOSE brackets the whole proposal phase: every protein's R read and
  // R_new written once (the bench's roofline unit).  Complexes kept or newly
  // registered (k_bfs); their rigid-move parameters (cx_params, in the first
  // workgroups of k_propose_free); every unit moved by coalesced
  // thread-per-slot streams: free receptors, cis dimers, free ligands
  // (k_propose_free), members of complexes of <= CXL proteins
  // (k_move_members, with their complex's parameters); the complexes' lay-down / alignment tests and new
  // records (k_cx_check); the few complexes whose tests fail, with several
  // ligands or many members (k_complex_heavy).
  {
    Bracket b_(s, KI_PROPOSE, st);
    const int gL = std::min(2048, (K.NB + T - 1) / T);  // grid-stride over the descriptor list
    const bool side = s->cx_stream != 0 && K.NB > 0 && !s->use_graphs;
    if (K.NB > 0 && (!side || s->cx_stream == 3)) {
      TIMED(KI_BFS, (k_bfs<<<gB, T, 0, st>>>(K, d)));
    }
    const int gC = K.NB > 0 ? std::min(gL, 512) : 0;  // grid-stride over the descriptor list
    const int gP3 = s->cx_params_wg > 0 ? std::min(s->cx_params_wg, 1 << 16) : gL;
    if (side && s->cx_stream == 3) {
      // the members' HBM stream first, alone; then the complexes' checks and
      // heavy path (dependent chains waiting on latency) beside the free
      // units' HBM stream
      const int rc = side_stream(s);
      if (rc != KMC_OK) return rc;
      hipStream_t sd = s->side;
      // cx_params only, alone (one thread per complex up to gL workgroups;
      // 512 / gL / 4 096 workgroups: equal at C5, 128 us, profiles/r06/ab_cx_params_wg_C5)
      k_propose_free<<<gP3, T, 0, st>>>(K, d, gP3);
      TIMED(KI_MOVE_MEMBERS, (k_move_members<<<gN, T, 0, st>>>(K, d)));
      HIPCHK(s, hipEventRecord(s->ev_fork, st));
      HIPCHK(s, hipStreamWaitEvent(sd, s->ev_fork, 0));
      TIMED_ON(KI_CX_CHECK, sd, (k_cx_check<<<gL, T, 0, sd>>>(K, d)));
      TIMED_ON(KI_CX_HEAVY, sd, (k_complex_heavy<<<1024, T, 0, sd>>>(K, d)));
      HIPCHK(s, hipEventRecord(s->ev_join, sd));
      TIMED(KI_PROPOSE_FREE, (k_propose_free<<<gN, T, 0, st>>>(K, d, 0)));  // the free units
      HIPCHK(s, hipStreamWaitEvent(st, s->ev_join, 0));
    } else if (side) {
      // the complex chain — BFS of the candidates, rigid-move parameters,
      // members, checks, heavy path — beside the free units (k_classify has
      // settled every free unit; disjoint slots, records and beads; shared
      // lists only through atomics): the free units stream HBM while the
      // complexes' dependent chains wait on latency
      const int rc = side_stream(s);
      if (rc != KMC_OK) return rc;
      hipStream_t sd = s->side;
      HIPCHK(s, hipEventRecord(s->ev_fork, st));
      HIPCHK(s, hipStreamWaitEvent(sd, s->ev_fork, 0));
      TIMED_ON(KI_BFS, sd, (k_bfs<<<gB, T, 0, sd>>>(K, d)));
      k_propose_free<<<gC, T, 0, sd>>>(K, d, gC);  // cx_params only (the bracket of the id is the free units')
      if (s->cx_stream == 1) {
        TIMED_ON(KI_MOVE_MEMBERS, sd, (k_move_members<<<gN, T, 0, sd>>>(K, d)));
        TIMED_ON(KI_CX_CHECK, sd, (k_cx_check<<<gL, T, 0, sd>>>(K, d)));
        TIMED_ON(KI_CX_HEAVY, sd, (k_complex_heavy<<<1024, T, 0, sd>>>(K, d)));
      }
      HIPCHK(s, hipEventRecord(s->ev_join, sd));
      TIMED(KI_PROPOSE_FREE, (k_propose_free<<<gN, T, 0, st>>>(K, d, 0)));  // the free units
      HIPCHK(s, hipStreamWaitEvent(st, s->ev_join, 0));
      if (s->cx_stream == 2) {  // the members' streams after the free units', on the main stream
        TIMED(KI_MOVE_MEMBERS, (k_move_members<<<gN, T, 0, st>>>(K, d)));
        TIMED(KI_CX_CHECK, (k_cx_check<<<gL, T, 0, st>>>(K, d)));
        TIMED(KI_CX_HEAVY, (k_complex_heavy<<<1024, T, 0, st>>>(K, d)));
      }
    } else {
      TIMED(KI_PROPOSE_FREE, (k_propose_free<<<gC + gN, T, 0, st>>>(K, d, gC)));
      if (K.NB > 0) {
        TIMED(KI_MOVE_MEMBERS, (k_move_members<<<gN, T, 0, st>>>(K, d)));
        TIMED(KI_CX_CHECK, (k_cx_check<<<gL, T, 0, st>>>(K, d)));
        TIMED(KI_CX_HEAVY, (k_complex_heavy<<<1024, T, 0, st>>>(K, d)));
      }
    }
  }
  if (K.dbg_recs) k_rec_check<<<std::min(2048, (2 * K.N + T - 1) / T), T, 0, st>>>(K, d);
  const int gX = std::min(2048, (K.N + T - 1) / T);  // grid-stride kernels over device-sized lists
  const int ntiles = s->ntiles;
  // collision candidates and reaction candidates, one staging of each tile
  TIMED(KI_PAIR_SCAN, (k_pair_scan<<<ntiles, PAIR_THREADS, 0, st>>>(K, d)));
  // the tiles too dense for the pair scan's LDS, one per workgroup, then the
  // exact tests of the candidates
  TIMED(KI_COL_EXACT, {
#if DENSE_KERNEL
    // (a second stream for it, forked after the pair scan and joined before
    // the rounds, cost 15 us per step at C3 for the 5 us launch it hides)
    k_col_dense<<<64, T, 0, st>>>(K, d);
    if (s->debug_sync && hipStreamSynchronize(st) != hipSuccess)
      return fail(s, KMC_ERR_HIP, "KMC_DEBUG_SYNC: k_col_dense failed in step " + std::to_string(s->launch_base));
#endif
    k_col_exact<<<std::max(gX, 64), T, 0, st>>>(K, d);
  });
  if (s->debug_sync) {
    const int rc = debug_check_lists(s);
    if (rc != KMC_OK) return rc;
  }
  TIMED(KI_COL_ROUNDS, {
    k_col_resolve<<<gX, T, 0, st>>>(K, d);
    if (s->debug_sync && hipStreamSynchronize(st) != hipSuccess)
      return fail(s, KMC_ERR_HIP, "KMC_DEBUG_SYNC: k_col_resolve failed in step " + std::to_string(s->launch_base));
    k_col_tail<<<1, 1024, 0, st>>>(K, d, 1);
  });
  // (the revert cannot run beside the reactions: an association snaps the
  // receptor in R_new, and a receptor of a rejected unit must be reverted
  // before that — DESIGN.md §8, the rejected REJ_SIDE variant)
  // the revert and the exact reaction tests (one launch, k_commit_rxn)
#ifndef COMMIT_RXN  // (A/B builds: 0 = the revert, then the reaction tests, in two launches)
#define COMMIT_RXN 1
#endif
#if COMMIT_RXN
  TIMED(KI_COMMIT, (k_commit_rxn<<<gX + (K.NA > 0 ? 1024 : 0), T, 0, st>>>(K, d, gX)));
#else
  TIMED(KI_COMMIT, {
    k_commit_rxn<<<gX, T, 0, st>>>(K, d, gX);
    if (K.NA > 0) k_commit_rxn<<<1024, T, 0, st>>>(K, d, 0);
  });
#endif
  if (K.NA > 0) TIMED(KI_MATCH, (k_match<<<1, 1024, 0, st>>>(K, d)));
  TIMED(KI_DISS_OBSERVE, {
    if (per == 4) k_diss_observe<4><<<gP, T, 0, st>>>(K, d);
    else k_diss_observe<1><<<gP, T, 0, st>>>(K, d);
    k_finalize<<<1, 1024, 0, st>>>(K, d, s->p.time_step, gP);
  });
  if (s->tnow) s->tslot = (s->tslot + 1) % TRING;
  // R_new becomes R (main.cpp:2164-2191): swap the bead buffers
  std::swap(d.cur, d.nxt);
  return KMC_OK;
}

// One step through a HIP graph: replay the graph captured with the same
// kernel arguments, or capture this step (launch_step's host side runs during
// the capture: it swaps the buffers exactly as an eager step) and replay it.
static int launch_step_graph(kmc_sim* s) {
  unsigned char key[sizeof(KParams) + sizeof(Dev)];
  std::memcpy(key, &s->K, sizeof(KParams));
  std::memcpy(key + sizeof(KParams), &s->d, sizeof(Dev));
  for (auto& g : s->graphs)
    if (g.valid && std::memcmp(g.key, key, sizeof key) == 0) {
      HIPCHK(s, hipGraphLaunch(g.exec, s->stream));
      std::swap(s->d.cur, s->d.nxt);
      ++s->graph_launches;
      return KMC_OK;
    }
  auto& g = s->graphs[s->graph_next];
  s->graph_next = (s->graph_next + 1) % kmc_sim::NGRAPH;
  if (g.exec) (void)hipGraphExecDestroy(g.exec);
  g.exec = nullptr;
  g.valid = false;
  HIPCHK(s, hipStreamBeginCapture(s->stream, hipStreamCaptureModeThreadLocal));
  const int rc = launch_step(s, false);
  hipGraph_t graph = nullptr;
  const hipError_t ec = hipStreamEndCapture(s->stream, &graph);
  if (rc != KMC_OK) {
    if (graph) (void)hipGraphDestroy(graph);
    return rc;
  }
  HIPCHK(s, ec);
  const hipError_t ei = hipGraphInstantiate(&g.exec, graph, nullptr, nullptr, 0);
  (void)hipGraphDestroy(graph);
  HIPCHK(s, ei);
  std::memcpy(g.key, key, sizeof key);
  g.valid = true;
  ++s->graph_captures;
  HIPCHK(s, hipGraphLaunch(g.exec, s->stream));
  ++s->graph_launches;
  return KMC_OK;
}

// Launch n steps from the current state, whose last completed step is `base`
// (s->step_done, or an earlier step while replaying from the snapshot);
// device obs records land in obs_buf.  Returns after the stream has drained,
// with the control block in ctl_host.
static int dd_after_step(kmc_sim* s);

static int run_chunk(kmc_sim* s, int64_t n, int64_t base, kmc_obs* out = nullptr) {
  HIPCHK(s, hipMemsetAsync(&s->d.ctl->obs_idx, 0, sizeof(uint32_t), s->stream));
  for (int64_t k = 0; k < n; ++k) {
    const bool rs = s->resort_every > 0 && ++s->since_resort >= s->resort_every;
    if (rs) s->since_resort = 0;
    // unit-state tags are (step mod 2^30): clear them when the tag wraps
    if (((base + k + 1) & 0x3fffffff) == 0)
      HIPCHK(s, hipMemsetAsync(s->d.ustate, 0, sizeof(uint32_t) * (size_t)s->K.N, s->stream));
    s->tnow = s->tmask && (s->tcount++ % s->tperiod) == 0;
    // graph replay for the plain steps: no re-sort, no full complex rebuild, no
    // event brackets, no debug poison
    const bool plain = !rs && !s->tnow && !s->poison && !s->need_full && !s->always_full &&
                       s->K.dbg_stage == 0 && !s->debug_sync;
    s->launch_base = base + k + 1;
    int rc = (s->use_graphs && plain) ? launch_step_graph(s) : launch_step(s, rs);
    if (rc != KMC_OK) return rc;
  }
  HIPCHK(s, hipGetLastError());
  if (s->dd_step_pending) {  // kmc_dd_step: the exchange rows and the jumpers, before the one wait
    const int rc = dd_after_step(s);
    if (rc != KMC_OK) return rc;
  }
  HIPCHK(s, hipMemcpyAsync(s->ctl_host, s->d.ctl, sizeof(Ctl), hipMemcpyDeviceToHost, s->stream));
  // the records in the same wait (used by the caller only if the chunk raised no error bit)
  if (out) HIPCHK(s, hipMemcpyAsync(out, s->obs_buf, sizeof(kmc_obs_dev) * n, hipMemcpyDeviceToHost, s->stream));
  HIPCHK(s, hipStreamSynchronize(s->stream));
  if (s->tmask)
    for (int slot = 0; slot < TRING; ++slot) harvest(s, slot);
  return KMC_OK;
}

// Steps run in chunks of up to 4096 launched back to back; the device error
// bits are read once per chunk.  A device snapshot of the state at most
// snap_span steps before the chunk's end is kept (taken at a chunk start when
// the last one is older), so a chunk that raised an error bit is undone by
// restoring it and replaying the steps between it and the chunk:
//  * an output list or edge buffer overflowed (ERR_EDGES): the lists are
//    doubled and the chunk replayed — with keyed draws the replay is the same
//    trajectory, so capacities never change results;
//  * anything else (geometry bound, unresolved conflicts, members overflow):
//    the steps before the failing one are replayed and kept, kmc_step returns
//    the error, and the state and kmc_current_step() are those of the last
//    good step.
int kmc_step(kmc_sim* s, int64_t nsteps, kmc_obs* out) {
  if (!s) return KMC_ERR_ARG;
  if (!s->have_state) return fail(s, KMC_ERR_ARG, "no state: call kmc_init_random / kmc_load_cpt / kmc_set_state");
  if (nsteps <= 0) return KMC_OK;
  static_assert(sizeof(kmc_obs_dev) == sizeof(kmc_obs), "obs layout");
  const int64_t chunk = 4096;
  if (!s->obs_buf) {
    HIPCHK(s, hipMalloc((void**)&s->obs_buf, sizeof(kmc_obs_dev) * chunk));
    s->obs_cap = chunk;
    s->d.obs = s->obs_buf;
  }
  int64_t done = 0;
  while (done < nsteps) {
    const int64_t n = std::min(chunk, nsteps - done);
    int rc = KMC_OK;
    // a decomposed window takes no snapshot: every step's import changes its
    // state (a replay from a snapshot would miss the imports), and the slab
    // driver keeps the checkpoint it rolls back to
    if (!s->K.dd && (!s->snap_valid || s->step_done + n - s->snap_step > s->snap_span)) {
      rc = snapshot(s, false);
      if (rc != KMC_OK) return rc;
      s->snap_valid = true;
      s->snap_step = s->step_done;
      s->snap_since = s->since_resort;
      ++s->n_snapshots;
    }
    bool copied = false;  // the chunk's records already in `out`
    for (;;) {
      rc = run_chunk(s, n, s->step_done, out ? out + done : nullptr);
      if (rc != KMC_OK) return rc;
      const uint32_t err = s->ctl_host->err;
      if (!err) {
        copied = out != nullptr;
        break;
      }
      // the failing step's own bits: later steps of the chunk ran on its
      // dropped entries, so their bits may be consequences
      const uint32_t cause = s->ctl_host->err_first;
      const int64_t bad = (int64_t)s->ctl_host->err_step;
      if (s->K.dd) {
        // no snapshot to undo to: the window's state is lost.  A list
        // overflow alone doubles the lists first, so that the handle the
        // driver rebuilds (kmc_list_growth) runs the step with room
        const bool grow = (cause & ~ERR_EDGES) == 0;
        if (grow && s->grow < 6) {
          s->grow += 1;
          if (alloc_lists(s) != KMC_OK) return fail(s, KMC_ERR_HIP, "growing the output lists failed");
        }
        s->have_state = false;
        s->clusters_valid = false;
        char m[200];
        snprintf(m, sizeof m, "dd: device error bits 0x%x at step %lld; the window's state is lost (list growth 2^%d)",
                 err, (long long)bad, s->grow);
        return fail(s, grow ? KMC_ERR_CAPACITY : (cause & ERR_GEOMETRY) ? KMC_ERR_GEOMETRY : KMC_ERR_CAPACITY, m);
      }
      // undo to the snapshot, then replay the steps between it and this
      // chunk (already returned by earlier calls: same trajectory, keyed
      // draws) without output
      rc = snapshot(s, true);
      if (rc != KMC_OK) return rc;
      s->since_resort = s->snap_since;
      s->need_full = true;  // the kept complexes may describe the undone steps
      ++s->n_replays;
      // a list overflow alone: double the lists (at most 64x the defaults)
      // and run the chunk again; any other bit is reported at once
      const bool grow = (cause & ~ERR_EDGES) == 0 && s->grow < 6;
      if (grow) {
        s->grow += 1;
        if (alloc_lists(s) != KMC_OK) return fail(s, KMC_ERR_HIP, "growing the output lists failed");
      }
      for (int64_t at = s->snap_step; at < s->step_done;) {
        const int64_t m = std::min(chunk, s->step_done - at);
        rc = run_chunk(s, m, at);
        if (rc != KMC_OK) return rc;
        if (s->ctl_host->err) {
          // the device is somewhere between the snapshot and step_done: go
          // back to the snapshot (still valid) and say so — the host's step
          // count must describe the device state
          rc = snapshot(s, true);
          if (rc != KMC_OK) {
            s->have_state = false;  // neither state is known: the caller must set one
            return rc;
          }
          const int64_t at_fail = at;
          s->step_done = s->snap_step;
          s->since_resort = s->snap_since;
          s->need_full = true;
          s->clusters_valid = false;
          char m2[200];
          snprintf(m2, sizeof m2,
                   "replay from the snapshot raised an error the original steps did not (in steps %lld..%lld); "
                   "state restored to step %lld",
                   (long long)at_fail + 1, (long long)(at_fail + m), (long long)s->step_done);
          return fail(s, KMC_ERR_HIP, m2);
        }
        at += m;
      }
      if (grow) continue;
      // keep the steps before the failing one
      const int64_t good = std::max<int64_t>(0, std::min<int64_t>(n, bad - (s->step_done + 1)));
      if (good > 0) {
        rc = run_chunk(s, good, s->step_done);
        if (rc != KMC_OK) return rc;
        if (out)
          HIPCHK(s, hipMemcpy(out + done, s->obs_buf, sizeof(kmc_obs_dev) * good, hipMemcpyDeviceToHost));
        s->step_done += good;
      }
      s->clusters_valid = good > 0;
      char m[200];
      snprintf(m, sizeof m, "device error bits 0x%x at step %lld; state kept at step %lld", err, (long long)bad,
               (long long)s->step_done);
      const int code = (cause & ERR_GEOMETRY) ? KMC_ERR_GEOMETRY : KMC_ERR_CAPACITY;
      return fail(s, code, m);
    }
    if (out && !copied)
      HIPCHK(s, hipMemcpy(out + done, s->obs_buf, sizeof(kmc_obs_dev) * n, hipMemcpyDeviceToHost));
    s->step_done += n;
    s->clusters_valid = true;
    if (s->debug_counts) {
      const uint32_t* l = s->ctl_host->last;
      fprintf(stderr, "kmc step %lld: candidates %u conflicts %u pending-units %u rejected %u rxn-pairs %u rl-edges %u cis-edges %u bfs-overflow %u outliers %u (list growth 2^%d, replays %lld, snapshots %lld, forced rebuilds %u)\n",
              (long long)s->step_done, l[0], l[1], l[2], l[3], l[4], l[5], l[6], l[7], s->ctl_host->last_outl, s->grow,
              (long long)s->n_replays, (long long)s->n_snapshots, s->ctl_host->n_forced);
      if (s->K.dbg_cand) {
        const uint32_t* c = s->ctl_host->cand_kind;
        const uint32_t* r = s->ctl_host->rxn_kind;
        fprintf(stderr, "kmc cand AA %u/%u AB %u/%u BB %u/%u (tested/colliding) rxn %u final %u gate %u accept %u "
                "refined-out %u\n",
                c[0], c[1], c[2], c[3], c[4], c[5], r[0], r[1], r[2], r[3], r[4]);
      }
#if WALK_STATS
      {
        unsigned long long w = 0, wo = 0;
        if (hipMemcpyFromSymbol(&w, HIP_SYMBOL(kmc_walk_pairs), sizeof w) == hipSuccess &&
            hipMemcpyFromSymbol(&wo, HIP_SYMBOL(kmc_walk_pairs_old), sizeof wo) == hipSuccess)
          fprintf(stderr, "kmc walk pairs %llu old-position items %llu (summed since the library loaded)\n", w, wo);
      }
#endif
      const uint64_t* t = s->ctl_host->stamps;
      if (t[16])
        fprintf(stderr, "kmc stamps heavy stage %llu align %llu writeback %llu records %llu (cycles summed over "
                "waves) complexes %llu max-cycles %llu members %llu\n",
                (unsigned long long)t[16], (unsigned long long)t[17], (unsigned long long)t[18],
                (unsigned long long)t[19], (unsigned long long)t[20], (unsigned long long)t[21],
                (unsigned long long)t[22]);
      if (t[0] | t[8])
        fprintf(stderr, "kmc stamps col %llu %llu %llu %llu %llu %llu %llu %llu rxn %llu %llu %llu %llu %llu %llu %llu %llu\n",
                (unsigned long long)t[0], (unsigned long long)t[1], (unsigned long long)t[2], (unsigned long long)t[3],
                (unsigned long long)t[4], (unsigned long long)t[5], (unsigned long long)t[6], (unsigned long long)t[7],
                (unsigned long long)t[8], (unsigned long long)t[9], (unsigned long long)t[10], (unsigned long long)t[11],
                (unsigned long long)t[12], (unsigned long long)t[13], (unsigned long long)t[14], (unsigned long long)t[15]);
    }
    done += n;
  }
  return KMC_OK;
}

// ---------------------------------------------------------------- diagnostics
// op: 0 sin, 1 cos, 2 atan2(x, y), 3 acos, 4 sqrt, 5 x / y, 6 round
__global__ void k_math(int op, const double* x, const double* y, double* out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double a = x[i], b = y[i], r = 0;
  switch (op) {
    case 0: r = kmcm::sin(a); break;
    case 1: r = kmcm::cos(a); break;
    case 2: r = kmcm::atan2(a, b); break;
    case 3: r = kmcm::acos(a); break;
    case 4: r = kmcm::sqrt_(a); break;
    case 5: r = a / b; break;
    default: r = kmcm::round_(a); break;
  }
  out[i] = r;
}

int kmc_device_math(int op, const double* x, const double* y, double* out, int64_t n) {
  if (n <= 0) return KMC_OK;
  double *dx = nullptr, *dy = nullptr, *dout = nullptr;
  size_t b = sizeof(double) * (size_t)n;
  if (hipMalloc(&dx, b) != hipSuccess || hipMalloc(&dy, b) != hipSuccess || hipMalloc(&dout, b) != hipSuccess)
    return KMC_ERR_HIP;
  int rc = KMC_OK;
  if (hipMemcpy(dx, x, b, hipMemcpyHostToDevice) != hipSuccess || hipMemcpy(dy, y, b, hipMemcpyHostToDevice) != hipSuccess)
    rc = KMC_ERR_HIP;
  if (rc == KMC_OK) {
    k_math<<<(int)((n + 255) / 256), 256>>>(op, dx, dy, dout, (int)n);
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(out, dout, b, hipMemcpyDeviceToHost) != hipSuccess)
      rc = KMC_ERR_HIP;
  }
  (void)hipFree(dx);
  (void)hipFree(dy);
  (void)hipFree(dout);
  return rc;
}

int kmc_get_clusters(kmc_sim* s, int32_t* row_len, int32_t* members) {
  if (!s || !row_len || !members) return KMC_ERR_ARG;
  if (!s->have_state || !s->clusters_valid)
    return fail(s, KMC_ERR_ARG, "no step simulated since the state was set (or the last chunk was undone)");
  const int NA = s->p.n_a, NB = s->p.n_b, N = NA + NB;
  std::vector<uint8_t> kind(N);
  std::vector<int32_t> off(NB), size(NB), mem(N), id_of(N), slot_of(N);
  HIPCHK(s, hipStreamSynchronize(s->stream));
  HIPCHK(s, hipMemcpy(kind.data(), s->d.ukind, N, hipMemcpyDeviceToHost));
  HIPCHK(s, hipMemcpy(off.data(), s->d.cx_off, sizeof(int32_t) * NB, hipMemcpyDeviceToHost));
  HIPCHK(s, hipMemcpy(size.data(), s->d.cx_size, sizeof(int32_t) * NB, hipMemcpyDeviceToHost));
  std::vector<int32_t> shuf(s->d.mcap);
  std::vector<uint32_t> stag(NB);
  mem.resize(s->d.mcap);
  HIPCHK(s, hipMemcpy(mem.data(), s->d.members, sizeof(int32_t) * s->d.mcap, hipMemcpyDeviceToHost));
  HIPCHK(s, hipMemcpy(shuf.data(), s->d.shuf, sizeof(int32_t) * s->d.mcap, hipMemcpyDeviceToHost));
  HIPCHK(s, hipMemcpy(stag.data(), s->d.shuf_tag, sizeof(uint32_t) * NB, hipMemcpyDeviceToHost));
  HIPCHK(s, hipMemcpy(id_of.data(), s->d.id_of, sizeof(int32_t) * N, hipMemcpyDeviceToHost));
  HIPCHK(s, hipMemcpy(slot_of.data(), s->d.slot_of, sizeof(int32_t) * N, hipMemcpyDeviceToHost));
  // unit tables of the last step's classification (slots are re-sorted only
  // right before a step, so they still use the current slot numbering)
  int64_t o = 0;
  for (int b = 0; b < NB; ++b) {
    int p = slot_of[NA + b];  // ligand b's slot
    if (kind[p] == U_FREE_B) {
      row_len[b] = 1;
      members[o++] = NA + b + 1;
    } else if (kind[p] == U_COMPLEX) {
      int lb = p - NA;
      row_len[b] = size[lb];
      // the row after the multi-ligand shuffles when this step shuffled it
      const int32_t* row = (stag[lb] == (uint32_t)s->step_done ? shuf.data() : mem.data()) + off[lb];
      for (int t = 0; t < size[lb]; ++t) members[o++] = id_of[row[t]] + 1;
    } else {
      row_len[b] = 0;
    }
  }
  return KMC_OK;
}

int kmc_set_timing(kmc_sim* s, uint64_t kernel_mask) {
  if (!s) return KMC_ERR_ARG;
  if (kernel_mask && s->tev.empty()) {
    s->tev.assign((size_t)TRING * KI_N * 2, nullptr);
    s->tused.assign((size_t)TRING * KI_N, 0);
    for (auto& e : s->tev) HIPCHK(s, hipEventCreate(&e));
  }
  s->tmask = kernel_mask;
  s->tcount = 0;
  for (int k = 0; k < KI_N; ++k) {
    s->kms[k] = 0;
    s->kcount[k] = 0;
  }
  return KMC_OK;
}

int kmc_set_timing_period(kmc_sim* s, int32_t every) {
  if (!s || every < 1) return KMC_ERR_ARG;
  s->tperiod = every;
  return KMC_OK;
}

int kmc_kernel_times(const kmc_sim* s, double* total_ms, int64_t* launches, int32_t n) {
  if (!s) return KMC_ERR_ARG;
  for (int k = 0; k < n && k < KI_N; ++k) {
    if (total_ms) total_ms[k] = s->kms[k];
    if (launches) launches[k] = s->kcount[k];
  }
  return KI_N;
}

const char* kmc_kernel_name(int32_t id) { return id >= 0 && id < KI_N ? KNAMES[id] : ""; }

}  // extern "C"

// ---------------------------------------------------------------- decomposed trajectory
// One slab's window of a trajectory split over several handles (SURVEY.md
// §8(f).4): the host driver (slabs.py) sets the window's
// proteins with their global indices and ownership, steps every handle, and
// moves the end-of-step state of each slab's boundary proteins to the
// handles that hold them as halo copies.  Exchanged record of one protein:
// 48 doubles (the kmc_state_view bead order: receptor ((j-1)·4 + k-1)·3 + c,
// ligand ((j-1)·2 + k-1)·3 + c in the first 24) and 8 ints (receptor st2 st3
// nei2 nei4 nei3, ligand st1..4 nei1..4; protein links are local reference
// index + 1, 0 = none).
__global__ void k_dd_export(KParams P, Dev d, int n, const int32_t* ids, double* beads, int32_t* ints) {
  const int NA = P.NA, NB = P.NB;
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < (size_t)n * 48) {
    const int i = (int)(t / 48), e = (int)(t % 48), slot = d.slot_of[ids[i]], bead = e / 3, c = e % 3;
    double v = 0.0;
    if (slot < NA) v = d.cur.A(slot, bead / 4 + 1, bead % 4 + 1, c);
    else if (e < 24) v = d.cur.B(slot - NA, bead / 2 + 1, bead % 2 + 1, c);
    beads[t] = v;
  }
  if (t < (size_t)n * 8) {
    const int i = (int)(t / 8), f = (int)(t % 8), slot = d.slot_of[ids[i]];
    int v = 0;
    bool link = false;
    if (slot < NA) {
      if (f < 5) v = d.a_int[(size_t)f * NA + slot];
      link = f == 2 || f == 4;
    } else {
      v = d.b_int[(size_t)f * NB + (slot - NA)];
      link = f >= 4;
    }
    if (link && v > 0) v = d.id_of[v - 1] + 1;
    ints[t] = v;
  }
}

// The owner's end-of-step state of halo proteins into R and the state rows;
// flags[i] |= 1 where a coordinate differed bit for bit from this handle's
// own result, 2 where a status or link did.
__global__ void k_dd_import(KParams P, Dev d, int n, const int32_t* ids, const double* beads, const int32_t* ints,
                            uint8_t* flags) {
  const int NA = P.NA, NB = P.NB;
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < (size_t)n * 48) {
    const int i = (int)(t / 48), e = (int)(t % 48), slot = d.slot_of[ids[i]], bead = e / 3, c = e % 3;
    double* dst = nullptr;
    if (slot < NA) dst = &d.cur.A(slot, bead / 4 + 1, bead % 4 + 1, c);
    else if (e < 24) dst = &d.cur.B(slot - NA, bead / 2 + 1, bead % 2 + 1, c);
    if (dst) {
      const double v = beads[t];
      if (__double_as_longlong(*dst) != __double_as_longlong(v)) {
        atomicOr((uint32_t*)&flags[i & ~3], 1u << (8 * (i & 3)));
        *dst = v;
      }
    }
  }
  if (t < (size_t)n * 8) {
    const int i = (int)(t / 8), f = (int)(t % 8), slot = d.slot_of[ids[i]];
    int32_t* dst = nullptr;
    bool link = false;
    if (slot < NA) {
      if (f < 5) dst = &d.a_int[(size_t)f * NA + slot];
      link = f == 2 || f == 4;
    } else {
      dst = &d.b_int[(size_t)f * NB + (slot - NA)];
      link = f >= 4;
    }
    if (dst) {
      int v = ints[t];
      if (link && v > 0) v = d.slot_of[v - 1] + 1;
      if (*dst != v) {
        atomicOr((uint32_t*)&flags[i & ~3], 2u << (8 * (i & 3)));
        *dst = v;
      }
    }
  }
}

// largest |x − x0| (periodic in x) of [1][1] over the proteins this slab owns
__global__ void k_dd_drift(KParams P, Dev d, uint32_t* out) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  float m = 0.0f;
  if (p < P.N) {
    const int r = d.id_of[p];
    if (d.dd_own[r]) {
      double dx = d.cur.P(p, 1, 1, 0) - d.dd_x0[r];
      dx = dx - P.box_x * kmcm::round_(dx / P.box_x);
      m = (float)kmcm::fabs_(dx);
    }
  }
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_down(m, o, 64));
  if (__lane_id() == 0) atomicMax(out, __float_as_uint(m));
}

// the owned proteins whose [1][1] is more than S from its x at the window's
// set (periodic in x): {local index, x} (slabs.py checks them against the
// windows)
__global__ void k_dd_jumpers(KParams P, Dev d, double S, int cap, int32_t* ids, double* xs, uint32_t* cnt) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P.N) return;
  const int r = d.id_of[p];
  if (!d.dd_own[r]) return;
  const double x = d.cur.P(p, 1, 1, 0);
  double dx = x - d.dd_x0[r];
  dx = dx - P.box_x * kmcm::round_(dx / P.box_x);
  if (!(kmcm::fabs_(dx) > S)) return;
  const uint32_t k = atomicAdd(cnt, 1u);
  if (k < (uint32_t)cap) {
    ids[k] = r;
    xs[k] = x;
  }
}

// the same list into the step's report (kmc_dd_step; read by kmc_dd_finish),
// with the step's collision / bond counters
__global__ void k_dd_jumpers_rep(KParams P, Dev d, double S) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p == 0) {
    d.dd_rep->xcol = d.ctl->dd_xcol;
    d.dd_rep->xbond = d.ctl->dd_xbond;
  }
  if (p >= P.N) return;
  const int r = d.id_of[p];
  if (!d.dd_own[r]) return;
  const double x = d.cur.P(p, 1, 1, 0);
  double dx = x - d.dd_x0[r];
  dx = dx - P.box_x * kmcm::round_(dx / P.box_x);
  if (!(kmcm::fabs_(dx) > S)) return;
  const uint32_t k = atomicAdd((uint32_t*)&d.dd_rep->n_jump, 1u);
  if (k < DD_JCAP) {
    d.dd_rep->jump_id[k] = r;
    d.dd_rep->jump_x[k] = x;
  }
}

// Rows of the exchange (kmc_dd_pack): row i = the end-of-step state of local
// protein ids[i] — 48 doubles, then 8 ints at byte 384 with the links as
// global reference index + 1.  One thread per double / int of a row.
__global__ void k_dd_pack(KParams P, Dev d, int n, const int32_t* ids, unsigned char* rows) {
  const int NA = P.NA, NB = P.NB;
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (size_t)n * 56) return;
  const int i = (int)(t / 56), e = (int)(t % 56), slot = d.slot_of[ids[i]];
  unsigned char* row = rows + (size_t)i * KMC_DD_ROW;
  if (e < 48) {
    const int bead = e / 3, c = e % 3;
    double v = 0.0;
    if (slot < NA) v = d.cur.A(slot, bead / 4 + 1, bead % 4 + 1, c);
    else if (e < 24) v = d.cur.B(slot - NA, bead / 2 + 1, bead % 2 + 1, c);
    reinterpret_cast<double*>(row)[e] = v;
    return;
  }
  const int f = e - 48;
  int v = 0;
  bool link = false;
  if (slot < NA) {
    if (f < 5) v = d.a_int[(size_t)f * NA + slot];
    link = f == 2 || f == 4;
  } else {
    v = d.b_int[(size_t)f * NB + (slot - NA)];
    link = f >= 4;
  }
  if (link && v > 0) v = d.gid[d.id_of[v - 1]] + 1;
  reinterpret_cast<int32_t*>(row + 384)[f] = v;
}

// The owners' rows over this window's halo copies (kmc_dd_unpack): one wave
// per row, lanes 0..47 the doubles, 48..55 the ints.  A link (global index +
// 1) is found in the window by a binary search of gid (increasing); a link to
// a protein the window does not hold is cut, clearing the status it carries
// (receptor nei2 -> st2 and nei4, nei3 -> st3; ligand nei j -> st j), as the
// window was cut when it was set.  The row overwrites the window's own result;
// rows that differed are counted, and band rows that differed or had a link
// cut make the step's check fail (DDRep::bad).
__global__ __launch_bounds__(256) void k_dd_unpack(KParams P, Dev d, int n, const int32_t* ids,
                                                   const unsigned char* rows, const uint8_t* band, uint8_t* cut) {
  const int NA = P.NA, NB = P.NB, N = P.N;
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;  // a whole wave
  const int r = ids[i], slot = d.slot_of[r];
  const bool rec = slot < NA;
  const unsigned char* row = rows + (size_t)i * KMC_DD_ROW;
  bool dif = false, difi = false, lost = false;
  double* dst = nullptr;
  double v = 0.0;
  if (lane < 48) {
    const int bead = lane / 3, c = lane % 3;
    if (rec) dst = &d.cur.A(slot, bead / 4 + 1, bead % 4 + 1, c);
    else if (lane < 24) dst = &d.cur.B(slot - NA, bead / 2 + 1, bead % 2 + 1, c);
    if (dst) {
      v = reinterpret_cast<const double*>(row)[lane];
      dif = __double_as_longlong(*dst) != __double_as_longlong(v);
    }
  }
  const int f = lane - 48;
  int32_t* dsti = nullptr;
  int vi = 0;
  if (f >= 0 && f < 8) {
    bool link;
    if (rec) {
      if (f < 5) dsti = &d.a_int[(size_t)f * NA + slot];
      link = f == 2 || f == 4;
    } else {
      dsti = &d.b_int[(size_t)f * NB + (slot - NA)];
      link = f >= 4;
    }
    vi = reinterpret_cast<const int32_t*>(row + 384)[f];
    if (link && vi > 0) {
      const int g = vi - 1;
      int lo = 0, hi = N;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (d.gid[mid] < g) lo = mid + 1;
        else hi = mid;
      }
      if (lo < N && d.gid[lo] == g) {
        vi = d.slot_of[lo] + 1;
      } else {
        vi = 0;
        lost = true;
      }
    }
  }
  const uint32_t lostf = (uint32_t)(__ballot(lost) >> 48) & 0xffu;  // bit f: link field f was cut
  if (dsti) {
    if (rec) {
      if ((f == 0 || f == 3) && (lostf & (1u << 2))) vi = 0;
      if (f == 1 && (lostf & (1u << 4))) vi = 0;
    } else if (f < 4 && (lostf & (1u << (4 + f)))) {
      vi = 0;
    }
    difi = *dsti != vi;
    if (difi) *dsti = vi;
  }
  if (dif) *dst = v;
  const bool anyb = __ballot(dif) != 0, anyi = __ballot(difi) != 0;
  if (lane == 0) {
    cut[r] = lostf != 0;
    if (anyb || anyi) atomicAdd(&d.dd_rep->differed, 1);
    if (anyi) atomicAdd(&d.dd_rep->links, 1);
    if (band[r] && (anyb || anyi || lostf)) atomicAdd(&d.dd_rep->bad, 1);
  }
}

extern "C" {

static int dd_stage(kmc_sim* s, int32_t n) {
  if (n <= s->dd_cap) return KMC_OK;
  dfree(s, s->dd_ids);
  dfree(s, s->dd_beads);
  dfree(s, s->dd_ints);
  dfree(s, s->dd_flags);
  s->dd_cap = std::max<int32_t>(n, 1024);
  int rc = dalloc(s, &s->dd_ids, (size_t)s->dd_cap);
  rc |= dalloc(s, &s->dd_beads, (size_t)s->dd_cap * 48);
  rc |= dalloc(s, &s->dd_ints, (size_t)s->dd_cap * 8);
  rc |= dalloc(s, &s->dd_flags, ((size_t)s->dd_cap + 3) & ~(size_t)3);
  return rc == KMC_OK ? KMC_OK : fail(s, KMC_ERR_HIP, "dd staging buffers");
}

int kmc_dd_set_state(kmc_sim* s, const kmc_state_view* v, const int32_t* gid, const uint8_t* own,
                     const int32_t* ctl5) {
  if (!s || !v || !gid || !own || !ctl5) return KMC_ERR_ARG;
  const int NA = s->p.n_a, NB = s->p.n_b, N = NA + NB;
  // monotone local numbering, global indices in range, ownership 0 / 1
  {
    const int rc = kmch_host::dd_check(N, gid, own, &s->err);
    if (rc != KMC_OK) return rc;
  }
  if (!s->dd_gid) {
    int rc = dalloc(s, &s->dd_gid, (size_t)N);
    rc |= dalloc(s, &s->dd_own, (size_t)N);
    rc |= dalloc(s, &s->dd_x0, (size_t)N);
    rc |= dalloc(s, &s->dd_scratch, 2);
    rc |= dalloc(s, &s->dd_rep, 1);
    rc |= dalloc(s, &s->dd_band, (size_t)N);
    rc |= dalloc(s, &s->dd_cut, (size_t)N);
    if (rc != KMC_OK) return fail(s, KMC_ERR_HIP, "dd buffers");
  }
  HIPCHK(s, hipMemsetAsync(s->dd_rep, 0, sizeof(DDRep), s->stream));
  HIPCHK(s, hipMemsetAsync(s->dd_band, 0, (size_t)N, s->stream));
  HIPCHK(s, hipMemsetAsync(s->dd_cut, 0, (size_t)N, s->stream));
  HIPCHK(s, hipStreamSynchronize(s->stream));
  s->dd_n_send = s->dd_n_recv = 0;
  std::vector<double> x0((size_t)N);
  for (int i = 0; i < NA; ++i) x0[i] = v->ra[i];  // bead [1][1], x: row 0 of the host layout
  for (int b = 0; b < NB; ++b) x0[NA + b] = v->rb[b];
  HIPCHK(s, hipMemcpy(s->dd_gid, gid, sizeof(int32_t) * N, hipMemcpyHostToDevice));
  HIPCHK(s, hipMemcpy(s->dd_own, own, (size_t)N, hipMemcpyHostToDevice));
  HIPCHK(s, hipMemcpy(s->dd_x0, x0.data(), sizeof(double) * N, hipMemcpyHostToDevice));
  // a window holds its slab's units in part of the box's x range: its tiles
  // are sized from the density where the proteins are (the share of 1024 x
  // buckets holding any), not from the box's mean — at twice the mean density
  // every occupied tile would overflow the LDS staging into the dense path
  {
    std::vector<uint8_t> occ(1024, 0);
    const double L = s->p.box_x;
    for (int i = 0; i < N; ++i) {
      const double u = x0[i] - L * std::floor(x0[i] / L);
      occ[std::min(1023, std::max(0, (int)(u / L * 1024.0)))] = 1;
    }
    int n_occ = 0;
    for (uint8_t o : occ) n_occ += o;
    const double f = std::max(1, n_occ) / 1024.0;
    const int t = choose_tile((double)N * s->K.cs * s->K.cs / std::max(1.0, f * L * s->p.box_y));
    if (t != s->K.tile) {
      s->K.tile = t;
      dfree(s, s->d.tout);
      dfree(s, s->d.tout_n);
      s->ntiles = ((s->K.ncx + t - 1) / t) * ((s->K.ncy + t - 1) / t);
      if (dalloc(s, &s->d.tout, (size_t)s->ntiles * TOUT_CAP) != KMC_OK || dalloc(s, &s->d.tout_n, (size_t)s->ntiles) != KMC_OK)
        return fail(s, KMC_ERR_HIP, "dd: tile buffers");
    }
  }
  s->K.dd = 1;
  s->d.gid = s->dd_gid;
  s->d.dd_own = s->dd_own;
  s->d.dd_x0 = s->dd_x0;
  s->d.dd_rep = s->dd_rep;
  int rc = set_state_impl(s, v);
  if (rc != KMC_OK) return rc;
  // the counters' offsets and the running largest complex of this slab's
  // share (the driver gives the global ones to one slab, zero to the others)
  Ctl c;
  HIPCHK(s, hipMemcpy(&c, s->d.ctl, sizeof c, hipMemcpyDeviceToHost));
  c.off_bond = ctl5[0];
  c.off_rl = ctl5[1];
  c.off_cis = ctl5[2];
  c.off_mono = ctl5[3];
  c.maxc = ctl5[4];
  c.dd_xcol = c.dd_xbond = 0;
  HIPCHK(s, hipMemcpy(s->d.ctl, &c, sizeof c, hipMemcpyHostToDevice));
  return KMC_OK;
}

int kmc_dd_export(kmc_sim* s, int32_t n, const int32_t* ids, double* beads, int32_t* ints) {
  if (!s || n < 0 || (n > 0 && (!ids || !beads || !ints))) return KMC_ERR_ARG;
  if (!s->have_state || !s->K.dd) return fail(s, KMC_ERR_ARG, "dd: no decomposed state");
  if (n == 0) return KMC_OK;
  for (int32_t i = 0; i < n; ++i)
    if (ids[i] < 0 || ids[i] >= s->K.N) return fail(s, KMC_ERR_ARG, "dd: index out of range");
  int rc = dd_stage(s, n);
  if (rc != KMC_OK) return rc;
  HIPCHK(s, hipMemcpyAsync(s->dd_ids, ids, sizeof(int32_t) * n, hipMemcpyHostToDevice, s->stream));
  k_dd_export<<<(unsigned)(((size_t)n * 48 + 255) / 256), 256, 0, s->stream>>>(s->K, s->d, n, s->dd_ids,
                                                                            s->dd_beads, s->dd_ints);
  HIPCHK(s, hipGetLastError());
  HIPCHK(s, hipMemcpyAsync(beads, s->dd_beads, sizeof(double) * 48 * n, hipMemcpyDeviceToHost, s->stream));
  HIPCHK(s, hipMemcpyAsync(ints, s->dd_ints, sizeof(int32_t) * 8 * n, hipMemcpyDeviceToHost, s->stream));
  HIPCHK(s, hipStreamSynchronize(s->stream));
  return KMC_OK;
}

int kmc_dd_import(kmc_sim* s, int32_t n, const int32_t* ids, const double* beads, const int32_t* ints,
                  uint8_t* flags) {
  if (!s || n < 0 || (n > 0 && (!ids || !beads || !ints || !flags))) return KMC_ERR_ARG;
  if (!s->have_state || !s->K.dd) return fail(s, KMC_ERR_ARG, "dd: no decomposed state");
  if (n == 0) return KMC_OK;
  for (int32_t i = 0; i < n; ++i) {
    if (ids[i] < 0 || ids[i] >= s->K.N) return fail(s, KMC_ERR_ARG, "dd: index out of range");
    const bool rec = ids[i] < s->K.NA;
    for (int f = 0; f < 8; ++f) {
      const bool link = rec ? (f == 2 || f == 4) : f >= 4;
      if (link && (ints[(size_t)i * 8 + f] < 0 || ints[(size_t)i * 8 + f] > s->K.N))
        return fail(s, KMC_ERR_ARG, "dd: link out of range");
    }
  }
  int rc = dd_stage(s, n);
  if (rc != KMC_OK) return rc;
  HIPCHK(s, hipMemcpyAsync(s->dd_ids, ids, sizeof(int32_t) * n, hipMemcpyHostToDevice, s->stream));
  HIPCHK(s, hipMemcpyAsync(s->dd_beads, beads, sizeof(double) * 48 * n, hipMemcpyHostToDevice, s->stream));
  HIPCHK(s, hipMemcpyAsync(s->dd_ints, ints, sizeof(int32_t) * 8 * n, hipMemcpyHostToDevice, s->stream));
  HIPCHK(s, hipMemsetAsync(s->dd_flags, 0, ((size_t)n + 3) & ~(size_t)3, s->stream));
  k_dd_import<<<(unsigned)(((size_t)n * 48 + 255) / 256), 256, 0, s->stream>>>(s->K, s->d, n, s->dd_ids,
                                                                            s->dd_beads, s->dd_ints, s->dd_flags);
  HIPCHK(s, hipGetLastError());
  HIPCHK(s, hipMemcpyAsync(flags, s->dd_flags, (size_t)n, hipMemcpyDeviceToHost, s->stream));
  HIPCHK(s, hipStreamSynchronize(s->stream));
  bool links = false;
  for (int32_t i = 0; i < n; ++i) links |= (flags[i] & 2) != 0;
  // the chunk snapshot no longer describes this state (a replay from it would
  // miss the import); kept complexes are rebuilt when a bond of a halo
  // protein differed
  s->snap_valid = false;
  if (links) s->need_full = true;
  s->clusters_valid = false;
  return KMC_OK;
}

int kmc_dd_drift(kmc_sim* s, double* max_dx) {
  if (!s || !max_dx) return KMC_ERR_ARG;
  if (!s->have_state || !s->K.dd) return fail(s, KMC_ERR_ARG, "dd: no decomposed state");
  HIPCHK(s, hipMemsetAsync(s->dd_scratch, 0, sizeof(uint32_t), s->stream));
  k_dd_drift<<<(s->K.N + 255) / 256, 256, 0, s->stream>>>(s->K, s->d, s->dd_scratch);
  HIPCHK(s, hipGetLastError());
  uint32_t bits = 0;
  HIPCHK(s, hipMemcpyAsync(&bits, s->dd_scratch, sizeof bits, hipMemcpyDeviceToHost, s->stream));
  HIPCHK(s, hipStreamSynchronize(s->stream));
  float f;
  std::memcpy(&f, &bits, sizeof f);
  *max_dx = f;
  return KMC_OK;
}

int kmc_dd_jumpers(kmc_sim* s, double S, int32_t cap, int32_t* ids, double* xs, int32_t* n) {
  if (!s || cap < 0 || !n || (cap > 0 && (!ids || !xs))) return KMC_ERR_ARG;
  if (!s->have_state || !s->K.dd) return fail(s, KMC_ERR_ARG, "dd: no decomposed state");
  int rc = dd_stage(s, cap);
  if (rc != KMC_OK) return rc;
  HIPCHK(s, hipMemsetAsync(s->dd_scratch + 1, 0, sizeof(uint32_t), s->stream));
  k_dd_jumpers<<<(s->K.N + 255) / 256, 256, 0, s->stream>>>(s->K, s->d, S, cap, s->dd_ids, s->dd_beads,
                                                           s->dd_scratch + 1);
  HIPCHK(s, hipGetLastError());
  uint32_t cnt = 0;
  HIPCHK(s, hipMemcpyAsync(&cnt, s->dd_scratch + 1, sizeof cnt, hipMemcpyDeviceToHost, s->stream));
  HIPCHK(s, hipStreamSynchronize(s->stream));
  const int32_t m = (int32_t)std::min<uint32_t>(cnt, (uint32_t)cap);
  if (m > 0) {
    HIPCHK(s, hipMemcpyAsync(ids, s->dd_ids, sizeof(int32_t) * m, hipMemcpyDeviceToHost, s->stream));
    HIPCHK(s, hipMemcpyAsync(xs, s->dd_beads, sizeof(double) * m, hipMemcpyDeviceToHost, s->stream));
    HIPCHK(s, hipStreamSynchronize(s->stream));
  }
  *n = (int32_t)cnt;  // may exceed cap: the caller asks again with room for all
  return KMC_OK;
}

// ---- the device-resident exchange
static bool dd_ready(kmc_sim* s) { return s && s->have_state && s->K.dd && s->dd_rep; }

int kmc_dd_plan(kmc_sim* s, int32_t n_send, const int32_t* send_ids, int32_t n_recv, const int32_t* recv_ids,
                const uint8_t* own, const uint8_t* band) {
  if (!s || n_send < 0 || n_recv < 0 || !own || !band || (n_send > 0 && !send_ids) || (n_recv > 0 && !recv_ids))
    return KMC_ERR_ARG;
  if (!dd_ready(s)) return fail(s, KMC_ERR_ARG, "dd: no decomposed state");
  const int N = s->K.N;
  for (int i = 0; i < N; ++i)
    if (own[i] > 1 || band[i] > 1 || (own[i] && band[i])) return fail(s, KMC_ERR_ARG, "dd: own / band flags");
  for (int32_t i = 0; i < n_send; ++i)
    if (send_ids[i] < 0 || send_ids[i] >= N || !own[send_ids[i]])
      return fail(s, KMC_ERR_ARG, "dd: a sent protein out of range or not owned");
  for (int32_t i = 0; i < n_recv; ++i)
    if (recv_ids[i] < 0 || recv_ids[i] >= N || own[recv_ids[i]])
      return fail(s, KMC_ERR_ARG, "dd: a received protein out of range or owned");
  if (n_send > s->dd_send_cap) {
    dfree(s, s->dd_send_ids);
    dfree(s, s->dd_sendbuf);
    s->dd_send_cap = std::max<int32_t>(n_send + n_send / 4, 1024);
    int rc = dalloc(s, &s->dd_send_ids, (size_t)s->dd_send_cap);
    rc |= dalloc(s, &s->dd_sendbuf, (size_t)s->dd_send_cap * KMC_DD_ROW);
    if (rc != KMC_OK) return fail(s, KMC_ERR_HIP, "dd: send buffers");
  }
  if (n_recv > s->dd_recv_cap) {
    dfree(s, s->dd_recv_ids);
    s->dd_recv_cap = std::max<int32_t>(n_recv + n_recv / 4, 1024);
    if (dalloc(s, &s->dd_recv_ids, (size_t)s->dd_recv_cap) != KMC_OK) return fail(s, KMC_ERR_HIP, "dd: receive ids");
  }
  if (n_send) HIPCHK(s, hipMemcpyAsync(s->dd_send_ids, send_ids, sizeof(int32_t) * n_send, hipMemcpyHostToDevice, s->stream));
  if (n_recv) HIPCHK(s, hipMemcpyAsync(s->dd_recv_ids, recv_ids, sizeof(int32_t) * n_recv, hipMemcpyHostToDevice, s->stream));
  HIPCHK(s, hipMemcpyAsync(s->dd_own, own, (size_t)N, hipMemcpyHostToDevice, s->stream));
  HIPCHK(s, hipMemcpyAsync(s->dd_band, band, (size_t)N, hipMemcpyHostToDevice, s->stream));
  HIPCHK(s, hipStreamSynchronize(s->stream));
  s->dd_n_send = n_send;
  s->dd_n_recv = n_recv;
  return KMC_OK;
}

void* kmc_dd_send_buffer(kmc_sim* s) { return s ? (void*)s->dd_sendbuf : nullptr; }

int kmc_dd_pack(kmc_sim* s, void* dst) {
  if (!dd_ready(s)) return s ? fail(s, KMC_ERR_ARG, "dd: no decomposed state") : KMC_ERR_ARG;
  unsigned char* out = dst ? (unsigned char*)dst : s->dd_sendbuf;
  const int32_t n = s->dd_n_send;
  if (n > 0) {
    k_dd_pack<<<(unsigned)(((size_t)n * 56 + 255) / 256), 256, 0, s->stream>>>(s->K, s->d, n, s->dd_send_ids, out);
    HIPCHK(s, hipGetLastError());
  }
  HIPCHK(s, hipStreamSynchronize(s->stream));
  return KMC_OK;
}

int kmc_dd_unpack(kmc_sim* s, const void* src, int32_t first, int32_t n) {
  if (!dd_ready(s)) return s ? fail(s, KMC_ERR_ARG, "dd: no decomposed state") : KMC_ERR_ARG;
  if (first < 0 || n < 0 || (int64_t)first + n > s->dd_n_recv || (n > 0 && !src))
    return fail(s, KMC_ERR_ARG, "dd: unpack range outside the receive plan");
  if (n == 0) return KMC_OK;
  k_dd_unpack<<<(unsigned)((n + 3) / 4), 256, 0, s->stream>>>(s->K, s->d, n, s->dd_recv_ids + first,
                                                              (const unsigned char*)src, s->dd_band, s->dd_cut);
  HIPCHK(s, hipGetLastError());
  return KMC_OK;
}

// (run_chunk, a kmc_dd_step's chunk) the plan's rows into the pack
// destination and the jumpers into the report, on the stream after the step
static int dd_after_step(kmc_sim* s) {
  const int32_t n = s->dd_n_send;
  if (n > 0)
    k_dd_pack<<<(unsigned)(((size_t)n * 56 + 255) / 256), 256, 0, s->stream>>>(s->K, s->d, n, s->dd_send_ids,
                                                                              s->dd_step_dst);
  k_dd_jumpers_rep<<<(s->K.N + 255) / 256, 256, 0, s->stream>>>(s->K, s->d, s->dd_step_S);
  HIPCHK(s, hipGetLastError());
  return KMC_OK;
}

int kmc_dd_step(kmc_sim* s, void* dst, double S, kmc_obs* out) {
  if (!dd_ready(s)) return s ? fail(s, KMC_ERR_ARG, "dd: no decomposed state") : KMC_ERR_ARG;
  s->dd_step_pending = true;
  s->dd_step_dst = dst ? (unsigned char*)dst : s->dd_sendbuf;
  s->dd_step_S = S;
  const int rc = kmc_step(s, 1, out);
  s->dd_step_pending = false;
  return rc;
}

int kmc_dd_finish(kmc_sim* s, kmc_dd_report* out) {
  static_assert(sizeof(DDRep) == sizeof(kmc_dd_report), "kmc_dd_report layout");
  if (!out) return KMC_ERR_ARG;
  if (!dd_ready(s)) return s ? fail(s, KMC_ERR_ARG, "dd: no decomposed state") : KMC_ERR_ARG;
  HIPCHK(s, hipMemcpyAsync(out, s->dd_rep, sizeof(DDRep), hipMemcpyDeviceToHost, s->stream));
  // the step's counts and lists start again at zero (the entries are
  // overwritten before they are read)
  HIPCHK(s, hipMemsetAsync(&s->dd_rep->bad, 0, offsetof(DDRep, jump_id) - offsetof(DDRep, bad), s->stream));
  HIPCHK(s, hipStreamSynchronize(s->stream));
  // a halo protein's bonds changed under the kept complexes: register them anew
  if (out->links) s->need_full = true;
  s->clusters_valid = false;
  return KMC_OK;
}

int kmc_dd_cut_count(kmc_sim* s, int32_t n, const int32_t* ids, int32_t* count) {
  if (!count || n < 0 || (n > 0 && !ids)) return KMC_ERR_ARG;
  if (!dd_ready(s)) return s ? fail(s, KMC_ERR_ARG, "dd: no decomposed state") : KMC_ERR_ARG;
  const int N = s->K.N;
  for (int32_t i = 0; i < n; ++i)
    if (ids[i] < 0 || ids[i] >= N) return fail(s, KMC_ERR_ARG, "dd: index out of range");
  std::vector<uint8_t> cut((size_t)N);
  HIPCHK(s, hipMemcpyAsync(cut.data(), s->dd_cut, (size_t)N, hipMemcpyDeviceToHost, s->stream));
  HIPCHK(s, hipStreamSynchronize(s->stream));
  int32_t c = 0;
  for (int32_t i = 0; i < n; ++i) c += cut[ids[i]] != 0;
  *count = c;
  return KMC_OK;
}

int kmc_list_growth(const kmc_sim* s) { return s ? s->grow : KMC_ERR_ARG; }

int kmc_set_list_growth(kmc_sim* s, int32_t level) {
  if (!s || level < -16 || level > 6) return KMC_ERR_ARG;
  if (level == s->grow) return KMC_OK;
  HIPCHK(s, hipStreamSynchronize(s->stream));
  s->grow = level;
  if (alloc_lists(s) != KMC_OK) return fail(s, KMC_ERR_HIP, "resizing the output lists failed");
  return KMC_OK;
}

int kmc_dd_counters(kmc_sim* s, int64_t* out) {
  if (!s || !out) return KMC_ERR_ARG;
  HIPCHK(s, hipStreamSynchronize(s->stream));
  Ctl c;
  HIPCHK(s, hipMemcpy(&c, s->d.ctl, sizeof c, hipMemcpyDeviceToHost));
  out[0] = c.dd_xcol;
  out[1] = c.dd_xbond;
  return KMC_OK;
}

}  // extern "C"
