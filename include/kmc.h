/* kmc.h — C-ABI of libkmc, the MI355X (gfx950) engine for the per-timestep
 * KMC diffusion–reaction loop of xiaopuren/KMC-with-a-diffusion-reaction-
 * algorithm.
 *
 * The reference has no plugin/FFI surface: its "interface"
 * is the set of global arrays main() mutates (main.cpp:102-168) and the
 * process/file contract (position.cpt in, bond.dat/position.cpt out,
 * main.cpp:226-270, 2206-2253).  This header is the drop-in boundary a host
 * program binds instead: plain pointers and sizes, no torch types, int return
 * codes (0 = ok, < 0 = error; kmc_last_error() has the message).  One handle
 * per GPU; a handle is used by one host thread at a time.
 *
 * Indices inside state buffers follow the reference exactly: proteins are
 * 1-based, receptors ("protein_A") are 1..n_a, ligands ("protein_B") are
 * n_a+1..n_a+n_b, and 0 means "no neighbour" (main.cpp:117, 1926-1928).
 */
#ifndef KMC_H
#define KMC_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KMC_OK 0
#define KMC_ERR_ARG (-1)       /* bad argument / size mismatch */
#define KMC_ERR_IO (-2)        /* file could not be opened or written */
#define KMC_ERR_FORMAT (-3)    /* malformed position.cpt */
#define KMC_ERR_STATE (-4)     /* bond links inconsistent (status vs res_nei) */
#define KMC_ERR_PLACEMENT (-5) /* random placement exhausted its attempts */
#define KMC_ERR_CAPACITY (-6)  /* a fixed device capacity was exceeded */
#define KMC_ERR_HIP (-7)       /* HIP runtime error */
#define KMC_ERR_GEOMETRY (-8)  /* a rigid body left the cell-list extent bound */
#define KMC_ERR_NODEVICE (-9)  /* no gfx950 device / kernels not loaded */

/* Physics + run parameters.  Defaults (kmc_params_default) equal the
 * reference globals at main.cpp:39-99. */
typedef struct kmc_params {
  int32_t n_a;               /* protein_A_tot_num (main.cpp:48) */
  int32_t n_b;               /* protein_B_tot_num (main.cpp:57) */
  double time_step;          /* ns (main.cpp:40) */
  double box_x, box_y, box_z;/* cell_range_x/y/z (main.cpp:43-45) */
  double pai;                /* 3.1415926 (main.cpp:71) */
  double ra_radius, ra_D, ra_rot_D;      /* main.cpp:72-74 */
  double rb_radius, rb_D, rb_rot_D;      /* main.cpp:76-78 */
  double mono_cis_ass_rate, mono_cis_diss_rate;           /* main.cpp:80-81 */
  double cis_D, cis_rot_D, cis_ass_rate, cis_diss_rate;   /* main.cpp:83-86 */
  double bond_D, bond_rot_D, ass_rate, diss_rate;         /* main.cpp:88-91 */
  double bond_dist_cutoff;   /* 18  (main.cpp:93) */
  double bond_thetapd_cutoff;/* 45  (main.cpp:95) */
  double bond_thetaot_cutoff;/* 90  (main.cpp:97) */
  double cis_thetaot_cutoff; /* 10  (main.cpp:98) */
  double cis_dist_cutoff;    /* 15  (main.cpp:99) */
  int64_t simu_step;         /* last step of a full run (main.cpp:39) */
  int32_t out_interval;      /* checkpoint / bond.dat cadence, 5000 (main.cpp:2206) */
  int32_t reserved0;
  uint64_t seed;             /* Philox key (replaces the clock seed of rand2) */
  uint32_t replica;          /* independent trajectory id (ensembles) */
  int32_t reserved1;
} kmc_params;

/* One record per simulated step: the bond.dat columns (main.cpp:2251) plus
 * the raw cluster sums they come from. */
typedef struct kmc_obs {
  int64_t step;                 /* mc_time_step */
  double t;                     /* mc_time_step * time_step */
  int32_t bond_num_rl;
  int32_t bond_num_mono_cis;
  int32_t bond_num_cis;
  int32_t bond_num;
  double cluster_size;          /* tot_proteins_in_cluster / tot_cluster_num */
  int32_t protein_num_in_max_complex;
  int32_t tot_proteins_in_cluster;
  int32_t tot_cluster_num;
  int32_t reserved;
} kmc_obs;

/* Host-side state buffers (caller-owned), structure-of-arrays, fp64.
 *   ra  : 48 * n_a doubles, ra[(((j-1)*4 + (k-1))*3 + c) * n_a + (i-1)]
 *         = R_{x,y,z}[i][j][k] of receptor i (j,k = 1..4; c = 0,1,2 → x,y,z)
 *   rb  : 24 * n_b doubles, rb[(((j-1)*2 + (k-1))*3 + c) * n_b + (b-1)]
 *         = R_{x,y,z}[n_a+b][j][k] of ligand b (j = 1..4, k = 1..2)
 *   a_int: 5 * n_a int32 in checkpoint order: protein_status[i][2],
 *         protein_status[i][3], res_nei[i][2], res_nei[i][4], res_nei[i][3]
 *         (a_int[f * n_a + (i-1)], main.cpp:240-244)
 *   b_int: 8 * n_b int32: protein_status[.][1..4] then res_nei[.][1..4]
 *   counters: bond_num, bond_num_rl, bond_num_cis, bond_num_mono_cis,
 *         protein_num_in_Max_Complex (main.cpp:261-265)
 *   step: the last completed mc_time_step (0 for a fresh configuration). */
typedef struct kmc_state_view {
  double* ra;
  double* rb;
  int32_t* a_int;
  int32_t* b_int;
  int32_t counters[5];
  int32_t reserved;
  int64_t step;
} kmc_state_view;

typedef struct kmc_sim kmc_sim;

/* Reference defaults (main.cpp:39-99); out_interval 5000, seed 1, replica 0. */
void kmc_params_default(kmc_params* p);

/* Create a simulation on HIP device `device` (-1 = current). */
int kmc_create(const kmc_params* p, int device, kmc_sim** out);
int kmc_destroy(kmc_sim* s);
const char* kmc_last_error(const kmc_sim* s);

/* Random initial configuration with the reference's placement rules
 * (main.cpp:281-447: rejection of overlapping receptors / ligands, random
 * orientations), drawn from the keyed RNG; O(N) with a hash grid, so it also
 * serves the 1e6–1e7-particle configurations the reference's O(N^2) goto
 * sampler cannot reach.  Resets counters and sets step = 0. */
int kmc_init_random(kmc_sim* s);

/* position.cpt reader / writer, byte-compatible with main.cpp:226-270 and
 * main.cpp:2206-2244.  After a load the next simulated step is saved+1
 * (main.cpp:267). */
int kmc_load_cpt(kmc_sim* s, const char* path);
int kmc_write_cpt(kmc_sim* s, const char* path);

/* Exact checkpoint: the full-precision state, counters,
 * step, seed and replica in a binary file (KMCSTAT1 layout, FNV-1a trailer).
 * With the keyed random streams a load continues the trajectory bit for bit;
 * a file of another size, seed or replica is refused (KMC_ERR_ARG), a corrupt
 * one gives KMC_ERR_FORMAT.  position.cpt (3 decimals) cannot do this
 * (main.cpp:2208-2209). */
int kmc_save_state(kmc_sim* s, const char* path);
int kmc_load_state(kmc_sim* s, const char* path);

/* Copy the state in / out of the device (host buffers sized as above). */
int kmc_set_state(kmc_sim* s, const kmc_state_view* v);
int kmc_get_state(kmc_sim* s, kmc_state_view* v);

/* Advance nsteps time steps of the diffusion–reaction loop (main.cpp:461-2308)
 * on the GPU.  `out` (may be NULL) receives nsteps records. */
int kmc_step(kmc_sim* s, int64_t nsteps, kmc_obs* out);

/* Last completed step number. */
int64_t kmc_current_step(const kmc_sim* s);

/* Per-kernel device time, measured with HIP events on the handle's stream:
 * kmc_set_timing(s, mask) brackets the launches of the kernels whose id bit
 * is set (ids: kmc_kernel_name(0..n-1); 0 disables and resets; returns 0),
 * kmc_set_timing_period(s, every) brackets them only in every `every`-th step
 * (default 1: every step; an event pair costs a few microseconds of queue
 * time), and kmc_kernel_times returns the accumulated milliseconds and
 * launch counts since set_timing (returns the number of kernel ids).  Used
 * by bench.py for the roofline of the dominant kernel. */
int kmc_set_timing(kmc_sim* s, uint64_t kernel_mask);
int kmc_set_timing_period(kmc_sim* s, int32_t every);
int kmc_kernel_times(const kmc_sim* s, double* total_ms, int64_t* launches, int32_t n);
const char* kmc_kernel_name(int32_t id);

/* BFS member rows of the last simulated step (results[i][.] of main.cpp:537,
 * after the multi-ligand shuffles): for each ligand b, row_len[b] members
 * (reference 1-based indices) are appended to `members` (n_a+n_b capacity);
 * non-root ligands have row_len 0.  Feeds cluster.log (main.cpp:2291-2305).
 * KMC_ERR_ARG before the first step after a state was set, and after a
 * kmc_step that failed without keeping a step (the rows would not describe
 * the current state). */
int kmc_get_clusters(kmc_sim* s, int32_t* row_len, int32_t* members);

/* Formatting helpers shared by every host driver.  Each returns the number of
 * characters written (excluding NUL) or < 0. */
int kmc_format_bond_line(const kmc_params* p, const kmc_obs* o, char* buf, size_t n);   /* main.cpp:2251 */

/* FNV-1a-64 hash of a host state view in reference order (beads x,y,z as
 * IEEE bits, then the ints, then counters and step): the per-step parity
 * fingerprint shared by the oracle, the reference trace and the GPU tests. */
uint64_t kmc_state_hash(const kmc_params* p, const kmc_state_view* v);

/* Host-only helpers (no device needed): the same formats and generator as
 * above on caller-owned host buffers. */
const char* kmc_host_last_error(void);
int kmc_host_load_cpt(const kmc_params* p, const char* path, kmc_state_view* v);
int kmc_host_write_cpt(const kmc_params* p, const kmc_state_view* v, const char* path);
int kmc_host_init_random(const kmc_params* p, kmc_state_view* v);
int kmc_host_save_state(const kmc_params* p, const kmc_state_view* v, const char* path);
int kmc_host_load_state(const kmc_params* p, const char* path, kmc_state_view* v);
/* parameter.log (main.cpp:178-205), test.gro frame (2258-2287, appended),
 * cluster.log block (2291-2305, appended) */
int kmc_host_write_parameter_log(const kmc_params* p, const char* path);
int kmc_host_append_gro(const kmc_params* p, const kmc_state_view* v, const char* path);
int kmc_host_append_cluster_log(const kmc_params* p, int64_t step, const int32_t* row_len, const int32_t* members,
                                const char* path);
/* bond-link consistency + rigid-body extent bound; KMC_OK or an error code */
int kmc_host_validate(const kmc_params* p, const kmc_state_view* v);
/* the arguments kmc_dd_set_state checks first: gid[0..n) increasing and in
 * [0, INT32_MAX), own[i] 0 or 1; KMC_OK or KMC_ERR_ARG */
int kmc_host_dd_check(int32_t n, const int32_t* gid, const uint8_t* own);

/* Domain decomposition of ONE trajectory over several handles (SURVEY.md
 * §8(f).4; the host driver is slabs.py).  The reference has no
 * counterpart: its step is one sequential loop (main.cpp:577, 1877-2058).
 * A handle created for the n_a + n_b proteins of one slab's window (the
 * proteins its slab owns plus halo copies of its neighbours') simulates the
 * window with the trajectory's own random streams:
 *   kmc_dd_set_state  the window in local numbering (receptors, then ligands,
 *                     each increasing in the global index gid[]: every order
 *                     the step takes is then the global one), own[i] = 1 for
 *                     the proteins this slab owns (the observables count only
 *                     those; a cis pair at its lower-index member), ctl5 =
 *                     the counters' offsets (bond, rl, cis, mono_cis) and the
 *                     running largest complex of this slab's share.
 *   kmc_dd_export     the end-of-step state of local proteins ids[0..n):
 *                     beads[n][48] (kmc_state_view bead order; a ligand uses
 *                     the first 24) and ints[n][8] (receptor st2 st3 nei2
 *                     nei4 nei3, ligand st1..4 nei1..4; links = local index+1).
 *   kmc_dd_import     the owners' end-of-step state of halo proteins, same
 *                     layout; flags[i] |= 1 where a coordinate differed from
 *                     this handle's own result, 2 where a status / link did.
 *   kmc_dd_drift      the largest periodic x displacement of an owned
 *                     protein since kmc_dd_set_state.
 *   kmc_dd_jumpers    the owned proteins displaced more than S since then:
 *                     *n of them (may exceed cap), the first cap as (local
 *                     index, x of bead [1][1]).
 *   kmc_dd_counters   out[0] collisions between an owned and a halo unit,
 *                     out[1] bonds formed between an owned and a halo protein,
 *                     both since kmc_dd_set_state. */
int kmc_dd_set_state(kmc_sim* s, const kmc_state_view* v, const int32_t* gid, const uint8_t* own,
                     const int32_t* ctl5);
int kmc_dd_export(kmc_sim* s, int32_t n, const int32_t* ids, double* beads, int32_t* ints);
int kmc_dd_import(kmc_sim* s, int32_t n, const int32_t* ids, const double* beads, const int32_t* ints,
                  uint8_t* flags);
int kmc_dd_drift(kmc_sim* s, double* max_dx);
int kmc_dd_jumpers(kmc_sim* s, double S, int32_t cap, int32_t* ids, double* xs, int32_t* n);
int kmc_dd_counters(kmc_sim* s, int64_t* out);

/* The halo exchange on device memory (the per-step path of slabs.py; the
 * host-buffer export / import above stay for diagnostics).  One exchanged
 * row is KMC_DD_ROW bytes: 48 doubles (kmc_dd_export's bead order) then 8
 * int32 (kmc_dd_export's fields) whose links are GLOBAL reference index + 1
 * (0 = none), so a row means the same thing in every window.
 *   kmc_dd_plan    once per partition (and after an ownership change):
 *                  send_ids[n_send] the local ids whose rows this window
 *                  sends, grouped by destination; recv_ids[n_recv] the local
 *                  ids of the rows it receives, grouped by source, each group
 *                  in its source's send order; own[N] replaces the ownership
 *                  of kmc_dd_set_state; band[N] = 1 for the halo proteins
 *                  whose end-of-step state must equal their owner's.  Sent
 *                  proteins must be owned, received ones not.
 *   kmc_dd_step    one step of the window (kmc_step) that also packs the
 *                  end-of-step rows of send_ids into device memory dst
 *                  (n_send rows; NULL: the handle's own send buffer,
 *                  kmc_dd_send_buffer) and lists the owned proteins more
 *                  than S (periodic x) from their x at kmc_dd_set_state —
 *                  all before the step's one wait.
 *   kmc_dd_pack    the rows alone, likewise (returns after the stream drained).
 *   kmc_dd_unpack  rows [first, first + n) of the receive plan from device
 *                  memory src (another handle's send buffer on this device,
 *                  or a collective's receive buffer), enqueued on the
 *                  handle's stream: each row's links go through a binary
 *                  search of the window's global indices; a link to a
 *                  protein the window does not hold is cut with its status;
 *                  the row overwrites this handle's own result and the
 *                  differences are counted.
 *   kmc_dd_finish  waits for the unpacks and returns the step's report: band
 *                  rows that differed or had a link cut (bad; > 0 means the
 *                  step must be redone from a wider partition), rows that
 *                  differed, rows whose status / links differed; kmc_dd_step's
 *                  jumpers (n_jump, the first KMC_DD_JCAP listed as local id
 *                  + x); the bonds formed since the last finish between an
 *                  owned and a halo protein (n_xb, the first KMC_DD_XCAP as
 *                  local id pairs); kmc_dd_counters' values.
 *   kmc_dd_cut_count  how many of ids[n] had a link cut at the last unpack
 *                  (their unit is not held whole by this window).
 * A decomposed window takes no chunk snapshot (the slab driver keeps the
 * checkpoint): a kmc_step that raises a device error leaves the window's
 * state undefined and returns the error; after a list overflow
 * (KMC_ERR_CAPACITY) the lists have already been doubled —
 * kmc_list_growth / kmc_set_list_growth carry that size to the handle the
 * driver rebuilds. */
#define KMC_DD_ROW 416
#define KMC_DD_JCAP 256
#define KMC_DD_XCAP 64
typedef struct kmc_dd_report {
  int64_t xcol, xbond;
  int32_t bad, differed, links, n_jump, n_xb, reserved;
  int32_t jump_id[KMC_DD_JCAP];
  double jump_x[KMC_DD_JCAP];
  int32_t xb[KMC_DD_XCAP][2];
} kmc_dd_report;
int kmc_dd_plan(kmc_sim* s, int32_t n_send, const int32_t* send_ids, int32_t n_recv, const int32_t* recv_ids,
                const uint8_t* own, const uint8_t* band);
int kmc_dd_step(kmc_sim* s, void* dst, double S, kmc_obs* out);
int kmc_dd_pack(kmc_sim* s, void* dst);
void* kmc_dd_send_buffer(kmc_sim* s);
int kmc_dd_unpack(kmc_sim* s, const void* src, int32_t first, int32_t n);
int kmc_dd_finish(kmc_sim* s, kmc_dd_report* out);
int kmc_dd_cut_count(kmc_sim* s, int32_t n, const int32_t* ids, int32_t* count);

/* Output-list capacities as 2^level times their defaults (kmc_step doubles
 * them itself after an overflow, up to level 6). */
int kmc_list_growth(const kmc_sim* s);
int kmc_set_list_growth(kmc_sim* s, int32_t level);

/* Diagnostics: the portable math of kmc_math.h evaluated on the host and on
 * the device (op 0 sin, 1 cos, 2 atan2(x,y), 3 acos, 4 sqrt, 5 x/y, 6 round)
 * — the GPU numerics test compares the two bit for bit. */
int kmc_host_math(int op, const double* x, const double* y, double* out, int64_t n);
int kmc_device_math(int op, const double* x, const double* y, double* out, int64_t n);

#ifdef __cplusplus
}
#endif
#endif /* KMC_H */
