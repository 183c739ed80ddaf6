// kmc_device.h — device-side data layout and geometry primitives of the HIP
// engine (gfx950).  Every arithmetic expression follows the reference's
// operation order (main.cpp line cited at each helper) so that, compiled with
// -ffp-contract=off, results are bit-identical to the sequential oracle.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kmc_math.h"
#include "kmc_philox.h"

namespace kmcd {

// ---------------------------------------------------------------- constants
// Derived parameters, computed once on the host with the same expressions as
// the reference (e.g. 2*sqrt(RB_A_D*time_step/6), main.cpp:585) and passed by
// value as a kernel argument.
struct KParams {
  int NA, NB, N;
  int ncx, ncy;         // collision cell grid (xy), cs = 130 Å
  double gx0, gy0, cs;  // grid origin and cell size
  double box_x, box_y, box_z, pai;
  double ra, rb;
  double amp_a, amp_b, amp_cis, amp_bond;  // 2*sqrt(D*dt/6)
  double rot_a, rot_b, rot_cis, rot_bond;  // sqrt(rotD*dt)
  double p_ass, p_mono, p_cis, p_diss, p_mdiss, p_cdiss;  // rate*dt
  double bond_cut, cis_cut, thetapd_cut, thetaot_cut, cis_theta_cut;
  // exact squared-distance thresholds: sqrt(s) < c  <=>  s < T(c)
  double T_aa, T_ab, T_bb, T_bond, T_cis;
  // k_col_exact's refinement from the records (col_refine): squared float distances below which a
  // ligand pair (2RB) / ligand–receptor pair (RA + RB + 0.3 Å) may collide, + 2.5 Å for the rounding
  float ref_bb, ref_ab;
  int col_refine;  // 1 (default; KMC_COL_REFINE=0 turns it off: the same results, more fp64 gathers)
  // the R–L reaction tests' refinement from the records (rxn_refine): squared float distance below which a
  // ligand site may lie within bond_cut of the receptor's site (+ 3 Å for the records' rounding); on unless
  // KMC_RXN_REFINE=0 or a set state's binding sites are not where the templates put them (sites_ok)
  float ref_rl;
  int rxn_refine;
  kmcr::Key key;
  int tcap;  // LDS tile record capacity (<= TCAP; lowered only to test the global path)
  int tile;  // cells per tile side of the LDS scans (<= TILE_MAX)
  int dbg_stage;  // debug timing only: stop the tile scans after stage 1 (load) / 2 (items); 0 = off
  int tout_cap;   // per-tile outlier bucket capacity (<= TOUT_CAP; lowered only by KMC_DEBUG_TOUT_CAP)
  int cx_serial;  // debug: complexes aligned by one lane (KMC_CX_SERIAL=1) instead of the whole wave
  uint32_t cx_limit;  // members[] cursor above which k_finalize latches a full complex rebuild (mcap / 2;
                      // lowered only by KMC_DEBUG_CX_LIMIT to exercise the rebuild)
  int htag_max;   // tile home entries tagged for the direct lookup (<= HTAG_MAX; lowered only by KMC_DEBUG_HTAG)
  int dbg_recs;   // debug (KMC_DEBUG_RECS=1): every record stamped with its step and checked before the pair scan
  int dbg_cand;   // diagnostics (KMC_DEBUG_CAND=1): candidate / reaction-pair outcome counts (Ctl::cand_kind)
  int dd;         // 1: this handle simulates one slab's window of a decomposed trajectory (kmc_dd_set_state):
                  // random streams keyed by the global reference index (Dev::gid), observables over the
                  // proteins this slab owns (Dev::dd_own); 0: the whole trajectory
};

// per-step control block in device memory (replayable without host writes)
struct Ctl {
  uint32_t step;          // mc_time_step being simulated
  uint32_t obs_idx;       // record index within the current kmc_step call
  uint32_t err;           // error bits (ERR_*)
  uint32_t err_step;      // first step whose kernels raised an error bit (k_finalize), 0 = none
  uint32_t err_first;     // the error bits raised by that step (its cause; later bits may be consequences)
  // per-step work-list counters
  uint32_t n_overflow;    // ligands whose BFS overflowed the register queue
  uint32_t cx_cursor;     // members[] allocation cursor (rows are kept across steps; k_cx_kill resets)
  uint32_t n_pend;        // units still pending after a round (pass C)
  uint32_t n_pqu, n_pqe;  // compacted pending units / conflict entries for the later rounds
  uint32_t n_cx;          // complexes registered by the BFS this step (cx_list)
  uint32_t n_heavy;       // entries of cx_heavy this step
  uint32_t full_now;      // k_cx_kill: no complex kept this step (every bonded ligand runs the BFS)
  uint32_t n_dirty[2];    // proteins whose bonds changed during step s: list s & 1
  uint32_t last[8];       // previous step's work counts (diagnostics): cand conf plist rej pairs rl cisc overflow
  uint32_t n_rl;          // R–L accepting edges
  uint32_t n_cisc;        // cis candidates
  uint32_t n_outl;        // records listed on the outlier list this step (more than a cell from home)
  uint32_t n_dense;       // blocks on the dense list this step (k_pair_scan -> k_col_exact)
  // observable bookkeeping (the per-step counts are reduced by k_finalize)
  int32_t off_bond, off_rl, off_cis, off_mono;  // counters − derived at load
  int32_t maxc;                                 // protein_num_in_Max_Complex
  uint32_t n_forced;      // diagnostics: full complex rebuilds k_finalize made (members[] half full, or a
                          // dirty list overflowed) since the state was set
  uint32_t last_outl;     // diagnostics: the previous step's outlier records (n_outl)
  uint32_t cand_kind[6];  // diagnostics (KMC_DEBUG_CAND) since the state was set: collision candidates
                          // of kind pair A-A, A-B, B-B (proposal kind + other kind), tested / colliding
  uint32_t rxn_kind[5];   // diagnostics (KMC_DEBUG_CAND): reaction pairs tested, final-final, within the
                          // first distance gate, accepting; R–L site tests the record refinement ruled out
  uint64_t vtag;          // BFS tag counter for the overflow path
  uint64_t stamps[24];    // diagnostic build (-DKMC_STAMPS) only: phase cycles (tile scans, complexes)
  // decomposed trajectories (KParams::dd), since kmc_dd_set_state: collisions found between a unit this
  // slab owns and a unit it holds as a halo copy; bonds formed between an owned and a halo protein
  uint32_t dd_xcol, dd_xbond;
};

// One slab window's per-step exchange report (kmc_dd_finish; the layout of
// kmc_dd_report in include/kmc.h): the unpacks count the checks, k_dd_jumpers
// lists the jumpers, the matching lists the cross-slab bonds.  xcol / xbond
// are filled on the host from Ctl.
#define DD_JCAP 256
#define DD_XCAP 64
struct DDRep {
  int64_t xcol, xbond;
  int32_t bad, differed, links, n_jump, n_xb, reserved;
  int32_t jump_id[DD_JCAP];
  double jump_x[DD_JCAP];
  int32_t xb[DD_XCAP][2];
};

enum : uint32_t {
  ERR_EDGES = 1u,      // an output list / reaction edge buffer full (kmc_step grows them and replays)
  ERR_GEOMETRY = 2u,    // rigid-body extent bound violated
  ERR_RESOLVE = 4u,     // collision resolution did not converge
  ERR_ALIGN = 8u,       // alignment repeat guard
  ERR_MEMBERS = 16u,    // members[] overflow
  ERR_RECORDS = 32u,    // record buffer overflow
};

enum : uint8_t { U_NONE = 0, U_FREE_A = 1, U_DIMER = 2, U_FREE_B = 3, U_COMPLEX = 4, U_DIMER_P = 5 };  // U_DIMER_P: a cis dimer's partner
enum : uint32_t { S_ACC = 1, S_PEND = 2, S_REJ = 3 };  // unit fate this step (atomicMax order)

// ---------------------------------------------------------------- layout
// Paired structure-of-arrays: every element is a double2 holding two
// coordinates of ONE protein, so a lane moves 16 bytes per access (one
// dwordx4) and a wave 1 KiB contiguous.  Element (row r, slot i) is double2
// number r·n + i (n = NA or NB).  Receptor rows (bead (j,k), 1-based):
//   (j-1)·4 + (k-1)              (x, y) of bead (j,k)                rows 0..15
//   16 + (j-1)/2·4 + (k-1), j odd (z of (j,k), z of (j+1,k))         rows 16..23
// Ligand rows: (j-1)·2 + (k-1) (x, y), rows 0..7; 8 + (j-1)/2·2 + (k-1) the z
// pairs, rows 8..11.  The host side (kmc_state_view) keeps the reference-order
// SoA `[(bead·3 + c)][n]`; k_gather_beads converts at the boundary.
#define ROWS_A 24
#define ROWS_B 12
// BEAD_BLOCK 1: the rows are blocked by 64 slots instead — element (r, i) is
// number ((i / 64)·rows + r)·64 + i mod 64, so the rows of one wave's 64
// slots form one contiguous run (rows × 1 KiB) rather than `rows` streams n
// elements apart; the buffers then hold a whole number of 64-slot blocks.
#ifndef BEAD_BLOCK
#define BEAD_BLOCK 1
#endif
#ifndef BEAD_BS  // slots per block (a power of two dividing 64; A/B builds: smaller blocks put a protein's rows
#define BEAD_BS 64  // fewer cache lines apart for the gathers, the streams' rows fewer bytes long)
#endif
#ifndef ROW_PERM  // (A/B builds) blocked layout: the rows the gathers read first in each block
#define ROW_PERM 0
#endif
__host__ __device__ __forceinline__ int bead_row(int r, int rows) {
#if ROW_PERM
  // receptor: [j][1] xy (0, 4, 8, 12) and their z pairs (16, 20) — the exact
  // collision test — then the [3][k] rows of the reaction gates, then the rest;
  // ligand: [j][1] xy (0, 2, 4, 6) and z (8, 10) first
  constexpr unsigned char PA[24] = {0, 6, 7, 8, 1, 9, 10, 11, 2, 12, 13, 14, 3, 15, 16, 17, 4, 18, 19, 20, 5, 21, 22, 23};
  constexpr unsigned char PB[12] = {0, 6, 1, 7, 2, 8, 3, 9, 4, 10, 5, 11};
  return rows == 24 ? PA[r] : PB[r];
#else
  (void)rows;
  return r;
#endif
}
__host__ __device__ __forceinline__ size_t bead_elem(int i, int r, int n, int rows) {
#if BEAD_BLOCK
  (void)n;
  return ((size_t)(i / BEAD_BS) * rows + bead_row(r, rows)) * BEAD_BS + (i % BEAD_BS);
#else
  (void)rows;
  return (size_t)r * n + i;
#endif
}
// slots a bead buffer of n proteins holds
__host__ __device__ __forceinline__ size_t bead_slots(int n) {
  return BEAD_BLOCK ? ((size_t)n + 63) / 64 * 64 : (size_t)n;
}
__host__ __device__ __forceinline__ size_t bead_off_a(int i, int j, int k, int c, int NA) {
  const int row = c < 2 ? (j - 1) * 4 + (k - 1) : 16 + ((j - 1) >> 1) * 4 + (k - 1);
  const int half = c < 2 ? c : ((j - 1) & 1);
  return bead_elem(i, row, NA, ROWS_A) * 2 + half;
}
__host__ __device__ __forceinline__ size_t bead_off_b(int i, int j, int k, int c, int NB) {
  const int row = c < 2 ? (j - 1) * 2 + (k - 1) : 8 + ((j - 1) >> 1) * 2 + (k - 1);
  const int half = c < 2 ? c : ((j - 1) & 1);
  return bead_elem(i, row, NB, ROWS_B) * 2 + half;
}
struct Beads {
  double* a;
  double* b;
  int NA, NB;
  __device__ __forceinline__ double& A(int i, int j, int k, int c) const { return a[bead_off_a(i, j, k, c, NA)]; }
  __device__ __forceinline__ double& B(int i, int j, int k, int c) const { return b[bead_off_b(i, j, k, c, NB)]; }
  // whole double2 rows (one 16-byte access)
  __device__ __forceinline__ double2& A2(int i, int row) const {
    return reinterpret_cast<double2*>(a)[bead_elem(i, row, NA, ROWS_A)];
  }
  __device__ __forceinline__ double2& B2(int i, int row) const {
    return reinterpret_cast<double2*>(b)[bead_elem(i, row, NB, ROWS_B)];
  }
  // (x, y) of a bead in one access
  __device__ __forceinline__ double2 Axy(int i, int j, int k) const { return A2(i, (j - 1) * 4 + (k - 1)); }
  __device__ __forceinline__ double2 Bxy(int i, int j, int k) const { return B2(i, (j - 1) * 2 + (k - 1)); }
  // protein p is 0-based over [0, NA+NB)
  __device__ __forceinline__ double& P(int p, int j, int k, int c) const {
    return p < NA ? A(p, j, k, c) : B(p - NA, j, k, c);
  }
};

// ---------------------------------------------------------------- geometry
// Euler matrix, main.cpp:613-623
struct Rot {
  double t[3][3];
};
__device__ __forceinline__ Rot euler(double theta, double phi, double psai) {
  double cth = kmcm::cos(theta), sth = kmcm::sin(theta);
  double cph = kmcm::cos(phi), sph = kmcm::sin(phi);
  double cps = kmcm::cos(psai), sps = kmcm::sin(psai);
  Rot r;
  r.t[0][0] = cps * cph - cth * sph * sps;
  r.t[0][1] = -sps * cph - cth * sph * cps;
  r.t[0][2] = sth * sph;
  r.t[1][0] = cps * sph + cth * cph * sps;
  r.t[1][1] = -sps * sph + cth * cph * cps;
  r.t[1][2] = -sth * cph;
  r.t[2][0] = sps * sth;
  r.t[2][1] = cps * sth;
  r.t[2][2] = cth;
  return r;
}
// x' = t·(o − c) + c, one component at a time, main.cpp:631-633
__device__ __forceinline__ double rx(const Rot& r, double ox, double oy, double oz, double cx, double cy,
                                     double cz) {
  return r.t[0][0] * (ox - cx) + r.t[0][1] * (oy - cy) + r.t[0][2] * (oz - cz) + cx;
}
__device__ __forceinline__ double ry(const Rot& r, double ox, double oy, double oz, double cx, double cy,
                                     double cz) {
  return r.t[1][0] * (ox - cx) + r.t[1][1] * (oy - cy) + r.t[1][2] * (oz - cz) + cy;
}
__device__ __forceinline__ double rz(const Rot& r, double ox, double oy, double oz, double cx, double cy,
                                     double cz) {
  return r.t[2][0] * (ox - cx) + r.t[2][1] * (oy - cy) + r.t[2][2] * (oz - cz) + cz;
}

// gettheta, main.cpp:2329-2366 (p1 is the origin in every call site)
__device__ __forceinline__ double gettheta(double p0x, double p0y, double p0z, double p2x, double p2y,
                                           double p2z) {
  double lx0 = 0.0 - p0x, ly0 = 0.0 - p0y, lz0 = 0.0 - p0z;
  double lr0 = kmcm::sqrt_(lx0 * lx0 + ly0 * ly0 + lz0 * lz0);
  double lx1 = p2x - 0.0, ly1 = p2y - 0.0, lz1 = p2z - 0.0;
  double lr1 = kmcm::sqrt_(lx1 * lx1 + ly1 * ly1 + lz1 * lz1);
  double conv = 180 / 3.14159;
  double doth1 = -(lx1 * lx0 + ly0 * ly1 + lz0 * lz1);
  double doth2 = doth1 / (lr1 * lr0);
  if (doth2 > 1) doth2 = 1;
  if (doth2 < -1) doth2 = -1;
  return kmcm::acos(doth2) * conv;
}

__device__ __forceinline__ bool AreSame(double a, double b) { return kmcm::fabs_(a - b) < 1.0E-8; }

__device__ __forceinline__ double d2(double dx, double dy, double dz) { return dx * dx + dy * dy + dz * dz; }

// relaxed agent-scope accesses for values other workgroups update in-launch
__device__ __forceinline__ uint32_t ld_state(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_state(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace kmcd
