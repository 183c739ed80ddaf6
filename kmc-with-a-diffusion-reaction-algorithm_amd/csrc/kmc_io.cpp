// kmc_io.cpp — host-side formats and initial configurations of libkmc.
//
//  * position.cpt reader (main.cpp:226-270) and writer (main.cpp:2206-2244),
//    byte-compatible with the reference (pinned by tests against files the
//    reference itself wrote, tests/golden/*.cpt.gz);
//  * the bond.dat line (main.cpp:2247-2253);
//  * random placement with the reference's rules (main.cpp:281-447) drawn from
//    the keyed Philox stream, O(N) through a hash grid so 1e6-1e7-particle
//    boxes are reachable (the reference's goto sampler is O(N^2));
//  * state validation: bond-link consistency and the rigid-body extent bound
//    the device cell list relies on.
#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/kmc.h"
#include "kmc_host.h"
#include "kmc_math.h"
#include "kmc_philox.h"
#include "kmc_state_hash.h"

namespace {

inline size_t RA(int na, int j, int k, int c, int i) { return (size_t)((((j - 1) * 4 + (k - 1)) * 3) + c) * na + i; }
inline size_t RB(int nb, int j, int k, int c, int i) { return (size_t)((((j - 1) * 2 + (k - 1)) * 3) + c) * nb + i; }

struct Tok {
  FILE* f;
  char buf[128];
  bool next(std::string* err) {
    int c;
    do {
      c = fgetc(f);
    } while (c == ' ' || c == '\n' || c == '\t' || c == '\r');
    if (c == EOF) {
      *err = "unexpected end of file";
      return false;
    }
    int n = 0;
    while (c != EOF && c != ' ' && c != '\n' && c != '\t' && c != '\r') {
      if (n < 127) buf[n++] = (char)c;
      c = fgetc(f);
    }
    buf[n] = 0;
    return true;
  }
  bool f64(double* out, std::string* err) {
    if (!next(err)) return false;
    char* e = nullptr;
    errno = 0;
    *out = strtod(buf, &e);  // istream >> double: strtod in the C locale
    if (e == buf || *e) {
      *err = std::string("bad number '") + buf + "'";
      return false;
    }
    return true;
  }
  bool i32(int32_t* out, std::string* err) {
    if (!next(err)) return false;
    char* e = nullptr;
    long v = strtol(buf, &e, 10);
    if (e == buf || *e) {
      *err = std::string("bad integer '") + buf + "'";
      return false;
    }
    *out = (int32_t)v;
    return true;
  }
};

}  // namespace

namespace kmch_host {

int load_cpt(const kmc_params* p, const char* path, kmc_state_view* v, std::string* err) {
  FILE* f = fopen(path, "rb");
  if (!f) {
    *err = std::string("cannot open ") + path;
    return KMC_ERR_IO;
  }
  Tok t{f, {0}};
  const int na = p->n_a, nb = p->n_b;
  int rc = KMC_OK;
  for (int i = 0; i < na && rc == KMC_OK; ++i) {
    for (int j = 1; j <= 4 && rc == KMC_OK; ++j)
      for (int k = 1; k <= 4 && rc == KMC_OK; ++k)
        for (int c = 0; c < 3; ++c)
          if (!t.f64(&v->ra[RA(na, j, k, c, i)], err)) {
            rc = KMC_ERR_FORMAT;
            break;
          }
    for (int q = 0; q < 5 && rc == KMC_OK; ++q)  // status2 status3 nei2 nei4 nei3
      if (!t.i32(&v->a_int[(size_t)q * na + i], err)) rc = KMC_ERR_FORMAT;
  }
  for (int i = 0; i < nb && rc == KMC_OK; ++i)
    for (int j = 1; j <= 4 && rc == KMC_OK; ++j) {
      for (int k = 1; k <= 2 && rc == KMC_OK; ++k)
        for (int c = 0; c < 3; ++c)
          if (!t.f64(&v->rb[RB(nb, j, k, c, i)], err)) {
            rc = KMC_ERR_FORMAT;
            break;
          }
      if (rc == KMC_OK && !t.i32(&v->b_int[(size_t)(j - 1) * nb + i], err)) rc = KMC_ERR_FORMAT;
      if (rc == KMC_OK && !t.i32(&v->b_int[(size_t)(4 + j - 1) * nb + i], err)) rc = KMC_ERR_FORMAT;
    }
  for (int q = 0; q < 5 && rc == KMC_OK; ++q)
    if (!t.i32(&v->counters[q], err)) rc = KMC_ERR_FORMAT;
  int32_t step = 0;
  if (rc == KMC_OK && !t.i32(&step, err)) rc = KMC_ERR_FORMAT;
  fclose(f);
  if (rc == KMC_OK) v->step = step;  // the run continues at step+1 (main.cpp:267)
  return rc;
}

int write_cpt(const kmc_params* p, const kmc_state_view* v, const char* path, std::string* err) {
  FILE* f = fopen(path, "wb");
  if (!f) {
    *err = std::string("cannot open ") + path;
    return KMC_ERR_IO;
  }
  const int na = p->n_a, nb = p->n_b;
  // fixed, setprecision(3), setw(10) per coordinate; setw(8) per int
  for (int i = 0; i < na; ++i) {
    for (int j = 1; j <= 4; ++j)
      for (int k = 1; k <= 4; ++k)
        fprintf(f, "%10.3f%10.3f%10.3f\n", v->ra[RA(na, j, k, 0, i)], v->ra[RA(na, j, k, 1, i)], v->ra[RA(na, j, k, 2, i)]);
    fprintf(f, "%8d%8d%8d%8d%8d\n", v->a_int[0 * (size_t)na + i], v->a_int[1 * (size_t)na + i],
            v->a_int[2 * (size_t)na + i], v->a_int[3 * (size_t)na + i], v->a_int[4 * (size_t)na + i]);
  }
  for (int i = 0; i < nb; ++i)
    for (int j = 1; j <= 4; ++j) {
      for (int k = 1; k <= 2; ++k)
        fprintf(f, "%10.3f%10.3f%10.3f\n", v->rb[RB(nb, j, k, 0, i)], v->rb[RB(nb, j, k, 1, i)], v->rb[RB(nb, j, k, 2, i)]);
      fprintf(f, "%8d%8d\n", v->b_int[(size_t)(j - 1) * nb + i], v->b_int[(size_t)(4 + j - 1) * nb + i]);
    }
  for (int q = 0; q < 5; ++q) fprintf(f, "%d\n", v->counters[q]);
  fprintf(f, "%lld\n", (long long)v->step);
  if (fclose(f) != 0) {
    *err = "write failed";
    return KMC_ERR_IO;
  }
  return KMC_OK;
}

// bond-link consistency (what every reference step maintains) and the
// extent bound of the 130 Å cell list (kmc_kernels.hip)
int validate(const kmc_params* p, const kmc_state_view* v, std::string* err) {
  const int na = p->n_a, nb = p->n_b, n = na + nb;
  char msg[256];
  for (int i = 0; i < na; ++i) {
    int st2 = v->a_int[0 * (size_t)na + i], st3 = v->a_int[1 * (size_t)na + i];
    int n2 = v->a_int[2 * (size_t)na + i], n4 = v->a_int[3 * (size_t)na + i], n3 = v->a_int[4 * (size_t)na + i];
    bool ok = (st2 == 0 || st2 == 1) && (st3 == 0 || st3 == 1) && (st2 == (n2 != 0)) && (st3 == (n3 != 0));
    if (ok && n2) {
      ok = n2 > na && n2 <= n && n4 >= 2 && n4 <= 4;
      if (ok) {
        int b = n2 - 1 - na;
        ok = v->b_int[(size_t)(4 + n4 - 1) * nb + b] == i + 1 && v->b_int[(size_t)(n4 - 1) * nb + b] == 1;
      }
    } else if (ok) {
      ok = n4 == 0;
    }
    if (ok && n3) ok = n3 >= 1 && n3 <= na && n3 != i + 1 && v->a_int[4 * (size_t)na + (n3 - 1)] == i + 1;
    if (!ok) {
      snprintf(msg, sizeof msg, "inconsistent bond state at receptor %d", i + 1);
      *err = msg;
      return KMC_ERR_STATE;
    }
  }
  for (int b = 0; b < nb; ++b) {
    if (v->b_int[0 * (size_t)nb + b] != 0 || v->b_int[4 * (size_t)nb + b] != 0) {
      snprintf(msg, sizeof msg, "ligand %d: site 1 is the virtual centre and cannot bind", na + b + 1);
      *err = msg;
      return KMC_ERR_STATE;
    }
    for (int j = 2; j <= 4; ++j) {
      int st = v->b_int[(size_t)(j - 1) * nb + b], ne = v->b_int[(size_t)(4 + j - 1) * nb + b];
      bool ok = (st == (ne != 0)) && (st == 0 || st == 1);
      if (ok && ne) ok = ne >= 1 && ne <= na && v->a_int[2 * (size_t)na + (ne - 1)] == na + b + 1 &&
                         v->a_int[3 * (size_t)na + (ne - 1)] == j;
      if (!ok) {
        snprintf(msg, sizeof msg, "inconsistent bond state at ligand %d site %d", na + b + 1, j);
        *err = msg;
        return KMC_ERR_STATE;
      }
    }
  }
  // extents: receptor beads within 0.3 Å (domain axis) / 20.3 Å (sites) of
  // [1][1] in xy; ligand [1][2] ≤ 30.3, subunit centres ≤ 35, sites ≤ 65 Å
  for (int i = 0; i < na; ++i) {
    double x0 = v->ra[RA(na, 1, 1, 0, i)], y0 = v->ra[RA(na, 1, 1, 1, i)];
    for (int j = 1; j <= 4; ++j)
      for (int k = 1; k <= 4; ++k) {
        double dx = v->ra[RA(na, j, k, 0, i)] - x0, dy = v->ra[RA(na, j, k, 1, i)] - y0;
        double lim = (k == 1 || k == 4) ? 0.3 : 20.3;
        if (!(dx * dx + dy * dy <= lim * lim)) {
          snprintf(msg, sizeof msg, "receptor %d bead [%d][%d] outside the rigid-body extent bound", i + 1, j, k);
          *err = msg;
          return KMC_ERR_GEOMETRY;
        }
      }
  }
  for (int b = 0; b < nb; ++b) {
    double x0 = v->rb[RB(nb, 1, 1, 0, b)], y0 = v->rb[RB(nb, 1, 1, 1, b)];
    for (int j = 1; j <= 4; ++j)
      for (int k = 1; k <= 2; ++k) {
        double dx = v->rb[RB(nb, j, k, 0, b)] - x0, dy = v->rb[RB(nb, j, k, 1, b)] - y0;
        double lim = j == 1 ? (k == 1 ? 0.3 : 30.3) : (k == 1 ? 35.0 : 65.0);
        if (!(dx * dx + dy * dy <= lim * lim)) {
          snprintf(msg, sizeof msg, "ligand %d bead [%d][%d] outside the rigid-body extent bound", na + b + 1, j, k);
          *err = msg;
          return KMC_ERR_GEOMETRY;
        }
      }
  }
  return KMC_OK;
}

// derived bond counters of a state: rl, mono-cis pairs, complex-cis pairs
void derived_counts(const kmc_params* p, const kmc_state_view* v, int* rl, int* mono, int* cis) {
  const int na = p->n_a;
  *rl = *mono = *cis = 0;
  for (int i = 0; i < na; ++i) {
    *rl += v->a_int[0 * (size_t)na + i];
    if (v->a_int[1 * (size_t)na + i] == 1) {
      int q = v->a_int[4 * (size_t)na + i] - 1;
      if (i < q) {
        if (v->a_int[0 * (size_t)na + i] == 0 && v->a_int[0 * (size_t)na + q] == 0) ++*mono;
        else ++*cis;
      }
    }
  }
}

// ------------------------------------------------------------------ placement
// main.cpp:281-447 with keyed draws: identical to the oracle's keyed
// placement (a hash grid only prunes pairs that cannot reject).
struct Grid {
  double cs, x0, y0;
  int nx, ny;
  std::vector<int> head, next;  // linked lists of item indices
  Grid(double box_x, double box_y, double cell, int cap) {
    cs = cell;
    x0 = -box_x / 2 - 2 * cell;
    y0 = -box_y / 2 - std::max(box_x, box_y) / 2 - 2 * cell;  // ligand y range uses box_x (sic)
    nx = (int)((box_x + 4 * cell) / cell) + 1;
    ny = (int)((box_y + std::max(box_x, box_y) + 4 * cell) / cell) + 1;
    head.assign((size_t)nx * ny, -1);
    next.assign(cap, -1);
  }
  int cx(double x) const { return std::min(std::max((int)std::floor((x - x0) / cs), 0), nx - 1); }
  int cy(double y) const { return std::min(std::max((int)std::floor((y - y0) / cs), 0), ny - 1); }
  void add(int item, double x, double y) {
    size_t c = (size_t)cy(y) * nx + cx(x);
    next[item] = head[c];
    head[c] = item;
  }
  template <typename F>
  bool any_near(double x, double y, F f) const {
    int X = cx(x), Y = cy(y);
    for (int yy = Y - 1; yy <= Y + 1; ++yy)
      for (int xx = X - 1; xx <= X + 1; ++xx) {
        if (xx < 0 || yy < 0 || xx >= nx || yy >= ny) continue;
        for (int it = head[(size_t)yy * nx + xx]; it >= 0; it = next[it])
          if (f(it)) return true;
      }
    return false;
  }
};

static void euler(double theta, double phi, double psai, double t[3][3]) {
  double cth = kmcm::cos(theta), sth = kmcm::sin(theta);
  double cph = kmcm::cos(phi), sph = kmcm::sin(phi);
  double cps = kmcm::cos(psai), sps = kmcm::sin(psai);
  t[0][0] = cps * cph - cth * sph * sps;
  t[0][1] = -sps * cph - cth * sph * cps;
  t[0][2] = sth * sph;
  t[1][0] = cps * sph + cth * cph * sps;
  t[1][1] = -sps * sph + cth * cph * cps;
  t[1][2] = -sth * cph;
  t[2][0] = sps * sth;
  t[2][1] = cps * sth;
  t[2][2] = cth;
}

int init_random(const kmc_params* p, kmc_state_view* v, std::string* err) {
  const int na = p->n_a, nb = p->n_b;
  const double RAd = p->ra_radius, RBd = p->rb_radius, pai = p->pai;
  const kmcr::Key key = kmcr::make_key(p->seed, p->replica);
  const int64_t MAXATT = 100000000;
  auto draw = [&](int prot1, uint32_t att, int slot) {
    double u0, u1;
    kmcr::uniform2(key, kmcr::DOM_INIT, (uint32_t)(prot1 - 1), att, 0, (uint32_t)(slot >> 1), &u0, &u1);
    return (slot & 1) ? u1 : u0;
  };
  const uint32_t ORIENT = 0xffffffffu;
  const double S3 = kmcm::sqrt_(3.0);
  // receptors: 2-D rejection vs earlier receptors (dist <= 2 R_A)
  Grid ga(p->box_x, p->box_y, 130.0, std::max(na, 1));
  std::vector<double> ax(na), ay(na);
  for (int i = 0; i < na; ++i) {
    double ti = 0, tj = 0;
    for (uint32_t att = 0;; ++att) {
      if (att >= MAXATT) {
        *err = "receptor placement failed";
        return KMC_ERR_PLACEMENT;
      }
      ti = draw(i + 1, att, 0) * p->box_x - p->box_x / 2;
      tj = draw(i + 1, att, 1) * p->box_y - p->box_y / 2;
      bool bad = ga.any_near(ti, tj, [&](int j) {
        double d = kmcm::sqrt_((ti - ax[j]) * (ti - ax[j]) + (tj - ay[j]) * (tj - ay[j]));
        return d <= RAd + RAd;
      });
      if (!bad) break;
    }
    ax[i] = ti;
    ay[i] = tj;
    ga.add(i, ti, tj);
    double tk = 0;
    double t[3][3];
    euler(0, 0, (2 * draw(i + 1, ORIENT, 0) - 1) * pai, t);
    for (int j = 1; j <= 4; ++j) {
      double cx = ti, cy = tj, cz = tk + (j * 2 - 2) * RAd;
      v->ra[RA(na, j, 1, 0, i)] = cx;
      v->ra[RA(na, j, 1, 1, i)] = cy;
      v->ra[RA(na, j, 1, 2, i)] = cz;
      double ox[5] = {0, 0, ti + RAd, ti - RAd, ti};
      double oy[5] = {0, 0, tj, tj, tj};
      double oz[5] = {0, 0, tk + (j * 2 - 2) * RAd, tk + (j * 2 - 2) * RAd, tk + (j * 2 - 1) * RAd};
      for (int k = 2; k <= 4; ++k) {
        v->ra[RA(na, j, k, 0, i)] = t[0][0] * (ox[k] - cx) + t[0][1] * (oy[k] - cy) + t[0][2] * (oz[k] - cz) + cx;
        v->ra[RA(na, j, k, 1, i)] = t[1][0] * (ox[k] - cx) + t[1][1] * (oy[k] - cy) + t[1][2] * (oz[k] - cz) + cy;
        v->ra[RA(na, j, k, 2, i)] = t[2][0] * (ox[k] - cx) + t[2][1] * (oy[k] - cy) + t[2][2] * (oz[k] - cz) + cz;
      }
    }
    for (int q = 0; q < 5; ++q) v->a_int[(size_t)q * na + i] = 0;
  }
  // ligands: 3-D rejection vs receptor domain centres and earlier ligands
  Grid gb(p->box_x, p->box_y, 130.0, std::max(nb, 1));
  std::vector<double> bx(nb), by(nb), bz(nb);
  for (int b = 0; b < nb; ++b) {
    int prot = na + b + 1;
    double ti = 0, tj = 0, tk = 0;
    for (uint32_t att = 0;; ++att) {
      if (att >= MAXATT) {
        *err = "ligand placement failed";
        return KMC_ERR_PLACEMENT;
      }
      ti = draw(prot, att, 0) * p->box_x - p->box_x / 2;
      tj = draw(prot, att, 1) * p->box_y - p->box_x / 2;  // sic: cell_range_x (main.cpp:358)
      tk = draw(prot, att, 2) * p->box_z;
      bool bad = ga.any_near(ti, tj, [&](int j) {
        for (int k = 1; k <= 4; ++k) {
          double X = v->ra[RA(na, k, 1, 0, j)], Y = v->ra[RA(na, k, 1, 1, j)], Z = v->ra[RA(na, k, 1, 2, j)];
          double d = kmcm::sqrt_((ti - X) * (ti - X) + (tj - Y) * (tj - Y) + (tk - Z) * (tk - Z));
          if (d <= RAd + RBd * 2 / S3 + RBd) return true;
        }
        return false;
      });
      if (!bad)
        bad = gb.any_near(ti, tj, [&](int j) {
          double d = kmcm::sqrt_((ti - bx[j]) * (ti - bx[j]) + (tj - by[j]) * (tj - by[j]) + (tk - bz[j]) * (tk - bz[j]));
          return d <= RBd * 2 / S3 + RBd * 2 / S3 + 2 * RBd;
        });
      if (!bad) break;
    }
    bx[b] = ti;
    by[b] = tj;
    bz[b] = tk;
    gb.add(b, ti, tj);
    // template R_x_0 (main.cpp:390-412), index [j][k]
    double ox[5][3] = {{0}}, oy[5][3] = {{0}}, oz[5][3] = {{0}};
    ox[1][2] = ti; oy[1][2] = tj; oz[1][2] = tk + RBd;
    ox[2][1] = ti; oy[2][1] = tj + RBd * 2 / S3; oz[2][1] = tk;
    ox[3][1] = ti - RBd; oy[3][1] = tj - RBd / S3; oz[3][1] = tk;
    ox[4][1] = ti + RBd; oy[4][1] = tj - RBd / S3; oz[4][1] = tk;
    ox[2][2] = ti; oy[2][2] = tj + RBd * (2 / S3 + 1); oz[2][2] = tk;
    ox[3][2] = ti - RBd * (S3 / 2 + 1); oy[3][2] = tj - RBd / S3 - RBd / 2; oz[3][2] = tk;
    ox[4][2] = ti + RBd * (S3 / 2 + 1); oy[4][2] = tj - RBd / S3 - RBd / 2; oz[4][2] = tk;
    double th = (2 * draw(prot, ORIENT, 0) - 1) * pai;
    double ph = (2 * draw(prot, ORIENT, 1) - 1) * pai;
    double ps = (2 * draw(prot, ORIENT, 2) - 1) * pai;
    double t[3][3];
    euler(th, ph, ps, t);
    v->rb[RB(nb, 1, 1, 0, b)] = ti;
    v->rb[RB(nb, 1, 1, 1, b)] = tj;
    v->rb[RB(nb, 1, 1, 2, b)] = tk;
    for (int j = 1; j <= 4; ++j)
      for (int k = 1; k <= 2; ++k) {
        if (j == 1 && k == 1) continue;
        v->rb[RB(nb, j, k, 0, b)] = t[0][0] * (ox[j][k] - ti) + t[0][1] * (oy[j][k] - tj) + t[0][2] * (oz[j][k] - tk) + ti;
        v->rb[RB(nb, j, k, 1, b)] = t[1][0] * (ox[j][k] - ti) + t[1][1] * (oy[j][k] - tj) + t[1][2] * (oz[j][k] - tk) + tj;
        v->rb[RB(nb, j, k, 2, b)] = t[2][0] * (ox[j][k] - ti) + t[2][1] * (oy[j][k] - tj) + t[2][2] * (oz[j][k] - tk) + tk;
      }
    for (int q = 0; q < 8; ++q) v->b_int[(size_t)q * nb + b] = 0;
  }
  for (int q = 0; q < 5; ++q) v->counters[q] = 0;
  v->step = 0;
  return KMC_OK;
}

// ---------------------------------------------------------------- exact checkpoint
// Layout (little-endian): "KMCSTAT1", u32 version, i32 n_a, i32 n_b,
// u32 replica, u64 seed, i64 step, i32 counters[5], i32 reserved, then the
// view's arrays in their SoA layout (ra, rb as f64; a_int, b_int as i32), then
// an FNV-1a-64 of every preceding byte.
namespace {
const char kStateMagic[8] = {'K', 'M', 'C', 'S', 'T', 'A', 'T', '1'};
struct StateHeader {
  char magic[8];
  uint32_t version;
  int32_t n_a, n_b;
  uint32_t replica;
  uint64_t seed;
  int64_t step;
  int32_t counters[5];
  int32_t reserved;
};
static_assert(sizeof(StateHeader) == 64, "state header layout");

struct Fnv {
  uint64_t h = 1469598103934665603ull;
  void add(const void* p, size_t n) {
    const unsigned char* b = (const unsigned char*)p;
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
  }
};
}  // namespace

int save_state(const kmc_params* p, const kmc_state_view* v, const char* path, std::string* err) {
  const size_t NA = (size_t)p->n_a, NB = (size_t)p->n_b;
  StateHeader hd;
  std::memset(&hd, 0, sizeof hd);
  std::memcpy(hd.magic, kStateMagic, 8);
  hd.version = 1;
  hd.n_a = p->n_a;
  hd.n_b = p->n_b;
  hd.replica = p->replica;
  hd.seed = p->seed;
  hd.step = v->step;
  for (int k = 0; k < 5; ++k) hd.counters[k] = v->counters[k];
  FILE* f = fopen(path, "wb");
  if (!f) {
    *err = std::string("cannot write ") + path;
    return KMC_ERR_IO;
  }
  Fnv h;
  auto put = [&](const void* d, size_t n) {
    h.add(d, n);
    return fwrite(d, 1, n, f) == n;
  };
  bool ok = put(&hd, sizeof hd) && put(v->ra, sizeof(double) * 48 * NA) && put(v->rb, sizeof(double) * 24 * NB) &&
            put(v->a_int, sizeof(int32_t) * 5 * NA) && put(v->b_int, sizeof(int32_t) * 8 * NB);
  uint64_t tr = h.h;
  ok = ok && fwrite(&tr, 1, sizeof tr, f) == sizeof tr;
  ok = (fclose(f) == 0) && ok;
  if (!ok) {
    *err = std::string("write failed: ") + path;
    return KMC_ERR_IO;
  }
  return KMC_OK;
}

int load_state(const kmc_params* p, const char* path, kmc_state_view* v, std::string* err) {
  const size_t NA = (size_t)p->n_a, NB = (size_t)p->n_b;
  FILE* f = fopen(path, "rb");
  if (!f) {
    *err = std::string("cannot open ") + path;
    return KMC_ERR_IO;
  }
  Fnv h;
  auto get = [&](void* d, size_t n) {
    if (fread(d, 1, n, f) != n) return false;
    h.add(d, n);
    return true;
  };
  StateHeader hd;
  int rc = KMC_OK;
  if (!get(&hd, sizeof hd) || std::memcmp(hd.magic, kStateMagic, 8) != 0 || hd.version != 1) {
    *err = std::string("not a KMCSTAT1 file: ") + path;
    rc = KMC_ERR_FORMAT;
  } else if (hd.n_a != p->n_a || hd.n_b != p->n_b || hd.seed != p->seed || hd.replica != p->replica) {
    *err = "state file is of another trajectory (n_a, n_b, seed or replica differ)";
    rc = KMC_ERR_ARG;
  } else if (!get(v->ra, sizeof(double) * 48 * NA) || !get(v->rb, sizeof(double) * 24 * NB) ||
             !get(v->a_int, sizeof(int32_t) * 5 * NA) || !get(v->b_int, sizeof(int32_t) * 8 * NB)) {
    *err = std::string("truncated state file: ") + path;
    rc = KMC_ERR_FORMAT;
  } else {
    uint64_t tr = 0, want = h.h;
    if (fread(&tr, 1, sizeof tr, f) != sizeof tr || tr != want) {
      *err = std::string("state file checksum mismatch: ") + path;
      rc = KMC_ERR_FORMAT;
    }
  }
  fclose(f);
  if (rc != KMC_OK) return rc;
  v->step = hd.step;
  for (int k = 0; k < 5; ++k) v->counters[k] = hd.counters[k];
  v->reserved = 0;
  return validate(p, v, err);
}

// The window of a decomposed trajectory (kmc_dd_set_state): its local
// numbering is monotone in the global one (receptors, then ligands: every
// order the step takes — unit keys, BFS roots, the greedy reactions — is then
// the global order restricted to the window), a global index fits an
// exchanged link (global index + 1 in an int32), and ownership is 0 or 1.
int dd_check(int32_t n, const int32_t* gid, const uint8_t* own, std::string* err) {
  if (n < 0 || (n > 0 && (!gid || !own))) return KMC_ERR_ARG;
  for (int32_t i = 0; i < n; ++i) {
    if (gid[i] < 0 || gid[i] >= INT32_MAX) {
      if (err) *err = "dd: global index out of range";
      return KMC_ERR_ARG;
    }
    if (i > 0 && gid[i] <= gid[i - 1]) {
      if (err) *err = "dd: global indices not increasing";
      return KMC_ERR_ARG;
    }
    if (own[i] > 1) {
      if (err) *err = "dd: ownership flag not 0 or 1";
      return KMC_ERR_ARG;
    }
  }
  return KMC_OK;
}

}  // namespace kmch_host

// ------------------------------------------------------------------ C ABI (host-only part)
extern "C" {

void kmc_params_default(kmc_params* p) {
  memset(p, 0, sizeof *p);
  p->n_a = 150;
  p->n_b = 50;
  p->time_step = 10;
  p->box_x = 5773;
  p->box_y = 5773;
  p->box_z = 1000;
  p->pai = 3.1415926;
  p->ra_radius = 20;
  p->ra_D = 1;
  p->ra_rot_D = 0.0174;
  p->rb_radius = 30;
  p->rb_D = 7.2614;
  p->rb_rot_D = 0.0061209;
  p->mono_cis_ass_rate = 0.000047;
  p->mono_cis_diss_rate = 0.000000000000112;
  p->cis_D = 0.5;
  p->cis_rot_D = 0.005;
  p->cis_ass_rate = 0.00096;
  p->cis_diss_rate = 0.000000000000112;
  p->bond_D = 0.5;
  p->bond_rot_D = 0.005;
  p->ass_rate = 0.04;
  p->diss_rate = 0.000000000000348;
  p->bond_dist_cutoff = 18;
  p->bond_thetapd_cutoff = 45;
  p->bond_thetaot_cutoff = 90;
  p->cis_thetaot_cutoff = 10;
  p->cis_dist_cutoff = 15;
  p->simu_step = 20000000;
  p->out_interval = 5000;
  p->seed = 1;
  p->replica = 0;
}

int kmc_format_bond_line(const kmc_params* p, const kmc_obs* o, char* buf, size_t n) {
  // setw(15) t, setw(5) rl, setw(5) mono, setw(10) cis, setw(10) bond,
  // setw(10) cluster_size (fixed, 3 decimals), setw(10) max complex
  (void)p;
  return snprintf(buf, n, "%15.3f%5d%5d%10d%10d%10.3f%10d\n", o->t, o->bond_num_rl, o->bond_num_mono_cis,
                  o->bond_num_cis, o->bond_num, o->cluster_size, o->protein_num_in_max_complex);
}

uint64_t kmc_state_hash(const kmc_params* p, const kmc_state_view* v) { return kmch::state_hash(p->n_a, p->n_b, v); }

// parameter.log, main.cpp:178-205 (default ostream float format = %g)
int kmc_host_write_parameter_log(const kmc_params* p, const char* path) {
  FILE* f = fopen(path, "wb");
  if (!f) return KMC_ERR_IO;
  auto L = [&](const char* k, double v) { fprintf(f, "%25s%15g\n", k, v); };
  fprintf(f, "%25s%15g%7g%7g\n\n", "box size: x y z", p->box_x, p->box_y, p->box_z);
  fprintf(f, "%25s%15d\n", "protein_A_tot_num", p->n_a);
  fprintf(f, "%25s%15d\n", "RB_A_tot_num", p->n_a * 4);
  fprintf(f, "%25s%15d\n", "protein_B_tot_num", p->n_b);
  fprintf(f, "%25s%15d\n\n", "RB_B_tot_num", p->n_b * 4);
  L("RB_A_D", p->ra_D);
  L("RB_A_rot_D", p->ra_rot_D);
  L("RB_B_D", p->rb_D);
  fprintf(f, "%25s%15g\n\n", "RB_B_rot_D", p->rb_rot_D);
  fprintf(f, "%25s\n", "R-L interaction:");
  L("bond_D", p->bond_D);
  L("bond_rot_D", p->bond_rot_D);
  L("Ass_Rate", p->ass_rate);
  fprintf(f, "%25s%15g\n\n", "Diss_Rate", p->diss_rate);
  fprintf(f, "%25s\n", "Cis interaction:");
  L("cis_D", p->cis_D);
  L("cis_rot_D", p->cis_rot_D);
  L("mono_cis_Ass_Rate", p->mono_cis_ass_rate);
  fprintf(f, "%25s%15g\n\n", "mono_cis_Diss_Rate", p->mono_cis_diss_rate);
  L("cis_Ass_Rate", p->cis_ass_rate);
  fprintf(f, "%25s%15g\n\n", "cis_Diss_Rate", p->cis_diss_rate);
  return fclose(f) == 0 ? KMC_OK : KMC_ERR_IO;
}

// test.gro frame, main.cpp:2258-2287 (appended): receptor domain centres and
// ligand subunit centres in nm, fixed with 3 decimals
int kmc_host_append_gro(const kmc_params* p, const kmc_state_view* v, const char* path) {
  FILE* f = fopen(path, "ab");
  if (!f) return KMC_ERR_IO;
  const int na = p->n_a, nb = p->n_b;
  fprintf(f, "Hello Gro!, t=%.3f\n", (double)(int)v->step * p->time_step);
  fprintf(f, "%d\n", na * 4 + nb * 3);
  for (int i = 0; i < na; ++i)
    for (int j = 1; j <= 4; ++j)
      fprintf(f, "%5dALA%7s%5d%8.3f%8.3f%8.3f\n", i + 1, "CA", i + 1, v->ra[RA(na, j, 1, 0, i)] / 10,
              v->ra[RA(na, j, 1, 1, i)] / 10, v->ra[RA(na, j, 1, 2, i)] / 10);
  for (int b = 0; b < nb; ++b)
    for (int j = 2; j <= 4; ++j)
      fprintf(f, "%5dLEU%7s%5d%8.3f%8.3f%8.3f\n", na + b + 1, "CA", na + b + 1, v->rb[RB(nb, j, 1, 0, b)] / 10,
              v->rb[RB(nb, j, 1, 1, b)] / 10, v->rb[RB(nb, j, 1, 2, b)] / 10);
  fprintf(f, "%8.3f%12.3f%12.3f\n", p->box_x / 10, p->box_y / 10, p->box_z / 10);
  return fclose(f) == 0 ? KMC_OK : KMC_ERR_IO;
}

// cluster.log block, main.cpp:2291-2305 (appended): for every ligand its BFS
// row (members in results[i][.] order, "  "-separated; empty for non-roots)
int kmc_host_append_cluster_log(const kmc_params* p, int64_t step, const int32_t* row_len, const int32_t* members,
                                const char* path) {
  FILE* f = fopen(path, "ab");
  if (!f) return KMC_ERR_IO;
  fprintf(f, "Hello Cluster!, t=%g\n", (double)(int)step * p->time_step);
  int64_t o = 0;
  for (int b = 0; b < p->n_b; ++b) {
    for (int t = 0; t < row_len[b]; ++t) fprintf(f, "%d  ", members[o++]);
    fputc('\n', f);
  }
  return fclose(f) == 0 ? KMC_OK : KMC_ERR_IO;
}

static thread_local std::string g_host_err;
const char* kmc_host_last_error(void) { return g_host_err.c_str(); }

int kmc_host_load_cpt(const kmc_params* p, const char* path, kmc_state_view* v) {
  return kmch_host::load_cpt(p, path, v, &g_host_err);
}
int kmc_host_write_cpt(const kmc_params* p, const kmc_state_view* v, const char* path) {
  return kmch_host::write_cpt(p, v, path, &g_host_err);
}
int kmc_host_init_random(const kmc_params* p, kmc_state_view* v) { return kmch_host::init_random(p, v, &g_host_err); }
int kmc_host_save_state(const kmc_params* p, const kmc_state_view* v, const char* path) {
  return kmch_host::save_state(p, v, path, &g_host_err);
}
int kmc_host_load_state(const kmc_params* p, const char* path, kmc_state_view* v) {
  return kmch_host::load_state(p, path, v, &g_host_err);
}
int kmc_host_validate(const kmc_params* p, const kmc_state_view* v) { return kmch_host::validate(p, v, &g_host_err); }
int kmc_host_dd_check(int32_t n, const int32_t* gid, const uint8_t* own) {
  return kmch_host::dd_check(n, gid, own, &g_host_err);
}

int kmc_host_math(int op, const double* x, const double* y, double* out, int64_t n) {
  for (int64_t i = 0; i < n; ++i) {
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
  return KMC_OK;
}

}  // extern "C"
