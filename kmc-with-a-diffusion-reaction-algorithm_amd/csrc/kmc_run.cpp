// kmc_run.cpp — drop-in replacement for the reference executable.
//
// Reproduces main.cpp's process/file contract on top of libkmc (include/kmc.h):
//   * writes parameter.log (main.cpp:169-205);
//   * resumes from ./position.cpt when it exists, continuing at saved step + 1
//     (main.cpp:226-270); otherwise truncates test.gro, bond.dat, cluster.log
//     and position.cpt and draws a random configuration (main.cpp:273-456);
//   * runs the diffusion–reaction loop on the GPU up to simu_step
//     (main.cpp:461-2308);
//   * every out_interval steps (5000, main.cpp:2206) rewrites position.cpt and
//     appends bond.dat, test.gro and cluster.log (main.cpp:2206-2305).
// Parameters that are compile-time #defines / globals in the reference
// (main.cpp:39-99) are command-line options here:
//   kmc_run [--n-a 150] [--n-b 50] [--steps 20000000] [--box 5773 5773 1000]
//           [--out-interval 5000] [--seed 1] [--replica 0] [--device 0]
//           [--set name=value ...]   (any kmc_params field, e.g. ass_rate=0.04)
//           [--state FILE]   exact checkpoint (include/kmc.h, KMCSTAT1): resumed
//                            from when it exists (instead of position.cpt) and
//                            rewritten with position.cpt every out_interval
#include <sys/stat.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/kmc.h"

namespace {

bool set_field(kmc_params* p, const std::string& k, const std::string& v) {
  double d = strtod(v.c_str(), nullptr);
#define F(name)            \
  if (k == #name) {        \
    p->name = (decltype(p->name))d; \
    return true;           \
  }
  F(n_a) F(n_b) F(time_step) F(box_x) F(box_y) F(box_z) F(pai) F(ra_radius) F(ra_D) F(ra_rot_D) F(rb_radius)
  F(rb_D) F(rb_rot_D) F(mono_cis_ass_rate) F(mono_cis_diss_rate) F(cis_D) F(cis_rot_D) F(cis_ass_rate)
  F(cis_diss_rate) F(bond_D) F(bond_rot_D) F(ass_rate) F(diss_rate) F(bond_dist_cutoff) F(bond_thetapd_cutoff)
  F(bond_thetaot_cutoff) F(cis_thetaot_cutoff) F(cis_dist_cutoff) F(simu_step) F(out_interval) F(replica)
#undef F
  if (k == "seed") {
    p->seed = strtoull(v.c_str(), nullptr, 10);
    return true;
  }
  return false;
}

int die(kmc_sim* s, int rc, const char* what) {
  fprintf(stderr, "kmc_run: %s failed (%d): %s\n", what, rc, s ? kmc_last_error(s) : kmc_host_last_error());
  return 1;
}

bool exists(const char* path) {
  struct stat st;
  return stat(path, &st) == 0;
}

void truncate(const char* path) {
  FILE* f = fopen(path, "wb");
  if (f) fclose(f);
}

}  // namespace

int main(int argc, char** argv) {
  kmc_params p;
  kmc_params_default(&p);
  int device = 0;
  std::string state_path;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> std::string {
      if (i + 1 >= argc) {
        fprintf(stderr, "kmc_run: %s needs a value\n", a.c_str());
        exit(2);
      }
      return argv[++i];
    };
    if (a == "--n-a") p.n_a = atoi(next().c_str());
    else if (a == "--n-b") p.n_b = atoi(next().c_str());
    else if (a == "--steps") p.simu_step = atoll(next().c_str());
    else if (a == "--box") {
      p.box_x = atof(next().c_str());
      p.box_y = atof(next().c_str());
      p.box_z = atof(next().c_str());
    } else if (a == "--out-interval") p.out_interval = atoi(next().c_str());
    else if (a == "--seed") p.seed = strtoull(next().c_str(), nullptr, 10);
    else if (a == "--replica") p.replica = (uint32_t)atoi(next().c_str());
    else if (a == "--device") device = atoi(next().c_str());
    else if (a == "--state") state_path = next();
    else if (a == "--set") {
      std::string kv = next();
      size_t eq = kv.find('=');
      if (eq == std::string::npos || !set_field(&p, kv.substr(0, eq), kv.substr(eq + 1))) {
        fprintf(stderr, "kmc_run: bad --set %s\n", kv.c_str());
        return 2;
      }
    } else {
      fprintf(stderr, "kmc_run: unknown option %s\n", a.c_str());
      return 2;
    }
  }
  if (p.out_interval <= 0) p.out_interval = 5000;

  int rc = kmc_host_write_parameter_log(&p, "parameter.log");
  if (rc) return die(nullptr, rc, "parameter.log");
  kmc_sim* s = nullptr;
  rc = kmc_create(&p, device, &s);
  if (rc) return die(nullptr, rc, "kmc_create");
  if (!state_path.empty() && exists(state_path.c_str())) {
    printf("STATE file is exist\n");
    rc = kmc_load_state(s, state_path.c_str());
    if (rc) return die(s, rc, state_path.c_str());
  } else if (exists("position.cpt")) {
    printf("CPT file is exist\n");
    rc = kmc_load_cpt(s, "position.cpt");
    if (rc) return die(s, rc, "position.cpt");
  } else {
    printf("CPT file not exist\n");
    truncate("test.gro");
    truncate("bond.dat");
    truncate("cluster.log");
    truncate("position.cpt");
    rc = kmc_init_random(s);
    if (rc) return die(s, rc, "random placement");
  }
  fflush(stdout);

  const int na = p.n_a, nb = p.n_b;
  std::vector<double> ra((size_t)48 * na + 1), rb((size_t)24 * nb + 1);
  std::vector<int32_t> ai((size_t)5 * na + 1), bi((size_t)8 * nb + 1), row((size_t)nb + 1),
      mem((size_t)na + nb + 1);
  kmc_state_view v{ra.data(), rb.data(), ai.data(), bi.data(), {0, 0, 0, 0, 0}, 0, 0};
  std::vector<kmc_obs> obs;
  int64_t step = kmc_current_step(s);
  while (step < p.simu_step) {
    int64_t next_out = (step / p.out_interval + 1) * p.out_interval;
    int64_t end = next_out < p.simu_step ? next_out : p.simu_step;
    int64_t n = end - step;
    obs.resize((size_t)n);
    rc = kmc_step(s, n, obs.data());
    if (rc) return die(s, rc, "kmc_step");
    step = end;
    if (step % p.out_interval == 0) {
      rc = kmc_write_cpt(s, "position.cpt");
      if (rc) return die(s, rc, "position.cpt");
      if (!state_path.empty()) {
        rc = kmc_save_state(s, state_path.c_str());
        if (rc) return die(s, rc, state_path.c_str());
      }
      char line[256];
      kmc_format_bond_line(&p, &obs.back(), line, sizeof line);
      FILE* f = fopen("bond.dat", "ab");
      if (!f) return die(s, KMC_ERR_IO, "bond.dat");
      fputs(line, f);
      fclose(f);
      rc = kmc_get_state(s, &v);
      if (rc) return die(s, rc, "state");
      rc = kmc_host_append_gro(&p, &v, "test.gro");
      if (rc) return die(s, rc, "test.gro");
      rc = kmc_get_clusters(s, row.data(), mem.data());
      if (rc) return die(s, rc, "clusters");
      rc = kmc_host_append_cluster_log(&p, step, row.data(), mem.data(), "cluster.log");
      if (rc) return die(s, rc, "cluster.log");
    }
  }
  kmc_destroy(s);
  return 0;
}
