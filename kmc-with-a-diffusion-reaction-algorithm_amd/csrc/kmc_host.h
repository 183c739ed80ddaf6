// kmc_host.h — host-only helpers of libkmc shared by the C-ABI entry points.
#pragma once
#include <string>

#include "../../include/kmc.h"

namespace kmch_host {
int load_cpt(const kmc_params* p, const char* path, kmc_state_view* v, std::string* err);
int write_cpt(const kmc_params* p, const kmc_state_view* v, const char* path, std::string* err);
int validate(const kmc_params* p, const kmc_state_view* v, std::string* err);
int init_random(const kmc_params* p, kmc_state_view* v, std::string* err);
int save_state(const kmc_params* p, const kmc_state_view* v, const char* path, std::string* err);
int load_state(const kmc_params* p, const char* path, kmc_state_view* v, std::string* err);
void derived_counts(const kmc_params* p, const kmc_state_view* v, int* rl, int* mono, int* cis);
int dd_check(int32_t n, const int32_t* gid, const uint8_t* own, std::string* err);
}  // namespace kmch_host

// host-only entry points (no device needed; also exported for tests)
extern "C" {
const char* kmc_host_last_error(void);
int kmc_host_load_cpt(const kmc_params* p, const char* path, kmc_state_view* v);
int kmc_host_write_cpt(const kmc_params* p, const kmc_state_view* v, const char* path);
int kmc_host_init_random(const kmc_params* p, kmc_state_view* v);
int kmc_host_save_state(const kmc_params* p, const kmc_state_view* v, const char* path);
int kmc_host_load_state(const kmc_params* p, const char* path, kmc_state_view* v);
int kmc_host_validate(const kmc_params* p, const kmc_state_view* v);
int kmc_host_dd_check(int32_t n, const int32_t* gid, const uint8_t* own);
int kmc_host_math(int op, const double* x, const double* y, double* out, int64_t n);
}
