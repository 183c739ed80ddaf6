// Microbenchmark (diagnostic, not product): the free-unit proposal's memory
// pattern — one thread per protein reads 24 double2 rows of R and writes 24
// rows of R_new — in the engine's row-major SoA (element (row r, slot i) at
// r*n + i), in a 64-protein-block AoSoA layout, and as a plain linear copy of
// the same bytes.  hipcc --offload-arch=gfx950 -O3 rows_copy.hip -o rows_copy
#include <hip/hip_runtime.h>
#include <cstdio>
#define ROWS 24
typedef double dv2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ double2 ldn(const double2* p) { dv2 v = __builtin_nontemporal_load((const dv2*)p); return make_double2(v.x, v.y); }
__device__ __forceinline__ void stn(double2* p, double2 v) { dv2 w; w.x = v.x; w.y = v.y; __builtin_nontemporal_store(w, (dv2*)p); }
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

__global__ void __launch_bounds__(256) soa(const double2* __restrict__ a, double2* __restrict__ b, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double2 r[ROWS];
#pragma unroll
  for (int k = 0; k < ROWS; ++k) r[k] = ldn(&a[(size_t)k * n + i]);
#pragma unroll
  for (int k = 0; k < ROWS; ++k) { r[k].x += 1.0; stn(&b[(size_t)k * n + i], r[k]); }
}
__global__ void __launch_bounds__(256) soa_plain(const double2* __restrict__ a, double2* __restrict__ b, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double2 r[ROWS];
#pragma unroll
  for (int k = 0; k < ROWS; ++k) r[k] = a[(size_t)k * n + i];
#pragma unroll
  for (int k = 0; k < ROWS; ++k) { r[k].x += 1.0; b[(size_t)k * n + i] = r[k]; }
}
__global__ void __launch_bounds__(256) aosoa(const double2* __restrict__ a, double2* __restrict__ b, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const size_t base = (size_t)(i >> 6) * ROWS * 64 + (i & 63);
  double2 r[ROWS];
#pragma unroll
  for (int k = 0; k < ROWS; ++k) r[k] = ldn(&a[base + k * 64]);
#pragma unroll
  for (int k = 0; k < ROWS; ++k) { r[k].x += 1.0; stn(&b[base + k * 64], r[k]); }
}
__global__ void __launch_bounds__(256) linear(const double2* __restrict__ a, double2* __restrict__ b, size_t m) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < m; i += (size_t)gridDim.x * blockDim.x) {
    double2 v = a[i];
    v.x += 1.0;
    b[i] = v;
  }
}

int main() {
  const int n = 750000;  // C3 receptors
  const size_t m = (size_t)ROWS * n;
  double2 *a, *b;
  CHK(hipMalloc(&a, m * sizeof(double2)));
  CHK(hipMalloc(&b, m * sizeof(double2)));
  CHK(hipMemset(a, 0, m * sizeof(double2)));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  const char* names[4] = {"soa_nt", "soa_plain", "aosoa_nt", "linear"};
  for (int v = 0; v < 4; ++v) {
    float best = 1e9;
    for (int rep = 0; rep < 20; ++rep) {
      CHK(hipEventRecord(e0));
      if (v == 0) soa<<<(n + 255) / 256, 256>>>(a, b, n);
      if (v == 1) soa_plain<<<(n + 255) / 256, 256>>>(a, b, n);
      if (v == 2) aosoa<<<(n + 255) / 256, 256>>>(a, b, n);
      if (v == 3) linear<<<4096, 256>>>(a, b, m);
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float ms;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      if (rep > 2 && ms < best) best = ms;
    }
    printf("%-10s %8.1f us  %6.2f TB/s\n", names[v], best * 1e3, 2.0 * m * 16 / (best * 1e-3) / 1e12);
  }
  return 0;
}
