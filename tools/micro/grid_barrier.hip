// Microbenchmark (diagnostic, not product): what a phase boundary costs on
// MI355X — a dependent kernel launch on one stream against a grid barrier
// inside one cooperative launch — with and without dirty data written in
// the phase (the barrier's release must make it visible across the XCDs'
// L2s, as a kernel boundary does).
//   hipcc --offload-arch=gfx950 -O3 grid_barrier.hip -o grid_barrier
// Every spin is bounded (a barrier that never completes sets a flag and lets
// the wave leave), and the cooperative launch refuses a grid that cannot be
// co-resident.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CHK(x)                                                 \
  do {                                                         \
    hipError_t e = (x);                                        \
    if (e != hipSuccess) {                                     \
      printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      return 1;                                                \
    }                                                          \
  } while (0)

struct Bar {
  unsigned count;
  unsigned timeout;
};

// write `words` ints per phase, spread over the grid (dirty L2 lines)
__device__ __forceinline__ void phase_work(int* buf, int words, int phase) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < words; i += gridDim.x * blockDim.x) buf[i] = phase + i;
}

__global__ void __launch_bounds__(256) k_phase(int* buf, int words, int phase) { phase_work(buf, words, phase); }

// monotone counter barrier: phase k completes when the counter reaches
// gridDim.x * (k + 1)
__device__ __forceinline__ void grid_barrier(Bar* b, unsigned target) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(&b->count, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    unsigned spins = 0;
    while (__hip_atomic_load(&b->count, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 24)) {
        __hip_atomic_fetch_add(&b->timeout, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
}

__global__ void __launch_bounds__(256) k_persist(int* buf, int words, int nphase, Bar* b) {
  for (int k = 0; k < nphase; ++k) {
    phase_work(buf, words, k);
    grid_barrier(b, gridDim.x * (unsigned)(k + 1));
  }
}

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  int* buf;
  Bar* bar;
  CHK(hipMalloc(&buf, 64 << 20));
  CHK(hipMalloc(&bar, sizeof(Bar)));
  hipStream_t st;
  CHK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  const int nphase = 40, reps = 5;
  int occ = 0;
  CHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_persist, 256, 0));
  printf("CUs %d, co-resident 256-thread workgroups per CU %d\n", ncu, occ);
  for (int words : {0, 1 << 14, 1 << 18, 1 << 22}) {
    // chain of dependent launches
    float best = 1e30f;
    for (int r = 0; r < reps; ++r) {
      CHK(hipEventRecord(e0, st));
      for (int k = 0; k < nphase; ++k) k_phase<<<2048, 256, 0, st>>>(buf, words, k);
      CHK(hipEventRecord(e1, st));
      CHK(hipEventSynchronize(e1));
      float ms;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    printf("words %8d  launches: %.2f us/phase\n", words, 1e3f * best / nphase);
    for (int per : {1, 2, 4}) {
      if (per > occ) continue;
      const int g = ncu * per;
      best = 1e30f;
      Bar zero{0, 0};
      for (int r = 0; r < reps; ++r) {
        CHK(hipMemcpyAsync(bar, &zero, sizeof zero, hipMemcpyHostToDevice, st));
        int np = nphase;
        void* args[] = {&buf, &words, &np, &bar};
        CHK(hipEventRecord(e0, st));
        CHK(hipLaunchCooperativeKernel((const void*)k_persist, dim3(g), dim3(256), args, 0, st));
        CHK(hipEventRecord(e1, st));
        CHK(hipEventSynchronize(e1));
        float ms;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
      }
      Bar h;
      CHK(hipMemcpy(&h, bar, sizeof h, hipMemcpyDeviceToHost));
      printf("words %8d  barrier, %4d WGs: %.2f us/phase (timeouts %u)\n", words, g, 1e3f * best / nphase,
             h.timeout);
    }
  }
  return 0;
}
