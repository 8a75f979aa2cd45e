// Grid-barrier cost on MI355X: one workgroup per CU, NB back-to-back barriers,
// flat (every workgroup bumps one counter) vs two-level (a counter per group
// of 32 workgroups, the group's last arrival bumps the global one).
//   hipcc -O3 --offload-arch=gfx950 barrier_lab.hip -o barrier_lab && ./barrier_lab
#include <hip/hip_runtime.h>
#include <stdio.h>

__device__ __forceinline__ void bar_flat(unsigned* c, unsigned target, int* err) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int spins = 0;
    while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1 << 22)) { *err = 1; break; }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
}

__device__ __forceinline__ void bar_two(unsigned* grp, unsigned* glob, unsigned k, int* err) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const int G = gridDim.x, g = blockIdx.x & 7, per = G / 8;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const unsigned t = __hip_atomic_fetch_add(grp + 64 * g, 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    if (t + 1 == k * per) __hip_atomic_fetch_add(glob, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int spins = 0;
    while (__hip_atomic_load(glob, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < k * 8) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1 << 22)) { *err = 1; break; }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
}

__global__ __launch_bounds__(256) void k_flat(unsigned* c, int nb, int* err) {
  for (int i = 1; i <= nb; ++i) bar_flat(c, i * gridDim.x, err);
}
__global__ __launch_bounds__(256) void k_two(unsigned* grp, unsigned* glob, int nb, int* err) {
  for (int i = 1; i <= nb; ++i) bar_two(grp, glob, i, err);
}
__global__ void k_empty() {}

int main() {
  int dev = 0, ncu = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const int G = ncu / 8 * 8, NB = 200;
  unsigned *c, *grp, *glob;
  int* err;
  hipMalloc(&c, 4096); hipMalloc(&grp, 8 * 64 * 4); hipMalloc(&glob, 256); hipMalloc(&err, 4);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  for (int rep = 0; rep < 3; ++rep) {
    float ms;
    hipMemset(c, 0, 4096); hipMemset(err, 0, 4);
    hipEventRecord(a);
    k_flat<<<G, 256>>>(c, NB, err);
    hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
    int e; hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost);
    printf("{\"barrier\": \"flat\", \"grid\": %d, \"us_per_barrier\": %.2f, \"err\": %d}\n", G, 1000 * ms / NB, e);
    hipMemset(grp, 0, 8 * 64 * 4); hipMemset(glob, 0, 256); hipMemset(err, 0, 4);
    hipEventRecord(a);
    k_two<<<G, 256>>>(grp, glob, NB, err);
    hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
    hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost);
    printf("{\"barrier\": \"two-level\", \"grid\": %d, \"us_per_barrier\": %.2f, \"err\": %d}\n", G, 1000 * ms / NB, e);
    // kernel boundary for comparison: NB empty dependent launches
    hipEventRecord(a);
    for (int i = 0; i < NB; ++i) k_empty<<<G, 256>>>();
    hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
    printf("{\"barrier\": \"kernel-boundary (empty launches, stream)\", \"grid\": %d, \"us_per_barrier\": %.2f}\n", G, 1000 * ms / NB);
  }
  return 0;
}
