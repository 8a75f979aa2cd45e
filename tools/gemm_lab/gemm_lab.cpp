// Standalone GEMM lab: times fx_gemm (csrc/kernels/gemm.hip, compiled into this
// binary, optionally as an ablation build -DFX_GEMM_ABL=1|2) on the GPT-3 6.7B
// layer shapes with random bf16 operands.  Build: tools/gemm_lab/build.sh
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <string.h>

extern "C" int fx_gemm(int, int, int, int, int, int, int, const void*, long, const void*, long,
                       void*, long, const void*, void*, long, int, hipStream_t, float*, float*);
extern "C" void fx_gemm_set_variant(int);
extern "C" void fx_gemm_set_debug(unsigned long long*);

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

static void fill(uint16_t* d, size_t n, unsigned seed) {
  std::vector<uint16_t> h(n);
  unsigned s = seed * 2654435761u + 1;
  for (size_t i = 0; i < n; ++i) {
    s = s * 1664525u + 1013904223u;
    float f = ((s >> 8) * (1.0f / 16777216.0f)) * 2.f - 1.f;
    unsigned u; memcpy(&u, &f, 4);
    h[i] = (uint16_t)(u >> 16);
  }
  CK(hipMemcpy(d, h.data(), n * 2, hipMemcpyHostToDevice));
}

int main(int argc, char** argv) {
  const int variant = argc > 1 ? atoi(argv[1]) : 0;
  const int iters = argc > 2 ? atoi(argv[2]) : 20;
  const char* stamp_case = argc > 3 ? argv[3] : nullptr;  // e.g. "out:fwd": dump stamps
  fx_gemm_set_variant(variant);
  const int T = 8192, H = getenv("LAB_H") ? atoi(getenv("LAB_H")) : 4096;
  struct Sh { const char* name; int K, N; } shapes[] = {
      {"qkv", H, 3 * H}, {"out", H, H}, {"fc1", H, 4 * H}, {"fc2", 4 * H, H}};
  size_t maxe = (size_t)T * 4 * H;
  uint16_t *x, *w, *dy, *c16, *aux;
  float* c32;
  CK(hipMalloc(&x, maxe * 2)); CK(hipMalloc(&w, maxe * 2)); CK(hipMalloc(&dy, maxe * 2));
  CK(hipMalloc(&c16, maxe * 2)); CK(hipMalloc(&aux, maxe * 2)); CK(hipMalloc(&c32, maxe * 4));
  fill(x, maxe, 1); fill(w, maxe, 2); fill(dy, maxe, 3); fill(aux, maxe, 4);
  CK(hipMemset(c32, 0, maxe * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (auto& s : shapes) {
    const int M = T, N = s.N, K = s.K;
    const double fl = 2.0 * M * N * K;
    // fwd: C[M,N] = x[M,K] w[N,K]^T ; dgrad: C[M,K] = dy[M,N] w[N,K] ; wgrad: C[N,K] = dy^T x
    struct Case { const char* nm; int la, lb, epi, m, n, k; const void* A; long lda; const void* B; long ldb; void* C; long ldc; } cases[] = {
        {"fwd", 0, 0, 0, M, N, K, x, K, w, K, c16, N},
        {"fwd_gelu", 0, 0, 1, M, N, K, x, K, w, K, c16, N},
        {"dgrad", 0, 1, 0, M, K, N, dy, N, w, K, c16, K},
        {"dgrad_dgelu", 0, 1, 2, M, K, N, dy, N, w, K, c16, K},
        {"wgrad", 1, 1, 3, N, K, M, dy, N, x, K, c32, K},
    };
    printf("{\"gemm\": \"%s\"", s.name);
    for (auto& c : cases) {
      const char* only = getenv("LAB_ONLY");  // e.g. "fc1:fwd"
      if (only) {
        char want[64];
        snprintf(want, sizeof(want), "%s:%s", s.name, c.nm);
        if (strcmp(want, only)) continue;
      }
      auto run = [&]() {
        int rc = fx_gemm(0, c.la, c.lb, c.epi, c.m, c.n, c.k, c.A, c.lda, c.B, c.ldb, c.C, c.ldc,
                         nullptr, aux, c.n, 1, 0, nullptr, nullptr);
        if (rc) { printf("rc %d\n", rc); exit(1); }
      };
      for (int i = 0; i < 3; ++i) run();
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < iters; ++i) run();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      printf(", \"%s\": %.1f", c.nm, fl / (ms / iters * 1e-3) / 1e12);
      if (getenv("LAB_HASH")) {
        // output checksum of one launch into a zeroed C: schedule variants of
        // the same kernel accumulate in the same order, so equal hashes
        const size_t bytes = (size_t)c.m * c.ldc * (c.epi == 3 ? 4 : 2);
        CK(hipMemset(c.C, 0, bytes));
        run();
        CK(hipDeviceSynchronize());
        std::vector<unsigned char> hb(bytes);
        CK(hipMemcpy(hb.data(), c.C, bytes, hipMemcpyDeviceToHost));
        unsigned long long hsh = 1469598103934665603ull;
        for (size_t i = 0; i < bytes; ++i) hsh = (hsh ^ hb[i]) * 1099511628211ull;
        printf(", \"%s_h\": \"%016llx\"", c.nm, hsh);
      }
      if (stamp_case) {
        char want[64];
        snprintf(want, sizeof(want), "%s:%s", s.name, c.nm);
        if (!strcmp(want, stamp_case)) {
          const int nst = 8 * 8 * 4 * 6;  // also covers 4 waves x 8 K-tiles x 8 stamps
          unsigned long long* d;
          CK(hipMalloc(&d, nst * 8));
          CK(hipMemset(d, 0, nst * 8));
          fx_gemm_set_debug(d);
          run();
          CK(hipDeviceSynchronize());
          fx_gemm_set_debug(nullptr);
          std::vector<unsigned long long> h(nst);
          CK(hipMemcpy(h.data(), d, nst * 8, hipMemcpyDeviceToHost));
          FILE* f = fopen("gpurun_out/stamps.txt", "w");
          for (int i = 0; i < nst; ++i) fprintf(f, "%llu\n", h[i]);
          fclose(f);
        }
      }
    }
    printf("}\n");
    fflush(stdout);
  }
  return 0;
}
