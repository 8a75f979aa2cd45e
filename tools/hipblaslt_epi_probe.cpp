// Probe: do hipBLASLt's GELU epilogues pay on gfx950 for the MLP GEMMs?
//   fc1 forward  Y = gelu(X W1^T + b1), aux = X W1^T + b1  (GELU_AUX_BIAS)
//   fc2 dgrad    dPre = (dY W2) * gelu'(aux), db1 = colsum  (DGELU_BGRAD)
// against the plain GEMMs (the separate bias+GeLU passes cost what
// profiles/r4_prof says they cost).  Also checks the epilogue's GeLU form
// against tanh-GeLU on a small shape.
//   hipcc --offload-arch=gfx950 -O2 tools/hipblaslt_epi_probe.cpp -lhipblaslt -o /tmp/probe
//   ./probe M H F
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <hipblaslt/hipblaslt.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    auto e_ = (x);                                                                 \
    if ((int)e_ != 0) {                                                            \
      fprintf(stderr, "%s:%d %s -> %d\n", __FILE__, __LINE__, #x, (int)e_);       \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

static hipblasLtHandle_t H_;
static void* g_ws;
static const size_t WS = 64ull << 20;

struct Gemm {
  hipblasLtMatmulDesc_t d;
  hipblasLtMatrixLayout_t la, lb, lc;
  hipblasLtMatmulAlgo_t algo;
  bool ok = false;
};

// column-major: D[m,n] = op(A) op(B); A is m x k (opA = T: stored k x m, ld k)
static Gemm make(int m, int n, int k, hipblasOperation_t ta, int lda, int ldb, int ldd,
                 hipblasLtEpilogue_t epi, void* bias, hipDataType bias_t, void* aux, long aux_ld) {
  Gemm g;
  CK(hipblasLtMatmulDescCreate(&g.d, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  hipblasOperation_t tb = HIPBLAS_OP_N;
  CK(hipblasLtMatmulDescSetAttribute(g.d, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
  CK(hipblasLtMatmulDescSetAttribute(g.d, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
  CK(hipblasLtMatmulDescSetAttribute(g.d, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi)));
  if (bias) {
    CK(hipblasLtMatmulDescSetAttribute(g.d, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)));
    CK(hipblasLtMatmulDescSetAttribute(g.d, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bias_t,
                                       sizeof(bias_t)));
  }
  if (aux) {
    CK(hipblasLtMatmulDescSetAttribute(g.d, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, &aux,
                                       sizeof(aux)));
    int64_t ld = aux_ld;
    CK(hipblasLtMatmulDescSetAttribute(g.d, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &ld, sizeof(ld)));
  }
  const int ar = ta == HIPBLAS_OP_T ? k : m, ac = ta == HIPBLAS_OP_T ? m : k;
  CK(hipblasLtMatrixLayoutCreate(&g.la, HIP_R_16BF, ar, ac, lda));
  CK(hipblasLtMatrixLayoutCreate(&g.lb, HIP_R_16BF, k, n, ldb));
  CK(hipblasLtMatrixLayoutCreate(&g.lc, HIP_R_16BF, m, n, ldd));
  hipblasLtMatmulPreference_t pref;
  CK(hipblasLtMatmulPreferenceCreate(&pref));
  size_t ws = WS;
  CK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws,
                                           sizeof(ws)));
  hipblasLtMatmulHeuristicResult_t res[8];
  int nres = 0;
  auto st = hipblasLtMatmulAlgoGetHeuristic(H_, g.d, g.la, g.lb, g.lc, g.lc, pref, 8, res, &nres);
  if (st == HIPBLAS_STATUS_SUCCESS && nres > 0) {
    g.algo = res[0].algo;
    g.ok = true;
  }
  printf("  heuristic epi=%d -> status %d, %d algos\n", (int)epi, (int)st, nres);
  return g;
}

static float run(Gemm& g, const void* A, const void* B, void* D, int iters, hipStream_t s) {
  const float one = 1.f, zero = 0.f;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i)
    CK(hipblasLtMatmul(H_, g.d, &one, A, g.la, B, g.lb, &zero, D, g.lc, D, g.lc, &g.algo, g_ws, WS, s));
  CK(hipEventRecord(e0, s));
  for (int i = 0; i < iters; ++i)
    CK(hipblasLtMatmul(H_, g.d, &one, A, g.la, B, g.lb, &zero, D, g.lc, D, g.lc, &g.algo, g_ws, WS, s));
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / iters * 1e3f;  // us
}

static void fill(std::vector<__hip_bfloat16>& v, float sc, unsigned seed) {
  srand(seed);
  for (auto& x : v) x = __float2bfloat16(sc * ((float)rand() / RAND_MAX - 0.5f));
}
static float gelu_tanh(float x) {
  return 0.5f * x * (1.f + tanhf(0.7978845608f * (x + 0.044715f * x * x * x)));
}
static float gelu_tanh_grad(float x) {
  const float t = tanhf(0.7978845608f * (x + 0.044715f * x * x * x));
  return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * 0.7978845608f * (1.f + 3 * 0.044715f * x * x);
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 8192, Hd = argc > 2 ? atoi(argv[2]) : 4096,
            F = argc > 3 ? atoi(argv[3]) : 16384;
  CK(hipblasLtCreate(&H_));
  CK(hipMalloc(&g_ws, WS));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  // ---------------- numerics on a small shape: GELU form of the epilogue
  {
    const int m = 256, n = 128, k = 64;  // D[m=F, n=tokens] = W1[m,k] X^T[k,n]
    std::vector<__hip_bfloat16> w(m * k), x(k * n), b(m);
    fill(w, 2.f, 1);
    fill(x, 2.f, 2);
    fill(b, 1.f, 3);
    void *dw, *dx, *db, *dy, *daux;
    CK(hipMalloc(&dw, w.size() * 2));
    CK(hipMalloc(&dx, x.size() * 2));
    CK(hipMalloc(&db, b.size() * 2));
    CK(hipMalloc(&dy, (size_t)m * n * 2));
    CK(hipMalloc(&daux, (size_t)m * n * 2));
    CK(hipMemcpy(dw, w.data(), w.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dx, x.data(), x.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, b.data(), b.size() * 2, hipMemcpyHostToDevice));
    // W1 stored row-major [m][k] = column-major k x m, ld k: opA = T
    Gemm g = make(m, n, k, HIPBLAS_OP_T, k, k, m, HIPBLASLT_EPILOGUE_GELU_AUX_BIAS, db, HIP_R_16BF,
                  daux, m);
    if (g.ok) {
      run(g, dw, dx, dy, 1, s);
      std::vector<__hip_bfloat16> y(m * n), aux(m * n);
      CK(hipMemcpy(y.data(), dy, y.size() * 2, hipMemcpyDeviceToHost));
      CK(hipMemcpy(aux.data(), daux, aux.size() * 2, hipMemcpyDeviceToHost));
      double et = 0, ee = 0, ea = 0, ny = 0;
      for (int j = 0; j < n; ++j)
        for (int i = 0; i < m; ++i) {
          float acc = __bfloat162float(b[i]);
          for (int kk = 0; kk < k; ++kk)
            acc += __bfloat162float(w[i * k + kk]) * __bfloat162float(x[j * k + kk]);
          const float yt = gelu_tanh(acc), ye = 0.5f * acc * (1.f + erff(acc * 0.70710678f));
          const float got = __bfloat162float(y[j * m + i]);
          et += (got - yt) * (got - yt);
          ee += (got - ye) * (got - ye);
          ea += pow(__bfloat162float(aux[j * m + i]) - acc, 2);
          ny += yt * yt;
        }
      printf("gelu epilogue: rel err vs tanh %.3e, vs erf %.3e; aux rel err %.3e\n",
             sqrt(et / ny), sqrt(ee / ny), sqrt(ea / ny));
    }
    // DGELU_BGRAD: D[m=F, n] = dgelu(W2^T-ish product, aux); here A = W (m x k col-major)
    {
      std::vector<__hip_bfloat16> a(m * k), gy(k * n), aux(m * n);
      fill(a, 2.f, 4);
      fill(gy, 2.f, 5);
      fill(aux, 4.f, 6);
      void *da, *dg, *dax, *dd, *dbg;
      CK(hipMalloc(&da, a.size() * 2));
      CK(hipMalloc(&dg, gy.size() * 2));
      CK(hipMalloc(&dax, aux.size() * 2));
      CK(hipMalloc(&dd, (size_t)m * n * 2));
      CK(hipMalloc(&dbg, (size_t)m * 4));
      CK(hipMemcpy(da, a.data(), a.size() * 2, hipMemcpyHostToDevice));
      CK(hipMemcpy(dg, gy.data(), gy.size() * 2, hipMemcpyHostToDevice));
      CK(hipMemcpy(dax, aux.data(), aux.size() * 2, hipMemcpyHostToDevice));
      for (hipDataType bt : {HIP_R_32F, HIP_R_16BF}) {
        Gemm g2 = make(m, n, k, HIPBLAS_OP_N, m, k, m, HIPBLASLT_EPILOGUE_DGELU_BGRAD, dbg, bt, dax,
                       m);
        if (!g2.ok) continue;
        run(g2, da, dg, dd, 1, s);
        std::vector<__hip_bfloat16> d(m * n);
        std::vector<float> bgf(m);
        std::vector<__hip_bfloat16> bgh(m);
        CK(hipMemcpy(d.data(), dd, d.size() * 2, hipMemcpyDeviceToHost));
        if (bt == HIP_R_32F) CK(hipMemcpy(bgf.data(), dbg, m * 4, hipMemcpyDeviceToHost));
        else CK(hipMemcpy(bgh.data(), dbg, m * 2, hipMemcpyDeviceToHost));
        double e = 0, nd = 0, eb = 0, nb = 0;
        std::vector<double> colsum(m, 0.0);
        for (int j = 0; j < n; ++j)
          for (int i = 0; i < m; ++i) {
            float acc = 0;
            for (int kk = 0; kk < k; ++kk)
              acc += __bfloat162float(a[kk * m + i]) * __bfloat162float(gy[j * k + kk]);
            const float ref = acc * gelu_tanh_grad(__bfloat162float(aux[j * m + i]));
            e += pow(__bfloat162float(d[j * m + i]) - ref, 2);
            nd += ref * ref;
            colsum[i] += ref;
          }
        for (int i = 0; i < m; ++i) {
          const float got = bt == HIP_R_32F ? bgf[i] : __bfloat162float(bgh[i]);
          eb += pow(got - colsum[i], 2);
          nb += colsum[i] * colsum[i];
        }
        printf("dgelu_bgrad (bias type %d): rel err %.3e, bias-grad rel err %.3e\n", (int)bt,
               sqrt(e / nd), sqrt(eb / nb));
      }
    }
  }
  // ---------------- timing at the model shape
  {
    void *X, *W1, *b1, *Y, *AUX, *W2, *GY, *DP, *BG;
    CK(hipMalloc(&X, (size_t)M * Hd * 2));
    CK(hipMalloc(&W1, (size_t)F * Hd * 2));
    CK(hipMalloc(&b1, (size_t)F * 2));
    CK(hipMalloc(&Y, (size_t)M * F * 2));
    CK(hipMalloc(&AUX, (size_t)M * F * 2));
    CK(hipMalloc(&W2, (size_t)Hd * F * 2));
    CK(hipMalloc(&GY, (size_t)M * Hd * 2));
    CK(hipMalloc(&DP, (size_t)M * F * 2));
    CK(hipMalloc(&BG, (size_t)F * 4));
    CK(hipMemset(X, 0, (size_t)M * Hd * 2));
    CK(hipMemset(W1, 0, (size_t)F * Hd * 2));
    CK(hipMemset(b1, 0, (size_t)F * 2));
    CK(hipMemset(W2, 0, (size_t)F * Hd * 2));
    CK(hipMemset(GY, 0, (size_t)M * Hd * 2));
    CK(hipMemset(AUX, 0, (size_t)M * F * 2));
    const double fl = 2.0 * M * Hd * F;
    // fc1 fwd: D[F, M] = W1 (stored [F][Hd] -> col-major Hd x F, opA = T) x X^T (Hd x M)
    Gemm p = make(F, M, Hd, HIPBLAS_OP_T, Hd, Hd, F, HIPBLASLT_EPILOGUE_DEFAULT, nullptr, HIP_R_16BF,
                  nullptr, 0);
    Gemm pb = make(F, M, Hd, HIPBLAS_OP_T, Hd, Hd, F, HIPBLASLT_EPILOGUE_BIAS, b1, HIP_R_16BF,
                   nullptr, 0);
    Gemm ga = make(F, M, Hd, HIPBLAS_OP_T, Hd, Hd, F, HIPBLASLT_EPILOGUE_GELU_AUX_BIAS, b1,
                   HIP_R_16BF, AUX, F);
    // fc2 dgrad: dPre[F, M] = W2 (stored [Hd][F] -> col-major F x Hd, opA = N) x dY^T (Hd x M)
    Gemm d = make(F, M, Hd, HIPBLAS_OP_N, F, Hd, F, HIPBLASLT_EPILOGUE_DEFAULT, nullptr, HIP_R_16BF,
                  nullptr, 0);
    Gemm dg = make(F, M, Hd, HIPBLAS_OP_N, F, Hd, F, HIPBLASLT_EPILOGUE_DGELU_BGRAD, BG, HIP_R_32F,
                   AUX, F);
    Gemm dg16 = make(F, M, Hd, HIPBLAS_OP_N, F, Hd, F, HIPBLASLT_EPILOGUE_DGELU_BGRAD, BG,
                     HIP_R_16BF, AUX, F);
    struct {
      const char* name;
      Gemm* g;
      const void *A, *B;
      void* D;
    } cases[] = {{"fc1 fwd plain", &p, W1, X, Y},
                 {"fc1 fwd +bias", &pb, W1, X, Y},
                 {"fc1 fwd gelu_aux_bias", &ga, W1, X, Y},
                 {"fc2 dgrad plain", &d, W2, GY, DP},
                 {"fc2 dgrad dgelu_bgrad f32", &dg, W2, GY, DP},
                 {"fc2 dgrad dgelu_bgrad bf16", &dg16, W2, GY, DP}};
    for (auto& c : cases) {
      if (!c.g->ok) {
        printf("{\"case\": \"%s\", \"M\": %d, \"H\": %d, \"F\": %d, \"us\": null}\n", c.name, M, Hd, F);
        continue;
      }
      float us = run(*c.g, c.A, c.B, c.D, 20, s);
      printf("{\"case\": \"%s\", \"M\": %d, \"H\": %d, \"F\": %d, \"us\": %.1f, \"tflops\": %.0f}\n",
             c.name, M, Hd, F, us, fl / us * 1e-6);
    }
  }
  return 0;
}
