// Front end of the gfx950 MFMA GEMM (the kernel: gemm5.hip).
//
//   C[M, N] = sum_k A[m, k] * B[k, n]      (fp32 accumulate)
//
// Each operand comes in one of two layouts, so every training GEMM of a
// linear layer runs WITHOUT a transposed copy:
//   KC  "k-contiguous":  A stored [M][K] / B stored [N][K]   (x, W of y = x W^T)
//   MC  "mn-contiguous": A stored [K][M] / B stored [K][N]   (W in dX = dY W,
//                                                              dY and x in dW = dY^T x)
// Epilogues (replacing reference K01/K02/K08; FusedLinear /
// fused_gemm_epilogue at `gpt/dygraph/single_model.py:29,81,375` and
// `language_model/utils.py:30-36`):
//   STORE      C = acc (+ bias[n])                      16-bit out
//   BIAS_GELU  aux = acc + bias ; C = gelu(aux)         FC1 forward (pre-activation kept for bwd)
//   DGELU      C = acc * gelu'(aux)                     FC2 data-gradient -> dH directly
//   F32        C32 = acc (+ C32 when beta)              weight gradient into fp32 main_grad
//
// This file only validates a call and fills GemmParams; every covered shape
// (K a multiple of 64, >= 128) runs on gemm5's hand-scheduled 4-wave kernel.
// Earlier kernel generations (8-wave, prefetching, persistent, 4-wave HIP)
// live in tools/gemm_lab/gemm_legacy.hip for lab A/Bs only.
#include <stdlib.h>

#include <map>
#include <tuple>
#include <vector>

#include "fx_common.h"
#include "gemm_common.h"

int fx_gemm5_launch(int dt, int la, int lb, int epi, const fxg::GemmParams& P, hipStream_t st);
long fx_gemm5_ws_bytes(int M, int N, int K);
void fx_gemm5_set_geom(int nf, int split);
void fx_gemm5_set_persist(int on);
void fx_gemm5_set_xrect(int on);

using namespace fxg;

static int g_gm = -1;  // FLEETX_GEMM_GM / fx_gemm_set_gm: force the tile-order M-group height

// Tile-order autotune (FLEETX_GEMM_TUNE, default on).  The M-group height
// `gm` of the tile order decides which A / B panels the 32 concurrent
// workgroups of an XCD share; the best value depends on the shape and the
// operand layouts (GPT-3 6.7B, one box: weight gradient of the QKV
// projection 1206 TF/s at gm 8 vs 1306 at gm 4, data gradient of FC1 1378 vs
// 1514 at gm 2, forward of QKV 1419 vs 1466 at gm 2; profiles/r4_gm/).  On a
// shape's first call outside stream capture, every candidate runs into a
// scratch output (fp32 / 16-bit store epilogue, beta 0, no norm partials)
// and the fastest is cached per (layouts, fp32 output, M, N, K).  The tile
// order never changes a tile's arithmetic: results are bitwise identical for
// every gm.
static int g_tune = -1;
static std::map<std::tuple<int, int, int, int, int, int>, int> g_gm_tuned;
// order codes: the M-group height, + 32 = within XCD rectangles, + 64 = the
// runner-up rectangle cut (gemm5.hip
// g5_tile_mn: each XCD's range of tile ids is one rectangle of the grid, so
// its L2 holds that rectangle's panels; 6.7B forward L2 misses -23 %,
// profiles/r5_xrect/)
static const int kGmCand[] = {1, 2, 4, 8, 16, 33, 34, 36, 40, 48, 97, 98, 100, 104};

static int gemm_tuned_gm(int dt, int la, int lb, int epi, const GemmParams& P0, hipStream_t st) {
  const int f32 = epi_wgrad(epi);
  const auto key = std::make_tuple(la, lb, f32, P0.M, P0.N, P0.K);
  auto it = g_gm_tuned.find(key);
  if (it != g_gm_tuned.end()) return it->second;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return 8;
  void* scratch = nullptr;
  if (hipMalloc(&scratch, (size_t)P0.M * P0.N * (f32 ? 4 : 2)) != hipSuccess) {
    (void)hipGetLastError();
    return 8;
  }
  GemmParams P = P0;
  P.C = scratch;
  P.ldc = P0.N;
  P.bias = nullptr;
  P.aux = nullptr;
  P.beta = 0;
  P.sq = nullptr;
  P.ctr = 0;
  const int tepi = f32 ? EPI_F32 : EPI_STORE;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  int best = 8;
  float bt = 1e30f;
  for (int gm : kGmCand) {
    P.gm = gm;
    if (fx_gemm5_launch(dt, la, lb, tepi, P, st) != 0) break;
    (void)hipEventRecord(e0, st);
    for (int r = 0; r < 3; ++r) (void)fx_gemm5_launch(dt, la, lb, tepi, P, st);
    (void)hipEventRecord(e1, st);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, e0, e1) == hipSuccess && ms < bt) {
      bt = ms;
      best = gm;
    }
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipFree(scratch);
  g_gm_tuned[key] = best;
  return best;
}

// Returns 0 when launched, < 0 when the shape / layout / epilogue is not
// covered (the caller falls back to hipBLASLt):
//   -1: K not a multiple of 64, < 128 or empty;  -2: an mn-contiguous extent
//   not a multiple of 8, or N not a multiple of 4;  -3: layout x epilogue
//   combo;  -4: an operand too large for 32-bit per-lane offsets;  -5: norm
//   partials requested outside the fp32 epilogue.
extern "C" int fx_gemm(int dt, int la, int lb, int epi, int M, int N, int K, const void* A,
                       long lda, const void* B, long ldb, void* C, long ldc, const void* bias,
                       void* aux, long ldaux, int beta, hipStream_t st, float* sq, float* ws) {
  int ctr = 0;
  if (epi == EPI_F32BT) {  // transposed 16-bit weight gradient: C[m][n] at C + n * ldc + m
    epi = EPI_F32B;
    ctr = 1;
  }
  if (M <= 0 || N <= 0 || K < 2 * BK || K % BK) return -1;
  if (sq != nullptr && !epi_wgrad(epi)) return -5;
  // 16-bit gradients accumulate (beta: micro-batches, pipeline schedules) in
  // the plain order only: one fp32 add + one rounding per write
  if (ctr && beta) return -6;
  if (N % 4 || (la == LAY_MC && M % 8) || (lb == LAY_MC && N % 8)) return -2;
  if (M < 8 || N < 8) return -2;
  const long a_span = la == LAY_KC ? (long)M * lda : (long)BK * lda + M;
  const long b_span = lb == LAY_KC ? (long)N * ldb : (long)BK * ldb + N;
  if (a_span >= (1L << 31) || b_span >= (1L << 31)) return -4;
  if ((long)(ctr ? N : M) * ldc * (epi == EPI_F32 ? 4 : 2) >= (1L << 31)) return -4;
  if (ctr && ldc < M) return -2;
  if (aux && (long)M * ldaux * 2 >= (1L << 31)) return -4;
  GemmParams P{};
  P.A = (const uint16_t*)A;
  P.B = (const uint16_t*)B;
  P.C = C;
  P.bias = (const uint16_t*)bias;
  P.aux = (uint16_t*)aux;
  P.lda = lda; P.ldb = ldb; P.ldc = ldc; P.ldaux = ldaux;
  P.M = M; P.N = N; P.K = K;
  P.beta = beta;
  P.sq = sq;
  P.ws = epi_wgrad(epi) ? ws : nullptr;
  P.ctr = ctr;
  if (g_gm < 0) {
    const char* e = getenv("FLEETX_GEMM_GM");
    g_gm = e ? atoi(e) : 0;
  }
  if (g_tune < 0) {
    const char* e = getenv("FLEETX_GEMM_TUNE");
    g_tune = e ? atoi(e) : 1;
  }
  P.gm = g_gm > 0 ? g_gm : (g_tune ? gemm_tuned_gm(dt, la, lb, epi, P, st) : 8);
  return fx_gemm5_launch(dt, la, lb, epi, P, st);
}

// Tile-order M-group height (tools/bench_gemm.py --gm sweeps; 0 = tuned / default).
extern "C" void fx_gemm_set_gm(int gm) { g_gm = gm > 0 ? gm : 0; }

// Shipped plan (fleetx_amd/ops/gemm_plan_gfx950.json, tools/gemm_plan.py):
// preload the tile order of a shape so its first call neither times
// candidates nor depends on box noise; a shape that is in the table is never
// re-tuned.
extern "C" void fx_gemm_set_tuned(int la, int lb, int f32, int M, int N, int K, int gm) {
  g_gm_tuned[std::make_tuple(la, lb, f32, M, N, K)] = gm;
}

// 0: no first-call tuning (shapes missing from the plan run gm 8:
// FLEETX_DETERMINISTIC); 1: tune them.  < 0 re-reads FLEETX_GEMM_TUNE.
extern "C" void fx_gemm_set_tune(int on) { g_tune = on; }

// Lab override of the tile geometry (4 / 8) and split-K slices (1 = none);
// 0 = the shape's plan.
extern "C" void fx_gemm_set_geom(int nf, int split) { fx_gemm5_set_geom(nf, split); }

// Persistent 16-bit launches on (1) / off (0, one workgroup per tile) for
// A/B runs and the bitwise test; < 0 = FLEETX_GEMM5_PERSIST.
extern "C" void fx_gemm_set_persist(int on) { fx_gemm5_set_persist(on); }

// XCD-rectangle tile mapping forced on (1) / off (2), 0 = per order code;
// < 0 = FLEETX_GEMM_XRECT
extern "C" void fx_gemm_set_xrect(int on) { fx_gemm5_set_xrect(on); }

// The tuned table: (la, lb, fp32 out, M, N, K, gm) rows, flattened.
extern "C" int fx_gemm_tuned(long* out, int cap) {
  int n = 0;
  for (const auto& kv : g_gm_tuned) {
    if (n + 7 > cap) break;
    out[n++] = std::get<0>(kv.first); out[n++] = std::get<1>(kv.first);
    out[n++] = std::get<2>(kv.first); out[n++] = std::get<3>(kv.first);
    out[n++] = std::get<4>(kv.first); out[n++] = std::get<5>(kv.first);
    out[n++] = kv.second;
  }
  return n / 7;
}

// Split-K workspace (bytes) fx_gemm wants in `ws` for an fp32 weight-gradient
// GEMM of this shape; 0 = it runs unsplit (gemm5.hip g5_split_plan).
extern "C" long fx_gemm_ws_bytes(int epi, int M, int N, int K) {
  if (!epi_wgrad(epi) || K < 2 * BK || K % BK) return 0;
  return fx_gemm5_ws_bytes(M, N, K);
}
