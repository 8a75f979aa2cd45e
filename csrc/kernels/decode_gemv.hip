// Skinny GEMM for decoding: y[M, N] = x[M, K] W[N, K]^T, M <= 16, with the
// decoder layer's element-wise work fused into the epilogue.
//
// Reference K19 / N-12: the inference program's
// fused_multi_transformer (`core/engine/inference_engine.py:103-109,127-129`).
// At decode batch sizes a decoder layer is four weight-streaming GEMVs; every
// weight byte is read once per token, so the layer is bound by HBM bandwidth
// and the goal is to stream W at the roofline while the small activations
// come from L2.  Epilogues turn each GEMV into a whole sub-layer:
//   EPI_BIAS      y = acc + b                               (out-proj, LM head)
//   EPI_GELU      y = gelu_tanh(acc + b)                    (FFN1)
//   EPI_RES       y = acc + b + res                         (FFN2 + residual)
//   EPI_QKV       acc + b scattered to q[M, H, D] and the KV cache at this
//                 token's position (k/v_cache[M, maxlen, H, D])   (QKV + cache append)
//
// CDNA4 mapping (cdna_hip_programming.md §5, "GEMV / M <= 16 decode weights":
// operand streamed once per block -> straight to VGPRs, deep unroll):
//  * a block owns 16 output columns (rows of W) and splits K over its 4
//    waves; each wave runs v_mfma_f32_16x16x32 with A = 16 W rows, B = 16 x
//    rows (rows >= M repeat row M-1 and are never stored).  (A cross-block
//    K split with an agent-scope slab reduction measured 2-10x SLOWER here:
//    the release/acquire pair per block costs more than the latency it
//    hides -- tools/bench_gemv.py, profiles/r2_decode/);
//  * per 64-k chunk every lane loads 32 CONTIGUOUS bytes of one W row (lane
//    group g = lane/16 covers bytes 32g..32g+31), so one wave instruction pair
//    reads 16 full 128-byte row segments; the two MFMA k-steps use the
//    matching permutation of k for x (a sum is order-free in k);
//  * loads run in batches of U = 4 or 8 64-k chunks on two register sets:
//    batch c+1 is in flight while batch c feeds the MFMAs;
//  * the 4 wave partials are summed through LDS and the epilogue runs one
//    output element per thread.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <type_traits>

#include "fx_common.h"

namespace {

enum { GV_BIAS = 0, GV_GELU = 1, GV_RES = 2, GV_QKV = 3 };

struct GemvArgs {
  const uint16_t* x;
  const uint16_t* w;
  const uint16_t* bias;
  const uint16_t* res;
  uint16_t* y;
  long ldx, ldw, ldy, ldres;
  int M, N, K;
  // QKV scatter
  uint16_t* kc;
  uint16_t* vc;
  const long* pos;
  int heads, head_dim, maxlen;
  // optional LayerNorm of x fused as a prologue (LN1 -> QKV, LN2 -> FFN1)
  const uint16_t* ln_w;
  const uint16_t* ln_b;
  float ln_eps;
};

template <typename T>
__device__ __forceinline__ floatx4 mma16(const short8& a, const short8& b, const floatx4& c) {
  if constexpr (std::is_same<T, bf16>::value)
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}

template <int U>
__device__ __forceinline__ void load_w(short8 (&wv)[U][2], const uint16_t* wp, int c) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const short8* p = reinterpret_cast<const short8*>(wp + (c + u) * 64);
    wv[u][0] = __builtin_nontemporal_load(p);
    wv[u][1] = __builtin_nontemporal_load(p + 1);
  }
}
// x operand: global (L2-resident activations) or, with the fused LayerNorm,
// the normalised rows staged in LDS (address space 3 -> ds_read_b128)
template <int U, bool XL>
__device__ __forceinline__ void load_x(short8 (&xv)[U][2], const uint16_t* xp, int c) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if constexpr (XL) {
      const __attribute__((address_space(3))) short8* p =
          (const __attribute__((address_space(3))) short8*)(xp + (c + u) * 64);
      xv[u][0] = p[0];
      xv[u][1] = p[1];
    } else {
      const short8* p = reinterpret_cast<const short8*>(xp + (c + u) * 64);
      xv[u][0] = p[0];
      xv[u][1] = p[1];
    }
  }
}
template <int U, bool XL>
__device__ __forceinline__ void load_batch(short8 (&wv)[U][2], short8 (&xv)[U][2],
                                           const uint16_t* wp, const uint16_t* xp, int c) {
  load_w<U>(wv, wp, c);
  load_x<U, XL>(xv, xp, c);
}

// Fused LayerNorm prologue: rows m < M of x [M, K] normalised (fp32 math,
// shifted one-pass moments: the row's first element is subtracted before the
// sums, so E[d^2] - E[d]^2 does not cancel) and stored as 16-bit rows in LDS.
// Every block recomputes the statistics of the same few rows (K * M * 2 bytes
// from L2) -- cheaper than a separate LayerNorm launch at decode sizes.
template <typename T, int NT, int MR>
__device__ __forceinline__ void ln_prologue(const GemvArgs& a, uint16_t* xs, float* scratch) {
  // MR >= M rows (1 / 4 / 16, chosen on the host); the loops over rows are
  // unrolled so the loads of every row are in flight together
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  constexpr int NW = NT / 64;
  const int K = a.K, nch = K / 8, M = a.M;
  float sh[MR], s1[MR], s2[MR];
#pragma unroll
  for (int m = 0; m < MR; ++m) {
    sh[m] = m < M ? Elt<T>::to_f(a.x[(long)m * a.ldx]) : 0.f;
    s1[m] = s2[m] = 0.f;
  }
  for (int c = t; c < nch; c += NT) {
    uint4 raw[MR];
#pragma unroll
    for (int m = 0; m < MR; ++m)
      if (m < M) raw[m] = *reinterpret_cast<const uint4*>(a.x + (long)m * a.ldx + c * 8);
#pragma unroll
    for (int m = 0; m < MR; ++m) {
      if (m >= M) continue;
      float v[8];
      unpack8<T>(raw[m], v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[j] - sh[m];
        s1[m] += d;
        s2[m] += d * d;
      }
    }
  }
#pragma unroll
  for (int m = 0; m < MR; ++m) {
    if (m >= M) continue;
    const float r1 = wave_sum(s1[m]), r2 = wave_sum(s2[m]);
    if (lane == 0) {
      scratch[(2 * m) * NW + w] = r1;
      scratch[(2 * m + 1) * NW + w] = r2;
    }
  }
  __syncthreads();
  float mean[MR], rstd[MR];
#pragma unroll
  for (int m = 0; m < MR; ++m) {
    float r1 = 0.f, r2 = 0.f;
    if (m < M) {
#pragma unroll
      for (int i = 0; i < NW; ++i) {
        r1 += scratch[(2 * m) * NW + i];
        r2 += scratch[(2 * m + 1) * NW + i];
      }
    }
    const float md = r1 / K;
    mean[m] = sh[m] + md;
    rstd[m] = rsqrtf(fmaxf(r2 / K - md * md, 0.f) + a.ln_eps);
  }
  for (int c = t; c < nch; c += NT) {
    float gw[8], gb[8];
    load8<T>(a.ln_w + c * 8, gw);
    load8<T>(a.ln_b + c * 8, gb);
    uint4 raw[MR];
#pragma unroll
    for (int m = 0; m < MR; ++m)
      if (m < M) raw[m] = *reinterpret_cast<const uint4*>(a.x + (long)m * a.ldx + c * 8);
#pragma unroll
    for (int m = 0; m < MR; ++m) {
      if (m >= M) continue;
      float v[8];
      unpack8<T>(raw[m], v);
      short8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        o[j] = (short)Elt<T>::from_f((v[j] - mean[m]) * rstd[m] * gw[j] + gb[j]);
      *(__attribute__((address_space(3))) short8*)(xs + (long)m * (K + 8) + c * 8) = o;
    }
  }
  __syncthreads();
}

template <typename T, int U>
__device__ __forceinline__ void mma_batch(floatx4& acc, const short8 (&wv)[U][2],
                                          const short8 (&xv)[U][2]) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    acc = mma16<T>(wv[u][0], xv[u][0], acc);
    acc = mma16<T>(wv[u][1], xv[u][1], acc);
  }
}

template <typename T, int EPI, int U, int GV_KS, int RW, int LNR>
__global__ __launch_bounds__(64 * GV_KS) void gemv_kernel(GemvArgs a) {
  constexpr bool LN = LNR > 0;  // LayerNorm prologue over up to LNR rows
  __shared__ float red[GV_KS * 256];
  extern __shared__ __attribute__((aligned(16))) uint16_t xs_dyn[];  // LN: normalised x [M][K]
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  // RW (16 / 8 / 4) output columns per block: the MFMA still takes 16 W rows,
  // rows r and r + RW are the same row (the coalescer merges the duplicate
  // lanes), so a narrow layer (N = 2048) spreads over 256-512 blocks
  // instead of 128 and every CU streams
  const int n0 = blockIdx.x * RW;
  const int r = lane & 15, g = lane >> 4;
  const int kw = a.K / GV_KS;  // multiple of 64 * U (host check)
  const int kb = w * kw;
  const int nrow = min(n0 + (r % RW), a.N - 1);
  const uint16_t* wp = a.w + (long)nrow * a.ldw + kb + 16 * g;
  // x rows >= M read row M-1 (no per-load select: their D rows are never stored)
  // LN rows in LDS are K + 8 elements apart: the 16 lanes' rows fall on different banks
  const uint16_t* xp = LN ? xs_dyn + (long)min(r, a.M - 1) * (a.K + 8) + kb + 16 * g
                          : a.x + (long)min(r, a.M - 1) * a.ldx + kb + 16 * g;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  const int nch = kw / 64;
  // two register sets: batch c+1's loads are in flight under batch c's MFMAs
  short8 wa[U][2], xa[U][2], wb[U][2], xb[U][2];
  if constexpr (LN) {
    // the first weight batches stream while the LayerNorm statistics are taken
    load_w<U>(wa, wp, 0);
    if (U < nch) load_w<U>(wb, wp, U);
    ln_prologue<T, 64 * GV_KS, LNR>(a, xs_dyn, red);
    load_x<U, true>(xa, xp, 0);
    if (U < nch) load_x<U, true>(xb, xp, U);
  } else {
    load_batch<U, false>(wa, xa, wp, xp, 0);
  }
  for (int c = 0; c < nch; c += 2 * U) {
    if (!LN || c > 0)
      if (c + U < nch) load_batch<U, LN>(wb, xb, wp, xp, c + U);
    mma_batch<T, U>(acc, wa, xa);
    if (c + U >= nch) break;
    if (c + 2 * U < nch) load_batch<U, LN>(wa, xa, wp, xp, c + 2 * U);
    mma_batch<T, U>(acc, wb, xb);
  }
  if constexpr (LN) __syncthreads();  // red[] doubled as the LN scratch
  // D[n][m]: lane holds n = 4g + j, m = r
#pragma unroll
  for (int j = 0; j < 4; ++j) red[w * 256 + (4 * g + j) * 16 + r] = acc[j];
  __syncthreads();
  const int t = threadIdx.x;  // (nn, m) = (t / 16, t % 16)
  if (t >= 256) return;
  const int nn = t >> 4, m = t & 15;
  const int n = n0 + nn;
  if (nn >= RW || m >= a.M || n >= a.N) return;
  float v = 0.f;
#pragma unroll
  for (int s2 = 0; s2 < GV_KS; ++s2) v += red[s2 * 256 + t];
  if (a.bias != nullptr) v += Elt<T>::to_f(a.bias[n]);
  if constexpr (EPI == GV_GELU) v = gelu_tanh(v);
  if constexpr (EPI == GV_RES) v += Elt<T>::to_f(a.res[(long)m * a.ldres + n]);
  const uint16_t o = Elt<T>::from_f(v);
  if constexpr (EPI == GV_QKV) {
    // packed [heads][3][head_dim] columns
    const int D = a.head_dim;
    const int h = n / (3 * D), tq = (n / D) % 3, d = n % D;
    if (tq == 0) {
      a.y[(long)m * a.ldy + h * D + d] = o;
    } else {
      uint16_t* cache = tq == 1 ? a.kc : a.vc;
      cache[(((long)m * a.maxlen + a.pos[m]) * a.heads + h) * D + d] = o;
    }
  } else {
    a.y[(long)m * a.ldy + n] = o;
  }
}

template <typename T, int EPI, int RW, int LNR>
void launch_u(const GemvArgs& a, int u, int ks, hipStream_t s) {
  const dim3 grid((a.N + RW - 1) / RW);
  const size_t lds = LNR > 0 ? (size_t)a.M * (a.K + 8) * 2 : 0;
  auto go = [&](void (*k)(GemvArgs), int threads) {
    if (lds > 65536)
      (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds);
    hipLaunchKernelGGL(k, grid, dim3(threads), lds, s, a);
  };
  if (ks == 8) {
    if (u >= 8) go(gemv_kernel<T, EPI, 8, 8, RW, LNR>, 512);
    else go(gemv_kernel<T, EPI, 4, 8, RW, LNR>, 512);
  } else {
    if (u >= 8) go(gemv_kernel<T, EPI, 8, 4, RW, LNR>, 256);
    else go(gemv_kernel<T, EPI, 4, 4, RW, LNR>, 256);
  }
}

template <typename T, int EPI, int LNR>
void launch_rw(const GemvArgs& a, int u, int ks, int rw, hipStream_t s) {
  if (rw == 4 && LNR == 0) launch_u<T, EPI, 4, LNR>(a, u, ks, s);
  else if (rw <= 8) launch_u<T, EPI, 8, LNR>(a, u, ks, s);
  else launch_u<T, EPI, 16, LNR>(a, u, ks, s);
}

// LayerNorm-fused GEMV: row-count bucket of the unrolled prologue
template <typename T, int EPI>
void launch_ln(const GemvArgs& a, int u, int ks, int rw, hipStream_t s) {
  if (a.M == 1) launch_rw<T, EPI, 1>(a, u, ks, rw, s);
  else launch_rw<T, EPI, 4>(a, u, ks, rw, s);  // M <= 4 (host check)
}

// columns per block (FLEETX_GEMV_ROWS pins 16 / 8 / 4 for tools/bench_gemv.py sweeps)
int rows_per_block(int N) {
  static const int pin = [] {
    const char* e = getenv("FLEETX_GEMV_ROWS");
    return e ? atoi(e) : 0;
  }();
  if (pin == 4 || pin == 8 || pin == 16) return pin;
  // measured (tools/bench_gemv.py, M = 1, weights streamed from HBM): 8
  // columns per block help only the narrowest layers (1.3B out-proj / FC2,
  // N = 2048: 5.1 -> 4.7 / 14.2 -> 12.4 us); 4 columns lose everywhere (the
  // duplicated lanes cost issue slots)
  return N <= 2048 ? 8 : 16;
}

}  // namespace

extern "C" {

// Returns the number of blocks launched (0 = shape not supported: M > 16,
// K % 1024 != 0, unaligned rows).
// ln_w / ln_b (optional, GELU and QKV epilogues): y = LayerNorm(x) W^T ... with
// the LayerNorm fused as a prologue (normalised rows staged in LDS, M*K*2 bytes).
int fx_decode_gemv(int dt, int epi, int M, int N, int K, const void* x, long ldx, const void* w,
                   long ldw, const void* bias, const void* res, long ldres, void* y, long ldy,
                   void* kc, void* vc, const long* pos, int heads, int head_dim, int maxlen,
                   const void* ln_w, const void* ln_b, float ln_eps, hipStream_t s) {
  if (M < 1 || M > 16 || K % 1024 != 0 || (ldx % 8) || (ldw % 8)) return 0;
  const bool ln = ln_w != nullptr;
  // fused LayerNorm for up to 4 rows (small-batch decode, where the separate
  // launch dominates: 1.3B decode 1.27 / 1.38 / 1.43 -> 1.11 / 1.30 / 1.38 ms per
  // token at batch 1 / 2 / 4); more rows take the LayerNorm kernel (a 16-row
  // prologue measured 1.38 -> 2.13 ms at batch 8)
  if (ln && (ln_b == nullptr || (epi != GV_GELU && epi != GV_QKV) || M > 4 ||
             (long)M * (K + 8) * 2 > 96 * 1024))
    return 0;
  static const int pin_ks = [] { const char* e = getenv("FLEETX_GEMV_KS"); return e ? atoi(e) : 0; }();
  static const int pin_u = [] { const char* e = getenv("FLEETX_GEMV_U"); return e ? atoi(e) : 0; }();
  // measured (tools/bench_gemv.py, M = 1, HBM-streamed weights): 4 waves with
  // 4-chunk batches win on every GPT-3 1.3B / 6.7B layer and the LM head
  // (1.3B FFN1 12.2 -> 8.8 us, LM head 57 -> 40 us = 5.2 TB/s); only the
  // narrow N <= 2048 layers prefer 8 waves on shorter K ranges
  int ks = (N <= 2048 && K % 2048 == 0) ? 8 : 4;
  if ((pin_ks == 4 || pin_ks == 8) && K % (64 * 4 * pin_ks) == 0) ks = pin_ks;
  GemvArgs a;
  a.x = (const uint16_t*)x; a.w = (const uint16_t*)w; a.bias = (const uint16_t*)bias;
  a.res = (const uint16_t*)res; a.y = (uint16_t*)y;
  a.ldx = ldx; a.ldw = ldw; a.ldy = ldy; a.ldres = ldres;
  a.M = M; a.N = N; a.K = K;
  a.kc = (uint16_t*)kc; a.vc = (uint16_t*)vc; a.pos = pos;
  a.heads = heads; a.head_dim = head_dim; a.maxlen = maxlen;
  a.ln_w = (const uint16_t*)ln_w; a.ln_b = (const uint16_t*)ln_b; a.ln_eps = ln_eps;
  int u = 4;
  if (pin_u == 8 && (K / (64 * ks)) % 8 == 0) u = 8;
  const int rw = rows_per_block(N);
#define FX_GV(T)                                                  \
  switch (epi) {                                                              \
    case GV_GELU:                                                             \
      if (ln) launch_ln<T, GV_GELU>(a, u, ks, rw, s);                         \
      else launch_rw<T, GV_GELU, 0>(a, u, ks, rw, s);                         \
      break;                                                                  \
    case GV_RES: launch_rw<T, GV_RES, 0>(a, u, ks, rw, s); break;             \
    case GV_QKV:                                                              \
      if (ln) launch_ln<T, GV_QKV>(a, u, ks, rw, s);                          \
      else launch_rw<T, GV_QKV, 0>(a, u, ks, rw, s);                          \
      break;                                                                  \
    default: launch_rw<T, GV_BIAS, 0>(a, u, ks, rw, s); break;                \
  }
  if (dt == 0) { FX_GV(bf16) } else { FX_GV(f16) }
#undef FX_GV
  return (N + rw - 1) / rw;
}

}  // extern "C"
