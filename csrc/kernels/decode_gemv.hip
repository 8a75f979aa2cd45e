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
__device__ __forceinline__ void load_batch(short8 (&wv)[U][2], short8 (&xv)[U][2],
                                           const uint16_t* wp, const uint16_t* xp, int c) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const short8* p = reinterpret_cast<const short8*>(wp + (c + u) * 64);
    wv[u][0] = __builtin_nontemporal_load(p);
    wv[u][1] = __builtin_nontemporal_load(p + 1);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const short8* p = reinterpret_cast<const short8*>(xp + (c + u) * 64);
    xv[u][0] = p[0];
    xv[u][1] = p[1];
  }
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

template <typename T, int EPI, int U, int GV_KS>
__global__ __launch_bounds__(64 * GV_KS) void gemv_kernel(GemvArgs a) {
  __shared__ float red[GV_KS * 256];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int n0 = blockIdx.x * 16;
  const int r = lane & 15, g = lane >> 4;
  const int kw = a.K / GV_KS;  // multiple of 64 * U (host check)
  const int kb = w * kw;
  const int nrow = min(n0 + r, a.N - 1);
  const uint16_t* wp = a.w + (long)nrow * a.ldw + kb + 16 * g;
  // x rows >= M read row M-1 (no per-load select: their D rows are never stored)
  const uint16_t* xp = a.x + (long)min(r, a.M - 1) * a.ldx + kb + 16 * g;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  const int nch = kw / 64;
  // two register sets: batch c+1's loads are in flight under batch c's MFMAs
  short8 wa[U][2], xa[U][2], wb[U][2], xb[U][2];
  load_batch<U>(wa, xa, wp, xp, 0);
  for (int c = 0; c < nch; c += 2 * U) {
    if (c + U < nch) load_batch<U>(wb, xb, wp, xp, c + U);
    mma_batch<T, U>(acc, wa, xa);
    if (c + U >= nch) break;
    if (c + 2 * U < nch) load_batch<U>(wa, xa, wp, xp, c + 2 * U);
    mma_batch<T, U>(acc, wb, xb);
  }
  // D[n][m]: lane holds n = 4g + j, m = r
#pragma unroll
  for (int j = 0; j < 4; ++j) red[w * 256 + (4 * g + j) * 16 + r] = acc[j];
  __syncthreads();
  const int t = threadIdx.x;  // (nn, m) = (t / 16, t % 16)
  if (t >= 256) return;
  const int nn = t >> 4, m = t & 15;
  const int n = n0 + nn;
  if (m >= a.M || n >= a.N) return;
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

template <typename T, int EPI>
void launch_u(const GemvArgs& a, int u, int ks, hipStream_t s) {
  const dim3 grid((a.N + 15) / 16);
  if (ks == 8) {
    if (u >= 8) hipLaunchKernelGGL((gemv_kernel<T, EPI, 8, 8>), grid, dim3(512), 0, s, a);
    else hipLaunchKernelGGL((gemv_kernel<T, EPI, 4, 8>), grid, dim3(512), 0, s, a);
  } else {
    if (u >= 8) hipLaunchKernelGGL((gemv_kernel<T, EPI, 8, 4>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((gemv_kernel<T, EPI, 4, 4>), grid, dim3(256), 0, s, a);
  }
}

}  // namespace

extern "C" {

// Returns the number of blocks launched (0 = shape not supported: M > 16,
// K % 1024 != 0, unaligned rows).
int fx_decode_gemv(int dt, int epi, int M, int N, int K, const void* x, long ldx, const void* w,
                   long ldw, const void* bias, const void* res, long ldres, void* y, long ldy,
                   void* kc, void* vc, const long* pos, int heads, int head_dim, int maxlen,
                   hipStream_t s) {
  if (M < 1 || M > 16 || K % 1024 != 0 || (ldx % 8) || (ldw % 8)) return 0;
  // many column tiles: 8 waves per block, each on a shorter K range (more
  // waves resident, shorter dependent chains); few tiles: 4 waves with two
  // batches of loads in flight each (tools/bench_gemv.py)
  const int ks = (N >= 8192 && K % 2048 == 0) ? 8 : 4;
  GemvArgs a;
  a.x = (const uint16_t*)x; a.w = (const uint16_t*)w; a.bias = (const uint16_t*)bias;
  a.res = (const uint16_t*)res; a.y = (uint16_t*)y;
  a.ldx = ldx; a.ldw = ldw; a.ldy = ldy; a.ldres = ldres;
  a.M = M; a.N = N; a.K = K;
  a.kc = (uint16_t*)kc; a.vc = (uint16_t*)vc; a.pos = pos;
  a.heads = heads; a.head_dim = head_dim; a.maxlen = maxlen;
  const int u = (K / (64 * ks)) % 8 == 0 && K / (64 * ks) >= 16 ? 8 : 4;
#define FX_GV(T)                                                  \
  switch (epi) {                                                  \
    case GV_GELU: launch_u<T, GV_GELU>(a, u, ks, s); break;           \
    case GV_RES: launch_u<T, GV_RES>(a, u, ks, s); break;             \
    case GV_QKV: launch_u<T, GV_QKV>(a, u, ks, s); break;             \
    default: launch_u<T, GV_BIAS>(a, u, ks, s); break;                \
  }
  if (dt == 0) { FX_GV(bf16) } else { FX_GV(f16) }
#undef FX_GV
  return (N + 15) / 16;
}

}  // extern "C"
