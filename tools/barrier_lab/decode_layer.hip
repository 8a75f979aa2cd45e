// One whole GPT decoder layer for a decode step (M <= 4 token rows) in ONE
// persistent launch: LN1 + QKV GEMV (+ K/V appended to the cache) ->
// split-K attention over the cache -> [combine] + out-proj GEMV + residual ->
// LN2 + FC1 GEMV + GeLU -> FC2 GEMV + residual, separated by grid-wide
// barriers instead of kernel boundaries.
//
// Reference K19 / N-12: the inference program's
// fused_multi_transformer (`core/engine/inference_engine.py:103-109,127-129`).
//
// Why: at decode sizes the five per-layer kernels of decode_gemv.hip /
// decode_attention each cost a fixed ~5-9 us (dispatch, the first weight
// round trip from HBM, LayerNorm prologue, reduction, drain) whatever their
// bytes -- a 1.3B out-projection GEMV streams 8 MB in 5-9 us, the same with
// its weights resident in the Infinity Cache (profiles/r3_decode/).  Here one
// launch per layer keeps every workgroup resident: a phase boundary is a
// grid barrier, and each workgroup issues the loads of its first weight batch
// of a phase right after the barrier, before the phase's prologue (weights do
// not depend on the activations), so the first HBM round trip overlaps the
// LayerNorm / attention-combine work.
//
// CDNA4 mapping:
//  * grid = one 256-thread workgroup per CU (all co-resident; the host sizes
//    it from the CU count); every phase walks its work items grid-stride;
//  * GEMV work item = 8 output columns (rows of W) x all K: MFMA
//    v_mfma_f32_16x16x32 with A = the 8 W rows twice (rows r and r + 8 are
//    the same row: the coalescer merges the duplicate lanes), B = the x rows
//    (rows >= M repeat row M-1, never stored), K split over the 4 waves,
//    reduced through LDS -- the decode_gemv.hip inner loop;
//  * LayerNorm of the few rows is recomputed by every workgroup into LDS
//    (cheaper than a phase); the attention partials are combined the same way
//    in the out-projection's prologue;
//  * grid barrier: every wave drains its stores, workgroup barrier, one lane
//    releases (agent scope) and bumps a counter, polls it with s_sleep, and
//    acquires; the spin is bounded (an error flag, checked by the host after
//    generation, instead of a hang if a workgroup could not become resident).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "fx_common.h"

namespace {

constexpr int NT = 256;  // threads per workgroup (4 waves)
constexpr int RW = 8;    // W rows per GEMV work item
constexpr int U = 4;     // 64-k chunks per load batch

struct DecLayer {
  const uint16_t* x;  // [M, h] residual stream in
  uint16_t* xout;     // [M, h] residual stream out
  uint16_t* q;        // scratch [M, h]: query heads
  float* apart;       // scratch [M * H * nsplit, D + 2]: attention partials
  uint16_t* x2;       // scratch [M, h]: x + attn
  uint16_t* f;        // scratch [M, ffn]: gelu(FC1)
  const uint16_t *ln1w, *ln1b, *wqkv, *bqkv, *wo, *bo, *ln2w, *ln2b, *w1, *b1, *w2, *b2;
  uint16_t *kc, *vc;  // [M, maxlen, H, D]
  const long* pos;    // [M] position of this token
  const int* lens;    // [M] valid keys after the append
  int M, h, ffn, heads, hd, maxlen, nsplit, chunk;
  float eps1, eps2, scale;
  unsigned* bar;      // grid-barrier counter (zeroed by the host per decode step)
  unsigned bar_base;  // counter value at this launch's start
  int* err;           // set when a barrier spin gives up
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

// LDS-only workgroup sync: waits for this wave's LDS operations, not for its
// global loads (a weight batch in flight stays in flight across it)
__device__ __forceinline__ void lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

// ------------------------------------------------------------------ barrier
__device__ __forceinline__ void grid_barrier(const DecLayer& a, unsigned k) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stores are done
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned target = a.bar_base + k * gridDim.x;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(a.bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int spins = 0;
    while (__hip_atomic_load(a.bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > (1 << 22)) {  // ~0.5 s: never hang the GPU; the host raises
        __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

// ------------------------------------------------------------------ LayerNorm -> LDS
// rows m < M of src [M, K] (global) normalised into xs [M][K + 8] (16-bit, LDS)
template <typename T>
__device__ __forceinline__ void ln_rows(const uint16_t* src, const uint16_t* gw, const uint16_t* gb, float eps,
                        int M, int K, uint16_t* xs, float* red) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int nch = K / 8;
  for (int m = 0; m < M; ++m) {
    const uint16_t* row = src + (long)m * K;
    const float sh = Elt<T>::to_f(row[0]);  // shifted moments: no cancellation
    float s1 = 0.f, s2 = 0.f;
    for (int c = t; c < nch; c += NT) {
      float v[8];
      load8<T>(row + c * 8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[j] - sh;
        s1 += d;
        s2 += d * d;
      }
    }
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    if (lane == 0) {
      red[2 * w] = s1;
      red[2 * w + 1] = s2;
    }
    lds_sync();
    const float r1 = red[0] + red[2] + red[4] + red[6];
    const float r2 = red[1] + red[3] + red[5] + red[7];
    const float md = r1 / K, mean = sh + md;
    const float rstd = rsqrtf(fmaxf(r2 / K - md * md, 0.f) + eps);
    for (int c = t; c < nch; c += NT) {
      float v[8], g[8], b[8];
      load8<T>(row + c * 8, v);
      load8<T>(gw + c * 8, g);
      load8<T>(gb + c * 8, b);
      short8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (short)Elt<T>::from_f((v[j] - mean) * rstd * g[j] + b[j]);
      *(__attribute__((address_space(3))) short8*)(xs + (long)m * (K + 8) + c * 8) = o;
    }
    lds_sync();
  }
}

// ------------------------------------------------------------------ GEMV
enum { E_QKV = 0, E_RES = 1, E_GELU = 2 };

template <bool XL>
__device__ __forceinline__ void ld_x(short8 (&xv)[U][2], const uint16_t* xp, int c) {
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
__device__ __forceinline__ void ld_w(short8 (&wv)[U][2], const uint16_t* wp, int c) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const short8* p = reinterpret_cast<const short8*>(wp + (c + u) * 64);
    wv[u][0] = __builtin_nontemporal_load(p);
    wv[u][1] = __builtin_nontemporal_load(p + 1);
  }
}

// Per-wave pointer into W for work item `it` (rows it*RW .. +RW-1, this
// wave's K quarter, this lane's 32-byte slice of a 64-k chunk).
__device__ __forceinline__ const uint16_t* wptr(const uint16_t* W, int N, int K, int it) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int row = min(it * RW + (r % RW), N - 1);
  return W + (long)row * K + w * (K / 4) + 16 * g;
}

// y[m, n] over this workgroup's items, epilogue EPI.  x: LDS rows [M][K + 8]
// (XL) or global rows [M][K].  `pre` = the first batch of this workgroup's
// first item, already in flight (issued before the preceding barrier).
template <typename T, int EPI, bool XL>
__device__ __forceinline__ void gemv_phase(const DecLayer& a, const uint16_t* W, const uint16_t* bias, int N,
                           int K, const uint16_t* x, const uint16_t* res, uint16_t* y,
                           float* red, short8 (&pre)[U][2]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int kw = K / 4, nch = kw / 64;
  const int items = (N + RW - 1) / RW;
  const long ldx = XL ? K + 8 : K;
  const uint16_t* xp = x + (long)min(r, a.M - 1) * ldx + w * kw + 16 * g;
  bool first = true;
  for (int it = blockIdx.x; it < items; it += gridDim.x) {
    const uint16_t* wp = wptr(W, N, K, it);
    short8 wa[U][2], xa[U][2], wb[U][2], xb[U][2];
    if (first) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        wa[u][0] = pre[u][0];
        wa[u][1] = pre[u][1];
      }
      first = false;
    } else {
      ld_w(wa, wp, 0);
    }
    ld_x<XL>(xa, xp, 0);
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < nch; c += 2 * U) {
      if (c + U < nch) {
        ld_w(wb, wp, c + U);
        ld_x<XL>(xb, xp, c + U);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        acc = mma16<T>(wa[u][0], xa[u][0], acc);
        acc = mma16<T>(wa[u][1], xa[u][1], acc);
      }
      if (c + U >= nch) break;
      if (c + 2 * U < nch) {
        ld_w(wa, wp, c + 2 * U);
        ld_x<XL>(xa, xp, c + 2 * U);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        acc = mma16<T>(wb[u][0], xb[u][0], acc);
        acc = mma16<T>(wb[u][1], xb[u][1], acc);
      }
    }
    // D[n][m]: lane holds n = 4g + j, m = r
#pragma unroll
    for (int j = 0; j < 4; ++j) red[w * 256 + (4 * g + j) * 16 + r] = acc[j];
    lds_sync();
    const int t = threadIdx.x, nn = t >> 4, m = t & 15, n = it * RW + nn;
    if (nn < RW && m < a.M && n < N) {
      float v = red[t] + red[256 + t] + red[512 + t] + red[768 + t];
      v += Elt<T>::to_f(bias[n]);
      if constexpr (EPI == E_GELU) v = gelu_tanh(v);
      if constexpr (EPI == E_RES) v += Elt<T>::to_f(res[(long)m * N + n]);
      const uint16_t o = Elt<T>::from_f(v);
      if constexpr (EPI == E_QKV) {  // packed [heads][3][head_dim] columns
        const int D = a.hd;
        const int hh = n / (3 * D), tq = (n / D) % 3, d = n % D;
        if (tq == 0) {
          a.q[(long)m * a.h + hh * D + d] = o;
        } else {
          uint16_t* cache = tq == 1 ? a.kc : a.vc;
          cache[(((long)m * a.maxlen + a.pos[m]) * a.heads + hh) * D + d] = o;
        }
      } else {
        y[(long)m * N + n] = o;
      }
    }
    lds_sync();
  }
}

// first batch of this workgroup's first item of a GEMV phase (issued early)
__device__ __forceinline__ void prefetch(short8 (&pre)[U][2], const uint16_t* W, int N, int K) {
  if ((int)blockIdx.x < (N + RW - 1) / RW) ld_w(pre, wptr(W, N, K, blockIdx.x), 0);
}

// ------------------------------------------------------------------ attention
// item = (m, head, split): partial (o[D], max, sum) over keys [split*chunk, ..)
template <typename T, int D>
__device__ __forceinline__ void attn_phase(const DecLayer& a) {
  constexpr int LPK = D / 8;     // lanes per key row
  constexpr int KPW = 64 / LPK;  // key rows per wave instruction
  constexpr int NW = NT / 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int sub = lane / LPK, c = (lane % LPK) * 8;
  __shared__ float sm_m[NW * LPK], sm_l[NW * LPK], sm_o[NW * LPK][8];
  const int items = a.M * a.heads * a.nsplit;
  for (int it = blockIdx.x; it < items; it += gridDim.x) {
    const int split = it % a.nsplit, mh = it / a.nsplit;
    const int m = mh / a.heads, hd = mh % a.heads;
    const int len = a.lens[m];
    const int k_lo = split * a.chunk, k_hi = min(len, k_lo + a.chunk);
    float qv[8];
    load8<T>(a.q + (long)m * a.h + hd * D + c, qv);
#pragma unroll
    for (int j = 0; j < 8; ++j) qv[j] *= a.scale;
    float mx = -INFINITY, l = 0.f, o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = 0.f;
    const long sks = (long)a.heads * D;
    const uint16_t* kb = a.kc + (long)m * a.maxlen * sks + hd * D + c;
    const uint16_t* vb = a.vc + (long)m * a.maxlen * sks + hd * D + c;
    for (int k0 = k_lo; k0 < k_hi; k0 += NW * KPW) {
      const int key = k0 + w * KPW + sub;
      const int kk = key < k_hi ? key : k_lo;
      const uint4 kraw = *reinterpret_cast<const uint4*>(kb + (long)kk * sks);
      const uint4 vraw = *reinterpret_cast<const uint4*>(vb + (long)kk * sks);
      float kv[8], vv[8];
      unpack8<T>(kraw, kv);
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) s += kv[j] * qv[j];
#pragma unroll
      for (int off = LPK / 2; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
      if (key >= k_hi) continue;
      const float mn = fmaxf(mx, s);
      const float al = __expf(mx - mn), p = __expf(s - mn);
      unpack8<T>(vraw, vv);
      l = l * al + p;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = o[j] * al + p * vv[j];
      mx = mn;
    }
    // merge the KPW lane groups, then the waves through LDS
#pragma unroll
    for (int off = LPK; off < 64; off <<= 1) {
      const float m2 = __shfl_xor(mx, off, 64), l2 = __shfl_xor(l, off, 64);
      float o2[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o2[j] = __shfl_xor(o[j], off, 64);
      const float M = fmaxf(mx, m2);
      if (M != -INFINITY) {
        const float e1 = __expf(mx - M), e2 = __expf(m2 - M);
        l = l * e1 + l2 * e2;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = o[j] * e1 + o2[j] * e2;
        mx = M;
      }
    }
    if (lane < LPK) {
      sm_m[w * LPK + lane] = mx;
      sm_l[w * LPK + lane] = l;
#pragma unroll
      for (int j = 0; j < 8; ++j) sm_o[w * LPK + lane][j] = o[j];
    }
    lds_sync();
    if (threadIdx.x < LPK) {
      float M = -INFINITY;
#pragma unroll
      for (int i = 0; i < NW; ++i) M = fmaxf(M, sm_m[i * LPK + threadIdx.x]);
      float L = 0.f, O[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) O[j] = 0.f;
      if (M != -INFINITY) {
#pragma unroll
        for (int i = 0; i < NW; ++i) {
          const int t = i * LPK + threadIdx.x;
          if (sm_m[t] == -INFINITY) continue;
          const float e = __expf(sm_m[t] - M);
          L += sm_l[t] * e;
#pragma unroll
          for (int j = 0; j < 8; ++j) O[j] += sm_o[t][j] * e;
        }
      }
      float* wp = a.apart + (long)it * (D + 2);
#pragma unroll
      for (int j = 0; j < 8; ++j) wp[threadIdx.x * 8 + j] = O[j];
      if (threadIdx.x == 0) {
        wp[D] = M;
        wp[D + 1] = L;
      }
    }
    lds_sync();
  }
}

// attention output o[M][h] from the partials, into LDS rows [M][h + 8]
template <typename T, int D>
__device__ __forceinline__ void attn_combine(const DecLayer& a, uint16_t* xs) {
  const int total = a.M * a.heads * D;
  for (int e = threadIdx.x; e < total; e += NT) {
    const int d = e % D, mh = e / D, m = mh / a.heads, hd = mh % a.heads;
    const float* base = a.apart + (long)mh * a.nsplit * (D + 2);
    float M = -INFINITY;
    for (int s = 0; s < a.nsplit; ++s) M = fmaxf(M, base[s * (D + 2) + D]);
    float L = 0.f, O = 0.f;
    if (M != -INFINITY) {
      for (int s = 0; s < a.nsplit; ++s) {
        const float* wp = base + s * (D + 2);
        if (wp[D] == -INFINITY) continue;
        const float ex = __expf(wp[D] - M);
        L += wp[D + 1] * ex;
        O += wp[d] * ex;
      }
    }
    xs[(long)m * (a.h + 8) + hd * D + d] = Elt<T>::from_f(L > 0.f ? O / L : 0.f);
  }
  lds_sync();
}

template <typename T, int D>
__global__ __launch_bounds__(NT) void decode_layer_kernel(DecLayer a) {
  extern __shared__ __attribute__((aligned(16))) uint16_t xs[];  // [M][h + 8]
  __shared__ float red[4 * 256];
  const int h = a.h;
  short8 pre[U][2];
  // Each phase first issues its first weight batch (no dependence on the
  // activations), then runs its prologue (LayerNorm / attention combine)
  // under those loads, then the GEMV.
  // 1. LN1 + QKV (+ K/V into the cache)
  prefetch(pre, a.wqkv, 3 * h, h);
  ln_rows<T>(a.x, a.ln1w, a.ln1b, a.eps1, a.M, h, xs, red);
  gemv_phase<T, E_QKV, true>(a, a.wqkv, a.bqkv, 3 * h, h, xs, nullptr, nullptr, red, pre);
  grid_barrier(a, 1);
  // 2. attention partials
  prefetch(pre, a.wo, h, h);
  attn_phase<T, D>(a);
  grid_barrier(a, 2);
  // 3. combine + out-proj + residual -> x2
  attn_combine<T, D>(a, xs);
  gemv_phase<T, E_RES, true>(a, a.wo, a.bo, h, h, xs, a.x, a.x2, red, pre);
  grid_barrier(a, 3);
  // 4. LN2 + FC1 + GeLU -> f
  prefetch(pre, a.w1, a.ffn, h);
  ln_rows<T>(a.x2, a.ln2w, a.ln2b, a.eps2, a.M, h, xs, red);
  gemv_phase<T, E_GELU, true>(a, a.w1, a.b1, a.ffn, h, xs, nullptr, a.f, red, pre);
  grid_barrier(a, 4);
  // 5. FC2 + residual -> xout
  prefetch(pre, a.w2, h, a.ffn);
  gemv_phase<T, E_RES, false>(a, a.w2, a.b2, h, a.ffn, a.f, a.x2, a.xout, red, pre);
}

}  // namespace

extern "C" {

// Barriers per launch: the host advances `bar_base` by this x grid per layer.
int fx_decode_layer_barriers() { return 4; }

int fx_decode_layer_grid() {
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (ncu <= 0) ncu = 256;
  }
  return ncu;
}

// Returns 0 when launched, < 0 when the shape is not covered (the caller then
// runs the per-kernel decode layer).
int fx_decode_layer(int dt, int M, int h, int ffn, int heads, int hd, int maxlen, int nsplit,
                    const void* x, void* xout, void* q, float* apart, void* x2, void* f,
                    const void* ln1w, const void* ln1b, const void* wqkv, const void* bqkv,
                    const void* wo, const void* bo, const void* ln2w, const void* ln2b,
                    const void* w1, const void* b1, const void* w2, const void* b2, void* kc,
                    void* vc, const long* pos, const int* lens, float eps1, float eps2,
                    float scale, unsigned* bar, unsigned bar_base, int* err, hipStream_t st) {
  if (M < 1 || M > 4 || h % 1024 || ffn % 1024 || heads * hd != h) return -1;
  if (hd != 64 && hd != 128) return -2;
  if (nsplit < 1 || !bqkv || !bo || !b1 || !b2) return -3;
  DecLayer a;
  a.x = (const uint16_t*)x; a.xout = (uint16_t*)xout; a.q = (uint16_t*)q; a.apart = apart;
  a.x2 = (uint16_t*)x2; a.f = (uint16_t*)f;
  a.ln1w = (const uint16_t*)ln1w; a.ln1b = (const uint16_t*)ln1b;
  a.wqkv = (const uint16_t*)wqkv; a.bqkv = (const uint16_t*)bqkv;
  a.wo = (const uint16_t*)wo; a.bo = (const uint16_t*)bo;
  a.ln2w = (const uint16_t*)ln2w; a.ln2b = (const uint16_t*)ln2b;
  a.w1 = (const uint16_t*)w1; a.b1 = (const uint16_t*)b1;
  a.w2 = (const uint16_t*)w2; a.b2 = (const uint16_t*)b2;
  a.kc = (uint16_t*)kc; a.vc = (uint16_t*)vc; a.pos = pos; a.lens = lens;
  a.M = M; a.h = h; a.ffn = ffn; a.heads = heads; a.hd = hd; a.maxlen = maxlen;
  a.nsplit = nsplit; a.chunk = (maxlen + nsplit - 1) / nsplit;
  a.eps1 = eps1; a.eps2 = eps2; a.scale = scale;
  a.bar = bar; a.bar_base = bar_base; a.err = err;
  const int grid = fx_decode_layer_grid();
  const size_t lds = (size_t)M * (h + 8) * 2;
  auto go = [&](void (*k)(DecLayer)) {
    if (lds > 65536)
      (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds);
    hipLaunchKernelGGL(k, dim3(grid), dim3(NT), lds, st, a);
  };
  if (dt == 0) go(hd == 128 ? decode_layer_kernel<bf16, 128> : decode_layer_kernel<bf16, 64>);
  else go(hd == 128 ? decode_layer_kernel<f16, 128> : decode_layer_kernel<f16, 64>);
  return 0;
}

}  // extern "C"
