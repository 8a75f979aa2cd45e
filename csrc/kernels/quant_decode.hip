// QAT fake-quant (abs-max, symmetric int-N) and single-token decode attention
// over a KV cache.
//
// Parity: reference K23 (paddleslim QAT: abs_max weights / moving-average
// abs_max activations, 8 bit; `pretrain_gpt_345M_mp8_qat.yaml:35-44`) and
// K18/K19 (generation decode with a KV cache, `single_model.py:109-114`,
// Paddle fused_multi_transformer decode path).
//
// Decode attention is memory bound (one query row per (batch, head)): split-K
// over the cached keys (see decode_attn_split_kernel).
#include "fx_common.h"

namespace {

template <typename T>
__global__ __launch_bounds__(256) void absmax_kernel(const uint16_t* __restrict__ x, long n,
                                                     float* __restrict__ out) {
  float m = 0.f;
  const long n8 = n / 8;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    float a[8];
    load8<T>(x + i * 8, a);
#pragma unroll
    for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(a[j]));
  }
  for (long i = n8 * 8 + blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    m = fmaxf(m, fabsf(Elt<T>::to_f(x[i])));
  m = wave_max(m);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    // non-negative floats order like their bit patterns
    atomicMax(reinterpret_cast<unsigned int*>(out), __float_as_uint(m));
  }
}

template <typename T>
__global__ __launch_bounds__(256) void fake_quant_kernel(const uint16_t* __restrict__ x,
                                                         uint16_t* __restrict__ y,
                                                         const float* __restrict__ scale, int bits,
                                                         long n) {
  const float s = fmaxf(*scale, 1e-8f);
  const float qmax = (float)((1 << (bits - 1)) - 1);
  const float inv = qmax / s, deq = s / qmax;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    float v = Elt<T>::to_f(x[i]);
    float q = fminf(fmaxf(rintf(v * inv), -qmax), qmax);
    y[i] = Elt<T>::from_f(q * deq);
  }
}

// Split-K ("flash-decoding") single-token attention over a KV cache.
// q: [B, H, D] (strides sqb, sqh); caches: [B, maxlen, H, D] (skb, sks, skh);
// out: [B, H, D] (sob, D contiguous, head stride D).
// Pass 1: grid = B*H*nsplit workgroups; split s of (b, h) scores keys
//   [s*chunk, min((s+1)*chunk, len)): D/8 lanes cover one key row with 16-byte
//   loads, each lane group keeps 4 keys in flight per step (the kernel is HBM
//   bound: every cached byte is read once), online softmax per lane group,
//   merged through LDS into one partial (m, l, o[D]) per workgroup.
// Pass 2: one workgroup per (b, h) merges the nsplit partials.
// Small-batch long-context decode thus spreads over B*H*nsplit >= ~2 waves of
// workgroups instead of B*H (a few CUs out of 256).
// merge another online-softmax state (m2, l2, o2) into (m, l, o)
__device__ __forceinline__ void merge_state(float& m, float& l, float* o, float m2, float l2,
                                            const float* o2) {
  const float M = fmaxf(m, m2);
  if (M == -INFINITY) return;
  const float a = __expf(m - M), c = __expf(m2 - M);
  l = l * a + l2 * c;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = o[j] * a + o2[j] * c;
  m = M;
}

template <typename T, int D, int NW>
__global__ __launch_bounds__(64 * NW) void decode_attn_split_kernel(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc,
    const uint16_t* __restrict__ vc, const int* __restrict__ lens, float* __restrict__ ws,
    int H, int nsplit, int chunk, long sqb, long sqh, long skb, long sks, long skh, float scale,
    uint16_t* __restrict__ out, long sob) {
  constexpr int LPK = D / 8;        // lanes per key row
  constexpr int KPW = 64 / LPK;     // key rows per wave instruction
  constexpr int U = 4;              // key rows per lane group per step
  const int split = blockIdx.x % nsplit, bh = blockIdx.x / nsplit;
  const int b = bh / H, hd = bh % H;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int sub = lane / LPK, c = (lane % LPK) * 8;
  const int len = lens[b];
  const int k_lo = split * chunk, k_hi = min(len, k_lo + chunk);
  float qv[8];
  load8<T>(q + b * sqb + hd * sqh + c, qv);
#pragma unroll
  for (int j = 0; j < 8; ++j) qv[j] *= scale;
  float m = -INFINITY, l = 0.f, o[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = 0.f;
  const uint16_t* kb = kc + b * skb + hd * skh + c;
  const uint16_t* vb = vc + b * skb + hd * skh + c;
  // wave w, step: keys k0 + u*KPW*NW + w*KPW + sub, u < U.  NW = 16 for few
  // (batch, head) pairs: a whole short context is one step (one memory round
  // trip) of one workgroup instead of several steps of 4 waves
  for (int k0 = k_lo; k0 < k_hi; k0 += NW * KPW * U) {
    float sc[U];
    int key[U];
    // K and V rows of the step are loaded together (V does not depend on the
    // scores): one memory round trip per step instead of two
    uint4 kraw[U], vraw[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      key[u] = k0 + (u * NW + w) * KPW + sub;
      const int kk = key[u] < k_hi ? key[u] : k_lo;  // in-range dummy row
      kraw[u] = *reinterpret_cast<const uint4*>(kb + (long)kk * sks);
      vraw[u] = *reinterpret_cast<const uint4*>(vb + (long)kk * sks);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float kv[8];
      unpack8<T>(kraw[u], kv);
      sc[u] = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) sc[u] += kv[j] * qv[j];
    }
#pragma unroll
    for (int off = LPK / 2; off > 0; off >>= 1)
#pragma unroll
      for (int u = 0; u < U; ++u) sc[u] += __shfl_xor(sc[u], off, 64);
    float mx = m;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (key[u] >= k_hi) sc[u] = -INFINITY;
      mx = fmaxf(mx, sc[u]);
    }
    if (mx == -INFINITY) continue;
    const float a = __expf(m - mx);
    l *= a;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] *= a;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (key[u] >= k_hi) continue;
      const float p = __expf(sc[u] - mx);
      float vv[8];
      unpack8<T>(vraw[u], vv);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] += p * vv[j];
      l += p;
    }
    m = mx;
  }
  // merge: the KPW lane groups of a wave share each column slice -> lane
  // shuffles; then one state per (wave, slice) through LDS, NW-way
#pragma unroll
  for (int off = LPK; off < 64; off <<= 1) {
    float o2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o2[j] = __shfl_xor(o[j], off, 64);
    const float m2 = __shfl_xor(m, off, 64), l2 = __shfl_xor(l, off, 64);
    merge_state(m, l, o, m2, l2, o2);
  }
  __shared__ float sm_m[NW * LPK], sm_l[NW * LPK], sm_o[NW * LPK][8];
  if (lane < LPK) {
    sm_m[w * LPK + lane] = m;
    sm_l[w * LPK + lane] = l;
#pragma unroll
    for (int j = 0; j < 8; ++j) sm_o[w * LPK + lane][j] = o[j];
  }
  __syncthreads();
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
        const float a = __expf(sm_m[t] - M);
        L += sm_l[t] * a;
#pragma unroll
        for (int j = 0; j < 8; ++j) O[j] += sm_o[t][j] * a;
      }
    }
    if (nsplit == 1) {  // one split: normalise and store the output directly
      const float inv = L > 0.f ? 1.f / L : 0.f;
      float r[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] = O[j] * inv;
      store8<T>(out + b * sob + hd * D + threadIdx.x * 8, r);
      return;
    }
    float* wp = ws + (long)blockIdx.x * (D + 2);
#pragma unroll
    for (int j = 0; j < 8; ++j) wp[threadIdx.x * 8 + j] = O[j];
    if (threadIdx.x == 0) {
      wp[D] = M;
      wp[D + 1] = L;
    }
  }
}

template <typename T, int D>
__global__ __launch_bounds__(D) void decode_attn_combine_kernel(const float* __restrict__ ws,
                                                               uint16_t* __restrict__ out, int H,
                                                               int nsplit, long sob) {
  const int bh = blockIdx.x, b = bh / H, hd = bh % H, d = threadIdx.x;
  const float* base = ws + (long)bh * nsplit * (D + 2);
  float M = -INFINITY;
  for (int s = 0; s < nsplit; ++s) M = fmaxf(M, base[s * (D + 2) + D]);
  float L = 0.f, O = 0.f;
  if (M != -INFINITY) {
    for (int s = 0; s < nsplit; ++s) {
      const float* wp = base + s * (D + 2);
      if (wp[D] == -INFINITY) continue;
      const float a = __expf(wp[D] - M);
      L += wp[D + 1] * a;
      O += wp[d] * a;
    }
  }
  out[b * sob + hd * D + d] = Elt<T>::from_f(L > 0.f ? O / L : 0.f);
}

}  // namespace

extern "C" void fx_absmax(int dtype, const void* x, long n, float* out, hipStream_t st) {
  long g = (n / 8 + 255) / 256;
  if (g > 1024) g = 1024;
  if (g < 1) g = 1;
  if (dtype == 0) absmax_kernel<bf16><<<(int)g, 256, 0, st>>>((const uint16_t*)x, n, out);
  else absmax_kernel<f16><<<(int)g, 256, 0, st>>>((const uint16_t*)x, n, out);
}

extern "C" int fx_fake_quant_fwd(int dtype, const void* x, void* y, const float* scale, int bits,
                                 long n, hipStream_t st) {
  long g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  if (dtype == 0)
    fake_quant_kernel<bf16><<<(int)g, 256, 0, st>>>((const uint16_t*)x, (uint16_t*)y, scale, bits, n);
  else
    fake_quant_kernel<f16><<<(int)g, 256, 0, st>>>((const uint16_t*)x, (uint16_t*)y, scale, bits, n);
  return 0;
}

// dt: 0 bf16 / 1 fp16; ws: fp32 workspace of B*H*nsplit*(D+2); chunk = keys per split
extern "C" int fx_decode_attn(int dt, const void* q, const void* kc, const void* vc, void* out,
                              const int* lens, int B, int H, int D, int maxlen, int nsplit,
                              float* ws, long sqb, long sqh, long skb, long sks, long skh,
                              long sob, float scale, hipStream_t st) {
  if (D != 64 && D != 128) return -1;
  if (nsplit < 1) return -2;
  const int chunk = (maxlen + nsplit - 1) / nsplit;
  const int g = B * H * nsplit;
  // few workgroups (small batch x heads): 16 waves each, so a short context
  // is one load step; many: 4 waves
  const bool wide = g < 256;
#define FX_DEC(TT, DD)                                                                           \
  do {                                                                                           \
    if (wide)                                                                                    \
      decode_attn_split_kernel<TT, DD, 16><<<g, 1024, 0, st>>>(                                  \
          (const uint16_t*)q, (const uint16_t*)kc, (const uint16_t*)vc, lens, ws, H, nsplit,     \
          chunk, sqb, sqh, skb, sks, skh, scale, (uint16_t*)out, sob);                           \
    else                                                                                         \
      decode_attn_split_kernel<TT, DD, 4><<<g, 256, 0, st>>>(                                    \
          (const uint16_t*)q, (const uint16_t*)kc, (const uint16_t*)vc, lens, ws, H, nsplit,     \
          chunk, sqb, sqh, skb, sks, skh, scale, (uint16_t*)out, sob);                           \
    if (nsplit > 1)                                                                              \
      decode_attn_combine_kernel<TT, DD><<<B * H, DD, 0, st>>>(ws, (uint16_t*)out, H, nsplit, sob); \
  } while (0)
  if (dt == 0) {
    if (D == 128) FX_DEC(bf16, 128); else FX_DEC(bf16, 64);
  } else if (dt == 1) {
    if (D == 128) FX_DEC(f16, 128); else FX_DEC(f16, 64);
  } else {
    return -3;
  }
#undef FX_DEC
  return 0;
}
