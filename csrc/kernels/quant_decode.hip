// QAT fake-quant (abs-max, symmetric int-N) and single-token decode attention
// over a KV cache.
//
// Parity: reference K23 (paddleslim QAT: abs_max weights / moving-average
// abs_max activations, 8 bit; `pretrain_gpt_345M_mp8_qat.yaml:35-44`) and
// K18/K19 (generation decode with a KV cache, `single_model.py:109-114`,
// Paddle fused_multi_transformer decode path).
//
// Decode attention is memory bound (one query row per (batch, head)): one
// workgroup per (batch, head), 16 lanes x 16 bytes cover a D=128 key row, so a
// wave scores 4 keys per step; online softmax per lane group, merged through
// LDS at the end.
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

// q: [B, H, D] (strides sqb, sqh); caches: [B, maxlen, H, D] (skb, sks, skh);
// out: [B, H, D] (sob, D contiguous, head stride D)
template <int D>
__global__ __launch_bounds__(256) void decode_attn_kernel(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc,
    const uint16_t* __restrict__ vc, uint16_t* __restrict__ out, const int* __restrict__ lens,
    int H, long sqb, long sqh, long skb, long sks, long skh, long sob, float scale) {
  constexpr int LPK = D / 8;        // lanes per key row
  constexpr int KPW = 64 / LPK;     // keys per wave step
  const int bh = blockIdx.x, b = bh / H, hd = bh % H;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int sub = lane / LPK, c = (lane % LPK) * 8;
  const int len = lens[b];
  float qv[8];
  load8<bf16>(q + b * sqb + hd * sqh + c, qv);
  float m = -INFINITY, l = 0.f, o[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = 0.f;
  const uint16_t* kb = kc + b * skb + hd * skh + c;
  const uint16_t* vb = vc + b * skb + hd * skh + c;
  for (int k0 = w * KPW; k0 < len; k0 += 4 * KPW) {
    const int key = k0 + sub;
    float kv[8], s = 0.f;
    const bool valid = key < len;
    if (valid) {
      load8<bf16>(kb + (long)key * sks, kv);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += kv[j] * qv[j];
    }
#pragma unroll
    for (int off = LPK / 2; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    s = valid ? s * scale : -INFINITY;
    if (valid) {
      const float mn = fmaxf(m, s);
      const float a = __expf(m - mn), p = __expf(s - mn);
      float vv[8];
      load8<bf16>(vb + (long)key * sks, vv);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = o[j] * a + p * vv[j];
      l = l * a + p;
      m = mn;
    }
  }
  // merge the KPW*4 partial states of each column slice through LDS
  __shared__ float sm_m[4 * 64], sm_l[4 * 64], sm_o[4 * 64][8];
  sm_m[threadIdx.x] = m;
  sm_l[threadIdx.x] = l;
#pragma unroll
  for (int j = 0; j < 8; ++j) sm_o[threadIdx.x][j] = o[j];
  __syncthreads();
  if (threadIdx.x < LPK) {
    float M = -INFINITY;
    for (int t = threadIdx.x; t < 256; t += LPK) M = fmaxf(M, sm_m[t]);
    float L = 0.f, O[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) O[j] = 0.f;
    for (int t = threadIdx.x; t < 256; t += LPK) {
      if (sm_m[t] == -INFINITY) continue;
      const float a = __expf(sm_m[t] - M);
      L += sm_l[t] * a;
#pragma unroll
      for (int j = 0; j < 8; ++j) O[j] += sm_o[t][j] * a;
    }
    const float inv = L > 0.f ? 1.f / L : 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) O[j] *= inv;
    store8<bf16>(out + b * sob + hd * D + threadIdx.x * 8, O);
  }
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

extern "C" int fx_decode_attn(const void* q, const void* kc, const void* vc, void* out,
                              const int* lens, int B, int H, int D, int maxlen, int nsplit,
                              long sqb, long sqh, long skb, long sks, long skh, long sob,
                              float scale, hipStream_t st) {
  (void)maxlen;
  (void)nsplit;
  if (D == 128)
    decode_attn_kernel<128><<<B * H, 256, 0, st>>>((const uint16_t*)q, (const uint16_t*)kc,
                                                  (const uint16_t*)vc, (uint16_t*)out, lens, H,
                                                  sqb, sqh, skb, sks, skh, sob, scale);
  else if (D == 64)
    decode_attn_kernel<64><<<B * H, 256, 0, st>>>((const uint16_t*)q, (const uint16_t*)kc,
                                                 (const uint16_t*)vc, (uint16_t*)out, lens, H, sqb,
                                                 sqh, skb, sks, skh, sob, scale);
  else
    return -1;
  return 0;
}
