// Fused top-k / top-p (nucleus) sampling over the vocabulary (K18).
//
// The reference samples with a chain of framework ops per decode step
// (softmax, topk, sort + cumsum + scatter for top-p, multinomial,
// log_softmax + gather for the score: single_model.py:907-988).  Here one
// workgroup of 1024 threads (16 wave64s) owns one batch row and does all of
// it in a single launch, never sorting:
//
//   1. row max / sum-exp of logits/T (softmax denominators) and the
//      logsumexp of the raw logits (for the token's log-prob score);
//   2. top-k threshold by 4-pass radix select (8 bits per pass) on the fp32
//      probability bits (non-negative floats order like their bit patterns);
//      histogram in LDS, keep p >= p_(k)  (ties kept, as topk + ">=" does);
//   3. top-p threshold by the same radix walk over probability MASS: the
//      largest T with mass(p >= T) > top_p, computed on the top-k survivors
//      without renormalising -- exactly the keep rule of
//      models/language_model/gpt/generation.py:top_p_filter (keep a token iff
//      the mass ranked strictly above it is <= top_p);
//   4. inverse-CDF draw in index order with the row's uniform u: per-thread
//      contiguous chunks, block exclusive scan of chunk masses, the owning
//      thread walks its chunk.
//
// Every pass re-reads the row from global memory (a 50k-entry fp32 row is
// 200 KB: L2-resident, larger than LDS); decode batches are small, so the
// kernel is latency- not bandwidth-bound and one launch replaces ~15.
#include "fx_common.h"

namespace {

constexpr int ST = 1024;          // threads per row
constexpr int SW = ST / 64;       // waves

struct Shared {
  float red[SW];
  float red2[SW];
  unsigned int hist[256];
  float mass[256];
  float scan[ST];
  unsigned int sel_prefix;
  float sel_above;
  unsigned int sel_k;
  int pick;
};

template <typename T>
__device__ __forceinline__ float ld(const T* p, long i);
template <>
__device__ __forceinline__ float ld<float>(const float* p, long i) { return p[i]; }
template <>
__device__ __forceinline__ float ld<uint16_t>(const uint16_t* p, long i) {
  return bf16_bits_to_float(p[i]);
}

__device__ __forceinline__ float block_max(float v, Shared& s) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) s.red[w] = v;
  __syncthreads();
  float r = s.red[0];
#pragma unroll
  for (int i = 1; i < SW; ++i) r = fmaxf(r, s.red[i]);
  return r;
}
__device__ __forceinline__ float block_sum(float v, Shared& s) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) s.red2[w] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < SW; ++i) r += s.red2[i];
  return r;
}

template <typename T>
__global__ __launch_bounds__(ST) void sample_kernel(const T* __restrict__ logits, long ld_row,
                                                   int V, float inv_temp, int top_k, float top_p,
                                                   const float* __restrict__ uniforms,
                                                   int64_t* __restrict__ out_ids,
                                                   float* __restrict__ out_lse,
                                                   float* __restrict__ out_probs) {
  __shared__ Shared s;
  const int tid = threadIdx.x;
  const long row = blockIdx.x;
  const T* lg = logits + row * ld_row;

  // ---- 1. softmax denominators
  float m = -INFINITY, mraw = -INFINITY;
  for (int i = tid; i < V; i += ST) {
    const float x = ld<T>(lg, i);
    m = fmaxf(m, x * inv_temp);
    mraw = fmaxf(mraw, x);
  }
  m = block_max(m, s);
  const float mr = block_max(mraw, s);
  float se = 0.f, ser = 0.f;
  for (int i = tid; i < V; i += ST) {
    const float x = ld<T>(lg, i);
    se += __expf(x * inv_temp - m);
    ser += __expf(x - mr);
  }
  se = block_sum(se, s);
  ser = block_sum(ser, s);
  const float inv_se = 1.f / se;
  if (tid == 0 && out_lse) out_lse[row] = mr + __logf(ser);
  auto prob = [&](int i) { return __expf(ld<T>(lg, i) * inv_temp - m) * inv_se; };

  // ---- 2. top-k threshold (radix select on the probability bits)
  unsigned int kth = 0u;  // keep p_bits >= kth
  if (top_k > 0 && top_k < V) {
    if (tid == 0) {
      s.sel_prefix = 0u;
      s.sel_k = (unsigned)top_k;
    }
    for (int shift = 24; shift >= 0; shift -= 8) {
      __syncthreads();
      for (int b = tid; b < 256; b += ST) s.hist[b] = 0u;
      __syncthreads();
      const unsigned int prefix = s.sel_prefix;
      const unsigned int hmask = shift == 24 ? 0u : (0xffffffffu << (shift + 8));
      for (int i = tid; i < V; i += ST) {
        const unsigned int key = __float_as_uint(prob(i));
        if ((key & hmask) == (prefix & hmask)) atomicAdd(&s.hist[(key >> shift) & 0xffu], 1u);
      }
      __syncthreads();
      if (tid == 0) {
        unsigned int need = s.sel_k, cum = 0u;
        int b = 255;
        for (; b > 0; --b) {
          if (cum + s.hist[b] >= need) break;
          cum += s.hist[b];
        }
        s.sel_k = need - cum;
        s.sel_prefix = prefix | ((unsigned)b << shift);
      }
    }
    __syncthreads();
    kth = s.sel_prefix;
  }

  // ---- 3. top-p threshold over the top-k survivors' mass
  unsigned int pth = 0u;
  if (top_p < 1.f) {
    if (tid == 0) {
      s.sel_prefix = 0u;
      s.sel_above = 0.f;
      s.sel_k = 0u;  // 0: searching, 1: keep all, 2: stop at the current prefix
    }
    for (int shift = 24; shift >= 0; shift -= 8) {
      __syncthreads();
      for (int b = tid; b < 256; b += ST) s.mass[b] = 0.f;
      __syncthreads();
      const unsigned int prefix = s.sel_prefix;
      const unsigned int hmask = shift == 24 ? 0u : (0xffffffffu << (shift + 8));
      for (int i = tid; i < V; i += ST) {
        const float p = prob(i);
        const unsigned int key = __float_as_uint(p);
        if (key >= kth && (key & hmask) == (prefix & hmask))
          atomicAdd(&s.mass[(key >> shift) & 0xffu], p);
      }
      __syncthreads();
      if (tid == 0) {
        float above = s.sel_above;
        int b = 255;
        bool found = false;
        for (; b >= 0; --b) {
          if (above + s.mass[b] > top_p) {
            found = true;
            break;
          }
          above += s.mass[b];
        }
        if (!found) {
          // total mass <= top_p: nothing is cut (first level), or float
          // rounding between levels -- keep the bin selected so far
          s.sel_k = shift == 24 ? 1u : 2u;
        } else {
          s.sel_above = above;
          s.sel_prefix = prefix | ((unsigned)b << shift);
        }
      }
      __syncthreads();
      if (s.sel_k != 0u) break;
    }
    __syncthreads();
    pth = s.sel_k == 1u ? 0u : s.sel_prefix;
  }
  const unsigned int thr = kth > pth ? kth : pth;

  // ---- 4. inverse-CDF draw in index order
  const int chunk = (V + ST - 1) / ST;
  const int lo = min(V, tid * chunk), hi = min(V, lo + chunk);
  float part = 0.f;
  int last = -1;
  for (int i = lo; i < hi; ++i) {
    const float p = prob(i);
    const bool keep = __float_as_uint(p) >= thr;
    if (keep) {
      part += p;
      last = i;
    }
    if (out_probs) out_probs[row * (long)V + i] = keep ? p : 0.f;
  }
  s.scan[tid] = part;
  if (tid == 0) s.pick = -1;
  __syncthreads();
  // Hillis-Steele inclusive scan over 1024 chunk masses
  for (int off = 1; off < ST; off <<= 1) {
    const float v = tid >= off ? s.scan[tid - off] : 0.f;
    __syncthreads();
    s.scan[tid] += v;
    __syncthreads();
  }
  const float total = s.scan[ST - 1];
  const float target = uniforms[row] * total;
  const float excl = s.scan[tid] - part;
  if (part > 0.f && target >= excl && target < excl + part) {
    float c = excl;
    int pick = last;
    for (int i = lo; i < hi; ++i) {
      const float p = prob(i);
      if (__float_as_uint(p) < thr) continue;
      c += p;
      if (target < c) {
        pick = i;
        break;
      }
    }
    atomicMax(&s.pick, pick);
  }
  __syncthreads();
  if (s.pick < 0 && last >= 0) atomicMax(&s.pick, last);  // rounding: u*total past the end
  __syncthreads();
  if (tid == 0) out_ids[row] = s.pick < 0 ? 0 : s.pick;
}

}  // namespace

extern "C" int fx_sample(int dtype, const void* logits, long ld_row, int B, int V, float inv_temp,
                         int top_k, float top_p, const float* uniforms, int64_t* out_ids,
                         float* out_lse, float* out_probs, hipStream_t st) {
  if (B <= 0 || V <= 0) return 0;
  if (dtype == 2)
    sample_kernel<float><<<B, ST, 0, st>>>((const float*)logits, ld_row, V, inv_temp, top_k,
                                           top_p, uniforms, out_ids, out_lse, out_probs);
  else if (dtype == 0)
    sample_kernel<uint16_t><<<B, ST, 0, st>>>((const uint16_t*)logits, ld_row, V, inv_temp,
                                              top_k, top_p, uniforms, out_ids, out_lse,
                                              out_probs);
  else
    return -1;
  return 0;
}
