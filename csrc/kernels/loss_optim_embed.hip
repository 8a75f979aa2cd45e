// Softmax cross-entropy (vocab-parallel capable), fused AdamW over flat fp32
// buffers, squared-norm partials, and the (vocab-parallel) embedding.
//
// Parity: reference K10 (VocabParallelEmbedding / nn.Embedding), K11
// (ParallelCrossEntropy / CrossEntropyLoss kept in fp32), K12-K14 (multi-
// precision AdamW, ClipGradByGlobalNorm, GradScaler) -- SURVEY.md §2.10.
//
// MI355X design notes:
//  * CE: one 256-thread workgroup per token row, online (max, sum-exp) in fp32
//    over 16-byte vector loads; logits never up-cast in memory.  The backward
//    overwrites the logits buffer in place with dlogits (saves V x tokens x 2B).
//    Vocab-parallel statistics are combined by two tiny RCCL all-reduces on
//    the host side (max, then [sum, target]).
//  * AdamW: the optimizer owns flat fp32 master/grad/m/v buffers (tensor
//    fusion, reference P09), so an update is ONE launch per parameter group;
//    the clip coefficient and found-inf flag are read from device memory, so
//    the step never syncs the host.
#include "fx_common.h"

namespace {

// --------------------------------------------------------------- CE stats
template <typename T>
__global__ __launch_bounds__(256) void ce_stats_kernel(
    const uint16_t* __restrict__ logits, const int64_t* __restrict__ labels, int rows, int V,
    long vocab_start, float* __restrict__ out_max, float* __restrict__ out_sum,
    float* __restrict__ out_tgt, int ignore_index) {
  const int row = blockIdx.x;
  const uint16_t* x = logits + (size_t)row * V;
  float m = -INFINITY, s = 0.f;
  const int nv = V / 8;
  for (int v = threadIdx.x; v < nv; v += 256) {
    float a[8];
    load8<T>(x + v * 8, a);
    float lm = a[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) lm = fmaxf(lm, a[j]);
    if (lm > m) {
      s *= __expf(m - lm);
      m = lm;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) s += __expf(a[j] - m);
  }
  for (int c = nv * 8 + threadIdx.x; c < V; c += 256) {
    float a = Elt<T>::to_f(x[c]);
    if (a > m) {
      s *= __expf(m - a);
      m = a;
    }
    s += __expf(a - m);
  }
  // block reduce (max, sum)
  __shared__ float sm[4], ss[4];
  float wm = wave_max(m);
  float ws = wave_sum(m == -INFINITY ? 0.f : s * __expf(m - wm));
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) {
    sm[w] = wm;
    ss[w] = ws;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = fmaxf(fmaxf(sm[0], sm[1]), fmaxf(sm[2], sm[3]));
    float S = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) S += ss[k] * __expf(sm[k] - M);
    out_max[row] = M;
    out_sum[row] = S;
    const long lab = labels[row];
    const long local = lab - vocab_start;
    float t = 0.f;
    if (lab != ignore_index && local >= 0 && local < V) t = Elt<T>::to_f(x[local]);
    out_tgt[row] = t;
  }
}

// dlogits = (softmax - onehot) * g[row], written in place (or to dx).
template <typename T>
__global__ __launch_bounds__(256) void ce_bwd_kernel(const uint16_t* __restrict__ logits,
                                                     uint16_t* __restrict__ dx,
                                                     const int64_t* __restrict__ labels,
                                                     const float* __restrict__ lse,
                                                     const float* __restrict__ g, int V,
                                                     long vocab_start, int ignore_index) {
  const int row = blockIdx.x;
  const uint16_t* x = logits + (size_t)row * V;
  uint16_t* d = dx + (size_t)row * V;
  const float L = lse[row];
  const float gr = g[row];
  const long lab = labels[row];
  const long local = (lab == ignore_index) ? -1 : lab - vocab_start;
  const int nv = V / 8;
  for (int v = threadIdx.x; v < nv; v += 256) {
    float a[8];
    load8<T>(x + v * 8, a);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float p = __expf(a[j] - L);
      if (v * 8 + j == local) p -= 1.f;
      a[j] = p * gr;
    }
    store8<T>(d + v * 8, a);
  }
  for (int c = nv * 8 + threadIdx.x; c < V; c += 256) {
    float p = __expf(Elt<T>::to_f(x[c]) - L);
    if (c == local) p -= 1.f;
    d[c] = Elt<T>::from_f(p * gr);
  }
}

// --------------------------------------------------------------- norms
// Segmented sum of squares: block b reduces fp32 chunk b = (address, length),
// any number of separate tensors in ONE launch (the fused gradient norm's
// epilogue slots plus the gradient ranges they do not cover).  A negative
// length -n marks a chunk that already holds sums of squares (epilogue
// slots): its n values are added, not squared.
__global__ __launch_bounds__(256) void sumsq_chunks_kernel(const int64_t* __restrict__ addr,
                                                           const int64_t* __restrict__ len,
                                                           float* __restrict__ partial) {
  const float* x = reinterpret_cast<const float*>(addr[blockIdx.x]);
  const long l = len[blockIdx.x];
  const bool plain = l < 0;
  const long n = plain ? -l : l;
  float s = 0.f;
  if (plain) {
    for (long i = threadIdx.x; i < n; i += 256) s += x[i];
  } else if ((reinterpret_cast<uintptr_t>(x) & 15) == 0) {
    const long n4 = n / 4;
    const float4* x4 = reinterpret_cast<const float4*>(x);
    for (long i = threadIdx.x; i < n4; i += 256) {
      const float4 v = x4[i];
      s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    }
    for (long i = n4 * 4 + threadIdx.x; i < n; i += 256) s += x[i] * x[i];
  } else {
    for (long i = threadIdx.x; i < n; i += 256) s += x[i] * x[i];
  }
  __shared__ float red[4];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// partial[block] = sum of squares over a grid-stride slice (fp32 input)
__global__ __launch_bounds__(256) void sumsq_f32_kernel(const float* __restrict__ x, long n,
                                                        float* __restrict__ partial) {
  float s = 0.f;
  const long n4 = n / 4;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    float4 v = x4[i];
    s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  for (long i = n4 * 4 + blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    s += x[i] * x[i];
  __shared__ float red[4];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// partial[block] = sum of squares of a 16-bit (bf16 / fp16) range, fp32
// accumulation: the gradient norm over 16-bit gradient storage reads 2 B per
// element (the torch form `g.float().square().sum()` wrote and re-read an
// fp32 copy: ~15 ms per 6.7B step); 16-byte loads, a non-finite element
// (fp16 overflow) makes the sum non-finite
template <typename T>
__global__ __launch_bounds__(256) void sumsq_16_kernel(const uint16_t* __restrict__ x, long n,
                                                       float* __restrict__ partial) {
  float s = 0.f;
  const long n8 = (reinterpret_cast<uintptr_t>(x) & 15) == 0 ? n / 8 : 0;
  const uint4* x8 = reinterpret_cast<const uint4*>(x);
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    float f[8];
    unpack8<T>(x8[i], f);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += f[j] * f[j];
  }
  for (long i = n8 * 8 + blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float f = Elt<T>::to_f(x[i]);
    s += f * f;
  }
  __shared__ float red[4];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// --------------------------------------------------------------- AdamW
// p (fp32 master), g (fp32), m, v (fp32); optional 16-bit model copy.
//  * gscale: device scalar multiplied into g (clip coefficient x 1/loss-scale);
//  * skip: device int (fp16 found-inf) -> no update at all;
//  * step: device int = number of APPLIED updates including this one (the
//    optimizer advances it only when skip == 0, so an overflowed step does
//    not advance Adam's bias corrections -- Paddle's beta_pow semantics);
//  * wd: decoupled decay (AdamW); l2: classic L2 term added to the ALREADY
//    clipped / unscaled gradient (Adam; Paddle applies regularisation after
//    gradient clipping).
// Streaming: 2 float4 groups per thread per iteration with every load issued
// before any math (8 x 16-byte loads in flight per lane), non-temporal
// accesses (each byte is touched once per step, keep it out of L2/MALL).
template <typename V>
__device__ __forceinline__ V ld_stream(const V* a, bool nt) {
  return nt ? __builtin_nontemporal_load(a) : *a;
}
template <typename V>
__device__ __forceinline__ void st_stream(V x, V* a, bool nt) {
  if (nt) __builtin_nontemporal_store(x, a); else *a = x;
}

// BS threads per block, U float4 groups per thread per pass (4U x 16-byte
// loads in flight per lane).  The default (256, 2) fills the chip; the
// forward-overlapped update runs (1024, 4) on a capped grid instead: few CUs,
// each with 256 KiB of loads in flight, so the GEMMs beside it keep the rest
// of the chip (optims/optimizer.py, _update_overlapped).
// G16: the gradient is stored in the model's 16-bit dtype (the bf16
// gradient storage of Distributed.comm.grad_dtype: 2 B read per parameter
// instead of 4 -- 28 instead of 30 B per parameter per step)
// The raw gradient group (4 x 16 bit or 4 x fp32) is loaded with the other
// streams and widened only in the compute loop: widening it at the load made
// the compiler wait for each group's gradient before issuing the next group's
// loads (4 loads in flight per lane instead of 4U; gfx950 ISA of the G16
// instance), and the G16 update ran 14 % longer than the fp32 one beside the
// forward GEMMs (profiles/r5_grad16/).
template <bool G16>
struct GradRaw { using type = floatx4; };
template <>
struct GradRaw<true> { using type = unsigned long long; };

template <bool G16>
__device__ __forceinline__ typename GradRaw<G16>::type adamw_ld_grad(const void* g, long i,
                                                                      bool nt) {
  return ld_stream(reinterpret_cast<const typename GradRaw<G16>::type*>(g) + i, nt);
}

template <typename T, bool G16>
__device__ __forceinline__ floatx4 adamw_widen(typename GradRaw<G16>::type h) {
  if constexpr (G16)
    return floatx4{Elt<T>::to_f((uint16_t)h), Elt<T>::to_f((uint16_t)(h >> 16)),
                   Elt<T>::to_f((uint16_t)(h >> 32)), Elt<T>::to_f((uint16_t)(h >> 48))};
  else
    return h;
}

template <typename T, bool G16>
__device__ __forceinline__ float adamw_grad1(const void* g, long i) {
  if constexpr (G16) return Elt<T>::to_f(reinterpret_cast<const uint16_t*>(g)[i]);
  else return reinterpret_cast<const float*>(g)[i];
}

// Packed master (PK, bf16 models): the fp32 master x is stored as the bf16
// parameter itself (hi) plus x's low 16 bits (lo), so the update reads and
// writes 2 + 2 B of master+parameter instead of 4 + 4 (fp32 master) + 2
// (parameter copy): 26 instead of 28 B per parameter with bf16 gradients.
// hi = x's high half rounded to nearest on the low half (ties toward zero);
// x = ((hi - (lo > 0x8000)) << 16) | lo is exact, so the master keeps every
// fp32 bit and the parameter differs from a round-to-nearest-even cast only
// when the low half is exactly 0x8000.
__device__ __forceinline__ float pk_decode(uint32_t hi, uint32_t lo) {
  const uint32_t top = hi - (lo > 0x8000u ? 1u : 0u);
  return __uint_as_float((top << 16) | lo);
}
__device__ __forceinline__ void pk_encode(float x, uint32_t& hi, uint32_t& lo) {
  const uint32_t b = __float_as_uint(x);
  lo = b & 0xffffu;
  hi = ((b >> 16) + (lo > 0x8000u ? 1u : 0u)) & 0xffffu;
}

// One element of the update with every rounding spelled out (explicit fma,
// no contraction left to the compiler): each kernel instance -- fp32 / 16-bit
// gradient, packed / fp32 master, vector body / scalar tail -- computes the
// same bits, whatever the vectorizer makes of the surrounding code.
__device__ __forceinline__ void adamw_elem(float& p, float& m, float& v, float g, float gs,
                                           float l2, float beta1, float beta2,
                                           float inv_sqrt_bc2, float eps, float decay,
                                           float step_size) {
#pragma clang fp contract(off)
  const float gr = __builtin_fmaf(g, gs, l2 * p);
  m = __builtin_fmaf(beta1, m, (1.f - beta1) * gr);
  v = __builtin_fmaf(beta2, v, ((1.f - beta2) * gr) * gr);
  const float denom = __builtin_fmaf(__builtin_sqrtf(v), inv_sqrt_bc2, eps);
  p = __builtin_fmaf(p, decay, -((step_size * m) / denom));
}

template <typename T, bool NT, int BS, int U, bool G16 = false, bool PK = false>
__global__ __launch_bounds__(BS) void adamw_flat_kernel(
    float* __restrict__ p, const void* __restrict__ g, float* __restrict__ m,
    float* __restrict__ v, uint16_t* __restrict__ p16, long n, float lr, float beta1,
    float beta2, float eps, float wd, float l2, const float* __restrict__ gscale,
    const int* __restrict__ skip, const int* __restrict__ step, const float* __restrict__ lr_dev) {
  if (skip && *skip) return;
  if (lr_dev != nullptr) lr = *lr_dev;  // graph mode: the scheduler's lr lives on the device
  const float gs = gscale ? *gscale : 1.f;
  const float t = (float)(*step);
  const float bc1 = 1.f - __powf(beta1, t);
  const float bc2 = 1.f - __powf(beta2, t);
  const float step_size = lr / bc1;
  const float inv_sqrt_bc2 = rsqrtf(bc2);
  const float decay = 1.f - lr * wd;
  const long n4 = n / 4;
  const long stride = (long)gridDim.x * (BS * U);
  for (long i0 = blockIdx.x * (long)(BS * U) + threadIdx.x; i0 < n4; i0 += stride) {
    floatx4 pp[U], mm[U], vv[U];
    unsigned long long ph[PK ? U : 1], pl[PK ? U : 1];  // PK: raw hi / lo halves
    typename GradRaw<G16>::type gg[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = i0 + (long)u * BS;
      if (i < n4) {
        if constexpr (PK) {
          ph[u] = ld_stream(reinterpret_cast<const unsigned long long*>(p16) + i, NT);
          pl[u] = ld_stream(reinterpret_cast<const unsigned long long*>(p) + i, NT);
        } else {
          pp[u] = ld_stream(reinterpret_cast<const floatx4*>(p) + i, NT);
        }
        gg[u] = adamw_ld_grad<G16>(g, i, NT);
        mm[u] = ld_stream(reinterpret_cast<const floatx4*>(m) + i, NT);
        vv[u] = ld_stream(reinterpret_cast<const floatx4*>(v) + i, NT);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = i0 + (long)u * BS;
      if (i >= n4) break;
      floatx4 pa, ma = mm[u], va = vv[u];
      if constexpr (PK) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          pa[j] = pk_decode((uint32_t)(ph[u] >> (16 * j)) & 0xffffu,
                            (uint32_t)(pl[u] >> (16 * j)) & 0xffffu);
      } else {
        pa = pp[u];
      }
      const floatx4 ga = adamw_widen<T, G16>(gg[u]);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float pj = pa[j], mj = ma[j], vj = va[j];
        adamw_elem(pj, mj, vj, ga[j], gs, l2, beta1, beta2, inv_sqrt_bc2, eps, decay, step_size);
        pa[j] = pj;
        ma[j] = mj;
        va[j] = vj;
      }
      st_stream(ma, reinterpret_cast<floatx4*>(m) + i, NT);
      st_stream(va, reinterpret_cast<floatx4*>(v) + i, NT);
      if constexpr (PK) {
        unsigned long long hw = 0, lw = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          uint32_t hj, lj;
          pk_encode(pa[j], hj, lj);
          hw |= (unsigned long long)hj << (16 * j);
          lw |= (unsigned long long)lj << (16 * j);
        }
        st_stream(hw, reinterpret_cast<unsigned long long*>(p16) + i, NT);
        st_stream(lw, reinterpret_cast<unsigned long long*>(p) + i, NT);
        continue;
      }
      st_stream(pa, reinterpret_cast<floatx4*>(p) + i, NT);
      if (p16) {
        ushort4 o;
        o.x = Elt<T>::from_f(pa[0]);
        o.y = Elt<T>::from_f(pa[1]);
        o.z = Elt<T>::from_f(pa[2]);
        o.w = Elt<T>::from_f(pa[3]);
        reinterpret_cast<ushort4*>(p16)[i] = o;
      }
    }
  }
  for (long i = n4 * 4 + blockIdx.x * (long)BS + threadIdx.x; i < n; i += (long)gridDim.x * BS) {
    uint16_t* plo = reinterpret_cast<uint16_t*>(p);
    float x = PK ? pk_decode(p16[i], plo[i]) : p[i];
    float mi = m[i], vi = v[i];
    adamw_elem(x, mi, vi, adamw_grad1<T, G16>(g, i), gs, l2, beta1, beta2, inv_sqrt_bc2, eps,
               decay, step_size);
    m[i] = mi;
    v[i] = vi;
    if constexpr (PK) {
      uint32_t hj, lj;
      pk_encode(x, hj, lj);
      p16[i] = (uint16_t)hj;
      plo[i] = (uint16_t)lj;
    } else {
      p[i] = x;
      if (p16) p16[i] = Elt<T>::from_f(x);
    }
  }
}

// packed-master helpers for checkpoints / tests: fp32 master <-> (hi, lo)
__global__ __launch_bounds__(256) void pk_split_kernel(const float* __restrict__ x,
                                                       uint16_t* __restrict__ hi,
                                                       uint16_t* __restrict__ lo, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    uint32_t h, l;
    pk_encode(x[i], h, l);
    hi[i] = (uint16_t)h;
    lo[i] = (uint16_t)l;
  }
}
__global__ __launch_bounds__(256) void pk_join_kernel(const uint16_t* __restrict__ hi,
                                                      const uint16_t* __restrict__ lo,
                                                      float* __restrict__ x, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    x[i] = pk_decode(hi[i], lo[i]);
}

template <typename T>
__global__ __launch_bounds__(256) void cast_f32_kernel(const float* __restrict__ x,
                                                       uint16_t* __restrict__ y, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    y[i] = Elt<T>::from_f(x[i]);
}

// acc(fp32) += x (16-bit), used by grad-accumulation hooks
template <typename T>
__global__ __launch_bounds__(256) void accum_f32_kernel(float* __restrict__ acc,
                                                        const uint16_t* __restrict__ x, long n,
                                                        int overwrite) {
  const long n8 = n / 8;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    float a[8];
    load8<T>(x + i * 8, a);
    float4* dst = reinterpret_cast<float4*>(acc + i * 8);
    float4 d0 = overwrite ? make_float4(0, 0, 0, 0) : dst[0];
    float4 d1 = overwrite ? make_float4(0, 0, 0, 0) : dst[1];
    d0.x += a[0]; d0.y += a[1]; d0.z += a[2]; d0.w += a[3];
    d1.x += a[4]; d1.y += a[5]; d1.z += a[6]; d1.w += a[7];
    dst[0] = d0;
    dst[1] = d1;
  }
  for (long i = n8 * 8 + blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    acc[i] = (overwrite ? 0.f : acc[i]) + Elt<T>::to_f(x[i]);
}

// --------------------------------------------------------------- embedding
// out[t] = (id in shard ? W[id - vstart] : 0) + (P ? P[pos[t]] : 0)
template <typename T>
__global__ __launch_bounds__(256) void embedding_fwd_kernel(
    const int64_t* __restrict__ ids, const int64_t* __restrict__ pos,
    const uint16_t* __restrict__ W, const uint16_t* __restrict__ P, uint16_t* __restrict__ out,
    int ntok, int h, long vstart, long vsize) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= ntok) return;
  const long id = ids[t] - vstart;
  const bool in = id >= 0 && id < vsize;
  const long pp = P ? pos[t] : 0;
  for (int c = lane * 8; c < h; c += 512) {
    float a[8];
    if (in) load8<T>(W + (size_t)id * h + c, a);
    else {
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] = 0.f;
    }
    if (P) {
      float b[8];
      load8<T>(P + (size_t)pp * h + c, b);
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += b[j];
    }
    store8<T>(out + (size_t)t * h + c, a);
  }
}

// dW[id - vstart] += dout[t] (fp32 atomics, 256 contiguous bytes per wave op)
template <typename T>
__global__ __launch_bounds__(256) void embedding_bwd_kernel(const int64_t* __restrict__ ids,
                                                            const uint16_t* __restrict__ dout,
                                                            float* __restrict__ dW, int ntok, int h,
                                                            long vstart, long vsize) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= ntok) return;
  const long id = ids[t] - vstart;
  if (id < 0 || id >= vsize) return;
  float* dst = dW + (size_t)id * h;
  const uint16_t* src = dout + (size_t)t * h;
  for (int c = lane; c < h; c += 64) atomicAdd(dst + c, Elt<T>::to_f(src[c]));
}

// Deterministic variant (Global.deterministic): ids pre-sorted (stable) with
// their token permutation; the wave at the head of each equal-id segment sums
// that segment's rows in token order and does a plain read-add-write, so the
// fp32 result is bitwise reproducible run to run (no atomics ordering).
template <typename T>
__global__ __launch_bounds__(256) void embedding_bwd_sorted_kernel(
    const int64_t* __restrict__ sid, const int64_t* __restrict__ perm,
    const uint16_t* __restrict__ dout, float* __restrict__ dW, int ntok, int h, long vstart,
    long vsize) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= ntok) return;
  const long id = sid[i];
  if (i > 0 && sid[i - 1] == id) return;  // not a segment head
  const long row = id - vstart;
  if (row < 0 || row >= vsize) return;
  int end = i + 1;
  while (end < ntok && sid[end] == id) ++end;
  float* dst = dW + (size_t)row * h;
  for (int c = lane; c < h; c += 64) {
    float acc = dst[c];
    for (int j = i; j < end; ++j) acc += Elt<T>::to_f(dout[(size_t)perm[j] * h + c]);
    dst[c] = acc;
  }
}

inline int grid_n(long n, int per = 256) {
  long g = (n + per - 1) / per;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

#define FX_DISPATCH_T(dtype, ...) \
  if (dtype == 0) {               \
    using T = bf16;               \
    __VA_ARGS__;                  \
  } else {                        \
    using T = f16;                \
    __VA_ARGS__;                  \
  }

extern "C" void fx_ce_stats(int dtype, const void* logits, const int64_t* labels, int rows, int V,
                            long vocab_start, float* out_max, float* out_sum, float* out_tgt,
                            int ignore_index, hipStream_t st) {
  FX_DISPATCH_T(dtype, ce_stats_kernel<T><<<rows, 256, 0, st>>>(
                           (const uint16_t*)logits, labels, rows, V, vocab_start, out_max, out_sum,
                           out_tgt, ignore_index));
}

extern "C" void fx_ce_bwd(int dtype, const void* logits, void* dx, const int64_t* labels,
                          const float* lse, const float* g, int rows, int V, long vocab_start,
                          int ignore_index, hipStream_t st) {
  FX_DISPATCH_T(dtype, ce_bwd_kernel<T><<<rows, 256, 0, st>>>(
                           (const uint16_t*)logits, (uint16_t*)dx, labels, lse, g, V, vocab_start,
                           ignore_index));
}

extern "C" int fx_sumsq_blocks(long n) { return grid_n(n / 4 + 1, 256) > 1024 ? 1024 : grid_n(n / 4 + 1, 256); }

extern "C" void fx_sumsq_chunks(const int64_t* addr, const int64_t* len, int nchunks,
                                float* partial, hipStream_t st) {
  if (nchunks > 0) sumsq_chunks_kernel<<<nchunks, 256, 0, st>>>(addr, len, partial);
}

extern "C" void fx_sumsq_16(int dtype, const void* x, long n, float* partial, int blocks,
                            hipStream_t st) {
  FX_DISPATCH_T(dtype, sumsq_16_kernel<T><<<blocks, 256, 0, st>>>(
                           reinterpret_cast<const uint16_t*>(x), n, partial));
}
extern "C" void fx_sumsq_f32(const float* x, long n, float* partial, int blocks, hipStream_t st) {
  sumsq_f32_kernel<<<blocks, 256, 0, st>>>(x, n, partial);
}

static int g_adamw_grid = 0, g_adamw_nt = 1, g_adamw_wide = 0;  // tuning knobs
static const float* g_adamw_lr = nullptr;     // graph mode: device learning rate
extern "C" void fx_set_adamw_lr_ptr(const void* p) { g_adamw_lr = (const float*)p; }
// grid: workgroup cap (0 = fill the chip); nt: non-temporal accesses;
// wide: 1 = 1024-thread blocks with 4 float4 groups per thread (the capped,
// forward-overlapped update), 0 = 256 x 2
extern "C" void fx_adamw_tune(int grid, int nt, int wide) {
  g_adamw_grid = grid;
  g_adamw_nt = nt;
  g_adamw_wide = wide;
}

template <typename T, bool NT, int BS, int U, bool G16 = false, bool PK = false>
static void adamw_launch(float* p, const void* g, float* m, float* v, void* p16, long n,
                         float lr, float beta1, float beta2, float eps, float wd, float l2,
                         const float* gscale, const int* skip, const int* step, hipStream_t st) {
  // at most 8 resident 256-thread blocks per CU (2 of 1024)
  const long per = (long)BS * U * 4;
  long blocks = (n + per - 1) / per;
  const long cap = 256L * (8 * 256 / BS) * 4;
  int grid = (int)(blocks < 1 ? 1 : (blocks > cap ? cap : blocks));
  if (g_adamw_grid > 0 && g_adamw_grid < grid) grid = g_adamw_grid;
  adamw_flat_kernel<T, NT, BS, U, G16, PK><<<grid, BS, 0, st>>>(p, g, m, v, (uint16_t*)p16, n, lr, beta1,
                                                      beta2, eps, wd, l2, gscale, skip, step,
                                                      g_adamw_lr);
}

extern "C" void fx_adamw_flat(int dtype, float* p, const float* g, float* m, float* v, void* p16,
                              long n, float lr, float beta1, float beta2, float eps, float wd,
                              float l2, const float* gscale, const int* skip, const int* step,
                              hipStream_t st) {
#define FX_ADAMW_ARGS p, g, m, v, p16, n, lr, beta1, beta2, eps, wd, l2, gscale, skip, step, st
  if (g_adamw_wide) {
    FX_DISPATCH_T(dtype, adamw_launch<T, true, 1024, 4>(FX_ADAMW_ARGS));
  } else if (g_adamw_nt) {
    FX_DISPATCH_T(dtype, adamw_launch<T, true, 256, 2>(FX_ADAMW_ARGS));
  } else {
    FX_DISPATCH_T(dtype, adamw_launch<T, false, 256, 2>(FX_ADAMW_ARGS));
  }
#undef FX_ADAMW_ARGS
}

// the same with a 16-bit gradient (model dtype)
extern "C" void fx_adamw_flat_g16(int dtype, float* p, const void* g, float* m, float* v,
                                  void* p16, long n, float lr, float beta1, float beta2, float eps,
                                  float wd, float l2, const float* gscale, const int* skip,
                                  const int* step, hipStream_t st) {
#define FX_ADAMW_ARGS p, g, m, v, p16, n, lr, beta1, beta2, eps, wd, l2, gscale, skip, step, st
  if (g_adamw_wide) {
    FX_DISPATCH_T(dtype, (adamw_launch<T, true, 1024, 4, true>(FX_ADAMW_ARGS)));
  } else if (g_adamw_nt) {
    FX_DISPATCH_T(dtype, (adamw_launch<T, true, 256, 2, true>(FX_ADAMW_ARGS)));
  } else {
    FX_DISPATCH_T(dtype, (adamw_launch<T, false, 256, 2, true>(FX_ADAMW_ARGS)));
  }
#undef FX_ADAMW_ARGS
}

// packed master (bf16 models only): `p` is the master's low-half array, `p16`
// the bf16 parameters (= the high halves), read and written
#define FX_ADAMW_PK(G16)                                                                     \
  do {                                                                                       \
    if (dtype != 0) return -1;                                                               \
    if (g_adamw_wide)                                                                        \
      adamw_launch<bf16, true, 1024, 4, G16, true>(FX_ADAMW_ARGS);                           \
    else if (g_adamw_nt)                                                                     \
      adamw_launch<bf16, true, 256, 2, G16, true>(FX_ADAMW_ARGS);                            \
    else                                                                                     \
      adamw_launch<bf16, false, 256, 2, G16, true>(FX_ADAMW_ARGS);                           \
    return 0;                                                                                \
  } while (0)
extern "C" int fx_adamw_flat_pk(int dtype, void* lo, const void* g, float* m, float* v, void* hi,
                                long n, float lr, float beta1, float beta2, float eps, float wd,
                                float l2, const float* gscale, const int* skip, const int* step,
                                hipStream_t st) {
  float* p = (float*)lo;
  void* p16 = hi;
#define FX_ADAMW_ARGS p, g, m, v, p16, n, lr, beta1, beta2, eps, wd, l2, gscale, skip, step, st
  FX_ADAMW_PK(false);
#undef FX_ADAMW_ARGS
}
extern "C" int fx_adamw_flat_pk_g16(int dtype, void* lo, const void* g, float* m, float* v,
                                    void* hi, long n, float lr, float beta1, float beta2,
                                    float eps, float wd, float l2, const float* gscale,
                                    const int* skip, const int* step, hipStream_t st) {
  float* p = (float*)lo;
  void* p16 = hi;
#define FX_ADAMW_ARGS p, g, m, v, p16, n, lr, beta1, beta2, eps, wd, l2, gscale, skip, step, st
  FX_ADAMW_PK(true);
#undef FX_ADAMW_ARGS
}
#undef FX_ADAMW_PK

// fp32 master <-> (bf16 parameter, low halves)
extern "C" void fx_pk_split(const float* x, void* hi, void* lo, long n, hipStream_t st) {
  pk_split_kernel<<<grid_n(n), 256, 0, st>>>(x, (uint16_t*)hi, (uint16_t*)lo, n);
}
extern "C" void fx_pk_join(const void* hi, const void* lo, float* x, long n, hipStream_t st) {
  pk_join_kernel<<<grid_n(n), 256, 0, st>>>((const uint16_t*)hi, (const uint16_t*)lo, x, n);
}

extern "C" void fx_cast_f32(int dtype, const float* x, void* y, long n, hipStream_t st) {
  FX_DISPATCH_T(dtype, cast_f32_kernel<T><<<grid_n(n), 256, 0, st>>>(x, (uint16_t*)y, n));
}

extern "C" void fx_accum_f32(int dtype, float* acc, const void* x, long n, int overwrite,
                             hipStream_t st) {
  FX_DISPATCH_T(dtype, accum_f32_kernel<T><<<grid_n(n / 8 + 1), 256, 0, st>>>(
                           acc, (const uint16_t*)x, n, overwrite));
}

extern "C" void fx_embedding_fwd(int dtype, const int64_t* ids, const int64_t* pos, const void* W,
                                 const void* P, void* out, int ntok, int h, long vstart,
                                 long vsize, hipStream_t st) {
  FX_DISPATCH_T(dtype, embedding_fwd_kernel<T><<<(ntok + 3) / 4, 256, 0, st>>>(
                           ids, pos, (const uint16_t*)W, (const uint16_t*)P, (uint16_t*)out, ntok,
                           h, vstart, vsize));
}

extern "C" void fx_embedding_bwd(int dtype, const int64_t* ids, const void* dout, float* dW,
                                 int ntok, int h, long vstart, long vsize, hipStream_t st) {
  FX_DISPATCH_T(dtype, embedding_bwd_kernel<T><<<(ntok + 3) / 4, 256, 0, st>>>(
                           ids, (const uint16_t*)dout, dW, ntok, h, vstart, vsize));
}

extern "C" void fx_embedding_bwd_sorted(int dtype, const int64_t* sid, const int64_t* perm,
                                        const void* dout, float* dW, int ntok, int h, long vstart,
                                        long vsize, hipStream_t st) {
  FX_DISPATCH_T(dtype, embedding_bwd_sorted_kernel<T><<<(ntok + 3) / 4, 256, 0, st>>>(
                           sid, perm, (const uint16_t*)dout, dW, ntok, h, vstart, vsize));
}
