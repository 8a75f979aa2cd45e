// Standalone fused (masked) softmax for materialised attention scores.
//
// Reference K04 / N-3: Paddle's `softmax_mask_fuse_upper_triangle` (causal,
// training path, `single_model.py:198`, `hybrid_model.py:277`) and the eval
// path's "additive mask + softmax" (`single_model.py:194-196`), i.e. the
// `incubate.softmax_mask_fuse{,_upper_triangle}` ops.  The training GPT path
// never materialises scores (flash_attn.hip); this kernel serves the
// unfused attention fallback (head_dim > 128) and users of the op API.
//
// Layout: x / y are [rows, Sk] row-major with rows = B*H*Sq (row r is query
// q = r % Sq of head-batch bh = r / Sq).  Causal: column c > q is masked (the
// upper triangle, as the reference op).  Additive mask: fp32/16-bit row
// (bh / mask_div) * Sq + q of a [*, Sq, Sk] tensor (mask_div = H broadcasts a
// [B, 1, Sq, Sk] mask over heads).
//
// CDNA4 mapping: one wave64 per row, four rows per 256-thread block.  For
// Sk <= 4096 (Sk % 8 == 0) the row lives in registers (NV 8-element chunks
// per lane), so x is read once and y written once -- the op is HBM bound and
// this is its minimum traffic; masked-out columns of a causal row are neither
// read nor exponentiated (about half the reads of a square causal score
// matrix).  Statistics are fp32; exp via the hardware exp2.
#include "fx_common.h"

namespace {

template <typename T> struct IO;
template <> struct IO<bf16> {
  static __device__ __forceinline__ void ld8(const void* p, long i, float* f) {
    load8<bf16>(reinterpret_cast<const uint16_t*>(p) + i, f);
  }
  static __device__ __forceinline__ void st8(void* p, long i, const float* f) {
    store8<bf16>(reinterpret_cast<uint16_t*>(p) + i, f);
  }
  static __device__ __forceinline__ float ld1(const void* p, long i) {
    return Elt<bf16>::to_f(reinterpret_cast<const uint16_t*>(p)[i]);
  }
  static __device__ __forceinline__ void st1(void* p, long i, float v) {
    reinterpret_cast<uint16_t*>(p)[i] = Elt<bf16>::from_f(v);
  }
};
template <> struct IO<f16> {
  static __device__ __forceinline__ void ld8(const void* p, long i, float* f) {
    load8<f16>(reinterpret_cast<const uint16_t*>(p) + i, f);
  }
  static __device__ __forceinline__ void st8(void* p, long i, const float* f) {
    store8<f16>(reinterpret_cast<uint16_t*>(p) + i, f);
  }
  static __device__ __forceinline__ float ld1(const void* p, long i) {
    return Elt<f16>::to_f(reinterpret_cast<const uint16_t*>(p)[i]);
  }
  static __device__ __forceinline__ void st1(void* p, long i, float v) {
    reinterpret_cast<uint16_t*>(p)[i] = Elt<f16>::from_f(v);
  }
};
template <> struct IO<float> {
  static __device__ __forceinline__ void ld8(const void* p, long i, float* f) {
    const float4* q = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(p) + i);
    float4 a = q[0], b = q[1];
    f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w;
    f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
  }
  static __device__ __forceinline__ void st8(void* p, long i, const float* f) {
    float4* q = reinterpret_cast<float4*>(reinterpret_cast<float*>(p) + i);
    q[0] = make_float4(f[0], f[1], f[2], f[3]);
    q[1] = make_float4(f[4], f[5], f[6], f[7]);
  }
  static __device__ __forceinline__ float ld1(const void* p, long i) {
    return reinterpret_cast<const float*>(p)[i];
  }
  static __device__ __forceinline__ void st1(void* p, long i, float v) {
    reinterpret_cast<float*>(p)[i] = v;
  }
};

constexpr float kLog2e = 1.4426950408889634f;

struct SmParams {
  const void* x;     // scores (fwd) / y (bwd)
  const void* dy;    // bwd only
  const void* mask;  // additive mask or nullptr
  void* out;         // y (fwd) / dx (bwd)
  long rows;
  int Sq, Sk;
  long mask_div;
  float scale;
};

__device__ __forceinline__ int valid_cols(int causal, int q, int Sk) {
  return causal ? min(q + 1, Sk) : Sk;
}

// -------------------------------------------------------------- register path
template <typename T, typename TM, int NV>
__global__ __launch_bounds__(256) void softmax_fwd_reg(SmParams P, int causal) {
  const int lane = threadIdx.x & 63;
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= P.rows) return;
  const int q = (int)(r % P.Sq);
  const int lim = valid_cols(causal, q, P.Sk);
  const long base = r * P.Sk;
  const long mbase = P.mask ? ((r / P.Sq) / P.mask_div * P.Sq + q) * (long)P.Sk : 0;
  const float sl = P.scale * kLog2e;  // work in the log2 domain
  float v[NV][8];
  float m = -INFINITY;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c0 = (j * 64 + lane) * 8;
    if (c0 < lim) {
      IO<T>::ld8(P.x, base + c0, v[j]);
      float mk[8];
      if (P.mask) {
        IO<TM>::ld8(P.mask, mbase + c0, mk);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) mk[e] = 0.f;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float t = v[j][e] * sl + mk[e] * kLog2e;
        if (c0 + e >= lim) t = -INFINITY;
        v[j][e] = t;
        m = fmaxf(m, t);
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[j][e] = -INFINITY;
    }
  }
  m = wave_max(m);
  const bool live = m != -INFINITY;  // a fully masked row outputs zeros
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NV; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[j][e] = live ? exp2f(v[j][e] - m) : 0.f;
      s += v[j][e];
    }
  s = wave_sum(s);
  const float inv = s > 0.f ? 1.f / s : 0.f;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c0 = (j * 64 + lane) * 8;
    if (c0 < P.Sk) {
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = v[j][e] * inv;
      IO<T>::st8(P.out, base + c0, o);
    }
  }
}

template <typename T, int NV>
__global__ __launch_bounds__(256) void softmax_bwd_reg(SmParams P, int causal) {
  const int lane = threadIdx.x & 63;
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= P.rows) return;
  const int q = (int)(r % P.Sq);
  const int lim = valid_cols(causal, q, P.Sk);
  const long base = r * P.Sk;
  float y[NV][8], g[NV][8];
  float dot = 0.f;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c0 = (j * 64 + lane) * 8;
    if (c0 < lim) {  // y == 0 on masked columns: nothing to read there
      IO<T>::ld8(P.x, base + c0, y[j]);
      IO<T>::ld8(P.dy, base + c0, g[j]);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if (c0 + e >= lim) y[j][e] = 0.f;
        dot += y[j][e] * g[j][e];
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) y[j][e] = g[j][e] = 0.f;
    }
  }
  dot = wave_sum(dot);
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c0 = (j * 64 + lane) * 8;
    if (c0 < P.Sk) {
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = P.scale * y[j][e] * (g[j][e] - dot);
      IO<T>::st8(P.out, base + c0, o);
    }
  }
}

// -------------------------------------------------------------- generic path
// Any Sk (three strided passes; the row is re-read from L2/HBM).
template <typename T, typename TM>
__global__ __launch_bounds__(256) void softmax_fwd_gen(SmParams P, int causal) {
  const int lane = threadIdx.x & 63;
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= P.rows) return;
  const int q = (int)(r % P.Sq);
  const int lim = valid_cols(causal, q, P.Sk);
  const long base = r * P.Sk;
  const long mbase = P.mask ? ((r / P.Sq) / P.mask_div * P.Sq + q) * (long)P.Sk : 0;
  const float sl = P.scale * kLog2e;
  auto val = [&](int c) {
    return IO<T>::ld1(P.x, base + c) * sl +
           (P.mask ? IO<TM>::ld1(P.mask, mbase + c) * kLog2e : 0.f);
  };
  float m = -INFINITY;
  for (int c = lane; c < lim; c += 64) m = fmaxf(m, val(c));
  m = wave_max(m);
  const bool live = m != -INFINITY;
  float s = 0.f;
  if (live)
    for (int c = lane; c < lim; c += 64) s += exp2f(val(c) - m);
  s = wave_sum(s);
  const float inv = s > 0.f ? 1.f / s : 0.f;
  for (int c = lane; c < P.Sk; c += 64)
    IO<T>::st1(P.out, base + c, (c < lim && live) ? exp2f(val(c) - m) * inv : 0.f);
}

template <typename T>
__global__ __launch_bounds__(256) void softmax_bwd_gen(SmParams P, int causal) {
  const int lane = threadIdx.x & 63;
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= P.rows) return;
  const int q = (int)(r % P.Sq);
  const int lim = valid_cols(causal, q, P.Sk);
  const long base = r * P.Sk;
  float dot = 0.f;
  for (int c = lane; c < lim; c += 64)
    dot += IO<T>::ld1(P.x, base + c) * IO<T>::ld1(P.dy, base + c);
  dot = wave_sum(dot);
  for (int c = lane; c < P.Sk; c += 64) {
    float o = 0.f;
    if (c < lim) {
      const float y = IO<T>::ld1(P.x, base + c);
      o = P.scale * y * (IO<T>::ld1(P.dy, base + c) - dot);
    }
    IO<T>::st1(P.out, base + c, o);
  }
}

template <typename T, typename TM>
void launch_fwd(const SmParams& P, int causal, hipStream_t st) {
  const int grid = fx_cdiv(P.rows, 4);
  const bool vec = (P.Sk % 8) == 0;
  if (vec && P.Sk <= 512)
    softmax_fwd_reg<T, TM, 1><<<grid, 256, 0, st>>>(P, causal);
  else if (vec && P.Sk <= 1024)
    softmax_fwd_reg<T, TM, 2><<<grid, 256, 0, st>>>(P, causal);
  else if (vec && P.Sk <= 2048)
    softmax_fwd_reg<T, TM, 4><<<grid, 256, 0, st>>>(P, causal);
  else if (vec && P.Sk <= 4096)
    softmax_fwd_reg<T, TM, 8><<<grid, 256, 0, st>>>(P, causal);
  else
    softmax_fwd_gen<T, TM><<<grid, 256, 0, st>>>(P, causal);
}

template <typename T>
void launch_bwd(const SmParams& P, int causal, hipStream_t st) {
  const int grid = fx_cdiv(P.rows, 4);
  const bool vec = (P.Sk % 8) == 0;
  if (vec && P.Sk <= 512)
    softmax_bwd_reg<T, 1><<<grid, 256, 0, st>>>(P, causal);
  else if (vec && P.Sk <= 1024)
    softmax_bwd_reg<T, 2><<<grid, 256, 0, st>>>(P, causal);
  else if (vec && P.Sk <= 2048)
    softmax_bwd_reg<T, 4><<<grid, 256, 0, st>>>(P, causal);
  else if (vec && P.Sk <= 4096)
    softmax_bwd_reg<T, 8><<<grid, 256, 0, st>>>(P, causal);
  else
    softmax_bwd_gen<T><<<grid, 256, 0, st>>>(P, causal);
}

}  // namespace

// dt / mdt: 0 bf16, 1 fp16, 2 fp32 (the mask may have its own dtype).
extern "C" int fx_softmax_fwd(int dt, int mdt, const void* x, const void* mask, void* y, long rows,
                              int Sq, int Sk, long mask_div, float scale, int causal,
                              hipStream_t st) {
  if (rows <= 0 || Sq <= 0 || Sk <= 0 || mask_div <= 0 || dt < 0 || dt > 2 || mdt < 0 || mdt > 2)
    return 1;
  SmParams P{x, nullptr, mask, y, rows, Sq, Sk, mask_div, scale};
  if (dt == 0) {
    if (mdt == 0) launch_fwd<bf16, bf16>(P, causal, st);
    else if (mdt == 1) launch_fwd<bf16, f16>(P, causal, st);
    else launch_fwd<bf16, float>(P, causal, st);
  } else if (dt == 1) {
    if (mdt == 0) launch_fwd<f16, bf16>(P, causal, st);
    else if (mdt == 1) launch_fwd<f16, f16>(P, causal, st);
    else launch_fwd<f16, float>(P, causal, st);
  } else {
    if (mdt == 0) launch_fwd<float, bf16>(P, causal, st);
    else if (mdt == 1) launch_fwd<float, f16>(P, causal, st);
    else launch_fwd<float, float>(P, causal, st);
  }
  FX_CHECK_LAUNCH();
  return 0;
}

extern "C" int fx_softmax_bwd(int dt, const void* y, const void* dy, void* dx, long rows, int Sq,
                              int Sk, float scale, int causal, hipStream_t st) {
  if (rows <= 0 || Sq <= 0 || Sk <= 0 || dt < 0 || dt > 2) return 1;
  SmParams P{y, dy, nullptr, dx, rows, Sq, Sk, 1, scale};
  if (dt == 0) launch_bwd<bf16>(P, causal, st);
  else if (dt == 1) launch_bwd<f16>(P, causal, st);
  else launch_bwd<float>(P, causal, st);
  FX_CHECK_LAUNCH();
  return 0;
}
