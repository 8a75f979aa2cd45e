// Fused GroupNorm (+ per-(b,c) FiLM scale/shift) (+ SiLU) for NCHW
// activations, forward and backward, gfx950 / wave64.
//
// Parity: reference Imagen UNet ``Block`` = GroupNorm -> x*(scale+1)+shift ->
// SiLU -> conv (``imagen/unet.py:331-344``), SURVEY.md K21: "GroupNorm+SiLU as a
// fused HIP kernel".
//
// Layout: x is [B, C, HW] contiguous, so each (b, c) is one contiguous row.
// Rows are cut into `nseg` segments (host picks nseg so the launch has enough
// workgroups to fill 256 CUs even for batch-1 super-resolution shapes).
//
//  fwd K1 gn_row_stats : per (row, seg) fp32 sum / sum-of-squares of the
//                        segment, combined across threads in fp64 -> part[row,seg,2]
//  fwd K2 gn_apply     : each WG sums its group's partials (fp64), normalises,
//                        applies gamma/beta, FiLM and SiLU, writes y; seg 0 of
//                        the group's first channel stores mean/rstd for backward
//  bwd K3 gn_bwd_reduce: recomputes z (pre-SiLU) from x and the saved stats and
//                        reduces A = sum dz*xhat, Bz = sum dz per (row, seg)
//  (host: tiny [B,C] / [B,G] combinations in PyTorch)
//  bwd K4 gn_bwd_apply : dx = rstd*(k*dz - g1 - xhat*g2), k = gamma*(1+scale)
// Every element pass is a single streaming read (K1, K3) or read+write (K2,
// K4) of 16-bit data, 8 elements per lane when the row length allows.
#include "fx_common.h"

namespace {

constexpr int GN_T = 256;

__device__ __forceinline__ double block_sum_d(double v, double* sh) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if (lane == 0) sh[w] = v;
  __syncthreads();
  double r = 0.0;
#pragma unroll
  for (int i = 0; i < GN_T / 64; ++i) r += sh[i];
  __syncthreads();
  return r;
}

__device__ __forceinline__ float block_sum_f(float v, float* sh) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = wave_sum(v);
  if (lane == 0) sh[w] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < GN_T / 64; ++i) r += sh[i];
  __syncthreads();
  return r;
}

__device__ __forceinline__ float sigmoidf_(float z) { return 1.f / (1.f + __expf(-z)); }

// segment [s0, s1) of a row; VEC: 8-wide (row length and s0 multiple of 8)
template <typename T, bool VEC, typename F>
__device__ __forceinline__ void for_segment(const uint16_t* row, long s0, long s1, F&& f) {
  if constexpr (VEC) {
    for (long i = s0 + threadIdx.x * 8; i < s1; i += GN_T * 8) {
      float v[8];
      load8<T>(row + i, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) f(i + j, v[j]);
    }
  } else {
    for (long i = s0 + threadIdx.x; i < s1; i += GN_T) f(i, Elt<T>::to_f(row[i]));
  }
}

template <typename T, bool VEC>
__global__ __launch_bounds__(GN_T) void gn_row_stats(const uint16_t* x, double* part, long hw,
                                                     int nseg, long seglen) {
  __shared__ double sh[GN_T / 64];
  const long row = blockIdx.x;
  const int seg = blockIdx.y;
  const long s0 = seg * seglen, s1 = min(hw, s0 + seglen);
  float s = 0.f, q = 0.f;
  for_segment<T, VEC>(x + row * hw, s0, s1, [&](long, float v) {
    s += v;
    q += v * v;
  });
  const double ds = block_sum_d((double)s, sh);
  const double dq = block_sum_d((double)q, sh);
  if (threadIdx.x == 0) {
    part[(row * nseg + seg) * 2 + 0] = ds;
    part[(row * nseg + seg) * 2 + 1] = dq;
  }
}

// group statistics from the partials of channels [g*cpg, (g+1)*cpg) of batch b
__device__ __forceinline__ void group_stats(const double* part, int b, int C, int g, int cpg,
                                            int nseg, long hw, float eps, double* sh, float& mean,
                                            float& rstd) {
  const long base = ((long)b * C + (long)g * cpg) * nseg;
  const int n = cpg * nseg;
  double s = 0.0, q = 0.0;
  for (int i = threadIdx.x; i < n; i += GN_T) {
    s += part[(base + i) * 2];
    q += part[(base + i) * 2 + 1];
  }
  s = block_sum_d(s, sh);
  q = block_sum_d(q, sh);
  const double cnt = (double)cpg * (double)hw;
  const double m = s / cnt;
  double var = q / cnt - m * m;
  var = var < 0.0 ? 0.0 : var;
  mean = (float)m;
  rstd = (float)(1.0 / sqrt(var + (double)eps));
}

template <typename T, bool VEC>
__global__ __launch_bounds__(GN_T) void gn_apply(const uint16_t* x, const double* part,
                                                 const float* gamma, const float* beta,
                                                 const float* scale, const float* shift,
                                                 uint16_t* y, float* mean_out, float* rstd_out,
                                                 int C, int G, long hw, int nseg, long seglen,
                                                 float eps, int silu) {
  __shared__ double sh[GN_T / 64];
  const long row = blockIdx.x;
  const int seg = blockIdx.y;
  const int b = row / C, c = row % C, cpg = C / G, g = c / cpg;
  float mean, rstd;
  group_stats(part, b, C, g, cpg, nseg, hw, eps, sh, mean, rstd);
  if (threadIdx.x == 0 && seg == 0 && c % cpg == 0) {
    mean_out[b * G + g] = mean;
    rstd_out[b * G + g] = rstd;
  }
  const float ga = gamma ? gamma[c] : 1.f, be = beta ? beta[c] : 0.f;
  const float s1 = scale ? scale[row] + 1.f : 1.f, sf = shift ? shift[row] : 0.f;
  // z = ((x-mean)*rstd*ga + be)*s1 + sf = x*A + Bc
  const float A = rstd * ga * s1, Bc = (be - mean * rstd * ga) * s1 + sf;
  const long s0 = seg * seglen, s1e = min(hw, s0 + seglen);
  const uint16_t* xr = x + row * hw;
  uint16_t* yr = y + row * hw;
  if constexpr (VEC) {
    for (long i = s0 + threadIdx.x * 8; i < s1e; i += GN_T * 8) {
      float v[8];
      load8<T>(xr + i, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float z = v[j] * A + Bc;
        v[j] = silu ? z * sigmoidf_(z) : z;
      }
      store8<T>(yr + i, v);
    }
  } else {
    for (long i = s0 + threadIdx.x; i < s1e; i += GN_T) {
      const float z = Elt<T>::to_f(xr[i]) * A + Bc;
      yr[i] = Elt<T>::from_f(silu ? z * sigmoidf_(z) : z);
    }
  }
}

// dz from dy at pre-activation z
__device__ __forceinline__ float dz_of(float dy, float z, int silu) {
  if (!silu) return dy;
  const float sg = sigmoidf_(z);
  return dy * sg * (1.f + z * (1.f - sg));
}

template <typename T, bool VEC>
__global__ __launch_bounds__(GN_T) void gn_bwd_reduce(const uint16_t* x, const uint16_t* dy,
                                                      const float* mean, const float* rstd,
                                                      const float* gamma, const float* beta,
                                                      const float* scale, const float* shift,
                                                      float* part, int C, int G, long hw, int nseg,
                                                      long seglen, int silu) {
  __shared__ float sh[GN_T / 64];
  const long row = blockIdx.x;
  const int seg = blockIdx.y;
  const int b = row / C, c = row % C, g = c / (C / G);
  const float mu = mean[b * G + g], rs = rstd[b * G + g];
  const float ga = gamma ? gamma[c] : 1.f, be = beta ? beta[c] : 0.f;
  const float s1 = scale ? scale[row] + 1.f : 1.f, sf = shift ? shift[row] : 0.f;
  const long s0 = seg * seglen, s1e = min(hw, s0 + seglen);
  const uint16_t* xr = x + row * hw;
  const uint16_t* gr = dy + row * hw;
  float a = 0.f, bz = 0.f;
  if constexpr (VEC) {
    for (long i = s0 + threadIdx.x * 8; i < s1e; i += GN_T * 8) {
      float v[8], d[8];
      load8<T>(xr + i, v);
      load8<T>(gr + i, d);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xh = (v[j] - mu) * rs;
        const float z = (xh * ga + be) * s1 + sf;
        const float dz = dz_of(d[j], z, silu);
        a += dz * xh;
        bz += dz;
      }
    }
  } else {
    for (long i = s0 + threadIdx.x; i < s1e; i += GN_T) {
      const float xh = (Elt<T>::to_f(xr[i]) - mu) * rs;
      const float z = (xh * ga + be) * s1 + sf;
      const float dz = dz_of(Elt<T>::to_f(gr[i]), z, silu);
      a += dz * xh;
      bz += dz;
    }
  }
  a = block_sum_f(a, sh);
  bz = block_sum_f(bz, sh);
  if (threadIdx.x == 0) {
    part[(row * nseg + seg) * 2 + 0] = a;
    part[(row * nseg + seg) * 2 + 1] = bz;
  }
}

// dx = rstd * (k*dz - g1 - xhat*g2);  k[row] = gamma*(1+scale), g1/g2 per (b,g)
template <typename T, bool VEC>
__global__ __launch_bounds__(GN_T) void gn_bwd_apply(const uint16_t* x, const uint16_t* dy,
                                                     const float* mean, const float* rstd,
                                                     const float* gamma, const float* beta,
                                                     const float* scale, const float* shift,
                                                     const float* g1, const float* g2,
                                                     uint16_t* dx, int C, int G, long hw,
                                                     long seglen, int silu) {
  const long row = blockIdx.x;
  const int seg = blockIdx.y;
  const int b = row / C, c = row % C, g = c / (C / G);
  const float mu = mean[b * G + g], rs = rstd[b * G + g];
  const float ga = gamma ? gamma[c] : 1.f, be = beta ? beta[c] : 0.f;
  const float s1 = scale ? scale[row] + 1.f : 1.f, sf = shift ? shift[row] : 0.f;
  const float k = ga * s1, a1 = g1[b * G + g], a2 = g2[b * G + g];
  const long s0 = seg * seglen, s1e = min(hw, s0 + seglen);
  const uint16_t* xr = x + row * hw;
  const uint16_t* gr = dy + row * hw;
  uint16_t* dr = dx + row * hw;
  if constexpr (VEC) {
    for (long i = s0 + threadIdx.x * 8; i < s1e; i += GN_T * 8) {
      float v[8], d[8];
      load8<T>(xr + i, v);
      load8<T>(gr + i, d);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xh = (v[j] - mu) * rs;
        const float z = (xh * ga + be) * s1 + sf;
        const float dz = dz_of(d[j], z, silu);
        v[j] = rs * (k * dz - a1 - xh * a2);
      }
      store8<T>(dr + i, v);
    }
  } else {
    for (long i = s0 + threadIdx.x; i < s1e; i += GN_T) {
      const float xh = (Elt<T>::to_f(xr[i]) - mu) * rs;
      const float z = (xh * ga + be) * s1 + sf;
      const float dz = dz_of(Elt<T>::to_f(gr[i]), z, silu);
      dr[i] = Elt<T>::from_f(rs * (k * dz - a1 - xh * a2));
    }
  }
}

}  // namespace

// segments per row: enough (rows*nseg >= ~2048 WGs) without segments < 2048 elems
extern "C" int fx_gn_nseg(long rows, long hw) {
  long nseg = 1;
  while (rows * nseg < 2048 && hw / (nseg * 2) >= 2048) nseg *= 2;
  return (int)nseg;
}

static inline long seg_len(long hw, int nseg) {
  long s = (hw + nseg - 1) / nseg;
  return (s + 7) / 8 * 8;  // keep segment starts 8-aligned for the vector path
}

#define GN_DISPATCH(KERNEL, dtype, vec, grid, st, ...)                                   \
  do {                                                                                   \
    if (dtype == 0) {                                                                    \
      if (vec) KERNEL<bf16, true><<<grid, GN_T, 0, st>>>(__VA_ARGS__);                   \
      else KERNEL<bf16, false><<<grid, GN_T, 0, st>>>(__VA_ARGS__);                      \
    } else {                                                                             \
      if (vec) KERNEL<f16, true><<<grid, GN_T, 0, st>>>(__VA_ARGS__);                    \
      else KERNEL<f16, false><<<grid, GN_T, 0, st>>>(__VA_ARGS__);                       \
    }                                                                                    \
  } while (0)

// part: fp64 [B*C, nseg, 2] scratch.  mean/rstd: fp32 [B*G] outputs.
extern "C" int fx_gn_fwd(int dtype, const void* x, const float* gamma, const float* beta,
                         const float* scale, const float* shift, void* y, double* part,
                         float* mean, float* rstd, int B, int C, int G, long hw, int nseg,
                         float eps, int silu, hipStream_t st) {
  if (C % G != 0 || nseg < 1) return -1;
  const long rows = (long)B * C;
  const long sl = seg_len(hw, nseg);
  const bool vec = (hw % 8) == 0;
  dim3 grid((unsigned)rows, (unsigned)nseg);
  GN_DISPATCH(gn_row_stats, dtype, vec, grid, st, (const uint16_t*)x, part, hw, nseg, sl);
  GN_DISPATCH(gn_apply, dtype, vec, grid, st, (const uint16_t*)x, part, gamma, beta, scale,
              shift, (uint16_t*)y, mean, rstd, C, G, hw, nseg, sl, eps, silu);
  return 0;
}

// part: fp32 [B*C, nseg, 2] (A, Bz) partial sums
extern "C" int fx_gn_bwd_reduce(int dtype, const void* x, const void* dy, const float* mean,
                                const float* rstd, const float* gamma, const float* beta,
                                const float* scale, const float* shift, float* part, int B, int C,
                                int G, long hw, int nseg, int silu, hipStream_t st) {
  const long rows = (long)B * C;
  const long sl = seg_len(hw, nseg);
  const bool vec = (hw % 8) == 0;
  dim3 grid((unsigned)rows, (unsigned)nseg);
  GN_DISPATCH(gn_bwd_reduce, dtype, vec, grid, st, (const uint16_t*)x, (const uint16_t*)dy, mean,
              rstd, gamma, beta, scale, shift, part, C, G, hw, nseg, sl, silu);
  return 0;
}

extern "C" int fx_gn_bwd_apply(int dtype, const void* x, const void* dy, const float* mean,
                               const float* rstd, const float* gamma, const float* beta,
                               const float* scale, const float* shift, const float* g1,
                               const float* g2, void* dx, int B, int C, int G, long hw, int nseg,
                               int silu, hipStream_t st) {
  const long rows = (long)B * C;
  const long sl = seg_len(hw, nseg);
  const bool vec = (hw % 8) == 0;
  dim3 grid((unsigned)rows, (unsigned)nseg);
  GN_DISPATCH(gn_bwd_apply, dtype, vec, grid, st, (const uint16_t*)x, (const uint16_t*)dy, mean,
              rstd, gamma, beta, scale, shift, g1, g2, (uint16_t*)dx, C, G, hw, sl, silu);
  return 0;
}
