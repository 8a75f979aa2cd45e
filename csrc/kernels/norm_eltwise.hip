// LayerNorm (+ fused residual/bias/dropout add), bias+GeLU, bias+dropout+add,
// and the column-tile reduction kernels that produce dgamma/dbeta/dbias.
//
// Parity: reference K07 (nn.LayerNorm eps 1e-5/1e-6/1e-12), K08 (gelu tanh /
// erf), K09 (residual dropout + add under upscale_in_train) -- SURVEY.md §2.10.
//
// MI355X design:
//  * row kernels: one wave64 per row, 16-byte vector loads (8 x 16-bit) with
//    lane-interleaved vectors so a wave instruction covers 1 KiB contiguous;
//    the row is cached in VGPRs between the statistics pass and the
//    normalisation pass (VPT template = vectors per lane);
//  * column reductions (dgamma, dbeta, dbias) use a 128-column x 16-row
//    tiling (256-byte row segments) with per-split fp32 partials and a tiny
//    finalize kernel -- no float atomics, bitwise reproducible.
#include "fx_common.h"

namespace {

struct DropCfg {
  uint32_t klo, khi, thr;  // drop when rand16 < thr
  float scale;             // 1/(1-p)
  int enabled;
  const uint64_t* salt;    // graph mode: per-replay device salt mixed into the key
};

// Graph mode (fx_set_dropout_salt): the key baked into a captured launch is
// re-keyed on the device by the step salt, so every replay draws new masks
// while forward, backward and recompute of one step agree.
__device__ __forceinline__ DropCfg resolve_drop(DropCfg d) {
  if (d.enabled && d.salt != nullptr) {
    const uint64_t k = salt_key(((uint64_t)d.khi << 32) | d.klo, *d.salt);
    d.klo = (uint32_t)k;
    d.khi = (uint32_t)(k >> 32);
  }
  return d;
}

__device__ __forceinline__ float drop_apply(float v, uint64_t idx, const DropCfg& d) {
  if (!d.enabled) return v;
  uint32_t h = elem_rand_pair(idx, d.klo, d.khi);
  uint32_t r = (idx & 1) ? (h >> 16) : (h & 0xffffu);
  return r >= d.thr ? v * d.scale : 0.f;
}

// The 8 consecutive elements idx0 .. idx0 + 7 of one 16-byte vector (idx0 a
// multiple of 8 at every call site: row * h + 8-aligned column): one hash per
// element PAIR, each pair's low / high halves for its even / odd element --
// the same masks as drop_apply per element, with half the hashing VALU.
__device__ __forceinline__ void drop_apply8(float* v, uint64_t idx0, const DropCfg& d) {
  if (!d.enabled) return;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t h = elem_rand_pair(idx0 + 2 * q, d.klo, d.khi);
    v[2 * q] = (h & 0xffffu) >= d.thr ? v[2 * q] * d.scale : 0.f;
    v[2 * q + 1] = (h >> 16) >= d.thr ? v[2 * q + 1] * d.scale : 0.f;
  }
}

// ---------------------------------------------------------------------------
// Fused forward:  s = residual + dropout(x + bias);  y = LN(s) * g + b
// Any of residual/bias may be null; dropout optional.  If s_out is null the
// sum is not stored (plain LN when residual & bias are null and no dropout).
// ---------------------------------------------------------------------------
// MASK: h is not a multiple of 512 (ViT-g 1408, ViT-B 768): the last vector
// of some lanes lies past the row end and is neither loaded nor counted.
template <typename T, int VPT, bool MASK = false>
__global__ __launch_bounds__(256) void add_ln_fwd_kernel(
    const uint16_t* __restrict__ x, const uint16_t* __restrict__ bias,
    const uint16_t* __restrict__ residual, const uint16_t* __restrict__ gamma,
    const uint16_t* __restrict__ beta, uint16_t* __restrict__ s_out,
    uint16_t* __restrict__ y, float* __restrict__ mean_out, float* __restrict__ rstd_out,
    int rows, int h, float eps, DropCfg drop_) {
  const DropCfg drop = resolve_drop(drop_);
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const size_t base = (size_t)row * h;
  // Every global load of the row is issued before the first use, each
  // optional operand under ONE wave-uniform branch around its whole batch: a
  // per-vector `if (ptr)` around the loads made hipcc wait for each load
  // before issuing the next (40 loads, 36 waits at h 4096; 3.5 TB/s).
  uint4 xr[VPT], rr[VPT], br[VPT];
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = (i * 64 + lane) * 8;
    xr[i] = rr[i] = br[i] = make_uint4(0, 0, 0, 0);
    if (!MASK || c < h) xr[i] = *reinterpret_cast<const uint4*>(x + base + c);
  }
  if (residual) {
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int c = (i * 64 + lane) * 8;
      if (!MASK || c < h) rr[i] = *reinterpret_cast<const uint4*>(residual + base + c);
    }
  }
  if (bias) {
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int c = (i * 64 + lane) * 8;
      if (!MASK || c < h) br[i] = *reinterpret_cast<const uint4*>(bias + c);
    }
  }
  float v[VPT][8];
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = (i * 64 + lane) * 8;
    if (MASK && c >= h) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = 0.f;
      continue;
    }
    unpack8<T>(xr[i], v[i]);
    if (bias) {
      float b[8];
      unpack8<T>(br[i], b);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] += b[j];
    }
    if (drop.enabled) {
      drop_apply8(v[i], base + c, drop);
    }
    if (residual) {
      float r[8];
      unpack8<T>(rr[i], r);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] += r[j];
    }
    if (s_out) {
      store8<T>(s_out + base + c, v[i]);
      // LN sees the value as stored (rounded) so fwd/bwd agree exactly; the
      // rounding happens in registers (no dependent reload of the store).
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = round_to<T>(v[i][j]);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) sum += v[i][j];
  }
  const float mean = wave_sum(sum) / h;
  float var = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    if (MASK && (i * 64 + lane) * 8 >= h) continue;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float d = v[i][j] - mean;
      var += d * d;
    }
  }
  const float rstd = rsqrtf(wave_sum(var) / h + eps);
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = (i * 64 + lane) * 8;
    if (MASK && c >= h) continue;
    float g[8], b[8], o[8];
    load8<T>(gamma + c, g);
    load8<T>(beta + c, b);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (v[i][j] - mean) * rstd * g[j] + b[j];
    store8<T>(y + base + c, o);
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// Generic-width fallback (h % 8 == 0): re-reads the row from cache.
template <typename T>
__global__ __launch_bounds__(256) void add_ln_fwd_generic(
    const uint16_t* __restrict__ x, const uint16_t* __restrict__ bias,
    const uint16_t* __restrict__ residual, const uint16_t* __restrict__ gamma,
    const uint16_t* __restrict__ beta, uint16_t* __restrict__ s_out,
    uint16_t* __restrict__ y, float* __restrict__ mean_out, float* __restrict__ rstd_out,
    int rows, int h, float eps, DropCfg drop_) {
  const DropCfg drop = resolve_drop(drop_);
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const size_t base = (size_t)row * h;
  const int nv = h / 8;
  auto value = [&](int c, float* v) {
    load8<T>(x + base + c, v);
    if (bias) {
      float b[8];
      load8<T>(bias + c, b);
      for (int j = 0; j < 8; ++j) v[j] += b[j];
    }
    if (drop.enabled)
      drop_apply8(v, base + c, drop);
    if (residual) {
      float r[8];
      load8<T>(residual + base + c, r);
      for (int j = 0; j < 8; ++j) v[j] += r[j];
    }
  };
  float sum = 0.f;
  for (int vi = lane; vi < nv; vi += 64) {
    float v[8];
    value(vi * 8, v);
    if (s_out) {
      store8<T>(s_out + base + vi * 8, v);
      for (int j = 0; j < 8; ++j) v[j] = round_to<T>(v[j]);
    }
    for (int j = 0; j < 8; ++j) sum += v[j];
  }
  const float mean = wave_sum(sum) / h;
  float var = 0.f;
  for (int vi = lane; vi < nv; vi += 64) {
    float v[8];
    if (s_out) load8<T>(s_out + base + vi * 8, v); else value(vi * 8, v);
    for (int j = 0; j < 8; ++j) { float d = v[j] - mean; var += d * d; }
  }
  const float rstd = rsqrtf(wave_sum(var) / h + eps);
  for (int vi = lane; vi < nv; vi += 64) {
    float v[8], g[8], b[8], o[8];
    if (s_out) load8<T>(s_out + base + vi * 8, v); else value(vi * 8, v);
    load8<T>(gamma + vi * 8, g);
    load8<T>(beta + vi * 8, b);
    for (int j = 0; j < 8; ++j) o[j] = (v[j] - mean) * rstd * g[j] + b[j];
    store8<T>(y + base + vi * 8, o);
  }
  if (lane == 0) { mean_out[row] = mean; rstd_out[row] = rstd; }
}

// ---------------------------------------------------------------------------
// Row backward:  ds = ds_in + LN'(dy);  dx = dropout'(ds)
//   s: the LN input (as stored), dx_out may alias ds_out when no dropout.
// ---------------------------------------------------------------------------
template <typename T, int VPT, bool MASK = false>
__global__ __launch_bounds__(256) void ln_bwd_row_kernel(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ s,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
    const uint16_t* __restrict__ gamma, const uint16_t* __restrict__ ds_in,
    uint16_t* __restrict__ ds_out, uint16_t* __restrict__ dx_out, int rows, int h,
    DropCfg drop_) {
  const DropCfg drop = resolve_drop(drop_);
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const size_t base = (size_t)row * h;
  const float mean = mean_in[row], rstd = rstd_in[row];
  float xh[VPT][8], gdy[VPT][8];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = (i * 64 + lane) * 8;
    if (MASK && c >= h) {
#pragma unroll
      for (int j = 0; j < 8; ++j) xh[i][j] = gdy[i][j] = 0.f;
      continue;
    }
    float a[8], g[8], d[8];
    load8<T>(s + base + c, a);
    load8<T>(gamma + c, g);
    load8<T>(dy + base + c, d);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      xh[i][j] = (a[j] - mean) * rstd;
      gdy[i][j] = d[j] * g[j];
      s1 += gdy[i][j];
      s2 += gdy[i][j] * xh[i][j];
    }
  }
  // ds_in's loads go out before the row reductions, all under one branch (a
  // per-vector `if (ds_in)` load after them was waited on one by one)
  uint4 dr[VPT];
  if (ds_in) {
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int c = (i * 64 + lane) * 8;
      dr[i] = make_uint4(0, 0, 0, 0);
      if (!MASK || c < h) dr[i] = *reinterpret_cast<const uint4*>(ds_in + base + c);
    }
  }
  const float m1 = wave_sum(s1) / h, m2 = wave_sum(s2) / h;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = (i * 64 + lane) * 8;
    if (MASK && c >= h) continue;
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = rstd * (gdy[i][j] - m1 - xh[i][j] * m2);
    if (ds_in) {
      float r[8];
      unpack8<T>(dr[i], r);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] += r[j];
    }
    store8<T>(ds_out + base + c, o);
    if (drop.enabled) {
      drop_apply8(o, base + c, drop);
      store8<T>(dx_out + base + c, o);
    } else if (dx_out != ds_out) {
      store8<T>(dx_out + base + c, o);
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void ln_bwd_row_generic(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ s,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
    const uint16_t* __restrict__ gamma, const uint16_t* __restrict__ ds_in,
    uint16_t* __restrict__ ds_out, uint16_t* __restrict__ dx_out, int rows, int h,
    DropCfg drop_) {
  const DropCfg drop = resolve_drop(drop_);
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const size_t base = (size_t)row * h;
  const float mean = mean_in[row], rstd = rstd_in[row];
  const int nv = h / 8;
  float s1 = 0.f, s2 = 0.f;
  for (int vi = lane; vi < nv; vi += 64) {
    float a[8], g[8], d[8];
    load8<T>(s + base + vi * 8, a);
    load8<T>(gamma + vi * 8, g);
    load8<T>(dy + base + vi * 8, d);
    for (int j = 0; j < 8; ++j) {
      float xh = (a[j] - mean) * rstd, gd = d[j] * g[j];
      s1 += gd;
      s2 += gd * xh;
    }
  }
  const float m1 = wave_sum(s1) / h, m2 = wave_sum(s2) / h;
  for (int vi = lane; vi < nv; vi += 64) {
    const int c = vi * 8;
    float a[8], g[8], d[8], o[8];
    load8<T>(s + base + c, a);
    load8<T>(gamma + c, g);
    load8<T>(dy + base + c, d);
    for (int j = 0; j < 8; ++j) o[j] = rstd * (d[j] * g[j] - m1 - (a[j] - mean) * rstd * m2);
    if (ds_in) {
      float r[8];
      load8<T>(ds_in + base + c, r);
      for (int j = 0; j < 8; ++j) o[j] += r[j];
    }
    store8<T>(ds_out + base + c, o);
    if (drop.enabled) {
      drop_apply8(o, base + c, drop);
      store8<T>(dx_out + base + c, o);
    } else if (dx_out != ds_out) {
      store8<T>(dx_out + base + c, o);
    }
  }
}

// ---------------------------------------------------------------------------
// Row backward + its column sums in one pass (h <= 4096):
//   ds = ds_in + LN'(dy),  dx = dropout'(ds)          (as ln_bwd_row_kernel)
//   dgamma = sum dy * xhat,  dbeta = sum dy,  dbias = sum dx (optional: the
//   bias of the linear that feeds the fused residual add)
// instead of the row kernel + two column-tile passes that re-read dy and s
// (reference K07's LayerNorm backward + the bias gradient of K09).  A row is
// WPR waves wide (1 / 2 / 4 for h <= 1536 / 3072 / 4096: each wave owns a
// slice of the columns and the row sums meet in LDS); each row group owns a
// contiguous run of rows and keeps its columns' sums in registers.  Register
// budget (<= 3 vectors per lane, two waves per SIMD; 4 spilled): gamma stays
// packed, and xhat / dy are re-derived from the packed row in the second
// pass instead of being held as floats.
// The row groups' sums meet in LDS in a fixed order and the block writes one
// partial row per array ([3][G][h] fp32); ln_cols_finalize_kernel adds the G
// rows in a fixed order -- bitwise reproducible.
// ---------------------------------------------------------------------------
template <typename T, int VPT, int WPR, bool MASK, bool DB>
__global__ __launch_bounds__(256, 2) void ln_bwd_cols_kernel(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ s,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
    const uint16_t* __restrict__ gamma, const uint16_t* __restrict__ ds_in,
    uint16_t* __restrict__ ds_out, uint16_t* __restrict__ dx_out, int rows, int h,
    int rows_per_group, float* __restrict__ part, DropCfg drop_) {
  constexpr int NG = 4 / WPR;                 // row groups per block
  __shared__ float red[4 * 512 * VPT];        // NG groups x h columns
  __shared__ float xs[2][4][2];               // WPR > 1: the waves' row sums, by row parity
  const DropCfg drop = resolve_drop(drop_);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int grp = w / WPR, half = w % WPR;
  const int hw = h / WPR, cbase = half * hw;
  const int r0 = min(rows, (blockIdx.x * NG + grp) * rows_per_group);
  const int r1 = min(rows, r0 + rows_per_group);
  uint4 gp[VPT];
  float ag[VPT][8], ab[VPT][8], ax[DB ? VPT : 1][8];
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = (i * 64 + lane) * 8;
    gp[i] = (!MASK || c < hw) ? *reinterpret_cast<const uint4*>(gamma + cbase + c)
                              : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ag[i][j] = ab[i][j] = 0.f;
      if (DB) ax[i][j] = 0.f;
    }
  }
  for (int k = 0; k < rows_per_group; ++k) {
    const int r = r0 + k;
    const bool live = r < r1;   // WPR > 1: every wave runs every iteration (LDS barrier)
    if (WPR == 1 && !live) break;
    const size_t base = (size_t)(live ? r : 0) * h + cbase;
    uint4 ca[VPT], cd[VPT], cr[VPT];
    float mean = 0.f, rstd = 0.f, s1 = 0.f, s2 = 0.f;
    if (live) {
#pragma unroll
      for (int i = 0; i < VPT; ++i) {
        const int c = (i * 64 + lane) * 8;
        if (MASK && c >= hw) continue;
        ca[i] = *reinterpret_cast<const uint4*>(s + base + c);
        cd[i] = *reinterpret_cast<const uint4*>(dy + base + c);
      }
      // ds_in under ONE branch around its batch (a per-vector `if` around a
      // load made hipcc wait for each: profiles/r6_norm/)
      if (ds_in) {
#pragma unroll
        for (int i = 0; i < VPT; ++i) {
          const int c = (i * 64 + lane) * 8;
          if (MASK && c >= hw) continue;
          cr[i] = *reinterpret_cast<const uint4*>(ds_in + base + c);
        }
      }
      mean = mean_in[r];
      rstd = rstd_in[r];
#pragma unroll
      for (int i = 0; i < VPT; ++i) {
        const int c = (i * 64 + lane) * 8;
        if (MASK && c >= hw) continue;
        float a[8], d[8], g[8];
        unpack8<T>(ca[i], a);
        unpack8<T>(cd[i], d);
        unpack8<T>(gp[i], g);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xh = (a[j] - mean) * rstd, gd = d[j] * g[j];
          s1 += gd;
          s2 += gd * xh;
          ag[i][j] += d[j] * xh;
          ab[i][j] += d[j];
        }
      }
    }
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    if constexpr (WPR > 1) {
      if (lane == 0) {
        xs[k & 1][w][0] = s1;
        xs[k & 1][w][1] = s2;
      }
      __syncthreads();
      s1 = xs[k & 1][WPR * grp][0];
      s2 = xs[k & 1][WPR * grp][1];
#pragma unroll
      for (int q = 1; q < WPR; ++q) {
        s1 += xs[k & 1][WPR * grp + q][0];
        s2 += xs[k & 1][WPR * grp + q][1];
      }
    }
    if (!live) continue;
    const float m1 = s1 / h, m2 = s2 / h;
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int c = (i * 64 + lane) * 8;
      if (MASK && c >= hw) continue;
      float a[8], d[8], g[8], o[8];
      unpack8<T>(ca[i], a);
      unpack8<T>(cd[i], d);
      unpack8<T>(gp[i], g);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = rstd * (d[j] * g[j] - m1 - (a[j] - mean) * rstd * m2);
      if (ds_in) {
        float rr[8];
        unpack8<T>(cr[i], rr);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] += rr[j];
      }
      store8<T>(ds_out + base + c, o);
      if (drop.enabled) {
        drop_apply8(o, base + c, drop);
        store8<T>(dx_out + base + c, o);
      } else if (dx_out != ds_out) {
        store8<T>(dx_out + base + c, o);
      }
      if (DB) {
#pragma unroll
        for (int j = 0; j < 8; ++j) ax[i][j] += round_to<T>(o[j]);
      }
    }
  }
  // block partials: the row groups' column sums, added in group order
#pragma unroll
  for (int arr = 0; arr < (DB ? 3 : 2); ++arr) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int c = (i * 64 + lane) * 8;
      if (MASK && c >= hw) continue;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        red[grp * h + cbase + c + j] = arr == 0 ? ag[i][j] : arr == 1 ? ab[i][j] : ax[DB ? i : 0][j];
    }
    __syncthreads();
    float* out = part + ((size_t)arr * gridDim.x + blockIdx.x) * h;
    for (int c = threadIdx.x; c < h; c += 256) {
      float v = red[c];
#pragma unroll
      for (int q = 1; q < NG; ++q) v += red[q * h + c];
      out[c] = v;
    }
  }
}

// Sum the G partial rows of each array ([narr][G][h]) per column in a fixed
// order: 32 lanes x 4 columns per partial row, 8 row phases, 16 loads in
// flight per thread; the 8 phases meet in LDS.  grid = (h / 128, narr).
struct LnColsOut {
  float* f32[3];
  uint16_t* t16[3];
  int acc[3];
};
template <typename T>
__global__ __launch_bounds__(256) void ln_cols_finalize_kernel(const float* __restrict__ part,
                                                               int G, int h, LnColsOut f) {
  __shared__ float tr[8][132];
  const int arr = blockIdx.y;
  const float* p = part + (size_t)arr * G * h;
  const int q = threadIdx.x & 31, sr = threadIdx.x >> 5;
  const int c0 = blockIdx.x * 128 + q * 4;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  if (c0 < h) {
    for (int k0 = sr; k0 < G; k0 += 128) {
      floatx4 v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int k = k0 + 8 * u;
        v[u] = k < G ? *reinterpret_cast<const floatx4*>(p + (size_t)k * h + c0)
                     : floatx4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) acc += v[u];
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) tr[sr][q * 4 + j] = acc[j];
  __syncthreads();
  const int c = threadIdx.x, gc = blockIdx.x * 128 + c;
  if (c >= 128 || gc >= h) return;
  float sum = 0.f;
#pragma unroll
  for (int t = 0; t < 8; ++t) sum += tr[t][c];
  if (f.f32[arr]) f.f32[arr][gc] = f.acc[arr] ? f.f32[arr][gc] + sum : sum;
  if (f.t16[arr]) f.t16[arr][gc] = Elt<T>::from_f(sum);
}

// ---------------------------------------------------------------------------
// Fused finalize of the column-sum partials: the LAST workgroup of each
// 128-column tile to finish (ticket per tile) sums the tile's `splits`
// partial rows in a fixed order (deterministic whoever arrives last) and
// writes the outputs -- instead of a separate finalize launch per reduction
// (~5-6 us each, 190-260 per training step).  Hand-off (cdna_hip_programming.md
// §6 G16, sc1 form): the partials are stored write-through (sc1), every
// storing wave drains them, workgroup barrier, one lane draws the ticket with
// a relaxed agent-scope add; the last one reads the partials with sc1 loads
// (16-byte buffer loads, aux = sc1).
// No agent release fence: that is a write-back of the whole XCD L2, and these
// kernels have just dirtied it with their dx output (measured: the
// fence form made the four column kernels 2.5-4x slower than kernel + separate
// finalize).  The last arriver resets the ticket (tickets are per stream,
// zeroed once at allocation).  Each tile's ticket has a 128-byte line of its
// own: device-scope atomics on one line serialise (~13 ns each), and with the
// tickets packed the ~1024 arrivals of a short launch queued for ~13 us.
// ---------------------------------------------------------------------------
typedef __attribute__((address_space(1))) float gf32;
typedef __attribute__((address_space(1))) int gi32;

__device__ __forceinline__ void st_part(float* p, float v) {   // sc1 store
  __hip_atomic_store((gf32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct ColFin {
  int* cnt;               // [col tiles x 32] tickets, one per 128-B line; nullptr = caller finalizes
  float* f32[2];          // fp32 outputs (e.g. main_grad) for partial 0 / 1
  uint16_t* t16[2];       // 16-bit outputs
  int acc[2];             // accumulate into f32 (1) or overwrite (0)
};

template <typename T>
__device__ __forceinline__ void colsum_tail(const float* __restrict__ p0,
                                            const float* __restrict__ p1, int cols, int np,
                                            const ColFin& f) {
  __shared__ int last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains
  __syncthreads();
  if (threadIdx.x == 0) {
    const int t = __hip_atomic_fetch_add((gi32*)(f.cnt + 32 * blockIdx.x), 1, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    last = t == (int)gridDim.y - 1;
    if (last)
      __hip_atomic_store((gi32*)(f.cnt + 32 * blockIdx.x), 0, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // keeps the loads below the ticket
  // The reducer reads splits x 128 fp32 per array.  sc1-stored partials are not
  // in any L2, so every read pays the fabric latency: issue them ALL at once
  // -- 16-byte sc1 buffer loads, 32 lanes per split row (4 columns each), 8
  // split rows per pass, 16 passes in flight per thread (128 split rows per
  // round trip; out-of-range rows read 0 through the buffer range check) --
  // then combine the 8 row phases through LDS in a fixed order.
  __shared__ float tr[8][132];
  const int q = threadIdx.x & 31, sr = threadIdx.x >> 5;
  const int c0 = blockIdx.x * 128 + q * 4;
  const int splits = gridDim.y;
  for (int which = 0; which < np; ++which) {
    const float* p = which ? p1 : p0;
    floatx4 s = {0.f, 0.f, 0.f, 0.f};
    if (c0 < cols) {
      const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), 0,
                                                        splits * cols * 4, 0x00020000);
      for (int k0 = sr; k0 < splits; k0 += 128) {
        floatx4 v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int k = k0 + 8 * u;
          const uint32_t off = k < splits ? (uint32_t)(k * cols + c0) * 4u : 0x80000000u;
          v[u] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16));
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) s += v[u];
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) tr[sr][q * 4 + j] = s[j];
    __syncthreads();
    const int c = threadIdx.x, gc = blockIdx.x * 128 + c;
    if (c < 128 && gc < cols) {
      float sum = 0.f;
#pragma unroll
      for (int t = 0; t < 8; ++t) sum += tr[t][c];
      if (f.f32[which]) f.f32[which][gc] = f.acc[which] ? f.f32[which][gc] + sum : sum;
      if (f.t16[which]) f.t16[which][gc] = Elt<T>::from_f(sum);
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Column-tile partial sums.  Block = 256 threads = 16 column groups (8 cols
// each -> 128 columns) x 16 row lanes.  Grid = (col tiles, splits).
// MODE 0: LN  -> p0 += dy*xhat, p1 += dy            (a = dy, b = s)
// MODE 1: sum -> p0 += a                             (plain column sum)
// ---------------------------------------------------------------------------
template <typename T, int MODE>
__global__ __launch_bounds__(256) void coltile_partial_kernel(
    const uint16_t* __restrict__ a, const uint16_t* __restrict__ b,
    const float* __restrict__ mean, const float* __restrict__ rstd,
    float* __restrict__ p0, float* __restrict__ p1, int rows, int cols, int rows_per_split,
    ColFin fin) {
  __shared__ float red[2][16][129];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int col = blockIdx.x * 128 + tx * 8;
  const int r0 = blockIdx.y * rows_per_split;
  const int r1 = min(rows, r0 + rows_per_split);
  float acc0[8], acc1[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc0[j] = acc1[j] = 0.f;
  if (col < cols) {
    // 4 rows' loads in flight per thread (the loop-carried adds otherwise
    // leave one row's latency exposed per iteration); added in row order
    int r = r0 + ty;
    for (; r + 48 < r1; r += 64) {
      float va[4][8], vb[MODE == 0 ? 4 : 1][8], m[4], rs[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const size_t off = (size_t)(r + 16 * q) * cols + col;
        load8<T>(a + off, va[q]);
        if (MODE == 0) {
          load8<T>(b + off, vb[q]);
          m[q] = mean[r + 16 * q];
          rs[q] = rstd[r + 16 * q];
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (MODE == 0) {
            acc0[j] += va[q][j] * (vb[MODE == 0 ? q : 0][j] - m[q]) * rs[q];
            acc1[j] += va[q][j];
          } else {
            acc0[j] += va[q][j];
          }
        }
      }
    }
    for (; r < r1; r += 16) {
      const size_t off = (size_t)r * cols + col;
      float va[8];
      load8<T>(a + off, va);
      if (MODE == 0) {
        float vb[8];
        load8<T>(b + off, vb);
        const float m = mean[r], rs = rstd[r];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          acc0[j] += va[j] * (vb[j] - m) * rs;
          acc1[j] += va[j];
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) acc0[j] += va[j];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[0][ty][tx * 8 + j] = acc0[j];
    red[1][ty][tx * 8 + j] = acc1[j];
  }
  __syncthreads();
  // 256 threads reduce 128 columns x 2 arrays over 16 rows
  const int which = threadIdx.x >> 7, c = threadIdx.x & 127;
  if (MODE == 0 || which == 0) {
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < 16; ++t) s += red[which][t][c];
    const int gc = blockIdx.x * 128 + c;
    if (gc < cols) st_part((which == 0 ? p0 : p1) + (size_t)blockIdx.y * cols + gc, s);
  }
  if (fin.cnt) colsum_tail<T>(p0, p1, cols, MODE == 0 ? 2 : 1, fin);
}

// Sum partials over splits; write fp32 and/or 16-bit outputs.
template <typename T>
__global__ void coltile_finalize_kernel(const float* __restrict__ p, int splits, int cols,
                                        float* __restrict__ out_f32, uint16_t* __restrict__ out_t,
                                        int accumulate) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= cols) return;
  // 8 independent partial loads in flight per thread: the grid is only
  // cols/256 blocks, so a serial dependent loop over the splits would expose
  // one L2 round trip per split (measured ~15 us per call at 32 splits)
  float a[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = 0.f;
  int k = 0;
  for (; k + 8 <= splits; k += 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] += p[(size_t)(k + j) * cols + c];
  }
  for (int j = 0; k + j < splits; ++j) a[j] += p[(size_t)(k + j) * cols + c];
  const float s = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  if (out_f32) out_f32[c] = accumulate ? out_f32[c] + s : s;
  if (out_t) out_t[c] = Elt<T>::from_f(s);
}

// ---------------------------------------------------------------------------
// bias + GeLU  (fwd stores y; bwd emits dx and column partials of dx)
// ---------------------------------------------------------------------------
template <typename T, bool ERF>
__global__ __launch_bounds__(256) void bias_gelu_fwd_kernel(
    const uint16_t* __restrict__ x, const uint16_t* __restrict__ bias, uint16_t* __restrict__ y,
    long n8, int cols) {
  for (long v = blockIdx.x * (long)blockDim.x + threadIdx.x; v < n8; v += (long)gridDim.x * blockDim.x) {
    const long off = v * 8;
    const int c = (int)(off % cols);
    float a[8], b[8];
    load8<T>(x + off, a);
    if (bias) load8<T>(bias + c, b);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float t = a[j] + (bias ? b[j] : 0.f);
      a[j] = ERF ? gelu_erf(t) : gelu_tanh(t);
    }
    store8<T>(y + off, a);
  }
}

template <typename T, bool ERF>
__global__ __launch_bounds__(256) void bias_gelu_bwd_kernel(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x,
    const uint16_t* __restrict__ bias, uint16_t* __restrict__ dx, float* __restrict__ part,
    int rows, int cols, int rows_per_split, ColFin fin) {
  __shared__ float red[16][129];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int col = blockIdx.x * 128 + tx * 8;
  const int r0 = blockIdx.y * rows_per_split;
  const int r1 = min(rows, r0 + rows_per_split);
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  if (col < cols) {
    float b[8];
    if (bias) load8<T>(bias + col, b);
    else {
#pragma unroll
      for (int j = 0; j < 8; ++j) b[j] = 0.f;
    }
    for (int r = r0 + ty; r < r1; r += 16) {
      const size_t off = (size_t)r * cols + col;
      float g[8], a[8];
      load8<T>(dy + off, g);
      load8<T>(x + off, a);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float t = a[j] + b[j];
        g[j] *= ERF ? gelu_erf_grad(t) : gelu_tanh_grad(t);
      }
      store8<T>(dx + off, g);
      // accumulate the rounded value so dbias == colsum(dx) exactly
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += round_to<T>(g[j]);
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[ty][tx * 8 + j] = acc[j];
  __syncthreads();
  if (threadIdx.x < 128) {
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < 16; ++t) s += red[t][threadIdx.x];
    const int gc = blockIdx.x * 128 + threadIdx.x;
    if (part && gc < cols) st_part(part + (size_t)blockIdx.y * cols + gc, s);
  }
  if (fin.cnt) colsum_tail<T>(part, nullptr, cols, 1, fin);
}

// ---------------------------------------------------------------------------
// out = residual + dropout(x + bias)      and its backward
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void bias_dropout_add_fwd_kernel(
    const uint16_t* __restrict__ x, const uint16_t* __restrict__ bias,
    const uint16_t* __restrict__ residual, uint16_t* __restrict__ out, long n8, int cols,
    DropCfg drop_) {
  const DropCfg drop = resolve_drop(drop_);
  for (long v = blockIdx.x * (long)blockDim.x + threadIdx.x; v < n8; v += (long)gridDim.x * blockDim.x) {
    const long off = v * 8;
    const int c = (int)(off % cols);
    float a[8];
    load8<T>(x + off, a);
    if (bias) {
      float b[8];
      load8<T>(bias + c, b);
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += b[j];
    }
    drop_apply8(a, (uint64_t)off, drop);
    if (residual) {
      float r[8];
      load8<T>(residual + off, r);
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += r[j];
    }
    store8<T>(out + off, a);
  }
}

// dx = dropout'(dout); column partials of dx (for dbias) if part != null.
template <typename T>
__global__ __launch_bounds__(256) void dropout_bwd_colsum_kernel(
    const uint16_t* __restrict__ dout, uint16_t* __restrict__ dx, float* __restrict__ part,
    int rows, int cols, int rows_per_split, DropCfg drop_, ColFin fin) {
  const DropCfg drop = resolve_drop(drop_);
  __shared__ float red[16][129];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int col = blockIdx.x * 128 + tx * 8;
  const int r0 = blockIdx.y * rows_per_split;
  const int r1 = min(rows, r0 + rows_per_split);
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  if (col < cols) {
    int r = r0 + ty;
    for (; r + 48 < r1; r += 64) {  // 4 rows' loads in flight, added in row order
      float g[4][8];
#pragma unroll
      for (int q = 0; q < 4; ++q) load8<T>(dout + (size_t)(r + 16 * q) * cols + col, g[q]);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const size_t off = (size_t)(r + 16 * q) * cols + col;
        drop_apply8(g[q], off, drop);
        if (dx) {
          store8<T>(dx + off, g[q]);
#pragma unroll
          for (int j = 0; j < 8; ++j) g[q][j] = round_to<T>(g[q][j]);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += g[q][j];
      }
    }
    for (; r < r1; r += 16) {
      const size_t off = (size_t)r * cols + col;
      float g[8];
      load8<T>(dout + off, g);
      drop_apply8(g, off, drop);
      if (dx) {
        store8<T>(dx + off, g);
#pragma unroll
        for (int j = 0; j < 8; ++j) g[j] = round_to<T>(g[j]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += g[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[ty][tx * 8 + j] = acc[j];
  __syncthreads();
  if (threadIdx.x < 128) {
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < 16; ++t) s += red[t][threadIdx.x];
    const int gc = blockIdx.x * 128 + threadIdx.x;
    if (part && gc < cols) st_part(part + (size_t)blockIdx.y * cols + gc, s);
  }
  if (fin.cnt) colsum_tail<T>(part, nullptr, cols, 1, fin);
}

// Plain dropout (embedding / generic): y = dropout(x)
template <typename T>
__global__ __launch_bounds__(256) void dropout_fwd_kernel(const uint16_t* __restrict__ x,
                                                          uint16_t* __restrict__ y, long n8,
                                                          DropCfg drop_) {
  const DropCfg drop = resolve_drop(drop_);
  for (long v = blockIdx.x * (long)blockDim.x + threadIdx.x; v < n8; v += (long)gridDim.x * blockDim.x) {
    const long off = v * 8;
    float a[8];
    load8<T>(x + off, a);
    drop_apply8(a, (uint64_t)off, drop);
    store8<T>(y + off, a);
  }
}

DropCfg make_drop(float p, uint64_t key) {
  DropCfg d;
  d.enabled = p > 0.f ? 1 : 0;
  d.klo = (uint32_t)(key & 0xffffffffu);
  d.khi = (uint32_t)(key >> 32);
  d.thr = (uint32_t)(p * 65536.0f + 0.5f);
  d.scale = p < 1.f ? 1.f / (1.f - p) : 0.f;
  d.salt = g_fx_dropout_salt;
  return d;
}

inline int grid_for(long n8) {
  long g = (n8 + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

inline int splits_for(int rows, int cols) {
  // ~1024 workgroups per column reduction (FLEETX_COLSUM_BLOCKS overrides)
  static const int blocks = [] {
    const char* e = getenv("FLEETX_COLSUM_BLOCKS");
    const int v = e ? atoi(e) : 0;
    return v > 0 ? v : 1024;
  }();
  int tiles = (cols + 127) / 128;
  int s = blocks / (tiles > 0 ? tiles : 1);
  if (s < 1) s = 1;
  int max_s = (rows + 15) / 16;
  if (s > max_s) s = max_s;
  if (s > 512) s = 512;
  return s;
}

}  // namespace

// ============================================================================
// host launchers (extern "C" ABI, called from the pybind module)
// dtype: 0 = bf16, 1 = fp16
// ============================================================================
#define FX_DISPATCH_T(dtype, ...)        \
  if (dtype == 0) {                      \
    using T = bf16;                      \
    __VA_ARGS__;                         \
  } else {                               \
    using T = f16;                       \
    __VA_ARGS__;                         \
  }

// Fused finalize arguments of the column-sum producers (cnt == nullptr: the
// caller runs coltile_finalize itself).
static ColFin make_fin(int* cnt, float* f0, void* t0, int acc0, float* f1, void* t1, int acc1) {
  ColFin f;
  f.cnt = cnt;
  f.f32[0] = f0; f.f32[1] = f1;
  f.t16[0] = (uint16_t*)t0; f.t16[1] = (uint16_t*)t1;
  f.acc[0] = acc0; f.acc[1] = acc1;
  return f;
}

extern "C" int fx_coltile_splits(int rows, int cols) { return splits_for(rows, cols); }

extern "C" void fx_add_ln_fwd(int dtype, const void* x, const void* bias, const void* residual,
                              const void* gamma, const void* beta, void* s_out, void* y,
                              float* mean, float* rstd, int rows, int h, float eps, float p,
                              uint64_t key, hipStream_t st) {
  DropCfg d = make_drop(p, key);
  dim3 grid((rows + 3) / 4), block(256);
  auto X = (const uint16_t*)x;
  auto B = (const uint16_t*)bias;
  auto R = (const uint16_t*)residual;
  auto G = (const uint16_t*)gamma;
  auto Be = (const uint16_t*)beta;
  auto S = (uint16_t*)s_out;
  auto Y = (uint16_t*)y;
#define LN_CASE(V)                                                                          \
  case V:                                                                                   \
    FX_DISPATCH_T(dtype, add_ln_fwd_kernel<T, V><<<grid, block, 0, st>>>(                   \
                             X, B, R, G, Be, S, Y, mean, rstd, rows, h, eps, d));           \
    break;
  if (h % 512 == 0 && h / 512 <= 16) {
    switch (h / 512) {
      LN_CASE(1) LN_CASE(2) LN_CASE(3) LN_CASE(4) LN_CASE(5) LN_CASE(6) LN_CASE(7) LN_CASE(8)
      LN_CASE(10) LN_CASE(12) LN_CASE(16)
      default:
        FX_DISPATCH_T(dtype, add_ln_fwd_generic<T><<<grid, block, 0, st>>>(
                                 X, B, R, G, Be, S, Y, mean, rstd, rows, h, eps, d));
    }
  } else if (h % 8 == 0 && h < 8 * 512) {
    // row held in registers, last vector masked (ViT-g 1408: 2.75 vectors per lane)
#define LNM_CASE(V)                                                                          \
  case V:                                                                                    \
    FX_DISPATCH_T(dtype, add_ln_fwd_kernel<T, V, true><<<grid, block, 0, st>>>(              \
                             X, B, R, G, Be, S, Y, mean, rstd, rows, h, eps, d));            \
    break;
    switch ((h + 511) / 512) {
      LNM_CASE(1) LNM_CASE(2) LNM_CASE(3) LNM_CASE(4) LNM_CASE(5) LNM_CASE(6) LNM_CASE(7)
      LNM_CASE(8)
    }
#undef LNM_CASE
  } else {
    FX_DISPATCH_T(dtype, add_ln_fwd_generic<T><<<grid, block, 0, st>>>(
                             X, B, R, G, Be, S, Y, mean, rstd, rows, h, eps, d));
  }
#undef LN_CASE
}

extern "C" void fx_ln_bwd_row(int dtype, const void* dy, const void* s, const float* mean,
                              const float* rstd, const void* gamma, const void* ds_in,
                              void* ds_out, void* dx_out, int rows, int h, float p, uint64_t key,
                              hipStream_t st) {
  DropCfg d = make_drop(p, key);
  dim3 grid((rows + 3) / 4), block(256);
  auto DY = (const uint16_t*)dy;
  auto S = (const uint16_t*)s;
  auto G = (const uint16_t*)gamma;
  auto DI = (const uint16_t*)ds_in;
  auto DS = (uint16_t*)ds_out;
  auto DX = (uint16_t*)dx_out;
#define LNB_CASE(V)                                                                       \
  case V:                                                                                 \
    FX_DISPATCH_T(dtype, ln_bwd_row_kernel<T, V><<<grid, block, 0, st>>>(                 \
                             DY, S, mean, rstd, G, DI, DS, DX, rows, h, d));              \
    break;
  if (h % 512 == 0 && h / 512 <= 8) {
    switch (h / 512) {
      LNB_CASE(1) LNB_CASE(2) LNB_CASE(3) LNB_CASE(4) LNB_CASE(5) LNB_CASE(6) LNB_CASE(7)
      LNB_CASE(8)
      default:
        FX_DISPATCH_T(dtype, ln_bwd_row_generic<T><<<grid, block, 0, st>>>(
                                 DY, S, mean, rstd, G, DI, DS, DX, rows, h, d));
    }
  } else if (h % 8 == 0 && h < 8 * 512) {
#define LNBM_CASE(V)                                                                      \
  case V:                                                                                 \
    FX_DISPATCH_T(dtype, ln_bwd_row_kernel<T, V, true><<<grid, block, 0, st>>>(           \
                             DY, S, mean, rstd, G, DI, DS, DX, rows, h, d));              \
    break;
    switch ((h + 511) / 512) {
      LNBM_CASE(1) LNBM_CASE(2) LNBM_CASE(3) LNBM_CASE(4) LNBM_CASE(5) LNBM_CASE(6)
      LNBM_CASE(7) LNBM_CASE(8)
    }
#undef LNBM_CASE
  } else {
    FX_DISPATCH_T(dtype, ln_bwd_row_generic<T><<<grid, block, 0, st>>>(
                             DY, S, mean, rstd, G, DI, DS, DX, rows, h, d));
  }
#undef LNB_CASE
}

// Fused LayerNorm backward (h <= 4096): waves per row, rows per row group
// and partial rows G (the caller sizes part = [3][G][h]).
static int ln_cols_wpr(int h) { return h <= 1536 ? 1 : h <= 3072 ? 2 : 4; }
static int ln_cols_rows_per_group(int rows, int h) {
  const int ng = 4 / ln_cols_wpr(h);
  int rpg = (rows + 512 * ng - 1) / (512 * ng);
  return rpg < 2 ? 2 : rpg;
}
// max_h: the caller's width limit (fleetx_amd/ops/norm.py, FLEETX_LN_BWD_FUSED:
// 1536 = one wave per row, the default; 4096 = also 2 / 4 waves per row).
// Measured (profiles/r3_colsum/wide_rows.txt): at h 4096 the per-row LDS
// barrier of 4 waves makes the pass 76-109 us against 60 us for the row
// kernel, more than the column passes it saves (7.75 vs 7.38 ms per 6.7B
// step); h 2048 is neutral.
extern "C" int fx_ln_bwd_cols_blocks(int rows, int h, int max_h) {
  if (rows <= 0 || h > (max_h < 4096 ? max_h : 4096) || h % (8 * ln_cols_wpr(h))) return 0;
  const int ng = 4 / ln_cols_wpr(h), rpg = ln_cols_rows_per_group(rows, h);
  return (rows + ng * rpg - 1) / (ng * rpg);
}

// Returns 0 when launched, -1 when the shape is not covered.
extern "C" int fx_ln_bwd_cols(int dtype, const void* dy, const void* s, const float* mean,
                              const float* rstd, const void* gamma, const void* ds_in,
                              void* ds_out, void* dx_out, int rows, int h, float p, uint64_t key,
                              float* part, int with_dbias, float* fg, void* tg, int accg,
                              float* fb, void* tb, int accb, float* fx, void* tx, int accx,
                              hipStream_t st) {
  const int G = fx_ln_bwd_cols_blocks(rows, h, 4096);
  if (G == 0) return -1;
  const int wpr = ln_cols_wpr(h), hw = h / wpr;
  const int rpg = ln_cols_rows_per_group(rows, h);
  DropCfg d = make_drop(p, key);
  auto DY = (const uint16_t*)dy;
  auto S = (const uint16_t*)s;
  auto GM = (const uint16_t*)gamma;
  auto DI = (const uint16_t*)ds_in;
  auto DS = (uint16_t*)ds_out;
  auto DX = (uint16_t*)dx_out;
  const int vpt = (hw + 511) / 512;
  const bool mask = hw % 512 != 0;
#define LNC_GO(V, W, M, DB)                                                                   \
  FX_DISPATCH_T(dtype, ln_bwd_cols_kernel<T, V, W, M, DB><<<G, 256, 0, st>>>(                 \
                           DY, S, mean, rstd, GM, DI, DS, DX, rows, h, rpg, part, d))
#define LNC_M(V, W)                                                                           \
  if (mask) {                                                                                 \
    if (with_dbias) { LNC_GO(V, W, true, true); } else { LNC_GO(V, W, true, false); }         \
  } else {                                                                                    \
    if (with_dbias) { LNC_GO(V, W, false, true); } else { LNC_GO(V, W, false, false); }       \
  }
#define LNC_V(V)                                                                              \
  case V:                                                                                     \
    if (wpr == 1) { LNC_M(V, 1) } else if (wpr == 2) { LNC_M(V, 2) } else { LNC_M(V, 4) }     \
    break;
  switch (vpt) {
    LNC_V(1) LNC_V(2) LNC_V(3)
    default: return -1;
  }
#undef LNC_V
#undef LNC_M
#undef LNC_GO
  LnColsOut f;
  f.f32[0] = fg; f.f32[1] = fb; f.f32[2] = fx;
  f.t16[0] = (uint16_t*)tg; f.t16[1] = (uint16_t*)tb; f.t16[2] = (uint16_t*)tx;
  f.acc[0] = accg; f.acc[1] = accb; f.acc[2] = accx;
  dim3 grid((h + 127) / 128, with_dbias ? 3 : 2);
  FX_DISPATCH_T(dtype, ln_cols_finalize_kernel<T><<<grid, 256, 0, st>>>(part, G, h, f));
  return 0;
}

// dgamma/dbeta partials (mode 0) or plain column sum partials (mode 1).
extern "C" void fx_coltile_partial(int dtype, int mode, const void* a, const void* b,
                                   const float* mean, const float* rstd, float* p0, float* p1,
                                   int rows, int cols, int splits, hipStream_t st, int* cnt,
                                   float* f0, void* t0, int acc0, float* f1, void* t1, int acc1) {
  const ColFin fin = make_fin(cnt, f0, t0, acc0, f1, t1, acc1);
  int rps = (rows + splits - 1) / splits;
  dim3 grid((cols + 127) / 128, splits), block(256);
  auto A = (const uint16_t*)a;
  auto B = (const uint16_t*)b;
  if (mode == 0) {
    FX_DISPATCH_T(dtype, coltile_partial_kernel<T, 0><<<grid, block, 0, st>>>(
                             A, B, mean, rstd, p0, p1, rows, cols, rps, fin));
  } else {
    FX_DISPATCH_T(dtype, coltile_partial_kernel<T, 1><<<grid, block, 0, st>>>(
                             A, B, mean, rstd, p0, p1, rows, cols, rps, fin));
  }
}

extern "C" void fx_coltile_finalize(int dtype, const float* part, int splits, int cols,
                                    float* out_f32, void* out_t, int accumulate, hipStream_t st) {
  dim3 grid((cols + 255) / 256), block(256);
  FX_DISPATCH_T(dtype, coltile_finalize_kernel<T><<<grid, block, 0, st>>>(
                           part, splits, cols, out_f32, (uint16_t*)out_t, accumulate));
}

extern "C" void fx_bias_gelu_fwd(int dtype, int erf, const void* x, const void* bias, void* y,
                                 long n, int cols, hipStream_t st) {
  long n8 = n / 8;
  if (erf) {
    FX_DISPATCH_T(dtype, bias_gelu_fwd_kernel<T, true><<<grid_for(n8), 256, 0, st>>>(
                             (const uint16_t*)x, (const uint16_t*)bias, (uint16_t*)y, n8, cols));
  } else {
    FX_DISPATCH_T(dtype, bias_gelu_fwd_kernel<T, false><<<grid_for(n8), 256, 0, st>>>(
                             (const uint16_t*)x, (const uint16_t*)bias, (uint16_t*)y, n8, cols));
  }
}

extern "C" void fx_bias_gelu_bwd(int dtype, int erf, const void* dy, const void* x,
                                 const void* bias, void* dx, float* part, int rows, int cols,
                                 int splits, hipStream_t st, int* cnt, float* out_f32,
                                 void* out_t, int acc) {
  const ColFin fin = make_fin(cnt, out_f32, out_t, acc, nullptr, nullptr, 0);
  int rps = (rows + splits - 1) / splits;
  dim3 grid((cols + 127) / 128, splits), block(256);
  if (erf) {
    FX_DISPATCH_T(dtype, bias_gelu_bwd_kernel<T, true><<<grid, block, 0, st>>>(
                             (const uint16_t*)dy, (const uint16_t*)x, (const uint16_t*)bias,
                             (uint16_t*)dx, part, rows, cols, rps, fin));
  } else {
    FX_DISPATCH_T(dtype, bias_gelu_bwd_kernel<T, false><<<grid, block, 0, st>>>(
                             (const uint16_t*)dy, (const uint16_t*)x, (const uint16_t*)bias,
                             (uint16_t*)dx, part, rows, cols, rps, fin));
  }
}

extern "C" void fx_bias_dropout_add_fwd(int dtype, const void* x, const void* bias,
                                        const void* residual, void* out, long n, int cols, float p,
                                        uint64_t key, hipStream_t st) {
  DropCfg d = make_drop(p, key);
  long n8 = n / 8;
  FX_DISPATCH_T(dtype, bias_dropout_add_fwd_kernel<T><<<grid_for(n8), 256, 0, st>>>(
                           (const uint16_t*)x, (const uint16_t*)bias, (const uint16_t*)residual,
                           (uint16_t*)out, n8, cols, d));
}

extern "C" void fx_dropout_bwd_colsum(int dtype, const void* dout, void* dx, float* part,
                                      int rows, int cols, int splits, float p, uint64_t key,
                                      hipStream_t st, int* cnt, float* out_f32, void* out_t,
                                      int acc) {
  const ColFin fin = make_fin(cnt, out_f32, out_t, acc, nullptr, nullptr, 0);
  DropCfg d = make_drop(p, key);
  int rps = (rows + splits - 1) / splits;
  dim3 grid((cols + 127) / 128, splits), block(256);
  FX_DISPATCH_T(dtype, dropout_bwd_colsum_kernel<T><<<grid, block, 0, st>>>(
                           (const uint16_t*)dout, (uint16_t*)dx, part, rows, cols, rps, d, fin));
}

extern "C" void fx_dropout_fwd(int dtype, const void* x, void* y, long n, float p, uint64_t key,
                               hipStream_t st) {
  DropCfg d = make_drop(p, key);
  long n8 = n / 8;
  FX_DISPATCH_T(dtype, dropout_fwd_kernel<T><<<grid_for(n8), 256, 0, st>>>(
                           (const uint16_t*)x, (uint16_t*)y, n8, d));
}

// graph-mode dropout salt (see resolve_drop): a device uint64 read by every
// dropout-bearing launch issued while it is set (nullptr = eager keys)
const uint64_t* g_fx_dropout_salt = nullptr;
extern "C" void fx_set_dropout_salt(const void* p) {
  g_fx_dropout_salt = reinterpret_cast<const uint64_t*>(p);
}
