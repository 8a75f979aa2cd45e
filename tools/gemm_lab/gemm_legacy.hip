// Dense GEMM for gfx950 on MFMA with fused transformer epilogues.
//
//   C[M, N] = sum_k A[m, k] * B[k, n]      (fp32 accumulate)
//
// Each operand comes in one of two layouts, so every training GEMM of a
// linear layer runs WITHOUT a transposed copy:
//   KC  "k-contiguous":  A stored [M][K] / B stored [N][K]   (x, W of y = x W^T)
//   MC  "mn-contiguous": A stored [K][M] / B stored [K][N]   (W in dX = dY W,
//                                                              dY and x in dW = dY^T x)
// Epilogues (replacing reference K01/K02/K08; FusedLinear /
// fused_gemm_epilogue at `gpt/dygraph/single_model.py:29,81,375` and
// `language_model/utils.py:30-36`):
//   STORE      C = acc (+ bias[n])                      16-bit out
//   BIAS_GELU  aux = acc + bias ; C = gelu(aux)         FC1 forward (pre-activation kept for bwd)
//   DGELU      C = acc * gelu'(aux)                     FC2 data-gradient -> dH directly
//   F32        C32 = acc (+ C32 when beta)              weight gradient into fp32 main_grad
//
// CDNA4 structure:
//  * 256x256x64 block tile, 512 threads = 8 waves as 2 (M) x 4 (N); each wave
//    owns 128x64 of C as 8x4 v_mfma_f32_16x16x32 tiles (128 accumulator regs),
//    1 workgroup per CU (128 KiB LDS), 2 waves per SIMD.
//  * MFMA operands are swapped (D = B^T-tile x A^T-tile) so a lane's 4 results
//    are 4 CONSECUTIVE n of one row: 8-byte (16-bit) / 16-byte (fp32) stores.
//  * Every K-tile is staged as 4 pieces of 16 KiB (A rows of the waves' first /
//    second M-quadrant, B cols of the first / second N-quadrant) straight
//    HBM -> LDS with global_load_lds (no VGPR staging).  The K loop runs one
//    C-quadrant (16 MFMAs) per phase; a piece is restaged for K-tile t+2 right
//    after its last read in tile t, so 5 pieces (10 loads per wave) stay in
//    flight across the raw s_barriers (counted vmcnt, never 0 in steady state).
//  * LDS images are XOR-swizzled on the per-lane GLOBAL address (the LDS-DMA
//    destination is lane-linear): KC pieces are read by ds_read_b128
//    conflict-free, MC pieces by ds_read_b64_tr_b16 (hardware transpose)
//    conflict-free.
//  * blockIdx is remapped XCD-contiguously, then grouped 8 tiles along M so
//    the 32 concurrent tiles of an XCD share A/B panels in that XCD's L2.
#include <stdlib.h>

#include <type_traits>

#include "fx_common.h"
#include "gemm_common.h"

typedef short v4s __attribute__((ext_vector_type(4)));
#define LDS_AS(p) ((__attribute__((address_space(3))) void*)(p))
#define LDSV4(p) ((__attribute__((address_space(3))) v4s*)(p))

// Ablation builds for tools/gemm_lab (never set in the library build):
// 1 = no MFMAs (operand reads kept alive), 2 = no global->LDS staging,
// 3 = neither staging nor LDS operand reads (MFMAs + barriers only).
#ifndef FX_GEMM_ABL
#define FX_GEMM_ABL 0
#endif
// FX_GEMM_STAMP=1 (lab only): s_memtime stamps of workgroup 0's phases.
#ifndef FX_GEMM_STAMP
#define FX_GEMM_STAMP 0
#endif

// gemm5.hip: the 4-wave kernel with the hand-scheduled K-loop
int fx_gemm5_launch(int dt, int la, int lb, int epi, const fxg::GemmParams& P, hipStream_t st);
long fx_gemm5_ws_bytes(int M, int N, int K);

namespace {

using namespace fxg;

// piece-local row (0..127) -> row of the 256-wide block tile.  The A pieces
// hold rows {wr*128 + h*64 + 0..63}, the B pieces cols {wc*64 + h*32 + 0..31}.
template <bool ISA>
__device__ __forceinline__ int tile_row(int pr, int h) {
  if constexpr (ISA) return (pr >> 6) * 128 + h * 64 + (pr & 63);
  else return (pr >> 5) * 64 + h * 32 + (pr & 31);
}

// Per-lane source offsets (elements) of this wave's two 1-KiB LDS-DMA
// instructions for piece half h (0/1), relative to the operand base; the
// K-tile term is added per tile.  Rows past the matrix edge are clamped (the
// results for them are never stored).
template <int LAY, bool ISA>
struct Stager {
  uint32_t off[2][2];  // [h][instr]
  __device__ __forceinline__ void init(int w, int lane, int rc0, int nrows, long ld) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int blk = 2 * w + u;
        if constexpr (LAY == LAY_KC) {
          const int pr = 8 * blk + (lane >> 3), c = lane & 7;
          const int kc = c ^ ((pr >> 1) & 7);
          int g = rc0 + tile_row<ISA>(pr, h);
          g = g < nrows ? g : nrows - 1;
          off[h][u] = (uint32_t)((long)g * ld + 8 * kc);
        } else {
          const int krow = 4 * blk + (lane >> 4), cc = lane & 15;
          const int key = (krow & 3) | (((krow >> 3) & 1) << 2);
          const int pr = 16 * ((cc >> 1) ^ key) + 8 * (cc & 1);
          int g = rc0 + tile_row<ISA>(pr, h);
          g = g + 8 <= nrows ? g : nrows - 8;
          off[h][u] = (uint32_t)((long)krow * ld + g);
        }
      }
  }
  // issue piece half h of K-tile k0 into LDS piece `dst` (this wave's 2 KiB)
  template <int H>
  __device__ __forceinline__ void issue(const uint16_t* base, long ld, int k0, char* dst,
                                        int w) const {
    if (FX_GEMM_ABL >= 2) return;
    const uint16_t* tb = base + (LAY == LAY_KC ? (long)k0 : (long)k0 * ld);
#pragma unroll
    for (int u = 0; u < 2; ++u)
      __builtin_amdgcn_global_load_lds((const void*)(tb + off[H][u]),
                                       LDS_AS(dst + (2 * w + u) * 1024), 16, 0, 0);
  }
};

// 16x16x32 operand fragment (8 16-bit values: row pr0 + (lane&15), k = 32s +
// 8(lane>>4) + 0..7) from a staged piece.
template <int LAY>
__device__ __forceinline__ short8 frag(const char* piece, int pr0, int s, int lane) {
  if constexpr (FX_GEMM_ABL == 3) {
    short8 r;
    asm volatile("; opaque" : "=v"(r));
    return r;
  } else if constexpr (LAY == LAY_KC) {
    const int r = lane & 15;
    const int c = 4 * s + (lane >> 4);
    return *reinterpret_cast<const short8*>(piece + (pr0 + r) * 128 + ((c ^ (r >> 1)) << 4));
  } else {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int key = q | ((g & 1) << 2);
    const int blk = (pr0 >> 4) ^ key;
    const char* b0 = piece + (32 * s + 8 * g + q) * 256 + (blk << 5) + 8 * p;
    v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDSV4(b0));
    v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDSV4(b0 + 4 * 256));
    short8 r;
    r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
    r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
    return r;
  }
}

template <typename T>
__device__ __forceinline__ floatx4 mma(const short8& x, const short8& y, const floatx4& c) {
  if constexpr (FX_GEMM_ABL == 1) {
    asm volatile("" ::"v"(x), "v"(y));
    return c;
  } else if constexpr (std::is_same<T, bf16>::value)
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, x),
                                                   __builtin_bit_cast(bf16x8, y), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, x),
                                                  __builtin_bit_cast(f16x8, y), c, 0, 0, 0);
}

__device__ __forceinline__ void cbar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Retire every outstanding LDS read (s_waitcnt lgkmcnt(0), vmcnt/expcnt
// untouched) as a REAL s_waitcnt the compiler's wait-insertion pass sees: the
// operands of the coming MFMAs are then known to be in registers, so the
// pass does not put an lgkmcnt(0) in front of them that would also wait for
// the prefetch reads issued in between.
__device__ __forceinline__ void lds_reads_done() { __builtin_amdgcn_s_waitcnt(0xC07F); }

// wait until at most 2*young LDS-DMA instructions of this wave are in flight
__device__ __forceinline__ void wait_young(int young) {
  switch (young) {
    case 5: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

// one C-quadrant x K=64: 16 MFMAs
template <typename T, int MI, int NI>
__device__ __forceinline__ void quadrant(floatx4 (&acc)[8][4], const short8 (&af)[4][2],
                                         const short8 (&bf)[2][2]) {
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
        acc[MI * 4 + mt][NI * 2 + nt] = mma<T>(bf[nt][s], af[mt][s], acc[MI * 4 + mt][NI * 2 + nt]);
  __builtin_amdgcn_s_setprio(0);
}

// one k-step (32) of a quadrant: 8 MFMAs, fenced against compiler motion so
// the LDS reads placed between k-steps stay there
template <typename T, int MI, int NI>
__device__ __forceinline__ void half_step(floatx4 (&acc)[8][4], const short8 (&af)[4],
                                          const short8 (&bf)[2]) {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
      acc[MI * 4 + mt][NI * 2 + nt] = mma<T>(bf[nt], af[mt], acc[MI * 4 + mt][NI * 2 + nt]);
  __builtin_amdgcn_s_setprio(0);
  __builtin_amdgcn_sched_barrier(0);
}

template <int LAY>
__device__ __forceinline__ void load_as(short8 (&af)[4], const char* piece, int wr, int s,
                                        int lane) {
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) af[mt] = frag<LAY>(piece, wr * 64 + mt * 16, s, lane);
}
template <int LAY>
__device__ __forceinline__ void load_bs(short8 (&bf)[2], const char* piece, int wc, int s,
                                        int lane) {
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) bf[nt] = frag<LAY>(piece, wc * 32 + nt * 16, s, lane);
}

template <int LAY>
__device__ __forceinline__ void load_a(short8 (&af)[4][2], const char* piece, int wr, int lane) {
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int s = 0; s < 2; ++s) af[mt][s] = frag<LAY>(piece, wr * 64 + mt * 16, s, lane);
}
template <int LAY>
__device__ __forceinline__ void load_b(short8 (&bf)[2][2], const char* piece, int wc, int lane) {
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int s = 0; s < 2; ++s) bf[nt][s] = frag<LAY>(piece, wc * 32 + nt * 16, s, lane);
}

template <typename T, int LA, int LB, int EPI, bool PF>
__global__ __launch_bounds__(512, 1) void gemm_kernel(GemmParams P) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 2, wc = w & 3;

  // XCD-contiguous block ids, then 8-tile-tall groups along M
  const int nwg = P.tiles_m * P.tiles_n;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int GM = P.gm;
  const int per_group = GM * P.tiles_n;
  const int group = wg / per_group, first_m = group * GM;
  const int gm = min(P.tiles_m - first_m, GM);
  const int in_group = wg - group * per_group;
  const int m0 = (first_m + in_group % gm) * BM;
  const int n0 = (in_group / gm) * BN;

  Stager<LA, true> sa;
  Stager<LB, false> sb;
  sa.init(w, lane, m0, P.M, P.lda);
  sb.init(w, lane, n0, P.N, P.ldb);
  const uint16_t* Ab = P.A;
  const uint16_t* Bb = P.B;

  floatx4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int nk = P.K / BK;
  const int npieces = 4 * nk;
  // piece n = 4u + idx of K-tile u: idx 0 = A half 0, 1 = B half 0, 2 = B half 1,
  // 3 = A half 1; LDS slot ((u & 1) * 4 + idx).  Piece n is issued at phase n - 7.
  auto issue = [&](int n) {
    const int u = n >> 2, idx = n & 3;
    char* dst = smem + ((u & 1) * 4 + idx) * PIECE;
    const int k0 = u * BK;
    if (idx == 0) sa.template issue<0>(Ab, P.lda, k0, dst, w);
    else if (idx == 1) sb.template issue<0>(Bb, P.ldb, k0, dst, w);
    else if (idx == 2) sb.template issue<1>(Bb, P.ldb, k0, dst, w);
    else sa.template issue<1>(Ab, P.lda, k0, dst, w);
  };
#pragma unroll
  for (int n = 0; n < 7; ++n)
    if (n < npieces) issue(n);

  if constexpr (!PF) {
    short8 af[4][2], bf0[2][2], bf1[2][2];
    for (int t = 0; t < nk; ++t) {
      const char* cur = smem + (t & 1) * TILE_BYTES;
      char* nxt = smem + ((t + 1) & 1) * TILE_BYTES;
      char* same = smem + (t & 1) * TILE_BYTES;
      const int P0 = 4 * t;
      const bool full = t + 3 <= nk;
      // ---- phase 0: quadrant (0,0) needs A half 0 + B half 0
      wait_young(full ? 5 : min(5, npieces - P0 - 2));
      cbar();
      load_b<LB>(bf0, cur + 1 * PIECE, wc, lane);
      load_a<LA>(af, cur + 0 * PIECE, wr, lane);
      if (P0 + 7 < npieces) sa.template issue<1>(Ab, P.lda, (t + 1) * BK, nxt + 3 * PIECE, w);
      quadrant<T, 0, 0>(acc, af, bf0);
      // ---- phase 1: quadrant (0,1) needs B half 1
      wait_young(full ? 5 : min(5, npieces - P0 - 3));
      cbar();
      load_b<LB>(bf1, cur + 2 * PIECE, wc, lane);
      if (P0 + 8 < npieces) sa.template issue<0>(Ab, P.lda, (t + 2) * BK, same + 0 * PIECE, w);
      quadrant<T, 0, 1>(acc, af, bf1);
      // ---- phase 2: quadrant (1,1) needs A half 1
      wait_young(full ? 5 : min(5, npieces - P0 - 4));
      cbar();
      load_a<LA>(af, cur + 3 * PIECE, wr, lane);
      if (P0 + 9 < npieces) sb.template issue<0>(Bb, P.ldb, (t + 2) * BK, same + 1 * PIECE, w);
      quadrant<T, 1, 1>(acc, af, bf1);
      // ---- phase 3: quadrant (1,0): operands already in registers
      if (P0 + 10 < npieces) sb.template issue<1>(Bb, P.ldb, (t + 2) * BK, same + 2 * PIECE, w);
      quadrant<T, 1, 0>(acc, af, bf0);
    }
  } else {
    // Fragment reads half a quadrant AHEAD of their MFMAs: each quadrant runs
    // as two k-steps of 8 MFMAs, and the operands of the next k-step are read
    // from LDS while the current one computes.  Fragment sets are per k-step
    // (A: 16 VGPRs, B: 8), so the prefetch costs ~8 VGPRs over no prefetch.
    // Piece n is first read at phase ~n-2 (issued at n-7): 4 in flight.
    short8 a0s0[4], a0s1[4], a1s0[4], a1s1[4], b0s0[2], b0s1[2], b1s0[2], b1s1[2];
    wait_young(min(5, npieces - 2));
    cbar();
    load_as<LA>(a0s0, smem + 0 * PIECE, wr, 0, lane);
    load_bs<LB>(b0s0, smem + 1 * PIECE, wc, 0, lane);
    for (int t = 0; t < nk; ++t) {
      const char* cur = smem + (t & 1) * TILE_BYTES;
      char* nxt = smem + ((t + 1) & 1) * TILE_BYTES;
      char* same = smem + (t & 1) * TILE_BYTES;
      const int P0 = 4 * t;
      const bool full = t + 3 <= nk;
      // q0: quadrant (A0,B0)
      wait_young(full ? 4 : max(0, min(4, npieces - P0 - 3)));
      cbar();
      if (P0 + 7 < npieces) sa.template issue<1>(Ab, P.lda, (t + 1) * BK, nxt + 3 * PIECE, w);
      lds_reads_done();
      load_as<LA>(a0s1, cur + 0 * PIECE, wr, 1, lane);
      load_bs<LB>(b0s1, cur + 1 * PIECE, wc, 1, lane);
      half_step<T, 0, 0>(acc, a0s0, b0s0);
      lds_reads_done();
      load_bs<LB>(b1s0, cur + 2 * PIECE, wc, 0, lane);
      half_step<T, 0, 0>(acc, a0s1, b0s1);
      // q1: quadrant (A0,B1)
      wait_young(full ? 4 : max(0, min(4, npieces - P0 - 4)));
      cbar();
      if (P0 + 8 < npieces) sa.template issue<0>(Ab, P.lda, (t + 2) * BK, same + 0 * PIECE, w);
      lds_reads_done();
      load_bs<LB>(b1s1, cur + 2 * PIECE, wc, 1, lane);
      half_step<T, 0, 1>(acc, a0s0, b1s0);
      lds_reads_done();
      load_as<LA>(a1s0, cur + 3 * PIECE, wr, 0, lane);
      half_step<T, 0, 1>(acc, a0s1, b1s1);
      // q2: quadrant (A1,B1)
      if (P0 + 9 < npieces) sb.template issue<0>(Bb, P.ldb, (t + 2) * BK, same + 1 * PIECE, w);
      lds_reads_done();
      load_as<LA>(a1s1, cur + 3 * PIECE, wr, 1, lane);
      half_step<T, 1, 1>(acc, a1s0, b1s0);
      half_step<T, 1, 1>(acc, a1s1, b1s1);
      // q3: quadrant (A1,B0); first k-step operands of tile t+1
      if (t + 1 < nk) {
        wait_young(full ? 4 : max(0, min(4, npieces - P0 - 6)));
        cbar();
        if (P0 + 10 < npieces) sb.template issue<1>(Bb, P.ldb, (t + 2) * BK, same + 2 * PIECE, w);
      }
      short8 an[4], bn[2];
      lds_reads_done();
      if (t + 1 < nk) {
        load_as<LA>(an, nxt + 0 * PIECE, wr, 0, lane);
        load_bs<LB>(bn, nxt + 1 * PIECE, wc, 0, lane);
      }
      half_step<T, 1, 0>(acc, a1s0, b0s0);
      lds_reads_done();
      half_step<T, 1, 0>(acc, a1s1, b0s1);
#pragma unroll
      for (int i = 0; i < 4; ++i) a0s0[i] = an[i];
#pragma unroll
      for (int i = 0; i < 2; ++i) b0s0[i] = bn[i];
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // ---- epilogue: lane holds C[m][n .. n+3]
  const int mrow = m0 + wr * 128 + (lane & 15);
  const int ncol = n0 + wc * 64 + 4 * (lane >> 4);
  float bv[4][4];
  if constexpr (EPI == EPI_STORE || EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_GELU_ERF) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = ncol + (j >> 1) * 32 + (j & 1) * 16;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        bv[j][e] = (P.bias != nullptr && n + e < P.N) ? Elt<T>::to_f(P.bias[n + e]) : 0.f;
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = mrow + (i >> 2) * 64 + (i & 3) * 16;
    if (m >= P.M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = ncol + (j >> 1) * 32 + (j & 1) * 16;
      if (n >= P.N) continue;
      const floatx4 a = acc[i][j];
      if constexpr (EPI == EPI_F32) {
        float* c = reinterpret_cast<float*>(P.C) + (long)m * P.ldc + n;
        float4 v = make_float4(a[0], a[1], a[2], a[3]);
        if (P.beta) {
          const float4 o = *reinterpret_cast<const float4*>(c);
          v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
        }
        *reinterpret_cast<float4*>(c) = v;
      } else {
        float v[4] = {a[0], a[1], a[2], a[3]};
        uint16_t* c = reinterpret_cast<uint16_t*>(P.C) + (long)m * P.ldc + n;
        if constexpr (EPI == EPI_STORE) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += bv[j][e];
        } else if constexpr (EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_GELU_ERF) {
          ushort4 hv;
          uint16_t* hp = reinterpret_cast<uint16_t*>(&hv);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float x = v[e] + bv[j][e];
            hp[e] = Elt<T>::from_f(x);
            v[e] = EPI == EPI_BIAS_GELU ? gelu_tanh(x) : gelu_erf(x);
          }
          *reinterpret_cast<ushort4*>(P.aux + (long)m * P.ldaux + n) = hv;
        } else {  // DGELU
          const ushort4 hv = *reinterpret_cast<const ushort4*>(P.aux + (long)m * P.ldaux + n);
          const uint16_t* hp = reinterpret_cast<const uint16_t*>(&hv);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float x = Elt<T>::to_f(hp[e]);
            v[e] *= EPI == EPI_DGELU ? gelu_tanh_grad(x) : gelu_erf_grad(x);
          }
        }
        ushort4 o;
        uint16_t* op = reinterpret_cast<uint16_t*>(&o);
#pragma unroll
        for (int e = 0; e < 4; ++e) op[e] = Elt<T>::from_f(v[e]);
        *reinterpret_cast<ushort4*>(c) = o;
      }
    }
  }
}

// ============================================================================
// Persistent kernel: one 512-thread workgroup per CU walks its tiles
// (tile L = round * grid + slot, XCD-remapped slot, GM-grouped order) with the
// piece stream running ACROSS tile boundaries: the next tile's first K-tiles
// are staged while this tile finishes, so there is no per-tile prologue, and
// the epilogue's stores drain under the next tile's MFMAs.
//  * staging by buffer_load ... lds: the descriptor's bounds check returns 0
//    for rows past the matrix edge (no clamping), all per-tile / per-K-tile
//    offsets are one scalar add;
//  * 16-bit epilogues go through a 4 KiB per-wave LDS staging slab (the LDS
//    above the two K-tile buffers) and leave as full 128-byte row segments,
//    16 bytes per lane; every epilogue memory op is an unconditional buffer
//    op (out-of-range lanes get an out-of-bounds offset), so the number of
//    VMEM ops an epilogue adds is exact and the counted vmcnt waits of the
//    next tile stay exact.
// ============================================================================
constexpr int STG_BYTES = 4096;
constexpr int SMEM_PK = SMEM + 8 * STG_BYTES;  // 160 KiB
constexpr uint32_t OOB = 0x80000000u;         // extents are < 2 GiB (host check)

#define FX_VMW(N) case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
__device__ __forceinline__ void vm_wait(int n) {
  switch (n) {
    FX_VMW(0) FX_VMW(1) FX_VMW(2) FX_VMW(3) FX_VMW(4) FX_VMW(5) FX_VMW(6) FX_VMW(7)
    FX_VMW(8) FX_VMW(9) FX_VMW(10) FX_VMW(11) FX_VMW(12) FX_VMW(13) FX_VMW(14) FX_VMW(15)
    FX_VMW(16) FX_VMW(17) FX_VMW(18) FX_VMW(19) FX_VMW(20) FX_VMW(21) FX_VMW(22) FX_VMW(23)
    FX_VMW(24) FX_VMW(25) FX_VMW(26) FX_VMW(27) FX_VMW(28) FX_VMW(29) FX_VMW(30) FX_VMW(31)
    FX_VMW(32) FX_VMW(33) FX_VMW(34) FX_VMW(35) FX_VMW(36) FX_VMW(37) FX_VMW(38) FX_VMW(39)
    FX_VMW(40) FX_VMW(41) FX_VMW(42) FX_VMW(43) FX_VMW(44) FX_VMW(45) FX_VMW(46) FX_VMW(47)
    FX_VMW(48) FX_VMW(49) FX_VMW(50) FX_VMW(51) FX_VMW(52) FX_VMW(53) FX_VMW(54) FX_VMW(55)
    FX_VMW(56) FX_VMW(57) FX_VMW(58) FX_VMW(59) FX_VMW(60) FX_VMW(61) FX_VMW(62)
    default: asm volatile("s_waitcnt vmcnt(63)" ::: "memory"); break;
  }
}
#undef FX_VMW


// B operand of the persistent kernel: piece h holds the CONTIGUOUS tile
// columns h*128 + [0, 128) (wave wc's quadrant ni = columns ni*128 + wc*32 +
// [0, 32)), so an mn-contiguous B piece reads whole 256-byte row segments.
template <bool ISA>
__device__ __forceinline__ int pk_tile_row(int pr) {
  return ISA ? tile_row<true>(pr, 0) : pr;
}

template <int LAY, bool ISA>
struct BufStager {
  __amdgpu_buffer_rsrc_t rs;
  uint32_t vo[2];
  uint32_t hdelta;
  long ld;
  __device__ __forceinline__ void init(const uint16_t* base, long ld_, int rows, int K, int w,
                                       int lane) {
    ld = ld_;
    const long extent = LAY == LAY_KC ? ((long)(rows - 1) * ld + K) * 2 : ((long)(K - 1) * ld + rows) * 2;
    rs = rsrc(base, extent);
    constexpr int G = ISA ? 64 : 128;
    hdelta = LAY == LAY_KC ? (uint32_t)(G * ld * 2) : (uint32_t)(G * 2);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int blk = 2 * w + u;
      if constexpr (LAY == LAY_KC) {
        const int pr = 8 * blk + (lane >> 3), c = lane & 7;
        const int kc = c ^ ((pr >> 1) & 7);
        vo[u] = (uint32_t)(((long)pk_tile_row<ISA>(pr) * ld + 8 * kc) * 2);
      } else {
        const int krow = 4 * blk + (lane >> 4), cc = lane & 15;
        const int key = (krow & 3) | (((krow >> 3) & 1) << 2);
        const int pr = 16 * ((cc >> 1) ^ key) + 8 * (cc & 1);
        vo[u] = (uint32_t)(((long)krow * ld + pk_tile_row<ISA>(pr)) * 2);
      }
    }
  }
  __device__ __forceinline__ uint32_t origin(int rc0) const {
    return LAY == LAY_KC ? (uint32_t)(rc0 * ld * 2) : (uint32_t)(rc0 * 2);
  }
  __device__ __forceinline__ uint32_t kterm(int kk) const {
    return LAY == LAY_KC ? (uint32_t)(kk * BK * 2) : (uint32_t)(kk * BK * ld * 2);
  }
  template <int H>
  __device__ __forceinline__ void issue(uint32_t off, char* dst, int w) const {
    if (FX_GEMM_ABL >= 2) return;
    const uint32_t o = off + H * hdelta;
#pragma unroll
    for (int u = 0; u < 2; ++u)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, LDS_AS(dst + (2 * w + u) * 1024), 16, vo[u] + o,
                                               0, 0, 0);
  }
};

typedef int intx4 __attribute__((ext_vector_type(4)));
typedef int intx2 __attribute__((ext_vector_type(2)));

// Epilogue of the persistent kernel (see gemm_pk_kernel).  Lane holds
// C[m][n .. n+3] for acc[i][j]: m = wr*128 + (i>>2)*64 + (i&3)*16 + (lane&15),
// n = wc*64 + (j>>1)*32 + (j&1)*16 + 4*(lane>>4).
template <typename T, int EPI>
__device__ __forceinline__ void pk_epilogue(const GemmParams& P, floatx4 (&acc)[8][4], int m0,
                                            int n0, int wr, int wc, int w, int lane, char* stg) {
  const int mrow = m0 + wr * 128 + (lane & 15);
  const int ncol = n0 + wc * 32 + 4 * (lane >> 4);  // + (j>>1)*128 + (j&1)*16
  if constexpr (EPI == EPI_F32) {
    const __amdgpu_buffer_rsrc_t rc = rsrc(P.C, ((long)(P.M - 1) * P.ldc + P.N) * 4);
    const bool beta = P.beta != 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = mrow + (i >> 2) * 64 + (i & 3) * 16;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = ncol + (j >> 1) * 128 + (j & 1) * 16;
        const uint32_t off = n < P.N ? (uint32_t)(((long)m * P.ldc + n) * 4) : OOB;
        floatx4 v = acc[i][j];
        if (beta) {
          const floatx4 o = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(rc, off, 0, 0));
          v += o;
        }
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(intx4, v), rc, off, 0, 0);
      }
    }
    return;
  } else {
    const long ext16 = ((long)(P.M - 1) * P.ldc + P.N) * 2;
    const __amdgpu_buffer_rsrc_t rc = rsrc(P.C, ext16);
    // bias of this lane's 16 columns
    float bv[4][4];
    constexpr bool USE_BIAS = EPI == EPI_STORE || EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_GELU_ERF;
    if constexpr (USE_BIAS) {
      if (P.bias != nullptr) {
        const __amdgpu_buffer_rsrc_t rb = rsrc(P.bias, (long)P.N * 2);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = ncol + (j >> 1) * 128 + (j & 1) * 16;
          const intx2 b = __builtin_amdgcn_raw_buffer_load_b64(rb, n < P.N ? (uint32_t)(n * 2) : OOB, 0, 0);
          const uint32_t lo = (uint32_t)b.x, hi = (uint32_t)b.y;
          bv[j][0] = Elt<T>::to_f(lo & 0xffff);
          bv[j][1] = Elt<T>::to_f(lo >> 16);
          bv[j][2] = Elt<T>::to_f(hi & 0xffff);
          bv[j][3] = Elt<T>::to_f(hi >> 16);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) bv[j][e] = 0.f;
      }
    }
    __amdgpu_buffer_rsrc_t ra;
    if constexpr (EPI != EPI_STORE) ra = rsrc(P.aux, ((long)(P.M - 1) * P.ldaux + P.N) * 2);
    // Two staging slabs of 16 rows x 128 B (C, and aux for BIAS_GELU): 16-byte
    // chunk ch of row r at r*128 + ((ch ^ (r&7)) << 4).  One m-tile (16 rows)
    // of the wave's 128x64 tile per round.
    char* stg_c = stg;
    char* stg_a = stg + 2048;
    const int rl = lane & 15, g = lane >> 4;
    const int rr = lane >> 3, rch = lane & 7;
    const int scol = n0 + (rch >> 2) * 128 + wc * 32 + (rch & 3) * 8;
    auto flush = [&](const char* slab, const __amdgpu_buffer_rsrc_t& r, long ld, int mbase) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int row = p * 8 + rr;
        const intx4 v = *reinterpret_cast<const intx4*>(slab + row * 128 + ((rch ^ (row & 7)) << 4));
        const uint32_t off = scol < P.N ? (uint32_t)(((long)(mbase + row) * ld + scol) * 2) : OOB;
        __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 0);
      }
    };
    auto put = [&](char* slab, int j, const float* v) {
      const int byte = j * 32 + 8 * g;
      const int ch = byte >> 4, e = (byte >> 3) & 1;
      uint2 pk;
      pk.x = (uint32_t)Elt<T>::from_f(v[0]) | ((uint32_t)Elt<T>::from_f(v[1]) << 16);
      pk.y = (uint32_t)Elt<T>::from_f(v[2]) | ((uint32_t)Elt<T>::from_f(v[3]) << 16);
      *reinterpret_cast<uint2*>(slab + rl * 128 + ((ch ^ (rl & 7)) << 4) + 8 * e) = pk;
    };
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int mbase = m0 + wr * 128 + (i >> 2) * 64 + (i & 3) * 16;
      const int m = mbase + rl;
      intx2 hb[4];
      if constexpr (EPI == EPI_DGELU || EPI == EPI_DGELU_ERF) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = ncol + (j >> 1) * 128 + (j & 1) * 16;
          const uint32_t off = n < P.N ? (uint32_t)(((long)m * P.ldaux + n) * 2) : OOB;
          hb[j] = __builtin_amdgcn_raw_buffer_load_b64(ra, off, 0, 0);
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const floatx4 a = acc[i][j];
        float y[4];
        if constexpr (EPI == EPI_STORE) {
#pragma unroll
          for (int e = 0; e < 4; ++e) y[e] = a[e] + bv[j][e];
        } else if constexpr (EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_GELU_ERF) {
          float h[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            h[e] = a[e] + bv[j][e];
            y[e] = EPI == EPI_BIAS_GELU ? gelu_tanh(h[e]) : gelu_erf(h[e]);
          }
          put(stg_a, j, h);
        } else {  // DGELU
          const uint32_t lo = (uint32_t)hb[j].x, hi = (uint32_t)hb[j].y;
          const float hx[4] = {Elt<T>::to_f(lo & 0xffff), Elt<T>::to_f(lo >> 16),
                               Elt<T>::to_f(hi & 0xffff), Elt<T>::to_f(hi >> 16)};
#pragma unroll
          for (int e = 0; e < 4; ++e)
            y[e] = a[e] * (EPI == EPI_DGELU ? gelu_tanh_grad(hx[e]) : gelu_erf_grad(hx[e]));
        }
        put(stg_c, j, y);
      }
      flush(stg_c, rc, P.ldc, mbase);
      if constexpr (EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_GELU_ERF) flush(stg_a, ra, P.ldaux, mbase);
    }
  }
}

// VMEM operations one epilogue issues per lane (exact: every one is an
// unconditional buffer op)
template <int EPI>
__device__ __forceinline__ int epi_vmem_ops(bool has_bias, bool beta) {
  if constexpr (EPI == EPI_F32) return beta ? 64 : 32;
  else if constexpr (EPI == EPI_STORE) return 16 + (has_bias ? 4 : 0);
  else if constexpr (EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_GELU_ERF) return 32 + (has_bias ? 4 : 0);
  else return 16 + 32;  // DGELU: 32 aux loads + 16 stores
}

template <typename T, int LA, int LB, int EPI, bool PF>
__global__ __launch_bounds__(512, 1) void gemm_pk_kernel(GemmParams P) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 2, wc = w & 3;
  const int G = gridDim.x;
  const int ntiles = P.tiles_m * P.tiles_n;
  const int pb = xcd_remap(blockIdx.x, G);
  if (pb >= ntiles) return;
  const int ntl = (ntiles - pb + G - 1) / G;
  const int nk = P.K / BK;
  const int npieces = 4 * ntl * nk;

  auto tile_org = [&](int lt, int& m0, int& n0) {
    const int L = lt * G + pb;
    const int per_group = P.gm * P.tiles_n;
    const int group = L / per_group, first_m = group * P.gm;
    const int gm = min(P.tiles_m - first_m, P.gm);
    const int in_group = L - group * per_group;
    m0 = (first_m + in_group % gm) * BM;
    n0 = (in_group / gm) * BN;
  };

  BufStager<LA, true> sa;
  BufStager<LB, false> sb;
  sa.init(P.A, P.lda, P.M, P.K, w, lane);
  sb.init(P.B, P.ldb, P.N, P.K, w, lane);

  int m0c, n0c, m0n = 0, n0n = 0;
  tile_org(0, m0c, n0c);
  if (ntl > 1) tile_org(1, m0n, n0n);
  uint32_t ao_c = sa.origin(m0c), bo_c = sb.origin(n0c);
  uint32_t ao_n = sa.origin(m0n), bo_n = sb.origin(n0n);
  int lt_c = 0, kk_c = 0;

  // prologue: pieces 0..6 = K-tiles 0 and 1 of tile 0 (nk >= 2)
  sa.template issue<0>(ao_c + sa.kterm(0), smem + 0 * PIECE, w);
  sb.template issue<0>(bo_c + sb.kterm(0), smem + 1 * PIECE, w);
  sb.template issue<1>(bo_c + sb.kterm(0), smem + 2 * PIECE, w);
  sa.template issue<1>(ao_c + sa.kterm(0), smem + 3 * PIECE, w);
  sa.template issue<0>(ao_c + sa.kterm(1), smem + TILE_BYTES + 0 * PIECE, w);
  sb.template issue<0>(bo_c + sb.kterm(1), smem + TILE_BYTES + 1 * PIECE, w);
  sb.template issue<1>(bo_c + sb.kterm(1), smem + TILE_BYTES + 2 * PIECE, w);

  floatx4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  const bool has_bias = P.bias != nullptr;
  const int ep_ops = epi_vmem_ops<EPI>(has_bias, P.beta != 0);
  int ep_hi = -1;  // pieces <= ep_hi were issued before the last epilogue's VMEM ops

  // wait until piece x (issued before phase P's own issue) has landed
  auto wait_piece = [&](int Pph, int x) {
    const int issued = min(npieces, Pph + 7);
    const int young = issued - 1 - x;
    const int n = 2 * young + (x <= ep_hi ? ep_ops : 0);
    if (n == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (n == 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    else vm_wait(n < 63 ? n : 63);
  };

  short8 a0s0[4], a0s1[4], a1s0[4], a1s1[4], b0s0[2], b0s1[2], b1s0[2], b1s1[2];
  short8 af[4][2], bf0[2][2], bf1[2][2];
  const bool grpB = w >= 4;
  if constexpr (PF) {
    wait_piece(0, 1);
    cbar();
    load_as<LA>(a0s0, smem + 0 * PIECE, wr, 0, lane);
    load_bs<LB>(b0s0, smem + 1 * PIECE, wc, 0, lane);
  } else {
    wait_piece(0, 1);
    cbar();
    if (grpB) cbar();  // group B runs one half-phase behind
  }

  const int KT = ntl * nk;
  for (int t = 0; t < KT; ++t) {
    const char* cur = smem + (t & 1) * TILE_BYTES;
    char* nxt = smem + ((t + 1) & 1) * TILE_BYTES;
    char* same = smem + (t & 1) * TILE_BYTES;
    const int P0 = 4 * t;
    // staging offsets of K-tiles t+1 and t+2 (possibly in the next tile)
    uint32_t a1o, b1o, a2o, b2o;
    {
      int kk = kk_c + 1;
      if (kk < nk) { a1o = ao_c + sa.kterm(kk); b1o = bo_c + sb.kterm(kk); }
      else { kk -= nk; a1o = ao_n + sa.kterm(kk); b1o = bo_n + sb.kterm(kk); }
      kk = kk_c + 2;
      if (kk < nk) { a2o = ao_c + sa.kterm(kk); b2o = bo_c + sb.kterm(kk); }
      else { kk -= nk; a2o = ao_n + sa.kterm(kk); b2o = bo_n + sb.kterm(kk); }
    }
    if constexpr (!PF) {
      // Staggered halves (T3+T4): every phase is a MEMORY half (operand
      // ds_reads, this wave's share of one piece, lgkmcnt drain) and an MFMA
      // half, each closed by a workgroup barrier.  Waves 4-7 run one half
      // behind waves 0-3 (one extra barrier at the start), so on every SIMD
      // one wave streams MFMAs while its partner reads LDS / issues loads.
      // Pieces read in phase k+1 are waited for (vmcnt) before the barrier that
      // opens group A's memory half of phase k+1: by group A after its MFMA
      // half, by group B after its memory half.
      auto mem_end = [&](int k) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (grpB && k + 2 < npieces) wait_piece(k + 1, k + 2);
        cbar();
      };
      auto mma_end = [&](int k) {
        if (!grpB && k + 2 < npieces) wait_piece(k + 1, k + 2);
        cbar();
      };
      // q0: quadrant (A0,B0)
      load_b<LB>(bf0, cur + 1 * PIECE, wc, lane);
      load_a<LA>(af, cur + 0 * PIECE, wr, lane);
      if (P0 + 7 < npieces) sa.template issue<1>(a1o, nxt + 3 * PIECE, w);
      mem_end(P0);
      quadrant<T, 0, 0>(acc, af, bf0);
      mma_end(P0);
      // q1: quadrant (A0,B1)
      load_b<LB>(bf1, cur + 2 * PIECE, wc, lane);
      if (P0 + 8 < npieces) sa.template issue<0>(a2o, same + 0 * PIECE, w);
      mem_end(P0 + 1);
      quadrant<T, 0, 1>(acc, af, bf1);
      mma_end(P0 + 1);
      // q2: quadrant (A1,B1)
      load_a<LA>(af, cur + 3 * PIECE, wr, lane);
      if (P0 + 9 < npieces) sb.template issue<0>(b2o, same + 1 * PIECE, w);
      mem_end(P0 + 2);
      quadrant<T, 1, 1>(acc, af, bf1);
      mma_end(P0 + 2);
      // q3: quadrant (A1,B0): operands already in registers
      if (P0 + 10 < npieces) sb.template issue<1>(b2o, same + 2 * PIECE, w);
      mem_end(P0 + 3);
      quadrant<T, 1, 0>(acc, af, bf0);
      mma_end(P0 + 3);
    } else {
      // q0: quadrant (A0,B0)
      wait_piece(P0, P0 + 2);
      cbar();
      if (P0 + 7 < npieces) sa.template issue<1>(a1o, nxt + 3 * PIECE, w);
      lds_reads_done();
      load_as<LA>(a0s1, cur + 0 * PIECE, wr, 1, lane);
      load_bs<LB>(b0s1, cur + 1 * PIECE, wc, 1, lane);
      half_step<T, 0, 0>(acc, a0s0, b0s0);
      lds_reads_done();
      load_bs<LB>(b1s0, cur + 2 * PIECE, wc, 0, lane);
      half_step<T, 0, 0>(acc, a0s1, b0s1);
      // q1: quadrant (A0,B1)
      wait_piece(P0 + 1, P0 + 3);
      cbar();
      if (P0 + 8 < npieces) sa.template issue<0>(a2o, same + 0 * PIECE, w);
      lds_reads_done();
      load_bs<LB>(b1s1, cur + 2 * PIECE, wc, 1, lane);
      half_step<T, 0, 1>(acc, a0s0, b1s0);
      lds_reads_done();
      load_as<LA>(a1s0, cur + 3 * PIECE, wr, 0, lane);
      half_step<T, 0, 1>(acc, a0s1, b1s1);
      // q2: quadrant (A1,B1)
      if (P0 + 9 < npieces) sb.template issue<0>(b2o, same + 1 * PIECE, w);
      lds_reads_done();
      load_as<LA>(a1s1, cur + 3 * PIECE, wr, 1, lane);
      half_step<T, 1, 1>(acc, a1s0, b1s0);
      half_step<T, 1, 1>(acc, a1s1, b1s1);
      // q3: quadrant (A1,B0); first k-step operands of K-tile t+1
      if (t + 1 < KT) {
        wait_piece(P0 + 3, P0 + 5);
        cbar();
        if (P0 + 10 < npieces) sb.template issue<1>(b2o, same + 2 * PIECE, w);
      }
      short8 an[4], bn[2];
      lds_reads_done();
      if (t + 1 < KT) {
        load_as<LA>(an, nxt + 0 * PIECE, wr, 0, lane);
        load_bs<LB>(bn, nxt + 1 * PIECE, wc, 0, lane);
      }
      half_step<T, 1, 0>(acc, a1s0, b0s0);
      lds_reads_done();
      half_step<T, 1, 0>(acc, a1s1, b0s1);
  #pragma unroll
      for (int i = 0; i < 4; ++i) a0s0[i] = an[i];
  #pragma unroll
      for (int i = 0; i < 2; ++i) b0s0[i] = bn[i];
    }

    if (++kk_c == nk) {
      // ------------------------------------------------------------ epilogue
      pk_epilogue<T, EPI>(P, acc, m0c, n0c, wr, wc, w, lane, smem + SMEM + w * STG_BYTES);
      ep_hi = min(npieces, P0 + 11) - 1;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
      kk_c = 0;
      ++lt_c;
      m0c = m0n; n0c = n0n; ao_c = ao_n; bo_c = bo_n;
      if (lt_c + 1 < ntl) {
        tile_org(lt_c + 1, m0n, n0n);
        ao_n = sa.origin(m0n);
        bo_n = sb.origin(n0n);
      }
    }
  }
  if constexpr (!PF) {
    if (!grpB) cbar();  // same barrier count for both groups
  }
}

// ============================================================================
// 4-wave kernel (default): 256 threads, one wave per SIMD, each wave owns a
// 128x128 block of C as 8x8 v_mfma_f32_16x16x32 tiles (256 accumulators, in
// the AGPR half of the register file).  Against the 8-wave layout this cuts
// the LDS operand reads per K-tile by a third (every A row is read by 2
// waves instead of 4) and doubles the MFMAs per barrier.
//  * whole K-tiles (A 256x64 + B 256x64 = 64 KiB) are staged by LDS-DMA two
//    tiles ahead into 2 buffers; per K-tile two barriers: B1 after the last
//    operand read of the tile (its buffer may then be restaged with K-tile
//    t+2) and B2 once K-tile t+1 has landed (its first operands are then read
//    under the remaining MFMAs);
//  * each k-step of 64 MFMAs carries the next k-step's 16 fragment reads (or
//    the 16 staging loads), interleaved in fixed groups so the matrix pipe
//    never waits for LDS.
// ============================================================================
constexpr int W4_TILE = 65536;
constexpr int W4_SMEM = 2 * W4_TILE;

// MFMA with the accumulator pinned to AGPRs: the builtin lets the register
// allocator rename a 256-register accumulator set every K-iteration (hundreds
// of v_accvgpr moves per tile); the tied "+a" operand keeps each accumulator
// in place.  Its operands come straight from ds_read (the compiler still
// inserts the lgkmcnt waits for them); consecutive MFMAs never share an
// accumulator (64 apart), and the epilogue pads the MFMA -> read hazard.
template <typename T>
__device__ __forceinline__ void mma_agpr(floatx4& acc, const short8& x, const short8& y) {
  if constexpr (FX_GEMM_ABL == 1) {
    asm volatile("" ::"v"(x), "v"(y));
  } else if constexpr (std::is_same<T, bf16>::value) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(x), "v"(y));
  } else {
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(x), "v"(y));
  }
}

template <int LAY>
struct Stage4 {
  __amdgpu_buffer_rsrc_t rs;
  uint32_t vo[8];
  long ld;
  __device__ __forceinline__ void init(const uint16_t* base, long ld_, int rows, int K, int w,
                                       int lane) {
    ld = ld_;
    const long extent = LAY == LAY_KC ? ((long)(rows - 1) * ld + K) * 2 : ((long)(K - 1) * ld + rows) * 2;
    rs = rsrc(base, extent);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int blk = w * 8 + u;
      if constexpr (LAY == LAY_KC) {
        const int row = 8 * blk + (lane >> 3), c = lane & 7;
        const int kc = c ^ ((row >> 1) & 7);
        vo[u] = (uint32_t)(((long)row * ld + 8 * kc) * 2);
      } else {
        const int krow = 2 * blk + (lane >> 5), cc = lane & 31;
        const int key = (krow & 3) | (((krow >> 3) & 1) << 2);
        const int col = 16 * ((cc >> 1) ^ key) + 8 * (cc & 1);
        vo[u] = (uint32_t)(((long)krow * ld + col) * 2);
      }
    }
  }
  __device__ __forceinline__ uint32_t origin(int rc0) const {
    return LAY == LAY_KC ? (uint32_t)(rc0 * ld * 2) : (uint32_t)(rc0 * 2);
  }
  __device__ __forceinline__ uint32_t kterm(int kk) const {
    return LAY == LAY_KC ? (uint32_t)(kk * BK * 2) : (uint32_t)(kk * BK * ld * 2);
  }
  __device__ __forceinline__ void issue(int u, uint32_t off, char* img, int w) const {
    if (FX_GEMM_ABL >= 2) return;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, LDS_AS(img + (w * 8 + u) * 1024), 16, vo[u] + off,
                                             0, 0, 0);
  }
};

// operand fragment from a 256-row x 64-k image: KC rows of 128 B, MC k-rows of 512 B
template <int LAY>
__device__ __forceinline__ short8 frag4(const char* img, int pr0, int s, int lane) {
  if constexpr (FX_GEMM_ABL == 3) {
    short8 r;
    asm volatile("; opaque" : "=v"(r));
    return r;
  } else if constexpr (LAY == LAY_KC) {
    const int r = lane & 15;
    const int c = 4 * s + (lane >> 4);
    return *reinterpret_cast<const short8*>(img + (pr0 + r) * 128 + ((c ^ (r >> 1)) << 4));
  } else {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int key = q | ((g & 1) << 2);
    const int blk = (pr0 >> 4) ^ key;
    const char* b0 = img + (32 * s + 8 * g + q) * 512 + (blk << 5) + 8 * p;
    v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDSV4(b0));
    v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDSV4(b0 + 4 * 512));
    short8 r;
    r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
    r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
    return r;
  }
}

template <typename T, int LA, int LB, int EPI>
__global__ __launch_bounds__(256, 1) void gemm4_kernel(GemmParams P) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1;

  const int nwg = P.tiles_m * P.tiles_n;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int per_group = P.gm * P.tiles_n;
  const int group = wg / per_group, first_m = group * P.gm;
  const int gm = min(P.tiles_m - first_m, P.gm);
  const int in_group = wg - group * per_group;
  const int m0 = (first_m + in_group % gm) * BM;
  const int n0 = (in_group / gm) * BN;

  Stage4<LA> sa;
  Stage4<LB> sb;
  sa.init(P.A, P.lda, P.M, P.K, w, lane);
  sb.init(P.B, P.ldb, P.N, P.K, w, lane);
  const uint32_t ao = sa.origin(m0), bo = sb.origin(n0);
  const int nk = P.K / BK;

  auto stage = [&](int t, int u) {  // staging load u (0..15) of K-tile t
    char* img = smem + (t & 1) * W4_TILE;
    if (u < 8) sa.issue(u, ao + sa.kterm(t), img, w);
    else sb.issue(u - 8, bo + sb.kterm(t), img + 32768, w);
  };

  floatx4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  short8 fa0[8], fb0[8], fa1[8], fb1[8];
#pragma unroll
  for (int u = 0; u < 16; ++u) stage(0, u);
  if (nk > 1) {
#pragma unroll
    for (int u = 0; u < 16; ++u) stage(1, u);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  cbar();
#pragma unroll
  for (int i = 0; i < 8; ++i) fa0[i] = frag4<LA>(smem, wr * 128 + i * 16, 0, lane);
#pragma unroll
  for (int j = 0; j < 8; ++j) fb0[j] = frag4<LB>(smem + 32768, wc * 128 + j * 16, 0, lane);

#if FX_GEMM_STAMP
#define STAMP4(id)                                                                   \
  do {                                                                               \
    if (P.dbg && blockIdx.x == 0 && t >= 8 && t < 16) {                              \
      const unsigned long long v_ = __builtin_amdgcn_s_memtime();                    \
      if (lane == 0) P.dbg[(w * 8 + (t - 8)) * 8 + (id)] = v_;                       \
    }                                                                                \
  } while (0)
#else
#define STAMP4(id) do {} while (0)
#endif
  // Per K-tile: six segments, five barriers.  The A and B halves of a buffer
  // are freed separately (after the last read of each), so the 16 staging
  // loads of K-tile t+2 spread over three segments instead of one burst (the
  // LDS-DMA path moves ~64 B/clk per CU: 64 KiB per K-tile is half of the
  // MFMA time and has to be spread to stay hidden).
  for (int t = 0; t < nk; ++t) {
    STAMP4(0);
    const char* ia = smem + (t & 1) * W4_TILE;
    const char* ib = ia + 32768;
    const char* na = smem + ((t + 1) & 1) * W4_TILE;
    const char* nb = na + 32768;
    const bool more = t + 2 < nk, next = t + 1 < nk;
    // S1: k-step 0 rows 0-1; read A k-half 1
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int r = 0; r < 4; ++r) fa1[4 * i + r] = frag4<LA>(ia, wr * 128 + (4 * i + r) * 16, 1, lane);
#pragma unroll
      for (int j = 0; j < 8; ++j) mma_agpr<T>(acc[i][j], fb0[j], fa0[i]);
    }
    __builtin_amdgcn_sched_barrier(0);
    lds_reads_done();
    cbar();  // A half of this buffer is free
    STAMP4(1);
    // S2: k-step 0 rows 2-3; stage A of K-tile t+2; read B k-half 1
#pragma unroll
    for (int i = 2; i < 4; ++i) {
      __builtin_amdgcn_sched_barrier(0);
      if (more) {
#pragma unroll
        for (int u = 0; u < 4; ++u) stage(t + 2, 4 * (i - 2) + u);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) fb1[4 * (i - 2) + r] = frag4<LB>(ib, wc * 128 + (4 * (i - 2) + r) * 16, 1, lane);
#pragma unroll
      for (int j = 0; j < 8; ++j) mma_agpr<T>(acc[i][j], fb0[j], fa0[i]);
    }
    __builtin_amdgcn_sched_barrier(0);
    lds_reads_done();
    cbar();  // B half of this buffer is free
    STAMP4(2);
    // S3: k-step 0 rows 4-7; stage B of K-tile t+2
#pragma unroll
    for (int i = 4; i < 8; ++i) {
      __builtin_amdgcn_sched_barrier(0);
      if (more) {
        stage(t + 2, 8 + 2 * (i - 4));
        stage(t + 2, 8 + 2 * (i - 4) + 1);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) mma_agpr<T>(acc[i][j], fb0[j], fa0[i]);
    }
    __builtin_amdgcn_sched_barrier(0);
    STAMP4(3);
    // S4: k-step 1 rows 0-3; then K-tile t+1's A must have landed
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 8; ++j) mma_agpr<T>(acc[i][j], fb1[j], fa1[i]);
    }
    __builtin_amdgcn_sched_barrier(0);
    STAMP4(4);
    if (next) {
      if (more) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      cbar();
    }
    STAMP4(5);
    // S5: k-step 1 rows 4-5; read A k-half 0 of K-tile t+1, then its B must have landed
#pragma unroll
    for (int i = 4; i < 6; ++i) {
      __builtin_amdgcn_sched_barrier(0);
      if (next) {
#pragma unroll
        for (int r = 0; r < 4; ++r) fa0[4 * (i - 4) + r] = frag4<LA>(na, wr * 128 + (4 * (i - 4) + r) * 16, 0, lane);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) mma_agpr<T>(acc[i][j], fb1[j], fa1[i]);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (next) {
      if (more) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      cbar();
    }
    STAMP4(6);
    // S6: k-step 1 rows 6-7; read B k-half 0 of K-tile t+1
#pragma unroll
    for (int i = 6; i < 8; ++i) {
      __builtin_amdgcn_sched_barrier(0);
      if (next) {
#pragma unroll
        for (int r = 0; r < 4; ++r) fb0[4 * (i - 6) + r] = frag4<LB>(nb, wc * 128 + (4 * (i - 6) + r) * 16, 0, lane);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) mma_agpr<T>(acc[i][j], fb1[j], fa1[i]);
    }
    __builtin_amdgcn_sched_barrier(0);
    STAMP4(7);
  }
#undef STAMP4

  // ---- epilogue (direct stores; lane holds C[m][n .. n+3])
  asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");  // last MFMAs -> accumulator reads
  const int mrow = m0 + wr * 128 + (lane & 15);
  const int ncol = n0 + wc * 128 + 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = mrow + i * 16;
    if (m >= P.M) continue;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int n = ncol + j * 16;
      if (n >= P.N) continue;
      const floatx4 a = acc[i][j];
      if constexpr (EPI == EPI_F32) {
        float* c = reinterpret_cast<float*>(P.C) + (long)m * P.ldc + n;
        float4 v = make_float4(a[0], a[1], a[2], a[3]);
        if (P.beta) {
          const float4 o = *reinterpret_cast<const float4*>(c);
          v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
        }
        *reinterpret_cast<float4*>(c) = v;
      } else {
        float v[4] = {a[0], a[1], a[2], a[3]};
        uint16_t* c = reinterpret_cast<uint16_t*>(P.C) + (long)m * P.ldc + n;
        if constexpr (EPI == EPI_STORE) {
          if (P.bias != nullptr) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += Elt<T>::to_f(P.bias[n + e]);
          }
        } else if constexpr (EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_GELU_ERF) {
          ushort4 hv;
          uint16_t* hp = reinterpret_cast<uint16_t*>(&hv);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float x = v[e] + (P.bias != nullptr ? Elt<T>::to_f(P.bias[n + e]) : 0.f);
            hp[e] = Elt<T>::from_f(x);
            v[e] = EPI == EPI_BIAS_GELU ? gelu_tanh(x) : gelu_erf(x);
          }
          *reinterpret_cast<ushort4*>(P.aux + (long)m * P.ldaux + n) = hv;
        } else {  // DGELU
          const ushort4 hv = *reinterpret_cast<const ushort4*>(P.aux + (long)m * P.ldaux + n);
          const uint16_t* hp = reinterpret_cast<const uint16_t*>(&hv);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float x = Elt<T>::to_f(hp[e]);
            v[e] *= EPI == EPI_DGELU ? gelu_tanh_grad(x) : gelu_erf_grad(x);
          }
        }
        ushort4 o;
        uint16_t* op = reinterpret_cast<uint16_t*>(&o);
#pragma unroll
        for (int e = 0; e < 4; ++e) op[e] = Elt<T>::from_f(v[e]);
        *reinterpret_cast<ushort4*>(c) = o;
      }
    }
  }
}

static int g_variant = -1;  // FLEETX_GEMM_PF: 5 = hand-scheduled 4-wave (gemm5.hip, default; K >= 128), 0 = plain 8-wave, 1 = prefetching, 2/3 = persistent, 4 = 4-wave HIP
static int g_gm = -1;       // FLEETX_GEMM_GM: M-group height of the tile order (default 8)

template <typename T, int LA, int LB, int EPI>
void launch(const GemmParams& P, hipStream_t st) {
  if (g_variant < 0) {
    const char* e = getenv("FLEETX_GEMM_PF");
    g_variant = e ? atoi(e) : 5;
  }
  if (g_variant == 5 && P.K >= 2 * BK) {
    fx_gemm5_launch(std::is_same<T, f16>::value ? 1 : 0, LA, LB, EPI, P, st);
    return;
  }
  if (g_variant == 4) {
    auto k4 = gemm4_kernel<T, LA, LB, EPI>;
    static bool attr4 = false;
    if (!attr4) {
      (void)hipFuncSetAttribute((const void*)k4, hipFuncAttributeMaxDynamicSharedMemorySize, W4_SMEM);
      attr4 = true;
    }
    hipLaunchKernelGGL(k4, dim3(P.tiles_m * P.tiles_n), dim3(256), W4_SMEM, st, P);
    return;
  }
  if (g_variant >= 2 && g_variant <= 3 && P.K >= 2 * BK && P.N % 8 == 0) {
    auto kp = g_variant == 2 ? gemm_pk_kernel<T, LA, LB, EPI, true> : gemm_pk_kernel<T, LA, LB, EPI, false>;
    static bool attr_pk[2] = {false, false};
    static int ncu = 0;
    if (!attr_pk[g_variant & 1]) {
      (void)hipFuncSetAttribute((const void*)kp, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM_PK);
      int dev = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
      if (ncu <= 0) ncu = 256;
      attr_pk[g_variant & 1] = true;
    }
    const int nt = P.tiles_m * P.tiles_n;
    hipLaunchKernelGGL(kp, dim3(nt < ncu ? nt : ncu), dim3(512), SMEM_PK, st, P);
    return;
  }
  auto k = g_variant ? gemm_kernel<T, LA, LB, EPI, true> : gemm_kernel<T, LA, LB, EPI, false>;
  static bool attr[2] = {false, false};
  if (!attr[g_variant ? 1 : 0]) {
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    attr[g_variant ? 1 : 0] = true;
  }
  hipLaunchKernelGGL(k, dim3(P.tiles_m * P.tiles_n), dim3(512), SMEM, st, P);
}

template <typename T>
int dispatch(int la, int lb, int epi, const GemmParams& P, hipStream_t st) {
  if (la == LAY_KC && lb == LAY_KC) {
    switch (epi) {
      case EPI_STORE: launch<T, LAY_KC, LAY_KC, EPI_STORE>(P, st); return 0;
      case EPI_BIAS_GELU: launch<T, LAY_KC, LAY_KC, EPI_BIAS_GELU>(P, st); return 0;
      case EPI_BIAS_GELU_ERF: launch<T, LAY_KC, LAY_KC, EPI_BIAS_GELU_ERF>(P, st); return 0;
      default: return -3;
    }
  }
  if (la == LAY_KC && lb == LAY_MC) {
    switch (epi) {
      case EPI_STORE: launch<T, LAY_KC, LAY_MC, EPI_STORE>(P, st); return 0;
      case EPI_DGELU: launch<T, LAY_KC, LAY_MC, EPI_DGELU>(P, st); return 0;
      case EPI_DGELU_ERF: launch<T, LAY_KC, LAY_MC, EPI_DGELU_ERF>(P, st); return 0;
      default: return -3;
    }
  }
  if (la == LAY_MC && lb == LAY_MC) {
    switch (epi) {
      case EPI_F32: launch<T, LAY_MC, LAY_MC, EPI_F32>(P, st); return 0;
      case EPI_STORE: launch<T, LAY_MC, LAY_MC, EPI_STORE>(P, st); return 0;
      default: return -3;
    }
  }
  return -3;
}

}  // namespace

extern "C" void fx_gemm_set_variant(int v) { g_variant = v; }
static unsigned long long* g_dbg = nullptr;
extern "C" void fx_gemm_set_debug(unsigned long long* p) { g_dbg = p; }

// Returns 0 when launched, < 0 when the shape / layout / epilogue is not
// covered (the caller falls back to hipBLASLt):
//   -1: K not a multiple of 64 / empty;  -2: an mn-contiguous extent not a
//   multiple of 8, or N not a multiple of 4;  -3: layout x epilogue combo;
//   -4: an operand too large for 32-bit per-lane offsets.
extern "C" int fx_gemm(int dt, int la, int lb, int epi, int M, int N, int K, const void* A,
                       long lda, const void* B, long ldb, void* C, long ldc, const void* bias,
                       void* aux, long ldaux, int beta, hipStream_t st, float* sq, float* ws) {
  if (M <= 0 || N <= 0 || K <= 0 || K % BK) return -1;
  if (sq != nullptr) {  // norm partials: the hand-scheduled kernel's fp32 epilogue only
    if (g_variant < 0) {
      const char* e = getenv("FLEETX_GEMM_PF");
      g_variant = e ? atoi(e) : 5;
    }
    if (epi != EPI_F32 || g_variant != 5 || K < 2 * BK) return -5;
  }
  if (N % 4 || (la == LAY_MC && M % 8) || (lb == LAY_MC && N % 8)) return -2;
  if (M < 8 || N < 8) return -2;
  const long a_span = la == LAY_KC ? (long)M * lda : (long)BK * lda + M;
  const long b_span = lb == LAY_KC ? (long)N * ldb : (long)BK * ldb + N;
  if (a_span >= (1L << 31) || b_span >= (1L << 31)) return -4;
  if ((long)M * ldc * (epi == EPI_F32 ? 4 : 2) >= (1L << 31)) return -4;
  if (aux && (long)M * ldaux * 2 >= (1L << 31)) return -4;
  GemmParams P{};
  P.A = (const uint16_t*)A;
  P.B = (const uint16_t*)B;
  P.C = C;
  P.bias = (const uint16_t*)bias;
  P.aux = (uint16_t*)aux;
  P.lda = lda; P.ldb = ldb; P.ldc = ldc; P.ldaux = ldaux;
  P.M = M; P.N = N; P.K = K;
  P.tiles_m = (M + BM - 1) / BM;
  P.tiles_n = (N + BN - 1) / BN;
  P.beta = beta;
  if (g_gm < 0) {
    const char* e = getenv("FLEETX_GEMM_GM");
    g_gm = e ? atoi(e) : 8;
  }
  P.gm = g_gm > 0 ? g_gm : 8;
  P.dbg = g_dbg;
  P.sq = sq;
  P.ws = epi == EPI_F32 ? ws : nullptr;
  return dt == 0 ? dispatch<bf16>(la, lb, epi, P, st) : dispatch<f16>(la, lb, epi, P, st);
}

// Split-K workspace (bytes) fx_gemm wants in `ws` for an fp32 weight-gradient
// GEMM of this shape; 0 = it runs unsplit (gemm5.hip g5_split_plan).
extern "C" long fx_gemm_ws_bytes(int epi, int M, int N, int K) {
  if (g_variant < 0) {
    const char* e = getenv("FLEETX_GEMM_PF");
    g_variant = e ? atoi(e) : 5;
  }
  if (epi != EPI_F32 || g_variant != 5 || K < 2 * BK || K % BK) return 0;
  return fx_gemm5_ws_bytes(M, N, K);
}
