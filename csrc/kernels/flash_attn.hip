// Fused (flash-style) multi-head attention for gfx950: forward, and backward
// as two atomic-free passes (dK/dV with keys on the MFMA lane, dQ with
// queries on the lane).  Causal and key-padding masks, in-kernel dropout on
// the attention probabilities from the counter hash of parallel/rng.py.
//
// Parity: replaces reference K03-K06 (matmul(q,k^T)*d^-1/2 ->
// softmax_mask_fuse_upper_triangle -> dropout(local_seed) -> matmul(.,v) ->
// head merge); `single_model.py:189-213`,
// `hybrid_model.py:268-298`.  The [b, a, s, s] score tensor is never
// materialised.
//
// CDNA4 structure (see docs/KERNELS.md):
//  * MFMA v_mfma_f32_32x32x16_bf16, wave64.  Forward computes S^T = K.Q^T so
//    each lane owns ONE query column: the row max / sum are in-lane plus one
//    lane^32 exchange, and the S^T accumulator is directly the B operand of
//    O^T = V^T.P^T (no LDS round trip for P).
//  * V^T fragments come from ds_read_b64_tr_b16 (hardware transpose).
//  * K/V tiles are stored as 8-row x 32-column subtiles with an in-group XOR
//    (conflict-free for both the b128 row reads and the tr_b16 reads;
//    verified by tools/lds_bank_sim.py), addressed by base + immediate.
//  * K/V tiles go HBM -> LDS by global_load_lds (no VGPR staging, no
//    ds_write pass); tile i+1 is in flight into the second LDS buffer while
//    tile i computes, one vmcnt drain + barrier per tile.
//  * blockIdx is remapped so the q-blocks of one (batch, head) run on one XCD
//    (shared K/V stay in that XCD's L2); causal grids are issued heaviest
//    block first across the XCD's heads (lpt_order).
#include <cstdlib>
#include <type_traits>

#include "fx_common.h"

typedef short v4s __attribute__((ext_vector_type(4)));
#define LDSV4(p) ((__attribute__((address_space(3))) v4s*)(p))

namespace {

constexpr float LOG2E = 1.4426950408889634f;
#define FA_DKDV_QT 32  // query rows per dK/dV tile
#ifndef FA_DKDV_V128_QT
#define FA_DKDV_V128_QT 32  // query rows per tile of the D = 128 V-in-registers dK/dV pass
#endif
#ifndef FA_DKDV64_QT
#define FA_DKDV64_QT 64  // query rows per tile of the 64-keys-per-wave dK/dV kernel
#endif
#ifndef FA_RESCALE_THR
#define FA_RESCALE_THR 8.0f  // log2 units; 0 = rescale on every growth
#endif
#ifndef FA_FWD_WAVES_DEFAULT
#define FA_FWD_WAVES_DEFAULT 4
#endif
constexpr float LN2 = 0.6931471805599453f;

// LDS image of a [rows][D] 16-bit tile: 8-row x 32-column subtiles of 512 B,
// the 16-byte chunk index XORed inside its 4-chunk group by (row>>2)&3.
// Conflict-free for the b128 row reads of the 32x32x16 operand and for the
// tr_b16 transposed reads (tools/lds_bank_sim.py), and -- unlike a whole-row
// XOR -- the chunk GROUP (ch>>2) and the row group (row>>3) enter additively:
// the reads of one tile then share a few per-lane base registers and differ
// by immediates (ds_read offset:), instead of one address add per read.
template <int D>
__device__ __forceinline__ int loff(int row, int ch) {
  return (16 * D) * (row >> 3) + 512 * (ch >> 2) + 64 * (row & 7) +
         16 * ((ch & 3) ^ ((row >> 2) & 3));
}
// inverse: byte offset (16-byte aligned) -> (row, chunk)
template <int D>
__device__ __forceinline__ void linv(int o, int& row, int& ch) {
  const int r8 = o / (16 * D), rem = o % (16 * D);
  row = 8 * r8 + ((rem & 511) >> 6);
  ch = 4 * (rem >> 9) + (((rem & 63) >> 4) ^ ((row >> 2) & 3));
}

// Fragment reads of the 32x32x16 operands from a tile image, addressed as a
// per-lane base (computed once per kernel) plus compile-time immediates:
//  * row(tile, blk, s): A/B operand of rows 32*blk + (lane&31), k-step s
//    (16 columns), lane half h = lane>>5 holding columns 8h..8h+7;
//  * tr(tile, t, ss, dt): transposed operand via ds_read_b64_tr_b16 -- lane
//    gets column dt*32 + (lane&31) of rows kb+{0..3} and kb+8+{0..3},
//    kb = 32t + 16ss + 4h.
// Both are loff() evaluated in closed form (checked against it for every
// lane in tools/lds_bank_sim.py --check-frag).
template <int D>
struct Frag {
  int rb0, rb1, tb0, tb1;
  __device__ __forceinline__ void init(int lane) {
    const int h = lane >> 5, r = lane & 31;
    const int rbase = 16 * D * (r >> 3) + 64 * (r & 7);
    rb0 = rbase + 16 * (h ^ ((r >> 2) & 3));
    rb1 = rbase + 16 * ((2 + h) ^ ((r >> 2) & 3));
    const int gi = (lane >> 4) & 1, q = (lane >> 2) & 3, p = lane & 3;
    const int tbase = 64 * (4 * h + q) + 8 * (p & 1);
    const int c = 2 * gi + (p >> 1);
    tb0 = tbase + 16 * (c ^ h);
    tb1 = tbase + 16 * (c ^ (2 + h)) + 16 * D;
  }
  __device__ __forceinline__ short8 row(const char* tile, int blk, int s) const {
    return *reinterpret_cast<const short8*>(tile + ((s & 1) ? rb1 : rb0) + 64 * D * blk +
                                            512 * (s >> 1));
  }
  __device__ __forceinline__ short8 tr(const char* tile, int t, int ss, int dt) const {
    const int o = 64 * D * t + 32 * D * ss + 512 * dt;
    v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDSV4(tile + tb0 + o));
    v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDSV4(tile + tb1 + o));
    short8 r;
    r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
    r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
    return r;
  }
  // All D/32 transposed fragments of (t, ss) -- tr(tile, t, ss, 0..D/32-1) --
  // issued from inline asm; the caller waits with tr_wait() before use.
  // Why: for the builtin form the compiler's wait-count pass cannot tell the
  // read from the LDS-DMA prefetch of the NEXT tile still in flight, and puts
  // an s_waitcnt vmcnt(0) before the first transposed read of every loop
  // iteration (gfx950 assembly of fa_fwd / fa_bwd_dq / fa_bwd_dkdv), so the
  // prefetch overlapped only the first half of a tile.  The tile read here
  // was completed by the previous iteration's vmcnt(0) + barrier.
  __device__ __forceinline__ void tr_issue(const char* tile, int t, int ss,
                                           v4s (&lo)[D / 32], v4s (&hi)[D / 32]) const {
    const uint32_t base = (uint32_t)(size_t)((const __attribute__((address_space(3))) char*)tile);
    const uint32_t a0 = base + tb0 + 64 * D * t + 32 * D * ss;
    const uint32_t a1 = base + tb1 + 64 * D * t + 32 * D * ss;
    if constexpr (D == 64) {
      asm volatile(
          "ds_read_b64_tr_b16 %0, %4\n\t"
          "ds_read_b64_tr_b16 %1, %5\n\t"
          "ds_read_b64_tr_b16 %2, %4 offset:512\n\t"
          "ds_read_b64_tr_b16 %3, %5 offset:512"
          : "=&v"(lo[0]), "=&v"(hi[0]), "=&v"(lo[1]), "=&v"(hi[1])
          : "v"(a0), "v"(a1));
    } else if constexpr (D == 96) {
      asm volatile(
          "ds_read_b64_tr_b16 %0, %6\n\t"
          "ds_read_b64_tr_b16 %1, %7\n\t"
          "ds_read_b64_tr_b16 %2, %6 offset:512\n\t"
          "ds_read_b64_tr_b16 %3, %7 offset:512\n\t"
          "ds_read_b64_tr_b16 %4, %6 offset:1024\n\t"
          "ds_read_b64_tr_b16 %5, %7 offset:1024"
          : "=&v"(lo[0]), "=&v"(hi[0]), "=&v"(lo[1]), "=&v"(hi[1]), "=&v"(lo[2]), "=&v"(hi[2])
          : "v"(a0), "v"(a1));
    } else {
      asm volatile(
          "ds_read_b64_tr_b16 %0, %8\n\t"
          "ds_read_b64_tr_b16 %1, %9\n\t"
          "ds_read_b64_tr_b16 %2, %8 offset:512\n\t"
          "ds_read_b64_tr_b16 %3, %9 offset:512\n\t"
          "ds_read_b64_tr_b16 %4, %8 offset:1024\n\t"
          "ds_read_b64_tr_b16 %5, %9 offset:1024\n\t"
          "ds_read_b64_tr_b16 %6, %8 offset:1536\n\t"
          "ds_read_b64_tr_b16 %7, %9 offset:1536"
          : "=&v"(lo[0]), "=&v"(hi[0]), "=&v"(lo[1]), "=&v"(hi[1]), "=&v"(lo[2]), "=&v"(hi[2]),
            "=&v"(lo[3]), "=&v"(hi[3])
          : "v"(a0), "v"(a1));
    }
  }
};

// Wait for tr_issue() results (and any other LDS / scalar-memory op in flight):
// the registers are operands, so no use can be scheduled above the wait.
template <int ND>
__device__ __forceinline__ void tr_wait(v4s (&lo)[ND], v4s (&hi)[ND]) {
  if constexpr (ND == 2)
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(lo[0]), "+v"(hi[0]), "+v"(lo[1]), "+v"(hi[1]));
  else if constexpr (ND == 3)
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(lo[0]), "+v"(hi[0]), "+v"(lo[1]), "+v"(hi[1]), "+v"(lo[2]), "+v"(hi[2]));
  else
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(lo[0]), "+v"(hi[0]), "+v"(lo[1]), "+v"(hi[1]), "+v"(lo[2]), "+v"(hi[2]),
                   "+v"(lo[3]), "+v"(hi[3]));
}
__device__ __forceinline__ short8 tr_join(const v4s& lo, const v4s& hi) {
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

// bf16 or fp16 inputs (T), fp32 accumulate; the 16-bit operands travel as raw lanes
template <typename T>
__device__ __forceinline__ floatx16 mfma(const short8& a, const short8& b, const floatx16& c) {
  if constexpr (std::is_same<T, bf16>::value)
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}

// fp32 -> 16-bit lane of type T (round to nearest even)
template <typename T>
__device__ __forceinline__ short cvt16(float x) {
  if constexpr (std::is_same<T, bf16>::value) return __builtin_bit_cast(short, (__bf16)x);
  else return __builtin_bit_cast(short, (_Float16)x);
}

// row index (within a 32-row C tile) held in register i for lane half h
__device__ __forceinline__ int crow(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

// Store one output row per lane pair from a 32x32 accumulator set in the
// transposed (column = row of the output) layout: lane l and l + 32 hold the
// two 8-byte halves of every 16 consecutive columns of the row.  One
// permlane32 swap per register pair gives lane l columns 8k..8k+7 and lane
// l + 32 columns 8k+8..8k+15 (k even), so the row leaves as whole 16-byte
// chunks -- half the store instructions and half the partial-line writes of
// the 8-byte pieces (the store tail of every attention workgroup).  `ok` must
// agree between lanes l and l + 32 (same row); every lane runs the swaps.
template <typename T, int D>
__device__ __forceinline__ void store_row16(uint16_t* rowp, const floatx16 (&acc)[D / 32],
                                            float scale, int h, int dval, bool row16, bool ok) {
  auto pk = [&](float x, float y) {
    return (uint32_t)Elt<T>::from_f(x * scale) | ((uint32_t)Elt<T>::from_f(y * scale) << 16);
  };
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
    for (int k = 0; k < 4; k += 2) {
      uint32_t a0 = pk(acc[dt][4 * k + 0], acc[dt][4 * k + 1]);
      uint32_t a1 = pk(acc[dt][4 * k + 2], acc[dt][4 * k + 3]);
      uint32_t b0 = pk(acc[dt][4 * k + 4], acc[dt][4 * k + 5]);
      uint32_t b1 = pk(acc[dt][4 * k + 6], acc[dt][4 * k + 7]);
      const auto r0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
      const auto r1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
      a0 = r0[0]; b0 = r0[1];
      a1 = r1[0]; b1 = r1[1];
      const int d0 = dt * 32 + 8 * k + 8 * h;  // this lane's 8 columns: d0 .. d0 + 7
      if (ok && d0 < dval) {
        if (row16 && d0 + 8 <= dval) {
          *reinterpret_cast<uint4*>(rowp + d0) = make_uint4(a0, a1, b0, b1);
        } else {  // unaligned rows / a head dim ending mid-chunk: 8-byte halves
          *reinterpret_cast<uint2*>(rowp + d0) = make_uint2(a0, a1);
          if (d0 + 4 < dval) *reinterpret_cast<uint2*>(rowp + d0 + 4) = make_uint2(b0, b1);
        }
      }
    }
}

// 16 zero bytes in global memory: the LDS-DMA source of tile columns past a
// head dim that is not a tile width (D = 88 on the 96 tile, 40 on 64), so
// q / k / v need no zero-padded copies.
__device__ __attribute__((aligned(16))) uint16_t fa_zero16[8] = {0, 0, 0, 0, 0, 0, 0, 0};

// Tile loader: ROWS x D 16-bit elements straight into the swizzled LDS image
// with global_load_lds (16 B per lane, 1 KiB per wave-instruction).  The LDS
// side is lane-linear, so the XOR swizzle is applied to the per-lane GLOBAL
// source address (rule: swizzle both sides or neither).  Rows past `nvalid`
// are clamped to the last valid row; the kernels mask them.
template <int D, int ROWS, int NW = 4>
struct Glds {
  static constexpr int RB = D * 2;
  static constexpr int NP = ROWS * RB / 1024;       // 1 KiB pieces in the tile
  static constexpr int NI = (NP + NW - 1) / NW;     // instructions per wave (NW waves)
  static_assert(NP * 1024 == ROWS * RB, "tile must split into 1 KiB pieces");
  // wave w loads pieces w*NI .. w*NI+NI-1 (the last waves fewer when NW does
  // not divide NP, e.g. 32 rows of D = 96); wave-uniform guard
  static __device__ __forceinline__ bool has(int w, int u) {
    return NP % NW == 0 || w * NI + u < NP;
  }
  static __device__ __forceinline__ void load(const uint16_t* base, long stride, int row0,
                                              int nvalid, char* tile, int w, int lane,
                                              int dv = D) {
    const int last = nvalid - 1;
#pragma unroll
    for (int u = 0; u < NI; ++u) {
      if (!has(w, u)) continue;
      const int blk = (w * NI + u) * 1024;
      int row, chl;
      linv<D>(blk + lane * 16, row, chl);
      int grow = row0 + row;
      grow = grow > last ? last : grow;
      // columns past the valid head dim (e.g. 88 of a 96 tile) read zeros
      const uint16_t* src = chl * 8 < dv ? base + (long)grow * stride + chl * 8 : fa_zero16;
      __builtin_amdgcn_global_load_lds((const void*)src,
                                       (__attribute__((address_space(3))) void*)(tile + blk), 16,
                                       0, 0);
    }
  }
};

// Same loads with the per-lane part of the address (row * stride + swizzled
// chunk) computed ONCE per kernel: a full tile then costs one wave-uniform
// scalar offset plus one 64-bit add per instruction instead of a 64-bit
// multiply chain per lane per tile.  Partial (tail) tiles take the clamping
// path above.
template <int D, int ROWS, int NW = 4>
struct GldsStream {
  using G = Glds<D, ROWS, NW>;
  const uint16_t* base;
  long stride;
  int nvalid, w, dv;
  unsigned zmask;  // bit u: this lane's piece u lies past the valid head dim
  long off[G::NI];
  __device__ __forceinline__ void init(const uint16_t* b, long s, int nv, int wave, int lane,
                                       int dvalid = D) {
    base = b;
    stride = s;
    nvalid = nv;
    w = wave;
    dv = dvalid;
    zmask = 0u;
#pragma unroll
    for (int u = 0; u < G::NI; ++u) {
      int row, chl;
      linv<D>((w * G::NI + u) * 1024 + lane * 16, row, chl);
      off[u] = (long)row * stride + chl * 8;
      if (chl * 8 >= dv) zmask |= 1u << u;
    }
  }
  __device__ __forceinline__ void load(int row0, char* tile, int lane) const {
    if (row0 + ROWS > nvalid || dv < D) {  // tail tile / partial head dim (wave-uniform)
      G::load(base, stride, row0, nvalid, tile, w, lane, dv);
      return;
    }
    const uint16_t* tb = base + (long)row0 * stride;
#pragma unroll
    for (int u = 0; u < G::NI; ++u)
      if (G::has(w, u))
        __builtin_amdgcn_global_load_lds((const void*)(tb + off[u]),
                                       (__attribute__((address_space(3))) void*)(
                                           tile + (w * G::NI + u) * 1024),
                                       16, 0, 0);
  }
};

__device__ __forceinline__ void glds_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// exp2 on the hardware unit (v_exp_f32): the inputs here are <= 0 after the
// row max is subtracted, and flushing results below 2^-126 to zero is exact
// enough for softmax -- libm exp2f adds a denormal-range fix-up per element.
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }
typedef float f2 __attribute__((ext_vector_type(2)));

struct AttnParams {
  const uint16_t *q, *k, *v, *o, *dout;
  uint16_t *out, *dq, *dk, *dv;
  float *lse, *delta;
  const int* kv_lens;
  const float* kbias;      // optional additive key bias [B, kb_b] (natural-log units)
  long kb_b;
  long sq_b, sq_s, sq_h;   // q strides (elements) batch / seq / head
  long sk_b, sk_s, sk_h;   // k (and v) strides
  long sv_b, sv_s, sv_h;
  long so_b, so_s, so_h;   // out / dout strides (same layout)
  long sdq_b, sdq_s, sdq_h;  // dq strides
  long sdk_b, sdk_s, sdk_h;  // dk / dv strides
  int B, H, Sq, Sk;
  float scale;
  uint32_t klo, khi, thr;
  float drop_scale;
  int dval;              // valid head dim (<= the tile's D; columns past it are zero)
  const uint64_t* salt;  // graph mode: per-replay device salt (fx_set_dropout_salt)
  int pair;              // causal forward: two query blocks per workgroup (fa_fwd_kernel)
  int row16;             // output rows 16-byte aligned (store_row16's 16-byte stores)
};

// per-(batch, head) dropout hash seed; under graph mode the baked key is
// re-keyed by the device salt first
__device__ __forceinline__ uint32_t attn_cb(const AttnParams& P, int bh) {
  uint32_t klo = P.klo, khi = P.khi;
  if (P.salt != nullptr) {
    const uint64_t k = salt_key(((uint64_t)khi << 32) | klo, *P.salt);
    klo = (uint32_t)k;
    khi = (uint32_t)(k >> 32);
  }
  return lowbias32((uint32_t)bh ^ khi) ^ klo;
}

// S^T tile rows are keys: register i of lane half h holds key crow(i, h) of
// its 32-row block.  Keys crow(4g..4g+3, h) = 8g + 4h + {0..3} are contiguous,
// so the bias arrives as one float4 per group.  Result: s*scale*log2e + bias*log2e.
__device__ __forceinline__ void key_bias_add1(floatx16& acc, const float* kb, int h, float sl2) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const float4 v = *reinterpret_cast<const float4*>(kb + 8 * g + 4 * h);
    acc[4 * g + 0] = acc[4 * g + 0] * sl2 + v.x * LOG2E;
    acc[4 * g + 1] = acc[4 * g + 1] * sl2 + v.y * LOG2E;
    acc[4 * g + 2] = acc[4 * g + 2] * sl2 + v.z * LOG2E;
    acc[4 * g + 3] = acc[4 * g + 3] * sl2 + v.w * LOG2E;
  }
}
__device__ __forceinline__ void key_bias_add(floatx16 (&acc)[2], const float* kb, int h, float sl2) {
  key_bias_add1(acc[0], kb, h, sl2);
  key_bias_add1(acc[1], kb + 32, h, sl2);
}

__device__ __forceinline__ int xcd_remap(int bid, int nblk) {
  const int xcd = bid & 7, pos = bid >> 3, q = nblk >> 3, r = nblk & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + pos;
}

// Causal work order (longest-processing-time first).  A causal block's cost
// grows with its distance from the diagonal, so dispatching (head, block) in
// head-major order leaves the heaviest blocks of the LAST heads to start near
// the end of the grid: the kernel's tail is one heavy block running alone.
// Here the grid is cut into chunks of G = B*H/8 heads (one XCD's contiguous
// share after xcd_remap, so a head's blocks still share that XCD's L2), and
// inside a chunk every head's heaviest block is issued first, then every
// head's second heaviest, and so on.  `rank` 0 = heaviest.  Bijective on
// [0, nblk) for any B*H.
__device__ __forceinline__ void lpt_order(int lid, int nper, int BH, int& bh, int& rank) {
  const int G = BH >= 8 ? BH >> 3 : 1;
  const int c = lid / (G * nper);
  const int j = lid - c * G * nper;
  const int Gc = min(G, BH - c * G);
  rank = j / Gc;
  bh = c * G + j % Gc;
}

// One 64-key tile of the forward for this wave's 32 queries: S^T = K.Q^T,
// online softmax (mask on diagonal / tail tiles, deferred rescale, dropout on
// P), O^T += V^T.P^T.  (the per-block forward kernel).  
template <typename T, int D, bool CAUSAL, bool DROP, bool KB>
__device__ __forceinline__ void fwd_tile(const AttnParams& P, const Frag<D>& F, const char* kt,
                                         const char* vt, const short8 (&qf)[D / 16],
                                         floatx16 (&oacc)[D / 32], float& m_run, float& lsum,
                                         int kb, int wq0, int qi, int kv_len, int b, int h,
                                         float sl2, uint32_t cb) {
  constexpr int KV = 64;
  // waves without a valid query (the tail block of S = 257) only help load
  if (wq0 < P.Sq && !(CAUSAL && kb > wq0 + 31)) {
    floatx16 sacc[2];
    // the tile's second 32-key half holds no unmasked key when every key in
    // it is past kv_len (the tail tile of S = 257) or above the causal
    // diagonal of all this wave's queries (wave-uniform); its P.V MFMAs are
    // skipped below.  Its scores are still computed (and masked to -inf by
    // the diagonal / tail pass): skipping those MFMAs too made the compiler
    // copy the first half's 16 accumulators on every tile to merge the two
    // paths, which cost more than the few MFMAs it saved on diagonal tiles.
    const bool half2 = (kb + 32 < kv_len && !(CAUSAL && kb + 32 > wq0 + 31));
    // all K fragments of the tile up front: the 16 LDS reads overlap each
    // other instead of one exposed LDS latency per MFMA
    short8 kfr[2][D / 16];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s = 0; s < D / 16; ++s) kfr[t][s] = F.row(kt, t, s);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int i = 0; i < 16; ++i) sacc[t][i] = 0.f;
#pragma unroll
      for (int s = 0; s < D / 16; ++s) sacc[t] = mfma<T>(kfr[t][s], qf[s], sacc[t]);
    }
    const bool need_mask = (CAUSAL && kb + KV - 1 > wq0) || (kb + KV > kv_len);
    if constexpr (KB) key_bias_add(sacc, P.kbias + (long)b * P.kb_b + kb, h, sl2);
    // Online softmax on the lane's 32 scores.  Without a key bias the raw
    // scores are maxed and the scale folds into one FMA before the exp2
    // (scale > 0 commutes with max).  Only tiles on the causal diagonal or
    // past kv_len run the per-element key index / compare / select pass
    // (wave-uniform branch, masked scores set to -inf in place).
    if (__builtin_expect(need_mask, 0)) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int key = kb + 32 * t + crow(i, h);
          if ((CAUSAL && key > qi) || key >= kv_len) sacc[t][i] = -INFINITY;
        }
    }
    {
      float mloc = -INFINITY;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) mloc = fmaxf(mloc, sacc[t][i]);
      mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
      if constexpr (!KB) mloc *= sl2;
      // Deferred rescale: the running max moves (and O / l are rescaled)
      // only when some row of the wave grew by more than FA_RESCALE_THR
      // (log2 units) -- otherwise p = exp2(s - m_run) stays <= 2^THR, exact
      // in fp32 and as bf16 operands (same relative precision).  The
      // decision precedes this tile's exp2, so O, l and P always share one
      // reference max (tests/test_kernels_gpu.py forces the branch mid-row).
      if (__any(mloc > m_run + FA_RESCALE_THR)) {
        const float m_new = fmaxf(m_run, mloc);
        const float alpha = fexp2(m_run - ((m_new == -INFINITY) ? 0.f : m_new));
        m_run = m_new;
        lsum *= alpha;
#pragma unroll
        for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
          for (int i = 0; i < 16; ++i) oacc[dt][i] *= alpha;
      }
      const float m_use = (m_run == -INFINITY) ? 0.f : m_run;
      // score pairs in packed fp32 (v_pk_fma_f32 / v_pk_add_f32: two lanes'
      // worth per VALU issue; the softmax VALU, not the MFMAs, bounds the
      // causal and D = 64 tiles)
      const f2 nm = {-m_use, -m_use}, sc2 = {sl2, sl2};
      // four independent partial sums (a single dependent chain of packed
      // adds stalls on the packed-VALU read-after-write hazard)
      f2 lacc[4] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
          const f2 sv = {sacc[t][i], sacc[t][i + 1]};
          const f2 a = KB ? sv + nm : __builtin_elementwise_fma(sv, sc2, nm);
          const f2 pv = {fexp2(a.x), fexp2(a.y)};
          lacc[(i >> 1) & 3] += pv;
          float p0 = pv.x, p1 = pv.y;
          if (DROP) {  // the keep scale 1/(1-p) is applied once, to O
            const int key = kb + 32 * t + crow(i, h);  // even
            const uint32_t hh = lowbias32((((uint32_t)qi) << 16 | ((uint32_t)key >> 1)) ^ cb);
            p0 = ((hh & 0xffffu) >= P.thr) ? p0 : 0.f;
            p1 = ((hh >> 16) >= P.thr) ? p1 : 0.f;
          }
          sacc[t][i] = p0;
          sacc[t][i + 1] = p1;
        }
      const f2 lt = (lacc[0] + lacc[1]) + (lacc[2] + lacc[3]);
      lsum += lt.x + lt.y;
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      if (t == 1 && !half2) continue;  // P = 0 there
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        v4s vlo[D / 32], vhi[D / 32];
        F.tr_issue(vt, t, ss, vlo, vhi);
        short8 pf;
#pragma unroll
        for (int j = 0; j < 8; ++j) pf[j] = cvt16<T>(sacc[t][8 * ss + j]);
        tr_wait(vlo, vhi);
#pragma unroll
        for (int dt = 0; dt < D / 32; ++dt)
          oacc[dt] = mfma<T>(tr_join(vlo[dt], vhi[dt]), pf, oacc[dt]);
      }
    }
  }
}

// ============================================================================
// forward: WG = 4 waves x 32 queries = 128 queries; KV tile = 64 keys
// ============================================================================
// Causal grids pair query blocks: workgroup p of a head runs block nq-1-p
// (the heaviest) and then block p (the lightest) through ONE K/V tile stream,
// so every workgroup carries the same nq+1 blocks' worth of tiles, the grid is
// half as many workgroups, and the second block's Q fragments and first K/V
// tile load under the first block's last tile instead of in a fresh
// workgroup's exposed prologue.  (fa_pair_grid(): FLEETX_FA_PAIR=0 restores
// one block per workgroup in LPT order.)
__device__ __forceinline__ bool fa_pair_on(const AttnParams& P) { return P.pair != 0; }

#ifdef FX_FA_LAB
// Lab builds: per-wave s_memrealtime (100 MHz) stamps of the forward (tools/fa_lab/stamp_fwd.py;
// 64 slots per wave: 0 XCC / HW id, 1 entry, 2 prologue done, 3 + 2 t after
// tile t's compute, 4 + 2 t after its barrier, 62 before the last finish, 63 end)
__device__ unsigned long long* fa_stamps = nullptr;
#define FA_STN(i, n)                                                    \
  do {                                                                  \
    if (stp) {                                                          \
      const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();   \
      if (lane == 0 && (i) < (n)) stp[(i)] = t_;                        \
    }                                                                   \
  } while (0)
#define FA_ST(i) FA_STN(i, 64)
// dK/dV pass: 128 slots per wave (slot 0 = key block; tile t at 3 + 2 t /
// 4 + 2 t, 126 before the dK / dV stores, 127 end; tools/fa_lab/stamp_bwd.py)
#define FA_ST2(i) FA_STN(i, 128)
#else
#define FA_ST(i) \
  do {           \
  } while (0)
#define FA_ST2(i) \
  do {            \
  } while (0)
#endif

template <typename T, int D, bool CAUSAL, bool DROP, bool KB, int NW>
__global__ __launch_bounds__(64 * NW, 8 / NW) void fa_fwd_kernel(AttnParams P) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int KV = 64, TB = KV * D * 2, QB = 32 * NW;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5;
#ifdef FX_FA_LAB
  unsigned long long* stp = fa_stamps ? fa_stamps + ((long)blockIdx.x * NW + w) * 64 : nullptr;
  if (stp) {
    int xcc, hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    if (lane == 0) stp[0] = ((unsigned long long)(xcc & 15) << 32) | (unsigned)hw;
  }
#endif
  FA_ST(1);
  Frag<D> F;
  F.init(lane);
  const int nq = (P.Sq + QB - 1) / QB;
  // work items of this workgroup: query block qa, then (paired causal) qb2 >= 0
  int bh, qa, qb2 = -1;
  if (CAUSAL && fa_pair_on(P)) {
    const int npair = (nq + 1) >> 1;
    const int lid = xcd_remap(blockIdx.x, npair * P.B * P.H);
    bh = lid / npair;
    const int p = lid - bh * npair;
    qa = nq - 1 - p;
    qb2 = p != qa ? p : -1;
  } else {
    const int nblk = nq * P.B * P.H;
    const int lid = xcd_remap(blockIdx.x, nblk);
    if constexpr (CAUSAL) {
      int rank;
      lpt_order(lid, nq, P.B * P.H, bh, rank);
      qa = nq - 1 - rank;
    } else {
      bh = lid / nq;
      qa = lid % nq;
    }
  }
  const int b = bh / P.H, hd = bh % P.H;

  const uint16_t* qp = P.q + b * P.sq_b + hd * P.sq_h;
  const uint16_t* kp = P.k + b * P.sk_b + hd * P.sk_h;
  const uint16_t* vp = P.v + b * P.sv_b + hd * P.sv_h;
  int kv_len = P.Sk;
  if (P.kv_lens) kv_len = min(kv_len, P.kv_lens[b]);

  auto load_q = [&](int qblock, short8 (&qf)[D / 16]) {
    const int qi_ = qblock * QB + w * 32 + (lane & 31);
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
      if (qi_ < P.Sq && 16 * s + 8 * h < P.dval)
        qf[s] = *reinterpret_cast<const short8*>(qp + (long)qi_ * P.sq_s + 16 * s + 8 * h);
      else
        qf[s] = (short8){0, 0, 0, 0, 0, 0, 0, 0};
    }
  };
  auto tiles_of = [&](int qblock) {
    const int e = CAUSAL ? min(kv_len, (qblock + 1) * QB) : kv_len;
    return (e + KV - 1) / KV;
  };

  int wq0 = qa * QB + w * 32;
  int qi = wq0 + (lane & 31);
  short8 qf[D / 16];
  load_q(qa, qf);
  const int ntA = tiles_of(qa);
  const int ntiles = ntA + (qb2 >= 0 ? tiles_of(qb2) : 0);

  floatx16 oacc[D / 32];
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) oacc[dt][i] = 0.f;
  float m_run = -INFINITY, lsum = 0.f;
  const float sl2 = P.scale * LOG2E;
  const uint32_t cb = DROP ? attn_cb(P, bh) : 0u;

  // O and lse of the current item (its rows are qi of the current wq0)
  auto finish = [&]() {
    const float ltot = lsum + __shfl_xor(lsum, 32, 64);
    const float inv = ltot > 0.f ? (DROP ? P.drop_scale : 1.f) / ltot : 0.f;
    if constexpr (D == 128) {
      store_row16<T, D>(P.out + b * P.so_b + hd * P.so_h + (long)qi * P.so_s, oacc, inv, h,
                        P.dval, P.row16, qi < P.Sq);
      if (qi < P.Sq && h == 0)
        P.lse[(long)bh * P.Sq + qi] = ltot > 0.f ? (m_run + log2f(ltot)) * LN2 : INFINITY;
    } else if (qi < P.Sq) {
      // D 64 / 96: 8-byte pieces (the swaps' registers would cost these
      // kernels a wave per SIMD)
      uint16_t* op = P.out + b * P.so_b + hd * P.so_h + (long)qi * P.so_s;
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          ushort4 o;
          o.x = Elt<T>::from_f(oacc[dt][4 * g + 0] * inv);
          o.y = Elt<T>::from_f(oacc[dt][4 * g + 1] * inv);
          o.z = Elt<T>::from_f(oacc[dt][4 * g + 2] * inv);
          o.w = Elt<T>::from_f(oacc[dt][4 * g + 3] * inv);
          if (dt * 32 + 8 * g + 4 * h < P.dval)
            *reinterpret_cast<ushort4*>(op + dt * 32 + 8 * g + 4 * h) = o;
        }
      if (h == 0)
        P.lse[(long)bh * P.Sq + qi] = ltot > 0.f ? (m_run + log2f(ltot)) * LN2 : INFINITY;
    }
  };

  // the tile stream covers both items (tile t >= ntA is tile t - ntA of the
  // second); rows are clamped at kv_len only -- causal masking is per element
  GldsStream<D, KV, NW> kld, vld;
  kld.init(kp, P.sk_s, kv_len, w, lane, P.dval);
  vld.init(vp, P.sv_s, kv_len, w, lane, P.dval);
  auto row_of = [&](int t) { return (t < ntA ? t : t - ntA) * KV; };
  if (ntiles > 0) {
    kld.load(0, smem, lane);
    vld.load(0, smem + 2 * TB, lane);
  }
  glds_wait();
  __syncthreads();
  FA_ST(2);

  short8 qn[D / 16];  // the second item's Q fragments, loaded under the first's last tile
  for (int it = 0; it < ntiles; ++it) {
    const int cur = it & 1;
    const char* kt = smem + cur * TB;
    const char* vt = smem + 2 * TB + cur * TB;
    const bool more = it + 1 < ntiles;
    const bool switch_item = qb2 >= 0 && it == ntA - 1;
    if (switch_item) load_q(qb2, qn);
    if (more) {
      kld.load(row_of(it + 1), smem + (cur ^ 1) * TB, lane);
      vld.load(row_of(it + 1), smem + 2 * TB + (cur ^ 1) * TB, lane);
    }
#ifdef FA_EXP_NOMASK  // lab timing experiment: the causal grid with the full tile body
    fwd_tile<T, D, false, DROP, KB>(P, F, kt, vt, qf, oacc, m_run, lsum, row_of(it), wq0, qi,
                                    kv_len, b, h, sl2, cb);
#else
    fwd_tile<T, D, CAUSAL, DROP, KB>(P, F, kt, vt, qf, oacc, m_run, lsum, row_of(it), wq0, qi,
                                     kv_len, b, h, sl2, cb);
#endif
    FA_ST(3 + 2 * it);
    if (switch_item) {
      finish();
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) oacc[dt][i] = 0.f;
      m_run = -INFINITY;
      lsum = 0.f;
#pragma unroll
      for (int s = 0; s < D / 16; ++s) qf[s] = qn[s];
      wq0 = qb2 * QB + w * 32;
      qi = wq0 + (lane & 31);
    }
    glds_wait();
    __syncthreads();
    FA_ST(4 + 2 * it);
  }
  if (qb2 >= 0 && ntA == 0) {  // kv_len == 0: no tile switched the items; both rows are empty
    finish();
    wq0 = qb2 * QB + w * 32;
    qi = wq0 + (lane & 31);
  }
  FA_ST(62);
  finish();
  FA_ST(63);
}

// ============================================================================
// backward dQ: WG = 4 waves x 32 queries; loop over 64-key tiles.
//   S^T = K.Q^T, dP^T = V.dO^T (queries on lanes), dQ^T += K^T.dS^T
// ============================================================================
template <typename T, int D, bool CAUSAL, bool DROP, bool KB, int NW = 4>
__global__ __launch_bounds__(64 * NW, 2) void fa_bwd_dq_kernel(AttnParams P) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int KV = 64, TB = KV * D * 2, QB = 32 * NW;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5;
  Frag<D> F;
  F.init(lane);
  const int nq = (P.Sq + QB - 1) / QB;
  const int nblk = nq * P.B * P.H;
  const int lid = xcd_remap(blockIdx.x, nblk);
  int bh, qblock;
  if constexpr (CAUSAL) {
    int rank;
    lpt_order(lid, nq, P.B * P.H, bh, rank);
    qblock = nq - 1 - rank;
  } else {
    bh = lid / nq;
    qblock = lid % nq;
  }
  const int b = bh / P.H, hd = bh % P.H;
  const uint16_t* qp = P.q + b * P.sq_b + hd * P.sq_h;
  const uint16_t* kp = P.k + b * P.sk_b + hd * P.sk_h;
  const uint16_t* vp = P.v + b * P.sv_b + hd * P.sv_h;
  const uint16_t* dop = P.dout + b * P.so_b + hd * P.so_h;
  int kv_len = P.Sk;
  if (P.kv_lens) kv_len = min(kv_len, P.kv_lens[b]);

  const int wq0 = qblock * QB + w * 32;
  const int qi = wq0 + (lane & 31);
  const bool qvalid = qi < P.Sq;
  short8 qf[D / 16], gf[D / 16];
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
    if (qvalid && 16 * s + 8 * h < P.dval) {
      qf[s] = *reinterpret_cast<const short8*>(qp + (long)qi * P.sq_s + 16 * s + 8 * h);
      gf[s] = *reinterpret_cast<const short8*>(dop + (long)qi * P.so_s + 16 * s + 8 * h);
    } else {
      qf[s] = (short8){0, 0, 0, 0, 0, 0, 0, 0};
      gf[s] = qf[s];
    }
  }
  const float lse2 = qvalid ? P.lse[(long)bh * P.Sq + qi] * LOG2E : INFINITY;
  float dlt = 0.f;  // delta = rowsum(dO . O), below (after the first tile's DMA is issued)
  const float sl2 = P.scale * LOG2E;
  const uint32_t cb = DROP ? attn_cb(P, bh) : 0u;

  int kv_end = kv_len;
  if (CAUSAL) kv_end = min(kv_end, (qblock + 1) * QB);
  const int ntiles = (kv_end + KV - 1) / KV;

  floatx16 dqacc[D / 32];
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) dqacc[dt][i] = 0.f;

  GldsStream<D, KV, NW> kld, vld;
  kld.init(kp, P.sk_s, kv_end, w, lane, P.dval);
  vld.init(vp, P.sv_s, kv_end, w, lane, P.dval);
  if (ntiles > 0) {
    kld.load(0, smem, lane);
    vld.load(0, smem + 2 * TB, lane);
  }
  // delta = rowsum(dO . O): taken here from the dO fragments already in
  // registers plus one load of the O row (in flight with the first K/V tile);
  // the dK/dV pass, launched after this one, reads the stored value
  {
    float part = 0.f;
    if (qvalid) {
      const uint16_t* orow = P.o + b * P.so_b + hd * P.so_h + (long)qi * P.so_s;
#pragma unroll
      for (int s = 0; s < D / 16; ++s) {
        if (16 * s + 8 * h >= P.dval) continue;
        float ov[8], gv[8];
        load8<T>(orow + 16 * s + 8 * h, ov);
        unpack8<T>(__builtin_bit_cast(uint4, gf[s]), gv);
#pragma unroll
        for (int j = 0; j < 8; ++j) part += ov[j] * gv[j];
      }
    }
    part += __shfl_xor(part, 32, 64);
    dlt = qvalid ? part : 0.f;
    if (qvalid && h == 0) P.delta[(long)bh * P.Sq + qi] = dlt;
  }
  glds_wait();
  __syncthreads();

  for (int it = 0; it < ntiles; ++it) {
    const int cur = it & 1;
    const char* kt = smem + cur * TB;
    const char* vt = smem + 2 * TB + cur * TB;
    const bool more = it + 1 < ntiles;
    if (more) {
      kld.load((it + 1) * KV, smem + (cur ^ 1) * TB, lane);
      vld.load((it + 1) * KV, smem + 2 * TB + (cur ^ 1) * TB, lane);
    }
    const int kb = it * KV;
    // waves without a valid query (the tail block of S = 257) only help load
    if (wq0 < P.Sq && !(CAUSAL && kb > wq0 + 31)) {
      const bool need_mask = (CAUSAL && kb + KV - 1 > wq0) || (kb + KV > kv_len);
      // second 32-key half fully masked (P = 0 there, so dS = 0): skipped as in
      // the forward (ViT-g backward 291.8 -> 280.0 us, causal D 64 / 128
      // neutral: profiles/r3_fahalf/)
      const bool half2 = (kb + 32 < kv_len && !(CAUSAL && kb + 32 > wq0 + 31));
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        if (t == 1 && !half2) continue;
        floatx16 sacc, dpacc;
#pragma unroll
        for (int i = 0; i < 16; ++i) sacc[i] = dpacc[i] = 0.f;
#pragma unroll
        for (int s = 0; s < D / 16; ++s) {
          sacc = mfma<T>(F.row(kt, t, s), qf[s], sacc);
          dpacc = mfma<T>(F.row(vt, t, s), gf[s], dpacc);
        }
        if constexpr (KB) key_bias_add1(sacc, P.kbias + (long)b * P.kb_b + kb + 32 * t, h, sl2);
        // masked scores -> -inf in place, on diagonal / tail tiles only
        if (__builtin_expect(need_mask, 0)) {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int key = kb + 32 * t + crow(i, h);
            if ((CAUSAL && key > qi) || key >= kv_len) sacc[i] = -INFINITY;
          }
        }
        const float sc = KB ? 1.f : sl2;
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
          // invalid query rows carry lse2 = +inf: p = exp2(-inf) = 0
          const float p0 = fexp2(__builtin_fmaf(sacc[i], sc, -lse2));
          const float p1 = fexp2(__builtin_fmaf(sacc[i + 1], sc, -lse2));
          float dp0 = dpacc[i], dp1 = dpacc[i + 1];
          if (DROP) {
            const int key = kb + 32 * t + crow(i, h);
            const uint32_t hh = lowbias32((((uint32_t)qi) << 16 | ((uint32_t)key >> 1)) ^ cb);
            dp0 = ((hh & 0xffffu) >= P.thr) ? dp0 : 0.f;
            dp1 = ((hh >> 16) >= P.thr) ? dp1 : 0.f;
            sacc[i] = p0 * __builtin_fmaf(dp0, P.drop_scale, -dlt);
            sacc[i + 1] = p1 * __builtin_fmaf(dp1, P.drop_scale, -dlt);
          } else {
            sacc[i] = p0 * (dp0 - dlt);
            sacc[i + 1] = p1 * (dp1 - dlt);
          }
        }
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          v4s klo[D / 32], khi[D / 32];
          F.tr_issue(kt, t, ss, klo, khi);
          short8 df;
#pragma unroll
          for (int j = 0; j < 8; ++j) df[j] = cvt16<T>(sacc[8 * ss + j]);
          tr_wait(klo, khi);
#pragma unroll
          for (int dt = 0; dt < D / 32; ++dt)
            dqacc[dt] = mfma<T>(tr_join(klo[dt], khi[dt]), df, dqacc[dt]);
        }
      }
    }
    glds_wait();
    __syncthreads();
  }
  store_row16<T, D>(P.dq + b * P.sdq_b + hd * P.sdq_h + (long)qi * P.sdq_s, dqacc, P.scale, h,
                    P.dval, P.row16, qvalid);
}


// swap a 32-bit value with the neighbouring lane (lane ^ 1) through DPP
__device__ __forceinline__ uint32_t dpp_swap1(uint32_t v) {
  // quad_perm [1, 0, 3, 2]
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
}

// ============================================================================
// backward dK/dV: WG = 4 waves x 32 keys = 128 keys; loop over 32-query tiles
//   S = Q.K^T, dP = dO.V^T (keys on lanes, queries in registers)
//   dV^T += dO^T.(P o Z),  dK^T += Q^T.dS
// The Q / dO tiles and their lse / delta row constants are double-buffered:
// tile i+1 streams into the second LDS buffer (global_load_lds) while tile i
// computes, one vmcnt drain + barrier per tile.
// Occupancy: the dK and dV accumulators (128 VGPRs) plus K fragments (32)
// stay in registers; this WG's V rows (128 x D) live in LDS instead of 32
// more VGPRs, and the query tile is 32 rows, so the kernel fits 256 VGPRs
// without spills -> 2 waves per SIMD (2 WGs per CU, 65 KB LDS each) instead
// of 1 wave per SIMD with every LDS / exp latency exposed.
// Dropout: lanes 2j, 2j+1 hold keys 2j, 2j+1 = the two 16-bit halves of ONE
// hash per query row, so each lane hashes every other query row and the
// pair trades results through DPP (one hash per two elements, as fwd / dQ).
// ============================================================================
// QT: query rows per tile (32, or 64 = half the barriers / DMA issue points
// per unit of work); VREG: this wave's V rows in 32 VGPRs instead of a
// 128-row LDS image (keeps two workgroups per CU at QT = 64).
template <typename T, int D, bool CAUSAL, bool DROP, bool KB, int QT, bool VREG, int NW = 4>
__device__ __forceinline__ void dkdv_body(const AttnParams& P, char* smem) {
  constexpr bool LEAN = D == 128 && VREG;
  constexpr int KR = 32 * NW;  // keys per workgroup
  constexpr int TB = QT * D * 2;
  // one buffer: [Q tile][dO tile][lse2 QT floats][delta QT floats]; then V rows
  constexpr int BUF = 2 * TB + 2 * QT * 4;
  char* vs = smem + 2 * BUF;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5;
  Frag<D> F;
  F.init(lane);
  const int nk = (P.Sk + KR - 1) / KR;
  const int nblk = nk * P.B * P.H;
  const int lid = xcd_remap(blockIdx.x, nblk);
  int bh, kblock;  // causal: low key blocks are the heavy ones
  if constexpr (CAUSAL) {
    lpt_order(lid, nk, P.B * P.H, bh, kblock);
  } else {
    bh = lid / nk;
    kblock = lid % nk;
  }
  const int b = bh / P.H, hd = bh % P.H;
  const uint16_t* qp = P.q + b * P.sq_b + hd * P.sq_h;
  const uint16_t* kp = P.k + b * P.sk_b + hd * P.sk_h;
  const uint16_t* vp = P.v + b * P.sv_b + hd * P.sv_h;
  const uint16_t* dop = P.dout + b * P.so_b + hd * P.so_h;
  int kv_len = P.Sk;
  if (P.kv_lens) kv_len = min(kv_len, P.kv_lens[b]);

  const int wk0 = kblock * KR + w * 32;
  const int ki = wk0 + (lane & 31);
  const bool kvalid = ki < kv_len;
  // per-key additive term of the exp2 argument; -inf masks keys past kv_len
  const float kb2 = !kvalid ? -INFINITY : (KB ? P.kbias[(long)b * P.kb_b + ki] * LOG2E : 0.f);
  short8 kf[D / 16];
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
    if (ki < P.Sk && 16 * s + 8 * h < P.dval)
      kf[s] = *reinterpret_cast<const short8*>(kp + (long)ki * P.sk_s + 16 * s + 8 * h);
    else
      kf[s] = (short8){0, 0, 0, 0, 0, 0, 0, 0};
  }
  // V rows of this WG's 128 keys -> LDS (rows past Sk clamp; those keys are
  // masked), or this wave's 32 rows -> registers
  short8 vf[VREG ? D / 16 : 1];
  if constexpr (VREG) {
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
      if (ki < P.Sk && 16 * s + 8 * h < P.dval)
        vf[s] = *reinterpret_cast<const short8*>(vp + (long)ki * P.sv_s + 16 * s + 8 * h);
      else
        vf[s] = (short8){0, 0, 0, 0, 0, 0, 0, 0};
    }
  } else {
    Glds<D, KR, NW>::load(vp, P.sv_s, kblock * KR, P.Sk, vs, w, lane, P.dval);
  }
  floatx16 dkacc[D / 32], dvacc[D / 32];
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) dkacc[dt][i] = dvacc[dt][i] = 0.f;
  const float sl2 = P.scale * LOG2E;
  const uint32_t cb = DROP ? attn_cb(P, bh) : 0u;

  const int q_begin = CAUSAL ? (kblock * KR / QT) * QT : 0;
  const int ntiles = P.Sq > q_begin ? (P.Sq - q_begin + QT - 1) / QT : 0;
  // row constants of tile qb: loaded BEFORE the tile's DMA is issued (vmcnt
  // retires in order), written to LDS after the compute of the current tile
  float nl = INFINITY, nd = 0.f;
  auto rowconst_load = [&](int qb) {
    if (tid < QT) {
      const int q = qb + tid;
      nl = q < P.Sq ? P.lse[(long)bh * P.Sq + q] * LOG2E : INFINITY;
      nd = q < P.Sq ? P.delta[(long)bh * P.Sq + q] : 0.f;
    }
  };
  auto rowconst_store = [&](char* buf) {
    if (tid < QT) {
      float* c = reinterpret_cast<float*>(buf + 2 * TB);
      c[tid] = nl;
      c[QT + tid] = nd;
    }
  };
#ifdef FX_FA_LAB
  unsigned long long* stp = fa_stamps ? fa_stamps + ((long)blockIdx.x * NW + w) * 128 : nullptr;
  if (stp && lane == 0) stp[0] = (unsigned long long)kblock;
#endif
  FA_ST2(1);
  GldsStream<D, QT, NW> qld, gld;
  qld.init(qp, P.sq_s, P.Sq, w, lane, P.dval);
  gld.init(dop, P.so_s, P.Sq, w, lane, P.dval);
  if (ntiles > 0) {
    rowconst_load(q_begin);
    qld.load(q_begin, smem, lane);
    gld.load(q_begin, smem + TB, lane);
    rowconst_store(smem);
  }
  glds_wait();
  __syncthreads();
  FA_ST2(2);

  for (int it = 0; it < ntiles; ++it) {
    const int qb = q_begin + it * QT;
    const char* cur = smem + (it & 1) * BUF;
    char* nxt = smem + ((it & 1) ^ 1) * BUF;
    const bool more = it + 1 < ntiles;
    if (more) {
      rowconst_load(qb + QT);
      qld.load(qb + QT, nxt, lane);
      gld.load(qb + QT, nxt + TB, lane);
    }
    const char* qt = cur;
    const char* gt = cur + TB;
    const float* lse_s = reinterpret_cast<const float*>(cur + 2 * TB);
    const float* dl_s = lse_s + QT;
    // else: whole tile above this wave's keys, or the wave holds no valid key
    if (wk0 < P.Sk && !(CAUSAL && qb + QT - 1 < wk0)) {
      // one 32-query slice at a time (not interleaved by the compiler: the
      // slices' fp32 tiles would not fit the 2-wave register budget together)
#pragma unroll 1
      for (int t = 0; t < QT / 32; ++t) {
        const int q0 = qb + 32 * t;
        if (CAUSAL && q0 + 31 < wk0) continue;
        uint32_t keep = 0u;  // bit i: element i survives dropout (one VGPR, not 16);
        // hashed before the MFMAs so its temporaries die before the accumulators live
        if (DROP) {
          // registers i, i+1 (i even) are query rows q, q+1 of this lane's key
#pragma unroll
          for (int i = 0; i < 16; i += 2) {
            const int q = qb + 32 * t + crow(i, h);
            const uint32_t mine =
                lowbias32((((uint32_t)(q + (lane & 1))) << 16 | ((uint32_t)ki >> 1)) ^ cb);
            const uint32_t other = dpp_swap1(mine);
            const uint32_t hq = (lane & 1) ? other : mine;   // hash of row q
            const uint32_t hq1 = (lane & 1) ? mine : other;  // hash of row q + 1
            const uint32_t r0 = (lane & 1) ? (hq >> 16) : (hq & 0xffffu);
            const uint32_t r1 = (lane & 1) ? (hq1 >> 16) : (hq1 & 0xffffu);
            keep |= (r0 >= P.thr ? 1u : 0u) << i;
            keep |= (r1 >= P.thr ? 1u : 0u) << (i + 1);
          }
        }
        // causal: only the 32-query slices that cross this wave's keys need
        // the per-element mask; it enters as the S accumulator's initial
        // value (-inf where key > query), before any tile register is live.
        // Keys past kv_len carry kb2 = -inf and query rows past Sq carry
        // lse = +inf, so their p is exp2(-inf) = 0 without a compare.
        floatx16 sacc, dpacc;
#pragma unroll
        for (int i = 0; i < 16; ++i) sacc[i] = dpacc[i] = 0.f;
        if (CAUSAL && __builtin_expect(q0 < wk0 + 31, 0)) {
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if (ki > q0 + crow(i, h)) sacc[i] = -INFINITY;
        }
        if constexpr (LEAN) {
          // D = 128 with V in registers: fragments one k-step ahead only (the
          // compiler would hoist all of them) so the 2-wave budget holds
          short8 qr = F.row(qt, t, 0), gr = F.row(gt, t, 0);
#pragma unroll
          for (int s = 0; s < D / 16; ++s) {
            asm volatile("" ::: "memory");
            short8 nq = qr, ng = gr;
            if (s + 1 < D / 16) {
              nq = F.row(qt, t, s + 1);
              ng = F.row(gt, t, s + 1);
            }
            sacc = mfma<T>(qr, kf[s], sacc);
            dpacc = mfma<T>(gr, vf[s], dpacc);
            qr = nq; gr = ng;
          }
        } else {
#pragma unroll
          for (int s = 0; s < D / 16; ++s) {
            sacc = mfma<T>(F.row(qt, t, s), kf[s], sacc);
            if constexpr (VREG) dpacc = mfma<T>(F.row(gt, t, s), vf[s], dpacc);
            else dpacc = mfma<T>(F.row(gt, t, s), F.row(vs, w, s), dpacc);
          }
        }
        // LEAN: P o Z and dS of the whole slice to 16-bit before the MFMA
        // phase, so the fp32 S / dP tiles die first
        short8 pfa[LEAN ? 2 : 1], dfa[LEAN ? 2 : 1];
        if constexpr (LEAN) {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int ql_ = 32 * t + crow(i, h);
            const float p = fexp2(__builtin_fmaf(sacc[i], sl2, kb2 - lse_s[ql_]));
            if (DROP) {
              const float z = ((keep >> i) & 1u) ? P.drop_scale : 0.f;
              pfa[i >> 3][i & 7] = cvt16<T>(p * z);
              dfa[i >> 3][i & 7] = cvt16<T>(p * (dpacc[i] * z - dl_s[ql_]));
            } else {
              pfa[i >> 3][i & 7] = cvt16<T>(p);
              dfa[i >> 3][i & 7] = cvt16<T>(p * (dpacc[i] - dl_s[ql_]));
            }
          }
        }
        // P o Z (for dV) and dS (for dK) straight to bf16, one 8-row half at a
        // time: no fp32 copies of the tile stay live across the MFMAs
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          short8 pf, df;
          if constexpr (LEAN) {
            pf = pfa[ss];
            df = dfa[ss];
          } else
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int i = 8 * ss + j;
            const int ql_ = 32 * t + crow(i, h);
            const float p = fexp2(__builtin_fmaf(sacc[i], sl2, kb2 - lse_s[ql_]));
            if (DROP) {
              const float z = ((keep >> i) & 1u) ? P.drop_scale : 0.f;
              pf[j] = cvt16<T>(p * z);
              df[j] = cvt16<T>(p * (dpacc[i] * z - dl_s[ql_]));  // dS
            } else {
              pf[j] = cvt16<T>(p);
              df[j] = cvt16<T>(p * (dpacc[i] - dl_s[ql_]));  // dS
            }
          }
          // (issued after P / dS are packed: the register budget of D = 128
          // has no room for the fragments while the tile's fp32 values live)
          v4s glo[D / 32], ghi[D / 32];
          F.tr_issue(gt, t, ss, glo, ghi);
          tr_wait(glo, ghi);
#pragma unroll
          for (int dt = 0; dt < D / 32; ++dt)
            dvacc[dt] = mfma<T>(tr_join(glo[dt], ghi[dt]), pf, dvacc[dt]);
          // the Q fragments only after the dO ones are consumed: D = 128 has
          // no registers for both sets at once
          v4s qlo[D / 32], qhi[D / 32];
          F.tr_issue(qt, t, ss, qlo, qhi);
          tr_wait(qlo, qhi);
#pragma unroll
          for (int dt = 0; dt < D / 32; ++dt)
            dkacc[dt] = mfma<T>(tr_join(qlo[dt], qhi[dt]), df, dkacc[dt]);
        }
      }
    }
    FA_ST2(3 + 2 * it);
    if (more) rowconst_store(nxt);
    glds_wait();
    __syncthreads();
    FA_ST2(4 + 2 * it);
  }
  FA_ST2(126);
  const long krow = b * P.sdk_b + hd * P.sdk_h + (long)ki * P.sdk_s;
  store_row16<T, D>(P.dk + krow, dkacc, P.scale, h, P.dval, P.row16, ki < P.Sk);
  store_row16<T, D>(P.dv + krow, dvacc, 1.f, h, P.dval, P.row16, ki < P.Sk);
  FA_ST2(127);
}

#ifdef FX_FA_LAB
#include FX_FA_LAB  // tools/fa_lab/fa_wave64.inc (lab builds only)
#endif


template <typename T, int D, bool CAUSAL, bool DROP, bool KB>
__global__ __launch_bounds__(256, 2) void fa_bwd_dkdv_kernel(AttnParams P) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  dkdv_body<T, D, CAUSAL, DROP, KB, FA_DKDV_QT, false>(P, smem);
}
template <typename T, int D, bool CAUSAL, bool DROP, bool KB, int NW = 4>
__global__ __launch_bounds__(64 * NW, 2) void fa_bwd_dkdv_q64v_kernel(AttnParams P) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // launched for D <= 96 only (D = 128 has no registers for V; it would spill)
  if constexpr (D <= 96) dkdv_body<T, D, CAUSAL, DROP, KB, 64, true, NW>(P, smem);
}

AttnParams make_params(const void* q, const void* k, const void* v, const long* qs,
                       const long* ks, const long* vs, int B, int H, int Sq, int Sk, float scale,
                       float p, uint64_t key) {
  AttnParams P{};
  P.q = (const uint16_t*)q;
  P.k = (const uint16_t*)k;
  P.v = (const uint16_t*)v;
  P.sq_b = qs[0]; P.sq_s = qs[1]; P.sq_h = qs[2];
  P.sk_b = ks[0]; P.sk_s = ks[1]; P.sk_h = ks[2];
  P.sv_b = vs[0]; P.sv_s = vs[1]; P.sv_h = vs[2];
  P.B = B; P.H = H; P.Sq = Sq; P.Sk = Sk;
  P.scale = scale;
  P.klo = (uint32_t)(key & 0xffffffffu);
  P.khi = (uint32_t)(key >> 32);
  P.thr = (uint32_t)(p * 65536.0f + 0.5f);
  P.drop_scale = p < 1.f ? 1.f / (1.f - p) : 0.f;
  P.salt = p > 0.f ? g_fx_dropout_salt : nullptr;
  return P;
}

}  // namespace

// Launch with dynamic LDS; above 64 KiB the kernel must opt in (up to the
// 160 KiB of a CU).
static void fa_launch(void (*kernel)(AttnParams), int grid, size_t smem, hipStream_t st,
                      const AttnParams& P, int threads = 256) {
  if (smem > 65536)
    (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)smem);
  hipLaunchKernelGGL(kernel, dim3(grid), dim3(threads), smem, st, P);
}

// Forward workgroup width: NW waves x 32 queries share one K/V tile stream
// (FLEETX_FA_FWD_WAVES = 4 or 8; see fwd_waves()).
template <typename T, int D, int NW>
static void fa_fwd_dispatch(bool causal, bool drop, bool kbias, int grid, size_t smem,
                            hipStream_t st, const AttnParams& P) {
  auto go = [&](void (*k)(AttnParams)) { fa_launch(k, grid, smem, st, P, 64 * NW); };
  if (causal) {
    if (drop) go(fa_fwd_kernel<T, D, true, true, false, NW>);
    else go(fa_fwd_kernel<T, D, true, false, false, NW>);
  } else if (kbias) {
    if (drop) go(fa_fwd_kernel<T, D, false, true, true, NW>);
    else go(fa_fwd_kernel<T, D, false, false, true, NW>);
  } else {
    if (drop) go(fa_fwd_kernel<T, D, false, true, false, NW>);
    else go(fa_fwd_kernel<T, D, false, false, false, NW>);
  }
}

static int tile_dim(int d) { return d <= 64 ? 64 : (d <= 96 ? 96 : 128); }

// Waves per workgroup (32 rows each) along a sequence of n rows for the
// 96-wide tile: 3 when that leaves fewer idle waves than 4.  ViT-g's 257
// tokens are 9 row tiles: 3 x 3 waves with none idle, against 3 x 4 with 3
// idle waves holding the last workgroup's slots for a single row.
static int waves_for(int n) {
  const int tiles = (n + 31) / 32;
  const int idle3 = (n + 95) / 96 * 3 - tiles, idle4 = (n + 127) / 128 * 4 - tiles;
  return idle3 < idle4 ? 3 : 4;
}

// FLEETX_FA_PAIR=0: one causal query block per workgroup (LPT order) instead of pairs
static bool fa_pair_grid() {
  static const bool on = [] {
    const char* e = getenv("FLEETX_FA_PAIR");
    return !(e && atoi(e) == 0);
  }();
  return on;
}

#ifdef FX_FA_LAB
// Lab variants (tools/fa_lab): FLEETX_FA_DKDV64 (dK/dV with 64 keys per wave),
// FLEETX_FA_DKDV_VREG (D = 128 dK/dV with V in registers), FLEETX_FA_DQ64 (dQ
// with 64 queries per wave), or the fx_fa_set_* switches (1 on, 0 off, < 0
// re-reads the environment)
static int g_dkdv64 = -1, g_dkdv_vreg = -1, g_dq64 = -1;
static bool lab_flag(int& g, const char* name) {
  if (g < 0) {
    const char* e = getenv(name);
    g = e ? (atoi(e) != 0) : 0;
  }
  return g != 0;
}
static bool dkdv64() { return lab_flag(g_dkdv64, "FLEETX_FA_DKDV64"); }
static bool dkdv_vreg() { return lab_flag(g_dkdv_vreg, "FLEETX_FA_DKDV_VREG"); }
static bool dq64() { return lab_flag(g_dq64, "FLEETX_FA_DQ64"); }
extern "C" int fx_fa_lab() { return 1; }
extern "C" void fx_fa_set_dkdv64(int on) { g_dkdv64 = on < 0 ? -1 : (on != 0); }
extern "C" void fx_fa_set_dkdv_vreg(int on) { g_dkdv_vreg = on < 0 ? -1 : (on != 0); }
extern "C" void fx_fa_set_dq64(int on) { g_dq64 = on < 0 ? -1 : (on != 0); }
extern "C" int fx_fa_set_stamps(void* p) {
  return hipMemcpyToSymbol(HIP_SYMBOL(fa_stamps), &p, sizeof(p)) == hipSuccess ? 1 : 0;
}
#else
extern "C" int fx_fa_set_stamps(void*) { return 0; }  // production build: no stamps
extern "C" int fx_fa_lab() { return 0; }  // production build: no lab variants
extern "C" void fx_fa_set_dkdv64(int) {}
extern "C" void fx_fa_set_dkdv_vreg(int) {}
extern "C" void fx_fa_set_dq64(int) {}
#endif

static int fwd_waves() {
  static int nw = [] {
    const char* e = getenv("FLEETX_FA_FWD_WAVES");
    const int v = e ? atoi(e) : FA_FWD_WAVES_DEFAULT;
    return v == 8 ? 8 : 4;
  }();
  return nw;
}

#define FA_DISPATCH_D(KERNEL, DD, causal, drop, kbias, grid, smem, st, P)         \
  do {                                                                          \
    if (causal) {                                                               \
      if (drop) fa_launch(KERNEL<T, DD, true, true, false>, grid, smem, st, P); \
      else fa_launch(KERNEL<T, DD, true, false, false>, grid, smem, st, P);     \
    } else if (kbias) {                                                         \
      if (drop) fa_launch(KERNEL<T, DD, false, true, true>, grid, smem, st, P); \
      else fa_launch(KERNEL<T, DD, false, false, true>, grid, smem, st, P);     \
    } else {                                                                    \
      if (drop) fa_launch(KERNEL<T, DD, false, true, false>, grid, smem, st, P); \
      else fa_launch(KERNEL<T, DD, false, false, false>, grid, smem, st, P);     \
    }                                                                           \
  } while (0)
// one tile width with NW waves per workgroup (block size 64 NW)
#define FA_DISPATCH_NW(KERNEL, DD, NW, causal, drop, kbias, grid, smem, st, P)                  \
  do {                                                                                        \
    if (causal) {                                                                             \
      if (drop) fa_launch(KERNEL<T, DD, true, true, false, NW>, grid, smem, st, P, 64 * NW);  \
      else fa_launch(KERNEL<T, DD, true, false, false, NW>, grid, smem, st, P, 64 * NW);      \
    } else if (kbias) {                                                                       \
      if (drop) fa_launch(KERNEL<T, DD, false, true, true, NW>, grid, smem, st, P, 64 * NW);  \
      else fa_launch(KERNEL<T, DD, false, false, true, NW>, grid, smem, st, P, 64 * NW);      \
    } else {                                                                                  \
      if (drop) fa_launch(KERNEL<T, DD, false, true, false, NW>, grid, smem, st, P, 64 * NW); \
      else fa_launch(KERNEL<T, DD, false, false, false, NW>, grid, smem, st, P, 64 * NW);     \
    }                                                                                         \
  } while (0)
// key bias is only instantiated for non-causal attention (BERT-style padding
// masks); causal + bias is rejected by the launchers.
#define FA_DISPATCH(KERNEL, D, causal, drop, kbias, grid, smem, st, P)                  \
  do {                                                                                  \
    if (D == 128) FA_DISPATCH_D(KERNEL, 128, causal, drop, kbias, grid, smem, st, P);   \
    else if (D == 96) FA_DISPATCH_D(KERNEL, 96, causal, drop, kbias, grid, smem, st, P); \
    else FA_DISPATCH_D(KERNEL, 64, causal, drop, kbias, grid, smem, st, P);             \
  } while (0)

// every output row starts 16-byte aligned (store_row16's 16-byte stores);
// FLEETX_FA_ROW16=0 forces the 8-byte fallback (tests/test_kernels_gpu.py)
static bool rows16(const void* base, const long* s) {
  const char* e = getenv("FLEETX_FA_ROW16");
  if (e && atoi(e) == 0) return false;
  return (reinterpret_cast<uintptr_t>(base) & 15) == 0 && s[0] % 8 == 0 && s[1] % 8 == 0 &&
         s[2] % 8 == 0;
}

// strides arrays are {batch, seq, head} in elements; head dim contiguous.
// kbias: optional [B, kb_stride] float additive key bias; kb_stride must be
// >= round_up(Sk, 128) (tiles read whole 64-key groups).
template <typename T>
static int flash_fwd_t(const void* q, const void* k, const void* v, void* out, float* lse,
                            const long* qs, const long* ks, const long* vs, const long* os,
                            const int* kv_lens, const float* kbias, long kb_stride, int B, int H,
                            int Sq, int Sk, int D, int causal, float scale, float p, uint64_t key,
                            hipStream_t st) {
  // D is the head dim of the tensors; the kernel runs the smallest tile width
  // >= D (64 / 96 / 128) with the columns past D read as zeros
  if (D % 8 || D <= 0 || D > 128) return -1;
  if (kbias && (causal || kb_stride < ((Sk + 127) / 128) * 128)) return -2;
  AttnParams P = make_params(q, k, v, qs, ks, vs, B, H, Sq, Sk, scale, p, key);
  P.dval = D;
  D = tile_dim(D);
  P.out = (uint16_t*)out;
  P.lse = lse;
  P.kv_lens = kv_lens;
  P.kbias = kbias;
  P.kb_b = kb_stride;
  P.so_b = os[0]; P.so_s = os[1]; P.so_h = os[2];
  P.row16 = rows16(out, os);
  const int nw = D == 96 ? waves_for(Sq) : fwd_waves();
  const int nq = (Sq + 32 * nw - 1) / (32 * nw);
  P.pair = causal && fa_pair_grid() ? 1 : 0;
  const int grid = (P.pair ? (nq + 1) / 2 : nq) * B * H;
  const size_t smem = 4 * 64 * D * 2;
  const bool drop = p > 0.f, kb = kbias != nullptr;
  if (nw == 8) {
    if (D == 128) fa_fwd_dispatch<T, 128, 8>(causal, drop, kb, grid, smem, st, P);
    else fa_fwd_dispatch<T, 64, 8>(causal, drop, kb, grid, smem, st, P);
  } else {
    if (D == 128) fa_fwd_dispatch<T, 128, 4>(causal, drop, kb, grid, smem, st, P);
    else if (D == 96 && nw == 3) fa_fwd_dispatch<T, 96, 3>(causal, drop, kb, grid, smem, st, P);
    else if (D == 96) fa_fwd_dispatch<T, 96, 4>(causal, drop, kb, grid, smem, st, P);
    else fa_fwd_dispatch<T, 64, 4>(causal, drop, kb, grid, smem, st, P);
  }
  return 0;
}

// o/dout share strides `os`; dq uses `dqs`; dk/dv share `dks`.
template <typename T>
static int flash_bwd_t(const void* q, const void* k, const void* v, const void* o,
                            const void* dout, const float* lse, float* delta, void* dq, void* dk,
                            void* dv, const long* qs, const long* ks, const long* vs,
                            const long* os, const long* dqs, const long* dks, const int* kv_lens,
                            const float* kbias, long kb_stride, int B, int H,
                            int Sq, int Sk, int D, int causal, float scale, float p, uint64_t key,
                            hipStream_t st) {
  if (D % 8 || D <= 0 || D > 128) return -1;
  if (kbias && (causal || kb_stride < ((Sk + 127) / 128) * 128)) return -2;
  AttnParams P = make_params(q, k, v, qs, ks, vs, B, H, Sq, Sk, scale, p, key);
  P.dval = D;
  D = tile_dim(D);
  P.o = (const uint16_t*)o;
  P.dout = (const uint16_t*)dout;
  P.lse = const_cast<float*>(lse);
  P.delta = delta;
  P.dq = (uint16_t*)dq;
  P.dk = (uint16_t*)dk;
  P.dv = (uint16_t*)dv;
  P.kv_lens = kv_lens;
  P.kbias = kbias;
  P.kb_b = kb_stride;
  P.so_b = os[0]; P.so_s = os[1]; P.so_h = os[2];
  P.sdk_b = dks[0]; P.sdk_s = dks[1]; P.sdk_h = dks[2];
  P.sdq_b = dqs[0]; P.sdq_s = dqs[1]; P.sdq_h = dqs[2];
  P.row16 = rows16(dq, dqs) && rows16(dk, dks) && rows16(dv, dks);
  const bool drop = p > 0.f, kb = kbias != nullptr;
  {
    const size_t smem = 4 * 64 * D * 2;
    if (D == 96 && waves_for(Sq) == 3) {
      const int nq = (Sq + 95) / 96;
      FA_DISPATCH_NW(fa_bwd_dq_kernel, 96, 3, causal, drop, kb, nq * B * H, smem, st, P);
#ifdef FX_FA_LAB
    } else if (D == 128 && dq64()) {
      FA_DISPATCH_D(fa_bwd_dq64_kernel, 128, causal, drop, kb, (Sq + 255) / 256 * B * H, smem,
                    st, P);
#endif
    } else {
      const int nq = (Sq + 127) / 128;
      FA_DISPATCH(fa_bwd_dq_kernel, D, causal, drop, kb, nq * B * H, smem, st, P);
    }
  }
  {
    // double-buffered Q/dO tiles + row constants, then the WG's V rows
    // D <= 96: 64-query tiles with V in registers (bwd 0.150 -> 0.144 ms at
    // B8 S1024 H16 D64, profiles/r3_dkdv/); D = 128 has no 32 VGPRs to spare.
    const int nk = (Sk + 127) / 128;
    if (D == 96 && waves_for(Sk) == 3) {
      const size_t smem = 2 * (2 * 64 * D * 2 + 2 * 64 * 4);
      FA_DISPATCH_NW(fa_bwd_dkdv_q64v_kernel, 96, 3, causal, drop, kb, (Sk + 95) / 96 * B * H,
                     smem, st, P);
    } else if (D <= 96) {
      const size_t smem = 2 * (2 * 64 * D * 2 + 2 * 64 * 4);
      FA_DISPATCH(fa_bwd_dkdv_q64v_kernel, D, causal, p > 0.f, kbias != nullptr, nk * B * H,
                  smem, st, P);
#ifdef FX_FA_LAB
    } else if (dkdv_vreg()) {
      // D = 128, V in registers: no V image in LDS
      const size_t smem = 2 * (2 * FA_DKDV_V128_QT * D * 2 + 2 * FA_DKDV_V128_QT * 4);
      FA_DISPATCH_D(fa_bwd_dkdv_v128_kernel, 128, causal, p > 0.f, kbias != nullptr, nk * B * H,
                    smem, st, P);
    } else if (dkdv64()) {
      // 64 keys per wave, one workgroup of 256 keys per CU
      const size_t smem = 2 * (2 * FA_DKDV64_QT * D * 2 + 2 * FA_DKDV64_QT * 4) + 256 * D * 2;
      FA_DISPATCH_D(fa_bwd_dkdv_k64_kernel, 128, causal, p > 0.f, kbias != nullptr,
                    (Sk + 255) / 256 * B * H, smem, st, P);
#endif
    } else {
      const size_t smem = 2 * (2 * FA_DKDV_QT * D * 2 + 2 * FA_DKDV_QT * 4) + 128 * D * 2;
      FA_DISPATCH(fa_bwd_dkdv_kernel, D, causal, p > 0.f, kbias != nullptr, nk * B * H, smem,
                  st, P);
    }
  }
  return 0;
}

// dt: 0 = bf16, 1 = fp16 (inputs, outputs and the MFMA operand type)
extern "C" int fx_flash_fwd(int dt, const void* q, const void* k, const void* v, void* out,
                            float* lse, const long* qs, const long* ks, const long* vs,
                            const long* os, const int* kv_lens, const float* kbias,
                            long kb_stride, int B, int H, int Sq, int Sk, int D, int causal,
                            float scale, float p, uint64_t key, hipStream_t st) {
  if (dt == 0)
    return flash_fwd_t<bf16>(q, k, v, out, lse, qs, ks, vs, os, kv_lens, kbias, kb_stride, B, H,
                             Sq, Sk, D, causal, scale, p, key, st);
  if (dt == 1)
    return flash_fwd_t<f16>(q, k, v, out, lse, qs, ks, vs, os, kv_lens, kbias, kb_stride, B, H,
                            Sq, Sk, D, causal, scale, p, key, st);
  return -3;
}

extern "C" int fx_flash_bwd(int dt, const void* q, const void* k, const void* v, const void* o,
                            const void* dout, const float* lse, float* delta, void* dq, void* dk,
                            void* dv, const long* qs, const long* ks, const long* vs,
                            const long* os, const long* dqs, const long* dks, const int* kv_lens,
                            const float* kbias, long kb_stride, int B, int H, int Sq, int Sk,
                            int D, int causal, float scale, float p, uint64_t key,
                            hipStream_t st) {
  if (dt == 0)
    return flash_bwd_t<bf16>(q, k, v, o, dout, lse, delta, dq, dk, dv, qs, ks, vs, os, dqs, dks,
                             kv_lens, kbias, kb_stride, B, H, Sq, Sk, D, causal, scale, p, key,
                             st);
  if (dt == 1)
    return flash_bwd_t<f16>(q, k, v, o, dout, lse, delta, dq, dk, dv, qs, ks, vs, os, dqs, dks,
                            kv_lens, kbias, kb_stride, B, H, Sq, Sk, D, causal, scale, p, key,
                            st);
  return -3;
}
