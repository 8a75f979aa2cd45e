// Shared definitions of the gfx950 GEMM kernels (gemm.hip, gemm5.hip).
#pragma once
#include <stdint.h>

#include "fx_common.h"

namespace fxg {

enum { LAY_KC = 0, LAY_MC = 1 };
enum { EPI_STORE = 0, EPI_BIAS_GELU = 1, EPI_DGELU = 2, EPI_F32 = 3, EPI_BIAS_GELU_ERF = 4,
       EPI_DGELU_ERF = 5,
       // weight gradient stored in 16 bits (fp32 accumulation, beta 0): the
       // bf16 gradient storage of Distributed.comm.grad_dtype
       EPI_F32B = 6,
       // fx_gemm only: EPI_F32B with C stored transposed (GemmParams::ctr)
       EPI_F32BT = 7 };

// the fp32-accumulating weight-gradient epilogues (split-K, norm partials)
constexpr bool epi_wgrad(int e) { return e == EPI_F32 || e == EPI_F32B; }

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int PIECE = 16384;            // bytes per staged piece (128 rows x 64 k x 2 B)
constexpr int TILE_BYTES = 4 * PIECE;   // one K-tile of A and B
constexpr int SMEM = 2 * TILE_BYTES;    // double buffer: 128 KiB

struct GemmParams {
  const uint16_t* A;
  const uint16_t* B;
  void* C;
  const uint16_t* bias;
  uint16_t* aux;
  long lda, ldb, ldc, ldaux;
  int M, N, K;
  int tiles_m, tiles_n;
  int beta;
  int gm;  // tiles per M-group of the block order (L2 reuse)
  unsigned long long* dbg;  // tools/gemm_lab timeline stamps (FX_GEMM_STAMP builds only)
  // EPI_F32 (gemm5 only): per-wave sums of squares of the stored values,
  // sq[4 * blockIdx.x + wave] -- the gradient-norm partials of a weight
  // gradient, taken from the accumulators instead of re-reading main_grad
  float* sq;
  // EPI_F32 split-K (gemm5): this launch covers tiles [tile0, tile0 + gridDim.x / ksplit);
  // with ksplit > 1 each tile's K range is cut into ksplit slices whose fp32
  // partial tiles go to ws[(local tile * ksplit + slice) * TILE * TILE]
  int tile0;
  int ksplit;
  float* ws;
  // persistent launch (gemm5, 16-bit outputs): gridDim.x resident workgroups
  // pull tiles from the 8 per-XCD queues of ring slot `qslot` (int 32 x for
  // XCD x, int 256 the finish count; the last workgroup to finish re-zeroes
  // the slot); -1 = one workgroup per tile
  int qslot;
  // EPI_F32B: 1 = this launch stores the 16-bit gradient, 0 = fp32 split-K
  // partial slabs (the combine stores the 16-bit result)
  int out16;
  // XCD rectangles (gemm5): > 0 = the tile grid is cut into xm x (8 / xm)
  // equal rectangles, rectangle r = tile ids [r * T / 8, (r + 1) * T / 8) = the
  // range xcd_remap / the persistent queues deal to XCD r; the gm order runs
  // inside each rectangle.  0 = the gm order over the whole grid.
  int xm;
  // EPI_F32B: 1 = C[m][n] is stored at C + n * ldc + m (the transposed
  // product of a wide weight gradient, fx_gemm EPI_F32BT); unsplit launches only
  int ctr;
};

__device__ __forceinline__ int xcd_remap(int bid, int nblk) {
  const int xcd = bid & 7, pos = bid >> 3, q = nblk >> 3, r = nblk & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + pos;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}

}  // namespace fxg
