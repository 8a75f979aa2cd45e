// Layout kernels: 16-bit 2-D transpose through LDS.
//
// Used to hand hipBLASLt the weight-gradient GEMM in its fastest operand
// layout.  dW[N,K] = dy[M,N]^T x[M,K] reduces over the token axis M, which is
// the *slow* axis of both row-major activations; hipBLASLt's "NT" kernels for
// that case sustain ~1.0 PFLOP/s on gfx950 while the "TN" kernels (reduction
// axis contiguous in both operands) reach ~1.35 PFLOP/s with fp32 accumulate
// (tools/bench_gemm.py).  Transposing dy and x to token-contiguous copies
// costs one read + one write of each at HBM speed, well under the GEMM saving.
//
// Tile: 64 x 256 elements per 256-thread workgroup (4 wave64s).  Loads are
// 16-byte vectors along the source row (8 elements), eight per thread; the
// tile is staged in LDS with a 2-element row pad, then each thread gathers 8
// source rows of one source column into one 16-byte store along the
// destination row.  R, C, ldx, ldy are multiples of 8 (checked on the host),
// so only whole 8-element chunks are ever bounds-checked.
//
// With ``part`` set the kernel also emits the fp32 column sums of its tile
// (part[tile_row][col]) -- the bias gradient of the GEMM whose dy is being
// transposed, for free while the tile is in registers; coltile_finalize
// reduces the tile rows.
#include "fx_common.h"

namespace {

// Tile: 64 source rows x 256 source columns per 256-thread workgroup.  A
// 64 x 64 tile reads 128-byte row pieces and measured 2.0-2.9 TB/s on the
// transformer shapes; 512-byte row pieces and 8 loads in flight per thread
// (16 KiB per wave) keep HBM streaming (tools/bench_gemm.py transpose_dy_hip).
constexpr int TR = 64, TC = 256;
constexpr int TPAD = 2;  // row stride 129 dwords: the 8-row column gathers spread over banks

template <typename T, bool COLSUM>
__global__ __launch_bounds__(256) void transpose16_kernel(const uint16_t* __restrict__ x,
                                                          uint16_t* __restrict__ y,
                                                          float* __restrict__ part, int R, int C,
                                                          long ldx, long ldy, int tiles_c) {
  __shared__ uint16_t t[TR][TC + TPAD];
  const int bc = blockIdx.x % tiles_c;
  const int br = blockIdx.x / tiles_c;
  const int r0 = br * TR, c0 = bc * TC;
  const int tid = threadIdx.x;
  uint4 v[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int r = (tid >> 5) + 8 * k, cc = (tid & 31) * 8;
    if (r0 + r < R && c0 + cc < C)
      v[k] = *reinterpret_cast<const uint4*>(x + (long)(r0 + r) * ldx + c0 + cc);
    else
      v[k] = make_uint4(0, 0, 0, 0);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int r = (tid >> 5) + 8 * k, cc = (tid & 31) * 8;
    uint32_t* d = reinterpret_cast<uint32_t*>(&t[r][cc]);
    d[0] = v[k].x;
    d[1] = v[k].y;
    d[2] = v[k].z;
    d[3] = v[k].w;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int id = tid + k * 256;
    const int c = id >> 3, rr = (id & 7) * 8;  // 8 lanes write one 128-byte output row piece
    uint16_t h[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] = t[rr + i][c];
    if (c0 + c < C && r0 + rr < R)
      *reinterpret_cast<uint4*>(y + (long)(c0 + c) * ldy + r0 + rr) =
          *reinterpret_cast<const uint4*>(h);
    if constexpr (COLSUM) {
      // rows outside R were zero-filled above; the 8 lanes of a column are adjacent
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) s += Elt<T>::to_f(h[i]);
      s += __shfl_xor(s, 1, 64);
      s += __shfl_xor(s, 2, 64);
      s += __shfl_xor(s, 4, 64);
      if ((id & 7) == 0 && c0 + c < C) part[(long)br * C + c0 + c] = s;
    }
  }
}

}  // namespace

extern "C" int fx_transpose16(int dtype, const void* x, void* y, float* part, int R, int C,
                              long ldx, long ldy, hipStream_t st) {
  if ((R | C) & 7 || ldx & 7 || ldy & 7) return -1;
  if (R == 0 || C == 0) return 0;
  const int tiles_c = (C + TC - 1) / TC;
  const long blocks = (long)tiles_c * ((R + TR - 1) / TR);
  if (blocks > 0x7fffffffL) return -2;
  const uint16_t* xs = reinterpret_cast<const uint16_t*>(x);
  uint16_t* ys = reinterpret_cast<uint16_t*>(y);
  const dim3 grid((unsigned)blocks), block(256);
  if (!part)
    transpose16_kernel<bf16, false><<<grid, block, 0, st>>>(xs, ys, part, R, C, ldx, ldy, tiles_c);
  else if (dtype == 0)
    transpose16_kernel<bf16, true><<<grid, block, 0, st>>>(xs, ys, part, R, C, ldx, ldy, tiles_c);
  else
    transpose16_kernel<f16, true><<<grid, block, 0, st>>>(xs, ys, part, R, C, ldx, ldy, tiles_c);
  return 0;
}
