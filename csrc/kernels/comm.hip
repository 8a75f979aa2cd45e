// Intra-node one-shot all-reduce over IPC-mapped peer memory (xGMI).
//
// the latency-bound tensor-parallel collectives (the
// three ParallelCrossEntropy all-reduces, `hybrid_model.py:799,822-824`; the
// per-layer decode all-reduces of an mp>1 InferenceEngine) move 4 KiB - 256 KiB.
// A ring all-reduce pays 2(n-1) link hops of latency for them; on MI355X the
// peers of a node are fully connected by point-to-point xGMI links, so ONE
// hop suffices: every rank pushes its whole payload into every peer's receive
// area and reduces what it received.
//
// Protocol ("data is the flag", cdna_hip_programming.md §6 Guideline 16, R2,
// at system scope):
//  * the payload travels as 8-byte granules {tag = epoch (hi 32), 4 data bytes
//    (lo 32)} written by ONE aligned 64-bit system-scope atomic store into the
//    peer's receive slot [parity][src][granule] -- no separate flag, no fence;
//  * the receiver polls its OWN (local HBM, uncached) slot granule by granule
//    with relaxed system-scope loads until the tag equals this call's epoch;
//  * epochs are per-block device counters (graph-replay safe: nothing is baked
//    into the launch); the grid is always FX_COMM_MAX_BLOCKS blocks, so every
//    block's epoch equals the number of calls so far, on every rank;
//  * receive slots alternate by epoch parity: a rank can never be two calls
//    ahead of a peer (call k+1 needs the peer's call-k+1 data), so parity k
//    is never overwritten while a peer still reads it;
//  * reduction runs in rank order 0..world-1 on every rank, so all ranks get
//    bitwise-identical results (tensor-parallel replicas stay in lock-step);
//  * every spin is bounded (`timeout` ticks of the 100 MHz s_memrealtime
//    clock, FLEETX_ONESHOT_TIMEOUT_S on the host, default 120 s so a peer's
//    checkpoint save or data stall does not trip it); a timeout never
//    produces a normal-looking result: the affected outputs are written as
//    NaN (so the loss / found-inf / NaN guard see it on the next step) and
//    *err is set, which the engine reads at every logging sync and raises;
//    while *err is set later calls do not spin at all (they see it at entry),
//    and the optimizer folds it into found_inf so the step is skipped.
//    The protocol itself survives a timeout: the late peer still finds this
//    rank's pushed granules of that call, and the next call uses the other
//    parity, so only the timed-out call's output is lost.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fx_common.h"

namespace {

constexpr int FX_COMM_MAX_WORLD = 8;
constexpr int FX_COMM_THREADS = 512;
constexpr int FX_COMM_MAX_BLOCKS = 64;

struct PeerTable {
  unsigned long long* recv[FX_COMM_MAX_WORLD];  // receive base of every rank (own included)
};

typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned int gu32;

__device__ __forceinline__ void put_granule(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store((gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ unsigned long long get_granule(const unsigned long long* p) {
  return __hip_atomic_load((gu64*)p,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// 4 payload bytes <-> 1 fp32 or 2 x 16-bit values
template <typename T>
struct Pack;
template <>
struct Pack<float> {
  static constexpr int PER = 1;
  __device__ static uint32_t load(const float* x, long i, long n) {
    return i < n ? __float_as_uint(x[i]) : 0u;
  }
  __device__ static void unpack(uint32_t w, float (&v)[2]) { v[0] = __uint_as_float(w); v[1] = 0.f; }
  __device__ static void store(float* y, long i, long n, const float (&v)[2]) {
    if (i < n) y[i] = v[0];
  }
};
template <typename T16>
struct Pack16 {
  static constexpr int PER = 2;
  __device__ static uint32_t load(const T16* x, long i, long n) {
    const uint16_t* u = reinterpret_cast<const uint16_t*>(x);
    const uint32_t lo = 2 * i < n ? u[2 * i] : 0u;
    const uint32_t hi = 2 * i + 1 < n ? u[2 * i + 1] : 0u;
    return lo | (hi << 16);
  }
  __device__ static void unpack(uint32_t w, float (&v)[2]) {
    v[0] = Elt<T16>::to_f((uint16_t)(w & 0xffff));
    v[1] = Elt<T16>::to_f((uint16_t)(w >> 16));
  }
  __device__ static void store(T16* y, long i, long n, const float (&v)[2]) {
    uint16_t* u = reinterpret_cast<uint16_t*>(y);
    if (2 * i < n) u[2 * i] = Elt<T16>::from_f(v[0]);
    if (2 * i + 1 < n) u[2 * i + 1] = Elt<T16>::from_f(v[1]);
  }
};
template <>
struct Pack<bf16> : Pack16<bf16> {};
template <>
struct Pack<f16> : Pack16<f16> {};

template <typename T, int OP>  // OP 0 = sum, 1 = max
__global__ __launch_bounds__(FX_COMM_THREADS) void ll_allreduce_kernel(
    const T* in, T* out, long n, int rank, int world, PeerTable pt, unsigned int* epochs,
    unsigned int* err, long slot, unsigned long long timeout) {
  __shared__ unsigned int s_epoch, s_err;
  const int b = blockIdx.x;
  if (threadIdx.x == 0) {
    s_epoch = epochs[b] + 1u;
    // a peer already timed out (dead or stalled): do not spin again -- every
    // granule not yet present becomes NaN at once
    s_err = __hip_atomic_load((gu32*)err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  const unsigned int e = s_epoch;
  const int par = e & 1;
  const long ng = (n + Pack<T>::PER - 1) / Pack<T>::PER;
  const long per_blk = (ng + gridDim.x - 1) / gridDim.x;
  const long g0 = (long)b * per_blk, g1 = min(ng, g0 + per_blk);
  const unsigned long long tag = (unsigned long long)e << 32;

  // 1) push this rank's granules into every peer's slot [par][rank]
  for (long g = g0 + threadIdx.x; g < g1; g += blockDim.x) {
    const unsigned long long v = tag | Pack<T>::load(in, g, n);
#pragma unroll
    for (int p = 0; p < FX_COMM_MAX_WORLD; ++p)
      if (p < world && p != rank)
        put_granule(pt.recv[p] + ((long)(par * FX_COMM_MAX_WORLD + rank)) * slot + g, v);
  }
  // 2) reduce in rank order; poll every peer granule until its tag is ours
  const unsigned long long* mine = pt.recv[rank];
  bool timed_out = s_err != 0u;
  for (long g = g0 + threadIdx.x; g < g1; g += blockDim.x) {
    float acc[2] = {0.f, 0.f};
    bool lost = false;
    for (int p = 0; p < world; ++p) {
      uint32_t w;
      if (p == rank) {
        w = Pack<T>::load(in, g, n);
      } else {
        const unsigned long long* src = mine + ((long)(par * FX_COMM_MAX_WORLD + p)) * slot + g;
        unsigned long long x = get_granule(src);
        if ((x >> 32) != e && !timed_out) {
          const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
          do {
            __builtin_amdgcn_s_sleep(1);
            x = get_granule(src);
            if (__builtin_amdgcn_s_memrealtime() - t0 > timeout) {
              timed_out = true;
              break;
            }
          } while ((x >> 32) != e);
        }
        if ((x >> 32) != e) lost = true;
        w = (uint32_t)x;
      }
      float v[2];
      Pack<T>::unpack(w, v);
      if (p == 0) {
        acc[0] = v[0];
        acc[1] = v[1];
      } else if (OP == 0) {
        acc[0] += v[0];
        acc[1] += v[1];
      } else {
        acc[0] = fmaxf(acc[0], v[0]);
        acc[1] = fmaxf(acc[1], v[1]);
      }
    }
    if (lost) acc[0] = acc[1] = __builtin_nanf("");
    Pack<T>::store(out, g, n, acc);
  }
  if (timed_out)
    __hip_atomic_store((gu32*)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (threadIdx.x == 0) epochs[b] = e;
}

template <typename T, int OP>
void launch(const void* in, void* out, long n, int rank, int world, const PeerTable& pt,
            unsigned int* epochs, unsigned int* err, long slot, unsigned long long timeout,
            int blocks, hipStream_t s) {
  hipLaunchKernelGGL((ll_allreduce_kernel<T, OP>), dim3(blocks), dim3(FX_COMM_THREADS), 0, s,
                     (const T*)in, (T*)out, n, rank, world, pt, epochs, err, slot, timeout);
}

}  // namespace

extern "C" {

int fx_comm_max_world() { return FX_COMM_MAX_WORLD; }
int fx_comm_max_blocks() { return FX_COMM_MAX_BLOCKS; }

// Receive area of `slot_granules` granules per (parity, source): uncached device
// memory (remote xGMI stores land in HBM; the local L2 must not serve stale
// granules), zeroed (tag 0 is never a live epoch).
void* fx_comm_alloc(long slot_granules) {
  void* p = nullptr;
  const size_t bytes = (size_t)2 * FX_COMM_MAX_WORLD * slot_granules * 8;
  if (hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached) != hipSuccess) return nullptr;
  if (hipMemset(p, 0, bytes) != hipSuccess) return nullptr;
  if (hipDeviceSynchronize() != hipSuccess) return nullptr;
  return p;
}

int fx_comm_free(void* p) { return (int)hipFree(p); }

int fx_comm_ipc_handle(void* p, char* out64) {
  hipIpcMemHandle_t h;
  const hipError_t r = hipIpcGetMemHandle(&h, p);
  if (r != hipSuccess) return (int)r;
  for (int i = 0; i < HIP_IPC_HANDLE_SIZE; ++i) out64[i] = h.reserved[i];
  return 0;
}

void* fx_comm_ipc_open(const char* in64) {
  hipIpcMemHandle_t h;
  for (int i = 0; i < HIP_IPC_HANDLE_SIZE; ++i) h.reserved[i] = in64[i];
  void* p = nullptr;
  if (hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) return nullptr;
  return p;
}

int fx_comm_ipc_close(void* p) { return (int)hipIpcCloseMemHandle(p); }

// dt: 0 bf16, 1 fp16, 2 fp32; op: 0 sum, 1 max.  `peers[world]` are the
// receive bases (own at [rank]); `timeout_ticks` bounds every wait for a
// peer granule (100 MHz ticks); returns the number of blocks launched.
int fx_comm_allreduce(int dt, int op, const void* in, void* out, long n, int rank, int world,
                      const uint64_t* peers, unsigned int* epochs, unsigned int* err,
                      long slot_granules, unsigned long long timeout_ticks, hipStream_t s) {
  PeerTable pt;
  for (int i = 0; i < FX_COMM_MAX_WORLD; ++i)
    pt.recv[i] = i < world ? reinterpret_cast<unsigned long long*>(peers[i]) : nullptr;
  // ALWAYS the full grid: every block's epoch is then the call count, so
  // consecutive calls alternate parity for EVERY granule whatever n is (a
  // size-dependent grid would let a granule be re-written with a newer tag of
  // the same parity while a slower peer still polls it).
  const int blocks = FX_COMM_MAX_BLOCKS;
#define FX_AR(T)                                                                          \
  (op == 0 ? launch<T, 0>(in, out, n, rank, world, pt, epochs, err, slot_granules, timeout_ticks, blocks, s) \
           : launch<T, 1>(in, out, n, rank, world, pt, epochs, err, slot_granules, timeout_ticks, blocks, s))
  if (dt == 0) FX_AR(bf16);
  else if (dt == 1) FX_AR(f16);
  else FX_AR(float);
#undef FX_AR
  return blocks;
}

}  // extern "C"
