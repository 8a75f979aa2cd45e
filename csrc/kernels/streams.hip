// CU-masked HIP streams (SURVEY §5.8 stream budget).
//
// The forward-overlapped AdamW of step N runs on a side stream beside step
// N+1's forward GEMMs.  A grid cap (optimizer.py overlap_grid) bounds how many
// workgroups it has in flight but lets the dispatcher put them on any CU; a
// CU mask pins the whole side stream to a fixed set of CUs instead, so every
// other CU runs GEMM tiles undisturbed.  The CUs are chosen evenly spaced and
// staggered (bit j*step + j%8): spread over every XCD whether the driver
// numbers mask bits XCD-major or XCD-interleaved.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

extern "C" {

// Creates a stream restricted to `ncu` CUs of the current device (clamped to
// [1, #CUs]); returns it (nullptr on failure) and the CU count in *got.
hipStream_t fx_cumask_stream_create(int ncu, int* got) {
  int dev = 0, total = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  if (hipDeviceGetAttribute(&total, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      total <= 0)
    return nullptr;
  if (ncu < 1) ncu = 1;
  if (ncu > total) ncu = total;
  const int words = (total + 31) / 32;
  std::vector<uint32_t> mask(words, 0u);
  const int step = total / ncu;
  int set = 0;
  for (int j = 0; j < ncu; ++j) {
    int b = j * step + (step > 1 ? j % (step < 8 ? step : 8) : 0);
    if (b >= total) b = total - 1;
    if (!(mask[b / 32] & (1u << (b % 32)))) ++set;
    mask[b / 32] |= 1u << (b % 32);
  }
  hipStream_t s = nullptr;
  if (hipExtStreamCreateWithCUMask(&s, (uint32_t)words, mask.data()) != hipSuccess) return nullptr;
  if (got) *got = set;
  return s;
}

int fx_stream_destroy(hipStream_t s) { return (int)hipStreamDestroy(s); }

}  // extern "C"
