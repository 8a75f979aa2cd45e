// Common device helpers for FleetX-AMD HIP kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

#define FX_WAVE 64

typedef __hip_bfloat16 bf16;
typedef __half f16;

typedef short short8 __attribute__((ext_vector_type(8)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// ---------------------------------------------------------------- conversions
__device__ __forceinline__ float bf16_bits_to_float(uint16_t u) {
  return __uint_as_float(((uint32_t)u) << 16);
}
__device__ __forceinline__ uint16_t float_to_bf16_bits(float f) {
  bf16 b = __float2bfloat16(f);
  return *reinterpret_cast<uint16_t*>(&b);
}
__device__ __forceinline__ float half_bits_to_float(uint16_t u) {
  __half h = *reinterpret_cast<__half*>(&u);
  return __half2float(h);
}
__device__ __forceinline__ uint16_t float_to_half_bits(float f) {
  __half h = __float2half(f);
  return *reinterpret_cast<uint16_t*>(&h);
}

// Element type traits: 16-bit storage types are moved as raw bits.
template <typename T> struct Elt;
template <> struct Elt<bf16> {
  static __device__ __forceinline__ float to_f(uint16_t u) { return bf16_bits_to_float(u); }
  static __device__ __forceinline__ uint16_t from_f(float f) { return float_to_bf16_bits(f); }
};
template <> struct Elt<f16> {
  static __device__ __forceinline__ float to_f(uint16_t u) { return half_bits_to_float(u); }
  static __device__ __forceinline__ uint16_t from_f(float f) { return float_to_half_bits(f); }
};

// Load / store 8 consecutive 16-bit elements as float[8].
template <typename T>
__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  const uint16_t* h = reinterpret_cast<const uint16_t*>(&v);
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = Elt<T>::to_f(h[j]);
}
template <typename T>
__device__ __forceinline__ void load8(const uint16_t* p, float* f) {
  unpack8<T>(*reinterpret_cast<const uint4*>(p), f);
}
template <typename T>
__device__ __forceinline__ void store8(uint16_t* p, const float* f) {
  uint4 v;
  uint16_t* h = reinterpret_cast<uint16_t*>(&v);
#pragma unroll
  for (int j = 0; j < 8; ++j) h[j] = Elt<T>::from_f(f[j]);
  *reinterpret_cast<uint4*>(p) = v;
}

// ---------------------------------------------------------------- reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---------------------------------------------------------------- RNG
// lowbias32 (C. Wellons) avalanche permutation; must match
// fleetx_amd/parallel/rng.py.
__device__ __forceinline__ uint32_t lowbias32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
// 16-bit uniform for flat element i (elementwise dropout).
__device__ __forceinline__ uint32_t elem_rand_pair(uint64_t i, uint32_t klo, uint32_t khi) {
  uint64_t pair = i >> 1;
  uint32_t c = lowbias32((uint32_t)(pair >> 32) ^ khi) ^ klo;
  return lowbias32((uint32_t)pair ^ c);
}

// splitmix64 finaliser: graph-mode re-keying of dropout streams
__host__ __device__ __forceinline__ uint64_t fx_mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
extern const uint64_t* g_fx_dropout_salt;  // host-side, set by fx_set_dropout_salt
__device__ __forceinline__ uint64_t salt_key(uint64_t key, uint64_t salt) {
  return fx_mix64(key ^ fx_mix64(salt + 0x9E3779B97F4A7C15ull)) & 0x7FFFFFFFFFFFFFFFull;
}

// Round-trip through the 16-bit storage type (what a store + reload would see).
template <typename T>
__device__ __forceinline__ float round_to(float f) {
  return Elt<T>::to_f(Elt<T>::from_f(f));
}

// ---------------------------------------------------------------- math
// tanh-GeLU via the identity 0.5 * (1 + tanh(u)) = 1 / (1 + exp(-2u)):
// one v_exp_f32 + one v_rcp_f32 instead of libm tanhf's polynomial chain.
__device__ __forceinline__ float gelu_tanh(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float u = k0 * (x + k1 * x * x * x);
  return x * __builtin_amdgcn_rcpf(1.f + __expf(-2.f * u));
}
__device__ __forceinline__ float gelu_tanh_grad(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float x2 = x * x;
  const float u = k0 * (x + k1 * x2 * x);
  const float s = __builtin_amdgcn_rcpf(1.f + __expf(-2.f * u));  // sigmoid(2u) = (1 + tanh u) / 2
  return s + 2.f * x * s * (1.f - s) * k0 * (1.f + 3.f * k1 * x2);
}
__device__ __forceinline__ float gelu_erf(float x) {
  return 0.5f * x * (1.f + erff(x * 0.7071067811865476f));
}
__device__ __forceinline__ float gelu_erf_grad(float x) {
  return 0.5f * (1.f + erff(x * 0.7071067811865476f)) +
         x * 0.3989422804014327f * __expf(-0.5f * x * x);
}

#define FX_CHECK_LAUNCH() (void)hipGetLastError()

static inline int fx_cdiv(long a, long b) { return (int)((a + b - 1) / b); }
