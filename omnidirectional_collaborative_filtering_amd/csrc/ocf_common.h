// Shared device/host helpers for libocf (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ocf.h"

typedef _Float16 ocf_h8 __attribute__((ext_vector_type(8)));
typedef __bf16 ocf_b8 __attribute__((ext_vector_type(8)));
typedef short ocf_s4 __attribute__((ext_vector_type(4)));
typedef float ocf_f16v __attribute__((ext_vector_type(16)));
typedef float ocf_f4 __attribute__((ext_vector_type(4)));

// Element-type codes used across the C ABI (see include/ocf.h).
enum {
  OCF_F32 = 0,
  OCF_F16 = 1,
  OCF_BF16 = 2,
};

// Activation codes (model.py:34 default 'tanh', train.py:52 'sigmoid').
enum {
  OCF_ACT_LINEAR = 0,
  OCF_ACT_SIGMOID = 1,
  OCF_ACT_TANH = 2,
  OCF_ACT_RELU = 3,
};

// Optimizer codes (train.py:50-51 Adagrad, train_jester.py:61 rmsprop, north_star Adam).
enum {
  OCF_OPT_SGD = 0,
  OCF_OPT_ADAGRAD = 1,
  OCF_OPT_RMSPROP = 2,
  OCF_OPT_ADAM = 3,
};



namespace ocf {

template <typename T> struct CvtT;
template <> struct CvtT<float> {
  static __device__ __forceinline__ float to(float x) { return x; }
  static __device__ __forceinline__ float from(float x) { return x; }
};
template <> struct CvtT<_Float16> {
  static __device__ __forceinline__ _Float16 to(float x) { return (_Float16)x; }
  static __device__ __forceinline__ float from(_Float16 x) { return (float)x; }
};
template <> struct CvtT<__bf16> {
  static __device__ __forceinline__ __bf16 to(float x) { return (__bf16)x; }
  static __device__ __forceinline__ float from(__bf16 x) { return (float)x; }
};

__device__ __forceinline__ float act_apply(int act, float z) {
  switch (act) {
    case OCF_ACT_SIGMOID: return 1.0f / (1.0f + __expf(-z));
    case OCF_ACT_TANH: return tanhf(z);
    case OCF_ACT_RELU: return z > 0.f ? z : 0.f;
    default: return z;
  }
}
// derivative expressed from the activation output a (and z for relu)
__device__ __forceinline__ float act_grad(int act, float a) {
  switch (act) {
    case OCF_ACT_SIGMOID: return a * (1.0f - a);
    case OCF_ACT_TANH: return 1.0f - a * a;
    case OCF_ACT_RELU: return a > 0.f ? 1.f : 0.f;
    default: return 1.0f;
  }
}

// Philox4x32-10 counter-based RNG (device dropout / reciprocal split in device-RNG mode).
__device__ __forceinline__ uint32_t mulhilo(uint32_t a, uint32_t b, uint32_t* hi) {
  uint64_t p = (uint64_t)a * (uint64_t)b;
  *hi = (uint32_t)(p >> 32);
  return (uint32_t)p;
}
__device__ __forceinline__ uint4 philox4(uint4 c, uint2 k) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0, hi1;
    uint32_t lo0 = mulhilo(0xD2511F53u, c.x, &hi0);
    uint32_t lo1 = mulhilo(0xCD9E8D57u, c.z, &hi1);
    c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  return c;
}
// ---- cache-policy loads / stores through buffer descriptors ----------------------------
typedef unsigned int ocf_u4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wt_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7FFFFFFF, 0x00020000);
}
// 16-B store / load with an explicit cache policy (aux bits: 2 = nt, 16 = sc1; 0 = plain)
template <int AUX, typename T16>
__device__ __forceinline__ void st_pol16(__amdgpu_buffer_rsrc_t r, void* base, uint32_t byte_off, const T16& v) {
  static_assert(sizeof(T16) == 16, "16-byte store");
  if constexpr (AUX == 0) {
    (void)r;
    *reinterpret_cast<T16*>(reinterpret_cast<char*>(base) + byte_off) = v;
  } else {
    (void)base;
    ocf_u4 u;
    __builtin_memcpy(&u, &v, 16);
    __builtin_amdgcn_raw_buffer_store_b128(u, r, byte_off, 0, AUX);
  }
}
template <int AUX>
__device__ __forceinline__ float4 ld_pol16(__amdgpu_buffer_rsrc_t r, const void* base, uint32_t byte_off) {
  if constexpr (AUX == 0) {
    (void)r;
    return *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(base) + byte_off);
  } else {
    (void)base;
    ocf_u4 u = __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, AUX);
    float4 f;
    __builtin_memcpy(&f, &u, 16);
    return f;
  }
}
// uniform in [0,1) with 24 random bits
__device__ __forceinline__ float philox_uniform(uint64_t seed, uint64_t stream, uint64_t idx) {
  uint4 c = make_uint4((uint32_t)idx, (uint32_t)(idx >> 32), (uint32_t)stream, (uint32_t)(stream >> 32));
  uint4 r = philox4(c, make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
  return (float)(r.x >> 8) * (1.0f / 16777216.0f);
}

}  // namespace ocf
