// dgi/csrc/common.h — shared device helpers for the gfx950 (CDNA4) kernels.
//
// Everything here is written for wave64 / MFMA on MI355X; there is no
// CUDA or multi-platform path.  bf16 values travel as raw 16-bit patterns
// (ushort) through memory and are widened to fp32 in registers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dgi {

constexpr int kWave = 64;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

typedef __attribute__((address_space(3))) short4v lds_short4;

__device__ __forceinline__ float bf16_to_f32(uint16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}

typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef float f32x2v __attribute__((ext_vector_type(2)));

// Round-to-nearest-even f32 -> bf16.  Written as a (vector) conversion so hipcc
// emits gfx950's v_cvt_pk_bf16_f32 (one VALU op for two values) instead of the
// 5-6 integer ops of a bit-manipulation RNE — the softmax / norm / epilogue
// loops are VALU-issue-bound and pay for every op here.
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  return __builtin_bit_cast(uint16_t, (__bf16)f);
}

__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  const f32x2v v = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2v));
}

// 16-byte vector = 8 bf16.
struct __attribute__((aligned(16))) bf16x8_raw { uint32_t w[4]; };

__device__ __forceinline__ void unpack8(const u32x4& v, float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(v[i] << 16);
    f[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ u32x4 pack8(const float* f) {
  u32x4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = pack_bf16x2(f[2 * i], f[2 * i + 1]);
  return r;
}

__device__ __forceinline__ bf16x8 as_bf16x8(const u32x4& v) {
  return __builtin_bit_cast(bf16x8, v);
}

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

}  // namespace dgi

#define DGI_CHECK_LAUNCH() \
  do { hipError_t e__ = hipGetLastError(); if (e__ != hipSuccess) return (int)e__; } while (0)
