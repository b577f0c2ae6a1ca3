// Shared device helpers for the gfx950 (CDNA4, MI355X) kernels of llm_weighted_consensus_amd.
//
// Conventions used by every kernel in csrc/kernels:
//   * wave64 everywhere: lane = threadIdx.x & 63, block sizes are multiples of 64;
//   * bf16 is carried as raw uint16 bits in memory and widened to f32 in registers;
//     loads/stores are 16 B per lane (8 bf16) wherever the row length allows it;
//   * every launcher takes a hipStream_t so the torch binding layer can put the kernel
//     on the caller's current stream (and hence inside a captured hipGraph).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#define LWC_HOST_DEVICE __host__ __device__ __forceinline__
#define LWC_DEVICE __device__ __forceinline__

namespace lwc {

typedef uint16_t bf16_t;
typedef short short8 __attribute__((ext_vector_type(8)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef float float4v __attribute__((ext_vector_type(4)));
typedef float float16v __attribute__((ext_vector_type(16)));
typedef uint32_t uint4v __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

LWC_DEVICE float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

// Round-to-nearest-even f32 -> bf16 (NaN stays NaN: hipcc lowers this to v_cvt_pk_bf16_f32).
LWC_DEVICE bf16_t f2bf(float f) {
  __hip_bfloat16 b = __float2bfloat16(f);
  return *reinterpret_cast<bf16_t*>(&b);
}

LWC_DEVICE uint32_t pack_bf16x2(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

// 16-byte vector of 8 bf16 <-> 8 floats.
LWC_DEVICE void unpack8(const uint4v& v, float (&f)[8]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(v[i] << 16);
    f[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
  }
}
LWC_DEVICE uint4v pack8(const float (&f)[8]) {
  uint4v v;
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = pack_bf16x2(f[2 * i], f[2 * i + 1]);
  return v;
}

LWC_DEVICE float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
LWC_DEVICE float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x <= 1024; `scratch` must hold >= 16 floats.
LWC_DEVICE float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = lane < nw ? scratch[lane] : 0.f;
  return wave_sum(r);
}
LWC_DEVICE float block_max(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = lane < nw ? scratch[lane] : -INFINITY;
  return wave_max(r);
}

// Reductions over the 4 lanes {l, l^16, l^32, l^48} holding one query row's tokens: two VALU
// half-swaps (v_permlane32_swap / v_permlane16_swap, gfx950) instead of LDS ds_bpermute round trips.
LWC_DEVICE float row_max4(float v) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  auto q = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(q[0]), __uint_as_float(q[1]));
}
LWC_DEVICE float row_sum4(float v) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  auto q = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(q[0]) + __uint_as_float(q[1]);
}


// A buffer resource built from explicitly wave-uniform parts (readfirstlane of the base address and the
// size).  Built straight from kernel arguments / tile indices, the compiler sometimes cannot prove the
// resource uniform and wraps EVERY buffer access through it in a readfirstlane "waterfall" loop (~10
// instructions and a branch per access, inside GEMM main loops too).
// e8m0 exponent of an MX block with max |x| = amax: the smallest e with amax * 2^-e <= 448 (e4m3's largest
// finite), from amax's own exponent and mantissa (448 = 0.875 * 2^9), so no rounding pushes a value past 448
LWC_DEVICE int mx_exp(float amax) {
  const int ea = __builtin_amdgcn_frexp_expf(amax);
  const float m = __builtin_amdgcn_frexp_mantf(amax);
  return min(127, max(-127, ea - 9 + (m > 0.875f ? 1 : 0)));
}

// max over each 16-lane DPP row (quad xor 1, quad xor 2, half-row mirror, row mirror)
LWC_DEVICE float row16_max(float x) {
  x = fmaxf(x, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0xB1, 0xF, 0xF, false)));
  x = fmaxf(x, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x4E, 0xF, 0xF, false)));
  x = fmaxf(x, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x141, 0xF, 0xF, false)));
  return fmaxf(x, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x140, 0xF, 0xF, false)));
}

LWC_DEVICE __amdgpu_buffer_rsrc_t uniform_rsrc(const void* base, int bytes) {
  const uint64_t a = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0,
                                           __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// Bijective XCD-aware remap of a linear workgroup id (cdna_hip_programming.md §5 "XCD swizzle
// must be bijective"): consecutive remapped ids land on the same XCD so neighbouring tiles share L2.
LWC_DEVICE int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

}  // namespace lwc

#define LWC_CHECK_LAUNCH() (void)hipGetLastError()
