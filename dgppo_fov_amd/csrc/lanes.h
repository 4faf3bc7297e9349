// Cross-lane primitives for the 64-wide CDNA4 wavefront shared by the attention and policy kernels.
// Reductions use DPP lane shuffles (VALU, no LDS round trip) within 16-lane rows and readlane to
// combine rows, instead of ds_bpermute-based __shfl_xor chains whose every step waits on the LDS.
#pragma once
#include <hip/hip_runtime.h>

namespace dgppo {
namespace lanes {

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float rlane(float v, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}

// all-reduce over each 16-lane row: quad_perm [1,0,3,2], [2,3,0,1], row_ror 4, row_ror 8
__device__ __forceinline__ float sum16(float v) {
  v += dppf<0xB1>(v);
  v += dppf<0x4E>(v);
  v += dppf<0x124>(v);
  return v + dppf<0x128>(v);
}
__device__ __forceinline__ float max16(float v) {
  v = fmaxf(v, dppf<0xB1>(v));
  v = fmaxf(v, dppf<0x4E>(v));
  v = fmaxf(v, dppf<0x124>(v));
  return fmaxf(v, dppf<0x128>(v));
}
// all-reduce over each 32-lane half (all 64 lanes must be active)
__device__ __forceinline__ float sum32(float v) {
  v = sum16(v);
  const float lo = rlane(v, 0) + rlane(v, 16), hi = rlane(v, 32) + rlane(v, 48);
  return (threadIdx.x & 32) ? hi : lo;
}
__device__ __forceinline__ float max32(float v) {
  v = max16(v);
  const float lo = fmaxf(rlane(v, 0), rlane(v, 16)), hi = fmaxf(rlane(v, 32), rlane(v, 48));
  return (threadIdx.x & 32) ? hi : lo;
}
// all-reduce over 8-lane groups: quad xor 1, 2 then row_half_mirror (lane i <-> 7 - i)
__device__ __forceinline__ float sum8(float v) {
  v += dppf<0xB1>(v);
  v += dppf<0x4E>(v);
  return v + dppf<0x141>(v);
}

// LDS visibility among the lanes of one wave (no workgroup barrier)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

}  // namespace lanes
}  // namespace dgppo
