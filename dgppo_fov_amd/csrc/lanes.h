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

// ---- transposed reduction over each 32-lane half ---------------------------------------------------
// treduce32(v, cnt): every lane of a half-wave holds V values; afterwards lane c holds the half-wave totals
// of the value indices base(c) + j for j < cnt (base returned; slots past cnt are padding).  Five
// exchange levels halve the per-lane count: DPP row_ror 8 (lane bit 3), row_half_mirror (bit 2),
// quad_perm xor 2 (bit 1), quad_perm xor 1 (bit 0) inside 16-lane rows, then ds_swizzle xor 16 across
// the two rows.  A lane whose bit is set keeps the upper half and sends the lower one: V + V/2 + ...
// exchanges instead of V full all-reduces, no LDS storage.  All 64 lanes must be active.
template <int KIND>
__device__ __forceinline__ float tr_xchg(float v) {
  if (KIND == 0) return dppf<0x128>(v);
  if (KIND == 1) return dppf<0x141>(v);
  if (KIND == 2) return dppf<0x4E>(v);
  if (KIND == 3) return dppf<0xB1>(v);
  return __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, v), 0x401F));
}
template <int C, int KIND, int N>
__device__ __forceinline__ void tr_level(float (&v)[N], bool hi) {
  constexpr int H = (C + 1) / 2;
#pragma unroll
  for (int j = 0; j < H; ++j) {
    const float lo = v[j];
    const float up = (j + H < C) ? v[j + H] : 0.0f;
    v[j] = (hi ? up : lo) + tr_xchg<KIND>(hi ? lo : up);
  }
}
template <int V>
constexpr int tr_final() {
  return (((((V + 1) / 2 + 1) / 2 + 1) / 2 + 1) / 2 + 1) / 2;
}
template <int V>
__device__ __forceinline__ int treduce32(float (&v)[V], int& cnt) {
  constexpr int H0 = (V + 1) / 2, H1 = (H0 + 1) / 2, H2 = (H1 + 1) / 2, H3 = (H2 + 1) / 2, H4 = (H3 + 1) / 2;
  const int c = threadIdx.x & 31;
  // cnt: the real (non-padding) values of this lane's subtree; an odd split gives the upper half one fewer
  cnt = V;
  const auto split = [&](bool hi, int H) { cnt = hi ? cnt - H : (cnt < H ? cnt : H); };
  tr_level<V, 0>(v, c & 8);
  split(c & 8, H0);
  tr_level<H0, 1>(v, c & 4);
  split(c & 4, H1);
  tr_level<H1, 2>(v, c & 2);
  split(c & 2, H2);
  tr_level<H2, 3>(v, c & 1);
  split(c & 1, H3);
  tr_level<H3, 4>(v, c & 16);
  split(c & 16, H4);
  return ((c & 8) ? H0 : 0) + ((c & 4) ? H1 : 0) + ((c & 2) ? H2 : 0) + ((c & 1) ? H3 : 0) + ((c & 16) ? H4 : 0);
}

// lanes below this one whose bit of m is set
__device__ __forceinline__ int mbcnt64(uint64_t m) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// LDS visibility among the lanes of one wave (no workgroup barrier)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

}  // namespace lanes
}  // namespace dgppo
