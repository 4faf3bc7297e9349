// Philox4x32-10 standard normals (Box-Muller), shared by dgppo_normal (nn.hip) and the fused policy step's
// in-kernel noise (policy.hip), so both produce the same bits for the same (element, seed, stream).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dgppo {
namespace noise {

__device__ __forceinline__ uint32_t philox_w(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                             uint32_t k1, int word) {
  for (int rnd = 0; rnd < 10; ++rnd) {
    if (rnd > 0) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
  }
  return word == 0 ? c0 : (word == 1 ? c1 : (word == 2 ? c2 : c3));
}

// Counter (element lo, element hi, stream lo, stream hi | kDomain): the domain bit keeps every noise word
// disjoint from the env-reset draws, whose counters are (draw, env, purpose, 0) under the same key (math32.h Rng)
constexpr uint32_t kDomain = 0x80000000u;

// element t of the standard-normal stream (seed, stream_id)
__device__ __forceinline__ float normal_at(int64_t t, uint64_t seed, uint64_t stream_id) {
#pragma clang fp contract(off)
  const uint32_t c0 = (uint32_t)t, c1 = (uint32_t)(t >> 32);
  const uint32_t c2 = (uint32_t)stream_id, c3 = (uint32_t)(stream_id >> 32) | kDomain;
  const uint32_t a = philox_w(c0, c1, c2, c3, (uint32_t)seed, (uint32_t)(seed >> 32), 0);
  const uint32_t b = philox_w(c0, c1, c2, c3, (uint32_t)seed, (uint32_t)(seed >> 32), 1);
  const float u1 = ((a >> 8) + 1) * (1.0f / 16777216.0f);  // (0, 1]
  const float u2 = (b >> 8) * (1.0f / 16777216.0f);
  return sqrtf(-2.0f * logf(u1)) * cosf(6.28318530717958648f * u2);
}

}  // namespace noise
}  // namespace dgppo
