// Deterministic float32 sin/cos/atan2 and Philox4x32-10 for the CDNA4 kernels.
//
// Bit-for-bit twin of oracle/math32.py: the same sequence of single-rounded fp32 operations.
// Every translation unit that includes this header is compiled with -ffp-contract=off, so no
// a*b+c is fused into an FMA behind our back (the NumPy oracle rounds every op).
//
// Reference call sites these replace (jnp.cos / jnp.sin / jnp.arctan2 in XLA):
//   env/obstacle.py:40-53 (Rectangle.create), env/obstacle.py:62-72 (Rectangle.inside),
//   env/lidar_env/lidar_bicycle_target.py:81-83 (heading init), :97-105 (bicycle dynamics),
//   env/utils.py:51-55 (ray angles).
// Random numbers replace jax.random threefry (env/utils.py:139-244, lidar_env/base.py:89-124).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#pragma clang fp contract(off)

namespace dgppo {

constexpr float kTwoOverPi = 0.636619772367581343f;
constexpr float kPio2_1 = 1.5703125f;
constexpr float kPio2_2 = 4.837512969970703125e-4f;
constexpr float kPio2_3 = 7.54978995489188216e-8f;
constexpr float kS1 = -1.6666654611e-1f, kS2 = 8.3321608736e-3f, kS3 = -1.9515295891e-4f;
constexpr float kC1 = 4.166664568298827e-2f, kC2 = -1.388731625493765e-3f, kC3 = 2.443315711809948e-5f;
constexpr float kT3P8 = 2.414213562373095f;
constexpr float kTP8 = 0.4142135623730950f;
constexpr float kA1 = 8.05374449538e-2f, kA2 = -1.38776856032e-1f, kA3 = 1.99777106478e-1f,
                kA4 = -3.33329491539e-1f;
constexpr float kPio4 = 0.785398163397448309616f;
constexpr float kPio2 = 1.57079632679489661923f;
constexpr float kPi = 3.14159265358979323846f;

__host__ __device__ inline void sincos32(float x, float* sn, float* cs) {
  const float j = rintf(x * kTwoOverPi);
  float r = x - j * kPio2_1;
  r = r - j * kPio2_2;
  r = r - j * kPio2_3;
  const int q = ((int)j) & 3;
  const float z = r * r;
  float ps = kS3;
  ps = ps * z + kS2;
  ps = ps * z + kS1;
  const float s = r + (r * z) * ps;
  float pc = kC3;
  pc = pc * z + kC2;
  pc = pc * z + kC1;
  const float c = (1.0f - 0.5f * z) + (z * z) * pc;
  *sn = q == 0 ? s : (q == 1 ? c : (q == 2 ? -s : -c));
  *cs = q == 0 ? c : (q == 1 ? -s : (q == 2 ? -c : s));
}

__host__ __device__ inline float atan2_32(float y, float x) {
  const float ax = fabsf(x), ay = fabsf(y);
  const bool swap = ay > ax;
  const float num = swap ? ax : ay;
  const float den = swap ? ay : ax;
  const float t = den == 0.0f ? 0.0f : num / den;
  const bool big = t > kTP8;
  const float xr = big ? (t - 1.0f) / (t + 1.0f) : t;
  const float y0 = big ? kPio4 : 0.0f;
  const float z = xr * xr;
  float p = kA1;
  p = p * z + kA2;
  p = p * z + kA3;
  p = p * z + kA4;
  p = ((p * z) * xr) + xr;
  float a = y0 + p;
  a = swap ? kPio2 - a : a;
  a = x < 0.0f ? kPi - a : a;
  return signbit(y) ? -a : a;
}

// ---- exp / log1p / logaddexp(0, x) ---------------------------------------------------------
// The VMAS contact force (env/vmas/physax/world.py `_get_constraint_forces`) evaluates
// jnp.logaddexp(0, (d_min - d) / k); these restate it as max(0, x) + log1p(exp(-|x|)) on a
// cephes expf (Cody-Waite ln2 split, degree-6 minimax) and logf (frexp + degree-9 minimax), with
// log1p from Goldberg's correction log(u) * y / (u - 1), u = 1 + y.
constexpr float kLog2e = 1.44269504088896341f;
constexpr float kLn2Hi = 0.693359375f, kLn2Lo = -2.12194440e-4f;
constexpr float kSqrtHalf = 0.707106781186547524f;

__host__ __device__ inline float exp32_nonpos(float x) {  // x <= 0; 0 below -87 (no subnormals)
  if (!(x >= -87.0f)) return 0.0f;
  const float n = rintf(x * kLog2e);
  float r = x - n * kLn2Hi;
  r = r - n * kLn2Lo;
  float p = 1.9875691500e-4f;
  p = p * r + 1.3981999507e-3f;
  p = p * r + 8.3334519073e-3f;
  p = p * r + 4.1665795894e-2f;
  p = p * r + 1.6666665459e-1f;
  p = p * r + 5.0000001201e-1f;
  p = ((p * r) * r + r) + 1.0f;
  const uint32_t eb = (uint32_t)((int)n + 127) << 23;  // 2^n, n in [-126, 0]
  float two_n;
  __builtin_memcpy(&two_n, &eb, 4);
  return p * two_n;
}

__host__ __device__ inline float log32_pos(float x) {  // x normal, > 0
  uint32_t b;
  __builtin_memcpy(&b, &x, 4);
  int e = (int)((b >> 23) & 0xFFu) - 126;
  b = (b & 0x807FFFFFu) | 0x3F000000u;  // mantissa in [0.5, 1)
  float m;
  __builtin_memcpy(&m, &b, 4);
  if (m < kSqrtHalf) {
    e -= 1;
    m = (m + m) - 1.0f;
  } else {
    m = m - 1.0f;
  }
  const float z = m * m;
  float p = 7.0376836292e-2f;
  p = p * m - 1.1514610310e-1f;
  p = p * m + 1.1676998740e-1f;
  p = p * m - 1.2420140846e-1f;
  p = p * m + 1.4249322787e-1f;
  p = p * m - 1.6668057665e-1f;
  p = p * m + 2.0000714765e-1f;
  p = p * m - 2.4999993993e-1f;
  p = p * m + 3.3333331174e-1f;
  const float fe = (float)e;
  float y = (p * m) * z;
  y = y + fe * kLn2Lo;
  y = y - 0.5f * z;
  return (m + y) + fe * kLn2Hi;
}

__host__ __device__ inline float log1p32(float y) {  // y in [0, 1]
  const float u = 1.0f + y;
  if (u == 1.0f) return y;
  return log32_pos(u) * (y / (u - 1.0f));
}

__host__ __device__ inline float logaddexp0_32(float x) {  // jnp.logaddexp(0, x), finite x
  const float amax = x > 0.0f ? x : 0.0f;
  return amax + log1p32(exp32_nonpos(-fabsf(x)));
}

// ---- Philox4x32-10 -------------------------------------------------------------------------
__host__ __device__ inline uint32_t philox4x32_w0(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                                  uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int rnd = 0; rnd < 10; ++rnd) {
    if (rnd > 0) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
  }
  return c0;
}

__host__ __device__ inline float bits_to_unit(uint32_t bits) {
  const uint32_t b = (bits >> 9) | 0x3F800000u;
  float f;
  __builtin_memcpy(&f, &b, 4);
  return f - 1.0f;
}

// One env's draw stream: draw d uses counter (d, env, purpose, 0), key (seed_lo, seed_hi).
struct Rng {
  uint32_t k0, k1, env, purpose, count;
  __host__ __device__ Rng(uint64_t seed, uint32_t env_index, uint32_t purp = 0)
      : k0((uint32_t)seed), k1((uint32_t)(seed >> 32)), env(env_index), purpose(purp), count(0) {}
  __host__ __device__ uint32_t next_bits() { return philox4x32_w0(count++, env, purpose, 0u, k0, k1); }
  // jax.random.uniform's map: max(lo, u * (hi - lo) + lo)
  __host__ __device__ float uniform(float lo, float hi) {
    const float u = bits_to_unit(next_bits());
    const float v = u * (hi - lo) + lo;
    return v < lo ? lo : v;
  }
};

}  // namespace dgppo
