"""Deterministic float32 sin/cos/atan2 and the Philox4x32-10 counter RNG — NumPy side.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  The HIP twin of every function here is
`dgppo_fov_amd/csrc/math32.h`; both evaluate the *same* sequence of single-rounded float32
operations (no FMA contraction on either side), so kernel and oracle agree bit for bit.

Why not libm: the reference calls `jnp.cos/jnp.sin/jnp.arctan2` (XLA polynomials) in
`env/obstacle.py:40-53` (Rectangle.create), `env/obstacle.py:62-72` (inside),
`env/lidar_env/lidar_bicycle_target.py:81-83,97-105` (heading init and bicycle dynamics) and
`env/utils.py:51-55` (ray angles).  No bit pattern of XLA's versions is reproducible here (JAX is
absent), so both sides of the parity check use this one cephes-style restatement (<=2 ulp).

Random numbers: the reference draws with `jax.random` threefry (`env/utils.py:139-244`,
`lidar_env/base.py:89-124`).  We use Philox4x32-10 keyed per (reset seed, env index); the
uint32 -> float conversion follows jax.random.uniform (mantissa fill, `max(minval, u*(max-min)+min)`).
"""
from __future__ import annotations

import numpy as np

F = np.float32
U32 = np.uint32

# Cody-Waite split of pi/2 (cephes DP1..DP3 doubled; the leading parts are exact in fp32)
TWO_OVER_PI = F(0.636619772367581343)
PIO2_1 = F(1.5703125)
PIO2_2 = F(4.837512969970703125e-4)
PIO2_3 = F(7.54978995489188216e-8)
# cephes sinf/cosf minimax polynomials on [-pi/4, pi/4]
S1, S2, S3 = F(-1.6666654611e-1), F(8.3321608736e-3), F(-1.9515295891e-4)
C1, C2, C3 = F(4.166664568298827e-2), F(-1.388731625493765e-3), F(2.443315711809948e-5)
# cephes atanf
T3P8 = F(2.414213562373095)
TP8 = F(0.4142135623730950)
A1, A2, A3, A4 = F(8.05374449538e-2), F(-1.38776856032e-1), F(1.99777106478e-1), F(-3.33329491539e-1)
PIO4 = F(0.785398163397448309616)
PIO2 = F(1.57079632679489661923)
PI = F(3.14159265358979323846)


def _f(x):
    return np.asarray(x, dtype=F)


def sincos(x):
    """(sin x, cos x) in float32; mirrors `dgppo_sincosf` in csrc/math32.h."""
    x = _f(x)
    with np.errstate(all="ignore"):
        j = np.rint(x * TWO_OVER_PI).astype(F)
        r = x - j * PIO2_1
        r = r - j * PIO2_2
        r = r - j * PIO2_3
        q = j.astype(np.int64) & 3
        z = r * r
        ps = S3
        ps = ps * z + S2
        ps = ps * z + S1
        s = r + (r * z) * ps
        pc = C3
        pc = pc * z + C2
        pc = pc * z + C1
        c = (F(1.0) - F(0.5) * z) + (z * z) * pc
    sin = np.where(q == 0, s, np.where(q == 1, c, np.where(q == 2, -s, -c))).astype(F)
    cos = np.where(q == 0, c, np.where(q == 1, -s, np.where(q == 2, -c, s))).astype(F)
    return sin, cos


def atan2(y, x):
    """atan2(y, x) in float32; mirrors `dgppo_atan2f` in csrc/math32.h.

    atan2(+-0, +-0) returns +-0 (the reference's jnp.arctan2 would give +-pi for x = -0)."""
    y = _f(y)
    x = _f(x)
    with np.errstate(all="ignore"):
        ax = np.abs(x)
        ay = np.abs(y)
        swap = ay > ax
        num = np.where(swap, ax, ay)
        den = np.where(swap, ay, ax)
        t = np.where(den == F(0.0), F(0.0), num / den).astype(F)
        big = t > TP8
        xr = np.where(big, (t - F(1.0)) / (t + F(1.0)), t).astype(F)
        y0 = np.where(big, PIO4, F(0.0)).astype(F)
        z = xr * xr
        p = A1
        p = p * z + A2
        p = p * z + A3
        p = p * z + A4
        p = ((p * z) * xr) + xr
        a = y0 + p
        a = np.where(swap, PIO2 - a, a).astype(F)
        a = np.where(x < F(0.0), PI - a, a).astype(F)
        a = np.where(np.signbit(y), -a, a).astype(F)
    return a


# --------------------------------------------------------------------------------------------
# exp / log1p / logaddexp(0, x): twins of exp32_nonpos / log32_pos / log1p32 / logaddexp0_32 in
# csrc/math32.h, restating jnp.logaddexp(0, .) of env/vmas/physax/world.py `_get_constraint_forces`.
# --------------------------------------------------------------------------------------------
LOG2E = F(1.44269504088896341)
LN2_HI, LN2_LO = F(0.693359375), F(-2.12194440e-4)
SQRT_HALF = F(0.707106781186547524)
EXP_P = [F(v) for v in (1.9875691500e-4, 1.3981999507e-3, 8.3334519073e-3, 4.1665795894e-2,
                        1.6666665459e-1, 5.0000001201e-1)]
LOG_P = [F(v) for v in (7.0376836292e-2, -1.1514610310e-1, 1.1676998740e-1, -1.2420140846e-1,
                        1.4249322787e-1, -1.6668057665e-1, 2.0000714765e-1, -2.4999993993e-1,
                        3.3333331174e-1)]


def exp_nonpos(x):
    """exp(x) for x <= 0 (0 below -87)."""
    x = _f(x)
    with np.errstate(all="ignore"):
        n = np.rint(x * LOG2E).astype(F)
        r = x - n * LN2_HI
        r = r - n * LN2_LO
        p = EXP_P[0]
        for c in EXP_P[1:]:
            p = p * r + c
        p = ((p * r) * r + r) + F(1.0)
        ni = np.clip(n, -126, 0).astype(np.int64)
        two_n = ((ni + 127).astype(U32) << U32(23)).view(F)
        out = (p * two_n).astype(F)
    return np.where(x >= F(-87.0), out, F(0.0)).astype(F)


def log_pos(x):
    """log(x) for normal x > 0."""
    x = _f(x)
    b = np.ascontiguousarray(x).view(U32).reshape(x.shape)
    e = ((b >> U32(23)) & U32(0xFF)).astype(np.int64) - 126
    m = ((b & U32(0x807FFFFF)) | U32(0x3F000000)).view(F)
    with np.errstate(all="ignore"):
        low = m < SQRT_HALF
        e = np.where(low, e - 1, e)
        m = np.where(low, (m + m) - F(1.0), m - F(1.0)).astype(F)
        z = m * m
        p = LOG_P[0]
        for c in LOG_P[1:]:
            p = p * m + c
        fe = e.astype(F)
        y = (p * m) * z
        y = y + fe * LN2_LO
        y = y - F(0.5) * z
        return ((m + y) + fe * LN2_HI).astype(F)


def log1p(y):
    """log(1 + y) for y in [0, 1]."""
    y = _f(y)
    u = F(1.0) + y
    with np.errstate(all="ignore"):
        v = log_pos(np.where(u == F(1.0), F(2.0), u)) * (y / (u - F(1.0)))
    return np.where(u == F(1.0), y, v).astype(F)


def logaddexp0(x):
    """jnp.logaddexp(0, x) for finite x."""
    x = _f(x)
    amax = np.where(x > F(0.0), x, F(0.0)).astype(F)
    return (amax + log1p(exp_nonpos(-np.abs(x)))).astype(F)


# --------------------------------------------------------------------------------------------
# Philox4x32-10
# --------------------------------------------------------------------------------------------
PHILOX_M0 = np.uint64(0xD2511F53)
PHILOX_M1 = np.uint64(0xCD9E8D57)
PHILOX_W0 = np.uint64(0x9E3779B9)
PHILOX_W1 = np.uint64(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10; all arguments uint32-valued arrays (broadcastable)."""
    c0, c1, c2, c3, k0, k1 = (np.asarray(v, dtype=np.uint64) & MASK32 for v in (c0, c1, c2, c3, k0, k1))
    c0, c1, c2, c3, k0, k1 = np.broadcast_arrays(c0, c1, c2, c3, k0, k1)
    for rnd in range(10):
        if rnd > 0:
            k0 = (k0 + PHILOX_W0) & MASK32
            k1 = (k1 + PHILOX_W1) & MASK32
        p0 = PHILOX_M0 * c0
        p1 = PHILOX_M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK32
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
    return tuple(v.astype(U32) for v in (c0, c1, c2, c3))


def bits_to_unit(bits):
    """uint32 -> float32 in [0, 1) exactly as jax.random.uniform does (23-bit mantissa fill)."""
    b = (np.asarray(bits, dtype=U32) >> U32(9)) | U32(0x3F800000)
    return b.view(F) - F(1.0)


def uniform(bits, minval, maxval):
    """jax.random.uniform's affine map: max(minval, u * (maxval - minval) + minval) in fp32."""
    lo = F(minval)
    hi = F(maxval)
    u = bits_to_unit(bits)
    return np.maximum(lo, u * (hi - lo) + lo).astype(F)


class PhiloxStream:
    """Per-env draw counter over Philox: draw d of env e uses counter (d, e, purpose, 0),
    key (seed_lo, seed_hi) and returns output word 0.  Mirrors `DgppoRng` in csrc/math32.h."""

    def __init__(self, seed: int, env_index, purpose: int = 0):
        self.k0 = np.uint64(seed & 0xFFFFFFFF)
        self.k1 = np.uint64((seed >> 32) & 0xFFFFFFFF)
        self.env = np.asarray(env_index, dtype=np.uint64)
        self.purpose = np.uint64(purpose)
        self.count = np.zeros(self.env.shape, dtype=np.uint64)

    def next_bits(self, active=None):
        out = philox4x32(self.count, self.env, self.purpose, 0, self.k0, self.k1)[0]
        if active is None:
            self.count = self.count + np.uint64(1)
        else:
            self.count = self.count + np.asarray(active, dtype=np.uint64)
        return out

    def uniform(self, minval, maxval, active=None):
        return uniform(self.next_bits(active), minval, maxval)
