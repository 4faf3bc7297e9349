// GraphTransformer attention core (dgppo/nn/gnn.py:78-117 + jraph segment_softmax / segment_sum)
// in the per-receiving-agent form (see include/dgppo_hip.h, dgppo_gnn_attn_args).
//
// Thread mapping: a receiver (graph g, agent i) owns a group of CP = pow2 >= C lanes, one lane per
// candidate edge; a 256-thread workgroup processes R = 256 / CP receivers per round and `gpb` whole
// graphs per block (rounds loop over their receivers); blocks are persistent (grid-stride).  Each
// lane gathers its sender's feature row ONCE into registers (D <= DM floats) plus the edge's 4
// features -- issued before the round's staging barrier so the gathers overlap it -- and the
// softmax logits, the softmax backward and the sender gradients are per-lane register math; the
// weighted sums over candidates (xbar, ebar, dqt) go through an LDS transpose so every output
// column is one lane's dot product.
//
// Agent mode (xa != NULL): nodes that never receive (goals, LiDAR hits, obstacles) are only ever
// SENDERS, so their features at a layer are the previous layer's Dense_4 + ReLU of their raw row
// (empty aggregation); the kernel recomputes them per candidate (D0 x D FMAs) instead of
// materialising (G, N, D) hidden features, and folds their gradient straight into the previous
// layer's Dense_4 weight/bias gradient (per-block partials, fixed order).
//
// Sender gradients accumulate in an LDS image of the block's graphs in fixed receiver order, and
// every reduction has a fixed order: bitwise-deterministic, no atomics.
#include <hip/hip_runtime.h>

#include "lds_attr.h"
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/dgppo_hip.h"
#include "lanes.h"

namespace dgppo {

// Row strides of qt / dqt / dbeta (0: packed) and beta_h = q_h . bk_h: precomputed (p.beta, Q-free form) or
// the dot over this thread's f-stripe [f0, F) step `stride` (the caller reduces the stripes).
__device__ __forceinline__ int64_t qt_ld(const dgppo_gnn_attn_args& p) { return p.qt_ld ? p.qt_ld : (int64_t)p.H * p.D; }
__device__ __forceinline__ int64_t dqt_ld(const dgppo_gnn_attn_args& p) {
  return p.dqt_ld ? p.dqt_ld : (int64_t)p.H * p.D;
}
__device__ __forceinline__ int64_t dbeta_ld(const dgppo_gnn_attn_args& p) { return p.dbeta_ld ? p.dbeta_ld : p.H; }
__device__ __forceinline__ float q_dot_bk(const dgppo_gnn_attn_args& p, int64_t row, int h, int f0, int stride) {
  if (p.beta) return f0 == 0 ? p.beta[row * p.beta_ld + h] : 0.0f;
  float acc = 0.0f;
  for (int f = f0; f < p.F; f += stride) acc += p.q[row * p.H * p.F + h * p.F + f] * p.bk[h * p.F + f];
  return acc;
}
namespace {

constexpr int kH = 3;         // heads (GraphTransformer num_heads of the reference GNN)
constexpr int kD0 = 8;        // max raw feature width in agent mode
constexpr int kMaxBlocks = 2048;

template <int CP>
__device__ __forceinline__ float group_sum(float v, float* scratch) {
  if constexpr (CP <= 64) {
#pragma unroll
    for (int o = CP / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
  } else {  // CP = 128: two waves per group
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) scratch[w] = v;
    __syncthreads();
    const float r = scratch[(w & ~1)] + scratch[(w | 1)];
    __syncthreads();
    return r;
  }
}

template <int CP>
__device__ __forceinline__ float group_max(float v, float* scratch) {
  if constexpr (CP <= 64) {
#pragma unroll
    for (int o = CP / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
  } else {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) scratch[w] = v;
    __syncthreads();
    const float r = fmaxf(scratch[(w & ~1)], scratch[(w | 1)]);
    __syncthreads();
    return r;
  }
}

// group_sum / group_max of all kH heads at once: for CP = 128 one LDS exchange (3 barriers) serves every
// head instead of one per head; same pairing and order as group_sum / group_max (bit-identical)
template <int CP, bool MAX>
__device__ __forceinline__ void group_red3(float (&v)[kH], float* scratch) {
  if constexpr (CP <= 64) {
#pragma unroll
    for (int h = 0; h < kH; ++h) v[h] = MAX ? group_max<CP>(v[h], nullptr) : group_sum<CP>(v[h], nullptr);
  } else {
#pragma unroll
    for (int h = 0; h < kH; ++h)
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float w = __shfl_xor(v[h], o, 64);
        v[h] = MAX ? fmaxf(v[h], w) : v[h] + w;
      }
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0)
#pragma unroll
      for (int h = 0; h < kH; ++h) scratch[w * kH + h] = v[h];
    __syncthreads();
#pragma unroll
    for (int h = 0; h < kH; ++h) {
      const float a = scratch[(w & ~1) * kH + h], b = scratch[(w | 1) * kH + h];
      v[h] = MAX ? fmaxf(a, b) : a + b;
    }
    __syncthreads();
  }
}

struct Cand {
  int s, e;
};

__device__ __forceinline__ Cand candidate(const dgppo_gnn_attn_args& p, int64_t g, int i, int c) {
  Cand k{-1, -1};
  if (c < p.C) {
    const int e = p.cand[i * p.C + c];
    k.e = e;
    if (p.sidx) k.s = p.sidx[(g * p.n_agents + i) * p.C + c];
    else if (e >= 0 && p.receivers[g * p.E + e] == i) k.s = p.senders[g * p.E + e];
  }
  return k;
}

__global__ __launch_bounds__(256) void sender_table_kernel(int32_t G, int32_t n, int32_t C, int32_t E,
                                                           const int32_t* cand, const int32_t* recv,
                                                           const int32_t* send, int32_t* sidx) {
  const int64_t total = (int64_t)G * n * C;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int c = (int)(t % C);
    const int64_t gi = t / C;
    const int i = (int)(gi % n);
    const int64_t g = gi / n;
    const int e = cand[i * C + c];
    sidx[t] = (e >= 0 && recv[g * E + e] == i) ? send[g * E + e] : -1;
  }
}

template <int DM>
__device__ __forceinline__ void load_row(const float* xr, int D, bool ok, float (&x)[DM]) {
  if (DM % 4 == 0 && D == DM && (((uintptr_t)xr & 15) == 0)) {
#pragma unroll
    for (int q = 0; q < DM / 4; ++q) {
      const float4 v = ok ? *(const float4*)(xr + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
      x[4 * q] = v.x, x[4 * q + 1] = v.y, x[4 * q + 2] = v.z, x[4 * q + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int d = 0; d < DM; ++d) x[d] = (ok && d < D) ? xr[d] : 0.0f;
  }
}

// LDS carve (floats), CR = candidate rows kept per receiver (C rounded up to 8, <= CP):
//   preW [kD0][DM] | preb [DM] | scratch [8] | qt [R][kH*DM] | xs [R*CR][DM+1] | a [R*CR][kH]
//   | ef [R*CR][4] | (bwd) g [R][kH*(DM+5)] | x0s [R*CR][kD0+1] | dxs [gpb][Nacc][D]
template <int CP, int DM>
struct Carve {
  static constexpr int R = 256 / CP;
  static constexpr int XP = DM + 1;
  float *preW, *preb, *scr, *qt, *xs, *a, *ef, *g, *x0s, *dxs;
  __device__ Carve(float* base, int CR, bool bwd) {
    preW = base;
    preb = preW + kD0 * DM;
    scr = preb + DM;
    qt = scr + 16;
    xs = qt + R * kH * DM;
    a = xs + R * CR * XP;
    ef = a + R * CR * kH;
    g = ef + R * CR * 4;
    x0s = g + (bwd ? R * kH * (DM + 5) : 0);
    dxs = x0s + (bwd ? R * CR * (kD0 + 1) : 0);
  }
  static size_t floats_fixed(int CR, bool bwd) {
    return (size_t)kD0 * DM + DM + 16 + R * kH * DM + (size_t)R * CR * (XP + kH + 4) +
           (bwd ? (size_t)R * kH * (DM + 5) + (size_t)R * CR * (kD0 + 1) : 0);
  }
};

__host__ __device__ inline int cand_rows(int C, int CP) {
  const int cr = (C + 7) & ~7;
  return cr < CP ? cr : CP;
}

// sender row of candidate k into x (and its raw row into x0 when it goes through the transform)
template <int DM>
__device__ __forceinline__ void gather_sender(const dgppo_gnn_attn_args& p, int64_t g, int s, bool ok, int D,
                                              const float* preW, const float* preb, float (&x)[DM],
                                              float (&x0)[kD0], bool& via_pre) {
  via_pre = false;
#pragma unroll
  for (int k = 0; k < kD0; ++k) x0[k] = 0.0f;
  if (p.xa == nullptr) {
    load_row<DM>(p.x + g * p.x_gstride + (int64_t)(ok ? s : 0) * D, D, ok, x);
    return;
  }
  if (!ok || s < p.n_agents) {
    load_row<DM>(p.xa + g * p.xa_gstride + (int64_t)(ok ? s : 0) * D, D, ok, x);
    return;
  }
  const float* xr = p.x + g * p.x_gstride + (int64_t)s * p.D0;
#pragma unroll
  for (int k = 0; k < kD0; ++k) x0[k] = k < p.D0 ? xr[k] : 0.0f;
  if (p.pre_W == nullptr) {  // raw rows used directly (D0 == D <= kD0)
#pragma unroll
    for (int d = 0; d < DM; ++d) x[d] = d < kD0 ? x0[d < kD0 ? d : 0] : 0.0f;
    return;
  }
  via_pre = true;
#pragma unroll
  for (int d = 0; d < DM; ++d) {
    float v = preb[d];
#pragma unroll
    for (int k = 0; k < kD0; ++k) v += x0[k] * preW[k * DM + d];
    x[d] = v > 0.0f ? v : 0.0f;
  }
}

__device__ __forceinline__ void stage_pre(const dgppo_gnn_attn_args& p, float* preW, float* preb, int DM) {
  if (p.xa == nullptr || p.pre_W == nullptr) return;
  for (int e = threadIdx.x; e < kD0 * DM; e += 256) {
    const int k = e / DM, d = e - k * DM;
    preW[e] = (k < p.D0 && d < p.D) ? p.pre_W[k * p.D + d] : 0.0f;
  }
  for (int d = threadIdx.x; d < DM; d += 256) preb[d] = d < p.D ? p.pre_b[d] : 0.0f;
}

template <int CP, int DM>
__global__ __launch_bounds__(256) void attn_fwd_kernel(dgppo_gnn_attn_args p, int gpb, int64_t nblk) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  using CV = Carve<CP, DM>;
  constexpr int R = CV::R, XP = CV::XP;
  const int n = p.n_agents, D = p.D, F = p.F, C = p.C, H = p.H;
  const int CR = cand_rows(C, CP);
  CV L(lds, CR, false);
  const int W = H * (D + 5);
  const int t = threadIdx.x, slot = t / CP, c = t % CP;
  const int lr = slot * CR + c;  // this lane's LDS row (valid when c < CR)
  stage_pre(p, L.preW, L.preb, DM);
  __syncthreads();
  for (int64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    const int64_t g0 = blk * gpb;
    const int ng = (int)((int64_t)p.G - g0 < gpb ? (int64_t)p.G - g0 : gpb);
    const int nrec = ng * n;
    for (int r0 = 0; r0 < nrec; r0 += R) {
      const int rl = r0 + slot;
      const bool active = rl < nrec;
      const int64_t g = g0 + (active ? rl / n : 0);
      const int i = active ? rl % n : 0;
      const int64_t row = g0 * n + rl;
      // gathers first (they overlap the staging barrier below)
      const Cand k = active ? candidate(p, g, i, c) : Cand{-1, -1};
      const bool ok = k.s >= 0;
      float x[DM], x0[kD0];
      bool via_pre;
      gather_sender<DM>(p, g, k.s, ok, D, L.preW, L.preb, x, x0, via_pre);
      float ef[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) ef[j] = ok ? p.ef[g * p.ef_gstride + (int64_t)k.e * 4 + j] : 0.0f;
      // stage qt; beta_h = q_h . bk_h as a group dot product
      for (int e = t; e < R * H * D; e += 256) {
        const int rr = e / (H * D), kk = e - rr * (H * D);
        if (r0 + rr < nrec) L.qt[rr * kH * DM + kk] = p.qt[(g0 * n + r0 + rr) * qt_ld(p) + kk];
      }
      float beta[kH];
#pragma unroll
      for (int h = 0; h < kH; ++h) {
        float acc = 0.0f;
        if (active && h < H)
          acc = q_dot_bk(p, row, h, c, CP);
        beta[h] = acc;
      }
      group_red3<CP, false>(beta, L.scr);
      __syncthreads();
      float lg[kH], mx[kH], a[kH];
#pragma unroll
      for (int h = 0; h < kH; ++h) {
        float acc = 0.0f;
        const float* qt = L.qt + slot * kH * DM + h * D;
#pragma unroll
        for (int d = 0; d < DM; ++d)
          if (d < D) acc += qt[d] * x[d];
        lg[h] = (ok && h < H) ? (acc + beta[h]) * p.scale : -INFINITY;
        mx[h] = lg[h];
      }
      group_red3<CP, true>(mx, L.scr);
      float ex[kH], sm[kH];
#pragma unroll
      for (int h = 0; h < kH; ++h) sm[h] = ex[h] = ok && h < H ? expf(lg[h] - mx[h]) : 0.0f;
      group_red3<CP, false>(sm, L.scr);
#pragma unroll
      for (int h = 0; h < kH; ++h) {
        a[h] = ok && h < H ? ex[h] / sm[h] : 0.0f;
        if (active && c < C && h < H && p.attn) p.attn[(row * H + h) * C + c] = a[h];
      }
      // LDS transpose: candidates' rows and weights, then one output column per lane
      if (c < CR) {
#pragma unroll
        for (int d = 0; d < DM; ++d) L.xs[lr * XP + d] = x[d];
#pragma unroll
        for (int h = 0; h < kH; ++h) L.a[lr * kH + h] = a[h];
#pragma unroll
        for (int j = 0; j < 4; ++j) L.ef[lr * 4 + j] = ef[j];
      }
      __syncthreads();
      if (active) {
        const int base = slot * CR;
        float* out = p.xcat + row * W;
        for (int o = c; o < W; o += CP) {
          float acc = 0.0f;
          if (o < H * D) {
            const int h = o / D, d = o - h * D;
            #pragma unroll 8
            for (int cc = 0; cc < CR; ++cc) acc += L.a[(base + cc) * kH + h] * L.xs[(base + cc) * XP + d];
          } else if (o < H * D + 4 * H) {
            const int q = o - H * D, h = q >> 2, j = q & 3;
            #pragma unroll 8
            for (int cc = 0; cc < CR; ++cc) acc += L.a[(base + cc) * kH + h] * L.ef[(base + cc) * 4 + j];
          } else {
            const int h = o - H * D - 4 * H;
            #pragma unroll 8
            for (int cc = 0; cc < CR; ++cc) acc += L.a[(base + cc) * kH + h];
          }
          out[o] = acc;
        }
      }
      __syncthreads();
    }
  }
}

// backward LDS carve (floats):
//   preW [kD0][DM] | preb [DM] | scratch [8] | qt [R][kH*DM] | g [R][kH*(DM+5)] | xs [R*CR][DM+1]
//   | a [R*CR][kH] | ps [R*CR][DM+1] | x0s [R*CR][kD0+1] | cb [R][n][DM] | dxs [gpb][N][D] (full mode)
template <int CP, int DM>
struct BwdCarve {
  static constexpr int R = 256 / CP;
  static constexpr int XP = DM + 1;
  float *preW, *preb, *scr, *qt, *g, *xs, *a, *ps, *x0s, *cb, *dxs;
  __device__ BwdCarve(float* base, int CR, int n) {
    preW = base;
    preb = preW + kD0 * DM;
    scr = preb + DM;
    qt = scr + 16;
    g = qt + R * kH * DM;
    xs = g + R * kH * (DM + 5);
    a = xs + R * CR * XP;
    ps = a + R * CR * kH;
    x0s = ps + R * CR * XP;
    cb = x0s + R * CR * (kD0 + 1);
    dxs = cb + R * n * DM;
  }
  static size_t floats_fixed(int CR, int n) {
    return (size_t)kD0 * DM + DM + 16 + R * kH * DM + R * kH * (DM + 5) + (size_t)R * CR * (2 * XP + kH + kD0 + 1) +
           (size_t)R * n * DM;
  }
};

// Backward.  Agent mode relies on the env layout of the candidate table (env/base.py
// agent_candidates): an agent sender j only ever appears at candidate slot c == j (the agent-agent
// block edge i*n + j), so the sender gradient of agent j is the fixed-order sum over the graph's
// receivers of their slot-j contributions -- one barrier, no serialised accumulation.
template <int CP, int DM>
__global__ __launch_bounds__(256) void attn_bwd_kernel(dgppo_gnn_attn_args p, int gpb, int64_t nblk) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  using CV = BwdCarve<CP, DM>;
  constexpr int R = CV::R, XP = CV::XP;
  constexpr int NTD = (DM + 31) / 32;  // 32-column tiles of the pre-gradient accumulator
  const int n = p.n_agents, D = p.D, F = p.F, C = p.C, H = p.H;
  const int CR = cand_rows(C, CP);
  CV L(lds, CR, n);
  const int W = H * (D + 5);
  const int t = threadIdx.x, slot = t / CP, c = t % CP;
  const int lane = t & 63, wave = t >> 6;
  const int lr = slot * CR + c;
  const bool agent_mode = p.xa != nullptr;
  const bool want_dxa = agent_mode && p.dxa != nullptr;
  const bool want_dx = !agent_mode && p.dx != nullptr;
  const bool want_pre = agent_mode && p.pre_W != nullptr && p.dpre_part != nullptr;
  const int N = p.N;
  typedef float f32x16 __attribute__((ext_vector_type(16)));
  f32x16 pacc[NTD];
#pragma unroll
  for (int q = 0; q < NTD; ++q)
#pragma unroll
    for (int r = 0; r < 16; ++r) pacc[q][r] = 0.0f;
  stage_pre(p, L.preW, L.preb, DM);
  __syncthreads();
  for (int64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    const int64_t g0 = blk * gpb;
    const int ng = (int)((int64_t)p.G - g0 < gpb ? (int64_t)p.G - g0 : gpb);
    const int nrec = ng * n;
    if (want_dx) {
      for (int e = t; e < ng * N * D; e += 256) L.dxs[e] = 0.0f;
      __syncthreads();
    }
    for (int r0 = 0; r0 < nrec; r0 += R) {
      const int rl = r0 + slot;
      const bool active = rl < nrec;
      const int gl = active ? rl / n : 0;
      const int64_t g = g0 + gl;
      const int i = active ? rl % n : 0;
      const int64_t row = g0 * n + rl;
      const Cand k = active ? candidate(p, g, i, c) : Cand{-1, -1};
      const bool ok = k.s >= 0;
      float x[DM], x0[kD0];
      bool via_pre;
      gather_sender<DM>(p, g, k.s, ok, D, L.preW, L.preb, x, x0, via_pre);
      float ef[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) ef[j] = ok ? p.ef[g * p.ef_gstride + (int64_t)k.e * 4 + j] : 0.0f;
      float a[kH];
#pragma unroll
      for (int h = 0; h < kH; ++h) a[h] = (ok && h < H) ? p.attn[(row * H + h) * C + c] : 0.0f;
      for (int e = t; e < R * H * D; e += 256) {
        const int rr = e / (H * D), kk = e - rr * (H * D);
        if (r0 + rr < nrec) L.qt[rr * kH * DM + kk] = p.qt[(g0 * n + r0 + rr) * qt_ld(p) + kk];
      }
      for (int e = t; e < R * W; e += 256) {
        const int rr = e / W, kk = e - rr * W;
        if (r0 + rr < nrec) L.g[rr * kH * (DM + 5) + kk] = p.dxcat[(g0 * n + r0 + rr) * W + kk];
      }
      __syncthreads();  // (1) qt / dxcat staged
      const float* gv = L.g + slot * kH * (DM + 5);  // dxbar (H*D) | debar (H*4) | dsig (H)
      float dl[kH], dbeta[kH], da[kH], dot[kH];
#pragma unroll
      for (int h = 0; h < kH; ++h) {
        da[h] = 0.0f;
        if (ok && h < H) {
#pragma unroll
          for (int d = 0; d < DM; ++d)
            if (d < D) da[h] += gv[h * D + d] * x[d];
#pragma unroll
          for (int j = 0; j < 4; ++j) da[h] += gv[H * D + h * 4 + j] * ef[j];
          da[h] += gv[H * D + H * 4 + h];
          if (p.da_add) da[h] += p.da_add[(row * H + h) * C + c];
        }
        dot[h] = a[h] * da[h];
      }
      group_red3<CP, false>(dot, L.scr);
#pragma unroll
      for (int h = 0; h < kH; ++h) dbeta[h] = dl[h] = (ok && h < H) ? a[h] * (da[h] - dot[h]) * p.scale : 0.0f;
      group_red3<CP, false>(dbeta, L.scr);
      if (active && c == 0)
        for (int h = 0; h < H; ++h) p.dbeta[row * dbeta_ld(p) + h] = dbeta[h];
      if (active)
        for (int kk = c; kk < H * F; kk += CP) {
          const int h = kk / F;
          if (p.dq) p.dq[row * H * F + kk] = (h == 0 ? dbeta[0] : h == 1 ? dbeta[1] : dbeta[2]) * p.bk[kk];
        }
      // sender contribution dx_s[d] = sum_h a_h dxbar_h[d] + dl_h qt_h[d]
      float contrib[DM];
      {
        const float* qt = L.qt + slot * kH * DM;
#pragma unroll
        for (int d = 0; d < DM; ++d) {
          float v = 0.0f;
#pragma unroll
          for (int h = 0; h < kH; ++h)
            if (h < H && d < D) v += a[h] * gv[h * D + d] + dl[h] * qt[h * D + d];
          contrib[d] = v;
        }
      }
      // LDS images for the column reductions
      if (c < CR) {
#pragma unroll
        for (int d = 0; d < DM; ++d) L.xs[lr * XP + d] = x[d];
#pragma unroll
        for (int h = 0; h < kH; ++h) L.a[lr * kH + h] = dl[h];
        if (want_pre) {
#pragma unroll
          for (int d = 0; d < DM; ++d) L.ps[lr * XP + d] = via_pre && x[d] > 0.0f ? contrib[d] : 0.0f;
#pragma unroll
          for (int kk = 0; kk < kD0; ++kk) L.x0s[lr * (kD0 + 1) + kk] = via_pre ? x0[kk] : 0.0f;
          L.x0s[lr * (kD0 + 1) + kD0] = via_pre ? 1.0f : 0.0f;
        }
      }
      if (want_dxa && c < n) {
#pragma unroll
        for (int d = 0; d < DM; ++d) L.cb[(slot * n + c) * DM + d] = (ok && k.s < n) ? contrib[d] : 0.0f;
      }
      __syncthreads();  // (2) images written
      if (active) {
        const int base = slot * CR;
        for (int o = c; o < H * D; o += CP) {
          const int h = o / D, d = o - h * D;
          float acc = 0.0f;
          #pragma unroll 8
          for (int cc = 0; cc < CR; ++cc) acc += L.a[(base + cc) * kH + h] * L.xs[(base + cc) * XP + d];
          p.dqt[row * dqt_ld(p) + o] = acc;
        }
      }
      if (want_dxa) {  // agent j of each graph in this round: sum of its receivers' slot-j rows, in order
        const int rounds_graphs = (R + n - 1) / n + 1;
        for (int e = t; e < rounds_graphs * n * D; e += 256) {
          const int q = e / (n * D), jd = e - q * (n * D), j = jd / D, d = jd - j * D;
          const int gg = (r0 / n) + q;  // local graph index
          if (gg >= ng) continue;
          const int s0 = gg * n - r0, s1 = s0 + n;  // this graph's receivers' slots in the round
          float acc = 0.0f;
          bool any = false;
          for (int s = s0 < 0 ? 0 : s0; s < (s1 < R ? s1 : R); ++s) {
            if (r0 + s >= nrec) break;
            acc += L.cb[(s * n + j) * DM + d];
            any = true;
          }
          if (any) p.dxa[(g0 + gg) * p.dxa_gstride + j * D + d] += acc;
        }
      }
      if (want_pre) {  // pre-gradient += x0s^T ps over this round's rows (MFMA, per-wave accumulators)
        const int rows = R * CR;
        for (int t0 = 2 * wave; t0 < rows; t0 += 8) {
          const int tr = t0 + (lane >> 5);
          const int m = lane & 31;
          const float av = (tr < rows && m <= kD0) ? L.x0s[tr * (kD0 + 1) + m] : 0.0f;
#pragma unroll
          for (int q = 0; q < NTD; ++q) {
            const int d = q * 32 + m;
            const float bv = (tr < rows && d < DM) ? L.ps[tr * XP + d] : 0.0f;
            pacc[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, pacc[q], 0, 0, 0);
          }
        }
      }
      if (want_dx) {  // full mode: serialised fixed-order accumulation into the graph image
        for (int rr = 0; rr < R; ++rr) {
          __syncthreads();
          if (slot == rr && ok) {
            float* dst = L.dxs + ((int64_t)gl * N + k.s) * D;
#pragma unroll
            for (int d = 0; d < DM; ++d)
              if (d < D) dst[d] += contrib[d];
          }
        }
      }
      __syncthreads();  // (3) round done
    }
    if (want_dx) {
      for (int e = t; e < ng * N * D; e += 256) {
        const int gg = e / (N * D), kk = e - gg * (N * D);
        p.dx[(g0 + gg) * p.dx_gstride + kk] += L.dxs[e];
      }
      __syncthreads();
    }
  }
  if (want_pre) {  // combine the 4 waves' accumulators in fixed order, write this block's partial
    float* red = L.xs;  // >= 4 * 32 * (32*NTD + 1) floats are available from xs onwards
    constexpr int RP = 32 * NTD + 1;
    for (int w = 0; w < 4; ++w) {
      if (wave == w) {
#pragma unroll
        for (int q = 0; q < NTD; ++q)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
            float* dst = red + m * RP + q * 32 + (lane & 31);
            *dst = (w == 0 ? 0.0f : *dst) + pacc[q][r];
          }
      }
      __syncthreads();
    }
    const int PK = p.D0 * D + D;
    for (int o = t; o < PK; o += 256) {
      const int m = o < p.D0 * D ? o / D : kD0;
      const int d = o < p.D0 * D ? o - m * D : o - p.D0 * D;
      p.dpre_part[(int64_t)blockIdx.x * PK + o] = red[m * RP + d];
    }
  }
}


// ---- raw gather / transform split (wave kernels prefetch the next sub-round's raw rows) ----------
typedef const __attribute__((address_space(4))) float* cfloat_p;  // uniform reads -> scalar loads

template <int DM>
struct Gath {
  Cand k;
  float x[DM];   // agent row / full-mode row (or transformed row after finish())
  float x0[kD0]; // raw row of a transformed sender
  float ef[4];
  bool via_pre;
};

template <int DM>
__device__ __forceinline__ void gath_load(const dgppo_gnn_attn_args& p, int64_t g, int i, int c, bool active, int D,
                                          Gath<DM>& r) {
  r.k = active ? candidate(p, g, i, c) : Cand{-1, -1};
  const int s = r.k.s;
  const bool ok = s >= 0;
  r.via_pre = false;
#pragma unroll
  for (int k = 0; k < kD0; ++k) r.x0[k] = 0.0f;
  if (p.xa == nullptr) {
    load_row<DM>(p.x + g * p.x_gstride + (int64_t)(ok ? s : 0) * D, D, ok, r.x);
  } else if (!ok || s < p.n_agents) {
    load_row<DM>(p.xa + g * p.xa_gstride + (int64_t)(ok ? s : 0) * D, D, ok, r.x);
  } else {
    const float* xr = p.x + g * p.x_gstride + (int64_t)s * p.D0;
#pragma unroll
    for (int k = 0; k < kD0; ++k) r.x0[k] = k < p.D0 ? xr[k] : 0.0f;
    r.via_pre = p.pre_W != nullptr;
#pragma unroll
    for (int d = 0; d < DM; ++d) r.x[d] = 0.0f;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) r.ef[j] = ok ? p.ef[g * p.ef_gstride + (int64_t)r.k.e * 4 + j] : 0.0f;
}

// non-agent senders of agent mode: relu(x0 pre_W + pre_b) (or the raw row itself without pre_W)
template <int DM>
__device__ __forceinline__ void gath_finish(const dgppo_gnn_attn_args& p, const float* preW, const float* preb,
                                            Gath<DM>& r) {
  if (p.xa == nullptr || r.k.s < p.n_agents) return;
  if (!r.via_pre) {
#pragma unroll
    for (int d = 0; d < DM; ++d) r.x[d] = d < kD0 ? r.x0[d < kD0 ? d : 0] : 0.0f;
    return;
  }
#pragma unroll
  for (int d = 0; d < DM; ++d) {
    float v = preb[d];
#pragma unroll
    for (int k = 0; k < kD0; ++k) v += r.x0[k] * preW[k * DM + d];
    r.x[d] = v > 0.0f ? v : 0.0f;
  }
}

// ================================================================================================
// Wave-independent kernels (CP <= 64): each WAVE owns whole graphs and walks their receivers RW =
// 64 / CP at a time, with all its LDS images private, so waves never wait on each other (no block
// barriers inside the loops; the hardware interleaves the waves' gathers).  Block barriers only at
// start (pre_W staging) and end (pre-gradient combine).
// ================================================================================================
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// per-wave LDS (floats): qt [RW][QP] | g [RW][GP] (bwd) | xs [RW*CR][XP] | a [RW*CR][kH]
//   | ef [RW*CR][4] | x0s [RW*CR][kD0+1] (bwd) | cb [gpw][n][DM] (bwd)
template <int CP, int DM>
struct WaveCarve {
  static constexpr int RW = 64 / CP;
  static constexpr int XP = DM + 1;
  static constexpr int QP = kH * DM;
  static constexpr int GP = kH * DM + 16;  // dxbar (H*DM) | debar (kH*4) | dsig (kH) | pad
  float *qt, *g, *xs, *a, *ef, *x0s, *cb;
  __device__ WaveCarve(float* base, int CR, int cbf, bool bwd) {
    qt = base;
    g = qt + RW * QP;
    xs = g + (bwd ? RW * GP : 0);
    a = xs + RW * CR * XP;
    ef = a + RW * CR * kH;
    x0s = ef + RW * CR * 4;
    cb = x0s + (bwd ? RW * CR * (kD0 + 1) : 0);
    (void)cbf;
  }
  static size_t floats(int CR, int cbf, bool bwd) {
    size_t f = (size_t)RW * QP + (size_t)RW * CR * (XP + kH + 4);
    if (bwd) f += (size_t)RW * GP + (size_t)RW * CR * (kD0 + 1) + cbf;
    return (f + 3) & ~(size_t)3;
  }
};

// shared block header: preW [kD0][DM] | preb [DM] | (then 4 wave regions)
template <int DM>
constexpr int wave_header_floats() {
  return ((kD0 * DM + DM) + 3) & ~3;
}

template <int CP, int DM>
__global__ __launch_bounds__(256) void attn_fwd_wave_kernel(dgppo_gnn_attn_args p, int gpw, int64_t nitems,
                                                            int wfloats) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  using CV = WaveCarve<CP, DM>;
  constexpr int RW = CV::RW, XP = CV::XP, QP = CV::QP;
  const int n = p.n_agents, D = p.D, F = p.F, C = p.C, H = p.H;
  const int CR = cand_rows(C, CP);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  CV L(lds + wave_header_floats<DM>() + wave * wfloats, CR, 0, false);
  const int W = H * (D + 5);
  const int slot = lane / CP, c = lane % CP;
  const int lr = slot * CR + c;
  float* preW = lds;
  float* preb = preW + kD0 * DM;
  stage_pre(p, preW, preb, DM);
  __syncthreads();
  const int64_t gw = (int64_t)blockIdx.x * 4 + wave, nw = (int64_t)gridDim.x * 4;
  // this wave's sub-rounds j = (its k-th item, r0): a flat sequence so the next one's gathers are
  // issued while the current one computes
  const int spi = (gpw * n + RW - 1) / RW;
  const int64_t my_items = gw < nitems ? (nitems - gw + nw - 1) / nw : 0;
  const int64_t J = my_items * spi;
  auto sub = [&](int64_t j, int64_t& g0, int& nrec, int& r0) {
    const int64_t item = gw + (j / spi) * nw;
    g0 = item * gpw;
    const int ng = (int)((int64_t)p.G - g0 < gpw ? (int64_t)p.G - g0 : gpw);
    nrec = ng * n;
    r0 = (int)(j % spi) * RW;
  };
  Gath<DM> cur, nxt;
  if (J > 0) {
    int64_t g0;
    int nrec, r0;
    sub(0, g0, nrec, r0);
    const int rl = r0 + slot;
    gath_load<DM>(p, g0 + (rl < nrec ? rl / n : 0), rl < nrec ? rl % n : 0, c, rl < nrec, D, cur);
  }
  for (int64_t j = 0; j < J; ++j) {
    int64_t g0;
    int nrec, r0;
    sub(j, g0, nrec, r0);
    const int rl = r0 + slot;
    const bool active = rl < nrec;
    const int64_t row = g0 * n + rl;
    // this sub-round's small loads first (in-order completion), then the next sub-round's gathers
    float qv[(RW * kH * DM + 63) / 64];
#pragma unroll
    for (int u = 0; u < (RW * kH * DM + 63) / 64; ++u) {
      const int e = lane + 64 * u, rr = e / (H * D), kk = e - rr * (H * D);
      qv[u] = (e < RW * H * D && r0 + rr < nrec) ? p.qt[(g0 * n + r0 + rr) * qt_ld(p) + kk] : 0.0f;
    }
    float bacc[kH];
#pragma unroll
    for (int h = 0; h < kH; ++h) {
      float acc = 0.0f;
      if (active && h < H)
        acc = q_dot_bk(p, row, h, c, CP);
      bacc[h] = acc;
    }
    if (j + 1 < J) {
      int64_t g0n;
      int nrecn, r0n;
      sub(j + 1, g0n, nrecn, r0n);
      const int rln = r0n + slot;
      gath_load<DM>(p, g0n + (rln < nrecn ? rln / n : 0), rln < nrecn ? rln % n : 0, c, rln < nrecn, D, nxt);
    }
#pragma unroll
    for (int u = 0; u < (RW * kH * DM + 63) / 64; ++u) {
      const int e = lane + 64 * u, rr = e / (H * D), kk = e - rr * (H * D);
      if (e < RW * H * D) L.qt[rr * QP + kk] = qv[u];
    }
    float beta[kH];
#pragma unroll
    for (int h = 0; h < kH; ++h) beta[h] = group_sum<CP>(bacc[h], nullptr);
    gath_finish<DM>(p, preW, preb, cur);
    const bool ok = cur.k.s >= 0;
    wave_sync();
    float lg[kH], mx[kH], a[kH];
#pragma unroll
    for (int h = 0; h < kH; ++h) {
      float acc = 0.0f;
      const float* qt = L.qt + slot * QP + h * D;
#pragma unroll
      for (int d = 0; d < DM; ++d)
        if (d < D) acc += qt[d] * cur.x[d];
      lg[h] = (ok && h < H) ? (acc + beta[h]) * p.scale : -INFINITY;
      mx[h] = group_max<CP>(lg[h], nullptr);
    }
#pragma unroll
    for (int h = 0; h < kH; ++h) {
      const float ex = ok && h < H ? expf(lg[h] - mx[h]) : 0.0f;
      const float sm = group_sum<CP>(ex, nullptr);
      a[h] = ok && h < H ? ex / sm : 0.0f;
      if (active && c < C && h < H && p.attn) p.attn[(row * H + h) * C + c] = a[h];
    }
    if (c < CR) {
#pragma unroll
      for (int d = 0; d < DM; ++d) L.xs[lr * XP + d] = cur.x[d];
#pragma unroll
      for (int h = 0; h < kH; ++h) L.a[lr * kH + h] = a[h];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) L.ef[lr * 4 + jj] = cur.ef[jj];
    }
    wave_sync();
    if (active) {
      const int base = slot * CR;
      float* out = p.xcat + row * W;
      for (int o = c; o < W; o += CP) {
        float acc = 0.0f;
        if (o < H * D) {
          const int h = o / D, d = o - h * D;
          #pragma unroll 8
          for (int cc = 0; cc < CR; ++cc) acc += L.a[(base + cc) * kH + h] * L.xs[(base + cc) * XP + d];
        } else if (o < H * D + 4 * H) {
          const int q = o - H * D, h = q >> 2, jj = q & 3;
          #pragma unroll 8
          for (int cc = 0; cc < CR; ++cc) acc += L.a[(base + cc) * kH + h] * L.ef[(base + cc) * 4 + jj];
        } else {
          const int h = o - H * D - 4 * H;
          #pragma unroll 8
          for (int cc = 0; cc < CR; ++cc) acc += L.a[(base + cc) * kH + h];
        }
        out[o] = acc;
      }
    }
    wave_sync();
    cur = nxt;
  }
}

template <int CP, int DM>
__global__ __launch_bounds__(256) void attn_bwd_wave_kernel(dgppo_gnn_attn_args p, int gpw, int64_t nitems,
                                                            int wfloats) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  using CV = WaveCarve<CP, DM>;
  constexpr int RW = CV::RW, XP = CV::XP, QP = CV::QP, GP = CV::GP;
  constexpr int NTD = (DM + 31) / 32;
  const int n = p.n_agents, D = p.D, F = p.F, C = p.C, H = p.H;
  const int CR = cand_rows(C, CP);
  float* preW = lds;
  float* preb = preW + kD0 * DM;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  CV L(lds + wave_header_floats<DM>() + wave * wfloats, CR, gpw * n * DM, true);
  const int W = H * (D + 5);
  const int slot = lane / CP, c = lane % CP;
  const int lr = slot * CR + c;
  const bool agent_mode = p.xa != nullptr;
  const bool want_dxa = agent_mode && p.dxa != nullptr;
  const bool want_pre = agent_mode && p.pre_W != nullptr && p.dpre_part != nullptr;
  typedef float f32x16 __attribute__((ext_vector_type(16)));
  f32x16 pacc[NTD];
#pragma unroll
  for (int q = 0; q < NTD; ++q)
#pragma unroll
    for (int r = 0; r < 16; ++r) pacc[q][r] = 0.0f;
  stage_pre(p, preW, preb, DM);
  __syncthreads();
  const int64_t gw = (int64_t)blockIdx.x * 4 + wave, nw = (int64_t)gridDim.x * 4;
  for (int64_t item = gw; item < nitems; item += nw) {
    const int64_t g0 = item * gpw;
    const int ng = (int)((int64_t)p.G - g0 < gpw ? (int64_t)p.G - g0 : gpw);
    const int nrec = ng * n;
    if (want_dxa) {
      for (int e = lane; e < ng * n * D; e += 64) L.cb[e] = 0.0f;
    }
    for (int r0 = 0; r0 < nrec; r0 += RW) {
      const int rl = r0 + slot;
      const bool active = rl < nrec;
      const int gl = active ? rl / n : 0;
      const int64_t g = g0 + gl;
      const int i = active ? rl % n : 0;
      const int64_t row = g0 * n + rl;
      const Cand k = active ? candidate(p, g, i, c) : Cand{-1, -1};
      const bool ok = k.s >= 0;
      float x[DM], x0[kD0];
      bool via_pre;
      gather_sender<DM>(p, g, k.s, ok, D, preW, preb, x, x0, via_pre);
      float ef[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) ef[j] = ok ? p.ef[g * p.ef_gstride + (int64_t)k.e * 4 + j] : 0.0f;
      float a[kH];
#pragma unroll
      for (int h = 0; h < kH; ++h) a[h] = (ok && h < H) ? p.attn[(row * H + h) * C + c] : 0.0f;
      for (int e = lane; e < RW * H * D; e += 64) {
        const int rr = e / (H * D), kk = e - rr * (H * D);
        if (r0 + rr < nrec) L.qt[rr * QP + kk] = p.qt[(g0 * n + r0 + rr) * qt_ld(p) + kk];
      }
      for (int e = lane; e < RW * W; e += 64) {  // dxcat row -> [dxbar | debar | dsig] at aligned offsets
        const int rr = e / W, kk = e - rr * W;
        if (r0 + rr < nrec) {
          const int dst = kk < H * D ? kk : (kk < H * D + 4 * H ? kH * DM + (kk - H * D) : kH * DM + 12 + (kk - H * D - 4 * H));
          L.g[rr * GP + dst] = p.dxcat[(g0 * n + r0 + rr) * W + kk];
        }
      }
      wave_sync();
      const float* gv = L.g + slot * GP;
      float dl[kH], dbeta[kH];
#pragma unroll
      for (int h = 0; h < kH; ++h) {
        float da = 0.0f;
        if (ok && h < H) {
#pragma unroll
          for (int d = 0; d < DM; ++d)
            if (d < D) da += gv[h * D + d] * x[d];
#pragma unroll
          for (int j = 0; j < 4; ++j) da += gv[kH * DM + h * 4 + j] * ef[j];
          da += gv[kH * DM + 12 + h];
          if (p.da_add) da += p.da_add[(row * H + h) * C + c];
        }
        const float dot = group_sum<CP>(a[h] * da, nullptr);
        dl[h] = (ok && h < H) ? a[h] * (da - dot) * p.scale : 0.0f;
        dbeta[h] = group_sum<CP>(dl[h], nullptr);
      }
      if (active && c == 0)
        for (int h = 0; h < H; ++h) p.dbeta[row * dbeta_ld(p) + h] = dbeta[h];
      if (active)
        for (int kk = c; kk < H * F; kk += CP) {
          const int h = kk / F;
          if (p.dq) p.dq[row * H * F + kk] = (h == 0 ? dbeta[0] : h == 1 ? dbeta[1] : dbeta[2]) * p.bk[kk];
        }
      float contrib[DM];
      {
        const float* qt = L.qt + slot * QP;
#pragma unroll
        for (int d = 0; d < DM; ++d) {
          float v = 0.0f;
#pragma unroll
          for (int h = 0; h < kH; ++h)
            if (h < H && d < D) v += a[h] * gv[h * D + d] + dl[h] * qt[h * D + d];
          contrib[d] = v;
        }
      }
      if (c < CR) {
#pragma unroll
        for (int d = 0; d < DM; ++d) L.xs[lr * XP + d] = x[d];
#pragma unroll
        for (int h = 0; h < kH; ++h) L.a[lr * kH + h] = dl[h];
      }
      wave_sync();
      if (active) {
        const int base = slot * CR;
        for (int o = c; o < H * D; o += CP) {
          const int h = o / D, d = o - h * D;
          float acc = 0.0f;
          #pragma unroll 8
          for (int cc = 0; cc < CR; ++cc) acc += L.a[(base + cc) * kH + h] * L.xs[(base + cc) * XP + d];
          p.dqt[row * dqt_ld(p) + o] = acc;
        }
      }
      if (want_dxa) {  // agent senders: the wave's graph image, slots in fixed order
        const bool mine = ok && k.s < n;
        for (int ss = 0; ss < RW; ++ss) {
          wave_sync();
          if (slot == ss && mine) {
            float* dst = L.cb + ((int64_t)gl * n + k.s) * D;
#pragma unroll
            for (int d = 0; d < DM; ++d)
              if (d < D) dst[d] += contrib[d];
          }
        }
      }
      if (want_pre) {  // transformed senders: x0s^T (dz) into the wave's MFMA accumulators
        wave_sync();   // dqt readers of xs are done: xs now holds dz
        if (c < CR) {
#pragma unroll
          for (int d = 0; d < DM; ++d) L.xs[lr * XP + d] = via_pre && x[d] > 0.0f ? contrib[d] : 0.0f;
#pragma unroll
          for (int kk = 0; kk < kD0; ++kk) L.x0s[lr * (kD0 + 1) + kk] = via_pre ? x0[kk] : 0.0f;
          L.x0s[lr * (kD0 + 1) + kD0] = via_pre ? 1.0f : 0.0f;
        }
        wave_sync();
        const int rows = RW * CR;
        for (int t0 = 0; t0 < rows; t0 += 2) {
          const int tr = t0 + (lane >> 5);
          const int m = lane & 31;
          const float av = (tr < rows && m <= kD0) ? L.x0s[tr * (kD0 + 1) + m] : 0.0f;
#pragma unroll
          for (int q = 0; q < NTD; ++q) {
            const int d = q * 32 + m;
            const float bv = (tr < rows && d < DM) ? L.xs[tr * XP + d] : 0.0f;
            pacc[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, pacc[q], 0, 0, 0);
          }
        }
      }
      wave_sync();
    }
    if (want_dxa) {
      wave_sync();
      for (int e = lane; e < ng * n * D; e += 64) {
        const int gg = e / (n * D), kk = e - gg * (n * D);
        p.dxa[(g0 + gg) * p.dxa_gstride + kk] += L.cb[e];
      }
      wave_sync();
    }
  }
  if (want_pre) {  // combine the 4 waves' accumulators in fixed order, write this block's partial
    __syncthreads();
    float* red = lds + wave_header_floats<DM>();  // wave regions are free now
    constexpr int RP = 32 * NTD + 1;
    for (int w = 0; w < 4; ++w) {
      if (wave == w) {
#pragma unroll
        for (int q = 0; q < NTD; ++q)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
            float* dst = red + m * RP + q * 32 + (lane & 31);
            *dst = (w == 0 ? 0.0f : *dst) + pacc[q][r];
          }
      }
      __syncthreads();
    }
    const int PK = p.D0 * D + D;
    for (int o = threadIdx.x; o < PK; o += 256) {
      const int m = o < p.D0 * D ? o / D : kD0;
      const int d = o < p.D0 * D ? o - m * D : o - p.D0 * D;
      p.dpre_part[(int64_t)blockIdx.x * PK + o] = red[m * RP + d];
    }
  }
}

int pick_cp(int C) {
  int cp = 8;
  while (cp < C) cp <<= 1;
  return cp;
}

// ================================================================================================
// Forward, row-block form (C <= 32, H = 3, D <= 32, sender table given): a 256-thread workgroup
// takes 16 consecutive receiver rows, each wave two rows per sub-round (32 lanes = candidates) for
// two sub-rounds.  The rows' qt and beta sit in LDS; every lane's sender row and edge features for
// both sub-rounds are gathered up front (one exposed gather latency per block); in agent mode the
// never-receiving senders' relu(x_raw pre_W + pre_b) is one MFMA tile product per wave and
// sub-round; the softmax reductions are DPP lane shuffles; the weighted sums read float4 rows.
// ================================================================================================
namespace fwd2 {
constexpr int kRows = 16, kSR = 2, kQP = 100;
// xs row pitch: x (DM floats; the pre-transform writes 32) then the edge features at column EC
template <int DM>
struct Pitch {
  // XSP = EC + 4 (12 / 20 / 36 floats): every 16 consecutive lanes' row starts fall on distinct 4-bank groups,
  // so the per-lane float4 row reads and the pre-transform's strided accesses are bank-conflict free (a 40-float
  // pitch put lanes L and L + 8 on the same banks)
  static constexpr int EC = DM <= 8 ? 8 : (DM <= 16 ? 16 : 32), XSP = EC + 4, AW = 64 * (XSP + 4);
};
template <int DM>
constexpr size_t lds_floats() {
  return (size_t)kRows * kQP + kD0 * 32 + 32 + 4 * Pitch<DM>::AW;
}
}  // namespace fwd2

// Register form of the row-block forward (round 6: the LDS-staged form it replaced is removed): each lane's pair row x stays in registers (pre mode: relu(x_raw pre_W + pre_b) by VALU
// FMAs against the LDS-resident pre_W), and the attention-weighted sums over the row's 32 candidates --
// xbar_h per head, [ebar_h | sig_h] of all heads -- are transposed DPP reductions (lanes::treduce32)
// whose totals each lane stores to its row of xcat.  LDS holds only the block's qt / beta rows and
// pre_W (7.5 KB instead of 56 KB), so occupancy is set by registers.
template <int DM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8))) void attn_fwd2r_kernel(
    dgppo_gnn_attn_args p) {
  using lanes::f32x4;
  constexpr int kRows = fwd2::kRows, kSR = fwd2::kSR, kQP = fwd2::kQP;
  static_assert(DM == 8 || DM == 16 || DM == 32, "fwd2r instantiations");
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* qts = lds;                 // [16][100]: qt_h (32-float stride per head) | beta_h at 96 + h
  float* preW = qts + kRows * kQP;  // [8][32]
  float* preb = preW + kD0 * 32;    // [32]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int slot = lane >> 5, c = lane & 31;
  const int n = p.n_agents, D = p.D, C = p.C, H = kH;
  const int nrows = p.G * n;
  const int row0 = blockIdx.x * kRows;
  const bool agent = p.xa != nullptr;
  const bool pre = DM == 32 && agent && p.pre_W != nullptr;
  // ---- stage qt (zero padded per head), beta_h = q_h . bk_h, pre weights
  for (int e = threadIdx.x; e < kRows * 96; e += 256) {
    const int r = e / 96, k = e - r * 96, h = k >> 5, d = k & 31;
    qts[r * kQP + k] = (row0 + r < nrows && d < D) ? p.qt[(int64_t)(row0 + r) * qt_ld(p) + h * D + d] : 0.0f;
  }
  {
    const int r = threadIdx.x >> 4, j = threadIdx.x & 15;
    const bool act = row0 + r < nrows;
#pragma unroll
    for (int h = 0; h < kH; ++h) {
      float acc = 0.0f;
      if (act) acc = q_dot_bk(p, (int64_t)(row0 + r), h, j, 16);
      acc = lanes::sum16(acc);
      if (j == 0) qts[r * kQP + 96 + h] = acc;
    }
  }
  if (pre) {
    const int k = threadIdx.x >> 5, d = threadIdx.x & 31;
    preW[threadIdx.x] = (k < p.D0 && d < D) ? p.pre_W[k * D + d] : 0.0f;
    if (threadIdx.x < 32) preb[threadIdx.x] = threadIdx.x < D ? p.pre_b[threadIdx.x] : 0.0f;
  }
  __syncthreads();
  const int TQ = (D + 3) >> 2, W = H * (D + 5);
  constexpr int NEV = kH * 5;
  // one sub-round at a time, gathers included: at 4 waves per SIMD the other waves hide the gather latency,
  // and a prefetch of the next sub-round's 32-float rows would not fit the register budget
#pragma unroll 1
  for (int sr = 0; sr < kSR; ++sr) {
    const int rl = 2 * wave + 8 * sr + slot;
    const int row = row0 + rl;
    const bool active = row < nrows;
    float x[DM];
    f32x4 ef;
    int s = -1;
    {
      const int g = active ? row / n : 0;
      const int i = active ? row - g * n : 0;
      int e = 0;
      if (active && c < C) {
        e = p.cand[i * C + c];
        s = p.sidx[(int64_t)row * C + c];
      }
      const bool okg = s >= 0;
      const float* er = p.ef + (int64_t)g * p.ef_gstride + (int64_t)(okg ? e : 0) * 4;
#pragma unroll
      for (int j = 0; j < 4; ++j) ef[j] = okg ? er[j] : 0.0f;
      if (!agent) {
        load_row<DM>(p.x + (int64_t)g * p.x_gstride + (int64_t)(okg ? s : 0) * D, D, okg, x);
      } else if (!okg || s < n) {
        load_row<DM>(p.xa + (int64_t)g * p.xa_gstride + (int64_t)(okg ? s : 0) * D, D, okg, x);
      } else {
        const float* xr = p.x + (int64_t)g * p.x_gstride + (int64_t)s * p.D0;
#pragma unroll
        for (int kk = 0; kk < DM; ++kk) x[kk] = (kk < kD0 && kk < p.D0) ? xr[kk < kD0 ? kk : 0] : 0.0f;
      }
    }
    const bool ok = s >= 0;
    if (pre && ok && s >= n) {  // never-receiving sender: relu(x_raw pre_W + pre_b) in place
      float xr[kD0];
#pragma unroll
      for (int k = 0; k < kD0; ++k) xr[k] = x[k];
#pragma unroll
      for (int q = 0; q < DM / 4; ++q) {
        const f32x4 b = *(const f32x4*)(preb + 4 * q);
        x[4 * q] = b[0];
        x[4 * q + 1] = b[1];
        x[4 * q + 2] = b[2];
        x[4 * q + 3] = b[3];
      }
#pragma unroll
      for (int k = 0; k < kD0; ++k)
#pragma unroll
        for (int q = 0; q < DM / 4; ++q) {
          const f32x4 w = *(const f32x4*)(preW + k * 32 + 4 * q);
          x[4 * q] += xr[k] * w[0];
          x[4 * q + 1] += xr[k] * w[1];
          x[4 * q + 2] += xr[k] * w[2];
          x[4 * q + 3] += xr[k] * w[3];
        }
#pragma unroll
      for (int d = 0; d < DM; ++d) x[d] = x[d] > 0.0f ? x[d] : 0.0f;
    }
    // logits, softmax over the row's candidates, attention weights out
    const float* qt = qts + rl * kQP;
    float aw[kH];
#pragma unroll
    for (int h = 0; h < kH; ++h) {
      float acc = 0.0f;
#pragma unroll
      for (int q = 0; q < DM / 4; ++q)
        if (q < TQ) {
          const f32x4 qq = ((const f32x4*)(qt + 32 * h))[q];
          acc += x[4 * q] * qq[0] + x[4 * q + 1] * qq[1] + x[4 * q + 2] * qq[2] + x[4 * q + 3] * qq[3];
        }
      const float lg = ok ? (acc + qt[96 + h]) * p.scale : -INFINITY;
      const float mx = lanes::max32(lg);
      const float ex = ok ? expf(lg - mx) : 0.0f;
      const float sm = lanes::sum32(ex);
      aw[h] = ok ? ex / sm : 0.0f;
      if (active && c < C && p.attn) p.attn[((int64_t)row * H + h) * C + c] = aw[h];
    }
    float* o = p.xcat + (int64_t)row * W;
    // xbar_h = sum_c a_h x_c
#pragma unroll
    for (int h = 0; h < kH; ++h) {
      float v[DM];
#pragma unroll
      for (int d = 0; d < DM; ++d) v[d] = aw[h] * x[d];
      int cnt;
      const int base = lanes::treduce32(v, cnt);
#pragma unroll
      for (int j = 0; j < lanes::tr_final<DM>(); ++j) {
        const int q = base + j;
        if (active && j < cnt && q < D) o[h * D + q] = v[j];
      }
    }
    // [ebar_h (4) | sig_h] of the three heads
    {
      float v[NEV];
#pragma unroll
      for (int h = 0; h < kH; ++h) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[h * 5 + j] = aw[h] * ef[j];
        v[h * 5 + 4] = aw[h];
      }
      int cnt;
      const int base = lanes::treduce32(v, cnt);
#pragma unroll
      for (int j = 0; j < lanes::tr_final<NEV>(); ++j) {
        const int q = base + j;
        const int h = q / 5, k = q - h * 5;
        if (active && j < cnt) o[k < 4 ? H * D + 4 * h + k : H * D + 4 * H + h] = v[j];
      }
    }
  }
}

bool fwd2_ok(const dgppo_gnn_attn_args* p) {
  static const bool off = [] {
    const char* e = getenv("DGPPO_ATTN_FWD1");
    return e && atoi(e) != 0;
  }();
  return !off && p->H == kH && p->C <= 32 && p->D <= 32 && p->F <= 64 && p->sidx != nullptr &&
         (int64_t)p->G * p->n_agents < (int64_t)1 << 30 && (p->xa == nullptr || p->D0 <= kD0);
}

void fwd2_launch(const dgppo_gnn_attn_args* p, hipStream_t s) {
  const int64_t rows = (int64_t)p->G * p->n_agents;
  const unsigned grid = (unsigned)((rows + fwd2::kRows - 1) / fwd2::kRows);
  const bool no_pre = !(p->xa && p->pre_W);
  const size_t bytes = ((size_t)fwd2::kRows * fwd2::kQP + kD0 * 32 + 32) * sizeof(float);
  if (p->D <= 8 && no_pre) hipLaunchKernelGGL(attn_fwd2r_kernel<8>, dim3(grid), dim3(256), bytes, s, *p);
  else if (p->D <= 16 && no_pre) hipLaunchKernelGGL(attn_fwd2r_kernel<16>, dim3(grid), dim3(256), bytes, s, *p);  // e.g. Omni's 10-wide first layer
  else hipLaunchKernelGGL(attn_fwd2r_kernel<32>, dim3(grid), dim3(256), bytes, s, *p);
}

// ================================================================================================
// Backward, row-block form (same scope as the row-block forward; agent mode, or full mode without
// dx).  A persistent workgroup walks blocks of (16 / n) whole graphs; each wave two rows per
// sub-round.  Per pair: da_h = dxbar_h . x + debar_h . ef + dsig_h, dl_h = a_h (da_h - sum_c a_h
// da_h) scale (DPP reductions), dbeta_h = sum_c dl_h, dqt_h = sum_c dl_h x (float4 LDS sums), and
// the sender gradient contrib = sum_h a_h dxbar_h + dl_h qt_h.  Agent senders' contribs go to an
// LDS image [row][agent][d] that is summed over receivers in fixed order per block; the
// transformed senders' dz = contrib * (x > 0) feed a 16x16x4 MFMA accumulation of
// [x_raw | 1]^T dz (the pre layer's weight and bias gradient), combined over waves in fixed order
// into one partial row per workgroup.  Deterministic: no atomics.
// ================================================================================================
namespace bwd2 {
constexpr int kRows = 16, kSR = 2, kMaxBlocks = 1024;
// per-head stride HS of the qt / dxbar rows, row pitches, xs pitch (x | x_raw | 1 in pre mode)
template <int DM>
struct Lay {
  static constexpr int HS = DM <= 8 ? 8 : (DM <= 16 ? 16 : 32), QP = 3 * HS + 4, GP = 3 * HS + 16;
  static constexpr int XSP = DM <= 8 ? 12 : (DM <= 16 ? 20 : 44), AW = 64 * (XSP + 4);
};
template <int DM>
size_t lds_floats(int n, int D) {
  using L = Lay<DM>;
  return (size_t)kRows * (L::QP + L::GP) + kD0 * 32 + 32 + 4 * L::AW + (size_t)kRows * n * D;
}
}  // namespace bwd2

// Register form of the row-block backward (round 6: the LDS-staged form it replaced is removed): a
// lane's pair row x stays in registers (pre mode: relu(x_raw pre_W + pre_b) by VALU FMAs against the
// LDS-resident pre_W), da / dl / dbeta and the sender gradient are lane-local math against the row's
// LDS-staged dxbar / qt, dqt_h = sum_c dl_h x_c is one transposed DPP reduction per head, and the pre
// layer's gradient [x_raw | 1]^T dz goes through the MFMA in four 16-pair chunks staged in a 2.8 KB
// per-wave area (instead of a 64-pair image).  The agent-sender image and its fixed-order sums are the
// same as the LDS form.
#ifndef DGPPO_DIAG_BWD
#define DGPPO_DIAG_BWD 0  // diagnostic builds only (time attribution, results invalid): 1 no pre transform, 2 no dqt, 4 no pre gradient
#endif
namespace bwd2r {
constexpr int kPS = 44;  // chunk staging row: dz (0..31) | x_raw (32..39) | 1 (40)
template <int DM>
size_t lds_floats(int n, int D) {
  using L = bwd2::Lay<DM>;
  return (size_t)bwd2::kRows * (L::QP + L::GP) + kD0 * 32 + 32 + 4 * 16 * kPS + (size_t)bwd2::kRows * n * D +
         4 * 256;
}
}  // namespace bwd2r

template <int DM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 8))) void attn_bwd2r_kernel(
    dgppo_gnn_attn_args p, int64_t nblk) {
  using lanes::f32x4;
  using lanes::wave_sync;
  using LY = bwd2::Lay<DM>;
  constexpr int kRows = bwd2::kRows, kSR = bwd2::kSR, HS = LY::HS, kQP = LY::QP, kGP = LY::GP;
  constexpr int kPS = bwd2r::kPS;
  static_assert(DM == 8 || DM == 16 || DM == 32, "bwd2r instantiations");
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* qts = lds;                 // [16][QP]: qt_h (HS stride per head)
  float* gs = qts + kRows * kQP;    // [16][GP]: dxbar_h (HS stride) | debar (3HS..+12) | dsig (3HS+12..+3)
  float* preW = gs + kRows * kGP;   // [8][32]
  float* preb = preW + kD0 * 32;    // [32]
  float* stg = preb + 32;           // per wave [16][kPS]: pre-gradient chunk staging
  float* cbi = stg + 4 * 16 * kPS;  // [rows][n][D] agent-sender contributions
  int* pse = reinterpret_cast<int*>(cbi + bwd2::kRows * p.n_agents * p.D);  // [2 sub-rounds][s, e][256]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i16 = lane & 15, kq = lane >> 4;
  const int slot = lane >> 5, c = lane & 31;
  const int n = p.n_agents, D = p.D, F = p.F, C = p.C, H = kH;
  const int gpb = kRows / n;
  const bool agent = p.xa != nullptr;
  const bool pre = DM == 32 && agent && p.pre_W != nullptr;
  const bool want_dxa = agent && p.dxa != nullptr;
  const bool want_pre = pre && p.dpre_part != nullptr;
  if (pre) {
    const int k = threadIdx.x >> 5, d = threadIdx.x & 31;
    preW[threadIdx.x] = (k < p.D0 && d < D) ? p.pre_W[k * D + d] : 0.0f;
    if (threadIdx.x < 32) preb[threadIdx.x] = threadIdx.x < D ? p.pre_b[threadIdx.x] : 0.0f;
  }
  __syncthreads();
  f32x4 gacc[2] = {f32x4{0.0f, 0.0f, 0.0f, 0.0f}, f32x4{0.0f, 0.0f, 0.0f, 0.0f}};  // [x_raw | 1]^T dz
  float* ws = stg + wave * 16 * kPS;
  const int TQ = (D + 3) >> 2, W = H * (D + 5);
  // A block's staged rows (qt, dxcat) and its pairs' senders / candidates are loaded into registers with every
  // load issued before the first use: one memory round trip per block (a runtime-bounded staging loop waits for
  // each load before its LDS store: 13 round trips per block at DM = 32; attn_bwd2r<32> 405 -> 380 us).  Issuing
  // the next block's loads before this block's epilogue instead spilled at DM = 32 and measured slower (579 us).
  static_assert(kSR == 2, "two sub-rounds per block");
  constexpr int NQS = (kRows * 3 * HS + 255) / 256, NGS = (kRows * kGP + 255) / 256, NXS = (kRows * DM + 255) / 256;
  float qv[NQS], gw[NGS];
  int sv[kSR], ev[kSR];
  // (tid: threadIdx.x behind an empty asm, so that the per-lane index math below is redone per block instead of
  // being hoisted out of the block loop as 64-bit addresses that then spill)
  auto load_block = [&](int64_t b, int tid) {
    const int64_t bg0 = b * gpb;
    const int bnrec = (int)((int64_t)p.G - bg0 < gpb ? (int64_t)p.G - bg0 : gpb) * n;
    const int64_t brow0 = bg0 * n;
    const int32_t* sb = p.sidx + brow0 * C;
    const float* qb = p.qt + brow0 * qt_ld(p);
    const float* xb = p.dxcat + brow0 * W;
    const int qld = (int)qt_ld(p);
#pragma unroll
    for (int sr = 0; sr < kSR; ++sr) {
      const int rl = 2 * (tid >> 6) + 8 * sr + ((tid >> 5) & 1), cc = tid & 31;
      const bool act = rl < bnrec;
      const int i = act ? rl - (rl / n) * n : 0;
      int s = -1, e = 0;
      if (act && cc < C) {
        e = p.cand[i * C + cc];
        s = sb[rl * C + cc];
      }
      sv[sr] = s;
      ev[sr] = e;
    }
#pragma unroll
    for (int k = 0; k < NQS; ++k) {
      const int e = tid + 256 * k;
      const int r = e / (3 * HS), kk = e - r * (3 * HS), h = kk / HS, d = kk - h * HS;
      qv[k] = (e < kRows * 3 * HS && r < bnrec && d < D) ? qb[r * qld + h * D + d] : 0.0f;
    }
#pragma unroll
    for (int k = 0; k < NGS; ++k) {
      const int e = tid + 256 * k;
      const int r = e / kGP, kk = e - r * kGP;
      int src = -1;
      if (kk < 3 * HS) src = (kk % HS) < D ? (kk / HS) * D + (kk % HS) : -1;
      else if (kk < 3 * HS + 12) src = H * D + (kk - 3 * HS);
      else if (kk < 3 * HS + 15) src = H * D + 4 * H + (kk - 3 * HS - 12);
      gw[k] = (e < kRows * kGP && r < bnrec && src >= 0) ? xb[r * W + src] : 0.0f;
    }
  };
  for (int64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    load_block(blk, tid);
    const int64_t g0 = blk * gpb;
    const int ng = (int)((int64_t)p.G - g0 < gpb ? (int64_t)p.G - g0 : gpb);
    const int nrec = ng * n;
    const int64_t row0 = g0 * n;
    // ---- block staging from the registers: qt rows, dxcat rows (split at aligned offsets), agent image cleared
#pragma unroll
    for (int k = 0; k < NQS; ++k) {
      const int e = tid + 256 * k;
      const int r = e / (3 * HS), kk = e - r * (3 * HS);
      if (e < kRows * 3 * HS) qts[r * kQP + kk] = qv[k];
    }
#pragma unroll
    for (int k = 0; k < NGS; ++k) {
      const int e = tid + 256 * k;
      if (e < kRows * kGP) gs[e] = gw[k];
    }
    if (want_dxa)
      for (int e = threadIdx.x; e < kRows * n * D; e += 256) cbi[e] = 0.0f;
#pragma unroll
    for (int sr = 0; sr < kSR; ++sr) {  // (through LDS: 4 fewer registers live across the sub-rounds)
      pse[(2 * sr) * 256 + tid] = sv[sr];
      pse[(2 * sr + 1) * 256 + tid] = ev[sr];
    }
    __syncthreads();
#pragma unroll 1
    for (int sr = 0; sr < kSR; ++sr) {
      const int rl = 2 * wave + 8 * sr + slot;
      const bool active = rl < nrec;
      const int64_t row = row0 + rl;
      // ---- the pair: sender, edge, attention, sender row
      const int gl = active ? rl / n : 0;
      const int64_t g = g0 + gl;
      const int s = pse[(2 * sr) * 256 + tid], e = pse[(2 * sr + 1) * 256 + tid];
      const bool ok = s >= 0;
      float av[kH];
#pragma unroll
      for (int h = 0; h < kH; ++h) av[h] = ok ? p.attn[(row * H + h) * C + c] : 0.0f;
      f32x4 ef;
      const float* er = p.ef + g * p.ef_gstride + (int64_t)(ok ? e : 0) * 4;
#pragma unroll
      for (int j = 0; j < 4; ++j) ef[j] = ok ? er[j] : 0.0f;
      float x[DM];
      if (!agent) {
        load_row<DM>(p.x + g * p.x_gstride + (int64_t)(ok ? s : 0) * D, D, ok, x);
      } else if (!ok || s < n) {
        load_row<DM>(p.xa + g * p.xa_gstride + (int64_t)(ok ? s : 0) * D, D, ok, x);
      } else {
        const float* xr = p.x + g * p.x_gstride + (int64_t)s * p.D0;
#pragma unroll
        for (int k = 0; k < DM; ++k) x[k] = (k < kD0 && k < p.D0) ? xr[k < kD0 ? k : 0] : 0.0f;
      }
      const bool viapre = pre && ok && s >= n;
      float xraw[kD0];
#pragma unroll
      for (int k = 0; k < kD0; ++k) xraw[k] = viapre ? x[k < DM ? k : 0] : 0.0f;
      if (viapre && !(DGPPO_DIAG_BWD & 1)) {  // relu(x_raw pre_W + pre_b)
#pragma unroll
        for (int q = 0; q < DM / 4; ++q) {
          const f32x4 b = *(const f32x4*)(preb + 4 * q);
          x[4 * q] = b[0];
          x[4 * q + 1] = b[1];
          x[4 * q + 2] = b[2];
          x[4 * q + 3] = b[3];
        }
#pragma unroll
        for (int k = 0; k < kD0; ++k)
#pragma unroll
          for (int q = 0; q < DM / 4; ++q) {
            const f32x4 w = *(const f32x4*)(preW + k * 32 + 4 * q);
            x[4 * q] += xraw[k] * w[0];
            x[4 * q + 1] += xraw[k] * w[1];
            x[4 * q + 2] += xraw[k] * w[2];
            x[4 * q + 3] += xraw[k] * w[3];
          }
#pragma unroll
        for (int d = 0; d < DM; ++d) x[d] = x[d] > 0.0f ? x[d] : 0.0f;
      }
      // ---- softmax backward
      const float* gv = gs + rl * kGP;
      float dl[kH], dbeta[kH];
#pragma unroll
      for (int h = 0; h < kH; ++h) {
        float da = 0.0f;
#pragma unroll
        for (int q = 0; q < DM / 4; ++q)
          if (q < TQ) {
            const f32x4 gq = ((const f32x4*)(gv + HS * h))[q];
            da += x[4 * q] * gq[0] + x[4 * q + 1] * gq[1] + x[4 * q + 2] * gq[2] + x[4 * q + 3] * gq[3];
          }
#pragma unroll
        for (int j = 0; j < 4; ++j) da += gv[3 * HS + 4 * h + j] * ef[j];
        da += gv[3 * HS + 12 + h];
        if (p.da_add && ok) da += p.da_add[(row * H + h) * C + c];
        da = ok ? da : 0.0f;
        const float dot = lanes::sum32(av[h] * da);
        dl[h] = ok ? av[h] * (da - dot) * p.scale : 0.0f;
        dbeta[h] = lanes::sum32(dl[h]);
      }
      if (active) {
        if (c < kH) p.dbeta[row * dbeta_ld(p) + c] = c == 0 ? dbeta[0] : c == 1 ? dbeta[1] : dbeta[2];
        for (int kk = c; kk < H * F; kk += 32) {
          const int h = kk / F;
          if (p.dq) p.dq[row * H * F + kk] = (h == 0 ? dbeta[0] : h == 1 ? dbeta[1] : dbeta[2]) * p.bk[kk];
        }
      }
      // ---- dqt_h = sum_c dl_h x_c (transposed reduction per head)
#pragma unroll
      for (int h = 0; h < kH; ++h) {
        float v[DM];
#pragma unroll
        for (int d = 0; d < DM; ++d) v[d] = dl[h] * x[d];
        int cnt;
        const int base = lanes::treduce32(v, cnt);
        float* o = p.dqt + row * dqt_ld(p) + h * D;
#pragma unroll
        for (int j = 0; j < lanes::tr_final<DM>(); ++j) {
          const int q = base + j;
          if (active && j < cnt && q < D && !(DGPPO_DIAG_BWD & 2)) o[q] = v[j];
        }
      }
      // ---- sender gradient of this pair: sum_h a_h dxbar_h + dl_h qt_h
      f32x4 cq[DM / 4];
      const float* qt = qts + rl * kQP;
#pragma unroll
      for (int q = 0; q < DM / 4; ++q) {
        cq[q] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        if (q < TQ)
#pragma unroll
          for (int h = 0; h < kH; ++h)
            cq[q] += av[h] * ((const f32x4*)(gv + HS * h))[q] + dl[h] * ((const f32x4*)(qt + HS * h))[q];
      }
      if (want_dxa && ok && s < n) {
        float* dst = cbi + (rl * n + s) * D;
        if ((D & 3) == 0) {
#pragma unroll
          for (int q = 0; q < DM / 4; ++q)
            if (q < TQ) ((f32x4*)dst)[q] = cq[q];
        } else {
#pragma unroll
          for (int q = 0; q < DM / 4; ++q)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (4 * q + j < D) dst[4 * q + j] = cq[q][j];
        }
      }
      // ---- pre layer gradient: gacc[ct] += [x_raw | 1]^T dz over the wave's pairs in 16-pair chunks staged in the
      // wave's area.  Only the pairs whose sender went through the pre layer carry a nonzero dz (never-receivers:
      // 16 of a receiver's 24 candidates at n = 8, 9 of 17 for own-goal envs), so they are compacted to the front
      // (ballot rank) and the chunk loop runs over ceil(count / 16) chunks, not 4; the other lanes fill the last
      // chunk's free slots with zero rows (lane l: chunk pos >> 4, slot pos & 15)
      if (want_pre && !(DGPPO_DIAG_BWD & 4)) {
        const uint64_t vb = __ballot(viapre);
        const int nvia = __popcll(vb);
        const int pos = viapre ? lanes::mbcnt64(vb) : nvia + lanes::mbcnt64(~vb);
        const int nch = (nvia + 15) >> 4;
#pragma unroll 1
        for (int ch = 0; ch < nch; ++ch) {
          if ((pos >> 4) == ch) {
            float* sp = ws + (pos & 15) * kPS;
#pragma unroll
            for (int q = 0; q < DM / 4; ++q) {
              f32x4 dz;
#pragma unroll
              for (int j = 0; j < 4; ++j) dz[j] = (viapre && x[4 * q + j] > 0.0f) ? cq[q][j] : 0.0f;
              ((f32x4*)sp)[q] = dz;
            }
            ((f32x4*)(sp + 32))[0] = f32x4{xraw[0], xraw[1], xraw[2], xraw[3]};
            ((f32x4*)(sp + 32))[1] = f32x4{xraw[4], xraw[5], xraw[6], xraw[7]};
            sp[40] = viapre ? 1.0f : 0.0f;
          }
          wave_sync();
#pragma unroll
          for (int ks = 0; ks < 4; ++ks) {
            const int pp = 4 * ks + kq;
            const float a = i16 <= kD0 ? ws[pp * kPS + 32 + i16] : 0.0f;
#pragma unroll
            for (int ct = 0; ct < 2; ++ct)
              gacc[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, ws[pp * kPS + 16 * ct + i16], gacc[ct], 0, 0, 0);
          }
          wave_sync();
        }
      }
    }
    // the agent rows' current d xa (the epilogue adds this block's sums to them)
    float dxv[NXS];
#pragma unroll
    for (int k = 0; k < NXS; ++k) {
      const int e = tid + 256 * k;
      const int gl = e / (n * D), jd = e - gl * (n * D);
      dxv[k] = (want_dxa && e < nrec * D) ? p.dxa[(g0 + gl) * p.dxa_gstride + jd] : 0.0f;
    }
    __syncthreads();
    if (want_dxa) {  // agent j of graph gl: sum over its receivers i in order
#pragma unroll
      for (int k = 0; k < NXS; ++k) {
        const int e = tid + 256 * k;
        if (e < nrec * D) {
          const int gl = e / (n * D), jd = e - gl * (n * D), j = jd / D, d = jd - j * D;
          float acc = 0.0f;
          for (int i = 0; i < n; ++i) acc += cbi[((gl * n + i) * n + j) * D + d];
          p.dxa[(g0 + gl) * p.dxa_gstride + jd] = dxv[k] + acc;
        }
      }
    }
    __syncthreads();  // the sub-rounds' staging reads and the image sums are done before the next block's writes
  }
  if (want_pre) {  // fixed-order combine of the 4 waves' accumulators -> this workgroup's partial row
    float* red = stg;  // [16][33] (the staging area is free now)
    for (int w = 0; w < 4; ++w) {
      if (wave == w) {
#pragma unroll
        for (int ct = 0; ct < 2; ++ct)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float* dst = red + (4 * kq + i) * 33 + 16 * ct + i16;
            *dst = (w == 0 ? 0.0f : *dst) + gacc[ct][i];
          }
      }
      __syncthreads();
    }
    const int PK = p.D0 * D + D;
    for (int o = threadIdx.x; o < PK; o += 256) {
      const int m = o < p.D0 * D ? o / D : kD0;
      const int d = o < p.D0 * D ? o - m * D : o - p.D0 * D;
      p.dpre_part[(int64_t)blockIdx.x * PK + o] = red[m * 33 + d];
    }
  }
}

bool bwd2_ok(const dgppo_gnn_attn_args* p) {
  static const bool off = [] {
    const char* e = getenv("DGPPO_ATTN_BWD1");
    return e && atoi(e) != 0;
  }();
  if (off || p->H != kH || p->C > 32 || p->D > 32 || p->F > 64 || !p->sidx || p->n_agents > bwd2::kRows) return false;
  if (p->xa == nullptr) return p->dx == nullptr && p->D <= 32;
  if (p->D0 > kD0) return false;
  if (p->pre_W && p->D > 32) return false;
  return bwd2r::lds_floats<32>(p->n_agents, p->D) * sizeof(float) <= 160 * 1024;
}

int64_t bwd2_grid(const dgppo_gnn_attn_args* p, int64_t* nblk) {
  // persistent-grid cap: the resident workgroups, 3 per CU for the DM = 32 instantiation (47.7 KB of LDS, 3 waves per
  // SIMD), 6 per CU for the narrower ones (512 / 2048 / 4096 measured no different)
  const bool wide = p->D > 16 || (p->xa && p->pre_W);  // the DM = 32 instantiation
  const int64_t cap = wide ? 768 : 1536;
  const int gpb = bwd2::kRows / p->n_agents;
  *nblk = (p->G + gpb - 1) / gpb;
  return *nblk < cap ? *nblk : cap;
}

void bwd2_launch(const dgppo_gnn_attn_args* p, hipStream_t s) {
  int64_t nblk;
  const unsigned grid = (unsigned)bwd2_grid(p, &nblk);
  const bool no_pre = !(p->xa && p->pre_W);
  const int v = p->D <= 8 && no_pre ? 0 : (p->D <= 16 && no_pre ? 1 : 2);  // DM 8 / 16 / 32
  const size_t bytes = (v == 0   ? bwd2r::lds_floats<8>(p->n_agents, p->D)
                        : v == 1 ? bwd2r::lds_floats<16>(p->n_agents, p->D)
                                 : bwd2r::lds_floats<32>(p->n_agents, p->D)) *
                       sizeof(float);
  const void* fn = v == 0 ? (const void*)attn_bwd2r_kernel<8>
                          : (v == 1 ? (const void*)attn_bwd2r_kernel<16> : (const void*)attn_bwd2r_kernel<32>);
  if (bytes > 64 * 1024) allow_lds(fn);
  hipLaunchKernelGGL(reinterpret_cast<void (*)(dgppo_gnn_attn_args, int64_t)>(const_cast<void*>(fn)), dim3(grid),
                     dim3(256), bytes, s, *p, nblk);
}

struct Plan {
  int cp, dm, gpb;
  int64_t nblk, grid;
  size_t bytes;
  bool wave;
  int wfloats;
};

template <int CP, int DM>
Plan plan_t(const dgppo_gnn_attn_args* p, bool bwd) {
  constexpr int R = 256 / CP;
  Plan pl{CP, DM, 1, 0, 0, 0, false, 0};
  const bool full_dx = bwd && p->xa == nullptr && p->dx != nullptr;
  // measured on MI355X (LidarSpread n8, 16384 graphs): the block-synchronous forward and the
  // wave-independent backward are the faster pair; DGPPO_ATTN_WAVE=0/1 forces either family
  static const int wave_env = [] {
    const char* e = getenv("DGPPO_ATTN_WAVE");
    return e ? atoi(e) : -1;
  }();
  const bool use_wave = wave_env < 0 ? bwd : wave_env != 0;
  if (CP <= 64 && !full_dx && use_wave) {  // wave-independent kernels
    constexpr int RW = 64 / CP;
    pl.wave = true;
    pl.gpb = RW >= p->n_agents ? RW / p->n_agents : 1;  // graphs per wave item
    const int cbf = bwd ? pl.gpb * p->n_agents * DM : 0;
    pl.wfloats = (int)WaveCarve<CP, DM>::floats(cand_rows(p->C, CP), cbf, bwd);
    size_t tot = wave_header_floats<DM>() + 4 * (size_t)pl.wfloats;
    if (bwd && tot < (size_t)wave_header_floats<DM>() + 32 * (32 * ((DM + 31) / 32) + 1))
      tot = wave_header_floats<DM>() + 32 * (32 * ((DM + 31) / 32) + 1);
    pl.bytes = tot * sizeof(float);
    pl.nblk = (p->G + pl.gpb - 1) / pl.gpb;  // wave items
    const int64_t blocks = (pl.nblk + 3) / 4;
    pl.grid = blocks < kMaxBlocks ? blocks : kMaxBlocks;
    return pl;
  }
  const size_t fixed = bwd ? BwdCarve<CP, DM>::floats_fixed(cand_rows(p->C, CP), p->n_agents)
                           : Carve<CP, DM>::floats_fixed(cand_rows(p->C, CP), false);
  pl.gpb = R >= p->n_agents ? R / p->n_agents : 1;
  const bool agent_mode = p->xa != nullptr;
  const bool dx = bwd && (agent_mode ? p->dxa != nullptr : p->dx != nullptr);
  const size_t per_graph = dx && !agent_mode ? (size_t)p->N * p->D : 0;
  while (pl.gpb > 1 && (fixed + pl.gpb * per_graph) * sizeof(float) > 64 * 1024) --pl.gpb;
  pl.bytes = (fixed + pl.gpb * per_graph) * sizeof(float);
  pl.nblk = (p->G + pl.gpb - 1) / pl.gpb;
  pl.grid = pl.nblk < kMaxBlocks ? pl.nblk : kMaxBlocks;
  return pl;
}

template <int DM>
Plan plan_cp(const dgppo_gnn_attn_args* p, bool bwd) {
  switch (pick_cp(p->C)) {
    case 8: return plan_t<8, DM>(p, bwd);
    case 16: return plan_t<16, DM>(p, bwd);
    case 32: return plan_t<32, DM>(p, bwd);
    case 64: return plan_t<64, DM>(p, bwd);
    default: return plan_t<128, DM>(p, bwd);
  }
}

Plan make_plan(const dgppo_gnn_attn_args* p, bool bwd) {
  if (p->D <= 8) return plan_cp<8>(p, bwd);
  if (p->D <= 32) return plan_cp<32>(p, bwd);
  return plan_cp<64>(p, bwd);
}

template <int CP, int DM>
void launch_t(const dgppo_gnn_attn_args* p, const Plan& pl, bool bwd, hipStream_t s) {
  if (pl.bytes > 64 * 1024)  // allow up to the CU's 160 KB
    allow_lds(bwd ? (const void*)attn_bwd_kernel<CP, DM> : (const void*)attn_fwd_kernel<CP, DM>);
  if (pl.wave) {
    if constexpr (CP <= 64) {
      if (pl.bytes > 64 * 1024)
        allow_lds(bwd ? (const void*)attn_bwd_wave_kernel<CP, DM> : (const void*)attn_fwd_wave_kernel<CP, DM>);
      if (bwd)
        hipLaunchKernelGGL((attn_bwd_wave_kernel<CP, DM>), dim3((unsigned)pl.grid), dim3(256), pl.bytes, s, *p,
                           pl.gpb, pl.nblk, pl.wfloats);
      else
        hipLaunchKernelGGL((attn_fwd_wave_kernel<CP, DM>), dim3((unsigned)pl.grid), dim3(256), pl.bytes, s, *p,
                           pl.gpb, pl.nblk, pl.wfloats);
    }
    return;
  }
  if (bwd)
    hipLaunchKernelGGL((attn_bwd_kernel<CP, DM>), dim3((unsigned)pl.grid), dim3(256), pl.bytes, s, *p, pl.gpb,
                       pl.nblk);
  else
    hipLaunchKernelGGL((attn_fwd_kernel<CP, DM>), dim3((unsigned)pl.grid), dim3(256), pl.bytes, s, *p, pl.gpb,
                       pl.nblk);
}

template <int DM>
void launch_cp(const dgppo_gnn_attn_args* p, const Plan& pl, bool bwd, hipStream_t s) {
  switch (pl.cp) {
    case 8: launch_t<8, DM>(p, pl, bwd, s); break;
    case 16: launch_t<16, DM>(p, pl, bwd, s); break;
    case 32: launch_t<32, DM>(p, pl, bwd, s); break;
    case 64: launch_t<64, DM>(p, pl, bwd, s); break;
    default: launch_t<128, DM>(p, pl, bwd, s); break;
  }
}

// ================================================================================================
// Forward, graph form, for candidate rows wider than the row-block kernels' 32 (dense graphs, e.g.
// LidarSpread n = 32: 32 agent + 32 goal + 8 hit candidates per agent).  One workgroup per graph:
// every sender row of the graph is staged ONCE in LDS (agent mode: the never-receivers' relu(x_raw W4
// + b4) computed once per node instead of once per (receiver, candidate) pair), then each wave takes a
// receiver row at a time with two candidates per lane (C <= 128): logits from LDS, softmax by wave
// shuffles (no barriers), the row's weights / senders / edge features in a per-wave LDS buffer, and the
// H (D + 5) weighted sums one output column per lane.
// ================================================================================================
namespace gfwd {
constexpr int kMaxC = 128;
constexpr int kMaxSlots = 16;
// sender-row pitch: DM + 1 for the 8-wide first layers (scalar reads); 36 for DM = 32 (float4 row reads,
// 16-byte aligned, bank-conflict free across 16 lanes)
template <int DM>
constexpr int row_pitch() { return DM == 32 ? 36 : DM + 1; }
// ns: rows staged in LDS; cp: per-wave candidate pitch; slots: per-wave rows computed on the fly (0: every row
// staged, the round-3 layout).  On-the-fly mode (agent mode with the pre transform, D = 32, Lidar layout
// [agents | goals | each receiver's own hits | pad]): only the agent and goal rows (shared by all receivers) are
// staged; a receiver's own hit rows -- used by that receiver alone -- are computed by the lane that attends over
// them (relu(x_raw W4 + b4), the staging's order of operations) into the wave's slots.  LidarSpread n = 32: 75 KB
// -> 37 KB of LDS per graph, 2 -> 4 resident graphs per CU.
struct Plan {
  int ns, cp, slots;
};
template <int DM>
size_t wave_floats(const Plan& pl) {
  return (size_t)pl.cp * (kH + 1 + 4) + (size_t)pl.slots * row_pitch<DM>();
}
template <int DM>
size_t lds_floats(int n, const Plan& pl) {
  const size_t w = 4 * wave_floats<DM>(pl);
  const size_t pw = (size_t)kD0 * DM + DM;                           // pre weights | bias
  const size_t st = (((size_t)pl.ns * kD0 + 3) & ~(size_t)3) + (pl.slots > 0 ? 0 : pw);  // staging temporaries
  return (size_t)pl.ns * row_pitch<DM>() + (size_t)n * (kH * DM + 4) + (pl.slots > 0 ? pw : 0) + (w > st ? w : st);
}
}  // namespace gfwd

// relu(x_raw pre_W + pre_b) for feature quad [c, c + 4): bias first, then k ascending -- the one order of operations
// of the staged and the on-the-fly never-receiver rows (the backward recomputes them the same way)
__device__ __forceinline__ lanes::f32x4 pre_quad(const float* raw, const float* PW, int D0, int D, int c) {
  lanes::f32x4 v = *reinterpret_cast<const lanes::f32x4*>(PW + D0 * D + c);
  for (int k = 0; k < D0; ++k) v += raw[k] * *reinterpret_cast<const lanes::f32x4*>(PW + k * D + c);
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = v[j] > 0.0f ? v[j] : 0.0f;
  return v;
}

template <int DM>
__global__ __launch_bounds__(256) void attn_fwd_graph_kernel(dgppo_gnn_attn_args p, int ns, int cp, int slots) {
  using lanes::f32x4;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int XP = gfwd::row_pitch<DM>(), QP = kH * DM + 4;
  constexpr bool V4 = DM == 32;  // float4 logits / weighted sums (rows zero-padded to DM)
  const int n = p.n_agents, D = p.D, F = p.F, C = p.C, H = kH;
  const int64_t g = blockIdx.x;
  const bool otf = V4 && slots > 0;       // rows >= ns computed on the fly (gfwd::Plan)
  float* X = lds;                         // [ns][XP] staged sender rows
  float* Q = X + (size_t)ns * XP;         // [n][QP]: qt_h (DM stride) | beta_h at kH DM + h
  float* PWp = Q + (size_t)n * QP;        // on the fly: the persistent pre weights [D0][D] | b [D]
  float* Wb = PWp + (otf ? kD0 * DM + DM : 0);  // per wave: A [cp][kH] | S [cp] | E [cp][4] | slots [slots][XP]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool agent = p.xa != nullptr;
  (void)F;
  // ---- stage the graph's sender rows (pre mode: raw rows and pre weights through LDS first, in the
  // per-wave buffers that are free until the row loop)
  const bool pre = agent && p.pre_W != nullptr;
  const int D0 = p.D0;
  float* R0 = Wb;                                          // [ns][D0] raw rows
  float* PW = otf ? PWp : R0 + (((size_t)ns * D0 + 3) & ~(size_t)3);  // [D0][D] | b [D] (16-byte aligned)
  if (pre) {
    for (int e = threadIdx.x; e < ns * D0; e += 256) R0[e] = p.x[g * p.x_gstride + e];
    for (int e = threadIdx.x; e < D0 * D; e += 256) PW[e] = p.pre_W[e];
    for (int e = threadIdx.x; e < D; e += 256) PW[D0 * D + e] = p.pre_b[e];
    __syncthreads();
  }
  if constexpr (V4) {  // a column quad per thread and step (float4 LDS / global accesses where aligned)
    const bool q4ok = (D & 3) == 0;
    for (int e = threadIdx.x; e < ns * (DM / 4); e += 256) {
      const int r = e / (DM / 4), c = 4 * (e - r * (DM / 4));
      f32x4 v = {0.0f, 0.0f, 0.0f, 0.0f};
      if (c < D) {
        if (agent && r >= n && pre && q4ok) {
          v = pre_quad(R0 + r * D0, PW, D0, D, c);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int d = c + j;
            float x = 0.0f;
            if (d < D) {
              if (!agent) {
                x = p.x[g * p.x_gstride + (int64_t)r * D + d];
              } else if (r < n) {
                x = p.xa[g * p.xa_gstride + (int64_t)r * D + d];
              } else if (pre) {
                float acc = PW[D0 * D + d];
                for (int k = 0; k < D0; ++k) acc += R0[r * D0 + k] * PW[k * D + d];
                x = acc > 0.0f ? acc : 0.0f;
              } else {
                x = p.x[g * p.x_gstride + (int64_t)r * D0 + d];
              }
            }
            v[j] = x;
          }
        }
      }
      *reinterpret_cast<f32x4*>(X + r * XP + c) = v;
    }
  }
  const int DS = V4 ? 0 : D;  // staged columns of the scalar path
  for (int e = threadIdx.x; e < ns * DS; e += 256) {
    const int r = e / DS, d = e - r * DS;
    float v;
    if (d >= D) {
      v = 0.0f;
    } else if (!agent) {
      v = p.x[g * p.x_gstride + (int64_t)r * D + d];
    } else if (r < n) {
      v = p.xa[g * p.xa_gstride + (int64_t)r * D + d];
    } else if (pre) {
      float acc = PW[D0 * D + d];
      for (int k = 0; k < D0; ++k) acc += R0[r * D0 + k] * PW[k * D + d];
      v = acc > 0.0f ? acc : 0.0f;
    } else {  // raw rows used directly (D0 == D)
      v = p.x[g * p.x_gstride + (int64_t)r * D0 + d];
    }
    X[r * XP + d] = v;
  }
  for (int e = threadIdx.x; e < n * H * DM; e += 256) {
    const int i = e / (H * DM), k = e - i * (H * DM), h = k / DM, d = k - h * DM;
    if (V4 || d < D) Q[i * QP + h * DM + d] = d < D ? p.qt[(g * n + i) * qt_ld(p) + h * D + d] : 0.0f;
  }
  for (int e = threadIdx.x; e < n * H; e += 256) {  // beta_h = q_h . bk_h
    const int i = e / H, h = e - i * H;
    Q[i * QP + kH * DM + h] = q_dot_bk(p, g * n + i, h, 0, 1);
  }
  __syncthreads();
  float* A = Wb + (size_t)wave * (cp * (kH + 1 + 4) + slots * XP);
  int* S = reinterpret_cast<int*>(A + cp * kH);
  float* E = A + cp * (kH + 1);
  float* HB = E + cp * 4;  // [slots][XP] this wave's on-the-fly rows (S = ns + slot)
  const int W = H * (D + 5);
  // the next row's senders and edge features are requested while this row computes
  int sn[2];
  f32x4 en[2];
  auto fetch = [&](int i) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int c = lane + 64 * u;
      const bool in = i < n && c < C;
      const int64_t row = g * n + (in ? i : 0);
      const int sd = in ? p.sidx[row * C + c] : -1;
      const int e = in ? p.cand[i * C + c] : 0;
      sn[u] = sd;
      en[u] = sd >= 0 ? *reinterpret_cast<const f32x4*>(p.ef + g * p.ef_gstride + (int64_t)e * 4)
                      : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    }
  };
  fetch(wave);
  for (int i = wave; i < n; i += 4) {
    const int64_t row = g * n + i;
    int sv[2] = {sn[0], sn[1]};
    const f32x4 ev[2] = {en[0], en[1]};
    fetch(i + 4);
    float lg[2][kH];
    // on-the-fly senders of this row get consecutive slots of the wave buffer (clamped: the host enables the mode
    // only when a receiver has at most `slots` of them)
    int slot[2];
    bool overflow = false;  // more on-the-fly senders than slots: the row's outputs become NaN (loud, not silent)
    {
      const bool f0 = otf && sv[0] >= ns, f1 = otf && sv[1] >= ns;
      const uint64_t m0 = __ballot(f0), m1 = __ballot(f1);
      const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
      slot[0] = __popcll(m0 & below);
      slot[1] = __popcll(m0) + __popcll(m1 & below);
      overflow = __popcll(m0) + __popcll(m1) > slots && otf;
#pragma unroll
      for (int u = 0; u < 2; ++u) slot[u] = slot[u] < slots ? slot[u] : (slots > 0 ? slots - 1 : 0);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int c = lane + 64 * u;
      const int sd = sv[u];
      const bool ok = sd >= 0;
      const bool fly = otf && sd >= ns;
      const float* xr = X + (ok && !fly ? sd : 0) * XP;
      if constexpr (V4) {
        f32x4 xv[DM / 4];
        if (fly) {  // this receiver's own never-receiver row: relu(x_raw W4 + b4) here, kept for the weighted sums
          const float* raw = p.x + g * p.x_gstride + (int64_t)sd * D0;
          float* hb = HB + slot[u] * XP;
#pragma unroll
          for (int q = 0; q < DM / 4; ++q) {
            xv[q] = 4 * q < D ? pre_quad(raw, PW, D0, D, 4 * q) : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
            reinterpret_cast<f32x4*>(hb)[q] = xv[q];
          }
        } else {
#pragma unroll
          for (int q = 0; q < DM / 4; ++q) xv[q] = reinterpret_cast<const f32x4*>(xr)[q];
        }
#pragma unroll
        for (int h = 0; h < kH; ++h) {
          const f32x4* qt4 = reinterpret_cast<const f32x4*>(Q + i * QP + h * DM);
          float acc = 0.0f;
#pragma unroll
          for (int q = 0; q < DM / 4; ++q) {
            const f32x4 qq = qt4[q];
            acc += qq[0] * xv[q][0] + qq[1] * xv[q][1] + qq[2] * xv[q][2] + qq[3] * xv[q][3];
          }
          lg[u][h] = ok ? (acc + Q[i * QP + kH * DM + h]) * p.scale : -INFINITY;
        }
      } else {
#pragma unroll
        for (int h = 0; h < kH; ++h) {
          const float* qt = Q + i * QP + h * DM;
          float acc = 0.0f;
#pragma unroll
          for (int d = 0; d < DM; ++d)
            if (d < D) acc += qt[d] * xr[d];
          lg[u][h] = ok ? (acc + Q[i * QP + kH * DM + h]) * p.scale : -INFINITY;
        }
      }
      if (c < C) {
        *reinterpret_cast<f32x4*>(E + c * 4) = ev[u];
        S[c] = fly ? ns + slot[u] : sd;
      }
    }
#pragma unroll
    for (int h = 0; h < kH; ++h) {
      float mx = fmaxf(lg[0][h], lg[1][h]);
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
      const float e0 = sv[0] >= 0 ? expf(lg[0][h] - mx) : 0.0f;
      const float e1 = sv[1] >= 0 ? expf(lg[1][h] - mx) : 0.0f;
      float sm = e0 + e1;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) sm += __shfl_xor(sm, o, 64);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int c = lane + 64 * u;
        const float a = sv[u] >= 0 ? (u == 0 ? e0 : e1) / sm : 0.0f;
        if (c < C) {
          A[c * kH + h] = a;
          if (p.attn) p.attn[(row * H + h) * C + c] = a;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if constexpr (V4) {
      // weighted sums as float4 tasks: lane t = lane & 31 owns column quad (head, q) of xbar, or head h's
      // edge quad, or the three sigmas; the two lane halves take the two halves of the candidates and are
      // combined by one shuffle (masked candidates have weight 0 and read row 0)
      const int TQ = (D + 3) >> 2, t = lane & 31, half = lane >> 5;
      const int kind = t < H * TQ ? 0 : (t < H * TQ + H ? 1 : (t == H * TQ + H ? 2 : 3));
      const int h = kind == 0 ? t / TQ : (kind == 1 ? t - H * TQ : 0), q = kind == 0 ? t - h * TQ : 0;
      const int Ch = (C + 1) >> 1, c0 = half * Ch, c1 = half ? C : Ch;
      f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f}, acc2 = acc;
      // one candidate's term (the S -> X reads of four candidates are issued before their FMAs)
      auto term = [&](int c) -> f32x4 {
        const int sd = S[c];
        const float* ar = A + c * kH;
        if (kind == 2) return f32x4{ar[0], ar[1], ar[2], 0.0f};
        const float a = sd >= 0 ? ar[h] : 0.0f;
        const float* xrow = sd >= ns ? HB + (sd - ns) * XP : X + (sd >= 0 ? sd : 0) * XP;
        const f32x4 v = kind == 0 ? reinterpret_cast<const f32x4*>(xrow)[q] : reinterpret_cast<const f32x4*>(E)[c];
        return a * v;
      };
      if (kind < 3) {
        int c = c0;
        for (; c + 4 <= c1; c += 4) {
          const f32x4 t0 = term(c), t1 = term(c + 1), t2 = term(c + 2), t3 = term(c + 3);
          acc += t0 + t1;
          acc2 += t2 + t3;
        }
        for (; c < c1; ++c) acc += term(c);
        acc += acc2;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] += __shfl_xor(acc[j], 32, 64);
      if (overflow) acc = f32x4{NAN, NAN, NAN, NAN};
      if (half == 0) {
        float* o = p.xcat + row * W;
        if (kind == 0) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (4 * q + j < D) o[h * D + 4 * q + j] = acc[j];
        } else if (kind == 1) {
#pragma unroll
          for (int j = 0; j < 4; ++j) o[H * D + 4 * h + j] = acc[j];
        } else if (kind == 2) {
#pragma unroll
          for (int j = 0; j < kH; ++j) o[H * D + 4 * H + j] = acc[j];
        }
      }
    } else
    // weighted sums, 8 candidates per step with independent partial sums (the per-candidate LDS reads
    // of one step do not wait on each other); masked candidates have weight 0 and read row 0
    for (int o = lane; o < W; o += 64) {
      const int kind = o < H * D ? 0 : (o < H * D + 4 * H ? 1 : 2);
      const int h = kind == 0 ? o / D : (kind == 1 ? (o - H * D) >> 2 : o - H * D - 4 * H);
      const int d = kind == 0 ? o - h * D : (kind == 1 ? (o - H * D) & 3 : 0);
      float part[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
      for (int c0 = 0; c0 < C; c0 += 8) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int c = c0 + u;
          if (c < C) {
            const int sd = S[c];
            const float a = A[c * kH + h];
            const float v = kind == 0 ? X[(sd >= 0 ? sd : 0) * XP + d] : (kind == 1 ? E[c * 4 + d] : 1.0f);
            part[u] += (sd >= 0 ? a : 0.0f) * v;
          }
        }
      }
      p.xcat[row * W + o] = ((part[0] + part[1]) + (part[2] + part[3])) + ((part[4] + part[5]) + (part[6] + part[7]));
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// Backward, graph form, full mode without sender gradients (the first layer: its senders are the raw
// node rows, whose gradient nobody needs): the same staging and row walk as attn_fwd_graph_kernel.
// Per pair da_h = dxbar_h . x + debar_h . ef + dsig_h (+ da_add), dl_h = a_h (da_h - sum_c a_h da_h)
// scale and dbeta_h = sum_c dl_h by wave shuffles; dqt_h = sum_c dl_h x_c one output column per lane.
template <int DM>
__global__ __launch_bounds__(256) void attn_bwd_graph_kernel(dgppo_gnn_attn_args p, int cp) {
  using lanes::f32x4;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int XP = DM + 1;
  const int n = p.n_agents, N = p.N, D = p.D, F = p.F, C = p.C, H = kH;
  const int W = H * (D + 5);
  const int64_t g = blockIdx.x;
  float* X = lds;                          // [N][XP]
  float* G = X + (size_t)N * XP;           // [n][W] dxcat rows
  float* Wb = G + (size_t)n * W;           // per wave: dl [cp][kH] | S [cp] (cp = C rounded to 4)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int e = threadIdx.x; e < N * D; e += 256) {
    const int r = e / D, d = e - r * D;
    X[r * XP + d] = p.x[g * p.x_gstride + (int64_t)r * D + d];
  }
  for (int e = threadIdx.x; e < n * W; e += 256) G[e] = p.dxcat[g * n * W + e];
  __syncthreads();
  float* Aw = Wb + wave * cp * (kH + 1);
  int* S = reinterpret_cast<int*>(Aw + cp * kH);
  for (int i = wave; i < n; i += 4) {
    const int64_t row = g * n + i;
    const float* gv = G + i * W;  // dxbar (H D) | debar (4 H) | dsig (H)
    int sv[2];
    float av[2][kH], da[2][kH];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int c = lane + 64 * u;
      const int sd = c < C ? p.sidx[row * C + c] : -1;
      sv[u] = sd;
      const bool ok = sd >= 0;
      const int e = c < C ? p.cand[i * C + c] : 0;
      const f32x4 ef = ok ? *reinterpret_cast<const f32x4*>(p.ef + g * p.ef_gstride + (int64_t)e * 4)
                          : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
      const float* xr = X + (ok ? sd : 0) * XP;
#pragma unroll
      for (int h = 0; h < kH; ++h) {
        av[u][h] = ok ? p.attn[(row * H + h) * C + c] : 0.0f;
        float acc = 0.0f;
#pragma unroll
        for (int d = 0; d < DM; ++d)
          if (d < D) acc += gv[h * D + d] * xr[d];
#pragma unroll
        for (int j = 0; j < 4; ++j) acc += gv[H * D + 4 * h + j] * ef[j];
        acc += gv[H * D + 4 * H + h];
        if (p.da_add && ok) acc += p.da_add[(row * H + h) * C + c];
        da[u][h] = ok ? acc : 0.0f;
      }
      if (c < C) S[c] = sd;
    }
    float dbeta[kH];
#pragma unroll
    for (int h = 0; h < kH; ++h) {
      float dot = av[0][h] * da[0][h] + av[1][h] * da[1][h];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) dot += __shfl_xor(dot, o, 64);
      float db = 0.0f;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int c = lane + 64 * u;
        const float dl = sv[u] >= 0 ? av[u][h] * (da[u][h] - dot) * p.scale : 0.0f;
        db += dl;
        if (c < C) Aw[c * kH + h] = dl;
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) db += __shfl_xor(db, o, 64);
      dbeta[h] = db;
    }
    if (lane < kH) p.dbeta[row * dbeta_ld(p) + lane] = lane == 0 ? dbeta[0] : (lane == 1 ? dbeta[1] : dbeta[2]);
    for (int kk = lane; kk < H * F; kk += 64) {
      const int h = kk / F;
      if (p.dq) p.dq[row * H * F + kk] = (h == 0 ? dbeta[0] : h == 1 ? dbeta[1] : dbeta[2]) * p.bk[kk];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int o = lane; o < H * D; o += 64) {  // dqt_h[d] = sum_c dl_h x_c[d]
      const int h = o / D, d = o - h * D;
      float part[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
      for (int c0 = 0; c0 < C; c0 += 8) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int c = c0 + u;
          if (c < C) {
            const int sd = S[c];
            part[u] += (sd >= 0 ? Aw[c * kH + h] : 0.0f) * X[(sd >= 0 ? sd : 0) * XP + d];
          }
        }
      }
      p.dqt[row * dqt_ld(p) + o] = ((part[0] + part[1]) + (part[2] + part[3])) + ((part[4] + part[5]) + (part[6] + part[7]));
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// Backward, graph form, agent mode at D = 32 (the dense graphs' second layer, e.g. LidarSpread n = 32: 72
// candidates per agent, 289 never-receiving senders per graph).  A persistent 512-thread workgroup takes one
// graph at a time: the graph's raw rows, agent rows, qt and dxbar rows are staged once in LDS and every
// never-receiver's relu(x_raw pre_W + pre_b) is computed ONCE per node (the forward's order of operations, so
// the ReLU gates agree bit for bit), instead of once per (receiver, candidate) pair.  A wave takes a receiver
// row at a time, candidates c = lane and lane + 64: the pair rows x come from LDS into registers, da / dl /
// dbeta are lane-local math with 64-lane DPP sums, dqt_h = sum_c dl_h x_c is a transposed DPP reduction per
// head, and the sender gradient contrib = sum_h a_h dxbar_h + dl_h qt_h goes (agent senders) into the wave's
// private LDS image of the graph's agent rows -- a receiver's candidates have distinct senders, so the lanes
// never collide -- or (never-receivers) through the ReLU gate into the pre layer's [x_raw | 1]^T dz, MFMA
// 16x16x4 over 16-pair chunks.  The wave images are summed in fixed wave order per graph and the MFMA
// accumulators in fixed wave order per workgroup: bitwise deterministic, no atomics.
namespace gbwd32 {
constexpr int kWaves = 8, kXP = 36, kQP = 96, kGP = 112, kPS = 44;
inline size_t lds_floats(int N, int n) {
  return (size_t)N * kXP + (size_t)N * kD0 + kD0 * 32 + 32 + (size_t)n * (kQP + kGP) +
         (size_t)kWaves * ((size_t)n * 32 + 16 * kPS);
}
}  // namespace gbwd32

__device__ __forceinline__ float sum64(float v) {
  v = lanes::sum16(v);
  return (lanes::rlane(v, 0) + lanes::rlane(v, 16)) + (lanes::rlane(v, 32) + lanes::rlane(v, 48));
}

__global__ __launch_bounds__(512) void attn_bwd_graph32_kernel(dgppo_gnn_attn_args p) {
  using lanes::f32x4;
  using lanes::wave_sync;
  using namespace gbwd32;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int n = p.n_agents, N = p.N, D = p.D, D0 = p.D0, F = p.F, C = p.C, H = kH;
  float* X = lds;                      // [N][36] sender rows (agents: xa; the rest: relu(x_raw W + b))
  float* R0 = X + (size_t)N * kXP;     // [N][8] raw rows, zero padded
  float* PW = R0 + (size_t)N * kD0;    // [8][32] pre_W | [32] pre_b
  float* Pb = PW + kD0 * 32;
  float* QT = Pb + 32;                 // [n][96] qt_h (32-float stride per head)
  float* GS = QT + (size_t)n * kQP;    // [n][112] dxbar_h (32 stride) | debar (96..107) | dsig (108..110)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i16 = lane & 15, kq = lane >> 4;
  float* dxw = GS + (size_t)n * kGP + (size_t)wave * (n * 32 + 16 * kPS);  // this wave's [n][32] agent image
  float* stg = dxw + n * 32;                                                // [16][44] MFMA chunk staging
  const bool want_pre = p.dpre_part != nullptr;
  const bool want_dxa = p.dxa != nullptr;
  {
    const int k = threadIdx.x >> 5, d = threadIdx.x & 31;
    if (threadIdx.x < kD0 * 32) PW[threadIdx.x] = (k < D0 && d < D) ? p.pre_W[k * D + d] : 0.0f;
    if (threadIdx.x < 32) Pb[threadIdx.x] = threadIdx.x < D ? p.pre_b[threadIdx.x] : 0.0f;
  }
  f32x4 gacc[2] = {f32x4{0.0f, 0.0f, 0.0f, 0.0f}, f32x4{0.0f, 0.0f, 0.0f, 0.0f}};  // [x_raw | 1]^T dz
  const int W = H * (D + 5);
  for (int64_t g = blockIdx.x; g < p.G; g += gridDim.x) {
    __syncthreads();  // the previous graph's readers are done
    for (int e = threadIdx.x; e < N * kD0; e += 512) {
      const int r = e >> 3, k = e & 7;
      R0[e] = k < D0 ? p.x[g * p.x_gstride + (int64_t)r * D0 + k] : 0.0f;
    }
    for (int e = threadIdx.x; e < n * 32; e += 512) {
      const int i = e >> 5, d = e & 31;
      X[i * kXP + d] = d < D ? p.xa[g * p.xa_gstride + (int64_t)i * D + d] : 0.0f;
    }
    for (int e = threadIdx.x; e < n * kQP; e += 512) {
      const int i = e / kQP, k = e - i * kQP, h = k >> 5, d = k & 31;
      QT[e] = d < D ? p.qt[(g * n + i) * qt_ld(p) + h * D + d] : 0.0f;
    }
    for (int e = threadIdx.x; e < n * kGP; e += 512) {
      const int i = e / kGP, k = e - i * kGP;
      int src = -1;
      if (k < 96) src = (k & 31) < D ? (k >> 5) * D + (k & 31) : -1;
      else if (k < 108) src = H * D + (k - 96);
      else if (k < 111) src = H * D + 4 * H + (k - 108);
      GS[e] = src >= 0 ? p.dxcat[(g * n + i) * W + src] : 0.0f;
    }
    if (want_dxa)
      for (int e = lane; e < n * 32; e += 64) dxw[e] = 0.0f;
    __syncthreads();
    // never-receivers' rows, in attn_fwd_graph_kernel's order of operations (bias, then k ascending)
    for (int e = threadIdx.x; e < (N - n) * 8; e += 512) {
      const int r = n + (e >> 3), c4 = 4 * (e & 7);
      f32x4 v = *reinterpret_cast<const f32x4*>(Pb + c4);
      for (int k = 0; k < D0; ++k) v += R0[r * kD0 + k] * *reinterpret_cast<const f32x4*>(PW + k * 32 + c4);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = (c4 + j < D && v[j] > 0.0f) ? v[j] : 0.0f;
      *reinterpret_cast<f32x4*>(X + r * kXP + c4) = v;
    }
    __syncthreads();
    for (int i = wave; i < n; i += kWaves) {
      const int64_t row = g * n + i;
      int sv[2];
      f32x4 ev[2];
      float av[2][kH];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int c = lane + 64 * u;
        const bool in = c < C;
        const int s = in ? p.sidx[row * C + c] : -1;
        const int e = in ? p.cand[i * C + c] : 0;
        sv[u] = s;
        ev[u] = s >= 0 ? *reinterpret_cast<const f32x4*>(p.ef + g * p.ef_gstride + (int64_t)e * 4)
                       : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int h = 0; h < kH; ++h) av[u][h] = s >= 0 ? p.attn[(row * H + h) * C + c] : 0.0f;
      }
      float x[2][32];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const f32x4* xr = reinterpret_cast<const f32x4*>(X + (sv[u] >= 0 ? sv[u] : 0) * kXP);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const f32x4 t = xr[q];
          x[u][4 * q] = t[0];
          x[u][4 * q + 1] = t[1];
          x[u][4 * q + 2] = t[2];
          x[u][4 * q + 3] = t[3];
        }
      }
      const float* gv = GS + i * kGP;
      const float* qv = QT + i * kQP;
      // softmax backward: da_h = dxbar_h . x + debar_h . ef + dsig_h (+ da_add)
      float dl[2][kH], dbeta[kH];
#pragma unroll
      for (int h = 0; h < kH; ++h) {
        float da[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          float acc = 0.0f;
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const f32x4 gq = reinterpret_cast<const f32x4*>(gv + 32 * h)[q];
            acc += x[u][4 * q] * gq[0] + x[u][4 * q + 1] * gq[1] + x[u][4 * q + 2] * gq[2] + x[u][4 * q + 3] * gq[3];
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) acc += gv[96 + 4 * h + j] * ev[u][j];
          acc += gv[108 + h];
          const int c = lane + 64 * u;
          if (p.da_add && sv[u] >= 0) acc += p.da_add[(row * H + h) * C + c];
          da[u] = sv[u] >= 0 ? acc : 0.0f;
        }
        const float dot = sum64(av[0][h] * da[0] + av[1][h] * da[1]);
#pragma unroll
        for (int u = 0; u < 2; ++u) dl[u][h] = sv[u] >= 0 ? av[u][h] * (da[u] - dot) * p.scale : 0.0f;
        dbeta[h] = sum64(dl[0][h] + dl[1][h]);
      }
      if (lane < kH) p.dbeta[row * dbeta_ld(p) + lane] = lane == 0 ? dbeta[0] : (lane == 1 ? dbeta[1] : dbeta[2]);
      if (p.dq)
        for (int kk = lane; kk < H * F; kk += 64) {
          const int h = kk / F;
          p.dq[row * H * F + kk] = (h == 0 ? dbeta[0] : h == 1 ? dbeta[1] : dbeta[2]) * p.bk[kk];
        }
      // dqt_h = sum_c dl_h x_c: both slots folded per lane, transposed reduction per half, halves combined
#pragma unroll 1
      for (int h = 0; h < kH; ++h) {  // one head at a time (register budget)
        const float l0 = h == 0 ? dl[0][0] : (h == 1 ? dl[0][1] : dl[0][2]);
        const float l1 = h == 0 ? dl[1][0] : (h == 1 ? dl[1][1] : dl[1][2]);
        float v[32];
#pragma unroll
        for (int d = 0; d < 32; ++d) v[d] = l0 * x[0][d] + l1 * x[1][d];
        int cnt;
        const int base = lanes::treduce32(v, cnt);
        const float tot = v[0] + __shfl_xor(v[0], 32, 64);
        if (lane < 32 && cnt > 0 && base < D) p.dqt[row * dqt_ld(p) + h * D + base] = tot;
      }
      // sender gradients
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (64 * u >= C) break;  // wave-uniform
        const int s = sv[u];
        f32x4 cq[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          cq[q] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
          for (int h = 0; h < kH; ++h)
            cq[q] += av[u][h] * reinterpret_cast<const f32x4*>(gv + 32 * h)[q] +
                     dl[u][h] * reinterpret_cast<const f32x4*>(qv + 32 * h)[q];
        }
        if (want_dxa && s >= 0 && s < n) {
          f32x4* dst = reinterpret_cast<f32x4*>(dxw + s * 32);
#pragma unroll
          for (int q = 0; q < 8; ++q) dst[q] += cq[q];
        }
        if (want_pre) {
          const bool viapre = s >= n;
#pragma unroll 1
          for (int ch = 0; ch < 4; ++ch) {
            if (64 * u + 16 * ch >= C) break;  // wave-uniform
            if (kq == ch) {
              float* sp = stg + i16 * kPS;
#pragma unroll
              for (int q = 0; q < 8; ++q) {  // the ReLU gate from the staged row (x is dead by now)
                const f32x4 xq = reinterpret_cast<const f32x4*>(X + (viapre ? s : 0) * kXP)[q];
                f32x4 dz;
#pragma unroll
                for (int j = 0; j < 4; ++j) dz[j] = (viapre && xq[j] > 0.0f) ? cq[q][j] : 0.0f;
                reinterpret_cast<f32x4*>(sp)[q] = dz;
              }
              const float* rr = R0 + (viapre ? s : 0) * kD0;
              const f32x4 r0 = reinterpret_cast<const f32x4*>(rr)[0], r1 = reinterpret_cast<const f32x4*>(rr)[1];
              const f32x4 z = {0.0f, 0.0f, 0.0f, 0.0f};
              reinterpret_cast<f32x4*>(sp + 32)[0] = viapre ? r0 : z;
              reinterpret_cast<f32x4*>(sp + 32)[1] = viapre ? r1 : z;
              sp[40] = viapre ? 1.0f : 0.0f;
            }
            wave_sync();
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
              const int pp = 4 * ks + kq;
              const float a = i16 <= kD0 ? stg[pp * kPS + 32 + i16] : 0.0f;
#pragma unroll
              for (int ct = 0; ct < 2; ++ct)
                gacc[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, stg[pp * kPS + 16 * ct + i16], gacc[ct], 0, 0, 0);
            }
            wave_sync();
          }
        }
      }
    }
    if (want_dxa) {  // agent j's gradient: the wave images in fixed wave order
      __syncthreads();
      const float* img = GS + (size_t)n * kGP;
      const size_t ws = (size_t)n * 32 + 16 * kPS;
      for (int e = threadIdx.x; e < n * D; e += 512) {
        const int j = e / D, d = e - j * D;
        float acc = 0.0f;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) acc += img[w * ws + j * 32 + d];
        p.dxa[g * p.dxa_gstride + j * D + d] += acc;
      }
    }
  }
  if (want_pre) {  // fixed-order combine of the 8 waves' accumulators -> this workgroup's partial row
    __syncthreads();
    float* red = GS + (size_t)n * kGP;  // [16][33] (the wave areas are free now)
    for (int w = 0; w < kWaves; ++w) {
      if (wave == w) {
#pragma unroll
        for (int ct = 0; ct < 2; ++ct)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float* dst = red + (4 * kq + r) * 33 + 16 * ct + i16;
            *dst = (w == 0 ? 0.0f : *dst) + gacc[ct][r];
          }
      }
      __syncthreads();
    }
    const int PK = D0 * D + D;
    for (int o = threadIdx.x; o < PK; o += 512) {
      const int m = o < D0 * D ? o / D : kD0;
      const int d = o < D0 * D ? o - m * D : o - D0 * D;
      p.dpre_part[(int64_t)blockIdx.x * PK + o] = red[m * 33 + d];
    }
  }
}

bool gbwd32_ok(const dgppo_gnn_attn_args* p) {
  static const bool off = [] {
    const char* e = getenv("DGPPO_ATTN_GRAPH");
    const char* e32 = getenv("DGPPO_ATTN_GBWD32");
    return (e && atoi(e) == 0) || (e32 && atoi(e32) == 0);
  }();
  return !off && p->H == kH && p->C > 32 && p->C <= gfwd::kMaxC && p->D > 8 && p->D <= 32 && p->sidx && p->xa &&
         p->pre_W && p->pre_b && p->D0 <= kD0 && !p->dx && p->N > p->n_agents &&
         gbwd32::lds_floats(p->N, p->n_agents) * sizeof(float) <= 160 * 1024;
}

// one resident 512-thread workgroup per CU (the LDS of one graph fills most of a CU)
int64_t gbwd32_grid(const dgppo_gnn_attn_args* p) {
  static const int64_t knob = [] {
    const char* e = getenv("DGPPO_GBWD32_BLOCKS");
    return e ? (int64_t)atoi(e) : (int64_t)0;
  }();
  const int64_t cap = knob > 0 ? knob : 256;
  return p->G < cap ? p->G : cap;
}

void gbwd32_launch(const dgppo_gnn_attn_args* p, hipStream_t s) {
  const size_t bytes = gbwd32::lds_floats(p->N, p->n_agents) * sizeof(float);
  if (bytes > 64 * 1024) allow_lds((const void*)attn_bwd_graph32_kernel);
  hipLaunchKernelGGL(attn_bwd_graph32_kernel, dim3((unsigned)gbwd32_grid(p)), dim3(512), bytes, s, *p);
}

size_t gbwd_lds_floats(const dgppo_gnn_attn_args* p) {
  return (size_t)p->N * (8 + 1) + (size_t)p->n_agents * kH * (p->D + 5) + 4 * (size_t)((p->C + 3) & ~3) * (kH + 1);
}

bool gbwd_ok(const dgppo_gnn_attn_args* p) {
  static const bool off = [] {
    const char* e = getenv("DGPPO_ATTN_GRAPH");
    return e && atoi(e) == 0;
  }();
  return !off && p->H == kH && p->C > 32 && p->C <= gfwd::kMaxC && p->D <= 8 && p->sidx && !p->xa && !p->dx &&
         gbwd_lds_floats(p) * sizeof(float) <= 160 * 1024;
}

void gbwd_launch(const dgppo_gnn_attn_args* p, hipStream_t s) {
  const size_t bytes = gbwd_lds_floats(p) * sizeof(float);
  if (bytes > 64 * 1024) allow_lds((const void*)attn_bwd_graph_kernel<8>);
  hipLaunchKernelGGL(attn_bwd_graph_kernel<8>, dim3((unsigned)p->G), dim3(256), bytes, s, *p, (p->C + 3) & ~3);
}

// on-the-fly rows in the graph-form forward: -1 = unset (DGPPO_ATTN_GRAPH_OTF, default 1), else 0 / 1
// (dgppo_gnn_set_graph_otf: A/B and the bit-identity test)
int g_graph_otf = -1;

gfwd::Plan gfwd_plan(const dgppo_gnn_attn_args* p) {
  // every row staged; per-wave candidate buffers at the call's C rounded to 4 (was kMaxC = 128: at the n = 32 first
  // layer 31.5 -> 26.6 KB per graph, 5 -> 6 resident graphs per CU)
  gfwd::Plan pl{p->N, (p->C + 3) & ~3, 0};
  if (g_graph_otf < 0) {
    const char* e = getenv("DGPPO_ATTN_GRAPH_OTF");
    g_graph_otf = (e && atoi(e) == 0) ? 0 : 1;
  }
  const int otf = g_graph_otf;
  const int n = p->n_agents, ns = 2 * n, slots = p->C - ns;
  // the Spread layout only: N = 2n + n k + 1 nodes and C = 2n + k candidates (every agent, every goal, the
  // receiver's own k hits), so a receiver has at most C - 2n candidates past the staged rows
  const bool spread_layout = n > 0 && p->N > ns + 1 && (p->N - 1 - ns) % n == 0 && p->C == ns + (p->N - 1 - ns) / n;
  if (otf && spread_layout && p->D > 8 && (p->D & 3) == 0 && p->xa && p->pre_W && p->D0 <= kD0 && slots >= 1 &&
      slots <= gfwd::kMaxSlots)
    pl = gfwd::Plan{ns, (p->C + 3) & ~3, slots};
  return pl;
}

size_t gfwd_bytes(const dgppo_gnn_attn_args* p, const gfwd::Plan& pl) {
  return (p->D <= 8 ? gfwd::lds_floats<8>(p->n_agents, pl) : gfwd::lds_floats<32>(p->n_agents, pl)) * sizeof(float);
}

bool gfwd_ok(const dgppo_gnn_attn_args* p) {
  static const bool off = [] {
    const char* e = getenv("DGPPO_ATTN_GRAPH");
    return e && atoi(e) == 0;
  }();
  // measured (LidarSpread n = 32): 1.6 ms vs 3.1 ms for the block kernel at D <= 8; at D = 32 the float4 form
  // (DGPPO_ATTN_GRAPH32=0 keeps the block kernel there)
  static const bool off32 = [] {
    const char* e = getenv("DGPPO_ATTN_GRAPH32");
    return e && atoi(e) == 0;
  }();
  if (off || p->H != kH || p->C <= 32 || p->C > gfwd::kMaxC || p->D > 32 || !p->sidx) return false;
  if (p->D > 8 && off32) return false;
  if (p->xa && p->D0 > kD0) return false;
  return gfwd_bytes(p, gfwd_plan(p)) <= 160 * 1024;
}

void gfwd_launch(const dgppo_gnn_attn_args* p, hipStream_t s) {
  const bool d8 = p->D <= 8;
  const gfwd::Plan pl = gfwd_plan(p);
  const size_t bytes = gfwd_bytes(p, pl);
  if (bytes > 64 * 1024) allow_lds(d8 ? (const void*)attn_fwd_graph_kernel<8> : (const void*)attn_fwd_graph_kernel<32>);
  if (d8)
    hipLaunchKernelGGL(attn_fwd_graph_kernel<8>, dim3((unsigned)p->G), dim3(256), bytes, s, *p, pl.ns, pl.cp, pl.slots);
  else
    hipLaunchKernelGGL(attn_fwd_graph_kernel<32>, dim3((unsigned)p->G), dim3(256), bytes, s, *p, pl.ns, pl.cp, pl.slots);
}

int run(const dgppo_gnn_attn_args* p, bool bwd, hipStream_t s) {
  if (!bwd && gfwd_ok(p)) {
    if (p->G > 0) gfwd_launch(p, s);
    return 0;
  }
  if (!bwd && fwd2_ok(p)) {
    if (p->G > 0) fwd2_launch(p, s);
    return 0;
  }
  if (bwd && gbwd32_ok(p)) {
    if (p->G > 0) gbwd32_launch(p, s);
    return 0;
  }
  if (bwd && gbwd_ok(p)) {
    if (p->G > 0) gbwd_launch(p, s);
    return 0;
  }
  if (bwd && bwd2_ok(p)) {
    if (p->G > 0) bwd2_launch(p, s);
    return 0;
  }
  const Plan pl = make_plan(p, bwd);
  if (pl.bytes > 160 * 1024) return DGPPO_EINVAL;
  if (pl.dm == 8) launch_cp<8>(p, pl, bwd, s);
  else if (pl.dm == 32) launch_cp<32>(p, pl, bwd, s);
  else launch_cp<64>(p, pl, bwd, s);
  return 0;
}

bool valid(const dgppo_gnn_attn_args* p) {
  if (!p || p->H < 1 || p->H > kH || p->D < 1 || p->D > 64 || p->F < 1 || p->F > 64 || p->C < 1 || p->C > 128 ||
      p->n_agents < 1 || !p->x || !p->ef || !p->qt || !p->bk || !p->cand || !p->receivers || !p->senders)
    return false;
  if (!p->q && !(p->beta && p->beta_ld >= p->H)) return false;  // beta = q . bk from q, or precomputed
  if ((p->qt_ld && p->qt_ld < (int64_t)p->H * p->D) || (p->dqt_ld && p->dqt_ld < (int64_t)p->H * p->D) ||
      (p->dbeta_ld && p->dbeta_ld < p->H))
    return false;
  if (p->xa && (p->D0 < 1 || p->D0 > kD0 || (!p->pre_W && p->D0 != p->D) || (p->pre_W && !p->pre_b)))
    return false;
  return true;
}

}  // namespace
}  // namespace dgppo

extern "C" int dgppo_gnn_sender_table(int32_t G, int32_t n_agents, int32_t C, int32_t E, const int32_t* cand,
                                      const int32_t* receivers, const int32_t* senders, int32_t* sidx,
                                      void* stream) {
  if (G < 0 || n_agents < 1 || C < 1 || E < 1 || !cand || !receivers || !senders || !sidx) return DGPPO_EINVAL;
  const int64_t total = (int64_t)G * n_agents * C;
  if (total == 0) return 0;
  int64_t nb = (total + 255) / 256;
  if (nb > 8192) nb = 8192;
  hipLaunchKernelGGL(dgppo::sender_table_kernel, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream, G, n_agents,
                     C, E, cand, receivers, senders, sidx);
  return (int)hipGetLastError();
}

extern "C" int64_t dgppo_gnn_attn_partial_blocks(const dgppo_gnn_attn_args* p) {
  if (!dgppo::valid(p)) return 0;
  if (dgppo::gbwd32_ok(p)) return dgppo::gbwd32_grid(p);
  if (dgppo::bwd2_ok(p)) {
    int64_t nblk;
    return dgppo::bwd2_grid(p, &nblk);
  }
  return dgppo::make_plan(p, true).grid;
}

extern "C" int dgppo_gnn_set_graph_otf(int32_t on) {
  if (on != 0 && on != 1) return DGPPO_EINVAL;
  dgppo::g_graph_otf = on;
  return 0;
}

extern "C" int dgppo_gnn_attn_fwd(const dgppo_gnn_attn_args* p, void* stream) {
  if (!dgppo::valid(p) || !p->xcat) return DGPPO_EINVAL;
  if (p->G == 0) return 0;
  if (dgppo::run(p, false, (hipStream_t)stream)) return DGPPO_EINVAL;
  return (int)hipGetLastError();
}

extern "C" int dgppo_gnn_attn_bwd(const dgppo_gnn_attn_args* p, void* stream) {
  if (!dgppo::valid(p) || !p->attn || !p->dxcat || !p->dqt || !p->dbeta) return DGPPO_EINVAL;
  if (p->G == 0) return 0;
  if (dgppo::run(p, true, (hipStream_t)stream)) return DGPPO_EINVAL;
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------------------------
// Edge columns past the first 4 (LidarOmniTarget's 10-wide edges).  The attention kernels keep their 4-wide edge
// registers; the EX extra columns enter the value messages through xcat_x = sum_c attn * efx (edge_wsum, one
// thread per output column) and the softmax backward through da_add (edge_da, one thread per (row, head, cand)).
// Both are gather-bound over (G*n) x C x EX floats, a few % of the attention kernels' traffic.  EX <= 16.
namespace dgppo {
namespace {

// one thread per (row, head): the candidate loop reads each edge's EX columns once (float2 pairs when EX is
// even) and keeps the EX sums in registers
template <int EXM>
__global__ __launch_bounds__(256) void edge_wsum_kernel(int64_t R, int32_t n, int32_t C, int32_t H, int32_t EX,
                                                        int32_t E, const float* __restrict__ attn,
                                                        const int32_t* __restrict__ cand,
                                                        const int32_t* __restrict__ sidx,
                                                        const float* __restrict__ efx, float* __restrict__ out) {
  const int64_t total = R * H;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int64_t r = t / H;
    const int h = (int)(t - r * H);
    const int64_t g = r / n;
    const int i = (int)(r - g * n);
    const float* ar = attn + t * C;
    const float* eg = efx + g * E * EX;
    float acc[EXM];
#pragma unroll
    for (int j = 0; j < EXM; ++j) acc[j] = 0.0f;
    for (int c = 0; c < C; ++c) {
      if (sidx[r * C + c] < 0) continue;
      const float a = ar[c];
      const float* er = eg + (int64_t)cand[i * C + c] * EX;
#pragma unroll
      for (int j = 0; j < EXM; ++j)
        if (j < EX) acc[j] += a * er[j];
    }
    float* o = out + r * H * EX + h * EX;
#pragma unroll
    for (int j = 0; j < EXM; ++j)
      if (j < EX) o[j] = acc[j];
  }
}

// one thread per (row, candidate): the edge's EX columns read once, one dot product per head; consecutive
// candidates of a row write consecutive floats of each head's da row
template <int EXM>
__global__ __launch_bounds__(256) void edge_da_kernel(int64_t R, int32_t n, int32_t C, int32_t H, int32_t EX,
                                                      int32_t E, const float* __restrict__ dxx,
                                                      const int32_t* __restrict__ cand,
                                                      const int32_t* __restrict__ sidx,
                                                      const float* __restrict__ efx, float* __restrict__ da) {
  const int64_t total = R * C;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int64_t r = t / C;
    const int c = (int)(t - r * C);
    const int64_t g = r / n;
    const int i = (int)(r - g * n);
    const bool ok = sidx[t] >= 0;
    float ev[EXM];
    const float* er = efx + (g * E + (ok ? cand[i * C + c] : 0)) * EX;
#pragma unroll
    for (int j = 0; j < EXM; ++j) ev[j] = (ok && j < EX) ? er[j] : 0.0f;
    for (int h = 0; h < H; ++h) {
      const float* gr = dxx + (r * H + h) * EX;
      float acc = 0.0f;
#pragma unroll
      for (int j = 0; j < EXM; ++j)
        if (j < EX) acc += gr[j] * ev[j];
      da[(r * H + h) * C + c] = ok ? acc : 0.0f;
    }
  }
}

unsigned grid_for(int64_t total) {
  int64_t nb = (total + 255) / 256;
  return (unsigned)(nb < 8192 ? nb : 8192);
}

}  // namespace
}  // namespace dgppo

extern "C" int dgppo_gnn_edge_wsum(int32_t G, int32_t n_agents, int32_t C, int32_t H, int32_t EX, int32_t E,
                                   const float* attn, const int32_t* cand, const int32_t* sidx, const float* efx,
                                   float* out, void* stream) {
  if (G < 0 || n_agents < 1 || C < 1 || H < 1 || EX < 1 || E < 1 || !attn || !cand || !sidx || !efx || !out)
    return DGPPO_EINVAL;
  const int64_t R = (int64_t)G * n_agents;
  if (R == 0) return 0;
  if (EX > 16) return DGPPO_EINVAL;
  const dim3 grid(dgppo::grid_for(R * H));
  if (EX <= 8)
    hipLaunchKernelGGL(dgppo::edge_wsum_kernel<8>, grid, dim3(256), 0, (hipStream_t)stream, R, n_agents, C, H, EX, E,
                       attn, cand, sidx, efx, out);
  else
    hipLaunchKernelGGL(dgppo::edge_wsum_kernel<16>, grid, dim3(256), 0, (hipStream_t)stream, R, n_agents, C, H, EX,
                       E, attn, cand, sidx, efx, out);
  return (int)hipGetLastError();
}

extern "C" int dgppo_gnn_edge_da(int32_t G, int32_t n_agents, int32_t C, int32_t H, int32_t EX, int32_t E,
                                 const float* dxx, const int32_t* cand, const int32_t* sidx, const float* efx,
                                 float* da_add, void* stream) {
  if (G < 0 || n_agents < 1 || C < 1 || H < 1 || EX < 1 || E < 1 || !dxx || !cand || !sidx || !efx || !da_add)
    return DGPPO_EINVAL;
  const int64_t R = (int64_t)G * n_agents;
  if (R == 0) return 0;
  if (EX > 16) return DGPPO_EINVAL;
  const dim3 grid(dgppo::grid_for(R * C));
  if (EX <= 8)
    hipLaunchKernelGGL(dgppo::edge_da_kernel<8>, grid, dim3(256), 0, (hipStream_t)stream, R, n_agents, C, H, EX, E,
                       dxx, cand, sidx, efx, da_add);
  else
    hipLaunchKernelGGL(dgppo::edge_da_kernel<16>, grid, dim3(256), 0, (hipStream_t)stream, R, n_agents, C, H, EX, E,
                       dxx, cand, sidx, efx, da_add);
  return (int)hipGetLastError();
}
