// GraphTransformer attention core (dgppo/nn/gnn.py:78-117 + jraph segment_softmax / segment_sum)
// in the per-receiving-agent form (see include/dgppo_hip.h, dgppo_gnn_attn_args).
//
// Thread mapping: a receiver (graph g, agent i) owns a group of CP = pow2 >= C lanes, one lane per
// candidate edge; a 256-thread workgroup processes R = 256 / CP receivers per round and `gpb` whole
// graphs (rounds loop over their receivers).  Each lane gathers its sender's feature row ONCE into
// registers (D <= DM floats) plus the edge's 4 features, so the softmax logits, the softmax
// backward and the sender gradients are per-lane register math; the weighted sums over candidates
// (xbar, ebar, dqt) go through an LDS transpose so every output column is one lane's dot product.
// Sender gradients of the backward accumulate in an LDS image of the block's graphs in fixed
// receiver order (bitwise-deterministic, no atomics) and are added to dx once per node.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dgppo_hip.h"

namespace dgppo {
namespace {

constexpr int kH = 3;  // heads (GraphTransformer num_heads of the reference GNN)

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

struct Cand {
  int s, e;
};

__device__ __forceinline__ Cand candidate(const dgppo_gnn_attn_args& p, int64_t g, int i, int c) {
  Cand k{-1, -1};
  if (c < p.C) {
    const int e = p.cand[i * p.C + c];
    k.e = e;
    if (e >= 0 && p.receivers[g * p.E + e] == i) k.s = p.senders[g * p.E + e];
  }
  return k;
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

// LDS carve (floats): qt [R][kH*DM] | beta/dbeta [R][4] | xs [256][DM+1] | a [256][kH] | ef [256][4]
//                     | g (bwd: dxcat) [R][kH*(DM+5)] | scratch[8] | dxs (bwd) [gpb][N][D]
template <int CP, int DM>
struct Carve {
  static constexpr int R = 256 / CP;
  static constexpr int XP = DM + 1;
  float *qt, *beta, *xs, *a, *ef, *g, *scr, *dxs;
  __device__ Carve(float* base) {
    qt = base;
    beta = qt + R * kH * DM;
    xs = beta + R * 4;
    a = xs + 256 * XP;
    ef = a + 256 * kH;
    g = ef + 256 * 4;
    scr = g + R * kH * (DM + 5);
    dxs = scr + 8;
  }
  static constexpr size_t floats_fixed() {
    return (size_t)R * kH * DM + R * 4 + 256 * XP + 256 * kH + 256 * 4 + R * kH * (DM + 5) + 8;
  }
};

template <int CP, int DM>
__global__ __launch_bounds__(256) void attn_fwd_kernel(dgppo_gnn_attn_args p, int gpb) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  using CV = Carve<CP, DM>;
  constexpr int R = CV::R, XP = CV::XP;
  CV L(lds);
  const int n = p.n_agents, D = p.D, F = p.F, C = p.C, H = p.H;
  const int W = H * (D + 5);
  const int t = threadIdx.x, slot = t / CP, c = t % CP;
  const int64_t g0 = (int64_t)blockIdx.x * gpb;
  const int ng = (int)((int64_t)p.G - g0 < gpb ? (int64_t)p.G - g0 : gpb);
  const int nrec = ng * n;
  for (int r0 = 0; r0 < nrec; r0 += R) {
    // stage qt and beta_h = q_h . bk_h of the round's receivers
    for (int e = t; e < R * H * D; e += 256) {
      const int rr = e / (H * D), k = e - rr * (H * D);
      if (r0 + rr < nrec) L.qt[rr * kH * DM + k] = p.qt[(g0 * n + r0 + rr) * H * D + k];
    }
    if (t < R * H) {
      const int rr = t / H, h = t - rr * H;
      float acc = 0.0f;
      if (r0 + rr < nrec) {
        const float* q = p.q + (g0 * n + r0 + rr) * H * F + h * F;
        for (int f = 0; f < F; ++f) acc += q[f] * p.bk[h * F + f];
      }
      L.beta[rr * 4 + h] = acc;
    }
    __syncthreads();
    const int rl = r0 + slot;
    const bool active = rl < nrec;
    const int64_t g = g0 + (active ? rl / n : 0);
    const int i = active ? rl % n : 0;
    const int64_t row = g0 * n + rl;
    const Cand k = active ? candidate(p, g, i, c) : Cand{-1, -1};
    const bool ok = k.s >= 0;
    float x[DM];
    load_row<DM>(p.x + g * p.x_gstride + (int64_t)(ok ? k.s : 0) * D, D, ok, x);
    float ef[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) ef[j] = ok ? p.ef[g * p.ef_gstride + (int64_t)k.e * 4 + j] : 0.0f;
    float lg[kH], mx[kH], a[kH];
#pragma unroll
    for (int h = 0; h < kH; ++h) {
      float acc = 0.0f;
      const float* qt = L.qt + slot * kH * DM + h * D;
#pragma unroll
      for (int d = 0; d < DM; ++d)
        if (d < D) acc += qt[d] * x[d];
      lg[h] = (ok && h < H) ? (acc + L.beta[slot * 4 + h]) * p.scale : -INFINITY;
      mx[h] = group_max<CP>(lg[h], L.scr);
    }
#pragma unroll
    for (int h = 0; h < kH; ++h) {
      const float ex = ok && h < H ? expf(lg[h] - mx[h]) : 0.0f;
      const float sm = group_sum<CP>(ex, L.scr);
      a[h] = ok && h < H ? ex / sm : 0.0f;
      if (active && c < C && h < H && p.attn) p.attn[(row * H + h) * C + c] = a[h];
    }
    // LDS transpose: candidates' rows and weights, then one output column per lane
#pragma unroll
    for (int d = 0; d < DM; ++d) L.xs[t * XP + d] = x[d];
#pragma unroll
    for (int h = 0; h < kH; ++h) L.a[t * kH + h] = a[h];
#pragma unroll
    for (int j = 0; j < 4; ++j) L.ef[t * 4 + j] = ef[j];
    __syncthreads();
    if (active) {
      const int base = slot * CP;
      float* out = p.xcat + row * W;
      for (int o = c; o < W; o += CP) {
        float acc = 0.0f;
        if (o < H * D) {
          const int h = o / D, d = o - h * D;
          for (int cc = 0; cc < C; ++cc) acc += L.a[(base + cc) * kH + h] * L.xs[(base + cc) * XP + d];
        } else if (o < H * D + 4 * H) {
          const int q = o - H * D, h = q >> 2, j = q & 3;
          for (int cc = 0; cc < C; ++cc) acc += L.a[(base + cc) * kH + h] * L.ef[(base + cc) * 4 + j];
        } else {
          const int h = o - H * D - 4 * H;
          for (int cc = 0; cc < C; ++cc) acc += L.a[(base + cc) * kH + h];
        }
        out[o] = acc;
      }
    }
    __syncthreads();
  }
}

template <int CP, int DM>
__global__ __launch_bounds__(256) void attn_bwd_kernel(dgppo_gnn_attn_args p, int gpb) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  using CV = Carve<CP, DM>;
  constexpr int R = CV::R, XP = CV::XP;
  CV L(lds);
  const int n = p.n_agents, D = p.D, F = p.F, C = p.C, H = p.H, N = p.N;
  const int W = H * (D + 5);
  const int t = threadIdx.x, slot = t / CP, c = t % CP;
  const int64_t g0 = (int64_t)blockIdx.x * gpb;
  const int ng = (int)((int64_t)p.G - g0 < gpb ? (int64_t)p.G - g0 : gpb);
  const int nrec = ng * n;
  const bool want_dx = p.dx != nullptr;
  if (want_dx)
    for (int e = t; e < ng * N * D; e += 256) L.dxs[e] = 0.0f;
  for (int r0 = 0; r0 < nrec; r0 += R) {
    for (int e = t; e < R * H * D; e += 256) {
      const int rr = e / (H * D), kk = e - rr * (H * D);
      if (r0 + rr < nrec) L.qt[rr * kH * DM + kk] = p.qt[(g0 * n + r0 + rr) * H * D + kk];
    }
    for (int e = t; e < R * W; e += 256) {
      const int rr = e / W, kk = e - rr * W;
      if (r0 + rr < nrec) L.g[rr * kH * (DM + 5) + kk] = p.dxcat[(g0 * n + r0 + rr) * W + kk];
    }
    __syncthreads();
    const int rl = r0 + slot;
    const bool active = rl < nrec;
    const int gl = active ? rl / n : 0;
    const int64_t g = g0 + gl;
    const int i = active ? rl % n : 0;
    const int64_t row = g0 * n + rl;
    const Cand k = active ? candidate(p, g, i, c) : Cand{-1, -1};
    const bool ok = k.s >= 0;
    float x[DM];
    load_row<DM>(p.x + g * p.x_gstride + (int64_t)(ok ? k.s : 0) * D, D, ok, x);
    float ef[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) ef[j] = ok ? p.ef[g * p.ef_gstride + (int64_t)k.e * 4 + j] : 0.0f;
    const float* gv = L.g + slot * kH * (DM + 5);  // dxbar (H*D) | debar (H*4) | dsig (H)
    float a[kH], dl[kH], dbeta[kH];
#pragma unroll
    for (int h = 0; h < kH; ++h) {
      a[h] = (ok && h < H) ? p.attn[(row * H + h) * C + c] : 0.0f;
      float da = 0.0f;
      if (ok && h < H) {
#pragma unroll
        for (int d = 0; d < DM; ++d)
          if (d < D) da += gv[h * D + d] * x[d];
#pragma unroll
        for (int j = 0; j < 4; ++j) da += gv[H * D + h * 4 + j] * ef[j];
        da += gv[H * D + H * 4 + h];
      }
      const float dot = group_sum<CP>(a[h] * da, L.scr);
      dl[h] = (ok && h < H) ? a[h] * (da - dot) * p.scale : 0.0f;
      dbeta[h] = group_sum<CP>(dl[h], L.scr);
    }
    if (active && c == 0)
      for (int h = 0; h < H; ++h) p.dbeta[row * H + h] = dbeta[h];
    if (active)
      for (int kk = c; kk < H * F; kk += CP) {
        const int h = kk / F;
        p.dq[row * H * F + kk] = (h == 0 ? dbeta[0] : h == 1 ? dbeta[1] : dbeta[2]) * p.bk[kk];
      }
    // dqt_h[d] = sum_c dl_c,h x_s[d]: LDS transpose as in the forward
#pragma unroll
    for (int d = 0; d < DM; ++d) L.xs[t * XP + d] = x[d];
#pragma unroll
    for (int h = 0; h < kH; ++h) L.a[t * kH + h] = dl[h];
    __syncthreads();
    if (active) {
      const int base = slot * CP;
      for (int o = c; o < H * D; o += CP) {
        const int h = o / D, d = o - h * D;
        float acc = 0.0f;
        for (int cc = 0; cc < C; ++cc) acc += L.a[(base + cc) * kH + h] * L.xs[(base + cc) * XP + d];
        p.dqt[row * H * D + o] = acc;
      }
    }
    // sender gradients dx_s[d] += sum_h a_h dxbar_h[d] + dl_h qt_h[d], receivers in fixed order
    if (want_dx) {
      float contrib[DM];
      const float* qt = L.qt + slot * kH * DM;
#pragma unroll
      for (int d = 0; d < DM; ++d) {
        float v = 0.0f;
#pragma unroll
        for (int h = 0; h < kH; ++h)
          if (h < H && d < D) v += a[h] * gv[h * D + d] + dl[h] * qt[h * D + d];
        contrib[d] = v;
      }
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
    __syncthreads();
  }
  if (want_dx) {
    for (int e = t; e < ng * N * D; e += 256) {
      const int gg = e / (N * D), kk = e - gg * (N * D);
      p.dx[(g0 + gg) * p.dx_gstride + kk] += L.dxs[e];
    }
  }
}

int pick_cp(int C) {
  int cp = 8;
  while (cp < C) cp <<= 1;
  return cp;
}

template <int CP, int DM>
int launch(const dgppo_gnn_attn_args* p, bool bwd, hipStream_t s) {
  constexpr int R = 256 / CP;
  size_t fixed = Carve<CP, DM>::floats_fixed();
  int gpb = R >= p->n_agents ? R / p->n_agents : 1;
  size_t per_graph = bwd && p->dx ? (size_t)p->N * p->D : 0;
  while (gpb > 1 && (fixed + gpb * per_graph) * sizeof(float) > 64 * 1024) --gpb;
  const size_t bytes = (fixed + gpb * per_graph) * sizeof(float);
  if (bytes > 160 * 1024) return DGPPO_EINVAL;
  if (bytes > 64 * 1024) {  // once per instantiation: allow up to the CU's 160 KB
    static bool raised[2] = {false, false};
    if (!raised[bwd]) {
      (void)hipFuncSetAttribute(bwd ? (const void*)attn_bwd_kernel<CP, DM> : (const void*)attn_fwd_kernel<CP, DM>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      raised[bwd] = true;
    }
  }
  const int blocks = (int)((p->G + gpb - 1) / gpb);
  if (bwd)
    hipLaunchKernelGGL((attn_bwd_kernel<CP, DM>), dim3(blocks), dim3(256), bytes, s, *p, gpb);
  else
    hipLaunchKernelGGL((attn_fwd_kernel<CP, DM>), dim3(blocks), dim3(256), bytes, s, *p, gpb);
  return 0;
}

template <int DM>
int launch_cp(const dgppo_gnn_attn_args* p, bool bwd, hipStream_t s) {
  switch (pick_cp(p->C)) {
    case 8: return launch<8, DM>(p, bwd, s);
    case 16: return launch<16, DM>(p, bwd, s);
    case 32: return launch<32, DM>(p, bwd, s);
    case 64: return launch<64, DM>(p, bwd, s);
    case 128: return launch<128, DM>(p, bwd, s);
  }
  return DGPPO_EINVAL;
}

int dispatch(const dgppo_gnn_attn_args* p, bool bwd, hipStream_t s) {
  if (p->D <= 8) return launch_cp<8>(p, bwd, s);
  if (p->D <= 32) return launch_cp<32>(p, bwd, s);
  return launch_cp<64>(p, bwd, s);
}

}  // namespace
}  // namespace dgppo

extern "C" int dgppo_gnn_attn_fwd(const dgppo_gnn_attn_args* p, void* stream) {
  if (!p || p->H < 1 || p->H > 3 || p->D < 1 || p->D > 64 || p->F < 1 || p->F > 64 || p->C < 1 || p->C > 128 ||
      p->n_agents < 1 || !p->x || !p->ef || !p->qt || !p->q || !p->bk || !p->xcat || !p->cand)
    return DGPPO_EINVAL;
  if (p->G == 0) return 0;
  if (dgppo::dispatch(p, false, (hipStream_t)stream)) return DGPPO_EINVAL;
  return (int)hipGetLastError();
}

extern "C" int dgppo_gnn_attn_bwd(const dgppo_gnn_attn_args* p, void* stream) {
  if (!p || p->H < 1 || p->H > 3 || p->D < 1 || p->D > 64 || p->F < 1 || p->F > 64 || p->C < 1 || p->C > 128 ||
      p->n_agents < 1 || !p->x || !p->ef || !p->qt || !p->attn || !p->dxcat || !p->dqt || !p->dq || !p->dbeta ||
      !p->cand)
    return DGPPO_EINVAL;
  if (p->G == 0) return 0;
  if (dgppo::dispatch(p, true, (hipStream_t)stream)) return DGPPO_EINVAL;
  return (int)hipGetLastError();
}
