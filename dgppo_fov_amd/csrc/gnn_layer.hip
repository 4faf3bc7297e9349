// Fused GraphTransformer layer forward: dgppo_gnn_layer_fwd (include/dgppo_hip.h, ABI 11), one kernel for
// what the unfused chain does in four launches (nn/layers.py GraphTransformer.fwd):
//
//   [qt | beta] = [x_i 1] QBW          Dense_0 / Dense_1 in the Q-free form   (dgppo/nn/gnn.py:86-93)
//   attention over each receiving agent's candidate edges -> xcat            (gnn.py:94-107, segment softmax)
//   Y = relu(xcat Wcat / H + x_i Wu + bu)   Dense_2 / Dense_3 messages, Dense_4 update, ReLU   (gnn.py:99-117)
//
// A 256-thread workgroup owns gpb = 16 / n whole graphs (16 receiving agents at n = 8).  The row-block
// attention kernels (attn.hip attn_fwd2r) gather every candidate's sender row from global memory per lane: a
// dependent, uncoalesced 128-byte gather behind the sender-table load.  Here the block's graphs are staged once
// with coalesced loads -- raw node rows, the agent rows of the previous layer -- and the never-receivers' layer
// features relu(x_raw pre_W + pre_b) are computed ONCE per node (the row-block kernels redo them per candidate
// lane, 16 of 24 lanes at n = 8), so the per-candidate reads are LDS reads.  The query-key products and the two
// dense layers around the attention run on v_mfma_f32_16x16x4_f32 over the block's 16 rows (B operands from
// global memory, L2-resident); the attention core itself (logits, softmax, attention-weighted sums by transposed
// DPP reductions) is attn_fwd2r's, one half-wave per receiving agent and one lane per candidate edge.
//
// Outputs: Y always; [qt | beta], attn and xcat only when the caller keeps them for the backward (training
// passes) -- the prepass's forward-only passes write Y alone.  The never-receivers' pre-transform runs in the
// row-block kernels' order of operations (bias, then k ascending, fma), so its ReLU gates are the ones
// attn_bwd2r recomputes, bit for bit.  Everything else agrees with the unfused chain to fp32 rounding
// (different summation orders; tests/test_gnn_layer_gpu.py).
#include <hip/hip_runtime.h>

#include "lds_attr.h"
#include <stdint.h>
#include <stdlib.h>

#include "../../include/dgppo_hip.h"
#include "lanes.h"

namespace dgppo {
namespace {

using lanes::f32x4;

constexpr int kH = 3, kRows = 16, kD0 = 8;

// DM = 8: full mode (raw node rows, D <= 8); DM = 32: agent mode (D = 32, never-receivers via pre_W)
template <int DM>
struct Lay {
  static constexpr int XP = DM + 4;                               // staged node row pitch (12 / 36 floats)
  static constexpr int HS = DM;                                   // per-head stride of a qt row
  static constexpr int QP = 3 * HS + 4;                           // qt row: qt_h at h*HS, beta_h at 3*HS + h
  static constexpr int XCP = ((3 * (DM + 5) + 3) / 4) * 4 + 4;    // xcat tile pitch (44 / 116)
};

struct Carve {
  int rx, qt, pre;  // float offsets: node rows at 0 | raw rows / xcat tile | qt rows | pre_W, pre_b
  size_t floats;
};

template <int DM>
Carve carve(int gpb, int N, bool agent) {
  using L = Lay<DM>;
  Carve c;
  const int xs = gpb * N * L::XP;
  const int raw = agent ? gpb * N * kD0 : 0;
  const int xct = kRows * L::XCP;
  c.rx = (xs + 3) & ~3;
  c.qt = c.rx + ((raw > xct ? raw : xct) + 3) / 4 * 4;
  c.pre = c.qt + kRows * L::QP;
  c.floats = (size_t)c.pre + (agent ? kD0 * 32 + 32 : 0);
  return c;
}

__device__ __forceinline__ f32x4 mma(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <int DM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8))) void gnn_layer_fwd_kernel(
    dgppo_gnn_layer_args p, int gpb, int o_rx, int o_qt, int o_pre) {
  using L = Lay<DM>;
  constexpr int XP = L::XP, HS = L::HS, QP = L::QP, XCP = L::XCP;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const dgppo_gnn_attn_args& a = p.a;
  float* xs = lds;           // [gpb * N][XP] every node's layer input row
  float* rx = lds + o_rx;    // agent mode: raw rows [gpb * N][8]; after staging: the xcat tile [16][XCP]
  float* qts = lds + o_qt;   // [16][QP]
  float* preW = lds + o_pre; // [8][32] | pre_b [32]
  float* preb = preW + kD0 * 32;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i16 = lane & 15, kq = lane >> 4;
  const int n = a.n_agents, N = a.N, D = a.D, F = a.F, C = a.C;
  constexpr bool agent = DM == 32;
  const int64_t g0 = (int64_t)blockIdx.x * gpb;
  const int ng = (int)((int64_t)a.G - g0 < gpb ? (int64_t)a.G - g0 : gpb);
  const int nrec = ng * n;
  const int64_t row0 = g0 * n;
  const int W = kH * D + kH;  // [qt | beta] width

  // ---- stage 1: the block's graphs into LDS (coalesced), qt rows cleared
  if constexpr (agent) {
    const int D0 = a.D0;
    for (int t = tid; t < ng * N * kD0; t += 256) {
      const int node = t >> 3, k = t & 7;
      const int g = node / N, j = node - g * N;
      rx[t] = k < D0 ? a.x[(g0 + g) * a.x_gstride + (int64_t)j * D0 + k] : 0.0f;
    }
    for (int t = tid; t < nrec * (DM / 4); t += 256) {
      const int r = t / (DM / 4), q = t - r * (DM / 4);
      const int g = r / n, i = r - g * n;
      *(f32x4*)(xs + (g * N + i) * XP + 4 * q) = *(const f32x4*)(a.xa + (g0 + g) * a.xa_gstride + (int64_t)i * D + 4 * q);
    }
    {
      const int k = tid >> 5, d = tid & 31;
      preW[tid] = k < D0 ? a.pre_W[k * D + d] : 0.0f;
      if (tid < 32) preb[tid] = a.pre_b[tid];
    }
  } else {
    for (int t = tid; t < ng * N * XP; t += 256) {
      const int node = t / XP, k = t - node * XP;
      const int g = node / N, j = node - g * N;
      xs[t] = k < D ? a.x[(g0 + g) * a.x_gstride + (int64_t)j * D + k] : 0.0f;
    }
  }
  for (int t = tid; t < kRows * QP; t += 256) qts[t] = 0.0f;
  __syncthreads();

  // ---- stage 2 (agent mode): never-receivers' rows relu(x_raw pre_W + pre_b), once per node, in attn_fwd2r /
  // attn_bwd2r's order of operations (bias, then fma over k ascending): the same ReLU gates as their recomputation
  if constexpr (agent) {
    const int nn = N - n;
    for (int t = tid; t < ng * nn * (DM / 4); t += 256) {
      const int q = t & (DM / 4 - 1), rr = t / (DM / 4);
      const int g = rr / nn, j = n + rr - g * nn;
      const float* xr = rx + (g * N + j) * kD0;
      const f32x4 b = *(const f32x4*)(preb + 4 * q);
      float v0 = b[0], v1 = b[1], v2 = b[2], v3 = b[3];
#pragma unroll
      for (int k = 0; k < kD0; ++k) {
        const float xk = xr[k];
        const f32x4 w = *(const f32x4*)(preW + k * 32 + 4 * q);
        v0 += xk * w[0];
        v1 += xk * w[1];
        v2 += xk * w[2];
        v3 += xk * w[3];
      }
      *(f32x4*)(xs + (g * N + j) * XP + 4 * q) =
          f32x4{v0 > 0.0f ? v0 : 0.0f, v1 > 0.0f ? v1 : 0.0f, v2 > 0.0f ? v2 : 0.0f, v3 > 0.0f ? v3 : 0.0f};
    }
  }
  // ---- stage 3: [qt | beta] = [x_i 1] QBW (16 x (D+1) x W) on MFMA; reads only the receivers' rows (stage 1)
  {
    const bool ract = i16 < nrec;
    const int gl = ract ? i16 / n : 0, il = ract ? i16 - gl * n : 0;
    const float* arow = xs + (gl * N + il) * XP;
    const int ntile = (W + 15) >> 4, ksteps = (D + 4) >> 2;
    for (int ct = wave; ct < ntile; ct += 4) {
      const int col = 16 * ct + i16;
      f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
      for (int ks = 0; ks < ksteps; ++ks) {
        const int k = 4 * ks + kq;
        const float av = !ract ? 0.0f : (k < D ? arow[k] : (k == D ? 1.0f : 0.0f));
        const float bv = (k <= D && col < W) ? p.QBW[k * W + col] : 0.0f;
        acc = mma(av, bv, acc);
      }
      if (col < W) {
        const int dst = col < kH * D ? (col / D) * HS + (col % D) : kH * HS + (col - kH * D);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 4 * kq + i;
          if (r < nrec) {
            qts[r * QP + dst] = acc[i];
            if (p.qb) p.qb[(row0 + r) * W + col] = acc[i];
          }
        }
      }
    }
  }
  __syncthreads();

  // ---- stage 4: attention core, one half-wave per receiving agent, one lane per candidate (attn_fwd2r's math)
  float* xc = rx;  // the raw rows are dead: xcat tile [16][XCP]
  {
    const int slot = lane >> 5, c = lane & 31;
    const int TQ = (D + 3) >> 2, WX = kH * (D + 5);
    constexpr int NEV = kH * 5;
#pragma unroll 1
    for (int sr = 0; sr < 2; ++sr) {
      const int rl = 2 * wave + 8 * sr + slot;
      const bool active = rl < nrec;
      const int64_t row = row0 + rl;
      const int gl = active ? rl / n : 0;
      const int i = active ? rl - gl * n : 0;
      int s = -1, e = 0;
      if (active && c < C) {
        e = a.cand[i * C + c];
        s = a.sidx[row * C + c];
      }
      const bool ok = s >= 0;
      f32x4 ef = {0.0f, 0.0f, 0.0f, 0.0f};
      if (ok) ef = *(const f32x4*)(a.ef + (g0 + gl) * a.ef_gstride + (int64_t)e * 4);
      float x[DM];
      {
        const float* xr = xs + (gl * N + (ok ? s : 0)) * XP;
#pragma unroll
        for (int q = 0; q < DM / 4; ++q) {
          const f32x4 v = ok ? *(const f32x4*)(xr + 4 * q) : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
          x[4 * q] = v[0], x[4 * q + 1] = v[1], x[4 * q + 2] = v[2], x[4 * q + 3] = v[3];
        }
      }
      const float* qt = qts + rl * QP;
      float aw[kH];
#pragma unroll
      for (int h = 0; h < kH; ++h) {
        float acc = 0.0f;
#pragma unroll
        for (int q = 0; q < DM / 4; ++q)
          if (q < TQ) {
            const f32x4 qq = ((const f32x4*)(qt + HS * h))[q];
            acc += x[4 * q] * qq[0] + x[4 * q + 1] * qq[1] + x[4 * q + 2] * qq[2] + x[4 * q + 3] * qq[3];
          }
        const float lg = ok ? (acc + qt[kH * HS + h]) * a.scale : -INFINITY;
        const float mx = lanes::max32(lg);
        const float ex = ok ? expf(lg - mx) : 0.0f;
        const float sm = lanes::sum32(ex);
        aw[h] = ok ? ex / sm : 0.0f;
        if (active && c < C && a.attn) a.attn[(row * kH + h) * C + c] = aw[h];
      }
      float* o = a.xcat ? a.xcat + row * WX : nullptr;
      float* ot = xc + rl * XCP;
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
          if (active && j < cnt && q < D) {
            ot[h * D + q] = v[j];
            if (o) o[h * D + q] = v[j];
          }
        }
      }
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
          if (active && j < cnt) {
            const int col = k < 4 ? kH * D + 4 * h + k : kH * D + 4 * kH + h;
            ot[col] = v[j];
            if (o) o[col] = v[j];
          }
        }
      }
    }
  }
  __syncthreads();

  // ---- stage 5: Y = relu(xcat Wcat / H + x_i Wu + bu) on MFMA (16 x 111 x F and 16 x D x F), a wave per 16 columns
  {
    const int WX = kH * (D + 5);
    const bool ract = i16 < nrec;
    const int gl = ract ? i16 / n : 0, il = ract ? i16 - gl * n : 0;
    const float* arow = xs + (gl * N + il) * XP;
    const float* xrow = xc + i16 * XCP;
    const int nct = (F + 15) >> 4;
    for (int ct = wave; ct < nct; ct += 4) {
      const int col = 16 * ct + i16;
      const bool cok = col < F;
      f32x4 am = {0.0f, 0.0f, 0.0f, 0.0f}, au = {0.0f, 0.0f, 0.0f, 0.0f};
      const int km = (WX + 3) >> 2;
      for (int ks = 0; ks < km; ++ks) {
        const int k = 4 * ks + kq;
        const float av = (ract && k < WX) ? xrow[k] : 0.0f;
        const float bv = (cok && k < WX) ? p.Wcat[k * F + col] : 0.0f;
        am = mma(av, bv, am);
      }
      const int ku = (D + 3) >> 2;
      for (int ks = 0; ks < ku; ++ks) {
        const int k = 4 * ks + kq;
        const float av = (ract && k < D) ? arow[k] : 0.0f;
        const float bv = (cok && k < D) ? p.Wu[k * F + col] : 0.0f;
        au = mma(av, bv, au);
      }
      const float bias = cok ? p.bu[col] : 0.0f;
      const float inv_h = 1.0f / (float)kH;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 4 * kq + i;
        if (r < nrec && cok) {
          const float y = (au[i] + bias) + am[i] * inv_h;
          p.Y[(row0 + r) * F + col] = y > 0.0f ? y : 0.0f;
        }
      }
    }
  }
}

bool supported(const dgppo_gnn_layer_args* p) {
  const dgppo_gnn_attn_args& a = p->a;
  if (a.H != kH || a.C < 1 || a.C > 32 || a.n_agents < 1 || a.n_agents > kRows || a.F < 1 || a.F > 64 || !a.sidx ||
      !a.cand || !a.x || !a.ef || !p->QBW || !p->Wcat || !p->Wu || !p->bu || !p->Y || a.G < 0 || a.N < a.n_agents)
    return false;
  if (((uintptr_t)a.ef & 15) || (a.ef_gstride & 3)) return false;
  if (a.xa == nullptr) {
    if (a.D < 1 || a.D > 8 || a.pre_W) return false;
  } else {
    if (a.D != 32 || a.D0 < 1 || a.D0 > kD0 || !a.pre_W || !a.pre_b) return false;
    if (((uintptr_t)a.xa & 15) || (a.xa_gstride & 3)) return false;
  }
  const int gpb = kRows / a.n_agents;
  const Carve c = a.xa ? carve<32>(gpb, a.N, true) : carve<8>(gpb, a.N, false);
  return c.floats * sizeof(float) <= 64 * 1024;
}

}  // namespace
}  // namespace dgppo

extern "C" int dgppo_gnn_layer_supported(const dgppo_gnn_layer_args* p) { return p && dgppo::supported(p) ? 1 : 0; }

extern "C" int dgppo_gnn_layer_fwd(const dgppo_gnn_layer_args* p, void* stream) {
  using namespace dgppo;
  if (!p || !supported(p)) return DGPPO_EINVAL;
  const dgppo_gnn_attn_args& a = p->a;
  if (a.G == 0) return 0;
  const int gpb = kRows / a.n_agents;
  const unsigned grid = (unsigned)((a.G + gpb - 1) / gpb);
  hipStream_t s = (hipStream_t)stream;
  if (a.xa) {
    const Carve c = carve<32>(gpb, a.N, true);
    hipLaunchKernelGGL(gnn_layer_fwd_kernel<32>, dim3(grid), dim3(256), c.floats * sizeof(float), s, *p, gpb, c.rx,
                       c.qt, c.pre);
  } else {
    const Carve c = carve<8>(gpb, a.N, false);
    hipLaunchKernelGGL(gnn_layer_fwd_kernel<8>, dim3(grid), dim3(256), c.floats * sizeof(float), s, *p, gpb, c.rx,
                       c.qt, c.pre);
  }
  return (int)hipGetLastError();
}
