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
  // xcat tile pitch (44 / 132): at DM = 32 a row also hosts its half-wave's 32 (a, sender) pairs (128 floats) for
  // the LDS-loop weighted sums; 132 = 4 mod 64 spreads the 16 rows stage 5's MFMA A reads touch over the banks
  static constexpr int XCP = DM == 32 ? 132 : ((3 * (DM + 5) + 3) / 4) * 4 + 4;
};

constexpr int kYP = 68;  // Y / carry tile pitch (64 + 4)

// dst[t] = ld(t) for t = tid, tid + 256, .. < total, U loads in flight per lane: a plain runtime-bounded copy loop
// waits for each global load before its LDS store (one memory round trip per 256 elements)
template <int U, class Ld>
__device__ __forceinline__ void stage_copy(float* dst, int total, int tid, Ld ld) {
  for (int t0 = tid; t0 < total; t0 += 256 * U) {
    float v[U];
#pragma unroll
    for (int j = 0; j < U; ++j) v[j] = t0 + 256 * j < total ? ld(t0 + 256 * j) : 0.0f;
#pragma unroll
    for (int j = 0; j < U; ++j)
      if (t0 + 256 * j < total) dst[t0 + 256 * j] = v[j];
  }
}

struct Carve {
  // float offsets: node rows at 0 | raw rows / xcat tile | qt rows | pre_W, pre_b | Y tile (zmean, tail) | tail
  // carries [16][kYP] | tail LayerNorm parameters [4][64]
  int rx, qt, pre, yt, hb, lnp;
  int floats;
};

template <int DM>
Carve carve(int gpb, int N, bool agent, bool ytile, bool tail) {
  using L = Lay<DM>;
  Carve c;
  const int xs = gpb * N * L::XP;
  const int raw = agent ? gpb * N * kD0 : 0;
  const int xct = kRows * L::XCP;
  c.rx = (xs + 3) & ~3;
  c.qt = c.rx + ((raw > xct ? raw : xct) + 3) / 4 * 4;
  c.pre = c.qt + kRows * L::QP;
  int o = c.pre + (agent ? kD0 * 32 + 32 : 0);
  // the Y tile reuses the xcat tile when that is wide enough (read by stage 5's MFMAs, then a barrier)
  c.yt = (ytile || tail) ? (L::XCP >= kYP ? c.rx : o) : 0;
  if ((ytile || tail) && L::XCP < kYP) o += kRows * kYP;
  c.hb = tail ? o : 0;
  o += tail ? kRows * kYP : 0;
  c.lnp = tail ? o : 0;
  o += tail ? 4 * 64 : 0;
  c.floats = o;
  return c;
}

__device__ __forceinline__ f32x4 mma(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// LayerNorm(64) (eps 1e-6) + ReLU in place over the 16 rows of a [16][kYP] tile: 8 lanes per row (threads 0..127;
// the others return), flax's mean / E[x^2] - mean^2 form as the GEMM epilogue computes it
__device__ __forceinline__ void ln_relu64(float* Y, const float* scale, const float* bias) {
  if (threadIdx.x >= kRows * 8) return;
  const int r = threadIdx.x >> 3, q = threadIdx.x & 7;
  float v[8];
  float s = 0.0f, s2 = 0.0f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    v[j] = Y[r * kYP + q * 8 + j];
    s += v[j];
    s2 += v[j] * v[j];
  }
#pragma unroll
  for (int o = 4; o > 0; o >>= 1) {
    s += __shfl_xor(s, o, 64);
    s2 += __shfl_xor(s2, o, 64);
  }
  const float mean = s / 64.0f;
  float var = s2 / 64.0f - mean * mean;
  var = var > 0.0f ? var : 0.0f;
  const float rstd = 1.0f / sqrtf(var + 1e-6f);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int col = q * 8 + j;
    const float o = ((v[j] - mean) * rstd) * scale[col] + bias[col];
    Y[r * kYP + col] = o > 0.0f ? o : 0.0f;
  }
}

// acc (16 rows x the wave's 16 columns 16 ct + (lane & 15)) = A (LDS tile [16][lda], K = 64) @ W (64 x ldw, global,
// columns 16 ct ..); every B operand loaded before the first MFMA
__device__ __forceinline__ f32x4 dense64(const float* A, int lda, const float* W, int ldw, int ct, int N) {
  const int lane = threadIdx.x & 63, i16 = lane & 15, kq = lane >> 4;
  const int col = 16 * ct + i16;
  float b[16];
#pragma unroll
  for (int ks = 0; ks < 16; ++ks) b[ks] = col < N ? W[(4 * ks + kq) * ldw + col] : 0.0f;
  f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int ks = 0; ks < 16; ++ks) acc = mma(A[i16 * lda + 4 * ks + kq], b[ks], acc);
  return acc;
}

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

#ifndef DGPPO_DIAG_FWD
#define DGPPO_DIAG_FWD 0  // diagnostic builds only (time attribution, results invalid): 1 no staging loads, 2 no xbar
#endif                    // reductions, 4 no [qt | beta] / message GEMMs, 8 no attn / xcat / qb stores
template <int DM, bool TAIL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(TAIL ? 3 : 4, 8))) void gnn_layer_fwd_kernel(
    dgppo_gnn_layer_args p, int gpb, Carve cv) {
  const int o_rx = cv.rx, o_qt = cv.qt, o_pre = cv.pre;
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
    // (one load per iteration: batching these loads -- eight in flight, or a float4 copy -- measured no faster
    // here, and the extra paths cost the kernel's later phases ~10%, 220 -> 242 us; DGPPO_LAYER_STAGE A/B)
    for (int t = tid; t < ng * N * kD0; t += 256) {
      const int node = t >> 3, k = t & 7;
      const int g = node / N, j = node - g * N;
      rx[t] = (k < D0 && !(DGPPO_DIAG_FWD & 1)) ? a.x[(g0 + g) * a.x_gstride + (int64_t)j * D0 + k] : 0.0f;
    }
    for (int t = tid; t < nrec * (DM / 4); t += 256) {
      const int r = t / (DM / 4), q = t - r * (DM / 4);
      const int g = r / n, i = r - g * n;
      *(f32x4*)(xs + (g * N + i) * XP + 4 * q) = (DGPPO_DIAG_FWD & 1) ? f32x4{0.0f, 0.0f, 0.0f, 0.0f} : *(const f32x4*)(a.xa + (g0 + g) * a.xa_gstride + (int64_t)i * D + 4 * q);
    }
    {
      const int k = tid >> 5, d = tid & 31;
      preW[tid] = k < D0 ? a.pre_W[k * D + d] : 0.0f;
      if (tid < 32) preb[tid] = a.pre_b[tid];
    }
  } else {
    const float* xb = a.x + g0 * a.x_gstride;
    if (a.x_gstride == (int64_t)N * D) {
      stage_copy<8>(xs, ng * N * XP, tid, [&](int t) {
        const int node = t / XP, k = t - node * XP;
        return (k < D && !(DGPPO_DIAG_FWD & 1)) ? xb[node * D + k] : 0.0f;
      });
    } else {
      const int xg = (int)a.x_gstride;
      stage_copy<8>(xs, ng * N * XP, tid, [&](int t) {
        const int node = t / XP, k = t - node * XP;
        const int g = node / N, j = node - g * N;
        return (k < D && !(DGPPO_DIAG_FWD & 1)) ? xb[g * xg + j * D + k] : 0.0f;
      });
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
  // ---- stage 3: [qt | beta] = [x_i 1] QBW (16 x (D+1) x W) on MFMA; reads only the receivers' rows (stage 1).
  // Every B operand of the wave's (at most two) column tiles is loaded before the first MFMA: one L2 round trip
  // instead of one per k-step.
  {
    constexpr int KS = (DM + 4) / 4;  // k-steps over D + 1 <= DM + 1 rows
    const bool ract = i16 < nrec;
    const int gl = ract ? i16 / n : 0, il = ract ? i16 - gl * n : 0;
    const float* arow = xs + (gl * N + il) * XP;
    const int ntile = (W + 15) >> 4;
    float bq[2][KS];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int col = 16 * (wave + 4 * t) + i16;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int k = 4 * ks + kq;
        bq[t][ks] = (k <= D && col < W) ? p.QBW[k * W + col] : 0.0f;
      }
    }
    float aq[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int k = 4 * ks + kq;
      aq[ks] = !ract ? 0.0f : (k < D ? arow[k] : (k == D ? 1.0f : 0.0f));
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int ct = wave + 4 * t;
      if (ct < ntile) {
        const int col = 16 * ct + i16;
        f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int ks = 0; ks < ((DGPPO_DIAG_FWD & 4) ? 0 : KS); ++ks) acc = mma(aq[ks], bq[t][ks], acc);
        if (col < W) {
          const int dst = col < kH * D ? (col / D) * HS + (col % D) : kH * HS + (col - kH * D);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int r = 4 * kq + i;
            if (r < nrec) {
              qts[r * QP + dst] = acc[i];
              if (p.qb && !(DGPPO_DIAG_FWD & 8)) p.qb[(row0 + r) * W + col] = acc[i];
            }
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
        if (active && c < C && a.attn && !(DGPPO_DIAG_FWD & 8)) a.attn[(row * kH + h) * C + c] = aw[h];
      }
      float* o = (a.xcat && !(DGPPO_DIAG_FWD & 8)) ? a.xcat + row * WX : nullptr;
      float* ot = xc + rl * XCP;
      {  // xbar_h = sum_c a_hc x_c by transposed DPP reductions (an LDS loop over the candidates measured slower)
#pragma unroll
        for (int h = 0; h < ((DGPPO_DIAG_FWD & 2) ? 0 : kH); ++h) {
          float v[DM];
#pragma unroll
          for (int dd = 0; dd < DM; ++dd) v[dd] = aw[h] * x[dd];
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

  // ---- stage 5: Y = relu(xcat Wcat / H + x_i Wu + bu) on MFMA (16 x 3(D+5) x F and 16 x D x F), a wave per 16
  // columns; the wave's B operands are all loaded before its first MFMA (one L2 round trip).  Y goes to global
  // memory and / or the Y tile (forward-only epilogues)
  const bool ytile = TAIL || p.zmean != nullptr;
  float* yt = lds + cv.yt;
  {
    constexpr int KM = (3 * (DM + 5) + 3) / 4, KU = DM / 4;
    const int WX = kH * (D + 5);
    const int ct = wave;
    const int col = 16 * ct + i16;
    const bool cok = col < F;
    f32x4 yv = {0.0f, 0.0f, 0.0f, 0.0f};
    if (16 * ct < F) {
      float bm[KM], bu4[KU];
#pragma unroll
      for (int ks = 0; ks < KM; ++ks) {
        const int k = 4 * ks + kq;
        bm[ks] = (cok && k < WX) ? p.Wcat[k * F + col] : 0.0f;
      }
#pragma unroll
      for (int ks = 0; ks < KU; ++ks) {
        const int k = 4 * ks + kq;
        bu4[ks] = (cok && k < D) ? p.Wu[k * F + col] : 0.0f;
      }
      const float bias = cok ? p.bu[col] : 0.0f;
      const bool ract = i16 < nrec;
      const int gl = ract ? i16 / n : 0, il = ract ? i16 - gl * n : 0;
      const float* arow = xs + (gl * N + il) * XP;
      const float* xrow = xc + i16 * XCP;
      f32x4 am = {0.0f, 0.0f, 0.0f, 0.0f}, au = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int ks = 0; ks < ((DGPPO_DIAG_FWD & 4) ? 0 : KM); ++ks) {
        const int k = 4 * ks + kq;
        am = mma((ract && k < WX) ? xrow[k] : 0.0f, bm[ks], am);
      }
#pragma unroll
      for (int ks = 0; ks < ((DGPPO_DIAG_FWD & 4) ? 0 : KU); ++ks) {
        const int k = 4 * ks + kq;
        au = mma((ract && k < D) ? arow[k] : 0.0f, bu4[ks], au);
      }
      const float inv_h = 1.0f / (float)kH;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 4 * kq + i;
        const float y = (au[i] + bias) + am[i] * inv_h;
        yv[i] = y > 0.0f ? y : 0.0f;
        if (p.Y && r < nrec && cok) p.Y[(row0 + r) * F + col] = yv[i];
      }
    }
    if (ytile) {
      __syncthreads();  // the Y tile may alias the xcat tile the MFMAs above read
      if (16 * ct < F && cok)
#pragma unroll
        for (int i = 0; i < 4; ++i) yt[(4 * kq + i) * kYP + col] = yv[i];
      __syncthreads();
    }
  }
  // ---- zmean: per-graph mean of the agent rows (agents in order, then / n)
  if (p.zmean) {
    for (int t = tid; t < ng * F; t += 256) {
      const int g = t / F, f = t - g * F;
      float sacc = 0.0f;
      for (int i = 0; i < n; ++i) sacc += yt[(g * n + i) * kYP + f];
      p.zmean[(g0 + g) * F + f] = sacc / n;
    }
  }
  // ---- value-net tail (forward only): MLP head -> GRUCell(h_in) -> Dense(n_out)
  if constexpr (TAIL) {
    const dgppo_gnn_value_tail& tl = p.tail;
    float* hb = lds + cv.hb;
    float* lnp = lds + cv.lnp;
    for (int t = tid; t < kRows * 64; t += 256) {
      const int r = t >> 6, f = t & 63;
      hb[r * kYP + f] = r < nrec ? tl.h_in[(row0 + r) * 64 + f] : 0.0f;
    }
    {
      const int q = tid >> 6;
      const float* src = q == 0 ? tl.ln0_s : q == 1 ? tl.ln0_b : q == 2 ? tl.ln1_s : tl.ln1_b;
      lnp[tid] = src[tid & 63];
    }
    __syncthreads();
    const int col = 16 * wave + i16;
    // head: two Dense(64) + LayerNorm + ReLU, in place in the Y tile
#pragma unroll 1
    for (int l = 0; l < 2; ++l) {
      const f32x4 acc = dense64(yt, kYP, l == 0 ? tl.W0 : tl.W1, 64, wave, 64);
      const float b = (l == 0 ? tl.b0 : tl.b1)[col];
      __syncthreads();
#pragma unroll
      for (int i = 0; i < 4; ++i) yt[(4 * kq + i) * kYP + col] = acc[i] + b;
      __syncthreads();
      ln_relu64(yt, lnp + 128 * l, lnp + 128 * l + 64);
      __syncthreads();
    }
    // GRU: wave w's column tiles w, w+4, w+8 = the r, z, n gates of hidden columns 16w .. 16w+15
    f32x4 gi[3], gh[3];
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      gi[t] = dense64(yt, kYP, tl.Wi, 192, wave + 4 * t, 192);
      gh[t] = dense64(hb, kYP, tl.Wh, 192, wave + 4 * t, 192);
    }
    const float bir = tl.bi[col], biz = tl.bi[64 + col], bin = tl.bi[128 + col], bhn = tl.bhn[col];
    float hn[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = 4 * kq + i;
      const float rg = sigm(gi[0][i] + bir + gh[0][i]);
      const float zg = sigm(gi[1][i] + biz + gh[1][i]);
      const float ng2 = tanhf(gi[2][i] + bin + rg * (gh[2][i] + bhn));
      hn[i] = (1.0f - zg) * ng2 + zg * hb[r * kYP + col];
    }
    __syncthreads();  // every wave has read hb
#pragma unroll
    for (int i = 0; i < 4; ++i) hb[(4 * kq + i) * kYP + col] = hn[i];
    __syncthreads();
    // output Dense (64 -> n_out <= 16): wave 0
    if (wave == 0) {
      const f32x4 acc = dense64(hb, kYP, tl.Wo, tl.n_out, 0, tl.n_out);
      const bool ok = i16 < tl.n_out;
      const float b = ok ? tl.bo[i16] : 0.0f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 4 * kq + i;
        if (ok && r < nrec) tl.out[(row0 + r) * tl.n_out + i16] = acc[i] + b;
      }
    }
  }
}

bool supported(const dgppo_gnn_layer_args* p) {
  const dgppo_gnn_attn_args& a = p->a;
  const bool tail = p->tail.on != 0;
  if (a.H != kH || a.C < 1 || a.C > 32 || a.n_agents < 1 || a.n_agents > kRows || a.F < 1 || a.F > 64 || !a.sidx ||
      !a.cand || !a.x || !a.ef || !p->QBW || !p->Wcat || !p->Wu || !p->bu || a.G < 0 || a.N < a.n_agents)
    return false;
  if (!p->Y && !p->zmean && !tail) return false;
  if (tail) {
    const dgppo_gnn_value_tail& t = p->tail;
    if (a.xa || a.F != 64 || p->Y || p->qb || a.attn || a.xcat || p->zmean || t.n_out < 1 || t.n_out > 16 || !t.W0 ||
        !t.b0 || !t.ln0_s || !t.ln0_b || !t.W1 || !t.b1 || !t.ln1_s || !t.ln1_b || !t.Wi || !t.bi || !t.Wh || !t.bhn ||
        !t.Wo || !t.bo || !t.h_in || !t.out)
      return false;
  }
  if (((uintptr_t)a.ef & 15) || (a.ef_gstride & 3)) return false;
  if (a.xa == nullptr) {
    if (a.D < 1 || a.D > 8 || a.pre_W) return false;
  } else {
    if (a.D != 32 || a.D0 < 1 || a.D0 > kD0 || !a.pre_W || !a.pre_b) return false;
    if (((uintptr_t)a.xa & 15) || (a.xa_gstride & 3)) return false;
  }
  const int gpb = kRows / a.n_agents;
  const bool yt = p->zmean != nullptr;
  const Carve c = a.xa ? carve<32>(gpb, a.N, true, yt, false) : carve<8>(gpb, a.N, false, yt, tail);
  return (size_t)c.floats * sizeof(float) <= 64 * 1024;
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
  const bool yt = p->zmean != nullptr, tail = p->tail.on != 0;
  const size_t b32 = (size_t)carve<32>(gpb, a.N, true, yt, false).floats * sizeof(float);
  const size_t b8 = (size_t)carve<8>(gpb, a.N, false, yt, tail).floats * sizeof(float);
#define GL_LAUNCH(DMv, TAILv, bytes)                                                                               \
  hipLaunchKernelGGL((gnn_layer_fwd_kernel<DMv, TAILv>), dim3(grid), dim3(256), bytes, s, *p, gpb,                  \
                     carve<DMv>(gpb, a.N, DMv == 32, yt, TAILv))
  if (a.xa) GL_LAUNCH(32, false, b32);
  else if (tail) GL_LAUNCH(8, true, b8);
  else GL_LAUNCH(8, false, b8);
#undef GL_LAUNCH
  return (int)hipGetLastError();
}
