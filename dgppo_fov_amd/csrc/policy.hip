// Fused policy step: one launch per env step of the rollouts (trainer/utils.py rollout / test_rollout
// acting with PPOPolicy.sample_action / get_action, policy.py:191-212) for the whole env batch.
//
//   GNN (GraphTransformer x L, per receiving agent) -> MLP head (Dense+LN+ReLU x 2) -> GRUCell ->
//   ScaleHid -> mean / std Dense -> TanhNormal sample (or mode) + log-prob
//
// A 256-thread workgroup owns kRowsG = 16 agent rows (16 / n whole graphs) and keeps every activation of the
// chain in LDS: the ~20 launches and HBM round trips of the unfused step collapse into one kernel
// whose HBM traffic is the graph rows it gathers, the carries and the outputs.  The kernel is
// latency-bound (a chain of dependent gathers and small GEMMs per workgroup), so the design
// shortens that chain:
//   * the (row, candidate) -> (sender, edge) tables are resolved once per workgroup at staging
//     (two dependent gather levels, every load in flight), and each attention sub-round prefetches
//     the next sub-round's raw sender rows and edge features while it computes;
//   * queries are never materialised: QT_h = A (Wq_h Wkt_h) + bq_h Wkt_h and beta_h = Q_h . bk_h
//     come from one GEMM against the query-key products dgppo_policy_prepare() writes to `work`;
//   * the layer-1 features of never-receiving senders, relu(x_raw Wu0 + bu0), are one MFMA tile
//     product per wave and sub-round; the attention-weighted sums read float4 rows from LDS.
// Dense layers run on v_mfma_f32_16x16x4_f32: A operand = activation rows from LDS, B operand =
// weight columns straight from global memory (L2-resident), each wave owning every 4th 16-column
// tile -- for the GRU's 192 columns that puts the r, z and n gates of one wave's 16 hidden units in
// the same wave, so the gate math is register local.
//
// Same math as the unfused path (nn/layers.py, algo/module/nets.py); summation orders differ, so
// results agree to fp32 rounding (tests/test_rollout_gpu.py checks both against float64).
#include <hip/hip_runtime.h>

#include "lds_attr.h"
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/dgppo_hip.h"
#include "lanes.h"
#include "noise.h"

namespace dgppo {
namespace {

using lanes::f32x4;
using lanes::wave_sync;
__device__ __forceinline__ float gsum32(float v) { return lanes::sum32(v); }
__device__ __forceinline__ float gmax32(float v) { return lanes::max32(v); }
__device__ __forceinline__ float gsum8(float v) { return lanes::sum8(v); }

constexpr int kRowsG = 16, kThreads = 256, kHeads = 3, kHid = 64;
// row tiles of 16, attention sub-rounds (a wave takes two rows per sub-round), pairs per thread
constexpr int kRT = kRowsG / 16, kSR = kRowsG / 8;
// raw node rows up to 12 wide and edge rows up to 4 + 6 (LidarOmniTarget: 10 / 10); the kernel is
// instantiated narrow (<= 8, 4: the Lidar / MPE envs, 240 VGPRs = 2 waves per SIMD) and wide
constexpr int kMaxD0 = 12, kMaxEX = 6, kCP = 32;
constexpr int kNarrowD0 = 8;
// register form: waves per SIMD the compiler must fit (VGPR budget 512 / kRegWaves)
#ifndef POLICY_REG_WAVES
#define POLICY_REG_WAVES 3
#endif
constexpr int kRegWaves = POLICY_REG_WAVES;
#ifndef DGPPO_DIAG_POL
#define DGPPO_DIAG_POL 0  // diagnostic builds only (time attribution, results invalid): 1 no layer-1 pre transform
#endif
// LDS pitches (floats); xs rows: x (0..31) | edge head (32..35) | extra edge columns (36..41)
constexpr int kX0P = 13, kQTP = 100, kXCP = 132, kY0P = 36, kYP = 68, kXSP = 44;
// work: per layer the (32 + 1) x 100 query-key matrix [QT_0 | QT_1 | QT_2 (32 cols each) | beta_0..2 | 0]
// (rows 0..D-1) and its bias row (row 32)
constexpr int kQKRows = 33, kQKCols = kQTP, kQKStride = kQKRows * kQKCols;

// phase timestamps for tuning (`make probe` builds this file with -DPOLICY_PROBE, scripts/policy_probe.py reads them): thread 0
// of each workgroup writes s_memrealtime (100 MHz) at phase k into p.h_out viewed as uint64[grid][32]
#ifdef POLICY_PROBE
#define PROBE(k)                                                                                      \
  do {                                                                                                \
    __syncthreads();                                                                                  \
    if (threadIdx.x == 0) ((uint64_t*)p.h_out)[blockIdx.x * 32 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define PROBE(k) \
  do {           \
  } while (0)
#endif

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }
__device__ __forceinline__ float softplusf(float x) { return x > 20.0f ? x : log1pf(expf(x)); }
__device__ __forceinline__ float log_ndtr(float z) {
  if (z > -10.0f) return logf(0.5f * erfcf(-z * 0.70710678118654752f));
  const float z2 = z * z;
  const float s = 1.0f - 1.0f / z2 + 3.0f / (z2 * z2) - 15.0f / (z2 * z2 * z2);
  return -0.5f * z2 - logf(-z) - 0.91893853320467274f + logf(s);
}
__device__ __forceinline__ float tanh_fldj(float x) { return 2.0f * (0.69314718055994531f - x - softplusf(-2.0f * x)); }

// ---- register-resident weight operands -------------------------------------------------------
// Frag<KS, CT>: the B operand of v_mfma_f32_16x16x4_f32 for KS k-steps of this wave's column tiles
// ct = wave + 4 t (t < CT): v[ks][t] = W[4 ks + (lane >> 4)][16 ct + (lane & 15)].  Every fragment of
// the step is loaded at kernel start, so each GEMM phase runs without a global-memory round trip.
template <int KS, int CT>
struct Frag {
  float v[KS][CT];
};

// raw buffer resource over `bytes` bytes at `base`: loads past the end return 0 (no per-load guards)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const float* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, bytes, 0x00020000);
}
__device__ __forceinline__ float buf_load(__amdgpu_buffer_rsrc_t r, int byte_off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, byte_off, 0, 0));
}

// W is K x ldw row-major; rows >= K read as 0.  Columns past the layer's width may read neighbouring
// data: those accumulator columns are never stored (acc_store checks col < N).
template <int KS, int CT>
__device__ __forceinline__ void frag_load(Frag<KS, CT>& f, const float* W, int ldw, int K) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const auto rs = buf_rsrc(W, K * ldw * 4);
  const int vo = ((lane >> 4) * ldw + wave * 16 + (lane & 15)) * 4;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int t = 0; t < CT; ++t) f.v[ks][t] = buf_load(rs, vo + (4 * ks * ldw + 64 * t) * 4);
}

// per-lane bias of the C columns 16 (wave + 4 t) + (lane & 15)
template <int CT>
__device__ __forceinline__ void bias_load(float (&b)[CT], const float* bias, int N) {
  const auto rs = buf_rsrc(bias, N * 4);
  const int col0 = (threadIdx.x >> 6) * 16 + (threadIdx.x & 15);
#pragma unroll
  for (int t = 0; t < CT; ++t) b[t] = buf_load(rs, (col0 + 64 * t) * 4);
}

// acc[t][rt] += A (32 x K, LDS, pitch lda) @ W: rows rt*16 + 4*(lane>>4) + r, col (wave + 4t)*16 + (lane&15)
template <int KS, int CT>
__device__ __forceinline__ void frag_mma(f32x4 (&acc)[CT][kRT], const float* A, int lda, int K, const Frag<KS, CT>& f) {
  const int lane = threadIdx.x & 63;
  const int i16 = lane & 15, kq = lane >> 4;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int k = 4 * ks + kq;
    float a[kRT];
#pragma unroll
    for (int rt = 0; rt < kRT; ++rt) a[rt] = k < K ? A[(16 * rt + i16) * lda + k] : 0.0f;
#pragma unroll
    for (int t = 0; t < CT; ++t)
#pragma unroll
      for (int rt = 0; rt < kRT; ++rt)
        acc[t][rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[rt], f.v[ks][t], acc[t][rt], 0, 0, 0);
  }
}

template <int CT>
__device__ __forceinline__ void acc_zero(f32x4 (&acc)[CT][kRT]) {
#pragma unroll
  for (int t = 0; t < CT; ++t)
#pragma unroll
    for (int rt = 0; rt < kRT; ++rt) acc[t][rt] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
}

// dst[row][col] = act(scale * acc + bias) for col < N
template <int CT>
__device__ __forceinline__ void acc_store(const f32x4 (&acc)[CT][kRT], float* dst, int ldd, int N, const float (&b)[CT],
                                          float scale, bool relu) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i16 = lane & 15, kq = lane >> 4;
#pragma unroll
  for (int t = 0; t < CT; ++t) {
    const int col = (wave + 4 * t) * 16 + i16;
    if (col >= N) continue;
#pragma unroll
    for (int rt = 0; rt < kRT; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = scale * acc[t][rt][r] + b[t];
        if (relu) v = v > 0.0f ? v : 0.0f;
        dst[(rt * 16 + 4 * kq + r) * ldd + col] = v;
      }
  }
}

// layer-1 features relu(x_raw Wu0 + bu0) of a workgroup's never-receiving nodes, computed once per node (MFMA) into
// LDS when the group has at most kPreMax of them (LidarSpread n = 8: 2 graphs x 73 nodes); rows of 32 floats, each
// row's float4 quads stored XOR-swizzled by (row & 7) so that lanes reading different rows spread over the banks
constexpr int kPreMax = 160;
struct Lds {
  float *x0, *qt, *xc, *y0, *yb, *preW, *preb, *lnp, *outW, *att, *pre;
  int *psrc, *pedge;  // alias att: consumed before the first attention sub-round
  float* hb;          // aliases att: the carries are written there after the GNN
};

// the register form's att region only hosts the pair tables (before the GNN) and the carries (after it)
constexpr int kAttReg = kRowsG * kYP > 2 * kRowsG * kCP ? kRowsG * kYP : 2 * kRowsG * kCP;
constexpr size_t lds_floats() {
  return (size_t)kRowsG * (kX0P + kQTP + kXCP + kY0P + kYP) + kMaxD0 * 32 + 32 + 4 * kHid + 2 * kHid * 4 + 8 +
         kAttReg + kPreMax * 32;
}

__device__ __forceinline__ Lds carve(float* base) {
  Lds L;
  L.x0 = base;
  L.qt = L.x0 + kRowsG * kX0P;
  L.xc = L.qt + kRowsG * kQTP;
  L.y0 = L.xc + kRowsG * kXCP;
  L.yb = L.y0 + kRowsG * kY0P;
  L.preW = L.yb + kRowsG * kYP;
  L.preb = L.preW + kMaxD0 * 32;
  L.lnp = L.preb + 32;           // ln0 scale, ln0 bias, ln1 scale, ln1 bias (64 each)
  L.outW = L.lnp + 4 * kHid;     // [Wm | Wsd] (64 x 2A, A <= 4) then bm, bsd
  L.att = L.outW + 2 * kHid * 4 + 8;
  L.psrc = (int*)L.att;
  L.hb = L.att;
  L.pedge = L.psrc + kRowsG * kCP;
  L.pre = L.att + kAttReg;  // (register form only)
  return L;
}

// raw sender row and edge features of the pair (row r, candidate c); raw rows are fetched for every
// sender (layer 0 uses them all, layer 1 those of never-receiving senders)
template <int MD0, int MEX>
struct PairG {
  float xr[MD0];
  f32x4 ef;
  float ex[MEX > 0 ? MEX : 1];  // edge columns 4.. (wide instantiation only)
  int s;
};

// cur = pg[sr] by selects (a dynamically indexed register array would live in scratch)
template <int MD0, int MEX>
__device__ __forceinline__ void pair_pick(const PairG<MD0, MEX> (&pg)[kSR], int sr, PairG<MD0, MEX>& cur) {
#pragma unroll
  for (int k = 0; k < MD0; ++k) cur.xr[k] = pg[0].xr[k];
#pragma unroll
  for (int j = 0; j < 4; ++j) cur.ef[j] = pg[0].ef[j];
#pragma unroll
  for (int j = 0; j < MEX; ++j) cur.ex[j] = pg[0].ex[j];
  cur.s = pg[0].s;
#pragma unroll
  for (int q = 1; q < kSR; ++q) {
    const bool tk = sr == q;
#pragma unroll
    for (int k = 0; k < MD0; ++k) cur.xr[k] = tk ? pg[q].xr[k] : cur.xr[k];
#pragma unroll
    for (int j = 0; j < 4; ++j) cur.ef[j] = tk ? pg[q].ef[j] : cur.ef[j];
#pragma unroll
    for (int j = 0; j < MEX; ++j) cur.ex[j] = tk ? pg[q].ex[j] : cur.ex[j];
    cur.s = tk ? pg[q].s : cur.s;
  }
}

// r / n for r < 32, n <= 32: (r * nmag) >> 16 with nmag = 65536 / n + 1 (exact in that range)
__device__ __forceinline__ int div_n(int r, int nmag) { return (r * nmag) >> 16; }

template <int MD0, int MEX>
__device__ __forceinline__ void pair_gather(const dgppo_policy_step_args& p, const Lds& L, int r, int c, int64_t g0,
                                            int nmag, PairG<MD0, MEX>& o) {
  const int s = L.psrc[r * kCP + c];
  const int e = L.pedge[r * kCP + c];
  const int64_t g = g0 + div_n(r, nmag);
  const bool ok = s >= 0;
  o.s = s;
  if (MEX == 0) {
    o.ef = ok ? *(const f32x4*)(p.edges + g * p.edges_gstride + (int64_t)e * 4) : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    o.ex[0] = 0.0f;
  } else {  // wider edge rows (8-byte aligned at best): scalar loads
    const float* er = p.edges + g * p.edges_gstride + (int64_t)(ok ? e : 0) * p.ED;
#pragma unroll
    for (int j = 0; j < 4; ++j) o.ef[j] = ok ? er[j] : 0.0f;
#pragma unroll
    for (int j = 0; j < MEX; ++j) o.ex[j] = (ok && 4 + j < p.ED) ? er[4 + j] : 0.0f;
  }
  const float* xr = p.nodes + g * p.nodes_gstride + (int64_t)(ok ? s : 0) * p.D0;
#pragma unroll
  for (int k = 0; k < MD0; ++k) o.xr[k] = (ok && k < p.D0) ? xr[k] : 0.0f;
}

// One GraphTransformer layer for the group's rows (register form; round 6 removed the LDS-staged form): a lane's pair keeps its sender row x in registers
// (layer 0: the raw row; layer 1: relu(x_raw Wu0 + bu0) by VALU FMAs against the LDS-resident Wu0, or
// the agent's layer-0 output row from LDS), the logits are lane-local dots against the row's QT_h, and
// the attention-weighted sums over the row's 32 candidates -- [xbar_h | ebar_h | sig_h | ebar_x_h] --
// are one transposed DPP reduction per head (lanes::treduce32), whose totals each lane writes to the
// row's xcat.  No per-pair LDS staging: the workgroup's LDS is its row activations only, so more
// workgroups are resident per CU, and the weighted sums need no LDS round trips.
template <int DX, bool layer0, int MD0, int MEX, int KQ, int KC, int KX, int KU, bool node_pre = false>
__device__ __forceinline__ void gt_layer_reg(const dgppo_policy_step_args& p, const dgppo_gt_layer& ly,
                                             const PairG<MD0, MEX> (&pg)[kSR], const Lds& L, const float* qk,
                                             const float* A, int lda, float* out, int ldo, int nmag, int pk) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = p.n_agents, D = ly.D, F = ly.F, H = kHeads;
  const int EX = MEX > 0 ? p.ED - 4 : 0;
  // [QT_h | beta_h] = A QK + qk_bias (kRowsG x 100)
  {
    Frag<KQ, 2> fq;
    float bq[2];
    frag_load(fq, qk, kQKCols, D);
    bias_load(bq, qk + 32 * kQKCols, kQKCols);
    f32x4 acc[2][kRT];
    acc_zero(acc);
    frag_mma(acc, A, lda, D, fq);
    acc_store(acc, L.qt, kQTP, kQKCols, bq, 1.0f, false);
  }
  __syncthreads();
  PROBE(pk);
  const int slot = lane >> 5, c = lane & 31;
  const float scale = rsqrtf((float)F);
  // x width DX: layer 0 the raw row (MD0), layer 1 the 32-wide hidden row.  Per head the DX weighted x
  // sums are one transposed reduction; the edge / sig sums of all heads ([ebar_h (4) | sig_h | ebar_x_h
  // (EX)] x 3) a second one, so at most DX + DX values are live
  constexpr int NE = 5 + MEX, NEV = kHeads * NE;
#pragma unroll
  for (int sr = 0; sr < kSR; ++sr) {  // unrolled: pg[sr] read directly, pg[0] dies after the first sub-round
    const PairG<MD0, MEX>& cur = pg[sr];
    const int r = 2 * wave + 8 * sr + slot;
    const bool ok = cur.s >= 0;
    float x[DX];
    if (layer0) {
#pragma unroll
      for (int d = 0; d < DX; ++d) x[d] = d < MD0 ? cur.xr[d] : 0.0f;
    } else if (ok && cur.s < n) {  // agent sender: the layer input row of the same graph
      const f32x4* src = (const f32x4*)(A + (div_n(r, nmag) * n + cur.s) * lda);
#pragma unroll
      for (int q = 0; q < DX / 4; ++q) {
        const f32x4 v = src[q];
        x[4 * q] = v[0];
        x[4 * q + 1] = v[1];
        x[4 * q + 2] = v[2];
        x[4 * q + 3] = v[3];
      }
    } else if constexpr (node_pre) {  // never-receiving sender: its row of the per-node table (masked pairs: node 0)
      const int m = ok ? div_n(r, nmag) * (p.N - n) + (cur.s - n) : 0;
      const float* src = L.pre + m * 32;
#pragma unroll
      for (int q = 0; q < DX / 4; ++q) {
        const f32x4 v = *(const f32x4*)(src + 4 * (q ^ (m & 7)));
        x[4 * q] = v[0];
        x[4 * q + 1] = v[1];
        x[4 * q + 2] = v[2];
        x[4 * q + 3] = v[3];
      }
    } else {  // never-receiving sender: relu(x_raw Wu0 + bu0) (masked pairs too; their weights are 0)
#pragma unroll
      for (int q = 0; q < DX / 4; ++q) {
        const f32x4 b = *(const f32x4*)(L.preb + 4 * q);
        x[4 * q] = b[0];
        x[4 * q + 1] = b[1];
        x[4 * q + 2] = b[2];
        x[4 * q + 3] = b[3];
      }
#pragma unroll
      for (int k = 0; k < (DGPPO_DIAG_POL ? 0 : MD0); ++k) {
        const float xk = cur.xr[k];
#pragma unroll
        for (int q = 0; q < DX / 4; ++q) {
          const f32x4 w = *(const f32x4*)(L.preW + k * 32 + 4 * q);
          x[4 * q] += xk * w[0];
          x[4 * q + 1] += xk * w[1];
          x[4 * q + 2] += xk * w[2];
          x[4 * q + 3] += xk * w[3];
        }
      }
#pragma unroll
      for (int d = 0; d < DX; ++d) x[d] = x[d] > 0.0f ? x[d] : 0.0f;
    }
    // logits (QT_h . x + beta_h) / sqrt(F) and the softmax over the row's 32 candidates
    const float* qt = L.qt + r * kQTP;
    float* o = L.xc + r * kXCP;
    float aw[kHeads];
#pragma unroll
    for (int h = 0; h < kHeads; ++h) {
      float acc = 0.0f;
#pragma unroll
      for (int q = 0; q < DX / 4; ++q) {
        const f32x4 qv = *(const f32x4*)(qt + 32 * h + 4 * q);
        acc += x[4 * q] * qv[0] + x[4 * q + 1] * qv[1] + x[4 * q + 2] * qv[2] + x[4 * q + 3] * qv[3];
      }
      const float lg = ok ? (acc + qt[96 + h]) * scale : -INFINITY;
      const float mx = gmax32(lg);
      const float ex = ok ? expf(lg - mx) : 0.0f;
      const float sm = gsum32(ex);
      aw[h] = ok ? ex / sm : 0.0f;
    }
    // xbar_h = sum_c a_h x_c
#pragma unroll
    for (int h = 0; h < kHeads; ++h) {
      float v[DX];
#pragma unroll
      for (int d = 0; d < DX; ++d) v[d] = aw[h] * x[d];
      int cnt;
      const int base = lanes::treduce32(v, cnt);
#pragma unroll
      for (int j = 0; j < lanes::tr_final<DX>(); ++j) {
        const int q = base + j;
        if (j < cnt && q < D) o[h * D + q] = v[j];
      }
    }
    // [ebar_h | sig_h | ebar_x_h] of the three heads
    {
      float v[NEV];
#pragma unroll
      for (int h = 0; h < kHeads; ++h) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[h * NE + j] = aw[h] * cur.ef[j];
        v[h * NE + 4] = aw[h];
#pragma unroll
        for (int j = 0; j < MEX; ++j) v[h * NE + 5 + j] = aw[h] * cur.ex[j];
      }
      int cnt;
      const int base = lanes::treduce32(v, cnt);
#pragma unroll
      for (int j = 0; j < lanes::tr_final<NEV>(); ++j) {
        const int q = base + j;
        const int h = q / NE, k = q - h * NE;
        int col = -1;
        if (j < cnt) {
          if (k < 4) col = H * D + 4 * h + k;
          else if (k == 4) col = H * D + 4 * H + h;
          else if (k - 5 < EX) col = H * (D + 5) + h * EX + (k - 5);
        }
        if (col >= 0) o[col] = v[j];
      }
    }
  }
  // message + update operands (after the barrier: loads hoisted into the attention would raise its
  // register pressure), then out = relu(xcat Wcat / H + A Wu + bu)
  __syncthreads();
  PROBE(pk + 1);
  Frag<KC, 1> fc;
  Frag<KX, 1> fx;
  Frag<KU, 1> fu;
  float bu[1];
  frag_load(fc, ly.Wcat, ly.F, kHeads * (ly.D + 5));
  frag_load(fx, ly.Wex, ly.F, EX > 0 ? kHeads * EX : 0);
  frag_load(fu, ly.Wu, ly.F, ly.D);
  bias_load(bu, ly.bu, ly.F);
  {
    f32x4 acc[1][kRT];
    acc_zero(acc);
    frag_mma(acc, L.xc, kXCP, H * (D + 5), fc);
    if (EX > 0) frag_mma(acc, L.xc + H * (D + 5), kXCP, H * EX, fx);
#pragma unroll
    for (int rt = 0; rt < kRT; ++rt) acc[0][rt] *= 1.0f / H;
    frag_mma(acc, A, lda, D, fu);
    acc_store(acc, out, ldo, F, bu, 1.0f, true);
  }
  __syncthreads();
}

// in-place LayerNorm (eps 1e-6) + ReLU over 64 columns of the kRowsG rows: 8 lanes per row
__device__ __forceinline__ void ln_relu64(float* Y, const float* scale, const float* bias) {
  if (threadIdx.x >= kRowsG * 8) return;  // whole waves
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
    const float o = (v[j] - mean) * rstd * scale[col] + bias[col];
    Y[r * kYP + col] = o > 0.0f ? o : 0.0f;
  }
}

// NP: the per-node layer-1 pre-transform table (narrow register form, two layers, <= kPreMax never-receiving nodes
// per group: the host picks this instantiation, node_pre_ok); its own instantiation, so that the raw sender rows die
// after layer 0 instead of staying live through layer 1 for the per-lane fallback
template <int MD0, int MEX, bool NP = false>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(MD0 <= kNarrowD0 ? kRegWaves : 1, 8))) void policy_step_kernel(dgppo_policy_step_args p) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const Lds L = carve(lds);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i16 = lane & 15, kq = lane >> 4;
  const int n = p.n_agents, A = p.A;
  const int nmag = 65536 / n + 1;
  const int gpg = kRowsG / n;  // graphs per row group
  const int64_t ngroups = (p.G + gpg - 1) / gpg;
  const bool two = p.n_layers == 2;
  // one row group per workgroup (a persistent loop would let LICM hoist every weight load into
  // registers across groups and spill)
  const int64_t grp = blockIdx.x;
  if (grp >= ngroups) return;
  const int64_t g0 = grp * gpg;
  const int ng = (int)((int64_t)p.G - g0 < gpg ? (int64_t)p.G - g0 : gpg);
  const int rows = ng * n;
  const int64_t row0 = g0 * n;
  PROBE(0);
  // ---- level 1 loads: candidate edges, agent rows, carries, small parameters, weight fragments
  constexpr int kPT = kRowsG * kCP / kThreads;  // pairs per thread
  int ed[kPT];
#pragma unroll
  for (int u = 0; u < kPT; ++u) {
    const int e = threadIdx.x + u * kThreads, r = e / kCP, c = e % kCP;
    ed[u] = (r < rows && c < p.C) ? p.cand[(r - div_n(r, nmag) * n) * p.C + c] : -1;
  }
  for (int e = threadIdx.x; e < kRowsG * kMaxD0; e += kThreads) {
    const int r = e / kMaxD0, k = e % kMaxD0;
    float v = 0.0f;
    const int gl = div_n(r, nmag);
    if (r < rows && k < p.D0) v = p.nodes[(g0 + gl) * p.nodes_gstride + (int64_t)(r - gl * n) * p.D0 + k];
    L.x0[r * kX0P + k] = v;
  }
  // carries: held in registers until the GNN has released the attention scratch they go to
  constexpr int kHT = kRowsG * kHid / kThreads;
  float hreg[kHT];
#pragma unroll
  for (int u = 0; u < kHT; ++u) {
    const int e = threadIdx.x + u * kThreads, r = e / kHid;
    hreg[u] = r < rows ? p.h_in[row0 * kHid + e] : 0.0f;
  }
  if (two) {
    for (int e = threadIdx.x; e < kMaxD0 * 32; e += kThreads) {
      const int k = e / 32, d = e % 32;
      L.preW[e] = (k < p.D0 && d < p.layer[0].F) ? p.layer[0].Wu[k * p.layer[0].F + d] : 0.0f;
    }
    if (threadIdx.x < 32) L.preb[threadIdx.x] = threadIdx.x < p.layer[0].F ? p.layer[0].bu[threadIdx.x] : 0.0f;
  }
  {
    const int q = threadIdx.x >> 6;  // wave-uniform selection (no private pointer array)
    const float* lsrc = q == 0 ? p.ln0_s : q == 1 ? p.ln0_b : q == 2 ? p.ln1_s : p.ln1_b;
    L.lnp[threadIdx.x] = lsrc[threadIdx.x & 63];
    // [Wm | Wsd] as (64, 2A) rows
    for (int e = threadIdx.x; e < kHid * 2 * A; e += kThreads) {
      const int k = e / (2 * A), j = e % (2 * A);
      L.outW[e] = j < A ? p.Wm[k * A + j] : p.Wsd[k * A + j - A];
    }
    if (threadIdx.x < 2 * A) L.outW[kHid * 2 * A + threadIdx.x] = threadIdx.x < A ? p.bm[threadIdx.x] : p.bsd[threadIdx.x - A];
  }
  // raw rows of the group's never-receiving nodes (graph gl, node n + j -> table row gl (N - n) + j), staged in the
  // xcat region (free until layer 0's attention) for the per-node layer-1 pre-transform
  constexpr int kPreLd = kPreMax * kNarrowD0 / kThreads;
  const int nnr = p.N - n;
  constexpr bool node_pre = NP && MD0 <= kNarrowD0;
  float prv[kPreLd];
  if constexpr (node_pre) {
#pragma unroll
    for (int u = 0; u < kPreLd; ++u) {
      const int e = threadIdx.x + u * kThreads, m = e >> 3, k = e & 7;
      const int gl = m / nnr, j = n + m - gl * nnr;
      prv[u] = (gl < ng && k < p.D0) ? p.nodes[(g0 + gl) * p.nodes_gstride + (int64_t)j * p.D0 + k] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < kPreLd; ++u) L.xc[threadIdx.x + u * kThreads] = prv[u];
  }
  const int tr = threadIdx.x >> 3, tq = threadIdx.x & 7;  // tail: row, action lane
  const bool nz_own = p.mode == 1 && tr < rows && tq < A;
  const float nz = (nz_own && p.noise) ? p.noise[(row0 + tr) * A + tq] : 0.0f;  // else drawn at the tail
  // ---- level 2: resolve the (row, candidate) pairs
  {
    int rc[kPT], sd[kPT];
#pragma unroll
    for (int u = 0; u < kPT; ++u) {
      const int r = (threadIdx.x + u * kThreads) / kCP;
      const int64_t gb = (g0 + div_n(r, nmag)) * p.idx_gstride;
      rc[u] = ed[u] >= 0 ? p.receivers[gb + ed[u]] : -1;
      sd[u] = ed[u] >= 0 ? p.senders[gb + ed[u]] : -1;
    }
#pragma unroll
    for (int u = 0; u < kPT; ++u) {
      const int e = threadIdx.x + u * kThreads, r = e / kCP;
      const bool ok = ed[u] >= 0 && rc[u] == r - div_n(r, nmag) * n;
      L.psrc[e] = ok ? sd[u] : -1;
      L.pedge[e] = ok ? ed[u] : 0;
    }
  }
  __syncthreads();
  // ---- the per-node layer-1 pre-transform: 16-node x 16-column tiles on MFMA, K = the raw width (<= 8) in two
  // steps, bias as the accumulator's start, ReLU on the way to the swizzled table
  if constexpr (node_pre) {
    const int ntile = (gpg * nnr + 15) >> 4;
    for (int t = wave; t < 2 * ntile; t += 4) {
      const int tile = t >> 1, ct = t & 1;
      const float b = L.preb[16 * ct + i16];
      f32x4 acc = {b, b, b, b};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(L.xc[(16 * tile + i16) * kNarrowD0 + 4 * ks + kq],
                                                   L.preW[(4 * ks + kq) * 32 + 16 * ct + i16], acc, 0, 0, 0);
      const int col = 16 * ct + i16;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = 16 * tile + 4 * kq + i;
        L.pre[m * 32 + 4 * ((col >> 2) ^ (m & 7)) + (col & 3)] = acc[i] > 0.0f ? acc[i] : 0.0f;
      }
    }
  }
  // ---- level 3: every pair this lane attends over (kSR sub-rounds), kept in registers for both layers
  PairG<MD0, MEX> pg[kSR];
  {
    const int slot = lane >> 5, c = lane & 31;
#pragma unroll
    for (int sr = 0; sr < kSR; ++sr) pair_gather(p, L, 2 * wave + 8 * sr + slot, c, g0, nmag, pg[sr]);
  }
  __syncthreads();  // the pair tables alias the attention scratch
  PROBE(1);
  // ---- GNN
  {
    constexpr int KX = MEX > 0 ? (kHeads * MEX + 3) / 4 : 1;
    gt_layer_reg<MD0, true, MD0, MEX, (MD0 + 3) / 4, (kHeads * (MD0 + 5) + 3) / 4, KX, (MD0 + 3) / 4>(
        p, p.layer[0], pg, L, p.work, L.x0, kX0P, two ? L.y0 : L.yb, two ? kY0P : kYP, nmag, 2);
    PROBE(4);
    if (two) {
      gt_layer_reg<32, false, MD0, MEX, 8, 28, KX, 8, node_pre>(p, p.layer[1], pg, L, p.work + kQKStride, L.y0, kY0P,
                                                               L.yb, kYP, nmag, 5);
      PROBE(7);
    }
  }
#pragma unroll
  for (int u = 0; u < kHT; ++u) {
    const int e = threadIdx.x + u * kThreads;
    L.hb[(e / kHid) * kYP + e % kHid] = hreg[u];
  }
  // head / GRU / ScaleHid operands: loaded after the GNN (holding them through the attention would
  // spill); each loaded one phase ahead of its GEMM
  // (fi during the second head layer, fh after gi, fs during the gate math) so that at most ~100
  // registers of fragments are live and the kernel fits 3-4 waves per SIMD
  Frag<16, 1> fh0, fh1, fs;
  Frag<16, 3> fi, fh;
  float bh0[1], bh1[1], bs[1], bi[3], bhn[1];
  frag_load(fh0, p.head_W0, kHid, kHid);
  frag_load(fh1, p.head_W1, kHid, kHid);
  bias_load(bh0, p.head_b0, kHid);
  bias_load(bh1, p.head_b1, kHid);
  bias_load(bi, p.gru_bi, 3 * kHid);
  bias_load(bhn, p.gru_bhn, kHid);
  bias_load(bs, p.bs, kHid);
  PROBE(12);
  // ---- MLP head: two Dense(64) + LN + ReLU, in place in L.yb
  {
    f32x4 acc[1][kRT];
    acc_zero(acc);
    frag_mma(acc, L.yb, kYP, kHid, fh0);
    __syncthreads();
    acc_store(acc, L.yb, kYP, kHid, bh0, 1.0f, false);
    __syncthreads();
    ln_relu64(L.yb, L.lnp, L.lnp + kHid);
    __syncthreads();
    frag_load(fi, p.gru_Wi, 3 * kHid, kHid);
    acc_zero(acc);
    frag_mma(acc, L.yb, kYP, kHid, fh1);
    __syncthreads();
    acc_store(acc, L.yb, kYP, kHid, bh1, 1.0f, false);
    __syncthreads();
    ln_relu64(L.yb, L.lnp + 2 * kHid, L.lnp + 3 * kHid);
    __syncthreads();
  }
  PROBE(8);
  // ---- GRU: gi = y Wi + bi, gh = h Wh; wave w's tiles w, w+4, w+8 = r, z, n of hidden cols 16w..16w+15
  {
    f32x4 gi[3][kRT], gh[3][kRT];
    acc_zero(gi);
    acc_zero(gh);
    frag_mma(gi, L.yb, kYP, kHid, fi);
    frag_load(fh, p.gru_Wh, 3 * kHid, kHid);
    frag_mma(gh, L.hb, kYP, kHid, fh);
    frag_load(fs, p.Ws, kHid, kHid);
    const int col = wave * 16 + i16;
    float hn[kRT][4];
#pragma unroll
    for (int rt = 0; rt < kRT; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rt * 16 + 4 * kq + r;
        const float rg = sigm(gi[0][rt][r] + bi[0] + gh[0][rt][r]);
        const float zg = sigm(gi[1][rt][r] + bi[1] + gh[1][rt][r]);
        const float ng = tanhf(gi[2][rt][r] + bi[2] + rg * (gh[2][rt][r] + bhn[0]));
        hn[rt][r] = (1.0f - zg) * ng + zg * L.hb[row * kYP + col];
      }
    __syncthreads();  // every wave has read hb
#pragma unroll
    for (int rt = 0; rt < kRT; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rt * 16 + 4 * kq + r;
        L.hb[row * kYP + col] = hn[rt][r];
#ifndef POLICY_PROBE
        if (row < rows) p.h_out[(row0 + row) * kHid + col] = hn[rt][r];
#endif
      }
    __syncthreads();
  }
  PROBE(9);
  // ---- ScaleHid: s = h' Ws + bs (into yb)
  {
    f32x4 acc[1][kRT];
    acc_zero(acc);
    frag_mma(acc, L.hb, kYP, kHid, fs);
    acc_store(acc, L.yb, kYP, kHid, bs, 1.0f, false);
  }
  __syncthreads();
  PROBE(10);
  // ---- mean / std heads + TanhNormal (policy.py:61-74, distribution.py:24-35): 8 lanes per row,
  // each summing 8 of the 64 features for all 2A outputs, then lane j < A finishes action dim j
  if (threadIdx.x < kRowsG * 8) {  // whole waves
    float part[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) part[j] = 0.0f;
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const int k = tq * 8 + kk;
      const float sv = L.yb[tr * kYP + k];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (j < 2 * A) part[j] += sv * L.outW[k * 2 * A + j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) part[j] = gsum8(part[j]);
    float mu = 0.0f, sraw = 0.0f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      mu = j == tq ? part[j] : mu;
      sraw = j == tq + A ? part[j] : sraw;
    }
    if (tq < A) {
      mu += L.outW[kHid * 2 * A + tq];
      sraw += L.outW[kHid * 2 * A + A + tq];
    }
    const float sd = softplusf(sraw + p.std_shift) + p.std_min;
    // in-kernel noise (noise == NULL): the same Philox element dgppo_normal would have written
    const float nzv = (nz_own && !p.noise) ? noise::normal_at((int64_t)(row0 + tr) * A + tq, *p.noise_seed, p.noise_stream)
                                           : nz;
    const float act = p.mode == 1 ? tanhf(mu + sd * nzv) : tanhf(mu);
    constexpr float kThr = 0.999f;
    const float inv_t = atanhf(kThr), log_eps = logf(1.0f - kThr);
    const float v = fminf(fmaxf(act, -kThr), kThr);
    float lp;
    if (v <= -kThr) lp = log_ndtr((-inv_t - mu) / sd) - log_eps;
    else if (v >= kThr) lp = log_ndtr((mu - inv_t) / sd) - log_eps;
    else {
      const float x = atanhf(v), z = (x - mu) / sd;
      lp = -0.5f * z * z - logf(sd) - 0.91893853320467274f - tanh_fldj(x);
    }
    if (tq >= A) lp = 0.0f;
    // sum over the action dims of the row (lanes tq < A of the 8-lane group)
    const float tot = gsum8(lp);
    if (tr < rows && tq < A) {
      p.action[(row0 + tr) * A + tq] = act;
      if (tq == 0 && p.log_pi) p.log_pi[row0 + tr] = tot;
    }
  }
  PROBE(11);
}

// work[l] = [Wq_h Wkt_h (D x 32 per head) | Wq_h bk_h] rows 0..D-1 and the bias row 32 =
// [bq_h Wkt_h | bq_h . bk_h]; one thread per entry, F-term dot products
__global__ __launch_bounds__(256) void policy_prepare_kernel(dgppo_policy_step_args p) {
  const int l = blockIdx.y;
  const dgppo_gt_layer& ly = p.layer[l];
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= kQKStride) return;
  const int k = idx / kQKCols, col = idx % kQKCols;
  const int D = ly.D, F = ly.F;
  float v = 0.0f;
  if ((k < D || k == 32) && col < 96 + kHeads) {
    const int h = col < 96 ? col / 32 : col - 96, d = col < 96 ? col % 32 : 0;
    if (col >= 96 || d < D) {
      const float* q = k < D ? ly.Wq + (int64_t)k * kHeads * F + h * F : ly.bq + h * F;
      for (int f = 0; f < F; ++f)
        v += q[f] * (col < 96 ? ly.Wkt[((int64_t)h * F + f) * D + d] : ly.bk[h * F + f]);
    }
  }
  p.work[(int64_t)l * kQKStride + idx] = v;
}

size_t lds_bytes() { return lds_floats() * sizeof(float); }

}  // namespace
}  // namespace dgppo

extern "C" int dgppo_policy_step_supported(const dgppo_policy_step_args* p) {
  if (!p) return 0;
  if (p->n_agents < 1 || p->n_agents > dgppo::kRowsG || p->C < 1 || p->C > dgppo::kCP || p->D0 < 1 ||
      p->D0 > dgppo::kMaxD0 || p->A < 1 || p->A > 4 || p->H != dgppo::kHeads || p->ED < 4 ||
      p->ED > 4 + dgppo::kMaxEX)
    return 0;
  for (int l = 0; l < p->n_layers && l < 2; ++l)
    if (p->ED > 4 && !p->layer[l].Wex) return 0;
  if (p->n_layers == 2)
    return p->layer[0].D == p->D0 && p->layer[0].F == 32 && p->layer[1].D == 32 && p->layer[1].F == 64;
  if (p->n_layers == 1) return p->layer[0].D == p->D0 && p->layer[0].F == 64;
  return 0;
}

extern "C" int64_t dgppo_policy_work_floats(void) { return 2 * (int64_t)dgppo::kQKStride; }

extern "C" int dgppo_policy_prepare(const dgppo_policy_step_args* p, void* stream) {
  if (!dgppo_policy_step_supported(p) || !p->work) return DGPPO_EINVAL;
  hipLaunchKernelGGL(dgppo::policy_prepare_kernel, dim3((dgppo::kQKStride + 255) / 256, p->n_layers), dim3(256), 0,
                     (hipStream_t)stream, *p);
  return (int)hipGetLastError();
}

extern "C" int dgppo_policy_step(const dgppo_policy_step_args* p, void* stream) {
  if (!dgppo_policy_step_supported(p) || !p->cand || !p->nodes || !p->edges || !p->receivers || !p->senders ||
      !p->h_in || !p->h_out || !p->action || (p->mode == 1 && !p->noise && !p->noise_seed) || !p->work || p->G < 0)
    return DGPPO_EINVAL;
  if (p->G == 0) return 0;
  const int gpg = dgppo::kRowsG / p->n_agents;
  const int64_t ngroups = (p->G + gpg - 1) / gpg;
  if (ngroups > INT32_MAX) return DGPPO_EINVAL;
  const int64_t grid = ngroups;
  const bool wide = p->D0 > dgppo::kNarrowD0 || p->ED > 4;
  const bool np = !wide && p->n_layers == 2 && (int64_t)gpg * (p->N - p->n_agents) <= dgppo::kPreMax;
  const void* fn = wide ? (const void*)dgppo::policy_step_kernel<dgppo::kMaxD0, dgppo::kMaxEX>
                        : (np ? (const void*)dgppo::policy_step_kernel<dgppo::kNarrowD0, 0, true>
                              : (const void*)dgppo::policy_step_kernel<dgppo::kNarrowD0, 0>);
  const size_t bytes = dgppo::lds_bytes();
  if (bytes > 64 * 1024) dgppo::allow_lds(fn);
  const dim3 g((unsigned)grid), b(dgppo::kThreads);
  const hipStream_t s = (hipStream_t)stream;
  if (wide) hipLaunchKernelGGL((dgppo::policy_step_kernel<dgppo::kMaxD0, dgppo::kMaxEX>), g, b, bytes, s, *p);
  else if (np) hipLaunchKernelGGL((dgppo::policy_step_kernel<dgppo::kNarrowD0, 0, true>), g, b, bytes, s, *p);
  else hipLaunchKernelGGL((dgppo::policy_step_kernel<dgppo::kNarrowD0, 0>), g, b, bytes, s, *p);
  return (int)hipGetLastError();
}
