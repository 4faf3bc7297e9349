// Hot path (2) kernels besides the GEMM: the GraphTransformer attention core, LayerNorm(+ReLU),
// GRU cell, agent mean, TanhNormal head, PPO / L2 losses, Dec-OCP GAE, global-norm clip + Adam,
// and Philox normal noise.  All fp32; forward and backward for everything that carries gradients.
//
// GraphTransformer (dgppo/nn/gnn.py:78-117).  In every DGPPO env graph only agent nodes receive
// messages (all other edges are masked to the pad node), so per receiving agent i and head h:
//   logit_c = (q_h . k_c) / sqrt(F),  k_c = x_{s_c} Wk_h + bk_h
//           = (qt_h . x_{s_c} + q_h . bk_h) / sqrt(F),  with qt_h = Wk_h q_h   (D-dim, not F-dim)
//   sum_c a_c (v_c + e_c) = xbar_h Wv_h + sig_h bv_h + ebar_h We_h
//           with xbar_h = sum_c a_c x_{s_c}, ebar_h = sum_c a_c ef_c, sig_h = sum_c a_c
// i.e. the per-edge K/V/E projections of the reference collapse into per-agent dense products
// (GEMMs over all agents of the batch, dgppo_gemm) plus this O(C * H * D) gather core.  The
// result equals the reference's up to fp32 rounding.
#include <hip/hip_runtime.h>

#include "lds_attr.h"
#include <math.h>
#include <stdint.h>

#include "../../include/dgppo_hip.h"
#include "noise.h"

namespace dgppo {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }
__device__ __forceinline__ float softplusf_(float x) { return x > 20.0f ? x : log1pf(expf(x)); }

// ---- LayerNorm (+ReLU) over rows of width F (flax LayerNorm, eps 1e-6, fast variance) --------
// ---- F = 64 LayerNorm: 16 lanes x float4 per row, 16 rows per 256-thread block ----------------
__device__ __forceinline__ float sum16(float v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ __launch_bounds__(256) void layernorm64_fwd_kernel(const float* x, const float* scale, const float* bias,
                                                              float* y, float* mean_out, float* rstd_out,
                                                              int64_t rows, int relu, float eps) {
  const int c4 = threadIdx.x & 15;
  const float4 sc = ((const float4*)scale)[c4], bi = ((const float4*)bias)[c4];
  for (int64_t r = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4); r < rows; r += (int64_t)gridDim.x * 16) {
    const float4 v = ((const float4*)(x + r * 64))[c4];
    const float s = sum16((v.x + v.y) + (v.z + v.w));
    const float s2 = sum16((v.x * v.x + v.y * v.y) + (v.z * v.z + v.w * v.w));
    const float mean = s / 64.0f;
    float var = s2 / 64.0f - mean * mean;
    var = var > 0.0f ? var : 0.0f;
    const float rstd = 1.0f / sqrtf(var + eps);
    float4 o;
    o.x = (v.x - mean) * rstd * sc.x + bi.x;
    o.y = (v.y - mean) * rstd * sc.y + bi.y;
    o.z = (v.z - mean) * rstd * sc.z + bi.z;
    o.w = (v.w - mean) * rstd * sc.w + bi.w;
    if (relu) {
      o.x = o.x > 0.0f ? o.x : 0.0f, o.y = o.y > 0.0f ? o.y : 0.0f;
      o.z = o.z > 0.0f ? o.z : 0.0f, o.w = o.w > 0.0f ? o.w : 0.0f;
    }
    ((float4*)(y + r * 64))[c4] = o;
    if (c4 == 0) {
      mean_out[r] = mean;
      rstd_out[r] = rstd;
    }
  }
}

// dx (overwrite) and this block's partial [dscale (64) | dbias (64)] over rows [b*rpb, (b+1)*rpb)
__global__ __launch_bounds__(256) void layernorm64_bwd_kernel(const float* x, const float* y, const float* dy,
                                                              const float* scale, const float* mean_in,
                                                              const float* rstd_in, float* dx, float* part,
                                                              int64_t rows, int relu, int64_t rpb) {
  __shared__ float red[16][2 * 64 + 4];
  const int c4 = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const float4 sc = ((const float4*)scale)[c4];
  float ds[4] = {0.0f, 0.0f, 0.0f, 0.0f}, db[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  const int64_t r0 = (int64_t)blockIdx.x * rpb;
  const int64_t r1 = r0 + rpb < rows ? r0 + rpb : rows;
  for (int64_t r = r0 + rl; r < r1; r += 16) {
    const float4 xv = ((const float4*)(x + r * 64))[c4];
    float4 g = ((const float4*)(dy + r * 64))[c4];
    if (relu) {
      const float4 yv = ((const float4*)(y + r * 64))[c4];
      g.x = yv.x > 0.0f ? g.x : 0.0f, g.y = yv.y > 0.0f ? g.y : 0.0f;
      g.z = yv.z > 0.0f ? g.z : 0.0f, g.w = yv.w > 0.0f ? g.w : 0.0f;
    }
    const float mean = mean_in[r], rstd = rstd_in[r];
    const float xh[4] = {(xv.x - mean) * rstd, (xv.y - mean) * rstd, (xv.z - mean) * rstd, (xv.w - mean) * rstd};
    const float gg[4] = {g.x, g.y, g.z, g.w};
    const float sv[4] = {sc.x, sc.y, sc.z, sc.w};
    float s1 = 0.0f, s2 = 0.0f, gx[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      ds[j] += gg[j] * xh[j];
      db[j] += gg[j];
      gx[j] = gg[j] * sv[j];
      s1 += gx[j];
      s2 += gx[j] * xh[j];
    }
    s1 = sum16(s1) / 64.0f;
    s2 = sum16(s2) / 64.0f;
    float4 o;
    o.x = rstd * (gx[0] - s1 - xh[0] * s2);
    o.y = rstd * (gx[1] - s1 - xh[1] * s2);
    o.z = rstd * (gx[2] - s1 - xh[2] * s2);
    o.w = rstd * (gx[3] - s1 - xh[3] * s2);
    ((float4*)(dx + r * 64))[c4] = o;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    red[rl][4 * c4 + j] = ds[j];
    red[rl][64 + 4 * c4 + j] = db[j];
  }
  __syncthreads();
  if (threadIdx.x < 128) {
    float acc = 0.0f;
    for (int q = 0; q < 16; ++q) acc += red[q][threadIdx.x];
    part[(int64_t)blockIdx.x * 128 + threadIdx.x] = acc;
  }
}

__global__ __launch_bounds__(256) void layernorm_fwd_kernel(const float* x, const float* scale, const float* bias,
                                                            float* y, float* mean_out, float* rstd_out,
                                                            int64_t rows, int F, int relu, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const float* xr = x + r * F;
  float s = 0.0f, s2 = 0.0f;
  for (int f = lane; f < F; f += 64) {
    const float v = xr[f];
    s += v;
    s2 += v * v;
  }
  s = wave_sum(s);
  s2 = wave_sum(s2);
  const float mean = s / F;
  float var = s2 / F - mean * mean;
  var = var > 0.0f ? var : 0.0f;
  const float rstd = 1.0f / sqrtf(var + eps);
  for (int f = lane; f < F; f += 64) {
    float v = (xr[f] - mean) * rstd * scale[f] + bias[f];
    if (relu) v = v > 0.0f ? v : 0.0f;
    y[r * F + f] = v;
  }
  if (lane == 0) {
    mean_out[r] = mean;
    rstd_out[r] = rstd;
  }
}

// dx (overwrite), and per-block partial sums of dscale / dbias -> part[(block, 2, F)]
__global__ __launch_bounds__(256) void layernorm_bwd_kernel(const float* x, const float* y, const float* dy,
                                                            const float* scale, const float* mean_in,
                                                            const float* rstd_in, float* dx, float* part,
                                                            int64_t rows, int F, int relu, int rows_per_block) {
  extern __shared__ __attribute__((aligned(16))) float acc[];  // 4 waves x 2F
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int t = threadIdx.x; t < 8 * F; t += 256) acc[t] = 0.0f;
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  for (int64_t r = r0 + wave; r < r0 + rows_per_block && r < rows; r += 4) {
    const float mean = mean_in[r], rstd = rstd_in[r];
    float s1 = 0.0f, s2 = 0.0f;
    for (int f = lane; f < F; f += 64) {
      float g = dy[r * F + f];
      if (relu && !(y[r * F + f] > 0.0f)) g = 0.0f;
      const float xh = (x[r * F + f] - mean) * rstd;
      acc[wave * 2 * F + f] += g * xh;
      acc[wave * 2 * F + F + f] += g;
      const float gx = g * scale[f];
      s1 += gx;
      s2 += gx * xh;
    }
    s1 = wave_sum(s1) / F;
    s2 = wave_sum(s2) / F;
    for (int f = lane; f < F; f += 64) {
      float g = dy[r * F + f];
      if (relu && !(y[r * F + f] > 0.0f)) g = 0.0f;
      const float xh = (x[r * F + f] - mean) * rstd;
      dx[r * F + f] = rstd * (g * scale[f] - s1 - xh * s2);
    }
  }
  __syncthreads();
  for (int t = threadIdx.x; t < 2 * F; t += 256)
    part[(int64_t)blockIdx.x * 2 * F + t] = acc[t] + acc[2 * F + t] + acc[4 * F + t] + acc[6 * F + t];
}

// ---- column sums (deterministic two-level) ----------------------------------------------------
__host__ inline bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// Row partition shared by every two-level reduction: at most kMaxParts partial rows, each block
// owning a contiguous run of >= min_rows rows.
constexpr int kMaxParts = 512;
struct RowSplit {
  int nb;
  int64_t rpb;
};
__host__ __device__ inline RowSplit row_split(int64_t rows, int64_t min_rows) {
  int64_t nb = (rows + min_rows - 1) / min_rows;
  if (nb > kMaxParts) nb = kMaxParts;
  if (nb < 1) nb = 1;
  return {(int)nb, (rows + nb - 1) / nb};
}

// part[b][c] = sum of rows [b*rpb, (b+1)*rpb) of x (grouped row addressing as in the GEMM).
// cols <= 256: 256/cols threads per column walk interleaved rows, combined in LDS in fixed order.
__global__ __launch_bounds__(256) void colsum_partial_kernel(const float* x, int64_t rows, int cols, int64_t ld,
                                                             int grp, int64_t gstride, float* part,
                                                             int64_t rows_per_block) {
  __shared__ float red[256];
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(rows, r0 + rows_per_block);
  if (cols <= 256) {
    const int tpc = 256 / cols;
    const int c = threadIdx.x % cols, j = threadIdx.x / cols;
    float s = 0.0f;
    if (j < tpc) {
      for (int64_t r = r0 + j; r < r1; r += tpc) {
        const int64_t off = grp > 0 ? (r / grp) * gstride + (r % grp) * ld : r * ld;
        s += x[off + c];
      }
    }
    red[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x < cols) {
      float t = 0.0f;
      for (int k = 0; k < tpc; ++k) t += red[k * cols + threadIdx.x];
      part[(int64_t)blockIdx.x * cols + threadIdx.x] = t;
    }
    return;
  }
  for (int c = threadIdx.x; c < cols; c += 256) {
    float s = 0.0f;
    for (int64_t r = r0; r < r1; ++r) {
      const int64_t off = grp > 0 ? (r / grp) * gstride + (r % grp) * ld : r * ld;
      s += x[off + c];
    }
    part[(int64_t)blockIdx.x * cols + c] = s;
  }
}

// out[c] = alpha * sum_b part[b * pstride + c] + beta * out[c]; 16 columns x 16 phases per block
__global__ __launch_bounds__(256) void colsum_final_kernel(const float* part, int nparts, int cols, int64_t pstride,
                                                           float* out, float alpha, float beta) {
  __shared__ float red[16][17];
  const int cl = threadIdx.x & 15, j = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  float s = 0.0f;
  if (c < cols) {
#pragma unroll 4
    for (int b = j; b < nparts; b += 16) s += part[(int64_t)b * pstride + c];
  }
  red[j][cl] = s;
  __syncthreads();
  if (threadIdx.x < 16 && c < cols) {
    float t = 0.0f;
    for (int q = 0; q < 16; ++q) t += red[q][cl];
    out[c] = alpha * t + (beta != 0.0f ? beta * out[c] : 0.0f);
  }
}

// ---- GRU cell (flax GRUCell) ------------------------------------------------------------------
// gi = x Wi + bi (rows, 3H: r|z|n), gh = h Wh (rows, 3H, no bias), bhn (H)
__global__ __launch_bounds__(256) void gru_fwd_kernel(const float* gi, const float* gh, const float* bhn,
                                                      const float* h, float* hn_out, int64_t rows, int H) {
  const int64_t total = rows * H;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int64_t r = t / H;
    const int j = (int)(t - r * H);
    const float* a = gi + r * 3 * H;
    const float* b = gh + r * 3 * H;
    const float rg = sigmoidf_(a[j] + b[j]);
    const float zg = sigmoidf_(a[H + j] + b[H + j]);
    const float ng = tanhf(a[2 * H + j] + rg * (b[2 * H + j] + bhn[j]));
    hn_out[t] = (1.0f - zg) * ng + zg * h[t];
  }
}

// dgi, dgh (overwrite), dh (+= direct path)
__global__ __launch_bounds__(256) void gru_bwd_kernel(const float* gi, const float* gh, const float* bhn,
                                                      const float* h, const float* dhn, float* dgi, float* dgh,
                                                      float* dh, int64_t rows, int H) {
  const int64_t total = rows * H;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int64_t r = t / H;
    const int j = (int)(t - r * H);
    const float* a = gi + r * 3 * H;
    const float* b = gh + r * 3 * H;
    const float rg = sigmoidf_(a[j] + b[j]);
    const float zg = sigmoidf_(a[H + j] + b[H + j]);
    const float hnp = b[2 * H + j] + bhn[j];
    const float ng = tanhf(a[2 * H + j] + rg * hnp);
    const float g = dhn[t];
    const float dz = g * (h[t] - ng);
    const float dn = g * (1.0f - zg);
    const float dn_pre = dn * (1.0f - ng * ng);
    const float dr = dn_pre * hnp;
    const float dr_pre = dr * rg * (1.0f - rg);
    const float dz_pre = dz * zg * (1.0f - zg);
    float* ai = dgi + r * 3 * H;
    float* bi = dgh + r * 3 * H;
    ai[j] = dr_pre;
    ai[H + j] = dz_pre;
    ai[2 * H + j] = dn_pre;
    bi[j] = dr_pre;
    bi[H + j] = dz_pre;
    bi[2 * H + j] = dn_pre * rg;
    dh[t] += g * zg;
  }
}

// ---- mean over the n agents of each graph: (G, n, F) <-> (G, F) ------------------------------
__global__ __launch_bounds__(256) void agent_mean_fwd_kernel(const float* x, float* y, int64_t G, int n, int F,
                                                             int64_t x_gstride) {
  const int64_t total = G * F;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int64_t g = t / F;
    const int f = (int)(t - g * F);
    float s = 0.0f;
    for (int i = 0; i < n; ++i) s += x[g * x_gstride + (int64_t)i * F + f];
    y[t] = s / n;
  }
}

// mask (optional, (G n, F) contiguous): the ReLU output that fed the mean; dx = mask > 0 ? dy / n : 0 (the ReLU
// backward fused, as dgppo_relu_bwd would apply it after the broadcast)
__global__ __launch_bounds__(256) void agent_mean_bwd_kernel(const float* dy, float* dx, int64_t G, int n, int F,
                                                             int64_t dx_gstride, const float* mask) {
  const int64_t total = G * n * F;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int64_t g = t / ((int64_t)n * F);
    const int64_t rem = t - g * n * F;
    const int i = (int)(rem / F), f = (int)(rem - (int64_t)(rem / F) * F);
    float v = dy[g * F + f] / n;
    if (mask && !(mask[t] > 0.0f)) v = 0.0f;
    dx[g * dx_gstride + (int64_t)i * F + f] = v;
  }
}

// ---- TanhNormal head (distribution.py:10-66 + tfp Normal / Tanh / Independent) ----------------
__device__ __forceinline__ float log_ndtr_f(float z) {
  if (z > -10.0f) return logf(0.5f * erfcf(-z * 0.70710678118654752f));
  // asymptotic series for the far left tail
  const float z2 = z * z;
  const float s = 1.0f - 1.0f / z2 + 3.0f / (z2 * z2) - 15.0f / (z2 * z2 * z2);
  return -0.5f * z2 - logf(-z) - 0.91893853320467274f + logf(s);
}
// d/dz log Phi(z) = phi(z) / Phi(z)
__device__ __forceinline__ float dlog_ndtr_f(float z) {
  const float lp = -0.5f * z * z - 0.91893853320467274f;
  return expf(lp - log_ndtr_f(z));
}
__device__ __forceinline__ float tanh_fldj_f(float x) {  // 2 (log 2 - x - softplus(-2x))
  return 2.0f * (0.69314718055994531f - x - softplusf_(-2.0f * x));
}

__global__ __launch_bounds__(256) void tanh_normal_kernel(dgppo_tanh_normal_args p) {
  constexpr float kThr = 0.999f;
  const float inv_t = atanhf(kThr);
  const float log_eps = logf(1.0f - kThr);
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < p.rows; r += (int64_t)gridDim.x * 256) {
    float lp_sum = 0.0f, ent_sum = 0.0f;
    for (int j = 0; j < p.A; ++j) {
      const int64_t k = r * p.A + j;
      const float mu = p.mean[k];
      const float sraw = p.std_raw[k] + p.std_shift;
      const float sd = softplusf_(sraw) + p.std_min;
      if (p.std_out) p.std_out[k] = sd;
      float a;
      if (p.mode == 0) a = tanhf(mu);                         // mode(): tanh(mean)
      else if (p.mode == 1) a = tanhf(mu + sd * p.noise[k]);  // sample
      else a = p.action[k];                                   // evaluate given actions
      if (p.mode <= 1 && p.action_out) p.action_out[k] = a;
      // log_prob with the threshold clip
      const float v = fminf(fmaxf(a, -kThr), kThr);
      float lp, dmu, dsd;
      if (v <= -kThr) {
        const float w = (-inv_t - mu) / sd;
        lp = log_ndtr_f(w) - log_eps;
        const float lam = dlog_ndtr_f(w);
        dmu = -lam / sd;
        dsd = -lam * w / sd;
      } else if (v >= kThr) {
        const float u = (mu - inv_t) / sd;
        lp = log_ndtr_f(u) - log_eps;
        const float lam = dlog_ndtr_f(u);
        dmu = lam / sd;
        dsd = -lam * u / sd;
      } else {
        const float x = atanhf(v);
        const float z = (x - mu) / sd;
        lp = -0.5f * z * z - logf(sd) - 0.91893853320467274f - tanh_fldj_f(x);
        dmu = z / sd;
        dsd = (z * z - 1.0f) / sd;
      }
      lp_sum += lp;
      float dmu_e = 0.0f, dsd_e = 0.0f;
      if (p.entropy_eps) {  // entropy = N entropy + fldj(mu + sd * eps_fixed[agent])
        const int agent = (int)(r % p.n_agents);
        const float eps = p.entropy_eps[agent * p.A + j];
        const float ysmp = mu + sd * eps;
        ent_sum += 1.41893853320467274f + logf(sd) + tanh_fldj_f(ysmp);
        const float dfl = -2.0f * tanhf(ysmp);
        dmu_e = dfl;
        dsd_e = 1.0f / sd + dfl * eps;
      }
      if (p.dmean) {  // backward: upstream dlog_pi[r], dentropy[r]
        const float glp = p.dlog_pi ? p.dlog_pi[r] : 0.0f;
        const float gen = p.dentropy ? p.dentropy[r] : 0.0f;
        const float dsd_tot = glp * dsd + gen * dsd_e;
        p.dmean[k] = glp * dmu + gen * dmu_e;
        p.dstd_raw[k] = dsd_tot * sigmoidf_(sraw);
      }
    }
    if (p.log_pi) p.log_pi[r] = lp_sum;
    if (p.entropy) p.entropy[r] = ent_sum;
  }
}

// ---- losses ------------------------------------------------------------------------------------
// block partial sums: part[block*8 + q]
__device__ __forceinline__ void block_sums(float* vals, int nv, float* part) {
  __shared__ float red[8][4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int q = 0; q < nv; ++q) {
    const float s = wave_sum(vals[q]);
    if (lane == 0) red[q][wave] = s;
  }
  __syncthreads();
  if (threadIdx.x < nv) {
    const int q = threadIdx.x;
    part[blockIdx.x * 8 + q] = red[q][0] + red[q][1] + red[q][2] + red[q][3];
  }
}

// PPO clipped surrogate (informarl.py:428-438): grads into dlog_pi / dentropy; stats partials:
// [sum max(l1,l2), sum entropy, sum (l2 > l1), sum |ratio - 1|]
__global__ __launch_bounds__(256) void ppo_loss_kernel(const float* log_pi, const float* log_pi_old, const float* adv,
                                                       const float* entropy, int64_t n, float clip_eps, float coef_ent,
                                                       float* dlog_pi, float* dentropy, float* part) {
  float v[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  const float inv_n = 1.0f / (float)n;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < n; t += (int64_t)gridDim.x * 256) {
    const float r = expf(log_pi[t] - log_pi_old[t]);
    const float A = adv[t];
    const float l1 = -r * A;
    const float rc = fminf(fmaxf(r, 1.0f - clip_eps), 1.0f + clip_eps);
    const float l2 = -rc * A;
    const float in_range = (r >= 1.0f - clip_eps && r <= 1.0f + clip_eps) ? 1.0f : 0.0f;
    float g;
    if (l1 > l2) g = -A * r;
    else if (l1 < l2) g = -A * r * in_range;
    else g = 0.5f * (-A * r) + 0.5f * (-A * r * in_range);  // jnp.maximum splits ties
    dlog_pi[t] = g * inv_n;
    dentropy[t] = -coef_ent * inv_n;
    v[0] += fmaxf(l1, l2);
    v[1] += entropy[t];
    v[2] += l2 > l1 ? 1.0f : 0.0f;
    v[3] += fabsf(r - 1.0f);
  }
  block_sums(v, 4, part);
}

// 0.5 * mean (pred - target)^2 (optax.l2_loss): grad = (pred - target) / n; partial [sum loss]
__global__ __launch_bounds__(256) void l2_loss_kernel(const float* pred, const float* target, int64_t n,
                                                      float* dpred, float* part) {
  float v[1] = {0.0f};
  const float inv_n = 1.0f / (float)n;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < n; t += (int64_t)gridDim.x * 256) {
    const float d = pred[t] - target[t];
    dpred[t] = d * inv_n;
    v[0] += 0.5f * d * d;
  }
  block_sums(v, 1, part);
}

__global__ __launch_bounds__(64) void partial_reduce_kernel(const float* part, int nparts, int nv, float* out,
                                                            float scale) {
  for (int v = 0; v < nv; ++v) {  // lanes stride the partials, fixed-order butterfly -> deterministic
    float s = 0.0f;
    for (int b = threadIdx.x; b < nparts; b += 64) s += part[b * 8 + v];
    s = wave_sum(s);
    if (threadIdx.x == 0) out[v] = s * scale;
  }
}

// ---- Dec-OCP GAE (dgppo/algo/utils.py:11-79), one 256-thread workgroup per env ----------------
// The reference scans the data from time T-1 down to 0 (lax.scan(reverse=True) over
// ts = arange(T)[::-1]) and its loop variable ii = T-1-k COUNTS the steps: at step ii the rows
// 0..ii of the (T+1)-row table are live, row t holds an n-step backup (n = ii - t + 1 for t >= 1,
// ii + 1 for t = 0) and the output is Q[k] = sum_t c_ii[t] row[t] with c_ii[0] = lambda^ii and
// c_ii[t] = lambda^(ii-t) (1 - lambda) (the rolled coefficient vector, closed form).  Every row
// entry evolves independently, so thread (column q, chunk c) keeps the entries t = c + C e of
// column q in registers (columns: the n*nh Vh heads, then the Vl column); the weighted sum is a
// reduction over the C lanes of the column.  The env's inputs are staged in LDS once, so the T
// sequential steps never wait on HBM.  Work is O(T^2) per column like the reference's row update
// (its max(.) is not reducible to an O(T) recursion).
template <int EPL>
__global__ __launch_bounds__(256) void gae_kernel(dgppo_gae_args p, int C) {
  extern __shared__ __attribute__((aligned(16))) float sh[];
  const int T = p.T, n = p.n_agents, nh = p.n_h, K = n * nh, Tp1 = T + 1;
  float* s_hs = sh;                 // (T, K)
  float* s_Vh = s_hs + T * K;       // (T+1, K)
  float* s_l = s_Vh + Tp1 * K;      // (T)
  float* s_Vl = s_l + T;            // (T+1)
  float* s_pw = s_Vl + Tp1;         // lambda^j, j = 0..T
  float* s_pw1 = s_pw + Tp1;        // lambda^j (1 - lambda)
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x;
  {
    const float* hs = p.hs + b * (int64_t)T * K;
    const float* Vh = p.Vh + b * (int64_t)Tp1 * K;
    for (int i = tid; i < T * K; i += 256) s_hs[i] = hs[i];
    for (int i = tid; i < Tp1 * K; i += 256) s_Vh[i] = Vh[i];
    for (int i = tid; i < T; i += 256) s_l[i] = p.l[b * T + i];
    for (int i = tid; i < Tp1; i += 256) {
      s_Vl[i] = p.Vl[b * Tp1 + i];
      const float pw = powf(p.lambda, (float)i);
      s_pw[i] = pw;
      s_pw1[i] = pw * (1.0f - p.lambda);
    }
  }
  __syncthreads();
  const int q = tid / C, c = tid - (tid / C) * C;
  if (q > K) return;  // padding columns (no barrier below)
  const bool is_l = q == K;
  const int a = is_l ? 0 : q / nh;
  const float gamma = p.gamma, omg = 1.0f - p.gamma;
  float row[EPL];
#pragma unroll
  for (int e = 0; e < EPL; ++e) row[e] = 0.0f;
  if (c == 0) row[0] = is_l ? s_Vl[T] : s_Vh[T * K + q];  // row 0 = V(x_T)
  for (int ii = 0; ii < T; ++ii) {
    const int k = T - 1 - ii;
    float hv = 0.0f, hmax = 0.0f, lv = 0.0f;
    if (is_l) {
      lv = s_l[k];
    } else {
      hv = s_hs[k * K + q];
      hmax = s_hs[k * K + a * nh];
      for (int h = 1; h < nh; ++h) hmax = fmaxf(hmax, s_hs[k * K + a * nh + h]);
    }
    const float base = omg * hmax;
    float acc = 0.0f;
#pragma unroll
    for (int e = 0; e < EPL; ++e) {
      if (e * C > ii) break;  // uniform: no live entry left in this or later slots
      const int t = c + C * e;
      if (t <= ii) {
        const float r = is_l ? lv + gamma * row[e] : fmaxf(hv, base + gamma * row[e]);
        row[e] = r;
        acc += (t == 0 ? s_pw[ii] : s_pw1[ii - t]) * r;
      }
    }
    for (int o = 1; o < C; o <<= 1) acc += __shfl_xor(acc, o, 64);
    if (c == 0) {
      if (is_l) p.Ql[b * T + k] = acc;
      else p.Qh[(b * T + k) * K + q] = acc;
    }
    // row ii + 1 <- V(x_k) for the next step
    const int t1 = ii + 1;
    if (c == t1 % C) {
      const float v = is_l ? s_Vl[k] : s_Vh[k * K + q];
      const int e1 = t1 / C;
#pragma unroll
      for (int e = 0; e < EPL; ++e)
        if (e == e1) row[e] = v;
    }
  }
}

// ---- DGPPO advantages (dgppo/algo/dgppo.py:239-259), one workgroup per env -------------------
//   Al = norm_t(Ql - Vl) (population std + 1e-8), cbf = (Vh_{t+1} - Vh_t)/dt + alpha Vh_t,
//   safe = all_h(cbf <= 0), A = -(where(safe, Al, 0) + max_h relu(cbf + eps) * w)
__global__ __launch_bounds__(256) void dgppo_adv_kernel(dgppo_adv_args p) {
  __shared__ float red[2][4];
  const int64_t b = blockIdx.x;
  const int T = p.T, n = p.n_agents, nh = p.n_h;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* Ql = p.Ql + b * T;
  const float* Vl = p.Vl + b * (T + 1);
  float s = 0.0f;
  for (int t = tid; t < T; t += 256) s += Ql[t] - Vl[t];
  s = wave_sum(s);
  if (lane == 0) red[0][wave] = s;
  __syncthreads();
  const float mean = (red[0][0] + red[0][1] + red[0][2] + red[0][3]) / T;
  float s2 = 0.0f;
  for (int t = tid; t < T; t += 256) {
    const float d = (Ql[t] - Vl[t]) - mean;
    s2 += d * d;
  }
  s2 = wave_sum(s2);
  if (lane == 0) red[1][wave] = s2;
  __syncthreads();
  const float sd = sqrtf((red[1][0] + red[1][1] + red[1][2] + red[1][3]) / T);
  const float* Vh = p.Vh + b * (int64_t)(T + 1) * n * nh;
  float safe_cnt = 0.0f;
  for (int q = tid; q < T * n; q += 256) {
    const int t = q / n, i = q - (q / n) * n;
    const float al = ((Ql[t] - Vl[t]) - mean) / (sd + 1e-8f);
    bool safe = true;
    float amax = 0.0f;
    for (int h = 0; h < nh; ++h) {
      const float v0 = Vh[((int64_t)t * n + i) * nh + h];
      const float v1 = Vh[((int64_t)(t + 1) * n + i) * nh + h];
      const float dv = (v1 - v0) / p.dt + p.alpha * v0;
      safe = safe && (dv <= 0.0f);
      const float ac = fmaxf(dv + p.cbf_eps, 0.0f);
      amax = h == 0 ? ac : fmaxf(amax, ac);
    }
    p.A[(b * T + t) * n + i] = -((safe ? al : 0.0f) + amax * p.cbf_weight);
    safe_cnt += safe ? 1.0f : 0.0f;
  }
  safe_cnt = wave_sum(safe_cnt);
  __syncthreads();
  if (lane == 0) red[0][wave] = safe_cnt;
  __syncthreads();
  if (tid == 0) p.safe_count[b] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
}

// ---- global norm / finite check, clipped Adam (optax.adam + apply_if_finite) ------------------
__global__ __launch_bounds__(256) void sumsq_partial_kernel(const float* g, int64_t n, float* part) {
  float v[2] = {0.0f, 0.0f};
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < n; t += (int64_t)gridDim.x * 256) {
    const float x = g[t];
    v[0] += x * x;
    v[1] += isfinite(x) ? 0.0f : 1.0f;
  }
  block_sums(v, 2, part);
}

// state[0] = global norm, state[1] = non-finite count, state[2] = adam step count (float)
__global__ __launch_bounds__(64) void norm_final_kernel(const float* part, int nparts, float* state) {
  float s = 0.0f, nf = 0.0f;
  for (int b = threadIdx.x; b < nparts; b += 64) {
    s += part[b * 8 + 0];
    nf += part[b * 8 + 1];
  }
  s = wave_sum(s);
  nf = wave_sum(nf);
  if (threadIdx.x == 0) {
    state[0] = sqrtf(s);
    state[1] = nf;
  }
}

__global__ __launch_bounds__(256) void adam_kernel(float* param, const float* grad, float* m, float* v, int64_t n,
                                                   const float* state, float lr, float b1, float omb1, float b2,
                                                   float omb2, float eps, float max_norm) {
  if (state[1] != 0.0f) return;  // apply_if_finite: skip the whole update
  const float gnorm = state[0];
  const float c = fmaxf(max_norm, gnorm);
  const float t = state[2] + 1.0f;
  const float bc1 = 1.0f - powf(b1, t);
  const float bc2 = 1.0f - powf(b2, t);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float g = (grad[i] / c) * max_norm;
    const float mi = b1 * m[i] + omb1 * g;  // optax: (1 - decay) folded in double, then rounded (weak type)
    const float vi = b2 * v[i] + omb2 * (g * g);
    m[i] = mi;
    v[i] = vi;
    param[i] = param[i] - lr * ((mi / bc1) / (sqrtf(vi / bc2) + eps));
  }
}

__global__ void adam_count_kernel(float* state) {
  if (threadIdx.x == 0 && state[1] == 0.0f) state[2] += 1.0f;
}

// ---- several nets' grad_norm + adam in two launches (dgppo_adam_multi): blockIdx.y = net.  The partials, the
// norm (wave 0 of every workgroup redoes norm_final_kernel's sums over the same partials) and the update are
// norm_final / adam_kernel's arithmetic, so the results are bit-identical to the per-net launches.
constexpr int kAdamParts = 512;  // = kLossBlocks: partial blocks per net
struct AdamMultiDev {
  dgppo_adam_multi_args a;
  float omb1, omb2;
};
__global__ __launch_bounds__(256) void sumsq_multi_kernel(AdamMultiDev d) {
  const dgppo_adam_net& t = d.a.net[blockIdx.y];
  float* part = d.a.workspace + (int64_t)blockIdx.y * kAdamParts * 8;
  float v[2] = {0.0f, 0.0f};
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < t.n; i += (int64_t)gridDim.x * 256) {
    const float x = t.grad[i];
    v[0] += x * x;
    v[1] += isfinite(x) ? 0.0f : 1.0f;
  }
  block_sums(v, 2, part);
  // the step count before this update, read by every workgroup of the second kernel (workgroup 0 rewrites state)
  if (blockIdx.x == 0 && threadIdx.x == 0) d.a.workspace[(int64_t)DGPPO_ADAM_MAX_NETS * kAdamParts * 8 + blockIdx.y] = t.state[2];
}
__global__ __launch_bounds__(256) void adam_multi_kernel(AdamMultiDev d) {
  const dgppo_adam_net& t = d.a.net[blockIdx.y];
  const float* part = d.a.workspace + (int64_t)blockIdx.y * kAdamParts * 8;
  __shared__ float nrm[2];
  if (threadIdx.x < 64) {
    float s = 0.0f, nf = 0.0f;
    for (int b = threadIdx.x; b < kAdamParts; b += 64) {
      s += part[b * 8 + 0];
      nf += part[b * 8 + 1];
    }
    s = wave_sum(s);
    nf = wave_sum(nf);
    if (threadIdx.x == 0) {
      nrm[0] = sqrtf(s);
      nrm[1] = nf;
    }
  }
  __syncthreads();
  const float gnorm = nrm[0], nf = nrm[1];
  const float count = d.a.workspace[(int64_t)DGPPO_ADAM_MAX_NETS * kAdamParts * 8 + blockIdx.y];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    t.state[0] = gnorm;
    t.state[1] = nf;
    if (nf == 0.0f) t.state[2] = count + 1.0f;
  }
  if (nf != 0.0f) return;  // apply_if_finite: skip the whole update
  const float b1 = (float)d.a.b1, b2 = (float)d.a.b2, max_norm = t.max_norm, lr = t.lr, eps = d.a.eps;
  const float c = fmaxf(max_norm, gnorm);
  const float tt = count + 1.0f;
  const float bc1 = 1.0f - powf(b1, tt);
  const float bc2 = 1.0f - powf(b2, tt);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < t.n; i += (int64_t)gridDim.x * 256) {
    const float g = (t.grad[i] / c) * max_norm;
    const float mi = b1 * t.m[i] + d.omb1 * g;
    const float vi = b2 * t.v[i] + d.omb2 * (g * g);
    t.m[i] = mi;
    t.v[i] = vi;
    t.param[i] = t.param[i] - lr * ((mi / bc1) / (sqrtf(vi / bc2) + eps));
  }
}

// ---- Philox normals (Box-Muller, noise.h) ----------------------------------------------------------
__global__ __launch_bounds__(256) void normal_kernel(float* out, int64_t n, const uint64_t* seed_ptr, uint64_t seed,
                                                     uint64_t stream_id) {
  const uint64_t sd = seed_ptr ? *seed_ptr : seed;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < n; t += (int64_t)gridDim.x * 256)
    out[t] = noise::normal_at(t, sd, stream_id);
}

__global__ __launch_bounds__(256) void relu_bwd_kernel(float* dy, const float* y, int64_t n) {
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < n; t += (int64_t)gridDim.x * 256)
    if (!(y[t] > 0.0f)) dy[t] = 0.0f;
}

static int grid_for(int64_t n) {
  const int64_t b = (n + 255) / 256;
  return (int)(b < 8192 ? (b < 1 ? 1 : b) : 8192);
}

// flax.linen.LSTMCell gate math for one step of `rows` carries (the --use-lstm option, dgppo/nn/rnn.py:15-30):
// g (rows, 4H) = [i | f | g | o] pre-activations (x W_i + h W_h + b, from the GEMMs) -> activated in place;
// c' = f c + i g, h' = o tanh(c').  A thread per (row, column); the gate columns of a row are H apart.
__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

__global__ __launch_bounds__(256) void lstm_cell_fwd_kernel(int64_t rows, int H, float* __restrict__ g,
                                                            const float* __restrict__ c_prev, float* __restrict__ c_out,
                                                            float* __restrict__ h_out) {
  const int64_t total = rows * H;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int64_t r = t / H;
    const int j = (int)(t - r * H);
    float* gr = g + r * 4 * H + j;
    const float i = sigm(gr[0]), f = sigm(gr[H]), gg = tanhf(gr[2 * H]), o = sigm(gr[3 * H]);
    const float c = f * (c_prev ? c_prev[t] : 0.0f) + i * gg;
    gr[0] = i, gr[H] = f, gr[2 * H] = gg, gr[3 * H] = o;
    c_out[t] = c;
    h_out[t] = o * tanhf(c);
  }
}

// backward of one step: g = the activated gates, c = c', dh = dL/dh' (incl. the recurrent part), dc = dL/dc' from
// the next step (null: 0) -> dg (rows, 4H) pre-activation gradients, dc_prev = dL/dc (null: not wanted)
__global__ __launch_bounds__(256) void lstm_cell_bwd_kernel(int64_t rows, int H, const float* __restrict__ g,
                                                            const float* __restrict__ c_prev,
                                                            const float* __restrict__ c, const float* __restrict__ dh,
                                                            const float* __restrict__ dc, float* __restrict__ dg,
                                                            float* __restrict__ dc_prev) {
  const int64_t total = rows * H;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int64_t r = t / H;
    const int j = (int)(t - r * H);
    const float* gr = g + r * 4 * H + j;
    const float i = gr[0], f = gr[H], gg = gr[2 * H], o = gr[3 * H];
    const float tc = tanhf(c[t]);
    const float cp = c_prev ? c_prev[t] : 0.0f;
    const float dcc = dh[t] * o * (1.0f - tc * tc) + (dc ? dc[t] : 0.0f);
    float* dr = dg + r * 4 * H + j;
    dr[0] = dcc * gg * i * (1.0f - i);
    dr[H] = dcc * cp * f * (1.0f - f);
    dr[2 * H] = dcc * i * (1.0f - gg * gg);
    dr[3 * H] = dh[t] * tc * o * (1.0f - o);
    if (dc_prev) dc_prev[t] = dcc * f;
  }
}

}  // namespace dgppo

using namespace dgppo;

#define DG_STREAM(s) ((hipStream_t)(s))

extern "C" int dgppo_relu_bwd(float* dy, const float* y, int64_t n, void* stream) {
  if (n < 0 || !dy || !y) return DGPPO_EINVAL;
  if (n == 0) return 0;
  hipLaunchKernelGGL(relu_bwd_kernel, dim3(grid_for(n)), dim3(256), 0, DG_STREAM(stream), dy, y, n);
  return (int)hipGetLastError();
}

extern "C" int dgppo_lstm_cell_fwd(int64_t rows, int32_t H, float* g, const float* c_prev, float* c_out, float* h_out,
                                   void* stream) {
  if (rows < 0 || H < 1 || !g || !c_out || !h_out) return DGPPO_EINVAL;
  if (rows == 0) return 0;
  hipLaunchKernelGGL(lstm_cell_fwd_kernel, dim3(grid_for(rows * H)), dim3(256), 0, DG_STREAM(stream), rows, H, g,
                     c_prev, c_out, h_out);
  return (int)hipGetLastError();
}

extern "C" int dgppo_lstm_cell_bwd(int64_t rows, int32_t H, const float* g, const float* c_prev, const float* c,
                                   const float* dh, const float* dc, float* dg, float* dc_prev, void* stream) {
  if (rows < 0 || H < 1 || !g || !c || !dh || !dg) return DGPPO_EINVAL;
  if (rows == 0) return 0;
  hipLaunchKernelGGL(lstm_cell_bwd_kernel, dim3(grid_for(rows * H)), dim3(256), 0, DG_STREAM(stream), rows, H, g,
                     c_prev, c, dh, dc, dg, dc_prev);
  return (int)hipGetLastError();
}

extern "C" int dgppo_layernorm_fwd(const float* x, const float* scale, const float* bias, float* y, float* mean,
                                   float* rstd, int64_t rows, int32_t F, int32_t relu, float eps, void* stream) {
  if (rows < 0 || F < 1 || !x || !scale || !bias || !y || !mean || !rstd) return DGPPO_EINVAL;
  if (rows == 0) return 0;
  if (F == 64 && aligned16(x) && aligned16(y) && aligned16(scale) && aligned16(bias)) {
    const int64_t g = (rows + 15) / 16;
    hipLaunchKernelGGL(layernorm64_fwd_kernel, dim3((unsigned)(g < 4096 ? g : 4096)), dim3(256), 0, DG_STREAM(stream),
                       x, scale, bias, y, mean, rstd, rows, relu, eps);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(layernorm_fwd_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, DG_STREAM(stream), x,
                     scale, bias, y, mean, rstd, rows, F, relu, eps);
  return (int)hipGetLastError();
}

extern "C" int64_t dgppo_layernorm_bwd_workspace_floats(int64_t rows, int32_t F) {
  return (int64_t)row_split(rows, 64).nb * 2 * F;
}

// dscale / dbias are ACCUMULATED (+=) so one call serves a whole parameter-gradient buffer
extern "C" int dgppo_layernorm_bwd(const float* x, const float* y, const float* dy, const float* scale,
                                   const float* mean, const float* rstd, float* dx, float* dscale, float* dbias,
                                   int64_t rows, int32_t F, int32_t relu, float* workspace, void* stream) {
  if (rows < 0 || F < 1 || !x || !dy || !scale || !dx || !dscale || !dbias || !workspace || (relu && !y))
    return DGPPO_EINVAL;
  if (rows == 0) return 0;
  const RowSplit sp = row_split(rows, 64);
  if (F == 64 && aligned16(x) && aligned16(dy) && aligned16(dx) && aligned16(scale) && (!relu || aligned16(y))) {
    hipLaunchKernelGGL(layernorm64_bwd_kernel, dim3(sp.nb), dim3(256), 0, DG_STREAM(stream), x, y, dy, scale, mean,
                       rstd, dx, workspace, rows, relu, sp.rpb);
  } else {
  hipLaunchKernelGGL(layernorm_bwd_kernel, dim3(sp.nb), dim3(256), 8 * F * sizeof(float), DG_STREAM(stream), x, y,
                     dy, scale, mean, rstd, dx, workspace, rows, F, relu, (int)sp.rpb);
  }
  hipLaunchKernelGGL(colsum_final_kernel, dim3((F + 15) / 16), dim3(256), 0, DG_STREAM(stream), workspace, sp.nb, F,
                     (int64_t)2 * F, dscale, 1.0f, 1.0f);
  hipLaunchKernelGGL(colsum_final_kernel, dim3((F + 15) / 16), dim3(256), 0, DG_STREAM(stream), workspace + F, sp.nb,
                     F, (int64_t)2 * F, dbias, 1.0f, 1.0f);
  return (int)hipGetLastError();
}

extern "C" int64_t dgppo_colsum_workspace_floats(int64_t rows, int32_t cols) {
  return (int64_t)row_split(rows, 64).nb * cols;
}

// out = alpha * colsum(x) + beta * out, deterministic
extern "C" int dgppo_colsum(const float* x, int64_t rows, int32_t cols, int64_t ld, int32_t grp, int64_t gstride,
                            float* out, float alpha, float beta, float* workspace, void* stream) {
  if (rows < 0 || cols < 1 || !x || !out || !workspace) return DGPPO_EINVAL;
  if (rows > 0 && rows <= 2048 && grp <= 0) {  // few rows (per-workgroup partials): one fixed-order pass, no split
    hipLaunchKernelGGL(colsum_final_kernel, dim3((cols + 15) / 16), dim3(256), 0, DG_STREAM(stream), x, (int)rows, cols,
                       ld, out, alpha, beta);
    return (int)hipGetLastError();
  }
  const RowSplit sp = row_split(rows, 64);
  const int nb = rows > 0 ? sp.nb : 0;
  if (nb > 0)
    hipLaunchKernelGGL(colsum_partial_kernel, dim3(nb), dim3(256), 0, DG_STREAM(stream), x, rows, cols, ld, grp,
                       gstride, workspace, sp.rpb);
  hipLaunchKernelGGL(colsum_final_kernel, dim3((cols + 15) / 16), dim3(256), 0, DG_STREAM(stream), workspace, nb,
                     cols, (int64_t)cols, out, alpha, beta);
  return (int)hipGetLastError();
}

extern "C" int dgppo_gru_fwd(const float* gi, const float* gh, const float* bhn, const float* h, float* h_new,
                             int64_t rows, int32_t H, void* stream) {
  if (rows < 0 || H < 1 || !gi || !gh || !bhn || !h || !h_new) return DGPPO_EINVAL;
  if (rows == 0) return 0;
  hipLaunchKernelGGL(gru_fwd_kernel, dim3(grid_for(rows * H)), dim3(256), 0, DG_STREAM(stream), gi, gh, bhn, h,
                     h_new, rows, H);
  return (int)hipGetLastError();
}

extern "C" int dgppo_gru_bwd(const float* gi, const float* gh, const float* bhn, const float* h, const float* dh_new,
                             float* dgi, float* dgh, float* dh, int64_t rows, int32_t H, void* stream) {
  if (rows < 0 || H < 1 || !gi || !gh || !bhn || !h || !dh_new || !dgi || !dgh || !dh) return DGPPO_EINVAL;
  if (rows == 0) return 0;
  hipLaunchKernelGGL(gru_bwd_kernel, dim3(grid_for(rows * H)), dim3(256), 0, DG_STREAM(stream), gi, gh, bhn, h,
                     dh_new, dgi, dgh, dh, rows, H);
  return (int)hipGetLastError();
}

extern "C" int dgppo_agent_mean_fwd(const float* x, float* y, int64_t G, int32_t n, int32_t F, int64_t x_gstride,
                                    void* stream) {
  if (G < 0 || n < 1 || F < 1 || !x || !y) return DGPPO_EINVAL;
  if (G == 0) return 0;
  hipLaunchKernelGGL(agent_mean_fwd_kernel, dim3(grid_for(G * F)), dim3(256), 0, DG_STREAM(stream), x, y, G, n, F,
                     x_gstride);
  return (int)hipGetLastError();
}

extern "C" int dgppo_agent_mean_bwd_masked(const float* dy, const float* mask, float* dx, int64_t G, int32_t n,
                                           int32_t F, int64_t dx_gstride, void* stream) {
  if (G < 0 || n < 1 || F < 1 || !dx || !dy) return DGPPO_EINVAL;
  if (G == 0) return 0;
  hipLaunchKernelGGL(agent_mean_bwd_kernel, dim3(grid_for(G * n * F)), dim3(256), 0, DG_STREAM(stream), dy, dx, G,
                     n, F, dx_gstride, mask);
  return (int)hipGetLastError();
}

extern "C" int dgppo_agent_mean_bwd(const float* dy, float* dx, int64_t G, int32_t n, int32_t F, int64_t dx_gstride,
                                    void* stream) {
  return dgppo_agent_mean_bwd_masked(dy, nullptr, dx, G, n, F, dx_gstride, stream);
}

extern "C" int dgppo_tanh_normal(const dgppo_tanh_normal_args* p, void* stream) {
  if (!p || p->rows < 0 || p->A < 1 || !p->mean || !p->std_raw || p->mode < 0 || p->mode > 2) return DGPPO_EINVAL;
  if (p->mode == 1 && !p->noise) return DGPPO_EINVAL;
  if (p->mode == 2 && !p->action) return DGPPO_EINVAL;
  if (p->dmean && !p->dstd_raw) return DGPPO_EINVAL;
  if (p->entropy_eps && p->n_agents < 1) return DGPPO_EINVAL;
  if (p->rows == 0) return 0;
  hipLaunchKernelGGL(tanh_normal_kernel, dim3(grid_for(p->rows)), dim3(256), 0, DG_STREAM(stream), *p);
  return (int)hipGetLastError();
}

static const int kLossBlocks = 512;

extern "C" int64_t dgppo_loss_workspace_floats(void) { return (int64_t)kLossBlocks * 8; }

// stats out (4 floats): [mean max(l1,l2), mean entropy, clip_frac, total_variation_dist]
extern "C" int dgppo_ppo_loss(const float* log_pi, const float* log_pi_old, const float* adv, const float* entropy,
                              int64_t n, float clip_eps, float coef_ent, float* dlog_pi, float* dentropy, float* stats,
                              float* workspace, void* stream) {
  if (n < 1 || !log_pi || !log_pi_old || !adv || !entropy || !dlog_pi || !dentropy || !stats || !workspace)
    return DGPPO_EINVAL;
  hipLaunchKernelGGL(ppo_loss_kernel, dim3(kLossBlocks), dim3(256), 0, DG_STREAM(stream), log_pi, log_pi_old, adv,
                     entropy, n, clip_eps, coef_ent, dlog_pi, dentropy, workspace);
  hipLaunchKernelGGL(partial_reduce_kernel, dim3(1), dim3(64), 0, DG_STREAM(stream), workspace, kLossBlocks, 4,
                     stats, 1.0f / (float)n);
  return (int)hipGetLastError();
}

extern "C" int dgppo_l2_loss(const float* pred, const float* target, int64_t n, float* dpred, float* loss,
                             float* workspace, void* stream) {
  if (n < 1 || !pred || !target || !dpred || !loss || !workspace) return DGPPO_EINVAL;
  hipLaunchKernelGGL(l2_loss_kernel, dim3(kLossBlocks), dim3(256), 0, DG_STREAM(stream), pred, target, n, dpred,
                     workspace);
  hipLaunchKernelGGL(partial_reduce_kernel, dim3(1), dim3(64), 0, DG_STREAM(stream), workspace, kLossBlocks, 1, loss,
                     1.0f / (float)n);
  return (int)hipGetLastError();
}

extern "C" int dgppo_gae(const dgppo_gae_args* p, void* stream) {
  if (!p || p->B < 0 || p->T < 1 || p->T > 1024 || p->n_agents < 1 || p->n_h < 1 || !p->hs || !p->l || !p->Vh ||
      !p->Vl || !p->Qh || !p->Ql)
    return DGPPO_EINVAL;
  const int K = p->n_agents * p->n_h, T = p->T;
  if (K > 255) return DGPPO_EINVAL;
  // LDS staging of one env: hs, Vh, l, Vl and the two coefficient tables
  const size_t shmem = ((size_t)T * K + (size_t)(T + 1) * K + T + 3 * (size_t)(T + 1)) * sizeof(float);
  if (shmem > 160 * 1024) return DGPPO_EINVAL;
  if (p->B == 0) return 0;
  int Kp = 1;
  while (Kp < K + 1) Kp <<= 1;
  const int C = 256 / Kp < 64 ? 256 / Kp : 64;  // lanes per column (one wave holds a whole column)
  const int epl = (T + 1 + C - 1) / C;
  const dim3 grid((unsigned)p->B), block(256);
  const hipStream_t s = DG_STREAM(stream);
  if (shmem > 64 * 1024) {
    const void* fns[4] = {(const void*)gae_kernel<16>, (const void*)gae_kernel<32>, (const void*)gae_kernel<64>,
                          (const void*)gae_kernel<128>};
    for (const void* f : fns) allow_lds(f);
  }
  if (epl <= 16) hipLaunchKernelGGL(gae_kernel<16>, grid, block, shmem, s, *p, C);
  else if (epl <= 32) hipLaunchKernelGGL(gae_kernel<32>, grid, block, shmem, s, *p, C);
  else if (epl <= 64) hipLaunchKernelGGL(gae_kernel<64>, grid, block, shmem, s, *p, C);
  else if (epl <= 128) hipLaunchKernelGGL(gae_kernel<128>, grid, block, shmem, s, *p, C);
  else return DGPPO_EINVAL;
  return (int)hipGetLastError();
}

extern "C" int dgppo_dgppo_advantages(const dgppo_adv_args* p, void* stream) {
  if (!p || p->B < 0 || p->T < 1 || p->n_agents < 1 || p->n_h < 1 || !p->Ql || !p->Vl || !p->Vh || !p->A ||
      !p->safe_count)
    return DGPPO_EINVAL;
  if (p->B == 0) return 0;
  hipLaunchKernelGGL(dgppo_adv_kernel, dim3((unsigned)p->B), dim3(256), 0, DG_STREAM(stream), *p);
  return (int)hipGetLastError();
}

// ---- InforMARL (dgppo/algo/informarl.py:310-340): cost-shaped loss and normalised advantages --------
// l[b, t] = -r[b, t] + w * sum_a sum_h max(c[b, t, a, h], 0)   (sum over h first, then a)
__global__ __launch_bounds__(256) void shaped_loss_kernel(const float* __restrict__ r, const float* __restrict__ c,
                                                          float w, float* __restrict__ l, int64_t BT, int32_t n,
                                                          int32_t nh) {
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < BT; t += (int64_t)gridDim.x * 256) {
    const float* cr = c + t * n * nh;
    float sa = 0.0f;
    for (int a = 0; a < n; ++a) {
      float sh = 0.0f;
      for (int h = 0; h < nh; ++h) sh += fmaxf(cr[a * nh + h], 0.0f);
      sa += sh;
    }
    l[t] = -r[t] + w * sa;
  }
}

// one workgroup per env: Al = Ql - Vl[:T], A[t, a] = -(Al - mean_t Al) / (std_t Al + 1e-8) for every agent
// (jnp.std: population); fixed-order block reductions
__global__ __launch_bounds__(256) void informarl_adv_kernel(const float* __restrict__ Ql, const float* __restrict__ Vl,
                                                            float* __restrict__ A, int32_t T, int32_t n) {
  __shared__ float red[256];
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x;
  const float* q = Ql + b * T;
  const float* v = Vl + b * (T + 1);
  float s = 0.0f;
  for (int t = tid; t < T; t += 256) s += q[t] - v[t];
  red[tid] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) red[tid] += red[tid + o];
    __syncthreads();
  }
  const float mean = red[0] / (float)T;
  __syncthreads();
  float s2 = 0.0f;
  for (int t = tid; t < T; t += 256) {
    const float d = (q[t] - v[t]) - mean;
    s2 += d * d;
  }
  red[tid] = s2;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) red[tid] += red[tid + o];
    __syncthreads();
  }
  const float den = sqrtf(red[0] / (float)T) + 1e-8f;
  for (int e = tid; e < T * n; e += 256) {
    const int t = e / n;
    A[b * T * n + e] = -(((q[t] - v[t]) - mean) / den);
  }
}

extern "C" int dgppo_cost_shaped_loss(const float* rewards, const float* costs, float cost_weight, float* l, int32_t B,
                                      int32_t T, int32_t n_agents, int32_t n_h, void* stream) {
  if (B < 0 || T < 1 || n_agents < 1 || n_h < 1 || !rewards || !costs || !l) return DGPPO_EINVAL;
  const int64_t BT = (int64_t)B * T;
  if (BT == 0) return 0;
  hipLaunchKernelGGL(shaped_loss_kernel, dim3(grid_for(BT)), dim3(256), 0, DG_STREAM(stream), rewards, costs,
                     cost_weight, l, BT, n_agents, n_h);
  return (int)hipGetLastError();
}

extern "C" int dgppo_informarl_advantages(const float* Ql, const float* Vl, float* A, int32_t B, int32_t T,
                                          int32_t n_agents, void* stream) {
  if (B < 0 || T < 1 || n_agents < 1 || !Ql || !Vl || !A) return DGPPO_EINVAL;
  if (B == 0) return 0;
  hipLaunchKernelGGL(informarl_adv_kernel, dim3((unsigned)B), dim3(256), 0, DG_STREAM(stream), Ql, Vl, A, T, n_agents);
  return (int)hipGetLastError();
}

extern "C" int dgppo_grad_norm(const float* grad, int64_t n, float* state, float* workspace, void* stream) {
  if (n < 0 || !grad || !state || !workspace) return DGPPO_EINVAL;
  hipLaunchKernelGGL(sumsq_partial_kernel, dim3(kLossBlocks), dim3(256), 0, DG_STREAM(stream), grad, n, workspace);
  hipLaunchKernelGGL(norm_final_kernel, dim3(1), dim3(64), 0, DG_STREAM(stream), workspace, kLossBlocks, state);
  return (int)hipGetLastError();
}

extern "C" int dgppo_adam(float* param, const float* grad, float* m, float* v, int64_t n, float* state, float lr,
                          double b1, double b2, float eps, float max_norm, void* stream) {
  if (n < 0 || !param || !grad || !m || !v || !state) return DGPPO_EINVAL;
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n)), dim3(256), 0, DG_STREAM(stream), param, grad, m, v, n, state, lr,
                     (float)b1, (float)(1.0 - b1), (float)b2, (float)(1.0 - b2), eps, max_norm);
  hipLaunchKernelGGL(adam_count_kernel, dim3(1), dim3(64), 0, DG_STREAM(stream), state);
  return (int)hipGetLastError();
}

extern "C" int64_t dgppo_adam_multi_workspace_floats(void) {
  return (int64_t)DGPPO_ADAM_MAX_NETS * kAdamParts * 8 + DGPPO_ADAM_MAX_NETS;
}

extern "C" int dgppo_adam_multi(const dgppo_adam_multi_args* a, void* stream) {
  if (!a || a->n_nets < 1 || a->n_nets > DGPPO_ADAM_MAX_NETS || !a->workspace) return DGPPO_EINVAL;
  int64_t nmax = 0;
  for (int k = 0; k < a->n_nets; ++k) {
    const dgppo_adam_net& t = a->net[k];
    if (t.n < 0 || !t.param || !t.grad || !t.m || !t.v || !t.state) return DGPPO_EINVAL;
    nmax = t.n > nmax ? t.n : nmax;
  }
  static_assert(kAdamParts == kLossBlocks, "the per-net partials are dgppo_grad_norm's");
  AdamMultiDev d;
  d.a = *a;
  d.omb1 = (float)(1.0 - a->b1);  // (1 - b) formed in double and rounded once, as dgppo_adam
  d.omb2 = (float)(1.0 - a->b2);
  hipLaunchKernelGGL(sumsq_multi_kernel, dim3(kAdamParts, a->n_nets), dim3(256), 0, DG_STREAM(stream), d);
  hipLaunchKernelGGL(adam_multi_kernel, dim3(grid_for(nmax), a->n_nets), dim3(256), 0, DG_STREAM(stream), d);
  return (int)hipGetLastError();
}

extern "C" int dgppo_normal(float* out, int64_t n, const uint64_t* seed_ptr, uint64_t seed, uint64_t stream_id,
                            void* stream) {
  if (n < 0 || !out) return DGPPO_EINVAL;
  if (n == 0) return 0;
  hipLaunchKernelGGL(normal_kernel, dim3(grid_for(n)), dim3(256), 0, DG_STREAM(stream), out, n, seed_ptr, seed,
                     stream_id);
  return (int)hipGetLastError();
}

// ---- minibatch assembly: gather the (env, t) rows of the selected envs (DGPPO.update, dgppo.py:275-289) ---
// jtu.tree_map(lambda x: x[idx], rollout) of the reference's minibatch scan: for every field, output row
// o = e * T + t (e over the selected envs, t over the episode) is the source row of env envs[e] at step t,
// wherever the rollout keeps it (time-major buffers: t stride B * row, env stride row).  One wave per output
// row and field, 16-byte moves where a row allows it (rows of 4-byte elements).
namespace dgppo {
struct GatherFields {
  dgppo_gather_field f[8];
};
__global__ __launch_bounds__(256) void gather_env_steps_kernel(GatherFields fs, const int64_t* __restrict__ envs,
                                                             int32_t T, int64_t rows) {
  const dgppo_gather_field& f = fs.f[blockIdx.y];
  const int lane = threadIdx.x & 63;
  const int64_t o = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (o >= rows) return;
  const int64_t e = o / T, t = o - e * T;
  const float* src = reinterpret_cast<const float*>(f.src) + t * f.src_tstride + envs[e] * f.src_estride;
  float* dst = reinterpret_cast<float*>(f.dst) + o * f.row_elems;
  const int64_t L = f.row_elems;
  if ((L & 3) == 0 && ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0) {
    for (int64_t j = lane; j < L / 4; j += 64) reinterpret_cast<float4*>(dst)[j] = reinterpret_cast<const float4*>(src)[j];
  } else {
    for (int64_t j = lane; j < L; j += 64) dst[j] = src[j];
  }
}
}  // namespace dgppo

extern "C" int dgppo_gather_env_steps(const dgppo_gather_field* fields, int32_t n_fields, const int64_t* envs,
                                      int32_t n_sel, int32_t T, void* stream) {
  if (n_fields < 1 || n_fields > 8 || !fields || !envs || n_sel < 0 || T < 1) return DGPPO_EINVAL;
  const int64_t rows = (int64_t)n_sel * T;
  if (rows == 0) return 0;
  dgppo::GatherFields fs{};
  for (int i = 0; i < n_fields; ++i) {
    if (!fields[i].src || !fields[i].dst || fields[i].row_elems < 1) return DGPPO_EINVAL;
    fs.f[i] = fields[i];
  }
  hipLaunchKernelGGL(dgppo::gather_env_steps_kernel, dim3((unsigned)((rows + 3) / 4), (unsigned)n_fields), dim3(256),
                     0, DG_STREAM(stream), fs, envs, T, rows);
  return (int)hipGetLastError();
}

// ---- InforMARL-Lagr (dgppo/algo/informarl_lagr.py:125-309) ------------------------------------------------
namespace dgppo {
__device__ __forceinline__ float block_sum256(float v, float* red) {
  const int tid = threadIdx.x;
  red[tid] = v;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) red[tid] += red[tid + o];
    __syncthreads();
  }
  const float s = red[0];
  __syncthreads();
  return s;
}

__global__ void clip_min0_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float v = x[i];
    y[i] = v < 0.0f ? 0.0f : v;  // jnp.clip(costs, a_min=0): NaN passes through
  }
}

// one workgroup per env: Al = -(norm_t (Ql - Vl)), Ah = norm_t (Qh - Vh) per (agent, h) (population std + 1e-8),
// A[t, a] = Al[t] - mean_h (Ah[t, a, h] lagr[a, h])   (informarl_lagr.py:205-221)
__global__ __launch_bounds__(256) void lagr_adv_kernel(const float* __restrict__ Ql, const float* __restrict__ Vl,
                                                       const float* __restrict__ Qh, const float* __restrict__ Vh,
                                                       const float* __restrict__ lagr, float* __restrict__ A,
                                                       float* __restrict__ Ah, int32_t T, int32_t n, int32_t nh) {
  __shared__ float red[256];
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x;
  const float* q = Ql + b * T;
  const float* v = Vl + b * (T + 1);
  float s = 0.0f;
  for (int t = tid; t < T; t += 256) s += q[t] - v[t];
  const float mean = block_sum256(s, red) / (float)T;
  float s2 = 0.0f;
  for (int t = tid; t < T; t += 256) {
    const float d = (q[t] - v[t]) - mean;
    s2 += d * d;
  }
  const float den = sqrtf(block_sum256(s2, red) / (float)T) + 1e-8f;
  // constraint advantages: (agent, h) columns, each normalised over t; Vh row stride (T+1) n nh
  const float* qh = Qh + b * T * n * nh;
  const float* vh = Vh + b * (int64_t)(T + 1) * n * nh;
  float* ah = Ah + b * T * n * nh;
  for (int col = 0; col < n * nh; ++col) {
    float cs = 0.0f;
    for (int t = tid; t < T; t += 256) cs += qh[t * n * nh + col] - vh[t * n * nh + col];
    const float cm = block_sum256(cs, red) / (float)T;
    float cs2 = 0.0f;
    for (int t = tid; t < T; t += 256) {
      const float d = (qh[t * n * nh + col] - vh[t * n * nh + col]) - cm;
      cs2 += d * d;
    }
    const float cden = sqrtf(block_sum256(cs2, red) / (float)T) + 1e-8f;
    for (int t = tid; t < T; t += 256) ah[t * n * nh + col] = ((qh[t * n * nh + col] - vh[t * n * nh + col]) - cm) / cden;
  }
  __syncthreads();
  for (int e = tid; e < T * n; e += 256) {
    const int t = e / n, a = e - t * n;
    float m = 0.0f;
    for (int h = 0; h < nh; ++h) m += ah[(int64_t)t * n * nh + a * nh + h] * lagr[a * nh + h];
    A[b * T * n + e] = -(((q[t] - v[t]) - mean) / den) - m / (float)nh;
  }
}

// one workgroup per (agent, h): delta = -mean_{b,t} (Vh (1 - gamma) + ratio Ah), ratio = exp(log_pi - log_pi_old);
// lagr = relu(lagr - lr delta)   (update_lagr, informarl_lagr.py:283-305).  Fixed-order block reduction.
__global__ __launch_bounds__(256) void lagr_update_kernel(const float* __restrict__ lp, const float* __restrict__ lp_old,
                                                          const float* __restrict__ Vh, const float* __restrict__ Ah,
                                                          float* __restrict__ lagr, float* __restrict__ lagr_mean_out,
                                                          int64_t rows, int32_t n, int32_t nh, float gamma, float lr) {
  __shared__ float red[256];
  const int col = blockIdx.x, a = col / nh;
  float s = 0.0f;
  for (int64_t r = threadIdx.x; r < rows; r += 256) {
    const float ratio = expf(lp[r * n + a] - lp_old[r * n + a]);
    s += Vh[r * n * nh + col] * (1.0f - gamma) + ratio * Ah[r * n * nh + col];
  }
  const float delta = -(block_sum256(s, red) / (float)rows);
  if (threadIdx.x == 0) {
    const float l = lagr[col] - delta * lr;
    lagr[col] = l > 0.0f ? l : 0.0f;
  }
  (void)lagr_mean_out;
}

__global__ void mean_kernel(const float* __restrict__ x, int32_t n, float* __restrict__ out) {
  if (threadIdx.x == 0) {
    float s = 0.0f;
    for (int i = 0; i < n; ++i) s += x[i];
    out[0] = s / (float)n;
  }
}
}  // namespace dgppo

extern "C" int dgppo_clip_min0(const float* x, float* y, int64_t n, void* stream) {
  if (n < 0 || !x || !y) return DGPPO_EINVAL;
  if (n == 0) return 0;
  hipLaunchKernelGGL(dgppo::clip_min0_kernel, dim3(grid_for(n)), dim3(256), 0, DG_STREAM(stream), x, y, n);
  return (int)hipGetLastError();
}

extern "C" int dgppo_lagr_advantages(const float* Ql, const float* Vl, const float* Qh, const float* Vh,
                                     const float* lagr, float* A, float* Ah, int32_t B, int32_t T, int32_t n_agents,
                                     int32_t n_h, void* stream) {
  if (B < 0 || T < 1 || n_agents < 1 || n_h < 1 || !Ql || !Vl || !Qh || !Vh || !lagr || !A || !Ah) return DGPPO_EINVAL;
  if (B == 0) return 0;
  hipLaunchKernelGGL(dgppo::lagr_adv_kernel, dim3((unsigned)B), dim3(256), 0, DG_STREAM(stream), Ql, Vl, Qh, Vh, lagr,
                     A, Ah, T, n_agents, n_h);
  return (int)hipGetLastError();
}

extern "C" int dgppo_lagr_update(const float* log_pi, const float* log_pi_old, const float* Vh, const float* Ah,
                                 float* lagr, float* lagr_mean, int64_t rows, int32_t n_agents, int32_t n_h,
                                 float gamma, float lr, void* stream) {
  if (rows < 1 || n_agents < 1 || n_h < 1 || !log_pi || !log_pi_old || !Vh || !Ah || !lagr) return DGPPO_EINVAL;
  hipLaunchKernelGGL(dgppo::lagr_update_kernel, dim3((unsigned)(n_agents * n_h)), dim3(256), 0, DG_STREAM(stream),
                     log_pi, log_pi_old, Vh, Ah, lagr, lagr_mean, rows, n_agents, n_h, gamma, lr);
  if (lagr_mean)
    hipLaunchKernelGGL(dgppo::mean_kernel, dim3(1), dim3(64), 0, DG_STREAM(stream), lagr, n_agents * n_h, lagr_mean);
  return (int)hipGetLastError();
}
