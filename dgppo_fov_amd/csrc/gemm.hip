// Batched fp32 GEMM on gfx950 matrix cores (v_mfma_f32_32x32x2_f32: exact f32 FMA chains, 157 TF/s
// peak = the fp32 VALU peak, operands one VGPR per lane).
//
//   C[b] = alpha * op(A[b]) @ op(B[b]) + beta * C[b] + bias + addend[b]   (optional ReLU)
//   op(A) is (M, K): A row-major (M, K) with lda, or trans_a: A stored (K, M) with lda.
//   op(B) is (K, N): B row-major (K, N) with ldb, or trans_b: B stored (N, K) with ldb.
//
// Every dense layer of the DGPPO networks (flax Dense y = x W + b, its dX = dY W^T and
// dW = X^T dY, db = colsum dY) is one call.  The shapes are skinny (rows ~10^5..10^6, weights
// <= 192 x 192) and HBM-bound, so three kernels split the work by shape:
//
//  rows   (!trans_a, N <= 192, K <= 256): panel kernel.  The small weight op(B) is staged ONCE per
//         workgroup into LDS (k-major); each wave owns 32 rows x all N columns and streams its
//         rows' A values straight from HBM into MFMA operands (16-byte loads: the K index is
//         permuted so lane half h covers k in [h*Kh, (h+1)*Kh) contiguously).  Grid-stride over
//         128-row panels.
//  wgrad  (trans_a, !trans_b, M <= 128 per group, N <= 192): weight gradient X^T dY with the
//         reduction over ~10^5 rows.  Each workgroup takes a contiguous row chunk, its 8 waves
//         interleave row pairs and keep the WHOLE (M x N) partial in accumulators, so every
//         input byte is read once; the bias gradient colsum(dY) rides along on the VALU.
//         Wave partials combine in LDS in fixed order, chunk partials in a fixed-order reduce:
//         bitwise-deterministic gradients without float atomics.
//  tile   everything else: 64 x 64 LDS-tiled MFMA, optional split-K (the original kernel).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/dgppo_hip.h"
#include "lanes.h"
#include "lds_attr.h"

namespace dgppo {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kBM = 64, kBN = 64, kBK = 32, kPitch = kBM + 1;

// 64 zero bytes in global memory: out-of-range lanes of the streamed A loads read these instead of
// taking a branch or a select, so the prefetch stays a plain straight-line load
__device__ float4 g_zero_row[4];
__device__ float g_sink[64];  // target of the epilogue stores a lane must not make (kept branch-free)

struct GemmTileArgs {
  int M, N, K, k_begin, k_end;
  bool ta, tb;
  const float* A;
  int64_t lda;
  const float* B;
  int64_t ldb;
  int a_grp, b_grp;
  int64_t a_gstride, b_gstride;
};

// address of stored row r under optional two-level grouping
__device__ __forceinline__ int64_t row_off(int r, int64_t ld, int grp, int64_t gstride) {
  if (grp <= 0) return (int64_t)r * ld;
  const int q = r / grp;
  return (int64_t)q * gstride + (int64_t)(r - q * grp) * ld;
}

__device__ __forceinline__ float load_a(const GemmTileArgs& g, int m, int k) {
  if (m >= g.M || k >= g.k_end) return 0.0f;
  return g.ta ? g.A[row_off(k, g.lda, g.a_grp, g.a_gstride) + m] : g.A[row_off(m, g.lda, g.a_grp, g.a_gstride) + k];
}
__device__ __forceinline__ float load_b(const GemmTileArgs& g, int k, int n) {
  if (n >= g.N || k >= g.k_end) return 0.0f;
  return g.tb ? g.B[row_off(n, g.ldb, g.b_grp, g.b_gstride) + k] : g.B[row_off(k, g.ldb, g.b_grp, g.b_gstride) + n];
}

__device__ __forceinline__ int64_t row_off64(int64_t r, int64_t ld, int grp, int64_t gstride) {
  if (grp <= 0) return r * ld;
  const int64_t q = r / grp;
  return q * gstride + (r - q * grp) * ld;
}

// accumulate the (m0, n0) 64x64 tile over [k_begin, k_end) into acc (this wave's 32x32 block)
__device__ __forceinline__ void gemm_tile(const GemmTileArgs& g, int m0, int n0, float* As, float* Bs, f32x16& acc) {
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  for (int kt = g.k_begin; kt < g.k_end; kt += kBK) {
    // stage: 64 x 32 of A and 32 x 64 of B, 8 floats per thread each; the fast global index
    // follows the contiguous dimension of the stored layout (coalesced)
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int idx = tid + r * 256;  // 0 .. 2047
      int m, k;
      if (g.ta) { m = idx & 63; k = idx >> 6; }   // stored (K, M): m fastest
      else { k = idx & 31; m = idx >> 5; }        // stored (M, K): k fastest
      As[k * kPitch + m] = load_a(g, m0 + m, kt + k);
      int n, kb;
      if (g.tb) { kb = idx & 31; n = idx >> 5; }  // stored (N, K): k fastest
      else { n = idx & 63; kb = idx >> 6; }       // stored (K, N): n fastest
      Bs[kb * kPitch + n] = load_b(g, kt + kb, n0 + n);
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < kBK; kk += 2) {
      const int k = kk + (lane >> 5);
      const float a = As[k * kPitch + wm + (lane & 31)];
      const float b = Bs[k * kPitch + wn + (lane & 31)];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
    __syncthreads();
  }
}

// The one epilogue order of every GEMM path (tiled, split-K reduce, rows / pf / breg via epi_load + epi_store):
// v = (alpha acc + bias) + (beta C + addend), ReLU last -- the dispatch (shape, DGPPO_ROWS_* knobs) never changes
// the bits of a result.  cp / dp are the C and addend elements (dp null when the call has no addend).
__device__ __forceinline__ float epi_combine(const dgppo_gemm_args& p, float acc, float bias, const float* cp,
                                             const float* dp) {
#pragma clang fp contract(off)  // the same roundings on every path: one explicit fma, then plain mul / adds
  float v = __builtin_fmaf(p.alpha, acc, bias);
  if (p.beta != 0.0f || dp) {
    float x = p.beta != 0.0f ? p.beta * *cp : 0.0f;
    if (dp) x = p.beta != 0.0f ? x + *dp : *dp;
    v += x;
  }
  return p.relu ? (v > 0.0f ? v : 0.0f) : v;
}

__global__ __launch_bounds__(256) void gemm_kernel(dgppo_gemm_args p) {
  __shared__ float As[kBK * kPitch];
  __shared__ float Bs[kBK * kPitch];
  const int tiles_n = (p.N + kBN - 1) / kBN;
  const int m0 = (blockIdx.x / tiles_n) * kBM;
  const int n0 = (blockIdx.x % tiles_n) * kBN;
  const int split = blockIdx.y;
  const int b = blockIdx.z;
  const int kchunk = ((p.K + p.split_k - 1) / p.split_k + kBK - 1) / kBK * kBK;
  GemmTileArgs g;
  g.M = p.M;
  g.N = p.N;
  g.K = p.K;
  g.k_begin = split * kchunk;
  g.k_end = min(p.K, g.k_begin + kchunk);
  g.ta = p.trans_a;
  g.tb = p.trans_b;
  g.A = p.A + (int64_t)b * p.stride_a;
  g.lda = p.lda;
  g.B = p.B + (int64_t)b * p.stride_b;
  g.ldb = p.ldb;
  g.a_grp = p.a_grp;
  g.b_grp = p.b_grp;
  g.a_gstride = p.a_gstride;
  g.b_gstride = p.b_gstride;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
  gemm_tile(g, m0, n0, As, Bs, acc);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  const int col = n0 + wn + (lane & 31);
  if (p.split_k > 1) {  // raw partial into the workspace slab (split, batch, M, N)
    float* W = p.workspace + ((int64_t)split * p.batch + b) * (int64_t)p.M * p.N;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = m0 + wm + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (row < p.M && col < p.N) W[(int64_t)row * p.N + col] = acc[r];
    }
    return;
  }
  float* C = p.C + (int64_t)b * p.stride_c;
  const float* D = p.addend ? p.addend + (int64_t)b * p.stride_add : nullptr;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = m0 + wm + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    if (row < p.M && col < p.N) {
      float* cp = C + row_off(row, p.ldc, p.c_grp, p.c_gstride) + col;
      const float* dp = D ? D + row_off(row, p.ld_add, p.add_grp, p.add_gstride) + col : nullptr;
      *cp = epi_combine(p, acc[r], p.bias ? p.bias[col] : 0.0f, cp, dp);
    }
  }
}

// split-K reduce: fixed split order -> deterministic
__global__ __launch_bounds__(256) void gemm_splitk_reduce(dgppo_gemm_args p) {
  const int64_t MN = (int64_t)p.M * p.N;
  const int64_t total = MN * p.batch;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int b = (int)(i / MN);
    const int64_t e = i - (int64_t)b * MN;
    const int row = (int)(e / p.N), col = (int)(e - (int64_t)row * p.N);
    float s = 0.0f;
    for (int sp = 0; sp < p.split_k; ++sp) s += p.workspace[((int64_t)sp * p.batch + b) * MN + e];
    float* C = p.C + (int64_t)b * p.stride_c + row_off(row, p.ldc, p.c_grp, p.c_gstride) + col;
    const float* dp =
        p.addend ? p.addend + (int64_t)b * p.stride_add + row_off(row, p.ld_add, p.add_grp, p.add_gstride) + col : nullptr;
    *C = epi_combine(p, s, p.bias ? p.bias[col] : 0.0f, C, dp);
  }
}


// ================================================================================================
// rows: C = alpha * A op(B) + beta C + bias + addend (relu) for M large, N <= 192, K <= kRowsMaxK.
// op(B) (K x N, rows zero-padded to a multiple of 16) is staged once per workgroup in LDS.  The work
// unit is one WAVE's (32-row panel, group of NTW 32-column tiles); waves walk the units round-robin
// (u = 4 block + wave + k * 4 grid, column group fastest, so the waves of a workgroup share their A
// panel through L2) -- fine-grained units keep every SIMD busy to the end instead of leaving a
// partially filled last round of whole-panel workgroups.  A is read 32 contiguous bytes per lane:
// in k-chunk c (16 values) lane half h holds k = 16 c + 8 h .. +7, i.e. MFMA k-step q of the chunk
// is k = 16 c + 8 h + q in half h (B rows follow the same map), so both halves of a row read one
// 64-byte run.  Chunk c + 1 (or the next unit's chunk 0) is in flight while chunk c's MFMAs issue;
// the first chunk is requested before B is staged.
// ================================================================================================
constexpr int kRowsMaxK = 256;
constexpr int kRowsLdsFloats = 12800;  // 50 KB: K16 * (N + 1) must fit

// Epilogue operands of one 32-row unit (rows m0 + (r & 3) + 8 (r >> 2) + 4 h, columns col0 + 32 t + i): the
// bias and, when EXTRA, beta * C + addend, requested as straight-line loads BEFORE the next unit's A
// prefetch and consumed after the MFMAs.  A load issued after the prefetch (or guarded by a branch) makes its
// in-order vmcnt wait cover the whole prefetch -- one HBM round trip per epilogue element when guarded.
// EXTRA bit 0: addend, bit 1: beta * C (only the operands a call has are loaded)
//
// EPI (dgppo_gemm_args.epi, ABI 9) fuses the elementwise pass that follows the GEMM into its epilogue:
//   1 relu mask:  v = mask > 0 ? v : 0 (the ReLU backward of the layer whose output `mask` is; replaces relu_bwd)
//   2 LayerNorm(64) + ReLU forward (flax LayerNorm eps 1e-6, nn/mlp.py:20-30): h = the GEMM result is stored to ln_h,
//     y = relu(((h - mean) rstd) scale + bias) to C, the row mean / rstd to ln_mean / ln_rstd (a wave owns whole
//     64-wide rows: NTW = 2, one column group)
//   3 LayerNorm(64) + ReLU backward: the GEMM result is dy; h from ln_h and the row mean / rstd EPI 2 stored in
//     ln_mean / ln_rstd give the ReLU gate by the same instruction sequence as EPI 2 (bit-identical decisions;
//     no statistics are recomputed), dx goes to C and the workgroup's [dscale | dbias] column partials to ln_part
//     (dgppo_gemm_partial_rows rows; the host sums them)
constexpr int kEpiMask = 1, kEpiLnFwd = 2, kEpiLnBwd = 3;
template <int NTW, int EPI>
struct EpiX {
  float m[(EPI == dgppo::kEpiMask || EPI == dgppo::kEpiLnBwd) ? NTW : 1][16];  // mask rows (1) / pre-LN rows (3)
  float sc[NTW], bi[NTW];                                        // LayerNorm scale / bias at this lane's columns
  float mo, ro;  // EPI 3: the forward's mean / rstd of register row (lane & 15) of this lane's half-wave
};
template <int NTW>
struct EpiAcc {  // EPI 3: this lane's column partials of dscale / dbias over the rows it has stored
  float ds[NTW], db[NTW];
};

__device__ __forceinline__ float swz16(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, v), 0x401F));
}
// all-reduce over the 32 lanes of a half-wave (every lane gets the identical sum)
__device__ __forceinline__ float red32(float v) {
  v = lanes::sum16(v);
  return v + swz16(v);
}
// row statistics of 64 values (v0 at column i, v1 at column 32 + i of the half-wave's 32 lanes): EPI 2 and 3
// call this with the same bits, so the bwd recomputes the fwd's mean / rstd exactly
__device__ __forceinline__ void ln_stats(float v0, float v1, float& mean, float& rstd) {
#pragma clang fp contract(off)
  const float s1 = red32(v0 + v1);
  const float s2 = red32(v0 * v0 + v1 * v1);
  mean = s1 / 64.0f;
  float var = s2 / 64.0f - mean * mean;
  var = var > 0.0f ? var : 0.0f;
  rstd = 1.0f / sqrtf(var + 1e-6f);
}
__device__ __forceinline__ float ln_pre(float v, float mean, float rstd, float sc, float bi) {
#pragma clang fp contract(off)
  return ((v - mean) * rstd) * sc + bi;
}

template <int NTW, int EXTRA, int EPI>
__device__ __forceinline__ void epi_load(const dgppo_gemm_args& p, const float* C, const float* Dd, int m0, int col0,
                                         int i, int h, float (&bv)[NTW], float (&xv)[NTW][16], EpiX<NTW, EPI>& ex) {
#pragma clang fp contract(off)  // epi_combine's roundings
  if (EPI == dgppo::kEpiLnBwd) {  // lane i of a half-wave fetches register row (i & 15)'s statistics
    const int row = m0 + (i & 3) + 8 * ((i & 15) >> 2) + 4 * h;
    const bool ok = row < p.M;
    ex.mo = *(ok ? p.ln_mean + row : (const float*)g_zero_row);
    ex.ro = *(ok ? p.ln_rstd + row : (const float*)g_zero_row);
  }
#pragma unroll
  for (int t = 0; t < NTW; ++t) {
    const int col = col0 + 32 * t + i;
    const bool cok = col < p.N;
    bv[t] = (p.bias && cok) ? p.bias[col] : 0.0f;
    if (EPI == dgppo::kEpiLnFwd || EPI == dgppo::kEpiLnBwd) {
      ex.sc[t] = p.ln_scale[col];  // N == 64: every column is real
      ex.bi[t] = p.ln_bias[col];
    }
    if (EXTRA || EPI == dgppo::kEpiMask || EPI == dgppo::kEpiLnBwd) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const bool ok = cok && row < p.M;
        float x = 0.0f;
        if (EXTRA & 2) {
          const float* cs = ok ? C + row_off(row, p.ldc, p.c_grp, p.c_gstride) + col : (const float*)g_zero_row;
          x = p.beta * *cs;
        }
        if (EXTRA & 1) {  // beta C + addend, or the addend alone (epi_combine's operand order)
          const float* ds = ok ? Dd + row_off(row, p.ld_add, p.add_grp, p.add_gstride) + col : (const float*)g_zero_row;
          x = (EXTRA & 2) ? x + *ds : *ds;
        }
        if (EXTRA) xv[t][r] = x;
        if (EPI == dgppo::kEpiMask) {
          const float* ms = ok ? p.mask + row_off(row, p.ld_mask, p.c_grp, p.c_gstride) + col : (const float*)g_zero_row;
          ex.m[t][r] = *ms;
        }
        if (EPI == dgppo::kEpiLnBwd) ex.m[t][r] = *(ok ? p.ln_h + (int64_t)row * 64 + col : (const float*)g_zero_row);
      }
    }
  }
}

template <int NTW, int EXTRA, int EPI>
__device__ __forceinline__ void epi_store(const dgppo_gemm_args& p, float* C, const f32x16 (&acc)[NTW], int m0,
                                          int col0, int i, int h, const float (&bv)[NTW], const float (&xv)[NTW][16],
                                          const EpiX<NTW, EPI>& ex, EpiAcc<NTW>& ea) {
#pragma clang fp contract(off)  // epi_combine's roundings
  if constexpr (EPI == dgppo::kEpiLnFwd || EPI == dgppo::kEpiLnBwd) {
    static_assert(NTW == 2 && EXTRA == 0, "LayerNorm epilogues: whole 64-wide rows, no beta C / addend");
    float mo = 0.0f, ro = 0.0f;  // this lane's row statistic to store (lanes i < 16: register r = i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = m0 + (r & 3) + 8 * (r >> 2) + 4 * h;
      const bool rok = row < p.M;
      const int64_t off = row_off(row, p.ldc, p.c_grp, p.c_gstride);
      float* dst0 = rok ? C + off + i : (float*)g_sink;
      float* dst1 = rok ? C + off + 32 + i : (float*)g_sink;
      if constexpr (EPI == dgppo::kEpiLnFwd) {
        const float v0 = __builtin_fmaf(p.alpha, acc[0][r], bv[0]);
        const float v1 = __builtin_fmaf(p.alpha, acc[1][r], bv[1]);
        float mean, rstd;
        ln_stats(v0, v1, mean, rstd);
        float* h0 = rok ? p.ln_h + (int64_t)row * 64 + i : (float*)g_sink;
        float* h1 = rok ? p.ln_h + (int64_t)row * 64 + 32 + i : (float*)g_sink;
        *h0 = v0;
        *h1 = v1;
        const float y0 = ln_pre(v0, mean, rstd, ex.sc[0], ex.bi[0]);
        const float y1 = ln_pre(v1, mean, rstd, ex.sc[1], ex.bi[1]);
        *dst0 = y0 > 0.0f ? y0 : 0.0f;
        *dst1 = y1 > 0.0f ? y1 : 0.0f;
        mo = i == r ? mean : mo;
        ro = i == r ? rstd : ro;
      } else {
        const float hv0 = ex.m[0][r], hv1 = ex.m[1][r];
        const float mean = __shfl(ex.mo, r, 32), rstd = __shfl(ex.ro, r, 32);  // lane r of this half
        const float dy0 = rok ? __builtin_fmaf(p.alpha, acc[0][r], bv[0]) : 0.0f;
        const float dy1 = rok ? __builtin_fmaf(p.alpha, acc[1][r], bv[1]) : 0.0f;
        const float g0 = ln_pre(hv0, mean, rstd, ex.sc[0], ex.bi[0]) > 0.0f ? dy0 : 0.0f;
        const float g1 = ln_pre(hv1, mean, rstd, ex.sc[1], ex.bi[1]) > 0.0f ? dy1 : 0.0f;
        const float xh0 = (hv0 - mean) * rstd, xh1 = (hv1 - mean) * rstd;
        ea.ds[0] += g0 * xh0;
        ea.ds[1] += g1 * xh1;
        ea.db[0] += g0;
        ea.db[1] += g1;
        const float gx0 = g0 * ex.sc[0], gx1 = g1 * ex.sc[1];
        const float s1 = red32(gx0 + gx1) / 64.0f;
        const float s2 = red32(gx0 * xh0 + gx1 * xh1) / 64.0f;
        *dst0 = rstd * ((gx0 - s1) - xh0 * s2);
        *dst1 = rstd * ((gx1 - s1) - xh1 * s2);
      }
    }
    if constexpr (EPI == dgppo::kEpiLnFwd) {
      const int row = m0 + (i & 3) + 8 * ((i & 15) >> 2) + 4 * h;
      if (i < 16 && row < p.M) {
        p.ln_mean[row] = mo;
        p.ln_rstd[row] = ro;
      }
    }
    return;
  }
#pragma unroll
  for (int t = 0; t < NTW; ++t) {
    const int col = col0 + 32 * t + i;
    if (col >= p.N) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = m0 + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (row < p.M) {
        float v = __builtin_fmaf(p.alpha, acc[t][r], bv[t]);
        if (EXTRA) v += xv[t][r];
        if (p.relu) v = v > 0.0f ? v : 0.0f;
        if (EPI == dgppo::kEpiMask) v = ex.m[t][r] > 0.0f ? v : 0.0f;
        C[row_off(row, p.ldc, p.c_grp, p.c_gstride) + col] = v;
      }
    }
  }
}

// EPI 3 at kernel end: this workgroup's [dscale (64) | dbias (64)] partial row, halves then waves in fixed order
// (red: >= 4 x 128 floats of the B staging area, free after the unit loop)
template <int NTW, int EPI>
__device__ __forceinline__ void epi_finish(const dgppo_gemm_args& p, EpiAcc<NTW>& ea, float* red, int i, int h,
                                           int wave) {
  if constexpr (EPI == dgppo::kEpiLnBwd) {
#pragma unroll
    for (int t = 0; t < NTW; ++t) {
      ea.ds[t] += __shfl_xor(ea.ds[t], 32, 64);
      ea.db[t] += __shfl_xor(ea.db[t], 32, 64);
    }
    __syncthreads();  // every wave is done reading the staged B
    if (h == 0) {
#pragma unroll
      for (int t = 0; t < NTW; ++t) {
        red[wave * 128 + 32 * t + i] = ea.ds[t];
        red[wave * 128 + 64 + 32 * t + i] = ea.db[t];
      }
    }
    __syncthreads();
    if (threadIdx.x < 128) {
      const float v = ((red[threadIdx.x] + red[128 + threadIdx.x]) + red[256 + threadIdx.x]) + red[384 + threadIdx.x];
      p.ln_part[(int64_t)blockIdx.x * 128 + threadIdx.x] = v;
    }
  }
}

template <int NTW, bool VEC, int EXTRA, int EPI = 0>
__global__ __launch_bounds__(256) void gemm_rows_kernel(dgppo_gemm_args p, int ncg) {
  extern __shared__ __attribute__((aligned(16))) float Bs[];  // [K16][NP] k-major
  const int NC = 32 * NTW * ncg, NP = NC + 1;
  const int K = p.K, N = p.N, M = p.M;
  const int K16 = (K + 15) & ~15;
  const int b = blockIdx.z;
  const float* A = p.A + (int64_t)b * p.stride_a;
  const float* B = p.B + (int64_t)b * p.stride_b;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = lane & 31, h = lane >> 5;
  const int panels = (M + 31) / 32;
  const int64_t nunits = (int64_t)panels * ncg;
  const int64_t ustep = (int64_t)gridDim.x * 4;
  const int nch = K16 / 16;
  auto row_ptr = [&](int64_t uu, bool& rok) -> const float* {
    const int row = (int)(uu / ncg) * 32 + i;
    rok = uu < nunits && row < M;
    return A + (rok ? row_off(row, p.lda, p.a_grp, p.a_gstride) : 0) + 8 * h;
  };
  // branch-free loads: an out-of-range lane reads A's first element and zeroes it afterwards, so the
  // loads stay straight-line code and the compiler waits only for the chunk it consumes (a guarded load
  // becomes a branch, after which every use waits for ALL loads in flight, prefetch included)
  auto load8 = [&](const float* Ar, bool rok, int c, float (&a)[8]) {
    const int k0 = 16 * c + 8 * h;
    if (VEC) {  // K % 8 == 0 and 16-byte aligned rows: a lane's 8 values are all in or all out
      const bool ok = rok && k0 < K;
      const float* src = ok ? Ar + 16 * c : (const float*)g_zero_row;
      const float4 v0 = *(const float4*)src, v1 = *(const float4*)(src + 4);
      a[0] = v0.x; a[1] = v0.y; a[2] = v0.z; a[3] = v0.w;
      a[4] = v1.x; a[5] = v1.y; a[6] = v1.z; a[7] = v1.w;
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const bool ok = rok && k0 + q < K;
        a[q] = *(ok ? Ar + 16 * c + q : (const float*)g_zero_row);
      }
    }
  };
  int64_t u = (int64_t)blockIdx.x * 4 + wave;
  bool rok;
  const float* Ar = row_ptr(u, rok);
  float a0[8], a1[8];
  load8(Ar, rok, 0, a0);  // the first unit's first chunk is requested before B is staged
  {  // stage op(B): 16 independent loads in flight per thread before their stores.  Index split
     // e -> (major, minor) by a float reciprocal (exact: e < 2^16, divisor <= 256) -- an integer
     // division per element would cost more VALU time than the whole GEMM's MFMAs
    const int total = K16 * NC;
    const int dv = p.trans_b ? K16 : NC;  // minor extent
    const float inv = 1.0f / (float)dv;
    for (int e0 = threadIdx.x; e0 < total; e0 += 256 * 16) {
      float v[16];
#pragma unroll
      for (int uu = 0; uu < 16; ++uu) {
        const int e = e0 + uu * 256;
        const int mj = (int)(((float)e + 0.5f) * inv), mn = e - mj * dv;
        const int k = p.trans_b ? mn : mj, n = p.trans_b ? mj : mn;
        v[uu] = (e < total && k < K && n < N)
                    ? (p.trans_b ? B[row_off(n, p.ldb, p.b_grp, p.b_gstride) + k]
                                 : B[row_off(k, p.ldb, p.b_grp, p.b_gstride) + n])
                    : 0.0f;
      }
#pragma unroll
      for (int uu = 0; uu < 16; ++uu) {
        const int e = e0 + uu * 256;
        if (e < total) {
          const int mj = (int)(((float)e + 0.5f) * inv), mn = e - mj * dv;
          const int k = p.trans_b ? mn : mj, n = p.trans_b ? mj : mn;
          Bs[k * NP + n] = v[uu];
        }
      }
    }
  }
  __syncthreads();
  float* C = p.C + (int64_t)b * p.stride_c;
  const float* Dd = p.addend ? p.addend + (int64_t)b * p.stride_add : nullptr;
  EpiAcc<NTW> ea = {};
  for (; u < nunits; u += ustep) {
    const int panel = (int)(u / ncg), cg = (int)(u - (int64_t)panel * ncg);
    const int m0 = panel * 32;
    f32x16 acc[NTW];
#pragma unroll
    for (int t = 0; t < NTW; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][r] = 0.0f;
    const float* bcol = Bs + 8 * h * NP + cg * 32 * NTW + i;
    float bv[NTW], xv[NTW][16];
    EpiX<NTW, EPI> ex;
    epi_load<NTW, EXTRA, EPI>(p, C, Dd, m0, cg * NTW * 32, i, h, bv, xv, ex);
    bool rokn = false;
    const float* Arn = Ar;
    for (int c = 0; c < nch; ++c) {
      if (c + 1 < nch) {
        load8(Ar, rok, c + 1, a1);
      } else {
        Arn = row_ptr(u + ustep, rokn);
        load8(Arn, rokn, 0, a1);
      }
      __builtin_amdgcn_sched_barrier(0);  // the prefetch is issued here, not sunk to its use
      const float* brow = bcol + 16 * c * NP;
#pragma unroll
      for (int q = 0; q < 8; ++q)
#pragma unroll
        for (int t = 0; t < NTW; ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[q], brow[q * NP + 32 * t], acc[t], 0, 0, 0);
#pragma unroll
      for (int q = 0; q < 8; ++q) a0[q] = a1[q];
    }
    Ar = Arn;
    rok = rokn;
    // epilogue: lane holds column (cg NTW + t) 32 + i, rows (r&3) + 8 (r>>2) + 4 h of the panel
    epi_store<NTW, EXTRA, EPI>(p, C, acc, m0, cg * NTW * 32, i, h, bv, xv, ex, ea);
  }
  epi_finish<NTW, EPI>(p, ea, Bs, i, h, wave);
}

// ================================================================================================
// rows, whole-unit prefetch form (K <= 16 NCH <= 64, 16-byte A rows): the same unit walk and LDS-staged B as
// gemm_rows_kernel, but a wave requests ALL of a unit's A bytes at once (NCH chunks, 32 B x NCH per lane) and
// the next unit's while the current one's MFMAs and stores issue.  At the update's shapes (131072 rows,
// K = 64) a wave owns one or two units, so the chunk-at-a-time pipeline above serialised NCH HBM round trips
// per unit; here one round trip covers the unit and every wave's bytes are in flight together.
// ================================================================================================
template <int NTW, int NCH, int EXTRA, int EPI = 0>
__global__ __launch_bounds__(256) void gemm_rows_pf_kernel(dgppo_gemm_args p, int ncg) {
  extern __shared__ __attribute__((aligned(16))) float Bs[];  // [K16][NP] k-major
  const int NC = 32 * NTW * ncg, NP = NC + 1;
  constexpr int K16 = 16 * NCH;
  const int K = p.K, N = p.N, M = p.M;
  const int b = blockIdx.z;
  const float* A = p.A + (int64_t)b * p.stride_a;
  const float* B = p.B + (int64_t)b * p.stride_b;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = lane & 31, h = lane >> 5;
  const int panels = (M + 31) / 32;
  const int64_t nunits = (int64_t)panels * ncg;
  const int64_t ustep = (int64_t)gridDim.x * 4;
  auto row_ptr = [&](int64_t uu, bool& rok) -> const float* {
    const int row = (int)(uu / ncg) * 32 + i;
    rok = uu < nunits && row < M;
    return A + (rok ? row_off(row, p.lda, p.a_grp, p.a_gstride) : 0) + 8 * h;
  };
  auto load_unit = [&](const float* Ar, bool rok, float (&a)[NCH][8]) {  // branch-free, as gemm_rows_kernel
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const bool ok = rok && 16 * c + 8 * h < K;
      const float* src = ok ? Ar + 16 * c : (const float*)g_zero_row;
      const float4 v0 = *(const float4*)src, v1 = *(const float4*)(src + 4);
      a[c][0] = v0.x; a[c][1] = v0.y; a[c][2] = v0.z; a[c][3] = v0.w;
      a[c][4] = v1.x; a[c][5] = v1.y; a[c][6] = v1.z; a[c][7] = v1.w;
    }
  };
  int64_t u = (int64_t)blockIdx.x * 4 + wave;
  bool rok;
  const float* Ar = row_ptr(u, rok);
  float a0[NCH][8], a1[NCH][8];
  load_unit(Ar, rok, a0);  // the first unit is requested before B is staged
  {
    const int total = K16 * NC;
    const int dv = p.trans_b ? K16 : NC;
    const float inv = 1.0f / (float)dv;
    for (int e0 = threadIdx.x; e0 < total; e0 += 256 * 16) {
      float v[16];
#pragma unroll
      for (int uu = 0; uu < 16; ++uu) {
        const int e = e0 + uu * 256;
        const int mj = (int)(((float)e + 0.5f) * inv), mn = e - mj * dv;
        const int k = p.trans_b ? mn : mj, n = p.trans_b ? mj : mn;
        v[uu] = (e < total && k < K && n < N)
                    ? (p.trans_b ? B[row_off(n, p.ldb, p.b_grp, p.b_gstride) + k]
                                 : B[row_off(k, p.ldb, p.b_grp, p.b_gstride) + n])
                    : 0.0f;
      }
#pragma unroll
      for (int uu = 0; uu < 16; ++uu) {
        const int e = e0 + uu * 256;
        if (e < total) {
          const int mj = (int)(((float)e + 0.5f) * inv), mn = e - mj * dv;
          const int k = p.trans_b ? mn : mj, n = p.trans_b ? mj : mn;
          Bs[k * NP + n] = v[uu];
        }
      }
    }
  }
  __syncthreads();
  float* C = p.C + (int64_t)b * p.stride_c;
  const float* Dd = p.addend ? p.addend + (int64_t)b * p.stride_add : nullptr;
  EpiAcc<NTW> ea = {};
  for (; u < nunits; u += ustep) {
    const int panel = (int)(u / ncg), cg = (int)(u - (int64_t)panel * ncg);
    const int m0 = panel * 32;
    // this unit's epilogue operands are requested before the next unit's prefetch (epi_load)
    float bv[NTW], xv[NTW][16];
    EpiX<NTW, EPI> ex;
    epi_load<NTW, EXTRA, EPI>(p, C, Dd, m0, cg * NTW * 32, i, h, bv, xv, ex);
    bool rokn;
    const float* Arn = row_ptr(u + ustep, rokn);
    load_unit(Arn, rokn, a1);  // the next unit's bytes are in flight during this unit's MFMAs and stores
    __builtin_amdgcn_sched_barrier(0);
    f32x16 acc[NTW];
#pragma unroll
    for (int t = 0; t < NTW; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][r] = 0.0f;
    const float* bcol = Bs + 8 * h * NP + cg * 32 * NTW + i;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const float* brow = bcol + 16 * c * NP;
#pragma unroll
      for (int q = 0; q < 8; ++q)
#pragma unroll
        for (int t = 0; t < NTW; ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[c][q], brow[q * NP + 32 * t], acc[t], 0, 0, 0);
    }
    epi_store<NTW, EXTRA, EPI>(p, C, acc, m0, cg * NTW * 32, i, h, bv, xv, ex, ea);
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int q = 0; q < 8; ++q) a0[c][q] = a1[c][q];
    Ar = Arn;
    rok = rokn;
  }
  epi_finish<NTW, EPI>(p, ea, Bs, i, h, wave);
}

// ================================================================================================
// rows, B-in-registers form (N <= 64: one column group; K <= 16 NCH <= 64): op(B) is staged in LDS once
// per workgroup as above, then every lane copies ITS MFMA B operands (NCH x 8 x NTW values) into
// registers, so the main loop issues MFMAs fed by the streamed A chunks and registers only (no LDS
// read per MFMA).  Same unit walk, A chunk pipeline and epilogue as gemm_rows_kernel.
// ================================================================================================
template <int NTW, int NCH, int EXTRA, int EPI = 0>
__global__ __launch_bounds__(256) void gemm_rows_breg_kernel(dgppo_gemm_args p) {
  extern __shared__ __attribute__((aligned(16))) float Bs[];  // [K16][NP] k-major
  constexpr int NC = 32 * NTW, NP = NC + 1, K16 = 16 * NCH;
  const int K = p.K, N = p.N, M = p.M;
  const int b = blockIdx.z;
  const float* A = p.A + (int64_t)b * p.stride_a;
  const float* B = p.B + (int64_t)b * p.stride_b;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = lane & 31, h = lane >> 5;
  const int64_t nunits = (M + 31) / 32;
  const int64_t ustep = (int64_t)gridDim.x * 4;
  auto row_ptr = [&](int64_t uu, bool& rok) -> const float* {
    const int row = (int)uu * 32 + i;
    rok = uu < nunits && row < M;
    return A + (rok ? row_off(row, p.lda, p.a_grp, p.a_gstride) : 0) + 8 * h;
  };
  auto load8 = [&](const float* Ar, bool rok, int c, float (&a)[8]) {  // branch-free, as gemm_rows_kernel
    const bool ok = rok && 16 * c + 8 * h < K;  // K % 8 == 0: a lane's 8 values are all in or all out
    const float* src = ok ? Ar + 16 * c : (const float*)g_zero_row;
    const float4 v0 = *(const float4*)src, v1 = *(const float4*)(src + 4);
    a[0] = v0.x; a[1] = v0.y; a[2] = v0.z; a[3] = v0.w;
    a[4] = v1.x; a[5] = v1.y; a[6] = v1.z; a[7] = v1.w;
  };
  int64_t u = (int64_t)blockIdx.x * 4 + wave;
  bool rok;
  const float* Ar = row_ptr(u, rok);
  float a0[8], a1[8];
  load8(Ar, rok, 0, a0);
  {
    const int total = K16 * NC;
    const int dv = p.trans_b ? K16 : NC;
    const float inv = 1.0f / (float)dv;
    for (int e0 = threadIdx.x; e0 < total; e0 += 256 * 16) {
      float v[16];
#pragma unroll
      for (int uu = 0; uu < 16; ++uu) {
        const int e = e0 + uu * 256;
        const int mj = (int)(((float)e + 0.5f) * inv), mn = e - mj * dv;
        const int k = p.trans_b ? mn : mj, n = p.trans_b ? mj : mn;
        v[uu] = (e < total && k < K && n < N)
                    ? (p.trans_b ? B[row_off(n, p.ldb, p.b_grp, p.b_gstride) + k]
                                 : B[row_off(k, p.ldb, p.b_grp, p.b_gstride) + n])
                    : 0.0f;
      }
#pragma unroll
      for (int uu = 0; uu < 16; ++uu) {
        const int e = e0 + uu * 256;
        if (e < total) {
          const int mj = (int)(((float)e + 0.5f) * inv), mn = e - mj * dv;
          const int k = p.trans_b ? mn : mj, n = p.trans_b ? mj : mn;
          Bs[k * NP + n] = v[uu];
        }
      }
    }
  }
  __syncthreads();
  float bf[NCH][8][NTW];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int q = 0; q < 8; ++q)
#pragma unroll
      for (int t = 0; t < NTW; ++t) bf[c][q][t] = Bs[(16 * c + 8 * h + q) * NP + 32 * t + i];
  float* C = p.C + (int64_t)b * p.stride_c;
  const float* Dd = p.addend ? p.addend + (int64_t)b * p.stride_add : nullptr;
  EpiAcc<NTW> ea = {};
  for (; u < nunits; u += ustep) {
    const int m0 = (int)u * 32;
    float bv[NTW], xv[NTW][16];
    EpiX<NTW, EPI> ex;
    epi_load<NTW, EXTRA, EPI>(p, C, Dd, m0, 0, i, h, bv, xv, ex);
    f32x16 acc[NTW];
#pragma unroll
    for (int t = 0; t < NTW; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][r] = 0.0f;
    bool rokn = false;
    const float* Arn = Ar;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      if (c + 1 < NCH) {
        load8(Ar, rok, c + 1, a1);
      } else {
        Arn = row_ptr(u + ustep, rokn);
        load8(Arn, rokn, 0, a1);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int q = 0; q < 8; ++q)
#pragma unroll
        for (int t = 0; t < NTW; ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[q], bf[c][q][t], acc[t], 0, 0, 0);
#pragma unroll
      for (int q = 0; q < 8; ++q) a0[q] = a1[q];
    }
    Ar = Arn;
    rok = rokn;
    epi_store<NTW, EXTRA, EPI>(p, C, acc, m0, 0, i, h, bv, xv, ex, ea);
  }
  epi_finish<NTW, EPI>(p, ea, Bs, i, h, wave);
}

// ================================================================================================
// wgrad: C = alpha * A^T B + beta C over K rows (+ bias_grad = alpha * colsum(B) + beta bias_grad)
// ================================================================================================
constexpr int kWWaves = 8;
constexpr int kWMaxChunks = 256;
constexpr int kWMinRows = 512;

__host__ __device__ inline int wgrad_chunks(int64_t K, int min_rows = kWMinRows, int max_chunks = kWMaxChunks) {
  int64_t c = (K + min_rows - 1) / min_rows;
  if (c > max_chunks) c = max_chunks;
  return c < 1 ? 1 : (int)c;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t wg_rsrc(const float* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, bytes, 0x00020000);
}
__device__ __forceinline__ float wg_load(__amdgpu_buffer_rsrc_t r, int byte_off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, byte_off, 0, 0));
}

// workspace layout: [batch][chunk][M*N + N]; U row pairs of loads in flight per wave.  Every load is unconditional --
// the row clamped into the chunk, the column into the matrix, out-of-range values zeroed by a select -- so a row
// pair's loads issue back to back (guarded loads each sat behind a branch and a 64-bit row division, which made the
// loop issue-bound: SALU ~ VALU instructions, PMC); FLAT (no row grouping) addresses rows as k * ld, grouped rows
// with 32-bit arithmetic.
// one wgrad problem of a grouped launch (dgppo_gemm_wgrad_grouped): the dgppo_gemm_args fields the kernel reads
struct WgradEntry {
  const float* A;
  const float* B;
  float* C;
  float* bias_grad;
  float* workspace;
  int64_t lda, ldb, ldc, stride_a, stride_b, stride_c, a_gstride, b_gstride, c_gstride;
  int32_t a_grp, b_grp, c_grp, M, N, K, batch, chunks, ngroups_n;
  float alpha, beta;
};
constexpr int kWgradGroupMax = 12;
struct WgradGroup {
  int32_t n;
  int32_t wg_begin[kWgradGroupMax + 1];   // workgroups of the wgrad kernel per entry (prefix)
  int32_t red_begin[kWgradGroupMax + 1];  // 32-element blocks of the reduce kernel per entry (prefix)
  WgradEntry e[kWgradGroupMax];
};

// chunk c and tile group grp of workgroup L of one problem (G tile groups): the G tile groups of a chunk read the
// same rows (each its own columns), so they are dispatched back to back on ONE XCD (workgroups go round-robin over
// the 8 XCDs: linear id L runs on XCD L % 8) and the later groups' reads hit that XCD's L2 instead of HBM.  Needs
// chunks % 8 == 0 (the launcher rounds), else chunk-major order.
__device__ __forceinline__ void wgrad_place(int L, int chunks, int G, int& c, int& grp) {
  if ((chunks & 7) == 0) {
    const int j = L >> 3;
    c = 8 * (j / G) + (L & 7);
    grp = j - (j / G) * G;
  } else {
    c = L / G;
    grp = L - c * G;
  }
}

template <int MT, int NT, int U, bool FLAT, bool PIPE, class P>
__device__ __forceinline__ void wgrad_body(const P& p, int chunks, int ngroups_n, int c, int grp, int b, float* red) {
  constexpr int CP = NT * 32 + 1;
  const int gm = grp / ngroups_n, gn = grp % ngroups_n;
  const int m0 = gm * MT * 32, n0 = gn * NT * 32;
  const int M = p.M, N = p.N;
  const int64_t K = p.K;
  const int64_t rpc = (K + chunks - 1) / chunks;
  const int64_t r0 = (int64_t)c * rpc;
  const int64_t r1 = r0 + rpc < K ? r0 + rpc : K;
  const float* A = p.A + (int64_t)b * p.stride_a;
  const float* B = p.B + (int64_t)b * p.stride_b;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int i = lane & 31, h = lane >> 5;
  const bool do_bias = p.bias_grad != nullptr && gm == 0;
  f32x16 acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mt][nt][r] = 0.0f;
  float bs[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) bs[nt] = 0.0f;
  bool mok[MT], nok[NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) mok[mt] = m0 + mt * 32 + i < M;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) nok[nt] = n0 + nt * 32 + i < N;
  int mcol[MT], ncol[NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) mcol[mt] = mok[mt] ? m0 + mt * 32 + i : 0;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) ncol[nt] = nok[nt] ? n0 + nt * 32 + i : 0;
  // row pairs (2q, 2q+1) of the chunk, interleaved over the waves; lane half h takes row 2q + h.  A stage = U row
  // pairs: every load first (clamped, unconditional), then the selects and MFMAs (one wait for all of them)
  // FLAT: each row pair is read through a buffer resource based at its first row (wave-uniform, SGPRs) with the
  // lane's 32-bit offset (h * ld + column): no per-lane 64-bit addresses, and a row past the matrix end reads 0
  int offA[MT], offB[NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) offA[mt] = 4 * (h * p.lda + mcol[mt]);
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) offB[nt] = 4 * (h * p.ldb + ncol[nt]);
  auto issue = [&](float (&a)[U][MT], float (&bb)[U][NT], int64_t kb) {
    if constexpr (FLAT) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t k0 = kb + 2 * kWWaves * u;  // wave-uniform
        const int64_t ku = k0 < r1 ? k0 : r0;
        const int64_t left = K - ku;
        const int64_t ba = left * p.lda * 4, bbn = left * p.ldb * 4;
        const auto ra = wg_rsrc(A + ku * p.lda, ba < 0x7FFFFFFF ? (int)ba : 0x7FFFFFFF);
        const auto rb = wg_rsrc(B + ku * p.ldb, bbn < 0x7FFFFFFF ? (int)bbn : 0x7FFFFFFF);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) a[u][mt] = wg_load(ra, offA[mt]);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) bb[u][nt] = wg_load(rb, offB[nt]);
      }
      return;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t k = kb + 2 * kWWaves * u + h;
      const int64_t kc = k < r1 ? k : r0;
      // grouped rows: 32-bit row arithmetic (K < 2^31), one division per row instead of row_off64's 64-bit one
      const float* Ar = A + (FLAT ? kc * p.lda : row_off((int)kc, p.lda, p.a_grp, p.a_gstride));
      const float* Br = B + (FLAT ? kc * p.ldb : row_off((int)kc, p.ldb, p.b_grp, p.b_gstride));
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) a[u][mt] = Ar[mcol[mt]];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) bb[u][nt] = Br[ncol[nt]];
    }
  };
  auto consume = [&](float (&a)[U][MT], float (&bb)[U][NT], int64_t kb) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool kok = kb + 2 * kWWaves * u + h < r1;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) a[u][mt] = (kok && mok[mt]) ? a[u][mt] : 0.0f;
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) bb[u][nt] = (kok && nok[nt]) ? bb[u][nt] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u][mt], bb[u][nt], acc[mt][nt], 0, 0, 0);
      if (do_bias)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) bs[nt] += bb[u][nt];
    }
  };
  constexpr int64_t S = 2 * kWWaves * U;  // rows one stage advances
  if constexpr (PIPE) {
    // two register stages: the next stage's loads are in flight while this stage's MFMAs run (without it each
    // stage waited for its own loads: the kernel was load-latency-bound, ~30% MFMA busy on M64 N192).  Same row
    // order as the single-stage loop; a stage past the chunk end loads clamped rows and adds zeros.
    float a0[U][MT], b0[U][NT], a1[U][MT], b1[U][NT];
    int64_t kb = r0 + 2 * wave;
    if (kb < r1) issue(a0, b0, kb);
    for (; kb < r1; kb += 2 * S) {
      issue(a1, b1, kb + S);
      __builtin_amdgcn_sched_barrier(0);
      consume(a0, b0, kb);
      __builtin_amdgcn_sched_barrier(0);
      if (kb + S < r1) {
        issue(a0, b0, kb + 2 * S);
        __builtin_amdgcn_sched_barrier(0);
        consume(a1, b1, kb + S);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  } else {
    for (int64_t k0 = r0 + 2 * wave; k0 < r1; k0 += S) {
      float a[U][MT], bb[U][NT];
      issue(a, bb, k0);
      consume(a, bb, k0);
    }
  }
  // combine the 8 wave partials: a fixed pairwise tree over four LDS slabs ((w0 + w4) + (w2 + w6)) + ((w1 + w5) +
  // (w3 + w7)), 3 rounds instead of 8 serial read-modify-write rounds; the total lands in slab 0
  constexpr int SL = MT * 32 * CP;
  float* bred = red + 4 * SL;
  auto put = [&](float* dst) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int r = 0; r < 16; ++r) dst[(mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * CP + nt * 32 + i] = acc[mt][nt][r];
  };
  auto add = [&](const float* src) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[mt][nt][r] += src[(mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * CP + nt * 32 + i];
  };
  static_assert(kWWaves == 8, "tree over 8 waves");
  if (wave >= 4) put(red + (wave - 4) * SL);
  __syncthreads();
  if (wave < 4) add(red + wave * SL);
  __syncthreads();
  if (wave == 2 || wave == 3) put(red + (wave - 2) * SL);
  __syncthreads();
  if (wave < 2) add(red + wave * SL);
  __syncthreads();
  if (wave == 1) put(red + SL);
  __syncthreads();
  if (wave == 0) {
    add(red + SL);
    put(red);
  }
  if (do_bias) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) bred[(wave * 2 + h) * (NT * 32) + nt * 32 + i] = bs[nt];
  }
  __syncthreads();
  const int64_t slab = (int64_t)M * N + N;
  const bool direct = chunks == 1;
  float* W = p.workspace + ((int64_t)b * chunks + c) * slab;
  float* Cb = p.C + (int64_t)b * p.stride_c;
  for (int e = threadIdx.x; e < MT * 32 * NT * 32; e += 512) {
    const int row = e / (NT * 32), col = e % (NT * 32);
    const int m = m0 + row, n = n0 + col;
    if (m >= M || n >= N) continue;
    const float v = red[row * CP + col];
    if (direct) {
      float* cp = Cb + row_off(m, p.ldc, p.c_grp, p.c_gstride) + n;
      *cp = p.alpha * v + (p.beta != 0.0f ? p.beta * *cp : 0.0f);
    } else {
      W[(int64_t)m * N + n] = v;
    }
  }
  if (do_bias) {
    for (int col = threadIdx.x; col < NT * 32; col += 512) {
      const int n = n0 + col;
      if (n >= N) continue;
      float s = 0.0f;
      for (int q = 0; q < 2 * kWWaves; ++q) s += bred[q * (NT * 32) + col];
      if (direct) {
        float* bp = p.bias_grad + (int64_t)b * N + n;
        *bp = p.alpha * s + (p.beta != 0.0f ? p.beta * *bp : 0.0f);
      } else {
        W[(int64_t)M * N + n] = s;
      }
    }
  }
}

template <int MT, int NT, int U, bool FLAT, bool PIPE>
__global__ __launch_bounds__(512) void gemm_wgrad_kernel(dgppo_gemm_args p, int chunks, int ngroups_n) {
  extern __shared__ __attribute__((aligned(16))) float red[];  // 4 x [MT*32][NT*32 + 1] + colsum [2*kWWaves][NT*32]
  int c, grp;
  wgrad_place(blockIdx.x, chunks, gridDim.x / chunks, c, grp);
  wgrad_body<MT, NT, U, FLAT, PIPE>(p, chunks, ngroups_n, c, grp, blockIdx.z, red);
}

// several wgrad problems in ONE launch (a network pass's weight gradients, deferred to the end of its backward):
// workgroup -> (problem, batch entry, chunk, tile group) from the prefix table; per problem the same chunking,
// tile order and fixed-order sums as its own launch, so every output is bit-identical to gemm_wgrad_kernel's
template <int MT, int NT>
__global__ __launch_bounds__(512) void gemm_wgrad_grouped_kernel(WgradGroup g) {
  extern __shared__ __attribute__((aligned(16))) float red[];
  const int L = blockIdx.x;
  int k = 0;
  for (int q = 1; q < g.n; ++q) k = L >= g.wg_begin[q] ? q : k;
  const WgradEntry& p = g.e[k];
  const int G = ((p.M + MT * 32 - 1) / (MT * 32)) * p.ngroups_n;
  const int per_b = p.chunks * G;
  const int Lk = L - g.wg_begin[k];
  const int b = Lk / per_b;
  int c, grp;
  wgrad_place(Lk - b * per_b, p.chunks, G, c, grp);
  if (p.a_grp <= 0 && p.b_grp <= 0)
    wgrad_body<MT, NT, 4, true, true>(p, p.chunks, p.ngroups_n, c, grp, b, red);
  else
    wgrad_body<MT, NT, 4, false, true>(p, p.chunks, p.ngroups_n, c, grp, b, red);
}

// chunk partials -> C / bias_grad: 32 output elements per block, 8 chunk subsets each (coalesced
// over elements), combined in LDS in fixed order
template <class P>
__device__ __forceinline__ void wgrad_reduce_body(const P& p, int chunks, int64_t blk) {
  __shared__ float red[8][33];
  const int64_t MN = (int64_t)p.M * p.N;
  const int64_t slab = MN + p.N;
  const int64_t total = slab * p.batch;
  const int j = threadIdx.x >> 5;
  const int64_t t = blk * 32 + (threadIdx.x & 31);
  const int b = (int)(t / slab);
  const int64_t e = t - (int64_t)b * slab;
  const bool ok = t < total && (e < MN || p.bias_grad);
  float s = 0.0f;
  if (ok) {
    const float* W = p.workspace + (int64_t)b * chunks * slab + e;
#pragma unroll 8
    for (int q = j; q < chunks; q += 8) s += W[(int64_t)q * slab];
  }
  red[j][threadIdx.x & 31] = s;
  __syncthreads();
  if (j == 0 && ok) {
    const int l = threadIdx.x;
    const float v = ((red[0][l] + red[1][l]) + (red[2][l] + red[3][l])) + ((red[4][l] + red[5][l]) + (red[6][l] + red[7][l]));
    float* dst;
    if (e < MN) {
      const int row = (int)(e / p.N), col = (int)(e - (int64_t)row * p.N);
      dst = p.C + (int64_t)b * p.stride_c + row_off(row, p.ldc, p.c_grp, p.c_gstride) + col;
    } else {
      dst = p.bias_grad + (int64_t)b * p.N + (e - MN);
    }
    *dst = p.alpha * v + (p.beta != 0.0f ? p.beta * *dst : 0.0f);
  }
}

__global__ __launch_bounds__(256) void gemm_wgrad_reduce(dgppo_gemm_args p, int chunks) {
  wgrad_reduce_body(p, chunks, blockIdx.x);
}

__global__ __launch_bounds__(256) void gemm_wgrad_grouped_reduce(WgradGroup g) {
  const int L = blockIdx.x;
  int k = 0;
  for (int q = 1; q < g.n; ++q) k = L >= g.red_begin[q] ? q : k;
  if (g.e[k].chunks <= 1) return;
  wgrad_reduce_body(g.e[k], g.e[k].chunks, L - g.red_begin[k]);
}

}  // namespace dgppo

namespace {
enum GemmPath { kPathTile = 0, kPathRows = 1, kPathWgrad = 2 };

int env_knob(const char* name, int dflt) {
  const char* v = getenv(name);
  return v ? atoi(v) : dflt;
}
// wgrad launch shape (measured, scripts/gemm_knobs.sh): at most 4 accumulator tiles per wave (M64 x N192 over
// 131072 rows: 96 -> 67 us; more workgroups across N beat re-reading the row chunk once) and >= 128 rows per
// chunk (small-K weight gradients such as the GRU's dWh over 16384 rows: 88 -> 65 us)
int wgrad_min_rows() {
  static int v = env_knob("DGPPO_WGRAD_MINROWS", 128);
  return v;
}
int wgrad_max_acc() {
  static int v = env_knob("DGPPO_WGRAD_MAXACC", 4);
  return v;
}
// row chunks (workgroups along K; 256 = one 512-thread workgroup per CU) and row pairs in flight per wave (2 / 4)
int wgrad_max_chunks() {
  static int v = env_knob("DGPPO_WGRAD_MAXCHUNKS", 256);
  return v;
}
// two register stages in the wgrad loop (loads of the next U row pairs in flight under this stage's MFMAs);
// DGPPO_WGRAD_PIPE=0: the single-stage loop
int wgrad_pipe() {
  static int v = env_knob("DGPPO_WGRAD_PIPE", 1);
  return v;
}
int wgrad_unroll() {  // default 4 with the branch-free loads: M64 N192 66.9 -> 64.2 us, update 179.8 -> 178.6 ms
  static int v = env_knob("DGPPO_WGRAD_U", 4);
  return v == 8 ? 8 : (v == 4 ? 4 : 2);
}


GemmPath gemm_path(const dgppo_gemm_args* p) {
  if (p->trans_a && !p->trans_b && p->N <= 192 && p->M <= 4096 && !p->bias && !p->addend && !p->relu)
    return kPathWgrad;
  if (!p->trans_a && p->N <= 192 && p->K <= dgppo::kRowsMaxK) {
    int nt = (p->N + 31) / 32;
    if (nt == 5) nt = 6;
    if (((p->K + 15) & ~15) * (32 * nt + 1) <= dgppo::kRowsLdsFloats) return kPathRows;
  }
  return kPathTile;
}

// row chunks of a wgrad call: whole groups of 8 above 8 (the kernel's XCD-aware order; fewer chunks, more rows each)
int wgrad_chunk_count(int64_t K) {
  int chunks = dgppo::wgrad_chunks(K, wgrad_min_rows(), wgrad_max_chunks());
  return chunks > 8 ? (chunks & ~7) : chunks;
}

// (MT, NT) tile-group shape for the wgrad kernel: MT * NT <= 12 accumulators of 16 per lane
void wgrad_shape(int M, int N, int* MT, int* NT) {
  const int mt = (M + 31) / 32, nt = (N + 31) / 32;
  const int macc = wgrad_max_acc();
  *NT = nt >= 6 ? 6 : nt >= 3 ? 3 : nt;   // 1, 2, 3 or 6 (groups of 3/6 cover larger N)
  if (nt == 4 || nt == 5) *NT = 3;
  // one M tile and four N tiles (e.g. the Q-free projections' Gaug = x^T [dqt | dbeta], N = 99): one pass over
  // the rows instead of a 96-column group plus a 3-column group that re-reads the whole A panel
  static const int nt4 = env_knob("DGPPO_WGRAD_NT4", 1);
  if (nt == 4 && mt == 1 && nt4 && macc >= 4) {
    *NT = 4;
    *MT = 1;
    return;
  }
  while (*NT > 1 && *NT > macc) *NT = *NT == 6 ? 3 : (*NT == 3 ? 1 : *NT - 1);
  const int mmax = macc / *NT > 0 ? macc / *NT : 1;
  *MT = mt < mmax ? mt : mmax;
  if (*MT > 4) *MT = 4;
  if (*MT == 3 && *NT == 6) *MT = 2;
}

template <int MT, int NT>
void launch_wgrad_t(const dgppo_gemm_args* p, int chunks, hipStream_t s) {
  const int gm = (p->M + MT * 32 - 1) / (MT * 32), gn = (p->N + NT * 32 - 1) / (NT * 32);
  const size_t lds = ((size_t)4 * MT * 32 * (NT * 32 + 1) + 2 * dgppo::kWWaves * NT * 32) * sizeof(float);
  const dim3 grid(chunks * gm * gn, 1, p->batch);
  const bool flat = p->a_grp <= 0 && p->b_grp <= 0;
#define DG_WL(U, FL, PP)                                                                                       \
  do {                                                                                                         \
    if (lds > 64 * 1024) dgppo::allow_lds((const void*)dgppo::gemm_wgrad_kernel<MT, NT, U, FL, PP>);         \
    hipLaunchKernelGGL((dgppo::gemm_wgrad_kernel<MT, NT, U, FL, PP>), grid, dim3(512), lds, s, *p, chunks, gn); \
  } while (0)
  const bool pipe = wgrad_pipe();
  if (wgrad_unroll() == 8 && MT * NT <= 4 && flat && pipe) {
    DG_WL(8, true, true);
  } else if (wgrad_unroll() >= 4 && MT * NT <= 4) {
    if (pipe) {
      if (flat) DG_WL(4, true, true);
      else DG_WL(4, false, true);
    } else {
      if (flat) DG_WL(4, true, false);
      else DG_WL(4, false, false);
    }
  } else {
    if (pipe) {
      if (flat) DG_WL(2, true, true);
      else DG_WL(2, false, true);
    } else {
      if (flat) DG_WL(2, true, false);
      else DG_WL(2, false, false);
    }
  }
#undef DG_WL
}

int launch_wgrad(const dgppo_gemm_args* p0, hipStream_t s) {
  // a grouping whose group stride is grp rows is the plain row layout: drop it (the flat kernel's addressing)
  dgppo_gemm_args q = *p0;
  if (q.a_grp > 0 && q.a_gstride == (int64_t)q.a_grp * q.lda) q.a_grp = 0;
  if (q.b_grp > 0 && q.b_gstride == (int64_t)q.b_grp * q.ldb) q.b_grp = 0;
  const dgppo_gemm_args* p = &q;
  int MT, NT;
  wgrad_shape(p->M, p->N, &MT, &NT);
  const int chunks = wgrad_chunk_count(p->K);
  if (chunks > 1 && !p->workspace) return DGPPO_EINVAL;
#define DG_W(a, b) \
  if (MT == a && NT == b) { launch_wgrad_t<a, b>(p, chunks, s); goto launched; }
  DG_W(1, 1) DG_W(1, 2) DG_W(1, 3) DG_W(1, 4) DG_W(1, 6) DG_W(2, 1) DG_W(2, 2) DG_W(2, 3) DG_W(2, 6)
  DG_W(3, 1) DG_W(3, 2) DG_W(3, 3) DG_W(4, 1) DG_W(4, 2) DG_W(4, 3)
#undef DG_W
  return DGPPO_EINVAL;
launched:
  if (chunks > 1) {
    const int64_t total = ((int64_t)p->M * p->N + p->N) * p->batch;
    hipLaunchKernelGGL(dgppo::gemm_wgrad_reduce, dim3((unsigned)((total + 31) / 32)), dim3(256), 0, s, *p, chunks);
  }
  return 0;
}

// column-tile groups: NTW tiles per wave unit, ncg groups across N
void rows_split(int N, int* ntw, int* ncg) {
  const int nt = (N + 31) / 32;  // two tiles per unit keep the operands within 168 registers
  static const int wide = env_knob("DGPPO_ROWS_NTW", 0);  // experiment: tiles per unit for N > 64
  if (nt <= 2) { *ntw = nt; *ncg = 1; }
  else if (wide == 3 && nt % 3 == 0) { *ntw = 3; *ncg = nt / 3; }
  else if (wide == 6 && nt == 6) { *ntw = 6; *ncg = 1; }
  else if (nt == 3) { *ntw = 1; *ncg = 3; }
  else { *ntw = 2; *ncg = (nt + 1) / 2; }
}

// kernel choice, grid and dynamic LDS of a rows-path call (shared by the launch and dgppo_gemm_partial_rows)
struct RowsPlan {
  int ntw, ncg, K16, grid;
  size_t lds;
  bool vec, use_pf, use_breg;
};
RowsPlan rows_plan(const dgppo_gemm_args* p) {
  RowsPlan r;
  rows_split(p->N, &r.ntw, &r.ncg);
  r.K16 = (p->K + 15) & ~15;
  r.lds = (size_t)r.K16 * (32 * r.ntw * r.ncg + 1) * sizeof(float);
  const int64_t units = (int64_t)((p->M + 31) / 32) * r.ncg;
  int per_cu = (int)((160 * 1024) / (r.lds > 0 ? r.lds : 1));
  per_cu = per_cu < 1 ? 1 : per_cu > 5 ? 5 : per_cu;
  static int knob = -2;
  if (knob == -2) {
    const char* v = getenv("DGPPO_ROWS_WG_PER_CU");
    knob = v ? atoi(v) : -1;
  }
  r.vec = (p->K % 8 == 0) && (p->lda % 4 == 0) && (((uintptr_t)p->A & 15) == 0) &&
          (p->a_grp <= 0 || p->a_gstride % 4 == 0) && (p->stride_a % 4 == 0);
  // kernel choice and workgroups per CU, measured on the update's shapes (scripts/ab_gemm_pf.sh,
  // profiles/r03_gemm_rows_ab.txt, 131072 rows): the whole-unit prefetch form wins for K <= 32 and for N > 64
  // (N99 K32 35.7 -> 27.8 us, N64 K32 + addend 39.8 -> 22.4, N192 K32 52.4 -> 41.3, N192 K64 68.8 -> 63.9) at 3
  // workgroups per CU; the B-in-registers form stays best for N <= 64, K = 64 at 2 (28.0 -> 24.4-24.8 us)
  static const int pf = env_knob("DGPPO_ROWS_PF", 1);
  static const int breg = env_knob("DGPPO_ROWS_BREG", 1);
  r.use_pf = r.vec && pf && r.K16 <= 64 && (r.K16 <= 32 || r.ncg > 1 || !breg);
  r.use_breg = !r.use_pf && r.vec && breg && r.ncg == 1 && r.K16 <= 64;
  if (r.use_pf && per_cu > 3) per_cu = 3;
  if (r.use_breg && per_cu > 2) per_cu = 2;
  if (knob > 0 && knob < per_cu) per_cu = knob;
  const int64_t want = (units + 3) / 4, cap = 256LL * per_cu;
  r.grid = (int)(want < cap ? want : cap);
  if (r.grid < 1) r.grid = 1;
  return r;
}

// EPI != 0 instantiates only the combinations the epilogue supports (LayerNorm: NTW 2, no beta C / addend;
// relu mask: any NTW, beta C allowed, no addend)
template <int EPI, int NTW, int EXTRA>
constexpr bool epi_combo() {
  return EPI == 0 || (EPI == dgppo::kEpiMask && (EXTRA == 0 || EXTRA == 2)) || (NTW == 2 && EXTRA == 0);
}

template <int NTW, int EPI>
int launch_rows_t(const dgppo_gemm_args* p, const RowsPlan& r, hipStream_t s) {
  const int extra = (p->addend != nullptr ? 1 : 0) | (p->beta != 0.0f ? 2 : 0);
  const int ncg = r.ncg, grid = r.grid, K16 = r.K16;
  const size_t lds = r.lds;
  bool done = false;
  if (r.use_pf) {
#define DG_PF(c, x)                                                                                               \
  if constexpr (epi_combo<EPI, NTW, x>())                                                                         \
    if (!done && K16 == 16 * c && extra == x) {                                                                   \
      hipLaunchKernelGGL((dgppo::gemm_rows_pf_kernel<NTW, c, x, EPI>), dim3(grid, 1, p->batch), dim3(256), lds, s, \
                         *p, ncg);                                                                               \
      done = true;                                                                                                \
    }
    DG_PF(1, 0) DG_PF(1, 1) DG_PF(1, 2) DG_PF(1, 3) DG_PF(2, 0) DG_PF(2, 1) DG_PF(2, 2) DG_PF(2, 3)
    DG_PF(3, 0) DG_PF(3, 1) DG_PF(3, 2) DG_PF(3, 3) DG_PF(4, 0) DG_PF(4, 1) DG_PF(4, 2) DG_PF(4, 3)
#undef DG_PF
  } else if (r.use_breg) {
#define DG_RB(c, x)                                                                                                  \
  if constexpr (epi_combo<EPI, NTW, x>())                                                                            \
    if (!done && K16 == 16 * c && extra == x) {                                                                      \
      hipLaunchKernelGGL((dgppo::gemm_rows_breg_kernel<NTW, c, x, EPI>), dim3(grid, 1, p->batch), dim3(256), lds, s, \
                         *p);                                                                                        \
      done = true;                                                                                                   \
    }
    DG_RB(1, 0) DG_RB(1, 1) DG_RB(1, 2) DG_RB(1, 3) DG_RB(2, 0) DG_RB(2, 1) DG_RB(2, 2) DG_RB(2, 3)
    DG_RB(3, 0) DG_RB(3, 1) DG_RB(3, 2) DG_RB(3, 3) DG_RB(4, 0) DG_RB(4, 1) DG_RB(4, 2) DG_RB(4, 3)
#undef DG_RB
  } else {
#define DG_R(v, x)                                                                                                  \
  if constexpr (epi_combo<EPI, NTW, x>())                                                                           \
    if (!done && r.vec == v && extra == x) {                                                                        \
      hipLaunchKernelGGL((dgppo::gemm_rows_kernel<NTW, v, x, EPI>), dim3(grid, 1, p->batch), dim3(256), lds, s, *p, \
                         ncg);                                                                                      \
      done = true;                                                                                                  \
    }
    DG_R(true, 0) DG_R(true, 1) DG_R(true, 2) DG_R(true, 3) DG_R(false, 0) DG_R(false, 1) DG_R(false, 2)
    DG_R(false, 3)
#undef DG_R
  }
  return done ? 0 : DGPPO_EINVAL;
}

int launch_rows(const dgppo_gemm_args* p, hipStream_t s) {
  const RowsPlan r = rows_plan(p);
  switch (p->epi) {
    case 0:
      switch (r.ntw) {
        case 1: return launch_rows_t<1, 0>(p, r, s);
        case 2: return launch_rows_t<2, 0>(p, r, s);
        case 3: return launch_rows_t<3, 0>(p, r, s);
        case 6: return launch_rows_t<6, 0>(p, r, s);
      }
      return DGPPO_EINVAL;
    case dgppo::kEpiMask:
      if (!p->mask || p->addend || p->relu) return DGPPO_EINVAL;
      if (r.ntw == 1) return launch_rows_t<1, dgppo::kEpiMask>(p, r, s);
      if (r.ntw == 2) return launch_rows_t<2, dgppo::kEpiMask>(p, r, s);
      return DGPPO_EINVAL;
    case dgppo::kEpiLnFwd:
    case dgppo::kEpiLnBwd:
      if (p->N != 64 || r.ntw != 2 || r.ncg != 1 || p->batch != 1 || p->addend || p->beta != 0.0f || p->relu ||
          !p->ln_scale || !p->ln_bias || !p->ln_h || !p->ln_mean || !p->ln_rstd ||
          (p->epi == dgppo::kEpiLnBwd && !p->ln_part))
        return DGPPO_EINVAL;
      return p->epi == dgppo::kEpiLnFwd ? launch_rows_t<2, dgppo::kEpiLnFwd>(p, r, s) : launch_rows_t<2, dgppo::kEpiLnBwd>(p, r, s);
  }
  return DGPPO_EINVAL;
}
}  // namespace

extern "C" int64_t dgppo_gemm_partial_rows(const dgppo_gemm_args* p) {
  if (!p || p->M < 1 || p->N < 1 || gemm_path(p) != kPathRows) return 0;
  return rows_plan(p).grid;
}

extern "C" int64_t dgppo_gemm_workspace_floats(const dgppo_gemm_args* p) {
  if (!p) return 0;
  switch (gemm_path(p)) {
    case kPathWgrad: {
      const int chunks = wgrad_chunk_count(p->K);
      return chunks > 1 ? (int64_t)chunks * p->batch * ((int64_t)p->M * p->N + p->N) : 0;
    }
    case kPathRows:
      return 0;
    default:
      if (p->split_k <= 1) return 0;
      return (int64_t)p->split_k * p->batch * (int64_t)p->M * p->N;
  }
}

extern "C" int dgppo_gemm(const dgppo_gemm_args* p, void* stream) {
  if (!p || p->M < 0 || p->N < 0 || p->K < 0 || p->batch < 1 || p->split_k < 1 || p->split_k > 4096)
    return DGPPO_EINVAL;
  if (p->M == 0 || p->N == 0) return 0;
  if (!p->A || !p->B || !p->C) return DGPPO_EINVAL;
  if (p->bias_grad && gemm_path(p) != kPathWgrad) return DGPPO_EINVAL;
  if (p->epi && gemm_path(p) != kPathRows) return DGPPO_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const GemmPath path = gemm_path(p);
  if (path == kPathWgrad) {
    if (launch_wgrad(p, s)) return DGPPO_EINVAL;
    return (int)hipGetLastError();
  }
  if (path == kPathRows) {
    if (launch_rows(p, s)) return DGPPO_EINVAL;
    return (int)hipGetLastError();
  }
  if (p->split_k > 1 && !p->workspace) return DGPPO_EINVAL;
  const int tiles = ((p->M + dgppo::kBM - 1) / dgppo::kBM) * ((p->N + dgppo::kBN - 1) / dgppo::kBN);
  hipLaunchKernelGGL(dgppo::gemm_kernel, dim3(tiles, p->split_k, p->batch), dim3(256), 0, s, *p);
  if (p->split_k > 1) {
    const int64_t total = (int64_t)p->M * p->N * p->batch;
    const int64_t nb = (total + 255) / 256;
    const int blocks = (int)(nb < 4096 ? nb : 4096);
    hipLaunchKernelGGL(dgppo::gemm_splitk_reduce, dim3(blocks), dim3(256), 0, s, *p);
  }
  return (int)hipGetLastError();
}

// ---- grouped weight gradients (ABI 13) ---------------------------------------------------------------------------
namespace {
bool wgrad_grouped_ok(const dgppo_gemm_args* p) {
  return p->M >= 1 && p->N >= 1 && p->K >= 0 && p->batch >= 1 && p->A && p->B && p->C && p->trans_a && !p->trans_b &&
         gemm_path(p) == kPathWgrad && !p->epi;
}
int64_t wgrad_grouped_floats(const dgppo_gemm_args* p) {
  const int chunks = wgrad_chunk_count(p->K);
  return chunks > 1 ? (int64_t)chunks * p->batch * ((int64_t)p->M * p->N + p->N) : 0;
}
}  // namespace

extern "C" int64_t dgppo_gemm_wgrad_grouped_workspace_floats(const dgppo_gemm_args* args, int n) {
  if (!args || n < 0) return 0;
  int64_t t = 0;
  for (int k = 0; k < n; ++k) t += wgrad_grouped_floats(args + k);
  return t;
}

extern "C" int dgppo_gemm_wgrad_grouped(const dgppo_gemm_args* args, int n, float* workspace, void* stream) {
  if (!args || n < 0) return DGPPO_EINVAL;
  for (int k = 0; k < n; ++k)
    if (!wgrad_grouped_ok(args + k)) return DGPPO_EINVAL;
  if (dgppo_gemm_wgrad_grouped_workspace_floats(args, n) > 0 && !workspace) return DGPPO_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  constexpr int MT = 2, NT = 2;
  const size_t lds = ((size_t)4 * MT * 32 * (NT * 32 + 1) + 2 * dgppo::kWWaves * NT * 32) * sizeof(float);
  int64_t off = 0;
  for (int k0 = 0; k0 < n; k0 += dgppo::kWgradGroupMax) {
    dgppo::WgradGroup g{};
    g.n = n - k0 < dgppo::kWgradGroupMax ? n - k0 : dgppo::kWgradGroupMax;
    int64_t wg = 0, rb = 0;
    for (int q = 0; q < g.n; ++q) {
      const dgppo_gemm_args& a = args[k0 + q];
      dgppo::WgradEntry& e = g.e[q];
      e.A = a.A, e.B = a.B, e.C = a.C, e.bias_grad = a.bias_grad;
      e.lda = a.lda, e.ldb = a.ldb, e.ldc = a.ldc;
      e.stride_a = a.stride_a, e.stride_b = a.stride_b, e.stride_c = a.stride_c;
      // a grouping whose group stride is grp rows is the plain row layout (the flat kernel's addressing)
      e.a_grp = (a.a_grp > 0 && a.a_gstride == (int64_t)a.a_grp * a.lda) ? 0 : a.a_grp;
      e.b_grp = (a.b_grp > 0 && a.b_gstride == (int64_t)a.b_grp * a.ldb) ? 0 : a.b_grp;
      e.c_grp = a.c_grp;
      e.a_gstride = a.a_gstride, e.b_gstride = a.b_gstride, e.c_gstride = a.c_gstride;
      e.M = a.M, e.N = a.N, e.K = a.K, e.batch = a.batch;
      e.alpha = a.alpha, e.beta = a.beta;
      e.chunks = wgrad_chunk_count(a.K);
      e.ngroups_n = (a.N + NT * 32 - 1) / (NT * 32);
      const int G = ((a.M + MT * 32 - 1) / (MT * 32)) * e.ngroups_n;
      e.workspace = e.chunks > 1 ? workspace + off : nullptr;
      off += wgrad_grouped_floats(&a);
      g.wg_begin[q] = (int32_t)wg;
      g.red_begin[q] = (int32_t)rb;
      wg += (int64_t)a.batch * e.chunks * G;
      if (e.chunks > 1) rb += ((int64_t)a.batch * ((int64_t)a.M * a.N + a.N) + 31) / 32;
    }
    g.wg_begin[g.n] = (int32_t)wg;
    g.red_begin[g.n] = (int32_t)rb;
    if (wg > 0x7FFFFFFF || rb > 0x7FFFFFFF) return DGPPO_EINVAL;
    if (lds > 64 * 1024) dgppo::allow_lds((const void*)dgppo::gemm_wgrad_grouped_kernel<MT, NT>);
    hipLaunchKernelGGL((dgppo::gemm_wgrad_grouped_kernel<MT, NT>), dim3((unsigned)wg), dim3(512), lds, s, g);
    if (rb > 0) hipLaunchKernelGGL(dgppo::gemm_wgrad_grouped_reduce, dim3((unsigned)rb), dim3(256), 0, s, g);
  }
  return (int)hipGetLastError();
}
