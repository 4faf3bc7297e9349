// Whole-sequence GRU (flax.linen.GRUCell(64) scanned over the rnn_step chunk, dgppo/nn/rnn.py,
// informarl.py:281-293 / 387-403) as ONE launch per direction.
//
// The input projection gi = x Wi + bi of every step is one big GEMM outside (rows x 192); the
// recurrence h_t = GRU(gi_t, h_{t-1}) runs here.  A 256-thread workgroup owns 16 sequence rows for
// all L steps (persistent over row blocks); Wh (64 x 192) stays in LDS; h_{t-1} is the MFMA A
// operand from LDS and wave w computes the r / z / n gate tiles (v_mfma_f32_16x16x4_f32) of ITS 16
// hidden columns, so the gate math, the carry and the backward's dh recurrence stay in registers
// (lane = one hidden column x 4 rows).  16-row blocks keep the serial step latency short (48 MFMAs
// of 32 cycles per wave per step) and give the short-sequence critics (Q = a few thousand) enough
// workgroups.
//
// Backward (reverse steps): recompute gh = h_{t-1} Wh (h_{t-1} re-read from the forward's hs),
// gate derivatives, write dgi = [dr, dz, dn] and dgh = [dr, dz, dn*r] for the weight-gradient GEMMs
// done outside over all rows, and carry dh_{t-1} = dh_t z + dgh Wh^T (MFMA, K = 192).  The bhn
// gradient (column sum of dn*r) is reduced per workgroup in fixed order.  Every global load of a
// step is issued before the step's stores (no load-after-store serialisation).
#include <hip/hip_runtime.h>

#include "lds_attr.h"
#include <stdint.h>
#include <stdlib.h>

#include "../../include/dgppo_hip.h"

namespace dgppo {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int kHid = 64, kG3 = 192, kRows = 16, kWP = 193, kHP = 65, kThreads = 256, kMaxBlocks = 1024;

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

// sink for the stores of padding rows (q >= Q): every store stays an unconditional straight-line
// instruction, so the compiler's wait counts stay exact (a guarded store or load is a branch, after
// which the next use waits for EVERY memory operation in flight)
__device__ float g_row_sink[kG3];
__device__ float4 g_zero_rows[16];  // a zero hidden row (64 floats) for padding rows / no initial carry

__device__ __forceinline__ int64_t seq_row(int q, int t, int L, int n) {
  return ((int64_t)(q / n) * L + t) * n + (q % n);
}

// lane l of wave w holds hidden column 16 w + (l & 15) for rows 4 (l >> 4) + r, r = 0..3
__device__ __forceinline__ int lane_row(int lane, int r) { return ((lane >> 4) << 2) + r; }

// gh tiles (r, z, n) of the wave's 16 hidden columns for the 16 rows of A (pitch kHP)
__device__ __forceinline__ void gh_tiles(const float* A, const float* Whs, int col, int lane, f32x4& ar, f32x4& az,
                                         f32x4& an) {
  const int i = lane & 15, kq = lane >> 4;
#pragma unroll
  for (int r = 0; r < 4; ++r) ar[r] = az[r] = an[r] = 0.0f;
#pragma unroll
  for (int kk = 0; kk < kHid / 4; ++kk) {
    const int k = 4 * kk + kq;
    const float a = A[i * kHP + k];
    const float* w = Whs + k * kWP + col;
    ar = __builtin_amdgcn_mfma_f32_16x16x4f32(a, w[0], ar, 0, 0, 0);
    az = __builtin_amdgcn_mfma_f32_16x16x4f32(a, w[kHid], az, 0, 0, 0);
    an = __builtin_amdgcn_mfma_f32_16x16x4f32(a, w[2 * kHid], an, 0, 0, 0);
  }
}

// Register form of the B operand (REGB): lane (i, kq) of wave w needs, for its 16 k-steps, exactly
// Wh[4 kk + kq][g 64 + 16 w + i] (g = r, z, n gate) -- 48 floats, loaded once per workgroup instead of
// staging Wh (48 KB) in LDS and reading one fragment from LDS per MFMA.  The same operands reach the
// same MFMAs in the same order, so results are bit-identical to the LDS form.
struct WhFrag {
  float v[3][kHid / 4];
};
__device__ __forceinline__ void wh_frag_load(const float* Wh, int col, int lane, WhFrag& f) {
  const int kq = lane >> 4;
#pragma unroll
  for (int kk = 0; kk < kHid / 4; ++kk) {
    const float* w = Wh + (int64_t)(4 * kk + kq) * kG3 + col;
    f.v[0][kk] = w[0];
    f.v[1][kk] = w[kHid];
    f.v[2][kk] = w[2 * kHid];
  }
}
__device__ __forceinline__ void gh_tiles_reg(const float* A, const WhFrag& f, int lane, f32x4& ar, f32x4& az,
                                             f32x4& an) {
  const int i = lane & 15, kq = lane >> 4;
#pragma unroll
  for (int r = 0; r < 4; ++r) ar[r] = az[r] = an[r] = 0.0f;
#pragma unroll
  for (int kk = 0; kk < kHid / 4; ++kk) {
    const float a = A[i * kHP + 4 * kk + kq];
    ar = __builtin_amdgcn_mfma_f32_16x16x4f32(a, f.v[0][kk], ar, 0, 0, 0);
    az = __builtin_amdgcn_mfma_f32_16x16x4f32(a, f.v[1][kk], az, 0, 0, 0);
    an = __builtin_amdgcn_mfma_f32_16x16x4f32(a, f.v[2][kk], an, 0, 0, 0);
  }
}

// Wh (64 x 192 row-major) -> LDS [k][kWP], all loads of a thread in flight before its stores
__device__ __forceinline__ void stage_wh(const float* Wh, float* Whs) {
  constexpr int n4 = kHid * kG3 / 4;  // 3072 float4 = 12 per thread
  if (((uintptr_t)Wh & 15) != 0) {    // unaligned view: scalar loads
    for (int e0 = threadIdx.x; e0 < kHid * kG3; e0 += kThreads * 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = e0 + u * kThreads < kHid * kG3 ? Wh[e0 + u * kThreads] : 0.0f;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = e0 + u * kThreads;
        if (e < kHid * kG3) Whs[(e / kG3) * kWP + (e % kG3)] = v[u];
      }
    }
    return;
  }
  float4 v[n4 / kThreads];
#pragma unroll
  for (int u = 0; u < n4 / kThreads; ++u) v[u] = ((const float4*)Wh)[threadIdx.x + u * kThreads];
#pragma unroll
  for (int u = 0; u < n4 / kThreads; ++u) {
    const int e = threadIdx.x + u * kThreads;
    const int k = (4 * e) / kG3, c = (4 * e) % kG3;
    float* d = Whs + k * kWP + c;
    d[0] = v[u].x, d[1] = v[u].y, d[2] = v[u].z, d[3] = v[u].w;
  }
}

// 16 rows x 64 (row r at src_row(r), or zero) -> LDS [16][kHP]: one float4 per thread
template <typename RowPtr>
__device__ __forceinline__ float4 load_rows16(RowPtr src_row) {
  const int e = threadIdx.x;  // 256 float4 = 16 rows x 16
  const float* r = src_row(e >> 4);
  return r ? ((const float4*)r)[e & 15] : make_float4(0.f, 0.f, 0.f, 0.f);
}
__device__ __forceinline__ void store_rows16(float* dst, float4 v) {
  const int e = threadIdx.x;
  float* d = dst + (e >> 4) * kHP + 4 * (e & 15);
  d[0] = v.x, d[1] = v.y, d[2] = v.z, d[3] = v.w;
}

template <bool REGB>
__global__ __launch_bounds__(kThreads) void gru_seq_fwd_kernel(dgppo_gru_seq_args p) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* Whs = lds;                                   // [64][kWP] (LDS form only)
  float* hb = REGB ? lds : Whs + kHid * kWP;          // [2][16][kHP]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int Q = p.Q, L = p.L, n = p.n_agents;
  const int nblk = (Q + kRows - 1) / kRows;
  const int col = w * 16 + (lane & 15);
  WhFrag wf;
  if constexpr (REGB) wh_frag_load(p.Wh, col, lane, wf);
  else stage_wh(p.Wh, Whs);
  const float bn = p.bhn[col];
  for (int blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    const int q0 = blk * kRows;
    const float4 h0v = load_rows16([&](int r) -> const float* {
      const int q = q0 + r;
      return (q < Q && p.h0) ? p.h0 + (int64_t)q * kHid : nullptr;
    });
    __syncthreads();  // previous block's readers of hb are done
    store_rows16(hb, h0v);
    __syncthreads();
    // gi of step t + 1 is loaded during step t (register double buffer); padding rows read row 0 and
    // store into the sink, so neither loads nor stores branch
    float gc[3][4], gx[3][4];
    auto load_gi = [&](int t, float (&g)[3][4]) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int q = q0 + lane_row(lane, r);
        const float* gp = p.gi + (q < Q ? seq_row(q, t, L, n) : 0) * kG3 + col;
        g[0][r] = gp[0];
        g[1][r] = gp[kHid];
        g[2][r] = gp[2 * kHid];
      }
    };
    load_gi(0, gc);
    for (int t = 0; t < L; ++t) {
      const float* hcur = hb + (t & 1) * kRows * kHP;
      float* hnext = hb + ((t + 1) & 1) * kRows * kHP;
      load_gi(t + 1 < L ? t + 1 : t, gx);
      __builtin_amdgcn_sched_barrier(0);
      f32x4 ar, az, an;
      if constexpr (REGB) gh_tiles_reg(hcur, wf, lane, ar, az, an);
      else gh_tiles(hcur, Whs, col, lane, ar, az, an);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = lane_row(lane, r), q = q0 + row;
        const bool ok = q < Q;
        const float rg = sigm(gc[0][r] + ar[r]);
        const float zg = sigm(gc[1][r] + az[r]);
        const float ng = tanhf(gc[2][r] + rg * (an[r] + bn));
        const float hn = ok ? (1.0f - zg) * ng + zg * hcur[row * kHP + col] : 0.0f;
        *(ok ? p.hs + seq_row(q, t, L, n) * kHid + col : g_row_sink + col) = hn;
        if (t == L - 1 && p.hT) *(ok ? p.hT + (int64_t)q * kHid + col : g_row_sink + col) = hn;
        hnext[row * kHP + col] = hn;
      }
#pragma unroll
      for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int r = 0; r < 4; ++r) gc[k][r] = gx[k][r];
      __syncthreads();
    }
  }
}

template <bool REGB>
__global__ __launch_bounds__(kThreads) void gru_seq_bwd_kernel(dgppo_gru_seq_args p) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* Whs = lds;                                 // [64][kWP] (LDS form only)
  float* hp = REGB ? lds : Whs + kHid * kWP;        // [16][kHP]   h_{t-1}
  float* dg = hp + kRows * kHP;     // [16][kWP]   dgh of this step
  float* red = dg + kRows * kWP;    // [4][64]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = lane & 15, kq = lane >> 4;
  const int Q = p.Q, L = p.L, n = p.n_agents;
  const int nblk = (Q + kRows - 1) / kRows;
  const int col = w * 16 + i;
  // REGB: the gh fragments and, for dh_{t-1} += dgh Wh^T, wt[kk] = Wh[col][4 kk + kq] (48 more floats)
  WhFrag wf;
  float wt[kG3 / 4];
  if constexpr (REGB) {
    wh_frag_load(p.Wh, col, lane, wf);
#pragma unroll
    for (int kk = 0; kk < kG3 / 4; ++kk) wt[kk] = p.Wh[(int64_t)col * kG3 + 4 * kk + kq];
  } else {
    stage_wh(p.Wh, Whs);
  }
  const float bn = p.bhn[col];
  float dbn = 0.0f;
  for (int blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    const int q0 = blk * kRows;
    float dh[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    // step t's loads (h_{t-1} rows, gi and upstream grads of the lane's 4 rows) are issued during step
    // t + 1 (register double buffer), branch-free: padding rows / the zero initial carry read the zero row
    float4 hv, hvx;
    float gc[4][4], gx[4][4];  // [r, z, n, dhs][row]
    auto load_step = [&](int t, float4& h, float (&g)[4][4]) {
      {
        const int q = q0 + (threadIdx.x >> 4);
        const float* hr = (const float*)g_zero_rows;
        if (q < Q) hr = t > 0 ? p.hs + seq_row(q, t - 1, L, n) * kHid : (p.h0 ? p.h0 + (int64_t)q * kHid : hr);
        h = ((const float4*)hr)[threadIdx.x & 15];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int q = q0 + lane_row(lane, r);
        const int64_t grow = q < Q ? seq_row(q, t, L, n) : 0;
        const float* gp = p.gi + grow * kG3 + col;
        g[0][r] = gp[0];
        g[1][r] = gp[kHid];
        g[2][r] = gp[2 * kHid];
        g[3][r] = p.dhs[grow * kHid + col];
      }
    };
    load_step(L - 1, hv, gc);
    for (int t = L - 1; t >= 0; --t) {
      load_step(t > 0 ? t - 1 : t, hvx, gx);
      __builtin_amdgcn_sched_barrier(0);
      float gr_[4], gz_[4], gn_[4], dd_[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool ok = q0 + lane_row(lane, r) < Q;
        gr_[r] = ok ? gc[0][r] : 0.0f;
        gz_[r] = ok ? gc[1][r] : 0.0f;
        gn_[r] = ok ? gc[2][r] : 0.0f;
        dd_[r] = ok ? gc[3][r] : 0.0f;
      }
      __syncthreads();  // previous step's readers of hp / dg are done
      store_rows16(hp, hv);
      __syncthreads();
      f32x4 ar, az, an;
      if constexpr (REGB) gh_tiles_reg(hp, wf, lane, ar, az, an);
      else gh_tiles(hp, Whs, col, lane, ar, az, an);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = lane_row(lane, r), q = q0 + row;
        float drp = 0.0f, dzp = 0.0f, dnr = 0.0f;
        if (q < Q) {
          const int64_t gr = seq_row(q, t, L, n);
          const float rg = sigm(gr_[r] + ar[r]);
          const float zg = sigm(gz_[r] + az[r]);
          const float ghn = an[r] + bn;
          const float ng = tanhf(gn_[r] + rg * ghn);
          const float hprev = hp[row * kHP + col];
          const float d = dd_[r] + dh[r];
          const float dn = d * (1.0f - zg);
          const float dz = d * (hprev - ng);
          const float dnp = dn * (1.0f - ng * ng);
          dzp = dz * zg * (1.0f - zg);
          drp = dnp * ghn * rg * (1.0f - rg);
          dnr = dnp * rg;
          float* dgi = p.dgi + gr * kG3;
          dgi[col] = drp;
          dgi[kHid + col] = dzp;
          dgi[2 * kHid + col] = dnp;
          float* dghr = p.dgh + gr * kG3;
          dghr[col] = drp;
          dghr[kHid + col] = dzp;
          dghr[2 * kHid + col] = dnr;
          dbn += dnr;
          dh[r] = d * zg;
        } else {
          dh[r] = 0.0f;
        }
        dg[row * kWP + col] = drp;
        dg[row * kWP + kHid + col] = dzp;
        dg[row * kWP + 2 * kHid + col] = dnr;
      }
      __syncthreads();
      // dh_{t-1} += dgh (16 x 192) Wh^T (192 x 64): this wave's 16 hidden columns
      f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
      if constexpr (REGB) {
#pragma unroll
        for (int kk = 0; kk < kG3 / 4; ++kk)
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(dg[i * kWP + 4 * kk + kq], wt[kk], acc, 0, 0, 0);
      } else {
#pragma unroll 8
        for (int kk = 0; kk < kG3 / 4; ++kk) {
          const int k = 4 * kk + kq;
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(dg[i * kWP + k], Whs[col * kWP + k], acc, 0, 0, 0);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) dh[r] += acc[r];
      hv = hvx;
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int r = 0; r < 4; ++r) gc[k][r] = gx[k][r];
    }
    if (p.dh0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int q = q0 + lane_row(lane, r);
        if (q < Q) p.dh0[(int64_t)q * kHid + col] = dh[r];
      }
    }
  }
  if (p.dbhn_part) {
    __syncthreads();
    red[kq * kHid + col] = dbn;
    __syncthreads();
    if (threadIdx.x < kHid) {
      const int c = threadIdx.x;
      p.dbhn_part[(int64_t)blockIdx.x * kHid + c] = (red[c] + red[kHid + c]) + (red[2 * kHid + c] + red[3 * kHid + c]);
    }
  }
}

size_t fwd_lds(bool regb) { return (size_t)((regb ? 0 : kHid * kWP) + 2 * kRows * kHP) * sizeof(float); }
size_t bwd_lds(bool regb) {
  return (size_t)((regb ? 0 : kHid * kWP) + kRows * kHP + kRows * kWP + 4 * kHid) * sizeof(float);
}
// B operand form (DGPPO_GRU_REGB=0 or dgppo_gru_set_form(0): Wh staged in LDS, the round-3 kernels; default:
// register fragments)
int g_regb = -1;
bool regb() {
  if (g_regb < 0) {
    const char* e = getenv("DGPPO_GRU_REGB");
    g_regb = (e && atoi(e) == 0) ? 0 : 1;
  }
  return g_regb == 1;
}

}  // namespace
}  // namespace dgppo

extern "C" int dgppo_gru_set_form(int32_t regb) {
  if (regb != 0 && regb != 1) return DGPPO_EINVAL;
  dgppo::g_regb = regb;
  return 0;
}

// persistent grid: at most kMaxBlocks workgroups, each looping over 16-row blocks
extern "C" int64_t dgppo_gru_seq_blocks(int32_t Q) {
  const int64_t nb = (Q + dgppo::kRows - 1) / dgppo::kRows;
  return nb < dgppo::kMaxBlocks ? nb : dgppo::kMaxBlocks;
}

extern "C" int dgppo_gru_seq_fwd(const dgppo_gru_seq_args* p, void* stream) {
  if (!p || p->Q < 0 || p->L < 1 || p->n_agents < 1 || p->H != dgppo::kHid || !p->gi || !p->Wh || !p->bhn || !p->hs ||
      (p->Q % p->n_agents) != 0)
    return DGPPO_EINVAL;
  if (p->Q == 0) return 0;
  const dim3 grid((unsigned)dgppo_gru_seq_blocks(p->Q));
  if (dgppo::regb()) {
    hipLaunchKernelGGL(dgppo::gru_seq_fwd_kernel<true>, grid, dim3(dgppo::kThreads), dgppo::fwd_lds(true),
                       (hipStream_t)stream, *p);
  } else {
    dgppo::allow_lds((const void*)dgppo::gru_seq_fwd_kernel<false>);
    hipLaunchKernelGGL(dgppo::gru_seq_fwd_kernel<false>, grid, dim3(dgppo::kThreads), dgppo::fwd_lds(false),
                       (hipStream_t)stream, *p);
  }
  return (int)hipGetLastError();
}

extern "C" int dgppo_gru_seq_bwd(const dgppo_gru_seq_args* p, void* stream) {
  if (!p || p->Q < 0 || p->L < 1 || p->n_agents < 1 || p->H != dgppo::kHid || !p->gi || !p->Wh || !p->bhn || !p->hs ||
      !p->dhs || !p->dgi || !p->dgh || (p->Q % p->n_agents) != 0)
    return DGPPO_EINVAL;
  if (p->Q == 0) return 0;
  const dim3 grid((unsigned)dgppo_gru_seq_blocks(p->Q));
  if (dgppo::regb()) {
    hipLaunchKernelGGL(dgppo::gru_seq_bwd_kernel<true>, grid, dim3(dgppo::kThreads), dgppo::bwd_lds(true),
                       (hipStream_t)stream, *p);
  } else {
    dgppo::allow_lds((const void*)dgppo::gru_seq_bwd_kernel<false>);
    hipLaunchKernelGGL(dgppo::gru_seq_bwd_kernel<false>, grid, dim3(dgppo::kThreads), dgppo::bwd_lds(false),
                       (hipStream_t)stream, *p);
  }
  return (int)hipGetLastError();
}
