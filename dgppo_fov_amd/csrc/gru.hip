// Whole-sequence GRU (flax.linen.GRUCell(64) scanned over the rnn_step chunk, dgppo/nn/rnn.py,
// informarl.py:281-293 / 387-403) as ONE launch per direction.
//
// The input projection gi = x Wi + bi of every step is one big GEMM outside (rows x 192); the
// recurrence h_t = GRU(gi_t, h_{t-1}) runs here: a 128-thread workgroup owns 32 sequence rows for
// all L steps, Wh (64 x 192) stays in LDS, h_{t-1} is the MFMA A operand from LDS and each wave
// computes the r / z / n gate tiles of ITS 32 hidden columns, so the gate math, the carry and the
// backward's dh recurrence stay in registers (lane = one hidden column, 16 rows).
//
// Backward (reverse steps): recompute gh = h_{t-1} Wh (h_{t-1} re-read from the forward's hs),
// gate derivatives, write dgi = [dr, dz, dn] and dgh = [dr, dz, dn*r] for the weight-gradient GEMMs
// done outside over all rows, and carry dh_{t-1} = dh_t z + dgh Wh^T (MFMA, K = 192).  The bhn
// gradient (column sum of dn*r) is reduced per workgroup in fixed order.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dgppo_hip.h"

namespace dgppo {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int kHid = 64, kG3 = 192, kRows = 32, kWP = 193, kHP = 65;

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

__device__ __forceinline__ int64_t seq_row(int q, int t, int L, int n) {
  return ((int64_t)(q / n) * L + t) * n + (q % n);
}

// gh tiles (r, z, n) of hidden block w for the 32 rows in A (pitch kHP)
__device__ __forceinline__ void gh_tiles(const float* A, const float* Whs, int col, int lane, f32x16& ar, f32x16& az,
                                         f32x16& an) {
  const int i = lane & 31, hh = lane >> 5;
#pragma unroll
  for (int r = 0; r < 16; ++r) ar[r] = az[r] = an[r] = 0.0f;
#pragma unroll 8
  for (int kk = 0; kk < kHid / 2; ++kk) {
    const int k = 2 * kk + hh;
    const float a = A[i * kHP + k];
    const float* w = Whs + k * kWP + col;
    ar = __builtin_amdgcn_mfma_f32_32x32x2f32(a, w[0], ar, 0, 0, 0);
    az = __builtin_amdgcn_mfma_f32_32x32x2f32(a, w[kHid], az, 0, 0, 0);
    an = __builtin_amdgcn_mfma_f32_32x32x2f32(a, w[2 * kHid], an, 0, 0, 0);
  }
}

__device__ __forceinline__ int tile_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

// Wh (64 x 192 row-major) -> LDS [k][kWP]: float4 loads, 8 in flight per thread
__device__ __forceinline__ void stage_wh(const float* Wh, float* Whs) {
  constexpr int n4 = kHid * kG3 / 4;
  if (((uintptr_t)Wh & 15) != 0) {  // unaligned view: scalar loads, 8 in flight
    for (int e0 = threadIdx.x; e0 < kHid * kG3; e0 += 128 * 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = e0 + u * 128 < kHid * kG3 ? Wh[e0 + u * 128] : 0.0f;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = e0 + u * 128;
        if (e < kHid * kG3) Whs[(e / kG3) * kWP + (e % kG3)] = v[u];
      }
    }
    return;
  }
  for (int e0 = threadIdx.x; e0 < n4; e0 += 128 * 8) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = e0 + u * 128;
      v[u] = e < n4 ? ((const float4*)Wh)[e] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = e0 + u * 128;
      if (e < n4) {
        const int k = (4 * e) / kG3, c = (4 * e) % kG3;
        float* d = Whs + k * kWP + c;
        d[0] = v[u].x, d[1] = v[u].y, d[2] = v[u].z, d[3] = v[u].w;
      }
    }
  }
}

__global__ __launch_bounds__(128) void gru_seq_fwd_kernel(dgppo_gru_seq_args p) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* Whs = lds;                   // [64][kWP]
  float* hb = Whs + kHid * kWP;       // [2][32][kHP]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int Q = p.Q, L = p.L, n = p.n_agents;
  const int nblk = (Q + kRows - 1) / kRows;
  stage_wh(p.Wh, Whs);
  const int col = w * 32 + (lane & 31);
  const float bn = p.bhn[col];
  for (int blk = blockIdx.x; blk < nblk; blk += gridDim.x) {  // persistent: Wh staged once
  const int q0 = blk * kRows;
  __syncthreads();
  for (int e = tid; e < kRows * kHid; e += 128) {
    const int r = e / kHid, k = e % kHid, q = q0 + r;
    hb[r * kHP + k] = (q < Q && p.h0) ? p.h0[(int64_t)q * kHid + k] : 0.0f;
  }
  __syncthreads();
  for (int t = 0; t < L; ++t) {
    const float* hcur = hb + (t & 1) * kRows * kHP;
    float* hnext = hb + ((t + 1) & 1) * kRows * kHP;
    f32x16 ar, az, an;
    gh_tiles(hcur, Whs, col, lane, ar, az, an);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = tile_row(r, lane), q = q0 + row;
      float hn = 0.0f;
      if (q < Q) {
        const int64_t gr = seq_row(q, t, L, n);
        const float* g = p.gi + gr * kG3;
        const float rg = sigm(g[col] + ar[r]);
        const float zg = sigm(g[kHid + col] + az[r]);
        const float ng = tanhf(g[2 * kHid + col] + rg * (an[r] + bn));
        hn = (1.0f - zg) * ng + zg * hcur[row * kHP + col];
        p.hs[gr * kHid + col] = hn;
        if (t == L - 1 && p.hT) p.hT[(int64_t)q * kHid + col] = hn;
      }
      hnext[row * kHP + col] = hn;
    }
    __syncthreads();
  }
  }
}

__global__ __launch_bounds__(128) void gru_seq_bwd_kernel(dgppo_gru_seq_args p) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* Whs = lds;                 // [64][kWP]
  float* hp = Whs + kHid * kWP;     // [32][kHP]   h_{t-1}
  float* dg = hp + kRows * kHP;     // [32][kWP]   dgh of this step
  float* red = dg + kRows * kWP;    // [2][64]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int i = lane & 31, hh = lane >> 5;
  const int Q = p.Q, L = p.L, n = p.n_agents;
  const int nblk = (Q + kRows - 1) / kRows;
  stage_wh(p.Wh, Whs);
  const int col = w * 32 + i;
  const float bn = p.bhn[col];
  float dbn = 0.0f;
  for (int blk = blockIdx.x; blk < nblk; blk += gridDim.x) {  // persistent: Wh staged once
  const int q0 = blk * kRows;
  float dh[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) dh[r] = 0.0f;
  for (int t = L - 1; t >= 0; --t) {
    __syncthreads();  // previous step's readers of hp / dg are done
    for (int e = tid; e < kRows * kHid; e += 128) {
      const int r = e / kHid, k = e % kHid, q = q0 + r;
      float v = 0.0f;
      if (q < Q) {
        if (t > 0) v = p.hs[seq_row(q, t - 1, L, n) * kHid + k];
        else if (p.h0) v = p.h0[(int64_t)q * kHid + k];
      }
      hp[r * kHP + k] = v;
    }
    __syncthreads();
    f32x16 ar, az, an;
    gh_tiles(hp, Whs, col, lane, ar, az, an);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = tile_row(r, lane), q = q0 + row;
      float drp = 0.0f, dzp = 0.0f, dnr = 0.0f;
      if (q < Q) {
        const int64_t gr = seq_row(q, t, L, n);
        const float* g = p.gi + gr * kG3;
        const float rg = sigm(g[col] + ar[r]);
        const float zg = sigm(g[kHid + col] + az[r]);
        const float ghn = an[r] + bn;
        const float ng = tanhf(g[2 * kHid + col] + rg * ghn);
        const float hprev = hp[row * kHP + col];
        const float d = p.dhs[gr * kHid + col] + dh[r];
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
    // dh_{t-1} += dgh (32 x 192) Wh^T (192 x 64): this wave's 32 hidden columns
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
#pragma unroll 8
    for (int kk = 0; kk < kG3 / 2; ++kk) {
      const int k = 2 * kk + hh;
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(dg[i * kWP + k], Whs[col * kWP + k], acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) dh[r] += acc[r];
  }
  if (p.dh0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int q = q0 + tile_row(r, lane);
      if (q < Q) p.dh0[(int64_t)q * kHid + col] = dh[r];
    }
  }
  }
  if (p.dbhn_part) {
    red[hh * kHid + col] = dbn;
    __syncthreads();
    if (tid < kHid) p.dbhn_part[(int64_t)blockIdx.x * kHid + tid] = red[tid] + red[kHid + tid];
  }
}

size_t fwd_lds() { return (size_t)(kHid * kWP + 2 * kRows * kHP) * sizeof(float); }
size_t bwd_lds() { return (size_t)(kHid * kWP + kRows * kHP + kRows * kWP + 2 * kHid) * sizeof(float); }

}  // namespace
}  // namespace dgppo

// persistent grid: at most 512 workgroups (2 per CU), each looping over 32-row blocks
extern "C" int64_t dgppo_gru_seq_blocks(int32_t Q) {
  const int64_t nb = (Q + dgppo::kRows - 1) / dgppo::kRows;
  return nb < 512 ? nb : 512;
}

extern "C" int dgppo_gru_seq_fwd(const dgppo_gru_seq_args* p, void* stream) {
  if (!p || p->Q < 0 || p->L < 1 || p->n_agents < 1 || p->H != dgppo::kHid || !p->gi || !p->Wh || !p->bhn || !p->hs ||
      (p->Q % p->n_agents) != 0)
    return DGPPO_EINVAL;
  if (p->Q == 0) return 0;
  static bool raised = false;
  if (!raised) {
    (void)hipFuncSetAttribute((const void*)dgppo::gru_seq_fwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    raised = true;
  }
  hipLaunchKernelGGL(dgppo::gru_seq_fwd_kernel, dim3((unsigned)dgppo_gru_seq_blocks(p->Q)), dim3(128),
                     dgppo::fwd_lds(), (hipStream_t)stream, *p);
  return (int)hipGetLastError();
}

extern "C" int dgppo_gru_seq_bwd(const dgppo_gru_seq_args* p, void* stream) {
  if (!p || p->Q < 0 || p->L < 1 || p->n_agents < 1 || p->H != dgppo::kHid || !p->gi || !p->Wh || !p->bhn || !p->hs ||
      !p->dhs || !p->dgi || !p->dgh || (p->Q % p->n_agents) != 0)
    return DGPPO_EINVAL;
  if (p->Q == 0) return 0;
  static bool raised = false;
  if (!raised) {
    (void)hipFuncSetAttribute((const void*)dgppo::gru_seq_bwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    raised = true;
  }
  hipLaunchKernelGGL(dgppo::gru_seq_bwd_kernel, dim3((unsigned)dgppo_gru_seq_blocks(p->Q)), dim3(128),
                     dgppo::bwd_lds(), (hipStream_t)stream, *p);
  return (int)hipGetLastError();
}
