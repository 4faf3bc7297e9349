// Batched fp32 GEMM on gfx950 matrix cores (v_mfma_f32_32x32x2_f32: exact f32 FMA chains in k
// order, 157 TF/s peak = the fp32 VALU peak, with operands one VGPR per lane).
//
//   C[b] = alpha * op(A[b]) @ op(B[b]) + beta * C[b] + bias + addend[b]   (optional ReLU)
//   op(A) is (M, K): A row-major (M, K) with lda, or trans_a: A stored (K, M) with lda.
//   op(B) is (K, N): B row-major (K, N) with ldb, or trans_b: B stored (N, K) with ldb.
//
// Every dense layer of the DGPPO networks (flax Dense y = x W + b, its dX = dY W^T and
// dW = X^T dY) is one call.  The weight-gradient shapes have a huge reduction dimension
// (K = rows of the minibatch, ~10^5) and tiny M, N: those run split-K into a workspace slab and a
// deterministic reduce kernel (no float atomics: bitwise-reproducible gradients).
//
// Tile: 64 x 64 per 256-thread workgroup, 4 waves in 2 x 2, each wave one 32 x 32 accumulator
// (16 fp32 per lane).  K advances 32 per LDS tile (16 MFMAs per wave per tile).  LDS images are
// k-major ([k][m] / [k][n], row pitch 65 floats) so the MFMA operand reads are lane-contiguous.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dgppo_hip.h"

namespace dgppo {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kBM = 64, kBN = 64, kBK = 32, kPitch = kBM + 1;

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
      float v = p.alpha * acc[r];
      if (p.beta != 0.0f) v += p.beta * *cp;
      if (p.bias) v += p.bias[col];
      if (D) v += D[row_off(row, p.ld_add, p.add_grp, p.add_gstride) + col];
      if (p.relu) v = v > 0.0f ? v : 0.0f;
      *cp = v;
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
    float v = p.alpha * s;
    if (p.beta != 0.0f) v += p.beta * *C;
    if (p.bias) v += p.bias[col];
    if (p.addend) v += p.addend[(int64_t)b * p.stride_add + row_off(row, p.ld_add, p.add_grp, p.add_gstride) + col];
    if (p.relu) v = v > 0.0f ? v : 0.0f;
    *C = v;
  }
}

}  // namespace dgppo

extern "C" int64_t dgppo_gemm_workspace_floats(const dgppo_gemm_args* p) {
  if (!p || p->split_k <= 1) return 0;
  return (int64_t)p->split_k * p->batch * (int64_t)p->M * p->N;
}

extern "C" int dgppo_gemm(const dgppo_gemm_args* p, void* stream) {
  if (!p || p->M < 0 || p->N < 0 || p->K < 0 || p->batch < 1 || p->split_k < 1 || p->split_k > 4096)
    return DGPPO_EINVAL;
  if (p->M == 0 || p->N == 0) return 0;
  if (!p->A || !p->B || !p->C) return DGPPO_EINVAL;
  if (p->split_k > 1 && !p->workspace) return DGPPO_EINVAL;
  hipStream_t s = (hipStream_t)stream;
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
