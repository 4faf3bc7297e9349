// Graph-form MFMA attention (gm): the GraphTransformer attention core (dgppo/nn/gnn.py:83-117 + jraph
// segment_softmax / segment_sum) for graphs of N <= 96 nodes with n <= 10 receiving agents (every n = 8 Lidar
// env, MPE, LidarLine, LidarOmniTarget), one WAVE per graph, every dot product on the fp32 MFMA
// (v_mfma_f32_32x32x2_f32, exact f32 products).  Included by attn.hip inside dgppo::(anonymous).
//
// Per graph the sender rows S (N x D: agent rows, never-receivers' relu(x_raw W4 + b4) in agent mode, or the
// node rows themselves) are staged once in wave-private LDS; the receivers' query rows r = (h, i) (H * n <= 32)
// are the N dimension of every tile product, the graph's nodes (up to 3 tiles of 32) the M dimension:
//   logits^T (nodes x rows) = S . QT^T           K = D    (per node tile: D/2 MFMA steps)
//   softmax over each row's candidate nodes      lane-local: a lane holds one row's 16 x NT node values, the
//                                                other half-wave the rest (one xor-32 exchange)
//   xbar^T (d x rows)       = S^T . A^T          K = nodes, the attention weights straight from the logits'
//                                                accumulator registers (the K order is chosen to match the
//                                                accumulator layout, so no transpose)
// The candidate structure (which node is candidate c of receiver i, and its edge) comes from the sender table
// as an inverse map inv[i][node] = (c << 16) | edge; non-candidate nodes are masked out of the softmax.  The edge
// terms (ebar_h = sum_c a_hc ef_c, sig_h = sum_c a_hc) and the attention outputs use the same map.
//
// Backward: recompute S and the softmax (the same instruction sequence: the never-receivers' ReLU gates and the
// weights are bit-identical to the forward's), then
//   da^T  = S . dXbar^T (+ debar . ef + dsig + da_add on candidates);  dl = a (da - sum a da) / sqrt(F)
//   dqt^T = S^T . dl^T;  dbeta = sum dl
//   dS    = A^T dXbar + dL^T QT  (nodes x d; K = rows, a / dl transposed through LDS one node tile at a time)
//   agents: dxa += dS;  never-receivers (agent mode with pre): dz = dS (S > 0),
//   [W4; b4] gradient += [x_raw | 1]^T dz accumulated in registers over the wave's graphs (K = nodes).
// Writes of xcat / dqt rows go through LDS so each graph's rows are stored contiguously.  Deterministic (fixed
// order everywhere, no atomics); the pre gradient is one partial row per workgroup, summed by the host.
namespace gm {

constexpr int kMaxNT = 3;  // node tiles of 32: N <= 96
typedef float f32x16 __attribute__((ext_vector_type(16)));

__host__ __device__ inline int pitch(int DM) { return DM + 1; }
// wave-private LDS carve (floats): S [NP][DM+1] (aliased by X [32][33] after the sender-row products) | inv
// [n][NP] (int) | EF [E][4] | T [n][16] | (bwd) P [2][32][33] | RAW [NP][kD0 + 1]
struct Carve {
  int s, inv, ef, t, p, raw, total;
};
__host__ __device__ inline Carve carve(int DM, int NT, int n, int E, bool bwd, bool raw) {
  Carve c;
  const int NP = NT * 32;
  const int sz = NP * pitch(DM) > 32 * 33 ? NP * pitch(DM) : 32 * 33;
  c.s = 0;
  c.inv = (sz + 3) & ~3;
  c.ef = c.inv + ((n * NP + 3) & ~3);
  c.t = c.ef + E * 4;
  c.p = c.t + n * 16;
  c.raw = c.p + (bwd ? 2 * 32 * 33 : 32 * 33);
  c.total = c.raw + (bwd && raw ? NP * (kD0 + 1) : 0);
  c.total = ((c.total + 3) & ~3) + 4;  // + a sink for stores a lane must not make (kept branch-free)
  return c;
}

// node of accumulator register j of node tile t in half-wave hf (the 32x32x2 C layout: row (j/4)*8 + hf*4 + j%4)
__device__ __forceinline__ int node_of(int t, int j, int hf) { return t * 32 + (j & 3) + 8 * (j >> 2) + 4 * hf; }

__device__ __forceinline__ float xor32(float v) { return __shfl_xor(v, 32, 64); }

// ---- per-graph staging shared by forward and backward --------------------------------------------------------
// S rows (agents / transformed never-receivers / node rows), the inverse candidate map and the edge head rows.
// Agent mode with pre: S[node >= n] = relu(x_raw W4 + b4) as one MFMA product per node tile (K = 8).
template <int DM, int NT>
__device__ __forceinline__ void stage(const dgppo_gnn_attn_args& p, int64_t g, float* S, int* inv, float* EF,
                                      float* RAW, const float (&w4)[4], float b4, bool agent, bool pre, float* Ac,
                                      float* sink) {
  constexpr int SP = DM + 1;
  constexpr int NP = NT * 32;
  const int l = threadIdx.x & 63, col = l & 31, hf = l >> 5;
  const int n = p.n_agents, D = p.D, N = p.N, C = p.C, E = p.E;
  // node rows read directly (full mode: every node; agent mode: the agents from xa; agent mode without pre: the
  // never-receivers' raw rows, D0 == D)
  for (int e = l; e < NP * DM; e += 64) {
    const int node = e / DM, d = e - node * DM;
    float v = 0.0f;
    if (node < N && d < D) {
      if (!agent) v = p.x[g * p.x_gstride + (int64_t)node * D + d];
      else if (node < n) v = p.xa[g * p.xa_gstride + (int64_t)node * D + d];
      else if (!pre) v = p.x[g * p.x_gstride + (int64_t)node * p.D0 + d];
    }
    if (!pre || node < n || node >= N) S[node * SP + d] = v;
  }
  if (pre) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int node = t * 32 + col;
      const bool nv = node >= n && node < N;
      f32x16 acc = {};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int k = hf * 4 + s;
        const int nc = node < N ? node : N - 1, kc = k < p.D0 ? k : p.D0 - 1;
        const float x = p.x[g * p.x_gstride + (int64_t)nc * p.D0 + kc];  // unconditional (branch-free)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32((nv && k < p.D0) ? x : 0.0f, w4[s], acc, 0, 0, 0);
      }
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int nd = node_of(t, j, hf);
        const float z = acc[j] + b4;
        float* dst = (nd >= n && nd < N && col < DM) ? S + nd * SP + col : sink;
        *dst = (col < D && z > 0.0f) ? z : 0.0f;
      }
    }
    if (RAW) {  // [x_raw | 1] rows of the never-receivers for the pre-layer gradient
      for (int e = l; e < NP * (kD0 + 1); e += 64) {
        const int node = e / (kD0 + 1), k = e - node * (kD0 + 1);
        const bool nv = node >= n && node < N;
        float v = 0.0f;
        if (nv && k < p.D0) v = p.x[g * p.x_gstride + (int64_t)node * p.D0 + k];
        else if (nv && k == p.D0) v = 1.0f;
        RAW[e] = v;
      }
    }
  }
  for (int e = l; e < n * NP; e += 64) inv[e] = -1;
  if (Ac)  // forward: the attention rows start at 0 (masked candidates keep it)
    for (int e = l; e < 32 * 33; e += 64) Ac[e] = 0.0f;
  for (int e = l; e < E; e += 64) {
    const lanes::f32x4 v = *(const lanes::f32x4*)(p.ef + g * p.ef_gstride + (int64_t)e * 4);
    *(lanes::f32x4*)(EF + e * 4) = v;
  }
  lanes::wave_sync();
  for (int e = l; e < n * C; e += 64) {
    const int i = e / C, c = e - i * C;
    const int s = p.sidx[(g * n + i) * C + c];
    if (s >= 0) inv[i * NP + s] = (c << 16) | p.cand[i * C + c];
  }
  lanes::wave_sync();
}

// logits^T tiles, candidate mask and softmax: on return lg[t][j] = a (the attention weight of this lane's row
// for node_of(t, j, hf)), vm = the candidate bits (bit t * 16 + j)
template <int DM, int NT>
__device__ __forceinline__ uint64_t softmax(const dgppo_gnn_attn_args& p, int64_t g, const float* S, const int* inv,
                                            int i, int h, bool rv, f32x16 (&lg)[NT]) {
  constexpr int SP = DM + 1, KH = DM / 2, NP = NT * 32;
  const int l = threadIdx.x & 63, col = l & 31, hf = l >> 5;
  const int D = p.D, n = p.n_agents;
  float qb[KH];
  const float* qrow = p.qt + (g * n + i) * qt_ld(p) + h * D;
#pragma unroll
  for (int s = 0; s < KH; ++s) {
    const int k = hf * KH + s;
    const float v = qrow[k < D ? k : D - 1];  // (i, h) of an idle row is (0, 0): a valid address
    qb[s] = (rv && k < D) ? v : 0.0f;
  }
  const float bv = p.beta[(g * n + i) * p.beta_ld + h];
  const float beta = rv ? bv : 0.0f;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    lg[t] = f32x16{};
#pragma unroll
    for (int s = 0; s < KH; ++s)
      lg[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(S[(t * 32 + col) * SP + hf * KH + s], qb[s], lg[t], 0, 0, 0);
  }
  uint64_t vm = 0;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int4 iv = *(const int4*)(inv + i * NP + t * 32 + 8 * q + 4 * hf);
      vm |= (uint64_t)((iv.x >= 0) | ((iv.y >= 0) << 1) | ((iv.z >= 0) << 2) | ((iv.w >= 0) << 3)) << (t * 16 + 4 * q);
    }
  if (!rv) vm = 0;
  float mx = -INFINITY;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const float x = (lg[t][j] + beta) * p.scale;
      lg[t][j] = x;
      mx = ((vm >> (t * 16 + j)) & 1) ? fmaxf(mx, x) : mx;
    }
  mx = fmaxf(mx, xor32(mx));
  float sm = 0.0f;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const bool v = (vm >> (t * 16 + j)) & 1;
      const float e = v ? expf(lg[t][j] - mx) : 0.0f;
      lg[t][j] = e;
      sm += e;
    }
  sm += xor32(sm);
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int j = 0; j < 16; ++j) lg[t][j] = ((vm >> (t * 16 + j)) & 1) ? lg[t][j] / sm : 0.0f;
  return vm;
}

// Y^T (d x rows) = S^T . V^T with V (rows x nodes) in the accumulator layout (lane = row, register = node)
template <int DM, int NT>
__device__ __forceinline__ f32x16 sender_sum(const float* S, const f32x16 (&v)[NT]) {
  constexpr int SP = DM + 1;
  const int l = threadIdx.x & 63, col = l & 31, hf = l >> 5;
  f32x16 acc = {};
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const float a = S[node_of(t, j, hf) * SP + (col < DM ? col : DM - 1)];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(col < DM ? a : 0.0f, v[t][j], acc, 0, 0, 0);
    }
  return acc;
}

// accumulator layout (lane = row r, register j = d) -> X[r][d] (pitch 33) in LDS
__device__ __forceinline__ void to_rows(float* X, const f32x16& acc) {
  const int l = threadIdx.x & 63, col = l & 31, hf = l >> 5;
#pragma unroll
  for (int j = 0; j < 16; ++j) X[col * 33 + (j & 3) + 8 * (j >> 2) + 4 * hf] = acc[j];
}

template <int DM, int NT>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2, 8))) void attn_gm_fwd_kernel(
    dgppo_gnn_attn_args p) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int NP = NT * 32;
  const int l = threadIdx.x & 63, col = l & 31, hf = l >> 5;
  const int n = p.n_agents, D = p.D, H = kH, NR = kH * n;
  const Carve cv = carve(DM, NT, n, p.E, false, false);
  float* S = lds + cv.s;
  int* inv = (int*)(lds + cv.inv);
  float* EF = lds + cv.ef;
  float* T = lds + cv.t;
  const bool agent = p.xa != nullptr, pre = agent && p.pre_W != nullptr;
  float w4[4] = {0.0f, 0.0f, 0.0f, 0.0f}, b4 = 0.0f;
  if (pre) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int k = hf * 4 + s;
      w4[s] = (k < p.D0 && col < D) ? p.pre_W[k * D + col] : 0.0f;
    }
    b4 = col < D ? p.pre_b[col] : 0.0f;
  }
  const int r = col;
  const bool rv = r < NR;
  const int h = rv ? r / n : 0, i = rv ? r - (r / n) * n : 0;
  const int W = H * (D + 5);
  for (int64_t g = blockIdx.x; g < p.G; g += gridDim.x) {
    stage<DM, NT>(p, g, S, inv, EF, nullptr, w4, b4, agent, pre, lds + cv.p, lds + cv.total - 4);
    f32x16 a[NT];
    const uint64_t vm = softmax<DM, NT>(p, g, S, inv, i, h, rv, a);
    const f32x16 xb = sender_sum<DM, NT>(S, a);
    // edge head sums and sig over the candidates, attention weights out
    float e4[4] = {0.0f, 0.0f, 0.0f, 0.0f}, sg = 0.0f;
    float* Ac = lds + cv.p;  // [row][c] attention weights (pitch 33; column 32 is the sink of non-candidates)
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int v = inv[i * NP + node_of(t, j, hf)];
        const bool ok = ((vm >> (t * 16 + j)) & 1) != 0;
        const int c = ok ? v >> 16 : 32, e = ok ? v & 0xFFFF : 0;
        const lanes::f32x4 f = *(const lanes::f32x4*)(EF + e * 4);
        const float av = a[t][j];  // 0 off the candidates
#pragma unroll
        for (int k = 0; k < 4; ++k) e4[k] += av * f[k];
        sg += av;
        Ac[col * 33 + c] = av;
      }
#pragma unroll
    for (int k = 0; k < 4; ++k) e4[k] += xor32(e4[k]);
    sg += xor32(sg);
    lanes::wave_sync();  // every lane is past its reads of S: X aliases it
    if (p.attn) {  // attention rows of the graph ((g n + i) H + h) C + c: contiguous
      float* ao = p.attn + g * n * H * p.C;
      for (int e = l; e < n * H * p.C; e += 64) {
        const int ii = e / (H * p.C), k = e - ii * (H * p.C), hh = k / p.C, c = k - hh * p.C;
        ao[e] = Ac[(hh * n + ii) * 33 + c];
      }
    }
    float* X = S;
    to_rows(X, xb);
    if (rv && hf == 0) {
#pragma unroll
      for (int k = 0; k < 4; ++k) T[i * 16 + 4 * h + k] = e4[k];
      T[i * 16 + 12 + h] = sg;
    }
    lanes::wave_sync();
    // xcat rows of the graph: [xbar_0 | xbar_1 | xbar_2 | ebar (12) | sig (3)], contiguous over the graph
    float* out = p.xcat + g * n * W;
    for (int e = l; e < n * W; e += 64) {
      const int ii = e / W, k = e - ii * W;
      float v;
      if (k < H * D) {
        const int hh = k / D;
        v = X[(hh * n + ii) * 33 + (k - hh * D)];
      } else {
        v = T[ii * 16 + (k - H * D)];
      }
      out[e] = v;
    }
    lanes::wave_sync();  // X / T are rewritten by the next graph's staging
  }
}

template <int DM, int NT>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 8))) void attn_gm_bwd_kernel(
    dgppo_gnn_attn_args p) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int NP = NT * 32, KH = DM / 2, SP = DM + 1;
  const int l = threadIdx.x & 63, col = l & 31, hf = l >> 5;
  const int n = p.n_agents, D = p.D, H = kH, NR = kH * n, N = p.N, C = p.C;
  const bool agent = p.xa != nullptr, pre = agent && p.pre_W != nullptr;
  const bool want_dxa = agent && p.dxa != nullptr;
  const bool want_pre = pre && p.dpre_part != nullptr;
  const bool want_ds = want_dxa || want_pre;
  const Carve cv = carve(DM, NT, n, p.E, true, want_pre);
  float* S = lds + cv.s;
  int* inv = (int*)(lds + cv.inv);
  float* EF = lds + cv.ef;
  float* Pa = lds + cv.p;
  float* Pd = Pa + 32 * 33;
  float* RAW = want_pre ? lds + cv.raw : nullptr;
  float w4[4] = {0.0f, 0.0f, 0.0f, 0.0f}, b4 = 0.0f;
  if (pre) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int k = hf * 4 + s;
      w4[s] = (k < p.D0 && col < D) ? p.pre_W[k * D + col] : 0.0f;
    }
    b4 = col < D ? p.pre_b[col] : 0.0f;
  }
  const int r = col;
  const bool rv = r < NR;
  const int h = rv ? r / n : 0, i = rv ? r - (r / n) * n : 0;
  const int W = H * (D + 5);
  f32x16 gacc = {};  // [x_raw | 1]^T dz over this wave's graphs (M = raw column, N = d)
  for (int64_t g = blockIdx.x; g < p.G; g += gridDim.x) {
    stage<DM, NT>(p, g, S, inv, EF, RAW, w4, b4, agent, pre, nullptr, lds + cv.total - 4);
    f32x16 a[NT];
    const uint64_t vm = softmax<DM, NT>(p, g, S, inv, i, h, rv, a);
    // da^T = S . dXbar^T
    const float* grow = p.dxcat + (g * n + i) * W;
    f32x16 da[NT];
    {
      float gb[KH];
#pragma unroll
      for (int s = 0; s < KH; ++s) {
        const int k = hf * KH + s;
        const float v = grow[h * D + (k < D ? k : D - 1)];
        gb[s] = (rv && k < D) ? v : 0.0f;
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        da[t] = f32x16{};
#pragma unroll
        for (int s = 0; s < KH; ++s)
          da[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(S[(t * 32 + col) * SP + hf * KH + s], gb[s], da[t], 0, 0, 0);
      }
    }
    float de[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float v = grow[H * D + 4 * h + k];
      de[k] = rv ? v : 0.0f;
    }
    const float dsv = grow[H * D + 4 * H + h];
    const float ds = rv ? dsv : 0.0f;
    // edge / sig / extra-column terms on the candidates, then the softmax backward
    float dot = 0.0f;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const bool ok = ((vm >> (t * 16 + j)) & 1) != 0;
        const int q = inv[i * NP + node_of(t, j, hf)];
        const int c = ok ? q >> 16 : 0, e = ok ? q & 0xFFFF : 0;
        const lanes::f32x4 f = *(const lanes::f32x4*)(EF + e * 4);
        float v = da[t][j];
#pragma unroll
        for (int k = 0; k < 4; ++k) v += de[k] * f[k];
        v += ds;
        if (p.da_add) v += p.da_add[((g * n + i) * H + h) * C + c];
        v = ok ? v : 0.0f;
        da[t][j] = v;
        dot += a[t][j] * v;
      }
    dot += xor32(dot);
    float db = 0.0f;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const float dl = ((vm >> (t * 16 + j)) & 1) ? a[t][j] * (da[t][j] - dot) * p.scale : 0.0f;
        da[t][j] = dl;
        db += dl;
      }
    db += xor32(db);
    if (rv && hf == 0) p.dbeta[(g * n + i) * dbeta_ld(p) + h] = db;
    // dqt^T = S^T . dl^T, rows written through LDS (P is free until the sender-gradient phase)
    {
      const f32x16 dq = sender_sum<DM, NT>(S, da);
      to_rows(Pa, dq);
      lanes::wave_sync();
      for (int e = l; e < n * H * D; e += 64) {
        const int ii = e / (H * D), k = e - ii * (H * D), hh = k / D;
        p.dqt[(g * n + ii) * dqt_ld(p) + k] = Pa[(hh * n + ii) * 33 + (k - hh * D)];
      }
      lanes::wave_sync();
    }
    if (want_ds) {
      // B operands of the sender gradient: dxbar and qt rows k = hf * 16 + s at column d = col
      float gx[16], qx[16];
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const int k = hf * 16 + s;
        const bool ok = k < NR && col < D;
        const int kc = k < NR ? k : NR - 1, cc = col < D ? col : D - 1;
        const int hk = kc / n, ik = kc - hk * n;
        const float gv = p.dxcat[(g * n + ik) * W + hk * D + cc];
        const float qv = p.qt[(g * n + ik) * qt_ld(p) + hk * D + cc];
        gx[s] = ok ? gv : 0.0f;
        qx[s] = ok ? qv : 0.0f;
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        // transpose this node tile's a / dl (lane = row) into P[row][node]
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const int nl = (j & 3) + 8 * (j >> 2) + 4 * hf;
          Pa[col * 33 + nl] = a[t][j];
          Pd[col * 33 + nl] = da[t][j];
        }
        lanes::wave_sync();
        f32x16 acc = {};
#pragma unroll
        for (int s = 0; s < 16; ++s) {
          const int k = hf * 16 + s;
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(Pa[k * 33 + col], gx[s], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(Pd[k * 33 + col], qx[s], acc, 0, 0, 0);
        }
        // acc: lane = d (col), register j = node_of(t, j, hf)
        if (want_dxa && t == 0) {  // agents are nodes 0..n-1: dS rows -> LDS (P is free now) -> dxa rows
          lanes::wave_sync();
#pragma unroll
          for (int j = 0; j < 16; ++j) Pa[((j & 3) + 8 * (j >> 2) + 4 * hf) * 33 + col] = acc[j];
          lanes::wave_sync();
          float* dst = p.dxa + g * p.dxa_gstride;
          for (int e = l; e < n * D; e += 64) {
            const int nd = e / D;
            dst[e] += Pa[nd * 33 + (e - nd * D)];
          }
        }
        if (want_pre) {
#pragma unroll
          for (int j = 0; j < 16; ++j) {
            const int nd = node_of(t, j, hf);
            const bool nv = nd >= n && nd < N && col < D;
            const float sv = S[nd * SP + col];  // pre => DM = 32: col is inside the row
            const float dz = (nv && sv > 0.0f) ? acc[j] : 0.0f;
            const float rw = RAW[nd * (kD0 + 1) + (col <= kD0 ? col : kD0)];
            gacc = __builtin_amdgcn_mfma_f32_32x32x2f32(col <= kD0 ? rw : 0.0f, dz, gacc, 0, 0, 0);
          }
        }
        lanes::wave_sync();  // P is rewritten by the next tile
      }
    }
  }
  if (want_pre) {  // this workgroup's partial row: [W4 rows (D0 x D) | b4 (D)]
    const int PK = p.D0 * D + D;
    float* part = p.dpre_part + (int64_t)blockIdx.x * PK;
    if (col < D) {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int k = (j & 3) + 8 * (j >> 2) + 4 * hf;
        if (k < p.D0) part[k * D + col] = gacc[j];
        else if (k == p.D0) part[p.D0 * D + col] = gacc[j];
      }
    }
  }
}

}  // namespace gm

// ---- dispatch ------------------------------------------------------------------------------------------------
// Off by default: measured 2.3-4.8x SLOWER than the row-block kernels at the bench shape (LidarSpread n8, 16384
// graphs: fwd D=8 209 vs 79 us, fwd D=32 708 vs 180, bwd D=8 391 vs 81, bwd D=32 877 vs 390; profiles/r04_attn_gm_*):
// the node-space softmax / weight / edge work is dense over the graph's 96 node slots per receiver row where the
// candidate-space kernels touch 24, so the MFMA products save less than the 4x elementwise work costs (PMC: 1.1-1.7x
// the VALU instructions of the row-block kernels on 16x fewer waves).  Kept, tested against the row-block kernels,
// for DGPPO_ATTN_GM=1 / dgppo_gnn_set_attn_kernel(1).
int g_attn_gm = -1;  // dgppo_gnn_set_attn_kernel
inline bool gm_enabled() {
  if (g_attn_gm < 0) {
    const char* e = getenv("DGPPO_ATTN_GM");
    g_attn_gm = (e && atoi(e) == 1) ? 1 : 0;
  }
  return g_attn_gm == 1;
}

inline int gm_dm(const dgppo_gnn_attn_args* p) {
  const bool pre = p->xa && p->pre_W;
  return (p->D <= 8 && !pre) ? 8 : (p->D <= 16 && !pre) ? 16 : 32;
}

inline bool gm_ok(const dgppo_gnn_attn_args* p, bool bwd) {
  if (!gm_enabled() || p->H != kH || p->n_agents * kH > 32 || p->N > 32 * gm::kMaxNT || p->D > 32 || !p->sidx ||
      !p->beta || p->q || p->E >= 65536 || p->C >= 32768)
    return false;
  if (p->xa && (p->D0 < 1 || p->D0 > kD0 || (p->pre_W && p->D0 >= 32)))
    return false;
  if (bwd && (p->dq || (!p->xa && p->dx)))  // full-mode sender gradients (deep GNN layers): the other kernels
    return false;
  const int NT = (p->N + 31) / 32;
  const gm::Carve cv = gm::carve(gm_dm(p), NT, p->n_agents, p->E, bwd, bwd && p->xa && p->pre_W && p->dpre_part);
  return (size_t)cv.total * sizeof(float) <= 64 * 1024;
}

inline int64_t gm_grid(const dgppo_gnn_attn_args* p) {
  const int64_t cap = 256 * 8;  // resident one-wave workgroups (2 per SIMD)
  return p->G < cap ? p->G : cap;
}

template <int DM, int NT>
void gm_launch_t(const dgppo_gnn_attn_args* p, bool bwd, hipStream_t s) {
  const gm::Carve cv = gm::carve(DM, NT, p->n_agents, p->E, bwd, bwd && p->xa && p->pre_W && p->dpre_part);
  const size_t bytes = (size_t)cv.total * sizeof(float);
  const unsigned grid = (unsigned)gm_grid(p);
  if (bwd) hipLaunchKernelGGL((gm::attn_gm_bwd_kernel<DM, NT>), dim3(grid), dim3(64), bytes, s, *p);
  else hipLaunchKernelGGL((gm::attn_gm_fwd_kernel<DM, NT>), dim3(grid), dim3(64), bytes, s, *p);
}

inline void gm_launch(const dgppo_gnn_attn_args* p, bool bwd, hipStream_t s) {
  const int NT = (p->N + 31) / 32, DM = gm_dm(p);
#define DG_GM(dm, nt) \
  if (DM == dm && NT == nt) return gm_launch_t<dm, nt>(p, bwd, s);
  DG_GM(8, 1) DG_GM(8, 2) DG_GM(8, 3) DG_GM(16, 1) DG_GM(16, 2) DG_GM(16, 3) DG_GM(32, 1) DG_GM(32, 2) DG_GM(32, 3)
#undef DG_GM
}
