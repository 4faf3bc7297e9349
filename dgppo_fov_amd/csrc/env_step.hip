// Fused env-step / env-reset kernels for gfx950 (MI355X): hot path (1) of DGPPO.
//
// One workgroup owns one environment for the whole transition, so every intermediate (agent
// states, obstacle records, per-ray hit distances, sorted hits) lives in LDS and each env touches
// HBM exactly once per input byte and once per output byte:
//   read : current graph states (agents, goals, lidar hits / MPE obstacles), obstacle records,
//          actions                                                       (~1 KB per env, n=8)
//   write: next graph nodes, edges, states, receivers, senders, reward, cost (~8.4 KB per env)
// The step is HBM-bound (~9 flop/B against a 20 flop/B fp32 ridge), so the design
// goal is coalesced streaming stores: lane-contiguous dword stores for nodes/states/indices and
// one dwordx4 store per edge row.
//
// Reference semantics (all in the reference's fp32 operation order, see include/dgppo_hip.h):
//   dynamics     lidar_env/base.py:142-149, mpe/base.py:129-135, lidar_bicycle_target.py:92-111
//   lidar        env/utils.py:49-79 (get_lidar), 115-136 (raytracing), env/obstacle.py:62-105
//   reward       lidar_spread.py:35-52, lidar_target.py:35-52, mpe_spread.py:32-49, mpe_target.py:32-49
//   cost         lidar_env/base.py:180-207, mpe/base.py:164-191
//   graph        lidar_env/base.py:227-271, mpe/base.py:211-241, utils/graph.py:35-44, 212-247
//   reset        lidar_env/base.py:89-124, lidar_bicycle_target.py:60-90, mpe/base.py:81-127,
//                env/utils.py:139-244
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>

#include "../../include/dgppo_hip.h"
#include "math32.h"
#include "vmas.h"

#pragma clang fp contract(off)

namespace dgppo {

constexpr int kMaxAgents = 64;
constexpr int kMaxObs = 16;
constexpr int kMaxRays = 128;

__device__ __forceinline__ float clampf_nan(float x, float lo, float hi) {
  // jnp.clip = minimum(maximum(x, lo), hi): NaN propagates (v_max/v_min_f32 would drop it)
  x = x < lo ? lo : x;
  return x > hi ? hi : x;
}
// clampf_nan for a NONZERO constant bound pair: IEEE maximum / minimum (v_maximum3 / v_minimum3, NaN-propagating)
// give the same value for every x (no signed-zero tie with a nonzero bound), NaN payload aside
__device__ __forceinline__ float clampk(float x, float lo, float hi) {
  return __builtin_elementwise_minimum(__builtin_elementwise_maximum(x, lo), hi);
}
__device__ __forceinline__ float min_nan(float a, float b) {
  // jnp.min / jnp.minimum semantics: NaN wins
  return (a != a || a < b) ? a : b;
}
__device__ __forceinline__ float sq2(float dx, float dy) { return dx * dx + dy * dy; }
__device__ __forceinline__ float norm2(float dx, float dy) { return sqrtf(sq2(dx, dy)); }

// ---- LDS carve (floats) -------------------------------------------------------------------------
struct Carve {
  int cur, curhit, obst, evec, act, nxt, alpha, hpt, hits, isin, red, samp, dist, dist_n, cull, total;
  __host__ __device__ Carve(int n, int sd, int O, int R, int k, bool lidar) {
    int off = 0;
    auto take = [&](int nf) { int o = off; off += (nf + 3) & ~3; return o; };
    cur = take(2 * n * sd + (lidar ? 0 : O * sd));  // agents, goals (+ MPE obstacle rows)
    curhit = take(lidar ? n * k * 2 : 0);
    obst = take(lidar ? O * DGPPO_OBST_FIELDS : 0);
    evec = take(lidar ? O * 8 : 0);
    act = take(n * 2);
    nxt = take(n * sd);
    alpha = take(lidar ? n * R * 2 : 0);  // 64-bit sort keys
    hpt = take(lidar ? n * R * 2 : 0);
    hits = take(lidar ? n * k * 2 : 0);
    isin = take(n);
    red = take(5 * n);  // d2goal, far, |a|^2, cost0, cost1
    samp = take(4 * n);  // reset: sampled positions / goals (n, 2) each
    // step: pairwise distance tasks; lidar_scan: the culling's work list (dist is dead by then)
    dist_n = 2 * n * n + n * (k > O ? k : O) > 256 ? 2 * n * n + n * (k > O ? k : O) : 256;
    dist = take(dist_n);
    // lidar_scan: unsafe masks | radii | count | alpha codes | (16-byte aligned) ray table
    cull = take(lidar ? ((2 * O + 4 + n * R + 3) & ~3) + 4 * R : 0);
    total = off;
  }
};

// persistent block rollout: episodes with T * 2n <= kActStage action floats stage them all in LDS (after the carve)
constexpr int kActStage = 4096;

// Sizes: compile-time where a specialisation fixes them (0 / -1 = read from cfg at run time)
template <int NA, int NO, int NR, int NK>
struct Dims {
  int n, O, R, k;
  __device__ __forceinline__ explicit Dims(const dgppo_env_cfg& c)
      : n(NA > 0 ? NA : c.n_agents), O(NO >= 0 ? NO : c.n_obs), R(NR > 0 ? NR : c.n_rays), k(NK > 0 ? NK : c.top_k) {}
};

struct GraphOut {
  float* nodes;
  float* edges;
  float* states;
  int32_t* recv;
  int32_t* send;
};

// ---- Rectangle helpers (env/obstacle.py) ------------------------------------------------------
__device__ __forceinline__ bool rect_inside(const float* rec, float px, float py, float r) {
  const float rel_x = px - rec[0];
  const float rel_y = py - rec[1];
  const float c = rec[5], s = rec[6];
  const float rel_xx = fabsf(rel_x * c + rel_y * s) - rec[2] / 2.0f;
  const float rel_yy = fabsf(rel_x * s - rel_y * c) - rec[3] / 2.0f;
  const bool down = (rel_xx < r) && (rel_yy < 0.0f);
  const bool up = (rel_xx < 0.0f) && (rel_yy < r);
  const bool corner = (rel_xx > 0.0f) && (rel_yy > 0.0f);
  const bool circle = sqrtf(rel_xx * rel_xx + rel_yy * rel_yy) < r;
  return down || up || (corner && circle);
}

// Rectangle.raytracing for one ray against the 4 edges of one obstacle.
//
// Exactly the reference's result, with most IEEE divisions skipped: an edge whose alpha or beta is
// PROVABLY outside [0, 1] contributes exactly 1e6 in the reference (valid = 0 -> 0*alpha + 1e6), so
// for it we only need the numerators and det, not the quotients.  The screens below are
// conservative (1.001 margin on the ratio, 1e-30 floor against underflow to -0, finite numerators
// only); everything else -- including det == 0 and NaN inputs, which make the reference's alpha NaN --
// takes the full divide-and-compare path.  The per-ray terms ax = x1-x2, ay = y1-y2 and per-edge
// vectors (x4-x3, y4-y3) are exactly the reference's sub-expressions, hoisted.
__device__ __forceinline__ float rect_raytrace(const float* rec, const float* evec, float x1, float y1, float ax,
                                               float ay) {
  float best = 0.0f;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float x3 = rec[8 + 2 * e], y3 = rec[9 + 2 * e];
    const float exe = evec[2 * e], eye = evec[2 * e + 1];  // x4 - x3, y4 - y3
    const float px = x1 - x3, py = y1 - y3;
    const float det = ax * eye - ay * exe;
    const float na = eye * px - exe * py;
    const float nb = (-ay) * px + ax * py;
    const float adet = fabsf(det);
    float a;
    if (!(adet > 0.0f)) {
      a = __builtin_nanf("");  // det == 0 (sign 0) or NaN: the reference's alpha is NaN
    } else {
      const float cl = adet < 1e-7f ? 1e-7f : (adet > 1e7f ? 1e7f : adet);
      const float detc = det < 0.0f ? -cl : cl;
      const float lim = cl * 1.001f;
      const float ana = fabsf(na), anb = fabsf(nb);
      const bool finite = ana <= 3.0e38f && anb <= 3.0e38f;
      const bool neg_d = detc < 0.0f;
      const bool out = finite && (ana > lim || anb > lim || (ana >= 1e-30f && ((na < 0.0f) != neg_d)) ||
                                  (anb >= 1e-30f && ((nb < 0.0f) != neg_d)));
      if (out) {
        a = 1e6f;
      } else {
        const float alpha = na / detc;
        const float beta = nb / detc;
        const bool valid = (alpha <= 1.0f) && (alpha >= 0.0f) && (beta <= 1.0f) && (beta >= 0.0f);
        a = valid ? alpha + 0.0f : (alpha != alpha ? alpha : 1e6f);
      }
    }
    best = e == 0 ? a : min_nan(best, a);
  }
  return best;
}

// ---- graph writer: nxt (agents), goal rows, hits / obstacle rows, all in LDS ------------------
template <int ENGINE, int GOAL, int SD, class D>
__device__ __forceinline__ void write_graph(const dgppo_env_cfg& cfg, const D& d, const float* nxt,
                                            const float* goal, const float* third, GraphOut out, bool edges_vec4,
                                            int tid, int nthr) {
  constexpr int ND = SD + 3;
  constexpr bool mpe = ENGINE == DGPPO_ENGINE_MPE;
  const int n = d.n, O = d.O, k = d.k;
  const int n_third = mpe ? O : (O > 0 ? n * k : 0);
  const int N = 2 * n + n_third + 1;
  const int n_ag = GOAL == DGPPO_GOAL_SPREAD ? n * n : n;
  const int E = n * n + n_ag + (mpe ? n * O : n_third);
  const int pad = N - 1;
  const float comm = cfg.comm_radius;

  // nodes (N, ND): [state | obs, goal, agent one-hot]; lidar hit rows carry [hx, hy, 0...]
#pragma unroll 1
  for (int idx = tid; idx < N * ND; idx += nthr) {
    const int r = idx / ND;
    const int c = idx - r * ND;
    float v = 0.0f;
    if (r < n) {
      v = c < SD ? nxt[r * SD + c] : (c == SD + 2 ? 1.0f : 0.0f);
    } else if (r < 2 * n) {
      v = c < SD ? goal[(r - n) * SD + c] : (c == SD + 1 ? 1.0f : 0.0f);
    } else if (r < 2 * n + n_third) {
      const int h = r - 2 * n;
      if (mpe) v = c < SD ? third[h * SD + c] : (c == SD ? 1.0f : 0.0f);
      else v = c < 2 ? third[h * 2 + c] : (c == SD ? 1.0f : 0.0f);
    }
    out.nodes[idx] = v;
  }
  // states (N, SD); pad row is -1.  4-wide rows into a 16-byte aligned buffer: one float4 per row and lane (the LDS
  // rows are 16-byte aligned: Carve regions are), else one float per element
  if (SD == 4 && (reinterpret_cast<uintptr_t>(out.states) & 15u) == 0) {
#pragma unroll 1
    for (int r = tid; r < N; r += nthr) {
      float4 v;
      if (r < n) {
        v = *reinterpret_cast<const float4*>(nxt + r * SD);
      } else if (r < 2 * n) {
        v = *reinterpret_cast<const float4*>(goal + (r - n) * SD);
      } else if (r < 2 * n + n_third) {
        const int h = r - 2 * n;
        v = mpe ? *reinterpret_cast<const float4*>(third + h * SD) : make_float4(third[h * 2], third[h * 2 + 1], 0.0f, 0.0f);
      } else {
        v = make_float4(-1.0f, -1.0f, -1.0f, -1.0f);
      }
      reinterpret_cast<float4*>(out.states)[r] = v;
    }
  } else {
#pragma unroll 1
    for (int idx = tid; idx < N * SD; idx += nthr) {
      const int r = idx / SD;
      const int c = idx - r * SD;
      float v;
      if (r < n) v = nxt[r * SD + c];
      else if (r < 2 * n) v = goal[(r - n) * SD + c];
      else if (r < 2 * n + n_third) {
        const int h = r - 2 * n;
        v = mpe ? third[h * SD + c] : (c < 2 ? third[h * 2 + c] : 0.0f);
      } else v = -1.0f;
      out.states[idx] = v;
    }
  }
  // edges: [agent-agent n*n][agent-goal][agent-lidar n*k | agent-obstacle n*O]
  const int n_aa = n * n;
  // Lidar double-integrator rows (SD = 4) with nthr a multiple of n (the n = 32 block kernel): a thread's sender
  // column j = tid % n is the same in every agent-agent / agent-goal iteration, so its agent and goal rows stay in
  // registers as float4s and each edge reads only the receiver's row (one broadcast float4 per wave and half-wave)
  // instead of eight scalar LDS reads; receiver i advances by nthr / n without a division.  Same arithmetic.
  if (SD == 4 && ENGINE != DGPPO_ENGINE_BICYCLE && !mpe && edges_vec4 && nthr % n == 0) {
    const int j = tid % n, di = nthr / n;
    float4* eo4 = reinterpret_cast<float4*>(out.edges);
    {
      const float4 sj = *reinterpret_cast<const float4*>(nxt + j * SD);
#pragma unroll 1
      for (int i = tid / n; i < n; i += di) {
        const float4 si = *reinterpret_cast<const float4*>(nxt + i * SD);
        const int e = i * n + j;
        const float d2 = sq2(si.x - sj.x, si.y - sj.y);
        const bool m = i == j ? ((d2 == 0.0f) & (cfg.c_self_dist < comm)) : (d2 < cfg.t2_comm);
        eo4[e] = make_float4(si.x - sj.x, si.y - sj.y, si.z - sj.z, si.w - sj.w);
        out.recv[e] = m ? i : pad;
        out.send[e] = m ? j : pad;
      }
    }
    if (GOAL == DGPPO_GOAL_SPREAD) {
      const float4 gj = *reinterpret_cast<const float4*>(goal + j * SD);
#pragma unroll 1
      for (int i = tid / n; i < n; i += di) {
        const float4 si = *reinterpret_cast<const float4*>(nxt + i * SD);
        const int eg = n_aa + i * n + j;
        eo4[eg] = make_float4(si.x - gj.x, si.y - gj.y, si.z - gj.z, si.w - gj.w);
        out.recv[eg] = i;
        out.send[eg] = n + j;
      }
    }
    if (GOAL != DGPPO_GOAL_SPREAD) {
#pragma unroll 1
      for (int q = tid; q < n; q += nthr) {
        const float4 si = *reinterpret_cast<const float4*>(nxt + q * SD);
        const float4 gq = *reinterpret_cast<const float4*>(goal + q * SD);
        eo4[n_aa + q] = make_float4(si.x - gq.x, si.y - gq.y, si.z - gq.z, si.w - gq.w);
        out.recv[n_aa + q] = q;
        out.send[n_aa + q] = n + q;
      }
    }
#pragma unroll 1
    for (int q = tid; q < n_third; q += nthr) {  // agent-lidar blocks (1, k) per agent
      const int i = q / k;
      const float2 si = *reinterpret_cast<const float2*>(nxt + i * SD);
      const float2 hq = *reinterpret_cast<const float2*>(third + 2 * q);
      const float f0 = si.x - hq.x, f1 = si.y - hq.y;
      const bool m = sq2(f0, f1) < cfg.t2_lidar;
      const int e = n_aa + n_ag + q;
      eo4[e] = make_float4(f0, f1, 0.0f, 0.0f);
      out.recv[e] = m ? i : pad;
      out.send[e] = m ? 2 * n + q : pad;
    }
    return;
  }
#pragma unroll 1
  for (int e = tid; e < E; e += nthr) {
    float f0, f1, f2, f3;
    int rv, sv;
    if (e < n_aa) {
      const int i = e / n, j = e - (e / n) * n;
      const float* si = nxt + i * SD;
      const float* sj = nxt + j * SD;
      if (ENGINE == DGPPO_ENGINE_BICYCLE) {  // state2feat = [x, y, v cos, v sin]
        f0 = si[0] - sj[0];
        f1 = si[1] - sj[1];
        f2 = si[4] * si[2] - sj[4] * sj[2];
        f3 = si[4] * si[3] - sj[4] * sj[3];
      } else {
        f0 = si[0] - sj[0];
        f1 = si[1] - sj[1];
        f2 = si[2] - sj[2];
        f3 = si[3] - sj[3];
      }
      // norm + (c_self_dist on the diagonal) < comm_radius on the squared norm: sqrtf is correctly
      // rounded and monotone, so sqrtf(x) < r <=> x < t2_comm; the diagonal's difference is exactly 0 or NaN
      const float d2 = sq2(si[0] - sj[0], si[1] - sj[1]);
      const bool m = i == j ? ((d2 == 0.0f) & (cfg.c_self_dist < comm)) : (d2 < cfg.t2_comm);
      rv = m ? i : pad;
      sv = m ? j : pad;
    } else if (e < n_aa + n_ag) {
      const int q = e - n_aa;
      int i, j;
      if (GOAL == DGPPO_GOAL_SPREAD) {
        i = q / n;
        j = q - i * n;
      } else {
        i = q;
        j = q;
      }
      const float* si = nxt + i * SD;
      const float* gj = goal + j * SD;
      if (ENGINE == DGPPO_ENGINE_BICYCLE) {
        f0 = si[0] - gj[0];
        f1 = si[1] - gj[1];
        f2 = si[4] * si[2] - gj[4] * gj[2];
        f3 = si[4] * si[3] - gj[4] * gj[3];
      } else {
        f0 = si[0] - gj[0];
        f1 = si[1] - gj[1];
        f2 = si[2] - gj[2];
        f3 = si[3] - gj[3];
      }
      rv = i;
      sv = n + j;
    } else {
      const int q = e - n_aa - n_ag;
      if (mpe) {  // agent-obstacle block (n, O), mask ||p_i - o|| < comm_radius
        const int i = q / O, o = q - (q / O) * O;
        const float* si = nxt + i * SD;
        const float* so = third + o * SD;
        f0 = si[0] - so[0];
        f1 = si[1] - so[1];
        f2 = si[2] - so[2];
        f3 = si[3] - so[3];
        const bool m = sq2(si[0] - so[0], si[1] - so[1]) < cfg.t2_comm;
        rv = m ? i : pad;
        sv = m ? 2 * n + o : pad;
      } else {  // agent-lidar blocks (1, k) per agent, mask ||p_i - hit|| < comm_radius - 0.1
        const int i = q / k, h = q - (q / k) * k;
        const float* si = nxt + i * SD;
        f0 = si[0] - third[(i * k + h) * 2 + 0];
        f1 = si[1] - third[(i * k + h) * 2 + 1];
        f2 = 0.0f;
        f3 = 0.0f;
        const bool m = sq2(f0, f1) < cfg.t2_lidar;
        rv = m ? i : pad;
        sv = m ? 2 * n + i * k + h : pad;
      }
    }
    if (edges_vec4) {
      reinterpret_cast<float4*>(out.edges)[e] = make_float4(f0, f1, f2, f3);
    } else {
      out.edges[4 * e + 0] = f0;
      out.edges[4 * e + 1] = f1;
      out.edges[4 * e + 2] = f2;
      out.edges[4 * e + 3] = f3;
    }
    out.recv[e] = rv;
    out.send[e] = sv;
  }
}

// MPE graph writer without divergent sections: every element's LDS source row is chosen by selects and read with
// one unconditional load, so an iteration costs one LDS round trip instead of one per row kind (the if-chains of
// write_graph serialise the kinds' LDS latencies across the wave).  Same values, same arithmetic.
template <int GOAL, int SD, class D>
__device__ __forceinline__ void write_graph_mpe(const dgppo_env_cfg& cfg, const D& d, const float* nxt,
                                                const float* goal, const float* obs, GraphOut out, bool edges_vec4,
                                                int tid, int nthr) {
  constexpr int ND = SD + 3;
  const int n = d.n, O = d.O;
  const int N = 2 * n + O + 1;
  const int n_ag = GOAL == DGPPO_GOAL_SPREAD ? n * n : n;
  const int n_aa = n * n;
  const int E = n_aa + n_ag + n * O;
  const int pad = N - 1;
  // row r's state row in LDS (the pad row reads row 0 and is masked)
  auto row_ptr = [&](int r) -> const float* {
    const float* p = r < n ? nxt + r * SD : (r < 2 * n ? goal + (r - n) * SD : obs + (r - 2 * n) * SD);
    return r < pad ? p : nxt;
  };
#pragma unroll 1
  for (int idx = tid; idx < N * ND; idx += nthr) {
    const int r = idx / ND;
    const int c = idx - r * ND;
    const float x = row_ptr(r)[c < SD ? c : 0];
    const int hot = r < n ? SD + 2 : (r < 2 * n ? SD + 1 : SD);  // agent / goal / obstacle one-hot column
    out.nodes[idx] = r == pad ? 0.0f : (c < SD ? x : (c == hot ? 1.0f : 0.0f));
  }
#pragma unroll 1
  for (int idx = tid; idx < N * SD; idx += nthr) {
    const int r = idx / SD;
    const int c = idx - r * SD;
    const float x = row_ptr(r)[c];
    out.states[idx] = r == pad ? -1.0f : x;
  }
#pragma unroll 1
  for (int e = tid; e < E; e += nthr) {
    const bool aa = e < n_aa, ag = !aa && e < n_aa + n_ag;
    const int q = aa ? e : (ag ? e - n_aa : e - n_aa - n_ag);
    int i, j;
    if (GOAL == DGPPO_GOAL_SPREAD || !ag) {
      const int m = ag || aa ? n : O;
      i = q / m;
      j = q - i * m;
    } else {
      i = q;
      j = q;
    }
    const float* si = nxt + i * SD;
    const float* so = aa ? nxt + j * SD : (ag ? goal + j * SD : obs + j * SD);
    const float s0 = si[0], s1 = si[1], s2 = si[2], s3 = si[3];
    const float o0 = so[0], o1 = so[1], o2 = so[2], o3 = so[3];
    const float f0 = s0 - o0, f1 = s1 - o1, f2 = s2 - o2, f3 = s3 - o3;
    const float d2 = sq2(s0 - o0, s1 - o1);
    bool m;
    if (aa) m = i == j ? ((d2 == 0.0f) & (cfg.c_self_dist < cfg.comm_radius)) : (d2 < cfg.t2_comm);
    else m = ag ? true : (d2 < cfg.t2_comm);
    const int sv0 = aa ? j : (ag ? n + j : 2 * n + j);
    if (edges_vec4) {
      reinterpret_cast<float4*>(out.edges)[e] = make_float4(f0, f1, f2, f3);
    } else {
      out.edges[4 * e + 0] = f0;
      out.edges[4 * e + 1] = f1;
      out.edges[4 * e + 2] = f2;
      out.edges[4 * e + 3] = f3;
    }
    out.recv[e] = m ? i : pad;
    out.send[e] = m ? sv0 : pad;
  }
}

// MPE step tasks (block_step phase B) without divergent sections, when they fit one pass of the workgroup: lane q
// reads the operands of every task kind it could be (dynamics of agent q, or one distance), all loads issued
// together, then computes and stores its own kind.  Same arithmetic as the generic task loop.
template <int GOAL, int SD>
__device__ __forceinline__ void mpe_tasks(const dgppo_env_cfg& cfg, float* lds, const Carve& cv, int n, int O, int q) {
  const float* cur = lds + cv.cur;
  const float* goal = cur + n * SD;
  const float* obs = cur + 2 * n * SD;
  float* dist = lds + cv.dist;
  const int n_aa = n * n;
  const int n_ga = GOAL == DGPPO_GOAL_SPREAD ? n * n : n;
  const int n_task = n + n_aa + n_ga + n * O;
  // dynamics operands (agent q)
  const int id = q < n ? q : 0;
  const float* x = cur + id * SD;
  const float* a = lds + cv.act + 2 * id;
  const float x0 = x[0], x1 = x[1], x2 = x[2], x3 = x[3], a0 = a[0], a1 = a[1];
  // distance operands: A - B with (A, B) = (agent i, agent j) | (goal gj, agent ai) | (agent i, obstacle o)
  const int t = q - n;
  const bool aa = t >= 0 && t < n_aa, ga = t >= n_aa && t < n_aa + n_ga;
  const int tg = t - n_aa, to = t - n_aa - n_ga;
  int ia, ib, slot;
  const float *pa, *pb;
  if (aa) {
    ia = t / n;
    ib = t - ia * n;
    pa = cur + ia * SD;
    pb = cur + ib * SD;
    slot = t;
  } else if (ga) {
    const int gj = GOAL == DGPPO_GOAL_SPREAD ? tg / n : tg;
    const int ai = GOAL == DGPPO_GOAL_SPREAD ? tg - gj * n : tg;
    ia = gj;
    ib = ai;
    pa = goal + gj * SD;
    pb = cur + ai * SD;
    slot = n_aa + tg;
  } else {
    const int tt = (to >= 0 && q < n_task) ? to : 0;  // lanes past the tasks read obstacle 0 of agent 0
    const int i = O > 0 ? tt / O : 0, o = tt - i * (O > 0 ? O : 1);
    ia = i;
    ib = o;
    pa = cur + i * SD;
    pb = obs + o * SD;
    slot = 2 * n_aa + tt;
  }
  const float pa0 = pa[0], pa1 = pa[1], pb0 = pb[0], pb1 = pb[1];
  if (q < n) {  // dynamics (mpe/base.py double integrator), then clip_state
    float y[SD];
    y[0] = x2 * cfg.dt + x0;
    y[1] = x3 * cfg.dt + x1;
    y[2] = (a0 * 10.0f) * cfg.dt + x2;
    y[3] = (a1 * 10.0f) * cfg.dt + x3;
#pragma unroll
    for (int c = 0; c < SD; ++c) lds[cv.nxt + q * SD + c] = clampf_nan(y[c], cfg.state_lo[c], cfg.state_hi[c]);
    const float an = norm2(a0, a1);
    lds[cv.red + 2 * n + q] = an * an;
  } else if (q < n_task) {
    float dj = norm2(pa0 - pb0, pa1 - pb1);
    if (aa && ia == ib) dj = dj + 1e6f;
    dist[slot] = dj;
  }
}

// ---- lidar: per-ray hit distance, then a stable NaN-last rank -> top-k hits -------------------
// jnp.argsort (stable, NaN last, -0 == +0) as one 64-bit key per ray: high word = the alpha bits
// mapped to an unsigned total order (every NaN -> 0xFFFFFFFF, -0 -> +0), low word = ray index.
__device__ __forceinline__ uint64_t sort_key(float a, int r) {
  uint32_t u = __float_as_uint(a + 0.0f);  // -0 -> +0
  uint32_t ord = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  if (a != a) ord = 0xFFFFFFFFu;
  return ((uint64_t)ord << 32) | (uint32_t)r;
}

template <int SD, class D>
__device__ __forceinline__ void lidar_scan(const D& d, const float* ray_dirs, float* lds, const Carve& cv, int tid,
                                           int nthr) {
  const int n = d.n, R = d.R, k = d.k, O = d.O;
  const float* nxt = lds + cv.nxt;
  const float* obst = lds + cv.obst;
  const float* evec = lds + cv.evec;
  uint64_t* keys = reinterpret_cast<uint64_t*>(lds + cv.alpha);
  float* hpt = lds + cv.hpt;
  if (R <= 32) {
    // Exact culling with a compacted work list, the workgroup form of the wave kernel's (proof in the
    // notes before namespace wv): a (agent, obstacle, ray) triple is left at the reference's 1e6
    // unless the ray is unsafe for the obstacle (ineligible obstacle, |d| > 1 or a near-parallel edge),
    // the agent lies outside [-2, 2]^2 or the ray segment meets the disc (c, rho + 0.01).  Survivors
    // are ray-cast by the whole workgroup, one list-sized round at a time, and min-combined per (agent, ray)
    // with an LDS atomic on an order-preserving code (NaN wins, as min_nan).  Work list: the dist region.
    uint32_t* unsafe = reinterpret_cast<uint32_t*>(lds + cv.cull);  // (O) bit r: ray r must be cast
    float* rho = lds + cv.cull + O;                                    // (O) circumradius bound, -1 ineligible
    int* cnt = reinterpret_cast<int*>(lds + cv.cull + 2 * O);
    uint32_t* aenc = reinterpret_cast<uint32_t*>(lds + cv.cull + 2 * O + 4);  // (n R) alpha codes
    float4* rayc = reinterpret_cast<float4*>(lds + cv.cull + ((2 * O + 4 + n * R + 3) & ~3));  // (R) [dx, dy, |d|^2, |d| bound]
    int* items = reinterpret_cast<int*>(lds + cv.dist);  // the step's distance tasks are dead here
    const int cap = n * R * O < cv.dist_n ? n * R * O : cv.dist_n;
    auto enc = [](float a) { return a != a ? 0u : __float_as_uint(a) + 1u; };
    for (int o = tid; o < O; o += nthr) {
      const float* rec = obst + o * DGPPO_OBST_FIELDS;
      const float cx = rec[0], cy = rec[1];
      float r2 = 0.0f;
      bool elig = (fabsf(cx) <= 2.0f) & (fabsf(cy) <= 2.0f);
      for (int q = 0; q < 4; ++q) {
        const float px = rec[8 + 2 * q], py = rec[9 + 2 * q];
        elig = elig & (fabsf(px) <= 2.0f) & (fabsf(py) <= 2.0f);
        const float dx = px - cx, dy = py - cy;
        r2 = fmaxf(r2, dx * dx + dy * dy);
      }
      const float rh = __builtin_amdgcn_sqrtf(r2) * 1.0001f + 1e-6f;
      rho[o] = elig & (rh <= 0.5f) ? rh : -1.0f;
      unsafe[o] = 0u;
    }
    for (int p = tid; p < n * R; p += nthr) aenc[p] = 0x49742400u + 1u;  // enc(1e6f)
    for (int r = tid; r < R; r += nthr) {
      const float dx = ray_dirs[2 * r], dy = ray_dirs[2 * r + 1], l2 = dx * dx + dy * dy;
      rayc[r] = make_float4(dx, dy, l2, __builtin_amdgcn_sqrtf(l2) * 1.0001f);
    }
    if (tid == 0) *cnt = 0;
    __syncthreads();
    for (int q = tid; q < O * R; q += nthr) {
      const int o = q / R, r = q - (q / R) * R;
      const float4 rc = rayc[r];
      const float dx = rc.x, dy = rc.y;
      bool safe = (rho[o] >= 0.0f) & (rc.w <= 1.0f);
      for (int e = 0; e < 4; ++e) safe = safe & (fabsf(dy * evec[o * 8 + 2 * e] - dx * evec[o * 8 + 2 * e + 1]) >= 1e-3f);
      if (!safe) atomicOr(unsafe + o, 1u << r);
    }
    __syncthreads();
    const int tot = n * R * O;
    const int lane = tid & 63;
    // One-pass form (32 rays, every lane's (agent slot, obstacle) bits in one 64-bit mask): lane tid keeps ray
    // r = tid & 31 and its ray constants in registers and tests agents i = (tid >> 5) + (nthr / 32) it against every
    // obstacle; the survivors are compacted once by a workgroup prefix of the per-lane counts instead of one ballot +
    // LDS atomic per 64 triples.  The item order differs, the alphas do not (atomicMin per (agent, ray)).  When the
    // survivors exceed the list (adversarial inputs), the multi-round loop below runs instead.
    const int slots = nthr >> 5, its = (n + slots - 1) / slots;
    bool one_pass = R == 32 && (nthr & 31) == 0 && its * O <= 64 && nthr <= 1024;
    if (one_pass) {
      const int r = tid & 31, a0 = tid >> 5;
      const float4 rc = rayc[r];
      const float dx = rc.x, dy = rc.y, rlen2 = rc.z, rlen = rc.w;
      uint64_t bits = 0ull;
#pragma unroll 1
      for (int it = 0; it < its; ++it) {
        const int i = a0 + slots * it;
        const bool ai = i < n;
        const int ic = ai ? i : 0;
        const float sx = nxt[ic * SD + 0], sy = nxt[ic * SD + 1];
        const bool qok = (fabsf(sx) <= 2.0f) & (fabsf(sy) <= 2.0f);
#pragma unroll 1
        for (int o = 0; o < O; ++o) {
          const float vx = obst[o * DGPPO_OBST_FIELDS] - sx, vy = obst[o * DGPPO_OBST_FIELDS + 1] - sy;
          const float perp = vx * dy - vy * dx, proj = vx * dx + vy * dy;
          const float Rl = (rho[o] + 0.01f) * rlen;
          const bool miss = qok & ((fabsf(perp) > Rl) | (proj < -Rl) | (proj > rlen2 + Rl));
          const bool keep = ai & (!miss | ((unsafe[o] >> r) & 1u));
          bits |= (uint64_t)keep << (it * O + o);
        }
      }
      // workgroup exclusive prefix of the per-lane counts: 7 ballots per wave, then the waves' totals in LDS
      const int c = __popcll(bits);
      int pre = 0, wtot = 0;
#pragma unroll
      for (int b = 0; b < 7; ++b) {
        const uint64_t bb = __ballot((c >> b) & 1);
        pre += __builtin_amdgcn_mbcnt_hi((uint32_t)(bb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bb, 0u)) << b;
        wtot += __popcll(bb) << b;
      }
      int* wsum = cnt + 1;  // (the 3 ints after the counter; nthr / 64 <= 3 waves used here, else the wave totals
      const int wid = tid >> 6, nw = nthr >> 6;  //  go to the item list's tail, see below)
      int* wt = nw <= 3 ? wsum : items + cv.dist_n - nw;
      if (lane == 0) wt[wid] = wtot;
      __syncthreads();
      int base = 0, all = 0;
      for (int w = 0; w < nw; ++w) {
        const int v = wt[w];
        base += w < wid ? v : 0;
        all += v;
      }
      __syncthreads();  // every wave read the totals before any item (possibly over them) is written
      const int capw = cv.dist_n - (nw <= 3 ? 0 : nw);
      one_pass = all <= capw;
      if (one_pass) {
        int pos = base + pre;
        while (bits) {
          const int q = __builtin_ctzll(bits);
          bits &= bits - 1ull;
          const int it = q / O, o = q - it * O;
          items[pos++] = (o << 16) | ((a0 + slots * it) * R + r);
        }
        __syncthreads();
#pragma unroll 1
        for (int j = tid; j < all; j += nthr) {
          const int code = items[j], o = code >> 16, p = code & 0xFFFF, i = p / R, rr = p - (p / R) * R;
          const float sx = nxt[i * SD + 0], sy = nxt[i * SD + 1];
          const float4 rc2 = rayc[rr];
          const float ex = sx + rc2.x;
          const float ey = sy + rc2.y;
          const float a = rect_raytrace(obst + o * DGPPO_OBST_FIELDS, evec + o * 8, sx, sy, sx - ex, sy - ey);
          atomicMin(aenc + p, enc(a));
        }
        __syncthreads();
      }
    }
#pragma unroll 1
    for (int t0 = 0; t0 < (one_pass ? 0 : tot); t0 += cap) {
      const int t1 = t0 + cap < tot ? t0 + cap : tot;
#pragma unroll 1
      for (int tb = t0; tb < t1; tb += nthr) {  // uniform trip count: every wave joins the ballots
        const int t = tb + tid;
        const bool valid = t < t1;
        const int tt = valid ? t : t0;
        const int o = tt / (n * R), p = tt - o * (n * R), i = p / R, r = p - (p / R) * R;
        const float sx = nxt[i * SD + 0], sy = nxt[i * SD + 1];
        const float4 rc = rayc[r];
        const float dx = rc.x, dy = rc.y, rlen2 = rc.z, rlen = rc.w;
        const float vx = obst[o * DGPPO_OBST_FIELDS] - sx, vy = obst[o * DGPPO_OBST_FIELDS + 1] - sy;
        const float perp = vx * dy - vy * dx, proj = vx * dx + vy * dy;
        const float Rl = (rho[o] + 0.01f) * rlen;
        const bool qok = (fabsf(sx) <= 2.0f) & (fabsf(sy) <= 2.0f);
        const bool miss = qok & ((fabsf(perp) > Rl) | (proj < -Rl) | (proj > rlen2 + Rl));
        const bool keep = valid & (!miss | ((unsafe[o] >> r) & 1u));
        const uint64_t kb = __ballot(keep);
        int base = 0;
        if (lane == 0 && kb) base = atomicAdd(cnt, (int)__popcll(kb));
        base = __shfl(base, 0);
        if (keep) {
          const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(kb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)kb, 0u));
          items[base + below] = (o << 16) | p;
        }
      }
      __syncthreads();
      const int m = *cnt;
#pragma unroll 1
      for (int j = tid; j < m; j += nthr) {
        const int code = items[j], o = code >> 16, p = code & 0xFFFF, i = p / R, r = p - (p / R) * R;
        const float sx = nxt[i * SD + 0], sy = nxt[i * SD + 1];
        const float4 rc = rayc[r];
        const float ex = sx + rc.x;
        const float ey = sy + rc.y;
        const float a = rect_raytrace(obst + o * DGPPO_OBST_FIELDS, evec + o * 8, sx, sy, sx - ex, sy - ey);
        atomicMin(aenc + p, enc(a));
      }
      __syncthreads();
      if (tid == 0) *cnt = 0;
      __syncthreads();
    }
#pragma unroll 1
    for (int p = tid; p < n * R; p += nthr) {
      const int i = p / R, r = p - (p / R) * R;
      const float sx = nxt[i * SD + 0], sy = nxt[i * SD + 1];
      const float4 rc = rayc[r];
      const float ex = sx + rc.x;
      const float ey = sy + rc.y;
      const uint32_t e = aenc[p];
      float a = e == 0u ? __builtin_nanf("") : __uint_as_float(e - 1u);
      a = a * (1.0f - lds[cv.isin + i]);
      keys[p] = sort_key(a, r);
      hpt[2 * p + 0] = sx + (ex - sx) * a;
      hpt[2 * p + 1] = sy + (ey - sy) * a;
    }
  } else {
#pragma unroll 1
  for (int p = tid; p < n * R; p += nthr) {
    asm volatile("" ::: "memory");  // keep obstacle LDS reads inside the loop (no LICM register blow-up)
    const int i = p / R, r = p - (p / R) * R;
    const float sx = nxt[i * SD + 0], sy = nxt[i * SD + 1];
    const float ex = sx + ray_dirs[2 * r + 0];
    const float ey = sy + ray_dirs[2 * r + 1];
    const float ax = sx - ex, ay = sy - ey;
    float a = 0.0f;
    for (int o = 0; o < O; ++o) {
      const float ao = rect_raytrace(obst + o * DGPPO_OBST_FIELDS, evec + o * 8, sx, sy, ax, ay);
      a = o == 0 ? ao : min_nan(a, ao);
    }
    a = a * (1.0f - lds[cv.isin + i]);
    keys[p] = sort_key(a, r);
    hpt[2 * p + 0] = sx + (ex - sx) * a;
    hpt[2 * p + 1] = sy + (ey - sy) * a;
  }
  }
  __syncthreads();
  float* hits = lds + cv.hits;
#pragma unroll 1
  for (int p = tid; p < n * R; p += nthr) {
    const int i = p / R;
    const uint64_t key = keys[p];
    const uint64_t* row = keys + i * R;
    int rank = 0;
#pragma unroll 8
    for (int j = 0; j < R; ++j) rank += row[j] < key ? 1 : 0;
    if (rank < k) {
      hits[(i * k + rank) * 2 + 0] = hpt[2 * p + 0];
      hits[(i * k + rank) * 2 + 1] = hpt[2 * p + 1];
    }
  }
}

// per-obstacle edge vectors (x4 - x3, y4 - y3) of Rectangle.raytracing, e -> points[e-1] - points[e]
__device__ __forceinline__ void stage_edge_vectors(int O, float* lds, const Carve& cv, int tid, int nthr) {
  for (int q = tid; q < O * 8; q += nthr) {
    const int o = q >> 3, e = (q >> 1) & 3, c = q & 1;
    const float* rec = lds + cv.obst + o * DGPPO_OBST_FIELDS;
    const int e4 = (e + 3) & 3;
    lds[cv.evec + q] = rec[8 + 2 * e4 + c] - rec[8 + 2 * e + c];
  }
}

__device__ __forceinline__ void agent_is_inside(int O, float* lds, const Carve& cv, int SD, int i) {
  const float* obst = lds + cv.obst;
  const float px = lds[cv.nxt + i * SD + 0], py = lds[cv.nxt + i * SD + 1];
  bool in = false;
  for (int o = 0; o < O; ++o) in = in || rect_inside(obst + o * DGPPO_OBST_FIELDS, px, py, 0.0f);
  lds[cv.isin + i] = in ? 1.0f : 0.0f;
}

#ifdef DGPPO_ENV_STAMPS
// diagnostic builds: wave 0's barrier-to-barrier phase times of the workgroup-per-env step kernel
__device__ unsigned long long g_blk_stamps[8];
#define BLK_STAMP(k)                                      \
  do {                                                    \
    const uint64_t now_ = __builtin_amdgcn_s_memtime();   \
    bst[k] += now_ - blast;                               \
    blast = now_;                                         \
  } while (0)
#else
#define BLK_STAMP(k) \
  do {               \
  } while (0)
#endif

// ---- the step kernel --------------------------------------------------------------------------
// Phases (one barrier each), every phase spread over the whole workgroup:
//   A  stage current rows, obstacles, clipped actions in LDS
//   B  task list: per-agent dynamics + |a|^2, and one pairwise distance per lane (agent-agent,
//      goal-agent, agent-hit / agent-obstacle) on the pre-step graph
//   C  per-agent row minima -> cost and reward terms; is-inside on the next state
//   D  reward/cost stores, ray cast of the next state (keys + hit points), stable rank -> top-k
//   E  stream the next graph out
// One env step of one workgroup's env.  LOAD: the current graph's rows come from io.states (and the
// obstacles from io.obstacles); otherwise they are already in LDS (the persistent rollout below carries the
// previous step's next rows over, bit-identical to re-reading what that step wrote).
template <int ENGINE, int GOAL, int SD, int BLOCK, int NA, int NO, int NR, int NK, bool LOAD, bool ACT_LDS = false>
__device__ __forceinline__ void block_step(const dgppo_env_cfg& cfg, const dgppo_env_step_io& io, float* lds,
                                           int64_t env) {
  constexpr bool mpe = ENGINE == DGPPO_ENGINE_MPE;
  const Dims<NA, NO, NR, NK> d(cfg);
  const int n = d.n, O = d.O, k = d.k;
  const bool lidar = !mpe && O > 0;
  const Carve cv(n, SD, O, d.R, k, !mpe);
  const int tid = threadIdx.x;
#ifdef DGPPO_ENV_STAMPS
  uint64_t bst[5] = {0, 0, 0, 0, 0}, blast = __builtin_amdgcn_s_memtime();
#endif

  // ---- A ------------------------------------------------------------------------------------
  if (LOAD) {
    const float* st = io.states + env * io.states_stride;
    const int n_cur = (2 * n + (mpe ? O : 0)) * SD;  // type_states(0), (1) [, (2) for MPE]
    for (int idx = tid; idx < n_cur; idx += BLOCK) lds[cv.cur + idx] = st[idx];
    if (lidar) {
      for (int idx = tid; idx < n * k * 2; idx += BLOCK) {  // type_states(2)[:, :2] = current hits
        const int h = idx >> 1, c = idx & 1;
        lds[cv.curhit + idx] = st[(2 * n + h) * SD + c];
      }
      const float* ob = io.obstacles + env * io.obstacles_stride;
      for (int idx = tid; idx < O * DGPPO_OBST_FIELDS; idx += BLOCK) lds[cv.obst + idx] = ob[idx];
    }
  }
  if (!ACT_LDS) {  // (ACT_LDS: the caller staged the clipped actions in LDS)
    const float* ac = io.action + env * io.action_stride;
    for (int idx = tid; idx < 2 * n; idx += BLOCK) lds[cv.act + idx] = clampf_nan(ac[idx], -1.0f, 1.0f);
  }
  __syncthreads();
  BLK_STAMP(0);

  // ---- B ------------------------------------------------------------------------------------
  const float* cur = lds + cv.cur;
  const float* goal = lds + cv.cur + n * SD;
  float* dist = lds + cv.dist;
  const int n_aa = n * n;
  const int n_ga = GOAL == DGPPO_GOAL_SPREAD ? n * n : n;
  const int n_t3 = lidar ? n * k : (mpe ? n * O : 0);
  const int n_task = n + n_aa + n_ga + n_t3;
  const bool bf = mpe && n_task <= BLOCK;  // the branch-free MPE form (one pass)
  if (bf) mpe_tasks<GOAL, SD>(cfg, lds, cv, n, O, tid);
#pragma unroll 1
  for (int q = bf ? n_task : tid; q < n_task; q += BLOCK) {
    if (q < n) {  // dynamics (lidar_env/base.py:142-149 / bicycle 92-111), then clip_state
      const int i = q;
      const float* x = cur + i * SD;
      const float* a = lds + cv.act + 2 * i;
      float y[SD];
      if (ENGINE == DGPPO_ENGINE_BICYCLE) {
        const float theta = atan2_32(x[3], x[2]);
        const float theta_next = theta + ((x[4] * a[0]) * cfg.dt) * 10.0f;
        float st_, ct_, sn_, cn_;
        sincos32(theta, &st_, &ct_);
        sincos32(theta_next, &sn_, &cn_);
        y[0] = x[0] + (x[4] * ct_) * cfg.dt;
        y[1] = x[1] + (x[4] * st_) * cfg.dt;
        y[2] = cn_;
        y[3] = sn_;
        y[4] = x[4] + (a[1] * cfg.dt) * 10.0f;
      } else {
        y[0] = x[2] * cfg.dt + x[0];
        y[1] = x[3] * cfg.dt + x[1];
        y[2] = (a[0] * 10.0f) * cfg.dt + x[2];
        y[3] = (a[1] * 10.0f) * cfg.dt + x[3];
      }
#pragma unroll
      for (int c = 0; c < SD; ++c) lds[cv.nxt + i * SD + c] = clampf_nan(y[c], cfg.state_lo[c], cfg.state_hi[c]);
      const float an = norm2(a[0], a[1]);
      lds[cv.red + 2 * n + i] = an * an;
      continue;
    }
    int t = q - n;
    if (t < n_aa) {  // agent-agent distance with the eye * 1e6 diagonal (lidar_env/base.py:185-187)
      const int i = t / n, j = t - (t / n) * n;
      float dj = norm2(cur[i * SD] - cur[j * SD], cur[i * SD + 1] - cur[j * SD + 1]);
      if (i == j) dj = dj + 1e6f;
      dist[t] = dj;
      continue;
    }
    t -= n_aa;
    if (t < n_ga) {  // goal j to agent i (spread, goal-major) or own goal (target)
      int gj, ai;
      if (GOAL == DGPPO_GOAL_SPREAD) {
        gj = t / n;
        ai = t - gj * n;
      } else {
        gj = t;
        ai = t;
      }
      dist[n_aa + t] = norm2(goal[gj * SD] - cur[ai * SD], goal[gj * SD + 1] - cur[ai * SD + 1]);
      continue;
    }
    t -= n_ga;
    if (lidar) {  // current hit h of agent i: ||hit - p_i|| (lidar_env/base.py:194-197)
      const int i = t / k;
      const float* hc = lds + cv.curhit + 2 * t;
      dist[2 * n_aa + t] = norm2(hc[0] - cur[i * SD], hc[1] - cur[i * SD + 1]);
    } else {  // MPE: ||p_i - o|| (mpe/base.py:179-181)
      const int i = t / O, o = t - (t / O) * O;
      const float* ob = cur + 2 * n * SD + o * SD;
      dist[2 * n_aa + t] = norm2(cur[i * SD] - ob[0], cur[i * SD + 1] - ob[1]);
    }
  }
  if (lidar) stage_edge_vectors(O, lds, cv, tid, BLOCK);
  __syncthreads();
  BLK_STAMP(1);

  // ---- C ------------------------------------------------------------------------------------
  for (int i = tid; i < n; i += BLOCK) {
    float md = dist[i * n];
    for (int j = 1; j < n; ++j) md = min_nan(md, dist[i * n + j]);
    float dg;
    if (GOAL == DGPPO_GOAL_SPREAD) {  // goal i's nearest agent
      dg = dist[n_aa + i * n];
      for (int j = 1; j < n; ++j) dg = min_nan(dg, dist[n_aa + i * n + j]);
    } else {
      dg = dist[n_aa + i];
    }
    lds[cv.red + i] = dg;
    lds[cv.red + n + i] = dg > cfg.dist2goal ? 1.0f : 0.0f;
    float c0 = cfg.c_agent_cost - md;
    float c1 = 0.0f;
    const int m3 = lidar ? k : (mpe ? O : 0);
    if (m3 > 0) {
      const float* row = dist + 2 * n_aa + i * m3;
      float mo = row[0];
      for (int h = 1; h < m3; ++h) mo = min_nan(mo, row[h]);
      c1 = cfg.c_obs_cost - mo;
    }
    c0 = c0 <= 0.0f ? c0 - 0.5f : c0 + 0.5f;
    c1 = c1 <= 0.0f ? c1 - 0.5f : c1 + 0.5f;
    if (mpe) {  // jnp.clip(cost, a_min=-1.0)
      c0 = c0 < -1.0f ? -1.0f : c0;
      c1 = c1 < -1.0f ? -1.0f : c1;
    } else {
      c0 = clampf_nan(c0, -1.0f, 1.0f);
      c1 = clampf_nan(c1, -1.0f, 1.0f);
    }
    lds[cv.red + 3 * n + i] = c0;
    lds[cv.red + 4 * n + i] = c1;
    if (lidar) agent_is_inside(O, lds, cv, SD, i);
  }
  __syncthreads();
  BLK_STAMP(2);

  // ---- D ------------------------------------------------------------------------------------
  if (tid == 0) {
    float sd_ = 0.0f, sf = 0.0f, sa = 0.0f;
    for (int i = 0; i < n; ++i) {
      sd_ = sd_ + lds[cv.red + i];
      sf = sf + lds[cv.red + n + i];
      sa = sa + lds[cv.red + 2 * n + i];
    }
    const float nn = (float)n;
    float r = 0.0f - (sd_ / nn) * 0.01f;
    r = r - (sf / nn) * 0.001f;
    r = r - (sa / nn) * 0.0001f;
    io.reward[env * io.reward_stride] = r;
  }
  for (int idx = tid; idx < 2 * n; idx += BLOCK) {
    const int i = idx >> 1, h = idx & 1;
    io.cost[env * io.cost_stride + idx] = lds[cv.red + (3 + h) * n + i];
  }
  if (lidar) {
    lidar_scan<SD>(d, io.ray_dirs, lds, cv, tid, BLOCK);
    __syncthreads();
  }
  BLK_STAMP(3);

  // ---- E ------------------------------------------------------------------------------------
  GraphOut out;
  out.nodes = io.nodes + env * io.nodes_stride;
  out.edges = io.edges + env * io.edges_stride;
  out.states = io.out_states + env * io.out_states_stride;
  out.recv = io.receivers + env * io.edge_index_stride;
  out.send = io.senders + env * io.edge_index_stride;
  const bool vec4 = ((io.edges_stride & 3) == 0) && ((reinterpret_cast<uintptr_t>(io.edges) & 15) == 0);
  const float* third = mpe ? cur + 2 * n * SD : lds + cv.hits;
  if constexpr (mpe) write_graph_mpe<GOAL, SD>(cfg, d, lds + cv.nxt, goal, third, out, vec4, tid, BLOCK);
  else write_graph<ENGINE, GOAL, SD>(cfg, d, lds + cv.nxt, goal, third, out, vec4, tid, BLOCK);
  BLK_STAMP(4);
#ifdef DGPPO_ENV_STAMPS
  if (tid == 0)
    for (int q = 0; q < 5; ++q) atomicAdd(&g_blk_stamps[q], (unsigned long long)bst[q]);
#endif
}

template <int ENGINE, int GOAL, int SD, int BLOCK, int NA, int NO, int NR, int NK>
__global__ __launch_bounds__(BLOCK) void env_step_kernel(dgppo_env_cfg cfg, dgppo_env_step_io io) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  block_step<ENGINE, GOAL, SD, BLOCK, NA, NO, NR, NK, true>(cfg, io, lds, blockIdx.x);
}

// Persistent rollout of the workgroup-per-env kernel (dgppo_env_rollout for every shape the wave kernels do
// not take: MPE, Lidar n = 32 / 8 obstacles, other sizes): one launch runs all T steps of one env per
// workgroup, step t reading graph t's rows from LDS (graph 0 from HBM) and writing graph t + 1 into the
// time-major (T + 1) buffers, reward[t], cost[t] -- the same arithmetic as T per-step launches, without their
// launch floor and their re-reads of every graph.
// (n = 32: at most 128 VGPRs, so the 1024 envs of BASELINE config 5's share are resident in one round, 4 per CU)
template <int ENGINE, int GOAL, int SD, int BLOCK, int NA, int NO, int NR, int NK>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(NA == 32 ? 4 : 1, 8))) void env_rollout_block_kernel(dgppo_env_cfg cfg, dgppo_env_rollout_io r,
                                                                   int stage_acts) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr bool mpe = ENGINE == DGPPO_ENGINE_MPE;
  const Dims<NA, NO, NR, NK> d(cfg);
  const int n = d.n, O = d.O, k = d.k;
  const bool lidar = !mpe && O > 0;
  const Carve cv(n, SD, O, d.R, k, !mpe);
  const int64_t env = blockIdx.x;
  // step t + 1's actions are requested before step t's graph stores: vmcnt counts stores too, so a load
  // issued after them would wait for the whole store drain of the previous step (one HBM round trip per step)
  static_assert(BLOCK >= 64, "2 n <= 64 actions per step, one per thread");
  const int na = 2 * n;
  const float* act0 = r.step.action + env * r.step.action_stride;
  // Small episodes (T * 2n <= kActStage floats, e.g. MPE): every step's clipped actions are staged in LDS once, so
  // the step loop issues no global load at all.  A per-step action load would be waited for with vmcnt(0) at the
  // next step (the graph writer's store count is not static), i.e. behind the whole previous step's store drain.
  // The host decides (stage_acts) and sized the dynamic LDS for it: the two can never disagree.
  const bool stage = stage_acts != 0;
  float* acts = lds + cv.total;
  if (stage) {
    for (int idx = threadIdx.x; idx < r.T * na; idx += BLOCK) {
      const int t = idx / na, j = idx - t * na;
      acts[idx] = clampf_nan(act0[(int64_t)t * r.t_action + j], -1.0f, 1.0f);
    }
    __syncthreads();
  }
  float a_nxt = (!stage && threadIdx.x < na) ? act0[threadIdx.x] : 0.0f;
#pragma unroll 1
  for (int t = 0; t < r.T; ++t) {
    if (threadIdx.x < na) lds[cv.act + threadIdx.x] = stage ? acts[t * na + threadIdx.x] : clampf_nan(a_nxt, -1.0f, 1.0f);
    if (!stage && t + 1 < r.T && threadIdx.x < na) a_nxt = act0[(t + 1) * r.t_action + threadIdx.x];
    dgppo_env_step_io q = r.step;
    q.states = r.step.out_states + t * r.t_states;
    q.action = r.step.action + t * r.t_action;
    q.nodes = r.step.nodes + (t + 1) * r.t_nodes;
    q.edges = r.step.edges + (t + 1) * r.t_edges;
    q.out_states = r.step.out_states + (t + 1) * r.t_states;
    q.receivers = r.step.receivers + (t + 1) * r.t_index;
    q.senders = r.step.senders + (t + 1) * r.t_index;
    q.reward = r.step.reward + t * r.t_reward;
    q.cost = r.step.cost + t * r.t_cost;
    if (t == 0) block_step<ENGINE, GOAL, SD, BLOCK, NA, NO, NR, NK, true, true>(cfg, q, lds, env);
    else block_step<ENGINE, GOAL, SD, BLOCK, NA, NO, NR, NK, false, true>(cfg, q, lds, env);
    __syncthreads();
    // graph t + 1 becomes the current graph: agent rows <- next rows, current hits <- next hits
    for (int idx = threadIdx.x; idx < n * SD; idx += BLOCK) lds[cv.cur + idx] = lds[cv.nxt + idx];
    if (lidar)
      for (int idx = threadIdx.x; idx < n * k * 2; idx += BLOCK) lds[cv.curhit + idx] = lds[cv.hits + idx];
    __syncthreads();
  }
}

// Rectangle.inside with r = 0 (raytracing's is_in): the rounded-corner term sqrt(.) < 0 never holds
__device__ __forceinline__ bool rect_inside0(const float* rec, float px, float py) {
  const float rel_x = px - rec[0];
  const float rel_y = py - rec[1];
  const float c = rec[5], s = rec[6];
  const float rel_xx = fabsf(rel_x * c + rel_y * s) - rec[2] / 2.0f;
  const float rel_yy = fabsf(rel_x * s - rel_y * c) - rec[3] / 2.0f;
  return (rel_xx < 0.0f) & (rel_yy < 0.0f);
}

// ---- wave-per-env Lidar step (n = 8 agents, R = 32 rays, top-k = 8) ----------------------------
// The BASELINE Lidar configs (LidarSpread / LidarTarget / LidarBicycleTarget, n = 8): one 64-lane
// wave owns one environment end to end, so no phase needs a workgroup barrier (LDS hand-offs
// between the lanes of one wave only need wave_sync) and 4096 envs are resident at once (16 waves
// per CU).  Lane l maps to the pair (i = l / 8, j = l % 8): the 64 agent-agent, 64 goal-agent and
// 64 agent-hit distances are one value per lane, row minima are 3 DPP steps, and each lane owns
// 4 of its agent's 32 rays (r = 4 (l % 8) + q) for the sort.
//
// Exact ray culling.  Rectangle.raytracing of a (ray, obstacle) pair is exactly 1e6 in the
// reference whenever no edge can be valid and no alpha is NaN.  A triple (agent, obstacle, ray) is
// skipped (left at 1e6) only when all of the following hold, evaluated with NaN-false comparisons:
//   * the obstacle is "eligible": its 4 corners lie in [-2, 2]^2 and its circumradius rho <= 0.5;
//     the agent position lies in [-2, 2]^2 and the ray vector |d| <= 1;
//   * for all 4 edges the IDEAL determinant |d_y e_x - d_x e_y| >= kDetMin = 1e-3 (the computed
//     det then differs by < 5e-7, so no clipping, no det == 0, no NaN);
//   * the segment S -> S + d misses the disc (c, rho + kCullMargin), kCullMargin = 0.01 (capsule test).
// With every coordinate in [-2, 2] the numerators carry < 1.4e-6 (na) / 2.4e-6 (nb) absolute error,
// so computed alpha / beta differ from the exact line parameters by < 2e-3 / 3e-3 near [0, 1]:
// alpha, beta in [0, 1] would put the two segments within 2e-3 |d| + 3e-3 |e| <= 5e-3 < kCullMargin
// of each other.  Every skipped triple is therefore provably the reference's 1e6.  All other triples
// (~65 of 768 per env at the bench distribution) go to a compacted work list, pooled over the 4 envs
// of a workgroup, and run the exact per-edge arithmetic (raytrace_nodiv / rect_raytrace), combined
// per ray with an LDS atomic min on an order-preserving encoding (NaN wins, as jnp.min).
#pragma clang diagnostic ignored "-Wbitwise-instead-of-logical"  // branch-free predicates on purpose
constexpr int kOmniSD = 7, kOmniED = 10, kOmniNC = 5;  // LidarOmniTarget state / edge width, costs
// 16-byte state rows (SD = 4) stored one float4 per lane instead of one dword per lane and column (A/B builds:
// -DDGPPO_ENV_ST4=0 restores the dword stores)
#ifndef DGPPO_ENV_ST4
#define DGPPO_ENV_ST4 1
#endif
// hit ranks of the non-miss rays against their row's compacted non-miss keys (-DDGPPO_ENV_CRANK=1) instead of all
// 32 keys: 100 fewer instructions per step, but the runtime-bounded loop waits for each key load (the unrolled
// 32-key loop has all 16 in flight) -- LidarSpread episode 1.34 vs 1.25-1.27 ms, so off by default
#ifndef DGPPO_ENV_CRANK
#define DGPPO_ENV_CRANK 0
#endif
// the persistent rollout's env index wave-uniform for the bicycle engine (-DDGPPO_ENV_UNI=0: per-lane everywhere, the
// round-5 form; =2: uniform for every engine).  Episode A/B (4096 envs, same box, 3 runs each): bicycle 1.306-1.316
// vs 1.341-1.352 ms uniform vs per-lane; LidarSpread 1.249-1.269 vs 1.240-1.255 and Omni 1.926-1.945 vs
// 1.889-1.894, so only the bicycle engine takes it
#ifndef DGPPO_ENV_UNI
#define DGPPO_ENV_UNI 1
#endif

namespace wv {
constexpr int NA = 8, NR = 32, NK = 8;
constexpr float kCullMargin = 0.01f;
constexpr float kDetMin = 1e-3f;
constexpr uint32_t kEncMiss = 0x49742400u + 1u;  // enc(1e6f)

// order-preserving encoding of a ray's alpha (>= +0, 1e6 or NaN) for an LDS atomic min; NaN wins
__device__ __forceinline__ uint32_t enc_alpha(float a) { return a != a ? 0u : __float_as_uint(a) + 1u; }
__device__ __forceinline__ float dec_alpha(uint32_t e) {
  return e == 0u ? __builtin_nanf("") : __uint_as_float(e - 1u);
}
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float rlf(float v, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
// minimum over each 8-lane group of values that are >= +0 or NaN (norms and squared norms): quad xor 1, xor 2,
// row_half_mirror.  v_minimum3_f32 (IEEE minimum: NaN-propagating) equals min_nan on such values but for the NaN
// payload; every lane of the three patterns reads a valid lane, so the moves need no old-value initialisation
template <int CTRL>
__device__ __forceinline__ float dppb(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xf, 0xf, true));
}
__device__ __forceinline__ float min8(float v) {
  v = __builtin_elementwise_minimum(v, dppb<0xB1>(v));
  v = __builtin_elementwise_minimum(v, dppb<0x4E>(v));
  return __builtin_elementwise_minimum(v, dppb<0x141>(v));
}
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ int mbcnt(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Rectangle.raytracing (env/obstacle.py:74-105) of one ray against one obstacle WITHOUT the two
// per-edge divisions, bit-identical to the reference.  With detc = sign(det) clip(|det|, 1e-7, 1e7)
// = +-cl and na' = sign(det) na, nb' = sign(det) nb (exact sign flips):
//   fl(na / detc) >= 0  <=>  na' >= 0     (unless 0 < |na'| < 1e-30: a tiny negative could round to -0)
//   fl(na / detc) <= 1  <=>  na' <= cl    (round-to-nearest: fl(x) <= 1 <=> x <= 1 + 2^-24, and the
//                                          float after cl exceeds cl (1 + 2^-24))
// so validity needs no quotient.  The smallest valid alpha is picked by exact-order cross products
// (fl(a c) < fl(b d) implies a/d <= b/c, and fl of the quotient is monotone), and divided once.
// NaN: the reference's alpha is NaN iff det == 0 / NaN or na is NaN (0 * inf, NaN propagation).
// Returns false for the cases this does not decide (denormal or > 1e30 numerators, tied cross
// products); the caller then runs the literal per-edge code (rect_raytrace).
__device__ __forceinline__ bool raytrace_nodiv(const float4 pA, const float4 pB, const float4 eA, const float4 eB,
                                               float x1, float y1, float ax, float ay, float* out) {
  const float px3[4] = {pA.x, pA.z, pB.x, pB.z}, py3[4] = {pA.y, pA.w, pB.y, pB.w};
  const float ex[4] = {eA.x, eA.z, eB.x, eB.z}, ey[4] = {eA.y, eA.w, eB.y, eB.w};
  float bn = 0.0f, bc = 1.0f;
  bool has = false, nan = false, weird = false;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float px = x1 - px3[e], py = y1 - py3[e];
    const float det = ax * ey[e] - ay * ex[e];
    const float na = ey[e] * px - ex[e] * py;
    const float nb = (-ay) * px + ax * py;
    const float adet = fabsf(det);
    nan = nan | !(adet > 0.0f) | (na != na);
    const float cl = fminf(fmaxf(adet, 1e-7f), 1e7f);
    const bool neg = det < 0.0f;
    const float nap = neg ? -na : na, nbp = neg ? -nb : nb;
    const float ana = fabsf(na), anb = fabsf(nb);
    weird = weird | (ana > 1e30f) | ((ana < 1e-30f) & (ana != 0.0f)) | ((anb < 1e-30f) & (anb != 0.0f));
    const bool valid = (nap >= 0.0f) & (nap <= cl) & (nbp >= 0.0f) & (nbp <= cl);
    const float p1 = nap * bc, p2 = bn * cl;
    weird = weird | (valid & has & (p1 == p2));
    const bool better = valid & (!has | (p1 < p2));
    bn = better ? nap : bn;
    bc = better ? cl : bc;
    has = has | valid;
  }
  *out = nan ? __builtin_nanf("") : (has ? bn / bc + 0.0f : 1e6f);
  return !weird;
}

// per-wave LDS carve (floats); every region 16-byte aligned
template <int SD, int O>
struct Carve {
  static constexpr int N = 2 * NA + NA * NK + 1;
  static constexpr int ND = SD + 3;
  static constexpr int cur = 0;  // agents (8 SD) then goals (8 SD)
  static constexpr int nxt = cur + 16 * SD;
  static constexpr int obst = nxt + ((NA * SD + 3) & ~3);
  static constexpr int evec = obst + O * DGPPO_OBST_FIELDS;
  static constexpr int rays = evec + O * 8;
  static constexpr int alpha = rays + 2 * NR;  // (8, 32) encoded alphas (uint32)
  static constexpr int hits = alpha + NA * NR;  // (8, 8, 2)
  static constexpr int olist = hits + NA * NK * 2;  // compacted non-miss rays
  static constexpr int uni = olist + NA * NR;  // union: items | keys
  static constexpr int key_stride = 2 * NR + 4;  // dwords per agent row of 64-bit keys (bank-padded)
  static constexpr int n_items = NA * O * NR;
  static constexpr int uni_size = n_items + 64 > NA * key_stride ? n_items + 64 : NA * key_stride;
  static_assert(rays - obst >= 64, "the 64-lane obstacle staging store stays below the ray table");
  static constexpr int total = (uni + uni_size + 3) & ~3;
};

// One env step of the wave-per-env kernel for this wave's env (the 4 waves of a workgroup pool their
// ray casts, so all four call it together).  REBUILD: the graph of the given states (reset: y = x, no
// reward / cost), else one env step.  LOAD: read the current agent / goal rows, current hits,
// obstacles and ray table from HBM (io.states / io.obstacles / io.ray_dirs); otherwise they are the
// LDS state the previous call left (persistent rollout: next agent rows and next hits become current,
// obstacles and rays stay staged), and only the action comes from HBM.
// Phase timers of the persistent rollout (diagnostic builds only: -DDGPPO_ENV_STAMPS, `make stamps`):
// s_memtime deltas per phase summed over the steps of each wave, added into g_env_stamps at the end.
#ifdef DGPPO_ENV_STAMPS
struct EnvStamps {
  uint64_t last, acc[16];
};
__device__ unsigned long long g_env_stamps[16];
#define ENV_STAMP(k)                                             \
  do {                                                           \
    if (stamps) {                                                \
      const uint64_t now_ = __builtin_amdgcn_s_memtime();        \
      stamps->acc[k] += now_ - stamps->last;                     \
      stamps->last = now_;                                       \
    }                                                            \
  } while (0)
#else
struct EnvStamps {};
#define ENV_STAMP(k) \
  do {               \
  } while (0)
#endif

// Culling data that depends only on the obstacles and the ray table (constant over an episode): the
// persistent rollout computes it once, the per-step kernel every call.  Lane l: ray rr = l & 31.
template <int O>
struct WaveConst {
  float rdx, rdy, rlen2, rlen, rho_l;  // ray rr, |ray|^2, |ray| bound, circumradius bound of obstacle l (< O)
  uint64_t elig_mask;                  // obstacles eligible for culling
  uint32_t unsafe[O];                  // rays whose determinant against an edge of obstacle o is near 0
};

template <int O>
__device__ __forceinline__ WaveConst<O> wave_const(const float* obst, const float* evec, const float* rays, int lane) {
  WaveConst<O> k;
  const int rr = lane & 31;
  k.rdx = rays[2 * rr], k.rdy = rays[2 * rr + 1];
  k.rlen2 = k.rdx * k.rdx + k.rdy * k.rdy;
  // obstacle o = lane (< O): circumradius (raw v_sqrt: the culling bounds carry margins) and eligibility
  {
    const int o = lane < O ? lane : 0;
    const float4* rec4 = reinterpret_cast<const float4*>(obst + o * DGPPO_OBST_FIELDS);
    const float4 c4 = rec4[0], pA = rec4[2], pB = rec4[3];
    const float pxs[4] = {pA.x, pA.z, pB.x, pB.z}, pys[4] = {pA.y, pA.w, pB.y, pB.w};
    float r2 = 0.0f;
    bool elig = (fabsf(c4.x) <= 2.0f) & (fabsf(c4.y) <= 2.0f);
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      elig = elig & (fabsf(pxs[p]) <= 2.0f) & (fabsf(pys[p]) <= 2.0f);
      const float dx = pxs[p] - c4.x, dy = pys[p] - c4.y;
      r2 = fmaxf(r2, dx * dx + dy * dy);
    }
    k.rho_l = __builtin_amdgcn_sqrtf(r2) * 1.0001f + 1e-6f;
    elig = elig & (k.rho_l <= 0.5f);
    k.elig_mask = __ballot(elig & (lane < O));
  }
  k.rlen = __builtin_amdgcn_sqrtf(k.rlen2) * 1.0001f;
#pragma unroll
  for (int pass = 0; pass < (O + 1) / 2; ++pass) {  // (obstacle 2 pass + half, ray lane & 31)
    const int o = 2 * pass + (lane >> 5) < O ? 2 * pass + (lane >> 5) : 0;
    const float4* e4 = reinterpret_cast<const float4*>(evec + o * 8);
    const float4 eA = e4[0], eB = e4[1];
    const float exs[4] = {eA.x, eA.z, eB.x, eB.z}, eys[4] = {eA.y, eA.w, eB.y, eB.w};
    bool safe = (((k.elig_mask >> o) & 1ull) != 0ull) & (k.rlen <= 1.0f);
#pragma unroll
    for (int e = 0; e < 4; ++e) safe = safe & (fabsf(k.rdy * exs[e] - k.rdx * eys[e]) >= kDetMin);
    const uint64_t b = __ballot(!safe);
    k.unsafe[2 * pass] = (uint32_t)b;
    if (2 * pass + 1 < O) k.unsafe[2 * pass + 1] = (uint32_t)(b >> 32);
  }
  return k;
}

// raw (unclamped) action components of lane gj of this wave's env: (a0, a1, the omni alpha or 0)
template <int AD>
__device__ __forceinline__ float3 wave_action(const dgppo_env_step_io& io, int64_t env, int gj) {
  const float* ac = io.action + env * io.action_stride;
  return make_float3(ac[AD * gj + 0], ac[AD * gj + 1], AD == 3 ? ac[AD * gj + AD - 1] : 0.0f);
}

// (pre: LOAD = false only — this step's raw actions, loaded by the caller one step ahead)
template <int ENGINE, int GOAL, int SD, int O, bool REBUILD, bool LOAD, int WPG = 4>
__device__ __forceinline__ void wave_body(const dgppo_env_cfg& cfg, const dgppo_env_step_io& io, float* smem,
                                          int* wg_items, float3 pre = make_float3(0.0f, 0.0f, 0.0f),
                                          EnvStamps* stamps = nullptr, const WaveConst<O>* pc = nullptr) {
  (void)stamps;
  static_assert(O >= 1 && O <= 4, "obstacle records are staged by one load per lane");
  // LidarOmniTarget (SD 7, own goals): omni dynamics, 5 costs, 10-wide edges; same LiDAR and graph rows
  constexpr bool OMNI = ENGINE == DGPPO_ENGINE_OMNI;
  static_assert(!OMNI || (SD == 7 && GOAL == DGPPO_GOAL_TARGET), "LidarOmniTarget layout");
  constexpr int AD = OMNI ? 3 : 2;   // action width
  constexpr int ED = OMNI ? 10 : 4;  // edge width
  constexpr int XS = 16 * SD - 64;   // agent + goal state floats past the first 64
  constexpr bool ST4 = SD == 4 && DGPPO_ENV_ST4;  // state rows stored as one float4 per lane
  using C = Carve<SD, O>;
  constexpr int N = C::N, ND = C::ND, pad = N - 1;
  constexpr int n_ag = GOAL == DGPPO_GOAL_SPREAD ? NA * NA : NA;
  int tid = threadIdx.x;
  // persistent loop: an opaque thread id per step keeps the per-lane addressing inside the loop (hoisted,
  // it costs ~80 VGPRs and a wave per SIMD of occupancy)
  if constexpr (!LOAD) asm volatile("" : "+v"(tid));
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid) >> 6;
  const int64_t env_raw = (int64_t)blockIdx.x * WPG + wid;
  // a wave past the last env replays the last env without storing anything: it must still join
  // the two workgroup barriers around the pooled ray cast
  const bool live = env_raw < io.n_env;
  const int64_t env = live ? env_raw : io.n_env - 1;
#ifdef DGPPO_DIAG_NOSTORE
  const bool st_live = false;  // diagnostic build: every graph / reward / cost store dropped
#else
  const bool st_live = live;
#endif
  float* lds = smem + wid * C::total;
  const int gi = lane >> 3, gj = lane & 7;

  // ---- A: every global load first (unconditional, clamped addresses), then stage in LDS -------
  const float3 araw = LOAD ? wave_action<AD>(io, env, gj) : pre;
  const float a0 = clampk(araw.x, -1.0f, 1.0f), a1 = clampk(araw.y, -1.0f, 1.0f);
  const float aw = OMNI ? clampk(araw.z, -1000.0f, 1000.0f) : 0.0f;  // omni alpha
  float hcx, hcy;
  if constexpr (LOAD) {
    const float* st = io.states + env * io.states_stride;
    const float* ob = io.obstacles + env * io.obstacles_stride;
    const float cv0 = st[lane];
    const int xsl = 64 + (lane < XS ? lane : XS - 1);
    const float cv1 = XS > 0 ? st[xsl] : 0.0f;
    hcx = st[(16 + lane) * SD + 0], hcy = st[(16 + lane) * SD + 1];
    const float obv = ob[lane < O * DGPPO_OBST_FIELDS ? lane : 0];
    const float rdv = io.ray_dirs[lane];
    // unconditional LDS stores: a store under a lane predicate lets the compiler sink its global load
    // into the predicated block, serialising a second HBM round trip
    lds[C::cur + lane] = cv0;
    if (XS > 0) lds[C::cur + xsl] = cv1;
    // omni obstacle cost reads every current hit: staged in the next-hit rows (rewritten in E)
    if (OMNI) reinterpret_cast<float2*>(lds + C::hits)[lane] = make_float2(hcx, hcy);
    lds[C::obst + lane] = obv;  // lanes >= 16 O land in evec / rays, both written after this
    lds[C::rays + lane] = rdv;
  } else {
    // persistent rollout: the previous step's next agent rows are this step's current rows (goals,
    // obstacles and rays unchanged); its hits (rows 16 + lane of its graph) are the current hits
    if (lane < NA * SD) lds[C::cur + lane] = lds[C::nxt + lane];
    const float2 hc = reinterpret_cast<const float2*>(lds + C::hits)[lane];
    hcx = hc.x, hcy = hc.y;
  }
  wave_sync();
  const float* cur = lds + C::cur;
  const float* goal = cur + NA * SD;
  float* nxt = lds + C::nxt;
  float* hits = lds + C::hits;
  const float* obst = lds + C::obst;
  const float* evec = lds + C::evec;
  const float* rays = lds + C::rays;

  ENV_STAMP(0);
  // ---- B: dynamics of agent j (every lane; lanes 0..7 store it), distances, edge vectors -------
  float x[SD];
#pragma unroll
  for (int c = 0; c < SD; ++c) x[c] = cur[gj * SD + c];
  const float cix = cur[gi * SD], ciy = cur[gi * SD + 1];
  const float gix = goal[gi * SD], giy = goal[gi * SD + 1];
  float ev;
  {
    const int o = (lane >> 3) < O ? (lane >> 3) : 0, e = (lane >> 1) & 3, c = lane & 1;
    const float* rec = obst + o * DGPPO_OBST_FIELDS;
    ev = rec[8 + 2 * ((e + 3) & 3) + c] - rec[8 + 2 * e + c];  // (x4 - x3, y4 - y3)
  }
  float y[SD];
  if constexpr (REBUILD) {
#pragma unroll
    for (int c = 0; c < SD; ++c) y[c] = x[c];
  } else if constexpr (OMNI) {  // agent_step_euler (lidar_omni_target.py:146-197)
    const float acc_x = a0 * 10.0f, acc_y = a1 * 10.0f, alw = aw * 5.0f;
    const float theta = atan2_32(x[3], x[2]);
    const float new_theta = theta + x[6] * cfg.dt;
    float sn_, cn_;
    sincos32(new_theta, &sn_, &cn_);
    y[0] = x[0] + x[4] * cfg.dt;
    y[1] = x[1] + x[5] * cfg.dt;
    y[2] = cn_;
    y[3] = sn_;
    y[4] = x[4] + acc_x * cfg.dt;
    y[5] = x[5] + acc_y * cfg.dt;
    y[6] = x[6] + alw * cfg.dt;
  } else if constexpr (ENGINE == DGPPO_ENGINE_BICYCLE) {
    const float theta = atan2_32(x[3], x[2]);
    const float theta_next = theta + ((x[4] * a0) * cfg.dt) * 10.0f;
    float st_, ct_, sn_, cn_;
    sincos32(theta, &st_, &ct_);
    sincos32(theta_next, &sn_, &cn_);
    y[0] = x[0] + (x[4] * ct_) * cfg.dt;
    y[1] = x[1] + (x[4] * st_) * cfg.dt;
    y[2] = cn_;
    y[3] = sn_;
    y[4] = x[4] + (a1 * cfg.dt) * 10.0f;
  } else {
    y[0] = x[2] * cfg.dt + x[0];
    y[1] = x[3] * cfg.dt + x[1];
    y[2] = (a0 * 10.0f) * cfg.dt + x[2];
    y[3] = (a1 * 10.0f) * cfg.dt + x[3];
  }
  if constexpr (!REBUILD) {
#pragma unroll
    for (int c = 0; c < SD; ++c) y[c] = clampf_nan(y[c], cfg.state_lo[c], cfg.state_hi[c]);
  }
  if (lane < NA) {
#pragma unroll
    for (int c = 0; c < SD; ++c) nxt[lane * SD + c] = y[c];
  }
  if (!pc && lane < O * 8) lds[C::evec + lane] = ev;  // (persistent: staged once with the constants)
  const float an = norm2(a0, a1);
  const float a2 = an * an;
  // Lidar / bicycle: the agent, hit and goal distance minima of agent gi over squared norms, then ONE sqrtf for all
  // three (lane (gi, 0): agents, (gi, 1): hits, (gi, >= 2): goals).  sqrtf is correctly rounded and monotone, so
  // sqrtf(min x) == min sqrtf(x) (NaN either way).  The agent-agent diagonal is sqrtf(0) + 1e6 = 1e6 or NaN (the
  // row minus itself): it enters the squared minimum as +inf / NaN and the 1e6 after the sqrtf
  float dmin = 0.0f;
  if constexpr (!OMNI) {
    float saa = sq2(cix - x[0], ciy - x[1]);
    if (gi == gj) saa = saa == 0.0f ? __builtin_inff() : __builtin_nanf("");
    const float sga = GOAL == DGPPO_GOAL_SPREAD ? sq2(gix - x[0], giy - x[1]) : sq2(gix - cix, giy - ciy);
    const float sh = sq2(hcx - cix, hcy - ciy);
    const float maa = min8(saa), mh = min8(sh), mg = min8(sga);
    dmin = sqrtf(gj == 0 ? maa : (gj == 1 ? mh : mg));
  }
  float daa = 0.0f, dga = 0.0f, dh = 0.0f;
  if constexpr (OMNI) {
    daa = norm2(cix - x[0], ciy - x[1]);
    if (gi == gj) daa = daa + 1e6f;
    dga = norm2(gix - cix, giy - ciy);
    // every agent's current hits and the origin row (see oracle get_cost_omni): minimum of the squared
    // norms, one sqrtf after it (sqrtf is correctly rounded and monotone, so sqrtf(min x) == min sqrtf(x);
    // NaN propagates through min_nan either way)
    const float* ch = lds + C::hits;
    float d2 = sq2(0.0f - cix, 0.0f - ciy);
#pragma unroll
    for (int t = 0; t < NA; ++t) {
      const float2 hv = reinterpret_cast<const float2*>(ch)[gj + 8 * t];
      d2 = min_nan(d2, sq2(hv.x - cix, hv.y - ciy));
    }
    dh = sqrtf(d2);
  }
  const float md = OMNI ? min8(daa) : 0.0f, dg = OMNI ? min8(dga) : 0.0f, mo = OMNI ? min8(dh) : 0.0f;

  ENV_STAMP(1);
  // ---- C: cost (lanes j < 2 of group i, 5 for omni), reward (lane 0) -------------------------
  if constexpr (OMNI) {
    float cq[kOmniNC];
    cq[0] = cfg.c_agent_cost - md;
    cq[1] = cfg.c_obs_cost - mo;
    cq[2] = -1.0f, cq[3] = -1.0f, cq[4] = -1.0f;  // FoV on the chain gi -> gi+1; the last agent is safe
    if (gi + 1 < NA) {
      const float xi0 = cix, xi1 = ciy, xi2 = cur[gi * SD + 2], xi3 = cur[gi * SD + 3];
      const float dx = cur[(gi + 1) * SD] - xi0, dy = cur[(gi + 1) * SD + 1] - xi1;
      const float lx = xi2 * dx + xi3 * dy;
      const float ly = (-xi3) * dx + xi2 * dy;
      const float nrm = norm2(lx, ly);
      cq[2] = cfg.c_cos_fov * (nrm + 1e-8f) - lx;
      cq[3] = nrm - cfg.fov_rmax;
      cq[4] = cfg.fov_dmin - nrm;
    }
    const int q = gj < kOmniNC ? gj : 0;
    float v = q == 0 ? cq[0] : (q == 1 ? cq[1] : (q == 2 ? cq[2] : (q == 3 ? cq[3] : cq[4])));
    v = v <= 0.0f ? v - 0.1f : v + 0.1f;
    v = clampk(v, -1.0f, 1.0f);
    if (!REBUILD && st_live & (gj < kOmniNC)) io.cost[env * io.cost_stride + kOmniNC * gi + gj] = v;
    const float far = dg > cfg.dist2goal ? 1.0f : 0.0f;
    const float w2 = aw * aw, o2 = x[6] * x[6];
    float s0 = 0.0f, s1 = 0.0f, s2 = 0.0f, s3 = 0.0f, s4 = 0.0f;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      s0 = s0 + rlf(dg, 8 * i);
      s1 = s1 + rlf(far, 8 * i);
      s2 = s2 + rlf(a2, i);
      s3 = s3 + rlf(w2, i);
      s4 = s4 + rlf(o2, i);
    }
    if (!REBUILD && st_live & (lane == 0)) {  // get_reward (lidar_omni_target.py:295-336)
      const float nn = (float)NA;
      float r = 0.0f - (s0 / nn) * 0.01f;
      r = r - (s1 / nn) * 0.001f;
      r = r - (s2 / nn) * 0.0001f;
      r = r - (s3 / nn) * cfg.rot_pen;
      r = r - ((s4 / nn) * cfg.rot_pen) * 0.5f;
      io.reward[env * io.reward_stride] = r;
    }
  } else {
    // lane (gi, 0): the agent cost c_agent - min(d_aa), lane (gi, 1): the obstacle cost c_obs - min(d_hit)
    float c = gj == 0 ? cfg.c_agent_cost - min_nan(dmin, 1e6f) : cfg.c_obs_cost - dmin;
    c = c <= 0.0f ? c - 0.5f : c + 0.5f;
    c = clampk(c, -1.0f, 1.0f);
    if (!REBUILD && st_live & (gj < 2)) io.cost[env * io.cost_stride + 2 * gi + gj] = c;
    const float far = dmin > cfg.dist2goal ? 1.0f : 0.0f;  // (read at lanes (i, 2): the goal distance)
    float sd_ = 0.0f, sf = 0.0f, sa = 0.0f;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      sd_ = sd_ + rlf(dmin, 8 * i + 2);
      sf = sf + rlf(far, 8 * i + 2);
      sa = sa + rlf(a2, i);  // lane i holds agent j = i
    }
    if (!REBUILD && st_live & (lane == 0)) {
      const float nn = (float)NA;
      float r = 0.0f - (sd_ / nn) * 0.01f;
      r = r - (sf / nn) * 0.001f;
      r = r - (sa / nn) * 0.0001f;
      io.reward[env * io.reward_stride] = r;
    }
  }
  wave_sync();  // nxt, evec visible

  ENV_STAMP(2);
  // ---- F1: the graph parts that do not depend on the lidar, issued as store packets spread over
  // the compute phases below so the HBM drains them while the ray cast runs (one burst would stall
  // every wave on a full store queue at once)
  float* no = io.nodes + env * io.nodes_stride;
  float* so = io.out_states + env * io.out_states_stride;
  float* eo = io.edges + env * io.edges_stride;
  int32_t* ro = io.receivers + env * io.edge_index_stride;
  int32_t* sno = io.senders + env * io.edge_index_stride;
  // edge rows as vector stores: the launchers send only 16-byte (4-wide) / 8-byte (10-wide) aligned edge
  // buffers here (wave_bufs_aligned); a runtime fallback branch would let the compiler merge both
  // paths into 4-byte stores
  auto put = [&](int e, float f0, float f1, float f2, float f3, int rv, int sv) {
    reinterpret_cast<float4*>(eo)[e] = make_float4(f0, f1, f2, f3);
    ro[e] = rv;
    sno[e] = sv;
  };
  // Omni's 10-wide edge rows: assembled in LDS (olist / items are free until the capsule tests) and stored
  // lane-contiguous by flush_wide; a 40-byte row per lane would cost a memory request per lane and store
  float* const wstage = lds + C::olist;
  static_assert(!OMNI || 64 * kOmniED <= C::total - C::olist, "wide edge staging fits");
  auto put_wide = [&](int e, int slot, const float (&f)[kOmniED], int rv, int sv) {
#pragma unroll
    for (int c = 0; c < kOmniED; ++c) wstage[slot * kOmniED + c] = f[c];
    ro[e] = rv;
    sno[e] = sv;
  };
  auto flush_wide = [&](int e0, int rows) {  // every lane; rows e0 .. e0 + rows - 1 from slots 0 .. rows - 1
    wave_sync();
    float* dst = eo + kOmniED * e0;
#pragma unroll
    for (int k = 0; k < (64 * kOmniED + 63) / 64; ++k)
      if (64 * k + lane < rows * kOmniED) dst[64 * k + lane] = wstage[64 * k + lane];
  };
  float si[SD];
#pragma unroll
  for (int c = 0; c < SD; ++c) si[c] = nxt[gi * SD + c];
  if (st_live) {  // store packet 1: agent-agent edges
    float sj[SD];
#pragma unroll
    for (int c = 0; c < SD; ++c) sj[c] = y[c];  // this lane's dynamics result is agent j's next state
    {  // agent-agent row l: mask norm + (comm_radius + 1 on the diagonal) < comm_radius, on |d|^2
      float f2, f3;
      if (ENGINE == DGPPO_ENGINE_BICYCLE) {
        f2 = si[4] * si[2] - sj[4] * sj[2];
        f3 = si[4] * si[3] - sj[4] * sj[3];
      } else {
        f2 = si[2] - sj[2];
        f3 = si[3] - sj[3];
      }
      const float dx = si[0] - sj[0], dy = si[1] - sj[1];
      const float d2 = dx * dx + dy * dy;
      const bool m = gi == gj ? ((d2 == 0.0f) & (cfg.c_self_dist < cfg.comm_radius)) : (d2 < cfg.t2_comm);
      if constexpr (OMNI) {  // [s_i - s_j | critical i -> i+1 | ||p_j^i|| | i_x_j] (lidar_omni_target.py:352-422)
        float f[kOmniED];
#pragma unroll
        for (int c = 0; c < SD; ++c) f[c] = si[c] - sj[c];
        f[7] = gj == gi + 1 ? 1.0f : 0.0f;
        const float gx = -(si[0] - sj[0]), gy = -(si[1] - sj[1]);
        const float lx = si[2] * gx + si[3] * gy;
        const float ly = (-si[3]) * gx + si[2] * gy;
        f[8] = norm2(lx, ly);
        f[9] = lx;
        put_wide(lane, lane, f, m ? gi : pad, m ? gj : pad);
        flush_wide(0, NA * NA);
      } else {
        put(lane, dx, dy, f2, f3, m ? gi : pad, m ? gj : pad);
      }
    }
  }

  ENV_STAMP(3);
  // ---- D: is-inside at the next state; culling masks; capsule tests -> item list -------------
  const float sxi = si[0], syi = si[1];
  const int oi = gj < O ? gj : 0;
  const bool in_o = (gj < O) & rect_inside0(obst + oi * DGPPO_OBST_FIELDS, sxi, syi);
  const uint64_t in_mask = __ballot(in_o);
  const int rr = lane & 31;
  const WaveConst<O> kc = pc ? *pc : wave_const<O>(obst, evec, rays, lane);
  const float rdx = kc.rdx, rdy = kc.rdy, rlen2 = kc.rlen2, rlen = kc.rlen, rho_l = kc.rho_l;
  uint32_t unsafe[O];
#pragma unroll
  for (int o = 0; o < O; ++o) unsafe[o] = kc.unsafe[o];
  ENV_STAMP(4);
  if (st_live) {  // store packet 2: agent-goal edges
    float sj[SD], sg[SD];
#pragma unroll
    for (int c = 0; c < SD; ++c) {
      sj[c] = y[c];
      sg[c] = goal[gj * SD + c];
    }
    if (GOAL == DGPPO_GOAL_SPREAD) {  // agent i -> goal j
      float f2, f3;
      if (ENGINE == DGPPO_ENGINE_BICYCLE) {
        f2 = si[4] * si[2] - sg[4] * sg[2];
        f3 = si[4] * si[3] - sg[4] * sg[3];
      } else {
        f2 = si[2] - sg[2];
        f3 = si[3] - sg[3];
      }
      put(NA * NA + lane, si[0] - sg[0], si[1] - sg[1], f2, f3, gi, NA + gj);
    } else if (OMNI & (lane < NA)) {  // agent j -> own goal j, zero-padded to 10 (lidar_omni_target.py:424-443)
      float f[kOmniED];
#pragma unroll
      for (int c = 0; c < kOmniED; ++c) f[c] = c < SD ? sj[c < SD ? c : 0] - sg[c < SD ? c : 0] : 0.0f;
      put_wide(NA * NA + lane, lane, f, lane, NA + lane);
    } else if (lane < NA) {  // agent j -> own goal j
      float f2, f3;
      if (ENGINE == DGPPO_ENGINE_BICYCLE) {
        f2 = sj[4] * sj[2] - sg[4] * sg[2];
        f3 = sj[4] * sj[3] - sg[4] * sg[3];
      } else {
        f2 = sj[2] - sg[2];
        f3 = sj[3] - sg[3];
      }
      put(NA * NA + lane, sj[0] - sg[0], sj[1] - sg[1], f2, f3, lane, NA + lane);
    }
    if constexpr (OMNI) flush_wide(NA * NA, NA);
  }
  ENV_STAMP(5);
  // capsule test of every (agent, obstacle, ray) triple: pair p = o * 8 + i, 2 pairs per step (lane
  // halves), o and i = 2 m + half known per step; survivors -> compacted item list
  int n_items = 0;
  {
    int* items = reinterpret_cast<int*>(lds + C::uni);
    const int h = lane >> 5;
    float qx[4], qy[4];
    bool qok[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      qx[m] = nxt[(2 * m + h) * SD];
      qy[m] = nxt[(2 * m + h) * SD + 1];
      qok[m] = (fabsf(qx[m]) <= 2.0f) & (fabsf(qy[m]) <= 2.0f);
    }
    // the lane's survivors as a bit mask (bit 4 o + m), then one wave-wide exclusive prefix of the
    // per-lane counts (4 ballots over the count bits) and a short per-lane write loop: no per-triple
    // ballot and predicated store (the item order does not matter: alphas combine by atomicMin)
    uint32_t kmask = 0u;
#pragma unroll
    for (int o = 0; o < O; ++o) {
      const float cx = obst[o * DGPPO_OBST_FIELDS], cy = obst[o * DGPPO_OBST_FIELDS + 1];
      const float Rl = (rlf(rho_l, o) + kCullMargin) * rlen;
      const bool forced = (unsafe[o] >> rr) & 1u;
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const float vx = cx - qx[m], vy = cy - qy[m];
        const float perp = vx * rdy - vy * rdx;
        const float proj = vx * rdx + vy * rdy;
        const bool miss = qok[m] & ((fabsf(perp) > Rl) | (proj < -Rl) | (proj > rlen2 + Rl));
        kmask |= (uint32_t)(!miss | forced) << (4 * o + m);
      }
    }
    if (!live) kmask = 0u;
    static_assert(4 * O <= 15, "per-lane survivor count fits 4 bits");
    const int cnt = __builtin_popcount(kmask);
    int pre = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const uint64_t bb = __ballot((cnt >> b) & 1);
      pre += mbcnt(bb) << b;
      n_items += __popcll(bb) << b;
    }
    while (kmask) {
      const int k = __builtin_ctz(kmask);
      kmask &= kmask - 1u;
      items[pre++] = (((k >> 2) * 8 + 2 * (k & 3) + h) << 5) | rr;
    }
  }
  ENV_STAMP(6);
  if (st_live) {  // store packet 3: node / state rows of agents and goals, pad rows
    // node rows 0..15 (agents, goals) and the pad row; state rows 0..15 and the pad row
#pragma unroll
    for (int k = 0; k < (16 * ND + 63) / 64; ++k) {
      const int idx = lane + 64 * k;
      const int r = idx / ND, c = idx - (idx / ND) * ND;
      const int rs = r < 16 ? r : 15;
      const float* src = rs < NA ? nxt + rs * SD : goal + (rs - NA) * SD;
      const float sv = src[c < SD ? c : 0];
      const float v = c < SD ? sv : (c == SD + 2 ? (r < NA ? 1.0f : 0.0f) : (c == SD + 1 ? (r < NA ? 0.0f : 1.0f) : 0.0f));
      if (idx < 16 * ND) no[idx] = v;
    }
    if constexpr (ST4) {
      // 16-byte state rows (SD = 4): lane r < 16 stores row r, lane 16 the pad row, one float4 each (the launchers
      // send only 16-byte aligned state buffers here: wave_bufs_aligned)
      const int rs = lane < 16 ? lane : 0;
      const float4 v = *reinterpret_cast<const float4*>(rs < NA ? nxt + rs * SD : goal + (rs - NA) * SD);
      if (lane <= 16)
        reinterpret_cast<float4*>(so)[lane < 16 ? lane : pad] = lane < 16 ? v : make_float4(-1.0f, -1.0f, -1.0f, -1.0f);
    } else {
#pragma unroll
      for (int k = 0; k < (16 * SD + 63) / 64; ++k) {
        const int idx = lane + 64 * k;
        const int r = idx / SD, c = idx - (idx / SD) * SD;
        const int rs = r < 16 ? r : 15;
        const float v = (rs < NA ? nxt + rs * SD : goal + (rs - NA) * SD)[c];
        if (idx < 16 * SD) so[idx] = v;
      }
      if (lane < SD) so[pad * SD + lane] = -1.0f;
    }
    if (lane < ND) no[pad * ND + lane] = 0.0f;
  }
  uint32_t* alpha = reinterpret_cast<uint32_t*>(lds + C::alpha);
  reinterpret_cast<uint4*>(alpha)[lane] = make_uint4(kEncMiss, kEncMiss, kEncMiss, kEncMiss);
  ENV_STAMP(7);
  if constexpr (WPG == 1) {
    // one env per workgroup: the wave ray-casts its own items, no workgroup barriers
    wave_sync();
    ENV_STAMP(8);
    for (int base = 0; base < n_items; base += 64) {
      const int g = base + lane;
      const bool act = g < n_items;
      const int it = reinterpret_cast<const int*>(lds + C::uni)[act ? g : 0];
      const int r = it & 31, p = (it >> 5) & 31, o = (p >> 3) < O ? (p >> 3) : 0, i = p & 7;
      const float sx = nxt[i * SD + 0], sy = nxt[i * SD + 1];
      const float2 rd = reinterpret_cast<const float2*>(rays)[r];
      const float* rec = obst + o * DGPPO_OBST_FIELDS;
      const float* evo = evec + o * 8;
      const float ex = sx + rd.x, ey = sy + rd.y;
      float a;
      const bool ok = raytrace_nodiv(reinterpret_cast<const float4*>(rec)[2], reinterpret_cast<const float4*>(rec)[3],
                                     reinterpret_cast<const float4*>(evo)[0], reinterpret_cast<const float4*>(evo)[1],
                                     sx, sy, sx - ex, sy - ey, &a);
      if (act & !ok) a = rect_raytrace(rec, evo, sx, sy, sx - ex, sy - ey);
      if (act) atomicMin(alpha + i * NR + r, enc_alpha(a));
    }
    ENV_STAMP(9);
    ENV_STAMP(10);
    wave_sync();
  } else {
  if (lane == 0) wg_items[wid] = n_items;
  __syncthreads();  // item lists of the 4 envs of this workgroup are complete
  ENV_STAMP(8);

  // exact ray cast of the surviving triples, pooled over the workgroup's WPG envs (balances the
  // per-env item counts; each item atomically min-combines into its own env's alpha row)
  {
    int starts[WPG], tot = 0;
#pragma unroll
    for (int w = 0; w < WPG; ++w) {
      starts[w] = tot;
      tot += wg_items[w];
    }
    for (int base = wid * 64; base < tot; base += 64 * WPG) {
      const int g = base + lane;
      const bool act = g < tot;
      const int gg = act ? g : 0;
      int w2 = 0;
#pragma unroll
      for (int w = 1; w < WPG; ++w) w2 = gg >= starts[w] ? w : w2;
      int k = gg;
#pragma unroll
      for (int w = 1; w < WPG; ++w) k = w2 == w ? gg - starts[w] : k;
      float* L = smem + w2 * C::total;
      const int it = reinterpret_cast<const int*>(L + C::uni)[k];
      const int r = it & 31, p = (it >> 5) & 31, o = (p >> 3) < O ? (p >> 3) : 0, i = p & 7;
      const float sx = L[C::nxt + i * SD + 0], sy = L[C::nxt + i * SD + 1];
      const float2 rd = reinterpret_cast<const float2*>(L + C::rays)[r];
      const float* rec = L + C::obst + o * DGPPO_OBST_FIELDS;
      const float* evo = L + C::evec + o * 8;
      const float4* rec4 = reinterpret_cast<const float4*>(rec);
      const float4* e4 = reinterpret_cast<const float4*>(evo);
      const float ex = sx + rd.x, ey = sy + rd.y;
      float a;
      const bool ok = raytrace_nodiv(rec4[2], rec4[3], e4[0], e4[1], sx, sy, sx - ex, sy - ey, &a);
      if (act & !ok) a = rect_raytrace(rec, evo, sx, sy, sx - ex, sy - ey);
      if (act) atomicMin(reinterpret_cast<uint32_t*>(L + C::alpha) + i * NR + r, enc_alpha(a));
    }
  }
  ENV_STAMP(9);
  ENV_STAMP(10);
  __syncthreads();  // every alpha row is final
  }
  ENV_STAMP(11);

  // ---- E: sort keys; misses ranked by popcount, the rest by comparison; top-k hit points ------
  uint64_t* keys = reinterpret_cast<uint64_t*>(lds + C::uni);  // items are dead now
  int* olist = reinterpret_cast<int*>(lds + C::olist);
  const float isin = ((in_mask >> (8 * gi)) & 0xFFull) ? 1.0f : 0.0f;
  int n_other = 0;
  // CRANK: each agent row keeps only its non-miss keys, compacted and padded with all-ones keys, and a non-miss ray
  // is ranked against that list (mrow = the longest row, wave-uniform) plus, for a NaN alpha, every miss of its row
  // (misses sort after every number and before NaN); a miss never ranks before a number, so the ranks are the
  // full row's.  Alphas here are >= +0, 1e6 or NaN, so the key's high word is the alpha bits (NaN -> all ones).
  static_assert(NA * C::key_stride + NA <= C::uni_size, "row counts fit behind the keys");
  int* rowcnt = reinterpret_cast<int*>(lds + C::uni + NA * C::key_stride);
  int mrow = 0;
  auto key_pos = [](float a, int r) {
    return ((uint64_t)(a != a ? 0xFFFFFFFFu : __float_as_uint(a)) << 32) | (uint32_t)r;
  };
  {
    const uint4 e4 = reinterpret_cast<const uint4*>(alpha + gi * NR)[gj];
    const float4 rA = reinterpret_cast<const float4*>(rays)[2 * gj], rB = reinterpret_cast<const float4*>(rays)[2 * gj + 1];
    const uint32_t ev4[4] = {e4.x, e4.y, e4.z, e4.w};
    const float rx[4] = {rA.x, rA.z, rB.x, rB.z}, ry[4] = {rA.y, rA.w, rB.y, rB.w};
    float av[4], hx[4], hy[4];
    bool miss[4];
    uint32_t sm[4];
    uint64_t obq[4];
    int hf = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      av[q] = dec_alpha(ev4[q]) * (1.0f - isin);
      miss[q] = av[q] == 1e6f;
      const float ex = sxi + rx[q], ey = syi + ry[q];
      hx[q] = sxi + (ex - sxi) * av[q];
      hy[q] = syi + (ey - syi) * av[q];
      sm[q] = (uint32_t)(__ballot(miss[q]) >> (8 * gi)) & 0xFFu;
      obq[q] = __ballot(!miss[q]);
      hf += __builtin_popcount((uint32_t)(__ballot(!miss[q] & (av[q] == av[q])) >> (8 * gi)) & 0xFFu);
    }
    uint64_t* krow = keys + gi * (C::key_stride / 2);
    const uint32_t below = (1u << gj) - 1u;
    if constexpr (DGPPO_ENV_CRANK) {
      const ulonglong2 ones = make_ulonglong2(~0ull, ~0ull);
      reinterpret_cast<ulonglong2*>(krow)[2 * gj] = ones;
      reinterpret_cast<ulonglong2*>(krow)[2 * gj + 1] = ones;
      int pos = 0, rc = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t nm = (uint32_t)(obq[q] >> (8 * gi)) & 0xFFu;
        pos += __builtin_popcount(nm & below);
        rc += __builtin_popcount(nm);
      }
      wave_sync();  // every lane's padding before any compacted key
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (!miss[q]) krow[pos] = key_pos(av[q], 4 * gj + q);
        pos += miss[q] ? 0 : 1;
      }
      if (gj == 0) rowcnt[gi] = rc;
      // the longest row: max of the two groups of each 16-lane row, then of the four rows
      const int m2 = max(rc, __builtin_amdgcn_mov_dpp(rc, 0x128, 0xf, 0xf, true));  // row_ror:8
      mrow = max(max(__builtin_amdgcn_readlane(m2, 0), __builtin_amdgcn_readlane(m2, 16)),
                 max(__builtin_amdgcn_readlane(m2, 32), __builtin_amdgcn_readlane(m2, 48)));
    } else {
      reinterpret_cast<ulonglong2*>(krow)[2 * gj] = make_ulonglong2(sort_key(av[0], 4 * gj), sort_key(av[1], 4 * gj + 1));
      reinterpret_cast<ulonglong2*>(krow)[2 * gj + 1] = make_ulonglong2(sort_key(av[2], 4 * gj + 2), sort_key(av[3], 4 * gj + 3));
    }
    int cnt = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) cnt += __builtin_popcount(sm[q] & below);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int rank = hf + cnt;
      if (miss[q] & (rank < NK)) {
        hits[(gi * NK + rank) * 2 + 0] = hx[q];
        hits[(gi * NK + rank) * 2 + 1] = hy[q];
      }
      cnt += (sm[q] >> gj) & 1u;
      if (!miss[q]) olist[n_other + mbcnt(obq[q])] = gi * NR + 4 * gj + q;
      n_other += __popcll(obq[q]);
    }
  }
  wave_sync();
  ENV_STAMP(12);
  for (int base = 0; base < n_other; base += 64) {
    const int t = base + lane;
    const int v = olist[t];  // past n_other: stale words (olist is followed by the key region)
    const int i = (v >> 5) & 7, r = v & 31;
    const uint64_t* krow = keys + i * (C::key_stride / 2);
    const float a = dec_alpha(alpha[i * NR + r]) * (((in_mask >> (8 * i)) & 0xFFull) ? 0.0f : 1.0f);
    const float sx = nxt[i * SD + 0], sy = nxt[i * SD + 1];
    const float2 rd = reinterpret_cast<const float2*>(rays)[r];
    int rank = 0;
    if constexpr (DGPPO_ENV_CRANK) {
      const uint64_t key = key_pos(a, r);
      for (int j = 0; j < mrow; j += 2) {
        const ulonglong2 kk = *reinterpret_cast<const ulonglong2*>(krow + j);
        rank += kk.x < key ? 1 : 0;
        rank += kk.y < key ? 1 : 0;
      }
      if (a != a) rank += NR - rowcnt[i];
    } else {
      const uint64_t key = krow[r];
#pragma unroll
      for (int j = 0; j < NR; j += 2) {
        const ulonglong2 kk = *reinterpret_cast<const ulonglong2*>(krow + j);
        rank += kk.x < key ? 1 : 0;
        rank += kk.y < key ? 1 : 0;
      }
    }
    if ((t < n_other) & (rank < NK)) {
      const float ex = sx + rd.x, ey = sy + rd.y;
      hits[(i * NK + rank) * 2 + 0] = sx + (ex - sx) * a;
      hits[(i * NK + rank) * 2 + 1] = sy + (ey - sy) * a;
    }
  }
  wave_sync();
  ENV_STAMP(13);

  // ---- F2: the hit rows and agent-lidar edges.  Node / state rows of the hits (and Omni's 10-wide edge
  // rows) are assembled in LDS (olist, keys and items are dead now) and written lane-contiguous: a row per
  // lane at a 28-40 byte stride would cost a memory request per lane and store instruction
  {
    const float2 hl = reinterpret_cast<const float2*>(hits)[lane];
    const float f0 = si[0] - hl.x;
    const float f1 = si[1] - hl.y;
    // Lidar: norm < comm_radius - 0.1; omni: norm < comm_radius (lidar_omni_target.py:446-489); on |d|^2
    const bool m = f0 * f0 + f1 * f1 < (OMNI ? cfg.t2_comm : cfg.t2_lidar);
    const int e = NA * NA + n_ag + lane;
    static_assert(64 * (ND + SD) <= C::total - C::olist && 64 * ED <= C::total - C::olist, "F2 staging fits");
    float* sn = lds + C::olist;  // (64, ND) hit node rows [x, y, 0.. | obstacle 1, goal 0, agent 0]
    float* ss = sn + 64 * ND;    // (64, SD) hit state rows [x, y, 0..]
#pragma unroll
    for (int c = 0; c < ND; ++c) sn[lane * ND + c] = c == 0 ? hl.x : (c == 1 ? hl.y : (c == SD ? 1.0f : 0.0f));
    if constexpr (!ST4) {
#pragma unroll
      for (int c = 0; c < SD; ++c) ss[lane * SD + c] = c == 0 ? hl.x : (c == 1 ? hl.y : 0.0f);
    }
    wave_sync();
    if (st_live) {
      if constexpr (ED == 4) reinterpret_cast<float4*>(eo)[e] = make_float4(f0, f1, 0.0f, 0.0f);
      ro[e] = m ? gi : pad;
      sno[e] = m ? 2 * NA + lane : pad;
      float* nd = no + 16 * ND;
      float* sdst = so + 16 * SD;
#pragma unroll
      for (int k = 0; k < ND; ++k) nd[64 * k + lane] = sn[64 * k + lane];
      if constexpr (ST4) {
        reinterpret_cast<float4*>(sdst)[lane] = make_float4(hl.x, hl.y, 0.0f, 0.0f);
      } else {
#pragma unroll
        for (int k = 0; k < SD; ++k) sdst[64 * k + lane] = ss[64 * k + lane];
      }
    }
    if constexpr (ED != 4) {
      wave_sync();  // (in-order LDS: the reads above are done before these writes)
      float* se = lds + C::olist;  // (64, ED) edge rows [f0, f1, 0..]
#pragma unroll
      for (int c = 0; c < ED; ++c) se[lane * ED + c] = c == 0 ? f0 : (c == 1 ? f1 : 0.0f);
      wave_sync();
      if (st_live) {
        float* ed = eo + ED * (NA * NA + n_ag);
#pragma unroll
        for (int k = 0; k < ED; ++k) ed[64 * k + lane] = se[64 * k + lane];
      }
    }
  }
  ENV_STAMP(14);
}

// One env step (REBUILD: the graph of the given states) for io.n_env envs, 4 per workgroup.
template <int ENGINE, int GOAL, int SD, int O, bool REBUILD = false>
__global__ __launch_bounds__(256) void lidar_step_wave_kernel(dgppo_env_cfg cfg, dgppo_env_step_io io) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ int wg_items[4];
  wave_body<ENGINE, GOAL, SD, O, REBUILD, true>(cfg, io, smem, wg_items);
}

constexpr int kRolloutActFloats = 16 * NA * 3;  // per wave: a 16-step action chunk (3 action floats max)

// Persistent rollout: T env steps per launch, a wave per env for the whole episode (the reference's
// lax.scan over env.step, trainer/utils.py:45-55, with the actions given).  Agent rows, hits,
// obstacles and rays stay in LDS between steps: per step the wave reads its env's actions (T, B, n, A)
// and writes graph t+1's rows into the time-major (T+1, B) buffer, reward[t] and cost[t].  No launch
// per step, and the 4096 waves drift out of phase, so one wave's store drain overlaps another's compute.
// rebuild_first: graph 0 is first built from its agent / goal / obstacle rows (after a states-only
// reset), else its current rows are loaded.
// (4 waves per SIMD: the whole 4096-env batch resident at once, as for the per-step kernel; without the
// bound the loop's hoisted addressing takes ~150 VGPRs and a quarter of the workgroups would run after
// the rest had finished their episodes)
// WPG: envs (waves) per workgroup — 4 pools the ray casts of 4 envs between two workgroup barriers per
// step, 1 casts each env's own items with wave-level syncs only
template <int ENGINE, int GOAL, int SD, int O, int WPG>
__global__ __launch_bounds__(64 * WPG) __attribute__((amdgpu_waves_per_eu(4))) void lidar_rollout_wave_kernel(
    dgppo_env_cfg cfg, dgppo_env_rollout_io r) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ int wg_items[WPG];
  const dgppo_env_step_io& g0 = r.step;
  if (r.rebuild_first) {
    wave_body<ENGINE, GOAL, SD, O, true, true, WPG>(cfg, g0, smem, wg_items);
  } else {  // stage graph 0's rows exactly as the LOAD prologue of a step does
    using C = Carve<SD, O>;
    constexpr int XS = 16 * SD - 64;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int64_t env_raw = (int64_t)blockIdx.x * WPG + wid;
    const int64_t env = env_raw < g0.n_env ? env_raw : g0.n_env - 1;
    float* lds = smem + wid * C::total;
    const float* st = g0.states + env * g0.states_stride;
    const float* ob = g0.obstacles + env * g0.obstacles_stride;
    const float cv0 = st[lane];
    const int xsl = 64 + (lane < XS ? lane : XS - 1);
    const float cv1 = XS > 0 ? st[xsl] : 0.0f;
    const float hcx = st[(16 + lane) * SD + 0], hcy = st[(16 + lane) * SD + 1];
    const float obv = ob[lane < O * DGPPO_OBST_FIELDS ? lane : 0];
    const float rdv = g0.ray_dirs[lane];
    reinterpret_cast<float2*>(lds + C::hits)[lane] = make_float2(hcx, hcy);
    lds[C::obst + lane] = obv;
    lds[C::rays + lane] = rdv;
    // the current agent rows go to the NEXT-row slot: the first step copies them over (goals in place)
    if (lane < NA * SD) lds[C::nxt + lane] = cv0;
    lds[C::cur + lane] = cv0;
    if (XS > 0) lds[C::cur + xsl] = cv1;
    wave_sync();
  }
  // actions arrive in chunks of KC steps staged in LDS, the next chunk loaded into registers one chunk
  // ahead: vmcnt counts stores too, so any wait on an action load also waits for the store drain before
  // it — once per chunk instead of once per step
  constexpr int AD = ENGINE == DGPPO_ENGINE_OMNI ? 3 : 2;
  constexpr int APS = NA * AD, KC = 16, PER = KC * APS / 64;  // action floats per step / per lane and chunk
  static_assert(PER * 64 == KC * APS, "chunk = whole lanes");
  // the wave index as a wave-uniform (SGPR) value: the env's output base pointers then live in SGPRs and every store
  // takes the SGPR-base + 32-bit lane offset form (one address VGPR per lane, no 64-bit address arithmetic per store)
  const int lane = threadIdx.x & 63, gj = lane & 7;
  constexpr bool UNI = DGPPO_ENV_UNI == 2 || (DGPPO_ENV_UNI == 1 && ENGINE == DGPPO_ENGINE_BICYCLE);
  const int wid = UNI ? (__builtin_amdgcn_readfirstlane(threadIdx.x) >> 6) : (int)(threadIdx.x >> 6);
  const int64_t env_raw = (int64_t)blockIdx.x * WPG + wid;
  const int64_t env = env_raw < g0.n_env ? env_raw : g0.n_env - 1;
  float* acts = smem + WPG * wv::Carve<SD, O>::total + wid * (KC * APS);
  auto load_chunk = [&](int t0, float (&v)[PER]) {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int idx = lane * PER + j, st = idx / APS, k = idx - st * APS;
      const int ts = t0 + st < r.T ? t0 + st : r.T - 1;
      v[j] = g0.action[ts * r.t_action + env * g0.action_stride + k];
    }
  };
  float cv[PER];
  if (r.T > 0) load_chunk(0, cv);
  // episode constants of the culling: the obstacle edge vectors (staged in LDS once; the steps skip
  // their rewrite) and the per-ray / per-obstacle bounds
  WaveConst<O> kc;
  {
    using Cv = wv::Carve<SD, O>;
    float* lw = smem + wid * Cv::total;
    const int o = (lane >> 3) < O ? (lane >> 3) : 0, e = (lane >> 1) & 3, c = lane & 1;
    const float* rec = lw + Cv::obst + o * DGPPO_OBST_FIELDS;
    const float ev = rec[8 + 2 * ((e + 3) & 3) + c] - rec[8 + 2 * e + c];
    wave_sync();
    if (lane < O * 8) lw[Cv::evec + lane] = ev;
    wave_sync();
    kc = wave_const<O>(lw + Cv::obst, lw + Cv::evec, lw + Cv::rays, lane);
  }
#ifdef DGPPO_ENV_STAMPS
  EnvStamps stv{};
  EnvStamps* stamps = &stv;
  stv.last = __builtin_amdgcn_s_memtime();
#else
  EnvStamps* stamps = nullptr;
#endif
  float* const nodes_e = g0.nodes + env * g0.nodes_stride;
  float* const edges_e = g0.edges + env * g0.edges_stride;
  float* const states_e = g0.out_states + env * g0.out_states_stride;
  int32_t* const recv_e = g0.receivers + env * g0.edge_index_stride;
  int32_t* const send_e = g0.senders + env * g0.edge_index_stride;
  float* const reward_e = g0.reward + env * g0.reward_stride;
  float* const cost_e = g0.cost + env * g0.cost_stride;
#pragma clang loop unroll(disable)
  for (int t = 0; t < r.T; ++t) {
    const int tc = t % KC;
    if (tc == 0) {
#pragma unroll
      for (int j = 0; j < PER; ++j) acts[lane * PER + j] = cv[j];
      wave_sync();
      if (t + KC < r.T) load_chunk(t + KC, cv);
    }
    const float* ar = acts + tc * APS + AD * gj;
    const float3 act = make_float3(ar[0], ar[1], AD == 3 ? ar[AD - 1] : 0.0f);
    // this env's rows of step t: base pointers with the env offset folded in and zero env strides (constants
    // after inlining), so the step does no 64-bit index arithmetic and keeps fewer values in SGPRs
    dgppo_env_step_io q = g0;
    q.nodes = nodes_e + (t + 1) * r.t_nodes;
    q.nodes_stride = 0;
    q.edges = edges_e + (t + 1) * r.t_edges;
    q.edges_stride = 0;
    q.out_states = states_e + (t + 1) * r.t_states;
    q.out_states_stride = 0;
    q.receivers = recv_e + (t + 1) * r.t_index;
    q.senders = send_e + (t + 1) * r.t_index;
    q.edge_index_stride = 0;
    q.reward = reward_e + t * r.t_reward;
    q.reward_stride = 0;
    q.cost = cost_e + t * r.t_cost;
    q.cost_stride = 0;
    wave_body<ENGINE, GOAL, SD, O, false, false, WPG>(cfg, q, smem, wg_items, act, stamps, &kc);
  }
#ifdef DGPPO_ENV_STAMPS
  if (lane == 0 && env_raw < g0.n_env)
    for (int k = 0; k < 16; ++k) atomicAdd(&g_env_stamps[k], (unsigned long long)stv.acc[k]);
#else
  (void)stamps;
#endif
}


// ---- MPE, n = 3 agents, 3 obstacles (BASELINE config 2): persistent rollout, a wave per env ------------------
// The workgroup-per-env block kernel spends each step on generic task loops between five barrier phases; at 1024
// envs one wave sits on each SIMD, so every phase's latency is exposed.  Here one 64-lane wave owns one env for the
// whole episode with fixed lane roles, the same fp32 arithmetic as block_step / write_graph_mpe (bit-identical,
// tests/test_rollout_gpu.py):
//   lanes 0..2       agent q's dynamics + clip (mpe/base.py:129-135), its next row into LDS
//   quads 0..2       agent i vs agent j = lane & 3 (the eye * 1e6 diagonal added after the root, mpe/base.py:173-176)
//   quads 3..5       goal g vs agent a (SPREAD: every a, goal g's nearest agent; TARGET: a = g only)
//   quads 6..8       agent i vs obstacle o (mpe/base.py:179-181)
//   lanes 36..38     ||a_i|| (get_reward's action norm)
// one sqrtf for all of them, the row minima as 2-step quad reductions (v_minimum3: NaN-propagating like min_nan,
// equal values on these >= +0 norms), costs on lanes 0..5, the reward on lane 0 from readlanes in the reference's
// order, then graph t + 1 (70 node floats, 40 state floats, 27 / 21 edges) from LDS rows with per-lane constant
// roles.  Agent rows double-buffer in LDS by step parity; actions arrive clipped in KC-step chunks (as the Lidar
// wave kernel: a chunk's load waits once for the store drain before it, not once per step).
namespace mpew {
constexpr int NA = 3, NO = 3, SD = 4, ND = SD + 3, N = 2 * NA + NO + 1, PAD = N - 1, KC = 32;
constexpr int A0 = 0, GL = A0 + 2 * NA * SD, OB = GL + NA * SD, ACT = OB + NO * SD;  // LDS floats per wave
constexpr int TOTAL = ACT + KC * 2 * NA;                                                  // 48 + 192 = 240
static_assert((KC * 2 * NA) % 64 == 0, "a chunk is whole lanes");

template <int GOAL>
__global__ __launch_bounds__(256) void mpe_rollout_wave_kernel(dgppo_env_cfg cfg, dgppo_env_rollout_io r) {
  constexpr bool SPREAD = GOAL == DGPPO_GOAL_SPREAD;
  constexpr int NAG = SPREAD ? NA * NA : NA, E = NA * NA + NAG + NA * NO;
  constexpr int PER = KC * 2 * NA / 64;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const dgppo_env_step_io& g0 = r.step;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x) >> 6;
  const int64_t env_raw = (int64_t)blockIdx.x * 4 + wid;
  if (env_raw >= g0.n_env) return;  // no workgroup barrier in this kernel: a surplus wave just leaves
  const int64_t env = env_raw;
  float* lds = smem + wid * TOTAL;
  // graph 0's state rows: agents -> agent slot 0, goals -> GL, obstacles -> OB (2n + O rows)
  {
    const float* st = g0.states + env * g0.states_stride;
    const float v = st[lane < 36 ? lane : 0];
    if (lane < 36) lds[lane < NA * SD ? A0 + lane : GL + (lane - NA * SD)] = v;
  }
  wv::wave_sync();
  // per-lane roles (constant over the episode)
  const int q4 = lane >> 2, c4 = lane & 3;
  bool dvalid = lane < 36 && c4 < 3;
  if (!SPREAD && q4 >= 3 && q4 < 6) dvalid = dvalid && c4 == 0;
  const bool diag = q4 < 3 && c4 == q4;
  const bool anorm = lane >= 36 && lane < 39;
  // operand rows (x, y) of the lane's distance: (cur?, offset)
  int oa, ob;
  bool ca, cb;
  if (q4 < 3) {
    ca = true, oa = q4 * SD, cb = true, ob = (c4 < 3 ? c4 : 0) * SD;
  } else if (q4 < 6) {
    const int gj = q4 - 3, ai = SPREAD ? (c4 < 3 ? c4 : 0) : gj;
    ca = false, oa = GL + gj * SD, cb = true, ob = ai * SD;
  } else {
    const int i = q4 < 9 ? q4 - 6 : 0;
    ca = true, oa = i * SD, cb = false, ob = OB + (c4 < 3 ? c4 : 0) * SD;
  }
  const int ag = lane < 3 ? lane : (anorm ? lane - 36 : 0);  // the agent whose action this lane reads
  // graph roles: node floats idx = lane + 64 k (k = 0, 1), state floats idx = lane, edge e = lane
  int nr[2], nc[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int idx = lane + 64 * k;
    nr[k] = idx / ND;
    nc[k] = idx - nr[k] * ND;
  }
  const int sr = lane >> 2, sc = lane & 3;
  int ei = 0, ej = 0, ekind = 0;  // kind 0 agent-agent, 1 agent-goal, 2 agent-obstacle
  if (lane < NA * NA) {
    ei = lane / NA, ej = lane - ei * NA, ekind = 0;
  } else if (lane < NA * NA + NAG) {
    const int qq = lane - NA * NA;
    ei = SPREAD ? qq / NA : qq, ej = SPREAD ? qq - ei * NA : qq, ekind = 1;
  } else if (lane < E) {
    const int qq = lane - NA * NA - NAG;
    ei = qq / NO, ej = qq - ei * NO, ekind = 2;
  }
  // actions: chunks of KC steps, the next chunk in registers one chunk ahead
  const float* act0 = g0.action + env * g0.action_stride;
  float* acts = lds + ACT;
  auto load_chunk = [&](int t0, float (&v)[PER]) {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int idx = lane * PER + j, st = idx / (2 * NA), kk = idx - st * (2 * NA);
      const int ts = t0 + st < r.T ? t0 + st : r.T - 1;
      v[j] = act0[(int64_t)ts * r.t_action + kk];
    }
  };
  float cv[PER];
  if (r.T > 0) load_chunk(0, cv);
  float* const nodes_e = g0.nodes + env * g0.nodes_stride;
  float* const edges_e = g0.edges + env * g0.edges_stride;
  float* const states_e = g0.out_states + env * g0.out_states_stride;
  int32_t* const recv_e = g0.receivers + env * g0.edge_index_stride;
  int32_t* const send_e = g0.senders + env * g0.edge_index_stride;
  float* const reward_e = g0.reward + env * g0.reward_stride;
  float* const cost_e = g0.cost + env * g0.cost_stride;
#pragma clang loop unroll(disable)
  for (int t = 0; t < r.T; ++t) {
    const int tc = t % KC;
    if (tc == 0) {
#pragma unroll
      for (int j = 0; j < PER; ++j) acts[lane * PER + j] = clampf_nan(cv[j], -1.0f, 1.0f);
      wv::wave_sync();
      if (t + KC < r.T) load_chunk(t + KC, cv);
    }
    const int cur = (t & 1) * NA * SD, nxt = NA * SD - cur;
    // ---- dynamics (lanes 0..2) and the action norms (lanes 36..38)
    const float2 a = *reinterpret_cast<const float2*>(acts + tc * 2 * NA + 2 * ag);
    const float4 x = *reinterpret_cast<const float4*>(lds + A0 + cur + ag * SD);
    float y[SD];
    y[0] = x.z * cfg.dt + x.x;
    y[1] = x.w * cfg.dt + x.y;
    y[2] = (a.x * 10.0f) * cfg.dt + x.z;
    y[3] = (a.y * 10.0f) * cfg.dt + x.w;
#pragma unroll
    for (int c = 0; c < SD; ++c) y[c] = clampf_nan(y[c], cfg.state_lo[c], cfg.state_hi[c]);
    if (lane < NA) *reinterpret_cast<float4*>(lds + A0 + nxt + lane * SD) = make_float4(y[0], y[1], y[2], y[3]);
    // ---- distances on the current rows, one root for every lane
    const float2 pa = *reinterpret_cast<const float2*>(lds + oa + (ca ? cur : 0));
    const float2 pb = *reinterpret_cast<const float2*>(lds + ob + (cb ? cur : 0));
    const float sq = anorm ? sq2(a.x, a.y) : sq2(pa.x - pb.x, pa.y - pb.y);
    float v = sqrtf(sq);
    if (diag) v = v + 1e6f;
    float m = dvalid ? v : __builtin_inff();
    m = __builtin_elementwise_minimum(m, wv::dppb<0xB1>(m));
    m = __builtin_elementwise_minimum(m, wv::dppb<0x4E>(m));
    // ---- costs (lane 2 i + h) and reward (lane 0), mpe/base.py:164-191 / get_reward
    float md[NA], dg[NA], mo[NA], a2[NA];
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      md[i] = wv::rlf(m, 4 * i);
      dg[i] = wv::rlf(m, 12 + 4 * i);
      mo[i] = wv::rlf(m, 24 + 4 * i);
      const float an = wv::rlf(v, 36 + i);
      a2[i] = an * an;
    }
    {
      const int ci = lane >> 1;
      const float mdi = ci == 0 ? md[0] : (ci == 1 ? md[1] : md[2]);
      const float moi = ci == 0 ? mo[0] : (ci == 1 ? mo[1] : mo[2]);
      float c = (lane & 1) == 0 ? cfg.c_agent_cost - mdi : cfg.c_obs_cost - moi;
      c = c <= 0.0f ? c - 0.5f : c + 0.5f;
      c = c < -1.0f ? -1.0f : c;  // jnp.clip(cost, a_min=-1.0)
      if (lane < 2 * NA) cost_e[t * r.t_cost + lane] = c;
    }
    if (lane == 0) {
      float sd_ = 0.0f, sf = 0.0f, sa = 0.0f;
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        sd_ = sd_ + dg[i];
        sf = sf + (dg[i] > cfg.dist2goal ? 1.0f : 0.0f);
        sa = sa + a2[i];
      }
      const float nn = (float)NA;
      float rw = 0.0f - (sd_ / nn) * 0.01f;
      rw = rw - (sf / nn) * 0.001f;
      rw = rw - (sa / nn) * 0.0001f;
      reward_e[t * r.t_reward] = rw;
    }
    wv::wave_sync();  // next agent rows visible
    // ---- graph t + 1 (write_graph_mpe)
    float* no = nodes_e + (int64_t)(t + 1) * r.t_nodes;
    float* so = states_e + (int64_t)(t + 1) * r.t_states;
    float* eo = edges_e + (int64_t)(t + 1) * r.t_edges;
    int32_t* ro = recv_e + (int64_t)(t + 1) * r.t_index;
    int32_t* sno = send_e + (int64_t)(t + 1) * r.t_index;
    auto row_off = [&](int rr) {
      return rr < NA ? A0 + nxt + rr * SD : (rr < 2 * NA ? GL + (rr - NA) * SD : (rr < PAD ? OB + (rr - 2 * NA) * SD : A0 + nxt));
    };
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int rr = nr[k], c = nc[k];
      const float xv = lds[row_off(rr) + (c < SD ? c : 0)];
      const int hot = rr < NA ? SD + 2 : (rr < 2 * NA ? SD + 1 : SD);
      const float val = rr == PAD ? 0.0f : (c < SD ? xv : (c == hot ? 1.0f : 0.0f));
      if (lane + 64 * k < N * ND) no[lane + 64 * k] = val;
    }
    {
      const float xv = lds[row_off(sr) + sc];
      if (lane < N * SD) so[lane] = sr == PAD ? -1.0f : xv;
    }
    {
      const float4 si = *reinterpret_cast<const float4*>(lds + A0 + nxt + ei * SD);
      const float4 sj = *reinterpret_cast<const float4*>(
          lds + (ekind == 0 ? A0 + nxt + ej * SD : (ekind == 1 ? GL + ej * SD : OB + ej * SD)));
      const float f0 = si.x - sj.x, f1 = si.y - sj.y, f2 = si.z - sj.z, f3 = si.w - sj.w;
      const float d2 = sq2(si.x - sj.x, si.y - sj.y);
      bool msk;
      if (ekind == 0) msk = ei == ej ? ((d2 == 0.0f) & (cfg.c_self_dist < cfg.comm_radius)) : (d2 < cfg.t2_comm);
      else msk = ekind == 1 ? true : (d2 < cfg.t2_comm);
      const int sv0 = ekind == 0 ? ej : (ekind == 1 ? NA + ej : 2 * NA + ej);
      if (lane < E) {
        reinterpret_cast<float4*>(eo)[lane] = make_float4(f0, f1, f2, f3);
        ro[lane] = msk ? ei : PAD;
        sno[lane] = msk ? sv0 : PAD;
      }
    }
  }
}
}  // namespace mpew
}  // namespace wv

// ---- LidarOmniTarget (dgppo/env/lidar_env/lidar_omni_target.py) --------------------------------
// Omni-wheel agents [x, y, cos th, sin th, vx, vy, omega], actions [ax, ay, alpha], 5 costs
// (agent collision, obstacle collision, FoV angle / max range / min distance on the chain i -> i+1),
// 10-wide edge features [s_i - s_j (7) | critical i -> i+1 | ||p_j^i|| | i_x_j] with
// p_j^i = R_i^T (p_j - p_i).  One workgroup per env (any n, O, R, k); the LiDAR is the Lidar
// engines' lidar_scan.  Same graph layout as LidarTarget (own-goal edges), edge rows 10 wide.

// nodes (N, 10), states (N, 7), edges (E, 10), receivers / senders (E) of the graph on `nxt`
__device__ void write_graph_omni(const dgppo_env_cfg& cfg, int n, int k, bool lidar, const float* nxt,
                                 const float* goal, const float* hits, GraphOut out, int tid, int nthr) {
  constexpr int SD = kOmniSD, ND = SD + 3, ED = kOmniED;
  const int nh = lidar ? n * k : 0;
  const int N = 2 * n + nh + 1, E = n * n + n + nh, pad = N - 1;
#pragma unroll 1
  for (int idx = tid; idx < N * ND; idx += nthr) {
    const int r = idx / ND, c = idx - (idx / ND) * ND;
    float v = 0.0f;
    if (r < n) v = c < SD ? nxt[r * SD + c] : (c == SD + 2 ? 1.0f : 0.0f);
    else if (r < 2 * n) v = c < SD ? goal[(r - n) * SD + c] : (c == SD + 1 ? 1.0f : 0.0f);
    else if (r < 2 * n + nh) v = c < 2 ? hits[(r - 2 * n) * 2 + c] : (c == SD ? 1.0f : 0.0f);
    out.nodes[idx] = v;
  }
#pragma unroll 1
  for (int idx = tid; idx < N * SD; idx += nthr) {
    const int r = idx / SD, c = idx - (idx / SD) * SD;
    float v;
    if (r < n) v = nxt[r * SD + c];
    else if (r < 2 * n) v = goal[(r - n) * SD + c];
    else if (r < 2 * n + nh) v = c < 2 ? hits[(r - 2 * n) * 2 + c] : 0.0f;
    else v = -1.0f;
    out.states[idx] = v;
  }
#pragma unroll 1
  for (int e = tid; e < E; e += nthr) {
    float f[ED];
#pragma unroll
    for (int c = 0; c < ED; ++c) f[c] = 0.0f;
    int rv, sv;
    if (e < n * n) {  // agent-agent (lidar_omni_target.py:352-422)
      const int i = e / n, j = e - (e / n) * n;
      const float* si = nxt + i * SD;
      const float* sj = nxt + j * SD;
#pragma unroll
      for (int c = 0; c < SD; ++c) f[c] = si[c] - sj[c];
      f[7] = j == i + 1 ? 1.0f : 0.0f;
      const float gx = -(si[0] - sj[0]), gy = -(si[1] - sj[1]);  // p_j - p_i
      const float lx = si[2] * gx + si[3] * gy;                 // R_i^T (p_j - p_i)
      const float ly = (-si[3]) * gx + si[2] * gy;
      f[8] = norm2(lx, ly);
      f[9] = lx;
      const float dx = si[0] - sj[0], dy = si[1] - sj[1];
      const float d2 = dx * dx + dy * dy;
      const bool m = i == j ? ((d2 == 0.0f) & (cfg.c_self_dist < cfg.comm_radius)) : (d2 < cfg.t2_comm);
      rv = m ? i : pad;
      sv = m ? j : pad;
    } else if (e < n * n + n) {  // own goal (lidar_omni_target.py:424-443), zero-padded
      const int i = e - n * n;
#pragma unroll
      for (int c = 0; c < SD; ++c) f[c] = nxt[i * SD + c] - goal[i * SD + c];
      rv = i;
      sv = n + i;
    } else {  // hits, masked at comm_radius (lidar_omni_target.py:446-489)
      const int q = e - n * n - n, i = q / k;
      f[0] = nxt[i * SD + 0] - hits[2 * q + 0];
      f[1] = nxt[i * SD + 1] - hits[2 * q + 1];
      const bool m = f[0] * f[0] + f[1] * f[1] < cfg.t2_comm;
      rv = m ? i : pad;
      sv = m ? 2 * n + q : pad;
    }
#pragma unroll
    for (int c = 0; c < ED; ++c) out.edges[(int64_t)e * ED + c] = f[c];
    out.recv[e] = rv;
    out.send[e] = sv;
  }
}

template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void omni_step_kernel(dgppo_env_cfg cfg, dgppo_env_step_io io) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int SD = kOmniSD, NC = kOmniNC;
  const Dims<0, -1, 0, 0> d(cfg);
  const int n = d.n, O = d.O, k = d.k;
  const bool lidar = O > 0;
  const Carve cv(n, SD, O, d.R, k, true);
  const int nh = lidar ? n * k : 0;
  const int n_ob = nh + 1;                                  // hit rows + the origin row (quirk, see oracle)
  const int o_act = cv.total;                               // (n, 3) clipped actions
  const int o_dd = o_act + ((3 * n + 3) & ~3);              // agent-agent distances (n, n)
  const int o_do = o_dd + ((n * n + 3) & ~3);               // agent-obstacle-row distances (n, nh + 1)
  const int o_red = o_do + ((n * n_ob + 3) & ~3);           // reward terms (5, n)
  const int o_fov = o_red + 5 * n;                          // FoV costs (3, n)
  const int tid = threadIdx.x;
  const int64_t env = blockIdx.x;

  // ---- A: stage agent / goal rows, every current hit, obstacles, clipped actions ------------------
  const float* st = io.states + env * io.states_stride;
  for (int idx = tid; idx < 2 * n * SD; idx += BLOCK) lds[cv.cur + idx] = st[idx];
  for (int idx = tid; idx < nh * 2; idx += BLOCK) lds[cv.curhit + idx] = st[(2 * n + (idx >> 1)) * SD + (idx & 1)];
  if (lidar) {
    const float* ob = io.obstacles + env * io.obstacles_stride;
    for (int idx = tid; idx < O * DGPPO_OBST_FIELDS; idx += BLOCK) lds[cv.obst + idx] = ob[idx];
  }
  const float* ac = io.action + env * io.action_stride;
  for (int idx = tid; idx < 3 * n; idx += BLOCK) {  // action_lim (lidar_omni_target.py:511-521)
    const float lim = (idx % 3) == 2 ? 1000.0f : 1.0f;
    lds[o_act + idx] = clampf_nan(ac[idx], -lim, lim);
  }
  __syncthreads();

  // ---- B: dynamics + per-agent reward terms + FoV costs; pairwise distance tasks ------------------
  const float* cur = lds + cv.cur;
  const float* goal = cur + n * SD;
  const int n_task = n + n * n + n * n_ob;
#pragma unroll 1
  for (int q = tid; q < n_task; q += BLOCK) {
    if (q < n) {
      const int i = q;
      const float* x = cur + i * SD;
      const float* a = lds + o_act + 3 * i;
      const float dt = cfg.dt;
      // agent_step_euler (lidar_omni_target.py:146-197)
      const float acc_x = a[0] * 10.0f, acc_y = a[1] * 10.0f, alpha = a[2] * 5.0f;
      const float theta = atan2_32(x[3], x[2]);
      const float new_theta = theta + x[6] * dt;
      float sn, cn;
      sincos32(new_theta, &sn, &cn);
      const float y[SD] = {x[0] + x[4] * dt, x[1] + x[5] * dt, cn, sn, x[4] + acc_x * dt, x[5] + acc_y * dt,
                           x[6] + alpha * dt};
#pragma unroll
      for (int c = 0; c < SD; ++c) lds[cv.nxt + i * SD + c] = clampf_nan(y[c], cfg.state_lo[c], cfg.state_hi[c]);
      // get_reward terms (lidar_omni_target.py:295-336) on the pre-step graph
      const float dg = norm2(goal[i * SD] - x[0], goal[i * SD + 1] - x[1]);
      const float an = norm2(a[0], a[1]);
      lds[o_red + i] = dg;
      lds[o_red + n + i] = dg > cfg.dist2goal ? 1.0f : 0.0f;
      lds[o_red + 2 * n + i] = an * an;
      lds[o_red + 3 * n + i] = a[2] * a[2];
      lds[o_red + 4 * n + i] = x[6] * x[6];
      // FoV costs on the chain i -> i+1 (lidar_omni_target.py:577-631); the last agent is safe (-1)
      float ha = -1.0f, hr = -1.0f, hc = -1.0f;
      if (i + 1 < n) {
        const float* xj = cur + (i + 1) * SD;
        const float dx = xj[0] - x[0], dy = xj[1] - x[1];
        const float lx = x[2] * dx + x[3] * dy;
        const float ly = (-x[3]) * dx + x[2] * dy;
        const float nrm = norm2(lx, ly);
        ha = cfg.c_cos_fov * (nrm + 1e-8f) - lx;
        hr = nrm - cfg.fov_rmax;
        hc = cfg.fov_dmin - nrm;
      }
      lds[o_fov + i] = ha;
      lds[o_fov + n + i] = hr;
      lds[o_fov + 2 * n + i] = hc;
      continue;
    }
    int t = q - n;
    if (t < n * n) {  // agent-agent, eye * 1e6 on the diagonal
      const int i = t / n, j = t - (t / n) * n;
      float dj = norm2(cur[i * SD] - cur[j * SD], cur[i * SD + 1] - cur[j * SD + 1]);
      if (i == j) dj = dj + 1e6f;
      lds[o_dd + t] = dj;
      continue;
    }
    t -= n * n;  // agent i vs obstacle row h: ||row_h - p_i||, row nh = the origin
    const int i = t / n_ob, h = t - (t / n_ob) * n_ob;
    const float ox = h < nh ? lds[cv.curhit + 2 * h] : 0.0f;
    const float oy = h < nh ? lds[cv.curhit + 2 * h + 1] : 0.0f;
    lds[o_do + t] = norm2(ox - cur[i * SD], oy - cur[i * SD + 1]);
  }
  if (lidar) stage_edge_vectors(O, lds, cv, tid, BLOCK);
  __syncthreads();

  // ---- C: costs (5 per agent, margin 0.1, clip [-1, 1]); is-inside at the next state -------------
  for (int i = tid; i < n; i += BLOCK) {
    float md = lds[o_dd + i * n];
    for (int j = 1; j < n; ++j) md = min_nan(md, lds[o_dd + i * n + j]);
    float c[NC];
    c[0] = cfg.c_agent_cost - md;
    c[1] = 0.0f;
    if (lidar) {
      float mo = lds[o_do + i * n_ob];
      for (int h = 1; h < n_ob; ++h) mo = min_nan(mo, lds[o_do + i * n_ob + h]);
      c[1] = cfg.c_obs_cost - mo;
    }
    c[2] = lds[o_fov + i];
    c[3] = lds[o_fov + n + i];
    c[4] = lds[o_fov + 2 * n + i];
#pragma unroll
    for (int q = 0; q < NC; ++q) {
      const float v = c[q] <= 0.0f ? c[q] - 0.1f : c[q] + 0.1f;
      io.cost[env * io.cost_stride + i * NC + q] = clampf_nan(v, -1.0f, 1.0f);
    }
    if (lidar) agent_is_inside(O, lds, cv, SD, i);
  }
  __syncthreads();

  // ---- D: reward (sequential means), LiDAR of the next state -----------------------------------
  if (tid == 0) {
    float s[5] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    for (int i = 0; i < n; ++i)
#pragma unroll
      for (int q = 0; q < 5; ++q) s[q] = s[q] + lds[o_red + q * n + i];
    const float nn = (float)n;
    float r = 0.0f - (s[0] / nn) * 0.01f;
    r = r - (s[1] / nn) * 0.001f;
    r = r - (s[2] / nn) * 0.0001f;
    r = r - (s[3] / nn) * cfg.rot_pen;
    r = r - ((s[4] / nn) * cfg.rot_pen) * 0.5f;
    io.reward[env * io.reward_stride] = r;
  }
  if (lidar) {
    lidar_scan<SD>(d, io.ray_dirs, lds, cv, tid, BLOCK);
    __syncthreads();
  }

  // ---- E: the next graph ------------------------------------------------------------------------
  GraphOut out;
  out.nodes = io.nodes + env * io.nodes_stride;
  out.edges = io.edges + env * io.edges_stride;
  out.states = io.out_states + env * io.out_states_stride;
  out.recv = io.receivers + env * io.edge_index_stride;
  out.send = io.senders + env * io.edge_index_stride;
  write_graph_omni(cfg, n, k, lidar, lds + cv.nxt, goal, lds + cv.hits, out, tid, BLOCK);
}

static size_t omni_step_lds_bytes(const dgppo_env_cfg& c) {
  const Carve cv(c.n_agents, kOmniSD, c.n_obs, c.n_rays, c.top_k, true);
  const int n = c.n_agents, nh = c.n_obs > 0 ? n * c.top_k : 0;
  const size_t fl = cv.total + ((3 * n + 3) & ~3) + ((n * n + 3) & ~3) + ((n * (nh + 1) + 3) & ~3) + 8 * n;
  return fl * sizeof(float);
}

// ---- reset ------------------------------------------------------------------------------------
// Thread 0 draws the obstacles, wave 0 runs the rejection sampler for agents and goals, thread 0 the
// headings (reset is once per episode, amortised over T = 128 steps); then the whole workgroup
// ray-casts and writes the graph.
__device__ bool inside_any(const float* obst, int O, float px, float py, float r) {
  bool in = false;
  for (int o = 0; o < O; ++o) in = in || rect_inside(obst + o * DGPPO_OBST_FIELDS, px, py, r);
  return in;
}

__device__ void make_rectangle(float* rec, float cx, float cy, float w, float h, float th) {
  float s, c;
  sincos32(th, &s, &c);
  const float hw = w / 2.0f, hh = h / 2.0f;
  const float bx[4] = {hw, -hw, -hw, hw};
  const float by[4] = {hh, hh, -hh, -hh};
  rec[0] = cx;
  rec[1] = cy;
  rec[2] = w;
  rec[3] = h;
  rec[4] = th;
  rec[5] = c;
  rec[6] = s;
  rec[7] = 0.0f;
  for (int p = 0; p < 4; ++p) {
    rec[8 + 2 * p] = (c * bx[p] + (-s) * by[p]) + cx;
    rec[9 + 2 * p] = (s * bx[p] + c * by[p]) + cy;
  }
}

// get_node_goal_rng (env/utils.py:139-244; dim 2, max_travel None; oracle/env.py node_goal_rng), the
// reference's sequential rejection sampler, run by one 64-lane wave, exactly: within a phase (agent i, then goal i) the placed
// points do not change and candidate t of the phase is the Philox draw pair at count p + 2 t, so lane l
// tests candidate b + l of batch b and the phase takes the lowest accepted index (ballot); candidate
// kMaxIter is taken regardless, as the sequential loop does.  Returns the phase's rejection count.
constexpr int kSampTab = 256;  // candidate pairs drawn ahead by the whole workgroup (reset LDS tail)

__device__ int sample_phase(const Rng& rng, uint32_t& count, uint32_t count0, const float* tab, bool goals,
                            float side, int n, float min_dist, float r_in, const float* obst, int O,
                            const float* pts, float& ox, float& oy) {
  constexpr int kMaxIter = 1024;
  const int lane = threadIdx.x & 63;
  for (int b = 0;; b += 64) {
    const int t = b + lane;
    const uint32_t k = (count - count0) / 2u + (uint32_t)t;  // candidate pair index since count0
    float cx, cy;
    if (k < (uint32_t)kSampTab) {
      cx = tab[2 * k];
      cy = tab[2 * k + 1];
    } else {
      Rng r = rng;
      r.count = count + 2u * (uint32_t)t;
      cx = r.uniform(0.0f, side);
      cy = r.uniform(0.0f, side);
    }
    float dmin = 0.0f;
    for (int j = 0; j < n; ++j) {
      const float d = norm2(pts[2 * j] - cx, pts[2 * j + 1] - cy);
      dmin = j == 0 ? d : min_nan(dmin, d);
    }
    bool bad = (dmin <= min_dist) || inside_any(obst, O, cx, cy, r_in);
    if (goals) bad = bad || cx < 0.0f || cy < 0.0f || cx > side || cy > side;
    const uint64_t m = __ballot((t <= kMaxIter) && (!bad || t == kMaxIter));
    if (m) {
      const int f = __ffsll((unsigned long long)m) - 1;
      ox = __shfl(cx, f, 64);
      oy = __shfl(cy, f, 64);
      count += 2u * (uint32_t)(b + f + 1);
      return b + f;
    }
  }
}

// max{x : sqrtf(x) <= r} (-1 when no x >= 0 qualifies): sqrtf is correctly rounded and monotone, so for a squared
// norm x (>= +0, +inf or NaN) `sqrtf(x) <= r` is `x <= T` exactly (NaN compares false either way).  Found by ulp
// steps from fl(r * r), within a few ulps of T.
__device__ float sq_le_threshold(float r) {
  if (!(r >= 0.0f)) return -1.0f;
  if (r == __builtin_inff()) return __builtin_inff();
  float T = r * r;
  if (T == __builtin_inff()) T = 3.40282347e38f;
  for (int i = 0; i < 16 && !(sqrtf(T) <= r); ++i) T = __uint_as_float(__float_as_uint(T) - 1u);
  for (int i = 0; i < 16; ++i) {
    const float U = __uint_as_float(__float_as_uint(T) + 1u);
    if (!(sqrtf(U) <= r)) break;
    T = U;
  }
  return T;
}

__device__ void node_goal_rng_wave(Rng& rng, const float* tab, float side, int n, float min_dist, float r_in,
                                   const float* obst, int O, float* pos, float* gl) {
  constexpr int kMaxIter = 1024;
  const int lane = threadIdx.x & 63;
  auto clear = [&]() {
    for (int i = lane; i < 2 * n; i += 64) {
      pos[i] = 0.0f;
      gl[i] = 0.0f;
    }
    wv::wave_sync();
  };
  clear();
  uint32_t count = rng.count;
  const uint32_t count0 = count;
  // The table's kSampTab candidates as wave bit masks (lane l holds candidates l + 64 q): rejected by an obstacle
  // (either phase), out of the area (goal phases), within min_dist of a point placed so far or of the origin (the
  // unplaced rows are zeros).  A candidate's distance test is `min_j d_j <= min_dist`, i.e. `any d_j <= min_dist`
  // unless some d_j is NaN (min_nan then makes the minimum NaN and the test false): the masks OR in one ballot per
  // placed point and track NaNs apart, so a phase is a first-set-bit search instead of n distances and O
  // rectangle tests per candidate -- the same first accepted candidate, the same count.  Past the table (or after
  // kMaxIter rejections) sample_phase runs as before.
  static_assert(kSampTab == 256, "4 candidates per lane");
  float tx[4], ty[4];
  uint64_t inobs[4], oob[4], nearA[4], nearG[4], nanA[4], nanG[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    tx[q] = tab[2 * (lane + 64 * q)];
    ty[q] = tab[2 * (lane + 64 * q) + 1];
    inobs[q] = __ballot(inside_any(obst, O, tx[q], ty[q], r_in));
    oob[q] = __ballot(tx[q] < 0.0f || ty[q] < 0.0f || tx[q] > side || ty[q] > side);
  }
  // `norm2(..) <= min_dist` on the squared norms (sq_le_threshold; NaN iff the squared norm is NaN): no root per
  // candidate and placed point
  const float t_le = sq_le_threshold(min_dist);
  auto origin_only = [&]() {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float x = sq2(0.0f - tx[q], 0.0f - ty[q]);
      nearA[q] = nearG[q] = __ballot(x <= t_le);
      nanA[q] = nanG[q] = __ballot(x != x);
    }
  };
  auto add_point = [&](uint64_t (&near)[4], uint64_t (&nan)[4], float px, float py) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float x = sq2(px - tx[q], py - ty[q]);
      near[q] |= __ballot(x <= t_le);
      nan[q] |= __ballot(x != x);
    }
  };
  auto phase = [&](bool goals, const float* pts, const uint64_t (&near)[4], const uint64_t (&nan)[4], float& ox,
                   float& oy) -> int {
    const int s = (int)((count - count0) / 2u);  // this phase's first candidate
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int lo = s - 64 * q;
      if (lo >= 64) continue;
      uint64_t good = ~(inobs[q] | (near[q] & ~nan[q]) | (goals ? oob[q] : 0ull));
      if (lo > 0) good &= ~0ull << lo;
      if (good) {
        const int k = 64 * q + __ffsll((unsigned long long)good) - 1;
        ox = tab[2 * k];
        oy = tab[2 * k + 1];
        count += 2u * (uint32_t)(k - s + 1);
        return k - s;
      }
    }
    return sample_phase(rng, count, count0, tab, goals, side, n, min_dist, r_in, obst, O, pts, ox, oy);
  };
  origin_only();
  int agent_id = 0;
  while (agent_id < n) {
    float cx, cy, gx, gy;
    const int it_agent = phase(false, pos, nearA, nanA, cx, cy);
    if (lane == 0) {
      pos[2 * agent_id] = cx;
      pos[2 * agent_id + 1] = cy;
    }
    add_point(nearA, nanA, cx, cy);
    wv::wave_sync();
    const int it = phase(true, gl, nearG, nanG, gx, gy);
    if (lane == 0) {
      gl[2 * agent_id] = gx;
      gl[2 * agent_id + 1] = gy;
    }
    add_point(nearG, nanG, gx, gy);
    wv::wave_sync();
    ++agent_id;
    if (it_agent >= kMaxIter || it >= kMaxIter) {  // no solution: start over (utils.py:229-232)
      agent_id = 0;
      clear();
      origin_only();
    }
  }
  rng.count = count;
}

template <int ENGINE, int GOAL, int SD, int BLOCK>
__global__ __launch_bounds__(BLOCK) void env_reset_kernel(dgppo_env_cfg cfg, dgppo_env_reset_io io, int states_only) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const bool mpe = ENGINE == DGPPO_ENGINE_MPE;
  const Dims<0, -1, 0, 0> d(cfg);
  const int n = d.n, O = d.O, k = d.k;
  const bool lidar = !mpe && O > 0;
  const Carve cv(n, SD, O, cfg.n_rays, k, !mpe);
  const int tid = threadIdx.x;
  const int64_t env = blockIdx.x;
  float* nxt = lds + cv.nxt;            // sampled agent states
  float* goal = lds + cv.cur + n * SD;  // sampled goal states
  float* third = lds + cv.cur + 2 * n * SD;  // MPE obstacle states
  float* obst = lds + cv.obst;
  __shared__ uint32_t rng_count;
  Rng rng(io.seed_ptr ? *io.seed_ptr : io.seed, (uint32_t)(io.env_offset + env));
  const float area = cfg.area_size;
  float* pos = lds + cv.samp;
  float* gl = pos + 2 * n;
  // obstacles: draw l of the reference's sequence (centres x / y per obstacle, then sizes, then angles) is the
  // Philox word at count l, so thread l draws it (staged in the candidate table, filled only afterwards) and
  // thread o builds rectangle o -- the same values as one thread drawing them in order
  float* tab = lds + cv.total;
  const int n_ob_draws = (!mpe && O > 0) ? 5 * O : 0;
  for (int l = tid; l < n_ob_draws; l += BLOCK) {
    Rng r = rng;
    r.count = (uint32_t)l;
    const float lo = l < 2 * O ? 0.0f : (l < 4 * O ? cfg.obs_len_lo : cfg.obs_theta_lo);
    const float hi = l < 2 * O ? area : (l < 4 * O ? cfg.obs_len_hi : cfg.obs_theta_hi);
    tab[l] = r.uniform(lo, hi);
  }
  __syncthreads();
  for (int o = tid; o < (n_ob_draws > 0 ? O : 0); o += BLOCK)
    make_rectangle(obst + o * DGPPO_OBST_FIELDS, tab[2 * o], tab[2 * o + 1], tab[2 * O + 2 * o], tab[2 * O + 2 * o + 1],
                   tab[4 * O + o]);
  if (tid == 0) rng_count = (uint32_t)n_ob_draws;
  __syncthreads();
  // the first kSampTab candidate pairs of the sampler's stream, drawn by every thread at once
  for (int k = tid; k < kSampTab; k += BLOCK) {
    Rng r = rng;
    r.count = rng_count + 2u * (uint32_t)k;
    tab[2 * k] = r.uniform(0.0f, area);
    tab[2 * k + 1] = r.uniform(0.0f, area);
  }
  __syncthreads();
  if (tid < 64) {  // agent / goal positions: the rejection sampler, one wave wide
    rng.count = rng_count;
    node_goal_rng_wave(rng, tab, area, n, cfg.c_min_dist, cfg.c_inside_r, obst, mpe ? 0 : O, pos, gl);
    if (tid == 0) rng_count = rng.count;
  }
  __syncthreads();
  for (int idx = tid; idx < n * SD; idx += BLOCK) {
    const int i = idx / SD, c = idx - (idx / SD) * SD;
    nxt[idx] = c < 2 ? pos[2 * i + c] : 0.0f;
    goal[idx] = c < 2 ? gl[2 * i + c] : 0.0f;
  }
  __syncthreads();
  if (tid == 0 && (ENGINE == DGPPO_ENGINE_OMNI || mpe)) {
    rng.count = rng_count;
    if (ENGINE == DGPPO_ENGINE_OMNI) {  // chain headings toward the next agent (lidar_omni_target.py:246-272)
      for (int i = 0; i + 1 < n; ++i) {
        const float dx = pos[2 * (i + 1)] - pos[2 * i], dy = pos[2 * (i + 1) + 1] - pos[2 * i + 1];
        const float nrm = norm2(dx, dy) + 1e-8f;
        nxt[i * SD + 2] = dx / nrm;
        nxt[i * SD + 3] = dy / nrm;
      }
      float s, c;  // the last agent (or the only one) draws its heading
      sincos32(rng.uniform(0.0f, 6.28318548202514648438f), &s, &c);
      nxt[(n - 1) * SD + 2] = c;
      nxt[(n - 1) * SD + 3] = s;
    }
    if (mpe) {  // obstacles (mpe/base.py:92-118); the reference loop is unbounded, we cap it
      for (int o = 0; o < O; ++o) {
        float cx = rng.uniform(0.0f, area), cy = rng.uniform(0.0f, area);
        for (int it = 0; it < (1 << 16); ++it) {
          float da = 0.0f, dg = 0.0f;
          for (int j = 0; j < n; ++j) {
            const float d1 = norm2(pos[2 * j] - cx, pos[2 * j + 1] - cy);
            const float d2 = norm2(gl[2 * j] - cx, gl[2 * j + 1] - cy);
            da = j == 0 ? d1 : min_nan(da, d1);
            dg = j == 0 ? d2 : min_nan(dg, d2);
          }
          const bool bad = da <= cfg.c_mpe_obs_agent || dg <= cfg.c_mpe_obs_goal || cx < cfg.c_mpe_obs_lo ||
                           cy < cfg.c_mpe_obs_lo || cx > cfg.c_mpe_obs_hi || cy > cfg.c_mpe_obs_hi;
          if (!bad) break;
          cx = rng.uniform(cfg.c_mpe_obs_lo, cfg.c_mpe_obs_hi);
          cy = rng.uniform(cfg.c_mpe_obs_lo, cfg.c_mpe_obs_hi);
        }
        for (int c = 0; c < SD; ++c) third[o * SD + c] = c == 0 ? cx : (c == 1 ? cy : 0.0f);
      }
    }
  }
  __syncthreads();
  if (ENGINE == DGPPO_ENGINE_BICYCLE) {  // headings: agent i's draw is the Philox word at count rng_count + i
    for (int i = tid; i < n; i += BLOCK) {
      Rng r = rng;
      r.count = rng_count + (uint32_t)i;
      float s, c;
      sincos32(r.uniform(0.0f, 6.28318548202514648438f), &s, &c);
      nxt[i * SD + 2] = c;
      nxt[i * SD + 3] = s;
    }
    __syncthreads();
  }
  if (states_only) {  // the wave step kernel builds the graph from these rows (dgppo_env_reset)
    if (lidar) {
      float* ob = io.obstacles + env * io.obstacles_stride;
      for (int idx = tid; idx < O * DGPPO_OBST_FIELDS; idx += BLOCK) ob[idx] = obst[idx];
    }
    float* so = io.out_states + env * io.out_states_stride;
    for (int idx = tid; idx < 2 * n * SD; idx += BLOCK) so[idx] = idx < n * SD ? nxt[idx] : goal[idx - n * SD];
    return;
  }
  if (lidar) {
    float* ob = io.obstacles + env * io.obstacles_stride;
    for (int idx = tid; idx < O * DGPPO_OBST_FIELDS; idx += BLOCK) ob[idx] = obst[idx];
    for (int i = tid; i < n; i += BLOCK) agent_is_inside(O, lds, cv, SD, i);
    stage_edge_vectors(O, lds, cv, tid, BLOCK);
    __syncthreads();
    lidar_scan<SD>(d, io.ray_dirs, lds, cv, tid, BLOCK);
    __syncthreads();
  }
  GraphOut out;
  out.nodes = io.nodes + env * io.nodes_stride;
  out.edges = io.edges + env * io.edges_stride;
  out.states = io.out_states + env * io.out_states_stride;
  out.recv = io.receivers + env * io.edge_index_stride;
  out.send = io.senders + env * io.edge_index_stride;
  if constexpr (ENGINE == DGPPO_ENGINE_OMNI) {
    write_graph_omni(cfg, n, k, lidar, nxt, goal, lds + cv.hits, out, tid, BLOCK);
  } else {
    const bool vec4 = ((io.edges_stride & 3) == 0) && ((reinterpret_cast<uintptr_t>(io.edges) & 15) == 0);
    write_graph<ENGINE, GOAL, SD>(cfg, d, nxt, goal, mpe ? third : lds + cv.hits, out, vec4, tid, BLOCK);
  }
}

// ---- reference env variants ------------------------------------------------------------------
// lidar_line.py, mpe_line.py, mpe_formation.py, mpe_corridor.py, mpe_connect_spread.py: the SPREAD
// double-integrator envs with `n_goals` goal node rows (2 landmarks / 1 landmark / one per agent),
// reward goals derived from them (landmark2goal), their own resets and (connect) a connectivity cost.
// One wave per env, plain loops: these configs are correctness rows, not the benchmarked path.
// Same fp32 operation order as oracle/env_variants.py (bit-exact, tests/test_env_variants_gpu.py).
namespace var {
constexpr int kT = 64;
constexpr int kLoopCap = 1 << 16;

__device__ __forceinline__ float max_nan(float a, float b) { return (a != a || a >= b) ? a : b; }

// reward goal k of n from the goal node rows (pitch 4): landmark2goal (lidar_line.py:137-142,
// mpe_line.py:112-121, mpe_formation.py:92-96), or the goal node itself
__device__ void reward_goal(const dgppo_env_cfg& c, const float* grow, int k, float* gx, float* gy) {
  const int n = c.n_agents;
  if (c.variant == DGPPO_VARIANT_LINE) {
    const float dx = grow[4] - grow[0], dy = grow[5] - grow[1];
    const float kk = c.goals_inner ? (float)(k + 1) : (float)k;
    const float m = c.goals_inner ? (float)(n + 1) : (float)(n - 1);
    *gx = grow[0] + (kk * dx) / m;
    *gy = grow[1] + (kk * dy) / m;
  } else if (c.variant == DGPPO_VARIANT_FORMATION) {
    // th_k = jnp.linspace(0, 2 pi, n + 1)[k] = 0 * (1 - s) + 2pi * s, s = k / n
    const float sk = (float)k / (float)n;
    const float th = 0.0f * (1.0f - sk) + 6.28318548202514648438f * sk;
    float sn, cs;
    sincos32(th, &sn, &cs);
    *gx = grow[0] + c.goal_radius * cs;
    *gy = grow[1] + c.goal_radius * sn;
  } else {
    *gx = grow[4 * k];
    *gy = grow[4 * k + 1];
  }
}

// get_graph for the variants: agents | goal rows | hits (Lidar) or obstacles (MPE) | pad
__device__ void write_graph_var(const dgppo_env_cfg& c, bool mpe, bool lidar, const float* nxt, const float* grow,
                                const float* third, GraphOut out, int tid, int nthr) {
  constexpr int SD = 4, ND = 7;
  const int n = c.n_agents, ng = c.n_goals, O = c.n_obs, k = c.top_k;
  const int t0 = n + ng;
  const int n_third = mpe ? O : (lidar ? n * k : 0);
  const int N = t0 + n_third + 1, pad = N - 1;
  for (int idx = tid; idx < N * ND; idx += nthr) {
    const int r = idx / ND, col = idx - r * ND;
    float v = 0.0f;
    if (r < n) v = col < SD ? nxt[r * SD + col] : (col == SD + 2 ? 1.0f : 0.0f);
    else if (r < t0) v = col < SD ? grow[(r - n) * SD + col] : (col == SD + 1 ? 1.0f : 0.0f);
    else if (r < t0 + n_third) {
      const int h = r - t0;
      if (mpe) v = col < SD ? third[h * SD + col] : (col == SD ? 1.0f : 0.0f);
      else v = col < 2 ? third[h * 2 + col] : (col == SD ? 1.0f : 0.0f);
    }
    out.nodes[idx] = v;
  }
  for (int idx = tid; idx < N * SD; idx += nthr) {
    const int r = idx / SD, col = idx - r * SD;
    float v;
    if (r < n) v = nxt[r * SD + col];
    else if (r < t0) v = grow[(r - n) * SD + col];
    else if (r < t0 + n_third) {
      const int h = r - t0;
      v = mpe ? third[h * SD + col] : (col < 2 ? third[h * 2 + col] : 0.0f);
    } else v = -1.0f;
    out.states[idx] = v;
  }
  const int n_aa = n * n, n_ag = n * ng;
  const int E = n_aa + n_ag + (mpe ? n * O : n_third);
  const float robs = c.obs_edge_radius;
  for (int e = tid; e < E; e += nthr) {
    float f[4];
    int rv, sv;
    if (e < n_aa) {  // agent-agent: s_i - s_j, mask ||p_i - p_j|| (+ comm + 1 on the diagonal) < comm
      const int i = e / n, j = e - i * n;
      const float* si = nxt + i * SD;
      const float* sj = nxt + j * SD;
      for (int q = 0; q < 4; ++q) f[q] = si[q] - sj[q];
      float dd = norm2(si[0] - sj[0], si[1] - sj[1]);
      if (i == j) dd = dd + c.c_self_dist;
      const bool m = dd < c.comm_radius;
      rv = m ? i : pad;
      sv = m ? j : pad;
    } else if (e < n_aa + n_ag) {  // agent-goal node, all connected
      const int q = e - n_aa, i = q / ng, j = q - i * ng;
      const float* si = nxt + i * SD;
      const float* gj = grow + j * SD;
      for (int t = 0; t < 4; ++t) f[t] = si[t] - gj[t];
      rv = i;
      sv = n + j;
    } else {
      const int q = e - n_aa - n_ag;
      if (mpe) {  // agent-obstacle, mask ||p_i - o|| < obs_edge_radius (comm, or comm * 100)
        const int i = q / O, o = q - i * O;
        const float* si = nxt + i * SD;
        const float* so = third + o * SD;
        for (int t = 0; t < 4; ++t) f[t] = si[t] - so[t];
        const bool m = norm2(si[0] - so[0], si[1] - so[1]) < robs;
        rv = m ? i : pad;
        sv = m ? t0 + o : pad;
      } else {  // agent-lidar (1, k) blocks, mask ||p_i - hit|| < comm - 0.1
        const int i = q / k, h = q - i * k;
        const float* si = nxt + i * SD;
        f[0] = si[0] - third[(i * k + h) * 2 + 0];
        f[1] = si[1] - third[(i * k + h) * 2 + 1];
        f[2] = 0.0f;
        f[3] = 0.0f;
        const bool m = norm2(f[0], f[1]) < c.c_lidar_active;
        rv = m ? i : pad;
        sv = m ? t0 + i * k + h : pad;
      }
    }
    for (int t = 0; t < 4; ++t) out.edges[4 * e + t] = f[t];
    out.recv[e] = rv;
    out.send[e] = sv;
  }
}

// LDS: the base Carve (nxt, obst, evec, lidar tables) + red [8][n] + reward goals [n][2]
__host__ __device__ inline size_t lds_floats(const dgppo_env_cfg& c) {
  const Carve cv(c.n_agents, 4, c.n_obs, c.n_rays, c.top_k, c.engine != DGPPO_ENGINE_MPE);
  return (size_t)cv.total + 10 * (size_t)c.n_agents + 8;
}

template <int ENGINE>
__global__ __launch_bounds__(kT) void step_kernel(dgppo_env_cfg cfg, dgppo_env_step_io io) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int SD = 4;
  constexpr bool mpe = ENGINE == DGPPO_ENGINE_MPE;
  const Dims<0, -1, 0, 0> d(cfg);
  const int n = d.n, O = d.O, k = d.k, ng = cfg.n_goals, t0 = n + ng;
  const bool lidar = !mpe && O > 0;
  const Carve cv(n, SD, O, d.R, k, !mpe);
  float* red = lds + cv.total;  // d2goal, far, |a|^2, min agent dist, c0, c1, c2, min obstacle dist
  float* rg = red + 8 * n;      // reward goals (n, 2)
  const int tid = threadIdx.x;
  const int64_t env = blockIdx.x;
  const float* st = io.states + env * io.states_stride;
  const int n_cur = (t0 + (mpe ? O : 0)) * SD;  // type_states(0), (1) [, (2) MPE obstacles]
  for (int idx = tid; idx < n_cur; idx += kT) lds[cv.cur + idx] = st[idx];
  if (lidar) {
    for (int idx = tid; idx < n * k * 2; idx += kT) lds[cv.curhit + idx] = st[(t0 + (idx >> 1)) * SD + (idx & 1)];
    const float* ob = io.obstacles + env * io.obstacles_stride;
    for (int idx = tid; idx < O * DGPPO_OBST_FIELDS; idx += kT) lds[cv.obst + idx] = ob[idx];
  }
  const float* ac = io.action + env * io.action_stride;
  for (int idx = tid; idx < 2 * n; idx += kT) lds[cv.act + idx] = clampf_nan(ac[idx], -1.0f, 1.0f);
  __syncthreads();
  const float* cur = lds + cv.cur;
  const float* grow = cur + n * SD;
  const float* obs = cur + t0 * SD;
  for (int i = tid; i < n; i += kT) {
    const float* x = cur + i * SD;
    const float* a = lds + cv.act + 2 * i;
    const float y[4] = {x[2] * cfg.dt + x[0], x[3] * cfg.dt + x[1], (a[0] * 10.0f) * cfg.dt + x[2],
                        (a[1] * 10.0f) * cfg.dt + x[3]};
    for (int q = 0; q < SD; ++q) lds[cv.nxt + i * SD + q] = clampf_nan(y[q], cfg.state_lo[q], cfg.state_hi[q]);
    const float an = norm2(a[0], a[1]);
    red[2 * n + i] = an * an;
    float md = 0.0f;
    for (int j = 0; j < n; ++j) {
      float dj = norm2(x[0] - cur[j * SD], x[1] - cur[j * SD + 1]);
      if (i == j) dj = dj + 1e6f;
      md = j == 0 ? dj : min_nan(md, dj);
    }
    red[3 * n + i] = md;
    float mo = 0.0f;
    if (lidar) {
      const float* hc = lds + cv.curhit + 2 * i * k;
      for (int h = 0; h < k; ++h) {
        const float dh = norm2(hc[2 * h] - x[0], hc[2 * h + 1] - x[1]);
        mo = h == 0 ? dh : min_nan(mo, dh);
      }
    } else if (mpe) {
      for (int o = 0; o < O; ++o) {
        const float dh = norm2(x[0] - obs[o * SD], x[1] - obs[o * SD + 1]);
        mo = o == 0 ? dh : min_nan(mo, dh);
      }
    }
    red[7 * n + i] = mo;
    reward_goal(cfg, grow, i, rg + 2 * i, rg + 2 * i + 1);
  }
  __syncthreads();
  for (int i = tid; i < n; i += kT) {  // reward goal i's nearest agent
    float dg = 0.0f;
    for (int a = 0; a < n; ++a) {
      const float da = norm2(rg[2 * i] - cur[a * SD], rg[2 * i + 1] - cur[a * SD + 1]);
      dg = a == 0 ? da : min_nan(dg, da);
    }
    red[i] = dg;
    red[n + i] = dg > cfg.dist2goal ? 1.0f : 0.0f;
  }
  __syncthreads();
  if (tid == 0) {
    float sd_ = 0.0f, sf = 0.0f, sa = 0.0f;
    for (int i = 0; i < n; ++i) {
      sd_ = sd_ + red[i];
      sf = sf + red[n + i];
      sa = sa + red[2 * n + i];
    }
    const float nn = (float)n;
    float r = 0.0f - (sd_ / nn) * 0.01f;
    r = r - (sf / nn) * 0.001f;
    r = r - (sa / nn) * 0.0001f;
    io.reward[env * io.reward_stride] = r;
    const bool connect = cfg.variant == DGPPO_VARIANT_CONNECT;
    float cm = 0.0f;
    if (connect) {  // (min_dist - connect_radius).max()
      for (int i = 0; i < n; ++i) {
        const float ci = red[3 * n + i] - cfg.connect_radius;
        cm = i == 0 ? ci : max_nan(cm, ci);
      }
    }
    const bool upper = !mpe || connect;
    const int nc = connect ? 3 : 2;
    for (int i = 0; i < n; ++i) {
      float cs[3];
      cs[0] = cfg.c_agent_cost - red[3 * n + i];
      cs[1] = (lidar || (mpe && O > 0)) ? cfg.c_obs_cost - red[7 * n + i] : 0.0f;
      cs[2] = cm;
      for (int h = 0; h < nc; ++h) {
        float v = cs[h] <= 0.0f ? cs[h] - 0.5f : cs[h] + 0.5f;
        v = upper ? clampf_nan(v, -1.0f, 1.0f) : (v < -1.0f ? -1.0f : v);
        io.cost[env * io.cost_stride + i * nc + h] = v;
      }
    }
  }
  if (lidar) {
    for (int i = tid; i < n; i += kT) agent_is_inside(O, lds, cv, SD, i);
    stage_edge_vectors(O, lds, cv, tid, kT);
    __syncthreads();
    lidar_scan<SD>(d, io.ray_dirs, lds, cv, tid, kT);
    __syncthreads();
  }
  GraphOut out;
  out.nodes = io.nodes + env * io.nodes_stride;
  out.edges = io.edges + env * io.edges_stride;
  out.states = io.out_states + env * io.out_states_stride;
  out.recv = io.receivers + env * io.edge_index_stride;
  out.send = io.senders + env * io.edge_index_stride;
  write_graph_var(cfg, mpe, lidar, lds + cv.nxt, grow, mpe ? obs : lds + cv.hits, out, tid, kT);
}

// get_node_goal_rng without obstacles, candidates (uniform(0, side), uniform(0, side_y)) (env/utils.py:139-244,
// oracle/env_variants.py node_goal_rng_y), sequential in one thread
__device__ void node_goal_rng_seq(Rng& rng, float side, float side_y, int n, float min_dist, float* pos, float* gl) {
  constexpr int kMaxIter = 1024;
  for (int i = 0; i < 2 * n; ++i) pos[i] = gl[i] = 0.0f;
  int agent_id = 0;
  while (agent_id < n) {
    float cx = rng.uniform(0.0f, side), cy = rng.uniform(0.0f, side_y);
    int it = 0;
    while (true) {
      float dmin = 0.0f;
      for (int j = 0; j < n; ++j) {
        const float dj = norm2(pos[2 * j] - cx, pos[2 * j + 1] - cy);
        dmin = j == 0 ? dj : min_nan(dmin, dj);
      }
      if (!(dmin <= min_dist) || it >= kMaxIter) break;
      ++it;
      cx = rng.uniform(0.0f, side);
      cy = rng.uniform(0.0f, side_y);
    }
    const int it_agent = it;
    pos[2 * agent_id] = cx;
    pos[2 * agent_id + 1] = cy;
    float gx = rng.uniform(0.0f, side), gy = rng.uniform(0.0f, side_y);
    it = 0;
    while (true) {
      float dmin = 0.0f;
      for (int j = 0; j < n; ++j) {
        const float dj = norm2(gl[2 * j] - gx, gl[2 * j + 1] - gy);
        dmin = j == 0 ? dj : min_nan(dmin, dj);
      }
      const bool outside = gx < 0.0f || gy < 0.0f || gx > side || gy > side;
      if (!(dmin <= min_dist || outside) || it >= kMaxIter) break;
      ++it;
      gx = rng.uniform(0.0f, side);
      gy = rng.uniform(0.0f, side_y);
    }
    gl[2 * agent_id] = gx;
    gl[2 * agent_id + 1] = gy;
    ++agent_id;
    if (it_agent >= kMaxIter || it >= kMaxIter) {
      agent_id = 0;
      for (int i = 0; i < 2 * n; ++i) pos[i] = gl[i] = 0.0f;
    }
  }
}

__device__ __forceinline__ float min_dist_row(const float* p, int n, int i) {  // with the eye * 1e6 diagonal
  float md = 0.0f;
  for (int j = 0; j < n; ++j) {
    float dj = norm2(p[2 * i] - p[2 * j], p[2 * i + 1] - p[2 * j + 1]);
    if (i == j) dj = dj + 1e6f;
    md = j == 0 ? dj : min_nan(md, dj);
  }
  return md;
}

template <int ENGINE>
__global__ __launch_bounds__(kT) void reset_kernel(dgppo_env_cfg cfg, dgppo_env_reset_io io) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int SD = 4;
  constexpr bool mpe = ENGINE == DGPPO_ENGINE_MPE;
  const Dims<0, -1, 0, 0> d(cfg);
  const int n = d.n, O = d.O, ng = cfg.n_goals, t0 = n + ng;
  const bool lidar = !mpe && O > 0;
  const Carve cv(n, SD, O, d.R, d.k, !mpe);
  float* grow = lds + cv.cur + n * SD;  // goal node rows
  float* obs = lds + cv.cur + t0 * SD;  // MPE obstacle rows
  float* pos = lds + cv.total;          // sampled agents (n, 2) | goals (n, 2) | reward goals (n, 2)
  float* gl = pos + 2 * n;
  float* rg = gl + 2 * n;
  const int tid = threadIdx.x;
  const int64_t env = blockIdx.x;
  if (tid == 0) {
    Rng rng(io.seed_ptr ? *io.seed_ptr : io.seed, (uint32_t)(io.env_offset + env));
    const float area = cfg.area_size;
    for (int i = 0; i < t0 * SD + (mpe ? O * SD : 0); ++i) lds[cv.cur + i] = 0.0f;
    if (cfg.variant == DGPPO_VARIANT_LINE || cfg.variant == DGPPO_VARIANT_FORMATION) {
      node_goal_rng_seq(rng, area, area, n, cfg.c_agent_cost, pos, gl);
      if (cfg.variant == DGPPO_VARIANT_LINE) {  // lidar_line.py:53-84, mpe_line.py:47-83
        float l0x, l0y;
        if (mpe && cfg.goals_inner) {
          l0x = rng.uniform(0.0f, area);
          l0y = rng.uniform(0.0f, area);
        } else {
          const float u0 = rng.uniform(0.0f, cfg.line_box_x), u1 = rng.uniform(0.0f, cfg.line_box_y);
          const float half = area / 2.0f;
          const float cx = (u0 - half) + 0.0f, cy = (u1 - 0.0f) + cfg.line_off_y;
          int reg = (int)rng.uniform(0.0f, 4.0f);
          reg = reg > 3 ? 3 : reg;
          const float ang = ((float)reg * 3.14159274101257324219f) / 2.0f;
          float sn, cs;
          sincos32(ang, &sn, &cs);
          const float rx = cs * cx + (-sn) * cy, ry = sn * cx + cs * cy;
          l0x = rx + half;
          l0y = ry + half;
        }
        float l1x = rng.uniform(0.0f, area), l1y = rng.uniform(0.0f, area);
        for (int it = 0; it < kLoopCap && norm2(l1x - l0x, l1y - l0y) < cfg.line_min_dist; ++it) {
          l1x = rng.uniform(0.0f, area);
          l1y = rng.uniform(0.0f, area);
        }
        grow[0] = l0x, grow[1] = l0y, grow[SD] = l1x, grow[SD + 1] = l1y;
      } else {  // mpe_formation.py:47-52
        grow[0] = rng.uniform(cfg.formation_lo, cfg.formation_hi);
        grow[1] = rng.uniform(cfg.formation_lo, cfg.formation_hi);
      }
      for (int i = 0; i < n; ++i) reward_goal(cfg, grow, i, rg + 2 * i, rg + 2 * i + 1);
      if (mpe) {  // obstacle rejection against the agents and the reward goals (mpe_line.py:86-112)
        for (int o = 0; o < O; ++o) {
          float cx = rng.uniform(0.0f, area), cy = rng.uniform(0.0f, area);
          for (int it = 0; it < kLoopCap; ++it) {
            float da = 0.0f, dg = 0.0f;
            for (int j = 0; j < n; ++j) {
              const float d1 = norm2(pos[2 * j] - cx, pos[2 * j + 1] - cy);
              const float d2 = norm2(rg[2 * j] - cx, rg[2 * j + 1] - cy);
              da = j == 0 ? d1 : min_nan(da, d1);
              dg = j == 0 ? d2 : min_nan(dg, d2);
            }
            const bool bad = da <= cfg.c_mpe_obs_agent || dg <= cfg.c_mpe_obs_goal || cx < cfg.c_mpe_obs_lo ||
                             cy < cfg.c_mpe_obs_lo || cx > cfg.c_mpe_obs_hi || cy > cfg.c_mpe_obs_hi;
            if (!bad) break;
            cx = rng.uniform(cfg.c_mpe_obs_lo, cfg.c_mpe_obs_hi);
            cy = rng.uniform(cfg.c_mpe_obs_lo, cfg.c_mpe_obs_hi);
          }
          obs[o * SD] = cx;
          obs[o * SD + 1] = cy;
        }
      } else if (O > 0) {  // lidar_line.py:86-122: no agent / goal inside an obstacle inflated by 1.1 r
        float* obst = lds + cv.obst;
        for (int o = 0; o < O; ++o) {
          float* rec = obst + o * DGPPO_OBST_FIELDS;
          for (int it = 0;; ++it) {
            const float cx = rng.uniform(0.0f, area), cy = rng.uniform(0.0f, area);
            const float w = rng.uniform(cfg.obs_len_lo, cfg.obs_len_hi), h = rng.uniform(cfg.obs_len_lo, cfg.obs_len_hi);
            const float th = rng.uniform(0.0f, 3.14159274101257324219f);
            make_rectangle(rec, cx, cy, w, h, th);
            bool in = false;
            for (int j = 0; j < n; ++j)
              in = in || rect_inside(rec, pos[2 * j], pos[2 * j + 1], cfg.c_obs_inflate) ||
                   rect_inside(rec, rg[2 * j], rg[2 * j + 1], cfg.c_obs_inflate);
            if (!in || it >= kLoopCap) break;
          }
        }
      }
    } else {  // corridor (mpe_corridor.py:40-53) / connect (mpe_connect_spread.py:47-94)
      const bool connect = cfg.variant == DGPPO_VARIANT_CONNECT;
      for (int it = 0;; ++it) {
        node_goal_rng_seq(rng, area, cfg.sample_side_y, n, connect ? cfg.c_connect_min : cfg.c_agent_cost, pos, gl);
        for (int j = 0; j < n; ++j) gl[2 * j + 1] = gl[2 * j + 1] + cfg.goal_shift_y;
        if (!connect) break;
        bool bad = false;
        for (int i = 0; i < n; ++i) {
          const float ma = min_dist_row(pos, n, i), mg = min_dist_row(gl, n, i);
          bad = bad || ma > cfg.connect_radius || ma < cfg.c_agent_cost || mg > cfg.connect_radius;
        }
        if (!bad || it + 1 >= kLoopCap) break;
      }
      for (int j = 0; j < n; ++j) grow[j * SD] = gl[2 * j], grow[j * SD + 1] = gl[2 * j + 1];
      if (connect) {
        obs[0] = rng.uniform(cfg.obs_radius, cfg.obs_x_hi);
        obs[1] = area / 2.0f;
      } else {
        obs[0] = cfg.obs_radius, obs[1] = area / 2.0f;
        obs[SD] = cfg.obs_x_hi, obs[SD + 1] = area / 2.0f;
      }
    }
    for (int i = 0; i < n; ++i)
      for (int q = 0; q < SD; ++q) lds[cv.nxt + i * SD + q] = q < 2 ? pos[2 * i + q] : 0.0f;
  }
  __syncthreads();
  if (lidar) {
    float* ob = io.obstacles + env * io.obstacles_stride;
    for (int idx = tid; idx < O * DGPPO_OBST_FIELDS; idx += kT) ob[idx] = lds[cv.obst + idx];
    for (int i = tid; i < n; i += kT) agent_is_inside(O, lds, cv, SD, i);
    stage_edge_vectors(O, lds, cv, tid, kT);
    __syncthreads();
    lidar_scan<SD>(d, io.ray_dirs, lds, cv, tid, kT);
    __syncthreads();
  }
  GraphOut out;
  out.nodes = io.nodes + env * io.nodes_stride;
  out.edges = io.edges + env * io.edges_stride;
  out.states = io.out_states + env * io.out_states_stride;
  out.recv = io.receivers + env * io.edge_index_stride;
  out.send = io.senders + env * io.edge_index_stride;
  write_graph_var(cfg, mpe, lidar, lds + cv.nxt, grow, mpe ? obs : lds + cv.hits, out, tid, kT);
}
}  // namespace var

// ---- host dispatch --------------------------------------------------------------------------
static int validate(const dgppo_env_cfg* c) {
  if (!c) return DGPPO_EINVAL;
  if (vmas::is_vmas(c)) return vmas::validate(c);
  if (c->engine < 0 || c->engine > 3 || c->goal_mode < 0 || c->goal_mode > 1) return DGPPO_EINVAL;
  if (c->n_agents < 1 || c->n_agents > kMaxAgents || c->n_obs < 0 || c->n_obs > kMaxObs) return DGPPO_EINVAL;
  if (c->engine == DGPPO_ENGINE_OMNI && c->goal_mode != DGPPO_GOAL_TARGET) return DGPPO_EINVAL;
  if (c->variant < DGPPO_VARIANT_NONE || c->variant > DGPPO_VARIANT_CONNECT) return DGPPO_EINVAL;
  if (c->variant != DGPPO_VARIANT_NONE) {  // variants: SPREAD double integrators; Lidar only for the line
    if (c->goal_mode != DGPPO_GOAL_SPREAD || (c->engine != DGPPO_ENGINE_MPE && c->engine != DGPPO_ENGINE_LIDAR))
      return DGPPO_EINVAL;
    if (c->engine == DGPPO_ENGINE_LIDAR && c->variant != DGPPO_VARIANT_LINE) return DGPPO_EINVAL;
    if (c->n_goals < 1 || c->n_goals > c->n_agents) return DGPPO_EINVAL;
    if (c->variant == DGPPO_VARIANT_LINE && c->n_goals != 2) return DGPPO_EINVAL;
    if (c->variant == DGPPO_VARIANT_FORMATION && c->n_goals != 1) return DGPPO_EINVAL;
  } else if (c->n_goals != 0 && c->n_goals != c->n_agents) {
    return DGPPO_EINVAL;
  }
  const int sd = c->engine == DGPPO_ENGINE_BICYCLE ? 5 : (c->engine == DGPPO_ENGINE_OMNI ? 7 : 4);
  if (c->state_dim != sd || c->node_dim != sd + 3) return DGPPO_EINVAL;
  if (c->engine != DGPPO_ENGINE_MPE && c->n_obs > 0) {
    if (c->n_rays < 1 || c->n_rays > kMaxRays || c->top_k < 1 || c->top_k > c->n_rays) return DGPPO_EINVAL;
  }
  return 0;
}

// Step-kernel selection: 0 = auto (wave-per-env kernel where the config allows), 1 = the
// workgroup-per-env kernel everywhere.  Initialised from DGPPO_ENV_STEP_KERNEL=block|auto, changed
// by dgppo_env_set_step_kernel (A/B timing and kernel-vs-kernel parity tests).
static int g_step_kernel = -1;
static bool wave_step_enabled() {
  if (g_step_kernel < 0) {
    const char* v = getenv("DGPPO_ENV_STEP_KERNEL");
    g_step_kernel = (v && strcmp(v, "block") == 0) ? 1 : 0;
  }
  return g_step_kernel == 0;
}

// ---- launch helpers ---------------------------------------------------------------------------
template <int ENGINE, int GOAL, int SD, int BLOCK, int NA, int NO, int NR, int NK>
static void launch_step(const dgppo_env_cfg& c, const dgppo_env_step_io& io, size_t shmem, hipStream_t s) {
  hipLaunchKernelGGL((env_step_kernel<ENGINE, GOAL, SD, BLOCK, NA, NO, NR, NK>), dim3((unsigned)io.n_env),
                     dim3(BLOCK), shmem, s, c, io);
}

template <int ENGINE, int GOAL, int SD, int BLOCK, int NA, int NO, int NR, int NK>
static void launch_rollout_block(const dgppo_env_cfg& c, const dgppo_env_rollout_io& r, size_t shmem, hipStream_t s,
                                 int stage) {
  hipLaunchKernelGGL((env_rollout_block_kernel<ENGINE, GOAL, SD, BLOCK, NA, NO, NR, NK>), dim3((unsigned)r.step.n_env),
                     dim3(BLOCK), shmem, s, c, r, stage);
}

// the same compile-time size selection as dispatch_step_sized
template <int ENGINE, int GOAL, int SD>
static void dispatch_rollout_block_sized(const dgppo_env_cfg& c, const dgppo_env_rollout_io& r, size_t shmem,
                                         hipStream_t s, int stage) {
  const int n = c.n_agents, O = c.n_obs, R = c.n_rays, k = c.top_k;
  if (ENGINE == DGPPO_ENGINE_MPE) {
    if (n == 3 && O == 3) return launch_rollout_block<ENGINE, GOAL, SD, 64, 3, 3, 0, 0>(c, r, shmem, s, stage);
    if (n == 3 && O == 0) return launch_rollout_block<ENGINE, GOAL, SD, 64, 3, 0, 0, 0>(c, r, shmem, s, stage);
    return launch_rollout_block<ENGINE, GOAL, SD, 64, 0, -1, 0, 0>(c, r, shmem, s, stage);
  }
  if (R == 32 && k == 8) {
    if (n == 8 && O == 3) return launch_rollout_block<ENGINE, GOAL, SD, 256, 8, 3, 32, 8>(c, r, shmem, s, stage);
    if (n == 32 && O == 8) return launch_rollout_block<ENGINE, GOAL, SD, 256, 32, 8, 32, 8>(c, r, shmem, s, stage);
  }
  if (n * R >= 256) return launch_rollout_block<ENGINE, GOAL, SD, 256, 0, -1, 0, 0>(c, r, shmem, s, stage);
  return launch_rollout_block<ENGINE, GOAL, SD, 128, 0, -1, 0, 0>(c, r, shmem, s, stage);
}

static void dispatch_rollout_block(const dgppo_env_cfg& c, const dgppo_env_rollout_io& r, size_t shmem, hipStream_t s,
                                   int stage) {
  const bool spread = c.goal_mode == DGPPO_GOAL_SPREAD;
  switch (c.engine) {
    case DGPPO_ENGINE_MPE:
      return spread ? dispatch_rollout_block_sized<DGPPO_ENGINE_MPE, DGPPO_GOAL_SPREAD, 4>(c, r, shmem, s, stage)
                    : dispatch_rollout_block_sized<DGPPO_ENGINE_MPE, DGPPO_GOAL_TARGET, 4>(c, r, shmem, s, stage);
    case DGPPO_ENGINE_BICYCLE:
      return spread ? dispatch_rollout_block_sized<DGPPO_ENGINE_BICYCLE, DGPPO_GOAL_SPREAD, 5>(c, r, shmem, s, stage)
                    : dispatch_rollout_block_sized<DGPPO_ENGINE_BICYCLE, DGPPO_GOAL_TARGET, 5>(c, r, shmem, s, stage);
    default:
      return spread ? dispatch_rollout_block_sized<DGPPO_ENGINE_LIDAR, DGPPO_GOAL_SPREAD, 4>(c, r, shmem, s, stage)
                    : dispatch_rollout_block_sized<DGPPO_ENGINE_LIDAR, DGPPO_GOAL_TARGET, 4>(c, r, shmem, s, stage);
  }
}

template <int ENGINE, int GOAL, int SD>
static void dispatch_step_sized(const dgppo_env_cfg& c, const dgppo_env_step_io& io, size_t shmem, hipStream_t s) {
  const int n = c.n_agents, O = c.n_obs, R = c.n_rays, k = c.top_k;
  if (ENGINE == DGPPO_ENGINE_MPE) {
    if (n == 3 && O == 3) return launch_step<ENGINE, GOAL, SD, 64, 3, 3, 0, 0>(c, io, shmem, s);
    if (n == 3 && O == 0) return launch_step<ENGINE, GOAL, SD, 64, 3, 0, 0, 0>(c, io, shmem, s);
    return launch_step<ENGINE, GOAL, SD, 64, 0, -1, 0, 0>(c, io, shmem, s);
  }
  if (R == 32 && k == 8) {  // the BASELINE.json Lidar configs: compile-time sizes
    if (n == 8 && O == 3) return launch_step<ENGINE, GOAL, SD, 256, 8, 3, 32, 8>(c, io, shmem, s);
    if (n == 32 && O == 8) return launch_step<ENGINE, GOAL, SD, 256, 32, 8, 32, 8>(c, io, shmem, s);
  }
  if (n * R >= 256) return launch_step<ENGINE, GOAL, SD, 256, 0, -1, 0, 0>(c, io, shmem, s);
  return launch_step<ENGINE, GOAL, SD, 128, 0, -1, 0, 0>(c, io, shmem, s);
}

static void dispatch_step(const dgppo_env_cfg& c, const dgppo_env_step_io& io, size_t shmem, hipStream_t s) {
  const bool spread = c.goal_mode == DGPPO_GOAL_SPREAD;
  switch (c.engine) {
    case DGPPO_ENGINE_MPE:
      return spread ? dispatch_step_sized<DGPPO_ENGINE_MPE, DGPPO_GOAL_SPREAD, 4>(c, io, shmem, s)
                    : dispatch_step_sized<DGPPO_ENGINE_MPE, DGPPO_GOAL_TARGET, 4>(c, io, shmem, s);
    case DGPPO_ENGINE_BICYCLE:
      return spread ? dispatch_step_sized<DGPPO_ENGINE_BICYCLE, DGPPO_GOAL_SPREAD, 5>(c, io, shmem, s)
                    : dispatch_step_sized<DGPPO_ENGINE_BICYCLE, DGPPO_GOAL_TARGET, 5>(c, io, shmem, s);
    default:
      return spread ? dispatch_step_sized<DGPPO_ENGINE_LIDAR, DGPPO_GOAL_SPREAD, 4>(c, io, shmem, s)
                    : dispatch_step_sized<DGPPO_ENGINE_LIDAR, DGPPO_GOAL_TARGET, 4>(c, io, shmem, s);
  }
}

template <int ENGINE, int GOAL, int SD>
static void dispatch_reset_sized(const dgppo_env_cfg& c, const dgppo_env_reset_io& io, size_t shmem, hipStream_t s,
                                 int states_only) {
  const dim3 grid((unsigned)io.n_env);
  // MPE and states-only resets need one wave (sampler; no workgroup ray cast): 64 threads, so many more
  // envs are resident per CU and their sequential sampling latencies overlap
  if (ENGINE == DGPPO_ENGINE_MPE || states_only)
    hipLaunchKernelGGL((env_reset_kernel<ENGINE, GOAL, SD, 64>), grid, dim3(64), shmem, s, c, io, states_only);
  else if (c.n_agents * c.n_rays >= 256)
    hipLaunchKernelGGL((env_reset_kernel<ENGINE, GOAL, SD, 256>), grid, dim3(256), shmem, s, c, io, states_only);
  else
    hipLaunchKernelGGL((env_reset_kernel<ENGINE, GOAL, SD, 128>), grid, dim3(128), shmem, s, c, io, states_only);
}

static void dispatch_reset(const dgppo_env_cfg& c, const dgppo_env_reset_io& io, size_t shmem, hipStream_t s,
                           int so) {
  const bool spread = c.goal_mode == DGPPO_GOAL_SPREAD;
  switch (c.engine) {
    case DGPPO_ENGINE_MPE:
      return spread ? dispatch_reset_sized<DGPPO_ENGINE_MPE, DGPPO_GOAL_SPREAD, 4>(c, io, shmem, s, so)
                    : dispatch_reset_sized<DGPPO_ENGINE_MPE, DGPPO_GOAL_TARGET, 4>(c, io, shmem, s, so);
    case DGPPO_ENGINE_BICYCLE:
      return spread ? dispatch_reset_sized<DGPPO_ENGINE_BICYCLE, DGPPO_GOAL_SPREAD, 5>(c, io, shmem, s, so)
                    : dispatch_reset_sized<DGPPO_ENGINE_BICYCLE, DGPPO_GOAL_TARGET, 5>(c, io, shmem, s, so);
    case DGPPO_ENGINE_OMNI:
      return dispatch_reset_sized<DGPPO_ENGINE_OMNI, DGPPO_GOAL_TARGET, kOmniSD>(c, io, shmem, s, so);
    default:
      return spread ? dispatch_reset_sized<DGPPO_ENGINE_LIDAR, DGPPO_GOAL_SPREAD, 4>(c, io, shmem, s, so)
                    : dispatch_reset_sized<DGPPO_ENGINE_LIDAR, DGPPO_GOAL_TARGET, 4>(c, io, shmem, s, so);
  }
}

}  // namespace dgppo

using namespace dgppo;

extern "C" int dgppo_abi_version(void) { return DGPPO_ABI_VERSION; }

extern "C" const char* dgppo_build_info(void) {
  return "libdgppo_hip gfx950 abi=" "1" " env_step+env_reset (fp-contract=off)";
}

// smallest fp32 x with sqrtf(x) >= r (IEEE sqrt is correctly rounded and monotone, so for every
// x >= 0: sqrtf(x) < r  <=>  x < t; NaN compares false on both sides)
static float sq_threshold(float r) {
  if (!(r > 0.0f)) return 0.0f;
  if (!(r < INFINITY)) return INFINITY;
  float x = r * r;
  while (x > 0.0f && sqrtf(x) >= r) x = nextafterf(x, 0.0f);
  while (!(sqrtf(x) >= r)) x = nextafterf(x, INFINITY);
  return x;
}

extern "C" int dgppo_env_cfg_finalize(dgppo_env_cfg* c) {
  if (!c) return DGPPO_EINVAL;
  if (vmas::is_vmas(c)) return vmas::finalize(c);
  const bool mpe = c->engine == DGPPO_ENGINE_MPE;
  const int n = c->n_agents;
  const bool omni = c->engine == DGPPO_ENGINE_OMNI;
  c->state_dim = c->engine == DGPPO_ENGINE_BICYCLE ? 5 : (omni ? kOmniSD : 4);
  c->node_dim = c->state_dim + 3;
  c->edge_dim = omni ? kOmniED : 4;
  c->action_dim = omni ? 3 : 2;
  c->n_cost = omni ? kOmniNC : (c->variant == DGPPO_VARIANT_CONNECT ? 3 : 2);
  // goal node rows: the variants' landmarks (line 2, formation 1), else one per agent
  const int ng = (c->variant != DGPPO_VARIANT_NONE && c->n_goals > 0) ? c->n_goals : n;
  c->n_goals = ng;
  const int n_ag = c->goal_mode == DGPPO_GOAL_SPREAD ? n * ng : n;
  if (mpe) {
    c->n_nodes = n + ng + c->n_obs + 1;
    c->n_edges = n * n + n_ag + n * c->n_obs;
  } else {
    const int hits = c->n_obs > 0 ? n * c->top_k : 0;
    c->n_nodes = n + ng + hits + 1;
    c->n_edges = n * n + n_ag + hits;
  }
  const float a = c->area_size;
  if (omni) {  // lidar_omni_target.py:502-509
    const float w = c->omni_max_w;
    const float lo[7] = {0.f, 0.f, -1.f, -1.f, -2.f, -2.f, -w}, hi[7] = {a, a, 1.f, 1.f, 2.f, 2.f, w};
    for (int i = 0; i < 7; ++i) { c->state_lo[i] = lo[i]; c->state_hi[i] = hi[i]; }
    // jnp.cos(jnp.deg2rad(fov_angle_deg)): fp32 product with fp32(pi / 180), cos by the shared fp32 routine
    float sb, cb;
    sincos32(c->fov_angle_deg * (float)(M_PI / 180.0), &sb, &cb);
    c->c_cos_fov = cb;
  } else if (c->engine == DGPPO_ENGINE_BICYCLE) {
    const float lo[5] = {0.f, 0.f, -1.f, -1.f, -0.5f}, hi[5] = {a, a, 1.f, 1.f, 0.5f};
    for (int i = 0; i < 5; ++i) { c->state_lo[i] = lo[i]; c->state_hi[i] = hi[i]; }
  } else {
    const float v = mpe ? 1.0f : 0.5f;
    // corridor / connect: the goals sit past the obstacles, y up to 2 area (mpe_corridor.py:55-58)
    const bool tall = c->variant == DGPPO_VARIANT_CORRIDOR || c->variant == DGPPO_VARIANT_CONNECT;
    const float lo[5] = {0.f, 0.f, -v, -v, 0.f}, hi[5] = {a, tall ? 2.0f * a : a, v, v, 0.f};
    for (int i = 0; i < 5; ++i) { c->state_lo[i] = lo[i]; c->state_hi[i] = hi[i]; }
  }
  if (c->obs_edge_radius == 0.f) c->obs_edge_radius = c->comm_radius;
  const double r = c->car_radius, orr = c->obs_radius, cr = c->comm_radius;
  if (c->c_agent_cost == 0.f) c->c_agent_cost = (float)(r * 2);
  if (c->c_obs_cost == 0.f) c->c_obs_cost = (float)(mpe ? r + orr : r);
  if (c->c_self_dist == 0.f) c->c_self_dist = (float)(cr + 1);
  if (c->c_lidar_active == 0.f) c->c_lidar_active = (float)(cr - 0.1);
  const double md = mpe ? 2 * r : 2.2 * r;
  if (c->c_min_dist == 0.f) c->c_min_dist = (float)md;
  if (c->c_inside_r == 0.f) c->c_inside_r = (float)(md / 2);
  if (c->c_mpe_obs_agent == 0.f) c->c_mpe_obs_agent = (float)(r + orr);
  if (c->c_mpe_obs_goal == 0.f) c->c_mpe_obs_goal = (float)(r * 2 + orr);
  if (c->c_mpe_obs_lo == 0.f) c->c_mpe_obs_lo = (float)(r * 3);
  if (c->c_mpe_obs_hi == 0.f) c->c_mpe_obs_hi = (float)(c->area_size - r * 3);
  c->t2_comm = sq_threshold(c->comm_radius);
  c->t2_lidar = sq_threshold(c->c_lidar_active);
  return validate(c);
}

extern "C" int dgppo_ray_table(int32_t n_rays, float sense_range, float* out) {
  if (n_rays < 1 || !out) return DGPPO_EINVAL;
  // jnp.linspace(start, stop, R): start * (1 - i/div) + stop * (i/div), endpoint = stop
  const float start = (float)(-M_PI);
  const float stop = (float)(M_PI - 2 * M_PI / n_rays);
  for (int i = 0; i < n_rays; ++i) {
    float th;
    if (n_rays == 1) th = start;
    else if (i == n_rays - 1) th = stop;
    else {
      const float step = (float)i / (float)(n_rays - 1);
      th = start * (1.0f - step) + stop * step;
    }
    float s, c;
    sincos32(th, &s, &c);
    out[2 * i + 0] = c * sense_range;
    out[2 * i + 1] = s * sense_range;
  }
  return 0;
}

extern "C" int dgppo_env_set_step_kernel(int mode) {
  if (mode < 0 || mode > 1) return DGPPO_EINVAL;
  wave_step_enabled();
  const int prev = g_step_kernel;
  g_step_kernel = mode;
  return prev;
}

static bool wave_bufs_aligned(const dgppo_env_cfg* cfg, const float* edges, int64_t edges_stride, int64_t t_edges,
                              const float* states, int64_t states_stride, int64_t t_states);

extern "C" int dgppo_env_step(const dgppo_env_cfg* cfg, const dgppo_env_step_io* io, void* stream) {
  if (validate(cfg) || !io || io->n_env < 0) return DGPPO_EINVAL;
  if (vmas::is_vmas(cfg)) return vmas::step(cfg, io, stream);
  if (io->n_env == 0) return 0;
  if (!io->states || !io->action || !io->nodes || !io->edges || !io->out_states || !io->receivers ||
      !io->senders || !io->reward || !io->cost)
    return DGPPO_EINVAL;
  const bool lidar = cfg->engine != DGPPO_ENGINE_MPE && cfg->n_obs > 0;
  if (lidar && (!io->obstacles || !io->ray_dirs)) return DGPPO_EINVAL;
  if (cfg->variant != DGPPO_VARIANT_NONE) {
    const size_t sh = var::lds_floats(*cfg) * sizeof(float);
    if (sh > 64 * 1024) return DGPPO_EINVAL;
    if (cfg->engine == DGPPO_ENGINE_MPE)
      hipLaunchKernelGGL(var::step_kernel<DGPPO_ENGINE_MPE>, dim3((unsigned)io->n_env), dim3(var::kT), sh,
                         (hipStream_t)stream, *cfg, *io);
    else
      hipLaunchKernelGGL(var::step_kernel<DGPPO_ENGINE_LIDAR>, dim3((unsigned)io->n_env), dim3(var::kT), sh,
                         (hipStream_t)stream, *cfg, *io);
    return (int)hipGetLastError();
  }
  const bool wave_shape = lidar && cfg->n_agents == wv::NA && cfg->n_rays == wv::NR && cfg->top_k == wv::NK &&
                          cfg->n_obs == 3 && wave_step_enabled() &&
                          wave_bufs_aligned(cfg, io->edges, io->edges_stride, 0, io->out_states, io->out_states_stride, 0);
  if (cfg->engine == DGPPO_ENGINE_OMNI && wave_shape) {
    const size_t sh = 4 * sizeof(float) * wv::Carve<kOmniSD, 3>::total;
    hipLaunchKernelGGL((wv::lidar_step_wave_kernel<DGPPO_ENGINE_OMNI, DGPPO_GOAL_TARGET, kOmniSD, 3>),
                       dim3((unsigned)((io->n_env + 3) / 4)), dim3(256), sh, (hipStream_t)stream, *cfg, *io);
    return (int)hipGetLastError();
  }
  if (cfg->engine == DGPPO_ENGINE_OMNI) {
    const size_t sh = omni_step_lds_bytes(*cfg);
    if (sh > 64 * 1024) return DGPPO_EINVAL;
    hipLaunchKernelGGL(omni_step_kernel<256>, dim3((unsigned)io->n_env), dim3(256), sh, (hipStream_t)stream, *cfg,
                       *io);
    return (int)hipGetLastError();
  }
  if (wave_shape) {
    const dim3 grid((unsigned)((io->n_env + 3) / 4)), block(256);
    const hipStream_t s = (hipStream_t)stream;
    const bool spread = cfg->goal_mode == DGPPO_GOAL_SPREAD;
    if (cfg->engine == DGPPO_ENGINE_BICYCLE) {
      const size_t sh = 4 * sizeof(float) * wv::Carve<5, 3>::total;
      if (spread) hipLaunchKernelGGL((wv::lidar_step_wave_kernel<DGPPO_ENGINE_BICYCLE, DGPPO_GOAL_SPREAD, 5, 3>), grid, block, sh, s, *cfg, *io);
      else hipLaunchKernelGGL((wv::lidar_step_wave_kernel<DGPPO_ENGINE_BICYCLE, DGPPO_GOAL_TARGET, 5, 3>), grid, block, sh, s, *cfg, *io);
    } else {
      const size_t sh = 4 * sizeof(float) * wv::Carve<4, 3>::total;
      if (spread) hipLaunchKernelGGL((wv::lidar_step_wave_kernel<DGPPO_ENGINE_LIDAR, DGPPO_GOAL_SPREAD, 4, 3>), grid, block, sh, s, *cfg, *io);
      else hipLaunchKernelGGL((wv::lidar_step_wave_kernel<DGPPO_ENGINE_LIDAR, DGPPO_GOAL_TARGET, 4, 3>), grid, block, sh, s, *cfg, *io);
    }
    return (int)hipGetLastError();
  }
  const Carve cv(cfg->n_agents, cfg->state_dim, cfg->n_obs, cfg->n_rays, cfg->top_k,
                 cfg->engine != DGPPO_ENGINE_MPE);
  const size_t shmem = (size_t)cv.total * sizeof(float);
  dispatch_step(*cfg, *io, shmem, (hipStream_t)stream);
  return (int)hipGetLastError();
}

// the wave kernels store edge rows as float4 (4-wide) / float2 (LidarOmniTarget's 10-wide) and 4-wide state rows
// as float4: those buffers, their per-env strides and (rollouts) their per-step strides must keep that alignment,
// else the generic kernels run
static bool wave_bufs_aligned(const dgppo_env_cfg* cfg, const float* edges, int64_t edges_stride, int64_t t_edges,
                              const float* states, int64_t states_stride, int64_t t_states) {
  const int64_t q = cfg->engine == DGPPO_ENGINE_OMNI ? 2 : 4;
  const bool e = (reinterpret_cast<uintptr_t>(edges) % (uintptr_t)(4 * q)) == 0 && edges_stride % q == 0 && t_edges % q == 0;
  const bool st4 = DGPPO_ENV_ST4 && cfg->state_dim == 4;
  const bool s = !st4 || ((reinterpret_cast<uintptr_t>(states) % 16u) == 0 && states_stride % 4 == 0 && t_states % 4 == 0);
  return e && s;
}

static bool wave_config(const dgppo_env_cfg* cfg, const float* edges, int64_t edges_stride, int64_t t_edges,
                        const float* states, int64_t states_stride, int64_t t_states) {
  const bool lidar = cfg->engine != DGPPO_ENGINE_MPE && cfg->n_obs > 0;
  return lidar && cfg->variant == DGPPO_VARIANT_NONE && cfg->n_agents == wv::NA && cfg->n_rays == wv::NR &&
         cfg->top_k == wv::NK && cfg->n_obs == 3 && wave_step_enabled() &&
         wave_bufs_aligned(cfg, edges, edges_stride, t_edges, states, states_stride, t_states);
}

// the initial graph of sampled agent / goal rows and obstacles: the wave step kernel in REBUILD mode, in place
static void launch_rebuild(const dgppo_env_cfg* cfg, const dgppo_env_step_io& st, hipStream_t s) {
  const dim3 grid((unsigned)((st.n_env + 3) / 4)), block(256);
  const bool spread = cfg->goal_mode == DGPPO_GOAL_SPREAD;
  if (cfg->engine == DGPPO_ENGINE_OMNI) {
    const size_t sh = 4 * sizeof(float) * wv::Carve<kOmniSD, 3>::total;
    hipLaunchKernelGGL((wv::lidar_step_wave_kernel<DGPPO_ENGINE_OMNI, DGPPO_GOAL_TARGET, kOmniSD, 3, true>), grid, block,
                       sh, s, *cfg, st);
  } else if (cfg->engine == DGPPO_ENGINE_BICYCLE) {
    const size_t sh = 4 * sizeof(float) * wv::Carve<5, 3>::total;
    if (spread)
      hipLaunchKernelGGL((wv::lidar_step_wave_kernel<DGPPO_ENGINE_BICYCLE, DGPPO_GOAL_SPREAD, 5, 3, true>), grid, block,
                         sh, s, *cfg, st);
    else
      hipLaunchKernelGGL((wv::lidar_step_wave_kernel<DGPPO_ENGINE_BICYCLE, DGPPO_GOAL_TARGET, 5, 3, true>), grid, block,
                         sh, s, *cfg, st);
  } else {
    const size_t sh = 4 * sizeof(float) * wv::Carve<4, 3>::total;
    if (spread)
      hipLaunchKernelGGL((wv::lidar_step_wave_kernel<DGPPO_ENGINE_LIDAR, DGPPO_GOAL_SPREAD, 4, 3, true>), grid, block,
                         sh, s, *cfg, st);
    else
      hipLaunchKernelGGL((wv::lidar_step_wave_kernel<DGPPO_ENGINE_LIDAR, DGPPO_GOAL_TARGET, 4, 3, true>), grid, block,
                         sh, s, *cfg, st);
  }
}

extern "C" int dgppo_env_reset_states(const dgppo_env_cfg* cfg, const dgppo_env_reset_io* io, void* stream) {
  if (validate(cfg) || !io || io->n_env < 0) return DGPPO_EINVAL;
  if (vmas::is_vmas(cfg)) return vmas::reset(cfg, io, stream);  // the full reset (graph 0 included)
  if (!wave_config(cfg, io->edges, io->edges_stride, 0, io->out_states, io->out_states_stride, 0))
    return dgppo_env_reset(cfg, io, stream);
  if (io->n_env == 0) return 0;
  if (!io->out_states || !io->obstacles) return DGPPO_EINVAL;
  const Carve cv(cfg->n_agents, cfg->state_dim, cfg->n_obs, cfg->n_rays, cfg->top_k, true);
  const size_t shmem = ((size_t)cv.total + 2 * kSampTab) * sizeof(float);
  dispatch_reset(*cfg, *io, shmem, (hipStream_t)stream, 1);
  return (int)hipGetLastError();
}

// envs per workgroup of the persistent rollout (DGPPO_ROLLOUT_WPG = 1, 4 or 8 forces it).  Per LidarSpread
// episode (reset + 128 steps, 4096 envs): 1 env 1.59 ms, 4 envs 1.37, 8 envs 1.34, 16 envs 1.41 (register
// spills); pooling the ray casts of more envs evens out their item counts between the barriers.  Below 2048
// envs the grid, not the pooling, sets the pace: LidarBicycleTarget at 512 envs (config 4's 8-GPU share)
// 8 envs 0.959 ms, 4 envs 0.838, 1 env 0.894 -- so 4 there.
static int rollout_wpg(int64_t n_env) {
  static const int forced = [] {
    const char* e = getenv("DGPPO_ROLLOUT_WPG");
    const int v = e ? atoi(e) : 0;
    return v == 1 || v == 4 || v == 8 ? v : 0;
  }();
  return forced ? forced : (n_env >= 2048 ? 8 : 4);
}

template <int ENGINE, int GOAL, int SD, int WPG>
static void launch_rollout_w(const dgppo_env_cfg& c, const dgppo_env_rollout_io& r, hipStream_t s) {
  const size_t sh = WPG * sizeof(float) * (wv::Carve<SD, 3>::total + wv::kRolloutActFloats);
  hipLaunchKernelGGL((wv::lidar_rollout_wave_kernel<ENGINE, GOAL, SD, 3, WPG>),
                     dim3((unsigned)((r.step.n_env + WPG - 1) / WPG)), dim3(64 * WPG), sh, s, c, r);
}

template <int ENGINE, int GOAL, int SD>
static void launch_rollout(const dgppo_env_cfg& c, const dgppo_env_rollout_io& r, hipStream_t s) {
  const int w = rollout_wpg(r.step.n_env);
  if (w == 4) launch_rollout_w<ENGINE, GOAL, SD, 4>(c, r, s);
  else if (w == 8) launch_rollout_w<ENGINE, GOAL, SD, 8>(c, r, s);
  else launch_rollout_w<ENGINE, GOAL, SD, 1>(c, r, s);
}

#ifdef DGPPO_ENV_STAMPS
// diagnostic builds: the phase sums since the last call (16 x u64 s_memtime ticks, summed over waves), then zeroed
extern "C" int dgppo_env_diag_block_stamps(unsigned long long* out) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(dgppo::g_blk_stamps), 8 * sizeof(unsigned long long));
  if (e == hipSuccess) {
    static const unsigned long long zero[8] = {};
    e = hipMemcpyToSymbol(HIP_SYMBOL(dgppo::g_blk_stamps), zero, sizeof(zero));
  }
  return (int)e;
}

extern "C" int dgppo_env_diag_stamps(unsigned long long* out) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(dgppo::wv::g_env_stamps), 16 * sizeof(unsigned long long));
  if (e == hipSuccess) {
    static const unsigned long long zero[16] = {};
    e = hipMemcpyToSymbol(HIP_SYMBOL(dgppo::wv::g_env_stamps), zero, sizeof(zero));
  }
  return (int)e;
}
#endif

extern "C" int dgppo_env_rollout(const dgppo_env_cfg* cfg, const dgppo_env_rollout_io* r, void* stream) {
  if (validate(cfg) || !r || r->T < 0 || r->step.n_env < 0) return DGPPO_EINVAL;
  if (vmas::is_vmas(cfg)) return vmas::rollout(cfg, r, stream);
  const dgppo_env_step_io& io = r->step;
  if (r->T == 0 && !r->rebuild_first) return 0;
  if (io.n_env == 0) return 0;
  if (!io.states || !io.action || !io.nodes || !io.edges || !io.out_states || !io.receivers || !io.senders ||
      !io.reward || !io.cost)
    return DGPPO_EINVAL;
  const bool lidar = cfg->engine != DGPPO_ENGINE_MPE && cfg->n_obs > 0;
  if (lidar && (!io.obstacles || !io.ray_dirs)) return DGPPO_EINVAL;
  const hipStream_t s = (hipStream_t)stream;
  if (wave_config(cfg, io.edges, io.edges_stride, r->t_edges, io.out_states, io.out_states_stride, r->t_states)) {
    const bool spread = cfg->goal_mode == DGPPO_GOAL_SPREAD;
    if (cfg->engine == DGPPO_ENGINE_OMNI) launch_rollout<DGPPO_ENGINE_OMNI, DGPPO_GOAL_TARGET, kOmniSD>(*cfg, *r, s);
    else if (cfg->engine == DGPPO_ENGINE_BICYCLE && spread) launch_rollout<DGPPO_ENGINE_BICYCLE, DGPPO_GOAL_SPREAD, 5>(*cfg, *r, s);
    else if (cfg->engine == DGPPO_ENGINE_BICYCLE) launch_rollout<DGPPO_ENGINE_BICYCLE, DGPPO_GOAL_TARGET, 5>(*cfg, *r, s);
    else if (spread) launch_rollout<DGPPO_ENGINE_LIDAR, DGPPO_GOAL_SPREAD, 4>(*cfg, *r, s);
    else launch_rollout<DGPPO_ENGINE_LIDAR, DGPPO_GOAL_TARGET, 4>(*cfg, *r, s);
    return (int)hipGetLastError();
  }
  // other configs: rebuild_first: a states-only reset (dgppo_env_reset_states) left graph 0 unbuilt when the
  // wave kernels took it (a misaligned per-step stride sends the rollout here)
  if (r->rebuild_first && wave_config(cfg, io.edges, io.edges_stride, 0, io.out_states, io.out_states_stride, 0))
    launch_rebuild(cfg, io, s);
  // the workgroup-per-env shapes: one persistent launch for all T steps (DGPPO_ENV_BLOCK_ROLLOUT=0: T launches)
  static const bool block_rollout = [] {
    const char* e = getenv("DGPPO_ENV_BLOCK_ROLLOUT");
    return !(e && atoi(e) == 0);
  }();
  // MPE n = 3 with 3 obstacles (BASELINE config 2): the wave-per-env persistent rollout (graph 0 is loaded: the MPE
  // reset always builds it); DGPPO_MPE_WAVE=0 or the block step kernels forced keep the workgroup-per-env kernel
  static const bool mpe_wave = [] {
    const char* e = getenv("DGPPO_MPE_WAVE");
    return !(e && atoi(e) == 0);
  }();
  if (block_rollout && mpe_wave && r->T > 0 && cfg->engine == DGPPO_ENGINE_MPE && cfg->variant == DGPPO_VARIANT_NONE &&
      cfg->n_agents == wv::mpew::NA && cfg->n_obs == wv::mpew::NO && wave_step_enabled() &&
      (reinterpret_cast<uintptr_t>(io.edges) % 16u) == 0 && io.edges_stride % 4 == 0 && r->t_edges % 4 == 0) {
    const size_t sh = 4 * sizeof(float) * wv::mpew::TOTAL;
    const dim3 grid((unsigned)((io.n_env + 3) / 4));
    if (cfg->goal_mode == DGPPO_GOAL_SPREAD)
      hipLaunchKernelGGL((wv::mpew::mpe_rollout_wave_kernel<DGPPO_GOAL_SPREAD>), grid, dim3(256), sh, s, *cfg, *r);
    else
      hipLaunchKernelGGL((wv::mpew::mpe_rollout_wave_kernel<DGPPO_GOAL_TARGET>), grid, dim3(256), sh, s, *cfg, *r);
    return (int)hipGetLastError();
  }
  if (block_rollout && r->T > 0 && cfg->variant == DGPPO_VARIANT_NONE && cfg->engine != DGPPO_ENGINE_OMNI &&
      cfg->n_agents <= 32) {  // (2 n actions per step staged one per thread of a >= 64-thread workgroup)
    const Carve cv(cfg->n_agents, cfg->state_dim, cfg->n_obs, cfg->n_rays, cfg->top_k,
                   cfg->engine != DGPPO_ENGINE_MPE);
    // the whole episode's actions are staged in LDS only when they fit kActStage AND the total stays within
    // the 64 KB default dynamic LDS (n = 32 / 8 obstacles carves 59 KB before staging); the kernel reads the flag
    const int64_t act_floats = (int64_t)r->T * 2 * cfg->n_agents;
    const int64_t act_lds = (act_floats + 3) & ~(int64_t)3;
    const bool stage = act_floats <= kActStage && (cv.total + act_lds) * (int64_t)sizeof(float) <= 64 * 1024;
    const int64_t extra = stage ? act_lds : 0;
    dispatch_rollout_block(*cfg, *r, (size_t)(cv.total + extra) * sizeof(float), s, stage ? 1 : 0);
    return (int)hipGetLastError();
  }
  for (int t = 0; t < r->T; ++t) {
    dgppo_env_step_io q = io;
    q.states = io.out_states + t * r->t_states;
    q.action = io.action + t * r->t_action;
    q.nodes = io.nodes + (t + 1) * r->t_nodes;
    q.edges = io.edges + (t + 1) * r->t_edges;
    q.out_states = io.out_states + (t + 1) * r->t_states;
    q.receivers = io.receivers + (t + 1) * r->t_index;
    q.senders = io.senders + (t + 1) * r->t_index;
    q.reward = io.reward + t * r->t_reward;
    q.cost = io.cost + t * r->t_cost;
    const int rc = dgppo_env_step(cfg, &q, stream);
    if (rc) return rc;
  }
  return 0;
}

extern "C" int dgppo_env_reset(const dgppo_env_cfg* cfg, const dgppo_env_reset_io* io, void* stream) {
  if (validate(cfg) || !io || io->n_env < 0) return DGPPO_EINVAL;
  if (vmas::is_vmas(cfg)) return vmas::reset(cfg, io, stream);
  if (io->n_env == 0) return 0;
  if (!io->nodes || !io->edges || !io->out_states || !io->receivers || !io->senders) return DGPPO_EINVAL;
  const bool lidar = cfg->engine != DGPPO_ENGINE_MPE && cfg->n_obs > 0;
  if (lidar && (!io->obstacles || !io->ray_dirs)) return DGPPO_EINVAL;
  const hipStream_t s = (hipStream_t)stream;
  if (cfg->variant != DGPPO_VARIANT_NONE) {
    const size_t sh = var::lds_floats(*cfg) * sizeof(float);
    if (sh > 64 * 1024) return DGPPO_EINVAL;
    if (cfg->engine == DGPPO_ENGINE_MPE)
      hipLaunchKernelGGL(var::reset_kernel<DGPPO_ENGINE_MPE>, dim3((unsigned)io->n_env), dim3(var::kT), sh, s, *cfg,
                         *io);
    else
      hipLaunchKernelGGL(var::reset_kernel<DGPPO_ENGINE_LIDAR>, dim3((unsigned)io->n_env), dim3(var::kT), sh, s,
                         *cfg, *io);
    return (int)hipGetLastError();
  }
  const Carve cv(cfg->n_agents, cfg->state_dim, cfg->n_obs, cfg->n_rays, cfg->top_k,
                 cfg->engine != DGPPO_ENGINE_MPE);
  const size_t shmem = ((size_t)cv.total + 2 * kSampTab) * sizeof(float);  // + the sampler's candidate table
  const bool wave = wave_config(cfg, io->edges, io->edges_stride, 0, io->out_states, io->out_states_stride, 0);
  if (!wave) {
    dispatch_reset(*cfg, *io, shmem, s, 0);
    return (int)hipGetLastError();
  }
  // sampled agent / goal rows and obstacles, then the wave-per-env step kernel in REBUILD mode builds
  // the initial graph from them in place (same LiDAR and graph code as every step)
  dispatch_reset(*cfg, *io, shmem, s, 1);
  dgppo_env_step_io st{};
  st.states = io->out_states;
  st.states_stride = io->out_states_stride;
  st.obstacles = io->obstacles;
  st.obstacles_stride = io->obstacles_stride;
  st.action = io->out_states;  // read, never used in REBUILD
  st.action_stride = io->out_states_stride;
  st.ray_dirs = io->ray_dirs;
  st.nodes = io->nodes;
  st.nodes_stride = io->nodes_stride;
  st.edges = io->edges;
  st.edges_stride = io->edges_stride;
  st.out_states = io->out_states;
  st.out_states_stride = io->out_states_stride;
  st.receivers = io->receivers;
  st.senders = io->senders;
  st.edge_index_stride = io->edge_index_stride;
  st.n_env = io->n_env;
  launch_rebuild(cfg, st, s);
  return (int)hipGetLastError();
}
