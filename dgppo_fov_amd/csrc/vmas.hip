// VMAS contact-physics environments on CDNA4: VMASWheel and VMASReverseTransport.
//
// Reference (behaviour restated, not translated):
//   env/vmas/vmas_wheel.py:90-122 reset, :124-216 step, :218-260 reward / cost, :262-307 graph,
//       :425-452 angle_dist / sample_valid_avoid_angle
//   env/vmas/vmas_reverse_transport.py:91-129 reset, :131-207 step, :209-250 reward / cost, :252-312 graph
//   env/vmas/physax/world.py:78-163 World.step + integration, :309-438 sphere-line / box-sphere contacts,
//       :440-468 soft constraint force; physax/geometry.py:8-102 closest points on lines / box sides
//   env/utils.py:139-244 get_node_goal_rng
// The NumPy twin is oracle/vmas.py; both evaluate the same single-rounded fp32 operations in the
// reference's order (this file is built with fp contraction off), so GPU and oracle agree bit for bit.
//
// Layout (one env):
//   states (4, 4): rows 0..2 agents [x, y, vx, vy]; row 3 (the graph's pad row, whose reference states are
//                  0-wide) carries the moving body: Wheel [line_angle, line_angvel, 0, 0],
//                  Transport [box_x, box_y, box_vx, box_vy]
//   record (8):    the per-episode constants in the `obstacles` buffer: Wheel [goal_angle, avoid_angle, 0..],
//                  Transport [goal_x, goal_y, o0x, o0y, o1x, o1y, o2x, o2y]
//   graph:         4 nodes (3 agents + pad), 9 agent-agent edges (i*3 + j, receiver i, sender j; the
//                  diagonal points at the pad node), nodes 13 (Wheel) / 20 (Transport) wide.
//
// Execution: one thread per env.  Each env's step is a short serial chain (Wheel: 3 world steps x 3
// contacts; Transport: 4 x 5 substeps x 3 agents x 4 box sides) on ~60 registers of state with no
// cross-env data, so a lane per env keeps all of it in VGPRs and needs no LDS or barriers; the rollout
// kernel carries the state in registers across all T steps (one launch per rollout), writing each graph
// once.  The HBM traffic per env step is the graph written (4x13|20 + 9x4 + 4x4 floats + 18 ints) plus
// 6 action floats read.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "dgppo_hip.h"
#include "math32.h"
#include "vmas.h"

#pragma clang fp contract(off)

namespace dgppo {
namespace vmas {

constexpr int kWheel = DGPPO_ENGINE_VMAS_WHEEL;
constexpr int kTransport = DGPPO_ENGINE_VMAS_TRANSPORT;
constexpr int kN = 3, kNodes = 4, kEdges = 9, kSD = 4, kRec = DGPPO_VMAS_FIELDS;
constexpr int kBlock = 64;
constexpr int kMaxIter = 1024;        // get_node_goal_rng max_iter (env/utils.py:139-244)
constexpr int kMaxDraws = 1 << 20;    // safety bound on a pathological resample chain (never reached here)

// constants: the reference's Python float64 expressions, rounded once to fp32 (jax_enable_x64 off)
constexpr double kLineMinDist = 4 / 6e2;  // world.py:19
constexpr double kAgentR = 0.03;
constexpr double kDeg = M_PI / 180.0;     // np.deg2rad(x) = x * (pi / 180)
constexpr float kPiF = (float)M_PI;
constexpr float kAgentCost = (float)(kAgentR * 2);

namespace wk {  // VMASWheel (vmas_wheel.py:53-64, 132-164; World defaults world.py:32-45)
constexpr float u_mult = (float)0.6, agent_drag = (float)(1 - 0.25), line_drag = (float)(1 - 0.015);
constexpr float sub_dt = (float)(0.1 / 1), moi = (float)((1.0 / 12) * 15.0 * (2.0 * 2.0)), max_w = (float)0.6;
constexpr float dmin = (float)(kAgentR + kLineMinDist), k = (float)1e-3, mult = 100.0f, semi = (float)1.2;
constexpr float half_len = (float)(2.0 / 2), side = (float)(0.99 * (2 * 1.2)), shift = (float)1.2;
constexpr float obs_hw = (float)(15 * kDeg), avoid_min = (float)(15 * kDeg + 1 * kDeg);
constexpr float goal_max = (float)(M_PI / 2), rew_deg = (float)(1 * kDeg);
constexpr int frame_skip = 3;
}  // namespace wk

namespace tk {  // VMASReverseTransport (vmas_reverse_transport.py:50-64, 139-161)
constexpr double x0r_d = 0.98 * (0.8 - 0.5 * 0.6);
constexpr float u_mult = (float)0.5, agent_drag = (float)(1 - 0.25), box_drag = (float)(1 - 0.25);
constexpr float sub_dt = (float)(0.1 / 5), box_mass = (float)10.0, dmin = (float)(kAgentR + kLineMinDist);
constexpr float k = (float)6e-3, mult = 500.0f, semi = (float)1.2, half = (float)(0.6 / 2);
constexpr float side = (float)(0.4 * 0.6), shift = (float)0.2, x0r = (float)x0r_d;
constexpr float obs_place_r = (float)(x0r_d - 1.5 * 0.15), noise_ub = (float)(30 * kDeg);
constexpr float obs_r = (float)0.15, contact_len = (float)(0.6 - 1e-2), dist2goal = (float)0.01;
constexpr int frame_skip = 4, substeps = 5;
}  // namespace tk

__device__ __forceinline__ float angle_dist(float a, float b) {
  float s, c;
  sincos32(a - b, &s, &c);
  return atan2_32(s, c);
}

__device__ __forceinline__ float clampf(float x, float lo, float hi) {
  const float y = x < lo ? lo : x;
  return y > hi ? hi : y;
}

__device__ __forceinline__ float nrm2(float dx, float dy) { return sqrtf(dx * dx + dy * dy); }

// _get_constraint_forces (world.py:440-468), not attractive: the force on a
__device__ __forceinline__ void constraint_force(float ax, float ay, float bx, float by, float dmin, float mult,
                                                 float k, float& fx, float& fy) {
  const float dx = ax - bx, dy = ay - by;
  const float d = nrm2(dx, dy);
  const float pen = logaddexp0_32(((dmin - d) * 1.0f) / k) * k;
  const float den = d > 0.0f ? d : 1e-8f;
  fx = ((mult * dx) / den) * pen;
  fy = ((mult * dy) / den) * pen;
  if (d < 1e-6f || d > dmin) {
    fx = 0.0f;
    fy = 0.0f;
  }
}

// geometry.py:8-34 with the line direction precomputed
__device__ __forceinline__ void closest_point_line(float lx, float ly, float rvx, float rvy, float half_len, float px,
                                                   float py, float& cx, float& cy) {
  const float dx = lx - px, dy = ly - py;
  const float dot = dx * rvx + dy * rvy;
  const float sg = dot > 0.0f ? 1.0f : (dot < 0.0f ? -1.0f : 0.0f);
  const float ad = fabsf(dot);
  const float dfc = half_len < ad ? half_len : ad;
  const float s = sg * dfc;
  cx = lx - s * rvx;
  cy = ly - s * rvy;
}

struct BoxDirs {  // (cos, sin) of box_rot = 0 and of box_rot + pi/2 (geometry.py:78-102)
  float c0, s0, c2, s2;
};

__device__ __forceinline__ BoxDirs box_dirs() {
  BoxDirs d;
  sincos32(0.0f, &d.s0, &d.c0);
  sincos32(0.0f + (float)(M_PI / 2), &d.s2, &d.c2);
  return d;
}

// get_closest_point_box (geometry.py:37-53): the first side whose closest point is strictly nearest
__device__ __forceinline__ void closest_point_box(const BoxDirs& r, float bx, float by, float px, float py,
                                                  float& cx, float& cy) {
  const float h = tk::half;
  const float lx[4] = {bx + r.c0 * h, bx - r.c0 * h, bx + r.c2 * h, bx - r.c2 * h};
  const float ly[4] = {by + r.s0 * h, by - r.s0 * h, by + r.s2 * h, by - r.s2 * h};
  float best = INFINITY;
  cx = INFINITY;
  cy = INFINITY;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float rvx = q < 2 ? r.c2 : r.c0, rvy = q < 2 ? r.s2 : r.s0;  // sides 0, 1 run along box_rot + pi/2
    float qx, qy;
    closest_point_line(lx[q], ly[q], rvx, rvy, h, px, py, qx, qy);
    const float d = nrm2(px - qx, py - qy);
    if (d < best) {
      best = d;
      cx = qx;
      cy = qy;
    }
  }
}

struct Env {
  float px[kN], py[kN], vx[kN], vy[kN];
  float b0, b1, b2, b3;    // Wheel: rot, w; Transport: box x, y, vx, vy
  float fcx[kN], fcy[kN];  // Wheel: the agents' contact forces of the last world step
  float rec[kRec];
};

__device__ __forceinline__ void integrate_agents(Env& e, const float Fx[kN], const float Fy[kN], float drag,
                                                 float dt, float semi, bool substep0) {
#pragma unroll
  for (int i = 0; i < kN; ++i) {
    float vx = e.vx[i], vy = e.vy[i];
    if (substep0) {
      vx = vx * drag;
      vy = vy * drag;
    }
    vx = vx + (Fx[i] / 1.0f) * dt;
    vy = vy + (Fy[i] / 1.0f) * dt;
    e.vx[i] = vx;
    e.vy[i] = vy;
    e.px[i] = clampf(e.px[i] + vx * dt, -semi, semi);
    e.py[i] = clampf(e.py[i] + vy * dt, -semi, semi);
  }
}

// one World.step of [line, agent_0..2] (world.py:78-105, 137-152, 309-359)
__device__ __forceinline__ void wheel_world_step(Env& e, const float fax[kN], const float fay[kN]) {
  float sn, cs;
  sincos32(e.b0, &sn, &cs);
  float torque = 0.0f, Fx[kN], Fy[kN];
#pragma unroll
  for (int i = 0; i < kN; ++i) {
    float cx, cy, fx, fy;
    closest_point_line(0.0f, 0.0f, cs, sn, wk::half_len, e.px[i], e.py[i], cx, cy);
    constraint_force(e.px[i], e.py[i], cx, cy, wk::dmin, wk::mult, wk::k, fx, fy);
    const float flx = -fx, fly = -fy;
    const float rx = cx - 0.0f, ry = cy - 0.0f;
    const float t = rx * fly - ry * flx;
    torque = i == 0 ? t : torque + t;
    e.fcx[i] = fx;
    e.fcy[i] = fy;
    Fx[i] = (0.0f + fax[i]) + fx;
    Fy[i] = (0.0f + fay[i]) + fy;
  }
  const float tq = 0.0f + torque;
  float w = e.b1 * wk::line_drag;
  w = w + (tq / wk::moi) * wk::sub_dt;
  const float nrm = sqrtf(w * w);
  if (nrm > wk::max_w) w = (w / nrm) * wk::max_w;
  e.b0 = e.b0 + w * wk::sub_dt;
  e.b1 = w;
  integrate_agents(e, Fx, Fy, wk::agent_drag, wk::sub_dt, wk::semi, true);
}

// one World.step of [box, agent_0..2] with 5 substeps (world.py:78-135, 361-438)
__device__ __forceinline__ void transport_world_step(Env& e, const BoxDirs& bd, const float fax[kN],
                                                     const float fay[kN]) {
  for (int sub = 0; sub < tk::substeps; ++sub) {
    float Fx[kN], Fy[kN], fbx = 0.0f, fby = 0.0f;
#pragma unroll
    for (int i = 0; i < kN; ++i) {
      float cx, cy, fx, fy;
      closest_point_box(bd, e.b0, e.b1, e.px[i], e.py[i], cx, cy);
      constraint_force(e.px[i], e.py[i], cx, cy, tk::dmin, tk::mult, tk::k, fx, fy);
      fbx = i == 0 ? -fx : fbx + -fx;
      fby = i == 0 ? -fy : fby + -fy;
      Fx[i] = (0.0f + fax[i]) + fx;
      Fy[i] = (0.0f + fay[i]) + fy;
    }
    const float Fbx = 0.0f + fbx, Fby = 0.0f + fby;
    float bvx = e.b2, bvy = e.b3;
    if (sub == 0) {
      bvx = bvx * tk::box_drag;
      bvy = bvy * tk::box_drag;
    }
    bvx = bvx + (Fbx / tk::box_mass) * tk::sub_dt;
    bvy = bvy + (Fby / tk::box_mass) * tk::sub_dt;
    e.b2 = bvx;
    e.b3 = bvy;
    e.b0 = clampf(e.b0 + bvx * tk::sub_dt, -tk::semi, tk::semi);
    e.b1 = clampf(e.b1 + bvy * tk::sub_dt, -tk::semi, tk::semi);
    integrate_agents(e, Fx, Fy, tk::agent_drag, tk::sub_dt, tk::semi, sub == 0);
  }
}

// ---- reward / cost of the pre-step state (vmas_wheel.py:218-260, vmas_reverse_transport.py:209-250) ----
__device__ __forceinline__ float margin(float c) { return c <= 0.0f ? c - 0.5f : c + 0.5f; }

__device__ __forceinline__ void agent_min_dist(const Env& e, float md[kN]) {
#pragma unroll
  for (int i = 0; i < kN; ++i) {
    float m = INFINITY;
#pragma unroll
    for (int j = 0; j < kN; ++j) {
      const float d = nrm2(e.px[i] - e.px[j], e.py[i] - e.py[j]) + (i == j ? 1e6f : 0.0f);
      m = d < m ? d : m;
    }
    md[i] = m;
  }
}

template <int KIND>
__device__ __forceinline__ float reward_cost(const Env& e, float cost[kN][2]) {
  float md[kN];
  agent_min_dist(e, md);
  if (KIND == kWheel) {
    const float ad = angle_dist(e.b0, e.rec[0]);
    float sq = (0.1f * ad) / kPiF;
    sq = sq * sq;
    float r = (-sq) * 0.5f;
    r = r - (ad > wk::rew_deg ? 1.0f : 0.0f) * 0.005f;
    const float ld = angle_dist(e.b0, e.rec[1]);
    const float cl = (wk::obs_hw - fabsf(ld)) / kPiF;
#pragma unroll
    for (int i = 0; i < kN; ++i) {
      const float ca = margin(kAgentCost - md[i]), cb = margin(cl);
      cost[i][0] = ca < -1.0f ? -1.0f : ca;
      cost[i][1] = cb < -1.0f ? -1.0f : cb;
    }
    return r;
  } else {
    const float d = nrm2(e.rec[0] - e.b0, e.rec[1] - e.b1);
    float r = (-d) * 0.01f;
    r = r - (d > tk::dist2goal ? 1.0f : 0.0f) * 0.001f;
    float om = INFINITY;
#pragma unroll
    for (int o = 0; o < 3; ++o) {
      const float od = nrm2(e.b0 - e.rec[2 + 2 * o], e.b1 - e.rec[3 + 2 * o]);
      om = od < om ? od : om;
    }
    const float cb = 2.0f * (tk::obs_r - om);
#pragma unroll
    for (int i = 0; i < kN; ++i) {
      const float ca = margin(4.0f * (kAgentCost - md[i])), cc = margin(cb);
      cost[i][0] = clampf(ca, -1.0f, 1.0f);
      cost[i][1] = clampf(cc, -1.0f, 1.0f);
    }
    return r;
  }
}

// ---- graph (get_graph + edge_blocks + GetGraph.to_padded) ---------------------------------------------
struct GraphOut {
  float* nodes;
  float* edges;
  float* states;
  int32_t* recv;
  int32_t* send;
};

template <int KIND>
__device__ void write_graph(const Env& e, const GraphOut& g) {
  constexpr int ND = KIND == kWheel ? 13 : 20;
  float row[ND];
  if (KIND == kWheel) {
    float s, c, sg, cg, so, co;
    sincos32(e.b0, &s, &c);
    sincos32(angle_dist(e.b0, e.rec[0]), &sg, &cg);
    sincos32(angle_dist(e.b0, e.rec[1]), &so, &co);
    row[4] = s;
    row[5] = c;
    row[6] = e.b1;
    row[9] = sg;
    row[10] = cg;
    row[11] = so;
    row[12] = co;
  } else {
    row[4] = e.b0;
    row[5] = e.b1;
    row[6] = e.b2;
    row[7] = e.b3;
    row[8] = e.rec[0] - e.b0;
    row[9] = e.rec[1] - e.b1;
    float ox[3], oy[3], od[3];
#pragma unroll
    for (int o = 0; o < 3; ++o) {
      ox[o] = e.rec[2 + 2 * o] - e.b0;
      oy[o] = e.rec[3 + 2 * o] - e.b1;
      od[o] = sqrtf((ox[o] * ox[o] + oy[o] * oy[o]) + 1e-6f);
    }
#pragma unroll
    for (int o = 0; o < 3; ++o) {  // stable argsort: rank = #{q : od[q] < od[o] or (== and q < o)}
      int pos = 0;
#pragma unroll
      for (int q = 0; q < 3; ++q) pos += (od[q] < od[o] || (od[q] == od[o] && q < o)) ? 1 : 0;
      const float vx = ox[o] / od[o], vy = oy[o] / od[o];
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        if (p == pos) {
          row[11 + 2 * p] = vx;
          row[12 + 2 * p] = vy;
          row[17 + p] = od[o];
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < kN; ++i) {
    row[0] = e.px[i];
    row[1] = e.py[i];
    row[2] = e.vx[i];
    row[3] = e.vy[i];
    if (KIND == kWheel) {
      row[7] = e.fcx[i];
      row[8] = e.fcy[i];
    } else {
      const float rx = e.px[i] - e.b0, ry = e.py[i] - e.b1;
      row[10] = (fabsf(rx) > tk::contact_len || fabsf(ry) > tk::contact_len) ? 1.0f : 0.0f;
    }
#pragma unroll
    for (int c = 0; c < ND; ++c) g.nodes[i * ND + c] = row[c];
  }
#pragma unroll
  for (int c = 0; c < ND; ++c) g.nodes[kN * ND + c] = 0.0f;
#pragma unroll
  for (int i = 0; i < kN; ++i) {
    g.states[i * kSD + 0] = e.px[i];
    g.states[i * kSD + 1] = e.py[i];
    g.states[i * kSD + 2] = e.vx[i];
    g.states[i * kSD + 3] = e.vy[i];
  }
  g.states[12] = e.b0;
  g.states[13] = e.b1;
  g.states[14] = KIND == kWheel ? 0.0f : e.b2;
  g.states[15] = KIND == kWheel ? 0.0f : e.b3;
#pragma unroll
  for (int i = 0; i < kN; ++i) {
#pragma unroll
    for (int j = 0; j < kN; ++j) {
      const int ed = i * kN + j;
      g.edges[ed * 4 + 0] = e.px[i] - e.px[j];
      g.edges[ed * 4 + 1] = e.py[i] - e.py[j];
      g.edges[ed * 4 + 2] = e.vx[i] - e.vx[j];
      g.edges[ed * 4 + 3] = e.vy[i] - e.vy[j];
      g.recv[ed] = i != j ? i : kNodes - 1;
      g.send[ed] = i != j ? j : kNodes - 1;
    }
  }
}

// ---- step ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void load_env(Env& e, const float* st, const float* rec) {
#pragma unroll
  for (int i = 0; i < kN; ++i) {
    e.px[i] = st[i * kSD + 0];
    e.py[i] = st[i * kSD + 1];
    e.vx[i] = st[i * kSD + 2];
    e.vy[i] = st[i * kSD + 3];
    e.fcx[i] = 0.0f;
    e.fcy[i] = 0.0f;
  }
  e.b0 = st[12];
  e.b1 = st[13];
  e.b2 = st[14];
  e.b3 = st[15];
#pragma unroll
  for (int q = 0; q < kRec; ++q) e.rec[q] = rec[q];
}

// reward / cost of the current state, then frame_skip world steps with the clipped, scaled actions
template <int KIND>
__device__ __forceinline__ float env_step(Env& e, const float* act, float cost[kN][2]) {
  const float r = reward_cost<KIND>(e, cost);
  float fax[kN], fay[kN];
  const float um = KIND == kWheel ? wk::u_mult : tk::u_mult;
#pragma unroll
  for (int i = 0; i < kN; ++i) {  // clip_action then action * u_multiplier (vmas_wheel.py:127, 168)
    fax[i] = clampf(act[2 * i + 0], -1.0f, 1.0f) * um;
    fay[i] = clampf(act[2 * i + 1], -1.0f, 1.0f) * um;
  }
  if (KIND == kWheel) {
    for (int f = 0; f < wk::frame_skip; ++f) wheel_world_step(e, fax, fay);
  } else {
    const BoxDirs bd = box_dirs();
    for (int f = 0; f < tk::frame_skip; ++f) transport_world_step(e, bd, fax, fay);
  }
  return r;
}

__device__ __forceinline__ void store_cost(float* c, const float cost[kN][2]) {
#pragma unroll
  for (int i = 0; i < kN; ++i) {
    c[2 * i + 0] = cost[i][0];
    c[2 * i + 1] = cost[i][1];
  }
}

template <int KIND>
__global__ __launch_bounds__(kBlock) void step_kernel(dgppo_env_step_io io) {
  const int b = blockIdx.x * kBlock + threadIdx.x;
  if (b >= io.n_env) return;
  Env e;
  load_env(e, io.states + b * io.states_stride, io.obstacles + b * io.obstacles_stride);
  float cost[kN][2];
  const float r = env_step<KIND>(e, io.action + b * io.action_stride, cost);
  io.reward[b * io.reward_stride] = r;
  store_cost(io.cost + b * io.cost_stride, cost);
  const GraphOut g{io.nodes + b * io.nodes_stride, io.edges + b * io.edges_stride,
                   io.out_states + b * io.out_states_stride, io.receivers + b * io.edge_index_stride,
                   io.senders + b * io.edge_index_stride};
  write_graph<KIND>(e, g);
}

// T steps, the env state in registers throughout (graph t+1, reward[t], cost[t] written per step)
template <int KIND>
__global__ __launch_bounds__(kBlock) void rollout_kernel(dgppo_env_rollout_io r) {
  const dgppo_env_step_io& io = r.step;
  const int b = blockIdx.x * kBlock + threadIdx.x;
  if (b >= io.n_env) return;
  Env e;
  load_env(e, io.out_states + b * io.out_states_stride, io.obstacles + b * io.obstacles_stride);
  for (int t = 0; t < r.T; ++t) {
    float cost[kN][2];
    const float rw = env_step<KIND>(e, io.action + t * r.t_action + b * io.action_stride, cost);
    io.reward[t * r.t_reward + b * io.reward_stride] = rw;
    store_cost(io.cost + t * r.t_cost + b * io.cost_stride, cost);
    const int64_t t1 = t + 1;
    const GraphOut g{io.nodes + t1 * r.t_nodes + b * io.nodes_stride, io.edges + t1 * r.t_edges + b * io.edges_stride,
                     io.out_states + t1 * r.t_states + b * io.out_states_stride,
                     io.receivers + t1 * r.t_index + b * io.edge_index_stride,
                     io.senders + t1 * r.t_index + b * io.edge_index_stride};
    write_graph<KIND>(e, g);
  }
}

// ---- reset ----------------------------------------------------------------------------------------------
// get_node_goal_rng (env/utils.py:139-244) for n = 3, no obstacles, as oracle/env.py:node_goal_rng: the
// candidates are compared with all 3 rows (unplaced ones are zero), goals are drawn and discarded (VMAS
// keeps the agent positions only), a row exceeding max_iter restarts the whole draw.
__device__ void sample_agents(Rng& rng, float side, float md, float sx[kN], float sy[kN]) {
  float gx[kN], gy[kN];
#pragma unroll
  for (int j = 0; j < kN; ++j) sx[j] = sy[j] = gx[j] = gy[j] = 0.0f;
  int id = 0;
  int draws = 0;
  while (id < kN && draws < kMaxDraws) {
    float cx = rng.uniform(0.0f, side), cy = rng.uniform(0.0f, side);
    int it = 0;
    while (true) {
      float dmin = INFINITY;
#pragma unroll
      for (int j = 0; j < kN; ++j) {
        const float d = nrm2(sx[j] - cx, sy[j] - cy);
        dmin = d < dmin ? d : dmin;
      }
      if (!(dmin <= md) || it >= kMaxIter) break;
      ++it;
      cx = rng.uniform(0.0f, side);
      cy = rng.uniform(0.0f, side);
    }
    const int it_agent = it;
#pragma unroll
    for (int j = 0; j < kN; ++j)
      if (j == id) {
        sx[j] = cx;
        sy[j] = cy;
      }
    float qx = rng.uniform(0.0f, side), qy = rng.uniform(0.0f, side);
    it = 0;
    while (true) {
      float dmin = INFINITY;
#pragma unroll
      for (int j = 0; j < kN; ++j) {
        const float d = nrm2(gx[j] - qx, gy[j] - qy);
        dmin = d < dmin ? d : dmin;
      }
      const bool outside = qx < 0.0f || qy < 0.0f || qx > side || qy > side;
      if (!(dmin <= md || outside) || it >= kMaxIter) break;
      ++it;
      qx = rng.uniform(0.0f, side);
      qy = rng.uniform(0.0f, side);
    }
#pragma unroll
    for (int j = 0; j < kN; ++j)
      if (j == id) {
        gx[j] = qx;
        gy[j] = qy;
      }
    draws += it_agent + it + 2;
    ++id;
    if (it_agent >= kMaxIter || it >= kMaxIter) {
      id = 0;
#pragma unroll
      for (int j = 0; j < kN; ++j) sx[j] = sy[j] = gx[j] = gy[j] = 0.0f;
    }
  }
}

template <int KIND>
__global__ __launch_bounds__(kBlock) void reset_kernel(dgppo_env_reset_io io) {
  const int b = blockIdx.x * kBlock + threadIdx.x;
  if (b >= io.n_env) return;
  const uint64_t seed = io.seed_ptr ? *io.seed_ptr : io.seed;
  const uint32_t env = (uint32_t)(io.env_offset + b);
  Env e;
  float ax[kN], ay[kN];
#pragma unroll
  for (int q = 0; q < kRec; ++q) e.rec[q] = 0.0f;
  if (KIND == kWheel) {  // vmas_wheel.py:90-122; keys split 6 ways -> purposes 1..6
    Rng r1(seed, env, 1), r2(seed, env, 2), r3(seed, env, 3), r4(seed, env, 4), r5(seed, env, 5), r6(seed, env, 6);
    const float line = r1.uniform((float)-M_PI, (float)M_PI);
    const float w = r2.uniform(-0.05f, 0.05f);
    sample_agents(r3, wk::side, kAgentCost, ax, ay);
#pragma unroll
    for (int i = 0; i < kN; ++i) {
      e.px[i] = ax[i] - wk::shift;
      e.py[i] = ay[i] - wk::shift;
      e.vx[i] = r4.uniform(-0.01f, 0.01f);
      e.vy[i] = r4.uniform(-0.01f, 0.01f);
    }
    const float goal = r5.uniform((float)-M_PI, (float)M_PI);
    // sample_valid_avoid_angle (vmas_wheel.py:435-452): the first valid draw nearest the goal, else draw 0
    float best = INFINITY, avoid = 0.0f;
    for (int q = 0; q < 8; ++q) {
      const float a = r6.uniform((float)-M_PI, (float)M_PI);
      const float dg = fabsf(angle_dist(a, goal)), dl = fabsf(angle_dist(a, line));
      const bool ok = dg > wk::avoid_min && dl > wk::avoid_min && dg < wk::goal_max;
      const float m = ok ? dg : INFINITY;
      if (q == 0 || m < best) {
        best = m;
        avoid = a;
      }
    }
    e.b0 = line;
    e.b1 = w;
    e.b2 = 0.0f;
    e.b3 = 0.0f;
    e.rec[0] = goal;
    e.rec[1] = avoid;
  } else {  // vmas_reverse_transport.py:91-129; keys split 5 ways -> purposes 1..5
    Rng r1(seed, env, 1), r2(seed, env, 2), r3(seed, env, 3), r4(seed, env, 4), r5(seed, env, 5);
    const float x0 = r1.uniform(0.0f, (float)(2 * M_PI));
    float s0, c0;
    sincos32(x0, &s0, &c0);
    const float bx = tk::x0r * c0, by = tk::x0r * s0;
    const float ga = (x0 + kPiF) + r4.uniform(-tk::noise_ub, tk::noise_ub);
    float sg, cg;
    sincos32(ga, &sg, &cg);
    e.rec[0] = tk::x0r * cg;
    e.rec[1] = tk::x0r * sg;
#pragma unroll
    for (int o = 0; o < 3; ++o) {
      const float oa = r5.uniform(0.0f, (float)(2 * M_PI));
      float so, co;
      sincos32(oa, &so, &co);
      e.rec[2 + 2 * o] = tk::obs_place_r * co;
      e.rec[3 + 2 * o] = tk::obs_place_r * so;
    }
    sample_agents(r2, tk::side, kAgentCost, ax, ay);
#pragma unroll
    for (int i = 0; i < kN; ++i) {
      e.px[i] = (ax[i] - tk::shift) + bx;
      e.py[i] = (ay[i] - tk::shift) + by;
      e.vx[i] = r3.uniform(-0.01f, 0.01f);
      e.vy[i] = r3.uniform(-0.01f, 0.01f);
    }
    e.b0 = bx;
    e.b1 = by;
    e.b2 = 0.0f;
    e.b3 = 0.0f;
  }
#pragma unroll
  for (int i = 0; i < kN; ++i) e.fcx[i] = e.fcy[i] = 0.0f;
  float* rec = io.obstacles + b * io.obstacles_stride;
#pragma unroll
  for (int q = 0; q < kRec; ++q) rec[q] = e.rec[q];
  const GraphOut g{io.nodes + b * io.nodes_stride, io.edges + b * io.edges_stride,
                   io.out_states + b * io.out_states_stride, io.receivers + b * io.edge_index_stride,
                   io.senders + b * io.edge_index_stride};
  write_graph<KIND>(e, g);
}

// ---- host entry points (called by the dgppo_env_* C-ABI) ------------------------------------------------
bool is_vmas(const dgppo_env_cfg* c) {
  return c && (c->engine == DGPPO_ENGINE_VMAS_WHEEL || c->engine == DGPPO_ENGINE_VMAS_TRANSPORT);
}

int validate(const dgppo_env_cfg* c) {
  if (!is_vmas(c) || c->n_agents != kN || c->variant != DGPPO_VARIANT_NONE) return DGPPO_EINVAL;
  const int nd = c->engine == kWheel ? 13 : 20;
  if (c->state_dim != kSD || c->node_dim != nd || c->n_nodes != kNodes || c->n_edges != kEdges) return DGPPO_EINVAL;
  return 0;
}

int finalize(dgppo_env_cfg* c) {
  if (!is_vmas(c)) return DGPPO_EINVAL;
  c->state_dim = kSD;
  c->node_dim = c->engine == kWheel ? 13 : 20;
  c->edge_dim = 4;
  c->action_dim = 2;
  c->n_cost = 2;
  c->n_goals = 0;
  c->n_nodes = kNodes;
  c->n_edges = kEdges;
  for (int i = 0; i < 8; ++i) c->state_lo[i] = c->state_hi[i] = 0.0f;  // state_lim: `pass` in the reference
  return validate(c);
}

static unsigned grid_of(int n_env) { return (unsigned)((n_env + kBlock - 1) / kBlock); }

int step(const dgppo_env_cfg* c, const dgppo_env_step_io* io, void* stream) {
  if (validate(c) || !io || io->n_env < 0) return DGPPO_EINVAL;
  if (io->n_env == 0) return 0;
  if (!io->states || !io->obstacles || !io->action || !io->nodes || !io->edges || !io->out_states ||
      !io->receivers || !io->senders || !io->reward || !io->cost)
    return DGPPO_EINVAL;
  const hipStream_t s = (hipStream_t)stream;
  if (c->engine == kWheel)
    hipLaunchKernelGGL(step_kernel<kWheel>, dim3(grid_of(io->n_env)), dim3(kBlock), 0, s, *io);
  else
    hipLaunchKernelGGL(step_kernel<kTransport>, dim3(grid_of(io->n_env)), dim3(kBlock), 0, s, *io);
  return (int)hipGetLastError();
}

int reset(const dgppo_env_cfg* c, const dgppo_env_reset_io* io, void* stream) {
  if (validate(c) || !io || io->n_env < 0) return DGPPO_EINVAL;
  if (io->n_env == 0) return 0;
  if (!io->obstacles || !io->nodes || !io->edges || !io->out_states || !io->receivers || !io->senders)
    return DGPPO_EINVAL;
  const hipStream_t s = (hipStream_t)stream;
  if (c->engine == kWheel)
    hipLaunchKernelGGL(reset_kernel<kWheel>, dim3(grid_of(io->n_env)), dim3(kBlock), 0, s, *io);
  else
    hipLaunchKernelGGL(reset_kernel<kTransport>, dim3(grid_of(io->n_env)), dim3(kBlock), 0, s, *io);
  return (int)hipGetLastError();
}

int rollout(const dgppo_env_cfg* c, const dgppo_env_rollout_io* r, void* stream) {
  if (validate(c) || !r || r->T < 0 || r->step.n_env < 0) return DGPPO_EINVAL;
  const dgppo_env_step_io& io = r->step;
  if (r->T == 0 || io.n_env == 0) return 0;  // graph 0 is always complete (reset writes it)
  if (!io.obstacles || !io.action || !io.nodes || !io.edges || !io.out_states || !io.receivers || !io.senders ||
      !io.reward || !io.cost)
    return DGPPO_EINVAL;
  const hipStream_t s = (hipStream_t)stream;
  if (c->engine == kWheel)
    hipLaunchKernelGGL(rollout_kernel<kWheel>, dim3(grid_of(io.n_env)), dim3(kBlock), 0, s, *r);
  else
    hipLaunchKernelGGL(rollout_kernel<kTransport>, dim3(grid_of(io.n_env)), dim3(kBlock), 0, s, *r);
  return (int)hipGetLastError();
}

}  // namespace vmas
}  // namespace dgppo
