/* dgppo_hip.h — C-ABI of libdgppo_hip.so, the MI355X (gfx950) hot paths of DGPPO.
 *
 * The reference (Tw6249/dgppo_fov) is pure JAX and has no FFI: every entry point below replaces a
 * jitted, vmapped JAX function.  The Python host layer (dgppo_fov_amd/) binds them with ctypes
 * (see INTEGRATION.md); no torch types cross this boundary — only device pointers, element
 * strides, sizes and a hipStream_t passed as void*.
 *
 * Conventions
 *   - Ownership: the caller allocates every device buffer; the library never allocates or frees.
 *   - Errors: functions return 0 on success, DGPPO_EINVAL (-22) for shape/argument violations
 *     (the reference's `assert`s), or a positive hipError_t from the launch.
 *   - Threading: stateless; launches are enqueued on `stream` (NULL = the null stream).
 *   - All floating point is IEEE fp32; env-step kernels are compiled without FMA contraction so
 *     that they reproduce the NumPy oracle (oracle/env.py) bit for bit.
 */
#ifndef DGPPO_HIP_H
#define DGPPO_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DGPPO_ABI_VERSION 14  /* 14: dgppo_gnn_layer_bwd removed (the fused layer backward measured slower than the attention backward + GEMMs), dgppo_gnn_set_attn_kernel removed with the graph-form MFMA attention kernels (2-5x slower); 13: dgppo_gemm_wgrad_grouped (a pass's weight gradients in one launch); 12: dgppo_adam_multi (the clipped Adam steps of several nets in two launches); 11: dgppo_gnn_layer_fwd (fused GraphTransformer layer forward); 10: in-kernel policy-step noise, dgppo_gnn_set_graph_otf; 9: dgppo_gnn_set_attn_kernel (graph-form MFMA attention selector); 8: VMAS engines (DGPPO_ENGINE_VMAS_*) through the dgppo_env_* entry points; 7: dgppo_lstm_cell_fwd / _bwd; 6: env variants (dgppo_env_cfg variant fields); 5: Q-free attention args (beta, qt/dqt/dbeta strides), dgppo_gather_env_steps; 4: dgppo_env_rollout, dgppo_env_reset_states; 3: dgppo_adam takes double b1 / b2; 2: dgppo_gnn_attn_args.da_add, wide-edge entry points, env cfg Omni fields */
#define DGPPO_EINVAL (-22)

/* engines */
#define DGPPO_ENGINE_LIDAR 0   /* LidarEnv double integrator: dgppo/env/lidar_env/base.py */
#define DGPPO_ENGINE_BICYCLE 1 /* LidarBicycleTarget: dgppo/env/lidar_env/lidar_bicycle_target.py */
#define DGPPO_ENGINE_MPE 2     /* MPE double integrator: dgppo/env/mpe/base.py */
#define DGPPO_ENGINE_OMNI 3    /* LidarOmniTarget omni-wheel + FoV costs: dgppo/env/lidar_env/lidar_omni_target.py */
#define DGPPO_ENGINE_VMAS_WHEEL 4     /* VMASWheel contact physics: dgppo/env/vmas/vmas_wheel.py */
#define DGPPO_ENGINE_VMAS_TRANSPORT 5 /* VMASReverseTransport contact physics: dgppo/env/vmas/vmas_reverse_transport.py */
/* goal wiring */
#define DGPPO_GOAL_SPREAD 0 /* every agent sees every goal: lidar_spread.py:86-91, mpe_spread.py:64-69 */
#define DGPPO_GOAL_TARGET 1 /* agent i sees goal i only: lidar_target.py:77-84, mpe_target.py:63-70 */
/* reference env variants (goal wiring SPREAD, double integrator); reset, reward goals and costs differ */
#define DGPPO_VARIANT_NONE 0      /* the base envs above */
#define DGPPO_VARIANT_LINE 1      /* lidar_line.py, mpe_line.py: 2 landmark goal nodes, reward goals on the segment */
#define DGPPO_VARIANT_FORMATION 2 /* mpe_formation.py: 1 landmark goal node, reward goals on a circle around it */
#define DGPPO_VARIANT_CORRIDOR 3  /* mpe_corridor.py: 2 fixed wall obstacles, always-connected obstacle edges */
#define DGPPO_VARIANT_CONNECT 4   /* mpe_connect_spread.py: + connectivity cost (n_cost 3), 1 obstacle */

/* Obstacle record (LidarEnv rectangles), 16 floats = 64 B per obstacle:
 *   [cx, cy, width, height, theta, cos(theta), sin(theta), type, p0x, p0y, p1x, p1y, p2x, p2y, p3x, p3y]
 * = Rectangle(type, center, width, height, theta, points) of env/obstacle.py:30-56 plus a cached cos/sin. */
#define DGPPO_OBST_FIELDS 16

/* VMAS engines (n_agents 3): graph of 4 nodes (3 agents + pad) and 9 agent-agent edges, node_dim 13 (Wheel)
 * / 20 (Transport), state_dim 4.  `states` rows 0..2 are the agents [x, y, vx, vy]; row 3 (the pad row,
 * 0-wide in the reference) carries the moving body: Wheel [line_angle, line_angvel, 0, 0], Transport
 * [box_x, box_y, box_vx, box_vy].  The `obstacles` buffer holds one record of DGPPO_VMAS_FIELDS floats per
 * env (written by reset, read by step / rollout): Wheel [goal_angle, avoid_angle, 0 x 6], Transport
 * [goal_x, goal_y, o0x, o0y, o1x, o1y, o2x, o2y].  All sizes / radii are fixed by the reference classes;
 * dgppo_env_cfg_finalize fills the layout fields from `engine`. */
#define DGPPO_VMAS_FIELDS 8

/* Static description of one environment family + size (the reference's env PARAMS,
 * env/__init__.py:31-55 make_env, and the graph layout of utils/graph.py:212-247). */
typedef struct dgppo_env_cfg {
  int32_t engine;     /* DGPPO_ENGINE_* */
  int32_t goal_mode;  /* DGPPO_GOAL_* */
  int32_t n_agents;   /* n */
  int32_t n_obs;      /* O */
  int32_t n_rays;     /* R (Lidar) */
  int32_t top_k;      /* k = top_k_rays (Lidar) */
  int32_t state_dim;  /* 4, or 5 for the bicycle */
  int32_t node_dim;   /* state_dim + 3 */
  int32_t n_nodes;    /* N, including the pad node (filled by dgppo_env_cfg_finalize) */
  int32_t n_edges;    /* E (filled by dgppo_env_cfg_finalize) */
  float dt;           /* 0.03 (env/__init__.py:53) */
  float comm_radius;  /* 0.5, or 10*area with full_observation */
  float car_radius;   /* 0.05 */
  float obs_radius;   /* MPE obstacle radius 0.05 */
  float area_size;    /* 1.5 */
  float dist2goal;    /* 0.01 */
  float obs_len_lo, obs_len_hi; /* Lidar obstacle side range [0.1, 0.3] */
  float obs_theta_lo, obs_theta_hi; /* obstacle angle range: [0, 2pi) Lidar, [-pi, pi) bicycle */
  float state_lo[8], state_hi[8]; /* state_lim() */
  /* Derived constants.  The reference forms them in Python float64 and rounds once to fp32 when they
   * meet an fp32 array, so the host computes them the same way; finalize fills any left at 0. */
  float c_agent_cost;   /* car_radius * 2                      (lidar_env/base.py:188, mpe/base.py:173) */
  float c_obs_cost;     /* Lidar car_radius / MPE car+obs rad.  (lidar_env/base.py:197, mpe/base.py:181) */
  float c_self_dist;    /* comm_radius + 1                      (lidar_spread.py:75) */
  float c_lidar_active; /* comm_radius - 0.1                    (lidar_spread.py:97) */
  float c_min_dist;     /* reset min distance 2.2r Lidar / 2r MPE (lidar_env/base.py:111, mpe/base.py:88) */
  float c_inside_r;     /* min_dist / 2                         (env/utils.py:173, 195) */
  float c_mpe_obs_agent, c_mpe_obs_goal; /* car+obs radius, 2*car+obs radius (mpe/base.py:104-105) */
  float c_mpe_obs_lo, c_mpe_obs_hi;     /* 3*car radius, area - 3*car radius (mpe/base.py:97-98) */
  /* Squared-distance thresholds (filled by finalize): the smallest fp32 x with sqrt(x) >= r, so the
   * reference's `norm(d) < r` masks are decided exactly as `|d|^2 < t2` (sqrt is correctly rounded
   * and monotone).  t2_comm: r = comm_radius (agent-agent edges); t2_lidar: r = c_lidar_active. */
  float t2_comm, t2_lidar;
  /* filled by finalize from the engine: edge feature / action / cost widths (4, 2, 2; Omni 10, 3, 5) */
  int32_t edge_dim, action_dim, n_cost;
  /* LidarOmniTarget PARAMS (lidar_omni_target.py:49-68): max_angular_vel (state limit of omega),
   * fov_angle_deg (FoV half-angle beta), max_sensor_range (r_max), min_safe_distance (D),
   * rotation_penalty; c_cos_fov = cos(deg2rad(fov_angle_deg)) in fp32 (filled by finalize). */
  float omni_max_w, fov_angle_deg, fov_rmax, fov_dmin, rot_pen, c_cos_fov;
  /* ABI 6: env variants (all zero for the base envs).  Graph layout: agents | n_goals goal rows |
   * hits or obstacles | pad.  Constants in Python float64 rounded once, like the fields above. */
  int32_t variant;        /* DGPPO_VARIANT_* */
  int32_t n_goals;        /* goal node rows (0 -> n_agents; line 2, formation 1) */
  int32_t goals_inner;    /* line: 1 = the n interior points of the segment (mpe_line.py n <= 3) */
  float goal_radius;      /* formation: reward goals on this circle (comm_radius, mpe_formation.py:92-96) */
  float obs_edge_radius;  /* MPE agent-obstacle edge mask radius (0 -> comm_radius; corridor/connect comm*100) */
  float connect_radius;   /* connect: 0.45 */
  float sample_side_y;    /* corridor/connect: get_node_goal_rng side_length_y */
  float goal_shift_y;     /* corridor/connect: goals += [0, goal_shift_y] after sampling */
  float line_min_dist;    /* line: landmark separation */
  float c_obs_inflate;    /* lidar_line: obstacle placement radius 1.1 car_radius */
  float formation_lo, formation_hi; /* formation: landmark coordinate range [R + 2r, area - R - 2r] */
  float c_connect_min;    /* connect: agent sampling min_dist 2.3 car_radius */
  float line_box_x, line_box_y, line_off_y; /* line: l0 candidate box [0, area - side] x [0, side], y offset area/2 - side */
  float obs_x_hi;         /* corridor / connect: area - obs_radius */
} dgppo_env_cfg;

/* Fills n_nodes / n_edges / node_dim / state_lo/hi and zero derived constants from the other
 * fields; returns 0 or DGPPO_EINVAL. */
int dgppo_env_cfg_finalize(dgppo_env_cfg* cfg);

/* Host-side helper: writes the (R, 2) ray end-offset table (cos th_r * range, sin th_r * range) to
 * HOST memory `out`, th = jnp.linspace(-pi, pi - 2pi/R, R) formed as JAX does in fp32
 * (dgppo/env/utils.py:51-55).  Copy it to the device and pass it as `ray_dirs`. */
int dgppo_ray_table(int32_t n_rays, float sense_range, float* out);

/* One batched env step: replaces `vmap(env.step)` —
 *   LidarEnv.step   dgppo/env/lidar_env/base.py:151-174 (+ get_lidar_data 126-140, get_cost 180-207,
 *                   get_graph 227-271, edge_blocks lidar_spread.py:54-96 / lidar_target.py:54-96,
 *                   bicycle dynamics lidar_bicycle_target.py:92-118)
 *   MPE.step        dgppo/env/mpe/base.py:137-158 (+ get_cost 164-191, get_graph 211-241,
 *                   edge_blocks mpe_spread.py:51-81 / mpe_target.py:51-80)
 * Inputs are the current graph's `states` (B, N, sd) — agents, goals, lidar hits / MPE obstacles are
 * read from their fixed rows exactly as GraphsTuple.type_states does — the Lidar obstacle records
 * (B, O, 16) of env_states, and the actions (B, n, 2).  Outputs are the next graph's nodes (B,N,nd),
 * edges (B,E,4), states (B,N,sd), receivers/senders (B,E) int32, plus reward (B,) and cost (B,n,2)
 * evaluated on the current graph.  Every pointer has its own per-env stride (in elements) so a step
 * can write straight into a (B, T+1, ...) rollout buffer.  Outputs must not alias inputs. */
typedef struct dgppo_env_step_io {
  const float* states;      int64_t states_stride;
  const float* obstacles;   int64_t obstacles_stride; /* Lidar only (may be NULL when n_obs == 0) */
  const float* action;      int64_t action_stride;
  const float* ray_dirs;    /* (R, 2): cos(th_r)*range, sin(th_r)*range (Lidar only) */
  float* nodes;             int64_t nodes_stride;
  float* edges;             int64_t edges_stride;
  float* out_states;        int64_t out_states_stride;
  int32_t* receivers;       int32_t* senders; int64_t edge_index_stride;
  float* reward;            int64_t reward_stride;
  float* cost;              int64_t cost_stride;
  int32_t n_env;
} dgppo_env_step_io;

int dgppo_env_step(const dgppo_env_cfg* cfg, const dgppo_env_step_io* io, void* stream);

/* Step-kernel selection (no reference counterpart; both kernels are bit-identical): 0 = auto (the
 * wave-per-env kernel for Lidar n=8 / 32 rays / top-8 / 3 obstacles, the workgroup-per-env kernel
 * otherwise), 1 = workgroup-per-env everywhere.  Returns the previous mode or DGPPO_EINVAL.
 * Initial mode: DGPPO_ENV_STEP_KERNEL=block|auto (default auto). */
int dgppo_env_set_step_kernel(int mode);

/* Batched reset: replaces `vmap(env.reset)(keys)` —
 *   LidarEnv.reset dgppo/env/lidar_env/base.py:89-124, LidarBicycleTarget.reset
 *   lidar_bicycle_target.py:60-90, MPE.reset dgppo/env/mpe/base.py:81-127, with the rejection
 *   sampler get_node_goal_rng dgppo/env/utils.py:139-244.
 * Env b draws from Philox4x32-10 keyed (seed, env_offset + b) (jax.random threefry is not
 * reproducible here).  Writes the initial graph (same fields as a step) and, for Lidar, the
 * obstacle records (B, O, 16). */
typedef struct dgppo_env_reset_io {
  uint64_t seed;
  const uint64_t* seed_ptr; /* optional device scalar; when non-NULL it overrides `seed` (lets a
                               captured hipGraph replay draw a fresh episode per replay) */
  int32_t env_offset;
  float* obstacles;         int64_t obstacles_stride; /* out (Lidar) */
  const float* ray_dirs;
  float* nodes;             int64_t nodes_stride;
  float* edges;             int64_t edges_stride;
  float* out_states;        int64_t out_states_stride;
  int32_t* receivers;       int32_t* senders; int64_t edge_index_stride;
  int32_t n_env;
} dgppo_env_reset_io;

int dgppo_env_reset(const dgppo_env_cfg* cfg, const dgppo_env_reset_io* io, void* stream);

/* The sampling half of dgppo_env_reset: obstacle records and the agent / goal rows of `out_states`
 * only (no graph); dgppo_env_rollout with rebuild_first = 1 then builds graph 0 itself.  Configs
 * without a persistent rollout kernel get the full reset (the graph is written too). */
int dgppo_env_reset_states(const dgppo_env_cfg* cfg, const dgppo_env_reset_io* io, void* stream);

/* T env steps with given actions in one call: replaces the env half of the reference's rollout scan
 * `lax.scan(body, ...)` over env.step (dgppo/trainer/utils.py:45-55) for a fixed action sequence.
 * `step` describes graph 0 and step 0: graph t's rows live at the graph pointers + t * t_<field>
 * (states / nodes / edges / receivers+senders, element strides, e.g. a time-major (T+1, B, ...)
 * buffer), the actions of step t at action + t * t_action, reward[t] / cost[t] at + t * t_reward /
 * t_cost.  Step t reads graph t and writes graph t+1, reward[t], cost[t]; rebuild_first = 1 first
 * writes graph 0's rows from its agent / goal states and obstacles (after dgppo_env_reset_states).
 * Lidar configs at n = 8, 32 rays, top-8, 3 obstacles run one persistent kernel (a wave per env for
 * all T steps, state in LDS); others loop dgppo_env_step (identical results). */
typedef struct dgppo_env_rollout_io {
  dgppo_env_step_io step;   /* graph 0 in / out (states == out_states), actions / reward / cost of step 0 */
  int32_t T;
  int32_t rebuild_first;
  int64_t t_states, t_nodes, t_edges, t_index, t_action, t_reward, t_cost;
} dgppo_env_rollout_io;

int dgppo_env_rollout(const dgppo_env_cfg* cfg, const dgppo_env_rollout_io* io, void* stream);

/* ---- hot path (2): DGPPO update building blocks ------------------------------------------------
 * Batched fp32 GEMM on the matrix cores (v_mfma_f32_32x32x2_f32):
 *   C[b] = alpha * op(A[b]) op(B[b]) + beta * C[b] + bias[N] + addend[b]   (optional ReLU)
 * op(A) = A (M,K) row-major, or trans_a: A stored (K,M); op(B) = B (K,N), or trans_b: stored (N,K).
 * Every flax `nn.Dense` of the reference networks (dgppo/nn/mlp.py:15-30, nn/gnn.py:86-111,
 * algo/module/policy.py:67-71, value.py:253,288, flax GRUCell) and its two backward GEMMs map here.
 * split_k > 1 computes K in slices into `workspace` (dgppo_gemm_workspace_floats floats) and reduces
 * them in a fixed order (bitwise-deterministic weight gradients, no float atomics). */
/* Row grouping (a_grp/b_grp/c_grp/add_grp > 0): stored row r lives at (r / grp) * gstride + (r % grp) * ld,
 * e.g. the n agent rows of every graph inside a (G, N, D) node tensor (grp = n, gstride = N*D).  Stored rows are M (A), K (trans_a A), K (B), N (trans_b B), M (C). */
typedef struct dgppo_gemm_args {
  int32_t M, N, K, batch;
  int32_t trans_a, trans_b;
  const float* A; int64_t lda, stride_a;
  const float* B; int64_t ldb, stride_b;
  float* C;       int64_t ldc, stride_c;
  int32_t a_grp, b_grp, c_grp, pad_;
  int64_t a_gstride, b_gstride, c_gstride;
  const float* bias;                          /* (N) or NULL */
  const float* addend; int64_t ld_add, stride_add; /* (M,N) per batch or NULL */
  int32_t add_grp, pad2_; int64_t add_gstride;     /* addend row grouping (independent of C's) */
  float alpha, beta;
  int32_t relu;
  int32_t split_k;
  float* workspace;
  float* bias_grad;  /* trans_a && !trans_b only: bias_grad[n] = alpha * sum_k B[k][n] + beta * bias_grad[n]
                        (the dense layer's db fused into its dW = X^T dY), or NULL */
  /* ABI 9: elementwise pass fused into the epilogue of the row-GEMM paths (!trans_a, N <= 192, K <= 256; else
   * DGPPO_EINVAL).  epi 0: none.  1: relu mask, C = mask > 0 ? result : 0 (mask rows addressed like C with
   * ld_mask; the ReLU backward of the layer that produced `mask`, nn/gnn.py:116).  2: LayerNorm(64) + ReLU
   * forward (flax LayerNorm eps 1e-6 + relu, nn/mlp.py:20-30; N == 64, no beta / addend / relu): ln_h (M, 64)
   * <- result, C <- relu(((ln_h - mean) rstd) ln_scale + ln_bias), ln_mean / ln_rstd (M) <- the row
   * statistics.  3: its backward: the result is dy; with ln_h, ln_mean and ln_rstd as epi 2 wrote them (the
   * ReLU gates are the forward's, bit for bit), C <- dx and the per-workgroup
   * partials [dscale (64) | dbias (64)] to ln_part (dgppo_gemm_partial_rows rows of 128; sum them, e.g. with
   * dgppo_colsum). */
  int32_t epi, pad3_;
  const float* mask; int64_t ld_mask;
  const float* ln_scale; const float* ln_bias;
  float* ln_h; float* ln_mean; float* ln_rstd; float* ln_part;
} dgppo_gemm_args;

int64_t dgppo_gemm_workspace_floats(const dgppo_gemm_args* args);
/* ABI 13: n weight-gradient GEMMs (each trans_a, !trans_b, on dgppo_gemm's weight-gradient path: N <= 192,
 * M <= 4096, no bias / addend / relu / epi) in one launch plus one partial-reduction launch (per 12 problems),
 * every output bit-identical to its own dgppo_gemm call -- a network pass's weight gradients deferred to the end
 * of its backward (dgppo/algo/informarl.py:357-457 grads of one loss).  `workspace`: the floats
 * dgppo_gemm_wgrad_grouped_workspace_floats(args, n) returns (their own region per problem).  The problems' C /
 * bias_grad regions must not overlap one another. */
int64_t dgppo_gemm_wgrad_grouped_workspace_floats(const dgppo_gemm_args* args, int n);
int dgppo_gemm_wgrad_grouped(const dgppo_gemm_args* args, int n, float* workspace, void* stream);
/* rows of ln_part an epi 3 call writes (its workgroup count; 0 when the call is not on the row-GEMM paths) */
int64_t dgppo_gemm_partial_rows(const dgppo_gemm_args* args);
int dgppo_gemm(const dgppo_gemm_args* args, void* stream);

/* GraphTransformer attention core (dgppo/nn/gnn.py:78-117 + jraph.segment_softmax/segment_sum),
 * per RECEIVING AGENT: only agents receive messages in the DGPPO env graphs, so with
 * qt_h = Wk_h q_h the logits are (qt_h . x_s + q_h . bk_h) / sqrt(F) and the aggregated message is
 * xbar_h Wv_h + sig_h bv_h + ebar_h We_h (see csrc/attn.hip).  fwd writes attn (G*n, H, C) and
 * xcat (G*n, H*(D+5)) = [xbar (H*D) | ebar (H*4) | sig (H)]; bwd consumes dxcat and writes dqt,
 * dq (= dbeta_h * bk_h), dbeta and the sender gradients.
 * cand (n, C): edge ids that may target agent i (checked against receivers at run time).
 * Sender features, two modes:
 *   full  (xa == NULL): x (G, N, D) holds every node's features; bwd ACCUMULATES dx (G, N, D).
 *   agent (xa != NULL): agent senders (node < n) read xa (G, n, D); other senders are nodes that
 *         never receive, so their features are a function of their raw row x (G, N, D0):
 *         relu(x pre_W + pre_b) (the previous layer's Dense_4 with an empty aggregation), or x
 *         itself when pre_W == NULL (D0 == D).  bwd ACCUMULATES dxa (G, n, D) and writes per-block
 *         partial gradients of [pre_W (D0*D) | pre_b (D)] into dpre_part
 *         (dgppo_gnn_attn_partial_blocks rows; reduce with dgppo_colsum). */
typedef struct dgppo_gnn_attn_args {
  int32_t G, N, E, n_agents, D, F, H, C;
  const int32_t* cand;
  const int32_t* receivers;
  const int32_t* senders;     /* (G, E) */
  const float* x; int64_t x_gstride;   /* node features (G, N, D) [full] / raw (G, N, D0) [agent mode] */
  const float* ef; int64_t ef_gstride; /* edge features (G, E, 4) */
  const float* q;   /* (G*n, H*F) */
  const float* qt;  /* (G*n, H*D) */
  const float* bk;  /* (H*F) */
  float* attn;      /* (G*n, H, C) */
  float* xcat;      /* (G*n, H*(D+5)) */
  const float* dxcat;
  float* dqt;
  float* dq;
  float* dbeta;     /* (G*n, H) */
  float* dx; int64_t dx_gstride;
  float scale;      /* 1/sqrt(F) */
  int32_t D0;       /* raw feature width (agent mode) */
  const float* xa; int64_t xa_gstride;  /* agent-mode agent rows (G, n, D) */
  const float* pre_W; const float* pre_b;
  float* dxa; int64_t dxa_gstride;
  float* dpre_part;
  const int32_t* sidx;  /* optional (G*n, C) sender table from dgppo_gnn_sender_table (else resolved per use) */
  const float* da_add;  /* optional (G*n, H, C) extra dL/d attn added in the softmax backward: the edge columns
                           past the first 4 (dgppo_gnn_edge_da) */
  /* Q-free form (ABI 5): beta (G*n, H) with row stride beta_ld = q_h . bk_h precomputed (then q is not
   * read and may be NULL); row strides of qt / dqt / dbeta (0 = packed H*D / H*D / H), so [qt | beta]
   * and [dqt | dbeta] can share one (G*n, H*D + H) buffer; dq == NULL skips the (G*n, H*F) dq rows. */
  const float* beta; int64_t beta_ld;
  int64_t qt_ld, dqt_ld, dbeta_ld;
} dgppo_gnn_attn_args;

int64_t dgppo_gnn_attn_partial_blocks(const dgppo_gnn_attn_args* args);
/* ABI 10, tuning / testing hook: 1 (default) = the graph-form forward computes each receiver's own
 * never-receiver rows on the fly (Lidar layout, D = 32 agent mode with pre_W: only agent and goal rows staged
 * in LDS), 0 = every row staged; bit-identical either way.  Process-wide; also DGPPO_ATTN_GRAPH_OTF=0|1. */
int dgppo_gnn_set_graph_otf(int32_t on);
/* sidx[(g*n + i)*C + c] = senders[g][cand[i][c]] if that edge's receiver is i, else -1: the
 * candidate resolution shared by every attention launch on one graph batch */
int dgppo_gnn_sender_table(int32_t G, int32_t n_agents, int32_t C, int32_t E, const int32_t* cand,
                           const int32_t* receivers, const int32_t* senders, int32_t* sidx, void* stream);
int dgppo_gnn_attn_fwd(const dgppo_gnn_attn_args* args, void* stream);
int dgppo_gnn_attn_bwd(const dgppo_gnn_attn_args* args, void* stream);
/* ABI 11: one GraphTransformer layer forward as ONE kernel (dgppo/nn/gnn.py:78-117: Dense_0 / Dense_1 queries and
 * keys, segment softmax over each receiving agent's incoming edges, Dense_2 / Dense_3 messages, Dense_4 update and
 * ReLU), replacing the [qt | beta] GEMM, dgppo_gnn_attn_fwd and the two message / update GEMMs of the layer:
 *   [qt | beta] = [x_i 1] QBW,   xcat = attention over the candidates (as dgppo_gnn_attn_fwd),
 *   Y = relu(xcat Wcat / H + x_i Wu + bu)
 * with x_i the receiving agent's input row (full mode: node i of x; agent mode: row i of xa).  Each workgroup
 * stages whole graphs (raw / agent rows, never-receivers' relu(x_raw pre_W + pre_b) computed once per node) in
 * LDS with coalesced loads, so the per-candidate reads are LDS reads.  `a` carries the graph and the sender mode
 * exactly as for dgppo_gnn_attn_fwd (sidx required; a.q / a.qt / a.beta are not read); a.attn, a.xcat and qb are
 * OPTIONAL outputs (what dgppo_gnn_attn_bwd and the weight gradients read; NULL in forward-only passes).  Scope:
 * H = 3, C <= 32, n <= 16, F <= 64, 4-wide edges; full mode with D <= 8, or agent mode with D = 32, D0 <= 8 and
 * pre_W (dgppo_gnn_layer_supported; otherwise use the unfused chain). */
/* Forward-only epilogues of the value networks (forward passes whose intermediates nobody reads):
 *   zmean (G, F): the per-graph mean of Y over its n agent rows (VlNet's agent mean, value.py:35-37, summed over
 *         the agents in order then divided by n, as dgppo_agent_mean_fwd); Y may then be NULL;
 *   tail (tail.on = 1, F = 64): DecRStateFn's head after a 1-layer GNN (value.py:67-79, dgppo.py:83-95): MLP
 *         (Dense(64) + LayerNorm + ReLU x 2) -> GRUCell(64) fed the carries h_in -> Dense(n_out), written to
 *         tail.out (G*n, n_out <= 16); Y, qb, a.attn and a.xcat must then be NULL. */
typedef struct dgppo_gnn_value_tail {
  const float* W0; const float* b0; const float* ln0_s; const float* ln0_b;  /* head Dense_0 (64 x 64), LayerNorm_0 */
  const float* W1; const float* b1; const float* ln1_s; const float* ln1_b;  /* head Dense_1, LayerNorm_1 */
  const float* Wi; const float* bi; const float* Wh; const float* bhn;      /* GRUCell: (64, 192) [r|z|n], (192), (64, 192), (64) */
  const float* Wo; const float* bo;                                         /* output Dense (64, n_out), (n_out) */
  const float* h_in;                                                        /* (G*n, 64) carries */
  float* out;                                                               /* (G*n, n_out) */
  int32_t n_out, on;
} dgppo_gnn_value_tail;
typedef struct dgppo_gnn_layer_args {
  dgppo_gnn_attn_args a;
  const float* QBW;                  /* (D+1, H*D + H): [x 1] QBW = [qt | beta] (Q-free query-key products) */
  float* qb;                         /* optional out (G*n, H*D + H) [qt | beta] rows */
  const float* Wcat;                 /* (H*(D+5), F) = [Wv (H*D); We (H*4); bv (H)] per head */
  const float* Wu; const float* bu;  /* Dense_4: (D, F), (F) */
  float* Y;                          /* (G*n, F) (NULL allowed with zmean or the tail) */
  float* zmean;                      /* optional out (G, F) */
  dgppo_gnn_value_tail tail;
} dgppo_gnn_layer_args;
int dgppo_gnn_layer_supported(const dgppo_gnn_layer_args* args);
int dgppo_gnn_layer_fwd(const dgppo_gnn_layer_args* args, void* stream);

/* Edge features wider than 4 (LidarOmniTarget's 10-wide edges, lidar_omni_target.py edge_dim): the attention
 * kernels see columns 0..3, the remaining EX columns efx (G, E, EX) go through these two.
 *   edge_wsum: out[r, h*EX + j] = sum_c attn[r, h, c] * efx[g, cand[i][c], j] over sidx[r][c] >= 0
 *              (the attention-weighted edge term of the value messages, dgppo/nn/gnn.py:99-104)
 *   edge_da:   da_add[r, h, c] = sum_j dxx[r, h*EX + j] * efx[g, cand[i][c], j] if sidx[r][c] >= 0 else 0
 * with r = g*n + i; EX <= 16. */
int dgppo_gnn_edge_wsum(int32_t G, int32_t n_agents, int32_t C, int32_t H, int32_t EX, int32_t E, const float* attn,
                        const int32_t* cand, const int32_t* sidx, const float* efx, float* out, void* stream);
int dgppo_gnn_edge_da(int32_t G, int32_t n_agents, int32_t C, int32_t H, int32_t EX, int32_t E, const float* dxx,
                      const int32_t* cand, const int32_t* sidx, const float* efx, float* da_add, void* stream);

/* flax LayerNorm (+ReLU) over rows of width F (dgppo/nn/mlp.py:27-29); bwd accumulates dscale/dbias */
int dgppo_layernorm_fwd(const float* x, const float* scale, const float* bias, float* y, float* mean, float* rstd,
                        int64_t rows, int32_t F, int32_t relu, float eps, void* stream);
int64_t dgppo_layernorm_bwd_workspace_floats(int64_t rows, int32_t F);
int dgppo_layernorm_bwd(const float* x, const float* y, const float* dy, const float* scale, const float* mean,
                        const float* rstd, float* dx, float* dscale, float* dbias, int64_t rows, int32_t F,
                        int32_t relu, float* workspace, void* stream);

/* dy *= (y > 0) in place (ReLU backward) */
int dgppo_relu_bwd(float* dy, const float* y, int64_t n, void* stream);

/* flax.linen.LSTMCell, one step of `rows` contiguous carries (the --use-lstm option; replaces the LSTMCell
 * branch of RNN.__call__, dgppo/nn/rnn.py:21-23).  fwd: g (rows, 4H) = [i | f | g | o] pre-activations
 * (x W_i + h W_h + b) are activated in place, c_out = f c_prev + i g, h_out = o tanh(c_out); c_prev may be NULL
 * (zero carry).  bwd: g = the activated gates, c = c_out, dh = dL/dh_out, dc = dL/dc_out from the next step
 * (NULL: 0) -> dg (rows, 4H) pre-activation gradients and dc_prev = dL/dc_prev (NULL: not written). */
int dgppo_lstm_cell_fwd(int64_t rows, int32_t H, float* g, const float* c_prev, float* c_out, float* h_out,
                        void* stream);
int dgppo_lstm_cell_bwd(int64_t rows, int32_t H, const float* g, const float* c_prev, const float* c, const float* dh,
                        const float* dc, float* dg, float* dc_prev, void* stream);

/* out = alpha * column_sums(x) + beta * out (deterministic; bias gradients) */
int64_t dgppo_colsum_workspace_floats(int64_t rows, int32_t cols);
int dgppo_colsum(const float* x, int64_t rows, int32_t cols, int64_t ld, int32_t grp, int64_t gstride, float* out,
                 float alpha, float beta, float* workspace, void* stream);

/* flax GRUCell (dgppo/nn/rnn.py:15-30): gi = x Wi + bi, gh = h Wh (r|z|n blocks), bhn = hn bias */
int dgppo_gru_fwd(const float* gi, const float* gh, const float* bhn, const float* h, float* h_new, int64_t rows,
                  int32_t H, void* stream);
int dgppo_gru_bwd(const float* gi, const float* gh, const float* bhn, const float* h, const float* dh_new,
                  float* dgi, float* dgh, float* dh, int64_t rows, int32_t H, void* stream);

/* Whole-sequence GRU (the rnn_step scans of informarl.py:281-293 / 387-403 and the 1-step carries
 * of act / get_Vh) in one launch per direction.  Q sequence rows (q = s * n_agents + a) over L steps;
 * step-t row of sequence row q in the (rows = Q*L) tensors: ((q / n_agents) * L + t) * n_agents +
 * q % n_agents.  gi = x Wi + bi for all rows is computed outside (one GEMM).  H must be 64.
 *   fwd: hs[row] = h_t (carry after step t), hT (optional) = h_{L-1}; h0 NULL = zero carries.
 *   bwd: from dhs (upstream grads on hs) writes dgi = [dr|dz|dn] and dgh = [dr|dz|dn*r] (pre-
 *        activation grads; dWi = x^T dgi, dbi = colsum dgi, dWh = h_{t-1}^T dgh are GEMMs outside),
 *        dh0 (optional), and dbhn_part[b][H] = per-workgroup column sums of dn*r over its rows
 *        (dgppo_gru_seq_blocks(Q) workgroups; reduce with dgppo_colsum). */
typedef struct dgppo_gru_seq_args {
  int32_t Q, L, n_agents, H;
  const float* gi;     /* (rows, 3H) */
  const float* Wh;     /* (H, 3H) */
  const float* bhn;    /* (H) */
  const float* h0;     /* (Q, H) or NULL */
  float* hs;           /* (rows, H): fwd output, bwd input */
  float* hT;           /* (Q, H) or NULL */
  const float* dhs;    /* (rows, H) */
  float* dgi;          /* (rows, 3H) */
  float* dgh;          /* (rows, 3H) */
  float* dh0;          /* (Q, H) or NULL */
  float* dbhn_part;    /* (blocks, H) or NULL */
} dgppo_gru_seq_args;

int64_t dgppo_gru_seq_blocks(int32_t Q);
int dgppo_gru_seq_fwd(const dgppo_gru_seq_args* args, void* stream);
int dgppo_gru_seq_bwd(const dgppo_gru_seq_args* args, void* stream);
/* ABI 10, tuning / testing hook: 1 (default) = Wh as per-lane register MFMA fragments, 0 = Wh staged in LDS
 * (the round-3 kernels); bit-identical results either way.  Process-wide; also DGPPO_GRU_REGB=0|1. */
int dgppo_gru_set_form(int32_t regb);

/* Fused policy step (one launch per env step of the rollouts): GNN -> MLP head -> GRUCell ->
 * ScaleHid -> mean/std -> TanhNormal sample (mode 1, standard-normal noise) or mode (mode 0), i.e.
 * PPOPolicy.sample_action / get_action (dgppo/algo/module/policy.py:191-203) for G graphs at once.
 * Parameter pointers are the layouts of dgppo_fov_amd/nn/layers.py (GraphTransformer: Wq (D, H F),
 * bq, Wkt (H, F, D), bk, Wcat (H (D+5), F) = [Wv; We; bv], Wu (D, F), bu; GRU Wi (64, 192) [r|z|n],
 * bi, Wh (64, 192), bhn).  dgppo_policy_step_supported() tells whether a configuration fits the
 * fused kernel (n <= 32, C <= 32, D0 <= 8, H = 3, actor GNN D0->32->64 or D0->64, A in {1, 2, 4}).
 * `work` (dgppo_policy_work_floats() floats) holds the per-layer query-key products
 * [Wq_h Wkt_h | Wq_h bk_h] and their biases; dgppo_policy_prepare() fills it from the current weights
 * and must run after every weight change (the rollouts call it once per rollout, inside the graph). */
typedef struct dgppo_gt_layer {
  const float *Wq, *bq, *Wkt, *bk, *Wcat, *Wu, *bu;
  int32_t D, F;
  const float* Wex; /* (H (ED - 4), F) weights of the edge columns past 4 (LidarOmniTarget), NULL for ED == 4 */
} dgppo_gt_layer;

typedef struct dgppo_policy_step_args {
  int32_t G, N, E, n_agents, C, D0, A, n_layers, H, mode;
  int32_t ED, pad_;    /* edge feature width: 4, or up to 10 (LidarOmniTarget) with layer[].Wex */
  const int32_t* cand;
  const float* nodes; int64_t nodes_gstride;   /* (G, N, D0), D0 <= 12 */
  const float* edges; int64_t edges_gstride;   /* (G, E, ED) */
  const int32_t* receivers;
  const int32_t* senders; int64_t idx_gstride; /* (G, E) */
  dgppo_gt_layer layer[2];
  const float *head_W0, *head_b0, *ln0_s, *ln0_b, *head_W1, *head_b1, *ln1_s, *ln1_b;
  const float *gru_Wi, *gru_bi, *gru_Wh, *gru_bhn;
  const float *Ws, *bs, *Wm, *bm, *Wsd, *bsd;
  float std_shift, std_min;
  const float* h_in;   /* (G n, 64) */
  float* h_out;        /* (G n, 64) */
  const float* noise;  /* (G n, A), mode 1; NULL: drawn in the kernel from noise_seed (ABI 10) */
  float* action;       /* (G n, A) */
  float* log_pi;       /* (G n) or NULL */
  float* work;         /* dgppo_policy_work_floats() floats */
  /* ABI 10, mode 1 with noise == NULL: element row * A + q of the standard-normal stream
   * (*noise_seed, noise_stream), bit-identical to dgppo_normal(buffer, G n A, noise_seed, 0, noise_stream) */
  const uint64_t* noise_seed;
  uint64_t noise_stream;
} dgppo_policy_step_args;

int dgppo_policy_step_supported(const dgppo_policy_step_args* args);
int64_t dgppo_policy_work_floats(void);
int dgppo_policy_prepare(const dgppo_policy_step_args* args, void* stream);
int dgppo_policy_step(const dgppo_policy_step_args* args, void* stream);

/* mean over the agents of each graph (RStateFn, dgppo/algo/module/value.py:29) */
int dgppo_agent_mean_fwd(const float* x, float* y, int64_t G, int32_t n, int32_t F, int64_t x_gstride, void* stream);
int dgppo_agent_mean_bwd(const float* dy, float* dx, int64_t G, int32_t n, int32_t F, int64_t dx_gstride,
                         void* stream);
/* ABI 10: the same with the ReLU backward of the rows that fed the mean fused in: dx = mask > 0 ? dy / n : 0,
 * mask (G n, F) contiguous (dgppo_agent_mean_bwd then dgppo_relu_bwd(dx, mask), in one pass) */
int dgppo_agent_mean_bwd_masked(const float* dy, const float* mask, float* dx, int64_t G, int32_t n, int32_t F,
                                int64_t dx_gstride, void* stream);

/* TanhNormal head (dgppo/algo/module/policy.py:61-74, distribution.py:10-66): std = softplus(raw +
 * std_shift) + std_min; mode 0 = tanh(mean), 1 = tanh(mean + std * noise), 2 = evaluate `action`.
 * log_pi / entropy summed over the A action dims; entropy uses a fixed per-agent eps (n_agents, A).
 * If dmean is set, writes the backward of (dlog_pi, dentropy) into dmean / dstd_raw. */
typedef struct dgppo_tanh_normal_args {
  int64_t rows;
  int32_t A, mode, n_agents, pad_;
  const float* mean;
  const float* std_raw;
  float std_shift, std_min;
  const float* noise;
  const float* action;
  float* action_out;
  float* std_out;
  float* log_pi;
  float* entropy;
  const float* entropy_eps;
  const float* dlog_pi;
  const float* dentropy;
  float* dmean;
  float* dstd_raw;
} dgppo_tanh_normal_args;

int dgppo_tanh_normal(const dgppo_tanh_normal_args* args, void* stream);

/* losses: PPO clipped surrogate + entropy bonus (dgppo/algo/informarl.py:428-438) and
 * optax.l2_loss mean (informarl.py:374, dgppo.py:310); gradients are d(mean loss)/d(input) */
int64_t dgppo_loss_workspace_floats(void);
int dgppo_ppo_loss(const float* log_pi, const float* log_pi_old, const float* adv, const float* entropy, int64_t n,
                   float clip_eps, float coef_ent, float* dlog_pi, float* dentropy, float* stats, float* workspace,
                   void* stream);
int dgppo_l2_loss(const float* pred, const float* target, int64_t n, float* dpred, float* loss, float* workspace,
                  void* stream);

/* compute_dec_ocp_gae (dgppo/algo/utils.py:11-79), one workgroup per env; the reference's
 * lax.scan(reverse=True) step counter drives the mask and coefficients.  Limits: n*nh <= 255,
 * T <= 1024 and one env's inputs (T*K + (T+1)*K + 4T + 3 floats) within 160 KiB of LDS. */
typedef struct dgppo_gae_args {
  int32_t B, T, n_agents, n_h;
  const float* hs;  /* (B, T, n, nh) costs */
  const float* l;   /* (B, T) */
  const float* Vh;  /* (B, T+1, n, nh) */
  const float* Vl;  /* (B, T+1) */
  float* Qh;        /* (B, T, n, nh) */
  float* Ql;        /* (B, T) */
  float gamma, lambda;
} dgppo_gae_args;

int dgppo_gae(const dgppo_gae_args* args, void* stream);

/* DGPPO advantages (dgppo/algo/dgppo.py:239-259): per env, Al = (Ql - Vl) normalised over T,
 * CBF derivative of Vh, A = -(where(safe, Al, 0) + max_h relu(cbf + cbf_eps) * cbf_weight);
 * safe_count[b] = number of safe (t, agent) pairs (for eval/safe_data). */
typedef struct dgppo_adv_args {
  int32_t B, T, n_agents, n_h;
  const float* Ql;  /* (B, T) */
  const float* Vl;  /* (B, T+1) */
  const float* Vh;  /* (B, T+1, n, nh) */
  float dt, alpha, cbf_eps, cbf_weight;
  float* A;         /* (B, T, n) */
  float* safe_count;/* (B) */
} dgppo_adv_args;

int dgppo_dgppo_advantages(const dgppo_adv_args* args, void* stream);

/* compute_norm_and_clip + optax.adam + apply_if_finite (dgppo/trainer/utils.py:105-118,
 * informarl.py:131-137): state = [global norm, non-finite count, adam step] on the device */
/* InforMARL (dgppo/algo/informarl.py:310-340): the GAE's cost-shaped loss
 *   l[b,t] = -rewards[b,t] + cost_weight * sum_a sum_h max(costs[b,t,a,h], 0)
 * and the per-env normalised advantages A[b,t,a] = -(Al - mean_t Al) / (std_t Al + 1e-8), Al = Ql - Vl[:, :T]
 * (Ql (B, T), Vl (B, T+1), A (B, T, n_agents)). */
int dgppo_cost_shaped_loss(const float* rewards, const float* costs, float cost_weight, float* l, int32_t B,
                           int32_t T, int32_t n_agents, int32_t n_h, void* stream);
int dgppo_informarl_advantages(const float* Ql, const float* Vl, float* A, int32_t B, int32_t T, int32_t n_agents,
                               void* stream);
int dgppo_grad_norm(const float* grad, int64_t n, float* state, float* workspace, void* stream);
/* b1 / b2 are doubles: (1 - b) is formed in double and rounded once, as optax's weakly typed
 * `(1 - decay) * g` does (ABI 3) */
int dgppo_adam(float* param, const float* grad, float* m, float* v, int64_t n, float* state, float lr, double b1,
               double b2, float eps, float max_norm, void* stream);

/* Replaces the per-train-state compute_norm_and_clip + apply_if_finite(adam) of DGPPO.update_inner's three updates
 * (trainer/utils.py:105-118, dgppo.py:275-289) in one call.
 * The grad_norm + adam pair of up to DGPPO_ADAM_MAX_NETS nets (each its own parameters, state, lr and clip norm) in
 * TWO launches instead of four per net (ABI 12): the sum-of-squares / non-finite partials of every net, then one
 * kernel whose workgroups each finish their net's norm from the partials (the arithmetic of dgppo_grad_norm's
 * second kernel) and apply the clipped Adam step; workgroup 0 of each net writes its state.  Every value is
 * bit-identical to dgppo_grad_norm + dgppo_adam per net.  workspace: dgppo_adam_multi_workspace_floats() floats. */
#define DGPPO_ADAM_MAX_NETS 4
typedef struct dgppo_adam_net {
  float* param;
  const float* grad;
  float* m;
  float* v;
  int64_t n;
  float* state; /* [global norm, non-finite count, adam step] */
  float lr;
  float max_norm;
} dgppo_adam_net;
typedef struct dgppo_adam_multi_args {
  int32_t n_nets;
  float eps;
  double b1, b2;
  float* workspace;
  dgppo_adam_net net[DGPPO_ADAM_MAX_NETS];
} dgppo_adam_multi_args;
int64_t dgppo_adam_multi_workspace_floats(void);
int dgppo_adam_multi(const dgppo_adam_multi_args* a, void* stream);

/* InforMARL-Lagr (dgppo/algo/informarl_lagr.py:125-309): y = max(x, 0) (the GAE's clipped costs, :196);
 * the merged advantage A = -norm_t(Ql - Vl) - mean_h(lagr norm_t(Qh - Vh)) with Ah = norm_t(Qh - Vh) out
 * (Ql (B,T), Vl (B,T+1), Qh (B,T,n,nh), Vh (B,T+1,n,nh), lagr (n,nh), :205-221); and update_lagr (:283-305):
 * lagr = relu(lagr - lr delta), delta = -mean over `rows` (env, t) of Vh (1 - gamma) + exp(log_pi -
 * log_pi_old) Ah, with lagr_mean (optional) = mean of the new multipliers. */
int dgppo_clip_min0(const float* x, float* y, int64_t n, void* stream);
int dgppo_lagr_advantages(const float* Ql, const float* Vl, const float* Qh, const float* Vh, const float* lagr,
                          float* A, float* Ah, int32_t B, int32_t T, int32_t n_agents, int32_t n_h, void* stream);
int dgppo_lagr_update(const float* log_pi, const float* log_pi_old, const float* Vh, const float* Ah, float* lagr,
                      float* lagr_mean, int64_t rows, int32_t n_agents, int32_t n_h, float gamma, float lr,
                      void* stream);

/* Minibatch assembly (the reference's `jtu.tree_map(lambda x: x[idx], rollout)`, dgppo.py:275-289): for
 * each field, output row o = e * T + t (e < n_sel) = the source row of env envs[e] at step t, read at
 * src + t * src_tstride + envs[e] * src_estride (elements), written contiguously (row_elems elements).
 * Fields (at most 8, a HOST array) are rows of 4-byte elements (fp32 / int32); `envs` is a DEVICE array. */
typedef struct dgppo_gather_field {
  const void* src; void* dst;
  int64_t row_elems, src_tstride, src_estride;
} dgppo_gather_field;

int dgppo_gather_env_steps(const dgppo_gather_field* fields, int32_t n_fields, const int64_t* envs, int32_t n_sel,
                           int32_t T, void* stream);

/* standard normal noise from Philox4x32-10 (Box-Muller); seed from *seed_ptr when non-NULL.  Element t uses
   counter (t lo, t hi, stream_id lo, stream_id hi | 0x80000000): the top bit is the noise domain, disjoint from
   the env-reset draws (counter (draw, env, purpose, 0)) under the same key.  Replaces the threefry draws of
   sample_action (policy.py:196-203, jax.random.normal inside tfd.Normal.sample). */
int dgppo_normal(float* out, int64_t n, const uint64_t* seed_ptr, uint64_t seed, uint64_t stream_id, void* stream);

/* Library / device introspection */
int dgppo_abi_version(void);
const char* dgppo_build_info(void);

#ifdef __cplusplus
}
#endif
#endif /* DGPPO_HIP_H */
