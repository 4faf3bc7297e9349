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

#define DGPPO_ABI_VERSION 1
#define DGPPO_EINVAL (-22)

/* engines */
#define DGPPO_ENGINE_LIDAR 0   /* LidarEnv double integrator: dgppo/env/lidar_env/base.py */
#define DGPPO_ENGINE_BICYCLE 1 /* LidarBicycleTarget: dgppo/env/lidar_env/lidar_bicycle_target.py */
#define DGPPO_ENGINE_MPE 2     /* MPE double integrator: dgppo/env/mpe/base.py */
/* goal wiring */
#define DGPPO_GOAL_SPREAD 0 /* every agent sees every goal: lidar_spread.py:86-91, mpe_spread.py:64-69 */
#define DGPPO_GOAL_TARGET 1 /* agent i sees goal i only: lidar_target.py:77-84, mpe_target.py:63-70 */

/* Obstacle record (LidarEnv rectangles), 16 floats = 64 B per obstacle:
 *   [cx, cy, width, height, theta, cos(theta), sin(theta), type, p0x, p0y, p1x, p1y, p2x, p2y, p3x, p3y]
 * = Rectangle(type, center, width, height, theta, points) of env/obstacle.py:30-56 plus a cached cos/sin. */
#define DGPPO_OBST_FIELDS 16

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
  float state_lo[5], state_hi[5]; /* state_lim() */
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

/* Library / device introspection */
int dgppo_abi_version(void);
const char* dgppo_build_info(void);

#ifdef __cplusplus
}
#endif
#endif /* DGPPO_HIP_H */
