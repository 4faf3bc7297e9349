"""ctypes binding of libdgppo_hip.so (include/dgppo_hip.h).

The product path has exactly one implementation — the HIP kernels in this library.  If the
library is missing or cannot be loaded, every op raises `NativeLibraryError`; there is no CPU or
PyTorch fallback.
"""
from __future__ import annotations

import ctypes
import os
import pathlib

PKG_DIR = pathlib.Path(__file__).resolve().parent
LIB_PATH = pathlib.Path(os.environ.get("DGPPO_HIP_LIB", PKG_DIR / "lib" / "libdgppo_hip.so"))

DGPPO_EINVAL = -22
DGPPO_ENGINE_LIDAR, DGPPO_ENGINE_BICYCLE, DGPPO_ENGINE_MPE, DGPPO_ENGINE_OMNI = 0, 1, 2, 3
DGPPO_ENGINE_VMAS_WHEEL, DGPPO_ENGINE_VMAS_TRANSPORT = 4, 5
DGPPO_VMAS_FIELDS = 8
DGPPO_GOAL_SPREAD, DGPPO_GOAL_TARGET = 0, 1
(DGPPO_VARIANT_NONE, DGPPO_VARIANT_LINE, DGPPO_VARIANT_FORMATION, DGPPO_VARIANT_CORRIDOR,
 DGPPO_VARIANT_CONNECT) = 0, 1, 2, 3, 4
DGPPO_OBST_FIELDS = 16

c_f32p = ctypes.c_void_p  # device pointers travel as raw addresses


class NativeLibraryError(RuntimeError):
    pass


class EnvCfg(ctypes.Structure):
    _fields_ = [
        ("engine", ctypes.c_int32),
        ("goal_mode", ctypes.c_int32),
        ("n_agents", ctypes.c_int32),
        ("n_obs", ctypes.c_int32),
        ("n_rays", ctypes.c_int32),
        ("top_k", ctypes.c_int32),
        ("state_dim", ctypes.c_int32),
        ("node_dim", ctypes.c_int32),
        ("n_nodes", ctypes.c_int32),
        ("n_edges", ctypes.c_int32),
        ("dt", ctypes.c_float),
        ("comm_radius", ctypes.c_float),
        ("car_radius", ctypes.c_float),
        ("obs_radius", ctypes.c_float),
        ("area_size", ctypes.c_float),
        ("dist2goal", ctypes.c_float),
        ("obs_len_lo", ctypes.c_float),
        ("obs_len_hi", ctypes.c_float),
        ("obs_theta_lo", ctypes.c_float),
        ("obs_theta_hi", ctypes.c_float),
        ("state_lo", ctypes.c_float * 8),
        ("state_hi", ctypes.c_float * 8),
        ("c_agent_cost", ctypes.c_float),
        ("c_obs_cost", ctypes.c_float),
        ("c_self_dist", ctypes.c_float),
        ("c_lidar_active", ctypes.c_float),
        ("c_min_dist", ctypes.c_float),
        ("c_inside_r", ctypes.c_float),
        ("c_mpe_obs_agent", ctypes.c_float),
        ("c_mpe_obs_goal", ctypes.c_float),
        ("c_mpe_obs_lo", ctypes.c_float),
        ("c_mpe_obs_hi", ctypes.c_float),
        ("t2_comm", ctypes.c_float),
        ("t2_lidar", ctypes.c_float),
        ("edge_dim", ctypes.c_int32),
        ("action_dim", ctypes.c_int32),
        ("n_cost", ctypes.c_int32),
        ("omni_max_w", ctypes.c_float),
        ("fov_angle_deg", ctypes.c_float),
        ("fov_rmax", ctypes.c_float),
        ("fov_dmin", ctypes.c_float),
        ("rot_pen", ctypes.c_float),
        ("c_cos_fov", ctypes.c_float),
        ("variant", ctypes.c_int32),
        ("n_goals", ctypes.c_int32),
        ("goals_inner", ctypes.c_int32),
        ("goal_radius", ctypes.c_float),
        ("obs_edge_radius", ctypes.c_float),
        ("connect_radius", ctypes.c_float),
        ("sample_side_y", ctypes.c_float),
        ("goal_shift_y", ctypes.c_float),
        ("line_min_dist", ctypes.c_float),
        ("c_obs_inflate", ctypes.c_float),
        ("formation_lo", ctypes.c_float),
        ("formation_hi", ctypes.c_float),
        ("c_connect_min", ctypes.c_float),
        ("line_box_x", ctypes.c_float),
        ("line_box_y", ctypes.c_float),
        ("line_off_y", ctypes.c_float),
        ("obs_x_hi", ctypes.c_float),
    ]


class EnvStepIO(ctypes.Structure):
    _fields_ = [
        ("states", c_f32p), ("states_stride", ctypes.c_int64),
        ("obstacles", c_f32p), ("obstacles_stride", ctypes.c_int64),
        ("action", c_f32p), ("action_stride", ctypes.c_int64),
        ("ray_dirs", c_f32p),
        ("nodes", c_f32p), ("nodes_stride", ctypes.c_int64),
        ("edges", c_f32p), ("edges_stride", ctypes.c_int64),
        ("out_states", c_f32p), ("out_states_stride", ctypes.c_int64),
        ("receivers", c_f32p), ("senders", c_f32p), ("edge_index_stride", ctypes.c_int64),
        ("reward", c_f32p), ("reward_stride", ctypes.c_int64),
        ("cost", c_f32p), ("cost_stride", ctypes.c_int64),
        ("n_env", ctypes.c_int32),
    ]


class EnvResetIO(ctypes.Structure):
    _fields_ = [
        ("seed", ctypes.c_uint64),
        ("seed_ptr", c_f32p),
        ("env_offset", ctypes.c_int32),
        ("obstacles", c_f32p), ("obstacles_stride", ctypes.c_int64),
        ("ray_dirs", c_f32p),
        ("nodes", c_f32p), ("nodes_stride", ctypes.c_int64),
        ("edges", c_f32p), ("edges_stride", ctypes.c_int64),
        ("out_states", c_f32p), ("out_states_stride", ctypes.c_int64),
        ("receivers", c_f32p), ("senders", c_f32p), ("edge_index_stride", ctypes.c_int64),
        ("n_env", ctypes.c_int32),
    ]


class EnvRolloutIO(ctypes.Structure):
    _fields_ = [
        ("step", EnvStepIO),
        ("T", ctypes.c_int32), ("rebuild_first", ctypes.c_int32),
        ("t_states", ctypes.c_int64), ("t_nodes", ctypes.c_int64), ("t_edges", ctypes.c_int64),
        ("t_index", ctypes.c_int64), ("t_action", ctypes.c_int64), ("t_reward", ctypes.c_int64),
        ("t_cost", ctypes.c_int64),
    ]


class GatherField(ctypes.Structure):
    _fields_ = [("src", c_f32p), ("dst", c_f32p), ("row_elems", ctypes.c_int64), ("src_tstride", ctypes.c_int64),
                ("src_estride", ctypes.c_int64)]


class GemmArgs(ctypes.Structure):
    _fields_ = [
        ("M", ctypes.c_int32), ("N", ctypes.c_int32), ("K", ctypes.c_int32), ("batch", ctypes.c_int32),
        ("trans_a", ctypes.c_int32), ("trans_b", ctypes.c_int32),
        ("A", c_f32p), ("lda", ctypes.c_int64), ("stride_a", ctypes.c_int64),
        ("B", c_f32p), ("ldb", ctypes.c_int64), ("stride_b", ctypes.c_int64),
        ("C", c_f32p), ("ldc", ctypes.c_int64), ("stride_c", ctypes.c_int64),
        ("a_grp", ctypes.c_int32), ("b_grp", ctypes.c_int32), ("c_grp", ctypes.c_int32), ("pad_", ctypes.c_int32),
        ("a_gstride", ctypes.c_int64), ("b_gstride", ctypes.c_int64), ("c_gstride", ctypes.c_int64),
        ("bias", c_f32p),
        ("addend", c_f32p), ("ld_add", ctypes.c_int64), ("stride_add", ctypes.c_int64),
        ("add_grp", ctypes.c_int32), ("pad2_", ctypes.c_int32), ("add_gstride", ctypes.c_int64),
        ("alpha", ctypes.c_float), ("beta", ctypes.c_float),
        ("relu", ctypes.c_int32),
        ("split_k", ctypes.c_int32),
        ("workspace", c_f32p),
        ("bias_grad", c_f32p),
        ("epi", ctypes.c_int32), ("pad3_", ctypes.c_int32),
        ("mask", c_f32p), ("ld_mask", ctypes.c_int64),
        ("ln_scale", c_f32p), ("ln_bias", c_f32p),
        ("ln_h", c_f32p), ("ln_mean", c_f32p), ("ln_rstd", c_f32p), ("ln_part", c_f32p),
    ]


class GruSeqArgs(ctypes.Structure):
    _fields_ = [
        ("Q", ctypes.c_int32), ("L", ctypes.c_int32), ("n_agents", ctypes.c_int32), ("H", ctypes.c_int32),
        ("gi", c_f32p), ("Wh", c_f32p), ("bhn", c_f32p), ("h0", c_f32p), ("hs", c_f32p), ("hT", c_f32p),
        ("dhs", c_f32p), ("dgi", c_f32p), ("dgh", c_f32p), ("dh0", c_f32p), ("dbhn_part", c_f32p),
    ]


class GtLayer(ctypes.Structure):
    _fields_ = [("Wq", c_f32p), ("bq", c_f32p), ("Wkt", c_f32p), ("bk", c_f32p), ("Wcat", c_f32p), ("Wu", c_f32p),
                ("bu", c_f32p), ("D", ctypes.c_int32), ("F", ctypes.c_int32), ("Wex", c_f32p)]


class PolicyStepArgs(ctypes.Structure):
    _fields_ = [
        ("G", ctypes.c_int32), ("N", ctypes.c_int32), ("E", ctypes.c_int32), ("n_agents", ctypes.c_int32),
        ("C", ctypes.c_int32), ("D0", ctypes.c_int32), ("A", ctypes.c_int32), ("n_layers", ctypes.c_int32),
        ("H", ctypes.c_int32), ("mode", ctypes.c_int32), ("ED", ctypes.c_int32), ("pad_", ctypes.c_int32),
        ("cand", c_f32p),
        ("nodes", c_f32p), ("nodes_gstride", ctypes.c_int64),
        ("edges", c_f32p), ("edges_gstride", ctypes.c_int64),
        ("receivers", c_f32p), ("senders", c_f32p), ("idx_gstride", ctypes.c_int64),
        ("layer", GtLayer * 2),
        ("head_W0", c_f32p), ("head_b0", c_f32p), ("ln0_s", c_f32p), ("ln0_b", c_f32p),
        ("head_W1", c_f32p), ("head_b1", c_f32p), ("ln1_s", c_f32p), ("ln1_b", c_f32p),
        ("gru_Wi", c_f32p), ("gru_bi", c_f32p), ("gru_Wh", c_f32p), ("gru_bhn", c_f32p),
        ("Ws", c_f32p), ("bs", c_f32p), ("Wm", c_f32p), ("bm", c_f32p), ("Wsd", c_f32p), ("bsd", c_f32p),
        ("std_shift", ctypes.c_float), ("std_min", ctypes.c_float),
        ("h_in", c_f32p), ("h_out", c_f32p), ("noise", c_f32p), ("action", c_f32p), ("log_pi", c_f32p),
        ("work", c_f32p),
        ("noise_seed", c_f32p), ("noise_stream", ctypes.c_uint64),  # ABI 10: in-kernel noise (noise NULL)
    ]


class GnnAttnArgs(ctypes.Structure):
    _fields_ = [
        ("G", ctypes.c_int32), ("N", ctypes.c_int32), ("E", ctypes.c_int32), ("n_agents", ctypes.c_int32),
        ("D", ctypes.c_int32), ("F", ctypes.c_int32), ("H", ctypes.c_int32), ("C", ctypes.c_int32),
        ("cand", c_f32p), ("receivers", c_f32p), ("senders", c_f32p),
        ("x", c_f32p), ("x_gstride", ctypes.c_int64),
        ("ef", c_f32p), ("ef_gstride", ctypes.c_int64),
        ("q", c_f32p), ("qt", c_f32p), ("bk", c_f32p),
        ("attn", c_f32p), ("xcat", c_f32p),
        ("dxcat", c_f32p), ("dqt", c_f32p), ("dq", c_f32p), ("dbeta", c_f32p),
        ("dx", c_f32p), ("dx_gstride", ctypes.c_int64),
        ("scale", ctypes.c_float), ("D0", ctypes.c_int32),
        ("xa", c_f32p), ("xa_gstride", ctypes.c_int64), ("pre_W", c_f32p), ("pre_b", c_f32p),
        ("dxa", c_f32p), ("dxa_gstride", ctypes.c_int64), ("dpre_part", c_f32p), ("sidx", c_f32p),
        ("da_add", c_f32p),
        ("beta", c_f32p), ("beta_ld", ctypes.c_int64),
        ("qt_ld", ctypes.c_int64), ("dqt_ld", ctypes.c_int64), ("dbeta_ld", ctypes.c_int64),
    ]


class GnnValueTail(ctypes.Structure):  # ABI 11 dgppo_gnn_value_tail
    _fields_ = [
        ("W0", c_f32p), ("b0", c_f32p), ("ln0_s", c_f32p), ("ln0_b", c_f32p),
        ("W1", c_f32p), ("b1", c_f32p), ("ln1_s", c_f32p), ("ln1_b", c_f32p),
        ("Wi", c_f32p), ("bi", c_f32p), ("Wh", c_f32p), ("bhn", c_f32p), ("Wo", c_f32p), ("bo", c_f32p),
        ("h_in", c_f32p), ("out", c_f32p), ("n_out", ctypes.c_int32), ("on", ctypes.c_int32),
    ]


class GnnLayerArgs(ctypes.Structure):  # ABI 11 dgppo_gnn_layer_args
    _fields_ = [
        ("a", GnnAttnArgs), ("QBW", c_f32p), ("qb", c_f32p), ("Wcat", c_f32p), ("Wu", c_f32p), ("bu", c_f32p),
        ("Y", c_f32p), ("zmean", c_f32p), ("tail", GnnValueTail),
    ]


ADAM_MAX_NETS = 4  # include/dgppo_hip.h DGPPO_ADAM_MAX_NETS


class AdamNet(ctypes.Structure):  # ABI 12 dgppo_adam_net
    _fields_ = [("param", c_f32p), ("grad", c_f32p), ("m", c_f32p), ("v", c_f32p), ("n", ctypes.c_int64),
                ("state", c_f32p), ("lr", ctypes.c_float), ("max_norm", ctypes.c_float)]


class AdamMultiArgs(ctypes.Structure):  # ABI 12 dgppo_adam_multi_args
    _fields_ = [("n_nets", ctypes.c_int32), ("eps", ctypes.c_float), ("b1", ctypes.c_double), ("b2", ctypes.c_double),
                ("workspace", c_f32p), ("net", AdamNet * ADAM_MAX_NETS)]


class TanhNormalArgs(ctypes.Structure):
    _fields_ = [
        ("rows", ctypes.c_int64),
        ("A", ctypes.c_int32), ("mode", ctypes.c_int32), ("n_agents", ctypes.c_int32), ("pad_", ctypes.c_int32),
        ("mean", c_f32p), ("std_raw", c_f32p),
        ("std_shift", ctypes.c_float), ("std_min", ctypes.c_float),
        ("noise", c_f32p), ("action", c_f32p), ("action_out", c_f32p), ("std_out", c_f32p),
        ("log_pi", c_f32p), ("entropy", c_f32p), ("entropy_eps", c_f32p),
        ("dlog_pi", c_f32p), ("dentropy", c_f32p), ("dmean", c_f32p), ("dstd_raw", c_f32p),
    ]


class GaeArgs(ctypes.Structure):
    _fields_ = [
        ("B", ctypes.c_int32), ("T", ctypes.c_int32), ("n_agents", ctypes.c_int32), ("n_h", ctypes.c_int32),
        ("hs", c_f32p), ("l", c_f32p), ("Vh", c_f32p), ("Vl", c_f32p), ("Qh", c_f32p), ("Ql", c_f32p),
        ("gamma", ctypes.c_float), ("lambda", ctypes.c_float),
    ]


class AdvArgs(ctypes.Structure):
    _fields_ = [
        ("B", ctypes.c_int32), ("T", ctypes.c_int32), ("n_agents", ctypes.c_int32), ("n_h", ctypes.c_int32),
        ("Ql", c_f32p), ("Vl", c_f32p), ("Vh", c_f32p),
        ("dt", ctypes.c_float), ("alpha", ctypes.c_float), ("cbf_eps", ctypes.c_float), ("cbf_weight", ctypes.c_float),
        ("A", c_f32p), ("safe_count", c_f32p),
    ]


_V, _I64, _I32, _F32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_float

# symbol -> (restype, argtypes); must match include/dgppo_hip.h (checked by tests/test_capi.py)
SIGNATURES = {
    "dgppo_abi_version": (ctypes.c_int, []),
    "dgppo_build_info": (ctypes.c_char_p, []),
    "dgppo_env_cfg_finalize": (ctypes.c_int, [ctypes.POINTER(EnvCfg)]),
    "dgppo_ray_table": (ctypes.c_int, [ctypes.c_int32, ctypes.c_float, ctypes.c_void_p]),
    "dgppo_env_step": (ctypes.c_int, [ctypes.POINTER(EnvCfg), ctypes.POINTER(EnvStepIO), ctypes.c_void_p]),
    "dgppo_env_set_step_kernel": (ctypes.c_int, [ctypes.c_int]),
    "dgppo_env_reset": (ctypes.c_int, [ctypes.POINTER(EnvCfg), ctypes.POINTER(EnvResetIO), ctypes.c_void_p]),
    "dgppo_env_reset_states": (ctypes.c_int, [ctypes.POINTER(EnvCfg), ctypes.POINTER(EnvResetIO), ctypes.c_void_p]),
    "dgppo_env_rollout": (ctypes.c_int, [ctypes.POINTER(EnvCfg), ctypes.POINTER(EnvRolloutIO), ctypes.c_void_p]),
    "dgppo_gemm_workspace_floats": (ctypes.c_int64, [ctypes.POINTER(GemmArgs)]),
    "dgppo_gemm_wgrad_grouped_workspace_floats": (ctypes.c_int64, [ctypes.POINTER(GemmArgs), ctypes.c_int]),
    "dgppo_gemm_wgrad_grouped": (ctypes.c_int, [ctypes.POINTER(GemmArgs), ctypes.c_int, c_f32p, ctypes.c_void_p]),
    "dgppo_gemm": (ctypes.c_int, [ctypes.POINTER(GemmArgs), ctypes.c_void_p]),
    "dgppo_gnn_attn_fwd": (ctypes.c_int, [ctypes.POINTER(GnnAttnArgs), ctypes.c_void_p]),
    "dgppo_gnn_attn_bwd": (ctypes.c_int, [ctypes.POINTER(GnnAttnArgs), ctypes.c_void_p]),
    "dgppo_relu_bwd": (ctypes.c_int, [_V, _V, _I64, _V]),
    "dgppo_lstm_cell_fwd": (ctypes.c_int, [_I64, ctypes.c_int32, _V, _V, _V, _V, _V]),
    "dgppo_lstm_cell_bwd": (ctypes.c_int, [_I64, ctypes.c_int32, _V, _V, _V, _V, _V, _V, _V, _V]),
    "dgppo_layernorm_fwd": (ctypes.c_int, [_V, _V, _V, _V, _V, _V, _I64, _I32, _I32, _F32, _V]),
    "dgppo_layernorm_bwd_workspace_floats": (ctypes.c_int64, [_I64, _I32]),
    "dgppo_layernorm_bwd": (ctypes.c_int, [_V, _V, _V, _V, _V, _V, _V, _V, _V, _I64, _I32, _I32, _V, _V]),
    "dgppo_colsum_workspace_floats": (ctypes.c_int64, [_I64, _I32]),
    "dgppo_colsum": (ctypes.c_int, [_V, _I64, _I32, _I64, _I32, _I64, _V, _F32, _F32, _V, _V]),
    "dgppo_gru_fwd": (ctypes.c_int, [_V, _V, _V, _V, _V, _I64, _I32, _V]),
    "dgppo_gru_bwd": (ctypes.c_int, [_V, _V, _V, _V, _V, _V, _V, _V, _I64, _I32, _V]),
    "dgppo_gru_seq_blocks": (ctypes.c_int64, [_I32]),
    "dgppo_gnn_attn_partial_blocks": (ctypes.c_int64, [_V]),
    "dgppo_gemm_partial_rows": (ctypes.c_int64, [ctypes.POINTER(GemmArgs)]),
    "dgppo_policy_step_supported": (ctypes.c_int, [_V]),
    "dgppo_policy_work_floats": (ctypes.c_int64, []),
    "dgppo_policy_prepare": (ctypes.c_int, [_V, _V]),
    "dgppo_policy_step": (ctypes.c_int, [_V, _V]),
    "dgppo_gnn_sender_table": (ctypes.c_int, [_I32, _I32, _I32, _I32, _V, _V, _V, _V, _V]),
    "dgppo_cost_shaped_loss": (ctypes.c_int, [_V, _V, ctypes.c_float, _V, _I32, _I32, _I32, _I32, _V]),
    "dgppo_informarl_advantages": (ctypes.c_int, [_V, _V, _V, _I32, _I32, _I32, _V]),
    "dgppo_gnn_edge_wsum": (ctypes.c_int, [_I32, _I32, _I32, _I32, _I32, _I32, _V, _V, _V, _V, _V, _V]),
    "dgppo_gnn_edge_da": (ctypes.c_int, [_I32, _I32, _I32, _I32, _I32, _I32, _V, _V, _V, _V, _V, _V]),
    "dgppo_gru_seq_fwd": (ctypes.c_int, [_V, _V]),
    "dgppo_gru_seq_bwd": (ctypes.c_int, [_V, _V]),
    "dgppo_agent_mean_fwd": (ctypes.c_int, [_V, _V, _I64, _I32, _I32, _I64, _V]),
    "dgppo_agent_mean_bwd": (ctypes.c_int, [_V, _V, _I64, _I32, _I32, _I64, _V]),
    "dgppo_agent_mean_bwd_masked": (ctypes.c_int, [_V, _V, _V, _I64, _I32, _I32, _I64, _V]),
    "dgppo_gru_set_form": (ctypes.c_int, [_I32]),
    "dgppo_gnn_set_graph_otf": (ctypes.c_int, [_I32]),
    "dgppo_tanh_normal": (ctypes.c_int, [ctypes.POINTER(TanhNormalArgs), ctypes.c_void_p]),
    "dgppo_loss_workspace_floats": (ctypes.c_int64, []),
    "dgppo_ppo_loss": (ctypes.c_int, [_V, _V, _V, _V, _I64, _F32, _F32, _V, _V, _V, _V, _V]),
    "dgppo_l2_loss": (ctypes.c_int, [_V, _V, _I64, _V, _V, _V, _V]),
    "dgppo_gae": (ctypes.c_int, [ctypes.POINTER(GaeArgs), ctypes.c_void_p]),
    "dgppo_dgppo_advantages": (ctypes.c_int, [ctypes.POINTER(AdvArgs), ctypes.c_void_p]),
    "dgppo_grad_norm": (ctypes.c_int, [_V, _I64, _V, _V, _V]),
    "dgppo_adam": (ctypes.c_int, [_V, _V, _V, _V, _I64, _V, _F32, ctypes.c_double, ctypes.c_double, _F32, _F32, _V]),
    "dgppo_adam_multi_workspace_floats": (ctypes.c_int64, []),
    "dgppo_adam_multi": (ctypes.c_int, [_V, _V]),
    "dgppo_normal": (ctypes.c_int, [_V, _I64, _V, ctypes.c_uint64, ctypes.c_uint64, _V]),
    "dgppo_clip_min0": (ctypes.c_int, [_V, _V, _I64, _V]),
    "dgppo_lagr_advantages": (ctypes.c_int, [_V, _V, _V, _V, _V, _V, _V, _I32, _I32, _I32, _I32, _V]),
    "dgppo_lagr_update": (ctypes.c_int, [_V, _V, _V, _V, _V, _V, _I64, _I32, _I32, _F32, _F32, _V]),
    "dgppo_gather_env_steps": (ctypes.c_int, [ctypes.POINTER(GatherField), _I32, _V, _I32, _I32, _V]),
    "dgppo_gnn_layer_supported": (ctypes.c_int, [ctypes.POINTER(GnnLayerArgs)]),
    "dgppo_gnn_layer_fwd": (ctypes.c_int, [ctypes.POINTER(GnnLayerArgs), ctypes.c_void_p]),
}

_LIB = None


ABI_VERSION = 14  # include/dgppo_hip.h DGPPO_ABI_VERSION


def load() -> ctypes.CDLL:
    """Load the HIP library once (torch must be imported first so one HIP runtime is shared)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    import torch  # noqa: F401  (loads torch's libamdhip64.so.7 first; ours binds to the same soname)

    if not LIB_PATH.exists():
        raise NativeLibraryError(
            f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` or `make`"
        )
    try:
        lib = ctypes.CDLL(str(LIB_PATH), mode=ctypes.RTLD_GLOBAL)
    except OSError as e:  # pragma: no cover
        raise NativeLibraryError(f"cannot load {LIB_PATH}: {e}") from e
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.dgppo_abi_version() != ABI_VERSION:  # the ctypes mirrors below describe ABI_VERSION's structs
        raise NativeLibraryError(f"{LIB_PATH} has ABI {lib.dgppo_abi_version()}, this package expects {ABI_VERSION}: "
                                 "rebuild it (make)")
    _LIB = lib
    return lib


def check(rc: int, what: str):
    if rc == DGPPO_EINVAL:
        raise ValueError(f"{what}: invalid arguments (DGPPO_EINVAL)")
    if rc != 0:
        raise RuntimeError(f"{what}: HIP error {rc}")


def ptr(t) -> int:
    return 0 if t is None else int(t.data_ptr())


def stream_handle(device=None) -> int:
    import torch

    return int(torch.cuda.current_stream(device).cuda_stream)


def require_gpu(device, what: str):
    """The kernels only run on the GPU; there is deliberately no CPU path."""
    import torch

    if torch.device(device).type != "cuda":
        raise NativeLibraryError(f"{what}: libdgppo_hip kernels need GPU tensors (got device {device})")
