"""ctypes binding of libtrafficrl.so (C ABI: include/trafficrl.h).

This is the binding the reference side would add: plain
pointers and sizes, torch tensors passed by data_ptr(), the current HIP stream
passed as a void*.  There is no CPU fallback: if the library is missing or no
HIP device is present, the env raises.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# TRX_LIB: an A/B build of the same library (tools/, never a fallback)
LIB_PATH = os.environ.get("TRX_LIB") or os.path.join(_HERE, "libtrafficrl.so")

TRX_OK, TRX_EINVAL, TRX_EHIP, TRX_EUNSUP = 0, -1, -2, -3
METHODS = {"msa": 0, "fw": 1, "cfw": 2, "gp": 3}
ABI_VERSION = 12
SP_SCIPY, SP_TORCH = 0, 1   # TRX_SP_* (include/trafficrl.h)
REWARD_MODES = {"delta": 0, "log_delta": 1, "neg_tstt": 2, "minimize_tstt": 3, "rel_improve": 4}

# Every symbol include/trafficrl.h declares (tests check the export table).
EXPORTS = (
    "trx_abi_version", "trx_last_error", "trx_graph_create", "trx_graph_destroy", "trx_graph_info",
    "trx_workspace_bytes", "trx_gp_state_bytes", "trx_assign", "trx_reset", "trx_step", "trx_observe", "trx_gat_forward",
    "trx_gat_backward", "trx_per_update", "trx_per_sample", "trx_graph_patch_memsets", "trx_gat_layer_infer",
    "trx_edge_head_infer", "trx_gat_prologue_infer", "trx_layer_tail_forward", "trx_layer_tail_workspace_floats",
    "trx_layer_tail_backward", "trx_att_dots_forward", "trx_att_dots_workspace_floats", "trx_att_dots_backward",
    "trx_small_ln_forward", "trx_small_ln_workspace_floats", "trx_small_ln_backward", "trx_edge_head_backward",
    "trx_graph_pool_forward", "trx_graph_pool_backward", "trx_bf16_round", "trx_multi_copy",
    "trx_per_update_range", "trx_per_add_range", "trx_per32_add_range", "trx_per32_update", "trx_per32_sample",
    "trx_per32_sample_weighted", "trx_damage_sample", "trx_multi_gather", "trx_episode_step", "trx_env_kernel_name",
    "trx_gat_layer_backward", "trx_gat_layer_backward_part_floats", "trx_partial_sum", "trx_partial_sum_multi",
    "trx_gat_prologue_backward",
    "trx_sac_loss", "trx_sac_adam", "trx_gat_tail_infer", "trx_edge_att_weights_backward",
    "trx_gat_layer0_infer", "trx_gat_layer0_prepare", "trx_gat_mid_infer",
    "trx_gat_layer_infer_multi", "trx_edge_head_infer_multi", "trx_edge_head_backward_multi",
    "trx_gat_prologue_infer_multi", "trx_gat_layer_backward_multi", "trx_gat_prologue_backward_multi",
)
MAX_NETS = 6   # TRX_MAX_NETS: networks per *_multi launch (ABI 11)


class TrxParams(ctypes.Structure):
    _fields_ = [
        ("method", ctypes.c_int32), ("iters", ctypes.c_int32),
        ("bpr_alpha", ctypes.c_float), ("bpr_beta", ctypes.c_float),
        ("capacity_damage", ctypes.c_float), ("_pad0", ctypes.c_float),
        ("unassigned_penalty", ctypes.c_double),
        ("reward_mode", ctypes.c_int32), ("sp_rule", ctypes.c_int32),
        ("reward_alpha", ctypes.c_double), ("reward_beta", ctypes.c_double),
        ("reward_gamma", ctypes.c_double), ("reward_clip", ctypes.c_double),
        ("gp_step", ctypes.c_double), ("gp_keep_paths", ctypes.c_int32), ("_pad2", ctypes.c_int32),
    ]


class TrxState(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in
                ("flow", "capacity", "damaged", "goal", "t", "tstt", "initial_tstt", "unassigned", "gp")]


GP_MAX_HOPS = 32  # kGpMaxHops (csrc/trx_internal.h)


def gp_layout(P: int, keep: int) -> dict:
    """Byte offsets of one env's GP path-set row (gp_layout, csrc/trx_internal.h)."""
    KP = keep + 1
    off = 0
    out = {}
    for name, nbytes in (("nkeys", 16), ("ord", P * 2), ("np", P), ("flow", P * KP * 8), ("mask", P * KP * 16),
                         ("len", P * KP), ("edges", P * KP * GP_MAX_HOPS)):
        out[name] = off
        off = (off + nbytes + 15) & ~15
    out["total"] = (off + 255) & ~255
    return out


_vp = ctypes.c_void_p
_lib = None

_i32, _f32 = ctypes.c_int32, ctypes.c_float


class TrxGatLayerArgs(ctypes.Structure):
    """trx_gat_layer_args (include/trafficrl.h)."""
    _fields_ = [
        ("num_graphs", _i32), ("nodes_per_graph", _i32), ("heads", _i32), ("channels", _i32), ("concat", _i32),
        ("max_graph_edges", _i32), ("in_dim", _i32),
        ("xh", _vp), ("x0", _vp), ("w0", _vp), ("rowptr", _vp), ("col", _vp),
        ("a_edge", _vp), ("a_edge_stride", _i32), ("a_edge_offset", _i32),
        ("att_src", _vp), ("att_dst", _vp), ("bias", _vp), ("negative_slope", _f32),
        ("ln_weight", _vp), ("ln_bias", _vp), ("ln_eps", _f32),
        ("residual", _i32), ("res", _vp), ("wp", _vp), ("bp", _vp),
        ("activation", _i32),
        ("out_f32", _vp), ("out_bf16", _vp), ("pool", _vp),
        ("save_alpha", _vp), ("save_asd", _vp), ("save_v", _vp), ("save_stats", _vp), ("exact", _i32),
    ]


class TrxGatLayer0Args(ctypes.Structure):
    """trx_gat_layer0_args (include/trafficrl.h)."""
    _fields_ = [
        ("num_graphs", _i32), ("nodes_per_graph", _i32), ("heads", _i32), ("channels", _i32),
        ("max_graph_edges", _i32), ("x0", _vp), ("w0", _vp), ("rowptr", _vp), ("col", _vp),
        ("a_edge", _vp), ("a_edge_stride", _i32), ("a_edge_offset", _i32), ("bias", _vp), ("negative_slope", _f32),
        ("ln_weight", _vp), ("ln_bias", _vp), ("ln_eps", _f32), ("wp", _vp), ("bp", _vp), ("u", _vp),
        ("stats", _vp), ("out_f32", _vp), ("out_bf16", _vp), ("desc", _vp),
    ]


class TrxGatMidArgs(ctypes.Structure):
    """trx_gat_mid_args (include/trafficrl.h)."""
    _fields_ = [
        ("num_graphs", _i32), ("nodes_per_graph", _i32), ("heads", _i32), ("channels", _i32),
        ("max_graph_edges", _i32), ("xh", _vp), ("rowptr", _vp), ("col", _vp),
        ("a_edge", _vp), ("a_edge_stride", _i32), ("a_edge_offset", _i32), ("att_src", _vp), ("att_dst", _vp),
        ("bias", _vp), ("negative_slope", _f32), ("ln_weight", _vp), ("ln_bias", _vp), ("ln_eps", _f32),
        ("desc", _vp), ("l0_heads", _i32), ("l0_w0", _vp), ("l0_bias", _vp), ("l0_ln_weight", _vp),
        ("l0_ln_bias", _vp), ("l0_wp", _vp), ("l0_bp", _vp), ("out_f32", _vp), ("out_bf16", _vp),
    ]


class TrxEdgeHeadArgs(ctypes.Structure):
    """trx_edge_head_args (include/trafficrl.h)."""
    _fields_ = [
        ("num_graphs", _i32), ("edges_per_graph", _i32), ("hidden", _i32), ("edge_dim", _i32),
        ("src", _vp), ("dst", _vp), ("p", _vp), ("c", _vp), ("ea", _vp), ("we", _vp), ("w2", _vp),
        ("b2", _vp), ("mask", _vp), ("softmax", _i32), ("out", _vp), ("logits", _vp),
        ("nodes_per_graph", _i32), ("u", _vp), ("action", _vp), ("exact", _i32),
    ]


class TrxGatTailArgs(ctypes.Structure):
    """trx_gat_tail_args (include/trafficrl.h)."""
    _fields_ = [
        ("num_graphs", _i32), ("nodes_per_graph", _i32), ("edges_per_graph", _i32), ("in_dim", _i32),
        ("channels", _i32), ("hidden", _i32), ("edge_dim", _i32), ("max_graph_edges", _i32),
        ("x", _vp), ("w_lin", _vp), ("rowptr", _vp), ("col", _vp), ("a_edge", _vp),
        ("a_edge_stride", _i32), ("a_edge_offset", _i32), ("att_src", _vp), ("att_dst", _vp), ("bias", _vp),
        ("negative_slope", _f32), ("ln_weight", _vp), ("ln_bias", _vp), ("ln_eps", _f32),
        ("w_nodes", _vp), ("w_ctx", _vp), ("b1", _vp), ("src", _vp), ("dst", _vp), ("ea", _vp), ("we", _vp),
        ("w2", _vp), ("b2", _vp), ("mask", _vp), ("softmax", _i32), ("out", _vp), ("logits", _vp), ("u", _vp),
        ("action", _vp), ("emb_bf16", _vp), ("pool", _vp),
    ]


MAX_GAT_LAYERS = 4


class TrxGatPrologueArgs(ctypes.Structure):
    """trx_gat_prologue_args (include/trafficrl.h)."""
    _fields_ = [
        ("num_graphs", _i32), ("nodes_per_graph", _i32), ("edges_per_graph", _i32), ("node_dim", _i32),
        ("edge_dim", _i32), ("node_x", _vp), ("edge_x", _vp),
        ("node_ln_w", _vp), ("node_ln_b", _vp), ("node_ln_eps", _f32),
        ("edge_ln_w", _vp), ("edge_ln_b", _vp), ("edge_ln_eps", _f32),
        ("src", _vp), ("dst", _vp), ("rowptr", _vp), ("pos_src", _vp),
        ("num_layers", _i32), ("heads", _i32 * MAX_GAT_LAYERS), ("channels", _i32 * MAX_GAT_LAYERS),
        ("lin_edge_w", _vp * MAX_GAT_LAYERS), ("att_edge", _vp * MAX_GAT_LAYERS),
        ("m_work", _vp), ("x0", _vp), ("ea", _vp), ("a_edge", _vp), ("exact", _i32),
    ]


class TrxGatLayerBwdArgs(ctypes.Structure):
    """trx_gat_layer_bwd_args (include/trafficrl.h)."""
    _fields_ = [
        ("num_graphs", _i32), ("nodes_per_graph", _i32), ("heads", _i32), ("channels", _i32),
        ("max_graph_edges", _i32), ("in_dim", _i32),
        ("rowptr", _vp), ("col", _vp), ("sptr", _vp), ("spos", _vp), ("xh", _vp), ("x0", _vp), ("w0", _vp),
        ("a_edge", _vp), ("a_edge_stride", _i32), ("a_edge_offset", _i32),
        ("att_src", _vp), ("att_dst", _vp), ("ln_weight", _vp), ("negative_slope", _f32),
        ("activation", _i32), ("residual", _i32), ("wp", _vp),
        ("alpha", _vp), ("asd", _vp), ("v", _vp), ("stats", _vp), ("y", _vp),
        ("gy", _vp), ("gy_bf16", _vp), ("g_pool", _vp),
        ("g_xh", _vp), ("g_res", _vp), ("g_x0", _vp), ("g_a_edge", _vp), ("part", _vp), ("exact", _i32),
    ]


class TrxGatPrologueBwdArgs(ctypes.Structure):
    """trx_gat_prologue_bwd_args (include/trafficrl.h)."""
    _fields_ = [
        ("num_graphs", _i32), ("nodes_per_graph", _i32), ("edges_per_graph", _i32), ("node_dim", _i32),
        ("edge_dim", _i32), ("A", _i32), ("node_x", _vp), ("edge_x", _vp),
        ("node_ln_w", _vp), ("node_ln_b", _vp), ("node_ln_eps", _f32),
        ("edge_ln_w", _vp), ("edge_ln_b", _vp), ("edge_ln_eps", _f32),
        ("src", _vp), ("dst", _vp), ("rowptr", _vp), ("pos_src", _vp),
        ("m_work", _vp), ("g_a_edge", _vp), ("g_x0", _vp), ("g_ea_head", _vp), ("part", _vp), ("exact", _i32),
    ]


class TrxSacLossArgs(ctypes.Structure):
    """trx_sac_loss_args (include/trafficrl.h)."""
    _fields_ = [
        ("num_graphs", _i32), ("edges_per_graph", _i32),
        ("next_probs", _vp), ("qt1", _vp), ("qt2", _vp), ("reward", _vp), ("done", _vp), ("q1", _vp), ("q2", _vp),
        ("logits", _vp), ("mask", _vp), ("action", _vp), ("weights", _vp), ("log_alpha", _vp),
        ("gamma", _f32), ("target_entropy", _f32), ("target_entropy_ratio", _f32), ("target_entropy_given", _i32),
        ("g_q1", _vp), ("g_q2", _vp), ("g_logits", _vp), ("td_error", _vp), ("part", _vp), ("out", _vp),
        ("g_log_alpha", _vp),
    ]


class TrxAdamSeg(ctypes.Structure):
    """trx_adam_seg (include/trafficrl.h): 48 bytes."""
    _fields_ = [("p", _vp), ("t", _vp), ("goff", ctypes.c_int64), ("moff", ctypes.c_int64), ("n", ctypes.c_int64),
                ("group", _i32), ("_pad", _i32)]


class TrxAdamArgs(ctypes.Structure):
    """trx_adam_args (include/trafficrl.h)."""
    _fields_ = [
        ("segs", _vp), ("blocks", _vp), ("nseg", _i32), ("nblocks", _i32), ("g_base", _vp), ("m", _vp), ("v", _vp),
        ("partial", _vp), ("step", _vp), ("scal", _vp), ("lr", _f32 * 3), ("max_norm", _f32 * 3),
        ("beta1", _f32), ("beta2", _f32), ("eps", _f32), ("tau", _f32), ("log_alpha_min", _f32),
        ("log_alpha_max", _f32),
    ]


MAX_ROUND = 48


class TrxRoundList(ctypes.Structure):
    """trx_round_list (include/trafficrl.h)."""
    _fields_ = [
        ("count", _i32), ("out_bf16", _i32 * MAX_ROUND), ("rows", ctypes.c_int64 * MAX_ROUND),
        ("cols", ctypes.c_int64 * MAX_ROUND), ("src_stride", ctypes.c_int64 * MAX_ROUND),
        ("src", _vp * MAX_ROUND), ("dst", _vp * MAX_ROUND), ("dst_stride", ctypes.c_int64 * MAX_ROUND),
    ]


class TrxEdgeHeadBwdIO(ctypes.Structure):   # trx_edge_head_bwd_io (ABI 11)
    _fields_ = [(n, _vp) for n in ("grad_logits", "grad_p", "grad_c", "grad_z", "grad_w2_part", "grad_we_part",
                                   "grad_ea")]


MAX_PSUM = 32


class TrxPsumList(ctypes.Structure):
    """trx_psum_list (include/trafficrl.h)."""
    _fields_ = [
        ("count", _i32), ("rows", _i32), ("width", _i32 * MAX_PSUM), ("out_cols", _i32 * MAX_PSUM),
        ("stride", ctypes.c_int64 * MAX_PSUM), ("out_ld", ctypes.c_int64 * MAX_PSUM),
        ("part", _vp * MAX_PSUM), ("out", _vp * MAX_PSUM),
    ]


MAX_COPY = 16


class TrxCopyList(ctypes.Structure):
    """trx_copy_list (include/trafficrl.h)."""
    _fields_ = [("count", _i32), ("_pad", _i32), ("bytes", ctypes.c_int64 * MAX_COPY), ("src", _vp * MAX_COPY),
                ("dst", _vp * MAX_COPY)]


def multi_copy(pairs, device):
    """One trx_multi_copy launch for [(dst, src), ...] (contiguous, same dtype and size)."""
    L = load()
    lst = TrxCopyList()
    lst.count = len(pairs)
    for k, (dst, src) in enumerate(pairs):
        assert dst.is_contiguous() and src.is_contiguous() and dst.dtype == src.dtype and dst.numel() == src.numel()
        lst.bytes[k] = dst.numel() * dst.element_size()
        lst.src[k], lst.dst[k] = src.data_ptr(), dst.data_ptr()
    check(L.trx_multi_copy(lst, stream_ptr(device)), "trx_multi_copy")


def multi_gather(pairs, idx, device):
    """One trx_multi_gather launch: dst[r] = src[idx[r]] along dim 0 for
    [(dst, src), ...] (contiguous, same dtype and row shape; idx int64 on the
    device, values < every src's row count -- not checked on the device)."""
    L = load()
    lst = TrxCopyList()
    lst.count = len(pairs)
    n = idx.numel()
    for k, (dst, src) in enumerate(pairs):
        assert dst.is_contiguous() and src.is_contiguous() and dst.dtype == src.dtype and dst.shape[0] == n
        assert dst.shape[1:] == src.shape[1:]
        lst.bytes[k] = (dst.numel() // max(1, n)) * dst.element_size()
        lst.src[k], lst.dst[k] = src.data_ptr(), dst.data_ptr()
    check(L.trx_multi_gather(lst, ptr(idx), n, stream_ptr(device)), "trx_multi_gather")


class TrafficRLError(RuntimeError):
    pass


def load():
    """Load libtrafficrl.so (importing torch first so both share one HIP runtime)."""
    global _lib
    if _lib is not None:
        return _lib
    import torch  # noqa: F401  -- torch's libamdhip64.so.7 must be the one resolved
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is not built. Build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
    L = ctypes.CDLL(LIB_PATH)
    L.trx_abi_version.restype = ctypes.c_int32
    L.trx_last_error.restype = ctypes.c_char_p
    L.trx_gat_layer_backward.argtypes = [ctypes.POINTER(TrxGatLayerBwdArgs), _vp]
    L.trx_gat_layer_backward_part_floats.argtypes = [_i32, _i32, _i32]
    L.trx_gat_layer_backward_part_floats.restype = ctypes.c_int64
    L.trx_partial_sum.argtypes = [_vp, _i32, _i32, ctypes.c_int64, _vp, _vp]
    L.trx_partial_sum_multi.argtypes = [ctypes.POINTER(TrxPsumList), _vp]
    L.trx_gat_prologue_backward.argtypes = [ctypes.POINTER(TrxGatPrologueBwdArgs), _vp]
    L.trx_sac_loss.argtypes = [ctypes.POINTER(TrxSacLossArgs), _vp]
    L.trx_sac_adam.argtypes = [ctypes.POINTER(TrxAdamArgs), _vp]
    L.trx_env_kernel_name.argtypes = [_vp, ctypes.POINTER(TrxParams)]
    L.trx_env_kernel_name.restype = ctypes.c_char_p
    L.trx_graph_create.argtypes = [ctypes.c_int32, ctypes.c_int32, _vp, _vp, _vp, _vp, ctypes.c_int32, _vp, _vp, _vp,
                                   ctypes.POINTER(_vp)]
    L.trx_graph_destroy.argtypes = [_vp]
    L.trx_graph_info.argtypes = [_vp, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32),
                                 ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_double)]
    L.trx_workspace_bytes.argtypes = [_vp, ctypes.c_int32]
    L.trx_workspace_bytes.restype = ctypes.c_int64
    L.trx_gp_state_bytes.argtypes = [_vp, ctypes.c_int32, ctypes.c_int32]
    L.trx_gp_state_bytes.restype = ctypes.c_int64
    L.trx_assign.argtypes = [_vp, ctypes.POINTER(TrxParams), ctypes.c_int32, ctypes.POINTER(TrxState), _vp, _vp, _vp]
    L.trx_reset.argtypes = [_vp, ctypes.POINTER(TrxParams), ctypes.c_int32, ctypes.POINTER(TrxState), _vp, _vp, _vp]
    L.trx_step.argtypes = [_vp, ctypes.POINTER(TrxParams), ctypes.c_int32, ctypes.POINTER(TrxState), _vp, _vp, _vp,
                           _vp, _vp, _vp]
    L.trx_observe.argtypes = [_vp, ctypes.c_int32, ctypes.POINTER(TrxState), _vp, _vp, _vp, _vp, _vp]
    L.trx_gat_forward.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _vp, _vp, _vp, ctypes.c_int32,
                                  _vp, _vp, _vp, ctypes.c_float, _vp, _vp, _vp, _vp]
    L.trx_gat_backward.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _vp, _vp, _vp, _vp, _vp, _vp,
                                   ctypes.c_int32, _vp, _vp, _vp, ctypes.c_float, _vp, _vp, _vp, _vp, _vp, _vp, _vp]
    L.trx_per_update.argtypes = [_vp, ctypes.c_int64, _vp, _vp, ctypes.c_int32, _vp]
    L.trx_per_sample.argtypes = [_vp, ctypes.c_int64, _vp, ctypes.c_int32, _vp, _vp, _vp]
    L.trx_graph_patch_memsets.argtypes = [_vp, ctypes.POINTER(ctypes.c_int32)]
    L.trx_gat_layer_infer.argtypes = [ctypes.POINTER(TrxGatLayerArgs), _vp]
    L.trx_edge_head_infer.argtypes = [ctypes.POINTER(TrxEdgeHeadArgs), _vp]
    L.trx_gat_layer0_infer.argtypes = [ctypes.POINTER(TrxGatLayer0Args), _vp]
    L.trx_gat_layer0_prepare.argtypes = [_i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp]
    L.trx_gat_mid_infer.argtypes = [ctypes.POINTER(TrxGatMidArgs), _vp]
    L.trx_gat_tail_infer.argtypes = [ctypes.POINTER(TrxGatTailArgs), _vp]
    L.trx_edge_att_weights_backward.argtypes = [ctypes.POINTER(TrxGatPrologueArgs), _vp, _i32, _vp, _vp]
    L.trx_gat_prologue_infer.argtypes = [ctypes.POINTER(TrxGatPrologueArgs), _vp]
    L.trx_edge_head_backward.argtypes = [ctypes.POINTER(TrxEdgeHeadArgs), _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]
    for name, st in (("trx_gat_layer_infer_multi", TrxGatLayerArgs), ("trx_edge_head_infer_multi", TrxEdgeHeadArgs),
                     ("trx_gat_prologue_infer_multi", TrxGatPrologueArgs),
                     ("trx_gat_layer_backward_multi", TrxGatLayerBwdArgs),
                     ("trx_gat_prologue_backward_multi", TrxGatPrologueBwdArgs)):
        getattr(L, name).argtypes = [ctypes.POINTER(st), _i32, _vp]
    L.trx_edge_head_backward_multi.argtypes = [ctypes.POINTER(TrxEdgeHeadArgs), ctypes.POINTER(TrxEdgeHeadBwdIO),
                                               _i32, _vp]
    L.trx_graph_pool_forward.argtypes = [_i32, _i32, _i32, _vp, _vp, _vp, _vp]
    L.trx_bf16_round.argtypes = [ctypes.POINTER(TrxRoundList), _vp]
    L.trx_multi_copy.argtypes = [ctypes.POINTER(TrxCopyList), _vp]
    L.trx_per_update_range.argtypes = [_vp, ctypes.c_int64, ctypes.c_int64, _vp, _i32, _vp]
    L.trx_per_add_range.argtypes = [_vp, ctypes.c_int64, ctypes.c_int64, _i32, _vp, ctypes.c_double, ctypes.c_double,
                                    _vp]
    L.trx_per32_add_range.argtypes = [_vp, ctypes.c_int64, ctypes.c_int64, _i32, _vp, ctypes.c_double,
                                      ctypes.c_double, _vp]
    L.trx_per32_update.argtypes = [_vp, ctypes.c_int64, _vp, _vp, _i32, _vp, ctypes.c_double, ctypes.c_double, _vp]
    L.trx_per32_sample.argtypes = [_vp, ctypes.c_int64, _vp, _i32, _vp, _vp, _vp]
    L.trx_per32_sample_weighted.argtypes = [_vp, ctypes.c_int64, _vp, _i32, _vp, ctypes.c_double, _vp, _vp, _vp, _vp]
    L.trx_episode_step.argtypes = [_i32, _vp, _vp, _vp, ctypes.c_double, ctypes.c_int64] + [_vp] * 9 + [_vp]
    L.trx_multi_gather.argtypes = [ctypes.POINTER(TrxCopyList), _vp, _i32, _vp]
    L.trx_damage_sample.argtypes = [_i32, _i32, _vp, _vp, _i32, _i32, _i32, _vp, _vp, _i32]
    L.trx_graph_pool_backward.argtypes = [_i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp]
    L.trx_layer_tail_forward.argtypes = [_i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _f32, _vp, _vp, _vp, _vp]
    L.trx_att_dots_forward.argtypes = [_i32, _i32, _i32, _vp, _i32, _vp, _vp, _vp, _vp, _vp]
    L.trx_att_dots_workspace_floats.argtypes = [_i32, _i32, _i32]
    L.trx_att_dots_workspace_floats.restype = ctypes.c_int64
    L.trx_att_dots_backward.argtypes = [_i32, _i32, _i32, _vp, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]
    L.trx_small_ln_forward.argtypes = [_i32, _i32, _vp, _vp, _vp, _f32, _vp, _vp, _vp]
    L.trx_small_ln_workspace_floats.argtypes = [_i32, _i32]
    L.trx_small_ln_workspace_floats.restype = ctypes.c_int64
    L.trx_small_ln_backward.argtypes = [_i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]
    L.trx_layer_tail_workspace_floats.argtypes = [_i32, _i32]
    L.trx_layer_tail_workspace_floats.restype = ctypes.c_int64
    L.trx_layer_tail_backward.argtypes = [_i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                          _vp]
    for name in ("trx_graph_create", "trx_graph_destroy", "trx_graph_info", "trx_assign", "trx_reset", "trx_step",
                 "trx_observe", "trx_gat_forward", "trx_gat_backward", "trx_per_update", "trx_per_sample",
                 "trx_graph_patch_memsets", "trx_gat_layer_infer", "trx_edge_head_infer", "trx_gat_prologue_infer",
                 "trx_layer_tail_forward", "trx_layer_tail_backward", "trx_att_dots_forward",
                 "trx_att_dots_backward", "trx_small_ln_forward", "trx_small_ln_backward",
                 "trx_edge_head_backward", "trx_graph_pool_forward", "trx_graph_pool_backward",
                 "trx_bf16_round", "trx_multi_copy",
                 "trx_per_update_range", "trx_per_add_range", "trx_per32_add_range", "trx_per32_update",
                 "trx_per32_sample", "trx_per32_sample_weighted", "trx_damage_sample", "trx_multi_gather",
                 "trx_episode_step", "trx_gat_layer_backward", "trx_partial_sum", "trx_gat_prologue_backward",
                 "trx_sac_loss", "trx_sac_adam", "trx_gat_tail_infer", "trx_edge_att_weights_backward",
                 "trx_gat_layer0_infer", "trx_gat_layer0_prepare", "trx_gat_mid_infer", "trx_partial_sum_multi"):
        getattr(L, name).restype = ctypes.c_int
    if L.trx_abi_version() != ABI_VERSION:
        raise ImportError(f"libtrafficrl ABI {L.trx_abi_version()} != {ABI_VERSION}")
    _lib = L
    return L


def check(rc: int, what: str):
    """Map C return codes to the reference's exception types."""
    if rc == TRX_OK:
        return
    msg = load().trx_last_error().decode(errors="replace")
    if rc == TRX_EINVAL:
        raise ValueError(f"{what}: {msg}")
    raise TrafficRLError(f"{what} failed ({rc}): {msg}")


def multi(struct_type, items):
    """A ctypes array of argument blocks for a *_multi entry point."""
    return (struct_type * len(items))(*items)


def ptr(t) -> ctypes.c_void_p:
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def stream_ptr(device=None) -> ctypes.c_void_p:
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def patch_graph_memsets(graph) -> int:
    """Rewrite the memset nodes of a torch.cuda.CUDAGraph captured with
    keep_graph=True (before instantiate) into fill kernels; returns how many
    were rewritten.  See trx_graph_patch_memsets in include/trafficrl.h."""
    L = load()
    n = ctypes.c_int32(0)
    check(L.trx_graph_patch_memsets(ctypes.c_void_p(graph.raw_cuda_graph()), ctypes.byref(n)),
          "trx_graph_patch_memsets")
    return int(n.value)
