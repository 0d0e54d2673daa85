"""ctypes binding of libreth_hip.so (the C ABI declared in include/reth_hip.h).

The library is built in-tree by ``__graft_entry__.build()`` (hipcc --offload-arch=gfx950).
There is no fallback: if the shared object is missing or cannot be loaded, every entry
point raises ``HipExtensionMissing`` -- the product never silently runs a CPU path.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RTH_LIB_PATH") or os.path.join(_HERE, "libreth_hip.so")  # override: kernel A/B runs

# element types (include/reth_hip.h)
RTH_U8, RTH_I32, RTH_I64, RTH_F32, RTH_F64 = 0, 1, 2, 3, 4
RTH_PRIO_RAW = 16  # priorities stored as given (no (w + 1e-6) ** alpha)
RTH_FRAMES = 8  # a frame-stack column's stored type: frame ids into the replay's frame store
SAMPLER_PER, SAMPLER_UNIFORM, SAMPLER_FIFO = 0, 1, 2
MAX_COLS = 8

c_i32, c_i64, c_u64, c_f32, c_f64, c_vp = (ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64,
                                          ctypes.c_float, ctypes.c_double, ctypes.c_void_p)


class HipExtensionMissing(ImportError):
    pass


class RethHipError(RuntimeError):
    pass


class ColDesc(ctypes.Structure):
    _fields_ = [("row_elems", c_i64), ("in_dtype", c_i32), ("out_dtype", c_i32), ("out_planes", c_i32),
                ("reserved", c_i32)]


class Sched(ctypes.Structure):
    """rth_schedule: Schedule (schedule.py) as method/start/end/max_steps"""
    _fields_ = [("method", c_i32), ("reserved", c_i32), ("start", c_f64), ("end", c_f64), ("max_steps", c_i64)]


SCHED_CONST, SCHED_LINEAR, SCHED_EXP = 0, 1, 2


class Src(ctypes.Structure):
    _fields_ = [("base_dev", c_vp), ("rows_dev", c_vp), ("row_stride_bytes", c_i64), ("src_dtype", c_i32),
                ("reserved", c_i32)]


class ConvShape(ctypes.Structure):
    """rth_conv_shape"""
    _fields_ = [("input", c_i32), ("cin", c_i32), ("hin", c_i32), ("win", c_i32), ("cout", c_i32), ("kh", c_i32),
                ("kw", c_i32), ("stride", c_i32)]


class WgradDeferred(ctypes.Structure):
    """rth_wgrad_deferred (include/reth_hip.h): a conv2 / conv3 weight gradient whose split
    partials rth_conv_wgrad_f32_partials wrote, finished by conv1's reduce launch"""
    _fields_ = [("partial", ctypes.c_void_p), ("gw", ctypes.c_void_p), ("splits", ctypes.c_int32),
                ("elems", ctypes.c_int32), ("nb", ctypes.c_int32), ("K", ctypes.c_int32)]


class BiasDeferred(ctypes.Structure):
    """rth_bias_deferred (include/reth_hip.h): a bias gradient whose slabs rth_relu_bias_grad
    wrote with db = NULL, finished by rth_conv_relu_wgrad_ex"""
    _fields_ = [("workspace", ctypes.c_void_p), ("db", ctypes.c_void_p), ("rows", ctypes.c_int64),
                ("C", ctypes.c_int32), ("slabs", ctypes.c_int32)]


CONV_F32_NHWC, CONV_U8_CHW = 0, 1
CONV_OUT_NCHW = 16  # flag: the conv writes NCHW (the last conv, feeding FC1)
CONV_PACK_DGRAD = 32  # rth_conv_pack_many flag: pack this forward shape's data-gradient kernel
CONV_IMPL_F32, CONV_IMPL_BF16X3, CONV_IMPL_X9 = 1, 2, 3  # rth_conv_impl: the kernel a launch runs
HEADS_FC2_ONLY = -1


class ActorTailArgs(ctypes.Structure):
    """rth_actor_tail_args"""
    _fields_ = [("q", c_vp), ("eps", c_vp), ("t_dev", c_vp), ("action", c_vp), ("qcache", c_vp),
                ("prev_s0", c_vp), ("prev_a", c_vp), ("prev_s1", c_vp), ("prev_r", c_vp), ("prev_done", c_vp),
                ("td_abs", c_vp), ("frames", c_vp), ("cur_slot", c_vp), ("r_out", c_vp), ("done_out", c_vp),
                ("s0_h", c_vp), ("s1_h", c_vp), ("seed", c_u64), ("N", c_i64), ("gamma_n", c_f32),
                ("p_reward", c_f32), ("p_done", c_f32), ("ring", c_i32), ("A", c_i32), ("ext_frames", c_i32)]

# name -> (restype, argtypes); must match include/reth_hip.h exactly
SIGNATURES = {
    "rth_last_error": (ctypes.c_char_p, []),
    "rth_version": (c_i32, []),
    "rth_build_id": (ctypes.c_char_p, []),
    "rth_graph_upload": (c_i32, [c_vp, c_vp]),
    "rth_stream_capture_deps": (c_i32, [c_vp]),
    # sum-tree
    "rth_sumtree_create": (c_i32, [c_i64, c_i32, ctypes.POINTER(c_vp)]),
    "rth_sumtree_destroy": (c_i32, [c_vp]),
    "rth_sumtree_clear": (c_i32, [c_vp, c_vp]),
    "rth_sumtree_update": (c_i32, [c_vp, c_vp, c_vp, c_i64, c_vp]),
    "rth_sumtree_find": (c_i32, [c_vp, c_vp, c_i64, c_vp, c_vp, c_vp]),
    "rth_sumtree_sample": (c_i32, [c_vp, c_i64, c_vp, c_u64, c_u64, c_vp, c_vp, c_vp]),
    "rth_sumtree_stats": (c_i32, [c_vp, c_vp, c_vp]),
    "rth_sumtree_export": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp]),
    "rth_sumtree_import": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp]),
    "rth_sumtree_capacity": (c_i64, [c_vp]),
    # PER
    "rth_per_normalize": (c_i32, [c_vp, c_i64, c_f32, c_vp, c_vp]),
    "rth_per_update": (c_i32, [c_vp, c_vp, c_vp, c_i32, c_i64, c_f64, c_vp]),
    "rth_per_sample": (c_i32, [c_vp, c_i64, c_f64, c_vp, c_u64, c_u64, c_vp, c_vp, c_vp]),
    # replay
    "rth_replay_create": (c_i32, [c_i64, c_i32, ctypes.POINTER(ColDesc), c_i32, ctypes.POINTER(Sched),
                                  ctypes.POINTER(Sched), c_i32, c_u64, ctypes.POINTER(c_vp)]),
    "rth_replay_destroy": (c_i32, [c_vp]),
    "rth_replay_append": (c_i32, [c_vp, ctypes.POINTER(Src), c_vp, c_i32, c_i64, c_vp, c_vp]),
    "rth_replay_sample": (c_i32, [c_vp, c_i64, c_vp, ctypes.POINTER(c_vp), c_vp, c_vp, c_vp]),
    "rth_replay_update_priorities": (c_i32, [c_vp, c_vp, c_vp, c_i32, c_i64, c_i32, c_vp]),
    "rth_replay_update_priorities_deferred": (c_i32, [c_vp, c_vp, c_vp, c_i32, c_i64, c_i32, c_vp]),
    "rth_replay_flush": (c_i32, [c_vp, c_vp]),
    "rth_replay_gather": (c_i32, [c_vp, c_vp, c_i64, ctypes.POINTER(c_vp), c_vp]),
    "rth_replay_info": (c_i32, [c_vp, ctypes.POINTER(c_i64), ctypes.POINTER(c_i64),
                                ctypes.POINTER(c_i64), ctypes.POINTER(c_i64), ctypes.POINTER(c_i64),
                                ctypes.POINTER(c_i64)]),
    "rth_uniform_indices": (c_i32, [c_i64, c_i64, c_vp, c_u64, c_u64, c_vp, c_vp, c_vp]),
    "rth_replay_tree": (c_vp, [c_vp]),
    "rth_replay_set_timing": (c_i32, [c_vp, ctypes.POINTER(c_vp), c_i32, ctypes.POINTER(c_i32)]),
    "rth_replay_column": (c_vp, [c_vp, c_i32]),
    "rth_replay_frames_attach": (c_i32, [c_vp, c_i64, c_i64, ctypes.POINTER(c_vp), ctypes.POINTER(c_vp)]),
    "rth_replay_push_frames": (c_i32, [c_vp, c_vp, c_i64, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_vp]),
    "rth_replay_frames_ids_out": (c_i32, [c_vp, c_i32]),
    "rth_copy_rows": (c_i32, [c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_i64, c_i64, c_i32, c_i32, c_i32, c_vp]),
    # actors
    "rth_eps_greedy": (c_i32, [c_vp, c_i64, c_i64, c_i32, c_vp, c_vp, c_vp, c_u64, c_u64, c_vp, c_vp, c_vp]),
    "rth_counter_add": (c_i32, [c_vp, c_i64, c_vp]),
    "rth_actor_prologue": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_vp, c_vp]),
    "rth_compact_flagged": (c_i32, [c_vp, c_vp, c_i64, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp]),
    "rth_actor_tail": (c_i32, [c_vp, ctypes.POINTER(ActorTailArgs), c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "rth_nstep_create": (c_i32, [c_i64, c_i32, c_f64, c_i32, c_i32, ctypes.POINTER(c_vp)]),
    "rth_nstep_destroy": (c_i32, [c_vp]),
    "rth_nstep_reset": (c_i32, [c_vp, c_vp]),
    "rth_nstep_push": (c_i32, [c_vp] + [c_vp] * 11 + [c_vp]),
    "rth_synth_env_step": (c_i32, [c_vp, c_i64, c_i32, c_i64, c_vp, c_vp, c_vp, c_u64, c_f32, c_f32,
                                   c_vp, c_vp, c_vp, c_vp, c_vp]),
    "rth_synth_env_reset": (c_i32, [c_vp, c_i64, c_i32, c_u64, c_vp, c_vp]),
    # learner
    "rth_td_huber": (c_i32, [c_vp] * 7 + [c_i64, c_i64, c_f32, c_i32, c_i32] + [c_vp] * 5 + [c_vp]),
    "rth_bias_relu": (c_i32, [c_vp, c_vp, c_i64, c_i32, c_vp]),
    "rth_relu_bias_grad_workspace": (c_i64, [c_i32]),
    "rth_heads_merge": (c_i32, [ctypes.POINTER(c_vp), c_i64, c_i64, c_i64, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp,
                                c_vp]),
    "rth_heads_split_grad": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i32, c_i32,
                                     ctypes.POINTER(c_vp), c_vp]),
    "rth_heads_backward": (c_i32, [c_vp, c_vp, c_i64, c_vp, c_i64, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                   c_vp]),
    "rth_td_heads_backward": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_f32, c_i32, c_vp,
                                      c_i64, c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "rth_heads_backward_branches": (c_i32, [c_vp, c_vp, c_i64, ctypes.POINTER(c_vp), c_i32, c_i64, c_i64, c_vp,
                                            ctypes.POINTER(c_vp), c_vp, c_vp, c_vp, c_vp]),
    "rth_td_heads_backward_branches": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_f32, c_i32,
                                               c_vp, c_i64, ctypes.POINTER(c_vp), c_i32, c_vp, c_vp, c_vp,
                                               ctypes.POINTER(c_vp), c_vp, c_vp, c_vp]),
    "rth_heads_fc2": (c_i32, [c_vp, c_i64, c_i64, c_i32, c_i32, ctypes.POINTER(c_vp), c_vp, c_vp]),
    "rth_heads_fc2_upto": (c_i32, [c_vp, c_i64, c_i64, c_vp, c_i32, c_i32, ctypes.POINTER(c_vp), c_vp, c_vp, c_vp,
                                   c_vp]),
    "rth_linear_relu_rows_upto": (c_i32, [c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_i64,
                                          c_vp]),
    "rth_conv_wgrad_x9_supported": (c_i32, [ctypes.POINTER(ConvShape)]),
    "rth_conv_wgrad_x9_workspace": (c_i64, [ctypes.POINTER(ConvShape)]),
    "rth_conv_wgrad_x9": (c_i32, [ctypes.POINTER(ConvShape), c_vp, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "rth_conv_wgrad_f32_supported": (c_i32, [ctypes.POINTER(ConvShape)]),
    "rth_conv_wgrad_f32_workspace": (c_i64, [ctypes.POINTER(ConvShape)]),
    "rth_conv_wgrad_f32": (c_i32, [ctypes.POINTER(ConvShape), c_vp, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "rth_conv_wgrad_f32_partials": (c_i32, [ctypes.POINTER(ConvShape), c_vp, c_i64, c_vp, c_vp, c_vp,
                                            ctypes.POINTER(WgradDeferred), c_vp]),
    "rth_relu_bias_grad": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_vp]),
    "rth_relu_bias_grad_nchw": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_vp]),
    "rth_conv_supported": (c_i32, [ctypes.POINTER(ConvShape)]),
    "rth_conv_packed_bytes": (c_i64, [ctypes.POINTER(ConvShape)]),
    "rth_conv_impl": (c_i32, [ctypes.POINTER(ConvShape), c_i64, c_vp]),
    "rth_conv_pack": (c_i32, [ctypes.POINTER(ConvShape), c_vp, c_vp, c_vp]),
    "rth_conv_wgrad_workspace": (c_i64, [ctypes.POINTER(ConvShape)]),
    "rth_conv_relu_wgrad": (c_i32, [ctypes.POINTER(ConvShape), c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp,
                                    c_vp]),
    "rth_conv_relu_wgrad_ex": (c_i32, [ctypes.POINTER(ConvShape), c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp,
                                       c_vp, c_i32, c_vp, c_i32, c_vp]),
    "rth_conv1_frames_relu_wgrad_ex": (c_i32, [ctypes.POINTER(ConvShape), c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp,
                                               c_vp, c_vp, c_i32, c_vp, c_i32, c_vp]),
    "rth_conv_pack_many": (c_i32, [c_i32, ctypes.POINTER(ConvShape), ctypes.POINTER(c_vp), ctypes.POINTER(c_vp),
                                   c_vp]),
    "rth_conv_bias_relu": (c_i32, [ctypes.POINTER(ConvShape), c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "rth_conv1_frames_bias_relu": (c_i32, [ctypes.POINTER(ConvShape), c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "rth_conv_bias_relu_upto": (c_i32, [ctypes.POINTER(ConvShape), c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "rth_conv_dgrad_supported": (c_i32, [ctypes.POINTER(ConvShape)]),
    "rth_conv_dgrad": (c_i32, [ctypes.POINTER(ConvShape), c_vp, c_i64, c_vp, c_vp, c_vp]),
    "rth_conv_dgrad_workspace": (c_i64, [ctypes.POINTER(ConvShape)]),
    "rth_fc_x9_supported": (c_i32, [c_i64, c_i64, c_i64]),
    "rth_fc_x9_workspace": (c_i64, [c_i64, c_i64, c_i64]),
    "rth_fc_x9": (c_i32, [c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_i32, c_vp, c_vp, c_vp]),
    "rth_fc_x9_rows_upto": (c_i32, [c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "rth_fc1_heads_supported": (c_i32, [c_i64, c_i64, c_i64, c_i32]),
    "rth_fc1_heads": (c_i32, [c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_i32, ctypes.POINTER(c_vp), c_vp, c_vp,
                              c_vp, c_vp]),
    "rth_fc_f32_supported": (c_i32, [c_i64, c_i64, c_i64]),
    "rth_fc_f32_workspace": (c_i64, [c_i64, c_i64, c_i64]),
    "rth_fc_f32": (c_i32, [c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_i32, c_vp, c_vp, c_vp]),
    "rth_conv_dgrad_ws": (c_i32, [ctypes.POINTER(ConvShape), c_vp, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "rth_conv_dgrad_prepacked": (c_i32, [ctypes.POINTER(ConvShape), c_vp, c_i64, c_vp, c_vp, c_vp]),
    "rth_conv_dgrad_relu_supported": (c_i32, [ctypes.POINTER(ConvShape)]),
    "rth_conv_dgrad_relu_prepacked": (c_i32, [ctypes.POINTER(ConvShape), c_vp, c_i64, c_vp, c_vp, c_vp, c_vp,
                                              ctypes.POINTER(c_i64), c_vp]),
    "rth_atari_create": (c_i32, [c_i32, c_i32, c_i32, c_i32, c_i32, ctypes.POINTER(c_vp)]),
    "rth_atari_destroy": (c_i32, [c_vp]),
    "rth_atari_step": (c_i32, [c_vp, c_vp, c_i64, c_vp, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "rth_atari_env_step": (c_i32, [c_vp, c_vp, c_i64, c_vp, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "rth_atari_synth_raw": (c_i32, [c_vp, c_i64, c_u64, c_vp, c_vp]),
    "rth_atari_synth_reset": (c_i32, [c_vp, c_i64, c_i64, c_u64, c_vp, c_vp, c_vp]),
    "rth_clip_adam_workspace": (c_i64, []),
    "rth_tree_update_timeouts": (c_i32, [ctypes.POINTER(c_i64)]),
    "rth_debug_conv_clock": (c_i32, [c_vp, c_i32]),
    "rth_clip_adam": (c_i32, [c_vp, c_i32, c_f64, c_f64, c_f64, c_f64, c_f64, c_vp, c_vp, c_vp, c_vp]),
    "rth_adam_prenormed": (c_i32, [c_vp, c_i32, c_f64, c_f64, c_f64, c_f64, c_f64, c_i32, c_vp, c_vp, c_vp, c_vp]),
    "rth_conv1_relu_wgrad_norm": (c_i32, [ctypes.POINTER(ConvShape), c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp,
                                          c_vp, c_vp, c_i32, c_vp, c_i32, c_vp, c_i32, c_f64, c_f64, c_f64, c_vp, c_vp,
                                          ctypes.POINTER(c_i32), c_vp]),
    # learner -> actor weights slot (perwez PUB/SUB CONFLATE)
    "rth_weights_create": (c_i32, [c_i64, c_i32, ctypes.POINTER(c_vp)]),
    "rth_weights_destroy": (c_i32, [c_vp]),
    "rth_weights_bytes": (c_i64, [c_vp]),
    "rth_weights_publish": (c_i32, [c_vp, c_i32, ctypes.POINTER(c_vp), ctypes.POINTER(c_i64), c_vp]),
    "rth_weights_fill": (c_i32, [c_vp, c_i32, ctypes.POINTER(c_vp), ctypes.POINTER(c_i64), c_vp]),
    "rth_weights_acquire": (c_i32, [c_vp, c_i32, ctypes.POINTER(c_vp), ctypes.POINTER(c_i64), c_vp, c_vp, c_vp, c_i64,
                                    c_vp, c_vp]),
    "rth_weights_version": (c_i32, [c_vp, ctypes.POINTER(c_i64)]),
    "rth_weights_version_ptr": (c_i32, [c_vp, ctypes.POINTER(c_vp)]),
    # LZ4 frames (host)
    "rth_lz4_frame_bound": (c_i32, [c_vp, c_i64, ctypes.POINTER(c_i64)]),
    "rth_lz4_frame_decompress": (c_i32, [c_vp, c_i64, c_vp, c_i64, ctypes.POINTER(c_i64)]),
    "rth_lz4_frame_compress_bound": (c_i64, [c_i64]),
    "rth_lz4_frame_compress": (c_i32, [c_vp, c_i64, c_vp, c_i64, ctypes.POINTER(c_i64)]),
    "rth_xxh32": (ctypes.c_uint32, [c_vp, c_i64, ctypes.c_uint32]),
}

_lib = None
_load_error = None

_SRC_EXT = (".hip", ".hpp", ".cpp", ".h")
# hipcc flags of the library (part of its build id).  The device code is compiled without the
# packed-FP32 VALU ops (v_pk_{add,mul,fma}_f32): on MI355X a kernel using them returned wrong
# sums -- single outputs off by one float4's worth of products, 6-60 % of launches -- whenever
# its waves shared the CUs with k_fc_x9t's bf16-MFMA waves of a concurrent launch on another
# stream, and exact results with the same source compiled without them (the victim's packed
# ops, not the other kernel's: scripts/diag_tail_concurrency.py, DESIGN.md "Packed FP32").
HIPCC_FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17", "-Wall",
               "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]


def source_files(root=None):
    """the library's sources, relative to the repo root, in path order"""
    root = root or os.path.dirname(_HERE)
    csrc = os.path.join(root, "reth_amd", "csrc")
    rel = sorted(f"reth_amd/csrc/{f}" for f in os.listdir(csrc) if f.endswith(_SRC_EXT))
    return rel + ["include/reth_hip.h"]


def source_build_id(root=None):
    """SHA-1 over "<git blob id> <path>\\n" of every library source, then the hipcc flags (the id
    compiled into the library as rth_build_id()); from git: `git ls-tree -r HEAD reth_amd/csrc
    include/reth_hip.h` lists the same blob ids"""
    import hashlib

    root = root or os.path.dirname(_HERE)
    h = hashlib.sha1()
    h.update((" ".join(HIPCC_FLAGS) + "\n").encode())
    for rel in source_files(root):
        with open(os.path.join(root, rel), "rb") as f:
            data = f.read()
        blob = hashlib.sha1(b"blob %d\0" % len(data) + data).hexdigest()
        h.update(f"{blob} {rel}\n".encode())
    return h.hexdigest()


def library_build_id(path=None):
    """the id compiled into a built library, read from its bytes (no dlopen); None if absent"""
    import re

    path = path or LIB_PATH
    try:
        with open(path, "rb") as f:
            m = re.search(rb"RTH_BUILD_ID:([0-9a-f]{40})", f.read())
    except OSError:
        return None
    return m.group(1).decode() if m else None


def _load():
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        _load_error = f"{LIB_PATH} not built (run __graft_entry__.build())"
        raise HipExtensionMissing(_load_error)
    try:
        lib = ctypes.CDLL(LIB_PATH)
    except OSError as e:  # pragma: no cover
        _load_error = str(e)
        raise HipExtensionMissing(f"cannot load {LIB_PATH}: {e}") from e
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def lib():
    """The loaded library (raises HipExtensionMissing -- never falls back)."""
    return _load()


def check(rc, what=""):
    if rc != 0:
        msg = _load().rth_last_error().decode(errors="replace")
        raise RethHipError(f"{what or 'libreth_hip'} failed ({rc}): {msg}")


def call(name, *args):
    rc = getattr(_load(), name)(*args)
    check(rc, name)
    return rc


def ptr(t):
    """Device pointer of a torch tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_ptr(stream=None):
    import torch

    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


def require_device(t, what):
    if t is not None and not t.is_cuda:
        raise ValueError(f"{what} must be a device (HIP) tensor, got {t.device}")
