"""ctypes bindings for the in-tree native libraries.

``libstereo_amd.so`` (HIP kernels + engine) is loaded after ``torch`` so that it binds to the HIP
runtime torch already mapped (same SONAME, one runtime per process).  On a machine with a GPU a
missing library is a hard error — there is no silent eager fallback for any op.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

LIBDIR = Path(__file__).resolve().parent / "lib"

_dev = None
_host = None


class NativeMissing(RuntimeError):
    pass


def _load(name: str):
    path = LIBDIR / name
    if not path.exists():
        raise NativeMissing(
            f"{path} not built — run `python -m stereoalgorithms_amd._build` (or __graft_entry__.build())")
    return C.CDLL(str(path), mode=C.RTLD_GLOBAL)


def dev():
    """libstereo_amd.so (requires torch imported first so the HIP runtime is shared)."""
    global _dev
    if _dev is None:
        import torch  # noqa: F401  (bind to torch's HIP runtime)
        # SA_NATIVE_LIB: an alternative build of the device library (kernel A/B experiments, e.g.
        # tools/exp_build.sh variants); it must export the same C API
        alt = os.environ.get("SA_NATIVE_LIB")
        _dev = C.CDLL(alt, mode=C.RTLD_GLOBAL) if alt else _load("libstereo_amd.so")
        _declare_dev(_dev)
    return _dev


def host():
    """libstereo_host.so (CPU only)."""
    global _host
    if _host is None:
        _host = _load("libstereo_host.so")
        _declare_host(_host)
    return _host


def available() -> bool:
    return (LIBDIR / "libstereo_amd.so").exists()


# ----------------------------------------------------------------------------- structs
class SaConvSrc(C.Structure):
    _fields_ = [("ptr", C.c_void_p), ("channels", C.c_int32), ("stride", C.c_int32)]


class SaConvArgs(C.Structure):
    _fields_ = [
        ("src", SaConvSrc * 4), ("nsrc", C.c_int32),
        ("N", C.c_int32), ("H", C.c_int32), ("W", C.c_int32), ("Cin", C.c_int32),
        ("KH", C.c_int32), ("KW", C.c_int32), ("sh", C.c_int32), ("sw", C.c_int32),
        ("ph", C.c_int32), ("pw", C.c_int32), ("dh", C.c_int32), ("dw", C.c_int32),
        ("Ho", C.c_int32), ("Wo", C.c_int32),
        ("weight", C.c_void_p), ("bias", C.c_void_p),
        ("Cout", C.c_int32), ("Kpad", C.c_int32),
        ("out", C.c_void_p), ("out_stride", C.c_int32),
        ("epi", C.c_int32), ("act", C.c_int32), ("act2", C.c_int32),
        ("alpha", C.c_float), ("scale", C.c_float),
        ("res", C.c_void_p), ("res_stride", C.c_int32),
        ("ctx", C.c_void_p), ("ctx_stride", C.c_int32),
        ("aux", C.c_void_p), ("aux_stride", C.c_int32),
        ("hbuf", C.c_void_p), ("h_stride", C.c_int32),
        ("rh", C.c_void_p), ("rh_stride", C.c_int32),
        ("stats", C.c_void_p),
        ("tile_cfg", C.c_int32), ("splitk", C.c_int32),
        ("ws", C.c_void_p), ("counters", C.c_void_p), ("ws_floats", C.c_int64),
        ("n_counters", C.c_int32),
        ("KD", C.c_int32), ("Di", C.c_int32), ("Do", C.c_int32), ("sd", C.c_int32), ("pd", C.c_int32),
        ("up", C.c_int32), ("cout_real", C.c_int32), ("gate", C.c_void_p), ("gate_stride", C.c_int32),
        ("stats_slots", C.c_int32), ("cin_real", C.c_int32),
        ("tapw", C.c_void_p), ("taps", C.c_int32),
        ("in_stats", C.c_void_p), ("in_slots", C.c_int32), ("in_eps", C.c_float),
    ]


class SaNormArgs(C.Structure):
    _fields_ = [
        ("x", C.c_void_p), ("x_stride", C.c_int32),
        ("stats", C.c_void_p),
        ("res", C.c_void_p), ("res_stride", C.c_int32),
        ("res_stats", C.c_void_p),
        ("out", C.c_void_p), ("out_stride", C.c_int32),
        ("N", C.c_int32), ("HW", C.c_int32), ("C", C.c_int32),
        ("act", C.c_int32), ("act2", C.c_int32),
        ("eps", C.c_float), ("alpha", C.c_float),
        ("stat_slots", C.c_int32), ("res_act", C.c_int32),
    ]


class SaAgclArgs(C.Structure):
    _fields_ = [
        ("f1", C.c_void_p), ("f1_stride", C.c_int32), ("f2", C.c_void_p), ("f2_stride", C.c_int32),
        ("flow", C.c_void_p), ("offset", C.c_void_p), ("offset_stride", C.c_int32),
        ("N", C.c_int32), ("H", C.c_int32), ("W", C.c_int32), ("C", C.c_int32),
        ("small_patch", C.c_int32), ("iter_mode", C.c_int32),
        ("out", C.c_void_p), ("out_stride", C.c_int32), ("out_channels", C.c_int32),
    ]


class SaCreHeadArgs(C.Structure):
    _fields_ = [
        ("w16", C.c_void_p), ("bias", C.c_void_p), ("cor", C.c_void_p), ("cor_stride", C.c_int32),
        ("wf16", C.c_void_p), ("fbias", C.c_void_p), ("flo", C.c_void_p), ("flo_stride", C.c_int32),
        ("fcopy", C.c_void_p), ("fcopy_stride", C.c_int32),
    ]


class SaEwArgs(C.Structure):
    _fields_ = [
        ("x", C.c_void_p), ("x_stride", C.c_int32), ("add", C.c_void_p), ("add_stride", C.c_int32),
        ("bcast", C.c_void_p), ("bcast_period", C.c_int64), ("out", C.c_void_p), ("out_stride", C.c_int32),
        ("P", C.c_int64), ("C", C.c_int32), ("act", C.c_int32), ("scale", C.c_float),
    ]


ACT = {"none": 0, "relu": 1, "leaky": 2, "tanh": 3, "sigmoid": 4, "relu6": 5}
EPI = {"store": 0, "gru_zr": 1, "gru_q": 2, "flow_acc": 3, "store_f32": 4, "gru_zrq": 6, "tapproj": 7}
PRE = {"raw": 0, "unit": 1, "imagenet": 2, "signed": 3}

_i = C.c_int
_p = C.c_void_p
_f = C.c_float


def _declare_dev(lib):
    sig = {
        "sa_conv2d": (_i, [C.POINTER(SaConvArgs), _p]),
        "sa_gru_level": (_i, [C.POINTER(SaConvArgs), C.POINTER(SaConvArgs), _p, _i, _p]),
        "sa_flow_head_tail": (_i, [_p, _i, _i, _p, _p, _p, _i, _i, _i, _p]),
        "sa_flow_head_tail_oc": (_i, [_p, _i, _i, _p, _i, _p, _p, _i, _i, _i, _p]),
        "sa_instnorm_apply": (_i, [C.POINTER(SaNormArgs), _p]),
        "sa_stats_reduce": (_i, [_p, _i, C.c_long, _p]),
        "sa_avgpool3s2": (_i, [_p, _i, _p, _i, _i, _i, _i, _i, _p]),
        "sa_avgpool_k": (_i, [_p, _i, _p, _i, _i, _i, _i, _i, _i, _p]),
        "sa_interp_bilinear": (_i, [_p, _i, _p, _i, _i, _i, _i, _i, _i, _i, _i, _f, _p]),
        "sa_corr1d_pyramid": (_i, [_p, _p, _i, _i, _i, _i, _i, _i, _i, _p, _p]),
        "sa_corr1d_lookup": (_i, [_p, _p, _i, _i, _i, _i, _i, _i, _p, _i, _i, _p, _i, _i, _p, _i, _p]),
        "sa_raft_motion_head": (_i, [_p, _p, _i, _i, _i, _i, _i, _i, _p, _p, _p, _p, _p, _i, _p, _i, _p, _i, _p]),
        "sa_raft_motion_encoder": (_i, [_p, _p, _i, _i, _i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i, _p]),
        "sa_raft_motion_encoder_stamps": (None, [_p]),
        "sa_raft_motion_encoder_variant": (None, [_i]),
        "sa_convex_upsample": (_i, [_p, _i, _p, _i, _i, _i, _i, _f, _p, _p]),
        "sa_preprocess": (_i, [_p, _i, _i, _i, _i, _p, _i, _i, _i, _p]),
        "sa_remap_bgr": (_i, [_p, _i, _i, _i, _p, _i, _i, _i, _p, _p]),
        "sa_reproject": (_i, [_p, _i, _f, _p, _i, _i, _i, _p, _p, _p, _p]),
        "sa_agcl_corr": (_i, [C.POINTER(SaAgclArgs), _p]),
        "sa_agcl_conv1x1": (_i, [C.POINTER(SaAgclArgs), _p, _p, _i, _p, _i, _p]),
        "sa_cre_motion_head": (_i, [C.POINTER(SaAgclArgs), C.POINTER(SaCreHeadArgs), _p]),
        "sa_cre_motion_head_pre": (_i, [C.POINTER(SaAgclArgs), C.POINTER(SaCreHeadArgs), _p]),
        "sa_linear_attention": (_i, [_p, _i, _p, _i, _p, _i, _p, _i, _i, _i, _i, _i, _i, _f, _p, _p]),
        "sa_linear_attention_ws_floats": (C.c_long, [_i, _i, _i, _i]),
        "sa_layernorm": (_i, [_p, _i, _p, _p, _p, _i, _p, _i, C.c_long, _i, _f, _p]),
        "sa_ew": (_i, [C.POINTER(SaEwArgs), _p]),
        "sa_flow_features": (_i, [_p, _i, C.c_long, _p, _i, _i, _p, _i, _p]),
        "sa_interp_flow": (_i, [_p, _p, _i, _i, _i, _i, _i, _i, _f, _p]),
        "sa_convex_upsample_c": (_i, [_p, _i, _p, _i, _i, _i, _i, _i, _f, _p, _i, _p]),
        "sa_dwconv3x3": (_i, [_p, _i, _p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _p]),
        "sa_norm_corr_volume": (_i, [_p, _i, _p, _i, _i, _i, _i, _i, _i, _p, _i, _p]),
        "sa_topk_disparity": (_i, [_p, _i, _i, _i, _i, _i, _i, _i, _p, _p, _p]),
        "sa_concat_volume": (_i, [_p, _i, _p, _i, _p, _p, _i, _i, _i, _i, _i, _p, _i, _p]),
        "sa_topk_regress": (_i, [_p, _i, _i, _p, _i, _i, _i, _i, _i, _p, _p]),
        "sa_spx_upsample": (_i, [_p, _i, _p, _i, _i, _i, _i, _f, _p, _p]),
        "sa_version": (C.c_char_p, []),
        "sa_last_error": (C.c_char_p, []),
        "sa_engine_create": (_p, [C.c_char_p, C.c_char_p, _i, _i, _i, _i, _i, _i, C.c_ulonglong]),
        "sa_engine_destroy": (None, [_p]),
        "sa_engine_set_q": (_i, [_p, _p]),
        "sa_engine_set_rectify_maps": (_i, [_p, _p, _p]),
        "sa_engine_run_device": (_i, [_p, _p, _p, _p, _p, _i, _p, _p, _p]),
        "sa_engine_run_host": (_i, [_p, _p, _p, _p, _p, _i]),
        "sa_engine_device_bytes": (C.c_longlong, [_p]),
        "sa_engine_host_buffers": (None, [_p, _p, _p, _p, _p]),
        "sa_engine_host_times": (_i, [_p, C.POINTER(C.c_float), _i]),
        "sa_engine_copy_stream": (C.c_void_p, [_p]),
        "sa_engine_aux_output": (_p, [_p, C.POINTER(_i)]),
        "sa_engine_stream": (_p, [_p]),
        "sa_engine_plan_path": (C.c_char_p, [_p]),
        "sa_engine_tactics_digest": (C.c_char_p, [_p]),
        "sa_engine_plan_export": (_i, [_p, C.c_char_p]),
        "sa_conv_plan_pin": (None, [_i]),
        "sa_engine_tuned_shapes": (C.c_long, [_p]),
        "sa_engine_plan_status": (None, [_p, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
        "sa_plan_build_id": (C.c_char_p, []),
        "sa_engine_nonzero_splitk_counters": (C.c_long, [_p]),
        "sa_conv_tune_count": (C.c_long, []),
        "sa_conv_tune_rejects": (C.c_long, []),
        "sa_conv_plan_clear": (None, []),
        "sa_conv_plan_put": (None, [C.c_char_p, _i, _i, _f]),
        "sa_conv_plan_save": (_i, [C.c_char_p, C.c_char_p]),
        "sa_conv_plan_load": (_i, [C.c_char_p]),
        "sa_conv_plan_cache_append": (None, [C.c_char_p, _i, _i, _f]),
        "sa_conv_plan_entries": (C.c_long, []),
        "sa_conv2d_tile_lds": (_i, [_i]),
        "sa_tapproj_stencil": (_i, [_p, _i, _i, _p, _p, _i, _i, _i, _p]),
        "sa_engine_stage_times": (_i, [_p, C.POINTER(C.c_float), C.POINTER(C.c_char_p), _i]),
        "sa_algorithm_create": (_p, [C.c_char_p, _i, C.c_char_p, C.c_char_p]),
        "sa_algorithm_run": (_i, [_p, _p, _p, _i, _i, _p, _p, _i]),
        "sa_algorithm_frame_size": (_i, [_p, C.POINTER(_i), C.POINTER(_i)]),
        "sa_algorithm_last_ms": (_f, [_p]),
        "sa_algorithm_destroy": (None, [_p]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.restype = res
        fn.argtypes = args
    size = getattr(lib, "sa_struct_size", None)
    if size is not None:
        size.restype, size.argtypes = C.c_long, [C.c_char_p]
        for st in (SaConvSrc, SaConvArgs, SaNormArgs, SaAgclArgs, SaEwArgs):
            n = size(st.__name__.encode())
            if n != C.sizeof(st):
                raise RuntimeError(f"{st.__name__}: ctypes layout {C.sizeof(st)} B != native {n} B "
                                   "(stereoalgorithms_amd/_native.py out of sync with csrc/include/sa/kernels.h)")


def _declare_host(lib):
    # geometry / calibration / image io; declared lazily by stereoalgorithms_amd.utils modules
    pass


def check(rc: int, what: str):
    if rc != 0:
        msg = ""
        try:
            msg = dev().sa_last_error().decode()
        except Exception:  # pragma: no cover
            pass
        raise RuntimeError(f"{what} failed (rc={rc}) {msg}")


def on_gpu_box() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:  # pragma: no cover
        return False


def require_native():
    """Fail loudly when the native library is missing on a GPU machine."""
    if not available():
        raise NativeMissing("libstereo_amd.so missing: build it before running on the GPU")
    return dev()


os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
