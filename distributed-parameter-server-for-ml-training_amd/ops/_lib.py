"""ctypes bindings of the psx native libraries (C ABI, see csrc/).

``kernels()`` loads ``_native/libpsx_kernels.so`` (HIP kernels for gfx950). It is loaded only
after ``import torch`` so that the kernels bind to the HIP runtime instance PyTorch-ROCm already
loaded (same soname ``libamdhip64.so.7``): our launches then go onto torch streams and are
captured by ``torch.cuda.CUDAGraph`` (hipGraph) like any torch op.

``runtime()`` loads ``_native/libpsx_runtime.so`` (host-only C++: server core, shared-memory
mailbox, CIFAR reader); it needs no GPU and is exercised by the CPU test-suite.

There is deliberately no Python fallback for the GPU kernels: if the library is missing on a
GPU box, every op raises ``NativeLibraryMissing``.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

from .. import NATIVE_DIR

_lock = threading.Lock()
_kern = None
_rt = None

vp = C.c_void_p
i32 = C.c_int
i64 = C.c_long
f32 = C.c_float
f64 = C.c_double
u32 = C.c_uint


class NativeLibraryMissing(RuntimeError):
    pass


class HipError(RuntimeError):
    pass


# name -> (restype, [argtypes])
_KERNEL_SIGS = {
    "psx_wgrad_reduce": (i32, [vp, i32, i32, i32, i32, i32, i32, i32, f32, vp, i32, vp]),
    "psx_wgrad_reduce_batch": (i32, [i32, vp, vp, vp, vp, vp, vp, vp, vp, f32, i32, vp]),
    "psx_conv2_workspace": (i64, [i32, i32, i32, i32, i32, i32]),
    "psx_conv_wgrad2": (i32, [vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, i32, i32, i32, vp]),
    "psx_conv_fwd2": (i32, [vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, i32, i32, vp, i32, vp,
                            vp]),
    "psx_conv_dgrad2": (i32, [vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, i32, i32, vp, i32, vp]),
    "psx_stem_conv": (i32, [vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, vp]),
    "psx_stem7_conv": (i32, [vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, vp]),
    "psx_conv_dgrad2_sc": (i32, [vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, i32, i32, vp, i32, vp,
                                 vp, i32, vp]),
    "psx_bgemm_f32": (i32, [vp, vp, vp, vp, i32, i32, i32, i32, i32, vp]),
    "psx_wino_workspace": (i64, [i32, i32, i32, i32, i32]),
    "psx_wino_ok": (i32, [i32, i32, i32, i32]),
    "psx_wino_weights": (i32, [vp, vp, i32, i32, i32, vp]),
    "psx_wino_weights_multi": (i32, [vp, vp, vp, vp, vp, i32, vp, vp]),
    "psx_wino_fused_ok": (i32, [i32, i32, i32, i32, i32]),
    "psx_wino_fused": (i32, [vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp]),
    "psx_wino_conv": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, vp, vp, vp, vp, vp]),
    "psx_wino_v_floats": (i64, [i32, i32, i32, i32]),
    "psx_wino_p_floats": (i64, [i32, i32, i32, i32, i32]),
    "psx_wino_wgrad_q": (i32, [i32, i32, i32, i32, i32]),
    "psx_wino_wgrad": (i32, [vp, vp, vp, vp, vp, i32, f32, vp, i32, i32, i32, i32, i32, vp, vp, vp, vp]),
    "psx_bgemm_tn_f32": (i32, [vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, vp]),
    "psx_wino_wout": (i32, [vp, vp, i32, f32, i32, i32, i32, vp]),
    "psx_wino_wgrad_fused_q": (i32, [i32, i32, i32, i32, i32]),
    "psx_wino_wgrad_fused": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, i32, f32, i32, i32, i32, i32, i32, vp]),
    "psx_bn_finalize": (i32, [vp, i32, i32, f32, vp, vp, f32, f32, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
    "psx_bn_eval_affine": (i32, [i32, vp, vp, vp, vp, f32, vp, vp, vp]),
    "psx_bn_apply": (i32, [vp, vp, vp, vp, vp, vp, vp, i64, i32, i32, i32, i32, vp]),
    "psx_bn_bwd_reduce": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, vp, vp, i32, vp]),
    "psx_bn_bwd_finalize": (i32, [vp, i32, i32, i32, i32, f32, vp, vp, vp, vp, vp, vp, f32, i32, vp]),
    "psx_bn_bwd_apply": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, i32, i32, vp]),
    "psx_bn_apply_fin": (i32, [vp, vp, vp, vp, vp, vp, vp, i64, i32, i32, i32, i32, vp]),
    "psx_bn_bwd_apply_fin": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, i32, i32, vp]),
    "psx_head_fwd_bwd": (i32, [vp, i32, i32, i32, vp, vp, i32, vp, vp, vp, vp, vp, vp, vp, i32, vp]),
    "psx_head_wgrad": (i32, [vp, vp, i32, i32, i32, vp, vp, f32, i32, vp]),
    "psx_sgd_apply": (i32, [vp, vp, vp, i64, f32, f32, f32, f32, i32, i32, vp, vp]),
    "psx_grad_aggregate": (i32, [vp, i32, i32, vp, i32, i64, f32, i32, vp]),
    "psx_set_deterministic": (i32, [i32]),
    "psx_det_slot_scale": (i32, []),
    "psx_sgd_apply_multi": (i32, [vp, vp, i32, vp, i64, f32, f32, f32, f32, i32, i32, vp, vp]),
    "psx_fp16_pack": (i32, [vp, vp, i64, f32, vp]),
    "psx_fp16_unpack": (i32, [vp, vp, i64, f32, vp]),
    "psx_param_unpack": (i32, [vp, vp, i32, vp, vp]),
    "psx_param_unpack_tiles": (i32, [vp, i32, vp, i32, i32, vp, vp, vp, i64, vp, i32, vp, i32, vp]),
    "psx_unpack_desc_size": (i32, []),
    "psx_synth_gen": (i32, [vp, vp, i32, i32, i32, i32, u32, u32, vp]),
    "psx_augment": (i32, [vp, vp, vp, vp, vp, i32, i32, i32, i32, u32, vp, i32, vp, vp, vp, i64, vp, i64, vp, vp, i64,
                          i32, vp]),
    "psx_nchw_to_nhwc": (i32, [vp, vp, i32, i32, i32, i32, i32, i32, vp]),
    "psx_maxpool3s2_fwd": (i32, [vp, vp, vp, i32, i32, i32, i32, i32, vp]),
    "psx_maxpool3s2_bwd": (i32, [vp, vp, vp, i32, i32, i32, i32, i32, vp]),
    "psx_topk_workspace_words": (i64, [i64]),
    "psx_topk_payload_words": (i32, [i32]),
    "psx_topk_encode": (i32, [vp, i32, vp, i64, i32, i32, vp, vp, vp]),
    "psx_topk_decode_add": (i32, [vp, vp, f32, i32, vp]),
}

_RUNTIME_SIGS = {
    "psx_ps_create": (vp, [i32, i32, f32, i32, i32]),
    "psx_ps_destroy": (None, [vp]),
    "psx_ps_register": (i32, [vp, C.c_char_p, i32, f64]),
    "psx_ps_heartbeat": (None, [vp, i32, f64]),
    "psx_ps_on_fetch": (C.c_int64, [vp, i32, f64]),
    "psx_ps_on_push": (i32, [vp, i32, C.c_int64, f64, C.POINTER(f32), C.POINTER(i32), C.POINTER(C.c_int64)]),
    "psx_ps_round_members": (i32, [vp, C.POINTER(i32), i32]),
    "psx_ps_on_applied": (None, [vp, f64]),
    "psx_ps_record_update_time": (None, [vp, f64]),
    "psx_ps_job_finished": (i32, [vp, i32]),
    "psx_ps_mark_dead": (i32, [vp, i32]),
    "psx_ps_check_timeouts": (i32, [vp, f64, f64, C.POINTER(i32), i32]),
    "psx_ps_sync_ready": (i32, [vp]),
    "psx_ps_global_step": (C.c_int64, [vp]),
    "psx_ps_set_global_step": (None, [vp, C.c_int64]),
    "psx_ps_rollback_to": (None, [vp, C.c_int64]),
    "psx_ps_num_active": (i32, [vp]),
    "psx_ps_metrics_json": (i32, [vp, f64, C.c_char_p, i32]),
    "psx_ps_staleness_hist": (i32, [vp, C.POINTER(C.c_int64), i32]),
    "psx_mbox_open": (vp, [C.c_char_p, i32, i32, i32, f64]),
    "psx_mbox_close": (None, [vp]),
    "psx_mbox_send": (i32, [vp, i32, i32, i32, i32, C.c_longlong, C.c_longlong, f64]),
    "psx_mbox_recv": (i32, [vp, C.POINTER(C.c_longlong), f64]),
    "psx_mbox_reply": (i32, [vp, i32, i32, i32, i32, C.c_longlong, C.c_longlong]),
    "psx_mbox_wait_reply": (C.c_longlong, [vp, i32, C.c_longlong, C.POINTER(C.c_longlong), f64]),
    "psx_cifar_count": (i64, [C.c_char_p, i32]),
    "psx_cifar_read": (i64, [C.c_char_p, i32, i32, vp, vp, i64, i32]),
}


_COMM_SIGS = {
    "psx_comm_load": (i32, [C.c_char_p]),
    "psx_comm_id_bytes": (i32, []),
    "psx_comm_unique_id": (i32, [C.c_char_p]),
    "psx_comm_init": (i32, [C.c_char_p, i32, i32, i32, C.POINTER(vp)]),
    "psx_comm_destroy": (i32, [vp]),
    "psx_comm_abort": (i32, [vp]),
    "psx_comm_async_error": (i32, [vp]),
    "psx_comm_count": (i32, [vp, C.POINTER(i32)]),
    "psx_comm_error_string": (C.c_char_p, [i32]),
    "psx_comm_reduce_sum": (i32, [vp, vp, vp, i64, i32, i32, vp]),
    "psx_comm_all_reduce_sum": (i32, [vp, vp, vp, i64, i32, vp]),
    "psx_comm_broadcast": (i32, [vp, vp, i64, i32, i32, vp]),
    "psx_comm_reduce_scatter_sum": (i32, [vp, vp, vp, i64, i32, vp]),
    "psx_comm_all_gather": (i32, [vp, vp, vp, i64, i32, vp]),
    "psx_comm_send": (i32, [vp, vp, i64, i32, i32, vp]),
    "psx_comm_recv": (i32, [vp, vp, i64, i32, i32, vp]),
    "psx_comm_group_start": (i32, []),
    "psx_comm_group_end": (i32, []),
    "psx_comm_gather": (i32, [vp, vp, vp, i64, i32, i32, i32, i32, i32, vp]),
}


def _declare(lib, sigs, optional=False):
    for name, (res, args) in sigs.items():
        if optional and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def _maybe_build(libname: str) -> str:
    path = os.path.join(NATIVE_DIR, libname)
    if not os.path.exists(path) and os.environ.get("PSX_NO_AUTOBUILD", "0") != "1":
        import importlib.util

        build_py = os.path.join(os.path.dirname(os.path.dirname(NATIVE_DIR)), "csrc", "build.py")
        if os.path.exists(build_py):
            spec = importlib.util.spec_from_file_location("_psx_build", build_py)
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
            mod.build()
    if not os.path.exists(path):
        raise NativeLibraryMissing(f"{path} not found; run `python csrc/build.py`")
    return path


def kernels():
    """The HIP kernel library (imports torch first so both share one HIP runtime)."""
    global _kern
    if _kern is None:
        with _lock:
            if _kern is None:
                import torch  # noqa: F401  (must precede the dlopen, see module docstring)

                alt = os.environ.get("PSX_KERNELS_LIB")  # dev A/B: another build of the kernel library
                if alt:
                    _kern = _declare(C.CDLL(os.path.abspath(alt), mode=C.RTLD_GLOBAL), _KERNEL_SIGS, optional=True)
                else:
                    _kern = _declare(C.CDLL(_maybe_build("libpsx_kernels.so"), mode=C.RTLD_GLOBAL), _KERNEL_SIGS)
    return _kern


_comm = None


def comm():
    """The native RCCL data-plane library (csrc/comm/rccl_comm.cpp); loaded after torch so it
    shares PyTorch's HIP runtime (RCCL itself is bound by psx_comm_load)."""
    global _comm
    if _comm is None:
        with _lock:
            if _comm is None:
                import torch  # noqa: F401

                _comm = _declare(C.CDLL(_maybe_build("libpsx_comm.so"), mode=C.RTLD_GLOBAL), _COMM_SIGS)
    return _comm


def runtime():
    global _rt
    if _rt is None:
        with _lock:
            if _rt is None:
                _rt = _declare(C.CDLL(_maybe_build("libpsx_runtime.so")), _RUNTIME_SIGS)
    return _rt


def check(rc: int, what: str) -> int:
    if rc != 0:
        raise HipError(f"{what} failed with code {rc}")
    return rc


def stream_ptr(stream=None) -> int:
    import torch

    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


def ptr(t) -> int | None:
    """Raw device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()
