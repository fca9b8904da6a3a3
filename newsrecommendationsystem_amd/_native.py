"""ctypes binding of libnrms_hip.so (C ABI: include/nrms_hip.h).

The library is the product path: if it is missing or fails to load, every
entry point raises — there is no eager / CPU fallback. Torch is imported first
so the library binds to the HIP runtime torch already loaded (same soname),
letting torch's stream handles and device pointers be passed straight in.
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load: shared HIP runtime)

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NRMS_LIB_PATH") or os.path.join(_PKG, "libnrms_hip.so")   # override: A/B builds
ABI_VERSION = 8

NRMS_PROJ_AUTO, NRMS_PROJ_DIRECT, NRMS_PROJ_FOLDED = 0, 1, 2
NRMS_GEMM_SPLIT_BF16X6, NRMS_GEMM_F32, NRMS_GEMM_SPLIT_F16X3 = 0, 1, 2
NRMS_OK, NRMS_ERR_INVALID_ARG, NRMS_ERR_UNSUPPORTED, NRMS_ERR_WORKSPACE, NRMS_ERR_HIP = 0, 1, 2, 3, 4
GEMM_ARITH_NAMES = {NRMS_GEMM_SPLIT_BF16X6: "split-bf16x6", NRMS_GEMM_F32: "f32",
                    NRMS_GEMM_SPLIT_F16X3: "split-f16x3"}

_p = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_sz = ctypes.c_size_t


class EncoderWeights(ctypes.Structure):
    """nrms_encoder_weights_t."""
    _fields_ = [("w_q", _p), ("b_q", _p), ("w_k", _p), ("b_k", _p), ("w_v", _p), ("b_v", _p),
                ("w_add", _p), ("b_add", _p), ("q_add", _p),
                ("d_model", _i32), ("n_heads", _i32), ("query_dim", _i32)]


_EW = ctypes.POINTER(EncoderWeights)

# name -> (restype, argtypes)
SIGNATURES = {
    "nrms_abi_version": (_i32, []),
    "nrms_set_gemm_arith": (_i32, [_i32]),
    "nrms_set_title_dedupe": (_i32, [_i32]),
    "nrms_set_token_compaction": (_i32, [_i32]),
    "nrms_set_thread_gemm_arith": (_i32, [_i32]),
    "nrms_set_thread_title_dedupe": (_i32, [_i32]),
    "nrms_set_thread_token_compaction": (_i32, [_i32]),
    "nrms_get_gemm_arith": (_i32, []),
    "nrms_status_string": (ctypes.c_char_p, [_i32]),
    "nrms_last_hip_error": (_i32, []),
    "nrms_embedding_gather": (_i32, [_p, _i64, _p, _i64, _i32, _p, _p]),
    "nrms_qkv_row_stride": (_i32, [_i32]),
    "nrms_qkv_project": (_i32, [_p, _i64, _p, _i64, _EW, _p, _i64, _p]),
    "nrms_qkv_project_workspace_size": (_sz, [_i32]),
    "nrms_qkv_project_ws": (_i32, [_p, _i64, _p, _i64, _EW, _p, _i64, _p, _sz, _p]),
    "nrms_self_attention": (_i32, [_p, _i64, _p, _i64, _p, _i64, _i32, _EW, _p, _p]),
    "nrms_additive_attention": (_i32, [_p, _i64, _i32, _EW, _p, _p, _p]),
    "nrms_additive_scores": (_i32, [_p, _i64, _EW, _p, _p]),
    "nrms_additive_pool": (_i32, [_p, _p, _i64, _i32, _i32, _p, _p]),
    "nrms_news_attention_pool_workspace_size": (_sz, [_i64, _i32, _i32]),
    "nrms_news_attention_pool": (_i32, [_p, _i64, _i64, _p, _i64, _p, _i64, _i32, _EW, _p, _p, _sz,
                                         _p]),
    "nrms_news_encode_workspace_size": (_sz, [_i64, _i32, _i64, _i32, _i32]),
    "nrms_news_encode": (_i32, [_p, _i64, _i32, _p, _i64, _EW, _i32, _p, _p, _sz, _p]),
    "nrms_news_encode_folded_workspace_size": (_sz, [_i64, _i32, _i32]),
    "nrms_news_encode_folded": (_i32, [_p, _i64, _i32, _p, _i64, _i64, _EW, _p, _p, _sz, _p]),
    "nrms_user_attention_pool_workspace_size": (_sz, [_i64, _i32, _i32]),
    "nrms_user_attention_pool": (_i32, [_p, _i64, _i64, _i32, _EW, _p, _p, _sz, _p]),
    "nrms_user_attention_pool_padded": (_i32, [_p, _i64, _i64, _i32, _p, _EW, _p, _p, _sz, _p]),
    "nrms_user_encode_workspace_size": (_sz, [_i64, _i32, _i32]),
    "nrms_user_encode": (_i32, [_p, _i64, _i32, _i64, _i64, _EW, _p, _p, _sz, _p]),
    "nrms_score": (_i32, [_p, _i64, _i32, _i64, _i64, _p, _i64, _i32, _p, _p]),
    "nrms_score_pairs": (_i32, [_p, _i64, _p, _i64, _p, _p, _i64, _i32, _p, _p]),
    "nrms_impression_metrics": (_i32, [_p, _p, _p, _i64, _p, _p]),
    # training kernels
    "nrms_dropout": (_i32, [_p, _p, _i64, ctypes.c_float, ctypes.c_uint64, _p]),
    "nrms_additive_forward_train": (_i32, [_p, _i64, _i32, _EW, _p, _p, _p, _p]),
    "nrms_additive_backward_workspace_size": (_sz, [_i64, _i32, _i32, _i32]),
    "nrms_additive_backward": (_i32, [_p, _i64, _i32, _EW, _p, _p, _p, _p, _p, _p, _p, _p, _sz, _p]),
    "nrms_self_attention_backward": (_i32, [_p, _p, _i64, _i32, _EW, _p, _p]),
    "nrms_qkv_project_backward_workspace_size": (_sz, [_i32]),
    "nrms_qkv_project_backward": (_i32, [_p, _i64, _EW, _p, _p, _p, _p, _p, _sz, _p]),
    "nrms_score_backward": (_i32, [_p, _i64, _i32, _i64, _i64, _p, _i64, _i32, _p, _p, _p, _p]),
    "nrms_embedding_backward": (_i32, [_p, _i64, _p, _i64, _i32, _i64, _p, _p]),
    "nrms_embedding_backward_workspace_size": (_sz, [_i64, _i64]),
    "nrms_embedding_backward_ws": (_i32, [_p, _i64, _p, _i64, _i32, _i64, _p, _p, _sz, _p]),
    "nrms_adam_step": (_i32, [_p, _p, _p, _p, _i64, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                              ctypes.c_float, _i64, _p]),
    "nrms_adam_step_multi": (_i32, [_p, _i32, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                    ctypes.c_float, _i64, _p]),
    "nrms_forward_workspace_size": (_sz, [_i64, _i32, _i32, _i32, _i64, _i32, _i32]),
    "nrms_forward": (_i32, [_p, _p, _i64, _i32, _i32, _i32, _p, _i64, _EW, _EW, _i32, _p, _p,
                            _sz, _p]),
    "nrms_forward_timed": (_i32, [_p, _p, _i64, _i32, _i32, _i32, _p, _i64, _EW, _EW, _i32, _p, _p,
                                  _sz, _p, _p, _i32]),
    "nrms_forward_stage_name": (ctypes.c_char_p, [_i32]),
    # host-side readers (HOST pointers)
    "nrms_behaviors_scan": (_i32, [_p, _i64, _p]),
    "nrms_behaviors_parse": (_i32, [_p, _i64, _p, _p, _p, _p, _p, _p, _p, _p, _p]),
    "nrms_news_parse": (_i32, [_p, _i64, _i32, _p, _p, _p, _p, _i64]),
}
NRMS_FORWARD_STAGES = 5

_lib = None


class NativeError(RuntimeError):
    pass


def load():
    """Load and type the library once; raise loudly if it is unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeError(
            f"{LIB_PATH} not found: build it with `python -m newsrecommendationsystem_amd.build` "
            "(there is no CPU or eager fallback for the NRMS HIP path)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    v = lib.nrms_abi_version()
    if v != ABI_VERSION:
        raise NativeError(f"libnrms_hip ABI {v} != expected {ABI_VERSION}")
    _lib = lib
    return lib


def check(status, what):
    if status != 0:
        lib = load()
        msg = lib.nrms_status_string(status).decode()
        hip = lib.nrms_last_hip_error()
        raise NativeError(f"{what} failed: {msg} (status {status}, hip error {hip})")


def call(name, *args):
    fn = getattr(load(), name)
    check(fn(*args), name)


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_handle(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class gemm_arith:
    """Context manager selecting the GEMM arithmetic (nrms_set_gemm_arith) for
    the enclosed calls; restores the previous mode on exit."""

    def __init__(self, mode):
        self.mode = mode

    def __enter__(self):
        prev = load().nrms_set_gemm_arith(self.mode)
        if prev < 0:
            raise NativeError(f"unknown GEMM arithmetic {self.mode}")
        self.prev = prev
        return self

    def __exit__(self, *exc):
        load().nrms_set_gemm_arith(self.prev)
        return False
