"""ctypes binding of the flr C ABI (``include/flr.h``, ``lib/libflr.so``).

The library is the product path: every aggregation op in :mod:`flr.ops`
calls through here.  There is no CPU or PyTorch fallback — if the shared
library is missing or fails to load, :func:`lib` raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("FLR_LIB", os.path.join(_PKG_ROOT, "lib", "libflr.so"))
HEADER_PATH = os.path.join(os.path.dirname(_PKG_ROOT), "include", "flr.h")

FLR_OK = 0
FLR_ERR_ARG = -1
FLR_ERR_HIP = -2
FLR_ERR_UNSUPPORTED = -3
FLR_ERR_WORKSPACE = -4
FLR_ERR_KRUM_N = -5

_c_void_p = ctypes.c_void_p
_i64 = ctypes.c_int64
_size_t = ctypes.c_size_t
_int = ctypes.c_int

# name -> (restype, argtypes); must list every function include/flr.h declares.
SIGNATURES = {
    "flr_version": (ctypes.c_char_p, []),
    "flr_build_info": (ctypes.c_char_p, []),
    "flr_set_knob": (_int, [ctypes.c_char_p, ctypes.c_char_p]),
    "flr_status_string": (ctypes.c_char_p, [_int]),
    "flr_last_error": (ctypes.c_char_p, []),
    "flr_pairwise_l2_workspace": (_size_t, [_i64, _i64]),
    "flr_pairwise_l2": (_int, [_c_void_p, _i64, _i64, _i64, _c_void_p, _c_void_p, _size_t, _c_void_p]),
    "flr_pairwise_l2_ex": (_int, [_c_void_p, _i64, _i64, _i64, _c_void_p, _c_void_p, _size_t, _c_void_p, _c_void_p,
                                  _c_void_p]),
    "flr_pw_slice_chunks": (_int, [_i64, _i64, _c_void_p, _c_void_p]),
    "flr_pairwise_sample_len": (_i64, [_i64]),
    "flr_pairwise_gsum_len": (_size_t, [_i64]),
    "flr_pairwise_pivot_len": (_i64, []),
    "flr_pairwise_sliced_workspace": (_size_t, [_i64, _i64, _i64]),
    "flr_pairwise_sample": (_int, [_c_void_p, _i64, _i64, _i64, _i64, _i64, _c_void_p, _c_void_p]),
    "flr_pairwise_pivot": (_int, [_c_void_p, _i64, _i64, _c_void_p, _c_void_p, _size_t, _c_void_p]),
    "flr_pairwise_gram_slices": (_int, [_c_void_p, _i64, _i64, _i64, _i64, _i64, _c_void_p, _c_void_p, _c_void_p,
                                        _size_t, _c_void_p, _c_void_p, _c_void_p]),
    "flr_pairwise_tail": (_int, [_c_void_p, _i64, _i64, _i64, _i64, _c_void_p, _c_void_p]),
    "flr_pairwise_finish": (_int, [_c_void_p, _c_void_p, _i64, _c_void_p, _c_void_p]),
    "flr_pairwise_l2_reference_workspace": (_size_t, [_i64, _i64]),
    "flr_pairwise_l2_reference_tiles": (_int, [_i64]),
    "flr_pairwise_l2_reference": (_int, [_c_void_p, _i64, _i64, _i64, _c_void_p, _c_void_p, _size_t, _i64, _i64,
                                         _c_void_p]),
    "flr_pairwise_l2_reference_tap": (_int, [_c_void_p, _i64, _i64, _i64, _c_void_p, _i64, _c_void_p, _c_void_p,
                                             _size_t, _i64, _i64, _c_void_p]),
    "flr_pairwise_l2_reference_tap_dead": (_int, [_c_void_p, _i64, _i64, _i64, _c_void_p, _i64, _c_void_p, _c_void_p,
                                                  _i64, _c_void_p, _c_void_p, _size_t, _i64, _i64, _c_void_p,
                                                  _c_void_p]),
    "flr_pairwise_l2_reference_partial": (_int, [_c_void_p, _i64, _i64, _i64, _int, _c_void_p, _size_t, _c_void_p]),
    "flr_pairwise_l2_reference_partial_tap": (_int, [_c_void_p, _i64, _i64, _i64, _c_void_p, _i64, _int, _c_void_p,
                                                     _size_t, _c_void_p]),
    "flr_pairwise_l2_reference_finish": (_int, [_c_void_p, _i64, _i64, _i64, _int, _c_void_p, _c_void_p, _c_void_p]),
    "flr_pairwise_l2_direct_workspace": (_size_t, [_i64, _i64]),
    "flr_pairwise_l2_direct": (_int, [_c_void_p, _i64, _i64, _i64, _c_void_p, _c_void_p, _size_t, _c_void_p]),
    "flr_krum_select": (_int, [_c_void_p, _i64, _i64, _c_void_p, _c_void_p, _c_void_p]),
    "flr_rows_mean_dead": (_int, [_c_void_p, _i64, _i64, _i64, _c_void_p, _i64, _i64, _c_void_p, _c_void_p, _i64,
                                  _c_void_p, _i64, _c_void_p, _c_void_p]),
    "flr_rows_mean": (_int, [_c_void_p, _i64, _i64, _i64, _c_void_p, _i64, _i64, _c_void_p, _c_void_p]),
    "flr_fedavg": (_int, [_c_void_p, _i64, _i64, _i64, _c_void_p, _c_void_p, _c_void_p]),
    "flr_trimmed_mean": (_int, [_c_void_p, _i64, _i64, _i64, _i64, _c_void_p, _c_void_p]),
    "flr_median_lower": (_int, [_c_void_p, _i64, _i64, _i64, _c_void_p, _c_void_p]),
    "flr_trimmed_mean_rows": (_int, [_c_void_p, _i64, _i64, _i64, _c_void_p, _i64, _i64, _c_void_p, _c_void_p]),
    "flr_median_lower_rows": (_int, [_c_void_p, _i64, _i64, _i64, _c_void_p, _i64, _c_void_p, _c_void_p]),
    "flr_clip_sgd_workspace": (_size_t, [_i64]),
    "flr_clip_sgd_step": (_int, [_c_void_p, _c_void_p, _c_void_p, _i64, _i64, _i64, ctypes.c_float, ctypes.c_float,
                                 ctypes.c_float, ctypes.c_float, _int, _c_void_p, _c_void_p, _size_t, _c_void_p]),
    "flr_clip_sgd_step_blocked": (_int, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _i64, _i64,
                                         ctypes.c_float,
                                         ctypes.c_float, ctypes.c_float, ctypes.c_float, _int, _c_void_p, _c_void_p,
                                         _size_t, _c_void_p]),
    "flr_clip_sgd_step_blocked_x": (_int, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _i64, _i64,
                                           ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float, _int,
                                           _c_void_p, _c_void_p, _i64, _i64, _c_void_p, _c_void_p, _i64,
                                           _c_void_p, _c_void_p, _size_t, _c_void_p]),
    "flr_clip_sgd_step_blocked_src": (_int, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _i64, _i64,
                                             ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float, _int,
                                             _c_void_p, _c_void_p, _i64, _i64, _c_void_p, _c_void_p, _i64,
                                             _c_void_p, _c_void_p, _c_void_p, _c_void_p, _size_t, _c_void_p]),
    "flr_clip_sgd_step_phase": (_int, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _i64, _i64,
                                       ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float, _int,
                                       _c_void_p, _c_void_p, _i64, _i64, _c_void_p, _c_void_p, _i64,
                                       _c_void_p, _c_void_p, _c_void_p, _int, _c_void_p, _size_t, _c_void_p]),
    "flr_batchnorm_relu_maxpool_fwd": (_int, [_c_void_p] * 7 + [_i64] * 4 + [ctypes.c_float, _c_void_p]),
    "flr_maxpool_relu_batchnorm_bwd": (_int, [_c_void_p] * 10 + [_i64] * 4 + [_c_void_p]),
    "flr_conv2d_workspace": (_size_t, [_i64] * 10),
    "flr_resnet_gru_num_params": (_i64, [_c_void_p]),
    "flr_train_clients_workspace": (_size_t, [_c_void_p, _i64, _i64, _i64]),
    "flr_train_clients": (_int, [_c_void_p, _c_void_p, _c_void_p, _i64, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                                 _i64, _i64, _i64, ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                 _i64, _c_void_p, _c_void_p, _c_void_p, _size_t, _c_void_p]),
    "flr_train_clients_ex": (_int, [_c_void_p, _c_void_p, _c_void_p, _i64, _c_void_p, _c_void_p, _c_void_p,
                                    _c_void_p, _i64, _i64, _i64, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                    ctypes.c_float, _i64, _c_void_p, _c_void_p, ctypes.c_uint, _c_void_p, _size_t,
                                    _c_void_p]),
    "flr_resnet_gru_reorder": (_int, [_c_void_p, _c_void_p, _c_void_p, _int, _c_void_p]),
    "flr_resnet_gru_live_params": (_i64, [_c_void_p, ctypes.c_float]),
    "flr_resnet_gru_dead_ranges": (_i64, [_c_void_p, ctypes.c_float, _c_void_p, _c_void_p, _i64]),
    "flr_resnet_gru_fill_dead": (_int, [_c_void_p, ctypes.c_float, _c_void_p, _c_void_p, _i64, _i64, _i64, _c_void_p]),
    "flr_vit_bert_num_params": (_i64, [_c_void_p]),
    "flr_train_vit_bert_workspace": (_size_t, [_c_void_p, _i64, _i64, _i64, _i64]),
    "flr_train_vit_bert": (_int, [_c_void_p, _c_void_p, _c_void_p, _i64, _c_void_p, _c_void_p, _c_void_p,
                                  _c_void_p, _i64, _i64, _i64, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                  ctypes.c_float, _i64, _c_void_p, _c_void_p, ctypes.c_uint, _i64, _c_void_p,
                                  _size_t, _c_void_p]),
    "flr_conv2d_tap_major_ok": (_int, [_i64, _i64]),
    "flr_conv2d_t_workspace": (_size_t, [_i64] * 10),
    "flr_conv2d_fwd_t": (_int, [_c_void_p, _c_void_p, _c_void_p] + [_i64] * 10 + [_c_void_p, _size_t, _c_void_p]),
    "flr_conv2d_bwd_data_t": (_int, [_c_void_p, _c_void_p, _c_void_p] + [_i64] * 10 + [_c_void_p, _size_t, _c_void_p]),
    "flr_conv2d_bwd_data_t_add": (_int, [_c_void_p] * 4 + [_i64] * 10 + [_c_void_p, _size_t, _c_void_p]),
    "flr_conv2d_fwd_t_ex": (_int, [_c_void_p, _c_void_p, _i64, _c_void_p] + [_i64] * 10 + [_c_void_p, _size_t,
                                                                                          _c_void_p]),
    "flr_conv2d_bwd_data_t_ex": (_int, [_c_void_p, _c_void_p, _i64, _c_void_p, _c_void_p] + [_i64] * 10 +
                                 [_c_void_p, _size_t, _c_void_p]),
    "flr_conv2d_bwd_weight_t": (_int, [_c_void_p, _c_void_p, _c_void_p] + [_i64] * 10 + [_int, _c_void_p, _size_t,
                                                                                         _c_void_p]),
    "flr_conv2d_bwd_weight_t_sq_slots": (_i64, [_i64] * 10),
    "flr_conv2d_bwd_weight_t_sq": (_int, [_c_void_p, _c_void_p, _c_void_p] + [_i64] * 10 + [_int, _c_void_p, _i64,
                                                                                            _c_void_p, _size_t,
                                                                                            _c_void_p]),
    "flr_conv2d_fwd": (_int, [_c_void_p, _c_void_p, _c_void_p] + [_i64] * 10 + [_c_void_p, _size_t, _c_void_p]),
    "flr_conv2d_bwd_data": (_int, [_c_void_p, _c_void_p, _c_void_p] + [_i64] * 10 + [_c_void_p, _size_t, _c_void_p]),
    "flr_conv2d_bwd_weight": (_int, [_c_void_p, _c_void_p, _c_void_p] + [_i64] * 10 + [_c_void_p, _size_t, _c_void_p]),
    "flr_conv2d_bwd_weight_reuse": (_int, [_c_void_p, _c_void_p, _c_void_p] + [_i64] * 10 + [_c_void_p, _size_t,
                                                                                            _c_void_p]),
    "flr_cross_entropy": (_int, [_c_void_p, _c_void_p, _i64, _i64, _i64, _c_void_p, _c_void_p, _c_void_p, _c_void_p]),
    "flr_mean_rows": (_int, [_c_void_p, _i64, _i64, _c_void_p, _c_void_p]),
    "flr_scale_client_rows": (_int, [_c_void_p, _c_void_p, _i64, _i64, _i64, _c_void_p]),
    "flr_broadcast_rows": (_int, [_c_void_p, _i64, _c_void_p, _i64, _i64, _c_void_p]),
    "flr_broadcast_rows_neg": (_int, [_c_void_p, _i64, _c_void_p, _i64, _i64, _i64, _c_void_p]),
    "flr_copy_rows": (_int, [_c_void_p, _i64, _i64, _c_void_p, _i64, _i64, _c_void_p]),
    "flr_tap_major_to_torch": (_int, [_c_void_p, _i64, _i64, _i64, _i64, _c_void_p, _i64, _c_void_p]),
    "flr_copy_rows_neg": (_int, [_c_void_p, _i64, _i64, _c_void_p, _i64, _i64, _i64, _c_void_p]),
    "flr_tap_major_to_torch_neg": (_int, [_c_void_p, _i64, _i64, _i64, _i64, _c_void_p, _i64, _i64, _c_void_p]),
    "flr_row_norms_workspace": (_size_t, [_i64]),
    "flr_row_norms": (_int, [_c_void_p, _i64, _i64, _i64, _c_void_p, _int, _c_void_p, _c_void_p, _size_t,
                             _c_void_p]),
    "flr_row_dots": (_int, [_c_void_p, _i64, _i64, _i64, _c_void_p, _c_void_p, _c_void_p, _size_t, _c_void_p]),
    "flr_weighted_rows": (_int, [_c_void_p, _i64, _i64, _i64, _c_void_p, _i64, _c_void_p, _c_void_p,
                                 ctypes.c_float, _c_void_p, _c_void_p]),
    "flr_batchnorm_fwd": (_int, [_c_void_p] * 7 + [_i64] * 3 + [ctypes.c_float, _int, _c_void_p]),
    "flr_batchnorm_bwd": (_int, [_c_void_p] * 10 + [_i64] * 3 + [_int, _c_void_p]),
    "flr_bgemm_workspace": (_size_t, [_i64] * 4),
    "flr_bgemm": (_int, [_c_void_p, _i64, _i64, _i64, _c_void_p, _i64, _i64, _i64, _c_void_p, _i64, _i64, _i64,
                         _c_void_p, _i64, _c_void_p, _i64, _i64, _i64, _i64, _c_void_p, _size_t, _c_void_p]),
    "flr_bgemm_ex": (_int, [_c_void_p, _i64, _i64, _i64, _c_void_p, _i64, _i64, _i64, _c_void_p, _i64, _i64, _i64,
                            _c_void_p, _i64, _c_void_p, _int, _c_void_p, _c_void_p, _c_void_p, _i64, _i64, _i64, _i64,
                            _c_void_p, _size_t, _c_void_p]),
    "flr_fill": (_int, [_c_void_p, _i64, ctypes.c_float, _c_void_p]),
    "flr_act_bwd": (_int, [_c_void_p, _c_void_p, _c_void_p, _int, _c_void_p, _i64, _c_void_p]),
    "flr_embedding_fwd": (_int, [_c_void_p, _i64, _i64, _c_void_p, _i64] * 3 + [_i64, _i64, _i64, _c_void_p,
                                                                                _c_void_p]),
    "flr_embedding_bwd_workspace": (_size_t, [_i64, _i64]),
    "flr_embedding_bwd": (_int, [_c_void_p, _c_void_p, _i64, _i64, _i64, _i64, _i64, _c_void_p, _i64, _int,
                                 _c_void_p, _size_t, _c_void_p]),
    "flr_layernorm_fwd": (_int, [_c_void_p, _i64, _c_void_p, _i64, _c_void_p, _c_void_p, _c_void_p, _i64, _c_void_p,
                                 _i64, _c_void_p, _c_void_p, _i64, _i64, _i64, ctypes.c_float, _c_void_p]),
    "flr_layernorm_bwd_workspace": (_size_t, [_i64, _i64, _i64]),
    "flr_layernorm_bwd": (_int, [_c_void_p, _i64, _c_void_p, _i64, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _i64,
                                 _c_void_p, _i64, _c_void_p, _c_void_p, _i64, _i64, _i64, _c_void_p, _size_t,
                                 _c_void_p]),
    "flr_vit_tokens": (_int, [_c_void_p, _c_void_p, _c_void_p, _i64, _i64, _i64, _i64, _c_void_p, _c_void_p]),
    "flr_attention_fwd": (_int, [_c_void_p, _i64, _i64, _i64, _i64, _c_void_p, _c_void_p, _c_void_p]),
    "flr_attention_bwd": (_int, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _i64, _i64, _i64, _i64, _c_void_p,
                                 _c_void_p]),
    "flr_sum_rows": (_int, [_c_void_p, _i64, _i64, _i64, _i64, _i64, _c_void_p, _i64, _c_void_p]),
    "flr_sum_rows_workspace": (_size_t, [_i64, _i64, _i64]),
    "flr_sum_rows_ex": (_int, [_c_void_p, _i64, _i64, _i64, _i64, _i64, _c_void_p, _i64, _c_void_p, _size_t,
                               _c_void_p]),
    "flr_maxpool2d_fwd": (_int, [_c_void_p] * 3 + [_i64] * 7 + [_c_void_p]),
    "flr_maxpool2d_bwd": (_int, [_c_void_p] * 3 + [_i64] * 7 + [_c_void_p]),
    "flr_gru_fwd_step": (_int, [_c_void_p] * 4 + [_i64] * 5 + [_c_void_p]),
    "flr_gru_bwd_step": (_int, [_c_void_p] * 6 + [_i64] * 5 + [_c_void_p]),
    "flr_gru_fwd_fused": (_int, [_c_void_p] * 5 + [_i64] * 5 + [_c_void_p]),
    "flr_gru_bwd_fused": (_int, [_c_void_p] * 7 + [_i64] * 5 + [_c_void_p]),
    "flr_gru_pack": (_int, [_c_void_p, _i64, _i64, _i64, _i64, _int, _c_void_p, _c_void_p]),
    "flr_gru_fwd_fused_ex": (_int, [_c_void_p, _c_void_p, _int] + [_c_void_p] * 3 + [_i64] * 5 + [_c_void_p]),
    "flr_gru_bwd_fused_ex": (_int, [_c_void_p, _int] + [_c_void_p] * 6 + [_i64] * 5 + [_c_void_p]),
    "flr_batchnorm_infer": (_int, [_c_void_p] * 7 + [_i64, _i64, ctypes.c_float, _int, _c_void_p]),
    "flr_classify_rows": (_int, [_c_void_p, _c_void_p, _i64, _i64, _i64, _i64, _c_void_p, _c_void_p, _c_void_p,
                                 _c_void_p]),
}

_lock = threading.Lock()
_lib = None


class FlrError(RuntimeError):
    """A C-ABI call returned a non-zero status."""

    def __init__(self, fn: str, status: int, detail: str = ""):
        self.status = status
        msg = f"{fn} failed: {status_string(status)} ({status})"
        if detail:
            msg += f": {detail}"
        super().__init__(msg)


def lib() -> ctypes.CDLL:
    """Load libflr.so once; raise loudly if it is absent (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"flr native library not found at {LIB_PATH}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (or make -C "
                "multimodal-fl-security_amd/csrc). There is no CPU fallback.")
        # torch must be imported first so its libamdhip64.so.7 is the runtime
        # this library binds to (same SONAME -> one HIP runtime per process).
        import torch  # noqa: F401
        handle = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
        return _lib


def set_knob(name: str, value) -> None:
    """Set (value None: unset) one of the library's A/B switches (FLR_*; the
    process environment is read once, when the library loads)."""
    check("flr_set_knob", lib().flr_set_knob(name.encode(), None if value is None else str(value).encode()))


def build_info() -> str:
    """'gfx950', or 'gfx950 ablation' for the tools build (make ABLATION=1)."""
    return lib().flr_build_info().decode()


def status_string(status: int) -> str:
    try:
        return lib().flr_status_string(status).decode()
    except Exception:  # pragma: no cover - only when the lib is unusable
        return "unknown"


def check(fn: str, status: int) -> None:
    if status != FLR_OK:
        detail = ""
        if status == FLR_ERR_HIP:
            detail = lib().flr_last_error().decode()
        raise FlrError(fn, status, detail)


def call(fn: str, *args) -> int:
    status = getattr(lib(), fn)(*args)
    check(fn, status)
    return status
