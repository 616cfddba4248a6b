"""spmv_amd — Python host mirror of the MI355X SpMV suite's C-ABI.

The product is C/HIP: ``lib/libspmv_hip.so`` (gfx950 kernels behind the
``extern "C"`` entry points of ``include/spmv.h``) and ``lib/libspmv_host.so``
(Matrix Market reader, format builders, generators, CPU loops; declared in
``include/spmv_host.h``).  This module binds both with ctypes so tests and
``bench.py`` drive exactly the calls the C drivers make.  PyTorch is used
only as plumbing: device memory (CUDA tensors on ROCm), the current HIP
stream and ``torch.distributed``.

There is no fallback: if ``libspmv_hip.so`` is missing or a HIP call fails,
``SpmvError`` is raised.  The five formats mirror the reference's five
programs (reference coo.c, csr.c, ell.c, sigma_c.c, cmrs.c) and kernels
(reference kernels/{Coo,Csr,Ell,Sigma_C,Cmrs}.cl).
"""
from __future__ import annotations

import ctypes
import os
import sys
from dataclasses import dataclass, field
from pathlib import Path

import numpy as np

PKG_DIR = Path(__file__).resolve().parent
LIB_DIR = PKG_DIR / "lib"
REPO_DIR = PKG_DIR.parent

FORMATS = ("coo", "csr", "ell", "sell", "cmrs")  # the reference's five
# §8f row 4: CSR with 16-bit column offsets; ELL + COO tail; CSR with fp32 values;
# SELL-C-σ with 16-bit column offsets; column-grouped CSR (gather-bound rows)
EXTRA_FORMATS = ("csr16", "hyb", "csrf32", "sell16", "csrg")
ALL_FORMATS = FORMATS + EXTRA_FORMATS
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)

# The reference's ReturnCode values (reference inc/enums.h:4-11).
SUCCESS, DEVICE_ERROR, PROGRAM_ERROR, FILE_ERROR, OTHER_ERROR = range(5)


class SpmvError(RuntimeError):
    """A C-ABI call returned a non-zero spmv_rc code."""

    def __init__(self, rc: int, what: str, detail: str = ""):
        super().__init__(f"{what} failed: rc={rc} {detail}".strip())
        self.rc = rc


# --------------------------------------------------------------- loading
_c_i64 = ctypes.c_int64
_c_i32 = ctypes.c_int32
_vp = ctypes.c_void_p


class Dims(ctypes.Structure):
    """``spmv_dims`` (include/spmv.h)."""

    _fields_ = [
        ("n_rows", _c_i64),
        ("n_cols", _c_i64),
        ("nnz", _c_i64),
        ("device", ctypes.c_int),
        ("stream", _vp),
    ]


class MtxInfo(ctypes.Structure):
    """``spmv_mtx_info`` (include/spmv_host.h)."""

    _fields_ = [
        ("n_rows", _c_i64),
        ("n_cols", _c_i64),
        ("nnz", _c_i64),
        ("symmetric", ctypes.c_int),
        ("pattern", ctypes.c_int),
        ("integer", ctypes.c_int),
    ]


class PlanOpts(ctypes.Structure):
    """``spmv_plan_opts`` (include/spmv.h)."""

    _fields_ = [
        ("lanes", _c_i32),
        ("variant", _c_i32),
        ("xwin", _c_i32),
        ("xwin_rows", _c_i32),
        ("head", _c_i32),
        ("index16", _c_i32),
        ("coo_pass", _c_i32),
        ("split", _c_i32),
        ("bigplan", _c_i32),
        ("reserved", _c_i32),
        ("H", _c_i64),
    ]


class PlanInfo(ctypes.Structure):
    """``spmv_plan_info`` (include/spmv.h)."""

    _fields_ = [(k, _c_i32) for k in ("format", "path", "lanes", "variant", "ki", "xcap", "xwin", "head", "single_pass",
                                      "index16", "split_T", "reserved")] + \
               [(k, _c_i64) for k in ("n_chunks", "big_tiles", "head_bytes", "ws_bytes", "owned_bytes", "H")] + \
               [("kernel", ctypes.c_char * 64), ("desc", ctypes.c_char * 320)]


_PP = ctypes.POINTER(_vp)
_PO = ctypes.POINTER(PlanOpts)

# name -> (restype, argtypes)
HIP_SYMBOLS = {
    "spmv_plan_opts_init": (None, [_PO]),
    "spmv_plan_coo": (ctypes.c_int, [Dims, _vp, _vp, _vp, _PO, _PP]),
    "spmv_plan_csr": (ctypes.c_int, [Dims, _vp, _vp, _vp, _PO, _PP]),
    "spmv_plan_ell": (ctypes.c_int, [Dims, _c_i32, _c_i64, _c_i32, _vp, _vp, _PO, _PP]),
    "spmv_plan_sell": (ctypes.c_int, [Dims, _c_i32, _c_i32, _c_i32, _c_i64, _vp, _vp, _vp, _vp, _PO, _PP]),
    "spmv_plan_cmrs": (ctypes.c_int, [Dims, _c_i32, _c_i64, _vp, _vp, _vp, _vp, _PO, _PP]),
    "spmv_plan_run": (ctypes.c_int, [_vp, _vp, _vp, _vp]),
    "spmv_plan_get_info": (ctypes.c_int, [_vp, ctypes.POINTER(PlanInfo)]),
    "spmv_plan_destroy": (ctypes.c_int, [_vp]),
    "spmv_set_option": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    "spmv_get_option": (ctypes.c_int, [ctypes.c_int]),
    "spmv_coo_ws_bytes": (ctypes.c_size_t, [_c_i64]),
    "spmv_coo_run": (ctypes.c_int, [Dims, _vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_size_t]),
    "spmv_coo_tail_bytes": (ctypes.c_size_t, [_c_i64]),
    "spmv_coo_tail_build": (ctypes.c_int, [Dims, _vp, _vp, ctypes.c_size_t]),
    "spmv_coo_run_tail": (ctypes.c_int, [Dims, _vp, _vp, _vp, _vp, _vp, _vp]),
    "spmv_csr_auto_lanes": (ctypes.c_int, [_c_i64, _c_i64]),
    "spmv_csr_run": (ctypes.c_int, [Dims, _vp, _vp, _vp, _vp, _vp, ctypes.c_int]),
    "spmv_csr_run_variant": (ctypes.c_int, [Dims, _vp, _vp, _vp, _vp, _vp, ctypes.c_int, ctypes.c_int]),
    "spmv_csr_tiled_ws_bytes": (ctypes.c_size_t, [_c_i64, _c_i64]),
    "spmv_csr_run_tiled": (ctypes.c_int, [Dims, _vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_size_t]),
    "spmv_csr_hot_ws_bytes": (ctypes.c_size_t, [_c_i64, _c_i64, _c_i64]),
    "spmv_csr_f32v_run_xwin": (ctypes.c_int, [Dims, _vp, _vp, _vp, _vp, _vp, ctypes.c_int, _c_i32, _vp, _c_i32]),
    "spmv_csr_f32v_run_tiled_hot": (ctypes.c_int, [Dims, _vp, _vp, _vp, _vp, _vp, _c_i64, _vp, _vp, _vp,
                                                   ctypes.c_size_t]),
    "spmv_csr_run_tiled_hot": (ctypes.c_int, [Dims, _vp, _vp, _vp, _vp, _vp, _c_i64, _vp, _vp, _vp,
                                              ctypes.c_size_t]),
    "spmv_csr_tiled_plan_len": (_c_i64, [_c_i64]),
    "spmv_csr_tiled_plan": (ctypes.c_int, [Dims, _vp, _vp]),
    "spmv_csr_tiled_tile": (_c_i64, [_c_i64, _c_i64]),
    "spmv_csr_run_tiled_plan": (ctypes.c_int, [Dims, _vp, _vp, _vp, _vp, _vp, _c_i64, _vp, _vp, _vp, _c_i64,
                                               _c_i64, _vp, ctypes.c_size_t]),
    "spmv_csrg_ws_bytes": (ctypes.c_size_t, [_c_i64, _c_i64]),
    "spmv_csrg_run": (ctypes.c_int, [Dims, _c_i32, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                     ctypes.c_size_t]),
    "spmv_csr16_run": (ctypes.c_int, [Dims, _vp, _vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_int]),
    "spmv_csr16_run_xwin": (ctypes.c_int, [Dims, _vp, _vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_int, _c_i32, _vp,
                                           _c_i32]),
    "spmv_hyb_ws_bytes": (ctypes.c_size_t, [_c_i64]),
    "spmv_hyb_run": (ctypes.c_int, [Dims, _c_i32, _c_i64, _c_i32, _vp, _vp, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp,
                                    ctypes.c_size_t]),
    "spmv_hyb_run_tail": (ctypes.c_int, [Dims, _c_i32, _c_i64, _c_i32, _vp, _vp, _c_i64, _vp, _vp, _vp, _vp, _vp,
                                         _vp]),
    "spmv_hyb_run_tail_xwin": (ctypes.c_int, [Dims, _c_i32, _c_i64, _c_i32, _vp, _vp, _c_i64, _vp, _vp, _vp, _vp,
                                              _vp, _vp, _vp, _c_i32]),
    "spmv_csr_xwin_bytes": (ctypes.c_size_t, [_c_i64, _c_i64, ctypes.c_int, _c_i32]),
    "spmv_csr_xwin_build": (ctypes.c_int, [Dims, _vp, _vp, ctypes.c_int, _c_i32, _vp, ctypes.c_size_t,
                                           ctypes.POINTER(_c_i32)]),
    "spmv_csr_run_xwin": (ctypes.c_int, [Dims, _vp, _vp, _vp, _vp, _vp, ctypes.c_int, _c_i32, _vp, _c_i32]),
    "spmv_ell_run": (ctypes.c_int, [Dims, _c_i32, _c_i64, _c_i32, _vp, _vp, _vp, _vp]),
    "spmv_ell_xwin_bytes": (ctypes.c_size_t, [_c_i64]),
    "spmv_ell_xwin_build": (ctypes.c_int, [Dims, _c_i32, _c_i64, _c_i32, _vp, _vp, ctypes.c_size_t,
                                           ctypes.POINTER(_c_i32)]),
    "spmv_ell_run_xwin": (ctypes.c_int, [Dims, _c_i32, _c_i64, _c_i32, _vp, _vp, _vp, _vp, _vp, _c_i32]),
    "spmv_sell_xwin_bytes": (ctypes.c_size_t, [_c_i64, _c_i32, _c_i32]),
    "spmv_sell_auto_ki": (ctypes.c_int, [_c_i64, _c_i32]),
    "spmv_sell_xwin_build": (ctypes.c_int, [Dims, _c_i32, _c_i32, _c_i64, _vp, _vp, _vp, ctypes.c_size_t,
                                            ctypes.POINTER(_c_i32)]),
    "spmv_sell_run_xwin": (ctypes.c_int, [Dims, _c_i32, _c_i32, _c_i32, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp,
                                          _vp, _c_i32]),
    "spmv_sell_run": (ctypes.c_int, [Dims, _c_i32, _c_i32, _c_i32, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp]),
    "spmv_sell16_fill": (ctypes.c_int, [Dims, _c_i32, _c_i32, _c_i64, _vp, _vp, _vp, _vp]),
    "spmv_sell16_run": (ctypes.c_int, [Dims, _c_i32, _c_i32, _c_i32, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                       _c_i32, _vp]),
    "spmv_sell16_head_bytes": (ctypes.c_size_t, [_c_i64, _c_i32, _c_i32]),
    "spmv_sell_head_bytes": (ctypes.c_size_t, [_c_i64, _c_i32, _c_i32]),
    "spmv_sell_head_fill": (ctypes.c_int, [Dims, _c_i32, _c_i32, _c_i32, _c_i64, _vp, _vp, _vp, _vp,
                                           ctypes.c_size_t]),
    "spmv_sell_run_xwin_head": (ctypes.c_int, [Dims, _c_i32, _c_i32, _c_i32, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp,
                                               _vp, _c_i32, _vp]),
    "spmv_sell16_head_fill": (ctypes.c_int, [Dims, _c_i32, _c_i32, _c_i32, _c_i64, _vp, _vp, _vp, _vp,
                                             ctypes.c_size_t]),
    "spmv_cmrs_run": (ctypes.c_int, [Dims, _c_i32, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp]),
    "spmv_coo_xwin_bytes": (ctypes.c_size_t, [_c_i64]),
    "spmv_coo_xwin_build": (ctypes.c_int, [Dims, _vp, _vp, ctypes.c_size_t, ctypes.POINTER(_c_i32)]),
    "spmv_coo_run_xwin": (ctypes.c_int, [Dims, _vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_size_t, _vp, _c_i32]),
    "spmv_cmrs_xwin_bytes": (ctypes.c_size_t, [Dims, _c_i32, _c_i64]),
    "spmv_cmrs_xwin_build": (ctypes.c_int, [Dims, _c_i32, _c_i64, _vp, _vp, _vp, ctypes.c_size_t,
                                            ctypes.POINTER(_c_i32)]),
    "spmv_cmrs_run_xwin": (ctypes.c_int, [Dims, _c_i32, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _c_i32]),
    "spmv_coo_hot_ws_bytes": (ctypes.c_size_t, [_c_i64, _c_i64]),
    "spmv_coo_run_hot": (ctypes.c_int, [Dims, _vp, _vp, _vp, _vp, _vp, _c_i64, _vp, _vp, ctypes.c_size_t]),
    "spmv_cmrs_hot_ws_bytes": (ctypes.c_size_t, [_c_i64, _c_i64, _c_i32, _c_i64]),
    "spmv_cmrs_run_tiled_hot": (ctypes.c_int, [Dims, _c_i32, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp, _c_i64, _vp, _vp,
                                               ctypes.c_size_t]),
    "spmv_cmrs_tiled_ws_bytes": (ctypes.c_size_t, [_c_i64, _c_i64, _c_i32]),
    "spmv_cmrs_run_tiled": (ctypes.c_int, [Dims, _c_i32, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_size_t]),
    "spmv_sell_split_ws_bytes": (ctypes.c_size_t, [_c_i64, _c_i32]),
    "spmv_sell_hot_ws_bytes": (ctypes.c_size_t, [_c_i64, _c_i32, _c_i64]),
    "spmv_hyb_hot_ws_bytes": (ctypes.c_size_t, [_c_i64, _c_i64]),
    "spmv_hyb_run_hot": (ctypes.c_int, [Dims, _c_i32, _c_i64, _c_i32, _vp, _vp, _c_i64, _vp, _vp, _vp, _vp, _vp,
                                        _c_i64, _vp, _vp, ctypes.c_size_t]),
    "spmv_sell_run_hot": (ctypes.c_int, [Dims, _c_i32, _c_i32, _c_i32, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp, _c_i32,
                                         _c_i64, _vp, _vp, _c_i64, _vp, _vp, ctypes.c_size_t]),
    "spmv_sell_run_split": (ctypes.c_int, [Dims, _c_i32, _c_i32, _c_i32, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                           _c_i32, _c_i32, _c_i64, _vp, _vp, _vp, ctypes.c_size_t]),
    "spmv_gen_banded_device": (ctypes.c_int, [_c_i64, ctypes.c_uint64, _c_i64, _c_i64, ctypes.c_int, _c_i32,
                                              _c_i32, _vp, _vp, _vp, _vp, ctypes.c_int, _vp]),
    "spmv_dev_csr_from_coo": (ctypes.c_int, [Dims, _vp, _vp, _vp, _vp, _vp, _vp]),
    "spmv_dev_ell_plan": (ctypes.c_int, [Dims, _vp, _c_i32, ctypes.POINTER(_c_i32), ctypes.POINTER(_c_i64)]),
    "spmv_dev_ell_fill": (ctypes.c_int, [Dims, _vp, _vp, _vp, _c_i32, _c_i64, _c_i32, _vp, _vp]),
    "spmv_dev_sell_plan": (ctypes.c_int, [Dims, _vp, _vp, _c_i32, _c_i32, _c_i32, _c_i64, _vp, _vp, _vp,
                                          ctypes.POINTER(_c_i64)]),
    "spmv_dev_sell_fill": (ctypes.c_int, [Dims, _vp, _vp, _vp, _c_i32, _c_i32, _c_i64, _vp, _vp, _vp, _vp, _vp]),
    "spmv_dev_cmrs_build": (ctypes.c_int, [Dims, _vp, _c_i32, _vp, _vp]),
    "spmv_dot_ws_bytes": (ctypes.c_size_t, [_c_i64]),
    "spmv_dot": (ctypes.c_int, [_c_i64, _vp, _vp, _vp, _vp, ctypes.c_size_t, ctypes.c_int, _vp]),
    "spmv_axpy_ratio": (ctypes.c_int, [_c_i64, _vp, _vp, ctypes.c_double, _vp, _vp, ctypes.c_int, _vp]),
    "spmv_xpay_ratio": (ctypes.c_int, [_c_i64, _vp, _vp, _vp, _vp, ctypes.c_int, _vp]),
    "spmv_scale_rsqrt": (ctypes.c_int, [_c_i64, _vp, _vp, _vp, ctypes.c_int, _vp]),
    "spmv_gather": (ctypes.c_int, [_c_i64, _vp, _vp, _vp, ctypes.c_int, _vp]),
    "spmv_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "spmv_set_device": (ctypes.c_int, [ctypes.c_int]),
    "spmv_device_name": (ctypes.c_int, [ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t]),
    "spmv_malloc": (ctypes.c_int, [ctypes.POINTER(_vp), ctypes.c_size_t]),
    "spmv_free": (ctypes.c_int, [_vp]),
    "spmv_memset": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_size_t, _vp]),
    "spmv_upload": (ctypes.c_int, [_vp, _vp, ctypes.c_size_t, _vp]),
    "spmv_download": (ctypes.c_int, [_vp, _vp, ctypes.c_size_t, _vp]),
    "spmv_stream_create": (ctypes.c_int, [ctypes.POINTER(_vp)]),
    "spmv_stream_destroy": (ctypes.c_int, [_vp]),
    "spmv_sync": (ctypes.c_int, [_vp]),
    "spmv_flush_cache": (ctypes.c_int, [_vp, ctypes.c_size_t]),
    "spmv_flush_cache_read": (ctypes.c_int, [_vp, ctypes.c_size_t]),
    "spmv_event_create": (ctypes.c_int, [ctypes.POINTER(_vp)]),
    "spmv_event_destroy": (ctypes.c_int, [_vp]),
    "spmv_event_record": (ctypes.c_int, [_vp, _vp]),
    "spmv_event_elapsed": (ctypes.c_int, [_vp, _vp, ctypes.POINTER(ctypes.c_double)]),
    "spmv_time_launch": (ctypes.c_int, [_vp, _vp, _vp, ctypes.POINTER(ctypes.c_double)]),
    "spmv_release": (ctypes.c_int, []),
    "spmv_multi_init": (ctypes.c_int, [ctypes.c_int, _vp, _vp]),
    "spmv_multi_free": (ctypes.c_int, [_vp]),
    "spmv_multi_size": (ctypes.c_int, [_vp]),
    "spmv_multi_device": (ctypes.c_int, [_vp, ctypes.c_int]),
    "spmv_multi_stream": (_vp, [_vp, ctypes.c_int]),
    "spmv_multi_allgatherv": (ctypes.c_int, [_vp, _vp, _vp]),
    "spmv_multi_sync": (ctypes.c_int, [_vp]),
    "spmv_multi_time": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_int, _vp]),
    "spmv_strerror": (ctypes.c_char_p, [ctypes.c_int]),
    "spmv_last_error": (ctypes.c_char_p, []),
    "spmv_version": (ctypes.c_char_p, []),
}

HOST_SYMBOLS = {
    "spmv_mtx_read_info": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(MtxInfo)]),
    "spmv_mtx_read": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(MtxInfo), _vp, _vp, _vp]),
    "spmv_mtx_write": (ctypes.c_int, [ctypes.c_char_p, _c_i64, _c_i64, _c_i64, _vp, _vp, _vp, ctypes.c_int]),
    "spmv_bin_write": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(MtxInfo), _vp, _vp, _vp]),
    "spmv_bin_read_info": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(MtxInfo)]),
    "spmv_bin_read": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(MtxInfo), _vp, _vp, _vp]),
    "spmv_coo_sort_by_row": (ctypes.c_int, [_c_i64, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp]),
    "spmv_csr_from_coo": (ctypes.c_int, [_c_i64, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp]),
    "spmv_csr_sort_rows": (ctypes.c_int, [_c_i64, _vp, _vp, _vp]),
    "spmv_csr_row_stats": (ctypes.c_int, [_c_i64, _vp, ctypes.POINTER(_c_i64), ctypes.POINTER(_c_i64), ctypes.POINTER(ctypes.c_double)]),
    "spmv_csr_pick_variant": (ctypes.c_int, [_c_i64, _vp]),
    "spmv_csr_variant_rule": (ctypes.c_int, [_c_i64, _c_i64, _c_i64]),
    "spmv_cmrs_variant_rule": (ctypes.c_int, [_c_i64, _c_i64, _c_i64]),
    "spmv_hot_columns_possible": (ctypes.c_int, [_c_i64, _c_i64]),
    "spmv_hot_columns": (_c_i64, [_c_i64, _c_i64, _vp, _c_i64, _vp, _vp]),
    "spmv_column_relabel": (_c_i64, [_c_i64, _c_i64, _vp, _vp, _vp, _vp]),
    "spmv_column_relabel_ex": (_c_i64, [_c_i64, _c_i64, _vp, _vp, _vp, _vp, _c_i32]),
    "spmv_csr_tiled_bigplan": (_c_i64, [_c_i64, _vp, _c_i64, _c_i32, _vp]),
    "spmv_ell_plan": (ctypes.c_int, [_c_i64, _vp, _c_i32, ctypes.POINTER(_c_i32), ctypes.POINTER(_c_i64)]),
    "spmv_ell_fill": (ctypes.c_int, [_c_i64, _vp, _vp, _vp, _c_i32, _c_i64, _c_i32, _vp, _vp]),
    "spmv_sell_plan": (ctypes.c_int, [_c_i64, _vp, _c_i32, _c_i32, _c_i32, ctypes.POINTER(_c_i64), ctypes.POINTER(_c_i64)]),
    "spmv_sell_fill": (ctypes.c_int, [_c_i64, _vp, _vp, _vp, _c_i32, _c_i32, _c_i32, _c_i64, _vp, _vp, _vp, _vp]),
    "spmv_cmrs_build": (ctypes.c_int, [_c_i64, _vp, _c_i32, _vp, _vp]),
    "spmv_cmrs_pick_variant": (ctypes.c_int, [_c_i64, _vp]),
    "spmv_sell_split_auto": (_c_i32, [_c_i64, _vp, _c_i32, _c_i32]),
    "spmv_sell_split_plan": (_c_i64, [_c_i64, _vp, _c_i32, _c_i32, _vp, _vp]),
    "spmv_partition_rows": (ctypes.c_int, [_c_i64, _vp, ctypes.c_int, _c_i64, _vp]),
    "spmv_coo_row_shard": (_c_i64, [_c_i64, _vp, _vp, _vp, _c_i64, _c_i64, _vp, _vp, _vp]),
    "spmv_partition_rows_weighted": (ctypes.c_int, [_c_i64, _vp, ctypes.c_int, _c_i64, ctypes.c_double, _vp]),
    "spmv_partition_rows_calibrated": (ctypes.c_int, [_c_i64, _vp, ctypes.c_int, _c_i64, ctypes.c_double, ctypes.c_int,
                                                      _vp, _vp, _vp]),
    "spmv_csr16_plan": (ctypes.c_int, [_c_i64, _vp, ctypes.POINTER(_c_i64), ctypes.POINTER(_c_i64)]),
    "spmv_hyb_plan": (ctypes.c_int, [_c_i64, _vp, _c_i32, _c_i32, ctypes.POINTER(_c_i32), ctypes.POINTER(_c_i64),
                                     ctypes.POINTER(_c_i64)]),
    "spmv_hyb_fill": (ctypes.c_int, [_c_i64, _vp, _vp, _vp, _c_i32, _c_i64, _c_i32, _vp, _vp, _vp, _vp, _vp]),
    "spmv_csr16_fill": (ctypes.c_int, [_c_i64, _vp, _vp, _vp, _vp]),
    "spmv_csrg_group": (_c_i32, [_c_i32, _c_i32]),
    "spmv_csrg_block_rows": (_c_i32, []),
    "spmv_csrg_plan": (ctypes.c_int, [_c_i64, _vp, _vp, _c_i32, ctypes.POINTER(_c_i64)]),
    "spmv_csrg_fill": (ctypes.c_int, [_c_i64, _vp, _vp, _vp, _c_i32, _vp, _vp, _vp, _vp, _vp]),
    "spmv_cpu_coo": (ctypes.c_int, [_c_i64, _c_i64, _vp, _vp, _vp, _vp, _vp, ctypes.c_int]),
    "spmv_cpu_csr": (ctypes.c_int, [_c_i64, _vp, _vp, _vp, _vp, _vp, ctypes.c_int]),
    "spmv_cpu_ell": (ctypes.c_int, [_c_i64, _c_i32, _c_i64, _c_i32, _vp, _vp, _vp, _vp, ctypes.c_int]),
    "spmv_cpu_sell": (ctypes.c_int, [_c_i64, _c_i32, _c_i32, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_int]),
    "spmv_cpu_cmrs": (ctypes.c_int, [_c_i64, _c_i32, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_int]),
    "spmv_cpu_threads": (ctypes.c_int, []),
    "spmv_check": (_c_i64, [_c_i64, _c_i64, _vp, _vp, _vp, _vp, _vp, ctypes.c_double, ctypes.c_double, ctypes.POINTER(_c_i64), ctypes.POINTER(ctypes.c_double)]),
    "spmv_gen_cantlike": (ctypes.c_int, [ctypes.c_int, _c_i64, ctypes.POINTER(_c_i64), ctypes.POINTER(_c_i64), _vp, _vp, _vp]),
    "spmv_gen_rmat": (ctypes.c_int, [_c_i64, _c_i64, ctypes.c_int, ctypes.c_uint64, _vp, _vp, _vp]),
    "spmv_gen_banded_csr": (ctypes.c_int, [_c_i64, ctypes.c_uint64, _c_i64, _c_i64, _vp, _vp, _vp]),
    "spmv_gen_random": (ctypes.c_int, [_c_i64, _c_i64, _c_i64, _c_i64, ctypes.c_uint64, ctypes.POINTER(_c_i64), _vp, _vp, _vp]),
    "spmv_splitmix64": (ctypes.c_uint64, [ctypes.c_uint64, ctypes.c_uint64]),
}

_LAUNCH_FN = ctypes.CFUNCTYPE(ctypes.c_int, _vp)

_hip = None
_host = None


def _bind(lib: ctypes.CDLL, table: dict) -> ctypes.CDLL:
    for name, (res, args) in table.items():
        fn = getattr(lib, name)  # AttributeError = symbol missing: loud
        fn.restype = res
        fn.argtypes = args
    return lib


def hip_lib() -> ctypes.CDLL:
    """libspmv_hip.so — raises if it was not built (no CPU fallback)."""
    global _hip
    if _hip is None:
        host_lib()  # its plans call the host rules: loaded first (RTLD_GLOBAL, soname libspmv_host.so)
        path = Path(os.environ.get("SPMV_HIP_LIB") or LIB_DIR / "libspmv_hip.so")  # override: A/B runs
        if not path.exists():
            raise SpmvError(PROGRAM_ERROR, "load libspmv_hip.so", f"{path} missing: run `make lib`")
        _hip = _bind(ctypes.CDLL(str(path), mode=ctypes.RTLD_GLOBAL), HIP_SYMBOLS)
    return _hip


def host_lib() -> ctypes.CDLL:
    global _host
    if _host is None:
        path = Path(os.environ.get("SPMV_HOST_LIB", LIB_DIR / "libspmv_host.so"))  # `make test-san` build
        if not path.exists():
            raise SpmvError(PROGRAM_ERROR, "load libspmv_host.so", f"{path} missing: run `make lib`")
        _host = _bind(ctypes.CDLL(str(path), mode=ctypes.RTLD_GLOBAL), HOST_SYMBOLS)
    return _host


def _ptr(a) -> int | None:
    """Raw address of a numpy array or torch tensor (None for empty)."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return a.data_ptr()


def _check(rc: int, what: str) -> None:
    if rc != SUCCESS:
        detail = hip_lib().spmv_last_error().decode() if _hip is not None else ""
        raise SpmvError(rc, what, detail)


# --------------------------------------------------------- host: inputs
@dataclass
class Coo:
    """Entries in FILE order (the order check_result accumulates in)."""

    n_rows: int
    n_cols: int
    row: np.ndarray
    col: np.ndarray
    val: np.ndarray
    symmetric: bool = False
    label: str = ""

    @property
    def nnz(self) -> int:
        return int(self.row.shape[0])


def read_mtx(path: str | os.PathLike) -> Coo:
    """Matrix Market reader with the reference's acceptance rules
    (reference inc/helper_functions.h:134-165, csr.c:77-91)."""
    lib = host_lib()
    info = MtxInfo()
    p = str(path).encode()
    rc = lib.spmv_mtx_read_info(p, ctypes.byref(info))
    if rc != SUCCESS:
        raise SpmvError(rc, f"read {path}")
    z = info.nnz
    row = np.empty(z, np.int32)
    col = np.empty(z, np.int32)
    val = np.empty(z, np.float64)
    _check_host(lib.spmv_mtx_read(p, ctypes.byref(info), _ptr(row), _ptr(col), _ptr(val)), f"read {path}")
    return Coo(info.n_rows, info.n_cols, row, col, val, bool(info.symmetric), str(path))


def _check_host(rc: int, what: str) -> None:
    if rc != SUCCESS:
        raise SpmvError(rc, what)


def write_mtx(path, m: Coo) -> None:
    _check_host(host_lib().spmv_mtx_write(str(path).encode(), m.n_rows, m.n_cols, m.nnz,
                                          _ptr(m.row), _ptr(m.col), _ptr(m.val), int(m.symmetric)),
                f"write {path}")


def gen_cantlike(mode: int = 0, copies: int = 1) -> Coo:
    """cant-like stand-in (include/spmv_host.h: spmv_gen_cantlike)."""
    lib = host_lib()
    n = _c_i64()
    z = _c_i64()
    _check_host(lib.spmv_gen_cantlike(mode, copies, ctypes.byref(n), ctypes.byref(z), None, None, None), "gen_cantlike")
    row = np.empty(z.value, np.int32)
    col = np.empty(z.value, np.int32)
    val = np.empty(z.value, np.float64)
    _check_host(lib.spmv_gen_cantlike(mode, copies, ctypes.byref(n), ctypes.byref(z), _ptr(row), _ptr(col), _ptr(val)), "gen_cantlike")
    label = f"cant-like stand-in (synthetic, mode {mode}, x{copies})"
    return Coo(n.value, n.value, row, col, val, mode == 2, label)


def gen_rmat(n: int = 10_000_000, nnz: int = 100_000_000, scale: int = 24, seed: int = 1) -> Coo:
    lib = host_lib()
    row = np.empty(nnz, np.int32)
    col = np.empty(nnz, np.int32)
    val = np.empty(nnz, np.float64)
    _check_host(lib.spmv_gen_rmat(n, nnz, scale, seed, _ptr(row), _ptr(col), _ptr(val)), "gen_rmat")
    return Coo(n, n, row, col, val, False, f"R-MAT {n} rows {nnz} entries (synthetic)")


def gen_random(n_rows: int, n_cols: int, min_len: int, max_len: int, seed: int = 1) -> Coo:
    lib = host_lib()
    z = _c_i64()
    _check_host(lib.spmv_gen_random(n_rows, n_cols, min_len, max_len, seed, ctypes.byref(z), None, None, None), "gen_random")
    row = np.empty(z.value, np.int32)
    col = np.empty(z.value, np.int32)
    val = np.empty(z.value, np.float64)
    _check_host(lib.spmv_gen_random(n_rows, n_cols, min_len, max_len, seed, ctypes.byref(z), _ptr(row), _ptr(col), _ptr(val)), "gen_random")
    return Coo(n_rows, n_cols, row, col, val, False, f"random {n_rows}x{n_cols} len {min_len}..{max_len}")


def gen_banded_csr(n: int, row_begin: int = 0, row_end: int | None = None, seed: int = 2):
    """Banded rows [row_begin,row_end) in CSR form (local row_ptr)."""
    row_end = n if row_end is None else row_end
    m = row_end - row_begin
    ptr = np.empty(m + 1, np.int64)
    col = np.empty(16 * m, np.int32)
    val = np.empty(16 * m, np.float64)
    _check_host(host_lib().spmv_gen_banded_csr(n, seed, row_begin, row_end, _ptr(ptr), _ptr(col), _ptr(val)), "gen_banded")
    return ptr, col, val


def ramp_x(n_cols: int) -> np.ndarray:
    """x[j] = j, the reference's input vector (reference csr.c:95-99)."""
    return np.arange(n_cols, dtype=np.float64)


# ------------------------------------------------------- host: formats
def csr_from_coo(m: Coo):
    ptr = np.empty(m.n_rows + 1, np.int64)
    col = np.empty(m.nnz, np.int32)
    val = np.empty(m.nnz, np.float64)
    _check_host(host_lib().spmv_csr_from_coo(m.n_rows, m.nnz, _ptr(m.row), _ptr(m.col), _ptr(m.val),
                                             _ptr(ptr), _ptr(col), _ptr(val)), "csr_from_coo")
    return ptr, col, val


def csr_sort_rows(n_rows: int, ptr, col, val) -> None:
    """Sort every row's entries by column, in place (spmv_csr_sort_rows)."""
    _check_host(host_lib().spmv_csr_sort_rows(n_rows, _ptr(ptr), _ptr(col), _ptr(val)), "csr_sort_rows")


def coo_sort_by_row(m: Coo):
    row = np.empty(m.nnz, np.int32)
    col = np.empty(m.nnz, np.int32)
    val = np.empty(m.nnz, np.float64)
    _check_host(host_lib().spmv_coo_sort_by_row(m.n_rows, m.nnz, _ptr(m.row), _ptr(m.col), _ptr(m.val),
                                                _ptr(row), _ptr(col), _ptr(val)), "coo_sort_by_row")
    return row, col, val


def row_stats(n_rows: int, ptr: np.ndarray):
    mn, mx, mean = _c_i64(), _c_i64(), ctypes.c_double()
    host_lib().spmv_csr_row_stats(n_rows, _ptr(ptr), ctypes.byref(mn), ctypes.byref(mx), ctypes.byref(mean))
    return mn.value, mx.value, mean.value


def ell_build(n_rows: int, ptr, col, val, ki: int = 2, max_padding: float | None = None):
    lib = host_lib()
    K, ld = _c_i32(), _c_i64()
    _check_host(lib.spmv_ell_plan(n_rows, _ptr(ptr), ki, ctypes.byref(K), ctypes.byref(ld)), "ell_plan")
    stored = K.value * ld.value
    nnz = int(ptr[-1]) if n_rows > 0 else 0
    if max_padding is not None and nnz > 0 and stored / nnz > max_padding:
        raise SpmvError(OTHER_ERROR, "ell_build", f"padding factor {stored / nnz:.1f} > {max_padding}")
    ecol = np.empty(max(stored, 1), np.int32)
    evalv = np.empty(max(stored, 1), np.float64)
    _check_host(lib.spmv_ell_fill(n_rows, _ptr(ptr), _ptr(col), _ptr(val), K.value, ld.value, ki,
                                  _ptr(ecol), _ptr(evalv)), "ell_fill")
    return dict(K=K.value, ld=ld.value, ki=ki, col=ecol, val=evalv, stored=stored)


def sell_build(n_rows: int, ptr, col, val, C: int = 64, sigma: int = 1024, ki: int = 2):
    lib = host_lib()
    ns, stored = _c_i64(), _c_i64()
    _check_host(lib.spmv_sell_plan(n_rows, _ptr(ptr), C, sigma, ki, ctypes.byref(ns), ctypes.byref(stored)), "sell_plan")
    sp = np.empty(ns.value + 1, np.int64)
    perm = np.empty(max(ns.value * C, 1), np.int32)
    scol = np.empty(max(stored.value, 1), np.int32)
    sval = np.empty(max(stored.value, 1), np.float64)
    _check_host(lib.spmv_sell_fill(n_rows, _ptr(ptr), _ptr(col), _ptr(val), C, sigma, ki, ns.value,
                                   _ptr(sp), _ptr(perm), _ptr(scol), _ptr(sval)), "sell_fill")
    return dict(C=C, sigma=sigma, ki=ki, n_slices=ns.value, slice_ptr=sp, perm=perm, col=scol,
                val=sval, stored=stored.value)


def sell_split_plan(s: dict, T: int | None = None):
    """Wide-slice split plan of a sell_build result: (T, chunk_slice,
    chunk_k0); T None = the library rule (0: no split)."""
    hl = host_lib()
    sp = np.ascontiguousarray(s["slice_ptr"], dtype=np.int64)
    if T is None:
        T = hl.spmv_sell_split_auto(s["n_slices"], _ptr(sp), s["C"], s["ki"])
    if T <= 0:
        return 0, np.zeros(0, np.int32), np.zeros(0, np.int32)
    n = hl.spmv_sell_split_plan(s["n_slices"], _ptr(sp), s["C"], T, None, None)
    if n < 0:
        raise SpmvError(OTHER_ERROR, "spmv_sell_split_plan", "bad plan arguments")
    cs, ck = np.zeros(max(n, 1), np.int32), np.zeros(max(n, 1), np.int32)
    hl.spmv_sell_split_plan(s["n_slices"], _ptr(sp), s["C"], T, _ptr(cs), _ptr(ck))
    return T, cs[:n], ck[:n]


def hot_columns(n_cols: int, col, H: int = 0):
    """spmv_hot_columns: (H, hot[H], col_hot) — the H most frequent columns
    and col with them renumbered n_cols + rank (H = 0: the library rule)."""
    col = np.ascontiguousarray(col, dtype=np.int32)
    hot = np.empty(max(H, 1 << 19), np.int32)
    out = np.empty(max(col.size, 1), np.int32)
    n = host_lib().spmv_hot_columns(n_cols, col.size, _ptr(col), H, _ptr(hot), _ptr(out))
    if n < 0:
        raise SpmvError(OTHER_ERROR, "spmv_hot_columns", "bad arguments")
    return int(n), hot[:n].copy(), out[: col.size]


def column_relabel(n_cols: int, col, ties: str = "id"):
    """spmv_column_relabel(_ex): (order, newid, col') — columns ranked by
    decreasing entry count, ties by column id or (ties="first") by first
    appearance in col; x' = x[order] is the input of the relabelled matrix,
    whose y is the original's, row for row."""
    if ties not in ("id", "first"):
        raise SpmvError(OTHER_ERROR, "spmv_column_relabel", f"ties must be 'id' or 'first', not {ties!r}")
    col = np.ascontiguousarray(col, dtype=np.int32)
    order = np.empty(n_cols, np.int32)
    newid = np.empty(n_cols, np.int32)
    out = np.empty(max(col.size, 1), np.int32)
    n = host_lib().spmv_column_relabel_ex(n_cols, col.size, _ptr(col), _ptr(order), _ptr(newid), _ptr(out),
                                          0 if ties == "id" else 1)
    if n < 0:
        raise SpmvError(OTHER_ERROR, "spmv_column_relabel", "bad arguments")
    return order, newid, out[: col.size]


TILED_ROW_CAP = 1024  # rows a tiled-CSR tile stages offsets for (staged.hip kTiledRowCap)


def csr_tiled_bigplan(n_rows: int, ptr: np.ndarray, nnz: int, cap: int = TILED_ROW_CAP):
    """spmv_csr_tiled_bigplan for the tile the library runs this matrix
    with (spmv_csr_tiled_tile): int32 plan, or None when no tile owns more
    than `cap` rows."""
    ptr = np.ascontiguousarray(ptr, dtype=np.int64)
    tile = int(hip_lib().spmv_csr_tiled_tile(n_rows, nnz))
    n = host_lib().spmv_csr_tiled_bigplan(n_rows, _ptr(ptr), tile, cap, None)
    if n < 0:
        raise SpmvError(OTHER_ERROR, "spmv_csr_tiled_bigplan", "bad arguments")
    plan = np.empty(max(n, 1), np.int32)
    host_lib().spmv_csr_tiled_bigplan(n_rows, _ptr(ptr), tile, cap, _ptr(plan))
    tiles = (nnz + tile - 1) // tile
    return plan if tiles > 0 and np.any(plan[:tiles] >= 0) else None


def relabel_columns(m: Coo):
    """(m', order): m with its columns relabelled hot-first (same rows, same
    entry order); run m' on x[order]."""
    order, _, c2 = column_relabel(m.n_cols, m.col)
    return Coo(m.n_rows, m.n_cols, m.row, c2, m.val, False, f"{m.label} (columns relabelled by degree)"), order


def gather_x(order, x, out=None, stream=None):
    """out[k] = x[order[k]] on the device (spmv_gather): the x a
    column-relabelled matrix takes.  order: int32 device tensor."""
    torch = _torch()
    if out is None:
        out = torch.empty(order.numel(), dtype=torch.float64, device=x.device)
    s = stream if stream is not None else torch.cuda.current_stream(x.device)
    _check(hip_lib().spmv_gather(order.numel(), _ptr(order), _ptr(x), _ptr(out), x.device.index or 0, s.cuda_stream),
           "spmv_gather")
    return out


def cmrs_build(n_rows: int, ptr, h: int = 8):
    ns = (n_rows + h - 1) // h
    sp = np.empty(ns + 1, np.int64)
    rin = np.empty(max(int(ptr[-1]), 1), np.uint8)
    _check_host(host_lib().spmv_cmrs_build(n_rows, _ptr(ptr), h, _ptr(sp), _ptr(rin)), "cmrs_build")
    return dict(h=h, n_strips=ns, strip_ptr=sp, row_in_strip=rin)


def hyb_build(n_rows: int, ptr, col, val, ki: int = 2, K: int = 0):
    """ELL part (first K entries per row) + row-sorted COO tail (§8f row 4)."""
    Kc, ld, tail = _c_i32(0), _c_i64(0), _c_i64(0)
    _check_host(host_lib().spmv_hyb_plan(n_rows, _ptr(ptr), ki, K, ctypes.byref(Kc), ctypes.byref(ld),
                                         ctypes.byref(tail)), "hyb_plan")
    stored = Kc.value * ld.value
    ec, ev = np.empty(max(stored, 1), np.int32), np.empty(max(stored, 1), np.float64)
    tr, tc = np.empty(max(tail.value, 1), np.int32), np.empty(max(tail.value, 1), np.int32)
    tv = np.empty(max(tail.value, 1), np.float64)
    _check_host(host_lib().spmv_hyb_fill(n_rows, _ptr(ptr), _ptr(col), _ptr(val), Kc.value, ld.value, ki, _ptr(ec),
                                         _ptr(ev), _ptr(tr), _ptr(tc), _ptr(tv)), "hyb_fill")
    return dict(K=Kc.value, ld=ld.value, ki=ki, stored=stored, tail_nnz=tail.value, ell_col=ec, ell_val=ev,
                tail_row=tr, tail_col=tc, tail_val=tv)


def csr16_build(col: np.ndarray):
    """16-bit column offsets per 64-entry block."""
    nnz = int(col.shape[0])
    nb, ne = _c_i64(0), _c_i64(0)
    _check_host(host_lib().spmv_csr16_plan(nnz, _ptr(col), ctypes.byref(nb), ctypes.byref(ne)), "csr16_plan")
    base = np.empty(max(nb.value, 1), np.int32)
    off = np.empty(max(nnz, 2), np.uint16)
    esc = np.empty(max(ne.value * 64, 1), np.int32)
    _check_host(host_lib().spmv_csr16_fill(nnz, _ptr(col), _ptr(base), _ptr(off), _ptr(esc)), "csr16_fill")
    return dict(n_blocks=nb.value, n_esc=ne.value, blk_base=base, col_off=off, col_esc=esc)


def csrg_build(n_rows: int, ptr, col, val, groups: int = 4):
    """Column-grouped CSR (spmv_host.h spmv_csrg_plan/fill): the entries
    group after group of 128-B x lines, as a CSR over (row, group) pairs,
    plus the per-row-block pair ranges of the reduce."""
    lib = host_lib()
    npairs = _c_i64(0)
    _check_host(lib.spmv_csrg_plan(n_rows, _ptr(ptr), _ptr(col), groups, ctypes.byref(npairs)), "csrg_plan")
    n = npairs.value
    nnz = int(ptr[n_rows])
    rows = int(host_lib().spmv_csrg_block_rows())  # SPMV_CSRG_ROWS as built into the host fill
    nb = (n_rows + rows - 1) // rows
    pair_ptr = np.empty(n + 1, np.int64)
    col_g = np.empty(max(nnz, 1), np.int32)
    val_g = np.empty(max(nnz, 1), np.float64)
    blk_off = np.empty(groups * (nb + 1), np.int32)
    pair_row = np.empty(max(n, 1), np.uint16)
    _check_host(lib.spmv_csrg_fill(n_rows, _ptr(ptr), _ptr(col), _ptr(val), groups, _ptr(pair_ptr), _ptr(col_g),
                                   _ptr(val_g), _ptr(blk_off), _ptr(pair_row)), "csrg_fill")
    return dict(groups=groups, n_pairs=n, nb=nb, pair_ptr=pair_ptr, col_g=col_g, val_g=val_g, blk_off=blk_off,
                pair_row=pair_row)


def partition_rows(n_rows: int, ptr: np.ndarray, parts: int, align: int = 1024,
                   row_weight: float = 0.0) -> np.ndarray:
    """Contiguous row ranges with ~nnz/parts entries each;
    row_weight > 0 balances entries + row_weight per row instead."""
    bounds = np.empty(parts + 1, np.int64)
    ptr = np.ascontiguousarray(ptr, dtype=np.int64)
    if row_weight:
        rc = host_lib().spmv_partition_rows_weighted(n_rows, _ptr(ptr), parts, align, float(row_weight), _ptr(bounds))
    else:
        rc = host_lib().spmv_partition_rows(n_rows, _ptr(ptr), parts, align, _ptr(bounds))
    _check_host(rc, "partition_rows")
    return bounds


def partition_rows_calibrated(n_rows: int, ptr: np.ndarray, parts: int, old_bounds, old_ms, align: int = 1024,
                              row_weight: float = 0.0) -> np.ndarray:
    """Re-cut rows into `parts` ranges of equal measured cost: each row
    costs its old shard's time per (entries + row_weight * rows) unit
    (spmv_partition_rows_calibrated)."""
    bounds = np.empty(parts + 1, np.int64)
    ptr = np.ascontiguousarray(ptr, dtype=np.int64)
    ob = np.ascontiguousarray(old_bounds, dtype=np.int64)
    ms = np.ascontiguousarray(old_ms, dtype=np.float64)
    if ms.size + 1 != ob.size:
        raise SpmvError(OTHER_ERROR, "partition_rows_calibrated", "one time per old shard")
    _check_host(host_lib().spmv_partition_rows_calibrated(n_rows, _ptr(ptr), parts, align, float(row_weight),
                                                          ms.size, _ptr(ob), _ptr(ms), _ptr(bounds)),
                "partition_rows_calibrated")
    return bounds


def partition_rows_damped(n_rows: int, old_bounds, new_bounds, damp: float = 0.5, align: int = 1024) -> np.ndarray:
    """Move every cut point of old_bounds the fraction `damp` of the way to
    new_bounds (aligned, monotone, ends kept).  Cold shard times are not
    linear in a shard's rows and entries (a flushed shard also re-reads x
    and its row offsets), so a full profile-guided re-cut overshoots; half
    steps settle instead."""
    ob = np.asarray(old_bounds, dtype=np.float64)
    nb = np.asarray(new_bounds, dtype=np.float64)
    if ob.shape != nb.shape or ob[0] != 0 or nb[0] != 0 or ob[-1] != n_rows or nb[-1] != n_rows:
        raise SpmvError(OTHER_ERROR, "partition_rows_damped", "bounds must share size and ends")
    b = np.rint((ob + damp * (nb - ob)) / align).astype(np.int64) * align
    b[0], b[-1] = 0, n_rows
    b = np.minimum(np.maximum.accumulate(b), n_rows)
    return b


def shard(m: Coo, lo: int, hi: int) -> Coo:
    """Rows [lo, hi) of m as a local matrix (row ids rebased, columns kept:
    x stays replicated)."""
    sel = (m.row >= lo) & (m.row < hi)
    return Coo(hi - lo, m.n_cols, (m.row[sel] - lo).astype(np.int32), m.col[sel], m.val[sel], m.symmetric,
               f"{m.label} rows [{lo},{hi})")


def bytes_alg(n_rows: int, n_cols: int, nnz: int) -> int:
    """Algorithmic bytes of one SpMV: fp64 values + int32
    columns + int32 row offsets + x read once + y written once."""
    return 12 * nnz + 4 * (n_rows + 1) + 8 * n_cols + 8 * n_rows


def check(m: Coo, x: np.ndarray, y: np.ndarray, rel_tol: float = 1e-6, abs_tol: float = 0.0):
    """Host check_result (reference inc/helper_functions.h:184-236)
    -> (bad_rows, first_bad)."""
    first = _c_i64()
    ref = ctypes.c_double()
    bad = host_lib().spmv_check(m.n_rows, m.nnz, _ptr(m.row), _ptr(m.col), _ptr(m.val), _ptr(x), _ptr(y),
                                abs_tol, rel_tol, ctypes.byref(first), ctypes.byref(ref))
    return int(bad), int(first.value)


# ------------------------------------------------------------- device
def _torch():
    import torch

    return torch


def _dev_tensor(arr: np.ndarray, device):
    torch = _torch()
    return torch.from_numpy(np.ascontiguousarray(arr)).to(device)


@dataclass
class DeviceMatrix:
    """One format resident in HBM, ready for repeated SpMV launches.

    The reference's five formats run through a C plan (spmv_plan_<fmt>,
    include/spmv.h): the library chooses and prepares the kernel path once,
    exactly as ./bin/<fmt> does, and run() is spmv_plan_run.  `arrays`
    holds the format's device arrays (torch tensors, owned here; the plan
    keeps pointers to them), `params` the plan's choices (spmv_plan_info).
    The §8f extra formats (csr16, csrf32, hyb, csrg) call their entry
    points of include/spmv_ext.h directly."""

    fmt: str
    n_rows: int
    n_cols: int
    nnz: int
    device: object
    arrays: dict = field(default_factory=dict)
    params: dict = field(default_factory=dict)
    stored_bytes: int = 0
    plan: object = None  # ctypes.c_void_p of an spmv_plan, or None

    def __del__(self):
        plan, self.plan = self.plan, None
        if plan is not None and _hip is not None and not sys.is_finalizing():
            _hip.spmv_plan_destroy(plan)

    @property
    def bytes_alg(self) -> int:
        return bytes_alg(self.n_rows, self.n_cols, self.nnz)

    @property
    def kernel(self) -> str:
        """The dominant kernel the plan launches (rocprofv3 name, no template args)."""
        return self.params.get("kernel", "")

    def dims(self, stream=None) -> Dims:
        torch = _torch()
        dev = torch.device(self.device)
        if stream is None:
            stream = torch.cuda.current_stream(dev)
        return Dims(self.n_rows, self.n_cols, self.nnz, dev.index or 0, stream.cuda_stream)

    def run(self, x, y, stream=None) -> None:
        """y = A x on `stream` (default: torch's current stream)."""
        lib = hip_lib()
        torch = _torch()
        a = self.arrays
        p = self.params
        if x.dtype != torch.float64 or y.dtype != torch.float64:
            raise SpmvError(OTHER_ERROR, "run", "x and y must be float64")
        if x.numel() < self.n_cols or y.numel() < self.n_rows:
            raise SpmvError(OTHER_ERROR, "run", "x or y too short")
        # raw data_ptr()s go to the C-ABI: a strided view or a tensor on
        # another device would give a wrong y or a GPU fault
        if not (x.is_contiguous() and y.is_contiguous()):
            raise SpmvError(OTHER_ERROR, "run", "x and y must be contiguous")
        here = torch.device(self.device)
        idx = here.index or 0  # the device dims() passes to the C-ABI
        for t in (x, y):
            if t.device.type != here.type or (t.device.index or 0) != idx:
                raise SpmvError(OTHER_ERROR, "run", f"x and y must be on {here.type}:{idx}")
        if self.plan is not None:
            st = stream if stream is not None else torch.cuda.current_stream(here)
            _check(lib.spmv_plan_run(self.plan, _ptr(x), _ptr(y), st.cuda_stream), f"spmv_plan_run ({self.fmt})")
            return
        d = self.dims(stream)
        if self.fmt == "csrf32" and p.get("variant") == 4:
            rc = lib.spmv_csr_f32v_run_tiled_hot(d, _ptr(a["row_ptr"]), _ptr(a["col"]), _ptr(a["val"]), _ptr(x),
                                                 _ptr(y), p["H"], _ptr(a.get("hot")), _ptr(a.get("own_lo")),
                                                 _ptr(a["ws"]), a["ws"].numel())
        elif self.fmt == "csrf32":
            rc = lib.spmv_csr_f32v_run_xwin(d, _ptr(a["row_ptr"]), _ptr(a["col"]), _ptr(a["val"]), _ptr(x), _ptr(y),
                                            p["lanes"], p.get("xwin_rows", 0), _ptr(a["win"]), p["xcap"])
        elif self.fmt == "csr16" and "win" in a:
            rc = lib.spmv_csr16_run_xwin(d, _ptr(a["row_ptr"]), _ptr(a["blk_base"]), _ptr(a["col_off"]),
                                         _ptr(a["col_esc"]), _ptr(a["val"]), _ptr(x), _ptr(y), p["lanes"],
                                         p.get("xwin_rows", 0), _ptr(a["win"]), p["xcap"])
        elif self.fmt == "csr16":
            rc = lib.spmv_csr16_run(d, _ptr(a["row_ptr"]), _ptr(a["blk_base"]), _ptr(a["col_off"]),
                                    _ptr(a["col_esc"]), _ptr(a["val"]), _ptr(x), _ptr(y), p["lanes"])
        elif self.fmt == "hyb" and p.get("H", 0) > 0:
            rc = lib.spmv_hyb_run_hot(d, p["K"], p["ld"], p["ki"], _ptr(a["ell_col"]), _ptr(a["ell_val"]),
                                      p["tail_nnz"], _ptr(a["tail_row"]), _ptr(a["tail_col"]), _ptr(a["tail_val"]),
                                      _ptr(x), _ptr(y), p["H"], _ptr(a["hot"]), _ptr(a["ws"]), a["ws"].numel())
        elif self.fmt == "hyb" and "win" in a:  # single-pass tail, or no tail (K = the longest row)
            rc = lib.spmv_hyb_run_tail_xwin(d, p["K"], p["ld"], p["ki"], _ptr(a["ell_col"]), _ptr(a["ell_val"]),
                                            p["tail_nnz"], _ptr(a["tail_row"]), _ptr(a["tail_col"]),
                                            _ptr(a["tail_val"]), _ptr(x), _ptr(y), _ptr(a.get("tails")),
                                            _ptr(a["win"]), p["xcap"])
        elif self.fmt == "hyb" and "tails" in a:
            rc = lib.spmv_hyb_run_tail(d, p["K"], p["ld"], p["ki"], _ptr(a["ell_col"]), _ptr(a["ell_val"]),
                                       p["tail_nnz"], _ptr(a["tail_row"]), _ptr(a["tail_col"]), _ptr(a["tail_val"]),
                                       _ptr(x), _ptr(y), _ptr(a["tails"]))
        elif self.fmt == "hyb":
            rc = lib.spmv_hyb_run(d, p["K"], p["ld"], p["ki"], _ptr(a["ell_col"]), _ptr(a["ell_val"]), p["tail_nnz"],
                                  _ptr(a["tail_row"]), _ptr(a["tail_col"]), _ptr(a["tail_val"]), _ptr(x), _ptr(y),
                                  _ptr(a["ws"]), a["ws"].numel())
        elif self.fmt == "csrg":
            rc = lib.spmv_csrg_run(d, p["groups"], p["n_pairs"], _ptr(a["pair_ptr"]), _ptr(a["col_g"]),
                                   _ptr(a["val_g"]), _ptr(a.get("own_lo")), _ptr(a["blk_off"]), _ptr(a["pair_row"]),
                                   _ptr(x), _ptr(y), _ptr(a["ws"]), a["ws"].numel())
        else:
            raise SpmvError(OTHER_ERROR, "run", f"format {self.fmt} has no plan and no entry point")
        _check(rc, f"spmv_{self.fmt}_run")


# the library's A/B switches (include/spmv_ext.h; placement and load policy only)
OPTIONS = {"xwin_remap": 1, "xcd_remap": 2, "stream_nt": 3, "csr_prefetch": 4}


def set_option(name: str, value: int | None) -> None:
    """spmv_set_option: None / -1 = each kernel's default, 0 off, 1 on."""
    _check(hip_lib().spmv_set_option(OPTIONS[name], -1 if value is None else int(value)), f"set_option {name}")


def get_option(name: str) -> int:
    return int(hip_lib().spmv_get_option(OPTIONS[name]))


def _tri(v) -> int:
    """None -> -1 (the library's rule), else 0 / 1."""
    return -1 if v is None else int(bool(v))


def plan_opts(**kw) -> PlanOpts:
    """spmv_plan_opts with the library defaults, then the given fields."""
    o = PlanOpts()
    hip_lib().spmv_plan_opts_init(ctypes.byref(o))
    for k, v in kw.items():
        setattr(o, k, v)
    return o


_PLAN_INFO_KEYS = ("lanes", "variant", "ki", "xcap", "xwin", "head", "single_pass", "index16", "split_T", "n_chunks",
                   "big_tiles", "head_bytes", "ws_bytes", "owned_bytes", "H")


def _attach_plan(dm: DeviceMatrix, what: str, create, *args, opts: PlanOpts) -> None:
    """Create the C plan of dm (spmv_plan_<fmt>) and copy its choices
    (spmv_plan_info) into dm.params."""
    plan = _vp()
    _check(create(dm.dims(), *args, ctypes.byref(opts), ctypes.byref(plan)), what)
    dm.plan = plan
    info = PlanInfo()
    _check(hip_lib().spmv_plan_get_info(plan, ctypes.byref(info)), "spmv_plan_get_info")
    for k in _PLAN_INFO_KEYS:
        dm.params[k] = int(getattr(info, k))
    dm.params["kernel"] = info.kernel.decode()
    dm.params["plan"] = info.desc.decode()


def plan_info(dm: DeviceMatrix) -> dict:
    """The plan's choices as a dict (the fields of spmv_plan_info)."""
    return {k: dm.params[k] for k in _PLAN_INFO_KEYS + ("kernel", "plan") if k in dm.params}


def _csr_xwin(dm: DeviceMatrix) -> None:
    """Per-row-group column windows for the x-window CSR kernel (the
    CSR16 / CSR-f32 formats of spmv_ext.h; CSR itself plans its own)."""
    torch = _torch()
    p, a = dm.params, dm.arrays
    rows = p.setdefault("xwin_rows", 0)
    nbytes = hip_lib().spmv_csr_xwin_bytes(dm.n_rows, dm.nnz, p["lanes"], rows)
    a["win"] = torch.empty(max(nbytes, 8), dtype=torch.uint8, device=dm.device)
    cap = _c_i32(0)
    _check(hip_lib().spmv_csr_xwin_build(dm.dims(), _ptr(a["row_ptr"]), _ptr(a["col"]), p["lanes"], rows,
                                         _ptr(a["win"]), a["win"].numel(), ctypes.byref(cap)), "spmv_csr_xwin_build")
    p["xcap"] = cap.value
    p["variant"] = 3


def _plan_coo(dm, row, col, val, *, xwin=None, coo_tail=None, hot=None):
    dm.arrays = dict(row=_dev_tensor(row, dm.device), col=_dev_tensor(col, dm.device), val=_dev_tensor(val, dm.device))
    o = plan_opts(xwin=_tri(xwin), coo_pass=_tri(coo_tail), H=-1 if hot is None else int(hot))
    a = dm.arrays
    _attach_plan(dm, "spmv_plan_coo", hip_lib().spmv_plan_coo, _ptr(a["row"]), _ptr(a["col"]), _ptr(a["val"]),
                 opts=o)
    dm.stored_bytes = 16 * dm.nnz


def _plan_csr(dm, *, lanes=0, variant=0, xwin=None, xwin_rows=0, hot=None, bigplan=True):
    a = dm.arrays
    o = plan_opts(lanes=int(lanes), variant=int(variant) if variant else -1, xwin=_tri(xwin), xwin_rows=int(xwin_rows),
                  bigplan=-1 if bigplan else 0, H=-1 if hot is None else int(hot))
    _attach_plan(dm, "spmv_plan_csr", hip_lib().spmv_plan_csr, _ptr(a["row_ptr"]), _ptr(a["col"]), _ptr(a["val"]),
                 opts=o)
    dm.params["xwin_rows"] = int(xwin_rows)
    dm.stored_bytes = 12 * dm.nnz + 8 * (dm.n_rows + 1)


def _plan_ell(dm, *, xwin=None):
    a, p = dm.arrays, dm.params
    _attach_plan(dm, "spmv_plan_ell", hip_lib().spmv_plan_ell, p["K"], p["ld"], p["ki"], _ptr(a["col"]), _ptr(a["val"]),
                 opts=plan_opts(xwin=_tri(xwin)))
    dm.stored_bytes = 12 * p["stored"]


def _plan_sell(dm, *, xwin=None, split=None, hot=None, head=None, index16=False):
    a, p = dm.arrays, dm.params
    o = plan_opts(xwin=_tri(xwin), split=-1 if split is None else int(split), H=-1 if hot is None else int(hot),
                  head=_tri(head), index16=int(bool(index16)))
    _attach_plan(dm, "spmv_plan_sell", hip_lib().spmv_plan_sell, p["C"], p["sigma"], p["ki"], p["n_slices"],
                 _ptr(a["slice_ptr"]), _ptr(a["perm"]), _ptr(a["col"]), _ptr(a["val"]), opts=o)
    per_slot = 10 if index16 else 12
    dm.stored_bytes = per_slot * p["stored"] + 8 * (p["n_slices"] + 1) + 4 * p["n_slices"] * p["C"]


def _plan_cmrs(dm, *, variant=None, xwin=None, hot=None):
    a, p = dm.arrays, dm.params
    v = -1 if variant is None else (1 if int(variant) == 0 else 2)  # python 0 strip runs / 1 tiles
    o = plan_opts(variant=v, xwin=_tri(xwin), H=-1 if hot is None else int(hot))
    _attach_plan(dm, "spmv_plan_cmrs", hip_lib().spmv_plan_cmrs, p["h"], p["n_strips"], _ptr(a["strip_ptr"]),
                 _ptr(a["row_in_strip"]), _ptr(a["col"]), _ptr(a["val"]), opts=o)
    dm.stored_bytes = 13 * dm.nnz + 8 * (p["n_strips"] + 1)


def to_device(m: Coo, fmt: str, device="cuda:0", *, lanes: int = 0, variant: int = 0, ki: int = 0, C: int = 64,
              sigma: int = 1024, h: int = 8, ell_max_padding: float | None = 64.0,
              xwin: bool | None = None, xwin_rows: int = 0, split: int | None = None,
              cmrs_variant: int | None = None, hot: int | None = None,
              csr16_max_escape: float | None = 0.5, groups: int = 0, head: bool = True,
              sell_head: bool | None = None, coo_tail: bool | None = None, bigplan: bool = True,
              hyb_k: int = 0) -> DeviceMatrix:
    """Build `fmt` on the host (libspmv_host.so), upload it and, for the
    reference's five formats and SELL16, create its C plan (spmv.h): the
    library picks the kernel path — x windows in LDS (CSR, ELL, SELL, CMRS
    by default; COO opt-in), the entry-balanced tiles for skewed rows, the
    SELL head copy / split, the single-pass COO — exactly as ./bin/<fmt>.
    The keywords override its rules: xwin (None = the library's default),
    variant (CSR: 0 = the skew rule, 1-4 forced), cmrs_variant (None rule,
    0 strip runs, 1 tiles), split (SELL: None rule, 0 off, T), hot (None =
    the hot-column rule, 0 none, H forced), sell_head (None/True = the head
    copy where the small-matrix kernel runs), coo_tail (None = the single
    pass where the tail plan accepts the matrix, True = it or raise, False =
    the carry pass), bigplan (tiled CSR's big-tile plan), hyb_k (HYB's ELL
    width: 0 = spmv_hyb_plan's rule, K > 0 forced)."""
    torch = _torch()
    device = torch.device(device)
    dm = DeviceMatrix(fmt, m.n_rows, m.n_cols, m.nnz, device)
    if fmt == "coo":
        row, col, val = coo_sort_by_row(m)
        _plan_coo(dm, row, col, val, xwin=xwin, coo_tail=coo_tail, hot=hot)
        return dm
    ptr, col, val = csr_from_coo(m)
    if fmt == "csr":
        dm.arrays = dict(row_ptr=_dev_tensor(ptr, device), col=_dev_tensor(col, device), val=_dev_tensor(val, device))
        _plan_csr(dm, lanes=lanes, variant=variant, xwin=xwin, xwin_rows=xwin_rows, hot=hot, bigplan=bigplan)
    elif fmt == "csrf32":
        # fp32 values, fp64 products and sums (§8f row 4): the row-group x-window
        # kernel, or for skewed rows the entry-balanced one with the hot table
        v = variant or host_lib().spmv_csr_pick_variant(m.n_rows, _ptr(ptr))
        dm.params = dict(lanes=lanes or hip_lib().spmv_csr_auto_lanes(m.n_rows, m.nnz), xwin_rows=xwin_rows,
                         variant=4 if v == 4 else 3, H=0)
        dm.arrays = dict(row_ptr=_dev_tensor(ptr, device), col=_dev_tensor(col, device),
                         val=_dev_tensor(val.astype(np.float32), device))
        dm.stored_bytes = 8 * m.nnz + 8 * (m.n_rows + 1)
        if v == 4:
            H, hot_cols, col_hot = hot_columns(m.n_cols, col, 0 if hot is None else hot) if hot != 0 else (0, None, col)
            dm.params["H"] = H
            if H > 0:
                dm.arrays["col"] = _dev_tensor(col_hot, device)
                dm.arrays["hot"] = _dev_tensor(hot_cols, device)
            dm.arrays["ws"] = torch.empty(hip_lib().spmv_csr_hot_ws_bytes(m.n_rows, m.nnz, H), dtype=torch.uint8,
                                          device=device)
            n_plan = hip_lib().spmv_csr_tiled_plan_len(m.nnz)
            if n_plan > 0:
                dm.arrays["own_lo"] = torch.empty(n_plan, dtype=torch.int32, device=device)
                _check(hip_lib().spmv_csr_tiled_plan(dm.dims(), _ptr(dm.arrays["row_ptr"]), _ptr(dm.arrays["own_lo"])),
                       "spmv_csr_tiled_plan")
        else:
            _csr_xwin(dm)
    elif fmt == "csr16":
        c = csr16_build(col)
        if csr16_max_escape is not None and c["n_esc"] > csr16_max_escape * max(c["n_blocks"], 1):
            # columns spread wider than 16 bits in most blocks (R-MAT): the
            # escapes store more than plain CSR; reported N/A like ELL padding
            raise SpmvError(OTHER_ERROR, "csr16_build", f"{c['n_esc']} of {c['n_blocks']} 64-entry blocks "
                            f"need 32-bit escapes (> {csr16_max_escape:.0%})")
        dm.params = dict(lanes=lanes or hip_lib().spmv_csr_auto_lanes(m.n_rows, m.nnz), n_blocks=c["n_blocks"],
                         n_esc=c["n_esc"])
        dm.arrays = dict(row_ptr=_dev_tensor(ptr, device), blk_base=_dev_tensor(c["blk_base"], device),
                         col_off=_dev_tensor(c["col_off"], device), col_esc=_dev_tensor(c["col_esc"], device),
                         val=_dev_tensor(val, device))
        dm.stored_bytes = 10 * m.nnz + 4 * c["n_blocks"] + 256 * c["n_esc"] + 8 * (m.n_rows + 1)
        if xwin is None or xwin:
            # windows of the x-window pipeline from the int32 columns (the
            # same values), uploaded only for the build
            dm.arrays["col"] = _dev_tensor(col, device)
            dm.params["xwin_rows"] = xwin_rows
            _csr_xwin(dm)
            dm.params.pop("variant", None)
            del dm.arrays["col"]
    elif fmt == "ell":
        ki = ki or 2  # measured best for ELL (profiles/round1_sweep.md)
        e = ell_build(m.n_rows, ptr, col, val, ki=ki, max_padding=ell_max_padding)
        dm.params = dict(K=e["K"], ld=e["ld"], ki=ki, stored=e["stored"])
        dm.arrays = dict(col=_dev_tensor(e["col"], device), val=_dev_tensor(e["val"], device))
        _plan_ell(dm, xwin=xwin)
    elif fmt in ("sell", "sell16"):
        # sell16: SELL-C-σ with 16-bit column offsets from each workgroup's
        # window base (§8f row 4), built by the plan on the device; refused
        # when a window spans > 65,536 columns (R-MAT), like csr16's escapes
        ki = ki or hip_lib().spmv_sell_auto_ki(m.n_rows, C)  # 1 (σ-window kernel) or 2 (small matrices)
        s = sell_build(m.n_rows, ptr, col, val, C=C, sigma=sigma, ki=ki)
        dm.params = dict(C=C, sigma=sigma, ki=ki, n_slices=s["n_slices"], stored=s["stored"])
        dm.arrays = dict(slice_ptr=_dev_tensor(s["slice_ptr"], device), perm=_dev_tensor(s["perm"], device),
                         col=_dev_tensor(s["col"], device), val=_dev_tensor(s["val"], device))
        if fmt == "sell":
            _plan_sell(dm, xwin=xwin, split=split, hot=hot, head=sell_head)
        else:
            _plan_sell(dm, xwin=True, split=0, hot=0, head=head, index16=True)
            del dm.arrays["col"]  # read at plan creation only: the runs read the plan's 16-bit offsets
    elif fmt == "csrg":
        # column-grouped CSR for gather-bound power-law matrices (R-MAT)
        # G = 4 measured best on the R-MAT (0.757-0.785 ms vs 0.768-0.83 at G = 8,
        # profiles/round3/rmat_tiled_r.log): more groups add pairs
        g = csrg_build(m.n_rows, ptr, col, val, groups=groups or 4)
        dm.params = dict(groups=g["groups"], n_pairs=g["n_pairs"])
        dm.arrays = {k: _dev_tensor(g[k], device) for k in ("pair_ptr", "col_g", "val_g", "blk_off")}
        dm.arrays["pair_row"] = _dev_tensor(g["pair_row"].view(np.int16), device)
        ws = hip_lib().spmv_csrg_ws_bytes(g["n_pairs"], m.nnz)
        dm.arrays["ws"] = torch.empty(max(ws, 16), dtype=torch.uint8, device=device)
        n_plan = hip_lib().spmv_csr_tiled_plan_len(m.nnz)
        if n_plan > 0:  # tile -> first pair table over the pair CSR, built once
            dm.arrays["own_lo"] = torch.empty(n_plan, dtype=torch.int32, device=device)
            pd = Dims(g["n_pairs"], m.n_cols, m.nnz, device.index or 0, torch.cuda.current_stream(device).cuda_stream)
            _check(hip_lib().spmv_csr_tiled_plan(pd, _ptr(dm.arrays["pair_ptr"]), _ptr(dm.arrays["own_lo"])),
                   "spmv_csr_tiled_plan")
        dm.stored_bytes = 12 * m.nnz + 10 * g["n_pairs"] + 4 * g["blk_off"].size
    elif fmt == "hyb":
        hb = hyb_build(m.n_rows, ptr, col, val, ki=ki or 2, K=hyb_k)
        dm.params = dict(K=hb["K"], ld=hb["ld"], ki=hb["ki"], tail_nnz=hb["tail_nnz"], stored=hb["stored"], H=0)
        if hot != 0:  # one table over the ELL and tail columns together
            ne, nt_ = hb["stored"], hb["tail_nnz"]
            both = np.concatenate([hb["ell_col"][:ne], hb["tail_col"][:nt_]])
            H, hot_cols, both_hot = hot_columns(m.n_cols, both, hot or 0)
            if H > 0:
                dm.params["H"] = H
                hb["ell_col"] = both_hot[:ne]
                hb["tail_col"] = np.concatenate([both_hot[ne:], np.zeros(max(1 - nt_, 0), np.int32)])
        ws = hip_lib().spmv_hyb_hot_ws_bytes(hb["tail_nnz"], dm.params["H"])
        dm.arrays = {k: _dev_tensor(hb[k], device) for k in ("ell_col", "ell_val", "tail_row", "tail_col", "tail_val")}
        dm.arrays["ws"] = torch.empty(max(ws, 16), dtype=torch.uint8, device=device)
        if dm.params["H"] > 0:
            dm.arrays["hot"] = _dev_tensor(hot_cols, device)
        elif hb["tail_nnz"] > 0 and coo_tail is not False:
            # single-pass tail (no carry pass) where every tail row ends
            # within 80 entries of its tile, as the COO format
            td = dm.dims()
            td.nnz = hb["tail_nnz"]
            tb = hip_lib().spmv_coo_tail_bytes(hb["tail_nnz"])
            tails = torch.empty(max(tb, 4), dtype=torch.uint8, device=device)
            rc = hip_lib().spmv_coo_tail_build(td, _ptr(dm.arrays["tail_row"]), _ptr(tails), tails.numel())
            if rc == SUCCESS:
                dm.arrays["tails"] = tails
                dm.params["single_pass"] = 1
            elif coo_tail:
                raise SpmvError(rc, "spmv_coo_tail_build (hyb tail)", hip_lib().spmv_last_error().decode())
        if (xwin is None or xwin) and ("tails" in dm.arrays or hb["tail_nnz"] == 0) and hb["stored"] > 0:
            # the ELL part through the x-window ELL kernel (same bits): one
            # cant-like matrix cold, a full ELL 12.26 vs 13.36 us (profiles/HISTORY.md §H9)
            a, p = dm.arrays, dm.params
            nbytes = hip_lib().spmv_ell_xwin_bytes(dm.n_rows)
            a["win"] = torch.empty(max(nbytes, 8), dtype=torch.uint8, device=device)
            cap = _c_i32(0)
            _check(hip_lib().spmv_ell_xwin_build(dm.dims(), p["K"], p["ld"], p["ki"], _ptr(a["ell_col"]),
                                                 _ptr(a["win"]), a["win"].numel(), ctypes.byref(cap)),
                   "spmv_ell_xwin_build (hyb)")
            p["xcap"] = cap.value
        dm.stored_bytes = 12 * hb["stored"] + 16 * hb["tail_nnz"]
        # the first (ELL) kernel; K = 0 runs the tail alone as COO
        dm.params["kernel"] = ("coo_staged_kernel" if hb["K"] == 0 else
                               "ell_xwin_kernel" if "win" in dm.arrays else "ell_kernel")
    elif fmt == "cmrs":
        c = cmrs_build(m.n_rows, ptr, h=h)
        dm.params = dict(h=h, n_strips=c["n_strips"])
        dm.arrays = dict(strip_ptr=_dev_tensor(c["strip_ptr"], device),
                         row_in_strip=_dev_tensor(c["row_in_strip"], device),
                         col=_dev_tensor(col, device), val=_dev_tensor(val, device))
        _plan_cmrs(dm, variant=cmrs_variant, xwin=xwin, hot=hot)
    else:
        raise SpmvError(OTHER_ERROR, "to_device", f"unknown format {fmt}")
    return dm


def device_build(m: Coo, fmt: str, device="cuda:0", *, lanes: int = 0, ki: int = 0, C: int = 64,
                 sigma: int = 1024, h: int = 8, xwin: bool | None = None, split: int | None = None,
                 cmrs_variant: int | None = None) -> DeviceMatrix:
    """Like to_device, but only the raw COO (file order) crosses PCIe: CSR,
    ELL, SELL and CMRS are built on the device by the spmv_dev_* builders
    (SURVEY.md §8f row 2); the arrays equal the host builders'.  The same C
    plans run them."""
    torch = _torch()
    device = torch.device(device)
    if fmt not in ("csr", "ell", "sell", "cmrs"):
        raise SpmvError(OTHER_ERROR, "device_build", "format must be csr, ell, sell or cmrs")
    lib = hip_lib()
    N, Z = m.n_rows, m.nnz
    d_row, d_col, d_val = (_dev_tensor(a, device) for a in (m.row, m.col, m.val))
    ptr = torch.empty(N + 1, dtype=torch.int64, device=device)
    col = torch.empty(max(Z, 1), dtype=torch.int32, device=device)
    val = torch.empty(max(Z, 1), dtype=torch.float64, device=device)
    dm = DeviceMatrix(fmt, N, m.n_cols, Z, device)
    d = dm.dims()
    _check(lib.spmv_dev_csr_from_coo(d, _ptr(d_row), _ptr(d_col), _ptr(d_val), _ptr(ptr), _ptr(col), _ptr(val)),
           "spmv_dev_csr_from_coo")
    del d_row, d_col, d_val
    if fmt == "csr":
        dm.arrays = dict(row_ptr=ptr, col=col, val=val)
        _plan_csr(dm, lanes=lanes, variant=3, xwin=xwin)
    elif fmt == "ell":
        ki = ki or 2
        K, ld = _c_i32(0), _c_i64(0)
        _check(lib.spmv_dev_ell_plan(d, _ptr(ptr), ki, ctypes.byref(K), ctypes.byref(ld)), "spmv_dev_ell_plan")
        stored = K.value * ld.value
        ec = torch.empty(max(stored, 1), dtype=torch.int32, device=device)
        ev = torch.empty(max(stored, 1), dtype=torch.float64, device=device)
        _check(lib.spmv_dev_ell_fill(d, _ptr(ptr), _ptr(col), _ptr(val), K.value, ld.value, ki, _ptr(ec), _ptr(ev)),
               "spmv_dev_ell_fill")
        dm.params = dict(K=K.value, ld=ld.value, ki=ki, stored=stored)
        dm.arrays = dict(col=ec, val=ev)
        _plan_ell(dm, xwin=xwin)
    elif fmt == "sell":
        ki = ki or hip_lib().spmv_sell_auto_ki(m.n_rows, C)  # as to_device
        ns = (N + C - 1) // C
        perm = torch.empty(max(ns * C, 1), dtype=torch.int32, device=device)
        sp = torch.empty(ns + 1, dtype=torch.int64, device=device)
        scol = torch.empty(max(ns, 1), dtype=torch.int32, device=device)
        stored = _c_i64(0)
        _check(lib.spmv_dev_sell_plan(d, _ptr(ptr), _ptr(col), C, sigma, ki, ns, _ptr(perm), _ptr(sp), _ptr(scol),
                                      ctypes.byref(stored)), "spmv_dev_sell_plan")
        sc = torch.empty(max(stored.value, 1), dtype=torch.int32, device=device)
        sv = torch.empty(max(stored.value, 1), dtype=torch.float64, device=device)
        _check(lib.spmv_dev_sell_fill(d, _ptr(ptr), _ptr(col), _ptr(val), C, ki, ns, _ptr(sp), _ptr(perm), _ptr(scol),
                                      _ptr(sc), _ptr(sv)), "spmv_dev_sell_fill")
        dm.params = dict(C=C, sigma=sigma, ki=ki, n_slices=ns, stored=stored.value)
        dm.arrays = dict(slice_ptr=sp, perm=perm, col=sc, val=sv)
        _plan_sell(dm, xwin=xwin, split=split)
    else:
        ns = (N + h - 1) // h
        stp = torch.empty(ns + 1, dtype=torch.int64, device=device)
        rin = torch.empty(max(Z, 1), dtype=torch.uint8, device=device)
        _check(lib.spmv_dev_cmrs_build(d, _ptr(ptr), h, _ptr(stp), _ptr(rin)), "spmv_dev_cmrs_build")
        dm.params = dict(h=h, n_strips=ns)
        dm.arrays = dict(strip_ptr=stp, row_in_strip=rin, col=col, val=val)
        _plan_cmrs(dm, variant=cmrs_variant, xwin=xwin)
    dm.arrays["row_ptr_csr"] = ptr
    return dm


def banded_to_device(n: int, fmt: str, device="cuda:0", row_begin: int = 0, row_end: int | None = None,
                     seed: int = 2, C: int = 64, sigma: int = 1024, ki: int = 2, lanes: int = 0,
                     variant: int = 0, xwin: bool = True, xwin_rows: int = 0) -> DeviceMatrix:
    """Rows [row_begin, row_end) of the banded matrix (BASELINE.json
    configs[4]) generated directly in HBM by spmv_gen_banded_device, as CSR
    or SELL, run by its C plan (no hot-column table: the banded columns
    are uniform).  Row ids are local to the shard; columns are global (x is
    the full, replicated vector)."""
    torch = _torch()
    device = torch.device(device)
    row_end = n if row_end is None else row_end
    m = row_end - row_begin
    dm = DeviceMatrix(fmt, m, n, 16 * m, device)
    stream = torch.cuda.current_stream(device)
    if fmt == "csr":
        ptr = torch.empty(m + 1, dtype=torch.int64, device=device)
        col = torch.empty(16 * m, dtype=torch.int32, device=device)
        val = torch.empty(16 * m, dtype=torch.float64, device=device)
        rc = hip_lib().spmv_gen_banded_device(n, seed, row_begin, row_end, 0, 0, 0, _ptr(ptr), None, _ptr(col),
                                              _ptr(val), device.index or 0, stream.cuda_stream)
        _check(rc, "spmv_gen_banded_device")
        dm.arrays = dict(row_ptr=ptr, col=col, val=val)
        _plan_csr(dm, lanes=lanes, variant=variant, xwin=xwin, xwin_rows=xwin_rows, hot=0)
    elif fmt == "sell":
        ns = (m + C - 1) // C
        sp = torch.empty(ns + 1, dtype=torch.int64, device=device)
        perm = torch.empty(ns * C, dtype=torch.int32, device=device)
        col = torch.empty(ns * C * 16, dtype=torch.int32, device=device)
        val = torch.empty(ns * C * 16, dtype=torch.float64, device=device)
        rc = hip_lib().spmv_gen_banded_device(n, seed, row_begin, row_end, 1, C, ki, _ptr(sp), _ptr(perm),
                                              _ptr(col), _ptr(val), device.index or 0, stream.cuda_stream)
        _check(rc, "spmv_gen_banded_device")
        dm.params = dict(C=C, sigma=sigma, ki=ki, n_slices=ns, stored=ns * C * 16)
        dm.arrays = dict(slice_ptr=sp, perm=perm, col=col, val=val)
        _plan_sell(dm, xwin=xwin, split=0, hot=0)
    else:
        raise SpmvError(OTHER_ERROR, "banded_to_device", "format must be csr or sell")
    return dm


def read_bin(path) -> Coo:
    """Binary cache written by write_bin / the drivers' --cache."""
    lib = host_lib()
    info = MtxInfo()
    p = str(path).encode()
    _check_host(lib.spmv_bin_read_info(p, ctypes.byref(info)), f"read {path}")
    row = np.empty(info.nnz, np.int32)
    col = np.empty(info.nnz, np.int32)
    val = np.empty(info.nnz, np.float64)
    _check_host(lib.spmv_bin_read(p, ctypes.byref(info), _ptr(row), _ptr(col), _ptr(val)), f"read {path}")
    return Coo(info.n_rows, info.n_cols, row, col, val, bool(info.symmetric), str(path))


def write_bin(path, m: Coo) -> None:
    info = MtxInfo(m.n_rows, m.n_cols, m.nnz, int(m.symmetric), 0, 0)
    _check_host(host_lib().spmv_bin_write(str(path).encode(), ctypes.byref(info), _ptr(m.row), _ptr(m.col),
                                          _ptr(m.val)), f"write {path}")


def flush_cache(stream=None, nbytes: int = 0) -> None:
    """Evict the 256 MiB Infinity Cache + L2s (512 MiB scratch write)."""
    torch = _torch()
    s = stream if stream is not None else torch.cuda.current_stream()
    _check(hip_lib().spmv_flush_cache(s.cuda_stream, nbytes), "spmv_flush_cache")


def device_name(device: int = 0) -> str:
    buf = ctypes.create_string_buffer(256)
    _check(hip_lib().spmv_device_name(device, buf, 256), "spmv_device_name")
    return buf.value.decode()
