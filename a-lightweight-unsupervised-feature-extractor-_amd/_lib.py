"""ctypes binding of libtrk_amd.so (the C ABI declared in include/trk_amd.h).

There is no CPU fallback anywhere in this package: if the shared library is
missing, or a call is made with host tensors, the call raises.
"""
from __future__ import annotations

import ctypes
import os
import re
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# TRK_LIB_PATH: another in-tree build of the same library (A/B experiments of two builds); the
# default is the package's own libtrk_amd.so
LIB_PATH = os.environ.get("TRK_LIB_PATH") or os.path.join(_HERE, "libtrk_amd.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "trk_amd.h")

TRK_F32, TRK_BF16, TRK_F64 = 0, 1, 2
TRK_NCHW, TRK_NHWC = 0, 1
TRK_LSAP_MAX_DIM = 2048
TRK_ENC_PARTS = 3  # per-ROI partial sums of the encoder GEMMs (trk_amd.h)

_lock = threading.Lock()
_lib = None


class TrkError(RuntimeError):
    """A libtrk_amd entry point returned a non-zero status."""


class CostParams(ctypes.Structure):
    # mirrors trk_cost_params (include/trk_amd.h)
    _fields_ = [("w_app", ctypes.c_float), ("w_bbox", ctypes.c_float),
                ("w_conf", ctypes.c_float), ("alpha", ctypes.c_float),
                ("beta", ctypes.c_float), ("maha_thr", ctypes.c_double),
                ("inf_cost", ctypes.c_float), ("topk", ctypes.c_int), ("gate", ctypes.c_int)]


_STEP_PTRS = ("x P pbox last_conf gmean gsinv enc bank bank_len bank_head alive tid miss age last_frame "
              "order n_live next_id ndet frame_id flags m1 row1 m2 row2 n2 ud freelist e2 b2 c2 ap_n ap_slot "
              "ap_det ap_kind ap_cost lsap_status result").split()


class StepState(ctypes.Structure):
    # mirrors trk_step_state (include/trk_amd.h): device pointers, in declaration order
    _fields_ = [(n, ctypes.c_void_p) for n in _STEP_PTRS]


class StepConfig(ctypes.Structure):
    # mirrors trk_step_config (include/trk_amd.h)
    _fields_ = [("S", ctypes.c_int64), ("cap", ctypes.c_int64), ("Nmax", ctypes.c_int64), ("T", ctypes.c_int64),
                ("lost_reid_after", ctypes.c_int), ("max_age", ctypes.c_int),
                ("init_conf_min", ctypes.c_double), ("conf_update_min", ctypes.c_double),
                ("cost_update_max", ctypes.c_double), ("reid_only_cost_max", ctypes.c_double),
                ("maha_thr", ctypes.c_double), ("ema_alpha", ctypes.c_float)]


def _declare(L):
    P, i32, i64, sz, f32, f64 = (ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_size_t,
                                 ctypes.c_float, ctypes.c_double)
    L.trk_abi_version.argtypes = []
    L.trk_abi_version.restype = i32
    L.trk_last_error.argtypes = []
    L.trk_last_error.restype = ctypes.c_char_p
    L.trk_set_tuning.argtypes = [ctypes.c_char_p, i32]
    L.trk_set_tuning.restype = i32
    L.trk_roi_align_workspace_bytes.argtypes = [i64, i64, i64, i64, i32]
    L.trk_roi_align_workspace_bytes.restype = sz
    L.trk_roi_align_fwd.argtypes = [P, i64, i64, i64, i64, i32, P, i64, f32, i32, i32, i32, i32,
                                    P, i32, i32, P, sz, P]
    L.trk_roi_align_fwd.restype = i32
    L.trk_build_cost.argtypes = [i64, i64, i64, P, P, P, i64, P, P, P, P, P, P, P, P, P, P,
                                 ctypes.POINTER(CostParams), P, P, P, P, P, P]
    L.trk_build_cost.restype = i32
    L.trk_cost_combine.argtypes = [i64, i64, P, P, P, P, P, P, P, P, ctypes.POINTER(CostParams),
                                   P, P, P, P, P]
    L.trk_cost_combine.restype = i32
    L.trk_lsap.argtypes = [i64, P, i32, i64, i64, P, P, i64, P, P, P, P, P, i64, f64, P]
    L.trk_lsap.restype = i32
    L.trk_dwconv5_nhwc.argtypes = [P, P, P, i64, i64, i64, i64, i32, P]
    L.trk_dwconv5_nhwc.restype = i32
    L.trk_act_mean.argtypes = [P, P, P, i64, i64, i64, i64, i32, i32, P]
    L.trk_act_mean.restype = i32
    L.trk_scale_rows.argtypes = [P, P, i64, i64, i64, i32, P]
    L.trk_scale_rows.restype = i32
    L.trk_act_scale_rows.argtypes = [P, P, i64, i64, i64, i64, i32, i32, P]
    L.trk_act_scale_rows.restype = i32
    L.trk_enc_g1_dwconv.argtypes = [P, i64, P, i64, P, P, P]
    L.trk_enc_g1_dwconv.restype = i32
    L.trk_enc_dsc_gemm.argtypes = [P, i64, i64, i64, P, P, i64, P, P, P]
    L.trk_enc_dsc_gemm.restype = i32
    L.trk_enc_rmb_front_means.argtypes = [P, i64, P, P, P, P, P, P, P, P, P]
    L.trk_enc_rmb_front_means.restype = i32
    L.trk_enc_se_means.argtypes = [P, i64, i64, P, P, i64, P, P, P, P]
    L.trk_enc_se_means.restype = i32
    L.trk_enc_transition_gemm.argtypes = [P, i64, i64, i64, P, i64, P, P, i64, P, P]
    L.trk_enc_transition_gemm.restype = i32
    L.trk_enc_transition_gemm2.argtypes = [P, i64, i64, i64, P, i64, P, P, P, i64, P, P]
    L.trk_enc_transition_gemm2.restype = i32
    L.trk_enc_sums_reduce.argtypes = [P, i64, i64, i64, P, P]
    L.trk_enc_sums_reduce.restype = i32
    L.trk_enc_se.argtypes = [P, i64, i64, i64, i64, P, P, i64, P, P, P, P, P, P]
    L.trk_enc_se.restype = i32
    L.trk_enc_head.argtypes = [P, i64, i64, i64, P, P, P, ctypes.c_double, P, P, P, f32, P, P, i64, P, P]
    L.trk_enc_head.restype = i32
    L.trk_nchw_to_nhwc.argtypes = [P, i64, i64, i64, i64, P, P]
    L.trk_nchw_to_nhwc.restype = i32
    L.trk_kf_predict.argtypes = [i64, P, P, P, P, P, P, P]
    L.trk_kf_predict.restype = i32
    L.trk_track_update.argtypes = [i64, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, i64, f32, f32,
                                   f32, f64, P]
    L.trk_track_update.restype = i32
    L.trk_track_init.argtypes = [i64, P, P, P, P, P, P, P, P, P, P, P, P, P, i64, P]
    L.trk_track_init.restype = i32
    SP, SC = ctypes.POINTER(StepState), ctypes.POINTER(StepConfig)
    L.trk_step_result_stride.argtypes = [i64, i64]
    L.trk_step_result_stride.restype = i64
    L.trk_step_begin.argtypes = [SP, SC, P, P, i64, P]
    L.trk_step_mid.argtypes = [SP, SC, i64, P, P, P, P, P, P]
    L.trk_step_end.argtypes = [SP, SC, i64, P, P, P, P, P]
    L.trk_step_apply.argtypes = [SP, SC, P, P, P, P, P]
    for n in ("trk_step_begin", "trk_step_mid", "trk_step_end", "trk_step_apply"):
        getattr(L, n).restype = i32
    L.trk_build_cost_dev.argtypes = [i64, i64, i64, P, P, P, i64, i64, P, P, P, P, P, P, P, P, P, P,
                                     ctypes.POINTER(CostParams), P, P, P, P]
    L.trk_build_cost_dev.restype = i32
    L.trk_cost_work_bytes.argtypes = [i64, i64]
    L.trk_cost_work_bytes.restype = i64
    L.trk_lsap_dev.argtypes = [i64, P, i32, i64, i64, P, P, i64, i64, i64, P, P, P, P, P, i64, f64, P]
    L.trk_lsap_dev.restype = i32
    L.trk_lsap_set_prof.argtypes = [P]
    L.trk_lsap_set_prof.restype = i32
    L.trk_enc_set_prof.argtypes = [P]
    L.trk_enc_set_prof.restype = i32
    L.trk_stream_gate.argtypes = [P, ctypes.c_uint32, i64, P]
    L.trk_stream_gate.restype = i32
    L.trk_cost_set_prof.argtypes = [P]
    L.trk_cost_set_prof.restype = i32
    L.trk_head_set_prof.argtypes = [P]
    L.trk_head_set_prof.restype = i32
    for name, (args, res) in _EXTRA.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res


# entry points added by later modules register here (register() also declares them
# on an already-loaded library)
_EXTRA: dict = {}


def register(entries: dict):
    _EXTRA.update(entries)
    if _lib is not None:
        for name, (args, res) in entries.items():
            fn = getattr(_lib, name)
            fn.argtypes = args
            fn.restype = res


def lib():
    """The loaded library; raises if it has not been built."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise TrkError(
                        f"{LIB_PATH} is missing: build it with `make -C {os.path.join(_HERE, 'csrc')}` "
                        "or __graft_entry__.build() (there is no CPU fallback)")
                L = ctypes.CDLL(LIB_PATH)
                _declare(L)
                if L.trk_abi_version() != 2:
                    raise TrkError("libtrk_amd ABI version mismatch")
                # TRK_TUNE="key=value,..." applies trk_set_tuning knobs at load (A/B runs)
                for kv in filter(None, os.environ.get("TRK_TUNE", "").split(",")):
                    k, v = kv.split("=")
                    if L.trk_set_tuning(k.strip().encode(), int(v)) != 0:
                        raise TrkError(f"TRK_TUNE: {L.trk_last_error().decode()}")
                _lib = L
    return _lib


def check(rc: int, what: str):
    if rc != 0:
        msg = lib().trk_last_error().decode(errors="replace")
        if rc == -1:
            raise ValueError(f"{what}: {msg}")
        if rc == -3:
            raise NotImplementedError(f"{what}: {msg}")
        raise TrkError(f"{what} failed ({rc}): {msg}")


def set_tuning(key: str, value: int):
    """Process-global performance knob (include/trk_amd.h trk_set_tuning)."""
    check(lib().trk_set_tuning(key.encode(), int(value)), "set_tuning")


def header_symbols():
    """Every function the public header declares (for the ABI export test)."""
    src = open(HEADER_PATH).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(trk_[a-z0-9_]+)\s*\(", src)))
