"""ctypes binding of libsvdw.so (the C ABI declared in include/svdw.h).

The product path has no CPU fallback: if the HIP library is missing or cannot
be loaded, every entry point raises.
"""
from __future__ import annotations

import ctypes as ct
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# SVDW_LIB: load another build of the library (tools/ab_lib.sh A/B runs of two builds)
LIB_PATH = os.environ.get("SVDW_LIB") or os.path.join(HERE, "libsvdw.so")

SVDW_OK = 0
ERRORS = {-1: "SVDW_EINVAL", -2: "SVDW_ERANGE", -3: "SVDW_EDEVICE", -4: "SVDW_ENOMEM"}


class SvdwError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


class Params(ct.Structure):
    _fields_ = [("device", ct.c_int), ("precision_bits", ct.c_uint32),
                ("lookup_bits", ct.c_uint32)]


class Mat(ct.Structure):
    _fields_ = [("phase", ct.c_uint32), ("rows", ct.c_uint32), ("cols", ct.c_uint32),
                ("off", ct.c_uint64), ("rs", ct.c_int64), ("cs", ct.c_int64)]

    def __repr__(self):
        return (f"Mat(phase={self.phase}, {self.rows}x{self.cols}, off={self.off}, "
                f"rs={self.rs}, cs={self.cs})")


class Vec(ct.Structure):
    _fields_ = [("phase", ct.c_uint32), ("len", ct.c_uint32), ("off", ct.c_uint64),
                ("stride", ct.c_int64)]

    def __repr__(self):
        return f"Vec(phase={self.phase}, len={self.len}, off={self.off}, stride={self.stride})"


class Payload(ct.Structure):
    _fields_ = [("u_t", Mat), ("v_t", Mat), ("m_times_vt", Mat), ("u_times_ut", Mat),
                ("v_times_vt", Mat)]


class SvdConfig(ct.Structure):
    _fields_ = [("max_norm", ct.c_double), ("eps_svd", ct.c_double), ("eps_u", ct.c_double),
                ("max_bits_d", ct.c_uint32)]


class KStat(ct.Structure):
    _fields_ = [("name", ct.c_char * 48), ("launches", ct.c_uint64), ("total_ms", ct.c_double),
                ("max_ms", ct.c_double), ("bytes", ct.c_double), ("ops", ct.c_double)]


class Segment(ct.Structure):
    _fields_ = [("phase", ct.c_uint32), ("lookup", ct.c_uint32), ("off", ct.c_uint64),
                ("n", ct.c_uint64)]


class EqCheck(ct.Structure):
    _fields_ = [("copies_checked", ct.c_uint64), ("copy_failures", ct.c_uint64),
                ("consts_checked", ct.c_uint64), ("const_failures", ct.c_uint64)]


class CheckResult(ct.Structure):
    _fields_ = [("gates_checked", ct.c_uint64), ("gate_failures", ct.c_uint64),
                ("lookups_checked", ct.c_uint64), ("lookup_failures", ct.c_uint64),
                ("copies_checked", ct.c_uint64), ("copy_failures", ct.c_uint64)]


class PhysParams(ct.Structure):
    _fields_ = [("k", ct.c_uint32), ("minimum_rows", ct.c_uint32), ("max_rows", ct.c_uint64),
                ("num_advice", ct.c_uint32 * 2), ("columns_used", ct.c_uint32 * 2),
                ("num_lookup_advice", ct.c_uint32 * 2), ("num_fixed", ct.c_uint32),
                ("constants", ct.c_uint64)]


class Region(ct.Structure):
    _fields_ = [("phase", ct.c_uint32), ("_pad", ct.c_uint32), ("off", ct.c_uint64),
                ("n", ct.c_uint64), ("loff", ct.c_uint64), ("nl", ct.c_uint64),
                ("rows", ct.c_uint64), ("tag", ct.c_char * 40)]


class InputDims(ct.Structure):
    _fields_ = [("m_rows", ct.c_uint32), ("m_cols", ct.c_uint32), ("u_rows", ct.c_uint32),
                ("u_cols", ct.c_uint32), ("v_rows", ct.c_uint32), ("v_cols", ct.c_uint32),
                ("d_len", ct.c_uint32)]


class DivScale(ct.Structure):
    _fields_ = [("shift_bits", ct.c_uint32), ("num_bits", ct.c_uint32)]


class Counts(ct.Structure):
    _fields_ = [("advice0", ct.c_uint64), ("advice1", ct.c_uint64), ("lookup0", ct.c_uint64),
                ("lookup1", ct.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_P = ct.c_void_p
_u32, _u64, _i32, _dbl = ct.c_uint32, ct.c_uint64, ct.c_int, ct.c_double
_u64p = ct.POINTER(ct.c_uint64)

# name -> (restype, argtypes); mirrors include/svdw.h one-for-one.
SIGNATURES = {
    "svdw_ctx_create": (_i32, [ct.POINTER(Params), ct.POINTER(_P)]),
    "svdw_ctx_destroy": (_i32, [_P]),
    "svdw_ctx_reset": (_i32, [_P]),
    "svdw_reserve": (_i32, [_P, _u32, _u64, _u64]),
    "svdw_sync": (_i32, [_P]),
    "svdw_query": (_i32, [_P]),
    "svdw_mark": (_i32, [_P, ct.POINTER(ct.c_uint64)]),
    "svdw_mark_done": (_i32, [_P, _u64]),
    "svdw_mark_wait": (_i32, [_P, _u64]),
    "svdw_stream_wait": (_i32, [_P, _P]),
    "svdw_stream_signal": (_i32, [_P, _P]),
    "svdw_debug_trace": (_i32, [_P]),
    "svdw_last_error": (ct.c_char_p, []),
    "svdw_abi_version": (_i32, []),
    "svdw_advice_len": (_u64, [_P, _u32]),
    "svdw_lookup_len": (_u64, [_P, _u32]),
    "svdw_advice_device_ptr": (_P, [_P, _u32]),
    "svdw_lookup_device_ptr": (_P, [_P, _u32]),
    "svdw_copy_advice": (_i32, [_P, _u32, _u64, _u64, _P]),
    "svdw_copy_lookup": (_i32, [_P, _u32, _u64, _u64, _P]),
    "svdw_zkmatrix_new": (_i32, [_P, _u32, _P, _u32, _u32, _i32, ct.POINTER(Mat)]),
    "svdw_zkvector_new": (_i32, [_P, _u32, _P, _u32, _i32, ct.POINTER(Vec)]),
    "svdw_transpose_matrix": (_i32, [ct.POINTER(Mat), ct.POINTER(Mat)]),
    "svdw_load_witness": (_i32, [_P, _u32, _P, ct.POINTER(Vec)]),
    "svdw_load_constant": (_i32, [_P, _u32, _P, ct.POINTER(Vec)]),
    "svdw_entries_less_than": (_i32, [_P, ct.POINTER(Vec), _u32]),
    "svdw_entries_in_desc_order": (_i32, [_P, ct.POINTER(Vec), _u32]),
    "svdw_check_mat_entries_bounded": (_i32, [_P, ct.POINTER(Mat), _P]),
    "svdw_check_mat_diff": (_i32, [_P, ct.POINTER(Mat), ct.POINTER(Mat), _P]),
    "svdw_check_mat_id": (_i32, [_P, ct.POINTER(Mat), ct.POINTER(Vec), _P]),
    "svdw_mat_times_diag_mat": (_i32, [_P, ct.POINTER(Mat), ct.POINTER(Vec), ct.POINTER(Mat)]),
    "svdw_rescale_matrix": (_i32, [_P, ct.POINTER(Mat), ct.POINTER(DivScale), ct.POINTER(Mat)]),
    "svdw_zkvector_inner_product": (_i32, [_P, _u32, ct.POINTER(Vec), ct.POINTER(Vec),
                                           ct.POINTER(DivScale), ct.POINTER(Vec)]),
    "svdw_zkvector_norm_square": (_i32, [_P, _u32, ct.POINTER(Vec), ct.POINTER(DivScale),
                                         ct.POINTER(Vec)]),
    "svdw_zkvector_dist_square": (_i32, [_P, _u32, ct.POINTER(Vec), ct.POINTER(Vec),
                                         ct.POINTER(DivScale), ct.POINTER(Vec)]),
    "svdw_zkvector_mul": (_i32, [_P, _u32, ct.POINTER(Vec), ct.POINTER(Mat), ct.POINTER(DivScale),
                                 ct.POINTER(Vec)]),
    "svdw_honest_prover_mat_mul": (_i32, [_P, _u32, ct.POINTER(Mat), ct.POINTER(Mat),
                                          ct.POINTER(Mat)]),
    "svdw_field_mat_vec_mul": (_i32, [_P, _u32, ct.POINTER(Mat), ct.POINTER(Vec),
                                      ct.POINTER(Vec)]),
    "svdw_verify_mul": (_i32, [_P, _u32, ct.POINTER(Mat), ct.POINTER(Mat), ct.POINTER(Mat), _P]),
    "svdw_err_calc": (_i32, [_u32, _u64, _dbl, _dbl, _dbl, ct.POINTER(_dbl), ct.POINTER(_dbl)]),
    "svdw_check_svd_phase0": (_i32, [_P, ct.POINTER(Mat), ct.POINTER(Mat), ct.POINTER(Mat),
                                     ct.POINTER(Vec), _dbl, _dbl, _u32, ct.POINTER(Payload)]),
    "svdw_check_svd_phase1": (_i32, [_P, ct.POINTER(Mat), ct.POINTER(Mat), ct.POINTER(Mat),
                                     ct.POINTER(Payload), _P]),
    "svdw_svd_witness": (_i32, [_P, _P, _P, _P, _P, _u32, _u32, _i32, ct.POINTER(SvdConfig), _P,
                                ct.POINTER(Counts)]),
    "svdw_set_gemm_impl": (_i32, [_P, _i32]),
    "svdw_set_option": (_i32, [_P, ct.c_char_p, ct.c_int64]),
    "svdw_graph_stats": (_i32, [_P, ct.POINTER(ct.c_uint64), ct.POINTER(ct.c_uint64)]),
    "svdw_profile_enable": (_i32, [_P, _i32]),
    "svdw_profile_filter": (_i32, [_P, ct.c_char_p]),
    "svdw_set_shard": (_i32, [_P, _u32, _u32]),
    "svdw_parse_svd_input": (_i32, [ct.c_char_p, _u64, _i32, ct.POINTER(InputDims), _P, _P, _P, _P]),
    "svdw_rlc_trace": (_i32, [_P, _P, _P, ct.POINTER(ct.c_uint32)]),
    "svdw_verify_mul_witness": (_i32, [_P, _P, _P, _u32, _u32, _u32, _i32, _P, ct.POINTER(Counts)]),
    "svdw_verify_mul_witness_on": (_i32, [_P, _P, _P, _P, _u32, _u32, _u32, _P, ct.POINTER(Counts)]),
    "svdw_parse_svd_input_device": (_i32, [_P, _P, _u64, _i32, ct.POINTER(InputDims), _P, _P, _P, _P]),
    "svdw_shard_segments": (_i32, [_P, ct.POINTER(Segment), _u64, _u64p]),
    "svdw_layout": (_i32, [_P, ct.POINTER(Region), _u64, _u64p]),
    "svdw_check_gates": (_i32, [_P, ct.POINTER(CheckResult)]),
    "svdw_physical_layout": (_i32, [_P, _u32, _u32, ct.POINTER(PhysParams)]),
    "svdw_break_points": (_i32, [_P, _u32, _u64p, _u64, _u64p]),
    "svdw_assign_columns": (_i32, [_P, _u32, _P, _P, _P]),
    "svdw_check_physical": (_i32, [_P, _u32, _P, _P, _u32, ct.POINTER(CheckResult)]),
    "svdw_equalities": (_i32, [_P, _u32, _P, _u64, _u64p, _P, _u64, _u64p]),
    "svdw_zkvector_norm": (_i32, [_P, _u32, ct.POINTER(Vec), ct.POINTER(DivScale), _u32, ct.POINTER(Vec)]),
    "svdw_zkvector_dist": (_i32, [_P, _u32, ct.POINTER(Vec), ct.POINTER(Vec), ct.POINTER(DivScale), _u32,
                                  ct.POINTER(Vec)]),
    "svdw_check_equalities": (_i32, [_P, _u32, _P, _P, ct.POINTER(EqCheck)]),
    "svdw_profile_collect": (_i32, [_P, ct.POINTER(KStat), _u32, ct.POINTER(_u32)]),
    "svdw_plan_svd": (_i32, [_u32, _u32, _u32, _u32, ct.POINTER(SvdConfig), ct.POINTER(Counts)]),
}

_lib = None


def lib():
    """Load libsvdw.so (raises if missing: there is no fallback path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} not built: run `python -m halo2_svd041_amd.build` "
                               "(hipcc --offload-arch=gfx950); no CPU fallback exists")
        L = ct.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc: int) -> None:
    if rc != SVDW_OK:
        raise SvdwError(rc, lib().svdw_last_error().decode())
