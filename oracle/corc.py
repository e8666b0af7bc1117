"""ctypes binding of oracle/svdw_oracle.c (TEST INFRASTRUCTURE ONLY).

Used by tests/ (as the parity checker), __graft_entry__.smoke() and the
cpu_baseline leg of bench.py. Builds the library on first use if missing.
"""
from __future__ import annotations

import ctypes as ct
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libsvdw_oracle.so")
_lib = None
SIZE_MAX = (1 << 64) - 1


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH) or (
                os.path.getmtime(LIB_PATH) < os.path.getmtime(os.path.join(HERE, "svdw_oracle.c"))):
            build()
        L = ct.CDLL(LIB_PATH)
        u64p = ct.POINTER(ct.c_uint64)
        L.orc_svd_witness.restype = ct.c_int
        L.orc_svd_witness.argtypes = [
            ct.c_void_p, ct.c_void_p, ct.c_void_p, ct.c_void_p, ct.c_size_t, ct.c_size_t,
            ct.c_int, ct.c_int, ct.c_void_p, ct.c_double, ct.c_double, ct.c_double, ct.c_int,
            ct.c_size_t, ct.c_size_t,
            ct.POINTER(u64p), ct.POINTER(ct.c_size_t), ct.POINTER(u64p), ct.POINTER(ct.c_size_t),
            ct.POINTER(u64p), ct.POINTER(ct.c_size_t)]
        L.orc_verify_mul_witness.restype = ct.c_int
        L.orc_verify_mul_witness.argtypes = [
            ct.c_void_p, ct.c_void_p, ct.c_void_p, ct.c_size_t, ct.c_size_t, ct.c_size_t, ct.c_int,
            ct.c_void_p, ct.POINTER(u64p), ct.POINTER(ct.c_size_t), ct.POINTER(u64p),
            ct.POINTER(ct.c_size_t)]
        L.orc_free.argtypes = [ct.c_void_p]
        L.orc_err_calc.argtypes = [ct.c_int, ct.c_size_t, ct.c_double, ct.c_double, ct.c_double,
                                   ct.POINTER(ct.c_double), ct.POINTER(ct.c_double)]
        for fn in ("orc_fe_mul", "orc_fe_add", "orc_fe_sub"):
            getattr(L, fn).argtypes = [ct.c_void_p, ct.c_void_p, ct.c_void_p]
        L.orc_fe_inv.argtypes = [ct.c_void_p, ct.c_void_p]
        L.orc_quantize.argtypes = [ct.c_double, ct.c_int, ct.c_void_p]
        _lib = L
    return _lib


def int_to_limbs(x: int) -> np.ndarray:
    return np.array([(x >> (64 * i)) & ((1 << 64) - 1) for i in range(4)], dtype=np.uint64)


def limbs_to_int(a) -> int:
    a = [int(x) for x in a]
    return a[0] | (a[1] << 64) | (a[2] << 128) | (a[3] << 192)


def _take(ptr, n) -> np.ndarray:
    if n == 0:
        out = np.zeros((0, 4), dtype=np.uint64)
    else:
        buf = ct.cast(ptr, ct.POINTER(ct.c_uint64 * (4 * n))).contents
        out = np.frombuffer(buf, dtype=np.uint64).reshape(n, 4).copy()
    lib().orc_free(ptr)
    return out


def svd_witness(m, u, v, d, p: int, lb: int, gamma: int, max_norm=100.0, eps_svd=1e-10,
                eps_u=1e-10, max_bits_d=30, row_lim=None, row_begin=0):
    """Returns (advice0, lookup0, advice1) as (n,4) uint64 arrays of canonical cells.
    row_lim / row_begin: only the rows [row_begin, row_begin + row_lim) of every
    row-parallel stage (the others are computed in full)."""
    m = np.ascontiguousarray(m, dtype=np.float64)
    u = np.ascontiguousarray(u, dtype=np.float64)
    v = np.ascontiguousarray(v, dtype=np.float64)
    d = np.ascontiguousarray(d, dtype=np.float64)
    N, M = m.shape
    g = int_to_limbs(gamma)
    a0, l0, a1 = (ct.POINTER(ct.c_uint64)() for _ in range(3))
    n0, nl0, n1 = ct.c_size_t(), ct.c_size_t(), ct.c_size_t()
    rc = lib().orc_svd_witness(
        m.ctypes.data, u.ctypes.data, v.ctypes.data, d.ctypes.data, N, M, p, lb,
        g.ctypes.data, max_norm, eps_svd, eps_u, max_bits_d, row_begin,
        SIZE_MAX if row_lim is None else row_lim,
        ct.byref(a0), ct.byref(n0), ct.byref(l0), ct.byref(nl0), ct.byref(a1), ct.byref(n1))
    if rc != 0:
        raise ValueError(f"orc_svd_witness failed: {rc}")
    return _take(a0, n0.value), _take(l0, nl0.value), _take(a1, n1.value)


def verify_mul_witness(a, b, p: int, gamma: int, b_wrong=None):
    """README.md:32-46 recipe: phase-0 loads of a, b (and b_wrong), c_s = a * (b_wrong
    or b); phase-1 verify_mul(a, b, c_s, gamma). Returns (advice0, advice1)."""
    a = np.ascontiguousarray(a, dtype=np.float64)
    b = np.ascontiguousarray(b, dtype=np.float64)
    bw = None if b_wrong is None else np.ascontiguousarray(b_wrong, dtype=np.float64)
    n, k = a.shape
    k2, m = b.shape
    if k2 != k or (bw is not None and bw.shape != b.shape):
        raise ValueError("verify_mul_witness: shape mismatch")
    g = int_to_limbs(gamma)
    a0, a1 = ct.POINTER(ct.c_uint64)(), ct.POINTER(ct.c_uint64)()
    n0, n1 = ct.c_size_t(), ct.c_size_t()
    rc = lib().orc_verify_mul_witness(a.ctypes.data, b.ctypes.data,
                                      None if bw is None else bw.ctypes.data, n, k, m, p,
                                      g.ctypes.data, ct.byref(a0), ct.byref(n0), ct.byref(a1),
                                      ct.byref(n1))
    if rc != 0:
        raise ValueError(f"orc_verify_mul_witness failed: {rc}")
    return _take(a0, n0.value), _take(a1, n1.value)


def err_calc(p, size, max_norm=100.0, eps_svd=1e-10, eps_u=1e-10):
    a, b = ct.c_double(), ct.c_double()
    lib().orc_err_calc(p, size, max_norm, eps_svd, eps_u, ct.byref(a), ct.byref(b))
    return a.value, b.value


def quantize(x: float, p: int) -> int:
    out = np.zeros(4, dtype=np.uint64)
    lib().orc_quantize(x, p, out.ctypes.data)
    return limbs_to_int(out)


def fe_op(name: str, a: int, b: int = None) -> int:
    out = np.zeros(4, dtype=np.uint64)
    A = int_to_limbs(a)
    if b is None:
        getattr(lib(), name)(A.ctypes.data, out.ctypes.data)
    else:
        B = int_to_limbs(b)
        getattr(lib(), name)(A.ctypes.data, B.ctypes.data, out.ctypes.data)
    return limbs_to_int(out)
