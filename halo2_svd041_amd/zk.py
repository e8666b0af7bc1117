"""Host-side mirror of the reference's ZkMatrix / ZkVector / SVD API.

Same names and argument meaning as the Rust reference (src/matrix/mod.rs,
src/svd/mod.rs); every call goes through the C ABI (include/svdw.h) into the
gfx950 kernels. Where the reference panics on a shape mismatch, these raise
`SvdwError(SVDW_EINVAL)`.

    ctx = Context(device=0, precision_bits=63, lookup_bits=19)
    m = ZkMatrix.new(ctx, m_f64); u = ZkMatrix.new(ctx, u_f64); ...
    payload = check_svd_phase0(ctx, m, u, v, d, err_svd, err_u, 30)
    check_svd_phase1(ctx, m, u, v, payload, gamma)
    cells = ctx.advice(0)            # (n, 4) uint64 canonical Fr, like Fr::to_repr
"""
from __future__ import annotations

import collections
import ctypes as ct
from dataclasses import dataclass
from typing import Optional

import numpy as np

from ._lib import (CheckResult, EqCheck, PhysParams, Counts, DivScale, InputDims, KStat, Mat, Params, Payload, Region, Segment, SvdConfig, SvdwError,
                   Vec, check, lib)

P_MOD = 21888242871839275222246405745257275088548364400416034343698204186575808495617

__all__ = ["Context", "ZkMatrix", "ZkVector", "honest_prover_mat_mul", "field_mat_vec_mul",
           "mat_times_diag_mat", "check_mat_diff", "check_mat_id", "check_mat_entries_bounded",
           "check_svd_phase0", "check_svd_phase1", "err_calc", "svd_witness", "plan_svd",
           "SvdwError", "SvdPayload", "SvdConfigPy", "P_MOD", "int_to_words", "words_to_int"]


def int_to_words(x: int) -> np.ndarray:
    x = int(x)
    if x < 0:
        raise ValueError("expected a non-negative integer")
    return np.array([(x >> (64 * i)) & ((1 << 64) - 1) for i in range(4)], dtype=np.uint64)


_M64 = (1 << 64) - 1


def _words_arg(x: int):
    """x mod p as the 4-word little-endian argument of the C calls (a ctypes
    array: no numpy round trip on the per-witness path)."""
    x = int(x) % P_MOD
    return (ct.c_uint64 * 4)(x & _M64, (x >> 64) & _M64, (x >> 128) & _M64, x >> 192)


def words_to_int(w) -> int:
    w = [int(v) for v in w]
    return w[0] | (w[1] << 64) | (w[2] << 128) | (w[3] << 192)


_torch = None


def _torch_mod():
    global _torch
    if _torch is None:
        import torch  # noqa: WPS433
        _torch = torch
    return _torch


def _device_ptr(a) -> Optional[int]:
    """torch CUDA tensor -> device pointer (float64, contiguous) or None."""
    if isinstance(a, np.ndarray):
        return None
    try:
        torch = _torch_mod()
    except ImportError:  # pragma: no cover
        return None
    if isinstance(a, torch.Tensor) and a.is_cuda:
        if a.dtype != torch.float64 or not a.is_contiguous():
            raise SvdwError(-1, "device input must be a contiguous float64 tensor")
        return a.data_ptr()
    return None


def _torch_stream(ctx: "Context") -> int:
    """torch's current stream on the context's device (hipStream_t as int)."""
    t = _torch_mod()
    raw = getattr(t._C, "_cuda_getCurrentRawStream", None)   # no Stream object per call
    if raw is not None:
        return raw(ctx.device)
    return t.cuda.current_stream(ctx.device).cuda_stream


def _after_torch(ctx: "Context") -> None:
    """The engine's streams wait (on the device) for work torch has queued on
    its current stream: tensors it is still writing, memory it still reads."""
    check(lib().svdw_stream_wait(ctx.handle, _torch_stream(ctx)))


def _before_torch(ctx: "Context") -> None:
    """torch's current stream waits for the engine's queued work (its outputs)."""
    check(lib().svdw_stream_signal(ctx.handle, _torch_stream(ctx)))


# svdw_set_option names that change the cell layout (not just the schedule)
LAYOUT_OPTIONS = ("rlc_prefix",)


class Context:
    """One engine context = the phase-0 and phase-1 halo2-base `Context`s of a
    circuit (examples/svd_example.rs:108,181), streams resident on `device`."""

    def __init__(self, device: int = 0, precision_bits: int = 32, lookup_bits: int = 19):
        self.precision_bits = precision_bits
        self.lookup_bits = lookup_bits
        self.device = device
        self._phys = None
        self.last_svd = None
        self.layout_opts = {}
        self._h = ct.c_void_p()
        # device input tensors whose reads may still be queued (include/svdw.h,
        # "Lifetime of device inputs"): id -> [tensor, sequence number of the
        # last call that read it], kept until a completion mark at or after that call
        # has completed, so torch's allocator cannot hand their memory to a
        # tensor written on another stream while a pipelined call still reads it
        self._held = {}
        self._seq = 0
        self._ckpts = collections.deque()      # (call sequence number, svdw_mark ticket)
        p = Params(device, precision_bits, lookup_bits)
        check(lib().svdw_ctx_create(ct.byref(p), ct.byref(self._h)))

    # Per-call completion, at a cost amortised over calls: every HOLD_EVERY-th
    # call that holds inputs records a completion mark (svdw_mark: an event on
    # each of the context's streams, no waits); a held tensor is released once
    # a mark at or after its last reader has completed. At most HOLD_CKPTS
    # marks are pending: beyond that the oldest is waited for. So back-to-back
    # calls on fresh tensors hold the inputs of at most
    # HOLD_EVERY * (HOLD_CKPTS + 1) calls, whatever the device's progress, and
    # each call costs one dict update plus an event query. (The marks replaced
    # a side stream ordered after the context by svdw_stream_signal: with 4
    # hardware queues per process that stream shared one with a context stream,
    # whose next call then waited behind it -- 3.5 % of a 512^2 step.)
    HOLD_EVERY = 8
    HOLD_CKPTS = 4

    def _hold(self, *tensors) -> None:
        """Keep device inputs alive until the calls reading them have run (see _held)."""
        self._seq += 1
        seq = self._seq
        held = self._held
        for t in tensors:
            held[id(t)] = [t, seq]
        ck = self._ckpts
        done = 0
        while ck:
            s0, ticket = ck[0]
            if len(ck) > self.HOLD_CKPTS:
                check(lib().svdw_mark_wait(self._h, ticket))
            else:
                rc = lib().svdw_mark_done(self._h, ticket)
                if rc < 0:
                    check(rc)
                if rc != 1:
                    break
            ck.popleft()
            done = s0
        if done:
            for k in [k for k, (_, s) in held.items() if s <= done]:
                del held[k]
        if seq % self.HOLD_EVERY == 0:
            ticket = ct.c_uint64(0)
            check(lib().svdw_mark(self._h, ct.byref(ticket)))
            ck.append((seq, ticket.value))

    def _release_all(self) -> None:
        self._held.clear()
        self._ckpts.clear()

    def close(self) -> None:
        if self._h:
            lib().svdw_ctx_destroy(self._h)      # (waits for the context's work)
            self._h = ct.c_void_p()
        self._release_all()

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def handle(self):
        return self._h

    def reset(self) -> None:
        check(lib().svdw_ctx_reset(self._h))     # (synchronises)
        self._release_all()

    def reserve(self, phase: int, advice: int, lookups: int) -> None:
        check(lib().svdw_reserve(self._h, phase, advice, lookups))

    def sync(self) -> None:
        check(lib().svdw_sync(self._h))
        self._release_all()

    def query(self) -> bool:
        """svdw_query: has everything queued on the context completed?"""
        rc = lib().svdw_query(self._h)
        if rc < 0:
            check(rc)
        if rc == 1:
            self._release_all()
        return rc == 1

    def advice_len(self, phase: int) -> int:
        return lib().svdw_advice_len(self._h, phase)

    def lookup_len(self, phase: int) -> int:
        return lib().svdw_lookup_len(self._h, phase)

    def advice_device_ptr(self, phase: int) -> int:
        return lib().svdw_advice_device_ptr(self._h, phase) or 0

    def lookup_device_ptr(self, phase: int) -> int:
        return lib().svdw_lookup_device_ptr(self._h, phase) or 0

    def advice(self, phase: int, off: int = 0, n: Optional[int] = None) -> np.ndarray:
        n = self.advice_len(phase) - off if n is None else n
        out = np.zeros((n, 4), dtype=np.uint64)
        check(lib().svdw_copy_advice(self._h, phase, off, n, out.ctypes.data))
        return out

    def lookups(self, phase: int, off: int = 0, n: Optional[int] = None) -> np.ndarray:
        n = self.lookup_len(phase) - off if n is None else n
        out = np.zeros((n, 4), dtype=np.uint64)
        check(lib().svdw_copy_lookup(self._h, phase, off, n, out.ctypes.data))
        return out

    def set_gemm_impl(self, impl: str) -> None:
        """'mfma' (matrix cores, default) or 'valu' (v_dot4): bit-identical GEMM paths."""
        check(lib().svdw_set_gemm_impl(self._h, {"mfma": 0, "valu": 1}[impl]))

    def set_option(self, name: str, value: int) -> None:
        """Options of svdw_set_option (include/svdw.h). Tuning knobs leave the
        cells bit-identical; the layout options (LAYOUT_OPTIONS) add cells and
        are recorded in `layout_opts`, so a replay of this context's witness
        (collect.plan's dry planner) sees the same layout."""
        check(lib().svdw_set_option(self._h, name.encode(), int(value)))
        if name in LAYOUT_OPTIONS:
            self.layout_opts[name] = int(value)

    def graph_stats(self) -> tuple:
        """(captures, replays) of the captured verify_mul_witness graph
        (svdw_graph_stats; option "graph")."""
        cap, rep = ct.c_uint64(0), ct.c_uint64(0)
        check(lib().svdw_graph_stats(self._h, ct.byref(cap), ct.byref(rep)))
        return cap.value, rep.value

    def set_shard(self, rank: int, world: int) -> None:
        """Row-block sharding of one witness over `world` contexts (svdw_set_shard)."""
        check(lib().svdw_set_shard(self._h, int(rank), int(world)))

    def shard_segments(self) -> list:
        """[(phase, lookup, off, n)] cell ranges this rank is the source of."""
        n = ct.c_uint64()
        check(lib().svdw_shard_segments(self._h, None, 0, ct.byref(n)))
        buf = (Segment * max(n.value, 1))()
        check(lib().svdw_shard_segments(self._h, buf, n.value, ct.byref(n)))
        return [(s.phase, s.lookup, s.off, s.n) for s in buf[:n.value]]

    def layout(self) -> list:
        """Virtual layout of the last witness (svdw_layout): dicts with phase, off,
        n, loff, nl, rows, tag for every appended region, in append order."""
        n = ct.c_uint64()
        check(lib().svdw_layout(self._h, None, 0, ct.byref(n)))
        buf = (Region * max(n.value, 1))()
        check(lib().svdw_layout(self._h, buf, n.value, ct.byref(n)))
        return [{"phase": r.phase, "off": r.off, "n": r.n, "loff": r.loff, "nl": r.nl,
                 "rows": r.rows, "tag": r.tag.decode()} for r in buf[:n.value]]

    def rlc_trace(self) -> Optional[dict]:
        """ctx_rlc of the last svd_witness with rlc_prefix (svdw_rlc_trace;
        parity unpinned): {"cells": (3, 4) uint64, "copies": [(phase, offset)]
        of its two E cells}, or None without the prefix."""
        cells = np.zeros((3, 4), dtype=np.uint64)
        copies = np.zeros(2, dtype=np.uint64)
        n = ct.c_uint32()
        check(lib().svdw_rlc_trace(self._h, cells.ctypes.data, copies.ctypes.data, ct.byref(n)))
        if not n.value:
            return None
        return {"cells": cells, "copies": [(int(c) >> 62, int(c) & ((1 << 62) - 1)) for c in copies]}

    def check_gates(self) -> dict:
        """Device constraint check of the last witness (svdw_check_gates)."""
        r = CheckResult()
        check(lib().svdw_check_gates(self._h, ct.byref(r)))
        return {"gates_checked": r.gates_checked, "gate_failures": r.gate_failures,
                "lookups_checked": r.lookups_checked, "lookup_failures": r.lookup_failures,
                "copies_checked": r.copies_checked, "copy_failures": r.copy_failures}

    def physical_layout(self, k: int, minimum_rows: int = 20) -> dict:
        """Virtual -> physical layout plan of the last witness (svdw_physical_layout)."""
        p = PhysParams()
        check(lib().svdw_physical_layout(self._h, k, minimum_rows, ct.byref(p)))
        self._phys = {"k": p.k, "minimum_rows": p.minimum_rows, "max_rows": p.max_rows,
                "num_advice": list(p.num_advice), "columns_used": list(p.columns_used),
                "num_lookup_advice": list(p.num_lookup_advice), "num_fixed": p.num_fixed,
                "constants": p.constants}
        return dict(self._phys)

    def break_points(self, phase: int) -> list:
        n = ct.c_uint64()
        check(lib().svdw_break_points(self._h, phase, None, 0, ct.byref(n)))
        buf = (ct.c_uint64 * max(n.value, 1))()
        check(lib().svdw_break_points(self._h, phase, buf, n.value, ct.byref(n)))
        return list(buf[:n.value])

    def assign_columns(self, phase: int, device=None):
        """(advice [cols, 2^k, 32] u8, selectors [cols, 2^k] u8, lookup [nl, 2^k, 32] u8)
        torch tensors on the device, filled by svdw_assign_columns."""
        import torch
        p = self._phys
        if p is None:
            raise RuntimeError("call physical_layout() after the witness first")
        dev = device or torch.device("cuda", self.device)
        rows = 1 << p["k"]
        nc, nl = p["columns_used"][phase], p["num_lookup_advice"][phase]
        adv = torch.empty((nc, rows, 32), dtype=torch.uint8, device=dev)
        sel = torch.empty((nc, rows), dtype=torch.uint8, device=dev)
        lk = torch.empty((nl, rows, 32), dtype=torch.uint8, device=dev)
        _after_torch(self)
        check(lib().svdw_assign_columns(self._h, phase, adv.data_ptr() if nc else None,
                                        sel.data_ptr() if nc else None, lk.data_ptr() if nl else None))
        _before_torch(self)
        return adv, sel, lk

    def check_physical(self, phase: int, adv, sel) -> dict:
        r = CheckResult()
        _after_torch(self)
        check(lib().svdw_check_physical(self._h, phase, adv.data_ptr(), sel.data_ptr(), adv.shape[0],
                                        ct.byref(r)))
        return {"gates_checked": r.gates_checked, "gate_failures": r.gate_failures,
                "copies_checked": r.copies_checked, "copy_failures": r.copy_failures}

    def equalities(self, phase: int):
        """Copy-constraint lists of the last witness (svdw_equalities), in assign
        order: copies (n, 3) uint64 [source phase (2: init_rand), source cell,
        destination cell], consts: list of (cell, value int)."""
        nc, nk = ct.c_uint64(), ct.c_uint64()
        check(lib().svdw_equalities(self._h, phase, None, 0, ct.byref(nc), None, 0, ct.byref(nk)))
        cp = np.zeros((max(nc.value, 1), 2), dtype=np.uint64)
        ks = np.zeros((max(nk.value, 1), 5), dtype=np.uint64)
        check(lib().svdw_equalities(self._h, phase, cp.ctypes.data, nc.value, ct.byref(nc),
                                    ks.ctypes.data, nk.value, ct.byref(nk)))
        cp, ks = cp[:nc.value], ks[:nk.value]
        out = np.empty((cp.shape[0], 3), dtype=np.uint64)
        out[:, 0] = cp[:, 0] >> np.uint64(62)
        out[:, 1] = cp[:, 0] & np.uint64((1 << 62) - 1)
        out[:, 2] = cp[:, 1]
        consts = [(int(r[0]), words_to_int(r[1:])) for r in ks]
        return out, consts

    def check_equalities(self, phase: int, columns0=None, columns1=None) -> dict:
        """Device check of the equality records (svdw_check_equalities) on the
        cell streams, or on assigned physical columns (torch tensors)."""
        r = EqCheck()
        p0 = columns0.data_ptr() if columns0 is not None else None
        p1 = columns1.data_ptr() if columns1 is not None else None
        if p0 is not None or p1 is not None:
            _after_torch(self)
        check(lib().svdw_check_equalities(self._h, phase, p0, p1, ct.byref(r)))
        return {"copies_checked": r.copies_checked, "copy_failures": r.copy_failures,
                "consts_checked": r.consts_checked, "const_failures": r.const_failures}

    def profile(self, on: bool = True, prefix: str = "") -> None:
        """Record HIP events around kernel launches (names starting with `prefix`)."""
        check(lib().svdw_profile_filter(self._h, prefix.encode()))
        check(lib().svdw_profile_enable(self._h, 1 if on else 0))

    def profile_collect(self) -> list:
        """Per-kernel {name, launches, total_ms, max_ms, bytes, ops}; drops the records."""
        n = ct.c_uint32()
        cap = 256   # distinct kernel names; collect() drops the records, so one call
        buf = (KStat * cap)()
        check(lib().svdw_profile_collect(self._h, buf, cap, ct.byref(n)))
        return [{"name": s.name.decode(), "launches": s.launches, "total_ms": s.total_ms,
                 "max_ms": s.max_ms, "bytes": s.bytes, "ops": s.ops} for s in buf[:min(n.value, cap)]]

    def load_witness(self, value: int, phase: int = 0) -> "ZkVector":
        v = Vec()
        w = int_to_words(int(value) % P_MOD)
        check(lib().svdw_load_witness(self._h, phase, w.ctypes.data, ct.byref(v)))
        return ZkVector(self, v)

    def load_constant(self, value: int, phase: int = 0) -> "ZkVector":
        v = Vec()
        w = int_to_words(int(value) % P_MOD)
        check(lib().svdw_load_constant(self._h, phase, w.ctypes.data, ct.byref(v)))
        return ZkVector(self, v)


class ZkMatrix:
    """src/matrix/mod.rs:219-420: a view (offset + strides) into a phase stream."""

    def __init__(self, ctx: Context, mat: Mat):
        self.ctx = ctx
        self.mat = mat

    @property
    def num_rows(self) -> int:
        return self.mat.rows

    @property
    def num_col(self) -> int:
        return self.mat.cols

    @classmethod
    def new(cls, ctx: Context, matrix, phase: int = 0) -> "ZkMatrix":
        """ZkMatrix::new (src/matrix/mod.rs:230-252)."""
        out = Mat()
        dp = _device_ptr(matrix)
        if dp is not None:
            rows, cols = matrix.shape
            _after_torch(ctx)
            check(lib().svdw_zkmatrix_new(ctx.handle, phase, dp, rows, cols, 1, ct.byref(out)))
            ctx._hold(matrix)
        else:
            a = np.ascontiguousarray(matrix, dtype=np.float64)
            if a.ndim != 2:
                raise SvdwError(-1, "ZkMatrix::new expects a 2-D matrix")
            check(lib().svdw_zkmatrix_new(ctx.handle, phase, a.ctypes.data, a.shape[0],
                                          a.shape[1], 0, ct.byref(out)))
        return cls(ctx, out)

    def transpose_matrix(self) -> "ZkMatrix":
        """ZkMatrix::transpose_matrix (src/matrix/mod.rs:408-419): no cells."""
        out = Mat()
        check(lib().svdw_transpose_matrix(ct.byref(self.mat), ct.byref(out)))
        return ZkMatrix(self.ctx, out)

    @staticmethod
    def verify_mul(ctx: Context, a: "ZkMatrix", b: "ZkMatrix", c_s: "ZkMatrix", init_rand: int,
                   phase: int = 1) -> None:
        """ZkMatrix::verify_mul (src/matrix/mod.rs:299-342)."""
        g = int_to_words(int(init_rand) % P_MOD)
        check(lib().svdw_verify_mul(ctx.handle, phase, ct.byref(a.mat), ct.byref(b.mat),
                                    ct.byref(c_s.mat), g.ctypes.data))

    @staticmethod
    def rescale_matrix(ctx: Context, c_s: "ZkMatrix", shift_bits: int = 0,
                       num_bits: int = 0) -> "ZkMatrix":
        """ZkMatrix::rescale_matrix (src/matrix/mod.rs:354-375). signed_div_scale's
        layout is parity unpinned (include/svdw.h, svdw_div_scale)."""
        out = Mat()
        cfg = DivScale(shift_bits, num_bits)
        check(lib().svdw_rescale_matrix(ctx.handle, ct.byref(c_s.mat), ct.byref(cfg), ct.byref(out)))
        return ZkMatrix(ctx, out)

    def values(self) -> np.ndarray:
        """Cell values (rows, cols, 4) uint64 (host copy, for inspection)."""
        cells = self.ctx.advice(self.mat.phase)
        idx = (self.mat.off + np.arange(self.mat.rows)[:, None] * self.mat.rs
               + np.arange(self.mat.cols)[None, :] * self.mat.cs)
        return cells[idx]


class ZkVector:
    """src/matrix/mod.rs:19-216."""

    def __init__(self, ctx: Context, vec: Vec):
        self.ctx = ctx
        self.vec = vec

    def size(self) -> int:
        return self.vec.len

    @classmethod
    def new(cls, ctx: Context, v, phase: int = 0) -> "ZkVector":
        """ZkVector::new (src/matrix/mod.rs:29-40)."""
        out = Vec()
        dp = _device_ptr(v)
        if dp is not None:
            _after_torch(ctx)
            check(lib().svdw_zkvector_new(ctx.handle, phase, dp, v.numel(), 1, ct.byref(out)))
            ctx._hold(v)
        else:
            a = np.ascontiguousarray(v, dtype=np.float64).ravel()
            check(lib().svdw_zkvector_new(ctx.handle, phase, a.ctypes.data, a.size, 0,
                                          ct.byref(out)))
        return cls(ctx, out)

    def values(self) -> np.ndarray:
        """Cell values (len, 4) uint64 (host copy, for inspection)."""
        cells = self.ctx.advice(self.vec.phase)
        return cells[self.vec.off + np.arange(self.vec.len) * self.vec.stride]

    def inner_product(self, x: "ZkVector", phase: int = 0, shift_bits: int = 0,
                      num_bits: int = 0) -> "ZkVector":
        """ZkVector::inner_product (src/matrix/mod.rs:79-106): 1-element vector."""
        out = Vec()
        cfg = DivScale(shift_bits, num_bits)
        check(lib().svdw_zkvector_inner_product(self.ctx.handle, phase, ct.byref(self.vec),
                                                ct.byref(x.vec), ct.byref(cfg), ct.byref(out)))
        return ZkVector(self.ctx, out)

    def _norm_square(self, phase: int = 0, shift_bits: int = 0, num_bits: int = 0) -> "ZkVector":
        """ZkVector::_norm_square (src/matrix/mod.rs:112-119): 1-element vector."""
        out = Vec()
        cfg = DivScale(shift_bits, num_bits)
        check(lib().svdw_zkvector_norm_square(self.ctx.handle, phase, ct.byref(self.vec),
                                              ct.byref(cfg), ct.byref(out)))
        return ZkVector(self.ctx, out)

    def norm(self, phase: int = 0, shift_bits: int = 0, num_bits: int = 0,
             sqrt_bits: int = 0) -> "ZkVector":
        """ZkVector::norm (src/matrix/mod.rs:124-131): qsqrt(_norm_square); qsqrt is
        the parameterised construction of svdw_zkvector_norm (parity unpinned)."""
        out = Vec()
        cfg = DivScale(shift_bits, num_bits)
        check(lib().svdw_zkvector_norm(self.ctx.handle, phase, ct.byref(self.vec), ct.byref(cfg),
                                       sqrt_bits, ct.byref(out)))
        return ZkVector(self.ctx, out)

    def dist(self, x: "ZkVector", phase: int = 0, shift_bits: int = 0, num_bits: int = 0,
             sqrt_bits: int = 0) -> "ZkVector":
        """ZkVector::dist (src/matrix/mod.rs:156-164): qsqrt(_dist_square(x))."""
        out = Vec()
        cfg = DivScale(shift_bits, num_bits)
        check(lib().svdw_zkvector_dist(self.ctx.handle, phase, ct.byref(self.vec), ct.byref(x.vec),
                                       ct.byref(cfg), sqrt_bits, ct.byref(out)))
        return ZkVector(self.ctx, out)

    def _dist_square(self, x: "ZkVector", phase: int = 0, shift_bits: int = 0,
                     num_bits: int = 0) -> "ZkVector":
        """ZkVector::_dist_square (src/matrix/mod.rs:135-148): 1-element vector."""
        out = Vec()
        cfg = DivScale(shift_bits, num_bits)
        check(lib().svdw_zkvector_dist_square(self.ctx.handle, phase, ct.byref(self.vec),
                                              ct.byref(x.vec), ct.byref(cfg), ct.byref(out)))
        return ZkVector(self.ctx, out)

    def mul(self, a: ZkMatrix, phase: int = 0, shift_bits: int = 0,
            num_bits: int = 0) -> "ZkVector":
        """ZkVector::mul (src/matrix/mod.rs:169-182): a . self, rescaled."""
        out = Vec()
        cfg = DivScale(shift_bits, num_bits)
        check(lib().svdw_zkvector_mul(self.ctx.handle, phase, ct.byref(self.vec), ct.byref(a.mat),
                                      ct.byref(cfg), ct.byref(out)))
        return ZkVector(self.ctx, out)

    def entries_less_than(self, max_bits: int) -> None:
        """ZkVector::entries_less_than (src/matrix/mod.rs:185-194)."""
        check(lib().svdw_entries_less_than(self.ctx.handle, ct.byref(self.vec), max_bits))

    def entries_in_desc_order(self, max_bits: int) -> None:
        """ZkVector::entries_in_desc_order (src/matrix/mod.rs:199-215)."""
        check(lib().svdw_entries_in_desc_order(self.ctx.handle, ct.byref(self.vec), max_bits))


def _bound_words(b: int) -> np.ndarray:
    if b < 0 or b >= (1 << 256):
        raise SvdwError(-1, "bound must be a non-negative 256-bit integer")
    return int_to_words(b)


def honest_prover_mat_mul(ctx: Context, a: ZkMatrix, b: ZkMatrix, phase: int = 0) -> ZkMatrix:
    """src/matrix/mod.rs:546-568."""
    out = Mat()
    check(lib().svdw_honest_prover_mat_mul(ctx.handle, phase, ct.byref(a.mat), ct.byref(b.mat),
                                           ct.byref(out)))
    return ZkMatrix(ctx, out)


def field_mat_vec_mul(ctx: Context, a: ZkMatrix, v: ZkVector, phase: int = 0) -> ZkVector:
    """src/matrix/mod.rs:574-599."""
    out = Vec()
    check(lib().svdw_field_mat_vec_mul(ctx.handle, phase, ct.byref(a.mat), ct.byref(v.vec),
                                       ct.byref(out)))
    return ZkVector(ctx, out)


def mat_times_diag_mat(ctx: Context, a: ZkMatrix, v: ZkVector) -> ZkMatrix:
    """src/matrix/mod.rs:610-627."""
    out = Mat()
    check(lib().svdw_mat_times_diag_mat(ctx.handle, ct.byref(a.mat), ct.byref(v.vec),
                                        ct.byref(out)))
    return ZkMatrix(ctx, out)


def check_mat_diff(ctx: Context, a: ZkMatrix, b: ZkMatrix, tol: int) -> None:
    """src/matrix/mod.rs:441-457."""
    check(lib().svdw_check_mat_diff(ctx.handle, ct.byref(a.mat), ct.byref(b.mat),
                                    _bound_words(tol).ctypes.data))


def check_mat_id(ctx: Context, a: ZkMatrix, scalar_id: ZkVector, tol: int) -> None:
    """src/matrix/mod.rs:461-483."""
    check(lib().svdw_check_mat_id(ctx.handle, ct.byref(a.mat), ct.byref(scalar_id.vec),
                                  _bound_words(tol).ctypes.data))


def check_mat_entries_bounded(ctx: Context, a: ZkMatrix, bnd: int) -> None:
    """src/matrix/mod.rs:490-501."""
    check(lib().svdw_check_mat_entries_bounded(ctx.handle, ct.byref(a.mat),
                                               _bound_words(bnd).ctypes.data))


def err_calc(p: int, size: int, max_norm: float, eps_svd: float, eps_u: float):
    """src/svd/mod.rs:155-163."""
    a, b = ct.c_double(), ct.c_double()
    check(lib().svdw_err_calc(p, size, max_norm, eps_svd, eps_u, ct.byref(a), ct.byref(b)))
    return a.value, b.value


@dataclass
class SvdPayload:
    u_t: ZkMatrix
    v_t: ZkMatrix
    m_times_vt: ZkMatrix
    u_times_ut: ZkMatrix
    v_times_vt: ZkMatrix
    raw: Payload


def check_svd_phase0(ctx: Context, m: ZkMatrix, u: ZkMatrix, v: ZkMatrix, d: ZkVector,
                     err_svd: float, err_u: float, max_bits_d: int) -> SvdPayload:
    """src/svd/mod.rs:32-116."""
    pl = Payload()
    check(lib().svdw_check_svd_phase0(ctx.handle, ct.byref(m.mat), ct.byref(u.mat),
                                      ct.byref(v.mat), ct.byref(d.vec), err_svd, err_u,
                                      max_bits_d, ct.byref(pl)))
    return SvdPayload(ZkMatrix(ctx, pl.u_t), ZkMatrix(ctx, pl.v_t), ZkMatrix(ctx, pl.m_times_vt),
                      ZkMatrix(ctx, pl.u_times_ut), ZkMatrix(ctx, pl.v_times_vt), pl)


def check_svd_phase1(ctx: Context, m: ZkMatrix, u: ZkMatrix, v: ZkMatrix, payload: SvdPayload,
                     init_rand: int) -> None:
    """src/svd/mod.rs:127-144."""
    g = int_to_words(int(init_rand) % P_MOD)
    check(lib().svdw_check_svd_phase1(ctx.handle, ct.byref(m.mat), ct.byref(u.mat),
                                      ct.byref(v.mat), ct.byref(payload.raw), g.ctypes.data))


@dataclass
class SvdConfigPy:
    """examples/svd_example.rs:115-118,160."""
    max_norm: float = 100.0
    eps_svd: float = 1e-10
    eps_u: float = 1e-10
    max_bits_d: int = 30

    def c(self) -> SvdConfig:
        return SvdConfig(self.max_norm, self.eps_svd, self.eps_u, self.max_bits_d)


def svd_witness(ctx: Context, m, u, v, d, gamma: int, cfg: SvdConfigPy = SvdConfigPy()) -> dict:
    """Whole witness of examples/svd_example.rs:98-200 (intended one-context
    semantics). Inputs: numpy arrays (host) or contiguous float64 torch CUDA
    tensors on the context's device (then nothing is copied over PCIe)."""
    cfgc = cfg.c()
    cnt = Counts()
    g = _words_arg(gamma)
    dps = [_device_ptr(x) for x in (m, u, v, d)]
    if all(p is not None for p in dps):
        N, M = m.shape
        _after_torch(ctx)
        check(lib().svdw_svd_witness(ctx.handle, *dps, N, M, 1, ct.byref(cfgc), g, ct.byref(cnt)))
        ctx._hold(m, u, v, d)       # pipelined: the stages read them after the call returns
    else:
        arrs = [np.ascontiguousarray(x, dtype=np.float64) for x in (m, u, v, d)]
        N, M = arrs[0].shape
        if arrs[1].shape != (N, N) or arrs[2].shape != (M, M) or arrs[3].size != min(N, M):
            raise SvdwError(-1, "svd_witness: shapes must be m NxM, u NxN, v MxM, d min(N,M)")
        check(lib().svdw_svd_witness(ctx.handle, *[a.ctypes.data for a in arrs], N, M, 0,
                                     ct.byref(cfgc), g, ct.byref(cnt)))
    ctx.last_svd = (int(N), int(M), cfg)        # for collect.plan (shard segment replay)
    return cnt.as_dict()


def verify_mul_witness(ctx: Context, a, b, gamma: int) -> dict:
    """The README.md:32-46 recipe in one call (svdw_verify_mul_witness): loads
    of a and b, c_s = a * b in phase 0, verify_mul(a, b, c_s, gamma) in phase 1.
    Inputs: numpy arrays or contiguous float64 torch tensors on the device."""
    cnt = Counts()
    g = _words_arg(gamma)
    dps = [_device_ptr(x) for x in (a, b)]
    if all(p is not None for p in dps):
        (N, K), M = a.shape, b.shape[1]
        if b.shape[0] != K:
            raise SvdwError(-1, "verify_mul_witness: a.num_col != b.num_rows")
        # (the hand-off to torch's stream inside the call, on the state that runs it)
        check(lib().svdw_verify_mul_witness_on(ctx.handle, _torch_stream(ctx), *dps, N, K, M, g, ct.byref(cnt)))
        ctx._hold(a, b)             # lanes: the call still runs beside the next one
    else:
        arrs = [np.ascontiguousarray(x, dtype=np.float64) for x in (a, b)]
        (N, K), M = arrs[0].shape, arrs[1].shape[1]
        if arrs[1].shape[0] != K:
            raise SvdwError(-1, "verify_mul_witness: a.num_col != b.num_rows")
        check(lib().svdw_verify_mul_witness(ctx.handle, arrs[0].ctypes.data, arrs[1].ctypes.data, N, K, M, 0,
                                            g, ct.byref(cnt)))
    return cnt.as_dict()


def parse_svd_input(src, mode: str = "serde") -> dict:
    """Arrays m, u, d, v of the example's input file (data/matrix.in; a path,
    bytes or str), parsed natively like serde_json's default float path
    ("serde", what examples/svd_example.rs:326-330 reads) or correctly rounded
    ("correct"); svdw_parse_svd_input."""
    if isinstance(src, (bytes, bytearray)):
        text = bytes(src)
    elif isinstance(src, str) and src.lstrip().startswith("{"):
        text = src.encode()
    else:
        with open(src, "rb") as fh:
            text = fh.read()
    md = {"serde": 0, "correct": 1}[mode]
    dims = InputDims()
    check(lib().svdw_parse_svd_input(text, len(text), md, ct.byref(dims), None, None, None, None))
    m = np.empty((dims.m_rows, dims.m_cols))
    u = np.empty((dims.u_rows, dims.u_cols))
    v = np.empty((dims.v_rows, dims.v_cols))
    d = np.empty(dims.d_len)
    check(lib().svdw_parse_svd_input(text, len(text), md, ct.byref(dims), m.ctypes.data,
                                     u.ctypes.data, d.ctypes.data, v.ctypes.data))
    return {"m": m, "u": u, "d": d, "v": v}


def parse_svd_input_device(ctx: "Context", src):
    """parse_svd_input on the device (svdw_parse_svd_input_device, serde mode):
    the text (a path, bytes, str, or a uint8 torch tensor already on the
    context's device) is staged to HBM and parsed there; returns device f64
    torch tensors m, u, d, v, ready for svd_witness (on_device)."""
    import torch
    dev = torch.device("cuda", ctx.device)
    if isinstance(src, torch.Tensor):
        t = src.to(dev, dtype=torch.uint8).contiguous()
    else:
        if isinstance(src, (bytes, bytearray)):
            text = bytes(src)
        elif isinstance(src, str) and src.lstrip().startswith("{"):
            text = src.encode()
        else:
            with open(src, "rb") as fh:
                text = fh.read()
        t = torch.frombuffer(bytearray(text), dtype=torch.uint8).to(dev)
    dims = InputDims()
    n = t.numel()
    _after_torch(ctx)                   # the text may still be in flight on torch's stream
    check(lib().svdw_parse_svd_input_device(ctx._h, t.data_ptr(), n, 0, ct.byref(dims),
                                            None, None, None, None))
    out = {"m": torch.empty((dims.m_rows, dims.m_cols), dtype=torch.float64, device=dev),
           "u": torch.empty((dims.u_rows, dims.u_cols), dtype=torch.float64, device=dev),
           "v": torch.empty((dims.v_rows, dims.v_cols), dtype=torch.float64, device=dev),
           "d": torch.empty(dims.d_len, dtype=torch.float64, device=dev)}
    _after_torch(ctx)                   # the outputs' memory may still be read on torch's stream
    check(lib().svdw_parse_svd_input_device(ctx._h, t.data_ptr(), n, 0, ct.byref(dims),
                                            out["m"].data_ptr(), out["u"].data_ptr(),
                                            out["d"].data_ptr(), out["v"].data_ptr()))
    ctx._hold(t)
    _before_torch(ctx)                  # torch kernels reading m, u, d, v run after the parse
    return out


def plan_svd(N: int, M: int, precision_bits: int, lookup_bits: int,
             cfg: SvdConfigPy = SvdConfigPy()) -> dict:
    """Closed-form cell counts (no device)."""
    cfgc = cfg.c()
    cnt = Counts()
    check(lib().svdw_plan_svd(N, M, precision_bits, lookup_bits, ct.byref(cfgc), ct.byref(cnt)))
    return cnt.as_dict()
