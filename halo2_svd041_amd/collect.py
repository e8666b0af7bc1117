"""Reassembly of a row-sharded witness over torch.distributed.

north_star: row blocks of one matrix shard across the GPUs of a node "with RCCL
all-gather over xGMI only to reassemble the witness column". `svdw_set_shard`
leaves every rank with the row blocks it computed, written at their global
offsets of full-size streams, and `svdw_shard_segments` names them; the union
over the ranks is the single-GPU witness. This module moves the
other ranks' segments in place, straight between the engines' device streams,
with no packing copies:

* ``gather``     - to one root;
* ``all_gather`` - to every rank.

Every rank's segments are closed-form: `plan()` replays the engine's dry
planner once per rank of the world (no device, no exchange; cached per shape)
and checks the own entry against the context's `shard_segments()`. Adjacent
segments of one owner are coalesced into spans, and the whole exchange of a
mode is ONE grouped point-to-point call (`batch_isend_irecv`: one RCCL group
over xGMI on the "nccl" backend), whatever the segment count. With the "gloo"
backend the same code runs on host tensors (CPU tests).

The reference has no multi-device path (its prover is single-threaded), so the
layout to reassemble is the single-context witness of
examples/svd_example.rs:98-200; the exchange itself is plumbing around it.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Sequence, Tuple

import numpy as np

Key = Tuple[int, int]                      # (phase, lookup)
Segment = Tuple[int, int, int, int, int]   # (owner rank, phase, lookup, off, n)

# calls into torch.distributed made by this module (tests assert O(1) per reassembly)
stats = {"collective_calls": 0, "p2p_ops": 0}


class _CudaCells:
    """__cuda_array_interface__ over `n` 32-byte cells at a device pointer."""

    def __init__(self, ptr: int, n: int):
        self.__cuda_array_interface__ = {
            "shape": (n, 32), "typestr": "|u1", "data": (ptr, False),
            "strides": None, "version": 3,
        }


def stream_tensors(ctx, device) -> Dict[Key, "object"]:
    """uint8 [n, 32] torch views of the context's four cell streams (no copy).

    The views alias engine memory: they are valid until the context grows its
    streams (a larger witness) or is closed."""
    import torch
    out = {}
    for phase in (0, 1):
        for lk in (0, 1):
            n = ctx.lookup_len(phase) if lk else ctx.advice_len(phase)
            if n == 0:
                out[(phase, lk)] = torch.empty((0, 32), dtype=torch.uint8, device=device)
                continue
            ptr = ctx.lookup_device_ptr(phase) if lk else ctx.advice_device_ptr(phase)
            out[(phase, lk)] = torch.as_tensor(_CudaCells(ptr, n), device=device)
    return out


def coalesce(segs: Sequence[Segment]) -> List[Segment]:
    """Merge segments of one owner that touch in the same stream."""
    out: List[Segment] = []
    for s in sorted(segs, key=lambda s: (s[1], s[2], s[3])):
        if out and out[-1][:3] == s[:3] and out[-1][3] + out[-1][4] == s[3]:
            o = out[-1]
            out[-1] = (o[0], o[1], o[2], o[3], o[4] + s[4])
        else:
            out.append(s)
    return out


_plan_cache: Dict[tuple, List[Segment]] = {}


def planned_segments(N: int, M: int, P: int, LB: int, world: int, cfg=None,
                      layout_opts=None) -> List[Segment]:
    """Every rank's owned segments of a row-sharded svd_witness (N x M, P, LB)
    from the dry planner (Context(device=-1)), coalesced, in an order every
    rank computes identically. layout_opts: the engine options of the witness
    that move cells (zk.LAYOUT_OPTIONS, e.g. rlc_prefix), replayed on the dry
    contexts."""
    from . import zk
    cfg = cfg or zk.SvdConfigPy()
    opts = tuple(sorted((layout_opts or {}).items()))
    key = (N, M, P, LB, world, cfg.max_norm, cfg.eps_svd, cfg.eps_u, cfg.max_bits_d, opts)
    if key not in _plan_cache:
        r_ = min(N, M)
        m, u, v, d = np.zeros((N, M)), np.zeros((N, N)), np.zeros((M, M)), np.zeros(r_)
        segs: List[Segment] = []
        for r in range(world):
            c = zk.Context(device=-1, precision_bits=P, lookup_bits=LB)
            try:
                for name, val in opts:
                    c.set_option(name, val)
                c.set_shard(r, world)
                zk.svd_witness(c, m, u, v, d, 1, cfg)
                segs += [(r, ph, lk, off, n) for ph, lk, off, n in c.shard_segments() if n]
            finally:
                c.close()
        _plan_cache[key] = coalesce(segs)
    return _plan_cache[key]


@dataclass
class Plan:
    mode: str
    rank: int
    world: int
    root: int
    segments: List[Segment]
    sends: List[Tuple[int, Segment]] = field(default_factory=list)   # (peer, segment)
    recvs: List[Tuple[int, Segment]] = field(default_factory=list)
    collectives: int = 1              # grouped calls per reassembly
    moved_cells: int = 0              # cells this rank sends + receives


def plan(ctx, rank: int, world: int, mode: str = "gather", root: int = 0) -> Plan:
    """Exchange plan for the last svd_witness of `ctx` (row-sharded rank `rank`)."""
    if mode not in ("gather", "all_gather"):
        raise ValueError(f"unknown reassembly mode {mode!r}")
    last = getattr(ctx, "last_svd", None)
    if last is None:
        raise RuntimeError("collect.plan needs a row-sharded svd_witness on this context first")
    N, M, cfg = last
    segs = planned_segments(N, M, ctx.precision_bits, ctx.lookup_bits, world, cfg,
                            getattr(ctx, "layout_opts", None))
    mine = coalesce([(rank, ph, lk, off, n) for ph, lk, off, n in ctx.shard_segments() if n])
    if mine != [s for s in segs if s[0] == rank]:
        raise RuntimeError("collect.plan: the context's shard segments differ from the planner's")
    p = Plan(mode, rank, world, root, segs)
    for s in segs:
        owner = s[0]
        if mode == "gather":
            if owner == root:
                continue
            if rank == owner:
                p.sends.append((root, s))
            elif rank == root:
                p.recvs.append((owner, s))
        else:
            if rank == owner:
                p.sends += [(peer, s) for peer in range(world) if peer != owner]
            else:
                p.recvs.append((owner, s))
    p.moved_cells = sum(s[4] for _, s in p.sends) + sum(s[4] for _, s in p.recvs)
    return p


def exchange(streams: Dict[Key, "object"], p: Plan, group=None) -> int:
    """Run the plan's sends and receives as one grouped point-to-point call.
    Returns the cells this rank moved."""
    import torch.distributed as dist
    ops = []
    # a deterministic order that pairs every send with its receive: sorted by
    # (segment, peer) on both sides
    for peer, (owner, ph, lk, off, n) in sorted(p.sends + p.recvs, key=lambda t: (t[1], t[0])):
        view = streams[(ph, lk)][off:off + n]
        if owner == p.rank:
            ops.append(dist.P2POp(dist.isend, view, peer, group=group))
        else:
            ops.append(dist.P2POp(dist.irecv, view, owner, group=group))
    if ops:
        stats["collective_calls"] += 1
        stats["p2p_ops"] += len(ops)
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    return p.moved_cells


def reassemble(ctx, p: Plan, group=None, device=None) -> int:
    """Reassemble the last (sharded) witness of `ctx` with plan `p` (from plan()).
    Stream-ordered, no host wait: torch's current stream (which the RCCL
    exchange follows) first waits on the device for the engine's queued
    witness, and the engine's streams then wait for the exchange, so a next
    witness cannot overwrite cells still being sent or received."""
    import torch
    from . import zk
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    zk._before_torch(ctx)
    moved = exchange(stream_tensors(ctx, device), p, group)
    zk._after_torch(ctx)
    return moved
