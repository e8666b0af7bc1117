"""Reassembly of a row-sharded witness over torch.distributed.

north_star: row blocks of one matrix shard across the GPUs of a node "with RCCL
all-gather over xGMI only to reassemble the witness column". `svdw_set_shard`
leaves every rank with the row blocks it computed, written at their global
offsets of full-size streams, and `svdw_shard_segments` names them; the union
over the ranks is the single-GPU witness. This module moves the
other ranks' segments in place, straight between the engines' device streams:

* ``gather``   - to one root (point-to-point sends, one per owned segment);
* ``all_gather`` - to every rank (each owner broadcasts its segments: on the
  "nccl" backend these are RCCL collectives over xGMI).

The reference has no multi-device path (its prover is single-threaded), so the
layout to reassemble is the single-context witness of
examples/svd_example.rs:98-200; the exchange itself is plumbing around it.
With the "gloo" backend the same code runs on host tensors (CPU tests).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

Key = Tuple[int, int]                      # (phase, lookup)
Segment = Tuple[int, int, int, int, int]   # (owner rank, phase, lookup, off, n)


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


def all_segments(own: Sequence[Tuple[int, int, int, int]], rank: int, world: int,
                 group=None) -> List[Segment]:
    """Every rank's owned segments (all_gather_object), in a rank-major order
    that all ranks agree on."""
    import torch.distributed as dist
    per_rank: List[Optional[list]] = [None] * world
    dist.all_gather_object(per_rank, [tuple(int(x) for x in s) for s in own], group=group)
    return [(r, ph, lk, off, n) for r in range(world) for (ph, lk, off, n) in per_rank[r] if n]


def gather(streams: Dict[Key, "object"], segs: Sequence[Segment], rank: int, root: int = 0,
           group=None) -> int:
    """Root receives every segment it does not own into `streams`; owners send.
    Returns the number of cells this rank moved (sent or received)."""
    import torch.distributed as dist
    ops, moved = [], 0
    for owner, ph, lk, off, n in segs:
        if owner == root:
            continue
        view = streams[(ph, lk)][off:off + n]
        if rank == owner:
            ops.append(dist.P2POp(dist.isend, view, root, group=group))
            moved += n
        elif rank == root:
            ops.append(dist.P2POp(dist.irecv, view, owner, group=group))
            moved += n
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    return moved


def all_gather(streams: Dict[Key, "object"], segs: Sequence[Segment], group=None) -> int:
    """Every rank ends with the whole witness: each owner broadcasts its
    segments in place. Returns the cells broadcast in total."""
    import torch.distributed as dist
    total = 0
    for owner, ph, lk, off, n in segs:
        dist.broadcast(streams[(ph, lk)][off:off + n], src=owner, group=group)
        total += n
    return total


def reassemble(ctx, rank: int, world: int, mode: str = "gather", root: int = 0,
               group=None, device=None) -> dict:
    """Reassemble the last (sharded) witness of `ctx` with the mode's collective.
    Returns {"cells": moved, "segments": count}."""
    import torch
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    ctx.sync()
    segs = all_segments(ctx.shard_segments(), rank, world, group)
    streams = stream_tensors(ctx, device)
    if mode == "gather":
        cells = gather(streams, segs, rank, root, group)
    elif mode == "all_gather":
        cells = all_gather(streams, segs, group)
    else:
        raise ValueError(f"unknown reassembly mode {mode!r}")
    torch.cuda.synchronize(device)
    return {"cells": cells, "segments": len(segs)}
