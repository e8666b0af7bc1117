"""Witness reassembly (halo2_svd041_amd.collect) on CPU: gloo ranks holding only
their own row blocks of a row-sharded witness (segments from the engine's dry
planner, the same layout svdw_set_shard gives on the GPU) end with the whole
witness after gather (root only) and all_gather (every rank)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _expected(key, n):
    """Distinct, recognisable cell bytes per (stream, cell index)."""
    ph, lk = key
    idx = np.arange(n, dtype=np.uint64)[:, None] * 131 + np.arange(32, dtype=np.uint64)[None, :]
    return torch.from_numpy(((idx + 7 * ph + 3 * lk) % 251).astype(np.uint8))


def _worker(rank, world, port, mode, shape, out, opts=None):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import halo2_svd041_amd as hs
        from halo2_svd041_amd import collect
        from conftest import gen_svd_input
        N, M, P = shape
        m, u, d, v = gen_svd_input(N, M, seed=3)
        ctx = hs.Context(device=-1, precision_bits=P, lookup_bits=19)   # planner
        for k, val in (opts or {}).items():
            ctx.set_option(k, val)
        ctx.set_shard(rank, world)
        cnt = hs.svd_witness(ctx, m, u, v, d, 99)
        sizes = {(0, 0): cnt["advice0"], (1, 0): cnt["advice1"],
                 (0, 1): cnt["lookup0"], (1, 1): cnt["lookup1"]}
        plan = collect.plan(ctx, rank, world, mode)          # planner replay, no exchange
        segs = plan.segments
        streams = {k: torch.zeros((n, 32), dtype=torch.uint8) for k, n in sizes.items()}
        for owner, ph, lk, off, n in segs:                    # this rank's own cells only
            if owner == rank:
                streams[(ph, lk)][off:off + n] = _expected((ph, lk), sizes[(ph, lk)])[off:off + n]
        calls0 = collect.stats["collective_calls"]
        moved = collect.exchange(streams, plan)
        calls = collect.stats["collective_calls"] - calls0
        ok = {}
        for k, n in sizes.items():
            ok[k] = bool(torch.equal(streams[k], _expected(k, n)))
        out[rank] = (ok, moved, len(segs), calls, len(plan.sends) + len(plan.recvs))
        ctx.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["gather", "all_gather"])
@pytest.mark.parametrize("world,shape,opts", [(2, (12, 12, 63), None), (3, (9, 13, 32), None),
                                              (2, (12, 12, 63), {"rlc_prefix": 1}),
                                              (3, (9, 13, 32), {"rlc_prefix": 1})])
def test_reassembly_gloo(mode, world, shape, opts):
    """rlc_prefix shifts every phase-1 segment by two cells: the plan's dry
    replay must see it (the option is recorded on the Python Context)."""
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, mode, shape, out, opts), nprocs=world, join=True)
    for rank in range(world):
        ok, moved, nseg, calls, nops = out[rank]
        assert nseg >= world
        # one grouped exchange per reassembly, whatever the segment count
        assert calls == (1 if nops else 0)
        if mode == "all_gather" or rank == 0:
            assert all(ok.values()), (rank, ok)
        else:                                        # non-roots keep their own rows only
            assert not all(ok.values())
        assert moved > 0
