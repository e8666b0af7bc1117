"""Reassembly on the device: the engine's streams as torch views
(collect.stream_tensors), and a two-shard witness moved into one context's
streams segment by segment equals the unsharded witness bit for bit (the
transport of the same segments over RCCL / gloo is covered by
tests/test_collect_cpu.py)."""
import numpy as np
import pytest
import torch

from conftest import gamma_for, gen_svd_input

pytestmark = pytest.mark.gpu


def test_stream_views_alias_engine_memory(gpu_ctx_factory):
    from halo2_svd041_amd import collect
    import halo2_svd041_amd as hs
    ctx = gpu_ctx_factory(63)
    m, u, d, v = gen_svd_input(7, 5, seed=11)
    hs.svd_witness(ctx, m, u, v, d, gamma_for(11))
    ctx.sync()
    views = collect.stream_tensors(ctx, torch.device("cuda", 0))
    for (ph, lk), t in views.items():
        host = ctx.lookups(ph) if lk else ctx.advice(ph)
        got = t.cpu().numpy().view(np.uint64).reshape(-1, 4) if t.numel() else np.zeros((0, 4), np.uint64)
        assert np.array_equal(got, host.reshape(-1, 4)), (ph, lk)


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_union_equals_single(gpu_ctx_factory, world):
    from halo2_svd041_amd import collect
    import halo2_svd041_amd as hs
    N, M, P = 19, 14, 42
    m, u, d, v = gen_svd_input(N, M, seed=5)
    g = gamma_for(5)
    full = gpu_ctx_factory(P)
    hs.svd_witness(full, m, u, v, d, g)
    full.sync()
    dev = torch.device("cuda", 0)
    shards = []
    for r in range(world):
        c = hs.Context(device=0, precision_bits=P, lookup_bits=19)
        c.set_shard(r, world)
        hs.svd_witness(c, m, u, v, d, g)
        c.sync()
        shards.append(c)
    try:
        root = collect.stream_tensors(shards[0], dev)
        for r in range(1, world):
            src = collect.stream_tensors(shards[r], dev)
            for ph, lk, off, n in shards[r].shard_segments():
                root[(ph, lk)][off:off + n].copy_(src[(ph, lk)][off:off + n])
        torch.cuda.synchronize()
        want = collect.stream_tensors(full, dev)
        for k in want:
            assert torch.equal(root[k], want[k]), k
    finally:
        for c in shards:
            c.close()
