"""Round-6 diagnostic: one rank with an RCCL process group initialised (as
bench.py --gpus N sets it up, before the engine context) against no process
group, same loop (fresh gamma, 3 warm-up steps, 30 timed). RCCL's streams take
hardware queues first; does a context stream end up sharing one that blocks?"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from bench import gen_input, step_gammas  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dist", type=int, default=1)
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--p", type=int, default=63)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--shard", type=int, default=0, help="row shard world (rank 0), 0: unsharded")
    ap.add_argument("--ctx-first", type=int, default=0, help="create the engine context before the group")
    a = ap.parse_args()
    import torch
    import halo2_svd041_amd as hs
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    ctx = hs.Context(device=0, precision_bits=a.p, lookup_bits=19) if a.ctx_first else None
    dist = None
    if a.dist:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29611")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        dist.barrier()
    if ctx is None:
        ctx = hs.Context(device=0, precision_bits=a.p, lookup_bits=19)
    if a.shard:
        ctx.set_shard(0, a.shard)
    m, u, d, v = gen_input(a.n, a.n, 0)
    inp = tuple(torch.tensor(np.ascontiguousarray(x), dtype=torch.float64, device=dev) for x in (m, u, v, d))
    for g in step_gammas(0, 3, offset=10 ** 6):
        hs.svd_witness(ctx, *inp, g)
    ctx.sync()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for g in step_gammas(0, a.steps):
        hs.svd_witness(ctx, *inp, g)
    ctx.sync()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    ms = (time.perf_counter() - t0) / a.steps * 1e3
    print(json.dumps({"dist": a.dist, "ctx_first": a.ctx_first, "shard": a.shard, "n": a.n, "ms": round(ms, 4)}))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
