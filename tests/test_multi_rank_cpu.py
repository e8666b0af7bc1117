"""Multi-GPU path of bench.py on CPU: two gloo ranks run the same replica logic
(own matrix per rank, max-over-ranks clock, summed cells) with the engine's
dry planner standing in for the device (no GPU here)."""
import os
import socket
import sys

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


def _worker(rank, world, port, out):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        import halo2_svd041_amd as hs
        N = M = 24
        m, u, d, v, g = bench.rank_workload(7, rank, N, M)
        cnt = hs.plan_svd(N, M, 63, 19)              # dry planner: same layout per rank
        cells = cnt["advice0"] + cnt["advice1"]
        elapsed = 1.0 + rank                          # rank 1 is the slow one
        t, c = bench.reduce_over_ranks(elapsed, cells, dist, torch.device("cpu"))
        out[rank] = (t, c, cells, float(m[0, 0]), g)
    finally:
        dist.destroy_process_group()


def test_two_rank_replicas_gloo():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    (t0, c0, cells0, m00, g0), (t1, c1, cells1, m01, g1) = out[0], out[1]
    assert t0 == t1 == 2.0                            # max over ranks
    assert c0 == c1 == cells0 + cells1                # whole-job cells
    assert cells0 == cells1
    assert m00 != m01 and g0 != g1                    # independent matrices per rank


def test_single_rank_reduce_is_identity():
    sys.path.insert(0, ROOT)
    import bench
    assert bench.reduce_over_ranks(0.5, 1234, None, None) == (0.5, 1234.0)


@pytest.mark.parametrize("extra", [[], ["--shard", "replicas"]])
def test_bench_gpus_flag_launches_ranks(extra):
    """`bench.py --gpus 2` outside torch.distributed starts two ranks itself (a
    torch.distributed.run child); --dry rehearses them on CPU (gloo + planner)."""
    import json
    import subprocess
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry",
                        "--n", "32", "--steps", "2", "--warmup", "1"] + extra,
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout                 # rank 0 prints one JSON line
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["ranks"] == 2
    assert out["scaling"] == ("weak" if extra else "strong")
    assert out["config"]["backend"] == "gloo"
    # the whole-witness roofline fraction is on every line; in rows mode against
    # N x peak, with the per-rank times and the reassembly record
    step = out["roofline"]["step"]
    assert step["bytes"] > 0 and step["frac"] is not None
    if not extra:
        assert step["peak"] == 2 * 8000.0
        assert len(step["rank_ms"]) == 2 and step["rank_ms_min"] <= step["rank_ms_max"]
        r = out["reassembly"]
        assert r["mode"] == "gather" and r["moved_GB_per_step"] > 0
        assert r["ms_per_step_with_reassembly"] > 0
    else:
        assert "reassembly" not in out
