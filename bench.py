#!/usr/bin/env python3
"""bench.py — SVD-verify witness generation throughput (advice cells / s).

One step = the whole witness of examples/svd_example.rs:98-200 for one
N x M matrix (ZkMatrix::new m,u,v + ZkVector::new d, check_svd_phase0 into
phase 0, check_svd_phase1 into phase 1), f64 inputs resident in HBM when the
clock starts, complete advice + lookup streams resident in HBM when it stops.

Default workload: BASELINE.json configs[3] shape (1024 x 1024, PRECISION_BITS=63,
LOOKUP_BITS=19) on one GPU. With --gpus N (torch.distributed.run, one rank per
GPU) every rank generates its own matrix (independent objects, no data-path
collective): weak scaling, value = cells of all ranks / max-over-ranks time.

Output: ONE JSON line on rank 0 (driver contract), including
  roofline     dominant kernel (k_stage, the cell-program stage kernel), from
               HIP events the engine records around each of its launches on
               its own stream during the timed steps (svdw_profile_*; only that
               kernel is bracketed, so the clock sees two event packets per
               stage launch and nothing else),
  cpu_baseline the single-threaded C oracle (oracle/svdw_oracle.c, a port of
               the reference algorithm) on a bounded row sample, rank 0 only.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
ORACLE_DIR = os.path.join(ROOT, "oracle")   # cpu_baseline leg only

P_MOD = 21888242871839275222246405745257275088548364400416034343698204186575808495617
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
METRIC = "advice cells/sec (SVD-verify witness gen, N×N) at 1/2/4/8 MI355X"


def gen_input(N, M, seed):
    """input-creator.py:23-30 recipe with a seeded RandomState."""
    rs = np.random.RandomState(seed)
    m = rs.uniform(-10, 10, size=(N, M))
    m = m / np.linalg.norm(m, ord=2) * rs.uniform(1, 100)
    U, D, V = np.linalg.svd(m)
    return m, U, D, V


def gamma_for(seed) -> int:
    return int.from_bytes(hashlib.sha256(f"svdw-gamma-{seed}".encode()).digest(), "little") % P_MOD


def roofline_from_profile(stats, steps):
    """Dominant kernel (largest total time) aggregated over all its launches."""
    by_kernel = {}
    for s in stats:
        k = s["name"].split(":")[0]
        agg = by_kernel.setdefault(k, {"launches": 0, "total_ms": 0.0, "bytes": 0.0, "ops": 0.0})
        for f in ("launches", "total_ms", "bytes", "ops"):
            agg[f] += s[f]
    name, agg = max(by_kernel.items(), key=lambda kv: kv[1]["total_ms"])
    avg_ms = agg["total_ms"] / agg["launches"]
    bytes_per_launch = agg["bytes"] / agg["launches"]
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
    breakdown = {k: round(v["total_ms"] / steps, 4) for k, v in
                 sorted(by_kernel.items(), key=lambda kv: -kv[1]["total_ms"])}
    return name, {
        "bound": "hbm",
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": None,
        "kernel": name,
        "avg_launch_ms": round(avg_ms, 5),
        "bytes_per_launch": round(bytes_per_launch),
        "launches_per_step": agg["launches"] / steps,
    }, breakdown


def rank_workload(seed, rank, N, M):
    """Rank r witnesses its own matrix (seed + r): independent objects, no
    data-path exchange (north_star: matrices shard embarrassingly)."""
    m, u, d, v = gen_input(N, M, seed + rank)
    return m, u, d, v, gamma_for(seed + rank)


def reduce_over_ranks(elapsed, cells_step, dist, device):
    """Job clock = slowest rank (max), cells = all ranks (sum). dist None: 1 rank."""
    if dist is None:
        return elapsed, float(cells_step)
    import torch
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    c = torch.tensor([float(cells_step)], dtype=torch.float64, device=device)
    dist.all_reduce(c, op=dist.ReduceOp.SUM)
    return float(t.item()), float(c.item())


def pmc_traffic(kernel, N, M, P, LB):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC
    summary of this exact workload (profiles/*_pmc_summary.json, written by
    tools/pmc_summary.py from separate --pmc FETCH_SIZE / WRITE_SIZE passes)."""
    import glob
    want = {"N": N, "M": M, "P": P, "LB": LB}
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_summary.json")), reverse=True):
        try:
            with open(f) as fh:
                s = json.load(fh)
        except (OSError, ValueError):
            continue
        if s.get("config") == want and kernel in s.get("kernels", {}):
            return s["kernels"][kernel]["traffic_per_launch"], os.path.relpath(f, ROOT)
    return None, None


def cpu_baseline(m, u, v, d, P, LB, g, rows):
    sys.path.insert(0, ORACLE_DIR)
    import corc  # oracle/ — the checker / reported baseline only
    t0 = time.perf_counter()
    a0, l0, a1 = corc.svd_witness(m, u, v, d, P, LB, g, row_lim=rows)
    dt = time.perf_counter() - t0
    cells = a0.shape[0] + a1.shape[0]
    return {"value": round(cells / dt, 1), "unit": "advice cells/s", "cores": 1, "kind": "port",
            "sample": (f"oracle/svdw_oracle.c single thread, same {m.shape[0]}x{m.shape[1]} P={P} "
                       f"witness restricted to rows [0,{rows}) of every row-parallel stage "
                       f"(+ all loads and d checks): {cells} advice cells in {dt:.2f} s"),
            "seconds": round(dt, 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--m", type=int, default=None)
    ap.add_argument("--p", type=int, default=63)
    ap.add_argument("--lb", type=int, default=19)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-rows", type=int, default=128)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true",
                    help="skip the engine's event profiler in the timed region")
    ap.add_argument("--profile-prefix", default="k_stage",
                    help="kernel-name prefix the timed-region profiler records ('' = all)")
    ap.add_argument("--breakdown", action="store_true", help="print per-kernel ms/step to stderr")
    ap.add_argument("--shard", choices=["replicas", "rows"], default="replicas",
                    help="N>1: one matrix per rank (weak scaling, default) or one matrix "
                         "row-block sharded over the ranks (strong scaling, BASELINE config 4)")
    ap.add_argument("--gather", choices=["none", "root", "all"], default="none",
                    help="--shard rows: also time reassembling the witness after each step "
                         "(RCCL point-to-point gather to rank 0, or all-gather by segment "
                         "broadcasts), reported beside the witness-only value")
    ap.add_argument("--no-check", action="store_true",
                    help="skip the untimed device constraint check of the last witness")
    ap.add_argument("--opt", action="append", default=[],
                    help="engine tuning option name=value (svdw_set_option), repeatable")
    args = ap.parse_args()
    N = args.n
    M = args.m or N

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    # Rehearsal on fewer GPUs than ranks (e.g. a 1-GPU box): BENCH_DIST_BACKEND=gloo
    # and ranks share devices round-robin. Timings are then not per-GPU numbers.
    backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(torch.cuda.device_count(), 1)
    dist = None
    if world > 1:
        import torch.distributed as dist  # noqa: F811
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(local)

    import halo2_svd041_amd as hs

    rows_mode = args.shard == "rows" and world > 1
    m, u, d, v, g = rank_workload(args.seed, 0 if rows_mode else rank, N, M)
    dev = torch.device("cuda", local)
    dm, du, dv, dd = (torch.tensor(np.ascontiguousarray(x), dtype=torch.float64, device=dev)
                      for x in (m, u, v, d))
    torch.cuda.synchronize()
    ctx = hs.Context(device=local, precision_bits=args.p, lookup_bits=args.lb)
    for kv in args.opt:
        name, _, val = kv.partition("=")
        ctx.set_option(name, int(val))
    if rows_mode:
        ctx.set_shard(rank, world)

    for _ in range(args.warmup):
        cnt = hs.svd_witness(ctx, dm, du, dv, dd, g)
    ctx.sync()

    if not args.no_profile:
        ctx.profile(True, args.profile_prefix)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        cnt = hs.svd_witness(ctx, dm, du, dv, dd, g)
    ctx.sync()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    stats = ctx.profile_collect() if not args.no_profile else []

    # The same kernel alone on the GPU (one untimed step with both streams
    # serialised): its intrinsic rate, reported beside the contended in-step rate.
    solo = None
    if not args.no_profile and not rows_mode:
        ctx.set_option("overlap", 0)
        ctx.set_option("phase1_overlap", 0)
        ctx.profile(True, args.profile_prefix)
        hs.svd_witness(ctx, dm, du, dv, dd, g)
        ctx.sync()
        solo_stats = ctx.profile_collect()
        ctx.profile(False)
        ctx.set_option("overlap", 1)
        ctx.set_option("phase1_overlap", 1)
        if solo_stats:
            _, solo, _ = roofline_from_profile(solo_stats, 1)

    reasm = None
    if rows_mode and args.gather != "none":
        # witness + reassembly per step, timed like the witness-only loop
        from halo2_svd041_amd import collect
        mode = "gather" if args.gather == "root" else "all_gather"
        collect.reassemble(ctx, rank, world, mode)        # warm the communicator
        dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        moved = 0
        for _ in range(args.steps):
            hs.svd_witness(ctx, dm, du, dv, dd, g)
            moved = collect.reassemble(ctx, rank, world, mode)["cells"]
        torch.cuda.synchronize()
        dist.barrier()
        el2 = time.perf_counter() - t1
        el2, moved_all = reduce_over_ranks(el2, moved, dist, dev if backend == "nccl"
                                           else torch.device("cpu"))
        extra = el2 / args.steps - elapsed / args.steps
        reasm = {"mode": mode, "ms_per_step_with_reassembly": round(el2 / args.steps * 1e3, 4),
                 "value_with_reassembly": round(cells_step * args.steps / el2, 1),
                 "reassembly_ms": round(extra * 1e3, 4),
                 "moved_GB_per_step": round(moved_all * 32 / 1e9 / (2 if mode == "gather" else world), 3)}

    # Untimed: the device constraint checker over the last witness (svdw_check_gates;
    # a row-sharded rank checks the rows it owns), summed over the ranks.
    check = None
    if not args.no_check:
        r = ctx.check_gates()
        keys = sorted(r)
        vals = [float(r[k]) for k in keys]
        if dist is not None:
            t = torch.tensor(vals, dtype=torch.float64,
                             device=dev if backend == "nccl" else torch.device("cpu"))
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
            vals = t.tolist()
        check = {k: int(x) for k, x in zip(keys, vals)}
        check["ok"] = check["gate_failures"] + check["copy_failures"] + check["lookup_failures"] == 0

    cells_step = cnt["advice0"] + cnt["advice1"]
    elapsed, cells_all = reduce_over_ranks(elapsed, cells_step, dist,
                                           dev if backend == "nccl" else torch.device("cpu"))
    if rows_mode:
        cells_all = float(cells_step)        # one witness, split over the ranks
    total_cells = cells_all * args.steps
    value = total_cells / elapsed

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "advice cells/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if rows_mode else "weak",
            "vs_baseline": None,
            "dtype": "bn254_fr (u32 limbs; exact multi-modular int8 MFMA GEMM)",
            "data": "synthetic (input-creator.py recipe, seeded; gamma = sha256 mod p)",
            "config": {
                "workload": (f"svd_verify_witness N={N} M={M} PRECISION_BITS={args.p} "
                             f"LOOKUP_BITS={args.lb}, "
                             + ("one matrix row-sharded over the GPUs" if rows_mode
                                else "one matrix per GPU")),
                "N": N, "M": M, "precision_bits": args.p, "lookup_bits": args.lb,
                "advice_cells_per_matrix": cells_step,
                "lookup_cells_per_matrix": cnt["lookup0"] + cnt["lookup1"],
                "parallelism": (f"row blocks x{world} of one matrix (witness kept sharded; "
                                f"reassembly timed separately with --gather)"
                                if rows_mode else f"replicas x{world} (no data-path collective)"),
            },
        }
        if stats:
            kname, roof, breakdown = roofline_from_profile(stats, args.steps)
            # the committed PMC summary is for the whole witness on one GPU
            traffic, src = (None, None) if rows_mode else pmc_traffic(kname, N, M, args.p,
                                                                         args.lb)
            if traffic is not None:
                roof["traffic"] = traffic
                roof["traffic_source"] = src
            if solo is not None and solo["kernel"] == roof["kernel"]:
                roof["standalone"] = {k: solo[k] for k in ("achieved", "frac", "avg_launch_ms")}
                roof["standalone"]["note"] = ("same kernel, one extra untimed step with the "
                                              "streams serialised (no concurrent products/scans)")
            # SURVEY.md §8(d) stage (i): the whole step against HBM, algorithmic
            # bytes = 32 B per advice + lookup cell + 8 B per f64 input entry
            if not rows_mode:
                step_bytes = (32 * (cells_step + cnt["lookup0"] + cnt["lookup1"])
                              + 8 * (N * M + N * N + M * M + min(N, M)))
                ach = step_bytes / (elapsed / args.steps) / 1e9
                roof["step"] = {"bytes": step_bytes, "achieved": round(ach, 1),
                                "frac": round(ach / roof["peak"], 4),
                                "note": "whole witness per step (all kernels, both streams)"}
            out["roofline"] = roof
            if args.breakdown:
                print(json.dumps({"ms_per_step_by_kernel": breakdown,
                                  "stats": stats}, indent=1), file=sys.stderr)
        if reasm is not None:
            out["reassembly"] = reasm
        if check is not None:
            out["witness_check"] = check
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(m, u, v, d, args.p, args.lb, g, args.cpu_rows)
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
