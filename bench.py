#!/usr/bin/env python3
"""bench.py — SVD-verify witness generation throughput (advice cells / s).

Workloads (BASELINE.json configs):
  svd        (default) one step = the whole witness of examples/svd_example.rs:98-200
             for one N x M matrix (ZkMatrix::new m,u,v + ZkVector::new d,
             check_svd_phase0 into phase 0, check_svd_phase1 into phase 1).
             1 GPU: configs[3]'s shape 1024 x 1024, PRECISION_BITS=63.
             --n 512 --p 32: configs[2]; --n 2048 --m 1024 --p 32: configs[4].
  verify_mul the README.md:32-46 recipe: ZkMatrix::new a, b; c_s =
             honest_prover_mat_mul(a, b) in phase 0; verify_mul(a, b, c_s, gamma)
             in phase 1 (configs[1]: 256 x 256, PRECISION_BITS=32).
f64 inputs are resident in HBM when the clock starts, the complete advice +
lookup streams are resident in HBM when it stops. Every step draws a fresh
gamma (sha256(seed, step) mod p), as a prover gets a fresh challenge per witness.

Multi-GPU: `--gpus N` without a torch.distributed environment starts N ranks
itself (a torch.distributed.run child process; this process never touches the
GPU) and exits with its status. One rank per GPU:
  --shard rows      (default for N > 1, configs[3]) one matrix row-block sharded
                    over the ranks (svdw_set_shard): strong scaling, the witness
                    stays sharded-resident; --gather root|all also times its
                    reassembly over RCCL, reported beside the witness-only value.
  --shard replicas  (configs[4]) one matrix per rank, no data-path collective:
                    weak scaling, value = cells of all ranks / max-over-ranks time.
--dry rehearses the launch and the rank logic on CPU (gloo, the engine's dry
planner instead of a device): no GPU, timings are host planning only.

Output: ONE JSON line on rank 0 (driver contract), including
  roofline     dominant kernel, from HIP events the engine records around each
               of its launches on its own stream during the timed steps
               (svdw_profile_*; filtered by --profile-prefix),
  cpu_baseline the single-threaded C oracle (oracle/svdw_oracle.c, a port of the
               reference algorithm) on a bounded sample of the same workload, in a
               child process pinned to core 0 (taskset -c 0) that runs to
               completion before this process first touches the GPU; rank 0, N=1.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import shutil
import socket
import subprocess
import sys
import time

import numpy as np

# Hardware queues per process (read by HIP at its first call, so before torch
# touches the GPU). The engine runs three streams and torch one; a rank's RCCL
# group adds its own, and with the box default of 4 some of them share a queue
# with a context stream: tools/r6/rccl1.py with the group created before the
# context, 1024^2 1.818 -> 1.804 ms and the 8-way rank 0.306 -> 0.302 ms at 8
# queues; created after it, 1.92 -> 1.80 and 0.368 -> 0.309 ms (DESIGN.md,
# round 6, r6w). One GPU without a group is unchanged (512^2 0.375 ms both).
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")

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


def gen_matmul_input(N, K, M, seed):
    """README.md:32-46 recipe operands: a (N x K), b (K x M), entries U(-1, 1)."""
    rs = np.random.RandomState(seed)
    return rs.uniform(-1, 1, size=(N, K)), rs.uniform(-1, 1, size=(K, M))


def gamma_for(seed) -> int:
    return int.from_bytes(hashlib.sha256(f"svdw-gamma-{seed}".encode()).digest(), "little") % P_MOD


def step_gammas(seed, steps, offset=0):
    """A fresh challenge per witness (the RLC gamma of svd_example.rs:181-184)."""
    return [gamma_for(f"{seed}-{offset + i}") for i in range(steps)]


def stage_stream_rate(stats, steps):
    """The k_stage launches of the stream that runs most of them (the engine
    tags every launch with its stream: @cell, @s2, @s3). Pipelined, that is
    st2, which carries every stage kernel of a call back to back: its busy time
    per step and its write rate while busy, against the step."""
    per = {}
    for s in stats:
        if not s["name"].startswith("k_stage") or "@" not in s["name"]:
            continue
        tag = s["name"].rsplit("@", 1)[1]
        agg = per.setdefault(tag, {"ms": 0.0, "bytes": 0.0, "launches": 0})
        agg["ms"] += s["total_ms"]
        agg["bytes"] += s["bytes"]
        agg["launches"] += s["launches"]
    if not per:
        return None
    tag, agg = max(per.items(), key=lambda kv: kv[1]["ms"])
    ach = agg["bytes"] / (agg["ms"] * 1e-3) / 1e9
    return {"stream": tag, "achieved": round(ach, 1), "frac": round(ach / HBM_PEAK_GBS, 4),
            "busy_ms_per_step": round(agg["ms"] / steps, 4), "launches_per_step": agg["launches"] / steps,
            "note": "k_stage launches of the stream carrying most of them: busy time per step and "
                    "its cell write rate while busy"}


def roofline_from_profile(stats, steps):
    """Dominant kernel (largest total time) aggregated over all its launches."""
    by_kernel = {}
    for s in stats:
        k = s["name"].split(":")[0].split("@")[0]
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


def sources_sha16():
    """Hash of the engine and kernel sources (halo2_svd041_amd/csrc): a PMC
    summary is only evidence for the build it was collected on."""
    import glob
    h = hashlib.sha256()
    for f in sorted(glob.glob(os.path.join(ROOT, "halo2_svd041_amd", "csrc", "*"))):
        if f.endswith((".hip", ".cpp", ".hpp")):
            h.update(os.path.basename(f).encode())
            with open(f, "rb") as fh:
                h.update(fh.read())
    return h.hexdigest()[:16]


def pmc_traffic(kernel, workload, N, M, P, LB, world=1, rank=0):
    """HBM bytes per launch of `kernel` from a committed rocprofv3 PMC summary
    of this exact workload AND these kernel sources (profiles/*_pmc_summary.json,
    written by tools/pmc_summary.py from separate --pmc FETCH_SIZE / WRITE_SIZE
    passes; a summary of other sources is refused). Returns (bytes, file, note)."""
    import glob
    want = {"N": N, "M": M, "P": P, "LB": LB}
    if world > 1:
        want.update({"world": world, "rank": rank})
    sha = sources_sha16()
    stale = []
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_summary.json")), reverse=True):
        try:
            with open(f) as fh:
                s = json.load(fh)
        except (OSError, ValueError):
            continue
        ks = s.get("kernels", {})
        # the profiler's family name (k_matvec_scan) or rocprof's kernel name (k_matvec_scan_dpp)
        pre = [k for k in ks if k.startswith(kernel + "_")]
        key = kernel if kernel in ks else (pre[0] if len(pre) == 1 else None)
        if s.get("config") == want and s.get("workload", "svd") == workload and key:
            if s.get("sources_sha16") != sha:
                stale.append(os.path.relpath(f, ROOT))
                continue
            return ks[key]["traffic_per_launch"], os.path.relpath(f, ROOT), None
    note = ("no PMC summary of these kernel sources (sha16 %s)" % sha
            + ("; refused summaries of other sources: %s" % ", ".join(stale) if stale else ""))
    return None, None, note


def gpu_only_chain(workload, N, M, P, LB):
    """The GPU-only schedule of this workload (tools/timeline.py --json over a
    rocprofv3 kernel trace of the same kernel sources, run with hold_us so the
    host has queued the whole step first): span, busy time and the critical
    chain's launches, kernel time and launch-boundary time."""
    import glob
    sha = sources_sha16()
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_chain_*.json")), reverse=True):
        try:
            with open(f) as fh:
                s = json.load(fh)
        except (OSError, ValueError):
            continue
        if (s.get("workload") == workload and s.get("config") == {"N": N, "M": M, "P": P, "LB": LB}
                and s.get("sources_sha16") == sha):
            s = dict(s)
            s["file"] = os.path.relpath(f, ROOT)
            return s
    return None


# ----------------------------------------------------------------- CPU baseline
def cpu_info():
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"cpu_model": model, "nproc": os.cpu_count(),
            "affinity": len(os.sched_getaffinity(0))}


def cpu_baseline_run(spec):
    """The C oracle on a bounded sample of the workload (runs in the child)."""
    sys.path.insert(0, ORACLE_DIR)
    import corc  # oracle/ — the checker / reported baseline only
    if spec["workload"] == "svd":
        m, u, d, v = gen_input(spec["N"], spec["M"], spec["seed"])
        g = step_gammas(spec["seed"], 1)[0]
        t0 = time.perf_counter()
        a0, l0, a1 = corc.svd_witness(m, u, v, d, spec["P"], spec["LB"], g, row_lim=spec["rows"])
        dt = time.perf_counter() - t0
        cells = a0.shape[0] + a1.shape[0]
        sample = (f"oracle/svdw_oracle.c single thread, same {spec['N']}x{spec['M']} P={spec['P']} "
                  f"witness restricted to rows [0,{spec['rows']}) of every row-parallel stage "
                  f"(+ all loads and d checks): {cells} advice cells in {dt:.2f} s")
    else:
        a, b = gen_matmul_input(spec["N"], spec["N"], spec["M"], spec["seed"])
        g = step_gammas(spec["seed"], 1)[0]
        t0 = time.perf_counter()
        a0, a1 = corc.verify_mul_witness(a, b, spec["P"], g)
        dt = time.perf_counter() - t0
        cells = a0.shape[0] + a1.shape[0]
        sample = (f"oracle/svdw_oracle.c single thread, the whole {spec['N']}x{spec['N']} . "
                  f"{spec['N']}x{spec['M']} P={spec['P']} verify_mul witness (loads, naive "
                  f"i-j-k Fr GEMM, Freivalds rows): {cells} advice cells in {dt:.2f} s")
    return {"value": round(cells / dt, 1), "unit": "advice cells/s", "cores": 1, "kind": "port",
            "sample": sample, "seconds": round(dt, 3), **cpu_info()}


def cpu_baseline_child(spec):
    """Runs the baseline in a fresh process pinned to core 0 (taskset -c 0) and
    waits for it; called before this process touches the GPU."""
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-baseline-child", json.dumps(spec)]
    if shutil.which("taskset"):
        cmd = ["taskset", "-c", "0"] + cmd
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        return {"error": r.stderr.strip()[-400:]}
    out = json.loads(r.stdout.strip().splitlines()[-1])
    out["pinning"] = "taskset -c 0" if cmd[0] == "taskset" else "none"
    return out


# ----------------------------------------------------------------- launcher
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n):
    """`bench.py --gpus N` outside torch.distributed: run N ranks as a child
    torch.distributed.run process (this process never initialises the GPU and
    never execs) and return its exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)]
    env = dict(os.environ)
    # the ranks read this process's arguments from the environment (torchrun's
    # own parser would claim abbreviations such as --n)
    env["BENCH_ARGV"] = json.dumps(sys.argv[1:])
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.run(cmd, env=env).returncode


# ----------------------------------------------------------------- workloads
class SvdWorkload:
    def __init__(self, hs, ctx, args, N, M, rank, rows_mode, dev):
        import torch
        self.hs, self.ctx = hs, ctx
        m, u, d, v, _ = rank_workload(args.seed, 0 if rows_mode else rank, N, M)
        self.host = (m, u, v, d)
        if dev is None:                       # dry planner: host arrays
            self.inp = (m, u, v, d)
        else:
            self.inp = tuple(torch.tensor(np.ascontiguousarray(x), dtype=torch.float64, device=dev)
                             for x in (m, u, v, d))

    def step(self, gamma):
        return self.hs.svd_witness(self.ctx, *self.inp, gamma)


class VerifyMulWorkload:
    """README.md:32-46 as one step: loads of a and b, c_s = a * b (phase 0),
    verify_mul(a, b, c_s, gamma) (phase 1)."""

    def __init__(self, hs, ctx, args, N, M, rank, rows_mode, dev):
        import torch
        self.hs, self.ctx = hs, ctx
        a, b = gen_matmul_input(N, N, M, args.seed + rank)
        self.host = (a, b)
        self.inp = (a, b) if dev is None else tuple(
            torch.tensor(np.ascontiguousarray(x), dtype=torch.float64, device=dev) for x in (a, b))

    def step(self, gamma):
        # the four modular calls in one (svdw_verify_mul_witness: same cells,
        # tests/test_verify_mul_config.py; no host waits between them)
        return self.hs.verify_mul_witness(self.ctx, *self.inp, gamma)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=None,
                    help="untimed steps (default 3; verify_mul 8: each of its two lanes "
                         "captures its launch graph on its second or third call)")
    ap.add_argument("--workload", choices=["svd", "verify_mul"], default="svd")
    ap.add_argument("--n", type=int, default=None, help="rows (default 1024 svd, 256 verify_mul)")
    ap.add_argument("--m", type=int, default=None)
    ap.add_argument("--p", type=int, default=None, help="PRECISION_BITS (default 63 svd, 32 verify_mul)")
    ap.add_argument("--lb", type=int, default=19)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-rows", type=int, default=128)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-baseline-child", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--no-profile", action="store_true",
                    help="skip the engine's event profiler in the timed region")
    ap.add_argument("--profile-prefix", default=None,
                    help="kernel-name prefix the timed-region profiler records "
                         "(default k_stage for svd, k_matvec_scan for verify_mul)")
    ap.add_argument("--breakdown", action="store_true", help="print per-kernel ms/step to stderr")
    ap.add_argument("--shard", choices=["replicas", "rows"], default=None,
                    help="N>1: one matrix row-block sharded over the ranks (default; strong "
                         "scaling, BASELINE config 4) or one matrix per rank (weak scaling, "
                         "config 5)")
    ap.add_argument("--gather", choices=["auto", "none", "root", "all"], default="auto",
                    help="--shard rows: also time reassembling the witness after each step "
                         "(RCCL gather to rank 0 or all-gather), reported beside the "
                         "witness-only value as the `reassembly` record (auto: root in "
                         "rows mode)")
    ap.add_argument("--no-check", action="store_true",
                    help="skip the untimed device constraint check of the last witness")
    ap.add_argument("--no-ingest", action="store_true",
                    help="skip the untimed device parse of the input as data/matrix.in text")
    ap.add_argument("--dry", action="store_true",
                    help="CPU rehearsal: gloo + the engine's dry planner, no GPU")
    ap.add_argument("--opt", action="append", default=[],
                    help="engine tuning option name=value (svdw_set_option), repeatable")
    argv = json.loads(os.environ["BENCH_ARGV"]) if "BENCH_ARGV" in os.environ else None
    args = ap.parse_args(argv)

    if args.cpu_baseline_child is not None:
        print(json.dumps(cpu_baseline_run(json.loads(args.cpu_baseline_child))), flush=True)
        return 0
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args.gpus)

    svd = args.workload == "svd"
    if args.warmup is None:
        args.warmup = 3 if svd else 8
    N = args.n or (1024 if svd else 256)
    M = args.m or N
    P = args.p or (63 if svd else 32)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    shard = args.shard or ("rows" if world > 1 and svd else "replicas")
    rows_mode = shard == "rows" and world > 1
    gather = args.gather if args.gather != "auto" else ("root" if rows_mode else "none")
    if rows_mode and not svd:
        raise SystemExit("bench.py: --shard rows is the SVD witness's row-block sharding")

    # CPU baseline first, in a pinned child, before this process touches the GPU
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.dry:
        cpu = cpu_baseline_child({"workload": args.workload, "N": N, "M": M, "P": P,
                                  "LB": args.lb, "seed": args.seed, "rows": args.cpu_rows})
        try:
            os.sched_setaffinity(0, set(os.sched_getaffinity(0)) - {0} or {0})
        except OSError:
            pass

    import torch
    backend = "gloo" if args.dry else os.environ.get("BENCH_DIST_BACKEND", "nccl")
    dist = None
    dev = None
    if not args.dry:
        # Rehearsal on fewer GPUs than ranks (BENCH_DIST_BACKEND=gloo): ranks share
        # devices round-robin; timings are then not per-GPU numbers.
        if backend != "nccl":
            local = local % max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist  # noqa: F811
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
        assert dist.get_world_size() == world == args.gpus
    red_dev = dev if backend == "nccl" else torch.device("cpu")

    import halo2_svd041_amd as hs
    ctx = hs.Context(device=-1 if args.dry else local, precision_bits=P, lookup_bits=args.lb)
    for kv in args.opt:
        name, _, val = kv.partition("=")
        ctx.set_option(name, int(val))
    if rows_mode:
        ctx.set_shard(rank, world)
    wl = (SvdWorkload if svd else VerifyMulWorkload)(hs, ctx, args, N, M, rank, rows_mode, dev)

    def sync():
        if not args.dry:
            ctx.sync()
            torch.cuda.synchronize()

    warm_g = step_gammas(args.seed, args.warmup, offset=10 ** 6)
    gammas = step_gammas(args.seed, args.steps)
    for g in warm_g:
        cnt = wl.step(g)
    sync()

    profile = not args.no_profile and not args.dry
    # events around the dominant kernel's launches only: at config 2's size,
    # events around all ten launches of a step doubled the step time
    prefix = args.profile_prefix if args.profile_prefix is not None else ("k_stage" if svd else "k_matvec_scan")
    # The timed steps run without the event profiler (its start markers cost
    # 0.5-3.5 % of a step); the dominant kernel's launches
    # are timed in a second, untimed pass of the same steps right after (for
    # verify_mul also because the timed steps replay the captured launch
    # graph, which the profiler would switch off).
    graph_vm = not svd and "graph=0" not in args.opt
    if dist is not None:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for g in gammas:
        cnt = wl.step(g)
    t_issued = time.perf_counter()          # host done enqueueing (the GPU may still run)
    sync()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    host_ms = (t_issued - t0) / args.steps * 1e3
    graph_stats = ctx.graph_stats() if profile and graph_vm else None
    prof_elapsed = None
    if profile:
        ctx.profile(True, prefix)
        sync()
        tp = time.perf_counter()
        for g in gammas:
            wl.step(g)
        sync()
        prof_elapsed = time.perf_counter() - tp
    stats = ctx.profile_collect() if profile else []
    cells_step = cnt["advice0"] + cnt["advice1"]

    # The same kernel alone on the GPU (one untimed step with the streams
    # serialised): its intrinsic rate, reported beside the contended in-step rate.
    solo = None
    gemm = None
    if profile and svd and not rows_mode:
        ctx.set_option("overlap", 0)
        ctx.set_option("phase1_overlap", 0)
        ctx.profile(True, "")
        wl.step(gammas[-1])
        sync()
        solo_stats = ctx.profile_collect()
        ctx.profile(False)
        ctx.set_option("overlap", 1)
        ctx.set_option("phase1_overlap", 1)
        if solo_stats:
            _, solo, _ = roofline_from_profile([x for x in solo_stats if x["name"].startswith(prefix)], 1)
            # SURVEY.md §8(d) stage (ii): the exact field GEMMs (N M^2 + N^3 + M^3
            # MACs) -- residue planes, int8 matrix-core GEMMs, CRT -- alone on the GPU
            gms = sum(x["total_ms"] for x in solo_stats
                      if x["name"].split("@")[0].startswith(("k_to_residues", "k_residues", "k_gemm", "k_crt")))
            macs = float(N) * M * M + float(N) ** 3 + float(M) ** 3
            if gms > 0:
                gemm = {"field_macs_per_step": macs, "ms": round(gms, 4),
                        "field_GMAC_s": round(macs / (gms * 1e-3) / 1e9, 1),
                        "note": "exact Fr GEMMs (residues + int8 MFMA GEMMs + CRT), streams serialised"}

    reasm = None
    if rows_mode and gather != "none":
        # witness + reassembly per step, timed like the witness-only loop
        # (scaling reported with and without reassembly); --dry: the
        # same plan and grouped exchange over gloo on host buffers
        from halo2_svd041_amd import collect
        mode = "gather" if gather == "root" else "all_gather"
        plan = collect.plan(ctx, rank, world, mode)
        if args.dry:
            sizes = {(0, 0): cnt["advice0"], (1, 0): cnt["advice1"],
                     (0, 1): cnt["lookup0"], (1, 1): cnt["lookup1"]}
            host = {k: torch.zeros((n, 32), dtype=torch.uint8) for k, n in sizes.items()}
            reassemble = lambda: collect.exchange(host, plan)             # noqa: E731
        else:
            reassemble = lambda: collect.reassemble(ctx, plan)           # noqa: E731
        reassemble()                                     # warm the communicator
        dist.barrier()
        sync()
        t1 = time.perf_counter()
        for g in gammas:
            wl.step(g)
            reassemble()
        sync()
        dist.barrier()
        el2 = time.perf_counter() - t1
        el2, _ = reduce_over_ranks(el2, 0, dist, red_dev)
        reasm = {"mode": mode, "root": 0 if mode == "gather" else None,
                 "collectives_per_step": plan.collectives,
                 "ms_per_step_with_reassembly": round(el2 / args.steps * 1e3, 4),
                 "value_with_reassembly": round(cells_step * args.steps / el2, 1),
                 "reassembly_ms": round((el2 - elapsed) / args.steps * 1e3, 4),
                 "moved_GB_per_step": round(plan.moved_cells * 32 / 1e9, 3),
                 "note": "witness then its stream-ordered reassembly over "
                         + ("gloo (dry rehearsal, host buffers)" if args.dry else "RCCL")
                         + ", max over ranks"}

    # Untimed: the device constraint checker over the last witness (svdw_check_gates;
    # a row-sharded rank checks the rows it owns), summed over the ranks.
    check = None
    if not args.no_check and not args.dry:
        r = ctx.check_gates()
        keys = sorted(r)
        vals = [float(r[k]) for k in keys]
        if dist is not None:
            t = torch.tensor(vals, dtype=torch.float64, device=red_dev)
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
            vals = t.tolist()
        check = {k: int(x) for k, x in zip(keys, vals)}
        bad = check["gate_failures"] + check["copy_failures"] + check["lookup_failures"]
        if not rows_mode:
            # every copy-constraint (equality) record, generated and checked on the
            # device (svdw_check_equalities): scan operands and constants included
            eq = [ctx.check_equalities(ph) for ph in (0, 1)]
            for k in ("copies_checked", "copy_failures", "consts_checked", "const_failures"):
                check["equality_" + k] = sum(int(x[k]) for x in eq)
            bad += check["equality_copy_failures"] + check["equality_const_failures"]
        check["ok"] = bad == 0

    # Untimed: the same input as data/matrix.in text (json.dump(indent=4), as
    # input-creator.py writes it) parsed on the device (svdw_parse_svd_input_device)
    ingest = None
    if svd and world == 1 and not args.dry and not args.no_ingest:
        m, u, v, d = wl.host
        text = json.dumps({"m": m.tolist(), "u": u.tolist(), "d": d.tolist(), "v": v.tolist()},
                          indent=4).encode()
        tt = torch.frombuffer(bytearray(text), dtype=torch.uint8).to(dev)
        hs.parse_svd_input_device(ctx, tt)
        ts = []
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            parsed = hs.parse_svd_input_device(ctx, tt)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        tdev = sorted(ts)[1]
        t0 = time.perf_counter()
        host = hs.parse_svd_input(text, "serde")
        thost = time.perf_counter() - t0
        same = all(np.array_equal(parsed[k].cpu().numpy().view(np.uint64), host[k].view(np.uint64))
                   for k in ("m", "u", "v", "d"))
        ingest = {"text_MB": round(len(text) / 1e6, 1), "device_parse_ms": round(tdev * 1e3, 3),
                  "device_GB_s": round(len(text) / tdev / 1e9, 1), "host_parse_ms": round(thost * 1e3, 1),
                  "bit_identical_to_host_parse": bool(same),
                  "note": "untimed; serde_json's default float path (1 ulp off correct rounding on ~10 % "
                          "of values, as the reference reads data/matrix.in), text resident in HBM"}
        del tt, parsed

    rank_ms = None
    if dist is not None:
        t = torch.zeros(world, dtype=torch.float64, device=red_dev)
        t[rank] = elapsed / args.steps * 1e3
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        rank_ms = [round(x, 4) for x in t.tolist()]
    elapsed, cells_all = reduce_over_ranks(elapsed, cells_step, dist, red_dev)
    if rows_mode:
        cells_all = float(cells_step)        # one witness, split over the ranks
    value = cells_all * args.steps / elapsed

    if rank == 0:
        if svd:
            workload = (f"svd_verify_witness N={N} M={M} PRECISION_BITS={P} LOOKUP_BITS={args.lb}, "
                        + ("one matrix row-sharded over the GPUs" if rows_mode
                           else "one matrix per GPU"))
        else:
            workload = (f"verify_mul (README.md:32-46 recipe, svdw_verify_mul_witness) a {N}x{N} . "
                        f"b {N}x{M} PRECISION_BITS={P}, one product per GPU")
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "advice cells/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            # host time to enqueue a step, rank 0 (pipelined: close to ms_per_step
            # means the host, not the GPU, bounds the step)
            "host_enqueue_ms_per_step": round(host_ms, 4),
            "higher_is_better": True,
            "scaling": "strong" if rows_mode else "weak",
            "vs_baseline": None,
            "dtype": "bn254_fr (u32 limbs; exact multi-modular int8 MFMA GEMM)",
            "data": ("dry planner rehearsal on CPU (no GPU: timings are host planning only)"
                     if args.dry else
                     "synthetic (input-creator.py recipe, seeded; fresh gamma = sha256 mod p "
                     "per step)"),
            "config": {
                "workload": workload,
                "N": N, "M": M, "precision_bits": P, "lookup_bits": args.lb,
                "advice_cells_per_step": cells_step,
                "lookup_cells_per_step": cnt["lookup0"] + cnt["lookup1"],
                "parallelism": (f"row blocks x{world} of one matrix (witness kept sharded; "
                                f"its reassembly timed in the `reassembly` record)"
                                if rows_mode else f"replicas x{world} (no data-path collective)"),
                "ranks": world,
                "backend": backend if world > 1 else None,
            },
        }
        # SURVEY.md §8(d) stage (i): the whole witness against HBM, algorithmic
        # bytes = 32 B per advice + lookup cell + 8 B per f64 input entry; with
        # N GPUs against N x peak (the node's aggregate HBM roofline)
        nin = (N * M + N * N + M * M + min(N, M)) if svd else (N * N + N * M)
        step_bytes = 32 * (cells_step + cnt["lookup0"] + cnt["lookup1"]) + 8 * nin
        ach = step_bytes / (elapsed / args.steps) / 1e9
        peak_all = HBM_PEAK_GBS * (world if rows_mode else 1)
        step = {"bytes": step_bytes, "achieved": round(ach, 1), "peak": peak_all,
                "frac": round(ach / peak_all, 4),
                "note": ("one witness row-sharded over %d GPUs: its bytes / ms_per_step / "
                         "(%d x peak)" % (world, world)) if rows_mode else
                        "whole witness per step (all kernels, all streams)"}
        if rows_mode and rank_ms:
            step["rank_ms_min"] = min(rank_ms)
            step["rank_ms_max"] = max(rank_ms)
            step["rank_ms"] = rank_ms
        if world > 1 and not rows_mode:           # replicas: every rank its own witness
            step["note"] = "each rank's whole witness per step against one GPU's peak"
        if stats:
            kname, roof, breakdown = roofline_from_profile(stats, args.steps)
            traffic, src, tnote = pmc_traffic(kname, args.workload, N, M, P, args.lb,
                                              world if rows_mode else 1, rank)
            if traffic is not None:
                roof["traffic"] = traffic
                roof["traffic_source"] = src
            else:
                roof["traffic_note"] = tnote
            roof["sources_sha16"] = sources_sha16()
            sst = stage_stream_rate(stats, args.steps)
            if sst is not None and roof["kernel"] == "k_stage":
                # against the step time of the profiled pass it was measured in
                sst["busy_frac_of_step"] = round(sst["busy_ms_per_step"] / (prof_elapsed / args.steps * 1e3), 4)
                sst["profiled_pass_ms_per_step"] = round(prof_elapsed / args.steps * 1e3, 4)
                roof["stage_stream"] = sst
            if solo is not None and solo["kernel"] == roof["kernel"]:
                roof["standalone"] = {k: solo[k] for k in ("achieved", "frac", "avg_launch_ms")}
                roof["standalone"]["note"] = ("same kernel, one extra untimed step with the "
                                              "streams serialised (no concurrent products/scans)")
            if args.breakdown:
                print(json.dumps({"ms_per_step_by_kernel": breakdown,
                                  "stats": stats}, indent=1), file=sys.stderr)
        else:                                     # (--dry / --no-profile: no kernel events)
            roof = {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": None, "traffic": None, "kernel": None}
        roof["step"] = step
        if not svd:
            # a 256^2 witness moves 26 MB: the step is bound by its dependent
            # launches and their boundaries, not by HBM (its whole-step fraction
            # says so); the GPU-only chain of the same sources, when committed
            roof["bound"] = "latency"
            ch = gpu_only_chain(args.workload, N, M, P, args.lb)
            roof["latency"] = ({"gpu_only_step_us": ch["span_us"], "gpu_busy_us": ch["busy_us"],
                                "critical_launches": ch["chain"]["launches"],
                                "critical_kernel_us": ch["chain"]["kernel_us"],
                                "critical_boundary_us": ch["chain"]["boundary_us"],
                                "critical_kernels": ch["chain"]["kernels"], "source": ch["file"],
                                "note": "GPU-only schedule (hold_us) of the same kernel sources; the "
                                        "per-kernel HBM fraction above is the dominant kernel's"}
                               if ch else {"note": "no committed GPU-only chain of these kernel sources "
                                                   "(profiles/*_chain_*.json)"})
        if stats:
            roof["timing_note"] = ("ms_per_step from the timed steps, profiler off; the kernel's "
                                   "launches timed by HIP events in a second, untimed pass of the same "
                                   "steps (%.4f ms per step with the events)" % (prof_elapsed / args.steps * 1e3))
            if graph_stats is not None:
                roof["timing_note"] += ("; the timed steps replay the captured launch graph (captures, "
                                        "replays = %d, %d), the profiled pass runs eagerly" % graph_stats)
        out["roofline"] = roof
        if gemm is not None:
            out["field_gemm"] = gemm
        if ingest is not None:
            out["ingest"] = ingest
        if reasm is not None:
            out["reassembly"] = reasm
        if check is not None:
            out["witness_check"] = check
        if cpu is not None:
            out["cpu_baseline"] = cpu
            if "value" in cpu:
                out["speedup_vs_cpu_baseline"] = round(value / cpu["value"], 1)
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
