#!/usr/bin/env python3
"""Turn a tools/final_r0N.sh run (gpurun_out/final_<tag>) into the committed
evidence under profiles/: PMC traffic summaries and GPU-only critical chains
tagged with the kernel-source hash the run was collected on (bench.py uses
only those of its own sources), kernel stats, timelines, bench lines.

    python tools/evidence.py r05          # locally, on the merged gpurun_out
    python tools/evidence.py r05 --pre    # on the GPU box, between the PMC /
                                          # timeline passes and the bench lines
"""
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(args, out=None):
    r = subprocess.run([sys.executable] + args, cwd=ROOT, capture_output=True, text=True)
    if r.returncode:
        raise SystemExit(r.stderr)
    if out:
        with open(os.path.join(ROOT, out), "w") as fh:
            fh.write(r.stdout)
    return r.stdout


def main():
    tag = sys.argv[1]
    pre = "--pre" in sys.argv[2:]
    src = os.path.join("gpurun_out", "final_" + tag)
    sha = open(os.path.join(ROOT, src, "sources_sha16")).read().strip()
    pro = "profiles"
    cfg = {"bench": "N=1024,M=1024,P=63,LB=19", "s8": "N=1024,M=1024,P=63,LB=19,world=8,rank=0",
           "vm": "N=256,M=256,P=32,LB=19", "512": "N=512,M=512,P=32,LB=19",
           "2048": "N=2048,M=1024,P=32,LB=19"}
    for name, c in cfg.items():
        d = os.path.join(src, "pmc_" + name)
        if not os.path.isdir(os.path.join(ROOT, d)):
            continue
        out = os.path.join(pro, f"{tag}_{name}_pmc_summary.json" if name != "bench" else f"{tag}_pmc_summary.json")
        run(["tools/pmc_summary.py", d, "--config", c, "--out", out,
             "--workload", "verify_mul" if name == "vm" else "svd"], out.replace(".json", ".txt"))
    chains = {"1024": ("svd", "N=1024,M=1024,P=63,LB=19"), "512": ("svd", "N=512,M=512,P=32,LB=19"),
              "s8": ("svd_shard8_rank0", "N=1024,M=1024,P=63,LB=19"), "vm": ("verify_mul", "N=256,M=256,P=32,LB=19")}
    for name, (wl, c) in chains.items():
        tr = os.path.join(src, "go_" + name, "run_kernel_trace.csv")
        if not os.path.exists(os.path.join(ROOT, tr)):
            continue
        run(["tools/timeline.py", tr, "--all", "--json", os.path.join(pro, f"{tag}_chain_{name}.json"),
             "--workload", wl, "--sha", sha, "--config", c], os.path.join(pro, f"{tag}_timeline_{name}.txt"))
    steady = os.path.join(src, "steady_1024", "run_kernel_trace.csv")
    if os.path.exists(os.path.join(ROOT, steady)):
        run(["tools/steady.py", steady], os.path.join(pro, f"{tag}_steady_b1024.txt"))
    if pre:
        print("pre-bench evidence for sources", sha, "written under profiles/ as", tag + "_*")
        return
    for f, dst in (("prof/run_kernel_stats.csv", f"{tag}_kernel_stats.csv"), ("bench.json", f"{tag}_bench.json"),
                   ("configs.jsonl", f"{tag}_configs.jsonl"), ("shard_sim.json", f"{tag}_shard_sim.json"),
                   ("ingest.jsonl", f"{tag}_ingest.jsonl")):
        p = os.path.join(ROOT, src, f)
        if os.path.exists(p):
            shutil.copy(p, os.path.join(ROOT, pro, dst))
    with open(os.path.join(ROOT, pro, f"{tag}_gpu_check.log"), "w") as fh:
        for f in ("pytest_gpu.log", "smoke.log"):
            p = os.path.join(ROOT, src, f)
            if os.path.exists(p):
                fh.write("".join(open(p).readlines()[-3:]))
    print("evidence for sources", sha, "written under profiles/ as", tag + "_*")


if __name__ == "__main__":
    main()
