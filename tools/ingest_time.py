#!/usr/bin/env python3
"""Device ingest timing at the BASELINE sizes (svdw_parse_svd_input_device on
text already in HBM) next to the host parser; json.dump(indent=4) text as
input-creator.py writes it.

    python tools/ingest_time.py [--sizes 512,1024,2048x1024]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="512,1024,2048x1024")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    torch.cuda.is_available()
    import halo2_svd041_amd as hs
    from bench import gen_input
    out = []
    with hs.Context(device=0, precision_bits=63, lookup_bits=19) as ctx:
        for sz in a.sizes.split(","):
            N, _, M = sz.partition("x")
            N, M = int(N), int(M or N)
            m, u, d, v = gen_input(N, M, 0)
            text = json.dumps({"m": m.tolist(), "u": u.tolist(), "d": d.tolist(), "v": v.tolist()},
                              indent=4).encode()
            t0 = time.perf_counter()
            hs.parse_svd_input(text, "serde")
            th = time.perf_counter() - t0
            t = torch.frombuffer(bytearray(text), dtype=torch.uint8).to("cuda:0")
            hs.parse_svd_input_device(ctx, t)
            ts = []
            for _ in range(a.reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                hs.parse_svd_input_device(ctx, t)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            td = sorted(ts)[len(ts) // 2]
            rec = {"N": N, "M": M, "text_MB": round(len(text) / 1e6, 1), "host_ms": round(th * 1e3, 1),
                   "device_ms": round(td * 1e3, 3), "device_GBps": round(len(text) / td / 1e9, 1)}
            print(json.dumps(rec), flush=True)
            out.append(rec)
    return 0


if __name__ == "__main__":
    sys.exit(main())
