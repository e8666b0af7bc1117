#!/usr/bin/env python3
"""Host-launch vs kernel-start lag per dispatch of the last witness step, from a
rocprofv3 --kernel-trace --hip-runtime-trace run (same clock).

    python tools/hostlag.py gpurun_out/prof_X   (dir with run_kernel_trace.csv, run_hip_api_trace.csv)
"""
import csv
import sys

d = sys.argv[1]
api = {}
calls = []
for r in csv.DictReader(open(f"{d}/run_hip_api_trace.csv")):
    api[int(r["Correlation_Id"])] = (r["Function"], int(r["Start_Timestamp"]))
    calls.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]))
ks = []
for r in csv.DictReader(open(f"{d}/run_kernel_trace.csv")):
    ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-40:],
               r["Stream_Id"], int(r["Correlation_Id"])))
ks.sort()
starts = [i for i, k in enumerate(ks) if "quantize" in k[2] and (i == 0 or "quantize" not in ks[i - 1][2])]
s0, s1 = starts[-2], starts[-1]
t0 = ks[s0][0]
print("stream  kstart   kend  hostcall  lag(kstart-host)  kernel")
for k in ks[s0:s1]:
    fn, ht = api.get(k[4], ("?", 0))
    print(f"s{k[3]} {(k[0]-t0)/1e3:8.1f} {(k[1]-t0)/1e3:8.1f} {(ht-t0)/1e3:9.1f} {(k[0]-ht)/1e3:9.1f}  {k[2]}")
# blocking-looking host calls (> 20 us) during the step
print("host calls > 20 us in the step window:")
for s, e, f in calls:
    if t0 - 500e3 <= s <= ks[s1][0] and e - s > 20e3:
        print(f"  {(s-t0)/1e3:9.1f} +{(e-s)/1e3:8.1f} us  {f}")
