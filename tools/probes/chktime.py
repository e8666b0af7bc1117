import sys, os, time
sys.path.insert(0, os.getcwd())
import numpy as np, torch
import halo2_svd041_amd as hs
from bench import gen_input, gamma_for
m, u, d, v = gen_input(1024, 1024, 0)
dev = torch.device("cuda", 0)
dm, du, dv, dd = (torch.tensor(np.ascontiguousarray(x), dtype=torch.float64, device=dev) for x in (m, u, v, d))
ctx = hs.Context(device=0, precision_bits=63, lookup_bits=19)
hs.svd_witness(ctx, dm, du, dv, dd, gamma_for(0)); ctx.sync()
ctx.check_gates()
t0 = time.perf_counter(); r = ctx.check_gates(); t = time.perf_counter() - t0
print("check_gates ms %.2f" % (t * 1e3), r)
