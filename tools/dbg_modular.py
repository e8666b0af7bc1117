import sys, os
sys.path[:0] = [".", "tests", "oracle"]
import numpy as np
import halo2_svd041_amd as hs
import corc
from conftest import gamma_for, gen_svd_input
N, M, P = 10, 13, 42
m, u, d, v = gen_svd_input(N, M, seed=17)
g = gamma_for(17)
a0, l0, a1 = corc.svd_witness(m, u, v, d, P, 19, g)
for trial in range(2):
    ctx = hs.Context(device=0, precision_bits=P, lookup_bits=19)
    zm = hs.ZkMatrix.new(ctx, m); zu = hs.ZkMatrix.new(ctx, u); zv = hs.ZkMatrix.new(ctx, v)
    zd = hs.ZkVector.new(ctx, d)
    es, eu = hs.err_calc(P, max(N, M), 100.0, 1e-10, 1e-10)
    pl = hs.check_svd_phase0(ctx, zm, zu, zv, zd, es, eu, 30)
    g0 = ctx.advice(0)
    bad = np.nonzero(np.any(g0 != a0[:g0.shape[0]], axis=1))[0]
    print("trial", trial, "n", g0.shape[0], a0.shape[0], "bad", bad.size, bad[:5], bad[-5:] if bad.size else "")
    if bad.size:
        i = bad[0]
        print(" got", [hex(int(x)) for x in g0[i]], "want", [hex(int(x)) for x in a0[i]])
        print(" got", [hex(int(x)) for x in g0[i+3]], "want", [hex(int(x)) for x in a0[i+3]])
    ctx.close()
