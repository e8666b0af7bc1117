"""Round-6 diagnostic: run bench.py with the Python layer's hold checkpoints
off (Context.HOLD_EVERY huge), to test whether the checkpoint stream stalls a
pipelined engine stream that shares its hardware queue."""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import halo2_svd041_amd.zk as zk  # noqa: E402

zk.Context.HOLD_EVERY = 10 ** 9
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
