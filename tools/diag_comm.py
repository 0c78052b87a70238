"""Diagnostic: where does a 2-rank hg_comm_init_rank with a missing peer spend its time?  Prints progress with flushes."""
import faulthandler
import sys
import time

faulthandler.dump_traceback_later(40, exit=True)
sys.path.insert(0, sys.argv[1] if len(sys.argv) > 1 else "halogen-pathtracer_amd")
from halogen import abi  # noqa: E402

t0 = time.time()
print("create", flush=True)
ctx = abi.Context(0)
ctx.resize(64, 64)
ctx.set_tiling(0, 2)
uid = abi.comm_unique_id()
print(f"uid {time.time() - t0:.2f}", flush=True)
try:
    abi.Comm.rank(ctx, 2, uid, 0)
    print("JOINED", flush=True)
except abi.HalogenError as e:
    print(f"FAILED-LOUDLY {time.time() - t0:.1f} {e}", flush=True)
print(f"closing {time.time() - t0:.2f}", flush=True)
ctx.close()
print(f"closed {time.time() - t0:.2f}", flush=True)
