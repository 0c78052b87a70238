"""leaf_dist's precondition, checked at run time.

The distributed leaf test (hg_device.h leaf_dist) scans leaf sizes with DPP row shifts and exchanges rays with
ds_bpermute: it is exact only when every lane of the wave is active.  The product build relies on the streaming
kernel calling it at the top level of ballot-exit loops.  The HG_CHECK_EXEC=1 build (make check_exec ->
halogen/check_exec/libhalogen_hip.so) checks EXEC on every call, falls back to the sequential leaf loop when a lane is
off and counts it (hg_counters.exec_fallbacks).  This test runs the streaming-kernel parity tests against that build
in a child process (HALOGEN_LIB): the goldens, the 24 fuzz scenes, full-size C3 rows against the live oracle and the
1-frame launches; gpu_render asserts the build flag and zero fallbacks after every render, and the images must still
be bit-exact.  The same build verifies every cost-order sort (hg_order_verify: the order must be a permutation of the
tiles, hg_counters.order_faults), and gpu_render asserts zero faults too."""
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
CHECK_LIB = ROOT / "halogen-pathtracer_amd" / "halogen" / "check_exec" / "libhalogen_hip.so"
SELECT = ["tests/test_gpu_parity.py::test_gpu_matches_golden", "tests/test_gpu_fuzz.py::test_gpu_fuzz_matches_oracle",
          "tests/test_gpu_parity.py::test_gpu_full_size_rows_match_oracle",
          "tests/test_gpu_per_frame.py::test_gpu_one_frame_launches_match_golden"]


@pytest.mark.gpu
@pytest.mark.timeout(1000)
def test_gpu_leaf_dist_never_runs_under_partial_exec(gpu):
    assert CHECK_LIB.exists(), f"{CHECK_LIB} not built (make -C halogen-pathtracer_amd check_exec)"
    env = dict(os.environ, HALOGEN_LIB=str(CHECK_LIB), HG_EXPECT_NO_EXEC_FALLBACK="1")
    cmd = [sys.executable, "-u", "-m", "pytest", "-q", "-x", "-m", "gpu", "-p", "no:cacheprovider", "-k",
           "(stream and not C2 and not C5) or one_frame_launches", *SELECT]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    tail = (r.stdout + r.stderr)[-3000:]
    assert r.returncode == 0, tail
    assert " passed" in r.stdout and " failed" not in r.stdout, tail
    n_passed = int(r.stdout.rsplit(" passed", 1)[0].split()[-1])
    assert n_passed >= 12 + 24 + 2 + 5, tail
