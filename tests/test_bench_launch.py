"""bench.py --gpus N without an outside launcher: the parent starts torch.distributed.run with N
ranks itself, before anything imports halogen or touches a GPU, relays rank 0's one JSON line and exits with the
launcher's status.  Driven here with the --dist-probe stub (gloo, no GPU); the GPU form is the driver's N > 1 run."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def _env(**extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                          "MASTER_PORT")}
    env.update(OMP_NUM_THREADS="1", **extra)
    return env


def test_gpus_requested_and_command():
    import bench
    assert bench.gpus_requested(["--gpus", "8", "--steps", "3"]) == 8
    assert bench.gpus_requested(["--steps", "3", "--gpus=4"]) == 4
    assert bench.gpus_requested(["--steps", "3"]) == 1
    assert bench.gpus_requested(["--gpus", "x"]) == 1
    cmd = bench.self_launch_command(["--gpus", "2", "--steps", "3"], 2, 29555)
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert "--nproc-per-node=2" in cmd and "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    assert cmd[-4:] == [str(ROOT / "bench.py"), "--gpus", "2", "--steps", "3"][-4:]


def test_no_self_launch_inside_a_rank_or_at_one_gpu():
    import bench
    old = os.environ.get("WORLD_SIZE")
    try:
        os.environ["WORLD_SIZE"] = "2"
        assert bench.self_launch(["--gpus", "2"]) is None
        del os.environ["WORLD_SIZE"]
        assert bench.self_launch(["--gpus", "1"]) is None
    finally:
        if old is not None:
            os.environ["WORLD_SIZE"] = old


@pytest.mark.parametrize("n", [2, 3])
def test_bench_starts_its_ranks_and_relays_one_line(n):
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", str(n), "--dist-probe"], cwd=ROOT,
                       env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["dist_probe"] and out["world"] == n and out["rank_sum"] == n * (n - 1) // 2, out


def test_a_failing_rank_fails_the_parent():
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--dist-probe"], cwd=ROOT,
                       env=_env(HALOGEN_BENCH_PROBE_FAIL_RANK="1"), capture_output=True, text=True, timeout=300)
    assert r.returncode != 0


def test_compact_summary_and_detail_split(tmp_path):
    """The line's last key (`summary`) carries the per-frame operating points; the per-format display tables go to the
    detail file and the line keeps the reference's display format."""
    import bench
    disp = {f: {"sync": {"frac_of_batched": 0.7}, "pipelined": {"frac_of_batched": 0.8}} for f in ("rgba32f", "rgba16f",
                                                                                                 "r11g11b10f")}
    result = {"value": 3500.0, "primary_miss_frac": 0.54, "roofline": {"frac": 0.56}, "config": {"workload": "C3"},
              "per_frame": {"frac_of_batched": 0.96, "strict": {"value": 3150.0, "frac_of_batched": 0.9,
                                                                  "per_launch": {"frac_of_batched": 0.85}},
                            "with_display_readback": disp},
              "camera_move": {"value": 1860.0, "upload_share": 0.003}, "framed": {"value": 1650.0}}
    out = tmp_path / "detail.json"
    bench.split_detail(result, str(out))
    assert set(result["per_frame"]["with_display_readback"]) == {"r11g11b10f", "other_formats"}
    assert json.loads(out.read_text())["with_display_readback"]["rgba16f"]["sync"]["frac_of_batched"] == 0.7
    s = bench.compact_summary(result)
    assert s["per_frame"]["strict"]["frac_of_batched"] == 0.9
    assert s["per_frame"]["display_r11g11b10f"]["at_once"] == 0.7
    assert s["per_frame"]["display_r11g11b10f"]["one_behind"] == 0.8
    assert s["camera_move"]["frac_of_batched"] == round(1860 / 3500, 3) and s["framed"] == 1650.0
    assert len(json.dumps(s)) < 1000
