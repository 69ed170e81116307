"""bench.py's multi-rank launch on CPU (VERDICT r4 "a multi-GPU bench that
cannot mis-measure"): `bench.py --gpus N` without torchrun starts N rank
processes itself, refuses a rank set that is not the one asked for, and
fails when one rank fails."""
import json
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_check_world():
    assert bench.check_world(1, 1, "nccl", 1) is None
    assert bench.check_world(8, 8, "nccl", 8) is None
    assert "WORLD_SIZE" in bench.check_world(8, 1, "nccl", 8)      # one rank cannot stand in for eight
    assert "needs 2 GPUs" in bench.check_world(2, 2, "nccl", 1)     # RCCL: one device per rank
    assert bench.check_world(2, 2, "gloo", 1) is None               # gloo rehearsal: ranks share a device
    assert bench.check_world(1, 1, "gloo", 0) == "no GPU visible"


def test_spawn_ranks_env(tmp_path):
    script = tmp_path / "rank.py"
    script.write_text(textwrap.dedent(f"""
        import json, os, sys
        keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
        with open(os.path.join({str(tmp_path)!r}, "r" + os.environ["RANK"] + ".json"), "w") as f:
            json.dump({{"env": {{k: os.environ[k] for k in keys}}, "argv": sys.argv[1:]}}, f)
    """))
    rc = bench.spawn_ranks(3, ["--gpus", "3", "--steps", "2"], script=str(script), poll_s=0.05)
    assert rc == 0
    seen = [json.load(open(tmp_path / f"r{r}.json")) for r in range(3)]
    ports = {s["env"]["MASTER_PORT"] for s in seen}
    assert len(ports) == 1
    for r, s in enumerate(seen):
        assert s["env"]["RANK"] == s["env"]["LOCAL_RANK"] == str(r)
        assert s["env"]["WORLD_SIZE"] == "3" and s["env"]["MASTER_ADDR"] == "127.0.0.1"
        assert s["argv"] == ["--gpus", "3", "--steps", "2"]


def test_spawn_ranks_one_failure_fails_the_run(tmp_path):
    script = tmp_path / "rank.py"
    script.write_text(textwrap.dedent("""
        import os, sys, time
        if os.environ["RANK"] == "1":
            sys.exit(7)
        time.sleep(60)          # the surviving rank would wait in a collective; it is terminated
    """))
    rc = bench.spawn_ranks(2, [], script=str(script), poll_s=0.05)
    assert rc == 7


@pytest.mark.parametrize("extra", [[], ["--backend", "gloo"]])
def test_bench_without_gpus_exits_nonzero(extra):
    """No GPU here: --gpus 2 must fail before printing a line, not fall back to one rank."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", *extra],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 2, p.stderr[-2000:]
    assert p.stdout.strip() == ""
    assert "GPU" in p.stderr


def test_bench_rank_count_mismatch_exits_nonzero():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 2
    assert p.stdout.strip() == ""
    assert "WORLD_SIZE" in p.stderr


def test_launch_refuses_when_amdsmi_cannot_count():
    """the launcher counts devices through amdsmi only; when
    amdsmi fails it refuses (exit 2) instead of falling back to a HIP call that
    would initialise the GPU in the parent before it starts the ranks."""
    import argparse
    import torch
    args = argparse.Namespace(gpus=2, backend="nccl")
    assert bench.launch_ranks(args, [], count=lambda: None) == 2
    assert bench.launch_ranks(args, [], count=lambda: 1) == 2           # RCCL: one device per rank
    assert not torch.cuda.is_initialized()


def test_count_devices_no_hip_does_not_initialise():
    import torch
    n = bench.count_devices_no_hip()
    assert n is None or n >= 0
    assert not torch.cuda.is_initialized()


def test_mlt_parity_zero_steps_is_reported_not_raised():
    """fewer mutations than chains leaves 0 steps per chain; the
    parity is skipped with a note before anything touches the context."""
    r = {"nx": 256, "ny": 256, "kind": "cornell_box_obj", "obj": "unused", "env": None}
    out = bench.cpu_baseline_mlt(None, r, 1, 1 << 18, 0, 1, 1.0)
    assert out["parity"] is None and "0 mutations per chain" in out["note"]


def test_shared_device_roofline_has_no_fractions():
    """a gloo rehearsal with ranks sharing one device reports no
    fraction of a chip peak, VALU issue included."""
    res = {"avg_kernel_ms": 100.0, "rays_per_launch": 10 ** 9, "scene_in_lds": False, "scene_bytes": 10 ** 8,
           "launch": {}, "fp64": False}
    out = bench.roofline("path", "cornell_1m:1920x1080", 2, res, 50.0, 2.0, shared_device=True)
    for k in ("achieved", "frac", "valu_issue_frac", "lds_frac", "valu_issue_frac_at_clock"):
        assert out.get(k) is None, k


def test_roofline_clock_fields():
    """The profiled clock (roofline_pmc.json clock_ghz, a GRBM_GUI_ACTIVE pass)
    rescales the VALU fraction from the 2.4-GHz peak to the running clock."""
    res = {"avg_kernel_ms": 227.0, "rays_per_launch": 7.6e9, "scene_in_lds": True, "scene_bytes": 10 ** 4,
           "launch": {}, "fp64": False}
    out = bench.roofline("path", "cornell:1920x1080", 2, res, None, None)
    pmc = bench.load_profile("roofline_pmc.json", "path:cornell:1920x1080")
    assert out["bound"] == "valu" and out["clock_ghz"] == round(pmc["clock_ghz"], 3)
    assert 1.9 < out["clock_ghz"] <= 2.4
    assert out["valu_issue_frac_at_clock"] == round(out["frac"] * bench.VALU_PEAK_CLOCK_GHZ / pmc["clock_ghz"], 4)
