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
