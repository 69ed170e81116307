"""The bench line's configuration blocks on the GPU: the
default command carries C2, the north-star (C4), C3 and C5 blocks; here the
same code path at a reduced frame (256x144) with --configs on, so the GPU suite
checks every block's fields, its RMSE against the oracle and its timing fields
each round.  bench.py runs as a child process, as the driver runs it."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def test_default_line_blocks():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--res", "256x144", "--spp", "64", "--steps", "2",
           "--warmup", "1", "--configs", "on", "--north-star", "on", "--ns-steps", "1", "--ns-pixels", "2048",
           "--cfg-steps", "1", "--cfg-cpu-seconds", "1", "--cpu-seconds", "1", "--c3-min-pixels", "4096"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads([x for x in p.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 1 and line["steps"] == 2 and line["rmse"] <= 1e-3
    assert line["cpu_baseline"]["kind"] == "port" and line["cpu_baseline"]["value"] > 0
    for key in ("north_star", "c3", "c5"):
        blk = line[key]
        assert blk["value"] > 0 and blk["steps"] == 1
        assert blk["ms_per_step"] > 0 and blk["rays_per_step"] > 0
        assert blk["rmse"] is not None and blk["rmse"] <= 1e-3, (key, blk["rmse"])
        assert blk["roofline"]["kernel"] in ("path_megakernel", "mlt_megakernel")
        assert blk["cpu_baseline"]["value"] > 0
    assert line["c3"]["dtype"] == "f64"                       # list world: fp64 kernels under precision auto
    assert line["c3"]["rmse_detail"]["pixels"] >= 4096
    par = line["c5"]["rmse_detail"]["path_exact"]
    assert par["samples_gpu"] == par["samples_oracle"]
    assert par["path_exact_chains"] >= 0.97 * par["chains"]
    assert par["rays_rel_diff"] <= 2e-3
    # the main (C2) block's collective timing is measured
    assert line["collective_ms"] >= 0.0
