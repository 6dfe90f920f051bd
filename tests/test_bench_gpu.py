"""bench.py end to end on the GPU at a small size: one JSON line with the driver's keys, the
MFMA roofline of the minibatch step and the env-step HBM view (the driver runs the full size)."""

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_emits_contract_line():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1",
           "--envs", "512", "--rollout", "8", "--minibatches", "4", "--epochs", "2",
           "--no-cpu-baseline"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
              "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1
    assert d["value"] > 0 and d["higher_is_better"] is True and d["scaling"] == "weak"
    # value = env-steps of the timed steps / their wall time
    assert abs(d["value"] - 512 * 8 * 2 / (d["ms_per_step"] * 2e-3)) / d["value"] < 0.01
    r = d["roofline"]
    assert r["bound"] == "mfma" and r["unit"] == "TFLOP/s" and 0 < r["frac"] < 1
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    e = d["roofline_env_step"]
    assert e["bound"] == "hbm" and 0 < e["frac"] < 1 and e["envs_per_launch"] == 512
