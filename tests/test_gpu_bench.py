"""bench.py end to end at a short clip: the driver runs it at round end, so every leg (clip stream, per-call
pass, roofline probe) must run on the current tree and print one well-formed contract line."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_line_short_clip():
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--seconds", "4", "--steps", "2",
                        "--warmup", "1", "--no-cpu-baseline"], capture_output=True, text=True, timeout=240, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in line, k
    assert line["value"] > 0 and line["n_gpus"] == 1 and line["steps"] == 2
    roof = line["roofline"]
    assert roof["bound"] == "mfma" and 0 < roof["frac"] < 1 and roof["launches_per_step"] > 0
    assert line["per_call"]["value"] > 0
