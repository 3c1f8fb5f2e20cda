"""The N-rank bench on the GPU: `profiles/rehearse_bench_ranks.py` runs bench.run in 2 spawned
ranks that share GPU 0 (gloo instead of RCCL, which refuses two ranks on one device), so the
8-GPU driver run's path -- ranks spawned before any GPU call, per-rank seeded families, barrier +
synchronize around the timed steps, MAX time and SUM families over the ranks -- runs on hardware
here.  The JSON line must count both ranks' families."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_two_ranks_on_one_gpu():
    fams, steps = 50_000, 3
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "profiles", "rehearse_bench_ranks.py"), "--ranks", "2", "--",
                        "--families", str(fams), "--steps", str(steps), "--warmup", "1", "--cpu-sample", "0",
                        "--no-tags-leg"], capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-3000:]  # rank 0 alone prints
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == steps and d["scaling"] == "weak"
    assert d["config"]["families_per_gpu"] == fams and d["config"]["parallelism"] == "family-sharded x2"
    # value = both ranks' families per step / the slower rank's step time
    total = d["value"] * d["ms_per_step"] / 1e3
    assert abs(total - 2 * fams) <= 2 * fams * 1e-2, (total, d)  # (ms_per_step is rounded)
    assert d["families_emitted"] > fams  # SUM over the ranks (each emits nearly all of its own)
    assert d["cpu_baseline"] is None     # the CPU leg runs at N = 1 only
