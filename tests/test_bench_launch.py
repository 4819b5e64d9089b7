"""bench.py --gpus N: the launch contract (VERDICT r03 Missing #1).

* CPU: a --gpus that disagrees with an outer launcher's WORLD_SIZE is refused before anything
  touches a GPU (no line with a wrong n_gpus can be printed);
* GPU: ``bench.py --gpus 2`` with no launcher around it starts its two rank processes itself
  (children, torch.distributed.run on 127.0.0.1 -- the reference's Trainer(gpus=N,
  accelerator='ddp'), sl_pipeline.py:157-170) and relays rank 0's line; over gloo both ranks share
  the one GPU of the test box.
"""
import json
import os
import pathlib
import subprocess
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]


def test_bench_refuses_world_size_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "1"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode != 0
    assert "misreport n_gpus" in (p.stderr + p.stdout)
    assert '"metric"' not in p.stdout


@pytest.mark.gpu
def test_bench_gpus2_launches_its_ranks():
    env = dict(os.environ, FIODE_BENCH_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--no-cpu-baseline", "--no-secondary", "--no-configs", "--prof-reps", "2"],
                       env=env, capture_output=True, text=True, timeout=600, cwd=str(ROOT))
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2
    assert rec["config"]["parallelism"] == "dp2"
    assert rec["config"]["global_batch"] == 256
    assert rec["process_group"] == {"backend": "gloo", "world_size": 2}
    assert rec["value"] > 0 and rec["device_status"]["status"] == 0
