"""bench.py's N > 1 path on the hardware: two ranks launched by torch.distributed.run
share the box's GPU over the gloo backend (the driver's 8-GPU run uses RCCL, one rank per GPU; the
code path -- rank-offset simulator indices, barrier + max-over-ranks timing, metric-sum all-reduce,
rank-0 JSON -- is the same).  Checks the JSON line's whole-job accounting and that the all-reduced
metric means are finite and plausible."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_gloo():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29531", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--batch", "64", "--L", "2000",
           "--dist-backend", "gloo", "--no-cpu-baseline", "--no-variants", "--no-batch1", "--no-pipeline"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]             # rank 0 prints, rank 1 does not
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["global_batch"] == 128
    assert rec["config"]["parallelism"] == "dp2"
    assert abs(rec["value"] - 2 * 64 * 2 / (rec["ms_per_step"] * 2 * 1e-3)) < 1e-6 * rec["value"]
    m = rec["metrics_mean"]
    assert all(v == v for v in m.values())                # finite, all-reduced over both ranks
    assert 0.0 < m["SSIM"] <= 1.0 and m["MSE"] >= 0.0
