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
           "--dist-backend", "gloo", "--no-cpu-baseline", "--no-variants", "--no-batch1", "--no-pipeline",
           "--config4-batch", "16", "--config4-chunks", "2", "--config4-archs", "RRCDNet,DSDN"]
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
    c4 = rec["configs"]["config4"]                       # the data-parallel driver at W = 2
    assert c4["n_gpus"] == 2 and c4["total_spectra"] == 2 * 2 * 16
    assert "config2" not in rec["configs"]               # single-GPU configs run at N = 1 only


def test_bench_gpus_flag_starts_its_own_ranks():
    """`python bench.py --gpus 2` without a launcher starts its two ranks itself
    (torch.distributed.run, before any GPU call) and rank 0 prints one line with n_gpus = 2; here both
    ranks share the box's one GPU over gloo."""
    env = dict(os.environ, OMP_NUM_THREADS="4")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--batch", "64", "--L", "2000", "--dist-backend", "gloo", "--no-cpu-baseline", "--no-variants",
           "--no-batch1", "--no-pipeline", "--no-configs"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["global_batch"] == 128 and rec["config"]["parallelism"] == "dp2"


def _config4(nproc, backend, port, tmp_path, total=48, archs="RRCDNet,DSDN"):
    out = tmp_path / f"c4_{nproc}_{backend}.json"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "tools", "config4.py"),
           "--total", str(total), "--archs", archs, "--batch", "10", "--L", "1200", "--dist-backend", backend,
           "--out", str(out)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(out.read_text())


def test_config4_sums_identical_for_one_and_two_ranks(tmp_path):
    """Config 4 (tools/config4.py -> evaluate_synthetic): the same N = 48 simulator spectra evaluated
    by 1 rank and by 2 ranks (gloo, both on the box's GPU; 24 + 24 indices, ragged 10-spectrum
    chunks) give bit-identical exact metric accumulators and means for RRCDNet and DSDN."""
    one = _config4(1, "gloo", 29541, tmp_path)
    two = _config4(2, "gloo", 29543, tmp_path)
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    for a in ("RRCDNet", "DSDN"):
        assert one["networks"][a]["acc"] == two["networks"][a]["acc"], a
        assert one["networks"][a]["means"] == two["networks"][a]["means"], a
        assert one["networks"][a]["acc"][-1] == 48


def test_rccl_leg_runs_one_rank(tmp_path):
    """The nccl (RCCL) backend path of bench.py and of the config-4 driver, executed once: one rank
    under torch.distributed.run (process group over RCCL, device-tensor barrier/all-reduce)."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", "29545", os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--steps", "2", "--warmup", "1", "--batch", "64", "--L", "2000",
           "--no-cpu-baseline", "--no-variants", "--no-batch1", "--config4-batch", "16", "--config4-chunks", "2",
           "--config2-n", "64", "--config2-batch", "32"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 1 and "dist_backend" not in rec["config"]
    c4 = rec["configs"]["config4"]
    assert c4["total_spectra"] == 32 and set(c4) >= {"RRCDNet", "DSDN", "ADSDN"}
    assert rec["configs"]["config2"]["spectra"] == 64 and "config5" in rec["configs"]
    one = _config4(1, "nccl", 29547, tmp_path, total=30, archs="ADSDN")
    assert one["dist_backend"] == "nccl" and one["networks"]["ADSDN"]["acc"][-1] == 30
