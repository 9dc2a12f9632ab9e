"""Host-side checks without a GPU: oracle vs the reference's golden vectors, module surfaces,
dataset format, sharding, and the world_size-2 metric all-reduce over gloo."""
import json
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import GOLDEN, INPUT_SETS, golden_inputs, golden_state_dict, golden_template, input_array, load_golden

ARCHS = ["DenoiseCNN", "RRCDNet", "DSDN", "ADSDN", "PIDN", "APIDN"]


# --- oracle pinned to the reference ------------------------------------------------------------
@pytest.mark.parametrize("arch", ARCHS)
def test_oracle_reproduces_reference_outputs(arch, inputs):
    from oracle.models import forward
    g = load_golden(arch)
    whichs = ["synth"] + (["trained"] if any(k.startswith("w::") for k in g.files) else [])
    for which in whichs:
        sd = golden_state_dict(arch, which)
        for name in INPUT_SETS:         # every input set, L = 7 ... 16384, for all six networks
            x = torch.from_numpy(input_array(inputs, name)).unsqueeze(1)
            y = forward(arch, sd, x).squeeze(1).numpy()
            ref = g[f"{which}_{name}"]
            assert np.abs(y - ref).max() <= 1e-6 * max(1.0, np.abs(ref).max()), (arch, which, name)


def test_oracle_metrics_match_skimage_golden():
    from oracle.metrics import per_spectrum
    g = np.load(os.path.join(GOLDEN, "metrics.npz"))
    p = per_spectrum(g["den"], g["clean"])
    ref = g["per_spectrum"]
    np.testing.assert_allclose(p[:, :2], ref[:, :2], rtol=1e-10)      # MSE, SSIM (fp64 in both)
    np.testing.assert_allclose(p[:, 2:], ref[:, 2:], rtol=1e-6)       # reference: float32 diff/ptp


def test_oracle_generator_distribution():
    """The numpy restatement of the engine's simulator against reference statistics (small n)."""
    from oracle.generator import generate
    with open(os.path.join(GOLDEN, "generator_stats.json")) as fh:
        ref = json.load(fh)
    c, x, s, sd, outs = generate(7, 0, 200, 10000)
    assert np.all(c.min(axis=1) == 0) and np.all(c.max(axis=1) > 0.9999)
    lens = np.concatenate([o["seg_lens"][:-1] for o in outs])
    assert lens.min() >= 1 and lens.max() <= 40 and abs(lens.mean() - 20.5) < 0.5
    assert s.min() >= 20 and s.max() < 37
    assert abs(np.mean(np.mean(c.astype(np.float64) ** 2, axis=1)) - ref["power_mean"]) < 0.02
    rq = np.array(ref["noise_std_quantiles"])
    assert rq[0] * 0.8 < np.median(sd) < rq[4]


def test_oracle_generator_is_counter_based():
    from oracle.generator import generate_one
    a = generate_one(11, 5, 500)
    b = generate_one(11, 5, 500)
    c = generate_one(11, 6, 500)
    assert np.array_equal(a["noisy"], b["noisy"]) and not np.array_equal(a["noisy"], c["noisy"])


# --- module surface ----------------------------------------------------------------------------
@pytest.mark.parametrize("arch", ARCHS)
def test_module_state_dict_is_reference_compatible(arch):
    import raman_mi355x as R
    g = load_golden(arch)
    m = R.MODELS[arch]()
    keys = json.loads(str(g["keys"]))
    shapes = json.loads(str(g["shapes"]))
    sd = m.state_dict()
    assert list(sd) == keys
    assert [list(v.shape) for v in sd.values()] == shapes
    m.load_state_dict(golden_state_dict(arch, "synth"), strict=True)


def test_module_unsupported_configuration_raises():
    import raman_mi355x as R
    with pytest.raises(NotImplementedError):
        R.DSDN(num_res_blocks=3)


@pytest.mark.parametrize("arch", ARCHS)
def test_eager_fallback_matches_reference_goldens(arch, inputs):
    """SURVEY.md §8(b) fallback: a CPU tensor runs the reference forward on the module's own
    submodules (an unchanged evaulate.py with DEVICE = "cpu", 1DCNN/evaulate.py:10): the golden
    checkpoints load strictly and reproduce the reference's fp32 CPU outputs within 1e-6."""
    import raman_mi355x as R
    g = load_golden(arch)
    whichs = ["synth"] + (["trained"] if any(k.startswith("w::") for k in g.files) else [])
    for which in whichs:
        m = R.MODELS[arch]()
        m.load_state_dict(golden_state_dict(arch, which), strict=True)
        m.eval()
        assert not m.uses_engine(torch.zeros(1, 1, 8))
        for name in ("main", "edge33", "edge7"):
            x = torch.from_numpy(input_array(inputs, name)).unsqueeze(1)
            with torch.no_grad():
                y = m(x).squeeze(1).numpy()
            ref = g[f"{which}_{name}"]
            assert np.abs(y - ref).max() <= 1e-6 * max(1.0, np.abs(ref).max()), (arch, which, name)


def test_eager_fallback_trains():
    """Training mode and requires_grad inputs take the eager path: BatchNorm uses batch statistics and
    updates its running stats, and gradients reach every parameter (RRCDNet/train.py:158-170)."""
    import raman_mi355x as R
    torch.manual_seed(0)
    m = R.RRCDNet().train()
    x = torch.rand(2, 1, 64)
    assert not m.uses_engine(x)
    rm0 = m.right_net[1].running_mean.clone()
    loss = torch.nn.functional.mse_loss(m(x), x)
    loss.backward()
    assert not torch.equal(m.right_net[1].running_mean, rm0)
    assert all(p.grad is not None for p in m.parameters())
    m.eval()
    xg = torch.rand(1, 1, 32, requires_grad=True)
    assert not m.uses_engine(xg)
    m(xg).sum().backward()
    assert xg.grad is not None


def test_checkpoint_round_trip(tmp_path):
    """torch.save(state_dict) -> torch.load(weights_only=True) -> strict load, as */evaulate.py:66."""
    import raman_mi355x as R
    sd = golden_state_dict("RRCDNet", "trained")
    path = tmp_path / "RRCDNet_best.pth"
    torch.save(sd, path)
    m = R.RRCDNet()
    m.load_state_dict(torch.load(path, map_location="cpu", weights_only=True))
    for k, v in m.state_dict().items():
        assert torch.equal(v, sd[k])


def test_dataset_format(tmp_path):
    from raman_mi355x.dataset import load_dataset, save_dataset
    rng = np.random.default_rng(0)
    c, n = rng.uniform(size=(3, 50)), rng.uniform(size=(3, 50))
    save_dataset(tmp_path / "test.npz", c, n, np.ones(3), np.ones(3) * 0.1)
    d = load_dataset(tmp_path / "test.npz")
    assert d["clean_signals"].dtype == np.float64 and d["snrs"].shape == (3, 1)
    np.testing.assert_array_equal(d["noisy_signals"], n)


# --- data parallelism --------------------------------------------------------------------------
def test_shard_partitions_exactly():
    from raman_mi355x.distributed import shard
    for n in (0, 1, 7, 1000, 1001):
        for w in (1, 2, 3, 8):
            parts = [shard(n, r, w) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[i][1] == parts[i + 1][0] for i in range(w - 1))
            assert max(b - a for a, b in parts) - min(b - a for a, b in parts) <= 1


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _allreduce_worker(rank, world, port, per, out):
    import torch.distributed as dist
    from raman_mi355x.distributed import all_reduce_sums, means, shard
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    lo, hi = shard(per.shape[0])
    sums = torch.cat([torch.from_numpy(per[lo:hi]).sum(0), torch.tensor([float(hi - lo)], dtype=torch.float64)])
    all_reduce_sums(sums)
    if rank == 0:
        out.update(means(sums))
    dist.barrier()
    dist.destroy_process_group()


def test_metric_allreduce_world2_gloo():
    """Rank-sharded metric sums all-reduced over gloo equal the single-process means."""
    g = np.load(os.path.join(GOLDEN, "metrics.npz"))
    per = g["per_spectrum"].astype(np.float64)
    port = _free_port()
    with mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_allreduce_worker, args=(2, port, per, out), nprocs=2, join=True)
        got = dict(out)
    exp = per.mean(axis=0)
    for i, k in enumerate(("MSE", "SSIM", "Smoothness", "Peak2Peak")):
        assert abs(got[k] - exp[i]) <= 1e-12 * max(1.0, abs(exp[i]))


def test_bench_algorithmic_flops_match_survey():
    """bench.py's roofline numerator: sum over Conv1d layers of 2*Cin*Cout*K*L,
    per spectrum at L = 10,000 and PIDN / APIDN at L = 16,384."""
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location("bench", os.path.join(os.path.dirname(__file__), "..", "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    survey = {"DenoiseCNN": 4.4314e9, "RRCDNet": 7.1424e9, "DSDN": 7.8720e9, "ADSDN": 7.8768e9,
              "PIDN": 7.3805e9, "APIDN": 7.3847e9}
    for arch, g in survey.items():
        assert abs(bench.flops_per_spectrum(arch, 10000) - g) / g < 5e-5, arch
    assert abs(bench.flops_per_spectrum("PIDN", 16384) - 12.092e9) / 12.092e9 < 5e-4
    assert abs(bench.flops_per_spectrum("APIDN", 16384) - 12.099e9) / 12.099e9 < 5e-4


def _bench_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench", os.path.join(os.path.dirname(__file__), "..", "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    return bench


@pytest.mark.parametrize("world", [1, 2, 8])
def test_bench_index_blocks_disjoint(world):
    """bench.py's legs never re-generate each other's spectra: every rank's headline batch, pipeline
    batches and config-4 shard (evaluate_synthetic: [first + r N/W, first + (r+1) N/W)), the config-4
    warm-up and the sustained (config 3) window, are pairwise disjoint simulator index ranges for W = 1, 2, 8."""
    from raman_mi355x.distributed import shard
    bench = _bench_module()
    B, B4, chunks = 8192, 8192, 4
    ranges = []
    for r in range(world):
        b = bench.index_blocks(world, r, B, bench.PIPELINE_STEPS, B4, chunks)
        ranges += [b["headline"], b["pipeline"]]
        lo, hi = shard(b["config4_total"], r, world)
        ranges.append((b["config4_first"] + lo, b["config4_first"] + hi))
    ranges.append((b["config4_warmup_first"], b["config4_warmup_first"] + 2 * world))
    for r in range(world):                  # the sustained window: up to 2^32 indices per rank
        s0 = bench.index_blocks(world, r, B, bench.PIPELINE_STEPS, B4, chunks)["sustained_first"]
        ranges.append((s0, s0 + (1 << 32)))
    ranges.sort()
    assert all(a[1] <= c[0] for a, c in zip(ranges, ranges[1:])), ranges
    assert ranges[0][0] == 0


def test_bench_gpus_flag_launches_ranks(monkeypatch):
    """`python bench.py --gpus N` without torchrun starts N ranks under torch.distributed.run (before any
    GPU call), forwarding its arguments; with WORLD_SIZE set (a launched rank) it does not re-launch."""
    bench = _bench_module()
    calls = []
    monkeypatch.setattr("subprocess.call", lambda cmd: calls.append(cmd) or 0)
    assert bench.launch_ranks(4, ["--gpus", "4", "--dist-backend", "gloo"]) == 0
    cmd = calls[0]
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=4" in cmd
    assert "--master-addr=127.0.0.1" in cmd and cmd[-4:] == ["--gpus", "4", "--dist-backend", "gloo"]
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench, "launch_ranks", lambda n, argv: calls.append(("launch", n)) or 7)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "3", "--dist-backend", "gloo"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 7 and calls[-1] == ("launch", 3)


def test_refgen_reproduces_reference_generator_bit_exact(inputs):
    """oracle.refgen against the spectra the reference's own generate_signals produced for the fixtures
    (tests/golden/make_golden.py: np.random.seed(20250410); gen(3); gen(2, L) for L in 7, 8, 33, 1000;
    gen(1, 16384), in that order on one global stream)."""
    from oracle.refgen import generate_signals
    np.random.seed(20250410)
    c, n, _, _ = generate_signals(3, signal_length=10000)
    np.testing.assert_array_equal(c, inputs["main_clean64"])
    np.testing.assert_array_equal(n, inputs["main_noisy64"])
    for L in (7, 8, 33, 1000):
        c, n, _, _ = generate_signals(2, signal_length=L, extreme_noise_prob=0.0 if L <= 100 else 0.05)
        np.testing.assert_array_equal(n.astype(np.float32), inputs[f"edge{L}_noisy"])
        np.testing.assert_array_equal(c.astype(np.float32), inputs[f"edge{L}_clean"])
    c, n, _, _ = generate_signals(1, signal_length=16384)
    np.testing.assert_array_equal(n.astype(np.float32), inputs["long_noisy"])


def test_spike_recovery_reproduces_reference_statistics():
    """tests/spike_stats.py on oracle.refgen (bit-exact with the reference generator) reproduces the
    spike statistics make_golden.py --spikes recovered from the reference's own spectra exactly:
    the recovery is deterministic and the GPU test compares like with like."""
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    from oracle.refgen import generate_signals
    from spike_stats import collect
    with open(os.path.join(GOLDEN, "generator_stats.json")) as fh:
        ref = json.load(fh)["spikes"]
    np.random.seed(20250410 + 1)
    clean, noisy, _, nstd = generate_signals(1000, extreme_noise_prob=1.0)
    assert collect(clean, noisy, nstd[:, 0]) == ref


def _acc_worker(rank, world, port, per, out):
    import torch.distributed as dist
    from raman_mi355x import _lib, engine
    from raman_mi355x.distributed import shard
    from test_abi import _acc_of
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    lo, hi = shard(per.shape[0])
    acc = torch.zeros(_lib.ACC_WORDS, dtype=torch.int64)
    for k in range(4):
        acc[k * _lib.ACC_STRIDE: k * _lib.ACC_STRIDE + _lib.ACC_LIMBS] = torch.tensor(_acc_of(per[lo:hi, k]))
    acc[_lib.ACC_COUNT] = hi - lo
    dist.all_reduce(acc, op=dist.ReduceOp.SUM)
    if rank == 0:
        out["sums"] = engine.acc_value(acc).tolist()
    dist.barrier()
    dist.destroy_process_group()


def test_exact_accumulator_allreduce_world2_gloo():
    """Config 4's reduction: exact metric accumulators of two rank shards, all-reduced (int64 SUM over
    gloo), give the same bits as one process over all spectra."""
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    from raman_mi355x import _lib, engine
    from test_abi import _acc_of
    g = np.load(os.path.join(GOLDEN, "metrics.npz"))
    per = g["per_spectrum"].astype(np.float64)
    acc = torch.zeros(_lib.ACC_WORDS, dtype=torch.int64)
    for k in range(4):
        acc[k * _lib.ACC_STRIDE: k * _lib.ACC_STRIDE + _lib.ACC_LIMBS] = torch.tensor(_acc_of(per[:, k]))
    acc[_lib.ACC_COUNT] = per.shape[0]
    one = engine.acc_value(acc).tolist()
    port = _free_port()
    with mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_acc_worker, args=(2, port, per, out), nprocs=2, join=True)
        two = out["sums"]
    assert one == two
    np.testing.assert_allclose(np.array(one[:4]) / one[4], per.mean(axis=0), rtol=1e-13)


def _team16_place(wg, teams, TT):
    """cbam.hip team16_forward's workgroup -> (team, tile, one-XCD candidate), restated: workgroups
    8r + x (r < R0 = tpx TT) form teams 8j + x (r = j TT + tile), the rest the remaining teams in order"""
    tpx = (teams * TT // 8) // TT
    R0 = tpx * TT
    if wg < 8 * R0:
        x, r = wg & 7, wg >> 3
        return (r // TT) * 8 + x, r % TT, x
    i = wg - 8 * R0
    return 8 * tpx + i // TT, i % TT, None


@pytest.mark.parametrize("teams,TT", [(16, 16), (9, 27), (1, 16), (3, 16), (8, 32), (12, 21), (2, 27), (5, 51)])
def test_team16_xcd_placement_is_a_bijection(teams, TT):
    """Every (team, tile) of the launch is owned by exactly one workgroup, and every team formed from
    workgroups 8r + x lies on one round-robin XCD x (L = 10,000: 16 one-XCD teams of 16; L = 16,384:
    8 of 27 plus one spread team)."""
    seen, xcd = {}, {}
    for wg in range(teams * TT):
        team, tile, x = _team16_place(wg, teams, TT)
        assert 0 <= team < teams and 0 <= tile < TT
        assert (team, tile) not in seen
        seen[(team, tile)] = wg
        if x is not None:
            assert wg % 8 == x and xcd.setdefault(team, x) == x
    assert len(seen) == teams * TT


def test_row_views_and_empty_batches_on_the_host():
    """engine._rows: (N, L) and (N, 1, L) -> contiguous (N, L), N = 0 included (no -1 in the view); and
    the eager (reference) forward of every module on an empty CPU batch returns an empty (0, 1, L)."""
    import raman_mi355x as R
    from raman_mi355x import engine
    for shape in [(3, 50), (3, 1, 50), (0, 50), (0, 1, 50)]:
        t = torch.zeros(shape)
        r = engine._rows(t)
        assert tuple(r.shape) == (shape[0], 50) and r.is_contiguous()
    x = torch.zeros((0, 1, 40))
    for name, cls in R.MODELS.items():
        with torch.no_grad():
            y = cls().eval()(x)
        assert tuple(y.shape) == (0, 1, 40), name
