"""On-device simulator vs the numpy restatement (same Philox draws) and vs reference statistics."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

SEED = 20250410


def _gpu(n, first=0, L=10000, **kw):
    from raman_mi355x import engine
    c, x, s, sd = engine.generate(n, SEED, first_index=first, signal_length=L, **kw)
    torch.cuda.synchronize()
    return c.cpu().numpy(), x.cpu().numpy(), s.cpu().numpy(), sd.cpu().numpy()


@pytest.mark.parametrize("L", [10000, 16384, 1000, 101, 7])
def test_matches_numpy_restatement(L):
    from oracle.generator import generate
    n = 6
    kw = dict(extreme_noise_prob=0.5)            # exercise the spike path often
    c, x, s, sd = _gpu(n, first=123, L=L, **kw)
    oc, ox, os_, osd, outs = generate(SEED, 123, n, L, **kw)
    assert np.array_equal(s, os_), "SNR draws differ"
    np.testing.assert_allclose(sd, osd, rtol=2e-6)
    # clean: identical segment structure; values equal up to division rounding
    np.testing.assert_allclose(c, oc, rtol=0, atol=1e-6)
    assert np.array_equal(np.diff(c, axis=1) != 0, np.diff(oc, axis=1) != 0)
    # noisy: logf/sincosf differ from numpy by a few ulp, scaled by sigma (<0.1)
    np.testing.assert_allclose(x, ox, rtol=0, atol=2e-6)


def test_index_ranges_are_independent_of_batching():
    c_all, x_all, _, _ = _gpu(16, first=0)
    c_sub, x_sub, _, _ = _gpu(4, first=10)
    assert np.array_equal(c_all[10:14], c_sub) and np.array_equal(x_all[10:14], x_sub)


def test_statistics_match_reference():
    """χ²/range checks against the distributional contract and reference-generated statistics."""
    with open(os.path.join(GOLDEN, "generator_stats.json")) as fh:
        ref = json.load(fh)
    n = 2000
    c, x, s, sd = _gpu(n)
    # per-row normalisation (数据集产生.py:38-40)
    assert np.all(c.min(axis=1) == 0.0)
    assert np.all(c.max(axis=1) > 0.9999)
    # segment lengths: U{1..40}, last (truncated) run excluded
    counts = np.zeros(41)
    for row in c:
        b = np.concatenate([[0], np.flatnonzero(np.diff(row) != 0) + 1, [row.size]])
        runs = np.diff(b)[:-1]
        np.add.at(counts, runs[runs <= 40], 1)
    obs = counts[1:]
    exp = np.full(40, obs.sum() / 40)
    chi2 = ((obs - exp) ** 2 / exp).sum()
    assert chi2 < 80.0, f"segment-length chi2 {chi2:.1f} (39 dof, p~1e-4 at 80)"
    ref_obs = np.array(ref["seg_len_counts"], float)
    ref_exp = ref_obs.sum() * obs / obs.sum()
    chi2_ref = ((ref_obs - ref_exp) ** 2 / np.maximum(ref_exp, 1)).sum()
    assert chi2_ref < 90.0, f"segment lengths vs reference chi2 {chi2_ref:.1f}"
    # SNR ~ U[20, 37): 17 equal bins
    h, _ = np.histogram(s, bins=17, range=(20, 37))
    chi2_snr = ((h - n / 17) ** 2 / (n / 17)).sum()
    assert s.min() >= 20 and s.max() < 37 and chi2_snr < 45, f"snr chi2 {chi2_snr:.1f}"
    # noise std range and signal power like the reference
    q = np.quantile(sd, [0.1, 0.5, 0.9])
    rq = np.array(ref["noise_std_quantiles"])[[1, 2, 3]]
    assert np.all(np.abs(q - rq) / rq < 0.1), (q, rq)
    power = np.mean(c.astype(np.float64) ** 2, axis=1).mean()
    assert abs(power - ref["power_mean"]) < 0.01
    # spiked fraction ~ Binomial(n, 0.05): detect >= 20 consecutive points beyond 4 sigma
    spiked = 0
    for r, sig in zip(x - c, sd):
        big = (np.abs(r) > 4 * sig).astype(np.int32)
        spiked += bool((np.convolve(big, np.ones(20, np.int32), "valid") == 20).any())
    frac = spiked / n
    assert abs(frac - 0.05) < 4 * np.sqrt(0.05 * 0.95 / n) + 0.005, frac
    assert abs(frac - ref["spiked_fraction"]) < 0.03


def test_spike_process_matches_reference():
    """The spike process (数据集产生.py:50-62) on the device simulator with every spectrum spiked
    (extreme_noise_prob = 1): spike count U{1,2,3}, width U{20..99}, start U{0..L-W-1}, amplitude/σ
    U[5,15), sign Bernoulli(0.5) — χ² against the uniform contract (p = 0.001 bounds) and two-sample
    χ² against the same statistics of 1000 reference-generated spectra (generator_stats.json
    "spikes", make_golden.py --spikes), both recovered by tests/spike_stats.py."""
    from spike_stats import chi2_two_sample, chi2_uniform, collect
    with open(os.path.join(GOLDEN, "generator_stats.json")) as fh:
        ref = json.load(fh)["spikes"]
    n = 2000
    c, x, s, sd = _gpu(n, first=5000, extreme_noise_prob=1.0)
    st = collect(c, x, sd)
    print({k: v for k, v in st.items()})
    # every spectrum carries 1..3 spikes (a count outside means two edges coincided: rare)
    assert st["count_hist"][0] + st["count_hist"][4] <= n // 200, st["count_hist"]
    assert st["overlapped_spectra"] < 0.08 * n
    bounds = {"count_hist": 13.8, "width_hist": 24.3, "amp_hist": 27.9, "start_hist": 27.9}   # chi2(dof) at p=1e-3
    for key, bound in bounds.items():
        h = st[key][1:4] if key == "count_hist" else st[key]
        r = ref[key][1:4] if key == "count_hist" else ref[key]
        u, t = chi2_uniform(h), chi2_two_sample(h, r)
        print(f"{key}: chi2 vs uniform {u:.1f}, vs reference {t:.1f} (bound {bound})")
        assert u < bound, (key, u)
        assert t < bound, (key, t)
    assert 20 <= st["width_min_max"][0] and st["width_min_max"][1] <= 99
    p = st["sign_pos"] / st["sign_n"]
    assert abs(p - 0.5) < 4 * np.sqrt(0.25 / st["sign_n"]), p
    pr = ref["sign_pos"] / ref["sign_n"]
    assert abs(p - pr) < 4 * np.sqrt(0.25 / st["sign_n"] + 0.25 / ref["sign_n"])
