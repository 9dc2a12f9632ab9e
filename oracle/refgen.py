"""numpy restatement of the REFERENCE simulator's exact draw sequence (TEST INFRASTRUCTURE — see
oracle/__init__).  Reference: 数据集产生.py:5-64 ``generate_signals``.

The reference draws from numpy's legacy global RNG in batch order, so the only way to regenerate its
data sets bit for bit (config 1's ``data/test.npz``: ``np.random.seed(20250410)``, 1,000 spectra,
SURVEY.md §8d) is to repeat that order exactly:

  1. per spectrum, per segment: ``randint(1, max_repeat + 1)`` then ``uniform(0, 1)`` (:28-35), the
     segment truncated at the end of the spectrum (:32);
  2. min-max normalisation with eps 1e-8 (:38-40);
  3. ``uniform(snr_lo, snr_hi, (n, 1))`` for all spectra (:44), sigma = sqrt(mean(clean^2) /
     10^(snr / 10)) (:43, :45), then ``randn(n, L)`` for all spectra at once (:46-47);
  4. ``rand(n) < p`` selects the spiked spectra (:50-51); per spiked spectrum ``randint(1, 4)`` spikes
     (:54), each ``randint(20, 100)`` wide (:56) at ``randint(0, L - width)`` (:57) with amplitude
     ``uniform(5, 15) * sigma`` (:58) and sign ``rand() > 0.5`` (:59-62).

Pinned bit-exact against the fixtures the reference itself produced (tests/golden/inputs.npz, made by
tests/golden/make_golden.py from the AST-extracted reference function): tests/test_cpu_host.py.
The ENGINE's generator is a different, counter-based stream (oracle/generator.py); its parity with
the reference is statistical.
"""
import numpy as np


def _clean_rows(rng, n, L, max_repeat):
    out = np.zeros((n, L))
    for row in out:                                   # :28-35, one spectrum at a time
        pos = 0
        while pos < L:
            run = min(rng.randint(1, max_repeat + 1), L - pos)
            row[pos:pos + run] = rng.uniform(0, 1)
            pos += run
    lo = out.min(axis=1, keepdims=True)               # :38-40
    hi = out.max(axis=1, keepdims=True)
    return (out - lo) / (hi - lo + 1e-8)


def _spikes(rng, noisy, sigma, p):
    n, L = noisy.shape
    for i in np.where(rng.rand(n) < p)[0]:            # :50-62
        for _ in range(rng.randint(1, 4)):
            width = rng.randint(20, 100)
            start = rng.randint(0, L - width)
            amp = rng.uniform(5, 15) * sigma[i]
            sign_up = rng.rand() > 0.5
            seg = noisy[i, start:start + width]
            noisy[i, start:start + width] = seg + amp if sign_up else seg - amp


def generate_signals(num_samples, signal_length=10000, snr_range=(20, 37), extreme_noise_prob=0.05,
                     max_repeat=40, rng=np.random):
    """(clean, noisy, snrs, noise_std) float64, exactly as 数据集产生.py:5-64 with the same global RNG."""
    clean = _clean_rows(rng, num_samples, signal_length, max_repeat)
    power = np.mean(clean ** 2, axis=1, keepdims=True)                      # :43
    snrs = rng.uniform(snr_range[0], snr_range[1], size=(num_samples, 1))   # :44
    sigma = np.sqrt(power / (10 ** (snrs / 10)))                            # :45
    noisy = clean + sigma * rng.randn(num_samples, signal_length)           # :46-47
    _spikes(rng, noisy, sigma, extreme_noise_prob)
    return clean, noisy, snrs, sigma
