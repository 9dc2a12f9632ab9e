"""Spike parameters recovered from (clean, noisy, noise_std) triples — test infrastructure for the
generator's distributional contract (数据集产生.py:50-62: per spiked spectrum U{1,2,3} spikes, each a
box of width U{20..99} starting at U{0..L-W-1}, amplitude U[5,15)·σ, sign Bernoulli(0.5)).

The residual r = (noisy − clean)/σ is N(0,1) noise plus a sum of ±a boxes.  A box edge is a step of
|a| >= 5: the difference of the means of the 10 samples after and before a position (noise std
0.45) peaks there.  Edges are the extrema of that difference beyond 2.5 (5.6 σ: no false edges in
practice), refined to the least-squares step position.  The spike count is #edges / 2 (exact unless
two edges coincide); width, start, amplitude and sign are read from spectra whose boxes do not
overlap (consecutive edge pairs of opposite sign and equal size), which drops ~3 % of the spiked
spectra — the same selection is applied to the reference's spectra the GPU generator is compared
with (make_golden.py --spikes), so it cancels in the two-sample tests.
"""
import numpy as np

W = 10          # half-window of the edge detector
THRESH = 2.5    # |mean after − mean before| threshold (the smallest step is 5)


def edges(r):
    """[(position, step)] of the box edges in the normalised residual r (1-D float64)."""
    L = r.size
    cs = np.concatenate([[0.0], np.cumsum(r)])
    i = np.arange(W, L - W + 1)
    d = (cs[i + W] - cs[i]) / W - (cs[i] - cs[i - W]) / W          # step at i: mean r[i:i+W] - mean r[i-W:i]
    out = []
    above = np.abs(d) > THRESH
    k = 0
    n = d.size
    while k < n:
        if not above[k]:
            k += 1
            continue
        j = k
        while j < n and above[j] and np.sign(d[j]) == np.sign(d[k]):
            j += 1
        m = k + int(np.argmax(np.abs(d[k:j])))
        p = int(i[m])
        # least-squares refinement of the step position within +-3 samples
        best, bp = None, p
        for q in range(max(W, p - 3), min(L - W, p + 3) + 1):
            a, b = r[q - W:q], r[q:q + W]
            sse = ((a - a.mean()) ** 2).sum() + ((b - b.mean()) ** 2).sum()
            if best is None or sse < best:
                best, bp = sse, q
        out.append((bp, float(d[m])))
        k = j
    return out


def spectrum_spikes(clean, noisy, sigma):
    """(n_spikes, [(start, width, amp_over_sigma, sign)] or None when boxes overlap)."""
    r = (noisy.astype(np.float64) - clean.astype(np.float64)) / float(sigma)
    e = edges(r)
    if not e:
        return 0, []
    n = len(e) // 2
    boxes = []
    if len(e) % 2:
        return n, None
    for k in range(0, len(e), 2):
        (p0, s0), (p1, s1) = e[k], e[k + 1]
        if np.sign(s0) == np.sign(s1) or not (0.6 < abs(s0) / abs(s1) < 1.67):
            return n, None
        if not 20 <= p1 - p0 <= 99:            # impossible for one box: an overlap paired the wrong edges
            return n, None
        amp = float(np.mean(r[p0 + 2:p1 - 2]))
        boxes.append((p0, p1 - p0, abs(amp), 1 if s0 > 0 else -1))
    return n, boxes


def collect(clean, noisy, sigma):
    """Histograms of the spike parameters over all spectra (sigma: per-spectrum noise std)."""
    L = clean.shape[1]
    counts = np.zeros(5, np.int64)         # spectra with 0, 1, 2, 3, >3 spikes
    widths, starts, amps, signs = [], [], [], []
    overlapped = 0
    for c, x, s in zip(clean, noisy, np.ravel(sigma)):
        n, boxes = spectrum_spikes(c, x, s)
        counts[min(n, 4)] += 1
        if boxes is None:
            overlapped += 1
            continue
        for p0, w, a, sg in boxes:
            widths.append(w)
            starts.append(p0 / (L - w))      # U[0, 1) for a start drawn from U{0..L-w-1}
            amps.append(a)
            signs.append(sg)
    widths = np.array(widths)
    return {
        "n": int(clean.shape[0]), "L": int(L),
        "count_hist": counts.tolist(),
        "width_hist": np.histogram(widths, bins=8, range=(20, 100))[0].tolist(),
        "amp_hist": np.histogram(amps, bins=10, range=(5, 15))[0].tolist(),
        "start_hist": np.histogram(starts, bins=10, range=(0, 1))[0].tolist(),
        "sign_pos": int(np.sum(np.array(signs) > 0)), "sign_n": int(len(signs)),
        "overlapped_spectra": int(overlapped),
        "width_min_max": [int(widths.min()), int(widths.max())] if widths.size else None,
    }


def chi2_uniform(h):
    h = np.asarray(h, float)
    e = h.sum() / h.size
    return float(((h - e) ** 2 / e).sum())


def chi2_two_sample(a, b):
    """χ² of two histograms over the same bins (dof = bins − 1 for non-empty bins)."""
    a, b = np.asarray(a, float), np.asarray(b, float)
    ka, kb = np.sqrt(b.sum() / a.sum()), np.sqrt(a.sum() / b.sum())
    m = (a + b) > 0
    return float((((ka * a - kb * b)[m]) ** 2 / (a + b)[m]).sum())
