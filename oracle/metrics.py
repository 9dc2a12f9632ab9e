"""numpy restatement of the evaluation metrics (TEST INFRASTRUCTURE — see oracle/__init__).

Reference: */evaulate.py:14-21 (``compute_mse``, ``compute_smoothness``, ``compute_peak_to_peak``),
:35 (``ssim(clean, denoised, data_range=clean.max() - clean.min())``) and :39 (mean over spectra).
SSIM follows scikit-image 0.18.3 ``skimage/metrics/_structural_similarity.py:127-214`` with the
reference's arguments: win_size 7, uniform filter (scipy.ndimage, mode 'reflect'), K1 0.01, K2 0.03,
sample covariance (7/6), mean over the image cropped by 3 on each side.  Because the crop removes
exactly the filter radius, every window that survives the crop lies inside [0, L), so the reflect
border never reaches the mean (restated here with plain windows).
"""
import numpy as np

WIN = 7
K1, K2 = 0.01, 0.03


def _box_mean(a, win=WIN):
    """mean of a[i : i+win] for i = 0 .. L-win (direct window sums, no running-sum cancellation)."""
    return np.lib.stride_tricks.sliding_window_view(a, win).sum(axis=1) / win


def ssim_1d(clean, den):
    x = np.asarray(clean, np.float64)
    y = np.asarray(den, np.float64)
    if x.shape[-1] < WIN:
        raise ValueError("win_size exceeds image extent")
    R = float(x.max() - x.min())
    C1, C2 = (K1 * R) ** 2, (K2 * R) ** 2
    cov = WIN / (WIN - 1)
    ux, uy = _box_mean(x), _box_mean(y)
    uxx, uyy, uxy = _box_mean(x * x), _box_mean(y * y), _box_mean(x * y)
    vx = cov * (uxx - ux * ux)
    vy = cov * (uyy - uy * uy)
    vxy = cov * (uxy - ux * uy)
    S = ((2 * ux * uy + C1) * (2 * vxy + C2)) / ((ux * ux + uy * uy + C1) * (vx + vy + C2))
    return float(S.mean())


def per_spectrum(den, clean):
    """Returns float64 (N, 4): MSE, SSIM, Smoothness, Peak2Peak (evaulate.py:34-37)."""
    den = np.atleast_2d(np.asarray(den))
    clean = np.atleast_2d(np.asarray(clean))
    out = np.empty((den.shape[0], 4), np.float64)
    for i, (y, c) in enumerate(zip(den, clean)):
        y64 = y.astype(np.float64)
        out[i, 0] = np.mean((y64 - c.astype(np.float64)) ** 2)
        out[i, 1] = ssim_1d(c, y)
        out[i, 2] = np.mean(np.abs(np.diff(y64)))
        out[i, 3] = y64.max() - y64.min()
    return out


def sums(den, clean):
    """[ΣMSE, ΣSSIM, ΣSmoothness, ΣPeak2Peak, count] — what the engine all-reduces across ranks."""
    p = per_spectrum(den, clean)
    return np.concatenate([p.sum(axis=0), [float(p.shape[0])]])
