"""The reference's on-disk data format (数据集产生.py:67-79, consumed by */evaulate.py:61-62 and
*/train.py:48-56): ``np.savez_compressed`` with float64 ``clean_signals`` / ``noisy_signals`` (N, L)
and ``snrs`` / ``noise_std`` (N, 1).  Loading never unpickles (``allow_pickle=False``)."""
import numpy as np

KEYS = ("clean_signals", "noisy_signals", "snrs", "noise_std")


def save_dataset(path, clean, noisy, snrs, noise_std):
    def host(a, two_d):
        a = a.detach().cpu().numpy() if hasattr(a, "detach") else np.asarray(a)
        a = a.astype(np.float64)
        return a.reshape(a.shape[0], -1) if two_d else a.reshape(-1, 1)
    np.savez_compressed(path, clean_signals=host(clean, True), noisy_signals=host(noisy, True),
                        snrs=host(snrs, False), noise_std=host(noise_std, False))


def load_dataset(path):
    with np.load(path, allow_pickle=False) as d:
        missing = [k for k in KEYS[:2] if k not in d.files]
        if missing:
            raise KeyError(f"{path}: missing {missing}")
        return {k: d[k] for k in KEYS if k in d.files}
