"""numpy restatement of the engine's per-spectrum simulator (TEST INFRASTRUCTURE — see oracle/__init__).

Distributional contract: 数据集产生.py:5-64 (``generate_signals``):
  * piecewise-constant clean signal, segment length U{1..max_repeat} (:31, ``randint(1, max_repeat+1)``),
    truncated at the end (:32), segment value U[0,1) (:33);
  * min-max normalisation with eps 1e-8 (:38-40);
  * Gaussian noise, sigma = sqrt(mean(clean^2) / 10^(snr/10)), snr ~ U[snr_lo, snr_hi) (:43-47);
  * with probability ``extreme_noise_prob`` (:50) 1..3 rectangular spikes (:54), width U{20..99} (:56),
    start U{0..L-width-1} (:57), amplitude U[5,15)*sigma (:58), sign + iff rand > 0.5 (:59-62),
    applied in order on top of the noise.

The reference draws from numpy's *global* RNG in batch order (all segments, then all SNRs, then all
noise, ...), so its streams cannot be reproduced per spectrum.  The engine instead keys a
Philox4x32-10 stream on (seed, spectrum index, draw tag, draw index) so that any index range can be
generated independently on any GPU; this module reproduces those draws exactly (integer draws
bit-exact, float transforms in the same float32 op order).  Parity with the reference itself is
statistical (tests/test_generator_gpu.py, against tests/golden/generator_stats.json).
"""
import numpy as np

PHILOX_M0 = np.uint64(0xD2511F53)
PHILOX_M1 = np.uint64(0xCD9E8D57)
PHILOX_W0 = np.uint32(0x9E3779B9)
PHILOX_W1 = np.uint32(0xBB67AE85)

TAG_SEG, TAG_SCALAR, TAG_SPIKE, TAG_NOISE = 1, 2, 3, 4
_MASK32 = np.uint64(0xFFFFFFFF)
_TWO_M24 = np.float32(1.0 / 16777216.0)


def philox4x32(c0, c1, c2, c3, seed):
    """Philox4x32-10 (Random123).  Counters are uint32 arrays (broadcastable); returns 4 uint32 arrays."""
    c = [np.asarray(v, dtype=np.uint32) for v in np.broadcast_arrays(c0, c1, c2, c3)]
    k0 = np.uint32(seed & 0xFFFFFFFF)
    k1 = np.uint32((seed >> 32) & 0xFFFFFFFF)
    with np.errstate(over="ignore"):
        for r in range(10):
            if r:
                k0 = np.uint32((int(k0) + int(PHILOX_W0)) & 0xFFFFFFFF)
                k1 = np.uint32((int(k1) + int(PHILOX_W1)) & 0xFFFFFFFF)
            p0 = PHILOX_M0 * c[0].astype(np.uint64)
            p1 = PHILOX_M1 * c[2].astype(np.uint64)
            hi0 = (p0 >> np.uint64(32)).astype(np.uint32)
            lo0 = (p0 & _MASK32).astype(np.uint32)
            hi1 = (p1 >> np.uint64(32)).astype(np.uint32)
            lo1 = (p1 & _MASK32).astype(np.uint32)
            c = [hi1 ^ c[1] ^ k0, lo1, hi0 ^ c[3] ^ k1, lo0]
    return c


def u24(x):
    """uint32 -> float32 in [0, 1) with 24 random bits (exact)."""
    return (np.asarray(x, dtype=np.uint32) >> np.uint32(8)).astype(np.float32) * _TWO_M24


def uniform(lo, hi, x):
    return np.float32(lo) + np.float32(np.float32(hi) - np.float32(lo)) * u24(x)


def randint(lo, hi, x):
    """[lo, hi) by 32x32->64 multiply-high (no modulo bias worth mentioning, bit-exact on GPU)."""
    span = np.uint64(hi - lo)
    return lo + ((np.asarray(x, dtype=np.uint32).astype(np.uint64) * span) >> np.uint64(32)).astype(np.int64)


def box_muller(xa, xb):
    u1 = ((np.asarray(xa, np.uint32) >> np.uint32(8)).astype(np.float32) + np.float32(1)) * _TWO_M24
    u2 = u24(xb)
    r = np.sqrt(np.float32(-2.0) * np.log(u1))
    th = np.float32(2.0 * np.pi) * u2
    return (r * np.cos(th)).astype(np.float32), (r * np.sin(th)).astype(np.float32)


def _ctr(index):
    index = int(index)
    return np.uint32(index & 0xFFFFFFFF), np.uint32(index >> 32)


def generate_one(seed, index, L=10000, snr_range=(20.0, 37.0), extreme_noise_prob=0.05,
                 max_repeat=40):
    """One spectrum; returns dict(clean, noisy float32 (L,), snr, noise_std float32, plus draws)."""
    s_lo, s_hi = _ctr(index)
    # --- segments (数据集产生.py:28-35) -------------------------------------------------------
    n_max = L  # every segment has length >= 1
    k = np.arange(n_max, dtype=np.int64)
    x = philox4x32((k >> 1).astype(np.uint32), TAG_SEG, s_lo, s_hi, seed)
    xs = np.stack(x)                                      # (4, n_max)
    lane = (k & 1) * 2
    lens = randint(1, max_repeat + 1, xs[lane, k])
    vals = u24(xs[lane + 1, k])
    ends = np.cumsum(lens)
    n_seg = int(np.searchsorted(ends, L, side="left")) + 1   # first segment reaching L
    starts = ends[:n_seg] - lens[:n_seg]
    vals = vals[:n_seg]
    raw = np.repeat(vals, np.minimum(lens[:n_seg], L - starts))
    assert raw.shape == (L,)
    # --- normalisation (:38-40) -------------------------------------------------------------
    mn = vals.min()
    mx = vals.max()
    den = np.float32(np.float32(mx - mn) + np.float32(1e-8))
    cvals = ((vals - mn) / den).astype(np.float32)
    clean = ((raw - mn) / den).astype(np.float32)
    seg_len = np.minimum(lens[:n_seg], L - starts).astype(np.float64)
    power = float(np.sum(seg_len * cvals.astype(np.float64) ** 2) / L)
    # --- scalars ------------------------------------------------------------------------------
    sc = philox4x32(0, TAG_SCALAR, s_lo, s_hi, seed)
    snr = uniform(snr_range[0], snr_range[1], sc[0])
    noise_std = np.float32(np.sqrt(power / (10.0 ** (float(snr) / 10.0))))
    extreme = bool(u24(sc[1]) < np.float32(extreme_noise_prob))
    n_spikes = int(randint(1, 4, sc[2])) if extreme else 0
    # --- noise (:43-47) -----------------------------------------------------------------------
    q = np.arange((L + 3) // 4, dtype=np.uint32)
    nz = philox4x32(q, TAG_NOISE, s_lo, s_hi, seed)
    z0, z1 = box_muller(nz[0], nz[1])
    z2, z3 = box_muller(nz[2], nz[3])
    z = np.stack([z0, z1, z2, z3], axis=1).reshape(-1)[:L]
    noisy = (clean + (noise_std * z).astype(np.float32)).astype(np.float32)
    # --- spikes (:50-62) ----------------------------------------------------------------------
    spikes = []
    for s in range(n_spikes):
        sx = philox4x32(s, TAG_SPIKE, s_lo, s_hi, seed)
        width = int(randint(20, 100, sx[0]))
        if L - width <= 0:          # the reference raises here (randint low >= high); we clamp
            width, start = L, 0
        else:
            start = int(randint(0, L - width, sx[1]))
        amp = np.float32(uniform(5.0, 15.0, sx[2]) * noise_std)
        sign = 1.0 if u24(sx[3]) > np.float32(0.5) else -1.0
        noisy[start:start + width] = (noisy[start:start + width] + np.float32(sign) * amp).astype(np.float32)
        spikes.append((start, width, float(sign * amp)))
    return dict(clean=clean, noisy=noisy, snr=np.float32(snr), noise_std=noise_std,
                seg_lens=lens[:n_seg], seg_vals=vals, spikes=spikes, extreme=extreme)


def generate(seed, first_index, n, L=10000, **kw):
    outs = [generate_one(seed, first_index + i, L, **kw) for i in range(n)]
    return (np.stack([o["clean"] for o in outs]), np.stack([o["noisy"] for o in outs]),
            np.array([o["snr"] for o in outs], np.float32),
            np.array([o["noise_std"] for o in outs], np.float32), outs)
