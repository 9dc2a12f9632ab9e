"""C-ABI checks that need no GPU: the library loads, exports every declared entry point, names the
reference state_dict keys, and packs (BN folding + MFMA fragment layout) exactly as documented."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from conftest import ROOT, golden_state_dict

ARCHS = ["DenoiseCNN", "RRCDNet", "DSDN", "ADSDN", "PIDN", "APIDN"]


@pytest.fixture(scope="module")
def lib():
    from raman_mi355x import _lib
    return _lib.lib()


def test_exports_every_declared_symbol(lib):
    with open(os.path.join(ROOT, "include", "raman_mi355x.h")) as fh:
        header = fh.read()
    declared = set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+(rdn_\w+)\s*\(", header, re.M))
    from raman_mi355x import _lib
    assert declared == set(_lib.EXPORTED), declared ^ set(_lib.EXPORTED)
    for name in declared:
        assert hasattr(lib, name), name
    assert lib.rdn_version() == 6


def test_library_built_from_these_sources(lib):
    """The .so carries the sha256 stamp of the sources it was compiled from (csrc/Makefile); the
    loader refuses a library whose stamp differs from this tree's sources."""
    from raman_mi355x import _lib
    assert lib.rdn_build_id().decode() == _lib.source_hash()


def test_plain_bf16_is_refused_and_unsafe_mode_is_explicit():
    import raman_mi355x as R
    from raman_mi355x import engine
    m = R.RRCDNet()
    for bad in ("bf16", "bfloat16", torch.bfloat16):
        with pytest.raises(ValueError, match="bf16-unsafe"):
            m.set_engine_dtype(bad)
    assert m.set_engine_dtype("bf16-unsafe").engine_dtype == "bf16-unsafe"
    assert engine._dtype("f16f8") == 3 and engine._dtype(torch.float32) == 0


@pytest.mark.parametrize("spelling", ["f16", "float16", torch.float16])
def test_every_f16_spelling_selects_the_same_arithmetic(spelling):
    """'f16', 'float16' and torch.float16 all mean the network's fastest mode within 2e-2: RDN_F16MIX
    on RRCDNet (plain f16 misses the bar there), RDN_F16 elsewhere; only 'f16-plain' opts out.  The
    functional engine API resolves the same way as the module."""
    import raman_mi355x as R
    from raman_mi355x import engine
    for arch in ARCHS:
        code = engine.resolve_dtype(arch, spelling)
        assert code == (5 if arch == "RRCDNet" else 4), (arch, code)
        m = R.MODELS[arch]().set_engine_dtype(spelling)
        assert m.engine_code == code and m.engine_dtype == "f16"
        assert engine.resolve_dtype(arch, "f16-plain") == 4
        assert R.MODELS[arch]().set_engine_dtype("f16-plain").engine_dtype == "f16-plain"
    assert engine.packed_size("RRCDNet", spelling) == engine.packed_size("RRCDNet", "f16mix")
    with pytest.raises(ValueError, match="resolves per network"):
        engine._dtype(spelling)


def test_16bit_dtypes_take_a_status_workspace(lib):
    """ABI v5: every 16-bit dtype on the fused networks takes a 256-byte workspace whose first word is
    the status word -- RDN_F16F8 / RDN_F16MIX report a saturated e4m3 plane through its range bit
    (rdn_forward_status: RDN_ERANGE = -6), every 16-bit dtype an input beyond [-4, 4] through its gate
    bit; fp32 needs none, and rdn_workspace_init refuses a too-small workspace (no GPU call is made)."""
    from raman_mi355x import _lib, engine
    n = ctypes.c_size_t()
    assert (engine.STATUS_RANGE, engine.STATUS_GATE) == (1, 2)
    for arch in (0, 1, 2, 4):
        for code, need in ((0, 0), (2, 256), (4, 256), (1, 256), (3, 256)):
            assert lib.rdn_workspace_size(arch, code, 8, 1000, ctypes.byref(n), None) == 0
            assert n.value == need, (arch, code, n.value)
            assert engine.needs_workspace(arch, code) == (need > 0)
    assert lib.rdn_workspace_size(1, 5, 8, 1000, ctypes.byref(n), None) == 0 and n.value == 256
    assert lib.rdn_workspace_init(1, 5, 8, 1000, None, 0, None) == -4
    assert lib.rdn_workspace_init(0, 0, 8, 1000, None, 0, None) == 0
    assert _lib.RDN_ERANGE == -6 and issubclass(_lib.RangeError, _lib.EngineError)


def test_f16mix_is_refused_for_other_networks_before_dispatch(lib):
    """RDN_F16MIX exists for RRCDNet only: every entry point refuses it for the other networks with
    RDN_EUNSUPPORTED before any per-network (e.g. CBAM) dispatch."""
    n = ctypes.c_size_t()
    for arch in (0, 2, 3, 4, 5):
        assert lib.rdn_workspace_size(arch, 5, 4, 1000, ctypes.byref(n), None) == -2
        assert b"RRCDNet" in lib.rdn_last_error()
        assert lib.rdn_forward(arch, 5, ctypes.c_void_p(1 << 32), ctypes.c_void_p(1 << 33), ctypes.c_void_p(1 << 34),
                               1, 1000, None, 0, None) == -2
        assert lib.rdn_forward_status(arch, 5, 1, 1000, None, 0, None) == -2
        assert lib.rdn_workspace_init(arch, 5, 1, 1000, None, 0, None) == -2


def test_blob_layout_tag(lib):
    """rdn_pack tags every blob with (arch, dtype); rdn_check_blob / rdn_get_correction_mask refuse a
    blob of another layout (an RDN_F16F8 blob is one record short of what RDN_F16MIX reads)."""
    from raman_mi355x import engine, _lib
    sd = golden_state_dict("RRCDNet", "synth")
    b8 = engine.pack("RRCDNet", sd, "f16f8", "cpu")
    bm = engine.pack("RRCDNet", sd, "f16mix", "cpu")
    engine.check_blob("RRCDNet", "f16f8", b8)
    engine.check_blob("RRCDNet", "f16", bm)
    assert engine.correction_mask("RRCDNet", "f16", bm) == 0x1f << 10
    with pytest.raises(_lib.EngineError, match="needs"):
        engine.check_blob("RRCDNet", "f16mix", b8)                 # too small for the F16MIX layout
    padded = torch.cat([b8, torch.zeros(bm.numel() - b8.numel(), dtype=torch.uint8)])
    with pytest.raises(_lib.EngineError, match="dtype 3, not arch 1 dtype 5"):
        engine.check_blob("RRCDNet", "f16mix", padded)
    with pytest.raises(_lib.EngineError, match="no layout tag"):
        engine.check_blob("RRCDNet", "f16mix", torch.zeros_like(bm))
    for arch in ARCHS:
        for dt in ("fp32", "f16-plain", "f16f8"):
            engine.check_blob(arch, dt, engine.pack(arch, golden_state_dict(arch, "synth"), dt, "cpu"))


def _acc_of(values):
    """Host restatement of the device accumulator (metrics.hip to_limbs): limbs of one metric."""
    from fractions import Fraction
    from raman_mi355x import _lib
    limbs = [0] * _lib.ACC_LIMBS
    for v in values:
        f = Fraction(v) * 2 ** _lib.ACC_FRAC_BITS
        mag = abs(f.numerator) // f.denominator                    # truncation toward zero
        for j in range(_lib.ACC_LIMBS):
            c = (mag >> (32 * j)) & 0xffffffff
            limbs[j] += -c if v < 0 else c
    return limbs


def test_exact_accumulator_rounds_the_exact_sum_once(lib):
    """rdn_acc_value: the exact total of the (2^-128-truncated) values, rounded once to double --
    independent of summation order (the reason config-4 sums are identical for any world size)."""
    from fractions import Fraction
    from raman_mi355x import engine, _lib
    rng = np.random.default_rng(5)
    vals = [np.concatenate([rng.uniform(-1, 1, 500) * 10.0 ** rng.integers(-12, 12, 500),
                            [1e-40, -3e-39, 2.0 ** 63, -(2.0 ** 62), 0.1, 0.2, 0.3]]) for _ in range(4)]
    acc = torch.zeros(_lib.ACC_WORDS, dtype=torch.int64)
    for k in range(4):
        acc[k * _lib.ACC_STRIDE: k * _lib.ACC_STRIDE + _lib.ACC_LIMBS] = torch.tensor(_acc_of(vals[k]))
    acc[_lib.ACC_COUNT] = 507
    out = engine.acc_value(acc).numpy()
    for k in range(4):
        exact = sum(Fraction(abs(Fraction(v)) * 2 ** 128).__floor__() * (1 if v >= 0 else -1) for v in vals[k])
        assert out[k] == float(Fraction(exact, 2 ** 128)), k
    assert out[4] == 507
    acc[_lib.ACC_LIMBS] = 1                                          # an out-of-range value in metric 0
    assert np.isnan(engine.acc_value(acc).numpy()[0])


def test_forward_status_without_gpu_reports_error_not_crash(lib):
    """rdn_forward_status synchronises the stream; on a host without a device it must fail cleanly."""
    rc = lib.rdn_forward_status(99, 0, 1, 100, None, 0, None)
    assert rc == -1 and b"unknown arch" in lib.rdn_last_error()
    rc = lib.rdn_workspace_init(99, 0, 1, 100, None, 0, None)
    assert rc == -1


@pytest.mark.parametrize("arch", ARCHS)
def test_param_names_are_reference_keys(arch):
    from raman_mi355x import engine
    from conftest import load_golden
    import json
    keys = json.loads(str(load_golden(arch)["keys"]))
    names = engine.param_names(arch)
    assert len(names) == len(set(names))
    assert set(names) <= set(keys)
    # everything except the BN step counters feeds the engine
    assert set(keys) - set(names) == {k for k in keys if k.endswith("num_batches_tracked")}
    # order follows the state_dict order (the forward order of the reference modules)
    assert names == [k for k in keys if k in set(names)]


def test_errors_are_reported_not_raised(lib):
    from raman_mi355x import engine, _lib
    n = ctypes.c_size_t()
    assert lib.rdn_packed_size(99, 0, ctypes.byref(n)) == -1
    assert b"bad argument" in lib.rdn_last_error()
    sd = golden_state_dict("DenoiseCNN", "synth")
    sd["layers.2.0.weight"] = sd["layers.2.0.weight"][:, :32]        # wrong shape
    with pytest.raises(_lib.EngineError, match="expected 12288 elements"):
        engine.pack("DenoiseCNN", sd, "fp32", "cpu")
    with pytest.raises(KeyError):
        engine.pack("DenoiseCNN", {}, "fp32", "cpu")
    # overlapping x / y are refused before anything touches the device (addresses are never read)
    base = 1 << 32
    assert lib.rdn_forward(1, 4, ctypes.c_void_p(base), ctypes.c_void_p(base), ctypes.c_void_p(base + 4 * 999),
                           2, 1000, None, 0, None) == -1
    assert b"overlap" in lib.rdn_last_error()


def _fold(sd, conv, bn):
    w = sd[conv + ".weight"].double().numpy()
    b = sd[conv + ".bias"].double().numpy()
    if bn:
        s = sd[bn + ".weight"].double().numpy() / np.sqrt(sd[bn + ".running_var"].double().numpy() + 1e-5)
        w = w * s[:, None, None]
        b = (b - sd[bn + ".running_mean"].double().numpy()) * s + sd[bn + ".bias"].double().numpy()
    return w.astype(np.float32), b.astype(np.float32)


def _bf16_to_f32(u16):
    return (u16.astype(np.uint32) << 16).view(np.float32)


def _f32_to_bf16(f):
    u = f.astype(np.float32).view(np.uint32).astype(np.uint64)
    return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)


SMALL = 64 * 256 * 4


@pytest.mark.parametrize("dtype", ["fp32", "bf16-unsafe", "bf16x3"])
def test_pack_layout_rrcdnet(dtype):
    """Unpack the blob with the layout documented in csrc/common.hpp and compare with BN folding."""
    from raman_mi355x import engine
    sd = golden_state_dict("RRCDNet", "trained")
    blob = engine.pack("RRCDNet", sd, dtype, "cpu").numpy()
    assert blob.size == engine.packed_size("RRCDNet", dtype)
    small = blob[:SMALL].view(np.float32).reshape(64, 256)
    # stem of the right branch: slot 0, BN folded
    w, b = _fold(sd, "right_net.0", "right_net.1")
    np.testing.assert_allclose(small[0, :192].reshape(64, 3), w[:, 0, :], rtol=1e-6)
    np.testing.assert_allclose(small[0, 192:], b, rtol=1e-6, atol=1e-7)
    # left head: slot 3
    w, b = _fold(sd, "left_net.19", None)
    np.testing.assert_array_equal(small[3, :192].reshape(64, 3), w[0])
    assert small[3, 192] == b[0]
    # big layer 16 = left_net.3.0 (first dilated conv) in every dtype's order
    big = blob[SMALL:]
    if dtype == "bf16-unsafe":
        layer, nbytes = 16, 24832              # the right head is big layer 15 in bf16
    else:
        layer, nbytes = 15, 49408
    w, b = _fold(sd, "left_net.3.0", None)
    L = big[layer * nbytes:(layer + 1) * nbytes]
    lane = np.arange(64)
    if dtype == "fp32":
        frag = L[:49152].view(np.float32).reshape(4, 12, 64, 4)
        for m in range(4):
            for tg in range(12):
                t, g = tg >> 2, tg & 3
                for i in range(4):
                    exp = w[16 * m + (lane & 15), 16 * g + 4 * (lane >> 4) + i, t]
                    np.testing.assert_array_equal(frag[m, tg, :, i], exp)
        np.testing.assert_array_equal(L[49152:49408].view(np.float32), b)
    elif dtype == "bf16-unsafe":
        # fused16.hip K order: element j of lane quarter q in k-step (t, u) is channel
        # 32u + 4q + (j & 3) + 16 (j >> 2) (common.hpp h16_channel)
        frag = L[:24576].view(np.uint16).reshape(4, 6, 64, 8)
        for m in range(4):
            for s in range(6):
                t, u = s >> 1, s & 1
                for j in range(8):
                    cin = 32 * u + 4 * (lane >> 4) + (j & 3) + 16 * (j >> 2)
                    exp = w[16 * m + (lane & 15), cin, t]
                    np.testing.assert_array_equal(frag[m, s, :, j], _f32_to_bf16(exp))
        np.testing.assert_array_equal(L[24576:24832].view(np.float32), b)
    else:
        frag = L[:49152].view(np.uint16).reshape(4, 6, 2, 64, 8)
        for m in range(4):
            for s in range(6):
                t, u = s >> 1, s & 1
                for j in range(8):
                    exp = w[16 * m + (lane & 15), 32 * u + 8 * (lane >> 4) + j, t]
                    hi = _bf16_to_f32(frag[m, s, 0, :, j])
                    lo = _bf16_to_f32(frag[m, s, 1, :, j])
                    np.testing.assert_array_equal(frag[m, s, 0, :, j], _f32_to_bf16(exp))
                    assert np.all(np.abs(hi.astype(np.float64) + lo - exp) <= 2.0 ** -16 * np.abs(exp) + 1e-30)
        np.testing.assert_array_equal(L[49152:49408].view(np.float32), b)


def test_bn_folding_matches_reference_math():
    """Folding is exact in fp64: conv(x, W') + b' == BN(conv(x, W) + b) to fp32 rounding."""
    sd = golden_state_dict("RRCDNet", "trained")
    x = torch.randn(2, 64, 300, dtype=torch.float64)
    w, b = _fold(sd, "right_net.5.0", "right_net.5.1")
    y_fold = torch.nn.functional.conv1d(x, torch.from_numpy(w).double(), torch.from_numpy(b).double(), padding=1)
    y = torch.nn.functional.conv1d(x, sd["right_net.5.0.weight"].double(), sd["right_net.5.0.bias"].double(), padding=1)
    y = torch.nn.functional.batch_norm(y, sd["right_net.5.1.running_mean"].double(), sd["right_net.5.1.running_var"].double(),
                                       sd["right_net.5.1.weight"].double(), sd["right_net.5.1.bias"].double(), False, 0, 1e-5)
    assert (y_fold - y).abs().max() / y.abs().max() < 1e-6


def test_pack_layout_f16f8():
    """RDN_F16F8 layer (common.hpp BIG_BYTES_H8): f16 hi fragments, e4m3 [lo | hi] correction fragments
    with per-(row, 32-channel block, tap) E8M0 scales; hi + lo reproduces the folded weight to ~2^-15."""
    from raman_mi355x import engine
    sd = golden_state_dict("RRCDNet", "trained")
    blob = engine.pack("RRCDNet", sd, "f16f8", "cpu").numpy()
    assert blob.size == engine.packed_size("RRCDNet", "f16f8") == SMALL + 29 * 50432
    w, b = _fold(sd, "left_net.3.0", None)          # big layer 15
    w64 = _fold_f64(sd, "left_net.3.0")
    L = blob[SMALL + 15 * 50432:SMALL + 16 * 50432]
    lane = np.arange(64)
    main = L[:24576].view(np.float16).reshape(4, 6, 64, 8)
    corr = L[24576:49152].reshape(4, 3, 64, 32)
    scales = L[49152:50176].view(np.uint32).reshape(4, 64)
    np.testing.assert_array_equal(L[50176:].view(np.float32), b)
    e4m3 = torch.from_numpy(corr.copy()).view(torch.float8_e4m3fn).float().numpy().astype(np.float64)
    chan = lambda byte: 32 * ((byte >> 3) >> 2) + 4 * ((byte >> 3) & 3) + (byte & 7 & 3) + 16 * ((byte & 7) >> 2)
    hi_full = np.zeros((64, 64, 3))
    lo_full = np.zeros((64, 64, 3))
    for m in range(4):
        for s in range(6):
            t, u = s >> 1, s & 1
            for j in range(8):
                cin = 32 * u + 4 * (lane >> 4) + (j & 3) + 16 * (j >> 2)
                hi_full[16 * m + (lane & 15), cin, t] = main[m, s, :, j]
        for t in range(3):
            for ln in range(64):
                r, g = ln & 15, ln >> 4
                for jj in range(16):
                    byte = 16 * g + jj
                    kb = byte >> 5
                    s_lo = float(2.0 ** (int((scales[m, r + 16 * kb] >> (8 * t)) & 0xFF) - 127))
                    s_hi = float(2.0 ** (int((scales[m, r + 16 * (2 + kb)] >> (8 * t)) & 0xFF) - 127))
                    co, ci = 16 * m + r, chan(byte)
                    lo_full[co, ci, t] = e4m3[m, t, ln, jj] * s_lo
                    # the e4m3 copy of hi is within 2^-4 relative of the f16 hi
                    assert abs(e4m3[m, t, ln, 16 + jj] * s_hi - hi_full[co, ci, t]) <= 2.0 ** -4 * abs(hi_full[co, ci, t]) + 1e-12
    np.testing.assert_array_equal(hi_full.astype(np.float16), w.astype(np.float16))
    err = np.abs(hi_full + lo_full - w64)
    assert err.max() <= 2.0 ** -14 * np.abs(w64).max(), err.max()


def test_pack_layout_f16mix_head_record():
    """RDN_F16MIX blob: the 29 f16 + e4m3 big layers, then the left head (left_net.19) as a ping-pong head
    record in an f16 + e4m3-sized slot: f16 fragments with cout 0 in rows 0 and 32 (M-tiles 0 and 2)
    and its weights' f16 rounding residue in rows 1 and 33, the bias at H8_BIAS_OFF (fused16.hpp head,
    read by fused_inplace.hip rrcdnet_hybrid); then the right head (right_net.18) as an f16 + e4m3 layer
    record with the head at couts 0 and 32 (inplace.hpp head_h8_mfma)."""
    from raman_mi355x import engine
    sd = golden_state_dict("RRCDNet", "trained")
    blob = engine.pack("RRCDNet", sd, "f16mix", "cpu").numpy()
    assert blob.size == engine.packed_size("RRCDNet", "f16mix") == SMALL + 31 * 50432
    # the big layers are the f16f8 blob's
    ref = engine.pack("RRCDNet", sd, "f16f8", "cpu").numpy()
    np.testing.assert_array_equal(blob[SMALL:SMALL + 29 * 50432], ref[SMALL:])
    lane = np.arange(64)
    # the right head's record: f16 fragments of cout 0 in rows 0 and 32, zeros elsewhere, bias copied
    wr, br = _fold(sd, "right_net.18", None)
    R2 = blob[SMALL + 30 * 50432:]
    main = R2[:24576].view(np.float16).reshape(4, 6, 64, 8)
    for s_ in range(6):
        t, u = s_ >> 1, s_ & 1
        for j in range(8):
            cin = 32 * u + 4 * (lane >> 4) + (j & 3) + 16 * (j >> 2)
            for m in (0, 2):
                got = main[m, s_, :, j]
                np.testing.assert_array_equal(got[(lane & 15) == 0], wr[0, cin, t][(lane & 15) == 0].astype(np.float16))
                assert np.all(got[(lane & 15) != 0] == 0)
        assert np.all(main[1, s_] == 0) and np.all(main[3, s_] == 0)
    rbias = R2[50176:].view(np.float32)
    assert rbias[0] == np.float32(br[0]) and rbias[32] == np.float32(br[0]) and np.count_nonzero(rbias) <= 2
    w, b = _fold(sd, "left_net.19", None)            # [1, 64, 3]
    R = blob[SMALL + 29 * 50432:SMALL + 30 * 50432]
    frag = R[:24576].view(np.float16).reshape(4, 6, 64, 8)
    lane = np.arange(64)
    for s_ in range(6):
        t, u = s_ >> 1, s_ & 1
        for j in range(8):
            cin = 32 * u + 4 * (lane >> 4) + (j & 3) + 16 * (j >> 2)
            exp = w[0, cin, t]
            for m in (0, 2):
                rows = lane & 15
                got = frag[m, s_, :, j]
                np.testing.assert_array_equal(got[rows == 0], exp[rows == 0].astype(np.float16))
                res = (exp.astype(np.float64) - exp.astype(np.float16).astype(np.float64))
                np.testing.assert_array_equal(got[rows == 1], res[rows == 1].astype(np.float16))
                assert np.all(got[rows >= 2] == 0)
            assert np.all(frag[1, s_] == 0) and np.all(frag[3, s_] == 0)
    bias = R[50176:].view(np.float32)
    assert bias[0] == b[0] and bias[32] == b[0] and np.count_nonzero(bias) <= 2


@pytest.mark.parametrize("arch,nbig", [("ADSDN", 32), ("APIDN", 30)])
def test_pack_layout_cbam_f16_pingpong_section(arch, nbig):
    """RDN_F16 on the CBAM networks: the in-place single-plane records (per-segment kernels) are followed
    by a ping-pong section for the team kernel (cbam.hip team16_forward): one fused16 record per big layer
    (f16 fragments in h16_channel K order, bias at 24576) and the head (conv_out) as the last record."""
    from raman_mi355x import engine
    sd = golden_state_dict(arch, "trained")
    blob = engine.pack(arch, sd, "f16", "cpu").numpy()
    off = SMALL + nbig * 49408
    assert blob.size == engine.packed_size(arch, "f16") == off + (nbig + 1) * 24832
    lane = np.arange(64)
    # big layer 2 (the first ResidualBlock's / block's first conv, BN folded)
    conv, bn = ("res_blocks.0.conv1", "res_blocks.0.bn1") if arch == "ADSDN" else ("res_blocks.1.0", "res_blocks.1.1")
    k = 2
    w, b = _fold(sd, conv, bn)
    R = blob[off + k * 24832:off + (k + 1) * 24832]
    frag = R[:24576].view(np.float16).reshape(4, 6, 64, 8)
    for m in range(4):
        for s_ in range(6):
            t, u = s_ >> 1, s_ & 1
            for j in range(8):
                cin = 32 * u + 4 * (lane >> 4) + (j & 3) + 16 * (j >> 2)
                np.testing.assert_array_equal(frag[m, s_, :, j], w[16 * m + (lane & 15), cin, t].astype(np.float16))
    np.testing.assert_array_equal(R[24576:].view(np.float32), b.astype(np.float32))
    # the head record: cout 0 in rows 0 and 32, bias copies at 0 and 32
    wh, bh = _fold(sd, "conv_out" if arch == "ADSDN" else "conv_out.0", None)
    H = blob[off + nbig * 24832:]
    hf = H[:24576].view(np.float16).reshape(4, 6, 64, 8)
    np.testing.assert_array_equal(hf[0, 0, 0, :4], wh[0, [0, 1, 2, 3], 0].astype(np.float16))
    hb = H[24576:].view(np.float32)
    assert hb[0] == bh[0] and hb[32] == bh[0]


def _fold_f64(sd, conv):
    return sd[conv + ".weight"].double().numpy()


@pytest.mark.slow
@pytest.mark.parametrize("arch,dtype", [("RRCDNet", "f16f8"), ("RRCDNet", "f16mix"), ("ADSDN", "f16"), ("ADSDN", "fp32"), ("DSDN", "bf16x3"),
                                        ("APIDN", "bf16-unsafe"), ("DenoiseCNN", "f16f8")])
def test_host_sanitizer_pack(arch, dtype, tmp_path):
    """pack.cpp + abi.cpp built with ASan + UBSan (csrc/Makefile `asan`): packing a
    trained reference state_dict into an exactly-sized buffer and every argument-error path run clean,
    and the sanitized packer writes the same bytes as the library's rdn_pack."""
    import subprocess
    import sys
    from raman_mi355x import engine
    csrc = os.path.join(ROOT, "data-simulation-and-noise-reduction-of-distributed-fiber-raman-intensity_amd", "csrc")
    subprocess.run(["make", "-C", csrc, "-j8", "asan", f"PYTHON={sys.executable}"], check=True, capture_output=True)
    sd = golden_state_dict(arch, "trained")
    with open(tmp_path / "t.bin", "wb") as fh:
        for k in engine.param_names(arch):
            t = sd[k].detach().float().contiguous().numpy()
            fh.write(np.int64(t.size).tobytes())
            fh.write(t.tobytes())
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(csrc, "build", "asan", "host_check"), str(engine._arch(arch)),
                        str(engine.resolve_dtype(arch, dtype)), str(tmp_path / "t.bin"), str(tmp_path / "blob.bin")],
                       capture_output=True, text=True, env=env)
    assert r.returncode == 0, f"rc {r.returncode}: {r.stdout} {r.stderr}"
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr
    blob = np.fromfile(tmp_path / "blob.bin", dtype=np.uint8)
    np.testing.assert_array_equal(blob, engine.pack(arch, sd, dtype, "cpu").numpy())


def test_correction_masks_recorded_in_blob():
    """RDN_F16F8 blobs record every layer as corrected, RDN_F16MIX (RRCDNet only) the compiled-in tail
    right_net.13-17 = big layers 10-14; the other networks refuse RDN_F16MIX."""
    from raman_mi355x import engine, _lib
    sd = golden_state_dict("RRCDNet", "trained")
    assert engine.correction_mask("RRCDNet", "f16f8", engine.pack("RRCDNet", sd, "f16f8", "cpu")) == (1 << 64) - 1
    assert engine.correction_mask("RRCDNet", "f16mix", engine.pack("RRCDNet", sd, "f16mix", "cpu")) == 0x1f << 10
    assert engine.default_correction_mask("RRCDNet") == 0x1f << 10
    for arch in ("DenoiseCNN", "DSDN", "PIDN", "ADSDN", "APIDN"):
        assert engine.default_correction_mask(arch) == 0
        with pytest.raises(_lib.EngineError, match="RRCDNet"):
            engine.pack(arch, golden_state_dict(arch, "synth"), "f16mix", "cpu")
