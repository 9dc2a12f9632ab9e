"""Thin tensor-level wrappers over the C ABI: weight packing, forward, simulator and metrics.

All compute runs in libraman_mi355x.so on the caller's current HIP stream; these functions only
check shapes/devices, allocate outputs through the PyTorch caching allocator and pass raw
pointers.  Nothing here has a CPU or PyTorch-op fallback.
"""
import ctypes
import os

import torch

from . import _lib

ARCHS = ("DenoiseCNN", "RRCDNet", "DSDN", "ADSDN", "PIDN", "APIDN")
ARCH_ID = {a: i for i, a in enumerate(ARCHS)}
CBAM_ARCHS = ("ADSDN", "APIDN")
CBAM_IDS = tuple(ARCH_ID[a] for a in CBAM_ARCHS)
# dtypes whose e4m3 correction planes bound the activations (|v| <= 1792): their forwards report a
# saturated tile through the workspace's status word (RangeError) and write NaN for it
RANGE_CODES = (3, 5)
# a fused network's 16-bit forward keeps a status word in its workspace (common.hpp STATUS_*): bit 0 an
# e4m3 activation saturated (RANGE_CODES only), bit 1 an input left [-4, 4] (the stems' input gate,
# models.INPUT_GATE: the 16-bit modes' domain; informational, rdn_forward_status does not fail on it)
STATUS_RANGE, STATUS_GATE, STATUS_TIMEOUT = 1, 2, 4
# Engine arithmetic modes (include/raman_mi355x.h rdn_dtype).  Every name here except
# "bf16-unsafe" meets its north-star tolerance on every golden fixture (fp32: 1e-5 max-relative;
# 16-bit modes: 2e-2 max-abs).  Single-rounding bf16 does NOT (0.24 on trained RRCDNet),
# so it is reachable only under that explicit name; plain "bf16" / torch.bfloat16 is refused with a
# pointer to the tolerance-meeting 16-bit modes instead of silently returning out-of-contract results.
DTYPE_ID = {"fp32": 0, "float32": 0, "bf16-unsafe": 1, "bf16_unsafe": 1, "bf16x3": 2, "f16f8": 3, "f16-plain": 4,
            "f16mix": 5}
DTYPE_NAME = {0: "fp32", 1: "bf16-unsafe", 2: "bf16x3", 3: "f16f8", 4: "f16-plain", 5: "f16mix"}
SAFE_16BIT = ("f16", "f16f8", "bf16x3")
F16, F16MIX = 4, 5
# every spelling of "f16" means one thing: the fastest arithmetic within the 2e-2 bar for the network
_F16_SPELLINGS = ("f16", "float16", "half")


def default_correction_mask(arch):
    """The layers RDN_F16MIX corrects for ``arch`` (0: plain f16 already meets the 2e-2 bar there)."""
    m = ctypes.c_uint64()
    _lib.check(_lib.lib().rdn_default_correction_mask(_arch(arch), ctypes.byref(m)), "rdn_default_correction_mask")
    return m.value


def correction_mask(arch, dtype, host_blob):
    """Correction mask recorded in a packed (host) blob."""
    m = ctypes.c_uint64()
    _lib.check(_lib.lib().rdn_get_correction_mask(_arch(arch), resolve_dtype(arch, dtype),
                                                  ctypes.c_void_p(host_blob.data_ptr()), host_blob.numel(),
                                                  ctypes.byref(m)), "rdn_get_correction_mask")
    return m.value


def check_blob(arch, dtype, host_blob):
    """Raise unless ``host_blob`` (a CPU uint8 tensor) was packed by rdn_pack for (arch, dtype)."""
    _lib.check(_lib.lib().rdn_check_blob(_arch(arch), resolve_dtype(arch, dtype), ctypes.c_void_p(host_blob.data_ptr()),
                                         host_blob.numel()), "rdn_check_blob")


def resolve_dtype(arch, dtype):
    """ABI dtype code (rdn_dtype) for a user dtype.  'f16' (also 'float16' and torch.float16) is the
    fastest arithmetic within the 2e-2 bar: plain f16 (RDN_F16) where that suffices, f16 with the
    compiled-in e4m3-corrected layers (RDN_F16MIX) where it does not (RRCDNet).  'f16-plain' forces
    RDN_F16 everywhere, 'f16mix' RDN_F16MIX.  An integer is taken as an ABI code unchanged."""
    if isinstance(dtype, int) and not isinstance(dtype, bool):
        if dtype not in DTYPE_NAME:
            raise ValueError(f"unknown engine dtype code {dtype}")
        return dtype
    if isinstance(dtype, torch.dtype):
        dtype = {torch.float32: "fp32", torch.bfloat16: "bf16", torch.float16: "f16"}.get(dtype, str(dtype))
    if dtype in _F16_SPELLINGS:
        return F16MIX if default_correction_mask(arch) else F16
    return _dtype(dtype)


def dtype_name(dtype, arch=None):
    """User-level name of a dtype: 'f16' for every f16 spelling (the network's fastest mode within
    2e-2), else the name of its ABI code ('f16-plain' = RDN_F16, 'f16mix' = RDN_F16MIX)."""
    if isinstance(dtype, torch.dtype) and dtype == torch.float16:
        return "f16"
    if isinstance(dtype, str) and dtype in _F16_SPELLINGS:
        return "f16"
    return DTYPE_NAME[resolve_dtype(arch, dtype) if arch is not None else _dtype(dtype)]


def _arch(arch):
    if isinstance(arch, int):
        return arch
    try:
        return ARCH_ID[arch]
    except KeyError:
        raise ValueError(f"unknown network {arch!r}; expected one of {ARCHS}") from None


def _dtype(dtype):
    """Code of an arch-independent dtype name ('f16' depends on the network: resolve_dtype)."""
    if isinstance(dtype, int) and dtype in DTYPE_NAME:
        return dtype
    if isinstance(dtype, torch.dtype):
        dtype = {torch.float32: "fp32", torch.bfloat16: "bf16", torch.float16: "f16"}.get(dtype, str(dtype))
    if dtype in _F16_SPELLINGS:
        raise ValueError("engine dtype 'f16' resolves per network: use resolve_dtype(arch, 'f16')")
    if dtype in ("bf16", "bfloat16"):
        raise ValueError("engine dtype 'bf16' (one bf16 rounding per operand) does not meet the 2e-2 bf16 "
                         "tolerance on trained weights (0.24 on trained RRCDNet); use 'f16', 'f16f8' or 'bf16x3' "
                         f"({', '.join(SAFE_16BIT)}: within 2e-2), or opt in explicitly with 'bf16-unsafe'")
    try:
        return DTYPE_ID[dtype]
    except (KeyError, TypeError):
        raise ValueError(f"unknown engine dtype {dtype!r}; expected one of 'fp32', 'f16', 'f16-plain', 'f16f8', "
                         "'bf16x3', 'bf16-unsafe'") from None


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def param_names(arch):
    """The state_dict keys the packer consumes, in order (folded BN stats included)."""
    L = _lib.lib()
    need = ctypes.c_size_t()
    _lib.check(L.rdn_param_names(_arch(arch), None, 0, ctypes.byref(need)), "rdn_param_names")
    buf = ctypes.create_string_buffer(need.value)
    _lib.check(L.rdn_param_names(_arch(arch), buf, need.value, ctypes.byref(need)), "rdn_param_names")
    return [s for s in buf.value.decode().split("\n") if s]


def packed_size(arch, dtype):
    n = ctypes.c_size_t()
    _lib.check(_lib.lib().rdn_packed_size(_arch(arch), resolve_dtype(arch, dtype), ctypes.byref(n)), "rdn_packed_size")
    return n.value


def pack(arch, state_dict, dtype, device):
    """Fold BN + lay out MFMA fragments on the host, then copy the blob to ``device``."""
    names = param_names(arch)
    missing = [k for k in names if k not in state_dict]
    if missing:
        raise KeyError(f"state_dict lacks {len(missing)} tensors the engine needs, e.g. {missing[:3]}")
    host = [state_dict[k].detach().to("cpu", torch.float32).contiguous() for k in names]
    ptrs = (ctypes.c_void_p * len(host))(*[t.data_ptr() for t in host])
    numels = (ctypes.c_int64 * len(host))(*[t.numel() for t in host])
    code = resolve_dtype(arch, dtype)
    size = packed_size(arch, code)
    blob = torch.empty(size, dtype=torch.uint8)
    _lib.check(_lib.lib().rdn_pack(_arch(arch), code, ptrs, numels, len(host),
                                   ctypes.c_void_p(blob.data_ptr()), size), "rdn_pack")
    return blob.to(device)


def _check_cuda_f32(t, name):
    if not (torch.is_tensor(t) and t.is_cuda):
        raise RuntimeError(f"raman_mi355x runs on the GPU only: {name} must be a CUDA (HIP) tensor")
    if t.dtype != torch.float32:
        raise TypeError(f"{name} must be float32, got {t.dtype}")


def _rows(t):
    """(N, L) or (N, 1, L) -> contiguous (N, L) (N = 0 included: no -1 in the shape)."""
    return t.reshape(t.shape[0], t.shape[-1] if t.dim() > 1 else 1).contiguous()


def _check_out(t, name, shape, device, dtype=torch.float32):
    """A caller-supplied output buffer the kernels write through a raw pointer: it must be exactly
    the size, type and device the launch assumes, and contiguous."""
    if not torch.is_tensor(t):
        raise TypeError(f"{name} must be a tensor")
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_cuda or t.device != torch.device(device):
        raise ValueError(f"{name} must live on {device}, got {t.device}")
    if tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name} must have shape {tuple(shape)}, got {tuple(t.shape)}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


def needs_workspace(arch, code):
    """A forward of (arch, code) takes a workspace: the CBAM team kernels (required) and the fused
    networks' 16-bit dtypes (their status word: range and input gate)."""
    return _arch(arch) in CBAM_IDS or code != 0


def has_status_word(arch, code):
    """Whether a workspace of (arch, code) starts with the fused networks' status word."""
    return _arch(arch) not in CBAM_IDS and code != 0


class Workspace:
    """Device scratch of a forward for (arch, dtype, L) on one device and stream, reused across
    forwards: the CBAM team kernels' slots and hand-off error word, and the fused networks' 16-bit status
    word (the range bit of RDN_F16F8 / RDN_F16MIX, the input-gate bit).  The status words are sticky: ``check()`` waits for the stream once and raises
    EngineError if any forward since the last check timed out, RangeError if one saturated the e4m3
    planes (rdn_forward_status), so a batched driver checks once at the end instead of host-syncing
    every batch."""

    def __init__(self, arch, dtype, n, L, device, stream=None):
        self.arch, self.code, self.L = _arch(arch), resolve_dtype(arch, dtype), int(L)
        self.device = torch.device(device)
        self.stream = stream if stream is not None else torch.cuda.current_stream(self.device)
        self.n = int(n)
        sz = ctypes.c_size_t()
        lib_ = _lib.lib()
        sp = ctypes.c_void_p(self.stream.cuda_stream)
        _lib.check(lib_.rdn_workspace_size(self.arch, self.code, self.n, self.L, ctypes.byref(sz), sp),
                   "rdn_workspace_size")
        self.bytes = sz.value
        self._fit_memo = {}
        self.buf = torch.empty(self.bytes, dtype=torch.uint8, device=self.device) if self.bytes else None
        _lib.check(lib_.rdn_workspace_init(self.arch, self.code, self.n, self.L, self.ptr, self.bytes, sp),
                   "rdn_workspace_init")

    @property
    def ptr(self):
        return ctypes.c_void_p(self.buf.data_ptr() if self.buf is not None else 0)

    def fits(self, arch, code, n, L, device):
        """Made for this network, dtype, length and device, large enough for n spectra, and bound to the
        stream the forward launches on (torch's current stream): check() waits for self.stream only, and
        rdn_workspace_init's reset is ordered on it."""
        if not ((self.arch, self.code, self.L, self.device) == (_arch(arch), code, int(L), torch.device(device))
                and torch.cuda.current_stream(self.device).cuda_stream == self.stream.cuda_stream):
            return False
        if self.arch in CBAM_IDS:
            # the CBAM layout (team or segment geometry) is the one the device and environment give now:
            # the size it had when made, and room for n spectra (memoised per batch size and the
            # RDN_CBAM_SEGMENTS switch: the batch-1 loop asks once per call)
            key = (int(n), os.environ.get("RDN_CBAM_SEGMENTS"))
            ok = self._fit_memo.get(key)
            if ok is None:
                ok = self.bytes_for(self.n) == self.bytes and self.bytes_for(n) <= self.bytes
                self._fit_memo[key] = ok
            return ok
        return self.n >= n or self.bytes_for(n) <= self.bytes

    def bytes_for(self, n):
        sz = ctypes.c_size_t()
        _lib.check(_lib.lib().rdn_workspace_size(self.arch, self.code, int(n), self.L, ctypes.byref(sz),
                                                 ctypes.c_void_p(self.stream.cuda_stream)), "rdn_workspace_size")
        return sz.value

    def status_word(self):
        """The status word of a fused network's 16-bit workspace (its first 4 bytes, rdn_forward_status's
        word: STATUS_RANGE | STATUS_GATE bits) as a device int32 tensor, without waiting.  A caller that
        reads it this way (models._EngineNet.forward: the call's one 4-byte host read) clears it with
        clear_status_word() (rdn_forward_status reads and clears)."""
        if not has_status_word(self.arch, self.code):
            raise ValueError("status_word: only the fused networks' 16-bit workspaces")
        return self.buf[:4].view(torch.int32)

    def clear_status_word(self):
        self.buf[:4].zero_()                       # on the current stream = the forwards' (fits())

    def read_status(self):
        """Wait for the workspace's stream and return its status word (0 for a CBAM workspace) without
        clearing it (check() clears it)."""
        if not has_status_word(self.arch, self.code):
            return 0
        with torch.cuda.stream(self.stream):
            return int(self.status_word().item())

    def check(self):
        """Wait for the stream, read and clear the status words of every forward since the last check, and
        return their flags (STATUS_RANGE | STATUS_GATE | STATUS_TIMEOUT, rdn_forward_status_ex).  Raises
        EngineError if a CBAM hand-off timed out, RangeError if a tile saturated the e4m3 planes; the
        input gate (an input beyond the 16-bit modes' domain) is only reported in the flags."""
        flags = ctypes.c_uint(0)
        _lib.check(_lib.lib().rdn_forward_status_ex(self.arch, self.code, self.n, self.L, self.ptr, self.bytes,
                                                    ctypes.c_void_p(self.stream.cuda_stream), ctypes.byref(flags)),
                   "rdn_forward_status_ex")
        return int(flags.value)


def _forward_args(arch, dtype, x, out, check, workspace, _ws_checked):
    """Shared argument checks of forward / forward_metrics: (n, L, arch id, code, y, workspace)."""
    _check_cuda_f32(x, "input")
    if x.dim() == 3 and x.shape[1] != 1:
        raise ValueError(f"expected (N, 1, L) input, got {tuple(x.shape)}")
    if x.dim() not in (2, 3):
        raise ValueError(f"expected (N, 1, L) input, got {tuple(x.shape)}")
    n, L = x.shape[0], x.shape[-1]
    a, code = _arch(arch), resolve_dtype(arch, dtype)
    y = torch.empty_like(x) if out is None else out
    if out is not None:
        _check_out(y, "out", x.shape, x.device)
    if y.data_ptr() < x.data_ptr() + x.numel() * 4 and x.data_ptr() < y.data_ptr() + y.numel() * 4:
        raise ValueError("out must not overlap the input (tiles re-read input halos while outputs are written)")
    ws = workspace
    if ws is None and (a in CBAM_IDS or (check and code in RANGE_CODES)):
        ws = Workspace(a, code, n, L, x.device)
    elif ws is not None and not _ws_checked and not ws.fits(a, code, n, L, x.device):
        raise ValueError("workspace was made for another network, dtype, length, device, stream or a smaller batch")
    return n, L, a, code, y, ws


def forward(arch, dtype, packed, x, out=None, check=True, workspace=None, _ws_checked=False):
    """y = Model(x) for x float32 (N, 1, L) (or (N, L)) on the GPU.

    ``dtype`` is an engine dtype name or ABI code (resolve_dtype).  The CBAM networks run one
    team-persistent kernel whose workgroups hand off statistics; RDN_F16F8 / RDN_F16MIX tiles whose
    activations leave the e4m3 planes' range write NaN.  With ``check`` (default) the call waits for
    the kernel and raises EngineError if a hand-off timed out, RangeError if a tile saturated
    (rdn_forward_status).  A batched caller passes one ``Workspace`` to every forward with
    ``check=False`` and calls ``workspace.check()`` once at the end (the status words are sticky);
    (``_ws_checked``: the caller has just verified ``workspace.fits`` for this input.)
    ``check=False`` without a workspace keeps the launch asynchronous and unchecked (benchmarks: the
    affected outputs are NaN).  On the CBAM networks (ADSDN / APIDN) a saturated tile's clamped CBAM
    statistics reach the other tiles of its spectrum through the team hand-off, so the whole spectrum
    is NaN, not just the tile: the team kernel's saturated tile publishes +inf maxima that taint its
    team (cbam.hip publish_stats / apply_cbam), and a segment-path launch (spectra longer than the
    co-resident teams hold) NaNs every spectrum of the chunk.  On the walk geometry (large 'f16' batches
    of RRCDNet) a saturated tile NaNs the rest of its spectrum, since its clamped values reach the next
    tiles through the carried rows.  The status word (RangeError from ``check`` or
    ``Workspace.check()``) remains the authoritative signal."""
    _check_cuda_f32(x, "input")
    x = x.contiguous()
    n, L, a, code, y, ws = _forward_args(arch, dtype, x, out, check, workspace, _ws_checked)
    L_ = _lib.lib()
    _lib.check(L_.rdn_forward(a, code, ctypes.c_void_p(packed.data_ptr()), ctypes.c_void_p(x.data_ptr()),
                              ctypes.c_void_p(y.data_ptr()), n, L,
                              ws.ptr if ws is not None else ctypes.c_void_p(0), ws.bytes if ws is not None else 0,
                              _stream(x.device)), "rdn_forward")
    if check and ws is not None:
        ws.check()
    return y


def forward_metrics(arch, dtype, packed, x, clean, out=None, sums=None, per_spectrum=False, acc=None, check=True,
                    workspace=None):
    """forward() and metrics() in one call (rdn_forward_metrics): y = Model(x), then each spectrum's MSE,
    SSIM, Smoothness and Peak2Peak against ``clean`` (float32 or float64, (N, L) or (N, 1, L)), added to
    ``sums`` / ``acc`` as metrics() does.  On the walk geometry (large batches of the f16 modes) the
    forward kernel computes the metrics itself after each spectrum's walk, so y is not read again by a
    second pass.  Returns (y, per (n, 4) or None, sums, fused)."""
    _check_cuda_f32(x, "input")
    x = x.contiguous()
    if not (torch.is_tensor(clean) and clean.is_cuda):
        raise RuntimeError("raman_mi355x runs on the GPU only: clean must be a CUDA (HIP) tensor")
    if clean.dtype not in (torch.float32, torch.float64):
        raise TypeError(f"clean must be float32 or float64, got {clean.dtype}")
    n, L, a, code, y, ws = _forward_args(arch, dtype, x, out, check, workspace, False)
    clean = _rows(clean)
    if tuple(clean.shape) != (n, L):
        raise ValueError(f"clean must be ({n}, {L}), got {tuple(clean.shape)}")
    if clean.device != x.device:
        raise ValueError(f"input on {x.device} but clean on {clean.device}")
    per = torch.empty((n, 4), dtype=torch.float64, device=x.device) if per_spectrum else None
    if sums is None:
        sums = torch.zeros(5, dtype=torch.float64, device=x.device)
    else:
        _check_out(sums, "sums", (5,), x.device, torch.float64)
    if acc is not None:
        _check_out(acc, "acc", (_lib.ACC_WORDS,), x.device, torch.int64)
    fused = ctypes.c_int(0)
    _lib.check(_lib.lib().rdn_forward_metrics(
        a, code, ctypes.c_void_p(packed.data_ptr()), ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(y.data_ptr()), n, L,
        ctypes.c_void_p(clean.data_ptr()), int(clean.dtype == torch.float64),
        ctypes.c_void_p(per.data_ptr() if per is not None else 0), ctypes.c_void_p(sums.data_ptr()),
        ctypes.c_void_p(acc.data_ptr() if acc is not None else 0),
        ws.ptr if ws is not None else ctypes.c_void_p(0), ws.bytes if ws is not None else 0, _stream(x.device),
        ctypes.byref(fused)), "rdn_forward_metrics")
    if check and ws is not None:
        ws.check()
    return y, per, sums, bool(fused.value)


def generate(n, seed, first_index=0, signal_length=10000, snr_range=(20.0, 37.0), extreme_noise_prob=0.05,
             max_repeat=40, device="cuda", out=None):
    """Device simulator (数据集产生.py:5-64 contract): returns clean, noisy (n, L), snr, noise_std (n,)."""
    device = torch.device(device)
    if device.type != "cuda":
        raise RuntimeError("raman_mi355x runs on the GPU only: the simulator needs a CUDA device")
    L = int(signal_length)
    if device.index is None:
        device = torch.device("cuda", torch.cuda.current_device())
    if out is None:
        clean = torch.empty((n, L), dtype=torch.float32, device=device)
        noisy = torch.empty((n, L), dtype=torch.float32, device=device)
    else:
        clean, noisy = out
        _check_out(clean, "out[0] (clean)", (n, L), device)
        _check_out(noisy, "out[1] (noisy)", (n, L), device)
        if clean.data_ptr() == noisy.data_ptr():
            raise ValueError("clean and noisy output buffers must be distinct")
    snr = torch.empty(n, dtype=torch.float32, device=device)
    nstd = torch.empty(n, dtype=torch.float32, device=device)
    prm = _lib.GenParams(L, float(snr_range[0]), float(snr_range[1]), float(extreme_noise_prob), int(max_repeat))
    _lib.check(_lib.lib().rdn_generate(int(seed), int(first_index), int(n), ctypes.byref(prm),
                                       ctypes.c_void_p(clean.data_ptr()), ctypes.c_void_p(noisy.data_ptr()),
                                       ctypes.c_void_p(snr.data_ptr()), ctypes.c_void_p(nstd.data_ptr()),
                                       _stream(device)), "rdn_generate")
    return clean, noisy, snr, nstd


def metrics(y, clean, sums=None, per_spectrum=True, acc=None):
    """Per-spectrum [MSE, SSIM, Smoothness, Peak2Peak] (fp64, (n, 4)) and accumulated fp64 sums [5].

    ``clean`` may be float32 (the device simulator) or float64 (a test.npz as evaulate.py:61-62 loads
    it; the metrics then see the same float64 clean values as evaulate.py:34-35).  ``acc``: an
    exact accumulator (new_acc) that this batch is added to (rdn_metrics_ex)."""
    _check_cuda_f32(y, "denoised")
    if not (torch.is_tensor(clean) and clean.is_cuda):
        raise RuntimeError("raman_mi355x runs on the GPU only: clean must be a CUDA (HIP) tensor")
    if clean.dtype not in (torch.float32, torch.float64):
        raise TypeError(f"clean must be float32 or float64, got {clean.dtype}")
    y = _rows(y)
    clean = _rows(clean)
    if y.shape != clean.shape:
        raise ValueError(f"shape mismatch {tuple(y.shape)} vs {tuple(clean.shape)}")
    n, L = y.shape
    if clean.device != y.device:
        raise ValueError(f"denoised on {y.device} but clean on {clean.device}")
    per = torch.empty((n, 4), dtype=torch.float64, device=y.device) if per_spectrum else None
    if sums is None:
        sums = torch.zeros(5, dtype=torch.float64, device=y.device)
    else:
        _check_out(sums, "sums", (5,), y.device, torch.float64)   # fp64 atomics into sums[0..4]
    if acc is not None:
        _check_out(acc, "acc", (_lib.ACC_WORDS,), y.device, torch.int64)
    _lib.check(_lib.lib().rdn_metrics_ex(ctypes.c_void_p(y.data_ptr()), ctypes.c_void_p(clean.data_ptr()),
                                         int(clean.dtype == torch.float64), n, L,
                                         ctypes.c_void_p(per.data_ptr() if per is not None else 0),
                                         ctypes.c_void_p(sums.data_ptr()),
                                         ctypes.c_void_p(acc.data_ptr() if acc is not None else 0),
                                         _stream(y.device)), "rdn_metrics_ex")
    return per, sums


def new_acc(device):
    """A zeroed exact metric accumulator (RDN_ACC_WORDS int64) on ``device``."""
    return torch.zeros(_lib.ACC_WORDS, dtype=torch.int64, device=device)


def acc_value(acc):
    """{ΣMSE, ΣSSIM, ΣSmoothness, ΣPeak2Peak, count} (float64 [5], CPU) of an exact accumulator: each
    sum is the exact total rounded once (rdn_acc_value)."""
    h = acc.detach().to("cpu", torch.int64).contiguous()
    if h.numel() != _lib.ACC_WORDS:
        raise ValueError(f"accumulator must have {_lib.ACC_WORDS} words")
    out = torch.empty(5, dtype=torch.float64)
    _lib.check(_lib.lib().rdn_acc_value(ctypes.cast(h.data_ptr(), ctypes.POINTER(ctypes.c_int64)),
                                        ctypes.cast(out.data_ptr(), ctypes.POINTER(ctypes.c_double))), "rdn_acc_value")
    return out
