"""fp32 PyTorch-CPU restatement of the six reference networks (TEST INFRASTRUCTURE — see oracle/__init__).

Each ``forward_<arch>(sd, x)`` consumes a reference-format ``state_dict`` (same keys as
``torch.save(model.state_dict())`` in */train.py) and a float32 ``(N, 1, L)`` tensor, and follows the
reference op order exactly (eval-mode BatchNorm, eps 1e-5).  No module objects are built, so this
file doubles as the specification of which key feeds which op.
"""
import torch
import torch.nn.functional as F

BN_EPS = 1e-5


def _conv(x, sd, key, dilation=1, padding=None):
    w = sd[key + ".weight"]
    b = sd.get(key + ".bias")
    if padding is None:
        padding = dilation * (w.shape[-1] // 2)
    return F.conv1d(x, w, b, padding=padding, dilation=dilation)


def _bn(x, sd, key):
    return F.batch_norm(x, sd[key + ".running_mean"], sd[key + ".running_var"],
                        sd[key + ".weight"], sd[key + ".bias"], False, 0.0, BN_EPS)


def _cbam(x, sd, key, ca="channel_attention", sa="spatial_attention"):
    """CBAM as in ADSDN/train.py:72-116 (ca/sa names) and APIDN/train.py:72-116 (``ca``/``sa``)."""
    avg = x.mean(dim=2)
    mx = x.amax(dim=2)

    def fc(v):
        h = F.linear(v, sd[f"{key}.{ca}.fc.0.weight"], sd.get(f"{key}.{ca}.fc.0.bias"))
        h = F.relu(h)
        return F.linear(h, sd[f"{key}.{ca}.fc.2.weight"], sd.get(f"{key}.{ca}.fc.2.bias"))

    x = x * torch.sigmoid(fc(avg) + fc(mx)).unsqueeze(-1)
    cat = torch.cat([x.mean(dim=1, keepdim=True), x.amax(dim=1, keepdim=True)], dim=1)
    s = _conv(cat, sd, f"{key}.{sa}.conv", padding=3)
    return x * torch.sigmoid(s)


def forward_denoisecnn(sd, x):
    """1DCNN/train.py:71-82: conv(1→64)+ReLU, 18×[conv(64→64)+ReLU], conv(64→1)."""
    h = F.relu(_conv(x, sd, "layers.0"))
    for i in range(2, 20):
        h = F.relu(_conv(h, sd, f"layers.{i}.0"))
    return _conv(h, sd, "layers.20")


def forward_rrcdnet(sd, x):
    """RRCDNet/train.py:77-98: right (BN, d=1) and left (dilated) branches, x − (r + l)/2."""
    r = F.relu(_bn(_conv(x, sd, "right_net.0"), sd, "right_net.1"))
    for i in range(3, 18):
        r = F.relu(_bn(_conv(r, sd, f"right_net.{i}.0"), sd, f"right_net.{i}.1"))
    r = _conv(r, sd, "right_net.18")

    h = F.relu(_bn(_conv(x, sd, "left_net.0"), sd, "left_net.1"))
    for i in range(3, 10):
        h = F.relu(_conv(h, sd, f"left_net.{i}.0", dilation=2))
    h = F.relu(_bn(_conv(h, sd, "left_net.10"), sd, "left_net.11"))
    for i in range(13, 19):
        h = F.relu(_conv(h, sd, f"left_net.{i}.0", dilation=2))
    left = _conv(h, sd, "left_net.19")
    return x - (r + left) / 2


def _n_blocks(sd, prefix="res_blocks"):
    idx = {int(k.split(".")[1]) for k in sd if k.startswith(prefix + ".")}
    return max(idx) + 1 if idx else 0


def forward_dsdn(sd, x):
    """DSDN/train.py:120-126 (ReLU applied twice after the stem: :80 and :121)."""
    h = F.relu(F.relu(_conv(x, sd, "down_sampling.conv")))
    h = F.relu(_conv(h, sd, "conv1"))
    h = F.relu(_conv(h, sd, "conv2"))
    for i in range(_n_blocks(sd)):
        k = f"res_blocks.{i}"
        o = F.relu(_bn(_conv(h, sd, k + ".conv1"), sd, k + ".bn1"))
        o = _bn(_conv(o, sd, k + ".conv2"), sd, k + ".bn2")
        h = F.relu(o + h)
    return _conv(h, sd, "conv_out")


def forward_adsdn(sd, x):
    """ADSDN/train.py:120-167: DSDN plus CBAM after the stem, after conv2 and inside each block."""
    h = _cbam(F.relu(_conv(x, sd, "down_sampling.conv")), sd, "down_sampling.cbam")
    h = F.relu(_conv(h, sd, "conv1"))
    h = F.relu(_conv(h, sd, "conv2"))
    h = _cbam(h, sd, "cbam")
    for i in range(_n_blocks(sd)):
        k = f"res_blocks.{i}"
        o = F.relu(_bn(_conv(h, sd, k + ".conv1"), sd, k + ".bn1"))
        o = _bn(_conv(o, sd, k + ".conv2"), sd, k + ".bn2")
        o = _cbam(o, sd, k + ".cbam")
        h = F.relu(o + h)
    return _conv(h, sd, "conv_out")


def forward_pidn(sd, x):
    """PIDN/train.py:101-106: no per-block residual, one global skip, Sigmoid head."""
    ident = F.relu(_conv(x, sd, "down_sampling.0"))
    h = ident
    for i in range(_n_blocks(sd)):
        k = f"res_blocks.{i}"
        h = F.relu(_bn(_conv(h, sd, k + ".0"), sd, k + ".1"))
        h = _bn(_conv(h, sd, k + ".3"), sd, k + ".4")
    return torch.sigmoid(_conv(h + ident, sd, "conv_out.0"))


def forward_apidn(sd, x):
    """APIDN/train.py:150-159: x += CBAM(block(x)) per block (bias-free CBAM), σ(conv_out(x + h))."""
    ident = F.relu(_conv(x, sd, "down_sampling.0"))
    h = ident
    for i in range(_n_blocks(sd)):
        k = f"res_blocks.{i}"
        o = F.relu(_bn(_conv(h, sd, k + ".0"), sd, k + ".1"))
        o = _bn(_conv(o, sd, k + ".3"), sd, k + ".4")
        h = h + _cbam(o, sd, k + ".5", ca="ca", sa="sa")
    return torch.sigmoid(_conv(h + ident, sd, "conv_out.0"))


FORWARD = {
    "DenoiseCNN": forward_denoisecnn,
    "RRCDNet": forward_rrcdnet,
    "DSDN": forward_dsdn,
    "ADSDN": forward_adsdn,
    "PIDN": forward_pidn,
    "APIDN": forward_apidn,
}

ARCHS = tuple(FORWARD)


@torch.no_grad()
def forward(arch, sd, x):
    """Run the CPU oracle.  ``sd`` values are cast to float32 CPU tensors; ``x`` is (N,1,L) float32."""
    sd = {k: (v.detach().to("cpu", torch.float32) if torch.is_tensor(v) and v.is_floating_point()
              else v) for k, v in sd.items()}
    x = torch.as_tensor(x, dtype=torch.float32).cpu()
    return FORWARD[arch](sd, x)
