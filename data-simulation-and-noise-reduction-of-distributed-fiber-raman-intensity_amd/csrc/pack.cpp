// Load-time weight preparation (host): BatchNorm folding + MFMA fragment layout.
//
// Replaces the reference's ``model.load_state_dict(torch.load(path))`` (*/evaulate.py:66): the
// state_dict tensors are consumed in the order of net_spec(), eval-mode BatchNorm1d
// (y = (x - mean) / sqrt(var + 1e-5) * gamma + beta) is folded into the preceding Conv1d in fp64,
// and each 64->64 layer is written as the A-operand fragments its kernel loads (common.hpp).
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "common.hpp"
#include "netspec.hpp"

namespace rdn {

static constexpr double BN_EPS = 1e-5;
uint64_t f16mix_default_mask(int arch);
void set_corr_mask(void* blob, uint64_t mask);


std::vector<Op> net_spec(int arch) {
  std::vector<Op> s;
  auto stem = [&](const std::string& c, const std::string& bn, int slot) { s.push_back({OpKind::STEM, c, bn, slot}); };
  auto big = [&](const std::string& c, const std::string& bn) { s.push_back({OpKind::BIG, c, bn, -1}); };
  auto head = [&](const std::string& c, int slot) { s.push_back({OpKind::HEAD, c, "", slot}); };
  auto cbam = [&](const std::string& p, int slot, bool bias, const char* ca, const char* sa) {
    Op o{OpKind::CBAM, p, "", slot};
    o.bias = bias;
    o.ca = ca;
    o.sa = sa;
    s.push_back(o);
  };
  switch (arch) {
    case DENOISECNN:                                   // 1DCNN/train.py:74-78
      stem("layers.0", "", 0);
      for (int i = 2; i < 20; ++i) big("layers." + std::to_string(i) + ".0", "");
      head("layers.20", 1);
      break;
    case RRCDNET:                                      // RRCDNet/train.py:77-90
      stem("right_net.0", "right_net.1", 0);
      for (int i = 3; i < 18; ++i) big("right_net." + std::to_string(i) + ".0", "right_net." + std::to_string(i) + ".1");
      head("right_net.18", 2);
      stem("left_net.0", "left_net.1", 1);
      for (int i = 3; i < 10; ++i) big("left_net." + std::to_string(i) + ".0", "");
      big("left_net.10", "left_net.11");
      for (int i = 13; i < 19; ++i) big("left_net." + std::to_string(i) + ".0", "");
      head("left_net.19", 3);
      break;
    case DSDN:                                         // DSDN/train.py:104-118
      stem("down_sampling.conv", "", 0);
      big("conv1", "");
      big("conv2", "");
      for (int i = 0; i < 15; ++i) {
        const std::string p = "res_blocks." + std::to_string(i);
        big(p + ".conv1", p + ".bn1");
        big(p + ".conv2", p + ".bn2");
      }
      head("conv_out", 1);
      break;
    case ADSDN:                                        // ADSDN/train.py:151-158
      stem("down_sampling.conv", "", 0);
      cbam("down_sampling.cbam", 2, true, "channel_attention", "spatial_attention");
      big("conv1", "");
      big("conv2", "");
      cbam("cbam", 5, true, "channel_attention", "spatial_attention");
      for (int i = 0; i < 15; ++i) {
        const std::string p = "res_blocks." + std::to_string(i);
        big(p + ".conv1", p + ".bn1");
        big(p + ".conv2", p + ".bn2");
        cbam(p + ".cbam", 8 + 3 * i, true, "channel_attention", "spatial_attention");
      }
      head("conv_out", 1);
      break;
    case PIDN:                                         // PIDN/train.py:75-99
      stem("down_sampling.0", "", 0);
      for (int i = 0; i < 15; ++i) {
        const std::string p = "res_blocks." + std::to_string(i);
        big(p + ".0", p + ".1");
        big(p + ".3", p + ".4");
      }
      head("conv_out.0", 1);
      break;
    case APIDN:                                        // APIDN/train.py:122-148
      stem("down_sampling.0", "", 0);
      for (int i = 0; i < 15; ++i) {
        const std::string p = "res_blocks." + std::to_string(i);
        big(p + ".0", p + ".1");
        big(p + ".3", p + ".4");
        cbam(p + ".5", 2 + 3 * i, false, "ca", "sa");
      }
      head("conv_out.0", 1);
      break;
    default:
      break;
  }
  return s;
}

static void conv_names(const Op& o, std::vector<std::string>& out) {
  out.push_back(o.conv + ".weight");
  out.push_back(o.conv + ".bias");
  if (!o.bn.empty()) {
    for (const char* k : {".weight", ".bias", ".running_mean", ".running_var"}) out.push_back(o.bn + k);
  }
}

std::vector<std::string> param_names(const std::vector<Op>& spec) {
  std::vector<std::string> out;
  for (const Op& o : spec) {
    if (o.kind != OpKind::CBAM) {
      conv_names(o, out);
      continue;
    }
    const std::string ca = o.conv + "." + o.ca + ".fc.", sa = o.conv + "." + o.sa + ".conv.";
    out.push_back(ca + "0.weight");
    if (o.bias) out.push_back(ca + "0.bias");
    out.push_back(ca + "2.weight");
    if (o.bias) out.push_back(ca + "2.bias");
    out.push_back(sa + "weight");
    if (o.bias) out.push_back(sa + "bias");
  }
  return out;
}

// Weight layout of the big section: the fused bf16 kernels (fused16.hip: non-CBAM networks, bf16)
// keep the head as an MFMA layer (M-row 0) in 24832-byte layers, K order permuted (h16_channel); every other (network, dtype) runs on the
// in-place 256-byte-row engine: f32 fragments, or bf16 hi/lo fragments (bf16 uses only hi).
static bool has_cbam(const std::vector<Op>& spec) {
  for (const Op& o : spec)
    if (o.kind == OpKind::CBAM) return true;
  return false;
}
// layouts: F32, F16F8, BF16 / F16 (fused16.hip, head as an MFMA layer), BF16X3 (also the in-place
// plain-bf16 mode of the CBAM networks), F16X = F16 on the CBAM networks (split-bf16 geometry, f16 hi)
constexpr int F16X = 100;
int big_layout(const std::vector<Op>& spec, int dtype) {
  if (dtype == F32) return F32;
  if (dtype == F16F8 || dtype == F16MIX) return F16F8;
  if (dtype == BF16 && !has_cbam(spec)) return BF16;
  if (dtype == F16) return has_cbam(spec) ? F16X : F16;
  return BF16X3;
}
int big_layers(const std::vector<Op>& spec, int dtype) {
  const int lay = big_layout(spec, dtype);
  const bool head_big = lay == BF16 || lay == F16;
  int n = 0;
  for (const Op& o : spec) n += o.kind == OpKind::BIG || (o.kind == OpKind::HEAD && head_big);
  // RDN_F16MIX: the left head (left_net.19) also as a ping-pong head record after the big layers
  // (fused_inplace.hip rrcdnet_hybrid runs the left branch on the ping-pong engine), then the right
  // head (right_net.18) as an f16 + e4m3 layer record (its MFMA head, inplace.hpp head_h8_mfma)
  if (dtype == F16MIX) n += 2;
  return n;
}

// ---- packing ----------------------------------------------------------------------------------

struct Folded {            // conv weight [cout][cin][3] and bias [cout] after BN folding, fp64
  int cout, cin;
  std::vector<double> w, b;
  double W(int co, int ci, int t) const { return w[((size_t)co * cin + ci) * 3 + t]; }
};

struct Reader {
  const float* const* t;
  const int64_t* numel;
  int n, i = 0;
  std::string err;
  const float* take(const std::string& name, int64_t expect) {
    if (i >= n) { err = "too few tensors: missing " + name; return nullptr; }
    if (numel[i] != expect) {
      err = name + ": expected " + std::to_string(expect) + " elements, got " + std::to_string(numel[i]);
      return nullptr;
    }
    if (!t[i]) { err = name + ": null pointer"; return nullptr; }
    return t[i++];
  }
};

static bool fold(Reader& rd, const Op& o, int cin, int cout, Folded& f) {
  const float* w = rd.take(o.conv + ".weight", (int64_t)cout * cin * 3);
  const float* b = w ? rd.take(o.conv + ".bias", cout) : nullptr;
  if (!b) return false;
  f.cout = cout;
  f.cin = cin;
  f.w.assign(w, w + (size_t)cout * cin * 3);
  f.b.assign(b, b + cout);
  if (o.bn.empty()) return true;
  const float* g = rd.take(o.bn + ".weight", cout);
  const float* be = g ? rd.take(o.bn + ".bias", cout) : nullptr;
  const float* mu = be ? rd.take(o.bn + ".running_mean", cout) : nullptr;
  const float* var = mu ? rd.take(o.bn + ".running_var", cout) : nullptr;
  if (!var) return false;
  for (int c = 0; c < cout; ++c) {
    const double s = (double)g[c] / std::sqrt((double)var[c] + BN_EPS);
    for (int k = 0; k < cin * 3; ++k) f.w[(size_t)c * cin * 3 + k] *= s;
    f.b[c] = (f.b[c] - (double)mu[c]) * s + (double)be[c];
  }
  return true;
}

static uint16_t to_bf16(double v) {      // fp64 -> fp32 -> bf16, round to nearest even
  const float f = (float)v;
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7f800000u) == 0x7f800000u) return (uint16_t)((u >> 16) | ((u & 0xffff) ? 0x40 : 0));
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// fp64 -> fp32 -> f16, each step round to nearest even.  The f16 step is integer arithmetic on the
// fp32 bits: the host's _Float16 conversion differed by one ulp near ties between the -O3 library
// and the -O1 sanitizer build of the same source (tests/test_abi.py test_host_sanitizer_pack)
static uint16_t to_f16(double v) {
  const float f = (float)v;
  uint32_t x;
  std::memcpy(&x, &f, 4);
  const uint32_t sign = (x >> 16) & 0x8000u, mant = x & 0x7fffffu;
  const int exp = (int)((x >> 23) & 0xffu);
  if (exp == 0xff) return (uint16_t)(sign | 0x7c00u | (mant ? 0x200u : 0u));    // inf / nan
  const int e = exp - 127 + 15;                                                  // f16 biased exponent
  if (e >= 31) return (uint16_t)(sign | 0x7c00u);                                // overflow
  if (e <= 0) {                                                                  // f16 subnormal / zero
    if (e < -10) return (uint16_t)sign;
    const uint32_t m = mant | 0x800000u;
    const int sh = 14 - e;
    uint32_t h = m >> sh;
    const uint32_t rem = m & ((1u << sh) - 1u), half = 1u << (sh - 1);
    if (rem > half || (rem == half && (h & 1u))) ++h;
    return (uint16_t)(sign | h);
  }
  uint32_t h = ((uint32_t)e << 10) | (mant >> 13);
  const uint32_t rem = mant & 0x1fffu;
  if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) ++h;                         // a carry rounds into the exponent
  return (uint16_t)(sign | h);
}

static double from16(uint16_t u, bool f16) {
  if (f16) {
    _Float16 h;
    std::memcpy(&h, &u, 2);
    return (double)(float)h;
  }
  const uint32_t b = (uint32_t)u << 16;
  float f;
  std::memcpy(&f, &b, 4);
  return (double)f;
}

// fused16.hip layout; f16: the RDN_F16 instantiation (same fragments, f16 bits)
static void pack_big_bf16(const Folded& f, uint8_t* dst, bool f16 = false) {
  uint16_t* frag = (uint16_t*)dst;
  for (int m = 0; m < 4; ++m)
    for (int s = 0; s < 6; ++s)
      for (int lane = 0; lane < 64; ++lane)
        for (int j = 0; j < 8; ++j) {
          const int t = s >> 1, u = s & 1;
          // a head (cout = 1) sits in M-tiles 0 and 2 (rows 0 and 32: the M-tile of either
          // output-channel half, fused16.hpp head); row 1 / 33 carries the residue of row 0's rounding
          const int co = (f.cout == 1 && m == 2 ? 0 : 16 * m) + (lane & 15), ci = h16_channel(4 * u + (lane >> 4), j);
          double v = co < f.cout ? f.W(co, ci, t) : 0.0;
          if (f.cout == 1 && co == 1) {
            const double w = f.W(0, ci, t);
            v = w - from16(f16 ? to_f16(w) : to_bf16(w), f16);
          }
          frag[(((m * 6 + s) * 64) + lane) * 8 + j] = f16 ? to_f16(v) : to_bf16(v);
        }
  float* bias = (float*)(dst + BIG_FRAG_BYTES_BF16);
  for (int c = 0; c < C; ++c) bias[c] = c < f.cout ? (float)f.b[c] : 0.f;
  if (f.cout == 1) bias[32] = (float)f.b[0];        // the head's copy in M-tile 2
}

static void pack_big_f32(const Folded& f, uint8_t* dst) {
  float* frag = (float*)dst;
  for (int m = 0; m < 4; ++m)
    for (int tg = 0; tg < 12; ++tg)
      for (int lane = 0; lane < 64; ++lane)
        for (int i = 0; i < 4; ++i) {
          const int t = tg >> 2, g = tg & 3;
          const int co = 16 * m + (lane & 15), ci = 16 * g + 4 * (lane >> 4) + i;
          frag[((m * 12 + tg) * 64 + lane) * 4 + i] = (float)f.W(co, ci, t);
        }
  float* bias = frag + BIG_FRAG_FLOATS_F32;
  for (int c = 0; c < C; ++c) bias[c] = (float)f.b[c];
}

// split-bf16 layout; f16: the in-place single-plane f16 mode of the CBAM networks (RDN_F16 there),
// which reads only the hi fragments, here f16(W)
static void pack_big_x3(const Folded& f, uint8_t* dst, bool f16 = false) {
  uint16_t* frag = (uint16_t*)dst;
  for (int m = 0; m < 4; ++m)
    for (int s = 0; s < 6; ++s)
      for (int lane = 0; lane < 64; ++lane)
        for (int j = 0; j < 8; ++j) {
          const int t = s >> 1, u = s & 1;
          const int co = 16 * m + (lane & 15), ci = 32 * u + 8 * (lane >> 4) + j;
          const float w = (float)f.W(co, ci, t);
          if (f16) {
            frag[((((m * 6 + s) * 2 + 0) * 64) + lane) * 8 + j] = to_f16(w);
            frag[((((m * 6 + s) * 2 + 1) * 64) + lane) * 8 + j] = 0;
            continue;
          }
          const uint16_t hi = to_bf16(w);
          const uint32_t hib = (uint32_t)hi << 16;
          float hf;
          std::memcpy(&hf, &hib, 4);
          const uint16_t lo = to_bf16((double)w - (double)hf);
          frag[((((m * 6 + s) * 2 + 0) * 64) + lane) * 8 + j] = hi;
          frag[((((m * 6 + s) * 2 + 1) * 64) + lane) * 8 + j] = lo;
        }
  float* bias = (float*)(dst + BIG_FRAG_FLOATS_F32 * 4);
  for (int c = 0; c < C; ++c) bias[c] = (float)f.b[c];
}

// ---- f16 + e4m3 correction layout (common.hpp BIG_BYTES_H8, inplace.hpp Op<MODE_H8>) --------------

// OCP e4m3fn (bias 7, max 448, subnormal step 2^-9), round to nearest even, saturating
static uint8_t to_e4m3(double v) {
  const uint8_t sign = v < 0 ? 0x80 : 0;
  double a = std::fabs(v);
  if (!(a > 0)) return sign;
  if (a >= 448.0) return sign | 0x7e;
  int e;
  std::frexp(a, &e);                      // a = f * 2^e, f in [0.5, 1)
  e -= 1;                                 // a in [2^e, 2^(e+1))
  if (e < -6) e = -6;                     // subnormal range shares the step of [2^-6, 2^-5)
  const double step = std::ldexp(1.0, e - 3);
  double q = std::nearbyint(a / step);    // default rounding mode: nearest even
  double r = q * step;
  if (r >= 448.0) return sign | 0x7e;
  // re-encode r exactly
  if (r < std::ldexp(1.0, -6)) return sign | (uint8_t)std::lround(r / std::ldexp(1.0, -9));
  int er;
  const double fr = std::frexp(r, &er);   // r = fr * 2^er
  const int E = er - 1 + 7;
  const int M = (int)std::lround((fr * 2.0 - 1.0) * 8.0);
  return sign | (uint8_t)((E << 3) | M);
}

// E8M0 block scale so that the block's largest magnitude lands in (224, 448]
static int e8m0_for(double amax) {
  if (!(amax > 0)) return 127;
  int e = (int)std::ceil(std::log2(amax / 448.0));
  while (std::ldexp(amax, -e) > 448.0) ++e;
  while (e > -127 && std::ldexp(amax, -(e - 1)) <= 448.0) --e;
  return e + 127 < 0 ? 0 : (e + 127 > 254 ? 254 : e + 127);
}

static void pack_big_h8(const Folded& f, uint8_t* dst) {
  uint16_t* main = (uint16_t*)dst;
  // hi / lo split of every weight: hi = f16(fp32(W)), lo = W - hi (fp64)
  std::vector<double> hi((size_t)C * C * 3), lo((size_t)C * C * 3);
  for (int co = 0; co < C; ++co)
    for (int ci = 0; ci < C; ++ci)
      for (int t = 0; t < 3; ++t) {
        const double w = co < f.cout ? f.W(co, ci, t) : 0.0;
        const double h = from16(to_f16(w), true);
        hi[((size_t)co * C + ci) * 3 + t] = h;
        lo[((size_t)co * C + ci) * 3 + t] = w - h;
      }
  auto H = [&](int co, int ci, int t) { return hi[((size_t)co * C + ci) * 3 + t]; };
  auto Lo = [&](int co, int ci, int t) { return lo[((size_t)co * C + ci) * 3 + t]; };
  for (int m = 0; m < 4; ++m)
    for (int s = 0; s < 6; ++s)
      for (int lane = 0; lane < 64; ++lane)
        for (int j = 0; j < 8; ++j) {
          const int t = s >> 1, u = s & 1;
          const int co = 16 * m + (lane & 15), ci = h16_channel(4 * u + (lane >> 4), j);
          main[(((m * 6 + s) * 64) + lane) * 8 + j] = to_f16(H(co, ci, t));     // exact: H is an f16 value
        }
  // e4m3 activation byte b of a plane holds channel h16_channel(b >> 3, b & 7); blocks of 32 bytes
  // = channels [0, 32) and [32, 64)
  auto chan = [](int b) { return h16_channel(b >> 3, b & 7); };
  uint8_t* corr = dst + H8_CORR_OFF;
  uint32_t* scales = (uint32_t*)(dst + H8_SCALE_OFF);
  for (int m = 0; m < 4; ++m)
    for (int r = 0; r < 16; ++r) {
      const int co = 16 * m + r;
      for (int t = 0; t < 3; ++t) {
        int sc[4];                     // kb 0/1: lo channels 0-31 / 32-63; kb 2/3: hi
        for (int kb = 0; kb < 4; ++kb) {
          double amax = 0;
          for (int b = 32 * (kb & 1); b < 32 * (kb & 1) + 32; ++b)
            amax = std::fmax(amax, std::fabs(kb < 2 ? Lo(co, chan(b), t) : H(co, chan(b), t)));
          sc[kb] = e8m0_for(amax);
          uint32_t& word = scales[m * 64 + r + 16 * kb];
          word = (word & ~(0xffu << (8 * t))) | ((uint32_t)sc[kb] << (8 * t));
        }
        for (int g = 0; g < 4; ++g) {
          uint8_t* lanebytes = corr + ((m * 3 + t) * 64 + r + 16 * g) * 32;
          for (int jj = 0; jj < 16; ++jj) {
            const int b = 16 * g + jj, ci = chan(b), kb = b >> 5;
            lanebytes[jj] = to_e4m3(std::ldexp(Lo(co, ci, t), -(sc[kb] - 127)));
            lanebytes[16 + jj] = to_e4m3(std::ldexp(H(co, ci, t), -(sc[2 + kb] - 127)));
          }
        }
      }
    }
  float* bias = (float*)(dst + H8_BIAS_OFF);
  for (int c = 0; c < C; ++c) bias[c] = c < f.cout ? (float)f.b[c] : 0.f;
}

// a head as fused16's head record (f16 fragments with the rounding residue in row 1, pack_big_bf16)
// inside an f16 + e4m3-sized record: the ping-pong engine reads the H8 blob with that record stride
// and its bias at H8_BIAS_OFF
static void pack_head_h8(const Folded& f, uint8_t* dst) {
  std::vector<uint8_t> rec(BIG_BYTES_BF16);
  pack_big_bf16(f, rec.data(), true);
  std::memcpy(dst, rec.data(), BIG_FRAG_BYTES_BF16);
  std::memcpy(dst + H8_BIAS_OFF, rec.data() + BIG_FRAG_BYTES_BF16, C * sizeof(float));
}

// a head (cout = 1) as an f16 + e4m3 layer record with its output channel at couts 0 and 32 (the
// first M-tile of either output-channel half of the in-place wave pair) and zeros elsewhere
static void pack_head_h8mfma(const Folded& f, uint8_t* dst) {
  Folded g;
  g.cout = C;
  g.cin = C;
  g.w.assign((size_t)C * C * 3, 0.0);
  g.b.assign(C, 0.0);
  for (int co : {0, 32}) {
    for (int k = 0; k < C * 3; ++k) g.w[(size_t)co * C * 3 + k] = f.w[k];
    g.b[co] = f.b[0];
  }
  pack_big_h8(g, dst);
}

static void pack_small_conv(const Folded& f, float* slot) {   // w[c*3+t], bias at 192 (+c)
  std::memset(slot, 0, SMALL_SLOT_FLOATS * sizeof(float));
  if (f.cin == 1) {
    for (int c = 0; c < f.cout; ++c) {
      for (int t = 0; t < 3; ++t) slot[3 * c + t] = (float)f.W(c, 0, t);
      slot[192 + c] = (float)f.b[c];
    }
  } else {
    for (int c = 0; c < f.cin; ++c)
      for (int t = 0; t < 3; ++t) slot[3 * c + t] = (float)f.W(0, c, t);
    slot[192] = (float)f.b[0];
  }
}

// CBAM: slot+0 fc.0.weight [4][64]; slot+1 fc.2.weight [64][4]; slot+2: fc.0.bias[4] @0,
// fc.2.bias[64] @4, sa.conv.weight [2][7] @68, sa.conv.bias @82 (zeros when the layer has no bias).
static bool pack_cbam(Reader& rd, const Op& o, float* small) {
  const std::string ca = o.conv + "." + o.ca + ".fc.", sa = o.conv + "." + o.sa + ".conv.";
  float* s0 = small + o.slot * SMALL_SLOT_FLOATS;
  float* s1 = s0 + SMALL_SLOT_FLOATS;
  float* s2 = s1 + SMALL_SLOT_FLOATS;
  std::memset(s0, 0, 3 * SMALL_SLOT_FLOATS * sizeof(float));
  const float* p;
  if (!(p = rd.take(ca + "0.weight", 4 * 64))) return false;
  std::memcpy(s0, p, 256 * sizeof(float));
  if (o.bias) {
    if (!(p = rd.take(ca + "0.bias", 4))) return false;
    std::memcpy(s2, p, 4 * sizeof(float));
  }
  if (!(p = rd.take(ca + "2.weight", 64 * 4))) return false;
  std::memcpy(s1, p, 256 * sizeof(float));
  if (o.bias) {
    if (!(p = rd.take(ca + "2.bias", 64))) return false;
    std::memcpy(s2 + 4, p, 64 * sizeof(float));
  }
  if (!(p = rd.take(sa + "weight", 14))) return false;
  std::memcpy(s2 + 68, p, 14 * sizeof(float));
  if (o.bias) {
    if (!(p = rd.take(sa + "bias", 1))) return false;
    s2[82] = p[0];
  }
  return true;
}

static size_t layer_bytes(int layout) {
  return layout == BF16 || layout == F16 ? BIG_BYTES_BF16 : layout == F16F8 ? BIG_BYTES_H8 : BIG_BYTES_F32;
}

// RDN_F16 on the CBAM networks: the in-place single-plane records (F16X: the per-segment kernels,
// for spectra longer than the co-resident teams hold) are followed by a ping-pong section (fused16
// layout, f16 fragments in h16_channel order, the head as its last record) for the team kernel
// cb::team16_forward
bool has_pp16_section(const std::vector<Op>& spec, int dtype) { return dtype == F16 && has_cbam(spec); }
size_t pp16_section_offset(const std::vector<Op>& spec, int dtype) {
  return SMALL_BYTES + (size_t)big_layers(spec, dtype) * layer_bytes(big_layout(spec, dtype));
}

size_t pp16_section_offset_arch(int arch) { return pp16_section_offset(net_spec(arch), F16); }

size_t packed_bytes(const std::vector<Op>& spec, int dtype) {
  size_t n = SMALL_BYTES + (size_t)big_layers(spec, dtype) * layer_bytes(big_layout(spec, dtype));
  if (has_pp16_section(spec, dtype)) n += (size_t)big_layers(spec, F16) * BIG_BYTES_BF16 + BIG_BYTES_BF16;
  return n;
}


// returns "" on success, else the error message
std::string pack(int arch, int dtype, const float* const* tensors, const int64_t* numels, int n, void* dst,
                 size_t cap) {
  const std::vector<Op> spec = net_spec(arch);
  if (spec.empty()) return "unknown arch " + std::to_string(arch);
  if (dtype != F32 && dtype != BF16 && dtype != BF16X3 && dtype != F16F8 && dtype != F16 && dtype != F16MIX)
    return "unknown dtype " + std::to_string(dtype);
  if (dtype == F16MIX && arch != RRCDNET)
    return "unsupported: RDN_F16MIX is built for RRCDNet (the other networks meet 2e-2 in plain RDN_F16)";
  const size_t need = packed_bytes(spec, dtype);
  if (cap < need) return "destination too small: need " + std::to_string(need) + " bytes";
  uint8_t* out = (uint8_t*)dst;
  std::memset(out, 0, need);
  float* small = (float*)out;
  uint8_t* big = out + SMALL_BYTES;
  const int layout = big_layout(spec, dtype);
  const size_t big_bytes = layer_bytes(layout);
  Reader rd{tensors, numels, n};
  int layer = 0;
  for (const Op& o : spec) {
    Folded f;
    switch (o.kind) {
      case OpKind::STEM:
        if (!fold(rd, o, 1, C, f)) return rd.err;
        pack_small_conv(f, small + o.slot * SMALL_SLOT_FLOATS);
        break;
      case OpKind::BIG:
        if (!fold(rd, o, C, C, f)) return rd.err;
        if (layout == BF16 || layout == F16) pack_big_bf16(f, big + layer * big_bytes, layout == F16);
        else if (layout == BF16X3 || layout == F16X) pack_big_x3(f, big + layer * big_bytes, layout == F16X);
        else if (layout == F16F8) pack_big_h8(f, big + layer * big_bytes);
        else pack_big_f32(f, big + layer * big_bytes);
        ++layer;
        break;
      case OpKind::HEAD:
        if (!fold(rd, o, C, 1, f)) return rd.err;
        pack_small_conv(f, small + o.slot * SMALL_SLOT_FLOATS);
        if (layout == BF16 || layout == F16) pack_big_bf16(f, big + (layer++) * big_bytes, layout == F16);
        else if (dtype == F16MIX && &o == &spec.back()) pack_head_h8(f, big + (size_t)F16MIX_LHEAD_REC * big_bytes);
        else if (dtype == F16MIX) pack_head_h8mfma(f, big + (size_t)F16MIX_RHEAD_REC * big_bytes);
        break;
      case OpKind::CBAM:
        if (!pack_cbam(rd, o, small)) return rd.err;
        break;
    }
  }
  if (rd.i != n) return "too many tensors: consumed " + std::to_string(rd.i) + " of " + std::to_string(n);
  if (has_pp16_section(spec, dtype)) {        // second pass: the ping-pong records (BIG, then the head)
    uint8_t* pp = out + pp16_section_offset(spec, dtype);
    Reader r2{tensors, numels, n};
    int k = 0;
    for (const Op& o : spec) {
      Folded f;
      switch (o.kind) {
        case OpKind::STEM:
          if (!fold(r2, o, 1, C, f)) return r2.err;
          break;
        case OpKind::BIG:
          if (!fold(r2, o, C, C, f)) return r2.err;
          pack_big_bf16(f, pp + (size_t)(k++) * BIG_BYTES_BF16, true);
          break;
        case OpKind::HEAD:
          if (!fold(r2, o, C, 1, f)) return r2.err;
          pack_big_bf16(f, pp + (size_t)(k++) * BIG_BYTES_BF16, true);
          break;
        case OpKind::CBAM: {
          std::vector<float> scratch(3 * SMALL_SLOT_FLOATS);
          Op o2 = o;
          o2.slot = 0;
          if (!pack_cbam(r2, o2, scratch.data())) return r2.err;
          break;
        }
      }
    }
  }
  if (dtype == F16F8 || dtype == F16MIX) set_corr_mask(out, dtype == F16F8 ? ~0ull : f16mix_default_mask(arch));
  ((uint32_t*)(out + (size_t)CORR_SLOT * SMALL_SLOT_FLOATS * 4))[TAG_WORD] = blob_tag(arch, dtype);
  return "";
}

uint32_t get_blob_tag(const void* blob) {
  return ((const uint32_t*)((const uint8_t*)blob + (size_t)CORR_SLOT * SMALL_SLOT_FLOATS * 4))[TAG_WORD];
}

// RDN_F16MIX: the big layers (execution order) that keep the e4m3 correction.  Plain f16 (RDN_F16)
// meets the 2e-2 bar on every golden fixture except trained RRCDNet (3.5e-2 fused / 2.6e-2 with the
// exact head input of the in-place path); the head's cancellation x - (r + l)/2 amplifies the
// rounding of the right branch's last layers most (tools/f16mix_select.py, greedy on the GPU), and
// correcting right_net.15-17 (big layers 12-14) brings it to 1.36e-2 with both heads split, 1.65e-2 with the left head in plain f16 (tools/f16mix_masks.py).  The
// pattern is compiled into the kernel (fused_inplace.hip RRCDNET_F16MIX_TAIL); the blob records it.
uint64_t f16mix_default_mask(int arch) {
  return arch == RRCDNET ? (((1ull << F16MIX_TAIL) - 1) << (15 - F16MIX_TAIL)) : 0;
}
void set_corr_mask(void* blob, uint64_t mask) {
  uint32_t* w = (uint32_t*)((uint8_t*)blob + (size_t)CORR_SLOT * SMALL_SLOT_FLOATS * 4);
  w[0] = (uint32_t)mask;
  w[1] = (uint32_t)(mask >> 32);
}
uint64_t get_corr_mask(const void* blob) {
  const uint32_t* w = (const uint32_t*)((const uint8_t*)blob + (size_t)CORR_SLOT * SMALL_SLOT_FLOATS * 4);
  return (uint64_t)w[1] << 32 | w[0];
}

}  // namespace rdn
