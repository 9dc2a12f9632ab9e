// Host-side description of each reference network: which state_dict tensors feed which packed
// layer, in the order the device kernels consume them.  Single source of truth for
// rdn_param_names() and rdn_pack().
#pragma once
#include <string>
#include <vector>

namespace rdn {

enum class OpKind {
  STEM,    // Conv1d(1, 64, 3) [+ BatchNorm1d]          -> small slot (fp32)
  BIG,     // Conv1d(64, 64, 3, d) [+ BatchNorm1d]      -> big section (MFMA fragments)
  HEAD,    // Conv1d(64, 1, 3)                          -> small slot (fp32) and, for bf16, a big layer
  CBAM,    // ChannelAttention fc.0/fc.2 + SpatialAttention conv (2->1, k7) -> two small slots
};

struct Op {
  OpKind kind;
  std::string conv;    // state_dict prefix of the Conv1d (CBAM: prefix of the CBAM module)
  std::string bn;      // state_dict prefix of the folded BatchNorm1d, "" if none
  int slot;            // small-section slot (STEM/HEAD/CBAM)
  bool bias = true;    // CBAM: Linear/Conv layers carry a bias (ADSDN) or not (APIDN)
  std::string ca = "channel_attention", sa = "spatial_attention";   // CBAM child names
};

std::vector<Op> net_spec(int arch);                     // empty for an unknown arch
std::vector<std::string> param_names(const std::vector<Op>& spec);
int big_layers(const std::vector<Op>& spec, int dtype);

}  // namespace rdn
