// RDN_F16: the fused 16-bit kernels of fused16.hip instantiated with f16 weights / activations and
// v_mfma_f32_16x16x32_f16 (namespace rdn::h16f, launcher launch_fused16_f16).
#define RDN_H16_F16 1
#include "fused16.hip"
