// RDN_F16 on the walk geometry (fused16.hpp "Walk instantiation"; namespace rdn::h16fw, launcher
// launch_fused16_f16_walk): one workgroup per spectrum walks 576-position tiles left to right with
// time-skewed layers, so no halo rows are recomputed.  Same MFMA products and roundings per output as
// fused16_f16.hip (bitwise equal outputs away from the spectrum's ends).
#define RDN_H16_F16 1
#define H16_NS h16fw
#define H16_LAUNCH launch_fused16_f16_walk
#define H16_ATTR_SLOT0 100
#define H16_WALK_T H16_WALK_ROWS
#include "fused16.hip"
