// RDN_F16 with 256-row tiles (namespace rdn::h16fs, launcher launch_fused16_f16_small): the latency
// geometry for launches too small to fill the chip (evaulate.py:29-32 calls the model one spectrum at
// a time).  At L = 10,000 a spectrum is 51 tiles of 198 own positions instead of 18 of 582: 2.8x
// the workgroups, each layer about 0.4x as long, 1.2x the total MFMA work (the halo is 58 of 256
// rows).  Same kernels and numerics as fused16_f16.hip; only the tile length differs.
#define RDN_H16_F16 1
#define H16_NS h16fs
#define H16_LAUNCH launch_fused16_f16_small
#define H16_ATTR_SLOT0 84
#define H16_TILE_ROWS 256
#include "fused16.hip"
