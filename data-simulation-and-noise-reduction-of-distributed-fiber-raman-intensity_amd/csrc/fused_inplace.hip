// Whole-network fused tile kernels on the in-place 256-byte-row tile (see inplace.hpp):
// exact-fp32 (MODE_F32), split-bf16 (MODE_X3) and f16 + e4m3-correction (MODE_H8) variants of 1DCNN, RRCDNet, DSDN and PIDN.
//
// Reference forwards: 1DCNN/train.py:71-82, RRCDNet/train.py:72-98, DSDN/train.py:72-126,
// PIDN/train.py:72-106.
#include <cstddef>

#include "inplace.hpp"
#include "host_util.hpp"
#include "metrics.hpp"
// the f16 ping-pong layers of fused16.hpp over the f16 + e4m3 blob (its leading f16 fragments):
// the plain layers of RDN_F16MIX (rrcdnet_hybrid below)
#define RDN_H16_F16 1
#define H16_NS h16x
#define H16_LAYER_BYTES BIG_BYTES_H8
#define H16_BIAS_OFF H8_BIAS_OFF
#include "fused16.hpp"
// the same over 256-row tiles: the ping-pong part of RDN_F16MIX's latency geometry (rrcdnet_short)
#undef H16_NS
#define H16_NS h16xs
#define H16_TILE_ROWS 256
#include "fused16.hpp"
#undef H16_TILE_ROWS
// the same on the walk geometry (512-position tiles, the in-place engine's 4 blocks): the ping-pong
// part of the RDN_F16MIX walk (rrcdnet_hybrid_walk.hpp)
#undef H16_NS
#define H16_NS h16xw
#define H16_WALK_T RDN_WALK_ROWS_MIX
#include "fused16.hpp"
#undef H16_WALK_T

namespace rdn {
namespace ip {

// Network bodies.  EDGE: the tile holds positions outside [0, L) (first / last tile of a
// spectrum), whose rows every write-back re-zeroes; interior tiles skip that per-row select.
#define IP_BODY(name) \
  template <int MODE, bool EDGE, int NBK, int TAIL> \
  __device__ __forceinline__ void name##_body(Tile& tl, float* y, int n, int L, int T, unsigned* status)

// MODE_H8 (RDN_F16F8 / RDN_F16MIX) bodies end with the range vote (inplace.hpp range_vote): a tile
// whose activations left the e4m3 planes' range writes NaN and raises the status word
template <int MODE, int N>
__device__ __forceinline__ void range_guard(const Tile& tl, unsigned* status, float (&o)[N]) {
  if constexpr (MODE == MODE_H8) {
    if (range_vote(tl, 0, status)) nan_rows(o);
  }
}

// RRCDNet's right-branch head outputs are parked in y (as fp32) over the left branch in the
// vectorized-head modes, whose 5 double rows per lane would otherwise hold 10 VGPRs through it
// (the f16f8 kernel spilled); the exact-fp32 and split modes keep their 2 doubles in registers.
// The rounding of r to fp32 is 2^-24 relative, far below those modes' operand error.
template <int MODE, int NBK>
__device__ __forceinline__ void park_rows(const Tile& tl, float* y, int n, const double (&r)[HeadOut<MODE, NBK>::ROWS],
                                          int H, int T) {
  float o[HeadOut<MODE, NBK>::ROWS];
  round_rows(r, o);
  store_out<MODE, NBK>(tl, y, n, o, H, T);
}
template <int MODE, int NBK>
__device__ __forceinline__ double parked_row(const Tile& tl, const float* y, int n, int k, int H, int T) {
  const int j = HeadOut<MODE, NBK>::row(k), p = tl.base + j;
  return HeadOut<MODE, NBK>::writer() && j >= H && j < H + T && p < tl.L ? (double)y[(size_t)n * tl.L + p] : 0.0;
}

// 128-row blocks per tile: 640-row tiles (the whole LDS, no guard rows) everywhere except DSDN,
// whose ResidualBlock identity lives in VGPRs (20 vs 16 f32x4 per lane at 640 rows: spills).
template <int ARCH> struct NetGeo { static constexpr int NBK = 5; };

#ifndef RDN_DSDN_NBK
#define RDN_DSDN_NBK 4
#endif
template <> struct NetGeo<DSDN> { static constexpr int NBK = RDN_DSDN_NBK; };

IP_BODY(denoisecnn) {
  constexpr int H = fused_halo(DENOISECNN);
  using G = Geo<MODE, false>;
  f32x4 id[16 * NBK / 4];
  LayerA<MODE> a;
  load_layer_a<MODE>(tl, 0, a);
  if (NBK == 4) zero_guards(tl.lds);
  stem<MODE, false, NBK>(tl, 0);
  __syncthreads();
  for (int i = 0; i < 18; ++i) conv<MODE, RELU, G::S, EDGE, NBK>(tl, 1, id, a, i + 1 < 18);
  double d[HeadOut<MODE, NBK>::ROWS];
  head<MODE, NBK>(tl, 1, d);
  float o[HeadOut<MODE, NBK>::ROWS];
  round_rows(d, o);
  range_guard<MODE>(tl, status, o);
  store_out<MODE, NBK>(tl, y, n, o, H, T);
}

IP_BODY(rrcdnet) {
  constexpr int H = fused_halo(RRCDNET);
  using G = Geo<MODE, false>;
  f32x4 id[16 * NBK / 4];
  LayerA<MODE> a;
  load_layer_a<MODE>(tl, 0, a);
  if (NBK == 4) zero_guards(tl.lds);
  stem<MODE, false, NBK>(tl, 0);
  __syncthreads();
  if constexpr (TAIL == 0) {
    for (int i = 0; i < 15; ++i) conv<MODE, RELU, G::S, EDGE, NBK>(tl, 1, id, a, true);
  } else {
    // RDN_F16MIX: plain f16 layers (the correction compiled out), the last of them also writing the
    // e4m3 planes, then TAIL corrected layers (right_net.15-17 for TAIL = 3: the layers whose f16
    // rounding the head's cancellation x - (r + l)/2 amplifies most, tools/f16mix_select.py).
    // (A wave split with all four M-tiles per wave -- half the LDS reads, twice the per-wave weight
    // fragments -- measured 10 % slower: the layer is not LDS-bound, the extra L1 weight traffic is.)
    for (int i = 0; i < 14 - TAIL; ++i) conv<MODE, RELU, G::S, EDGE, NBK, false, false, false>(tl, 1, id, a, true);
    conv<MODE, RELU, G::S, EDGE, NBK, false, true, true>(tl, 1, id, a, true);
    for (int i = 0; i < TAIL; ++i) conv<MODE, RELU, G::S, EDGE, NBK, true, true, true>(tl, 1, id, a, i + 1 < TAIL);
    load_layer_a<MODE>(tl, tl.layer, a);                // the left branch's first layer (f16 + e4m3)
  }
  using HO = HeadOut<MODE, NBK>;
  double r[HO::ROWS];
  head<MODE, NBK>(tl, 2, r);
  if constexpr (HO::VEC) park_rows<MODE, NBK>(tl, y, n, r, H, T);
  __syncthreads();               // the left stem overwrites the rows the right head just read
  stem<MODE, false, NBK>(tl, 1);
  __syncthreads();
  if constexpr (TAIL == 0) {
    for (int i = 0; i < 14; ++i) conv<MODE, RELU, G::S, EDGE, NBK>(tl, i == 7 ? 1 : 2, id, a, i + 1 < 14);
  } else {
    // plain f16; the last layer writes the e4m3 lo plane the head reads
    for (int i = 0; i < 13; ++i) conv<MODE, RELU, G::S, EDGE, NBK, false, false, false>(tl, i == 7 ? 1 : 2, id, a, true);
    conv<MODE, RELU, G::S, EDGE, NBK, false, true, false>(tl, 2, id, a, false);
  }
  double l[HO::ROWS];
  head<MODE, NBK>(tl, 3, l);
  float o[HO::ROWS];
#pragma unroll
  for (int k = 0; k < HO::ROWS; ++k) {      // x - (r + l)/2 from the unrounded heads, one rounding
    const int p = tl.base + HO::row(k);
    const float xv = in_range(p, L) ? tl.x[p] : 0.f;
    const double rv = HO::VEC ? parked_row<MODE, NBK>(tl, y, n, k, H, T) : r[k];
    o[k] = (float)((double)xv - (rv + l[k]) * 0.5);
  }
  range_guard<MODE>(tl, status, o);
  store_out<MODE, NBK>(tl, y, n, o, H, T);
}

IP_BODY(dsdn) {
  constexpr int H = fused_halo(DSDN);
  using G = Geo<MODE, true>;
  f32x4 id[16 * NBK / 4];
  LayerA<MODE> a;
  load_layer_a<MODE>(tl, 0, a);
  if (NBK == 4) zero_guards(tl.lds);
  stem<MODE, false, NBK>(tl, 0);
  __syncthreads();
  conv<MODE, RELU, G::S, EDGE, NBK>(tl, 1, id, a, true);                        // conv1
  conv<MODE, RELU | SAVE_ID, G::S, EDGE, NBK>(tl, 1, id, a, true);              // conv2 -> first block identity
  for (int b = 0; b < 15; ++b) {
    conv<MODE, RELU, G::S, EDGE, NBK>(tl, 1, id, a, true);                      // relu(bn1(conv1 x))
    conv<MODE, RELU | ADD_ID | SAVE_ID, G::S, EDGE, NBK>(tl, 1, id, a, b < 14); // relu(bn2(conv2 .) + x)
  }
  double d[HeadOut<MODE, NBK>::ROWS];
  head<MODE, NBK>(tl, 1, d);
  float o[HeadOut<MODE, NBK>::ROWS];
  round_rows(d, o);
  range_guard<MODE>(tl, status, o);
  store_out<MODE, NBK>(tl, y, n, o, H, T);
}

IP_BODY(pidn) {
  constexpr int H = fused_halo(PIDN);
  using G = Geo<MODE, false>;
  f32x4 id[16 * NBK / 4];
  LayerA<MODE> a;
  load_layer_a<MODE>(tl, 0, a);
  if (NBK == 4) zero_guards(tl.lds);
  stem<MODE, false, NBK>(tl, 0);
  __syncthreads();
  for (int b = 0; b < 15; ++b) {
    conv<MODE, RELU, G::S, EDGE, NBK>(tl, 1, id, a, true);
    conv<MODE, 0, G::S, EDGE, NBK>(tl, 1, id, a, b < 14);
  }
  stem<MODE, true, NBK>(tl, 0);       // + identity (the stem output), recomputed from x
  __syncthreads();
  double d[HeadOut<MODE, NBK>::ROWS];
  head<MODE, NBK>(tl, 1, d);
  float o[HeadOut<MODE, NBK>::ROWS];
  round_rows(d, o);
#pragma unroll
  for (int k = 0; k < HeadOut<MODE, NBK>::ROWS; ++k) o[k] = 1.0f / (1.0f + expf(-o[k]));
  range_guard<MODE>(tl, status, o);
  store_out<MODE, NBK>(tl, y, n, o, H, T);
}

// Short last tiles: the last tile of a spectrum holds only the positions left over by the full
// tiles before it (at L = 10,000 RRCDNet: 106 of its 640 rows), so it runs on the fewest 128-row
// blocks that reach position L + 1 (2 or 3 blocks, wrapped geometry; 4 = the guarded 512-row
// geometry).  Rows at positions >= L are re-zeroed by every write-back, so the garbage a wrapped
// tap (d <= 2) reads from the tile's other end never survives past them; the left end erodes into
// the halo exactly as in the full tile.  RRCDNet at L = 10,000 executes 3.3 % fewer rows (+1 %
// measured: a short tile still fetches every layer's weights).  DSDN (512-row tiles, identity in
// VGPRs) keeps one geometry: the extra bodies raised its spills.
// RDN_F16MIX: corrected layers at the end of RRCDNet's right branch (pack.cpp f16mix_default_mask)
constexpr int RRCDNET_F16MIX_TAIL = F16MIX_TAIL;

// RDN_F16MIX on full tiles: the plain f16 layers run on fused16's ping-pong tile (two 640 x 128-B
// buffers, one barrier per layer, no write-back lag: 8 % fewer cycles per layer than the in-place
// tile's f16 plane), then the activations move once into the in-place tile for the layers the
// e4m3 planes serve (the producer of the corrected tail, the tail itself, the last left layer) and
// the two heads, which read the f16 + e4m3-lo planes (HeadOut, vectorized).  The big-layer
// fragments of the H8 blob start with fused16's [m][k-step][lane][8 x f16] map (pack.cpp
// pack_big_h8 / pack_big_bf16, same h16_channel K order), so both halves read one blob.

namespace hyb640 {
#define PPNS h16x
#define HNBK 5
#include "rrcdnet_hybrid.hpp"
#undef PPNS
#undef HNBK
}  // namespace hyb640
namespace hyb256 {
#define PPNS h16xs
#define HNBK 2
#include "rrcdnet_hybrid.hpp"
#undef PPNS
#undef HNBK
}  // namespace hyb256

// RDN_F16MIX reads one record past an RDN_F16F8 blob's end: a blob whose layout tag (pack.cpp) is not
// RDN_F16MIX RRCDNet's gets NaN outputs instead of a read past it (one scalar load per workgroup)
__device__ __forceinline__ bool f16mix_blob_ok(const uint8_t* blob) {
  const uint32_t tag = ((const __attribute__((address_space(4))) uint32_t*)blob)[CORR_SLOT * SMALL_SLOT_FLOATS + TAG_WORD];
  return tag == blob_tag(RRCDNET, F16MIX);
}
__device__ __forceinline__ void nan_outputs(const Tile& tl, float* y, int n, int T) {
  for (int j = __builtin_amdgcn_workitem_id_x(); j < T; j += THREADS) {
    const int p = tl.base + fused_halo(RRCDNET) + j;
    if (p < tl.L) y[(size_t)n * tl.L + p] = __uint_as_float(0x7fc00000u);
  }
}

// The all-corrected body of a spiked tile (RDN_F16F8 on the RDN_F16MIX blob, which carries every
// layer's e4m3 correction fragments)
template <bool EDGE, int NBK>
__device__ __forceinline__ void rrcdnet_f16f8_tile(Tile& tl, float* y, int n, int L, int T, unsigned* status) {
  rrcdnet_body<MODE_H8, EDGE, NBK, 0>(tl, y, n, L, T, status);
}

// Whether any input of the tile's rows [base, base + WB) inside [0, L) lies outside [lo, hi]
// (workgroup-uniform; a vote word per wave at the end of the LDS, read before a barrier that precedes
// any other LDS write)
__device__ __forceinline__ bool window_outside(const Tile& tl, float lo, float hi) {
  bool out = false;
  if (lo <= hi) {
    for (int r = __builtin_amdgcn_workitem_id_x(); r < TileGeo<5>::WB; r += THREADS) {
      const int p = tl.base + r;
      if (in_range(p, tl.L)) {
        const float v = tl.x[p];
        out = out || v < lo || v > hi;
      }
    }
  }
  unsigned* vote = (unsigned*)(tl.lds + TileGeo<5>::LDS) - THREADS / 64;
  const bool wave_out = __builtin_amdgcn_ballot_w64(out) != 0;
  if ((__builtin_amdgcn_workitem_id_x() & 63) == 0) vote[__builtin_amdgcn_workitem_id_x() >> 6] = wave_out ? 1u : 0u;
  __syncthreads();
  bool any = false;
#pragma unroll
  for (int k = 0; k < THREADS / 64; ++k) any = any || vote[k] != 0;
  __syncthreads();
  return any;
}

// RDN_F16MIX RRCDNet: hybrid bodies on 640-row tiles, the in-place body on short last tiles; a tile
// whose input window leaves [F16MIX_WIN_LO, F16MIX_WIN_HI] (a spike) runs every layer corrected.
// Tile `id` (spectrum id / tiles, tile id % tiles) of a launch (one tile per workgroup, or the walk
// kernel's fallback loop over a spiked spectrum's tiles).
template <int TAIL>
__device__ __forceinline__ void rrcdnet_hybrid_tile(char* lds, const uint8_t* blob, const float* x, float* y, int L,
                                                    int T, int tiles, unsigned* status, int64_t id) {
  int n;
  Tile tl = make_tile_at(lds, blob, x, L, T, tiles, fused_halo(RRCDNET), id, n);
  tl.status = status;
  const int need = L - tl.base + 2;
  if (tl.base >= 0 && tl.base + TileGeo<5>::WB <= L) {
    if (!hyb640::rrcdnet_hybrid_body<false, TAIL>(tl, y, n, L, T, status))
      rrcdnet_f16f8_tile<false, 5>(tl, y, n, L, T, status);        // spiked tile: every layer corrected
  } else if (need <= 512) {
    // short last tile (the in-place body on the fewest blocks): all layers corrected when spiked
    const bool spiked = window_outside(tl, F16MIX_WIN_LO, F16MIX_WIN_HI);
    if (need <= 256) spiked ? rrcdnet_f16f8_tile<true, 2>(tl, y, n, L, T, status) : rrcdnet_body<MODE_H8, true, 2, TAIL>(tl, y, n, L, T, status);
    else if (need <= 384) spiked ? rrcdnet_f16f8_tile<true, 3>(tl, y, n, L, T, status) : rrcdnet_body<MODE_H8, true, 3, TAIL>(tl, y, n, L, T, status);
    else spiked ? rrcdnet_f16f8_tile<true, 4>(tl, y, n, L, T, status) : rrcdnet_body<MODE_H8, true, 4, TAIL>(tl, y, n, L, T, status);
  } else if (!hyb640::rrcdnet_hybrid_body<true, TAIL>(tl, y, n, L, T, status)) {
    rrcdnet_f16f8_tile<true, 5>(tl, y, n, L, T, status);
  }
}
template <int TAIL>
__global__ __launch_bounds__(THREADS) void rrcdnet_hybrid(const uint8_t* __restrict__ blob, const float* __restrict__ x,
                                                          float* __restrict__ y, int L, int T, int tiles,
                                                          unsigned* __restrict__ status) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  if (!f16mix_blob_ok(blob)) {
    int n;
    const Tile tl = make_tile(lds, blob, x, L, T, tiles, fused_halo(RRCDNET), n);
    return nan_outputs(tl, y, n, T);
  }
  rrcdnet_hybrid_tile<TAIL>(lds, blob, x, y, L, T, tiles, status, __builtin_amdgcn_workgroup_id_x());
}

#include "rrcdnet_hybrid_walk.hpp"

// Whether any input of spectrum xs lies outside [lo, hi] (workgroup-uniform; vote words at the end of
// the LDS, behind everything the kernels use)
__device__ __forceinline__ bool spectrum_outside(char* lds, const float* xs, int L, float lo, float hi) {
  bool out = false;
  if (lo <= hi) {
    for (int p = __builtin_amdgcn_workitem_id_x(); p < L; p += THREADS) {
      const float v = xs[p];
      out = out || v < lo || v > hi;
    }
  }
  unsigned* vote = (unsigned*)(lds + 163840) - THREADS / 64;
  const bool wave_out = __builtin_amdgcn_ballot_w64(out) != 0;
  if ((__builtin_amdgcn_workitem_id_x() & 63) == 0) vote[__builtin_amdgcn_workitem_id_x() >> 6] = wave_out ? 1u : 0u;
  __syncthreads();
  bool any = false;
#pragma unroll
  for (int k = 0; k < THREADS / 64; ++k) any = any || vote[k] != 0;
  __syncthreads();
  return any;
}

// RDN_F16MIX RRCDNet on the walk geometry: one workgroup per spectrum (rrcdnet_hybrid_walk.hpp); a
// spectrum with a spike takes the tiled hybrid tile by tile (T, tiles: the 640-row geometry)
template <int TAIL>
__device__ __forceinline__ void hybrid_walk_spectrum(char* lds, const uint8_t* __restrict__ blob,
                                                     const float* __restrict__ x, float* __restrict__ y, int L, int T,
                                                     int tiles, int ntiles, unsigned* __restrict__ status, int n) {
  static_assert(TAIL == F16MIX_TAIL, "the walk body is written for the compiled-in tail");
  if (!f16mix_blob_ok(blob)) {
    for (int p = __builtin_amdgcn_workitem_id_x(); p < L; p += THREADS) y[(size_t)n * L + p] = __uint_as_float(0x7fc00000u);
    return;
  }
  if (spectrum_outside(lds, x + (size_t)n * L, L, F16MIX_WIN_LO, F16MIX_WIN_HI)) {
    for (int t = 0; t < tiles; ++t) {
      rrcdnet_hybrid_tile<TAIL>(lds, blob, x, y, L, T, tiles, status, (int64_t)n * tiles + t);
      __syncthreads();               // the next tile's stem overwrites what this one read last
    }
    return;
  }
  int n_;
  Tile tl = make_tile_at(lds, blob, x, L, 0, 1, 0, n, n_);
  tl.status = status;
  tl.cs_cur = tl.cs_prev = tl.dn_prev = 0;
  tl.dnext = 1;
  tl.first = true;
  hybw::PP::Tile t16 = hybw::PP::init_tile(lds, blob, blob + SMALL_BYTES, tl.x, L, 0);
  t16.status = status;
#if defined(RDN_HYB_STAMPS) && RDN_HYB_STAMPS
  for (int k = 0; k < 5; ++k) t16.lst[k] = 0;
  tl.bwork = tl.bwait = 0;
#endif
  hybw::PP::Frags F0, F1;
  hybw::PP::load_frags(t16, 0, F1);
  hybw::PP::StemX xs = hybw::PP::walk_stem_load(t16, 0, hybw::RIGHT_C0);
  y += (size_t)n * L;
  hybw::Stamps st;
  // the first tile, the interior tiles, the tiles reaching L: three straight runs of one body each (the
  // two bodies under one per-tile branch made the register allocator spill ~160 VGPRs)
  hybw::tile<true>(tl, t16, y, 0, ntiles, F0, F1, xs, status, st);
  t16.first = false;
  int t = 1;
  for (; t < ntiles && (t + 1) * hybw::PP::WT <= L; ++t) hybw::tile<false>(tl, t16, y, t, ntiles, F0, F1, xs, status, st);
  for (; t < ntiles; ++t) hybw::tile<true>(tl, t16, y, t, ntiles, F0, F1, xs, status, st);
  st.flush(status);
#if defined(RDN_HYB_STAMPS) && RDN_HYB_STAMPS
  if (status && (__builtin_amdgcn_workitem_id_x() & 63) == 0)      // every wave's view: words 32 + 5 w + k
    for (int k = 0; k < 5; ++k) atomicAdd((unsigned long long*)status + 32 + 5 * (__builtin_amdgcn_workitem_id_x() >> 6) + k, t16.lst[k]);
  if (status && (__builtin_amdgcn_workitem_id_x() & 63) == 0) {     // words 80 + 2 w: corrected-layer work / wait
    atomicAdd((unsigned long long*)status + 80 + 2 * (__builtin_amdgcn_workitem_id_x() >> 6), tl.bwork);
    atomicAdd((unsigned long long*)status + 81 + 2 * (__builtin_amdgcn_workitem_id_x() >> 6), tl.bwait);
  }
#endif
}
// MET: the spectrum's metrics follow its walk in the same workgroup (metrics.hpp walk_metrics; a
// separate instantiation, so the plain forward's register allocation does not see the epilogue).  The
// epilogue reads y and mo from the kernel-argument segment after the walk (an opaque pointer, so the
// loads are not hoisted to the kernel's start): held in SGPRs across the walk, they cost 44 more
// spilled VGPRs in the tile loop.  HybWalkArgs mirrors the parameter list (the kernarg layout).
struct HybWalkArgs {
  const uint8_t* blob;
  const float* x;
  float* y;
  int L, T, tiles, ntiles;
  unsigned* status;
  met::MetricOut mo;
};
static_assert(offsetof(HybWalkArgs, y) == 16 && offsetof(HybWalkArgs, L) == 24 && offsetof(HybWalkArgs, mo) == 48,
              "HybWalkArgs mirrors rrcdnet_hybrid_walk's parameters (kernarg layout: natural alignment, in order)");
template <int TAIL, bool MET>
__global__ __launch_bounds__(THREADS) void rrcdnet_hybrid_walk(const uint8_t* __restrict__ blob,
                                                               const float* __restrict__ x, float* __restrict__ y,
                                                               int L, int T, int tiles, int ntiles,
                                                               unsigned* __restrict__ status, met::MetricOut mo) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  wave_priority();
  const int n = __builtin_amdgcn_workgroup_id_x();
  hybrid_walk_spectrum<TAIL>(lds, blob, x, y, L, T, tiles, ntiles, status, n);
  if (MET) {
    __syncthreads();                   // the walk's (or the spiked fallback's) last LDS use is done
    const char* ka = (const char*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(ka));
    const HybWalkArgs* a = (const HybWalkArgs*)ka;
    met::walk_metrics(a->y + (size_t)n * a->L, a->L, n, lds, a->mo);
  }
}

// RDN_F16MIX RRCDNet on 256-row tiles (the hybrid body on h16xs + the 2-block in-place tile): the
// latency geometry for launches too small to fill the chip (launch_fused_inplace_short)
template <int TAIL>
__global__ __launch_bounds__(THREADS) void rrcdnet_short(const uint8_t* __restrict__ blob, const float* __restrict__ x,
                                                         float* __restrict__ y, int L, int T, int tiles,
                                                         unsigned* __restrict__ status) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  int n;
  Tile tl = make_tile(lds, blob, x, L, T, tiles, fused_halo(RRCDNET), n);
  tl.status = status;
  if (!f16mix_blob_ok(blob)) return nan_outputs(tl, y, n, T);
  if (tl.base >= 0 && tl.base + TileGeo<2>::WB <= L) {
    if (!hyb256::rrcdnet_hybrid_body<false, TAIL>(tl, y, n, L, T, status))
      rrcdnet_f16f8_tile<false, 2>(tl, y, n, L, T, status);
  } else if (!hyb256::rrcdnet_hybrid_body<true, TAIL>(tl, y, n, L, T, status)) {
    rrcdnet_f16f8_tile<true, 2>(tl, y, n, L, T, status);
  }
}

#define IP_KERNEL(name, arch)                                                                              \
  template <int MODE, int TAIL = 0>                                                                         \
  __global__ __launch_bounds__(THREADS) void name(const uint8_t* __restrict__ blob, const float* __restrict__ x, \
                                                 float* __restrict__ y, int L, int T, int tiles,            \
                                                 unsigned* __restrict__ status) {                           \
    extern __shared__ __attribute__((aligned(16))) char lds[];                                             \
    int n;                                                                                                 \
    Tile tl = make_tile(lds, blob, x, L, T, tiles, fused_halo(arch), n);                                   \
    tl.status = status;                                                                                    \
    constexpr int NBK = NetGeo<arch>::NBK;                                                                 \
    const int need = L - tl.base + 2;  /* rows up to position L + 1: short last tiles */                     \
    if (tl.base >= 0 && tl.base + TileGeo<NBK>::WB <= L) name##_body<MODE, false, NBK, TAIL>(tl, y, n, L, T, status); \
    else if (NBK == 5 && need <= 256) name##_body<MODE, true, NBK == 5 ? 2 : NBK, TAIL>(tl, y, n, L, T, status);  \
    else if (NBK == 5 && need <= 384) name##_body<MODE, true, NBK == 5 ? 3 : NBK, TAIL>(tl, y, n, L, T, status);  \
    else if (NBK == 5 && need <= 512) name##_body<MODE, true, NBK == 5 ? 4 : NBK, TAIL>(tl, y, n, L, T, status);  \
    else name##_body<MODE, true, NBK, TAIL>(tl, y, n, L, T, status);                                             \
  }

IP_KERNEL(denoisecnn, DENOISECNN)
IP_KERNEL(rrcdnet, RRCDNET)
IP_KERNEL(dsdn, DSDN)
IP_KERNEL(pidn, PIDN)

}  // namespace ip

typedef void (*fused_kernel_t)(const uint8_t*, const float*, float*, int, int, int, unsigned*);

template <int MODE>
static fused_kernel_t pick(int arch) {
  switch (arch) {
    case DENOISECNN: return ip::denoisecnn<MODE>;
    case RRCDNET: return ip::rrcdnet<MODE>;
    case DSDN: return ip::dsdn<MODE>;
    case PIDN: return ip::pidn<MODE>;
    default: return nullptr;
  }
}

// RDN_F16MIX RRCDNet with 256-row tiles (ip::rrcdnet_short)
hipError_t launch_fused_inplace_short(const uint8_t* blob, const float* x, float* y, int64_t n, int L,
                                      unsigned* status, hipStream_t stream) {
  const fused_kernel_t k = ip::rrcdnet_short<ip::RRCDNET_F16MIX_TAIL>;
  const hipError_t e = ensure_dynamic_lds((const void*)k, 92, (int)ip::TileGeo<2>::LDS, stream_device(stream));
  if (e != hipSuccess) return e;
  const int H = fused_halo(RRCDNET), T = ip::TileGeo<2>::WB - 2 * H, tiles = (L + T - 1) / T;
  const int64_t chunk = (int64_t)(0x7fffffff / tiles);
  for (int64_t n0 = 0; n0 < n; n0 += chunk) {
    const int64_t nn = n - n0 < chunk ? n - n0 : chunk;
    hipLaunchKernelGGL(k, dim3((unsigned)(nn * tiles)), dim3(THREADS), ip::TileGeo<2>::LDS, stream, blob, x + n0 * L,
                       y + n0 * L, L, T, tiles, status);
  }
  return hipGetLastError();
}

// RDN_F16MIX RRCDNet on the walk geometry (ip::rrcdnet_hybrid_walk): one workgroup per spectrum
hipError_t launch_fused_inplace_walk(const uint8_t* blob, const float* x, float* y, int64_t n, int L, unsigned* status,
                                     const met::MetricOut* mo, hipStream_t stream) {
  const bool met = mo && mo->clean;
  const auto k = met ? ip::rrcdnet_hybrid_walk<ip::RRCDNET_F16MIX_TAIL, true> : ip::rrcdnet_hybrid_walk<ip::RRCDNET_F16MIX_TAIL, false>;
  // attribute slots 93 / 94, host_util.hpp
  const hipError_t e = ensure_dynamic_lds((const void*)k, met ? 94 : 93, 163840, stream_device(stream));
  if (e != hipSuccess) return e;
  const int H = fused_halo(RRCDNET), T = ip::TileGeo<5>::WB - 2 * H, tiles = (L + T - 1) / T;
  const int ntiles = (int)(((int64_t)L + walk_shift(RRCDNET) + RDN_WALK_ROWS_MIX - 1) / RDN_WALK_ROWS_MIX);
  for (int64_t n0 = 0; n0 < n; n0 += 0x7fffffff) {
    const int64_t nn = n - n0 < 0x7fffffff ? n - n0 : 0x7fffffff;
    hipLaunchKernelGGL(k, dim3((unsigned)nn), dim3(THREADS), 163840, stream, blob, x + n0 * L, y + n0 * L, L, T, tiles,
                       ntiles, status, met::chunk(mo, n0, L));
  }
  return hipGetLastError();
}

// dtype: F32 (exact fp32), BF16X3 (split bf16) or F16F8 (f16 + e4m3 correction); see common.hpp
// status: the workspace's range word (RDN_F16F8 / RDN_F16MIX; NULL: a saturated tile's NaN outputs only)
hipError_t launch_fused_inplace(int arch, int dtype, const uint8_t* blob, const float* x, float* y, int64_t n, int L,
                                unsigned* status, hipStream_t stream) {
  if (arch < 0 || arch >= 8 || dtype < 0 || dtype > F16MIX) return hipErrorInvalidValue;
  const fused_kernel_t k = dtype == BF16X3 ? pick<ip::MODE_X3>(arch)
                           : dtype == F16F8 ? pick<ip::MODE_H8>(arch)
                           : dtype == F16MIX ? (arch == RRCDNET ? ip::rrcdnet_hybrid<ip::RRCDNET_F16MIX_TAIL> : nullptr)
                           : dtype == F32   ? pick<ip::MODE_F32>(arch) : nullptr;
  if (!k) return hipErrorInvalidValue;
  const int nbk = arch == DSDN ? ip::NetGeo<DSDN>::NBK : ip::NetGeo<RRCDNET>::NBK;
  const int wb = 128 * nbk;
  const uint32_t lds = nbk == 4 ? ip::TileGeo<4>::LDS : ip::TileGeo<5>::LDS;
  // attribute slots 8-39 and 70-77 (RDN_F16MIX), host_util.hpp
  const int slot = dtype == F16MIX ? 70 + arch : 8 + dtype * 8 + arch;
  const hipError_t e = ensure_dynamic_lds((const void*)k, slot, (int)lds, stream_device(stream));
  if (e != hipSuccess) return e;
  const int H = fused_halo(arch), T = wb - 2 * H, tiles = (L + T - 1) / T;
  const int64_t chunk = (int64_t)(0x7fffffff / tiles);
  for (int64_t n0 = 0; n0 < n; n0 += chunk) {
    const int64_t nn = n - n0 < chunk ? n - n0 : chunk;
    hipLaunchKernelGGL(k, dim3((unsigned)(nn * tiles)), dim3(THREADS), lds, stream, blob, x + n0 * L,
                       y + n0 * L, L, T, tiles, status);
  }
  return hipGetLastError();
}

}  // namespace rdn
