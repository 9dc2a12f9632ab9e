// RDN_F16MIX RRCDNet hybrid on the walk geometry (included once by fused_inplace.hip, namespace hybw):
// one workgroup walks a spectrum's 576-position tiles (RDN_WALK_ROWS_MIX) left to right (fused16.hpp "Walk
// instantiation"),
// no halo rows recomputed.  Per tile, as the tiled hybrid (rrcdnet_hybrid.hpp): the right stem and
// layers 0-8 on the ping-pong walk engine (h16xw), layer 9 staged into the in-place tile's three
// planes, the corrected tail (layers 10-14) and the MFMA right head on the in-place walk engine
// (inplace.hpp WalkGeo, conv<..., WALK>), then the left branch and its head on the ping-pong engine,
// and the combine x - (r + l)/2.  Each layer's carry rows live in a slot behind the tile (128-B rows
// for the ping-pong layers' outputs, 256-B plane rows for the outputs the corrected layers and the
// right head read): 12,032 B.
//
// Range guard: tl.amax (the corrected layers' running max, inplace.hpp h8_track) is reset once per
// spectrum, not per tile, so the first tile whose activations saturate NaNs its own outputs and those
// of every later tile of the spectrum: the clamped values reach the next tile through its carry rows,
// so none of its outputs could be trusted (tests/test_range_gpu.py test_walk_saturation_nans_rest_of_
// spectrum).  The 640-row tiles, which carry nothing, NaN only the saturated tile.
//
// Spectra with an input outside [F16MIX_WIN_LO, F16MIX_WIN_HI] (a spike) take the tiled hybrid for
// every tile of the spectrum instead (rrcdnet_hybrid_tile: its per-tile spiked fallback corrects every
// layer of a spiked tile; the walk would need full-precision carries across such a tile's boundary):
// ~3 % of the simulator's spectra.

namespace hybw {
namespace PP = h16xw;
constexpr int WNBK = (RDN_WALK_ROWS_MIX + 127) / 128;    // in-place blocks (the last may be half)
using WG = WalkGeo<WNBK>;
static_assert(PP::WT == WG::WB && PP::CG == WG::GRD, "one walk tile, two engines");
constexpr int RIGHT_C0 = walk_shift(RRCDNET) - 16;   // the right stem's extra shift (both heads at 28)
constexpr int CARRY_BYTES = 9 * 2 * 128 + 6 * 2 * 256 + 52 * 128;   // layers 0-8 | 9-14 | left 15-28
static_assert(PP::CARRY_OFF + CARRY_BYTES <= 163840 - 64, "carry slots below the vote words");
static_assert(WG::LDS <= PP::CARRY_OFF, "the in-place tile inside the ping-pong buffers");

// layer 9's outputs, split in VGPRs into the in-place tile's planes (rrcdnet_hybrid.hpp H8Stage on the
// walk rows: r0 includes the carry rows in front)
struct H8Stage {
  f16x8 hi[PP::NT];
  uint32_t e_hi[PP::NT][2], e_lo[PP::NT][2];
  float amax = 0.f;
  __device__ __forceinline__ void put(int n, PP::f32x8 v, bool valid) {
    const PP::f32x8 t = valid ? v : (PP::f32x8)(0.f);
    h8_track<true>(amax, __builtin_shufflevector(t, t, 0, 1, 2, 3));
    h8_track<true>(amax, __builtin_shufflevector(t, t, 4, 5, 6, 7));
    const f32x4 a = h8_sat<true>(__builtin_shufflevector(v, v, 0, 1, 2, 3));
    const f32x4 b = h8_sat<true>(__builtin_shufflevector(v, v, 4, 5, 6, 7));
    const H8Split sa = h8_split(a), sb = h8_split(b);
    hi[n] = __builtin_shufflevector(sa.hi, sb.hi, 0, 1, 2, 3, 4, 5, 6, 7);
    e_hi[n][0] = sa.hi8;
    e_hi[n][1] = sb.hi8;
    e_lo[n][0] = sa.lo8;
    e_lo[n][1] = sb.lo8;
  }
  template <bool EDGE>
  __device__ __forceinline__ void write(char* lds, const PP::Tile& t) const {
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    const int tid = PP::tid(), w = tid >> 6, lane = tid & 63;
    const int g = 4 * (w / PP::RB) + (lane >> 4), r0 = PP::CG + PP::rblock(w) * PP::RW + (lane & 15);
#pragma unroll
    for (int n = 0; n < PP::NT; ++n) {
      const int r = r0 + 16 * n;
      const bool ok = !EDGE || in_range(t.base + r, t.L);
      *(f16x8*)(lds + off_f32(r, 16 * g)) = ok ? hi[n] : (f16x8)((_Float16)0);
      *(u32x2*)(lds + off_f32(r, 128 + 8 * g)) = ok ? u32x2{e_hi[n][0], e_hi[n][1]} : u32x2{0u, 0u};
      *(u32x2*)(lds + off_f32(r, 192 + 8 * g)) = ok ? u32x2{e_lo[n][0], e_lo[n][1]} : u32x2{0u, 0u};
    }
  }
};

// layer 9's carry rows of the in-place tile (plane rows CG - 2, CG - 1) from its slot (zeros on the
// spectrum's first tile); after the staged layer's barrier nothing reads the tile
__device__ __forceinline__ void stage_carry(char* lds, const PP::Tile& t) {
  typedef unsigned int u32x4c __attribute__((ext_vector_type(4)));
  const int tid = PP::tid(), lane = tid & 63;
  if (__builtin_amdgcn_readfirstlane(tid >> 6) == PP::WAVES - 1 && lane < 32) {
    const int k = lane >> 4, sl = lane & 15, pr = WG::GRD - 2 + k;
    const u32x4c v = t.first ? u32x4c{0u, 0u, 0u, 0u} : *(const u32x4c*)(lds + t.cs_prev + k * ROWB_F32 + 16 * sl);
    *(u32x4c*)(lds + pr * ROWB_F32 + ((sl ^ swz256(pr)) << 4)) = v;
  }
}

// Diagnostic builds (tools/hyb_stamps.py with RDN_WALK=1, -DRDN_HYB_STAMPS=1): phase stamps summed over
// each spectrum's tiles (hyb640::HybStamps, flushed once per spectrum); nothing in the product build
using Stamps = hyb640::HybStamps;

template <bool EDGE>
__device__ __forceinline__ void tile(Tile& tl, PP::Tile& t16, float* y, int t, int ntiles, PP::Frags& F0, PP::Frags& F1,
                                     PP::StemX& xs, unsigned* status, Stamps& st) {
  constexpr int TAIL = F16MIX_TAIL, PPL = 14 - TAIL;      // 9 plain right layers, layer 9 staged
  static_assert(PPL % 2 == 1, "the staged layer reads BUF1");
  using HO = HeadOut<MODE_H8, WNBK>;
  const int L = tl.L;
  f32x4 id[16 * WNBK / 4];
  LayerA<MODE_H8> a;
  // right branch: stem shifted by RIGHT_C0, layers 0-8
  PP::walk_start(t16, t, RIGHT_C0);
  PP::stem(t16, 0, PP::BUF0, xs);
  F0 = F1;
  PP::lds_barrier();
  st(0);
  for (int i = 0; i < PPL / 2; ++i) {
    PP::layer<PP::RELU, EDGE>(t16, PP::BUF0, PP::BUF1, 1, F0, F1);
    PP::layer<PP::RELU, EDGE>(t16, PP::BUF1, PP::BUF0, 1, F1, F0);
  }
  PP::layer<PP::RELU, EDGE>(t16, PP::BUF0, PP::BUF1, 1, F0, F1);
  st(1);
  {
    H8Stage stg;
    PP::layer<PP::STAGE, EDGE>(t16, PP::BUF1, PP::BUF0, 1, F1, F0, false, nullptr, nullptr, &stg);
#if RDN_STAGE_FIRST
    // A/B: the planes' LDS stores ahead of the tail's 26 operand loads per wave (whose issue waits on
    // the texture path), the loads k-step-outer so the first k-step's fragments arrive first
    stg.write<EDGE>(tl.lds, t16);
    stage_carry(tl.lds, t16);
    load_layer_a<MODE_H8, true>(tl, PPL + 1, a);
#else
    load_layer_a<MODE_H8>(tl, PPL + 1, a);
    stg.write<EDGE>(tl.lds, t16);
    stage_carry(tl.lds, t16);
#endif
    tl.amax = fmaxf(tl.amax, stg.amax);
  }
  // hand the walk state to the in-place tile: its logical row 0 is buffer row CG
  tl.base = t16.base + PP::CG;
  tl.cs_prev = t16.cs_prev;
  tl.dn_prev = 1;
  tl.cs_cur = t16.cs_cur;
  tl.dnext = 1;
  tl.first = t16.first;
  tl.layer = PPL + 1;
  lds_barrier();
  st(2);
  const uint8_t* rhead = tl.big + (size_t)F16MIX_RHEAD_REC * BIG_BYTES_H8;
  for (int i = 0; i < TAIL; ++i)
    conv<MODE_H8, RELU, 1, EDGE, WNBK, true, true, true, true>(tl, 1, id, a, true, i + 1 < TAIL ? nullptr : rhead);
  st(3);
  // the left branch's stem inputs and layer-15 operands, fetched before the right head: their latency
  // hides under its MFMAs (F0 is free since the staged layer)
  const PP::StemX xl = PP::walk_stem_load(t16, t, 0);
  t16.layer = 15;
  PP::load_frags(t16, 15, F0);
  float rk[HO::ROWS];
  head_h8_mfma<WNBK, true>(tl, a, rk);
  st(4);
  // left branch: layers 15-28 and the head on the ping-pong engine
  t16.cs_cur = tl.cs_cur;
  t16.dn_prev = 0;                      // the stem recomputes its carry rows
  t16.base = t * PP::WT - PP::CG;
  PP::lds_barrier();                    // the left stem overwrites the rows the right head read
  PP::stem(t16, 1, PP::BUF0, xl);
  PP::lds_barrier();
  st(5);
  for (int i = 0; i < 7; ++i) {        // left layer j has d = 1 at j = 7, else 2; the head reads with d = 1
    t16.dnext = 2 * i + 1 == 7 ? 1 : 2;
    PP::layer<PP::RELU, EDGE>(t16, PP::BUF0, PP::BUF1, 2, F0, F1);
    t16.dnext = i == 6 ? 1 : 2;
    PP::layer<PP::RELU, EDGE>(t16, PP::BUF1, PP::BUF0, 2 * i + 1 == 7 ? 1 : 2, F1, F0);
  }
  st(6);
  float xv[HO::ROWS];
#pragma unroll
  for (int k = 0; k < HO::ROWS; ++k) {  // the combine's x, fetched before the left head
    const int p = tl.base + HO::row(k);
    xv[k] = in_range(p, L) ? tl.x[p] : 0.f;
  }
  // the next tile's stem inputs and layer-0 operands, fetched unconditionally (past the last tile:
  // harmless reads), so neither xs nor F1 stays live across a tile for the loop's last iteration
  xs = PP::walk_stem_load(t16, t + 1, RIGHT_C0);
  float l[PP::HN];
  PP::head<EDGE>(t16, PP::BUF0, F0, F1, true, l, 0);
  st(7);
  // the left head's rows to the right head's lanes through LDS (BUF1, unread since layer 28's
  // barrier); the tail's range vote rides on the same barrier
  float* lrow = (float*)(tl.lds + PP::BUF1);
  if ((PP::tid() & 63) < PP::HEAD_LANES) {
#pragma unroll
    for (int k = 0; k < PP::HN; ++k) {
      const int j = PP::head_row(k);
      if (j < PP::WB) lrow[j] = l[k];
    }
  }
  range_vote_post(tl, PP::BUF1 + 4 * PP::WB);
  PP::lds_barrier();
  const bool sat = range_vote_read(tl, PP::BUF1 + 4 * PP::WB, status);
  float o[HO::ROWS];
#pragma unroll
  for (int k = 0; k < HO::ROWS; ++k)        // x - (r + l)/2, one rounding
    o[k] = (float)((double)xv[k] - ((double)rk[k] + (double)lrow[min(PP::CG + HO::row(k), PP::WB - 1)]) * 0.5);
  if (sat) nan_rows(o);
  if (HO::writer()) {
#pragma unroll
    for (int k = 0; k < HO::ROWS; ++k) {
      const int p = tl.base + HO::row(k);
      if (HO::row(k) < WG::WB && in_range(p, L)) y[p] = o[k];
    }
  }
  PP::lds_barrier();                    // the next tile's stem and layers overwrite BUF0 / BUF1
  st(8);
}

}  // namespace hybw
