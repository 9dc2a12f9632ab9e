// Whole-network fused tile kernels for the single-rounding 16-bit modes: RDN_F16 (this file compiled
// with RDN_H16_F16=1, fused16_f16.hip: v_mfma_f32_16x16x32_f16, f16 weights and activations -- the
// headline mode, within the 2e-2 bar on every golden fixture) and RDN_BF16 ('bf16-unsafe':
// v_mfma_f32_16x16x32_bf16, bf16 -- NOT within 2e-2 on trained weights).  fp32 accumulation in both.
// The two instantiations share every line below; only the element type, the MFMA and the namespace
// (h16 / h16f, so rocprof tells them apart) differ.
//
// Geometry.  One workgroup = one tile of WB = 640 consecutive positions of one spectrum (its T
// output positions plus a halo on each side).  LDS holds two ping-pong activation buffers of
// 640 rows x 128 B (64 channels x bf16) = the CU's whole 160 KiB.  There are no guard rows: a tap
// that falls off one end of the tile wraps to the other end.  Those rows lie outside every
// output's receptive field (the halo covers the full depth of the stack), so any finite value
// serves; positions outside [0, L) of the spectrum itself are re-zeroed by every epilogue — the
// zero padding each reference Conv1d applies.
//
// Each Conv1d(64,64,3,d) is an implicit GEMM  Y[64 cout][640 pos] = W[64][192] . X~[192][640]
// whose B operand is read straight from the activation buffer at row offsets (t-1)*d (no
// im2col).  Wave w owns row block w % 4 (RW = 160 rows, NT = 10 N-tiles; walk: rblock) and output channels
// 32h .. 32h+31 (h = w / 4: two M-tiles), so the two waves of a SIMD (w, w + 4) split the output
// channels of the same rows.  The split halves the weights a wave holds (12 A-fragments, 12 KB per
// layer, loaded from L2/L1 by every wave: 96 KB per CU per layer instead of 192 KB -- the vector
// memory path, not the MFMA, bounded the all-channels-per-wave layout) at the price of twice the
// LDS B reads (480 KB per CU per layer at 256 B/clk: half the MFMA time).  The layer's
// operands are double-buffered (two Frags, the network bodies alternate them): the next layer's
// 14 loads are spread one per 4 steps, so the vector-memory traffic of the CU's
// 8 waves is smooth instead of a burst at the layer's end.  N-tiles are the outer loop, so each
// N-tile's ReLU (+ residual), rounding and ds_write_b128 run one N-tile behind the MFMAs, spread
// over the layer (a k-step-outer loop bunched all of them, issue-bound, into its last sixth).
// Accumulators start at the folded bias.  One LDS barrier per layer.
//
// Channel order inside an LDS row (= K order of the packed A-fragments, csrc/pack.cpp): 16-B slot
// g = 4u + q holds channels h16_channel(g, j) = 32u + 4q + (j & 3) + 16 (j >> 2), j = 0..7 — the
// 8 output channels lane quarter q of M-tiles 2u and 2u+1 holds after an MFMA (C/D map) AND the 8
// K-elements lane quarter q of k-step (t, u) feeds in (B map).  Slots are XOR-swizzled by
// (row & 7): B reads (ds_read_b128) and epilogue writes (ds_write_b128) are bank-conflict-free.
//
// Reference forwards: 1DCNN/train.py:71-82, RRCDNet/train.py:72-98, DSDN/train.py:72-126,
// PIDN/train.py:72-106.
#include "common.hpp"
#include "host_util.hpp"

#ifndef RDN_H16_F16
#define RDN_H16_F16 0
#endif
#ifndef H16_NS
#if RDN_H16_F16
#define H16_NS h16f
#define H16_LAUNCH launch_fused16_f16
#define H16_ATTR_SLOT0 56
#else
#define H16_NS h16
#define H16_LAUNCH launch_fused16
#define H16_ATTR_SLOT0 0
#endif
#endif
// big-layer stride and bias offset of the blob this instantiation reads: the fused16 layout
// (BIG_BYTES_BF16, common.hpp) or, for the f16 layers of RDN_F16MIX (fused_inplace.hip), the
// f16 + e4m3 layout, whose leading f16 fragment section has the same [m 4][kstep 6][lane 64][8] map
#ifndef H16_LAYER_BYTES
#define H16_LAYER_BYTES BIG_BYTES_BF16
#define H16_BIAS_OFF BIG_FRAG_BYTES_BF16
#endif

namespace rdn {
namespace H16_NS {

#if defined(H16_WALK_T)
// Walk instantiation (fused16_walk.hip): one workgroup walks a spectrum's tiles left to right and
// every executed MFMA row is an output row.  Layer l of a tile computes WT rows at positions shifted
// left by its cumulative dilation c_l (row r <-> position tile_base + r - CG - c_l), so its taps read
// rows r - 2d, r - d, r of the previous layer's buffer; the CG rows in front of the computed rows
// carry the previous tile's last 2d rows of that layer (copied through a per-layer carry slot,
// layer_carry).  No halo is recomputed and the workgroup's start is paid once per spectrum.
constexpr bool WALK = true;
constexpr int WT = H16_WALK_T;                        // positions a layer advances per tile
constexpr int CG = 4;                                  // carry rows in front of the computed rows (2 d_max)
constexpr int WB = CG + WT;                            // buffer rows
constexpr int CARRY_ROWS = 88;                        // sum of 2 d over the 64-channel readers (RRCDNet: 88)
#else
constexpr bool WALK = false;
constexpr int CG = 0;
#ifdef H16_TILE_ROWS
constexpr int WB = H16_TILE_ROWS;                     // latency instantiation (fused16_small.hip): short tiles
#else
constexpr int WB = H16_WB;                            // 640 rows per tile, halo included
#endif
constexpr int WT = WB;                                // rows a layer computes
constexpr int CARRY_ROWS = 0;
#endif
constexpr int ROWB = 128;                             // 64 channels x 16 bit
constexpr uint32_t BUF_BYTES = WB * ROWB;             // 81920
constexpr uint32_t BUF0 = 0, BUF1 = BUF_BYTES;
constexpr uint32_t CARRY_OFF = 2 * BUF_BYTES;         // walk: the layers' carry slots
constexpr uint32_t LDS_BYTES = CARRY_OFF + CARRY_ROWS * ROWB;   // 163840 (640 rows): the whole LDS of a CU
static_assert(LDS_BYTES <= 163840, "LDS of one CU");
constexpr int LAYER_BYTES = H16_LAYER_BYTES;          // [m 4][k-step 6][lane 64][8 x 16 bit] ... bias[64] f32
constexpr int BIAS_OFF = H16_BIAS_OFF;
#ifndef RDN_H16_PF
#define RDN_H16_PF 3
#endif
#ifndef RDN_H16_ESPLIT
#define RDN_H16_ESPLIT 0
#endif
#ifndef RDN_PRIO_SWITCH
// Ping-pong layers: the two waves of a SIMD (w, w + 4: the two channel halves) share its MFMA pipe, and
// at equal priority the arbiter favours the older wave, so waves 0-3 finish a layer's MFMA stream ~1k
// cycles before waves 4-7, which then run it alone (one wave per SIMD) up to the barrier
// (tools/hyb_stamps.py, per-wave layer stamps).  RDN_PRIO_SWITCH = k > 0: waves 4-7 raise their
// priority when they reach N-tile k of a layer (and drop it at the next layer's start), so that both
// waves of a SIMD reach the barrier together
#define RDN_PRIO_SWITCH 0
#endif
#ifndef RDN_H16_SGB
#define RDN_H16_SGB 0
#endif
// A tile holding positions outside [0, L) stores its layer outputs unmasked (the MFMA loop is the
// interior tiles' own) and each wave then zeroes its rows outside [0, L) -- a few stores after the
// loop, before the barrier (zero_outside; a per-lane range check and select in every epilogue made
// the edge tiles ~10 % slower, and the CBAM team kernel waits for them).  The 32x32x16 MFMA form
// measured 5 % slower (same MFMA busy, lower clock) and is not built.
constexpr int WAVES = 8;
constexpr int THREADS = 64 * WAVES;
constexpr int MH = 2;                                 // output-channel halves (32 channels each)
constexpr int RB = WAVES / MH;                        // row blocks
constexpr int RW = WT / RB;                           // 160 rows per wave
constexpr int NR = 16;
constexpr int KS = 6;                                 // 3 taps x 2 x 32 channels
constexpr int NFRAG = 12;                             // 2 M-tiles x 6 k-steps
constexpr int NBIAS = 2;
constexpr int HEAD_LANES = 16;
constexpr int NT = RW / NR;                           // N-tiles per wave (10 / 5)
constexpr int HN = (NT + MH - 1) / MH;                // head N-tiles per wave (the two halves split the rows)
static_assert(RW % NR == 0, "rows per wave must be whole N-tiles");
static_assert(WALK || (WB % 64) == 0, "stem rows lane + 64k cover the tile");

typedef float f32x8 __attribute__((ext_vector_type(8)));
#if RDN_H16_F16
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
typedef f16x8_t V;
typedef _Float16 E;
__device__ __forceinline__ f32x4 mma(V a, V b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0); }
#else
typedef bf16x8 V;
typedef __bf16 E;
__device__ __forceinline__ f32x4 mma(V a, V b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }
#endif
// Thread index the compiler cannot treat as loop-invariant (per-lane addresses are recomputed where
// they are used instead of being hoisted across the network's layers and spilled)
__device__ __forceinline__ int tid() {
  int t = __builtin_amdgcn_workitem_id_x();
  asm volatile("" : "+v"(t));
  return t;
}
__device__ __forceinline__ int soff(int row, int slot) { return row * ROWB + ((slot ^ (row & 7)) << 4); }
__device__ __forceinline__ int wrap(int row) { return row < 0 ? row + WB : (row >= WB ? row - WB : row); }
__device__ __forceinline__ bool in_range(int p, int L) { return (unsigned)p < (unsigned)L; }
// LDS-only workgroup barrier: this wave's LDS traffic drains, its global loads (next layer's
// weights) stay in flight.  One asm statement, so no memory access moves across it.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

struct Tile {
  char* lds;
  const float* x;        // this spectrum
  int L;
  int base;              // spectrum position of tile row 0
  const float* small;    // small section of the blob
  const uint8_t* big;    // big-layer section
  __amdgpu_buffer_rsrc_t wrsrc;   // buffer resource over the big-layer section (scalar-offset loads)
  int layer;             // big layer whose fragments are in VGPRs
  // per-lane LDS offsets, computed once per tile (no address arithmetic at each layer's start):
  // koff[d + 2][u] = soff(r0 + d, 4u + q) for tap shift d in -2..2 (no wrap), r0 = this lane's
  // first row (rblock(w) * RW + lane % 16); walk: koff[d + 4][u] for d in -4..0, r0 = CG + ...
  int koff[5][KS / 3];
  int r0;
  // walk only (layer_carry): the carry slot of the layer being computed (its last 2 dnext rows, for
  // the next tile), the previous layer's slot and row count (0: none, the stem recomputes its rows),
  // the dilation of the layer that reads this one, and whether this is the spectrum's first tile
  int cs_cur, cs_prev, dn_prev, dnext;
  bool first;
  unsigned* status;      // the launch's status word (input gate, STATUS_GATE) or NULL
#if defined(RDN_HYB_STAMPS) && RDN_HYB_STAMPS
  // diagnostic (tools/hyb_stamps.py): the walk's ReLU layers, wave 0's view -- entry to the first MFMA
  // issue (fill), to the last MFMA issue, to the last epilogue's store, to past the barrier; layers
  unsigned long long lst[5];
#endif
};

struct Frags {            // one layer's operands in VGPRs: this wave's A-fragments and folded bias
  V a[NFRAG];             // [M-tile 2][k-step 6]
  f32x4 bias[NBIAS];
};
// this wave's output-channel half (channels 32h .. 32h + 31), wave-uniform
__device__ __forceinline__ int mhalf() { return __builtin_amdgcn_readfirstlane(tid() >> 6) / RB; }
// the row block of wave w (channel half w / RB).  Tiles: w % RB.  Walk: the second half's row blocks
// are rotated by two, so the two waves a SIMD holds (w and w + 4: a workgroup's waves go to its
// SIMDs cyclically, MI355X_MICROARCH.md §LDS) own row blocks two apart -- on a spectrum's short last
// tile, whose upper row blocks lie beyond L and skip their MFMAs, every SIMD keeps one busy wave
// instead of two SIMDs carrying both waves of the live row blocks
static_assert(!WALK || (RB == 4 && MH == 2), "the walk's row-block rotation is written for 4 x 2 waves");
__device__ __forceinline__ int rblock(int w) { return WALK ? (w + 2 * (w / RB)) % RB : w % RB; }

// Operand loads as raw buffer loads: lane offset in a VGPR, layer/fragment offset in an SGPR, so
// the loads of a layer cost no address VALU.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
struct LaneOff {          // this lane's byte offsets of the A-fragment and bias loads
  int a, b;
};
// One opaque tid() per layer, not one per load.  The blob's fragments are 16x16x32 A-operands,
// fragment (m, s = 2t + u) lane r + 16q = W[16m + r][slot 4u + q of tap t] (pack.cpp).
__device__ __forceinline__ LaneOff lane_off() {
  const int lane = tid() & 63;
  return {lane * 16, (lane >> 4) * 16};
}
// operand i of half h of big layer `layer`, in the order of first use: the two bias vectors (the
// accumulators' start at k-step 0), then the A-fragments by k-step, both M-tiles of a step together.
// The loads are counted in order (vmcnt), so the operands issued last -- those of k-step 5 -- are the
// ones the next layer needs last (bias last: the next layer's first MFMA waited on the load issued
// two steps before the barrier).
__device__ __forceinline__ void load_op(const Tile& tl, int layer, int h, int i, const LaneOff& lo, Frags& F) {
  const int base = layer * LAYER_BYTES;
  if (i < NBIAS) {
    const int so = base + BIAS_OFF + 64 * (2 * h + i);
    F.bias[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(tl.wrsrc, lo.b, so, 0));
  } else {
    const int f = i - NBIAS, m = f & 1, s = f >> 1;
    const int so = base + ((2 * h + m) * 6 + s) * 1024;
    F.a[m * 6 + s] = __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b128(tl.wrsrc, lo.a, so, 0));
  }
}
constexpr int NLOAD = NFRAG + NBIAS;

__device__ __forceinline__ void load_frags(const Tile& tl, int layer, Frags& F) {
  const LaneOff lo = lane_off();
  const int h = mhalf();
#pragma unroll
  for (int i = 0; i < NLOAD; ++i) load_op(tl, layer, h, i, lo, F);
}

// Accumulators of one N-tile: M-tiles 2h, 2h + 1 (16 channels x 16 positions each), started at the
// folded bias.
struct Acc {
  f32x4 v[2];
};
__device__ __forceinline__ void mstep(const Frags& F, int s, V b, Acc& acc) {
#pragma unroll
  for (int m = 0; m < 2; ++m) {
#if defined(RDN_ABLATE_NOMFMA)
    if (s == 0) acc.v[m] = F.bias[m];
    asm volatile("" : "+v"(acc.v[m]) : "v"(F.a[m * 6 + s]), "v"(b));
#else
    acc.v[m] = mma(F.a[m * 6 + s], b, s == 0 ? F.bias[m] : acc.v[m]);
#endif
  }
}

// Conv1d(1, 64, 3, padding=1) (+ folded BN) + ReLU in fp32, one (row, 16-B slot) item per lane
// and step.  ACCUM adds the result onto the resident row (PIDN/train.py:105, identity recomputed
// from x).  out_lo / out_hi (lo <= hi): returns whether any input this thread read at the tile's
// rows lies outside [lo, hi] (the RDN_F16MIX spiked-tile test, rrcdnet_hybrid.hpp), else false.
// Wave w computes slot w (8 channels, its 32 weights scalar-loaded once) for rows lane + 64k, and
// every x value of those rows is fetched before the first is used (buffer loads: positions outside
// [0, L) read 0 by the range check of the resource) -- one memory latency per stem (a loop of one
// (row, slot) item per lane and step waited on its loads ten times: 7 % of the RDN_F16MIX hybrid,
// which runs two stems per tile); channel pairs on v_pk_fma_f32 and a packed ReLU after the rounding
// (without ACCUM).
// The stem's x values: rows lane + 64k by buffer loads (positions outside [0, L) read 0 by the range
// check of the resource), plus the two positions just outside the tile's rows; the taps -1 / +1 come
// from the neighbouring lanes (DPP wave shifts) in stem, so a lane issues NK + 2 loads instead of
// 3 NK (every wave fetches the whole tile's x: one load per row, not three).  A caller may issue them
// early (stem_load) and hand them to the stem later, so their latency hides under other work (the
// RDN_F16MIX hybrid fetches its left stem's inputs before the right head).
constexpr int STEM_NK = (WB + 63) / 64;
struct StemX {
  float x0[STEM_NK];
  float xe0, xe1;               // positions base - 1 and base + 64 STEM_NK
};
__device__ __forceinline__ StemX stem_load(const Tile& tl) {
  StemX s;
  const int lane = tid() & 63;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)tl.x, 0, tl.L * 4, 0x00020000);
#pragma unroll
  for (int k = 0; k < STEM_NK; ++k)
    s.x0[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, 4 * (tl.base + lane + 64 * k), 0, 0));
  s.xe0 = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, 4 * (tl.base - 1), 0, 0));
  s.xe1 = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, 4 * (tl.base + 64 * STEM_NK), 0, 0));
  return s;
}
// x at row lane + 64k - 1 / + 1: the wave shifted by one lane, the vacated lane from the
// neighbouring 64-row chunk (or the position outside the tile's rows)
__device__ __forceinline__ float stem_xm(const StemX& s, int k) {
  const float prev = k == 0 ? s.xe0 : __int_as_float(__builtin_amdgcn_readlane(__float_as_int(s.x0[k - 1]), 63));
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(prev), __float_as_int(s.x0[k]), 0x138, 0xf, 0xf, false));
}
__device__ __forceinline__ float stem_xp(const StemX& s, int k) {
  const float next = k == STEM_NK - 1 ? s.xe1 : __int_as_float(__builtin_amdgcn_readlane(__float_as_int(s.x0[k + 1]), 0));
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(next), __float_as_int(s.x0[k]), 0x130, 0xf, 0xf, false));
}

// Conv1d(1, 64, 3, padding=1) (+ folded BN) + ReLU in fp32.  ACCUM adds the result onto the resident
// row (PIDN/train.py:105, identity recomputed from x).  out_lo / out_hi (lo <= hi): returns whether any
// input this thread read at the tile's rows lies outside [lo, hi] (the RDN_F16MIX spiked-tile test,
// rrcdnet_hybrid.hpp), else false.
// Wave w computes slot w (8 channels, its 32 weights scalar-loaded once) for rows lane + 64k, and
// every x value of those rows is fetched before the first is used -- one memory latency per stem (a
// loop of one (row, slot) item per lane and step waited on its loads ten times: 7 % of the RDN_F16MIX
// hybrid, which runs two stems per tile); channel pairs on v_pk_fma_f32 and a packed ReLU after the
// rounding (without ACCUM).
template <bool ACCUM = false>
__device__ __forceinline__ bool stem(const Tile& tl, int sslot, uint32_t dst, const StemX& xs, float out_lo = 1.f,
                                     float out_hi = 0.f) {
  const float* swp = tl.small + sslot * SMALL_SLOT_FLOATS;
  asm volatile("" : "+s"(swp));      // no reuse of scalar-loaded weights across the layers in between
  const cfloat* sw = (const cfloat*)swp;
  bool outside = false;
#if defined(RDN_ABLATE_NOSTEM)         // diagnostic (tools/ablate.py): the stem's cost, wrong results
  return outside;
#endif
  static_assert(WAVES == 8, "one slot per wave, rows lane + 64k");
  constexpr int NK = STEM_NK;
  const int g = __builtin_amdgcn_readfirstlane(tid() >> 6), lane = tid() & 63;
  float wb[8], wm[8], w0[8], wp[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = h16_channel(g, j);
    wb[j] = sw[192 + c];
    wm[j] = sw[3 * c + 0];
    w0[j] = sw[3 * c + 1];
    wp[j] = sw[3 * c + 2];
  }
  bool over = false;              // an input beyond the 16-bit modes' domain (STATUS_GATE)
#pragma unroll
  for (int k = 0; k < NK; ++k) over = over || fabsf(xs.x0[k]) > INPUT_GATE;
  // every wave reads all the tile's x: wave 0 reports
  if (tl.status && g == 0 && __builtin_amdgcn_ballot_w64(over) != 0 && lane == 0) raise_status(tl.status, STATUS_GATE);
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int row = lane + 64 * k;
    const int p = tl.base + row;
    const bool valid = in_range(p, tl.L);
    if (out_lo <= out_hi) outside = outside || xs.x0[k] < out_lo || xs.x0[k] > out_hi;
    const float xmk = stem_xm(xs, k), xpk = stem_xp(xs, k);
    // walk: rows beyond the buffer are not stored; ACCUM skips the carry rows in front (they hold the
    // previous tile's rows, identity already added)
    if (WALK && (row >= WB || (ACCUM && row < CG))) continue;
    V* ptr = (V*)(tl.lds + dst + soff(row, g));
    V v;
    if (!ACCUM) {
      // channel pairs by v_pk_fma_f32 (each half one fmaf, same order), ReLU after the rounding
      // (rounding is monotone and keeps 0: the same value), rows outside [0, L) zeroed last
      typedef float f32x2 __attribute__((ext_vector_type(2)));
      const f32x2 xm2 = {xmk, xmk}, x02 = {xs.x0[k], xs.x0[k]}, xp2 = {xpk, xpk};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        f32x2 a = {wb[2 * q], wb[2 * q + 1]};
        a = __builtin_elementwise_fma(f32x2{wm[2 * q], wm[2 * q + 1]}, xm2, a);
        a = __builtin_elementwise_fma(f32x2{w0[2 * q], w0[2 * q + 1]}, x02, a);
        a = __builtin_elementwise_fma(f32x2{wp[2 * q], wp[2 * q + 1]}, xp2, a);
        v[2 * q] = (E)a[0];
        v[2 * q + 1] = (E)a[1];
      }
      v = __builtin_elementwise_max(v, (V)((E)0.f));
      if (!valid) v = (V)((E)0.f);
      *ptr = v;
      continue;
    }
    v = *ptr;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float a = wb[j];
      a = fmaf(wm[j], xmk, a);
      a = fmaf(w0[j], xs.x0[k], a);
      a = fmaf(wp[j], xpk, a);
      a = fmaxf(a, 0.f);
      a += (float)v[j];
      v[j] = (E)(valid ? a : 0.f);
    }
    *ptr = v;
  }
  return outside;
}
template <bool ACCUM = false>
__device__ __forceinline__ bool stem(const Tile& tl, int sslot, uint32_t dst, float out_lo = 1.f, float out_hi = 0.f) {
  return stem<ACCUM>(tl, sslot, dst, stem_load(tl), out_lo, out_hi);
}

enum Epi : int {
  RELU = 0,       // relu(acc + b)
  LINEAR = 1,     // acc + b                (PIDN block output: BN without ReLU)
  RES_RELU = 2,   // relu(acc + b + dst)    (DSDN ResidualBlock: out += identity; relu)
  LINEAR_SAVE = 3,  // acc + b, the dst slot's previous content saved to idv[n] first (the CBAM
                    // networks' ResidualBlock identity, held in VGPRs across the CBAM: cbam.hip)
  STAGE = 4,        // acc + b handed to stg->put(n, v) (VGPRs) instead of stored: the caller writes
                    // the layer's output after the barrier, in another LDS layout (RDN_F16MIX hybrid)
};

// LDS byte addresses of this lane's B fragment for k-step s = (tap t, part u) of N-tile n, from
// the tile's per-lane offsets: a tap shift keeps the swizzle of a 640-row wrap (640 = 0 mod 16),
// so the wrapped taps of the first / last wave (only (n = 0, t = 0) and (n = NT-1, t = 2) can leave
// the tile) are the unwrapped offset -/+ one buffer.
struct BAddr {
  static constexpr int U = KS / 3;      // k-steps per tap
  int m[KS], first[U], last[U];
  __device__ __forceinline__ BAddr(const Tile& tl, uint32_t src, int dil) {
    const bool d1 = dil == 1;
    if constexpr (WALK) {     // taps at rows r - 2d, r - d, r; the carry rows in front: no wrap
#pragma unroll
      for (int u = 0; u < U; ++u) {
        m[u] = (int)src + (d1 ? tl.koff[2][u] : tl.koff[0][u]);
        m[U + u] = (int)src + (d1 ? tl.koff[3][u] : tl.koff[2][u]);
        m[2 * U + u] = (int)src + tl.koff[4][u];
        first[u] = last[u] = 0;
      }
      return;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      m[u] = (int)src + (d1 ? tl.koff[1][u] : tl.koff[0][u]);
      m[U + u] = (int)src + tl.koff[2][u];
      m[2 * U + u] = (int)src + (d1 ? tl.koff[3][u] : tl.koff[4][u]);
    }
    const bool wl = tl.r0 < dil, wh = tl.r0 + NR * (NT - 1) + dil >= WB;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      first[u] = m[u] + (wl ? (int)BUF_BYTES : 0);
      last[u] = m[2 * U + u] + NR * (NT - 1) * ROWB - (wh ? (int)BUF_BYTES : 0);
    }
  }
  __device__ __forceinline__ int at(int n, int s) const {
    const int t = s / U, u = s % U;
    if (WALK) return m[s] + n * NR * ROWB;
    if (n == 0 && t == 0) return first[u];
    if (n == NT - 1 && t == 2) return last[u];
    return m[s] + n * NR * ROWB;
  }
};

// steps between two of the next layer's operand loads: 4 on the 640-row tile (16x16x32: 3 is
// -0.5 %, 2 is -2 %), as many as fit otherwise
#ifndef RDN_H16_LDSTEP
#define RDN_H16_LDSTEP 4
#endif
constexpr int LDSTEP = (KS * NT - 1) / (NLOAD - 1) < RDN_H16_LDSTEP ? (KS * NT - 1) / (NLOAD - 1) : RDN_H16_LDSTEP;
static_assert(LDSTEP >= 1 && LDSTEP * (NLOAD - 1) < KS * NT, "every operand load of the next layer must be issued");

// One Conv1d(64, 64, 3, dilation=dil, padding=dil) over the tile, src -> dst: this wave's 32
// output channels x NT N-tiles from the operands in F, while the next layer's operands stream into
// G (header).
// Per-channel sum / max of a layer's output over tile rows [lo, hi), accumulated in its epilogue
// from the unrounded fp32 values: this lane's 8 channels (slot 4h + q) over its rows (the CBAM
// channel statistics of the conv that produces u, cbam.hip team16_forward)
struct ChanStats {
  f32x8 sum, max;
  int lo, hi;
};

// Rows of this wave's block [r0, r0 + RW) at spectrum positions outside [0, L): its channel half
// (slots 4h .. 4h + 3) set to zero (the Conv1d zero padding of the next layer's input)
__device__ __forceinline__ void zero_outside(const Tile& tl, uint32_t dst, int r0, int h, int lane) {
  const int front = min(RW, max(0, -tl.base - r0));                 // rows at positions < 0
  const int back = max(front, min(RW, tl.L - tl.base - r0));       // first row at a position >= L
  const int nb = front + (RW - back);
  for (int i = lane; i < 4 * nb; i += 64) {
    const int k = i >> 2, r = r0 + (k < front ? k : back + (k - front));
    *(V*)(tl.lds + dst + soff(r, 4 * h + (i & 3))) = (V)((E)0);
  }
}

// Walk: the carry rows of the layer being computed and the previous layer's carry slot.  The waves
// of the last row block (each its channel half) (a) fill dst rows [CG - 2 dnext, CG), which the next
// layer's taps of its first rows read, from this layer's slot, written by the previous tile (zeros
// on the spectrum's first tile: positions < 0), and (b) save the last 2 dn_prev rows of src, the
// previous layer's output, which this layer only reads, into that layer's slot for the next tile.
// No wave reads dst rows [0, CG) during this layer and none writes src: no barrier of their own.
// Split in two so that the loads' latency hides under the layer's first N-tile: carry_load before
// the MFMA loop, carry_store after its first N-tile (then the slot bookkeeping).
struct Carry {
  V a, b;               // (a): the value for dst's carry row; (b): src's last row for the slot
};
__device__ __forceinline__ Carry carry_load(const Tile& tl, uint32_t src, bool has_dst) {
  Carry c;
  const int w = __builtin_amdgcn_readfirstlane(tid() >> 6), lane = tid() & 63;
  if (rblock(w) == RB - 1) {
    const int k = lane >> 2, g = 4 * (w / RB) + (lane & 3);
    if (has_dst && k < 2 * tl.dnext)
      c.a = tl.first ? (V)((E)0) : *(const V*)(tl.lds + tl.cs_cur + k * ROWB + 16 * g);
    if (k < 2 * tl.dn_prev) c.b = *(const V*)(tl.lds + src + soff(CG + WT - 2 * tl.dn_prev + k, g));
  }
  return c;
}
// rowb: bytes per carry row of this layer's slot (the staged layer's outputs are 256-B plane rows)
__device__ __forceinline__ void carry_store(Tile& tl, uint32_t dst, bool has_dst, const Carry& c, int rowb = ROWB) {
  const int w = __builtin_amdgcn_readfirstlane(tid() >> 6), lane = tid() & 63;
  if (rblock(w) == RB - 1) {
    const int k = lane >> 2, g = 4 * (w / RB) + (lane & 3);
    if (has_dst && k < 2 * tl.dnext) *(V*)(tl.lds + dst + soff(CG - 2 * tl.dnext + k, g)) = c.a;
    if (k < 2 * tl.dn_prev) *(V*)(tl.lds + tl.cs_prev + k * ROWB + 16 * g) = c.b;
  }
  tl.cs_prev = tl.cs_cur;
  tl.dn_prev = tl.dnext;
  tl.cs_cur += 2 * tl.dnext * rowb;
}

struct NoStage {
  __device__ void put(int, f32x8, bool) {}
};
template <int EPI, bool EDGE, class SG = NoStage>
__device__ __forceinline__ void layer(Tile& tl, uint32_t src, uint32_t dst, int dil, const Frags& F, Frags& G,
                                      bool has_next = true, V* idv = nullptr, ChanStats* cs = nullptr,
                                      SG* stg = nullptr, V* walk_id = nullptr) {
  const int lane = tid() & 63, w = __builtin_amdgcn_readfirstlane(tid() >> 6), h = w / RB;
  const int next = tl.layer + 1;
  asm volatile("" : "+s"(src), "+s"(dst));   // per-layer addresses: not hoisted out of a network's loop (spills)
  const BAddr ba(tl, src, dil);
  // (a) not for STAGE: its outputs go to the in-place tile, whose carry rows the caller fills
  // (rrcdnet_hybrid_walk.hpp stage_carry) from a slot of 256-B plane rows
  constexpr bool CA = EPI != STAGE;
  constexpr int CROW = EPI == STAGE ? 2 * ROWB : ROWB;
  Carry cc;
  if constexpr (WALK) {
    tl.base -= dil;                          // this layer's outputs: positions shifted by its dilation
    cc = carry_load(tl, src, CA);
  }
  const int pos0 = tl.base + CG + rblock(w) * RW;
#if RDN_PRIO_SWITCH
  if (h) __builtin_amdgcn_s_setprio(0);
#endif

  // Idle waves of a short last tile: every row of this wave lies at position >= L + 2, beyond the
  // reach (d <= 2) of any row that matters, so it skips the layer's MFMAs and only zeroes its dst
  // rows.  Left unwritten they would hold whatever an earlier workgroup left in the LDS, and the
  // wrapped taps of rows 0, 1 read them: that stays in the halo, but it made the halo rows of the
  // 256-row hybrid arbitrarily large, which the range guard of its staged layer and corrected tail
  // then saw (a false RDN_ERANGE after a saturating launch on the same CUs).  Its SIMD partner wave
  // has the MFMA pipe to itself; it still fetches the next layer's operands and meets the barrier.
  // (walk: every row at a position >= L is zero, the same rule without the halo's reach)
  if (EDGE && pos0 >= tl.L + (WALK ? 0 : 2)) {
    if constexpr (WALK) carry_store(tl, dst, CA, cc, CROW);
    if constexpr (EPI != STAGE) zero_outside(tl, dst, pos0 - tl.base, h, lane);
    if (WALK && walk_id) *walk_id = *(const V*)(tl.lds + src + (h ? tl.koff[2][1] : tl.koff[2][0]));
    if (has_next) load_frags(tl, next, G);
    if constexpr (EPI == LINEAR_SAVE) {
#pragma unroll
      for (int n = 0; n < NT; ++n) idv[n] = (V)((E)0);
    }
    tl.layer += 1;
    lds_barrier();
    return;
  }
  const LaneOff lo = lane_off();

  // bias (+ identity), ReLU, zero rows outside [0, L), round, store 8 channels as one 16-B slot
  // Walk RES_RELU (DSDN's second block conv, in place over the block input): the identity of output
  // row r is block-input row r - 2 (the input is two layers less shifted), which the epilogue of the
  // N-tile before may already have overwritten: each N-tile's identity is read at its first k-step,
  // ahead of that epilogue in this wave's LDS order, and N-tile 0's -- two rows of the previous row
  // block, or the carry rows that layer_carry (a) rewrites -- by the layer before, ahead of its
  // closing barrier (walk_id)
  V idn[2];
  const int sid = (int)dst + (h ? tl.koff[2][1] : tl.koff[2][0]);   // walk: row r0 - 2 of the block input
  auto store_slot = [&](V* p, f32x8 v, bool valid, int n) {
    if constexpr (EPI == RES_RELU) {
      if constexpr (WALK) v += __builtin_convertvector(n == 0 ? *walk_id : idn[n & 1], f32x8);
      else v += __builtin_convertvector(*p, f32x8);
    }
#if RDN_H16_F16
    // ReLU after the rounding, on packed f16 (4 v_pk_max_f16 instead of 8 v_max_f32; the rounding is
    // monotone, so max(f16(v), 0) = f16(max(v, 0)) up to the sign of a zero)
    V hv = __builtin_convertvector(v, V);
    if (EPI != LINEAR && EPI != LINEAR_SAVE) hv = __builtin_elementwise_max(hv, (V)((E)0));
    if (EDGE && !valid) hv = (V)((E)0);
#if defined(RDN_ABLATE_NOSTORE)            // diagnostic builds only (tools/ablate.py)
    if (hv[0] == (E)1234.f)
#endif
    *p = hv;
#else
    if (EPI != LINEAR && EPI != LINEAR_SAVE) v = __builtin_elementwise_max(v, (f32x8)(0.f));
    if (EDGE && !valid) v = (f32x8)(0.f);
#if defined(RDN_ABLATE_NOSTORE)
    if (v[0] == 123456.f)
#endif
    *p = __builtin_convertvector(v, V);
#endif
  };
  constexpr int K0 = WALK ? 4 : 2;                                      // koff index of tap shift 0
  const int sa = (int)dst + (h ? tl.koff[K0][1] : tl.koff[K0][0]);   // slot 4h + q of row r0
  auto epilogue = [&](int n, const Acc& a) {
    // positions outside [0, L): only the N-tiles that straddle 0 or L (a wave-uniform, scalar test)
    // pay the per-lane check and select; the other N-tiles of an edge tile store unmasked
    constexpr bool valid = true;             // rows outside [0, L): zero_outside after the loop
    if constexpr (EPI == STAGE) {
      // valid: the row's position lies in [0, L) (only there may the range guard see the value: the
      // rows of an edge tile beyond L + 1 are computed from rows no wave keeps current)
      stg->put(n, __builtin_shufflevector(a.v[0], a.v[1], 0, 1, 2, 3, 4, 5, 6, 7),
               !EDGE || in_range(pos0 + NR * n + (lane & 15), tl.L));
      return;
    }
    V* p = (V*)(tl.lds + sa + n * NR * ROWB);
    if constexpr (EPI == LINEAR_SAVE) idv[n] = *p;
    const f32x8 v = __builtin_shufflevector(a.v[0], a.v[1], 0, 1, 2, 3, 4, 5, 6, 7);
    if constexpr (EPI == LINEAR_SAVE) {
      if (cs) {
        const int r = pos0 - tl.base + NR * n + (lane & 15);
        if (r >= cs->lo && r < cs->hi) {
          cs->sum += v;
          cs->max = __builtin_elementwise_max(cs->max, v);
        }
      }
    }
    store_slot(p, v, valid, n);
  };

#if defined(RDN_HYB_STAMPS) && RDN_HYB_STAMPS
  constexpr bool LST = WALK && EPI == RELU;
  unsigned long long lt[5] = {__builtin_amdgcn_s_memtime(), 0, 0, 0, 0};
#endif
  Acc prev;
  constexpr int PF = RDN_H16_PF;       // B fragments in flight ahead of the step that consumes them
  constexpr int K = KS * NT;           // steps (N-tile n, k-step s), k = KS n + s
  // RDN_H16_ESPLIT = e > 1 (f16 RELU / LINEAR layers): the previous N-tile's rounding and ReLU at step
  // 1, its ds_write_b128 at step e, so one step no longer carries the whole epilogue (diagnostic A/B)
  constexpr bool ESPLIT = RDN_H16_ESPLIT > 1 && RDN_H16_F16 && (EPI == RELU || EPI == LINEAR);
  V pend;
  V B[PF + 1];
#pragma unroll
  for (int k = 0; k < PF; ++k) B[k] = *(const V*)(tl.lds + ba.at(k / KS, k % KS));
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    Acc acc;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int k = KS * n + s, kp = k + PF;
#if RDN_PRIO_SWITCH
      if (n == RDN_PRIO_SWITCH && s == 0 && h) __builtin_amdgcn_s_setprio(1);
#endif
#if defined(RDN_ABLATE_NOLDS)
      if (kp < K) { B[kp % (PF + 1)] = B[(k + 1) % (PF + 1)]; asm volatile("" : "+v"(B[kp % (PF + 1)])); }
#else
      if (kp < K) B[kp % (PF + 1)] = *(const V*)(tl.lds + ba.at(kp / KS, kp % KS));
#endif
      if constexpr (WALK && EPI == RES_RELU) {
        if (n > 0 && s == 0) idn[n & 1] = *(const V*)(tl.lds + sid + n * NR * ROWB);
      }
      mstep(F, s, B[k % (PF + 1)], acc);
#if defined(RDN_HYB_STAMPS) && RDN_HYB_STAMPS
      if (LST && k == 0) lt[1] = __builtin_amdgcn_s_memtime();
      if (LST && k == K - 1) lt[2] = __builtin_amdgcn_s_memtime();
#endif
      if constexpr (ESPLIT) {
        if (n > 0 && s == 1) {
          V hv = __builtin_convertvector(__builtin_shufflevector(prev.v[0], prev.v[1], 0, 1, 2, 3, 4, 5, 6, 7), V);
          if (EPI == RELU) hv = __builtin_elementwise_max(hv, (V)((E)0));
          pend = hv;
        }
        if (n > 0 && s == RDN_H16_ESPLIT) *(V*)(tl.lds + sa + (n - 1) * NR * ROWB) = pend;
      } else {
        if (n > 0 && s == 1) epilogue(n - 1, prev);
      }
      if (WALK && n == 1 && s == 0) carry_store(tl, dst, CA, cc, CROW);
#if !defined(RDN_ABLATE_NOALOAD)
      // the next layer's operands, one buffer load every LDSTEP-th step: the vector-memory traffic
      // of the CU's 8 waves spreads over the layer
      if (has_next && k % LDSTEP == 0 && k / LDSTEP < NLOAD) load_op(tl, next, h, k / LDSTEP, lo, G);
#endif
#if RDN_H16_SGB
      // explicit interleave inside the step (diagnostic A/B): MFMA, VALU, B read, MFMA, VALU, store, load
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, RDN_H16_SGB, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 16, 0);
      __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
#endif
      __builtin_amdgcn_sched_barrier(0);
    }
    prev = acc;
  }
  epilogue(NT - 1, prev);
#if !defined(RDN_ABLATE_NOZERO)           // diagnostic builds only (tools/ablate.py): wrong results
  if constexpr (EDGE && EPI != STAGE) zero_outside(tl, dst, pos0 - tl.base, h, lane);
#endif
  // walk: the next layer's (RES_RELU) N-tile-0 identity, rows r0 - 2 of this layer's input (stable
  // until the barrier below)
  if (WALK && walk_id) *walk_id = *(const V*)(tl.lds + src + (h ? tl.koff[2][1] : tl.koff[2][0]));
  tl.layer += 1;
#if defined(RDN_HYB_STAMPS) && RDN_HYB_STAMPS
  if (LST) lt[3] = __builtin_amdgcn_s_memtime();
#endif
#if defined(RDN_ABLATE_NOBARRIER)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#else
  lds_barrier();
#endif
#if defined(RDN_HYB_STAMPS) && RDN_HYB_STAMPS
  if (LST) {
    lt[4] = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int k = 0; k < 4; ++k) tl.lst[k] += lt[k + 1] - lt[k];
    tl.lst[4] += 1;
  }
#endif
}

// Conv1d(64, 1, 3) head, packed as a big layer whose M-tiles 0 and 2 (channels 0 and 32) both hold
// cout 0 in row 0 and its weights' rounding residue in row 1 (pack.cpp pack_big_bf16: the two
// partial sums add in fp32, so the head's weights are exact to ~2^-22 at no extra MFMA; the head
// feeds the RRCDNet cancellation x - (r + l)/2).  Half h computes N-tiles h*HN .. h*HN + HN-1 of
// its row block (those < NT) from its first M-tile / its 32-channel tile; out[j] = cout 0 of row
// head_row(j), in lanes 0..HEAD_LANES-1 (regs 0 and 1 hold rows 0 and 1 there in both MFMA forms).
// No write, no barrier; the next layer's operands stream into G.
template <bool EDGE>
__device__ __forceinline__ void head(Tile& tl, uint32_t src, const Frags& F, Frags& G, bool has_next,
                                     float (&out)[HN], int next_layer = -1) {
  const int w = __builtin_amdgcn_readfirstlane(tid() >> 6), h = w / RB;
  const int next = next_layer >= 0 ? next_layer : tl.layer + 1;
  const BAddr ba(tl, src, 1);
  Carry cc;
  if constexpr (WALK) {
    tl.base -= 1;
    cc = carry_load(tl, src, false);
  }
  const int pos0 = tl.base + CG + rblock(w) * RW + NR * HN * h;
  if (EDGE && pos0 >= tl.L + (WALK ? 0 : 2)) {
    if constexpr (WALK) carry_store(tl, 0, false, cc);
    if (has_next) load_frags(tl, next, G);
#pragma unroll
    for (int j = 0; j < HN; ++j) out[j] = 0.f;
    tl.layer += 1;
    return;
  }
  const LaneOff lo = lane_off();
  // N-tile of step j, clamped (the reads of a skipped N-tile stay inside the buffer)
  auto ntile = [&](int j) { return min(h * HN + j, NT - 1); };
  constexpr int PF = RDN_H16_PF, K = KS * HN;
  V B[PF + 1];
#pragma unroll
  for (int k = 0; k < PF; ++k) B[k] = *(const V*)(tl.lds + ba.at(ntile(k / KS), k % KS));
#pragma unroll
  for (int j = 0; j < HN; ++j) {
    Acc acc;
    const bool live = h * HN + j < NT;     // wave-uniform
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int k = KS * j + s, kp = k + PF;
      if (kp < K) B[kp % (PF + 1)] = *(const V*)(tl.lds + ba.at(ntile(kp / KS), kp % KS));
      if (live) {
        acc.v[0] = mma(F.a[s], B[k % (PF + 1)], s == 0 ? F.bias[0] : acc.v[0]);
      }
      if (WALK && j == 1 && s == 0) carry_store(tl, 0, false, cc);
      // the next layer's NLOAD operand loads spread over the head's K steps (operand i at step
      // i * K / NLOAD: every one is issued however few N-tiles the head has)
      if (has_next) {
#pragma unroll
        for (int i = 0; i < NLOAD; ++i)
          if (i * K / NLOAD == k) load_op(tl, next, h, i, lo, G);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    out[j] = acc.v[0][0] + acc.v[0][1];
  }
  tl.layer += 1;
}

// tile over positions [base, base + WB) of the spectrum at x; big: the blob's big-layer section
__device__ __forceinline__ Tile init_tile(char* lds, const uint8_t* blob, const uint8_t* big, const float* x, int L,
                                          int base) {
  Tile tl;
  tl.lds = lds;
  tl.x = x;
  tl.L = L;
  tl.base = base;
  tl.small = (const float*)blob;
  tl.big = big;
  // raw buffer over the big-layer section (stride 0, 2 GiB bound; dword 3 = 0x00020000, the raw
  // 32-bit data format of the gfx9 buffer descriptor)
  tl.wrsrc = __builtin_amdgcn_make_buffer_rsrc((void*)tl.big, 0, 0x7fffffff, 0x00020000);
  tl.layer = 0;
  const int t = tid();
  const int q = (t & 63) >> 4;
  tl.r0 = CG + rblock(t >> 6) * RW + (t & 15);
  constexpr int D0 = WALK ? -4 : -2;
#pragma unroll
  for (int d = 0; d < 5; ++d)
#pragma unroll
    for (int u = 0; u < 2; ++u) tl.koff[d][u] = soff(tl.r0 + D0 + d, 4 * u + q);
  tl.cs_cur = tl.cs_prev = (int)CARRY_OFF;
  tl.dn_prev = 0;
  tl.dnext = 1;
  tl.first = true;
  tl.status = nullptr;
  return tl;
}

__device__ __forceinline__ Tile make_tile(char* lds, const uint8_t* blob, const float* x, int L, int T, int tiles,
                                          int halo, int& n_out) {
  const int n = __builtin_amdgcn_workgroup_id_x() / tiles, tile = __builtin_amdgcn_workgroup_id_x() - n * tiles;
  n_out = n;
  return init_tile(lds, blob, blob + SMALL_BYTES, x + (size_t)n * L, L, tile * T - halo);
}

// tile row of head output j of this lane (lanes 0..HEAD_LANES-1); a row no tile owns (WB) for the
// skipped N-tile of an odd NT
__device__ __forceinline__ int head_row(int j) {
  const int w = tid() >> 6, n = HN * (w / RB) + j;
  return n < NT ? CG + rblock(w) * RW + NR * n + (tid() & (HEAD_LANES - 1)) : WB;
}

__device__ __forceinline__ void store_out(const Tile& tl, float* y, int n, const float (&v)[HN], int halo, int T) {
  if ((tid() & 63) >= HEAD_LANES) return;
#pragma unroll
  for (int k = 0; k < HN; ++k) {
    const int j = head_row(k);
    const int p = tl.base + j;
    if (j >= halo && j < halo + T && p < tl.L) y[(size_t)n * tl.L + p] = v[k];
  }
}

// walk: start tile t (stem row CG at position t WT - c0: a shallower branch starts c0 further left)
__device__ __forceinline__ void walk_start(Tile& tl, int t, int c0) {
  tl.base = t * WT - CG - c0;
  tl.cs_cur = tl.cs_prev = (int)CARRY_OFF;
  tl.dn_prev = 0;
  tl.dnext = 1;
  tl.layer = 0;
}
// the stem inputs of tile t (fetched ahead: their latency hides under the previous tile's last layer)
__device__ __forceinline__ StemX walk_stem_load(const Tile& tl, int t, int c0) {
  Tile s = tl;
  s.base = t * WT - CG - c0;
  return stem_load(s);
}

// walk: head outputs at positions inside [0, L)
__device__ __forceinline__ void store_out_walk(const Tile& tl, float* y, const float (&v)[HN]) {
  if ((tid() & 63) >= HEAD_LANES) return;
#pragma unroll
  for (int k = 0; k < HN; ++k) {
    const int j = head_row(k);
    const int p = tl.base + j;
    if (j < WB && in_range(p, tl.L)) y[p] = v[k];
  }
}

}  // namespace H16_NS
}  // namespace rdn
