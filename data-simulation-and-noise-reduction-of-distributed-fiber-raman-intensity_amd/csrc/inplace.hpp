// Device building blocks for tiles with 256-byte activation rows, updated IN PLACE
// (fused_inplace.hip: whole-network kernels; cbam.hip: CBAM-network segments):
//   MODE_F32   exact-fp32 MFMA (v_mfma_f32_16x16x4_f32), activations fp32;
//   MODE_X3    split-bf16 MFMA: every operand is held as a bf16 pair v = hi + lo and each product
//              is computed as hi*hi + hi*lo + lo*hi (3 x v_mfma_f32_16x16x32_bf16, fp32 accumulate),
//              ~16 significant bits per operand.  This is the bf16 mode that meets the 2e-2
//              tolerance on trained weights, where a single bf16 rounding of weights and
//              activations does not (tools/precision_sweep.py: 0.20 vs 4e-4 on trained RRCDNet).
//
// One 512-thread workgroup owns WB = 512 positions of one spectrum (halo included); the 132 KB
// buffer (516 rows x 256 B) holds the whole tile.  Wave w = (m = w & 3, nh = w >> 2) computes
// output channels [16m, 16m+16) for rows [256nh, 256nh+256) and keeps them in accumulators until
// the workgroup barrier, after which every wave overwrites its outputs in place.  A-operands
// (weights) come straight from L2 (<= 12 KB per wave per layer).  fp32 accumulation is split over
// S partial sums (k-steps dealt round-robin), which roughly halves the error of one 192-term
// fp32 chain (tools/precision_sweep.py, SURVEY.md §7 "fp32 parity definition").
//
// Reference forwards: 1DCNN/train.py:71-82, RRCDNet/train.py:72-98, DSDN/train.py:72-126,
// PIDN/train.py:72-106.
#pragma once
#include "common.hpp"

namespace rdn {
namespace ip {

constexpr int MODE_F32 = 0, MODE_B1 = 1, MODE_X3 = 2, MODE_H8 = 3, MODE_F16 = 4;
// single-plane 16-bit modes (one MFMA per product, one rounding per operand)
__host__ __device__ constexpr bool single16(int mode) { return mode == MODE_B1 || mode == MODE_F16; }
constexpr uint32_t LDS_BYTES = ACT_BYTES_F32;                    // 132096 (512 rows + guards)

// Tile geometry by number of 128-row blocks: NBK = 4 -> 512 rows with 2 zero guard rows per side
// (the CBAM segment kernels, which keep scratch behind the buffer); NBK = 5 -> 640 rows, no guard
// rows, the whole 160 KiB LDS (fused_inplace.hip).  Without guards a tap that leaves the tile
// wraps to its other end: those rows are outside every output's receptive field (the halo covers
// the stack's depth), so any finite value serves; spectrum positions outside [0, L) are re-zeroed
// by the write-backs of edge tiles.
template <int NBK> struct TileGeo {
  static constexpr int WB = 128 * NBK;
  static constexpr bool HALF = false;
  static constexpr bool WRAP = NBK != 4;
  static constexpr int GRD = WRAP ? 0 : GUARD;
  static constexpr uint32_t LDS = (WB + 2 * GRD) * ROWB_F32;
  __device__ static int row(int r) { return WRAP ? (r < 0 ? r + WB : (r >= WB ? r - WB : r)) : r + GRD; }
};
// Walk geometry (the RDN_F16MIX walk, rrcdnet_hybrid_walk.hpp; fused16.hpp "Walk instantiation"):
// NBK blocks of computed rows behind GRD = 4 carry rows (the previous tile's last 2d rows of the
// layer's input, taps r - 2d, r - d, r: nothing is read past the computed rows), no wrap.
// WB = RDN_WALK_ROWS_MIX computed rows in NBK blocks; when WB = 128 NBK - 64 the last block is half
// (HALF): its rows are those of the waves of quarters nq = 0, 1, and the waves of quarters 2, 3 skip it.
#ifndef RDN_HALF_REMAP
#define RDN_HALF_REMAP 0
#endif
#ifndef RDN_TAIL_SWAP
#define RDN_TAIL_SWAP 0       // A/B: the half block on waves 4-7 instead of 0-3 (inplace.hpp conv)
#endif
#ifndef RDN_TAIL_EARLY
#define RDN_TAIL_EARLY 0      // A/B: next-layer operand loads of the half block's idle waves one block early
                              // (1: all; 2: the fragments, bias and scales at the last block; 3: k-step 0 only)
#endif
#ifndef RDN_STAGE_FIRST
#define RDN_STAGE_FIRST 0     // A/B (the hybrid walk): layer 9's plane stores before the tail's operand loads
#endif
#ifndef RDN_TAIL_SGB
// A/B: the corrected layers' write-back VALU (e4m3 split of block j-2) interleaved between the last
// N-tile's MFMAs of the k-step, RDN_TAIL_SGB VALU per MFMA (sched_group_barrier); 0 = off
#define RDN_TAIL_SGB 0
#endif
#ifndef RDN_TAIL_STAG
#define RDN_TAIL_STAG 0       // diagnostic A/B: the in-place write-back of waves 4-7 one k-step late
#endif
template <int NBK> struct WalkGeo {
  static constexpr int WB = RDN_WALK_ROWS_MIX;
  static constexpr bool HALF = WB == 128 * NBK - 64;
  static_assert(WB == 128 * NBK || HALF, "whole blocks, or a last half block");
  static constexpr bool WRAP = false;
  static constexpr int GRD = 4;
  static constexpr uint32_t LDS = (WB + GRD) * ROWB_F32;
  __device__ static int row(int r) { return r + GRD; }
};
template <int NBK, bool WALK> struct GeoOf { using T = TileGeo<NBK>; };
template <int NBK> struct GeoOf<NBK, true> { using T = WalkGeo<NBK>; };
static_assert(TileGeo<4>::LDS == LDS_BYTES, "CBAM geometry");
static_assert(TileGeo<5>::LDS == 163840, "fused geometry fills the LDS");
// bytes per packed big layer and offset of its bias: f32 / split-bf16 / bf16 49408 (bias at 49152),
// f16 + e4m3 correction 50432 (bias at 50176)
template <int MODE> struct LayerBytes {
  static constexpr int BYTES = BIG_BYTES_F32, BIAS = BIG_FRAG_FLOATS_F32 * 4;
};

enum Epi : int { RELU = 1, ADD_ID = 2, SAVE_ID = 4 };

struct Tile {
  char* lds;
  const float* x;
  int L;
  int base;
  const uint8_t* big;
  int layer;
  const float* small;
  uint64_t corr;        // MODE_H8: bit i = big layer i consumes the e4m3 correction (CORR_SLOT)
  float amax;           // MODE_H8: running max of the values h8_sat saw (range guard, h8_track)
  unsigned* status;     // the launch's status word (input gate, STATUS_GATE) or NULL
  // walk only (conv<..., WALK>): this layer's carry slot (LDS byte offset), the previous layer's slot
  // and its carry rows' dilation, the dilation of the layer reading this one, first tile of a spectrum
  int cs_cur, cs_prev, dn_prev, dnext;
  bool first;
#if defined(RDN_HYB_STAMPS) && RDN_HYB_STAMPS
  // diagnostic (tools/hyb_stamps.py): this wave's cycles working / waiting at the corrected walk layers'
  // block barriers (flushed once per spectrum by rrcdnet_hybrid_walk)
  unsigned long long bwork, bwait;
#endif
};

__device__ __forceinline__ bool in_range(int p, int L) { return p >= 0 && p < L; }

// Thread index the compiler cannot treat as loop-invariant: per-lane addresses derived from it are
// recomputed where they are used instead of being hoisted out of the callers' layer / spectrum
// loops (where, with 256 VGPRs taken by the conv, they are spilled to scratch and reloaded).
__device__ __forceinline__ int opaque_tid() {
  int t = __builtin_amdgcn_workitem_id_x();
  asm volatile("" : "+v"(t));
  return t;
}

// ---- operand traits -------------------------------------------------------------------------
template <int MODE> struct Op;

template <> struct Op<MODE_F32> {
  // k-step = (tap t, 16-channel group g), 4 MFMAs of K=4; lane quarter q carries cin 16g+4q+i
  static constexpr int KSTEPS = 12;
  struct A { f32x4 w; };
  struct B { f32x4 v; };
  __device__ static A load_a(const uint8_t* layer, int m, int s, int lane) {
    return A{((const f32x4*)layer)[(m * 12 + s) * 64 + lane]};
  }
  __device__ static B load_b(const char* act, int prow, int s, int q) {
    const int g = s & 3;
    return B{*(const f32x4*)(act + off_f32(prow, 64 * g + 16 * q))};
  }
  __device__ static int tap(int s) { return s >> 2; }
  // precomputed-address forms: PLANES byte addresses per k-step / store, plus a row offset that
  // is a multiple of 16 rows (leaves the row swizzle unchanged -> ds_* immediate offsets)
  static constexpr int PLANES = 1;
  __device__ static int bslot(int s, int q, int) { return 4 * (s & 3) + q; }
  __device__ static int sbyte(int c0, int) { return 4 * c0; }
  __device__ static B load_b_at(const char* act, const uint32_t (&ad)[PLANES], uint32_t off) {
    return B{*(const f32x4*)(act + ad[0] + off)};
  }
  __device__ static void store4_at(char* act, const uint32_t (&ad)[PLANES], uint32_t off, f32x4 v, float* = nullptr) {
    *(f32x4*)(act + ad[0] + off) = v;
  }
  __device__ static f32x4 mma(const A& a, const B& b, f32x4 acc, uint32_t, int) {
#pragma unroll
    for (int i = 0; i < 4; ++i) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w[i], b.v[i], acc, 0, 0, 0);
    return acc;
  }
  // 4 channels [c0, c0+4) of a row
  __device__ static void store4(char* act, int prow, int c0, f32x4 v, float* = nullptr) {
    *(f32x4*)(act + off_f32(prow, 4 * c0)) = v;
  }
  __device__ static f32x4 load4(const char* act, int prow, int c0) { return *(const f32x4*)(act + off_f32(prow, 4 * c0)); }
};

__device__ __forceinline__ float bf2f(__bf16 h) { return (float)h; }

template <> struct Op<MODE_X3> {
  // k-step = (tap t, 32-channel half u); row = [hi 64 ch bf16 | lo 64 ch bf16]
  static constexpr int KSTEPS = 6;
  struct A { bf16x8 hi, lo; };
  struct B { bf16x8 hi, lo; };
  __device__ static A load_a(const uint8_t* layer, int m, int s, int lane) {
    const bf16x8* f = (const bf16x8*)layer + ((m * 6 + s) * 2) * 64 + lane;
    return A{f[0], f[64]};
  }
  __device__ static B load_b(const char* act, int prow, int s, int q) {
    const int u = s & 1;
    return B{*(const bf16x8*)(act + off_f32(prow, 64 * u + 16 * q)),
             *(const bf16x8*)(act + off_f32(prow, 128 + 64 * u + 16 * q))};
  }
  __device__ static int tap(int s) { return s >> 1; }
  static constexpr int PLANES = 2;
  __device__ static int bslot(int s, int q, int p) { return 8 * p + 4 * (s & 1) + q; }
  __device__ static int sbyte(int c0, int p) { return 128 * p + 2 * c0; }
  __device__ static B load_b_at(const char* act, const uint32_t (&ad)[PLANES], uint32_t off) {
    return B{*(const bf16x8*)(act + ad[0] + off), *(const bf16x8*)(act + ad[1] + off)};
  }
  __device__ static void store4_at(char* act, const uint32_t (&ad)[PLANES], uint32_t off, f32x4 v, float* = nullptr) {
    const bf16x4 hi = __builtin_convertvector(v, bf16x4);           // 2 x v_cvt_pk_bf16_f32 (RNE)
    // hi back to f32 straight from the packed bits (one shift / mask each, no re-conversion)
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    const u32x2 hb = __builtin_bit_cast(u32x2, hi);
    const f32x4 hf = {__uint_as_float(hb.x << 16), __uint_as_float(hb.x & 0xffff0000u),
                      __uint_as_float(hb.y << 16), __uint_as_float(hb.y & 0xffff0000u)};
    const bf16x4 lo = __builtin_convertvector(v - hf, bf16x4);
    *(bf16x4*)(act + ad[0] + off) = hi;
    *(bf16x4*)(act + ad[1] + off) = lo;
  }
  __device__ static f32x4 mma(const A& a, const B& b, f32x4 acc, uint32_t, int) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.lo, b.hi, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.hi, b.lo, acc, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.hi, b.hi, acc, 0, 0, 0);
  }
  __device__ static void store4(char* act, int prow, int c0, f32x4 v, float* = nullptr) {
    const bf16x4 hi = __builtin_convertvector(v, bf16x4);           // 2 x v_cvt_pk_bf16_f32
    const bf16x4 lo = __builtin_convertvector(v - __builtin_convertvector(hi, f32x4), bf16x4);
    *(bf16x4*)(act + off_f32(prow, 2 * c0)) = hi;
    *(bf16x4*)(act + off_f32(prow, 128 + 2 * c0)) = lo;
  }
  __device__ static f32x4 load4(const char* act, int prow, int c0) {
    const bf16x4 hi = *(const bf16x4*)(act + off_f32(prow, 2 * c0));
    const bf16x4 lo = *(const bf16x4*)(act + off_f32(prow, 128 + 2 * c0));
    return __builtin_convertvector(hi, f32x4) + __builtin_convertvector(lo, f32x4);
  }
};

// plain bf16 (MODE_B1, 'bf16-unsafe') or f16 (MODE_F16, RDN_F16) on the same 256-byte rows (used by
// the CBAM networks): hi plane only, one MFMA per product.
typedef _Float16 h16x8_t __attribute__((ext_vector_type(8)));
typedef _Float16 h16x4_t __attribute__((ext_vector_type(4)));
template <typename E> struct S16Types;
template <> struct S16Types<__bf16> {
  typedef bf16x8 V8;
  typedef bf16x4 V4;
  __device__ static f32x4 mma(V8 a, V8 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }
};
template <> struct S16Types<_Float16> {
  typedef h16x8_t V8;
  typedef h16x4_t V4;
  __device__ static f32x4 mma(V8 a, V8 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0); }
};
template <typename E> struct OpS16 {
  typedef typename S16Types<E>::V8 V8;
  typedef typename S16Types<E>::V4 V4;
  static constexpr int KSTEPS = 6;
  struct A { V8 hi; };
  struct B { V8 hi; };
  __device__ static A load_a(const uint8_t* layer, int m, int s, int lane) {
    return A{((const V8*)layer)[((m * 6 + s) * 2) * 64 + lane]};
  }
  __device__ static B load_b(const char* act, int prow, int s, int q) {
    return B{*(const V8*)(act + off_f32(prow, 64 * (s & 1) + 16 * q))};
  }
  __device__ static int tap(int s) { return s >> 1; }
  static constexpr int PLANES = 1;
  __device__ static int bslot(int s, int q, int) { return 4 * (s & 1) + q; }
  __device__ static int sbyte(int c0, int) { return 2 * c0; }
  __device__ static B load_b_at(const char* act, const uint32_t (&ad)[PLANES], uint32_t off) {
    return B{*(const V8*)(act + ad[0] + off)};
  }
  __device__ static void store4_at(char* act, const uint32_t (&ad)[PLANES], uint32_t off, f32x4 v, float* = nullptr) {
    *(V4*)(act + ad[0] + off) = __builtin_convertvector(v, V4);
  }
  __device__ static f32x4 mma(const A& a, const B& b, f32x4 acc, uint32_t, int) {
    return S16Types<E>::mma(a.hi, b.hi, acc);
  }
  __device__ static void store4(char* act, int prow, int c0, f32x4 v, float* = nullptr) {
    *(V4*)(act + off_f32(prow, 2 * c0)) = __builtin_convertvector(v, V4);
  }
  __device__ static f32x4 load4(const char* act, int prow, int c0) {
    return __builtin_convertvector(*(const V4*)(act + off_f32(prow, 2 * c0)), f32x4);
  }
};
template <> struct Op<MODE_B1> : OpS16<__bf16> {};
template <> struct Op<MODE_F16> : OpS16<_Float16> {};

// f16 main product + block-scaled e4m3 correction (RDN_F16F8).  Row = [hi: 64 ch f16 (128 B) |
// e4m3(hi / 4) (64 B) | e4m3(lo * 2^9) (64 B)], v = hi + lo, channels in h16_channel order within
// each plane (the 8 outputs of lane quarter q of an M-tile pair {2u, 2u+1} are 16-B f16 slot 4u+q
// and 8-B e4m3 slot 4u+q).  One k-step per tap:
//   W.X ~= W_hi.X_hi (2 x v_mfma_f32_16x16x32_f16, K = 64)
//        + [W_lo | W_hi] . [X_hi | X_lo]  (1 x v_mfma_scale_f32_16x16x128_f8f6f4, e4m3, K = 128),
// i.e. the two correction products of the split-bf16 mode in ONE fp8 MFMA at 2x the 16-bit rate:
// 64 MFMA cycles per (tap, 16 x 16 tile) instead of 96.  W_lo/W_hi e4m3 carry per-32-channel E8M0
// scales (packed on the host); the activation planes use fixed scales (common.hpp H8_*), and the
// stored activation saturates at +-1792 so that no conversion leaves the e4m3 range
// (v_cvt_*_fp8 returns NaN there).  CPU emulation on trained RRCDNet (tools/precision_sweep.py):
// 1.5e-3 max-abs, vs 0.030 for plain f16 and 0.20 for plain bf16.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4v __attribute__((ext_vector_type(4)));
typedef short s16x2 __attribute__((ext_vector_type(2)));

// 4 floats -> 4 e4m3 bytes of v / div (v_cvt_scalef32_pk_fp8_f32: the division is free)
__device__ __forceinline__ uint32_t pk_e4m3_div(f32x4 v, float div) {
  // both halves are overwritten: seed the tied destination with a source that dies here (v[0]),
  // so no zero-initialising v_mov is needed
  s16x2 o = __builtin_bit_cast(s16x2, v[0]);
  o = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(o, v[0], v[1], div, false);
  o = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(o, v[2], v[3], div, true);
  return __builtin_bit_cast(uint32_t, o);
}
__device__ __forceinline__ f32x4 unpk_e4m3(uint32_t w) {
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  const f32x2 a = __builtin_amdgcn_cvt_pk_f32_fp8((int)w, false), b = __builtin_amdgcn_cvt_pk_f32_fp8((int)w, true);
  return f32x4{a[0], a[1], b[0], b[1]};
}
// saturate (and, with RELU, rectify) in one v_med3 per value
template <bool RELU>
__device__ __forceinline__ f32x4 h8_sat(f32x4 v) {
  const float lo = RELU ? 0.f : -H8_SAT;
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = __builtin_amdgcn_fmed3f(v[i], lo, H8_SAT);
  return v;
}
// Range guard of the e4m3 correction planes: h8_sat clamps |v| to H8_SAT, so every value it sees
// first enters a per-lane running max (two v_max3 per 4 values; a rectified layer needs no |.|, its
// negative values become 0).  The kernels vote the max at the end of a tile (range_vote): a tile
// that saturated writes NaN outputs and raises the launch's status word (rdn_forward_status:
// RDN_ERANGE) -- a clamped activation never reaches an output silently.
template <bool RELU>
__device__ __forceinline__ void h8_track(float& m, f32x4 v) {
  // spelled as asm: the same maxima written with fmaxf made the compiler re-schedule the in-place
  // epilogue into 56-350 VGPRs of spills (the f16f8 / hybrid kernels sit at 241-256 VGPRs)
  if (RELU) {
    asm("v_max3_f32 %0, %0, %1, %2" : "+v"(m) : "v"(v[0]), "v"(v[1]));
    asm("v_max3_f32 %0, %0, %1, %2" : "+v"(m) : "v"(v[2]), "v"(v[3]));
  } else {
    asm("v_max3_f32 %0, %0, |%1|, |%2|" : "+v"(m) : "v"(v[0]), "v"(v[1]));
    asm("v_max3_f32 %0, %0, |%1|, |%2|" : "+v"(m) : "v"(v[2]), "v"(v[3]));
  }
}
// split a saturated activation into its three plane encodings
struct H8Split {
  f16x4 hi;
  uint32_t hi8, lo8;
};
__device__ __forceinline__ H8Split h8_split(f32x4 r) {
  const f16x4 h = __builtin_convertvector(r, f16x4);
  // lo = r - f32(h) in one v_fma_mix_f32 per value (f16 source operand, exact), and the e4m3 copy
  // of hi converted from r itself (its 3-bit mantissa cannot tell r from f16(r) except at
  // double-rounding ties): no f16 -> f32 round trip.  14 VALU per 4 values instead of 18.
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  const u32x2 hb = __builtin_bit_cast(u32x2, h);
  f32x4 lo;
  // the compiler turns fma(f32(h), -1, r) into cvt + sub; the mixed-precision FMA is spelled out
  asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(lo[0]) : "v"(hb.x), "v"(r[0]));
  asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(lo[1]) : "v"(hb.x), "v"(r[1]));
  asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(lo[2]) : "v"(hb.y), "v"(r[2]));
  asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(lo[3]) : "v"(hb.y), "v"(r[3]));
  return H8Split{h, pk_e4m3_div(r, H8_HI_DIV), pk_e4m3_div(lo, H8_LO_DIV)};
}

template <> struct LayerBytes<MODE_H8> {
  static constexpr int BYTES = BIG_BYTES_H8, BIAS = H8_BIAS_OFF;
};

template <> struct Op<MODE_H8> {
  static constexpr int KSTEPS = 3;
  struct A { f16x8 h[2]; i32x8 c; };
  struct B { f16x8 h[2]; i32x8 c; };
  __device__ static A load_a(const uint8_t* layer, int m, int s, int lane) {
    const f16x8* f = (const f16x8*)layer + (m * 6 + 2 * s) * 64 + lane;
    return A{{f[0], f[64]}, *(const i32x8*)(layer + H8_CORR_OFF + ((m * 3 + s) * 64 + lane) * 32)};
  }
  // the f16 fragments only (the next layer is uncorrected: its e4m3 fragments are never read)
  __device__ static void load_a_main(const uint8_t* layer, int m, int s, int lane, A& a) {
    const f16x8* f = (const f16x8*)layer + (m * 6 + 2 * s) * 64 + lane;
    a.h[0] = f[0];
    a.h[1] = f[64];
  }
  __device__ static int tap(int s) { return s; }
  static constexpr int PLANES = 4;
  // B fragment of k-step s: f16 slots q (channels 0-31) and 4+q (32-63), e4m3 hi / lo bytes 16q..16q+15
  __device__ static int bslot(int, int q, int p) { return 4 * p + q; }
  // stores: byte of channels [c0, c0+4) in plane p (0 f16, 1 e4m3 hi, 2 e4m3 lo)
  __device__ static int sbyte(int c0, int p) {
    const int mt = c0 >> 4, slot = 4 * (mt >> 1) + ((c0 >> 2) & 3), half = mt & 1;
    return p == 0 ? 16 * slot + 8 * half : (p == 1 ? 128 : 192) + 8 * slot + 4 * half;
  }
  __device__ static B load_b_at(const char* act, const uint32_t (&ad)[PLANES], uint32_t off) {
    const i32x4v ch = *(const i32x4v*)(act + ad[2] + off), cl = *(const i32x4v*)(act + ad[3] + off);
    return B{{*(const f16x8*)(act + ad[0] + off), *(const f16x8*)(act + ad[1] + off)},
             __builtin_shufflevector(ch, cl, 0, 1, 2, 3, 4, 5, 6, 7)};
  }
  // per-layer correction (RDN_F16MIX): without it only the f16 planes are read
  __device__ static B load_b_at(const char* act, const uint32_t (&ad)[PLANES], uint32_t off, bool cin) {
    B b;
    b.h[0] = *(const f16x8*)(act + ad[0] + off);
    b.h[1] = *(const f16x8*)(act + ad[1] + off);
    if (cin) {
      const i32x4v ch = *(const i32x4v*)(act + ad[2] + off), cl = *(const i32x4v*)(act + ad[3] + off);
      b.c = __builtin_shufflevector(ch, cl, 0, 1, 2, 3, 4, 5, 6, 7);
    }
    return b;
  }
  __device__ static B load_b(const char* act, int prow, int s, int q) {
    uint32_t ad[PLANES];
#pragma unroll
    for (int p = 0; p < PLANES; ++p) ad[p] = off_f32(prow, 16 * bslot(s, q, p));
    return load_b_at(act, ad, 0);
  }
  __device__ static void put(char* act, uint32_t a0, uint32_t a1, uint32_t a2, f32x4 v, float* amax) {
    if (amax) h8_track<false>(*amax, v);
    const H8Split x = h8_split(h8_sat<false>(v));
    *(f16x4*)(act + a0) = x.hi;
    *(uint32_t*)(act + a1) = x.hi8;
    *(uint32_t*)(act + a2) = x.lo8;
  }
  __device__ static void store4_at(char* act, const uint32_t (&ad)[PLANES], uint32_t off, f32x4 v, float* amax = nullptr) {
    put(act, ad[0] + off, ad[1] + off, ad[2] + off, v, amax);
  }
  __device__ static f32x4 mma(const A& a, const B& b, f32x4 acc, uint32_t sa, int s) {
    const int sb = (__builtin_amdgcn_workitem_id_x() & 32) ? H8_LO_E8M0 : H8_HI_E8M0;   // lanes 32-63: the lo blocks
    if (s == 0) acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a.c, b.c, acc, 0, 0, 0, (int)sa, 0, sb);
    else if (s == 1) acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a.c, b.c, acc, 0, 0, 1, (int)sa, 0, sb);
    else acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a.c, b.c, acc, 0, 0, 2, (int)sa, 0, sb);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a.h[0], b.h[0], acc, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a.h[1], b.h[1], acc, 0, 0, 0);
  }
  // the three MFMAs of mma one by one (conv interleaves them over its two M-tiles)
  __device__ static f32x4 mma_c(const A& a, const B& b, f32x4 acc, uint32_t sa, int s) {
    const int sb = (__builtin_amdgcn_workitem_id_x() & 32) ? H8_LO_E8M0 : H8_HI_E8M0;
    if (s == 0) return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a.c, b.c, acc, 0, 0, 0, (int)sa, 0, sb);
    if (s == 1) return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a.c, b.c, acc, 0, 0, 1, (int)sa, 0, sb);
    return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a.c, b.c, acc, 0, 0, 2, (int)sa, 0, sb);
  }
  __device__ static f32x4 mma_h(const A& a, const B& b, f32x4 acc, int u) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a.h[u], b.h[u], acc, 0, 0, 0);
  }
  __device__ static f32x4 mma(const A& a, const B& b, f32x4 acc, uint32_t sa, int s, bool cin) {
    if (cin) return mma(a, b, acc, sa, s);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a.h[0], b.h[0], acc, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a.h[1], b.h[1], acc, 0, 0, 0);
  }
  __device__ static void store4(char* act, int prow, int c0, f32x4 v, float* amax = nullptr) {
    put(act, off_f32(prow, sbyte(c0, 0)), off_f32(prow, sbyte(c0, 1)), off_f32(prow, sbyte(c0, 2)), v, amax);
  }
  __device__ static f32x4 load4(const char* act, int prow, int c0) {
    const f16x4 h = *(const f16x4*)(act + off_f32(prow, sbyte(c0, 0)));
    const uint32_t l = *(const uint32_t*)(act + off_f32(prow, sbyte(c0, 2)));
    return __builtin_convertvector(h, f32x4) + unpk_e4m3(l) * H8_LO_DIV;
  }
};

__device__ __forceinline__ void zero_guards(char* lds) {
  const int t = __builtin_amdgcn_workitem_id_x();           // 4 guard rows x 256 B = 64 lanes x 16 B
  if (t < 64) {
    const int r = t >> 4, slot = t & 15;
    const int prow = r < 2 ? r : ROWS - 4 + r;
    *(f32x4*)(lds + prow * ROWB_F32 + slot * 16) = f32x4{0.f, 0.f, 0.f, 0.f};
  }
}

__device__ __forceinline__ const cfloat* small_slot(const Tile& tl, int slot) {
  const float* p = tl.small + slot * SMALL_SLOT_FLOATS;
  asm volatile("" : "+s"(p));     // keep scalar-loaded weights from living across layers
  return (const cfloat*)p;
}

// Conv1d(1, 64, 3, padding=1) (+ folded BN) + ReLU, one row per thread, fp32; ACCUM adds the
// result onto the resident row (PIDN/train.py:105, identity recomputed from x).
template <int MODE, bool ACCUM = false, int NBK = 4>
__device__ __forceinline__ void stem(Tile& tl, int slot) {
  using TG = TileGeo<NBK>;
  const cfloat* sw = small_slot(tl, slot);
  bool over = false;              // an input beyond the 16-bit modes' domain (STATUS_GATE)
  for (int j = opaque_tid(); j < TG::WB; j += THREADS) {
  const int pr = TG::row(j);
  const int p = tl.base + j;
  const float xm = in_range(p - 1, tl.L) ? tl.x[p - 1] : 0.f;
  const float x0 = in_range(p, tl.L) ? tl.x[p] : 0.f;
  const float xp = in_range(p + 1, tl.L) ? tl.x[p + 1] : 0.f;
  const bool valid = in_range(p, tl.L);
  over = over || fabsf(x0) > INPUT_GATE;
#pragma unroll
  for (int cb = 0; cb < 16; ++cb) {
    f32x4 v = ACCUM ? Op<MODE>::load4(tl.lds, pr, 4 * cb) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = cb * 4 + i;
      float a = sw[192 + c];
      a = fmaf(sw[3 * c + 0], xm, a);
      a = fmaf(sw[3 * c + 1], x0, a);
      a = fmaf(sw[3 * c + 2], xp, a);
      a = fmaxf(a, 0.f);
      if (ACCUM) a += v[i];
      v[i] = valid ? a : 0.f;
    }
    Op<MODE>::store4(tl.lds, pr, 4 * cb, v, &tl.amax);
  }
  }
  if (tl.status && __builtin_amdgcn_ballot_w64(over) != 0 && (__builtin_amdgcn_workitem_id_x() & 63) == 0)
    raise_status(tl.status, STATUS_GATE);
}

// Conv1d(64, 1, 3, padding=1): the head, fp32 weights, fp64 or exact-ish accumulation, rounded once
// by the caller after the network's own combine (RRCDNet x - (r + l)/2, RRCDNet/train.py:98, a
// cancellation; PIDN/APIDN sigmoid).
//
// Row mapping of the results (HeadOut): fp32 / split-bf16 tiles, one row per thread (row tid + 512k
// in out[k]); the 16-bit tiles (f16 + e4m3, single-plane f16/bf16), the B-fragment arrangement of the
// convs -- lane (q, c16) of wave w reads the 16-B f16 slots 4u + q of rows 128k + 16w + c16 + t - 1
// (conflict-free ds_read_b128, like the conv B reads, instead of per-row 8-B reads that hit the same
// banks 4-way: the row-per-thread head cost 10 % of the f16 RRCDNet kernel), accumulates its 16
// channels x 3 taps, and the 4 quarters are summed across lanes (v_permlane16/32_swap): out[k] is
// row 128k + 16w + c16, on every quarter's lanes.
constexpr int HEAD_ROWS = 2;      // rows per thread of the row-per-thread head: ceil(640 / 512)
template <int MODE, int NBK = 4> struct HeadOut {
  static constexpr bool VEC = MODE == MODE_H8 || single16(MODE);
  static constexpr int ROWS = VEC ? NBK : HEAD_ROWS;
  __device__ static int row(int k) {
    const int t = __builtin_amdgcn_workitem_id_x();
    return VEC ? 128 * k + 16 * (t >> 6) + (t & 15) : t + THREADS * k;
  }
  __device__ static bool writer() { return !VEC || (__builtin_amdgcn_workitem_id_x() & 48) == 0; }
};

__device__ __forceinline__ float quarter_sum(float v) {
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  const float h = __uint_as_float(a[0]) + __uint_as_float(a[1]);          // lanes l, l ^ 32
  const auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(h), __float_as_uint(h), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);                   // and the other 16-lane row
}

template <int MODE, int NBK = 4>
__device__ __forceinline__ void head(const Tile& tl, int slot, double (&out)[HeadOut<MODE, NBK>::ROWS]) {
  using TG = TileGeo<NBK>;
  const cfloat* hw = small_slot(tl, slot);
  if constexpr (HeadOut<MODE, NBK>::VEC) {
    const int tid = opaque_tid(), lane = tid & 63, w = tid >> 6, q = lane >> 4, c16 = lane & 15;
    // channel of element jj of 16-B f16 slot s: h16_channel order (f16 + e4m3 tile), natural otherwise
    auto chan = [&](int s, int jj) { return MODE == MODE_H8 ? h16_channel(s, jj) : 8 * s + jj; };
    float wv[3][16];
    const float* hwv = (const float*)hw;
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) wv[t][i] = hwv[3 * chan(4 * (i >> 3) + q, i & 7) + t];
    const float bias = hw[192];
    if constexpr (MODE == MODE_H8) {
      // f16 plane by v_fma_mix_f32 (the f16 operand converted inside the FMA), e4m3-lo plane into a
      // separate packed accumulator (v_pk_fma_f32 on the pairs v_cvt_pk_f32_fp8 returns), scaled by
      // H8_LO_DIV (a power of two) once per row.  The NBK rows of a lane are independent sums,
      // interleaved innermost: one row's 48-term sum is a dependent FMA chain, and the head of a
      // single chain per row waited on FMA latency (the hybrid's right head + park: 11.6k cycles per
      // tile, tools/hyb_stamps.py)
      typedef float f32x2 __attribute__((ext_vector_type(2)));
      typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
      float acc[NBK];
      f32x2 accl[NBK];
#pragma unroll
      for (int k = 0; k < NBK; ++k) acc[k] = 0.f, accl[k] = f32x2{0.f, 0.f};
#pragma unroll
      for (int t = 0; t < 3; ++t) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int sl = 4 * u + q;
          u32x4 h[NBK];
          u32x2 lo[NBK];
#pragma unroll
          for (int k = 0; k < NBK; ++k) {
            const int pr = TG::row(128 * k + 16 * w + c16 + t - 1);
            h[k] = *(const u32x4*)(tl.lds + off_f32(pr, 16 * sl));
            lo[k] = *(const u32x2*)(tl.lds + off_f32(pr, 192 + 8 * sl));
          }
#pragma unroll
          for (int d = 0; d < 4; ++d) {
#pragma unroll
            for (int k = 0; k < NBK; ++k)
              asm("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,0]" : "+v"(acc[k]) : "v"(h[k][d]), "v"(wv[t][8 * u + 2 * d]));
#pragma unroll
            for (int k = 0; k < NBK; ++k)
              asm("v_fma_mix_f32 %0, %1, %2, %0 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
                  : "+v"(acc[k]) : "v"(h[k][d]), "v"(wv[t][8 * u + 2 * d + 1]));
          }
#pragma unroll
          for (int e = 0; e < 2; ++e) {
#pragma unroll
            for (int k = 0; k < NBK; ++k) {
              const f32x2 l0 = __builtin_amdgcn_cvt_pk_f32_fp8((int)lo[k][e], false);
              const f32x2 l1 = __builtin_amdgcn_cvt_pk_f32_fp8((int)lo[k][e], true);
              accl[k] = __builtin_elementwise_fma(f32x2{wv[t][8 * u + 4 * e], wv[t][8 * u + 4 * e + 1]}, l0, accl[k]);
              accl[k] = __builtin_elementwise_fma(f32x2{wv[t][8 * u + 4 * e + 2], wv[t][8 * u + 4 * e + 3]}, l1, accl[k]);
            }
          }
        }
      }
#pragma unroll
      for (int k = 0; k < NBK; ++k)
        out[k] = (double)quarter_sum(fmaf(accl[k][0] + accl[k][1], H8_LO_DIV, acc[k])) + (double)bias;
    } else {
#pragma unroll
    for (int k = 0; k < NBK; ++k) {
      float acc = 0.f;
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const int pr = TG::row(128 * k + 16 * w + c16 + t - 1);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int sl = 4 * u + q;
          f32x4 v0, v1;
          {
            typedef typename Op<MODE>::V8 V8;
            const V8 h = *(const V8*)(tl.lds + off_f32(pr, 16 * sl));
            v0 = __builtin_convertvector(__builtin_shufflevector(h, h, 0, 1, 2, 3), f32x4);
            v1 = __builtin_convertvector(__builtin_shufflevector(h, h, 4, 5, 6, 7), f32x4);
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            acc = fmaf(wv[t][8 * u + e], v0[e], acc);
            acc = fmaf(wv[t][8 * u + 4 + e], v1[e], acc);
          }
        }
      }
      out[k] = (double)quarter_sum(acc) + (double)bias;
    }
    }
  } else {
    static_assert(TG::WB <= HEAD_ROWS * THREADS, "head rows per thread");
#pragma unroll
    for (int k = 0; k < HEAD_ROWS; ++k) {
      const int j = opaque_tid() + THREADS * k;
      out[k] = 0.0;
      if (j >= TG::WB) continue;
      double a = (double)hw[192];
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const int prow = TG::row(j + t - 1);
#pragma unroll 4
        for (int cb = 0; cb < 16; ++cb) {
          const f32x4 v = Op<MODE>::load4(tl.lds, prow, 4 * cb);
#pragma unroll
          for (int i = 0; i < 4; ++i) a = fma((double)hw[3 * (cb * 4 + i) + t], (double)v[i], a);
        }
      }
      out[k] = a;
    }
  }
}
template <int N>
__device__ __forceinline__ void round_rows(const double (&d)[N], float (&f)[N]) {
#pragma unroll
  for (int k = 0; k < N; ++k) f[k] = (float)d[k];
}

// LDS-only workgroup barrier: waits for this wave's LDS traffic, NOT for its outstanding global
// loads (the prefetched weights stay in flight across it).  One asm statement, so the compiler
// cannot move memory accesses across the barrier either.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Work split of one layer (512 rows x 64 couts) over the 8 waves: wave w owns the M-tile pair
// {2mp, 2mp+1} (mp = w & 1, 32 couts) and, in each of the 4 row blocks of 128, the 32 rows
// 128j + 32nq + [0, 32) (nq = w >> 1, 2 N-tiles).  Every B fragment read from LDS feeds both
// M-tiles (2 x 3 split-bf16 MFMAs), so each activation row is read by 2 waves, not 4.
constexpr int IP_MT = 2, IP_NT = 2, IP_NB = 4, IP_BR = WB / IP_NB;

// A-operands (this wave's weights) of a whole layer: [M-tile][k-step].  Loaded once per layer
// from L2 (the four waves of a pair hit the same lines at the same time: mostly L1 hits); the
// next layer's k-step s is fetched right after its last use in the current layer.
template <int MODE>
struct LayerA {
  typename Op<MODE>::A v[IP_MT][Op<MODE>::KSTEPS];
  f32x4 bias[IP_MT];           // lane quarter q's 4 output channels of each M-tile (accumulator init)
  uint32_t sc[IP_MT];          // MODE_H8: E8M0 scales of the correction fragments (byte t = tap t)
  __device__ __forceinline__ typename Op<MODE>::A (&operator[](int mm))[Op<MODE>::KSTEPS] { return v[mm]; }
};

template <int MODE>
__device__ __forceinline__ f32x4 load_bias(const uint8_t* wl, int m) {
  return *(const f32x4*)(wl + LayerBytes<MODE>::BIAS + (16 * m + 4 * ((__builtin_amdgcn_workitem_id_x() & 63) >> 4)) * 4);
}
template <int MODE>
__device__ __forceinline__ uint32_t load_scale(const uint8_t* wl, int m) {
  return MODE == MODE_H8 ? ((const uint32_t*)(wl + H8_SCALE_OFF))[m * 64 + (__builtin_amdgcn_workitem_id_x() & 63)] : 0u;
}

template <int MODE, bool SOUTER = false>
__device__ __forceinline__ void load_layer_a(const Tile& tl, int layer, LayerA<MODE>& a) {
  const int tid = opaque_tid(), mp = (tid >> 6) & 1, lane = tid & 63;
  const uint8_t* wl = tl.big + (size_t)layer * LayerBytes<MODE>::BYTES;
  if constexpr (SOUTER) {            // k-step outer: the first k-step's fragments of both M-tiles first
#pragma unroll
    for (int mm = 0; mm < IP_MT; ++mm) a.bias[mm] = load_bias<MODE>(wl, IP_MT * mp + mm), a.sc[mm] = load_scale<MODE>(wl, IP_MT * mp + mm);
#pragma unroll
    for (int s = 0; s < Op<MODE>::KSTEPS; ++s)
#pragma unroll
      for (int mm = 0; mm < IP_MT; ++mm) a[mm][s] = Op<MODE>::load_a(wl, IP_MT * mp + mm, s, lane);
    return;
  }
#pragma unroll
  for (int mm = 0; mm < IP_MT; ++mm) {
    a.bias[mm] = load_bias<MODE>(wl, IP_MT * mp + mm);
    a.sc[mm] = load_scale<MODE>(wl, IP_MT * mp + mm);
#pragma unroll
    for (int s = 0; s < Op<MODE>::KSTEPS; ++s) a[mm][s] = Op<MODE>::load_a(wl, IP_MT * mp + mm, s, lane);
  }
}

// Compensated fp32 accumulation (MODE_F32): the exact-fp32 MFMA is a k-ordered fmaf chain, one
// rounding per product, and over the 192-term reduction those roundings (not the fp32 storage of
// the activations) dominate the error: a plain chain is ~8e-6 from the float64 forward on trained
// RRCDNet, as far as the fp32 reference itself, so the two differ by up to 1.3e-5.  The chain is
// therefore cut into chunks of RDN_F32_CHUNK k-steps (64 products); each chunk's sum is added to a
// running total by an error-free TwoSum and the rounding error is injected as the next chunk's
// accumulator start (no extra VGPRs over two plain partial sums).  CPU emulation of this exact
// scheme: 4e-6 from the float64 forward (tools/precision_sweep.py --fp32).
#ifndef RDN_F32_COMP
#define RDN_F32_COMP 1
#endif
#ifndef RDN_F32_CHUNK
#define RDN_F32_CHUNK 4
#endif
// hi + c = s + e exactly (Knuth TwoSum, 6 flops); hi <- s, c <- e.  Scalar ops on purpose (packed
// f32 VALU next to MFMAs costs more than it saves, MI355X_MICROARCH.md cycle constants).
__device__ __forceinline__ void two_sum(f32x4& hi, f32x4& c) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float a = hi[k], b = c[k];
    const float s = a + b;
    const float bb = s - a;
    const float e = (a - (s - bb)) + (b - bb);
    hi[k] = s;
    c[k] = e;
  }
}

// One Conv1d(64,64,3,d) over the tile, updated in place with a one-block lag.
//
// Block j reads input rows down to 128j - d, i.e. the tail of block j-1, so block j-1's outputs
// may overwrite their rows only once EVERY wave has finished block j: the barrier after block j.
// They are then written while block j+1 computes (after its first k-step), so the LDS stores and
// their epilogue VALU overlap the MFMA stream instead of forming a separate write phase.
// Sequence: C0 | C1 | S0+C2 | S1+C3 | S2 S3 |.   id[16] = [block][N-tile][M-tile] identities.
// EDGE = false: the tile holds no position outside [0, L) (interior tiles of a spectrum), so the
// write-back skips the per-row zeroing.
// MODE_H8 per-layer correction (RDN_F16F8: every layer; RDN_F16MIX: the layers of the blob's mask,
// CORR_SLOT): cin = this layer reads the e4m3 planes and runs the correction MFMA, otherwise only
// the f16 product (one MFMA per product); cout = its output is written with the e4m3 planes, which
// the next layer needs if it is corrected, and every reader of load4 (head, identity re-add, CBAM)
// needs: `out_full` marks such a last conv.  Both are wave-uniform (scalar branches).
// MODE_H8 per-layer correction (RDN_F16F8: every layer; RDN_F16MIX: RRCDNet's calibrated tail):
// CIN = this layer reads the e4m3 planes and runs the correction MFMA, otherwise only the f16
// product (one MFMA per product); COUT = its output is written with the e4m3 planes, which the next
// layer needs if it is corrected and every load4 reader (head, identity re-add, CBAM) needs; LOADC =
// the next layer's e4m3 weight fragments are prefetched (only a corrected layer reads them).  All
// three are template parameters: as wave-uniform runtime branches inside the k-step stream they cost
// the all-corrected kernel 18 % and the uncorrected one 38 % (measured), and a per-layer runtime
// dispatch between instantiations inside one loop made the compiler spill 1,400-8,000 VGPRs, so a
// mixed network is written as straight runs of one instantiation each (fused_inplace.hip).
// WALK (WalkGeo, the RDN_F16MIX walk): taps at rows r - 2d, r - d, r, outputs dil positions further
// left than the inputs (tl.base), and the carry rows: the last wave (a) fills the carry rows in front
// from this layer's slot (written by the previous tile; zeros on a spectrum's first tile) once block 0,
// their only reader, is done, and (b) saves the input's last 2 dn_prev rows into the previous layer's
// slot for the next tile before the last block's write-back overwrites them (fused16.hpp layer_carry).
template <int MODE, int EPI, int S, bool EDGE = true, int NBK = 4, bool CIN = true, bool COUT = true,
          bool LOADC = true, bool WALK = false>
__device__ __forceinline__ void conv(Tile& tl, int dil, f32x4 (&id)[16 * NBK / 4], LayerA<MODE>& a, bool has_next,
                                     const uint8_t* next_rec = nullptr) {
  using O = Op<MODE>;
  constexpr bool cin = MODE != MODE_H8 || CIN;
  constexpr bool cout = MODE != MODE_H8 || COUT;
  using TG = typename GeoOf<NBK, WALK>::T;
  constexpr int NB = NBK, NT = IP_NT, MT = IP_MT, BR = IP_BR;
  constexpr int TS = O::KSTEPS / 3;                  // k-steps per tap
  const int tid = opaque_tid();
  const int lane = tid & 63, w = tid >> 6;
  const int mp = w & 1, nq = w >> 1;
  const int q = lane >> 4, c16 = lane & 15;
  const uint8_t* wcur = tl.big + (size_t)tl.layer * LayerBytes<MODE>::BYTES;
  // the record whose operands has_next prefetches: the next layer's, or next_rec (RDN_F16MIX: the
  // right head's record after the last corrected layer)
  const uint8_t* wnext = next_rec ? next_rec : wcur + LayerBytes<MODE>::BYTES;
  // bf16 modes start the accumulators at the folded bias; exact fp32 keeps the reference's
  // order (sum of products, then + bias) for its 1e-5 parity
  constexpr bool BIAS_INIT = MODE != MODE_F32;
  // S <= 0: one compensated chain (two_sum) of -S k-step chunks (S = 0: RDN_F32_CHUNK)
  constexpr bool COMP = MODE == MODE_F32 && RDN_F32_COMP && S <= 0;
  constexpr int CH = S == 0 ? RDN_F32_CHUNK : -S;
  constexpr int SP = COMP ? 1 : S;                           // MFMA accumulator sets
  f32x4 bias_l[MT];
  uint32_t sc_l[MT];
#pragma unroll
  for (int mm = 0; mm < MT; ++mm) bias_l[mm] = a.bias[mm], sc_l[mm] = a.sc[mm];
  // WalkGeo HALF: the last block holds 64 rows.  RDN_HALF_REMAP = 0: the waves of quarters 2, 3 have no
  // rows there (wave-uniform) and the others run their two N-tiles; RDN_HALF_REMAP = 1: every wave runs
  // ONE N-tile of it, rows 16 nq + [0, 16) (its usual B / store addresses moved by -16 nq rows, a multiple
  // of 16: same swizzle, one address add per access), so the half block costs half a block
  constexpr bool REMAP = TG::HALF && RDN_HALF_REMAP;
  static_assert(!REMAP || MODE == MODE_H8, "the half-block remap is written for the f16 + e4m3 write-back");
  // RDN_TAIL_SWAP: the half block's rows go to the waves of quarters 2-3 (4-7: the younger wave of each
  // SIMD, which finishes the full blocks last), shifted down by 64 rows, and waves 0-3 idle there instead
  // -- with RDN_TAIL_EARLY those fetch the next layer's operands in block NB - 2, where they have slack
  constexpr bool SWAP = TG::HALF && !REMAP && RDN_TAIL_SWAP;
  const bool half_idle = TG::HALF && !REMAP && ((__builtin_amdgcn_readfirstlane(tid >> 6) >> 1) >= 2) != SWAP;
  const uint32_t hsw = SWAP && (__builtin_amdgcn_readfirstlane(tid >> 6) >> 1) >= 2 ? 64u * ROWB_F32 : 0u;
  auto swapped = [&](int j) { return SWAP && j == NB - 1; };
  const bool stag_late = RDN_TAIL_STAG && __builtin_amdgcn_readfirstlane(tid >> 6) >= 4;
  constexpr bool SGB = RDN_TAIL_SGB && !RDN_TAIL_STAG && MODE == MODE_H8 && cin && !(EPI & (ADD_ID | SAVE_ID));
  const uint32_t hoff = REMAP ? (uint32_t)(16 * ROWB_F32) * (uint32_t)__builtin_amdgcn_readfirstlane(nq) : 0u;
  // the remapped block's rows of this wave start 16 nq, not 32 nq, rows into it
  auto remapped = [&](int j) { return REMAP && j == NB - 1; };
  typedef unsigned int u32x4c __attribute__((ext_vector_type(4)));
  u32x4c carry_a = {0u, 0u, 0u, 0u}, carry_b = {0u, 0u, 0u, 0u};
  const bool cwave = WALK && __builtin_amdgcn_readfirstlane(tid >> 6) == THREADS / 64 - 1;
  if constexpr (WALK) {
    tl.base -= dil;
    if (cwave) {                      // lane = (row k, 16-B slot): 4 rows of 256 B
      const int k = lane >> 4, sl = lane & 15;
      if (k < 2 * tl.dnext && !tl.first) carry_a = *(const u32x4c*)(tl.lds + tl.cs_cur + k * ROWB_F32 + 16 * sl);
      if (k < 2 * tl.dn_prev) {
        const int pr = TG::GRD + TG::WB - 2 * tl.dn_prev + k;
        carry_b = *(const u32x4c*)(tl.lds + pr * ROWB_F32 + ((sl ^ swz256(pr)) << 4));
      }
    }
  }

  // LDS byte addresses of this lane's B fragments for every k-step (row = first row of the wave's
  // share of block 0), and of its output stores; blocks and N-tiles add multiples of 16 rows,
  // which leave the row swizzle unchanged (-> ds_* immediate offsets).
  uint32_t badr[O::KSTEPS][O::PLANES], sadr[MT][O::PLANES];
  const int prow0 = TG::GRD + (BR / 4) * nq + c16;
#pragma unroll
  for (int s = 0; s < O::KSTEPS; ++s) {
    const int pr = prow0 + (O::tap(s) - (WALK ? 2 : 1)) * dil;  // < 0 (wave 0, tap 0) only in WRAP geometry: block 0 uses bfirst
#pragma unroll
    for (int p = 0; p < O::PLANES; ++p) badr[s][p] = pr * ROWB_F32 + ((O::bslot(s, q, p) ^ swz256(pr)) << 4);
  }
  // WRAP: the taps that can leave the tile -- tap 0 of block 0, N-tile 0 (waves nq = 0) and tap 2 of
  // the last block, last N-tile (nq = 3) -- read through wrapped absolute addresses
  uint32_t bfirst[TS][O::PLANES], blast[TS][O::PLANES];
  if (TG::WRAP) {
    const int pf = TG::row(prow0 - dil), pl = TG::row(prow0 + BR * (NB - 1) + 16 * (NT - 1) + dil);
#pragma unroll
    for (int s = 0; s < TS; ++s)
#pragma unroll
      for (int p = 0; p < O::PLANES; ++p) {
        bfirst[s][p] = pf * ROWB_F32 + ((O::bslot(s, q, p) ^ swz256(pf)) << 4);
        blast[s][p] = pl * ROWB_F32 + ((O::bslot(2 * TS + s, q, p) ^ swz256(pl)) << 4);
      }
  }
  // a second set of B addresses 64 KiB up: blocks 2 and 3 then fit the 16-bit ds_read offset
  // (no v_add per read); block 4 still adds
  uint32_t badr2[O::KSTEPS][O::PLANES];
#pragma unroll
  for (int s = 0; s < O::KSTEPS; ++s)
#pragma unroll
    for (int p = 0; p < O::PLANES; ++p) {
      badr2[s][p] = badr[s][p] + 2 * BR * ROWB_F32;
      asm volatile("" : "+v"(badr2[s][p]));         // a register of its own, not re-derived per read
    }
  auto ldb = [&](const uint32_t (&ad)[O::PLANES], uint32_t off) -> typename O::B {
    if constexpr (MODE == MODE_H8) return O::load_b_at(tl.lds, ad, off, cin);
    else return O::load_b_at(tl.lds, ad, off);
  };
  auto read_b = [&](int j, int s, int i) -> typename O::B {
    if (TG::WRAP && j == 0 && s < TS && i == 0) return ldb(bfirst[s], 0);
    if (TG::WRAP && j == NB - 1 && s >= 2 * TS && i == NT - 1) return ldb(blast[s - 2 * TS], 0);
    if (remapped(j)) return ldb(j >= 2 ? badr2[s] : badr[s], (uint32_t)(BR * (j >= 2 ? j - 2 : j)) * ROWB_F32 - hoff);
    if (swapped(j)) return ldb(badr2[s], (uint32_t)(BR * (j - 2) + 16 * i) * ROWB_F32 - hsw);
    if (j >= 2) return ldb(badr2[s], (uint32_t)(BR * (j - 2) + 16 * i) * ROWB_F32);
    return ldb(badr[s], (uint32_t)(BR * j + 16 * i) * ROWB_F32);
  };
#pragma unroll
  for (int mm = 0; mm < MT; ++mm)
#pragma unroll
    for (int p = 0; p < O::PLANES; ++p) {
      const int b = O::sbyte(16 * (MT * mp + mm) + 4 * q, p);
      sadr[mm][p] = prow0 * ROWB_F32 + ((((b >> 4) ^ swz256(prow0)) << 4) | (b & 15));
    }

  f32x4 res[NB][NT][MT];
#if defined(RDN_HYB_STAMPS) && RDN_HYB_STAMPS
  // diagnostic (tools/hyb_stamps.py, walk): wave 0's time per block of each corrected walk layer, from
  // the layer's start (block 0 includes the operand wait) to each block's barrier, then the last two
  // write-backs; summed into the status workspace's words 16 + j (one atomic per block and layer)
  unsigned long long bst_t = __builtin_amdgcn_s_memtime(), bst[NB + 1];
#pragma unroll
  for (int k = 0; k <= NB; ++k) bst[k] = 0;
  auto bstamp = [&](int k) {
    const unsigned long long nt = __builtin_amdgcn_s_memtime();
    bst[k] += nt - bst_t;
    bst_t = nt;
  };
#else
  auto bstamp = [&](int) {};
#endif
  // write-back of N-tile i, M-tile mm of block j (bias / identity, ReLU, zero padding, round)
  auto store_piece = [&](int j, int i, int mm) {
    const int rb = BR * j + (BR / 4) * nq;            // first row of this wave's share of block j
    const bool inside = !EDGE || (tl.base + rb >= 0 && tl.base + rb + BR / 4 <= tl.L);
    const int row = rb + 16 * i + c16;
    const bool zero = !inside && !in_range(tl.base + row, tl.L);         // conv zero padding
    f32x4 v = res[j][i][mm];
    if (!BIAS_INIT && !COMP) v += bias_l[mm];
    if (EPI & ADD_ID) v += id[(j * NT + i) * MT + mm];
    if (EPI & RELU) v = __builtin_elementwise_max(v, f32x4{0.f, 0.f, 0.f, 0.f});
    if (EDGE && zero) v = f32x4{0.f, 0.f, 0.f, 0.f};
    if (EPI & SAVE_ID) id[(j * NT + i) * MT + mm] = v;
#if defined(RDN_ABLATE_NOSTORE)
    if (v[0] == 123456.f)
#endif
    O::store4_at(tl.lds, sadr[mm], (uint32_t)(BR * j + 16 * i) * ROWB_F32, v);
  };
  // MODE_H8: both M-tiles of N-tile i in one write-back, 16-B f16 slot + two 8-B e4m3 slots (3
  // stores instead of 6); ReLU folded into the saturating med3
  auto store_pair = [&](int j, int i) {
    if constexpr (MODE == MODE_H8) {                // (instantiated in every mode, called in MODE_H8)
      const int rb = BR * j + (remapped(j) ? 16 : BR / 4) * nq - (swapped(j) ? 64 : 0);
      const bool inside = !EDGE || (tl.base + rb >= 0 && tl.base + rb + (remapped(j) ? 16 : BR / 4) <= tl.L);
      const bool zero = !inside && !in_range(tl.base + rb + 16 * i + c16, tl.L);
      if (!cout) {                 // plain f16 output (the next layer is uncorrected): no e4m3 planes
        f16x4 hv[MT];
  #pragma unroll
        for (int mm = 0; mm < MT; ++mm) {
          f32x4 v = res[j][i][mm];
          if (EPI & ADD_ID) v += id[(j * NT + i) * MT + mm];
          if (EPI & RELU) v = __builtin_elementwise_max(v, f32x4{0.f, 0.f, 0.f, 0.f});
          if (EDGE && zero) v = f32x4{0.f, 0.f, 0.f, 0.f};
          if (EPI & SAVE_ID) id[(j * NT + i) * MT + mm] = v;
          hv[mm] = __builtin_convertvector(v, f16x4);
        }
        *(f16x8*)(tl.lds + sadr[0][0] + (uint32_t)(BR * j + 16 * i) * ROWB_F32 - (remapped(j) ? hoff : 0u) - (swapped(j) ? hsw : 0u)) =
            __builtin_shufflevector(hv[0], hv[1], 0, 1, 2, 3, 4, 5, 6, 7);
        return;
      }
      H8Split x[MT];
  #pragma unroll
      for (int mm = 0; mm < MT; ++mm) {
        f32x4 v = res[j][i][mm];
        if (EPI & ADD_ID) v += id[(j * NT + i) * MT + mm];
        if (EDGE && zero) v = f32x4{0.f, 0.f, 0.f, 0.f};      // the range guard sees rows in [0, L) only
        h8_track<(EPI & RELU) != 0>(tl.amax, v);
        v = (EPI & RELU) ? h8_sat<true>(v) : h8_sat<false>(v);
        if (EPI & SAVE_ID) id[(j * NT + i) * MT + mm] = v;
        x[mm] = h8_split(v);
      }
      const uint32_t off = (uint32_t)(BR * j + 16 * i) * ROWB_F32 - (remapped(j) ? hoff : 0u) - (swapped(j) ? hsw : 0u);
      typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  #if defined(RDN_ABLATE_NOSTORE)
      if (x[0].hi8 == 0x12345678u)
  #endif
      {
        *(f16x8*)(tl.lds + sadr[0][0] + off) = __builtin_shufflevector(x[0].hi, x[1].hi, 0, 1, 2, 3, 4, 5, 6, 7);
        *(u32x2*)(tl.lds + sadr[0][1] + off) = u32x2{x[0].hi8, x[1].hi8};
        *(u32x2*)(tl.lds + sadr[0][2] + off) = u32x2{x[0].lo8, x[1].lo8};
      }
    }
  };
  // (walk, a spectrum's short last tiles) block j's rows all lie 8 or more positions beyond L: no
  // output inside [0, L) reaches them within the remaining corrected layers and the head (d = 1: 6
  // positions), so the block skips its MFMAs, B reads and write-back (its rows keep older values,
  // which only feed rows beyond L: never stored, never tracked by the range guard)
  auto beyond = [&](int j) { return WALK && EDGE && tl.base + BR * j >= tl.L + 8; };
  // the block whose k-steps retire this layer's operands, after which the next layer's are fetched: the
  // last block; RDN_TAIL_EARLY: for the waves that own no rows of a last half block, the block before
  // (their last use), so half of the CU's operand loads -- bound by the texture path, ~3k cycles per
  // corrected layer -- leave a block earlier instead of queueing with the others' in the half block
  auto load_next = [&](int j) {
    if constexpr (RDN_TAIL_EARLY && TG::HALF && !REMAP) return half_idle ? j == NB - 2 : j == NB - 1;
    return j == NB - 1;
  };
  auto store_block = [&](int j) {
    if ((j == NB - 1 && half_idle) || beyond(j)) return;
    if constexpr (MODE == MODE_H8) {
#pragma unroll
      for (int i = 0; i < (remapped(j) ? 1 : NT); ++i) store_pair(j, i);
    } else {
#pragma unroll
      for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int mm = 0; mm < MT; ++mm) store_piece(j, i, mm);
    }
  };

  // B fragments are software-pipelined one k-step ahead: the reads for k-step s+1 are issued
  // before the MFMAs of k-step s, so LDS latency hides under 2 x 3 x 16-cycle MFMA chains; the
  // first k-step of block j+1 is read before the barrier that ends block j (its rows are not
  // among those the write-backs around that barrier touch: blocks j-2 and j-1).
  typename O::B bnext[NT];
#pragma unroll
  for (int i = 0; i < NT; ++i) bnext[i] = read_b(0, 0, i);
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const bool skip = (j == NB - 1 && half_idle) || beyond(j);   // no rows of this wave / none needed
    f32x4 part[SP][NT][MT];
    f32x4 hi[COMP ? NT : 1][COMP ? MT : 1];          // COMP: running total, starts at the bias
#pragma unroll
    for (int k = 0; k < SP; ++k)
#pragma unroll
      for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int mm = 0; mm < MT; ++mm)
          part[k][i][mm] = k == 0 && BIAS_INIT ? a.bias[mm] : f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (COMP) {
#pragma unroll
      for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int mm = 0; mm < MT; ++mm) hi[i][mm] = bias_l[mm];
    }
    if (has_next && (RDN_TAIL_EARLY >= 2 ? j == NB - 1 : load_next(j))) {   // last use of this layer's bias
#pragma unroll
      for (int mm = 0; mm < MT; ++mm) a.bias[mm] = load_bias<MODE>(wnext, MT * mp + mm), a.sc[mm] = load_scale<MODE>(wnext, MT * mp + mm);
    }
    // B fragments rotate per N-tile: the reads of N-tile i for the next k-step (or for k-step 0 of
    // block j+1) are issued as soon as its MFMAs of this k-step are issued, so they fly under the
    // MFMAs of the other N-tile(s) instead of trailing the whole k-step -- same VGPRs as one set.
#pragma unroll
    for (int s = 0; s < O::KSTEPS; ++s) {
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        if (!skip && !(remapped(j) && i > 0)) {
#pragma unroll
        for (int mm = 0; mm < MT; ++mm) {
          if constexpr (MODE == MODE_H8 && !(EPI & (ADD_ID | SAVE_ID))) {
            // the M-tiles' chains interleaved (e4m3 MFMAs, then each f16 half): no MFMA issues right
            // behind the one whose result it adds to (+0.8 % on the hybrid, bit-equal: each chain keeps
            // its order; the f16 MFMAs ahead of the e4m3 one cost 6 %, ablate_m.log).  Not on the
            // residual convs, whose identity VGPRs leave no room for the longer live ranges (DSDN
            // f16f8 spilled 5 more VGPRs)
            if (mm > 0) break;
            if (cin) {
#pragma unroll
              for (int m2 = 0; m2 < MT; ++m2) part[s % SP][i][m2] = O::mma_c(a[m2][s], bnext[i], part[s % SP][i][m2], sc_l[m2], s);
            }
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
              for (int m2 = 0; m2 < MT; ++m2) part[s % SP][i][m2] = O::mma_h(a[m2][s], bnext[i], part[s % SP][i][m2], u);
          } else if constexpr (MODE == MODE_H8) {
            part[s % SP][i][mm] = O::mma(a[mm][s], bnext[i], part[s % SP][i][mm], sc_l[mm], s, cin);
          } else {
            part[s % SP][i][mm] = O::mma(a[mm][s], bnext[i], part[s % SP][i][mm], sc_l[mm], s);
          }
        }
        if (s + 1 < O::KSTEPS) bnext[i] = read_b(j, s + 1, i);
        else if (j + 1 < NB && !(j + 1 == NB - 1 && half_idle) && !(remapped(j + 1) && i > 0)) bnext[i] = read_b(j + 1, 0, i);
        }
        if constexpr (SGB) {
          if (i == NT - 1 && j >= 2 && s < NT && !beyond(j - 2)) {
            store_pair(j - 2, s);
            // MFMA, B read, V VALU (x4), MFMA, V VALU (x2), the three plane stores
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
              __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
              __builtin_amdgcn_sched_group_barrier(0x002, RDN_TAIL_SGB, 0);
            }
#pragma unroll
            for (int g = 0; g < 2; ++g) {
              __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
              __builtin_amdgcn_sched_group_barrier(0x002, RDN_TAIL_SGB, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x200, 3, 0);
          }
        }
        if constexpr (COMP) {
          // fold a finished chunk into the running totals (the rounding error becomes the next
          // chunk's accumulator start), staggered by one N-tile so that the VALU neither waits for
          // the MFMAs it reads nor holds back the MFMAs that read it: N-tile i < NT-1 right after
          // N-tile i+1's MFMAs of the chunk's last k-step, the last N-tile right after N-tile 0's
          // MFMAs of the next k-step
          const bool chunk_end = s % CH == CH - 1 && s + 1 < O::KSTEPS;
          const bool chunk_next = s % CH == 0 && s > 0;
          if (chunk_end && i > 0) {
#pragma unroll
            for (int mm = 0; mm < MT; ++mm) two_sum(hi[i - 1][mm], part[0][i - 1][mm]);
          }
          if (chunk_next && i == 0) {
#pragma unroll
            for (int mm = 0; mm < MT; ++mm) two_sum(hi[NT - 1][mm], part[0][NT - 1][mm]);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
#if defined(RDN_ABLATE_NOALOAD_TAIL)       // diagnostic builds only (tools/ablate.py): wrong results
      if (has_next && load_next(j) && tl.layer < 0) {
#else
      if (has_next && (RDN_TAIL_EARLY == 3 && s > 0 ? j == NB - 1 : load_next(j))) {   // last use of a[.][s]
#endif
#pragma unroll
        for (int mm = 0; mm < MT; ++mm) {
          if constexpr (MODE == MODE_H8 && !LOADC) O::load_a_main(wnext, MT * mp + mm, s, lane, a[mm][s]);
          else a[mm][s] = O::load_a(wnext, MT * mp + mm, s, lane);
        }
      }
      if (WALK && j == 1 && s == 0 && cwave) {         // block 0 (the carry rows' reader) is done
        const int k = lane >> 4, sl = lane & 15;
        if (k < 2 * tl.dnext) {
          const int pr = TG::GRD - 2 * tl.dnext + k;
          *(u32x4c*)(tl.lds + pr * ROWB_F32 + ((sl ^ swz256(pr)) << 4)) = carry_a;
        }
        if (k < 2 * tl.dn_prev) *(u32x4c*)(tl.lds + tl.cs_prev + k * ROWB_F32 + 16 * sl) = carry_b;
      }
      if (j >= 2 && !beyond(j - 2)) {
        constexpr int NP = NT * MT;
        if constexpr (MODE == MODE_H8 && RDN_TAIL_STAG) {
          // waves 4-7 (row quarters 2-3) share their SIMDs with waves 0-3: their write-backs run one
          // k-step later, so the two waves of a SIMD do not issue their e4m3-split VALU together
          if (!stag_late) {
            if (s < NT) store_pair(j - 2, s);
          } else if (s >= 1 && s - 1 < NT) {
            store_pair(j - 2, s - 1);
          }
        } else if constexpr (MODE == MODE_H8) {
          if (!SGB && s < NT) store_pair(j - 2, s);
        } else if constexpr (O::KSTEPS >= NP) {
          if (s < NP) store_piece(j - 2, s / MT, s % MT);
        } else {
#pragma unroll
          for (int pc = s * NP / O::KSTEPS; pc < (s + 1) * NP / O::KSTEPS; ++pc) store_piece(j - 2, pc / MT, pc % MT);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int mm = 0; mm < MT; ++mm) {
        f32x4 v = part[0][i][mm];
        if constexpr (COMP) {
          v = hi[i][mm] + v;                          // total + last chunk (+ pending error): one rounding
        } else {
#pragma unroll
          for (int k = 1; k < SP; ++k) v += part[k][i][mm];
        }
        res[j][i][mm] = v;
      }
#if defined(RDN_HYB_STAMPS) && RDN_HYB_STAMPS
    const unsigned long long pre_b = __builtin_amdgcn_s_memtime();
#endif
#if defined(RDN_ABLATE_NOBARRIER)         // diagnostic builds only (tools/ablate.py): wrong results
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#else
    lds_barrier();                 // every wave is done reading the rows block j needed
#endif
#if defined(RDN_HYB_STAMPS) && RDN_HYB_STAMPS
    if (WALK && MODE == MODE_H8) {
      const unsigned long long post_b = __builtin_amdgcn_s_memtime();
      tl.bwork += pre_b - bst_t;
      tl.bwait += post_b - pre_b;
    }
#endif
    bstamp(j);
  }
  store_block(NB - 2);
  store_block(NB - 1);
#if defined(RDN_HYB_STAMPS) && RDN_HYB_STAMPS
  const unsigned long long pre_s = __builtin_amdgcn_s_memtime();
#endif
  lds_barrier();                   // the layer's output is complete
#if defined(RDN_HYB_STAMPS) && RDN_HYB_STAMPS
  if (WALK && MODE == MODE_H8) {
    tl.bwork += pre_s - bst_t;
    tl.bwait += __builtin_amdgcn_s_memtime() - pre_s;
  }
#endif
  bstamp(NB);
#if defined(RDN_HYB_STAMPS) && RDN_HYB_STAMPS
  if (WALK && MODE == MODE_H8 && tl.status && tid == 0) {
#pragma unroll
    for (int k = 0; k <= NB; ++k) atomicAdd((unsigned long long*)tl.status + 16 + k, bst[k]);
  }

#endif
  tl.layer += 1;
  if constexpr (WALK) {
    tl.cs_prev = tl.cs_cur;
    tl.dn_prev = tl.dnext;
    tl.cs_cur += 2 * tl.dnext * ROWB_F32;
  }
}

// Conv1d(64, 1, 3) head on the MFMA for the f16 + e4m3 tile (RDN_F16MIX RRCDNet's right head): the
// corrected layer product W.X ~= W_hi.X_hi + [W_lo | W_hi].[X_hi | X_lo] with one meaningful output
// channel, whose record (pack.cpp pack_head_h8mfma) holds the head at couts 0 and 32, so the operands
// a conv prefetched for M-tile 2 mp of every wave (a[0], its bias and scales) are the head's.  Rows
// as HeadOut<MODE_H8, NBK> (N-tile 8k + w, row 128k + 16w + c16): out[k] on the lanes of quarter 0,
// which HeadOut::writer() selects.  Replaces the VALU head (48 per-lane weight loads, 16 channels x 3
// taps of fma_mix / e4m3-decode FMAs per row and lane, a cross-quarter sum: 12.9k cycles per tile in
// the hybrid, tools/hyb_stamps.py) by 9 MFMAs and 12 conflict-free B reads per row block.
// WALK: taps r - 2, r - 1, r, outputs one position further left; the last wave saves the input's last
// 2 rows into its carry slot (conv's (b)).
template <int NBK, bool WALK = false>
__device__ __forceinline__ void head_h8_mfma(Tile& tl, const LayerA<MODE_H8>& a, float (&out)[NBK]) {
  using O = Op<MODE_H8>;
  using TG = typename GeoOf<NBK, WALK>::T;
  const int tid = opaque_tid(), lane = tid & 63, w = tid >> 6, q = lane >> 4, c16 = lane & 15;
  if constexpr (WALK) {
    tl.base -= 1;
    if (__builtin_amdgcn_readfirstlane(w) == THREADS / 64 - 1) {
      typedef unsigned int u32x4c __attribute__((ext_vector_type(4)));
      const int k = lane >> 4, sl = lane & 15;
      if (k < 2 * tl.dn_prev) {
        const int pr = TG::GRD + TG::WB - 2 * tl.dn_prev + k;
        *(u32x4c*)(tl.lds + tl.cs_prev + k * ROWB_F32 + 16 * sl) = *(const u32x4c*)(tl.lds + pr * ROWB_F32 + ((sl ^ swz256(pr)) << 4));
      }
    }
  }
  f32x4 acc[NBK];
#pragma unroll
  for (int k = 0; k < NBK; ++k) acc[k] = a.bias[0];
  // WalkGeo HALF: waves 4-7 own no rows of the last, half block (N-tile 8k + w)
  const bool half_idle = TG::HALF && __builtin_amdgcn_readfirstlane(w) >= 4;
#pragma unroll
  for (int s = 0; s < O::KSTEPS; ++s) {
#pragma unroll
    for (int k = 0; k < NBK; ++k) {
      if (k == NBK - 1 && half_idle) continue;
      const typename O::B b = O::load_b(tl.lds, TG::row(128 * k + 16 * w + c16 + s - (WALK ? 2 : 1)), s, q);
      acc[k] = O::mma(a.v[0][s], b, acc[k], a.sc[0], s);
    }
  }
#pragma unroll
  for (int k = 0; k < NBK; ++k) out[k] = acc[k][0];
}

// partial sums per accumulator (S <= 0: one chain with compensated chunk sums, see two_sum): F32
// compensates on the plain stacks (1DCNN, RRCDNet, PIDN; measured on the GPU with RDN_F32_CHUNK = 4:
// trained RRCDNet 1.25e-5 -> 7.4e-6 vs the fp32 reference, 8.1e-6 -> 4.3e-6 vs float64, -8 %
// throughput).  The residual networks keep one plain chain: DSDN holds 64 VGPRs of identity
// (compensated it spills 224 B per lane, -11 %), and on the CBAM networks (CbamGeo, RDN_F32_COMP_RES = 1:
// chunks of RDN_F32_CHUNK_RES k-steps) compensation buys nothing measurable: at inputs x1 - x100 the
// plain chain is already within 0.65x of the reference fp32's own distance from float64, and at x1000
// the CBAM gating is chaotic -- the distance is a draw whose size the summation order sets, not its
// accuracy (APIDN x1000 vs the reference's distance: plain 5.0x, 6-step chunks 1.6x, 4-step 2.0x,
// 3-step 6.1x, 2-step 1.4x; against the fp32 noise floor of tests/test_range_gpu.py the plain chain is
// the closest of all, 0.95x) -- for -2.3 % (6-step) to -5 % (4-step) of fp32 throughput
// (profiles/r05/ablate/fp32_rescomp.log).  Split-bf16 / f16f8 error is dominated by the operand split,
// one chain.
#ifndef RDN_F32_COMP_RES
#define RDN_F32_COMP_RES 0
#endif
#ifndef RDN_F32_CHUNK_RES
#define RDN_F32_CHUNK_RES 4
#endif
template <int MODE, bool RES> struct Geo { static constexpr int S = 1; };
template <> struct Geo<MODE_F32, false> { static constexpr int S = RDN_F32_COMP ? 0 : 2; };
template <int MODE> struct CbamGeo { static constexpr int S = 1; };
template <> struct CbamGeo<MODE_F32> { static constexpr int S = RDN_F32_COMP && RDN_F32_COMP_RES ? -RDN_F32_CHUNK_RES : 1; };

// the blob's per-layer correction mask (common.hpp CORR_SLOT), a scalar load
__device__ __forceinline__ uint64_t corr_mask(const uint8_t* blob) {
  const cfloat* p = (const cfloat*)(blob + CORR_SLOT * SMALL_SLOT_FLOATS * 4);
  const uint32_t lo = __float_as_uint(p[0]), hi = __float_as_uint(p[1]);
  return (uint64_t)hi << 32 | lo;
}

// tile `id` = (spectrum n, tile index within it) of a launch: workgroup `id` of a one-tile-per-workgroup
// grid, or the persistent kernels' loop index
__device__ __forceinline__ Tile make_tile_at(char* lds, const uint8_t* blob, const float* x, int L, int T, int tiles,
                                             int halo, int64_t id, int& n_out) {
  const int n = (int)(id / tiles), tile = (int)(id - (int64_t)n * tiles);
  n_out = n;
  Tile tl;
  tl.lds = lds;
  tl.x = x + (size_t)n * L;
  tl.L = L;
  tl.base = tile * T - halo;
  tl.small = (const float*)blob;
  tl.big = blob + SMALL_BYTES;
  tl.layer = 0;
  tl.corr = corr_mask(blob);
  tl.amax = 0.f;
  tl.status = nullptr;
  return tl;
}
__device__ __forceinline__ Tile make_tile(char* lds, const uint8_t* blob, const float* x, int L, int T,
                                          int tiles, int halo, int& n_out) {
  return make_tile_at(lds, blob, x, L, T, tiles, halo, __builtin_amdgcn_workgroup_id_x(), n_out);
}

// End-of-tile range vote of the MODE_H8 kernels (h8_track): whether any lane of the workgroup saw a
// value beyond H8_SAT.  Workgroup-uniform; one LDS word per wave at `vote_off`, which no wave may be
// reading or about to write between the two barriers (callers pass a region their last phase is
// done with).  A saturated tile raises *status (if given: the launch's workspace word, a relaxed
// agent-scope vector store from one lane) and its caller writes NaN outputs.
__device__ __forceinline__ bool range_vote(const Tile& tl, uint32_t vote_off, unsigned* status) {
  unsigned* vote = (unsigned*)(tl.lds + vote_off);
  const int tid = __builtin_amdgcn_workitem_id_x();
  __syncthreads();
  const bool wave_sat = __builtin_amdgcn_ballot_w64(tl.amax > H8_SAT) != 0;
  if ((tid & 63) == 0) vote[tid >> 6] = wave_sat ? 1u : 0u;
  __syncthreads();
  bool sat = false;
#pragma unroll
  for (int k = 0; k < THREADS / 64; ++k) sat = sat || vote[k] != 0;
  __syncthreads();
  if (sat && status && tid == 0) raise_status(status, STATUS_RANGE);
  return sat;
}
// The same vote split around a caller's barrier (the RDN_F16MIX hybrid publishes it with its own
// LDS hand-off, one barrier instead of three): post this wave's word, then -- after a barrier, with
// nothing writing the words again in the tile -- read every wave's
__device__ __forceinline__ void range_vote_post(const Tile& tl, uint32_t vote_off) {
  const int tid = __builtin_amdgcn_workitem_id_x();
  const bool wave_sat = __builtin_amdgcn_ballot_w64(tl.amax > H8_SAT) != 0;
  if ((tid & 63) == 0) ((unsigned*)(tl.lds + vote_off))[tid >> 6] = wave_sat ? 1u : 0u;
}
__device__ __forceinline__ bool range_vote_read(const Tile& tl, uint32_t vote_off, unsigned* status) {
  const unsigned* vote = (const unsigned*)(tl.lds + vote_off);
  bool sat = false;
#pragma unroll
  for (int k = 0; k < THREADS / 64; ++k) sat = sat || vote[k] != 0;
  if (sat && status && __builtin_amdgcn_workitem_id_x() == 0) raise_status(status, STATUS_RANGE);
  return sat;
}
template <int N>
__device__ __forceinline__ void nan_rows(float (&o)[N]) {
#pragma unroll
  for (int k = 0; k < N; ++k) o[k] = __uint_as_float(0x7fc00000u);
}

template <int MODE, int NBK = 4>
__device__ __forceinline__ void store_out(const Tile& tl, float* y, int n, const float (&v)[HeadOut<MODE, NBK>::ROWS],
                                          int halo, int T) {
  using HO = HeadOut<MODE, NBK>;
  if (!HO::writer()) return;
#pragma unroll
  for (int k = 0; k < HO::ROWS; ++k) {
    const int j = HO::row(k);
    const int p = tl.base + j;
    if (j >= halo && j < halo + T && p < tl.L) y[(size_t)n * tl.L + p] = v[k];
  }
}

}  // namespace ip
}  // namespace rdn
