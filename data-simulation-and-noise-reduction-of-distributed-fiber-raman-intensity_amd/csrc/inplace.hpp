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

constexpr int MODE_F32 = 0, MODE_B1 = 1, MODE_X3 = 2;
#ifndef RDN_IP_SPREAD_STORE
#define RDN_IP_SPREAD_STORE 1
#endif
constexpr uint32_t LDS_BYTES = ACT_BYTES_F32;                    // 132096 (512 rows + guards)

// Tile geometry by number of 128-row blocks: NBK = 4 -> 512 rows with 2 zero guard rows per side
// (the CBAM segment kernels, which keep scratch behind the buffer); NBK = 5 -> 640 rows, no guard
// rows, the whole 160 KiB LDS (fused_inplace.hip).  Without guards a tap that leaves the tile
// wraps to its other end: those rows are outside every output's receptive field (the halo covers
// the stack's depth), so any finite value serves; spectrum positions outside [0, L) are re-zeroed
// by the write-backs of edge tiles.
template <int NBK> struct TileGeo {
  static constexpr int WB = 128 * NBK;
  static constexpr bool WRAP = NBK != 4;
  static constexpr int GRD = WRAP ? 0 : GUARD;
  static constexpr uint32_t LDS = (WB + 2 * GRD) * ROWB_F32;
  __device__ static int row(int r) { return WRAP ? (r < 0 ? r + WB : (r >= WB ? r - WB : r)) : r + GRD; }
};
static_assert(TileGeo<4>::LDS == LDS_BYTES, "CBAM geometry");
static_assert(TileGeo<5>::LDS == 163840, "fused geometry fills the LDS");
constexpr int BIG_BYTES = BIG_BYTES_F32;                         // both modes: 49408 B per layer
constexpr int BIAS_OFF = BIG_FRAG_FLOATS_F32 * 4;                // 49152

enum Epi : int { RELU = 1, ADD_ID = 2, SAVE_ID = 4 };

struct Tile {
  char* lds;
  const float* x;
  int L;
  int base;
  const uint8_t* big;
  int layer;
  const float* small;
};

__device__ __forceinline__ bool in_range(int p, int L) { return p >= 0 && p < L; }

// Thread index the compiler cannot treat as loop-invariant: per-lane addresses derived from it are
// recomputed where they are used instead of being hoisted out of the callers' layer / spectrum
// loops (where, with 256 VGPRs taken by the conv, they are spilled to scratch and reloaded).
__device__ __forceinline__ int opaque_tid() {
  int t = threadIdx.x;
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
  __device__ static void store4_at(char* act, const uint32_t (&ad)[PLANES], uint32_t off, f32x4 v) {
    *(f32x4*)(act + ad[0] + off) = v;
  }
  __device__ static f32x4 mma(const A& a, const B& b, f32x4 acc) {
#pragma unroll
    for (int i = 0; i < 4; ++i) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w[i], b.v[i], acc, 0, 0, 0);
    return acc;
  }
  // 4 channels [c0, c0+4) of a row
  __device__ static void store4(char* act, int prow, int c0, f32x4 v) { *(f32x4*)(act + off_f32(prow, 4 * c0)) = v; }
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
  __device__ static void store4_at(char* act, const uint32_t (&ad)[PLANES], uint32_t off, f32x4 v) {
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
  __device__ static f32x4 mma(const A& a, const B& b, f32x4 acc) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.lo, b.hi, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.hi, b.lo, acc, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.hi, b.hi, acc, 0, 0, 0);
  }
  __device__ static void store4(char* act, int prow, int c0, f32x4 v) {
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

// plain bf16 on the same 256-byte rows (used by the CBAM segments): hi plane only, one MFMA.
template <> struct Op<MODE_B1> {
  static constexpr int KSTEPS = 6;
  struct A { bf16x8 hi; };
  struct B { bf16x8 hi; };
  __device__ static A load_a(const uint8_t* layer, int m, int s, int lane) {
    return A{((const bf16x8*)layer)[((m * 6 + s) * 2) * 64 + lane]};
  }
  __device__ static B load_b(const char* act, int prow, int s, int q) {
    return B{*(const bf16x8*)(act + off_f32(prow, 64 * (s & 1) + 16 * q))};
  }
  __device__ static int tap(int s) { return s >> 1; }
  static constexpr int PLANES = 1;
  __device__ static int bslot(int s, int q, int) { return 4 * (s & 1) + q; }
  __device__ static int sbyte(int c0, int) { return 2 * c0; }
  __device__ static B load_b_at(const char* act, const uint32_t (&ad)[PLANES], uint32_t off) {
    return B{*(const bf16x8*)(act + ad[0] + off)};
  }
  __device__ static void store4_at(char* act, const uint32_t (&ad)[PLANES], uint32_t off, f32x4 v) {
    *(bf16x4*)(act + ad[0] + off) = __builtin_convertvector(v, bf16x4);
  }
  __device__ static f32x4 mma(const A& a, const B& b, f32x4 acc) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.hi, b.hi, acc, 0, 0, 0);
  }
  __device__ static void store4(char* act, int prow, int c0, f32x4 v) {
    *(bf16x4*)(act + off_f32(prow, 2 * c0)) = __builtin_convertvector(v, bf16x4);
  }
  __device__ static f32x4 load4(const char* act, int prow, int c0) {
    return __builtin_convertvector(*(const bf16x4*)(act + off_f32(prow, 2 * c0)), f32x4);
  }
};

__device__ __forceinline__ void zero_guards(char* lds) {
  const int t = threadIdx.x;           // 4 guard rows x 256 B = 64 lanes x 16 B
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
__device__ __forceinline__ void stem(const Tile& tl, int slot) {
  using TG = TileGeo<NBK>;
  const cfloat* sw = small_slot(tl, slot);
  for (int j = opaque_tid(); j < TG::WB; j += THREADS) {
  const int pr = TG::row(j);
  const int p = tl.base + j;
  const float xm = in_range(p - 1, tl.L) ? tl.x[p - 1] : 0.f;
  const float x0 = in_range(p, tl.L) ? tl.x[p] : 0.f;
  const float xp = in_range(p + 1, tl.L) ? tl.x[p + 1] : 0.f;
  const bool valid = in_range(p, tl.L);
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
    Op<MODE>::store4(tl.lds, pr, 4 * cb, v);
  }
  }
}

// Conv1d(64, 1, 3, padding=1), one row per thread (row j = threadIdx.x + THREADS * k in out[k]),
// fp32 weights and accumulate.
constexpr int HEAD_ROWS = 2;      // rows per thread: ceil(640 / 512)
template <int MODE, int NBK = 4>
__device__ __forceinline__ void head(const Tile& tl, int slot, float (&out)[HEAD_ROWS]) {
  using TG = TileGeo<NBK>;
  static_assert(TG::WB <= HEAD_ROWS * THREADS, "head rows per thread");
  const cfloat* hw = small_slot(tl, slot);
#pragma unroll
  for (int k = 0; k < HEAD_ROWS; ++k) {
  const int j = opaque_tid() + THREADS * k;
  out[k] = 0.f;
  if (j >= TG::WB) continue;
  float a = hw[192];
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const int prow = TG::row(j + t - 1);
#pragma unroll 4
    for (int cb = 0; cb < 16; ++cb) {
      const f32x4 v = Op<MODE>::load4(tl.lds, prow, 4 * cb);
#pragma unroll
      for (int i = 0; i < 4; ++i) a = fmaf(hw[3 * (cb * 4 + i) + t], v[i], a);
    }
  }
  out[k] = a;
  }
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
  __device__ __forceinline__ typename Op<MODE>::A (&operator[](int mm))[Op<MODE>::KSTEPS] { return v[mm]; }
};

__device__ __forceinline__ f32x4 load_bias(const uint8_t* wl, int m) {
  return *(const f32x4*)(wl + BIAS_OFF + (16 * m + 4 * ((threadIdx.x & 63) >> 4)) * 4);
}

template <int MODE>
__device__ __forceinline__ void load_layer_a(const Tile& tl, int layer, LayerA<MODE>& a) {
  const int tid = opaque_tid(), mp = (tid >> 6) & 1, lane = tid & 63;
  const uint8_t* wl = tl.big + (size_t)layer * BIG_BYTES;
#pragma unroll
  for (int mm = 0; mm < IP_MT; ++mm) {
    a.bias[mm] = load_bias(wl, IP_MT * mp + mm);
#pragma unroll
    for (int s = 0; s < Op<MODE>::KSTEPS; ++s) a[mm][s] = Op<MODE>::load_a(wl, IP_MT * mp + mm, s, lane);
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
template <int MODE, int EPI, int S, bool EDGE = true, int NBK = 4>
__device__ __forceinline__ void conv(Tile& tl, int dil, f32x4 (&id)[16 * NBK / 4], LayerA<MODE>& a, bool has_next) {
  using O = Op<MODE>;
  using TG = TileGeo<NBK>;
  constexpr int NB = NBK, NT = IP_NT, MT = IP_MT, BR = IP_BR;
  constexpr int TS = O::KSTEPS / 3;                  // k-steps per tap
  const int tid = opaque_tid();
  const int lane = tid & 63, w = tid >> 6;
  const int mp = w & 1, nq = w >> 1;
  const int q = lane >> 4, c16 = lane & 15;
  const uint8_t* wcur = tl.big + (size_t)tl.layer * BIG_BYTES;
  const uint8_t* wnext = wcur + BIG_BYTES;
  // bf16 modes start the accumulators at the folded bias; exact fp32 keeps the reference's
  // order (sum of products, then + bias) for its 1e-5 parity
  constexpr bool BIAS_INIT = MODE != MODE_F32;
  f32x4 bias_l[MT];
#pragma unroll
  for (int mm = 0; mm < MT; ++mm) bias_l[mm] = a.bias[mm];

  // LDS byte addresses of this lane's B fragments for every k-step (row = first row of the wave's
  // share of block 0), and of its output stores; blocks and N-tiles add multiples of 16 rows,
  // which leave the row swizzle unchanged (-> ds_* immediate offsets).
  uint32_t badr[O::KSTEPS][O::PLANES], sadr[MT][O::PLANES];
  const int prow0 = TG::GRD + (BR / 4) * nq + c16;
#pragma unroll
  for (int s = 0; s < O::KSTEPS; ++s) {
    const int pr = prow0 + (O::tap(s) - 1) * dil;  // < 0 (wave 0, tap 0) only in WRAP geometry: block 0 uses bfirst
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
  auto read_b = [&](int j, int s, int i) -> typename O::B {
    if (TG::WRAP && j == 0 && s < TS && i == 0) return O::load_b_at(tl.lds, bfirst[s], 0);
    if (TG::WRAP && j == NB - 1 && s >= 2 * TS && i == NT - 1) return O::load_b_at(tl.lds, blast[s - 2 * TS], 0);
    return O::load_b_at(tl.lds, badr[s], (uint32_t)(BR * j + 16 * i) * ROWB_F32);
  };
#pragma unroll
  for (int mm = 0; mm < MT; ++mm)
#pragma unroll
    for (int p = 0; p < O::PLANES; ++p) {
      const int b = O::sbyte(16 * (MT * mp + mm) + 4 * q, p);
      sadr[mm][p] = prow0 * ROWB_F32 + ((((b >> 4) ^ swz256(prow0)) << 4) | (b & 15));
    }

  f32x4 res[NB][NT][MT];
  // write-back of N-tile i, M-tile mm of block j (bias / identity, ReLU, zero padding, round)
  auto store_piece = [&](int j, int i, int mm) {
    const int rb = BR * j + (BR / 4) * nq;            // first row of this wave's share of block j
    const bool inside = !EDGE || (tl.base + rb >= 0 && tl.base + rb + BR / 4 <= tl.L);
    const int row = rb + 16 * i + c16;
    const bool zero = !inside && !in_range(tl.base + row, tl.L);         // conv zero padding
    f32x4 v = res[j][i][mm];
    if (!BIAS_INIT) v += bias_l[mm];
    if (EPI & ADD_ID) v += id[(j * NT + i) * MT + mm];
    if (EPI & RELU) v = __builtin_elementwise_max(v, f32x4{0.f, 0.f, 0.f, 0.f});
    if (EDGE && zero) v = f32x4{0.f, 0.f, 0.f, 0.f};
    if (EPI & SAVE_ID) id[(j * NT + i) * MT + mm] = v;
#if defined(RDN_ABLATE_NOSTORE)
    if (v[0] == 123456.f)
#endif
    O::store4_at(tl.lds, sadr[mm], (uint32_t)(BR * j + 16 * i) * ROWB_F32, v);
  };
  auto store_block = [&](int j) {
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int mm = 0; mm < MT; ++mm) store_piece(j, i, mm);
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
    f32x4 part[S][NT][MT];
#pragma unroll
    for (int k = 0; k < S; ++k)
#pragma unroll
      for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int mm = 0; mm < MT; ++mm)
          part[k][i][mm] = k == 0 && BIAS_INIT ? a.bias[mm] : f32x4{0.f, 0.f, 0.f, 0.f};
    if (j == NB - 1 && has_next) {                    // last use of this layer's bias
#pragma unroll
      for (int mm = 0; mm < MT; ++mm) a.bias[mm] = load_bias(wnext, MT * mp + mm);
    }
#pragma unroll
    for (int s = 0; s < O::KSTEPS; ++s) {
      typename O::B bcur[NT];
#pragma unroll
      for (int i = 0; i < NT; ++i) bcur[i] = bnext[i];
      if (s + 1 < O::KSTEPS) {
#pragma unroll
        for (int i = 0; i < NT; ++i) {
#if defined(RDN_ABLATE_NOLDS)          // diagnostic builds only (tools/ablate.py): reuse block reads
          bnext[i] = bcur[i];
          asm volatile("" : "+v"(reinterpret_cast<f32x4&>(bnext[i])) ::);
#else
          bnext[i] = read_b(j, s + 1, i);
#endif
        }
      }
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        const typename O::B& b = bcur[i];
#pragma unroll
        for (int mm = 0; mm < MT; ++mm) {
#if defined(RDN_ABLATE_NOMFMA)
          part[s % S][i][mm] += *(const f32x4*)&b;
#else
          part[s % S][i][mm] = O::mma(a[mm][s], b, part[s % S][i][mm]);
#endif
        }
      }
      if (j == NB - 1 && has_next) {                                   // last use of a[.][s]
#pragma unroll
        for (int mm = 0; mm < MT; ++mm) a[mm][s] = O::load_a(wnext, MT * mp + mm, s, lane);
      }
#if RDN_IP_SPREAD_STORE
      // lagged write-back of block j-2, one (N-tile, M-tile) piece per k-step: the LDS write
      // bursts of the 8 waves spread over the block instead of landing on its first k-step
      if (j >= 2 && s < NT * MT) store_piece(j - 2, s / MT, s % MT);
#else
      if (s == 0 && j >= 2) store_block(j - 2);                        // lagged write-back
#endif
      // keep B-fragment reads within their k-step (VGPR budget of 2 waves/SIMD)
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int mm = 0; mm < MT; ++mm) {
        f32x4 v = part[0][i][mm];
#pragma unroll
        for (int k = 1; k < S; ++k) v += part[k][i][mm];
        res[j][i][mm] = v;
      }
    if (j + 1 < NB) {
#pragma unroll
      for (int i = 0; i < NT; ++i) bnext[i] = read_b(j + 1, 0, i);
    }
    lds_barrier();                 // every wave is done reading the rows block j needed
  }
  store_block(NB - 2);
  store_block(NB - 1);
  lds_barrier();                   // the layer's output is complete
  tl.layer += 1;
}

// partial sums per accumulator: F32 splits the fp32 chain 2 ways (128 accumulator VGPRs); the
// residual net (DSDN) needs 64 VGPRs of identity and keeps one chain; split-bf16 error is
// dominated by the operand split, one chain.
template <int MODE, bool RES> struct Geo { static constexpr int S = 1; };
template <> struct Geo<MODE_F32, false> { static constexpr int S = 2; };

__device__ __forceinline__ Tile make_tile(char* lds, const uint8_t* blob, const float* x, int L, int T,
                                          int tiles, int halo, int& n_out) {
  const int n = blockIdx.x / tiles, tile = blockIdx.x - n * tiles;
  n_out = n;
  Tile tl;
  tl.lds = lds;
  tl.x = x + (size_t)n * L;
  tl.L = L;
  tl.base = tile * T - halo;
  tl.small = (const float*)blob;
  tl.big = blob + SMALL_BYTES;
  tl.layer = 0;
  return tl;
}

__device__ __forceinline__ void store_out(const Tile& tl, float* y, int n, const float (&v)[HEAD_ROWS], int halo, int T) {
#pragma unroll
  for (int k = 0; k < HEAD_ROWS; ++k) {
    const int j = opaque_tid() + THREADS * k;
    const int p = tl.base + j;
    if (j >= halo && j < halo + T && p < tl.L) y[(size_t)n * tl.L + p] = v[k];
  }
}

}  // namespace ip
}  // namespace rdn
