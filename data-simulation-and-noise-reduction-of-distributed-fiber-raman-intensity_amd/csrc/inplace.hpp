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
constexpr uint32_t LDS_BYTES = ACT_BYTES_F32;                    // 132096
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
template <int MODE, bool ACCUM = false>
__device__ __forceinline__ void stem(const Tile& tl, int slot) {
  const cfloat* sw = small_slot(tl, slot);
  const int j = threadIdx.x;
  const int p = tl.base + j;
  const float xm = in_range(p - 1, tl.L) ? tl.x[p - 1] : 0.f;
  const float x0 = in_range(p, tl.L) ? tl.x[p] : 0.f;
  const float xp = in_range(p + 1, tl.L) ? tl.x[p + 1] : 0.f;
  const bool valid = in_range(p, tl.L);
#pragma unroll
  for (int cb = 0; cb < 16; ++cb) {
    f32x4 v = ACCUM ? Op<MODE>::load4(tl.lds, j + GUARD, 4 * cb) : f32x4{0.f, 0.f, 0.f, 0.f};
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
    Op<MODE>::store4(tl.lds, j + GUARD, 4 * cb, v);
  }
}

// Conv1d(64, 1, 3, padding=1), one row per thread, fp32 weights and accumulate.
template <int MODE>
__device__ __forceinline__ float head(const Tile& tl, int slot) {
  const cfloat* hw = small_slot(tl, slot);
  const int j = threadIdx.x;
  float a = hw[192];
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const int prow = j + GUARD + t - 1;
#pragma unroll 4
    for (int cb = 0; cb < 16; ++cb) {
      const f32x4 v = Op<MODE>::load4(tl.lds, prow, 4 * cb);
#pragma unroll
      for (int i = 0; i < 4; ++i) a = fmaf(hw[3 * (cb * 4 + i) + t], v[i], a);
    }
  }
  return a;
}

// LDS-only workgroup barrier: waits for this wave's LDS traffic, NOT for its outstanding global
// loads (the prefetched weights stay in flight across it).  One asm statement, so the compiler
// cannot move memory accesses across the barrier either.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// A-operands of (layer, k-step 0), loaded one k-step ahead of their use (software pipelining):
// every k-step issues the global (L2) load of the next k-step's weights, and the last k-step of a
// layer issues the next layer's first one, so no MFMA chain waits on an L2 round trip.
template <int MODE>
__device__ __forceinline__ typename Op<MODE>::A load_a0(const Tile& tl, int layer) {
  const int m = (threadIdx.x >> 6) & 3, lane = threadIdx.x & 63;
  return Op<MODE>::load_a(tl.big + (size_t)layer * BIG_BYTES, m, 0, lane);
}

// One Conv1d(64,64,3,d) over the tile; S partial sums per accumulator (k-steps dealt round-robin).
// `a` holds this layer's k-step-0 A-operand on entry and the next layer's on exit.
template <int MODE, int EPI, int S>
__device__ __forceinline__ void conv(Tile& tl, int dil, f32x4 (&id)[16], typename Op<MODE>::A& a, bool has_next) {
  using O = Op<MODE>;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int m = w & 3, nh = w >> 2;
  const int q = lane >> 4, c16 = lane & 15;
  const uint8_t* wl = tl.big + (size_t)tl.layer * BIG_BYTES;
  const f32x4 bias = *(const f32x4*)(wl + BIAS_OFF + (16 * m + 4 * q) * 4);

  f32x4 part[S][16];
#pragma unroll
  for (int k = 0; k < S; ++k)
#pragma unroll
    for (int n = 0; n < 16; ++n) part[k][n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < O::KSTEPS; ++s) {
    const int t = O::tap(s);
    const typename O::A cur = a;
    if (s + 1 < O::KSTEPS) a = O::load_a(wl, m, s + 1, lane);
    else if (has_next) a = O::load_a(wl + BIG_BYTES, m, 0, lane);
#pragma unroll
    for (int n = 0; n < 16; ++n) {
      const int prow = GUARD + nh * 256 + n * 16 + c16 + (t - 1) * dil;
      const typename O::B b = O::load_b(tl.lds, prow, s, q);
      part[s % S][n] = O::mma(cur, b, part[s % S][n]);
      // bound how far the scheduler hoists B-fragment reads (VGPR pressure at 2 waves/SIMD)
      if ((n & 3) == 3) __builtin_amdgcn_sched_barrier(0);
    }
  }
  lds_barrier();                   // every read of the layer input is done: overwrite in place
  // rows outside [0, L) are re-zeroed (every reference Conv1d zero-pads); only waves whose 256
  // rows straddle a spectrum end pay for the per-lane select
  const int r0 = tl.base + nh * 256;
  const bool wave_inside = r0 >= 0 && r0 + 256 <= tl.L;
#pragma unroll
  for (int n = 0; n < 16; ++n) {
    const int row = nh * 256 + n * 16 + c16;
    f32x4 v = part[0][n];
#pragma unroll
    for (int k = 1; k < S; ++k) v += part[k][n];
    v += bias;
    if (EPI & ADD_ID) v += id[n];
    if (EPI & RELU) v = __builtin_elementwise_max(v, f32x4{0.f, 0.f, 0.f, 0.f});
    if (!wave_inside && !in_range(tl.base + row, tl.L)) v = f32x4{0.f, 0.f, 0.f, 0.f};
    if (EPI & SAVE_ID) id[n] = v;
    O::store4(tl.lds, row + GUARD, 16 * m + 4 * q, v);
  }
  lds_barrier();
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

__device__ __forceinline__ void store_out(const Tile& tl, float* y, int n, float v, int halo, int T) {
  const int j = threadIdx.x;
  const int p = tl.base + j;
  if (j >= halo && j < halo + T && p < tl.L) y[(size_t)n * tl.L + p] = v;
}

}  // namespace ip
}  // namespace rdn
