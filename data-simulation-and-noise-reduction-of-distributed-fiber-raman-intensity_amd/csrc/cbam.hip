// ADSDN / APIDN (CBAM networks) on MI355X: one launch per CBAM-delimited segment.
//
// CBAM's channel attention pools every channel over the WHOLE spectrum (AdaptiveAvg/MaxPool1d,
// ADSDN/train.py:75-76, APIDN/train.py:75-76), a global dependency in each of the 15-17 blocks, so
// these networks cannot stay in one tile for their whole depth.  Each segment kernel is a tile of
// the in-place 256-byte-row engine (inplace.hpp) that
//   prologue  applies the PENDING CBAM of the previous segment to its output u (read from HBM):
//             ca[c] = sigmoid(fc(avg_L u) + fc(max_L u)) from the per-channel sums/maxima the
//             previous segment accumulated, then the spatial attention
//             sa[p] = sigmoid(conv7([mean_c(u*ca); max_c(u*ca)])) on the tile rows +-3, and forms
//             the block output h = [h_prev +] u*ca*sa [then ReLU] (ADSDN/train.py:113-116,143-147;
//             APIDN/train.py:113-116,154-156); or computes h = relu(stem(x)) for the first segment;
//   body      runs the segment's Conv1d(64,64,3) layers on the tile in LDS (BN folded);
//   epilogue  writes the new u (and h, the next residual) to HBM and accumulates the per-channel
//             sum (fp64) and max of u over the tile's own positions for the next CBAM; or, for
//             the last segment, runs the head (ADSDN: conv_out; APIDN: sigmoid(conv_out(h + h0))).
// Intermediates live in HBM as fp32 [n][L][64] (256 B per position).
#include <atomic>
#include <cstdlib>
#include <vector>

#include "inplace.hpp"
#include "host_util.hpp"
// the ping-pong engine (fused16.hpp) in f16 over the blob's ping-pong section (pack.cpp
// has_pp16_section): the convs of the RDN_F16 team kernel (team16_forward below)
#define RDN_H16_F16 1
#define H16_NS h16c
#define H16_LAYER_BYTES BIG_BYTES_BF16
#define H16_BIAS_OFF BIG_FRAG_BYTES_BF16
#include "fused16.hpp"

namespace rdn {
namespace cb {

using namespace ip;

enum Pro : int { PRO_STEM = 0, PRO_CBAM = 1 };
enum Res : int { RES_NONE = 0, RES_ADD = 1, RES_ADD_RELU = 2 };
enum EpiKind : int { EPI_STORE = 0, EPI_HEAD = 1 };

struct Seg {
  int pro, res, store_h;        // prologue kind, residual form, write h to HBM
  int cbam_slot, bias;          // CBAM being applied (first of its 3 small slots); CBAM has biases
  int n_convs, epi0, epi1;      // body: number of convs (0..2) and their epilogues (RELU or 0)
  int layer0;                   // big-layer index of the first conv
  int epi;                      // EPI_STORE or EPI_HEAD
  int head_slot, head_sigmoid, head_add_stem;
  int halo;                     // rows of halo needed by the body (+ head)
  const float* h_in;            // [n][L][64] previous residual input (RES_ADD*)
  const float* u_in;            // [n][L][64] previous segment output (PRO_CBAM)
  const double* sum_in;         // [n][64]
  const unsigned* max_in;       // [n][64] order-preserving encoding of float
  float* h_out;
  float* u_out;
  double* sum_out;
  unsigned* max_out;
  unsigned* range;              // status words: [0] MODE_H8 range, this forward; [1] range, sticky; [2] the
                                // input gate (STATUS_GATE, raised by the first segment's stem), sticky
};

__device__ __forceinline__ unsigned f2ord(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(unsigned o) {
  return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}
__device__ __forceinline__ float sigm(float v) { return 1.0f / (1.0f + expf(-v)); }
// sigmoid from v_exp_f32 (2^x) and v_rcp_f32 (~1 ulp each): the f16 team kernel's channel / spatial
// attention, which it rounds to f16 before use (the fp32 kernels and every network output use sigm);
// exp2 overflow gives rcp(inf) = 0 = sigmoid(-inf)
__device__ __forceinline__ float sigm_fast(float v) {
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * v));
}

// LDS scratch behind the activation buffer
constexpr int S1_OFF = ACT_BYTES_F32;                 // mean_c(u*ca) for rows -3 .. 514   (518 f32)
constexpr int S2_OFF = S1_OFF + 520 * 4;              // max_c(u*ca)
constexpr int SA_OFF = S2_OFF + 520 * 4;              // spatial attention per window row (512 f32)
constexpr int CA_OFF = SA_OFF + 512 * 4;              // channel attention (64 f32)
constexpr int H1_OFF = CA_OFF + 64 * 4;               // MLP hidden (2 x 4 f32)
constexpr int RED_OFF = H1_OFF + 16 * 4;              // cross-wave reduction (8 waves x 64 x {f64 sum, u32 max})
constexpr uint32_t SEG_LDS_BYTES = RED_OFF + 8 * 64 * 12;  // 146,528 B

template <int MODE>
__device__ void prologue_cbam(Tile& tl, const Seg& sg, int n) {
  char* lds = tl.lds;
  float* s1 = (float*)(lds + S1_OFF) + 3;       // index -3 .. 514
  float* s2 = (float*)(lds + S2_OFF) + 3;
  float* sa = (float*)(lds + SA_OFF);
  float* ca = (float*)(lds + CA_OFF);
  float* h1 = (float*)(lds + H1_OFF);
  const int tid = __builtin_amdgcn_workitem_id_x(), lane = tid & 63, w = tid >> 6;
  const float* cw = tl.small + sg.cbam_slot * SMALL_SLOT_FLOATS;   // fc.0.weight [4][64]
  const float* cw2 = cw + SMALL_SLOT_FLOATS;                       // fc.2.weight [64][4]
  const float* cmisc = cw2 + SMALL_SLOT_FLOATS;                    // fc.0.bias[4], fc.2.bias[64], sa.w[2][7], sa.b

  // -- channel attention: hidden units of the shared MLP for the avg- and max-pooled vectors
  if (tid < 8) {
    const int j = tid & 3, which = tid >> 2;        // which: 0 = avg, 1 = max
    float a = sg.bias ? cmisc[j] : 0.f;
    for (int c = 0; c < 64; ++c) {
      const float v = which == 0 ? (float)(sg.sum_in[(size_t)n * 64 + c] / (double)tl.L)
                                 : ord2f(sg.max_in[(size_t)n * 64 + c]);
      a = fmaf(cw[j * 64 + c], v, a);
    }
    h1[tid] = fmaxf(a, 0.f);
  }
  __syncthreads();
  if (tid < 64) {
    float oa = sg.bias ? cmisc[4 + tid] : 0.f, om = oa;
    for (int j = 0; j < 4; ++j) {
      oa = fmaf(cw2[tid * 4 + j], h1[j], oa);
      om = fmaf(cw2[tid * 4 + j], h1[4 + j], om);
    }
    ca[tid] = sigm(oa + om);
  }
  __syncthreads();

  // -- spatial statistics of u*ca for window rows -3 .. 514: 16 lanes per row, 4 channels each
  const int sub = lane & 15, rgrp = lane >> 4;
  const f32x4 cav = *(const f32x4*)(ca + 4 * sub);
  for (int r = w * 4 + rgrp - 3; r < WB + 3; r += WAVES * 4) {
    const int p = tl.base + r;
    float sm = 0.f, mx = -INFINITY;
    if (p >= 0 && p < tl.L) {
      const f32x4 u = *(const f32x4*)(sg.u_in + ((size_t)n * tl.L + p) * 64 + 4 * sub);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float v = u[i] * cav[i];
        sm += v;
        mx = fmaxf(mx, v);
      }
    }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      sm += __shfl_xor(sm, o);
      mx = fmaxf(mx, __shfl_xor(mx, o));
    }
    if (sub == 0) {
      const bool in = p >= 0 && p < tl.L;           // conv7 zero-pads the [mean; max] map
      s1[r] = in ? sm * (1.0f / 64.0f) : 0.f;
      s2[r] = in ? mx : 0.f;
    }
  }
  __syncthreads();
  // -- spatial attention per window row
  {
    const int r = tid;
    float a = sg.bias ? cmisc[82] : 0.f;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      a = fmaf(cmisc[68 + k], s1[r + k - 3], a);
      a = fmaf(cmisc[75 + k], s2[r + k - 3], a);
    }
    sa[r] = sigm(a);
  }
  __syncthreads();
  // -- h = [h_prev +] u*ca*sa [relu] into the tile, and (valid rows) to HBM
  const int H = sg.halo, T = WB - 2 * H;
  for (int r = w * 4 + rgrp; r < WB; r += WAVES * 4) {
    const int p = tl.base + r;
    f32x4 h = f32x4{0.f, 0.f, 0.f, 0.f};
    if (p >= 0 && p < tl.L) {
      const size_t off = ((size_t)n * tl.L + p) * 64 + 4 * sub;
      const f32x4 u = *(const f32x4*)(sg.u_in + off);
      const float s = sa[r];
#pragma unroll
      for (int i = 0; i < 4; ++i) h[i] = (u[i] * cav[i]) * s;
      if (sg.res != RES_NONE) {
        const f32x4 hp = *(const f32x4*)(sg.h_in + off);
        h += hp;
        if (sg.res == RES_ADD_RELU)
#pragma unroll
          for (int i = 0; i < 4; ++i) h[i] = fmaxf(h[i], 0.f);
      }
      if (sg.store_h && r >= H && r < H + T) *(f32x4*)(sg.h_out + off) = h;
    }
    Op<MODE>::store4(lds, r + GUARD, 4 * sub, h, &tl.amax);
  }
}

// h = relu(stem(x)) for the first segment; also stored to HBM when it is a residual (APIDN)
template <int MODE>
__device__ void prologue_stem(Tile& tl, const Seg& sg, int n) {
  stem<MODE>(tl, 0);
  __syncthreads();
  if (!sg.store_h) return;
  const int tid = opaque_tid(), lane = tid & 63, w = tid >> 6, sub = lane & 15, rgrp = lane >> 4;
  const int H = sg.halo, T = WB - 2 * H;
  for (int r = w * 4 + rgrp; r < WB; r += WAVES * 4) {
    const int p = tl.base + r;
    if (p >= 0 && p < tl.L && r >= H && r < H + T)
      *(f32x4*)(sg.h_out + ((size_t)n * tl.L + p) * 64 + 4 * sub) = Op<MODE>::load4(tl.lds, r + GUARD, 4 * sub);
  }
}

// u (tile rows [H, H+T)) to HBM + per-channel sum / max over them
template <int MODE>
__device__ void epilogue_store(Tile& tl, const Seg& sg, int n) {
  char* lds = tl.lds;
  const int tid = opaque_tid(), lane = tid & 63, w = tid >> 6, sub = lane & 15, rgrp = lane >> 4;
  const int H = sg.halo, T = WB - 2 * H;
  double sm[4] = {0, 0, 0, 0};
  float mx[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  for (int r = H + w * 4 + rgrp; r < H + T; r += WAVES * 4) {
    const int p = tl.base + r;
    if (p >= tl.L) break;
    const f32x4 u = Op<MODE>::load4(lds, r + GUARD, 4 * sub);
    *(f32x4*)(sg.u_out + ((size_t)n * tl.L + p) * 64 + 4 * sub) = u;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      sm[i] += (double)u[i];
      mx[i] = fmaxf(mx[i], u[i]);
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    for (int o = 16; o < 64; o <<= 1) {
      sm[i] += __shfl_xor(sm[i], o);
      mx[i] = fmaxf(mx[i], __shfl_xor(mx[i], o));
    }
  }
  double* rs = (double*)(lds + RED_OFF);
  unsigned* rm = (unsigned*)(lds + RED_OFF + 8 * 64 * 8);
  if (rgrp == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      rs[w * 64 + 4 * sub + i] = sm[i];
      rm[w * 64 + 4 * sub + i] = f2ord(mx[i]);
    }
  }
  __syncthreads();
  if (tid < 64) {
    const int c = tid;
    double s = 0.0;
    unsigned m = 0;
    for (int k = 0; k < WAVES; ++k) {
      s += rs[k * 64 + c];
      m = max(m, rm[k * 64 + c]);
    }
    atomicAdd(&sg.sum_out[(size_t)n * 64 + c], s);
    atomicMax(&sg.max_out[(size_t)n * 64 + c], m);
  }
}

template <int MODE>
__global__ __launch_bounds__(THREADS) void segment(const uint8_t* __restrict__ blob, const float* __restrict__ x,
                                                   float* __restrict__ y, int L, int T, int tiles, Seg sg) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  using G = CbamGeo<MODE>;
  int n;
  Tile tl = make_tile(lds, blob, x, L, T, tiles, sg.halo, n);
  tl.layer = sg.layer0;
  f32x4 id[16];
  LayerA<MODE> a;
  if (sg.n_convs) load_layer_a<MODE>(tl, sg.layer0, a);
  zero_guards(lds);
  if (sg.pro == PRO_STEM) {
    tl.status = sg.range + 2;            // the stem reads every x: the input-gate word
    prologue_stem<MODE>(tl, sg, n);
    tl.status = nullptr;
  } else {
    prologue_cbam<MODE>(tl, sg, n);
  }
  __syncthreads();
  for (int i = 0; i < sg.n_convs; ++i) {
    const bool more = i + 1 < sg.n_convs;
    if ((i ? sg.epi1 : sg.epi0) & RELU) conv<MODE, RELU, G::S>(tl, 1, id, a, more);
    else conv<MODE, 0, G::S>(tl, 1, id, a, more);
  }
  // MODE_H8 range guard (inplace.hpp range_vote): a saturated tile raises this forward's word and the
  // sticky one; the head segment writes NaN if any segment of the forward saturated
  bool sat = false;
  if constexpr (MODE == MODE_H8) {
    sat = range_vote(tl, RED_OFF, sg.range + 1);
    if (sat && __builtin_amdgcn_workitem_id_x() == 0) __hip_atomic_store(sg.range, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (sg.epi == EPI_STORE) {
    epilogue_store<MODE>(tl, sg, n);
    return;
  }
  if (sg.head_add_stem) {
    stem<MODE, true>(tl, 0);
    __syncthreads();
  }
  double d[HeadOut<MODE>::ROWS];
  head<MODE>(tl, sg.head_slot, d);
  float v[HeadOut<MODE>::ROWS];
  round_rows(d, v);
  if (sg.head_sigmoid) {
#pragma unroll
    for (int k = 0; k < HeadOut<MODE>::ROWS; ++k) v[k] = sigm(v[k]);
  }
  if constexpr (MODE == MODE_H8) {
    if (sat || __hip_atomic_load(sg.range, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) nan_rows(v);
  }
  store_out<MODE>(tl, y, n, v, sg.halo, T);
}


// ---- team-persistent forward ---------------------------------------------------------------------
//
// The whole network in ONE launch.  The grid is `teams` x TT co-resident workgroups (one per CU:
// the tile takes 143 KB of LDS); the TT workgroups of a team own the TT tiles of one spectrum and
// walk the spectra team, team + teams, ...  Each keeps its tile (512 rows + the whole network's
// TEAM_HALO rows per side, refreshed from the neighbours' published edge rows at every CBAM) in LDS
// from the stem to the head.  CBAM is pointwise except the +-3-row spatial conv and the channel pool
// over the whole spectrum: at each
// CBAM every tile publishes the per-channel sum (fp64) and max of u over its own positions to a
// slot, the team meets at a counter, and every tile reduces the TT slots in tile order (so the
// result is deterministic) into ca.  Hand-off per MI355X_MICROARCH.md §Workgroup dispatch (first
// row of the sc1 table): slots written with sc1 stores by wave 0, `s_waitcnt vmcnt(0)`, one agent
// atomic add by lane 0; lane 0 polls the counter with sc1 loads, a workgroup barrier, then sc1 loads
// of the slots.  The ResidualBlock identity (the block input, all tile rows) is parked in a
// per-workgroup fp32 buffer in memory (sc1 stores / loads: written and read back by the same CU).
// A wait that exceeds SPIN_TICKS (0.3 s) raises the error word and falls through instead of hanging.

// Halo exchange: the tiles of a team meet at every CBAM anyway, so instead of recomputing the whole
// network's halo (85 / 77 rows per side for ADSDN / APIDN: 30 / 28 tiles per spectrum at L = 10,000)
// each tile keeps TEAM_HALO rows per side and, with its statistics, publishes the EDGE_ROWS rows of
// u its neighbours' halos need.  Between two CBAMs a tile runs at most 2 convs (k = 3, d = 1), so
// with h valid on rows [3, WB - 3) after a CBAM, u is valid on [5, WB - 5) at the next one; the
// neighbours supply rows [0, 5) and [WB - 5, WB), the +-3-row spatial conv then yields h valid on
// [3, WB - 3) again, and the head (+-1 row) reads only rows inside it: TEAM_HALO >= 4.
constexpr int TEAM_HALO = 6;
constexpr int EDGE_ROWS = 5;
constexpr int EDGE_BYTES = EDGE_ROWS * 64 * 4;       // one edge, fp32
constexpr int STAT_BYTES = 64 * 8 + 64 * 4;        // per-tile stats: 64 fp64 sums, 64 ordered u32 maxima
constexpr int SLOT_BYTES = STAT_BYTES + 2 * EDGE_BYTES;   // + the tile's first / last EDGE_ROWS own-edge rows
static_assert(2 * TEAM_HALO - EDGE_ROWS >= TEAM_HALO - 1 && TEAM_HALO >= 4, "edge rows lie in the tile's own rows");
// A wait is bounded by wall-clock time: SPIN_TICKS of the 100 MHz s_memrealtime counter (0.3 s),
// checked every 64 polls by one thread, which raises the error words; SPIN_LIMIT polls remain as a
// backstop (a poll round of the tagged hand-off is a memory round trip plus a workgroup vote, so a
// count alone stood for seconds, not the 0.3 s its comment promised: ADVICE r03).
constexpr unsigned long long SPIN_TICKS = 30000000ull;
constexpr unsigned SPIN_LIMIT = 1u << 22;
#ifndef RDN_TEAM_SLEEP
#define RDN_TEAM_SLEEP 2                           // s_sleep units (64 clocks) between two polls
#endif
constexpr int TEAM_CTR_STRIDE = 16;                // u32s between team counters (64 B)

struct TeamArgs {
  int TT;               // workgroups (tiles) per team
  int teams;
  int T;                // output positions per tile
  int halo;
  int64_t n;            // spectra
  char* slots;          // [teams][2][TT][SLOT_BYTES]
  unsigned* counters;   // [teams][TEAM_CTR_STRIDE], zeroed before the launch
  char* hsave;          // [teams * TT][WB][64] f32
  unsigned* err;         // status words: [0] hand-off error, this launch (fast-fail, NaN outputs); [1] hand-off
                         // error, sticky; [2] MODE_H8 range, sticky; [3] the input gate (STATUS_GATE: the stems
                         // read every x), sticky -- the sticky words are read and cleared by cbam_status
  unsigned long long* stamps;   // RDN_TEAM_STAMPS diagnostics: [grid][NSTAMP] cycle sums per phase
  int force_miss;       // test knob (RDN_CBAM_FORCE_MISS=k): workgroup 0 skips its k-th arrival
  int xcd;              // team16: 1 = same-XCD teams may hand off through their XCD's L2
  unsigned tag0;        // team16: this launch's first granule tag - 1 (tags never repeat across launches)
};
#ifndef RDN_TEAM_STAMPS
#define RDN_TEAM_STAMPS 0
#endif
constexpr int NSTAMP = 16;
constexpr int STAMP_BYTES = RDN_TEAM_STAMPS ? 256 * NSTAMP * 8 : 0;

// diagnostics (RDN_TEAM_STAMPS=1, tools/team_stamps.py): s_memtime deltas summed per phase by
// wave 0; compiled out otherwise
struct Stamps {
  unsigned long long acc[NSTAMP], t;
  __device__ __forceinline__ void init() {
    if (RDN_TEAM_STAMPS) {
      for (int k = 0; k < NSTAMP; ++k) acc[k] = 0;
      t = __builtin_amdgcn_s_memtime();
    }
  }
  __device__ __forceinline__ void operator()(int k) {
    if (RDN_TEAM_STAMPS) {
      const unsigned long long n = __builtin_amdgcn_s_memtime();
      acc[k] += n - t;
      t = n;
    }
  }
};

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// sc1 (L1-bypassing) 16-B access to this workgroup's identity buffer
__device__ __forceinline__ void hs_store(__amdgpu_buffer_rsrc_t r, int off, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off, 0, 16);
}
__device__ __forceinline__ f32x4 hs_load(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16));
}

// Row k (0 .. 15) of the pointwise passes for lane group rgrp of wave w: 16 lanes x 4 channels per
// row, 32 rows per pass step.  fp32 rows (16 x 16 B) take 4 consecutive rows per wave (conflict-free
// ds_read_b128); the bf16 planes (16 x 8 B, ds_read_b64 in 32-lane groups) pair rows r and r + 4,
// whose swizzles put the plane in opposite halves of the 256 B of banks.
template <int MODE>
__device__ __forceinline__ int pw_row(int w, int rgrp, int k) {
  if (MODE == MODE_F32) return 32 * k + 4 * w + rgrp;
  return 32 * k + 8 * (w >> 1) + 2 * (w & 1) + 4 * (rgrp & 1) + (rgrp >> 1);
}

// The ResidualBlock identity (the block input, all WB tile rows).  Plain bf16 keeps it in the free
// lo plane of its own LDS row (the activation is bf16 there, so the copy is exact); fp32 and
// split-bf16 park it as fp32 in the workgroup's buffer in memory.
// f16f8 parks it in its own two-plane form (f16 hi + e4m3 lo: 12 B per 4 values instead of 16, the
// value its LDS row holds): 96 KB per tile, so the 30 tiles of an XCD keep it in their 4 MB L2.
// IdRaw: the identity as fetched (converted to f32 only where it is added).
typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));
template <int MODE> struct IdRaw { typedef u32x4 T; };
template <> struct IdRaw<MODE_H8> { typedef u32x3 T; };
template <int MODE>
__device__ __forceinline__ void id_store(char* lds, __amdgpu_buffer_rsrc_t hs, int r, int sub, f32x4 h) {
  if constexpr (single16(MODE)) {
    typedef typename Op<MODE>::V4 V4;
    *(V4*)(lds + off_f32(r + GUARD, 128 + 8 * sub)) = __builtin_convertvector(h, V4);
  }
  else if (MODE == MODE_H8) {
    const H8Split x = h8_split(h8_sat<false>(h));
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    const u32x2 hb = __builtin_bit_cast(u32x2, x.hi);
    __builtin_amdgcn_raw_buffer_store_b96(u32x3{hb.x, hb.y, x.lo8}, hs, (r * 16 + sub) * 12, 0, 16);
  } else hs_store(hs, (r * 64 + 4 * sub) * 4, h);
}
template <int MODE>
__device__ __forceinline__ typename IdRaw<MODE>::T id_fetch(__amdgpu_buffer_rsrc_t hs, int r, int sub) {
  if constexpr (MODE == MODE_H8) return __builtin_amdgcn_raw_buffer_load_b96(hs, (r * 16 + sub) * 12, 0, 16);
  else return __builtin_amdgcn_raw_buffer_load_b128(hs, (r * 64 + 4 * sub) * 4, 0, 16);
}
template <int MODE>
__device__ __forceinline__ f32x4 id_value(typename IdRaw<MODE>::T v) {
  if constexpr (MODE == MODE_H8) {
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    const f16x4 hi = __builtin_bit_cast(f16x4, u32x2{v.x, v.y});
    return __builtin_convertvector(hi, f32x4) + unpk_e4m3(v.z) * H8_LO_DIV;
  } else return __builtin_bit_cast(f32x4, v);
}
template <int MODE>
__device__ __forceinline__ f32x4 id_load(const char* lds, __amdgpu_buffer_rsrc_t hs, int r, int sub) {
  if constexpr (single16(MODE)) {
    typedef typename Op<MODE>::V4 V4;
    return __builtin_convertvector(*(const V4*)(lds + off_f32(r + GUARD, 128 + 8 * sub)), f32x4);
  } else {
    return id_value<MODE>(id_fetch<MODE>(hs, r, sub));
  }
}

// block input (all WB tile rows) -> identity (used after the stem; later blocks save it from the
// CBAM write-back that produces it)
template <int MODE>
__device__ __forceinline__ void save_identity(const Tile& tl, __amdgpu_buffer_rsrc_t hs) {
  const int tid = opaque_tid(), lane = tid & 63, w = tid >> 6, sub = lane & 15, rgrp = lane >> 4;
#pragma unroll 4
  for (int k = 0; k < WB / 32; ++k) {
    const int r = pw_row<MODE>(w, rgrp, k);
    id_store<MODE>(tl.lds, hs, r, sub, Op<MODE>::load4(tl.lds, r + GUARD, 4 * sub));
  }
}

// 8 channels [8k, 8k+8) of tile row r as f32
template <int MODE>
__device__ __forceinline__ void load8(const char* lds, int r, int k, float (&v)[8]) {
  const int pr = r + GUARD;
  if (MODE == MODE_H8) {          // f16 + e4m3 planes in h16_channel order: two 4-channel reads
    const f32x4 a = Op<MODE>::load4(lds, pr, 8 * k), b = Op<MODE>::load4(lds, pr, 8 * k + 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[i] = a[i];
      v[4 + i] = b[i];
    }
  } else if (MODE == MODE_F32) {
    const f32x4 a = *(const f32x4*)(lds + off_f32(pr, 32 * k)), b = *(const f32x4*)(lds + off_f32(pr, 32 * k + 16));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[i] = a[i];
      v[4 + i] = b[i];
    }
  } else if constexpr (MODE == MODE_F16) {
    const h16x8_t hi = *(const h16x8_t*)(lds + off_f32(pr, 16 * k));
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (float)hi[i];
  } else {
    const bf16x8 hi = *(const bf16x8*)(lds + off_f32(pr, 16 * k));
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (float)hi[i];
    if (MODE == MODE_X3) {
      const bf16x8 lo = *(const bf16x8*)(lds + off_f32(pr, 128 + 16 * k));
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] += (float)lo[i];
    }
  }
}

// per-channel sum / max of u over the tile's own positions -> slot (sc1); arrive at the counter
template <int MODE>
__device__ __forceinline__ void publish_stats(const Tile& tl, const TeamArgs& ta, char* slot, unsigned* ctr, Stamps& st,
                                              bool arrive = true) {
  char* lds = tl.lds;
  const int tid = opaque_tid(), lane = tid & 63, w = tid >> 6, sub = lane & 15, rgrp = lane >> 4;
  const int H = ta.halo, T = ta.T;
  const int rend = H + min(T, tl.L - tl.base - H);     // the last tile of a spectrum ends at L
  // edge rows for the neighbours (sc1 stores, issued first so that they drain under the statistics
  // pass): block 0 = rows [2H - 5, 2H) (the left neighbour's rows [WB - 5, WB)), block 1 = rows
  // [T, T + 5) (the right neighbour's rows [0, 5))
  if (tid < 2 * EDGE_ROWS * 16) {
    const int e = tid / (EDGE_ROWS * 16), k = (tid / 16) % EDGE_ROWS, c4 = tid & 15;
    const int r = e == 0 ? 2 * H - EDGE_ROWS + k : T + k;
    const __amdgpu_buffer_rsrc_t sr = __builtin_amdgcn_make_buffer_rsrc((void*)slot, 0, SLOT_BYTES, 0x00020000);
    const f32x4 u = Op<MODE>::load4(lds, r + GUARD, 4 * c4);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, u), sr, STAT_BYTES + e * EDGE_BYTES + (k * 64 + 4 * c4) * 4, 0, 16);
  }
  // fp32 partials over <= T / 32 rows per lane, fp64 from the cross-wave sum on
  f32x4 sm = {0.f, 0.f, 0.f, 0.f}, mx = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll 4
  for (int k = 0; k < WB / 32; ++k) {
    const int r = H + pw_row<MODE>(w, rgrp, k);
    if (r >= rend) break;              // pw_row is increasing in k
    const f32x4 u = Op<MODE>::load4(lds, r + GUARD, 4 * sub);
    sm += u;
    mx = __builtin_elementwise_max(mx, u);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    for (int o = 16; o < 64; o <<= 1) {
      sm[i] += __shfl_xor(sm[i], o);
      mx[i] = fmaxf(mx[i], __shfl_xor(mx[i], o));
    }
  }
  float* rs = (float*)(lds + RED_OFF);
  unsigned* rm = (unsigned*)(lds + RED_OFF + 8 * 64 * 8);
  unsigned* rsat = (unsigned*)(lds + RED_OFF + 8 * 64 * 4);       // per-wave saturation votes (MODE_H8)
  if (rgrp == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      rs[w * 64 + 4 * sub + i] = sm[i];
      rm[w * 64 + 4 * sub + i] = f2ord(mx[i]);
    }
  }
  if constexpr (MODE == MODE_H8) {
    const bool wave_sat = __builtin_amdgcn_ballot_w64(tl.amax > H8_SAT) != 0;
    if (lane == 0) rsat[w] = wave_sat ? 1u : 0u;
  }
  // the edge stores drain under the statistics pass; every storing wave waits for them before the
  // barrier that precedes the arrival
  if (tid < 2 * EDGE_ROWS * 16) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  st(8);
  __syncthreads();
  st(9);
  if (tid < 64) {
    const int c = tid;
    double s = 0.0;
    unsigned m = 0;
#pragma unroll
    for (int k = 0; k < WAVES; ++k) {
      s += (double)rs[k * 64 + c];
      m = max(m, rm[k * 64 + c]);
    }
    // MODE_H8: a tile whose activations saturated so far publishes +inf maxima -- stored activations
    // are clamped to +-1792, so an infinite pooled maximum taints the whole team's spectrum (apply_cbam)
    if constexpr (MODE == MODE_H8) {
      bool sat = false;
#pragma unroll
      for (int k = 0; k < WAVES; ++k) sat = sat || rsat[k] != 0;
      if (sat) m = f2ord(INFINITY);
    }
    __hip_atomic_store((double*)slot + c, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store((unsigned*)(slot + 512) + c, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");      // every lane's slot stores have landed
    if (c == 0 && arrive) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// the team has arrived at `target`: lane 0 polls (sc1), the workgroup barrier releases the rest.
// A wait that exceeds SPIN_TICKS (a team member never arrived: the co-residency the grid is
// sized for was broken, e.g. by a concurrent kernel) raises the error word and falls through; once
// the word is up every later wait of every workgroup falls through at once, so the grid drains in
// about one SPIN_TICKS, the outputs of the affected spectra are NaN (team_forward) and the host
// reports RDN_EHIP (cbam_status).
__device__ __forceinline__ void team_wait(const TeamArgs& ta, unsigned* ctr, unsigned target) {
  if (__builtin_amdgcn_workitem_id_x() == 0) {
    unsigned it = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(RDN_TEAM_SLEEP);
      if ((++it & 63) == 0 && __hip_atomic_load(ta.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
      if (it > SPIN_LIMIT || ((it & 63) == 0 && __builtin_amdgcn_s_memrealtime() - t0 > SPIN_TICKS)) {
        __hip_atomic_store(ta.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(ta.err + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // sticky word
        break;
      }
    }
  }
  __syncthreads();
}

// Apply a CBAM whose statistics sit in the team's slots (`slots0`: TT slots of this barrier) to u
// in the tile: h = [identity +] u*ca*sa [then ReLU] (ADSDN/train.py:113-116,143-147;
// APIDN/train.py:113-116,154-156), written over u (and, with save_next, as the next block's
// identity).
constexpr int ID_ITERS = WB / (WAVES * 4);          // rows per thread in the pointwise pass (16)
// identity rows fetched ahead of the spatial pass (the rest at the write-back): all 16 for fp32 and
// f16f8 (3 VGPRs per row there), 8 for split-bf16 (16 spill there; measured 18.8k vs 16.5k APIDN
// spectra/s); plain bf16 keeps its identity in LDS
template <int MODE> constexpr int ID_PRE = MODE == MODE_X3 ? 8 : 16;

// Returns whether a tile of the team had saturated (MODE_H8: an infinite pooled maximum, publish_stats).
template <int MODE>
__device__ __forceinline__ bool apply_cbam(Tile& tl, const TeamArgs& ta, const char* slots0, int cbam_slot, bool bias, int res,
                           bool save_next, __amdgpu_buffer_rsrc_t hs, Stamps& st) {
  char* lds = tl.lds;
  float* s1 = (float*)(lds + S1_OFF) + 3;       // index -3 .. 514
  float* s2 = (float*)(lds + S2_OFF) + 3;
  float* sa = (float*)(lds + SA_OFF);
  float* ca = (float*)(lds + CA_OFF);
  float* h1 = (float*)(lds + H1_OFF);
  double* red = (double*)(lds + RED_OFF);        // pooled avg / max per channel (2 x 64)
  const int tid = opaque_tid(), lane = tid & 63, w = tid >> 6;
  const float* cw = tl.small + cbam_slot * SMALL_SLOT_FLOATS;      // fc.0.weight [4][64]
  const float* cw2 = cw + SMALL_SLOT_FLOATS;                       // fc.2.weight [64][4]
  const float* cmisc = cw2 + SMALL_SLOT_FLOATS;                    // fc.0.bias[4], fc.2.bias[64], sa.w[2][7], sa.b
  // the CBAM's weights, fetched under the statistics round trip
  const float cwv = cw[(w & 3) * 64 + lane];                       // hidden unit w & 3, channel lane
  const float b1 = bias ? cmisc[w & 3] : 0.f;
  const f32x4 cw2v = *(const f32x4*)(cw2 + 4 * lane);              // channel lane's 4 hidden weights
  const float b2 = bias ? cmisc[4 + lane] : 0.f;

  // -- halo refresh, fetched first so that its round trip overlaps the slots': u of rows [0, 5)
  //    from the left neighbour's block 1, rows [WB - 5, WB) from the right neighbour's block 0
  //    (first / last tile of a spectrum: no neighbour, rows outside [0, L))
  const int edge_e = tid / (EDGE_ROWS * 16), edge_k = (tid / 16) % EDGE_ROWS;
  bool has_edge = false;
  f32x4 edge_u = {0.f, 0.f, 0.f, 0.f};
  if (tid < 2 * EDGE_ROWS * 16) {
    const int tile = (tl.base + ta.halo) / ta.T;
    const int nb = edge_e == 0 ? tile - 1 : tile + 1;
    if (nb >= 0 && nb < ta.TT) {
      const __amdgpu_buffer_rsrc_t sr = __builtin_amdgcn_make_buffer_rsrc((void*)slots0, 0, ta.TT * SLOT_BYTES, 0x00020000);
      edge_u = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
          sr, nb * SLOT_BYTES + STAT_BYTES + (1 - edge_e) * EDGE_BYTES + (edge_k * 64 + 4 * (tid & 15)) * 4, 0, 16));
      has_edge = true;
    }
  }
  // -- the spectrum's per-channel mean and max over the TT slots: 8 tile-strided partials per
  //    channel (all waves, sc1 buffer loads issued together: they are L2 / fabric round trips),
  //    then combined in a fixed order (deterministic)
  {
    const __amdgpu_buffer_rsrc_t sr = __builtin_amdgcn_make_buffer_rsrc((void*)slots0, 0, ta.TT * SLOT_BYTES, 0x00020000);
    const int c = tid & 63, part = tid >> 6;             // part = 0..7 (WAVES)
    double sp = 0.0;
    unsigned mp = 0;
    constexpr int PER = 8;                               // slots per batch per thread
    for (int t0 = part; t0 < ta.TT; t0 += WAVES * PER) {
      typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
      u32x2 sv[PER];
      unsigned mv[PER];
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int t = t0 + WAVES * k;
        const int off = (t < ta.TT ? t : 0) * SLOT_BYTES;
        sv[k] = __builtin_amdgcn_raw_buffer_load_b64(sr, off + 8 * c, 0, 16);
        mv[k] = __builtin_amdgcn_raw_buffer_load_b32(sr, off + 512 + 4 * c, 0, 16);
      }
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        if (t0 + WAVES * k < ta.TT) {
          sp += __builtin_bit_cast(double, sv[k]);
          mp = max(mp, mv[k]);
        }
      }
    }
    double* rs = (double*)(lds + S1_OFF);               // 8 x 64 partials in the spatial-pass scratch
    unsigned* rm = (unsigned*)(lds + SA_OFF);           // (S1+S2: 4160 B, SA: 2048 B; refilled below)
    static_assert(S2_OFF + 520 * 4 - S1_OFF >= 8 * 64 * 8 && CA_OFF - SA_OFF >= 8 * 64 * 4, "partials fit");
    rs[part * 64 + c] = sp;
    rm[part * 64 + c] = mp;
    __syncthreads();
    if (tid < 64) {
      double sum = 0.0;
      unsigned m = 0;
#pragma unroll
      for (int k = 0; k < WAVES; ++k) {
        sum += rs[k * 64 + tid];
        m = max(m, rm[k * 64 + tid]);
      }
      red[tid] = (double)(float)(sum / (double)tl.L);
      red[64 + tid] = (double)ord2f(m);
    }
  }
  // halo refresh (the edge rows fetched above): into rows [0, 5) / [WB - 5, WB)
  if (has_edge) Op<MODE>::store4(lds, (edge_e == 0 ? edge_k : WB - EDGE_ROWS + edge_k) + GUARD, 4 * (tid & 15), edge_u);
  __syncthreads();
  st(10);
  // MODE_H8: a tile of the team that saturated (its +inf maxima, publish_stats) taints the spectrum
  const bool taint = MODE == MODE_H8 && red[64] == (double)INFINITY;
  // -- channel attention: hidden unit (w & 3) of the shared MLP for the avg (w < 4) or max pooled
  //    vector, one wave each (64 lanes = 64 channels, butterfly sum)
  {
    float a = cwv * (float)red[(w >> 2) * 64 + lane];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o);
    if (lane == 0) h1[w] = fmaxf(a + b1, 0.f);
  }
  __syncthreads();
  if (tid < 64) {
    float oa = b2, om = b2;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      oa = fmaf(cw2v[j], h1[j], oa);
      om = fmaf(cw2v[j], h1[4 + j], om);
    }
    ca[tid] = sigm(oa + om);
  }
  __syncthreads();
  st(11);

  // -- identities of this thread's pointwise rows, in flight during the spatial pass
  const int sub = lane & 15, rgrp = lane >> 4;
  typename IdRaw<MODE>::T idr[ID_ITERS];
  if (!single16(MODE) && res != RES_NONE) {
#pragma unroll
    for (int k = 0; k < ID_PRE<MODE>; ++k) idr[k] = id_fetch<MODE>(hs, pw_row<MODE>(w, rgrp, k), sub);
  }
  // -- spatial statistics of u*ca: one tile row per thread (rows beyond the tile: 0; they feed
  //    only halo rows)
  for (int r = tid - 3; r < WB + 3; r += THREADS) {
    const int p = tl.base + r;
    const bool in = p >= 0 && p < tl.L && r >= 0 && r < WB;   // conv7 zero-pads the [mean; max] map
    float sm = 0.f, mx = -INFINITY;
    if (in) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float u[8];
        load8<MODE>(lds, r, k, u);
        const f32x4 c0 = *(const f32x4*)(ca + 8 * k), c1 = *(const f32x4*)(ca + 8 * k + 4);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float v = u[i] * (i < 4 ? c0[i] : c1[i - 4]);
          sm += v;
          mx = fmaxf(mx, v);
        }
      }
    }
    s1[r] = in ? sm * (1.0f / 64.0f) : 0.f;
    s2[r] = in ? mx : 0.f;
  }
  __syncthreads();
  st(12);
  {
    const int r = tid;
    float a = bias ? cmisc[82] : 0.f;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      a = fmaf(cmisc[68 + k], s1[r + k - 3], a);
      a = fmaf(cmisc[75 + k], s2[r + k - 3], a);
    }
    sa[r] = sigm(a);
  }
  __syncthreads();
  st(13);
  // -- h = [identity +] u*ca*sa [relu], in place (rows outside [0, L) stay zero: u and identity are)
  const f32x4 cav = *(const f32x4*)(ca + 4 * sub);
#pragma unroll
  for (int k = 0; k < ID_ITERS; ++k) {
    const int r = pw_row<MODE>(w, rgrp, k);
    const f32x4 u = Op<MODE>::load4(lds, r + GUARD, 4 * sub);
    const float sr = sa[r];
    f32x4 h;
#pragma unroll
    for (int i = 0; i < 4; ++i) h[i] = (u[i] * cav[i]) * sr;
    if (res != RES_NONE) {
      h += single16(MODE) || k >= ID_PRE<MODE> ? id_load<MODE>(lds, hs, r, sub) : id_value<MODE>(idr[k]);
      if (res == RES_ADD_RELU) h = __builtin_elementwise_max(h, f32x4{0.f, 0.f, 0.f, 0.f});
    }
    const int p = tl.base + r;
    if (p < 0 || p >= tl.L) h = f32x4{0.f, 0.f, 0.f, 0.f};
    Op<MODE>::store4(lds, r + GUARD, 4 * sub, h, &tl.amax);
    if (save_next) id_store<MODE>(lds, hs, r, sub, h);
  }
  __syncthreads();
  return taint;
}

template <int MODE, bool ADS>
__global__ __launch_bounds__(THREADS) void team_forward(const uint8_t* __restrict__ blob, const float* __restrict__ x,
                                                        float* __restrict__ y, int L, TeamArgs ta) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  using G = CbamGeo<MODE>;
  const int team = __builtin_amdgcn_workgroup_id_x() / ta.TT, tile = __builtin_amdgcn_workgroup_id_x() - team * ta.TT;
  const __amdgpu_buffer_rsrc_t hs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(ta.hsave + (size_t)__builtin_amdgcn_workgroup_id_x() * WB * 64 * 4), 0, WB * 64 * 4, 0x00020000);
  unsigned* ctr = ta.counters + (size_t)team * TEAM_CTR_STRIDE;
  char* tslots = ta.slots + (size_t)team * 2 * ta.TT * SLOT_BYTES;
  constexpr int NL = ADS ? 32 : 30;             // big layers
  // the next layer's weights: prefetched by the conv before a CBAM (held across it), or loaded
  constexpr bool RELOAD_A = false;
  unsigned nbar = 0;
  f32x4 id[16];
  Stamps stamp;
  stamp.init();
  zero_guards(lds);
  for (int64_t n = team; n < ta.n; n += ta.teams) {
    Tile tl;
    tl.lds = lds;
    tl.x = x + (size_t)n * L;
    tl.L = L;
    tl.base = tile * ta.T - ta.halo;
    tl.small = (const float*)blob;
    tl.big = blob + SMALL_BYTES;
    tl.layer = 0;
    tl.corr = corr_mask(blob);
    tl.amax = 0.f;
    tl.status = ta.err + 3;               // the stems raise the input gate
    LayerA<MODE> a;
    load_layer_a<MODE>(tl, 0, a);
    bool tainted = false;                 // MODE_H8: a tile of this spectrum saturated (apply_cbam)
    // stats of u -> team -> apply.  The identity rows are fetched while the team assembles; the
    // next layer's operands are loaded only now (held across this VALU-heavy code they spill).
    auto cbam = [&](int slot, int res, bool save_next) {
      char* mine = tslots + ((size_t)(nbar & 1) * ta.TT + tile) * SLOT_BYTES;
      const bool skip = ta.force_miss > 0 && __builtin_amdgcn_workgroup_id_x() == 0 && nbar + 1 == (unsigned)ta.force_miss;
      publish_stats<MODE>(tl, ta, mine, ctr, stamp, !skip);
      stamp(3);
      team_wait(ta, ctr, (nbar + 1) * (unsigned)ta.TT);
      stamp(4);
      tainted = apply_cbam<MODE>(tl, ta, tslots + (size_t)(nbar & 1) * ta.TT * SLOT_BYTES, slot, ADS, res, save_next, hs,
                                 stamp) || tainted;
      stamp(5);
      ++nbar;
      if (RELOAD_A && tl.layer < NL) load_layer_a<MODE>(tl, tl.layer, a);
    };
    stem<MODE>(tl, 0);
    __syncthreads();
    if (ADS) {
      // ADSDN/train.py:160-167: cbam(relu(conv_ds x)); relu(conv1); relu(conv2); cbam;
      // 15 x relu(cbam(bn2(conv2(relu(bn1(conv1 x))))) + x); conv_out
      cbam(2, RES_NONE, false);
      conv<MODE, RELU, G::S>(tl, 1, id, a, true);
      conv<MODE, RELU, G::S>(tl, 1, id, a, !RELOAD_A);
      cbam(5, RES_NONE, true);                   // block 0's identity
      for (int b = 0; b < 15; ++b) {
        conv<MODE, RELU, G::S>(tl, 1, id, a, true);
        conv<MODE, 0, G::S>(tl, 1, id, a, !RELOAD_A && tl.layer + 1 < NL);
        cbam(8 + 3 * b, RES_ADD_RELU, b < 14);
      }
    } else {
      // APIDN/train.py:150-159: h = relu(conv_ds x); 15 x x += cbam(bn(conv(relu(bn(conv x)))));
      // sigmoid(conv_out(x + h))
      save_identity<MODE>(tl, hs);
      for (int b = 0; b < 15; ++b) {
        stamp(7);
        conv<MODE, RELU, G::S>(tl, 1, id, a, true);
        stamp(1);
        conv<MODE, 0, G::S>(tl, 1, id, a, !RELOAD_A && tl.layer + 1 < NL);
        stamp(2);
        cbam(2 + 3 * b, RES_ADD, b < 14);
      }
      stem<MODE, true>(tl, 0);       // + h, recomputed from x
      __syncthreads();
    }
    double d[HeadOut<MODE>::ROWS];
    head<MODE>(tl, 1, d);
    float v[HeadOut<MODE>::ROWS];
    round_rows(d, v);
    if (!ADS) {
#pragma unroll
      for (int k = 0; k < HeadOut<MODE>::ROWS; ++k) v[k] = sigm(v[k]);
    }
    // a timed-out hand-off anywhere in the grid: this spectrum's CBAM statistics may be incomplete,
    // so its outputs are NaN rather than plausible-looking garbage
    if (__hip_atomic_load(ta.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
#pragma unroll
      for (int k = 0; k < HeadOut<MODE>::ROWS; ++k) v[k] = __uint_as_float(0x7fc00000u);   // quiet NaN (bit pattern: -fno-honor-nans build)
    }
    // MODE_H8 range guard: a tile whose activations saturated raises the sticky range word (err[2],
    // the authoritative signal: its CBAM statistics reached the whole team) and writes NaN
    if constexpr (MODE == MODE_H8) {
      // (and every other tile of a spectrum one of whose tiles saturated: its clamped statistics
      // reached them through the hand-offs -- the whole spectrum is NaN, not just that tile)
      if (range_vote(tl, RED_OFF, ta.err + 2) || tainted) nan_rows(v);
    }
    store_out<MODE>(tl, y, (int)n, v, ta.halo, ta.T);
    __syncthreads();                 // the next spectrum's stem overwrites the rows the head read
    stamp(6);
  }
  if (RDN_TEAM_STAMPS && __builtin_amdgcn_workitem_id_x() == 0 && ta.stamps)
    for (int k = 0; k < NSTAMP; ++k) ta.stamps[(size_t)__builtin_amdgcn_workgroup_id_x() * NSTAMP + k] = stamp.acc[k];
}


// ---- team-persistent forward on the ping-pong engine (RDN_F16) ------------------------------------
//
// The same team protocol as team_forward (statistics + edge rows published per tile, one counter
// barrier per CBAM, deterministic slot reduction, spin limit -> error word), with the convs on the
// f16 ping-pong engine of fused16.hpp: 640-row tiles (T = 628 own positions, TEAM_HALO = 6 per
// side: 16 tiles per spectrum at L = 10,000), two 80 KiB activation buffers, one barrier per conv.
// Every CBAM's input u ends in BUF0; BUF1 is free during the CBAM and holds its scratch.  The
// ResidualBlock identity (the block input, which conv2 overwrites in BUF0) is saved by conv2's
// epilogue (fused16.hpp LINEAR_SAVE) into 10 x 8 f16 per lane, in that epilogue's (row, slot)
// layout, which every pointwise pass of the CBAM below uses: lane (w, q, c16) owns rows
// 160 (w % 4) + 16 n + c16 (n < 10) at 16-B slot 4 (w / 4) + q, i.e. channels h16_channel(slot, j).
// Statistics in fp32 per lane, fp64 across waves and tiles; ca / sa in fp32; u, h and the identity
// are f16 (the mode's storage).  ADSDN/train.py:72-167, APIDN/train.py:72-159.
namespace t16 {
using V = h16c::V;
constexpr int WB16 = h16c::WB;
constexpr int NT = h16c::NT;
constexpr int EDGE16_BYTES = EDGE_ROWS * h16c::ROWB;        // one edge, f16 rows
// The hand-off carries its own completion -- every 4-byte word of a slot
// travels as an 8-byte granule {word, tag} written by one sc1 store (tag = the CBAM's sequence
// number + 1; the slots are zeroed before each launch), and a consumer polls the granules it needs
// until every tag is current.  The producer neither drains its stores nor meets a counter, and the
// consumer's poll IS its read (one memory round trip after the last producer's stores land instead
// of drain + counter add + counter poll + slot loads: MI355X_MICROARCH.md handoff-1to1 vs
// handoff-flag).  Slot = 64 channel sums (f32: each tile's sum of its fp32 lane partials, rounded
// once) | 64 ordered maxima | 2 x EDGE_ROWS rows of u (f16) as 4-byte words.
constexpr int G_SUM = 0, G_MAX = 64, G_EDGE = 128;               // granule indices within a slot
// The spatial mean over channels runs as two MFMAs per row group (A = ca), the spatial conv7 two
// rows per thread in one round, the channel-attention MLP's 8 hidden sums as one lane butterfly
// (DESIGN.md §3 CBAM table; a per-wave conv7 with recomputed halo rows measured 0.4-2 % slower).
// Teams placed on one XCD each (team16_forward) hand off through that XCD's L2 (plain slot stores)
// once the launch's first CBAM has confirmed the placement.
constexpr int POLL_PER = 4;                                      // poll rounds batched per wave
// s_getreg operand of HW_REG_XCC_ID (id 20), bits [3:0]
constexpr int HWREG_XCC_ID = (3 << 11) | 20;
constexpr int EDGE16_WORDS = EDGE16_BYTES / 4;                   // 160 per edge
constexpr int SLOT16_BYTES = (G_EDGE + 2 * EDGE16_WORDS) * 8;    // 448 granules = 3584 B
// CBAM scratch in BUF1
constexpr int SC = h16c::BUF1;
constexpr int RED16_OFF = SC;                                  // [4 row blocks][64] f32 sums, then u32 maxima
constexpr int SLP_OFF = RED16_OFF + 2 * 4 * 64 * 4;            // [8 waves][64] f64 slot partials, then u32
constexpr int POOL_OFF = SLP_OFF + 8 * 64 * 12;                // [2][64] f64: pooled avg / max
constexpr int CA16_OFF = POOL_OFF + 2 * 64 * 8;                // channel attention, one copy per wave (8 x 64 f32)
constexpr int SA16_OFF = CA16_OFF + 8 * 64 * 4;                // spatial attention per tile row
constexpr int M1_OFF = SA16_OFF + WB16 * 4;                    // [mean_c; max_c] map, rows -3 .. WB + 2
constexpr int M2_OFF = M1_OFF + (WB16 + 8) * 4;
constexpr int VOTE16_OFF = M2_OFF + (WB16 + 8) * 4;           // [2][8] u32 workgroup votes (wg_all)
static_assert(VOTE16_OFF + 2 * 8 * 4 <= (int)h16c::LDS_BYTES, "CBAM scratch fits BUF1");

// Workgroup-wide AND of a per-thread predicate: a wave ballot, one LDS word per wave (two parity
// sets, so a vote needs one barrier), read back by every thread.  (__syncthreads_and would declare
// static LDS, which a kernel holding all 160 KiB dynamically cannot have.)
__device__ __forceinline__ bool wg_all(char* lds, bool v, unsigned& parity) {
  unsigned* vote = (unsigned*)(lds + VOTE16_OFF) + 8 * (parity & 1);
  const bool wave_ok = __builtin_amdgcn_ballot_w64(v) == ~0ull;
  if ((h16c::tid() & 63) == 0) vote[h16c::tid() >> 6] = wave_ok ? 1u : 0u;
  __syncthreads();
  bool all = true;
#pragma unroll
  for (int k = 0; k < h16c::WAVES; ++k) all = all && vote[k] != 0;
  ++parity;
  return all;
}

struct Lane {             // this lane's (row, slot) items of the pointwise passes
  int w, h, rb, q, c16;
  __device__ __forceinline__ Lane() {
    const int t = h16c::tid();
    w = __builtin_amdgcn_readfirstlane(t >> 6);
    h = w / h16c::RB;
    rb = w % h16c::RB;
    q = (t & 63) >> 4;
    c16 = t & 15;
  }
  __device__ __forceinline__ int row(int n) const { return rb * h16c::RW + 16 * n + c16; }
  __device__ __forceinline__ int slot() const { return 4 * h + q; }
};
// sum / max over the 16 lanes of a row by DPP (pair, quad, half-row mirror, row mirror): every lane
// of the row ends with the row's value, one VALU op per step
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float row_sum(float v) {
  v += dpp<0xB1>(v);
  v += dpp<0x4E>(v);
  v += dpp<0x141>(v);
  return v + dpp<0x140>(v);
}
__device__ __forceinline__ float row_max(float v) {
  v = fmaxf(v, dpp<0xB1>(v));
  v = fmaxf(v, dpp<0x4E>(v));
  v = fmaxf(v, dpp<0x141>(v));
  return fmaxf(v, dpp<0x140>(v));
}
// over lanes l, l ^ 16, l ^ 32, l ^ 48 (v_permlane32/16_swap)
__device__ __forceinline__ float quarter_max(float v) {
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  const float h = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(h), __float_as_uint(h), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

// per-channel sum / max of u (BUF0) over the tile's own positions and its edge rows -> slot (sc1);
// arrive at the team counter
typedef unsigned int gu32x2 __attribute__((ext_vector_type(2)));
template <int AUX>
__device__ __forceinline__ void slot_store64(gu32x2 v, __amdgpu_buffer_rsrc_t sr, int off) {
  __builtin_amdgcn_raw_buffer_store_b64(v, sr, off, 0, AUX);
}
template <int AUX>
__device__ __forceinline__ void slot_store128(u32x4 v, __amdgpu_buffer_rsrc_t sr, int off) {
  __builtin_amdgcn_raw_buffer_store_b128(v, sr, off, 0, AUX);
}
// xmode: XM_PROBE = the launch's first CBAM (sc1 stores; every sum granule's tag carries
// bit 31 when this tile cannot hand off through its XCD's L2), XM_L2 = plain stores (the line stays
// in the team's one L2, which every member's L1-bypassing loads read), XM_SC1 = sc1 stores
enum XMode : int { XM_PROBE = 0, XM_L2 = 1, XM_SC1 = 2 };
constexpr unsigned TAG_OFF_XCD = 0x80000000u;
__device__ __forceinline__ void publish16(const h16c::Tile& tl, const TeamArgs& ta, char* slot, unsigned* ctr,
                                          bool arrive, const h16c::ChanStats* pre, unsigned tag, int xmode,
                                          bool local, Stamps& st) {
  char* lds = tl.lds;
  const Lane ln;
  const int tid = h16c::tid();
  const int H = ta.halo, T = ta.T;
  const int rend = H + min(T, tl.L - tl.base - H);
  // this lane's channel partials: accumulated by the conv that produced u (pre: its epilogue, from
  // the unrounded values), or from u in BUF0
  h16c::f32x8 sm = (h16c::f32x8)(0.f), mx = (h16c::f32x8)(-INFINITY);
  if (pre) {
    sm = pre->sum;
    mx = pre->max;
  } else {
    const char* b0 = lds + h16c::BUF0 + (ln.h ? tl.koff[2][1] : tl.koff[2][0]);
    V uv[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) uv[n] = *(const V*)(b0 + n * 16 * h16c::ROWB);
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const int r = ln.row(n);
      if (r >= H && r < rend) {
        const h16c::f32x8 u = __builtin_convertvector(uv[n], h16c::f32x8);
        sm += u;
        mx = __builtin_elementwise_max(mx, u);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sm[j] = row_sum(sm[j]);
    mx[j] = row_max(mx[j]);
  }
  float* rs = (float*)(lds + RED16_OFF);
  unsigned* rm = (unsigned*)(lds + RED16_OFF + 4 * 64 * 4);
  if (ln.c16 == 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = h16_channel(ln.slot(), j);
      rs[ln.rb * 64 + c] = sm[j];
      rm[ln.rb * 64 + c] = f2ord(mx[j]);
    }
  }
  st(14);
  __syncthreads();
  st(15);
  // one store phase, no drain, no arrival: the statistics (wave 0: granules {f32 sum, tag} and
  // {ordered max, tag}) and the edge rows (u, f16) for the neighbours (waves 1-2: two granules per
  // 16-B sc1 store): block 0 = rows [2H - 5, 2H) (the left neighbour's rows [WB - 5, WB)), block 1 =
  // rows [T, T + 5).  arrive = false (test knob) publishes nothing.
  if (!arrive) return;
  const __amdgpu_buffer_rsrc_t sr = __builtin_amdgcn_make_buffer_rsrc((void*)slot, 0, SLOT16_BYTES, 0x00020000);
  if (tid < 64) {
    const int c = tid;
    double sv = 0.0;
    unsigned m = 0;
#pragma unroll
    for (int k = 0; k < h16c::RB; ++k) {
      sv += (double)rs[k * 64 + c];
      m = max(m, rm[k * 64 + c]);
    }
    const unsigned tsum = xmode == XM_PROBE && !local ? tag | TAG_OFF_XCD : tag;
    if (xmode == XM_L2) {
      slot_store64<0>(gu32x2{__float_as_uint((float)sv), tsum}, sr, 8 * (G_SUM + c));
      slot_store64<0>(gu32x2{m, tag}, sr, 8 * (G_MAX + c));
    } else {
      slot_store64<16>(gu32x2{__float_as_uint((float)sv), tsum}, sr, 8 * (G_SUM + c));
      slot_store64<16>(gu32x2{m, tag}, sr, 8 * (G_MAX + c));
    }
  } else if (tid < 64 + 2 * EDGE_ROWS * 8) {
    const int i = tid - 64, e = i / (EDGE_ROWS * 8), k = (i / 8) % EDGE_ROWS, g = i & 7;
    const int r = e == 0 ? WB16 - T - EDGE_ROWS + k : T + k;
    const u32x4 v = *(const u32x4*)(lds + h16c::BUF0 + h16c::soff(r, g));
    const int g0 = G_EDGE + e * EDGE16_WORDS + (k * 8 + g) * 4;
    if (xmode == XM_L2) {
      slot_store128<0>(u32x4{v[0], tag, v[1], tag}, sr, 8 * g0);
      slot_store128<0>(u32x4{v[2], tag, v[3], tag}, sr, 8 * g0 + 16);
    } else {
      slot_store128<16>(u32x4{v[0], tag, v[1], tag}, sr, 8 * g0);
      slot_store128<16>(u32x4{v[2], tag, v[3], tag}, sr, 8 * g0 + 16);
    }
  }
  (void)ctr;
}

// apply the CBAM whose statistics sit in the team's slots to u (BUF0): h = [identity +] u*ca*sa
// [then ReLU], written over u; idv: the identity (LINEAR_SAVE layout) for res != RES_NONE
template <bool EDGE>
__device__ __forceinline__ void apply16(const h16c::Tile& tl, const TeamArgs& ta, const char* slots0, int cbam_slot,
                                        bool bias, int res, const V* idv, Stamps& st, unsigned tag, int& xmode,
                                        bool local) {
  char* lds = tl.lds;
  const Lane ln;
  const int tid = h16c::tid(), lane = tid & 63, w = ln.w;
  const float* cw = tl.small + cbam_slot * SMALL_SLOT_FLOATS;      // fc.0.weight [4][64]
  const float* cw2 = cw + SMALL_SLOT_FLOATS;                       // fc.2.weight [64][4]
  const float* cmisc = cw2 + SMALL_SLOT_FLOATS;                    // fc.0.bias[4], fc.2.bias[64], sa.w[2][7], sa.b
  f32x4 w1v;                                                       // fc.0 column `lane` (4 hidden units)
#pragma unroll
  for (int j = 0; j < 4; ++j) w1v[j] = cw[j * 64 + lane];
  const f32x4 cw2v = *(const f32x4*)(cw2 + 4 * lane);
  const float b2 = bias ? cmisc[4 + lane] : 0.f;
  const __amdgpu_buffer_rsrc_t sr = __builtin_amdgcn_make_buffer_rsrc((void*)slots0, 0, ta.TT * SLOT16_BYTES, 0x00020000);

  // the granules this thread needs, polled until every tag is `tag` (uniform loop: one workgroup
  // vote per round): the halo refresh (threads < 80: u of rows [0, 5) from the left neighbour's
  // block 1, rows [WB - 5, WB) from the right neighbour's block 0; first / last tile: no
  // neighbour) and the spectrum's per-channel sums / maxima from the TT slots (thread (c, part):
  // slots part + 8k), combined in a fixed order
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  const int edge_e = tid / (EDGE_ROWS * 8), edge_k = (tid / 8) % EDGE_ROWS, edge_g = tid & 7;
  int eoff = -1;
  if (tid < 2 * EDGE_ROWS * 8) {
    const int tile = (tl.base + ta.halo) / ta.T;
    const int nb = edge_e == 0 ? tile - 1 : tile + 1;
    if (nb >= 0 && nb < ta.TT)
      eoff = nb * SLOT16_BYTES + 8 * (G_EDGE + (1 - edge_e) * EDGE16_WORDS + (edge_k * 8 + edge_g) * 4);
  }
  u32x4 ea = {0u, 0u, 0u, 0u}, eb = {0u, 0u, 0u, 0u};
  bool edge_ok = eoff < 0;
  {
    const int c = tid & 63, part = tid >> 6;
    // slots per thread per poll batch: 4 -> one batch (one round trip) for up to 32 tiles, i.e. up to
    // L = 20,096 (L = 16,384: 27 tiles; 2 per thread made that two batches polled one after the other)
    constexpr int PER = POLL_PER, STEP = h16c::WAVES * PER;
    const int nbatch = (ta.TT + STEP - 1) / STEP;
    // this tile's own slot is not polled: its granules are the values publish16 stored, recomputed
    // from the same LDS partials in the same order (same bits), so the last tile to publish goes on
    // without a round trip through memory for its own statistics
    const int own = (tl.base + ta.halo) / ta.T;
    double sp = 0.0;
    unsigned mp = 0;
    bool failed = false, off_xcd = false;
    unsigned vparity = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int b = 0; b < nbatch; ++b) {
      u32x2 sv[PER], mv[PER];
      bool ok[PER];
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int t = part + STEP * b + h16c::WAVES * k;
        ok[k] = t >= ta.TT || t == own;
        if (t == own) {
          const float* rs = (const float*)(lds + RED16_OFF);
          const unsigned* rm = (const unsigned*)(lds + RED16_OFF + 4 * 64 * 4);
          double s0 = 0.0;
          unsigned m0 = 0;
#pragma unroll
          for (int j = 0; j < h16c::RB; ++j) {
            s0 += (double)rs[j * 64 + c];
            m0 = max(m0, rm[j * 64 + c]);
          }
          sv[k] = u32x2{__float_as_uint((float)s0), tag};
          mv[k] = u32x2{m0, tag};
        }
      }
      for (unsigned it = 0;; ++it) {
#pragma unroll
        for (int k = 0; k < PER; ++k) {
          if (!ok[k]) {
            const int off = (part + STEP * b + h16c::WAVES * k) * SLOT16_BYTES;
            sv[k] = __builtin_amdgcn_raw_buffer_load_b64(sr, off + 8 * (G_SUM + c), 0, 16);
            mv[k] = __builtin_amdgcn_raw_buffer_load_b64(sr, off + 8 * (G_MAX + c), 0, 16);
          }
        }
        if (b == 0 && !edge_ok) {
          ea = __builtin_amdgcn_raw_buffer_load_b128(sr, eoff, 0, 16);
          eb = __builtin_amdgcn_raw_buffer_load_b128(sr, eoff + 16, 0, 16);
        }
        bool mine = true;
#pragma unroll
        for (int k = 0; k < PER; ++k) {
          ok[k] = ok[k] || ((sv[k][1] & ~TAG_OFF_XCD) == tag && mv[k][1] == tag);
          mine = mine && ok[k];
        }
        if (b == 0) {
          edge_ok = edge_ok || (ea[1] == tag && ea[3] == tag && eb[1] == tag && eb[3] == tag);
          mine = mine && edge_ok;
        }
        if (wg_all(lds, mine, vparity)) break;
        // a wait that exceeds SPIN_LIMIT rounds or SPIN_TICKS (a team member never published: co-residency
        // broken) raises the error words; once they are up every wait falls through (NaN outputs)
        if (failed || it > SPIN_LIMIT) {
          if (tid == 0 && !failed) {
            __hip_atomic_store(ta.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(ta.err + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          failed = true;
          break;
        }
        // every 64 rounds: thread 0 raises the error words once the wait passed SPIN_TICKS, and the
        // workgroup reads them in one vote (thread 0 sees its own store: the break is uniform)
        if ((it & 63) == 63 && tid == 0 && __builtin_amdgcn_s_memrealtime() - t0 > SPIN_TICKS) {
          __hip_atomic_store(ta.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(ta.err + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if ((it & 63) == 63 &&
            !wg_all(lds, __hip_atomic_load(ta.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0, vparity)) {
          failed = true;
          break;
        }
        __builtin_amdgcn_s_sleep(RDN_TEAM_SLEEP);
      }
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        if (part + STEP * b + h16c::WAVES * k < ta.TT) {
          sp += (double)__uint_as_float(sv[k][0]);
          mp = max(mp, mv[k][0]);
          off_xcd = off_xcd || (sv[k][1] & TAG_OFF_XCD) != 0;
        }
      }
    }
    double* ps = (double*)(lds + SLP_OFF);
    unsigned* pm = (unsigned*)(lds + SLP_OFF + 8 * 64 * 8);
    ps[part * 64 + c] = sp;
    pm[part * 64 + c] = mp;
    // the launch's first CBAM: every member has now seen every member's placement bit (its own:
    // `local`), so the whole team takes the same decision
    if (xmode == XM_PROBE) xmode = wg_all(lds, local && !off_xcd && !failed, vparity) ? XM_L2 : XM_SC1;
  }
  if (eoff >= 0) {
    const int r = edge_e == 0 ? edge_k : WB16 - EDGE_ROWS + edge_k;
    *(u32x4*)(lds + h16c::BUF0 + h16c::soff(r, edge_g)) = u32x4{ea[0], ea[2], eb[0], eb[2]};
  }
  __syncthreads();
  st(10);
  // the spatial pass's u rows (below), fetched now: their LDS latency hides under the MLP's chain
  constexpr int SROWS = WB16 / h16c::WAVES;    // 80 rows per wave
  static_assert(SROWS % 16 == 0, "whole 16-row groups per wave");
  V ua[SROWS / 16], ub[SROWS / 16];
#pragma unroll
  for (int k = 0; k < SROWS / 16; ++k) {
    const int r = SROWS * w + ln.c16 + 16 * k;
    ua[k] = *(const V*)(lds + h16c::BUF0 + h16c::soff(r, ln.q));
    ub[k] = *(const V*)(lds + h16c::BUF0 + h16c::soff(r, ln.q + 4));
  }
  // channel attention, evaluated whole by every wave (no barrier): the pooled avg / max of channel
  // `lane` from the 8 partials in a fixed order, the 4 + 4 hidden units as sums over the 64 lanes
  float cav;
  {
    const double* ps = (const double*)(lds + SLP_OFF);
    const unsigned* pm = (const unsigned*)(lds + SLP_OFF + 8 * 64 * 8);
    double sum = 0.0;
    unsigned m = 0;
#pragma unroll
    for (int k = 0; k < h16c::WAVES; ++k) {
      sum += ps[k * 64 + lane];
      m = max(m, pm[k * 64 + lane]);
    }
    const float pa = (float)sum * __builtin_amdgcn_rcpf((float)tl.L), px = ord2f(m);
    // the 8 hidden sums (fc.0 row j of the pooled avg / max, over the 64 lanes = channels) by one
    // butterfly instead of 8 separate reductions: lane halves swap (avg | max), then lane quarters
    // (j pairs), rows of 8 (ror 8), and 3 DPP adds finish each 8-lane group; lane 8g of the wave then
    // holds hidden sum (avg if g < 4 else max, j = {0, 2, 1, 3}[g & 3])
    float t[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(w1v[j] * pa), __float_as_uint(w1v[j] * px), false, false);
      t[j] = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
    }
    float u[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(t[2 * k]), __float_as_uint(t[2 * k + 1]), false, false);
      u[k] = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
    }
    const bool hi8 = (lane & 8) != 0;
    float r = (hi8 ? u[1] : u[0]) + dpp<0x128>(hi8 ? u[0] : u[1]);     // row_ror:8
    r += dpp<0xB1>(r);
    r += dpp<0x4E>(r);
    r += dpp<0x141>(r);
    float oa = 2.f * b2;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int g = j == 0 ? 0 : j == 1 ? 2 : j == 2 ? 1 : 3;          // lane group of hidden unit j
      const float b1 = bias ? cmisc[j] : 0.f;
      const float ha = fmaxf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(r), 8 * g)) + b1, 0.f);
      const float hm = fmaxf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(r), 32 + 8 * g)) + b1, 0.f);
      oa = fmaf(cw2v[j], ha + hm, oa);
    }
    cav = sigm_fast(oa);
  }
  // this lane's 8 channels of ca through the wave's own LDS row (in-order within a wave)
  float* caw = (float*)(lds + CA16_OFF) + 64 * w;
  caw[lane] = cav;
  st(11);

  // spatial statistics of u*ca in packed f16 (the mode's storage precision: u is f16, ca rounds to
  // f16): wave w takes rows 80w .. 80w + 79, lane (q, c16) the rows 80w + c16 + 16k (k < 5) at
  // slots q and q + 4 (16 channels), the 4 quarters (all 64 channels) by lane swaps -- every row's
  // [mean; max] completes inside one wave; partial sums / maxima to f32
  char* b0 = lds + h16c::BUF0 + (ln.h ? tl.koff[2][1] : tl.koff[2][0]);
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  // ca of this lane's pointwise slot; of slots q and q + 4 (h16_channel(g, j): channels j < 4 and
  // j >= 4 are 4 consecutive channels each, so two 16-B LDS reads per slot)
  auto ca_slot = [&](int g) {
    const int c0 = h16_channel(g, 0);
    const f32x4 lo = *(const f32x4*)(caw + c0), hi = *(const f32x4*)(caw + c0 + 16);
    return __builtin_convertvector(__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7), V);
  };
  const V cah = ca_slot(ln.slot()), cq0 = ca_slot(ln.q), cq4 = ca_slot(ln.q + 4);
  float* m1 = (float*)(lds + M1_OFF) + 3;      // [mean_c; max_c] of rows -3 .. WB + 2, zero outside
  float* m2 = (float*)(lds + M2_OFF) + 3;      // the tile and [0, L)
  {
#pragma unroll
    for (int k = 0; k < SROWS / 16; ++k) {
      const V va = ua[k] * cq0, vb = ub[k] * cq4;
      const V vm = __builtin_elementwise_max(va, vb);
      // sum_c ca_c u_c of row c16 on the idle MFMA pipe: A = ca (every row of the 16 x 32 A-operand
      // the same, its K order the B-fragment channel order of slots q / q + 4: cq0 / cq4), B = the
      // two u fragments this lane holds anyway; every output row is the sum, exact f16 products
      // accumulated in fp32 -- no pk_add tree and no cross-lane sum
      const f32x4 dsum = h16c::mma(cq4, ub[k], h16c::mma(cq0, ua[k], (f32x4)(0.f)));
      const float sm = dsum[0];
      const h2 x2 = __builtin_elementwise_max(
          __builtin_elementwise_max(__builtin_shufflevector(vm, vm, 0, 1), __builtin_shufflevector(vm, vm, 2, 3)),
          __builtin_elementwise_max(__builtin_shufflevector(vm, vm, 4, 5), __builtin_shufflevector(vm, vm, 6, 7)));
      const float mx = quarter_max(fmaxf((float)x2[0], (float)x2[1]));
      // (rows at positions outside [0, L) hold u = 0 -- conv2's zero_outside, and no neighbour refreshes
      // an edge tile's outer halo -- so their mean and max come out 0, the map's zero padding, with no
      // per-row check)
      if (ln.q == 0) {
        const int r = SROWS * w + ln.c16 + 16 * k;
        m1[r] = sm * (1.0f / 64.0f);
        m2[r] = mx;
      }
    }
    if (tid < 6) {                             // rows beyond the tile feed only halo rows: 0
      const int r = tid < 3 ? tid - 3 : WB16 + tid - 3;
      m1[r] = 0.f;
      m2[r] = 0.f;
    }
  }
  __syncthreads();
  st(12);
  // the product pass's u rows (below), fetched now: their latency hides under conv7
  V uv[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n) uv[n] = *(const V*)(b0 + n * 16 * h16c::ROWB);
  // sa = sigmoid(conv7([mean_c; max_c]))
  float* sa = (float*)(lds + SA16_OFF);
  // two adjacent rows per thread (their 7-tap windows share 6 rows): the 320 row pairs of the tile
  // in one round instead of 640 rows in two
  for (int i = tid; i < WB16 / 2; i += h16c::THREADS) {
    const int r = 2 * i;
    float a0 = bias ? cmisc[82] : 0.f, a1 = a0;
    float p1[8], p2[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      p1[k] = m1[r + k - 3];
      p2[k] = m2[r + k - 3];
    }
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      a0 = fmaf(cmisc[68 + k], p1[k], a0);
      a0 = fmaf(cmisc[75 + k], p2[k], a0);
      a1 = fmaf(cmisc[68 + k], p1[k + 1], a1);
      a1 = fmaf(cmisc[75 + k], p2[k + 1], a1);
    }
    sa[r] = sigm_fast(a0);
    sa[r + 1] = sigm_fast(a1);
  }
  __syncthreads();
  st(13);
  // h = [identity +] u*ca*sa [relu], in place, packed f16.  Rows at positions outside [0, L) stay zero
  // without a check: u is 0 there (conv2's zero_outside; the stem's for the first CBAM), ca and sa are
  // finite, and the identity -- the block input, an earlier h -- is 0 there too
  float sv[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n) sv[n] = sa[ln.row(n)];
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    V* pu = (V*)(b0 + n * 16 * h16c::ROWB);
    V hv = (uv[n] * cah) * (V)((_Float16)sv[n]);
    if (res != RES_NONE) {
      hv += idv[n];
      if (res == RES_ADD_RELU) hv = __builtin_elementwise_max(hv, (V)((_Float16)0));
    }
    *pu = hv;
  }
  __syncthreads();
}

// The spectra of team `team`: a contiguous range.  Teams 0 .. nloc-1 sit on one XCD each; the rest
// (L = 16,384: 27-tile teams, 9 per chip, the ninth spread over the XCDs' spare CUs) hand off across
// XCDs and run ~3 % slower per spectrum (tools/team_stamps.py: 4.61e7 vs 4.47e7 cycles), so with
// XCD-local hand-offs they take 31/32 of a local team's share and the launch's teams finish together.
__device__ __forceinline__ void team_range(const TeamArgs& ta, int team, int nloc, int64_t& lo, int64_t& hi) {
  const int64_t ws = ta.xcd && nloc < ta.teams ? 31 : 32;
  auto cum = [&](int t) -> int64_t { return t <= nloc ? 32LL * t : 32LL * nloc + ws * (t - nloc); };
  const int64_t W = cum(ta.teams);
  lo = (ta.n * cum(team) + W - 1) / W;         // rounded up: with fewer spectra than teams, team 0
  hi = (ta.n * cum(team + 1) + W - 1) / W;     // takes spectrum 0
}

template <bool ADS, bool EDGE>
__device__ __forceinline__ void team16_spectra(char* lds, const uint8_t* blob, const uint8_t* big16, const float* x,
                                               float* y, int L, const TeamArgs& ta, int team, int tile,
                                               bool local, int nloc) {
  unsigned* ctr = ta.counters + (size_t)team * TEAM_CTR_STRIDE;
  int xmode = ta.xcd ? XM_PROBE : XM_SC1;
  char* tslots = ta.slots + (size_t)team * 2 * ta.TT * SLOT16_BYTES;
  unsigned nbar = 0;
  Stamps st;
  st.init();
  int64_t n_lo, n_hi;
  team_range(ta, team, nloc, n_lo, n_hi);
  for (int64_t n = n_lo; n < n_hi; ++n) {
    h16c::Tile tl = h16c::init_tile(lds, blob, big16, x + (size_t)n * L, L, tile * ta.T - ta.halo);
    tl.status = ta.err + 3;               // the stems raise the input gate
    h16c::Frags F0, F1;
    V id[NT];
    h16c::ChanStats cs;
    auto conv2_stats = [&]() -> h16c::ChanStats* {   // the block's conv2 accumulates u's statistics
      cs.sum = (h16c::f32x8)(0.f);
      cs.max = (h16c::f32x8)(-INFINITY);
      cs.lo = ta.halo;
      cs.hi = ta.halo + min(ta.T, L - tl.base - ta.halo);
      return &cs;
    };
    auto cbam = [&](int slot, int res, const h16c::ChanStats* pre) {
      char* mine = tslots + ((size_t)(nbar & 1) * ta.TT + tile) * SLOT16_BYTES;
      const bool skip = ta.force_miss > 0 && __builtin_amdgcn_workgroup_id_x() == 0 && nbar + 1 == (unsigned)ta.force_miss;
      st(1);
      publish16(tl, ta, mine, ctr, !skip, pre, ta.tag0 + nbar + 1, xmode, local, st);
      st(3);
      st(4);
      apply16<EDGE>(tl, ta, tslots + (size_t)(nbar & 1) * ta.TT * SLOT16_BYTES, slot, ADS, res, id, st,
                    ta.tag0 + nbar + 1, xmode, local);
      st(5);
      ++nbar;
    };
    h16c::load_frags(tl, 0, F0);
    h16c::stem(tl, 0, h16c::BUF0);
    h16c::lds_barrier();
    if (ADS) {
      // ADSDN/train.py:160-167: cbam(relu(conv_ds x)); relu(conv1); relu(conv2); cbam;
      // 15 x relu(cbam(bn2(conv2(relu(bn1(conv1 x))))) + x); conv_out
      cbam(2, RES_NONE, nullptr);
      h16c::layer<h16c::RELU, EDGE>(tl, h16c::BUF0, h16c::BUF1, 1, F0, F1);
      h16c::layer<h16c::RELU, EDGE>(tl, h16c::BUF1, h16c::BUF0, 1, F1, F0);
      cbam(5, RES_NONE, nullptr);
      for (int b = 0; b < 15; ++b) {
        h16c::layer<h16c::RELU, EDGE>(tl, h16c::BUF0, h16c::BUF1, 1, F0, F1);
        h16c::layer<h16c::LINEAR_SAVE, EDGE>(tl, h16c::BUF1, h16c::BUF0, 1, F1, F0, true, id, conv2_stats());
        cbam(8 + 3 * b, RES_ADD_RELU, &cs);
      }
    } else {
      // APIDN/train.py:150-159: h = relu(conv_ds x); 15 x x += cbam(bn(conv(relu(bn(conv x)))));
      // sigmoid(conv_out(x + h))
      for (int b = 0; b < 15; ++b) {
        h16c::layer<h16c::RELU, EDGE>(tl, h16c::BUF0, h16c::BUF1, 1, F0, F1);
        h16c::layer<h16c::LINEAR_SAVE, EDGE>(tl, h16c::BUF1, h16c::BUF0, 1, F1, F0, true, id, conv2_stats());
        cbam(2 + 3 * b, RES_ADD, &cs);
      }
      h16c::stem<true>(tl, 0, h16c::BUF0);       // + h, recomputed from x
      h16c::lds_barrier();
    }
    float o[h16c::HN];
    h16c::head<EDGE>(tl, h16c::BUF0, F0, F1, false, o);
    const bool failed = __hip_atomic_load(ta.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
#pragma unroll
    for (int k = 0; k < h16c::HN; ++k) {
      if (!ADS) o[k] = sigm(o[k]);
      if (failed) o[k] = __uint_as_float(0x7fc00000u);     // quiet NaN: an incomplete CBAM hand-off
    }
    h16c::store_out(tl, y, (int)n, o, ta.halo, ta.T);
    __syncthreads();                 // the next spectrum's stem overwrites the rows the head read
    st(6);
  }
  if (RDN_TEAM_STAMPS && __builtin_amdgcn_workitem_id_x() == 0 && ta.stamps)
    for (int k = 0; k < NSTAMP; ++k) ta.stamps[(size_t)__builtin_amdgcn_workgroup_id_x() * NSTAMP + k] = st.acc[k];
}
}  // namespace t16

template <bool ADS>
__global__ __launch_bounds__(h16c::THREADS) void team16_forward(const uint8_t* __restrict__ blob,
                                                                const uint8_t* __restrict__ big16,
                                                                const float* __restrict__ x, float* __restrict__ y,
                                                                int L, TeamArgs ta) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int wg = __builtin_amdgcn_workgroup_id_x();
  int team = wg / ta.TT, tile = wg - team * ta.TT;
  bool local = false;
  // XCD-aware teams: workgroups are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md), so
  // workgroups 8r + x, r < R0, sit on XCD x; they form teams 8j + x of TT tiles (r = j TT + tile),
  // each on one XCD, and the workgroups from 8 R0 on form the remaining teams in order.  A member
  // whose XCC_ID is not x reports it at the first CBAM and its team hands off through sc1 instead.
  const int tpx = (ta.teams * ta.TT / 8) / ta.TT, R0 = tpx * ta.TT;
  if (wg < 8 * R0) {
    const int xc = wg & 7, r = wg >> 3;
    team = (r / ta.TT) * 8 + xc;
    tile = r % ta.TT;
    local = (__builtin_amdgcn_s_getreg(t16::HWREG_XCC_ID) & 0xf) == (unsigned)xc;
  } else {
    team = 8 * tpx + (wg - 8 * R0) / ta.TT;
    tile = (wg - 8 * R0) % ta.TT;
  }
  const int base = tile * ta.T - ta.halo;
  // a tile holds positions outside [0, L) for every spectrum or for none (one L per launch)
#if defined(RDN_ABLATE_ALLEDGE)          // diagnostic: every tile on the edge-tile code
  if (false) t16::team16_spectra<ADS, false>(lds, blob, big16, x, y, L, ta, team, tile, local, 8 * tpx);
#else
  if (base >= 0 && base + t16::WB16 <= L) t16::team16_spectra<ADS, false>(lds, blob, big16, x, y, L, ta, team, tile, local, 8 * tpx);
#endif
  else t16::team16_spectra<ADS, true>(lds, blob, big16, x, y, L, ta, team, tile, local, 8 * tpx);
}

}  // namespace cb

// ---- host ----------------------------------------------------------------------------------------

static constexpr int64_t CBAM_CHUNK = 1024;       // spectra per pass (bounds the workspace)

static size_t act_bytes(int64_t n, int64_t L) { return (size_t)n * L * 64 * sizeof(float); }
// The segment path's workspace: [256 B status: the MODE_H8 range words, [0] this forward's chunk, [1]
// sticky (cbam_status)] [4 activation buffers] [2 x statistics], 256-B aligned
static char* seg_base(void* ws) { return (char*)(((uintptr_t)ws + 255) & ~(uintptr_t)255); }
static unsigned* seg_range(void* ws) { return (unsigned*)seg_base(ws); }

// Team-persistent geometry: TEAM_HALO rows per side (refreshed from the neighbours at every CBAM),
// TT tiles per spectrum, as many teams as the device holds co-resident: the occupancy API's
// workgroups per CU for this kernel (LDS-bound: 1) x the CUs of the stream's device.
struct TeamGeo {
  int halo, T, TT, teams;
  size_t slots, counters, hsave, total;
};
typedef void (*team_kernel_t)(const uint8_t*, const float*, float*, int, cb::TeamArgs);
static team_kernel_t team_kernel(int arch, int mode) {
  using namespace cb;
  const bool ads = arch == ADSDN;
  if (mode == ip::MODE_F32) return ads ? team_forward<ip::MODE_F32, true> : team_forward<ip::MODE_F32, false>;
  if (mode == ip::MODE_X3) return ads ? team_forward<ip::MODE_X3, true> : team_forward<ip::MODE_X3, false>;
  if (mode == ip::MODE_H8) return ads ? team_forward<ip::MODE_H8, true> : team_forward<ip::MODE_H8, false>;
  if (mode == ip::MODE_F16) return ads ? team_forward<ip::MODE_F16, true> : team_forward<ip::MODE_F16, false>;
  return ads ? team_forward<ip::MODE_B1, true> : team_forward<ip::MODE_B1, false>;
}
// team kernel of RDN_F16 on the ping-pong engine (cb::team16_forward): its own team mode
constexpr int MODE_P16 = 8;
typedef void (*team16_kernel_t)(const uint8_t*, const uint8_t*, const float*, float*, int, cb::TeamArgs);
static team16_kernel_t team16_kernel(int arch) {
  return arch == ADSDN ? cb::team16_forward<true> : cb::team16_forward<false>;
}
size_t pp16_section_offset_arch(int arch);   // pack.cpp: the RDN_F16 blob's ping-pong section
static int dtype_mode(int dtype) {
  return dtype == F32 ? ip::MODE_F32 : dtype == BF16X3 ? ip::MODE_X3 : dtype == F16F8 ? ip::MODE_H8
       : dtype == F16 ? ip::MODE_F16 : ip::MODE_B1;
}
// attribute slots 40-49 (team kernels) and 64-68 (segment kernels), host_util.hpp
static int team_slot(int arch, int mode) { return mode == MODE_P16 ? 80 + (arch == ADSDN) : 40 + 2 * mode + (arch == ADSDN); }
static const void* team_fn(int arch, int mode) {
  return mode == MODE_P16 ? (const void*)team16_kernel(arch) : (const void*)team_kernel(arch, mode);
}
static int team_lds(int mode) { return mode == MODE_P16 ? (int)h16c::LDS_BYTES : (int)cb::SEG_LDS_BYTES; }
// the team kernel RDN_<dtype> runs (RDN_F16: the ping-pong one)
static int team_mode(int dtype) { return dtype == F16 ? MODE_P16 : dtype_mode(dtype); }

static int team_blocks_query(int arch, int mode, int dev) {
  const void* k = team_fn(arch, mode);
  if (ensure_dynamic_lds(k, team_slot(arch, mode), team_lds(mode), dev) != hipSuccess) {
    (void)hipGetLastError();          // no team geometry (the segment path runs); leave no sticky error behind
    return 0;
  }
  int cur = 0, nb = 0;
  if (hipGetDevice(&cur) != hipSuccess) return 0;
  if (cur != dev && hipSetDevice(dev) != hipSuccess) return 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, THREADS, team_lds(mode)) != hipSuccess) nb = 0;
  if (cur != dev) (void)hipSetDevice(cur);
  return nb;
}

// co-resident workgroups per CU of the team kernel on `dev` (0 on any failure), cached per (kernel,
// device): the occupancy query ran three times per call of the batch-1 loop (the forward's workspace
// check and launch, the status read)
static int team_blocks_per_cu(int arch, int mode, int dev) {
  static std::atomic<int> known[MAX_DEVICES * ATTR_SLOTS];           // blocks + 1; 0 = not queried yet
  const int slot = team_slot(arch, mode);
  if (dev < 0 || dev >= MAX_DEVICES) return 0;
  const int c = known[dev * ATTR_SLOTS + slot].load(std::memory_order_relaxed);
  if (c > 0) return c - 1;
  const int nb = team_blocks_query(arch, mode, dev);
  known[dev * ATTR_SLOTS + slot].store(nb + 1, std::memory_order_relaxed);
  return nb;
}

static TeamGeo team_geo(int arch, int mode, int64_t L, int dev) {
  TeamGeo g{};
  const bool p16 = mode == MODE_P16;
  g.halo = cb::TEAM_HALO;                  // halos refreshed from the neighbours at every CBAM
  g.T = (p16 ? cb::t16::WB16 : WB) - 2 * g.halo;
  g.TT = (int)((L + g.T - 1) / g.T);
  // the ping-pong team kernel spreads L evenly over its TT tiles (T = ceil(L / TT) own positions;
  // the rows beyond them up to the tile's end are its right halo): the last tile then holds few
  // rows outside [0, L) (9 instead of 54 at L = 10,000), whose zeroing after every conv made it
  // the slowest member of its team (+0.5-0.7 % against tiles that each own WB - 2 halo).
  if (p16) g.T = (int)((L + g.TT - 1) / g.TT);
  const int resident = device_cus(dev) * team_blocks_per_cu(arch, mode, dev);
  g.teams = resident > 0 ? resident / g.TT : 0;
  const char* env = getenv("RDN_CBAM_SEGMENTS");       // diagnostics: force the per-segment path
  if (env && env[0] == '1') g.teams = 0;
  if (g.teams > 0) {
    g.slots = (size_t)g.teams * 2 * g.TT * (p16 ? cb::t16::SLOT16_BYTES : cb::SLOT_BYTES);
    g.counters = (size_t)g.teams * cb::TEAM_CTR_STRIDE * 4;
    g.hsave = p16 ? 0 : (size_t)g.teams * g.TT * WB * 64 * 4;     // p16: the identity lives in VGPRs
    g.total = g.slots + g.counters + g.hsave + 256 + 4 * 256 + cb::STAMP_BYTES;
  }
  return g;
}

size_t cbam_workspace_bytes(int arch, int dtype, int64_t n, int64_t L, hipStream_t stream) {
  const TeamGeo g = team_geo(arch, team_mode(dtype), L, stream_device(stream));
  if (g.teams > 0) return g.total;
  const int64_t c = n < CBAM_CHUNK ? n : CBAM_CHUNK;
  return 256 + 4 * act_bytes(c, L) + 2 * (size_t)c * 64 * (sizeof(double) + sizeof(unsigned)) + 256;
}

// workspace carve-up of the team kernel: slots | counters | identity buffers | error word | stamps
static char* team_base(void* ws) { return (char*)(((uintptr_t)ws + 255) & ~(uintptr_t)255); }
static char* team_hsave(const TeamGeo& g, void* ws) {
  return team_base(ws) + ((g.slots + g.counters + 255) & ~(size_t)255);
}
static unsigned* team_err(const TeamGeo& g, void* ws) { return (unsigned*)(team_hsave(g, ws) + g.hsave); }

// One launch for the whole network (see cb::team_forward).
static hipError_t launch_team(int arch, int mode, const TeamGeo& g, const uint8_t* blob, const float* x, float* y,
                              int64_t n, int L, void* ws, hipStream_t stream) {
  using namespace cb;
  const hipError_t ea = ensure_dynamic_lds(team_fn(arch, mode), team_slot(arch, mode), team_lds(mode), stream_device(stream));
  if (ea != hipSuccess) return ea;
  char* base = team_base(ws);
  TeamArgs ta{};
  ta.TT = g.TT;
  ta.teams = g.teams;
  ta.T = g.T;
  ta.halo = g.halo;
  ta.n = n;
  ta.slots = base;
  ta.counters = (unsigned*)(base + g.slots);
  ta.hsave = team_hsave(g, ws);
  ta.err = team_err(g, ws);
  const char* miss = getenv("RDN_CBAM_FORCE_MISS");     // test knob: see TeamArgs::force_miss
  ta.force_miss = miss ? atoi(miss) : 0;
  const char* xcd = getenv("RDN_T16_XCD_OFF");          // A/B knob: every team hands off through sc1
  ta.xcd = xcd && xcd[0] == '1' ? 0 : 1;
  ta.stamps = cb::STAMP_BYTES ? (unsigned long long*)((char*)ws + g.total - cb::STAMP_BYTES) : nullptr;
  // counters and this launch's error word start at 0 (the hand-off counts arrivals monotonically);
  // the sticky word after it collects every launch's timeouts until cbam_status reads and clears it
  // the tagged hand-off starts from tag 0 in every slot granule, and each launch
  // takes tags from a range no earlier launch used (ta.tag0, below): no granule of an earlier launch
  // -- in memory or left in an XCD's L2 by plain stores -- carries a tag this launch
  // waits for.  MODE_P16 keeps no identity buffer, so slots | counters | padding | err[0] are one
  // contiguous range: one fill instead of three (the sticky words err[1..3] behind it stay); the batch-1
  // loop of evaulate.py pays every launch's fills
  hipError_t e;
  if (mode == MODE_P16 && g.hsave == 0 && (char*)ta.err >= base + g.slots + g.counters) {
    e = hipMemsetAsync(base, 0, (size_t)((char*)ta.err - base) + 4, stream);
  } else {
    e = hipMemsetAsync(ta.counters, 0, g.counters, stream);
    if (e == hipSuccess) e = hipMemsetAsync(ta.err, 0, 4, stream);
    if (e == hipSuccess && mode == MODE_P16) e = hipMemsetAsync(ta.slots, 0, g.slots, stream);
  }
  if (e != hipSuccess) return e;
  const int64_t teams = n < g.teams ? n : g.teams;    // never more teams than spectra
  ta.teams = (int)teams;
  {
    // CBAMs per team in this launch (ADSDN 17, APIDN 15 per spectrum); tags stay below bit 31
    // (cbam.hip TAG_OFF_XCD), and the range restarts from 0 when it would reach it
    static std::atomic<unsigned> next_tag{0};
    const unsigned span = (unsigned)(((n + teams - 1) / teams) * 17 + 2);
    unsigned t = next_tag.load(), base;
    do {
      base = t + span < 0x7fff0000u ? t : 0u;
    } while (!next_tag.compare_exchange_weak(t, base + span));
    ta.tag0 = base;
  }
  if (mode == MODE_P16) {
    const uint8_t* big16 = blob + pp16_section_offset_arch(arch);
    hipLaunchKernelGGL(team16_kernel(arch), dim3((unsigned)(teams * g.TT)), dim3(THREADS), (uint32_t)team_lds(mode),
                       stream, blob, big16, x, y, L, ta);
  } else {
    hipLaunchKernelGGL(team_kernel(arch, mode), dim3((unsigned)(teams * g.TT)), dim3(THREADS), SEG_LDS_BYTES, stream,
                       blob, x, y, L, ta);
  }
  return hipGetLastError();
}

typedef void (*seg_kernel_t)(const uint8_t*, const float*, float*, int, int, int, cb::Seg);

hipError_t launch_cbam_forward(int arch, int dtype, const uint8_t* blob, const float* x, float* y, int64_t n, int L,
                               void* ws, size_t ws_bytes, hipStream_t stream) {
  using namespace cb;
  const int mode = dtype_mode(dtype);
  const seg_kernel_t k = mode == ip::MODE_F32 ? segment<ip::MODE_F32>
                         : mode == ip::MODE_X3 ? segment<ip::MODE_X3>
                         : mode == ip::MODE_H8 ? segment<ip::MODE_H8>
                         : mode == ip::MODE_F16 ? segment<ip::MODE_F16> : segment<ip::MODE_B1>;
  const int dev = stream_device(stream);
  const hipError_t ea = ensure_dynamic_lds((const void*)k, 64 + mode, (int)SEG_LDS_BYTES, dev);
  if (ea != hipSuccess) return ea;
  const int tmode = team_mode(dtype);
  const TeamGeo tg = team_geo(arch, tmode, L, dev);
  if (tg.teams > 0) {
    if (ws_bytes < tg.total) return hipErrorInvalidValue;
    return launch_team(arch, tmode, tg, blob, x, y, n, L, ws, stream);
  }
  const bool adsdn = arch == ADSDN;
  const int64_t chunk = n < CBAM_CHUNK ? n : CBAM_CHUNK;
  if (ws_bytes < cbam_workspace_bytes(arch, dtype, chunk, L, stream)) return hipErrorInvalidValue;
  char* base = seg_base(ws) + 256;
  float* act[4];
  for (int i = 0; i < 4; ++i) act[i] = (float*)(base + i * act_bytes(chunk, L));
  double* sums[2];
  unsigned* maxs[2];
  char* st = base + 4 * act_bytes(chunk, L);
  for (int i = 0; i < 2; ++i) {
    sums[i] = (double*)(st + i * chunk * 64 * 8);
    maxs[i] = (unsigned*)(st + 2 * chunk * 64 * 8 + i * chunk * 64 * 4);
  }

  unsigned* range = seg_range(ws);
  for (int64_t n0 = 0; n0 < n; n0 += chunk) {
    const int64_t nn = n - n0 < chunk ? n - n0 : chunk;
    const float* xs = x + n0 * L;
    float* ys = y + n0 * L;
    // this chunk's range word starts clear (the sticky word behind it is cleared by cbam_status)
    if (mode == ip::MODE_H8) {
      const hipError_t er = hipMemsetAsync(range, 0, 4, stream);
      if (er != hipSuccess) return er;
    }
    // segment list (ADSDN/train.py:160-167, APIDN/train.py:150-159)
    std::vector<Seg> segs;
    auto mk = [&](int pro, int res, int store_h, int slot, int nconv, int e0, int e1, int layer0, int epi) {
      Seg s{};
      s.pro = pro; s.res = res; s.store_h = store_h; s.cbam_slot = slot; s.bias = adsdn;
      s.n_convs = nconv; s.epi0 = e0; s.epi1 = e1; s.layer0 = layer0; s.epi = epi;
      s.head_slot = 1; s.head_sigmoid = !adsdn; s.head_add_stem = !adsdn;
      s.range = range;
      s.halo = nconv + (epi == EPI_HEAD ? 1 : 0);
      return s;
    };
    if (adsdn) {
      segs.push_back(mk(PRO_STEM, RES_NONE, 0, 0, 0, 0, 0, 0, EPI_STORE));              // u0 = relu(stem x)
      segs.push_back(mk(PRO_CBAM, RES_NONE, 0, 2, 2, RELU, RELU, 0, EPI_STORE));        // cbam(u0); conv1, conv2
      segs.push_back(mk(PRO_CBAM, RES_NONE, 1, 5, 2, RELU, 0, 2, EPI_STORE));           // h = cbam(u1); block 0
      for (int b = 1; b < 15; ++b)
        segs.push_back(mk(PRO_CBAM, RES_ADD_RELU, 1, 8 + 3 * (b - 1), 2, RELU, 0, 2 + 2 * b, EPI_STORE));
      segs.push_back(mk(PRO_CBAM, RES_ADD_RELU, 0, 8 + 3 * 14, 0, 0, 0, 0, EPI_HEAD)); // h15; conv_out
    } else {
      segs.push_back(mk(PRO_STEM, RES_NONE, 1, 0, 2, RELU, 0, 0, EPI_STORE));           // h0 = relu(stem x); block 0
      for (int b = 1; b < 15; ++b)
        segs.push_back(mk(PRO_CBAM, RES_ADD, 1, 2 + 3 * (b - 1), 2, RELU, 0, 2 * b, EPI_STORE));
      segs.push_back(mk(PRO_CBAM, RES_ADD, 0, 2 + 3 * 14, 0, 0, 0, 0, EPI_HEAD));       // h15; sigmoid(conv_out(h15 + h0))
    }
    hipError_t e;
    // ping-pong: segment i writes u / h / stats into slot i&1 and reads slot (i&1)^1
    for (size_t i = 0; i < segs.size(); ++i) {
      Seg& s = segs[i];
      const int pi = (int)(i & 1), qi = pi ^ 1;
      s.u_in = act[qi];
      s.u_out = act[pi];
      s.h_in = act[2 + qi];
      s.h_out = act[2 + pi];
      s.sum_in = sums[qi];
      s.max_in = maxs[qi];
      s.sum_out = sums[pi];
      s.max_out = maxs[pi];
      // this segment's output stats were the previous-but-one segment's: clear them (stream order)
      e = hipMemsetAsync(sums[pi], 0, (size_t)chunk * 64 * 8, stream);
      if (e == hipSuccess) e = hipMemsetAsync(maxs[pi], 0, (size_t)chunk * 64 * 4, stream);
      if (e != hipSuccess) return e;
      const int T = WB - 2 * s.halo, tiles = (L + T - 1) / T;
      hipLaunchKernelGGL(k, dim3((unsigned)(nn * tiles)), dim3(THREADS), SEG_LDS_BYTES, stream, blob, xs, ys, L, T, tiles, s);
      e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
  }
  return hipSuccess;
}

// A new workspace: clear the sticky status words -- the team kernel's hand-off error, range and input-
// gate words (err[1..3]), or the segment path's range and gate words (the caller checked the size).
hipError_t cbam_workspace_init(int arch, int dtype, int64_t L, void* ws, size_t ws_bytes, hipStream_t stream) {
  const TeamGeo tg = team_geo(arch, team_mode(dtype), L, stream_device(stream));
  if (tg.teams <= 0) {
    if (!ws) return hipSuccess;
    return hipMemsetAsync(seg_range(ws), 0, 12, stream);
  }
  if (!ws || ws_bytes < tg.total) return hipErrorInvalidValue;
  return hipMemsetAsync(team_err(tg, ws) + 1, 0, 12, stream);         // the sticky words
}

// After CBAM forwards on `stream`: wait for them, then read and clear the sticky status words.
// *timed_out = 1 if a team wait of any forward since the last read exceeded its spin limit (outputs
// of affected spectra are NaN); *out_of_range = 1 if a MODE_H8 activation saturated; *gate = 1 if an
// input left [-INPUT_GATE, INPUT_GATE].  The caller checked the workspace size.
hipError_t cbam_status(int arch, int dtype, int64_t L, void* ws, size_t ws_bytes, hipStream_t stream,
                       int* timed_out, int* out_of_range, int* gate) {
  *timed_out = 0;
  *out_of_range = 0;
  *gate = 0;
  hipError_t e = hipSuccess;
  const TeamGeo tg = team_geo(arch, team_mode(dtype), L, stream_device(stream));
  unsigned* words;
  if (tg.teams <= 0) {
    if (!ws) return hipStreamSynchronize(stream);
    words = seg_range(ws);                                              // [1] range, [2] gate (sticky)
  } else {
    if (!ws || ws_bytes < tg.total) return hipErrorInvalidValue;
    words = team_err(tg, ws);                                           // [1] timeout, [2] range, [3] gate
  }
  // the words' copy is ordered behind the forwards on their stream; one wait covers both (the
  // batch-1 module path pays this per call)
  unsigned w[4] = {0, 0, 0, 0};
  e = read_words(w, words, sizeof(w), stream);
  if (e != hipSuccess) return e;
  if (tg.teams <= 0) {
    *out_of_range = w[1] != 0;
    *gate = w[2] != 0;
    if (w[1] || w[2]) e = hipMemsetAsync(words + 1, 0, 8, stream);     // on the forwards' stream (ordered)
  } else {
    *timed_out = w[1] != 0;
    *out_of_range = w[2] != 0;
    *gate = w[3] != 0;
    if (w[1] || w[2] || w[3]) e = hipMemsetAsync(words + 1, 0, 12, stream);
  }
  return e;
}

}  // namespace rdn
