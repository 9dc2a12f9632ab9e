// Whole-network fused tile kernels for the f16 + e4m3-correction mode (RDN_F16F8) of 1DCNN,
// RRCDNet and PIDN: four waves per workgroup, one per SIMD, each holding ALL 64 output channels.
//
// Arithmetic per Conv1d(64,64,3,d) (inplace.hpp Op<MODE_H8>): per tap, two f16 MFMAs (K = 64) for
// W_hi.X_hi plus one block-scaled e4m3 MFMA (K = 128) for W_lo.X_hi + W_hi.X_lo.  That is 64 MFMA
// cycles per (tap, 16x16 tile) against 96 for split bf16, but it reads the same 64 B of activation
// per lane per tap, so with the split-bf16 geometry (8 waves, 2 M-tiles each) the LDS traffic per
// MFMA cycle rises 1.5x and the kernel stops being MFMA-bound (tools/ablate.py, PMC: 39 % MFMA busy).
// Here each wave computes 4 M-tiles from every B fragment it reads: half the LDS reads and stores
// per MFMA cycle.  The price is registers: the layer's A operands for 4 M-tiles (192 VGPRs), so one
// wave per SIMD with the 512-register budget (VGPR + AGPR).
//
// Geometry.  One workgroup = one tile of WB = 640 positions (the CU's whole 160 KiB LDS as one
// in-place buffer of 256-byte rows: [f16 hi | e4m3 hi | e4m3 lo * 2^11], h16_channel order), no
// guard rows (a tap that leaves the tile wraps; see inplace.hpp TileGeo).  A layer runs as NB = 5
// blocks of 128 rows; wave w owns rows 128j + 32w + [0, 32) of block j (2 N-tiles) x 64 couts.
// Write-back lags two blocks (block j-2 is stored while block j computes, one (N-tile, M-tile
// pair) piece per k-step: a 16-B f16 slot + two 8-B e4m3 slots), one LDS barrier per block.
//
// Reference forwards: 1DCNN/train.py:71-82, RRCDNet/train.py:72-98, PIDN/train.py:72-106.
#include "inplace.hpp"

namespace rdn {
namespace h8 {

using ip::Tile;
using O = ip::Op<ip::MODE_H8>;
using ip::f16x4;
using ip::f16x8;

constexpr int WAVES = 4;
constexpr int THREADS = 64 * WAVES;
constexpr int WB = 640, NB = 5, BR = 128;       // rows per tile, blocks per layer, rows per block
constexpr int NT = 2, MT = 4;                   // N-tiles (16 rows) per wave per block, M-tiles (16 couts)
constexpr int RPT = (WB + THREADS - 1) / THREADS;   // stem / head rows per thread
constexpr uint32_t LDS_BYTES = WB * ROWB_F32;   // 163840
static_assert(BR == WAVES * NT * 16, "block = waves x N-tiles x 16 rows");

__device__ __forceinline__ int wrap(int r) { return r < 0 ? r + WB : (r >= WB ? r - WB : r); }
__device__ __forceinline__ bool in_range(int p, int L) { return (unsigned)p < (unsigned)L; }
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

struct Frags {                 // one layer's operands: A fragments [M-tile][tap], bias, E8M0 scales
  O::A a[MT][3];
  f32x4 bias[MT];
  uint32_t sc[MT];
};

__device__ __forceinline__ void load_frags_tap(const Tile& tl, int layer, int t, Frags& F) {
  const uint8_t* wl = tl.big + (size_t)layer * BIG_BYTES_H8;
  const int lane = ip::opaque_tid() & 63;
#pragma unroll
  for (int m = 0; m < MT; ++m) F.a[m][t] = O::load_a(wl, m, t, lane);
}
__device__ __forceinline__ void load_frags_misc(const Tile& tl, int layer, Frags& F) {
  const uint8_t* wl = tl.big + (size_t)layer * BIG_BYTES_H8;
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    F.bias[m] = ip::load_bias<ip::MODE_H8>(wl, m);
    F.sc[m] = ip::load_scale<ip::MODE_H8>(wl, m);
  }
}
__device__ __forceinline__ void load_frags(const Tile& tl, int layer, Frags& F) {
  load_frags_misc(tl, layer, F);
#pragma unroll
  for (int t = 0; t < 3; ++t) load_frags_tap(tl, layer, t, F);
}

// Conv1d(1, 64, 3, padding=1) (+ folded BN) + ReLU in fp32, one row per thread per pass;
// ACCUM adds the result onto the resident row (PIDN/train.py:105: identity recomputed from x).
template <bool ACCUM = false>
__device__ __forceinline__ void tile_stem(const Tile& tl, int slot) {
  const cfloat* sw = ip::small_slot(tl, slot);
  for (int j = ip::opaque_tid(); j < WB; j += THREADS) {
    const int p = tl.base + j;
    const float xm = in_range(p - 1, tl.L) ? tl.x[p - 1] : 0.f;
    const float x0 = in_range(p, tl.L) ? tl.x[p] : 0.f;
    const float xp = in_range(p + 1, tl.L) ? tl.x[p + 1] : 0.f;
    const bool valid = in_range(p, tl.L);
#pragma unroll
    for (int cb = 0; cb < 16; ++cb) {
      f32x4 v = ACCUM ? O::load4(tl.lds, j, 4 * cb) : f32x4{0.f, 0.f, 0.f, 0.f};
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
      O::store4(tl.lds, j, 4 * cb, v);
    }
  }
}

// Conv1d(64, 1, 3, padding=1) in fp32, row j = tid + THREADS k in out[k]
__device__ __forceinline__ void tile_head(const Tile& tl, int slot, float (&out)[RPT]) {
  const cfloat* hw = ip::small_slot(tl, slot);
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int j = ip::opaque_tid() + THREADS * k;
    out[k] = 0.f;
    if (j >= WB) continue;
    float a = hw[192];
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const int r = wrap(j + t - 1);
#pragma unroll 4
      for (int cb = 0; cb < 16; ++cb) {
        const f32x4 v = O::load4(tl.lds, r, 4 * cb);
#pragma unroll
        for (int i = 0; i < 4; ++i) a = fmaf(hw[3 * (cb * 4 + i) + t], v[i], a);
      }
    }
    out[k] = a;
  }
}

__device__ __forceinline__ void tile_store_out(const Tile& tl, float* y, int n, const float (&v)[RPT], int halo, int T) {
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int j = ip::opaque_tid() + THREADS * k;
    const int p = tl.base + j;
    if (j < WB && j >= halo && j < halo + T && p < tl.L) y[(size_t)n * tl.L + p] = v[k];
  }
}

// One Conv1d(64, 64, 3, dilation=dil, padding=dil) + folded BN (+ ReLU) in place over the tile.
// Block j reads rows down to 128j - d (the tail of block j-1), so block j-1's outputs may only be
// written once every wave has finished block j: after the barrier that ends block j.  They are
// written during block j+1 (lag 2 in block index from the block that produced them).
template <bool RELU, bool EDGE>
__device__ __forceinline__ void conv(Tile& tl, int dil, Frags& F, bool has_next) {
  const int tid = ip::opaque_tid();
  const int lane = tid & 63, w = tid >> 6, q = lane >> 4, c16 = lane & 15;
  const int next = tl.layer + 1;
  f32x4 bias_l[MT];
  uint32_t sc_l[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) bias_l[m] = F.bias[m], sc_l[m] = F.sc[m];

  // this lane's rows: 128 j + 32 w + 16 i + c16.  B addresses per (tap, plane) for j = i = 0;
  // blocks and N-tiles add multiples of 16 rows (swizzle unchanged -> immediate offsets).
  const int r0 = 32 * w + c16;
  uint32_t badr[3][O::PLANES];
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const int r = r0 + (t - 1) * dil;               // < 0 only for wave 0, tap 0: block 0 uses bfirst
#pragma unroll
    for (int p = 0; p < O::PLANES; ++p) badr[t][p] = r * ROWB_F32 + ((O::bslot(t, q, p) ^ swz256(r)) << 4);
  }
  // the only taps that can leave the tile: tap 0 of (block 0, N-tile 0) and tap 2 of (block NB-1,
  // N-tile NT-1); wrapped absolute addresses (equal to the plain ones for waves that stay inside)
  uint32_t bfirst[O::PLANES], blast[O::PLANES];
  {
    const int rf = wrap(r0 - dil), rl = wrap(r0 + BR * (NB - 1) + 16 * (NT - 1) + dil);
#pragma unroll
    for (int p = 0; p < O::PLANES; ++p) {
      bfirst[p] = rf * ROWB_F32 + ((O::bslot(0, q, p) ^ swz256(rf)) << 4);
      blast[p] = rl * ROWB_F32 + ((O::bslot(2, q, p) ^ swz256(rl)) << 4);
    }
  }
  auto read_b = [&](int j, int t, int i) -> O::B {
    if (j == 0 && t == 0 && i == 0) return O::load_b_at(tl.lds, bfirst, 0);
    if (j == NB - 1 && t == 2 && i == NT - 1) return O::load_b_at(tl.lds, blast, 0);
    return O::load_b_at(tl.lds, badr[t], (uint32_t)(BR * j + 16 * i) * ROWB_F32);
  };
  // store addresses of M-tile pair u (channels 32u + ...: f16 slot 4u+q, e4m3 slots 4u+q)
  uint32_t sadr[2][3];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int slot = 4 * u + q;
    const int b[3] = {16 * slot, 128 + 8 * slot, 192 + 8 * slot};
#pragma unroll
    for (int p = 0; p < 3; ++p) sadr[u][p] = r0 * ROWB_F32 + ((((b[p] >> 4) ^ swz256(r0)) << 4) | (b[p] & 15));
  }

  f32x4 res[NB][NT][MT];
  // write-back of N-tile i, M-tile pair u of block j: ReLU, zero padding, split, 3 stores
  auto store_piece = [&](int j, int i, int u) {
    const int row = BR * j + 32 * w + 16 * i + c16;
    f32x4 v0 = ip::h8_sat<RELU>(res[j][i][2 * u]), v1 = ip::h8_sat<RELU>(res[j][i][2 * u + 1]);
    if (EDGE && !in_range(tl.base + row, tl.L)) v0 = v1 = f32x4{0.f, 0.f, 0.f, 0.f};
    const ip::H8Split x0 = ip::h8_split(v0), x1 = ip::h8_split(v1);
    const uint32_t off = (uint32_t)(BR * j + 16 * i) * ROWB_F32;
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    *(f16x8*)(tl.lds + sadr[u][0] + off) = __builtin_shufflevector(x0.hi, x1.hi, 0, 1, 2, 3, 4, 5, 6, 7);
    *(u32x2*)(tl.lds + sadr[u][1] + off) = u32x2{x0.hi8, x1.hi8};
    *(u32x2*)(tl.lds + sadr[u][2] + off) = u32x2{x0.lo8, x1.lo8};
  };

  O::B bnext[NT];
#pragma unroll
  for (int i = 0; i < NT; ++i) bnext[i] = read_b(0, 0, i);
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    f32x4 part[NT][MT];
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int m = 0; m < MT; ++m) part[i][m] = bias_l[m];
    if (j == NB - 1 && has_next) load_frags_misc(tl, next, F);        // bias / scales copied above
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      O::B bcur[NT];
#pragma unroll
      for (int i = 0; i < NT; ++i) bcur[i] = bnext[i];
      if (t + 1 < 3) {
#pragma unroll
        for (int i = 0; i < NT; ++i) bnext[i] = read_b(j, t + 1, i);
      }
#pragma unroll
      for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int m = 0; m < MT; ++m) part[i][m] = O::mma(F.a[m][t], bcur[i], part[i][m], sc_l[m], t);
      if (j == NB - 1 && has_next) load_frags_tap(tl, next, t, F);    // last use of tap t's fragments
      // lagged write-back of block j-2: pieces (i, u) = (0,0) | (0,1) | (1,0) (1,1) over the 3 taps
      if (j >= 2) {
        if (t == 0) store_piece(j - 2, 0, 0);
        if (t == 1) store_piece(j - 2, 0, 1);
        if (t == 2) { store_piece(j - 2, 1, 0); store_piece(j - 2, 1, 1); }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int m = 0; m < MT; ++m) res[j][i][m] = part[i][m];
    if (j + 1 < NB) {
#pragma unroll
      for (int i = 0; i < NT; ++i) bnext[i] = read_b(j + 1, 0, i);
    }
    lds_barrier();                 // every wave is done reading the rows of block j (and j-1's tail)
  }
#pragma unroll
  for (int j = NB - 2; j < NB; ++j)
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int u = 0; u < 2; ++u) store_piece(j, i, u);
  lds_barrier();
  tl.layer += 1;
}

#define H8_BODY(name) template <bool EDGE> __device__ __forceinline__ void name##_body(Tile& tl, float* y, int n, int L, int T)

// 1DCNN/train.py:71-82 — conv(1->64)+ReLU, 18 x [conv+ReLU], conv(64->1)
H8_BODY(denoisecnn) {
  constexpr int H = fused_halo(DENOISECNN);
  Frags F;
  load_frags(tl, 0, F);
  tile_stem(tl, 0);
  __syncthreads();
  for (int i = 0; i < 18; ++i) conv<true, EDGE>(tl, 1, F, i + 1 < 18);
  float o[RPT];
  tile_head(tl, 1, o);
  tile_store_out(tl, y, n, o, H, T);
}

// RRCDNet/train.py:77-98 — right (BN, d=1) and left (dilated) branches, y = x - (r + l) / 2
H8_BODY(rrcdnet) {
  constexpr int H = fused_halo(RRCDNET);
  Frags F;
  load_frags(tl, 0, F);
  tile_stem(tl, 0);
  __syncthreads();
  for (int i = 0; i < 15; ++i) conv<true, EDGE>(tl, 1, F, true);
  float r[RPT];
  tile_head(tl, 2, r);
  __syncthreads();               // the left stem overwrites the rows the right head just read
  tile_stem(tl, 1);
  __syncthreads();
  for (int i = 0; i < 14; ++i) conv<true, EDGE>(tl, i == 7 ? 1 : 2, F, i + 1 < 14);
  float l[RPT];
  tile_head(tl, 3, l);
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int p = tl.base + ip::opaque_tid() + THREADS * k;
    const float xv = in_range(p, L) ? tl.x[p] : 0.f;
    r[k] = xv - (r[k] + l[k]) / 2.0f;
  }
  tile_store_out(tl, y, n, r, H, T);
}

// PIDN/train.py:101-106 — h = relu(stem x); 15 x [conv+BN+ReLU, conv+BN]; sigmoid(conv_out(y + h))
H8_BODY(pidn) {
  constexpr int H = fused_halo(PIDN);
  Frags F;
  load_frags(tl, 0, F);
  tile_stem(tl, 0);
  __syncthreads();
  for (int b = 0; b < 15; ++b) {
    conv<true, EDGE>(tl, 1, F, true);
    conv<false, EDGE>(tl, 1, F, b < 14);
  }
  tile_stem<true>(tl, 0);             // + identity (the stem output), recomputed from x
  __syncthreads();
  float o[RPT];
  tile_head(tl, 1, o);
#pragma unroll
  for (int k = 0; k < RPT; ++k) o[k] = 1.0f / (1.0f + expf(-o[k]));
  tile_store_out(tl, y, n, o, H, T);
}

#define H8_KERNEL(name, arch)                                                                             \
  __global__ __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu(1, 1)))                      \
  void name(const uint8_t* __restrict__ blob, const float* __restrict__ x, float* __restrict__ y, int L, int T, \
            int tiles) {                                                                                  \
    extern __shared__ __attribute__((aligned(16))) char lds[];                                            \
    int n;                                                                                                \
    Tile tl = ip::make_tile(lds, blob, x, L, T, tiles, fused_halo(arch), n);                              \
    if (tl.base >= 0 && tl.base + WB <= L) name##_body<false>(tl, y, n, L, T);                            \
    else name##_body<true>(tl, y, n, L, T);                                                               \
  }

H8_KERNEL(denoisecnn, DENOISECNN)
H8_KERNEL(rrcdnet, RRCDNET)
H8_KERNEL(pidn, PIDN)

}  // namespace h8

typedef void (*fused_kernel_t)(const uint8_t*, const float*, float*, int, int, int);

// true if (arch) has a 4-wave f16f8 kernel; DSDN (its ResidualBlock identity needs registers this
// geometry does not have) runs the 8-wave in-place kernel (fused_inplace.hip)
// (RDN_H8_GENERIC=1: diagnostic builds, tools/ablate.py — every network on the 8-wave kernel)
#ifndef RDN_H8_GENERIC
#define RDN_H8_GENERIC 0
#endif
bool has_fused_h8(int arch) { return !RDN_H8_GENERIC && (arch == DENOISECNN || arch == RRCDNET || arch == PIDN); }

hipError_t launch_fused_h8(int arch, const uint8_t* blob, const float* x, float* y, int64_t n, int L,
                           hipStream_t stream) {
  fused_kernel_t k = nullptr;
  switch (arch) {
    case DENOISECNN: k = h8::denoisecnn; break;
    case RRCDNET: k = h8::rrcdnet; break;
    case PIDN: k = h8::pidn; break;
    default: return hipErrorInvalidValue;
  }
  static bool attr_set[8] = {};
  if (!attr_set[arch]) {
    const hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h8::LDS_BYTES);
    if (e != hipSuccess) return e;
    attr_set[arch] = true;
  }
  const int H = fused_halo(arch), T = h8::WB - 2 * H, tiles = (L + T - 1) / T;
  const int64_t chunk = (int64_t)(0x7fffffff / tiles);
  for (int64_t n0 = 0; n0 < n; n0 += chunk) {
    const int64_t nn = n - n0 < chunk ? n - n0 : chunk;
    hipLaunchKernelGGL(k, dim3((unsigned)(nn * tiles)), dim3(h8::THREADS), h8::LDS_BYTES, stream, blob,
                       x + n0 * L, y + n0 * L, L, T, tiles);
  }
  return hipGetLastError();
}

}  // namespace rdn
