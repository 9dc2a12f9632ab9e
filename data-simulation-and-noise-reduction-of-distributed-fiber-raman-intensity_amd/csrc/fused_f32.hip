// Fused conv-stack tile kernels, exact-fp32 MFMA path (v_mfma_f32_16x16x4_f32).
//
// Same tiling as the bf16 path (fused_bf16.hip): one 512-thread workgroup owns WB = 512 positions
// of one spectrum and keeps the 64-channel activations in LDS for the whole network.  fp32 rows
// are 256 B, so a single 132 KB buffer is updated IN PLACE: every wave accumulates its whole
// share of the layer (16 N-tiles x one 16-channel M-tile = 64 accumulator VGPRs), the workgroup
// synchronises, and only then are the outputs written back.  At 1/16 of the bf16 MFMA rate the
// layer is ~50k cycles long, so the serialised write-back (~1.5k cycles) is a few percent.
// Wave w = (m = w & 3, nh = w >> 2) computes output channels [16m, 16m+16) for rows
// [256 nh, 256 nh + 256); its 48 A-operands (the layer's weights for those channels) are loaded
// from L2 into VGPRs once per layer.  ResNet identities (DSDN) stay in VGPRs of the lane that
// wrote them, so no second buffer is needed.
//
// Reference forwards reproduced here: 1DCNN/train.py:71-82, RRCDNet/train.py:72-98,
// DSDN/train.py:72-126, PIDN/train.py:72-106.
#include "common.hpp"

namespace rdn {
namespace f32k {

constexpr uint32_t ACT = 0;
constexpr uint32_t LDS_BYTES = ACT_BYTES_F32;                    // 132096
constexpr int BIG_FLOATS = BIG_BYTES_F32 / 4;                    // 12352

enum Epi : int { RELU = 1, ADD_ID = 2, SAVE_ID = 4 };

struct Tile {
  char* lds;
  const float* x;
  int L;
  int base;
  const float* big;
  int layer;
  const float* small;
};

__device__ __forceinline__ bool in_range(int p, int L) { return p >= 0 && p < L; }

__device__ __forceinline__ void zero_guards(char* lds) {
  // 4 guard rows x 256 B = 1 KiB -> 64 lanes x 16 B
  const int t = threadIdx.x;
  if (t < 64) {
    const int r = t >> 4, slot = t & 15;
    const int prow = r < 2 ? r : ROWS - 4 + r;
    *(f32x4*)(lds + ACT + prow * ROWB_F32 + slot * 16) = f32x4{0.f, 0.f, 0.f, 0.f};
  }
}

__device__ __forceinline__ const cfloat* small_slot(const Tile& tl, int slot) {
  const float* p = tl.small + slot * SMALL_SLOT_FLOATS;
  asm volatile("" : "+s"(p));     // keep scalar-loaded weights from living across layers
  return (const cfloat*)p;
}

// Conv1d(1, 64, 3, padding=1) (+ folded BN) + ReLU; ACCUM adds it onto the resident row.
template <bool ACCUM = false>
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
    f32x4* slotp = (f32x4*)(tl.lds + ACT + off_f32(j + GUARD, cb * 16));
    f32x4 v;
    if (ACCUM) v = *slotp;
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
    *slotp = v;
  }
}

// Conv1d(64, 1, 3, padding=1), one row per thread.
__device__ __forceinline__ float head(const Tile& tl, int slot) {
  const cfloat* hw = small_slot(tl, slot);
  const int j = threadIdx.x;
  float a = hw[192];
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const int prow = j + GUARD + t - 1;
#pragma unroll 4
    for (int cb = 0; cb < 16; ++cb) {
      const f32x4 v = *(const f32x4*)(tl.lds + ACT + off_f32(prow, cb * 16));
#pragma unroll
      for (int i = 0; i < 4; ++i) a = fmaf(hw[3 * (cb * 4 + i) + t], v[i], a);
    }
  }
  return a;
}

template <int EPI>
__device__ __forceinline__ void conv(Tile& tl, int dil, f32x4 (&id)[16]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int m = w & 3, nh = w >> 2;
  const int q = lane >> 4, c16 = lane & 15;
  const float* wl = tl.big + (size_t)tl.layer * BIG_FLOATS;
  const f32x4 bias = *(const f32x4*)(wl + BIG_FRAG_FLOATS_F32 + 16 * m + 4 * q);

  f32x4 acc[16];
#pragma unroll
  for (int n = 0; n < 16; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int tg = 0; tg < 12; ++tg) {
    const int t = tg >> 2, g = tg & 3;
    const f32x4 W = ((const f32x4*)wl)[(m * 12 + tg) * 64 + lane];
#pragma unroll
    for (int n = 0; n < 16; ++n) {
      const int prow = GUARD + nh * 256 + n * 16 + c16 + (t - 1) * dil;
      const f32x4 B = *(const f32x4*)(tl.lds + ACT + off_f32(prow, 64 * g + 16 * q));
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(W[i], B[i], acc[n], 0, 0, 0);
    }
  }
  __syncthreads();                 // every read of the layer input is done: overwrite in place
#pragma unroll
  for (int n = 0; n < 16; ++n) {
    const int row = nh * 256 + n * 16 + c16;
    const bool valid = in_range(tl.base + row, tl.L);
    f32x4 v = acc[n] + bias;
    if (EPI & ADD_ID) v += id[n];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float a = v[r];
      if (EPI & RELU) a = fmaxf(a, 0.f);
      v[r] = valid ? a : 0.f;
    }
    if (EPI & SAVE_ID) id[n] = v;
    *(f32x4*)(tl.lds + ACT + off_f32(row + GUARD, 64 * m + 16 * q)) = v;
  }
  __syncthreads();
  tl.layer += 1;
}

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
  tl.big = (const float*)(blob + SMALL_BYTES);
  tl.layer = 0;
  return tl;
}

__device__ __forceinline__ void store_out(const Tile& tl, float* y, int n, float v, int halo, int T) {
  const int j = threadIdx.x;
  const int p = tl.base + j;
  if (j >= halo && j < halo + T && p < tl.L) y[(size_t)n * tl.L + p] = v;
}

}  // namespace f32k

using namespace f32k;

__global__ __launch_bounds__(THREADS) void denoisecnn_f32(const uint8_t* __restrict__ blob,
                                                        const float* __restrict__ x, float* __restrict__ y,
                                                        int L, int T, int tiles) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  constexpr int H = fused_halo(DENOISECNN);
  int n;
  Tile tl = make_tile(lds, blob, x, L, T, tiles, H, n);
  f32x4 id[16];
  zero_guards(lds);
  stem(tl, 0);
  __syncthreads();
  for (int i = 0; i < 18; ++i) conv<RELU>(tl, 1, id);
  store_out(tl, y, n, head(tl, 1), H, T);
}

__global__ __launch_bounds__(THREADS) void rrcdnet_f32(const uint8_t* __restrict__ blob,
                                                     const float* __restrict__ x, float* __restrict__ y,
                                                     int L, int T, int tiles) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  constexpr int H = fused_halo(RRCDNET);
  int n;
  Tile tl = make_tile(lds, blob, x, L, T, tiles, H, n);
  f32x4 id[16];
  zero_guards(lds);
  stem(tl, 0);
  __syncthreads();
  for (int i = 0; i < 15; ++i) conv<RELU>(tl, 1, id);
  const float r = head(tl, 2);
  __syncthreads();               // the left stem overwrites the buffer the right head just read
  stem(tl, 1);
  __syncthreads();
  for (int i = 0; i < 14; ++i) conv<RELU>(tl, i == 7 ? 1 : 2, id);
  const float l = head(tl, 3);
  const int p = tl.base + (int)threadIdx.x;
  const float xv = in_range(p, L) ? tl.x[p] : 0.f;
  store_out(tl, y, n, xv - (r + l) / 2.0f, H, T);
}

__global__ __launch_bounds__(THREADS) void dsdn_f32(const uint8_t* __restrict__ blob,
                                                  const float* __restrict__ x, float* __restrict__ y,
                                                  int L, int T, int tiles) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  constexpr int H = fused_halo(DSDN);
  int n;
  Tile tl = make_tile(lds, blob, x, L, T, tiles, H, n);
  f32x4 id[16];
  zero_guards(lds);
  stem(tl, 0);
  __syncthreads();
  conv<RELU>(tl, 1, id);                       // conv1
  conv<RELU | SAVE_ID>(tl, 1, id);             // conv2 -> first block identity
  for (int b = 0; b < 15; ++b) {
    conv<RELU>(tl, 1, id);                     // relu(bn1(conv1 x))
    conv<RELU | ADD_ID | SAVE_ID>(tl, 1, id);  // relu(bn2(conv2 .) + x)
  }
  store_out(tl, y, n, head(tl, 1), H, T);
}

__global__ __launch_bounds__(THREADS) void pidn_f32(const uint8_t* __restrict__ blob,
                                                  const float* __restrict__ x, float* __restrict__ y,
                                                  int L, int T, int tiles) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  constexpr int H = fused_halo(PIDN);
  int n;
  Tile tl = make_tile(lds, blob, x, L, T, tiles, H, n);
  f32x4 id[16];
  zero_guards(lds);
  stem(tl, 0);
  __syncthreads();
  for (int b = 0; b < 15; ++b) {
    conv<RELU>(tl, 1, id);
    conv<0>(tl, 1, id);
  }
  stem<true>(tl, 0);             // + identity (the stem output), recomputed from x
  __syncthreads();
  const float v = head(tl, 1);
  store_out(tl, y, n, 1.0f / (1.0f + expf(-v)), H, T);
}

}  // namespace rdn

namespace rdn {

typedef void (*fused_kernel_t)(const uint8_t*, const float*, float*, int, int, int);

hipError_t launch_fused_f32(int arch, const uint8_t* blob, const float* x, float* y, int64_t n, int L,
                            hipStream_t stream) {
  fused_kernel_t k = nullptr;
  switch (arch) {
    case DENOISECNN: k = denoisecnn_f32; break;
    case RRCDNET: k = rrcdnet_f32; break;
    case DSDN: k = dsdn_f32; break;
    case PIDN: k = pidn_f32; break;
    default: return hipErrorInvalidValue;
  }
  static bool attr_set[8] = {};
  if (!attr_set[arch]) {
    const hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)f32k::LDS_BYTES);
    if (e != hipSuccess) return e;
    attr_set[arch] = true;
  }
  const int H = fused_halo(arch), T = WB - 2 * H, tiles = (L + T - 1) / T;
  const int64_t chunk = (int64_t)(0x7fffffff / tiles);
  for (int64_t n0 = 0; n0 < n; n0 += chunk) {
    const int64_t nn = n - n0 < chunk ? n - n0 : chunk;
    hipLaunchKernelGGL(k, dim3((unsigned)(nn * tiles)), dim3(THREADS), f32k::LDS_BYTES, stream, blob,
                       x + n0 * L, y + n0 * L, L, T, tiles);
  }
  return hipGetLastError();
}

}  // namespace rdn
