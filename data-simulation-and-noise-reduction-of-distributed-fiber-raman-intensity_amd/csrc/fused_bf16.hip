// Fused conv-stack tile kernels, bf16 MFMA path (v_mfma_f32_16x16x32_bf16, fp32 accumulate).
//
// One 512-thread workgroup = one tile of WB = 512 positions of one spectrum.  LDS holds two
// ping-pong activation buffers (516 rows x 64 ch bf16, 2 guard rows per side) and one 24.8 KB
// weight slot.  Each Conv1d(64,64,3,d) is an implicit GEMM
//     Y[64 cout][512 pos] = W[64][192 = 3 taps x 64 cin] . X~[192][512]
// whose B operand is read straight from the activation buffer at row offsets (t-1)*d: no im2col.
// Wave w owns rows [64w, 64w+64) = 4 N-tiles of 16 positions and all 64 output channels
// (4 M-tiles); its 24 A-fragments (the layer's weights) are read from the slot while it works
// on N-tile 0 and stay in VGPRs for N-tiles 1..3, after which the slot is refilled with the next
// layer's weights by LDS-DMA (global_load_lds_dwordx4) under the remaining 3 N-tiles.
// BatchNorm is folded into W and bias on the host; bias + ReLU (+ residual) run in the epilogue,
// which also re-zeroes rows outside [0, L) — the zero padding every reference Conv1d applies.
//
// Reference forwards reproduced here: 1DCNN/train.py:71-82, RRCDNet/train.py:72-98,
// DSDN/train.py:72-126, PIDN/train.py:72-106.
#include "common.hpp"

namespace rdn {
namespace bf {

constexpr uint32_t ACT0 = 0;
constexpr uint32_t ACT1 = ACT_BYTES_BF16;
constexpr uint32_t WSLOT = 2 * ACT_BYTES_BF16;                  // 132096
constexpr uint32_t LDS_BYTES = WSLOT + BIG_BYTES_BF16;          // 156928
constexpr int BIG_CHUNKS = BIG_BYTES_BF16 / 16;                 // 1552

enum Epi : int {
  EPI_RELU = 0,        // relu(acc + b)
  EPI_LINEAR = 1,      // acc + b               (PIDN block output: BN without ReLU)
  EPI_RES_RELU = 2,    // relu(acc + b + dst)   (DSDN ResidualBlock: out += identity; relu)
};

struct Tile {
  char* lds;
  const float* x;        // this spectrum's input
  int L;
  int base;              // global position of logical row 0
  const uint8_t* big;    // big-layer section of the blob
  int n_big;
  int layer;             // index of the big layer whose weights sit in WSLOT
  const float* small;    // small section
};

__device__ __forceinline__ bool in_range(int p, int L) { return p >= 0 && p < L; }

// LDS-DMA the packed weights of big layer `idx` into the weight slot (16 B per lane, 1 KiB per
// wave-instruction; wave w issues instructions w, w+8, w+16, w+24).
__device__ __forceinline__ void issue_weight_dma(const Tile& tl, int idx) {
  if (idx >= tl.n_big) return;
  const uint8_t* src = tl.big + (size_t)idx * BIG_BYTES_BF16;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int k0 = 0; k0 < 32; k0 += WAVES) {
    const int k = k0 + w;
    const int chunk = k * 64 + lane;
    if (k * 64 < BIG_CHUNKS && chunk < BIG_CHUNKS) {
      __builtin_amdgcn_global_load_lds((const void*)(src + (size_t)chunk * 16),
                                       (lds_ptr_t)(tl.lds + WSLOT + k * 1024), 16, 0, 0);
    }
  }
}

__device__ __forceinline__ void zero_guards(char* lds) {
  // 4 guard rows x 128 B per buffer = 512 B; 2 buffers -> 64 lanes x 16 B
  const int t = threadIdx.x;
  if (t < 64) {
    const int buf = t >> 5, r = (t >> 3) & 3, slot = t & 7;
    const int prow = r < 2 ? r : ROWS - 4 + r;
    *(f32x4*)(lds + (buf ? ACT1 : ACT0) + prow * ROWB_BF16 + slot * 16) = f32x4{0.f, 0.f, 0.f, 0.f};
  }
}

// stem: Conv1d(1, 64, 3, padding=1) (+ folded BN) + ReLU, one row per thread, fp32 math.
// ACCUM: add the stem output to the row already in dst instead of overwriting it
// (PIDN/train.py:105 ``x + identity`` with the identity recomputed from x).
template <bool ACCUM = false>
__device__ __forceinline__ void stem(const Tile& tl, int slot, uint32_t dst) {
  const float* swp = tl.small + slot * SMALL_SLOT_FLOATS;
  asm volatile("" : "+s"(swp));   // no reuse of scalar-loaded weights across the 30 layers in between
  const cfloat* sw = (const cfloat*)swp;
  const int j = threadIdx.x;
  const int p = tl.base + j;
  const float xm = in_range(p - 1, tl.L) ? tl.x[p - 1] : 0.f;
  const float x0 = in_range(p, tl.L) ? tl.x[p] : 0.f;
  const float xp = in_range(p + 1, tl.L) ? tl.x[p + 1] : 0.f;
  const bool valid = in_range(p, tl.L);
#pragma unroll
  for (int cb = 0; cb < 8; ++cb) {
    bf16x8* slotp = (bf16x8*)(tl.lds + dst + off_bf16(j + GUARD, cb * 16));
    bf16x8 v;
    if (ACCUM) v = *slotp;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int c = cb * 8 + i;
      float a = sw[192 + c];
      a = fmaf(sw[3 * c + 0], xm, a);
      a = fmaf(sw[3 * c + 1], x0, a);
      a = fmaf(sw[3 * c + 2], xp, a);
      a = fmaxf(a, 0.f);
      if (ACCUM) a += (float)v[i];
      v[i] = (__bf16)(valid ? a : 0.f);
    }
    *slotp = v;
  }
}

// One Conv1d(64, 64, 3, dilation=dil, padding=dil) over the whole tile, src -> dst.
template <int EPI>
__device__ __forceinline__ void conv(Tile& tl, uint32_t src, uint32_t dst, int dil) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int q = lane >> 4, c16 = lane & 15;
  const char* wslot = tl.lds + WSLOT;
  bf16x8 A[4][6];
  f32x4 bias[4];
  const int r0 = tl.base + w * 64;                  // this wave's 64 rows straddle no spectrum end?
  const bool wave_inside = r0 >= 0 && r0 + 64 <= tl.L;

#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const int row = w * 64 + n * 16 + c16;          // logical row this lane's accumulators map to
    f32x4 acc[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 6; ++s) {
      const int t = s >> 1, u = s & 1;
      if (n == 0) {
#pragma unroll
        for (int m = 0; m < 4; ++m) A[m][s] = *(const bf16x8*)(wslot + ((m * 6 + s) * 64 + lane) * 16);
      }
      const int prow = GUARD + w * 64 + n * 16 + c16 + (t - 1) * dil;
      const bf16x8 B = *(const bf16x8*)(tl.lds + src + off_bf16(prow, 64 * u + 16 * q));
#pragma unroll
      for (int m = 0; m < 4; ++m) acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[m][s], B, acc[m], 0, 0, 0);
    }
    if (n == 0) {
#pragma unroll
      for (int m = 0; m < 4; ++m)
        bias[m] = *(const f32x4*)(wslot + BIG_FRAG_BYTES_BF16 + (16 * m + 4 * q) * 4);
    }
    // ---- epilogue for this N-tile: bias (+ identity), ReLU, zero rows outside [0, L) ----
    const bool valid = wave_inside || in_range(tl.base + row, tl.L);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const uint32_t o = dst + off_bf16(row + GUARD, 32 * m + 8 * q);
      f32x4 v = acc[m] + bias[m];
      if (EPI == EPI_RES_RELU) v += __builtin_convertvector(*(const bf16x4*)(tl.lds + o), f32x4);
      if (EPI == EPI_RELU || EPI == EPI_RES_RELU) v = __builtin_elementwise_max(v, f32x4{0.f, 0.f, 0.f, 0.f});
      if (!valid) v = f32x4{0.f, 0.f, 0.f, 0.f};
      *(bf16x4*)(tl.lds + o) = __builtin_convertvector(v, bf16x4);
    }
    if (n == 0) {
      // every wave now holds this layer's A-fragments and bias in VGPRs: refill the slot
      __syncthreads();
      issue_weight_dma(tl, tl.layer + 1);
    }
  }
  tl.layer += 1;
  __syncthreads();      // dst complete; s_waitcnt vmcnt(0) before it lands the next weights
}

// head: Conv1d(64, 1, 3, padding=1) as the same implicit GEMM with only M-row 0 populated
// (packed as a big layer whose other 63 output rows are zero).  Lanes with q == 0 return the
// output of position row w*64 + 16n + (lane & 15) in out[n].
__device__ __forceinline__ void head(Tile& tl, uint32_t src, float (&out)[4]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int q = lane >> 4, c16 = lane & 15;
  const char* wslot = tl.lds + WSLOT;
  bf16x8 A[6];
  float b0 = 0.f;
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 6; ++s) {
      const int t = s >> 1, u = s & 1;
      if (n == 0) A[s] = *(const bf16x8*)(wslot + (s * 64 + lane) * 16);
      const int prow = GUARD + w * 64 + n * 16 + c16 + (t - 1);
      const bf16x8 B = *(const bf16x8*)(tl.lds + src + off_bf16(prow, 64 * u + 16 * q));
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[s], B, acc, 0, 0, 0);
    }
    if (n == 0) b0 = *(const float*)(wslot + BIG_FRAG_BYTES_BF16);
    out[n] = acc[0] + b0;
    if (n == 0) {
      __syncthreads();
      issue_weight_dma(tl, tl.layer + 1);
    }
  }
  tl.layer += 1;
}

__device__ __forceinline__ Tile make_tile(char* lds, const uint8_t* blob, const float* x, int L, int T,
                                          int tiles, int halo, int n_big, int& n_out, int& t_out) {
  const int n = blockIdx.x / tiles, tile = blockIdx.x - n * tiles;
  n_out = n;
  t_out = tile;
  Tile tl;
  tl.lds = lds;
  tl.x = x + (size_t)n * L;
  tl.L = L;
  tl.base = tile * T - halo;
  tl.small = (const float*)blob;
  tl.big = blob + SMALL_BYTES;
  tl.n_big = n_big;
  tl.layer = 0;
  return tl;
}

// position row of out[k] for this lane (meaningful in lanes with (lane >> 4) == 0)
__device__ __forceinline__ int head_row(int k) { return (threadIdx.x >> 6) * 64 + k * 16 + (threadIdx.x & 15); }

__device__ __forceinline__ void store_out(const Tile& tl, float* y, int n, const float (&v)[4], int halo, int T) {
  if ((threadIdx.x & 63) >= 16) return;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int j = head_row(k);
    const int p = tl.base + j;
    if (j >= halo && j < halo + T && p < tl.L) y[(size_t)n * tl.L + p] = v[k];
  }
}

}  // namespace bf

using namespace bf;

// 1DCNN/train.py:71-82 — conv(1->64)+ReLU, 18 x [conv+ReLU], conv(64->1)
__global__ __launch_bounds__(THREADS) void denoisecnn_bf16(const uint8_t* __restrict__ blob,
                                                         const float* __restrict__ x, float* __restrict__ y,
                                                         int L, int T, int tiles) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  constexpr int H = fused_halo(DENOISECNN);
  int n, tile;
  Tile tl = make_tile(lds, blob, x, L, T, tiles, H, 19, n, tile);
  zero_guards(lds);
  issue_weight_dma(tl, 0);
  stem(tl, 0, ACT0);
  __syncthreads();
  uint32_t cur = ACT0, nxt = ACT1;
  for (int i = 0; i < 18; ++i) {
    conv<EPI_RELU>(tl, cur, nxt, 1);
    const uint32_t t = cur; cur = nxt; nxt = t;
  }
  float o[4];
  head(tl, cur, o);
  store_out(tl, y, n, o, H, T);
}

// RRCDNet/train.py:77-98 — right (BN, d=1) and left (dilated) branches, y = x - (r + l) / 2
__global__ __launch_bounds__(THREADS) void rrcdnet_bf16(const uint8_t* __restrict__ blob,
                                                      const float* __restrict__ x, float* __restrict__ y,
                                                      int L, int T, int tiles) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  constexpr int H = fused_halo(RRCDNET);
  int n, tile;
  Tile tl = make_tile(lds, blob, x, L, T, tiles, H, 31, n, tile);
  zero_guards(lds);
  issue_weight_dma(tl, 0);
  // right_net: conv+BN+ReLU, 15 x [conv+BN+ReLU], conv(64->1)
  stem(tl, 0, ACT0);
  __syncthreads();
  uint32_t cur = ACT0, nxt = ACT1;
  for (int i = 0; i < 15; ++i) {
    conv<EPI_RELU>(tl, cur, nxt, 1);
    const uint32_t t = cur; cur = nxt; nxt = t;
  }
  float r[4];
  head(tl, cur, r);
  // left_net: conv+BN+ReLU, 7 x [conv d2 + ReLU], conv+BN+ReLU, 6 x [conv d2 + ReLU], conv(64->1)
  stem(tl, 1, nxt);            // the head above reads `cur` only
  __syncthreads();
  cur = nxt; nxt = cur == ACT0 ? ACT1 : ACT0;
  for (int i = 0; i < 14; ++i) {
    conv<EPI_RELU>(tl, cur, nxt, i == 7 ? 1 : 2);
    const uint32_t t = cur; cur = nxt; nxt = t;
  }
  float l[4];
  head(tl, cur, l);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int p = tl.base + head_row(k);
    const float xv = in_range(p, L) ? tl.x[p] : 0.f;
    r[k] = xv - (r[k] + l[k]) / 2.0f;
  }
  store_out(tl, y, n, r, H, T);
}

// DSDN/train.py:120-126 — relu(relu(stem)), relu(conv1), relu(conv2), 15 ResNet blocks, conv_out
__global__ __launch_bounds__(THREADS) void dsdn_bf16(const uint8_t* __restrict__ blob,
                                                   const float* __restrict__ x, float* __restrict__ y,
                                                   int L, int T, int tiles) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  constexpr int H = fused_halo(DSDN);
  int n, tile;
  Tile tl = make_tile(lds, blob, x, L, T, tiles, H, 33, n, tile);
  zero_guards(lds);
  issue_weight_dma(tl, 0);
  stem(tl, 0, ACT0);
  __syncthreads();
  conv<EPI_RELU>(tl, ACT0, ACT1, 1);        // conv1
  conv<EPI_RELU>(tl, ACT1, ACT0, 1);        // conv2
  for (int b = 0; b < 15; ++b) {            // x in ACT0 is the block identity
    conv<EPI_RELU>(tl, ACT0, ACT1, 1);      // relu(bn1(conv1 x))
    conv<EPI_RES_RELU>(tl, ACT1, ACT0, 1);  // relu(bn2(conv2 .) + x), written over x in place
  }
  float o[4];
  head(tl, ACT0, o);
  store_out(tl, y, n, o, H, T);
}

// PIDN/train.py:101-106 — h = relu(stem x); 15 x [conv+BN+ReLU, conv+BN]; sigmoid(conv_out(y + h))
__global__ __launch_bounds__(THREADS) void pidn_bf16(const uint8_t* __restrict__ blob,
                                                   const float* __restrict__ x, float* __restrict__ y,
                                                   int L, int T, int tiles) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  constexpr int H = fused_halo(PIDN);
  int n, tile;
  Tile tl = make_tile(lds, blob, x, L, T, tiles, H, 31, n, tile);
  zero_guards(lds);
  issue_weight_dma(tl, 0);
  stem(tl, 0, ACT0);
  __syncthreads();
  for (int b = 0; b < 15; ++b) {
    conv<EPI_RELU>(tl, ACT0, ACT1, 1);
    conv<EPI_LINEAR>(tl, ACT1, ACT0, 1);
  }
  stem<true>(tl, 0, ACT0);      // + identity (the stem output), recomputed in fp32 from x
  __syncthreads();
  float o[4];
  head(tl, ACT0, o);
#pragma unroll
  for (int k = 0; k < 4; ++k) o[k] = 1.0f / (1.0f + expf(-o[k]));
  store_out(tl, y, n, o, H, T);
}

}  // namespace rdn

namespace rdn {

typedef void (*fused_kernel_t)(const uint8_t*, const float*, float*, int, int, int);

// Host launcher: one workgroup per (spectrum, tile); tiles along L overlap by 2*halo.
hipError_t launch_fused_bf16(int arch, const uint8_t* blob, const float* x, float* y, int64_t n, int L,
                             hipStream_t stream) {
  fused_kernel_t k = nullptr;
  switch (arch) {
    case DENOISECNN: k = denoisecnn_bf16; break;
    case RRCDNET: k = rrcdnet_bf16; break;
    case DSDN: k = dsdn_bf16; break;
    case PIDN: k = pidn_bf16; break;
    default: return hipErrorInvalidValue;
  }
  static bool attr_set[8] = {};
  if (!attr_set[arch]) {
    const hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bf::LDS_BYTES);
    if (e != hipSuccess) return e;
    attr_set[arch] = true;
  }
  const int H = fused_halo(arch), T = WB - 2 * H, tiles = (L + T - 1) / T;
  const int64_t chunk = (int64_t)(0x7fffffff / tiles);
  for (int64_t n0 = 0; n0 < n; n0 += chunk) {
    const int64_t nn = n - n0 < chunk ? n - n0 : chunk;
    hipLaunchKernelGGL(k, dim3((unsigned)(nn * tiles)), dim3(THREADS), bf::LDS_BYTES, stream, blob,
                       x + n0 * L, y + n0 * L, L, T, tiles);
  }
  return hipGetLastError();
}

}  // namespace rdn
