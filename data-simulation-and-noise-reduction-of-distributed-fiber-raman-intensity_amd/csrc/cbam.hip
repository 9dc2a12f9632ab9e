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
#include <vector>

#include "inplace.hpp"

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
};

__device__ __forceinline__ unsigned f2ord(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(unsigned o) {
  return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}
__device__ __forceinline__ float sigm(float v) { return 1.0f / (1.0f + expf(-v)); }

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
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
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
    Op<MODE>::store4(lds, r + GUARD, 4 * sub, h);
  }
}

// h = relu(stem(x)) for the first segment; also stored to HBM when it is a residual (APIDN)
template <int MODE>
__device__ void prologue_stem(Tile& tl, const Seg& sg, int n) {
  stem<MODE>(tl, 0);
  __syncthreads();
  if (!sg.store_h) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, sub = lane & 15, rgrp = lane >> 4;
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
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, sub = lane & 15, rgrp = lane >> 4;
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
  if (threadIdx.x < 64) {
    const int c = threadIdx.x;
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
  using G = Geo<MODE, true>;
  int n;
  Tile tl = make_tile(lds, blob, x, L, T, tiles, sg.halo, n);
  tl.layer = sg.layer0;
  f32x4 id[16];
  LayerA<MODE> a;
  if (sg.n_convs) load_layer_a<MODE>(tl, sg.layer0, a);
  zero_guards(lds);
  if (sg.pro == PRO_STEM) prologue_stem<MODE>(tl, sg, n);
  else prologue_cbam<MODE>(tl, sg, n);
  __syncthreads();
  for (int i = 0; i < sg.n_convs; ++i) {
    const bool more = i + 1 < sg.n_convs;
    if ((i ? sg.epi1 : sg.epi0) & RELU) conv<MODE, RELU, G::S>(tl, 1, id, a, more);
    else conv<MODE, 0, G::S>(tl, 1, id, a, more);
  }
  if (sg.epi == EPI_STORE) {
    epilogue_store<MODE>(tl, sg, n);
    return;
  }
  if (sg.head_add_stem) {
    stem<MODE, true>(tl, 0);
    __syncthreads();
  }
  float v[HEAD_ROWS];
  head<MODE>(tl, sg.head_slot, v);
  if (sg.head_sigmoid) {
#pragma unroll
    for (int k = 0; k < HEAD_ROWS; ++k) v[k] = sigm(v[k]);
  }
  store_out(tl, y, n, v, sg.halo, T);
}

}  // namespace cb

// ---- host ----------------------------------------------------------------------------------------

static constexpr int64_t CBAM_CHUNK = 1024;       // spectra per pass (bounds the workspace)

static size_t act_bytes(int64_t n, int64_t L) { return (size_t)n * L * 64 * sizeof(float); }

size_t cbam_workspace_bytes(int, int, int64_t n, int64_t L) {
  const int64_t c = n < CBAM_CHUNK ? n : CBAM_CHUNK;
  return 4 * act_bytes(c, L) + 2 * (size_t)c * 64 * (sizeof(double) + sizeof(unsigned)) + 256;
}

typedef void (*seg_kernel_t)(const uint8_t*, const float*, float*, int, int, int, cb::Seg);

hipError_t launch_cbam_forward(int arch, int dtype, const uint8_t* blob, const float* x, float* y, int64_t n, int L,
                               void* ws, size_t ws_bytes, hipStream_t stream) {
  using namespace cb;
  const int mode = dtype == F32 ? ip::MODE_F32 : dtype == BF16X3 ? ip::MODE_X3 : ip::MODE_B1;
  const seg_kernel_t k = mode == ip::MODE_F32 ? segment<ip::MODE_F32>
                         : mode == ip::MODE_X3 ? segment<ip::MODE_X3> : segment<ip::MODE_B1>;
  static bool attr_set[3] = {};
  const int mi = mode == ip::MODE_F32 ? 0 : mode == ip::MODE_X3 ? 1 : 2;
  if (!attr_set[mi]) {
    const hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)SEG_LDS_BYTES);
    if (e != hipSuccess) return e;
    attr_set[mi] = true;
  }
  const bool adsdn = arch == ADSDN;
  const int64_t chunk = n < CBAM_CHUNK ? n : CBAM_CHUNK;
  if (ws_bytes < cbam_workspace_bytes(arch, dtype, chunk, L)) return hipErrorInvalidValue;
  char* base = (char*)(((uintptr_t)ws + 255) & ~(uintptr_t)255);
  float* act[4];
  for (int i = 0; i < 4; ++i) act[i] = (float*)(base + i * act_bytes(chunk, L));
  double* sums[2];
  unsigned* maxs[2];
  char* st = base + 4 * act_bytes(chunk, L);
  for (int i = 0; i < 2; ++i) {
    sums[i] = (double*)(st + i * chunk * 64 * 8);
    maxs[i] = (unsigned*)(st + 2 * chunk * 64 * 8 + i * chunk * 64 * 4);
  }

  for (int64_t n0 = 0; n0 < n; n0 += chunk) {
    const int64_t nn = n - n0 < chunk ? n - n0 : chunk;
    const float* xs = x + n0 * L;
    float* ys = y + n0 * L;
    // segment list (ADSDN/train.py:160-167, APIDN/train.py:150-159)
    std::vector<Seg> segs;
    auto mk = [&](int pro, int res, int store_h, int slot, int nconv, int e0, int e1, int layer0, int epi) {
      Seg s{};
      s.pro = pro; s.res = res; s.store_h = store_h; s.cbam_slot = slot; s.bias = adsdn;
      s.n_convs = nconv; s.epi0 = e0; s.epi1 = e1; s.layer0 = layer0; s.epi = epi;
      s.head_slot = 1; s.head_sigmoid = !adsdn; s.head_add_stem = !adsdn;
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

}  // namespace rdn
