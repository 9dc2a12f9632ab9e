// Whole-network fused kernels and host launcher of the single-rounding 16-bit modes (device
// building blocks: fused16.hpp).  Reference forwards: 1DCNN/train.py:71-82, RRCDNet/train.py:72-98,
// DSDN/train.py:72-126, PIDN/train.py:72-106.
#include "fused16.hpp"
#include "host_util.hpp"
#include "metrics.hpp"

namespace rdn {

#if !defined(H16_WALK_T)
namespace H16_NS {

// Network bodies; EDGE: the tile holds positions outside [0, L) (first/last tile of a spectrum),
// whose rows every epilogue re-zeroes.  Interior tiles skip that per-row select.
#define H16_BODY(name) template <bool EDGE> __device__ __forceinline__ void name##_body(Tile& tl, float* y, int n, int L, int T)

// The bodies alternate the two operand buffers F0 / F1: a layer computes from one while the next
// layer's operands stream into the other (fused16.hpp layer).

// 1DCNN/train.py:71-82 — conv(1->64)+ReLU, 18 x [conv+ReLU], conv(64->1)
H16_BODY(denoisecnn) {
  constexpr int H = fused_halo(DENOISECNN);
  Frags F0, F1;
  load_frags(tl, 0, F0);
  stem(tl, 0, BUF0);
  lds_barrier();
  for (int i = 0; i < 9; ++i) {
    layer<RELU, EDGE>(tl, BUF0, BUF1, 1, F0, F1);
    layer<RELU, EDGE>(tl, BUF1, BUF0, 1, F1, F0);
  }
  float o[HN];
  head<EDGE>(tl, BUF0, F0, F1, false, o);
  store_out(tl, y, n, o, H, T);
}

// RRCDNet/train.py:77-98 — right (BN, d=1) and left (dilated) branches, y = x - (r + l) / 2
H16_BODY(rrcdnet) {
  constexpr int H = fused_halo(RRCDNET);
  Frags F0, F1;
  load_frags(tl, 0, F0);
  // right_net: conv+BN+ReLU, 15 x [conv+BN+ReLU], conv(64->1)
  stem(tl, 0, BUF0);
  lds_barrier();
  for (int i = 0; i < 7; ++i) {
    layer<RELU, EDGE>(tl, BUF0, BUF1, 1, F0, F1);
    layer<RELU, EDGE>(tl, BUF1, BUF0, 1, F1, F0);
  }
  layer<RELU, EDGE>(tl, BUF0, BUF1, 1, F0, F1);
  {
    float r[HN];
    head<EDGE>(tl, BUF1, F1, F0, true, r);
    store_out(tl, y, n, r, H, T);   // parked in the output (re-read below): no VGPRs held across the left branch
  }
  // left_net: conv+BN+ReLU, 7 x [conv d2 + ReLU], conv+BN+ReLU, 6 x [conv d2 + ReLU], conv(64->1)
  stem(tl, 1, BUF0);             // the head above reads BUF1 only
  lds_barrier();
  for (int i = 0; i < 7; ++i) {
    layer<RELU, EDGE>(tl, BUF0, BUF1, 2, F0, F1);
    layer<RELU, EDGE>(tl, BUF1, BUF0, 2 * i + 1 == 7 ? 1 : 2, F1, F0);
  }
  float l[HN];
  head<EDGE>(tl, BUF0, F0, F1, false, l);
  // y = x - (right + left) / 2 on this tile's output rows (the lanes that stored r re-read it)
  if ((tid() & 63) < HEAD_LANES) {
#pragma unroll
    for (int k = 0; k < HN; ++k) {
      const int j = head_row(k);
      const int p = tl.base + j;
      if (j >= H && j < H + T && p < L) {
        float* yp = y + (size_t)n * L + p;
        *yp = tl.x[p] - (*yp + l[k]) / 2.0f;
      }
    }
  }
}

// DSDN/train.py:120-126 — relu(relu(stem)), relu(conv1), relu(conv2), 15 ResNet blocks, conv_out
H16_BODY(dsdn) {
  constexpr int H = fused_halo(DSDN);
  Frags F0, F1;
  load_frags(tl, 0, F0);
  stem(tl, 0, BUF0);
  lds_barrier();
  layer<RELU, EDGE>(tl, BUF0, BUF1, 1, F0, F1);           // conv1
  layer<RELU, EDGE>(tl, BUF1, BUF0, 1, F1, F0);           // conv2
  for (int b = 0; b < 15; ++b) {               // x in BUF0 is the block identity
    layer<RELU, EDGE>(tl, BUF0, BUF1, 1, F0, F1);         // relu(bn1(conv1 x))
    layer<RES_RELU, EDGE>(tl, BUF1, BUF0, 1, F1, F0);     // relu(bn2(conv2 .) + x), written over x in place
  }
  float o[HN];
  head<EDGE>(tl, BUF0, F0, F1, false, o);
  store_out(tl, y, n, o, H, T);
}

// PIDN/train.py:101-106 — h = relu(stem x); 15 x [conv+BN+ReLU, conv+BN]; sigmoid(conv_out(y + h))
H16_BODY(pidn) {
  constexpr int H = fused_halo(PIDN);
  Frags F0, F1;
  load_frags(tl, 0, F0);
  stem(tl, 0, BUF0);
  lds_barrier();
  for (int b = 0; b < 15; ++b) {
    layer<RELU, EDGE>(tl, BUF0, BUF1, 1, F0, F1);
    layer<LINEAR, EDGE>(tl, BUF1, BUF0, 1, F1, F0);
  }
  stem<true>(tl, 0, BUF0);       // + identity (the stem output), recomputed in fp32 from x
  lds_barrier();
  float o[HN];
  head<EDGE>(tl, BUF0, F0, F1, false, o);
#pragma unroll
  for (int k = 0; k < HN; ++k) o[k] = 1.0f / (1.0f + expf(-o[k]));
  store_out(tl, y, n, o, H, T);
}

#define H16_KERNEL(name, arch)                                                                            \
  __global__ __launch_bounds__(THREADS) void name(const uint8_t* __restrict__ blob, const float* __restrict__ x, \
                                                  float* __restrict__ y, int L, int T, int tiles,          \
                                                  unsigned* __restrict__ status) {                         \
    extern __shared__ __attribute__((aligned(16))) char lds[];                                             \
    int n;                                                                                                 \
    Tile tl = make_tile(lds, blob, x, L, T, tiles, fused_halo(arch), n);                                   \
    tl.status = status;                                                                                    \
    if (tl.base >= 0 && tl.base + WB <= L) name##_body<false>(tl, y, n, L, T);                             \
    else name##_body<true>(tl, y, n, L, T);                                                                \
  }

H16_KERNEL(denoisecnn, DENOISECNN)
H16_KERNEL(rrcdnet, RRCDNET)
H16_KERNEL(dsdn, DSDN)
H16_KERNEL(pidn, PIDN)

}  // namespace H16_NS

typedef void (*fused_kernel_t)(const uint8_t*, const float*, float*, int, int, int, unsigned*);

// Host launcher: one workgroup per (spectrum, tile); tiles along L overlap by 2*halo.
// status: the workspace's status word (the input gate, STATUS_GATE) or NULL
hipError_t H16_LAUNCH(int arch, const uint8_t* blob, const float* x, float* y, int64_t n, int L, unsigned* status,
                      hipStream_t stream) {
  fused_kernel_t k = nullptr;
  switch (arch) {
    case DENOISECNN: k = H16_NS::denoisecnn; break;
    case RRCDNET: k = H16_NS::rrcdnet; break;
    case DSDN: k = H16_NS::dsdn; break;
    case PIDN: k = H16_NS::pidn; break;
    default: return hipErrorInvalidValue;
  }
  // attribute slots 0-7 (bf16) / 56-63 (f16), host_util.hpp
  const hipError_t e = ensure_dynamic_lds((const void*)k, H16_ATTR_SLOT0 + arch, (int)H16_NS::LDS_BYTES, stream_device(stream));
  if (e != hipSuccess) return e;
  const int H = fused_halo(arch), T = H16_NS::WB - 2 * H, tiles = (L + T - 1) / T;
  const int64_t chunk = (int64_t)(0x7fffffff / tiles);
  for (int64_t n0 = 0; n0 < n; n0 += chunk) {
    const int64_t nn = n - n0 < chunk ? n - n0 : chunk;
    hipLaunchKernelGGL(k, dim3((unsigned)(nn * tiles)), dim3(H16_NS::THREADS), H16_NS::LDS_BYTES, stream, blob,
                       x + n0 * L, y + n0 * L, L, T, tiles, status);
  }
  return hipGetLastError();
}

#else  // H16_WALK_T

namespace H16_NS {

// Walk bodies (fused16.hpp "Walk instantiation"): one workgroup per spectrum walks its tiles left to
// right.  A tile's stem writes rows [0, WB) at positions base + row (base = t WT - CG - c0: the stem
// of a branch whose stack is shallower starts c0 positions further left, so both heads of RRCDNet end
// at the same positions); every layer then shifts by its dilation (layer() / head()), and tl.dnext
// names the dilation of the layer that reads it (the carry rows it needs).  The last head of a tile
// prefetches the next tile's layer 0 into the other operand buffer (copied after the next stem) and
// the next stem's x (StemX) is fetched before it.

// 1DCNN/train.py:71-82 — conv(1->64)+ReLU, 18 x [conv+ReLU], conv(64->1); head at shift 19
constexpr int DENOISECNN_SHIFT = walk_shift(DENOISECNN);
static_assert(DENOISECNN_SHIFT == 18 + 1, "18 layers and the head, d = 1");
template <bool EDGE>
__device__ __forceinline__ void denoisecnn_tile(Tile& tl, float* y, int t, int ntiles, Frags& F0, Frags& F1, StemX& xs) {
  walk_start(tl, t, 0);
  stem(tl, 0, BUF0, xs);
  F0 = F1;                            // layer 0's operands, prefetched by the last head (or the kernel)
  lds_barrier();
  for (int i = 0; i < 9; ++i) {
    layer<RELU, EDGE>(tl, BUF0, BUF1, 1, F0, F1);
    layer<RELU, EDGE>(tl, BUF1, BUF0, 1, F1, F0);
  }
  // the next tile's stem inputs and layer-0 operands, fetched unconditionally (past the last tile:
  // harmless reads), so neither xs nor F1 stays live across a tile for the loop's last iteration
  xs = walk_stem_load(tl, t + 1, 0);
  float o[HN];
  head<EDGE>(tl, BUF0, F0, F1, true, o, 0);
  store_out_walk(tl, y, o);
  lds_barrier();                      // the next tile's stem overwrites BUF0
}

// RRCDNet/train.py:77-98 — right (BN, d = 1) and left (dilated) branches, y = x - (r + l) / 2: both
// heads at shift 28 (right: stem shifted by 12, 15 layers, head; left: 7 x (2, 2|1) = 27, head)
constexpr int RRCDNET_SHIFT = walk_shift(RRCDNET), RRCDNET_RIGHT_C0 = RRCDNET_SHIFT - 16;
static_assert(RRCDNET_SHIFT == 13 * 2 + 1 + 1, "left: 13 layers d = 2, one d = 1, the head");
template <bool EDGE>
__device__ __forceinline__ void rrcdnet_tile(Tile& tl, float* y, int t, int ntiles, Frags& F0, Frags& F1, StemX& xs) {
  walk_start(tl, t, RRCDNET_RIGHT_C0);
  stem(tl, 0, BUF0, xs);
  F0 = F1;                            // layer 0's operands, prefetched by the last head (or the kernel)
  lds_barrier();
  for (int i = 0; i < 7; ++i) {
    layer<RELU, EDGE>(tl, BUF0, BUF1, 1, F0, F1);
    layer<RELU, EDGE>(tl, BUF1, BUF0, 1, F1, F0);
  }
  layer<RELU, EDGE>(tl, BUF0, BUF1, 1, F0, F1);
  const StemX xl = walk_stem_load(tl, t, 0);
  float r[HN];
  head<EDGE>(tl, BUF1, F1, F0, true, r);
  // left_net: conv+BN+ReLU, 7 x [conv d2 + ReLU], conv+BN+ReLU, 6 x [conv d2 + ReLU], conv(64->1)
  tl.base = t * WT - CG;
  tl.dn_prev = 0;                     // the stem recomputes its carry rows
  stem(tl, 1, BUF0, xl);             // the head above reads BUF1 only
  lds_barrier();
  for (int i = 0; i < 7; ++i) {
    // left layer j has d = 1 at j = 7, else 2; the head reads the last with d = 1
    tl.dnext = 2 * i + 1 == 7 ? 1 : 2;
    layer<RELU, EDGE>(tl, BUF0, BUF1, 2, F0, F1);
    tl.dnext = i == 6 ? 1 : 2;
    layer<RELU, EDGE>(tl, BUF1, BUF0, 2 * i + 1 == 7 ? 1 : 2, F1, F0);
  }
  tl.dnext = 1;
  float xv[HN];
#pragma unroll
  for (int k = 0; k < HN; ++k) {      // the combine's x, fetched before the left head
    const int p = tl.base - 1 + head_row(k);
    xv[k] = head_row(k) < WB && in_range(p, tl.L) ? tl.x[p] : 0.f;
  }
  xs = walk_stem_load(tl, t + 1, RRCDNET_RIGHT_C0);
  float l[HN];
  head<EDGE>(tl, BUF0, F0, F1, true, l, 0);
#pragma unroll
  for (int k = 0; k < HN; ++k) l[k] = xv[k] - (r[k] + l[k]) / 2.0f;
  store_out_walk(tl, y, l);
  lds_barrier();
}

// PIDN/train.py:101-106 — h = relu(stem x); 15 x [conv+BN+ReLU, conv+BN]; sigmoid(conv_out(y + h)):
// head at shift 31.  The identity h is recomputed from x at the last layer's shift (stem<true>), on the
// computed rows only: the carry rows in front already hold the previous tile's y + h (layer_carry
// saved them after its stem<true>)
constexpr int PIDN_SHIFT = walk_shift(PIDN);
static_assert(PIDN_SHIFT == 30 + 1, "30 layers and the head, d = 1");
template <bool EDGE>
__device__ __forceinline__ void pidn_tile(Tile& tl, float* y, int t, int ntiles, Frags& F0, Frags& F1, StemX& xs) {
  walk_start(tl, t, 0);
  stem(tl, 0, BUF0, xs);
  F0 = F1;
  lds_barrier();
  for (int b = 0; b < 15; ++b) {
    layer<RELU, EDGE>(tl, BUF0, BUF1, 1, F0, F1);
    layer<LINEAR, EDGE>(tl, BUF1, BUF0, 1, F1, F0);
  }
  stem<true>(tl, 0, BUF0);            // + identity, at this shift (stem_load reads x at tl.base)
  lds_barrier();
  xs = walk_stem_load(tl, t + 1, 0);
  float o[HN];
  head<EDGE>(tl, BUF0, F0, F1, true, o, 0);
#pragma unroll
  for (int k = 0; k < HN; ++k) o[k] = 1.0f / (1.0f + expf(-o[k]));
  store_out_walk(tl, y, o);
  lds_barrier();
}

// DSDN/train.py:120-126 — relu(relu(stem)), relu(conv1), relu(conv2), 15 ResNet blocks, conv_out:
// head at shift 33.  Each block's second conv adds the block input two rows up (fused16.hpp layer,
// walk RES_RELU); the block's first conv hands it the identity of its first N-tile (walk_id).
constexpr int DSDN_SHIFT = walk_shift(DSDN);
static_assert(DSDN_SHIFT == 32 + 1, "32 layers and the head, d = 1");
template <bool EDGE>
__device__ __forceinline__ void dsdn_tile(Tile& tl, float* y, int t, int ntiles, Frags& F0, Frags& F1, StemX& xs) {
  walk_start(tl, t, 0);
  stem(tl, 0, BUF0, xs);
  F0 = F1;
  lds_barrier();
  layer<RELU, EDGE>(tl, BUF0, BUF1, 1, F0, F1);           // conv1
  layer<RELU, EDGE>(tl, BUF1, BUF0, 1, F1, F0);           // conv2
  for (int b = 0; b < 15; ++b) {                           // x in BUF0 is the block identity
    V id0;
    layer<RELU, EDGE>(tl, BUF0, BUF1, 1, F0, F1, true, nullptr, nullptr, (NoStage*)nullptr, &id0);
    layer<RES_RELU, EDGE>(tl, BUF1, BUF0, 1, F1, F0, true, nullptr, nullptr, (NoStage*)nullptr, &id0);
  }
  xs = walk_stem_load(tl, t + 1, 0);
  float o[HN];
  head<EDGE>(tl, BUF0, F0, F1, true, o, 0);
  store_out_walk(tl, y, o);
  lds_barrier();
}

#define H16_WALK_KERNEL(name, SHIFT, C0)                                                                   \
  __global__ __launch_bounds__(THREADS) void name##_walk(const uint8_t* __restrict__ blob,                 \
                                                         const float* __restrict__ x, float* __restrict__ y, \
                                                         int L, int ntiles, unsigned* __restrict__ status, \
                                                         met::MetricOut mo) {                               \
    extern __shared__ __attribute__((aligned(16))) char lds[];                                             \
    wave_priority();                                                                                       \
    const int n = __builtin_amdgcn_workgroup_id_x();                                                       \
    Tile tl = init_tile(lds, blob, blob + SMALL_BYTES, x + (size_t)n * L, L, 0);                           \
    tl.status = status;                                                                                    \
    y += (size_t)n * L;                                                                                    \
    Frags F0, F1;                                                                                          \
    load_frags(tl, 0, F1);                                                                                 \
    StemX xs = walk_stem_load(tl, 0, C0);                                                                  \
    for (int t = 0; t < ntiles; ++t) {                                                                     \
      if (t == 0 || (t + 1) * WT > L) name##_tile<true>(tl, y, t, ntiles, F0, F1, xs);                    \
      else name##_tile<false>(tl, y, t, ntiles, F0, F1, xs);                                               \
      tl.first = false;                                                                                    \
    }                                                                                                      \
    if (mo.clean) met::walk_metrics(y, L, n, lds, mo);  /* the metric epilogue: y read back from L2 */    \
  }

H16_WALK_KERNEL(denoisecnn, DENOISECNN_SHIFT, 0)
H16_WALK_KERNEL(rrcdnet, RRCDNET_SHIFT, RRCDNET_RIGHT_C0)
H16_WALK_KERNEL(pidn, PIDN_SHIFT, 0)
H16_WALK_KERNEL(dsdn, DSDN_SHIFT, 0)

}  // namespace H16_NS

typedef void (*walk_kernel_t)(const uint8_t*, const float*, float*, int, int, unsigned*, met::MetricOut);

// Host launcher: one workgroup per spectrum (the grid should hold many spectra per CU: a spectrum is
// one CU's sequential walk); ntiles = ceil((L + head shift) / WT).  mo (may be NULL): the metric
// epilogue's outputs (metrics.hpp walk_metrics), computed by each spectrum's workgroup after its walk.
hipError_t H16_LAUNCH(int arch, const uint8_t* blob, const float* x, float* y, int64_t n, int L, unsigned* status,
                      const met::MetricOut* mo, hipStream_t stream) {
  walk_kernel_t k = nullptr;
  int shift = 0;
  switch (arch) {
    case DENOISECNN: k = H16_NS::denoisecnn_walk; shift = H16_NS::DENOISECNN_SHIFT; break;
    case RRCDNET: k = H16_NS::rrcdnet_walk; shift = H16_NS::RRCDNET_SHIFT; break;
    case PIDN: k = H16_NS::pidn_walk; shift = H16_NS::PIDN_SHIFT; break;
    case DSDN: k = H16_NS::dsdn_walk; shift = H16_NS::DSDN_SHIFT; break;
    default: return hipErrorInvalidValue;
  }
  const hipError_t e = ensure_dynamic_lds((const void*)k, H16_ATTR_SLOT0 + arch, (int)H16_NS::LDS_BYTES, stream_device(stream));
  if (e != hipSuccess) return e;
  const int ntiles = (int)(((int64_t)L + shift + H16_NS::WT - 1) / H16_NS::WT);
  for (int64_t n0 = 0; n0 < n; n0 += 0x7fffffff) {
    const int64_t nn = n - n0 < 0x7fffffff ? n - n0 : 0x7fffffff;
    hipLaunchKernelGGL(k, dim3((unsigned)nn), dim3(H16_NS::THREADS), H16_NS::LDS_BYTES, stream, blob, x + n0 * L,
                       y + n0 * L, L, ntiles, status, met::chunk(mo, n0, L));
  }
  return hipGetLastError();
}

#endif  // H16_WALK_T

}  // namespace rdn
