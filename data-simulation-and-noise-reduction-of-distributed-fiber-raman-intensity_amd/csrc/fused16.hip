// Whole-network fused kernels and host launcher of the single-rounding 16-bit modes (device
// building blocks: fused16.hpp).  Reference forwards: 1DCNN/train.py:71-82, RRCDNet/train.py:72-98,
// DSDN/train.py:72-126, PIDN/train.py:72-106.
#include "fused16.hpp"
#include "host_util.hpp"

namespace rdn {
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
                                                  float* __restrict__ y, int L, int T, int tiles) {        \
    extern __shared__ __attribute__((aligned(16))) char lds[];                                             \
    int n;                                                                                                 \
    Tile tl = make_tile(lds, blob, x, L, T, tiles, fused_halo(arch), n);                                   \
    if (tl.base >= 0 && tl.base + WB <= L) name##_body<false>(tl, y, n, L, T);                             \
    else name##_body<true>(tl, y, n, L, T);                                                                \
  }

H16_KERNEL(denoisecnn, DENOISECNN)
H16_KERNEL(rrcdnet, RRCDNET)
H16_KERNEL(dsdn, DSDN)
H16_KERNEL(pidn, PIDN)

}  // namespace H16_NS

typedef void (*fused_kernel_t)(const uint8_t*, const float*, float*, int, int, int);

// Host launcher: one workgroup per (spectrum, tile); tiles along L overlap by 2*halo.
hipError_t H16_LAUNCH(int arch, const uint8_t* blob, const float* x, float* y, int64_t n, int L,
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
                       x + n0 * L, y + n0 * L, L, T, tiles);
  }
  return hipGetLastError();
}

}  // namespace rdn
