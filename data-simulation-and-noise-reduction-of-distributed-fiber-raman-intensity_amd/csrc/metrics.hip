// Evaluation metrics on the device, one 256-thread workgroup per spectrum, fp64 arithmetic.
//
// Reference: */evaulate.py:14-21 (MSE, Smoothness = mean|diff|, Peak2Peak), :35 skimage 0.18.3
// structural_similarity(clean, denoised, data_range = clean.max() - clean.min()) with its
// defaults (7-wide uniform filter, K1 0.01, K2 0.03, sample covariance 7/6, mean over the image
// cropped by 3).  The crop removes exactly the filter radius, so every surviving window lies in
// [0, L) and the 'reflect' border never contributes: S is evaluated for window starts
// i = 0 .. L-7 (centres 3 .. L-4).  Per-spectrum values replace the per-spectrum host loop of
// evaulate.py:29-37 and its .cpu() sync; the sums are what ranks all-reduce.
#include "common.hpp"

namespace rdn {
namespace met {

constexpr int MT = 256;

template <typename T, typename Op>
__device__ __forceinline__ T block_reduce(T v, T* scratch, Op op) {
  for (int o = 32; o > 0; o >>= 1) v = op(v, __shfl_xor(v, o));
  const int w = __builtin_amdgcn_workitem_id_x() >> 6, lane = __builtin_amdgcn_workitem_id_x() & 63;
  __syncthreads();
  if (lane == 0) scratch[w] = v;
  __syncthreads();
  T r = scratch[0];
  for (int i = 1; i < MT / 64; ++i) r = op(r, scratch[i]);
  return r;
}

__global__ __launch_bounds__(MT) void metrics_kernel(const float* __restrict__ y, const float* __restrict__ clean,
                                                     int L, double* __restrict__ per, double* __restrict__ sums) {
  __shared__ double red[MT / 64];
  const int tid = __builtin_amdgcn_workitem_id_x();
  const float* yy = y + (size_t)__builtin_amdgcn_workgroup_id_x() * L;
  const float* cc = clean + (size_t)__builtin_amdgcn_workgroup_id_x() * L;
  const auto add = [](double a, double b) { return a + b; };
  const auto mx = [](double a, double b) { return a > b ? a : b; };
  const auto mn = [](double a, double b) { return a < b ? a : b; };

  double se = 0.0, sm = 0.0, ymax = -INFINITY, ymin = INFINITY, cmax = -INFINITY, cmin = INFINITY;
  for (int p = tid; p < L; p += MT) {
    const double a = yy[p], c = cc[p];
    se += (a - c) * (a - c);
    if (p + 1 < L) sm += fabs((double)yy[p + 1] - a);
    ymax = fmax(ymax, a);
    ymin = fmin(ymin, a);
    cmax = fmax(cmax, c);
    cmin = fmin(cmin, c);
  }
  se = block_reduce(se, red, add);
  sm = block_reduce(sm, red, add);
  ymax = block_reduce(ymax, red, mx);
  ymin = block_reduce(ymin, red, mn);
  cmax = block_reduce(cmax, red, mx);
  cmin = block_reduce(cmin, red, mn);

  const double R = cmax - cmin;
  const double C1 = (0.01 * R) * (0.01 * R), C2 = (0.03 * R) * (0.03 * R);
  const double cov = 7.0 / 6.0;
  double ss = 0.0;
  for (int i = tid; i + 7 <= L; i += MT) {
    double sx = 0, sy = 0, sxx = 0, syy = 0, sxy = 0;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      const double a = cc[i + k], b = yy[i + k];
      sx += a;
      sy += b;
      sxx += a * a;
      syy += b * b;
      sxy += a * b;
    }
    const double ux = sx / 7, uy = sy / 7;
    const double vx = cov * (sxx / 7 - ux * ux), vy = cov * (syy / 7 - uy * uy), vxy = cov * (sxy / 7 - ux * uy);
    ss += ((2 * ux * uy + C1) * (2 * vxy + C2)) / ((ux * ux + uy * uy + C1) * (vx + vy + C2));
  }
  ss = block_reduce(ss, red, add);

  if (tid == 0) {
    const double m4[4] = {se / L, ss / (L - 6), sm / (L - 1), ymax - ymin};
    if (per) {
      for (int k = 0; k < 4; ++k) per[(size_t)__builtin_amdgcn_workgroup_id_x() * 4 + k] = m4[k];
    }
    if (sums) {
      for (int k = 0; k < 4; ++k) atomicAdd(&sums[k], m4[k]);
      atomicAdd(&sums[4], 1.0);
    }
  }
}

}  // namespace met

hipError_t launch_metrics(const float* y, const float* clean, int64_t n, int L, double* per, double* sums,
                          hipStream_t stream) {
  const int64_t chunk = 0x7fffffff;
  for (int64_t n0 = 0; n0 < n; n0 += chunk) {
    const int64_t nn = n - n0 < chunk ? n - n0 : chunk;
    hipLaunchKernelGGL(met::metrics_kernel, dim3((unsigned)nn), dim3(met::MT), 0, stream, y + n0 * L, clean + n0 * L, L,
                       per ? per + n0 * 4 : nullptr, sums);
  }
  return hipGetLastError();
}

}  // namespace rdn
