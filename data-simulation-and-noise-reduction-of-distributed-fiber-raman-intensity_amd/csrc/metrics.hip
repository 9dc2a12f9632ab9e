// Evaluation metrics on the device, one 256-thread workgroup per spectrum, fp64 arithmetic.
//
// Reference: */evaulate.py:14-21 (MSE, Smoothness = mean|diff|, Peak2Peak), :35 skimage 0.18.3
// structural_similarity(clean, denoised, data_range = clean.max() - clean.min()) with its
// defaults (7-wide uniform filter, K1 0.01, K2 0.03, sample covariance 7/6, mean over the image
// cropped by 3).  The crop removes exactly the filter radius, so every surviving window lies in
// [0, L) and the 'reflect' border never contributes: S is evaluated for window starts
// i = 0 .. L-7 (centres 3 .. L-4).  Per-spectrum values replace the per-spectrum host loop of
// evaulate.py:29-37 and its .cpu() sync; the sums are what ranks all-reduce.
//
// The clean reference is read as fp32 (the on-device simulator's output) or fp64 (a test.npz loaded
// as the reference loads it, 数据集产生.py:73-78 / evaulate.py:61-62: the metrics then see the same
// float64 clean values as evaulate.py:34-35).
//
// Exact accumulation (rdn_metrics_ex `acc`): every per-spectrum value is added, without rounding,
// into a fixed-point integer accumulator (RDN_ACC_LIMBS int64 limbs of 32 bits per metric, weight
// 2^(32 j - 128)), so the sums are the same bits whatever the order of the atomics, the batch
// split or the number of ranks whose accumulators are all-reduced; rdn_acc_value rounds once.
#include "common.hpp"
#include "../../include/raman_mi355x.h"

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

// Limb j (32 bits at weight 2^(32 j - RDN_ACC_FRAC_BITS)) of the fixed-point image of v, truncated
// toward zero below 2^-128, signed like v.  Returns false if |v| >= 2^64 or v is not finite (the
// metric's out-of-range word counts those; rdn_acc_value then reports NaN for that sum).
__device__ __forceinline__ bool to_limbs(double v, long long (&limb)[RDN_ACC_LIMBS]) {
  for (int j = 0; j < RDN_ACC_LIMBS; ++j) limb[j] = 0;
  const unsigned long long bits = __double_as_longlong(v);
  const int be = (int)((bits >> 52) & 0x7ff);
  if (be == 0x7ff) return false;                                   // inf / NaN
  if (be == 0) return true;                                        // zero / subnormal (< 2^-1022)
  const unsigned long long m = (bits & ((1ull << 52) - 1)) | (1ull << 52);
  const int s = be - 1075 + RDN_ACC_FRAC_BITS;                     // bit position of m's LSB
  if (s + 53 > 32 * RDN_ACC_LIMBS) return false;
  const bool neg = bits >> 63;
#pragma unroll
  for (int j = 0; j < RDN_ACC_LIMBS; ++j) {
    const int o = 32 * j - s;                                      // m's bit at limb j's bit 0
    unsigned long long c = 0;
    if (o >= 0 && o < 53) c = (m >> o) & 0xffffffffull;
    else if (o < 0 && o > -32) c = (m << (-o)) & 0xffffffffull;
    limb[j] = neg ? -(long long)c : (long long)c;
  }
  return true;
}

template <typename TC>
__global__ __launch_bounds__(MT) void metrics_kernel(const float* __restrict__ y, const TC* __restrict__ clean,
                                                     int L, double* __restrict__ per, double* __restrict__ sums,
                                                     long long* __restrict__ acc) {
  __shared__ double red[MT / 64];
  const int tid = __builtin_amdgcn_workitem_id_x();
  const float* yy = y + (size_t)__builtin_amdgcn_workgroup_id_x() * L;
  const TC* cc = clean + (size_t)__builtin_amdgcn_workgroup_id_x() * L;
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

  const double m4[4] = {se / L, ss / (L - 6), sm / (L - 1), ymax - ymin};
  if (tid == 0) {
    if (per) {
      for (int k = 0; k < 4; ++k) per[(size_t)__builtin_amdgcn_workgroup_id_x() * 4 + k] = m4[k];
    }
    if (sums) {
      for (int k = 0; k < 4; ++k) atomicAdd(&sums[k], m4[k]);
      atomicAdd(&sums[4], 1.0);
    }
  }
  // exact accumulator: lanes 0..3 of wave 0 each own one metric (integer atomics: order-free)
  if (acc && tid < 4) {
    long long limb[RDN_ACC_LIMBS];
    const bool ok = to_limbs(m4[tid], limb);
    long long* a = acc + tid * RDN_ACC_STRIDE;
    if (ok) {
#pragma unroll
      for (int j = 0; j < RDN_ACC_LIMBS; ++j)
        if (limb[j]) atomicAdd((unsigned long long*)&a[j], (unsigned long long)limb[j]);
    } else {
      atomicAdd((unsigned long long*)&a[RDN_ACC_LIMBS], 1ull);   // this metric's out-of-range count
    }
    if (tid == 0) atomicAdd((unsigned long long*)&acc[RDN_ACC_COUNT], 1ull);
  }
}

}  // namespace met

template <typename TC>
static hipError_t launch_metrics_t(const float* y, const TC* clean, int64_t n, int L, double* per, double* sums,
                                   long long* acc, hipStream_t stream) {
  const int64_t chunk = 0x7fffffff;
  for (int64_t n0 = 0; n0 < n; n0 += chunk) {
    const int64_t nn = n - n0 < chunk ? n - n0 : chunk;
    hipLaunchKernelGGL(met::metrics_kernel<TC>, dim3((unsigned)nn), dim3(met::MT), 0, stream, y + n0 * L,
                       clean + n0 * L, L, per ? per + n0 * 4 : nullptr, sums, acc);
  }
  return hipGetLastError();
}

hipError_t launch_metrics(const float* y, const void* clean, bool clean_f64, int64_t n, int L, double* per,
                          double* sums, long long* acc, hipStream_t stream) {
  return clean_f64 ? launch_metrics_t(y, (const double*)clean, n, L, per, sums, acc, stream)
                   : launch_metrics_t(y, (const float*)clean, n, L, per, sums, acc, stream);
}

}  // namespace rdn
