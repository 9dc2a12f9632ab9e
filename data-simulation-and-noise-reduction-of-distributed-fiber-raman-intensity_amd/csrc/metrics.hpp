// Per-spectrum evaluation metrics in fp64, shared by the standalone metrics kernel (metrics.hip) and
// the metric epilogue of the walk kernels (fused16.hip walk, rrcdnet_hybrid_walk): one workgroup of
// MET_THREADS threads per spectrum, the same per-thread partition and reduction order in both, so a
// spectrum's four values are the same bits whichever path computed them.
//
// Reference: */evaulate.py:14-21 (MSE, Smoothness = mean|diff|, Peak2Peak), :35 skimage 0.18.3
// structural_similarity(clean, denoised, data_range = clean.max() - clean.min()) with its defaults
// (7-wide uniform filter, K1 0.01, K2 0.03, sample covariance 7/6, mean over the image cropped by 3).
// The crop removes exactly the filter radius, so every surviving window lies in [0, L) and the
// 'reflect' border never contributes: S is evaluated for window starts i = 0 .. L-7 (centres 3 .. L-4).
//
// Exact accumulation (`acc`): every per-spectrum value is added, without rounding, into a fixed-point
// integer accumulator (RDN_ACC_LIMBS int64 limbs of 32 bits per metric, weight 2^(32 j - 128)), so the
// sums are the same bits whatever the order of the atomics, the batch split or the number of ranks
// whose accumulators are all-reduced; rdn_acc_value rounds once.
#pragma once
#include "common.hpp"

namespace rdn {
namespace met {

constexpr int MET_THREADS = 512;      // = the fused kernels' workgroup (8 waves)

template <typename T, typename Op>
__device__ __forceinline__ T block_reduce(T v, T* scratch, Op op) {
  for (int o = 32; o > 0; o >>= 1) v = op(v, __shfl_xor(v, o));
  const int w = __builtin_amdgcn_workitem_id_x() >> 6, lane = __builtin_amdgcn_workitem_id_x() & 63;
  __syncthreads();
  if (lane == 0) scratch[w] = v;
  __syncthreads();
  T r = scratch[0];
  for (int i = 1; i < MET_THREADS / 64; ++i) r = op(r, scratch[i]);
  return r;
}
// Six reductions in one round trip through the scratch (each value reduced exactly as block_reduce
// would: lane butterfly, then the waves in order): sums [0, 2), maxima [2, 4), minima [4, 6)
constexpr int RED_DOUBLES = 6 * (MET_THREADS / 64);
__device__ __forceinline__ void block_reduce6(double (&v)[6], double* scratch) {
  const int w = __builtin_amdgcn_workitem_id_x() >> 6, lane = __builtin_amdgcn_workitem_id_x() & 63;
  auto op = [](int k, double a, double b) { return k < 2 ? a + b : k < 4 ? (a > b ? a : b) : (a < b ? a : b); };
#pragma unroll
  for (int k = 0; k < 6; ++k)
    for (int o = 32; o > 0; o >>= 1) v[k] = op(k, v[k], __shfl_xor(v[k], o));
  __syncthreads();
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < 6; ++k) scratch[k * (MET_THREADS / 64) + w] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    double r = scratch[k * (MET_THREADS / 64)];
    for (int i = 1; i < MET_THREADS / 64; ++i) r = op(k, r, scratch[k * (MET_THREADS / 64) + i]);
    v[k] = r;
  }
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

// The four metrics of spectrum n (denoised values through yv(p), clean cc[0..L)), every thread of the
// MET_THREADS-thread workgroup taking part; red: RED_DOUBLES doubles of LDS.  Results: per[n],
// sums, acc of mo (each optional).
template <typename TC, class YV>
__device__ __forceinline__ void spectrum_metrics(YV yv, const TC* __restrict__ cc, int L, int64_t n, double* red,
                                                 const MetricOut& mo) {
  const int tid = __builtin_amdgcn_workitem_id_x();
  const auto add = [](double a, double b) { return a + b; };

  double se = 0.0, sm = 0.0, ymax = -INFINITY, ymin = INFINITY, cmax = -INFINITY, cmin = INFINITY;
  for (int p = tid; p < L; p += MET_THREADS) {
    const double a = yv(p), c = cc[p];
    se += (a - c) * (a - c);
    if (p + 1 < L) sm += fabs((double)yv(p + 1) - a);
    ymax = fmax(ymax, a);
    ymin = fmin(ymin, a);
    cmax = fmax(cmax, c);
    cmin = fmin(cmin, c);
  }
  double r6[6] = {se, sm, ymax, cmax, ymin, cmin};
  block_reduce6(r6, red);
  se = r6[0], sm = r6[1], ymax = r6[2], cmax = r6[3], ymin = r6[4], cmin = r6[5];

  const double R = cmax - cmin;
  const double C1 = (0.01 * R) * (0.01 * R), C2 = (0.03 * R) * (0.03 * R);
  const double cov = 7.0 / 6.0;
  double ss = 0.0;
  for (int i = tid; i + 7 <= L; i += MET_THREADS) {
    double sx = 0, sy = 0, sxx = 0, syy = 0, sxy = 0;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      const double a = cc[i + k], b = yv(i + k);
      sx += a;
      sy += b;
      sxx += a * a;
      syy += b * b;
      sxy += a * b;
    }
    // window means by one multiplication each (five fp64 divisions per window were most of the loop)
    constexpr double inv7 = 1.0 / 7.0;
    const double ux = sx * inv7, uy = sy * inv7;
    const double vx = cov * (sxx * inv7 - ux * ux), vy = cov * (syy * inv7 - uy * uy), vxy = cov * (sxy * inv7 - ux * uy);
    ss += ((2 * ux * uy + C1) * (2 * vxy + C2)) / ((ux * ux + uy * uy + C1) * (vx + vy + C2));
  }
  ss = block_reduce(ss, red, add);

  const double m4[4] = {se / L, ss / (L - 6), sm / (L - 1), ymax - ymin};
  if (tid == 0) {
    if (mo.per) {
      for (int k = 0; k < 4; ++k) mo.per[n * 4 + k] = m4[k];
    }
    if (mo.sums) {
      for (int k = 0; k < 4; ++k) atomicAdd(&mo.sums[k], m4[k]);
      atomicAdd(&mo.sums[4], 1.0);
    }
  }
  // exact accumulator: lanes 0..3 of wave 0 each own one metric (integer atomics: order-free)
  if (mo.acc && tid < 4) {
    long long limb[RDN_ACC_LIMBS];
    const bool ok = to_limbs(m4[tid], limb);
    long long* a = mo.acc + tid * RDN_ACC_STRIDE;
    if (ok) {
#pragma unroll
      for (int j = 0; j < RDN_ACC_LIMBS; ++j)
        if (limb[j]) atomicAdd((unsigned long long*)&a[j], (unsigned long long)limb[j]);
    } else {
      atomicAdd((unsigned long long*)&a[RDN_ACC_LIMBS], 1ull);   // this metric's out-of-range count
    }
    if (tid == 0) atomicAdd((unsigned long long*)&mo.acc[RDN_ACC_COUNT], 1ull);
  }
}

// The metric epilogue of a walk kernel: spectrum n's denoised row y (written by this workgroup's
// waves) is read back once every wave's stores have completed, through L1-bypassing (sc1) buffer loads
// from the L2 they landed in (no L1 line of y this CU may hold from an earlier spectrum -- the rows of
// neighbouring spectra share lines -- is trusted); the LDS is free once the walk's last barrier passed.
// One workgroup per CU and one spectrum at a time leave no other workgroup to hide memory latency, so
// y and clean are first staged into the LDS with eight loads in flight per thread (one round trip per
// 4096 values, not one per value), and the metric loops then read the LDS; spectra too long for the
// LDS read memory directly.  The values are the same either way (the same routine on the same numbers).
template <typename T, class LD>
__device__ __forceinline__ void stage_row(T* dst, int L, LD ld) {
  const int tid = __builtin_amdgcn_workitem_id_x();
  for (int p0 = 0; p0 < L; p0 += 8 * MET_THREADS) {
    T v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int p = p0 + tid + k * MET_THREADS;
      v[k] = p < L ? ld(p) : (T)0;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int p = p0 + tid + k * MET_THREADS;
      if (p < L) dst[p] = v[k];
    }
  }
}
template <typename TC>
__device__ __forceinline__ void walk_metrics_t(const float* y, const TC* cc, int L, int64_t n, char* lds,
                                               const MetricOut& mo) {
  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc((void*)y, 0, L * 4, 0x00020000);
  const auto yg = [&](int p) { return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(yr, 4 * p, 0, 16)); };
  double* red = (double*)lds;
  constexpr int RED = RED_DOUBLES * 8, LDS_MAX = 163840;
  const int yb = (L * 4 + 15) & ~15;
  if (RED + yb + (size_t)L * sizeof(TC) <= (size_t)LDS_MAX) {
    float* ys = (float*)(lds + RED);
    TC* cs = (TC*)(lds + RED + yb);
    stage_row(ys, L, yg);
    stage_row(cs, L, [&](int p) { return cc[p]; });
    __syncthreads();
    spectrum_metrics([&](int p) { return ys[p]; }, (const TC*)cs, L, n, red, mo);
  } else {
    spectrum_metrics(yg, cc, L, n, red, mo);
  }
}
__device__ __forceinline__ void walk_metrics(const float* y, int L, int64_t n, char* lds, const MetricOut& mo) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // this wave's y stores are in L2
  __syncthreads();
  if (mo.clean_f64) walk_metrics_t(y, (const double*)mo.clean + (size_t)n * L, L, n, lds, mo);
  else walk_metrics_t(y, (const float*)mo.clean + (size_t)n * L, L, n, lds, mo);
  __syncthreads();                                      // the LDS the next use may overwrite
}

}  // namespace met
}  // namespace rdn
