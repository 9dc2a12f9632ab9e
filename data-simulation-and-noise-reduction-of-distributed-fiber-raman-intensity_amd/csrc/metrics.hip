// Evaluation metrics on the device: one 512-thread workgroup per spectrum, fp64 arithmetic
// (metrics.hpp spectrum_metrics, shared with the walk kernels' metric epilogue, so both paths give a
// spectrum the same bits).
//
// Reference: */evaulate.py:14-21 (MSE, Smoothness, Peak2Peak), :35 skimage 0.18.3
// structural_similarity; see metrics.hpp.  Per-spectrum values replace the per-spectrum host loop of
// evaulate.py:29-37 and its .cpu() sync; the sums are what ranks all-reduce.
//
// The clean reference is read as fp32 (the on-device simulator's output) or fp64 (a test.npz loaded
// as the reference loads it, 数据集产生.py:73-78 / evaulate.py:61-62: the metrics then see the same
// float64 clean values as evaulate.py:34-35).
#include "metrics.hpp"

namespace rdn {
namespace met {

template <typename TC>
__global__ __launch_bounds__(MET_THREADS) void metrics_kernel(const float* __restrict__ y, const TC* __restrict__ clean,
                                                              int L, MetricOut mo) {
  __shared__ double red[RED_DOUBLES];
  const int64_t n = __builtin_amdgcn_workgroup_id_x();
  const float* yy = y + (size_t)n * L;
  spectrum_metrics([&](int p) { return yy[p]; }, clean + (size_t)n * L, L, n, red, mo);
}

}  // namespace met

template <typename TC>
static hipError_t launch_metrics_t(const float* y, const TC* clean, int64_t n, int L, double* per, double* sums,
                                   long long* acc, hipStream_t stream) {
  const int64_t chunk = 0x7fffffff;
  for (int64_t n0 = 0; n0 < n; n0 += chunk) {
    const int64_t nn = n - n0 < chunk ? n - n0 : chunk;
    const met::MetricOut mo{clean + n0 * L, sizeof(TC) == 8, per ? per + n0 * 4 : nullptr, sums, acc};
    hipLaunchKernelGGL(met::metrics_kernel<TC>, dim3((unsigned)nn), dim3(met::MET_THREADS), 0, stream, y + n0 * L,
                       clean + n0 * L, L, mo);
  }
  return hipGetLastError();
}

hipError_t launch_metrics(const float* y, const void* clean, bool clean_f64, int64_t n, int L, double* per,
                          double* sums, long long* acc, hipStream_t stream) {
  return clean_f64 ? launch_metrics_t(y, (const double*)clean, n, L, per, sums, acc, stream)
                   : launch_metrics_t(y, (const float*)clean, n, L, per, sums, acc, stream);
}

}  // namespace rdn
