// On-device Raman spectrum simulator: one 256-thread workgroup per spectrum.
//
// Distributional contract: 数据集产生.py:5-64 (generate_signals).  Instead of numpy's global,
// batch-ordered RNG the engine keys a Philox4x32-10 stream on (seed; draw index, draw tag,
// spectrum index), so spectrum i is the same on any GPU, in any batch, at any world size
// (SURVEY.md §3.3, §8e).  Draw layout (mirrored bit-for-bit by oracle/generator.py):
//   TAG_SEG    counter k>>1 : segment k length (U{1..max_repeat}) and value (U[0,1))
//   TAG_SCALAR counter 0    : [snr, extreme?, n_spikes, -]
//   TAG_SPIKE  counter s    : spike s [width, start, amplitude, sign]
//   TAG_NOISE  counter p>>2 : 4 Box-Muller normals for positions p..p+3
// Float transforms are written under `fp contract(off)` (and the file is built with
// -ffp-contract=off) so that no FMA fusion makes them differ from the float32 numpy restatement.
#include "common.hpp"

// Every float op below is rounded on its own, exactly like the numpy restatement: no FMA fusion.
#pragma clang fp contract(off)

namespace rdn {
namespace gen {

constexpr int GT = 256;
enum : uint32_t { TAG_SEG = 1, TAG_SCALAR = 2, TAG_SPIKE = 3, TAG_NOISE = 4 };

struct Params {
  int L;
  float snr_lo, snr_hi, extreme_prob;
  int max_repeat;
};

struct U4 { uint32_t x, y, z, w; };

__device__ __forceinline__ U4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint64_t seed) {
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c0 = hi1 ^ c1 ^ k0;
    c1 = lo1;
    c2 = hi0 ^ c3 ^ k1;
    c3 = lo0;
  }
  return U4{c0, c1, c2, c3};
}

__device__ __forceinline__ float u24(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }
__device__ __forceinline__ float uniform(float lo, float hi, uint32_t x) {
  return lo + (hi - lo) * u24(x);
}
__device__ __forceinline__ int randint(int lo, int hi, uint32_t x) {
  return lo + (int)(((uint64_t)x * (uint64_t)(hi - lo)) >> 32);
}
__device__ __forceinline__ void box_muller(uint32_t a, uint32_t b, float& z0, float& z1) {
  const float u1 = ((float)(a >> 8) + 1.0f) * (1.0f / 16777216.0f);
  const float u2 = u24(b);
  const float r = sqrtf(-2.0f * logf(u1));
  const float th = 6.2831854820251465f * u2;
  float s, c;
  sincosf(th, &s, &c);
  z0 = r * c;
  z1 = r * s;
}

template <typename T, typename Op>
__device__ __forceinline__ T block_reduce(T v, T* scratch, Op op) {
  for (int o = 32; o > 0; o >>= 1) v = op(v, __shfl_xor(v, o));
  const int w = __builtin_amdgcn_workitem_id_x() >> 6, lane = __builtin_amdgcn_workitem_id_x() & 63;
  __syncthreads();
  if (lane == 0) scratch[w] = v;
  __syncthreads();
  T r = scratch[0];
  for (int i = 1; i < GT / 64; ++i) r = op(r, scratch[i]);
  return r;
}

__global__ __launch_bounds__(GT) void generate_kernel(uint64_t seed, uint64_t first, Params prm, float* __restrict__ clean,
                                                      float* __restrict__ noisy, float* __restrict__ snr_out,
                                                      float* __restrict__ std_out) {
  __shared__ int s_scan[GT];
  __shared__ double s_red[GT / 64];
  __shared__ float s_redf[GT / 64];
  __shared__ float s_spk[3][3];      // start, width, signed amplitude
  __shared__ int s_nspk;
  __shared__ float s_sigma;
  const int tid = __builtin_amdgcn_workitem_id_x();
  const uint64_t idx = first + __builtin_amdgcn_workgroup_id_x();
  const uint32_t ilo = (uint32_t)idx, ihi = (uint32_t)(idx >> 32);
  const int L = prm.L;
  float* cl = clean + (size_t)__builtin_amdgcn_workgroup_id_x() * L;
  float* nz = noisy + (size_t)__builtin_amdgcn_workgroup_id_x() * L;

  // ---- phase A: piecewise-constant segments (raw values into `clean`) --------------------------
  float mn = INFINITY, mx = -INFINITY;
  int pos = 0;
  for (int kb = 0; pos < L; kb += GT) {
    const int k = kb + tid;
    const U4 r = philox((uint32_t)(k >> 1), TAG_SEG, ilo, ihi, seed);
    const uint32_t xl = (k & 1) ? r.z : r.x, xv = (k & 1) ? r.w : r.y;
    const int len = randint(1, prm.max_repeat + 1, xl);
    const float val = u24(xv);
    // inclusive scan of segment lengths (Hillis-Steele in LDS)
    s_scan[tid] = len;
    __syncthreads();
    for (int o = 1; o < GT; o <<= 1) {
      const int add = tid >= o ? s_scan[tid - o] : 0;
      __syncthreads();
      s_scan[tid] += add;
      __syncthreads();
    }
    const int end = pos + s_scan[tid];
    const int start = end - len;
    if (start < L) {
      mn = fminf(mn, val);
      mx = fmaxf(mx, val);
      const int e = end < L ? end : L;
      for (int p = start; p < e; ++p) cl[p] = val;
    }
    pos += s_scan[GT - 1];
    __syncthreads();
  }
  mn = block_reduce(mn, s_redf, [](float a, float b) { return fminf(a, b); });
  mx = block_reduce(mx, s_redf, [](float a, float b) { return fmaxf(a, b); });
  const float den = (mx - mn) + 1e-8f;

  // ---- phase B: signal power of the normalised signal (数据集产生.py:38-43) --------------------
  double ps = 0.0;
  for (int p = tid; p < L; p += GT) {
    const float c = __fdiv_rn(cl[p] - mn, den);
    ps += (double)c * (double)c;
  }
  ps = block_reduce(ps, s_red, [](double a, double b) { return a + b; });

  if (tid == 0) {
    const U4 sc = philox(0u, TAG_SCALAR, ilo, ihi, seed);
    const float snr = uniform(prm.snr_lo, prm.snr_hi, sc.x);
    const float sigma = (float)sqrt((ps / L) / pow(10.0, (double)snr / 10.0));
    const bool extreme = u24(sc.y) < prm.extreme_prob;
    const int ns = extreme ? randint(1, 4, sc.z) : 0;
    for (int s = 0; s < ns; ++s) {
      const U4 sp = philox((uint32_t)s, TAG_SPIKE, ilo, ihi, seed);
      int width = randint(20, 100, sp.x), start = 0;
      if (L - width <= 0) width = L;               // the reference would raise here
      else start = randint(0, L - width, sp.y);
      const float amp = uniform(5.0f, 15.0f, sp.z) * sigma;
      s_spk[s][0] = (float)start;
      s_spk[s][1] = (float)width;
      s_spk[s][2] = u24(sp.w) > 0.5f ? amp : -amp;
    }
    s_nspk = ns;
    s_sigma = sigma;
    if (snr_out) snr_out[__builtin_amdgcn_workgroup_id_x()] = snr;
    if (std_out) std_out[__builtin_amdgcn_workgroup_id_x()] = sigma;
  }
  __syncthreads();
  const float sigma = s_sigma;
  const int ns = s_nspk;

  // ---- phase C: normalise, add noise and spikes (数据集产生.py:38-62) --------------------------
  for (int p0 = 4 * tid; p0 < L; p0 += 4 * GT) {
    const U4 r = philox((uint32_t)(p0 >> 2), TAG_NOISE, ilo, ihi, seed);
    float z[4];
    box_muller(r.x, r.y, z[0], z[1]);
    box_muller(r.z, r.w, z[2], z[3]);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int p = p0 + i;
      if (p >= L) break;
      const float c = __fdiv_rn(cl[p] - mn, den);
      float v = c + sigma * z[i];
      for (int s = 0; s < ns; ++s) {
        const int st = (int)s_spk[s][0], w = (int)s_spk[s][1];
        if (p >= st && p < st + w) v = v + s_spk[s][2];
      }
      cl[p] = c;
      nz[p] = v;
    }
  }
}

}  // namespace gen

hipError_t launch_generate(uint64_t seed, uint64_t first, int64_t n, int L, float snr_lo, float snr_hi,
                           float extreme_prob, int max_repeat, float* clean, float* noisy, float* snr,
                           float* nstd, hipStream_t stream) {
  const gen::Params prm{L, snr_lo, snr_hi, extreme_prob, max_repeat};
  const int64_t chunk = 0x7fffffff;
  for (int64_t n0 = 0; n0 < n; n0 += chunk) {
    const int64_t nn = n - n0 < chunk ? n - n0 : chunk;
    hipLaunchKernelGGL(gen::generate_kernel, dim3((unsigned)nn), dim3(gen::GT), 0, stream, seed, first + n0, prm,
                       clean + n0 * L, noisy + n0 * L, snr ? snr + n0 : nullptr, nstd ? nstd + n0 : nullptr);
  }
  return hipGetLastError();
}

}  // namespace rdn
