// Probe (diagnostic, not product): v_fma_mix_f32 lo-split vs the cvt+sub split on gfx950, incl.
// f16-subnormal inputs.  hipcc --offload-arch=gfx950 -O3 tools/split_probe.hip -o tools/split_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
__global__ void k(const float* r, float* lo_mix, float* lo_ref, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (2 * i + 1 >= n) return;
  float r0 = r[2 * i], r1 = r[2 * i + 1];
  f16x2 h = {(_Float16)r0, (_Float16)r1};
  unsigned hb = __builtin_bit_cast(unsigned, h);
  float a, b;
  asm volatile("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(a) : "v"(hb), "v"(r0));
  asm volatile("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(b) : "v"(hb), "v"(r1));
  lo_mix[2 * i] = a; lo_mix[2 * i + 1] = b;
  lo_ref[2 * i] = r0 - (float)h[0]; lo_ref[2 * i + 1] = r1 - (float)h[1];
}
int main() {
  const int n = 1 << 20;
  std::vector<float> r(n);
  unsigned s = 12345;
  for (int i = 0; i < n; ++i) {
    s = s * 1664525u + 1013904223u;
    float u = (s >> 8) * (1.0f / 16777216.0f);
    float mag = std::ldexp(1.0f, -(int)(i % 30));  // 1 .. 2^-29: f16 normal, subnormal, zero
    r[i] = (i & 1 ? -1.f : 1.f) * u * mag * 7.f;
  }
  float *dr, *dm, *dref;
  hipMalloc(&dr, n * 4); hipMalloc(&dm, n * 4); hipMalloc(&dref, n * 4);
  hipMemcpy(dr, r.data(), n * 4, hipMemcpyHostToDevice);
  k<<<n / 2 / 256, 256>>>(dr, dm, dref, n);
  std::vector<float> m(n), ref(n);
  hipMemcpy(m.data(), dm, n * 4, hipMemcpyDeviceToHost);
  hipMemcpy(ref.data(), dref, n * 4, hipMemcpyDeviceToHost);
  int bad = 0, bad_small = 0; double worst = 0;
  for (int i = 0; i < n; ++i)
    if (m[i] != ref[i]) {
      ++bad;
      if (std::fabs(r[i]) < 6.2e-5f) ++bad_small;
      worst = std::fmax(worst, std::fabs(m[i] - ref[i]));
      if (bad <= 5) printf("r=%.9g mix=%.9g ref=%.9g\n", r[i], m[i], ref[i]);
    }
  printf("mismatches %d of %d (|r| < f16 normal min: %d), worst abs %.3g\n", bad, n, bad_small, worst);
  return 0;
}
