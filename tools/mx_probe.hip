// Probe of the gfx950 block-scaled MFMA and fp8 conversions used by the f16f8 engine mode:
//   v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 operands): A/B lane maps and per-lane E8M0 scales,
//   v_cvt_pk_fp8_f32: rounding and out-of-range behaviour.
// Build: hipcc --offload-arch=gfx950 -O2 tools/mx_probe.hip -o tools/mx_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// lane l holds A[row l&15][k = 32 (l>>4) + j] and B[k = 32 (l>>4) + j][col l&15], j = 0..31 (assumed)
__global__ void mx_kernel(const unsigned char* a, const unsigned char* b, const int* sa, const int* sb, float* d) {
  const int l = threadIdx.x;
  i32x8 av, bv;
  memcpy(&av, a + l * 32, 32);
  memcpy(&bv, b + l * 32, 32);
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, c, 0, 0, 0, sa[l], 0, sb[l]);
  for (int i = 0; i < 4; ++i) d[(4 * (l >> 4) + i) * 16 + (l & 15)] = c[i];   // C/D: row 4(l>>4)+i, col l&15
}

template <int OPSEL>
__global__ void mx_kernel_sel(const unsigned char* a, const unsigned char* b, const int* sa, const int* sb, float* d) {
  const int l = threadIdx.x;
  i32x8 av, bv;
  memcpy(&av, a + l * 32, 32);
  memcpy(&bv, b + l * 32, 32);
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  const int sav = sa[l] << (8 * OPSEL), sbv = sb[l] << (8 * OPSEL);
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, c, 0, 0, OPSEL, sav, OPSEL, sbv);
  for (int i = 0; i < 4; ++i) d[(4 * (l >> 4) + i) * 16 + (l & 15)] = c[i];
}

__global__ void cvt2_kernel(unsigned* out) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(1.0f, 2.0f, 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(4.0f, -1.0f, w, true);
  out[0] = (unsigned)w;
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  const f32x2 lo = __builtin_amdgcn_cvt_pk_f32_fp8(w, false), hi = __builtin_amdgcn_cvt_pk_f32_fp8(w, true);
  out[1] = __float_as_uint(lo[0]); out[2] = __float_as_uint(lo[1]); out[3] = __float_as_uint(hi[0]); out[4] = __float_as_uint(hi[1]);
}

__global__ void cvt3_kernel(const float* x, unsigned* out, int n) {
  const int i = threadIdx.x;
  if (i >= n) return;
  int w;
  w = __builtin_amdgcn_cvt_pk_fp8_f32(x[i], -x[i], 0, false);
  out[i] = (unsigned)w;
  typedef short s16x2 __attribute__((ext_vector_type(2)));
  s16x2 o = {0, 0};
  o = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(o, x[i], -x[i], 4.0f, false);
  out[32 + i] = (unsigned)(unsigned short)o[0];
}

__global__ void cvt_kernel(const float* x, unsigned* out, int n) {
  const int i = threadIdx.x;
  if (i < n) out[i] = (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(x[i], -x[i], 0, false);
}

static float e4m3_to_f(unsigned char v) {
  const int s = v >> 7, e = (v >> 3) & 15, m = v & 7;
  if (e == 15 && m == 7) return NAN;
  const float mag = e == 0 ? std::ldexp((float)m, -9) : std::ldexp(1.f + m / 8.f, e - 7);
  return s ? -mag : mag;
}
static unsigned char f_to_e4m3_exact(float f) {   // f must be exactly representable
  for (int v = 0; v < 256; ++v)
    if (e4m3_to_f((unsigned char)v) == f) return (unsigned char)v;
  fprintf(stderr, "not representable %g\n", f);
  exit(2);
}

int main(int argc, char** argv) {
  unsigned char ha[64 * 32], hb[64 * 32];
  int hsa[64], hsb[64];
  float A[16][128], B[128][16];
  srand(7);
  for (int l = 0; l < 64; ++l) {
    hsa[l] = 127 + (l % 5) - 2;            // 2^-2 .. 2^2
    hsb[l] = 127 + (l % 3) - 1;
    for (int j = 0; j < 32; ++j) {
      const float va = (float)(rand() % 15 - 7) / 2.f, vb = (float)(rand() % 13 - 6) / 4.f;
      ha[l * 32 + j] = f_to_e4m3_exact(va);
      hb[l * 32 + j] = f_to_e4m3_exact(vb);
      A[l & 15][32 * (l >> 4) + j] = std::ldexp(va, hsa[l] - 127);
      B[32 * (l >> 4) + j][l & 15] = std::ldexp(vb, hsb[l] - 127);
    }
  }
  unsigned char *da, *db;
  int *dsa, *dsb;
  float* dd;
  hipMalloc(&da, sizeof ha); hipMalloc(&db, sizeof hb); hipMalloc(&dsa, sizeof hsa); hipMalloc(&dsb, sizeof hsb);
  hipMalloc(&dd, 256 * 4);
  hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice); hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
  hipMemcpy(dsa, hsa, sizeof hsa, hipMemcpyHostToDevice); hipMemcpy(dsb, hsb, sizeof hsb, hipMemcpyHostToDevice);
  float D[256], Du[256];
  mx_kernel<<<1, 64>>>(da, db, dsa, dsb, dd);
  hipMemcpy(D, dd, sizeof D, hipMemcpyDeviceToHost);
  int unit[64];
  for (int l = 0; l < 64; ++l) unit[l] = 127;
  hipMemcpy(dsa, unit, sizeof unit, hipMemcpyHostToDevice); hipMemcpy(dsb, unit, sizeof unit, hipMemcpyHostToDevice);
  mx_kernel<<<1, 64>>>(da, db, dsa, dsb, dd);
  hipMemcpy(Du, dd, sizeof Du, hipMemcpyDeviceToHost);
  if (FILE* f = fopen(argc > 1 ? argv[1] : "mx_probe.bin", "wb")) {
    fwrite(ha, 1, sizeof ha, f); fwrite(hb, 1, sizeof hb, f); fwrite(hsa, 4, 64, f); fwrite(hsb, 4, 64, f);
    fwrite(D, 4, 256, f); fwrite(Du, 4, 256, f); fclose(f);
  }
  double maxerr = 0, maxref = 0;
  for (int r = 0; r < 16; ++r)
    for (int c = 0; c < 16; ++c) {
      double ref = 0;
      for (int k = 0; k < 128; ++k) ref += (double)A[r][k] * B[k][c];
      maxerr = fmax(maxerr, fabs(ref - D[r * 16 + c]));
      maxref = fmax(maxref, fabs(ref));
    }
  printf("mfma_scale 16x16x128 e4m3, assumed lane map k = 32(l>>4)+j: max|err| %.3g (max|ref| %.3g) %s\n", maxerr,
         maxref, maxerr <= 1e-4 * maxref ? "MATCH" : "MISMATCH");

  for (int sel = 1; sel < 4; ++sel) {
    hipMemcpy(dsa, hsa, sizeof hsa, hipMemcpyHostToDevice); hipMemcpy(dsb, hsb, sizeof hsb, hipMemcpyHostToDevice);
    if (sel == 1) mx_kernel_sel<1><<<1, 64>>>(da, db, dsa, dsb, dd);
    if (sel == 2) mx_kernel_sel<2><<<1, 64>>>(da, db, dsa, dsb, dd);
    if (sel == 3) mx_kernel_sel<3><<<1, 64>>>(da, db, dsa, dsb, dd);
    float Ds[256];
    hipMemcpy(Ds, dd, sizeof Ds, hipMemcpyDeviceToHost);
    double md = 0;
    for (int i = 0; i < 256; ++i) md = fmax(md, fabs(Ds[i] - D[i]));
    printf("opsel %d with the scale in byte %d: max|D_sel - D_byte0| = %g\n", sel, sel, md);
  }
  {
    unsigned* dc;
    hipMalloc(&dc, 64);
    cvt2_kernel<<<1, 1>>>(dc);
    unsigned hc[5];
    hipMemcpy(hc, dc, sizeof hc, hipMemcpyDeviceToHost);
    float f[4];
    memcpy(f, hc + 1, 16);
    printf("cvt_pk_fp8 (1,2) lo then (4,-1) hi -> 0x%08x ; unpack lo %g %g hi %g %g\n", hc[0], f[0], f[1], f[2], f[3]);
  }
  float hx[16] = {1.f, 1.0625f, 1.1875f, 0.015625f, 0.001953125f, 0.0009765625f, 448.f, 464.f, 480.f, 1000.f, 1e6f, -3.3f, 0.3f, 1e-5f, 240.f, 250.f};
  float* dx;
  unsigned* dout;
  hipMalloc(&dx, sizeof hx); hipMalloc(&dout, 64);
  hipMemcpy(dx, hx, sizeof hx, hipMemcpyHostToDevice);
  cvt_kernel<<<1, 64>>>(dx, dout, 16);
  unsigned hout[16];
  hipMemcpy(hout, dout, sizeof hout, hipMemcpyDeviceToHost);
  for (int i = 0; i < 16; ++i)
    printf("cvt_pk_fp8_f32(%g) -> 0x%02x = %g ; (%g) -> %g\n", hx[i], hout[i] & 0xff, e4m3_to_f(hout[i] & 0xff), -hx[i],
           e4m3_to_f((hout[i] >> 8) & 0xff));
  {
    unsigned* d3;
    hipMalloc(&d3, 64 * 4);
    cvt3_kernel<<<1, 64>>>(dx, d3, 16);
    unsigned h3[64];
    hipMemcpy(h3, d3, sizeof h3, hipMemcpyDeviceToHost);
    for (int i = 0; i < 16; ++i)
      printf("clamp cvt(%g) -> %g, %g ; scalef32(scale 4) cvt(%g) -> %g, %g\n", hx[i], e4m3_to_f(h3[i] & 0xff),
             e4m3_to_f((h3[i] >> 8) & 0xff), hx[i], e4m3_to_f(h3[32 + i] & 0xff), e4m3_to_f((h3[32 + i] >> 8) & 0xff));
  }
  return 0;
}
