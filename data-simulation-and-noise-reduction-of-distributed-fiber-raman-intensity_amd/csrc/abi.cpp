// C ABI (include/raman_mi355x.h): argument checking, error reporting and dispatch.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <string>

#include "../../include/raman_mi355x.h"
#include "common.hpp"
#include "netspec.hpp"
#include "host_util.hpp"

namespace rdn {
std::string pack(int arch, int dtype, const float* const* tensors, const int64_t* numels, int n, void* dst, size_t cap);
size_t packed_bytes(const std::vector<Op>& spec, int dtype);
void set_corr_mask(void* blob, uint64_t mask);
uint64_t get_corr_mask(const void* blob);
uint32_t get_blob_tag(const void* blob);
uint64_t f16mix_default_mask(int arch);
hipError_t launch_fused16(int arch, const uint8_t* blob, const float* x, float* y, int64_t n, int L, unsigned* status,
                          hipStream_t s);
hipError_t launch_fused16_f16(int arch, const uint8_t* blob, const float* x, float* y, int64_t n, int L, unsigned* status,
                              hipStream_t s);
hipError_t launch_fused16_f16_walk(int arch, const uint8_t* blob, const float* x, float* y, int64_t n, int L,
                                   unsigned* status, const met::MetricOut* mo, hipStream_t s);
hipError_t launch_fused16_f16_small(int arch, const uint8_t* blob, const float* x, float* y, int64_t n, int L,
                                   unsigned* status, hipStream_t s);
hipError_t launch_fused_inplace_walk(const uint8_t* blob, const float* x, float* y, int64_t n, int L, unsigned* status,
                                     const met::MetricOut* mo, hipStream_t s);
hipError_t launch_fused_inplace_short(const uint8_t* blob, const float* x, float* y, int64_t n, int L, unsigned* status,
                                      hipStream_t s);
hipError_t launch_fused_inplace(int arch, int dtype, const uint8_t* blob, const float* x, float* y, int64_t n, int L,
                                unsigned* status, hipStream_t s);

hipError_t launch_cbam_forward(int arch, int dtype, const uint8_t* blob, const float* x, float* y, int64_t n, int L,
                               void* ws, size_t ws_bytes, hipStream_t s);
size_t cbam_workspace_bytes(int arch, int dtype, int64_t n, int64_t L, hipStream_t s);
hipError_t cbam_status(int arch, int dtype, int64_t L, void* ws, size_t ws_bytes, hipStream_t s, int* timed_out,
                       int* out_of_range, int* gate);
hipError_t cbam_workspace_init(int arch, int dtype, int64_t L, void* ws, size_t ws_bytes, hipStream_t s);
hipError_t launch_generate(uint64_t seed, uint64_t first, int64_t n, int L, float snr_lo, float snr_hi, float extreme_prob,
                           int max_repeat, float* clean, float* noisy, float* snr, float* nstd, hipStream_t s);
hipError_t launch_metrics(const float* y, const void* clean, bool clean_f64, int64_t n, int L, double* per, double* sums,
                          long long* acc, hipStream_t s);
}  // namespace rdn

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

int hip_check(hipError_t e, const char* what) {
  if (e == hipSuccess) return RDN_OK;
  return fail(RDN_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

bool valid_arch(int a) { return a >= RDN_DENOISECNN && a <= RDN_APIDN; }
bool valid_dtype(int d) { return d >= RDN_F32 && d <= RDN_F16MIX; }
bool is_cbam(int a) { return a == RDN_ADSDN || a == RDN_APIDN; }
// the dtypes whose e4m3 correction planes bound the activations (RDN_ERANGE, inplace.hpp range_vote)
bool range_checked(int d) { return d == RDN_F16F8 || d == RDN_F16MIX; }
// the fused networks' 16-bit forwards keep a status word in the first 4 bytes of a RANGE_WS_BYTES
// workspace (common.hpp STATUS_*): the range bit of the range-checked dtypes and, for every 16-bit
// dtype, the input gate bit raised by the stems
bool status_word(int d) { return d != RDN_F32; }
constexpr size_t RANGE_WS_BYTES = 256;
const char* range_msg() {
  return "an activation left the range of the e4m3 correction planes (|v| > 1792, RDN_F16F8 / RDN_F16MIX): the "
         "affected tiles' outputs are NaN; inputs this large need RDN_F32 or RDN_BF16X3";
}
// RDN_F16MIX exists for RRCDNet only (checked before any per-network dispatch)
bool unsupported(int arch, int dtype) { return dtype == RDN_F16MIX && arch != RDN_RRCDNET; }
int fail_unsupported(const char* fn) {
  return fail(RDN_EUNSUPPORTED, std::string(fn) + ": RDN_F16MIX is built for RRCDNet; the other networks run RDN_F16");
}

static_assert(rdn::BLOB_MAGIC == RDN_BLOB_MAGIC, "blob tag magic");
static_assert(sizeof(long long) == sizeof(int64_t), "accumulator words");

}  // namespace

#define RDN_GUARD_BEGIN try {
#define RDN_GUARD_END                                     \
  }                                                       \
  catch (const std::exception& ex) {                      \
    return fail(RDN_EINVAL, std::string("exception: ") + ex.what()); \
  }                                                       \
  catch (...) {                                           \
    return fail(RDN_EINVAL, "unknown exception");         \
  }

extern "C" {

#ifndef RDN_SOURCE_HASH
#define RDN_SOURCE_HASH "unstamped"
#endif

int rdn_version(void) { return RDN_ABI_VERSION; }

const char* rdn_build_id(void) { return RDN_SOURCE_HASH; }

const char* rdn_last_error(void) { return g_err.c_str(); }

int rdn_param_names(int arch, char* buf, size_t cap, size_t* needed) {
  RDN_GUARD_BEGIN
  if (!valid_arch(arch)) return fail(RDN_EINVAL, "unknown arch " + std::to_string(arch));
  std::string all;
  for (const std::string& s : rdn::param_names(rdn::net_spec(arch))) {
    all += s;
    all += '\n';
  }
  if (needed) *needed = all.size() + 1;
  if (buf && cap) {
    const size_t n = all.size() + 1 <= cap ? all.size() + 1 : cap;
    std::memcpy(buf, all.c_str(), n);
    buf[n - 1] = '\0';
    if (n < all.size() + 1) return fail(RDN_ESIZE, "buffer too small for parameter names");
  }
  return RDN_OK;
  RDN_GUARD_END
}

int rdn_packed_size(int arch, int dtype, size_t* bytes) {
  RDN_GUARD_BEGIN
  if (!valid_arch(arch) || !valid_dtype(dtype) || !bytes) return fail(RDN_EINVAL, "rdn_packed_size: bad argument");
  *bytes = rdn::packed_bytes(rdn::net_spec(arch), dtype);
  return RDN_OK;
  RDN_GUARD_END
}

int rdn_pack(int arch, int dtype, const float* const* tensors, const int64_t* numels, int n_tensors, void* dst,
             size_t cap) {
  RDN_GUARD_BEGIN
  if (!valid_arch(arch) || !valid_dtype(dtype) || !tensors || !numels || !dst || n_tensors < 0)
    return fail(RDN_EINVAL, "rdn_pack: bad argument");
  const std::string err = rdn::pack(arch, dtype, tensors, numels, n_tensors, dst, cap);
  if (!err.empty()) {
    const bool shape = err.find("expected") != std::string::npos || err.find("tensors") != std::string::npos;
    return fail(err.find("too small") != std::string::npos ? RDN_ESIZE : shape ? RDN_ESHAPE : RDN_EINVAL, err);
  }
  return RDN_OK;
  RDN_GUARD_END
}

int rdn_check_blob(int arch, int dtype, const void* host_blob, size_t bytes) {
  RDN_GUARD_BEGIN
  if (!valid_arch(arch) || !valid_dtype(dtype) || !host_blob) return fail(RDN_EINVAL, "rdn_check_blob: bad argument");
  if (unsupported(arch, dtype)) return fail_unsupported("rdn_check_blob");
  const size_t need = rdn::packed_bytes(rdn::net_spec(arch), dtype);
  if (bytes < need) return fail(RDN_ESIZE, "rdn_check_blob: blob of " + std::to_string(bytes) + " bytes, the layout needs " +
                                               std::to_string(need));
  const uint32_t tag = rdn::get_blob_tag(host_blob);
  if (tag != rdn::blob_tag(arch, dtype)) {
    if ((tag & 0xffff0000u) != RDN_BLOB_MAGIC) return fail(RDN_EINVAL, "rdn_check_blob: not an rdn_pack blob (no layout tag)");
    return fail(RDN_EINVAL, "rdn_check_blob: blob packed for arch " + std::to_string((tag >> 8) & 0xff) + " dtype " +
                                std::to_string(tag & 0xff) + ", not arch " + std::to_string(arch) + " dtype " +
                                std::to_string(dtype));
  }
  return RDN_OK;
  RDN_GUARD_END
}

int rdn_default_correction_mask(int arch, uint64_t* mask) {
  RDN_GUARD_BEGIN
  if (!valid_arch(arch) || !mask) return fail(RDN_EINVAL, "rdn_default_correction_mask: bad argument");
  *mask = rdn::f16mix_default_mask(arch);
  return RDN_OK;
  RDN_GUARD_END
}

int rdn_get_correction_mask(int arch, int dtype, const void* host_blob, size_t bytes, uint64_t* mask) {
  RDN_GUARD_BEGIN
  if (!valid_arch(arch) || !valid_dtype(dtype) || !host_blob || !mask)
    return fail(RDN_EINVAL, "rdn_get_correction_mask: bad argument");
  if (dtype != RDN_F16F8 && dtype != RDN_F16MIX) return fail(RDN_EINVAL, "rdn_get_correction_mask: not a correction layout");
  const int chk = rdn_check_blob(arch, dtype, host_blob, bytes);
  if (chk != RDN_OK) return chk;
  *mask = rdn::get_corr_mask(host_blob);
  return RDN_OK;
  RDN_GUARD_END
}

int rdn_workspace_size(int arch, int dtype, int64_t n, int64_t L, size_t* bytes, void* stream) {
  RDN_GUARD_BEGIN
  if (!valid_arch(arch) || !valid_dtype(dtype) || !bytes || n < 0 || L < 1)
    return fail(RDN_EINVAL, "rdn_workspace_size: bad argument");
  if (unsupported(arch, dtype)) return fail_unsupported("rdn_workspace_size");
  *bytes = is_cbam(arch) ? rdn::cbam_workspace_bytes(arch, dtype, n, L, (hipStream_t)stream)
                          : status_word(dtype) ? RANGE_WS_BYTES : 0;
  return RDN_OK;
  RDN_GUARD_END
}

int rdn_workspace_init(int arch, int dtype, int64_t n, int64_t L, void* ws, size_t ws_bytes, void* stream) {
  RDN_GUARD_BEGIN
  if (!valid_arch(arch) || !valid_dtype(dtype) || n < 0 || L < 1 || L > 0x7fffffff)
    return fail(RDN_EINVAL, "rdn_workspace_init: bad argument");
  if (unsupported(arch, dtype)) return fail_unsupported("rdn_workspace_init");
  const hipStream_t s = (hipStream_t)stream;
  if (!is_cbam(arch)) {
    if (!status_word(dtype)) return RDN_OK;
    if (!ws || ws_bytes < RANGE_WS_BYTES)
      return fail(RDN_ESIZE, "rdn_workspace_init: workspace too small, need " + std::to_string(RANGE_WS_BYTES) + " bytes");
    return hip_check(hipMemsetAsync(ws, 0, 4, s), "rdn_workspace_init");
  }
  const size_t need = rdn::cbam_workspace_bytes(arch, dtype, n, L, s);
  if (ws_bytes < need || (need && !ws))
    return fail(RDN_ESIZE, "rdn_workspace_init: workspace too small, need " + std::to_string(need) + " bytes");
  return hip_check(rdn::cbam_workspace_init(arch, dtype, L, ws, ws_bytes, s), "rdn_workspace_init");
  RDN_GUARD_END
}

// Latency geometry: a launch whose 640-row tiles would occupy at most half the CUs (the reference's
// evaulate.py calls the model one spectrum at a time: 18 workgroups at L = 10,000) runs RDN_F16 /
// RDN_F16MIX on 256-row tiles instead (2.8x the workgroups, each layer ~0.4x as long).  RDN_SHORT_TILES
// = 0 / 1 forces either geometry (tests compare the two).
static bool short_tiles(int arch, int64_t n, int64_t L, hipStream_t s) {
  const char* env = std::getenv("RDN_SHORT_TILES");
  if (env && (env[0] == '0' || env[0] == '1')) return env[0] == '1';
  const int64_t T = rdn::H16_WB - 2 * rdn::fused_halo(arch), tiles = (L + T - 1) / T;
  const int cus = rdn::device_cus(rdn::stream_device(s));
  return cus > 0 && 2 * n * tiles <= cus;
}

// Walk geometry (one workgroup walks a whole spectrum, no halo recompute: fused16_walk.hip for RDN_F16
// on DenoiseCNN / RRCDNet / DSDN / PIDN -- the networks with a walk_shift -- in 576-row tiles;
// rrcdnet_hybrid_walk.hpp for RDN_F16MIX RRCDNet, 576-row tiles, RDN_WALK_ROWS_MIX) when
// its predicted time -- rounds of the CUs x tiles per spectrum x rows per tile -- is below that of the
// 640-row tiles (rounds x 640 rows): large batches.  RDN_WALK = 0 / 1 forces either geometry (tests
// compare the two).
static bool walk_tiles(int arch, int dtype, int64_t n, int64_t L, hipStream_t s) {
  if (!rdn::walk_shift(arch) || (dtype != RDN_F16 && dtype != RDN_F16MIX)) return false;
  const int64_t rows = dtype == RDN_F16MIX ? RDN_WALK_ROWS_MIX : rdn::H16_WALK_ROWS;
  const char* env = std::getenv("RDN_WALK");
  if (env && (env[0] == '0' || env[0] == '1')) return env[0] == '1';
  const int64_t cus = rdn::device_cus(rdn::stream_device(s));
  if (cus <= 0) return false;
  const int64_t T = rdn::H16_WB - 2 * rdn::fused_halo(arch), tiles = (L + T - 1) / T;
  const int64_t wt = (L + rdn::walk_shift(arch) + rows - 1) / rows;
  const int64_t walk_rows = (n + cus - 1) / cus * wt * rows;
  const int64_t tile_rows = (n * tiles + cus - 1) / cus * rdn::H16_WB;
  return walk_rows < tile_rows;
}

// The forward of rdn_forward / rdn_forward_metrics.  mo (may be NULL): metrics of y against mo->clean;
// on the walk geometry the forward kernel computes them (each spectrum's workgroup after its walk,
// *fused = true), otherwise the metrics kernel runs after the forward on the same stream.
static int forward_impl(const char* who, int arch, int dtype, const void* packed, const float* x, float* y, int64_t n,
                        int64_t L, void* ws, size_t ws_bytes, const rdn::met::MetricOut* mo, hipStream_t s, bool* fused) {
  if (!valid_arch(arch) || !valid_dtype(dtype)) return fail(RDN_EINVAL, std::string(who) + ": unknown arch/dtype");
  // x / y may be NULL for an empty batch (an empty torch tensor's data pointer); the blob may not
  if (!packed || (n > 0 && (!x || !y))) return fail(RDN_EINVAL, std::string(who) + ": null pointer");
  if (n < 0 || L < 1 || L > 0x7fffffff) return fail(RDN_EINVAL, std::string(who) + ": need n >= 0 and 1 <= L < 2^31");
  if (mo && L < 7) return fail(RDN_EINVAL, std::string(who) + ": need L >= 7 (SSIM window)");
  if (n == 0) return RDN_OK;
  {  // tiles re-read their input halos while other tiles' outputs (and parked head rows) land in y
    const uintptr_t xb = (uintptr_t)x, yb = (uintptr_t)y, bytes = (uintptr_t)(n * L) * sizeof(float);
    if (xb < yb + bytes && yb < xb + bytes) return fail(RDN_EINVAL, std::string(who) + ": x and y overlap");
  }
  if (unsupported(arch, dtype)) return fail_unsupported(who);
  const uint8_t* blob = (const uint8_t*)packed;
  hipError_t e = hipSuccess;
  bool done = false;          // metrics computed by the forward kernel
  if (is_cbam(arch)) {
    const size_t need = rdn::cbam_workspace_bytes(arch, dtype, n, L, s);
    if (ws_bytes < need || (need && !ws))
      return fail(RDN_ESIZE, std::string(who) + ": workspace too small, need " + std::to_string(need) + " bytes");
    e = rdn::launch_cbam_forward(arch, dtype, blob, x, y, n, (int)L, ws, ws_bytes, s);
  } else {
    // status word of the 16-bit dtypes (optional: without a workspace a saturated tile still writes NaN,
    // and the input gate is not reported)
    unsigned* status = status_word(dtype) && ws && ws_bytes >= RANGE_WS_BYTES ? (unsigned*)ws : nullptr;
    const bool shrt = dtype != RDN_BF16 && short_tiles(arch, n, L, s);
    const bool walk = dtype != RDN_BF16 && !shrt && walk_tiles(arch, dtype, n, L, s);
    if (dtype == RDN_BF16) e = rdn::launch_fused16(arch, blob, x, y, n, (int)L, status, s);
    else if (dtype == RDN_F16 && walk) e = rdn::launch_fused16_f16_walk(arch, blob, x, y, n, (int)L, status, mo, s), done = true;
    else if (dtype == RDN_F16)
      e = shrt ? rdn::launch_fused16_f16_small(arch, blob, x, y, n, (int)L, status, s)
               : rdn::launch_fused16_f16(arch, blob, x, y, n, (int)L, status, s);
    else if (dtype == RDN_F16MIX && walk) e = rdn::launch_fused_inplace_walk(blob, x, y, n, (int)L, status, mo, s), done = true;
    else if (dtype == RDN_F16MIX && shrt) e = rdn::launch_fused_inplace_short(blob, x, y, n, (int)L, status, s);
    else e = rdn::launch_fused_inplace(arch, dtype, blob, x, y, n, (int)L, status, s);
  }
  if (e != hipSuccess) return hip_check(e, who);
  done = done && mo;
  if (fused) *fused = done;
  if (mo && !done) e = rdn::launch_metrics(y, mo->clean, mo->clean_f64 != 0, n, (int)L, mo->per, mo->sums, mo->acc, s);
  return hip_check(e, who);
}

int rdn_forward(int arch, int dtype, const void* packed, const float* x, float* y, int64_t n, int64_t L, void* ws,
                size_t ws_bytes, void* stream) {
  RDN_GUARD_BEGIN
  return forward_impl("rdn_forward", arch, dtype, packed, x, y, n, L, ws, ws_bytes, nullptr, (hipStream_t)stream, nullptr);
  RDN_GUARD_END
}

int rdn_forward_metrics(int arch, int dtype, const void* packed, const float* x, float* y, int64_t n, int64_t L,
                        const void* clean, int clean_is_f64, double* per_spectrum, double* sums, int64_t* acc, void* ws,
                        size_t ws_bytes, void* stream, int* fused) {
  RDN_GUARD_BEGIN
  if (!clean && n > 0) return fail(RDN_EINVAL, "rdn_forward_metrics: null clean pointer");
  if (clean_is_f64 != 0 && clean_is_f64 != 1) return fail(RDN_EINVAL, "rdn_forward_metrics: clean_is_f64 must be 0 or 1");
  const rdn::met::MetricOut mo{clean, clean_is_f64, per_spectrum, sums, (long long*)acc};
  bool f = false;
  const int rc = forward_impl("rdn_forward_metrics", arch, dtype, packed, x, y, n, L, ws, ws_bytes, &mo, (hipStream_t)stream, &f);
  if (fused) *fused = rc == RDN_OK && f ? 1 : 0;
  return rc;
  RDN_GUARD_END
}

// rdn_forward_status / rdn_forward_status_ex: wait for the stream, read and clear every sticky status
// word, report all of them through *flags, fail on a hand-off timeout (RDN_EHIP) or a saturated
// activation (RDN_ERANGE); the input gate is informational (flags only).
static int forward_status(const char* who, int arch, int dtype, int64_t n, int64_t L, void* ws, size_t ws_bytes,
                          hipStream_t s, unsigned* flags) {
  if (flags) *flags = 0;
  if (!valid_arch(arch) || !valid_dtype(dtype)) return fail(RDN_EINVAL, std::string(who) + ": unknown arch/dtype");
  if (n < 0 || L < 1 || L > 0x7fffffff) return fail(RDN_EINVAL, std::string(who) + ": bad n / L");
  if (unsupported(arch, dtype)) return fail_unsupported(who);
  if (!is_cbam(arch)) {
    if (!status_word(dtype) || !ws || ws_bytes < RANGE_WS_BYTES) return hip_check(hipStreamSynchronize(s), who);
    // the word's copy is ordered behind the forwards on their stream: one wait covers both
    unsigned w = 0;
    int rc = hip_check(rdn::read_words(&w, ws, sizeof(w), s), who);
    if (rc != RDN_OK) return rc;
    if (!w) return RDN_OK;
    if (flags) *flags = w & (RDN_STATUS_RANGE | RDN_STATUS_GATE);
    // cleared on the forwards' stream: ordered before the next forward enqueued there
    rc = hip_check(hipMemsetAsync(ws, 0, 4, s), who);
    // the input-gate bit is informational (the module's fp32 re-run decision): only the range bit fails
    return rc != RDN_OK || !(w & rdn::STATUS_RANGE) ? rc : fail(RDN_ERANGE, range_msg());
  }
  // n = 0 with no workspace: nothing ran.  With one, its sticky words may hold earlier forwards' bits
  // (a workspace made for an empty batch and reused for larger ones): read them
  if (n == 0 && !ws) return hip_check(hipStreamSynchronize(s), who);
  const size_t need = rdn::cbam_workspace_bytes(arch, dtype, n, L, s);
  if (ws_bytes < need || (need && !ws))
    return fail(RDN_ESIZE, std::string(who) + ": workspace smaller than this device's CBAM geometry needs (" +
                               std::to_string(need) + " bytes)");
  int timed_out = 0, out_of_range = 0, gate = 0;
  const int rc = hip_check(rdn::cbam_status(arch, dtype, L, ws, ws_bytes, s, &timed_out, &out_of_range, &gate), who);
  if (rc != RDN_OK) return rc;
  if (flags)
    *flags = (out_of_range ? RDN_STATUS_RANGE : 0u) | (gate ? RDN_STATUS_GATE : 0u) | (timed_out ? RDN_STATUS_TIMEOUT : 0u);
  if (timed_out)
    return fail(RDN_EHIP, "CBAM team hand-off timed out: a workgroup of a spectrum's team never arrived (the "
                          "grid's co-residency was broken, e.g. by a concurrent kernel on the device); the "
                          "affected spectra's outputs are NaN");
  if (out_of_range) return fail(RDN_ERANGE, range_msg());
  return RDN_OK;
}

int rdn_forward_status(int arch, int dtype, int64_t n, int64_t L, void* ws, size_t ws_bytes, void* stream) {
  RDN_GUARD_BEGIN
  return forward_status("rdn_forward_status", arch, dtype, n, L, ws, ws_bytes, (hipStream_t)stream, nullptr);
  RDN_GUARD_END
}

int rdn_forward_status_ex(int arch, int dtype, int64_t n, int64_t L, void* ws, size_t ws_bytes, void* stream,
                          unsigned* flags) {
  RDN_GUARD_BEGIN
  return forward_status("rdn_forward_status_ex", arch, dtype, n, L, ws, ws_bytes, (hipStream_t)stream, flags);
  RDN_GUARD_END
}

int rdn_generate(uint64_t seed, uint64_t first_index, int64_t n, const rdn_gen_params* p, float* clean, float* noisy,
                 float* snr_db, float* noise_std, void* stream) {
  RDN_GUARD_BEGIN
  if (!p || (n > 0 && (!clean || !noisy))) return fail(RDN_EINVAL, "rdn_generate: null pointer");
  if (n < 0 || p->signal_length < 1 || p->signal_length > 0x7fffffff || p->max_repeat < 1 || !(p->snr_hi >= p->snr_lo))
    return fail(RDN_EINVAL, "rdn_generate: bad parameters");
  if (n == 0) return RDN_OK;
  return hip_check(rdn::launch_generate(seed, first_index, n, (int)p->signal_length, p->snr_lo, p->snr_hi,
                                        p->extreme_noise_prob, p->max_repeat, clean, noisy, snr_db, noise_std,
                                        (hipStream_t)stream),
                   "generate");
  RDN_GUARD_END
}

int rdn_metrics(const float* y, const float* clean, int64_t n, int64_t L, double* per_spectrum, double* sums,
                void* stream) {
  RDN_GUARD_BEGIN
  if (n > 0 && (!y || !clean)) return fail(RDN_EINVAL, "rdn_metrics: null pointer");
  if (n < 0 || L < 7 || L > 0x7fffffff) return fail(RDN_EINVAL, "rdn_metrics: need L >= 7 (SSIM window)");
  if (n == 0) return RDN_OK;
  return hip_check(rdn::launch_metrics(y, clean, false, n, (int)L, per_spectrum, sums, nullptr, (hipStream_t)stream),
                   "metrics");
  RDN_GUARD_END
}

int rdn_metrics_ex(const float* y, const void* clean, int clean_is_f64, int64_t n, int64_t L, double* per_spectrum,
                   double* sums, int64_t* acc, void* stream) {
  RDN_GUARD_BEGIN
  if (n > 0 && (!y || !clean)) return fail(RDN_EINVAL, "rdn_metrics_ex: null pointer");
  if (clean_is_f64 != 0 && clean_is_f64 != 1) return fail(RDN_EINVAL, "rdn_metrics_ex: clean_is_f64 must be 0 or 1");
  if (n < 0 || L < 7 || L > 0x7fffffff) return fail(RDN_EINVAL, "rdn_metrics_ex: need L >= 7 (SSIM window)");
  if (n == 0) return RDN_OK;
  return hip_check(rdn::launch_metrics(y, clean, clean_is_f64 == 1, n, (int)L, per_spectrum, sums, (long long*)acc,
                                       (hipStream_t)stream),
                   "metrics");
  RDN_GUARD_END
}

// Exact accumulator -> doubles: the limbs are carried into base-2^32 digits of the signed total
// (sign-magnitude after one negation), whose leading 64 bits with a sticky bit for the rest
// convert to double with one round-to-nearest-even.
static double acc_to_double(const int64_t* limb) {
  int64_t l[RDN_ACC_LIMBS];
  for (int j = 0; j < RDN_ACC_LIMBS; ++j) l[j] = limb[j];
  auto carry = [&](uint32_t (&d)[RDN_ACC_LIMBS + 2]) {
    __int128 c = 0;
    for (int j = 0; j < RDN_ACC_LIMBS; ++j) {
      const __int128 t = (__int128)l[j] + c;
      d[j] = (uint32_t)(t & 0xffffffff);
      c = (t - (__int128)d[j]) / ((__int128)1 << 32);
    }
    d[RDN_ACC_LIMBS] = (uint32_t)(c & 0xffffffff);
    d[RDN_ACC_LIMBS + 1] = (uint32_t)((c >> 32) & 0xffffffff);
    return c < 0;
  };
  uint32_t d[RDN_ACC_LIMBS + 2];
  bool neg = carry(d);
  if (neg) {
    for (int j = 0; j < RDN_ACC_LIMBS; ++j) l[j] = -l[j];
    carry(d);
  }
  int top = RDN_ACC_LIMBS + 1;
  while (top >= 0 && d[top] == 0) --top;
  if (top < 0) return 0.0;
  const int hb = 32 * top + (31 - __builtin_clz(d[top]));     // highest set bit
  auto bit = [&](int i) -> uint64_t { return i < 0 ? 0 : (d[i >> 5] >> (i & 31)) & 1u; };
  uint64_t u = 0;
  const int lo = hb - 63;
  for (int i = hb; i >= lo; --i) u = (u << 1) | bit(i);
  bool sticky = false;
  for (int i = lo - 1; i >= 0 && !sticky; --i) sticky = bit(i);
  const double v = std::ldexp((double)(u | (sticky ? 1u : 0u)), lo - RDN_ACC_FRAC_BITS);
  return neg ? -v : v;
}

int rdn_acc_value(const int64_t* acc, double* sums) {
  RDN_GUARD_BEGIN
  if (!acc || !sums) return fail(RDN_EINVAL, "rdn_acc_value: null pointer");
  for (int k = 0; k < 4; ++k) {
    const int64_t* a = acc + k * RDN_ACC_STRIDE;
    sums[k] = a[RDN_ACC_LIMBS] ? std::nan("") : acc_to_double(a);
  }
  sums[4] = (double)acc[RDN_ACC_COUNT];
  return RDN_OK;
  RDN_GUARD_END
}

}  // extern "C"
