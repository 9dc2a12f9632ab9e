/*
 * raman_mi355x — C ABI of the MI355X (gfx950) Raman-denoising inference engine.
 *
 * Plain pointers and sizes only: no PyTorch or HIP types cross this boundary (a HIP stream is
 * passed as `void*`).  Every entry point returns RDN_OK (0) or a negative RDN_E* code and leaves
 * a message for rdn_last_error() (thread-local).  No exception crosses the ABI.  All device
 * buffers are owned by the caller (e.g. the PyTorch caching allocator); the library keeps no
 * device state of its own, enqueues on the caller's stream and never synchronises it.
 *
 * Reference interfaces these entry points replace (paths relative to the reference repo):
 *   rdn_param_names / rdn_packed_size / rdn_pack
 *       -> Model().load_state_dict(torch.load(path))            <model>/evaulate.py:65-66
 *          (the reference keeps nn.Module parameters; the engine folds eval-mode BatchNorm and
 *           re-lays the weights out as MFMA operand fragments once, at load time)
 *   rdn_forward
 *       -> Model.forward(x), x float32 (N, 1, L)                   <model>/evaulate.py:30-32, :84-85
 *          DenoiseCNN 1DCNN/train.py:71-82 · RRCDNet RRCDNet/train.py:72-98 · DSDN DSDN/train.py:101-126
 *          ADSDN ADSDN/train.py:150-167 · PIDN PIDN/train.py:72-106 · APIDN APIDN/train.py:119-159
 *   rdn_generate
 *       -> generate_signals(num_samples, signal_length, snr_range, extreme_noise_prob, max_repeat)
 *                                                                  数据集产生.py:5-64
 *   rdn_metrics / rdn_metrics_ex / rdn_acc_value
 *       -> compute_mse / compute_smoothness / compute_peak_to_peak + skimage SSIM, averaged
 *                                                                  <model>/evaulate.py:14-39
 *   rdn_forward_metrics
 *       -> the body of evaluate(): model(input) then the four metrics of each spectrum, averaged
 *                                                                  <model>/evaulate.py:25-39
 */
#ifndef RAMAN_MI355X_H
#define RAMAN_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RDN_ABI_VERSION 6

typedef enum {
  RDN_DENOISECNN = 0, /* 1DCNN/train.py   class DenoiseCNN */
  RDN_RRCDNET = 1,    /* RRCDNet/train.py class RRCDNet    */
  RDN_DSDN = 2,       /* DSDN/train.py    class DSDN       */
  RDN_ADSDN = 3,      /* ADSDN/train.py   class ADSDN      */
  RDN_PIDN = 4,       /* PIDN/train.py    class PIDN       */
  RDN_APIDN = 5       /* APIDN/train.py   class APIDN      */
} rdn_arch;

/* Arithmetic of the 64->64 convolutions (stems, activations math: fp32; heads: fp32 operands,
 * fp64 accumulation, one final rounding).
 *   RDN_F32    exact-fp32 MFMA, fp32 activations, compensated (chunked TwoSum) accumulation
 *                                                               (1e-5 parity mode)
 *   RDN_BF16   one bf16 MFMA per product, bf16 activations: NO tolerance guarantee (misses the
 *              2e-2 bf16 bar on trained RRCDNet: 0.24); the Python layer names it 'bf16-unsafe' 
 *   RDN_BF16X3 split bf16: operands as bf16 hi+lo pairs, three bf16 MFMAs per product
 *              (hi*hi + hi*lo + lo*hi), ~16-bit operands        (bf16 MFMA at 2e-2-safe accuracy)
 *   RDN_F16F8  f16 main product (v = hi + lo, hi = f16(v)) plus both correction products
 *              W_lo*X_hi + W_hi*X_lo as ONE block-scaled e4m3 MFMA at twice the 16-bit rate; f16 hi
 *              + e4m3 lo activations (~15 significant bits).  2e-2-safe at 2/3 of the MFMA cycles
 *              of RDN_BF16X3.  Range: the e4m3 planes hold |activation| <= 1792 (hi / 4 in e4m3); a
 *              tile whose activations exceed it writes NaN outputs and raises the workspace's range
 *              word (rdn_forward_status: RDN_ERANGE) -- never a silently clamped value.  Inputs of
 *              normalised intensity stay far inside it (trained networks: max |activation| 9-28);
 *              ~100x larger inputs need RDN_F32 or RDN_BF16X3.
 *   RDN_F16    one f16 MFMA per product (v_mfma_f32_16x16x32_f16, the bf16 rate), f16 weights and
 *              activations (11 significant bits), fp32 accumulation: the fastest mode within the 2e-2
 *              bf16 bar on the golden fixtures of 1DCNN, DSDN, ADSDN, PIDN and APIDN (worst 6.9e-3,
 *              trained DSDN) -- NOT on trained RRCDNet (3.6e-2): use RDN_F16MIX there.  Activations
 *              must stay below the f16 range (65504); a larger one becomes inf, never a silent wrong
 *              value.
 *   RDN_F16MIX RRCDNet only: RDN_F16 arithmetic with the RDN_F16F8 correction kept on the last five
 *              layers of the right branch (the ones the head's cancellation x - (r + l)/2 amplifies),
 *              and every layer corrected on a tile whose input window leaves [-0.3, 1.3] (a spike):
 *              within 2e-2 (1.19e-2 on the trained fixture, 1.54e-2 worst over config 1's 1000
 *              spectra).  The corrected layers have RDN_F16F8's range and range guard (RDN_ERANGE);
 *              on the walk geometry a saturated tile NaNs the rest of its spectrum (its clamped values
 *              travel on in the carried rows), on the tile geometries the tile alone.
 *              One hybrid kernel: the plain layers, the whole left branch and its head
 *              on the RDN_F16 ping-pong engine, the corrected tail and the right head on the in-place
 *              tile.  The corrected layers are compiled in; rdn_get_correction_mask reads them back
 *              from a packed blob.
 * RDN_F16 / RDN_F16MIX launches that would occupy at most half the CUs with 640-row tiles (e.g. one
 * spectrum per call, evaulate.py:29-32) run on 256-row tiles (same arithmetic and, for RDN_F16MIX, the
 * same hybrid composition); the environment variable RDN_SHORT_TILES=0/1 forces either.  Launches large
 * enough to give every CU several spectra run RDN_F16 (DenoiseCNN, RRCDNet, DSDN, PIDN) and RDN_F16MIX
 * on the walk geometry instead: one workgroup walks a whole spectrum with time-skewed layers and no
 * halo recompute (same per-output arithmetic; RDN_WALK=0/1 forces either). */
typedef enum { RDN_F32 = 0, RDN_BF16 = 1, RDN_BF16X3 = 2, RDN_F16F8 = 3, RDN_F16 = 4, RDN_F16MIX = 5 } rdn_dtype;

enum {
  RDN_OK = 0,
  RDN_EINVAL = -1,       /* bad argument (null pointer, unknown arch/dtype, n or L < 1)      */
  RDN_EUNSUPPORTED = -2, /* combination not built                                            */
  RDN_ESHAPE = -3,       /* a tensor handed to rdn_pack has the wrong number of elements      */
  RDN_ESIZE = -4,        /* destination / workspace buffer too small                          */
  RDN_EHIP = -5,         /* a HIP runtime call failed (message carries hipGetErrorString)     */
  RDN_ERANGE = -6        /* rdn_forward_status: an RDN_F16F8 / RDN_F16MIX activation left the
                            e4m3 planes' range; the affected tiles' outputs are NaN          */
};

/* ABI version (RDN_ABI_VERSION) of the loaded library. */
int rdn_version(void);

/* Build stamp: sha256 prefix of the sources this library was compiled from (csrc/Makefile). */
const char* rdn_build_id(void);

/* Message of the last failing call on this thread ("" if none). */
const char* rdn_last_error(void);

/* The reference state_dict keys rdn_pack consumes, in order, '\n'-separated, NUL-terminated.
 * Writes at most `cap` bytes to `buf` (may be NULL with cap 0); `*needed` receives the size. */
int rdn_param_names(int arch, char* buf, size_t cap, size_t* needed);

/* Bytes of the packed weight blob for (arch, dtype). */
int rdn_packed_size(int arch, int dtype, size_t* bytes);

/* Fold eval-mode BatchNorm (eps 1e-5) into the preceding Conv1d (in fp64) and lay every layer out
 * as MFMA operand fragments.  `tensors[i]` is a HOST fp32 pointer to the tensor named by line i
 * of rdn_param_names (row-major, torch layout), `numels[i]` its element count.  Writes the blob
 * into host memory `dst` (cap bytes); the caller copies it to the device. */
int rdn_pack(int arch, int dtype, const float* const* tensors, const int64_t* numels, int n_tensors,
             void* dst, size_t cap);

/* Blob layout tag: rdn_pack writes RDN_BLOB_MAGIC | arch << 8 | dtype into a word of the small
 * section, and rdn_check_blob verifies that a host blob was packed for (arch, dtype) and is at
 * least rdn_packed_size bytes.  The blob layouts differ per dtype (e.g. an RDN_F16MIX blob holds one
 * more record than an RDN_F16F8 one): rdn_forward needs a blob packed for the same (arch, dtype).
 * The RDN_F16MIX kernels also check the tag on the device and write NaN outputs on a mismatch. */
#define RDN_BLOB_MAGIC 0x52440000u
int rdn_check_blob(int arch, int dtype, const void* host_blob, size_t bytes);

/* Per-layer correction mask (bit i = big layer i, execution order of rdn_param_names' convs, runs
 * the e4m3 correction).  default: the RDN_F16MIX pattern of `arch` (0 = plain RDN_F16 already meets
 * 2e-2 there, and RDN_F16MIX is not built); get: read back from a packed RDN_F16F8 (all ones) or
 * RDN_F16MIX host blob. */
int rdn_default_correction_mask(int arch, uint64_t* mask);
int rdn_get_correction_mask(int arch, int dtype, const void* host_blob, size_t bytes, uint64_t* mask);

/* Device scratch rdn_forward takes for a batch on the device of `stream`: the CBAM networks' team
 * geometry (depends on the device's CU count and occupancy; required); every 16-bit dtype on the fused
 * networks 256 bytes whose first 4 bytes are the status word (optional; ABI v5), 0 otherwise (RDN_F32).
 * Status word bits, sticky until read: RDN_STATUS_RANGE an RDN_F16F8 / RDN_F16MIX activation left the
 * e4m3 planes' range (the tile's outputs are NaN; rdn_forward_status returns RDN_ERANGE);
 * RDN_STATUS_GATE an input value left [-4, 4], the 16-bit modes' domain (normalised intensity: every
 * simulated spectrum lies in [-1, 2]) -- set by the kernels' stems, which read every input anyway;
 * informational (rdn_forward_status does not fail on it; rdn_forward_status_ex reports it): the Python
 * module reads the word once per call and re-runs such a batch in RDN_F32.  Without the workspace a
 * saturated tile still writes NaN, but neither bit is reported.  The CBAM networks' workspaces hold the
 * same information in words of their own (the team kernels' and segment kernels' stems raise the gate
 * there too, ABI v6); read it with rdn_forward_status_ex. */
#define RDN_STATUS_RANGE 1u
#define RDN_STATUS_GATE 2u
#define RDN_STATUS_TIMEOUT 4u   /* rdn_forward_status_ex only: a CBAM team hand-off timed out */
int rdn_workspace_size(int arch, int dtype, int64_t n, int64_t L, size_t* bytes, void* stream);

/* Prepare a newly allocated workspace for rdn_forward on `stream`: clears its status words -- the
 * CBAM hand-off error word and the range word (both sticky across forwards until rdn_forward_status
 * reads and clears them, so one status call after many forwards that share a workspace covers all
 * of them). */
int rdn_workspace_init(int arch, int dtype, int64_t n, int64_t L, void* workspace, size_t workspace_bytes,
                       void* stream);

/* y[n][L] = Model(x[n][L]) on the device.  x, y: fp32 device pointers (the (N,1,L) tensor is
 * (N,L) contiguous) that must not overlap (RDN_EINVAL: tiles re-read input halos while outputs are
 * written); packed: device copy of the rdn_pack blob; stream: hipStream_t or NULL.  n = 0 launches
 * nothing and returns RDN_OK; x and y may then be NULL (every entry point below that takes a batch
 * accepts NULL data pointers for n = 0 the same way). */
int rdn_forward(int arch, int dtype, const void* packed, const float* x, float* y, int64_t n, int64_t L,
                void* workspace, size_t workspace_bytes, void* stream);

/* Completion status of every rdn_forward enqueued on `stream` with this workspace since the last
 * status call (or rdn_workspace_init): waits for the stream (hipStreamSynchronize), then reads and
 * clears the workspace's sticky status words (the fused networks' word: cleared on `stream`).  RDN_EHIP if a CBAM team wait timed out (co-residency
 * broken by a concurrent kernel; the affected spectra's outputs are NaN) or the stream reported an
 * error; RDN_ERANGE if an RDN_F16F8 / RDN_F16MIX activation left the e4m3 planes' range (NaN tiles;
 * for the CBAM networks the CBAM statistics of the saturated tile also reached the rest of its
 * spectrum, so the status word, not the NaN, is the authoritative signal); RDN_ESIZE if the workspace
 * is smaller than this device's team geometry needs; RDN_OK otherwise.  Replaces nothing in the
 * reference (its forward is synchronous PyTorch): the Python module calls it after each
 * range-checked or CBAM forward (and re-runs a saturated batch in RDN_F32), the batched evaluate
 * drivers once at the end. */
int rdn_forward_status(int arch, int dtype, int64_t n, int64_t L, void* workspace, size_t workspace_bytes,
                       void* stream);
/* rdn_forward_status that also reports WHICH status words were set (ABI v6): *flags (may be NULL)
 * receives RDN_STATUS_RANGE | RDN_STATUS_GATE | RDN_STATUS_TIMEOUT as read before the words were
 * cleared, so a caller learns of the input gate (informational: no error code) without reading the
 * workspace itself.  rdn_forward_status clears the same words and drops the gate bit: a C caller that
 * needs it calls this form.  Every network keeps the gate: the fused networks' status word, and the
 * CBAM networks' team / segment workspaces (their stems raise it, ABI v6). */
int rdn_forward_status_ex(int arch, int dtype, int64_t n, int64_t L, void* workspace, size_t workspace_bytes,
                          void* stream, unsigned* flags);

/* rdn_forward followed by rdn_metrics_ex(y, clean, ...) on the same stream (ABI v6): y = Model(x), then
 * each spectrum's MSE, SSIM, Smoothness and Peak2Peak against clean (fp32 or fp64 [n][L], device) into
 * per_spectrum / sums / acc (each may be NULL; sums and acc ACCUMULATED, as rdn_metrics_ex).  Where the
 * forward runs on the walk geometry (RDN_F16 on DenoiseCNN / RRCDNet / DSDN / PIDN, RDN_F16MIX on
 * RRCDNet, large batches) the forward kernel computes them itself -- each spectrum's workgroup right
 * after its walk, from the y rows it just wrote (read back from L2) -- so the separate metrics pass over
 * y is gone; *fused (may be NULL) is then 1.  Otherwise the metrics kernel follows the forward (*fused
 * = 0).  Both paths give every spectrum the same bits (one shared fp64 routine).  L must be >= 7. */
int rdn_forward_metrics(int arch, int dtype, const void* packed, const float* x, float* y, int64_t n, int64_t L,
                        const void* clean, int clean_is_f64, double* per_spectrum, double* sums, int64_t* acc,
                        void* workspace, size_t workspace_bytes, void* stream, int* fused);
/* Simulator parameters; defaults of 数据集产生.py:5-7 are {10000, 20, 37, 0.05, 40}. */
typedef struct {
  int64_t signal_length;
  float snr_lo;
  float snr_hi;
  float extreme_noise_prob;
  int32_t max_repeat;
} rdn_gen_params;

/* Generate spectra first_index .. first_index+n-1 of the stream `seed` (counter-based Philox,
 * so any index range is reproducible on any device).  clean/noisy: fp32 [n][L] device;
 * snr_db / noise_std: fp32 [n] device (either may be NULL). */
int rdn_generate(uint64_t seed, uint64_t first_index, int64_t n, const rdn_gen_params* params,
                 float* clean, float* noisy, float* snr_db, float* noise_std, void* stream);

/* Per-spectrum MSE, SSIM, Smoothness, Peak2Peak of denoised y against clean (both fp32 [n][L],
 * device), computed in fp64.  per_spectrum: fp64 [n][4] device (may be NULL).  sums: fp64 [5]
 * device, ACCUMULATED (+=) as {ΣMSE, ΣSSIM, ΣSmoothness, ΣPeak2Peak, count} (may be NULL).
 * L must be >= 7 (SSIM window). */
int rdn_metrics(const float* y, const float* clean, int64_t n, int64_t L, double* per_spectrum,
                double* sums, void* stream);

/* Exact metric accumulator: RDN_ACC_WORDS int64 on the device.  Metric k (MSE, SSIM, Smoothness,
 * Peak2Peak) owns words [k * RDN_ACC_STRIDE, ...): RDN_ACC_LIMBS limbs, limb j holding the sum of the
 * spectra's 32-bit chunks of weight 2^(32 j - RDN_ACC_FRAC_BITS) (values truncated toward zero below
 * 2^-128), then a count of values that were non-finite or >= 2^64 in magnitude; word RDN_ACC_COUNT
 * counts spectra.  Integer addition is associative, so the accumulated bits do not depend on the
 * batch split, the atomics' order or the number of ranks whose accumulators are summed (all-reduce
 * SUM over int64), for up to 2^31 spectra per accumulator. */
#define RDN_ACC_LIMBS 6
#define RDN_ACC_FRAC_BITS 128
#define RDN_ACC_STRIDE (RDN_ACC_LIMBS + 1)
#define RDN_ACC_COUNT (4 * RDN_ACC_STRIDE)
#define RDN_ACC_WORDS (RDN_ACC_COUNT + 1)

/* rdn_metrics with the clean reference in fp32 (clean_is_f64 = 0) or fp64 (1, e.g. a test.npz as
 * the reference loads it), and an optional exact accumulator `acc` (device, RDN_ACC_WORDS int64,
 * ACCUMULATED).  per_spectrum, sums and acc may each be NULL. */
int rdn_metrics_ex(const float* y, const void* clean, int clean_is_f64, int64_t n, int64_t L, double* per_spectrum,
                   double* sums, int64_t* acc, void* stream);

/* Host: {ΣMSE, ΣSSIM, ΣSmoothness, ΣPeak2Peak, count} from a HOST copy of an exact accumulator, each
 * sum the exact accumulated value rounded once to the nearest double (NaN for a metric with an
 * out-of-range value). */
int rdn_acc_value(const int64_t* acc, double* sums);

#ifdef __cplusplus
}
#endif

#endif /* RAMAN_MI355X_H */
