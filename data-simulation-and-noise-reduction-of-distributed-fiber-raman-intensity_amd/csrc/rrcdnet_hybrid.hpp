// (no include guard: included once per tile length, inside namespaces ip::hyb640 and ip::hyb256)
// RDN_F16MIX RRCDNet hybrid body, included by fused_inplace.hip once per tile length: PPNS names the
// ping-pong engine instantiation (fused16.hpp: h16x, 640 rows; h16xs, 256 rows) and HNBK the in-place
// tile's 128-row blocks (5 / 2) of the same length.
// The producer of the corrected tail (the layer before it, which writes the e4m3 planes) runs on the
// ping-pong engine with its outputs staged in VGPRs as the in-place tile's three planes and written
// after the layer's barrier: no in-place plain layer and no conversion pass (+1 %, bit-equal).

// the staged outputs of one ping-pong layer as the in-place H8 row planes: lane (w, q, c16) holds
// N-tile n's row (w % RB) * RW + 16 n + c16 at 16-B slot 4 (w / RB) + q -- the f16 slot, and the
// 8-B e4m3 (hi / 4) and e4m3 (lo * 2^9) slots of the same 8 channels (h16_channel order in every
// plane, inplace.hpp Op<MODE_H8>::sbyte)
struct H8Stage {
  f16x8 hi[PPNS::NT];
  uint32_t e_hi[PPNS::NT][2], e_lo[PPNS::NT][2];
  float amax = 0.f;              // range guard (inplace.hpp h8_track): merged into the tile's after the layer
  // valid: the row lies in [0, L); rows outside are written as zeros (write) and never tracked -- on
  // an edge tile the rows beyond L + 1 are computed from stale LDS rows (the ping-pong engine's idle
  // waves skip them), whose values are arbitrary and would raise a false range error
  __device__ __forceinline__ void put(int n, PPNS::f32x8 v, bool valid) {
    const PPNS::f32x8 t = valid ? v : (PPNS::f32x8)(0.f);
    h8_track<true>(amax, __builtin_shufflevector(t, t, 0, 1, 2, 3));
    h8_track<true>(amax, __builtin_shufflevector(t, t, 4, 5, 6, 7));
    const f32x4 a = h8_sat<true>(__builtin_shufflevector(v, v, 0, 1, 2, 3));
    const f32x4 b = h8_sat<true>(__builtin_shufflevector(v, v, 4, 5, 6, 7));
    const H8Split sa = h8_split(a), sb = h8_split(b);
    hi[n] = __builtin_shufflevector(sa.hi, sb.hi, 0, 1, 2, 3, 4, 5, 6, 7);
    e_hi[n][0] = sa.hi8;
    e_hi[n][1] = sb.hi8;
    e_lo[n][0] = sa.lo8;
    e_lo[n][1] = sb.lo8;
  }
  // after the layer's barrier (every read of its input done): rows outside [0, L) as zeros
  template <bool EDGE>
  __device__ __forceinline__ void write(char* lds, const PPNS::Tile& t) const {
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    const int tid = PPNS::tid(), w = tid >> 6, lane = tid & 63;
    const int g = 4 * (w / PPNS::RB) + (lane >> 4), r0 = (w % PPNS::RB) * PPNS::RW + (lane & 15);
#pragma unroll
    for (int n = 0; n < PPNS::NT; ++n) {
      const int r = r0 + 16 * n;
      const bool ok = !EDGE || in_range(t.base + r, t.L);
      *(f16x8*)(lds + off_f32(r, 16 * g)) = ok ? hi[n] : (f16x8)((_Float16)0);
      *(u32x2*)(lds + off_f32(r, 128 + 8 * g)) = ok ? u32x2{e_hi[n][0], e_hi[n][1]} : u32x2{0u, 0u};
      *(u32x2*)(lds + off_f32(r, 192 + 8 * g)) = ok ? u32x2{e_lo[n][0], e_lo[n][1]} : u32x2{0u, 0u};
    }
  }
};

// Diagnostic builds (tools/hyb_stamps.py, -DRDN_HYB_STAMPS=1): s_memtime at the phase boundaries of
// the hybrid body, summed over workgroups into the range workspace behind its status word (u64
// [1 + phase], [1 + HYB_PHASES] = workgroups).  In the product build every stamp compiles to nothing.
#ifndef RDN_HYB_STAMPS
#define RDN_HYB_STAMPS 0
#endif
constexpr int HYB_PHASES = 10;
struct HybStamps {
  unsigned long long t, acc[HYB_PHASES];
  __device__ __forceinline__ HybStamps() {
    if (RDN_HYB_STAMPS) {
      for (int k = 0; k < HYB_PHASES; ++k) acc[k] = 0;
      t = __builtin_amdgcn_s_memtime();
    }
  }
  __device__ __forceinline__ void operator()(int k) {
    if (RDN_HYB_STAMPS) {
      const unsigned long long n = __builtin_amdgcn_s_memtime();
      acc[k] += n - t;
      t = n;
    }
  }
  __device__ __forceinline__ void flush(unsigned* status) {
    if (RDN_HYB_STAMPS && status && __builtin_amdgcn_workitem_id_x() == 0) {
      unsigned long long* w = (unsigned long long*)status;
      for (int k = 0; k < HYB_PHASES; ++k) atomicAdd(w + 1 + k, acc[k]);
      atomicAdd(w + 1 + HYB_PHASES, 1ull);
    }
  }
};

// The ping-pong view of the same tile (rows [base, base + WB) of spectrum n).
__device__ __forceinline__ PPNS::Tile pp_tile(const Tile& tl) {
  return PPNS::init_tile(tl.lds, (const uint8_t*)tl.small, tl.big, tl.x, tl.L, tl.base);
}

// Returns false, having written nothing, when the tile's input window leaves [F16MIX_WIN_LO,
// F16MIX_WIN_HI] (common.hpp): the caller then runs the all-corrected body on the tile.
template <bool EDGE, int TAIL>
__device__ __forceinline__ bool rrcdnet_hybrid_body(Tile& tl, float* y, int n, int L, int T, unsigned* status) {
  constexpr int H = fused_halo(RRCDNET), NBK = HNBK, PP = 14 - TAIL;   // ping-pong layers of the right branch
  using HO = HeadOut<MODE_H8, NBK>;
  HybStamps st;
  PPNS::Tile t16 = pp_tile(tl);
  t16.status = tl.status;        // the right stem reads every x of the tile: the input gate
  PPNS::Frags F0, F1;            // alternating operand buffers (fused16.hpp layer)
  PPNS::load_frags(t16, 0, F0);
  const PPNS::StemX xr = PPNS::stem_load(t16);
  {
    // the stem tests its inputs against the window.  Every wave reads the x of ALL the tile's rows
    // (wave w computes channel slot w of rows lane + 64k), so each wave's ballot is already the
    // tile's vote: no LDS vote words and no second barrier (2.5k cycles per tile, tools/hyb_stamps.py)
    const bool out = PPNS::stem(t16, 0, PPNS::BUF0, xr, F16MIX_WIN_LO, F16MIX_WIN_HI);
    st(0);
    const bool spiked = __builtin_amdgcn_ballot_w64(out) != 0;
    // the stem's rows are complete before layer 0 reads them; on a spiked tile, before the fallback
    // body overwrites the LDS
    PPNS::lds_barrier();
    if (spiked) return false;
  }
  st(1);
  f32x4 id[16 * NBK / 4];
  LayerA<MODE_H8> a;
  // layers 0 .. PP - 1 plain, layer PP (the tail's producer) staged into the in-place planes
  for (int i = 0; i < PP / 2; ++i) {
    PPNS::layer<PPNS::RELU, EDGE>(t16, PPNS::BUF0, PPNS::BUF1, 1, F0, F1);
    PPNS::layer<PPNS::RELU, EDGE>(t16, PPNS::BUF1, PPNS::BUF0, 1, F1, F0);
  }
  st(2);
  {
    H8Stage stg;
    if constexpr (PP % 2 == 1) {
      PPNS::layer<PPNS::RELU, EDGE>(t16, PPNS::BUF0, PPNS::BUF1, 1, F0, F1);
      PPNS::layer<PPNS::STAGE, EDGE>(t16, PPNS::BUF1, PPNS::BUF0, 1, F1, F0, false, nullptr, nullptr, &stg);
    } else {
      PPNS::layer<PPNS::STAGE, EDGE>(t16, PPNS::BUF0, PPNS::BUF1, 1, F0, F1, false, nullptr, nullptr, &stg);
    }
    // the tail's operands, issued before the staged planes are written so that their latency hides
    // under the stores; then an LDS-only barrier (the first conv waits for its k-step's operands
    // alone, not for all 96 VGPRs of them as a __syncthreads would)
    load_layer_a<MODE_H8>(tl, PP + 1, a);
    stg.write<EDGE>(tl.lds, t16);
    tl.amax = fmaxf(tl.amax, stg.amax);
  }
  tl.layer = PP + 1;
  lds_barrier();
  st(3);
  // the last corrected layer prefetches the right head's record (its operands: a[0])
  const uint8_t* rhead = tl.big + (size_t)F16MIX_RHEAD_REC * BIG_BYTES_H8;
  for (int i = 0; i < TAIL; ++i)
    conv<MODE_H8, RELU, 1, EDGE, NBK, true, true, true>(tl, 1, id, a, true, i + 1 < TAIL ? nullptr : rhead);
  st(4);
  // the left stem's inputs, fetched now: their latency hides under the right head (whose operands
  // are in registers already: no vector-memory wait in it)
  const PPNS::StemX xl = PPNS::stem_load(t16);
  float rk[HO::ROWS];            // the right head's rows, kept over the left branch
  head_h8_mfma<NBK>(tl, a, rk);
  st(5);
  // left branch: layers 15-28 and the head on the ping-pong engine (f16 activations into the head,
  // whose weights carry their rounding residue: tools/head_fusion_emul.py puts this at 1.52e-2 on
  // trained RRCDNet against 1.44e-2 with the split head, the bar being 2e-2)
  t16.layer = 15;
  PPNS::load_frags(t16, 15, F0);
  // the left stem overwrites the rows the right head just read: an LDS-only barrier (a __syncthreads
  // would also wait for the vector-memory loads in flight: the left stem's x and F0)
  PPNS::lds_barrier();
  st(6);
  PPNS::stem(t16, 1, PPNS::BUF0, xl);
  PPNS::lds_barrier();
  st(7);
  for (int i = 0; i < 7; ++i) {  // left layers 15-28 (the one at 22 with d = 1)
    PPNS::layer<PPNS::RELU, EDGE>(t16, PPNS::BUF0, PPNS::BUF1, 2, F0, F1);
    PPNS::layer<PPNS::RELU, EDGE>(t16, PPNS::BUF1, PPNS::BUF0, 2 * i + 1 == 7 ? 1 : 2, F1, F0);
  }
  st(8);
  // the combine's inputs (x and the parked right-head rows of this lane's output rows), fetched
  // before the left head so that their latency hides under it
  float xv[HO::ROWS], rv[HO::ROWS];
#pragma unroll
  for (int k = 0; k < HO::ROWS; ++k) {
    const int p = tl.base + HO::row(k);
    xv[k] = in_range(p, L) ? tl.x[p] : 0.f;
    rv[k] = rk[k];
  }
  float l[PPNS::HN];
  PPNS::head<EDGE>(t16, PPNS::BUF0, F0, F1, false, l);
  // hand the left head's rows (ping-pong lane layout) to the right head's (HeadOut) through LDS
  // (BUF1: no longer read since layer 28's closing barrier), then y = x - (r + l)/2; the corrected
  // tail's range vote (one word per wave behind the rows) rides on the same barrier
  float* lrow = (float*)(tl.lds + PPNS::BUF1);
  if ((PPNS::tid() & 63) < PPNS::HEAD_LANES) {
#pragma unroll
    for (int k = 0; k < PPNS::HN; ++k) {
      const int j = PPNS::head_row(k);
      if (j < PPNS::WB) lrow[j] = l[k];
    }
  }
  range_vote_post(tl, PPNS::BUF1 + 4 * PPNS::WB);
  PPNS::lds_barrier();
  const bool sat = range_vote_read(tl, PPNS::BUF1 + 4 * PPNS::WB, status);
  float o[HO::ROWS];
#pragma unroll
  for (int k = 0; k < HO::ROWS; ++k)        // x - (r + l)/2, one rounding
    o[k] = (float)((double)xv[k] - ((double)rv[k] + (double)lrow[HO::row(k)]) * 0.5);
  if (sat) nan_rows(o);
  store_out<MODE_H8, NBK>(tl, y, n, o, H, T);
  st(9);
  st.flush(status);
  return true;
}

