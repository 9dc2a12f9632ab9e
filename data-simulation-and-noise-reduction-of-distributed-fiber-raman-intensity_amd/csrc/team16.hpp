// Team-persistent CBAM forward on the f16 ping-pong engine (RDN_F16 on ADSDN / APIDN), included by
// cbam.hip once per engine geometry:
//   T16_ENG     the fused16.hpp instantiation (namespace) whose tiles / convs it runs
//   T16_NS      namespace of this instantiation's team code
//   T16_KERNEL  kernel name
//   T16_MINW    __launch_bounds__ minimum waves per SIMD (2 for the 4-wave, 2-workgroups-per-CU form)
// Needs cb:: (TeamArgs, Stamps, TEAM_HALO, EDGE_ROWS, f2ord / ord2f, sigm, quarter_sum, RES_*).
// ---- team-persistent forward on the ping-pong engine (RDN_F16) ------------------------------------
//
// The same team protocol as team_forward (statistics + edge rows published per tile, one counter
// barrier per CBAM, deterministic slot reduction, spin limit -> error word), with the convs on the
// f16 ping-pong engine of fused16.hpp: 640-row tiles (T = 628 own positions, TEAM_HALO = 6 per
// side: 16 tiles per spectrum at L = 10,000), two 80 KiB activation buffers, one barrier per conv.
// Every CBAM's input u ends in BUF0; BUF1 is free during the CBAM and holds its scratch.  The
// ResidualBlock identity (the block input, which conv2 overwrites in BUF0) is saved by conv2's
// epilogue (fused16.hpp LINEAR_SAVE) into 10 x 8 f16 per lane, in that epilogue's (row, slot)
// layout, which every pointwise pass of the CBAM below uses: lane (w, q, c16) owns rows
// 160 (w % 4) + 16 n + c16 (n < 10) at 16-B slot 4 (w / 4) + q, i.e. channels h16_channel(slot, j).
// Statistics in fp32 per lane, fp64 across waves and tiles; ca / sa in fp32; u, h and the identity
// are f16 (the mode's storage).  ADSDN/train.py:72-167, APIDN/train.py:72-159.
namespace T16_NS {
using V = T16_ENG::V;
constexpr int WB16 = T16_ENG::WB;
constexpr int NT = T16_ENG::NT;
constexpr int EDGE16_BYTES = EDGE_ROWS * T16_ENG::ROWB;        // one edge, f16 rows
// RDN_T16_TAGGED (default): the hand-off carries its own completion -- every 4-byte word of a slot
// travels as an 8-byte granule {word, tag} written by one sc1 store (tag = the CBAM's sequence
// number + 1; the slots are zeroed before each launch), and a consumer polls the granules it needs
// until every tag is current.  The producer neither drains its stores nor meets a counter, and the
// consumer's poll IS its read (one memory round trip after the last producer's stores land instead
// of drain + counter add + counter poll + slot loads: MI355X_MICROARCH.md handoff-1to1 vs
// handoff-flag).  Slot = 64 channel sums (f32: each tile's sum of its fp32 lane partials, rounded
// once) | 64 ordered maxima | 2 x EDGE_ROWS rows of u (f16) as 4-byte words.
#ifndef RDN_T16_TAGGED
#define RDN_T16_TAGGED 1
#endif
constexpr int G_SUM = 0, G_MAX = 64, G_EDGE = 128;               // granule indices within a slot
constexpr bool RDN_T16_TAGGED_ON = RDN_T16_TAGGED;
// RDN_T16_SA_LOCAL=1: per-wave conv7 with recomputed halo rows instead of a separate pass (one
// barrier fewer): measured 0.4 % (ADSDN) / 2 % (APIDN) SLOWER with the tagged hand-off (the extra
// 16-lane group and the wave-serial conv7 cost more than the barrier), so off
#ifndef RDN_T16_SA_LOCAL
#define RDN_T16_SA_LOCAL 0
#endif
constexpr int EDGE16_WORDS = EDGE16_BYTES / 4;                   // 160 per edge
#if RDN_T16_TAGGED
constexpr int SLOT16_BYTES = (G_EDGE + 2 * EDGE16_WORDS) * 8;    // 448 granules = 3584 B
#else
constexpr int SLOT16_BYTES = STAT_BYTES + 2 * EDGE16_BYTES;
#endif
// CBAM scratch in BUF1
constexpr int SC = T16_ENG::BUF1;
constexpr int RED16_OFF = SC;                                  // [4 row blocks][64] f32 sums, then u32 maxima
constexpr int SLP_OFF = RED16_OFF + 2 * 4 * 64 * 4;            // [8 waves][64] f64 slot partials, then u32
constexpr int POOL_OFF = SLP_OFF + 8 * 64 * 12;                // [2][64] f64: pooled avg / max
constexpr int CA16_OFF = POOL_OFF + 2 * 64 * 8;                // channel attention, one copy per wave (8 x 64 f32)
constexpr int SA16_OFF = CA16_OFF + 8 * 64 * 4;                // spatial attention per tile row
constexpr int M1_OFF = SA16_OFF + WB16 * 4;                    // [mean_c; max_c] map, rows -3 .. WB + 2
constexpr int M2_OFF = M1_OFF + (WB16 + 8) * 4;
constexpr int VOTE16_OFF = M2_OFF + (WB16 + 8) * 4;           // [2][8] u32 workgroup votes (wg_all)
static_assert(VOTE16_OFF + 2 * 8 * 4 <= (int)T16_ENG::LDS_BYTES, "CBAM scratch fits BUF1");

// Workgroup-wide AND of a per-thread predicate: a wave ballot, one LDS word per wave (two parity
// sets, so a vote needs one barrier), read back by every thread.  (__syncthreads_and would declare
// static LDS, which a kernel holding all 160 KiB dynamically cannot have.)
__device__ __forceinline__ bool wg_all(char* lds, bool v, unsigned& parity) {
  unsigned* vote = (unsigned*)(lds + VOTE16_OFF) + 8 * (parity & 1);
  const bool wave_ok = __builtin_amdgcn_ballot_w64(v) == ~0ull;
  if ((T16_ENG::tid() & 63) == 0) vote[T16_ENG::tid() >> 6] = wave_ok ? 1u : 0u;
  __syncthreads();
  bool all = true;
#pragma unroll
  for (int k = 0; k < T16_ENG::WAVES; ++k) all = all && vote[k] != 0;
  ++parity;
  return all;
}

struct Lane {             // this lane's (row, slot) items of the pointwise passes
  int w, h, rb, q, c16;
  __device__ __forceinline__ Lane() {
    const int t = T16_ENG::tid();
    w = __builtin_amdgcn_readfirstlane(t >> 6);
    h = w / T16_ENG::RB;
    rb = w % T16_ENG::RB;
    q = (t & 63) >> 4;
    c16 = t & 15;
  }
  __device__ __forceinline__ int row(int n) const { return rb * T16_ENG::RW + 16 * n + c16; }
  __device__ __forceinline__ int slot() const { return 4 * h + q; }
};
// sum / max over the 16 lanes of a row by DPP (pair, quad, half-row mirror, row mirror): every lane
// of the row ends with the row's value, one VALU op per step
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float row_sum(float v) {
  v += dpp<0xB1>(v);
  v += dpp<0x4E>(v);
  v += dpp<0x141>(v);
  return v + dpp<0x140>(v);
}
__device__ __forceinline__ float row_max(float v) {
  v = fmaxf(v, dpp<0xB1>(v));
  v = fmaxf(v, dpp<0x4E>(v));
  v = fmaxf(v, dpp<0x141>(v));
  return fmaxf(v, dpp<0x140>(v));
}
// over lanes l, l ^ 16, l ^ 32, l ^ 48 (v_permlane32/16_swap)
__device__ __forceinline__ float quarter_max(float v) {
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  const float h = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(h), __float_as_uint(h), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

// per-channel sum / max of u (BUF0) over the tile's own positions and its edge rows -> slot (sc1);
// arrive at the team counter
__device__ __forceinline__ void publish16(const T16_ENG::Tile& tl, const TeamArgs& ta, char* slot, unsigned* ctr,
                                          bool arrive, const T16_ENG::ChanStats* pre, unsigned tag) {
  char* lds = tl.lds;
  const Lane ln;
  const int tid = T16_ENG::tid();
  const int H = ta.halo, T = ta.T;
  const int rend = H + min(T, tl.L - tl.base - H);
  // this lane's channel partials: accumulated by the conv that produced u (pre: its epilogue, from
  // the unrounded values), or from u in BUF0
  T16_ENG::f32x8 sm = (T16_ENG::f32x8)(0.f), mx = (T16_ENG::f32x8)(-INFINITY);
  if (pre) {
    sm = pre->sum;
    mx = pre->max;
  } else {
    const char* b0 = lds + T16_ENG::BUF0 + (ln.h ? tl.koff[2][1] : tl.koff[2][0]);
    V uv[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) uv[n] = *(const V*)(b0 + n * 16 * T16_ENG::ROWB);
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const int r = ln.row(n);
      if (r >= H && r < rend) {
        const T16_ENG::f32x8 u = __builtin_convertvector(uv[n], T16_ENG::f32x8);
        sm += u;
        mx = __builtin_elementwise_max(mx, u);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sm[j] = row_sum(sm[j]);
    mx[j] = row_max(mx[j]);
  }
  float* rs = (float*)(lds + RED16_OFF);
  unsigned* rm = (unsigned*)(lds + RED16_OFF + 4 * 64 * 4);
  if (ln.c16 == 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = h16_channel(ln.slot(), j);
      rs[ln.rb * 64 + c] = sm[j];
      rm[ln.rb * 64 + c] = f2ord(mx[j]);
    }
  }
  __syncthreads();
#if RDN_T16_TAGGED
  // one store phase, no drain, no arrival: the statistics (wave 0: granules {f32 sum, tag} and
  // {ordered max, tag}) and the edge rows (u, f16) for the neighbours (waves 1-2: two granules per
  // 16-B sc1 store): block 0 = rows [2H - 5, 2H) (the left neighbour's rows [WB - 5, WB)), block 1 =
  // rows [T, T + 5).  arrive = false (test knob) publishes nothing.
  if (!arrive) return;
  const __amdgpu_buffer_rsrc_t sr = __builtin_amdgcn_make_buffer_rsrc((void*)slot, 0, SLOT16_BYTES, 0x00020000);
  if (tid < 64) {
    const int c = tid;
    double sv = 0.0;
    unsigned m = 0;
#pragma unroll
    for (int k = 0; k < T16_ENG::RB; ++k) {
      sv += (double)rs[k * 64 + c];
      m = max(m, rm[k * 64 + c]);
    }
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    __builtin_amdgcn_raw_buffer_store_b64(u32x2{__float_as_uint((float)sv), tag}, sr, 8 * (G_SUM + c), 0, 16);
    __builtin_amdgcn_raw_buffer_store_b64(u32x2{m, tag}, sr, 8 * (G_MAX + c), 0, 16);
  } else if (tid < 64 + 2 * EDGE_ROWS * 8) {
    const int i = tid - 64, e = i / (EDGE_ROWS * 8), k = (i / 8) % EDGE_ROWS, g = i & 7;
    const int r = e == 0 ? 2 * H - EDGE_ROWS + k : T + k;
    const u32x4 v = *(const u32x4*)(lds + T16_ENG::BUF0 + T16_ENG::soff(r, g));
    const int g0 = G_EDGE + e * EDGE16_WORDS + (k * 8 + g) * 4;
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{v[0], tag, v[1], tag}, sr, 8 * g0, 0, 16);
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{v[2], tag, v[3], tag}, sr, 8 * g0 + 16, 0, 16);
  }
  (void)ctr;
#else
  // one store phase: the statistics (wave 0) and the edge rows (u, f16) for the neighbours (waves
  // 1-2): block 0 = rows [2H - 5, 2H) (the left neighbour's rows [WB - 5, WB)), block 1 = rows
  // [T, T + 5); every storing wave drains its stores, the workgroup barrier, then the arrival
  if (tid < 64) {
    const int c = tid;
    double sv = 0.0;
    unsigned m = 0;
#pragma unroll
    for (int k = 0; k < T16_ENG::RB; ++k) {
      sv += (double)rs[k * 64 + c];
      m = max(m, rm[k * 64 + c]);
    }
    __hip_atomic_store((double*)slot + c, sv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store((unsigned*)(slot + 512) + c, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else if (tid < 64 + 2 * EDGE_ROWS * 8) {
    const int i = tid - 64, e = i / (EDGE_ROWS * 8), k = (i / 8) % EDGE_ROWS, g = i & 7;
    const int r = e == 0 ? 2 * H - EDGE_ROWS + k : T + k;
    const __amdgpu_buffer_rsrc_t sr = __builtin_amdgcn_make_buffer_rsrc((void*)slot, 0, SLOT16_BYTES, 0x00020000);
    const u32x4 v = *(const u32x4*)(lds + T16_ENG::BUF0 + T16_ENG::soff(r, g));
    __builtin_amdgcn_raw_buffer_store_b128(v, sr, STAT_BYTES + e * EDGE16_BYTES + (k * 8 + g) * 16, 0, 16);
  }
  if (tid < 64 + 2 * EDGE_ROWS * 8) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0 && arrive) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  (void)tag;
#endif
}

// apply the CBAM whose statistics sit in the team's slots to u (BUF0): h = [identity +] u*ca*sa
// [then ReLU], written over u; idv: the identity (LINEAR_SAVE layout) for res != RES_NONE
__device__ __forceinline__ void apply16(const T16_ENG::Tile& tl, const TeamArgs& ta, const char* slots0, int cbam_slot,
                                        bool bias, int res, const V* idv, Stamps& st, unsigned tag) {
  char* lds = tl.lds;
  const Lane ln;
  const int tid = T16_ENG::tid(), lane = tid & 63, w = ln.w;
  const float* cw = tl.small + cbam_slot * SMALL_SLOT_FLOATS;      // fc.0.weight [4][64]
  const float* cw2 = cw + SMALL_SLOT_FLOATS;                       // fc.2.weight [64][4]
  const float* cmisc = cw2 + SMALL_SLOT_FLOATS;                    // fc.0.bias[4], fc.2.bias[64], sa.w[2][7], sa.b
  f32x4 w1v;                                                       // fc.0 column `lane` (4 hidden units)
#pragma unroll
  for (int j = 0; j < 4; ++j) w1v[j] = cw[j * 64 + lane];
  const f32x4 cw2v = *(const f32x4*)(cw2 + 4 * lane);
  const float b2 = bias ? cmisc[4 + lane] : 0.f;
  const __amdgpu_buffer_rsrc_t sr = __builtin_amdgcn_make_buffer_rsrc((void*)slots0, 0, ta.TT * SLOT16_BYTES, 0x00020000);

#if RDN_T16_TAGGED
  // the granules this thread needs, polled until every tag is `tag` (uniform loop: one workgroup
  // vote per round): the halo refresh (threads < 80: u of rows [0, 5) from the left neighbour's
  // block 1, rows [WB - 5, WB) from the right neighbour's block 0; first / last tile: no
  // neighbour) and the spectrum's per-channel sums / maxima from the TT slots (thread (c, part):
  // slots part + 8k), combined in a fixed order
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  const int edge_e = tid / (EDGE_ROWS * 8), edge_k = (tid / 8) % EDGE_ROWS, edge_g = tid & 7;
  int eoff = -1;
  if (tid < 2 * EDGE_ROWS * 8) {
    const int tile = (tl.base + ta.halo) / ta.T;
    const int nb = edge_e == 0 ? tile - 1 : tile + 1;
    if (nb >= 0 && nb < ta.TT)
      eoff = nb * SLOT16_BYTES + 8 * (G_EDGE + (1 - edge_e) * EDGE16_WORDS + (edge_k * 8 + edge_g) * 4);
  }
  u32x4 ea = {0u, 0u, 0u, 0u}, eb = {0u, 0u, 0u, 0u};
  bool edge_ok = eoff < 0;
  double* pool = (double*)(lds + POOL_OFF);
  {
    const int c = tid & 63, part = tid >> 6;
    constexpr int PER = 2, STEP = T16_ENG::WAVES * PER;
    const int nbatch = (ta.TT + STEP - 1) / STEP;
    double sp = 0.0;
    unsigned mp = 0;
    bool failed = false;
    unsigned vparity = 0;
    for (int b = 0; b < nbatch; ++b) {
      u32x2 sv[PER], mv[PER];
      bool ok[PER];
#pragma unroll
      for (int k = 0; k < PER; ++k) ok[k] = part + STEP * b + T16_ENG::WAVES * k >= ta.TT;
      for (unsigned it = 0;; ++it) {
#pragma unroll
        for (int k = 0; k < PER; ++k) {
          if (!ok[k]) {
            const int off = (part + STEP * b + T16_ENG::WAVES * k) * SLOT16_BYTES;
            sv[k] = __builtin_amdgcn_raw_buffer_load_b64(sr, off + 8 * (G_SUM + c), 0, 16);
            mv[k] = __builtin_amdgcn_raw_buffer_load_b64(sr, off + 8 * (G_MAX + c), 0, 16);
          }
        }
        if (b == 0 && !edge_ok) {
          ea = __builtin_amdgcn_raw_buffer_load_b128(sr, eoff, 0, 16);
          eb = __builtin_amdgcn_raw_buffer_load_b128(sr, eoff + 16, 0, 16);
        }
        bool mine = true;
#pragma unroll
        for (int k = 0; k < PER; ++k) {
          ok[k] = ok[k] || (sv[k][1] == tag && mv[k][1] == tag);
          mine = mine && ok[k];
        }
        if (b == 0) {
          edge_ok = edge_ok || (ea[1] == tag && ea[3] == tag && eb[1] == tag && eb[3] == tag);
          mine = mine && edge_ok;
        }
        if (wg_all(lds, mine, vparity)) break;
        // a wait that exceeds SPIN_LIMIT rounds (a team member never published: co-residency
        // broken) raises the error words; once they are up every wait falls through (NaN outputs)
        if (failed || it > SPIN_LIMIT) {
          if (tid == 0 && !failed) {
            __hip_atomic_store(ta.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(ta.err + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          failed = true;
          break;
        }
        if ((it & 63) == 63 &&
            !wg_all(lds, __hip_atomic_load(ta.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0, vparity)) {
          failed = true;
          break;
        }
        __builtin_amdgcn_s_sleep(RDN_TEAM_SLEEP);
      }
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        if (part + STEP * b + T16_ENG::WAVES * k < ta.TT) {
          sp += (double)__uint_as_float(sv[k][0]);
          mp = max(mp, mv[k][0]);
        }
      }
    }
    double* ps = (double*)(lds + SLP_OFF);
    unsigned* pm = (unsigned*)(lds + SLP_OFF + 8 * 64 * 8);
    ps[part * 64 + c] = sp;
    pm[part * 64 + c] = mp;
  }
  if (eoff >= 0) {
    const int r = edge_e == 0 ? edge_k : WB16 - EDGE_ROWS + edge_k;
    *(u32x4*)(lds + T16_ENG::BUF0 + T16_ENG::soff(r, edge_g)) = u32x4{ea[0], ea[2], eb[0], eb[2]};
  }
  __syncthreads();
#else
  // halo refresh, fetched first: u of rows [0, 5) from the left neighbour's block 1, rows
  // [WB - 5, WB) from the right neighbour's block 0 (first / last tile: no neighbour)
  const int edge_e = tid / (EDGE_ROWS * 8), edge_k = (tid / 8) % EDGE_ROWS, edge_g = tid & 7;
  bool has_edge = false;
  u32x4 edge_u = {0u, 0u, 0u, 0u};
  if (tid < 2 * EDGE_ROWS * 8) {
    const int tile = (tl.base + ta.halo) / ta.T;
    const int nb = edge_e == 0 ? tile - 1 : tile + 1;
    if (nb >= 0 && nb < ta.TT) {
      edge_u = __builtin_amdgcn_raw_buffer_load_b128(
          sr, nb * SLOT16_BYTES + STAT_BYTES + (1 - edge_e) * EDGE16_BYTES + (edge_k * 8 + edge_g) * 16, 0, 16);
      has_edge = true;
    }
  }
  // the spectrum's per-channel mean and max over the TT slots, combined in a fixed order
  double* pool = (double*)(lds + POOL_OFF);
  {
    const int c = tid & 63, part = tid >> 6;
    double sp = 0.0;
    unsigned mp = 0;
    constexpr int PER = 2;                 // 16 slots per batch (TT = 16 at L = 10,000)
    for (int t0 = part; t0 < ta.TT; t0 += T16_ENG::WAVES * PER) {
      typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
      u32x2 sv[PER];
      unsigned mv[PER];
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int t = t0 + T16_ENG::WAVES * k;
        const int off = (t < ta.TT ? t : 0) * SLOT16_BYTES;
        sv[k] = __builtin_amdgcn_raw_buffer_load_b64(sr, off + 8 * c, 0, 16);
        mv[k] = __builtin_amdgcn_raw_buffer_load_b32(sr, off + 512 + 4 * c, 0, 16);
      }
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        if (t0 + T16_ENG::WAVES * k < ta.TT) {
          sp += __builtin_bit_cast(double, sv[k]);
          mp = max(mp, mv[k]);
        }
      }
    }
    double* ps = (double*)(lds + SLP_OFF);
    unsigned* pm = (unsigned*)(lds + SLP_OFF + 8 * 64 * 8);
    ps[part * 64 + c] = sp;
    pm[part * 64 + c] = mp;
  }
  if (has_edge) {
    const int r = edge_e == 0 ? edge_k : WB16 - EDGE_ROWS + edge_k;
    *(u32x4*)(lds + T16_ENG::BUF0 + T16_ENG::soff(r, edge_g)) = edge_u;
  }
  __syncthreads();
#endif
  st(10);
  // channel attention, evaluated whole by every wave (no barrier): the pooled avg / max of channel
  // `lane` from the 8 partials in a fixed order, the 4 + 4 hidden units as sums over the 64 lanes
  float cav;
  {
    const double* ps = (const double*)(lds + SLP_OFF);
    const unsigned* pm = (const unsigned*)(lds + SLP_OFF + 8 * 64 * 8);
    double sum = 0.0;
    unsigned m = 0;
#pragma unroll
    for (int k = 0; k < T16_ENG::WAVES; ++k) {
      sum += ps[k * 64 + lane];
      m = max(m, pm[k * 64 + lane]);
    }
    const float pa = (float)(sum / (double)tl.L), px = ord2f(m);
    float oa = b2, om = b2;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float b1 = bias ? cmisc[j] : 0.f;
      const float ha = fmaxf(quarter_sum(row_sum(w1v[j] * pa)) + b1, 0.f);
      const float hm = fmaxf(quarter_sum(row_sum(w1v[j] * px)) + b1, 0.f);
      oa = fmaf(cw2v[j], ha, oa);
      om = fmaf(cw2v[j], hm, om);
    }
    cav = sigm(oa + om);
  }
  // this lane's 8 channels of ca through the wave's own LDS row (in-order within a wave)
  float* caw = (float*)(lds + CA16_OFF) + 64 * w;
  caw[lane] = cav;
  st(11);

  // spatial statistics of u*ca in packed f16 (the mode's storage precision: u is f16, ca rounds to
  // f16): wave w takes rows 80w .. 80w + 79, lane (q, c16) the rows 80w + c16 + 16k (k < 5) at
  // slots q and q + 4 (16 channels), the 4 quarters (all 64 channels) by lane swaps -- every row's
  // [mean; max] completes inside one wave; partial sums / maxima to f32
  char* b0 = lds + T16_ENG::BUF0 + (ln.h ? tl.koff[2][1] : tl.koff[2][0]);
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  V cah, cq0, cq4;           // ca of this lane's pointwise slot; of slots q and q + 4
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    cah[j] = (_Float16)caw[h16_channel(ln.slot(), j)];
    cq0[j] = (_Float16)caw[h16_channel(ln.q, j)];
    cq4[j] = (_Float16)caw[h16_channel(ln.q + 4, j)];
  }
  float* m1 = (float*)(lds + M1_OFF) + 3;      // [mean_c; max_c] of rows -3 .. WB + 2, zero outside
  float* m2 = (float*)(lds + M2_OFF) + 3;      // the tile and [0, L)
  constexpr int SROWS = WB16 / T16_ENG::WAVES;    // 80 rows per wave
  static_assert(SROWS % 16 == 0, "whole 16-row groups per wave");
#if RDN_T16_SA_LOCAL
  // RDN_T16_SA_LOCAL: each wave also forms [mean; max] of the 3 + 3 rows around its own
  // 80 (one extra 16-lane group, lanes c16 < 6; rows outside the tile are 0) and then runs the conv7
  // of its own rows from its own LDS writes (in order within a wave): no workgroup barrier and no
  // separate pass between the spatial statistics and sa.  A halo row is written by two waves with
  // the same value.
  float* sa = (float*)(lds + SA16_OFF);
  {
    constexpr int KG = SROWS / 16;
    auto srow = [&](int k) {                   // row of group k for this lane (k == KG: the halo group)
      return k < KG ? SROWS * w + ln.c16 + 16 * k
                    : (ln.c16 < 3 ? SROWS * w - 3 + ln.c16 : SROWS * w + SROWS + min(ln.c16, 5) - 3);
    };
    V ua[KG + 1], ub[KG + 1];
#pragma unroll
    for (int k = 0; k <= KG; ++k) {
      const int r = min(max(srow(k), 0), WB16 - 1);
      ua[k] = *(const V*)(lds + T16_ENG::BUF0 + T16_ENG::soff(r, ln.q));
      ub[k] = *(const V*)(lds + T16_ENG::BUF0 + T16_ENG::soff(r, ln.q + 4));
    }
#pragma unroll
    for (int k = 0; k <= KG; ++k) {
      const V va = ua[k] * cq0, vb = ub[k] * cq4;
      const V vs = va + vb, vm = __builtin_elementwise_max(va, vb);
      const h2 s2 = (__builtin_shufflevector(vs, vs, 0, 1) + __builtin_shufflevector(vs, vs, 2, 3)) +
                    (__builtin_shufflevector(vs, vs, 4, 5) + __builtin_shufflevector(vs, vs, 6, 7));
      const h2 x2 = __builtin_elementwise_max(
          __builtin_elementwise_max(__builtin_shufflevector(vm, vm, 0, 1), __builtin_shufflevector(vm, vm, 2, 3)),
          __builtin_elementwise_max(__builtin_shufflevector(vm, vm, 4, 5), __builtin_shufflevector(vm, vm, 6, 7)));
      const float sm = quarter_sum((float)s2[0] + (float)s2[1]);
      const float mx = quarter_max(fmaxf((float)x2[0], (float)x2[1]));
      if (ln.q == 0 && (k < KG || ln.c16 < 6)) {
        const int r = srow(k);
        const bool in = r >= 0 && r < WB16 && T16_ENG::in_range(tl.base + r, tl.L);
        m1[r] = in ? sm * (1.0f / 64.0f) : 0.f;
        m2[r] = in ? mx : 0.f;
      }
    }
    // sa = sigmoid(conv7([mean_c; max_c])) of this wave's rows
#pragma unroll
    for (int i = 0; i < (SROWS + 63) / 64; ++i) {
      const int j = lane + 64 * i;
      if (j < SROWS) {
        const int r = SROWS * w + j;
        float a = bias ? cmisc[82] : 0.f;
#pragma unroll
        for (int k = 0; k < 7; ++k) {
          a = fmaf(cmisc[68 + k], m1[r + k - 3], a);
          a = fmaf(cmisc[75 + k], m2[r + k - 3], a);
        }
        sa[r] = sigm(a);
      }
    }
  }
  __syncthreads();
  st(12);
#else
  {
    V ua[SROWS / 16], ub[SROWS / 16];
#pragma unroll
    for (int k = 0; k < SROWS / 16; ++k) {
      const int r = SROWS * w + ln.c16 + 16 * k;
      ua[k] = *(const V*)(lds + T16_ENG::BUF0 + T16_ENG::soff(r, ln.q));
      ub[k] = *(const V*)(lds + T16_ENG::BUF0 + T16_ENG::soff(r, ln.q + 4));
    }
#pragma unroll
    for (int k = 0; k < SROWS / 16; ++k) {
      const V va = ua[k] * cq0, vb = ub[k] * cq4;
      const V vs = va + vb, vm = __builtin_elementwise_max(va, vb);
      const h2 s2 = (__builtin_shufflevector(vs, vs, 0, 1) + __builtin_shufflevector(vs, vs, 2, 3)) +
                    (__builtin_shufflevector(vs, vs, 4, 5) + __builtin_shufflevector(vs, vs, 6, 7));
      const h2 x2 = __builtin_elementwise_max(
          __builtin_elementwise_max(__builtin_shufflevector(vm, vm, 0, 1), __builtin_shufflevector(vm, vm, 2, 3)),
          __builtin_elementwise_max(__builtin_shufflevector(vm, vm, 4, 5), __builtin_shufflevector(vm, vm, 6, 7)));
      const float sm = quarter_sum((float)s2[0] + (float)s2[1]);
      const float mx = quarter_max(fmaxf((float)x2[0], (float)x2[1]));
      if (ln.q == 0) {
        const int r = SROWS * w + ln.c16 + 16 * k;
        const bool in = T16_ENG::in_range(tl.base + r, tl.L);
        m1[r] = in ? sm * (1.0f / 64.0f) : 0.f;
        m2[r] = in ? mx : 0.f;
      }
    }
    if (tid < 6) {                             // rows beyond the tile feed only halo rows: 0
      const int r = tid < 3 ? tid - 3 : WB16 + tid - 3;
      m1[r] = 0.f;
      m2[r] = 0.f;
    }
  }
  __syncthreads();
  st(12);
  // sa = sigmoid(conv7([mean_c; max_c]))
  float* sa = (float*)(lds + SA16_OFF);
  for (int r = tid; r < WB16; r += T16_ENG::THREADS) {
    float a = bias ? cmisc[82] : 0.f;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      a = fmaf(cmisc[68 + k], m1[r + k - 3], a);
      a = fmaf(cmisc[75 + k], m2[r + k - 3], a);
    }
    sa[r] = sigm(a);
  }
  __syncthreads();
  st(13);
#endif
  V uv[NT];
  // h = [identity +] u*ca*sa [relu], in place, packed f16; rows outside [0, L) zero
  float sv[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    uv[n] = *(const V*)(b0 + n * 16 * T16_ENG::ROWB);
    sv[n] = sa[ln.row(n)];
  }
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int r = ln.row(n);
    V* pu = (V*)(b0 + n * 16 * T16_ENG::ROWB);
    V hv = (uv[n] * cah) * (V)((_Float16)sv[n]);
    if (res != RES_NONE) {
      hv += idv[n];
      if (res == RES_ADD_RELU) hv = __builtin_elementwise_max(hv, (V)((_Float16)0));
    }
    if (!T16_ENG::in_range(tl.base + r, tl.L)) hv = (V)((_Float16)0);
    *pu = hv;
  }
  __syncthreads();
}

template <bool ADS, bool EDGE>
__device__ __forceinline__ void team16_spectra(char* lds, const uint8_t* blob, const uint8_t* big16, const float* x,
                                               float* y, int L, const TeamArgs& ta, int team, int tile) {
  unsigned* ctr = ta.counters + (size_t)team * TEAM_CTR_STRIDE;
  char* tslots = ta.slots + (size_t)team * 2 * ta.TT * SLOT16_BYTES;
  unsigned nbar = 0;
  Stamps st;
  st.init();
  for (int64_t n = team; n < ta.n; n += ta.teams) {
    T16_ENG::Tile tl = T16_ENG::init_tile(lds, blob, big16, x + (size_t)n * L, L, tile * ta.T - ta.halo);
    T16_ENG::Frags F0, F1;
    V id[NT];
    T16_ENG::ChanStats cs;
    auto conv2_stats = [&]() -> T16_ENG::ChanStats* {   // the block's conv2 accumulates u's statistics
      cs.sum = (T16_ENG::f32x8)(0.f);
      cs.max = (T16_ENG::f32x8)(-INFINITY);
      cs.lo = ta.halo;
      cs.hi = ta.halo + min(ta.T, L - tl.base - ta.halo);
      return &cs;
    };
    auto cbam = [&](int slot, int res, const T16_ENG::ChanStats* pre) {
      char* mine = tslots + ((size_t)(nbar & 1) * ta.TT + tile) * SLOT16_BYTES;
      const bool skip = ta.force_miss > 0 && __builtin_amdgcn_workgroup_id_x() == 0 && nbar + 1 == (unsigned)ta.force_miss;
      st(1);
      publish16(tl, ta, mine, ctr, !skip, pre, nbar + 1);
      st(3);
#if !RDN_T16_TAGGED
      team_wait(ta, ctr, (nbar + 1) * (unsigned)ta.TT);
#endif
      st(4);
      apply16(tl, ta, tslots + (size_t)(nbar & 1) * ta.TT * SLOT16_BYTES, slot, ADS, res, id, st, nbar + 1);
      st(5);
      ++nbar;
    };
    T16_ENG::load_frags(tl, 0, F0);
    T16_ENG::stem(tl, 0, T16_ENG::BUF0);
    T16_ENG::lds_barrier();
    if (ADS) {
      // ADSDN/train.py:160-167: cbam(relu(conv_ds x)); relu(conv1); relu(conv2); cbam;
      // 15 x relu(cbam(bn2(conv2(relu(bn1(conv1 x))))) + x); conv_out
      cbam(2, RES_NONE, nullptr);
      T16_ENG::layer<T16_ENG::RELU, EDGE>(tl, T16_ENG::BUF0, T16_ENG::BUF1, 1, F0, F1);
      T16_ENG::layer<T16_ENG::RELU, EDGE>(tl, T16_ENG::BUF1, T16_ENG::BUF0, 1, F1, F0);
      cbam(5, RES_NONE, nullptr);
      for (int b = 0; b < 15; ++b) {
        T16_ENG::layer<T16_ENG::RELU, EDGE>(tl, T16_ENG::BUF0, T16_ENG::BUF1, 1, F0, F1);
        T16_ENG::layer<T16_ENG::LINEAR_SAVE, EDGE>(tl, T16_ENG::BUF1, T16_ENG::BUF0, 1, F1, F0, true, id, conv2_stats());
        cbam(8 + 3 * b, RES_ADD_RELU, &cs);
      }
    } else {
      // APIDN/train.py:150-159: h = relu(conv_ds x); 15 x x += cbam(bn(conv(relu(bn(conv x)))));
      // sigmoid(conv_out(x + h))
      for (int b = 0; b < 15; ++b) {
        T16_ENG::layer<T16_ENG::RELU, EDGE>(tl, T16_ENG::BUF0, T16_ENG::BUF1, 1, F0, F1);
        T16_ENG::layer<T16_ENG::LINEAR_SAVE, EDGE>(tl, T16_ENG::BUF1, T16_ENG::BUF0, 1, F1, F0, true, id, conv2_stats());
        cbam(2 + 3 * b, RES_ADD, &cs);
      }
      T16_ENG::stem<true>(tl, 0, T16_ENG::BUF0);       // + h, recomputed from x
      T16_ENG::lds_barrier();
    }
    float o[T16_ENG::HN];
    T16_ENG::head<EDGE>(tl, T16_ENG::BUF0, F0, F1, false, o);
    const bool failed = __hip_atomic_load(ta.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
#pragma unroll
    for (int k = 0; k < T16_ENG::HN; ++k) {
      if (!ADS) o[k] = sigm(o[k]);
      if (failed) o[k] = __uint_as_float(0x7fc00000u);     // quiet NaN: an incomplete CBAM hand-off
    }
    T16_ENG::store_out(tl, y, (int)n, o, ta.halo, ta.T);
    __syncthreads();                 // the next spectrum's stem overwrites the rows the head read
    st(6);
  }
  if (RDN_TEAM_STAMPS && __builtin_amdgcn_workitem_id_x() == 0 && ta.stamps)
    for (int k = 0; k < NSTAMP; ++k) ta.stamps[(size_t)__builtin_amdgcn_workgroup_id_x() * NSTAMP + k] = st.acc[k];
}
}  // namespace T16_NS

template <bool ADS>
__global__ __launch_bounds__(T16_ENG::THREADS, T16_MINW) void T16_KERNEL(const uint8_t* __restrict__ blob,
                                                                const uint8_t* __restrict__ big16,
                                                                const float* __restrict__ x, float* __restrict__ y,
                                                                int L, TeamArgs ta) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int team = __builtin_amdgcn_workgroup_id_x() / ta.TT, tile = __builtin_amdgcn_workgroup_id_x() - team * ta.TT;
  const int base = tile * ta.T - ta.halo;
  // a tile holds positions outside [0, L) for every spectrum or for none (one L per launch)
#if defined(RDN_ABLATE_ALLEDGE)          // diagnostic: every tile on the edge-tile code
  if (false) T16_NS::team16_spectra<ADS, false>(lds, blob, big16, x, y, L, ta, team, tile);
#else
  if (base >= 0 && base + T16_NS::WB16 <= L) T16_NS::team16_spectra<ADS, false>(lds, blob, big16, x, y, L, ta, team, tile);
#endif
  else T16_NS::team16_spectra<ADS, true>(lds, blob, big16, x, y, L, ta, team, tile);
}

