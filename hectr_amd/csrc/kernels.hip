// kernels.hip - gfx950 kernels of the CKKS engine.
//
// NTT: negacyclic, psi merged into the twiddles, forward Cooley-Tukey
// (natural -> bit-reversed), inverse Gentleman-Sande (bit-reversed ->
// natural), the ordering of oracle/ckks_oracle.c:ntt_limb/intt_limb.  For a
// butterfly on local element j at distance t the twiddle is
//     tw[(base + j) >> (log2 t + 1)]
// with base = n for a whole-limb tile, n1 for a column tile of the n1 x n2
// decomposition and (n1 + row) * n2 for a row tile.  One workgroup owns one
// LDS tile; each round keeps 2^R elements per thread in registers for R
// radix-2 stages (R <= 4), so a 256-point sub-transform costs two LDS round
// trips.
//
// All other kernels are elementwise over (limb, coefficient) and stream HBM
// with one 8-byte word per lane, canonical residues in and out.
#include "gpqhe_internal.h"
#include "ntt_device.h"
#include "tables.h"

#include <type_traits>

#include <map>
#include <string.h>
#include <tuple>

#define TPB 256

static inline dim3 grid1(size_t n, unsigned tpb = TPB)
{
  return dim3((unsigned)((n + tpb - 1) / tpb));
}

__device__ __forceinline__ unsigned brev_dev(unsigned x, unsigned bits)
{
  return __brev(x) >> (32 - bits);
}


// ===========================================================================
// Live kernel statistics (gpqhe_prof_enable / gpqhe_prof_collect): HIP events
// around each launch on the engine stream.
// ===========================================================================
// kernel names as rocprofv3 reports them (template arguments <fwd>/<inv> stand
// for the INV flag), so bench.py can match its statistics to a PMC profile
static const char *kc_names[KC_COUNT] = {
  "ntt_whole_kernel<fwd>", "ntt_whole_kernel<inv>", "modup_kernel", "ks_inner_kernel", "tensor_kernel",
  "down_conv_kernel", "down_combine_kernel", "ks_cols_kernel", "ks_rows_kernel", "dn_cols_kernel", "dn_rows_kernel",
  "d2_rows_kernel", "ntt2_cols_kernel<fwd>", "ntt3_rows_kernel<fwd>", "ntt3_rows_kernel<inv>",
  "ntt2_cols_kernel<inv>", "ks_cols4_kernel", "ntt_small_kernel<fwd>", "ntt_small_kernel<inv>",
  "gemv_inner_kernel", "ksq_kernel<drop>", "ksq_kernel<keep>", "modup_small_kernel", "moddown_small_kernel",
  "gemv_win_kernel", "gemv_fbc_kernel", "gemv_fold_kernel", "gemv_c0_kernel"};

struct ProfEntry {
  int cls;
  hipEvent_t a, b;
  double bytes;
};
static bool g_prof = false;
static std::vector<ProfEntry> g_prof_entries;
static std::vector<hipEvent_t> g_ev_pool;

static hipEvent_t prof_event()
{
  if (!g_ev_pool.empty()) {
    hipEvent_t e = g_ev_pool.back();
    g_ev_pool.pop_back();
    return e;
  }
  hipEvent_t e;
  HIP_CHECK(hipEventCreate(&e));
  return e;
}

ProfScope::ProfScope(int c, double b) : cls(c), bytes(b)
{
  if (!g_prof)
    return;
  a = prof_event();
  HIP_CHECK(hipEventRecord(a, G.stream));
}

ProfScope::~ProfScope()
{
  if (!a)
    return;
  hipEvent_t b = prof_event();
  HIP_CHECK(hipEventRecord(b, G.stream));
  g_prof_entries.push_back({cls, a, b, bytes});
}

bool k_prof_on()
{
  return g_prof;
}

// hectx_exit: the timing events (pooled and still recorded)
void k_prof_release()
{
  for (const ProfEntry &e : g_prof_entries) {
    g_ev_pool.push_back(e.a);
    g_ev_pool.push_back(e.b);
  }
  g_prof_entries.clear();
  for (hipEvent_t e : g_ev_pool)
    HIP_CHECK(hipEventDestroy(e));
  g_ev_pool.clear();
}

extern "C" void gpqhe_prof_enable(int on)
{
  g_prof = on != 0;
}

extern "C" unsigned gpqhe_prof_collect(gpqhe_kstat_t *out, unsigned max)
{
  if (G.stream)
    HIP_CHECK(hipStreamSynchronize(G.stream));
  double us[KC_COUNT] = {0}, bytes[KC_COUNT] = {0};
  unsigned cnt[KC_COUNT] = {0};
  for (const ProfEntry &e : g_prof_entries) {
    float ms = 0;
    HIP_CHECK(hipEventElapsedTime(&ms, e.a, e.b));
    us[e.cls] += 1e3 * ms;
    bytes[e.cls] += e.bytes;
    cnt[e.cls]++;
    g_ev_pool.push_back(e.a);
    g_ev_pool.push_back(e.b);
  }
  g_prof_entries.clear();
  unsigned k = 0;
  for (int c = 0; c < KC_COUNT && k < max; c++) {
    if (!cnt[c])
      continue;
    memset(&out[k], 0, sizeof(out[k]));
    strncpy(out[k].name, kc_names[c], sizeof(out[k].name) - 1);
    out[k].launches = cnt[c];
    out[k].total_us = us[c];
    out[k].bytes = bytes[c];
    k++;
  }
  return k;
}

// ===========================================================================
// NTT rounds on an LDS tile.
// Tile: nsub sub-transforms of T = 2^logT points; element (sub, j) at
// lds[sub * SS + j * ES].  base(sub) = base0 + sub * bstep.
// ===========================================================================
// In one round a group holds elements b + k*tlo (k < E).  Stage s of the
// round uses the 2^s (forward) or 2^(R-1-s) (inverse) twiddles
//   tw[Bs + u],  Bs = (base + b_high) >> (log2 t + 1 + log2(u-range)),
// i.e. contiguous runs, so a radix-16 group loads exactly 15 twiddle pairs.
template <int LOGE, bool SUB_MAJOR>
__device__ __forceinline__ void fwd_round(uint64_t *lds, int nsub, int logT, int log_thi, int SS, int ES,
                                          uint64_t base0, uint64_t bstep, const uint64_t *__restrict__ tw,
                                          const uint64_t *__restrict__ twp, uint64_t q)
{
  constexpr int E = 1 << LOGE;
  const int log_tlo = log_thi - LOGE + 1;
  const int tlo = 1 << log_tlo;
  const int gps = (1 << logT) >> LOGE;  // groups per sub
  const int total = nsub * gps;
  for (int g = threadIdx.x; g < total; g += blockDim.x) {
    int sub, grp;
    if (SUB_MAJOR) {
      sub = g / gps;
      grp = g - sub * gps;
    } else {
      sub = g % nsub;
      grp = g / nsub;
    }
    const int bhi = (grp >> log_tlo) << (log_thi + 1);
    const int b = bhi | (grp & (tlo - 1));
    const uint64_t bb = base0 + (uint64_t)sub * bstep + (uint64_t)bhi;
    uint64_t W[E - 1], WP[E - 1];
#pragma unroll
    for (int s = 0; s < LOGE; s++) {
      const uint64_t Bs = bb >> (log_thi - s + 1);
#pragma unroll
      for (int u = 0; u < (1 << s); u++) {
        W[(1 << s) - 1 + u] = tw[Bs + u];
        WP[(1 << s) - 1 + u] = twp[Bs + u];
      }
    }
    uint64_t x[E];
#pragma unroll
    for (int k = 0; k < E; k++)
      x[k] = lds[sub * SS + (b + k * tlo) * ES];
#pragma unroll
    for (int s = 0; s < LOGE; s++) {
      const int half = E >> (s + 1);
#pragma unroll
      for (int k = 0; k < E; k++) {
        if (k & half)
          continue;
        const int wi = (1 << s) - 1 + (k >> (LOGE - s));
        const uint64_t U = x[k];
        const uint64_t V = mul_shoup(x[k + half], W[wi], WP[wi], q);
        x[k] = add_mod(U, V, q);
        x[k + half] = sub_mod(U, V, q);
      }
    }
#pragma unroll
    for (int k = 0; k < E; k++)
      lds[sub * SS + (b + k * tlo) * ES] = x[k];
  }
}

template <int LOGE, bool SUB_MAJOR>
__device__ __forceinline__ void inv_round(uint64_t *lds, int nsub, int logT, int log_tlo, int SS, int ES,
                                          uint64_t base0, uint64_t bstep, const uint64_t *__restrict__ tw,
                                          const uint64_t *__restrict__ twp, uint64_t q)
{
  constexpr int E = 1 << LOGE;
  const int log_thi = log_tlo + LOGE - 1;
  const int tlo = 1 << log_tlo;
  const int gps = (1 << logT) >> LOGE;
  const int total = nsub * gps;
  for (int g = threadIdx.x; g < total; g += blockDim.x) {
    int sub, grp;
    if (SUB_MAJOR) {
      sub = g / gps;
      grp = g - sub * gps;
    } else {
      sub = g % nsub;
      grp = g / nsub;
    }
    const int bhi = (grp >> log_tlo) << (log_thi + 1);
    const int b = bhi | (grp & (tlo - 1));
    const uint64_t bb = base0 + (uint64_t)sub * bstep + (uint64_t)bhi;
    // stage s uses 2^(LOGE-1-s) twiddles; slot offset = E - 2^(LOGE-s)
    uint64_t W[E - 1], WP[E - 1];
#pragma unroll
    for (int s = 0; s < LOGE; s++) {
      const uint64_t Bs = bb >> (log_tlo + s + 1);
#pragma unroll
      for (int u = 0; u < (1 << (LOGE - 1 - s)); u++) {
        W[E - (1 << (LOGE - s)) + u] = tw[Bs + u];
        WP[E - (1 << (LOGE - s)) + u] = twp[Bs + u];
      }
    }
    uint64_t x[E];
#pragma unroll
    for (int k = 0; k < E; k++)
      x[k] = lds[sub * SS + (b + k * tlo) * ES];
#pragma unroll
    for (int s = 0; s < LOGE; s++) {
      const int half = 1 << s;
#pragma unroll
      for (int k = 0; k < E; k++) {
        if (k & half)
          continue;
        const int wi = E - (1 << (LOGE - s)) + (k >> (s + 1));
        const uint64_t U = x[k], V = x[k + half];
        x[k] = add_mod(U, V, q);
        x[k + half] = mul_shoup(sub_mod(U, V, q), W[wi], WP[wi], q);
      }
    }
#pragma unroll
    for (int k = 0; k < E; k++)
      lds[sub * SS + (b + k * tlo) * ES] = x[k];
  }
}

// Forward: rounds from the largest distance down; first round takes the
// remainder so later rounds are full radix-16.
template <bool SUB_MAJOR>
__device__ __forceinline__ void tile_fwd(uint64_t *lds, int nsub, int logT, int SS, int ES, uint64_t base0, uint64_t bstep,
                         const uint64_t *tw, const uint64_t *twp, uint64_t q)
{
  int remaining = logT;
  int log_thi = logT - 1;
  int first = logT % 4 ? logT % 4 : 4;
  while (remaining > 0) {
    const int r = first;
    switch (r) {
    case 1: fwd_round<1, SUB_MAJOR>(lds, nsub, logT, log_thi, SS, ES, base0, bstep, tw, twp, q); break;
    case 2: fwd_round<2, SUB_MAJOR>(lds, nsub, logT, log_thi, SS, ES, base0, bstep, tw, twp, q); break;
    case 3: fwd_round<3, SUB_MAJOR>(lds, nsub, logT, log_thi, SS, ES, base0, bstep, tw, twp, q); break;
    default: fwd_round<4, SUB_MAJOR>(lds, nsub, logT, log_thi, SS, ES, base0, bstep, tw, twp, q); break;
    }
    __syncthreads();
    remaining -= r;
    log_thi -= r;
    first = 4;
  }
}

template <bool SUB_MAJOR>
__device__ __forceinline__ void tile_inv(uint64_t *lds, int nsub, int logT, int SS, int ES, uint64_t base0, uint64_t bstep,
                         const uint64_t *tw, const uint64_t *twp, uint64_t q)
{
  int log_tlo = 0;
  int remaining = logT;
  while (remaining > 0) {
    const int r = remaining >= 4 ? 4 : remaining;
    switch (r) {
    case 1: inv_round<1, SUB_MAJOR>(lds, nsub, logT, log_tlo, SS, ES, base0, bstep, tw, twp, q); break;
    case 2: inv_round<2, SUB_MAJOR>(lds, nsub, logT, log_tlo, SS, ES, base0, bstep, tw, twp, q); break;
    case 3: inv_round<3, SUB_MAJOR>(lds, nsub, logT, log_tlo, SS, ES, base0, bstep, tw, twp, q); break;
    default: inv_round<4, SUB_MAJOR>(lds, nsub, logT, log_tlo, SS, ES, base0, bstep, tw, twp, q); break;
    }
    __syncthreads();
    remaining -= r;
    log_tlo += r;
  }
}

// Whole limb in one LDS tile (n <= 4096: 32 KiB).  grid.y = limb.
template <bool inverse>
__global__ void __launch_bounds__(TPB) ntt_whole_kernel(LimbSet s, unsigned logn, DevTables t)
{
  extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
  const unsigned n = 1u << logn;
  const unsigned v = blockIdx.y;
  uint64_t *x = s.limb(v, logn);
  const unsigned m = s.mod(v);
  const ModConst mc = t.mc[m];
  for (unsigned i = threadIdx.x; i < n; i += blockDim.x)
    lds[i] = x[i];
  __syncthreads();
  if constexpr (!inverse) {
    tile_fwd<true>(lds, 1, logn, 0, 1, n, 0, t.tw + ((size_t)m << logn), t.twp + ((size_t)m << logn), mc.q);
    for (unsigned i = threadIdx.x; i < n; i += blockDim.x)
      x[i] = lds[i];
  } else {
    tile_inv<true>(lds, 1, logn, 0, 1, n, 0, t.itw + ((size_t)m << logn), t.itwp + ((size_t)m << logn), mc.q);
    for (unsigned i = threadIdx.x; i < n; i += blockDim.x)
      x[i] = mul_shoup(lds[i], mc.ninv, mc.ninvp, mc.q);
  }
}

template <int LOGT, bool INV>
__global__ void __launch_bounds__(256) ntt2_cols_kernel(LimbSet s, LimbSet o, unsigned logn, Tw2 tw,
                                                         const ModConst *mcs, const uint64_t *post)
{
  constexpr int T = 1 << LOGT, C = 4096 / T, CP = C + 1;
  __shared__ __attribute__((aligned(16))) uint64_t lds[T * CP];
  const unsigned n2 = 1u << (logn - LOGT);
  unsigned v, tile;
  pm_decode(s, n2 / C, v, tile);
  const unsigned m = s.mod(v);
  const ModConst mc = mcs[m];
  const uint64_t *x = s.limb(v, logn) + (size_t)tile * C;
  uint64_t *y = o.limb(v, logn) + (size_t)tile * C;
  // final scale of the inverse: n^-1, or a caller constant per limb slot (e.g.
  // n^-1 times the ModUp factor [(Q_j/q_i)^-1]_{q_i}, folded into the INTT)
  uint64_t sw = 0, swp = 0;
  if (INV) {
    sw = post ? post[2 * (v % s.per)] : mc.ninv;
    swp = post ? post[2 * (v % s.per) + 1] : mc.ninvp;
  }
  with_arith(mc.q, m, logn, tw, [&](const auto &ar) { cols_tile<LOGT, INV>(ar, x, y, n2, lds, sw, swp); });
}

template <int LOGN2, bool INV>
__global__ void __launch_bounds__(256) ntt3_rows_kernel(LimbSet s, LimbSet o, unsigned logn, Tw2 tw,
                                                         const ModConst *mcs)
{
  using T = Row8<LOGN2>;
  __shared__ __attribute__((aligned(16))) uint64_t lds[T::WORDS];
  const unsigned n1 = 1u << (logn - LOGN2);
  unsigned v, tile;
  pm_decode(s, n1 / T::R, v, tile);
  const unsigned m = s.mod(v);
  const uint64_t q = mcs[m].q;
  const unsigned row0 = tile * T::R;
  const uint64_t *x = s.limb(v, logn) + ((size_t)row0 << LOGN2);
  uint64_t *y = o.limb(v, logn) + ((size_t)row0 << LOGN2);
  with_arith(q, m, logn, tw, [&](const auto &ar) { rows8_tile<LOGN2, INV>(ar, x, y, lds, n1 + row0); });
}

// Row pass of the batched NTT: a workgroup owns (basis slot, row tile) and a
// range of polynomials; QN 256-thread quarters stream their own polys (the
// next one's words prefetched) and share the tile's twiddles staged once in
// LDS (RowTw; FP64 moduli forward and inverse from it, integer moduli the
// forward ones), instead of every tile re-fetching its 20 twiddle pairs per
// thread from L2.
// (launch bound: two workgroups per CU, 128 VGPRs; the inverse takes 8-byte
// twiddle entries (W8) to fit: with 16-byte ones it spilled 16 VGPRs, and at
// one workgroup per CU it ran slower still)
#ifndef NTT_ROWS_SQ
#define NTT_ROWS_SQ 1
#endif
// POST (inverse, DIN): every output word times the slot's constant post[2 slot]
// (Shoup companion post[2 slot + 1]), canonical -- the ModDown's n^-1
// [(D/d)^-1]_d on the dropped limbs before dn_cols' pre-scaled form
// (k_ntt_rows_down).
template <int LOGN2, bool INV, int QN, bool W8 = false, bool DIN = false, bool POST = false>
__global__ void __launch_bounds__(256 * QN, 2 * QN) ntt_rows_q_kernel(LimbSet s, LimbSet o, unsigned logn, Tw2 tw,
                                                             const ModConst *mcs, unsigned members,
                                                             const uint64_t *post)
{
  using T = Row8<LOGN2>;
  __shared__ __attribute__((aligned(16))) uint64_t rt[QN][T::WORDS];
  // (integer moduli stage 16-byte forward entries whatever W8 says)
  __shared__ __attribute__((aligned(16))) uint64_t rtw[2 * RowTw<LOGN2>::ENTRIES];
  const unsigned n1 = 1u << (logn - LOGN2), tiles = n1 / T::R, per = s.per, polys = s.count / per;
  unsigned grp, mi;  // group = (slot, tile); members = poly ranges
  if (!xcd_group(members, per * tiles, grp, mi))
    return;
  const unsigned pb0 = (unsigned)(((size_t)mi * polys) / members), pb1 = (unsigned)(((size_t)(mi + 1) * polys) / members);
  if (pb0 >= pb1)
    return;
  const unsigned slot = grp / tiles, tile = grp % tiles, m = s.mod(slot);
  const uint64_t q = mcs[m].q;
  const unsigned row0 = tile * T::R;
  const size_t toff = (size_t)row0 << LOGN2;
  // the poly stream is wave-uniform (scalar: SGPR stream bases, 32-bit lane
  // offsets, a pair loop without exec masks; as the split key switch's ksq)
  const int qi = NTT_ROWS_SQ ? (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 8) : (int)(threadIdx.x >> 8);
  const int th = threadIdx.x & 255, row = th / T::TA, l = th % T::TA;
  uint64_t *lq = rt[qi];
  auto fetch = [&](uint64_t (&w)[8], unsigned p) {
    const auto x = sgpr_ptr<NTT_ROWS_SQ>(s.limb(p * per + slot, logn) + toff);
    if constexpr (INV && DIN) {
      // the thread's round-C words 8 h + k of its row, 16-byte loads
      const auto v2 = (gptr<const u64x2>)(x + (unsigned)((row << LOGN2) + 8 * l));
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const u64x2 v = v2[i];
        w[2 * i] = v.x;
        w[2 * i + 1] = v.y;
      }
    } else {
#pragma unroll
      for (int k = 0; k < 8; k++)
        w[k] = INV ? x[(unsigned)((th & ~63) * 8 + (th & 63) + 64 * k)] : x[(unsigned)((row << LOGN2) + l + T::TA * k)];
    }
  };
  with_arith(q, m, logn, tw, [&](const auto &ar0) {
    using A0 = std::decay_t<decltype(ar0)>;
    constexpr bool F = std::is_same<A0, ArF64>::value;
    // FP64: (w, w/q) of this direction; integer: the forward (w, w') pairs
    if constexpr (W8 && F)
      RowTw<LOGN2>::template stage<true>(rtw, INV ? (const uint64_t *)ar0.itw : (const uint64_t *)ar0.tw, n1 + row0,
                                         threadIdx.x, 256 * QN);
    else
      RowTw<LOGN2>::stage(rtw, INV && F ? (const uint64_t *)ar0.itw : (const uint64_t *)ar0.tw, n1 + row0, threadIdx.x,
                          256 * QN);
    __syncthreads();
    const auto ar = [&] {
      if constexpr (F)
        return row_policy<LOGN2, W8>(ar0, rtw, (int64_t)T::R - (int64_t)(n1 + row0), INV ? rtw : nullptr);
      else
        return row_policy<LOGN2, false>(ar0, rtw, (int64_t)T::R - (int64_t)(n1 + row0));
    }();
    // POST: the slot's scale (FP64: as double with its quotient factor)
    uint64_t pw = 0, pwp = 0;
    double pqd = 0, pqi = 0, pwd = 0, pwq = 0;
    if constexpr (POST) {
      pw = post[2 * slot];
      pwp = post[2 * slot + 1];
      if constexpr (F) {
        pqd = (double)q;
        pqi = 1.0 / pqd;
        pwd = f64_from_u52(pw);
        pwq = pwd * pqi;
      }
    }
    unsigned p = pb0 + qi;
    uint64_t nx[8];
    if (p < pb1)
      fetch(nx, p);
    for (; p < pb1; p += QN) {
      uint64_t w[8];
#pragma unroll
      for (int k = 0; k < 8; k++)
        w[k] = nx[k];
      if (p + QN < pb1)
        fetch(nx, p + QN);
      wave_sync();
      if constexpr (INV && DIN) {
        using V = typename std::decay_t<decltype(ar)>::V;
        V r[8];
#pragma unroll
        for (int k = 0; k < 8; k++)
          r[k] = std::decay_t<decltype(ar)>::load(w[k]);
        rows8_inv<LOGN2>(r, lq, ar, n1 + row0, th);
        const auto y = sgpr_ptr<NTT_ROWS_SQ>(o.limb(p * per + slot, logn) + toff);
#pragma unroll
        for (int k = 0; k < 8; k++) {
          if constexpr (POST && F) {  // (constants hoisted out of the poly loop)
            y[(unsigned)((row << LOGN2) + l + T::TA * k)] =
                f64_canon(f64_mulmod(f64_from_u52(ar.canon(r[k])), pwd, pwq, pqd), pqd, pqi);
          } else if constexpr (POST) {
            y[(unsigned)((row << LOGN2) + l + T::TA * k)] = mul_shoup(ar.canon(r[k]), pw, pwp, q);
          } else {
            y[(unsigned)((row << LOGN2) + l + T::TA * k)] = ar.canon(r[k]);
          }
        }
      } else {
        rows8_tile_words<LOGN2, INV>(ar, w, sgpr_ptr<NTT_ROWS_SQ>(o.limb(p * per + slot, logn) + toff), lq, n1 + row0,
                                     th);
      }
    }
  });
}

// The row pass of the two-pass NTT (n = n1 x 2^LOGN2; ntt2_launch): the
// batched form when every slot has polys enough to share a workgroup's
// staged twiddles, else one tile per workgroup.
template <int LOGN2>
static bool ntt_rows_launch(bool inv, const LimbSet &in, const LimbSet &out, const uint64_t *post = nullptr)
{
  const unsigned logn = G.logn, n = G.n;
  const unsigned blocks = in.count * (n / 4096);
  const Tw2 tw{G.tw2, G.itw2, G.twd, G.itwd};
  constexpr int QN = 2;
  const unsigned polys = in.count / in.per, groups = in.per * (n / 2048);
  if (polys >= 4 * QN && in.per == out.per) {  // config 2: 7.75 -> 7.50 ms roundtrip
    // ~12 polys per quarter stream (two pair ranges per group of 48 polys:
    // one wave of workgroups): forward 86.6 -> 76.2, inverse 99 -> 96 us per
    // group against ~4 per quarter; ~24 (107 us inverse) and ~8 were slower,
    // and a second poly in flight (PF = 2) no faster
    const unsigned members = std::max(1u, polys / (12 * QN));
    // inverse: 8-byte staged twiddles (w only, quotient from the product):
    // 94 VGPRs, no spills (16-byte entries spilled 16 at this launch bound),
    // 107 -> 98 us per 48-poly group; the forward pass measured 86 -> 88 us
    // with them and keeps 16-byte (w, w/q) entries
    // inverse: each thread loads its round-C words directly (16-byte loads,
    // no transpose through LDS): 94.6 -> 88.4-90.5 us per 48-poly group
    auto k = inv ? (post ? ntt_rows_q_kernel<LOGN2, true, QN, true, true, true> : ntt_rows_q_kernel<LOGN2, true, QN, true, true>)
                 : ntt_rows_q_kernel<LOGN2, false, QN>;
    hipLaunchKernelGGL(k, dim3(xcd_blocks(members, groups)), dim3(256 * QN), 0, G.stream, in, out, logn, tw, G.dev.mc,
                       members, post);
  } else if (post) {
    return false;  // (the batched form only)
  } else if (inv) {
    hipLaunchKernelGGL((ntt3_rows_kernel<LOGN2, true>), dim3(2 * blocks), dim3(256), 0, G.stream, in, out, logn, tw,
                       G.dev.mc);
  } else {
    hipLaunchKernelGGL((ntt3_rows_kernel<LOGN2, false>), dim3(2 * blocks), dim3(256), 0, G.stream, in, out, logn, tw,
                       G.dev.mc);
  }
  return true;
}

template <int LOGT1, int LOGN2>
static void ntt2_launch(const LimbSet &s, const LimbSet &o, bool inverse, const uint64_t *post)
{
  const unsigned logn = G.logn, n = G.n;
  const unsigned blocks = s.count * (n / 4096);
  const Tw2 tw{G.tw2, G.itw2, G.twd, G.itwd};
  const double pass_bytes = 16.0 * n * s.count;
  // row pass: ntt_rows_q_kernel when every slot has polys enough to share
  // a workgroup's staged twiddles, else one tile per workgroup
  // every limb of the set on an FP64 modulus: the LDS-twiddle column pass
  bool allf = GPQHE_COLSF && G.twd != nullptr;
  for (unsigned i = 0; i < s.per; i++)
    allf &= G.q[s.mods[i]] < (1ull << 51);
  auto cols_launch = [&](bool inv, const LimbSet &in, const LimbSet &out) {
    // (several tiles per workgroup with the next tile's words requested ahead
    // measured slower: 86 -> 103 us forward, 73 -> 88 us inverse per 48-poly group)
    if (allf)
      ntt2_colsf_launch(LOGT1, inv, blocks, in, out, post);
    else if (inv)
      hipLaunchKernelGGL((ntt2_cols_kernel<LOGT1, true>), dim3(blocks), dim3(256), 0, G.stream, in, out, logn, tw,
                         G.dev.mc, post);
    else
      hipLaunchKernelGGL((ntt2_cols_kernel<LOGT1, false>), dim3(blocks), dim3(256), 0, G.stream, in, out, logn, tw,
                         G.dev.mc, (const uint64_t *)nullptr);
  };
  auto rows_launch = [&](bool inv, const LimbSet &in, const LimbSet &out) { ntt_rows_launch<LOGN2>(inv, in, out); };
  if (!inverse) {
    {
      ProfScope ps(KC_NTT2_COLS_FWD, pass_bytes);
      cols_launch(false, s, o);
    }
    ProfScope ps(KC_NTT3_ROWS_FWD, pass_bytes);
    rows_launch(false, o, o);
  } else {
    {
      ProfScope ps(KC_NTT3_ROWS_INV, pass_bytes);
      rows_launch(true, s, o);
    }
    ProfScope ps(KC_NTT2_COLS_INV, pass_bytes);
    cols_launch(true, o, o);
  }
  HIP_CHECK(hipGetLastError());
}

// two-pass path for this ring degree?
static bool ntt2_ok()
{
  return G.logn >= 13 && G.logn <= 17;
}

// Out-of-place NTT (in and out have the same geometry; out may equal in);
// `post` (inverse only) replaces n^-1 by per-slot Shoup pairs post[2 (v % per)].
static void ntt_small_launch(const LimbSet &s, const LimbSet &in, bool inverse);

void k_ntt_ex(const LimbSet &in, const LimbSet &out, bool inverse, const uint64_t *post)
{
  if (!in.count)
    return;
  if (G.logn >= 10 && G.logn <= 12 && !post) {
    ntt_small_launch(out, in.base == out.base && !in.ngp ? LimbSet{} : in, inverse);
    return;
  }
  switch (G.logn) {
  case 13: ntt2_launch<6, 7>(in, out, inverse, post); return;
  case 14: ntt2_launch<7, 7>(in, out, inverse, post); return;
  case 15: ntt2_launch<7, 8>(in, out, inverse, post); return;
  case 16: ntt2_launch<8, 8>(in, out, inverse, post); return;
  case 17: ntt2_launch<8, 9>(in, out, inverse, post); return;
  default: gpqhe_die("k_ntt_ex: ring degree 2^%u not supported", G.logn);
  }
}

void k_ntt_rows(const LimbSet &in, const LimbSet &out, bool inverse)
{
  if (!in.count)
    return;
  ProfScope ps(inverse ? KC_NTT3_ROWS_INV : KC_NTT3_ROWS_FWD, 16.0 * G.n * in.count);
  switch (G.logn) {
  case 13: ntt_rows_launch<7>(inverse, in, out); break;
  case 14: ntt_rows_launch<7>(inverse, in, out); break;
  case 15: ntt_rows_launch<8>(inverse, in, out); break;
  case 16: ntt_rows_launch<8>(inverse, in, out); break;
  case 17: ntt_rows_launch<9>(inverse, in, out); break;
  default: gpqhe_die("k_ntt_rows: ring degree 2^%u not supported", G.logn);
  }
  HIP_CHECK(hipGetLastError());
}

// Whole-limb NTT for n = 2^10 .. 2^12 (HECTR's own ring): one block of n/8
// threads per limb, radix-8 register rounds (3 stages each, the last round
// takes the remaining logn mod 3 stages on 8 / 2^r groups per thread), lazy
// butterflies on the limb's arithmetic policy.  Round r covers global stages
// [3r, 3r + 3): thread t's group starts at pos0 = (t / D8) 8 D8 + t % D8 with
// D8 = n >> (3r + 3) the group's smallest distance, twiddle base n + pos0.
// coef != nullptr (forward only): round 0 reads the signed integer
// coefficients shared by every limb and lifts them mod q (encoding), instead
// of a separate lift launch.
__device__ __forceinline__ uint64_t lift_i64(int64_t v, const ModConst &c)
{
  if (v >= 0)
    return reduce64((uint64_t)v, c);
  const uint64_t r = reduce64((uint64_t)(-(v + 1)), c) + 1;  // |v| mod q in [1, q]
  return r == c.q ? 0 : c.q - r;
}

// small_fwd / small_inv: ntt_device.h

template <int LOGN, bool INV>
__global__ void __launch_bounds__(512) ntt_small_kernel(LimbSet s, Tw2 tw, const ModConst *mcs,
                                                         const int64_t *coef, LimbSet in, unsigned clog)
{
  constexpr int n = 1 << LOGN;
  __shared__ __attribute__((aligned(16))) uint64_t lds[n];
  const unsigned v = blockIdx.x;
  uint64_t *x = s.limb(v, LOGN);
  const uint64_t *xi = in.base ? in.limb(v, LOGN) : x;  // out of place: same geometry
  const unsigned m = s.mod(v);
  const ModConst mc = mcs[m];
  with_arith(mc.q, m, LOGN, tw, [&](const auto &ar) {
    using A = std::decay_t<decltype(ar)>;
    using V = typename A::V;
    if constexpr (!INV) {
      small_fwd<LOGN>(
          ar, lds,
          [&](int, int i) {
            // coef: n >> clog values per group, coefficient i = j 2^clog holds
            // value j, the others are 0
            if (!coef)
              return A::load(xi[i]);
            return A::load((i & ((1 << clog) - 1))
                               ? 0
                               : lift_i64(coef[((size_t)(v / s.per) << (LOGN - clog)) + (i >> clog)], mc));
          },
          [&](int, int i, V a) { x[i] = ar.canon(a); });
    } else {
      small_inv<LOGN>(
          ar, lds, [&](int, int i) { return A::load(xi[i]); },
          [&](int, int i, V a) { x[i] = ar.mulc(a, mc.ninv, mc.ninvp); });
    }
  });
}

// In-place forward transform of limb v of s (ntt_small_kernel<LOGN, false>
// without a lift), for workgroups attached to another launch (SpecAttach).
template <int LOGN>
__device__ __forceinline__ void ntt_fwd_small_body(const LimbSet &s, const Tw2 &tw, const ModConst *mcs, unsigned v,
                                                   uint64_t *lds)
{
  uint64_t *x = s.limb(v, LOGN);
  const unsigned m = s.mod(v);
  const ModConst mc = mcs[m];
  with_arith(mc.q, m, LOGN, tw, [&](const auto &ar) {
    using A = std::decay_t<decltype(ar)>;
    small_fwd<LOGN>(
        ar, lds, [&](int, int i) { return A::load(x[i]); }, [&](int, int i, typename A::V a) { x[i] = ar.canon(a); });
  });
}

// The same lift + forward transform with the (few) coefficients passed by
// value in the kernel arguments: group g's value j at ca.v[g row + j] is
// coefficient j 2^clog, the others are 0.  No upload, no host-memory reads.
template <int LOGN>
__global__ void __launch_bounds__(512) lift_ntt_arg_kernel(LimbSet s, Tw2 tw, const ModConst *mcs, CoefArg ca)
{
  constexpr int n = 1 << LOGN;
  __shared__ __attribute__((aligned(16))) uint64_t lds[n];
  const unsigned v = blockIdx.x;
  uint64_t *x = s.limb(v, LOGN);
  const unsigned m = s.mod(v), g = v / s.per, clog = ca.clog;
  const ModConst mc = mcs[m];
  with_arith(mc.q, m, LOGN, tw, [&](const auto &ar) {
    using A = std::decay_t<decltype(ar)>;
    small_fwd<LOGN>(
        ar, lds,
        [&](int, int i) {
          // round 0 holds elements th + k n/8: for clog >= 6 the value index
          // i >> clog is wave-uniform, so a scalar load reads the argument
          // (per-lane reads of by-value arguments cost ~3.5 us, ubench_small)
          const int j = clog >= 6 ? __builtin_amdgcn_readfirstlane(i >> clog) : i >> clog;
          return A::load((i & ((1 << clog) - 1)) ? 0 : lift_i64(ca.v[g * ca.row + j], mc));
        },
        [&](int, int i, typename A::V a) { x[i] = ar.canon(a); });
  });
}

void k_lift_ntt_arg(const LimbSet &s, const int64_t *coef_host, unsigned clog)
{
  const unsigned row = G.n >> clog, groups = s.count / s.per;
  if (G.logn < 10 || G.logn > 12 || (size_t)groups * row > CoefArg::MAX)
    gpqhe_die("k_lift_ntt_arg: %u x %u coefficients at n = %u", groups, row, G.n);
  CoefArg ca;
  memcpy(ca.v, coef_host, (size_t)groups * row * 8);
  ca.clog = clog;
  ca.row = row;
  ProfScope ps(KC_NTT_SMALL_FWD, 8.0 * G.n * s.count);
  const Tw2 tw{G.tw2, G.itw2, G.twd, G.itwd};
  auto go = [&](auto kern, unsigned threads) {
    hipLaunchKernelGGL(kern, dim3(s.count), dim3(threads), 0, G.stream, s, tw, G.dev.mc, ca);
  };
  if (G.logn == 12)
    go(lift_ntt_arg_kernel<12>, 512);
  else if (G.logn == 11)
    go(lift_ntt_arg_kernel<11>, 256);
  else
    go(lift_ntt_arg_kernel<10>, 128);
  HIP_CHECK(hipGetLastError());
}

// Encoding: lift the signed coefficients into every limb of s, then the
// forward NTT (one launch for n <= 2^12).  clog > 0 (n <= 2^12 only): each
// group's row holds only every 2^clog-th coefficient (the others are zero:
// an encoding of s slots has nonzero coefficients at stride n / 2s only).
void k_lift_ntt(const LimbSet &s, const int64_t *coef, unsigned clog)
{
  if (G.logn >= 10 && G.logn <= 12) {
    ProfScope ps(KC_NTT_SMALL_FWD, 8.0 * G.n * (s.count + 1));
    const Tw2 tw{G.tw2, G.itw2, G.twd, G.itwd};
    auto go = [&](auto kern, unsigned threads) {
      hipLaunchKernelGGL(kern, dim3(s.count), dim3(threads), 0, G.stream, s, tw, G.dev.mc, coef, LimbSet{}, clog);
    };
    if (G.logn == 12)
      go(ntt_small_kernel<12, false>, 512);
    else if (G.logn == 11)
      go(ntt_small_kernel<11, false>, 256);
    else
      go(ntt_small_kernel<10, false>, 128);
    HIP_CHECK(hipGetLastError());
    return;
  }
  if (clog)
    gpqhe_die("k_lift_ntt: strided coefficients need n <= 2^12");
  k_lift_i64(s, coef);
  k_ntt(s, false);
}

// ntt_small_kernel over s; `in` (same geometry, base != nullptr): read the
// input from there (out of place).
static void ntt_small_launch(const LimbSet &s, const LimbSet &in, bool inverse)
{
  const unsigned logn = G.logn, n = G.n;
  ProfScope ps(inverse ? KC_NTT_SMALL_INV : KC_NTT_SMALL_FWD, 16.0 * n * s.count);
  const Tw2 tw{G.tw2, G.itw2, G.twd, G.itwd};
  auto go = [&](auto kern, unsigned threads) {
    hipLaunchKernelGGL(kern, dim3(s.count), dim3(threads), 0, G.stream, s, tw, G.dev.mc, (const int64_t *)nullptr,
                       in, 0u);
  };
  if (logn == 12)
    inverse ? go(ntt_small_kernel<12, true>, 512) : go(ntt_small_kernel<12, false>, 512);
  else if (logn == 11)
    inverse ? go(ntt_small_kernel<11, true>, 256) : go(ntt_small_kernel<11, false>, 256);
  else
    inverse ? go(ntt_small_kernel<10, true>, 128) : go(ntt_small_kernel<10, false>, 128);
  HIP_CHECK(hipGetLastError());
}

void k_ntt(const LimbSet &s, bool inverse)
{
  if (!s.count)
    return;
  const unsigned logn = G.logn, n = G.n;
  if (s.count > 65535)
    gpqhe_die("k_ntt: %u limbs in one launch", s.count);
  if (logn >= 10 && logn <= 12) {
    ntt_small_launch(s, LimbSet{}, inverse);
    return;
  }
  if (logn <= 12) {
    ProfScope ps(inverse ? KC_NTT_WHOLE_INV : KC_NTT_WHOLE_FWD, 16.0 * n * s.count);
    if (inverse)
      hipLaunchKernelGGL(ntt_whole_kernel<true>, dim3(1, s.count), dim3(TPB), n * 8, G.stream, s, logn, G.dev);
    else
      hipLaunchKernelGGL(ntt_whole_kernel<false>, dim3(1, s.count), dim3(TPB), n * 8, G.stream, s, logn, G.dev);
    HIP_CHECK(hipGetLastError());
    return;
  }
  if (!ntt2_ok())
    gpqhe_die("k_ntt: ring degree 2^%u not supported", logn);
  k_ntt_ex(s, s, inverse, nullptr);
}

// ===========================================================================
// Elementwise kernels
// ===========================================================================
// out = a op b over npoly x lvl limbs; op 0 add, 1 sub.
__global__ void binop_kernel(uint64_t *out, const uint64_t *a, const uint64_t *b, unsigned logn, unsigned lvl,
                             size_t os, size_t as, size_t bs, int op, const ModConst *mc)
{
  const size_t n = (size_t)1 << logn;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned limb = blockIdx.y, p = blockIdx.z;
  if (i >= n)
    return;
  const uint64_t q = mc[limb].q;
  const uint64_t x = a[p * as + ((size_t)limb << logn) + i], y = b[p * bs + ((size_t)limb << logn) + i];
  out[p * os + ((size_t)limb << logn) + i] = op ? sub_mod(x, y, q) : add_mod(x, y, q);
}

void k_binop(uint64_t *out, const uint64_t *a, const uint64_t *b, unsigned npoly, unsigned lvl, size_t os,
             size_t as, size_t bs, int op)
{
  hipLaunchKernelGGL(binop_kernel, dim3((G.n + TPB - 1) / TPB, lvl, npoly), dim3(TPB), 0, G.stream, out, a, b,
                     G.logn, lvl, os, as, bs, op, G.dev.mc);
  HIP_CHECK(hipGetLastError());
}

__global__ void neg_kernel(uint64_t *x, unsigned logn, size_t ps, const ModConst *mc)
{
  const size_t n = (size_t)1 << logn;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n)
    return;
  uint64_t *p = x + blockIdx.z * ps + ((size_t)blockIdx.y << logn) + i;
  *p = neg_mod(*p, mc[blockIdx.y].q);
}

void k_neg(uint64_t *x, unsigned npoly, unsigned lvl, size_t ps)
{
  hipLaunchKernelGGL(neg_kernel, dim3((G.n + TPB - 1) / TPB, lvl, npoly), dim3(TPB), 0, G.stream, x, G.logn, ps,
                     G.dev.mc);
  HIP_CHECK(hipGetLastError());
}

// Canonical product a b mod q of canonical residues (FP64 for q < 2^51).
__device__ __forceinline__ uint64_t mulmod_vv(uint64_t a, uint64_t b, const ModConst &m)
{
  if (m.q < F64_QMAX) {
    const double q = (double)m.q, qinv = 1.0 / q, y = f64_from_u52(b);
    return f64_canon(f64_mulmod(f64_from_u52(a), y, y * qinv, q), q, qinv);
  }
  return mul_mod(a, b, m);
}

// Eight words of tensor poly P (d0 for even P, d1 for odd) at off + pos[k]
// (off: limb/tile offset inside the poly), canonical mod m.q.
__device__ __forceinline__ void d01_fetch8(const D01Src &s, unsigned P, size_t off, const int (&pos)[8],
                                           const ModConst &m, uint64_t (&v)[8])
{
  const uint64_t *pa = s.a + (P >> 1) * s.in_stride + off, *pb = s.b + (P >> 1) * s.in_stride + off;
  if (!(P & 1)) {
#pragma unroll
    for (int k = 0; k < 8; k++)
      v[k] = mulmod_vv(pa[pos[k]], pb[pos[k]], m);
    return;
  }
  if (m.q < F64_QMAX) {
    const double q = (double)m.q, qinv = 1.0 / q;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const double a0 = f64_from_u52(pa[pos[k]]), a1 = f64_from_u52(pa[s.in_pstride + pos[k]]);
      const double b0 = f64_from_u52(pb[pos[k]]), b1 = f64_from_u52(pb[s.in_pstride + pos[k]]);
      v[k] = f64_canon(f64_mulmod(a0, b1, b1 * qinv, q) + f64_mulmod(a1, b0, b0 * qinv, q), q, qinv);
    }
  } else {
#pragma unroll
    for (int k = 0; k < 8; k++)
      v[k] = add_mod(mul_mod(pa[pos[k]], pb[s.in_pstride + pos[k]], m),
                     mul_mod(pa[s.in_pstride + pos[k]], pb[pos[k]], m), m.q);
  }
}

// f0 += P d0, f1 += P d1 of pair i at words off .. off + 7 (8 consecutive
// words, 16-byte loads), in FP64 for m.q < 2^51 (caller's guarantee).  Bounds:
// f0, f1 arrive with |.| < 3q (two MAC products); they are reduced to
// |.| <= q/2 first, d0 = a0 b0 is < 1.25 q, d1 = a0 b1 + a1 b0 is reduced to
// <= q/2, and each P d term is < 1.5 q, so every value stays an exact integer
// below 2^53 and the results are < 2q (canonicalised by the caller).
__device__ __forceinline__ void d01_fold_f64(const D01Src &s, unsigned i, size_t off, const ModConst &m,
                                             double (&f0)[8], double (&f1)[8])
{
  const double q = (double)m.q, qinv = 1.0 / q, P = f64_from_u52(m.pmod), Pq = P * qinv;
  auto ld8 = [](const uint64_t *src, double (&x)[8]) {
    const ulonglong2 *v2 = (const ulonglong2 *)src;
#pragma unroll
    for (int h = 0; h < 4; h++) {
      const ulonglong2 w = v2[h];
      x[2 * h] = f64_from_u52(w.x);
      x[2 * h + 1] = f64_from_u52(w.y);
    }
  };
  double d0[8], d1[8];
  {
    double a0[8], a1[8], b0[8], b1[8];
    const uint64_t *pa = s.a + i * s.in_stride + off, *pb = s.b + i * s.in_stride + off;
    ld8(pa, a0);
    ld8(pb, b0);
    ld8(pa + s.in_pstride, a1);
    ld8(pb + s.in_pstride, b1);
#pragma unroll
    for (int k = 0; k < 8; k++) {
      d0[k] = f64_mulmod(a0[k], b0[k], b0[k] * qinv, q);
      d1[k] = f64_red(f64_mulmod(a0[k], b1[k], b1[k] * qinv, q) + f64_mulmod(a1[k], b0[k], b0[k] * qinv, q), q,
                      qinv);
    }
  }
#pragma unroll
  for (int k = 0; k < 8; k++) {
    f0[k] = f64_red(f0[k], q, qinv) + f64_mulmod(d0[k], P, Pq, q);
    f1[k] = f64_red(f1[k], q, qinv) + f64_mulmod(d1[k], P, Pq, q);
  }
}

// Tensor of count ciphertext pairs: d0 = a0 b0, d1 = a0 b1 + a1 b0 into
// d01 [count][2][lvl][n]; d2 = a1 b1 into d2 [count][lvl][n].  Two adjacent
// coefficients per thread (16-byte accesses).  Moduli below 2^51 use the exact
// FP64 product (f64_mulmod with a variable second operand: both factors < q,
// so ab / q < 2^51, the quotient estimate is off by < 1.25 and every
// intermediate is an integer below 2^53); wider moduli use Barrett.
__global__ void __launch_bounds__(256) tensor_kernel(uint64_t *d01, uint64_t *d2, const uint64_t *a,
                                                     const uint64_t *b, unsigned logn, unsigned lvl, size_t in_stride,
                                                     size_t in_pstride, size_t d01_stride, size_t d2_stride,
                                                     const ModConst *mc)
{
  const size_t n = (size_t)1 << logn;
  const size_t i = 2 * ((size_t)blockIdx.x * blockDim.x + threadIdx.x);
  const unsigned limb = blockIdx.y, c = blockIdx.z;
  if (i >= n)
    return;
  const ModConst m = mc[limb];
  const size_t off = ((size_t)limb << logn) + i;
  const uint64_t *pa = a + c * in_stride, *pb = b + c * in_stride;
  const ulonglong2 A0 = *(const ulonglong2 *)(pa + off), A1 = *(const ulonglong2 *)(pa + in_pstride + off);
  const ulonglong2 B0 = *(const ulonglong2 *)(pb + off), B1 = *(const ulonglong2 *)(pb + in_pstride + off);
  uint64_t r0[2], r1[2], r2[2];
  const uint64_t a0[2] = {A0.x, A0.y}, a1[2] = {A1.x, A1.y}, b0[2] = {B0.x, B0.y}, b1[2] = {B1.x, B1.y};
  if (m.q < F64_QMAX) {
    const double q = (double)m.q, qinv = 1.0 / q;
#pragma unroll
    for (int e = 0; e < 2; e++) {
      const double x0 = f64_from_u52(a0[e]), x1 = f64_from_u52(a1[e]);
      const double y0 = f64_from_u52(b0[e]), y1 = f64_from_u52(b1[e]);
      r0[e] = f64_canon(f64_mulmod(x0, y0, y0 * qinv, q), q, qinv);
      r1[e] = f64_canon(f64_mulmod(x0, y1, y1 * qinv, q) + f64_mulmod(x1, y0, y0 * qinv, q), q, qinv);
      r2[e] = f64_canon(f64_mulmod(x1, y1, y1 * qinv, q), q, qinv);
    }
  } else {
#pragma unroll
    for (int e = 0; e < 2; e++) {
      r0[e] = mul_mod(a0[e], b0[e], m);
      r1[e] = add_mod(mul_mod(a0[e], b1[e], m), mul_mod(a1[e], b0[e], m), m.q);
      r2[e] = mul_mod(a1[e], b1[e], m);
    }
  }
  uint64_t *o = d01 + c * d01_stride;
  *(ulonglong2 *)(o + off) = make_ulonglong2(r0[0], r0[1]);
  *(ulonglong2 *)(o + ((size_t)lvl << logn) + off) = make_ulonglong2(r1[0], r1[1]);
  *(ulonglong2 *)(d2 + c * d2_stride + off) = make_ulonglong2(r2[0], r2[1]);
}

void k_tensor(uint64_t *d01, uint64_t *d2c, const uint64_t *a, const uint64_t *b, unsigned lvl,
              size_t in_stride, size_t in_pstride, unsigned count, size_t d_stride)
{
  ProfScope ps(KC_TENSOR, 8.0 * G.n * lvl * count * 7);  // read 4 limbs, write 3 limbs
  hipLaunchKernelGGL(tensor_kernel, dim3((G.n / 2 + TPB - 1) / TPB, lvl, count), dim3(TPB), 0, G.stream, d01, d2c, a,
                     b, G.logn, lvl, in_stride, in_pstride, d_stride, (size_t)lvl << G.logn, G.dev.mc);
  HIP_CHECK(hipGetLastError());
}

__global__ void dec_kernel(uint64_t *pt, const uint64_t *c0, const uint64_t *c1, const uint64_t *s, unsigned logn,
                           const ModConst *mc)
{
  const size_t n = (size_t)1 << logn;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n)
    return;
  const ModConst m = mc[blockIdx.y];
  const size_t off = ((size_t)blockIdx.y << logn) + i;
  pt[off] = add_mod(c0[off], mul_mod(c1[off], s[off], m), m.q);
}

void k_dec(uint64_t *pt, const uint64_t *c0, const uint64_t *c1, const uint64_t *s, unsigned lvl)
{
  hipLaunchKernelGGL(dec_kernel, dim3((G.n + TPB - 1) / TPB, lvl), dim3(TPB), 0, G.stream, pt, c0, c1, s, G.logn,
                     G.dev.mc);
  HIP_CHECK(hipGetLastError());
}

// One launch for a queued elementwise program: thread (limb, k) applies the
// ops in queue order to its element.  Each op reads and writes only element
// (limb, k) of its operands, so every value is the one of the sequential
// binop / neg / copy / dec launches.
__global__ void ew_prog_kernel(EwProg pr, unsigned logn, const ModConst *mc)
{
  const size_t n = (size_t)1 << logn;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n)
    return;
  const unsigned l = blockIdx.y;
  const ModConst m = mc[l];
  const size_t off = ((size_t)l << logn) + i;
  for (unsigned j = 0; j < pr.count; j++) {
    const EwOp &o = pr.op[j];
    if (l >= o.lvl)
      continue;
    const uint64_t x = o.a[off];
    uint64_t r;
    switch (o.kind) {
    case EW_ADD:
      r = add_mod(x, o.b[off], m.q);
      break;
    case EW_SUB:
      r = sub_mod(x, o.b[off], m.q);
      break;
    case EW_NEG:
      r = neg_mod(x, m.q);
      break;
    case EW_DEC:
      r = add_mod(x, mul_mod(o.b[off], o.s[off], m), m.q);
      break;
    default:
      r = x;
    }
    o.out[off] = r;
  }
}

void k_ew_prog(const EwProg &p)
{
  unsigned lv = 0;
  for (unsigned j = 0; j < p.count; j++)
    lv = std::max(lv, p.op[j].lvl);
  if (!lv)
    return;
  hipLaunchKernelGGL(ew_prog_kernel, dim3((G.n + TPB - 1) / TPB, lv), dim3(TPB), 0, G.stream, p, G.logn, G.dev.mc);
  HIP_CHECK(hipGetLastError());
}

// Small samples (ternary or CBD-21) lifted to every limb of dst.
__global__ void sample_small_kernel(LimbSet dst, unsigned logn, ChachaKey key, uint64_t stream, int cbd,
                                    const ModConst *mc)
{
  const unsigned k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= (1u << logn))
    return;
  uint32_t b[16];
  chacha20_block(b, key, stream, k);
  int v;
  if (cbd) {
    v = __popc(b[0] & 0x1FFFFFu) - __popc(b[1] & 0x1FFFFFu);
  } else {
    const uint32_t r = b[0] & 3u;
    v = r < 2 ? 0 : (r == 2 ? 1 : -1);
  }
  for (unsigned l = 0; l < dst.count; l++) {
    const uint64_t q = mc[dst.mod(l)].q;
    dst.limb(l, logn)[k] = v >= 0 ? (uint64_t)v : q - (uint64_t)(-v);
  }
}

// Encryption noise in one launch: polynomial y of `npoly` (rows of dst.per
// limbs) draws from ChaCha stream `stream + y`; y = 0 is ternary (v), the
// others CBD (e0, e1) -- the same streams and values as npoly separate
// k_sample_small calls in that order.  With ec, encryption e's e0 (y = 3 e + 1)
// also takes the integer coefficients of its plaintext (EncCoef): the caller
// then combines without m, as NTT(e0 + m) = NTT(e0) + NTT(m) mod q.
__device__ __forceinline__ int enc_noise_value(const ChachaKey &key, uint64_t stream, unsigned y, unsigned k)
{
  uint32_t b[16];
  chacha20_block(b, key, stream + y, k);
  if (y % 3)  // (v, e0, e1) per encryption: ternary v, CBD e0 / e1
    return __popc(b[0] & 0x1FFFFFu) - __popc(b[1] & 0x1FFFFFu);
  const uint32_t r = b[0] & 3u;
  return r < 2 ? 0 : (r == 2 ? 1 : -1);
}

// Coefficient k of noise poly y into its limbs (sample_enc_kernel without a
// plaintext; the attached sampler of gemv_inner_kernel).
__device__ __forceinline__ void enc_noise_store(const LimbSet &dst, unsigned logn, const ChachaKey &key,
                                                uint64_t stream, const ModConst *mc, unsigned y, unsigned k)
{
  const int v = enc_noise_value(key, stream, y, k);
  for (unsigned l = y * dst.per; l < (y + 1) * dst.per; l++) {
    const uint64_t q = mc[dst.mod(l)].q;
    dst.limb(l, logn)[k] = v >= 0 ? (uint64_t)v : q - (uint64_t)(-v);
  }
}

__global__ void sample_enc_kernel(LimbSet dst, unsigned logn, ChachaKey key, uint64_t stream, const ModConst *mc,
                                  EncCoef ec, int has_ec)
{
  const unsigned k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= (1u << logn))
    return;
  const unsigned y = blockIdx.y;
  const int v = enc_noise_value(key, stream, y, k);
  bool addm = false;
  int64_t mco = 0;
  if (has_ec && y % 3 == 1) {
    const int row = ec.row_of[y / 3];
    if (row >= 0 && !(k & ((1u << ec.clog) - 1))) {
      // for clog >= 6 the index is wave-uniform (blocks of whole waves): a
      // scalar load of the by-value argument (per-lane reads: ubench_small)
      const unsigned i = (unsigned)row * ec.row + (k >> ec.clog);
      mco = ec.p ? ec.p[i] : ec.v[ec.clog >= 6 ? __builtin_amdgcn_readfirstlane(i) : i];
      addm = true;
    }
  }
  for (unsigned l = y * dst.per; l < (y + 1) * dst.per; l++) {
    const ModConst &m = mc[dst.mod(l)];
    uint64_t r = v >= 0 ? (uint64_t)v : m.q - (uint64_t)(-v);
    if (addm)
      r = add_mod(r, lift_i64(mco, m), m.q);
    dst.limb(l, logn)[k] = r;
  }
}

// The noise alone (speculation, keygen paths): no 2.6 KB EncCoef argument to
// copy into every launch
__global__ void sample_noise_kernel(LimbSet dst, unsigned logn, ChachaKey key, uint64_t stream, const ModConst *mc)
{
  const unsigned k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < (1u << logn))
    enc_noise_store(dst, logn, key, stream, mc, blockIdx.y, k);
}

void k_sample_enc(const LimbSet &dst, uint64_t stream, unsigned npoly, const EncCoef *ec)
{
  const dim3 grid((G.n + TPB - 1) / TPB, npoly);
  if (ec)
    hipLaunchKernelGGL(sample_enc_kernel, grid, dim3(TPB), 0, G.stream, dst, G.logn, G.key, stream, G.dev.mc, *ec, 1);
  else
    hipLaunchKernelGGL(sample_noise_kernel, grid, dim3(TPB), 0, G.stream, dst, G.logn, G.key, stream, G.dev.mc);
  HIP_CHECK(hipGetLastError());
}

void k_sample_small(const LimbSet &dst, uint64_t stream, int cbd)
{
  hipLaunchKernelGGL(sample_small_kernel, grid1(G.n), dim3(TPB), 0, G.stream, dst, G.logn, G.key, stream, cbd,
                     G.dev.mc);
  HIP_CHECK(hipGetLastError());
}

__global__ void sample_uniform_kernel(LimbSet dst, unsigned logn, ChachaKey key, uint64_t stream, unsigned nb,
                                      const ModConst *mc)
{
  const unsigned k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= (1u << logn))
    return;
  const unsigned l = blockIdx.y;
  const unsigned m = dst.mod(l);
  const ModConst c = mc[m];
  uint32_t b[16];
  chacha20_block(b, key, stream, k * nb + m / 4);
  const uint32_t *w = b + 4 * (m % 4);
  const uint64_t lo = (uint64_t)w[0] | ((uint64_t)w[1] << 32), hi = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
  // (hi 2^64 + lo) mod q
  const uint64_t r64 = reduce64(reduce64(~0ull, c) + 1, c);  // 2^64 mod q
  const uint64_t v = add_mod(mul_mod(reduce64(hi, c), r64, c), reduce64(lo, c), c.q);
  dst.limb(l, logn)[k] = v;
}

void k_sample_uniform(const LimbSet &dst, uint64_t stream)
{
  const unsigned nb = (G.nmod + 3) / 4;
  hipLaunchKernelGGL(sample_uniform_kernel, dim3((G.n + TPB - 1) / TPB, dst.count), dim3(TPB), 0, G.stream, dst,
                     G.logn, G.key, stream, nb, G.dev.mc);
  HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------
// GPU CKKS encoder (he_ecd for large slot counts): the special inverse FFT of
// host_math.cpp (fft_special_enc) stage by stage with the same operations in
// the same order (IEEE products, sums and division, no contraction: this file
// is built with -ffp-contract=off), then bit reversal, / s, x scale and
// llround.  Bit-identical to the host encoder and the oracle.
//   stages with len > FFT_LDS: one launch each, a thread per butterfly;
//   stages with len <= FFT_LDS: one launch, a block per FFT_LDS-element chunk
//   in LDS (the chunks are independent below that length).
// ---------------------------------------------------------------------------
constexpr unsigned FFT_LDS = 2048;
static_assert(FFT_LDS == GPQHE_DCD_ONEPASS, "k_decode's one-launch bound");

__device__ __forceinline__ void fft_enc_bfly(double2 &x, double2 &y, const double2 w)
{
  const double2 a = make_double2(x.x + y.x, x.y + y.y);
  const double2 d = make_double2(x.x - y.x, x.y - y.y);
  x = a;
  y = make_double2(d.x * w.x - d.y * w.y, d.x * w.y + d.y * w.x);
}

__global__ void fft_enc_stage_kernel(double2 *v, unsigned s, unsigned len, const double2 *ksi, const unsigned *rot)
{
  const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= s / 2)
    return;
  const unsigned h = len >> 1, lq = len << 2, M = 4 * s;
  const unsigned i = (t / h) * len, j = t % h;
  const unsigned idx = (lq - rot[j] % lq) * (M / lq);
  fft_enc_bfly(v[i + j], v[i + j + h], ksi[idx]);
}

__global__ void __launch_bounds__(512) fft_enc_lds_kernel(double2 *v, unsigned s, unsigned len0, const double2 *ksi,
                                                          const unsigned *rot)
{
  __shared__ double2 c[FFT_LDS];
  const unsigned base = blockIdx.x * len0, M = 4 * s;
  for (unsigned e = threadIdx.x; e < len0; e += blockDim.x)
    c[e] = v[base + e];
  __syncthreads();
  for (unsigned len = len0; len >= 2; len >>= 1) {
    const unsigned h = len >> 1, lq = len << 2;
    for (unsigned t = threadIdx.x; t < len0 / 2; t += blockDim.x) {
      const unsigned i = (t / h) * len, j = t % h;
      const unsigned idx = (lq - rot[j] % lq) * (M / lq);
      fft_enc_bfly(c[i + j], c[i + j + h], ksi[idx]);
    }
    __syncthreads();
  }
  for (unsigned e = threadIdx.x; e < len0; e += blockDim.x)
    v[base + e] = c[e];
}

// coef[k gap] = llround(re(u_k) / s * scale), coef[(k + s) gap] = im, 0
// elsewhere; u = bit-reversed v.  One thread per coefficient slot pair.
__global__ void fft_enc_round_kernel(int64_t *coef, const double2 *v, unsigned s, unsigned logs, unsigned n,
                                     double scale, int *overflow)
{
  const unsigned k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n / 2)
    return;
  const unsigned gap = n / (2 * s);
  int64_t lo = 0, hi = 0;
  if (k % gap == 0) {
    const unsigned slot = k / gap;
    const double2 u = v[logs ? __brev(slot) >> (32 - logs) : 0];
    const double re = u.x / (double)s * scale, im = u.y / (double)s * scale;
    if (fabs(re) >= 9.2e18 || fabs(im) >= 9.2e18)
      *overflow = 1;
    lo = llround(re);
    hi = llround(im);
  }
  coef[k] = lo;
  coef[k + n / 2] = hi;
}

struct FftDev {
  double2 *ksi;
  unsigned *rot;
};
static std::map<unsigned, FftDev> g_fft;

static const FftDev &fft_dev(unsigned s)
{
  if (!s || (s & (s - 1)) || s > G.n / 2)
    gpqhe_die("bad slot count %u", s);
  auto it = g_fft.find(s);
  if (it == g_fft.end()) {
    std::vector<double> ksi(2 * (4 * (size_t)s + 1));
    std::vector<unsigned> rot(s);
    hm_fft_tables(s, ksi.data(), rot.data());
    FftDev d;
    HIP_CHECK(hipMalloc(&d.ksi, ksi.size() * 8));
    HIP_CHECK(hipMalloc(&d.rot, rot.size() * 4));
    HIP_CHECK(hipMemcpy(d.ksi, ksi.data(), ksi.size() * 8, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(d.rot, rot.data(), rot.size() * 4, hipMemcpyHostToDevice));
    it = g_fft.emplace(s, d).first;
  }
  return it->second;
}

void k_encode_coeffs(int64_t *coef, double *work, unsigned s, double scale)
{
  const unsigned n = G.n;
  const FftDev &T = fft_dev(s);
  double2 *v = (double2 *)work;
  unsigned len = s;
  for (; len > FFT_LDS; len >>= 1)
    hipLaunchKernelGGL(fft_enc_stage_kernel, dim3((s / 2 + TPB - 1) / TPB), dim3(TPB), 0, G.stream, v, s, len, T.ksi,
                       T.rot);
  if (len >= 2)
    hipLaunchKernelGGL(fft_enc_lds_kernel, dim3(s / len), dim3(std::min(512u, std::max(64u, len / 2))), 0, G.stream,
                       v, s, len, T.ksi, T.rot);
  int *ovf = (int *)(work + 2 * (size_t)s);
  HIP_CHECK(hipMemsetAsync(ovf, 0, sizeof(int), G.stream));
  hipLaunchKernelGGL(fft_enc_round_kernel, dim3((n / 2 + TPB - 1) / TPB), dim3(TPB), 0, G.stream, coef, v, s,
                     (unsigned)__builtin_ctz(s), n, scale, ovf);
  HIP_CHECK(hipGetLastError());
  int h = 0;
  HIP_CHECK(hipMemcpyAsync(&h, ovf, sizeof(int), hipMemcpyDeviceToHost, G.stream));
  HIP_CHECK(hipStreamSynchronize(G.stream));
  if (h)
    gpqhe_die("encode overflow (|value * scale| >= 2^63)");
}

// ---------------------------------------------------------------------------
// GPU CKKS decoder (he_dcd): the centred CRT lift (Garner) of the 2s
// coefficients the slots read, / scale, and the special forward FFT of
// host_math.cpp (hm_decode: crt_center, fft_special_dec) with the same
// integer steps and the same IEEE operations in the same order (no
// contraction), so bit-identical to the host decoder and the oracle
// (oracle/ckks_oracle.c crt_center / he_dcd_ex).  Only the s decoded values
// cross PCIe instead of nl limbs of n residues.
//   fft_dec_lds_kernel: a block per FFT_LDS-element chunk of the bit-reversed
//     vector lifts its elements straight into LDS and runs the stages
//     len = 2 .. chunk there;
//   fft_dec_stage_kernel: the stages with len > FFT_LDS, a thread per butterfly.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void fft_dec_bfly(double2 &x, double2 &y, const double2 w)
{
  const double2 a = x;
  const double2 b = make_double2(y.x * w.x - y.y * w.y, y.x * w.y + y.y * w.x);
  x = make_double2(a.x + b.x, a.y + b.y);
  y = make_double2(a.x - b.x, a.y - b.y);
}

// Centred lift of coefficient k over q_0..q_{nl-1} (nl <= NLM), as double.
// ginv[i * ld + j] = (q_j mod q_i)^-1 mod q_i.  Words above nl stay zero, so
// the fixed-length loops give the host's values exactly.
template <int NLM>
__device__ double dcd_crt_center(const uint64_t *c, unsigned k, unsigned nl, unsigned logn, const ModConst *mc,
                                 const uint64_t *ginv, unsigned ld)
{
  constexpr int U = NLM <= 16 ? NLM + 1 : 1;  // registers up to 16 limbs
  if (nl == 1) {
    const uint64_t v = c[k], q = mc[0].q;
    return v > q / 2 ? -(double)(q - v) : (double)v;
  }
  uint64_t v[NLM];
#pragma unroll U
  for (int i = 0; i < NLM; i++) {
    v[i] = 0;
    if (i < (int)nl) {
      const ModConst m = mc[i];
      uint64_t t = c[((size_t)i << logn) + k];
#pragma unroll U
      for (int j = 0; j < i; j++) {
        t = sub_mod(t, reduce64(v[j], m), m.q);
        t = mul_mod(t, ginv[i * ld + j], m);
      }
      v[i] = t;
    }
  }
  // val = v_{nl-1}; val = val q_i + v_i for i = nl-2 .. 0 (Horner from 0);
  // Q = prod q_i
  uint64_t val[NLM + 1], Q[NLM + 1];
#pragma unroll U
  for (int w = 0; w <= NLM; w++)
    val[w] = Q[w] = 0;
  Q[0] = 1;
#pragma unroll U
  for (int i = NLM - 1; i >= 0; i--) {
    if (i < (int)nl) {
      const uint64_t q = mc[i].q;
      uint64_t cv = v[i], cq = 0;
#pragma unroll U
      for (int w = 0; w <= NLM; w++) {
        uint64_t lo = val[w] * q, hi = __umul64hi(val[w], q);
        lo += cv;
        hi += lo < cv;
        val[w] = lo;
        cv = hi;
        uint64_t ql = Q[w] * q, qh = __umul64hi(Q[w], q);
        ql += cq;
        qh += ql < cq;
        Q[w] = ql;
        cq = qh;
      }
    }
  }
  // negative iff 2 val > Q
  int cmp = 0;
  uint64_t carry = 0;
  uint64_t twice[NLM + 1];
#pragma unroll U
  for (int w = 0; w <= NLM; w++) {
    twice[w] = (val[w] << 1) | carry;
    carry = val[w] >> 63;
  }
#pragma unroll U
  for (int w = NLM; w >= 0; w--)
    if (!cmp && twice[w] != Q[w])
      cmp = twice[w] > Q[w] ? 1 : -1;
  const bool neg = cmp > 0;
  if (neg) {
    uint64_t b = 0;
#pragma unroll U
    for (int w = 0; w <= NLM; w++) {
      const uint64_t d = Q[w] - val[w], d2 = d - b;
      b = (Q[w] < val[w]) | (d < b);
      val[w] = d2;
    }
  }
  double d = 0;
#pragma unroll U
  for (int w = NLM; w >= 0; w--)
    d = d * 18446744073709551616.0 + (double)val[w];
  return neg ? -d : d;
}

// One chunk of len0 elements at base: lift into sh, stages 2 .. len0, store.
template <int NLM>
__device__ __forceinline__ void dcd_chunk(double2 *sh, double2 *v, unsigned base, const uint64_t *c, unsigned nl,
                                          unsigned logn, unsigned s, unsigned logs, unsigned len0, double scale,
                                          const ModConst *mc, const uint64_t *ginv, unsigned ld, const double2 *ksi,
                                          const unsigned *rot)
{
  const unsigned M = 4 * s, gap = (1u << logn) / (2 * s);
  for (unsigned e = threadIdx.x; e < len0; e += blockDim.x) {
    const unsigned slot = logs ? __brev(base + e) >> (32 - logs) : 0;  // v = bit-reversed u
    const double re = dcd_crt_center<NLM>(c, slot * gap, nl, logn, mc, ginv, ld);
    const double im = dcd_crt_center<NLM>(c, (slot + s) * gap, nl, logn, mc, ginv, ld);
    sh[e] = make_double2(re / scale, im / scale);
  }
  __syncthreads();
  for (unsigned len = 2; len <= len0; len <<= 1) {
    const unsigned h = len >> 1, lq = len << 2;
    for (unsigned t = threadIdx.x; t < len0 / 2; t += blockDim.x) {
      const unsigned i = (t / h) * len, j = t % h;
      fft_dec_bfly(sh[i + j], sh[i + j + h], ksi[(rot[j] % lq) * (M / lq)]);
    }
    __syncthreads();
  }
  for (unsigned e = threadIdx.x; e < len0; e += blockDim.x)
    v[base + e] = sh[e];
}

template <int NLM>
__global__ void __launch_bounds__(512) fft_dec_lds_kernel(double2 *v, const uint64_t *c, unsigned nl, unsigned logn,
                                                          unsigned s, unsigned logs, unsigned len0, double scale,
                                                          const ModConst *mc, const uint64_t *ginv, unsigned ld,
                                                          const double2 *ksi, const unsigned *rot)
{
  __shared__ double2 sh[FFT_LDS];
  dcd_chunk<NLM>(sh, v, blockIdx.x * len0, c, nl, logn, s, logs, len0, scale, mc, ginv, ld, ksi, rot);
}

__global__ void fft_dec_stage_kernel(double2 *v, unsigned s, unsigned len, const double2 *ksi, const unsigned *rot)
{
  const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= s / 2)
    return;
  const unsigned h = len >> 1, lq = len << 2, M = 4 * s;
  const unsigned i = (t / h) * len, j = t % h;
  fft_dec_bfly(v[i + j], v[i + j + h], ksi[(rot[j] % lq) * (M / lq)]);
}

static uint64_t *g_ginv = nullptr;  // [L][L] Garner inverses of the current context

static void garner_table()
{
  if (g_ginv)
    return;
  const unsigned ld = G.L;
  std::vector<uint64_t> h((size_t)ld * ld, 0);
  for (unsigned i = 0; i < ld; i++)
    for (unsigned j = 0; j < i; j++)
      h[(size_t)i * ld + j] = hm_inv_mod(G.q[j] % G.q[i], G.q[i]);
  HIP_CHECK(hipMalloc(&g_ginv, h.size() * 8));
  HIP_CHECK(hipMemcpy(g_ginv, h.data(), h.size() * 8, hipMemcpyHostToDevice));
}

void k_decode(double *z, const uint64_t *coef, unsigned nl, unsigned s, double scale)
{
  const FftDev &T = fft_dev(s);
  if (nl < 1 || nl > G.L)
    gpqhe_die("he_dcd: bad level %u", nl);
  const unsigned ld = G.L;
  garner_table();
  double2 *v = (double2 *)z;
  const unsigned logs = (unsigned)__builtin_ctz(s), len0 = std::min(s, FFT_LDS);
  const dim3 grid(s / len0), block(std::min(512u, std::max(64u, len0 / 2)));
#define GPQHE_DCD(NLM)                                                                                     \
  hipLaunchKernelGGL(fft_dec_lds_kernel<NLM>, grid, block, 0, G.stream, v, coef, nl, G.logn, s, logs, len0, \
                     scale, G.dev.mc, g_ginv, ld, T.ksi, T.rot)
  if (nl <= 2)
    GPQHE_DCD(2);
  else if (nl <= 4)
    GPQHE_DCD(4);
  else if (nl <= 8)
    GPQHE_DCD(8);
  else if (nl <= 16)
    GPQHE_DCD(16);
  else
    GPQHE_DCD(GPQHE_MAXMOD);
#undef GPQHE_DCD
  for (unsigned len = 2 * len0; len <= s; len <<= 1)
    hipLaunchKernelGGL(fft_dec_stage_kernel, dim3((s / 2 + TPB - 1) / TPB), dim3(TPB), 0, G.stream, v, s, len,
                       T.ksi, T.rot);
  HIP_CHECK(hipGetLastError());
}

// The decoder's tail of a small-N control step: the inverse transform of the
// plaintext's nl <= 2 limbs and the decoder (s <= FFT_LDS) in one workgroup,
// which reads what it wrote after a barrier.  Same values as
// ntt_small_kernel<inv> + fft_dec_lds_kernel.  Measured non-levers: the
// queued elementwise program inside this workgroup too (one CU streams the
// program's ~1.2 MB: 44 us against 19 us for the three launches), and the
// transforms in one workgroup per limb with the last one to finish decoding
// (the agent-scope release / acquire that hand-off needs: 42 us).
template <int LOGN>
__global__ void __launch_bounds__(512) inv_dcd_kernel(const uint64_t *pt, unsigned nl, uint64_t *c, double2 *z,
                                                       unsigned s, unsigned logs, double scale, Tw2 tw,
                                                       const ModConst *mcs, const uint64_t *ginv, unsigned ld,
                                                       const double2 *ksi, const unsigned *rot)
{
  constexpr int n = 1 << LOGN;
  __shared__ __attribute__((aligned(16))) uint64_t lds[n];
  for (unsigned l = 0; l < nl; l++) {
    __syncthreads();  // the previous transform's LDS use
    const ModConst mc = mcs[l];
    const uint64_t *xi = pt + ((size_t)l << LOGN);
    uint64_t *x = c + ((size_t)l << LOGN);
    with_arith(mc.q, l, LOGN, tw, [&](const auto &ar) {
      using A = std::decay_t<decltype(ar)>;
      small_inv<LOGN>(
          ar, lds, [&](int, int i) { return A::load(xi[i]); },
          [&](int, int i, typename A::V a) { x[i] = ar.mulc(a, mc.ninv, mc.ninvp); });
    });
  }
  __syncthreads();
  dcd_chunk<2>((double2 *)lds, z, 0, c, nl, LOGN, s, logs, s, scale, mcs, ginv, ld, ksi, rot);
}

void k_ew_decode(const EwProg &p, double *z, const uint64_t *pt, unsigned nl, unsigned s, double scale, uint64_t *c)
{
  const FftDev &T = fft_dev(s);
  if (nl < 1 || nl > 2 || nl > G.L || s > FFT_LDS || G.logn < 10 || G.logn > 12)
    gpqhe_die("k_ew_decode: n = %u, %u limbs, %u slots", G.n, nl, s);
  garner_table();
  const unsigned logs = (unsigned)__builtin_ctz(s);
  k_ew_prog(p);
  const Tw2 tw{G.tw2, G.itw2, G.twd, G.itwd};
  ProfScope ps(KC_NTT_SMALL_INV, 16.0 * G.n * nl);
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(1), dim3(G.n / 8), 0, G.stream, pt, nl, c, (double2 *)z, s, logs, scale, tw,
                       G.dev.mc, g_ginv, G.L, T.ksi, T.rot);
  };
  if (G.logn == 12)
    go(inv_dcd_kernel<12>);
  else if (G.logn == 11)
    go(inv_dcd_kernel<11>);
  else
    go(inv_dcd_kernel<10>);
  HIP_CHECK(hipGetLastError());
}

void k_fft_free()
{
  for (auto &kv : g_fft) {
    HIP_CHECK(hipFree(kv.second.ksi));
    HIP_CHECK(hipFree(kv.second.rot));
  }
  g_fft.clear();
  if (g_ginv)
    HIP_CHECK(hipFree(g_ginv));
  g_ginv = nullptr;
}

__global__ void lift_i64_kernel(LimbSet dst, const int64_t *coef, unsigned logn, const ModConst *mc)
{
  const unsigned k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= (1u << logn))
    return;
  const unsigned l = blockIdx.y;
  const ModConst c = mc[dst.mod(l)];
  dst.limb(l, logn)[k] = lift_i64(coef[((size_t)(l / dst.per) << logn) + k], c);  // one coefficient row per group
}

void k_lift_i64(const LimbSet &dst, const int64_t *coef)
{
  hipLaunchKernelGGL(lift_i64_kernel, dim3((G.n + TPB - 1) / TPB, dst.count), dim3(TPB), 0, G.stream, dst, coef,
                     G.logn, G.dev.mc);
  HIP_CHECK(hipGetLastError());
}

// c0 = v pk0 + e0 + m, c1 = v pk1 + e1 (all NTT domain, lvl limbs).
__global__ void enc_kernel(uint64_t *c0, uint64_t *c1, const uint64_t *v, const uint64_t *e0, const uint64_t *e1,
                           const uint64_t *pk0, const uint64_t *pk1, const uint64_t *mp, unsigned logn,
                           const ModConst *mc)
{
  const size_t n = (size_t)1 << logn;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n)
    return;
  const ModConst m = mc[blockIdx.y];
  const size_t o = ((size_t)blockIdx.y << logn) + i;
  c0[o] = add_mod(add_mod(e0[o], mul_mod(v[o], pk0[o], m), m.q), mp[o], m.q);
  c1[o] = add_mod(e1[o], mul_mod(v[o], pk1[o], m), m.q);
}

void k_enc_combine(uint64_t *c0, uint64_t *c1, const uint64_t *v, const uint64_t *e0, const uint64_t *e1,
                   const uint64_t *pk0, const uint64_t *pk1, const uint64_t *m, unsigned lvl)
{
  hipLaunchKernelGGL(enc_kernel, dim3((G.n + TPB - 1) / TPB, lvl), dim3(TPB), 0, G.stream, c0, c1, v, e0, e1, pk0,
                     pk1, m, G.logn, G.dev.mc);
  HIP_CHECK(hipGetLastError());
}

__global__ void enc_batch_kernel(EncBatch bt, const uint64_t *vee, const uint64_t *pk0, const uint64_t *pk1,
                                 unsigned logn, unsigned lvl, const ModConst *mc)
{
  const size_t n = (size_t)1 << logn;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n)
    return;
  const unsigned e = blockIdx.z;
  const ModConst m = mc[blockIdx.y];
  const size_t o = ((size_t)blockIdx.y << logn) + i, w = (size_t)lvl << logn;
  const uint64_t *v = vee + 3 * e * w;
  const uint64_t c0 = add_mod(v[w + o], mul_mod(v[o], pk0[o], m), m.q);
  bt.c0[e][o] = bt.m[e] ? add_mod(c0, bt.m[e][o], m.q) : c0;  // m == nullptr: already in e0 (EncCoef)
  bt.c1[e][o] = add_mod(v[2 * w + o], mul_mod(v[o], pk1[o], m), m.q);
}

void k_enc_combine_batch(const EncBatch &b, unsigned k, const uint64_t *vee, const uint64_t *pk0,
                         const uint64_t *pk1, unsigned lvl)
{
  hipLaunchKernelGGL(enc_batch_kernel, dim3((G.n + TPB - 1) / TPB, lvl, k), dim3(TPB), 0, G.stream, b, vee, pk0, pk1,
                     G.logn, lvl, G.dev.mc);
  HIP_CHECK(hipGetLastError());
}

// The combine with m evaluated in NTT form from its coefficients: output k
// holds m(psi^(2 brev(k) + 1)) = sum_j r_j y^j with y = psi^((2 brev(k) + 1)
// 2^clog) (value j is coefficient j 2^clog), psi^e read as tw[brev(e mod n)]
// and negated for e >= n (psi^n = -1).  The noise can then be sampled and
// transformed before the plaintext exists (api.cpp: the speculative noise of
// the small-N step).  Four lanes share an output: lane b sums the terms
// j = 4a + b by Horner's rule in z = y^4 and multiplies by y^b, and the four
// meet by lane shuffles -- a quarter of the serial chain of one lane per
// output; each step's four values are read with uniform (scalar) loads of the
// by-value argument, and the lane picks its own.  Lane 0 of the four writes
// c0, lane 1 c1.  Every value is canonical, so the residues equal those of
// NTT(m) added by enc_batch_kernel.
__global__ void enc_batch_m_kernel(EncBatch bt, EncM em, const uint64_t *vee, const uint64_t *pk0,
                                   const uint64_t *pk1, unsigned logn, unsigned lvl, const ModConst *mc,
                                   const uint64_t *tw)
{
  const unsigned n = 1u << logn;
  const unsigned g = blockIdx.x * blockDim.x + threadIdx.x, i = g >> 2, b = g & 3;
  if (i >= n)
    return;
  const unsigned l = blockIdx.y, e = blockIdx.z;
  const ModConst m = mc[l];
  const size_t o = ((size_t)l << logn) + i, w = (size_t)lvl << logn;
  const uint64_t *v = vee + 3 * e * w;
  // the combine's noise and key words requested before the evaluation, whose
  // serial products they would otherwise wait behind (lane 0: e0, pk0; lane
  // 1: e1, pk1; lanes 2, 3 read lane 1's words, unused)
  const uint64_t nv = v[o], ne = v[(b == 0 ? 1 : 2) * w + o], nk = (b == 0 ? pk0 : pk1)[o];
  uint64_t mh = 0;
  const int r = em.row_of[e];
  if (r >= 0) {  // (uniform)
    const uint64_t *cv = em.v + ((size_t)r * lvl + l) * em.row;
    const unsigned br = __brev(i) >> (32 - logn);
    const unsigned ex = ((2 * br + 1) << em.clog) & (2 * n - 1);
    const uint64_t y0 = tw[(size_t)l * n + (__brev(ex & (n - 1)) >> (32 - logn))];
    const uint64_t y = ex >= n ? m.q - y0 : y0;
    const uint64_t y2 = mul_mod(y, y, m), y4 = mul_mod(y2, y2, m);
    uint64_t acc = 0;
    for (int a = (int)em.row / 4 - 1; a >= 0; a--) {
      const uint64_t c0v = cv[4 * a], c1v = cv[4 * a + 1], c2v = cv[4 * a + 2], c3v = cv[4 * a + 3];
      acc = add_mod(mul_mod(acc, y4, m), b == 0 ? c0v : b == 1 ? c1v : b == 2 ? c2v : c3v, m.q);
    }
    if (b)
      acc = mul_mod(acc, b == 1 ? y : b == 2 ? y2 : mul_mod(y2, y, m), m);
    mh = add_mod(acc, __shfl_xor(acc, 1), m.q);
    mh = add_mod(mh, __shfl_xor(mh, 2), m.q);
  } else if (bt.m[e] && b == 0) {
    mh = bt.m[e][o];
  }
  if (b == 0)
    bt.c0[e][o] = add_mod(add_mod(ne, mul_mod(nv, nk, m), m.q), mh, m.q);
  else if (b == 1)
    bt.c1[e][o] = add_mod(ne, mul_mod(nv, nk, m), m.q);
}

void k_enc_combine_m(const EncBatch &b, const EncM &em, unsigned k, const uint64_t *vee, const uint64_t *pk0,
                     const uint64_t *pk1, unsigned lvl)
{
  if (G.logn > 12 || em.row < 4 || em.row > EncM::MAXROW || (em.row & (em.row - 1)))
    gpqhe_die("k_enc_combine_m: %u values per row at n = %u", em.row, G.n);
  hipLaunchKernelGGL(enc_batch_m_kernel, dim3((4 * G.n + TPB - 1) / TPB, lvl, k), dim3(TPB), 0, G.stream, b, em, vee,
                     pk0, pk1, G.logn, lvl, G.dev.mc, G.dev.tw);
  HIP_CHECK(hipGetLastError());
}

// c0 = e - a s + m
__global__ void enc_sk_kernel(uint64_t *c0, const uint64_t *a, const uint64_t *e, const uint64_t *s,
                              const uint64_t *mp, unsigned logn, const ModConst *mc)
{
  const size_t n = (size_t)1 << logn;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n)
    return;
  const ModConst m = mc[blockIdx.y];
  const size_t o = ((size_t)blockIdx.y << logn) + i;
  c0[o] = add_mod(sub_mod(e[o], mul_mod(a[o], s[o], m), m.q), mp ? mp[o] : 0, m.q);
}

void k_enc_sk_combine(uint64_t *c0, const uint64_t *a, const uint64_t *e, const uint64_t *s, const uint64_t *m,
                      unsigned lvl)
{
  hipLaunchKernelGGL(enc_sk_kernel, dim3((G.n + TPB - 1) / TPB, lvl), dim3(TPB), 0, G.stream, c0, a, e, s, m,
                     G.logn, G.dev.mc);
  HIP_CHECK(hipGetLastError());
}

// evk digit: b = e - a s (+ [P]_q s' on limbs [lo, hi)), all nmod limbs.
__global__ void evk_kernel(uint64_t *b, const uint64_t *a, const uint64_t *e, const uint64_t *s,
                           const uint64_t *sp, unsigned lo, unsigned hi, unsigned logn, const ModConst *mc)
{
  const size_t n = (size_t)1 << logn;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n)
    return;
  const unsigned l = blockIdx.y;
  const ModConst m = mc[l];
  const size_t o = ((size_t)l << logn) + i;
  uint64_t r = sub_mod(e[o], mul_mod(a[o], s[o], m), m.q);
  if (l >= lo && l < hi)
    r = add_mod(r, mul_mod(m.pmod, sp[o], m), m.q);
  b[o] = r;
}

void k_evk_combine(uint64_t *b, const uint64_t *a, const uint64_t *e, const uint64_t *s, const uint64_t *sprime,
                   unsigned lo, unsigned hi)
{
  hipLaunchKernelGGL(evk_kernel, dim3((G.n + TPB - 1) / TPB, G.nmod), dim3(TPB), 0, G.stream, b, a, e, s, sprime,
                     lo, hi, G.logn, G.dev.mc);
  HIP_CHECK(hipGetLastError());
}

__device__ __forceinline__ unsigned auto_index(unsigned k, uint64_t g, unsigned logn)
{
  const uint64_t mask = (2ull << logn) - 1;
  const uint64_t e = ((2ull * brev_dev(k, logn) + 1) * g) & mask;
  return brev_dev((unsigned)(e >> 1), logn);
}

__global__ void automorph_kernel(uint64_t *out, const uint64_t *in, unsigned logn, uint64_t g)
{
  const size_t n = (size_t)1 << logn;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n)
    return;
  const size_t off = (size_t)blockIdx.y << logn;
  out[off + i] = in[off + auto_index((unsigned)i, g, logn)];
}

void k_automorph(uint64_t *out, const uint64_t *in, unsigned nlimbs, uint64_t g)
{
  hipLaunchKernelGGL(automorph_kernel, dim3((G.n + TPB - 1) / TPB, nlimbs), dim3(TPB), 0, G.stream, out, in,
                     G.logn, g);
  HIP_CHECK(hipGetLastError());
}

__global__ void square_kernel(uint64_t *out, const uint64_t *in, unsigned logn, const ModConst *mc)
{
  const size_t n = (size_t)1 << logn;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n)
    return;
  const size_t o = ((size_t)blockIdx.y << logn) + i;
  out[o] = mul_mod(in[o], in[o], mc[blockIdx.y]);
}

void k_square(uint64_t *out, const uint64_t *in, unsigned nlimbs)
{
  hipLaunchKernelGGL(square_kernel, dim3((G.n + TPB - 1) / TPB, nlimbs), dim3(TPB), 0, G.stream, out, in, G.logn,
                     G.dev.mc);
  HIP_CHECK(hipGetLastError());
}

__global__ void mul_pt_kernel(uint64_t *out, const uint64_t *a, const uint64_t *pt, unsigned logn, size_t ps,
                              const ModConst *mc)
{
  const size_t n = (size_t)1 << logn;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n)
    return;
  const ModConst m = mc[blockIdx.y];
  const size_t o = ((size_t)blockIdx.y << logn) + i;
  const size_t p = blockIdx.z * ps;
  out[p + o] = mul_mod(a[p + o], pt[o], m);
}

void k_mul_pt(uint64_t *out, const uint64_t *a, const uint64_t *pt, unsigned lvl, size_t pstride)
{
  hipLaunchKernelGGL(mul_pt_kernel, dim3((G.n + TPB - 1) / TPB, lvl, 2), dim3(TPB), 0, G.stream, out, a, pt,
                     G.logn, pstride, G.dev.mc);
  HIP_CHECK(hipGetLastError());
}

__global__ void add_pt_kernel(uint64_t *out, const uint64_t *a, const uint64_t *pt, unsigned logn, size_t ps,
                              const ModConst *mc)
{
  const size_t n = (size_t)1 << logn;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n)
    return;
  const ModConst m = mc[blockIdx.y];
  const size_t o = ((size_t)blockIdx.y << logn) + i;
  out[o] = add_mod(a[o], pt[o], m.q);
  out[ps + o] = a[ps + o];
}

void k_add_pt(uint64_t *out, const uint64_t *a, const uint64_t *pt, unsigned lvl, size_t pstride)
{
  hipLaunchKernelGGL(add_pt_kernel, dim3((G.n + TPB - 1) / TPB, lvl), dim3(TPB), 0, G.stream, out, a, pt, G.logn,
                     pstride, G.dev.mc);
  HIP_CHECK(hipGetLastError());
}

// ===========================================================================
// Basis conversion constants, cached per (kind, level) in device memory.
// ===========================================================================
// (UpTable / DownTable: tables.h)
static unsigned basis_qp(unsigned lvl, unsigned *mods)
{
  for (unsigned t = 0; t < lvl; t++)
    mods[t] = t;
  for (unsigned k = 0; k < G.K; k++)
    mods[lvl + k] = G.L + k;
  return lvl + G.K;
}


// Row length n2 of the fused kernels' 4-step split (n = n1 x n2).
static unsigned ks_logn2()
{
  return G.logn >= 17 ? 9 : G.logn >= 15 ? 8 : 7;
}

static std::map<unsigned, UpTable> g_up;

static UpTable &up_table(unsigned lvl)
{
  auto it = g_up.find(lvl);
  if (it != g_up.end())
    return it->second;
  if (G.alpha > 8)
    gpqhe_die("digit size alpha=%u > 8 unsupported", G.alpha);
  unsigned mods[GPQHE_MAXMOD];
  const unsigned nm = basis_qp(lvl, mods);
  const unsigned ndig = (lvl + G.alpha - 1) / G.alpha;
  std::vector<UpDigit> dig(ndig);
  std::vector<uint64_t> c((size_t)ndig * 8 * nm, 0);
  std::vector<double> cd((size_t)ndig * 8 * nm * 2, 0.0);
  for (unsigned j = 0; j < ndig; j++) {
    const unsigned lo = j * G.alpha, hi = std::min(lo + G.alpha, lvl);
    dig[j].lo = lo;
    dig[j].na = hi - lo;
    for (unsigned i = lo; i < hi; i++) {
      uint64_t hat = 1;
      for (unsigned i2 = lo; i2 < hi; i2++)
        if (i2 != i)
          hat = hm_mul_mod(hat, G.q[i2] % G.q[i], G.q[i]);
      dig[j].y[i - lo] = hm_inv_mod(hat, G.q[i]);
      dig[j].yp[i - lo] = (uint64_t)(((unsigned __int128)dig[j].y[i - lo] << 64) / G.q[i]);
      for (unsigned t = 0; t < nm; t++) {
        const uint64_t qt = G.q[mods[t]];
        uint64_t h = 1;
        for (unsigned i2 = lo; i2 < hi; i2++)
          if (i2 != i)
            h = hm_mul_mod(h, G.q[i2] % qt, qt);
        c[((size_t)j * 8 + (i - lo)) * nm + t] = hm_mul_mod(h, G.mc[mods[t]].r64, qt);  // Montgomery form
        cd[2 * (((size_t)j * 8 + (i - lo)) * nm + t)] = (double)h;
        cd[2 * (((size_t)j * 8 + (i - lo)) * nm + t) + 1] = (double)h / (double)qt;
      }
    }
  }
  std::vector<uint64_t> ysc(2 * (size_t)lvl);
  for (unsigned i = 0; i < lvl; i++) {
    const UpDigit &d = dig[i / G.alpha];
    const uint64_t w = hm_mul_mod(G.mc[i].ninv, d.y[i - d.lo], G.q[i]);
    ysc[2 * i] = w;
    ysc[2 * i + 1] = (uint64_t)(((unsigned __int128)w << 64) / G.q[i]);
  }
  UpTable tab;
  tab.ndig = ndig;
  tab.nm = nm;
  tab.f64 = G.twd != nullptr;
  for (unsigned t = 0; t < nm; t++)
    tab.f64 &= G.q[mods[t]] < (1ull << 51);
  HIP_CHECK(hipMalloc(&tab.cd, cd.size() * 8));
  HIP_CHECK(hipMemcpy(tab.cd, cd.data(), cd.size() * 8, hipMemcpyHostToDevice));
  HIP_CHECK(hipMalloc(&tab.ysc, ysc.size() * 8));
  HIP_CHECK(hipMemcpy(tab.ysc, ysc.data(), ysc.size() * 8, hipMemcpyHostToDevice));
  HIP_CHECK(hipMalloc(&tab.dig, ndig * sizeof(UpDigit)));
  HIP_CHECK(hipMalloc(&tab.c, c.size() * 8));
  HIP_CHECK(hipMemcpy(tab.dig, dig.data(), ndig * sizeof(UpDigit), hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(tab.c, c.data(), c.size() * 8, hipMemcpyHostToDevice));
  return g_up[lvl] = tab;
}

const UpTable &k_up_table(unsigned lvl)
{
  return up_table(lvl);
}


// D[p][j][t][k] = FBC(digit j of xc[p]) mod basis_t (coefficient domain);
// own limbs copy xc (the uniform NTT afterwards reproduces the NTT-domain
// limb exactly).  One thread per coefficient walks every target: the digit's
// y_i = x_i [(Qj/q_i)^-1] are formed once, each target sums y_i [Qj/q_i]_t
// 2^64 lazily in 128 bits and pays one Montgomery REDC.
// grid: (n / TPB, ndig, count).
__global__ void modup_kernel(uint64_t *D, const uint64_t *xc, unsigned logn, unsigned lvl, unsigned L, unsigned nm,
                             unsigned ndig, size_t x_stride, size_t d_stride, UpTable tab, const ModConst *mc)
{
  const size_t n = (size_t)1 << logn;
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n)
    return;
  const unsigned j = blockIdx.y, p = blockIdx.z;
  const UpDigit *dg = tab.dig + j;
  const unsigned lo = dg->lo, na = dg->na;
  const uint64_t *x = xc + p * x_stride;
  uint64_t *out = D + p * d_stride + (((size_t)j * nm) << logn) + k;
  uint64_t y[8];
#pragma unroll
  for (unsigned i = 0; i < 8; i++)
    if (i < na)
      y[i] = mul_shoup(x[((size_t)(lo + i) << logn) + k], dg->y[i], dg->yp[i], mc[lo + i].q);
  const uint64_t *cj = tab.c + (size_t)j * 8 * nm;
  for (unsigned t = 0; t < nm; t++) {
    uint64_t r;
    if (t >= lo && t < lo + na) {
      r = x[((size_t)t << logn) + k];
    } else {
      const ModConst mt = mc[basis_mod(t, lvl, L)];
      unsigned __int128 acc = 0;
#pragma unroll
      for (unsigned i = 0; i < 8; i++)
        if (i < na)
          acc += (unsigned __int128)y[i] * cj[i * nm + t];
      r = redc128((uint64_t)(acc >> 64), (uint64_t)acc, mt);
    }
    out[(size_t)t << logn] = r;
  }
}

void k_modup(uint64_t *D, const uint64_t *xc, unsigned count, size_t x_stride, size_t d_stride, unsigned lvl)
{
  UpTable &tab = up_table(lvl);
  ProfScope ps(KC_MODUP, 8.0 * G.n * count * (lvl + tab.ndig * tab.nm));
  hipLaunchKernelGGL(modup_kernel, dim3((G.n + TPB - 1) / TPB, tab.ndig, count), dim3(TPB), 0, G.stream, D, xc,
                     G.logn, lvl, G.L, tab.nm, tab.ndig, x_stride, d_stride, tab, G.dev.mc);
  HIP_CHECK(hipGetLastError());
}

// Key-switch inner product (NTT domain, basis_qp(lvl)):
//   s0 = sum_j D_j[t][perm k] evk_b[j][t][k] + [P] c0[t][perm k]  (t < lvl)
//   s1 = sum_j D_j[t][perm k] evk_a[j][t][k] + [P] c1[t][perm k]  (t < lvl)
// evk == null skips the digit sum; accumulate: acc += pt * s, else acc = s.
// grid: (n / TPB, nm, count).
__global__ void ks_inner_kernel(uint64_t *acc0, const uint64_t *D, unsigned logn, unsigned lvl, unsigned L,
                                unsigned nm, unsigned nmod, unsigned ndig, size_t d_stride, size_t acc_stride,
                                const uint64_t *evk, uint64_t g, const uint64_t *c0, const uint64_t *c1,
                                size_t c_stride, size_t c_pstride, const uint64_t *pt, int accumulate,
                                const ModConst *mc)
{
  const size_t n = (size_t)1 << logn;
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n)
    return;
  // grid (n/TPB, count, nm): basis slot slowest so one evk limb serves every
  // ciphertext of the chunk from L2 before the next limb is touched
  const unsigned p = blockIdx.y, t = blockIdx.z;
  const unsigned m = basis_mod(t, lvl, L);
  const ModConst mm = mc[m];
  const size_t src = g == 1 ? k : auto_index((unsigned)k, g, logn);
  uint64_t s0 = 0, s1 = 0;
  if (evk) {
    const uint64_t *d = D + p * d_stride + ((size_t)t << logn) + src;
    for (unsigned j = 0; j < ndig; j++) {
      const uint64_t dv = d[((size_t)j * nm) << logn];
      const uint64_t *eb = evk + (((size_t)(2 * j) * nmod + m) << logn);
      const uint64_t *ea = evk + (((size_t)(2 * j + 1) * nmod + m) << logn);
      s0 = add_mod(s0, mul_mod(dv, eb[k], mm), mm.q);
      s1 = add_mod(s1, mul_mod(dv, ea[k], mm), mm.q);
    }
  }
  if (t < lvl) {
    if (c0)
      s0 = add_mod(s0, mul_shoup(c0[p * c_stride + ((size_t)t << logn) + src], mm.pmod, mm.pmodp, mm.q), mm.q);
    if (c1)
      s1 = add_mod(s1, mul_shoup(c1[p * c_stride + ((size_t)t << logn) + src], mm.pmod, mm.pmodp, mm.q), mm.q);
  }
  uint64_t *o0 = acc0 + p * acc_stride + ((size_t)t << logn) + k;
  uint64_t *o1 = o0 + ((size_t)nm << logn);
  if (accumulate) {
    const uint64_t w = pt[((size_t)t << logn) + k];
    *o0 = add_mod(*o0, mul_mod(w, s0, mm), mm.q);
    *o1 = add_mod(*o1, mul_mod(w, s1, mm), mm.q);
  } else {
    *o0 = s0;
    *o1 = s1;
  }
  (void)c_pstride;
}

// he_gemv's diagonal sum in one launch: for each non-zero diagonal e,
//   acc0 += pt_e * (sum_j D_j[perm_e k] evk_e,b[j] + [P] x0[perm_e k])
//   acc1 += pt_e * (sum_j D_j[perm_e k] evk_e,a[j])          (rotations)
//   acc0 += pt_e * [P] x0[k], acc1 += pt_e * [P] x1[k]        (identity)
// with the hoisted ModUp D of x; replaces one ks_inner launch per diagonal.
// A block covers 64 coefficients of one basis slot with 8 diagonal lanes, one
// per wave (wave g sums diagonals g, g + 8, ...); the 8 partial sums meet in
// LDS.  The diagonal index is wave-uniform, so its key / plaintext pointers and
// Galois element come from the kernel arguments by scalar loads: per-lane reads
// of by-value arguments took ~3.5 us more per launch (scripts/ubench_small).
// grid: (n / 64, nm, jobs), 512 threads.
// sp.npoly > 0: the last z slice samples the next step's noise instead
// (SpecAttach): workgroup (x, y) of it covers coefficients [512 b, 512 b + 512)
// of noise poly b / (n / 512), b = y gridDim.x + x.
// Test switch GPQHE_SPEC_ATTACH_TAKE=0: no launch takes the attached
// speculative work, so api.cpp flush_gemvs runs its fallback launches (the
// path a disagreement between spec_attach's prediction and a launch's own
// eligibility test would take; tests/test_gpu_parity.py switch off-paths)
static bool spec_take()
{
  static const bool take = !(getenv("GPQHE_SPEC_ATTACH_TAKE") && atoi(getenv("GPQHE_SPEC_ATTACH_TAKE")) == 0);
  return take;
}

struct SpecSmp {
  LimbSet dst;
  ChachaKey key;
  uint64_t stream;
  unsigned npoly;
};
__global__ void __launch_bounds__(512) gemv_inner_kernel(GemvJobs jobs, unsigned logn, unsigned lvl, unsigned L,
                                                          unsigned nm, unsigned nmod, unsigned ndig,
                                                          const ModConst *mc, SpecSmp sp)
{
  if (sp.npoly && blockIdx.z == gridDim.z - 1) {
    const unsigned b = blockIdx.y * gridDim.x + blockIdx.x, bpp = (1u << logn) / 512;
    if (b < sp.npoly * bpp)
      enc_noise_store(sp.dst, logn, sp.key, sp.stream, mc, b / bpp, (b % bpp) * 512 + threadIdx.x);
    return;
  }
  __shared__ uint64_t part[2][8][64];
  // blockIdx.z: the job (gemvs queued together run in one launch)
  const GemvJob &job = jobs.j[blockIdx.z];
  uint64_t *acc = job.acc;
  const uint64_t *D = job.D, *x0 = job.x0, *x1 = job.x1, *y0 = job.y0, *y1 = job.y1;
  const GemvDiags &dg = job.dg;
  const int accumulate = job.accumulate;
  const unsigned c = threadIdx.x % 64, gl = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
  const size_t k = (size_t)blockIdx.x * 64 + c;
  const unsigned t = blockIdx.y;
  const unsigned m = basis_mod(t, lvl, L);
  const ModConst mm = mc[m];
  const size_t tl = (size_t)t << logn;
  uint64_t a0 = 0, a1 = 0;
  for (unsigned e = gl; e < dg.count; e += 8) {
    const uint64_t g = dg.g[e];
    const size_t src = g == 1 ? k : auto_index((unsigned)k, g, logn);
    uint64_t s0 = 0, s1 = 0;
    const uint64_t *evk = dg.evk[e];
    if (evk) {
      for (unsigned j = 0; j < ndig; j++) {
        const uint64_t dv = D[(((size_t)j * nm) << logn) + tl + src];
        s0 = add_mod(s0, mul_mod(dv, evk[(((size_t)(2 * j) * nmod + m) << logn) + k], mm), mm.q);
        s1 = add_mod(s1, mul_mod(dv, evk[(((size_t)(2 * j + 1) * nmod + m) << logn) + k], mm), mm.q);
      }
    }
    if (t < lvl) {
      const uint64_t v0 = y0 ? sub_mod(x0[tl + src], y0[tl + src], mm.q) : x0[tl + src];
      s0 = add_mod(s0, mul_shoup(v0, mm.pmod, mm.pmodp, mm.q), mm.q);
      if (!evk) {
        const uint64_t v1 = y1 ? sub_mod(x1[tl + src], y1[tl + src], mm.q) : x1[tl + src];
        s1 = add_mod(s1, mul_shoup(v1, mm.pmod, mm.pmodp, mm.q), mm.q);
      }
    }
    const uint64_t w = dg.pt[e][tl + k];
    a0 = add_mod(a0, mul_mod(w, s0, mm), mm.q);
    a1 = add_mod(a1, mul_mod(w, s1, mm), mm.q);
  }
  part[0][gl][c] = a0;
  part[1][gl][c] = a1;
  __syncthreads();
  if (gl < 2) {
    uint64_t r = 0;
#pragma unroll
    for (int i = 0; i < 8; i++)
      r = add_mod(r, part[gl][i][c], mm.q);
    uint64_t *o = acc + ((size_t)gl * nm << logn) + tl + k;
    *o = accumulate ? add_mod(r, *o, mm.q) : r;
  }
}

void k_gemv_inner_jobs(const GemvJobs &jobs, unsigned njobs, unsigned lvl)
{
  const unsigned nm = lvl + G.K, ndig = (lvl + G.alpha - 1) / G.alpha;
  if (njobs < 1 || njobs > GemvJobs::MAX)
    gpqhe_die("k_gemv_inner_jobs: %u jobs", njobs);
  double diags = 0;
  for (unsigned i = 0; i < njobs; i++)
    diags += jobs.j[i].dg.count;
  ProfScope ps(KC_GEMV_INNER, 8.0 * G.n * diags * (ndig * nm + 2 * nm + 2 * lvl));
  // the next step's noise sampling rides along in one more z slice (g_sa)
  SpecSmp sp{};
  if (g_sa.sample && spec_take() && G.n >= 512 && (size_t)g_sa.npoly * (G.n / 512) <= (size_t)(G.n / 64) * nm) {
    sp.dst = g_sa.noise;
    sp.key = G.key;
    sp.stream = g_sa.stream;
    sp.npoly = g_sa.npoly;
    g_sa.sample = false;
  }
  hipLaunchKernelGGL(gemv_inner_kernel, dim3(G.n / 64, nm, njobs + (sp.npoly ? 1 : 0)), dim3(512), 0, G.stream, jobs,
                     G.logn, lvl, G.L, nm, G.nmod, ndig, G.dev.mc, sp);
  HIP_CHECK(hipGetLastError());
}

void k_gemv_inner(uint64_t *acc, const uint64_t *D, const uint64_t *x0, const uint64_t *x1, unsigned lvl,
                  const GemvDiags &dg, bool accumulate)
{
  GemvJobs jobs;
  jobs.j[0] = GemvJob{acc, D, x0, x1, dg, accumulate ? 1 : 0};
  k_gemv_inner_jobs(jobs, 1, lvl);
}

// acc layout per ciphertext p: acc0 at acc + p*acc_stride, acc1 right after
// it (nm limbs later).
void k_ks_inner(uint64_t *acc, const uint64_t *D, unsigned count, size_t d_stride, size_t acc_stride,
                const uint64_t *evk, unsigned lvl, uint64_t g, const uint64_t *c0, const uint64_t *c1,
                size_t c_stride, const uint64_t *pt, bool accumulate)
{
  const unsigned nm = lvl + G.K, ndig = (lvl + G.alpha - 1) / G.alpha;
  // reads D and c0/c1 per ciphertext + the evk once, writes 2 nm limbs per ciphertext
  const double kb = 8.0 * G.n *
                    ((double)count * (ndig * nm * (evk ? 1 : 0) + (c0 ? lvl : 0) + (c1 ? lvl : 0) +
                                      (accumulate ? 5 : 2) * nm) + (evk ? 2.0 * ndig * nm : 0));
  ProfScope ps(KC_KS_INNER, kb);
  hipLaunchKernelGGL(ks_inner_kernel, dim3((G.n + TPB - 1) / TPB, count, nm), dim3(TPB), 0, G.stream, acc, D,
                     G.logn, lvl, G.L, nm, G.nmod, ndig, d_stride, acc_stride, evk, g, c0, c1, c_stride,
                     (size_t)0, pt, accumulate ? 1 : 0, G.dev.mc);
  HIP_CHECK(hipGetLastError());
}


// ===========================================================================
// Fused key switching for ciphertext batches (n = 2^13 .. 2^16).
//
//   y      = INTT(d2) with n^-1 (Qj/q_i)^-1 folded into the last pass
//   T1     = forward column pass of FBC_{j->t}(y)  (ks_cols_kernel; the
//            converted digit never reaches HBM)
//   acc    = sum_j NTTrows(T1[j][t]) evk_j[t] + P (d0, d1)   (ks_rows_kernel;
//            own-digit limbs come straight from the NTT-form d2)
// Block orders: ks_cols walks the targets fastest (a digit's y tile is reused
// from L2 by all its targets); ks_rows walks ciphertexts fastest and basis
// slots slowest (each evk tile and twiddle table is read from HBM once per
// chunk).
// ===========================================================================


template <int LOGT>
__global__ void __launch_bounds__(256) ks_cols_kernel(const uint64_t *ybuf, size_t y_stride, uint64_t *T1,
                                                       size_t t1_stride, unsigned logn, unsigned lvl, unsigned L,
                                                       unsigned nm, unsigned ndig, unsigned ngroups, UpTable tab,
                                                       Tw2 tw, const ModConst *mcs)
{
  constexpr int T = 1 << LOGT, C = 4096 / T, LEA = LOGT - 4, EA = 1 << LEA, CP = C + 1;
  __shared__ __attribute__((aligned(16))) uint64_t lds[T * CP];
  const unsigned n2 = 1u << (logn - LOGT);
  const unsigned tiles = n2 / C;
  unsigned grp, t;  // group = (p, j, tile) on one XCD; members = basis targets
  if (!xcd_group(nm, ngroups, grp, t))
    return;
  const unsigned tile = grp % tiles, pj = grp / tiles, p = pj / ndig, j = pj % ndig;
  const UpDigit *dg = tab.dig + j;
  const unsigned lo = dg->lo, na = dg->na;
  if (t >= lo && t < lo + na)
    return;  // own limb: the row pass reads it from the NTT-form d2
  const unsigned m = basis_mod(t, lvl, L);
  const ModConst mc = mcs[m];
  const uint64_t q = mc.q, q2 = 2 * q;
  const uint64_t *yb = ybuf + p * y_stride + ((size_t)lo << logn) + (size_t)tile * C;
  uint64_t cc[8];
#pragma unroll
  for (unsigned i = 0; i < 8; i++)
    cc[i] = i < na ? tab.c[((size_t)j * 8 + i) * nm + t] : 0;
  uint64_t *out = T1 + p * t1_stride + (((size_t)j * nm + t) << logn) + (size_t)tile * C;
  const uint64_t *tw2 = tw.fwd + ((size_t)m << (logn + 1));
  const int th = threadIdx.x;
#pragma unroll
  for (int it = 0; it < C / 16; it++) {
    const int item = th + 256 * it, c = item % C, l = item / C;
    uint64_t r[EA];
#pragma unroll
    for (int k = 0; k < EA; k++) {
      const size_t idx = (size_t)(l + 16 * k) * n2 + c;
      unsigned __int128 acc = 0;
#pragma unroll
      for (unsigned i = 0; i < 8; i++)
        if (i < na)
          acc += (unsigned __int128)yb[((size_t)i << logn) + idx] * cc[i];
      r[k] = redc128((uint64_t)(acc >> 64), (uint64_t)acc, mc);
    }
    fwd_stages<LEA>(r, tw2, T, LOGT - 1, q);
#pragma unroll
    for (int k = 0; k < EA; k++)
      lds[(l + 16 * k) * CP + c] = r[k];
  }
  __syncthreads();
  {
    const int c = th % C, g = th / C;
    uint64_t r[16];
#pragma unroll
    for (int k = 0; k < 16; k++)
      r[k] = lds[(16 * g + k) * CP + c];
    fwd_stages<4>(r, tw2, T + 16 * g, 3, q);
    const bool f64 = q < F64_QMAX && tw.fwdd;  // T1 is read lazily: doubles on FP64 moduli
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const uint64_t v = canon4(r[k], q, q2);
      out[(size_t)(16 * g + k) * n2 + c] = f64 ? (uint64_t)__double_as_longlong((double)v) : v;
    }
  }
}

// Multi-target variant for digits of at most 4 limbs: the block loads its
// (p, j, tile) digit values into registers once and converts them for NT
// targets in turn (the single-target kernel re-reads them through L2 for every
// target and waits on those loads most of its time).  Column tiles are double
// buffered in LDS, so one barrier per target suffices.
template <int LOGT, int NT, bool INVC, bool F64>
__global__ void __launch_bounds__(256, 2) ks_cols4_kernel(const uint64_t *ybuf, size_t y_stride, uint64_t *T1,
                                                           size_t t1_stride, unsigned logn, unsigned lvl,
                                                           unsigned L, unsigned nm, unsigned ndig, unsigned members,
                                                           unsigned ngroups, UpTable tab, Tw2 tw,
                                                           const ModConst *mcs)
{
  constexpr int T = 1 << LOGT, C = 4096 / T, LEA = LOGT - 4, EA = 1 << LEA, CP = C + 1, IT = C / 16;
  __shared__ __attribute__((aligned(16))) uint64_t lds[2][T * CP];
  const unsigned n2 = 1u << (logn - LOGT);
  const unsigned tiles = n2 / C;
  unsigned grp, mi;  // group = (p, j, tile) on one XCD; members = target batches
  if (!xcd_group(members, ngroups, grp, mi))
    return;
  const unsigned tile = grp % tiles, pj = grp / tiles, p = pj / ndig, j = pj % ndig;
  const UpDigit *dg = tab.dig + j;
  const unsigned lo = dg->lo, na = dg->na;
  if (mi * NT >= nm - na)
    return;
  const uint64_t *yb = ybuf + p * y_stride + ((size_t)lo << logn) + (size_t)tile * C;
  const int th = threadIdx.x;
  uint64_t y[IT][4][EA];
  if constexpr (!INVC) {
#pragma unroll
    for (int it = 0; it < IT; it++) {
      const int item = th + 256 * it, c = item % C, l = item / C;
      const unsigned vo = (unsigned)l * n2 + c;  // 32-bit per-thread offset, uniform bases
#pragma unroll
      for (int i = 0; i < 4; i++)
#pragma unroll
        for (int k = 0; k < EA; k++) {
          const uint64_t v = i < (int)na ? (yb + ((size_t)i << logn) + (size_t)(16 * k) * n2)[vo] : 0;
          y[it][i][k] = F64 ? (uint64_t)__double_as_longlong(f64_from_u52(v)) : v;
        }
    }
  } else {
    // the digit arrives after the inverse row pass (d2_rows_kernel): run the
    // inverse column pass with n^-1 [(Qj/q_i)^-1] here, limb by limb
    auto load_limb = [&](auto I) {
      constexpr int i = decltype(I)::value;
      if (i >= (int)na) {
#pragma unroll
        for (int it = 0; it < IT; it++)
#pragma unroll
          for (int k = 0; k < EA; k++)
            y[it][i][k] = 0;
        return;
      }
      const unsigned mi_ = lo + i;
      const uint64_t *src = yb + ((size_t)i << logn);
      if (i)
        __syncthreads();
      with_arith_t<F64>(mcs[mi_].q, mi_, logn, tw, [&](const auto &ar) {
        using A = std::decay_t<decltype(ar)>;
        using V = typename A::V;
        {
          const int c = th % C, g = th / C;
          const unsigned vo = (unsigned)(16 * g) * n2 + c;
          V r[16];
#pragma unroll
          for (int k = 0; k < 16; k++)
            r[k] = A::load((src + (size_t)k * n2)[vo]);
          ar.template inv<4>(r, T + 16 * g, 0);
#pragma unroll
          for (int k = 0; k < 16; k++)
            lds[0][(16 * g + k) * CP + c] = A::bits(r[k]);
        }
        __syncthreads();
#pragma unroll
        for (int it = 0; it < IT; it++) {
          const int item = th + 256 * it, c = item % C, l = item / C;
          V r[EA];
#pragma unroll
          for (int k = 0; k < EA; k++)
            r[k] = A::unbits(lds[0][(l + 16 * k) * CP + c]);
          ar.template inv<LEA>(r, T, 4);
#pragma unroll
          for (int k = 0; k < EA; k++)
            y[it][i][k] = F64 ? ar.canon_d(r[k]) : ar.canon(r[k]);  // (scaled by d2_rows)
        }
      });
    };
    load_limb(std::integral_constant<int, 0>{});
    load_limb(std::integral_constant<int, 1>{});
    load_limb(std::integral_constant<int, 2>{});
    load_limb(std::integral_constant<int, 3>{});
    __syncthreads();
  }
  for (int u = 0; u < NT; u++) {
    const unsigned ui = mi * NT + u;
    if (ui >= nm - na)
      break;
    const unsigned t = ui < lo ? ui : ui + na;  // skip the digit's own limbs
    const unsigned m = basis_mod(t, lvl, L);
    const ModConst mc = mcs[m];
    const uint64_t q = mc.q, q2 = 2 * q;
    uint64_t cc[4];
#pragma unroll
    for (int i = 0; i < 4; i++)
      cc[i] = i < (int)na ? tab.c[((size_t)j * 8 + i) * nm + t] : 0;
    uint64_t *buf = lds[u & 1];
    uint64_t *out = T1 + p * t1_stride + (((size_t)j * nm + t) << logn) + (size_t)tile * C;
    with_arith_t<F64>(q, m, logn, tw, [&](const auto &ar) {
      using A = std::decay_t<decltype(ar)>;
      using V = typename A::V;
#pragma unroll
      for (int it = 0; it < IT; it++) {
        const int item = th + 256 * it, c = item % C, l = item / C;
        V r[EA];
        bool done = false;
        if constexpr (F64 && std::is_same<A, ArF64>::value) {
          {
            double cw[4], cq[4];
#pragma unroll
            for (int i = 0; i < 4; i++) {
              cw[i] = i < (int)na ? tab.cd[2 * (((size_t)j * 8 + i) * nm + t)] : 0.0;
              cq[i] = i < (int)na ? tab.cd[2 * (((size_t)j * 8 + i) * nm + t) + 1] : 0.0;
            }
#pragma unroll
            for (int k = 0; k < EA; k++) {
              auto yd = [&](int i) { return __longlong_as_double((long long)y[it][i][k]); };
              const double v = fbc_term(yd(0), cw[0], cq[0], ar.q) + fbc_term(yd(1), cw[1], cq[1], ar.q) +
                               fbc_term(yd(2), cw[2], cq[2], ar.q);
              r[k] = f64_red(v, ar.q, ar.qinv) + fbc_term(yd(3), cw[3], cq[3], ar.q);  // |.| < 1.5 q
            }
            done = true;
          }
        }
        if (!done) {
#pragma unroll
          for (int k = 0; k < EA; k++) {
            unsigned __int128 acc = 0;
#pragma unroll
            for (int i = 0; i < 4; i++)
              acc += (unsigned __int128)y[it][i][k] * cc[i];
            r[k] = A::load(redc128((uint64_t)(acc >> 64), (uint64_t)acc, mc));
          }
        }
        ar.template fwd<LEA>(r, T, LOGT - 1);
#pragma unroll
        for (int k = 0; k < EA; k++)
          buf[(l + 16 * k) * CP + c] = A::bits(r[k]);
      }
      __syncthreads();
      const int c = th % C, g = th / C;
      const unsigned vo = (unsigned)(16 * g) * n2 + c;
      V r[16];
#pragma unroll
      for (int k = 0; k < 16; k++)
        r[k] = A::unbits(buf[(16 * g + k) * CP + c]);
      ar.template fwd<4>(r, T + 16 * g, 3);
#pragma unroll
      for (int k = 0; k < 16; k++)
        ST_STREAM(ar.store_lazy(r[k]), &(out + (size_t)k * n2)[vo]);  // T1 / conv: read lazily by the row passes
    });
    (void)q2;
  }
}

// Key layout used by ks_rows: inside every 2048-element row tile, element
// 8 th + k (the 8 consecutive residues thread th owns after the row pass)
// sits at k 256 + th, so each thread's key words are loaded coalesced.
__device__ __forceinline__ unsigned own_perm(unsigned idx)
{
  const unsigned e = idx & 2047;
  return (idx & ~2047u) + ((e & 7) << 8) + (e >> 3);
}

// Relinearization inner product with the forward row pass fused in front:
// for (basis slot t, 2048-element row tile, ciphertext p) and each digit j,
// the column-transformed limb T1[j][t] (own digit: the NTT-form d2 limb) gets
// its row pass and is multiplied into the Montgomery-form key; both
// accumulators stay in registers.  P (d0, d1) is added on the q limbs; limbs
// t >= drop_lo leave after the inverse row pass (input of dn_cols).
template <int LOGN2>
__global__ void __launch_bounds__(256, 3) ks_rows_kernel(const uint64_t *T1, size_t t1_stride, const uint64_t *d2n,
                                                       size_t d2_stride, D01Src d01,
                                                       const uint64_t *evkm, uint64_t *acc, size_t acc_stride,
                                                       unsigned logn, unsigned lvl, unsigned L, unsigned nm,
                                                       unsigned nmod, unsigned ndig, unsigned alpha, unsigned count,
                                                       unsigned drop_lo, Tw2 tw,
                                                       const ModConst *mcs)
{
  using T = Row8<LOGN2>;
  __shared__ __attribute__((aligned(16))) uint64_t lds[T::WORDS];
  const unsigned n1 = 1u << (logn - LOGN2);
  const unsigned tiles = n1 / T::R;
  unsigned grp, p;  // group = (basis slot t, tile) on one XCD; members = ciphertexts
  if (!xcd_group(count, nm * tiles, grp, p))
    return;
  const unsigned t = grp / tiles, tile = grp % tiles;
  const unsigned m = basis_mod(t, lvl, L);
  const ModConst mc = mcs[m];
  const uint64_t q = mc.q, q2 = 2 * q;
  const unsigned row0 = tile * T::R;
  const size_t toff = (size_t)row0 << LOGN2;  // tile offset inside a limb
  const int th = threadIdx.x, row = th / T::TA, l = th % T::TA, h = th % T::TA;
  // natural-layout tile <-> ownership (8 th + k) through the swizzled LDS tile
  auto load_own = [&](const uint64_t *src, uint64_t (&r)[8]) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int e = th + 256 * i;
      lds[T::at(e >> LOGN2, e & (T::N2 - 1))] = src[e];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 8; k++)
      r[k] = lds[T::at(row, 8 * h + k)];
  };
  auto store_own = [&](uint64_t *dst, const uint64_t (&r)[8]) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 8; k++)
      lds[T::at(row, 8 * h + k)] = r[k];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int e = th + 256 * i;
      dst[e] = lds[T::at(e >> LOGN2, e & (T::N2 - 1))];
    }
  };
  // 64-bit lazy accumulators in [0, 2q): each product v * evk_mont is reduced
  // by a REDC without its final correction (v, evk < q gives a result < 2q)
  uint64_t a0[8], a1[8];
#pragma unroll
  for (int k = 0; k < 8; k++)
    a0[k] = a1[k] = 0;
  auto mac = [&](uint64_t &a, uint64_t v, uint64_t w) {
    const uint64_t lo = v * w, hi = mulhi64(v, w);
    const uint64_t r = hi + mulhi64(lo * mc.qneg_inv, q) + (lo != 0);
    a = lazy_lt2q(a + r, q2);
  };
  with_arith(q, m, logn, tw, [&](const auto &ar) {
    using A = std::decay_t<decltype(ar)>;
    using V = typename A::V;
    constexpr bool F = std::is_same<A, ArF64>::value;  // FP64 moduli: plain key, FP64 products
    V f0[8], f1[8];
    for (unsigned j = 0; j < ndig; j++) {
      const uint64_t *eb = evkm + (((size_t)(2 * j) * nmod + m) << logn) + toff + th;
      const uint64_t *ea = evkm + (((size_t)(2 * j + 1) * nmod + m) << logn) + toff + th;
      V r[8];
      const bool own = t < lvl && t / alpha == j;
      if (own) {
        uint64_t v[8];
        load_own(d2n + p * d2_stride + ((size_t)t << logn) + toff, v);  // own digit: NTT-form d2
#pragma unroll
        for (int k = 0; k < 8; k++)
          r[k] = A::load(v[k]);
      } else {
        // converted limb from ks_cols (column pass done)
        const uint64_t *x = T1 + p * t1_stride + (((size_t)j * nm + t) << logn) + toff;
#pragma unroll
        for (int k = 0; k < 8; k++)
          r[k] = A::load_lazy(x[(row << LOGN2) + l + T::TA * k]);
        __syncthreads();
        rows8_fwd_raw<LOGN2>(r, lds, ar, n1 + row0);
      }
      if constexpr (F) {
        // |accumulator| grows by < 1.5 q per digit; fold it back every 4 digits
        const bool fold = (j & 3) == 3;
#pragma unroll
        for (int k = 0; k < 8; k++) {
          const double wb = (double)eb[256 * k], wa = (double)ea[256 * k];
          const double tb = f64_mulmod_h(r[k], wb, ar.q, ar.qinv);
          const double ta = f64_mulmod_h(r[k], wa, ar.q, ar.qinv);
          f0[k] = j ? f0[k] + tb : tb;
          f1[k] = j ? f1[k] + ta : ta;
          if (fold) {
            f0[k] = f64_red(f0[k], ar.q, ar.qinv);
            f1[k] = f64_red(f1[k], ar.q, ar.qinv);
          }
        }
      } else {
#pragma unroll
        for (int k = 0; k < 8; k++) {
          const uint64_t v = ar.canon(r[k]);
          mac(a0[k], v, eb[256 * k]);
          mac(a1[k], v, ea[256 * k]);
        }
      }
    }
    if constexpr (F) {
#pragma unroll
      for (int k = 0; k < 8; k++) {
        a0[k] = ar.canon(f0[k]);
        a1[k] = ar.canon(f1[k]);
      }
    } else {
#pragma unroll
      for (int k = 0; k < 8; k++) {
        a0[k] = a0[k] >= q ? a0[k] - q : a0[k];
        a1[k] = a1[k] >= q ? a1[k] - q : a1[k];
      }
      (void)f0;
      (void)f1;
    }
    if (t < lvl) {
      // round C ownership: words 8 h + k of the thread's row
      int pos[8];
#pragma unroll
      for (int k = 0; k < 8; k++)
        pos[k] = (row << LOGN2) + 8 * h + k;
      uint64_t c[8];
      d01_fetch8(d01, 2 * p, ((size_t)t << logn) + toff, pos, mc, c);
#pragma unroll
      for (int k = 0; k < 8; k++)
        a0[k] = add_mod(a0[k], mul_shoup(c[k], mc.pmod, mc.pmodp, q), q);
      d01_fetch8(d01, 2 * p + 1, ((size_t)t << logn) + toff, pos, mc, c);
#pragma unroll
      for (int k = 0; k < 8; k++)
        a1[k] = add_mod(a1[k], mul_shoup(c[k], mc.pmod, mc.pmodp, q), q);
    }
    uint64_t *o0 = acc + p * acc_stride + ((size_t)t << logn) + toff;
    uint64_t *o1 = o0 + ((size_t)nm << logn);
    if (t < drop_lo) {
      store_own(o0, a0);
      store_own(o1, a1);
      return;
    }
    // limb dropped by the following ModDown: inverse row pass here (the
    // registers hold round C's ownership); dn_cols finishes the INTT
    auto inv_store = [&](uint64_t *dst, const uint64_t (&a)[8]) {
      V r[8];
#pragma unroll
      for (int k = 0; k < 8; k++)
        r[k] = A::load(a[k]);
      __syncthreads();
      rows8_inv<LOGN2>(r, lds, ar, n1 + row0);
#pragma unroll
      for (int k = 0; k < 8; k++)
        dst[(row << LOGN2) + l + T::TA * k] = ar.canon(r[k]);
    };
    inv_store(o0, a0);
    inv_store(o1, a1);
  });
}

// ks_colsf_kernel takes the digit tile and all its targets (at most 12) when
// every modulus is on FP64 and the row length is one it is built for
// the mixed-set column kernel for `targets` targets per digit at T = 2^LOGT1
template <int LOGT1>
static bool colsm_ks_ok(unsigned targets)
{
  return GPQHE_COLSM && targets <= 8 && LOGT1 <= 7;
}

static bool ks_colsf_ok(const UpTable &tab, unsigned lvl)
{
  const unsigned na_min = lvl - (tab.ndig - 1) * G.alpha;
  return GPQHE_COLSF && FBC64_KS_INVC && tab.f64 && G.alpha <= 4 && G.logn >= 13 && G.logn <= 17 &&
         tab.nm - na_min <= (G.logn >= 14 ? 12u : 8u);
}

// ModUp of d2 (its INTT finished here when invc) into T1 [count][ndig][nm]:
// the digit's limbs converted to every other basis slot, forward column pass.
template <int LOGT1>
static void ks_cols_stage(const uint64_t *y, uint64_t *T1, unsigned count, unsigned lvl, bool invc)
{
  // invc: y holds only the inverse row pass of d2 (d2_rows_kernel, unscaled);
  // ks_cols4 runs the inverse column pass with the full n^-1 [(Qj/q_i)^-1]
  const UpTable &tab = up_table(lvl);
  const unsigned nm = tab.nm, ndig = tab.ndig, n = G.n;
  const size_t y_stride = (size_t)lvl * n, t1_stride = (size_t)ndig * nm * n;
  const Tw2 tw{G.tw2, G.itw2, G.twd, G.itwd};
  const unsigned tiles = n / 4096;
  const double own = (double)G.alpha * ndig;  // digit slots not converted (approx. for partial digits)
  {
    // reads the digit's alpha limbs once per target set (registers), writes
    // the converted + column-transformed limbs
    ProfScope ps(invc || G.alpha <= 4 ? KC_KS_COLS4 : KC_KS_COLS, 8.0 * n * count * ((double)lvl + ndig * nm - own));
    const unsigned ngroups = tiles * count * ndig;
    const unsigned na_min = lvl - (ndig - 1) * G.alpha;
    if (invc) {
      constexpr unsigned NT = 8;  // all targets of a digit tile: its INTT columns run once
      const unsigned members = (nm - na_min + NT - 1) / NT;
      auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(xcd_blocks(members, ngroups)), dim3(256), 0, G.stream, y, y_stride, T1,
                           t1_stride, G.logn, lvl, G.L, nm, ndig, members, ngroups, tab, tw, G.dev.mc);
      };
      if (ks_colsf_ok(tab, lvl)) {
        // up to 12 targets per block (the digit's column INTT once per tile)
        const int nt = nm - na_min <= 8 ? 8 : 12;
        ks_colsf_launch(LOGT1, nt, dim3(xcd_blocks(1, ngroups)), y, y_stride, T1, t1_stride, lvl, nm, ndig, 1,
                        ngroups, tab, tw);
      } else if (!tab.f64 && colsm_ks_ok<LOGT1>(nm - na_min)) {
        ks_colsm_launch(LOGT1, dim3(xcd_blocks(members, ngroups)), y, y_stride, T1, t1_stride, lvl, nm, ndig, members,
                        ngroups, tab, tw);
      } else {
        tab.f64 && FBC64_KS_INVC ? go(ks_cols4_kernel<LOGT1, NT, true, true>)
                                 : go(ks_cols4_kernel<LOGT1, NT, true, false>);
      }
    } else if (G.alpha <= 4) {
      constexpr unsigned NT = 4;
      const unsigned members = (nm - na_min + NT - 1) / NT;
      auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(xcd_blocks(members, ngroups)), dim3(256), 0, G.stream, y, y_stride, T1,
                           t1_stride, G.logn, lvl, G.L, nm, ndig, members, ngroups, tab, tw, G.dev.mc);
      };
      tab.f64 && FBC64_KS_NT4 ? go(ks_cols4_kernel<LOGT1, NT, false, true>)
                              : go(ks_cols4_kernel<LOGT1, NT, false, false>);
    } else {
      hipLaunchKernelGGL((ks_cols_kernel<LOGT1>), dim3(xcd_blocks(nm, ngroups)), dim3(256), 0, G.stream, y,
                         y_stride, T1, t1_stride, G.logn, lvl, G.L, nm, ndig, ngroups, tab, tw, G.dev.mc);
    }
  }
  HIP_CHECK(hipGetLastError());
}

template <int LOGT1, int LOGN2>
static void ks_fused_launch(const uint64_t *y, uint64_t *T1, const uint64_t *d2n, const D01Src &d01,
                            const uint64_t *evkm, uint64_t *acc, unsigned count, unsigned lvl, unsigned drop_lo,
                            bool invc)
{
  ks_cols_stage<LOGT1>(y, T1, count, lvl, invc);
  const UpTable &tab = up_table(lvl);
  const unsigned nm = tab.nm, ndig = tab.ndig, n = G.n;
  const size_t t1_stride = (size_t)ndig * nm * n, d2_stride = (size_t)lvl * n, acc_stride = 2 * (size_t)nm * n;
  const Tw2 tw{G.tw2, G.itw2, G.twd, G.itwd};
  // reads T1 (+ own d2 limbs, the four input limbs of d0/d1 on q limbs) per
  // ciphertext and the key once, writes acc
  ProfScope ps(KC_KS_ROWS, 8.0 * n * ((double)count * (ndig * nm + 4.0 * lvl + 2 * nm) + 2.0 * ndig * nm));
  hipLaunchKernelGGL((ks_rows_kernel<LOGN2>), dim3(xcd_blocks(count, nm * (n / 2048))), dim3(256), 0, G.stream, T1,
                     t1_stride, d2n, d2_stride, d01, evkm, acc, acc_stride, G.logn, lvl, G.L, nm, G.nmod, ndig,
                     G.alpha, count, drop_lo, tw, G.dev.mc);
  HIP_CHECK(hipGetLastError());
}

// d2 = a1 b1 of `count` pairs fused with the INTT's inverse row pass: block
// = (limb, pair, 2048-element row tile), limb-major (one modulus' twiddles
// hot at a time).  Writes the NTT-form d2 when asked (the own-digit limbs of ks_rows)
// and its inverse row pass (the column pass completes the INTT); replaces the
// tensor kernel and the separate row pass (d0, d1 are formed by their
// consumers, D01Src).
// ysc (split key switch with the INTT's column pass in ks_cols4): the ModUp
// factor n^-1 [(Qj/q_i)^-1]_{q_i} per limb is applied here, where the kernel
// waits on HBM with VALU to spare, instead of in the VALU-bound ks_cols4.
template <int LOGN2>
__global__ void __launch_bounds__(256) d2_rows_kernel(uint64_t *d2, uint64_t *y, const uint64_t *a,
                                                       const uint64_t *b, size_t in_stride, size_t in_pstride,
                                                       unsigned logn, unsigned lvl, unsigned count, Tw2 tw,
                                                       const ModConst *mcs, const uint64_t *ysc)
{
  using T = Row8<LOGN2>;
  __shared__ __attribute__((aligned(16))) uint64_t lds[T::WORDS];
  const unsigned n1 = 1u << (logn - LOGN2), tiles = n1 / T::R;
  const unsigned blk = blockIdx.x, limb = blk / (count * tiles), rem = blk - limb * count * tiles;
  const unsigned p = rem / tiles, tile = rem - p * tiles;
  const ModConst mc = mcs[limb];
  const unsigned row0 = tile * T::R;
  const size_t off = ((size_t)limb << logn) + ((size_t)row0 << LOGN2);
  // b null: the c1 of a ciphertext alone (the ModUp of he_gemv / he_rot
  // batches on prime sets without the all-FP64 form, k_modup_c1_split)
  const uint64_t *pa = a + p * in_stride + in_pstride + off, *pb = b ? b + p * in_stride + in_pstride + off : pa;
  // this thread's 8 consecutive words 8 th + k are exactly its round-C
  // elements of the inverse row pass: 16-byte loads, no transpose through LDS
  const int th = threadIdx.x, row = th / T::TA, l = th % T::TA;
  uint64_t A1[8], B1[8];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const ulonglong2 x = ((const ulonglong2 *)(pa + 8 * th))[i];
    A1[2 * i] = x.x;
    A1[2 * i + 1] = x.y;
    if (b) {
      const ulonglong2 z = ((const ulonglong2 *)(pb + 8 * th))[i];
      B1[2 * i] = z.x;
      B1[2 * i + 1] = z.y;
    }
  }
  uint64_t *yo = y + (size_t)p * lvl * ((size_t)1 << logn) + off;
  with_arith(mc.q, limb, logn, tw, [&](const auto &ar) {
    using A = std::decay_t<decltype(ar)>;
    typename A::V r[8];
    uint64_t raw[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
      if constexpr (std::is_same<A, ArF64>::value) {
        // exact FP64 product of canonical residues, |.| < 1.5 q (a valid
        // inverse-pass input); canonical only for the optional d2 copy
        r[k] = b ? f64_mulmod_h(f64_from_u52(A1[k]), f64_from_u52(B1[k]), ar.q, ar.qinv) : f64_from_u52(A1[k]);
        if (d2)
          raw[k] = ar.canon(r[k]);
        if (ysc) {
          // times s: |r| <= q/2 after the reduction, so with the recomputed
          // s / q the quotient is off by < 1/2 + 0.75 q 2^-52: |r s - .| < 0.9 q
          const double sd = f64_from_u52(ysc[2 * limb]);
          r[k] = f64_mulmod_h(f64_red(r[k], ar.q, ar.qinv), sd, ar.q, ar.qinv);
        }
      } else {
        raw[k] = b ? mul_mod(A1[k], B1[k], mc) : A1[k];
        r[k] = A::load(ysc ? mul_shoup(raw[k], ysc[2 * limb], ysc[2 * limb + 1], mc.q) : raw[k]);
      }
    }
    if (d2) {  // the NTT-form copy for the streaming ks_rows (the split key switch forms it from a, b)
      ulonglong2 *dn = (ulonglong2 *)(d2 + (size_t)p * lvl * ((size_t)1 << logn) + off + 8 * th);
#pragma unroll
      for (int i = 0; i < 4; i++)
        dn[i] = make_ulonglong2(raw[2 * i], raw[2 * i + 1]);
    }
    rows8_inv<LOGN2>(r, lds, ar, n1 + row0);
#pragma unroll
    for (int k = 0; k < 8; k++)
      // streaming store: the batch's row-pass output (256 pairs: 1 GiB) is read
      // back from HBM by ks_cols4 anyway (d2_rows 649 -> 641 us, 40.4k ->
      // 40.6k ct-mult/s, same box)
      ST_STREAM(ar.canon(r[k]), &yo[(row << LOGN2) + l + T::TA * k]);
  });
}

// d2_rows_kernel for the split key switch (ysc) when every limb is on an FP64
// modulus: a workgroup owns (limb, row tile) and a range of pairs; QN
// 256-thread quarters stream their own pairs (the next pair's a1, b1 words
// requested while the current one is transformed) and share the tile's
// inverse twiddles, staged once in LDS as 8-byte entries (RowTw, the quotient
// from the product: ArF64Row<., true>, as ntt_rows_q_kernel's inverse).  The
// per-tile kernel fetched every twiddle from L2 at every round and waited on
// one pair's loads at a time (sq_wait_any 0.49).  Same values: canonical
// outputs of the same exact residue arithmetic.
// ONE: y = INTT_rows(a1 x s) (b unused): the ModUp of a ciphertext's c1 alone
// (he_gemv / he_rot batches, k_modup_c1_split).
// Launch bound: hip-clang reads the second argument as amdgpu_waves_per_eu, so
// 2 QN = 4 waves per SIMD caps the kernel at 128 VGPRs; it needs 114-118 (QN =
// 2, LOGN2 7-9; 96-100 for ONE) with no spills (-Rpass-analysis=
// kernel-resource-usage), and two 512-thread workgroups per CU are its
// intended occupancy.
template <int LOGN2, int QN, bool ONE = false>
__global__ void __launch_bounds__(256 * QN, 2 * QN) d2_rows_q_kernel(uint64_t *y, const uint64_t *a, const uint64_t *b,
                                                                     size_t in_stride, size_t in_pstride,
                                                                     unsigned logn, unsigned lvl, unsigned count,
                                                                     unsigned members, Tw2 tw, const ModConst *mcs,
                                                                     const uint64_t *ysc)
{
  using T = Row8<LOGN2>;
  __shared__ __attribute__((aligned(16))) uint64_t rt[QN][T::WORDS];
  __shared__ __attribute__((aligned(16))) uint64_t rtw[RowTw<LOGN2>::ENTRIES];
  const unsigned n1 = 1u << (logn - LOGN2), tiles = n1 / T::R;
  unsigned grp, mi;  // group = (limb, tile) on one XCD; members = pair ranges
  if (!xcd_group(members, lvl * tiles, grp, mi))
    return;
  const unsigned pb0 = (unsigned)(((size_t)mi * count) / members), pb1 = (unsigned)(((size_t)(mi + 1) * count) / members);
  if (pb0 >= pb1)
    return;
  const unsigned limb = grp / tiles, tile = grp % tiles;
  const double q = (double)mcs[limb].q, qinv = 1.0 / q;
  const unsigned row0 = tile * T::R;
  const size_t off = ((size_t)limb << logn) + ((size_t)row0 << LOGN2);
  // (the pair stream wave-uniform: scalar stream bases, as ntt_rows_q_kernel)
  const int qi = NTT_ROWS_SQ ? (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 8) : (int)(threadIdx.x >> 8);
  const int th = threadIdx.x & 255, row = th / T::TA, l = th % T::TA;
  uint64_t *lq = rt[qi];
  const size_t o = (size_t)limb << (logn + 1);
  RowTw<LOGN2>::template stage<true>(rtw, (const uint64_t *)(tw.invd + o), n1 + row0, threadIdx.x, 256 * QN);
  ArF64 ar0{q, qinv, tw.fwdd + o, tw.invd + o, q < (double)F64_LAZY};
  const auto ar = row_policy<LOGN2, true>(ar0, rtw, (int64_t)T::R - (int64_t)(n1 + row0), rtw);
  const double sd = f64_from_u52(ysc[2 * limb]);
  // this thread's 8 consecutive words 8 th + k: its round-C elements
  auto fetch = [&](uint64_t (&A1)[8], uint64_t (&B1)[8], unsigned p) {
    const auto pa = (gptr<const u64x2>)(sgpr_ptr<NTT_ROWS_SQ>(a + p * in_stride + in_pstride + off) + 8u * th);
    const auto pb = (gptr<const u64x2>)(sgpr_ptr<NTT_ROWS_SQ>((ONE ? a : b) + p * in_stride + in_pstride + off) + 8u * th);
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const u64x2 x = pa[i];
      A1[2 * i] = x.x;
      A1[2 * i + 1] = x.y;
      if constexpr (!ONE) {
        const u64x2 z = pb[i];
        B1[2 * i] = z.x;
        B1[2 * i + 1] = z.y;
      }
    }
  };
  unsigned p = pb0 + qi;
  uint64_t nA[8], nB[8];
  if (p < pb1)
    fetch(nA, nB, p);
  __syncthreads();  // the staged twiddles
  for (; p < pb1; p += QN) {
    double r[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
      // exact FP64 product of canonical residues, then times the ModUp factor
      // s: |r| <= q/2 after the reduction, so with the recomputed s / q the
      // quotient is off by < 1/2 + 0.75 q 2^-52: |r s - .| < 0.9 q
      if constexpr (ONE)
        r[k] = f64_from_u52(nA[k]);
      else
        r[k] = f64_mulmod_h(f64_from_u52(nA[k]), f64_from_u52(nB[k]), q, qinv);
      r[k] = f64_mulmod_h(f64_red(r[k], q, qinv), sd, q, qinv);
    }
    if (p + QN < pb1)
      fetch(nA, nB, p + QN);  // the next pair's words, in flight meanwhile
    wave_sync();              // the previous pair's rounds have finished with the LDS tile
    rows8_inv<LOGN2>(r, lq, ar, n1 + row0, th);
    const auto yo = sgpr_ptr<NTT_ROWS_SQ>(y + (size_t)p * lvl * ((size_t)1 << logn) + off);
#pragma unroll
    for (int k = 0; k < 8; k++)
      ST_STREAM(ar.canon(r[k]), &yo[(unsigned)((row << LOGN2) + l + T::TA * k)]);
  }
}

bool k_ks_fused_ok()
{
  return ntt2_ok() && G.alpha <= 8 && G.K <= 4;  // K <= 4: the fused ModDown drops at most 5 limbs
}

// d2 = a1 b1 and its INTT: the inverse row pass (d2_rows_kernel), plus the
// column pass unless ks_cols4 runs it (cols = false).
template <int LOGT1, int LOGN2>
static void d2_intt_launch(uint64_t *d2, uint64_t *ybuf, const uint64_t *a, const uint64_t *b, size_t in_stride,
                           size_t in_pstride, unsigned count, unsigned lvl, const UpTable &tab, bool cols)
{
  const Tw2 tw{G.tw2, G.itw2, G.twd, G.itwd};
  const unsigned n = G.n;
  bool allf = !cols && !d2 && b && G.twd != nullptr && GPQHE_D2Q;
  for (unsigned i = 0; i < lvl; i++)
    allf &= G.q[i] < (1ull << 51);
  if (allf) {
    // ~12 pairs per quarter stream, as the NTT batch's row pass
    ProfScope ps(KC_D2_ROWS, 8.0 * n * lvl * count * 3);
    constexpr int QN = 2;
    const unsigned groups = lvl * (n / 2048), members = std::max(1u, count / (12 * QN));
    hipLaunchKernelGGL((d2_rows_q_kernel<LOGN2, QN>), dim3(xcd_blocks(members, groups)), dim3(256 * QN), 0, G.stream,
                       ybuf, a, b, in_stride, in_pstride, G.logn, lvl, count, members, tw, G.dev.mc,
                       (const uint64_t *)tab.ysc);
    HIP_CHECK(hipGetLastError());
    return;
  }
  {
    // reads a1, b1; writes its inverse row pass (and d2 when asked)
    ProfScope ps(KC_D2_ROWS, 8.0 * n * lvl * count * ((b ? 2 : 1) + 1 + (d2 ? 1 : 0)));
    hipLaunchKernelGGL((d2_rows_kernel<LOGN2>), dim3(lvl * count * (n / 2048)), dim3(256), 0, G.stream, d2, ybuf, a,
                       b, in_stride, in_pstride, G.logn, lvl, count, tw, G.dev.mc,
                       cols ? (const uint64_t *)nullptr : (const uint64_t *)tab.ysc);
  }
  if (!cols)  // the column pass runs inside ks_cols4 (invc)
    return;
  LimbSet ys{};
  ys.base = ybuf;
  ys.stride = (size_t)lvl * n;
  ys.per = lvl;
  ys.count = lvl * count;
  for (unsigned i = 0; i < lvl; i++)
    ys.mods[i] = (uint8_t)i;
  ProfScope ps(KC_NTT2_COLS_INV, 16.0 * n * ys.count);
  hipLaunchKernelGGL((ntt2_cols_kernel<LOGT1, true>), dim3(ys.count * (n / 4096)), dim3(256), 0, G.stream, ys, ys,
                     G.logn, tw, G.dev.mc, (const uint64_t *)tab.ysc);
  HIP_CHECK(hipGetLastError());
}

D01Src k_mul_keyswitch_fused(uint64_t *acc, uint64_t *d2, uint64_t *ybuf, uint64_t *T1, const uint64_t *a,
                             const uint64_t *b, size_t in_stride, size_t in_pstride, const uint64_t *evkm,
                             unsigned count, unsigned lvl, unsigned drop_lo)
{
  const UpTable &tab = up_table(lvl);
  // invc: d2's INTT column pass runs inside ks_cols4 (one block per digit tile
  // and all its targets: 31.4k vs 30.7k ct-mult/s at N=2^16, L=8 against a
  // separate ntt2_cols pass).  A digit with more than 8 targets (config 5: 12)
  // would repeat the column INTT per block (7.6k vs 7.8k), so it keeps the
  // separate pass.
  const unsigned ndig = (lvl + G.alpha - 1) / G.alpha, na_min = lvl - (ndig - 1) * G.alpha;
  const bool invc = G.alpha <= 4 && tab.nm - na_min <= 8;
  const D01Src src{a, b, in_stride, in_pstride};
  switch (G.logn) {
  case 13: d2_intt_launch<6, 7>(d2, ybuf, a, b, in_stride, in_pstride, count, lvl, tab, !invc); break;
  case 14: d2_intt_launch<7, 7>(d2, ybuf, a, b, in_stride, in_pstride, count, lvl, tab, !invc); break;
  case 15: d2_intt_launch<7, 8>(d2, ybuf, a, b, in_stride, in_pstride, count, lvl, tab, !invc); break;
  case 16: d2_intt_launch<8, 8>(d2, ybuf, a, b, in_stride, in_pstride, count, lvl, tab, !invc); break;
  case 17: d2_intt_launch<8, 9>(d2, ybuf, a, b, in_stride, in_pstride, count, lvl, tab, !invc); break;
  default: gpqhe_die("fused key switching needs 2^13 <= n <= 2^17");
  }
  switch (G.logn) {
  case 13: ks_fused_launch<6, 7>(ybuf, T1, d2, src, evkm, acc, count, lvl, drop_lo, invc); break;
  case 14: ks_fused_launch<7, 7>(ybuf, T1, d2, src, evkm, acc, count, lvl, drop_lo, invc); break;
  case 15: ks_fused_launch<7, 8>(ybuf, T1, d2, src, evkm, acc, count, lvl, drop_lo, invc); break;
  case 16: ks_fused_launch<8, 8>(ybuf, T1, d2, src, evkm, acc, count, lvl, drop_lo, invc); break;
  case 17: ks_fused_launch<8, 9>(ybuf, T1, d2, src, evkm, acc, count, lvl, drop_lo, invc); break;
  default: gpqhe_die("fused key switching needs 2^13 <= n <= 2^17");
  }
  return src;
}

// Montgomery-form copy of a key (x 2^64 mod q per limb), used by the fused
// inner product.
__global__ void to_mont_kernel(uint64_t *out, const uint64_t *in, unsigned logn, unsigned nmod, unsigned logn2,
                               int f64, const ModConst *mc)
{
  const size_t n = (size_t)1 << logn;
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n)
    return;
  const unsigned limb = blockIdx.y % nmod;
  const size_t base = (size_t)blockIdx.y << logn;
  const ModConst m = mc[limb];
  const size_t dst = logn2 ? own_perm((unsigned)k) : k;
  // moduli on the FP64 path multiply the plain key; the others use REDC
  out[base + dst] = f64 && m.q < F64_QMAX ? in[base + k] : mul_mod(in[base + k], m.r64, m);
}

// Montgomery copy (x 2^64 mod q) of nlimbs_total limbs (limb slot = index %
// nmod), laid out for ks_rows when the fused path serves this ring degree.
void k_to_mont(uint64_t *out, const uint64_t *in, unsigned nlimbs_total)
{
  const unsigned logn2 = k_ks_fused_ok() ? ks_logn2() : 0;
  hipLaunchKernelGGL(to_mont_kernel, dim3((G.n + TPB - 1) / TPB, nlimbs_total), dim3(TPB), 0, G.stream, out, in,
                     G.logn, G.nmod, logn2, G.twd ? 1 : 0, G.dev.mc);
  HIP_CHECK(hipGetLastError());
}

static std::map<std::pair<unsigned, int>, DownTable> g_down;

// mode 0: basis_qp(lvl) / P -> q_0..q_{lvl-1}         (key switching)
// mode 1: basis_qp(lvl) / (q_{lvl-1} P) -> q_0..q_{lvl-2} (fused rescale)
// mode 2: q_0..q_{lvl-1} / q_{lvl-1} -> q_0..q_{lvl-2}  (plain rescale)
static DownTable &down_table(unsigned lvl, int mode)
{
  auto key = std::make_pair(lvl, mode);
  auto it = g_down.find(key);
  if (it != g_down.end())
    return it->second;
  unsigned mods[GPQHE_MAXMOD];
  const unsigned nm = mode == 2 ? lvl : basis_qp(lvl, mods);
  if (mode == 2)
    for (unsigned t = 0; t < lvl; t++)
      mods[t] = t;
  const unsigned keep = mode == 0 ? lvl : lvl - 1, nd = nm - keep;
  std::vector<uint64_t> y(nd), yp(nd), c((size_t)nd * keep), dinv(keep), dinvp(keep);
  std::vector<double> cd((size_t)nd * keep * 2);
  for (unsigned d = 0; d < nd; d++) {
    const uint64_t qd = G.q[mods[keep + d]];
    uint64_t hat = 1;
    for (unsigned d2 = 0; d2 < nd; d2++)
      if (d2 != d)
        hat = hm_mul_mod(hat, G.q[mods[keep + d2]] % qd, qd);
    y[d] = hm_inv_mod(hat, qd);
    yp[d] = (uint64_t)(((unsigned __int128)y[d] << 64) / qd);
    for (unsigned t = 0; t < keep; t++) {
      const uint64_t qt = G.q[mods[t]];
      uint64_t h = 1;
      for (unsigned d2 = 0; d2 < nd; d2++)
        if (d2 != d)
          h = hm_mul_mod(h, G.q[mods[keep + d2]] % qt, qt);
      c[(size_t)d * keep + t] = hm_mul_mod(h, G.mc[mods[t]].r64, qt);  // Montgomery form
      cd[2 * ((size_t)d * keep + t)] = (double)h;
      cd[2 * ((size_t)d * keep + t) + 1] = (double)h / (double)qt;
    }
  }
  for (unsigned t = 0; t < keep; t++) {
    const uint64_t qt = G.q[mods[t]];
    uint64_t dp = 1;
    for (unsigned d = 0; d < nd; d++)
      dp = hm_mul_mod(dp, G.q[mods[keep + d]] % qt, qt);
    dinv[t] = hm_inv_mod(dp, qt);
    dinvp[t] = (uint64_t)(((unsigned __int128)dinv[t] << 64) / qt);
  }
  std::vector<uint64_t> ysc(2 * (size_t)nd);
  for (unsigned d = 0; d < nd; d++) {
    const unsigned md = mods[keep + d];
    const uint64_t w = hm_mul_mod(G.mc[md].ninv, y[d], G.q[md]);
    ysc[2 * d] = w;
    ysc[2 * d + 1] = (uint64_t)(((unsigned __int128)w << 64) / G.q[md]);
  }
  // folded factors of the split key switch (see DownTable)
  std::vector<uint64_t> ksc(nm), kps(2 * (size_t)nm), cf((size_t)nd * keep);
  std::vector<double> cdf((size_t)nd * keep * 2);
  for (unsigned t = 0; t < nm; t++) {
    const unsigned m = mods[t];
    ksc[t] = t < keep ? dinv[t] : ysc[2 * (t - keep)];
    kps[2 * t] = hm_mul_mod(G.mc[m].pmod, ksc[t], G.q[m]);
    kps[2 * t + 1] = (uint64_t)(((unsigned __int128)kps[2 * t] << 64) / G.q[m]);
  }
  for (unsigned d = 0; d < nd; d++)
    for (unsigned t = 0; t < keep; t++) {
      const uint64_t qt = G.q[mods[t]];
      const uint64_t di = hm_inv_mod(G.q[mods[keep + d]] % qt, qt);
      cf[(size_t)d * keep + t] = hm_mul_mod(di, G.mc[mods[t]].r64, qt);  // Montgomery form
      cdf[2 * ((size_t)d * keep + t)] = (double)di;
      cdf[2 * ((size_t)d * keep + t) + 1] = (double)di / (double)qt;
    }
  DownTable tab;
  tab.keep = keep;
  tab.nd = nd;
  auto up = [](auto *&dst, const auto &v) {
    HIP_CHECK(hipMalloc(&dst, v.size() * 8));
    HIP_CHECK(hipMemcpy(dst, v.data(), v.size() * 8, hipMemcpyHostToDevice));
  };
  up(tab.ksc, ksc);
  up(tab.kps, kps);
  up(tab.cf, cf);
  up(tab.cdf, cdf);
  tab.f64 = G.twd != nullptr;
  for (unsigned t = 0; t < nm; t++)
    tab.f64 &= G.q[mods[t]] < (1ull << 51);
  HIP_CHECK(hipMalloc(&tab.cd, cd.size() * 8));
  HIP_CHECK(hipMemcpy(tab.cd, cd.data(), cd.size() * 8, hipMemcpyHostToDevice));
  HIP_CHECK(hipMalloc(&tab.ysc, ysc.size() * 8));
  HIP_CHECK(hipMemcpy(tab.ysc, ysc.data(), ysc.size() * 8, hipMemcpyHostToDevice));
  HIP_CHECK(hipMalloc(&tab.y, nd * 8));
  HIP_CHECK(hipMalloc(&tab.yp, nd * 8));
  HIP_CHECK(hipMalloc(&tab.c, c.size() * 8));
  HIP_CHECK(hipMalloc(&tab.dinv, keep * 8));
  HIP_CHECK(hipMalloc(&tab.dinvp, keep * 8));
  HIP_CHECK(hipMemcpy(tab.y, y.data(), nd * 8, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(tab.yp, yp.data(), nd * 8, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(tab.c, c.data(), c.size() * 8, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(tab.dinv, dinv.data(), keep * 8, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(tab.dinvp, dinvp.data(), keep * 8, hipMemcpyHostToDevice));
  return g_down[key] = tab;
}

// conv[p][t][k] = sum_d y_d(x_d[k]) [Dprod/d]_t  (coefficient domain); one
// thread per coefficient walks every keep target (lazy 128-bit sums, REDC).
// grid: (n / TPB, npoly)
__global__ void down_conv_kernel(uint64_t *conv, const uint64_t *X, unsigned logn, unsigned lvl, unsigned L,
                                 size_t x_pstride, DownTable tab, const ModConst *mc)
{
  const size_t n = (size_t)1 << logn;
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n)
    return;
  const unsigned p = blockIdx.y;
  const uint64_t *x = X + p * x_pstride;
  uint64_t y[8];
#pragma unroll
  for (unsigned d = 0; d < 8; d++)
    if (d < tab.nd) {
      const unsigned bd = tab.keep + d;
      y[d] = mul_shoup(x[((size_t)bd << logn) + k], tab.y[d], tab.yp[d], mc[basis_mod(bd, lvl, L)].q);
    }
  uint64_t *o = conv + (((size_t)p * tab.keep) << logn) + k;
  for (unsigned t = 0; t < tab.keep; t++) {
    const ModConst mt = mc[basis_mod(t, lvl, L)];
    unsigned __int128 acc = 0;
#pragma unroll
    for (unsigned d = 0; d < 8; d++)
      if (d < tab.nd)
        acc += (unsigned __int128)y[d] * tab.c[(size_t)d * tab.keep + t];
    o[(size_t)t << logn] = redc128((uint64_t)(acc >> 64), (uint64_t)acc, mt);
  }
}

// out[p][t] = (X[p][t] - conv[p][t]) * Dprod^-1
__global__ void down_combine_kernel(uint64_t *out, uint64_t *out2, unsigned half, size_t out_pstride,
                                    const uint64_t *X, size_t x_pstride, const uint64_t *conv, unsigned logn,
                                    unsigned lvl, unsigned L, DownTable tab, const ModConst *mc)
{
  const size_t n = (size_t)1 << logn;
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n)
    return;
  const unsigned t = blockIdx.y, p = blockIdx.z;
  const uint64_t q = mc[basis_mod(t, lvl, L)].q;
  const size_t o = ((size_t)t << logn) + k;
  const uint64_t v = sub_mod(X[p * x_pstride + o], conv[(((size_t)p * tab.keep + t) << logn) + k], q);
  uint64_t *dst = p < half ? out + p * out_pstride : out2 + (p - half) * out_pstride;
  dst[o] = mul_shoup(v, tab.dinv[t], tab.dinvp[t], q);
}

// Fused small-N ModUp (n = 2^10 .. 2^12): digit j of c1 (NTT domain, x[p]) to
// basis slot t, in one workgroup: the inverse transform of each of the
// digit's limbs, its products y_i = x_i [(Q_j/q_i)^-1] and the sum
// sum_i y_i [Q_j/q_i]_t (128-bit, one REDC) in registers, then the forward
// transform mod q_t.  The digit's own slots are the input limbs themselves.
// Replaces copy + INTT + modup_kernel + NTT (four launches) with one; every
// value equals theirs (canonical residues at each step).
// grid: (nm, ndig, count), n / 8 threads.
// DIFF: input p is not in memory but the c1 difference of two fresh
// encryptions formed from their noise at load, (v_a pk1 + e1_a) - (v_b pk1 +
// e1_b) as enc_batch_kernel and the queued he_sub form it (the speculative
// ModUp of the small-N step, api.cpp SpecModup).
template <int LOGN, bool DIFF>
__device__ __forceinline__ void modup_small_body(uint64_t *D, const XPtrs &x1, size_t d_stride, unsigned lvl,
                                                 unsigned L, unsigned nm, const Tw2 &tw, const UpTable &tab,
                                                 const ModConst *mcs, const C1Diffs &cd, const uint64_t *pk1,
                                                 unsigned t, unsigned j, unsigned p, uint64_t *lds)
{
  constexpr int n = 1 << LOGN;
  const UpDigit *dg = tab.dig + j;
  const unsigned lo = dg->lo, na = dg->na;
  const uint64_t *x = x1.p[p];
  uint64_t *out = D + p * d_stride + (((size_t)j * nm + t) << LOGN);
  const int th = threadIdx.x;
  // input word e of limb ms
  auto xin = [&](unsigned ms, int e, const ModConst &m) -> uint64_t {
    const size_t o = ((size_t)ms << LOGN) + e;
    if constexpr (DIFF) {
      const size_t w = (size_t)lvl << LOGN;
      const uint64_t *a = cd.va[p], *b = cd.vb[p];
      const uint64_t ca = add_mod(a[2 * w + o], mul_mod(a[o], pk1[o], m), m.q);
      const uint64_t cb = add_mod(b[2 * w + o], mul_mod(b[o], pk1[o], m), m.q);
      return sub_mod(ca, cb, m.q);
    } else {
      return x[o];
    }
  };
  if (t >= lo && t < lo + na) {
    const ModConst m = mcs[t];
#pragma unroll
    for (int k = 0; k < 8; k++)
      out[th + k * (n / 8)] = xin(t, th + k * (n / 8), m);
    return;
  }
  unsigned __int128 acc[8];
#pragma unroll
  for (int k = 0; k < 8; k++)
    acc[k] = 0;
  const uint64_t *cj = tab.c + (size_t)j * 8 * nm;
  for (unsigned i = 0; i < na; i++) {
    const unsigned ms = lo + i;
    const ModConst mc = mcs[ms];
    const uint64_t cw = cj[i * nm + t], yw = dg->y[i], ywp = dg->yp[i];
    if (i)
      __syncthreads();
    with_arith(mc.q, ms, LOGN, tw, [&](const auto &ar) {
      using A = std::decay_t<decltype(ar)>;
      small_inv<LOGN>(
          ar, lds, [&](int, int e) { return A::load(xin(ms, e, mc)); },
          [&](int k, int, typename A::V a) {
            const uint64_t y = mul_shoup(ar.mulc(a, mc.ninv, mc.ninvp), yw, ywp, mc.q);
            acc[k] += (unsigned __int128)y * cw;
          });
    });
  }
  __syncthreads();
  const unsigned mt = basis_mod(t, lvl, L);
  const ModConst mc = mcs[mt];
  uint64_t r[8];
#pragma unroll
  for (int k = 0; k < 8; k++)
    r[k] = redc128((uint64_t)(acc[k] >> 64), (uint64_t)acc[k], mc);
  with_arith(mc.q, mt, LOGN, tw, [&](const auto &ar) {
    using A = std::decay_t<decltype(ar)>;
    small_fwd<LOGN>(
        ar, lds, [&](int k, int) { return A::load(r[k]); },
        [&](int, int e, typename A::V a) { out[e] = ar.canon(a); });
  });
}

template <int LOGN, bool DIFF>
__global__ void __launch_bounds__(512) modup_small_kernel(uint64_t *D, XPtrs x1, size_t d_stride, unsigned lvl,
                                                           unsigned L, unsigned nm, Tw2 tw, UpTable tab,
                                                           const ModConst *mcs, C1Diffs cd, const uint64_t *pk1)
{
  __shared__ __attribute__((aligned(16))) uint64_t lds[1 << LOGN];
  modup_small_body<LOGN, DIFF>(D, x1, d_stride, lvl, L, nm, tw, tab, mcs, cd, pk1, blockIdx.x, blockIdx.y, blockIdx.z,
                               lds);
}

// The speculative ModUp in two halves (ModupHalves; api.cpp spec_attach).
// First half, workgroup b < np lvl: difference p = b / lvl at input limb
// ms = b % lvl, formed at load as modup_small_body<., true> forms it; the
// value goes to its digit's own slot of D (modup_small_body's copy), and the
// inverse transform times [(Q_j/q_ms)^-1] to Y[p][ms] (the y its inverse
// callback forms).  Every other workgroup of modup_small_kernel ran this
// inverse transform again for its own target slot.
template <int LOGN>
__device__ __forceinline__ void modup_inv_half_body(const ModupHalves &mh, const UpTable &tab, const Tw2 &tw,
                                                    const ModConst *mcs, unsigned b, uint64_t *lds)
{
  const unsigned p = b / mh.lvl, ms = b % mh.lvl, nm = tab.nm;
  unsigned j = 0;
  while (j + 1 < tab.ndig && ms >= tab.dig[j + 1].lo)
    j++;
  const UpDigit *dg = tab.dig + j;
  const uint64_t yw = dg->y[ms - dg->lo], ywp = dg->yp[ms - dg->lo];
  const ModConst mc = mcs[ms];
  const size_t w = (size_t)mh.lvl << LOGN, o = (size_t)ms << LOGN;
  const uint64_t *va = mh.cd.va[p] + o, *vb = mh.cd.vb[p] + o, *pk = mh.pk1 + o;
  uint64_t *own = mh.D + p * mh.d_stride + (((size_t)j * nm + ms) << LOGN);
  uint64_t *y = mh.Y + (size_t)p * w + o;
  // every load first, the own-slot stores after: a store between two
  // elements' loads (which it may alias) kept the compiler from issuing the
  // next element's loads before it, one memory round trip per element
  // (down_fwd 13.7 -> 19 us with the loads inside small_inv's load callback).
  // small_inv's first round reads element 8 th + k into slot k for n = 2^10 ..
  // 2^12, so the values go in by slot.
  const int th = threadIdx.x;
  uint64_t xr[8];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const int e = 8 * th + k;
    const uint64_t ca = add_mod(va[2 * w + e], mul_mod(va[e], pk[e], mc), mc.q);
    const uint64_t cb = add_mod(vb[2 * w + e], mul_mod(vb[e], pk[e], mc), mc.q);
    xr[k] = sub_mod(ca, cb, mc.q);
  }
#pragma unroll
  for (int k = 0; k < 8; k++)
    own[8 * th + k] = xr[k];
  with_arith(mc.q, ms, LOGN, tw, [&](const auto &ar) {
    using A = std::decay_t<decltype(ar)>;
    small_inv<LOGN>(
        ar, lds, [&](int k, int) { return A::load(xr[k]); },
        [&](int, int e, typename A::V a) { y[e] = mul_shoup(ar.mulc(a, mc.ninv, mc.ninvp), yw, ywp, mc.q); });
  });
}

// Second half, grid (nm, ndig, np): slot t outside digit j, the conversion sum
// of Y in 128 bits, one REDC, the forward transform mod q_t (modup_small_body's
// tail, same order of terms).
template <int LOGN>
__global__ void __launch_bounds__(512) modup_fwd_half_kernel(ModupHalves mh, unsigned L, Tw2 tw, UpTable tab,
                                                              const ModConst *mcs)
{
  constexpr int n = 1 << LOGN;
  __shared__ __attribute__((aligned(16))) uint64_t lds[n];
  const unsigned t = blockIdx.x, j = blockIdx.y, p = blockIdx.z, nm = tab.nm;
  const UpDigit *dg = tab.dig + j;
  const unsigned lo = dg->lo, na = dg->na;
  if (t >= lo && t < lo + na)
    return;  // the first half wrote the digit's own slots
  const int th = threadIdx.x;
  const uint64_t *cj = tab.c + (size_t)j * 8 * nm;
  const uint64_t *y = mh.Y + ((size_t)p * mh.lvl << LOGN);
  unsigned __int128 acc[8];
#pragma unroll
  for (int k = 0; k < 8; k++)
    acc[k] = 0;
  for (unsigned i = 0; i < na; i++) {
    const uint64_t cw = cj[i * nm + t];
    const uint64_t *yi = y + ((size_t)(lo + i) << LOGN);
#pragma unroll
    for (int k = 0; k < 8; k++)
      acc[k] += (unsigned __int128)yi[th + k * (n / 8)] * cw;
  }
  const unsigned mt = basis_mod(t, mh.lvl, L);
  const ModConst mc = mcs[mt];
  uint64_t r[8];
#pragma unroll
  for (int k = 0; k < 8; k++)
    r[k] = redc128((uint64_t)(acc[k] >> 64), (uint64_t)acc[k], mc);
  uint64_t *out = mh.D + p * mh.d_stride + (((size_t)j * nm + t) << LOGN);
  with_arith(mc.q, mt, LOGN, tw, [&](const auto &ar) {
    using A = std::decay_t<decltype(ar)>;
    small_fwd<LOGN>(
        ar, lds, [&](int k, int) { return A::load(r[k]); },
        [&](int, int e, typename A::V a) { out[e] = ar.canon(a); });
  });
}

SpecAttach g_sa;
struct SpecNtt {  // down_inv_small_kernel's attached forward transforms
  LimbSet s;
};

// Fused small-N ModDown (+ rescale by its mode): output slot t of poly p in
// one workgroup: the inverse transform of each dropped limb, the conversion
// sum in registers, the forward transform mod q_t, and
// out = (X[t] - conv) [D^-1]_t.  Replaces INTT + down_conv + NTT +
// down_combine; X is only read (the in-place call of he_rescale is safe: each
// output word is written by the thread that read X at that word).
// grid: (keep, npoly), n / 8 threads.
template <int LOGN>
__global__ void __launch_bounds__(512) moddown_small_kernel(uint64_t *out, uint64_t *out2, unsigned half,
                                                             size_t out_pstride, const uint64_t *X, size_t x_pstride,
                                                             unsigned lvl, unsigned L, Tw2 tw, DownTable tab,
                                                             const ModConst *mcs)
{
  __shared__ __attribute__((aligned(16))) uint64_t lds[1 << LOGN];
  const unsigned t = blockIdx.x, p = blockIdx.y;
  const uint64_t *x = X + p * x_pstride;
  unsigned __int128 acc[8];
#pragma unroll
  for (int k = 0; k < 8; k++)
    acc[k] = 0;
  for (unsigned d = 0; d < tab.nd; d++) {
    const unsigned bd = tab.keep + d, md = basis_mod(bd, lvl, L);
    const ModConst mc = mcs[md];
    const uint64_t *src = x + ((size_t)bd << LOGN);
    const uint64_t cw = tab.c[(size_t)d * tab.keep + t], yw = tab.y[d], ywp = tab.yp[d];
    if (d)
      __syncthreads();
    with_arith(mc.q, md, LOGN, tw, [&](const auto &ar) {
      using A = std::decay_t<decltype(ar)>;
      small_inv<LOGN>(
          ar, lds, [&](int, int e) { return A::load(src[e]); },
          [&](int k, int, typename A::V a) {
            const uint64_t y = mul_shoup(ar.mulc(a, mc.ninv, mc.ninvp), yw, ywp, mc.q);
            acc[k] += (unsigned __int128)y * cw;
          });
    });
  }
  __syncthreads();
  const unsigned mt = basis_mod(t, lvl, L);
  const ModConst mc = mcs[mt];
  uint64_t r[8];
#pragma unroll
  for (int k = 0; k < 8; k++)
    r[k] = redc128((uint64_t)(acc[k] >> 64), (uint64_t)acc[k], mc);
  const uint64_t *xt = x + ((size_t)t << LOGN);
  uint64_t *dst = (p < half ? out + p * out_pstride : out2 + (p - half) * out_pstride) + ((size_t)t << LOGN);
  const uint64_t dinv = tab.dinv[t], dinvp = tab.dinvp[t];
  with_arith(mc.q, mt, LOGN, tw, [&](const auto &ar) {
    using A = std::decay_t<decltype(ar)>;
    small_fwd<LOGN>(
        ar, lds, [&](int k, int) { return A::load(r[k]); },
        [&](int, int e, typename A::V a) {
          dst[e] = mul_shoup(sub_mod(xt[e], ar.canon(a), mc.q), dinv, dinvp, mc.q);
        });
  });
}

// The same ModDown in two launches when two or more limbs are dropped (the
// batched he_gemv's / P q_top): the dropped limbs' inverse transforms run in
// workgroups of their own, side by side, instead of one after another inside
// one workgroup (the fused kernel's chain is nd + 1 transforms, this one's 2).
// down_inv_small_kernel, grid (nd, npoly): Y[p][d] = INTT(X[p][keep + d])
// [(D/d)^-1]_d, coefficient domain, canonical (the fused kernel's y).
// (1-D grid: nd npoly workgroups, then sn.count more that run the forward
// transform of limb b - nd npoly of sn.s in place: the next step's noise,
// SpecAttach)
template <int LOGN>
__global__ void __launch_bounds__(512) down_inv_small_kernel(uint64_t *Y, const uint64_t *X, size_t x_pstride,
                                                              unsigned lvl, unsigned L, Tw2 tw, DownTable tab,
                                                              const ModConst *mcs, unsigned npoly, SpecNtt sn)
{
  __shared__ __attribute__((aligned(16))) uint64_t lds[1 << LOGN];
  if (blockIdx.x >= tab.nd * npoly) {
    ntt_fwd_small_body<LOGN>(sn.s, tw, mcs, blockIdx.x - tab.nd * npoly, lds);
    return;
  }
  const unsigned d = blockIdx.x % tab.nd, p = blockIdx.x / tab.nd;
  const unsigned bd = tab.keep + d, md = basis_mod(bd, lvl, L);
  const ModConst mc = mcs[md];
  const uint64_t *src = X + p * x_pstride + ((size_t)bd << LOGN);
  uint64_t *y = Y + (((size_t)p * tab.nd + d) << LOGN);
  const uint64_t yw = tab.y[d], ywp = tab.yp[d];
  with_arith(mc.q, md, LOGN, tw, [&](const auto &ar) {
    using A = std::decay_t<decltype(ar)>;
    small_inv<LOGN>(
        ar, lds, [&](int, int e) { return A::load(src[e]); },
        [&](int, int e, typename A::V a) { y[e] = mul_shoup(ar.mulc(a, mc.ninv, mc.ninvp), yw, ywp, mc.q); });
  });
}

// down_fwd_small_kernel, grid (keep, npoly): conversion sum of Y to slot t,
// forward transform mod q_t, out = (X[t] - conv) [D^-1]_t, as the fused
// kernel (thread th holds elements th + k n/8 before a forward transform).
// (Rows y >= npoly of the grid: the next step's first ModUp half,
// modup_inv_half_body, workgroup (y - npoly) keep + x < mh.np mh.lvl.)
template <int LOGN>
__global__ void __launch_bounds__(512) down_fwd_small_kernel(uint64_t *out, uint64_t *out2, unsigned half,
                                                              size_t out_pstride, const uint64_t *Y,
                                                              const uint64_t *X, size_t x_pstride, unsigned lvl,
                                                              unsigned L, Tw2 tw, DownTable tab, const ModConst *mcs,
                                                              unsigned npoly, ModupHalves mh, UpTable utab)
{
  constexpr int n = 1 << LOGN;
  __shared__ __attribute__((aligned(16))) uint64_t lds[n];
  if (blockIdx.y >= npoly) {
    const unsigned b = (blockIdx.y - npoly) * gridDim.x + blockIdx.x;
    if (b < mh.np * mh.lvl)
      modup_inv_half_body<LOGN>(mh, utab, tw, mcs, b, lds);
    return;
  }
  const unsigned t = blockIdx.x, p = blockIdx.y;
  const int th = threadIdx.x;
  // X's words of this thread's outputs (the forward transform's last round
  // leaves elements 8 th + k with the thread), requested before the
  // conversion sum and the transform
  const uint64_t *xt = X + p * x_pstride + ((size_t)t << LOGN);
  uint64_t xk[8];
#pragma unroll
  for (int k = 0; k < 8; k++)
    xk[k] = xt[8 * th + k];
  unsigned __int128 acc[8];
#pragma unroll
  for (int k = 0; k < 8; k++)
    acc[k] = 0;
  for (unsigned d = 0; d < tab.nd; d++) {
    const uint64_t *y = Y + (((size_t)p * tab.nd + d) << LOGN);
    const uint64_t cw = tab.c[(size_t)d * tab.keep + t];
#pragma unroll
    for (int k = 0; k < 8; k++)
      acc[k] += (unsigned __int128)y[th + k * (n / 8)] * cw;
  }
  const unsigned mt = basis_mod(t, lvl, L);
  const ModConst mc = mcs[mt];
  uint64_t r[8];
#pragma unroll
  for (int k = 0; k < 8; k++)
    r[k] = redc128((uint64_t)(acc[k] >> 64), (uint64_t)acc[k], mc);
  uint64_t *dst = (p < half ? out + p * out_pstride : out2 + (p - half) * out_pstride) + ((size_t)t << LOGN);
  const uint64_t dinv = tab.dinv[t], dinvp = tab.dinvp[t];
  with_arith(mc.q, mt, LOGN, tw, [&](const auto &ar) {
    using A = std::decay_t<decltype(ar)>;
    small_fwd<LOGN>(
        ar, lds, [&](int k, int) { return A::load(r[k]); },
        [&](int k, int e, typename A::V a) {
          dst[e] = mul_shoup(sub_mod(xk[k], ar.canon(a), mc.q), dinv, dinvp, mc.q);
        });
  });
}

// ModUp of NTT-domain inputs x1.p[0..count) (lvl limbs each, e.g. c1 of a
// ciphertext, left unchanged) into D [count][ndig][nm] (NTT domain): one fused
// launch for n <= 2^12, else copy + INTT + modup_kernel + NTT.
void k_modup_ntt(uint64_t *D, const XPtrs &x1, unsigned count, size_t d_stride, unsigned lvl)
{
  UpTable &tab = up_table(lvl);
  const unsigned nm = tab.nm, ndig = tab.ndig, n = G.n;
  if (count > XPtrs::MAX)
    gpqhe_die("k_modup_ntt: %u inputs (max %u)", count, XPtrs::MAX);
  if (G.logn >= 10 && G.logn <= 12) {
    ProfScope ps(KC_MODUP_SMALL, 8.0 * n * count * ((double)ndig * lvl + ndig * nm));
    const Tw2 tw{G.tw2, G.itw2, G.twd, G.itwd};
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(nm, ndig, count), dim3(n / 8), 0, G.stream, D, x1, d_stride, lvl, G.L, nm, tw,
                         tab, G.dev.mc, C1Diffs{}, (const uint64_t *)nullptr);
    };
    if (G.logn == 12)
      go(modup_small_kernel<12, false>);
    else if (G.logn == 11)
      go(modup_small_kernel<11, false>);
    else
      go(modup_small_kernel<10, false>);
    HIP_CHECK(hipGetLastError());
    return;
  }
  const size_t w = (size_t)lvl * n;
  uint64_t *c1c = (uint64_t *)pool_alloc((size_t)count * w * 8);
  for (unsigned i = 0; i < count; i++)
    HIP_CHECK(hipMemcpyAsync(c1c + i * w, x1.p[i], w * 8, hipMemcpyDeviceToDevice, G.stream));
  unsigned mods[GPQHE_MAXMOD];
  for (unsigned l = 0; l < lvl; l++)
    mods[l] = l;
  auto limbs = [](uint64_t *base, const unsigned *md, unsigned per, unsigned groups, size_t stride) {
    LimbSet ls{};
    ls.base = base;
    ls.per = per;
    ls.count = per * groups;
    ls.stride = stride;
    for (unsigned i = 0; i < per; i++)
      ls.mods[i] = (uint8_t)md[i];
    return ls;
  };
  k_ntt(limbs(c1c, mods, lvl, count, w), true);
  k_modup(D, c1c, count, w, d_stride, lvl);
  basis_qp(lvl, mods);
  k_ntt(limbs(D, mods, nm, count * ndig, (size_t)nm * n), false);
  pool_free(c1c);
}

// k_modup_ntt of np c1 differences formed from encryption noise (C1Diffs) at
// load, n <= 2^12.
void k_modup_ntt_diffs(uint64_t *D, const C1Diffs &cd, unsigned np, size_t d_stride, const uint64_t *pk1,
                       unsigned lvl)
{
  UpTable &tab = up_table(lvl);
  const unsigned nm = tab.nm, ndig = tab.ndig, n = G.n;
  if (G.logn < 10 || G.logn > 12 || !np || np > GPQHE_MAXGRP)
    gpqhe_die("k_modup_ntt_diffs: %u inputs at n = %u", np, n);
  ProfScope ps(KC_MODUP_SMALL, 8.0 * n * np * ((double)ndig * lvl + ndig * nm));
  const Tw2 tw{G.tw2, G.itw2, G.twd, G.itwd};
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(nm, ndig, np), dim3(n / 8), 0, G.stream, D, XPtrs{}, d_stride, lvl, G.L, nm, tw, tab,
                       G.dev.mc, cd, pk1);
  };
  if (G.logn == 12)
    go(modup_small_kernel<12, true>);
  else if (G.logn == 11)
    go(modup_small_kernel<11, true>);
  else
    go(modup_small_kernel<10, true>);
  HIP_CHECK(hipGetLastError());
}

void k_modup_fwd_diffs(const ModupHalves &mh)
{
  UpTable &tab = up_table(mh.lvl);
  if (G.logn < 10 || G.logn > 12 || !mh.np || mh.np > GPQHE_MAXGRP)
    gpqhe_die("k_modup_fwd_diffs: %u inputs at n = %u", mh.np, G.n);
  ProfScope ps(KC_MODUP_SMALL, 8.0 * G.n * mh.np * ((double)mh.lvl + (double)tab.ndig * tab.nm));
  const Tw2 tw{G.tw2, G.itw2, G.twd, G.itwd};
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(tab.nm, tab.ndig, mh.np), dim3(G.n / 8), 0, G.stream, mh, G.L, tw, tab, G.dev.mc);
  };
  if (G.logn == 12)
    go(modup_fwd_half_kernel<12>);
  else if (G.logn == 11)
    go(modup_fwd_half_kernel<11>);
  else
    go(modup_fwd_half_kernel<10>);
  HIP_CHECK(hipGetLastError());
}

// X: npoly polynomials over basis_qp(lvl) (NTT domain, nm limbs each, stride
// x_pstride); their drop limbs are overwritten (INTT in place).  With out2,
// the first npoly/2 results go to out and the rest to out2 (two ciphertexts
// of one batched he_gemv flush).
void k_moddown(uint64_t *out, size_t out_pstride, uint64_t *X, size_t x_pstride, unsigned npoly, unsigned lvl,
               int mode, uint64_t *out2)
{
  DownTable &tab = down_table(lvl, mode);
  if (G.logn >= 10 && G.logn <= 12) {
    // one fused launch (moddown_small_kernel), or the inverse transforms of
    // two or more dropped limbs in workgroups of their own first
    ProfScope ps(KC_DOWN_SMALL, 8.0 * G.n * npoly * (tab.nd + 2.0 * tab.keep));
    const Tw2 tw{G.tw2, G.itw2, G.twd, G.itwd};
    const unsigned half = out2 ? npoly / 2 : npoly;
    if (tab.nd >= 2) {
      uint64_t *Y = (uint64_t *)pool_alloc(((size_t)npoly * tab.nd << G.logn) * 8);
      // the next step's speculative transforms and ModUp ride along (g_sa)
      SpecNtt sn{};
      unsigned xn = 0;
      if (g_sa.ntt && !g_sa.sample && spec_take()) {  // (transforms only of noise already sampled in stream order)
        sn.s = g_sa.noise;
        xn = g_sa.noise.count;
        g_sa.ntt = false;
      }
      // the next step's first ModUp half reads the noise transformed by the
      // inverse launch: only with it
      ModupHalves mh{};
      UpTable ut{};
      unsigned ry = 0;
      if (xn && g_sa.modup_inv) {
        mh = g_sa.mh;
        ut = up_table(mh.lvl);
        ry = (mh.np * mh.lvl + tab.keep - 1) / tab.keep;
        g_sa.modup_inv = false;
        g_sa.modup_inv_done = true;
      }
      auto go2 = [&](auto kinv, auto kfwd) {
        hipLaunchKernelGGL(kinv, dim3(tab.nd * npoly + xn), dim3(G.n / 8), 0, G.stream, Y, X, x_pstride, lvl, G.L, tw,
                           tab, G.dev.mc, npoly, sn);
        hipLaunchKernelGGL(kfwd, dim3(tab.keep, npoly + ry), dim3(G.n / 8), 0, G.stream, out, out2, half, out_pstride,
                           Y, X, x_pstride, lvl, G.L, tw, tab, G.dev.mc, npoly, mh, ut);
      };
      if (G.logn == 12)
        go2(down_inv_small_kernel<12>, down_fwd_small_kernel<12>);
      else if (G.logn == 11)
        go2(down_inv_small_kernel<11>, down_fwd_small_kernel<11>);
      else
        go2(down_inv_small_kernel<10>, down_fwd_small_kernel<10>);
      HIP_CHECK(hipGetLastError());
      pool_free(Y);
      return;
    }
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(tab.keep, npoly), dim3(G.n / 8), 0, G.stream, out, out2, half, out_pstride, X,
                         x_pstride, lvl, G.L, tw, tab, G.dev.mc);
    };
    if (G.logn == 12)
      go(moddown_small_kernel<12>);
    else if (G.logn == 11)
      go(moddown_small_kernel<11>);
    else
      go(moddown_small_kernel<10>);
    HIP_CHECK(hipGetLastError());
    return;
  }
  unsigned mods[GPQHE_MAXMOD];
  basis_qp(lvl, mods);
  LimbSet ds{};
  ds.base = X + ((size_t)tab.keep << G.logn);
  ds.stride = x_pstride;
  ds.per = tab.nd;
  ds.count = tab.nd * npoly;
  for (unsigned d = 0; d < tab.nd; d++)
    ds.mods[d] = (uint8_t)mods[tab.keep + d];
  k_ntt(ds, true);
  uint64_t *conv = (uint64_t *)pool_alloc((size_t)npoly * tab.keep * G.n * 8);
  {
  ProfScope ps(KC_DOWN_CONV, 8.0 * G.n * npoly * (tab.nd + tab.keep));
  if (tab.nd > 8)
    gpqhe_die("ModDown over %u moduli unsupported (max 8)", tab.nd);
  hipLaunchKernelGGL(down_conv_kernel, dim3((G.n + TPB - 1) / TPB, npoly), dim3(TPB), 0, G.stream, conv,
                     X, G.logn, lvl, G.L, x_pstride, tab, G.dev.mc);
  HIP_CHECK(hipGetLastError());
  }
  LimbSet cs{};
  cs.base = conv;
  cs.stride = (size_t)tab.keep * G.n;
  cs.per = tab.keep;
  cs.count = tab.keep * npoly;
  for (unsigned t = 0; t < tab.keep; t++)
    cs.mods[t] = (uint8_t)mods[t];
  k_ntt(cs, false);
  ProfScope ps(KC_DOWN_COMBINE, 8.0 * G.n * npoly * tab.keep * 3);
  hipLaunchKernelGGL(down_combine_kernel, dim3((G.n + TPB - 1) / TPB, tab.keep, npoly), dim3(TPB), 0, G.stream,
                     out, out2, out2 ? npoly / 2 : npoly, out_pstride, X, x_pstride, conv, G.logn, lvl, G.L, tab,
                     G.dev.mc);
  HIP_CHECK(hipGetLastError());
  pool_free(conv);
}

// ===========================================================================
// Fused ModDown for ciphertext batches (mode 0 / 1, n = 2^13 .. 2^16).
//
//   Y    = INTT(X drop limbs) with n^-1 [(Dprod/d)^-1]_d folded into the last
//          pass (in place)
//   conv = forward column pass of FBC_{drop->t}(Y)      (dn_cols_kernel)
//   out  = (X_t - NTTrows(conv_t)) Dprod^-1              (dn_rows_kernel)
// The converted polynomial never reaches HBM in coefficient form and the
// combine is the row pass's epilogue.
// ===========================================================================
// PRE (split key switch): the drop limbs arrive already scaled by
// n^-1 [(Dprod/d)^-1]_d (folded into the key) and conv takes the folded
// constants [d^-1]_t (conv x [Dprod^-1]_t: the kept slots' epilogue has no
// multiply); else the scaling runs here and conv uses [Dprod/d]_t.
template <int LOGT, int NT, bool X5, bool F64, bool PRE = false>
__global__ void __launch_bounds__(256, 2) dn_cols_kernel(const uint64_t *X, size_t x_pstride, size_t x_off, uint64_t *conv,
                                                          unsigned logn, unsigned lvl, unsigned L, unsigned members,
                                                          unsigned ngroups, DownTable tab, Tw2 tw,
                                                          const ModConst *mcs)
{
  constexpr int T = 1 << LOGT, C = 4096 / T, LEA = LOGT - 4, EA = 1 << LEA, CP = C + 1, IT = C / 16;
  __shared__ __attribute__((aligned(16))) uint64_t lds[T * CP];
  // fifth drop limb (mode 1 with K = 4), thread-private slots (it EA + k) 256 + th
  __shared__ uint64_t y5[X5 ? 4096 : 1];
  const unsigned n2 = 1u << (logn - LOGT);
  const unsigned tiles = n2 / C;
  unsigned grp, mi;  // group = (poly, tile) on one XCD; members = target batches
  if (!xcd_group(members, ngroups, grp, mi))
    return;
  const unsigned tile = grp % tiles, p = grp / tiles;
  const unsigned keep = tab.keep, nd = tab.nd;
  if (mi * NT >= keep)
    return;
  const uint64_t *yb = X + p * x_pstride + x_off + (size_t)tile * C;
  const int th = threadIdx.x;
  // Drop limbs arrive after the inverse row pass (ks_rows); the inverse column
  // pass with n^-1 [(Dprod/d)^-1]_d runs here.  Limbs 0..3 stay in registers.
  uint64_t y[IT][4][EA];
#pragma unroll
  for (int d = 0; d < 5; d++) {
    if (d >= (int)nd)
      break;
    const unsigned md = basis_mod(keep + d, lvl, L);
    const uint64_t w = tab.ysc[2 * d], wp = tab.ysc[2 * d + 1];
    const uint64_t *src = yb + ((size_t)d << logn);
    if (d)
      __syncthreads();
    with_arith_t<F64>(mcs[md].q, md, logn, tw, [&](const auto &ar) {
      using A = std::decay_t<decltype(ar)>;
      using V = typename A::V;
      {
        // 32-bit per-thread offset + uniform per-row base (scalar address
        // arithmetic; 64-bit per-element offsets cost 32 VGPRs and spilled)
        const int c = th % C, g = th / C;
        const unsigned vo = (unsigned)(16 * g) * n2 + c;
        V r[16];
#pragma unroll
        for (int k = 0; k < 16; k++)
          r[k] = A::load((src + (size_t)k * n2)[vo]);
        ar.template inv<4>(r, T + 16 * g, 0);
#pragma unroll
        for (int k = 0; k < 16; k++)
          lds[(16 * g + k) * CP + c] = A::bits(r[k]);
      }
      __syncthreads();
#pragma unroll
      for (int it = 0; it < IT; it++) {
        const int item = th + 256 * it, c = item % C, l = item / C;
        V r[EA];
#pragma unroll
        for (int k = 0; k < EA; k++)
          r[k] = A::unbits(lds[(l + 16 * k) * CP + c]);
        ar.template inv<LEA>(r, T, 4);
#pragma unroll
        for (int k = 0; k < EA; k++) {
          // FP64 conversion: canonical doubles; integer sums: canonical words
          const uint64_t v = PRE ? (F64 ? ar.canon_d(r[k]) : ar.canon(r[k]))
                                 : (F64 ? ar.mulc_d(r[k], w, wp) : ar.mulc(r[k], w, wp));
          if (d < 4)
            y[it][d < 4 ? d : 0][k] = v;
          else if constexpr (X5)
            y5[(it * EA + k) * 256 + th] = v;
        }
      }
    });
  }
#pragma unroll
  for (int d = 0; d < 4; d++)
    if (d >= (int)nd)
#pragma unroll
      for (int it = 0; it < IT; it++)
#pragma unroll
        for (int k = 0; k < EA; k++)
          y[it][d][k] = 0;
  __syncthreads();
  for (int u = 0; u < NT; u++) {
    const unsigned t = mi * NT + u;
    if (t >= keep)
      break;
    const unsigned m = basis_mod(t, lvl, L);
    const ModConst mc = mcs[m];
    const uint64_t q = mc.q, q2 = 2 * q;
    const uint64_t *ctab = PRE ? tab.cf : tab.c;
    const double *cdtab = PRE ? tab.cdf : tab.cd;
    uint64_t cc[5];
#pragma unroll
    for (int d = 0; d < 5; d++)
      cc[d] = d < (int)nd ? ctab[(size_t)d * keep + t] : 0;
    if (u)
      __syncthreads();  // the previous target's round B has read the tile
    uint64_t *out = conv + (((size_t)p * keep + t) << logn) + (size_t)tile * C;
    with_arith_t<F64>(q, m, logn, tw, [&](const auto &ar) {
      using A = std::decay_t<decltype(ar)>;
      using V = typename A::V;
#pragma unroll
      for (int it = 0; it < IT; it++) {
        const int item = th + 256 * it, c = item % C, l = item / C;
        V r[EA];
        bool done = false;
        if constexpr (F64 && std::is_same<A, ArF64>::value) {
          {
            // FP64 conversion: sources are canonical doubles, constants plain
            double cw[5], cq[5];
#pragma unroll
            for (int d = 0; d < 5; d++) {
              cw[d] = d < (int)nd ? cdtab[2 * ((size_t)d * keep + t)] : 0.0;
              cq[d] = d < (int)nd ? cdtab[2 * ((size_t)d * keep + t) + 1] : 0.0;
            }
#pragma unroll
            for (int k = 0; k < EA; k++) {
              auto yd = [&](int d) { return __longlong_as_double((long long)y[it][d][k]); };
              double v = fbc_term(yd(0), cw[0], cq[0], ar.q) + fbc_term(yd(1), cw[1], cq[1], ar.q) +
                         fbc_term(yd(2), cw[2], cq[2], ar.q);
              v = f64_red(v, ar.q, ar.qinv) + fbc_term(yd(3), cw[3], cq[3], ar.q);
              if constexpr (X5)
                v = f64_red(v + fbc_term(__longlong_as_double((long long)y5[(it * EA + k) * 256 + th]), cw[4],
                                         cq[4], ar.q),
                            ar.q, ar.qinv);
              r[k] = v;  // |v| < 2 q
            }
            done = true;
          }
        }
        if (!done) {
#pragma unroll
          for (int k = 0; k < EA; k++) {
            unsigned __int128 acc = 0;
#pragma unroll
            for (int d = 0; d < 4; d++)
              acc += (unsigned __int128)y[it][d][k] * cc[d];
            if constexpr (X5)
              acc += (unsigned __int128)y5[(it * EA + k) * 256 + th] * cc[4];
            r[k] = A::load(redc128((uint64_t)(acc >> 64), (uint64_t)acc, mc));
          }
        }
        ar.template fwd<LEA>(r, T, LOGT - 1);
#pragma unroll
        for (int k = 0; k < EA; k++)
          lds[(l + 16 * k) * CP + c] = A::bits(r[k]);
      }
      __syncthreads();
      const int c = th % C, g = th / C;
      const unsigned vo = (unsigned)(16 * g) * n2 + c;
      V r[16];
#pragma unroll
      for (int k = 0; k < 16; k++)
        r[k] = A::unbits(lds[(16 * g + k) * CP + c]);
      ar.template fwd<4>(r, T + 16 * g, 3);
#pragma unroll
      for (int k = 0; k < 16; k++)
        ST_STREAM(ar.store_lazy(r[k]), &(out + (size_t)k * n2)[vo]);  // T1 / conv: read lazily by the row passes
    });
    (void)q2;
  }
}

// Forward row pass of conv on 8-element row tiles with the combine as its
// epilogue.  The epilogue operand X_t is fetched at kernel start so its
// latency overlaps the row pass.  (The key switch added P (d0, d1) to X.)
// PRE: conv is pre-scaled (dn_cols' pre form: conv' = conv [D^-1]_t), so
// out = X [D^-1]_t - rowNTT(conv'), the same residue.
template <int LOGN2, bool PRE = false>
__global__ void __launch_bounds__(256) dn_rows_kernel(const uint64_t *conv, uint64_t *out, size_t out_pstride,
                                                       const uint64_t *X, size_t x_pstride, unsigned logn,
                                                       unsigned lvl, unsigned L, unsigned npoly, DownTable tab,
                                                       Tw2 tw, const ModConst *mcs)
{
  using T = Row8<LOGN2>;
  __shared__ __attribute__((aligned(16))) uint64_t lds[T::WORDS];
  const unsigned n1 = 1u << (logn - LOGN2);
  const unsigned tiles = n1 / T::R;
  const unsigned keep = tab.keep;
  unsigned grp, p;  // group = (target t, tile) on one XCD; members = polynomials
  if (!xcd_group(npoly, keep * tiles, grp, p))
    return;
  const unsigned t = grp / tiles, tile = grp % tiles;
  const unsigned m = basis_mod(t, lvl, L);
  const ModConst mc = mcs[m];
  const uint64_t q = mc.q;
  const unsigned row0 = tile * T::R;
  const size_t toff = ((size_t)t << logn) + ((size_t)row0 << LOGN2);
  const uint64_t *x = conv + (((size_t)p * keep) << logn) + toff;
  const uint64_t *xs = X + p * x_pstride + toff;
  const int th = threadIdx.x, row = th / T::TA, l = th % T::TA, h = th % T::TA;
  uint64_t xv[8];
#pragma unroll
  for (int i = 0; i < 8; i++)
    xv[i] = xs[wl_elem(i)];
  uint64_t cv[8];
  with_arith(q, m, logn, tw, [&](const auto &ar) {
    using A = std::decay_t<decltype(ar)>;
    typename A::V r[8];
#pragma unroll
    for (int k = 0; k < 8; k++)
      r[k] = A::load_lazy(x[(row << LOGN2) + l + T::TA * k]);  // conv (dn_cols, lazy)
    rows8_fwd<LOGN2>(r, cv, lds, ar, n1 + row0);
  });
  wave_sync();
#pragma unroll
  for (int k = 0; k < 8; k++)
    lds[T::at2(row, 8 * h, k)] = cv[k];
  wave_sync();
  const uint64_t dinv = tab.dinv[t], dinvp = tab.dinvp[t];
  uint64_t *o = out + p * out_pstride + toff;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int e = wl_elem(i);
    const uint64_t c = lds[T::wl(th, i)];
    if constexpr (PRE) {
      o[e] = sub_mod(mulc_canon(xv[i], dinv, dinvp, q), c, q);
    } else if (q < F64_QMAX) {
      // exact FP64 product: |X - conv| < q, the product < 1.25 q
      const double qd = (double)q, qinv = 1.0 / qd, di = f64_from_u52(dinv);
      o[e] = f64_canon(f64_mulmod(f64_from_u52(xv[i]) - f64_from_u52(c), di, di * qinv, qd), qd, qinv);
    } else {
      o[e] = mul_shoup(sub_mod(xv[i], c, q), dinv, dinvp, q);
    }
  }
}

// conv [npoly][keep] <- forward column pass of FBC(INTT(drop limbs)); the drop
// limbs of poly p sit at X + p x_pstride + x_off (inverse row pass done)
template <int LOGT1>
static void dn_cols_stage(uint64_t *conv, const uint64_t *X, size_t x_pstride, size_t x_off, unsigned npoly,
                          unsigned lvl, const DownTable &tab, bool pre)
{
  const unsigned n = G.n, keep = tab.keep, tiles = n / 4096;
  const Tw2 tw{G.tw2, G.itw2, G.twd, G.itwd};
  {
    // reads the nd row-transformed drop limbs, writes keep column-transformed
    // limbs; NT = 8: one block per (poly, tile) owns every keep target, so
    // the INTT columns run once
    ProfScope ps(KC_DN_COLS, 8.0 * n * npoly * (tab.nd + keep));
    constexpr unsigned NT = 8;
    const unsigned members = (keep + NT - 1) / NT, ngroups = npoly * tiles;
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(xcd_blocks(members, ngroups)), dim3(256), 0, G.stream, X, x_pstride, x_off,
                         conv, G.logn, lvl, G.L, members, ngroups, tab, tw, G.dev.mc);
    };
    if (pre) {
      if (tab.f64 && FBC64_DN && GPQHE_COLSF)
        dn_colsf_launch(LOGT1, dim3(xcd_blocks(members, ngroups)), X, x_pstride, x_off, conv, lvl, members, ngroups, tab,
                        tw);
      else if (tab.f64 && FBC64_DN)
        tab.nd <= 4 ? go(dn_cols_kernel<LOGT1, NT, false, true, true>) : go(dn_cols_kernel<LOGT1, NT, true, true, true>);
      else if (GPQHE_COLSM && LOGT1 <= 7)  // (T = 256 spilled 92 B/lane and ran slower: not used)
        dn_colsm_launch(LOGT1, dim3(xcd_blocks(members, ngroups)), X, x_pstride, x_off, conv, lvl, members, ngroups, tab,
                        tw);
      else
        tab.nd <= 4 ? go(dn_cols_kernel<LOGT1, NT, false, false, true>)
                    : go(dn_cols_kernel<LOGT1, NT, true, false, true>);
    } else if (tab.f64 && FBC64_DN) {
      tab.nd <= 4 ? go(dn_cols_kernel<LOGT1, NT, false, true>) : go(dn_cols_kernel<LOGT1, NT, true, true>);
    } else {
      tab.nd <= 4 ? go(dn_cols_kernel<LOGT1, NT, false, false>) : go(dn_cols_kernel<LOGT1, NT, true, false>);
    }
  }
  HIP_CHECK(hipGetLastError());
}

template <int LOGT1, int LOGN2>
static void dn_fused_launch(uint64_t *conv, uint64_t *out, size_t out_pstride, const uint64_t *X, size_t x_pstride,
                            unsigned npoly, unsigned lvl, const DownTable &tab, bool pre)
{
  const unsigned n = G.n, keep = tab.keep;
  const Tw2 tw{G.tw2, G.itw2, G.twd, G.itwd};
  dn_cols_stage<LOGT1>(conv, X, x_pstride, (size_t)keep << G.logn, npoly, lvl, tab, pre);
  // reads conv and X, writes out
  ProfScope ps(KC_DN_ROWS, 8.0 * n * npoly * keep * 3.0);
  hipLaunchKernelGGL((pre ? dn_rows_kernel<LOGN2, true> : dn_rows_kernel<LOGN2, false>),
                     dim3(xcd_blocks(npoly, keep * (n / 2048))), dim3(256), 0, G.stream, conv, out, out_pstride, X,
                     x_pstride, G.logn, lvl, G.L, npoly, tab, tw, G.dev.mc);
  HIP_CHECK(hipGetLastError());
}

// The inverse row pass of the dropped limbs dr before k_moddown_fused, each
// word times n^-1 [(D/d)^-1]_d (the DownTable's ysc): then the fused ModDown
// takes the pre-scaled column kernels (pre = true), as the split key switch's
// dropped slots do.  False (nothing launched) when the batched row form does
// not apply: then k_ntt_rows and pre = false.
bool k_ntt_rows_down(const LimbSet &dr, unsigned lvl, int mode, bool s79)
{
  const char *sw = getenv("GPQHE_DN_PRE");  // (read per call: tests switch it in-process)
  const bool on = !(sw && atoi(sw) == 0);
  const DownTable &tab = down_table(lvl, mode);
  if (!on || !dr.count || dr.per != tab.nd || dr.ngp)
    return false;
  bool ok;
  {
    ProfScope ps(KC_NTT3_ROWS_INV, 16.0 * G.n * dr.count);
    switch (G.logn) {
    case 13: ok = ntt_rows_launch<7>(true, dr, dr, tab.ysc); break;
    case 14: ok = ntt_rows_launch<7>(true, dr, dr, tab.ysc); break;
    case 15: ok = ntt_rows_launch<8>(true, dr, dr, tab.ysc); break;
    case 16: ok = s79 ? ntt_rows_launch<9>(true, dr, dr, tab.ysc) : ntt_rows_launch<8>(true, dr, dr, tab.ysc); break;
    case 17: ok = ntt_rows_launch<9>(true, dr, dr, tab.ysc); break;
    default: ok = false;
    }
  }
  HIP_CHECK(hipGetLastError());
  return ok;
}

void k_moddown_fused(uint64_t *out, size_t out_pstride, uint64_t *X, size_t x_pstride, unsigned npoly, unsigned lvl,
                     int mode, bool pre, bool s79)
{
  if (mode != 0 && mode != 1)
    gpqhe_die("fused ModDown: mode %d", mode);
  const DownTable &tab = down_table(lvl, mode);
  if (tab.nd > 5)
    gpqhe_die("fused ModDown over %u moduli unsupported (max 5)", tab.nd);
  uint64_t *conv = (uint64_t *)pool_alloc((size_t)npoly * tab.keep * G.n * 8);
  switch (G.logn) {
  case 13: dn_fused_launch<6, 7>(conv, out, out_pstride, X, x_pstride, npoly, lvl, tab, pre); break;
  case 14: dn_fused_launch<7, 7>(conv, out, out_pstride, X, x_pstride, npoly, lvl, tab, pre); break;
  case 15: dn_fused_launch<7, 8>(conv, out, out_pstride, X, x_pstride, npoly, lvl, tab, pre); break;
  case 16:
    if (s79)  // (the split key switch's 128 x 512 tiling: the column kernels' T = 128 forms)
      dn_fused_launch<7, 9>(conv, out, out_pstride, X, x_pstride, npoly, lvl, tab, pre);
    else
      dn_fused_launch<8, 8>(conv, out, out_pstride, X, x_pstride, npoly, lvl, tab, pre);
    break;
  case 17: dn_fused_launch<8, 9>(conv, out, out_pstride, X, x_pstride, npoly, lvl, tab, pre); break;
  default: gpqhe_die("fused ModDown needs 2^13 <= n <= 2^17");
  }
  pool_free(conv);
}

// ===========================================================================
// ct x ct relinearization [+ rescale] of `count` pairs, split key switch:
//   d2_rows  d2 = a1 b1, inverse row pass                  -> y
//   ks_cols4 inverse column pass, ModUp conversion, forward column pass -> T1
//   ksq<drop> key inner product of the dropped slots, inverse row pass -> accd
//   dn_cols  their INTT + conversion to the kept slots, forward column pass -> conv
//   ksq<keep> key inner product of the kept slots + P (d0, d1), minus
//             NTTrows(conv), times D^-1                       -> out
// The kept slots' accumulators never reach HBM.  Digits per key: 1 or 2.
// ===========================================================================
static bool split_ndig_ok(unsigned ndig)
{
  // the key tile (2 ndig x 16 KB) + the pair streams' padded row tiles (+ the
  // staged row twiddles for 1-2 digits) fit the LDS up to three digits;
  // longer keys take the streaming ks_rows path
  return ndig >= 1 && ndig <= 3;
}

bool k_mul_split_ok(unsigned lvl)
{
  const unsigned ndig = (lvl + G.alpha - 1) / G.alpha;
  return k_ks_fused_ok() && split_ndig_ok(ndig);
}

// Stages [s0, s1) of the split key switch (0 d2_rows, 1 ks_cols, 2
// ksq<drop>, 3 dn_cols, 4 ksq<keep>) on the engine stream; ws is the chunk's
// workspace (k_mul_split_ws_words), or null for all five stages from the pool.
template <int LOGT1, int LOGN2>
static void mul_split_launch(uint64_t *out, size_t out_pstride, const uint64_t *a, const uint64_t *b,
                             size_t in_stride, size_t in_pstride, const uint64_t *evkm, unsigned count, unsigned lvl,
                             bool rescale, uint64_t *ws, int s0, int s1)
{
  const UpTable &up = up_table(lvl);
  const DownTable &dn = down_table(lvl, rescale ? 1 : 0);
  const unsigned nm = up.nm, ndig = up.ndig, keep = dn.keep, nd = dn.nd, n = G.n;
  if (nd > 5)
    gpqhe_die("split key switch: ModDown over %u moduli unsupported (max 5)", nd);
  const unsigned na_min = lvl - (ndig - 1) * G.alpha;
  // the column INTT inside the ModUp kernel: up to 8 targets per digit, or 12
  // on the all-FP64 column kernel (config 5)
  const bool invc = G.alpha <= 4 && (nm - na_min <= 8 || ks_colsf_ok(up, lvl) || (!up.f64 && colsm_ks_ok<LOGT1>(nm - na_min)));
  // workspace: the caller's (k_mul_split_ws_words) or the pool's
  const bool own = !ws;
  if (own && (s0 != 0 || s1 != 5))
    gpqhe_die("split key switch: a stage range needs the caller's workspace");
  if (own)
    ws = (uint64_t *)pool_alloc(k_mul_split_ws_words(count, lvl, rescale) * 8);
  uint64_t *y = ws;
  uint64_t *T1 = y + (size_t)count * lvl * n;
  uint64_t *accd = T1 + (size_t)count * ndig * nm * n;
  uint64_t *conv = accd + (size_t)2 * count * nd * n;
  const D01Src d01{a, b, in_stride, in_pstride};
  const bool allf = up.f64 && dn.f64;
  for (int st = s0; st < s1; st++) {
    switch (st) {
    case 0: d2_intt_launch<LOGT1, LOGN2>(nullptr, y, a, b, in_stride, in_pstride, count, lvl, up, !invc); break;
    case 1: ks_cols_stage<LOGT1>(y, T1, count, lvl, invc); break;
    case 2: {
      // reads T1 (+ the inputs on a dropped q slot) per pair, the key once per
      // workgroup; writes the inverse row pass of the nd dropped slots
      ProfScope ps(KC_KSQ_DROP, 8.0 * n * count * ((double)ndig * nd + 2.0 * nd + (rescale ? 4.0 - 1.0 : 0.0)));
      ksq_run(LOGN2, ndig, allf, false, T1, d01, evkm, accd, (size_t)nd * n, nullptr, dn.ksc, dn.kps, count, lvl,
              nm, keep, nd);
      break;
    }
    case 3: dn_cols_stage<LOGT1>(conv, accd, (size_t)nd * n, 0, 2 * count, lvl, dn, true); break;
    case 4: {
      // reads T1 (ndig - 1 converted limbs), the four input limbs and the two
      // conv limbs per pair and kept slot; writes the two output limbs
      ProfScope ps(KC_KSQ_KEEP, 8.0 * n * count * keep * ((double)ndig - 1.0 + 4.0 + 2.0 + 2.0));
      ksq_run(LOGN2, ndig, allf, true, T1, d01, evkm, out, out_pstride, conv, dn.ksc, dn.kps, count, lvl, nm, 0,
              keep);
      break;
    }
    }
  }
  if (own)
    pool_free(ws);
}

size_t k_mul_split_ws_words(unsigned count, unsigned lvl, bool rescale)
{
  const unsigned ndig = (lvl + G.alpha - 1) / G.alpha, nm = lvl + G.K;
  const unsigned nd = G.K + (rescale ? 1 : 0), keep = rescale ? lvl - 1 : lvl;
  return (size_t)count * ((size_t)lvl + (size_t)ndig * nm + 2 * nd + 2 * keep) * G.n;
}

void k_mul_relin_split(uint64_t *out, size_t out_pstride, const uint64_t *a, const uint64_t *b, size_t in_stride,
                       size_t in_pstride, const uint64_t *evkm, unsigned count, unsigned lvl, bool rescale, uint64_t *ws,
                       int s0, int s1)
{
  switch (G.logn) {
  case 13: mul_split_launch<6, 7>(out, out_pstride, a, b, in_stride, in_pstride, evkm, count, lvl, rescale, ws, s0, s1); break;
  case 14: mul_split_launch<7, 7>(out, out_pstride, a, b, in_stride, in_pstride, evkm, count, lvl, rescale, ws, s0, s1); break;
  case 15: mul_split_launch<7, 8>(out, out_pstride, a, b, in_stride, in_pstride, evkm, count, lvl, rescale, ws, s0, s1); break;
  // 2^16 = 128 x 512: one NTT stage moves from the VALU-bound column kernels
  // to the row passes of the memory-bound ksq kernels (41.5-41.9k -> 42.0k
  // ct-mult/s against 256 x 256, same box)
  case 16: mul_split_launch<7, 9>(out, out_pstride, a, b, in_stride, in_pstride, evkm, count, lvl, rescale, ws, s0, s1); break;
  case 17: mul_split_launch<8, 9>(out, out_pstride, a, b, in_stride, in_pstride, evkm, count, lvl, rescale, ws, s0, s1); break;
  default: gpqhe_die("split key switch needs 2^13 <= n <= 2^17");
  }
}

// ModUp of the c1 of `count` ciphertexts (he_gemv / he_rot batches,
// gemv_win.hip) through the split key switch's first two kernels: y = the
// inverse row pass of c1 x n^-1 [(Q_j/q_i)^-1] (d2_rows_q_kernel<ONE> when
// every modulus is below 2^51, else d2_rows_kernel on c1 alone), then the
// column INTT, the conversion and the forward column pass (ks_cols) -> T1
// [count][ndig][nm][n] (own-digit slots not written), then the forward row
// pass of every converted slot: T1 ends in NTT form.  False when this ring has
// no split key switch.
template <int LOGT1, int LOGN2>
static bool modup_c1_launch(uint64_t *T1, uint64_t *ybuf, const uint64_t *x, size_t x_stride, size_t x_pstride,
                            unsigned count, unsigned lvl)
{
  const UpTable &up = up_table(lvl);
  const unsigned nm = up.nm, ndig = up.ndig, n = G.n;
  const unsigned na_min = lvl - (ndig - 1) * G.alpha;
  const bool invc = G.alpha <= 4 && (nm - na_min <= 8 || ks_colsf_ok(up, lvl) ||
                                     (!up.f64 && colsm_ks_ok<LOGT1>(nm - na_min)));
  if (!up.f64 || !invc || !GPQHE_D2Q || !G.twd) {
    // any other prime set (60-bit q_0 / P: the mixed-set column kernels):
    // the relinearization's first two stages on c1 alone
    d2_intt_launch<LOGT1, LOGN2>(nullptr, ybuf, x, nullptr, x_stride, x_pstride, count, lvl, up, !invc);
  } else {
    const Tw2 tw{G.tw2, G.itw2, G.twd, G.itwd};
    ProfScope ps(KC_D2_ROWS, 8.0 * n * lvl * count * 2);
    constexpr int QN = 2;
    const unsigned groups = lvl * (n / 2048), members = std::max(1u, count / (12 * QN));
    hipLaunchKernelGGL((d2_rows_q_kernel<LOGN2, QN, true>), dim3(xcd_blocks(members, groups)), dim3(256 * QN), 0,
                       G.stream, ybuf, x, (const uint64_t *)nullptr, x_stride, x_pstride, G.logn, lvl, count, members,
                       tw, G.dev.mc, (const uint64_t *)up.ysc);
    HIP_CHECK(hipGetLastError());
  }
  ks_cols_stage<LOGT1>(ybuf, T1, count, lvl, invc);
  for (unsigned j = 0; j < ndig; j++) {
    const unsigned lo = j * G.alpha, hi = std::min(lo + G.alpha, lvl);
    for (unsigned r = 0; r < 2; r++) {  // the slots before and after the digit
      const unsigned t0 = r ? hi : 0, t1 = r ? nm : lo;
      if (t0 >= t1)
        continue;
      LimbSet ls{};
      ls.base = T1 + ((size_t)j * nm + t0) * n;
      ls.per = t1 - t0;
      ls.count = ls.per * count;
      ls.stride = (size_t)ndig * nm * n;
      for (unsigned t = t0; t < t1; t++)
        ls.mods[t - t0] = (uint8_t)(t < lvl ? t : G.L + (t - lvl));
      ProfScope ps(KC_NTT3_ROWS_FWD, 16.0 * n * ls.count);
      ntt_rows_launch<LOGN2>(false, ls, ls);
      HIP_CHECK(hipGetLastError());
    }
  }
  return true;
}

bool k_modup_c1_split(uint64_t *T1, uint64_t *ybuf, const uint64_t *x, size_t x_stride, size_t x_pstride,
                      unsigned count, unsigned lvl)
{
  if (!k_ks_fused_ok() || (lvl + G.alpha - 1) / G.alpha > 3)
    return false;
  switch (G.logn) {
  case 13: return modup_c1_launch<6, 7>(T1, ybuf, x, x_stride, x_pstride, count, lvl);
  case 14: return modup_c1_launch<7, 7>(T1, ybuf, x, x_stride, x_pstride, count, lvl);
  case 15: return modup_c1_launch<7, 8>(T1, ybuf, x, x_stride, x_pstride, count, lvl);
  case 16: return modup_c1_launch<7, 9>(T1, ybuf, x, x_stride, x_pstride, count, lvl);
  case 17: return modup_c1_launch<8, 9>(T1, ybuf, x, x_stride, x_pstride, count, lvl);
  default: return false;
  }
}

// Benchmark input generator (oracle: poly_fill_uniform).
__global__ void fill_uniform_kernel(uint64_t *data, unsigned logn, unsigned nlimbs, uint64_t seed,
                                    const ModConst *mc)
{
  const size_t n = (size_t)1 << logn;
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n)
    return;
  const unsigned m = blockIdx.y;
  const size_t p = blockIdx.z;
  const uint64_t base = seed ^ (0x48454354520001ull + m);
  const uint64_t idx = p * n + k;
  const uint64_t v = splitmix64_mix(base + (idx + 1) * 0x9E3779B97F4A7C15ull);
  data[((p * nlimbs + m) << logn) + k] = v % mc[m].q;
}

void k_fill_uniform(uint64_t *data, size_t npolys, unsigned nlimbs, uint64_t seed)
{
  for (size_t p0 = 0; p0 < npolys; p0 += 65535) {
    const size_t cnt = std::min<size_t>(65535, npolys - p0);
    hipLaunchKernelGGL(fill_uniform_kernel, dim3((G.n + TPB - 1) / TPB, nlimbs, (unsigned)cnt), dim3(TPB), 0,
                       G.stream, data + p0 * nlimbs * G.n, G.logn, nlimbs, seed, G.dev.mc);
    HIP_CHECK(hipGetLastError());
  }
}

// ===========================================================================
// Tables
// ===========================================================================
void tables_upload()
{
  const size_t n = G.n, nm = G.nmod;
  std::vector<uint64_t> tw(nm * n), twp(nm * n), itw(nm * n), itwp(nm * n);
  for (unsigned m = 0; m < nm; m++) {
    const uint64_t q = G.q[m], psi = G.psi[m], ipsi = hm_inv_mod(psi, q);
    // powers in natural order, then permuted by bit reversal
    std::vector<uint64_t> pw(n), ipw(n);
    pw[0] = ipw[0] = 1;
    for (size_t k = 1; k < n; k++) {
      pw[k] = hm_mul_mod(pw[k - 1], psi, q);
      ipw[k] = hm_mul_mod(ipw[k - 1], ipsi, q);
    }
    for (size_t k = 0; k < n; k++) {
      const unsigned e = hm_brev((unsigned)k, G.logn);
      tw[m * n + k] = pw[e];
      itw[m * n + k] = ipw[e];
      twp[m * n + k] = (uint64_t)(((unsigned __int128)pw[e] << 64) / q);
      itwp[m * n + k] = (uint64_t)(((unsigned __int128)ipw[e] << 64) / q);
    }
  }
  HIP_CHECK(hipMalloc(&G.dev.mc, nm * sizeof(ModConst)));
  HIP_CHECK(hipMalloc(&G.dev.tw, nm * n * 8));
  HIP_CHECK(hipMalloc(&G.dev.twp, nm * n * 8));
  HIP_CHECK(hipMalloc(&G.dev.itw, nm * n * 8));
  HIP_CHECK(hipMalloc(&G.dev.itwp, nm * n * 8));
  HIP_CHECK(hipMemcpy(G.dev.mc, G.mc, nm * sizeof(ModConst), hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(G.dev.tw, tw.data(), nm * n * 8, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(G.dev.twp, twp.data(), nm * n * 8, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(G.dev.itw, itw.data(), nm * n * 8, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(G.dev.itwp, itwp.data(), nm * n * 8, hipMemcpyHostToDevice));
  std::vector<uint64_t> f2(2 * nm * n), i2(2 * nm * n);
  for (size_t k = 0; k < nm * n; k++) {
    f2[2 * k] = tw[k];
    f2[2 * k + 1] = twp[k];
    i2[2 * k] = itw[k];
    i2[2 * k + 1] = itwp[k];
  }
  HIP_CHECK(hipMalloc((void **)&G.tw2, 2 * nm * n * 8));
  HIP_CHECK(hipMalloc((void **)&G.itw2, 2 * nm * n * 8));
  HIP_CHECK(hipMemcpy((void *)G.tw2, f2.data(), 2 * nm * n * 8, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy((void *)G.itw2, i2.data(), 2 * nm * n * 8, hipMemcpyHostToDevice));
  // FP64 twiddles (w, w / q) for the moduli below 2^51 (others unused)
  std::vector<double> fd(2 * nm * n), id(2 * nm * n);
  for (size_t m = 0; m < nm; m++) {
    const double qd = (double)G.q[m];
    for (size_t k = 0; k < n; k++) {
      const size_t j = m * n + k;
      fd[2 * j] = (double)tw[j];
      fd[2 * j + 1] = (double)tw[j] / qd;
      id[2 * j] = (double)itw[j];
      id[2 * j + 1] = (double)itw[j] / qd;
    }
  }
  HIP_CHECK(hipMalloc((void **)&G.twd, 2 * nm * n * 8));
  HIP_CHECK(hipMalloc((void **)&G.itwd, 2 * nm * n * 8));
  HIP_CHECK(hipMemcpy((void *)G.twd, fd.data(), 2 * nm * n * 8, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy((void *)G.itwd, id.data(), 2 * nm * n * 8, hipMemcpyHostToDevice));
}

// ModUp / ModDown constant tables of every level, built at init rather than
// at their first use inside a caller's loop (each is a few small uploads).
void tables_prewarm()
{
  for (unsigned lvl = 1; lvl <= G.L; lvl++) {
    if (G.alpha <= 8)
      up_table(lvl);
    if (G.K + 1 <= 8)
      down_table(lvl, 0);
    if (lvl >= 2) {
      if (G.K + 1 <= 8)
        down_table(lvl, 1);
      down_table(lvl, 2);
    }
  }
}

void tables_free()
{
  HIP_CHECK(hipFree(G.dev.mc));
  HIP_CHECK(hipFree(G.dev.tw));
  HIP_CHECK(hipFree(G.dev.twp));
  HIP_CHECK(hipFree(G.dev.itw));
  HIP_CHECK(hipFree(G.dev.itwp));
  HIP_CHECK(hipFree((void *)G.tw2));
  HIP_CHECK(hipFree((void *)G.itw2));
  HIP_CHECK(hipFree((void *)G.twd));
  HIP_CHECK(hipFree((void *)G.itwd));
  G.tw2 = G.itw2 = nullptr;
  G.twd = G.itwd = nullptr;
  G.dev = DevTables{};
  for (auto &kv : g_up) {
    HIP_CHECK(hipFree(kv.second.dig));
    HIP_CHECK(hipFree(kv.second.c));
    HIP_CHECK(hipFree(kv.second.ysc));
    HIP_CHECK(hipFree(kv.second.cd));
  }
  g_up.clear();
  for (auto &kv : g_down) {
    HIP_CHECK(hipFree(kv.second.y));
    HIP_CHECK(hipFree(kv.second.yp));
    HIP_CHECK(hipFree(kv.second.c));
    HIP_CHECK(hipFree(kv.second.dinv));
    HIP_CHECK(hipFree(kv.second.dinvp));
    HIP_CHECK(hipFree(kv.second.ysc));
    HIP_CHECK(hipFree(kv.second.cd));
  }
  g_down.clear();
  k_fft_free();
}
