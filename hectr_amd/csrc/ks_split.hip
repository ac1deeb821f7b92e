// ks_split.hip - the split key switch's inner-product kernels (gfx950): the
// dropped basis slots (inverse row pass out) and the kept slots (ModDown
// epilogue fused).  Orchestrated by kernels.hip:mul_split_launch.
#include "ntt_device.h"

#include <algorithm>
#include <numeric>

// pair streams of ksq_kernel<drop> on FP64 prime sets (3: 168 VGPRs, 2: 256)
#ifndef KSQ_DROP_QN
#define KSQ_DROP_QN 3
#endif
#ifndef KSQ_KEEP_QN
#define KSQ_KEEP_QN 3
#endif
// three-digit keys (config 5), kept slots: staged forward row twiddles
#ifndef KSQ_C5_KEEP_LTW
#define KSQ_C5_KEEP_LTW 1
#endif
// three-digit keys, dropped slots: 2 = forward row twiddles staged (16 KB),
// the inverse ones from L2; 0 = both from L2
// grids of whole waves of workgroups (ksq_launch): same box, single stream,
// keep 1855 -> 1824-1848, drop 1159 -> 1105-1116 us per chunk; two streams
// (whose kernels fill each other's tails) unchanged.  0 off, 2 shorter ranges
// (slower)
#ifndef KSQ_FILL
#define KSQ_FILL 1
#endif
// the dropped slots' run-time lazy choice (ArF64Row LZC): -4 per element in
// the forward passes, one branch per call in the inverse ones (52 B/lane of
// spills; drop 1114 -> 1107 us per chunk, same box); -2 per element in both
// (44 B); -1 per call in both spilled 92 B (1196 -> 1258 us)
#ifndef KSQ_DROP_LZM
#define KSQ_DROP_LZM -4
#endif
// mixed prime sets: each arithmetic class's slot runs on its own kernel
#ifndef KSQ_SPLIT_AR
#define KSQ_SPLIT_AR 1
#endif
// the pair stream as a wave-uniform scalar (sgpr_ptr, below): bit 0 the
// dropped slots' kernel, bit 1 the kept slots'
#ifndef KSQ_DROP_PF1
#define KSQ_DROP_PF1 1
#endif
#ifndef KSQ_SCALAR_Q
#define KSQ_SCALAR_Q 3
#endif
#ifndef KSQ_C5_DROP_LTW
#define KSQ_C5_DROP_LTW 2
#endif

// ===========================================================================
// Key switch split at the ModDown boundary, key tile shared by quarter streams.
//
// One workgroup of QN x 256 threads owns a (basis slot t, 2048-element row
// tile) and a range of ciphertext pairs; each 256-thread quarter works through
// its own pairs (p = first + quarter + QN k) on its own LDS row tile, and the
// key words of every digit for (t, tile) are loaded into LDS once per
// workgroup and read by all quarters.  That keeps the key stationary (no
// per-pair key traffic) at QN waves per SIMD instead of the two that one
// 80 KB private key tile per 256 threads allows.
//
// Per pair and slot t: f0, f1 = sum over digits j of x_j (b_j, a_j)[t], x_j
// the forward row pass of the converted limb T1[j][t], or for the digit that
// owns a q limb t, d2 = a1 b1 itself (NTT domain, formed from the inputs: no
// d2 copy); on q limbs + P (d0, d1) with d0 = a0 b0, d1 = a0 b1 + a1 b0.
//   KEEP = false (slots t >= drop_lo, the limbs the ModDown divides out): the
//     inverse row pass of (f0, f1) goes to accd (dn_cols finishes the INTT
//     and converts).
//   KEEP = true (t < drop_lo): the ModDown epilogue follows at once, so the
//     accumulators never reach HBM: out = (f - NTTrows(conv)) D^-1 with conv
//     from dn_cols (the key switch of the dropped limbs ran first).
// The ModDown's constant factors are folded in (DownTable ksc / kps): the key
// tile is scaled by s_t as it is staged (kept slots: D^-1, so f arrives as
// f D^-1 and conv as conv D^-1 from dn_cols' folded constants; dropped slots:
// the INTT's n^-1 [(D/d)^-1]_d), and P (d0, d1) by [P s_t]_t.
// Inputs a, b are read here and by d2_rows only; out may alias them when each
// output word sits where the same pair's input word of the same slot was
// (he_mul(c, c, b)): the thread that writes it has read it.
// ===========================================================================
// (Measured non-levers, removed: non-temporal loads of the streamed operands
// -- keep 1853 -> 2140 us per chunk, a thread's two input halves share cache
// lines; loads one phase ahead in the kept slots' kernel -- 1868 -> 1960 /
// 2215 us, spills; one kernel per lazy-reduction policy with the slots
// launched in runs of one policy -- keep 1869, drop 1213 us.  DESIGN 5b.)

// the policy with its lazy-reduction choice fixed (LZ 0 / 1; -1 as it is)
template <int LZ>
__device__ __forceinline__ ArF64 with_lz(ArF64 a)
{
  if constexpr (LZ >= 0)
    a.lz = LZ != 0;
  return a;
}
template <int LZ>
__device__ __forceinline__ ArInt with_lz(const ArInt &a)
{
  return a;
}

// AR: the slots' arithmetic -- 1 every modulus below 2^51 (FP64; 3 / 4: and
// every one below / above 2^50, the lazy-reduction policy fixed), 2 every one
// integer, 0 chosen per slot at run time (both bodies in one kernel: its
// registers are the larger body's, so mixed prime sets launch each class's
// slot runs on their own kernel instead, KSQ_SPLIT_AR).  The slots are
// [t_lo, t_lo + t_n); conv (kept slots) holds cv_n slots per poly.
template <int LOGN2, int NDIG, int QN, int AR, bool KEEP, int LTW>
__global__ void __launch_bounds__(256 * QN, 1)
    ksq_kernel(const uint64_t *T1, size_t t1_stride, D01Src d01, const uint64_t *evkm, uint64_t *dst,
               size_t dst_pstride, const uint64_t *conv, const uint64_t *ksc, const uint64_t *kps, unsigned logn,
               unsigned lvl, unsigned L, unsigned nm, unsigned nmod, unsigned alpha, unsigned count, unsigned members,
               unsigned t_lo, unsigned t_n, unsigned cv_n, Tw2 tw, const ModConst *mcs)
{
  constexpr bool ALLF = AR == 1 || AR >= 3;
  using T = Row8<LOGN2>;
  constexpr int NX = KEEP ? NDIG - 1 : NDIG;  // converted limbs per slot at most
  __shared__ __attribute__((aligned(16))) uint64_t kl[2 * NDIG][2048];  // (b_j, a_j), order k 256 + th
  __shared__ __attribute__((aligned(16))) uint64_t rt[QN][T::WORDS];    // row tile per quarter
  // LTW: the tile's row-pass twiddles (RowTw), read by every quarter: with
  // every modulus on FP64 (ALLF) as 8-byte entries (forward, and inverse for
  // the dropped slots unless LTW == 2: those from L2), else the forward ones
  // as 16-byte entries
  constexpr bool GINV = ALLF && !KEEP && LTW == 2;
  constexpr int TWW = !LTW ? 2 : (ALLF && (KEEP || GINV)) ? RowTw<LOGN2>::ENTRIES : 2 * RowTw<LOGN2>::ENTRIES;
  __shared__ __attribute__((aligned(16))) uint64_t rtw[TWW];
  const unsigned n1 = 1u << (logn - LOGN2);
  const unsigned tiles = n1 / T::R;
  unsigned grp, mi;  // group = (slot, tile) on one XCD; members = pair ranges
  if (!xcd_group(members, t_n * tiles, grp, mi))
    return;
  const unsigned pb0 = (unsigned)(((size_t)mi * count) / members), pb1 = (unsigned)(((size_t)(mi + 1) * count) / members);
  if (pb0 >= pb1)
    return;
  const unsigned t = t_lo + grp / tiles, tile = grp % tiles;
  const unsigned m = basis_mod(t, lvl, L);
  const ModConst mc = mcs[m];
  const uint64_t q = mc.q, q2 = 2 * q;
  const unsigned row0 = tile * T::R;
  const size_t toff = (size_t)row0 << LOGN2;
  const bool f64 = ALLF || (AR == 0 && q < F64_QMAX && tw.fwdd);  // key words as plain doubles (to_mont_kernel)
  const uint64_t sk = ksc[t];  // the folded ModDown factor of this slot
  // [P s_t]_t and its Shoup companion, read before any store of the kernel
  // (a uniform load a store may clobber is a vector load, and its wait,
  // vmcnt(0), also waited out every prefetch in flight)
  const uint64_t kp0 = kps[2 * t], kp1 = kps[2 * t + 1];
  for (unsigned idx = threadIdx.x; idx < 2 * NDIG * 2048; idx += 256 * QN) {
    const unsigned c = idx >> 11, w = idx & 2047;
    // plain (FP64 moduli) or Montgomery form: either way x s_t stays in its form
    const uint64_t e = mul_mod(evkm[(((size_t)c * nmod + m) << logn) + toff + w], sk, mc);
    kl[c][w] = f64 ? (uint64_t)__double_as_longlong((double)e) : e;
  }
  __syncthreads();
  // the quarter (pair stream) is wave-uniform: as a scalar, the pair index,
  // the loop bound tests and the streams' base addresses live in SGPRs (no
  // exec-masked pair loop, 32-bit lane offsets)
  constexpr bool SQ = (KSQ_SCALAR_Q >> (KEEP ? 1 : 0)) & 1;
  const int qi = SQ ? (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 8) : (int)(threadIdx.x >> 8);
  const int th = threadIdx.x & 255, row = th / T::TA, l = th % T::TA;
  // this lane's word offset in a row tile (32-bit, so a uniform base in SGPRs
  // plus it is one global access with a scalar base)
  const unsigned lo = (unsigned)((row << LOGN2) + l);
  uint64_t *lq = rt[qi];
  const unsigned jo = t < lvl ? t / alpha : NDIG;  // the digit owning q limb t (none on P limbs)
  const int nx = jo < NDIG ? NDIG - 1 : NDIG;
  auto jof = [&](int u) -> unsigned { return (unsigned)u < jo ? (unsigned)u : (unsigned)u + 1; };
  auto fetch = [&](uint64_t (&x)[8], unsigned j, unsigned p) {
    gptr<const uint64_t> s = sgpr_ptr<SQ>(T1 + p * t1_stride + (((size_t)j * nm + t) << logn) + toff);
#pragma unroll
    for (int k = 0; k < 8; k++)
      x[k] = s[lo + T::TA * k];
  };
  unsigned p = pb0 + qi;
  // PF1 (the dropped slots' two digits): one tile buffer, each converted limb
  // requested one phase ahead (the next digit of this pair, or the first of
  // the next pair) instead of every digit of the next pair at once -- 16 VGPRs
  // fewer
  constexpr bool PF1 = !KEEP && NX > 1 && KSQ_DROP_PF1;
  constexpr int NB = PF1 ? 1 : (NX > 0 ? NX : 1);
  uint64_t xn[NB][8];
  if (p < pb1)
#pragma unroll
    for (int u = 0; u < NB; u++)
      if (u < nx)
        fetch(xn[u], jof(u), p);
  auto mac_i = [&](uint64_t &a, uint64_t v, uint64_t w) {  // Montgomery MAC, lazy [0, 2q)
    const uint64_t lo = v * w, hi = mulhi64(v, w);
    const uint64_t r = hi + mulhi64(lo * mc.qneg_inv, q) + (lo != 0);
    a = lazy_lt2q(a + r, q2);
  };
  with_arith_ar<AR>(q, m, logn, tw, [&](const auto &ar0) {
    using A0 = std::decay_t<decltype(ar0)>;
    constexpr bool F = std::is_same<A0, ArF64>::value;
    // 8-byte entries (ALLF: A0 is ArF64); the kept slots' 16-byte forward
    // entries measured slower (more spills: 2.00 vs 1.91 ms per chunk)
    constexpr bool W8 = LTW && ALLF;
    if constexpr (W8) {
      RowTw<LOGN2>::template stage<true>(rtw, (const uint64_t *)ar0.tw, n1 + row0, threadIdx.x, 256 * QN);
      if constexpr (!KEEP && !GINV)  // the dropped slots' inverse row pass
        RowTw<LOGN2>::template stage<true>(rtw + RowTw<LOGN2>::ENTRIES, (const uint64_t *)ar0.itw, n1 + row0,
                                           threadIdx.x, 256 * QN);
      __syncthreads();
    } else if constexpr (LTW) {
      RowTw<LOGN2>::stage(rtw, (const uint64_t *)ar0.tw, n1 + row0, threadIdx.x, 256 * QN);
      __syncthreads();
    }
    // the pair loop, with the FP64 lazy-reduction choice as a compile-time
    // constant (lzc: 1 / 0, -1 integer or run-time)
    auto pairs = [&](auto lzc) {
    constexpr int LZ = decltype(lzc)::value;
    const auto ar = [&] {
      if constexpr (LTW && F) {
        return row_policy<LOGN2, W8, GINV, LZ>(ar0, rtw, (int64_t)T::R - (int64_t)(n1 + row0),
                                               W8 && !KEEP && !GINV ? rtw + RowTw<LOGN2>::ENTRIES : nullptr);
      } else if constexpr (LTW) {
        return row_policy<LOGN2>(ar0, rtw, (int64_t)T::R - (int64_t)(n1 + row0));
      } else {
        return with_lz<LZ>(ar0);
      }
    }();
    using A = std::decay_t<decltype(ar)>;
    using V = typename A::V;
    for (; p < pb1; p += QN) {
      const unsigned pn = p + QN;
      // f: FP64 accumulators (|.| < 3 q before each fold); a: integer lazy ones
      V f0[8], f1[8];
      uint64_t a0[8], a1[8];
      if (nx == 0)  // one-digit keys: a q slot has no converted limb
#pragma unroll
        for (int k = 0; k < 8; k++) {
          f0[k] = f1[k] = 0;
          a0[k] = a1[k] = 0;
        }
      // the dropped q slot's first half of input words is requested here, so
      // its latency overlaps the converted limb's row pass (1037 -> 1018 us)
      const size_t ioff = p * d01.in_stride + ((size_t)t << logn) + toff;  // (uniform)
      gptr<const uint64_t> pin[4] = {sgpr_ptr<SQ>(d01.a + ioff), sgpr_ptr<SQ>(d01.b + ioff), sgpr_ptr<SQ>(d01.a + ioff + d01.in_pstride),
                                sgpr_ptr<SQ>(d01.b + ioff + d01.in_pstride)};  // a0, b0, a1, b1
      const unsigned lin = 8u * (unsigned)th;
      uint64_t inw[4][4];
      auto ld_in = [&](int h) {
#pragma unroll
        for (int a = 0; a < 4; a++) {
          gptr<const u64x2> v2 = (gptr<const u64x2>)(pin[a] + (lin + 4 * h));
          const u64x2 w0 = v2[0];
          const u64x2 w1 = v2[1];
          inw[a][0] = w0.x;
          inw[a][1] = w0.y;
          inw[a][2] = w1.x;
          inw[a][3] = w1.y;
        }
      };
      // (the kept slots' kernel cannot hold them: requesting the conv and
      // input words here spilled at three streams, 1.89 -> 2.73 ms per chunk,
      // and two streams with the room for them ran 2.04 vs 1.90 ms)
      constexpr bool EARLY = !KEEP;
      uint64_t cvw[KEEP && EARLY ? 2 : 1][8];
      if constexpr (KEEP && EARLY) {
#pragma unroll
        for (int half = 0; half < 2; half++) {
          gptr<const uint64_t> cv = sgpr_ptr<SQ>(conv + (((size_t)(2 * p + half) * cv_n + t) << logn) + toff);
#pragma unroll
          for (int k = 0; k < 8; k++)
            cvw[half][k] = cv[lo + T::TA * k];
        }
      }
      if (EARLY && jo < NDIG)
        ld_in(0);
#pragma unroll
      for (int u = 0; u < NX; u++) {
        if (u >= nx)
          continue;
        const unsigned j = jof(u);
        V r[8];
        uint64_t (&xb)[8] = xn[PF1 ? 0 : u];
#pragma unroll
        for (int k = 0; k < 8; k++)
          r[k] = A::load_lazy(xb[k]);  // T1 (ks_cols4, lazy)
        if constexpr (PF1) {
          if (u + 1 < nx)
            fetch(xb, jof(u + 1), p);  // this pair's next digit
          else if (pn < pb1)
            fetch(xb, jof(0), pn);  // the next pair's first
        } else if (pn < pb1) {
          fetch(xb, j, pn);  // next pair's tile, in flight meanwhile
        }
        wave_sync();            // the previous phase has finished with the LDS tile
        rows8_fwd_raw<LOGN2>(r, lq, ar, n1 + row0, th);
        if constexpr (F) {
#pragma unroll
          for (int k = 0; k < 8; k++) {
            const double eb = __longlong_as_double((long long)kl[2 * j][256 * k + th]);
            const double ea = __longlong_as_double((long long)kl[2 * j + 1][256 * k + th]);
            const double tb = f64_mulmod_h(r[k], eb, ar.q, ar.qinv);
            const double ta = f64_mulmod_h(r[k], ea, ar.q, ar.qinv);
            f0[k] = u ? f0[k] + tb : tb;
            f1[k] = u ? f1[k] + ta : ta;
            if (u == 1) {  // two products (< 3 q): fold before the next term
              f0[k] = f64_red(f0[k], ar.q, ar.qinv);
              f1[k] = f64_red(f1[k], ar.q, ar.qinv);
            }
          }
        } else {
#pragma unroll
          for (int k = 0; k < 8; k++) {
            const uint64_t v = ar.canon(r[k]);
            if (u == 0)
              a0[k] = a1[k] = 0;
            mac_i(a0[k], v, kl[2 * j][256 * k + th]);
            mac_i(a1[k], v, kl[2 * j + 1][256 * k + th]);
          }
        }
      }
      if (jo < NDIG) {
        // q limb: own digit x = a1 b1 (the NTT-form d2 limb) and P (d0, d1),
        // from the four input words at this thread's natural positions 8 th + k
        if constexpr (F) {
          const double Pd = f64_from_u52(kp0), Pq = Pd * ar.qinv;  // [P s_t]_t
#pragma unroll
          for (int h = 0; h < 2; h++) {
            if (h || !EARLY)
              ld_in(h);
            auto iw = [&](int a, int e) { return inw[a][e]; };
#pragma unroll
            for (int e = 0; e < 4; e++) {
              const int k = 4 * h + e;
              const double A0 = f64_from_u52(iw(0, e)), B0 = f64_from_u52(iw(1, e));
              const double A1 = f64_from_u52(iw(2, e)), B1 = f64_from_u52(iw(3, e));
              const double eb = __longlong_as_double((long long)kl[2 * jo][256 * k + th]);
              const double ea = __longlong_as_double((long long)kl[2 * jo + 1][256 * k + th]);
              const double x = f64_mulmod_h(A1, B1, ar.q, ar.qinv);  // |x| < 1.5 q
              const double d0 = f64_mulmod_h(A0, B0, ar.q, ar.qinv);
              const double d1 = f64_red(f64_mulmod_h(A0, B1, ar.q, ar.qinv) + f64_mulmod_h(A1, B0, ar.q, ar.qinv),
                                        ar.q, ar.qinv);
              // |f| <= q/2 + 1.5 q after the fold, then + two products < 1.5 q
              const double g0 = f64_red(f0[k], ar.q, ar.qinv) + f64_mulmod_h(x, eb, ar.q, ar.qinv);
              const double g1 = f64_red(f1[k], ar.q, ar.qinv) + f64_mulmod_h(x, ea, ar.q, ar.qinv);
              f0[k] = f64_red(g0, ar.q, ar.qinv) + f64_mulmod(d0, Pd, Pq, ar.q);
              f1[k] = f64_red(g1, ar.q, ar.qinv) + f64_mulmod(d1, Pd, Pq, ar.q);
            }
          }
        } else {
#pragma unroll
          for (int h = 0; h < 2; h++) {
            if (h || !EARLY)
              ld_in(h);
#pragma unroll
            for (int e = 0; e < 4; e++) {
              const int k = 4 * h + e;
              const uint64_t A0 = inw[0][e], B0 = inw[1][e], A1 = inw[2][e], B1 = inw[3][e];
              const uint64_t x = mul_mod(A1, B1, mc);
              mac_i(a0[k], x, kl[2 * jo][256 * k + th]);
              mac_i(a1[k], x, kl[2 * jo + 1][256 * k + th]);
              const uint64_t d0 = mul_mod(A0, B0, mc);
              const uint64_t d1 = add_mod(mul_mod(A0, B1, mc), mul_mod(A1, B0, mc), q);
              const uint64_t c0 = a0[k] >= q ? a0[k] - q : a0[k], c1 = a1[k] >= q ? a1[k] - q : a1[k];
              a0[k] = add_mod(c0, mul_shoup(d0, kp0, kp1, q), q);
              a1[k] = add_mod(c1, mul_shoup(d1, kp0, kp1, q), q);
            }
          }
        }
      } else if constexpr (!F) {
#pragma unroll
        for (int k = 0; k < 8; k++) {
          a0[k] = a0[k] >= q ? a0[k] - q : a0[k];
          a1[k] = a1[k] >= q ? a1[k] - q : a1[k];
        }
      }
      // (f0, f1) / (a0, a1): this thread's words 8 th + k of slot t (natural order)
      if constexpr (KEEP) {
#pragma unroll
        for (int half = 0; half < 2; half++) {
          const unsigned poly = 2 * p + half;
          gptr<const uint64_t> cv = sgpr_ptr<SQ>(conv + (((size_t)poly * cv_n + t) << logn) + toff);
          V r[8];
#pragma unroll
          for (int k = 0; k < 8; k++)
            r[k] = A::load_lazy(EARLY ? cvw[half][k] : cv[lo + T::TA * k]);  // conv (lazy)
          wave_sync();
          rows8_fwd_raw<LOGN2>(r, lq, ar, n1 + row0, th);
          // out = f D^-1 - NTTrows(conv D^-1): both factors already folded in
          uint64_t o[8];
          if constexpr (F) {
#pragma unroll
            for (int k = 0; k < 8; k++)
              o[k] = ar.canon(f64_red(half ? f1[k] : f0[k], ar.q, ar.qinv) - r[k]);  // |.| < 3.1 q
          } else {
#pragma unroll
            for (int k = 0; k < 8; k++)
              o[k] = sub_mod(half ? a1[k] : a0[k], ar.canon(r[k]), q);
          }
          // The wave's 64 threads hold its 4 KiB of consecutive words, 64 B
          // each: transposed through the wave's own rows of the LDS tile
          // (free again after the row pass) so that each 16-byte store
          // instruction writes 1 KiB contiguous (consecutive lanes 16 B
          // apart).  Lanes 64 B apart store at ~4.2 TB/s against ~5.6 for
          // that shape (copy kernels, scripts/ubench_lanes.hip): keep 1839 -
          // 1853 -> 1798 - 1814 us per chunk, same box.
          const unsigned e0 = (uint32_t)__builtin_amdgcn_readfirstlane((th & ~63) * 8), ln = (unsigned)th & 63;
          u64x2 *wr = (u64x2 *)(lq + (e0 >> LOGN2) * T::RS);
          wave_sync();  // the row pass's last reads of these words
#pragma unroll
          for (int i = 0; i < 4; i++)
            wr[4 * ln + i] = u64x2{o[2 * i], o[2 * i + 1]};
          wave_sync();
          gptr<u64x2> d2 = (gptr<u64x2>)sgpr_ptr<SQ>(dst + poly * dst_pstride + ((size_t)t << logn) + toff + e0);
#pragma unroll
          for (int i = 0; i < 4; i++)  // (non-temporal stores here: 1840 -> 2245 us per chunk)
            d2[64 * i + ln] = wr[64 * i + ln];
        }
      } else {
#pragma unroll
        for (int half = 0; half < 2; half++) {
          V r[8];
#pragma unroll
          for (int k = 0; k < 8; k++) {
            if constexpr (F)
              r[k] = f64_red(half ? f1[k] : f0[k], ar.q, ar.qinv);
            else
              r[k] = A::load(half ? a1[k] : a0[k]);
          }
          wave_sync();
          rows8_inv<LOGN2>(r, lq, ar, n1 + row0, th);
          gptr<uint64_t> o = sgpr_ptr<SQ>(dst + (2 * p + half) * dst_pstride + ((size_t)(t - t_lo) << logn) + toff);
#pragma unroll
          for (int k = 0; k < 8; k++)
            ST_STREAM(ar.canon(r[k]), &o[lo + T::TA * k]);
        }
      }
    }
    };
    // (run-time choice: one branch per transform call for the kept slots,
    // 1811 vs 1831 us per chunk; KSQ_DROP_LZM for the dropped ones, whose
    // registers the all-branch form spills)
    pairs(std::integral_constant<int, !F ? -1 : AR < 3 ? (KEEP ? -1 : KSQ_DROP_LZM) : AR == 3 ? 1 : 0>{});
  });
}

// (DROP_LTW: the dropped slots' form of LTW; 0: it reads its twiddles from
// L2, 2: the forward ones staged only, for keys whose tile leaves less room)
template <int LOGN2, int NDIG, int QN, int AR, int LTW, int DROP_LTW = LTW>
static void ksq_launch(bool keep_stage, const uint64_t *T1, const D01Src &d01, const uint64_t *evkm, uint64_t *dst,
                       size_t dst_pstride, const uint64_t *conv, const uint64_t *ksc, const uint64_t *kps, unsigned count,
                       unsigned lvl, unsigned nm, unsigned t_lo, unsigned t_n, unsigned cv_n)
{
  const unsigned n = G.n, groups = t_n * (n / 2048);
  // pair ranges of about 8 pairs per quarter stream (128 pairs at N=2^16:
  // 3 pairs 38.5k, 5-50 pairs 39.2-39.3k ct-mult/s, same box); more, shorter
  // ranges while the grid would not give every CU two workgroups
  const unsigned per = 8 * QN;
  unsigned members = std::max(1u, (count + per - 1) / per);
  while (members < count && (size_t)groups * members < 2 * 256)
    members++;
  if (KSQ_FILL && count >= 64) {
    // one workgroup per CU (the key tile's LDS): a grid of whole waves of
    // 256 workgroups leaves no partly idle last wave.  1: fewer, longer pair
    // ranges; 2: more, shorter ones
    const unsigned step = 256 / std::gcd(groups, 256u);
    if (step <= 16) {  // (else the rounding would cut the ranges to a few pairs)
    const unsigned lo = std::max(step, members / step * step), hi = (members + step - 1) / step * step;
    members = std::min(count, KSQ_FILL == 1 ? lo : hi);
    }
  }
  const Tw2 tw{G.tw2, G.itw2, G.twd, G.itwd};
  const size_t t1_stride = (size_t)NDIG * nm * n;
  auto kern = keep_stage ? ksq_kernel<LOGN2, NDIG, QN, AR, true, LTW> : ksq_kernel<LOGN2, NDIG, QN, AR, false, DROP_LTW>;
  hipLaunchKernelGGL(kern, dim3(xcd_blocks(members, groups)), dim3(256 * QN), 0, G.stream, T1, t1_stride, d01, evkm,
                     dst, dst_pstride, conv, ksc, kps, G.logn, lvl, G.L, nm, G.nmod, G.alpha, count,
                     members, t_lo, t_n, cv_n, tw, G.dev.mc);
  HIP_CHECK(hipGetLastError());
}

// f(integral_constant<AR>) for the FP64 class (AR 1: the lazy-reduction
// policy chosen per slot at run time)
template <class F>
static void with_f64_class(int, F &&f)
{
  f(std::integral_constant<int, 1>{});
}

// ar: the slots' arithmetic class (ksq_kernel AR)
template <int LOGN2>
static void ksq_dispatch(unsigned ndig, int ar, bool keep_stage, const uint64_t *T1, const D01Src &d01,
                         const uint64_t *evkm, uint64_t *dst, size_t dst_pstride, const uint64_t *conv,
                         const uint64_t *ksc, const uint64_t *kps, unsigned count, unsigned lvl, unsigned nm, unsigned t_lo,
                         unsigned t_n, unsigned cv_n)
{
#define KSQ_ARGS keep_stage, T1, d01, evkm, dst, dst_pstride, conv, ksc, kps, count, lvl, nm, t_lo, t_n, cv_n
  // LDS: the key tile (2 ndig x 16 KB) + 16 KB per quarter stream (+ 32 KB of
  // row twiddles where they fit) <= 160 KB
  switch (ndig) {
  case 1:
    // two streams (256 VGPRs); four (1024 threads, 128 VGPRs) spilled 58-193:
    // 68.2k -> 77.6k ct-mult/s at N=2^16, L=4, dnum=1 (same box)
    ksq_launch<LOGN2, 1, 2, 0, 1>(KSQ_ARGS);
    break;
  case 2:
    // (four streams for the kept slots, 128 VGPRs: 36.4k vs 38.1k ct-mult/s)
    if (ar == 1 || ar >= 3)
      with_f64_class(ar, [&](auto arc) {
        constexpr int A = decltype(arc)::value;
        if ((!keep_stage && KSQ_DROP_QN == 2) || (keep_stage && KSQ_KEEP_QN == 2))
          ksq_launch<LOGN2, 2, 2, A, 1>(KSQ_ARGS);
        else
          ksq_launch<LOGN2, 2, 3, A, 1>(KSQ_ARGS);
      });
    else if (ar == 2)  // integer moduli: two streams, 256 VGPRs (three spilled 180: drop 2.60 -> 1.78 ms per chunk)
      ksq_launch<LOGN2, 2, 2, 2, 1>(KSQ_ARGS);
    else
      ksq_launch<LOGN2, 2, 2, 0, 1>(KSQ_ARGS);
    break;
  case 3:
    // 96 KB of key tile: two streams and the row twiddles from L2 (config 5:
    // 7.76k vs 7.51k ct-mult/s for the streaming ks_rows form; one stream with
    // staged twiddles 7.50k, same box)
    if (ar == 1 || ar >= 3)
      with_f64_class(ar, [&](auto arc) {
        constexpr int A = decltype(arc)::value;
        if (keep_stage ? KSQ_C5_KEEP_LTW != 0 : KSQ_C5_DROP_LTW != 0)
          // the forward row twiddles staged (16 KB): 96 KB of key + two row
          // tiles + those fit (the dropped slots' inverse ones too would not)
          ksq_launch<LOGN2, 3, 2, A, 1, 2 * (KSQ_C5_DROP_LTW != 0)>(KSQ_ARGS);
        else
          ksq_launch<LOGN2, 3, 2, A, 0>(KSQ_ARGS);
      });
    else if (ar == 2)
      ksq_launch<LOGN2, 3, 2, 2, 0>(KSQ_ARGS);
    else
      ksq_launch<LOGN2, 3, 2, 0, 0>(KSQ_ARGS);
    break;
  default: gpqhe_die("split key switch: %u digits", ndig);
  }
#undef KSQ_ARGS
}

// Slots [t_lo, t_lo + t_n) of one stage.  Mixed prime sets (FP64 and 60-bit
// moduli) launch each run of same-class slots on its class's kernel
// (KSQ_SPLIT_AR): the dropped slots' outputs are relative to t_lo, so a run
// starting at a writes from dst + (a - t_lo) limbs; the kept slots' outputs
// and conv are indexed by the absolute slot.
template <int LOGN2>
static void ksq_stage(unsigned ndig, bool allf, bool keep_stage, const uint64_t *T1, const D01Src &d01,
                      const uint64_t *evkm, uint64_t *dst, size_t dst_pstride, const uint64_t *conv, const uint64_t *ksc,
                      const uint64_t *kps, unsigned count, unsigned lvl, unsigned nm, unsigned t_lo, unsigned t_n)
{
  if (allf || !KSQ_SPLIT_AR || ndig == 1) {
    ksq_dispatch<LOGN2>(ndig, allf ? 1 : 0, keep_stage, T1, d01, evkm, dst, dst_pstride, conv, ksc, kps, count, lvl, nm,
                        t_lo, t_n, t_n);
    return;
  }
  auto cls = [&](unsigned t) {
    const unsigned m = t < lvl ? t : G.L + (t - lvl);
    if (!(G.twd != nullptr && G.q[m] < (1ull << 51)))
      return 2;
    return 1;
  };
  for (unsigned a = t_lo; a < t_lo + t_n;) {
    const int c = cls(a);
    unsigned b = a + 1;
    while (b < t_lo + t_n && cls(b) == c)
      b++;
    uint64_t *d = keep_stage ? dst : dst + ((size_t)(a - t_lo) << G.logn);
    ksq_dispatch<LOGN2>(ndig, c, keep_stage, T1, d01, evkm, d, dst_pstride, conv, ksc, kps, count, lvl, nm, a, b - a,
                        t_n);
    a = b;
  }
}

void ksq_run(unsigned logn2, unsigned ndig, bool allf, bool keep_stage, const uint64_t *T1, const D01Src &d01,
             const uint64_t *evkm, uint64_t *dst, size_t dst_pstride, const uint64_t *conv, const uint64_t *ksc,
             const uint64_t *kps, unsigned count, unsigned lvl, unsigned nm, unsigned t_lo, unsigned t_n)
{
#ifdef KSQ_DEV  // analysis builds: the bench's instantiations only (N=2^16: 128 x 512)
  if (logn2 == 9 && ndig == 2 && allf) {
    ksq_launch<9, 2, 3, 1, 1>(keep_stage, T1, d01, evkm, dst, dst_pstride, conv, ksc, kps, count, lvl, nm, t_lo, t_n, t_n);
    return;
  }
  gpqhe_die("KSQ_DEV build");
#else
  switch (logn2) {
  case 7: ksq_stage<7>(ndig, allf, keep_stage, T1, d01, evkm, dst, dst_pstride, conv, ksc, kps, count, lvl, nm, t_lo, t_n); break;
  case 8: ksq_stage<8>(ndig, allf, keep_stage, T1, d01, evkm, dst, dst_pstride, conv, ksc, kps, count, lvl, nm, t_lo, t_n); break;
  case 9: ksq_stage<9>(ndig, allf, keep_stage, T1, d01, evkm, dst, dst_pstride, conv, ksc, kps, count, lvl, nm, t_lo, t_n); break;
  default: gpqhe_die("split key switch: row length 2^%u", logn2);
  }
#endif
}
