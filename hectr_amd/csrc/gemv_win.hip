// gemv_win.hip - HECTR's he_gemv (reference src/hempc.c:257-259) and he_rot
// over a batch of independent ciphertexts at n = 2^13 .. 2^17 (he_gemv_batch /
// he_rot_batch, and he_gemv / he_rot on one object at those sizes):
//
//   ModUp  Dc = NTT(FBC(INTT(c1) x [(Q_j/q_i)^-1]))  k_modup_c1_split: the split
//          on every slot outside a digit             key switch's d2_rows (c1
//                                                    form) + ks_cols + row pass
//   acc = sum_d pt_d sigma_d(KS_d(c0, c1))           gemv_win_kernel (basis QP)
//   out = ModDown(acc) by P q_top (gemv) or P (rot)  k_moddown_fused
//
// Basis slots on moduli below 2^51 run the inner products in FP64 (exact
// products, ntt_device.h); wider ones (HECTR-like 59-61-bit q0 / P) in 64-bit
// integers with Montgomery-form keys (gemv_win_kernel<., ., INT>).
//
// The oracle's hoisted gemv (oracle/ckks_oracle.c gemv_apply): one ModUp per
// ciphertext, the rotated inner products accumulated in the extended basis,
// one ModDown per output.  Every step is exact modular arithmetic on canonical
// residues, so the outputs are the oracle's bit for bit whatever the order of
// the sums.
//
// The inner products (gemv_win_kernel).  Diagonal d reads D at the Galois
// permutation pi_d = auto_index(., 5^d) of each output position.  Blocks of
// 64 consecutive NTT positions (the top b = logn - 6 index bits) map to
// blocks: block e (odd, mod 2^(b+1)) reads block 5^d e, and inside a block the
// map is a permutation of the 64 positions, affine in the bit-reversed
// offset.  The blocks form two orbits under x5 (e = +-5^i), and output block
// o of an orbit reads source blocks o + d.  One wave owns one output block; a
// workgroup of 16 waves owns (basis slot, orbit, segment) for three
// ciphertexts and advances along the segment 16 output blocks at a time.
// The source blocks those outputs read sit in an LDS ring of 32 blocks
// (centred doubles), each loaded from HBM once; a wave reads its sources
// from the ring at the permuted lane (conflict-free: a permutation of its
// own 64 lanes), multiplies them by its output positions' key words -- one
// load per word serves the three ciphertexts -- and keeps the accumulators
// in registers.  The keys are pre-multiplied by their diagonal (pt_d x evk_d,
// P x pt_d; gemv_fold_kernel) and interleaved per position, so a lane's key
// words for a diagonal are one 16-byte-aligned run; the workgroups of one
// (slot, orbit, segment) are placed on one XCD (xcd_group), so they share the
// keys through its L2.
#include "ntt_device.h"
#include "tables.h"

#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <type_traits>
#include <vector>

__device__ __forceinline__ unsigned gw_brev(unsigned x, unsigned bits)
{
  return __builtin_bitreverse32(x) >> (32 - bits);
}

// NTT-domain position whose value sigma_g moves to k (kernels.hip auto_index)
__device__ __forceinline__ unsigned gw_auto_index(unsigned k, uint64_t g, unsigned logn)
{
  const uint64_t mask = (2ull << logn) - 1;
  const uint64_t e = ((2ull * gw_brev(k, logn) + 1) * g) & mask;
  return gw_brev((unsigned)(e >> 1), logn);
}

// ---------------------------------------------------------------------------
// Folded keys, output order, interleaved: slot t's block at gw_kbase(t), then
// [(e n + k) 2 ndig + w] for output position k:
//   w < ndig:           [pt_d]_t[k] [b_{d,w}]_t[k]
//   ndig <= w < 2 ndig: [pt_d]_t[k] [a_{d,w-ndig}]_t[k]
// and after all slots' blocks (gw_kbase(nm)) the q slots' P pt_d words,
// [(t E + e) n + k] for t < lvl (gemv_c0_kernel; the identity's c1 term).
// pt null: 1 (a rotation).  FP64 slots: the residues as doubles; integer
// slots: Montgomery forms x 2^64 mod q, as 30-bit halves (gw_split) when every
// integer modulus is below 2^60.
// grid: (n / 256, nm, diagonals of this launch)
// ---------------------------------------------------------------------------
// the start of slot t's key block (in words, E diagonals)
__host__ __device__ __forceinline__ size_t gw_kbase(unsigned t, unsigned ndig, unsigned E, unsigned logn)
{
  return ((size_t)t * 2 * ndig * E) << logn;
}

struct FoldArgs {
  static constexpr unsigned MAX = 16;
  const uint64_t *pt[MAX], *evk[MAX];
  unsigned e0;       // the launch's first diagonal in K
  uint64_t intmask;  // bit t: basis slot t on 64-bit integer arithmetic (modulus >= 2^51)
  unsigned split;    // integer slots' moduli all below 2^60: words stored as 30-bit halves (gw_split)
};

// x < 2^60 as its 30-bit halves in the two 32-bit words (x0 | x1 << 32), the
// operands of v_mad_u64_u32
__host__ __device__ __forceinline__ uint64_t gw_split(uint64_t x)
{
  return (x & ((1ull << 30) - 1)) | ((x >> 30) << 32);
}

__global__ void __launch_bounds__(256) gemv_fold_kernel(double *K, FoldArgs fa, unsigned Etot, unsigned ndig,
                                                        unsigned logn, unsigned lvl, unsigned L, unsigned nmod,
                                                        unsigned nm, const ModConst *mcs)
{
  const unsigned k = blockIdx.x * 256 + threadIdx.x, t = blockIdx.y, e = blockIdx.z;
  const unsigned m = basis_mod(t, lvl, L);
  const ModConst mc = mcs[m];
  const uint64_t *pt = fa.pt[e], *ev = fa.evk[e];
  const uint64_t w = pt ? pt[((size_t)t << logn) + k] : 1;
  const unsigned kw = 2 * ndig;
  const bool isint = (fa.intmask >> t) & 1;
  // FP64 slots: the residue as a double; integer slots: its Montgomery form
  // x 2^64 mod q (bits), so the kernel's REDC of y x returns y x mod q
  auto put = [&](double *o, uint64_t v) {
    if (isint) {
      const uint64_t m = mul_mod(v, mc.r64, mc);
      *(uint64_t *)o = fa.split ? gw_split(m) : m;
    } else {
      *(uint64_t *)o = (uint64_t)__double_as_longlong((double)v);
    }
  };
  double *o = K + gw_kbase(t, ndig, Etot, logn) + ((((size_t)fa.e0 + e) << logn) + k) * kw;
  for (unsigned j = 0; j < ndig; j++) {
    put(o + j, ev ? mul_mod(w, ev[(((size_t)(2 * j) * nmod + m) << logn) + k], mc) : 0);
    put(o + ndig + j, ev ? mul_mod(w, ev[(((size_t)(2 * j + 1) * nmod + m) << logn) + k], mc) : 0);
  }
  if (t < lvl)
    put(K + gw_kbase(nm, ndig, Etot, logn) + ((((size_t)t * Etot + fa.e0 + e) << logn) + k), mul_mod(w, mc.pmod, mc));
}

// ---------------------------------------------------------------------------
// ModUp conversion: Dc[p][slot] = sum_i y_i [Q_j/q_i]_t mod q_t for each digit
// j and each basis slot t outside it (slots in that order), y the digit's
// scaled coefficient-domain limbs.  One thread per coefficient.
// grid: (n / 256, count)
// ---------------------------------------------------------------------------
struct GwMods {
  double q[GPQHE_MAXMOD / 2], qinv[GPQHE_MAXMOD / 2];  // per basis slot of basis_qp(lvl)
  uint64_t qi[GPQHE_MAXMOD / 2], qni[GPQHE_MAXMOD / 2];  // the same as integers, -q^-1 mod 2^64
};

__global__ void __launch_bounds__(256) gemv_fbc_kernel(uint64_t *Dc, size_t d_stride, const uint64_t *y,
                                                       size_t y_stride, const double *cd, GwMods md, unsigned logn,
                                                       unsigned lvl, unsigned nm, unsigned ndig, unsigned alpha)
{
  const size_t k = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t p = blockIdx.y;
  const uint64_t *yp = y + p * y_stride + k;
  uint64_t *dp = Dc + p * d_stride + k;
  unsigned slot = 0;
  for (unsigned j = 0; j < ndig; j++) {
    const unsigned lo = j * alpha, na = min(alpha, lvl - lo);
    double yv[8];
#pragma unroll
    for (unsigned i = 0; i < 8; i++)
      yv[i] = i < na ? f64_from_u52(yp[(size_t)(lo + i) << logn]) : 0.0;
    for (unsigned t = 0; t < nm; t++) {
      if (t >= lo && t < lo + na)
        continue;
      const double q = md.q[t], qinv = md.qinv[t];
      const double *c = cd + 2 * ((size_t)j * 8 * nm + t);  // ([Q_j/q_i]_t, that / q_t) at i stride 2 nm
      // |term| < q (y < 2^51); two terms, then a reduction: |.| < 2.5 q
      double s = 0;
#pragma unroll
      for (unsigned i = 0; i < 8; i++) {
        if (i < na) {
          s += f64_mulmod(yv[i], c[2 * i * nm], c[2 * i * nm + 1], q);
          if (i & 1)
            s = f64_red(s, q, qinv);
        }
      }
      dp[(size_t)slot++ << logn] = f64_canon(s, q, qinv);
    }
  }
}

// ---------------------------------------------------------------------------
// The windowed inner products (see the file comment).
// ---------------------------------------------------------------------------
struct GemvWin {
  static constexpr unsigned MAXE = 16;
  const uint64_t *x;  // ciphertext p: c0 at x + p x_stride, c1 at + x_pstride
  size_t x_stride, x_pstride;
  const uint64_t *Dc;  // compact ModUp digits [count][S][n]
  size_t d_stride;
  const double *K;   // folded keys (gw_kbase: [nm][Etot][n][2 ndig])
  const double *Kp;  // the q slots' P pt_d words [lvl][Etot][n]
  uint64_t *acc;    // [count][2][nm][n]
  size_t acc_stride;
  int16_t yi[GPQHE_MAXMOD / 2][3];  // slot t, digit j: its Dc slot, -1: the own digit (c1 limb t)
  int32_t d[MAXE];                  // rotations of this launch's diagonals, ascending
  uint32_t hm[MAXE];                // g_e mod 64
  const uint32_t *tab;              // the launch's orbit table (gemv_tab_kernel)
  GwMods md;
  uint8_t slot[GPQHE_MAXMOD / 2];   // the launch's basis slots (one arithmetic class)
  unsigned ns;
  unsigned E, e0, Etot, accumulate;
  unsigned logn, lvl, nm, count, nseg, alpha;
};

struct GemvTab {
  uint64_t g[GemvWin::MAXE];  // g_e mod 2n
  unsigned E, logn;
};

__device__ __forceinline__ double gw_center(double v, double q)
{
  return v > 0.5 * q ? v - q : v;
}

// ---------------------------------------------------------------------------
// The orbit table of one launch (gemv_tab_kernel): row (orb, o), 32 words, for
// orbit position o of orbit orb (block value e = +-5^o mod 2^(b+1)): word e <
// E holds C_{o,e} mod 64, the constant of the permutation from output block o
// to its source through diagonal e (source offset j'_hi = C + g_e j_hi mod
// 64), word 16 the block of position o.  One scalar row load per output
// block replaces the 64-bit arithmetic per diagonal.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) gemv_tab_kernel(uint32_t *tab, GemvTab ta)
{
  const unsigned bb = ta.logn - 6, P = 1u << (bb - 1);
  const unsigned idx = blockIdx.x * 256 + threadIdx.x, row = idx / 32, w = idx % 32;
  if (row >= 2 * P)
    return;
  const uint64_t emask = (2ull << bb) - 1, nmask2 = (2ull << ta.logn) - 1;
  uint64_t ev = 1, bse = 5;
  for (unsigned r = row % P; r; r >>= 1, bse = (bse * bse) & emask)
    if (r & 1)
      ev = (ev * bse) & emask;
  if (row >= P)
    ev = (emask + 1 - ev) & emask;
  uint32_t v = 0;
  if (w == 16)
    v = gw_brev((unsigned)(ev >> 1), bb);
  else if (w < ta.E)
    v = (uint32_t)((((ta.g[w] * ev) & nmask2) >> (bb + 1)) & 63);
  tab[idx] = v;
}

// C ciphertexts per workgroup share every key word a lane loads (the keys'
// L2 traffic is the kernel's largest): as many as the ring (C x 32 blocks x
// ndig words x 512 B) and the registers allow -- the c0 term runs in its own
// pass (gemv_c0_kernel), so the ring holds the digits only: two digits 4
// ciphertexts (128 KB) against 3 with c0 in the ring (inner products 31.5 ->
// 24.5 us per ciphertext at N=2^16, L=8, 16 slots, same box), three digits 3
// (144 KB) against 2. With C0IN (the c0 word in the ring): 3 for two digits,
// 2 for three (and for one: 3 spills there)
template <int NDIG, bool C0IN = false>
constexpr int gw_cts()
{
  return C0IN ? (NDIG != 2 ? 2 : 3) : (NDIG >= 3 ? 3 : 4);
}

// One ring word: a centred double (FP64 slots) or a canonical residue
// (integer slots).
union GwWord {
  double d;
  uint64_t u;
};

// Montgomery REDC of a 128-bit sum v < q 2^64: v 2^-64 mod q in [0, 2q)
__device__ __forceinline__ uint64_t gw_redc(uint64_t hi, uint64_t lo, uint64_t q, uint64_t qni)
{
  return hi + mulhi64(lo * qni, q) + (lo != 0);
}

// (hi:lo) += y w
__device__ __forceinline__ void gw_mac128(uint64_t &hi, uint64_t &lo, uint64_t y, uint64_t w)
{
  const uint64_t pl = y * w, ph = mulhi64(y, w);
  lo += pl;
  hi += ph + (lo < pl);
}

// the split form (moduli below 2^60, operands gw_split): y w as four 32 x 32
// products of 30-bit halves into three 64-bit sums -- s00 += y0 w0, s01 +=
// y0 w1 + y1 w0, s11 += y1 w1 -- each term below 2^60, so up to 2^3 products'
// sums stay below 2^63 with no carries: four v_mad_u64_u32 per product
// instead of a 64 x 64 -> 128-bit product (about eight multiplies and the
// carries)
struct GwAcc3 {
  uint64_t s00 = 0, s01 = 0, s11 = 0;
  __device__ __forceinline__ void mac(uint64_t y, uint64_t w)
  {
    const uint32_t y0 = (uint32_t)y, y1 = (uint32_t)(y >> 32), w0 = (uint32_t)w, w1 = (uint32_t)(w >> 32);
    s00 += (uint64_t)y0 * w0;
    s01 += (uint64_t)y0 * w1;
    s01 += (uint64_t)y1 * w0;
    s11 += (uint64_t)y1 * w1;
  }
  // REDC of s00 + s01 2^30 + s11 2^60 (< q 2^64): [0, 2q)
  __device__ __forceinline__ uint64_t redc(uint64_t q, uint64_t qni) const
  {
    uint64_t lo = s00 + (s01 << 30);
    uint64_t hi = (s01 >> 34) + (lo < s00);
    const uint64_t u = s11 << 60;
    lo += u;
    hi += (s11 >> 4) + (lo < u);
    return gw_redc(hi, lo, q, qni);
  }
};

// INT: the slots of this launch are on 64-bit integer moduli (q >= 2^51: the
// 60-bit q_0 / P of HECTR-like prime sets).  Their key words are Montgomery
// forms (gemv_fold_kernel), a diagonal's products are summed in 128 bits
// (at most ndig + 1 <= 4 products of residues below q < 2^61: below q 2^64)
// and reduced by one REDC, the accumulators kept in [0, 2q).
// LZ (FP64 slots with q < 2^50, at most two digits; chosen per workgroup
// around the advance loop): the accumulators are reduced every third diagonal
// instead of every one.  With centred ring values
// |y| <= q/2 < 2^49 a product is below q (1/2 + 1.5 |y| 2^-52) < 0.69 q, so
// three diagonals of two products (three with C0IN's c0 term) on top of
// |acc| <= q/2 stay below 4.7 q < 2^52.3 (6.9 q < 2^52.8), and one more
// canonical word added at the output below 2^53.
// C0IN: the q slots' c0 term in this kernel (c0 a ring word, its P pt_d word
// from a.Kp per diagonal) instead of gemv_c0_kernel's pass -- the form for
// three digits (a fourth ring word costs one ciphertext per workgroup, 3 -> 2,
// against a separate pass that measured slower there) and for launches of a
// few diagonals (a rotation: the separate pass's fixed cost).
// the diagonal at which an advance requests the next advance's source block
// (and the c0 pass its accumulator words): 8 against before diagonal 0 (the
// round-5 A/B, profiles/r5_ab_gemv_srcat.json: 4 and 12 within noise of 8)
constexpr int GW_SRC_AT = 8;
// the integer forms' counted loop: at the last diagonal (1) or at GW_SRC_AT
#ifndef GW_INT_SRC_LAST
#define GW_INT_SRC_LAST 1
#endif
// KF (launches of 8 diagonals and more): the FP64 key words are requested on
// every path of the unrolled diagonal loop (past E at the last diagonal's
// address); else under each diagonal's branch, where the compiler's wait
// counts at the joins turn conservative but a launch of a few diagonals (a
// rotation) does not request 16 diagonals' words
template <int NDIG, int W, bool INT, bool SPLIT = false, bool C0IN = false, bool KF = false>
__global__ void __launch_bounds__(1024) gemv_win_kernel(GemvWin a)
{
  constexpr int C = gw_cts<NDIG, C0IN>(), RING = 32, NWD = NDIG + (C0IN ? 1 : 0), KW = 2 * NDIG;
  __shared__ GwWord ring[C][RING][NWD][64];
  const unsigned logn = a.logn, bb = logn - 6, P = 1u << (bb - 1);
  const unsigned nmem = (a.count + C - 1) / C;
  unsigned grp, mi;
  if (!xcd_group(nmem, a.ns * 2 * a.nseg, grp, mi))
    return;
  const unsigned t = a.slot[grp / (2 * a.nseg)], orb = (grp / a.nseg) & 1, seg = grp % a.nseg;
  const unsigned SEG = P / a.nseg, o0 = seg * SEG;
  const unsigned wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), L = threadIdx.x & 63;
  const unsigned p0 = mi * C;
  const unsigned nc = min((unsigned)C, a.count - p0);  // ciphertexts of this workgroup (the last may have fewer)
  const double q = a.md.q[t], qinv = a.md.qinv[t];
  const uint64_t qi = a.md.qi[t], qni = a.md.qni[t], q2 = 2 * qi;
  const bool qs = t < a.lvl;
  const int E = (int)a.E, dmin = a.d[0], dmax = a.d[E - 1];
  const bool ident = dmin == 0;
  const unsigned jo = qs ? t / a.alpha : 0;  // the own digit's ring word (c1) on a q slot
  const unsigned jh = gw_brev(L, 6);
  unsigned gj[W];  // g_e j_hi mod 64
#pragma unroll
  for (int e = 0; e < W; e++)
    gj[e] = e < E ? (a.hm[e] * jh) & 63 : 0;
  // the ring words: digit j (its ModUp limb, or c1 for the own digit)
  const uint64_t *sp[C][NWD];
#pragma unroll
  for (int c = 0; c < C; c++) {
    const unsigned pc = p0 + ((unsigned)c < nc ? c : 0);
    const uint64_t *xb = a.x + (size_t)pc * a.x_stride;
#pragma unroll
    for (int j = 0; j < NDIG; j++) {
      const int yi = a.yi[t][j];
      sp[c][j] = yi < 0 ? xb + a.x_pstride + ((size_t)t << logn) : a.Dc + (size_t)pc * a.d_stride + ((size_t)yi << logn);
    }
    if constexpr (C0IN)
      sp[c][NWD - 1] = xb + ((size_t)(qs ? t : 0) << logn);
  }
  const double *Kt = a.K + gw_kbase(t, NDIG, a.Etot, logn) + ((size_t)a.e0 << logn) * KW;
  // the q slots' [P pt_d] words (the identity's c1 term; with C0IN every
  // diagonal's c0 term -- else gemv_c0_kernel's)
  const double *Kpid = a.Kp + (((size_t)(qs ? t : 0) * a.Etot + a.e0) << logn);
  const size_t apoly = (size_t)a.nm << logn;
  const uint32_t *tabo = a.tab + (size_t)orb * P * 32;
  uint64_t pv[C][NWD];
  auto load_src = [&](unsigned s) {
    const size_t off = ((size_t)tabo[(s & (P - 1)) * 32 + 16] << 6) + L;
#pragma unroll
    for (int c = 0; c < C; c++)
#pragma unroll
      for (int w = 0; w < NWD; w++)
        pv[c][w] = sp[c][w][off];  // (C0IN P slots: slot 0's c0, unused)
  };
  auto store_src = [&](unsigned s) {
    const unsigned slot = s & (RING - 1);
#pragma unroll
    for (int c = 0; c < C; c++)
#pragma unroll
      for (int w = 0; w < NWD; w++) {
        if constexpr (INT)
          ring[c][slot][w][L].u = SPLIT ? gw_split(pv[c][w]) : pv[c][w];
        else
          ring[c][slot][w][L].d = gw_center(f64_from_u52(pv[c][w]), q);
      }
  };
  const unsigned nadv = SEG / 16;
  auto advances = [&](auto lzc) {
  constexpr bool LZ = decltype(lzc)::value;
  for (unsigned adv = 0; adv < nadv; adv++) {
    const unsigned ob = o0 + adv * 16;
    if (adv == 0) {
      for (unsigned s = ob + dmin + wv; s < ob + 16 + dmax; s += 16) {
        load_src(s);
        store_src(s);
      }
    } else {
      store_src(ob + dmax + wv);  // prefetched during the previous advance
    }
    __syncthreads();
    // the next advance's new block, requested at diagonal e_src (in flight
    // over the rest of the advance): loads return in order, so requested
    // before the first diagonals' key words it would hold them up, and every
    // wave of the workgroup would wait out its HBM latency together
    const bool more = adv + 1 < nadv;
    const int e_src = min(GW_SRC_AT, E - 1);
    const unsigned o = ob + wv;
    const uint32_t *tr = tabo + (o & (P - 1)) * 32;
    const size_t koff = ((size_t)tr[16] << 6) + L;
    // the identity's [P pt_0] word, requested before the first key words (at
    // its use it would wait out its own latency and every load before it)
    const uint64_t kpid = ident && qs ? ((const uint64_t *)Kpid)[koff] : 0;
    // accumulators: |.| <= q/2 (+ tiny) between diagonals (FP64), [0, 2q) (INT)
    double a0[C], a1[C];
    uint64_t u0[C], u1[C];
#pragma unroll
    for (int c = 0; c < C; c++) {
      a0[c] = a1[c] = 0.0;
      u0[c] = u1[c] = 0;
    }
    // INT: one diagonal's products (key words ku), the accumulators in [0, 2q)
    auto int_diag = [&](int e, const uint64_t *ku, unsigned slot, unsigned sl) {
      if (ident && e == 0) {  // the identity: [P pt_0] (c0, c1) on q slots (c0 here only with C0IN)
        if (qs) {
          const uint64_t kpi = kpid;
#pragma unroll
          for (int c = 0; c < C; c++) {
            const uint64_t y1 = ring[c][slot][jo][sl].u;
            if constexpr (SPLIT) {
              GwAcc3 b1;
              b1.mac(y1, kpi);
              u1[c] = b1.redc(qi, qni);
              if constexpr (C0IN) {
                GwAcc3 b0;
                b0.mac(ring[c][slot][NDIG][sl].u, kpi);
                u0[c] = b0.redc(qi, qni);
              }
            } else {
              u1[c] = gw_redc(mulhi64(y1, kpi), y1 * kpi, qi, qni);
              if constexpr (C0IN) {
                const uint64_t y0 = ring[c][slot][NDIG][sl].u;
                u0[c] = gw_redc(mulhi64(y0, kpi), y0 * kpi, qi, qni);
              }
            }
          }
        }
        return;
      }
#pragma unroll
      for (int c = 0; c < C; c++) {
        if constexpr (SPLIT) {
          GwAcc3 b0, b1;
#pragma unroll
          for (int j = 0; j < NDIG; j++) {
            const uint64_t yv = ring[c][slot][j][sl].u;
            b0.mac(yv, ku[j]);
            b1.mac(yv, ku[NDIG + j]);
          }
          if (C0IN && qs)
            b0.mac(ring[c][slot][NWD - 1][sl].u, ku[KW]);
          u0[c] = lazy_lt2q(u0[c] + b0.redc(qi, qni), q2);
          u1[c] = lazy_lt2q(u1[c] + b1.redc(qi, qni), q2);
        } else {
          uint64_t h0 = 0, l0 = 0, h1 = 0, l1 = 0;
#pragma unroll
          for (int j = 0; j < NDIG; j++) {
            const uint64_t yv = ring[c][slot][j][sl].u;
            gw_mac128(h0, l0, yv, ku[j]);
            gw_mac128(h1, l1, yv, ku[NDIG + j]);
          }
          if (C0IN && qs)
            gw_mac128(h0, l0, ring[c][slot][NWD - 1][sl].u, ku[KW]);
          u0[c] = lazy_lt2q(u0[c] + gw_redc(h0, l0, qi, qni), q2);
          u1[c] = lazy_lt2q(u1[c] + gw_redc(h1, l1, qi, qni), q2);
        }
      }
    };
    if constexpr (INT) {
      // one diagonal at a time with the next diagonal's key words in flight
      // (unrolled over 16 like the FP64 forms, the compiler unrolled it only
      // partly and indexed the key sets through gpr_idx: 60-bit gemv 70.4 ->
      // 73.3 us, same box, profiles/r6_ab_session1.txt).  The next advance's
      // source block is requested at the last diagonal: requested earlier, the
      // wait for the next diagonal's keys at the loop head (vmcnt(0): the
      // count differs between the iterations) waited it out as well
      uint64_t kc[KW + 1], kn[KW + 1];  // (word KW: the P pt_d word, C0IN q slots)
      auto load_keys1 = [&](int e, uint64_t (&kk)[KW + 1]) {
        const ulonglong2 *kp = (const ulonglong2 *)(Kt + ((((size_t)e) << logn) + koff) * KW);
#pragma unroll
        for (int w = 0; w < KW / 2; w++) {
          const ulonglong2 v = kp[w];
          kk[2 * w] = v.x;
          kk[2 * w + 1] = v.y;
        }
        kk[KW] = C0IN && qs ? ((const uint64_t *)Kpid)[((size_t)e << logn) + koff] : 0;
      };
      load_keys1(0, kn);
      for (int e = 0; e < E; e++) {
#pragma unroll
        for (int w = 0; w <= KW; w++)
          kc[w] = kn[w];
        if (e + 1 < E)
          load_keys1(e + 1, kn);
        if (e == (GW_INT_SRC_LAST ? E - 1 : e_src) && more)
          load_src(ob + 16 + dmax + wv);
        int_diag(e, kc, (o + a.d[e]) & (RING - 1), gw_brev((tr[e] + ((a.hm[e] * jh) & 63)) & 63, 6));
      }
    }
    // key words two diagonals ahead (a ring of three sets): the L2 latency of
    // a diagonal's keys overlaps the two before it
    constexpr int KD = 3;
    uint64_t kw[KD][KW + 1];  // (word KW: the P pt_d word, C0IN q slots)
    auto load_keys = [&](int e, int ea) {  // set e % KD <- diagonal ea's words
      const ulonglong2 *kp = (const ulonglong2 *)(Kt + ((((size_t)ea) << logn) + koff) * KW);
#pragma unroll
      for (int w = 0; w < KW / 2; w++) {
        const ulonglong2 v = kp[w];
        kw[e % KD][2 * w] = v.x;
        kw[e % KD][2 * w + 1] = v.y;
      }
      if constexpr (C0IN) {  // (P slots: zero -- the product below adds nothing)
        const uint64_t v = ((const uint64_t *)Kpid)[((size_t)ea << logn) + koff];
        kw[e % KD][KW] = qs ? v : 0;
      }
    };
    // (KF: key words requested on every path, past E at the last diagonal's:
    // a load under the diagonal's branch left the compiler's wait counts
    // conservative at the joins, a full vmcnt(0) after it)
    constexpr bool UNR = !INT;  // the unrolled loop below runs this launch
#pragma unroll
    for (int e = 0; e < KD - 1; e++)
      if (UNR && (KF || e < E))
        load_keys(e, KF ? min(e, E - 1) : e);
#pragma unroll
    for (int e = 0; e < W; e++) {
      if constexpr (KF)
        if (e + KD - 1 < W)
          load_keys(e + KD - 1, min(e + KD - 1, E - 1));
      if (UNR && e < E) {
        if constexpr (!KF)
          if (e + KD - 1 < W && e + KD - 1 < E)
            load_keys(e + KD - 1, e + KD - 1);
        if (e == e_src && more)
          load_src(ob + 16 + dmax + wv);
        const uint64_t *ku = kw[e % KD];
        auto k = [&](int w) { return __longlong_as_double((long long)ku[w]); };
        const unsigned slot = (o + a.d[e]) & (RING - 1);
        const unsigned sl = gw_brev((tr[e] + gj[e]) & 63, 6);  // the lane of this output's source
        if constexpr (INT) {
          int_diag(e, ku, slot, sl);
        } else if (ident && e == 0) {  // the identity: [P pt_0] (c0 with C0IN, c1) on q slots
          if (qs) {
            const double kpi = __longlong_as_double((long long)kpid);
#pragma unroll
            for (int c = 0; c < C; c++) {
              a1[c] = f64_mulmod_h(ring[c][slot][jo][sl].d, kpi, q, qinv);
              if constexpr (C0IN)
                a0[c] = f64_mulmod_h(ring[c][slot][NWD - 1][sl].d, kpi, q, qinv);
            }
          }
        } else {
#pragma unroll
          for (int c = 0; c < C; c++) {
            double s0 = a0[c], s1 = a1[c];  // |acc| <= q/2 (+ tiny) between diagonals
#pragma unroll
            for (int j = 0; j < NDIG; j++) {
              const double yv = ring[c][slot][j][sl].d;
              if (j == 2) {  // three digits: fold before the third product
                s0 = f64_red(s0, q, qinv);
                s1 = f64_red(s1, q, qinv);
              }
              s0 += f64_mulmod_h(yv, k(j), q, qinv);
              s1 += f64_mulmod_h(yv, k(NDIG + j), q, qinv);
            }
            if constexpr (C0IN)
              s0 += f64_mulmod_h(ring[c][slot][NWD - 1][sl].d, k(KW), q, qinv);
            if (!LZ || NDIG > 2 || e % 3 == 2) {
              a0[c] = f64_red(s0, q, qinv);  // (|s0| < 3.2 q before; LZ: < 6.9 q)
              a1[c] = f64_red(s1, q, qinv);
            } else {
              a0[c] = s0;
              a1[c] = s1;
            }
          }
        }
      }
    }
#pragma unroll
    for (int c = 0; c < C; c++) {
      if ((unsigned)c >= nc)
        continue;
      uint64_t *op = a.acc + (size_t)(p0 + c) * a.acc_stride + ((size_t)t << logn) + koff;
      if constexpr (INT) {
        uint64_t s0 = u0[c] >= qi ? u0[c] - qi : u0[c], s1 = u1[c] >= qi ? u1[c] - qi : u1[c];
        if (a.accumulate) {
          s0 = add_mod(s0, op[0], qi);
          s1 = add_mod(s1, op[apoly], qi);
        }
        op[0] = s0;
        op[apoly] = s1;
      } else {
        double s0 = a0[c], s1 = a1[c];
        if (a.accumulate) {
          s0 += f64_from_u52(op[0]);
          s1 += f64_from_u52(op[apoly]);
        }
        op[0] = f64_canon(s0, q, qinv);
        op[apoly] = f64_canon(s1, q, qinv);
      }
    }
    __syncthreads();  // the ring slots the next advance overwrites were read here
  }
  };
  if (!INT && NDIG <= 2 && q < (double)F64_LAZY)
    advances(std::true_type{});
  else
    advances(std::false_type{});
}

// ---------------------------------------------------------------------------
// The c0 term of the q slots: acc0[t][k] += sum_d [P pt_d]_t[k] c0[pi_d k],
// run after the digit inner products of the same diagonals (gemv_win_kernel)
// with the same orbit walk and LDS ring, one ring word per ciphertext, so a
// workgroup carries 8 ciphertexts per key word.  The P pt_d words are the
// fold's separate q-slot array (a.Kp).
// FP64: |product| <= 0.875 q (centred ring values, q < 2^51); reduced every
// second diagonal, so |acc| < 2.25 q, and < 3.25 q with the word it adds to.
// ---------------------------------------------------------------------------
template <int W, bool INT, bool SPLIT>
__global__ void __launch_bounds__(1024) gemv_c0_kernel(GemvWin a)
{
  constexpr int C = 8, RING = 32, KD = 3;
  __shared__ GwWord ring[C][RING][64];
  const unsigned logn = a.logn, bb = logn - 6, P = 1u << (bb - 1);
  const unsigned nmem = (a.count + C - 1) / C;
  unsigned grp, mi;
  if (!xcd_group(nmem, a.ns * 2 * a.nseg, grp, mi))
    return;
  const unsigned t = a.slot[grp / (2 * a.nseg)], orb = (grp / a.nseg) & 1, seg = grp % a.nseg;
  const unsigned SEG = P / a.nseg, o0 = seg * SEG;
  const unsigned wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), L = threadIdx.x & 63;
  const unsigned p0 = mi * C;
  const unsigned nc = min((unsigned)C, a.count - p0);
  const double q = a.md.q[t], qinv = a.md.qinv[t];
  const uint64_t qi = a.md.qi[t], qni = a.md.qni[t], q2 = 2 * qi;
  const int E = (int)a.E, dmin = a.d[0], dmax = a.d[E - 1];
  const unsigned jh = gw_brev(L, 6);
  const uint64_t *sp[C];
#pragma unroll
  for (int c = 0; c < C; c++)
    sp[c] = a.x + (size_t)(p0 + ((unsigned)c < nc ? c : 0)) * a.x_stride + ((size_t)t << logn);
  const uint64_t *Kpt = (const uint64_t *)a.Kp + (((size_t)t * a.Etot + a.e0) << logn);
  const uint32_t *tabo = a.tab + (size_t)orb * P * 32;
  uint64_t pv[C];
  auto load_src = [&](unsigned s) {
    const size_t off = ((size_t)tabo[(s & (P - 1)) * 32 + 16] << 6) + L;
#pragma unroll
    for (int c = 0; c < C; c++)
      pv[c] = sp[c][off];
  };
  auto store_src = [&](unsigned s) {
    const unsigned slot = s & (RING - 1);
#pragma unroll
    for (int c = 0; c < C; c++) {
      if constexpr (INT)
        ring[c][slot][L].u = SPLIT ? gw_split(pv[c]) : pv[c];
      else
        ring[c][slot][L].d = gw_center(f64_from_u52(pv[c]), q);
    }
  };
  const unsigned nadv = SEG / 16;
  for (unsigned adv = 0; adv < nadv; adv++) {
    const unsigned ob = o0 + adv * 16;
    if (adv == 0) {
      for (unsigned s = ob + dmin + wv; s < ob + 16 + dmax; s += 16) {
        load_src(s);
        store_src(s);
      }
    } else {
      store_src(ob + dmax + wv);
    }
    __syncthreads();
    const bool more = adv + 1 < nadv;
    const int e_src = min(GW_SRC_AT, E - 1);
    const unsigned o = ob + wv;
    const uint32_t *tr = tabo + (o & (P - 1)) * 32;
    const size_t koff = ((size_t)tr[16] << 6) + L;
    // the accumulator words this advance updates and the next advance's new
    // block: requested at diagonal e_src, behind the first key words (as in
    // gemv_win_kernel)
    uint64_t av[C];
    auto load_acc = [&]() {
#pragma unroll
      for (int c = 0; c < C; c++)
        av[c] = (unsigned)c < nc ? a.acc[(size_t)(p0 + c) * a.acc_stride + ((size_t)t << logn) + koff] : 0;
    };
    double f[C];
    uint64_t u[C];
#pragma unroll
    for (int c = 0; c < C; c++) {
      f[c] = 0.0;
      u[c] = 0;
    }
    // (key words requested on every path, past E at the last diagonal's:
    // loads under the diagonal's branch left the compiler's wait counts
    // conservative at the joins -- a full vmcnt(0) after each)
    uint64_t kd[KD];
#pragma unroll
    for (int e = 0; e < KD - 1; e++)
      kd[e] = Kpt[((size_t)min(e, E - 1) << logn) + koff];
#pragma unroll
    for (int e = 0; e < W; e++) {
      if (e + KD - 1 < W)
        kd[(e + KD - 1) % KD] = Kpt[((size_t)min(e + KD - 1, E - 1) << logn) + koff];
      if (e < E) {
        if (e == e_src) {
          if (more)
            load_src(ob + 16 + dmax + wv);
          load_acc();
        }
        const uint64_t kw = kd[e % KD];
        const unsigned slot = (o + a.d[e]) & (RING - 1);
        const unsigned sl = gw_brev((tr[e] + ((a.hm[e] * jh) & 63)) & 63, 6);
#pragma unroll
        for (int c = 0; c < C; c++) {
          if constexpr (INT) {
            const uint64_t y = ring[c][slot][sl].u;
            uint64_t r;
            if constexpr (SPLIT) {
              GwAcc3 b;
              b.mac(y, kw);
              r = b.redc(qi, qni);
            } else {
              r = gw_redc(mulhi64(y, kw), y * kw, qi, qni);
            }
            u[c] = lazy_lt2q(u[c] + r, q2);
          } else {
            f[c] += f64_mulmod_h(ring[c][slot][sl].d, __longlong_as_double((long long)kw), q, qinv);
            if (e & 1)
              f[c] = f64_red(f[c], q, qinv);
          }
        }
      }
    }
#pragma unroll
    for (int c = 0; c < C; c++) {
      if ((unsigned)c >= nc)
        continue;
      uint64_t *op = a.acc + (size_t)(p0 + c) * a.acc_stride + ((size_t)t << logn) + koff;
      if constexpr (INT)
        op[0] = add_mod(u[c] >= qi ? u[c] - qi : u[c], av[c], qi);
      else
        op[0] = f64_canon(f[c] + f64_from_u52(av[c]), q, qinv);
    }
    __syncthreads();  // the ring slots the next advance overwrites were read here
  }
}

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------
static GwMods gw_mods(unsigned lvl)
{
  GwMods md{};
  const unsigned nm = lvl + G.K;
  for (unsigned t = 0; t < nm; t++) {
    const unsigned m = t < lvl ? t : G.L + (t - lvl);
    const uint64_t qq = G.q[m];
    md.q[t] = (double)qq;
    md.qinv[t] = 1.0 / (double)qq;
    md.qi[t] = qq;
    md.qni[t] = G.mc[m].qneg_inv;
  }
  return md;
}

// bit t: basis slot t of basis_qp(lvl) on 64-bit integer arithmetic (the
// modulus is not below 2^51, or this ring has no FP64 twiddles): the
// kernels' own choice (with_arith)
static uint64_t gw_intmask(unsigned lvl)
{
  uint64_t mask = 0;
  for (unsigned t = 0; t < lvl + G.K; t++)
    if (!G.twd || G.q[t < lvl ? t : G.L + (t - lvl)] >= F64_QMAX)
      mask |= 1ull << t;
  return mask;
}

// the integer slots' split form (GwAcc3) applies: every integer modulus below 2^60
static bool gw_split_ok(unsigned lvl)
{
  for (unsigned t = 0; t < lvl + G.K; t++)
    if (((gw_intmask(lvl) >> t) & 1) && G.q[t < lvl ? t : G.L + (t - lvl)] >= (1ull << 60))
      return false;
  return true;
}

bool k_gemv_win_ok(unsigned lvl)
{
  if (G.logn < 13 || G.logn > 17 || G.alpha > 8)
    return false;
  const unsigned ndig = (lvl + G.alpha - 1) / G.alpha, nm = lvl + G.K;
  if (ndig < 1 || ndig > 3 || nm > GPQHE_MAXMOD / 2)
    return false;
  // integer slots need the split key switch's ModUp (k_modup_c1_split): the
  // fallback conversion below is FP64 only
  return gw_intmask(lvl) == 0 ? G.twd != nullptr : k_ks_fused_ok();
}

static uint64_t gw_pow(uint64_t b, uint64_t e, uint64_t mask)
{
  uint64_t r = 1;
  for (; e; e >>= 1, b = (b * b) & mask)
    if (e & 1)
      r = (r * b) & mask;
  return r;
}

// 5^d and 5^-d mod 2n (5 has order n / 2 there)
static void gw_galois(unsigned d, uint64_t &g, uint64_t &gi)
{
  const uint64_t mask = (2ull << G.logn) - 1, ord = G.n / 2;
  g = gw_pow(5, d % ord, mask);
  gi = gw_pow(5, (ord - d % ord) % ord, mask);
}

size_t k_gemv_fold_words(unsigned E, unsigned lvl)
{
  const unsigned ndig = (lvl + G.alpha - 1) / G.alpha, nm = lvl + G.K;
  return gw_kbase(nm, ndig, E, G.logn) + ((size_t)lvl * E << G.logn);
}

double *k_gemv_fold(const GemvDiagIn *dg, unsigned E, unsigned lvl)
{
  const unsigned ndig = (lvl + G.alpha - 1) / G.alpha, nm = lvl + G.K;
  double *K = (double *)pool_alloc(k_gemv_fold_words(E, lvl) * 8);
  for (unsigned e0 = 0; e0 < E; e0 += FoldArgs::MAX) {
    const unsigned cnt = std::min(FoldArgs::MAX, E - e0);
    FoldArgs fa{};
    fa.e0 = e0;
    fa.intmask = gw_intmask(lvl);
    fa.split = gw_split_ok(lvl);
    for (unsigned e = 0; e < cnt; e++) {
      fa.pt[e] = dg[e0 + e].pt;
      fa.evk[e] = dg[e0 + e].evk;
    }
    ProfScope ps(KC_GEMV_FOLD, 8.0 * G.n * cnt * nm * ((double)(2 * ndig + 1) + (2 * ndig + 2)));
    hipLaunchKernelGGL(gemv_fold_kernel, dim3(G.n / 256, nm, cnt), dim3(256), 0, G.stream, K, fa, E, ndig, G.logn, lvl,
                       G.L, G.nmod, nm, G.dev.mc);
    HIP_CHECK(hipGetLastError());
  }
  return K;
}

static void gemv_chunk(uint64_t *y, size_t y_stride, size_t y_pstride, const uint64_t *x, size_t x_stride,
                       size_t x_pstride, unsigned cnt, unsigned lvl, const double *K, const unsigned *d, unsigned E,
                       int mode)
{
  const UpTable &up = k_up_table(lvl);
  const unsigned n = G.n, logn = G.logn, nm = up.nm, ndig = up.ndig, alpha = G.alpha;
  const GwMods md = gw_mods(lvl);
  // ModUp digits: the split key switch's ModUp kernels (T1 layout: digit j,
  // slot t at j nm + t), else the INTT / conversion / NTT sequence below
  // (compact: digit j's targets outside it, in slot order)
  std::vector<int> yi((size_t)nm * 3, -1);
  const size_t ys = (size_t)lvl * n, as = 2 * (size_t)nm * n;
  size_t ds = (size_t)ndig * nm * n;
  uint64_t *ws = (uint64_t *)pool_alloc((size_t)cnt * (ys + ds + as) * 8);
  uint64_t *ybuf = ws, *Dc = ybuf + cnt * ys, *acc = Dc + cnt * ds;
  if (k_modup_c1_split(Dc, ybuf, x, x_stride, x_pstride, cnt, lvl)) {
    for (unsigned j = 0; j < ndig; j++)
      for (unsigned t = 0; t < nm; t++)
        if (!(t >= j * alpha && t < std::min(j * alpha + alpha, lvl)))
          yi[(size_t)t * 3 + j] = (int)(j * nm + t);
  } else {
    if (gw_intmask(lvl))
      gpqhe_die("gemv batch: no ModUp form for integer moduli at this ring");
    unsigned mods[GPQHE_MAXMOD], S = 0;
    for (unsigned j = 0; j < ndig; j++) {
      const unsigned lo = j * alpha, hi = std::min(lo + alpha, lvl);
      for (unsigned t = 0; t < nm; t++) {
        if (t >= lo && t < hi)
          continue;
        yi[(size_t)t * 3 + j] = (int)S;
        mods[S++] = t < lvl ? t : G.L + (t - lvl);
      }
    }
    ds = (size_t)S * n;  // (within the ndig nm n words reserved per ciphertext)
    // 1. y = INTT(c1) x n^-1 [(Q_j/q_i)^-1]
    LimbSet in{}, yo{};
    in.base = (uint64_t *)x + x_pstride;
    in.per = lvl;
    in.count = lvl * cnt;
    in.stride = x_stride;
    yo = in;
    yo.base = ybuf;
    yo.stride = ys;
    for (unsigned i = 0; i < lvl; i++)
      in.mods[i] = yo.mods[i] = (uint8_t)i;
    k_ntt_ex(in, yo, true, up.ysc);
    // 2. conversion to every slot outside each digit, 3. their forward NTT
    {
      ProfScope ps(KC_GEMV_FBC, 8.0 * n * cnt * ((double)lvl + S));
      hipLaunchKernelGGL(gemv_fbc_kernel, dim3(n / 256, cnt), dim3(256), 0, G.stream, Dc, ds, ybuf, ys, up.cd, md,
                         logn, lvl, nm, ndig, alpha);
      HIP_CHECK(hipGetLastError());
    }
    LimbSet dl{};
    dl.base = Dc;
    dl.per = S;
    dl.count = S * cnt;
    dl.stride = ds;
    for (unsigned i = 0; i < S; i++)
      dl.mods[i] = (uint8_t)mods[i];
    k_ntt(dl, false);
  }
  // 4. the inner products, diagonals in launches spanning at most 16
  // rotations (the LDS ring: 16 output blocks and the 15 more sources they
  // read); segments of >= 16 blocks, enough workgroups to fill the chip
  // the c0 term in the main kernel (C0IN) for three digits and for a few
  // diagonals, else in gemv_c0_kernel's pass (see gemv_win_kernel)
  const bool c0in = ndig >= 3 || E < 4;
  const unsigned P = 1u << (logn - 7), cpw = c0in ? (ndig != 2 ? 2 : 3) : (ndig >= 3 ? 3 : 4);  // (cpw: gw_cts)
  unsigned nseg = 1;
  while (nseg < P / 16 && (size_t)nm * 2 * nseg * ((cnt + cpw - 1) / cpw) < 1024)
    nseg *= 2;
  GemvWin a{};
  a.x = x;
  a.x_stride = x_stride;
  a.x_pstride = x_pstride;
  a.Dc = Dc;
  a.d_stride = ds;
  a.K = K;
  a.Kp = K + gw_kbase(nm, ndig, E, logn);
  a.acc = acc;
  a.acc_stride = as;
  for (unsigned t = 0; t < nm; t++)
    for (unsigned j = 0; j < 3; j++)
      a.yi[t][j] = (int16_t)yi[(size_t)t * 3 + j];
  a.md = md;
  a.Etot = E;
  a.logn = logn;
  a.lvl = lvl;
  a.nm = nm;
  a.count = cnt;
  a.nseg = nseg;
  a.alpha = alpha;
  // the basis slots by arithmetic class: one launch per class and diagonal run
  const uint64_t imask = gw_intmask(lvl);
  GemvWin acls[2] = {a, a};  // [0] FP64 slots, [1] integer slots
  GemvWin qcls[2] = {a, a};  // their q slots (the c0 term)
  for (unsigned t = 0; t < nm; t++) {
    GemvWin &c = acls[(imask >> t) & 1];
    c.slot[c.ns++] = (uint8_t)t;
    if (t < lvl) {
      GemvWin &cq = qcls[(imask >> t) & 1];
      cq.slot[cq.ns++] = (uint8_t)t;
    }
  }
  const bool split = gw_split_ok(lvl);
  uint32_t *tab = (uint32_t *)pool_alloc((size_t)2 * P * 32 * 4);
  bool first = true;
  for (unsigned e0 = 0; e0 < E;) {
    unsigned e1 = e0;
    while (e1 < E && e1 - e0 < GemvWin::MAXE && d[e1] - d[e0] < 16)
      e1++;
    a.E = e1 - e0;
    a.e0 = e0;
    a.accumulate = first ? 0 : 1;
    GemvTab ta{};
    ta.E = a.E;
    ta.logn = logn;
    for (unsigned e = 0; e < a.E; e++) {
      uint64_t g, gi;
      gw_galois(d[e0 + e], g, gi);
      a.d[e] = (int32_t)d[e0 + e];
      a.hm[e] = (uint32_t)(g & 63);
      ta.g[e] = g;
    }
    hipLaunchKernelGGL(gemv_tab_kernel, dim3((2 * P * 32 + 255) / 256), dim3(256), 0, G.stream, tab, ta);
    HIP_CHECK(hipGetLastError());
    a.tab = tab;
    auto setup = [&](GemvWin &c) {
      memcpy(c.d, a.d, sizeof a.d);
      memcpy(c.hm, a.hm, sizeof a.hm);
      c.tab = a.tab;
      c.E = a.E;
      c.e0 = a.e0;
      c.accumulate = a.accumulate;
    };
    {
      // reads each ciphertext's ModUp digits once, the folded keys once per
      // slot, orbit and ciphertext group, writes (or updates) the accumulators
      ProfScope ps(KC_GEMV_WIN, 8.0 * n * ((double)cnt * (ndig * nm + (c0in ? lvl : 0) + (first ? 2.0 : 4.0) * nm) +
                                           (double)a.E * (nm * 2 * ndig + (c0in ? lvl : 0))));
      for (int ic = 0; ic < 2; ic++) {
        GemvWin &c = acls[ic];
        if (!c.ns)
          continue;
        setup(c);
        const dim3 grid(xcd_blocks((cnt + cpw - 1) / cpw, c.ns * 2 * nseg));
        auto go = [&](auto kern) { hipLaunchKernelGGL(kern, grid, dim3(1024), 0, G.stream, c); };
        // (KF: the FP64 forms of launches of 8 diagonals and more)
        auto form = [&](auto c0) {
          constexpr bool C0 = decltype(c0)::value;
          switch (ndig * 2 + ic) {
          case 2:
            c.E >= 8 ? go(gemv_win_kernel<1, 16, false, false, C0, true>) : go(gemv_win_kernel<1, 16, false, false, C0>);
            break;
          case 3:
            if (split)
              go(gemv_win_kernel<1, 16, true, true, C0>);
            else
              go(gemv_win_kernel<1, 16, true, false, C0>);
            break;
          case 4:
            c.E >= 8 ? go(gemv_win_kernel<2, 16, false, false, C0, true>) : go(gemv_win_kernel<2, 16, false, false, C0>);
            break;
          case 5:
            if (split)
              go(gemv_win_kernel<2, 16, true, true, C0>);
            else
              go(gemv_win_kernel<2, 16, true, false, C0>);
            break;
          default: break;
          }
        };
        if (ndig >= 3) {  // (always C0IN)
          if (!ic)
            c.E >= 8 ? go(gemv_win_kernel<3, 16, false, false, true, true>) : go(gemv_win_kernel<3, 16, false, false, true>);
          else if (split)
            go(gemv_win_kernel<3, 16, true, true, true>);
          else
            go(gemv_win_kernel<3, 16, true, false, true>);
        } else if (c0in) {
          form(std::true_type{});
        } else {
          form(std::false_type{});
        }
        HIP_CHECK(hipGetLastError());
      }
    }
    if (!c0in) {
      // the q slots' c0 term: reads c0 once per ciphertext, the P pt_d words
      // once per slot, orbit and group of 8, updates the accumulators' poly 0
      ProfScope ps(KC_GEMV_C0, 8.0 * n * ((double)cnt * 3.0 * lvl + (double)a.E * lvl));
      for (int ic = 0; ic < 2; ic++) {
        GemvWin &c = qcls[ic];
        if (!c.ns)
          continue;
        setup(c);
        // segments: one workgroup per CU at least (the c0 pass streams; its
        // ring fill at each segment start is not hidden by compute)
        unsigned nseg0 = 1;
        while (nseg0 < P / 16 && (size_t)c.ns * 2 * nseg0 * ((cnt + 7) / 8) < 256)
          nseg0 *= 2;
        c.nseg = nseg0;
        const dim3 grid(xcd_blocks((cnt + 7) / 8, c.ns * 2 * nseg0));
        auto go = [&](auto kern) { hipLaunchKernelGGL(kern, grid, dim3(1024), 0, G.stream, c); };
        if (!ic)
          go(gemv_c0_kernel<16, false, false>);
        else if (split)
          go(gemv_c0_kernel<16, true, true>);
        else
          go(gemv_c0_kernel<16, true, false>);
        HIP_CHECK(hipGetLastError());
      }
    }
    first = false;
    e0 = e1;
  }
  pool_free(tab);
  // 5. ModDown of both accumulators of every ciphertext: the dropped slots'
  // inverse row pass, then the fused conversion (dn_cols) and combine (dn_rows)
  if (!E)
    HIP_CHECK(hipMemsetAsync(acc, 0, (size_t)cnt * as * 8, G.stream));
  const unsigned keep = mode == 1 ? lvl - 1 : lvl, nd = nm - keep;
  const bool fused = k_ks_fused_ok() && nd <= 5;
  bool pre = false, s79 = false;
  if (fused) {
    LimbSet dr{};
    dr.base = acc + ((size_t)keep << logn);
    dr.per = nd;
    dr.count = nd * 2 * cnt;
    dr.stride = (size_t)nm * n;
    for (unsigned d = 0; d < nd; d++)
      dr.mods[d] = (uint8_t)(keep + d < lvl ? keep + d : G.L + (keep + d - lvl));
    // the ModDown scale on the row pass's output, so dn_cols runs its
    // pre-scaled (staged-constant) form
    // (n = 2^16: on 512-element rows, so the ModDown's column kernels run
    // their T = 128 forms, as the split key switch's: GPQHE_DN_S79=0 keeps
    // 256 x 256)
    const char *sw = getenv("GPQHE_DN_S79");
    s79 = logn == 16 && !(sw && atoi(sw) == 0);
    pre = k_ntt_rows_down(dr, lvl, mode, s79);
    if (!pre) {
      s79 = false;
      k_ntt_rows(dr, dr, true);
    }
  }
  auto down = [&](uint64_t *o, uint64_t *X, unsigned npoly) {
    if (fused)
      k_moddown_fused(o, y_pstride, X, (size_t)nm * n, npoly, lvl, mode, pre, s79);
    else
      k_moddown(o, y_pstride, X, (size_t)nm * n, npoly, lvl, mode);
  };
  if (y_stride == 2 * y_pstride) {
    down(y, acc, 2 * cnt);
  } else {
    for (unsigned c = 0; c < cnt; c++)  // (one ciphertext: an object's own layout)
      down(y + c * y_stride, acc + c * as, 2);
  }
  pool_free(ws);
}

void k_gemv_batch_ex(uint64_t *y, size_t y_stride, size_t y_pstride, const uint64_t *x, size_t x_stride,
                     size_t x_pstride, size_t count, unsigned lvl, const double *K, const unsigned *d, unsigned E,
                     int mode)
{
  const unsigned ndig = (lvl + G.alpha - 1) / G.alpha, nm = lvl + G.K;
  const size_t per_ct = ((size_t)lvl + (size_t)ndig * nm + 2 * (size_t)nm) * G.n * 8;
  const size_t budget = (size_t)8 << 30;
  size_t chunk = std::max<size_t>(1, std::min<size_t>(budget / per_ct, 65535 / (3 * nm)));
  if (const char *e = getenv("GPQHE_GEMV_CHUNK"))  // test hook: several chunks on a small batch
    chunk = std::max<size_t>(1, std::min<size_t>(chunk, strtoul(e, nullptr, 0)));
  for (size_t c0 = 0; c0 < count; c0 += chunk) {
    const unsigned cnt = (unsigned)std::min(chunk, count - c0);
    gemv_chunk(y + c0 * y_stride, y_stride, y_pstride, x + c0 * x_stride, x_stride, x_pstride, cnt, lvl, K, d, E,
               mode);
  }
}

void k_gemv_batch(uint64_t *y, const uint64_t *x, size_t count, unsigned lvl, const double *K, const unsigned *d,
                  unsigned E, int mode)
{
  const size_t n = G.n, keep = mode == 1 ? lvl - 1 : lvl;
  k_gemv_batch_ex(y, 2 * keep * n, keep * n, x, 2 * (size_t)lvl * n, (size_t)lvl * n, count, lvl, K, d, E, mode);
}
