// ntt_device.h - device building blocks shared by the gfx950 kernel files:
// modular / FP64 arithmetic policies, the 4-step NTT column and row passes on
// LDS tiles, and the XCD-aware block mapping.
#pragma once

#include "gpqhe_internal.h"

#include <type_traits>

// ===========================================================================
// NTT v2 (two-pass, n = 2^13 .. 2^16): 4096-element tiles, 256 threads,
// Harvey lazy butterflies (values in [0, 4q) inside a pass, canonical at every
// pass boundary), interleaved (w, w') twiddle pairs (one 16-byte load), round
// A loaded straight from HBM into registers, prime-major workgroup order so
// the workgroups resident at one time share one prime's twiddle table.
// ===========================================================================
struct Tw2 {
  const uint64_t *fwd;  // [nmod][n][2] (w, floor(w 2^64 / q))
  const uint64_t *inv;
  const double *fwdd;   // [nmod][n][2] (w, w / q) as doubles (moduli < 2^51)
  const double *invd;
};

__device__ __forceinline__ uint64_t lazy_lt2q(uint64_t x, uint64_t q2)
{
  return x >= q2 ? x - q2 : x;
}

__device__ __forceinline__ uint64_t canon4(uint64_t x, uint64_t q, uint64_t q2)
{
  x = x >= q2 ? x - q2 : x;
  return x >= q ? x - q : x;
}

// forward CT stages on E = 2^LE registers; twiddle run of stage s starts at
// bb >> (log_thi - s + 1); inputs < 4q, outputs < 4q
template <int LE>
__device__ __forceinline__ void fwd_stages(uint64_t (&x)[1 << LE], const uint64_t *__restrict__ tw2, uint64_t bb,
                                           int log_thi, uint64_t q)
{
  constexpr int E = 1 << LE;
  const uint64_t q2 = 2 * q;
#pragma unroll
  for (int s = 0; s < LE; s++) {
    const uint64_t Bs = bb >> (log_thi - s + 1);
    const int half = E >> (s + 1);
#pragma unroll
    for (int k = 0; k < E; k++) {
      if (k & half)
        continue;
      const uint64_t i2 = 2 * (Bs + (uint64_t)(k >> (LE - s)));
      const uint64_t w = tw2[i2], wp = tw2[i2 + 1];
      const uint64_t U = lazy_lt2q(x[k], q2);
      const uint64_t V = mul_shoup_lazy(x[k + half], w, wp, q);
      x[k] = U + V;
      x[k + half] = U - V + q2;
    }
  }
}

// inverse GS stages; inputs < 2q, outputs < 2q
template <int LE>
__device__ __forceinline__ void inv_stages(uint64_t (&x)[1 << LE], const uint64_t *__restrict__ tw2, uint64_t bb,
                                           int log_tlo, uint64_t q)
{
  constexpr int E = 1 << LE;
  const uint64_t q2 = 2 * q;
#pragma unroll
  for (int s = 0; s < LE; s++) {
    const uint64_t Bs = bb >> (log_tlo + s + 1);
    const int half = 1 << s;
#pragma unroll
    for (int k = 0; k < E; k++) {
      if (k & half)
        continue;
      const uint64_t i2 = 2 * (Bs + (uint64_t)(k >> (s + 1)));
      const uint64_t w = tw2[i2], wp = tw2[i2 + 1];
      const uint64_t U = x[k], V = x[k + half];
      x[k] = lazy_lt2q(U + V, q2);
      x[k + half] = mul_shoup_lazy(U - V + q2, w, wp, q);
    }
  }
}

// ---------------------------------------------------------------------------
// FP64 butterflies for moduli q < 2^51 (the FP64 pipe is full rate on gfx950
// and twice as fast as 64-bit integer Shoup per butterfly, scripts/ubench_bfly).
// Values are signed doubles holding exact integers:
//   mulmod: h = fl(y w), l = fma(y, w, -h) (exact), qt = rint(y fl(w/q)),
//           T = fma(-qt, q, h) + l = y w - qt q exactly.  The quotient error
//           is below 1/2 + |y| 2^-52, so for |y| <= 2q < 2^52 |T| < 1.5 q.
//   red:    x - rint(x fl(1/q)) q, |result| <= q/2 (+ negligible).
// CT: X = red(x[k]), T = mulmod(x[k+h]); outputs X +- T, |.| < 2q.
// GS: outputs red(U + V) and mulmod(U - V) with |U - V| < 2q.
// Every intermediate is an integer below 2^53, so the residues are exact and
// the canonical outputs equal the integer path's bit for bit.
// ---------------------------------------------------------------------------
__device__ __forceinline__ double f64_mulmod(double y, double w, double wq, double q)
{
  const double h = y * w;
  const double l = __fma_rn(y, w, -h);
  const double qt = rint(y * wq);
  return __fma_rn(-qt, q, h) + l;
}

// The same product with the quotient estimated from h itself, for a w whose
// w / q is not at hand (twiddles staged as 8-byte entries, key words, data x
// data products): qt = rint(fl(h) fl(1/q)) is off by < 1/2 + 1.5 |y| 2^-52,
// the bound of a recomputed fl(w fl(1/q)) quotient, one multiply fewer.
__device__ __forceinline__ double f64_mulmod_h(double y, double w, double q, double qinv)
{
  const double h = y * w;
  const double l = __fma_rn(y, w, -h);
  const double qt = rint(h * qinv);
  return __fma_rn(-qt, q, h) + l;
}

__device__ __forceinline__ double f64_red(double x, double q, double qinv)
{
  return __fma_rn(-rint(x * qinv), q, x);
}

// u64 <-> f64 for integers below 2^52 without the generic conversions (4 and
// ~7 instructions): 2^52 + x has x as its mantissa bits.
__device__ __forceinline__ double f64_from_u52(uint64_t x)
{
  return __longlong_as_double((long long)(x | 0x4330000000000000ull)) - 0x1p52;
}

// canonical residue of x (integer, |x| < 2^53): reduce, lift negatives by
// q and read the mantissa of 2^52 + v
__device__ __forceinline__ uint64_t f64_canon(double x, double q, double qinv)
{
  const double v = f64_red(x, q, qinv);
  const double b = v < 0 ? q + 0x1p52 : 0x1p52;
  return (uint64_t)__double_as_longlong(v + b) & ((1ull << 52) - 1);
}

// Bounds (|y| = b q; the quotient estimate is off by < 1/2 + |y| 2^-52, so
// |T| <= q (1/2 + |y| 2^-52), and every value must stay an exact integer
// below 2^53):
// * lz (q < 2^50): the reduction of the CT input X (forward) / of U + V
//   (inverse) is skipped on every odd stage of a call.  Forward: b stays
//   below 2.55.  Inverse: a 3-stage call maps b to 1 + b/2, a 4-stage call to
//   2 + b; the chains between canonical values here are at most 4 + 4 stages,
//   so b <= 5 (5 q < 2^52.4).
// * q >= 2^50: X / U + V reduced every stage; the inverse products T grow by
//   up to q/2 a stage, so they are reduced at the last stage of every call
//   (<= 4 stages: b < 2.5).  Canonical outputs are bit-identical either way.
template <int LE>
__device__ __forceinline__ void fwd_stages_f(double (&x)[1 << LE], const double *__restrict__ twd, uint64_t bb,
                                             int log_thi, double q, double qinv, bool lz = false)
{
  constexpr int E = 1 << LE;
#pragma unroll
  for (int s = 0; s < LE; s++) {
    const uint64_t Bs = bb >> (log_thi - s + 1);
    const int half = E >> (s + 1);
    if (!(lz && (s & 1))) {
#pragma unroll
      for (int k = 0; k < E; k++)
        if (!(k & half))
          x[k] = f64_red(x[k], q, qinv);
    }
#pragma unroll
    for (int k = 0; k < E; k++) {
      if (k & half)
        continue;
      const uint64_t i2 = 2 * (Bs + (uint64_t)(k >> (LE - s)));
      const double X = x[k];
      const double T = f64_mulmod(x[k + half], twd[i2], twd[i2 + 1], q);
      x[k] = X + T;
      x[k + half] = X - T;
    }
  }
}

template <int LE>
__device__ __forceinline__ void inv_stages_f(double (&x)[1 << LE], const double *__restrict__ twd, uint64_t bb,
                                             int log_tlo, double q, double qinv, bool lz = false)
{
  constexpr int E = 1 << LE;
#pragma unroll
  for (int s = 0; s < LE; s++) {
    const uint64_t Bs = bb >> (log_tlo + s + 1);
    const int half = 1 << s;
    const bool red = !(lz && (s & 1));
#pragma unroll
    for (int k = 0; k < E; k++) {
      if (k & half)
        continue;
      const uint64_t i2 = 2 * (Bs + (uint64_t)(k >> (s + 1)));
      const double U = x[k], V = x[k + half];
      x[k] = U + V;
      x[k + half] = f64_mulmod(U - V, twd[i2], twd[i2 + 1], q);
    }
    if (red) {
#pragma unroll
      for (int k = 0; k < E; k++)
        if (!(k & half))
          x[k] = f64_red(x[k], q, qinv);
    }
    if (!lz && s == LE - 1) {
      // q >= 2^50: |T| <= q/2 + |U - V| q 2^-52 can grow by q/2 a stage, so
      // the products are reduced at the last stage of every call (calls span
      // at most 4 stages: |.| < 2.5 q, exact, throughout)
#pragma unroll
      for (int k = 0; k < E; k++)
        if (k & half)
          x[k] = f64_red(x[k], q, qinv);
    }
  }
}

#ifndef F64_LZ_CALL
#define F64_LZ_CALL 1
#endif

// Arithmetic policies: the NTT kernels are written once against these.  Both
// read and write canonical u64 residues; ArF64 requires q < 2^51.
struct ArInt {
  using V = uint64_t;
  uint64_t q;
  const uint64_t *tw;   // this modulus' forward (w, w') pairs
  const uint64_t *itw;  // and inverse
  __device__ static V load(uint64_t x) { return x; }
  __device__ uint64_t canon(V x) const { return canon4(x, q, 2 * q); }  // x < 4q
  // forward-transform intermediates between a column and a row pass (T1,
  // conv, the NTT's own): canonical words on integer moduli
  __device__ static V load_lazy(uint64_t b) { return b; }
  __device__ uint64_t store_lazy(V x) const { return canon(x); }
  __device__ static uint64_t bits(V x) { return x; }
  __device__ static V unbits(uint64_t b) { return b; }
  template <int LE>
  __device__ void fwd(V (&x)[1 << LE], uint64_t bb, int log_thi) const { fwd_stages<LE>(x, tw, bb, log_thi, q); }
  template <int LE>
  __device__ void inv(V (&x)[1 << LE], uint64_t bb, int log_tlo) const { inv_stages<LE>(x, itw, bb, log_tlo, q); }
  // canonical x w for a constant w < q (Shoup pair)
  __device__ uint64_t mulc(V x, uint64_t w, uint64_t wp) const { return mul_shoup(x, w, wp, q); }
  __device__ uint64_t mulc_d(V x, uint64_t w, uint64_t wp) const { return mulc(x, w, wp); }  // (FP64 only)
  __device__ uint64_t canon_d(V x) const { return canon(x); }                              // (FP64 only)
};

struct ArF64 {
  using V = double;
  double q, qinv;
  const double *tw;   // this modulus' forward (w, w / q) pairs
  const double *itw;  // and inverse
  bool lz = false;    // q < 2^50: lazy reduction on alternate stages (fwd_stages_f)
  __device__ static V load(uint64_t x) { return f64_from_u52(x); }  // x canonical (< q)
  __device__ uint64_t canon(V x) const { return f64_canon(x, q, qinv); }
  // forward-transform intermediates (T1, conv, the NTT's own): the lazy
  // double itself (|x| < 2q, an exact integer), no canonicalisation, no
  // conversion -- a stage boundary inside one pass sees the same values
  __device__ static V load_lazy(uint64_t b) { return unbits(b); }
  __device__ static uint64_t store_lazy(V x) { return bits(x); }
  __device__ static uint64_t bits(V x) { return (uint64_t)__double_as_longlong(x); }
  __device__ static V unbits(uint64_t b) { return __longlong_as_double((long long)b); }
  // (one uniform branch per call on lz: passed into the stages, it is
  // if-converted -- both reductions computed, one selected -- see ArF64Row)
  template <int LE>
  __device__ void fwd(V (&x)[1 << LE], uint64_t bb, int log_thi) const
  {
#if F64_LZ_CALL
    if (lz)
      fwd_stages_f<LE>(x, tw, bb, log_thi, q, qinv, true);
    else
      fwd_stages_f<LE>(x, tw, bb, log_thi, q, qinv, false);
#else
    fwd_stages_f<LE>(x, tw, bb, log_thi, q, qinv, lz);
#endif
  }
  template <int LE>
  __device__ void inv(V (&x)[1 << LE], uint64_t bb, int log_tlo) const
  {
#if F64_LZ_CALL
    if (lz)
      inv_stages_f<LE>(x, itw, bb, log_tlo, q, qinv, true);
    else
      inv_stages_f<LE>(x, itw, bb, log_tlo, q, qinv, false);
#else
    inv_stages_f<LE>(x, itw, bb, log_tlo, q, qinv, lz);
#endif
  }
  __device__ uint64_t mulc(V x, uint64_t w, uint64_t) const
  {
    const double wd = f64_from_u52(w);
    return canon(f64_mulmod(x, wd, wd / q, q));
  }
  // x (|x| < 2^53) as the bits of a canonical double in [0, q) (FP64 basis
  // conversion input)
  __device__ uint64_t canon_d(V x) const
  {
    const double v = f64_red(x, q, qinv);
    return (uint64_t)__double_as_longlong(v < 0 ? v + q : v);
  }
  // x w as the bits of a canonical double in [0, q) (FP64 basis conversion input)
  __device__ uint64_t mulc_d(V x, uint64_t w, uint64_t) const
  {
    const double wd = f64_from_u52(w);
    const double v = f64_red(f64_mulmod(x, wd, wd / q, q), q, qinv);
    return (uint64_t)__double_as_longlong(v < 0 ? v + q : v);
  }
};

// ArF64 for the all-FP64 column passes (cols_f64.hip): the twiddles from an
// LDS table holding entries [0, T) of the modulus' (w, w / q) table -- a T-row
// column pass reads no others -- and the lazy-reduction choice fixed at
// compile time, so a transform is straight-line code with no global loads.
// Same stages as ArF64, so the same bits.
// SB: a scheduling barrier after every forward stage, so the compiler does
// not hoist all of a 16-element round's LDS twiddle reads (60 VGPRs) to its
// start (the T = 256 ModDown columns then spill 20 B/lane; with it, none).
template <int LE, bool SB>
__device__ __forceinline__ void fwd_stages_fl(double (&x)[1 << LE], const double *__restrict__ twd, uint64_t bb,
                                              int log_thi, double q, double qinv, bool lz)
{
  if constexpr (!SB) {
    fwd_stages_f<LE>(x, twd, bb, log_thi, q, qinv, lz);
  } else {
    constexpr int E = 1 << LE;
#pragma unroll
    for (int s = 0; s < LE; s++) {
      const uint64_t Bs = bb >> (log_thi - s + 1);
      const int half = E >> (s + 1);
      if (!(lz && (s & 1))) {
#pragma unroll
        for (int k = 0; k < E; k++)
          if (!(k & half))
            x[k] = f64_red(x[k], q, qinv);
      }
#pragma unroll
      for (int k = 0; k < E; k++) {
        if (k & half)
          continue;
        const uint64_t i2 = 2 * (Bs + (uint64_t)(k >> (LE - s)));
        const double X = x[k];
        const double T = f64_mulmod(x[k + half], twd[i2], twd[i2 + 1], q);
        x[k] = X + T;
        x[k + half] = X - T;
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

template <bool LZ, bool SB = false>
struct ArF64C : ArF64 {
  const double *twl;  // LDS: [T][2]
  template <int LE>
  __device__ __forceinline__ void fwd(V (&x)[1 << LE], uint64_t bb, int log_thi) const
  {
    fwd_stages_fl<LE, SB>(x, twl, bb, log_thi, q, qinv, LZ);
  }
  template <int LE>
  __device__ __forceinline__ void inv(V (&x)[1 << LE], uint64_t bb, int log_tlo) const
  {
    inv_stages_f<LE>(x, twl, bb, log_tlo, q, qinv, LZ);
  }
};

template <bool LZ, bool SB = false>
__device__ __forceinline__ ArF64C<LZ, SB> make_f64c(double q, const double *twl)
{
  ArF64C<LZ, SB> a;
  a.q = q;
  a.qinv = 1.0 / q;
  a.tw = a.itw = nullptr;
  a.lz = LZ;
  a.twl = twl;
  return a;
}

// ONE: every modulus on the non-lazy policy (one instantiation of f; the
// non-lazy stages are exact for every q < 2^51)
template <bool SB = false, int ONE = 0, class F>
__device__ __forceinline__ void with_f64c(double q, const double *twl, F &&f)
{
  if (!ONE && q < (double)(1ull << 50))
    f(make_f64c<true, SB>(q, twl));
  else
    f(make_f64c<false, SB>(q, twl));
}

// FP64 fast basis conversion term y c mod q_t for canonical y < q_i < 2^51 and
// a constant c < q_t < 2^51 with cq = fl(c / q_t): y c / q_t < 2^51, so the
// quotient estimate is off by at most 1, |result| <= q_t and every
// intermediate is an integer below 2^53 (exact).  Sums of up to three terms
// stay below 2^53; longer sums are reduced in between (f64_red).
__device__ __forceinline__ double fbc_term(double y, double c, double cq, double q)
{
  return f64_mulmod(y, c, cq, q);
}

// Streaming stores for the pipeline intermediates (read back once by the next
// kernel); GPQHE_PLAIN_STORES builds the plain-store variant for A/B runs.
#ifdef GPQHE_PLAIN_STORES
#define ST_STREAM(v, p) (*(p) = (v))
#else
#define ST_STREAM(v, p) __builtin_nontemporal_store((v), (p))
#endif

constexpr uint64_t F64_QMAX = 1ull << 51;  // ArF64 applies to moduli below this

// x w mod q, canonical, for canonical x and a constant w < q with its Shoup
// companion wp: the exact FP64 product below F64_QMAX (as dn_rows_kernel's
// epilogue), 64-bit Shoup above
__device__ __forceinline__ uint64_t mulc_canon(uint64_t x, uint64_t w, uint64_t wp, uint64_t q)
{
  if (q < F64_QMAX) {
    const double qd = (double)q, qinv = 1.0 / qd, wd = f64_from_u52(w);
    return f64_canon(f64_mulmod(f64_from_u52(x), wd, wd * qinv, qd), qd, qinv);
  }
  return mul_shoup(x, w, wp, q);
}
constexpr uint64_t F64_LAZY = 1ull << 50;  // and its lazy stage reduction below this

// Forward row passes with the twiddles of one row tile staged in LDS.  A
// 2^LOGN2-point row pass of global row rho uses, at its stage of level lam
// (0 .. LOGN2-1), the 2^lam twiddles tw[rho 2^lam + g]; the R rows
// [rho0, rho0 + R) of a tile need R 2^lam consecutive entries per level,
// stored at R (2^lam - 1) (R (2^LOGN2 - 1) 16-byte entries in all, ~32 KB).
// A stage whose run starts at Bs = bb >> shift is at level LOGN2 - shift.
template <int LOGN2>
struct RowTw {
  static constexpr int R = 2048 >> LOGN2, ENTRIES = R * ((1 << LOGN2) - 1);
  const uint64_t *lds;  // ENTRIES x 2 words
  int64_t rel;          // R - rho0
  __device__ __forceinline__ uint64_t idx(uint64_t i, int shift) const
  {
    return (uint64_t)((int64_t)i + (rel << (LOGN2 - shift)) - R);
  }
  // copy the tile's entries of a [n][2] table (16-byte entries) into lds; W8:
  // only the first word of each (8-byte entries: FP64 w, w / q recomputed)
  template <bool W8 = false>
  static __device__ __forceinline__ void stage(uint64_t *dst, const uint64_t *tab, unsigned rho0, unsigned tid,
                                               unsigned nthreads)
  {
    for (unsigned e = tid; e < (unsigned)ENTRIES; e += nthreads) {
      const unsigned lam = 31 - __clz(e / R + 1);  // level of entry e: R (2^lam - 1) <= e
      const unsigned g = e - R * ((1u << lam) - 1);
      const size_t src = ((size_t)rho0 << lam) + g;
      if (W8)
        dst[e] = tab[2 * src];
      else
        ((ulonglong2 *)dst)[e] = ((const ulonglong2 *)tab)[src];
    }
  }
};

// ArF64 / ArInt with the forward twiddles from a RowTw table (the inverse
// stays on the global table).  ArF64Row<.., true>: 8-byte entries (w only,
// w / q recomputed as w fl(1/q)) for both directions (itl: inverse).  The
// recomputed quotient constant widens the estimate's error to 1.5 |y| 2^-52,
// so on moduli >= 2^50 the products are reduced every stage (inverse) and
// every other stage (forward): |.| < 1.75 q throughout, exact; below 2^50
// the lazy bounds of fwd_stages_f / inv_stages_f hold with room to spare.
// GINV: 8-byte forward entries staged, the inverse on the global table (for
// kernels whose LDS leaves room for one direction only)
template <int LOGN2, bool W8 = false, bool GINV = false, int LZC = -1>
struct ArF64Row : ArF64 {
  RowTw<LOGN2> rt;
  const uint64_t *itl = nullptr;
  // LZC: the lazy-reduction choice -- 0 / 1 at compile time, -1 one uniform
  // branch per call (fwd / inv below), -2 per element at run time (which the
  // compiler if-converts: both reductions computed, one selected, so every
  // modulus pays the wide one; fewer registers than -1 in some kernels);
  // -3 / -4: per call forward and per element inverse / the reverse
  __device__ __forceinline__ double2 twf(const uint64_t *tab, uint64_t e) const
  {
    if constexpr (W8) {
      const double w = __longlong_as_double((long long)tab[e]);
      return make_double2(w, w * qinv);
    } else {
      return ((const double2 *)tab)[e];
    }
  }
  // The lazy-reduction choice is made once per call (LZ below), not per
  // element: a run-time lz inside the stages is if-converted (both
  // reductions computed, one selected), so every modulus paid the wide one.
  template <int LE>
  __device__ __forceinline__ void fwd(V (&x)[1 << LE], uint64_t bb, int log_thi) const
  {
    constexpr int FM = LZC == -3 ? -1 : LZC == -4 ? -2 : LZC;
    if constexpr (FM != -1)
      fwd_p<LE, FM>(x, bb, log_thi);
    else if (lz)
      fwd_p<LE, 1>(x, bb, log_thi);
    else
      fwd_p<LE, 0>(x, bb, log_thi);
  }
  template <int LE>
  __device__ __forceinline__ void inv(V (&x)[1 << LE], uint64_t bb, int log_tlo) const
  {
    constexpr int IM = LZC == -3 ? -2 : LZC == -4 ? -1 : LZC;
    if (GINV || (!W8 && !itl))  // (uniform) no staged inverse table: the global one
      ArF64::inv<LE>(x, bb, log_tlo);
    else if constexpr (IM != -1)
      inv_p<LE, IM>(x, bb, log_tlo);
    else if (lz)
      inv_p<LE, 1>(x, bb, log_tlo);
    else
      inv_p<LE, 0>(x, bb, log_tlo);
  }
  template <int LE, int LZM>
  __device__ __forceinline__ void fwd_p(V (&x)[1 << LE], uint64_t bb, int log_thi) const
  {
    constexpr int E = 1 << LE;
    const bool LZ = LZM < 0 ? lz : LZM != 0;
#pragma unroll
    for (int s = 0; s < LE; s++) {
      const int shift = log_thi - s + 1;
      const uint64_t Bs = bb >> shift;
      const int half = E >> (s + 1);
      if (!(LZ && (s & 1))) {  // lazy reduction: see fwd_stages_f
#pragma unroll
        for (int k = 0; k < E; k++)
          if (!(k & half))
            x[k] = f64_red(x[k], q, qinv);
      }
#pragma unroll
      for (int k = 0; k < E; k++) {
        if (k & half)
          continue;
        const uint64_t e = rt.idx(Bs + (uint64_t)(k >> (LE - s)), shift);
        const double X = x[k];
        double T;
        if constexpr (W8) {
          T = f64_mulmod_h(x[k + half], __longlong_as_double((long long)rt.lds[e]), q, qinv);
        } else {
          const double2 w = twf(rt.lds, e);
          T = f64_mulmod(x[k + half], w.x, w.y, q);
        }
        if (W8 && !LZ && (s & 1))
          T = f64_red(T, q, qinv);  // recomputed w/q on a wide modulus: see below
        x[k] = X + T;
        x[k + half] = X - T;
      }
    }
  }
  template <int LE, int LZM>
  __device__ __forceinline__ void inv_p(V (&x)[1 << LE], uint64_t bb, int log_tlo) const
  {
    const bool LZ = LZM < 0 ? lz : LZM != 0;
    {
      constexpr int E = 1 << LE;
#pragma unroll
      for (int s = 0; s < LE; s++) {
        const int shift = log_tlo + s + 1;
        const uint64_t Bs = bb >> shift;
        const int half = 1 << s;
#pragma unroll
        for (int k = 0; k < E; k++) {
          if (k & half)
            continue;
          const uint64_t e = rt.idx(Bs + (uint64_t)(k >> (s + 1)), shift);
          const double U = x[k], V_ = x[k + half];
          x[k] = U + V_;
          if constexpr (W8) {
            x[k + half] = f64_mulmod_h(U - V_, __longlong_as_double((long long)itl[e]), q, qinv);
          } else {
            const double2 w = twf(itl, e);
            x[k + half] = f64_mulmod(U - V_, w.x, w.y, q);
          }
          if (W8 && !LZ)  // recomputed w/q on a wide modulus: see above
            x[k + half] = f64_red(x[k + half], q, qinv);
        }
        if (!(LZ && (s & 1))) {  // lazy reduction: see inv_stages_f
#pragma unroll
          for (int k = 0; k < E; k++)
            if (!(k & half))
              x[k] = f64_red(x[k], q, qinv);
        }
        if (!W8 && !LZ && s == LE - 1) {  // wide moduli: bounded products, see inv_stages_f
#pragma unroll
          for (int k = 0; k < E; k++)
            if (k & half)
              x[k] = f64_red(x[k], q, qinv);
        }
      }
    }
  }
};

template <int LOGN2>
struct ArIntRow : ArInt {
  RowTw<LOGN2> rt;
  template <int LE>
  __device__ void fwd(V (&x)[1 << LE], uint64_t bb, int log_thi) const
  {
    constexpr int E = 1 << LE;
    const uint64_t q2 = 2 * q;
#pragma unroll
    for (int s = 0; s < LE; s++) {
      const int shift = log_thi - s + 1;
      const uint64_t Bs = bb >> shift;
      const int half = E >> (s + 1);
#pragma unroll
      for (int k = 0; k < E; k++) {
        if (k & half)
          continue;
        const uint64_t e = rt.idx(Bs + (uint64_t)(k >> (LE - s)), shift);
        const ulonglong2 w = ((const ulonglong2 *)rt.lds)[e];
        const uint64_t U = lazy_lt2q(x[k], q2);
        const uint64_t V_ = mul_shoup_lazy(x[k + half], w.x, w.y, q);
        x[k] = U + V_;
        x[k + half] = U - V_ + q2;
      }
    }
  }
};

template <int LOGN2, bool W8 = false, bool GINV = false, int LZC = -1>
__device__ __forceinline__ ArF64Row<LOGN2, W8, GINV, LZC> row_policy(const ArF64 &a, const uint64_t *lds, int64_t rel,
                                                                     const uint64_t *ilds = nullptr)
{
  ArF64Row<LOGN2, W8, GINV, LZC> r;
  static_cast<ArF64 &>(r) = a;
  if constexpr (LZC >= 0)
    r.lz = LZC != 0;  // (the base class's global-table passes see the constant)
  r.rt = RowTw<LOGN2>{lds, rel};
  r.itl = ilds;
  return r;
}

template <int LOGN2, bool W8 = false, bool GINV = false>
__device__ __forceinline__ ArIntRow<LOGN2> row_policy(const ArInt &a, const uint64_t *lds, int64_t rel,
                                                      const uint64_t * = nullptr)
{
  static_assert(!W8, "integer twiddles need their Shoup companions");
  ArIntRow<LOGN2> r;
  static_cast<ArInt &>(r) = a;
  r.rt = RowTw<LOGN2>{lds, rel};
  return r;
}

// Run f with the arithmetic policy of modulus index m (q = its prime).
template <class F>
__device__ __forceinline__ void with_arith(uint64_t q, unsigned m, unsigned logn, const Tw2 &tw, F &&f)
{
  const size_t o = (size_t)m << (logn + 1);
  if (q < F64_QMAX && tw.fwdd)
    f(ArF64{(double)q, 1.0 / (double)q, tw.fwdd + o, tw.invd + o, q < F64_LAZY});
  else
    f(ArInt{q, tw.fwd + o, tw.inv + o});
}

// FP64 basis conversion (fbc_term) where it measured faster than the 128-bit
// integer sums + REDC (same box, per 64-pair chunk at N=2^16, L=8): the INVC
// ks_cols4 (323 vs 388 us) and dn_cols (296 vs 309 us).  The NT = 4 ks_cols4
// (config 5) keeps the integer sums (308 vs 488 us with FP64).  Both forms are
// exact, so the choice never changes a bit.
constexpr bool FBC64_KS_INVC = true, FBC64_DN = true, FBC64_KS_NT4 = false;

// with_arith for kernels instantiated per prime set: ALL_F64 (every modulus
// < 2^51, FP64 tables present) keeps only the FP64 policy in the code.
template <bool ALL_F64, class F>
__device__ __forceinline__ void with_arith_t(uint64_t q, unsigned m, unsigned logn, const Tw2 &tw, F &&f)
{
  if constexpr (ALL_F64) {
    const size_t o = (size_t)m << (logn + 1);
    f(ArF64{(double)q, 1.0 / (double)q, tw.fwdd + o, tw.invd + o, q < F64_LAZY});
  } else {
    with_arith(q, m, logn, tw, f);
  }
}

// The same by arithmetic class: AR 1 every modulus FP64, 2 every one integer
// (the caller launched the slots of one class), 0 chosen per modulus.
template <int AR, class F>
__device__ __forceinline__ void with_arith_ar(uint64_t q, unsigned m, unsigned logn, const Tw2 &tw, F &&f)
{
  if constexpr (AR == 2) {
    const size_t o = (size_t)m << (logn + 1);
    f(ArInt{q, tw.fwd + o, tw.inv + o});
  } else {
    with_arith_t<AR == 1 || AR >= 3>(q, m, logn, tw, f);
  }
}

// Row-tile LDS swizzle: column c of a row lives at c ^ ((c >> 4) & 15).  Round
// B reads 16 consecutive columns per thread at a 16-column lane stride; the
// XOR spreads those lanes over distinct banks (8-way conflict without it).
__device__ __forceinline__ int rswz(int c)
{
  return c ^ ((c >> 4) & 15);
}

// block -> (limb, tile) in prime-major order: all tiles of all limbs that use
// basis slot t run before slot t + 1.
__device__ __forceinline__ void pm_decode(const LimbSet &s, unsigned tiles, unsigned &v, unsigned &tile)
{
  const unsigned groups = s.count / s.per;
  const unsigned b = blockIdx.x;
  const unsigned t = b / (groups * tiles);
  const unsigned rem = b - t * groups * tiles;
  const unsigned grp = rem / tiles;
  tile = rem - grp * tiles;
  v = grp * s.per + t;
}

// Column pass: tile = T rows x C columns (T C = 4096).
template <int LOGT, bool INV, class A>
__device__ __forceinline__ void cols_tile(const A &ar, const uint64_t *x, uint64_t *y, unsigned n2, uint64_t *lds,
                                          uint64_t sw, uint64_t swp)
{
  using V = typename A::V;
  constexpr int T = 1 << LOGT, C = 4096 / T, LEA = LOGT - 4, EA = 1 << LEA, CP = C + 1;
  const int t = threadIdx.x;
  if constexpr (!INV) {
    // round A: rows l + 16 k (distances T/2 .. 16)
#pragma unroll
    for (int it = 0; it < C / 16; it++) {
      const int item = t + 256 * it, c = item % C, l = item / C;
      const unsigned vo = (unsigned)l * n2 + c;  // 32-bit per-thread offset, uniform row bases
      V r[EA];
#pragma unroll
      for (int k = 0; k < EA; k++)
        r[k] = A::load((x + (size_t)(16 * k) * n2)[vo]);
      ar.template fwd<LEA>(r, T, LOGT - 1);
#pragma unroll
      for (int k = 0; k < EA; k++)
        lds[(l + 16 * k) * CP + c] = A::bits(r[k]);
    }
    __syncthreads();
    // round B: rows 16 g + k (distances 8 .. 1)
    const int c = t % C, g = t / C;
    const unsigned vo = (unsigned)(16 * g) * n2 + c;
    V r[16];
#pragma unroll
    for (int k = 0; k < 16; k++)
      r[k] = A::unbits(lds[(16 * g + k) * CP + c]);
    ar.template fwd<4>(r, T + 16 * g, 3);
#pragma unroll
    for (int k = 0; k < 16; k++)
      (y + (size_t)k * n2)[vo] = ar.store_lazy(r[k]);  // the row pass (ntt3_rows) reads it lazily
  } else {
    {
      const int c = t % C, g = t / C;
      const unsigned vo = (unsigned)(16 * g) * n2 + c;
      V r[16];
#pragma unroll
      for (int k = 0; k < 16; k++)
        r[k] = A::load((x + (size_t)k * n2)[vo]);
      ar.template inv<4>(r, T + 16 * g, 0);
#pragma unroll
      for (int k = 0; k < 16; k++)
        lds[(16 * g + k) * CP + c] = A::bits(r[k]);
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < C / 16; it++) {
      const int item = t + 256 * it, c = item % C, l = item / C;
      const unsigned vo = (unsigned)l * n2 + c;
      V r[EA];
#pragma unroll
      for (int k = 0; k < EA; k++)
        r[k] = A::unbits(lds[(l + 16 * k) * CP + c]);
      ar.template inv<LEA>(r, T, 4);
#pragma unroll
      for (int k = 0; k < EA; k++)
        (y + (size_t)(16 * k) * n2)[vo] = ar.mulc(r[k], sw, swp);
    }
  }
}


// ---------------------------------------------------------------------------
// Row pass, 8 elements per thread: tile = R x N2 with R N2 = 2048 (16 KiB of
// LDS, no padding), three register rounds of 3, 3 and LOGN2 - 6 stages.
// Half the registers of the 16-element form, so twice the waves per CU to
// overlap one block's butterflies with another's loads.
//   round A: thread (row, l < TA = N2/8)    elements l + TA k
//   round B: thread (row, m < 8, l' < TA/8) elements m TA + l' + (TA/8) k
//   round C: thread (row, h < TA)           elements 8 h + k (consecutive)
// LDS swizzle (conflict-free for all four access patterns, checked offline):
// column c of row r sits at c ^ ((c >> 3) & (TA - 1)) (^ (r & 1) << 4 for
// N2 = 128).
// ---------------------------------------------------------------------------
// Every exchange of the 8-element row passes stays inside one row, and a
// row belongs to one wave (TA = N2 / 8 threads per row, 64 / TA rows per
// wave), so the row passes synchronise per wave, not per block: LDS
// operations of one wave execute in order, the fences only keep the compiler
// from moving them across the exchange.  Waves of a block never wait for each
// other.
// A wave-uniform pointer pinned to SGPRs where it is used (the split key
// switch's and the NTT row passes' pair / poly streams): the compiler
// otherwise hoists (uniform base + lane offset) out of the stream loop as
// 64-bit VGPR pairs, one per stream, and spills them (each reload's vmcnt(0)
// then also waits out the prefetches in flight).  The pointer must be
// wave-uniform.
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
template <class P>
using gptr = __attribute__((address_space(1))) P *;  // a global-memory pointer
template <bool SQ = true, class P>
__device__ __forceinline__ gptr<P> sgpr_ptr(P *p)
{
  if constexpr (!SQ) {
    return (gptr<P>)p;
  } else {
  // (readfirstlane: an opaque scalar; the cast back to the global address
  // space keeps global_load / global_store, not flat, instructions)
  // (the builtin returns int: each half goes through uint32_t, or the low
  // one would be sign-extended into the high one)
  const uint64_t v = (uint64_t)(uintptr_t)p;
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  const uint64_t s = ((uint64_t)hi << 32) | lo;
  return (gptr<P>)(P *)(uintptr_t)s;
  }
}

__device__ __forceinline__ void wave_sync()
{
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Word i < 8 of this thread in a wave-local coalesced walk over a
// 2048-element row tile: wave w covers elements [512 w, 512 w + 512), which
// are exactly its own rows.
__device__ __forceinline__ int wl_elem(int i)
{
  return (threadIdx.x & ~63) * 8 + (threadIdx.x & 63) + 64 * i;
}

template <int LOGN2>
struct Row8 {
  static constexpr int N2 = 1 << LOGN2, R = 2048 / N2, TA = N2 / 8, TB = TA / 8, EC = 1 << (LOGN2 - 6);
  // LDS layout: one pad word per 8 (row stride RS = 9 N2 / 8).  Column c of
  // a row sits at c + c / 8, so every per-thread element set of rounds A, B, C
  // and of the coalesced transposes is one base plus compile-time offsets
  // (one address VGPR per round, not one per element), and all of them are
  // conflict-free for ds_read_b64 except two-way on 3 banks in round A.
  static constexpr int RS = N2 + N2 / 8, WORDS = R * RS;
  static __device__ __forceinline__ int padc(int c) { return c + (c >> 3); }
  static __device__ __forceinline__ int at(int row, int c) { return row * RS + padc(c); }
  // column c0 + d with (c0 & 7) + (d & 7) < 8: base + constant
  static __device__ __forceinline__ int at2(int row, int c0, int d) { return row * RS + padc(c0) + padc(d); }
  // word wl_elem(i) of local thread th (wave-local coalesced walk)
  static __device__ __forceinline__ int wl(int th, int i)
  {
    const int e0 = (th & ~63) * 8;  // the wave's first element: a row start
    return (e0 >> LOGN2) * RS + ((64 * i) >> LOGN2) * RS + padc(th & 63) + padc((64 * i) & (N2 - 1));
  }
};

// forward row pass of one tile, rounds A..C: round A input in r (the
// thread's A elements), canonical result in out (the thread's C elements)
// forward row pass of one tile leaving the thread's C elements lazy in r
// (|.| < 2q for ArF64, < 4q for ArInt)
template <int LOGN2, class A>
__device__ __forceinline__ void rows8_fwd_raw(typename A::V (&r)[8], uint64_t *lds, const A &ar, uint64_t rowbase0,
                                              const int th = (int)threadIdx.x)
{
  using T = Row8<LOGN2>;
  using V = typename A::V;
  const int row = th / T::TA;
  const uint64_t rb = (rowbase0 + row) << LOGN2;
  {
    const int l = th % T::TA;
    ar.template fwd<3>(r, rb, LOGN2 - 1);
#pragma unroll
    for (int k = 0; k < 8; k++)
      lds[T::at2(row, l, T::TA * k)] = A::bits(r[k]);
  }
  wave_sync();
  {
    const int mb = (th % T::TA) / T::TB, l2 = th % T::TB, c0 = mb * T::TA + l2;
#pragma unroll
    for (int k = 0; k < 8; k++)
      r[k] = A::unbits(lds[T::at2(row, c0, T::TB * k)]);
    ar.template fwd<3>(r, rb + mb * T::TA, LOGN2 - 4);
#pragma unroll
    for (int k = 0; k < 8; k++)
      lds[T::at2(row, c0, T::TB * k)] = A::bits(r[k]);
  }
  wave_sync();
  const int h = th % T::TA;
#pragma unroll
  for (int k = 0; k < 8; k++)
    r[k] = A::unbits(lds[T::at2(row, 8 * h, k)]);
#pragma unroll
  for (int j = 0; j < 8 / T::EC; j++) {
    V g[T::EC];
#pragma unroll
    for (int e = 0; e < T::EC; e++)
      g[e] = r[j * T::EC + e];
    ar.template fwd<LOGN2 - 6>(g, rb + 8 * h + T::EC * j, LOGN2 - 7);
#pragma unroll
    for (int e = 0; e < T::EC; e++)
      r[j * T::EC + e] = g[e];
  }
}

template <int LOGN2, class A>
__device__ __forceinline__ void rows8_fwd(typename A::V (&r)[8], uint64_t (&out)[8], uint64_t *lds, const A &ar,
                                          uint64_t rowbase0, const int th = (int)threadIdx.x)
{
  using T = Row8<LOGN2>;
  using V = typename A::V;
  const int row = th / T::TA;
  const uint64_t rb = (rowbase0 + row) << LOGN2;
  {
    const int l = th % T::TA;
    ar.template fwd<3>(r, rb, LOGN2 - 1);
#pragma unroll
    for (int k = 0; k < 8; k++)
      lds[T::at2(row, l, T::TA * k)] = A::bits(r[k]);
  }
  wave_sync();
  {
    const int mb = (th % T::TA) / T::TB, l2 = th % T::TB, c0 = mb * T::TA + l2;
#pragma unroll
    for (int k = 0; k < 8; k++)
      r[k] = A::unbits(lds[T::at2(row, c0, T::TB * k)]);
    ar.template fwd<3>(r, rb + mb * T::TA, LOGN2 - 4);
#pragma unroll
    for (int k = 0; k < 8; k++)
      lds[T::at2(row, c0, T::TB * k)] = A::bits(r[k]);
  }
  wave_sync();
  const int h = th % T::TA;
#pragma unroll
  for (int k = 0; k < 8; k++)
    r[k] = A::unbits(lds[T::at2(row, 8 * h, k)]);
#pragma unroll
  for (int j = 0; j < 8 / T::EC; j++) {
    V g[T::EC];
#pragma unroll
    for (int e = 0; e < T::EC; e++)
      g[e] = r[j * T::EC + e];
    ar.template fwd<LOGN2 - 6>(g, rb + 8 * h + T::EC * j, LOGN2 - 7);
#pragma unroll
    for (int e = 0; e < T::EC; e++)
      out[j * T::EC + e] = ar.canon(g[e]);
  }
}

// inverse row pass of one tile: input r = thread's C elements (canonical or
// bounded as the policy's inverse allows), result r = thread's A elements
// (lazy; canonicalise with ar.canon)
template <int LOGN2, class A>
__device__ __forceinline__ void rows8_inv(typename A::V (&r)[8], uint64_t *lds, const A &ar, uint64_t rowbase0,
                                          const int th = (int)threadIdx.x)
{
  using T = Row8<LOGN2>;
  using V = typename A::V;
  const int row = th / T::TA;
  const uint64_t rb = (rowbase0 + row) << LOGN2;
  {
    const int h = th % T::TA;
#pragma unroll
    for (int j = 0; j < 8 / T::EC; j++) {
      V g[T::EC];
#pragma unroll
      for (int e = 0; e < T::EC; e++)
        g[e] = r[j * T::EC + e];
      ar.template inv<LOGN2 - 6>(g, rb + 8 * h + T::EC * j, 0);
#pragma unroll
      for (int e = 0; e < T::EC; e++)
        r[j * T::EC + e] = g[e];
    }
#pragma unroll
    for (int k = 0; k < 8; k++)
      lds[T::at2(row, 8 * h, k)] = A::bits(r[k]);
  }
  wave_sync();
  {
    const int mb = (th % T::TA) / T::TB, l2 = th % T::TB, c0 = mb * T::TA + l2;
#pragma unroll
    for (int k = 0; k < 8; k++)
      r[k] = A::unbits(lds[T::at2(row, c0, T::TB * k)]);
    ar.template inv<3>(r, rb + mb * T::TA, LOGN2 - 6);
#pragma unroll
    for (int k = 0; k < 8; k++)
      lds[T::at2(row, c0, T::TB * k)] = A::bits(r[k]);
  }
  wave_sync();
  {
    const int l = th % T::TA;
#pragma unroll
    for (int k = 0; k < 8; k++)
      r[k] = A::unbits(lds[T::at2(row, l, T::TA * k)]);
    ar.template inv<3>(r, rb, LOGN2 - 3);
  }
}

// Inverse row pass of one tile whose words the thread already holds in the
// wave-local coalesced order (raw[i] = word wl_elem(i)).
template <int LOGN2, bool INV, class A>
__device__ __forceinline__ void rows8_tile_raw(const A &ar, const uint64_t (&raw)[8], uint64_t *y, uint64_t *lds,
                                               uint64_t rowbase0)
{
  static_assert(INV, "forward tiles load their own words");
  using T = Row8<LOGN2>;
  using V = typename A::V;
  const int th = threadIdx.x, row = th / T::TA, h = th % T::TA, l = th % T::TA;
#pragma unroll
  for (int i = 0; i < 8; i++)
    lds[T::wl(th, i)] = raw[i];
  wave_sync();
  V r[8];
#pragma unroll
  for (int k = 0; k < 8; k++)
    r[k] = A::load(lds[T::at2(row, 8 * h, k)]);
  wave_sync();
  rows8_inv<LOGN2>(r, lds, ar, rowbase0);
#pragma unroll
  for (int k = 0; k < 8; k++)
    y[(row << LOGN2) + l + T::TA * k] = ar.canon(r[k]);
}

// One row-pass tile from words the thread already holds (w: forward -- the
// row-pass input words (row << LOGN2) + l + TA k, lazy; inverse -- the
// coalesced words wl_elem(i), canonical), output canonical to y in the other
// layout.  th: the thread's index in its 256-thread tile group.
template <int LOGN2, bool INV, class A, class Y>
__device__ __forceinline__ void rows8_tile_words(const A &ar, const uint64_t (&w)[8], Y y, uint64_t *lds,
                                                 uint64_t rowbase0, const int th)
{
  using T = Row8<LOGN2>;
  using V = typename A::V;
  const int row = th / T::TA, h = th % T::TA, l = th % T::TA;
  V r[8];
  if constexpr (!INV) {
#pragma unroll
    for (int k = 0; k < 8; k++)
      r[k] = A::load_lazy(w[k]);
    uint64_t out[8];
    rows8_fwd<LOGN2>(r, out, lds, ar, rowbase0, th);
    wave_sync();
#pragma unroll
    for (int k = 0; k < 8; k++)
      lds[T::at2(row, 8 * h, k)] = out[k];
    wave_sync();
#pragma unroll
    for (int i = 0; i < 8; i++)
      y[(unsigned)((th & ~63) * 8 + (th & 63) + 64 * i)] = lds[T::wl(th, i)];
  } else {
#pragma unroll
    for (int i = 0; i < 8; i++)
      lds[T::wl(th, i)] = w[i];
    wave_sync();
#pragma unroll
    for (int k = 0; k < 8; k++)
      r[k] = A::load(lds[T::at2(row, 8 * h, k)]);
    wave_sync();
    rows8_inv<LOGN2>(r, lds, ar, rowbase0, th);
#pragma unroll
    for (int k = 0; k < 8; k++)
      y[(unsigned)((row << LOGN2) + l + T::TA * k)] = ar.canon(r[k]);
  }
}

template <int LOGN2, bool INV, class A>
__device__ __forceinline__ void rows8_tile(const A &ar, const uint64_t *x, uint64_t *y, uint64_t *lds,
                                           uint64_t rowbase0)
{
  using T = Row8<LOGN2>;
  using V = typename A::V;
  const int th = threadIdx.x, row = th / T::TA;
  V r[8];
  if constexpr (!INV) {
    const int l = th % T::TA;
#pragma unroll
    for (int k = 0; k < 8; k++)
      r[k] = A::load_lazy(x[(row << LOGN2) + l + T::TA * k]);  // written by cols_tile<fwd>
    uint64_t out[8];
    rows8_fwd<LOGN2>(r, out, lds, ar, rowbase0);
    const int h = th % T::TA;
    wave_sync();
#pragma unroll
    for (int k = 0; k < 8; k++)
      lds[T::at2(row, 8 * h, k)] = out[k];
    wave_sync();
#pragma unroll
    for (int i = 0; i < 8; i++)
      y[wl_elem(i)] = lds[T::wl(th, i)];
  } else {
#pragma unroll
    for (int i = 0; i < 8; i++)
      lds[T::wl(th, i)] = x[wl_elem(i)];
    wave_sync();
    const int h = th % T::TA;
#pragma unroll
    for (int k = 0; k < 8; k++)
      r[k] = A::load(lds[T::at2(row, 8 * h, k)]);
    wave_sync();
    rows8_inv<LOGN2>(r, lds, ar, rowbase0);
    const int l = th % T::TA;
#pragma unroll
    for (int k = 0; k < 8; k++)
      y[(row << LOGN2) + l + T::TA * k] = ar.canon(r[k]);
  }
}


// ---------------------------------------------------------------------------
// Whole-limb NTT rounds for n = 2^10 .. 2^12 (one block of n/8 threads per
// limb, radix-8 register rounds; kernels.hip: ntt_small_kernel and the fused
// small-N ModUp / ModDown / decode kernels).
// ---------------------------------------------------------------------------
// The rounds as device functions: the first loads and the last stores are the
// caller's (load(k, i) -> V, store(k, i, V) for element i held in slot k).
// The last inverse round and the first forward round both give thread th the
// elements th + k n/8 (k < 8), so a caller can finish an inverse transform,
// combine per element in registers and start a forward transform on the
// result without an LDS pass (modup_small_kernel, moddown_small_kernel).
template <int LOGN, class A, class LD, class ST>
__device__ __forceinline__ void small_fwd(const A &ar, uint64_t *lds, LD &&load, ST &&store)
{
  using V = typename A::V;
  constexpr int n = 1 << LOGN, FULL = LOGN / 3, REM = LOGN % 3;
  const int th = threadIdx.x;
  V a[8];
#pragma unroll
  for (int r = 0; r < FULL; r++) {
    const int d8 = n >> (3 * r + 3), pos0 = (th / d8) * 8 * d8 + th % d8;
#pragma unroll
    for (int k = 0; k < 8; k++)
      a[k] = r ? A::unbits(lds[pos0 + k * d8]) : load(k, pos0 + k * d8);
    ar.template fwd<3>(a, (uint64_t)n + pos0, LOGN - 3 * r - 1);
    if (r + 1 < FULL || REM) {
#pragma unroll
      for (int k = 0; k < 8; k++)
        lds[pos0 + k * d8] = A::bits(a[k]);
      __syncthreads();
    } else {
#pragma unroll
      for (int k = 0; k < 8; k++)
        store(k, pos0 + k * d8, a[k]);
    }
  }
  if constexpr (REM > 0) {
    // last REM stages (distances 2^(REM-1) .. 1): thread t owns 8
    // consecutive elements = 8 / 2^REM groups
    constexpr int EG = 1 << REM;
#pragma unroll
    for (int k = 0; k < 8; k++)
      a[k] = A::unbits(lds[8 * th + k]);
#pragma unroll
    for (int j = 0; j < 8 / EG; j++) {
      V g[EG];
#pragma unroll
      for (int e = 0; e < EG; e++)
        g[e] = a[j * EG + e];
      ar.template fwd<REM>(g, (uint64_t)n + 8 * th + EG * j, REM - 1);
#pragma unroll
      for (int e = 0; e < EG; e++)
        store(j * EG + e, 8 * th + j * EG + e, g[e]);
    }
  }
}

template <int LOGN, class A, class LD, class ST>
__device__ __forceinline__ void small_inv(const A &ar, uint64_t *lds, LD &&load, ST &&store)
{
  using V = typename A::V;
  constexpr int n = 1 << LOGN, FULL = LOGN / 3, REM = LOGN % 3;
  const int th = threadIdx.x;
  V a[8];
  if constexpr (REM > 0) {
    constexpr int EG = 1 << REM;
#pragma unroll
    for (int k = 0; k < 8; k++)
      a[k] = load(k, 8 * th + k);
#pragma unroll
    for (int j = 0; j < 8 / EG; j++) {
      V g[EG];
#pragma unroll
      for (int e = 0; e < EG; e++)
        g[e] = a[j * EG + e];
      ar.template inv<REM>(g, (uint64_t)n + 8 * th + EG * j, 0);
#pragma unroll
      for (int e = 0; e < EG; e++)
        lds[8 * th + j * EG + e] = A::bits(g[e]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int rr = 0; rr < FULL; rr++) {
    const int r = FULL - 1 - rr;  // smallest distances first
    const int d8 = n >> (3 * r + 3), pos0 = (th / d8) * 8 * d8 + th % d8;
#pragma unroll
    for (int k = 0; k < 8; k++)
      a[k] = (rr || REM) ? A::unbits(lds[pos0 + k * d8]) : load(k, pos0 + k * d8);
    ar.template inv<3>(a, (uint64_t)n + pos0, LOGN - 3 * r - 3);
    if (rr + 1 < FULL) {
      __syncthreads();  // every group of this round has read its inputs
#pragma unroll
      for (int k = 0; k < 8; k++)
        lds[pos0 + k * d8] = A::bits(a[k]);
      __syncthreads();
    } else {
#pragma unroll
      for (int k = 0; k < 8; k++)
        store(k, pos0 + k * d8, a[k]);
    }
  }
}


__device__ __forceinline__ unsigned basis_mod(unsigned t, unsigned lvl, unsigned L)
{
  return t < lvl ? t : L + (t - lvl);
}

// XCD-aware grouping: workgroups are dealt round-robin over the 8 XCDs, so
// blocks b and b + 8 share one XCD's L2.  Map block b to (group g, member i)
// such that the `members` blocks of a group share b % 8 and are dispatched
// close together; groups are padded to a multiple of 8 (extra blocks exit).
// Placement only affects speed, never correctness.
__device__ __forceinline__ bool xcd_group(unsigned members, unsigned ngroups, unsigned &g, unsigned &i)
{
  const unsigned b = blockIdx.x, x = b & 7, s = b >> 3;
  i = s % members;
  g = (s / members) * 8 + x;
  return g < ngroups;
}

static inline unsigned xcd_blocks(unsigned members, unsigned ngroups)
{
  return ((ngroups + 7) / 8) * 8 * members;
}

// The all-FP64 column kernels of the split key switch (cols_f64.hip), used in
// place of ks_cols4_kernel<., 8, true, true> / dn_cols_kernel<., 8, ., true,
// true> for column lengths 2^6, 2^7; -DGPQHE_COLSF=0 builds the old ones
// (same-box A/B).
#ifndef GPQHE_COLSF
#define GPQHE_COLSF 1
#endif
// d2_rows_q_kernel (pair ranges per workgroup, staged twiddles) for the split
// key switch's first pass on FP64 prime sets; -DGPQHE_D2Q=0: d2_rows_kernel
#ifndef GPQHE_D2Q
#define GPQHE_D2Q 1
#endif
struct UpTable;
struct DownTable;
void ks_colsf_launch(int logt, int nt, dim3 grid, const uint64_t *y, size_t y_stride, uint64_t *T1, size_t t1_stride,
                     unsigned lvl, unsigned nm, unsigned ndig, unsigned members, unsigned ngroups, const UpTable &tab,
                     const Tw2 &tw);
void ntt2_colsf_launch(int logt, bool inv, unsigned blocks, const LimbSet &in, const LimbSet &out,
                       const uint64_t *post);
// cols_mixed.hip: the same for prime sets mixing FP64 and wider integer
// moduli (GPQHE_COLSM; replaces ks_cols4_kernel<., 8, true, false> and
// dn_cols_kernel<., 8, ., false, true>)
// (Measured non-levers, removed: more targets than one block's 8 as target
// batches re-running the column INTT, and dn_colsm at T = 256)
#ifndef GPQHE_COLSM
#define GPQHE_COLSM 1
#endif
void ks_colsm_launch(int logt, dim3 grid, const uint64_t *y, size_t y_stride, uint64_t *T1, size_t t1_stride,
                     unsigned lvl, unsigned nm, unsigned ndig, unsigned members, unsigned ngroups, const UpTable &tab,
                     const Tw2 &tw);
void dn_colsm_launch(int logt, dim3 grid, const uint64_t *X, size_t x_pstride, size_t x_off, uint64_t *conv,
                     unsigned lvl, unsigned members, unsigned ngroups, const DownTable &tab, const Tw2 &tw);
void dn_colsf_launch(int logt, dim3 grid, const uint64_t *X, size_t x_pstride, size_t x_off, uint64_t *conv,
                     unsigned lvl, unsigned members, unsigned ngroups, const DownTable &tab, const Tw2 &tw);

// Split key switch, kept / dropped basis slots (ks_split.hip): one launch of
// ksq_kernel for row length 2^logn2 and ndig digits.
// ksc / kps: the folded ModDown factors per basis slot (DownTable).
void ksq_run(unsigned logn2, unsigned ndig, bool allf, bool keep_stage, const uint64_t *T1, const D01Src &d01,
             const uint64_t *evkm, uint64_t *dst, size_t dst_pstride, const uint64_t *conv, const uint64_t *ksc,
             const uint64_t *kps, unsigned count, unsigned lvl, unsigned nm, unsigned t_lo, unsigned t_n);
