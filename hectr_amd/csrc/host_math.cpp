// host_math.cpp - host-side number theory and the CKKS special FFT.
//
// Prime rule: largest prime below 2^bits congruent to 1 mod 2n, distinct from
// those already chosen; psi = h^((q-1)/2n) for the smallest h >= 2 with
// psi^n = -1.  Encode: inverse special FFT over the 4s-th roots with
// rotation group 5^j, coefficients at stride n/(2s), llround(value * scale).
// Decode: centred CRT lift (Garner), / scale, forward special FFT.
// These are the definitions of oracle/ckks_oracle.c; the complex arithmetic
// is spelled out in real operations and built with -ffp-contract=off so the
// doubles round identically.
#include "gpqhe_internal.h"

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;

void gpqhe_die(const char *fmt, ...)
{
  va_list ap;
  va_start(ap, fmt);
  fprintf(stderr, "gpqhe: ");
  vfprintf(stderr, fmt, ap);
  fprintf(stderr, "\n");
  va_end(ap);
  abort();
}

uint64_t hm_mul_mod(uint64_t a, uint64_t b, uint64_t q)
{
  return (uint64_t)(((u128)a * b) % q);
}

uint64_t hm_pow_mod(uint64_t b, uint64_t e, uint64_t q)
{
  uint64_t r = 1 % q, x = b % q;
  while (e) {
    if (e & 1)
      r = hm_mul_mod(r, x, q);
    x = hm_mul_mod(x, x, q);
    e >>= 1;
  }
  return r;
}

uint64_t hm_inv_mod(uint64_t a, uint64_t q)
{
  a %= q;
  if (!a)
    gpqhe_die("inverse of 0 mod %llu", (unsigned long long)q);
  return hm_pow_mod(a, q - 2, q);
}

void hm_modconst(ModConst &m, uint64_t q)
{
  memset(&m, 0, sizeof(m));
  m.q = q;
  m.k = 64 - (unsigned)__builtin_clzll(q);
  m.mu = (uint64_t)(((u128)1 << (2 * m.k)) / q);
  uint64_t inv = 1;  // q^-1 mod 2^64 by Newton iteration (q odd)
  for (int i = 0; i < 6; i++)
    inv *= 2 - q * inv;
  m.qneg_inv = (uint64_t)0 - inv;
  m.r64 = (uint64_t)(((u128)1 << 64) % q);
}

static bool is_prime64(uint64_t n)
{
  static const uint64_t bases[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
  if (n < 2)
    return false;
  for (uint64_t p : bases)
    if (n % p == 0)
      return n == p;
  uint64_t d = n - 1;
  unsigned r = 0;
  while (!(d & 1)) {
    d >>= 1;
    r++;
  }
  for (uint64_t a : bases) {
    uint64_t x = hm_pow_mod(a, d, n);
    if (x == 1 || x == n - 1)
      continue;
    bool composite = true;
    for (unsigned j = 1; j < r && composite; j++) {
      x = hm_mul_mod(x, x, n);
      if (x == n - 1)
        composite = false;
    }
    if (composite)
      return false;
  }
  return true;
}

uint64_t hm_pick_prime(unsigned bits, uint64_t two_n, const uint64_t *used, unsigned nused)
{
  const uint64_t top = 1ull << bits;
  uint64_t c = (top / two_n) * two_n + 1;
  while (c >= top)
    c -= two_n;
  for (; c > (top >> 1); c -= two_n) {
    bool dup = false;
    for (unsigned i = 0; i < nused; i++)
      dup |= used[i] == c;
    if (!dup && is_prime64(c))
      return c;
  }
  gpqhe_die("no %u-bit NTT prime for 2n=%llu", bits, (unsigned long long)two_n);
}

uint64_t hm_find_psi(uint64_t q, uint64_t n)
{
  for (uint64_t h = 2;; h++) {
    const uint64_t psi = hm_pow_mod(h, (q - 1) / (2 * n), q);
    if (hm_pow_mod(psi, n, q) == q - 1)
      return psi;
  }
}

unsigned hm_brev(unsigned x, unsigned bits)
{
  unsigned r = 0;
  for (unsigned i = 0; i < bits; i++) {
    r = (r << 1) | (x & 1);
    x >>= 1;
  }
  return r;
}

// ---------------------------------------------------------------------------
// Special FFT
// ---------------------------------------------------------------------------
struct cplx {
  double re, im;
};

static inline cplx cmul(cplx a, cplx b)
{
  return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}

struct FftTables {
  std::vector<cplx> ksi;
  std::vector<unsigned> rot;
  explicit FftTables(unsigned s)
  {
    const unsigned M = 4 * s;
    ksi.resize(M + 1);
    rot.resize(s);
    for (unsigned k = 0; k <= M; k++) {
      const double ang = 2.0 * M_PI * (double)k / (double)M;
      ksi[k] = {cos(ang), sin(ang)};
    }
    unsigned r = 1;
    for (unsigned j = 0; j < s; j++) {
      rot[j] = r;
      r = (unsigned)((5ull * r) % M);
    }
  }
};

// Tables of the special FFT for s slots, for the GPU encoder: ksi[k] =
// exp(2 pi i k / 4s) for k <= 4s as (re, im) pairs, rot[j] = 5^j mod 4s.
void hm_fft_tables(unsigned s, double *ksi, unsigned *rot)
{
  FftTables T(s);
  for (unsigned k = 0; k <= 4 * s; k++) {
    ksi[2 * k] = T.ksi[k].re;
    ksi[2 * k + 1] = T.ksi[k].im;
  }
  for (unsigned j = 0; j < s; j++)
    rot[j] = T.rot[j];
}

static void bitrev_perm(cplx *v, unsigned s)
{
  const unsigned lb = (unsigned)__builtin_ctz(s);
  for (unsigned i = 0; i < s; i++) {
    const unsigned j = hm_brev(i, lb);
    if (i < j) {
      cplx t = v[i];
      v[i] = v[j];
      v[j] = t;
    }
  }
}

static void fft_special_dec(cplx *v, unsigned s)
{
  FftTables T(s);
  const unsigned M = 4 * s;
  bitrev_perm(v, s);
  for (unsigned len = 2; len <= s; len <<= 1) {
    const unsigned h = len >> 1, lq = len << 2;
    for (unsigned i = 0; i < s; i += len)
      for (unsigned j = 0; j < h; j++) {
        const unsigned idx = (T.rot[j] % lq) * (M / lq);
        const cplx a = v[i + j], b = cmul(v[i + j + h], T.ksi[idx]);
        v[i + j] = {a.re + b.re, a.im + b.im};
        v[i + j + h] = {a.re - b.re, a.im - b.im};
      }
  }
}

static void fft_special_enc(cplx *v, unsigned s)
{
  FftTables T(s);
  const unsigned M = 4 * s;
  for (unsigned len = s; len >= 2; len >>= 1) {
    const unsigned h = len >> 1, lq = len << 2;
    for (unsigned i = 0; i < s; i += len)
      for (unsigned j = 0; j < h; j++) {
        const unsigned idx = (lq - T.rot[j] % lq) * (M / lq);
        const cplx x = v[i + j], y = v[i + j + h];
        const cplx a = {x.re + y.re, x.im + y.im};
        const cplx b = cmul({x.re - y.re, x.im - y.im}, T.ksi[idx]);
        v[i + j] = a;
        v[i + j + h] = b;
      }
  }
  bitrev_perm(v, s);
  for (unsigned i = 0; i < s; i++)
    v[i] = {v[i].re / (double)s, v[i].im / (double)s};
}

void hm_encode_coeffs(int64_t *coef, const double *z, unsigned s, unsigned n, double scale)
{
  if (!s || (s & (s - 1)) || s > n / 2)
    gpqhe_die("bad slot count %u", s);
  std::vector<cplx> u(s);
  for (unsigned i = 0; i < s; i++)
    u[i] = {z[2 * i], z[2 * i + 1]};
  fft_special_enc(u.data(), s);
  memset(coef, 0, (size_t)n * sizeof(int64_t));
  const unsigned gap = n / (2 * s);
  for (unsigned k = 0; k < s; k++) {
    const double re = u[k].re * scale, im = u[k].im * scale;
    if (fabs(re) >= 9.2e18 || fabs(im) >= 9.2e18)
      gpqhe_die("encode overflow (|value * scale| >= 2^63)");
    coef[(size_t)k * gap] = llround(re);
    coef[(size_t)(k + s) * gap] = llround(im);
  }
}

// Centred CRT lift of residues over q_0..q_{nl-1} (Garner), as double.
static double crt_center(const uint64_t *res, unsigned nl)
{
  if (nl == 1) {
    const uint64_t v = res[0], q = G.q[0];
    return v > q / 2 ? -(double)(q - v) : (double)v;
  }
  uint64_t v[GPQHE_MAXMOD];
  for (unsigned i = 0; i < nl; i++) {
    const uint64_t qi = G.q[i];
    uint64_t t = res[i];
    for (unsigned j = 0; j < i; j++) {
      const uint64_t vj = v[j] % qi;
      t = t >= vj ? t - vj : t + qi - vj;
      t = hm_mul_mod(t, hm_inv_mod(G.q[j] % qi, qi), qi);
    }
    v[i] = t;
  }
  uint64_t val[GPQHE_MAXMOD + 1], Q[GPQHE_MAXMOD + 1];
  memset(val, 0, sizeof(val));
  memset(Q, 0, sizeof(Q));
  val[0] = v[nl - 1];
  Q[0] = 1;
  for (int i = (int)nl - 2; i >= 0; i--) {
    u128 carry = v[i];
    for (unsigned w = 0; w <= nl; w++) {
      const u128 x = (u128)val[w] * G.q[i] + carry;
      val[w] = (uint64_t)x;
      carry = x >> 64;
    }
  }
  for (unsigned i = 0; i < nl; i++) {
    u128 carry = 0;
    for (unsigned w = 0; w <= nl; w++) {
      const u128 x = (u128)Q[w] * G.q[i] + carry;
      Q[w] = (uint64_t)x;
      carry = x >> 64;
    }
  }
  bool neg = false;
  {
    uint64_t twice[GPQHE_MAXMOD + 1];
    uint64_t c = 0;
    for (unsigned w = 0; w <= nl; w++) {
      twice[w] = (val[w] << 1) | c;
      c = val[w] >> 63;
    }
    for (int w = (int)nl; w >= 0; w--)
      if (twice[w] != Q[w]) {
        neg = twice[w] > Q[w];
        break;
      }
  }
  if (neg) {
    uint64_t b = 0;
    for (unsigned w = 0; w <= nl; w++) {
      const u128 x = (u128)Q[w] - val[w] - b;
      val[w] = (uint64_t)x;
      b = (uint64_t)(x >> 64) & 1;
    }
  }
  double d = 0;
  for (int w = (int)nl; w >= 0; w--)
    d = d * 18446744073709551616.0 + (double)val[w];
  return neg ? -d : d;
}

void hm_decode(double *z, const uint64_t *c, unsigned nl, unsigned s, unsigned n, double scale)
{
  if (!s || (s & (s - 1)) || s > n / 2)
    gpqhe_die("bad slot count %u", s);
  const unsigned gap = n / (2 * s);
  std::vector<cplx> u(s);
  uint64_t res[GPQHE_MAXMOD];
  for (unsigned k = 0; k < s; k++) {
    for (unsigned m = 0; m < nl; m++)
      res[m] = c[(size_t)m * n + (size_t)k * gap];
    const double re = crt_center(res, nl);
    for (unsigned m = 0; m < nl; m++)
      res[m] = c[(size_t)m * n + (size_t)(k + s) * gap];
    const double im = crt_center(res, nl);
    u[k] = {re / scale, im / scale};
  }
  fft_special_dec(u.data(), s);
  for (unsigned i = 0; i < s; i++) {
    z[2 * i] = u[i].re;
    z[2 * i + 1] = u[i].im;
  }
}
