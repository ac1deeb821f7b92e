// host_math.cpp - host-side number theory and the CKKS special FFT.
//
// Prime rule: largest prime below 2^bits congruent to 1 mod 2n, distinct from
// those already chosen; psi = h^((q-1)/2n) for the smallest h >= 2 with
// psi^n = -1.  Encode: inverse special FFT over the 4s-th roots with
// rotation group 5^j, coefficients at stride n/(2s), llround(value * scale).
// Decode (centred CRT lift, / scale, forward special FFT) runs on the GPU:
// kernels.hip k_decode.
// These are the definitions of oracle/ckks_oracle.c; the complex arithmetic
// is spelled out in real operations and built with -ffp-contract=off so the
// doubles round identically.
#include "gpqhe_internal.h"

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <map>
#include <memory>

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
// The tables of one slot count, built once: the control loop encodes at one
// size every step, and 4s + 1 cos / sin pairs cost more than its FFT.
static const FftTables &fft_tables(unsigned s)
{
  static std::map<unsigned, std::unique_ptr<FftTables>> cache;
  std::unique_ptr<FftTables> &t = cache[s];
  if (!t)
    t.reset(new FftTables(s));
  return *t;
}

void hm_fft_tables(unsigned s, double *ksi, unsigned *rot)
{
  const FftTables &T = fft_tables(s);
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

static void fft_special_enc(cplx *v, unsigned s)
{
  const FftTables &T = fft_tables(s);
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

void hm_encode_slots(int64_t *v, const double *z, unsigned s, double scale)
{
  if (!s || (s & (s - 1)))
    gpqhe_die("bad slot count %u", s);
  std::vector<cplx> u(s);
  for (unsigned i = 0; i < s; i++)
    u[i] = {z[2 * i], z[2 * i + 1]};
  fft_special_enc(u.data(), s);
  for (unsigned k = 0; k < s; k++) {
    const double re = u[k].re * scale, im = u[k].im * scale;
    if (fabs(re) >= 9.2e18 || fabs(im) >= 9.2e18)
      gpqhe_die("encode overflow (|value * scale| >= 2^63)");
    v[k] = llround(re);
    v[k + s] = llround(im);
  }
}

void hm_encode_coeffs(int64_t *coef, const double *z, unsigned s, unsigned n, double scale)
{
  if (!s || (s & (s - 1)) || s > n / 2)
    gpqhe_die("bad slot count %u", s);
  std::vector<int64_t> v(2 * (size_t)s);
  hm_encode_slots(v.data(), z, s, scale);
  memset(coef, 0, (size_t)n * sizeof(int64_t));
  const unsigned gap = n / (2 * s);
  for (unsigned k = 0; k < 2 * s; k++)
    coef[(size_t)k * gap] = v[k];
}
