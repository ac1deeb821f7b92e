/*
 * ckks_oracle.c - CPU restatement of the GPQHE CKKS engine behind HECTR's
 *                 he_* C API (include/gpqhe.h).
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker and the CPU
 * baseline ("port") for the MI355X product library (libgpqhe.so).  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load it;
 * the product never links, loads or calls it.
 *
 * What it restates.  GPQHE is an empty submodule in the reference
 * (/root/reference/.gitmodules:1-3, unpinned: Makefile:25 tracks branch HEAD,
 * https://github.com/OChicken/GPQHE.git), so its source is absent.  The
 * algorithm is the published full-RNS CKKS scheme (Cheon-Han-Kim-Kim-Song,
 * SAC'18; hybrid key switching, Han-Ki CT-RSA'20; hoisted rotations,
 * Halevi-Shoup CRYPTO'18) restricted to the contract HECTR's call sites
 * impose (reference src/hempc.c:216-274, src/ctr.c:445-618):
 *   hectx_init(logn=12, q=2^109, slots=16, Delta=2^50)   ctr.c:514-518
 *   he_keypair / he_genrk (slots rotation keys)          ctr.c:529,532
 *   he_ecd / he_enc_pk / he_dec / he_dcd                 ctr.c:466-492
 *   he_sub / he_gemv / he_add / he_neg / he_copy_ct / he_moddown
 *                                                        hempc.c:253-266
 *
 * Parity status.  Bit-exactness against GPQHE itself is "parity unpinned"
 * (no GPQHE source, tests or vectors exist in the reference).  This oracle
 * is pinned (a) against an independent Python big-integer model of the
 * NTT / CRT / key-switch identities (tests/ckks_model.py), and (b) end to
 * end against the reference's own committed encrypted run
 * tests/results/cstr-hempc.bin and plaintext run cstr-mpc.bin (written at
 * reference tests/hectr.c:751-756,812-817) through hectr_amd/cstr.py.
 *
 * Every algorithmic choice that affects output bits (prime selection, root
 * choice, NTT ordering, RNG streams, fast basis conversion, rounding in
 * encode, hoisting order in gemv) is defined here and mirrored by the
 * product kernels; arithmetic tricks (Shoup/Barrett/lazy reduction) do not
 * affect bits because every stored residue is canonical in [0, q).
 */
#define _GNU_SOURCE
#include "../include/gpqhe.h"

#include <complex.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef unsigned __int128 u128;

#define MAXMOD 64

static void die(const char *fmt, ...)
{
  va_list ap;
  va_start(ap, fmt);
  fprintf(stderr, "gpqhe-oracle: ");
  vfprintf(stderr, fmt, ap);
  fprintf(stderr, "\n");
  va_end(ap);
  abort();
}

static void *xmalloc(size_t bytes)
{
  void *p = aligned_alloc(64, (bytes + 63) & ~(size_t)63);
  if (!p)
    die("out of memory (%zu bytes)", bytes);
  return p;
}

static void *xcalloc(size_t bytes)
{
  void *p = xmalloc(bytes);
  memset(p, 0, bytes);
  return p;
}

/* ======================================================================== */
/* Modular arithmetic (64-bit words, primes < 2^62).                        */
/* ======================================================================== */
typedef struct {
  uint64_t q;
  uint64_t mu;  /* floor(2^(2k) / q), Barrett */
  unsigned k;   /* bit length of q */
} modulus_t;

static void modulus_init(modulus_t *m, uint64_t q)
{
  m->q = q;
  m->k = 64 - (unsigned)__builtin_clzll(q);
  m->mu = (uint64_t)(((u128)1 << (2 * m->k)) / q);
}

static inline uint64_t add_mod(uint64_t a, uint64_t b, uint64_t q)
{
  uint64_t r = a + b;
  return r >= q ? r - q : r;
}

static inline uint64_t sub_mod(uint64_t a, uint64_t b, uint64_t q)
{
  return a >= b ? a - b : a + q - b;
}

static inline uint64_t neg_mod(uint64_t a, uint64_t q)
{
  return a ? q - a : 0;
}

/* a, b < q: Barrett on the 128-bit product. */
static inline uint64_t mul_mod(const modulus_t *m, uint64_t a, uint64_t b)
{
  u128 z = (u128)a * b;
  uint64_t t = (uint64_t)(z >> (m->k - 1));
  uint64_t est = (uint64_t)(((u128)t * m->mu) >> (m->k + 1));
  uint64_t r = (uint64_t)z - est * m->q;
  while (r >= m->q)
    r -= m->q;
  return r;
}

static inline uint64_t shoup_pre(uint64_t w, uint64_t q)
{
  return (uint64_t)(((u128)w << 64) / q);
}

/* w < q, any a < 2^64. */
static inline uint64_t mul_shoup(uint64_t a, uint64_t w, uint64_t wp, uint64_t q)
{
  uint64_t qh = (uint64_t)(((u128)a * wp) >> 64);
  uint64_t r = a * w - qh * q;
  return r >= q ? r - q : r;
}

static uint64_t pow_mod(uint64_t b, uint64_t e, uint64_t q)
{
  u128 r = 1, x = b % q;
  while (e) {
    if (e & 1)
      r = (r * x) % q;
    x = (x * x) % q;
    e >>= 1;
  }
  return (uint64_t)r;
}

static uint64_t inv_mod(uint64_t a, uint64_t q)
{
  a %= q;
  if (!a)
    die("inverse of 0");
  return pow_mod(a, q - 2, q);
}

static int is_prime64(uint64_t n)
{
  static const uint64_t bases[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
  if (n < 2)
    return 0;
  for (unsigned i = 0; i < 12; i++) {
    if (n % bases[i] == 0)
      return n == bases[i];
  }
  uint64_t d = n - 1;
  unsigned r = 0;
  while (!(d & 1)) {
    d >>= 1;
    r++;
  }
  for (unsigned i = 0; i < 12; i++) {
    uint64_t x = pow_mod(bases[i], d, n);
    if (x == 1 || x == n - 1)
      continue;
    int comp = 1;
    for (unsigned j = 1; j < r; j++) {
      x = (uint64_t)(((u128)x * x) % n);
      if (x == n - 1) {
        comp = 0;
        break;
      }
    }
    if (comp)
      return 0;
  }
  return 1;
}

/* Largest prime p < 2^bits with p = 1 (mod 2n), not already used. */
static uint64_t pick_prime(unsigned bits, uint64_t two_n, const uint64_t *used, unsigned nused)
{
  uint64_t top = (uint64_t)1 << bits;
  uint64_t c = (top / two_n) * two_n + 1;
  while (c >= top)
    c -= two_n;
  for (; c > (top >> 1); c -= two_n) {
    int dup = 0;
    for (unsigned i = 0; i < nused; i++)
      dup |= used[i] == c;
    if (!dup && is_prime64(c))
      return c;
  }
  die("no %u-bit NTT prime for 2n=%llu", bits, (unsigned long long)two_n);
  return 0;
}

/* psi = h^((q-1)/2n) for the smallest h >= 2 with psi^n = -1. */
static uint64_t find_psi(uint64_t q, uint64_t n)
{
  for (uint64_t h = 2;; h++) {
    uint64_t psi = pow_mod(h, (q - 1) / (2 * n), q);
    if (pow_mod(psi, n, q) == q - 1)
      return psi;
  }
}

static unsigned brev(unsigned x, unsigned bits)
{
  unsigned r = 0;
  for (unsigned i = 0; i < bits; i++) {
    r = (r << 1) | (x & 1);
    x >>= 1;
  }
  return r;
}

/* ======================================================================== */
/* ChaCha20 counter-mode RNG and samplers.                                   */
/* ======================================================================== */
#define ROTL32(v, c) (((v) << (c)) | ((v) >> (32 - (c))))
#define QR(a, b, c, d)                                                         \
  a += b; d ^= a; d = ROTL32(d, 16);                                           \
  c += d; b ^= c; b = ROTL32(b, 12);                                           \
  a += b; d ^= a; d = ROTL32(d, 8);                                            \
  c += d; b ^= c; b = ROTL32(b, 7)

/* state: constants | key[8] | counter | 0 | stream_lo | stream_hi */
static void chacha20_block(uint32_t out[16], const uint32_t key[8], uint64_t stream, uint32_t counter)
{
  uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                    key[0], key[1], key[2], key[3], key[4], key[5], key[6], key[7],
                    counter, 0u, (uint32_t)stream, (uint32_t)(stream >> 32)};
  uint32_t x[16];
  memcpy(x, s, sizeof(x));
  for (int i = 0; i < 10; i++) {
    QR(x[0], x[4], x[8], x[12]);
    QR(x[1], x[5], x[9], x[13]);
    QR(x[2], x[6], x[10], x[14]);
    QR(x[3], x[7], x[11], x[15]);
    QR(x[0], x[5], x[10], x[15]);
    QR(x[1], x[6], x[11], x[12]);
    QR(x[2], x[7], x[8], x[13]);
    QR(x[3], x[4], x[9], x[14]);
  }
  for (int i = 0; i < 16; i++)
    out[i] = x[i] + s[i];
}

static inline uint64_t splitmix64_mix(uint64_t z)
{
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

/* ======================================================================== */
/* Context                                                                   */
/* ======================================================================== */
static struct {
  int init;
  unsigned logn, n, L, K, nmod, dnum, alpha, slots;
  double delta;
  uint64_t q[MAXMOD];
  modulus_t mod[MAXMOD];
  uint64_t psi[MAXMOD];
  uint64_t *tw[MAXMOD], *twp[MAXMOD];   /* psi^brev(k) and Shoup companions  */
  uint64_t *itw[MAXMOD], *itwp[MAXMOD]; /* psi^-brev(k) and Shoup companions */
  uint64_t ninv[MAXMOD], ninvp[MAXMOD];
  uint64_t P_mod_q[MAXMOD]; /* [prod special primes] mod q_i */
  uint32_t key[8];
  uint64_t counter;
} C;

static void check_ctx(void)
{
  if (!C.init)
    die("context not initialised (hectx_init)");
}

static void set_seed_words(uint64_t seed)
{
  uint64_t z = seed;
  for (int i = 0; i < 4; i++) {
    z += 0x9E3779B97F4A7C15ull;
    uint64_t x = splitmix64_mix(z);
    C.key[2 * i] = (uint32_t)x;
    C.key[2 * i + 1] = (uint32_t)(x >> 32);
  }
  C.counter = 0;
}

void gpqhe_set_seed(uint64_t seed)
{
  set_seed_words(seed);
}

static uint64_t default_seed(void)
{
  const char *e = getenv("GPQHE_SEED");
  if (e && *e)
    return strtoull(e, NULL, 0);
  uint64_t s = 0;
  FILE *f = fopen("/dev/urandom", "rb");
  if (!f || fread(&s, sizeof(s), 1, f) != 1)
    die("cannot read /dev/urandom");
  fclose(f);
  return s;
}

void hectx_init_params(const gpqhe_params_t *p)
{
  if (C.init)
    hectx_exit();
  if (p->logn < 4 || p->logn > 17)
    die("logn %u out of range", p->logn);
  if (p->nlimbs < 1 || p->nspecial < 1 || p->nlimbs + p->nspecial > MAXMOD)
    die("bad limb counts L=%u K=%u", p->nlimbs, p->nspecial);
  if (p->q0_bits > 61 || p->qi_bits > 61 || p->p_bits > 61 || p->q0_bits < 20 || p->qi_bits < 20 || p->p_bits < 20)
    die("prime sizes must be within [20, 61] bits");
  memset(&C, 0, sizeof(C));
  C.logn = p->logn;
  C.n = 1u << p->logn;
  C.L = p->nlimbs;
  C.K = p->nspecial;
  C.nmod = C.L + C.K;
  C.dnum = p->dnum ? p->dnum : p->nlimbs;
  if (C.dnum > C.L)
    C.dnum = C.L;
  C.alpha = (C.L + C.dnum - 1) / C.dnum;
  C.dnum = (C.L + C.alpha - 1) / C.alpha;
  C.slots = p->slots ? p->slots : C.n / 2;
  if (C.slots & (C.slots - 1) || C.slots > C.n / 2)
    die("slots %u must be a power of two <= n/2", C.slots);
  C.delta = p->delta;
  const uint64_t two_n = 2ull * C.n;
  unsigned nused = 0;
  C.q[nused] = pick_prime(p->q0_bits, two_n, C.q, nused);
  nused++;
  for (unsigned i = 1; i < C.L; i++, nused++)
    C.q[nused] = pick_prime(p->qi_bits, two_n, C.q, nused);
  for (unsigned i = 0; i < C.K; i++, nused++)
    C.q[nused] = pick_prime(p->p_bits, two_n, C.q, nused);
  for (unsigned m = 0; m < C.nmod; m++) {
    const uint64_t q = C.q[m];
    modulus_init(&C.mod[m], q);
    C.psi[m] = find_psi(q, C.n);
    const uint64_t ipsi = inv_mod(C.psi[m], q);
    C.tw[m] = xmalloc(C.n * 8);
    C.twp[m] = xmalloc(C.n * 8);
    C.itw[m] = xmalloc(C.n * 8);
    C.itwp[m] = xmalloc(C.n * 8);
    for (unsigned k = 0; k < C.n; k++) {
      unsigned e = brev(k, C.logn);
      C.tw[m][k] = pow_mod(C.psi[m], e, q);
      C.twp[m][k] = shoup_pre(C.tw[m][k], q);
      C.itw[m][k] = pow_mod(ipsi, e, q);
      C.itwp[m][k] = shoup_pre(C.itw[m][k], q);
    }
    C.ninv[m] = inv_mod(C.n, q);
    C.ninvp[m] = shoup_pre(C.ninv[m], q);
  }
  for (unsigned i = 0; i < C.nmod; i++) {
    uint64_t acc = 1;
    for (unsigned k = 0; k < C.K; k++)
      acc = mul_mod(&C.mod[i], acc, C.q[C.L + k] % C.q[i]);
    C.P_mod_q[i] = acc;
  }
  set_seed_words(p->seed ? p->seed : default_seed());
  C.init = 1;
}

static unsigned env_u(const char *name, unsigned dflt)
{
  const char *e = getenv(name);
  return (e && *e) ? (unsigned)strtoul(e, NULL, 0) : dflt;
}

/* Derivation of the RNS chain from HECTR's (logn, q, slots, Delta). */
void hectx_init(unsigned int logn, MPI q, unsigned int slots, uint64_t Delta)
{
  gpqhe_params_t p;
  memset(&p, 0, sizeof(p));
  unsigned logq = gpqhe_mpi_get_nbits(q) - 1;
  unsigned logd = 63 - (unsigned)__builtin_clzll(Delta);
  p.logn = env_u("GPQHE_LOGN", logn);
  p.slots = slots;
  p.delta = (double)Delta;
  p.qi_bits = logd;
  p.nspecial = 1;
  p.p_bits = 60;
  unsigned L = env_u("GPQHE_NLIMBS", 0);
  if (L) {
    p.nlimbs = L;
    p.q0_bits = 60;
  } else {
    L = 2;
    while (logq > (L - 1) * logd + 61)
      L++;
    p.nlimbs = L;
    p.q0_bits = logq - (L - 1) * logd;
  }
  p.dnum = env_u("GPQHE_DNUM", p.nlimbs);
  p.seed = 0;
  hectx_init_params(&p);
}

void hectx_exit(void)
{
  if (!C.init)
    return;
  for (unsigned m = 0; m < C.nmod; m++) {
    free(C.tw[m]);
    free(C.twp[m]);
    free(C.itw[m]);
    free(C.itwp[m]);
  }
  memset(&C, 0, sizeof(C));
}

void hectx_info(gpqhe_info_t *info)
{
  check_ctx();
  memset(info, 0, sizeof(*info));
  info->logn = C.logn;
  info->n = C.n;
  info->nlimbs = C.L;
  info->nspecial = C.K;
  info->dnum = C.dnum;
  info->alpha = C.alpha;
  info->slots = C.slots;
  info->delta = C.delta;
  for (unsigned m = 0; m < C.nmod; m++) {
    info->primes[m] = C.q[m];
    info->psi[m] = C.psi[m];
  }
}

void gpqhe_set_stream(void *stream)
{
  (void)stream;
}

void gpqhe_set_streams(unsigned int n)
{
  (void)n;
}

void gpqhe_sync(void)
{
}

/* no speculation here: every he_gemv and he_dcd runs as called */
unsigned gpqhe_spec_gemv_taken(void)
{
  return 0;
}

unsigned gpqhe_spec_dcd_taken(void)
{
  return 0;
}

void gpqhe_prof_enable(int on)
{
  (void)on;
}

unsigned gpqhe_prof_collect(gpqhe_kstat_t *out, unsigned max)
{
  (void)out;
  (void)max;
  return 0;
}

/* ======================================================================== */
/* NTT (negacyclic, merged psi; CT forward natural->bit-reversed, GS inverse */
/* bit-reversed->natural).  Output index k holds a(psi^(2 brev(k) + 1)).     */
/* ======================================================================== */
static void ntt_limb(uint64_t *a, unsigned m_idx)
{
  const uint64_t q = C.q[m_idx];
  const uint64_t *w = C.tw[m_idx], *wp = C.twp[m_idx];
  const size_t n = C.n;
  size_t t = n;
  for (size_t m = 1; m < n; m <<= 1) {
    t >>= 1;
    for (size_t i = 0; i < m; i++) {
      const size_t j1 = 2 * i * t;
      const uint64_t S = w[m + i], Sp = wp[m + i];
      for (size_t j = j1; j < j1 + t; j++) {
        uint64_t U = a[j];
        uint64_t V = mul_shoup(a[j + t], S, Sp, q);
        a[j] = add_mod(U, V, q);
        a[j + t] = sub_mod(U, V, q);
      }
    }
  }
}

static void intt_limb(uint64_t *a, unsigned m_idx)
{
  const uint64_t q = C.q[m_idx];
  const uint64_t *w = C.itw[m_idx], *wp = C.itwp[m_idx];
  const size_t n = C.n;
  size_t t = 1;
  for (size_t m = n >> 1; m >= 1; m >>= 1) {
    size_t j1 = 0;
    for (size_t i = 0; i < m; i++) {
      const uint64_t S = w[m + i], Sp = wp[m + i];
      for (size_t j = j1; j < j1 + t; j++) {
        uint64_t U = a[j], V = a[j + t];
        a[j] = add_mod(U, V, q);
        a[j + t] = mul_shoup(sub_mod(U, V, q), S, Sp, q);
      }
      j1 += 2 * t;
    }
    t <<= 1;
  }
  for (size_t j = 0; j < n; j++)
    a[j] = mul_shoup(a[j], C.ninv[m_idx], C.ninvp[m_idx], q);
}

/* NTT-domain automorphism X -> X^g: out[k] = in[perm(k)]. */
static unsigned auto_index(unsigned k, uint64_t g)
{
  const uint64_t two_n = 2ull * C.n;
  uint64_t e = ((2ull * brev(k, C.logn) + 1) * g) % two_n;
  return brev((unsigned)((e - 1) >> 1), C.logn);
}

static uint64_t galois_of_rot(unsigned r)
{
  return pow_mod(5, r, 2ull * C.n);
}

/* ======================================================================== */
/* Multi-precision integer (MPI) handle.                                     */
/* ======================================================================== */
struct gpqhe_mpi {
  unsigned nwords;
  uint64_t w[64];
};

MPI gpqhe_mpi_set_ui(MPI w, unsigned long u)
{
  if (!w)
    w = xcalloc(sizeof(*w));
  memset(w->w, 0, sizeof(w->w));
  w->w[0] = u;
  w->nwords = 1;
  return w;
}

void gpqhe_mpi_lshift(MPI x, MPI a, unsigned int n)
{
  uint64_t src[64], dst[64];
  memcpy(src, a->w, sizeof(src));
  memset(dst, 0, sizeof(dst));
  unsigned ws = n / 64, bs = n % 64;
  for (int i = 63; i >= 0; i--) {
    int s = i - (int)ws;
    if (s < 0)
      continue;
    uint64_t v = src[s] << bs;
    if (bs && s > 0)
      v |= src[s - 1] >> (64 - bs);
    dst[i] = v;
  }
  memcpy(x->w, dst, sizeof(dst));
  x->nwords = 64;
}

void gpqhe_mpi_release(MPI a)
{
  free(a);
}

unsigned gpqhe_mpi_get_nbits(MPI a)
{
  for (int i = 63; i >= 0; i--)
    if (a->w[i])
      return (unsigned)(i * 64 + 64 - __builtin_clzll(a->w[i]));
  return 0;
}

/* ======================================================================== */
/* Objects                                                                   */
/* ======================================================================== */
#define OBJ_WORDS(o) ((size_t)(o)->npoly * (o)->cap * C.n)
#define LIMB(o, p, l) ((o)->data + ((size_t)(p) * (o)->cap + (l)) * C.n)

static void obj_alloc(void *vo, unsigned npoly, unsigned cap)
{
  check_ctx();
  he_ct_t *o = vo;
  memset(o, 0, sizeof(*o));
  o->npoly = npoly;
  o->cap = cap;
  o->data = xcalloc((size_t)npoly * cap * C.n * 8);
}

static void obj_free(void *vo)
{
  he_ct_t *o = vo;
  free(o->data);
  memset(o, 0, sizeof(*o));
}

void he_alloc_pk(he_pk_t *pk) { obj_alloc(pk, 2, C.L); }
void he_free_pk(he_pk_t *pk) { obj_free(pk); }
void he_alloc_sk(poly_mpi_t *sk) { obj_alloc(sk, 1, C.nmod); }
void he_free_sk(poly_mpi_t *sk) { obj_free(sk); }
void he_alloc_ct(he_ct_t *ct) { obj_alloc(ct, 2, C.L); }
void he_free_ct(he_ct_t *ct) { obj_free(ct); }
void he_alloc_pt(he_pt_t *pt) { obj_alloc(pt, 1, C.nmod); }
void he_free_pt(he_pt_t *pt) { obj_free(pt); }

/* evk payload is allocated lazily by the key generator (size depends on
 * dnum); rk[0] stays empty (identity rotation). */
void he_alloc_evk(he_evk_t *evk)
{
  check_ctx();
  memset(evk, 0, sizeof(*evk));
}

void he_free_evk(he_evk_t *evk) { obj_free(evk); }

static unsigned obj_export_limbs(const he_ct_t *o)
{
  return o->nlimbs;
}

size_t he_export(const void *vo, uint64_t *host)
{
  const he_ct_t *o = vo;
  unsigned nl = obj_export_limbs(o);
  size_t w = 0;
  for (unsigned p = 0; p < o->npoly; p++)
    for (unsigned l = 0; l < nl; l++) {
      memcpy(host + w, LIMB(o, p, l), C.n * 8);
      w += C.n;
    }
  return w;
}

void he_import(void *vo, const uint64_t *host, unsigned int nlimbs, double scale, uint32_t flags)
{
  he_ct_t *o = vo;
  if (!o->data) {
    /* evk payloads are allocated lazily: the caller sets galois and dnum */
    const uint32_t g = o->galois, dn = o->dnum;
    if (!dn || dn != C.dnum)
      die("he_import into an unallocated object (evk needs dnum=%u)", C.dnum);
    obj_alloc(o, 2 * dn, C.nmod);
    o->galois = g;
    o->dnum = dn;
  }
  if (nlimbs > o->cap)
    die("he_import: %u limbs > capacity %u", nlimbs, o->cap);
  size_t w = 0;
  for (unsigned p = 0; p < o->npoly; p++)
    for (unsigned l = 0; l < nlimbs; l++) {
      memcpy(LIMB(o, p, l), host + w, C.n * 8);
      w += C.n;
    }
  o->nlimbs = nlimbs;
  o->scale = scale;
  o->flags = flags;
}

void he_evk_meta(const he_evk_t *evk, uint32_t *galois, uint32_t *dnum)
{
  *galois = evk->galois;
  *dnum = evk->dnum;
}

/* ======================================================================== */
/* Sampling (ChaCha20 streams; one fresh stream id per sampled polynomial). */
/* ======================================================================== */
static uint64_t next_stream(void)
{
  return C.counter++;
}

/* ternary: P(0) = 1/2, P(+1) = P(-1) = 1/4 */
static void sample_ternary(int8_t *out, uint64_t stream)
{
  for (unsigned k = 0; k < C.n; k++) {
    uint32_t b[16];
    chacha20_block(b, C.key, stream, k);
    uint32_t r = b[0] & 3u;
    out[k] = (int8_t)(r < 2 ? 0 : (r == 2 ? 1 : -1));
  }
}

/* centered binomial, eta = 21 (sigma = 3.24) */
static void sample_cbd(int8_t *out, uint64_t stream)
{
  for (unsigned k = 0; k < C.n; k++) {
    uint32_t b[16];
    chacha20_block(b, C.key, stream, k);
    out[k] = (int8_t)(__builtin_popcount(b[0] & 0x1FFFFFu) - __builtin_popcount(b[1] & 0x1FFFFFu));
  }
}

/* uniform residues for the moduli mods[0..nm): 128 random bits mod q */
static void sample_uniform(uint64_t *out, const unsigned *mods, unsigned nm, uint64_t stream)
{
  const unsigned nb = (C.nmod + 3) / 4; /* blocks per coefficient */
  for (unsigned t = 0; t < nm; t++) {
    const unsigned m = mods[t];
    const uint64_t q = C.q[m];
    for (unsigned k = 0; k < C.n; k++) {
      uint32_t b[16];
      chacha20_block(b, C.key, stream, k * nb + m / 4);
      const uint32_t *w = b + 4 * (m % 4);
      u128 v = (u128)w[0] | ((u128)w[1] << 32) | ((u128)w[2] << 64) | ((u128)w[3] << 96);
      out[(size_t)t * C.n + k] = (uint64_t)(v % q);
    }
  }
}

static void lift_small(uint64_t *dst, const int8_t *src, unsigned m)
{
  const uint64_t q = C.q[m];
  for (unsigned k = 0; k < C.n; k++)
    dst[k] = src[k] >= 0 ? (uint64_t)src[k] : q - (uint64_t)(-src[k]);
}

/* ======================================================================== */
/* CKKS special FFT (canonical embedding over the 4s-th roots, rotation     */
/* group 5^j).  Decode: z_j = sum_k u_k xi^(k 5^j); encode is its inverse.  */
/* ======================================================================== */
static void fft_tables(unsigned s, double complex **ksi, unsigned **rot)
{
  const unsigned M = 4 * s;
  *ksi = xmalloc((size_t)(M + 1) * sizeof(double complex));
  *rot = xmalloc((size_t)s * sizeof(unsigned));
  for (unsigned k = 0; k <= M; k++) {
    double ang = 2.0 * M_PI * (double)k / (double)M;
    (*ksi)[k] = CMPLX(cos(ang), sin(ang));
  }
  unsigned r = 1;
  for (unsigned j = 0; j < s; j++) {
    (*rot)[j] = r;
    r = (unsigned)((5ull * r) % M);
  }
}

/* explicit (ac - bd, ad + bc): no __muldc3, no contraction -> reproducible */
static inline double complex cmul(double complex a, double complex b)
{
  return CMPLX(creal(a) * creal(b) - cimag(a) * cimag(b), creal(a) * cimag(b) + cimag(a) * creal(b));
}

static void bitrev_perm(double complex *v, unsigned s)
{
  unsigned lb = (unsigned)__builtin_ctz(s);
  for (unsigned i = 0; i < s; i++) {
    unsigned j = brev(i, lb);
    if (i < j) {
      double complex t = v[i];
      v[i] = v[j];
      v[j] = t;
    }
  }
}

static void fft_special_dec(double complex *v, unsigned s)
{
  double complex *ksi;
  unsigned *rot;
  fft_tables(s, &ksi, &rot);
  const unsigned M = 4 * s;
  bitrev_perm(v, s);
  for (unsigned len = 2; len <= s; len <<= 1) {
    const unsigned h = len >> 1, lq = len << 2;
    for (unsigned i = 0; i < s; i += len)
      for (unsigned j = 0; j < h; j++) {
        unsigned idx = (rot[j] % lq) * (M / lq);
        double complex a = v[i + j], b = cmul(v[i + j + h], ksi[idx]);
        v[i + j] = CMPLX(creal(a) + creal(b), cimag(a) + cimag(b));
        v[i + j + h] = CMPLX(creal(a) - creal(b), cimag(a) - cimag(b));
      }
  }
  free(ksi);
  free(rot);
}

static void fft_special_enc(double complex *v, unsigned s)
{
  double complex *ksi;
  unsigned *rot;
  fft_tables(s, &ksi, &rot);
  const unsigned M = 4 * s;
  for (unsigned len = s; len >= 2; len >>= 1) {
    const unsigned h = len >> 1, lq = len << 2;
    for (unsigned i = 0; i < s; i += len)
      for (unsigned j = 0; j < h; j++) {
        unsigned idx = (lq - rot[j] % lq) * (M / lq);
        double complex x = v[i + j], y = v[i + j + h];
        double complex a = CMPLX(creal(x) + creal(y), cimag(x) + cimag(y));
        double complex b = cmul(CMPLX(creal(x) - creal(y), cimag(x) - cimag(y)), ksi[idx]);
        v[i + j] = a;
        v[i + j + h] = b;
      }
  }
  bitrev_perm(v, s);
  for (unsigned i = 0; i < s; i++)
    v[i] = CMPLX(creal(v[i]) / (double)s, cimag(v[i]) / (double)s);
  free(ksi);
  free(rot);
}

/* Encode z[slots] at `scale` into integer coefficients (int64, n of them). */
static void encode_coeffs(int64_t *coef, const double complex *z, unsigned s, double scale)
{
  if (!s || (s & (s - 1)) || s > C.n / 2)
    die("bad slot count %u", s);
  double complex *u = xmalloc((size_t)s * sizeof(double complex));
  memcpy(u, z, (size_t)s * sizeof(double complex));
  fft_special_enc(u, s);
  memset(coef, 0, (size_t)C.n * sizeof(int64_t));
  const unsigned gap = C.n / (2 * s);
  for (unsigned k = 0; k < s; k++) {
    double re = creal(u[k]) * scale, im = cimag(u[k]) * scale;
    if (fabs(re) >= 9.2e18 || fabs(im) >= 9.2e18)
      die("encode overflow (|value * scale| >= 2^63)");
    coef[(size_t)k * gap] = llround(re);
    coef[(size_t)(k + s) * gap] = llround(im);
  }
  free(u);
}

static void lift_i64(uint64_t *dst, const int64_t *src, unsigned m)
{
  const uint64_t q = C.q[m];
  for (unsigned k = 0; k < C.n; k++) {
    int64_t v = src[k];
    dst[k] = v >= 0 ? (uint64_t)v % q : (q - ((uint64_t)(-(v + 1)) % q) - 1) % q;
  }
}

/* ======================================================================== */
/* Polynomial helpers over a "modulus list" (RNS basis at a level).          */
/* ======================================================================== */
/* Basis at level lvl: q_0..q_{lvl-1} followed by the K special primes. */
static unsigned basis_qp(unsigned lvl, unsigned *mods)
{
  for (unsigned t = 0; t < lvl; t++)
    mods[t] = t;
  for (unsigned k = 0; k < C.K; k++)
    mods[lvl + k] = C.L + k;
  return lvl + C.K;
}

/* Fast basis conversion: x (coefficient domain, limbs over `from[0..nf)`)
 * -> residues mod `to` (coefficient domain):
 *   y_i = x_i * [(F/f_i)^-1]_{f_i};  out = sum_i y_i * [F/f_i]_to  (mod to). */
static void fbc(uint64_t *out, unsigned to, const uint64_t *const *x, const unsigned *from, unsigned nf)
{
  const modulus_t *mt = &C.mod[to];
  uint64_t ymul[MAXMOD], ymulp[MAXMOD], cto[MAXMOD];
  for (unsigned i = 0; i < nf; i++) {
    const modulus_t *mi = &C.mod[from[i]];
    uint64_t hat = 1, hat_t = 1;
    for (unsigned j = 0; j < nf; j++) {
      if (j == i)
        continue;
      hat = mul_mod(mi, hat, C.q[from[j]] % mi->q);
      hat_t = mul_mod(mt, hat_t, C.q[from[j]] % mt->q);
    }
    ymul[i] = inv_mod(hat, mi->q);
    ymulp[i] = shoup_pre(ymul[i], mi->q);
    cto[i] = hat_t;
  }
  for (unsigned k = 0; k < C.n; k++) {
    uint64_t acc = 0;
    for (unsigned i = 0; i < nf; i++) {
      uint64_t y = mul_shoup(x[i][k], ymul[i], ymulp[i], C.q[from[i]]);
      acc = add_mod(acc, mul_mod(mt, y % mt->q, cto[i]), mt->q);
    }
    out[k] = acc;
  }
}

/* ModUp of the c1 polynomial at level lvl.
 * c1n: NTT-domain limbs 0..lvl-1 (stride n); c1c: same in coefficient domain.
 * D: output [ndig][lvl+K][n], NTT domain, basis_qp(lvl). */
static unsigned modup(uint64_t *D, const uint64_t *c1n, const uint64_t *c1c, unsigned lvl)
{
  unsigned mods[MAXMOD];
  const unsigned nm = basis_qp(lvl, mods);
  const unsigned ndig = (lvl + C.alpha - 1) / C.alpha;
  const size_t n = C.n;
#pragma omp parallel for collapse(2) schedule(dynamic) if (!omp_in_parallel())
  for (unsigned j = 0; j < ndig; j++)
    for (unsigned t = 0; t < nm; t++) {
      const unsigned lo = j * C.alpha;
      const unsigned hi = lo + C.alpha < lvl ? lo + C.alpha : lvl;
      uint64_t *dst = D + ((size_t)j * nm + t) * n;
      if (t >= lo && t < hi) {
        memcpy(dst, c1n + (size_t)t * n, n * 8);
        continue;
      }
      const uint64_t *x[MAXMOD];
      unsigned from[MAXMOD];
      for (unsigned i = lo; i < hi; i++) {
        x[i - lo] = c1c + (size_t)i * n;
        from[i - lo] = i;
      }
      fbc(dst, mods[t], x, from, hi - lo);
      ntt_limb(dst, mods[t]);
    }
  return ndig;
}

/* Approximate division by the product of the "drop" moduli:
 *   out_t = (X_t - NTT(FBC(INTT(X_drop)))_t) * [Dprod^-1]_t   for t in keep.
 * X: limbs with moduli xm[0..nx) (NTT domain); keep/drop index into X. */
static void moddown(uint64_t *out, const uint64_t *X, const unsigned *xm,
                    const unsigned *keep, unsigned nk, const unsigned *drop, unsigned nd)
{
  const size_t n = C.n;
  uint64_t *xc = xmalloc((size_t)nd * n * 8);
  const uint64_t *xp[MAXMOD];
  unsigned from[MAXMOD];
  for (unsigned d = 0; d < nd; d++) {
    memcpy(xc + (size_t)d * n, X + (size_t)drop[d] * n, n * 8);
    intt_limb(xc + (size_t)d * n, xm[drop[d]]);
    xp[d] = xc + (size_t)d * n;
    from[d] = xm[drop[d]];
  }
#pragma omp parallel for schedule(dynamic) if (!omp_in_parallel())
  for (unsigned t = 0; t < nk; t++) {
    const unsigned m = xm[keep[t]];
    const modulus_t *mm = &C.mod[m];
    uint64_t *conv = xmalloc(n * 8);
    fbc(conv, m, xp, from, nd);
    ntt_limb(conv, m);
    uint64_t dp = 1;
    for (unsigned d = 0; d < nd; d++)
      dp = mul_mod(mm, dp, C.q[from[d]] % mm->q);
    const uint64_t dinv = inv_mod(dp, mm->q), dinvp = shoup_pre(dinv, mm->q);
    const uint64_t *x = X + (size_t)keep[t] * n;
    uint64_t *o = out + (size_t)t * n;
    for (size_t k = 0; k < n; k++)
      o[k] = mul_shoup(sub_mod(x[k], conv[k], mm->q), dinv, dinvp, mm->q);
    free(conv);
  }
  free(xc);
}

/* ======================================================================== */
/* Keys                                                                      */
/* ======================================================================== */
void he_keypair(he_pk_t *pk, poly_mpi_t *sk)
{
  check_ctx();
  const size_t n = C.n;
  int8_t *small = xmalloc(n);
  /* s: ternary, stored over all L+K moduli in NTT form */
  sample_ternary(small, next_stream());
  for (unsigned m = 0; m < C.nmod; m++) {
    lift_small(LIMB(sk, 0, m), small, m);
    ntt_limb(LIMB(sk, 0, m), m);
  }
  sk->nlimbs = C.nmod;
  sk->scale = 0;
  /* pk = (-a s + e, a) mod Q_L */
  unsigned mods[MAXMOD];
  for (unsigned t = 0; t < C.L; t++)
    mods[t] = t;
  sample_uniform(LIMB(pk, 1, 0), mods, C.L, next_stream());
  sample_cbd(small, next_stream());
  for (unsigned m = 0; m < C.L; m++) {
    uint64_t *b = LIMB(pk, 0, m);
    const uint64_t *a = LIMB(pk, 1, m), *s = LIMB(sk, 0, m);
    lift_small(b, small, m);
    ntt_limb(b, m);
    for (size_t k = 0; k < n; k++)
      b[k] = sub_mod(b[k], mul_mod(&C.mod[m], a[k], s[k]), C.q[m]);
  }
  pk->nlimbs = C.L;
  free(small);
}

/* Key switching sigma(s) or s^2 (sprime, NTT over all moduli) -> s. */
static void gen_evk(he_evk_t *evk, const uint64_t *sprime, const poly_mpi_t *sk, uint32_t galois)
{
  const size_t n = C.n;
  if (evk->data)
    obj_free(evk);
  obj_alloc(evk, 2 * C.dnum, C.nmod);
  evk->nlimbs = C.nmod;
  evk->galois = galois;
  evk->dnum = C.dnum;
  unsigned mods[MAXMOD];
  for (unsigned t = 0; t < C.nmod; t++)
    mods[t] = t;
  int8_t *small = xmalloc(n);
  for (unsigned j = 0; j < C.dnum; j++) {
    sample_uniform(LIMB(evk, 2 * j + 1, 0), mods, C.nmod, next_stream());
    sample_cbd(small, next_stream());
    const unsigned lo = j * C.alpha, hi = lo + C.alpha < C.L ? lo + C.alpha : C.L;
    for (unsigned m = 0; m < C.nmod; m++) {
      const modulus_t *mm = &C.mod[m];
      uint64_t *b = LIMB(evk, 2 * j, m);
      const uint64_t *a = LIMB(evk, 2 * j + 1, m), *s = LIMB(sk, 0, m);
      lift_small(b, small, m);
      ntt_limb(b, m);
      for (size_t k = 0; k < n; k++)
        b[k] = sub_mod(b[k], mul_mod(mm, a[k], s[k]), mm->q);
      if (m >= lo && m < hi) {
        const uint64_t *sp = sprime + (size_t)m * n;
        for (size_t k = 0; k < n; k++)
          b[k] = add_mod(b[k], mul_mod(mm, C.P_mod_q[m], sp[k]), mm->q);
      }
    }
  }
  free(small);
}

static void gen_rot_key(he_evk_t *evk, uint64_t g, const poly_mpi_t *sk)
{
  const size_t n = C.n;
  uint64_t *sp = xmalloc((size_t)C.nmod * n * 8);
  for (unsigned m = 0; m < C.nmod; m++) {
    const uint64_t *s = LIMB(sk, 0, m);
    for (unsigned k = 0; k < C.n; k++)
      sp[(size_t)m * n + k] = s[auto_index(k, g)];
  }
  gen_evk(evk, sp, sk, (uint32_t)g);
  free(sp);
}

void he_genrk(he_evk_t rk[], const poly_mpi_t *sk)
{
  check_ctx();
  if (rk[0].data)
    obj_free(&rk[0]);
  rk[0].galois = 1;
  for (unsigned r = 1; r < C.slots; r++)
    gen_rot_key(&rk[r], galois_of_rot(r), sk);
}

void he_genrot(he_evk_t *evk, unsigned int rot, const poly_mpi_t *sk)
{
  check_ctx();
  gen_rot_key(evk, galois_of_rot(rot), sk);
}

void he_genrlk(he_evk_t *rlk, const poly_mpi_t *sk)
{
  check_ctx();
  const size_t n = C.n;
  uint64_t *s2 = xmalloc((size_t)C.nmod * n * 8);
  for (unsigned m = 0; m < C.nmod; m++) {
    const uint64_t *s = LIMB(sk, 0, m);
    for (size_t k = 0; k < n; k++)
      s2[(size_t)m * n + k] = mul_mod(&C.mod[m], s[k], s[k]);
  }
  gen_evk(rlk, s2, sk, 1);
  free(s2);
}

/* ======================================================================== */
/* Encoding / encryption                                                     */
/* ======================================================================== */
static void encode_into(he_pt_t *pt, const gpqhe_complex_t *z, unsigned s, double scale,
                        unsigned nlimbs, int special)
{
  int64_t *coef = xmalloc((size_t)C.n * sizeof(int64_t));
  encode_coeffs(coef, (const double complex *)z, s, scale);
  for (unsigned m = 0; m < nlimbs; m++) {
    lift_i64(LIMB(pt, 0, m), coef, m);
    ntt_limb(LIMB(pt, 0, m), m);
  }
  if (special)
    for (unsigned k = 0; k < C.K; k++) {
      lift_i64(LIMB(pt, 0, C.L + k), coef, C.L + k);
      ntt_limb(LIMB(pt, 0, C.L + k), C.L + k);
    }
  pt->nlimbs = nlimbs;
  pt->scale = scale;
  pt->flags = special ? GPQHE_F_SPECIAL : 0;
  free(coef);
}

void he_ecd_ex(he_pt_t *pt, const gpqhe_complex_t z[], unsigned int slots, double scale, unsigned int nlimbs)
{
  check_ctx();
  if (nlimbs < 1 || nlimbs > C.L)
    die("he_ecd_ex: bad level %u", nlimbs);
  encode_into(pt, z, slots, scale, nlimbs, 0);
}

void he_ecd(he_pt_t *pt, const gpqhe_complex_t z[])
{
  he_ecd_ex(pt, z, C.slots, C.delta, C.L);
}

/* Centered CRT lift of coefficient residues (Garner), as double. */
static double crt_center(const uint64_t *res, unsigned nl)
{
  if (nl == 1) {
    uint64_t v = res[0], q = C.q[0];
    return v > q / 2 ? -(double)(q - v) : (double)v;
  }
  uint64_t v[MAXMOD];
  for (unsigned i = 0; i < nl; i++) {
    const modulus_t *mi = &C.mod[i];
    uint64_t t = res[i];
    for (unsigned j = 0; j < i; j++) {
      t = sub_mod(t, v[j] % mi->q, mi->q);
      t = mul_mod(mi, t, inv_mod(C.q[j] % mi->q, mi->q));
    }
    v[i] = t;
  }
  /* value = v0 + q0 (v1 + q1 (v2 + ...)) as a little-endian word array */
  uint64_t val[MAXMOD + 1], Q[MAXMOD + 1];
  memset(val, 0, sizeof(val));
  memset(Q, 0, sizeof(Q));
  val[0] = v[nl - 1];
  Q[0] = 1;
  for (int i = (int)nl - 2; i >= 0; i--) {
    u128 carry = v[i];
    for (unsigned w = 0; w <= nl; w++) {
      u128 x = (u128)val[w] * C.q[i] + carry;
      val[w] = (uint64_t)x;
      carry = x >> 64;
    }
  }
  for (unsigned i = 0; i < nl; i++) {
    u128 carry = 0;
    for (unsigned w = 0; w <= nl; w++) {
      u128 x = (u128)Q[w] * C.q[i] + carry;
      Q[w] = (uint64_t)x;
      carry = x >> 64;
    }
  }
  /* negative iff 2*val > Q */
  int neg = 0;
  {
    uint64_t twice[MAXMOD + 1];
    uint64_t c = 0;
    for (unsigned w = 0; w <= nl; w++) {
      twice[w] = (val[w] << 1) | c;
      c = val[w] >> 63;
    }
    for (int w = (int)nl; w >= 0; w--) {
      if (twice[w] != Q[w]) {
        neg = twice[w] > Q[w];
        break;
      }
    }
  }
  if (neg) {
    uint64_t b = 0;
    for (unsigned w = 0; w <= nl; w++) {
      u128 x = (u128)Q[w] - val[w] - b;
      val[w] = (uint64_t)x;
      b = (uint64_t)(x >> 64) & 1;
    }
  }
  double d = 0;
  for (int w = (int)nl; w >= 0; w--)
    d = d * 18446744073709551616.0 + (double)val[w];
  return neg ? -d : d;
}

void he_dcd_ex(gpqhe_complex_t z[], const he_pt_t *pt, unsigned int slots)
{
  check_ctx();
  const unsigned s = slots, nl = pt->nlimbs;
  const size_t n = C.n;
  if (!s || (s & (s - 1)) || s > C.n / 2)
    die("bad slot count %u", s);
  uint64_t *c = xmalloc((size_t)nl * n * 8);
  for (unsigned m = 0; m < nl; m++) {
    memcpy(c + (size_t)m * n, LIMB(pt, 0, m), n * 8);
    if (!(pt->flags & GPQHE_F_COEFF))
      intt_limb(c + (size_t)m * n, m);
  }
  const unsigned gap = C.n / (2 * s);
  double complex *u = xmalloc((size_t)s * sizeof(double complex));
  uint64_t res[MAXMOD];
  for (unsigned k = 0; k < s; k++) {
    for (unsigned m = 0; m < nl; m++)
      res[m] = c[(size_t)m * n + (size_t)k * gap];
    double re = crt_center(res, nl);
    for (unsigned m = 0; m < nl; m++)
      res[m] = c[(size_t)m * n + (size_t)(k + s) * gap];
    double im = crt_center(res, nl);
    u[k] = CMPLX(re / pt->scale, im / pt->scale);
  }
  fft_special_dec(u, s);
  memcpy(z, u, (size_t)s * sizeof(double complex));
  free(u);
  free(c);
}

void he_dcd(gpqhe_complex_t z[], const he_pt_t *pt)
{
  he_dcd_ex(z, pt, C.slots);
}

void he_enc_pk(he_ct_t *ct, const he_pt_t *pt, const he_pk_t *pk)
{
  check_ctx();
  const size_t n = C.n;
  const unsigned lvl = pt->nlimbs;
  int8_t *v = xmalloc(n), *e0 = xmalloc(n), *e1 = xmalloc(n);
  sample_ternary(v, next_stream());
  sample_cbd(e0, next_stream());
  sample_cbd(e1, next_stream());
  uint64_t *tv = xmalloc(n * 8);
  for (unsigned m = 0; m < lvl; m++) {
    const modulus_t *mm = &C.mod[m];
    lift_small(tv, v, m);
    ntt_limb(tv, m);
    uint64_t *c0 = LIMB(ct, 0, m), *c1 = LIMB(ct, 1, m);
    lift_small(c0, e0, m);
    ntt_limb(c0, m);
    lift_small(c1, e1, m);
    ntt_limb(c1, m);
    const uint64_t *p0 = LIMB(pk, 0, m), *p1 = LIMB(pk, 1, m), *mp = LIMB(pt, 0, m);
    for (size_t k = 0; k < n; k++) {
      c0[k] = add_mod(add_mod(c0[k], mul_mod(mm, tv[k], p0[k]), mm->q), mp[k], mm->q);
      c1[k] = add_mod(c1[k], mul_mod(mm, tv[k], p1[k]), mm->q);
    }
  }
  ct->nlimbs = lvl;
  ct->scale = pt->scale;
  ct->flags = 0;
  free(tv);
  free(v);
  free(e0);
  free(e1);
}

void he_enc_sk(he_ct_t *ct, const he_pt_t *pt, const poly_mpi_t *sk)
{
  check_ctx();
  const size_t n = C.n;
  const unsigned lvl = pt->nlimbs;
  unsigned mods[MAXMOD];
  for (unsigned t = 0; t < lvl; t++)
    mods[t] = t;
  sample_uniform(LIMB(ct, 1, 0), mods, lvl, next_stream());
  int8_t *e = xmalloc(n);
  sample_cbd(e, next_stream());
  for (unsigned m = 0; m < lvl; m++) {
    const modulus_t *mm = &C.mod[m];
    uint64_t *c0 = LIMB(ct, 0, m);
    const uint64_t *a = LIMB(ct, 1, m), *s = LIMB(sk, 0, m), *mp = LIMB(pt, 0, m);
    lift_small(c0, e, m);
    ntt_limb(c0, m);
    for (size_t k = 0; k < n; k++)
      c0[k] = add_mod(sub_mod(c0[k], mul_mod(mm, a[k], s[k]), mm->q), mp[k], mm->q);
  }
  ct->nlimbs = lvl;
  ct->scale = pt->scale;
  ct->flags = 0;
  free(e);
}

void he_dec(he_pt_t *pt, const he_ct_t *ct, const poly_mpi_t *sk)
{
  check_ctx();
  const size_t n = C.n;
  for (unsigned m = 0; m < ct->nlimbs; m++) {
    const modulus_t *mm = &C.mod[m];
    const uint64_t *c0 = LIMB(ct, 0, m), *c1 = LIMB(ct, 1, m), *s = LIMB(sk, 0, m);
    uint64_t *o = LIMB(pt, 0, m);
    for (size_t k = 0; k < n; k++)
      o[k] = add_mod(c0[k], mul_mod(mm, c1[k], s[k]), mm->q);
  }
  pt->nlimbs = ct->nlimbs;
  pt->scale = ct->scale;
  pt->flags = 0;
}

/* ======================================================================== */
/* Evaluation                                                                */
/* ======================================================================== */
static void check_scales(const he_ct_t *a, const he_ct_t *b, const char *op)
{
  double r = a->scale / b->scale;
  if (fabs(r - 1.0) > 1e-9)
    die("%s: scale mismatch (%g vs %g)", op, a->scale, b->scale);
}

static unsigned min_u(unsigned a, unsigned b) { return a < b ? a : b; }

static void addsub(he_ct_t *out, const he_ct_t *a, const he_ct_t *b, int sub)
{
  check_ctx();
  check_scales(a, b, sub ? "he_sub" : "he_add");
  const unsigned lvl = min_u(a->nlimbs, b->nlimbs);
  const double scale = a->scale;
  const size_t n = C.n;
  for (unsigned p = 0; p < 2; p++)
    for (unsigned m = 0; m < lvl; m++) {
      const uint64_t q = C.q[m];
      const uint64_t *x = LIMB(a, p, m), *y = LIMB(b, p, m);
      uint64_t *o = LIMB(out, p, m);
      for (size_t k = 0; k < n; k++)
        o[k] = sub ? sub_mod(x[k], y[k], q) : add_mod(x[k], y[k], q);
    }
  out->nlimbs = lvl;
  out->scale = scale;
  out->flags = 0;
}

void he_add(he_ct_t *out, const he_ct_t *a, const he_ct_t *b) { addsub(out, a, b, 0); }
void he_sub(he_ct_t *out, const he_ct_t *a, const he_ct_t *b) { addsub(out, a, b, 1); }

void he_neg(he_ct_t *ct)
{
  check_ctx();
  for (unsigned p = 0; p < 2; p++)
    for (unsigned m = 0; m < ct->nlimbs; m++) {
      uint64_t *o = LIMB(ct, p, m);
      for (size_t k = 0; k < C.n; k++)
        o[k] = neg_mod(o[k], C.q[m]);
    }
}

void he_copy_ct(he_ct_t *dst, const he_ct_t *src)
{
  check_ctx();
  if (dst == src)
    return;
  for (unsigned p = 0; p < 2; p++)
    memcpy(LIMB(dst, p, 0), LIMB(src, p, 0), (size_t)src->nlimbs * C.n * 8);
  dst->nlimbs = src->nlimbs;
  dst->scale = src->scale;
  dst->flags = src->flags;
}

void he_moddown(he_ct_t *ct)
{
  check_ctx();
  if (ct->nlimbs < 2)
    die("he_moddown: ciphertext at the lowest level");
  ct->nlimbs--;
}

void he_add_pt(he_ct_t *out, const he_ct_t *a, const he_pt_t *pt)
{
  check_ctx();
  check_scales(a, (const he_ct_t *)pt, "he_add_pt");
  const unsigned lvl = min_u(a->nlimbs, pt->nlimbs);
  for (unsigned m = 0; m < lvl; m++) {
    const uint64_t q = C.q[m];
    const uint64_t *x0 = LIMB(a, 0, m), *x1 = LIMB(a, 1, m), *y = LIMB(pt, 0, m);
    uint64_t *o0 = LIMB(out, 0, m), *o1 = LIMB(out, 1, m);
    for (size_t k = 0; k < C.n; k++) {
      o0[k] = add_mod(x0[k], y[k], q);
      o1[k] = x1[k];
    }
  }
  out->nlimbs = lvl;
  out->scale = a->scale;
  out->flags = 0;
}

void he_mul_pt(he_ct_t *out, const he_ct_t *a, const he_pt_t *pt)
{
  check_ctx();
  const unsigned lvl = min_u(a->nlimbs, pt->nlimbs);
  const double scale = a->scale * pt->scale;
  for (unsigned p = 0; p < 2; p++)
    for (unsigned m = 0; m < lvl; m++) {
      const uint64_t *x = LIMB(a, p, m), *y = LIMB(pt, 0, m);
      uint64_t *o = LIMB(out, p, m);
      for (size_t k = 0; k < C.n; k++)
        o[k] = mul_mod(&C.mod[m], x[k], y[k]);
    }
  out->nlimbs = lvl;
  out->scale = scale;
  out->flags = 0;
}

/* Inner product of the ModUp digits with an evk, optionally through the
 * NTT-domain automorphism g, plus P * sigma_g(c0) into acc0.
 * acc0/acc1: [nm][n] over basis_qp(lvl).  c0 may be NULL. */
static void ks_inner(uint64_t *acc0, uint64_t *acc1, const uint64_t *D, unsigned ndig, unsigned lvl,
                     const he_evk_t *evk, uint64_t g, const uint64_t *c0, int accumulate_pt,
                     const uint64_t *pt)
{
  unsigned mods[MAXMOD];
  const unsigned nm = basis_qp(lvl, mods);
  const size_t n = C.n;
  if (evk && evk->dnum != C.dnum)
    die("evk dnum %u != context dnum %u", evk->dnum, C.dnum);
  unsigned *perm = NULL;
  if (g != 1) {
    perm = xmalloc(n * sizeof(unsigned));
    for (unsigned k = 0; k < C.n; k++)
      perm[k] = auto_index(k, g);
  }
#pragma omp parallel for schedule(dynamic) if (!omp_in_parallel())
  for (unsigned t = 0; t < nm; t++) {
    const unsigned m = mods[t];
    const modulus_t *mm = &C.mod[m];
    const uint64_t q = mm->q;
    uint64_t *o0 = acc0 + (size_t)t * n, *o1 = acc1 + (size_t)t * n;
    for (size_t k = 0; k < n; k++) {
      const size_t src = perm ? perm[k] : k;
      uint64_t s0 = 0, s1 = 0;
      for (unsigned j = 0; j < ndig; j++) {
        const uint64_t d = D[((size_t)j * nm + t) * n + src];
        s0 = add_mod(s0, mul_mod(mm, d, LIMB(evk, 2 * j, m)[k]), q);
        s1 = add_mod(s1, mul_mod(mm, d, LIMB(evk, 2 * j + 1, m)[k]), q);
      }
      if (c0 && t < lvl)
        s0 = add_mod(s0, mul_mod(mm, C.P_mod_q[m], c0[(size_t)t * n + src]), q);
      if (accumulate_pt) {
        const uint64_t w = pt[(size_t)t * n + k];
        o0[k] = add_mod(o0[k], mul_mod(mm, w, s0), q);
        o1[k] = add_mod(o1[k], mul_mod(mm, w, s1), q);
      } else {
        o0[k] = s0;
        o1[k] = s1;
      }
    }
  }
  free(perm);
}

/* Divide (acc0, acc1) over basis_qp(lvl) by P (drop_top = 0) or by
 * P * q_{lvl-1} (drop_top = 1); write into ct limbs 0.. */
static void ks_finish(he_ct_t *out, const uint64_t *acc0, const uint64_t *acc1, unsigned lvl, int drop_top)
{
  unsigned mods[MAXMOD], keep[MAXMOD], drop[MAXMOD];
  const unsigned nm = basis_qp(lvl, mods);
  unsigned nk = 0, nd = 0;
  for (unsigned t = 0; t < nm; t++) {
    if (t >= lvl || (drop_top && t == lvl - 1))
      drop[nd++] = t;
    else
      keep[nk++] = t;
  }
  const size_t n = C.n;
  uint64_t *o = xmalloc((size_t)nk * n * 8);
  moddown(o, acc0, mods, keep, nk, drop, nd);
  memcpy(LIMB(out, 0, 0), o, (size_t)nk * n * 8);
  moddown(o, acc1, mods, keep, nk, drop, nd);
  memcpy(LIMB(out, 1, 0), o, (size_t)nk * n * 8);
  free(o);
  out->nlimbs = nk;
  out->flags = 0;
}

/* Tensor + relinearize [+ rescale]. */
static void mul_core(he_ct_t *out, const he_ct_t *a, const he_ct_t *b, const he_evk_t *rlk, int rescale)
{
  const unsigned lvl = min_u(a->nlimbs, b->nlimbs);
  if (rescale && lvl < 2)
    die("he_mul_rescale: no level left to rescale");
  const size_t n = C.n;
  const double scale = a->scale * b->scale;
  unsigned mods[MAXMOD];
  const unsigned nm = basis_qp(lvl, mods);
  uint64_t *d01 = xmalloc((size_t)2 * lvl * n * 8); /* d0 | d1 */
  uint64_t *d2n = xmalloc((size_t)lvl * n * 8), *d2c = xmalloc((size_t)lvl * n * 8);
  for (unsigned m = 0; m < lvl; m++) {
    const modulus_t *mm = &C.mod[m];
    const uint64_t *a0 = LIMB(a, 0, m), *a1 = LIMB(a, 1, m), *b0 = LIMB(b, 0, m), *b1 = LIMB(b, 1, m);
    uint64_t *d0 = d01 + (size_t)m * n, *d1 = d01 + (size_t)(lvl + m) * n, *d2 = d2n + (size_t)m * n;
    for (size_t k = 0; k < n; k++) {
      d0[k] = mul_mod(mm, a0[k], b0[k]);
      d1[k] = add_mod(mul_mod(mm, a0[k], b1[k]), mul_mod(mm, a1[k], b0[k]), mm->q);
      d2[k] = mul_mod(mm, a1[k], b1[k]);
    }
    memcpy(d2c + (size_t)m * n, d2, n * 8);
    intt_limb(d2c + (size_t)m * n, m);
  }
  const unsigned ndig = (lvl + C.alpha - 1) / C.alpha;
  uint64_t *D = xmalloc((size_t)ndig * nm * n * 8);
  modup(D, d2n, d2c, lvl);
  uint64_t *acc0 = xmalloc((size_t)nm * n * 8), *acc1 = xmalloc((size_t)nm * n * 8);
  ks_inner(acc0, acc1, D, ndig, lvl, rlk, 1, d01, 0, NULL);
  /* add P * d1 to acc1 (acc0 got P * d0 through the c0 argument) */
  for (unsigned t = 0; t < lvl; t++) {
    const modulus_t *mm = &C.mod[t];
    const uint64_t *d1 = d01 + (size_t)(lvl + t) * n;
    uint64_t *o = acc1 + (size_t)t * n;
    for (size_t k = 0; k < n; k++)
      o[k] = add_mod(o[k], mul_mod(mm, C.P_mod_q[t], d1[k]), mm->q);
  }
  ks_finish(out, acc0, acc1, lvl, rescale);
  out->scale = rescale ? scale / (double)C.q[lvl - 1] : scale;
  free(acc0);
  free(acc1);
  free(D);
  free(d01);
  free(d2n);
  free(d2c);
}

void he_mul(he_ct_t *out, const he_ct_t *a, const he_ct_t *b, const he_evk_t *rlk)
{
  check_ctx();
  mul_core(out, a, b, rlk, 0);
}

void he_mul_rescale(he_ct_t *out, const he_ct_t *a, const he_ct_t *b, const he_evk_t *rlk)
{
  check_ctx();
  mul_core(out, a, b, rlk, 1);
}

void he_rescale(he_ct_t *ct)
{
  check_ctx();
  const unsigned lvl = ct->nlimbs;
  if (lvl < 2)
    die("he_rescale: ciphertext at the lowest level");
  const size_t n = C.n;
  unsigned mods[MAXMOD], keep[MAXMOD], drop[1] = {lvl - 1};
  for (unsigned t = 0; t < lvl; t++)
    mods[t] = keep[t] = t;
  uint64_t *o = xmalloc((size_t)(lvl - 1) * n * 8);
  for (unsigned p = 0; p < 2; p++) {
    moddown(o, LIMB(ct, p, 0), mods, keep, lvl - 1, drop, 1);
    memcpy(LIMB(ct, p, 0), o, (size_t)(lvl - 1) * n * 8);
  }
  free(o);
  ct->scale /= (double)C.q[lvl - 1];
  ct->nlimbs = lvl - 1;
}

static const he_evk_t *find_rot_key(const he_evk_t rk[], unsigned r, uint64_t g)
{
  const he_evk_t *k = &rk[r];
  if (!k->data || k->galois != (uint32_t)g)
    die("rotation key for r=%u (galois %llu) missing", r, (unsigned long long)g);
  return k;
}

void he_rot(he_ct_t *out, const he_ct_t *in, unsigned int rot, const he_evk_t rk[])
{
  check_ctx();
  const unsigned lvl = in->nlimbs;
  const size_t n = C.n;
  rot %= C.slots;
  if (!rot) {
    he_copy_ct(out, in);
    return;
  }
  const uint64_t g = galois_of_rot(rot);
  const he_evk_t *k = find_rot_key(rk, rot, g);
  unsigned mods[MAXMOD];
  const unsigned nm = basis_qp(lvl, mods);
  uint64_t *c1c = xmalloc((size_t)lvl * n * 8);
  for (unsigned m = 0; m < lvl; m++) {
    memcpy(c1c + (size_t)m * n, LIMB(in, 1, m), n * 8);
    intt_limb(c1c + (size_t)m * n, m);
  }
  const unsigned ndig = (lvl + C.alpha - 1) / C.alpha;
  uint64_t *D = xmalloc((size_t)ndig * nm * n * 8);
  modup(D, LIMB(in, 1, 0), c1c, lvl);
  uint64_t *acc0 = xmalloc((size_t)nm * n * 8), *acc1 = xmalloc((size_t)nm * n * 8);
  ks_inner(acc0, acc1, D, ndig, lvl, k, g, LIMB(in, 0, 0), 0, NULL);
  const double scale = in->scale;
  ks_finish(out, acc0, acc1, lvl, 0);
  out->scale = scale;
  free(acc0);
  free(acc1);
  free(D);
  free(c1c);
}

/* y = M x, diagonal method (Halevi-Shoup) with hoisted ModUp and a single
 * ModDown-and-rescale by P * q_{lvl-1} at the end.  Diagonal d is encoded at
 * scale q_{lvl-1} over the QP basis so that y keeps x's scale exactly. */
/* The non-zero diagonals of M (diagonal d: M[i][(i + d) mod s]), encoded at
 * scale q_{lvl-1} over basis_qp(lvl) in NTT form: *pt [cnt][nm][n], rot[e]
 * the rotation of the e-th one (ascending).  Returns cnt. */
static unsigned gemv_diags(uint64_t **pt, unsigned *rot, const gpqhe_complex_t M[], unsigned lvl)
{
  const unsigned s = C.slots;
  const size_t n = C.n;
  unsigned mods[MAXMOD];
  const unsigned nm = basis_qp(lvl, mods);
  const double complex *Mz = (const double complex *)M;
  int64_t *coef = xmalloc(n * sizeof(int64_t));
  double complex *diag = xmalloc((size_t)s * sizeof(double complex));
  uint64_t *all = xmalloc((size_t)s * nm * n * 8);
  const double qtop = (double)C.q[lvl - 1];
  unsigned cnt = 0;
  for (unsigned d = 0; d < s; d++) {
    int nz = 0;
    for (unsigned i = 0; i < s; i++) {
      diag[i] = Mz[(size_t)i * s + (i + d) % s];
      nz |= creal(diag[i]) != 0.0 || cimag(diag[i]) != 0.0;
    }
    if (!nz)
      continue;
    encode_coeffs(coef, diag, s, qtop);
    uint64_t *ptl = all + (size_t)cnt * nm * n;
    for (unsigned t = 0; t < nm; t++) {
      lift_i64(ptl + (size_t)t * n, coef, mods[t]);
      ntt_limb(ptl + (size_t)t * n, mods[t]);
    }
    rot[cnt++] = d;
  }
  free(diag);
  free(coef);
  *pt = all;
  return cnt;
}

/* y = sum over the encoded diagonals e of pt_e * rot_{rot[e]}(x): one hoisted
 * ModUp of x, the inner products in the extended basis, one ModDown by
 * P q_{lvl-1}. */
static void gemv_apply(he_ct_t *y, const he_ct_t *x, const he_evk_t rk[], const uint64_t *pts,
                       const unsigned *rot, unsigned cnt)
{
  const unsigned lvl = x->nlimbs;
  const size_t n = C.n;
  unsigned mods[MAXMOD];
  const unsigned nm = basis_qp(lvl, mods);
  uint64_t *c1c = xmalloc((size_t)lvl * n * 8);
  for (unsigned m = 0; m < lvl; m++) {
    memcpy(c1c + (size_t)m * n, LIMB(x, 1, m), n * 8);
    intt_limb(c1c + (size_t)m * n, m);
  }
  const unsigned ndig = (lvl + C.alpha - 1) / C.alpha;
  uint64_t *D = xmalloc((size_t)ndig * nm * n * 8);
  modup(D, LIMB(x, 1, 0), c1c, lvl);
  uint64_t *acc0 = xcalloc((size_t)nm * n * 8), *acc1 = xcalloc((size_t)nm * n * 8);
  for (unsigned e = 0; e < cnt; e++) {
    const unsigned d = rot[e];
    const uint64_t *ptl = pts + (size_t)e * nm * n;
    if (d == 0) {
      /* acc += pt * P * (c0, c1) on the q limbs (P limbs: 0) */
      for (unsigned t = 0; t < lvl; t++) {
        const modulus_t *mm = &C.mod[t];
        const uint64_t *c0 = LIMB(x, 0, t), *c1 = LIMB(x, 1, t), *w = ptl + (size_t)t * n;
        uint64_t *o0 = acc0 + (size_t)t * n, *o1 = acc1 + (size_t)t * n;
        for (size_t k = 0; k < n; k++) {
          uint64_t pw = mul_mod(mm, w[k], C.P_mod_q[t]);
          o0[k] = add_mod(o0[k], mul_mod(mm, pw, c0[k]), mm->q);
          o1[k] = add_mod(o1[k], mul_mod(mm, pw, c1[k]), mm->q);
        }
      }
      continue;
    }
    const uint64_t g = galois_of_rot(d);
    const he_evk_t *k = find_rot_key(rk, d, g);
    ks_inner(acc0, acc1, D, ndig, lvl, k, g, LIMB(x, 0, 0), 1, ptl);
  }
  const double scale = x->scale;
  ks_finish(y, acc0, acc1, lvl, 1);
  y->scale = scale;
  free(acc0);
  free(acc1);
  free(D);
  free(c1c);
}

void he_gemv(he_ct_t *y, const gpqhe_complex_t M[], const he_ct_t *x, const he_evk_t rk[])
{
  check_ctx();
  const unsigned lvl = x->nlimbs;
  if (lvl < 2)
    die("he_gemv: input at the lowest level");
  uint64_t *pts;
  unsigned *rot = xmalloc((size_t)C.slots * sizeof(unsigned));
  const unsigned cnt = gemv_diags(&pts, rot, M, lvl);
  gemv_apply(y, x, rk, pts, rot, cnt);
  free(pts);
  free(rot);
}

/* ======================================================================== */
/* Batched entry points                                                      */
/* ======================================================================== */
static he_ct_t ct_view(const uint64_t *base, unsigned nlimbs)
{
  he_ct_t c = {0};
  c.data = (uint64_t *)base;
  c.nlimbs = c.cap = nlimbs;
  c.npoly = 2;
  c.scale = 1.0;
  return c;
}

/* Independent ciphertexts, one thread each (the per-ciphertext kernels'
 * own parallel loops stay serial inside); the diagonals are encoded once. */
void he_gemv_batch(uint64_t *y, const gpqhe_complex_t M[], const uint64_t *x, size_t count, unsigned int nlimbs,
                   const he_evk_t rk[])
{
  check_ctx();
  if (nlimbs < 2 || nlimbs > C.L)
    die("he_gemv_batch: bad level %u", nlimbs);
  uint64_t *pts;
  unsigned *rot = xmalloc((size_t)C.slots * sizeof(unsigned));
  const unsigned cnt = gemv_diags(&pts, rot, M, nlimbs);
  const size_t in_words = (size_t)2 * nlimbs * C.n, out_words = (size_t)2 * (nlimbs - 1) * C.n;
#pragma omp parallel for schedule(dynamic)
  for (size_t i = 0; i < count; i++) {
    he_ct_t cx = ct_view(x + i * in_words, nlimbs), cy = ct_view(y + i * out_words, nlimbs - 1);
    gemv_apply(&cy, &cx, rk, pts, rot, cnt);
  }
  free(pts);
  free(rot);
}

void he_rot_batch(uint64_t *out, const uint64_t *x, size_t count, unsigned int nlimbs, unsigned int rot,
                  const he_evk_t rk[])
{
  check_ctx();
  if (nlimbs < 1 || nlimbs > C.L)
    die("he_rot_batch: bad level %u", nlimbs);
  const size_t words = (size_t)2 * nlimbs * C.n;
#pragma omp parallel for schedule(dynamic)
  for (size_t i = 0; i < count; i++) {
    he_ct_t cx = ct_view(x + i * words, nlimbs), co = ct_view(out + i * words, nlimbs);
    he_rot(&co, &cx, rot, rk);
  }
}
void he_mul_rescale_batch(uint64_t *out, const uint64_t *a, const uint64_t *b,
                          size_t count, unsigned int nlimbs, const he_evk_t *rlk)
{
  check_ctx();
  const size_t in_words = (size_t)2 * nlimbs * C.n, out_words = (size_t)2 * (nlimbs - 1) * C.n;
#pragma omp parallel for schedule(dynamic)
  for (size_t i = 0; i < count; i++) {
    he_ct_t ca = {0}, cb = {0}, co = {0};
    ca.data = (uint64_t *)a + i * in_words;
    ca.nlimbs = ca.cap = nlimbs;
    ca.npoly = 2;
    ca.scale = 1.0;
    cb = ca;
    cb.data = (uint64_t *)b + i * in_words;
    co.data = out + i * out_words;
    co.cap = nlimbs - 1;
    co.npoly = 2;
    mul_core(&co, &ca, &cb, rlk, 1);
  }
}

void poly_ntt_batch(uint64_t *data, size_t npolys, unsigned int nlimbs)
{
  check_ctx();
#pragma omp parallel for collapse(2) schedule(static)
  for (size_t p = 0; p < npolys; p++)
    for (unsigned m = 0; m < nlimbs; m++)
      ntt_limb(data + (p * nlimbs + m) * C.n, m);
}

void poly_intt_batch(uint64_t *data, size_t npolys, unsigned int nlimbs)
{
  check_ctx();
#pragma omp parallel for collapse(2) schedule(static)
  for (size_t p = 0; p < npolys; p++)
    for (unsigned m = 0; m < nlimbs; m++)
      intt_limb(data + (p * nlimbs + m) * C.n, m);
}

/* value(p, limb, k) = splitmix64 output #(p*n + k) of the stream seeded with
 * seed ^ (0x48454354520001 + limb), reduced mod q_limb. */
void poly_fill_uniform(uint64_t *data, size_t npolys, unsigned int nlimbs, uint64_t seed)
{
  check_ctx();
  for (size_t p = 0; p < npolys; p++)
    for (unsigned m = 0; m < nlimbs; m++) {
      const uint64_t base = seed ^ (0x48454354520001ull + m);
      uint64_t *o = data + (p * nlimbs + m) * C.n;
      for (size_t k = 0; k < C.n; k++) {
        uint64_t idx = p * C.n + k;
        o[k] = splitmix64_mix(base + (idx + 1) * 0x9E3779B97F4A7C15ull) % C.q[m];
      }
    }
}
