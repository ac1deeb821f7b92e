// gpqhe_internal.h - shared definitions of the MI355X CKKS engine
// (libgpqhe.so): modular arithmetic, RNG, device tables, host context.
//
// Arithmetic contract: every residue stored in HBM is canonical in [0, q).
// Primes are < 2^61, so 64-bit lanes hold [0, 4q) lazily where a kernel
// wants it.  The algorithms (prime/root choice, NTT ordering, basis
// conversion, RNG streams, encode rounding) are the ones the CPU oracle
// (oracle/ckks_oracle.c) defines, so outputs are bit-identical to it.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include <vector>

#include "../../include/gpqhe.h"

#define GPQHE_MAXMOD 64

#define HIP_CHECK(expr)                                                        \
  do {                                                                         \
    hipError_t err_ = (expr);                                                  \
    if (err_ != hipSuccess)                                                    \
      gpqhe_die("HIP error %s at %s:%d: %s", hipGetErrorName(err_), __FILE__, \
                __LINE__, hipGetErrorString(err_));                            \
  } while (0)

[[noreturn]] void gpqhe_die(const char *fmt, ...);

// ---------------------------------------------------------------------------
// Per-modulus constants (device copy in ModTab array).
// ---------------------------------------------------------------------------
struct ModConst {
  uint64_t q;
  uint64_t mu;     // floor(2^(2k) / q), Barrett
  uint32_t k;      // bit length of q
  uint32_t pad;
  uint64_t ninv, ninvp;  // n^-1 and Shoup companion
  uint64_t pmod, pmodp;  // [P]_q (product of the special primes) + Shoup
  uint64_t qneg_inv;     // -q^-1 mod 2^64 (Montgomery REDC)
  uint64_t r64;          // 2^64 mod q
};


// ---------------------------------------------------------------------------
// Modular arithmetic (host + device).
// ---------------------------------------------------------------------------
__host__ __device__ __forceinline__ uint64_t mulhi64(uint64_t a, uint64_t b)
{
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul64hi(a, b);
#else
  return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}

__host__ __device__ __forceinline__ uint64_t add_mod(uint64_t a, uint64_t b, uint64_t q)
{
  uint64_t r = a + b;
  return r >= q ? r - q : r;
}

__host__ __device__ __forceinline__ uint64_t sub_mod(uint64_t a, uint64_t b, uint64_t q)
{
  return a >= b ? a - b : a + q - b;
}

__host__ __device__ __forceinline__ uint64_t neg_mod(uint64_t a, uint64_t q)
{
  return a ? q - a : 0;
}

// Barrett product of a, b < q (k = bitlen(q) <= 61).
__host__ __device__ __forceinline__ uint64_t mul_mod(uint64_t a, uint64_t b, const ModConst &m)
{
  const uint64_t lo = a * b, hi = mulhi64(a, b);
  const uint64_t t = (hi << (65 - m.k)) | (lo >> (m.k - 1));
  const uint64_t plo = t * m.mu, phi = mulhi64(t, m.mu);
  const uint64_t est = (phi << (63 - m.k)) | (plo >> (m.k + 1));
  uint64_t r = lo - est * m.q;
  r = r >= m.q ? r - m.q : r;
  return r >= m.q ? r - m.q : r;
}

// Shoup product: w < q constant with wp = floor(w 2^64 / q); a < 2^64.
__host__ __device__ __forceinline__ uint64_t mul_shoup(uint64_t a, uint64_t w, uint64_t wp, uint64_t q)
{
  const uint64_t qh = mulhi64(a, wp);
  const uint64_t r = a * w - qh * q;
  return r >= q ? r - q : r;
}

// Shoup without the final correction: result in [0, 2q).
__host__ __device__ __forceinline__ uint64_t mul_shoup_lazy(uint64_t a, uint64_t w, uint64_t wp, uint64_t q)
{
  return a * w - mulhi64(a, wp) * q;
}

// Montgomery REDC of a 128-bit (hi:lo) sum v < 8 q 2^61: returns v 2^-64 mod q
// (canonical).  Used with constants pre-multiplied by 2^64 so the result is
// the plain residue.
__host__ __device__ __forceinline__ uint64_t redc128(uint64_t hi, uint64_t lo, const ModConst &m)
{
  const uint64_t mq = lo * m.qneg_inv;
  uint64_t t = hi + mulhi64(mq, m.q) + (lo != 0);
  return t >= m.q ? t - m.q : t;
}

// x mod q for arbitrary 64-bit x (q < 2^61): reduce via Barrett on (0:x).
__host__ __device__ __forceinline__ uint64_t reduce64(uint64_t x, const ModConst &m)
{
  const uint64_t t = x >> (m.k - 1);
  const uint64_t plo = t * m.mu, phi = mulhi64(t, m.mu);
  const uint64_t est = (phi << (63 - m.k)) | (plo >> (m.k + 1));
  uint64_t r = x - est * m.q;
  r = r >= m.q ? r - m.q : r;
  return r >= m.q ? r - m.q : r;
}

// ---------------------------------------------------------------------------
// ChaCha20 block (state: constants | key | counter | 0 | stream lo | hi).
// ---------------------------------------------------------------------------
struct ChachaKey {
  uint32_t k[8];
};

#define GPQHE_ROTL32(v, c) (((v) << (c)) | ((v) >> (32 - (c))))
#define GPQHE_QR(a, b, c, d)                                                   \
  a += b; d ^= a; d = GPQHE_ROTL32(d, 16);                                     \
  c += d; b ^= c; b = GPQHE_ROTL32(b, 12);                                     \
  a += b; d ^= a; d = GPQHE_ROTL32(d, 8);                                      \
  c += d; b ^= c; b = GPQHE_ROTL32(b, 7)

__host__ __device__ __forceinline__ void chacha20_block(uint32_t out[16], const ChachaKey &key,
                                                        uint64_t stream, uint32_t counter)
{
  uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                    key.k[0], key.k[1], key.k[2], key.k[3], key.k[4], key.k[5], key.k[6], key.k[7],
                    counter, 0u, (uint32_t)stream, (uint32_t)(stream >> 32)};
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 16; i++)
    x[i] = s[i];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    GPQHE_QR(x[0], x[4], x[8], x[12]);
    GPQHE_QR(x[1], x[5], x[9], x[13]);
    GPQHE_QR(x[2], x[6], x[10], x[14]);
    GPQHE_QR(x[3], x[7], x[11], x[15]);
    GPQHE_QR(x[0], x[5], x[10], x[15]);
    GPQHE_QR(x[1], x[6], x[11], x[12]);
    GPQHE_QR(x[2], x[7], x[8], x[13]);
    GPQHE_QR(x[3], x[4], x[9], x[14]);
  }
#pragma unroll
  for (int i = 0; i < 16; i++)
    out[i] = x[i] + s[i];
}

__host__ __device__ __forceinline__ uint64_t splitmix64_mix(uint64_t z)
{
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// ---------------------------------------------------------------------------
// Limb sets: `count` limbs, limb v at base + (v / per) * stride + (v % per) * n,
// reduced modulo mods[v % per].  Passed by value to kernels.
// ---------------------------------------------------------------------------
#define GPQHE_MAXGRP 8
struct LimbSet {
  uint64_t *base;
  size_t stride;      // words between groups of `per` limbs
  uint32_t per;
  uint32_t count;
  uint8_t mods[GPQHE_MAXMOD];
  // ngp > 0: group g starts at gp[g] instead (separately allocated objects
  // batched into one launch, g < ngp <= GPQHE_MAXGRP)
  uint64_t *gp[GPQHE_MAXGRP];
  uint32_t ngp;

  __host__ __device__ __forceinline__ uint64_t *limb(uint32_t v, uint32_t logn) const
  {
    if (ngp)
      return gp[v / per] + ((size_t)(v % per) << logn);
    return base + (size_t)(v / per) * stride + ((size_t)(v % per) << logn);
  }
  __host__ __device__ __forceinline__ uint32_t mod(uint32_t v) const { return mods[v % per]; }
};

// ---------------------------------------------------------------------------
// Host context (process-global singleton).
// ---------------------------------------------------------------------------
struct DevTables {
  ModConst *mc;        // [nmod]
  uint64_t *tw, *twp;  // [nmod][n] psi^brev(k) (+ Shoup)
  uint64_t *itw, *itwp;
};

struct Context {
  bool init = false;
  unsigned logn = 0, n = 0, L = 0, K = 0, nmod = 0, dnum = 0, alpha = 0, slots = 0;
  double delta = 0;
  uint64_t q[GPQHE_MAXMOD];
  uint64_t psi[GPQHE_MAXMOD];
  ModConst mc[GPQHE_MAXMOD];
  ChachaKey key;
  uint64_t counter = 0;
  DevTables dev{};
  const uint64_t *tw2 = nullptr, *itw2 = nullptr;  // interleaved (w, w') pairs [nmod][n][2]
  const double *twd = nullptr, *itwd = nullptr;    // interleaved (w, w / q) doubles [nmod][n][2]
  hipStream_t stream = nullptr;
  hipStream_t own_stream = nullptr;
  int device = 0;
};

extern Context G;

// ---------------------------------------------------------------------------
// Host helpers (host_math.cpp)
// ---------------------------------------------------------------------------
uint64_t hm_pow_mod(uint64_t b, uint64_t e, uint64_t q);
uint64_t hm_inv_mod(uint64_t a, uint64_t q);
void hm_modconst(ModConst &m, uint64_t q);
uint64_t hm_mul_mod(uint64_t a, uint64_t b, uint64_t q);
uint64_t hm_pick_prime(unsigned bits, uint64_t two_n, const uint64_t *used, unsigned nused);
uint64_t hm_find_psi(uint64_t q, uint64_t n);
unsigned hm_brev(unsigned x, unsigned bits);
void hm_fft_tables(unsigned s, double *ksi, unsigned *rot);
// GPU encoder: work (device, 2 s + 2 doubles) holds z (s complex values) and
// is overwritten; writes the n signed coefficients of hm_encode_coeffs (same
// operations, same order: bit-identical).  Synchronises (overflow check).
void k_encode_coeffs(int64_t *coef, double *work, unsigned s, double scale);
void hm_encode_coeffs(int64_t *coef, const double *z_interleaved, unsigned s, unsigned n, double scale);
// The 2s non-zero coefficients of that encoding only: v[k] is coefficient
// k n / 2s (the same values, no n-word array).
void hm_encode_slots(int64_t *v, const double *z_interleaved, unsigned s, double scale);
// GPU decoder: z (device, s complex values) <- the centred CRT lift of the
// coefficient limbs coef [nl][n] (device), / scale, forward special FFT --
// bit-identical to the oracle's he_dcd; asynchronous on the engine stream.
// Up to GPQHE_DCD_ONEPASS slots one launch writes each value of z once, so z
// may be mapped pinned host memory.
#define GPQHE_DCD_ONEPASS 2048u
void k_decode(double *z, const uint64_t *coef, unsigned nl, unsigned s, double scale);

// ---------------------------------------------------------------------------
// Device memory pool (stream-ordered reuse on the engine stream).
// ---------------------------------------------------------------------------
void *pool_alloc(size_t bytes);
void pool_free(void *p);
void pool_release_all();

// ---------------------------------------------------------------------------
// Kernel launchers (kernels.hip)
// ---------------------------------------------------------------------------
void k_ntt(const LimbSet &s, bool inverse);
// out of place (in and out of the same geometry; out may equal in); post: per-slot
// Shoup pairs replacing n^-1 (inverse only, n >= 2^13)
void k_ntt_ex(const LimbSet &in, const LimbSet &out, bool inverse, const uint64_t *post);
// The row pass alone of the two-pass transform (n >= 2^13): what
// k_moddown_fused expects of the dropped limbs (inverse), or the second half
// of a forward transform whose column pass ran elsewhere
void k_ntt_rows(const LimbSet &in, const LimbSet &out, bool inverse);
void k_binop(uint64_t *out, const uint64_t *a, const uint64_t *b, unsigned npoly, unsigned lvl,
             size_t out_pstride, size_t a_pstride, size_t b_pstride, int op);
void k_neg(uint64_t *x, unsigned npoly, unsigned lvl, size_t pstride);
// d01 [count][2][lvl][n] (stride d_stride) <- (a0 b0, a0 b1 + a1 b0); d2 [count][lvl][n] <- a1 b1
void k_tensor(uint64_t *d01, uint64_t *d2, const uint64_t *a, const uint64_t *b, unsigned lvl,
              size_t in_stride, size_t in_pstride, unsigned count, size_t d_stride);
void k_dec(uint64_t *pt, const uint64_t *c0, const uint64_t *c1, const uint64_t *s, unsigned lvl);
// Deferred elementwise program (the small-N latency path, api.cpp): queued
// he_add / he_sub / he_neg / he_copy_ct / he_dec polys, applied in queue order
// to every element (limb, k) by one launch.  Op: out = a + b, a - b, -a, a, or
// a + b s (decryption: a = c0, b = c1, s = the secret key), limbs < lvl.
enum { EW_ADD = 0, EW_SUB = 1, EW_NEG = 2, EW_COPY = 3, EW_DEC = 4 };
struct EwOp {
  uint64_t *out;
  const uint64_t *a, *b, *s;
  uint32_t kind, lvl;
};
struct EwProg {
  static constexpr unsigned MAX = 16;
  EwOp op[MAX];
  unsigned count;
};
void k_ew_prog(const EwProg &p);
// k_ew_prog(p), then he_dcd of the NTT-form plaintext pt (nl <= 2 limbs,
// s <= GPQHE_DCD_ONEPASS, n = 2^10 .. 2^12) in one more launch; c: nl n
// words of workspace; z as k_decode's.
void k_ew_decode(const EwProg &p, double *z, const uint64_t *pt, unsigned nl, unsigned s, double scale, uint64_t *c);
// Plaintext coefficients added to the queued encryptions' e0 before their
// transform (NTT(e0 + m) = NTT(e0) + NTT(m) mod q): the combine then needs no
// NTT-form plaintext.  Encryption e of a launch takes row row_of[e] (-1: none),
// n >> clog values per row (value j is coefficient j 2^clog, the others are
// 0), from v (by value) or, when p is set, from device-readable memory.
struct EncCoef {
  static constexpr unsigned MAX = 320;
  int64_t v[MAX];
  const int64_t *p;
  int32_t row_of[GPQHE_MAXGRP];
  uint32_t clog, row;
};
void k_sample_enc(const LimbSet &dst, uint64_t stream, unsigned npoly, const EncCoef *ec = nullptr);
void k_sample_small(const LimbSet &dst, uint64_t stream, int cbd);
void k_sample_uniform(const LimbSet &dst, uint64_t stream);
void k_lift_i64(const LimbSet &dst, const int64_t *coef);
// lift + forward NTT (group g: coef + g (n >> clog); clog > 0: only every
// 2^clog-th coefficient is stored, the others are zero; n <= 2^12)
void k_lift_ntt(const LimbSet &dst, const int64_t *coef, unsigned clog = 0);
// The same with at most CoefArg::MAX coefficients in total (host memory,
// n >> clog per group), passed to the kernel by value (n <= 2^12).
struct CoefArg {
  static constexpr unsigned MAX = 320;
  int64_t v[MAX];
  unsigned clog, row;
};
void k_lift_ntt_arg(const LimbSet &dst, const int64_t *coef_host, unsigned clog);
void k_enc_combine(uint64_t *c0, uint64_t *c1, const uint64_t *v, const uint64_t *e0, const uint64_t *e1,
                   const uint64_t *pk0, const uint64_t *pk1, const uint64_t *m, unsigned lvl);
// up to GPQHE_MAXGRP public-key encryptions in one launch: encryption i takes
// v, e0, e1 from vee + (3 i + {0, 1, 2}) * lvl * n
struct EncBatch {
  uint64_t *c0[GPQHE_MAXGRP], *c1[GPQHE_MAXGRP];
  const uint64_t *m[GPQHE_MAXGRP];  // nullptr: m was added to e0 (EncCoef)
};
void k_enc_combine_batch(const EncBatch &b, unsigned k, const uint64_t *vee, const uint64_t *pk0,
                         const uint64_t *pk1, unsigned lvl);
// The same combine for plaintexts given by coefficients: encryption e with
// row_of[e] >= 0 adds m in NTT form evaluated from its `row` coefficient
// values (value j = coefficient j 2^clog; limb l's values, reduced mod q_l,
// at v + (row_of[e] lvl + l) row); the others add b.m[e] if set.  n <= 2^12,
// row a power of two in [4, MAXROW].
struct EncM {
  static constexpr unsigned MAX = 320, MAXROW = 64;
  uint64_t v[MAX];
  int32_t row_of[GPQHE_MAXGRP];
  uint32_t row, clog;
};
void k_enc_combine_m(const EncBatch &b, const EncM &em, unsigned k, const uint64_t *vee, const uint64_t *pk0,
                     const uint64_t *pk1, unsigned lvl);
// The c1 of the difference of two fresh encryptions without their plaintexts:
// c1(a_i) - c1(b_i), c1(x) = v pk1 + e1 of the sampled noise (v, e0, e1) at
// va[i] / vb[i] (NTT form, lvl limbs each).  k_modup_ntt_diffs: their ModUp,
// each value formed at load (n <= 2^12).
struct C1Diffs {
  const uint64_t *va[GPQHE_MAXGRP], *vb[GPQHE_MAXGRP];
};
void k_modup_ntt_diffs(uint64_t *D, const C1Diffs &cd, unsigned np, size_t d_stride, const uint64_t *pk1,
                       unsigned lvl);
void k_enc_sk_combine(uint64_t *c0, const uint64_t *a, const uint64_t *e, const uint64_t *s, const uint64_t *m,
                      unsigned lvl);
void k_evk_combine(uint64_t *b, const uint64_t *a, const uint64_t *e, const uint64_t *s, const uint64_t *sprime,
                   unsigned lo, unsigned hi);
void k_automorph(uint64_t *out, const uint64_t *in, unsigned nlimbs, uint64_t g);
void k_square(uint64_t *out, const uint64_t *in, unsigned nlimbs);
void k_modup(uint64_t *D, const uint64_t *xc, unsigned count, size_t x_stride, size_t d_stride, unsigned lvl);
struct XPtrs {
  static constexpr unsigned MAX = 8;
  const uint64_t *p[MAX];
};
// The next small-N step's noise carried by this step's kernels (api.cpp
// flush_gemvs; no launches of its own): extra workgroups of
// gemv_inner_kernel sample it (sample), of down_inv_small_kernel run its
// forward transforms (ntt).  Each launcher takes its part and clears the
// flag; the values equal those of the separate launches.
// The next step's speculative ModUp in two halves (ModupHalves): the first,
// per (difference p, input limb i), writes the difference (NTT form) into its
// digit's own slot of D and Y[p][i] = INTT(x_i) [(Q_j/q_i)^-1] (coefficient
// form); the second, per (slot t, digit j, p) outside the digit, the
// conversion sum of Y and the forward transform mod q_t into D.  Together they
// write what modup_small_kernel<., DIFF> writes, value for value.
struct ModupHalves {
  C1Diffs cd{};
  const uint64_t *pk1 = nullptr;
  uint64_t *D = nullptr, *Y = nullptr;  // D [np][ndig][nm][n] (stride d_stride), Y [np][lvl][n]
  size_t d_stride = 0;
  unsigned np = 0, lvl = 0;
};
void k_modup_fwd_diffs(const ModupHalves &mh);  // the second half (n <= 2^12)
struct SpecAttach {
  bool sample = false, ntt = false;
  LimbSet noise{};      // 3k polys x lvl limbs (per = lvl)
  uint64_t stream = 0;  // poly y draws from ChaCha stream stream + y
  unsigned npoly = 0;   // 3k
  // the first ModUp half, as extra workgroups of down_fwd_small_kernel (only
  // in the launch after the one that took ntt: it reads the transformed noise)
  bool modup_inv = false, modup_inv_done = false;
  ModupHalves mh{};
};
extern SpecAttach g_sa;
void k_modup_ntt(uint64_t *D, const XPtrs &x1, unsigned count, size_t d_stride, unsigned lvl);
// acc [count][2][lvl+K][n] (stride acc_stride): acc0 then acc1
// he_gemv diagonals of one launch (passed by value as kernel arguments)
struct GemvDiags {
  static constexpr unsigned MAX = 32;
  const uint64_t *evk[MAX];  // key of the rotation, nullptr for the identity
  const uint64_t *pt[MAX];   // encoded diagonal (over basis_qp(lvl))
  uint64_t g[MAX];           // Galois element (1: identity)
  unsigned count;
};
void k_gemv_inner(uint64_t *acc, const uint64_t *D, const uint64_t *x0, const uint64_t *x1, unsigned lvl,
                  const GemvDiags &dg, bool accumulate);
struct GemvJob {
  uint64_t *acc;
  const uint64_t *D, *x0, *x1;
  GemvDiags dg;
  int accumulate;
  // non-null: the input is x - y, a queued he_sub not yet run (api.cpp
  // he_gemv), formed where the kernel reads it
  const uint64_t *y0 = nullptr, *y1 = nullptr;
};
struct GemvJobs {
  static constexpr unsigned MAX = 2;  // kernel arguments: ~0.8 KB per job
  GemvJob j[MAX];
};
void k_gemv_inner_jobs(const GemvJobs &jobs, unsigned njobs, unsigned lvl);
void k_ks_inner(uint64_t *acc, const uint64_t *D, unsigned count, size_t d_stride, size_t acc_stride,
                const uint64_t *evk, unsigned lvl, uint64_t g, const uint64_t *c0, const uint64_t *c1,
                size_t c_stride, const uint64_t *pt, bool accumulate);
// mode 0: divide by P; 1: by P q_{lvl-1}; 2: by q_{lvl-1} (X over q limbs only)
// out2: the last nx_poly/2 outputs go there instead (see kernels.hip)
void k_moddown(uint64_t *out, size_t out_pstride, uint64_t *X, size_t x_pstride, unsigned nx_poly,
               unsigned lvl, int mode, uint64_t *out2 = nullptr);
void k_fill_uniform(uint64_t *data, size_t npolys, unsigned nlimbs, uint64_t seed);
void k_mul_pt(uint64_t *out, const uint64_t *a, const uint64_t *pt, unsigned lvl, size_t pstride);
void k_add_pt(uint64_t *out, const uint64_t *a, const uint64_t *pt, unsigned lvl, size_t pstride);
bool k_ks_fused_ok();
// The tensor terms d0 = a0 b0 (poly 2 i) and d1 = a0 b1 + a1 b0 (poly 2 i + 1)
// of ciphertext pair i are never materialized: the key switch forms them from
// the input pairs (pair i at a / b + i * in_stride, c1 at + in_pstride; limb t
// word k at (t << logn) + k) and adds P (d0, d1) to its accumulators.
struct D01Src {
  const uint64_t *a, *b;
  size_t in_stride, in_pstride;
};
// d2 = a1 b1 of `count` pairs -> INTT -> ModUp -> key inner product + P (d0,
// d1) into acc [count][2][lvl + K] (NTT domain).  Limbs t >= drop_lo leave after
// the inverse row pass (the input k_moddown_fused expects).  d2 [count][lvl],
// ybuf [count][lvl] and T1 [count][ndig][lvl + K] are workspaces.  Every read
// of a and b happens here, so the ModDown may write over them (in place).
D01Src k_mul_keyswitch_fused(uint64_t *acc, uint64_t *d2, uint64_t *ybuf, uint64_t *T1, const uint64_t *a,
                             const uint64_t *b, size_t in_stride, size_t in_pstride, const uint64_t *evkm,
                             unsigned count, unsigned lvl, unsigned drop_lo);
// Tensor + relinearization [+ rescale] of `count` pairs through the split key
// switch (kernels.hip: ModUp, the dropped slots' inner product, ModDown
// conversion, then the kept slots' inner product with the ModDown epilogue).
// out may equal a or b only with one pair and out_pstride == in_pstride.
bool k_mul_split_ok(unsigned lvl);
// ws: a workspace of k_mul_split_ws_words(count, lvl, rescale) words, or null
// (the pool's, on the engine stream)
size_t k_mul_split_ws_words(unsigned count, unsigned lvl, bool rescale);
// s0, s1: run only stages [s0, s1) (0 d2_rows, 1 ks_cols, 2 ksq<drop>, 3
// dn_cols, 4 ksq<keep>) -- a batch split into sub-chunks on several streams
// issues them in its own order; a stage range needs the caller's ws
void k_mul_relin_split(uint64_t *out, size_t out_pstride, const uint64_t *a, const uint64_t *b, size_t in_stride,
                       size_t in_pstride, const uint64_t *evkm, unsigned count, unsigned lvl, bool rescale,
                       uint64_t *ws = nullptr, int s0 = 0, int s1 = 5);
// ModDown (mode 0: / P, 1: / P q_{lvl-1}) of X whose drop limbs hold the
// inverse row pass of their NTT form (k_mul_keyswitch_fused with drop_lo =
// keep).
// pre: the drop limbs' row pass also applied n^-1 [(D/d)^-1]_d
// (k_ntt_rows_down), so the pre-scaled column kernels run.
// s79 (n = 2^16): the drop limbs' row pass ran on 512-element rows
// (k_ntt_rows_down with s79), so the 128 x 512 tiling follows, as the split
// key switch's; otherwise k_ntt_ex's 256 x 256.
void k_moddown_fused(uint64_t *out, size_t out_pstride, uint64_t *X, size_t x_pstride, unsigned npoly,
                     unsigned lvl, int mode, bool pre = false, bool s79 = false);
bool k_ntt_rows_down(const LimbSet &dr, unsigned lvl, int mode, bool s79 = false);
bool k_prof_on();
void k_prof_release();
// Live kernel statistics (gpqhe_prof_enable): HIP events around one launch
// on the engine stream, per kernel class (names: kernels.hip kc_names).
enum KClass {
  KC_NTT_WHOLE_FWD, KC_NTT_WHOLE_INV, KC_MODUP, KC_KS_INNER, KC_TENSOR, KC_DOWN_CONV, KC_DOWN_COMBINE, KC_KS_COLS,
  KC_KS_ROWS, KC_DN_COLS, KC_DN_ROWS, KC_D2_ROWS, KC_NTT2_COLS_FWD, KC_NTT3_ROWS_FWD, KC_NTT3_ROWS_INV,
  KC_NTT2_COLS_INV, KC_KS_COLS4, KC_NTT_SMALL_FWD, KC_NTT_SMALL_INV, KC_GEMV_INNER, KC_KSQ_DROP, KC_KSQ_KEEP,
  KC_MODUP_SMALL, KC_DOWN_SMALL, KC_GEMV_WIN, KC_GEMV_FBC, KC_GEMV_FOLD, KC_GEMV_C0, KC_COUNT
};
struct ProfScope {
  int cls;
  double bytes;
  hipEvent_t a = nullptr;
  ProfScope(int c, double b);  // b: the launch's algorithmic bytes
  ~ProfScope();
  ProfScope(const ProfScope &) = delete;
  ProfScope &operator=(const ProfScope &) = delete;
};
void k_to_mont(uint64_t *out, const uint64_t *in, unsigned nlimbs_total);
struct UpTable;
const UpTable &k_up_table(unsigned lvl);  // ModUp conversion tables of a level (kernels.hip)
// he_gemv / he_rot over a ciphertext batch on the windowed FP64 path
// (gemv_win.hip): every modulus of basis_qp(lvl) below 2^51, 2^13 <= n <= 2^17,
// at most three digits
bool k_gemv_win_ok(unsigned lvl);
// ModUp of the c1 of count ciphertexts (c0 at x + c x_stride, c1 at + x_pstride)
// through the split key switch's ModUp kernels: T1 [count][ndig][nm][n] in NTT
// form on every slot outside its digit (own-digit slots unwritten); ybuf
// [count][lvl][n] workspace.  False when the ring / prime set has no such form.
bool k_modup_c1_split(uint64_t *T1, uint64_t *ybuf, const uint64_t *x, size_t x_stride, size_t x_pstride,
                      unsigned count, unsigned lvl);
struct GemvDiagIn {
  unsigned d;           // rotation (0: the identity)
  const uint64_t *pt;   // encoded diagonal over basis_qp(lvl) (NTT form); null: 1
  const uint64_t *evk;  // rotation key (null for d = 0)
};
// Keys folded with their diagonals, in source order: [nm][E][2 ndig + 1][n]
// doubles (pool memory; the caller caches and frees it)
double *k_gemv_fold(const GemvDiagIn *dg, unsigned E, unsigned lvl);
size_t k_gemv_fold_words(unsigned E, unsigned lvl);
// y [count][2][keep][n] = ModDown(sum over the folded diagonals d[e] of the
// rotated key switch of x [count][2][lvl][n]); mode 1: by P q_{lvl-1} (he_gemv,
// keep = lvl - 1), 0: by P (he_rot, keep = lvl)
void k_gemv_batch(uint64_t *y, const uint64_t *x, size_t count, unsigned lvl, const double *K, const unsigned *d,
                  unsigned E, int mode);
// The same with explicit layouts: ciphertext c's poly p at x + c x_stride +
// p x_pstride (y likewise); y_stride != 2 y_pstride runs one ModDown per
// ciphertext (an object's own layout, count 1)
void k_gemv_batch_ex(uint64_t *y, size_t y_stride, size_t y_pstride, const uint64_t *x, size_t x_stride,
                     size_t x_pstride, size_t count, unsigned lvl, const double *K, const unsigned *d, unsigned E,
                     int mode);
void tables_upload();
void tables_prewarm();
void tables_free();
