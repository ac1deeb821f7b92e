/*
 * gpqhe.h - C ABI of the MI355X-native CKKS engine (libgpqhe.so).
 *
 * This header is the drop-in boundary for OChicken/HECTR: HECTR includes
 * "../GPQHE/src/gpqhe.h" (reference src/hectr.h:35, src/ctr.c:23,
 * tests/hectr.c:23) and links -lgpqhe (reference tests/Makefile:25).
 * GPQHE itself is an empty submodule in the reference (.gitmodules:1-3), so
 * every signature below is inferred from its call sites; each declaration
 * cites the reference line(s) it serves.  Declarations marked [ext] are
 * additions that HECTR does not call (benchmarks, tests, serialization).
 *
 * Pure C99, no HIP types: it compiles under gcc -Wall -Wextra -Wpedantic
 * (reference Makefile:21) and is include-guarded (tests/hectr.c:22-23
 * includes it twice).  All functions return void and abort with a message on
 * error, matching the void-return convention of every call site
 * (reference src/hempc.c:246-273, src/ctr.c:461-475,524-541).
 *
 * Two implementations export this ABI:
 *   libgpqhe.so          - the product: host C++ + gfx950 HIP kernels; the
 *                          `data` pointers of all objects are device memory.
 *   oracle/libgpqhe_oracle.so - test infrastructure only: the CPU C
 *                          restatement used as the parity checker and CPU
 *                          baseline; `data` pointers are host memory.
 */
#ifndef GPQHE_H
#define GPQHE_H

#include <stddef.h>
#include <stdint.h>
/* HECTR's sources call abort / exit / malloc without including <stdlib.h>
   themselves (reference src/mpc.c:211, tests/hectr.c:938): the GPQHE header
   they include provides it. */
#include <stdlib.h>

#ifdef __cplusplus
extern "C" {
typedef struct gpqhe_c128 { double re, im; } gpqhe_complex_t;
#else
typedef _Complex double gpqhe_complex_t;
#endif

/* ------------------------------------------------------------------------ */
/* Multi-precision integer handle (libgcrypt-style).                        */
/* HECTR: `MPI q = mpi_set_ui(NULL, 1); mpi_lshift(q, q, 109);`             */
/*        `mpi_release(q);`   (reference src/ctr.c:515-516,607)              */
/* <gcrypt.h> is not part of the boundary, so the header supplies its own.  */
/* ------------------------------------------------------------------------ */
typedef struct gpqhe_mpi *MPI;
MPI      gpqhe_mpi_set_ui(MPI w, unsigned long u);
void     gpqhe_mpi_lshift(MPI x, MPI a, unsigned int n);
void     gpqhe_mpi_release(MPI a);
unsigned gpqhe_mpi_get_nbits(MPI a);
#define mpi_set_ui(w, u)     gpqhe_mpi_set_ui((w), (u))
#define mpi_lshift(x, a, n)  gpqhe_mpi_lshift((x), (a), (n))
#define mpi_release(a)       gpqhe_mpi_release(a)
#define mpi_get_nbits(a)     gpqhe_mpi_get_nbits(a)

/* ------------------------------------------------------------------------ */
/* Object types.  The caller owns the struct storage (on the stack, even in  */
/* a VLA: `he_evk_t rk[slots]`, reference src/ctr.c:521), so sizeof must be */
/* complete here; he_alloc_* attaches the payload, he_free_* releases it.    */
/*                                                                           */
/* Payload layout (both implementations): `data` holds npoly polynomials,   */
/* each `cap` limbs of n = 2^logn uint64 residues, limb-major:               */
/*   data[(p * cap + limb) * n + coeff]                                       */
/* Limb order is q_0 .. q_{L-1} then the special primes p_0 .. p_{K-1}.      */
/* Residues are canonical (in [0, q)) and in NTT (evaluation) order unless   */
/* flags say otherwise.                                                      */
/* ------------------------------------------------------------------------ */
#define GPQHE_OBJECT_FIELDS                                                    \
  uint64_t *data;   /* residues (device memory in libgpqhe.so)            */  \
  uint32_t nlimbs;  /* limbs in use = current level                        */ \
  uint32_t cap;     /* limbs allocated per polynomial                      */ \
  uint32_t npoly;   /* polynomials held                                    */ \
  uint32_t galois;  /* evk: Galois element (1 = relinearization key)      */  \
  double   scale;   /* CKKS scaling factor of the encoded message          */ \
  uint32_t flags;   /* GPQHE_F_* bits                                      */ \
  uint32_t dnum;    /* evk: key-switch digits                              */ \
  uint64_t reserved;

#define GPQHE_F_COEFF   1u  /* residues are in coefficient order (not NTT)  */
#define GPQHE_F_SPECIAL 2u  /* pt also carries the special-prime limbs      */

typedef struct he_ct_s    { GPQHE_OBJECT_FIELDS } he_ct_t;    /* ciphertext (c0, c1)   */
typedef struct he_pt_s    { GPQHE_OBJECT_FIELDS } he_pt_t;    /* plaintext             */
typedef struct he_pk_s    { GPQHE_OBJECT_FIELDS } he_pk_t;    /* public key (b, a)     */
typedef struct he_evk_s   { GPQHE_OBJECT_FIELDS } he_evk_t;   /* key-switching key     */
typedef struct poly_mpi_s { GPQHE_OBJECT_FIELDS } poly_mpi_t; /* secret key s (QP, NTT)*/

/* ------------------------------------------------------------------------ */
/* Context (process-global singleton: no ctx argument on any call).          */
/* ------------------------------------------------------------------------ */

/* reference src/ctr.c:514-518 (logn=12, q=2^109, slots, Delta=2^50), :617.
 * The modulus chain is derived from log2(q) and log2(Delta): L limbs with
 * q_1..q_{L-1} of log2(Delta) bits and q_0 taking the rest (q=2^109,
 * Delta=2^50 -> q_0: 59 bits, q_1: 50 bits), one 60-bit special prime,
 * dnum = L.  Environment overrides (for the unchanged caller):
 * GPQHE_LOGN, GPQHE_NLIMBS, GPQHE_DNUM, GPQHE_SEED. */
void hectx_init(unsigned int logn, MPI q, unsigned int slots, uint64_t Delta);
void hectx_exit(void);

typedef struct gpqhe_params {
  uint32_t logn;      /* ring degree n = 2^logn, 4 <= logn <= 17          */
  uint32_t nlimbs;    /* L: primes of the ciphertext modulus Q            */
  uint32_t nspecial;  /* K: special primes of P (key switching)           */
  uint32_t dnum;      /* key-switch digits; a digit spans ceil(L/dnum) limbs */
  uint32_t slots;     /* packed complex slots, power of two <= n/2        */
  uint32_t q0_bits;   /* bit size of q_0                                  */
  uint32_t qi_bits;   /* bit size of q_1 .. q_{L-1}                       */
  uint32_t p_bits;    /* bit size of the special primes                   */
  double   delta;     /* default encoding scale                           */
  uint64_t seed;      /* RNG seed (0: from GPQHE_SEED or /dev/urandom)    */
} gpqhe_params_t;
/* [ext] explicit parameters (benchmarks: n=2^16, L=8, ...). */
void hectx_init_params(const gpqhe_params_t *params);

typedef struct gpqhe_info {
  uint32_t logn, n, nlimbs, nspecial, dnum, alpha, slots, reserved;
  double   delta;
  uint64_t primes[64]; /* q_0..q_{L-1}, p_0..p_{K-1}                      */
  uint64_t psi[64];    /* primitive 2n-th roots used by the NTT          */
} gpqhe_info_t;
void hectx_info(gpqhe_info_t *info);                  /* [ext] */
void gpqhe_set_seed(uint64_t seed);                   /* [ext] reset RNG  */
/* [ext] HIP stream (hipStream_t) the engine launches on; NULL = its own.
 * Ignored by the oracle. */
void gpqhe_set_stream(void *stream);
void gpqhe_sync(void);                                /* [ext] */
/* [ext] he_mul_rescale_batch: run a batch as 1 or 2 sub-chunks on their own
 * HIP streams (default 2: one sub-chunk's compute-bound kernels overlap the
 * other's memory-bound ones).  Bits never depend on it; ignored by the
 * oracle. */
void gpqhe_set_streams(unsigned int n);

/* ------------------------------------------------------------------------ */
/* Allocation: reference src/ctr.c:461-465,524-527,537-541,608-616;         */
/* src/hempc.c:246-251,268-273.                                              */
/* ------------------------------------------------------------------------ */
void he_alloc_pk(he_pk_t *pk);     void he_free_pk(he_pk_t *pk);
void he_alloc_sk(poly_mpi_t *sk);  void he_free_sk(poly_mpi_t *sk);
void he_alloc_evk(he_evk_t *evk);  void he_free_evk(he_evk_t *evk);
void he_alloc_ct(he_ct_t *ct);     void he_free_ct(he_ct_t *ct);
void he_alloc_pt(he_pt_t *pt);     void he_free_pt(he_pt_t *pt);

/* ------------------------------------------------------------------------ */
/* Keys                                                                      */
/* ------------------------------------------------------------------------ */
void he_keypair(he_pk_t *pk, poly_mpi_t *sk);                 /* ctr.c:529  */
/* Rotation keys: rk[r] switches sigma_{5^r}(s) -> s, r = 1..slots-1;
 * rk[0] is the identity (no payload).                            ctr.c:532  */
void he_genrk(he_evk_t rk[], const poly_mpi_t *sk);
void he_genrlk(he_evk_t *rlk, const poly_mpi_t *sk);           /* [ext] s^2 */
void he_genrot(he_evk_t *evk, unsigned int rot, const poly_mpi_t *sk); /* [ext] */

/* ------------------------------------------------------------------------ */
/* Encoding / encryption                                                     */
/* ------------------------------------------------------------------------ */
/* z[slots] -> pt at level L, scale Delta.     reference src/ctr.c:466-470   */
void he_ecd(he_pt_t *pt, const gpqhe_complex_t z[]);
/* pt -> z[slots].                              reference src/ctr.c:492       */
void he_dcd(gpqhe_complex_t z[], const he_pt_t *pt);
/* [ext] encode with explicit slots / scale / level. */
void he_ecd_ex(he_pt_t *pt, const gpqhe_complex_t z[], unsigned int slots,
               double scale, unsigned int nlimbs);
void he_dcd_ex(gpqhe_complex_t z[], const he_pt_t *pt, unsigned int slots);
void he_enc_pk(he_ct_t *ct, const he_pt_t *pt, const he_pk_t *pk); /* ctr.c:471-475 */
void he_enc_sk(he_ct_t *ct, const he_pt_t *pt, const poly_mpi_t *sk); /* [ext] */
void he_dec(he_pt_t *pt, const he_ct_t *ct, const poly_mpi_t *sk);   /* ctr.c:489 */

/* ------------------------------------------------------------------------ */
/* Evaluation                                                                */
/* ------------------------------------------------------------------------ */
/* out = a +/- b.  Operands at different levels are aligned by dropping
 * limbs; scales must agree.  `out` may alias an operand and may hold an
 * earlier ciphertext (reference src/hempc.c:266 writes into ct_up).         */
void he_add(he_ct_t *out, const he_ct_t *a, const he_ct_t *b); /* hempc.c:261,266 */
void he_sub(he_ct_t *out, const he_ct_t *a, const he_ct_t *b); /* hempc.c:253,255 */
void he_neg(he_ct_t *ct);                                       /* hempc.c:262 */
void he_copy_ct(he_ct_t *dst, const he_ct_t *src);              /* hempc.c:264 */
/* Drop the top limb without changing the scale.                hempc.c:265  */
void he_moddown(he_ct_t *ct);
/* y = M x for a slots x slots complex matrix M (row-major, M[i*slots+j]),
 * diagonal method with hoisted rotations; y is one level below x and keeps
 * x's scale.                                                  hempc.c:257,259 */
void he_gemv(he_ct_t *y, const gpqhe_complex_t M[], const he_ct_t *x,
             const he_evk_t rk[]);
/* [ext] rotation by `rot` slots (uses rk[rot]). */
void he_rot(he_ct_t *out, const he_ct_t *in, unsigned int rot, const he_evk_t rk[]);
/* [ext] ct x ct multiply + relinearize (no rescale); scale = a.scale*b.scale */
void he_mul(he_ct_t *out, const he_ct_t *a, const he_ct_t *b, const he_evk_t *rlk);
/* [ext] divide by the top prime; drops one level.                           */
void he_rescale(he_ct_t *ct);
/* [ext] fused multiply + relinearize + rescale (ModDown by P*q_top at once). */
void he_mul_rescale(he_ct_t *out, const he_ct_t *a, const he_ct_t *b, const he_evk_t *rlk);
void he_mul_pt(he_ct_t *out, const he_ct_t *a, const he_pt_t *pt);  /* [ext] */
void he_add_pt(he_ct_t *out, const he_ct_t *a, const he_pt_t *pt);  /* [ext] */

/* ------------------------------------------------------------------------ */
/* [ext] Batched entry points for the benchmarks (configs 2, 3, 5).          */
/* Pointers address implementation memory (device memory for libgpqhe.so):  */
/* count contiguous ciphertexts laid out [count][2][nlimbs][n].              */
/* ------------------------------------------------------------------------ */
void he_mul_rescale_batch(uint64_t *out, const uint64_t *a, const uint64_t *b,
                          size_t count, unsigned int nlimbs, const he_evk_t *rlk);
/* he_gemv over `count` independent ciphertexts that share M and the rotation
 * keys (HECTR's encrypted matrix-vector step, reference src/hempc.c:257,259,
 * with its rotation keys from src/ctr.c:521,526-532, batched across a
 * ciphertext batch): x [count][2][nlimbs][n] -> y [count][2][nlimbs-1][n],
 * each y_i = M x_i with the residues he_gemv gives it.  y must not overlap x. */
void he_gemv_batch(uint64_t *y, const gpqhe_complex_t M[], const uint64_t *x,
                   size_t count, unsigned int nlimbs, const he_evk_t rk[]);
/* he_rot of `count` ciphertexts by the same rotation:
 * x [count][2][nlimbs][n] -> out [count][2][nlimbs][n]; no overlap. */
void he_rot_batch(uint64_t *out, const uint64_t *x, size_t count,
                  unsigned int nlimbs, unsigned int rot, const he_evk_t rk[]);
/* npolys contiguous polynomials [npolys][nlimbs][n], limb i mod q_i. */
void poly_ntt_batch(uint64_t *data, size_t npolys, unsigned int nlimbs);
void poly_intt_batch(uint64_t *data, size_t npolys, unsigned int nlimbs);
/* Fill [npolys][nlimbs][n] with splitmix64-derived residues < q_limb
 * (deterministic in seed; benchmark input generator). */
void poly_fill_uniform(uint64_t *data, size_t npolys, unsigned int nlimbs, uint64_t seed);

/* ------------------------------------------------------------------------ */
/* [ext] Live kernel statistics: when enabled, every kernel launch is        */
/* bracketed by HIP events on the engine stream; collect returns, per kernel */
/* class (one kernel symbol each), launches, device time and algorithmic     */
/* bytes (bytes the launch must read + write at minimum), then resets.       */
/* The oracle returns 0 classes.                                             */
/* ------------------------------------------------------------------------ */
typedef struct gpqhe_kstat {
  char     name[40];
  uint32_t launches;
  uint32_t reserved;
  double   total_us;
  double   bytes;
} gpqhe_kstat_t;
void     gpqhe_prof_enable(int on);
unsigned gpqhe_prof_collect(gpqhe_kstat_t *out, unsigned max);
/* [ext] he_gemv calls served by the speculated gemv of the small-N step     */
/* (api.cpp SpecGemv) since hectx_init; the oracle returns 0.                */
unsigned gpqhe_spec_gemv_taken(void);
/* [ext] he_dcd calls of the small-N step served by the replay of the last   */
/* step's elementwise tail and decode (api.cpp SpecDcd); the oracle: 0.      */
unsigned gpqhe_spec_dcd_taken(void);

/* ------------------------------------------------------------------------ */
/* [ext] Serialization (host buffers): residues in the payload layout above, */
/* npoly x nlimbs x n words.  Used for fixtures and cross-engine parity.     */
/* ------------------------------------------------------------------------ */
size_t he_export(const void *obj, uint64_t *host);   /* any he_*_t / poly_mpi_t */
void   he_import(void *obj, const uint64_t *host, unsigned int nlimbs,
                 double scale, uint32_t flags);
void   he_evk_meta(const he_evk_t *evk, uint32_t *galois, uint32_t *dnum);

#ifdef __cplusplus
}
#endif

#endif /* GPQHE_H */
