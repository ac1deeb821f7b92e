/*
 * lapacke_subset.c - the six LAPACKE routines HECTR's plaintext control code
 * calls (reference src/matrices.c:36-122), for small dense matrices.
 *
 *   dgetrf / zgetrf  LU with partial pivoting (LAPACK xGETF2 order; pivot on
 *                    the largest |a| (complex: |re| + |im|, as IZAMAX))
 *   dgetri / zgetri  inverse from the LU factors: inv(U), then inv(A) L =
 *                    inv(U), then the column interchanges in reverse (xGETRI)
 *   dgesvd           one-sided Jacobi SVD, jobu = jobvt = 'A' (full U and VT;
 *                    singular values descending)
 *   zgeev            Householder Hessenberg reduction, single-shift complex
 *                    QR (Wilkinson shift) to Schur form T = Z^H A Z, right
 *                    eigenvectors by back substitution in T, v = Z x,
 *                    normalised to unit 2-norm with the largest component
 *                    real (xGEEV's convention)
 *
 * Harness portability only: this is the host-side
 * numerical library of the unchanged HECTR harness, not part of the CKKS
 * engine.  Results agree with reference LAPACK to rounding; eigenvector
 * phase and singular-vector signs are not unique, and HECTR's uses (expm as
 * V diag(e^l) V^-1, pinv as V S^-1 U^T) do not depend on them.
 */
#include "include/lapacke.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

typedef double _Complex zc;

static inline size_t ix(int layout, lapack_int i, lapack_int j, lapack_int ld)
{
  return layout == LAPACK_ROW_MAJOR ? (size_t)i * ld + j : (size_t)j * ld + i;
}

static inline double zabs1(zc z) { return fabs(creal(z)) + fabs(cimag(z)); }

static int bad_layout(int layout) { return layout != LAPACK_ROW_MAJOR && layout != LAPACK_COL_MAJOR; }

/* ------------------------------------------------------------------------ */
/* LU factorisation and inverse (real and complex share the code by macro). */
/* ------------------------------------------------------------------------ */
#define DEFINE_GETRF(NAME, T, ABS)                                                                     \
  lapack_int NAME(int layout, lapack_int m, lapack_int n, T *a, lapack_int lda, lapack_int *ipiv)     \
  {                                                                                                    \
    if (bad_layout(layout))                                                                            \
      return -1;                                                                                       \
    if (m < 0)                                                                                         \
      return -2;                                                                                       \
    if (n < 0)                                                                                         \
      return -3;                                                                                       \
    lapack_int info = 0;                                                                               \
    const lapack_int k = m < n ? m : n;                                                                \
    for (lapack_int j = 0; j < k; j++) {                                                               \
      lapack_int p = j;                                                                                \
      double best = ABS(a[ix(layout, j, j, lda)]);                                                     \
      for (lapack_int i = j + 1; i < m; i++) {                                                         \
        const double v = ABS(a[ix(layout, i, j, lda)]);                                                \
        if (v > best) {                                                                                \
          best = v;                                                                                    \
          p = i;                                                                                       \
        }                                                                                              \
      }                                                                                                \
      ipiv[j] = p + 1;                                                                                 \
      if (a[ix(layout, p, j, lda)] != 0) {                                                             \
        if (p != j)                                                                                    \
          for (lapack_int c = 0; c < n; c++) {                                                         \
            T t = a[ix(layout, j, c, lda)];                                                            \
            a[ix(layout, j, c, lda)] = a[ix(layout, p, c, lda)];                                       \
            a[ix(layout, p, c, lda)] = t;                                                              \
          }                                                                                            \
        const T r = 1.0 / a[ix(layout, j, j, lda)];                                                    \
        for (lapack_int i = j + 1; i < m; i++)                                                         \
          a[ix(layout, i, j, lda)] *= r;                                                               \
      } else if (!info) {                                                                              \
        info = j + 1;                                                                                  \
      }                                                                                                \
      for (lapack_int i = j + 1; i < m; i++) {                                                         \
        const T l = a[ix(layout, i, j, lda)];                                                          \
        if (l != 0)                                                                                    \
          for (lapack_int c = j + 1; c < n; c++)                                                       \
            a[ix(layout, i, c, lda)] -= l * a[ix(layout, j, c, lda)];                                  \
      }                                                                                                \
    }                                                                                                  \
    return info;                                                                                       \
  }

#define DEFINE_GETRI(NAME, T)                                                                          \
  lapack_int NAME(int layout, lapack_int n, T *a, lapack_int lda, const lapack_int *ipiv)             \
  {                                                                                                    \
    if (bad_layout(layout))                                                                            \
      return -1;                                                                                       \
    if (n < 0)                                                                                         \
      return -2;                                                                                       \
    for (lapack_int i = 0; i < n; i++)                                                                 \
      if (a[ix(layout, i, i, lda)] == 0)                                                               \
        return i + 1;                                                                                  \
    /* inv(U) in place (upper triangle), column by column */                                          \
    for (lapack_int j = 0; j < n; j++) {                                                               \
      a[ix(layout, j, j, lda)] = 1.0 / a[ix(layout, j, j, lda)];                                       \
      const T ajj = -a[ix(layout, j, j, lda)];                                                         \
      /* x = inv(U)[0:j, 0:j] * U[0:j, j], then scale by -1 / U[j, j] */                              \
      for (lapack_int i = 0; i < j; i++) {                                                             \
        T s = 0;                                                                                       \
        for (lapack_int c = i; c < j; c++)                                                             \
          s += a[ix(layout, i, c, lda)] * a[ix(layout, c, j, lda)];                                    \
        a[ix(layout, i, j, lda)] = s;                                                                  \
      }                                                                                                \
      for (lapack_int i = 0; i < j; i++)                                                               \
        a[ix(layout, i, j, lda)] *= ajj;                                                               \
    }                                                                                                  \
    /* solve inv(A) L = inv(U) for inv(A), columns n-2 .. 0 */                                         \
    T *work = (T *)malloc(sizeof(T) * (size_t)(n ? n : 1));                                            \
    if (!work)                                                                                         \
      return -1011;                                                                                    \
    for (lapack_int j = n - 2; j >= 0; j--) {                                                          \
      for (lapack_int i = j + 1; i < n; i++) {                                                         \
        work[i] = a[ix(layout, i, j, lda)];                                                            \
        a[ix(layout, i, j, lda)] = 0;                                                                  \
      }                                                                                                \
      for (lapack_int r = 0; r < n; r++) {                                                             \
        T s = 0;                                                                                       \
        for (lapack_int i = j + 1; i < n; i++)                                                         \
          s += a[ix(layout, r, i, lda)] * work[i];                                                     \
        a[ix(layout, r, j, lda)] -= s;                                                                 \
      }                                                                                                \
    }                                                                                                  \
    free(work);                                                                                        \
    /* column interchanges, in reverse order */                                                        \
    for (lapack_int j = n - 2; j >= 0; j--) {                                                          \
      const lapack_int jp = ipiv[j] - 1;                                                               \
      if (jp != j)                                                                                     \
        for (lapack_int r = 0; r < n; r++) {                                                           \
          T t = a[ix(layout, r, j, lda)];                                                              \
          a[ix(layout, r, j, lda)] = a[ix(layout, r, jp, lda)];                                        \
          a[ix(layout, r, jp, lda)] = t;                                                               \
        }                                                                                              \
    }                                                                                                  \
    return 0;                                                                                          \
  }

DEFINE_GETRF(LAPACKE_dgetrf, double, fabs)
DEFINE_GETRF(LAPACKE_zgetrf, zc, zabs1)
DEFINE_GETRI(LAPACKE_dgetri, double)
DEFINE_GETRI(LAPACKE_zgetri, zc)

/* ------------------------------------------------------------------------ */
/* SVD: one-sided Jacobi on a tall matrix W (M x N, M >= N, row-major).      */
/* ------------------------------------------------------------------------ */
/* Complete the orthonormal columns U[:, j] (j in `have`) to a basis of R^M:
 * Gram-Schmidt (twice) on the unit vectors e_r, taking the one with the
 * largest residual each time. */
static void complete_basis(double *U, lapack_int M, unsigned char *have)
{
  double *v = malloc(sizeof(double) * (size_t)M), *best = malloc(sizeof(double) * (size_t)M);
  for (lapack_int j = 0; j < M; j++) {
    if (have[j])
      continue;
    double bn = -1;
    for (lapack_int r = 0; r < M; r++) {
      for (lapack_int i = 0; i < M; i++)
        v[i] = i == r;
      for (int pass = 0; pass < 2; pass++)
        for (lapack_int c = 0; c < M; c++) {
          if (!have[c])
            continue;
          double d = 0;
          for (lapack_int i = 0; i < M; i++)
            d += U[(size_t)i * M + c] * v[i];
          for (lapack_int i = 0; i < M; i++)
            v[i] -= d * U[(size_t)i * M + c];
        }
      double nv = 0;
      for (lapack_int i = 0; i < M; i++)
        nv += v[i] * v[i];
      if (nv > bn) {
        bn = nv;
        memcpy(best, v, sizeof(double) * (size_t)M);
      }
    }
    bn = sqrt(bn);
    for (lapack_int i = 0; i < M; i++)
      U[(size_t)i * M + j] = best[i] / bn;
    have[j] = 1;
  }
  free(v);
  free(best);
}

/* W (M x N, M >= N) = U diag(s) V^T; U is M x M, V is N x N (row-major). */
static int svd_tall(double *W, lapack_int M, lapack_int N, double *s, double *U, double *V)
{
  for (lapack_int i = 0; i < N; i++)
    for (lapack_int j = 0; j < N; j++)
      V[(size_t)i * N + j] = i == j;
  for (int sweep = 0; sweep < 80; sweep++) {
    int rotated = 0;
    for (lapack_int p = 0; p < N; p++)
      for (lapack_int q = p + 1; q < N; q++) {
        double al = 0, be = 0, ga = 0;
        for (lapack_int i = 0; i < M; i++) {
          const double x = W[(size_t)i * N + p], y = W[(size_t)i * N + q];
          al += x * x;
          be += y * y;
          ga += x * y;
        }
        if (ga == 0 || fabs(ga) <= DBL_EPSILON * sqrt(al * be))
          continue;
        rotated = 1;
        const double zeta = (be - al) / (2 * ga);
        const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1 + zeta * zeta));
        const double c = 1 / sqrt(1 + t * t), sn = c * t;
        for (lapack_int i = 0; i < M; i++) {
          const double x = W[(size_t)i * N + p], y = W[(size_t)i * N + q];
          W[(size_t)i * N + p] = c * x - sn * y;
          W[(size_t)i * N + q] = sn * x + c * y;
        }
        for (lapack_int i = 0; i < N; i++) {
          const double x = V[(size_t)i * N + p], y = V[(size_t)i * N + q];
          V[(size_t)i * N + p] = c * x - sn * y;
          V[(size_t)i * N + q] = sn * x + c * y;
        }
      }
    if (!rotated)
      break;
  }
  for (lapack_int j = 0; j < N; j++) {
    double nn = 0;
    for (lapack_int i = 0; i < M; i++)
      nn += W[(size_t)i * N + j] * W[(size_t)i * N + j];
    s[j] = sqrt(nn);
  }
  /* sort descending (selection sort, permuting W and V columns alike) */
  for (lapack_int j = 0; j < N; j++) {
    lapack_int b = j;
    for (lapack_int k = j + 1; k < N; k++)
      if (s[k] > s[b])
        b = k;
    if (b == j)
      continue;
    double t = s[j];
    s[j] = s[b];
    s[b] = t;
    for (lapack_int i = 0; i < M; i++) {
      t = W[(size_t)i * N + j];
      W[(size_t)i * N + j] = W[(size_t)i * N + b];
      W[(size_t)i * N + b] = t;
    }
    for (lapack_int i = 0; i < N; i++) {
      t = V[(size_t)i * N + j];
      V[(size_t)i * N + j] = V[(size_t)i * N + b];
      V[(size_t)i * N + b] = t;
    }
  }
  unsigned char *have = calloc((size_t)M, 1);
  const double tiny = (s[0] > 0 ? s[0] : 1.0) * DBL_EPSILON * (double)(M > N ? M : N);
  for (lapack_int j = 0; j < M; j++)
    for (lapack_int i = 0; i < M; i++)
      U[(size_t)i * M + j] = 0;
  for (lapack_int j = 0; j < N; j++) {
    if (s[j] <= tiny)
      continue;
    for (lapack_int i = 0; i < M; i++)
      U[(size_t)i * M + j] = W[(size_t)i * N + j] / s[j];
    have[j] = 1;
  }
  complete_basis(U, M, have);
  free(have);
  return 0;
}

lapack_int LAPACKE_dgesvd(int layout, char jobu, char jobvt, lapack_int m, lapack_int n, double *a, lapack_int lda,
                          double *s, double *u, lapack_int ldu, double *vt, lapack_int ldvt, double *superb)
{
  if (bad_layout(layout))
    return -1;
  if (jobu != 'A' && jobu != 'a')
    return -2;  /* only the full factorisation HECTR asks for (src/matrices.c:71) */
  if (jobvt != 'A' && jobvt != 'a')
    return -3;
  if (m < 0)
    return -4;
  if (n < 0)
    return -5;
  const lapack_int k = m < n ? m : n;
  if (!k)
    return 0;
  const int tall = m >= n;
  const lapack_int M = tall ? m : n, N = tall ? n : m;
  double *W = malloc(sizeof(double) * (size_t)M * N), *Ub = malloc(sizeof(double) * (size_t)M * M),
         *Vb = malloc(sizeof(double) * (size_t)N * N);
  if (!W || !Ub || !Vb)
    return -1011;
  for (lapack_int i = 0; i < m; i++)
    for (lapack_int j = 0; j < n; j++) {
      const double v = a[ix(layout, i, j, lda)];
      if (tall)
        W[(size_t)i * N + j] = v;
      else
        W[(size_t)j * N + i] = v;  /* W = A^T */
    }
  svd_tall(W, M, N, s, Ub, Vb);
  /* tall: A = Ub S Vb^T.  wide: A^T = Ub S Vb^T, so A = Vb S Ub^T. */
  for (lapack_int i = 0; i < m; i++)
    for (lapack_int j = 0; j < m; j++)
      u[ix(layout, i, j, ldu)] = tall ? Ub[(size_t)i * M + j] : Vb[(size_t)i * N + j];
  for (lapack_int i = 0; i < n; i++)
    for (lapack_int j = 0; j < n; j++)
      vt[ix(layout, i, j, ldvt)] = tall ? Vb[(size_t)j * N + i] : Ub[(size_t)j * M + i];
  if (superb)
    for (lapack_int i = 0; i + 1 < k; i++)
      superb[i] = 0;
  free(W);
  free(Ub);
  free(Vb);
  return 0;
}

/* ------------------------------------------------------------------------ */
/* Complex eigenproblem.                                                     */
/* ------------------------------------------------------------------------ */
/* G = [[c, s], [-conj(s), c]] with G (x, y)^T = (r, 0)^T. */
static void zgivens(zc x, zc y, double *c, zc *s)
{
  const double ay = cabs(y);
  if (ay == 0) {
    *c = 1;
    *s = 0;
    return;
  }
  const double ax = cabs(x);
  if (ax == 0) {
    *c = 0;
    *s = conj(y) / ay;
    return;
  }
  const double t = hypot(ax, ay);
  *c = ax / t;
  *s = (x / ax) * conj(y) / t;
}

lapack_int LAPACKE_zgeev(int layout, char jobvl, char jobvr, lapack_int n, zc *a, lapack_int lda, zc *w, zc *vl,
                         lapack_int ldvl, zc *vr, lapack_int ldvr)
{
  (void)vl;
  (void)ldvl;
  if (bad_layout(layout))
    return -1;
  if (jobvl != 'N' && jobvl != 'n')
    return -2;  /* left eigenvectors are not needed by HECTR (src/matrices.c:99) */
  const int want_v = jobvr == 'V' || jobvr == 'v';
  if (!want_v && jobvr != 'N' && jobvr != 'n')
    return -3;
  if (n < 0)
    return -4;
  if (!n)
    return 0;
  const size_t N = (size_t)n;
  zc *H = malloc(sizeof(zc) * N * N), *Z = malloc(sizeof(zc) * N * N), *v = malloc(sizeof(zc) * N);
  if (!H || !Z || !v)
    return -1011;
#define HH(i, j) H[(size_t)(i) * N + (j)]
#define ZZ(i, j) Z[(size_t)(i) * N + (j)]
  for (lapack_int i = 0; i < n; i++)
    for (lapack_int j = 0; j < n; j++) {
      HH(i, j) = a[ix(layout, i, j, lda)];
      ZZ(i, j) = i == j;
    }
  /* Householder reduction to upper Hessenberg form, Z accumulates */
  for (lapack_int k = 0; k + 2 < n; k++) {
    double nx = 0;
    for (lapack_int i = k + 1; i < n; i++)
      nx += creal(HH(i, k) * conj(HH(i, k)));
    nx = sqrt(nx);
    if (nx == 0)
      continue;
    const zc x0 = HH(k + 1, k);
    const zc ph = cabs(x0) > 0 ? x0 / cabs(x0) : 1.0;
    const zc alpha = -ph * nx;
    for (lapack_int i = k + 1; i < n; i++)
      v[i] = HH(i, k);
    v[k + 1] -= alpha;
    double nv = 0;
    for (lapack_int i = k + 1; i < n; i++)
      nv += creal(v[i] * conj(v[i]));
    nv = sqrt(nv);
    if (nv == 0)
      continue;
    for (lapack_int i = k + 1; i < n; i++)
      v[i] /= nv;
    /* H <- (I - 2 v v^H) H */
    for (lapack_int j = 0; j < n; j++) {
      zc d = 0;
      for (lapack_int i = k + 1; i < n; i++)
        d += conj(v[i]) * HH(i, j);
      for (lapack_int i = k + 1; i < n; i++)
        HH(i, j) -= 2.0 * v[i] * d;
    }
    /* H <- H (I - 2 v v^H), Z <- Z (I - 2 v v^H) */
    for (lapack_int r = 0; r < n; r++) {
      zc d = 0, e = 0;
      for (lapack_int i = k + 1; i < n; i++) {
        d += HH(r, i) * v[i];
        e += ZZ(r, i) * v[i];
      }
      for (lapack_int i = k + 1; i < n; i++) {
        HH(r, i) -= 2.0 * d * conj(v[i]);
        ZZ(r, i) -= 2.0 * e * conj(v[i]);
      }
    }
    for (lapack_int i = k + 2; i < n; i++)
      HH(i, k) = 0;
  }
  /* shifted QR iteration to Schur form (upper triangular T), Z accumulates */
  double hnorm = 0;
  for (size_t i = 0; i < N * N; i++)
    hnorm = fmax(hnorm, zabs1(H[i]));
  lapack_int info = 0, hi = n - 1, its = 0;
  double *cs = malloc(sizeof(double) * N);
  zc *ss = malloc(sizeof(zc) * N);
  while (hi > 0) {
    lapack_int l = hi;
    for (; l > 0; l--) {
      double sc = zabs1(HH(l - 1, l - 1)) + zabs1(HH(l, l));
      if (sc == 0)
        sc = hnorm;
      if (zabs1(HH(l, l - 1)) <= DBL_EPSILON * sc) {
        HH(l, l - 1) = 0;
        break;
      }
    }
    if (l == hi) {
      hi--;
      its = 0;
      continue;
    }
    if (++its > 60) {
      info = hi + 1;
      break;
    }
    /* Wilkinson shift: eigenvalue of the trailing 2x2 closest to H[hi][hi];
       exceptional shifts every 10 iterations without deflation */
    zc mu;
    if (its % 10 == 0) {
      mu = HH(hi, hi) + 0.75 * cabs(HH(hi, hi - 1));
    } else {
      const zc p = HH(hi - 1, hi - 1), q = HH(hi - 1, hi), r = HH(hi, hi - 1), d = HH(hi, hi);
      const zc tr = 0.5 * (p - d), disc = csqrt(tr * tr + q * r);
      const zc m1 = d + tr + disc, m2 = d + tr - disc;  /* (p + d) / 2 +- disc */
      mu = cabs(m1 - d) < cabs(m2 - d) ? m1 : m2;
    }
    for (lapack_int i = l; i <= hi; i++)
      HH(i, i) -= mu;
    for (lapack_int k = l; k < hi; k++) {
      zgivens(HH(k, k), HH(k + 1, k), &cs[k], &ss[k]);
      for (lapack_int j = k; j < n; j++) {
        const zc x = HH(k, j), y = HH(k + 1, j);
        HH(k, j) = cs[k] * x + ss[k] * y;
        HH(k + 1, j) = -conj(ss[k]) * x + cs[k] * y;
      }
    }
    for (lapack_int k = l; k < hi; k++) {
      const lapack_int rmax = k + 2 < hi ? k + 2 : hi;
      for (lapack_int r = 0; r <= rmax; r++) {
        const zc x = HH(r, k), y = HH(r, k + 1);
        HH(r, k) = cs[k] * x + conj(ss[k]) * y;
        HH(r, k + 1) = -ss[k] * x + cs[k] * y;
      }
      for (lapack_int r = 0; r < n; r++) {
        const zc x = ZZ(r, k), y = ZZ(r, k + 1);
        ZZ(r, k) = cs[k] * x + conj(ss[k]) * y;
        ZZ(r, k + 1) = -ss[k] * x + cs[k] * y;
      }
    }
    for (lapack_int i = l; i <= hi; i++)
      HH(i, i) += mu;
  }
  free(cs);
  free(ss);
  for (lapack_int i = 0; i < n; i++)
    w[i] = HH(i, i);
  if (!info && want_v) {
    const double smlnum = DBL_MIN * ((double)n / DBL_EPSILON);
    zc *x = malloc(sizeof(zc) * N);
    for (lapack_int k = n - 1; k >= 0; k--) {
      const zc lk = HH(k, k);
      const double smin = fmax(DBL_EPSILON * zabs1(lk), smlnum);
      for (lapack_int i = 0; i < n; i++)
        x[i] = 0;
      x[k] = 1;
      for (lapack_int i = k - 1; i >= 0; i--) {
        zc s = 0;
        for (lapack_int j = i + 1; j <= k; j++)
          s += HH(i, j) * x[j];
        zc d = HH(i, i) - lk;
        if (zabs1(d) < smin)
          d = smin;
        x[i] = -s / d;
      }
      /* v = Z x, unit 2-norm, largest component real */
      double nn = 0, big = -1;
      lapack_int ib = 0;
      for (lapack_int r = 0; r < n; r++) {
        zc t = 0;
        for (lapack_int j = 0; j <= k; j++)
          t += ZZ(r, j) * x[j];
        v[r] = t;
        const double m2 = creal(t * conj(t));
        nn += m2;
        if (m2 > big) {
          big = m2;
          ib = r;
        }
      }
      const zc rot = conj(v[ib]) / cabs(v[ib]) / sqrt(nn);
      for (lapack_int r = 0; r < n; r++) {
        zc t = v[r] * rot;
        if (r == ib)
          t = creal(t);
        vr[ix(layout, r, k, ldvr)] = t;
      }
    }
    free(x);
  }
#undef HH
#undef ZZ
  free(H);
  free(Z);
  free(v);
  return info;
}
