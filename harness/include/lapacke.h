/*
 * lapacke.h - the LAPACKE subset HECTR's harness calls, implemented in
 * harness/lapacke_subset.c (liblapacke.so), so the unchanged reference
 * sources build on a host without LAPACK development files (SURVEY 8(f),
 * harness portability).  Call sites: reference src/matrices.c:43-54 (getrf /
 * getri), :71 (dgesvd, jobu = jobvt = 'A'), :99 (zgeev, jobvl = 'N',
 * jobvr = 'V'); src/hectr.h:34 includes this header.
 *
 * Signatures, argument meaning, return codes and the ipiv convention (1-based
 * row interchanges) are LAPACKE's.  Row- and column-major layouts are both
 * accepted.  The algorithms are the textbook ones for the small dense
 * matrices of a control loop (n <= a few dozen): partial-pivoting LU,
 * one-sided Jacobi SVD, Householder Hessenberg + shifted complex QR.
 */
#ifndef HECTR_PORT_LAPACKE_H
#define HECTR_PORT_LAPACKE_H

#include <complex.h>

#ifdef __cplusplus
extern "C" {
#endif

#ifndef lapack_int
#define lapack_int int
#endif
#ifndef lapack_complex_double
#define lapack_complex_double double _Complex
#endif

#define LAPACK_ROW_MAJOR 101
#define LAPACK_COL_MAJOR 102

lapack_int LAPACKE_dgetrf(int matrix_layout, lapack_int m, lapack_int n, double *a, lapack_int lda,
                          lapack_int *ipiv);
lapack_int LAPACKE_dgetri(int matrix_layout, lapack_int n, double *a, lapack_int lda, const lapack_int *ipiv);
lapack_int LAPACKE_zgetrf(int matrix_layout, lapack_int m, lapack_int n, lapack_complex_double *a, lapack_int lda,
                          lapack_int *ipiv);
lapack_int LAPACKE_zgetri(int matrix_layout, lapack_int n, lapack_complex_double *a, lapack_int lda,
                          const lapack_int *ipiv);
lapack_int LAPACKE_dgesvd(int matrix_layout, char jobu, char jobvt, lapack_int m, lapack_int n, double *a,
                          lapack_int lda, double *s, double *u, lapack_int ldu, double *vt, lapack_int ldvt,
                          double *superb);
lapack_int LAPACKE_zgeev(int matrix_layout, char jobvl, char jobvr, lapack_int n, lapack_complex_double *a,
                         lapack_int lda, lapack_complex_double *w, lapack_complex_double *vl, lapack_int ldvl,
                         lapack_complex_double *vr, lapack_int ldvr);

#ifdef __cplusplus
}
#endif

#endif /* HECTR_PORT_LAPACKE_H */
