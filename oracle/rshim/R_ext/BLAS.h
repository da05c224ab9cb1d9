/* oracle/rshim/R_ext/BLAS.h — BLAS prototypes (gfortran calling convention,
 * hidden character lengths as size_t). Implemented in rshim.c. */
#ifndef RSHIM_BLAS_H
#define RSHIM_BLAS_H
#include <stddef.h>
void dgemv_(const char *trans, const int *m, const int *n, const double *alpha,
            const double *a, const int *lda, const double *x, const int *incx,
            const double *beta, double *y, const int *incy, size_t ltrans);
void dgemm_(const char *transa, const char *transb, const int *m, const int *n,
            const int *k, const double *alpha, const double *a, const int *lda,
            const double *b, const int *ldb, const double *beta, double *c,
            const int *ldc, size_t la, size_t lb);
#endif
