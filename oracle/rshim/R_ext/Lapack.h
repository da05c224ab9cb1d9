/* oracle/rshim/R_ext/Lapack.h — LAPACK prototypes used by the reference
 * (forwarded by rshim.c to a runtime-loaded LP64 LAPACK). */
#ifndef RSHIM_LAPACK_H
#define RSHIM_LAPACK_H
#include <stddef.h>
void dgeevx_(const char *balanc, const char *jobvl, const char *jobvr,
             const char *sense, const int *n, double *a, const int *lda,
             double *wr, double *wi, double *vl, const int *ldvl, double *vr,
             const int *ldvr, int *ilo, int *ihi, double *scale, double *abnrm,
             double *rconde, double *rcondv, double *work, const int *lwork,
             int *iwork, int *info, size_t, size_t, size_t, size_t);
void dgetrf_(const int *m, const int *n, double *a, const int *lda, int *ipiv,
             int *info);
void dgetri_(const int *n, double *a, const int *lda, const int *ipiv,
             double *work, const int *lwork, int *info);
#endif
