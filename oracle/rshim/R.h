/* oracle/rshim/R.h — minimal stand-in for R's C API, written for this
 * repository (test infrastructure only).  It lets the reference's own C
 * sources under /root/reference/src compile unmodified into
 * oracle/_ref/libpht_ref.so, with R's RNG supplied by the R-compatible
 * restatement in phasetype_amd/csrc/rstream.c and BLAS/LAPACK by rshim.c. */
#ifndef RSHIM_R_H
#define RSHIM_R_H
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <float.h>
#include <limits.h>
#include <stddef.h>

#ifndef TRUE
#define TRUE 1
#endif
#ifndef FALSE
#define FALSE 0
#endif

#define F77_CALL(x) x##_
#define F77_NAME(x) x##_
#define FCONE , (size_t)1

void Rprintf(const char *fmt, ...);
void REprintf(const char *fmt, ...);
char *R_alloc(size_t n, int size);
void R_FlushConsole(void);
void R_CheckUserInterrupt(void);
void GetRNGstate(void);
void PutRNGstate(void);
void *rshim_calloc(size_t n, size_t size);
void rshim_free(void *p);
#define R_Calloc(n, t) ((t *)rshim_calloc((size_t)(n), sizeof(t)))
#define R_Free(p) (rshim_free((void *)(p)), (p) = NULL)

#include "Rmath.h"
#endif
