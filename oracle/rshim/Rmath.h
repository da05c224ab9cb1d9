/* oracle/rshim/Rmath.h — the nmath entry points the reference calls. */
#ifndef RSHIM_RMATH_H
#define RSHIM_RMATH_H
double unif_rand(void);
double exp_rand(void);
double norm_rand(void);
double runif(double a, double b);
double rexp(double scale);
double rgamma(double a, double scale);
double dexp(double x, double scale, int give_log);
#endif
