/* Minimal declarations of the R C API used by r/src/recoup_amd_shim.c -- for a compile check
 * of the shim against include/recoup_amd.h where R itself is not installed
 * (tests/test_r_shim.py), and for tests/rmini/rmini.c, a small emulation of these functions
 * that lets the tests execute the shim.  Not R's header. */
#ifndef RCP_RSTUB_R_H
#define RCP_RSTUB_R_H
#include <stddef.h>
typedef struct SEXPREC* SEXP;
typedef ptrdiff_t R_xlen_t;
typedef unsigned int SEXPTYPE;
void Rf_error(const char*, ...);
char* R_alloc(size_t, int);
int R_IsNA(double);
#define ISNA(x) R_IsNA(x)
#define TRUE 1
#define FALSE 0
#endif
