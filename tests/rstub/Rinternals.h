/* see R.h in this directory */
#ifndef RCP_RSTUB_RINTERNALS_H
#define RCP_RSTUB_RINTERNALS_H
#include "R.h"
enum { INTSXP = 13, LGLSXP = 10, REALSXP = 14, STRSXP = 16, VECSXP = 19, EXTPTRSXP = 22 };
extern SEXP R_NilValue, R_NamesSymbol, R_DimNamesSymbol;
extern int R_NaInt;
#define NA_INTEGER R_NaInt
R_xlen_t XLENGTH(SEXP);
int LENGTH(SEXP);
double* REAL(SEXP);
int* INTEGER(SEXP);
int* LOGICAL(SEXP);
int TYPEOF(SEXP);
int asInteger(SEXP);
double asReal(SEXP);
int asLogical(SEXP);
SEXP PROTECT(SEXP);
void UNPROTECT(int);
SEXP allocVector(SEXPTYPE, R_xlen_t);
SEXP allocMatrix(SEXPTYPE, int, int);
SEXP VECTOR_ELT(SEXP, R_xlen_t);
SEXP SET_VECTOR_ELT(SEXP, R_xlen_t, SEXP);
SEXP STRING_ELT(SEXP, R_xlen_t);
void SET_STRING_ELT(SEXP, R_xlen_t, SEXP);
SEXP mkChar(const char*);
const char* CHAR(SEXP);
SEXP setAttrib(SEXP, SEXP, SEXP);
SEXP R_MakeExternalPtr(void*, SEXP, SEXP);
void* R_ExternalPtrAddr(SEXP);
void R_ClearExternalPtr(SEXP);
void R_SetExternalPtrAddr(SEXP, void*);
typedef void (*R_CFinalizer_t)(SEXP);
void R_RegisterCFinalizerEx(SEXP, R_CFinalizer_t, int);
/* S4 objects and their slots (S4Vectors::Rle: "values", "lengths") */
SEXP install(const char*);
int IS_S4_OBJECT(SEXP);
int R_has_slot(SEXP, SEXP);
SEXP R_do_slot(SEXP, SEXP);
typedef void* (*DL_FUNC)(void);
typedef struct { const char* name; DL_FUNC fun; int numArgs; } R_CallMethodDef;
typedef struct _DllInfo DllInfo;
int R_registerRoutines(DllInfo*, const void*, const R_CallMethodDef*, const void*, const void*);
int R_useDynamicSymbols(DllInfo*, int);
#endif
