/* rmini.c -- a small emulation of the R C API subset that r/src/recoup_amd_shim.c uses
 * (declared in tests/rstub), so the tests can EXECUTE the .Call shim where R is not installed.
 * Test infrastructure only: it is linked with the shim and librecoup_amd.so into
 * tests/rmini/build/librmini_shim.so and driven from Python (tests/rmini/rmini.py).
 *
 * What it models of R, and what it checks:
 *   - vectors (integer, logical, double, character, list), matrices (dims kept), names, and a
 *     matrix's dimnames (a list of two: row names, column names; each NULL or character of the
 *     dimension's length -- what R's dimnames<- insists on);
 *   - Rf_error as a longjmp back to rmini_call's setjmp (R's error unwinding), after which the
 *     protect stack is reset, as R resets it;
 *   - the PROTECT stack: rmini_call reports the depth a routine left behind (must be 0);
 *   - external pointers with C finalizers: rmini_run_finalizers runs them all (what R's
 *     garbage collector eventually does), rmini_live_handles counts pointers still holding an
 *     address;
 *   - allocation failure: rmini_fail_alloc_after(k) makes the k-th next R allocation raise the
 *     error R raises when it cannot allocate, so the tests can check that no library handle is
 *     held only by a C local across an R allocation (it would leak).
 * Memory handed out is never reclaimed (a test process is short-lived). */
#include <limits.h>
#include <math.h>
#include <setjmp.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "Rinternals.h"

enum { NILSXP = 0, CHARSXP = 9, S4SXP = 25 };

struct SEXPREC {
    int type;
    R_xlen_t len;
    void* data;
    SEXP names;
    SEXP dimnames;
    int nrow, ncol;
    void* addr;
    R_CFinalizer_t fin;
};

static struct SEXPREC nil_obj = {NILSXP, 0, NULL, NULL, NULL, 0, 0, NULL, NULL};
static struct SEXPREC names_sym = {NILSXP, 0, NULL, NULL, NULL, 0, 0, NULL, NULL};
static struct SEXPREC dimnames_sym = {NILSXP, 0, NULL, NULL, NULL, 0, 0, NULL, NULL};
SEXP R_NilValue = &nil_obj;
SEXP R_NamesSymbol = &names_sym;
SEXP R_DimNamesSymbol = &dimnames_sym;
int R_NaInt = INT_MIN;

static jmp_buf* err_jmp = NULL;
static char err_msg[4096];
static int protect_depth = 0;
static long fail_after = -1; /* allocations left before an injected failure; -1 = never */

#define MAX_EXT 4096
static SEXP ext_tab[MAX_EXT];
static int n_ext = 0;

void Rf_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(err_msg, sizeof err_msg, fmt, ap);
    va_end(ap);
    if (!err_jmp) {
        fprintf(stderr, "rmini: Rf_error outside rmini_call: %s\n", err_msg);
        abort();
    }
    longjmp(*err_jmp, 1);
}

static void count_alloc(void) {
    if (fail_after < 0) return;
    if (fail_after == 0) {
        fail_after = -1;
        Rf_error("cannot allocate vector (injected by rmini)");
    }
    --fail_after;
}

static size_t elt_size(int type) {
    switch (type) {
    case INTSXP:
    case LGLSXP: return sizeof(int);
    case REALSXP: return sizeof(double);
    case STRSXP:
    case VECSXP:
    case S4SXP: return sizeof(SEXP);
    case CHARSXP: return 1;
    default: return 0;
    }
}

static SEXP new_obj(int type, R_xlen_t n) {
    SEXP s = (SEXP)calloc(1, sizeof *s);
    if (!s) abort();
    s->type = type;
    s->len = n;
    size_t es = elt_size(type);
    if (es) {
        s->data = calloc((size_t)(n > 0 ? n : 1) + (type == CHARSXP), es);
        if (!s->data) abort();
    }
    if (type == STRSXP || type == VECSXP)
        for (R_xlen_t i = 0; i < n; ++i) ((SEXP*)s->data)[i] = type == STRSXP ? NULL : R_NilValue;
    return s;
}

SEXP allocVector(SEXPTYPE t, R_xlen_t n) {
    count_alloc();
    return new_obj((int)t, n);
}

SEXP allocMatrix(SEXPTYPE t, int nrow, int ncol) {
    count_alloc();
    SEXP s = new_obj((int)t, (R_xlen_t)nrow * ncol);
    s->nrow = nrow;
    s->ncol = ncol;
    return s;
}

char* R_alloc(size_t n, int size) {
    count_alloc();
    char* p = (char*)calloc(n ? n : 1, (size_t)size);
    if (!p) abort();
    return p;
}

int R_IsNA(double x) {
    if (!isnan(x)) return 0;
    uint64_t u;
    memcpy(&u, &x, 8);
    return (uint32_t)(u & 0xffffffffu) == 1954u;
}

static void need(SEXP s, int type, const char* what) {
    if (!s || s->type != type) Rf_error("rmini: %s() on an object of type %d", what, s ? s->type : -1);
}

R_xlen_t XLENGTH(SEXP s) { return s->len; }
int LENGTH(SEXP s) { return (int)s->len; }
double* REAL(SEXP s) { need(s, REALSXP, "REAL"); return (double*)s->data; }
int* INTEGER(SEXP s) {
    if (!s || (s->type != INTSXP && s->type != LGLSXP)) Rf_error("rmini: INTEGER() on type %d", s ? s->type : -1);
    return (int*)s->data;
}
int* LOGICAL(SEXP s) {
    if (!s || (s->type != INTSXP && s->type != LGLSXP)) Rf_error("rmini: LOGICAL() on type %d", s ? s->type : -1);
    return (int*)s->data;
}
int TYPEOF(SEXP s) { return s->type; }

int asInteger(SEXP s) {
    if (s->len < 1) return R_NaInt;
    if (s->type == INTSXP || s->type == LGLSXP) return ((int*)s->data)[0];
    if (s->type == REALSXP) {
        double v = ((double*)s->data)[0];
        return isnan(v) ? R_NaInt : (int)v;
    }
    return R_NaInt;
}

double asReal(SEXP s) {
    if (s->len < 1) return NAN;
    if (s->type == REALSXP) return ((double*)s->data)[0];
    if (s->type == INTSXP || s->type == LGLSXP) {
        int v = ((int*)s->data)[0];
        return v == R_NaInt ? NAN : (double)v;
    }
    return NAN;
}

int asLogical(SEXP s) {
    if (s->len < 1) return R_NaInt;
    if (s->type == LGLSXP || s->type == INTSXP) {
        int v = ((int*)s->data)[0];
        return v == R_NaInt ? R_NaInt : v != 0;
    }
    if (s->type == REALSXP) return ((double*)s->data)[0] != 0;
    return R_NaInt;
}

SEXP PROTECT(SEXP s) {
    ++protect_depth;
    return s;
}

void UNPROTECT(int n) {
    protect_depth -= n;
    if (protect_depth < 0) Rf_error("rmini: UNPROTECT below the stack base");
}

SEXP VECTOR_ELT(SEXP s, R_xlen_t i) {
    need(s, VECSXP, "VECTOR_ELT");
    if (i < 0 || i >= s->len) Rf_error("rmini: VECTOR_ELT index %ld of %ld", (long)i, (long)s->len);
    return ((SEXP*)s->data)[i];
}

SEXP SET_VECTOR_ELT(SEXP s, R_xlen_t i, SEXP v) {
    need(s, VECSXP, "SET_VECTOR_ELT");
    if (i < 0 || i >= s->len) Rf_error("rmini: SET_VECTOR_ELT index %ld of %ld", (long)i, (long)s->len);
    ((SEXP*)s->data)[i] = v;
    return v;
}

SEXP STRING_ELT(SEXP s, R_xlen_t i) {
    need(s, STRSXP, "STRING_ELT");
    if (i < 0 || i >= s->len) Rf_error("rmini: STRING_ELT index %ld of %ld", (long)i, (long)s->len);
    return ((SEXP*)s->data)[i];
}

void SET_STRING_ELT(SEXP s, R_xlen_t i, SEXP v) {
    need(s, STRSXP, "SET_STRING_ELT");
    if (i < 0 || i >= s->len) Rf_error("rmini: SET_STRING_ELT index %ld of %ld", (long)i, (long)s->len);
    ((SEXP*)s->data)[i] = v;
}

SEXP mkChar(const char* c) {
    count_alloc();
    size_t n = strlen(c);
    SEXP s = new_obj(CHARSXP, (R_xlen_t)n);
    memcpy(s->data, c, n);
    return s;
}

const char* CHAR(SEXP s) {
    need(s, CHARSXP, "CHAR");
    return (const char*)s->data;
}

SEXP setAttrib(SEXP s, SEXP name, SEXP v) {
    if (name == R_NamesSymbol) {
        s->names = v;
        return v;
    }
    if (name != R_DimNamesSymbol) Rf_error("rmini: only names and dimnames attributes are modelled");
    if (s->nrow == 0 && s->ncol == 0 && s->len != 0) Rf_error("'dimnames' applied to non-array");
    if (v->type != VECSXP || v->len != 2) Rf_error("length of 'dimnames' [%ld] must match that of 'dims' [2]",
                                                   (long)v->len);
    for (int k = 0; k < 2; ++k) {
        SEXP d = ((SEXP*)v->data)[k];
        int want = k == 0 ? s->nrow : s->ncol;
        if (d->type == NILSXP) continue;
        if (d->type != STRSXP) Rf_error("rmini: dimnames[[%d]] is neither NULL nor character", k + 1);
        if (d->len != want)
            Rf_error("length of 'dimnames' [%d] not equal to array extent", k + 1);
        for (R_xlen_t i = 0; i < d->len; ++i)
            if (!((SEXP*)d->data)[i]) Rf_error("rmini: dimnames[[%d]][%ld] unset", k + 1, (long)i + 1);
    }
    s->dimnames = v;
    return v;
}

SEXP R_MakeExternalPtr(void* p, SEXP tag, SEXP prot) {
    count_alloc();
    SEXP s = new_obj(EXTPTRSXP, 1);
    s->addr = p;
    if (n_ext == MAX_EXT) Rf_error("rmini: too many external pointers");
    ext_tab[n_ext++] = s;
    return s;
}

void* R_ExternalPtrAddr(SEXP s) {
    need(s, EXTPTRSXP, "R_ExternalPtrAddr");
    return s->addr;
}

void R_ClearExternalPtr(SEXP s) {
    need(s, EXTPTRSXP, "R_ClearExternalPtr");
    s->addr = NULL;
}

void R_SetExternalPtrAddr(SEXP s, void* p) {
    need(s, EXTPTRSXP, "R_SetExternalPtrAddr");
    s->addr = p;
}

void R_RegisterCFinalizerEx(SEXP s, R_CFinalizer_t f, int onexit) {
    need(s, EXTPTRSXP, "R_RegisterCFinalizerEx");
    s->fin = f;
}

/* ---------------------------------------------------------------- registration */
static const R_CallMethodDef* routines = NULL;

int R_registerRoutines(DllInfo* dll, const void* c, const R_CallMethodDef* call, const void* f, const void* e) {
    routines = call;
    return 1;
}

int R_useDynamicSymbols(DllInfo* dll, int v) { return 1; }

extern void R_init_recoup(DllInfo* dll);

/* ---------------------------------------------------------------- driver API (Python) */
int rmini_init(void) {
    R_init_recoup(NULL);
    return routines ? 0 : -1;
}

/* registered routine by name: its entry point and arity (0 / -1 when absent) */
DL_FUNC rmini_routine(const char* name, int* nargs) {
    for (const R_CallMethodDef* r = routines; r && r->name; ++r)
        if (strcmp(r->name, name) == 0) {
            *nargs = r->numArgs;
            return r->fun;
        }
    *nargs = -1;
    return NULL;
}

typedef SEXP (*F0)(void);
typedef SEXP (*F1)(SEXP);
typedef SEXP (*F4)(SEXP, SEXP, SEXP, SEXP);
typedef SEXP (*F7)(SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP);
typedef SEXP (*F9)(SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP);
typedef SEXP (*F10)(SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP);
typedef SEXP (*F13)(SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP);
typedef SEXP (*F14)(SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP);
typedef SEXP (*F15)(SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP);
typedef SEXP (*F17)(SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP,
                    SEXP, SEXP);
typedef SEXP (*F18)(SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP,
                    SEXP, SEXP, SEXP);
typedef SEXP (*F19)(SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP,
                    SEXP, SEXP, SEXP, SEXP);

/* .Call(name, a[0], ..., a[nargs-1]): 0 and *out on success; 1 and the message
 * (rmini_error) when the routine raised an R error.  *depth: the protect stack depth the
 * routine returned with (R requires 0; after an error R resets it, and so does this). */
int rmini_call(const char* name, int nargs, SEXP* a, SEXP* out, int* depth) {
    int k = 0;
    DL_FUNC f = rmini_routine(name, &k);
    if (!f || k != nargs) {
        snprintf(err_msg, sizeof err_msg, "rmini: no routine %s with %d arguments", name, nargs);
        return 2;
    }
    jmp_buf jb;
    jmp_buf* saved = err_jmp;
    err_jmp = &jb;
    protect_depth = 0;
    if (setjmp(jb)) {
        err_jmp = saved;
        *depth = protect_depth;
        protect_depth = 0;
        return 1;
    }
    SEXP r = R_NilValue;
    switch (nargs) {
    case 1: r = ((F1)f)(a[0]); break;
    case 4: r = ((F4)f)(a[0], a[1], a[2], a[3]); break;
    case 7: r = ((F7)f)(a[0], a[1], a[2], a[3], a[4], a[5], a[6]); break;
    case 9: r = ((F9)f)(a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7], a[8]); break;
    case 10: r = ((F10)f)(a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7], a[8], a[9]); break;
    case 13: r = ((F13)f)(a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7], a[8], a[9], a[10], a[11], a[12]); break;
    case 14:
        r = ((F14)f)(a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7], a[8], a[9], a[10], a[11], a[12], a[13]);
        break;
    case 15:
        r = ((F15)f)(a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7], a[8], a[9], a[10], a[11], a[12], a[13], a[14]);
        break;
    case 17:
        r = ((F17)f)(a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7], a[8], a[9], a[10], a[11], a[12], a[13], a[14],
                     a[15], a[16]);
        break;
    case 18:
        r = ((F18)f)(a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7], a[8], a[9], a[10], a[11], a[12], a[13], a[14],
                     a[15], a[16], a[17]);
        break;
    case 19:
        r = ((F19)f)(a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7], a[8], a[9], a[10], a[11], a[12], a[13], a[14],
                     a[15], a[16], a[17], a[18]);
        break;
    default:
        err_jmp = saved;
        snprintf(err_msg, sizeof err_msg, "rmini: arity %d not modelled", nargs);
        return 2;
    }
    err_jmp = saved;
    *depth = protect_depth;
    protect_depth = 0;
    *out = r;
    return 0;
}

const char* rmini_error(void) { return err_msg; }
void rmini_fail_alloc_after(long k) { fail_after = k; }

/* R's garbage collector, eventually: every finalizer runs once */
int rmini_run_finalizers(void) {
    int ran = 0;
    for (int i = 0; i < n_ext; ++i)
        if (ext_tab[i]->fin) {
            R_CFinalizer_t f = ext_tab[i]->fin;
            ext_tab[i]->fin = NULL;
            f(ext_tab[i]);
            ++ran;
        }
    return ran;
}

/* external pointers that still hold an address */
int rmini_live_handles(void) {
    int n = 0;
    for (int i = 0; i < n_ext; ++i) n += ext_tab[i]->addr != NULL;
    return n;
}

/* live handles no finalizer will ever release (a leak) */
int rmini_unguarded_handles(void) {
    int n = 0;
    for (int i = 0; i < n_ext; ++i) n += ext_tab[i]->addr != NULL && ext_tab[i]->fin == NULL;
    return n;
}

SEXP rmini_strings(int n, const char** c);

/* S4 objects: named slots (a list of n SEXPs with a names vector); symbols are CHARSXPs */
SEXP install(const char* name) { return mkChar(name); }
int IS_S4_OBJECT(SEXP s) { return s->type == S4SXP; }
static SEXP slot_of(SEXP obj, SEXP sym) {
    if (obj->type != S4SXP || !obj->names) return NULL;
    SEXP* slots = (SEXP*)obj->data;
    SEXP* nm = (SEXP*)obj->names->data;
    for (R_xlen_t i = 0; i < obj->len; ++i)
        if (strcmp((const char*)nm[i]->data, (const char*)sym->data) == 0) return slots[i];
    return NULL;
}
int R_has_slot(SEXP obj, SEXP sym) { return slot_of(obj, sym) != NULL; }
SEXP R_do_slot(SEXP obj, SEXP sym) {
    SEXP v = slot_of(obj, sym);
    if (!v) Rf_error("no slot of name \"%s\" for this object", (const char*)sym->data);
    return v;
}
SEXP rmini_s4(int n, const char** names, const SEXP* slots) {
    SEXP s = new_obj(S4SXP, n);
    for (int i = 0; i < n; ++i) ((SEXP*)s->data)[i] = slots[i];
    s->names = rmini_strings(n, names);
    return s;
}

SEXP rmini_vector(int type, R_xlen_t n, const void* src) {
    SEXP s = new_obj(type, n);
    if (src && n > 0) memcpy(s->data, src, (size_t)n * elt_size(type));
    return s;
}

SEXP rmini_string(const char* c) {
    SEXP s = new_obj(STRSXP, 1);
    size_t n = strlen(c);
    SEXP ch = new_obj(CHARSXP, (R_xlen_t)n);
    memcpy(ch->data, c, n);
    ((SEXP*)s->data)[0] = ch;
    return s;
}

SEXP rmini_strings(int n, const char** c) {
    SEXP s = new_obj(STRSXP, n);
    for (int i = 0; i < n; ++i) {
        size_t k = strlen(c[i]);
        SEXP ch = new_obj(CHARSXP, (R_xlen_t)k);
        memcpy(ch->data, c[i], k);
        ((SEXP*)s->data)[i] = ch;
    }
    return s;
}

SEXP rmini_list(int n, const SEXP* elts) {
    SEXP s = new_obj(VECSXP, n);
    for (int i = 0; i < n; ++i) ((SEXP*)s->data)[i] = elts[i];
    return s;
}

int rmini_type(SEXP s) { return s->type; }
R_xlen_t rmini_length(SEXP s) { return s->len; }
void* rmini_data(SEXP s) { return s->data; }
SEXP rmini_names(SEXP s) { return s->names ? s->names : R_NilValue; }
SEXP rmini_dimnames(SEXP s) { return s->dimnames ? s->dimnames : R_NilValue; }
int rmini_dim(SEXP s, int k) { return k == 0 ? s->nrow : s->ncol; }
SEXP rmini_nil(void) { return R_NilValue; }
