/* tests/rstub/rstub.c -- R C API emulation + ctypes driver for the .Call shim
 * (test infrastructure; see README.md). */
#include <setjmp.h>
#include <stdarg.h>

#include "R.h"
#include "R_ext/Rdynload.h"
#include "Rinternals.h"

static struct SEXPREC nil = {NILSXP, 0, 0, 0, NULL};
SEXP R_NilValue = &nil;

static void **pool = NULL;
static size_t npool = 0, cappool = 0;
static void *track(void *p) {
  if (npool == cappool) {
    cappool = cappool ? 2 * cappool : 1024;
    pool = (void **)realloc(pool, cappool * sizeof(void *));
  }
  pool[npool++] = p;
  return p;
}
void rs_reset(void) {
  for (size_t i = 0; i < npool; ++i) free(pool[i]);
  npool = 0;
}

static jmp_buf *jb = NULL;
static char errbuf[1024];
void error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(errbuf, sizeof(errbuf), fmt, ap);
  va_end(ap);
  if (jb) longjmp(*jb, 1);
  fprintf(stderr, "R error outside a call: %s\n", errbuf);
  abort();
}
const char *rs_error(void) { return errbuf; }

static size_t elt_size(int type) {
  switch (type) {
    case INTSXP: case LGLSXP: return sizeof(int);
    case REALSXP: return sizeof(double);
    case STRSXP: case VECSXP: return sizeof(SEXP);
    case CHARSXP: return 1;
    default: return 0;
  }
}
SEXP allocVector(int type, R_xlen_t n) {
  SEXP x = (SEXP)track(calloc(1, sizeof(struct SEXPREC)));
  x->type = type;
  x->len = n;
  x->nrow = (int)n;
  x->ncol = 1;
  x->data = track(calloc((size_t)(n > 0 ? n : 1) + (type == CHARSXP), elt_size(type)));
  if (type == STRSXP || type == VECSXP)
    for (R_xlen_t i = 0; i < n; ++i) ((SEXP *)x->data)[i] = R_NilValue;
  return x;
}
SEXP allocMatrix(int type, int nrow, int ncol) {
  SEXP x = allocVector(type, (R_xlen_t)nrow * ncol);
  x->nrow = nrow;
  x->ncol = ncol;
  return x;
}
SEXP ScalarLogical(int v) {
  SEXP x = allocVector(LGLSXP, 1);
  ((int *)x->data)[0] = v;
  return x;
}
SEXP ScalarReal(double v) {
  SEXP x = allocVector(REALSXP, 1);
  ((double *)x->data)[0] = v;
  return x;
}
SEXP mkChar(const char *s) {
  size_t n = strlen(s);
  SEXP x = allocVector(CHARSXP, (R_xlen_t)n);
  memcpy(x->data, s, n);
  return x;
}
int TYPEOF(SEXP x) { return x->type; }
int length(SEXP x) { return (int)x->len; }
int *INTEGER(SEXP x) { return (int *)x->data; }
int asInteger(SEXP x) {
  if (x->len < 1) return NA_LOGICAL;
  if (x->type == REALSXP) return (int)((double *)x->data)[0];
  return ((int *)x->data)[0];
}
double *REAL(SEXP x) { return (double *)x->data; }
const char *CHAR(SEXP x) { return (const char *)x->data; }
SEXP STRING_ELT(SEXP x, R_xlen_t i) { return ((SEXP *)x->data)[i]; }
void SET_STRING_ELT(SEXP x, R_xlen_t i, SEXP v) { ((SEXP *)x->data)[i] = v; }
SEXP VECTOR_ELT(SEXP x, R_xlen_t i) { return ((SEXP *)x->data)[i]; }
SEXP SET_VECTOR_ELT(SEXP x, R_xlen_t i, SEXP v) { ((SEXP *)x->data)[i] = v; return v; }
SEXP PROTECT(SEXP x) { return x; }
void UNPROTECT(int n) { (void)n; }
char *R_alloc(size_t n, int size) { return (char *)track(calloc(n ? n : 1, (size_t)size)); }

static const R_CallMethodDef *routines = NULL;
int R_registerRoutines(DllInfo *info, const void *c, const R_CallMethodDef *call, const void *f,
                       const void *e) {
  (void)info; (void)c; (void)f; (void)e;
  routines = call;
  return 1;
}

/* ---- ctypes driver */
void R_init_kmer_spans(DllInfo *info);
int rs_init(void) { R_init_kmer_spans(NULL); return routines != NULL; }
int rs_nroutines(void) { int n = 0; while (routines && routines[n].name) ++n; return n; }
const char *rs_routine_name(int i) { return routines[i].name; }
int rs_routine_nargs(int i) { return routines[i].numArgs; }

SEXP rs_str(int n, const char **s, const int *lens) {
  SEXP x = allocVector(STRSXP, n);
  for (int i = 0; i < n; ++i) {
    SEXP c = allocVector(CHARSXP, lens[i]);
    memcpy(c->data, s[i], (size_t)lens[i]);
    SET_STRING_ELT(x, i, c);
  }
  return x;
}
SEXP rs_int(int n, const int *v) { SEXP x = allocVector(INTSXP, n); memcpy(x->data, v, (size_t)n * sizeof(int)); return x; }
SEXP rs_real(int n, const double *v) { SEXP x = allocVector(REALSXP, n); memcpy(x->data, v, (size_t)n * sizeof(double)); return x; }

typedef SEXP (*fn1)(SEXP);
typedef SEXP (*fn2)(SEXP, SEXP);
typedef SEXP (*fn5)(SEXP, SEXP, SEXP, SEXP, SEXP);
SEXP rs_call(const char *name, SEXP *a, int nargs) {
  const R_CallMethodDef *m = NULL;
  for (int i = 0; routines && routines[i].name; ++i)
    if (!strcmp(routines[i].name, name)) m = &routines[i];
  errbuf[0] = 0;
  if (!m || m->numArgs != nargs) { snprintf(errbuf, sizeof(errbuf), "no routine %s/%d", name, nargs); return NULL; }
  jmp_buf here;
  jb = &here;
  SEXP r = NULL;
  if (setjmp(here) == 0) {
    if (nargs == 1) r = ((fn1)m->fun)(a[0]);
    else if (nargs == 2) r = ((fn2)m->fun)(a[0], a[1]);
    else if (nargs == 5) r = ((fn5)m->fun)(a[0], a[1], a[2], a[3], a[4]);
  }
  jb = NULL;
  return r;
}
int rs_type(SEXP x) { return x->type; }
long rs_length(SEXP x) { return (long)x->len; }
int rs_nrow(SEXP x) { return x->nrow; }
int rs_ncol(SEXP x) { return x->ncol; }
SEXP rs_elt(SEXP x, long i) { return ((SEXP *)x->data)[i]; }
void *rs_data(SEXP x) { return x->data; }
