/* minimal Rinternals.h for tests/rstub (see README.md) */
#pragma once
#include <stddef.h>
typedef ptrdiff_t R_xlen_t;
typedef struct SEXPREC *SEXP;
struct SEXPREC {
  int type;
  R_xlen_t len;
  int nrow, ncol;
  void *data;
};
#define NILSXP 0
#define LGLSXP 10
#define CHARSXP 9
#define INTSXP 13
#define REALSXP 14
#define STRSXP 16
#define VECSXP 19
extern SEXP R_NilValue;
int TYPEOF(SEXP x);
int length(SEXP x);
int *INTEGER(SEXP x);
double *REAL(SEXP x);
const char *CHAR(SEXP x);
SEXP STRING_ELT(SEXP x, R_xlen_t i);
void SET_STRING_ELT(SEXP x, R_xlen_t i, SEXP v);
SEXP VECTOR_ELT(SEXP x, R_xlen_t i);
SEXP SET_VECTOR_ELT(SEXP x, R_xlen_t i, SEXP v);
SEXP allocVector(int type, R_xlen_t n);
SEXP allocMatrix(int type, int nrow, int ncol);
SEXP mkChar(const char *s);
#define NA_LOGICAL (-2147483647 - 1)
SEXP ScalarLogical(int x);
SEXP ScalarReal(double x);
int asInteger(SEXP x);
SEXP PROTECT(SEXP x);
void UNPROTECT(int n);
/* as in R, error() is a macro for Rf_error (glibc also exports error(3)) */
#define error Rf_error
void Rf_error(const char *fmt, ...) __attribute__((noreturn));
char *R_alloc(size_t n, int size);
