/* minimal R_ext/Rdynload.h for tests/rstub (see README.md) */
#pragma once
typedef void *(*DL_FUNC)(void);
typedef struct {
  const char *name;
  DL_FUNC fun;
  int numArgs;
} R_CallMethodDef;
typedef struct DllInfo DllInfo;
int R_registerRoutines(DllInfo *info, const void *c, const R_CallMethodDef *call, const void *f,
                       const void *e);
