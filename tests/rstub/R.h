/* minimal R.h for tests/rstub (see README.md) */
#pragma once
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#define Rprintf printf
