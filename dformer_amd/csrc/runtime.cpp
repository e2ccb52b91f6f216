// Host-side runtime of libdformer_hip.so: error reporting and ABI version.
#include <stdarg.h>
#include <stdio.h>

#include "../../include/dformer_hip.h"

static thread_local char g_err[512] = "";

void dfm_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

extern "C" const char* dfm_last_error(void) { return g_err; }
extern "C" int dfm_abi_version(void) { return 1; }
