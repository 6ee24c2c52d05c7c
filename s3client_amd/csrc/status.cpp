// status.cpp -- the C-ABI's last-error string and version (include/s3hash.h).
#include "status.hpp"

#include <cstdarg>
#include <cstdio>

#include "../../include/s3hash.h"

namespace s3h::host {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

}  // namespace s3h::host

extern "C" {

const char* s3h_last_error(void) { return s3h::host::g_err.c_str(); }
int s3h_api_version(void) { return S3H_API_VERSION; }

}  // extern "C"
