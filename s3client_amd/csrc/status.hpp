// status.hpp -- error reporting shared by every translation unit of libs3hash.so: the C-ABI's
// thread-local last-error string (s3h_last_error) and the wall clock the host path and the
// route model time themselves with.  HIP-free (the host-concurrency sanitizer build links it).
#pragma once
#include <chrono>
#include <string>

namespace s3h::host {

// Last error message of the calling thread (s3h_last_error returns it).
extern thread_local std::string g_err;

// Sets g_err from a printf format and returns `code` (an s3h_status).
int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

// Seconds on the steady clock (an arbitrary epoch): for intervals only.
inline double wall_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

inline double seconds_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

}  // namespace s3h::host
