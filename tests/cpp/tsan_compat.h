// tsan_compat.h -- force-included into the ThreadSanitizer build of host_concurrency_test.cpp
// only.  GCC 11's libtsan does not intercept pthread_cond_clockwait, which libstdc++ uses for
// condition_variable::wait_for / wait_until when glibc has it; the sanitizer then loses track
// of the mutex the wait releases and re-acquires and reports a "double lock" that is not there
// (GCC bug 101978).  Without this macro libstdc++ waits through pthread_cond_timedwait, which
// the sanitizer does intercept.
#include <bits/c++config.h>
#undef _GLIBCXX_USE_PTHREAD_COND_CLOCKWAIT
