"""The host path's concurrent machinery under ThreadSanitizer and AddressSanitizer (CPU; VERDICT
r5 item 4).

tests/cpp/host_concurrency_test.cpp links the HIP-free units exactly as they ship -- the
per-device merge queue (host_queue.hpp), the copy-thread pool (copy_pool.hpp), the CPU route and
the split route's driver (route_plan.cpp), topology.cpp, status.cpp and the CPU drop-in -- with
a fake device executor that stages every part through a CopyPool, hashes it with the drop-in,
sleeps, fails or throws.  32 concurrent callers mix algorithm sets (SHA-256, MD5, both), slice
sizes, memory parts and file ranges and injected faults; 8 run the split driver at once with a
fake GPU side (memory parts and file ranges, file descriptors counted); 16 run the CPU route.
Each caller must receive exactly its own status, message and digests.  Built twice with g++
(-fsanitize=thread; -fsanitize=address,undefined) and run; any sanitizer report fails the test.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRCS = ["tests/cpp/host_concurrency_test.cpp", "s3client_amd/csrc/status.cpp",
        "s3client_amd/csrc/topology.cpp", "s3client_amd/csrc/route_plan.cpp",
        "s3client_amd/csrc/cpu/lib_hash.cpp", "s3client_amd/csrc/cpu/lib_md5.cpp"]
BUILDS = {
    # GCC 11's libtsan misses pthread_cond_clockwait (tests/cpp/tsan_compat.h)
    "tsan": (["-fsanitize=thread", "-include", "tests/cpp/tsan_compat.h"],
             {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"}),
    "asan": (["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
              "-fno-omit-frame-pointer"],
             {"ASAN_OPTIONS": "detect_leaks=1:halt_on_error=1",
              "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"}),
}


@pytest.mark.parametrize("kind", sorted(BUILDS))
def test_host_concurrency_under_sanitizer(kind, tmp_path):
    flags, env = BUILDS[kind]
    exe = os.path.join(ROOT, "tests", "cpp", "build", f"host_concurrency_{kind}")
    os.makedirs(os.path.dirname(exe), exist_ok=True)
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-pthread", *flags, "-Iinclude", *SRCS, "-o", exe]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    r = subprocess.run([exe, str(tmp_path)], cwd=ROOT, capture_output=True, text=True, timeout=600,
                       env={**os.environ, **env})
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-6000:]
    assert "WARNING: ThreadSanitizer" not in out and "ERROR: AddressSanitizer" not in out, out[-6000:]
    assert "runtime error" not in out, out[-6000:]  # UBSan
    assert "host concurrency ok" in r.stdout
    assert "failed as injected" in r.stdout and "fds" in r.stdout
