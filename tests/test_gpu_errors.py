"""A launch that faults must fail its call, never return wrong digests (the reference's
sha256::sha256, lib/hash/sha256.cpp:147-160, always returns the message's digest).

The flag-synchronised kernels (two-group skew, shared-SIMD skew, dual-digest group kernels)
bound every producer/consumer wait; a wait that times out ORs kErrSyncTimeout into the plan's
device error word (sha256_kernels.hip flag_wait_ge) and every host entry point reads the word
(capi.hip plan_check).  tests/cpp/build/libs3hash_stall.so (Makefile target `stall`) is the product
source built with producers that stop publishing after their first step: every consumer wait
times out, and every entry point must report S3H_EHIP.  The same probe against the product
library must succeed with the oracle's digests.  Each library runs in its own child process
(S3H_LIBRARY is read when s3client_amd is imported)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STALL = os.path.join(ROOT, "tests", "cpp", "build", "libs3hash_stall.so")
PROBE = os.path.join(ROOT, "tests", "gpu_stall_probe.py")
S3H_EHIP = -3


def _probe(lib=None):
    env = dict(os.environ)
    env.pop("S3H_LIBRARY", None)
    if lib:
        env["S3H_LIBRARY"] = lib
    r = subprocess.run([sys.executable, PROBE], capture_output=True, text=True, env=env,
                       cwd=ROOT, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


PRODUCT = os.path.join(ROOT, "s3client_amd", "lib", "libs3hash.so")


def exported_abi(path: str) -> set:
    """The C-ABI symbols (s3h_*) a library exports (nm -D --defined-only)."""
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True,
                         check=True).stdout
    return {l.split()[-1] for l in out.splitlines() if l.split() and l.split()[-1].startswith("s3h_")}


def stale_stall_library() -> str:
    """"" when the forced-fault build exports exactly the product's C-ABI; otherwise why not
    (a stale prebuilt stall library once lacked a new entry point and failed a GPU run)."""
    want, got = exported_abi(PRODUCT), exported_abi(STALL)
    if want == got:
        return ""
    return (f"{STALL} is stale -- rebuild it with `make stall`: missing {sorted(want - got)}, "
            f"extra {sorted(got - want)}")


@pytest.mark.gpu
def test_forced_stall_fails_every_entry_point():
    if not os.path.exists(STALL):  # test-only build, not part of `make all`
        pytest.skip("forced-fault library not built: run `make stall` (__graft_entry__.build() does)")
    stale = stale_stall_library()
    assert not stale, stale
    res = _probe(STALL)
    assert res.pop("library").endswith("libs3hash_stall.so")
    assert res.pop("control_1000_parts") == 0  # barrier kernels are unaffected
    assert len(res) == 16, sorted(res)
    for name, out in res.items():
        assert out != 0, f"{name}: succeeded although every consumer wait timed out"
        assert isinstance(out, list), f"{name}: {out}"
        code, msg = out
        assert code == S3H_EHIP and "synchronisation timeout" in msg, (name, msg)


@pytest.mark.gpu
def test_product_library_passes_the_same_probe():
    res = _probe()
    assert res.pop("library").endswith(os.path.join("lib", "libs3hash.so"))
    assert all(v == 0 for v in res.values()), {k: v for k, v in res.items() if v != 0}


def test_stall_library_exports_the_product_abi():
    """CPU: the forced-fault library the GPU test loads is built from the same source as the
    product (Makefile `stall`, rebuilt whenever capi.hip changes) -- same exported C-ABI."""
    if not (os.path.exists(STALL) and os.path.exists(PRODUCT)):
        pytest.skip("libraries not built")
    assert not stale_stall_library(), stale_stall_library()
    assert len(exported_abi(PRODUCT)) > 50

