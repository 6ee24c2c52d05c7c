"""AUTO's kernel policy: "efficiency" runs skewp where
"throughput" runs the shared-SIMD skews kernel (4,097 - 32 x CUs parts), "power" (the default)
runs skews there only when the board's power cap (sysfs hwmon power1_cap) is at least the
1,500 W skews needs to hold its clock; same digests; elsewhere every policy agrees."""
import os
import subprocess
import sys

import numpy as np
import pytest

import s3client_amd as s3

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_policy_switch_cpu():
    prev = s3.kernel_policy("efficiency")
    try:
        assert s3.kernel_policy("throughput") == "efficiency"
        assert s3.kernel_policy("power") == "throughput"
        assert s3._native.lib().s3h_kernel_policy(7, None) == -1
    finally:
        s3.kernel_policy(prev)
    code = "import s3client_amd as s3;print(s3.kernel_policy('throughput'))"
    env0 = {k: v for k, v in os.environ.items()
            if k not in ("S3H_PREFER_EFFICIENCY", "S3H_KERNEL_POLICY")}
    for env, want in (({}, "power"),
                      ({"S3H_PREFER_EFFICIENCY": "1"}, "efficiency"),
                      ({"S3H_PREFER_EFFICIENCY": "0"}, "power"),
                      ({"S3H_KERNEL_POLICY": "throughput"}, "throughput"),
                      ({"S3H_KERNEL_POLICY": "efficiency"}, "efficiency")):
        r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True,
                           env={**env0, **env}, timeout=60)
        assert r.returncode == 0 and r.stdout.strip() == want, r.stderr


@pytest.mark.gpu
def test_efficiency_policy_picks_skewp_same_digests(torch_cuda, oracle):
    torch = torch_cuda
    rng = np.random.default_rng(61)
    cap = s3.device_power_cap(0)
    print("board power cap", cap, "W")
    k_pow = "skewp" if 0 < cap < 1500 else "skews"
    cases = {8192: ("skews", "skewp", k_pow), 1024: ("skew", "skew", "skew"),
             30000: ("pair", "pair", "pair")}
    for n, (k_thr, k_eff, k_pw) in cases.items():
        lens = rng.integers(0, 1500, n).astype(np.uint64)
        offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
        host = rng.integers(0, 256, int(lens.sum()) + 64, dtype=np.uint8)
        data = torch.from_numpy(host).cuda()
        want = oracle.batch(host, offs, lens)
        prev = s3.kernel_policy("throughput")
        try:
            for policy, kname in (("throughput", k_thr), ("efficiency", k_eff), ("power", k_pw)):
                s3.kernel_policy(policy)
                with s3.Plan(offs, lens) as p:
                    assert p.info()["kernel"] == kname, (n, policy)
                got = s3.sha256_batch_device(data, offs, lens).cpu().numpy().view(np.uint32)
                assert np.array_equal(got, want), (n, policy)
        finally:
            s3.kernel_policy(prev)
