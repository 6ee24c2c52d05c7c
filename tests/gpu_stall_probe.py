"""Child process of tests/test_gpu_errors.py: every entry point that can run a
flag-synchronised kernel, called through whichever libs3hash.so S3H_LIBRARY names, with the
outcome of each call printed as one JSON object ({name: 0 | [status, message]}).

Run against tests/cpp/build/libs3hash_stall.so (producers stop publishing after one step, so
every consumer wait times out) every call must fail with S3H_EHIP; against the product library
the same calls must succeed with the oracle's digests."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import s3client_amd as s3  # noqa: E402
from s3client_amd import _native  # noqa: E402
from tests.oracle_lib import Oracle  # noqa: E402


def main():
    orc = Oracle()
    rng = np.random.default_rng(11)
    res = {"library": os.path.relpath(_native.LIB_PATH, ROOT)}

    def parts(n, lo=0, hi=2000):
        lens = rng.integers(lo, hi, n)
        offs = np.concatenate([[0], np.cumsum(lens + 5)[:-1]])
        host = rng.integers(0, 256, int(offs[-1] + lens[-1]) + 64, dtype=np.uint8)
        return host, offs, lens, torch.from_numpy(host).cuda()

    def outcome(name, fn, want=None):
        try:
            got = fn()
        except s3.S3HashError as e:
            res[name] = [e.code, str(e)]
            return
        if want is not None and not np.array_equal(np.asarray(got).view(np.uint32).reshape(want.shape), want):
            res[name] = "WRONG DIGESTS RETURNED AS SUCCESS"
            return
        res[name] = 0

    # 3,000 parts: two-group skew kernel (2,049-4,096); 5,000: shared-SIMD skew (4,097-8,192)
    # -- under the "throughput" policy: the default "power" policy runs skewp (barrier
    # synchronised, not stalled by this build) there on a board capped below 1.5 kW
    s3.kernel_policy("throughput")
    for n, tag in ((3000, "skew_pairs"), (5000, "skews")):
        host, offs, lens, data = parts(n)
        want = orc.batch(host, offs, lens)
        outcome(f"batch_device_{tag}",
                lambda: s3.sha256_batch_device(data, offs, lens).cpu().numpy(), want)

        def plan_then_status():
            plan = s3.Plan(offs, lens)
            out = torch.zeros((n, 8), dtype=torch.int32, device="cuda")
            plan.launch(data, out)  # asynchronous: returns OK either way
            plan.status()           # the launch's verdict
            plan.close()
            return out.cpu().numpy()
        outcome(f"plan_status_{tag}", plan_then_status, want)
        views = [host[int(o):int(o) + int(L)] for o, L in zip(offs, lens)]
        outcome(f"batch_host_{tag}", lambda: s3.sha256_batch_host(views, ndevices=1), want)
        # verification against the true digests: success must mean "no part differs"
        ok = np.zeros((n, 1), dtype=np.uint32)
        outcome(f"verify_host_{tag}",
                lambda: s3.verify_batch_host(views, want, ndevices=1).astype(np.uint32)[:, None], ok)
        exp = torch.from_numpy(want.view(np.int32)).cuda()
        outcome(f"verify_device_{tag}",
                lambda: s3.verify_batch_device(data, offs, lens, exp)[1].cpu().numpy()
                .astype(np.uint32)[:, None], ok)
        m5 = orc.md5_batch(host, offs, lens)
        outcome(f"dual_device_{tag}",
                lambda: np.concatenate([x.cpu().numpy().view(np.uint32) for x in
                                        s3.sha256_md5_batch_device(data, offs, lens)], axis=1),
                np.concatenate([want, m5], axis=1))
        outcome(f"dual_host_{tag}",
                lambda: np.concatenate(s3.sha256_md5_batch_host(views, ndevices=1), axis=1),
                np.concatenate([want, m5], axis=1))

        def streamed():
            st = s3.Stream(n)
            half = [v[:len(v) // 2] for v in views]
            rest = [v[len(v) // 2:] for v in views]
            st.update(half)
            st.update(rest)
            d = st.final()
            st.close()
            return d
        outcome(f"stream_host_{tag}", streamed, want)
    # control: 1,000 parts run the barrier-synchronised skew kernel, which cannot time out
    host, offs, lens, data = parts(1000)
    outcome("control_1000_parts", lambda: s3.sha256_batch_device(data, offs, lens).cpu().numpy(),
            orc.batch(host, offs, lens))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
