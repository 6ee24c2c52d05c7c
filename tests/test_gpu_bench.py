"""bench.py's multi-GPU plumbing on the GPU box (pytest -m gpu): `python bench.py --gpus 2`
with NO external launcher starts its two ranks itself (a child torch.distributed.run), and
rank 0's single JSON line carries both ranks' devices, per-rank fixture parity and no errors.
On a one-GPU box the two ranks share the device (S3H_BENCH_SHARE_GPU=1, the rehearsal mode);
the driver's N-GPU runs use the same code with one device per rank."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_self_launches_two_ranks(torch_cuda):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["S3H_BENCH_SHARE_GPU"] = "1"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2",
                        "--warmup", "1", "--no-c4", "--no-host-resident"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and "errors" not in line, line.get("errors")
    assert [d["rank"] for d in line["devices"]] == [0, 1]
    assert all(d["pci_bus_id"].count(":") == 2 and d["arch"].startswith("gfx950") for d in line["devices"])
    assert line["distinct_devices"] == 1  # shared on purpose here
    per = line["parity"]["per_rank"]
    assert [p["rank"] for p in per] == [0, 1] and all(p["fixtures_checked"] >= 4 for p in per)
    assert line["parity"]["mismatches"] == 0
    assert "timed 2 steps" in line["phases_s"]
    assert "[bench rank 0] timed 2 steps" in r.stderr
