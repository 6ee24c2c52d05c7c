import os, sys, time
os.environ["S3H_TRACE_HOST"] = "1"
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np, torch
import s3client_amd as s3
from s3client_amd import hashing as H
n, L = 1024, 1 << 20
host = torch.empty(n * L, dtype=torch.uint8, pin_memory=True)
h = host.numpy(); h[:] = 1
views = [h[i * L:(i + 1) * L] for i in range(n)]
s3.sha256_batch_host(views)
for _ in range(3):
    t = time.perf_counter(); a = H._host_parts(views); t1 = time.perf_counter()
    s3.sha256_batch_host(views); t2 = time.perf_counter()
    print(f"marshal {1e3*(t1-t):.3f} ms, call {1e3*(t2-t1):.3f} ms", flush=True)
