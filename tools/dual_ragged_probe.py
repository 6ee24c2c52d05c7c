import sys, time, json, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np, torch
import s3client_amd as s3
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "tools"))
from route_gpu_side_probe import gen, best
MIB = 1 << 20
rng = np.random.default_rng(606)
lens = rng.integers(1 * MIB, 16 * MIB, 300); lens[:4] = [0, 1, 55, 64]
host, offs, lens = gen(torch, s3, lens)
data = torch.from_numpy(host).cuda()
def row(name, fn):
    t, ts = best(fn); print(json.dumps({"case": name, "s": t, "all": ts}), flush=True)
row("device sha ragged300", lambda: (s3.sha256_batch_device(data, offs, lens), torch.cuda.synchronize()))
row("device dual ragged300", lambda: (s3.sha256_md5_batch_device(data, offs, lens), torch.cuda.synchronize()))
row("device md5 ragged300", lambda: (s3.md5_batch_device(data, offs, lens), torch.cuda.synchronize()))
with s3.Plan(offs, lens) as p: print("sha plan", p.info(), flush=True)
pb = torch.empty(host.size, dtype=torch.uint8, pin_memory=True); pb.numpy()[:] = host
h = pb.numpy(); views = [h[int(o):int(o)+int(L)] for o, L in zip(offs, lens)]
row("host sha ragged300", lambda: s3.sha256_batch_host(views))
row("host md5 ragged300", lambda: s3.md5_batch_host(views))
row("host dual ragged300", lambda: s3.sha256_md5_batch_host(views))
for sb in (256 << 10, 1 << 20, 4 << 20):
    row(f"host dual ragged300 slice {sb}", lambda: s3.sha256_md5_batch_host(views, slice_bytes=sb))
eq = np.full(300, 16 * MIB, dtype=np.uint64); eo = np.arange(300, dtype=np.uint64) * np.uint64(16 * MIB)
d2 = torch.empty(300 * 16 * MIB, dtype=torch.uint8, device="cuda")
row("device dual equal300x16MiB", lambda: (s3.sha256_md5_batch_device(d2, eo, eq), torch.cuda.synchronize()))
row("device sha equal300x16MiB", lambda: (s3.sha256_batch_device(d2, eo, eq), torch.cuda.synchronize()))
