import sys, hashlib, struct
sys.path.insert(0, '.')
import numpy as np, torch
import s3client_amd as s3
for L in (0, 3, 100, 1000):
    host = np.arange(max(L,1), dtype=np.uint8)
    d = torch.from_numpy(host).cuda()
    for k in ("skew", "quad"):
        out = s3.sha256_batch_device(d, [0], [L], kernel=k).cpu().numpy().view(np.uint32)
        print(L, k, [hex(x) for x in out[0]])
    want = struct.unpack("<8I", hashlib.sha256(host[:L].tobytes()).digest())
    print(L, "want", [hex(x) for x in want])
