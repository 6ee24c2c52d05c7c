"""Same-box A/B: C2 (1,024 x 8 MiB) from one pageable host buffer through the batch host path
(s3h_sha256_batch_host) and as 1,024 streamed objects appended in 64 KiB / 1 MiB chunks
(s3h_stream_update_host), with a new stream object per pass or one object reused (final()
restarts it).  Rounds alternate; one JSON line with each variant's GiB/s."""
import sys, os, time, json
sys.path.insert(0, os.getcwd())
import numpy as np, torch
import s3client_amd as s3
MIB=1<<20; n=1024; L=8*MIB
lens=np.full(n,L,dtype=np.uint64); offs=np.arange(n,dtype=np.uint64)*np.uint64(L)
dev=torch.empty(n*L,dtype=torch.uint8,device="cuda"); s3.generate_parts(dev,offs,lens,np.arange(n),20241008)
host=torch.empty(n*L,dtype=torch.uint8); host.copy_(dev); del dev; torch.cuda.empty_cache()
gib=n*L/2**30
ref=s3.sha256_batch_host(s3.BufferParts(host,offs,lens))
def batch():
    return s3.sha256_batch_host(s3.BufferParts(host,offs,lens))
def stream(cb, reuse):
    keep = s3.Stream(n) if reuse else None
    def f():
        st = keep or s3.Stream(n)
        for k in range(L//cb):
            st.update(s3.BufferParts(host, offs+np.uint64(k*cb), np.full(n,cb,dtype=np.uint64)))
        out = st.final()
        if not reuse:
            st.close()
        return out
    return f
fns={"batch":batch,"stream_64k_new_object":stream(64<<10, False),"stream_1m_new_object":stream(1<<20, False),
     "stream_64k_reused_object":stream(64<<10, True),"stream_1m_reused_object":stream(1<<20, True)}
res={k:[] for k in fns}
for k,f in fns.items(): assert np.array_equal(f(),ref), k
for r in range(4):
    for k,f in fns.items():
        t0=time.perf_counter(); out=f(); res[k].append(round(gib/(time.perf_counter()-t0),2))
        assert np.array_equal(out,ref)
print(json.dumps({k:{"runs":v,"median":float(np.median(v))} for k,v in res.items()}))
