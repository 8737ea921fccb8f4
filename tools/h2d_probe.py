import time, torch, numpy as np
torch.cuda.init(); x=torch.zeros(1,device='cuda')
for n in (16, 16000*8, 1<<20, 4<<20):
    a=np.random.rand(n).astype(np.float32)
    for mode in ("pageable","pinned"):
        ts=[]
        for i in range(10):
            b=np.random.rand(n).astype(np.float32)   # fresh buffer each time
            torch.cuda.synchronize(); t=time.perf_counter()
            t0=torch.from_numpy(b)
            if mode=="pinned": t0=t0.pin_memory(); y=t0.to('cuda',non_blocking=True); torch.cuda.synchronize()
            else: y=t0.to('cuda')
            ts.append((time.perf_counter()-t)*1e3)
        print(n*4, mode, "ms median", round(sorted(ts)[5],3), "first", round(ts[0],3))
