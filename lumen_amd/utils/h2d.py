"""Small host -> device uploads that never stall the host.

A copy from pageable host memory (``torch.tensor(list).to("cuda")``, ``torch.from_numpy(a).to(dev)``
and even ``.to(dev, non_blocking=True)`` of a pageable tensor) makes HIP stage the bytes through
its own pinned bounce buffer: the calling thread blocks until the stream has drained up to the
copy -- measured 6.4 ms of host time for a 64 KiB copy behind 17.7 ms of queued GEMMs
(tools/probes/h2d_stall.py) versus 0.06 ms from pinned memory.  In a pipelined loop (decode step i on the
host while the GPU runs step i - 1, an admitted request's prefill launched while its vision tower
still runs) that stall serialises host and device.

:func:`h2d` copies the data into a block of torch's caching pinned-host allocator and issues an
asynchronous copy; the allocator records the copy's stream event and only hands the block out
again once the copy has completed, so the host buffer's lifetime is safe without any fencing here.
"""
from __future__ import annotations

import numpy as np
import torch

_SMALL = 1 << 26     # above this a one-off pinned block costs more than it saves


def h2d(data, device, dtype=None) -> torch.Tensor:
    """list / numpy array / CPU tensor -> tensor on ``device`` (asynchronous for CUDA targets)."""
    dev = torch.device(device)
    if isinstance(data, torch.Tensor):
        t = data if dtype is None else data.to(dtype)
    elif isinstance(data, np.ndarray):
        t = torch.from_numpy(np.ascontiguousarray(data))
        if dtype is not None:
            t = t.to(dtype)
    else:
        t = torch.as_tensor(data, dtype=dtype)
    if dev.type != "cuda":
        return t.to(dev)
    if t.device.type == "cuda":
        return t.to(dev)
    if t.numel() * t.element_size() > _SMALL or torch.cuda.is_current_stream_capturing():
        return t.to(dev)
    pinned = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    pinned.copy_(t)
    return pinned.to(dev, non_blocking=True)


def h2d_ahead(data, device, dtype=None) -> torch.Tensor:
    """:func:`h2d` for a prefill's small inputs (token ids, cache slots) queued behind other work:
    an integer array of <= 896 values travels in the arguments of one tiny kernel (ops_llm.cpp:
    upload_small), so it lands as soon as the queue ahead drains, not 20-70 us later per
    hipMemcpyAsync (a side-stream copy does not help: the blit kernel waits its turn behind the
    busy queue's kernels; profiles/r5_ttft_*).  Anything else: :func:`h2d`."""
    dev = torch.device(device)
    if dev.type == "cuda" and dtype in (None, torch.long) and not torch.cuda.is_current_stream_capturing():
        a = data.numpy() if isinstance(data, torch.Tensor) and not data.is_cuda else data
        if not isinstance(a, torch.Tensor):
            a = np.asarray(a)
            if a.dtype.kind in "iu" and 0 < a.size <= 896 and (dtype is not None or a.dtype == np.int64):
                a32 = a.reshape(-1).astype(np.int32)
                if int(a32.min()) == int(a.min()) and int(a32.max()) == int(a.max()):
                    from ..ops import hip_ops

                    out = torch.empty(a.shape, dtype=torch.long, device=dev)
                    hip_ops().upload_small(torch.from_numpy(a32), out.view(-1))
                    return out
    return h2d(data, device, dtype)
