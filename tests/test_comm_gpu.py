"""IPC one-shot and two-shot all-reduce (csrc/comm.hip) on the GPU.

The box has one MI355X, so the group is 2 or 4 processes sharing cuda:0: the IPC
mapping, flag protocol, parity double-buffering, device-side epochs and hipGraph
replay are the same code paths as 8 GPUs over xGMI (only the link differs).
Bootstrap (handle exchange) runs over gloo.  Reference: fp32 sum of the inputs.
"""
import multiprocessing as mp
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _ar_worker(rank, world, port, q, one_shot_max=1 << 20):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from lumen_amd.parallel.comm import Communicator

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = {"rank": rank}
    try:
        comm = Communicator(None, dev, ipc=True, ipc_max_bytes=one_shot_max)
        assert comm.custom is not None
        errs = []
        # one-shot sizes, then two-shot ones (above one_shot_max: reduce-scatter + all-gather), with
        # slices that do not divide evenly over the ranks / blocks, interleaved with one-shot calls
        for it, (n, dt) in enumerate([(4096, torch.bfloat16), (8, torch.bfloat16), (4096 * 3, torch.float32),
                                      (65536 * 4, torch.bfloat16), (1024, torch.float32), (4096, torch.bfloat16),
                                      (624 * 4096, torch.bfloat16), (300008, torch.float32), (8, torch.bfloat16),
                                      (624 * 4096, torch.bfloat16)]):
            parts = [torch.randn(n, generator=torch.Generator().manual_seed(100 * it + r)) for r in range(world)]
            ref = sum(p.to(dt).float() for p in parts)
            x = parts[rank].to(dt).to(dev)
            comm.all_reduce(x)
            torch.cuda.synchronize()
            errs.append(float((x.float().cpu() - ref).abs().max() / ref.abs().max()))
        res["errs"] = errs
        # hipGraph capture: the epoch advances on the device, so replays stay in step
        x = torch.zeros(2048, dtype=torch.bfloat16, device=dev)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            comm.all_reduce(x)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            comm.all_reduce(x)
        vals = []
        for k in range(3):
            x.fill_(float(rank + 1 + k))
            g.replay()
            torch.cuda.synchronize()
            vals.append(float(x[0]))
        res["graph"] = vals
        # one-shot and two-shot calls of varying sizes (different block partitions of the
        # buffer) alternating inside ONE graph, replayed back to back: every block of a call must use
        # the same parity (a single per-rank epoch)
        sizes = [(2048, torch.bfloat16), (200000, torch.bfloat16), (8, torch.bfloat16), (130000, torch.float32),
                 (40000, torch.bfloat16), (300000, torch.bfloat16), (16, torch.float32)]
        xs = [torch.zeros(n, dtype=dt, device=dev) for n, dt in sizes]
        with torch.cuda.stream(s):
            for t in xs:
                comm.all_reduce(t)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g2 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g2):
            for t in xs:
                comm.all_reduce(t)
        mix = []
        for k in range(4):
            for j, t in enumerate(xs):
                t.copy_(torch.arange(t.numel(), device=dev, dtype=torch.float32).remainder(7).to(t.dtype)
                        * (rank + 1) + k + j)
            g2.replay()
            torch.cuda.synchronize()
            ok = True
            for j, t in enumerate(xs):
                base = torch.arange(t.numel(), device=dev, dtype=torch.float32).remainder(7)
                want = base * sum(r + 1 for r in range(world)) + world * (k + j)
                ok = ok and bool(torch.equal(t.float(), want.to(t.dtype).float()))
            mix.append(ok)
        res["graph_mix"] = mix
        res["error_flag"] = comm.custom.error()
        res["stats"] = dict(comm.stats)
        dist.barrier()
        comm.close()
    except Exception as e:  # noqa: BLE001
        res["exc"] = repr(e)
    finally:
        q.put(res)
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_ipc_all_reduce_processes_one_gpu(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_ar_worker, args=(r, world, port, q, 1 << 18)) for r in range(world)]
    for p in ps:
        p.start()
    out = sorted([q.get(timeout=100) for _ in range(world)], key=lambda d: d["rank"])
    for p in ps:
        p.join(30)
    graph = [float(sum(r + 1 + k for r in range(world))) for k in range(3)]
    for r in out:
        assert "exc" not in r, r
        assert max(r["errs"]) < 1e-2, r["errs"]
        assert r["graph"] == graph, r["graph"]
        assert r["graph_mix"] == [True] * 4, r["graph_mix"]
        assert not r["error_flag"]
        assert r["stats"]["ipc_calls"] >= 11 and r["stats"]["ipc2_calls"] >= 4
    for r in out[1:]:
        assert r["errs"] == out[0]["errs"]       # every rank holds the same (bitwise) result
