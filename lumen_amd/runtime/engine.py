"""Continuous-batching generation engine for the VLM decoder (paged KV cache, TP-aware).

The reference generates one request at a time on ORT, copying the whole KV cache
host<->device every token (packages/lumen-vlm/src/lumen_vlm/backends/onnxrt_backend.py:
298-492).  Here one engine thread owns the device:

* requests are admitted while the native block manager can reserve
  ``prompt + max_new_tokens`` tokens (no preemption needed at 288 GB/GPU);
* each admitted request is prefilled (its ``prefill`` callable builds the input
  embeddings — vision tower + token embeddings — on the engine thread), its first
  token sampled and streamed immediately (TTFT);
* chunked prefill: a prompt longer than ``prefill_chunk`` tokens (env
  ``LUMEN_PREFILL_CHUNK``, default 2048) is prefilled ``prefill_chunk`` tokens per engine
  iteration, with a decode step of the running requests between chunks, so a long
  prompt never stalls the other streams for its whole prefill (each chunk attends the
  cached prefix: :meth:`LLM.prefill` ``prefix_blocks``);
* all running requests then advance together: one batched decode step per
  iteration (paged flash-decoding), sampling from on-device top-k candidates;
* finished sequences release their blocks.

Tensor parallelism: rank 0 runs this loop and broadcasts every step (prefill inputs,
decode token ids / positions / slots / block tables) to follower ranks running
:func:`follower_loop`, so every rank issues the same kernels and collectives; only
rank 0 samples (the candidate merge makes logits identical on all ranks anyway).
"""
from __future__ import annotations

import itertools
import logging
import os
import queue
import threading
import time
from dataclasses import dataclass, field
from typing import Any, Callable, Iterator, Optional, Sequence

import numpy as np
import torch

from .. import ops
from ..ops import llm as lops
from ..parallel.comm import TPGroupUnavailable
from ..utils.h2d import h2d, h2d_ahead
from .kv_cache import BLOCK, PagedKVCache

log = logging.getLogger("lumen.engine")

# look-ahead greedy decode on the graph path (LUMEN_DECODE_LOOKAHEAD=0: one synchronous step at a time)
_LOOKAHEAD = os.environ.get("LUMEN_DECODE_LOOKAHEAD", "1") != "0"


@dataclass
class SamplingParams:
    max_new_tokens: int = 512
    temperature: float = 0.0
    top_p: float = 1.0
    repetition_penalty: float = 1.0
    stop_token_ids: tuple = ()
    seed: Optional[int] = None


@dataclass
class GenRequest:
    rid: int
    prefill_args: Any                       # opaque, handed to the engine's prefill builder
    prompt_len: int
    params: SamplingParams
    out: "queue.Queue" = field(default_factory=queue.Queue)
    tokens: list = field(default_factory=list)
    t_submit: float = 0.0
    t_admit: Optional[float] = None         # prefill started (left the admission queue)
    t_first: Optional[float] = None
    t_done: Optional[float] = None
    finish_reason: Optional[str] = None
    ctx: int = 0                            # tokens in the KV cache
    rng: Any = None
    x: Any = None                           # prefill input embeddings while the prompt is being chunk-prefilled
    done: int = 0                           # prompt tokens prefilled so far

    def stream(self, timeout: Optional[float] = None) -> Iterator[tuple]:
        """yields ("token", id) ... then ("done", reason) | raises the engine error."""
        while True:
            kind, val = self.out.get(timeout=timeout)
            if kind == "error":
                raise val
            yield kind, val
            if kind == "done":
                return


class Sampler:
    """Greedy / temperature + nucleus sampling from per-row top-k candidates (vocab-parallel).

    ``spec`` (built on rank 0, broadcast with every TP step) carries everything that
    changes the local logits shard or the collective shapes: k, per-row 1/T and the
    repetition-penalty token sets."""

    K_SAMPLE = 64

    def __init__(self, llm):
        self.llm = llm
        self.d2h = 0          # host round trips of the candidate gather (gloo groups only)

    @staticmethod
    def spec(reqs: Sequence[GenRequest]) -> dict:
        sample = any(r.params.temperature > 0 for r in reqs)
        pens = [float(r.params.repetition_penalty) for r in reqs]
        use_pen = any(abs(p - 1.0) > 1e-6 for p in pens)
        return {"k": Sampler.K_SAMPLE if sample else 8,
                "inv": [1.0 / r.params.temperature if r.params.temperature > 0 else 1.0 for r in reqs] if sample else None,
                "pen": pens if use_pen else None,
                "pen_ids": [list(r.tokens) for r in reqs] if use_pen else None}

    def candidates(self, logits: torch.Tensor, spec: dict):
        if spec["pen"] is not None:
            lops.rep_penalty_(logits, [[t - self.llm.v0 for t in ids] for ids in spec["pen_ids"]], spec["pen"])
        if spec["inv"] is not None:
            logits.mul_(h2d(spec["inv"], logits.device, torch.float32)[:, None])
        k = spec["k"]
        v, i, lse = ops.row_topk(logits, k, with_lse=True, index_offset=self.llm.v0)
        tp = self.llm.tp
        if tp.enabled:
            # ONE all-gather of the packed (values, indices, lse) rows -- vocab ids < 2^24 are exact
            # in fp32 -- and the merge (global top-k, lse of the shard lse's) on the device
            import torch.distributed as dist

            B = v.shape[0]
            packed = torch.cat([v, i.to(torch.float32), lse.view(B, 1)], 1).contiguous()
            if packed.is_cuda and dist.get_backend(tp.group) == "gloo":    # gloo gathers host tensors only
                packed = packed.cpu()
                self.d2h += 1
            parts = [torch.empty_like(packed) for _ in range(tp.world)]
            dist.all_gather(parts, packed, group=tp.group)
            allp = torch.stack(parts, 1)                                   # [B, world, 2k + 1]
            vals, ids = allp[..., :k].reshape(B, -1), allp[..., k:2 * k].reshape(B, -1)
            lse = torch.logsumexp(allp[..., 2 * k], 1)
            v, order = torch.topk(vals, k, dim=1)
            i = torch.gather(ids, 1, order).to(torch.int32)
        return v, i, lse

    def pick(self, cands, reqs: Sequence[GenRequest]) -> list[int]:
        v, i, lse = (t.cpu().numpy() for t in cands)
        out = []
        for b, r in enumerate(reqs):
            if r.params.temperature > 0:
                out.append(lops.sample_from_candidates(v[b], i[b], float(lse[b]), r.params.temperature,
                                                       r.params.top_p, r.rng))
            else:
                out.append(int(i[b, 0]))
        return out


class TPSync:
    """Step channel from rank 0 (the engine) to the follower ranks of a TP group.

    Transport:

    * ``bus`` (default when every rank of the group is on this node -- always, for
      :class:`~lumen_amd.parallel.tp.TPServingGroup`): a host shared-memory ring
      (:mod:`lumen_amd.parallel.step_bus`).  A follower's host reads the step straight from shared
      memory -- no collective and no device->host copy per token -- and launches its step while
      the leader launches its own.
    * ``bcast``: ONE broadcast of a 4 KiB prefix of an int32 buffer per step (GPU buffer for RCCL,
      host for gloo), plus a sized remainder for long descriptors; the follower copies the prefix
      to the host to parse it.

    A decode step is an 8-int header (op, batch, table width, top-k, flags, message length)
    followed by the step descriptor -- ids, positions, cache slots, context lengths, block table;
    nothing is pickled.  ``flags``: 1 = replay the captured graph, 2 = token ids come from the
    previous replay's in-graph arg-max (look-ahead step), 4 = the graph's in-graph TP sampler is
    this step's sampler (the follower does nothing after the replay).  Prefill / control messages
    and decode steps whose sampling needs per-row state (temperatures, repetition-penalty token
    sets) travel pickled (bus) or as an object broadcast (bcast).
    ``capacity`` (ints after the header) must hold 4 * batch + batch * table width of the
    largest decode step: :func:`tp_sync_capacity`.
    """

    OBJ, DECODE, OBJ_BIG = 1, 2, 3
    F_GRAPH, F_DEV_IDS, F_INGRAPH = 1, 2, 4

    def __init__(self, group=None, src: int = 0, device: Optional[torch.device] = None, capacity: int = 1 << 15,
                 transport: Optional[str] = None):
        import torch.distributed as dist

        self.group, self.src = group, src
        if device is None:
            be = dist.get_backend(group) if dist.is_initialized() else "gloo"
            device = torch.device("cuda", torch.cuda.current_device()) if be == "nccl" else torch.device("cpu")
        self.device = device
        self.capacity = int(capacity)
        self.buf = torch.zeros(8 + self.capacity, dtype=torch.int32, device=device)
        self.prefix = min(1024, 8 + self.capacity)          # ints per step's first broadcast
        self.stats = {"tensor_steps": 0, "object_steps": 0, "two_part_steps": 0, "d2h": 0}
        self.bus = None
        transport = transport or os.environ.get("LUMEN_TP_STEP_TRANSPORT", "bus")
        if transport == "bus":
            self.bus = self._open_bus()
        self.transport = "bus" if self.bus is not None else "bcast"

    def _open_bus(self):
        """Collective: a shared-memory bus when all ranks share this host and the host library
        has it (every rank agrees, else all fall back to broadcasts)."""
        import socket

        import torch.distributed as dist

        from ..parallel import step_bus

        rank, world = dist.get_rank(self.group), dist.get_world_size(self.group)
        hosts = [None] * world
        dist.all_gather_object(hosts, (socket.gethostname(), step_bus.available()), group=self.group)
        if len({h for h, _ in hosts}) != 1 or not all(ok for _, ok in hosts):
            return None
        slot = max(1 << 18, 4 * (8 + self.capacity) + 64)
        name = [None]
        bus, err = None, None
        if rank == self.src:
            try:
                name[0] = step_bus.StepBus.unique_name()
                bus = step_bus.StepBus(name[0], None, nslots=64, slot_bytes=slot, nreaders=world - 1)
            except Exception as e:  # noqa: BLE001 - agreed fallback below
                name[0], err = None, e
        dist.broadcast_object_list(name, src=self.src, group=self.group)
        if name[0] is not None and rank != self.src:
            try:
                bus = step_bus.StepBus(name[0], rank if rank < self.src else rank - 1)
            except Exception as e:  # noqa: BLE001
                bus, err = None, e
        oks = [None] * world
        dist.all_gather_object(oks, bus is not None, group=self.group)
        if rank == self.src and bus is not None:
            bus.unlink()                       # every rank holds its mapping (or gave up): drop the name
        if not all(oks):
            if bus is not None:
                bus.close()
            log.warning("TP step bus unavailable (%s); stepping over broadcasts", err)
            return None
        return bus

    def _bcast(self, t: torch.Tensor) -> None:
        import torch.distributed as dist

        dist.broadcast(t, src=self.src, group=self.group)

    def send(self, msg) -> None:
        import pickle

        import torch.distributed as dist

        self.stats["object_steps"] += 1
        if self.bus is not None:
            data = pickle.dumps(msg, protocol=pickle.HIGHEST_PROTOCOL)
            head = np.zeros(8, np.int32)
            if 32 + len(data) <= self.bus.slot_bytes:
                head[0] = self.OBJ
                self.bus.publish(head.tobytes() + data)
                return
            head[0] = self.OBJ_BIG
            self.bus.publish(head)
        else:
            self.buf[:8].fill_(0)
            self.buf[0] = self.OBJ
            self._bcast(self.buf[:self.prefix])
        dist.broadcast_object_list([msg], src=self.src, group=self.group)

    def send_decode(self, ids, pos, slots, bt, ctx, spec, graph: bool, ingraph: bool = False) -> None:
        """``ids`` None: the previous replay's in-graph arg-max feeds this step (look-ahead)."""
        B, W = len(pos), bt.shape[1]
        if spec["inv"] is not None or spec["pen"] is not None or 4 * B + B * W > self.capacity:
            self.send(("decode", ids, pos, slots, bt, ctx, spec, graph, ingraph))
            return
        n = 8 + 4 * B + B * W
        flags = (self.F_GRAPH if graph else 0) | (self.F_DEV_IDS if ids is None else 0) | \
            (self.F_INGRAPH if ingraph else 0)
        msg = np.zeros(n, np.int32)
        msg[:8] = [self.DECODE, B, W, spec["k"], flags, n, 0, 0]
        if ids is not None:
            msg[8:8 + B] = np.asarray(ids, np.int64).astype(np.int32)
        msg[8 + B:] = np.concatenate([np.asarray(pos, np.int32), np.asarray(slots, np.int64).astype(np.int32),
                                      np.asarray(ctx, np.int32), np.asarray(bt, np.int32).reshape(-1)])
        self.stats["tensor_steps"] += 1
        if self.bus is not None:
            self.bus.publish(msg)
            return
        self.buf[:n].copy_(torch.from_numpy(msg), non_blocking=self.device.type == "cuda")
        self._bcast(self.buf[:self.prefix])
        if n > self.prefix:
            self._bcast(self.buf[self.prefix:n])
            self.stats["two_part_steps"] += 1

    def _parse_decode(self, p: np.ndarray):
        h = p[:8].tolist()
        B, W, k, flags = h[1], h[2], h[3], h[4]
        p = p[8:8 + 4 * B + B * W]
        ids = None if flags & self.F_DEV_IDS else p[:B].astype(np.int64)
        pos = p[B:2 * B].copy()
        slots = p[2 * B:3 * B].astype(np.int64)
        ctx = p[3 * B:4 * B].copy()
        bt = p[4 * B:].reshape(B, W).copy()
        return ("decode", ids, pos, slots, bt, ctx, {"k": k, "inv": None, "pen": None, "pen_ids": None},
                bool(flags & self.F_GRAPH), bool(flags & self.F_INGRAPH))

    def _recv_obj(self):
        import torch.distributed as dist

        obj = [None]
        dist.broadcast_object_list(obj, src=self.src, group=self.group)
        return obj[0]

    def recv(self):
        if self.bus is not None:
            import pickle

            from ..parallel.step_bus import BusClosed

            while True:
                try:
                    m = self.bus.next(timeout_ms=1000)
                except BusClosed:
                    return ("stop",)
                if m is not None:
                    break
                if not self.bus.writer_alive():
                    return ("stop",)
            op = int(np.frombuffer(m[:4], np.int32)[0])
            if op == self.OBJ:
                return pickle.loads(m[32:])     # written by this group's own leader process
            if op == self.OBJ_BIG:
                return self._recv_obj()
            return self._parse_decode(np.frombuffer(m, np.int32))
        self._bcast(self.buf[:self.prefix])
        p = self.buf[:self.prefix].cpu().numpy()
        self.stats["d2h"] += 1
        if int(p[0]) == self.OBJ:
            return self._recv_obj()
        n = int(p[5])
        if n > self.prefix:
            self._bcast(self.buf[self.prefix:n])
            p = self.buf[:n].cpu().numpy()
            self.stats["d2h"] += 1
        return self._parse_decode(p)

    def close(self) -> None:
        if self.bus is not None:
            self.bus.close()
            self.bus = None


def tp_sync_capacity(max_batch: int, max_position: int) -> int:
    """Descriptor ints of the largest decode step: 4 per row + the block table (64-token blocks)."""
    return max_batch * (4 + -(-max_position // 64))


class DecodeGraphs:
    """hipGraph-captured decode steps, one graph per (padded batch-size, table-width) bucket.

    A decode step is ~5 kernels per layer (hundreds per token) whose host launch cost
    dominates small-batch decode; replaying a captured graph issues them in one call.
    Inputs live in ONE device buffer per graph (positions, context lengths, block table of
    fixed width, cache slots) filled by ONE H2D copy from a pinned staging buffer; padded
    rows use slot -1 (no cache write) and context 1, and their logits are ignored.

    The graph also holds the greedy sampler: the row top-8 candidates + row lse go to one
    packed result buffer (one D2H per step) and the arg-max token is written straight into the
    batch bucket's token-id buffer, which every graph of that bucket embeds from -- so the NEXT
    step can be launched before the host has read this one (:meth:`launch` with ``ids=None``;
    LLMEngine's look-ahead decode).  Under TP the vocab-parallel merge is captured too: each
    rank's shard top-8 + lse go into its row of a [world, B, 20] fp32 block, ONE all-reduce
    (the IPC one-shot kernel) gives every rank every shard's candidates, and the global top-8,
    the lse of the shard lse's and the arg-max are computed on every rank identically -- so the
    followers never read anything back and look-ahead works under TP.  The last word of the
    result buffer is the IPC all-reduce error flag, copied after the step's last all-reduce:
    the leader sees it in the same D2H as the tokens, before emitting them.  Staging and result
    buffers are double-buffered and fenced by the event of the launch that last used them.
    """

    BUCKETS = (1, 2, 4, 8, 16, 32, 64, 128)
    K_GREEDY = 8

    def __init__(self, llm, kv: PagedKVCache, max_batch: int, max_blocks: int):
        self.llm, self.kv = llm, kv
        self.max_blocks = max_blocks
        self.buckets = [b for b in self.BUCKETS if b <= max(max_batch, 1)] or [1]
        if self.buckets[-1] < max_batch:
            self.buckets.append(max_batch)
        self.graphs: dict[tuple, dict] = {}
        self.ids: dict[int, torch.Tensor] = {}       # batch bucket -> device token ids (shared by its graphs)
        self.pool = None
        self.in_graph_sampler = not llm.tp.enabled or os.environ.get("LUMEN_TP_INGRAPH_SAMPLER", "1") == "1"
        self._stream = None     # the capture stream, private to this instance (see _capture_stream)

    def _bucket(self, B: int) -> int:
        for b in self.buckets:
            if b >= B:
                return b
        raise ValueError(f"batch {B} exceeds graph buckets {self.buckets}")

    def _width(self, w: int) -> int:
        """block-table width bucket: the decode kernel's split count follows the width,
        so short contexts must not pay for the maximum-length table."""
        for b in (8, 32, 128):
            if w <= b and b <= self.max_blocks:
                return b
        return self.max_blocks

    @staticmethod
    def _layout(Bp: int, W: int) -> dict:
        """byte offsets of (slots i64, pos i32, ctx i32, bt i32) in the step buffer"""
        o_pos = 8 * Bp
        o_ctx = o_pos + 4 * Bp
        o_bt = o_ctx + 4 * Bp
        return {"slots": (0, Bp), "pos": (o_pos, Bp), "ctx": (o_ctx, Bp), "bt": (o_bt, Bp * W),
                "bytes": -(-(o_bt + 4 * Bp * W) // 16) * 16}

    def _capture_stream(self, d: torch.device) -> torch.cuda.Stream:
        """One stream per engine that nothing else ever uses.  The split-K tickets and
        workspaces the kernels key by stream are baked into the graphs captured on it; a
        stream from PyTorch's recycled pool could later be handed to another thread's eager
        split-K work while a graph replays, and the two would share counters."""
        if self._stream is None:
            self._stream = ops.private_stream(d)
        return self._stream

    def _capture(self, Bp: int, W: int) -> dict:
        d = self.llm.embed.device
        lay = self._layout(Bp, W)
        dbuf = torch.zeros(lay["bytes"], dtype=torch.uint8, device=d)

        def views(buf):
            o, n = lay["slots"]
            v = {"slots": buf[o:o + 8 * n].view(torch.int64)}
            for k in ("pos", "ctx"):
                o, n = lay[k]
                v[k] = buf[o:o + 4 * n].view(torch.int32)
            o, n = lay["bt"]
            v["bt"] = buf[o:o + 4 * n].view(torch.int32).view(Bp, W)
            return v

        st = views(dbuf)
        st["slots"].fill_(-1)
        st["ctx"].fill_(1)
        if Bp not in self.ids:
            self.ids[Bp] = torch.zeros(Bp, dtype=torch.long, device=d)
        ids = self.ids[Bp]
        k = self.K_GREEDY
        res = torch.zeros(2 * Bp * k + Bp + 1, dtype=torch.float32, device=d) if self.in_graph_sampler else None
        tp = self.llm.tp
        KP = 2 * k + 4                      # per-row candidate record: k values, k ids, lse, pad to 16 B
        gat = torch.zeros((tp.world, Bp, KP), dtype=torch.float32, device=d) if res is not None and tp.enabled \
            else None
        loc = torch.zeros(2 * Bp * k + Bp, dtype=torch.float32, device=d) if gat is not None else None
        ws: dict = {}

        def run():
            logits = self.llm.decode(ids, st["pos"], st["slots"], self.kv, st["bt"], st["ctx"], workspace=ws)
            if res is not None:
                v = res[:Bp * k].view(Bp, k)
                i = res[Bp * k:2 * Bp * k].view(torch.int32).view(Bp, k)
                lse = res[2 * Bp * k:2 * Bp * k + Bp]
                hip = ops.hip_ops()
                if gat is None:
                    hip.row_topk(logits, k, 1.0, v, i, lse, int(self.llm.v0))
                else:
                    lv = loc[:Bp * k].view(Bp, k)
                    li = loc[Bp * k:2 * Bp * k].view(torch.int32).view(Bp, k)
                    hip.row_topk(logits, k, 1.0, lv, li, loc[2 * Bp * k:], int(self.llm.v0))
                    gat.zero_()
                    own = gat[tp.rank]
                    own[:, :k].copy_(lv)
                    own[:, k:2 * k].copy_(li)                 # global vocab ids < 2^24: exact in fp32
                    own[:, 2 * k].copy_(loc[2 * Bp * k:])
                    self.llm._all_reduce(gat)
                    vals = gat[:, :, :k].permute(1, 0, 2).reshape(Bp, tp.world * k)
                    gids = gat[:, :, k:2 * k].permute(1, 0, 2).reshape(Bp, tp.world * k)
                    tv, order = torch.topk(vals, k, dim=1)
                    v.copy_(tv)
                    i.copy_(torch.gather(gids, 1, order))
                    lse.copy_(torch.logsumexp(gat[:, :, 2 * k], 0))
                    comm = getattr(self.llm, "comm", None)
                    if comm is not None:
                        comm.error_into(res[2 * Bp * k + Bp:].view(torch.int32))
                ids.copy_(i[:, 0])                                   # greedy next token, on the device
            return logits

        s = self._capture_stream(d)
        s.wait_stream(torch.cuda.current_stream(d))
        with torch.cuda.stream(s):
            for _ in range(2):
                run()
        torch.cuda.current_stream(d).wait_stream(s)
        g = torch.cuda.CUDAGraph()
        if self.pool is None:
            self.pool = torch.cuda.graph_pool_handle()
        # captured on the warm-up stream: the split-K tickets / workspaces the kernels key by stream
        # already exist (a first request inside the capture would record its zero-fill into every replay)
        # thread_local: a multi-service engine process runs other services' batch loops on other
        # threads meanwhile; the default (global) mode would fail their HIP calls during the capture
        # (ops.CAPTURE_LOCK: one capture at a time in the process, see there)
        with ops.CAPTURE_LOCK, torch.cuda.graph(g, pool=self.pool, stream=s, capture_error_mode="thread_local"):
            out = run()
        pin = lambda t: torch.empty(t.shape, dtype=t.dtype).pin_memory()  # noqa: E731
        ent = {"g": g, "st": st, "dbuf": dbuf, "out": out, "ws": ws, "res": res, "lay": lay, "Bp": Bp, "W": W,
               "h_step": [pin(dbuf) for _ in range(2)], "h_ids": [pin(ids) for _ in range(2)],
               "h_res": [pin(res) for _ in range(2)] if res is not None else None,
               "ev": [None, None], "par": 0}
        ent["h_views"] = [views(h) for h in ent["h_step"]]
        self.graphs[(Bp, W)] = ent
        return ent

    def _entry(self, B: int, width: int) -> dict:
        key = (self._bucket(B), self._width(width))
        return self.graphs[key] if key in self.graphs else self._capture(*key)

    def launch(self, ids, pos, slots, bt, ctx, fetch: bool = True) -> dict:
        """Stage + replay one step (host arrays; ``ids=None``: the token ids the previous
        replay of this batch bucket wrote on the device).  Returns a handle for
        :meth:`tokens` / :meth:`logits`.  ``fetch=False`` (TP followers): no result copy."""
        B = len(pos)
        e = self._entry(B, bt.shape[1])
        Bp, W = e["Bp"], e["W"]
        par = e["par"]
        e["par"] ^= 1
        if e["ev"][par] is not None:
            e["ev"][par].synchronize()        # the copies that last used these pinned buffers are done
        hv = e["h_views"][par]
        w = min(bt.shape[1], W)
        sl, po, cx, tb = (hv[k].numpy() for k in ("slots", "pos", "ctx", "bt"))
        sl[:] = -1
        sl[:B] = slots
        po[:] = 0
        po[:B] = pos
        cx[:] = 1
        cx[:B] = ctx
        tb[:] = 0
        tb[:B, :w] = bt[:, :w]
        e["dbuf"].copy_(e["h_step"][par], non_blocking=True)
        if ids is not None:
            hi = e["h_ids"][par].numpy()
            hi[:] = 0
            hi[:B] = ids
            self.ids[Bp].copy_(e["h_ids"][par], non_blocking=True)
        e["g"].replay()
        if e["res"] is not None and fetch:
            e["h_res"][par].copy_(e["res"], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        e["ev"][par] = ev
        return {"e": e, "par": par, "B": B, "ev": ev}

    def tokens(self, h: dict):
        """(values [B, 8], ids [B, 8], lse [B]) numpy of a launched step (waits for it); sets
        ``h["err"]`` from the step's all-reduce error word (TP)."""
        e, B = h["e"], h["B"]
        h["ev"].synchronize()
        r = e["h_res"][h["par"]]
        Bp, k = e["Bp"], self.K_GREEDY
        h["err"] = int(r[2 * Bp * k + Bp:].view(torch.int32)[0])
        v = r[:Bp * k].view(Bp, k)[:B].numpy()
        i = r[Bp * k:2 * Bp * k].view(torch.int32).view(Bp, k)[:B].numpy()
        return v, i, r[2 * Bp * k:2 * Bp * k + B].numpy()

    def run(self, ids, pos, slots, bt, ctx) -> torch.Tensor:
        """Replay one step and return its logits [B, V/tp] (device, valid until the next replay)."""
        h = self.launch(ids, pos, slots, bt, ctx)
        return h["e"]["out"][:h["B"]]


class LLMEngine:
    def __init__(self, llm, kv: PagedKVCache, prefill_builder: Callable[[Any], torch.Tensor], max_batch: int = 64,
                 max_prefill_per_step: int = 4, tp_sync: Optional[TPSync] = None, name: str = "vlm",
                 use_graphs: Optional[bool] = None, prefill_chunk: Optional[int] = None,
                 follower_args: Optional[Callable[[Any], Any]] = None):
        """``follower_args``: what the TP followers receive instead of the prefill arguments
        (the VLM strips the image: only rank 0 decodes it and runs the vision tower)."""
        self.llm = llm
        self.kv = kv
        self.build = prefill_builder
        self.max_batch = max_batch
        self.max_prefill = max_prefill_per_step
        self.sync = tp_sync
        self.sampler = Sampler(llm)
        self._ids = itertools.count(1)
        self._waiting: "queue.Queue[GenRequest]" = queue.Queue()
        self._running: list[GenRequest] = []
        self._prefilling: list[GenRequest] = []
        self.prefill_chunk = max(16, int(prefill_chunk or os.environ.get("LUMEN_PREFILL_CHUNK", 2048)))
        self._stop = threading.Event()
        self._ws: dict = {}
        self._pending: Optional[tuple] = None     # (request ids, handle) of a look-ahead decode step in flight
        self.device = llm.embed.device
        self.stats = {"prefills": 0, "prefill_chunks": 0, "decode_steps": 0, "tokens": 0}
        if use_graphs is None:
            use_graphs = os.environ.get("LUMEN_HIP_GRAPHS", "1") == "1"
        self.graphs: Optional[DecodeGraphs] = None
        # under TP every rank captures / replays the same decode graphs in lockstep (the leader's
        # step descriptor says when); the in-graph all-reduces are the IPC one-shot kernel or RCCL
        if use_graphs and llm.tp.enabled:
            use_graphs = os.environ.get("LUMEN_TP_GRAPHS", "1") == "1"
        if use_graphs and self.device.type == "cuda":
            self.graphs = DecodeGraphs(llm, kv, max_batch, -(-llm.cfg.max_position // 64))
        self.follower_args = follower_args
        self._thread = threading.Thread(target=self._loop, name=f"lumen-{name}-engine", daemon=True)
        self._thread.start()

    # ------------------------------------------------------------------ public API
    def submit(self, prefill_args: Any, prompt_len: int, params: SamplingParams) -> GenRequest:
        if self._stop.is_set():
            raise RuntimeError("engine stopped")
        need = prompt_len + params.max_new_tokens
        if need > self.kv.capacity_tokens:
            raise ValueError(f"request needs {need} KV tokens, cache holds {self.kv.capacity_tokens}")
        if prompt_len + params.max_new_tokens > self.llm.cfg.max_position:
            params.max_new_tokens = max(1, self.llm.cfg.max_position - prompt_len)
        r = GenRequest(rid=next(self._ids), prefill_args=prefill_args, prompt_len=prompt_len, params=params,
                       t_submit=time.perf_counter(), rng=np.random.default_rng(params.seed))
        self._waiting.put(r)
        return r

    def close(self) -> None:
        self._stop.set()
        self._thread.join(timeout=10)
        if self.sync is not None:
            try:
                self.sync.send(("stop",))
            except Exception:  # pragma: no cover
                pass
            self.sync.close()

    # ------------------------------------------------------------------ loop
    def _emit(self, r: GenRequest, tok: int) -> bool:
        """record token; returns True when the request finished."""
        p = r.params
        if tok in p.stop_token_ids:
            r.finish_reason = "eos_token"
            return True
        r.tokens.append(tok)
        r.out.put(("token", tok))
        self.stats["tokens"] += 1
        if len(r.tokens) >= p.max_new_tokens:
            r.finish_reason = "length"
            return True
        return False

    def _finish(self, r: GenRequest) -> None:
        self.kv.blocks.release(r.rid)
        r.t_done = time.perf_counter()
        r.out.put(("done", r.finish_reason or "stop"))

    def _fail(self, reqs, e: BaseException) -> None:
        for r in reqs:
            try:
                self.kv.blocks.release(r.rid)
            except Exception:
                pass
            r.out.put(("error", e))

    def cancel(self, r: GenRequest) -> None:
        r.params.max_new_tokens = len(r.tokens)   # finishes at the next step

    def _admit(self) -> list[GenRequest]:
        adm = []
        while (len(self._running) + len(self._prefilling) + len(adm) < self.max_batch
               and len(self._prefilling) + len(adm) < self.max_prefill):
            try:
                r = self._waiting.get_nowait()
            except queue.Empty:
                break
            if not self.kv.blocks.reserve(r.rid, r.prompt_len + r.params.max_new_tokens):
                self._waiting.put(r)   # retry when blocks free up
                break
            adm.append(r)
        return adm

    @torch.no_grad()
    def _prefill_chunk(self, r: GenRequest, budget: int) -> int:
        """Prefill up to ``budget`` more prompt tokens of ``r``; returns the tokens consumed.
        On the last chunk the first token is sampled and ``r`` joins the running batch."""
        if r.x is None:
            if r.t_admit is None:
                r.t_admit = time.perf_counter()
            if self.sync is not None:
                # followers must enter the build (its vocab-parallel embedding all-reduce)
                # together with us: announce it before building the inputs
                fa = self.follower_args(r.prefill_args) if self.follower_args is not None else r.prefill_args
                self.sync.send(("pbuild", r.rid, fa))
                x = self.build(r.prefill_args)
                if x.shape[0] != r.prompt_len:
                    raise RuntimeError(f"prefill built {x.shape[0]} rows for a {r.prompt_len}-token prompt")
            else:
                x = self.build(r.prefill_args)
                r.prompt_len = x.shape[0]
            r.x, r.done = x, 0
        T = r.prompt_len
        s = r.done
        e = min(T, s + max(1, budget))
        last = e == T
        slots = self.kv.slots(r.rid, s, e - s)
        tab = np.asarray(self.kv.blocks.table(r.rid), np.int64)[: -(-e // BLOCK)] if s > 0 else None
        spec = Sampler.spec([r]) if last else None
        if self.sync is not None:
            self.sync.send(("pchunk", r.rid, s, e, slots, tab, spec, last))
        logits = self.llm.prefill(r.x[s:e], self.kv, h2d_ahead(slots, self.device), start_pos=s,
                                  prefix_blocks=h2d_ahead(tab, self.device) if tab is not None else None)
        r.done = e
        self.stats["prefill_chunks"] += 1
        if not last:
            return e - s
        r.x = None
        r.ctx = T
        tok = self.sampler.pick(self.sampler.candidates(logits, spec), [r])[0]
        r.t_first = time.perf_counter()
        self.stats["prefills"] += 1
        self._prefilling.remove(r)
        if self._emit(r, tok):
            self._finish(r)
        else:
            self._running.append(r)
        return e - s

    def _prefill_round(self) -> None:
        """One engine iteration's prefill work: up to ``prefill_chunk`` prompt tokens,
        oldest request first.  (Packing several prompts into one forward measured neutral for
        Llama-3-8B fp8 and slower for FastVLM-0.5B batch 16, profiles/r2_prefill_pack_v1.txt,
        so chunks run per request.)"""
        budget = self.prefill_chunk
        for r in list(self._prefilling):
            if budget <= 0:
                break
            try:
                budget -= self._prefill_chunk(r, budget)
            except Exception as e:  # noqa: BLE001 - surfaced to the caller
                log.exception("prefill failed")
                if r in self._prefilling:
                    self._prefilling.remove(r)
                r.x = None
                self._fail([r], e)

    def _greedy_graph_ok(self, reqs, spec) -> bool:
        """the in-graph greedy sampler serves this step: graphs on, every request greedy without
        repetition penalty, batch and table within the graph buckets (any TP size)"""
        g = self.graphs
        return (g is not None and g.in_graph_sampler and _LOOKAHEAD
                and spec["inv"] is None and spec["pen"] is None and spec["k"] <= g.K_GREEDY
                and len(reqs) <= g.buckets[-1])

    def _graph_ready(self, reqs) -> bool:
        """the step's graph exists or captures now (a capture failure disables graphs).  Under
        TP the capture runs collectives, so it happens inside the launch, after the followers
        received the step (they capture the same graph at the same point)."""
        w = max(len(self.kv.blocks.table(r.rid)) for r in reqs)
        if w > self.graphs.max_blocks:
            return False
        if self.sync is not None:
            return True
        try:
            self.graphs._entry(len(reqs), w)
            return True
        except Exception as e:  # noqa: BLE001 - capture unsupported: eager launches from now on
            log.warning("hipGraph decode disabled: %s", e)
            self.graphs = None
            return False

    def _step_inputs(self, reqs, ahead: int):
        """positions / slots / block table / context lengths of the step that feeds position
        r.ctx + ahead of every request"""
        pos = np.array([r.ctx + ahead for r in reqs], np.int32)
        slots = np.concatenate([self.kv.slots(r.rid, r.ctx + ahead, 1) for r in reqs])
        bt = self.kv.block_table([r.rid for r in reqs])
        return pos, slots, bt, pos + 1

    def _can_look_ahead(self, reqs) -> bool:
        """every request surely runs one more step after this one (no length finish, its reserved
        blocks cover the next position) and nothing waits to join the batch"""
        if self._prefilling or not self._waiting.empty():
            return False
        for r in reqs:
            if len(r.tokens) + 1 >= r.params.max_new_tokens:
                return False
            if len(self.kv.blocks.table(r.rid)) * BLOCK <= r.ctx + 1:
                return False
        return True

    @torch.no_grad()
    def _decode(self) -> None:
        reqs = self._running
        B = len(reqs)
        spec = Sampler.spec(reqs)
        if self._greedy_graph_ok(reqs, spec) and self._graph_ready(reqs):
            # look-ahead decode: the step after this one is launched (token ids taken from this
            # step's in-graph arg-max) BEFORE this step's tokens are read, so the host work of
            # reading, streaming and scheduling overlaps the GPU instead of idling it between steps
            rids = [r.rid for r in reqs]
            pend, self._pending = self._pending, None
            if pend is not None and pend[0] == rids:
                h = pend[1]
            else:
                ids = np.array([r.tokens[-1] for r in reqs], np.int64)
                h = self._launch_greedy(ids, self._step_inputs(reqs, 0), spec)
            nxt = self._launch_greedy(None, self._step_inputs(reqs, 1), spec) if self._can_look_ahead(reqs) else None
            _v, i, _lse = self.graphs.tokens(h)
            if h.get("err"):
                # an IPC all-reduce of this step gave up on a peer: its tokens are garbage
                self._pending = None
                raise TPGroupUnavailable("tensor-parallel peer not responding (IPC all-reduce timed out)")
            toks = [int(i[b, 0]) for b in range(B)]
            self.stats["decode_steps"] += 1
            still = []
            for r, t in zip(reqs, toks):
                r.ctx += 1
                if self._emit(r, t):
                    self._finish(r)
                else:
                    still.append(r)
            self._running = still
            if nxt is not None and len(still) == B:
                self._pending = (rids, nxt)
                self.stats["lookahead_steps"] = self.stats.get("lookahead_steps", 0) + 1
            return
        self._pending = None
        ids = np.array([r.tokens[-1] for r in reqs], np.int64)
        pos = np.array([r.ctx for r in reqs], np.int32)
        slots = np.concatenate([self.kv.slots(r.rid, r.ctx, 1) for r in reqs])
        bt = self.kv.block_table([r.rid for r in reqs])
        ctx = pos + 1
        graph = self.graphs is not None and bt.shape[1] <= self.graphs.max_blocks
        if self.sync is not None:
            self.sync.send_decode(ids, pos, slots, bt, ctx, spec, graph)
        logits = self._decode_step(ids, pos, slots, bt, ctx, graph)
        toks = self.sampler.pick(self.sampler.candidates(logits, spec), reqs)
        self.stats["decode_steps"] += 1
        comm = getattr(self.llm, "comm", None)
        if comm is not None:
            comm.check()    # before emitting; the tokens' D2H already waited for the step
        still = []
        for r, t in zip(reqs, toks):
            r.ctx += 1
            if self._emit(r, t):
                self._finish(r)
            else:
                still.append(r)
        self._running = still

    def _launch_greedy(self, ids, inputs, spec) -> dict:
        """One in-graph-sampled step (``ids`` None: look-ahead, ids from the device); under TP the
        followers get the descriptor first and replay the same graph."""
        if self.sync is not None:
            self.sync.send_decode(ids, *inputs, spec, graph=True, ingraph=True)
        try:
            return self.graphs.launch(ids, *inputs)
        except Exception:
            if self.sync is not None:
                raise            # TP ranks must not diverge
            log.warning("hipGraph decode disabled", exc_info=True)
            self.graphs = None
            raise

    def _decode_step(self, ids, pos, slots, bt, ctx, graph: bool = True) -> torch.Tensor:
        d = self.device
        if graph and self.graphs is not None and bt.shape[1] <= self.graphs.max_blocks:
            try:
                return self.graphs.run(ids, pos, slots, bt, ctx)
            except Exception as e:  # noqa: BLE001 - capture unsupported: fall back to eager launches
                if self.sync is not None:
                    raise            # TP ranks must not diverge: surface instead of falling back
                log.warning("hipGraph decode disabled: %s", e)
                self.graphs = None
        return self.llm.decode(h2d(ids, d), h2d(pos, d), h2d(slots, d), self.kv, h2d(bt, d), h2d(ctx, d),
                               workspace=self._ws)

    def _loop(self) -> None:
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        while not self._stop.is_set():
            self._prefilling.extend(self._admit())
            if not self._prefilling and not self._running:
                try:
                    r = self._waiting.get(timeout=0.05)
                    self._waiting.put(r)
                except queue.Empty:
                    pass
                continue
            if self._prefilling:
                self._prefill_round()
            if self._running:
                try:
                    self._decode()
                except Exception as e:  # noqa: BLE001
                    log.exception("decode step failed")
                    self._fail(self._running, e)
                    self._running = []
                    self._pending = None


def follower_loop(llm, kv: PagedKVCache, prefill_builder: Callable[[Any], torch.Tensor], sync: TPSync,
                  max_batch: int = 64) -> dict:
    """Non-zero TP ranks: replay rank 0's steps so every collective is matched.  Greedy decode
    steps (flag ``ingraph``) are a descriptor read from the step bus + one graph launch: the
    graph samples on the device, so the follower never reads a result back.  Returns the
    follower's counters (also written as JSON to ``$LUMEN_TP_FOLLOWER_STATS`` when set)."""
    sampler = Sampler(llm)
    ws: dict = {}
    xs: dict = {}                            # rid -> prefill embeddings of prompts being chunk-prefilled
    dev = llm.embed.device
    graphs = None
    if dev.type == "cuda" and os.environ.get("LUMEN_HIP_GRAPHS", "1") == "1" and \
            os.environ.get("LUMEN_TP_GRAPHS", "1") == "1":
        graphs = DecodeGraphs(llm, kv, max_batch, -(-llm.cfg.max_position // 64))   # the leader's buckets
    stats = {"decode_steps": 0, "ingraph_steps": 0, "lookahead_steps": 0, "prefill_chunks": 0}
    while True:
        msg = sync.recv()
        kind = msg[0]
        if kind == "stop":
            break
        with torch.no_grad():
            if kind == "pbuild":
                _, rid, args = msg
                xs[rid] = prefill_builder(args)
            elif kind == "pchunk":
                _, rid, s, e, slots, tab, spec, last = msg
                x = xs[rid] if not last else xs.pop(rid)
                logits = llm.prefill(x[s:e], kv, h2d(slots, dev), start_pos=s,
                                     prefix_blocks=h2d(tab, dev) if tab is not None else None)
                stats["prefill_chunks"] += 1
                if last:
                    sampler.candidates(logits, spec)
            elif kind == "decode":
                _, ids, pos, slots, bt, ctx, spec, graph, ingraph = msg
                stats["decode_steps"] += 1
                if graph and graphs is not None and ingraph:
                    graphs.launch(ids, pos, slots, bt, ctx, fetch=False)
                    stats["ingraph_steps"] += 1
                    stats["lookahead_steps"] += ids is None
                    continue
                if graph and graphs is not None:
                    logits = graphs.run(ids, pos, slots, bt, ctx)
                else:
                    logits = llm.decode(h2d(ids, dev), h2d(pos, dev), h2d(slots, dev), kv, h2d(bt, dev),
                                        h2d(ctx, dev), workspace=ws)
                sampler.candidates(logits, spec)
    stats["d2h"] = sync.stats["d2h"] + sampler.d2h
    stats["transport"] = sync.transport
    path = os.environ.get("LUMEN_TP_FOLLOWER_STATS")
    if path:
        import json

        with open(f"{path}.rank{llm.tp.rank}", "w") as f:
            json.dump(stats, f)
    sync.close()
    return stats
