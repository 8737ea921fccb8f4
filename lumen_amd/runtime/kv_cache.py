"""Paged KV cache: device block pools + the native block manager (csrc/host/kv_blocks.cpp).

Per layer one k pool [NB, Hkv, 64, D] and one transposed v pool [NB, Hkv, D, 64]
(bf16; layouts in csrc/llm.h).  Pools are zero-initialised once so never-written
slots hold finite values (masked lanes multiply them by 0).  The number of blocks
defaults to a fraction of the free HBM — with 288 GB per MI355X, the Llama-3-8B
TP-shard leaves room for ~10^6 cached tokens per GPU.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence

import numpy as np
import torch

from .._native import load_host

BLOCK = 64


class BlockManager:
    """ctypes front of the C++ block manager."""

    def __init__(self, num_blocks: int):
        lib = load_host()
        if lib is None:
            raise RuntimeError("lumen host library (_lumen_host.so) not built: python -m lumen_amd._build")
        self.lib = lib
        lib.lumen_kv_create.restype = ctypes.c_void_p
        lib.lumen_kv_create.argtypes = [ctypes.c_int]
        for fn in ("lumen_kv_free_blocks", "lumen_kv_num_seqs"):
            getattr(lib, fn).argtypes = [ctypes.c_void_p]
        lib.lumen_kv_destroy.argtypes = [ctypes.c_void_p]
        lib.lumen_kv_reserve.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int]
        lib.lumen_kv_can_reserve.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int]
        lib.lumen_kv_table.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_int), ctypes.c_int]
        lib.lumen_kv_fork.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64]
        lib.lumen_kv_release.argtypes = [ctypes.c_void_p, ctypes.c_int64]
        self.num_blocks = num_blocks
        self.h = lib.lumen_kv_create(num_blocks)

    def __del__(self):
        h, self.h = getattr(self, "h", None), None
        if h:
            self.lib.lumen_kv_destroy(h)

    def free_blocks(self) -> int:
        return self.lib.lumen_kv_free_blocks(self.h)

    def num_seqs(self) -> int:
        return self.lib.lumen_kv_num_seqs(self.h)

    def reserve(self, seq: int, n_tokens: int) -> bool:
        return self.lib.lumen_kv_reserve(self.h, seq, n_tokens) >= 0

    def can_reserve(self, seq: int, n_tokens: int) -> bool:
        return bool(self.lib.lumen_kv_can_reserve(self.h, seq, n_tokens))

    def table(self, seq: int) -> list[int]:
        buf = (ctypes.c_int * 4096)()
        n = self.lib.lumen_kv_table(self.h, seq, buf, 4096)
        if n < 0:
            raise KeyError(seq)
        if n > 4096:
            buf = (ctypes.c_int * n)()
            self.lib.lumen_kv_table(self.h, seq, buf, n)
        return list(buf[:n])

    def fork(self, src: int, dst: int) -> int:
        return self.lib.lumen_kv_fork(self.h, src, dst)

    def release(self, seq: int) -> None:
        self.lib.lumen_kv_release(self.h, seq)


def kv_dtype_from_env(default=torch.bfloat16):
    """LUMEN_KV_DTYPE=fp8 -> OCP e4m3fn paged cache (half the HBM per token; decode attention
    widens it to bf16 in registers), bf16 (default) otherwise."""
    v = os.environ.get("LUMEN_KV_DTYPE", "").strip().lower()
    if v in ("fp8", "e4m3", "float8_e4m3fn"):
        return torch.float8_e4m3fn
    if v in ("bf16", "bfloat16"):
        return torch.bfloat16
    return default


class PagedKVCache:
    def __init__(self, num_layers: int, num_kv_heads: int, head_dim: int, num_blocks: Optional[int] = None,
                 device=None, dtype=torch.bfloat16, hbm_fraction: float = 0.5, max_blocks: int = 1 << 20):
        device = torch.device(device) if device is not None else torch.device("cpu")
        per_block = num_layers * 2 * num_kv_heads * BLOCK * head_dim * torch.tensor([], dtype=dtype).element_size()
        if num_blocks is None or num_blocks <= 0:
            if device.type == "cuda":
                free, _ = torch.cuda.mem_get_info(device)
                num_blocks = int(free * hbm_fraction) // per_block
            else:
                num_blocks = 256
        num_blocks = max(4, min(int(num_blocks), max_blocks))
        self.num_blocks = num_blocks
        self.num_layers, self.Hkv, self.D = num_layers, num_kv_heads, head_dim
        self.device = device
        self.k = [torch.zeros((num_blocks, num_kv_heads, BLOCK, head_dim), device=device, dtype=dtype)
                  for _ in range(num_layers)]
        self.v = [torch.zeros((num_blocks, num_kv_heads, head_dim, BLOCK), device=device, dtype=dtype)
                  for _ in range(num_layers)]
        self.blocks = BlockManager(num_blocks)
        self.bytes = per_block * num_blocks

    @property
    def capacity_tokens(self) -> int:
        return self.num_blocks * BLOCK

    def slots(self, seq: int, start: int, n: int) -> np.ndarray:
        """cache slots (block * 64 + offset) of positions [start, start + n) of ``seq``."""
        tab = np.asarray(self.blocks.table(seq), np.int64)
        p = np.arange(start, start + n)
        return tab[p // BLOCK] * BLOCK + p % BLOCK

    def block_table(self, seqs: Sequence[int], width: Optional[int] = None) -> np.ndarray:
        tabs = [self.blocks.table(s) for s in seqs]
        w = max(1, width or max((len(t) for t in tabs), default=1))
        out = np.zeros((len(seqs), w), np.int32)
        for i, t in enumerate(tabs):
            out[i, :len(t)] = t[:w]
        return out
