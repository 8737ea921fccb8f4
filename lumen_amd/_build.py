"""In-tree builder for the lumen_amd native libraries (gfx950 only).

Produces two shared objects next to this file:

* ``_lumen_hip.so``  — every ``csrc/*.hip`` kernel + ``csrc/ops.cpp`` registered as
  ``torch.ops.lumen.*`` (PyTorch-ROCm custom ops, HIP stream aware).
* ``_lumen_host.so`` — host-only C++ runtime pieces (``csrc/host/*.cpp``: DB-net
  geometry, KV block manager, batching queue) exposed through a plain C ABI and
  loaded with ctypes, so they work with or without a GPU.

The builder drives ``hipcc --offload-arch=gfx950`` directly (no JIT cache under
~/.cache), compiles translation units in parallel and only rebuilds what is
out of date, so the built ``.so`` travels with the repo snapshot to a GPU box.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
BUILD = PKG.parent / "build" / "lumen_amd"
HIP_SO = PKG / "_lumen_hip.so"
HOST_SO = PKG / "_lumen_host.so"
ARCH = os.environ.get("LUMEN_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _torch_paths():
    import torch

    root = Path(torch.__file__).resolve().parent
    inc = [root / "include", root / "include" / "torch" / "csrc" / "api" / "include"]
    lib = root / "lib"
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _hip_flags():
    inc, _, abi = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    flags = [
        f"--offload-arch={ARCH}",
        "-O3",
        "-fPIC",
        "-std=c++17",
        "-D__HIP_PLATFORM_AMD__=1",
        "-DUSE_ROCM=1",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-DTORCH_EXTENSION_NAME=_lumen_hip",
        "-Wno-unused-result",
        "-Wno-deprecated-declarations",
        "-Wno-unused-command-line-argument",
        f"-I{CSRC}",
        f"-I{py_inc}",
    ]
    for p in inc:
        flags.append(f"-isystem{p}")
    return flags


def _needs(obj: Path, src: Path, deps: list[Path]) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return src.stat().st_mtime > t or any(d.stat().st_mtime > t for d in deps)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        # hipcc can leave a fresh-looking object behind when the device pass fails, which
        # the mtime check would then take as up to date: remove it
        if "-o" in cmd:
            Path(cmd[cmd.index("-o") + 1]).unlink(missing_ok=True)
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
        raise RuntimeError(f"compile failed: {cmd[-1] if cmd else ''}")


# Per-source extra flags.  attention.hip: MFMA accumulators in VGPRs — the online softmax
# rescales O and reads S with VALU ops, and with AGPR accumulators hipcc shuttles all of
# them through v_accvgpr_read/write every 64-key chunk (~40 extra VALU ops per chunk).
PER_FILE_FLAGS = {
    "attention.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"],
}


def _local_deps(src: Path, seen: set | None = None) -> list[Path]:
    """Headers of csrc/ that ``src`` includes (``#include "x.h"``), transitively: a source is rebuilt
    when one of ITS headers changes, not when any header does (gemm_f8.hip alone compiles for
    ~8 minutes)."""
    import re

    seen = set() if seen is None else seen
    for name in re.findall(r'^\s*#\s*include\s+"([^"]+)"', src.read_text(errors="ignore"), re.M):
        h = src.parent / name
        if h.exists() and h not in seen:
            seen.add(h)
            _local_deps(h, seen)
    return sorted(seen)


def build(verbose: bool = False, jobs: int | None = None) -> dict:
    """Compile (incrementally) and link both native libraries. Returns paths."""
    BUILD.mkdir(parents=True, exist_ok=True)
    jobs = jobs or min(8, os.cpu_count() or 4)

    # ---- HIP kernel library + torch op registration
    flags = _hip_flags()
    srcs = sorted(CSRC.glob("*.hip")) + sorted(CSRC.glob("*.cpp"))
    objs = []
    todo = []
    for s in srcs:
        o = BUILD / (s.name + ".o")
        objs.append(o)
        if _needs(o, s, _local_deps(s)):
            lang = ["-x", "hip"] if s.suffix == ".hip" else ["-x", "hip"]
            todo.append([HIPCC, *flags, *PER_FILE_FLAGS.get(s.name, []), *lang, "-c", str(s), "-o", str(o)])
    with cf.ThreadPoolExecutor(jobs) as ex:
        list(ex.map(_run, todo))
    if todo or not HIP_SO.exists() or any(o.stat().st_mtime > HIP_SO.stat().st_mtime for o in objs):
        _, lib, _ = _torch_paths()
        link = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(HIP_SO),
                f"-L{lib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-lamdhip64",
                f"-Wl,-rpath,{lib}"]
        _run(link)
        if verbose:
            print("linked", HIP_SO)

    # ---- host-only runtime library (C ABI, no torch / HIP dependency)
    host_dir = CSRC / "host"
    hsrcs = sorted(host_dir.glob("*.cpp")) if host_dir.exists() else []
    if hsrcs:
        hobjs, htodo = [], []
        for s in hsrcs:
            o = BUILD / ("host_" + s.name + ".o")
            hobjs.append(o)
            if _needs(o, s, _local_deps(s)):      # host headers and the shared csrc/*.h layouts
                htodo.append(["g++", "-O3", "-fPIC", "-std=c++17", "-pthread", f"-I{host_dir}", "-c", str(s),
                              "-o", str(o)])
        with cf.ThreadPoolExecutor(jobs) as ex:
            list(ex.map(_run, htodo))
        if htodo or not HOST_SO.exists() or any(o.stat().st_mtime > HOST_SO.stat().st_mtime for o in hobjs):
            _run(["g++", "-shared", "-fPIC", "-pthread", *map(str, hobjs), "-o", str(HOST_SO)])
    return {"hip": str(HIP_SO), "host": str(HOST_SO) if hsrcs else None}


if __name__ == "__main__":
    print(build(verbose=True))
