"""Register-pressure guard: the hot gfx950 kernels must compile without scratch spills.

A spill turns the 256x256 GEMM into a 2.5 ms kernel (seen when a second activation
switch was added to the shared epilogue); this cross-compiles each hot source with
the resource-usage remarks and fails on any ScratchSize > 0.  CPU-only (hipcc).
"""
import re
import shutil
import subprocess
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import pytest

CSRC = Path(__file__).resolve().parents[1] / "lumen_amd" / "csrc"
HOT = ["gemm.hip", "gemm_skinny.hip", "attention.hip", "llm.hip", "conv.hip", "norm.hip", "topk.hip"]
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


def _scratch(src: str):
    out = subprocess.run([HIPCC, "-x", "hip", "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", str(CSRC / src),
                          "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
    names = re.findall(r"Function Name: (\S+)", out.stderr)
    scratch = [int(x) for x in re.findall(r"ScratchSize \[bytes/lane\]: (\d+)", out.stderr)]
    return src, out.returncode, list(zip(names, scratch))


@pytest.mark.skipif(not Path(HIPCC).exists(), reason="hipcc not available")
def test_hot_kernels_do_not_spill():
    with ThreadPoolExecutor(4) as ex:
        res = list(ex.map(_scratch, HOT))
    bad = []
    for src, rc, ks in res:
        assert rc == 0, f"{src} failed to compile"
        assert ks, f"{src}: no kernels reported"
        bad += [(src, n, s) for n, s in ks if s > 0]
    assert not bad, f"kernels with scratch spills: {bad}"
