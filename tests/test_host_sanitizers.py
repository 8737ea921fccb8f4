"""Race detection / sanitizers for the host C++ runtime.

The host libraries (DB-net geometry, similarity transform, paged-KV block manager)
are compiled together with a stress driver under AddressSanitizer + UBSan and,
separately, ThreadSanitizer (4 threads hammering the block manager).  GPU
sanitizers are not available on this pool; the HIP kernels are covered by the
numerics tests and the no-spill resource guard instead.
"""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HOST = ROOT / "lumen_amd" / "csrc" / "host"
DRIVER = Path(__file__).parent / "native" / "host_stress.cpp"
CXX = shutil.which("g++")


@pytest.mark.skipif(CXX is None, reason="g++ not available")
@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_host_runtime_under_sanitizer(tmp_path, san):
    exe = tmp_path / f"stress_{san.split(',')[0]}"
    srcs = [str(DRIVER), str(HOST / "geometry.cpp"), str(HOST / "kv_blocks.cpp")]
    cmd = [CXX, "-std=c++17", "-O1", "-g", f"-fsanitize={san}", "-fno-omit-frame-pointer", "-pthread", *srcs,
           "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    run = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300,
                         env={"ASAN_OPTIONS": "detect_leaks=1", "TSAN_OPTIONS": "halt_on_error=1"})
    assert run.returncode == 0, run.stdout + run.stderr
    assert "ok boxes=" in run.stdout
