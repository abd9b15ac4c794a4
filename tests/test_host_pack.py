"""CPU: the upload's 24-bit column packer (gx::host_pack24, gx_host.cpp; the SSE4.1/SSSE3 path
and the scalar one), through a small C++ harness linked against the built libgx.so."""
import shutil
import subprocess

import pytest

from conftest import ROOT


def test_host_pack24_roundtrip(tmp_path):
    lib = ROOT / "ldbc_graphalytics_platforms_graphblas_amd" / "libgx.so"
    if not lib.exists() or shutil.which("g++") is None:
        pytest.skip("libgx.so not built or no g++")
    exe = tmp_path / "pack24_check"
    subprocess.run(["g++", "-O2", "-std=c++17", str(ROOT / "tests" / "native" / "pack24_check.cpp"), "-o", str(exe),
                    f"-L{lib.parent}", "-lgx", f"-Wl,-rpath,{lib.parent}"], check=True, capture_output=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "pack24 ok" in out.stdout
