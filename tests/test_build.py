"""Build-level guards (CPU, no GPU): the PageRank hot kernel must not spill registers.

k_pr_pull_units runs 16 waves per CU (launch bounds 1024 threads, 4 waves per SIMD), so it has
128 VGPRs; an edit that pushed it past them (round 3: 34 VGPRs spilled to scratch) made the
launch 2x slower without failing any parity test.  This compiles gx_pr_sorted.hip with the
compiler's resource report and checks the product instantiation."""
import re
import subprocess

import pytest

from conftest import ROOT

HIPCC = "/opt/rocm/bin/hipcc"


def resource_report(src):
    cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", f"-I{ROOT}/include",
           f"-I{ROOT}/ldbc_graphalytics_platforms_graphblas_amd/csrc", "-c", str(src), "-o", "/dev/null",
           "-Rpass-analysis=kernel-resource-usage"]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert res.returncode == 0, res.stderr[-2000:]
    kernels, cur = {}, None
    for line in res.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            kernels[cur] = {}
            continue
        m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[bytes/lane\])?: (\d+)", line)
        if m and cur:
            kernels[cur][m.group(1).strip()] = int(m.group(2))
    return kernels


def test_pagerank_kernel_does_not_spill():
    import shutil
    if not shutil.which(HIPCC):
        pytest.skip("hipcc not available")
    ks = resource_report(ROOT / "ldbc_graphalytics_platforms_graphblas_amd" / "csrc" / "gx_pr_sorted.hip")
    prod = [k for k in ks if "k_pr_pull_units" in k and "ILb0ELi0E" in k]
    assert prod, sorted(ks)
    for k in prod:
        assert ks[k].get("VGPRs Spill", 0) == 0 and ks[k].get("ScratchSize", 0) == 0, (k, ks[k])
        assert ks[k].get("VGPRs", 0) <= 128, (k, ks[k])
