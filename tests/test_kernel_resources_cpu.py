"""Build-time guard on the gfx950 code objects: no kernel may use scratch (private memory).

A kernel that spills or keeps an argument block or array on the stack pays a per-lane
scratch write and a load per access -- the tree update once copied its 176-byte argument
block to scratch in every lane (12 MB of writes per launch) because an out-of-line call
took the arguments by reference.  hipcc reports each kernel's ScratchSize with
-Rpass-analysis=kernel-resource-usage; this compiles every HIP source for gfx950 (device
code only, no GPU needed) and checks them all."""
import os
import re
import shutil
import subprocess
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _resources(src):
    cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-c", "-o", os.devnull,
           "-I", os.path.join(ROOT, "reth_amd", "csrc"), "-I", os.path.join(ROOT, "include"),
           "-Rpass-analysis=kernel-resource-usage", src]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    kernels, name = {}, None
    for line in out.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            name = m.group(1)
        m = re.search(r"ScratchSize \[bytes/lane\]: (\d+)", line)
        if m and name:
            kernels[name] = int(m.group(1))
    return src, kernels


@pytest.mark.skipif(not shutil.which(HIPCC) and not os.path.exists(HIPCC), reason="hipcc not available")
def test_no_kernel_uses_scratch():
    import __graft_entry__ as g

    srcs = [os.path.join(ROOT, "reth_amd", "csrc", s) for s in g.HIP_SOURCES if s.endswith(".hip")]
    with ThreadPoolExecutor(max_workers=4) as ex:
        results = list(ex.map(_resources, srcs))
    n = sum(len(k) for _, k in results)
    assert n >= 30, f"only {n} kernels reported: the remark format may have changed"
    bad = {name: size for _, k in results for name, size in k.items() if size}
    assert not bad, f"kernels using scratch (bytes/lane): {bad}"
