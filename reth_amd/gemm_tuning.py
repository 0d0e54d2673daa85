"""GEMM algorithm selection for the library GEMMs left on the path (FC1 forward / data /
weight gradient on hipBLASLt or rocBLAS): PyTorch's TunableOp benchmarks the candidate
solutions of both libraries for each (shape, layout) once and keeps the fastest.

The fp32 GEMMs stay fp32 (gfx950 has no xf32; every candidate is an fp32-MFMA or fp32 VALU
kernel); the numerical check rejects a candidate that differs from the default solution by
more than fp32 round-off.  Results for the Ape-X shapes on MI355X are committed in
reth_amd/tuned/ and read at start; a shape not in the file is tuned on first use (outside
graph capture -- the loop runs eager steps before it captures) and recorded in a scratch
file, not in the package.  Measured: 0.622 vs 0.649-0.657 ms per Pong step on one box
(DESIGN.md).
"""
import os
import tempfile

import torch

_ROOT = os.path.dirname(os.path.abspath(__file__))
RESULTS = os.environ.get("RTH_TUNABLEOP_IN") or os.path.join(_ROOT, "tuned", "tunableop_results_mi355x.csv")


def enable(tune_missing=True, max_tuning_ms=30):
    """switch TunableOp on for this process (idempotent); returns the committed results file
    used, or None"""
    if not torch.cuda.is_available() or os.environ.get("RTH_NO_TUNED_GEMM"):
        return None
    tun = torch.cuda.tunable
    if tun.is_enabled():
        return RESULTS if os.path.exists(RESULTS) else None
    # where newly tuned shapes are written at exit (RTH_TUNABLEOP_OUT: regenerate the committed file)
    scratch = os.environ.get("RTH_TUNABLEOP_OUT") or os.path.join(tempfile.gettempdir(),
                                                                 f"reth_tunableop_{os.getpid()}_%d.csv")
    tun.set_filename(scratch)
    tun.set_numerical_check_tolerances(True, 1e-5, 1e-5)
    tun.set_max_tuning_duration(int(max_tuning_ms))
    tun.enable(True)
    tun.tuning_enable(bool(tune_missing))
    used = None
    if os.path.exists(RESULTS):
        try:
            used = RESULTS if tun.read_file(RESULTS) else None
        except RuntimeError:  # another torch / ROCm build: validators differ, tune afresh
            used = None
    return used
