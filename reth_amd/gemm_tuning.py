"""GEMM algorithm selection for the library GEMMs left on the path (FC1 forward / data /
weight gradient on hipBLASLt or rocBLAS): PyTorch's TunableOp benchmarks the candidate
solutions of both libraries for each (shape, layout) once and keeps the fastest.

The fp32 GEMMs stay fp32 (gfx950 has no xf32; every candidate is an fp32-MFMA or fp32 VALU
kernel); the numerical check rejects a candidate that differs from the default solution by
more than fp32 round-off.  Results for the Ape-X shapes on MI355X are committed in
reth_amd/tuned/ and read at start; a shape not in the file runs the library's default
solution unless tuning is asked for (then it is tuned on first use, outside graph capture --
the loop runs eager steps before it captures -- and recorded in a scratch file, not in the
package).  Measured: 0.622 vs 0.649-0.657 ms per Pong step on one box
(DESIGN.md).
"""
import os
import tempfile

import torch

_ROOT = os.path.dirname(os.path.abspath(__file__))
RESULTS = os.environ.get("RTH_TUNABLEOP_IN") or os.path.join(_ROOT, "tuned", "tunableop_results_mi355x.csv")


_STATE = {}  # what the first enable() changed: restored by the matching last restore()
_USERS = [0]  # enable() calls not yet matched by restore(): TunableOp stays on while any is open


def enable(tune_missing=None, max_tuning_ms=30):
    """switch TunableOp on for this process; returns the committed results file used, or None.
    Reference counted: every enable() is matched by one restore(), and the state found by the
    first is put back only by the last, so closing one ApexDQN never switches tuned selection
    off under another still running in the process.  Selection is read-only by default: shapes
    missing from the committed file run the library's default solution (deterministic, the
    same on every rank); tune_missing (or RTH_TUNE_MISSING=1) benchmarks them on first use
    instead, and restore() reports which shapes that tuned."""
    if not torch.cuda.is_available() or os.environ.get("RTH_NO_TUNED_GEMM"):
        return None
    tun = torch.cuda.tunable
    _USERS[0] += 1
    if _USERS[0] > 1 or tun.is_enabled():  # already on (ours, or the caller's own): nothing to change
        return RESULTS if os.path.exists(RESULTS) else None
    if tune_missing is None:
        tune_missing = bool(os.environ.get("RTH_TUNE_MISSING"))
    _STATE.update(enabled=tun.is_enabled(), tuning=tun.tuning_is_enabled(), filename=tun.get_filename(),
                  max_ms=tun.get_max_tuning_duration())
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
        except RuntimeError:  # another torch / ROCm build: validators differ
            used = None
    _STATE["known"] = {tuple(r[:2]) for r in tun.get_results()}
    return used


def tuned_at_runtime():
    """(op, shape) entries selected by benchmarking in this process (not from the committed file)"""
    if "known" not in _STATE:
        return []
    return sorted({tuple(r[:2]) for r in torch.cuda.tunable.get_results()} - _STATE["known"])


def restore():
    """match one enable() (ApexDQN.close); the last open one puts TunableOp back to the state
    the first found and logs the shapes tuned at runtime, if any"""
    if _USERS[0] > 0:
        _USERS[0] -= 1
    if _USERS[0] > 0 or not _STATE:
        return
    tun = torch.cuda.tunable
    new = tuned_at_runtime()
    if new:
        import warnings

        warnings.warn(f"TunableOp tuned {len(new)} GEMM shape(s) at runtime (not in {RESULTS}): {new}")
    tun.tuning_enable(_STATE["tuning"])
    tun.enable(_STATE["enabled"])
    tun.set_max_tuning_duration(_STATE["max_ms"])
    if _STATE["filename"]:
        tun.set_filename(_STATE["filename"])
    _STATE.clear()
