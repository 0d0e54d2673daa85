"""TunableOp selection (reth_amd/gemm_tuning.py) is reference counted: closing one user
(ApexDQN.close -> restore) leaves tuned selection on for another still open in the process;
the last restore puts back the state the first enable found."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_enable_restore_is_reference_counted(dev):
    from reth_amd import gemm_tuning

    tun = torch.cuda.tunable
    was = tun.is_enabled()
    if was:
        pytest.skip("TunableOp already enabled by the environment")
    gemm_tuning.enable()
    gemm_tuning.enable()
    assert tun.is_enabled()
    gemm_tuning.restore()
    assert tun.is_enabled(), "one close switched tuned selection off under the other user"
    gemm_tuning.restore()
    assert tun.is_enabled() == was
    gemm_tuning.restore()  # an unmatched restore is a no-op
    assert tun.is_enabled() == was
