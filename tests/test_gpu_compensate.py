"""lphy_hip_compensate (phy.cpp:150-180, lora_phy::compensate_offsets) on the
GPU against the oracle's restatement, which test_oracle_vs_reference.py pins
to the reference build: the rotation by e^{-j 2 pi cfo n / (N osr)} and the
integer time shift, bit for bit, through the host and device entry points."""
import numpy as np
import pytest

from test_oracle_vs_reference import COMP_CASES, _nan_bits_equal

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("sf,osr,cfo,toff", COMP_CASES)
def test_compensate_host_matches_oracle(oracle, lphy, sf, osr, cfo, toff):
    rng = np.random.default_rng(sf * 13 + osr)
    n = 7 * (1 << sf) * osr
    x = ((rng.standard_normal(n) + 1j * rng.standard_normal(n)) * 2.0).astype(np.complex64)
    x[3] = complex(np.inf, 0.5)
    d = lphy.Demodulator(sf, osr=osr)
    got = d.compensate_host(x, cfo, toff)
    _nan_bits_equal(np.asarray(got, np.complex64).view(np.float32),
                    oracle.compensate_offsets(x, sf, cfo, toff, osr).view(np.float32))


def test_compensate_device_on_stream(oracle, lphy):
    import torch
    sf, cfo, toff = 8, 0.3, -40.2
    rng = np.random.default_rng(3)
    n = 9 << sf
    x = ((rng.standard_normal(n) + 1j * rng.standard_normal(n))).astype(np.complex64)
    d = lphy.Demodulator(sf)
    s = torch.cuda.Stream()
    t = torch.from_numpy(x.view(np.float32).copy()).cuda()
    torch.cuda.current_stream().synchronize()
    rc = d.lib.lphy_hip_compensate(d.ctx, t.data_ptr(), n, cfo, toff, s.cuda_stream)
    assert rc == 0
    s.synchronize()
    got = t.cpu().numpy().view(np.complex64)
    _nan_bits_equal(got.view(np.float32), oracle.compensate_offsets(x, sf, cfo, toff).view(np.float32))
