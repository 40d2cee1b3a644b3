"""The test-only build (lib/test/liblphy_hip.so: -DLPHY_TEST_PATHS
-DLPHY_DEBUG_BOUNDS) and the product library's boundary:

* the product library rejects the comparison / test flags with -EINVAL and
  has no index counter (-ENOTSUP);
* the test build's device index checks (every LDS address of the transform
  and argmax tiles through Geo::addr / at8, the IQ loads, the doubled
  down-chirp and rotation-table indices, the frame-slot ring, symbol and
  frame-record stores; csrc/lphy_fft.h bound_check) stay at zero over every
  SF, mode and launch path, impaired and ragged frames included, while its
  outputs equal the product library's bit for bit.

`LPHY_LIB=test python -m pytest tests -m gpu` runs the whole suite through
the checked build; conftest.py then fails the session on any violation."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_product_rejects_test_flags(lphy):
    d = lphy.Demodulator(7, lib_path=lphy.HIP_SO)
    iq = np.zeros((2, 66 * 128), np.complex64)
    for fl in (lphy.F_EXACT_ROTATION, lphy.F_SCAN_FIRST, lphy.F_DEBUG_RECHECK, 128):
        with pytest.raises(lphy.LphyError) as e:
            d.demod_host(iq, 2, iq.shape[1], 2, fl)
        assert e.value.rc == -22
    with pytest.raises(lphy.LphyError) as e:
        d.bounds_violations()
    assert e.value.rc == -95  # -ENOTSUP


def _frames(oracle, sf, nf, seed, tail=0):
    rng = np.random.default_rng(seed)
    N = 1 << sf
    base = oracle.modulate(oracle.encode(bytes(range(10))), sf)
    t = np.arange(base.size)
    out = np.zeros((nf, base.size + tail), np.complex64)
    for f in range(nf):
        x = base * np.exp(2j * np.pi * rng.uniform(-0.45, 0.45) / N * t)
        x = np.roll(x, int(rng.integers(-N // 3, N // 3 + 1)))
        x = x + [0.0, 0.05, 0.6][f % 3] * (rng.standard_normal(x.size) + 1j * rng.standard_normal(x.size))
        out[f, :base.size] = (x * [1.0, 2.5, 0.4][f % 3]).astype(np.complex64)
        if tail:
            out[f, base.size:] = 0.2
        if f % 11 == 5:
            out[f, int(rng.integers(0, out.shape[1]))] = np.complex64(complex(np.nan, 0.0))
    return out


@pytest.mark.parametrize("sf", [5, 7, 8, 9, 10, 11, 12])
@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("variant", ["fused", "unfused", "hann"])
def test_bounds_checked_build_matches_product(oracle, lphy, sf, mode, variant):
    nf = {5: 97, 7: 77, 8: 41, 9: 23, 10: 13, 11: 7, 12: 5}[sf]
    tail = (1 << sf) // 3 if mode == 1 else 0
    iq = _frames(oracle, sf, nf, seed=sf * 7 + mode, tail=tail)
    win = lphy.WINDOW_HANN if variant == "hann" else lphy.WINDOW_NONE
    flags = lphy.F_DECODE | (lphy.F_UNFUSED if variant == "unfused" else 0)
    p = lphy.Demodulator(sf, window=win, lib_path=lphy.HIP_SO)
    t = lphy.Demodulator(sf, window=win, test_build=True)
    t.bounds_violations(reset=True)
    a = p.demod_host(iq, nf, iq.shape[1], mode, flags)
    b = t.demod_host(iq, nf, iq.shape[1], mode, flags)
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])
    np.testing.assert_array_equal(a[2].view(np.uint8), b[2].view(np.uint8))
    if mode != 0:  # the comparison schedules too
        t.demod_host(iq, nf, iq.shape[1], mode, flags | lphy.F_SCAN_FIRST)
    t.demod_host(iq, nf, iq.shape[1], mode, flags | lphy.F_EXACT_ROTATION)
    assert t.bounds_violations() == 0
