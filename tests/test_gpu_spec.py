"""Speculative normalisation of the fused kernel (k_frames, modes 1/2; for
SF 11-12 the separate launches with DemodArgs::spec_big): the
frame is estimated with the max-abs of its first two symbols, each symbol
unit folds its own samples' max-abs, and the frame end either confirms the
normalisation or settles the frame in k_post (exact estimate + certificate
check against the exact rate, else the whole-frame re-run).  Every output
bit against the oracle (LoRaDemod.cpp:50-197) and against the pre-scan
schedule (LPHY_F_SCAN_FIRST), on frames built to take each branch:
  - the maximum inside the two estimate symbols (confirmed),
  - a larger sample late in the frame (settled: exact scale, exact rate),
  - CFO so that the time shift is negative or positive (the samples no
    symbol window covers are scanned at the frame end),
  - mode 1 frames with a partial last symbol holding the maximum,
  - NaN / inf late in the frame (whole-frame re-run),
  - no-scratch frames (the speculation is off: -ERANGE as the reference)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _bits(x):
    return np.asarray(x, np.float32).view(np.uint32)


def _build(oracle, sf, nf, seed, tail=0):
    rng = np.random.default_rng(seed)
    N = 1 << sf
    base = oracle.modulate(oracle.encode(bytes(range(24))), sf)
    fs = base.size + tail
    t = np.arange(base.size, dtype=np.float64)
    iq = np.zeros((nf, fs), np.complex64)
    for f in range(nf):
        x = base * np.exp(2j * np.pi * rng.uniform(-0.45, 0.45) / N * t)
        x = x + [0.0, 0.02, 0.3][f % 3] * (rng.standard_normal(base.size) + 1j * rng.standard_normal(base.size))
        x = x * [1.0, 0.7, 2.5, 1.3][f % 4]
        iq[f, :base.size] = x.astype(np.complex64)
        if tail:
            iq[f, base.size:] = (0.1 * rng.standard_normal(tail)).astype(np.complex64)
        kind = f % 7
        S = base.size // N
        if kind == 1:    # spike in a late symbol
            iq[f, int(rng.integers(3 * N, S * N))] *= np.complex64(4.0)
        elif kind == 2:  # spike inside the estimate symbols
            iq[f, int(rng.integers(0, 2 * N))] *= np.complex64(4.0)
        elif kind == 3:  # the frame's very last sample / the partial symbol
            iq[f, fs - 1] = np.complex64(complex(6.0, -1.0))
        elif kind == 4:  # a barely larger sample late (scale differs in the last bits)
            j = int(rng.integers(2 * N, S * N))
            iq[f, j] = iq[f, j] * np.complex64(1.0 + 1e-6) + np.complex64(0.001)
        elif kind == 5 and f % 2:
            iq[f, int(rng.integers(2 * N, S * N))] = np.complex64(complex(np.nan, 1.0))
        elif kind == 6 and f % 2:
            iq[f, int(rng.integers(2 * N, S * N))] = np.complex64(complex(np.inf, 0.0))
    return iq


@pytest.mark.parametrize("sf,nf", [(7, 515), (5, 301), (8, 203), (9, 97), (10, 41), (11, 29), (12, 15)])
@pytest.mark.parametrize("mode", [1, 2])
def test_speculative_normalisation(oracle, lphy, sf, nf, mode):
    tail = (1 << sf) // 2 + 3 if mode == 1 else 0  # a partial last symbol
    iq = _build(oracle, sf, nf, seed=sf * 31 + mode, tail=tail)
    fs = iq.shape[1]
    d = lphy.Demodulator(sf)
    a = d.demod_host(iq, nf, fs, mode, lphy.F_DECODE)
    dt = lphy.Demodulator(sf, test_build=True)  # the pre-scan schedule: test build only
    b = dt.demod_host(iq, nf, fs, mode, lphy.F_DECODE | lphy.F_SCAN_FIRST)
    assert dt.bounds_violations() == 0
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])
    np.testing.assert_array_equal(a[2].view(np.uint8), b[2].view(np.uint8))
    for f in range(0, nf, max(1, nf // 60)):
        src = iq[f] if mode == 1 else oracle.dechirp(iq[f], sf)
        r, osyms, osync, omet = oracle.lora_demodulate(src, sf)
        ctx = f"sf {sf} mode {mode} frame {f}"
        assert a[2]["status"][f] == 0, ctx
        np.testing.assert_array_equal(a[0][f], osyms, err_msg=ctx)
        assert a[2]["sync_word"][f] == osync, ctx
        assert _bits(a[2]["cfo"][f]) == _bits(omet[0]), ctx
        assert _bits(a[2]["time_offset"][f]) == _bits(omet[1]), ctx


@pytest.mark.parametrize("sf", [9, 10])
@pytest.mark.parametrize("how", ["hann", "exact_rotation"])
def test_estimate_maxabs_in_symbol0(oracle, lphy, sf, how):
    """Frames whose max-abs lies in sync symbol 0, with symbol 1's own
    maximum smaller but still > 1: both estimate units must be scaled by the
    frame's (symbol 0's) maximum, LoRaDemod.cpp:60-78.  Hann windows and
    LPHY_F_EXACT_ROTATION route SF 9-10 modes 1/2 to k_frames, whose EB tiles
    fold the estimate symbols' max-abs only when both units share a tile
    (SF <= 9); at SF 10 the two-symbol scan must supply it."""
    N = 1 << sf
    rng = np.random.default_rng(1000 + sf)
    base = oracle.modulate(oracle.encode(bytes(range(12))), sf)
    t = np.arange(base.size, dtype=np.float64)
    nf = 24
    iq = np.zeros((nf, base.size), np.complex64)
    for f in range(nf):
        x = base * np.exp(2j * np.pi * rng.uniform(-0.4, 0.4) / N * t) * (1.5 + 0.1 * (f % 5))
        x = x + 0.05 * (rng.standard_normal(base.size) + 1j * rng.standard_normal(base.size))
        x = x.astype(np.complex64)
        j = int(rng.integers(0, N))
        x[j] = np.complex64(complex(3.0 + 0.25 * (f % 4), -0.5))  # the frame's maximum, symbol 0
        iq[f] = x
    window = lphy.WINDOW_HANN if how == "hann" else lphy.WINDOW_NONE
    flags = lphy.F_DECODE | (lphy.F_EXACT_ROTATION if how == "exact_rotation" else 0)
    d = lphy.Demodulator(sf, window=window, test_build=how == "exact_rotation")
    syms, _, meta = d.demod_host(iq, nf, iq.shape[1], 2, flags)
    for f in range(nf):
        dech = oracle.dechirp(iq[f], sf)
        m0 = np.max(np.maximum(np.abs(dech[:N].real), np.abs(dech[:N].imag)))
        m1 = np.max(np.maximum(np.abs(dech[N:2 * N].real), np.abs(dech[N:2 * N].imag)))
        assert m0 > m1 > 1.0
        r, osyms, osync, omet = oracle.lora_demodulate(dech, sf, hann=how == "hann")
        ctx = f"sf {sf} {how} frame {f}"
        assert meta["status"][f] == 0, ctx
        assert _bits(meta["cfo"][f]) == _bits(omet[0]), ctx
        assert _bits(meta["time_offset"][f]) == _bits(omet[1]), ctx
        assert meta["sync_word"][f] == osync, ctx
        np.testing.assert_array_equal(syms[f], osyms, err_msg=ctx)


def test_speculation_off_without_scratch(oracle, lphy):
    sf = 7
    iq = _build(oracle, sf, 64, seed=5)
    d = lphy.Demodulator(sf)
    syms, _, meta = d.demod_host(iq, 64, iq.shape[1], 2, lphy.F_NO_SCRATCH)
    for f in range(64):
        dech = oracle.dechirp(iq[f], sf)
        mx = np.max(np.maximum(np.abs(dech.real), np.abs(dech.imag)))
        if mx > 1.0:
            assert meta["status"][f] == -34
        elif np.isfinite(iq[f]).all():
            r, osyms, osync, omet = oracle.lora_demodulate(dech, sf)
            np.testing.assert_array_equal(syms[f], osyms)
