"""The fused kernel's certified fast rotation (per-frame table + argmax
certificate, csrc/lphy_hip.hip "Certified fast rotation") against the exact
per-sample rotation of the reference (LoRaDemod.cpp:152-163,
phy.cpp:217-229), which LPHY_F_EXACT_ROTATION forces for every symbol.

Every output bit must agree: symbols, payload bytes and the 32-byte frame
records.  Inputs are chosen to stress the certificate: deep noise (near-ties
between the two largest bins), large CFO and time offsets (non-zero t_off,
symbols whose window shift is not applied, large phases), exact two-tone
ties, NaN / Inf samples, zero frames and big amplitudes (mode 0 is not
normalised).  The recheck counter shows the fallback actually ran."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _impaired(oracle, sf, nf, seed, plen=32, snr_db=None, cfo_bins=0.4, gain=(1.0,),
              max_delay=0):
    rng = np.random.default_rng(seed)
    N = 1 << sf
    frames = []
    for f in range(nf):
        p = rng.integers(0, 256, plen, dtype=np.uint8).tobytes()
        x = oracle.modulate(oracle.encode(p), sf).astype(np.complex128)
        t = np.arange(x.size)
        x = x * np.exp(2j * np.pi * rng.uniform(-cfo_bins, cfo_bins) / N * t)
        if max_delay:
            x = np.roll(x, int(rng.integers(-max_delay, max_delay + 1)))
        if snr_db is not None:
            s = np.sqrt(10 ** (-snr_db / 10) / 2)
            x = x + s * (rng.standard_normal(x.size) + 1j * rng.standard_normal(x.size))
        frames.append((x * gain[f % len(gain)]).astype(np.complex64))
    return np.stack(frames)


def _both(lphy, d, iq, mode):
    """The product library's run and the exact rotation's (test build:
    LPHY_F_EXACT_ROTATION is not in the product library)."""
    nf, fs = iq.shape
    a = d.demod_host(iq, nf, fs, mode, lphy.F_DECODE)
    n_fast = d.recheck_count(reset=True)
    dt = lphy.Demodulator(d.sf, d.bw_hz, d.osr, d.window, test_build=True)
    b = dt.demod_host(iq, nf, fs, mode, lphy.F_DECODE | lphy.F_EXACT_ROTATION)
    n_exact = dt.recheck_count(reset=True)
    assert dt.bounds_violations() == 0
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])
    np.testing.assert_array_equal(a[2].view(np.uint8), b[2].view(np.uint8))
    return a, n_fast, n_exact


MODES = [0, 1, 2]


@pytest.mark.parametrize("sf", [5, 6, 7, 8, 9, 10])
@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("snr", [None, -8.0, -16.0, -24.0])
def test_fast_equals_exact_noise(oracle, lphy, sf, mode, snr):
    nf = {5: 300, 6: 260, 7: 240, 8: 120, 9: 60, 10: 40}[sf]
    iq = _impaired(oracle, sf, nf, seed=sf * 31 + mode + int(snr or 0), snr_db=snr,
                   gain=(1.0, 0.3, 2.5), max_delay=3)
    if mode == 1:
        iq = np.stack([oracle.dechirp(x, sf) for x in iq])
    d = lphy.Demodulator(sf)
    (syms, _, meta), n_fast, n_exact = _both(lphy, d, iq, mode)
    assert n_exact >= nf * syms.shape[1]  # every live symbol re-ran exactly
    # spot-check against the oracle
    for f in range(0, nf, max(1, nf // 5)):
        if mode == 0:
            r, osyms, osync, _ = oracle.demodulate(iq[f], sf)
        else:
            x = oracle.dechirp(iq[f], sf) if mode == 2 else iq[f]
            r, osyms, osync, _ = oracle.lora_demodulate(x, sf)
        np.testing.assert_array_equal(syms[f], osyms)
        assert meta["sync_word"][f] == osync


@pytest.mark.parametrize("sf", [7, 9])
@pytest.mark.parametrize("hann", [False, True])
def test_fast_equals_exact_window_big_cfo(oracle, lphy, sf, hann):
    """Hann window, CFO up to +-3 bins and delays of up to 40 samples."""
    iq = _impaired(oracle, sf, 150 if sf == 7 else 40, seed=5 + sf + hann, snr_db=-12.0,
                   cfo_bins=3.0, max_delay=40)
    d = lphy.Demodulator(sf, 125000, 1, lphy.WINDOW_HANN if hann else lphy.WINDOW_NONE)
    for mode in MODES:
        x = np.stack([oracle.dechirp(v, sf) for v in iq]) if mode == 1 else iq
        _both(lphy, d, x, mode)


def test_fast_path_rechecks_ties_and_specials(oracle, lphy):
    """Frames the certificate must refuse: all-zero data symbols, NaN / Inf
    samples, a zero frame, huge and tiny amplitudes, exact two-tone ties;
    plus clean frames that must need no re-check."""
    sf, N = 7, 128
    base = oracle.modulate(oracle.encode(bytes(range(16))), sf)
    fs = base.size
    frames = [base.copy() for _ in range(12)]
    frames[1][2 * N:] = 0  # data symbols all zero: every bin 0
    frames[2][700] = np.nan
    frames[3][1000] = np.inf
    frames[4][300] = complex(np.nan, 0.5)
    frames[5] = np.zeros_like(base)
    frames[6] = base * 1e20
    frames[7] = base * 1e-30
    iq = np.stack(frames).astype(np.complex64)
    d = lphy.Demodulator(sf)
    for mode in (0, 2):
        _, n_fast, _ = _both(lphy, d, iq, mode)
        assert n_fast > 0
    # pre-dechirped two-tone symbols (mode 1): bins 5 and 40 of equal power
    # (the estimated CFO rotation separates them; outputs must still agree)
    t = np.arange(N)
    tone = ((np.exp(2j * np.pi * 5 * t / N) + np.exp(2j * np.pi * 40 * t / N)) / 2).astype(np.complex64)
    tie = np.tile(tone, fs // N)
    _both(lphy, d, np.stack([tie] * 4), 1)
    # clean frames alone: the certificate holds for every symbol
    clean = np.stack([base] * 16).astype(np.complex64)
    _, n_fast, _ = _both(lphy, d, clean, 2)
    assert n_fast == 0


def test_fast_path_equal_power_fixture(oracle, lphy):
    """equal_power_iq (equal_power_bin_test.cpp:35): tie -> bin 0, repeated
    to a whole frame so the fused path's symbol units see it."""
    from pathlib import Path
    raw = np.fromfile(Path(__file__).parent / "golden" / "equal_power_iq.bin", np.complex64)
    sf, N = 7, 128
    sym = np.resize(raw, N)
    frame = np.tile(sym, 20).astype(np.complex64)  # long enough for the fused launch
    iq = np.stack([frame] * 8)
    d = lphy.Demodulator(sf)
    for mode in MODES:
        (syms, _, meta), n_fast, _ = _both(lphy, d, iq, mode)
        x = oracle.dechirp(frame, sf) if mode == 2 else frame
        r, osyms, _, _ = (oracle.demodulate(frame, sf) if mode == 0
                          else oracle.lora_demodulate(x, sf))
        np.testing.assert_array_equal(syms[0], osyms)
