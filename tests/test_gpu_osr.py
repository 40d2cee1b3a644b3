"""GPU parity for oversampled input (osr > 1) against the CPU oracle, bit
for bit: the estimate's best-of-osr phase selection by detector power
(LoRaDetector.hpp:64, glibc log10f; LoRaDemod.cpp:93-113 with the
lowest-bin tie-break, phy.cpp:106-121 without), the time shift in
oversampled samples and the symbol reads of every osr-th sample
(LoRaDemod.cpp:144-163, phy.cpp:208-229), the oversampled modulator
(LoRaMod.cpp:8-43) and estimate_offsets over whole buffers (phy.cpp:81-148).
The oracle's osr handling is pinned to the reference build in
tests/test_oracle_vs_reference.py (test_oversampled_*)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _bits(x):
    return np.asarray(x, np.float32).view(np.uint32)


def _frames(oracle, sf, osr, nf, plen, seed, snr=None, cfo=0.0, max_delay=0):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(nf):
        iq = oracle.modulate(oracle.encode(rng.integers(0, 256, plen, dtype=np.uint8).tobytes()),
                             sf, osr=osr)
        if cfo:
            iq = (iq * np.exp(2j * np.pi * cfo / ((1 << sf) * osr) * np.arange(iq.size))).astype(np.complex64)
        d = int(rng.integers(0, max_delay + 1)) if max_delay else 0
        if d:
            iq = np.concatenate([np.zeros(d, np.complex64), iq[:-d]])
        if snr is not None:
            s = np.sqrt(10 ** (-snr / 10) / 2)
            iq = (iq + s * (rng.standard_normal(iq.size) + 1j * rng.standard_normal(iq.size))).astype(np.complex64)
        out.append(iq)
    return np.stack(out)


def _tie_frames(sf, osr, nsym, amps):
    """Phase 0 alternating (peak N/2), phase 1 constant (peak 0): equal
    detector power, different bins (see test_oracle_vs_reference)."""
    N = 1 << sf
    out = []
    for a in amps:
        x = np.zeros((nsym, N, osr), np.complex64)
        x[:, :, 0] = a * np.where(np.arange(N) % 2 == 0, 1.0, -1.0)
        x[:, :, 1] = a
        out.append(x.reshape(-1))
    return np.stack(out)


CASES = [  # sf, osr, frames, payload bytes, snr, cfo, max delay (samples), hann
    (7, 2, 6, 16, None, 0.0, 0, False),
    (7, 2, 8, 16, -8.0, 0.2, 200, False),
    (7, 4, 5, 8, None, -0.3, 400, False),
    (8, 3, 4, 12, 0.0, 0.1, 90, True),
    (9, 2, 4, 8, -12.0, 0.0, 0, False),
    (5, 8, 6, 8, None, 0.05, 255, False),
    (10, 2, 3, 4, None, 0.0, 1500, False),
    (11, 4, 2, 4, None, 0.4, 300, True),
    (12, 2, 2, 4, -5.0, 0.0, 100, False),
]

LAUNCH = [0, 32]  # osr > 1 always runs the separate kernels; both flags agree


@pytest.mark.parametrize("sf,osr,nf,plen,snr,cfo,dly,hann", CASES)
@pytest.mark.parametrize("launch", LAUNCH)
def test_oversampled_demodulate(oracle, lphy, sf, osr, nf, plen, snr, cfo, dly, hann, launch):
    iq = _frames(oracle, sf, osr, nf, plen, seed=sf * 17 + osr, snr=snr, cfo=cfo, max_delay=dly)
    d = lphy.Demodulator(sf, 125000, osr, lphy.WINDOW_HANN if hann else lphy.WINDOW_NONE)
    fs = iq.shape[1]
    syms, pay, meta = d.demod_host(iq, nf, fs, lphy.MODE_DEMODULATE, lphy.F_DECODE | launch)
    for f in range(nf):
        r, osyms, osync, omet = oracle.demodulate(iq[f], sf, osr=osr, hann=hann)
        np.testing.assert_array_equal(syms[f], osyms, err_msg=f"frame {f}")
        assert meta["sync_word"][f] == osync
        assert _bits(meta["cfo"][f]) == _bits(omet[0])
        assert _bits(meta["time_offset"][f]) == _bits(omet[1])
        np.testing.assert_array_equal(pay[f], oracle.decode(osyms)[1])
    syms, pay, meta = d.demod_host(iq, nf, fs, lphy.MODE_LORA_DEMODULATE, lphy.F_DECODE | launch)
    for f in range(nf):
        r, osyms, osync, omet = oracle.lora_demodulate(iq[f], sf, osr=osr, hann=hann)
        np.testing.assert_array_equal(syms[f], osyms, err_msg=f"frame {f}")
        assert meta["sync_word"][f] == osync
        assert _bits(meta["cfo"][f]) == _bits(omet[0])
        assert _bits(meta["time_offset"][f]) == _bits(omet[1])


@pytest.mark.parametrize("sf,osr", [(2, 2), (7, 2), (7, 4), (10, 2)])
def test_oversampled_power_tie(oracle, lphy, sf, osr):
    x = _tie_frames(sf, osr, 6, [0.5, 0.25, 3.0, 1.0])
    nf, fs = x.shape
    d = lphy.Demodulator(sf, 125000, osr)
    for mode in (lphy.MODE_DEMODULATE, lphy.MODE_LORA_DEMODULATE):
        syms, _, meta = d.demod_host(x, nf, fs, mode, 32)
        for f in range(nf):
            if mode == lphy.MODE_DEMODULATE:
                r, osyms, osync, omet = oracle.demodulate(x[f], sf, osr=osr)
            else:
                r, osyms, osync, omet = oracle.lora_demodulate(x[f], sf, osr=osr)
            np.testing.assert_array_equal(syms[f], osyms)
            assert _bits(meta["cfo"][f]) == _bits(omet[0])
            assert _bits(meta["time_offset"][f]) == _bits(omet[1])


@pytest.mark.parametrize("sf,osr", [(7, 2), (9, 4), (5, 3), (12, 2)])
def test_oversampled_modulate_and_estimate(oracle, lphy, sf, osr):
    rng = np.random.default_rng(sf * osr)
    syms = rng.integers(0, 1 << min(sf, 8), 9, dtype=np.uint16)
    d = lphy.Demodulator(sf, 125000, osr)
    a = d.modulate_host(syms, 1.0, 0x34)
    b = oracle.modulate(syms, sf, osr=osr, sync=0x34)
    np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))
    noisy = (b + 0.3 * (rng.standard_normal(b.size) + 1j * rng.standard_normal(b.size))).astype(np.complex64)
    step = (1 << sf) * osr
    for n in (1, 2, 5):
        m = d.estimate_host(noisy[: n * step])
        o = oracle.estimate_offsets(noisy[: n * step], sf, osr)
        assert _bits(m["cfo"]) == _bits(o[0]) and _bits(m["time_offset"]) == _bits(o[1])
