"""GPU parity: the HIP path (through the C ABI) against the CPU oracle on the
same inputs.  Bit-exact on every integer output (symbol indices, sync word,
decoded bytes, CRC flag, return status) and on the float32 bit patterns of
the per-frame cfo / time_offset estimates."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _frames(oracle, sf, bw, nframes, payload_len, seed, snr_db=None, delay=0):
    rng = np.random.default_rng(seed)
    out, payloads = [], []
    for _ in range(nframes):
        p = rng.integers(0, 256, payload_len, dtype=np.uint8).tobytes()
        iq = oracle.modulate(oracle.encode(p), sf, bw_hz=bw)
        if delay:
            iq = np.concatenate([np.zeros(delay, np.complex64), iq[:-delay]])
        if snr_db is not None:
            sig = np.sqrt(10 ** (-snr_db / 10) / 2)
            noise = sig * (rng.standard_normal(iq.size) + 1j * rng.standard_normal(iq.size))
            iq = (iq + noise).astype(np.complex64)
        out.append(iq)
        payloads.append(p)
    return np.stack(out), payloads


def _bits(x):
    return np.asarray(x, np.float32).view(np.uint32)


CASES = [
    # sf, bw, frames, payload bytes, snr, delay, hann
    (7, 125000, 6, 32, None, 0, False),
    (7, 125000, 4, 32, -10.0, 0, False),
    (7, 125000, 4, 16, -18.0, 3, False),
    (7, 250000, 3, 16, None, 0, False),
    (8, 125000, 4, 32, None, 0, True),
    (8, 500000, 3, 12, 0.0, 0, False),
    (9, 125000, 4, 32, -10.0, 0, False),
    (9, 125000, 4, 32, -15.0, 0, False),
    (10, 125000, 2, 16, None, 5, False),
    (11, 125000, 2, 8, -5.0, 0, False),
    (12, 125000, 2, 8, None, 0, False),
    (12, 500000, 1, 4, -10.0, 0, True),
    (5, 125000, 3, 8, None, 0, False),
    (6, 250000, 3, 8, 3.0, 0, False),
]


@pytest.mark.parametrize("sf,bw,nf,plen,snr,delay,hann", CASES)
def test_mode_demodulate_vs_oracle(oracle, lphy, sf, bw, nf, plen, snr, delay, hann):
    """lora_phy::demodulate + decode (phy.cpp:182-261) per frame."""
    iq, _ = _frames(oracle, sf, bw, nf, plen, seed=sf * 100 + nf, snr_db=snr, delay=delay)
    d = lphy.Demodulator(sf, bw, 1, lphy.WINDOW_HANN if hann else lphy.WINDOW_NONE)
    fs = iq.shape[1]
    syms, pay, meta = d.demod_host(iq, nf, fs, lphy.MODE_DEMODULATE, lphy.F_DECODE)
    for f in range(nf):
        r, osyms, osync, omet = oracle.demodulate(iq[f], sf, bw_hz=bw, hann=hann)
        assert r == syms.shape[1]
        np.testing.assert_array_equal(syms[f], osyms)
        assert meta["sync_word"][f] == osync
        assert _bits(meta["cfo"][f]) == _bits(omet[0])
        assert _bits(meta["time_offset"][f]) == _bits(omet[1])
        rr, obytes, ocrc = oracle.decode(osyms)
        np.testing.assert_array_equal(pay[f], obytes)
        assert meta["crc_ok"][f] == ocrc


@pytest.mark.parametrize("sf,bw,nf,plen,snr,delay,hann", CASES)
@pytest.mark.parametrize("fused", [False, True])
def test_mode_lora_demodulate_vs_oracle(oracle, lphy, sf, bw, nf, plen, snr, delay, hann, fused):
    """external dechirp -> lora_demodulate -> lora_decode (LoRaDemod.cpp:50-197)."""
    iq, payloads = _frames(oracle, sf, bw, nf, plen, seed=sf * 7 + nf, snr_db=snr, delay=delay)
    dech = np.stack([oracle.dechirp(x, sf, bw) for x in iq])
    d = lphy.Demodulator(sf, bw, 1, lphy.WINDOW_HANN if hann else lphy.WINDOW_NONE)
    fs = iq.shape[1]
    mode = lphy.MODE_DECHIRP_LORA_DEMODULATE if fused else lphy.MODE_LORA_DEMODULATE
    syms, pay, meta = d.demod_host(iq if fused else dech, nf, fs, mode, lphy.F_DECODE)
    for f in range(nf):
        r, osyms, osync, omet = oracle.lora_demodulate(dech[f], sf, hann=hann)
        np.testing.assert_array_equal(syms[f], osyms)
        assert meta["sync_word"][f] == osync
        assert _bits(meta["cfo"][f]) == _bits(omet[0])
        assert _bits(meta["time_offset"][f]) == _bits(omet[1])
        rr, obytes = oracle.lora_decode(osyms)
        np.testing.assert_array_equal(pay[f], obytes)
        if snr is None and bw == 125000 and sf >= 6 and not hann and not delay:
            assert pay[f].tobytes() == payloads[f]


def test_modulate_bit_exact(oracle, lphy):
    """GPU lora_modulate (LoRaMod.cpp:8-43) == oracle, every float bit."""
    rng = np.random.default_rng(3)
    for sf, bw in [(7, 125000), (9, 250000), (12, 500000), (2, 125000)]:
        syms = rng.integers(0, 256, 10, dtype=np.uint16)
        d = lphy.Demodulator(sf, bw)
        a = d.modulate_host(syms, 1.0, 0x34)
        b = oracle.modulate(syms, sf, bw_hz=bw, sync=0x34)
        np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))


def test_modulate_repeated_contexts(oracle, lphy):
    """Stress: many producer calls with fresh contexts and varying sizes
    (guards the phase-scratch hand-off between the two modulate kernels)."""
    rng = np.random.default_rng(11)
    for k in range(24):
        sf = int(rng.integers(2, 10))
        bw = [125000, 250000, 500000][k % 3]
        syms = rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint16)
        a = lphy.Demodulator(sf, bw).modulate_host(syms, 1.0, 0x12)
        b = oracle.modulate(syms, sf, bw_hz=bw)
        np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32), err_msg=f"iter {k}")


def test_zero_and_overrange_frames(oracle, lphy):
    sf, N = 7, 128
    d = lphy.Demodulator(sf)
    zero = np.zeros((1, 10 * N), np.complex64)
    syms, _, meta = d.demod_host(zero, 1, 10 * N, lphy.MODE_DEMODULATE)
    r, osyms, osync, omet = oracle.demodulate(zero[0], sf)
    np.testing.assert_array_equal(syms[0], osyms)
    assert _bits(meta["cfo"][0]) == _bits(omet[0])
    big = np.full((1, N), 2.0 + 0j, np.complex64)  # scratch_buffer_error_test.cpp:16
    syms, _, meta = d.demod_host(big, 1, N, lphy.MODE_LORA_DEMODULATE, lphy.F_NO_SCRATCH)
    assert meta["status"][0] == -34  # -ERANGE
    syms, _, meta = d.demod_host(big, 1, N, lphy.MODE_LORA_DEMODULATE)
    r, osyms, osync, omet = oracle.lora_demodulate(big[0], sf)
    np.testing.assert_array_equal(syms[0], osyms)
