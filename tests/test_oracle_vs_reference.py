"""Pin the CPU oracle (oracle/lphy_oracle.c) to the reference library itself
(oracle/_ref/libloraref.so, compiled from /root/reference's sources by
oracle/Makefile) on seeded random inputs: every output bit of each function
on the hot path.  Skipped where the reference build is absent (GPU boxes)."""
import numpy as np
import pytest


def _iq(rng, n, scale=1.0):
    return ((rng.standard_normal(n) + 1j * rng.standard_normal(n)) * scale).astype(np.complex64)


def _frame(oracle, rng, sf, bw, plen, snr=None, delay=0, cfo=0.0):
    iq = oracle.modulate(oracle.encode(rng.integers(0, 256, plen, dtype=np.uint8).tobytes()), sf, bw_hz=bw)
    if cfo:
        iq = (iq * np.exp(2j * np.pi * cfo / (1 << sf) * np.arange(iq.size))).astype(np.complex64)
    if delay:
        iq = np.concatenate([np.zeros(delay, np.complex64), iq[:-delay]])
    if snr is not None:
        s = np.sqrt(10 ** (-snr / 10) / 2)
        iq = (iq + s * (rng.standard_normal(iq.size) + 1j * rng.standard_normal(iq.size))).astype(np.complex64)
    return iq


def _bits(x):
    return np.asarray(x, np.float32).view(np.uint32)


@pytest.mark.parametrize("sf", range(1, 13))
def test_fft_bit_exact(oracle, reference, sf):
    rng = np.random.default_rng(sf)
    for _ in range(4):
        x = _iq(rng, 1 << sf, scale=10.0 ** rng.uniform(-3, 3))
        np.testing.assert_array_equal(oracle.fft(x).view(np.uint32), reference.fft(x).view(np.uint32))


@pytest.mark.parametrize("sf,bw", [(s, b) for s in (2, 5, 7, 9, 12) for b in (125000, 250000, 500000)])
def test_modulate_and_dechirp_bit_exact(oracle, reference, sf, bw):
    rng = np.random.default_rng(sf * 7 + bw // 125000)
    syms = rng.integers(0, 1 << min(sf, 8), 12, dtype=np.uint16)
    for sync in (0x12, 0x34, 0xAB):
        a = oracle.modulate(syms, sf, bw_hz=bw, sync=sync)
        b = reference.modulate(syms, sf, bw_hz=bw, sync=sync)
        np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))
    x = _iq(rng, 5 * (1 << sf))
    np.testing.assert_array_equal(oracle.dechirp(x, sf, bw).view(np.uint32),
                                  reference.dechirp(x, sf, bw).view(np.uint32))


CASES = [(sf, bw, plen, snr, delay, cfo, hann)
         for sf, bw, plen, snr, delay, cfo, hann in [
             (7, 125000, 32, None, 0, 0.0, False), (7, 125000, 16, -10.0, 0, 0.0, False),
             (7, 125000, 20, -18.0, 3, 0.0, False), (7, 250000, 8, None, 0, 0.3, False),
             (8, 125000, 32, None, 11, -0.2, True), (8, 500000, 12, 0.0, 0, 0.45, False),
             (9, 125000, 32, -10.0, 0, 0.0, False), (9, 125000, 32, -15.0, 0, 0.0, False),
             (10, 125000, 16, None, 5, 0.1, False), (11, 125000, 8, -5.0, 0, 0.0, False),
             (12, 125000, 4, None, 0, -0.35, False), (5, 125000, 8, None, 0, 0.0, False),
             (6, 250000, 8, 3.0, 2, 0.0, True), (3, 125000, 6, None, 0, 0.0, False)]]


@pytest.mark.parametrize("sf,bw,plen,snr,delay,cfo,hann", CASES)
def test_demodulate_paths_bit_exact(oracle, reference, sf, bw, plen, snr, delay, cfo, hann):
    """lora_phy::demodulate + decode and dechirp -> lora_demodulate ->
    lora_decode, every output including the float metrics' bits."""
    rng = np.random.default_rng(sf * 1000 + plen + delay)
    for rep in range(3):
        iq = _frame(oracle, rng, sf, bw, plen, snr, delay, cfo)
        a = oracle.demodulate(iq, sf, bw_hz=bw, hann=hann)
        b = reference.demodulate(iq, sf, bw_hz=bw, hann=hann)
        assert a[0] == b[0] and a[2] == b[2]
        np.testing.assert_array_equal(a[1], b[1])
        np.testing.assert_array_equal(_bits(a[3][:2]), _bits(b[3][:2]))
        np.testing.assert_array_equal(oracle.decode(a[1])[1], reference.decode(b[1])[1])
        x = oracle.dechirp(iq, sf, bw)
        for scratch in (True, False):
            a = oracle.lora_demodulate(x, sf, hann=hann, scratch=scratch)
            b = reference.lora_demodulate(x, sf, hann=hann, scratch=scratch)
            assert a[0] == b[0] and a[2] == b[2]
            np.testing.assert_array_equal(a[1], b[1])
            np.testing.assert_array_equal(_bits(a[3][:2]), _bits(b[3][:2]))


def test_noise_frames_large_phase(oracle, reference):
    """Pure noise: bogus CFO estimates drive the rotation angle past 120 rad
    (glibc sincosf's large-argument path)."""
    rng = np.random.default_rng(77)
    for sf in (7, 8):
        for _ in range(4):
            x = _iq(rng, 60 * (1 << sf))
            a = oracle.lora_demodulate(x, sf)
            b = reference.lora_demodulate(x, sf)
            np.testing.assert_array_equal(a[1], b[1])
            np.testing.assert_array_equal(_bits(a[3][:2]), _bits(b[3][:2]))


def test_encode_decode_roundtrip(oracle, reference):
    rng = np.random.default_rng(5)
    for n in (0, 1, 2, 7, 32, 255):
        p = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        np.testing.assert_array_equal(oracle.encode(p), reference.encode(p))
        syms = oracle.encode(p) ^ rng.integers(0, 2, 2 * n, dtype=np.uint16) << rng.integers(0, 8, 2 * n, dtype=np.uint16)
        np.testing.assert_array_equal(oracle.decode(syms)[1], reference.decode(syms)[1])
        assert oracle.decode(syms)[2] == reference.decode(syms)[2]


def _osr_frame(oracle, rng, sf, osr, plen, snr, delay, cfo):
    """A frame modulated at osr samples per chip, delayed by a fraction of a
    symbol, with carrier offset and noise."""
    iq = oracle.modulate(oracle.encode(rng.integers(0, 256, plen, dtype=np.uint8).tobytes()),
                         sf, osr=osr)
    if cfo:
        iq = (iq * np.exp(2j * np.pi * cfo / ((1 << sf) * osr) * np.arange(iq.size))).astype(np.complex64)
    if delay:
        iq = np.concatenate([np.zeros(delay, np.complex64), iq[:-delay]])
    if snr is not None:
        s = np.sqrt(10 ** (-snr / 10) / 2)
        iq = (iq + s * (rng.standard_normal(iq.size) + 1j * rng.standard_normal(iq.size))).astype(np.complex64)
    return iq


def _tie_frame(sf, osr, nsym, amp):
    """Oversampled input whose phases tie on detector power with different
    argmax bins: phase 0 carries an alternating sequence (peak at N/2),
    phase 1 a constant one (peak at 0).  LoRaDemod.cpp:102 breaks the tie
    towards the lower bin, phy.cpp:114 keeps the first phase."""
    N = 1 << sf
    x = np.zeros((nsym, N, osr), np.complex64)
    x[:, :, 0] = amp * np.where(np.arange(N) % 2 == 0, 1.0, -1.0)
    if osr > 1:
        x[:, :, 1] = amp
    return x.reshape(-1)


OSR_CASES = [  # sf, osr, payload bytes, snr, delay, cfo, hann
    (7, 2, 16, None, 0, 0.0, False), (7, 2, 16, -8.0, 37, 0.2, False),
    (7, 4, 8, None, 301, -0.3, False), (8, 3, 12, 0.0, 5, 0.1, True),
    (9, 2, 8, -12.0, 0, 0.0, False), (5, 8, 8, None, 17, 0.05, False),
    (10, 2, 4, None, 700, 0.0, False), (12, 2, 4, -5.0, 0, 0.0, False),
    (11, 4, 4, None, 33, 0.4, True)]


@pytest.mark.parametrize("sf,osr,plen,snr,delay,cfo,hann", OSR_CASES)
def test_oversampled_paths_bit_exact(oracle, reference, sf, osr, plen, snr, delay, cfo, hann):
    """osr > 1: the estimate picks the best of osr phases by detector power
    (log10f), symbols read every osr-th sample after the time shift."""
    rng = np.random.default_rng(sf * 31 + osr * 7 + delay)
    for rep in range(2):
        iq = _osr_frame(oracle, rng, sf, osr, plen, snr, delay, cfo)
        a = oracle.demodulate(iq, sf, osr=osr, hann=hann)
        b = reference.demodulate(iq, sf, osr=osr, hann=hann)
        assert a[0] == b[0] and a[2] == b[2]
        np.testing.assert_array_equal(a[1], b[1])
        np.testing.assert_array_equal(_bits(a[3][:2]), _bits(b[3][:2]))
        nsym = iq.size // ((1 << sf) * osr)
        for n in (1, 3, nsym):  # estimate_offsets over n whole symbols
            seg = iq[: n * (1 << sf) * osr]
            np.testing.assert_array_equal(_bits(oracle.estimate_offsets(seg, sf, osr, hann)),
                                          _bits(reference.estimate_offsets(seg, sf, osr, hann)))
        for scratch in (True, False):
            a = oracle.lora_demodulate(iq, sf, osr=osr, hann=hann, scratch=scratch)
            b = reference.lora_demodulate(iq, sf, osr=osr, hann=hann, scratch=scratch)
            assert a[0] == b[0] and a[2] == b[2]
            np.testing.assert_array_equal(a[1], b[1])
            np.testing.assert_array_equal(_bits(a[3][:2]), _bits(b[3][:2]))


@pytest.mark.parametrize("sf,osr,amp", [(2, 2, 0.5), (7, 2, 0.25), (7, 4, 3.0), (10, 2, 1.0)])
def test_oversampled_power_tie(oracle, reference, sf, osr, amp):
    x = _tie_frame(sf, osr, 6, amp)
    a = oracle.demodulate(x, sf, osr=osr)
    b = reference.demodulate(x, sf, osr=osr)
    np.testing.assert_array_equal(a[1], b[1])
    np.testing.assert_array_equal(_bits(a[3][:2]), _bits(b[3][:2]))
    a1 = oracle.lora_demodulate(x, sf, osr=osr)
    b1 = reference.lora_demodulate(x, sf, osr=osr)
    np.testing.assert_array_equal(a1[1], b1[1])
    np.testing.assert_array_equal(_bits(a1[3][:2]), _bits(b1[3][:2]))
    # the two tie rules pick different phases here
    assert _bits(a[3][1]) != _bits(a1[3][1])


# Non-finite samples: GCC's std::complex<float> product calls __mulsc3 when
# both result parts are NaN (C99 Annex G recovery of infinities), in the
# dechirp, the rotation and every KISS butterfly.  The oracle restates it.
NONFINITE = [(complex(-np.inf, np.nan)), complex(np.inf, 0.25), complex(np.inf, np.inf),
             complex(np.nan, 3.0), complex(0.5, np.nan), complex(-np.inf, -np.inf),
             complex(3e38, 3e38), complex(np.nan, np.inf)]


def _nan_bits_equal(a, b):
    a = np.asarray(a, np.float32).reshape(-1)
    b = np.asarray(b, np.float32).reshape(-1)
    na, nb = np.isnan(a), np.isnan(b)
    np.testing.assert_array_equal(na, nb)
    np.testing.assert_array_equal(a[~na].view(np.uint32), b[~nb].view(np.uint32))


def _nonfinite_frames(oracle, sf, rng):
    base = _frame(oracle, rng, sf, 125000, 8)
    out = []
    for v in NONFINITE:
        for pos in (3, (1 << sf) + 5, base.size - 7):
            x = base.copy()
            x[pos] = v
            out.append(x)
    return out


@pytest.mark.parametrize("sf", [2, 7, 8])
def test_nonfinite_samples_bit_exact(oracle, reference, sf):
    rng = np.random.default_rng(900 + sf)
    for iq in _nonfinite_frames(oracle, sf, rng):
        a = oracle.demodulate(iq, sf)
        b = reference.demodulate(iq, sf)
        assert a[0] == b[0] and a[2] == b[2]
        np.testing.assert_array_equal(a[1], b[1])
        _nan_bits_equal(a[3][:2], b[3][:2])
        x = oracle.dechirp(iq, sf, 125000)
        _nan_bits_equal(x.view(np.float32), reference.dechirp(iq, sf, 125000).view(np.float32))
        for inp in (x, iq):
            a = oracle.lora_demodulate(inp, sf)
            b = reference.lora_demodulate(inp, sf)
            assert a[0] == b[0] and a[2] == b[2]
            np.testing.assert_array_equal(a[1], b[1])
            _nan_bits_equal(a[3][:2], b[3][:2])
        # FFT bins bit for bit, except that a NaN's sign/payload follows the
        # host's operand order (x86 keeps the first NaN operand); NaN
        # positions must agree
        fa, fb = oracle.fft(iq[: 1 << sf]), reference.fft(iq[: 1 << sf])
        _nan_bits_equal(fa.view(np.float32), fb.view(np.float32))


COMP_CASES = [  # sf, osr, cfo, time_offset
    (7, 1, 0.37, 95.54), (7, 1, -0.21, -12.4), (8, 1, 0.0, 0.0), (9, 2, 0.45, 300.2),
    (12, 1, -0.5, 1e9), (7, 1, 3.0, -2.6e9), (5, 4, 0.1, float("nan")), (10, 1, 1e-4, 0.49)]


@pytest.mark.parametrize("sf,osr,cfo,toff", COMP_CASES)
def test_compensate_offsets_bit_exact(oracle, reference, sf, osr, cfo, toff):
    """phy.cpp:150-180: rotation by -2 pi cfo n / (N osr), then the integer
    shift by round(time_offset) (no shift when it is out of range or NaN)."""
    rng = np.random.default_rng(sf * 13 + osr)
    x = _iq(rng, 7 * (1 << sf) * osr, scale=2.0)
    x[3] = complex(np.inf, 0.5)  # Annex G product inside the rotation
    _nan_bits_equal(oracle.compensate_offsets(x, sf, cfo, toff, osr).view(np.float32),
                    reference.compensate_offsets(x, sf, cfo, toff, osr).view(np.float32))


# ---- LoRaCodes.hpp helpers: oracle vs the reference header
def test_codes_gray_and_hamming_exhaustive(oracle, reference):
    for v in range(0, 65536, 7):
        for tb in (0, 1):
            assert oracle.gray(v, tb) == reference.gray(v, tb)
    for x in range(256):
        for op in range(8):
            assert oracle.hamming(x, op) == reference.hamming(x, op), (x, op)


@pytest.mark.parametrize("ppm,rdd", [(p, r) for p in (5, 7, 8, 10, 12) for r in (0, 1, 2, 4)])
def test_codes_interleaver(oracle, reference, ppm, rdd):
    rng = np.random.default_rng(ppm * 10 + rdd)
    cw = rng.integers(0, 1 << (4 + rdd), 3 * ppm + 2, dtype=np.uint8)
    a, b = oracle.interleave(cw, ppm, rdd), reference.interleave(cw, ppm, rdd)
    np.testing.assert_array_equal(a, b)
    syms = rng.integers(0, 1 << ppm, 3 * (4 + rdd) + 1, dtype=np.uint16)
    np.testing.assert_array_equal(oracle.deinterleave(syms, ppm, rdd), reference.deinterleave(syms, ppm, rdd))
    # round trip of whole blocks
    np.testing.assert_array_equal(oracle.deinterleave(a, ppm, rdd), cw[: len(a) // (4 + rdd) * ppm])


@pytest.mark.parametrize("kind", [0, 1, 2])
def test_codes_whitening_and_checksums(oracle, reference, kind):
    rng = np.random.default_rng(40 + kind)
    for rdd in (0, 1, 2, 3, 4):
        for bit_ofs in (0, 1, 7, 100):
            buf = rng.integers(0, 256, 255, dtype=np.uint8)
            np.testing.assert_array_equal(oracle.whiten(buf, kind, bit_ofs, rdd),
                                          reference.whiten(buf, kind, bit_ofs, rdd))
    for n in (0, 1, 2, 5, 64, 255):
        buf = rng.integers(0, 256, max(n, 2), dtype=np.uint8)[: max(n, 2)]
        assert oracle.checksum(buf[:n] if kind != 1 else buf, kind) == \
            reference.checksum(buf[:n] if kind != 1 else buf, kind)
    # whitening_test.cpp:30-31 known answer
    w = oracle.whiten(np.frombuffer(bytes.fromhex("DEADBEEF700D"), np.uint8), 2, 0, 4)
    assert w.tobytes() == bytes.fromhex("215290102CF2")
