"""GPU parity: the HIP path (through the C ABI) against the CPU oracle on the
same inputs.  Bit-exact on every integer output (symbol indices, sync word,
decoded bytes, CRC flag, return status) and on the float32 bit patterns of
the per-frame cfo / time_offset estimates."""
import numpy as np
import torch
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
    (12, 125000, 3, 16, 0.0, 0, True),
    (5, 125000, 3, 8, None, 0, False),
    (6, 250000, 3, 8, 3.0, 0, False),
]


# launch paths: the fused single launch (default, SF <= 10) and the
# separate prologue / symbol kernels
LAUNCH = [0, 32]


@pytest.mark.parametrize("sf,bw,nf,plen,snr,delay,hann", CASES)
@pytest.mark.parametrize("launch", LAUNCH)
def test_mode_demodulate_vs_oracle(oracle, lphy, sf, bw, nf, plen, snr, delay, hann, launch):
    """lora_phy::demodulate + decode (phy.cpp:182-261) per frame."""
    iq, _ = _frames(oracle, sf, bw, nf, plen, seed=sf * 100 + nf, snr_db=snr, delay=delay)
    d = lphy.Demodulator(sf, bw, 1, lphy.WINDOW_HANN if hann else lphy.WINDOW_NONE)
    fs = iq.shape[1]
    syms, pay, meta = d.demod_host(iq, nf, fs, lphy.MODE_DEMODULATE, lphy.F_DECODE | launch)
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
@pytest.mark.parametrize("launch", LAUNCH)
def test_mode_lora_demodulate_vs_oracle(oracle, lphy, sf, bw, nf, plen, snr, delay, hann, fused,
                                        launch):
    """external dechirp -> lora_demodulate -> lora_decode (LoRaDemod.cpp:50-197)."""
    iq, payloads = _frames(oracle, sf, bw, nf, plen, seed=sf * 7 + nf, snr_db=snr, delay=delay)
    dech = np.stack([oracle.dechirp(x, sf, bw) for x in iq])
    d = lphy.Demodulator(sf, bw, 1, lphy.WINDOW_HANN if hann else lphy.WINDOW_NONE)
    fs = iq.shape[1]
    mode = lphy.MODE_DECHIRP_LORA_DEMODULATE if fused else lphy.MODE_LORA_DEMODULATE
    syms, pay, meta = d.demod_host(iq if fused else dech, nf, fs, mode, lphy.F_DECODE | launch)
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


@pytest.mark.parametrize("sf,osr,nf,nsyms", [(7, 1, 1, 64), (7, 1, 5, 64), (8, 1, 3, 64), (9, 1, 2, 64),
                                              (5, 3, 4, 21), (7, 2, 2, 30), (3, 3, 3, 7), (2, 1, 2, 5),
                                              (10, 1, 2, 64), (7, 1, 70, 64), (11, 2, 2, 30), (12, 1, 3, 20)])
def test_modulate_batch_frames(oracle, lphy, sf, osr, nf, nsyms):
    """lphy_hip_modulate_batch, frame by frame == the oracle: k_mod_fast (f
    rows in LDS: up to SF 9 at 66 symbols, few frames, osr 2-3 too), its
    split form with the rows interleaved in the phase buffer (SF 10-12,
    several frames, osr 2 at SF 11) and the batch form (70 frames)."""
    rng = np.random.default_rng(sf * 100 + nf)
    syms = rng.integers(0, 1 << min(sf, 8), (nf, nsyms), dtype=np.uint16)
    d = lphy.Demodulator(sf, 125000, osr)
    dev = torch.device("cuda", 0)
    step = (1 << sf) * osr
    iq = torch.zeros(nf * (nsyms + 2) * step * 2, dtype=torch.float32, device=dev)
    s_t = torch.from_numpy(syms.reshape(-1).astype(np.int16)).to(dev)
    d.modulate_batch(s_t, nf, nsyms, iq, 1.0, 0x34, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = iq.cpu().numpy().view(np.complex64).reshape(nf, -1)
    for f in range(nf):
        b = oracle.modulate(syms[f], sf, osr=osr, sync=0x34)
        np.testing.assert_array_equal(got[f].view(np.uint32), b.view(np.uint32), err_msg=f"frame {f}")


@pytest.mark.parametrize("sf", [5, 6, 7, 8, 9, 10, 11, 12])
def test_modulate_candidate_chain(oracle, lphy, sf):
    """The one-launch modulator (k_mod_fast: candidate windows around each
    symbol's pivot, chained by lookups; f rows in LDS up to SF 9, in the
    phase buffer from SF 10) == the oracle's serial walk, every float bit,
    over random packets and constant-symbol ones (all 0, all N-1, a repeated
    value); and the chain, not its serial fallback, is what ran for nearly
    every packet (lphy_hip_test_counter kCtrModSerial)."""
    rng = np.random.default_rng(sf * 31)
    N = 1 << sf
    d = lphy.Demodulator(sf, test_build=True)
    d.mod_serial_count(reset=True)
    packets = [rng.integers(0, N, 64, dtype=np.uint16) for _ in range(40 if sf <= 9 else 15)]
    packets += [np.zeros(64, np.uint16), np.full(64, N - 1, np.uint16), np.full(30, N // 3, np.uint16),
                rng.integers(0, N, 200, dtype=np.uint16), rng.integers(0, N, 1, dtype=np.uint16)]
    for k, syms in enumerate(packets):
        a = d.modulate_host(syms, 1.0, 0x34)
        b = oracle.modulate(syms, sf, sync=0x34)
        np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32), err_msg=f"packet {k}")
    slow = d.mod_serial_count()
    assert slow <= len(packets) // 10, f"{slow} of {len(packets)} packets took the serial walk"


@pytest.mark.parametrize("sf,osr", [(5, 1), (7, 1), (8, 1), (9, 1), (10, 1), (12, 1), (7, 2), (5, 3), (9, 2)])
def test_modulate_forced_serial_fallback(oracle, lphy, sf, osr):
    """k_mod_fast's serial fallback (the whole frame walked in order by one
    thread, taken when a candidate chain leaves its windows) forced for
    every packet by the test build's switch: every float bit == the oracle's,
    and the fallback counter counts every packet."""
    rng = np.random.default_rng(sf * 7 + osr)
    N = 1 << sf
    d = lphy.Demodulator(sf, 125000, osr, test_build=True)
    d.mod_force_serial(True)
    d.mod_serial_count(reset=True)
    packets = [rng.integers(0, N, 64, dtype=np.uint16) for _ in range(3)] + [np.zeros(5, np.uint16)]
    for k, syms in enumerate(packets):
        a = d.modulate_host(syms, 1.0, 0x34)
        b = oracle.modulate(syms, sf, osr=osr, sync=0x34)
        np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32), err_msg=f"packet {k}")
    assert d.mod_serial_count() == len(packets)
    d.mod_force_serial(False)
    a = d.modulate_host(packets[0], 1.0, 0x34)
    np.testing.assert_array_equal(a.view(np.uint32), oracle.modulate(packets[0], sf, osr=osr, sync=0x34).view(np.uint32))
    assert d.mod_serial_count() == 0


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


@pytest.mark.parametrize("sf,nf", [(7, 3001), (8, 1203), (9, 517), (10, 129), (5, 2049)])
def test_large_batch_fused_equals_unfused(oracle, lphy, sf, nf):
    """Many frames through the fused ticket scheduler (look-ahead, partial
    groups, waits) against the separate launches, every output bit; the
    first frames also against the oracle.  Frames get random CFO-like
    rotations, delays and noise so that normalisation, offsets and the
    large-phase sincos branch all occur."""
    rng = np.random.default_rng(sf * 1000 + nf)
    N = 1 << sf
    base = oracle.modulate(oracle.encode(bytes(range(16))), sf)
    fs = base.size
    t = np.arange(fs, dtype=np.float64)
    iq = np.empty((nf, fs), np.complex64)
    for f in range(nf):
        x = base * np.exp(2j * np.pi * rng.uniform(-0.4, 0.4) / N * t)
        x = np.roll(x, int(rng.integers(0, 4)))
        sig = [0.0, 0.05, 0.5, 2.0][f % 4]
        x = x + sig * (rng.standard_normal(fs) + 1j * rng.standard_normal(fs))
        iq[f] = (x * [1.0, 0.5, 3.0][f % 3]).astype(np.complex64)
    d = lphy.Demodulator(sf)
    for mode in (lphy.MODE_DEMODULATE, lphy.MODE_DECHIRP_LORA_DEMODULATE):
        a = d.demod_host(iq, nf, fs, mode, lphy.F_DECODE)
        b = d.demod_host(iq, nf, fs, mode, lphy.F_DECODE | lphy.F_UNFUSED)
        np.testing.assert_array_equal(a[0], b[0])
        np.testing.assert_array_equal(a[1], b[1])
        np.testing.assert_array_equal(a[2].view(np.uint8), b[2].view(np.uint8))
    for f in range(4):
        r, osyms, osync, omet = oracle.lora_demodulate(oracle.dechirp(iq[f], sf, 125000), sf)
        np.testing.assert_array_equal(a[0][f], osyms)
        assert _bits(a[2]["cfo"][f]) == _bits(omet[0])


def test_fused_no_scratch_mixed(oracle, lphy):
    """-ERANGE frames (rescale needed, no scratch) interleaved with normal
    ones in one fused batch."""
    sf, N = 7, 128
    base = oracle.modulate(oracle.encode(bytes(range(8))), sf)
    fs = base.size
    nf = 37
    iq = np.stack([base * (2.0 if f % 3 == 1 else 0.9) for f in range(nf)]).astype(np.complex64)
    d = lphy.Demodulator(sf)
    for flags in (lphy.F_NO_SCRATCH, lphy.F_NO_SCRATCH | lphy.F_UNFUSED):
        syms, _, meta = d.demod_host(iq, nf, fs, lphy.MODE_DECHIRP_LORA_DEMODULATE, flags)
        for f in range(nf):
            dech = oracle.dechirp(iq[f], sf, 125000)
            if f % 3 == 1:
                assert meta["status"][f] == -34
            else:
                assert meta["status"][f] == 0
                r, osyms, osync, omet = oracle.lora_demodulate(dech, sf)
                np.testing.assert_array_equal(syms[f], osyms)


def test_nonfinite_frames_maxabs(oracle, lphy):
    """The fused max-abs scan's fast form (v_max3 + NaN sentinel) against the
    reference's per-sample fold (LoRaDemod.cpp:62-66) on frames carrying a
    NaN real part beside a large imaginary part (the sample is hidden), a
    NaN imaginary part (the real part still counts), inf, values whose
    dechirp overflows, and a NaN in the partial-symbol tail (scanned only
    without the fused dechirp).  Both normalising modes, fused and separate
    launches, every output against the oracle."""
    sf, N = 7, 128
    base = oracle.modulate(oracle.encode(bytes(range(16))), sf)
    tail = 5
    fs = base.size + tail
    frames = []
    for k in range(8):
        x = np.concatenate([base * 0.8, np.zeros(tail, np.complex64)]).astype(np.complex64)
        if k == 1:
            x[300] = np.complex64(complex(np.nan, 5.0))
        elif k == 2:
            x[301] = np.complex64(complex(3.0, np.nan))
        elif k == 3:
            x[4000] = np.complex64(complex(np.inf, 0.25))
        elif k == 4:
            x[777] = np.complex64(complex(3.0e38, -3.0e38))
        elif k == 5:
            x[fs - 2] = np.complex64(complex(np.nan, 7.0))
        elif k == 6:
            x[fs - 1] = np.complex64(complex(9.0, 0.0))
        elif k == 7:
            x[40] = np.complex64(complex(-np.inf, np.nan))
        frames.append(x)
    iq = np.stack(frames)
    nf = iq.shape[0]
    d = lphy.Demodulator(sf)
    for mode in (lphy.MODE_LORA_DEMODULATE, lphy.MODE_DECHIRP_LORA_DEMODULATE):
        # the fused dechirp takes whole symbols only (-EINVAL otherwise)
        x = iq if mode == lphy.MODE_LORA_DEMODULATE else np.ascontiguousarray(iq[:, :base.size])
        for flags in (0, lphy.F_UNFUSED):
            syms, _, meta = d.demod_host(x, nf, x.shape[1], mode, flags)
            for f in range(nf):
                src = x[f] if mode == lphy.MODE_LORA_DEMODULATE else oracle.dechirp(x[f], sf)
                r, osyms, osync, omet = oracle.lora_demodulate(src, sf)
                ctx = f"mode {mode} flags {flags} frame {f}"
                assert meta["status"][f] == 0, ctx
                np.testing.assert_array_equal(syms[f], osyms, err_msg=ctx)
                assert _bits(meta["cfo"][f]) == _bits(omet[0]), ctx
                assert _bits(meta["time_offset"][f]) == _bits(omet[1]), ctx


@pytest.mark.parametrize("sf,nf,S", [(7, 2048 * 5 + 123, 19), (8, 2048 * 3 + 77, 11), (6, 2048 * 3 + 5, 33)])
def test_fused_frame_groups(oracle, lphy, sf, nf, S):
    """k_frames' frame groups (F = WT/2 frames share estimate-only tiles):
    several groups per wave, a partial last group, and S with F*S not a
    multiple of the tile (dead padding units), fused against the separate
    launches on every output bit, the first frames against the oracle."""
    rng = np.random.default_rng(sf * 7 + nf)
    N = 1 << sf
    base = oracle.modulate(oracle.encode(bytes(range(S // 2 - 1 if S % 2 == 0 else S // 2))), sf)
    fs = S * N
    base = np.resize(base, fs).astype(np.complex64)
    t = np.arange(fs, dtype=np.float32)
    cfo = rng.uniform(-0.4, 0.4, nf).astype(np.float32)
    iq = base[None, :] * np.exp((2j * np.pi / N) * cfo[:, None] * t[None, :]).astype(np.complex64)
    sig = np.array([0.0, 0.05, 0.5, 2.0], np.float32)[np.arange(nf) % 4]
    iq += sig[:, None] * (rng.standard_normal((nf, fs), np.float32) +
                          1j * rng.standard_normal((nf, fs), np.float32)).astype(np.complex64)
    iq *= np.array([1.0, 0.5, 3.0], np.float32)[np.arange(nf) % 3][:, None]
    iq = np.ascontiguousarray(iq.astype(np.complex64))
    d = lphy.Demodulator(sf)
    for mode in (lphy.MODE_DEMODULATE, lphy.MODE_DECHIRP_LORA_DEMODULATE):
        a = d.demod_host(iq, nf, fs, mode, 0)
        b = d.demod_host(iq, nf, fs, mode, lphy.F_UNFUSED)
        np.testing.assert_array_equal(a[0], b[0])
        np.testing.assert_array_equal(a[2].view(np.uint8), b[2].view(np.uint8))
    for f in (0, 1, nf - 1):
        r, osyms, osync, omet = oracle.lora_demodulate(oracle.dechirp(iq[f], sf, 125000), sf)
        np.testing.assert_array_equal(a[0][f], osyms)
        assert _bits(a[2]["cfo"][f]) == _bits(omet[0])


@pytest.mark.parametrize("n", [8, 64, 66, 130, 512])
def test_decode_finalize_vs_oracle(oracle, lphy, n):
    """The finalisation's decode (Hamming 8,4 syndromes as parities, 16-byte
    symbol loads with a scalar tail) and its byte-wise SX1272 checksum
    against the oracle (LoRaDecoder.cpp:7-21, LoRaCodes.hpp:69-105, 250-281);
    every low-byte value occurs in both nibble positions."""
    rng = np.random.default_rng(n)
    d = lphy.Demodulator(7)
    for rep in range(4):
        syms = rng.integers(0, 1 << 16, n, dtype=np.uint16)
        if rep == 0:
            syms[: min(n, 256)] = np.arange(min(n, 256), dtype=np.uint16) * 257
        rc, out, meta = d.decode_host(syms)
        r, obytes, ocrc = oracle.decode(syms)
        assert rc == 0 and r == n // 2
        np.testing.assert_array_equal(out, obytes)
        assert meta["crc_ok"] == ocrc


@pytest.mark.parametrize("sf,mode", [(11, 0), (12, 0), (11, 1)])
def test_separate_launch_rechecks_stable(oracle, lphy, sf, mode):
    """k_demod (SF 11-12) with many symbols left to k_post's exact re-check:
    a workgroup that reads its frame record after another one flagged the
    frame (kStatusRecheck) must still demodulate its own symbol (k_post
    recomputes the sentinels only).  Repeated runs agree bit for bit, and
    sampled frames match the oracle."""
    rng = np.random.default_rng(sf * 10 + mode)
    N = 1 << sf
    nf = 96
    base = oracle.modulate(oracle.encode(bytes(range(32))), sf)
    fs = base.size
    t = np.arange(fs, dtype=np.float32)
    cfo = rng.uniform(-0.4, 0.4, nf).astype(np.float32)
    iq = base[None, :] * np.exp((2j * np.pi / N) * cfo[:, None] * t[None, :]).astype(np.complex64)
    sig = np.float32(np.sqrt(10 ** 1.2 / 2))  # -12 dB: near-ties, many re-checks
    iq += sig * (rng.standard_normal((nf, fs), np.float32) +
                 1j * rng.standard_normal((nf, fs), np.float32)).astype(np.complex64)
    iq = np.ascontiguousarray(iq.astype(np.complex64))
    d = lphy.Demodulator(sf)
    runs = [d.demod_host(iq, nf, fs, mode, lphy.F_DECODE) for _ in range(4)]
    for r in runs[1:]:
        np.testing.assert_array_equal(r[0], runs[0][0])
        np.testing.assert_array_equal(r[2].view(np.uint8), runs[0][2].view(np.uint8))
    for f in (0, 1, nf // 2, nf - 1):
        if mode == 0:
            r, osyms, osync, omet = oracle.demodulate(iq[f], sf)
        else:
            r, osyms, osync, omet = oracle.lora_demodulate(iq[f], sf)
        np.testing.assert_array_equal(runs[0][0][f], osyms, err_msg=f"frame {f}")


@pytest.mark.parametrize("per,nf", [(64, 300), (60, 300), (8, 513), (6, 5)])
def test_decode_batch_rows_vs_oracle(oracle, lphy, per, nf):
    """lphy_hip_decode_batch (k_finalize) over whole workgroups of rows:
    rows of 8k symbols go through the LDS-staged block form (a partial last
    workgroup included), others through the row-per-thread form; rows whose
    record carries a non-zero status are left untouched (bytes and record),
    as the per-row form leaves them.  Every decoded row and CRC flag against
    the oracle (LoRaDecoder.cpp:7-21, LoRaCodes.hpp:69-105, 250-281)."""
    import torch
    rng = np.random.default_rng(per * 1000 + nf)
    d = lphy.Demodulator(7)
    dev = torch.device("cuda:0")
    syms = rng.integers(0, 1 << 16, (nf, per), dtype=np.uint16)
    syms[::7, :] = rng.integers(0, 256, (len(syms[::7]), per), dtype=np.uint16)  # clean low bytes too
    meta = np.zeros(nf, lphy.META_DTYPE)
    skip = rng.random(nf) < 0.1
    meta["status"][skip] = -34
    meta["crc_ok"] = 7
    t_syms = torch.from_numpy(syms.view(np.int16).reshape(-1).copy()).to(dev)
    t_pay = torch.full((nf * (per // 2),), 0xAB, dtype=torch.uint8, device=dev)
    t_meta = torch.from_numpy(meta.view(np.uint8).reshape(-1).copy()).to(dev)
    d.decode_batch(t_syms, nf, per, t_pay, t_meta, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    pay = t_pay.cpu().numpy().reshape(nf, per // 2)
    out = t_meta.cpu().numpy().view(lphy.META_DTYPE)
    for f in range(nf):
        if skip[f]:
            assert (pay[f] == 0xAB).all() and out["crc_ok"][f] == 7 and out["status"][f] == -34
            continue
        r, obytes, ocrc = oracle.decode(syms[f])
        assert r == per // 2
        np.testing.assert_array_equal(pay[f], obytes)
        assert out["crc_ok"][f] == ocrc and out["status"][f] == 0
