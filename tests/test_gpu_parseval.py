"""The Parseval certificate of the wave kernel (csrc/lphy_wave.h, k_wave,
SF 7-12; SF 7-9 with units spanning frames): a symbol unit whose every symbol carries most of its
energy in one bin is proven from that bin and the symbol's energy alone,
without its FFT (|Y_k| - sqrt(N E - |Y_k|^2) > 4 B); any other unit runs the
transform and the runner-up certificate, and whatever neither proves is
re-run exactly (k_post).  These tests pin each branch:

* the runner-up straddle: one frame per call, every data symbol two pure
  tones with a constant amplitude ratio r, r - 1 swept geometrically
  across the runner-up bound (two comparable tones give Parseval no
  candidate): frames above it are certified by the transform, frames
  below re-run every data symbol exactly;
* the Parseval straddle: one clean tone plus a half-symbol tone that adds
  energy but nothing to the winner's bin, swept so the exact Parseval lead
  crosses 4 B: frames well above it are proven by Parseval entirely, frames
  below take the transform;
* three tones (a main tone and two side tones of 0.8 of its amplitude):
  less than half the energy in the winner, so Parseval cannot prove it,
  while the runner-up certificate can: the transform path takes over and
  nothing is re-run;
* AWGN frames across SNRs (every path mixed).
Every output bit is compared with the oracle (LoRaDemod.cpp:50-197,
phy.cpp:182-243).  The Parseval count is the test build's counter
(lphy_hip_test_counter), the re-runs lphy_hip_recheck_count."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _bits(x):
    return np.asarray(x, np.float32).view(np.uint32)


def _tones_frame(oracle, sf, gains, seed, cfo=0.2, roll=True):
    """One frame whose every data symbol is len(gains) tones (distinct
    random bins) with relative amplitudes `gains` (a callable of the symbol
    index giving the list), under a small CFO and delay."""
    rng = np.random.default_rng(seed)
    N = 1 << sf
    S = 64
    base = rng.integers(0, N, S)
    x = None
    g0 = gains(0)
    for t in range(len(g0)):
        # side tone t in its own part of the spectrum (never on another tone)
        off = 0 if t == 0 else int(rng.integers((2 * t - 1) * N // 8, 2 * t * N // 8 + 1))
        syms = ((base + off) % N).astype(np.uint16)
        xt = oracle.modulate(syms, sf).astype(np.complex128)
        g = np.ones(xt.size)
        for s in range(S):
            g[(s + 2) * N:(s + 3) * N] = gains(s)[t]
        if t > 0:
            g[:2 * N] = 0.0  # the sync symbols: one tone
        x = xt * g if x is None else x + xt * g
    n = np.arange(x.size)
    x = x * np.exp(2j * np.pi * rng.uniform(-cfo, cfo) / N * n)
    if roll:
        x = np.roll(x, int(rng.integers(-N // 8, N // 8 + 1)))
    return x.astype(np.complex64)


def _check_one(oracle, sf, x, mode, syms, meta, ctx):
    if mode == 0:
        r, osyms, osync, omet = oracle.demodulate(x, sf)
    else:
        src = x if mode == 1 else oracle.dechirp(x, sf)
        r, osyms, osync, omet = oracle.lora_demodulate(src, sf)
    assert meta["status"][0] == 0, ctx
    np.testing.assert_array_equal(syms[0], osyms, err_msg=ctx)
    assert meta["sync_word"][0] == osync, ctx
    assert _bits(meta["cfo"][0]) == _bits(omet[0]), ctx
    assert _bits(meta["time_offset"][0]) == _bits(omet[1]), ctx


def _product_one(oracle, dp, sf, x, mode, ctx):
    """The same frame through the product library (lib/liblphy_hip.so, the
    fused kernel the tests force with fused_min_frames 0): every output bit
    against the oracle; returns its exact re-run count."""
    dp.recheck_count(reset=True)
    syms, _, meta = dp.demod_host(x[None, :], 1, x.size, mode, 0x1)  # F_DECODE
    n = dp.recheck_count(reset=True)
    _check_one(oracle, sf, x, mode, syms, meta, ctx)
    return n


def _pure_tone_frame(sf, amps, gains, seed, nsym=64):
    """Mode-1 input (dechirped samples) built directly: two sync symbols of
    one tone each, then data symbols of len(amps) pure integer tones at
    distinct random bins, tone t of symbol s with amplitude amps[t] *
    gains(s)[t].  No wrap-around phase step (a modulated chirp's dechirp
    has one, which leaks energy out of the peak and breaks an amplitude
    tie), so the peaks are the amplitudes times N."""
    rng = np.random.default_rng(seed)
    N = 1 << sf
    n = np.arange(N)
    tone = lambda k: np.exp(2j * np.pi * k * n / N)
    # both sync symbols at bin 0: the estimate (LoRaDemod.cpp:80-136) then
    # finds cfo 0 and time offset 0, so the data tones stay on integer bins
    # (a fractional rotation would leak each tone into the others' bins and
    # break a tie by far more than the sweeps' ratios)
    out = [tone(0), tone(0)]
    for s in range(nsym):
        bins = rng.choice(N, len(amps), replace=False)
        g = gains(s)
        out.append(sum(amps[t] * g[t] * tone(int(bins[t])) for t in range(len(amps))))
    return np.concatenate(out).astype(np.complex64)


@pytest.mark.parametrize("sf", [7, 8, 9, 10, 11, 12])
def test_runner_up_threshold_straddled(oracle, lphy, sf):
    """One frame per call (mode 1), every data symbol two pure tones at a
    constant amplitude ratio r.  Two comparable tones give the Parseval
    certificate no candidate (their lag autocorrelations average the two
    frequencies) and no lead beyond the runner-up's, so these symbols go to
    the transform: above the runner-up bound every symbol is certified,
    below it every data symbol is re-run exactly; the switch lies where
    |X_a| - |X_b| = N (r - 1) / 2 meets 4 B."""
    d = lphy.Demodulator(sf, test_build=True)
    dp = lphy.Demodulator(sf)  # the product library's code objects, same frames
    ks = 2.0 ** np.linspace(-22, -8, 29)
    rows = []
    for i, k in enumerate(ks):
        x = _pure_tone_frame(sf, [0.5, 0.5], lambda s, k=k: [1.0, (1.0 + k) if s % 2 else 1.0 / (1.0 + k)],
                             seed=7000 + 31 * sf + i)
        d.recheck_count(reset=True)
        d.parseval_count(reset=True)
        syms, _, meta = d.demod_host(x[None, :], 1, x.size, 1, lphy.F_DECODE)
        n_exact, n_pv = d.recheck_count(reset=True), d.parseval_count(reset=True)
        _check_one(oracle, sf, x, 1, syms, meta, f"sf {sf} r-1 {k:.3g}")
        n_prod = _product_one(oracle, dp, sf, x, 1, f"product sf {sf} r-1 {k:.3g}")
        rows.append((k, n_exact, n_pv, n_prod))
    assert d.bounds_violations() == 0
    msg = "\n".join(f"r-1 {k:.3g}: exact {n} parseval {p} product exact {q}" for k, n, p, q in rows)
    # the product build takes the same decisions: the same symbols re-run
    assert all(n == q for _, n, _, q in rows), msg
    rows = [r[:3] for r in rows]
    certified = [k for k, n, p in rows if n == 0]
    rerun = [k for k, n, p in rows if n == 64]
    assert certified and rerun, msg
    assert max(rerun) < min(certified) < 2.0 ** -9, msg
    assert all(p <= 2 for _, _, p in rows), msg  # Parseval: the one-tone sync symbols at most


KU = 2.0 ** -24


def _burst_frame(sf, c, seed, a=0.3, nsym=64):
    """Mode-1 input: sync symbols at bin 0 (cfo 0, time offset 0), then data
    symbols of one tone (amplitude a, random bin k) plus, in the symbol's
    second half only, a tone of amplitude c at a bin j = k + 2m (m != 0).
    A half-symbol tone at an even distance from k has no projection on bin
    k, so |Y_k| = N a exactly, while it adds N c^2 / 2 to N E: the Parseval
    lead is N (a - c / sqrt 2) for every symbol.  The candidate reads the
    first eighth (lag 1) and quarter (lag LPS) of each symbol, where the
    tone is clean; the transform's runner-up (~ N c / 2) stays far below
    N a, so the runner-up certificate holds throughout."""
    rng = np.random.default_rng(seed)
    N = 1 << sf
    n = np.arange(N)
    out = [np.ones(N), np.ones(N)]
    for s in range(nsym):
        k = int(rng.integers(0, N))
        m = int(rng.integers(1, N // 2 - 1))
        j = (k + 2 * m) % N
        y = a * np.exp(2j * np.pi * k * n / N)
        y[N // 2:] += c * np.exp(2j * np.pi * j * n[N // 2:] / N)
        out.append(y)
    return np.concatenate(out).astype(np.complex64)


def _parseval_leads(x, sf):
    """Per data symbol: the exact Parseval lead of the normalised samples
    (LoRaDemod.cpp:60-78's max-abs scale; cfo 0, so no rotation) and the
    runner-up certificate's bound B (cert_bound with kWaveExtra, rate 0)."""
    N = 1 << sf
    xd = x.astype(np.complex128)
    mx = max(np.abs(x.real).max(), np.abs(x.imag).max())
    scale = 1.0 / np.float32(mx) if mx > 1.0 else 1.0
    y = xd[2 * N:].reshape(-1, N) * np.float64(np.float32(scale))
    Y = np.fft.fft(y, axis=1)
    P = np.abs(Y) ** 2
    k = P.argmax(axis=1)
    yk = np.sqrt(P[np.arange(len(k)), k])
    lead = yk - np.sqrt(np.maximum(N * (np.abs(y) ** 2).sum(axis=1) - yk ** 2, 0.0))
    L = (sf + 1) // 2
    A = N * np.sqrt(2.0)
    B = KU * A * (24 + 12 * L + 64) * 1.001
    return lead, B, A


@pytest.mark.parametrize("sf", [7, 8, 9, 10, 11, 12])
def test_parseval_threshold_straddled(oracle, lphy, sf):
    """One frame per call (mode 1), every data symbol a clean tone plus a
    half-symbol tone that adds energy but nothing to the winner's bin
    (_burst_frame), swept so the exact Parseval lead N a delta crosses the
    certificate's 4 B + the Parseval charges: frames whose every symbol leads by a clear margin are proven by
    Parseval entirely (66 symbols with the sync symbols), frames where some
    symbol's lead is below 4 B are not (their units take the transform,
    which certifies them: nothing is re-run).  Every output bit equals the
    oracle's."""
    d = lphy.Demodulator(sf, test_build=True)
    dp = lphy.Demodulator(sf)  # the product library's code objects, same frames
    a = 0.3
    rows = []
    for i, dl in enumerate(2.0 ** np.linspace(-20, -6, 43)):
        x = _burst_frame(sf, np.sqrt(2.0) * a * (1.0 - dl), seed=9000 + 31 * sf + i, a=a)
        d.recheck_count(reset=True)
        d.parseval_count(reset=True)
        syms, _, meta = d.demod_host(x[None, :], 1, x.size, 1, lphy.F_DECODE)
        n_exact, n_pv = d.recheck_count(reset=True), d.parseval_count(reset=True)
        _check_one(oracle, sf, x, 1, syms, meta, f"sf {sf} delta {dl:.3g}")
        assert _product_one(oracle, dp, sf, x, 1, f"product sf {sf} delta {dl:.3g}") == 0
        lead, B, A = _parseval_leads(x, sf)
        rows.append((dl, lead.min() / B, n_exact, n_pv))
    assert d.bounds_violations() == 0
    msg = "\n".join(f"delta {k:.3g}: min lead {r:.3g} B, exact {n}, parseval {p}" for k, r, n, p in rows)
    assert all(n == 0 for _, _, n, _ in rows), msg
    # the charges beyond 4 B: kPvErr u A on |Y_k| and E's 32 u, well inside 8 B
    proven = [r for _, r, _, p in rows if p == 66]
    short = [r for _, r, _, p in rows if p < 66]
    assert proven and short, msg
    assert all(p == 66 for _, r, _, p in rows if r > 8.0), msg
    assert all(p < 66 for _, r, _, p in rows if r < 4.0), msg


@pytest.mark.parametrize("sf", [7, 8, 9, 10, 11, 12])
def test_three_tones_take_the_transform(oracle, lphy, sf):
    d = lphy.Demodulator(sf, test_build=True)
    dp = lphy.Demodulator(sf)
    for i in range(3):
        x = _tones_frame(oracle, sf, lambda s: [1.0, 0.8, 0.8], seed=8000 + sf * 7 + i)
        d.recheck_count(reset=True)
        d.parseval_count(reset=True)
        syms, _, meta = d.demod_host(x[None, :], 1, x.size, 2, lphy.F_DECODE)
        n_exact, n_pv = d.recheck_count(reset=True), d.parseval_count(reset=True)
        _check_one(oracle, sf, x, 2, syms, meta, f"sf {sf} frame {i}")
        assert _product_one(oracle, dp, sf, x, 2, f"product sf {sf} frame {i}") == 0
        # Parseval proves the one-tone sync symbols at most (SF 12: its
        # units hold one symbol each); the data symbols: the transform
        assert n_pv <= 2 and n_exact == 0, (n_pv, n_exact)


@pytest.mark.parametrize("sf,nf", [(7, 3200), (8, 1600), (9, 800), (10, 400), (11, 200), (12, 100)])
@pytest.mark.parametrize("mode", [0, 2])
def test_awgn_mixed_paths(oracle, lphy, sf, nf, mode):
    """AWGN from 30 dB down to -10 dB per-sample SNR over the batch's frames
    (one SNR per frame): high-SNR frames take Parseval, low ones the
    transform (after one attempt per frame), near-ties the exact re-run."""
    N = 1 << sf
    rng = np.random.default_rng(900 + sf)
    base = oracle.modulate(oracle.encode(bytes(range(32))), sf).astype(np.complex128)
    n = np.arange(base.size)
    snrs = np.linspace(30, -10, nf)
    iq = np.zeros((nf, base.size), np.complex64)
    for f in range(nf):
        sig = np.sqrt(10 ** (-snrs[f] / 10) / 2)
        x = base * np.exp(2j * np.pi * rng.uniform(-0.3, 0.3) / N * n)
        x = x + sig * (rng.standard_normal(x.size) + 1j * rng.standard_normal(x.size))
        iq[f] = x.astype(np.complex64)
    dt = lphy.Demodulator(sf, test_build=True)
    dt.parseval_count(reset=True)
    got = dt.demod_host(iq, nf, iq.shape[1], mode, lphy.F_DECODE)
    n_pv = dt.parseval_count(reset=True)
    # the product library's fused launch over the same batch
    prod = lphy.Demodulator(sf).demod_host(iq, nf, iq.shape[1], mode, lphy.F_DECODE)
    # the separate launches (no Parseval) as the whole-batch reference
    ref = lphy.Demodulator(sf).demod_host(iq, nf, iq.shape[1], mode, lphy.F_DECODE | lphy.F_UNFUSED)
    for out in (got, prod):
        np.testing.assert_array_equal(out[0], ref[0])
        np.testing.assert_array_equal(out[1], ref[1])
        np.testing.assert_array_equal(out[2].view(np.uint8), ref[2].view(np.uint8))
    assert 0 < n_pv < nf * 66, n_pv
    for f in range(0, nf, max(1, nf // 25)):
        if mode == 0:
            r, osyms, osync, omet = oracle.demodulate(iq[f], sf)
        else:
            r, osyms, osync, omet = oracle.lora_demodulate(oracle.dechirp(iq[f], sf), sf)
        ctx = f"sf {sf} mode {mode} frame {f} snr {snrs[f]:.1f}"
        for out, who in ((got, "test build"), (prod, "product")):
            assert out[2]["status"][f] == 0, (who, ctx)
            np.testing.assert_array_equal(out[0][f], osyms, err_msg=f"{who} {ctx}")
            assert out[2]["sync_word"][f] == osync, (who, ctx)
            assert _bits(out[2]["cfo"][f]) == _bits(omet[0]), (who, ctx)
            assert _bits(out[2]["time_offset"][f]) == _bits(omet[1]), (who, ctx)


@pytest.mark.parametrize("sf,nf", [(11, 24), (12, 12)])
def test_hann_frames_take_the_wave_kernel(oracle, lphy, sf, nf):
    """Hann-windowed frames at SF 11-12 run on k_wave (round 6; SF 12 with
    three waves per workgroup, wave_wpb): the Parseval counter, which only
    k_wave's certificate moves, proves clean windowed symbols there, and
    every output bit equals the oracle's windowed lora_demodulate
    (LoRaDemod.cpp:16-24, 97-98) and the separate launches'."""
    rng = np.random.default_rng(4400 + sf)
    N = 1 << sf
    iq = []
    for f in range(nf):
        p = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
        x = oracle.modulate(oracle.encode(p), sf).astype(np.complex128)
        n = np.arange(x.size)
        x = x * np.exp(2j * np.pi * rng.uniform(-0.3, 0.3) / N * n) * [0.6, 1.0, 1.7][f % 3]
        iq.append(x.astype(np.complex64))
    iq = np.stack(iq)
    d = lphy.Demodulator(sf, window=lphy.WINDOW_HANN, test_build=True)
    d.parseval_count(reset=True)
    got = d.demod_host(iq, nf, iq.shape[1], 2, lphy.F_DECODE)
    n_pv = d.parseval_count(reset=True)
    prod = lphy.Demodulator(sf, window=lphy.WINDOW_HANN).demod_host(iq, nf, iq.shape[1], 2, lphy.F_DECODE)
    ref = lphy.Demodulator(sf, window=lphy.WINDOW_HANN).demod_host(iq, nf, iq.shape[1], 2,
                                                                   lphy.F_DECODE | lphy.F_UNFUSED)
    for out in (got, prod):
        np.testing.assert_array_equal(out[0], ref[0])
        np.testing.assert_array_equal(out[1], ref[1])
        np.testing.assert_array_equal(out[2].view(np.uint8), ref[2].view(np.uint8))
    # (a windowed tone keeps 2/3 of its energy in its bin, less the chirp's
    # wrap-around leak: a part of the units pass, SF 11 ~28 %; any means
    # k_wave ran)
    assert n_pv > 0, n_pv
    for f in range(0, nf, 4):
        r, osyms, osync, omet = oracle.lora_demodulate(oracle.dechirp(iq[f], sf), sf, hann=True)
        ctx = f"sf {sf} hann frame {f}"
        assert got[2]["status"][f] == 0, ctx
        np.testing.assert_array_equal(got[0][f], osyms, err_msg=ctx)
        assert got[2]["sync_word"][f] == osync, ctx
        assert _bits(got[2]["cfo"][f]) == _bits(omet[0]), ctx
        assert _bits(got[2]["time_offset"][f]) == _bits(omet[1]), ctx
