"""Adversarial near-ties for the certified fast path.

Symbol units of the fused kernels do not run KISS's exact arithmetic: they
rotate with a per-frame table and (k_wave2) 64th-root twiddles, and prove
the argmax with a certificate (|X_best| - 4B > |X_second|); a symbol the
certificate cannot prove is re-run exactly (k_post).  If the bound B were
too small, a near-tie could flip silently.  These frames are built to sit
on both sides of the threshold: every data symbol is two tones (symbols a
and b, the reference's strict `>` with the first maximum winning,
LoRaDetector.hpp:46-58) whose amplitude ratio is 1 + k 2^-23, k swept
geometrically from 1 to 2^10 over the frame's symbols, under CFO and delay.
Every output (symbols, sync word, cfo / time_offset bits) must equal the
oracle's, and lphy_hip_recheck_count must show the exact re-run fired.

Kernels: SF 7-8 k_frames (modes 1/2: symbol tiles on the matrix cores,
lphy_mfma.h, whose f16 roundings the certificate charges; mode 0 packed
f32); SF 9 k_wave2s, SF 11-12 k_wave (no window) and, with a Hann window,
k_frames (SF 9) or the separate launches' certified k_demod (SF 11-12)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _bits(x):
    return np.asarray(x, np.float32).view(np.uint32)


def _two_tone_frames(oracle, sf, nf, seed):
    rng = np.random.default_rng(seed)
    N = 1 << sf
    S = 64
    ks = np.unique(np.round(2.0 ** np.linspace(0, 10, S)).astype(np.int64))
    frames = []
    for f in range(nf):
        a = rng.integers(0, 256, S).astype(np.uint16) % N
        b = (a + rng.integers(1, N, S)).astype(np.uint16) % N
        xa = oracle.modulate(a, sf).astype(np.complex128)
        xb = oracle.modulate(b, sf).astype(np.complex128)
        # per-symbol amplitude ratio 1 + k 2^-23 (tone b larger or smaller)
        k = ks[(np.arange(S) + f) % ks.size]
        r = 1.0 + k * 2.0 ** -23
        gain_b = np.ones(xa.size)
        for s in range(S):
            gain_b[(s + 2) * N:(s + 3) * N] = r[s] if (s + f) % 2 else 1.0 / r[s]
        x = xa + xb * gain_b
        t = np.arange(x.size)
        x = x * np.exp(2j * np.pi * rng.uniform(-0.4, 0.4) / N * t) * [0.7, 1.0, 1.9][f % 3]
        x = np.roll(x, int(rng.integers(-N // 4, N // 4 + 1)))
        frames.append(x.astype(np.complex64))
    return np.stack(frames)


@pytest.mark.parametrize("sf,nf", [(7, 48), (8, 24), (9, 20), (11, 6), (12, 4)])
@pytest.mark.parametrize("mode", [0, 2])
@pytest.mark.parametrize("hann", [False, True])
def test_near_ties_straddling_the_certificate(oracle, lphy, sf, nf, mode, hann):
    if sf <= 8 and hann:
        pytest.skip("SF 7-8 take k_frames either way")
    iq = _two_tone_frames(oracle, sf, nf, seed=sf * 13 + mode + 7 * hann)
    d = lphy.Demodulator(sf, window=lphy.WINDOW_HANN if hann else lphy.WINDOW_NONE)
    d.recheck_count(reset=True)
    syms, _, meta = d.demod_host(iq, nf, iq.shape[1], mode, lphy.F_DECODE)
    n_exact = d.recheck_count(reset=True)
    for f in range(nf):
        if mode == 0:
            r, osyms, osync, omet = oracle.demodulate(iq[f], sf, hann=hann)
        else:
            r, osyms, osync, omet = oracle.lora_demodulate(oracle.dechirp(iq[f], sf), sf, hann=hann)
        ctx = f"sf {sf} mode {mode} hann {hann} frame {f}"
        assert meta["status"][f] == 0, ctx
        np.testing.assert_array_equal(syms[f], osyms, err_msg=ctx)
        assert meta["sync_word"][f] == osync, ctx
        assert _bits(meta["cfo"][f]) == _bits(omet[0]), ctx
        assert _bits(meta["time_offset"][f]) == _bits(omet[1]), ctx
    # the sweep reaches margins far below the bound: some symbols must have
    # gone to the exact re-run, and far above it: not all of them
    assert 0 < n_exact < nf * 66, f"{n_exact} exact re-runs of {nf * 66} symbols"
