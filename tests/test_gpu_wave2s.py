"""k_wave2s (csrc/lphy_wave2.h), the default fused kernel at SF 9: units of
SPW = 8 consecutive symbols of a wave's frame stream, per-frame records in an
LDS ring, the 64 x 8 exchange through LDS buffers shared by the CU's 8 waves
under compare-and-swap locks.

* Short frames.  A unit of 8 stream positions can hold several frame ends
  when a frame has fewer than 8 symbols, and k_wave2s closes at most one
  frame per unit (the speculation's frame-end check, wclose2).  The library
  therefore sends frames shorter than a unit to k_wave
  (lphy_kernels.h use_wave2s).  These batches (>= 768 frames, the product's
  fused crossover at SF 9, and the suite's fused default) have 2-9 symbols
  per frame, a later symbol louder than the estimate symbols in some frames
  (the settle path) and impairments; every output bit against the oracle
  (LoRaDemod.cpp:50-197, phy.cpp:182-243).
* Lock fail-safe.  wbuf_acquire caps its sweeps so a lost lock can never
  hang the GPU; at the cap the unit uses no buffer and is left to the exact
  re-run (a symbol unit: kSymRecheck; an estimate unit: the frame to
  kStatusFixup).  LPHY_F_DEBUG_LOCKFAIL (test build) makes every third
  acquisition fail and the others try once, so this path runs on every call:
  the outputs must equal the oracle's and the product library's bit for
  bit, with re-runs counted."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _bits(x):
    return np.asarray(x, np.float32).view(np.uint32)


def _frames(oracle, sf, nf, nbytes, seed, loud_every=3):
    """nf frames of `nbytes` payload bytes (2 nbytes data symbols + 2 sync),
    CFO, noise, gain; every `loud_every`-th frame has a late sample larger
    than any in its estimate symbols (the speculative normalisation settles
    it)."""
    rng = np.random.default_rng(seed)
    N = 1 << sf
    out = []
    for f in range(nf):
        pay = bytes(rng.integers(0, 256, nbytes, dtype=np.uint8))
        x = oracle.modulate(oracle.encode(pay), sf).astype(np.complex128)
        t = np.arange(x.size)
        x = x * np.exp(2j * np.pi * rng.uniform(-0.4, 0.4) / N * t) * [0.8, 1.0, 2.2][f % 3]
        x = x + 0.05 * (rng.standard_normal(x.size) + 1j * rng.standard_normal(x.size))
        x = x.astype(np.complex64)
        if loud_every and f % loud_every == 1 and x.size > 2 * N:
            j = int(rng.integers(2 * N, x.size))
            x[j] = np.complex64(complex(6.0, -2.0))
        out.append(x)
    return np.stack(out)


def _check(oracle, sf, iq, mode, syms, meta, frames, what):
    for f in frames:
        if mode == 0:
            r, osyms, osync, omet = oracle.demodulate(iq[f], sf)
        else:
            src = iq[f] if mode == 1 else oracle.dechirp(iq[f], sf)
            r, osyms, osync, omet = oracle.lora_demodulate(src, sf)
        ctx = f"{what} mode {mode} frame {f}"
        assert meta["status"][f] == 0, ctx
        np.testing.assert_array_equal(syms[f], osyms, err_msg=ctx)
        assert meta["sync_word"][f] == osync, ctx
        assert _bits(meta["cfo"][f]) == _bits(omet[0]), ctx
        assert _bits(meta["time_offset"][f]) == _bits(omet[1]), ctx


@pytest.mark.parametrize("nbytes", [0, 1, 2, 3, 4])  # 2, 4, 6, 8, 10 symbols per frame
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_short_frames_sf9(oracle, lphy, nbytes, mode):
    sf, nf = 9, 800
    iq = _frames(oracle, sf, nf, nbytes, seed=900 + 10 * nbytes + mode)
    d = lphy.Demodulator(sf)
    syms, pay, meta = d.demod_host(iq, nf, iq.shape[1], mode, lphy.F_DECODE)
    # the separate launches as a second reference over the whole batch
    s2, p2, m2 = d.demod_host(iq, nf, iq.shape[1], mode, lphy.F_DECODE | lphy.F_UNFUSED)
    np.testing.assert_array_equal(syms, s2)
    np.testing.assert_array_equal(pay, p2)
    np.testing.assert_array_equal(meta.view(np.uint8), m2.view(np.uint8))
    _check(oracle, sf, iq, mode, syms, meta, range(0, nf, 7), f"S={2 * nbytes + 2}")


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_lock_fail_safe_sf9(oracle, lphy, mode):
    sf, nf = 9, 900
    iq = _frames(oracle, sf, nf, 32, seed=77 + mode)
    fs = iq.shape[1]
    ref = lphy.Demodulator(sf).demod_host(iq, nf, fs, mode, lphy.F_DECODE)
    dt = lphy.Demodulator(sf, test_build=True)
    dt.recheck_count(reset=True)
    got = dt.demod_host(iq, nf, fs, mode, lphy.F_DECODE | lphy.F_DEBUG_LOCKFAIL)
    n_exact = dt.recheck_count(reset=True)
    assert dt.bounds_violations() == 0
    np.testing.assert_array_equal(got[0], ref[0])
    np.testing.assert_array_equal(got[1], ref[1])
    np.testing.assert_array_equal(got[2].view(np.uint8), ref[2].view(np.uint8))
    # every third acquisition failed: about a third of the symbol units went
    # to the exact re-run (and the frames of a third of the estimate units
    # were re-run whole, which this count does not include)
    assert n_exact >= nf * 64 // 8, n_exact
    _check(oracle, sf, iq, mode, got[0], got[2], range(0, nf, 29), "lockfail")
