"""Frames of few symbols through k_wave (csrc/lphy_wave.h) at SF 7-10,
where a unit holds SPW = 8 / 4 symbols and one estimate unit holds the two
estimate symbols of EPU = 4 / 2 frames of a wave (halves 2j, 2j + 1: frame
j of the group).  Frames of 2-10 symbols: every frame's last unit is
partial (its halves past the last symbol load nothing), several groups end
a wave's frames with fewer than EPU frames (the estimate unit's other halves
load nothing and are not live), and the batch sizes give waves 0 to 5
frames each (1,024 waves on the GPU).  Some frames carry a late sample
louder than their estimate symbols (the speculative normalisation settles
them, re-running their estimate unit alone).  Every output byte against the
separate launches over the whole batch and against the oracle
(LoRaDemod.cpp:50-197, phy.cpp:182-243) on a sample.

test_units_spanning_frames: SF 7-10 with S >= SPW symbols per frame, where a
wave's frames form one symbol stream and a unit holds the end of one frame
and the start of the next (WSchedSpan): S = SPW (units aligned with
frames), S just above SPW and S of the bench's 66, frames delayed both ways
(windows shifted up to the frame's edges), batches of one to many estimate
groups per wave."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _bits(x):
    return np.asarray(x, np.float32).view(np.uint32)


def _frames(oracle, sf, nf, nbytes, seed, loud_every=3, delay=False):
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
        if delay:
            x = np.roll(x, int(rng.integers(-N // 4, N // 4 + 1)))
        x = x.astype(np.complex64)
        if loud_every and f % loud_every == 1 % loud_every and x.size > 2 * N:
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


@pytest.mark.parametrize("sf,nf", [(9, 800), (9, 3001), (10, 2050), (10, 5000)])
@pytest.mark.parametrize("nbytes", [0, 1, 2, 3, 4])  # 2, 4, 6, 8, 10 symbols per frame
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_short_frames(oracle, lphy, sf, nf, nbytes, mode):
    iq = _frames(oracle, sf, nf, nbytes, seed=900 + 10 * nbytes + mode + sf)
    d = lphy.Demodulator(sf)
    syms, pay, meta = d.demod_host(iq, nf, iq.shape[1], mode, lphy.F_DECODE)
    # the separate launches as a second reference over the whole batch
    s2, p2, m2 = d.demod_host(iq, nf, iq.shape[1], mode, lphy.F_DECODE | lphy.F_UNFUSED)
    np.testing.assert_array_equal(syms, s2)
    np.testing.assert_array_equal(pay, p2)
    np.testing.assert_array_equal(meta.view(np.uint8), m2.view(np.uint8))
    _check(oracle, sf, iq, mode, syms, meta, range(0, nf, max(1, nf // 40)), f"SF{sf} S={2 * nbytes + 2}")


@pytest.mark.parametrize("sf,nbytes,nf", [(7, 15, 3000), (7, 16, 20000), (7, 32, 5000), (8, 7, 2500),
                                          (8, 8, 9000), (8, 32, 3000), (9, 3, 4000), (9, 5, 9000),
                                          (9, 32, 1500), (10, 1, 3000), (10, 3, 5000), (10, 32, 800)])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_units_spanning_frames(oracle, lphy, sf, nbytes, nf, mode):
    iq = _frames(oracle, sf, nf, nbytes, seed=1700 + 10 * nbytes + mode + sf, delay=True)
    d = lphy.Demodulator(sf)
    syms, pay, meta = d.demod_host(iq, nf, iq.shape[1], mode, lphy.F_DECODE)
    s2, p2, m2 = d.demod_host(iq, nf, iq.shape[1], mode, lphy.F_DECODE | lphy.F_UNFUSED)
    np.testing.assert_array_equal(syms, s2)
    np.testing.assert_array_equal(pay, p2)
    np.testing.assert_array_equal(meta.view(np.uint8), m2.view(np.uint8))
    _check(oracle, sf, iq, mode, syms, meta, range(0, nf, max(1, nf // 40)), f"SF{sf} S={2 * nbytes + 2}")


@pytest.mark.parametrize("sf,nbytes,nf", [(7, 16, 20000), (8, 8, 12000), (9, 5, 6000), (10, 3, 5000)])
@pytest.mark.parametrize("mode", [1, 2])
def test_spanning_units_every_frame_settles(oracle, lphy, sf, nbytes, nf, mode):
    """Every frame carries a late sample louder than its estimate symbols, so
    every frame's speculative normalisation is overturned at its end and
    queued for a batched settle (wsettle: EPU frames per unit, then the
    remainder after a wave's last unit); waves hold more than EPU frames."""
    iq = _frames(oracle, sf, nf, nbytes, seed=2300 + 10 * nbytes + mode + sf, loud_every=1, delay=True)
    d = lphy.Demodulator(sf)
    syms, pay, meta = d.demod_host(iq, nf, iq.shape[1], mode, lphy.F_DECODE)
    s2, p2, m2 = d.demod_host(iq, nf, iq.shape[1], mode, lphy.F_DECODE | lphy.F_UNFUSED)
    np.testing.assert_array_equal(syms, s2)
    np.testing.assert_array_equal(pay, p2)
    np.testing.assert_array_equal(meta.view(np.uint8), m2.view(np.uint8))
    _check(oracle, sf, iq, mode, syms, meta, range(0, nf, max(1, nf // 40)), f"SF{sf} S={2 * nbytes + 2}")
