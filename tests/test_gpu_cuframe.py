"""The single-read CU-resident kernel (csrc/lphy_cuframe.h: SF 7, 56..70
whole symbols per frame) against the separate-launch path (exact per-sample
rotation, LPHY_F_UNFUSED) and the CPU oracle.

Every output must agree byte for byte: symbols, decoded payloads and the
32-byte frame records.  Frame counts are chosen so workgroups hold 0, 1, 2
and many frames (the register-slot / frame-buffer pipeline's prologue and
tail), payload sizes span the kernel's whole symbol range, and impairments
exercise time shifts that straddle symbol slots, CFO, noise (near-ties left
to k_post's exact re-check), gains on both sides of the normalisation, the
Hann window, non-finite samples and the no-scratch -ERANGE status."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SF, N = 7, 128


def _frames(oracle, nf, plen, seed, snr_db=None, cfo_bins=0.0, max_delay=0, gains=(1.0,)):
    rng = np.random.default_rng(seed)
    out = []
    for f in range(nf):
        p = rng.integers(0, 256, plen, dtype=np.uint8).tobytes()
        x = oracle.modulate(oracle.encode(p), SF).astype(np.complex128)
        t = np.arange(x.size)
        if cfo_bins:
            x = x * np.exp(2j * np.pi * rng.uniform(-cfo_bins, cfo_bins) / N * t)
        if max_delay:
            x = np.roll(x, int(rng.integers(-max_delay, max_delay + 1)))
        if snr_db is not None:
            s = np.sqrt(10 ** (-snr_db / 10) / 2)
            x = x + s * (rng.standard_normal(x.size) + 1j * rng.standard_normal(x.size))
        out.append((x * gains[f % len(gains)]).astype(np.complex64))
    return np.stack(out)


def _run(lphy, d, iq, mode, flags=0):
    """The resident kernel is opt-in (LPHY_F_RESIDENT); the comparisons
    below run it against LPHY_F_UNFUSED, where the flag has no effect."""
    nf, fs = iq.shape
    return d.demod_host(iq, nf, fs, mode, flags | lphy.F_DECODE | lphy.F_RESIDENT)


def _same(a, b, what):
    np.testing.assert_array_equal(a[0], b[0], err_msg=f"{what}: symbols")
    np.testing.assert_array_equal(a[1], b[1], err_msg=f"{what}: payload")
    np.testing.assert_array_equal(a[2].view(np.uint8), b[2].view(np.uint8), err_msg=f"{what}: records")


def _oracle_check(oracle, iq, mode, res, frames):
    syms, pay, meta = res
    for f in frames:
        if mode == 0:
            r, osyms, osync, omet = oracle.demodulate(iq[f], SF)
        else:
            x = oracle.dechirp(iq[f], SF) if mode == 2 else iq[f]
            r, osyms, osync, omet = oracle.lora_demodulate(x, SF)
        np.testing.assert_array_equal(syms[f], osyms, err_msg=f"frame {f}")
        assert meta["sync_word"][f] == osync
        np.testing.assert_array_equal(np.array([meta["cfo"][f], meta["time_offset"][f]], np.float32).view(np.uint32),
                                      np.asarray(omet[:2], np.float32).view(np.uint32))


@pytest.mark.parametrize("plen", [27, 29, 32, 34])  # 56, 60, 66, 70 symbols
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_cuframe_clean_and_impaired(oracle, lphy, plen, mode):
    d = lphy.Demodulator(SF)
    for nf, kw, seed in [(700, {}, 1), (300, dict(snr_db=-12.0, cfo_bins=0.45, max_delay=50, gains=(1.0, 0.3, 2.5)), 2)]:
        iq = _frames(oracle, nf, plen, seed + plen * 10 + mode, **kw)
        if mode == 1:
            iq = np.stack([oracle.dechirp(x, SF) for x in iq])
        a = _run(lphy, d, iq, mode)
        b = _run(lphy, d, iq, mode, lphy.F_UNFUSED)
        _same(a, b, f"mode {mode} plen {plen} nf {nf}")
        _oracle_check(oracle, iq, mode, a, range(0, nf, nf // 7))


@pytest.mark.parametrize("nf", [1, 2, 3, 255, 256, 257, 513, 1031])
def test_cuframe_frame_counts(oracle, lphy, nf):
    """Workgroups with 0..5 frames: the pipeline's prologue and tail."""
    d = lphy.Demodulator(SF)
    iq = _frames(oracle, nf, 32, 50 + nf, snr_db=-5.0, cfo_bins=0.2, max_delay=20)
    for mode in (0, 2):
        _same(_run(lphy, d, iq, mode), _run(lphy, d, iq, mode, lphy.F_UNFUSED), f"mode {mode} nf {nf}")


def test_cuframe_window_specials_and_noscratch(oracle, lphy):
    base = _frames(oracle, 64, 32, 77, snr_db=-8.0, cfo_bins=0.3, max_delay=30)
    iq = base.copy()
    iq[3, 500] = np.nan
    iq[5, 2000] = complex(np.inf, 0.5)
    iq[7] = 0
    iq[9] *= 1e20
    iq[11] *= 1e-30
    iq[13, 3 * N:] = 0
    dh = lphy.Demodulator(SF, 125000, 1, lphy.WINDOW_HANN)
    dn = lphy.Demodulator(SF)
    for d in (dn, dh):
        for mode in (0, 1, 2):
            x = np.stack([oracle.dechirp(v, SF) for v in iq]) if mode == 1 else iq
            _same(_run(lphy, d, x, mode), _run(lphy, d, x, mode, lphy.F_UNFUSED), f"mode {mode}")
            if mode:
                _same(_run(lphy, d, x, mode, lphy.F_NO_SCRATCH),
                      _run(lphy, d, x, mode, lphy.F_NO_SCRATCH | lphy.F_UNFUSED), f"noscratch mode {mode}")
    # exact rotation forced: every symbol goes through k_post's recheck
    a = _run(lphy, dn, base, 2, lphy.F_EXACT_ROTATION)
    _same(a, _run(lphy, dn, base, 2), "exact vs fast")
    assert dn.recheck_count(reset=True) >= 64 * 66


def test_cuframe_large_batch_payloads(oracle, lphy):
    """65,536-frame-scale batch slice through the device entry point: every
    payload recovered, identical to the separate launches."""
    import torch
    nf, plen = 4096, 32
    rng = np.random.default_rng(9)
    pay = rng.integers(0, 256, (nf, plen), dtype=np.uint8)
    d = lphy.Demodulator(SF)
    dev = torch.device("cuda:0")
    syms_in = torch.from_numpy(lphy.encode_payloads(pay).view(np.int16).reshape(-1).copy()).to(dev)
    fs = 66 * N
    iq = torch.empty(nf * fs * 2, dtype=torch.float32, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    d.modulate_batch(syms_in, nf, 64, iq, 1.0, 0x12, st)
    outs = []
    for flags in (lphy.F_DECODE | lphy.F_RESIDENT, lphy.F_DECODE | lphy.F_UNFUSED):
        s = torch.zeros(nf * 64, dtype=torch.int16, device=dev)
        m = torch.zeros(nf * 32, dtype=torch.uint8, device=dev)
        p = torch.zeros(nf * 32, dtype=torch.uint8, device=dev)
        d.demod_batch(iq, nf, fs, s, m, lphy.MODE_DECHIRP_LORA_DEMODULATE, flags, payload=p, stream=st)
        torch.cuda.synchronize()
        outs.append((s.cpu().numpy(), p.cpu().numpy(), m.cpu().numpy()))
    for x, y in zip(outs[0], outs[1]):
        np.testing.assert_array_equal(x, y)
    np.testing.assert_array_equal(outs[0][1].reshape(nf, plen), pay)
