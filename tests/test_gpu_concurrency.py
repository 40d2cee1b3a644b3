"""Concurrency and ordering at SF 7-12 (the fused wave kernel, with units
spanning frames at SF 7-10, and the separate launches) and SF <= 10 with
LPHY_F_UNFUSED:

* two lphy_hip_demod_batch calls on ONE context issued on two streams at
  once give the single-stream results bit for bit (the SF 11-12
  speculation records are per-call scratch, not context state);
* LPHY_F_DEBUG_RECHECK, separate launches: marks every estimated frame
  "has open symbols" (kStatusRecheck) before the symbol kernel runs - the
  state a symbol may observe when another workgroup's certificate failed
  first - so the round-2 race (such a symbol skipped and never written) is
  exercised on every frame deterministically; fused kernels (k_frames,
  k_wave): every symbol is left uncertified, so k_post's exact re-run
  produces all of them (lphy_hip_recheck_count must cover every data
  symbol).  The output buffer is poisoned first and no poison may survive in
  any frame.  Every frame is compared with the oracle."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

POISON = 0xA5A5  # never a bin index (N <= 4096) nor the recheck sentinel


def _noisy_frames(oracle, sf, nf, snr_db, seed):
    rng = np.random.default_rng(seed)
    N = 1 << sf
    base = oracle.modulate(oracle.encode(bytes(range(16))), sf)
    fs = base.size
    t = np.arange(fs, dtype=np.float32)
    cfo = rng.uniform(-0.4, 0.4, nf).astype(np.float32)
    iq = base[None, :] * np.exp((2j * np.pi / N) * cfo[:, None] * t[None, :]).astype(np.complex64)
    sig = np.float32(np.sqrt(10 ** (-snr_db / 10) / 2))
    iq += sig * (rng.standard_normal((nf, fs), np.float32) +
                 1j * rng.standard_normal((nf, fs), np.float32)).astype(np.complex64)
    iq *= np.array([1.0, 2.5, 0.5], np.float32)[np.arange(nf) % 3][:, None]
    return np.ascontiguousarray(iq.astype(np.complex64)), fs


def _dev_run(lphy, d, iq_t, nf, fs, mode, flags, stream, poison=True):
    dev = iq_t.device
    per = d.syms_per_frame(fs, mode)
    syms = torch.full((nf * per,), POISON - 65536, dtype=torch.int16, device=dev) if poison else \
        torch.zeros(nf * per, dtype=torch.int16, device=dev)
    pay = torch.zeros(nf * (per // 2), dtype=torch.uint8, device=dev)
    meta = torch.zeros(nf * 32, dtype=torch.uint8, device=dev)
    d.demod_batch(iq_t, nf, fs, syms, meta, mode, flags, payload=pay, stream=stream)
    return syms, pay, meta


def _host(lphy, syms, pay, meta, nf, per):
    return (syms.cpu().numpy().view(np.uint16).reshape(nf, per), pay.cpu().numpy().reshape(nf, per // 2),
            meta.cpu().numpy().view(lphy.META_DTYPE))


@pytest.mark.parametrize("sf,mode", [(12, 2), (11, 2), (12, 1), (11, 0), (10, 2), (9, 1), (8, 1), (7, 2)])
@pytest.mark.parametrize("unfused", [False, True])
def test_two_streams_one_context(oracle, lphy, sf, mode, unfused):
    nf = 40
    iq, fs = _noisy_frames(oracle, sf, nf, -8.0, seed=sf * 3 + mode)
    iq2 = np.ascontiguousarray(iq[::-1])  # a different batch on the other stream
    d = lphy.Demodulator(sf)
    dev = torch.device("cuda", 0)
    a_t = torch.from_numpy(iq.view(np.float32).copy()).to(dev)
    b_t = torch.from_numpy(iq2.view(np.float32).copy()).to(dev)
    per = d.syms_per_frame(fs, mode)
    F = lphy.F_DECODE | (lphy.F_UNFUSED if unfused else 0)
    # single-stream references, one after the other
    s0 = torch.cuda.current_stream()
    ra = _host(lphy, *_dev_run(lphy, d, a_t, nf, fs, mode, F, s0.cuda_stream), nf, per)
    rb = _host(lphy, *_dev_run(lphy, d, b_t, nf, fs, mode, F, s0.cuda_stream), nf, per)
    torch.cuda.synchronize()
    for rep in range(3):
        st1, st2 = torch.cuda.Stream(), torch.cuda.Stream()
        torch.cuda.synchronize()
        with torch.cuda.stream(st1):
            oa = _dev_run(lphy, d, a_t, nf, fs, mode, F, st1.cuda_stream)
        with torch.cuda.stream(st2):
            ob = _dev_run(lphy, d, b_t, nf, fs, mode, F, st2.cuda_stream)
        torch.cuda.synchronize()
        for got, ref in ((_host(lphy, *oa, nf, per), ra), (_host(lphy, *ob, nf, per), rb)):
            np.testing.assert_array_equal(got[0], ref[0], err_msg=f"rep {rep}")
            np.testing.assert_array_equal(got[1], ref[1])
            np.testing.assert_array_equal(got[2].view(np.uint8), ref[2].view(np.uint8))


@pytest.mark.parametrize("sf,mode,unfused", [(12, 2, True), (11, 1, True), (12, 0, True),
                                             (12, 2, False), (11, 2, False), (10, 2, False), (9, 1, False),
                                             (9, 2, True), (7, 0, True), (8, 2, False), (7, 2, False),
                                             (7, 0, False)])
def test_forced_recheck_no_symbol_lost(oracle, lphy, sf, mode, unfused):
    nf = 24 if sf >= 11 else 96
    iq, fs = _noisy_frames(oracle, sf, nf, -12.0, seed=sf * 11 + mode)
    d = lphy.Demodulator(sf)
    dev = torch.device("cuda", 0)
    x_t = torch.from_numpy(iq.view(np.float32).copy()).to(dev)
    per = d.syms_per_frame(fs, mode)
    base = lphy.F_DECODE | (lphy.F_UNFUSED if unfused else 0)
    st = torch.cuda.current_stream().cuda_stream
    plain = _host(lphy, *_dev_run(lphy, d, x_t, nf, fs, mode, base, st, poison=False), nf, per)
    dt = lphy.Demodulator(sf, test_build=True)  # LPHY_F_DEBUG_RECHECK: test build only
    dt.recheck_count(reset=True)
    forced = _host(lphy, *_dev_run(lphy, dt, x_t, nf, fs, mode, base | lphy.F_DEBUG_RECHECK, st), nf, per)
    assert dt.bounds_violations() == 0
    live = forced[2]["status"] == 0
    assert live.all()
    if not unfused:
        # the fused kernels leave every symbol uncertified under the flag:
        # k_post's exact re-run must have produced each one
        n = dt.recheck_count()
        assert n >= nf * per, f"{n} exact re-runs for {nf * per} data symbols"
    assert not (forced[0] == POISON).any(), "a symbol was never written"
    np.testing.assert_array_equal(forced[0], plain[0])
    np.testing.assert_array_equal(forced[1], plain[1])
    np.testing.assert_array_equal(forced[2].view(np.uint8), plain[2].view(np.uint8))
    for f in range(nf):
        if mode == lphy.MODE_DEMODULATE:
            r, osyms, osync, omet = oracle.demodulate(iq[f], sf)
        else:
            src = iq[f] if mode == lphy.MODE_LORA_DEMODULATE else oracle.dechirp(iq[f], sf)
            r, osyms, osync, omet = oracle.lora_demodulate(src, sf)
        np.testing.assert_array_equal(forced[0][f], osyms, err_msg=f"frame {f}")
