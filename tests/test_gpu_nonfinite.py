"""Non-finite IQ on the GPU against the oracle (C99 Annex G complex products).

The reference multiplies std::complex<float> values with GCC's inline
formula and calls __mulsc3 when both parts of a product come out NaN, which
turns some of them back into infinities (oracle/lphy_oracle.c cmul_recover,
pinned against the reference build in test_oracle_vs_reference.py).  The
hot kernels use the plain product and send every frame where that could
matter (a non-finite max-abs, a NaN bin) to the exact re-run in k_post; this
test checks every output of such frames, in every mode and launch path,
across the SF range (fused k_frames up to SF10, k_demod workgroup tiles at
SF11-12) and for oversampled input."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

VALUES = [complex(-np.inf, np.nan), complex(np.inf, 0.25), complex(np.inf, np.inf),
          complex(np.nan, 3.0), complex(0.5, np.nan), complex(-np.inf, -np.inf),
          complex(3e38, 3e38), complex(np.nan, np.inf)]


def _frames(oracle, sf, osr, nsyms_payload, seed):
    rng = np.random.default_rng(seed)
    base = oracle.modulate(oracle.encode(rng.integers(0, 256, nsyms_payload, dtype=np.uint8).tobytes()),
                           sf, osr=osr)
    n = base.size
    frames = [base.copy()]  # one clean frame beside the broken ones
    for k, v in enumerate(VALUES):
        for pos in (5, (1 << sf) * osr + 3, n // 2 + 1, n - 2):
            x = (base * (0.7 if k % 2 else 1.6)).astype(np.complex64)  # both sides of the rescale
            x[pos] = v
            frames.append(x)
    return np.stack(frames)


def _nan_bits_equal(a, b):
    a = np.asarray(a, np.float32).reshape(-1)
    b = np.asarray(b, np.float32).reshape(-1)
    na, nb = np.isnan(a), np.isnan(b)
    np.testing.assert_array_equal(na, nb)
    np.testing.assert_array_equal(a[~na].view(np.uint32), b[~nb].view(np.uint32))


# (5, 1) and (8, 1): the fused k_frames' EB tiles fold the estimate symbols'
# max-abs over team pairs of 4 and 32 lanes (NaN / inf there must reach the
# exact re-run as the 2-symbol scan made them)
@pytest.mark.parametrize("sf,osr", [(7, 1), (9, 1), (11, 1), (8, 2), (5, 1), (8, 1)])
@pytest.mark.parametrize("flags", [0, 32, 64])  # 32 = F_DECODE, 64 = F_EXACT_ROTATION
def test_nonfinite_frames_all_modes(oracle, lphy, sf, osr, flags):
    iq = _frames(oracle, sf, osr, 6, seed=sf * 10 + osr)
    nf, fs = iq.shape
    # flags 64 = LPHY_F_EXACT_ROTATION: the test build's comparison flag
    d = lphy.Demodulator(sf, osr=osr, test_build=flags == lphy.F_EXACT_ROTATION)
    modes = [lphy.MODE_DEMODULATE, lphy.MODE_LORA_DEMODULATE]
    if osr == 1:
        modes.append(lphy.MODE_DECHIRP_LORA_DEMODULATE)
    for mode in modes:
        syms, pay, meta = d.demod_host(iq, nf, fs, mode, flags | lphy.F_DECODE)
        for f in range(nf):
            if mode == lphy.MODE_DEMODULATE:
                rc, osyms, osync, omet = oracle.demodulate(iq[f], sf, osr=osr)
            else:
                src = oracle.dechirp(iq[f], sf) if mode == lphy.MODE_DECHIRP_LORA_DEMODULATE else iq[f]
                rc, osyms, osync, omet = oracle.lora_demodulate(src, sf, osr=osr)
            where = f"mode {mode} flags {flags} frame {f}"
            assert meta[f]["status"] == (rc if rc < 0 else 0), where
            if rc < 0:
                continue
            np.testing.assert_array_equal(syms[f], osyms, err_msg=where)
            assert meta[f]["sync_word"] == osync, where
            _nan_bits_equal([meta[f]["cfo"], meta[f]["time_offset"]], omet[:2])
            _, obytes, ocrc = oracle.decode(osyms)
            np.testing.assert_array_equal(pay[f], obytes, err_msg=where)
            assert bool(meta[f]["crc_ok"]) == bool(ocrc), where
