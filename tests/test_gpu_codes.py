"""GPU batch forms of the LoRaCodes.hpp helpers (csrc/lphy_codes.hip, SURVEY
8f rank 3) against the CPU oracle (pinned to the reference header by
test_oracle_vs_reference.py): Gray mapping over every 16-bit value, every
Hamming / parity op over every byte with its flags, the diagonal
(de)interleaver for the SX127x geometries (ppm 5..12, rdd 0..4) on batches
of frames with strides, the three whitening generators at several bit
offsets, and the checksums — bit for bit, row by row."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    return torch, torch.device("cuda:0")


def test_gpu_gray_all_values(oracle, lphy, torch_dev):
    torch, dev = torch_dev
    v = np.arange(65536, dtype=np.uint16)
    for tb in (0, 1):
        t = torch.from_numpy(v.view(np.int16).copy()).to(dev)
        lphy.gray_batch(t, tb)
        got = t.cpu().numpy().view(np.uint16)
        want = np.array([oracle.gray(int(x), tb) for x in v[::1]], np.uint16)
        np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("op", range(8))
def test_gpu_hamming_all_bytes(oracle, lphy, torch_dev, op):
    torch, dev = torch_dev
    x = np.tile(np.arange(256, dtype=np.uint8), 37)
    t = torch.from_numpy(x.copy()).to(dev)
    fl = torch.zeros(x.size, dtype=torch.uint8, device=dev)
    lphy.hamming_batch(t, op, fl)
    got, gfl = t.cpu().numpy(), fl.cpu().numpy()
    for i in range(256):
        o, f = oracle.hamming(i, op)
        assert got[i] == o and gfl[i] == f, (i, op)
    np.testing.assert_array_equal(got.reshape(37, 256), np.tile(got[:256], (37, 1)))


@pytest.mark.parametrize("ppm,rdd", [(p, r) for p in (5, 7, 8, 10, 12) for r in (0, 1, 2, 4)])
def test_gpu_interleaver_batch(oracle, lphy, torch_dev, ppm, rdd):
    torch, dev = torch_dev
    rng = np.random.default_rng(ppm * 10 + rdd)
    frames, ncw = 301, 5 * ppm + 3
    cw_stride, sym_stride = ncw + 5, (ncw // ppm) * (4 + rdd) + 3
    cw = rng.integers(0, 1 << (4 + rdd), (frames, cw_stride), dtype=np.uint8)
    tcw = torch.from_numpy(cw.copy()).to(dev)
    tsy = torch.full((frames, sym_stride), -1, dtype=torch.int16, device=dev)
    lphy.interleave_batch(tcw, frames, cw_stride, ncw, tsy, sym_stride, ppm, rdd)
    sy = tsy.cpu().numpy().view(np.uint16)
    nsy = (ncw // ppm) * (4 + rdd)
    for f in range(frames):
        np.testing.assert_array_equal(sy[f, :nsy], oracle.interleave(cw[f, :ncw], ppm, rdd))
        assert (sy[f, nsy:] == 0xFFFF).all()  # past the row's blocks: untouched
    # deinterleave random symbols (and back to the codewords above)
    rs = rng.integers(0, 1 << ppm, (frames, sym_stride), dtype=np.uint16)
    trs = torch.from_numpy(rs.view(np.int16).copy()).to(dev)
    tout = torch.full((frames, cw_stride), 0xAB, dtype=torch.uint8, device=dev)
    lphy.deinterleave_batch(trs, frames, sym_stride, nsy, tout, cw_stride, ppm, rdd)
    out = tout.cpu().numpy()
    for f in range(frames):
        np.testing.assert_array_equal(out[f, : (nsy // (4 + rdd)) * ppm], oracle.deinterleave(rs[f, :nsy], ppm, rdd))
    lphy.deinterleave_batch(tsy, frames, sym_stride, nsy, tout, cw_stride, ppm, rdd)
    np.testing.assert_array_equal(tout.cpu().numpy()[:, : (ncw // ppm) * ppm], cw[:, : (ncw // ppm) * ppm])


@pytest.mark.parametrize("kind", [0, 1, 2])
def test_gpu_whitening_and_checksums(oracle, lphy, torch_dev, kind):
    torch, dev = torch_dev
    rng = np.random.default_rng(60 + kind)
    frames, length, stride = 513, 200, 211
    buf = rng.integers(0, 256, (frames, stride), dtype=np.uint8)
    for rdd in (0, 1, 4):
        for bit_ofs in (0, 3, 100):
            t = torch.from_numpy(buf.copy()).to(dev)
            lphy.whiten_batch(t, frames, stride, length, kind, bit_ofs, rdd)
            got = t.cpu().numpy()
            for f in range(0, frames, 37):
                np.testing.assert_array_equal(got[f, :length], oracle.whiten(buf[f, :length], kind, bit_ofs, rdd))
            np.testing.assert_array_equal(got[:, length:], buf[:, length:])
            lphy.whiten_batch(t, frames, stride, length, kind, bit_ofs, rdd)  # involution
            np.testing.assert_array_equal(t.cpu().numpy(), buf)
    out = torch.zeros(frames, dtype=torch.int16, device=dev)
    t = torch.from_numpy(buf.copy()).to(dev)
    lphy.checksum_batch(t, frames, stride, length, kind, out)
    got = out.cpu().numpy().view(np.uint16)
    for f in range(frames):
        assert got[f] == oracle.checksum(buf[f, :length] if kind != 1 else buf[f, :2], kind), f
