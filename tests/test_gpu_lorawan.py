"""LoRaWAN helpers on the GPU (csrc/lphy_lorawan.hip)
against the oracle (pinned to lorawan.cpp + tiny-AES by
tests/test_lorawan_cpu.py): batched compute_mic over ragged, unaligned
frames with per-frame keys; the MIC append build_frame does; parse_frame's
checks on decoded rows (valid, MIC mismatch, short, FOpts overrun, unknown
key); the reference's own outcomes from tests/golden/lorawan_v1.json; and a
whole uplink chain on the device: MIC append -> lora_encode ->
lora_modulate -> demodulate + decode -> parse."""
import json
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLD = json.loads((Path(__file__).resolve().parent / "golden" / "lorawan_v1.json").read_text())
KAT = bytes([0x40, 0x04, 0x03, 0x02, 0x01, 0x80, 0x01, 0x00, 0x01, 0xA6, 0x94, 0x64, 0x26, 0x15])


@pytest.fixture(scope="module")
def dev():
    import torch
    return torch, torch.device("cuda:0")


def _desc(rows):
    import numpy as np
    from lphy import LORAWAN_DESC_DTYPE
    d = np.zeros(len(rows), LORAWAN_DESC_DTYPE)
    for i, (off, n, da, fc, key, up) in enumerate(rows):
        d[i] = (off, n, da, fc, key, up, 0)
    return d


def test_gpu_mic_known_answer(lphy):
    assert lphy.lorawan_mic(bytes([2] * 16), True, 0x01020304, 1, KAT) == 0x82B5C3D6
    for c in GOLD["mic"][:20]:
        assert lphy.lorawan_mic(bytes.fromhex(c["key"]), c["uplink"], c["devaddr"], c["fcnt"],
                                bytes.fromhex(c["data"])) == c["mic"]


def test_gpu_mic_batch_ragged(oracle, lphy, dev):
    torch, d = dev
    rng = np.random.default_rng(11)
    nk, nf = 37, 4099
    keys = rng.integers(0, 256, (nk, 16), dtype=np.uint8)
    lens = rng.integers(0, 300, nf)
    lens[:300] = np.arange(300)
    offs = np.concatenate([[0], np.cumsum(lens + rng.integers(0, 7, nf))])[:-1] + 3  # unaligned
    buf = rng.integers(0, 256, int(offs[-1] + lens[-1] + 8), dtype=np.uint8)
    rows = [(int(offs[i]), int(lens[i]), int(rng.integers(0, 2**32)), int(rng.integers(0, 2**32)),
             int(rng.integers(0, nk)), int(rng.integers(0, 2))) for i in range(nf)]
    desc = _desc(rows)
    t_buf = torch.from_numpy(buf.copy()).to(d)
    t_desc = torch.from_numpy(desc.view(np.uint8).copy()).to(d)
    t_keys = torch.from_numpy(keys.reshape(-1).copy()).to(d)
    t_mic = torch.zeros(nf, dtype=torch.int32, device=d)
    lphy.lorawan_mic_batch(t_buf, t_desc, t_keys, t_mic)
    got = t_mic.cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(t_buf.cpu().numpy(), buf)  # read-only without APPEND
    for i, (off, n, da, fc, k, up) in enumerate(rows):
        want = oracle.lorawan_mic(keys[k], up, da, fc, buf[off:off + n].tobytes())
        assert got[i] == want, (i, n)


def test_gpu_mic_append_and_bad_key(oracle, lphy, dev):
    torch, d = dev
    rng = np.random.default_rng(12)
    nf, row = 515, 64
    buf = rng.integers(0, 256, nf * row, dtype=np.uint8)
    keys = rng.integers(0, 256, (2, 16), dtype=np.uint8)
    rows = [(i * row + 1, int(rng.integers(0, 58)), i, 7 * i, i % 3, i & 1) for i in range(nf)]  # key 2: absent
    t_buf = torch.from_numpy(buf.copy()).to(d)
    t_mic = torch.full((nf,), -1, dtype=torch.int32, device=d)
    lphy.lorawan_mic_batch(t_buf, torch.from_numpy(_desc(rows).view(np.uint8).copy()).to(d),
                           torch.from_numpy(keys.reshape(-1).copy()).to(d), t_mic, lphy.LW_APPEND)
    out, mic = t_buf.cpu().numpy(), t_mic.cpu().numpy().view(np.uint32)
    want_buf = buf.copy()
    for i, (off, n, da, fc, k, up) in enumerate(rows):
        if k >= 2:
            assert mic[i] == 0
            continue
        m = oracle.lorawan_mic(keys[k], up, da, fc, buf[off:off + n].tobytes())
        assert mic[i] == m
        want_buf[off + n:off + n + 4] = np.frombuffer(m.to_bytes(4, "little"), np.uint8)
    np.testing.assert_array_equal(out, want_buf)


def _parse_rows(lphy, torch, d, rows_bytes, stride, keys, key_index=None, lens=None):
    nf = len(rows_bytes)
    buf = np.zeros((nf, stride), np.uint8)
    for i, b in enumerate(rows_bytes):
        buf[i, :len(b)] = np.frombuffer(b, np.uint8)
    t_out = torch.zeros(nf * 32, dtype=torch.uint8, device=d)
    t_lens = torch.from_numpy(np.array(lens, np.int32)).to(d) if lens is not None else None
    t_ki = torch.from_numpy(np.array(key_index, np.int32)).to(d) if key_index is not None else None
    lphy.lorawan_parse_batch(torch.from_numpy(buf.reshape(-1).copy()).to(d), nf, stride,
                             stride if lens is None else 0, torch.from_numpy(np.array(keys, np.uint8).reshape(-1).copy()).to(d),
                             t_out, lens=t_lens, key_index=t_ki)
    return t_out.cpu().numpy().view(lphy.LORAWAN_FRAME_DTYPE)


def _same(rec, want):
    for k in ("status", "devaddr", "mic", "calc_mic", "payload_offset", "payload_len", "fcnt", "mhdr",
              "fctrl", "fopts_len"):
        assert int(rec[k]) == want[k], (k, int(rec[k]), want[k])


def test_gpu_parse_golden(oracle, lphy, dev):
    """The reference's parse_frame outcomes (golden), row by row, per-row
    lengths and keys."""
    torch, d = dev
    frames = GOLD["frames"]
    keys = [list(bytes.fromhex(c["key"])) for c in frames]
    rows = [bytes.fromhex(c["decoded"]) for c in frames]
    recs = _parse_rows(lphy, torch, d, rows, 256, keys, key_index=list(range(len(rows))),
                       lens=[len(r) for r in rows])
    for c, r, rec in zip(frames, rows, recs):
        assert int(rec["status"]) == c["parse_ret"], c["variant"]
        _same(rec, oracle.lorawan_parse(bytes.fromhex(c["key"]), r))
        if c["parse_ret"] >= 0:
            po, pl = int(rec["payload_offset"]), int(rec["payload_len"])
            assert r[po:po + pl].hex() == c["frame"]["payload"]


def test_gpu_parse_uniform_rows(oracle, lphy, dev):
    torch, d = dev
    rng = np.random.default_rng(13)
    key = rng.integers(0, 256, 16, dtype=np.uint8)
    nf, L = 2053, 40
    rows = []
    for i in range(nf):
        fol = int(rng.integers(0, 16))
        body = bytearray(rng.integers(0, 256, L - 4, dtype=np.uint8).tobytes())
        body[5] = (body[5] & 0xF0) | fol
        mic = oracle.lorawan_mic(key, ((body[0] >> 5) & 1) == 0, int.from_bytes(body[1:5], "little"),
                                 int.from_bytes(body[6:8], "little"), bytes(body))
        b = bytes(body) + mic.to_bytes(4, "little")
        if i % 5 == 1:
            b = b[:-1] + bytes([b[-1] ^ 0x40])  # MIC mismatch
        rows.append(b)
    recs = _parse_rows(lphy, torch, d, rows, L, [key])
    for r, rec in zip(rows, recs):
        _same(rec, oracle.lorawan_parse(key, r))
    st = recs["status"]
    assert (st[1::5] == -22).all() and (st >= 0).sum() > nf // 2
    # short rows and an absent key
    recs = _parse_rows(lphy, torch, d, [b"\x40" * n for n in range(12)], 16, [key], lens=list(range(12)))
    assert (recs["status"] == -34).all() and (recs["mic"] == 0).all()
    recs = _parse_rows(lphy, torch, d, rows[:4], L, [key], key_index=[0, 1, 0, 5])
    assert list(recs["status"][[1, 3]]) == [-126, -126]


def test_gpu_parse_row_length_bounds(oracle, lphy, dev):
    """A per-row length past the row (`stride`) or past 65535 is -ERANGE for
    that row alone, with nothing of the row read; the other rows parse."""
    torch, d = dev
    rng = np.random.default_rng(14)
    key = rng.integers(0, 256, 16, dtype=np.uint8)
    L = 40
    body = bytearray(rng.integers(0, 256, L - 4, dtype=np.uint8).tobytes())
    body[5] &= 0xF0
    mic = oracle.lorawan_mic(key, ((body[0] >> 5) & 1) == 0, int.from_bytes(body[1:5], "little"),
                             int.from_bytes(body[6:8], "little"), bytes(body))
    row = bytes(body) + mic.to_bytes(4, "little")
    lens = [L, L + 1, 70000, 0x7FFFFFFF, L]
    recs = _parse_rows(lphy, torch, d, [row] * len(lens), L, [key], lens=lens)
    assert list(recs["status"]) == [L - 12, -34, -34, -34, L - 12]
    assert (recs["mic"][1:4] == 0).all() and (recs["devaddr"][1:4] == 0).all()


def test_gpu_uplink_chain(oracle, lphy, dev):
    """MIC append -> lora_encode -> modulate -> demodulate+decode -> parse,
    all on the device (SF7, 64-symbol frames, 32-byte LoRaWAN frames)."""
    torch, d = dev
    rng = np.random.default_rng(14)
    nf, L = 3000, 32
    keys = rng.integers(0, 256, (16, 16), dtype=np.uint8)
    kidx = rng.integers(0, 16, nf).astype(np.int32)
    rows = np.zeros((nf, L), np.uint8)
    descs = []
    for i in range(nf):
        body = bytearray(rng.integers(0, 256, L - 4, dtype=np.uint8).tobytes())
        body[0] = (int(rng.integers(0, 8)) << 5) | int(rng.integers(0, 4))
        body[5] = (body[5] & 0xF0) | 3
        rows[i, :L - 4] = np.frombuffer(bytes(body), np.uint8)
        descs.append((i * L, L - 4, int.from_bytes(body[1:5], "little"), int.from_bytes(body[6:8], "little"),
                      int(kidx[i]), int(((body[0] >> 5) & 1) == 0)))
    t_rows = torch.from_numpy(rows.reshape(-1).copy()).to(d)
    t_keys = torch.from_numpy(keys.reshape(-1).copy()).to(d)
    st = torch.cuda.current_stream().cuda_stream
    lphy.lorawan_mic_batch(t_rows, torch.from_numpy(_desc(descs).view(np.uint8).copy()).to(d), t_keys,
                           None, lphy.LW_APPEND, stream=st)
    syms = torch.zeros(nf * 2 * L, dtype=torch.int16, device=d)
    lphy.lora_encode_batch(t_rows, nf, L, L, syms, 2 * L, stream=st)
    dm = lphy.Demodulator(7)
    fs = (2 * L + 2) * 128
    iq = torch.empty(nf * fs * 2, dtype=torch.float32, device=d)
    dm.modulate_batch(syms, nf, 2 * L, iq, 1.0, 0x12, st)
    s2 = torch.zeros(nf * 2 * L, dtype=torch.int16, device=d)
    meta = torch.zeros(nf * 32, dtype=torch.uint8, device=d)
    pay = torch.zeros(nf * L, dtype=torch.uint8, device=d)
    dm.demod_batch(iq, nf, fs, s2, meta, lphy.MODE_DECHIRP_LORA_DEMODULATE, lphy.F_DECODE, payload=pay, stream=st)
    out = torch.zeros(nf * 32, dtype=torch.uint8, device=d)
    lphy.lorawan_parse_batch(pay, nf, L, L, t_keys, out, key_index=torch.from_numpy(kidx).to(d), stream=st)
    torch.cuda.synchronize()
    recs = out.cpu().numpy().view(lphy.LORAWAN_FRAME_DTYPE)
    built = t_rows.cpu().numpy().reshape(nf, L)
    np.testing.assert_array_equal(pay.cpu().numpy().reshape(nf, L), built)
    assert (recs["status"] == L - 12 - 3).all()
    for i in range(0, nf, 97):
        m = oracle.lorawan_mic(keys[kidx[i]], descs[i][5], descs[i][2], descs[i][3], rows[i, :L - 4].tobytes())
        assert int(recs["mic"][i]) == m == int.from_bytes(built[i, L - 4:].tobytes(), "little")
    np.testing.assert_array_equal(syms.cpu().numpy().view(np.uint16).reshape(nf, 2 * L)[:8],
                                  np.stack([oracle.encode(built[i]) for i in range(8)]))
