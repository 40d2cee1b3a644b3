"""Streaming ingestion (lphy_hip_demod_stream).

Input is the reference receive runner's byte format: float32 (I, Q) pairs
back to back (rx_runner.cpp:61-79). It is read from a file and from a pipe
with short writes, and demodulated in chunks that do not divide the frame
count. Every output is checked bit for bit against the one-shot batch path
(lphy_hip_demod_host), and the first frames against the CPU oracle."""
import os
import tempfile
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _frames(oracle, sf, nf, seed):
    rng = np.random.default_rng(seed)
    N = 1 << sf
    iq = np.stack([oracle.modulate(oracle.encode(rng.integers(0, 256, 16, dtype=np.uint8).tobytes()), sf)
                   for _ in range(nf)]).astype(np.complex128)
    t = np.arange(iq.shape[1])
    for f in range(nf):
        x = iq[f] * np.exp(2j * np.pi * rng.uniform(-0.3, 0.3) / N * t) * [1.0, 2.5, 0.7][f % 3]
        iq[f] = x + 0.1 * (rng.standard_normal(x.size) + 1j * rng.standard_normal(x.size))
    return iq.astype(np.complex64)


def _same(a, b):
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])
    np.testing.assert_array_equal(a[2].view(np.uint8), b[2].view(np.uint8))


def _oracle_frame(oracle, lphy, x, sf, mode):
    if mode == lphy.MODE_DEMODULATE:
        return oracle.demodulate(x, sf)[1]
    return oracle.lora_demodulate(oracle.dechirp(x, sf), sf)[1]


@pytest.mark.parametrize("mode", [0, 2])
def test_stream_file_matches_batch(oracle, lphy, mode):
    sf, nf = 7, 37
    iq = _frames(oracle, sf, nf, 5 + mode)
    fs = iq.shape[1]
    d = lphy.Demodulator(sf)
    ref = d.demod_host(iq, nf, fs, mode, lphy.F_DECODE)
    with tempfile.TemporaryFile() as fh:
        fh.write(iq.tobytes())
        fh.write(b"\x01" * 100)  # a trailing partial frame
        fh.flush()
        fh.seek(0)
        syms, pay, meta, tail = d.demod_stream(fh.fileno(), fs, mode, lphy.F_DECODE,
                                               chunk_frames=8, capacity=64)
    assert tail == 100
    assert syms.shape[0] == nf
    _same((syms, pay, meta), ref)
    for f in range(3):
        np.testing.assert_array_equal(syms[f], _oracle_frame(oracle, lphy, iq[f], sf, mode))


def test_stream_pipe_short_writes_and_cap(oracle, lphy):
    sf, nf = 8, 21
    iq = _frames(oracle, sf, nf, 11)
    fs = iq.shape[1]
    mode = lphy.MODE_DECHIRP_LORA_DEMODULATE
    d = lphy.Demodulator(sf)
    ref = d.demod_host(iq, nf, fs, mode, lphy.F_DECODE)
    data = iq.tobytes()

    def run(max_frames, chunk):
        r, w = os.pipe()

        def writer():
            try:
                for i in range(0, len(data), 7001):  # short, unaligned writes
                    os.write(w, data[i:i + 7001])
            except BrokenPipeError:
                pass
            finally:
                os.close(w)

        th = threading.Thread(target=writer)
        th.start()
        try:
            out = d.demod_stream(r, fs, mode, lphy.F_DECODE, chunk_frames=chunk,
                                 max_frames=max_frames, capacity=nf)
        finally:
            os.close(r)
            th.join()
        return out

    syms, pay, meta, tail = run(0, 5)
    assert tail == 0 and syms.shape[0] == nf
    _same((syms, pay, meta), ref)
    syms, pay, meta, tail = run(10, 4)  # stops after max_frames
    assert syms.shape[0] == 10
    _same((syms, pay, meta), tuple(x[:10] for x in ref))


def test_stream_argument_errors(lphy):
    import ctypes as C
    d = lphy.Demodulator(7)
    n, t = C.c_size_t(0), C.c_size_t(0)
    meta = np.zeros(4, lphy.META_DTYPE)
    syms = np.zeros(4 * 64, np.uint16)
    lib = d.lib
    assert lib.lphy_hip_demod_stream(d.ctx, -1, 66 * 128, 4, 0, 0, 4, syms.ctypes.data, None,
                                     meta.ctypes.data, C.byref(n), C.byref(t)) == -22
    # no frame length (chunk_frames = 0 is valid: the library picks ~64 MiB chunks)
    assert lib.lphy_hip_demod_stream(d.ctx, 0, 0, 0, 0, 0, 4, syms.ctypes.data, None,
                                     meta.ctypes.data, C.byref(n), C.byref(t)) == -22
    # no capacity: the C ABI cannot bound the writes into the caller's arrays
    assert lib.lphy_hip_demod_stream(d.ctx, 0, 66 * 128, 4, 0, 0, 0, syms.ctypes.data, None,
                                     meta.ctypes.data, C.byref(n), C.byref(t)) == -22
    # LPHY_F_DECODE without a payload array
    assert lib.lphy_hip_demod_stream(d.ctx, 0, 66 * 128, 4, 0, lphy.F_DECODE, 4, syms.ctypes.data,
                                     None, meta.ctypes.data, C.byref(n), C.byref(t)) == -22
    # the fused dechirp needs whole symbols: the first chunk's launch refuses
    with tempfile.TemporaryFile() as fh:
        fh.write(np.zeros(2 * (66 * 128 + 3), np.float32).tobytes())
        fh.flush()
        fh.seek(0)
        with pytest.raises(lphy.LphyError):
            d.demod_stream(fh.fileno(), 66 * 128 + 3, lphy.MODE_DECHIRP_LORA_DEMODULATE, 0,
                           chunk_frames=2, capacity=2)


@pytest.mark.parametrize("copy", ["map", "pread"])
def test_stream_reader_pool_offset_and_resume(oracle, lphy, monkeypatch, copy):
    """Chunks above the reader pool's threshold (4 MiB): the readers copy
    out of a mapping of the file (default) or pread it (LPHY_STREAM_COPY).
    The stream starts at a non-zero file offset, stops at max_frames and a
    second call resumes from the descriptor's offset; a partial frame
    trails."""
    if copy == "pread":
        monkeypatch.setenv("LPHY_STREAM_COPY", "pread")
    else:
        monkeypatch.delenv("LPHY_STREAM_COPY", raising=False)
    sf, nf, head = 7, 150, 24
    iq = _frames(oracle, sf, nf, 29)
    fs = iq.shape[1]
    mode = lphy.MODE_DECHIRP_LORA_DEMODULATE
    d = lphy.Demodulator(sf)
    ref = d.demod_host(iq, nf, fs, mode, lphy.F_DECODE)
    with tempfile.TemporaryFile() as fh:
        fh.write(b"\x7f" * head)
        fh.write(iq.tobytes())
        fh.write(b"\x02" * 40)
        fh.flush()
        fh.seek(head)
        a = d.demod_stream(fh.fileno(), fs, mode, lphy.F_DECODE, chunk_frames=70,
                           max_frames=100, capacity=nf)
        assert a[0].shape[0] == 100 and a[3] == 0
        assert os.lseek(fh.fileno(), 0, os.SEEK_CUR) == head + 100 * fs * 8
        b = d.demod_stream(fh.fileno(), fs, mode, lphy.F_DECODE, chunk_frames=70, capacity=nf)
    assert b[0].shape[0] == nf - 100 and b[3] == 40
    got = tuple(np.concatenate([x, y]) for x, y in zip(a[:3], b[:3]))
    _same(got, ref)
    for f in (0, 99, 100, nf - 1):
        np.testing.assert_array_equal(got[0][f], _oracle_frame(oracle, lphy, iq[f], sf, mode))
