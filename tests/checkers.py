"""ctypes bindings for the two CPU checkers (TEST INFRASTRUCTURE ONLY).

* ``Oracle``    -> oracle/_build/liblphy_oracle.so  (our C restatement)
* ``Reference`` -> oracle/_ref/libloraref.so        (the reference itself,
                   compiled from /root/reference's own sources by
                   oracle/Makefile; absent on boxes where it was never built)

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  The product never does.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
ORACLE_SO = ROOT / "oracle" / "_build" / "liblphy_oracle.so"
REF_SO = ROOT / "oracle" / "_ref" / "libloraref.so"

_f32p = C.POINTER(C.c_float)
_u16p = C.POINTER(C.c_uint16)
_u8p = C.POINTER(C.c_uint8)


def _p(a, t):
    return a.ctypes.data_as(t) if a is not None else None


def _cf(iq: np.ndarray) -> np.ndarray:
    """complex64 / interleaved float32 -> contiguous float32 view."""
    iq = np.ascontiguousarray(iq)
    if iq.dtype == np.complex64:
        return iq.view(np.float32)
    assert iq.dtype == np.float32
    return iq


def build_oracle() -> None:
    import subprocess
    subprocess.run(["make", "-s", "-C", str(ROOT / "oracle"), "oracle"], check=True)


def _u8(x) -> np.ndarray:
    """bytes / list / array -> a fresh contiguous uint8 array."""
    if isinstance(x, (bytes, bytearray)):
        return np.frombuffer(bytes(x), np.uint8).copy()
    return np.array(x, np.uint8, copy=True)


class _LoRaWANMixin:
    """compute_mic / AES-128 (lorawan.cpp:35-98, aes.c) on either library."""

    def _lw_types(self, L, pre):
        getattr(L, pre + "aes128").argtypes = [_u8p, _u8p]
        getattr(L, pre + "lorawan_mic").argtypes = [_u8p, C.c_int, C.c_uint32, C.c_uint32, _u8p, C.c_size_t]
        getattr(L, pre + "lorawan_mic").restype = C.c_uint32

    def aes128(self, key, block):
        k, b = _u8(key), _u8(block)
        getattr(self.lib, self._p + "aes128")(_p(k, _u8p), _p(b, _u8p))
        return b

    def lorawan_mic(self, key, uplink, devaddr, fcnt, data):
        k = _u8(key)
        d = np.frombuffer(bytes(data) + b"\0", np.uint8)
        return int(getattr(self.lib, self._p + "lorawan_mic")(_p(k, _u8p), int(uplink), devaddr & 0xFFFFFFFF,
                                                               fcnt & 0xFFFFFFFF, _p(d, _u8p), len(data)))


class Oracle(_LoRaWANMixin):
    _p = "orc_"

    def __init__(self, path: Path = ORACLE_SO):
        if not path.exists():
            build_oracle()
        L = self.lib = C.CDLL(str(path))
        L.orc_genchirp.argtypes = [_f32p, C.c_int, C.c_int, C.c_int, C.c_float,
                                   C.c_int, C.c_float, _f32p, C.c_float]
        L.orc_fft.argtypes = [_f32p, _f32p, C.c_int]
        L.orc_dechirp.argtypes = [_f32p, _f32p, C.c_size_t, C.c_uint, C.c_uint]
        L.orc_detect.argtypes = [_f32p, _f32p, C.c_int, _f32p, _f32p, _f32p]
        L.orc_detect.restype = C.c_size_t
        L.orc_lora_modulate.argtypes = [_u16p, C.c_size_t, _f32p, C.c_uint, C.c_uint,
                                        C.c_uint, C.c_float, C.c_uint8]
        L.orc_lora_modulate.restype = C.c_size_t
        L.orc_lora_encode.argtypes = [_u8p, C.c_size_t, _u16p]
        L.orc_lora_encode.restype = C.c_size_t
        L.orc_lora_decode.argtypes = [_u16p, C.c_size_t, _u8p]
        L.orc_lora_decode.restype = C.c_ssize_t
        L.orc_sx1272_checksum.argtypes = [_u8p, C.c_int]
        L.orc_sx1272_checksum.restype = C.c_uint16
        L.orc_decode_hamming84.argtypes = [C.c_uint8]
        L.orc_decode_hamming84.restype = C.c_uint8
        L.orc_encode_hamming84.argtypes = [C.c_uint8]
        L.orc_encode_hamming84.restype = C.c_uint8
        L.orc_lora_demodulate.argtypes = [C.c_uint, C.c_int, _f32p, C.c_size_t, _u16p,
                                          C.c_uint, _u8p, C.c_size_t, _f32p]
        L.orc_lora_demodulate.restype = C.c_ssize_t
        L.orc_demodulate.argtypes = [C.c_uint, C.c_uint, C.c_uint, C.c_int, _f32p,
                                     C.c_size_t, _u16p, C.c_size_t, _f32p, C.c_uint8, _u8p]
        L.orc_demodulate.restype = C.c_ssize_t
        L.orc_estimate_offsets.argtypes = [C.c_uint, C.c_uint, C.c_int, _f32p,
                                           C.c_size_t, _f32p]
        L.orc_decode.argtypes = [_u16p, C.c_size_t, _u8p, C.c_size_t, _u8p]
        L.orc_decode.restype = C.c_ssize_t
        L.orc_compensate_offsets.argtypes = [C.c_uint, C.c_uint, C.c_float, C.c_float,
                                             _f32p, C.c_size_t]
        L.orc_gray.argtypes = [C.c_uint16, C.c_int]
        L.orc_gray.restype = C.c_uint16
        L.orc_interleave.argtypes = [_u8p, C.c_size_t, _u16p, C.c_size_t, C.c_size_t]
        L.orc_deinterleave.argtypes = [_u16p, C.c_size_t, _u8p, C.c_size_t, C.c_size_t]
        L.orc_whiten.argtypes = [_u8p, C.c_size_t, C.c_int, C.c_int, C.c_uint]
        L.orc_hamming.argtypes = [C.c_uint8, C.c_int, _u8p]
        L.orc_hamming.restype = C.c_uint8
        L.orc_checksum.argtypes = [_u8p, C.c_size_t, C.c_int]
        L.orc_checksum.restype = C.c_uint16
        L.orc_bench.argtypes = [C.c_int, C.c_uint, C.c_uint, _f32p, C.c_size_t,
                                C.c_size_t, _u8p, C.c_int]
        L.orc_bench.restype = C.c_double
        self._lw_types(L, "orc_")
        L.orc_lorawan_parse.argtypes = [_u8p, _u8p, C.c_size_t, C.POINTER(C.c_int64)]


    # --- LoRaCodes.hpp helpers -------------------------
    def gray(self, v, to_binary):
        return getattr(self.lib, self._p + "gray")(int(v), int(to_binary))

    def interleave(self, cw, ppm, rdd):
        cw = np.ascontiguousarray(cw, np.uint8)
        out = np.zeros(max((len(cw) // ppm) * (4 + rdd), 1), np.uint16)
        getattr(self.lib, self._p + "interleave")(_p(cw, _u8p), len(cw), _p(out, _u16p), ppm, rdd)
        return out[: (len(cw) // ppm) * (4 + rdd)]

    def deinterleave(self, syms, ppm, rdd):
        syms = np.ascontiguousarray(syms, np.uint16)
        out = np.zeros(max((len(syms) // (4 + rdd)) * ppm, 1), np.uint8)
        getattr(self.lib, self._p + "deinterleave")(_p(syms, _u16p), len(syms), _p(out, _u8p), ppm, rdd)
        return out[: (len(syms) // (4 + rdd)) * ppm]

    def whiten(self, buf, kind, bit_ofs=0, rdd=4):
        b = np.array(buf, np.uint8, copy=True)
        getattr(self.lib, self._p + "whiten")(_p(b, _u8p), len(b), kind, bit_ofs, rdd)
        return b

    def hamming(self, x, op):
        fl = np.zeros(1, np.uint8)
        out = getattr(self.lib, self._p + "hamming")(int(x), op, _p(fl, _u8p))
        return int(out), int(fl[0])

    def checksum(self, buf, kind):
        b = np.ascontiguousarray(np.frombuffer(bytes(buf), np.uint8)) if not isinstance(buf, np.ndarray) else np.ascontiguousarray(buf, np.uint8)
        return getattr(self.lib, self._p + "checksum")(_p(b, _u8p), len(b), kind)

    def lorawan_parse(self, key, data):
        """parse_frame's checks on decoded bytes -> dict (lphy_oracle.c)."""
        k = _u8(key)
        d = np.frombuffer(bytes(data) + b"\0", np.uint8)
        rec = np.zeros(10, np.int64)
        self.lib.orc_lorawan_parse(_p(k, _u8p), _p(d, _u8p), len(data), rec.ctypes.data_as(C.POINTER(C.c_int64)))
        names = ("status", "devaddr", "mic", "calc_mic", "payload_offset", "payload_len", "fcnt", "mhdr",
                 "fctrl", "fopts_len")
        return {n: int(v) for n, v in zip(names, rec)}

    # --- producers -----------------------------------------------------
    def genchirp(self, N, osr, NN, f0, down, ampl, phase, bw_scale):
        out = np.zeros(2 * NN, np.float32)
        ph = np.array([phase], np.float32)
        self.lib.orc_genchirp(_p(out, _f32p), N, osr, NN, f0, int(down), ampl,
                              _p(ph, _f32p), bw_scale)
        return out.view(np.complex64), float(ph[0])

    def modulate(self, syms, sf, osr=1, bw_hz=125000, ampl=1.0, sync=0x12):
        syms = np.ascontiguousarray(syms, np.uint16)
        n = len(syms)
        out = np.zeros(2 * (n + 2) * (1 << sf) * osr, np.float32)
        self.lib.orc_lora_modulate(_p(syms, _u16p), n, _p(out, _f32p), sf, osr,
                                   bw_hz, ampl, sync)
        return out.view(np.complex64)

    def encode(self, payload):
        payload = np.ascontiguousarray(np.frombuffer(bytes(payload), np.uint8))
        out = np.zeros(2 * len(payload), np.uint16)
        self.lib.orc_lora_encode(_p(payload, _u8p), len(payload), _p(out, _u16p))
        return out

    def estimate_offsets(self, iq, sf, osr=1, hann=False):
        """phy.cpp:81-148 over the whole buffer -> (cfo, time_offset)."""
        x = _cf(iq)
        met = np.zeros(2, np.float32)
        self.lib.orc_estimate_offsets(sf, osr, int(hann), _p(x, _f32p), len(x) // 2,
                                      _p(met, _f32p))
        return met

    def compensate_offsets(self, iq, sf, cfo, time_offset, osr=1):
        """phy.cpp:150-180 on a copy -> compensated complex64 samples."""
        x = _cf(np.array(iq, np.complex64))
        self.lib.orc_compensate_offsets(sf, osr, cfo, time_offset, _p(x, _f32p), len(x) // 2)
        return x.view(np.complex64)

    def dechirp(self, iq, sf, bw_hz=125000):
        x = _cf(np.asarray(iq, np.complex64))
        out = np.zeros_like(x)
        self.lib.orc_dechirp(_p(x, _f32p), _p(out, _f32p), len(x) // 2, sf, bw_hz)
        return out.view(np.complex64)

    # --- consumers -----------------------------------------------------
    def fft(self, x):
        x = _cf(np.asarray(x, np.complex64))
        out = np.zeros_like(x)
        self.lib.orc_fft(_p(x, _f32p), _p(out, _f32p), len(x) // 2)
        return out.view(np.complex64)

    def lora_demodulate(self, samples, sf, osr=1, hann=False, scratch=True):
        x = _cf(samples)
        count = len(x) // 2
        total = count // ((1 << sf) * osr)
        out = np.zeros(max(total, 1), np.uint16)
        sync = np.zeros(1, np.uint8)
        met = np.zeros(2, np.float32)
        r = self.lib.orc_lora_demodulate(sf, int(hann), _p(x, _f32p), count,
                                         _p(out, _u16p), osr, _p(sync, _u8p),
                                         count if scratch else 0, _p(met, _f32p))
        return r, out[: max(r, 0)], int(sync[0]), met

    def demodulate(self, iq, sf, bw_hz=125000, osr=1, hann=False, cap=None, sync=0x12):
        x = _cf(iq)
        count = len(x) // 2
        total = count // ((1 << sf) * osr)
        cap = max(total - 2, 0) if cap is None else cap
        syms = np.zeros(max(cap, 1), np.uint16)
        met = np.zeros(2, np.float32)
        so = np.zeros(1, np.uint8)
        r = self.lib.orc_demodulate(sf, bw_hz, osr, int(hann), _p(x, _f32p), count,
                                    _p(syms, _u16p), cap, _p(met, _f32p), sync,
                                    _p(so, _u8p))
        return r, syms[: max(r, 0)], int(so[0]), met

    def decode(self, syms, cap=None):
        syms = np.ascontiguousarray(syms, np.uint16)
        cap = len(syms) // 2 if cap is None else cap
        out = np.zeros(max(len(syms) // 2, 1), np.uint8)
        crc = np.zeros(1, np.uint8)
        r = self.lib.orc_decode(_p(syms, _u16p), len(syms), _p(out, _u8p), cap,
                                _p(crc, _u8p))
        return r, out[: max(r, 0)], int(crc[0])

    def lora_decode(self, syms):
        syms = np.ascontiguousarray(syms, np.uint16)
        out = np.zeros(max(len(syms) // 2, 1), np.uint8)
        r = self.lib.orc_lora_decode(_p(syms, _u16p), len(syms), _p(out, _u8p))
        return r, out[: max(r, 0)]

    def sx_checksum(self, data):
        d = np.ascontiguousarray(np.frombuffer(bytes(data), np.uint8))
        return self.lib.orc_sx1272_checksum(_p(d, _u8p), len(d))

    def bench(self, mode, sf, iq, frames, frame_samples, threads, bw_hz=125000):
        x = _cf(iq)
        ndata = frame_samples // (1 << sf) - 2
        out = np.zeros(frames * (ndata // 2), np.uint8)
        t = self.lib.orc_bench(mode, sf, bw_hz, _p(x, _f32p), frames, frame_samples,
                               _p(out, _u8p), threads)
        return t, out


class Reference(_LoRaWANMixin):
    """The reference library (oracle/_ref), when it has been built."""
    _p = "ref_"

    def __init__(self, path: Path = REF_SO):
        if not path.exists():
            raise FileNotFoundError(path)
        L = self.lib = C.CDLL(str(path))
        for n in ("ref_sizeof_workspace", "ref_sizeof_demod_workspace",
                  "ref_sizeof_params", "ref_sizeof_metrics"):
            getattr(L, n).restype = C.c_size_t
        L.ref_fft.argtypes = [_f32p, _f32p, C.c_int]
        L.ref_dechirp.argtypes = [_f32p, _f32p, C.c_size_t, C.c_uint, C.c_uint]
        L.ref_detect.argtypes = [_f32p, _f32p, C.c_int, _f32p, _f32p, _f32p]
        L.ref_detect.restype = C.c_size_t
        L.ref_genchirp.argtypes = [_f32p, C.c_int, C.c_int, C.c_int, C.c_float,
                                   C.c_int, C.c_float, _f32p, C.c_float]
        L.ref_lora_modulate.argtypes = [_u16p, C.c_size_t, _f32p, C.c_uint, C.c_uint,
                                        C.c_uint, C.c_float, C.c_uint8]
        L.ref_lora_modulate.restype = C.c_size_t
        L.ref_lora_encode.argtypes = [_u8p, C.c_size_t, _u16p, C.c_uint]
        L.ref_lora_encode.restype = C.c_size_t
        L.ref_lora_decode.argtypes = [_u16p, C.c_size_t, _u8p]
        L.ref_lora_decode.restype = C.c_ssize_t
        L.ref_sx1272_checksum.argtypes = [_u8p, C.c_int]
        L.ref_sx1272_checksum.restype = C.c_uint16
        L.ref_decode_hamming84.argtypes = [C.c_uint8]
        L.ref_decode_hamming84.restype = C.c_uint8
        L.ref_lora_demodulate.argtypes = [C.c_uint, C.c_int, _f32p, C.c_size_t, _u16p,
                                          C.c_uint, _u8p, C.c_int, _f32p]
        L.ref_lora_demodulate.restype = C.c_ssize_t
        L.ref_demodulate.argtypes = [C.c_uint, C.c_uint, C.c_uint, C.c_int, C.c_uint8,
                                     _f32p, C.c_size_t, _u16p, C.c_size_t, _f32p, _u8p]
        L.ref_demodulate.restype = C.c_ssize_t
        L.ref_estimate_offsets.argtypes = [C.c_uint, C.c_uint, C.c_uint, C.c_int,
                                           _f32p, C.c_size_t, _f32p]
        L.ref_decode.argtypes = [C.c_uint, _u16p, C.c_size_t, _u8p, C.c_size_t, _u8p]
        L.ref_decode.restype = C.c_ssize_t
        L.ref_compensate_offsets.argtypes = [C.c_uint, C.c_uint, C.c_float, C.c_float,
                                             _f32p, C.c_size_t]
        L.ref_gray.argtypes = [C.c_uint16, C.c_int]
        L.ref_gray.restype = C.c_uint16
        L.ref_interleave.argtypes = [_u8p, C.c_size_t, _u16p, C.c_size_t, C.c_size_t]
        L.ref_deinterleave.argtypes = [_u16p, C.c_size_t, _u8p, C.c_size_t, C.c_size_t]
        L.ref_whiten.argtypes = [_u8p, C.c_size_t, C.c_int, C.c_int, C.c_uint]
        L.ref_hamming.argtypes = [C.c_uint8, C.c_int, _u8p]
        L.ref_hamming.restype = C.c_uint8
        L.ref_checksum.argtypes = [_u8p, C.c_size_t, C.c_int]
        L.ref_checksum.restype = C.c_uint16
        self._lw_types(L, "ref_")
        _u32p = C.POINTER(C.c_uint32)
        L.ref_lorawan_build.argtypes = [_u8p, _u32p, _u8p, C.c_size_t, _u8p, C.c_size_t, _u16p,
                                        C.c_size_t, _u8p, C.c_size_t]
        L.ref_lorawan_build.restype = C.c_long
        L.ref_lorawan_parse.argtypes = [_u8p, _u16p, C.c_size_t, _u8p, C.c_size_t, _u32p, _u8p, _u8p]
        L.ref_lorawan_parse.restype = C.c_long
        for n in ("ref_bench_modeA", "ref_bench_modeB"):
            getattr(L, n).argtypes = [C.c_uint, C.c_uint, _f32p, C.c_size_t,
                                      C.c_size_t, _u8p, C.c_int]
            getattr(L, n).restype = C.c_double


    # --- LoRaCodes.hpp helpers -------------------------
    def gray(self, v, to_binary):
        return getattr(self.lib, self._p + "gray")(int(v), int(to_binary))

    def interleave(self, cw, ppm, rdd):
        cw = np.ascontiguousarray(cw, np.uint8)
        out = np.zeros(max((len(cw) // ppm) * (4 + rdd), 1), np.uint16)
        getattr(self.lib, self._p + "interleave")(_p(cw, _u8p), len(cw), _p(out, _u16p), ppm, rdd)
        return out[: (len(cw) // ppm) * (4 + rdd)]

    def deinterleave(self, syms, ppm, rdd):
        syms = np.ascontiguousarray(syms, np.uint16)
        out = np.zeros(max((len(syms) // (4 + rdd)) * ppm, 1), np.uint8)
        getattr(self.lib, self._p + "deinterleave")(_p(syms, _u16p), len(syms), _p(out, _u8p), ppm, rdd)
        return out[: (len(syms) // (4 + rdd)) * ppm]

    def whiten(self, buf, kind, bit_ofs=0, rdd=4):
        b = np.array(buf, np.uint8, copy=True)
        getattr(self.lib, self._p + "whiten")(_p(b, _u8p), len(b), kind, bit_ofs, rdd)
        return b

    def hamming(self, x, op):
        fl = np.zeros(1, np.uint8)
        out = getattr(self.lib, self._p + "hamming")(int(x), op, _p(fl, _u8p))
        return int(out), int(fl[0])

    def checksum(self, buf, kind):
        b = np.ascontiguousarray(np.frombuffer(bytes(buf), np.uint8)) if not isinstance(buf, np.ndarray) else np.ascontiguousarray(buf, np.uint8)
        return getattr(self.lib, self._p + "checksum")(_p(b, _u8p), len(b), kind)

    def lorawan_build(self, key, mtype, major, devaddr, fctrl, fcnt, fopts, payload, cap=None, tmp_cap=None):
        """lorawan::build_frame -> (return value, symbols, tmp bytes)."""
        k = _u8(key)
        hdr = np.array([mtype, major, devaddr & 0xFFFFFFFF, fctrl, fcnt & 0xFFFF], np.uint32)
        fo = np.frombuffer(bytes(fopts) + b"\0", np.uint8)
        pl = np.frombuffer(bytes(payload) + b"\0", np.uint8)
        need = 12 + len(fopts) + len(payload)
        cap = 2 * need if cap is None else cap
        tmp_cap = need if tmp_cap is None else tmp_cap
        syms = np.zeros(max(cap, 1), np.uint16)
        tmp = np.zeros(max(tmp_cap, need, 1), np.uint8)
        r = self.lib.ref_lorawan_build(_p(k, _u8p), hdr.ctypes.data_as(C.POINTER(C.c_uint32)), _p(fo, _u8p),
                                       len(fopts), _p(pl, _u8p), len(payload), _p(syms, _u16p), cap,
                                       _p(tmp, _u8p), tmp_cap)
        return int(r), syms[: max(int(r), 0)], tmp

    def lorawan_parse(self, key, syms, tmp_cap=None):
        """lorawan::parse_frame -> (return value, Frame fields dict)."""
        k = _u8(key)
        sy = np.ascontiguousarray(syms, np.uint16)
        tmp_cap = len(sy) // 2 if tmp_cap is None else tmp_cap
        tmp = np.zeros(max(len(sy) // 2, tmp_cap, 1), np.uint8)
        out = np.zeros(7, np.uint32)
        fo, pl = np.zeros(256, np.uint8), np.zeros(65536, np.uint8)
        r = self.lib.ref_lorawan_parse(_p(k, _u8p), _p(sy, _u16p), len(sy), _p(tmp, _u8p), tmp_cap,
                                       out.ctypes.data_as(C.POINTER(C.c_uint32)), _p(fo, _u8p), _p(pl, _u8p))
        f = dict(zip(("mtype", "major", "devaddr", "fctrl", "fcnt"), (int(v) for v in out[:5])))
        f["fopts"], f["payload"] = fo[: out[5]].tobytes(), pl[: out[6]].tobytes()
        return int(r), f

    def fft(self, x):
        x = _cf(np.asarray(x, np.complex64))
        out = np.zeros_like(x)
        self.lib.ref_fft(_p(x, _f32p), _p(out, _f32p), len(x) // 2)
        return out.view(np.complex64)

    def estimate_offsets(self, iq, sf, osr=1, hann=False, bw_hz=125000):
        x = _cf(iq)
        met = np.zeros(2, np.float32)
        self.lib.ref_estimate_offsets(sf, bw_hz, osr, int(hann), _p(x, _f32p), len(x) // 2,
                                      _p(met, _f32p))
        return met

    def compensate_offsets(self, iq, sf, cfo, time_offset, osr=1):
        x = _cf(np.array(iq, np.complex64))
        self.lib.ref_compensate_offsets(sf, osr, cfo, time_offset, _p(x, _f32p), len(x) // 2)
        return x.view(np.complex64)

    def dechirp(self, iq, sf, bw_hz=125000):
        x = _cf(np.asarray(iq, np.complex64))
        out = np.zeros_like(x)
        self.lib.ref_dechirp(_p(x, _f32p), _p(out, _f32p), len(x) // 2, sf, bw_hz)
        return out.view(np.complex64)

    def detect(self, x):
        x = _cf(np.asarray(x, np.complex64))
        out = np.zeros_like(x)
        p, pa, fi = (np.zeros(1, np.float32) for _ in range(3))
        idx = self.lib.ref_detect(_p(x, _f32p), _p(out, _f32p), len(x) // 2,
                                  _p(p, _f32p), _p(pa, _f32p), _p(fi, _f32p))
        return idx, float(p[0]), float(pa[0]), float(fi[0]), out.view(np.complex64)

    def genchirp(self, N, osr, NN, f0, down, ampl, phase, bw_scale):
        out = np.zeros(2 * NN, np.float32)
        ph = np.array([phase], np.float32)
        self.lib.ref_genchirp(_p(out, _f32p), N, osr, NN, f0, int(down), ampl,
                              _p(ph, _f32p), bw_scale)
        return out.view(np.complex64), float(ph[0])

    def modulate(self, syms, sf, osr=1, bw_hz=125000, ampl=1.0, sync=0x12):
        syms = np.ascontiguousarray(syms, np.uint16)
        n = len(syms)
        out = np.zeros(2 * (n + 2) * (1 << sf) * osr, np.float32)
        self.lib.ref_lora_modulate(_p(syms, _u16p), n, _p(out, _f32p), sf, osr,
                                   bw_hz, ampl, sync)
        return out.view(np.complex64)

    def encode(self, payload, sf=7):
        payload = np.ascontiguousarray(np.frombuffer(bytes(payload), np.uint8))
        out = np.zeros(2 * len(payload), np.uint16)
        self.lib.ref_lora_encode(_p(payload, _u8p), len(payload), _p(out, _u16p), sf)
        return out

    def lora_demodulate(self, samples, sf, osr=1, hann=False, scratch=True):
        x = _cf(samples)
        count = len(x) // 2
        total = count // ((1 << sf) * osr)
        out = np.zeros(max(total, 1), np.uint16)
        sync = np.zeros(1, np.uint8)
        met = np.zeros(2, np.float32)
        r = self.lib.ref_lora_demodulate(sf, int(hann), _p(x, _f32p), count,
                                         _p(out, _u16p), osr, _p(sync, _u8p),
                                         int(scratch), _p(met, _f32p))
        return r, out[: max(r, 0)], int(sync[0]), met

    def demodulate(self, iq, sf, bw_hz=125000, osr=1, hann=False, cap=None, sync=0x12):
        x = _cf(iq)
        count = len(x) // 2
        total = count // ((1 << sf) * osr)
        cap = max(total - 2, 0) if cap is None else cap
        syms = np.zeros(max(cap, 1), np.uint16)
        met = np.zeros(2, np.float32)
        so = np.zeros(1, np.uint8)
        r = self.lib.ref_demodulate(sf, bw_hz, osr, int(hann), sync, _p(x, _f32p),
                                    count, _p(syms, _u16p), cap, _p(met, _f32p),
                                    _p(so, _u8p))
        return r, syms[: max(r, 0)], int(so[0]), met

    def decode(self, syms, cap=None):
        syms = np.ascontiguousarray(syms, np.uint16)
        cap = len(syms) // 2 if cap is None else cap
        out = np.zeros(max(len(syms) // 2, 1), np.uint8)
        crc = np.zeros(1, np.uint8)
        r = self.lib.ref_decode(7, _p(syms, _u16p), len(syms), _p(out, _u8p), cap,
                                _p(crc, _u8p))
        return r, out[: max(r, 0)], int(crc[0])

    def bench(self, mode, sf, iq, frames, frame_samples, threads, bw_hz=125000):
        x = _cf(iq)
        ndata = frame_samples // (1 << sf) - 2
        out = np.zeros(frames * (ndata // 2), np.uint8)
        fn = self.lib.ref_bench_modeB if mode == 1 else self.lib.ref_bench_modeA
        t = fn(sf, bw_hz, _p(x, _f32p), frames, frame_samples, _p(out, _u8p), threads)
        return t, out


def reference_available() -> bool:
    return REF_SO.exists()
