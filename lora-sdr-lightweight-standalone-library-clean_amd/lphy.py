"""Python binding of the MI355X LoRa PHY C ABI (include/lphy_hip.h).

Thin ctypes layer used by tests/, bench.py and __graft_entry__: it loads
lib/liblphy_hip.so (built in-tree by the package Makefile) and exposes the
batch entry points on device pointers (torch tensors) plus the host-buffer
conveniences.  There is no fallback: when the library or a HIP device is
missing, calls raise.

lib/test/liblphy_hip.so is the test-only build (Makefile `test`): the same
kernels with device index checks (-DLPHY_DEBUG_BOUNDS, counted in
bounds_violations()) and the comparison flags F_EXACT_ROTATION /
F_SCAN_FIRST / F_DEBUG_RECHECK (csrc/lphy_testing.h), which the product
library rejects.  Demodulator(..., test_build=True) uses it; LPHY_LIB=test
makes it the default (a whole test run under the index checks).
"""
from __future__ import annotations

import ctypes as C
import errno
import os
from pathlib import Path

import numpy as np

PKG = Path(__file__).resolve().parent
LIB_DIR = PKG / "lib"
HIP_SO = LIB_DIR / "liblphy_hip.so"
TEST_SO = LIB_DIR / "test" / "liblphy_hip.so"
# LPHY_LIB=test: the test build; LPHY_LIB=<path>: another build of the
# library (timing experiments, tools/ubench/variants.py)
_ENV_LIB = os.environ.get("LPHY_LIB", "")
DEFAULT_SO = TEST_SO if _ENV_LIB == "test" else (Path(_ENV_LIB) if _ENV_LIB else HIP_SO)
SHIM_SO = LIB_DIR / "liblora_phy_amd.so"

MODE_DEMODULATE = 0
MODE_LORA_DEMODULATE = 1
MODE_DECHIRP_LORA_DEMODULATE = 2
F_DECODE = 1
F_NO_SCRATCH = 2
F_STAGE_PROLOGUE = 4
F_STAGE_SYMBOLS = 8
F_STAGE_FINAL = 16
F_UNFUSED = 32  # separate prologue / symbol launches (lphy_hip.h)
# test-only build (csrc/lphy_testing.h; the product library returns -EINVAL):
F_EXACT_ROTATION = 64  # every symbol with the reference's per-sample rotation
F_SCAN_FIRST = 256  # modes 1/2: whole-frame max-abs pre-scan (no speculation)
F_DEBUG_RECHECK = 512  # every symbol / estimated frame left to the exact re-run
F_FRAMES_KERNEL = 1024  # SF 7-10: k_frames where k_wave would run (test build; matrix-core tests)
WINDOW_NONE = 0
WINDOW_HANN = 1
# Smallest batch new Demodulators send to the fused kernels
# (lphy_hip_ctx_set_fused_min_frames); None keeps the library's measured
# per-SF crossover.  The test suite sets 0 (tests/conftest.py) so that its
# small batches run the fused kernels.
FUSED_MIN_FRAMES = None


class FrameMeta(C.Structure):
    _fields_ = [
        ("cfo", C.c_float), ("time_offset", C.c_float), ("rate", C.c_float),
        ("scale", C.c_float), ("t_off", C.c_int32), ("status", C.c_int32),
        ("sw0", C.c_uint16), ("sw1", C.c_uint16), ("sync_word", C.c_uint8),
        ("crc_ok", C.c_uint8), ("normalised", C.c_uint8), ("have_sync", C.c_uint8),
    ]


assert C.sizeof(FrameMeta) == 32

META_DTYPE = np.dtype([
    ("cfo", "<f4"), ("time_offset", "<f4"), ("rate", "<f4"), ("scale", "<f4"),
    ("t_off", "<i4"), ("status", "<i4"), ("sw0", "<u2"), ("sw1", "<u2"),
    ("sync_word", "u1"), ("crc_ok", "u1"), ("normalised", "u1"), ("have_sync", "u1"),
])
assert META_DTYPE.itemsize == 32

_vp = C.c_void_p
_sz = C.c_size_t

EXPORTS = (
    "lphy_hip_ctx_create", "lphy_hip_ctx_destroy", "lphy_hip_ctx_share", "lphy_hip_ctx_reserve",
    "lphy_hip_ctx_set_fused_min_frames",
    "lphy_hip_syms_per_frame", "lphy_hip_recheck_count", "lphy_hip_bounds_violations",
    "lphy_hip_demod_batch", "lphy_hip_decode_batch", "lphy_hip_estimate_batch",
    "lphy_hip_compensate", "lphy_hip_modulate_batch", "lphy_hip_demod_host",
    "lphy_hip_decode_host", "lphy_hip_estimate_host", "lphy_hip_compensate_host",
    "lphy_hip_modulate_host", "lphy_hip_demod_stream", "lphy_hip_sync", "lphy_hip_version",
    "lphy_hip_gray_batch", "lphy_hip_interleave_batch", "lphy_hip_deinterleave_batch",
    "lphy_hip_whiten_batch", "lphy_hip_hamming_batch", "lphy_hip_checksum_batch",
    "lphy_hip_lora_encode_batch", "lphy_hip_lorawan_mic_batch", "lphy_hip_lorawan_parse_batch",
    "lphy_hip_lorawan_mic_host",
)

WHITEN_SX1232, WHITEN_SX1272, WHITEN_SX1272_LFSR = 0, 1, 2
CODE_ENC84, CODE_DEC84, CODE_ENC74, CODE_DEC74 = 0, 1, 2, 3
CODE_ENCP54, CODE_CHKP54, CODE_ENCP64, CODE_CHKP64 = 4, 5, 6, 7
SUM_SX1272_CRC, SUM_HEADER, SUM_CHECKSUM8 = 0, 1, 2

_LIBS: dict = {}


class LphyError(RuntimeError):
    def __init__(self, rc: int, what: str):
        name = errno.errorcode.get(-rc, str(rc))
        super().__init__(f"{what} failed: -{name} ({rc})")
        self.rc = rc


def use(path) -> C.CDLL:
    """Make the library at `path` the default of later load() / Demodulator
    calls (experiment builds: tools/ubench) and load it."""
    global DEFAULT_SO
    DEFAULT_SO = Path(path)
    return load(DEFAULT_SO)


def load(path: Path | None = None) -> C.CDLL:
    """Load liblphy_hip.so (raises if it was not built); `path` picks another
    build (TEST_SO), default DEFAULT_SO."""
    path = Path(path or DEFAULT_SO)
    if str(path) in _LIBS:
        return _LIBS[str(path)]
    if not path.exists():
        raise FileNotFoundError(f"{path} missing: build with __graft_entry__.build()")
    # One HIP runtime per process: torch ships its own libamdhip64 (SONAME
    # libamdhip64.so.7) and asks for it by the unversioned name.  Loaded
    # first, it also satisfies our NEEDED libamdhip64.so.7; loaded after
    # /opt/rocm's copy, a second runtime instance appears and torch then
    # sees no device.  So bring torch's in before ours when torch exists.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(str(path))
    L.lphy_hip_ctx_create.argtypes = [C.POINTER(_vp), C.c_int, C.c_uint, C.c_uint, C.c_uint, C.c_int]
    L.lphy_hip_ctx_destroy.argtypes = [_vp]
    L.lphy_hip_ctx_destroy.restype = None
    L.lphy_hip_ctx_share.argtypes = [C.POINTER(_vp), _vp, C.c_uint]
    L.lphy_hip_ctx_reserve.argtypes = [_vp, _sz, _sz]
    L.lphy_hip_ctx_set_fused_min_frames.argtypes = [_vp, C.c_long]
    L.lphy_hip_bounds_violations.argtypes = [_vp, C.POINTER(C.c_ulonglong), C.c_int]
    L.lphy_hip_syms_per_frame.argtypes = [_vp, _sz, C.c_int]
    L.lphy_hip_syms_per_frame.restype = _sz
    L.lphy_hip_demod_batch.argtypes = [_vp, _vp, _sz, _sz, _vp, _vp, _vp, C.c_int, C.c_uint, _vp]
    L.lphy_hip_decode_batch.argtypes = [_vp, _vp, _sz, _sz, _vp, _vp, _vp]
    L.lphy_hip_estimate_batch.argtypes = [_vp, _vp, _sz, _sz, _sz, _vp, _vp]
    L.lphy_hip_compensate.argtypes = [_vp, _vp, _sz, C.c_float, C.c_float, _vp]
    L.lphy_hip_modulate_batch.argtypes = [_vp, _vp, _sz, _sz, _vp, C.c_float, C.c_uint8, _vp]
    L.lphy_hip_demod_host.argtypes = [_vp, _vp, _sz, _sz, _vp, _vp, _vp, C.c_int, C.c_uint]
    L.lphy_hip_decode_host.argtypes = [_vp, _vp, _sz, _vp, _vp]
    L.lphy_hip_estimate_host.argtypes = [_vp, _vp, _sz, _vp]
    L.lphy_hip_compensate_host.argtypes = [_vp, _vp, _sz, C.c_float, C.c_float]
    L.lphy_hip_modulate_host.argtypes = [_vp, _vp, _sz, _vp, C.c_float, C.c_uint8]
    L.lphy_hip_demod_stream.argtypes = [_vp, C.c_int, _sz, _sz, C.c_int, C.c_uint, _sz, _vp, _vp,
                                        _vp, C.POINTER(_sz), C.POINTER(_sz)]
    L.lphy_hip_sync.argtypes = [_vp]
    L.lphy_hip_recheck_count.argtypes = [_vp, C.POINTER(C.c_ulonglong), C.c_int]
    L.lphy_hip_version.restype = C.c_char_p
    L.lphy_hip_gray_batch.argtypes = [_vp, _sz, C.c_int, _vp]
    L.lphy_hip_interleave_batch.argtypes = [_vp, _sz, _sz, _sz, _vp, _sz, C.c_uint, C.c_uint, _vp]
    L.lphy_hip_deinterleave_batch.argtypes = [_vp, _sz, _sz, _sz, _vp, _sz, C.c_uint, C.c_uint, _vp]
    L.lphy_hip_whiten_batch.argtypes = [_vp, _sz, _sz, _sz, C.c_int, C.c_int, C.c_uint, _vp]
    L.lphy_hip_hamming_batch.argtypes = [_vp, _sz, C.c_int, _vp, _vp]
    L.lphy_hip_checksum_batch.argtypes = [_vp, _sz, _sz, _sz, C.c_int, _vp, _vp]
    L.lphy_hip_lora_encode_batch.argtypes = [_vp, _sz, _sz, _sz, _vp, _sz, _vp]
    L.lphy_hip_lorawan_mic_batch.argtypes = [_vp, _vp, _sz, _vp, _sz, _vp, C.c_uint, _vp]
    L.lphy_hip_lorawan_parse_batch.argtypes = [_vp, _sz, _sz, _vp, _sz, _vp, _sz, _vp, _vp, _vp]
    L.lphy_hip_lorawan_mic_host.argtypes = [C.c_int, _vp, C.c_int, C.c_uint32, C.c_uint32, _vp, _sz,
                                            C.POINTER(C.c_uint32)]
    _LIBS[str(path)] = L
    return L


def _chk(rc: int, what: str) -> None:
    if rc != 0:
        raise LphyError(rc, what)


def _ptr(a) -> int | None:
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return a.data_ptr()  # torch tensor


def _dev_buf(t, name: str, device: int, nbytes: int, itemsize: int | None = None) -> int:
    """Pointer of a device tensor after checking what the C ABI cannot: it
    lives on the context's HIP device, is contiguous, has the element size
    the kernels write (when given) and holds at least `nbytes`.  A wrong
    buffer would otherwise become a silent out-of-bounds device access."""
    if t is None or isinstance(t, np.ndarray) or not hasattr(t, "data_ptr"):
        raise ValueError(f"{name}: expected a device tensor, got {type(t).__name__}")
    if t.device.type != "cuda" or (t.device.index or 0) != device:
        raise ValueError(f"{name}: tensor on {t.device}, context on cuda:{device}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: tensor must be contiguous")
    if itemsize is not None and t.element_size() != itemsize:
        raise ValueError(f"{name}: {itemsize}-byte elements expected, got {t.dtype}")
    have = t.numel() * t.element_size()
    if have < nbytes:
        raise ValueError(f"{name}: {have} bytes, the call writes/reads {nbytes}")
    return t.data_ptr()


class Demodulator:
    """One (sf, bw, osr, window) configuration on one HIP device."""

    def __init__(self, sf: int, bw_hz: int = 125000, osr: int = 1,
                 window: int = WINDOW_NONE, device: int = 0, test_build: bool = False,
                 lib_path=None):
        self.lib = load(lib_path or (TEST_SO if test_build else None))
        self.sf, self.N, self.bw_hz, self.osr = sf, 1 << sf, bw_hz, osr
        self.window, self.device = window, device
        h = _vp()
        _chk(self.lib.lphy_hip_ctx_create(C.byref(h), device, sf, bw_hz, osr, window),
             "lphy_hip_ctx_create")
        self.ctx = h
        if FUSED_MIN_FRAMES is not None:
            self.set_fused_min_frames(FUSED_MIN_FRAMES)

    def set_fused_min_frames(self, frames: int) -> None:
        """Smallest batch that takes the fused kernels on this context
        (< 0: the library's measured per-SF crossover)."""
        _chk(self.lib.lphy_hip_ctx_set_fused_min_frames(self.ctx, int(frames)),
             "lphy_hip_ctx_set_fused_min_frames")

    def close(self):
        if self.ctx:
            self.lib.lphy_hip_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def syms_per_frame(self, frame_samples: int, mode: int) -> int:
        return self.lib.lphy_hip_syms_per_frame(self.ctx, frame_samples, mode)

    # --- device batch API (torch tensors) --------------------------------
    def demod_batch(self, iq, frames, frame_samples, syms, meta, mode, flags=0,
                    payload=None, stream=None):
        per = self.syms_per_frame(frame_samples, mode)
        dv = self.device
        p_iq = _dev_buf(iq, "iq", dv, frames * frame_samples * 8, None)
        p_syms = _dev_buf(syms, "syms", dv, frames * per * 2, 2)
        p_meta = _dev_buf(meta, "meta", dv, frames * 32, None)
        p_pay = None
        if flags & F_DECODE:
            p_pay = _dev_buf(payload, "payload", dv, frames * (per // 2), 1)
        _chk(self.lib.lphy_hip_demod_batch(self.ctx, p_iq, frames, frame_samples,
                                           p_syms, p_pay, p_meta, mode, flags, stream),
             "lphy_hip_demod_batch")

    def modulate_batch(self, syms, frames, nsyms, iq, amplitude=1.0, sync=0x12, stream=None):
        dv = self.device
        p_syms = _dev_buf(syms, "syms", dv, frames * nsyms * 2, 2) if nsyms else None
        p_iq = _dev_buf(iq, "iq", dv, frames * (nsyms + 2) * self.N * self.osr * 8, None)
        _chk(self.lib.lphy_hip_modulate_batch(self.ctx, p_syms, frames, nsyms, p_iq,
                                              amplitude, sync, stream),
             "lphy_hip_modulate_batch")

    def decode_batch(self, syms, frames, syms_per_frame, payload, meta, stream=None):
        dv = self.device
        p_syms = _dev_buf(syms, "syms", dv, frames * syms_per_frame * 2, 2)
        p_pay = _dev_buf(payload, "payload", dv, frames * (syms_per_frame // 2), 1)
        p_meta = _dev_buf(meta, "meta", dv, frames * 32, None)
        _chk(self.lib.lphy_hip_decode_batch(self.ctx, p_syms, frames, syms_per_frame,
                                            p_pay, p_meta, stream),
             "lphy_hip_decode_batch")

    # --- streaming ingestion (lphy_hip_demod_stream) --------------------
    def demod_stream(self, fd: int, frame_samples: int, mode: int, flags: int = 0,
                     chunk_frames: int = 0, max_frames: int = 0, capacity: int = 0):
        """Demodulate the float32 I/Q frames read from `fd` until EOF or
        max_frames.  The result arrays hold `capacity` frames (default:
        max_frames); at most min(max_frames, capacity) frames are read.
        chunk_frames = 0 lets the library pick ~64 MiB chunks (its pinned slots
        are kept with the context for the next call).  Returns (symbols,
        payload, meta, tail_bytes) for the whole frames read."""
        cap = capacity or max_frames
        if cap <= 0:
            raise ValueError("capacity or max_frames required")
        max_frames = min(max_frames, cap) if max_frames else cap
        per = self.syms_per_frame(frame_samples, mode)
        syms = np.zeros(max(cap * per, 1), np.uint16)
        payload = np.zeros(max(cap * (per // 2), 1), np.uint8)
        meta = np.zeros(cap, META_DTYPE)
        nout, tail = _sz(0), _sz(0)
        _chk(self.lib.lphy_hip_demod_stream(self.ctx, fd, frame_samples, chunk_frames, mode, flags,
                                            max_frames, syms.ctypes.data, payload.ctypes.data,
                                            meta.ctypes.data, C.byref(nout), C.byref(tail)),
             "lphy_hip_demod_stream")
        n = nout.value
        return (syms[: n * per].reshape(n, per), payload[: n * (per // 2)].reshape(n, per // 2),
                meta[:n], tail.value)

    # --- host convenience ----------------------------------------------
    def demod_host(self, iq: np.ndarray, frames: int, frame_samples: int, mode: int,
                   flags: int = 0):
        iq = np.ascontiguousarray(iq, np.complex64).reshape(-1)
        assert iq.size == frames * frame_samples
        per = self.syms_per_frame(frame_samples, mode)
        syms = np.zeros(max(frames * per, 1), np.uint16)
        payload = np.zeros(max(frames * (per // 2), 1), np.uint8)
        meta = np.zeros(frames, META_DTYPE)
        _chk(self.lib.lphy_hip_demod_host(self.ctx, iq.ctypes.data, frames, frame_samples,
                                          syms.ctypes.data, payload.ctypes.data,
                                          meta.ctypes.data, mode, flags),
             "lphy_hip_demod_host")
        return (syms[: frames * per].reshape(frames, per),
                payload[: frames * (per // 2)].reshape(frames, per // 2), meta)

    def decode_host(self, syms: np.ndarray):
        syms = np.ascontiguousarray(syms, np.uint16)
        out = np.zeros(max(len(syms) // 2, 1), np.uint8)
        meta = np.zeros(1, META_DTYPE)
        rc = self.lib.lphy_hip_decode_host(self.ctx, syms.ctypes.data, len(syms),
                                           out.ctypes.data, meta.ctypes.data)
        return rc, out[: len(syms) // 2], meta[0]

    def estimate_host(self, iq: np.ndarray):
        iq = np.ascontiguousarray(iq, np.complex64).reshape(-1)
        meta = np.zeros(1, META_DTYPE)
        _chk(self.lib.lphy_hip_estimate_host(self.ctx, iq.ctypes.data, iq.size,
                                             meta.ctypes.data), "lphy_hip_estimate_host")
        return meta[0]

    def compensate_host(self, iq: np.ndarray, cfo: float, time_offset: float):
        x = np.array(iq, np.complex64, copy=True).reshape(-1)
        _chk(self.lib.lphy_hip_compensate_host(self.ctx, x.ctypes.data, x.size, cfo,
                                               time_offset), "lphy_hip_compensate_host")
        return x

    def modulate_host(self, syms: np.ndarray, amplitude=1.0, sync=0x12):
        syms = np.ascontiguousarray(syms, np.uint16)
        out = np.zeros((len(syms) + 2) * self.N * self.osr, np.complex64)
        _chk(self.lib.lphy_hip_modulate_host(self.ctx, syms.ctypes.data, len(syms),
                                             out.ctypes.data, amplitude, sync),
             "lphy_hip_modulate_host")
        return out

    def bounds_violations(self, reset: bool = True) -> int:
        """Device index checks that failed since the last reset (test build
        only: the product library returns -ENOTSUP).  Synchronises."""
        n = C.c_ulonglong(0)
        _chk(self.lib.lphy_hip_bounds_violations(self.ctx, C.byref(n), int(reset)),
             "lphy_hip_bounds_violations")
        return int(n.value)

    def reserve(self, frames: int, frame_samples: int) -> None:
        _chk(self.lib.lphy_hip_ctx_reserve(self.ctx, frames, frame_samples), "lphy_hip_ctx_reserve")

    def parseval_count(self, reset: bool = True) -> int:
        """Test build only: symbols the wave kernel (k_wave, SF 7-12) certified by
        the Parseval certificate, without their FFT (device sync)."""
        fn = self.lib.lphy_hip_test_counter
        fn.argtypes = [_vp, C.c_int, C.POINTER(C.c_ulonglong), C.c_int]
        n = C.c_ulonglong(0)
        _chk(fn(self.ctx, 1, C.byref(n), int(reset)), "lphy_hip_test_counter")  # kCtrParseval
        return int(n.value)

    def mod_serial_count(self, reset: bool = True) -> int:
        """Test build only: frames the one-launch modulator (k_mod_fast) gave
        to its serial walk because the candidate chain left its windows
        (device sync)."""
        fn = self.lib.lphy_hip_test_counter
        fn.argtypes = [_vp, C.c_int, C.POINTER(C.c_ulonglong), C.c_int]
        n = C.c_ulonglong(0)
        _chk(fn(self.ctx, 2, C.byref(n), int(reset)), "lphy_hip_test_counter")  # kCtrModSerial
        return int(n.value)

    def mod_force_serial(self, on: bool) -> None:
        """Test build only: k_mod_fast takes its serial walk for every frame."""
        fn = self.lib.lphy_hip_test_mod_force_serial
        fn.argtypes = [_vp, C.c_int]
        _chk(fn(self.ctx, int(bool(on))), "lphy_hip_test_mod_force_serial")

    def recheck_count(self, reset: bool = True) -> int:
        """Symbols the fused kernel re-ran with the exact rotation (device sync)."""
        n = C.c_ulonglong(0)
        _chk(self.lib.lphy_hip_recheck_count(self.ctx, C.byref(n), int(reset)),
             "lphy_hip_recheck_count")
        return int(n.value)


def hamming84_encode_table() -> np.ndarray:
    """encodeHamming84sx (LoRaCodes.hpp:229-242) for nibbles 0..15 (producer)."""
    t = np.zeros(16, np.uint16)
    for x in range(16):
        d = [(x >> i) & 1 for i in range(4)]
        t[x] = (x | (d[0] ^ d[1] ^ d[2]) << 4 | (d[1] ^ d[2] ^ d[3]) << 5
                | (d[0] ^ d[1] ^ d[3]) << 6 | (d[0] ^ d[2] ^ d[3]) << 7)
    return t


def encode_payloads(payloads: np.ndarray) -> np.ndarray:
    """lora_encode for a [frames, bytes] uint8 array -> [frames, 2*bytes] uint16."""
    t = hamming84_encode_table()
    p = np.asarray(payloads, np.uint8)
    out = np.empty(p.shape[:-1] + (2 * p.shape[-1],), np.uint16)
    out[..., 0::2] = t[p >> 4]
    out[..., 1::2] = t[p & 0x0F]
    return out


# --- LoRaCodes.hpp batch kernels (device tensors) -------
def _dptr(t, name, nbytes, itemsize=None):
    return _dev_buf(t, name, t.device.index or 0, nbytes, itemsize)


def gray_batch(syms, to_binary: bool, stream=None):
    """binaryToGray16 / grayToBinary16 in place on a uint16 (int16) tensor."""
    n = syms.numel()
    _chk(load().lphy_hip_gray_batch(_dptr(syms, "syms", n * 2, 2), n, int(to_binary), stream),
         "lphy_hip_gray_batch")


def interleave_batch(cw, frames, cw_stride, cw_per_frame, syms, sym_stride, ppm, rdd, stream=None):
    _chk(load().lphy_hip_interleave_batch(_dptr(cw, "cw", frames * cw_stride, 1), frames, cw_stride,
                                          cw_per_frame, _dptr(syms, "syms", frames * sym_stride * 2, 2),
                                          sym_stride, ppm, rdd, stream), "lphy_hip_interleave_batch")


def deinterleave_batch(syms, frames, sym_stride, syms_per_frame, cw, cw_stride, ppm, rdd, stream=None):
    _chk(load().lphy_hip_deinterleave_batch(_dptr(syms, "syms", frames * sym_stride * 2, 2), frames,
                                            sym_stride, syms_per_frame, _dptr(cw, "cw", frames * cw_stride, 1),
                                            cw_stride, ppm, rdd, stream), "lphy_hip_deinterleave_batch")


def whiten_batch(buf, frames, stride, length, kind, bit_ofs=0, rdd=4, stream=None):
    _chk(load().lphy_hip_whiten_batch(_dptr(buf, "buf", frames * stride, 1), frames, stride, length, kind,
                                      bit_ofs, rdd, stream), "lphy_hip_whiten_batch")


def hamming_batch(buf, op, flags=None, stream=None):
    n = buf.numel()
    pf = _dptr(flags, "flags", n, 1) if flags is not None else None
    _chk(load().lphy_hip_hamming_batch(_dptr(buf, "buf", n, 1), n, op, pf, stream), "lphy_hip_hamming_batch")


def checksum_batch(buf, frames, stride, length, kind, out, stream=None):
    _chk(load().lphy_hip_checksum_batch(_dptr(buf, "buf", frames * stride, 1), frames, stride, length, kind,
                                        _dptr(out, "out", frames * 2, 2), stream), "lphy_hip_checksum_batch")


def lora_encode_batch(data, frames, stride, length, syms, sym_stride, stream=None):
    """lora_encode (LoRaEncoder.cpp:6-18) per row on device tensors."""
    _chk(load().lphy_hip_lora_encode_batch(_dptr(data, "data", frames * stride, 1), frames, stride, length,
                                           _dptr(syms, "syms", frames * sym_stride * 2, 2), sym_stride, stream),
         "lphy_hip_lora_encode_batch")


# --- LoRaWAN (lorawan.cpp) ----------------------------
LW_APPEND = 1
# lphy_lorawan_desc / lphy_lorawan_frame (include/lphy_hip.h) as numpy dtypes
LORAWAN_DESC_DTYPE = np.dtype([("offset", "<u8"), ("len", "<u4"), ("devaddr", "<u4"), ("fcnt", "<u4"),
                               ("key", "<u4"), ("uplink", "<u4"), ("reserved", "<u4")])
LORAWAN_FRAME_DTYPE = np.dtype([("status", "<i4"), ("devaddr", "<u4"), ("mic", "<u4"), ("calc_mic", "<u4"),
                                ("payload_offset", "<u4"), ("payload_len", "<u4"), ("fcnt", "<u2"),
                                ("mhdr", "u1"), ("fctrl", "u1"), ("fopts_len", "u1"), ("reserved", "u1", 3)])


def lorawan_mic_batch(data, desc, keys, mic=None, flags=0, stream=None):
    """compute_mic for every descriptor row.  data: uint8 device tensor;
    desc: device tensor holding len(desc) LORAWAN_DESC_DTYPE records (bytes);
    keys: uint8 device tensor of 16-byte keys; mic: int32 device tensor."""
    frames = desc.numel() * desc.element_size() // 32
    nkeys = keys.numel() // 16
    pm = _dptr(mic, "mic", frames * 4, 4) if mic is not None else None
    _chk(load().lphy_hip_lorawan_mic_batch(_dptr(data, "data", 1, 1), _dptr(desc, "desc", frames * 32), frames,
                                           _dptr(keys, "keys", nkeys * 16, 1), nkeys, pm, flags, stream),
         "lphy_hip_lorawan_mic_batch")


def lorawan_parse_batch(data, frames, stride, length, keys, out, lens=None, key_index=None, stream=None):
    """parse_frame's checks on `frames` rows of decoded bytes; out: device
    tensor of frames * 32 bytes (view it as LORAWAN_FRAME_DTYPE on the host)."""
    nkeys = keys.numel() // 16
    pl = _dptr(lens, "lens", frames * 4, 4) if lens is not None else None
    pk = _dptr(key_index, "key_index", frames * 4, 4) if key_index is not None else None
    _chk(load().lphy_hip_lorawan_parse_batch(_dptr(data, "data", (frames - 1) * stride + 1 if frames else 0, 1),
                                             frames, stride, pl, length, _dptr(keys, "keys", nkeys * 16, 1),
                                             nkeys, pk, _dptr(out, "out", frames * 32), stream),
         "lphy_hip_lorawan_parse_batch")


def lorawan_mic(key, uplink, devaddr, fcnt, data, device=0):
    """One compute_mic on the GPU from host bytes."""
    k = np.frombuffer(bytes(key), np.uint8)
    d = np.frombuffer(bytes(data) + b"\0", np.uint8)
    out = C.c_uint32()
    _chk(load().lphy_hip_lorawan_mic_host(device, k.ctypes.data, int(uplink), devaddr & 0xFFFFFFFF,
                                          fcnt & 0xFFFFFFFF, d.ctypes.data, len(data), C.byref(out)),
         "lphy_hip_lorawan_mic_host")
    return out.value
