#!/usr/bin/env python3
"""Generate tests/golden/lorawan_v1.json from the REFERENCE (TEST
INFRASTRUCTURE ONLY): lorawan::compute_mic, build_frame and parse_frame
(src/lorawan/lorawan.cpp with tiny-AES src/lorawan/aes.c) compiled from
/root/reference's sources into oracle/_ref/libloraref.so (oracle/Makefile).

  aes      FIPS-197 appendix C.1 and seeded single blocks through the
           reference's AES_ECB_encrypt
  mic      seeded compute_mic cases, data lengths 0..300, both directions,
           plus the reference's own known answer (lorawan_mic_test.cpp:10-11)
  frames   seeded build_frame -> parse_frame round trips (all MTypes, FOpts
           0..15 bytes, payloads 0..222 bytes), with the decoded bytes, and
           tampered variants: a flipped MIC byte (-EINVAL), a single
           symbol bit error Hamming corrects (still valid), an FCtrl whose
           FOpts length runs into the MIC (-ERANGE), truncated frames

Usage: python tests/golden/make_lorawan_golden.py   (from the repo root)
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parents[1] / "tests"))
from checkers import Reference  # noqa: E402


def main() -> None:
    ref = Reference()
    rng = np.random.default_rng(20261016)
    out: dict = {"version": 1, "aes": [], "mic": [], "frames": []}
    fips_key, fips_pt = bytes(range(16)), bytes.fromhex("00112233445566778899aabbccddeeff")
    out["aes"].append({"key": fips_key.hex(), "in": fips_pt.hex(), "out": ref.aes128(fips_key, fips_pt).tobytes().hex()})
    for _ in range(16):
        k, b = rng.bytes(16), rng.bytes(16)
        out["aes"].append({"key": k.hex(), "in": b.hex(), "out": ref.aes128(k, b).tobytes().hex()})
    kat = bytes([0x40, 0x04, 0x03, 0x02, 0x01, 0x80, 0x01, 0x00, 0x01, 0xA6, 0x94, 0x64, 0x26, 0x15])
    cases = [(bytes([2] * 16), 1, 0x01020304, 1, kat)]
    for n in list(range(0, 70)) + [95, 96, 97, 127, 128, 129, 200, 255, 256, 300]:
        cases.append((rng.bytes(16), int(rng.integers(0, 2)), int(rng.integers(0, 2**32)),
                      int(rng.integers(0, 2**32)), rng.bytes(n)))
    for k, up, da, fc, d in cases:
        out["mic"].append({"key": k.hex(), "uplink": up, "devaddr": da, "fcnt": fc, "data": d.hex(),
                           "mic": ref.lorawan_mic(k, up, da, fc, d)})
    for i in range(48):
        key = rng.bytes(16)
        mtype, major = int(rng.integers(0, 8)), int(rng.integers(0, 4))
        devaddr, fcnt = int(rng.integers(0, 2**32)), int(rng.integers(0, 2**16))
        nfo = int(rng.integers(0, 16))
        fctrl = int(rng.integers(0, 256))
        npay = int(rng.choice([0, 1, 5, 11, 12, 13, 31, 51, 115, 222]))
        fopts, payload = rng.bytes(nfo), rng.bytes(npay)
        r, syms, tmp = ref.lorawan_build(key, mtype, major, devaddr, fctrl, fcnt, fopts, payload)
        variants = [("clean", syms.copy())]
        t = syms.copy()
        t[-1] ^= 0x0F  # MIC nibble: beyond Hamming's reach (4 bits)
        variants.append(("mic_flip", t))
        t = syms.copy()
        t[int(rng.integers(0, len(t)))] ^= 1 << int(rng.integers(0, 8))  # one bit: corrected
        variants.append(("bit_error", t))
        variants.append(("truncated", syms[: 2 * int(rng.integers(0, 12))].copy()))
        for name, sy in variants:
            pr, frame = ref.lorawan_parse(key, sy)
            dec = ref.decode(sy)[1] if len(sy) else np.zeros(0, np.uint8)
            out["frames"].append({
                "key": key.hex(), "build": {"mtype": mtype, "major": major, "devaddr": devaddr, "fctrl": fctrl,
                                            "fcnt": fcnt, "fopts": fopts.hex(), "payload": payload.hex(),
                                            "ret": r, "bytes": tmp[: r // 2].tobytes().hex() if r > 0 else ""},
                "variant": name, "symbols": sy.astype(np.uint16).tobytes().hex(), "decoded": bytes(dec).hex(),
                "parse_ret": pr, "frame": {k2: (v.hex() if isinstance(v, bytes) else v) for k2, v in frame.items()}})
    # FOpts length past the MIC, with a valid MIC over the bytes (:172)
    key = bytes(range(16, 32))
    body = bytes([0x40, 1, 2, 3, 4, 0x0F, 9, 0]) + b"\x01\x02"
    mic = ref.lorawan_mic(key, 1, 0x04030201, 9, body)
    data = body + mic.to_bytes(4, "little")
    sy = ref.encode(np.frombuffer(data, np.uint8))
    pr, frame = ref.lorawan_parse(key, sy)
    out["frames"].append({"key": key.hex(), "build": None, "variant": "fopts_overrun",
                          "symbols": sy.astype(np.uint16).tobytes().hex(), "decoded": data.hex(),
                          "parse_ret": pr,
                          "frame": {k2: (v.hex() if isinstance(v, bytes) else v) for k2, v in frame.items()}})
    (HERE / "lorawan_v1.json").write_text(json.dumps(out, indent=0) + "\n")
    print("aes", len(out["aes"]), "mic", len(out["mic"]), "frames", len(out["frames"]))


if __name__ == "__main__":
    main()
