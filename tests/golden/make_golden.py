#!/usr/bin/env python3
"""Generate the golden fixtures from the REFERENCE (TEST INFRASTRUCTURE ONLY).

Runs only in the dev container, where oracle/_ref/libloraref.so can be built
from /root/reference's own sources (oracle/Makefile).  Writes:

  tests/golden/manifest.json    cases: input recipe or stored-IQ key, input
                                SHA-256, and the reference's outputs for
                                lora_phy::demodulate + decode (phy.cpp) and
                                for dechirp -> lora_demodulate -> lora_decode
                                (LoRaDemod.cpp, e2e_chain_test.cpp:80-106)
  tests/golden/golden_v1.npz    expected symbol arrays + the stored inputs
  tests/golden/modulation_tests.bin
                                the reference's bit_exact_test input format
                                (bit_exact_test.cpp:62-105: u32 count, then per
                                record u8 0, u32 sf/bw_khz/cr_idx/flags/len,
                                payload, u32 n, f64 IQ) for every profile of
                                tests/profiles.yaml, which the reference could
                                not run because the file was missing (BW250/500:
                                expected bytes = the reference's own decode).

Usage: python tests/golden/make_golden.py   (from the repo root)
"""
from __future__ import annotations

import base64
import json
import struct
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(HERE))

from checkers import Oracle, Reference  # noqa: E402
from recipes import make_iq, sha256  # noqa: E402

REF_VECTORS = Path("/root/reference/vectors/golden")


def fbits(x) -> str:
    return "%08x" % np.float32(x).view(np.uint32)


def ramp32() -> str:  # e2e_chain_test.cpp:63-66
    return bytes(i & 0xFF for i in range(32)).hex()


def crc_payload(rng, n: int, oracle) -> str:
    """n-byte payload whose last two bytes are the sx1272 checksum of
    payload[2:n-2], so lora_phy::decode reports crc_ok (phy.cpp:252-259)."""
    body = bytearray(rng.integers(0, 256, n - 2, dtype=np.uint8).tobytes())
    c = oracle.sx_checksum(bytes(body[2:]))
    return (bytes(body) + bytes([c & 0xFF, c >> 8])).hex()


def run_reference(ref: Reference, iq: np.ndarray, sf: int, bw: int, hann: bool,
                  apis: list[str], scratch: bool = True) -> dict:
    out = {}
    N = 1 << sf
    if "demodulate" in apis:
        r, syms, sync, met = ref.demodulate(iq, sf, bw_hz=bw, hann=hann)
        d = {"ret": int(r), "sync": int(sync), "cfo": fbits(met[0]), "toff": fbits(met[1]),
             "syms": syms.astype(np.uint16)}
        if r >= 0:
            n2 = len(syms) & ~1
            k, pay, crc = ref.decode(syms[:n2])
            d.update(decode_ret=int(k), bytes=pay.tobytes().hex(), crc_ok=int(crc))
        out["demodulate"] = d
    if "lora_demodulate" in apis:
        dech = ref.dechirp(iq, sf, bw) if iq.size % N == 0 else None
        x = dech if dech is not None else iq
        r, syms, sync, met = ref.lora_demodulate(x, sf, hann=hann, scratch=scratch)
        d = {"ret": int(r), "sync": int(sync), "cfo": fbits(met[0]), "toff": fbits(met[1]),
             "syms": syms.astype(np.uint16), "input": "dechirped" if dech is not None else "raw"}
        if r >= 0:
            n2 = len(syms) & ~1
            pay = np.zeros(max(n2 // 2, 1), np.uint8)
            k = ref.lib.ref_lora_decode(np.ascontiguousarray(syms[:n2]).ctypes.data_as(
                __import__("ctypes").POINTER(__import__("ctypes").c_uint16)), n2,
                pay.ctypes.data_as(__import__("ctypes").POINTER(__import__("ctypes").c_uint8)))
            d.update(decode_ret=int(k), bytes=pay[: max(k, 0)].tobytes().hex())
        out["lora_demodulate"] = d
    return out


def main() -> None:
    ref, orc = Reference(), Oracle()
    rng = np.random.default_rng(20251015)
    cases = []

    def add(name, recipe=None, iq=None, sf=7, bw=125000, hann=False,
            apis=("demodulate", "lora_demodulate"), scratch=True, store=False):
        if iq is None:
            recipe = dict(recipe, sf=sf, bw=bw)
            iq = make_iq(orc, recipe)
        cases.append({"name": name, "recipe": recipe, "iq": iq, "sf": sf, "bw": bw,
                      "hann": hann, "apis": list(apis), "scratch": scratch,
                      "store": store or recipe is None})

    # 1. tests/profiles.yaml profiles with the e2e 32-byte ramp payload
    for name, sf, bw in [("sf7_bw125_cr45", 7, 125000), ("sf7_bw125_cr47", 7, 125000),
                         ("sf8_bw125_cr45", 8, 125000), ("sf9_bw250_cr48", 9, 250000),
                         ("sf10_bw250_cr47", 10, 250000), ("sf11_bw500_cr45", 11, 500000),
                         ("sf12_bw500_cr45", 12, 500000)]:
        add("profile_" + name, {"payload_hex": ramp32()}, sf=sf, bw=bw, store=sf <= 8)
    # 2. clean random payloads at BW125 across SF (CR is never read by the
    #    library)
    for sf in range(5, 13):
        n = 16 if sf <= 10 else 8
        add(f"clean_sf{sf}", {"payload_hex": rng.integers(0, 256, n, dtype=np.uint8).tobytes().hex()},
            sf=sf, store=sf <= 8)
    # 3. BASELINE C4: SF9 BW125 AWGN at -10 / -15 dB, seeded
    for snr in (-10.0, -15.0):
        for k in range(3):
            add(f"awgn_sf9_{int(-snr)}db_{k}",
                {"payload_hex": rng.integers(0, 256, 32, dtype=np.uint8).tobytes().hex(),
                 "snr_db": snr, "seed": 1234 + k + (100 if snr < -12 else 0)}, sf=9)
    # 4. timing offsets and deep noise (symbol errors, non-zero t_off)
    add("awgn_sf7_m18db_delay3", {"payload_hex": rng.integers(0, 256, 16, dtype=np.uint8).tobytes().hex(),
                                  "snr_db": -18.0, "seed": 7, "delay": 3}, sf=7, store=True)
    add("awgn_sf8_m12db_delay17", {"payload_hex": rng.integers(0, 256, 20, dtype=np.uint8).tobytes().hex(),
                                   "snr_db": -12.0, "seed": 8, "delay": 17}, sf=8)
    add("awgn_sf10_m20db", {"payload_hex": rng.integers(0, 256, 8, dtype=np.uint8).tobytes().hex(),
                            "snr_db": -20.0, "seed": 10}, sf=10)
    add("delay_sf11_bw125_9", {"payload_hex": rng.integers(0, 256, 6, dtype=np.uint8).tobytes().hex(),
                               "delay": 9}, sf=11)
    # 5. pure noise: bogus CFO up to ~1 bin -> rotation angles beyond 120 rad
    #    (glibc's large-argument sincosf path)
    for sf, ns, seed in [(7, 66, 1), (7, 66, 2), (8, 40, 3), (9, 30, 4)]:
        add(f"noise_sf{sf}_{seed}", {"noise_only": True, "nsyms": ns, "seed": seed}, sf=sf)
    # 6. long frame: 255-byte payload (512 data symbols) -> angles > 120 rad
    add("long_sf7_255B", {"payload_hex": rng.integers(0, 256, 255, dtype=np.uint8).tobytes().hex()}, sf=7)
    # 7. Hann window (lora_demod_init / init with window_hann)
    add("hann_sf8_clean", {"payload_hex": rng.integers(0, 256, 12, dtype=np.uint8).tobytes().hex()},
        sf=8, hann=True)
    add("hann_sf9_m8db", {"payload_hex": rng.integers(0, 256, 12, dtype=np.uint8).tobytes().hex(),
                          "snr_db": -8.0, "seed": 99}, sf=9, hann=True)
    # 8. CRC-carrying payloads (crc_ok = 1 after decode)
    for sf in (7, 9):
        add(f"crc_sf{sf}", {"payload_hex": crc_payload(rng, 24, orc)}, sf=sf)
    # 9. sync words other than 0x12
    add("sync_34_sf8", {"payload_hex": rng.integers(0, 256, 8, dtype=np.uint8).tobytes().hex(),
                        "sync": 0x34}, sf=8)
    # 10. edge cases of lora_demodulate (stored inputs)
    N = 128
    add("zero_frame_sf7", iq=np.zeros(10 * N, np.complex64), sf=7)
    add("overrange_sf7_noscratch", iq=np.full(N, 2.0 + 0j, np.complex64), sf=7,
        apis=("lora_demodulate",), scratch=False)
    add("overrange_sf7_scratch", iq=(np.full(4 * N, 2.0 + 0j) * np.exp(1j * np.arange(4 * N) * 0.37)).astype(np.complex64),
        sf=7, apis=("lora_demodulate",))
    add("one_symbol_sf7", iq=make_iq(orc, {"payload_hex": "", "sf": 7, "bw": 125000})[:N], sf=7,
        apis=("lora_demodulate",))
    tail = make_iq(orc, {"payload_hex": "a5c3", "sf": 7, "bw": 125000})
    add("tail_samples_sf7", iq=np.concatenate([tail, tail[:37]]).astype(np.complex64), sf=7,
        apis=("lora_demodulate",))
    # the reference's own fixtures (data files under vectors/golden)
    ep = base64.b64decode((REF_VECTORS / "equal_power_iq.b64").read_text())
    add("ref_equal_power_sf2", iq=np.frombuffer(ep, np.complex64).copy(), sf=2,
        apis=("lora_demodulate",))
    sw = base64.b64decode((REF_VECTORS / "sync_word_iq.b64").read_text())
    sw_iq = np.frombuffer(sw[: (len(sw) // 8) * 8], np.complex64).copy()

    # ---- run the reference ------------------------------------------------
    manifest, arrays = {"version": 1, "cases": []}, {}
    for c in cases:
        iq = c["iq"]
        res = run_reference(ref, iq, c["sf"], c["bw"], c["hann"], c["apis"], c["scratch"])
        ent = {"name": c["name"], "sf": c["sf"], "bw": c["bw"], "hann": c["hann"],
               "scratch": c["scratch"], "samples": int(iq.size), "sha256": sha256(iq),
               "recipe": c["recipe"], "stored": bool(c["store"]), "results": {}}
        if c["store"]:
            arrays[f"{c['name']}__iq"] = iq
        for api, d in res.items():
            arrays[f"{c['name']}__{api}__syms"] = d.pop("syms")
            ent["results"][api] = d
        manifest["cases"].append(ent)

    # lora_modulate known answers: reference output bits + the first 35 samples
    # of the reference's sync_word_iq.b64 (sync 0xAB, SF7, no data symbols)
    mods = []
    for name, syms, sf, bw, sync in [("mod_sync_ab_sf7", [], 7, 125000, 0xAB),
                                     ("mod_sf9_bw250", [0, 1, 255, 128, 77], 9, 250000, 0x12),
                                     ("mod_sf12_bw500", [3, 200], 12, 500000, 0x34),
                                     ("mod_no_alloc_sf7", [0, 1, 12, 34, 56], 7, 125000, 0x12)]:
        out = ref.modulate(np.array(syms, np.uint16), sf, bw_hz=bw, sync=sync)
        mods.append({"name": name, "syms": syms, "sf": sf, "bw": bw, "sync": sync,
                     "sha256": sha256(out), "samples": int(out.size)})
        if out.size <= 4096:
            arrays[f"{name}__iq"] = out
    manifest["modulate"] = mods
    arrays["ref_sync_word_iq_b64"] = sw_iq
    manifest["ref_sync_word_prefix_match"] = int(
        np.argmax(sw_iq[:256].view(np.uint64) != arrays["mod_sync_ab_sf7__iq"][: sw_iq[:256].size].view(np.uint64)))

    # encode/decode known answers (roundtrip_test.cpp:30-31)
    manifest["encode_known"] = {"payload_hex": "deadbeef",
                                "symbols": [int(x) for x in ref.encode(bytes.fromhex("deadbeef"))]}
    hd = [int(ref.lib.ref_decode_hamming84(b)) for b in range(256)]
    manifest["hamming84_decode_table"] = hd
    manifest["checksum_known"] = {"Hello": int(ref.lib.ref_sx1272_checksum(
        np.frombuffer(b"Hello", np.uint8).ctypes.data_as(__import__("ctypes").POINTER(__import__("ctypes").c_uint8)), 5))}

    (HERE / "manifest.json").write_text(json.dumps(manifest, indent=1, sort_keys=False))
    np.savez_compressed(HERE / "golden_v1.npz", **arrays)

    # modulation_tests.bin in the reference's own format, every profile of
    # tests/profiles.yaml.  BW125: the ramp payload, which the reference
    # recovers.  BW250/500: the reference's lora_modulate at that bandwidth
    # does not round-trip through its own dechirp + lora_demodulate (SURVEY
    # §0.8: e2e fails those four profiles), so the record's expected bytes
    # are what the reference's chain decodes (bit_exact_test.cpp:143-166),
    # i.e. the reference's own output for the stored samples.
    recs = []
    for sf, bw, cr in [(7, 125000, 1), (7, 125000, 3), (8, 125000, 1), (9, 250000, 4), (10, 250000, 3),
                       (11, 500000, 1), (12, 500000, 1)]:
        payload = bytes.fromhex(ramp32())
        iq = ref.modulate(ref.encode(payload, sf), sf, bw_hz=bw)
        if bw != 125000:
            r, syms, _, _ = ref.lora_demodulate(ref.dechirp(iq, sf, bw_hz=bw), sf)
            payload = ref.decode(syms)[1][: len(syms) // 2].tobytes()
        body = struct.pack("<B5I", 0, sf, bw // 1000, cr, 0, len(payload)) + payload
        body += struct.pack("<I", iq.size) + np.stack([iq.real, iq.imag], 1).astype("<f8").tobytes()
        recs.append(body)
    (HERE / "modulation_tests.bin").write_bytes(struct.pack("<I", len(recs)) + b"".join(recs))
    print(f"{len(manifest['cases'])} cases, {len(arrays)} arrays written")


if __name__ == "__main__":
    main()
