"""CPU oracle against the committed golden fixtures (reference outputs):
bit-exact symbols, sync word, cfo / time_offset float bits, decoded bytes,
CRC flag and return codes for every case and both APIs, plus the
modulate / encode / Hamming / checksum known answers."""
import ctypes as C
import struct

import numpy as np
import pytest

import golden_cases as G

CASES = G.case_names()


@pytest.mark.parametrize("name", CASES)
def test_golden_input_integrity(oracle, name):
    G.case_iq(oracle, G.case(name))  # size + SHA-256 of stored / regenerated IQ


@pytest.mark.parametrize("name", CASES)
def test_oracle_demodulate_golden(oracle, name):
    c = G.case(name)
    res = c["results"].get("demodulate")
    if res is None:
        pytest.skip("lora_demodulate-only case")
    iq = G.case_iq(oracle, c)
    r, syms, sync, met = oracle.demodulate(iq, c["sf"], bw_hz=c["bw"], hann=c["hann"])
    assert r == res["ret"]
    np.testing.assert_array_equal(syms, G.expected_syms(c, "demodulate"))
    assert sync == res["sync"]
    assert G.fbits(met[0]) == res["cfo"] and G.fbits(met[1]) == res["toff"]
    if r >= 0:
        k, pay, crc = oracle.decode(syms[: len(syms) & ~1])
        assert k == res["decode_ret"] and pay.tobytes().hex() == res["bytes"]
        assert crc == res["crc_ok"]


@pytest.mark.parametrize("name", CASES)
def test_oracle_lora_demodulate_golden(oracle, name):
    c = G.case(name)
    res = c["results"]["lora_demodulate"]
    iq = G.case_iq(oracle, c)
    x = G.lora_input(oracle, c, iq)
    r, syms, sync, met = oracle.lora_demodulate(x, c["sf"], hann=c["hann"], scratch=c["scratch"])
    assert r == res["ret"]
    np.testing.assert_array_equal(syms, G.expected_syms(c, "lora_demodulate"))
    assert sync == res["sync"]
    assert G.fbits(met[0]) == res["cfo"] and G.fbits(met[1]) == res["toff"]
    if r >= 0:
        k, pay = oracle.lora_decode(syms[: len(syms) & ~1])
        assert k == res["decode_ret"] and pay[: max(k, 0)].tobytes().hex() == res["bytes"]


@pytest.mark.parametrize("m", G.MANIFEST["modulate"], ids=lambda m: m["name"])
def test_oracle_modulate_known_answers(oracle, m):
    from recipes import sha256
    out = oracle.modulate(np.array(m["syms"], np.uint16), m["sf"], bw_hz=m["bw"], sync=m["sync"])
    assert out.size == m["samples"] and sha256(out) == m["sha256"]


def test_oracle_matches_reference_sync_word_fixture(oracle):
    """vectors/golden/sync_word_iq.b64 (reference data file): its first
    samples are lora_modulate(sync 0xAB, SF7) exactly."""
    arr = G.arrays()
    ref_iq = arr["ref_sync_word_iq_b64"]
    ours = oracle.modulate(np.zeros(0, np.uint16), 7, sync=0xAB)
    n = G.MANIFEST["ref_sync_word_prefix_match"]
    assert n >= 32
    np.testing.assert_array_equal(ours[:n].view(np.uint64), ref_iq[:n].view(np.uint64))


def test_encode_known_answer(oracle):
    k = G.MANIFEST["encode_known"]
    np.testing.assert_array_equal(oracle.encode(bytes.fromhex(k["payload_hex"])), k["symbols"])


def test_hamming84_table(oracle):
    L = oracle.lib
    L.orc_decode_hamming84.restype = C.c_uint8
    L.orc_decode_hamming84.argtypes = [C.c_uint8]
    got = [int(L.orc_decode_hamming84(b)) for b in range(256)]
    assert got == G.MANIFEST["hamming84_decode_table"]


def test_checksum_known_answer(oracle):
    for s, v in G.MANIFEST["checksum_known"].items():
        assert oracle.sx_checksum(s.encode()) == v


def test_modulation_tests_bin_records(oracle):
    """vectors/golden/modulation_tests.bin in the reference's record format
    (SURVEY §4), one record per profile of the reference's tests/profiles.yaml:
    each record's IQ is the oracle's lora_modulate of the ramp payload at the
    profile's SF / bandwidth, and its expected bytes are what the dechirp +
    lora_demodulate + lora_decode chain gives (BW125: the payload itself;
    BW250/500, where the reference's chain does not round-trip, SURVEY §0.8:
    its own decode, bit_exact_test.cpp:143-166)."""
    blob = (G.HERE / "modulation_tests.bin").read_bytes()
    (count,) = struct.unpack_from("<I", blob, 0)
    off, n = 4, 0
    hdr = struct.Struct("<B5I")
    ramp = bytes(i & 0xFF for i in range(32))
    seen = []
    for _ in range(count):
        kind, sf, bw_khz, cr, _res, plen = hdr.unpack_from(blob, off)
        off += hdr.size
        payload = blob[off:off + plen]
        off += plen
        (nsamp,) = struct.unpack_from("<I", blob, off)
        off += 4
        ri = np.frombuffer(blob[off:off + 16 * nsamp], "<f8").reshape(nsamp, 2)
        off += 16 * nsamp
        iq = (ri[:, 0] + 1j * ri[:, 1]).astype(np.complex64)
        assert kind == 0
        np.testing.assert_array_equal(iq.view(np.uint64),
                                      oracle.modulate(oracle.encode(ramp), sf, bw_hz=1000 * bw_khz).view(np.uint64))
        r, syms, sync, _ = oracle.lora_demodulate(oracle.dechirp(iq, sf, bw_hz=1000 * bw_khz), sf)
        k, pay = oracle.lora_decode(syms)
        assert pay.tobytes() == payload
        assert (payload == ramp) == (bw_khz == 125)
        seen.append((sf, bw_khz, cr))
        n += 1
    assert off == len(blob)
    assert seen == [(7, 125, 1), (7, 125, 3), (8, 125, 1), (9, 250, 4), (10, 250, 3), (11, 500, 1), (12, 500, 1)]
