"""The HIP path against the committed golden fixtures (the reference's own
outputs, tests/golden/make_golden.py): every case, both APIs, both launch
paths, bit-exact symbols / sync word / cfo / time_offset / decoded bytes /
CRC flag / error status, plus the modulate known answers."""
import numpy as np
import pytest

import golden_cases as G

pytestmark = pytest.mark.gpu
LAUNCH = [0, 32]  # fused single launch, separate launches (lphy.F_UNFUSED)


def _dem(lphy, c):
    return lphy.Demodulator(c["sf"], c["bw"], 1, lphy.WINDOW_HANN if c["hann"] else lphy.WINDOW_NONE)


@pytest.mark.parametrize("launch", LAUNCH)
@pytest.mark.parametrize("name", G.case_names())
def test_demodulate_golden(oracle, lphy, name, launch):
    c = G.case(name)
    res = c["results"].get("demodulate")
    if res is None:
        pytest.skip("lora_demodulate-only case")
    iq = G.case_iq(oracle, c)
    d = _dem(lphy, c)
    syms, _, meta = d.demod_host(iq, 1, iq.size, lphy.MODE_DEMODULATE, launch)
    assert res["ret"] == syms.shape[1]
    np.testing.assert_array_equal(syms[0], G.expected_syms(c, "demodulate"))
    assert meta["sync_word"][0] == res["sync"]
    assert G.fbits(meta["cfo"][0]) == res["cfo"] and G.fbits(meta["time_offset"][0]) == res["toff"]
    n2 = syms.shape[1] & ~1
    rc, pay, m = d.decode_host(syms[0][:n2])
    assert rc == 0 and res["decode_ret"] == n2 // 2 and pay.tobytes().hex() == res["bytes"]
    assert m["crc_ok"] == res["crc_ok"]


@pytest.mark.parametrize("launch", LAUNCH)
@pytest.mark.parametrize("name", G.case_names())
def test_lora_demodulate_golden(oracle, lphy, name, launch):
    c = G.case(name)
    res = c["results"]["lora_demodulate"]
    iq = G.case_iq(oracle, c)
    d = _dem(lphy, c)
    flags = launch | (0 if c["scratch"] else lphy.F_NO_SCRATCH)
    runs = [(lphy.MODE_LORA_DEMODULATE, G.lora_input(oracle, c, iq))]
    if res["input"] == "dechirped":
        runs.append((lphy.MODE_DECHIRP_LORA_DEMODULATE, iq))  # dechirp fused on the GPU
    expect = G.expected_syms(c, "lora_demodulate")
    for mode, x in runs:
        syms, _, meta = d.demod_host(x, 1, x.size, mode, flags)
        if res["ret"] < 0:
            assert meta["status"][0] == res["ret"]
            continue
        assert meta["status"][0] == 0
        assert res["ret"] == syms.shape[1]
        np.testing.assert_array_equal(syms[0], expect)
        assert meta["sync_word"][0] == res["sync"]
        assert G.fbits(meta["cfo"][0]) == res["cfo"]
        assert G.fbits(meta["time_offset"][0]) == res["toff"]
        n2 = syms.shape[1] & ~1
        rc, pay, _ = d.decode_host(syms[0][:n2])
        assert rc == 0 and res["decode_ret"] == n2 // 2 and pay.tobytes().hex() == res["bytes"]


@pytest.mark.parametrize("m", G.MANIFEST["modulate"], ids=lambda m: m["name"])
def test_modulate_golden(lphy, m):
    from recipes import sha256
    out = lphy.Demodulator(m["sf"], m["bw"]).modulate_host(np.array(m["syms"], np.uint16), 1.0, m["sync"])
    assert out.size == m["samples"] and sha256(out) == m["sha256"]
