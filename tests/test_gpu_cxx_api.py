"""The lora_phy:: C++ drop-in (include/lora_phy/phy.hpp + liblora_phy_amd.so,
GPU behind the C ABI) against the reference library: the same probe source
(tests/cpp/lora_phy_api_probe.cpp) is built against both and must print
identical transcripts — return codes, symbols, sync words, cfo / time_offset
bits, CRC flags and payload bytes over the scenarios of the reference's own
tests (error_code, roundtrip, no_alloc, e2e_chain profiles, bit_exact on
modulation_tests.bin, equal_power_bin, scratch_buffer_error,
odd_symbol_count, sync_word) and impaired frames."""
import os
import subprocess
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "lora-sdr-lightweight-standalone-library-clean_amd"
REF_PROBE = ROOT / "oracle" / "_ref" / "lora_phy_api_probe_ref"


def prod_env(**kw):
    """The probes run the drop-in with the library's own launch choices (a
    packet at a time takes the separate launches by default,
    fused_min_frames)."""
    env = {k: v for k, v in os.environ.items() if k not in ("LPHY_FUSED_MIN_FRAMES", "LD_LIBRARY_PATH")}
    env.update(kw)
    return env


def fused_env():
    """The same drop-in with every call on the fused kernels: the test build
    of liblphy_hip.so (lib/test/, found first through LD_LIBRARY_PATH by
    liblora_phy_amd.so) reads LPHY_FUSED_MIN_FRAMES; the product library
    takes no launch choice from the environment."""
    return prod_env(LD_LIBRARY_PATH=str(PKG / "lib" / "test"), LPHY_FUSED_MIN_FRAMES="0")


def loaded_hip_lib(exe, env) -> str:
    """The liblphy_hip.so the dynamic loader picks for `exe` under `env`."""
    out = subprocess.run(["ldd", str(exe)], capture_output=True, text=True, env=env, check=True).stdout
    return next(l.split("=>")[1].split("(")[0].strip() for l in out.splitlines() if "liblphy_hip.so" in l)


def test_cxx_api_transcript_matches_reference(tmp_path):
    if not REF_PROBE.exists():
        pytest.skip("reference probe not built (oracle/Makefile probe)")
    exe = tmp_path / "probe_amd"
    subprocess.run(["g++", "-O2", "-std=gnu++17", "-ffp-contract=off", f"-I{ROOT / 'include'}",
                    "-o", str(exe), str(ROOT / "tests" / "cpp" / "lora_phy_api_probe.cpp"),
                    f"-L{PKG / 'lib'}", "-llora_phy_amd", f"-Wl,-rpath,{PKG / 'lib'}"], check=True)
    golden = str(ROOT / "tests" / "golden")
    ref = subprocess.run([str(REF_PROBE), golden], capture_output=True, text=True, timeout=300)
    assert ref.returncode == 0, ref.stderr
    b = ref.stdout.splitlines()
    # default launch choices, then the fused kernels forced for every call
    assert loaded_hip_lib(exe, prod_env()) == str(PKG / "lib" / "liblphy_hip.so")
    assert loaded_hip_lib(exe, fused_env()) == str(PKG / "lib" / "test" / "liblphy_hip.so")
    for env in (prod_env(), fused_env()):
        ours = subprocess.run([str(exe), golden], capture_output=True, text=True, timeout=300, env=env)
        assert ours.returncode == 0, ours.stderr
        a = ours.stdout.splitlines()
        assert len(a) == len(b) and len(b) >= 25
        bad = [(x, y) for x, y in zip(a, b) if x != y]
        assert not bad, "\n".join(f"ours: {x[:300]}\nref:  {y[:300]}" for x, y in bad[:5])


LW_REF_PROBE = ROOT / "oracle" / "_ref" / "lorawan_api_probe_ref"


def test_lorawan_api_transcript_matches_reference(tmp_path):
    """lorawan:: drop-in (include/lorawan/lorawan.hpp, GPU MIC + decode)
    against the reference's lorawan.cpp + tiny-AES: the same probe
    (tests/cpp/lorawan_api_probe.cpp) built against both."""
    if not LW_REF_PROBE.exists():
        pytest.skip("reference lorawan probe not built (oracle/Makefile lwprobe)")
    exe = tmp_path / "lwprobe_amd"
    subprocess.run(["g++", "-O2", "-std=gnu++17", f"-I{ROOT / 'include'}", "-o", str(exe),
                    str(ROOT / "tests" / "cpp" / "lorawan_api_probe.cpp"), f"-L{PKG / 'lib'}", "-llora_phy_amd",
                    f"-Wl,-rpath,{PKG / 'lib'}"], check=True)
    ours = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=prod_env())
    assert ours.returncode == 0, ours.stderr
    ref = subprocess.run([str(LW_REF_PROBE)], capture_output=True, text=True, timeout=300)
    assert ref.returncode == 0, ref.stderr
    a, b = ours.stdout.splitlines(), ref.stdout.splitlines()
    assert len(a) == len(b) and len(b) >= 400
    assert b[0] == "mic kat 82b5c3d6"
    bad = [(x, y) for x, y in zip(a, b) if x != y]
    assert not bad, "\n".join(f"ours: {x[:300]}\nref:  {y[:300]}" for x, y in bad[:5])


T_REF_PROBE = ROOT / "oracle" / "_ref" / "lora_phy_threads_probe_ref"


@pytest.mark.parametrize("threads,sf,frames", [(2, 9, 10), (4, 7, 8), (2, 12, 3)])
def test_cxx_api_threads_match_reference(tmp_path, threads, sf, frames):
    """Separate workspaces on separate threads at the same SF, concurrently
    (tests/cpp/lora_phy_threads_probe.cpp): the drop-in gives each workspace
    its own context (stream + staging) at init, so the threads run side by
    side, and each thread's transcript equals the reference's."""
    if not T_REF_PROBE.exists():
        pytest.skip("reference threads probe not built (oracle/Makefile tprobe)")
    exe = tmp_path / "tprobe_amd"
    subprocess.run(["g++", "-O2", "-std=gnu++17", "-ffp-contract=off", f"-I{ROOT / 'include'}",
                    "-o", str(exe), str(ROOT / "tests" / "cpp" / "lora_phy_threads_probe.cpp"),
                    f"-L{PKG / 'lib'}", "-llora_phy_amd", f"-Wl,-rpath,{PKG / 'lib'}", "-lpthread"], check=True)
    args = [str(threads), str(sf), str(frames)]
    ours = subprocess.run([str(exe)] + args, capture_output=True, text=True, timeout=300, env=prod_env())
    assert ours.returncode == 0, ours.stderr
    ref = subprocess.run([str(T_REF_PROBE)] + args, capture_output=True, text=True, timeout=300)
    assert ref.returncode == 0, ref.stderr
    a, b = ours.stdout.splitlines(), ref.stdout.splitlines()
    assert len(b) == threads * frames * 2 and len(a) == len(b)
    bad = [(x, y) for x, y in zip(a, b) if x != y]
    assert not bad, "\n".join(f"ours: {x[:300]}\nref:  {y[:300]}" for x, y in bad[:5])
