"""The reference's own test harness and runners against the drop-in
(VERDICT r4 missing 2).  oracle/Makefile `harness` compiles the UNMODIFIED
reference sources - tests/*.cpp with -Dmain=<name>_main and test_main.cpp,
as its CMakeLists.txt:37-64 does, and runners/{rx,tx}_runner.cpp
(CMakeLists.txt:28-33) - twice: against include/ + liblora_phy_amd.so (the
GPU drop-in) and against the reference's own sources (the CPU library), plus
one executable per test so that sync_word_test's heap overflow
aborts only itself.  Both run here from one working directory holding copies
of the data files the tests open (tests/golden/ref_harness: the reference's
tests/profiles.yaml and vectors/golden/*.b64, and the committed
modulation_tests.bin, which the reference tree lacks).

Asserted: every test's exit status is the reference build's, and equals
SURVEY §0.8's pattern with bit_exact now passing on the committed
modulation_tests.bin (its BW250/500 records hold the reference's own decode,
tests/golden/make_golden.py); the deterministic tests print the same lines;
tx_runner | rx_runner prints the reference's payload hex.

sync_word_test writes lora_modulate's 256 samples (2 sync symbols at SF 7)
into a 255-sample vector (sync_word_test.cpp:27-29): undefined behaviour
whose outcome depends on the heap layout, so the drop-in's exit status is
not asserted for it.  Instead its fault is pinned (VERDICT r5
weak 3): every test executable carries tests/cpp/crash_trace.cpp, whose
fatal-signal backtrace must show the fault inside the C library's heap
code called straight from sync_word_test_main (the test's next allocation or
free after the overflow), with no frame in liblphy_hip.so or
liblora_phy_amd.so; and both builds of the test under AddressSanitizer
(oracle/Makefile harness_asan, recovering) must report that one overflowing
write, into the test's own 2040-byte buffer, from lora_modulate - and no
other memory error."""
import os
import re
import shutil
import subprocess
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]
H = ROOT / "oracle" / "_ref" / "harness"
DATA = ROOT / "tests" / "golden" / "ref_harness"

# SURVEY §0.8 (reference, measured), bit_exact with the file present
EXPECTED = {
    "bit_exact_test": 0,
    "e2e_chain_test": 1,          # the 4 BW250/500 profiles do not round-trip
    "no_alloc_test": 0,
    "performance_test": 0,
    "roundtrip_test": 0,
    "whitening_test": 0,
    "equal_power_bin_test": 0,
    "sync_word_test": None,       # overflows its heap buffer: aborts (non-zero)
    "error_code_test": 1,         # error_code_test.cpp:101, :159
    "odd_symbol_count_test": 0,
    "scratch_buffer_error_test": 0,
    "lorawan_mic_test": 0,
}


def _need():
    for side in ("amd", "ref"):
        if not (H / side / "lora_phy_tests").exists():
            pytest.skip("reference harness not built (make -C oracle harness, needs /root/reference)")


@pytest.fixture
def workdir(tmp_path):
    _need()
    shutil.copytree(DATA, tmp_path, dirs_exist_ok=True)
    shutil.copy(ROOT / "tests" / "golden" / "modulation_tests.bin", tmp_path / "vectors" / "golden")
    return tmp_path


def _run(exe, cwd, timeout=300, **kw):
    return subprocess.run([str(exe)], cwd=cwd, capture_output=True, text=True, timeout=timeout, **kw)


LIBS = ("liblphy_hip.so", "liblora_phy_amd.so")


def _fault_frames(trace: str):
    """The backtrace crash_trace.cpp wrote: the frames after the handler's own
    and libc's signal trampoline."""
    lines = [l for l in trace.splitlines() if l and not l.startswith("lphy-crash-trace")]
    return lines[2:]  # (the handler, the kernel's sigreturn frame in libc)


def _assert_heap_fault_in_test(trace: str, ctx: str):
    """The fault happened in the C library's heap code (malloc / free /
    operator new, or abort from there) called directly by sync_word_test_main:
    the overflow's aftermath in the test's own allocation, no frame of ours."""
    assert "lphy-crash-trace: signal" in trace and "lphy-crash-trace: end" in trace, ctx
    frames = _fault_frames(trace)
    assert not any(lib in f for f in frames for lib in LIBS), f"{ctx}: a frame in the drop-in\n{trace}"
    k = next(i for i, f in enumerate(frames) if "sync_word_test_main" in f)
    above = frames[:k]  # (innermost first)
    assert above and all("libc.so" in f or "libstdc++.so" in f for f in above), f"{ctx}\n{trace}"
    assert any(re.search(r"\((malloc|free|_Znwm|cfree)\+", f) for f in above), f"{ctx}\n{trace}"


@pytest.mark.parametrize("name", sorted(EXPECTED))
def test_reference_test_against_drop_in(workdir, name):
    ours = _run(H / "amd" / name, workdir)
    ref = _run(H / "ref" / name, workdir)
    want = EXPECTED[name]
    ctx = f"{name}: ours rc {ours.returncode}\n{ours.stdout[-2000:]}{ours.stderr[-2000:]}\n" \
          f"ref rc {ref.returncode}\n{ref.stdout[-1000:]}{ref.stderr[-1000:]}"
    if want is None:
        # undefined behaviour (above): the reference build aborts; whether and
        # where the drop-in's process dies depends on its heap layout, so the
        # fault site is pinned instead of the status
        assert ref.returncode != 0, ctx
        return
    assert ref.returncode == want, ctx
    assert ours.returncode == want, ctx
    if name != "performance_test":  # (timing lines)
        assert ours.stdout.splitlines() == ref.stdout.splitlines(), ctx
        assert ours.stderr.splitlines() == ref.stderr.splitlines(), ctx
    else:
        lines = [l for l in ours.stdout.splitlines() if " pps, " in l]
        assert len(lines) == 7, ctx  # one per profile of tests/profiles.yaml


def test_lora_phy_tests_binary(workdir):
    """The reference's single test executable (test_main.cpp runs every
    test in turn).  sync_word_test.cpp:27-29 writes 256 samples into 255:
    glibc reports it as "malloc(): corrupted top size" (abort) under the
    reference build; under the drop-in's heap layout it has surfaced as a
    segfault or "double free" instead.  The reference build dies by that
    signal; the tests before sync_word report on stderr (unbuffered) the
    same lines in both builds; where a build dies, its fault lies in the
    heap code called from sync_word_test_main (crash_trace.cpp)."""
    out = {}
    for side in ("amd", "ref"):
        trace = workdir / f"trace_{side}.txt"
        p = _run(H / side / "lora_phy_tests", workdir, env=dict(os.environ, LPHY_CRASH_TRACE=str(trace)))
        out[side] = (p, trace.read_text() if trace.exists() else "")
    ours, ref = out["amd"][0], out["ref"][0]
    assert ref.returncode < 0, (ref.returncode, ref.stderr[-2000:])
    strip = lambda s: [l for l in s.splitlines() if "corrupted" not in l and "double free" not in l]
    a, b = strip(ours.stderr), strip(ref.stderr)
    # (a drop-in that survives the overflow goes on to the later tests)
    assert a[:len(b)] == b, (ours.stderr[-3000:], ref.stderr[-3000:])
    for side, (p, trace) in out.items():
        if p.returncode < 0:
            _assert_heap_fault_in_test(trace, f"lora_phy_tests ({side}) rc {p.returncode}")


def test_sync_word_fault_pinned(workdir):
    """sync_word_test alone (oracle/Makefile's per-test executable), both
    builds: a fatal signal's backtrace (crash_trace.cpp) lies in the heap
    code called from sync_word_test_main, never in the drop-in's libraries."""
    for side in ("amd", "ref"):
        trace = workdir / f"trace_sw_{side}.txt"
        p = _run(H / side / "sync_word_test", workdir, env=dict(os.environ, LPHY_CRASH_TRACE=str(trace)))
        if side == "ref":
            assert p.returncode < 0, p.stderr[-2000:]
        if p.returncode < 0:
            _assert_heap_fault_in_test(trace.read_text(), f"sync_word_test ({side}) rc {p.returncode}")


def _asan_reports(text: str):
    return ["ERROR: AddressSanitizer" + r for r in text.split("ERROR: AddressSanitizer")[1:]]


def test_sync_word_overflow_under_asan(workdir):
    """Both builds of sync_word_test under AddressSanitizer (recovering: the
    overflowing bytes land in ASan's redzone, nothing is corrupted): every
    report is a heap-buffer-overflow WRITE by lora_modulate (the reference's
    genChirp loop; the drop-in's copy of the packet's samples out of its
    pinned staging, 2,048 B) just past the test's own 2,040-byte vector
    (255 samples, sync_word_test.cpp:27), called from sync_word_test.cpp:28;
    no other memory error; and the test then reaches the same verdict in
    both builds."""
    rc = {}
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:protect_shadow_gap=0:halt_on_error=0:symbolize=1")
    for side in ("amd", "ref"):
        exe = H / "asan" / side / "sync_word_test"
        if not exe.exists():
            pytest.skip("oracle/_ref/harness/asan not built (make -C oracle harness)")
        p = _run(exe, workdir, env=env)
        reps = _asan_reports(p.stderr)
        ctx = f"{side}: rc {p.returncode}\n{p.stderr[-6000:]}"
        assert reps, ctx
        for r in reps:
            assert "heap-buffer-overflow" in r and re.search(r"WRITE of size \d+", r), ctx
            head = r.split("allocated by thread")[0]
            assert "lora_modulate" in head and "sync_word_test.cpp:28" in head, ctx
            assert re.search(r"located \d+ bytes (after|to the right of) 2040-byte region", r), ctx
            assert "sync_word_test.cpp:27" in r.split("allocated by thread")[1], ctx
        if side == "amd":
            assert "lphy_hip_modulate_host" in reps[0], ctx  # (the pinned-mirror copy)
        rc[side] = p.returncode
    assert rc["amd"] == rc["ref"], rc


@pytest.mark.parametrize("payload,sf", [("48656c6c6f", 7), ("48656c6c6f", 9), ("deadbeef00112233", 8),
                                        ("00", 12), ("0123456789abcdef0123456789abcdef", 10)])
def test_tx_rx_runner_pipe(workdir, payload, sf):
    out = {}
    for side in ("amd", "ref"):
        tx = subprocess.run([str(H / side / "tx_runner"), f"--payload={payload}", f"--sf={sf}", "--stdout"],
                            cwd=workdir, capture_output=True, timeout=120)
        assert tx.returncode == 0, tx.stderr
        rx = subprocess.run([str(H / side / "rx_runner"), f"--sf={sf}", "--report-offsets"], input=tx.stdout,
                            cwd=workdir, capture_output=True, timeout=120)
        assert rx.returncode == 0, rx.stderr
        out[side] = (tx.stdout, rx.stdout.decode())
    assert out["amd"][0] == out["ref"][0]  # the IQ, byte for byte
    assert out["amd"][1] == out["ref"][1], out
    if payload == "48656c6c6f" and sf == 7:
        assert out["ref"][1].splitlines()[0] == "Payload: 0ca9a0a0a3"
