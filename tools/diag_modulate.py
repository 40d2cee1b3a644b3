"""Diagnostic: GPU lora_modulate vs CPU oracle vs compiled reference."""
import sys, os
sys.path.insert(0, "tests"); sys.path.insert(0, "lora-sdr-lightweight-standalone-library-clean_amd")
import numpy as np
import lphy
from checkers import Oracle, Reference
flags = open("/proc/cpuinfo").read().split("flags")[1].split("\n")[0]
print("cpu fma:", " fma " in flags, "avx2:", " avx2 " in flags, open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0])
o = Oracle(); r = Reference()
rng = np.random.default_rng(3)
for sf, bw in [(7, 125000), (9, 250000), (12, 500000), (2, 125000)]:
    syms = rng.integers(0, 256, 10, dtype=np.uint16)
    for rep in range(3):
        a = lphy.Demodulator(sf, bw).modulate_host(syms, 1.0, 0x34)
        b = o.modulate(syms, sf, bw_hz=bw, sync=0x34)
        c = r.modulate(syms, sf, bw_hz=bw, sync=0x34)
        print(sf, bw, rep, "gpu==oracle", np.array_equal(a.view(np.uint32), b.view(np.uint32)),
              "oracle==ref", np.array_equal(b.view(np.uint32), c.view(np.uint32)),
              "first diff", int(np.argmax(a.view(np.uint32) != b.view(np.uint32))))
