"""The Python binding refuses buffers the C ABI cannot check (lphy.py
_dev_buf): host memory, the wrong device, non-contiguous views, the wrong
element size, or fewer bytes than the call reads / writes.  The CPU tests
exercise the checks alone; the GPU test drives them through a live context."""
import numpy as np
import pytest
import torch


def test_dev_buf_rejects_host_memory(lphy):
    with pytest.raises(ValueError, match="device tensor"):
        lphy._dev_buf(np.zeros(8, np.float32), "iq", 0, 32)
    with pytest.raises(ValueError, match="cpu"):
        lphy._dev_buf(torch.zeros(8), "iq", 0, 32)
    with pytest.raises(ValueError, match="device tensor"):
        lphy._dev_buf(None, "payload", 0, 1)


@pytest.mark.gpu
def test_demod_batch_argument_checks(lphy):
    dev = torch.device("cuda", 0)
    d = lphy.Demodulator(7)
    frames, fs = 4, 66 * 128
    per = d.syms_per_frame(fs, lphy.MODE_LORA_DEMODULATE)
    iq = torch.zeros(frames * fs * 2, dtype=torch.float32, device=dev)
    syms = torch.zeros(frames * per, dtype=torch.int16, device=dev)
    meta = torch.zeros(frames * 32, dtype=torch.uint8, device=dev)
    pay = torch.zeros(frames * (per // 2), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    d.demod_batch(iq, frames, fs, syms, meta, lphy.MODE_LORA_DEMODULATE, lphy.F_DECODE, payload=pay,
                  stream=st)
    torch.cuda.synchronize()
    bad = [
        dict(iq=iq[:-2]),                                   # IQ short by one sample
        dict(syms=torch.zeros(frames * per, dtype=torch.int32, device=dev)),  # 4-byte symbols
        dict(syms=syms[: frames * per - 1]),                # one symbol short
        dict(meta=meta[:-1]),                               # one meta byte short
        dict(payload=pay[:-1]),                             # one payload byte short
        dict(payload=None),                                 # F_DECODE without payload
        dict(iq=iq.cpu()),                                  # host tensor
        dict(syms=torch.zeros(2 * frames * per, dtype=torch.int16, device=dev)[::2]),  # strided
    ]
    for kw in bad:
        args = dict(iq=iq, syms=syms, meta=meta, payload=pay)
        args.update(kw)
        with pytest.raises(ValueError):
            d.demod_batch(args["iq"], frames, fs, args["syms"], args["meta"],
                          lphy.MODE_LORA_DEMODULATE, lphy.F_DECODE, payload=args["payload"], stream=st)
    with pytest.raises(ValueError):
        d.decode_batch(syms, frames, per, pay[:-1], meta, stream=st)
    with pytest.raises(ValueError):
        d.modulate_batch(syms, frames, per, iq[:-2], stream=st)
