"""A/B timing of cc_adam_step over the config-2 parameter arena (151,015,936 bf16 elements) across
library builds, interleaved in one process.  Usage: python tools/adam_bench.py lib1.so [lib2.so ...]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crosscoder_amd._lib import SIGNATURES  # noqa: E402

NUMEL = 2 * 16384 * 4608 + 16384 + 4608


def load(path):
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        f = getattr(lib, name, None)  # (an older build may lack newer entry points)
        if f is not None:
            f.restype, f.argtypes = res, args
    return lib


def main():
    libs = [(os.path.basename(p), load(p)) for p in sys.argv[1:]]
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    p = (torch.randn(NUMEL, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    gr = (torch.randn(NUMEL, device=dev, generator=g) * 1e-4).to(torch.bfloat16)
    m = (torch.randn(NUMEL, device=dev, generator=g) * 1e-5).to(torch.bfloat16)
    v = (torch.rand(NUMEL, device=dev, generator=g) * 1e-8).to(torch.bfloat16)
    coef = torch.ones(1, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    res = {}
    for rnd in range(6):
        for name, L in libs:
            fn = lambda: L.cc_adam_step(P(p), P(gr), P(m), P(v), NUMEL, P(coef), 5e-5, 0.9, 0.999, 1e-8, 7, 0, 1, st)  # noqa
            assert fn() == 0
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                fn()
            e.record()
            torch.cuda.synchronize()
            res.setdefault(name, []).append(s.elapsed_time(e) / 10)
    for name, ts in res.items():
        ts.sort()
        med = ts[len(ts) // 2]
        print(f"adam {name:28s} median {med*1e3:7.1f} us  min {ts[0]*1e3:7.1f} us  {14 * NUMEL / med / 1e9:6.2f} TB/s")


if __name__ == "__main__":
    main()
