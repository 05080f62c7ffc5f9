"""Diagnostic: MN/MN weight-gradient-shaped GEMM (M = h, N = n*d, contraction over the batch) with the
activation operand's row stride h (a power of two) vs padded strides, in one process.
Usage: python tools/stride_bench.py [lib.so]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import crosscoder_amd  # noqa: F401,E402
from crosscoder_amd import _lib  # noqa: E402

B, n, d, h = 4096, 2, 2304, 16384
K = n * d
PEAK = 256 * 2.4e9 * 4096 / 1e12


def main():
    L = _lib.load(sys.argv[1]) if len(sys.argv) > 1 else _lib.load()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    C = torch.empty(h, K, device=dev)
    cases = {}
    for pa in (0, 64, 128):
        for pb in (0, 64):
            A = torch.randn(B, h + pa, device=dev, generator=g).to(torch.bfloat16)
            Bm = torch.randn(B, K + pb, device=dev, generator=g).to(torch.bfloat16)
            cases[f"lda h+{pa:3d} ldb K+{pb:2d}"] = (A, Bm)
    flop = 2.0 * B * K * h
    res = {}
    for _ in range(5):
        for name, (A, Bm) in cases.items():
            fn = lambda: L.cc_gemm_f32out(P(A), 1, A.shape[1], P(Bm), 1, Bm.shape[1], P(C), K, h, K, B, 1, st)  # noqa
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
        print(f"MN/MN {name}: median {med * 1e3:7.1f} us  {flop / med / 1e9:7.1f} TF/s ({flop / med / 1e9 / PEAK * 100:4.1f}%)")


if __name__ == "__main__":
    main()
