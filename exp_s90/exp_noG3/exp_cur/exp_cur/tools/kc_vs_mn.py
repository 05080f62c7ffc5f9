"""Diagnostic: the weight-gradient GEMM shape (16384 x 4608, contraction 4096) as MN/MN (operands
[B][h], [B][K] as the step stores them) vs KC/KC (operands transposed to [h][B], [K][B]).
Usage: python tools/kc_vs_mn.py"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import crosscoder_amd  # noqa: F401,E402
from crosscoder_amd import _lib  # noqa: E402

B, K, h = 4096, 4608, 16384
PEAK = 256 * 2.4e9 * 4096 / 1e12


def main():
    L = _lib.load()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    bf = torch.bfloat16
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    acts = torch.relu(torch.randn(B, h, device=dev, generator=g)).to(bf)  # [B][h]
    grec = (torch.randn(B, K, device=dev, generator=g) * 1e-3).to(bf)     # [B][K]
    actsT = acts.t().contiguous()                                         # [h][B]
    grecT = grec.t().contiguous()                                         # [K][B]
    mask = torch.ones(h, K, device=dev, dtype=bf)
    out = torch.empty(h, K, device=dev, dtype=bf)
    tn = torch.zeros(K, device=dev)
    parts = torch.empty(1 << 21, device=dev)
    cases = {
        "MN/MN wgrad_enc (no L1)": lambda: L.cc_wgrad_enc(P(acts), P(grec), P(out), P(parts), B, h, K, 1, st),
        # KC/KC through the d_acts entry: rows = h (as 'B'), cols = K (as 'h'), contraction = B (as 'K')
        "KC/KC d_acts-shaped": lambda: L.cc_dacts_bwd(P(actsT), P(grecT), P(mask), P(tn), 0.0, P(out), P(parts), h, B,
                                                      K, 1, st),
    }
    flop = 2.0 * B * K * h
    res = {}
    for _ in range(5):
        for name, fn in cases.items():
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
        print(f"{name:28s} median {med * 1e3:7.1f} us  {flop / med / 1e9:7.1f} TF/s ({flop / med / 1e9 / PEAK * 100:4.1f}%)")


if __name__ == "__main__":
    main()
