"""The W_dec^T + decoder-norms pass alone (config 2: W_dec [16384][4608] bf16) across library builds, beside
a plain device copy of the same bytes (the HBM reference).  Usage: python tools/transpose_probe.py lib.so ..."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gemm_bench import load  # noqa: E402

h, n, d = 16384, 2, 2304
K = n * d


def timed(fn, reps=20):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    libs = [(os.path.basename(p), load(p)) for p in sys.argv[1:]]
    dev = torch.device("cuda:0")
    W = (torch.randn(h, K, device=dev) * 0.02).to(torch.bfloat16)
    Wt = torch.empty(K, h, device=dev, dtype=torch.bfloat16)
    cp = torch.empty_like(W)
    part = torch.empty(h * n * (d // 64), device=dev)
    norms, tot, inv = torch.empty(h, n, device=dev), torch.empty(h, device=dev), torch.empty(h, n, device=dev)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    nbytes = 2 * W.numel() * 2
    res = {}
    for rnd in range(7):
        res.setdefault("torch copy (same bytes)", []).append(timed(lambda: cp.copy_(W)))
        for name, L in libs:
            if rnd == 0:
                Wt.zero_()
                assert L.cc_transpose_dec_norms(P(W), h, n, d, P(Wt), P(part), P(norms), P(tot), P(inv), st) == 0
                torch.cuda.synchronize()
                assert torch.equal(Wt, W.t()), name
            res.setdefault(f"transpose {name}", []).append(
                timed(lambda: L.cc_transpose_b16(P(W), h, K, K, P(Wt), h, st)))
            res.setdefault(f"transpose+norms {name}", []).append(
                timed(lambda: L.cc_transpose_dec_norms(P(W), h, n, d, P(Wt), P(part), P(norms), P(tot), P(inv), st)))
    for k, v in res.items():
        v.sort()
        print(f"{k:40s} median {v[len(v) // 2]:6.1f} us  {nbytes / v[len(v) // 2] / 1e3:6.0f} GB/s")


if __name__ == "__main__":
    main()
