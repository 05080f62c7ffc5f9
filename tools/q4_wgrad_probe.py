"""Probe: is the 4-wave assembly K loop (tools/exp/libg4a*.so: q4_kloop + a plain bf16 store epilogue) faster than
the ping-pong on the weight-gradient shape, where the product runs dW_dec and dW_enc as ONE launch of 2 x 1152 tiles
(9 full waves)?  A single 1152-tile launch is 4.5 waves, so the standalone comparison is made at the dual launch's
tile count: q4 on M = 2 h rows (2304 tiles) against the product's cc_wgrad_both_t (the same two GEMMs, pp dual launch,
its epilogues incl. the L1 term, squared sums and transposed operands).  Timing only; interleaved, medians.
Usage: python tools/q4_wgrad_probe.py tools/exp/libg4a.so tools/exp/libg4ans.so"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import crosscoder_amd  # noqa: F401,E402
from crosscoder_amd import ops  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    bf = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    B, n, d, h = 4096, 2, 2304, 16384
    K = n * d
    r = lambda *s, sc=1.0: (torch.randn(*s, device=dev, generator=g) * sc).to(bf)  # noqa: E731
    actsT, g_reconT, g_preT, xT = r(h, B), r(K, B, sc=1e-3), r(h, B, sc=1e-3), r(K, B)
    W = r(h, K, sc=0.05)
    norms = torch.rand(h, n, device=dev) + 0.5
    colsum = torch.rand(h, device=dev)
    gd, ge = torch.empty(h, K, device=dev, dtype=bf), torch.empty(h, K, device=dev, dtype=bf)
    sq = torch.empty(ops.wgrad_parts(h, K, bf), device=dev)
    sq2 = torch.empty_like(sq)
    cases = {"pp dual (cc_wgrad_both_t)": lambda: ops.wgrad_both_t(actsT, g_reconT, W, norms, colsum, 1e-4, gd, sq,
                                                                    g_preT, xT, ge, sq2, n, d)}
    A2 = torch.cat([actsT, g_preT], 0)  # [2h][B]: dW_dec's then dW_enc's rows, contraction over B
    C2 = torch.empty(2 * h, K, device=dev, dtype=bf)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    for p in sys.argv[1:]:
        L = ctypes.CDLL(p)
        L.g4_gemm_bf16.restype = ctypes.c_int
        L.g4_gemm_bf16.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int64] * 6 + [ctypes.c_void_p]
        # (one operand for both halves: x^T stands in for g_recon^T -- the loop's timing does not depend on it)
        cases[f"q4 {os.path.basename(p)} M=2h"] = (lambda L=L: L.g4_gemm_bf16(P(A2), P(xT), P(C2), 2 * h, K, B, B, B, K,
                                                                               st))
    res = {k: [] for k in cases}
    for fn in cases.values():
        for _ in range(3):
            fn()
    torch.cuda.synchronize()
    for _ in range(6):
        for name, fn in cases.items():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(5):
                fn()
            e.record()
            torch.cuda.synchronize()
            res[name].append(s.elapsed_time(e) / 5)
    flop = 2 * 2.0 * h * K * B
    for name, ts in res.items():
        ts.sort()
        med = ts[len(ts) // 2]
        print(f"{name:36s} median {med * 1e3:7.1f} us  min {ts[0] * 1e3:7.1f} us  {flop / med / 1e9:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
