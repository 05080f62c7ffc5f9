"""Main-loop rate vs per-tile fixed cost of a GEMM, by sweeping the contraction length K at a fixed output shape:
T(K) = a + b K, fitted over K in {2304, 4608, 9216}.  b is the K loop's cost per 64-deep K step and tile wave, a the
K-independent part (prologue, epilogue element work, output stores).  Compares hipBLASLt (torch.matmul), the
product's G1 encode (8-wave ping-pong + the FAST bias / ReLU / colsum / l0 epilogue) and the 4-wave experiment
(tools/exp/g4h.hip: libs given as arguments).  Diagnostic only.
Usage: python tools/gemm_ksweep.py [tools/exp/libg4h_*.so ...]"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import crosscoder_amd  # noqa: F401,E402
from crosscoder_amd import ops  # noqa: E402


def timed(fn, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) / reps * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    dev = torch.device("cuda:0")
    bf = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    M, N = 4096, 16384
    libs = []
    for p in sys.argv[1:]:
        L = ctypes.CDLL(p)
        L.g4_gemm_bf16.restype = ctypes.c_int
        L.g4_gemm_bf16.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int64] * 6 + [ctypes.c_void_p]
        libs.append((os.path.basename(p), L))
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    res = {}
    for K in (2304, 4608, 9216):
        A = (torch.randn(M, K, device=dev, generator=g)).to(bf)
        Bm = (torch.randn(N, K, device=dev, generator=g) * 0.02).to(bf)
        C = torch.empty(M, N, device=dev, dtype=bf)
        b = torch.zeros(N, device=dev, dtype=bf)
        cases = {"hipBLASLt": lambda: torch.matmul(A, Bm.t(), out=C),
                 "ours G1 encode (pp)": lambda: ops.encode_fwd(A, Bm, b, C, True)}
        for name, L in libs:
            cases[name] = (lambda L=L: L.g4_gemm_bf16(P(A), P(Bm), P(C), M, N, K, K, K, N, st))
        for name, fn in cases.items():
            res.setdefault(name, {})[K] = timed(fn)
    for name, r in res.items():
        ks = sorted(r)
        # least squares over the three points
        n = len(ks)
        mk = sum(ks) / n
        mt = sum(r[k] for k in ks) / n
        b = sum((k - mk) * (r[k] - mt) for k in ks) / sum((k - mk) ** 2 for k in ks)
        a = mt - b * mk
        print(f"{name:28s} " + "  ".join(f"K={k}: {r[k]:7.1f} us" for k in ks) +
              f"   fit: {a:6.1f} us + {b * 4608:6.1f} us per K=4608 (= {b * 64 * 1e3 / 4:6.1f} ns per K step per tile wave)",
              flush=True)


if __name__ == "__main__":
    main()
