"""Ceiling check: torch.matmul (hipBLASLt) on the five step-GEMM shapes of config 2, random
bf16 operands, in the same operand layouts the step's kernels read, next to our kernels
(tools/gemm_bench.py).  Diagnostic only -- the product never calls hipBLASLt.

  python tools/blas_ref.py [B n d h]
"""
import sys

import torch

B, n, d, h = (int(v) for v in sys.argv[1:5]) if len(sys.argv) >= 5 else (4096, 2, 2304, 16384)
K = n * d
PEAK = 256 * 2.4e9 * 4096 / 1e12


def timed(fn, reps=10):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) / reps)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    dev = torch.device("cuda:0")
    bf = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    r = lambda *s, sc=1.0: (torch.randn(*s, device=dev, generator=g) * sc).to(bf)  # noqa: E731
    x, W_enc, W_dec = r(B, K), r(h, K, sc=0.02), r(h, K, sc=0.02)
    acts = torch.relu(r(B, h))
    g_recon, g_pre = r(B, K, sc=1e-3), r(B, h, sc=1e-3)
    W_dec_t, acts_t, g_recon_t, g_pre_t, x_t = (t.t().contiguous() for t in (W_dec, acts, g_recon, g_pre, x))
    cases = {
        # name: (fn, flop)  -- bf16 out unless noted; KC/KC = both operands contraction-contiguous
        "G1 x.W_enc^T (KC/KC, bf16 out)": lambda: torch.matmul(x, W_enc.t()),
        "G2 acts.W_dec_t^T (KC/KC)": lambda: torch.matmul(acts, W_dec_t.t()),
        "G2 acts.W_dec (MN, bf16 out)": lambda: torch.matmul(acts, W_dec),
        "G3 g_recon.W_dec^T (KC/KC)": lambda: torch.matmul(g_recon, W_dec.t()),
        "G4 acts_t.g_recon_t^T (KC/KC)": lambda: torch.matmul(acts_t, g_recon_t.t()),
        "G5 g_pre_t.x_t^T (KC/KC)": lambda: torch.matmul(g_pre_t, x_t.t()),
        "G4 acts^T.g_recon (MN/MN)": lambda: torch.matmul(acts.t(), g_recon),
    }
    flop = 2.0 * B * K * h
    for name, fn in cases.items():
        try:
            ms = timed(fn)
        except Exception as e:  # noqa: BLE001
            print(f"{name:40s} failed: {e}")
            continue
        print(f"{name:40s} {ms*1e3:8.1f} us  {flop/ms/1e9:7.1f} TF/s  ({flop/ms/1e9/PEAK*100:4.1f}% of peak)", flush=True)


if __name__ == "__main__":
    main()
