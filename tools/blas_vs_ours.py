"""Same-operand, interleaved timing of hipBLASLt (torch.matmul) against our GEMM kernels on the G1/G3
shape of config 2 (M = B = 4096, N = h = 16384, K = n*d = 4608, both operands K-contiguous, bf16 out)
and on the weight-gradient shape (M = h, N = K, contraction over B).  Diagnostic only.
Usage: python tools/blas_vs_ours.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import crosscoder_amd  # noqa: F401,E402
from crosscoder_amd import ops  # noqa: E402

B, n, d, h = 4096, 2, 2304, 16384
K = n * d
PEAK = 256 * 2.4e9 * 4096 / 1e12


def main():
    dev = torch.device("cuda:0")
    bf = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    r = lambda *s, sc=1.0: (torch.randn(*s, device=dev, generator=g) * sc).to(bf)  # noqa: E731
    x, W = r(B, K), r(h, K, sc=0.02)
    b = torch.zeros(h, device=dev, dtype=bf)
    acts = torch.relu(torch.matmul(x, W.t()))  # (G3's activation mask input)
    acts_t = torch.empty(h, B, device=dev, dtype=bf)
    out = torch.empty(B, h, device=dev, dtype=bf)
    xt = x.t().contiguous()
    gp_t = torch.relu(r(h, B))  # a [h][B] operand like g_pre^T
    dW = torch.empty(h, K, device=dev, dtype=bf)
    g_recon = r(B, K, sc=1e-3)  # G3's data: d_acts = g_recon . W_dec^T
    gp = torch.empty(h, B, device=dev, dtype=bf)
    tn = torch.rand(h, device=dev) * 0.1
    cases = {
        "hipBLASLt x.W^T": lambda: torch.matmul(x, W.t(), out=out),
        "hipBLASLt g_recon.W^T (G3 data)": lambda: torch.matmul(g_recon, W.t(), out=out),
        "ours G3 d_acts^T (G3 data)": lambda: ops.dacts_bwd_t(g_recon, W, acts, tn, 1e-4, gp),
        "ours G1 encode (bias+relu, bf16 out)": lambda: ops.encode_fwd(x, W, b, acts, True),
        "ours G1 encode + acts^T": lambda: ops.encode_fwd_t(x, W, b, acts, acts_t, True),
        "hipBLASLt g_pre^T.x (h x K, over B)": lambda: torch.matmul(gp_t, xt.t(), out=dW),
    }
    res = {k: [] for k in cases}
    for _ in range(3):
        for fn in cases.values():
            fn()
    torch.cuda.synchronize()
    for _ in range(6):
        for name, fn in cases.items():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                fn()
            e.record()
            torch.cuda.synchronize()
            res[name].append(s.elapsed_time(e) / 10)
    flop = 2.0 * B * K * h
    for name, ts in res.items():
        ts.sort()
        med = ts[len(ts) // 2]
        print(f"{name:45s} median {med * 1e3:7.1f} us  min {ts[0] * 1e3:7.1f} us  {flop / med / 1e9:7.1f} TF/s "
              f"({flop / med / 1e9 / PEAK * 100:4.1f}% of peak)", flush=True)


if __name__ == "__main__":
    main()
