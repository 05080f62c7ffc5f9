"""Timing of the stand-alone loss kernel (latent-sharded step: fp32 reconstruction -> loss row terms, g_recon
and g_recon^T) at config-2 shapes across library builds, interleaved in one process.
Usage: python tools/loss_bench.py lib1.so [lib2.so ...]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gemm_bench import load  # noqa: E402

B, n, d = 4096, 2, 2304
K = n * d


def main():
    libs = [(os.path.basename(p), load(p)) for p in sys.argv[1:]]
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    recon = torch.randn(B, K, device=dev, generator=g)
    x = torch.randn(B, K, device=dev, generator=g).to(torch.bfloat16)
    b_dec = torch.randn(K, device=dev, generator=g).to(torch.bfloat16)
    mu = torch.randn(K, device=dev, generator=g)
    gr = torch.empty(B, K, device=dev, dtype=torch.bfloat16)
    grt = torch.empty(K, B, device=dev, dtype=torch.bfloat16)
    rp = torch.empty(2 * n * 8 * B, device=dev)
    cp = torch.empty(B // 32 + 1, K, device=dev)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    nbytes = B * K * (4 + 2 + 2 + 2)
    outs = {}
    res = {}
    for rnd in range(7):
        for name, L in libs:
            for rows in (B, B // 2):
                fn = lambda: L.cc_loss_fwd_bwd_rows_t(P(recon), P(b_dec), P(x), P(mu), P(gr), P(grt), P(rp), P(cp),  # noqa: E731
                                                      2.0 / B, 0, rows, B, n, d, 1, st)
                assert fn() == 0
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(20):
                    fn()
                e.record()
                torch.cuda.synchronize()
                res.setdefault((name, rows), []).append(s.elapsed_time(e) / 20)
            if rnd == 0:
                outs[name] = (gr.clone(), grt.clone(), rp.clone(), cp.clone())
    ref = next(iter(outs.values()))
    for (name, rows), ts in sorted(res.items()):
        ts.sort()
        med = ts[len(ts) // 2]
        same = all(torch.equal(a, b) for a, b in zip(outs[name], ref))
        print(f"loss rows {rows:5d} {name:28s} median {med * 1e3:6.1f} us  min {ts[0] * 1e3:6.1f} us  "
              f"{nbytes * rows / B / med / 1e6:6.0f} GB/s  outputs identical to the first lib: {same}")


if __name__ == "__main__":
    main()
