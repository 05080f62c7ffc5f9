"""A/B timing of the step's HBM-bound prep / loss kernels (config-2 shapes) across library builds,
interleaved in ONE process.  Usage: python tools/small_bench.py lib1.so [lib2.so ...]
Prints each kernel's median time and the HBM rate of its algorithmic bytes."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import crosscoder_amd  # noqa: F401,E402
from crosscoder_amd._lib import SIGNATURES  # noqa: E402

B, n, d = 4096, 2, 2304
K = n * d


def load(path):
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        f = getattr(lib, name, None)
        if f is not None:
            f.restype, f.argtypes = res, args
    return lib


def main():
    libs = [(os.path.basename(p), load(p)) for p in sys.argv[1:]]
    dev = torch.device("cuda:0")
    bf = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    raw = torch.randn(B, K, device=dev, generator=g).to(bf)
    factor = torch.tensor([1.3, 0.8], device=dev)
    x = torch.empty(B, K, device=dev, dtype=bf)
    x_t = torch.empty(K, B, device=dev, dtype=bf)
    L0 = libs[0][1]
    xcol = torch.empty(L0.cc_prep_part_rows(B), K, device=dev)
    recon = torch.randn(B, K, device=dev, generator=g)
    b_dec = torch.zeros(K, device=dev, dtype=bf)
    x_mean = torch.zeros(K, device=dev)
    g_recon = torch.empty(B, K, device=dev, dtype=bf)
    g_t = torch.empty(K, B, device=dev, dtype=bf)
    ncb = L0.cc_loss_col_blocks(d)
    row_part = torch.empty(2, n * ncb, B, device=dev)
    col_part = torch.empty(L0.cc_loss_part_rows(B), K, device=dev)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    nbytes = {"prep_t": B * K * 2 * 3 + xcol.numel() * 4,
              "loss_t": B * K * (4 + 2 + 2 + 2) + row_part.numel() * 4 + col_part.numel() * 4}

    def calls(L):
        return {
            "prep_t": lambda: L.cc_prep_input_t(P(raw), 1, P(factor), 2, P(x), P(x_t), P(xcol), B, n, d, 1, st),
            "loss_t": lambda: L.cc_loss_fwd_bwd_rows_t(P(recon), P(b_dec), P(x), P(x_mean), P(g_recon), P(g_t),
                                                       P(row_part), P(col_part), 2.0 / B, 0, B, B, n, d, 1, st),
        }

    res = {}
    for _ in range(3):
        for name, L in libs:
            for k, f in calls(L).items():
                assert f() == 0
    torch.cuda.synchronize()
    for _ in range(15):
        for name, L in libs:
            for k, f in calls(L).items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    f()
                e1.record()
                e1.synchronize()
                res.setdefault((k, name), []).append(e0.elapsed_time(e1) / 10 * 1e3)
    for (k, name), ts in sorted(res.items()):
        ts.sort()
        med = ts[len(ts) // 2]
        print(f"{k:8s} {name:28s} median {med:7.2f} us  min {ts[0]:7.2f} us  {nbytes[k] / med / 1e6:6.2f} TB/s")


if __name__ == "__main__":
    main()
