"""Bit-identity of two library builds on the step GEMMs' outputs incl. the epilogue partial slabs
(column sums, l1 / l0 / squared-gradient partials).  Usage: python tools/epi_bits.py a.so b.so"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import crosscoder_amd  # noqa: F401,E402
from crosscoder_amd._lib import SIGNATURES  # noqa: E402

B, n, d, h = 4096, 2, 2304, 16384
K = n * d


def load(path):
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        f = getattr(lib, name, None)
        if f is not None:
            f.restype, f.argtypes = res, args
    return lib


def main():
    libs = [load(p) for p in sys.argv[1:3]]
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    bf = torch.bfloat16
    x = torch.randn(B, K, device=dev, generator=g).to(bf)
    W = (torch.randn(h, K, device=dev, generator=g) * 0.02).to(bf)
    b_enc = (torch.randn(h, device=dev, generator=g) * 0.1).to(bf)
    tn = torch.rand(h, device=dev, generator=g)
    g_recon = (torch.randn(B, K, device=dev, generator=g) * 1e-3).to(bf)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    outs = []
    for L in libs:
        acts = torch.empty(B, h, device=dev, dtype=bf)
        actsT = torch.empty(h, B, device=dev, dtype=bf)
        colp = torch.zeros(1 << 20, device=dev)
        l1p = torch.zeros(1 << 16, device=dev)
        l0p = torch.zeros(1 << 16, device=dev)
        mbits = torch.zeros(B * h // 32 + 4096, device=dev, dtype=torch.int32)
        assert L.cc_encode_fwd_t(P(x), P(W), P(b_enc), P(tn), P(acts), P(actsT), 1, P(colp), P(l1p), P(l0p), P(mbits),
                                 B, K, h, 1, st) == 0
        gpT = torch.empty(h, B, device=dev, dtype=bf)
        colp3 = torch.zeros(1 << 20, device=dev)
        assert L.cc_dacts_bwd_t(P(g_recon), P(W), P(acts), P(tn), 1e-4, P(mbits), P(gpT), B, P(colp3), B, K, h, 1,
                                st) == 0
        norms = torch.rand(h, n, device=dev, generator=torch.Generator(device=dev).manual_seed(1)) + 0.5
        colsum = torch.rand(h, device=dev, generator=torch.Generator(device=dev).manual_seed(2))
        gW, gW2 = torch.empty(h, K, device=dev, dtype=bf), torch.empty(h, K, device=dev, dtype=bf)
        sq1, sq2 = torch.zeros(1 << 20, device=dev), torch.zeros(1 << 20, device=dev)
        grT, xT = g_recon.t().contiguous(), x.t().contiguous()
        assert L.cc_wgrad_both_t(P(actsT), P(grT), P(W), P(norms), P(colsum), 1e-4, P(gW), P(sq1), P(gpT), P(xT),
                                 P(gW2), P(sq2), B, h, n, d, 1, st) == 0
        torch.cuda.synchronize()
        outs.append((acts, actsT, colp, l1p, l0p, gpT, colp3, gW, sq1, gW2, sq2))
    names = ["acts", "acts^T", "G1 colsum partials", "l1 partials", "l0 partials", "g_pre^T", "G3 colsum partials",
             "dW_dec", "dW_dec sq partials", "dW_enc", "dW_enc sq partials"]
    for nm, a, b in zip(names, outs[0], outs[1]):
        same = torch.equal(a.view(torch.int16) if a.dtype == bf else a.view(torch.int32),
                           b.view(torch.int16) if b.dtype == bf else b.view(torch.int32))
        print(f"{nm:22s} bit-identical: {same}", flush=True)
        assert same, nm


if __name__ == "__main__":
    main()
