"""Diagnostic: per-wave cycle split {prologue, DMA wait, barrier, compute} of the GEMM K loop from a
CC_STAMPS build (s_memtime stamps; stamps perturb timing, read the SHARES)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import crosscoder_amd  # noqa: F401,E402
from crosscoder_amd._lib import SIGNATURES  # noqa: E402

B, n, d, h = 4096, 2, 2304, 16384
K = n * d


def main():
    for path in sys.argv[1:]:
        L = ctypes.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        dev = torch.device("cuda:0")
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(B, K, device=dev, generator=g).to(torch.bfloat16)
        W = (torch.randn(h, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        acts = torch.randn(B, h, device=dev, generator=g).to(torch.bfloat16)
        C1 = torch.empty(B, h, device=dev)
        C2 = torch.empty(h, K, device=dev)
        buf = torch.zeros(2048 * 8 * 6, dtype=torch.int64, device=dev)
        L.cc_debug_set_stamp_buffer(ctypes.c_void_p(buf.data_ptr()))
        P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        cases = {
            "G1-like KC/KC 4096x16384x4608": lambda: L.cc_gemm_f32out(P(x), 0, K, P(W), 0, K, P(C1), h, B, h, K, 1, st),
            "G5-like MN/MN 16384x4608x4096": lambda: L.cc_gemm_f32out(P(acts), 1, h, P(x), 1, K, P(C2), K, h, K, B, 1, st),
        }
        for name, fn in cases.items():
            for _ in range(3):
                buf.zero_()
                assert fn() == 0
                torch.cuda.synchronize()
            v = buf.view(-1, 6).double()
            v = v[v[:, 4] > 0]
            tot = v[:, 4].mean()
            print(f"{os.path.basename(path)} {name}: blocks*waves={v.shape[0]} nk={int(v[0,5])} "
                  f"loop cycles/wave={tot:.0f} cycles/step={tot / v[0,5]:.0f}  shares: "
                  f"prologue {v[:,0].mean()/tot:.3f} dma-wait {v[:,1].mean()/tot:.3f} "
                  f"barrier {v[:,2].mean()/tot:.3f} compute {v[:,3].mean()/tot:.3f}")


if __name__ == "__main__":
    main()
