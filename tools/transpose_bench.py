"""cc_transpose_b16 throughput at the step's shapes (x / g_recon [4096][4608], W_dec [16384][4608]),
both block orders, next to torch's t().contiguous().  Usage: python tools/transpose_bench.py"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import crosscoder_amd  # noqa: F401,E402
from crosscoder_amd import _lib, ops  # noqa: E402
from aux_bench import timeit  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    L = _lib.load()
    L.cc_debug_set_transpose_order.argtypes = [ctypes.c_int]
    for rows, cols in ((4096, 4608), (16384, 4608), (4608, 16384)):
        src = torch.randn(rows, cols, device=dev).to(torch.bfloat16)
        dst = torch.empty(cols, rows, dtype=torch.bfloat16, device=dev)
        nbytes = 2 * src.numel() * 2
        res = []
        for order in (0, 1):
            L.cc_debug_set_transpose_order(order)
            t = timeit(lambda: ops.transpose(src, out=dst), reps=20)
            assert torch.equal(dst, src.t())
            res.append(f"order {order}: {t * 1e6:6.1f} us ({nbytes / t / 1e12:.2f} TB/s)")
        t = timeit(lambda: dst.copy_(src.t()), reps=20)
        res.append(f"torch: {t * 1e6:6.1f} us ({nbytes / t / 1e12:.2f} TB/s)")
        print(f"[{rows}][{cols}] bf16 -> transposed  " + " | ".join(res))
    L.cc_debug_set_transpose_order(-1)


if __name__ == "__main__":
    main()
