"""Per-CU rate of the epilogue's store pattern (tools/exp/store_rate.hip): one 512-thread workgroup per
CU writing 128-KB tiles (16 x 1-KB wave-instructions per wave), 1 / 32 / 256 workgroups.
Usage: python tools/store_rate.py"""
import ctypes
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "exp", "libstore_rate.so"))
    lib.store_run.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda:0")
    ld = 16 * 512  # 16 tiles of 512 B side by side per row band (8 KB rows, like a bf16 [.][4096] matrix)
    tiles_per_wg = 8
    buf = torch.empty(256 * tiles_per_wg // 16 * 256 * ld + (1 << 20), dtype=torch.uint8, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for blocks in (1, 8, 32, 128, 256):
        for _ in range(3):
            lib.store_run(ctypes.c_void_p(buf.data_ptr()), ld, blocks, 16, tiles_per_wg, st)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ts = []
        for _ in range(10):
            e0.record()
            lib.store_run(ctypes.c_void_p(buf.data_ptr()), ld, blocks, 16, tiles_per_wg, st)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        ts.sort()
        us = ts[len(ts) // 2]
        per_wg = tiles_per_wg * 128 * 1024
        print(f"{blocks:4d} workgroups: {us:8.1f} us  per tile {us / tiles_per_wg:6.2f} us  per CU {per_wg / us / 1e3:6.1f} GB/s  "
              f"chip {blocks * per_wg / us / 1e6:6.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
