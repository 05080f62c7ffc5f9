"""Sustained bf16 MFMA throughput, 16x16x32 vs 32x32x16, register-resident operands, every CU busy for
~3 s per case (the package power cap sets the clock): tools/exp/mfma_power.hip -> libmfma_power.so.
Also zero operands (less toggling -> less power -> higher clock).  Usage: python tools/mfma_power.py"""
import ctypes
import os
import re
import subprocess
import threading
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PEAK = 256 * 2.4e9 * 4096 / 1e12


def sample(stop, out):
    while not stop.is_set():
        try:
            s = subprocess.run(["rocm-smi", "--showpower", "--showclocks"], capture_output=True, text=True,
                               timeout=5).stdout
            p = re.search(r"Package Power \(W\): ([\d.]+)", s)
            c = re.search(r"sclk clock level: \d+: \((\d+)Mhz\)", s)
            if p and c:
                out.append((float(p.group(1)), float(c.group(1))))
        except Exception:  # noqa: BLE001
            pass
        time.sleep(0.25)


def main():
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "exp", "libmfma_power.so"))
    lib.mfma_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda:0")
    blocks, iters = 256 * 4, 20000
    out = torch.empty(blocks * 512, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    # flops per launch: per wave per trip 8 x (16*16*32*2) = 2 x 2 x (32*32*16*2) = 131072
    flop = blocks * 8 * iters * 131072.0
    for kind, zero in ((16, 0), (32, 0), (16, 1), (32, 1), (16, 0), (32, 0)):
        assert lib.mfma_run(kind, ctypes.c_void_p(out.data_ptr()), blocks, 100, zero, st) == 0
        torch.cuda.synchronize()
        stop, smp = threading.Event(), []
        th = threading.Thread(target=sample, args=(stop, smp))
        th.start()
        n, t0 = 0, time.perf_counter()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        times = []
        while time.perf_counter() - t0 < 3.0:
            e0.record()
            lib.mfma_run(kind, ctypes.c_void_p(out.data_ptr()), blocks, iters, zero, st)
            e1.record()
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1))
            n += 1
        stop.set()
        th.join()
        ms = sorted(times[1:] or times)[len(times[1:] or times) // 2]
        pw = [p for p, _ in smp[1:]] or [0]
        ck = [c for _, c in smp[1:]] or [0]
        tf = flop / (ms * 1e-3) / 1e12
        print(f"mfma {kind}x{kind} zero={zero}: {ms:7.2f} ms/launch  {tf:7.1f} TF/s ({tf / PEAK * 100:5.1f}% of 2.4 GHz peak)"
              f"  power mean {sum(pw) / len(pw):6.0f} W  sclk mean {sum(ck) / len(ck):5.0f} MHz  launches {n}",
              flush=True)


if __name__ == "__main__":
    main()
