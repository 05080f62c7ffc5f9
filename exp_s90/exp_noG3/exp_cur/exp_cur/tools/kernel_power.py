"""Power and clock of each step kernel run alone, back to back for ~3 s, sampled with rocm-smi in a
background thread: tells which kernels hold the chip at its package power cap (then the clock drops
and energy per kernel, not cycles, sets its time).  Config-2 shapes, random operands.
Usage: python tools/kernel_power.py [name-substring ...]"""
import ctypes
import os
import re
import subprocess
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import crosscoder_amd  # noqa: F401,E402
from crosscoder_amd import ops  # noqa: E402

B, n, d, h = 4096, 2, 2304, 16384
K = n * d


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
    dev = torch.device("cuda:0")
    bf = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    r = lambda *s, sc=1.0: (torch.randn(*s, device=dev, generator=g) * sc).to(bf)  # noqa: E731
    x, W, W2 = r(B, K), r(h, K, sc=0.02), r(h, K, sc=0.02)
    b_enc = torch.zeros(h, device=dev, dtype=bf)
    acts, acts_t = torch.relu(r(B, h)), torch.empty(h, B, device=dev, dtype=bf)
    recon = torch.empty(B, K, device=dev)
    g_recon = r(B, K, sc=1e-3)
    g_pre_t = torch.empty(h, B, device=dev, dtype=bf)
    tn = torch.ones(h, device=dev)
    norms = torch.ones(h, n, device=dev)
    colsum = torch.ones(h, device=dev)
    gW, gW2 = torch.empty(h, K, device=dev, dtype=bf), torch.empty(h, K, device=dev, dtype=bf)
    parts = torch.empty(1 << 20, device=dev)
    parts2 = torch.empty(1 << 20, device=dev)
    W2T = W2.t().contiguous()
    actsT, grT, gpT, xT = acts.t().contiguous(), g_recon.t().contiguous(), r(h, B, sc=1e-3), x.t().contiguous()
    nws = ops.decode_ws_floats(B, h, K, bf)
    dws = torch.empty(max(nws, 1), device=dev)
    P = [r(75_000_000, sc=0.02) for _ in range(4)]
    coef = torch.ones(1, device=dev)
    cases = {
        "G1 encode (+acts^T)": lambda: ops.encode_fwd_t(x, W, b_enc, acts, acts_t, True, colsum_part=parts, l0_part=parts2),
        "G2 decode": lambda: ops.decode_partial_t(acts, W2T, recon, dws),
        "G3 d_acts": lambda: ops.dacts_bwd_t(g_recon, W2, acts, tn, 1e-4, g_pre_t, colsum_part=parts),
        "G4+G5 wgrad": lambda: ops.wgrad_both_t(actsT, grT, W2, norms, colsum, 1e-4, gW, parts, gpT, xT, gW2, parts2, n, d),
        "adam (75M params)": lambda: ops.adam_step(P[0], P[1], P[2], P[3], coef, 5e-5, 0.9, 0.999, 1e-8, 3),
        "hipBLASLt G1 shape (plain)": lambda: torch.matmul(x, W.t(), out=acts),
        "ours G1 plain (bias+relu)": lambda: ops.encode_fwd(x, W, b_enc, acts, True),
        "idle": None,
    }
    only = sys.argv[1:]
    for name, fn in cases.items():
        if only and not any(o in name for o in only):
            continue
        torch.cuda.synchronize()
        stop, out = threading.Event(), []
        th = threading.Thread(target=sample, args=(stop, out))
        n_launch = 0
        t0 = time.perf_counter()
        if fn is None:
            th.start()
            time.sleep(2.0)
        else:
            for _ in range(20):
                fn()
            torch.cuda.synchronize()
            th.start()
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < 3.0:
                for _ in range(10):
                    fn()
                n_launch += 10
                torch.cuda.synchronize()
        el = time.perf_counter() - t0
        stop.set()
        th.join()
        pw = [p for p, _ in out[1:]] or [0]
        ck = [c for _, c in out[1:]] or [0]
        us = el / n_launch * 1e6 if n_launch else 0
        print(f"{name:22s} {us:8.1f} us/launch  power {min(pw):6.0f}-{max(pw):6.0f} W (mean {sum(pw)/len(pw):6.0f})  "
              f"sclk {min(ck):5.0f}-{max(ck):5.0f} MHz (mean {sum(ck)/len(ck):5.0f})  samples {len(out)}", flush=True)


if __name__ == "__main__":
    main()
