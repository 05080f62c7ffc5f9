"""Whole-step timing of the shipped schedule, config 2, for in-process or same-box A/B of library
builds: python tools/step_ab.py [--lib path/to/variant.so] [--spans] [--rounds R]
(--lib: load this build instead of the in-tree library -- tools only; --spans: per-launch HIP-event
averages as well).  Earlier scheduling variants and their measurements: DESIGN.md section 8."""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib")
    ap.add_argument("--spans", action="store_true")
    ap.add_argument("--rounds", type=int, default=10)
    args = ap.parse_args()
    import crosscoder_amd as ca

    if args.lib:
        ca._lib.load(args.lib)  # first load wins: every later call uses this build
    import bench
    from crosscoder_amd import engine

    torch.cuda.set_device(0)
    B, n, d, h = bench.CONFIGS[2]
    cfg = bench.make_cfg(B, n, d, h)
    tr = ca.Trainer(cfg, buffer=ca.SyntheticBuffer(cfg, rows=B * 8, seed=0), crosscoder=ca.CrossCoder(cfg))
    timer = bench.EventTimer() if args.spans else None
    for _ in range(5):
        tr.step()
    res = []
    for _ in range(args.rounds):
        torch.cuda.synchronize()
        if timer is not None:
            timer.enabled = True
            engine.TIMER = timer
        t0 = time.perf_counter()
        for _ in range(20):
            tr.step()
        torch.cuda.synchronize()
        engine.TIMER = None
        res.append((time.perf_counter() - t0) / 20 * 1e3)
    res.sort()
    print(f"{args.lib or 'in-tree'}: median {res[len(res) // 2]:.4f} ms/step  min {res[0]:.4f}")
    if timer is not None:
        print("   ", {k: round(v, 4) for k, v in timer.averages_ms().items()})


if __name__ == "__main__":
    main()
