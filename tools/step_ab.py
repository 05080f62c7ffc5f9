"""A/B of whole-step variants on ONE device, interleaved (cdna guide rule 24): config-2 Trainer.step
with the early loss copy on/off.  Usage: python tools/step_ab.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import crosscoder_amd as ca  # noqa: E402


def main():
    torch.cuda.set_device(0)
    cfg = bench.make_cfg(bench.H_LOCAL, 100)
    tr = ca.Trainer(cfg, buffer=ca.SyntheticBuffer(cfg, rows=bench.B * 8, seed=0), crosscoder=ca.CrossCoder(cfg))
    variants = {"early copy": True, "copy after step": False}
    res = {k: [] for k in variants}
    for _ in range(3):
        tr.step()
    for _ in range(6):
        for name, flag in variants.items():
            tr.early_loss_copy = flag
            tr.step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(10):
                tr.step()
            torch.cuda.synchronize()
            res[name].append((time.perf_counter() - t0) / 10 * 1e3)
    for name, ts in res.items():
        ts.sort()
        print(f"{name:18s} median {ts[len(ts) // 2]:.4f} ms/step  min {ts[0]:.4f}")


if __name__ == "__main__":
    main()
