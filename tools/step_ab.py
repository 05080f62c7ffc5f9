"""A/B of whole-step variants on ONE device, interleaved (cdna guide rule 24): config-2 Trainer.step
with the early loss copy and the side-stream decoder-half Adam on/off.  Usage: python tools/step_ab.py"""
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
    from crosscoder_amd import engine
    variants = {"early copy": (True, False, 0), "side Adam, 192 blocks": (True, True, 192),
                "side Adam, 256 blocks": (True, True, 256), "side Adam, 384 blocks": (True, True, 384)}
    res = {k: [] for k in variants}
    for _ in range(3):
        tr.step()
    for _ in range(12):
        for name, (flag, side, nb) in variants.items():
            tr.early_loss_copy = flag
            tr.overlap_decoder_adam = side
            engine.DEC_ADAM_BLOCKS = nb
            tr.step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(20):
                tr.step()
            torch.cuda.synchronize()
            res[name].append((time.perf_counter() - t0) / 20 * 1e3)
    for name, ts in res.items():
        ts.sort()
        print(f"{name:24s} median {ts[len(ts) // 2]:.4f} ms/step  min {ts[0]:.4f}")


if __name__ == "__main__":
    main()
