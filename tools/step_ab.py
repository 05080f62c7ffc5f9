"""A/B of whole-step variants on ONE device, interleaved (cdna guide rule 24): config-2 Trainer.step
with the transposed (KC/KC) weight-gradient operands on/off.  Usage: python tools/step_ab.py
(per-launch times of the same variants: python tools/step_ab.py --spans)"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import crosscoder_amd as ca  # noqa: E402
from crosscoder_amd import engine  # noqa: E402


def main():
    torch.cuda.set_device(0)
    cfg = bench.make_cfg(bench.H_LOCAL, 100)
    tr = ca.Trainer(cfg, buffer=ca.SyntheticBuffer(cfg, rows=bench.B * 8, seed=0), crosscoder=ca.CrossCoder(cfg))
    cc = tr.crosscoder
    dev = torch.device("cuda:0")
    wss = {}
    for flag in ("1", "0"):
        os.environ["CC_TRANSPOSED_WGRAD"] = flag
        wss["transposed wgrad" if flag == "1" else "batch-major wgrad"] = engine.StepWorkspace(
            bench.B, cc.n_models, cfg["d_in"], cc.d_hidden, cc.dtype, dev)
    spans = "--spans" in sys.argv
    timers = {k: bench.EventTimer() for k in wss} if spans else {}
    for t in timers.values():
        t.enabled = True
    res = {k: [] for k in wss}
    for ws in wss.values():
        cc._ws = ws
        for _ in range(3):
            tr.step()
    for _ in range(10):
        for name, ws in wss.items():
            cc._ws = ws
            tr.step()
            torch.cuda.synchronize()
            if spans:
                engine.TIMER = timers[name]
            t0 = time.perf_counter()
            for _ in range(20):
                tr.step()
            torch.cuda.synchronize()
            engine.TIMER = None
            res[name].append((time.perf_counter() - t0) / 20 * 1e3)
    for name, ts in res.items():
        ts.sort()
        print(f"{name:24s} median {ts[len(ts) // 2]:.4f} ms/step  min {ts[0]:.4f}")
        if spans:
            print("   ", {k: round(v, 4) for k, v in timers[name].averages_ms().items()})


if __name__ == "__main__":
    main()
