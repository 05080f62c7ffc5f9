"""Probe: one Trainer.step_async() captured into a HIP graph (torch.cuda.graph, both streams) and
replayed, against eager steps -- the launch / inter-kernel overhead a graph would remove.  Timing only:
the replay repeats the captured step's arguments (same batch, lr, Adam step).  Usage:
python tools/graph_probe.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import crosscoder_amd as ca
    import bench

    torch.cuda.set_device(0)
    B, n, d, h = bench.CONFIGS[2]
    cfg = bench.make_cfg(B, n, d, h)
    tr = ca.Trainer(cfg, buffer=ca.SyntheticBuffer(cfg, rows=B * 8, seed=0), crosscoder=ca.CrossCoder(cfg))
    for _ in range(5):
        tr.step()
    tr.synchronize()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        tr.step_async()  # warm the side-stream / workspace state on the capture stream
        tr.synchronize()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            tr.step_async()
            tr.synchronize()  # join the side stream into the capture
    torch.cuda.synchronize()
    res = {"eager": [], "graph": []}
    for _ in range(6):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            tr.step_async()
        tr.synchronize()
        torch.cuda.synchronize()
        res["eager"].append((time.perf_counter() - t0) / 20 * 1e3)
        t0 = time.perf_counter()
        for _ in range(20):
            g.replay()
        torch.cuda.synchronize()
        res["graph"].append((time.perf_counter() - t0) / 20 * 1e3)
    for k, v in res.items():
        v.sort()
        print(f"{k:6s} median {v[len(v) // 2]:.4f} ms/step  min {v[0]:.4f}", flush=True)


if __name__ == "__main__":
    main()
