"""Host-side cost of one Trainer step: time spent in step_async() (enqueue only), in the wait for the
loss copy, and in the rest of step(), against the GPU step time (config 2).  Tells whether the host
keeps ahead of the GPU.  Usage: python tools/host_enqueue.py"""
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
    torch.cuda.synchronize()
    enq, wait, tot = [], [], []
    t_start = time.perf_counter()
    N = 40
    for _ in range(N):
        t0 = time.perf_counter()
        tr.step_async(on_losses=tr._copy_losses)
        t1 = time.perf_counter()
        tr._copied.synchronize()
        t2 = time.perf_counter()
        tr._host[:6].tolist()
        tr.step_counter += 1
        t3 = time.perf_counter()
        enq.append((t1 - t0) * 1e3)
        wait.append((t2 - t1) * 1e3)
        tot.append((t3 - t0) * 1e3)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t_start) / N * 1e3
    med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
    print(f"per step: wall {el:.3f} ms; step_async enqueue median {med(enq):.3f} ms (max {max(enq):.3f}); "
          f"wait for the loss copy {med(wait):.3f} ms; host total {med(tot):.3f} ms", flush=True)


if __name__ == "__main__":
    main()
