"""Host-side probe (diagnostic, one GPU): per step, how long the host takes to enqueue the step and how
long it then waits for the losses.  A wait near zero means the host, not the GPU, sets the step time.

    python tools/host_probe.py [--sharded] [--recon-chunks C] [--steps N]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.distributed as dist

import bench
import crosscoder_amd as ca


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sharded", action="store_true")
    ap.add_argument("--recon-chunks", type=int, default=None)
    ap.add_argument("--steps", type=int, default=40)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    B, n, d, h = bench.CONFIGS[2]
    cfg = bench.make_cfg(B, n, d, h)
    buf = ca.SyntheticBuffer(cfg, rows=B * 8, n_models=n, seed=0)
    if args.sharded:
        from crosscoder_amd import sharded
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        dist.init_process_group("nccl", device_id=torch.device("cuda:0"), rank=0, world_size=1)
        tr = sharded.ShardedTrainer(cfg, buffer=buf, recon_chunks=args.recon_chunks)
        inner, name = tr.engine, "step"
    else:
        tr = ca.Trainer(cfg, buffer=buf)
        inner, name = tr, "_launch_step"
    launch = getattr(inner, name)
    marks = []

    def timed(*a, **k):
        t0 = time.perf_counter()
        r = launch(*a, **k)
        marks.append((t0, time.perf_counter()))
        return r

    setattr(inner, name, timed)
    for _ in range(5):
        tr.step()
    torch.cuda.synchronize()
    marks.clear()
    ends = []
    t_start = time.perf_counter()
    for _ in range(args.steps):
        tr.step()
        ends.append(time.perf_counter())
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t_start) / args.steps
    enq = [b - a for a, b in marks]
    wait = [e - b for (a, b), e in zip(marks, ends)]
    pre = [a - e for (a, _), e in zip(marks[1:], ends[:-1])]
    med = lambda v: sorted(v)[len(v) // 2] * 1e6
    print(f"{'sharded' if args.sharded else 'single'} chunks={args.recon_chunks}: step {wall * 1e3:.3f} ms | "
          f"host enqueue {med(enq):.0f} us, wait for losses {med(wait):.0f} us, between steps {med(pre):.0f} us")
    if args.sharded:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
