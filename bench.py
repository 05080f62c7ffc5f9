"""Benchmark: activations/sec of the full crosscoder training step (fwd + bwd + clip + Adam).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]

N = 1: BASELINE config 2 — CrossCoder 2x2304->16384, batch 4096, bf16 on one MI355X
(synthetic normalised activations, reference init with seed 49), timed through
Trainer.step() (the reference's step contract, incl. its per-step loss-dict host copy).
N > 1 (torchrun, one rank per GPU): the dictionary is latent-sharded — every rank owns a
16384-latent slice (so the whole job trains 2x2304 -> 16384*N, BASELINE config 3 at N = 8)
on the same 4096-row batch, with an RCCL all-reduce of the fp32 partial reconstructions.
Per-GPU work is fixed (weak scaling); `value` counts config-2-equivalent activations
(batch x h_total / 16384) per second over the whole job.

The JSON line also carries `roofline` (dominant kernel's achieved TFLOP/s from HIP events
around every launch of it in the timed region, vs the bf16 dense MFMA peak) and
`cpu_baseline` (the oracle CPU step timed on this host, rank 0, N = 1 only).
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import crosscoder_amd as ca  # noqa: E402
from crosscoder_amd import engine  # noqa: E402

B, N_MODELS, D_MODEL, H_LOCAL = 4096, 2, 2304, 16384
PEAK_BF16_TFLOPS = 256 * 2.4e9 * 4096 / 1e12  # 256 CU x 2.4 GHz x 4096 bf16 FLOP/clk/CU (dense)


class EventTimer:
    """HIP events on torch's current stream (the stream every launch uses) around named spans.

    `only` restricts recording to one span name: inside the timed region only the roofline kernel
    is bracketed (each timing event costs the stream a few microseconds); the per-kernel breakdown
    comes from an attribution pass of its own."""

    def __init__(self):
        self.rec = {}
        self.enabled = False
        self.only = None

    class _Span:
        def __init__(self, t, name):
            self.t, self.name = t, name
            self.on = t.enabled and (t.only is None or t.only == name)

        def __enter__(self):
            if self.on:
                self.s = torch.cuda.Event(enable_timing=True)
                self.s.record()

        def __exit__(self, *a):
            if self.on:
                e = torch.cuda.Event(enable_timing=True)
                e.record()
                self.t.rec.setdefault(self.name, []).append((self.s, e))

    def span(self, name):
        return EventTimer._Span(self, name)

    def averages_ms(self):
        return {k: sum(s.elapsed_time(e) for s, e in v) / len(v) for k, v in self.rec.items()}


SPAN_EVERY = 4  # timed steps per roofline-kernel sample (events around the launch)

# span name -> kernel-name prefix in the rocprofv3 traces
SPAN_KERNEL = {"G1_encode": "gemm_pp_kernel<true, true, 1>", "G2_decode": "gemm_pp_kernel<true, false, 2>",
               "G3_dacts": "gemm_pp_kernel<true, true, 3>", "G4G5_wgrad": "gemm_pp_dual_kernel<false, false, 4, 5>",
               "adam": "adam_bulk_kernel"}


def pmc_traffic(span):
    """HBM bytes per launch of the span's kernel from the newest committed PMC summary
    (profiles/*_pmc_traffic.json, written by tools/pmc_traffic.py from separate FETCH_SIZE /
    WRITE_SIZE passes of this bench), or None."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json")))
    if not files or span not in SPAN_KERNEL:
        return None, None
    with open(files[-1]) as f:
        doc = json.load(f)
    for name, v in doc["kernels"].items():
        if name.startswith(SPAN_KERNEL[span]):
            return v["hbm_bytes"], os.path.relpath(files[-1], ROOT)
    return None, None


def make_cfg(h, steps_total):
    return {
        "seed": 49, "batch_size": B, "buffer_mult": 128, "lr": 5e-5, "num_tokens": 400_000_000, "l1_coeff": 2,
        "beta1": 0.9, "beta2": 0.999, "dict_size": h, "seq_len": 1024, "enc_dtype": "bf16", "model_name": "synthetic",
        "device": f"cuda:{torch.cuda.current_device()}", "model_batch_size": 4, "log_every": 100,
        "save_every": 30000, "dec_init_norm": 0.08, "d_in": D_MODEL,
    }


def cpu_baseline(seconds_budget=20.0):
    """Oracle (reference PyTorch fp32 step restated, CPU) on a bounded sample of config 1."""
    from oracle import cpu_reference as O

    # this process's CPU share: OMP_NUM_THREADS (16 per GPU on the box), else the affinity mask
    cores = int(os.environ.get("OMP_NUM_THREADS") or 0) or len(os.sched_getaffinity(0))
    torch.set_num_threads(cores)
    cfg = {"seed": 49, "dict_size": H_LOCAL, "d_in": D_MODEL, "enc_dtype": "fp32", "dec_init_norm": 0.08,
           "batch_size": B, "num_tokens": 400_000_000, "lr": 5e-5, "beta1": 0.9, "beta2": 0.999, "l1_coeff": 2}
    P = O.init_params(cfg)
    tr = O.OracleTrainer(cfg, P)
    g = torch.Generator().manual_seed(0)
    x = torch.randn(B, N_MODELS, D_MODEL, generator=g)
    tr.step(x)  # warm-up
    times = []
    t_start = time.perf_counter()
    while len(times) < 5 and (time.perf_counter() - t_start) < seconds_budget:
        t0 = time.perf_counter()
        tr.step(x)
        times.append(time.perf_counter() - t0)
    times.sort()
    med = times[len(times) // 2]
    return {"value": B / med, "unit": "activations/s", "cores": cores, "kind": "port",
            "sample": f"oracle fp32 Trainer.step, config 1 (B={B}, 2x{D_MODEL}->{H_LOCAL}), "
                      f"median of {len(times)} steps after 1 warm-up, {med:.2f} s/step"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--force-sharded", action="store_true",
                    help="diagnostic: run the latent-sharded step even on one rank (1-rank RCCL group)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    sharded_path = world > 1 or args.force_sharded
    if sharded_path:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"), rank=rank, world_size=world)
    h_total = H_LOCAL * world
    cfg = make_cfg(h_total, args.warmup + args.steps)

    if not sharded_path:
        cc = ca.CrossCoder(cfg)
        buf = ca.SyntheticBuffer(cfg, rows=B * 8, seed=0)
        tr = ca.Trainer(cfg, buffer=buf, crosscoder=cc)
    else:
        from crosscoder_amd import sharded

        buf = ca.SyntheticBuffer(cfg, rows=B * 8, seed=0)  # same seed on every rank: replicated batch
        tr = sharded.ShardedTrainer(cfg, buffer=buf)

    timer = EventTimer()
    engine.TIMER = timer
    for _ in range(args.warmup):
        tr.step()
    # attribution pass (not timed): every kernel bracketed by events
    attrib = EventTimer()
    engine.TIMER = attrib
    attrib.enabled = True
    for _ in range(max(3, min(args.steps, 10))):
        tr.step()
    torch.cuda.synchronize()
    kern = attrib.averages_ms()
    gemms = {k: v for k, v in kern.items() if k.startswith("G")}
    dom = max(gemms, key=gemms.get)
    engine.TIMER = timer
    timer.only = dom  # the roofline kernel, measured live inside the timed region
    if sharded_path:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        # the roofline launch is bracketed on every SPAN_EVERY-th timed step (each event record
        # idles the stream ~6 us, tools/event_cost.py: sampling keeps that out of most steps)
        timer.enabled = i % SPAN_EVERY == 0
        last = tr.step()
    torch.cuda.synchronize()
    if sharded_path:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    timer.enabled = False
    if sharded_path:
        t = torch.tensor([elapsed], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()

    ms = elapsed / args.steps * 1e3
    acts_equiv = B * (h_total / H_LOCAL)
    value = acts_equiv / (elapsed / args.steps)
    dom_ms = timer.averages_ms()[dom]
    gemm_flop = 2.0 * B * N_MODELS * D_MODEL * H_LOCAL  # per GEMM (per rank)
    # G4G5_wgrad is one launch computing both weight gradients (cc_wgrad_both)
    dom_flop = gemm_flop * (2 if dom == "G4G5_wgrad" else 1)
    achieved = dom_flop / (dom_ms * 1e-3) / 1e12
    step_flop = 5 * gemm_flop
    if engine.transposed_wgrad(B, N_MODELS * D_MODEL, H_LOCAL, torch.bfloat16):  # KC/KC form (cc_wgrad_both_t)
        SPAN_KERNEL["G4G5_wgrad"] = "gemm_pp_dual_kernel<true, true, 4, 5>"
    traffic, traffic_src = pmc_traffic(dom)
    # algorithmic operand/output bytes of the dominant launch (each input read once, output written once)
    es = 2  # bf16
    K_ = N_MODELS * D_MODEL
    alg = {"G1_encode": (B * K_ + H_LOCAL * K_ + B * H_LOCAL) * es,
           "G2_decode": (B * H_LOCAL + H_LOCAL * K_) * es + B * K_ * 4,
           "G3_dacts": (B * K_ + H_LOCAL * K_ + 2 * B * H_LOCAL) * es,
           "G4G5_wgrad": (2 * B * H_LOCAL + 2 * B * K_ + 3 * H_LOCAL * K_) * es}
    dom_alg_bytes = alg.get(dom)
    result = {
        "metric": "activations/sec per train step (fwd+bwd+Adam), 2x2304->16384; % bf16 MFMA peak",
        "value": round(value, 1),
        "unit": "activations/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic (seeded N(0,1) activations scaled per model, reference init seed 49)",
        "config": {"workload": f"crosscoder train step 2x{D_MODEL}->{h_total}, batch {B}, latent-sharded over "
                               f"{world} GPU(s) ({H_LOCAL} latents per GPU)",
                   "global_batch": B, "n_models": N_MODELS, "d_model": D_MODEL, "dict_size": h_total,
                   "parallelism": f"latent{world}"},
        "step_mfma_frac": round(step_flop / (ms * 1e-3) / 1e12 / PEAK_BF16_TFLOPS, 4),
        "kernels_ms": {k: round(v, 4) for k, v in sorted(kern.items())},
        "roofline": {"bound": "mfma", "kernel": dom, "kernel_ms": round(dom_ms, 4),
                     "kernel_samples": len(timer.rec.get(dom, [])), "achieved": round(achieved, 1),
                     "peak": round(PEAK_BF16_TFLOPS, 1), "unit": "TFLOP/s", "frac": round(achieved / PEAK_BF16_TFLOPS, 4),
                     "traffic": traffic, "traffic_unit": "HBM bytes per launch (PMC)", "traffic_source": traffic_src,
                     "algorithmic_bytes": dom_alg_bytes},
        "last_loss": {k: round(v, 6) for k, v in last.items()},
    }
    if rank == 0:
        if world == 1 and not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline()
        print(json.dumps(result), flush=True)
    if sharded_path:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
