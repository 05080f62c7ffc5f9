"""Benchmark: activations/sec of the full crosscoder training step (fwd + bwd + clip + Adam).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config C] [--batch B] [--n-models n]
                  [--d-model d] [--dict-size h] [--no-cpu-baseline]

Workloads are BASELINE.json's configs (synthetic normalised activations, reference init seed 49, bf16):
  config 2  CrossCoder 2x2304->16384, batch 4096          -- the default at N = 1 (the metric's config)
  config 3  2x2304->131072 (2^17), batch 4096, latent-sharded over the N ranks -- the default at N > 1
  config 4  2x3584->65536, batch 8192                       config 5  4x2304->32768, batch 4096
(--batch / --n-models / --d-model / --dict-size override single fields).  N > 1 (torchrun, one rank per
GPU): the FIXED dictionary of the config is split into N latent slices (strong scaling) with an RCCL
all-reduce of the fp32 partial reconstructions; every rank processes the same batch.

`value` is the activations (batch rows, each seen by all n models) the whole job trains per second -- the
metric's own unit, on whatever workload runs.  At N = 1 that is config 2, the metric's config.  N > 1 runs
config 3 (2^17 latents, as BASELINE.json's north_star asks), whose rows cost 8x a config-2 row, so its
`value` is not comparable with the N = 1 line: the strong-scaling point of comparison is `n1_same_workload`
(config 3 on one GPU, measured in the same job on rank 0 before the sharded run), and `metric_equiv_acts_per_s` = value x n.d.h / (2.2304.16384)
restates the throughput in config-2 rows of equal FLOP (10.n.d.h FLOP of step work per row).
`latent_acts_per_s` = value x dict_size.

The JSON line also carries `roofline` (dominant kernel's achieved TFLOP/s from HIP events around its
launches inside the timed region, vs the bf16 dense MFMA peak), `hbm` (achieved GB/s of the
streaming kernels: Adam halves, input prep -- and the loss kernel where G2 does not carry the loss in its
epilogue -- from an untimed attribution pass) and `cpu_baseline` (the oracle CPU step timed on this host,
rank 0, N = 1 only).
"""
import argparse
import datetime
import json
import os
import signal
import socket
import subprocess
import sys
import threading
import time

# one HIP hardware queue per stream (HIP's default is 4 per process): the latent-sharded step uses the
# compute stream, the side stream and RCCL's streams, and on a shared queue the side stream's decoder-half
# Adam serialises behind the compute stream instead of running beside G1 (+0.2 ms per step, DESIGN.md
# section 6; neutral for the single-GPU step).  Must be set before the process touches the GPU.
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# (crosscoder_amd -- the HIP library -- is imported by the rank processes only: the launcher parent of an
# N > 1 run touches no GPU, see launch_ranks)
ca = engine = None

CONFIGS = {2: (4096, 2, 2304, 16384), 3: (4096, 2, 2304, 131072), 4: (8192, 2, 3584, 65536),
           5: (4096, 4, 2304, 32768)}  # (batch, n_models, d_model, dict_size)
PEAK_BF16_TFLOPS = 256 * 2.4e9 * 4096 / 1e12  # 256 CU x 2.4 GHz x 4096 bf16 FLOP/clk/CU (dense)
PEAK_HBM_GBS = 8000.0  # HBM3E spec (MI355X_MICROARCH.md; ~6300 measured for a float4 copy)


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
SPAN_KERNEL = {"G1_encode": "gemm_pp_kernel<true, true, 1", "G2_decode": "gemm_pp_main_splitk_kernel<true, false, 7",
               "G3_dacts": "gemm_q4_kernel<3, true>", "G4G5_wgrad": "gemm_pp_dual_tail_kernel<true, true, 4, 5>",
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


def rocprof_average(span):
    """The dominant kernel's average duration in the newest committed rocprofv3 --stats summary of this bench
    (profiles/*_step_kernel_stats.csv) -- the figure the live event samples are checked against -- or None."""
    import csv
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_step_kernel_stats.csv")))
    if not files or span not in SPAN_KERNEL:
        return None
    with open(files[-1]) as f:
        for row in csv.DictReader(f):
            name = row["Name"].replace("void ", "").replace("cc::", "")
            if name.startswith(SPAN_KERNEL[span]):
                return {"avg_ms": round(float(row["AverageNs"]) * 1e-6, 4), "calls": int(row["Calls"]),
                        "min_ms": round(float(row["MinNs"]) * 1e-6, 4), "source": os.path.relpath(files[-1], ROOT)}
    return None


def n1_same_workload(cfg, steps=10, warmup=3):
    """The 1-GPU point of the N > 1 strong-scaling curve, measured INSIDE this job: rank 0 runs the same workload
    (the whole dictionary) as a single-GPU Trainer on its own GPU before the sharded trainer is built, `warmup`
    untimed then `steps` timed steps (barrier-free: one process), and frees it again.  Same synthetic buffer and
    init as the sharded run."""
    B = cfg["batch_size"]
    cc = ca.CrossCoder(cfg)
    buf = ca.SyntheticBuffer(cfg, rows=B * 8, n_models=cfg["n_models"], seed=0)
    tr = ca.Trainer(cfg, buffer=buf, crosscoder=cc)
    for _ in range(warmup):
        tr.step()
    tr.synchronize()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        tr.step()
    tr.synchronize()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    words = clock_words(tr)
    clk = effective_clock(words)
    del tr, cc, buf
    torch.cuda.empty_cache()
    return {"value": round(B / dt, 1), "ms_per_step": round(dt * 1e3, 4), "steps": steps, "warmup": warmup,
            "effective_sclk_ghz": clk["effective_sclk_ghz"] if clk else None,
            "source": "measured in this job: rank 0, one GPU, single-GPU Trainer on the whole dictionary, before "
                      "the sharded run"}


def _sync(dev):
    if torch.device(dev).type == "cuda":
        torch.cuda.synchronize()


def timed_steps(tr, steps, dev="cuda"):
    """Wall time per step of `steps` steps between barrier + synchronize on both sides, max over ranks."""
    dist.barrier()
    _sync(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        tr.step()
    _sync(dev)
    dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.item() / steps


def allreduce_algbw(rows, K, iters=10, dev="cuda"):
    """Achieved bandwidth of one exchange slice's all-reduce alone (fp32 [rows, K], synchronous), the collective the
    sharded step issues: algbw = bytes / time (max over ranks), busbw = algbw x 2 (G - 1) / G (ring traffic)."""
    x = torch.ones(rows, K, device=dev)
    for _ in range(2):
        dist.all_reduce(x)
    _sync(dev)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        dist.all_reduce(x)
    _sync(dev)
    t = torch.tensor([(time.perf_counter() - t0) / iters], device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ms = t.item() * 1e3
    G = dist.get_world_size()
    algbw = x.numel() * 4 / (ms * 1e-3) / 1e9
    del x
    return {"bytes": rows * K * 4, "ms": round(ms, 4), "algbw_GB_s": round(algbw, 1),
            "busbw_GB_s": round(algbw * 2 * (G - 1) / G, 1)}


def measure_exchange(tr, comm, K, dev="cuda", steps=5, slices=None):
    """The latent-sharded step's exchange, measured in warm-up (not the timed region): each candidate form runs one
    settling step and `steps` timed steps (max over ranks); the fastest is left set on the trainer; plus the
    bandwidth one slice's all-reduce reaches alone.  "auto": the all-reduce in 1, 2 and 4 batch slices (unless
    `slices` fixes the count) and the reduce-scatter.  Every rank picks the same form (the times are all-reduced)."""
    cands = []
    for c in (("all_reduce", "reduce_scatter") if comm == "auto" else (comm,)):
        if c == "all_reduce" and comm == "auto" and slices is None:
            cands += [(f"all_reduce x{s}", c, s) for s in (1, 2, 4)]
        else:
            s = slices or tr.backend.recon_chunks
            cands.append((c if c == "reduce_scatter" or comm != "auto" else f"all_reduce x{s}", c, s))
    trial = {}
    for name, c, s in cands:
        tr.engine.comm, tr.backend.recon_chunks = c, s
        tr.step()
        trial[name] = round(timed_steps(tr, steps, dev) * 1e3, 4)
    pick = min(trial, key=trial.get)
    _, tr.engine.comm, tr.backend.recon_chunks = next(x for x in cands if x[0] == pick)
    chunks = tr.backend.row_chunks()
    return {"comm": tr.engine.comm, "chosen_by": "auto (fastest in warm-up)" if comm == "auto" else "--comm",
            "trial_ms_per_step": trial, "slices": len(chunks),
            "slice_allreduce": allreduce_algbw(chunks[0][1] - chunks[0][0], K, dev=dev)}


def exchange_exposed(kern, exchange):
    """Move the attribution pass's exchange spans out of `kern` into `exchange`: the compute stream's idle time in
    the exchange per step (events around each slice's wait / synchronous collective on the compute stream; each
    bracketing event costs a few us) and in the 24-byte sums all-reduce."""
    waits = {k: v for k, v in kern.items() if k.startswith("exchange_wait")}
    exchange["exposed_ms_per_step"] = round(sum(waits.values()), 4)
    exchange["exposed_ms_by_slice"] = {k[len("exchange_wait"):]: round(v, 4) for k, v in sorted(waits.items())}
    exchange["sums_allreduce_ms"] = round(kern.get("sums_allreduce", 0.0), 4)
    for k in list(waits) + ["sums_allreduce"]:
        kern.pop(k, None)
    return exchange


def clock_words(tr):
    """The clock words of the fused G4G5 launch's tile-sum scratch (crosscoder_amd.ops.wgrad_clock) of the trainer's
    step workspace, or None (shapes where the fused launch does not serve)."""
    from crosscoder_amd import ops

    ws = getattr(getattr(tr, "crosscoder", None), "_ws", None)  # (the step workspace; the sharded step's too)
    ts = getattr(ws, "tile_sum", None)
    if ts is not None:
        return ops.wgrad_clock(ts)
    return None


def effective_clock(words):
    """Shader clock the chip held over the roofline launches of the timed region: s_memtime ticks / s_memrealtime
    (100 MHz) ticks, both from the last workgroup of each fused G4G5 launch over its lifetime."""
    if words is None:
        return None
    w = words.tolist()
    if w[1] <= 0 or w[2] <= 0:
        return None
    return {"effective_sclk_ghz": round(w[0] / (w[1] * 10.0), 4), "launches": int(w[2]),
            "window_ms": round(w[1] * 1e-5, 3),
            "source": "s_memtime / s_memrealtime of the last workgroup of each G4G5 launch (gemm.hip WgradTail::clock)"}


def make_cfg(B, n, d, h):
    return {
        "seed": 49, "batch_size": B, "buffer_mult": 128, "lr": 5e-5, "num_tokens": 400_000_000, "l1_coeff": 2,
        "beta1": 0.9, "beta2": 0.999, "dict_size": h, "seq_len": 1024, "enc_dtype": "bf16", "model_name": "synthetic",
        "device": f"cuda:{torch.cuda.current_device()}", "model_batch_size": 4, "log_every": 100,
        "save_every": 30000, "dec_init_norm": 0.08, "d_in": d, "n_models": n,
    }


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(B, n, d, h):
    """Oracle (the reference's PyTorch fp32 step restated, CPU) on a bounded sample of the same workload:
    `rows` batch rows of normalised synthetic activations (Buffer.next scaling, buffer.py:115-125) for the
    config's crosscoder, median of 5 steps after 1 warm-up; the per-step cost is linear in the rows."""
    from oracle import cpu_reference as O

    # this process's CPU share: OMP_NUM_THREADS (16 per GPU on the box), else the affinity mask
    cores = int(os.environ.get("OMP_NUM_THREADS") or 0) or len(os.sched_getaffinity(0))
    torch.set_num_threads(cores)
    # ~3 s per oracle step on the box's 16 threads at config 2 (4096 rows): keep every config near that
    rows = max(256, min(B, int(B * (2 * 2304 * 16384) / (n * d * h)) // 256 * 256))
    cfg = {"seed": 49, "dict_size": h, "d_in": d, "enc_dtype": "fp32", "dec_init_norm": 0.08,
           "batch_size": rows, "num_tokens": 400_000_000, "lr": 5e-5, "beta1": 0.9, "beta2": 0.999, "l1_coeff": 2}
    P = O.init_params(cfg, n_models=n)
    tr = O.OracleTrainer(cfg, P, n_models=n)
    g = torch.Generator().manual_seed(0)
    scales = torch.tensor([(1 / 0.2759, 1 / 0.2442, 1 / 0.31, 1 / 0.27)[i % 4] for i in range(n)])
    buf = (torch.randn(rows, n, d, generator=g) * scales[None, :, None]).to(torch.bfloat16)
    factor = torch.tensor([(d ** 0.5) / buf[:, i].float().norm(dim=-1).mean().item() for i in range(n)]).to(
        torch.bfloat16)
    x = O.buffer_next(buf, factor)  # normalised: ||x_n|| ~ sqrt(d)
    tr.step(x)  # warm-up
    times = []
    t_start = time.perf_counter()
    while len(times) < 5 and (time.perf_counter() - t_start) < 25.0:
        t0 = time.perf_counter()
        tr.step(x)
        times.append(time.perf_counter() - t0)
    times.sort()
    med = times[len(times) // 2]
    return {"value": round(rows / med, 1), "unit": "activations/s", "cores": cores, "kind": "port",
            "cpu_model": cpu_model(),
            "sample": f"oracle fp32 Trainer.step on {rows} normalised rows of the {n}x{d}->{h} crosscoder "
                      f"(bench batch {B}; cost is linear in rows), median of {len(times)} steps after 1 "
                      f"warm-up, {med:.2f} s/step"}


def hbm_rows(kern, B, n, d, h_local, es=2):
    """Achieved HBM rate of the streaming kernels from the attribution pass (algorithmic bytes: every
    operand read once, every output written once)."""
    K = n * d
    enc = h_local * K + h_local  # encoder half of the arena (W_enc + b_enc)
    dec = h_local * K + K
    per = 7 * es  # Adam: p, g, m, v read + p, m, v written
    # the decoder half: W_dec's first hs rows on the side stream beside G1, the rest + b_dec after G1
    hs = min(h_local, int(h_local * engine.DEC_SIDE_ROWS) // 8 * 8)
    byts = {"adam": enc * per, "adam_dec": hs * K * per, "adam_dec_rest": (dec - hs * K) * per,
            "prep": B * K * es + 2 * B * K * es,            # raw batch in; x and x^T out
            "loss": B * K * 4 + B * K * es + 2 * B * K * es,  # recon fp32 + x in; g_recon and g_recon^T out
            "dec_norms_T": 2 * h_local * K * es}             # W_dec in, W_dec^T out (+ norms)
    out = {}
    for k, b in byts.items():
        if k in kern and kern[k] > 0:
            gbs = b / (kern[k] * 1e-3) / 1e9
            out[k] = {"ms": round(kern[k], 4), "bytes": b, "GB_s": round(gbs, 1),
                      "frac": round(gbs / PEAK_HBM_GBS, 3)}
    if "adam_dec" in out:
        out["adam_dec"]["note"] = ("W_dec's first rows, side stream, concurrent with the next step's prep / G1; "
                                   "also writes the decoder norms' per-block partials of the updated W_dec")
    if "adam_dec_rest" in out:
        out["adam_dec_rest"]["note"] = "the decoder half's remaining rows + b_dec, main stream after G1"
    if "dec_norms_T" in out:
        out["dec_norms_T"]["note"] = "side stream, concurrent with G1"
    return out


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args, argv):
    """`--gpus N` (N > 1) without a torchrun wrapper: start N rank processes under torch.distributed.run as
    ONE child process group (subprocess: this parent never execs and touches no GPU -- it imports no HIP
    library and only counts devices), relay rank 0's JSON line, and return non-zero if any rank fails or the
    deadline passes (the whole group is then killed).  Returns the exit code."""
    n = args.gpus
    one_device = os.environ.get("CC_BENCH_ONE_DEVICE") == "1"  # rehearsal: every rank on cuda:0, gloo
    if not one_device and not args.launcher_check:
        # (torch counts through amdsmi on ROCm -- falling back to hipGetDeviceCount, which loads the HIP runtime
        # without creating a context; the parent launches no kernel and never execs)
        have = torch.cuda.device_count()
        if have < n:
            print(f"bench.py: --gpus {n} needs {n} visible GPUs, found {have}; no measurement made",
                  file=sys.stderr, flush=True)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + argv
    env = dict(os.environ, CC_BENCH_LAUNCHED="1")
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=None, text=True, env=env, start_new_session=True)
    lines = []

    def pump():  # rank output: the JSON line is kept, everything else goes to stderr
        for line in p.stdout:
            if line.startswith("{"):
                lines.append(line.strip())
            else:
                sys.stderr.write(line)
                sys.stderr.flush()

    th = threading.Thread(target=pump, daemon=True)
    th.start()
    try:
        rc = p.wait(timeout=args.deadline)
    except subprocess.TimeoutExpired:
        print(f"bench.py: the {n} ranks did not finish within --deadline {args.deadline} s; killing them",
              file=sys.stderr, flush=True)
        for sig in (signal.SIGTERM, signal.SIGKILL):
            try:
                os.killpg(p.pid, sig)
            except ProcessLookupError:
                break
            try:
                p.wait(timeout=10)
                break
            except subprocess.TimeoutExpired:
                continue
        return 124
    th.join(timeout=10)
    if rc != 0:
        print(f"bench.py: rank launcher exited with {rc}", file=sys.stderr, flush=True)
        return rc
    if not lines:
        print("bench.py: the ranks printed no result line", file=sys.stderr, flush=True)
        return 3
    try:
        n_gpus = json.loads(lines[-1]).get("n_gpus")
    except json.JSONDecodeError:
        n_gpus = None
    if n_gpus != n:
        print(f"bench.py: the result line reports n_gpus {n_gpus}, asked for {n}", file=sys.stderr, flush=True)
        return 3
    print(lines[-1], flush=True)
    return 0


def launcher_check(args):
    """--launcher-check (CPU test of the N-rank launch, no GPU and no HIP library): every rank joins a gloo group
    and all-reduces its rank; rank 0 prints a line shaped like the bench's."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=args.pg_timeout))
    t = torch.tensor([float(rank)])
    dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"metric": "launcher-check", "n_gpus": world, "world_size_pg": dist.get_world_size(),
                          "rank_sum": t.item()}), flush=True)
    if args.launcher_check == "hang" and rank == world - 1:
        time.sleep(3600)  # a rank that never returns: the parent's deadline must end the run
    dist.destroy_process_group()
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs (ranks) of this node; N > 1 without a torchrun wrapper starts the N ranks itself")
    ap.add_argument("--deadline", type=float, default=1200.0,
                    help="N > 1 launched by this script: seconds before every rank is killed (exit 124)")
    ap.add_argument("--pg-timeout", type=float, default=300.0, help="torch.distributed collective timeout, s")
    ap.add_argument("--launcher-check", nargs="?", const="ok", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, choices=sorted(CONFIGS), default=None,
                    help="BASELINE.json config (default: 2 on one GPU, 3 when sharded over N > 1)")
    ap.add_argument("--batch", type=int)
    ap.add_argument("--n-models", type=int)
    ap.add_argument("--d-model", type=int)
    ap.add_argument("--dict-size", type=int, help="the WHOLE dictionary (split over the ranks when N > 1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--comm", choices=("auto", "all_reduce", "reduce_scatter"), default=None,
                    help="latent-sharded step: the partial-reconstruction exchange (default N > 1: auto = time both "
                         "during warm-up, run the faster; one rank: all_reduce)")
    ap.add_argument("--no-n1", action="store_true",
                    help="N > 1: skip the in-job one-GPU measurement of the same workload (n1_same_workload)")
    ap.add_argument("--recon-chunks", type=int, default=None,
                    help="latent-sharded step: batch slices the all-reduce is overlapped by (default N > 1: timed "
                         "in warm-up with --comm auto, 1 / 2 / 4; one rank: 1)")
    ap.add_argument("--force-sharded", action="store_true",
                    help="diagnostic: run the latent-sharded step even on one rank (1-rank RCCL group)")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")

    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:  # no torchrun wrapper: this process becomes the launcher of the N ranks
            return launch_ranks(args, sys.argv[1:])
    elif int(os.environ["WORLD_SIZE"]) != args.gpus and not args.force_sharded:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}", file=sys.stderr, flush=True)
        return 2
    if args.launcher_check:
        return launcher_check(args)
    return run_rank(args)


def run_rank(args):
    global ca, engine
    import crosscoder_amd as ca
    from crosscoder_amd import engine

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the N > 1 flow on a one-GPU box (never a measurement): every rank on cuda:0, gloo
    # collectives (RCCL refuses two ranks on one device)
    one_device = os.environ.get("CC_BENCH_ONE_DEVICE") == "1"
    if one_device:
        local = 0
    elif local >= torch.cuda.device_count():
        print(f"bench.py: rank {rank} needs cuda:{local}, {torch.cuda.device_count()} GPUs visible", file=sys.stderr,
              flush=True)
        return 2
    torch.cuda.set_device(local)
    sharded_path = world > 1 or args.force_sharded
    backend = None
    if sharded_path:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        pg_timeout = datetime.timedelta(seconds=args.pg_timeout)
        if one_device:
            dist.init_process_group("gloo", rank=rank, world_size=world, timeout=pg_timeout)
        else:
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"), rank=rank, world_size=world,
                                    timeout=pg_timeout)
        backend = dist.get_backend()
        if dist.get_world_size() != world:
            print(f"bench.py: process group has {dist.get_world_size()} ranks, WORLD_SIZE {world}", file=sys.stderr,
                  flush=True)
            return 2
    config = args.config if args.config is not None else (2 if world == 1 else 3)
    B, n, d, h_total = CONFIGS[config]
    B = args.batch or B
    n = args.n_models or n
    d = args.d_model or d
    h_total = args.dict_size or h_total
    custom = (B, n, d, h_total) != CONFIGS[config]
    h_local = h_total // world
    K = n * d
    cfg = make_cfg(B, n, d, h_total)

    if not sharded_path:
        cc = ca.CrossCoder(cfg)
        buf = ca.SyntheticBuffer(cfg, rows=B * 8, n_models=n, seed=0)
        tr = ca.Trainer(cfg, buffer=buf, crosscoder=cc)
    else:
        from crosscoder_amd import sharded

        n1 = None
        if world > 1 and not args.no_n1:
            # the strong-scaling curve's own 1-GPU point, measured in this job before the sharded trainer exists
            if rank == 0:
                n1 = n1_same_workload(cfg)
            dist.barrier()
        comm = args.comm or ("auto" if world > 1 else "all_reduce")
        buf = ca.SyntheticBuffer(cfg, rows=B * 8, n_models=n, seed=0)  # same seed on every rank: replicated batch
        tr = sharded.ShardedTrainer(cfg, buffer=buf, comm="all_reduce" if comm == "auto" else comm,
                                    recon_chunks=args.recon_chunks)

    timer = EventTimer()
    engine.TIMER = timer
    for _ in range(args.warmup):
        tr.step()
    exchange = measure_exchange(tr, comm, K, slices=args.recon_chunks) if sharded_path else None
    # attribution pass (not timed): every kernel bracketed by events
    attrib = EventTimer()
    engine.TIMER = attrib
    attrib.enabled = True
    for _ in range(max(3, min(args.steps, 10))):
        tr.step()
    torch.cuda.synchronize()
    kern = attrib.averages_ms()
    if exchange is not None:
        exchange_exposed(kern, exchange)
    gemms = {k: v for k, v in kern.items() if k.startswith("G")}
    dom = max(gemms, key=gemms.get)
    engine.TIMER = timer
    timer.only = dom  # the roofline kernel, measured live inside the timed region
    clk = clock_words(tr)
    if clk is not None:
        clk.zero_()
    if sharded_path:
        dist.barrier()
    torch.cuda.synchronize()
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

    clock = effective_clock(clk)
    step_s = elapsed / args.steps
    ms = step_s * 1e3
    rows_per_s = B / step_s  # activations (batch rows) trained per second by the whole job: `value`
    # config-2 rows of equal step work (10.n.d.h FLOP per row): config 2 counts 1, config 3 (2^17 latents) 8
    per_row = (n * d * h_total) / (2 * 2304 * 16384)
    dom_ms = timer.averages_ms()[dom]
    samples = sorted(s_.elapsed_time(e_) for s_, e_ in timer.rec.get(dom, []))
    gemm_flop = 2.0 * B * K * h_local  # per GEMM (per rank)
    # G4G5_wgrad is one launch computing both weight gradients (cc_wgrad_both)
    dom_flop = gemm_flop * (2 if dom == "G4G5_wgrad" else 1)
    achieved = dom_flop / (dom_ms * 1e-3) / 1e12
    step_flop = 5 * 2.0 * B * K * h_total  # whole job
    if not engine.transposed_wgrad(B, K, h_local, torch.bfloat16):  # batch-major MN/MN form (cc_wgrad_both)
        SPAN_KERNEL["G4G5_wgrad"] = "gemm_pp_dual_kernel<false, false, 4, 5>"
    traffic, traffic_src = pmc_traffic(dom) if (config, world, custom) == (2, 1, False) else (None, None)
    # algorithmic operand/output bytes of the dominant launch (each input read once, output written once)
    es = 2  # bf16
    alg = {"G1_encode": (B * K + h_local * K + 2 * B * h_local) * es,
           "G2_decode": (B * h_local + h_local * K + 3 * B * K) * es,  # + x in, g_recon / g_recon^T out (fused loss)
           "G3_dacts": (B * K + h_local * K + B * h_local) * es + B * h_local // 8,  # (+ G1's mask bits, g_pre^T out)
           "G4G5_wgrad": (2 * B * h_local + 2 * B * K + 3 * h_local * K) * es}
    dom_alg_bytes = alg.get(dom)
    name = f"{n}x{d}->{h_total}"
    result = {
        "metric": "activations/sec per train step (fwd+bwd+Adam), 2x2304->16384; % bf16 MFMA peak",
        "value": round(rows_per_s, 1),
        "unit": "activations/s",
        "n_gpus": world,
        # the ranks of the process group the collectives ran over (dist.get_world_size()) and its backend
        # ("nccl" = RCCL); 1 / null for the single-GPU step, which has no collectives
        "world_size_pg": dist.get_world_size() if sharded_path else 1,
        "pg_backend": backend,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic (seeded N(0,1) activations scaled per model, normalised as Buffer.next; reference "
                "init seed 49)",
        "config": {"workload": f"crosscoder train step {name}, batch {B}"
                               + (f", latent-sharded over {world} GPUs ({h_local} latents per GPU)" if world > 1
                                  else ""),
                   "baseline_config": None if custom else config,
                   "global_batch": B, "n_models": n, "d_model": d, "dict_size": h_total,
                   "parallelism": f"latent{world}"},
        "metric_equiv_acts_per_s": round(rows_per_s * per_row, 1),
        "metric_equiv_per_row": per_row,
        "latent_acts_per_s": round(rows_per_s * h_total, 1),
        # N > 1: the same workload on one GPU, measured in this job on rank 0 before the sharded run, so the
        # strong-scaling curve has its own 1-GPU point (the driver's N = 1 run is the metric's config 2, a
        # different dictionary): efficiency = value / (N x n1_same_workload.value)
        "n1_same_workload": n1 if world > 1 else None,
        "exchange": exchange,
        "step_mfma_frac": round(step_flop / step_s / 1e12 / (PEAK_BF16_TFLOPS * world), 4),
        "kernels_ms": {k: round(v, 4) for k, v in sorted(kern.items())},
        "roofline": {"bound": "mfma", "kernel": dom, "kernel_name": SPAN_KERNEL.get(dom), "kernel_ms": round(dom_ms, 4),
                     "kernel_samples": len(samples),
                     "kernel_ms_min_med_max": [round(samples[0], 4), round(samples[len(samples) // 2], 4),
                                               round(samples[-1], 4)] if samples else None,
                     "rocprof": rocprof_average(dom) if (config, world, custom) == (2, 1, False) else None,
                     "achieved": round(achieved, 1),
                     "peak": round(PEAK_BF16_TFLOPS, 1), "unit": "TFLOP/s", "frac": round(achieved / PEAK_BF16_TFLOPS, 4),
                     "traffic": traffic, "traffic_unit": "HBM bytes per launch (PMC)", "traffic_source": traffic_src,
                     "algorithmic_bytes": dom_alg_bytes},
        # the shader clock over the timed region's roofline launches (DVFS under the package power cap: the same
        # build runs faster on a box that holds a higher clock, so round-over-round comparisons need it)
        "effective_sclk_ghz": clock["effective_sclk_ghz"] if clock else None,
        "clock": clock,
        "hbm": hbm_rows(kern, B, n, d, h_local),
        "last_loss": {k: round(v, 6) for k, v in last.items()},
    }
    if rank == 0:
        if world == 1 and not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline(B, n, d, h_total)
        print(json.dumps(result), flush=True)
    if sharded_path:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
