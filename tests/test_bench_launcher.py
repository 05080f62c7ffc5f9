"""bench.py's N-rank entry, on the CPU: `--gpus N` without a torchrun wrapper starts the N
ranks itself and relays rank 0's line, refuses to run with fewer GPUs than asked, and kills ranks that pass its
deadline.  The rank bodies here are the gloo `--launcher-check` (no GPU, no HIP library); the GPU rehearsal of
the real step (`CC_BENCH_ONE_DEVICE=1 python bench.py --gpus 2`) is in tests/test_gpu_sharded.py."""
import json
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    env["PYTHONDONTWRITEBYTECODE"] = "1"
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, env=env, timeout=timeout,
                       cwd=ROOT)
    return p, time.monotonic() - t0


def json_lines(out):
    return [json.loads(s) for s in out.splitlines() if s.startswith("{")]


def test_gpus_2_launches_two_ranks_without_torchrun():
    p, _ = run(["--gpus", "2", "--launcher-check"])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = json_lines(p.stdout)
    assert len(lines) == 1, p.stdout
    assert lines[0]["n_gpus"] == 2 and lines[0]["world_size_pg"] == 2
    assert lines[0]["rank_sum"] == 1.0  # ranks 0 + 1 took part in the collective


def test_gpus_more_than_visible_exits_nonzero_without_a_line():
    import torch

    n = max(8, torch.cuda.device_count() + 1)
    p, _ = run(["--gpus", str(n)])
    assert p.returncode != 0
    assert json_lines(p.stdout) == []
    assert "visible GPUs" in p.stderr


def test_world_size_mismatch_exits_nonzero():
    p, _ = run(["--gpus", "4", "--launcher-check"], env_extra={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode == 2
    assert json_lines(p.stdout) == []


def test_deadline_kills_a_hung_rank():
    p, dt = run(["--gpus", "2", "--launcher-check", "hang", "--deadline", "25"], timeout=200)
    assert p.returncode == 124, (p.returncode, p.stderr[-2000:])
    assert dt < 120
    assert "deadline" in p.stderr


@pytest.mark.parametrize("n", [3])
def test_gpus_n_relays_rank0_line(n):
    p, _ = run(["--gpus", str(n), "--launcher-check"])
    assert p.returncode == 0, p.stderr[-2000:]
    (line,) = json_lines(p.stdout)
    assert line["n_gpus"] == n and line["rank_sum"] == float(sum(range(n)))


def test_effective_clock_from_tile_sum_words():
    """bench.py's clock report: shader-clock ticks over 100 MHz wall ticks (gemm.hip WgradTail::clock layout:
    [sclk ticks, wall ticks, launches, ...]); no launch recorded gives no report."""
    import importlib.util
    import torch
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    words = torch.zeros(8, dtype=torch.int64)
    assert bench.effective_clock(words) is None
    words[0], words[1], words[2] = 1_720_000_000, 100_000_000, 3     # 1 s of wall ticks at 1.72 GHz
    rep = bench.effective_clock(words)
    assert rep["effective_sclk_ghz"] == pytest.approx(1.72)
    assert rep["launches"] == 3 and rep["window_ms"] == pytest.approx(1000.0)
    assert bench.effective_clock(None) is None


def _load_bench():
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    return bench


class _FakeShardedTrainer:
    """ShardedTrainer's surface measure_exchange uses (engine.comm, backend.row_chunks, step), with a step whose time
    depends on the exchange form (reduce_scatter slower on rank 1: every rank must still pick the same form)."""

    def __init__(self, rank):
        import torch.distributed as dist

        self.rank, self.dist = rank, dist
        self.engine = type("E", (), {"comm": "all_reduce"})()
        bk = self.backend = type("Bk", (), {"recon_chunks": 2})()
        bk.row_chunks = lambda: [(r0, r0 + 32 // bk.recon_chunks) for r0 in range(0, 32, 32 // bk.recon_chunks)]
        self.comms = []

    def step(self):
        import torch

        self.comms.append((self.engine.comm, self.backend.recon_chunks))
        ar = 0.002 if self.backend.recon_chunks == 2 else 0.004 + 0.002 * self.rank
        time.sleep(ar if self.engine.comm == "all_reduce" else 0.006 + 0.004 * self.rank)
        t = torch.ones(4)
        self.dist.all_reduce(t)


def _exchange_rank(rank, world, port, q):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        bench = _load_bench()
        tr = _FakeShardedTrainer(rank)
        ex = bench.measure_exchange(tr, "auto", K=8, dev="cpu", steps=3)
        kern = {"G1_encode": 0.5, "exchange_wait0": 0.12, "exchange_wait1": 0.01, "sums_allreduce": 0.02}
        bench.exchange_exposed(kern, ex)
        q.put((rank, ex, kern, (tr.engine.comm, tr.backend.recon_chunks), sorted(set(tr.comms))))
    finally:
        dist.destroy_process_group()


def test_sharded_bench_exchange_fields_over_two_gloo_ranks():
    """The N > 1 line's exchange evidence, its host logic over 2 gloo ranks: the exchange
    forms (the all-reduce in 1, 2 and 4 batch slices, the reduce-scatter) are timed in warm-up (max over ranks), the
    fastest is left set on the trainer -- the same on every rank --,
    one slice's all-reduce bandwidth is measured, and the attribution pass's exchange spans become the exposed time
    per step (removed from the kernel table)."""
    import random

    import torch.multiprocessing as mp

    world, port = 2, 27000 + random.randint(0, 900)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_exchange_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r[0], r[1:]) for r in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank in range(world):
        ex, kern, comm, tried = res[rank]
        assert tried == [("all_reduce", 1), ("all_reduce", 2), ("all_reduce", 4), ("reduce_scatter", 2)]
        assert comm == ("all_reduce", 2) and ex["comm"] == "all_reduce"
        assert set(ex) == {"comm", "chosen_by", "trial_ms_per_step", "slices", "slice_allreduce",
                           "exposed_ms_per_step", "exposed_ms_by_slice", "sums_allreduce_ms"}
        tr_ms = ex["trial_ms_per_step"]
        assert set(tr_ms) == {"all_reduce x1", "all_reduce x2", "all_reduce x4", "reduce_scatter"}
        assert min(tr_ms["reduce_scatter"], tr_ms["all_reduce x1"], tr_ms["all_reduce x4"]) > tr_ms["all_reduce x2"] > 0
        assert ex["slices"] == 2 and ex["slice_allreduce"]["bytes"] == 16 * 8 * 4
        assert ex["slice_allreduce"]["busbw_GB_s"] == pytest.approx(ex["slice_allreduce"]["algbw_GB_s"], rel=0.01)
        assert ex["exposed_ms_per_step"] == pytest.approx(0.13) and ex["sums_allreduce_ms"] == 0.02
        assert ex["exposed_ms_by_slice"] == {"0": 0.12, "1": 0.01}
        assert kern == {"G1_encode": 0.5}
    # (the forms' times are all-reduced: both ranks report the same trial table)
    assert res[0][0]["trial_ms_per_step"] == res[1][0]["trial_ms_per_step"]
