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
