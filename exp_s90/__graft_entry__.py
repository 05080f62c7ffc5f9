"""Driver entry points: build() compiles the gfx950 HIP library in-tree (and the oracle's
checker inputs); smoke() runs one tiny fused training step on cuda:0 and checks it against
the CPU oracle."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "crosscoder-model-diff-replication_amd")


def build() -> None:
    jobs = str(min(8, os.cpu_count() or 1))
    subprocess.run(["make", "-C", os.path.join(PKG, "csrc"), f"-j{jobs}"], check=True)
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import crosscoder_amd  # noqa: F401
    from crosscoder_amd import _lib

    lib = _lib.load()
    assert lib.cc_version() >= 100


def smoke() -> None:
    import math

    import torch

    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import crosscoder_amd as ca
    from oracle import cpu_reference as O

    dev = torch.device("cuda:0")
    B, n, d, h = 256, 2, 64, 512
    cfg = {"seed": 49, "batch_size": B, "buffer_mult": 128, "lr": 5e-5, "num_tokens": B * 100, "l1_coeff": 2,
           "beta1": 0.9, "beta2": 0.999, "dict_size": h, "seq_len": 1024, "enc_dtype": "fp32", "device": "cuda:0",
           "dec_init_norm": 0.08, "d_in": d, "log_every": 100, "save_every": 30000}
    buf = ca.SyntheticBuffer(cfg, rows=B, seed=0)
    cc = ca.CrossCoder(cfg)
    raw, factor = buf.next_raw()
    x_cpu = O.buffer_next(raw.cpu(), factor.cpu())
    P = {k: getattr(cc, k).detach().cpu().clone() for k in O.PARAM_ORDER}
    ref = O.OracleTrainer(dict(cfg, device="cpu"), P)
    d_ref = ref.step(x_cpu)
    buf.buffer_pointer = 0
    tr = ca.Trainer(cfg, buffer=buf, crosscoder=cc)
    d_gpu = tr.step()
    torch.cuda.synchronize()
    for k in ("loss", "l2_loss", "l1_loss", "l0_loss", "explained_variance"):
        assert math.isclose(d_gpu[k], d_ref[k], rel_tol=1e-5, abs_tol=1e-6), (k, d_gpu[k], d_ref[k])
    st = tr.optimizer.state  # (orders after the side-stream decoder-half Adam)
    for k in O.PARAM_ORDER:
        a, b = getattr(cc, k).detach().cpu(), ref.P[k].detach()
        assert (a - b).abs().max().item() <= 0.01 * cfg["lr"], k  # fp32: Adam's update agrees to 1 % of lr
        m = st[getattr(cc, k)]["exp_avg"].cpu()
        assert (m - ref.m[k]).norm().item() <= 1e-5 * ref.m[k].norm().item(), k
    print("smoke ok:", {k: round(v, 6) for k, v in d_gpu.items()})


if __name__ == "__main__":
    build()
    if len(sys.argv) > 1 and sys.argv[1] == "smoke":
        smoke()
