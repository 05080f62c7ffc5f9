"""HBM throughput of the kernels around the step at the reference's sizes, next to the
torch ops they replace: the Buffer.refresh shuffle of the 523,776 x 2 x 2304 bf16 buffer, the
decoder-norm analytics and the scale fold over a 2x2304->16384 crosscoder.
Usage: python tools/aux_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import crosscoder_amd as ca  # noqa: E402
from crosscoder_amd import ops  # noqa: E402


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    ts.sort()
    return ts[len(ts) // 2] * 1e-3


def main():
    dev = torch.device("cuda:0")
    rows, n, d, h = 523776, 2, 2304, 16384
    buf = torch.empty(rows, n, d, dtype=torch.bfloat16, device=dev).normal_()
    out = torch.empty_like(buf)
    perm = torch.randperm(rows).to(dev)
    nbytes = 2 * buf.numel() * 2 + rows * 8
    t = timeit(lambda: ops.gather_rows(buf, perm, out=out))
    t_ref = timeit(lambda: buf[perm])
    print(f"shuffle {rows}x{n}x{d} bf16 ({buf.numel() * 2 / 1e9:.2f} GB): cc_gather_rows {t * 1e3:.2f} ms "
          f"({nbytes / t / 1e12:.2f} TB/s) | torch buffer[perm] {t_ref * 1e3:.2f} ms ({nbytes / t_ref / 1e12:.2f} TB/s)")
    del buf, out
    cfg = {"seed": 49, "dict_size": h, "d_in": d, "enc_dtype": "bf16", "dec_init_norm": 0.08, "device": "cuda:0"}
    cc = ca.CrossCoder(cfg)
    a = cc.arena()
    wbytes = h * n * d * 2
    t = timeit(lambda: ops.decoder_stats(a.W_dec_hk, n, d))
    W = cc.W_dec.detach()

    def ref_stats():
        norms = W.norm(dim=-1)
        rel = norms[:, 1] / norms.sum(dim=-1)
        cos = (W[:, 0, :] * W[:, 1, :]).sum(dim=-1) / (W[:, 0, :].norm(dim=-1) * W[:, 1, :].norm(dim=-1))
        return rel, cos

    t_ref = timeit(ref_stats)
    print(f"decoder stats (W_dec {wbytes / 1e6:.0f} MB): cc_decoder_stats {t * 1e6:.1f} us ({wbytes / t / 1e12:.2f} TB/s)"
          f" | torch analysis.py ops {t_ref * 1e6:.1f} us")
    s = torch.tensor([1.0, 1.0], device=dev)
    t = timeit(lambda: ops.fold_scaling(a.W_enc_hk, a.W_dec_hk, a.b_dec_flat, s, n, d))
    fbytes = 2 * 2 * wbytes
    print(f"fold scaling (W_enc + W_dec in place): cc_fold_scaling {t * 1e6:.1f} us ({fbytes / t / 1e12:.2f} TB/s)")


if __name__ == "__main__":
    main()
