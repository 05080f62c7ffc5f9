"""A/B of whole-step variants on ONE device, interleaved (cdna guide rule 24): config-2 Trainer.step
with individual scheduling features switched off.  Usage: python tools/step_ab.py [--spans]
(--spans: per-launch HIP-event averages of each variant as well)."""
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
    ws_t = engine.StepWorkspace(bench.B, cc.n_models, cfg["d_in"], cc.d_hidden, cc.dtype, dev)
    os.environ["CC_TRANSPOSED_WGRAD"] = "0"
    ws_b = engine.StepWorkspace(bench.B, cc.n_models, cfg["d_in"], cc.d_hidden, cc.dtype, dev)
    os.environ.pop("CC_TRANSPOSED_WGRAD")
    part = ws_t.norm_part

    defaults = (tr.mapped_losses, tr.overlap_decoder_adam, engine.DEC_ADAM_BLOCKS)

    def setup(ws, mapped=defaults[0], fused=True, side=defaults[1], blocks=defaults[2], fused_adam="serial",
              tails=True, fence_all=0, after_enc=True, dec_one=1, xmean_after=True):
        def f():
            cc._ws = ws
            engine.XMEAN_AFTER_G1 = xmean_after
            ca._lib.load().cc_debug_set_dec_one_launch(dec_one)
            engine.SIDE_AFTER_ENC = after_enc
            engine.FUSED_TAILS = tails
            ca._lib.load().cc_debug_set_tail_fence(fence_all)
            engine.FUSED_DEC_ADAM = fused_adam
            tr.mapped_losses = mapped
            tr.overlap_decoder_adam = side
            engine.DEC_ADAM_BLOCKS = blocks
            ws.norm_part = part if (fused and ws is ws_t) else None
            ws.norms_token = None
        return f

    variants = {"default": setup(ws_t), "fused dec Adam beside G1": setup(ws_t, fused_adam=True),
                "fused dec Adam serial": setup(ws_t, side=False), "flat dec Adam serial": setup(ws_t, side=False,
                                                                                             fused_adam=False),
                "side Adam 384 blocks": setup(ws_t, blocks=384), "batch-major wgrad": setup(ws_b),
                "separate tails": setup(ws_t, tails=False), "tails fence all": setup(ws_t, fence_all=1),
                "mapped losses": setup(ws_t, mapped=True), "side Adam 128 blocks": setup(ws_t, blocks=128),
                "side Adam 192 blocks": setup(ws_t, blocks=192), "side Adam beside enc": setup(ws_t, after_enc=False),
                "G2 two launches": setup(ws_t, dec_one=0), "x mean before G1": setup(ws_t, xmean_after=False)}
    only = [a.split("=", 1)[1] for a in sys.argv if a.startswith("--only=")]
    if only:
        variants = {k: v for k, v in variants.items() if k in only[0].split(",")}
    spans = "--spans" in sys.argv
    timers = {k: bench.EventTimer() for k in variants} if spans else {}
    for t in timers.values():
        t.enabled = True
    res = {k: [] for k in variants}
    for f in variants.values():
        f()
        for _ in range(3):
            tr.step()
    for _ in range(10):
        for name, f in variants.items():
            f()
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
    if os.environ.get("STEPAB_HIPRIO"):  # every launch on a high-priority stream (the side stream stays at 0)
        torch.cuda.set_device(0)
        hs = torch.cuda.Stream(priority=-int(os.environ["STEPAB_HIPRIO"]))
        print("main stream priority", hs.priority, "range", torch.cuda.Stream.priority_range())
        with torch.cuda.stream(hs):
            main()
    else:
        main()
