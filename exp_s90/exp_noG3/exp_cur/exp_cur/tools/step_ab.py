"""Whole-step timing of config 2 on ONE device, for same-box A/B: schedule variants of the decoder-half
Adam are defined HERE (monkeypatching engine.adam inside this process) -- the product keeps a single
schedule -- and library builds via --lib.  Variants run interleaved, 20 steps per sample.
  python tools/step_ab.py [--lib path/to/variant.so] [--spans] [--rounds R] [--only=a,b]
The variants below are the round-2 schedule experiments behind profiles/r02_step_ab_*.txt: they assume the
W_dec^T workspace copy (ws.W_dec_t), which the step no longer keeps since round 3 (G2 reads W_dec itself);
round-3 A/Bs are whole source trees timed by tools/ab_trees.sh / ab_multi.sh instead."""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def fused_dec_adam(blocks):
    """Decoder half as the 64x64-tile Adam that also writes W_dec^T + the norm partials (one HBM pass,
    cc_adam_dec_transposed) with a capped grid, beside the next step's G1."""
    from crosscoder_amd import engine, ops

    def adam(ws, P, G, M, V, lr, beta1, beta2, eps, step, side_stream=None):
        coef = ws.clip_out[0:1]
        dev = P.data.device
        ops.adam_step(P.enc_part(), G.enc_part(), M.enc_part(), V.enc_part(), coef, lr, beta1, beta2, eps, step)
        enc_done = torch.cuda.Event()
        enc_done.record(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side_stream):
            side_stream.wait_event(enc_done)
            ops.adam_dec_transposed(P.W_dec_hk, G.W_dec_hk, M.W_dec_hk, V.W_dec_hk, coef, lr, beta1, beta2, eps, step,
                                    ws.W_dec_t, ws.norm_part, max_blocks=blocks)
            ops.adam_step(P.b_dec_flat, G.b_dec_flat, M.b_dec_flat, V.b_dec_flat, coef, lr, beta1, beta2, eps, step)
            ops.dec_norms_finalize(ws.norm_part, ws.h, ws.n, ws.d, ws.norms, ws.tn, ws.inv_norms)
            ws.norms_token = engine._norms_token(P)
            done = torch.cuda.Event()
            done.record(side_stream)
        P.pending = done
    return adam


def serial_adam(norms_beside):
    """The whole Adam as one flat launch on the main stream (no decoder half beside G1); the next step's
    W_dec^T + decoder norms then either on the side stream beside prep / G1 (norms_beside) or on the main
    stream before G2 (forward's decoder_norms)."""
    from crosscoder_amd import engine

    def adam(ws, P, G, M, V, lr, beta1, beta2, eps, step, side_stream=None):
        coef = ws.clip_out[0:1]
        from crosscoder_amd import ops
        with engine._span("adam"):
            ops.adam_step(P.data, G.data, M.data, V.data, coef, lr, beta1, beta2, eps, step)
        if not norms_beside:
            return
        dev = P.data.device
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side_stream):
            side_stream.wait_event(ev)
            engine.norms_for_next(ws, P)
            done = torch.cuda.Event()
            done.record(side_stream)
        P.pending = done
    return adam


def dec_adam_side_norms_main():
    """Decoder-half Adam on the side stream as shipped, but W_dec^T + the decoder norms on the main stream
    before G2 (forward's decoder_norms), after the wait for the side stream."""
    from crosscoder_amd import engine, ops

    def adam(ws, P, G, M, V, lr, beta1, beta2, eps, step, side_stream=None):
        coef = ws.clip_out[0:1]
        dev = P.data.device
        with engine._span("adam"):
            ops.adam_step(P.enc_part(), G.enc_part(), M.enc_part(), V.enc_part(), coef, lr, beta1, beta2, eps, step)
        enc_done = torch.cuda.Event()
        enc_done.record(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side_stream):
            side_stream.wait_event(enc_done)
            ops.adam_step(P.dec_part(), G.dec_part(), M.dec_part(), V.dec_part(), coef, lr, beta1, beta2, eps, step,
                          max_blocks=engine.DEC_ADAM_BLOCKS)
            done = torch.cuda.Event()
            done.record(side_stream)
        P.pending = done
    return adam


def dec_adam_with_enc():
    """Decoder-half Adam on the side stream from the moment the clip coefficient exists (event recorded
    BEFORE the encoder-half Adam), so the two halves share the HBM instead of running back to back."""
    from crosscoder_amd import engine, ops

    def adam(ws, P, G, M, V, lr, beta1, beta2, eps, step, side_stream=None):
        coef = ws.clip_out[0:1]
        dev = P.data.device
        ready = torch.cuda.Event()
        ready.record(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side_stream):
            side_stream.wait_event(ready)
            ops.adam_step(P.dec_part(), G.dec_part(), M.dec_part(), V.dec_part(), coef, lr, beta1, beta2, eps, step,
                          max_blocks=engine.DEC_ADAM_BLOCKS)
            engine.norms_for_next(ws, P)
            done = torch.cuda.Event()
            done.record(side_stream)
        with engine._span("adam"):
            ops.adam_step(P.enc_part(), G.enc_part(), M.enc_part(), V.enc_part(), coef, lr, beta1, beta2, eps, step)
        P.pending = done
    return adam


class SidePriority:
    """Variant: the side stream (decoder-half Adam, W_dec^T + norms, loss tail) created with high priority."""

    def __init__(self, tr):
        self.tr = tr

    def on(self):
        self.saved = self.tr._side
        self.tr._side = torch.cuda.Stream(device=self.tr.crosscoder.arena().data.device, priority=-1)

    def off(self):
        self.tr._side = self.saved


class TwoPassLoss:
    """Variant: G2 to the fp32 reconstruction, then the separate loss kernel (cc_decode_fwd_ws_t +
    cc_loss_fwd_bwd_rows_t: the round-2 form) instead of the loss in G2's epilogue (cc_decode_loss_t)."""

    def __init__(self, tr):
        self.tr = tr

    def on(self):
        ws = self.tr.crosscoder._ws
        self.saved, ws.fused_ncb = ws.fused_ncb, 0

    def off(self):
        self.tr.crosscoder._ws.fused_ncb = self.saved


def flat_dec_adam(blocks):
    from crosscoder_amd import engine

    shipped = engine.adam

    def adam(*a, **k):
        old = engine.DEC_ADAM_BLOCKS
        engine.DEC_ADAM_BLOCKS = blocks
        try:
            shipped(*a, **k)
        finally:
            engine.DEC_ADAM_BLOCKS = old
    return adam


class G2FromWdec:
    """Variant: G2 reads W_dec directly (MN operand, cc_decode_fwd_ws) and the side stream computes only
    the decoder norms -- no W_dec^T pass (302 MB of HBM traffic less per step)."""

    def __init__(self, tr):
        from crosscoder_amd import engine, ops
        self.engine, self.ops, self.tr = engine, ops, tr
        self.saved = (ops.decode_partial_t, engine._decoder_derived)

    def on(self):
        engine, ops, tr = self.engine, self.ops, self.tr
        P = tr.crosscoder.arena()
        plain_decode = self.saved[0].__globals__["decode_partial"]

        def decode_partial_t(acts, W_dec_t, recon, ws=None):
            plain_decode(acts, P.W_dec_hk, recon, ws)

        def decoder_derived(ws, P_):
            with engine._span("dec_norms"):
                ops.dec_norms(P_.W_dec_hk, ws.h, ws.n, ws.d, norms=ws.norms, total=ws.tn, inv_norms=ws.inv_norms)

        ops.decode_partial_t = decode_partial_t
        engine._decoder_derived = decoder_derived
        tr.crosscoder._ws.norms_token = None

    def off(self):
        self.ops.decode_partial_t, self.engine._decoder_derived = self.saved
        self.tr.crosscoder._ws.norms_token = None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib")
    ap.add_argument("--spans", action="store_true")
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--only")
    args = ap.parse_args()
    import crosscoder_amd as ca

    if args.lib:
        ca._lib.load(args.lib)  # first load wins: every later call uses this build
    import bench
    from crosscoder_amd import engine

    torch.cuda.set_device(0)
    B, n, d, h = bench.CONFIGS[2]
    cfg = bench.make_cfg(B, n, d, h)
    tr = ca.Trainer(cfg, buffer=ca.SyntheticBuffer(cfg, rows=B * 8, seed=0), crosscoder=ca.CrossCoder(cfg))
    shipped = engine.adam
    tr.step()
    g2mn = G2FromWdec(tr)
    # name -> (adam function, setup, teardown)
    variants = {"shipped": (shipped, None, None)}
    for b in (64, 96, 128, 192, 256, 384, 512, 768, 1024, 2048):
        variants[f"fused dec Adam {b} blocks"] = (fused_dec_adam(b), None, None)
    for b in (512, 1024):
        variants[f"flat dec Adam {b} blocks"] = (flat_dec_adam(b), None, None)
    variants["dec Adam beside G1 + norms on main"] = (dec_adam_side_norms_main(), None, None)
    tp = TwoPassLoss(tr)
    variants["two-pass decode + loss"] = (shipped, tp.on, tp.off)
    variants["serial Adam + norms beside G1"] = (serial_adam(True), None, None)
    variants["serial Adam + norms before G2"] = (serial_adam(False), None, None)
    variants["G2 from W_dec (no W_dec^T pass)"] = (shipped, g2mn.on, g2mn.off)
    variants["dec Adam with enc Adam"] = (dec_adam_with_enc(), None, None)
    sp = SidePriority(tr)
    variants["side stream high priority"] = (shipped, sp.on, sp.off)
    variants["dec Adam with enc Adam + side high priority"] = (dec_adam_with_enc(), sp.on, sp.off)
    if args.only:
        keep = args.only.split(",")
        variants = {k: v for k, v in variants.items() if k in keep}
    timers = {k: bench.EventTimer() for k in variants} if args.spans else {}
    res = {k: [] for k in variants}

    def use(v):
        fn, setup, _ = v
        tr.synchronize()
        torch.cuda.synchronize()
        engine.adam = fn
        if setup:
            setup()

    def drop(v):
        tr.synchronize()
        torch.cuda.synchronize()
        if v[2]:
            v[2]()

    for v in variants.values():
        use(v)
        for _ in range(3):
            tr.step()
        drop(v)
    for _ in range(args.rounds):
        for name, v in variants.items():
            use(v)
            tr.step()  # switch-over step (the previous variant's side-stream work drains)
            tr.synchronize()
            torch.cuda.synchronize()
            if args.spans:
                timers[name].enabled = True
                engine.TIMER = timers[name]
            t0 = time.perf_counter()
            for _ in range(20):
                tr.step()
            torch.cuda.synchronize()
            engine.TIMER = None
            res[name].append((time.perf_counter() - t0) / 20 * 1e3)
            drop(v)
    engine.adam = shipped
    print(f"library: {args.lib or 'in-tree'}")
    for name, ts in res.items():
        ts.sort()
        print(f"{name:28s} median {ts[len(ts) // 2]:.4f} ms/step  min {ts[0]:.4f}")
        if args.spans:
            print("   ", {k: round(v, 4) for k, v in timers[name].averages_ms().items()})


if __name__ == "__main__":
    main()
