"""Where the grad tail's time goes inside the fused G4G5 launch: times, on the same config-2 step operands,
the dual weight-gradient GEMM alone, the dual GEMM + the stand-alone grad tail, and the fused launch
(cc_wgrad_both_clip_t) -- of the in-tree library and of experiment builds given on the command line
(tools/build_variant.sh NAME -DCC_EXP_TAIL_NOBIAS / -DCC_EXP_TAIL_NOCLIP / -DCC_EXP_TAIL_NOARRIVE).
Interleaved, HIP events, median of rounds.   python tools/tail_probe.py [variant.so ...]"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import crosscoder_amd as ca  # noqa: E402
from crosscoder_amd import _lib, engine, ops  # noqa: E402


def typed(path):
    lib = ctypes.CDLL(path)
    for name in ("cc_wgrad_both_t", "cc_grad_tail", "cc_wgrad_both_clip_t"):
        res, args = _lib.SIGNATURES[name]
        getattr(lib, name).restype = res
        getattr(lib, name).argtypes = args
    return lib


def main():
    torch.cuda.set_device(0)
    B, n, d, h = bench.CONFIGS[2]
    cfg = bench.make_cfg(B, n, d, h)
    tr = ca.Trainer(cfg, buffer=ca.SyntheticBuffer(cfg, rows=B * 2, seed=0), crosscoder=ca.CrossCoder(cfg))
    for _ in range(2):
        tr.step()
    tr.synchronize()
    torch.cuda.synchronize()
    ws, P, G = tr.crosscoder._ws, tr.crosscoder.arena(), tr.optimizer.grads
    l1s = 2.0 / B
    libs = [("in-tree", _lib.load())] + [(os.path.basename(p), typed(p)) for p in sys.argv[1:]]
    shipped_lib = ops.lib

    def run(kind):
        if kind in ("dual", "dual+tail"):
            ops.wgrad_both_t(ws.acts_t, ws.g_recon_t, P.W_dec_hk, ws.inv_norms, ws.colsum_acts, l1s, G.W_dec_hk,
                             ws.sq_slice(1), ws.g_pre_t, ws.x_t, G.W_enc_hk, ws.sq_slice(0), n, d)
            if kind == "dual+tail":
                ops.grad_tail(ws.gpre_colpart, G.b_enc, ws.sq_slice(2), engine.loss_colpart(ws), G.b_dec_flat,
                              ws.sq_slice(3), ws.sq, ws.sq_off, 1.0, True, ws.clip_out, ws.tail_ctr[1:2])
        else:
            ops.wgrad_both_clip_t(ws.acts_t, ws.g_recon_t, P.W_dec_hk, ws.inv_norms, ws.colsum_acts, l1s, G.W_dec_hk,
                                  ws.sq_slice(1), ws.g_pre_t, ws.x_t, G.W_enc_hk, ws.sq_slice(0), n, d,
                                  ws.gpre_colpart, G.b_enc, ws.sq_slice(2), engine.loss_colpart(ws), G.b_dec_flat,
                                  ws.sq_slice(3), ws.sq, ws.sq_off, 1.0, True, ws.clip_out, ws.tail_ctr[1:2], ws.wg_part)

    cases = [("in-tree", "dual"), ("in-tree", "dual+tail")] + [(nm, "fused") for nm, _ in libs]
    res = {c: [] for c in cases}
    for rnd in range(7):
        for c in cases:
            L = dict(libs)[c[0]]
            ops.lib = lambda L=L: L  # noqa: E731
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            run(c[1])
            e0.record()
            for _ in range(5):
                run(c[1])
            e1.record()
            torch.cuda.synchronize()
            if rnd:
                res[c].append(e0.elapsed_time(e1) / 5 * 1e3)
    ops.lib = shipped_lib
    for c, ts in res.items():
        ts.sort()
        print(f"{c[0]:24s} {c[1]:10s} median {ts[len(ts) // 2]:8.1f} us  min {ts[0]:8.1f}")


if __name__ == "__main__":
    main()
