"""A/B timing of the five step GEMMs (config-2 shapes) across library builds, interleaved in
ONE process (cdna guide rule 24).  Usage: python tools/gemm_bench.py lib1.so [lib2.so ...]
Env: CC_GEMM_B (batch rows, default 4096: e.g. 2048 for one of two batch slices), CC_GEMM_ONLY (comma list of
the names below)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import crosscoder_amd  # noqa: F401,E402
from crosscoder_amd._lib import SIGNATURES  # noqa: E402

B, n, d, h = int(os.environ.get("CC_GEMM_B", 4096)), 2, 2304, 16384
K = n * d
PEAK = 256 * 2.4e9 * 4096 / 1e12


def load(path):
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        f = getattr(lib, name, None)  # (an older build may lack newer entry points)
        if f is not None:
            f.restype, f.argtypes = res, args
    return lib


def main():
    # each argument: path/to/lib.so[@pp_mask][#nostore]  (the mask selects the ping-pong loop per layout; #nostore:
    # debug build, the ping-pong epilogues skip their output tiles' HBM stores)
    libs = []
    for arg in sys.argv[1:]:
        spec, _, flag = arg.partition("#")
        path, _, mask = spec.partition("@")
        label = os.path.relpath(path)
        libs.append((label + (f"@{mask}" if mask else "") + (f"#{flag}" if flag else ""), load(path),
                     (int(mask) if mask else None, flag == "nostore")))
    dev = torch.device("cuda:0")
    bf = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(B, K, device=dev, generator=g).to(bf)
    W = (torch.randn(h, K, device=dev, generator=g) * 0.02).to(bf)
    W2 = (torch.randn(h, K, device=dev, generator=g) * 0.02).to(bf)
    b_enc = torch.zeros(h, device=dev, dtype=bf)
    acts = torch.empty(B, h, device=dev, dtype=bf)
    recon = torch.empty(B, K, device=dev)
    g_recon = (torch.randn(B, K, device=dev, generator=g) * 1e-3).to(bf)
    g_pre = torch.empty(B, h, device=dev, dtype=bf)
    tn = torch.ones(h, device=dev)
    norms = torch.ones(h, n, device=dev)
    colsum = torch.ones(h, device=dev)
    gW = torch.empty(h, K, device=dev, dtype=bf)
    gW2 = torch.empty(h, K, device=dev, dtype=bf)
    parts2 = torch.empty(1 << 20, device=dev)
    parts = torch.empty(1 << 20, device=dev)
    # the transposed operands must carry the real G1 / G3 outputs (all-zero operands run at higher clocks)
    acts.copy_(torch.relu(torch.randn(B, h, device=dev, generator=g)).to(bf))
    g_pre.copy_((torch.randn(B, h, device=dev, generator=g) * 1e-3).to(bf))
    actsT, grT, gpT, xT = acts.t().contiguous(), g_recon.t().contiguous(), g_pre.t().contiguous(), x.t().contiguous()
    W2T = W2.t().contiguous()
    actsT2 = torch.empty(h, B, device=dev, dtype=bf)
    gpT2 = torch.empty(h, B, device=dev, dtype=bf)
    nws = libs[0][1].cc_decode_ws_floats(B, h, K, 1) if hasattr(libs[0][1], "cc_decode_ws_floats") else 0
    dws = torch.empty(max(nws, 1), device=dev)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    N0 = ctypes.c_void_p(0)
    mbits = torch.zeros(B * h // 32 + 4096, device=dev, dtype=torch.int32)

    def calls(L):
        return {
            "G1_encode": lambda: L.cc_encode_fwd(P(x), P(W), P(b_enc), P(tn), P(acts), 1, P(parts), P(parts), P(parts),
                                                 B, K, h, 1, st),
            # (as the step calls it: no l1 partials -- that selects the whole-tile FAST epilogue)
            "G1_encode_T": lambda: L.cc_encode_fwd_t(P(x), P(W), P(b_enc), P(tn), P(acts), P(actsT2), 1, P(parts),
                                                     N0, P(parts), P(mbits), N0, N0, B, K, h, 1, st),
            "G2_decode": lambda: L.cc_decode_fwd(P(acts), P(W2), N0, P(recon), N0, B, h, K, 1, st),
            "G2_decode_ws": lambda: L.cc_decode_fwd_ws(P(acts), P(W2), P(recon), P(dws), nws, B, h, K, 1, st),
            "G2_decode_ws_T": lambda: L.cc_decode_fwd_ws_t(P(acts), P(W2T), P(recon), P(dws), nws, B, h, K, 1, st),
            "G3_dacts_T": lambda: L.cc_dacts_bwd_t(P(g_recon), P(W2), P(acts), P(tn), 1e-4, P(mbits), P(gpT2), B,
                                                   P(parts), N0, N0, B, K, h, 1, st),
            "G3_dacts": lambda: L.cc_dacts_bwd(P(g_recon), P(W2), P(acts), P(tn), 1e-4, P(g_pre), P(parts), B, K, h, 1,
                                               st),
            "G4_wgrad_dec": lambda: L.cc_wgrad_dec(P(acts), P(g_recon), P(W2), P(norms), P(colsum), 1e-4, P(gW),
                                                   P(parts), B, h, n, d, 1, st),
            "G4_no_l1term": lambda: L.cc_wgrad_dec(P(acts), P(g_recon), P(W2), P(norms), P(colsum), 0.0, P(gW),
                                                   P(parts), B, h, n, d, 1, st),
            "G5_wgrad_enc": lambda: L.cc_wgrad_enc(P(g_pre), P(x), P(gW), P(parts), B, h, K, 1, st),
            "G4G5_both_x0.5": lambda: L.cc_wgrad_both(P(acts), P(g_recon), P(W2), P(norms), P(colsum), 1e-4, P(gW),
                                                      P(parts), P(g_pre), P(x), P(gW2), P(parts2), B, h, n, d, 1, st),
            "G4G5_both_T_x0.5": lambda: L.cc_wgrad_both_t(P(actsT), P(grT), P(W2), P(norms), P(colsum), 1e-4, P(gW),
                                                          P(parts), P(gpT), P(xT), P(gW2), P(parts2), B, h, n, d, 1,
                                                          st),
            "G4G5_both_T_noL1_x0.5": lambda: L.cc_wgrad_both_t(P(actsT), P(grT), P(W2), P(norms), P(colsum), 0.0,
                                                               P(gW), P(parts), P(gpT), P(xT), P(gW2), P(parts2), B,
                                                               h, n, d, 1, st),
            "G5_on_G4_data": lambda: L.cc_wgrad_enc(P(acts), P(g_recon), P(gW), P(parts), B, h, K, 1, st),
        }

    flop = 2.0 * B * K * h
    res = {}
    for rnd in range(5):
        for path, L, (mask, nostore) in libs:
            if mask is not None:
                L.cc_debug_set_pp_mask(mask)
            if hasattr(L, "cc_debug_set_epi_store"):
                L.cc_debug_set_epi_store(0 if nostore else 1)
            only = os.environ.get("CC_GEMM_ONLY")
            for name, fn in calls(L).items():
                if only and name not in only.split(","):
                    continue
                for _ in range(2):
                    assert fn() == 0
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(10):
                    fn()
                e.record()
                torch.cuda.synchronize()
                res.setdefault((path, name), []).append(s.elapsed_time(e) / 10 / (2 if name.startswith("G4G5") else 1))
    for (p, name), ts in sorted(res.items(), key=lambda kv: (kv[0][1], kv[0][0])):
        ts.sort()
        med = ts[len(ts) // 2]
        print(f"B={B} {name:14s} {p:34s} median {med*1e3:7.1f} us  min {ts[0]*1e3:7.1f} us  {flop/med/1e9:7.1f} TF/s "
              f"({flop/med/1e9/PEAK*100:4.1f}% peak)")


if __name__ == "__main__":
    main()
