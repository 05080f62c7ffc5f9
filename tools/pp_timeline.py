"""Diagnostic: per-block wall-clock timeline of the ping-pong GEMM kernels from a CC_PP_STAMPS build
(records [start, main-loop end, end, hw id] per block, 100 MHz s_memrealtime).
Usage: python tools/pp_timeline.py path/to/ppstamps.so [case-substring ...]"""
import ctypes
import os
import sys
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import crosscoder_amd  # noqa: F401,E402
from crosscoder_amd._lib import SIGNATURES  # noqa: E402

B, n, d, h = 4096, 2, 2304, 16384
K = n * d


def analyse(name, rec, nb0=None):
    rec = rec.view(-1, 4).cpu().long()
    t0 = rec[:, 0].min().item()
    st, mid, en = (rec[:, 0] - t0).double() / 100.0, (rec[:, 1] - t0).double() / 100.0, (rec[:, 2] - t0).double() / 100.0
    hw, xcc = rec[:, 3] & 0xFFFFFFFF, rec[:, 3] >> 32
    cu_key = (xcc << 16) | ((hw >> 8) & 0xFF)
    span = en.max().item()
    dur, epi = en - st, en - mid
    print(f"{name}: blocks {rec.shape[0]}, kernel span {span:.1f} us, last block start {st.max():.1f} us, "
          f"tile {dur.mean():.1f} us "
          f"(min {dur.min():.1f} max {dur.max():.1f}), epilogue {epi.mean():.1f} us, main loop {(mid - st).mean():.1f} us")
    if nb0 is not None:
        for lab, sl in (("first GEMM", slice(0, nb0)), ("second GEMM", slice(nb0, None))):
            print(f"   {lab}: tile {dur[sl].mean():.1f} us, epilogue {epi[sl].mean():.1f} us, "
                  f"main {(mid[sl] - st[sl]).mean():.1f} us")
    per_cu = defaultdict(list)
    for i in range(rec.shape[0]):
        per_cu[cu_key[i].item()].append(i)
    counts = sorted(len(v) for v in per_cu.values())
    gaps, ends, busy = [], [], []
    for v in per_cu.values():
        v.sort(key=lambda i: st[i].item())
        for a, b in zip(v, v[1:]):
            gaps.append(st[b].item() - en[a].item())
        ends.append(en[v[-1]].item())
        busy.append(sum(dur[i].item() for i in v))
    print(f"   CUs {len(per_cu)}, tiles per CU min {counts[0]} max {counts[-1]}; "
          f"gap between tiles on a CU: mean {sum(gaps) / max(1, len(gaps)):.2f} us max {max(gaps or [0]):.1f}; "
          f"CU finish: first {min(ends):.1f} last {max(ends):.1f} us; busy/span {sum(busy) / len(busy) / span:.3f}")
    # per-XCD mean tile time
    px = defaultdict(list)
    for i in range(rec.shape[0]):
        px[xcc[i].item()].append(dur[i].item())
    print("   tile us by XCD: " + " ".join(f"{k}:{sum(v) / len(v):.1f}" for k, v in sorted(px.items())))
    # start-time histogram by round (how synchronised the epilogues are)
    order = torch.argsort(st)
    rounds = [order[i:i + 256] for i in range(0, rec.shape[0], 256)]
    print("   per 256-block round: start spread " + " ".join(
        f"{(st[r].max() - st[r].min()).item():.0f}" for r in rounds[:10]) + " us")


def main():
    L = ctypes.CDLL(sys.argv[1])
    for nm, (res, args) in SIGNATURES.items():
        f = getattr(L, nm, None)
        if f is not None:
            f.restype, f.argtypes = res, args
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    bf = torch.bfloat16
    x = torch.randn(B, K, device=dev, generator=g).to(bf)
    W = (torch.randn(h, K, device=dev, generator=g) * 0.02).to(bf)
    b_enc = torch.zeros(h, device=dev, dtype=bf)
    acts = torch.relu(torch.randn(B, h, device=dev, generator=g)).to(bf)
    g_recon = (torch.randn(B, K, device=dev, generator=g) * 1e-3).to(bf)
    g_pre = (torch.randn(B, h, device=dev, generator=g) * 1e-3).to(bf)
    tn = torch.ones(h, device=dev)
    norms = torch.ones(h, n, device=dev)
    colsum = torch.ones(h, device=dev)
    gW, gW2 = torch.empty(h, K, device=dev, dtype=bf), torch.empty(h, K, device=dev, dtype=bf)
    parts, parts2 = torch.empty(1 << 20, device=dev), torch.empty(1 << 20, device=dev)
    buf = torch.zeros(4 * 4096, dtype=torch.int64, device=dev)
    L.cc_debug_set_stamp_buffer(ctypes.c_void_p(buf.data_ptr()))
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    cases = {
        "G1 encode (KC/KC)": (lambda: L.cc_encode_fwd(P(x), P(W), P(b_enc), P(tn), P(acts), 1, P(parts), P(parts),
                                                      P(parts), B, K, h, 1, st), None),
        "G4+G5 dual (MN/MN)": (lambda: L.cc_wgrad_both(P(acts), P(g_recon), P(W), P(norms), P(colsum), 1e-4, P(gW),
                                                       P(parts), P(g_pre), P(x), P(gW2), P(parts2), B, h, n, d, 1, st),
                               (h // 256) * (K // 256)),
        "G4+G5 dual, no L1 term": (lambda: L.cc_wgrad_both(P(acts), P(g_recon), P(W), P(norms), P(colsum), 0.0,
                                                           P(gW), P(parts), P(g_pre), P(x), P(gW2), P(parts2), B, h,
                                                           n, d, 1, st), (h // 256) * (K // 256)),
        "G5 alone (MN/MN)": (lambda: L.cc_wgrad_enc(P(g_pre), P(x), P(gW2), P(parts2), B, h, K, 1, st), None),
        "G4 no L1 term (MN/MN)": (lambda: L.cc_wgrad_dec(P(acts), P(g_recon), P(W), P(norms), P(colsum), 0.0, P(gW),
                                                         P(parts), B, h, n, d, 1, st), None),
    }
    W2 = (torch.randn(h, K, device=dev, generator=g) * 0.02).to(bf)
    rec = torch.empty(B, K, device=dev)
    nws = L.cc_decode_ws_floats(B, h, K, 1)
    ws = torch.empty(max(1, nws), device=dev)
    cases["G2 split-K leftover pass"] = (lambda: L.cc_decode_fwd_ws(P(acts), P(W2), P(rec), P(ws), nws, B, h, K, 1, st),
                                         None)
    aT, grT, gpT, xT = acts.t().contiguous(), g_recon.t().contiguous(), g_pre.t().contiguous(), x.t().contiguous()
    cases["G4+G5 dual (KC/KC, batch-contiguous operands)"] = (
        lambda: L.cc_wgrad_both_t(P(aT), P(grT), P(W), P(norms), P(colsum), 1e-4, P(gW), P(parts), P(gpT), P(xT),
                                  P(gW2), P(parts2), B, h, n, d, 1, st), (h // 256) * (K // 256))
    aT2 = torch.empty(h, B, device=dev, dtype=bf)
    cases["G1 encode + acts^T (as in the step)"] = (
        lambda: L.cc_encode_fwd_t(P(x), P(W), P(b_enc), P(tn), P(acts), P(aT2), 1, P(parts), P(parts), P(parts), B, K,
                                  h, 1, st), None)
    only = sys.argv[2:]
    for name, (fn, nb0) in cases.items():
        if only and not any(o in name for o in only):
            continue
        for _ in range(20):  # warm clocks
            assert fn() == 0
        buf.zero_()
        assert fn() == 0
        torch.cuda.synchronize()
        nrec = (buf.view(-1, 4)[:, 2] > 0).sum().item()
        analyse(name, buf[: 4 * nrec], nb0)


if __name__ == "__main__":
    main()
