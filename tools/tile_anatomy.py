"""Anatomy of a ping-pong GEMM tile from in-kernel clock stamps (probe library built with -DCC_PP_STAMPS:
exp_stamps/libstamps.so, see pp_tile's PP_STAMP points).  Static tile order (the gemm_bench calls pass no tile
counters), config-2 shapes.  Per tile: prologue (entry -> first operands landed), K loop, drain, epilogue (LDS
image + stores issued), and the gap to the workgroup's next tile (tile boundary + the next tile's entry).

  [CC_NOSTORE=1] python tools/tile_anatomy.py exp_stamps/libstamps.so [G1|G3|G4G5 ...]
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import crosscoder_amd  # noqa: F401,E402
from crosscoder_amd._lib import SIGNATURES  # noqa: E402

B, n, d, h = int(os.environ.get("CC_GEMM_B", 4096)), 2, 2304, 16384
K = n * d


def main():
    L = ctypes.CDLL(sys.argv[1])
    for name, (res, args) in SIGNATURES.items():
        f = getattr(L, name, None)
        if f is not None:
            f.restype, f.argtypes = res, args
    L.cc_debug_set_stamps.restype = None
    L.cc_debug_set_stamps.argtypes = [ctypes.c_void_p]
    which = sys.argv[2:] or ["G1", "G3", "G4G5"]
    if os.environ.get("CC_NOSTORE"):  # the epilogues skip their output tiles' HBM stores
        L.cc_debug_set_epi_store(0)
        print("(CC_NOSTORE: no output-tile stores)")
    dev = torch.device("cuda:0")
    bf = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(B, K, device=dev, generator=g).to(bf)
    W = (torch.randn(h, K, device=dev, generator=g) * 0.02).to(bf)
    W2 = (torch.randn(h, K, device=dev, generator=g) * 0.02).to(bf)
    b_enc = torch.zeros(h, device=dev, dtype=bf)
    acts = torch.relu(torch.randn(B, h, device=dev, generator=g)).to(bf)
    g_recon = (torch.randn(B, K, device=dev, generator=g) * 1e-3).to(bf)
    g_pre = (torch.randn(B, h, device=dev, generator=g) * 1e-3).to(bf)
    tn = torch.ones(h, device=dev)
    norms = torch.ones(h, n, device=dev)
    colsum = torch.ones(h, device=dev)
    gW = torch.empty(h, K, device=dev, dtype=bf)
    gW2 = torch.empty(K, h, device=dev, dtype=bf)
    parts = torch.empty(1 << 20, device=dev)
    parts2 = torch.empty(1 << 20, device=dev)
    actsT, grT, gpT, xT = acts.t().contiguous(), g_recon.t().contiguous(), g_pre.t().contiguous(), x.t().contiguous()
    acts2 = torch.empty(B, h, device=dev, dtype=bf)
    actsT2 = torch.empty(h, B, device=dev, dtype=bf)
    gpT2 = torch.empty(h, B, device=dev, dtype=bf)
    mbits = torch.zeros(B * h // 32 + 4096, device=dev, dtype=torch.int32)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    N0 = ctypes.c_void_p(0)
    calls = {
        # (as the step calls it: no l1 partials -- that selects the whole-tile FAST epilogue)
        "G1": (lambda: L.cc_encode_fwd_t(P(x), P(W), P(b_enc), P(tn), P(acts2), P(actsT2), 1, P(parts), N0,
                                         P(parts), P(mbits), N0, N0, B, K, h, 1, st), (B // 256) * (h // 256)),
        "G3": (lambda: L.cc_dacts_bwd_t(P(g_recon), P(W2), P(acts), P(tn), 1e-4, P(mbits), P(gpT2), B, P(parts), N0,
                                        N0, B, K, h, 1, st), (B // 256) * (h // 256)),
        "G4G5": (lambda: L.cc_wgrad_both_t(P(actsT), P(grT), P(W2), P(norms), P(colsum), 1e-4, P(gW), P(parts), P(gpT),
                                           P(xT), P(gW2), P(parts2), B, h, n, d, 1, st), 2 * (h // 256) * (K // 256)),
    }
    for name in which:
        fn, ntiles = calls[name]
        stamps = torch.zeros(ntiles * 12, device=dev, dtype=torch.int64)
        for _ in range(20):
            assert fn() == 0
        L.cc_debug_set_stamps(P(stamps))
        assert fn() == 0
        L.cc_debug_set_stamps(None)
        torch.cuda.synchronize()
        s = stamps.view(ntiles, 12).cpu().numpy().astype(np.int64)
        cyc = s[:, 4] - s[:, 0]
        wall_us = (s[:, 6] - s[:, 5]) * 0.01
        ghz = np.median(cyc / (wall_us * 1e3))
        us = lambda c: c / (ghz * 1e3)  # noqa: E731
        seg = {"prologue": us(s[:, 1] - s[:, 0]), "k_loop": us(s[:, 2] - s[:, 1]), "drain": us(s[:, 3] - s[:, 2]),
               "epilogue": us(s[:, 4] - s[:, 3]), "tile": us(s[:, 4] - s[:, 0])}
        if (s[:, 7] > 0).all():  # the LDS epilogue's own points: element work, direct stores, transposed stores
            seg.update({"epi_core": us(s[:, 7] - s[:, 3]), "epi_store": us(s[:, 8] - s[:, 7]),
                        "epi_store_t": us(s[:, 9] - s[:, 8]), "epi_return": us(s[:, 4] - s[:, 9])})
        if (s[:, 10] > 0).all():  # G1's fast core: element loop, mask / l0 stores, the barrier after it
            seg.update({"core_loop": us(s[:, 10] - s[:, 3]), "core_bits": us(s[:, 11] - s[:, 10]),
                        "core_sync": us(s[:, 7] - s[:, 11])})
        # static order: XCD x = t % 8 runs i = t // 8 on workgroup w = i % nwx, wave of tiles k = i // nwx
        nwx = 32
        t = np.arange(ntiles)
        x_, i_ = t % 8, t // 8
        w_, k_ = i_ % nwx, i_ // nwx
        gaps = []
        order = np.lexsort((k_, w_, x_))
        for a, b in zip(order[:-1], order[1:]):
            if x_[a] == x_[b] and w_[a] == w_[b]:
                gaps.append((s[b, 5] - s[a, 6]) * 0.01)
        t0 = s[:, 5].min()
        span = (s[:, 6].max() - t0) * 0.01
        print(f"== {name}: {ntiles} tiles, clock {ghz:.2f} GHz (s_memtime / wall), launch span {span:.1f} us "
              f"(first tile entry -> last tile end)")
        for k, v in seg.items():
            print(f"   {k:9s} median {np.median(v):7.2f} us  mean {np.mean(v):7.2f}  p10 {np.percentile(v, 10):7.2f}  "
                  f"p90 {np.percentile(v, 90):7.2f}")
        gaps = np.array(gaps)
        print(f"   gap to the workgroup's next tile: median {np.median(gaps):.2f} us mean {np.mean(gaps):.2f}")
        for k in range(int(k_.max()) + 1):
            m = k_ == k
            st0 = (s[m, 5] - t0) * 0.01
            print(f"   wave {k}: start {np.median(st0):7.1f} us (spread p10-p90 {np.percentile(st0, 10):7.1f}-"
                  f"{np.percentile(st0, 90):7.1f}), prologue {np.median(seg['prologue'][m]):5.2f} "
                  f"k_loop {np.median(seg['k_loop'][m]):6.2f} drain {np.median(seg['drain'][m]):5.2f} "
                  f"epilogue {np.median(seg['epilogue'][m]):5.2f}")


if __name__ == "__main__":
    main()
