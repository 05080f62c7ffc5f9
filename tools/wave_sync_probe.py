"""Probe for VERDICT r03 item 4 (G4G5's fetch above its L2 panel floor): the dual weight-gradient launch
(cc_wgrad_both_t, config-2 shapes, static tile order) with and without per-XCD wave synchronisation
(cc_debug_set_wave_sync: every workgroup of an XCD finishes its tile of wave k before any starts wave k + 1,
so the 32 concurrent tiles that share 4 A and 8 B panels stream them at the same K position).

  python tools/wave_sync_probe.py          interleaved timing of both forms + bit-identity of their outputs
  python tools/wave_sync_probe.py 0|1      20 launches of one form only (for rocprofv3 --pmc FETCH_SIZE passes)
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import crosscoder_amd  # noqa: F401,E402
from crosscoder_amd import _lib  # noqa: E402

B, n, d, h = 4096, 2, 2304, 16384
K = n * d
PEAK = 2.5e3  # TF/s, dense bf16


def main():
    L = _lib.load_debug()
    dev = torch.device("cuda:0")
    bf = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    acts = torch.relu(torch.randn(B, h, device=dev, generator=g)).to(bf)
    g_recon = (torch.randn(B, K, device=dev, generator=g) * 1e-3).to(bf)
    g_pre = (torch.randn(B, h, device=dev, generator=g) * 1e-3).to(bf)
    x = torch.randn(B, K, device=dev, generator=g).to(bf)
    W2 = (torch.randn(h, K, device=dev, generator=g) * 0.02).to(bf)
    actsT, grT, gpT, xT = acts.t().contiguous(), g_recon.t().contiguous(), g_pre.t().contiguous(), x.t().contiguous()
    norms = torch.ones(h, n, device=dev)
    colsum = torch.ones(h, device=dev)
    gW = torch.empty(h, K, device=dev, dtype=bf)
    gW2 = torch.empty(K, h, device=dev, dtype=bf)
    parts = torch.empty(1 << 20, device=dev)
    parts2 = torch.empty(1 << 20, device=dev)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def run(mode):
        L.cc_debug_set_wave_sync(mode)
        rc = L.cc_wgrad_both_t(P(actsT), P(grT), P(W2), P(norms), P(colsum), 1e-4, P(gW), P(parts), P(gpT), P(xT),
                               P(gW2), P(parts2), B, h, n, d, 1, st)
        assert rc == 0, rc

    if len(sys.argv) > 1:
        mode = int(sys.argv[1])
        for _ in range(20):
            run(mode)
        torch.cuda.synchronize()
        L.cc_debug_set_wave_sync(0)
        print(f"wave_sync={mode}: 20 launches done")
        return

    outs = {}
    for mode in (0, 1):
        run(mode)
        torch.cuda.synchronize()
        outs[mode] = (gW.clone(), gW2.clone(), parts[:4096].clone(), parts2[:4096].clone())
    same = all(torch.equal(a, b) for a, b in zip(outs[0], outs[1]))
    print(f"outputs bit-identical across forms: {same}")
    flop = 2 * 2.0 * B * K * h
    res = {0: [], 1: []}
    for _ in range(6):
        for mode in (0, 1):
            for _ in range(2):
                run(mode)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                run(mode)
            e.record()
            torch.cuda.synchronize()
            res[mode].append(s.elapsed_time(e) / 10)
    L.cc_debug_set_wave_sync(0)
    for mode, ts in res.items():
        ts.sort()
        med = ts[len(ts) // 2]
        print(f"G4G5 dual (cc_wgrad_both_t, static order) wave_sync={mode}: median {med * 1e3:7.1f} us "
              f"min {ts[0] * 1e3:7.1f} us  {flop / med / 1e9:7.1f} TF/s ({flop / med / 1e9 / PEAK * 100:4.1f}% of dense peak)"
              f"  (includes a 32 B memset launch when 1)")
    if not same:
        sys.exit(1)


if __name__ == "__main__":
    main()
