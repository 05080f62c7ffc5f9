"""GPU idle time between back-to-back kernels on ONE stream, by what precedes / follows a GEMM.
Run under `rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python tools/gap_probe.py`, then
`python tools/gap_probe.py DIR/.../run_kernel_trace.csv`.  Each pattern is a repeated sequence of launches
(config-2 G3 = cc_dacts_bwd_t, G1 = cc_encode_fwd_t, the W_dec^T transpose as a streaming kernel, a 1-block
tiny kernel), separated by 20 ms of idle; the report prints the median gap for every (previous, next) pair."""
import glob
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PATTERNS = {
    "G3 G3": ["G3", "G3"],
    "G1 G1": ["G1", "G1"],
    "T G3": ["T", "G3"],
    "tiny G3": ["tiny", "G3"],
    "tiny G1": ["tiny", "G1"],
    "G3 tiny tiny": ["G3", "tiny", "tiny"],
    "T tiny": ["T", "tiny"],
    "G1 T": ["G1", "T"],
}


def run():
    import ctypes

    sys.path.insert(0, ROOT)
    import crosscoder_amd  # noqa: F401
    from crosscoder_amd import _lib

    L = _lib.load()
    dev = torch.device("cuda:0")
    bf = torch.bfloat16
    B, n, d, h = 4096, 2, 2304, 16384
    K = n * d
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(B, K, device=dev, generator=g).to(bf)
    W = (torch.randn(h, K, device=dev, generator=g) * 0.02).to(bf)
    b_enc = torch.zeros(h, device=dev, dtype=bf)
    acts = torch.relu(torch.randn(B, h, device=dev, generator=g)).to(bf)
    actsT = torch.empty(h, B, device=dev, dtype=bf)
    g_recon = (torch.randn(B, K, device=dev, generator=g) * 1e-3).to(bf)
    gpT = torch.empty(h, B, device=dev, dtype=bf)
    WT = torch.empty(K, h, device=dev, dtype=bf)
    tn = torch.ones(h, device=dev)
    parts = torch.empty(1 << 22, device=dev)
    mbits = torch.zeros(B * h // 32 + 4096, device=dev, dtype=torch.int32)
    small = torch.zeros(64, device=dev)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    k = {
        "G1": lambda: L.cc_encode_fwd_t(P(x), P(W), P(b_enc), P(tn), P(acts), P(actsT), 1, P(parts), P(parts),
                                        P(parts), P(mbits), B, K, h, 1, st),
        "G3": lambda: L.cc_dacts_bwd_t(P(g_recon), P(W), P(acts), P(tn), 1e-4, P(mbits), P(gpT), B, P(parts), B, K,
                                       h, 1, st),
        "T": lambda: L.cc_transpose_b16(P(W), h, K, K, P(WT), h, st),
        "tiny": lambda: small.add_(1.0),
    }
    for f in k.values():
        r = f()
        assert isinstance(r, torch.Tensor) or r == 0, r
    torch.cuda.synchronize()
    for _ in range(3):
        for name, seq in PATTERNS.items():
            torch.cuda.synchronize()
            time.sleep(0.02)
            for _ in range(6):
                for s in seq:
                    k[s]()
    torch.cuda.synchronize()
    print("done")


def report(csv_path):
    import csv

    rows = []
    with open(csv_path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()

    def short(nm):
        if "gemm_pp_kernel<true, true, 3" in nm:
            return "G3"
        if "gemm_pp_kernel<true, true, 1" in nm:
            return "G1"
        if "transpose" in nm:
            return "T"
        if "elementwise" in nm or "add" in nm.lower():
            return "tiny"
        return nm[:30]

    gaps = {}
    for (s0, e0, n0), (s1, e1, n1) in zip(rows, rows[1:]):
        gap = (s1 - e0) / 1e3
        if gap > 1000:  # the 20 ms separators
            continue
        gaps.setdefault((short(n0), short(n1)), []).append(gap)
    durs = {}
    for s, e, nm in rows:
        durs.setdefault(short(nm), []).append((e - s) / 1e3)
    for key, v in sorted(gaps.items()):
        v.sort()
        print(f"{key[0]:>5s} -> {key[1]:<5s} n={len(v):3d} median gap {v[len(v)//2]:7.1f} us  min {v[0]:7.1f}  "
              f"max {v[-1]:7.1f}")
    for key, v in sorted(durs.items()):
        v.sort()
        print(f"duration {key:>5s} median {v[len(v)//2]:8.1f} us")


if __name__ == "__main__":
    if len(sys.argv) > 1:
        for p in sys.argv[1:]:
            for f in glob.glob(p) if "*" in p else [p]:
                report(f)
    else:
        run()
