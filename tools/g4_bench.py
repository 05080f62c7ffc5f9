"""Experiment: the 4-wave 128x128-per-wave GEMM (tools/exp/g4w.hip -> tools/exp/libg4w.so) against
hipBLASLt and the product's G1 kernel on the same operands, interleaved; plus a correctness check.
Usage: python tools/g4_bench.py [path/to/libg4w.so ...]"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import crosscoder_amd  # noqa: F401,E402
from crosscoder_amd import ops  # noqa: E402

PEAK = 256 * 2.4e9 * 4096 / 1e12


def load(path):
    lib = ctypes.CDLL(path)
    lib.g4_gemm_bf16.restype = ctypes.c_int
    lib.g4_gemm_bf16.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int64] * 6 + [ctypes.c_void_p]
    return lib


def main():
    paths = sys.argv[1:] or [os.path.join(ROOT, "tools", "exp", "libg4w.so")]
    libs = [(os.path.basename(p), load(p)) for p in paths]
    dev = torch.device("cuda:0")
    bf = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    r = lambda *s, sc=1.0: (torch.randn(*s, device=dev, generator=g) * sc).to(bf)  # noqa: E731
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    shapes = {"G1/G3 4096x16384x4608": (4096, 16384, 4608), "G4/G5 16384x4608x4096": (16384, 4608, 4096)}
    for sname, (M, N, K) in shapes.items():
        A, Bm = r(M, K), r(N, K, sc=0.02)
        C = torch.empty(M, N, device=dev, dtype=bf)
        ref = torch.matmul(A, Bm.t())
        cases = {"hipBLASLt": lambda: torch.matmul(A, Bm.t(), out=C)}
        if sname.startswith("G1"):
            b = torch.zeros(N, device=dev, dtype=bf)
            acts = torch.empty(M, N, device=dev, dtype=bf)
            cases["ours G1 encode (8-wave pp)"] = lambda: ops.encode_fwd(A, Bm, b, acts, False)
        for name, L in libs:
            C2 = torch.empty(M, N, device=dev, dtype=bf)
            rc = L.g4_gemm_bf16(P(A), P(Bm), P(C2), M, N, K, K, K, N, st)
            assert rc == 0, rc
            torch.cuda.synchronize()
            err = ((C2.float() - ref.float()).norm() / ref.float().norm()).item()
            print(f"{sname} {name}: rel err vs hipBLASLt {err:.2e}", flush=True)
            assert err < 1e-2 or "nostore" in name or name.endswith("ns.so")  # (timing-only builds store nothing)
            cases[name] = (lambda L=L, C2=C2: L.g4_gemm_bf16(P(A), P(Bm), P(C2), M, N, K, K, K, N, st))
        res = {k: [] for k in cases}
        for _ in range(3):
            for fn in cases.values():
                fn()
        torch.cuda.synchronize()
        for _ in range(6):
            for name, fn in cases.items():
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(10):
                    fn()
                e.record()
                torch.cuda.synchronize()
                res[name].append(s.elapsed_time(e) / 10)
        flop = 2.0 * M * N * K
        for name, ts in res.items():
            ts.sort()
            med = ts[len(ts) // 2]
            print(f"{sname} {name:32s} median {med * 1e3:7.1f} us  min {ts[0] * 1e3:7.1f} us  "
                  f"{flop / med / 1e9:7.1f} TF/s ({flop / med / 1e9 / PEAK * 100:4.1f}% of peak)", flush=True)


if __name__ == "__main__":
    main()
