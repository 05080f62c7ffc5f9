"""G3 and G4G5 (config-2 shapes) alone and with CUs held by another stream's kernel, static vs dynamic tile order.

A spin kernel of N workgroups x 512 threads, each holding 96 KB of LDS (no GEMM workgroup fits beside one), runs
for T us on a second stream, enqueued just before the GEMM: a stand-in for RCCL's all-reduce kernel beside G3 in
the latent-sharded step, or any side-stream kernel.  Timing: HIP events around the GEMM launch on its stream.
Usage: python tools/contention_probe.py [reps]   (test-only debug library: it carries the spin kernel)"""
import ctypes
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crosscoder_amd import _lib, ops  # noqa: E402

B, n, d, h = 4096, 2, 2304, 16384
K = n * d


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda:0")
    L = _lib.load_debug()
    bf = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(B, K, device=dev, generator=g).to(bf)
    W = (torch.randn(h, K, device=dev, generator=g) * 0.02).to(bf)
    acts = torch.relu(torch.randn(B, h, device=dev, generator=g)).to(bf)
    g_recon = (torch.randn(B, K, device=dev, generator=g) * 1e-3).to(bf)
    tn = torch.ones(h, device=dev)
    inv = torch.ones(h, n, device=dev)
    colsum = torch.ones(h, device=dev)
    actsT, grT, xT = acts.t().contiguous(), g_recon.t().contiguous(), x.t().contiguous()
    gpT = torch.empty(h, B, device=dev, dtype=bf)
    gpart = torch.empty(ops.col_part_rows(B), h, device=dev)
    mbits = torch.empty(ops.mask_bits_words(B, h), device=dev, dtype=torch.int32)
    ops.encode_fwd_t(x, W, torch.zeros(h, device=dev, dtype=bf), acts.clone(), torch.empty_like(actsT), True,
                     mask_bits=mbits)
    gW, gW2 = torch.empty(h, K, device=dev, dtype=bf), torch.empty(h, K, device=dev, dtype=bf)
    nw = ops.wgrad_parts(h, K, bf)
    sq = torch.zeros(2 * nw + ops.reduce_parts(h) + ops.reduce_parts(K), device=dev)
    off = [0, nw, 2 * nw, 2 * nw + ops.reduce_parts(h), sq.numel()]
    gbe, gbd = torch.empty(h, device=dev, dtype=bf), torch.empty(K, device=dev, dtype=bf)
    lcol = torch.randn(ops.col_part_rows(B), K, device=dev) * 1e-3
    clip = torch.empty(8, device=dev)
    tail = torch.zeros(1, device=dev, dtype=torch.int32)
    tsum = torch.empty(ops.wgrad_tile_sums(h, K), device=dev)
    ctr = torch.zeros(2, ops.TILE_CTR_WORDS, device=dev, dtype=torch.int32)
    hog = torch.cuda.Stream(device=dev)

    def g3(c):
        ops.dacts_bwd_t(g_recon, W, acts, tn, 1e-4, gpT, colsum_part=gpart, mask_bits=mbits, tile_ctr=c)

    def g45(c):
        ops.wgrad_both_clip_t(actsT, grT, W, inv, colsum, 1e-4, gW, sq[off[1]:off[2]], gpT, xT, gW2, sq[off[0]:off[1]],
                              n, d, gpart, gbe, sq[off[2]:off[3]], lcol, gbd, sq[off[3]:off[4]], sq, off, 1.0, True, clip,
                              tail, tsum, tile_ctr=c)

    with _lib.debug_library():
        cases = [(name, fn, mode, blocks, us) for name, fn, k in (("G3", g3, 0), ("G4G5", g45, 1))
                 for mode in ("static", "dynamic") for blocks, us in ((0, 0), (16, 200), (32, 200))]
        times = {c[:2] + c[2:]: [] for c in cases}
        for _ in range(reps + 1):
            for name, fn, mode, blocks, us in cases:
                c = ctr[0 if name == "G3" else 1] if mode == "dynamic" else None
                torch.cuda.synchronize()
                main = torch.cuda.current_stream(dev)
                if blocks:
                    ops.check(L.cc_debug_spin(blocks, 96 * 1024, us * 1000, ctypes.c_void_p(hog.cuda_stream)))
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record(main)
                fn(c)
                e.record(main)
                torch.cuda.synchronize()
                times[(name, fn, mode, blocks, us)].append(s.elapsed_time(e) * 1e3)
        assert not bool(ctr.any())
        print(f"# {reps} reps after 1 warm-up, median us (min-max); spin: N workgroups x 96 KB LDS for T us on another stream")
        for (name, fn, mode, blocks, us), v in times.items():
            v = v[1:]
            print(f"{name:5s} {mode:8s} hold {blocks:2d} CUs {us:3d} us: {statistics.median(v):7.1f} "
                  f"({min(v):.1f}-{max(v):.1f})")


if __name__ == "__main__":
    main()
