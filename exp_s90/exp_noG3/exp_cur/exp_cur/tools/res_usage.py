"""Summarise hipcc -Rpass-analysis=kernel-resource-usage output: kernel, VGPR, AGPR, spills, LDS."""
import re
import sys

txt = open(sys.argv[1] if len(sys.argv) > 1 else "crosscoder-model-diff-replication_amd/csrc/asm/gemm.hip.resource.txt").read()
for blk in re.split(r"remark: [^\n]*Function Name: ", txt)[1:]:
    name = blk.split()[0]
    get = lambda k: (re.search(k + r": (\d+)", blk) or [None, "?"])[1]  # noqa: E731
    lds = get(r"LDS Size \[bytes/block\]")
    print(f"{name[:60]:60s} vgpr {get('VGPRs'):>4} agpr {get('AGPRs'):>3} vspill {get('VGPRs Spill'):>3} "
          f"sspill {get('SGPRs Spill'):>3} lds {lds:>6}")
