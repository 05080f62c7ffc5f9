"""Summarise rocprofv3 --pmc csv passes per kernel (mean over dispatches)."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "p*", "pmc_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        short = name.split("(")[0].replace("void ", "").replace("cc::", "")
        if "gemm_kernel" in name:
            short = "gemm" + name[name.index("<"):name.index(">") + 1]
        vals[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
keys = ["SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "GRBM_GUI_ACTIVE",
        "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_MFMA", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_WAIT_INST_LDS",
        "FETCH_SIZE", "WRITE_SIZE", "TCC_HIT_sum", "TCC_MISS_sum"]
for k, d in sorted(vals.items()):
    m = {c: sum(v) / len(v) for c, v in d.items()}
    if "gemm" not in k and "adam" not in k:
        continue
    print(k)
    for c in keys:
        if c in m:
            print(f"   {c:26s} {m[c]:16.4g}")
    if "SQ_WAVE_CYCLES" in m:
        w = m["SQ_WAVE_CYCLES"]
        print(f"   wait_any {m['SQ_WAIT_ANY']/w:.2f} wait_inst {m['SQ_WAIT_INST_ANY']/w:.2f} active {m['SQ_ACTIVE_INST_ANY']/w:.2f}")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
        print(f"   mfma_busy/(gui_active*256CU/8xcd) {m['SQ_VALU_MFMA_BUSY_CYCLES']/(m['GRBM_GUI_ACTIVE']/8*256*4):.3f}")
    if "FETCH_SIZE" in m:
        print(f"   fetch MB (x2 gfx950 corr) {2*m['FETCH_SIZE']*1024/1e6:.1f}   write MB {m.get('WRITE_SIZE',0)*1024/1e6:.1f}")
