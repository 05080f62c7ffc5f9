"""Per-kernel HBM traffic per launch from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

  python tools/pmc_traffic.py FETCH_DIR WRITE_DIR OUT.json [label]

FETCH_SIZE / WRITE_SIZE are in KiB.  gfx950 correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE
reports half the bytes of wide (16 B/lane) coalesced streaming reads -- every kernel of this step
reads that way (LDS-DMA 16 B/lane or 16-B vector loads) -- so fetch bytes = 2 x FETCH_SIZE x 1024;
write bytes = WRITE_SIZE x 1024 (exact for 16-B stores).  Counts include Infinity-Cache hits
(memory-side L2 requests), i.e. bytes that crossed the L2 -> fabric boundary.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("cc::", "").strip()
    return n


def per_kernel(d, counter):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                vals[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


def main():
    fdir, wdir, out = sys.argv[1:4]
    label = sys.argv[4] if len(sys.argv) > 4 else ""
    fetch, nf = per_kernel(fdir, "FETCH_SIZE")
    write, _ = per_kernel(wdir, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        fb = 2.0 * fetch.get(k, 0.0) * 1024
        wb = write.get(k, 0.0) * 1024
        kernels[k] = {"fetch_bytes": round(fb), "write_bytes": round(wb), "hbm_bytes": round(fb + wb),
                      "dispatches": nf.get(k, 0)}
    doc = {"label": label,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
                     "`python bench.py --steps 3 --warmup 1 --no-cpu-baseline`; mean per dispatch; "
                     "fetch = 2 x FETCH_SIZE KiB (gfx950 wide-read correction), write = WRITE_SIZE KiB",
           "kernels": kernels}
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    for k, v in kernels.items():
        if v["hbm_bytes"] > 1e6:
            print(f"{k[:60]:60s} fetch {v['fetch_bytes'] / 1e6:9.1f} MB  write {v['write_bytes'] / 1e6:8.1f} MB")


if __name__ == "__main__":
    main()
