"""GPU idle time a stream-ordering primitive inserts between two back-to-back kernels on one stream.
Run under `rocprofv3 --kernel-trace --output-format csv -d DIR -- python tools/event_cost.py`, then
`python tools/event_cost.py DIR/..._kernel_trace.csv`.  Patterns are separated by 20 ms idle."""
import glob
import os
import sys
import time

import torch

PATTERNS = ["none", "event record", "wait (done event, other stream)", "aux.wait_stream(main)",
            "record + host query", "pinned copy + record", "device-scope record", "device-scope wait_stream",
            "device-scope ping-pong (aux waits main, main waits aux)", "two event records",
            "pinned copy + record + record"]


def run():
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from crosscoder_amd import ops
    from crosscoder_amd import _hip as H
    dev = torch.device("cuda:0")
    src = torch.randn(4096, 4608, device=dev).to(torch.bfloat16)
    dst = torch.empty(4608, 4096, dtype=torch.bfloat16, device=dev)
    aux = torch.cuda.Stream()
    host = torch.empty(8, pin_memory=True)
    small = torch.zeros(8, device=dev)
    k = lambda: ops.transpose(src, out=dst)  # noqa: E731
    for _ in range(3):
        for p in PATTERNS:
            done = torch.cuda.Event()
            with torch.cuda.stream(aux):
                done.record(aux)
            torch.cuda.synchronize()
            time.sleep(0.02)
            for _ in range(20):
                k()
                if p == "event record":
                    torch.cuda.Event().record()
                elif p.startswith("wait"):
                    torch.cuda.current_stream().wait_event(done)
                elif p.startswith("aux.wait_stream"):
                    aux.wait_stream(torch.cuda.current_stream())
                elif p == "record + host query":
                    e = torch.cuda.Event()
                    e.record()
                    e.query()
                elif p == "device-scope record":
                    H.DeviceEvent().record()
                elif p == "device-scope wait_stream":
                    H.wait_stream(aux, torch.cuda.current_stream())
                elif p.startswith("device-scope ping-pong"):
                    H.wait_stream(aux, torch.cuda.current_stream())
                    with torch.cuda.stream(aux):
                        k()
                    H.wait_stream(torch.cuda.current_stream(), aux)
                elif p == "two event records":
                    torch.cuda.Event().record()
                    torch.cuda.Event().record()
                elif p == "pinned copy + record + record":
                    host.copy_(small, non_blocking=True)
                    torch.cuda.Event().record()
                    torch.cuda.Event().record()
                elif p.startswith("pinned"):
                    host.copy_(small, non_blocking=True)
                    torch.cuda.Event().record()
            torch.cuda.synchronize()


def analyze(path):
    import csv
    tr = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    tr = [r for r in tr if "transpose" in r["Kernel_Name"]]
    groups, cur = [], [tr[0]]
    for a, b in zip(tr, tr[1:]):
        if int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) > 5e6:
            groups.append(cur)
            cur = []
        cur.append(b)
    groups.append(cur)
    res = {}
    for gi, g in enumerate(groups):
        gaps = sorted(int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) for a, b in zip(g, g[1:]))
        res.setdefault(PATTERNS[gi % len(PATTERNS)], []).append(gaps[len(gaps) // 2] / 1e3)
    for p, v in res.items():
        print(f"{p:36s} median gap between kernels: {' '.join(f'{x:5.1f}' for x in v)} us")


if __name__ == "__main__":
    if len(sys.argv) > 1:
        analyze(sys.argv[1] if sys.argv[1].endswith(".csv") else glob.glob(sys.argv[1] + "/**/*kernel_trace.csv",
                                                                            recursive=True)[0])
    else:
        run()
