"""Idle gap a cross-stream fork costs the forking stream (run under rocprofv3 --kernel-trace; read the trace with
--trace).  Per pattern, 20 repetitions of: main: spin 64 blocks 40 us [fork] ; side: spin 1 block 5 us after the
fork ; main: spin 64 blocks 40 us.  Forks: torch event record, device-scope event record (_hip.DeviceEvent), and
the event recorded by the first main launch itself (hipExtLaunchKernel stopEvent, cc_debug_spin_ev).
Usage: python tools/event_probe.py ; python tools/event_probe.py --trace TRACE.csv"""
import csv
import ctypes
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PATTERNS = ["torch event", "device event", "ext-launch stop event", "none"]


def run():
    import torch

    from crosscoder_amd import _hip, _lib
    L = _lib.load_debug()
    main = torch.cuda.current_stream()
    side = torch.cuda.Stream()
    sp = lambda st: ctypes.c_void_p(st.cuda_stream)  # noqa: E731
    for pat in PATTERNS:
        for _ in range(20):
            torch.cuda.synchronize()
            if pat == "ext-launch stop event":
                ev = _hip.DeviceEvent()
                assert L.cc_debug_spin_ev(64, 40_000, sp(main), ev._ev) == 0
                ev.wait(side)
            else:
                assert L.cc_debug_spin(64, 0, 40_000, sp(main)) == 0
                if pat == "torch event":
                    e = torch.cuda.Event()
                    e.record(main)
                    side.wait_event(e)
                elif pat == "device event":
                    _hip.DeviceEvent().record(main).wait(side)
            if pat != "none":
                assert L.cc_debug_spin(1, 0, 5_000, sp(side)) == 0
            assert L.cc_debug_spin(64, 0, 40_000, sp(main)) == 0
    torch.cuda.synchronize()


def trace(path):
    tr = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    tr = [r for r in tr if "debug_spin" in r["Kernel_Name"]]
    qmain = tr[0]["Queue_Id"]
    i = 0
    for pat in PATTERNS:
        gaps, side_after = [], []
        for _ in range(20):
            a = tr[i]
            side = None
            if pat != "none":
                side = next(r for r in tr[i + 1:i + 4] if r["Queue_Id"] != qmain)
            b = next(r for r in tr[i + 1:i + 4] if r["Queue_Id"] == qmain)
            gaps.append((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3)
            if side is not None:
                side_after.append((int(side["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3)
            i += 3 if pat != "none" else 2
        sa = f", side spin starts {statistics.median(side_after):6.2f} us after the first main spin ends " \
             f"(min {min(side_after):.2f})" if side_after else ""
        print(f"{pat:24s} main-stream gap median {statistics.median(gaps):6.2f} us{sa}")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--trace":
        trace(sys.argv[2])
    else:
        run()
