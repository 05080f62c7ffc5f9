"""One steady-state step's kernel timeline from a rocprofv3 kernel trace (csv): start / end offsets
from the step's prep kernel, duration, HW queue.  With the HIP API trace of the same run (rocprofv3
--hip-runtime-trace) each kernel also shows when the host made its launch call (same clock), so a kernel that
starts right after its launch call was waiting for the host.
Usage: python tools/step_timeline.py KERNEL_TRACE.csv [step] [HIP_API_TRACE.csv]"""
import csv
import sys


def main():
    tr = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    short = lambda n: n.split("(")[0].replace("void ", "").replace("cc::", "")[:60]  # noqa: E731
    starts = [i for i, r in enumerate(tr) if "prep_kernel" in r["Kernel_Name"]]
    a, b = starts[k], starts[k + 1]
    t0 = int(tr[a]["Start_Timestamp"])
    api = {}
    if len(sys.argv) > 3:
        api = {r["Correlation_Id"]: int(r["Start_Timestamp"]) for r in csv.DictReader(open(sys.argv[3]))}
    for r in tr[a:b + 1]:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        host = api.get(r.get("Correlation_Id"))
        hs = f" host {(host - t0) / 1e3:8.1f}" if host is not None else ""
        print(f"{s / 1e3:8.1f} {e / 1e3:8.1f} {(e - s) / 1e3:7.1f}  q{r['Queue_Id']}{hs}  {short(r['Kernel_Name'])}")


if __name__ == "__main__":
    main()
