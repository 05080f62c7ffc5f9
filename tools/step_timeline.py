"""One steady-state step's kernel timeline from a rocprofv3 kernel trace (csv): start / end offsets
from the step's prep kernel, duration, HW queue.  Usage: python tools/step_timeline.py TRACE.csv [step]"""
import csv
import sys


def main():
    tr = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    short = lambda n: n.split("(")[0].replace("void ", "").replace("cc::", "")[:60]  # noqa: E731
    starts = [i for i, r in enumerate(tr) if "prep_kernel" in r["Kernel_Name"]]
    a, b = starts[k], starts[k + 1]
    t0 = int(tr[a]["Start_Timestamp"])
    for r in tr[a:b + 1]:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        print(f"{s / 1e3:8.1f} {e / 1e3:8.1f} {(e - s) / 1e3:7.1f}  q{r['Queue_Id']}  {short(r['Kernel_Name'])}")


if __name__ == "__main__":
    main()
