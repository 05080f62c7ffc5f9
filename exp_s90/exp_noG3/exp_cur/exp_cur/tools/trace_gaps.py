"""Per-step busy time vs wall span from a rocprofv3 kernel trace (csv): where the step goes."""
import csv
import sys
from collections import defaultdict

tr = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
short = lambda n: n.split("(")[0].replace("void ", "").replace("cc::", "")[:48]  # noqa: E731
# steps start at each prep_kernel launch
starts = [i for i, r in enumerate(tr) if "prep_kernel" in r["Kernel_Name"]]
steps = [(starts[k], starts[k + 1]) for k in range(len(starts) - 1)]
gaps = defaultdict(list)
busy_tot = span_tot = 0
for a, b in steps[2:]:
    span = int(tr[b]["Start_Timestamp"]) - int(tr[a]["Start_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tr[a:b])
    busy_tot += busy
    span_tot += span
    for i in range(a, b):
        g = int(tr[i + 1]["Start_Timestamp"]) - int(tr[i]["End_Timestamp"])
        gaps[short(tr[i]["Kernel_Name"]) + " -> " + short(tr[i + 1]["Kernel_Name"])].append(g)
n = len(steps) - 2
print(f"steps {n}: span {span_tot / n / 1e3:.1f} us/step, kernel busy {busy_tot / n / 1e3:.1f} us/step")
for k, v in sorted(gaps.items(), key=lambda kv: -sum(kv[1])):
    print(f"  gap {sum(v) / len(v) / 1e3:7.1f} us  {k}")
