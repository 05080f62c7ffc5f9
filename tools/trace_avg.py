"""Steady-state per-step averages from a rocprofv3 kernel trace of bench.py: for the last N steps (prep kernel to
prep kernel; the timed steps) the mean step span, each kernel's mean start / end offset and duration in the step
(by launch position), and the compute stream's idle time.  Usage: python tools/trace_avg.py TRACE.csv [N]"""
import csv
import statistics
import sys


def main():
    tr = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    short = lambda s: s.split("(")[0].replace("void ", "").replace("cc::", "")[:52]  # noqa: E731
    starts = [i for i, r in enumerate(tr) if "prep_kernel" in r["Kernel_Name"]]
    n = min(n, len(starts) - 1)  # (consecutive prep launches: n + 1 of them bound n steps)
    steps = list(zip(starts[-n - 1:-1], starts[-n:]))
    spans, rows, idle = [], {}, []
    for a, b in steps:
        t0 = int(tr[a]["Start_Timestamp"])
        spans.append((int(tr[b]["Start_Timestamp"]) - t0) / 1e3)
        seen = {}
        busy_end, gap = t0, 0.0
        for r in tr[a:b]:
            k = (short(r["Kernel_Name"]), r["Queue_Id"])
            seen[k] = seen.get(k, 0) + 1
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            rows.setdefault(k + (seen[k],), []).append(((s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3))
            if r["Queue_Id"] == tr[a]["Queue_Id"]:
                gap += max(0, s - busy_end) / 1e3
                busy_end = max(busy_end, e)
        gap += max(0, int(tr[b]["Start_Timestamp"]) - busy_end) / 1e3
        idle.append(gap)
    print(f"# {len(steps)} steps: span mean {statistics.mean(spans):.1f} us, median {statistics.median(spans):.1f}, "
          f"min {min(spans):.1f}, max {max(spans):.1f}; compute-stream idle mean {statistics.mean(idle):.1f} us")
    print("#   start     end    dur  queue  kernel (means over the steps)")
    for k, v in sorted(rows.items(), key=lambda kv: statistics.mean(x[0] for x in kv[1])):
        if len(v) < len(steps) // 2:
            continue
        print(f"{statistics.mean(x[0] for x in v):8.1f} {statistics.mean(x[1] for x in v):8.1f} "
              f"{statistics.mean(x[2] for x in v):7.1f}  q{k[1]}  {k[0]}")


if __name__ == "__main__":
    main()
