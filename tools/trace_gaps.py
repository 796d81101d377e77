"""Timeline of a rocprofv3 --kernel-trace CSV: per-kernel totals and the idle gaps between
consecutive kernels (the GPU waiting on the host), for the last `--window-ms` of the trace.

    python tools/trace_gaps.py run_kernel_trace.csv [--window-ms 25] [--top 25]
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--window-ms", type=float, default=25.0)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(a.csv)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]))
    rows.sort()
    end = rows[-1][1]
    rows = [x for x in rows if x[0] >= end - a.window_ms * 1e6]
    t0 = rows[0][0]
    busy = collections.defaultdict(float)
    count = collections.Counter()
    gaps = []
    last_end = rows[0][0]
    for s, e, k in rows:
        busy[k] += (e - s) / 1e6
        count[k] += 1
        if s > last_end:
            gaps.append(((s - last_end) / 1e6, (last_end - t0) / 1e6, k))
        last_end = max(last_end, e)
    span = (last_end - t0) / 1e6
    print(f"window {span:.3f} ms, kernels {len(rows)}, busy {sum(busy.values()):.3f} ms, "
          f"idle {sum(g[0] for g in gaps):.3f} ms")
    for k, v in sorted(busy.items(), key=lambda x: -x[1])[: a.top]:
        print(f"  {v:8.3f} ms  {count[k]:4d}x  {k[:90]}")
    print("largest gaps (ms, at ms, next kernel):")
    for g in sorted(gaps, reverse=True)[:12]:
        print(f"  {g[0]:7.3f} at {g[1]:8.3f}  {g[2][:80]}")


if __name__ == "__main__":
    main()
