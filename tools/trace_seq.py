"""Kernel sequence of the last `--window-ms` of a rocprofv3 --kernel-trace CSV: start (relative), duration
and the gap since the previous kernel ended, one line per kernel (for finding launch-bound stretches).

    python tools/trace_seq.py run_kernel_trace.csv [--window-ms 1.5]
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--window-ms", type=float, default=1.5)
    a = ap.parse_args()
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:70])
                  for r in csv.DictReader(open(a.csv)))
    end = rows[-1][1]
    rows = [x for x in rows if x[0] >= end - a.window_ms * 1e6]
    t0, prev = rows[0][0], rows[0][0]
    for s, e, k in rows:
        print(f"{(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f}  gap {(s - prev) / 1e3:7.1f}  {k}")
        prev = e


if __name__ == "__main__":
    main()
