"""Summarises rocprofv3 CSV output (kernel stats + PMC passes) into a small
JSON committed under profiles/.  FETCH_SIZE is doubled for wide coalesced
streaming reads on gfx950 and WRITE_SIZE taken as is
(/opt/skills/guides/MI355X_MICROARCH.md, section HBM); both are reported in
KiB by rocprofv3 and converted to bytes here.

usage: profile_summary.py <stats_dir> <fetch_dir> <write_dir> <out.json> [bench_stats.log]

With the profiled bench's own output (its JSON line), "timed_region" holds the NTT pass kernels'
summed durations per transform over exactly the bench's timed steps (the last steps x passes
launches of the trace) next to that same run's ms_per_step: the kernels of a step cannot take
longer than the step, so the first is <= the second by construction of one run.
"""
import collections
import csv
import glob
import json
import sys


def load(pattern):
    files = glob.glob(pattern) or glob.glob(pattern.replace("/*", "/**/*"), recursive=True)
    return list(csv.DictReader(open(files[0]))) if files else []


def short(name):
    return name.split("(")[0].replace("void ", "")


def main():
    stats_dir, fetch_dir, write_dir, out = sys.argv[1:5]
    summary = {"kernels": {}, "pmc_bytes_per_launch": {}}
    for r in load(f"{stats_dir}/*kernel_stats.csv"):
        summary["kernels"][short(r["Name"])] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                                "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"]),
                                                "pct": float(r["Percentage"])}
    # Steady state: the median launch duration over the second half of each kernel's launches in
    # the kernel trace (the first launches include clock ramp-up and table builds).
    durs = collections.defaultdict(list)
    for r in sorted(load(f"{stats_dir}/*kernel_trace.csv"), key=lambda r: int(r["Start_Timestamp"])):
        durs[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for k, d in durs.items():
        if k in summary["kernels"] and d:
            tail = sorted(d[len(d) // 2:])
            summary["kernels"][k]["steady_median_ns"] = float(tail[len(tail) // 2])
    if len(sys.argv) > 5:
        line = [l for l in open(sys.argv[5]) if l.startswith('{"metric"')][-1]
        bench = json.loads(line)
        passes = int(bench["roofline"]["kernel"].split()[0])
        ntt = sorted((r for r in load(f"{stats_dir}/*kernel_trace.csv") if "ntt_pass_kernel" in r["Kernel_Name"]),
                     key=lambda r: int(r["Start_Timestamp"]))[-bench["steps"] * passes:]
        summary["timed_region"] = {
            "steps": bench["steps"], "launches": len(ntt),
            "kernel_ms_per_transform": sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in ntt)
            / bench["steps"] / 1e6,
            "bench_ms_per_step_same_run": bench["ms_per_step"]}
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in (fetch_dir, write_dir):
        for r in load(f"{d}/*counter_collection.csv"):
            per[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in per.items():
        rec = {}
        if "FETCH_SIZE" in cs:
            v = cs["FETCH_SIZE"]
            rec["fetch_bytes_corrected"] = 2 * 1024 * sum(v) / len(v)
        if "WRITE_SIZE" in cs:
            v = cs["WRITE_SIZE"]
            rec["write_bytes"] = 1024 * sum(v) / len(v)
        if rec:
            rec["hbm_bytes"] = rec.get("fetch_bytes_corrected", 0) + rec.get("write_bytes", 0)
            summary["pmc_bytes_per_launch"][k] = rec
    json.dump(summary, open(out, "w"), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
