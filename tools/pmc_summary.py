"""Summarises rocprofv3 --pmc passes (counter_collection.csv) per kernel: the mean of each counter
over the kernel's dispatches, the mean dispatch duration, the effective clock
(GRBM_GUI_ACTIVE / 8 XCDs / duration, MI355X_MICROARCH.md "DVFS give-back") and the HBM bytes
(FETCH_SIZE x 2 for wide coalesced reads on gfx950 + WRITE_SIZE, both KiB).

usage: pmc_summary.py <out.json> <pass_dir> [<pass_dir> ...]
"""
import collections
import csv
import glob
import json
import sys


def short(name):
    return name.split("(")[0].replace("void ", "")


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    durs = collections.defaultdict(list)
    for d in dirs:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            seen = set()
            for r in csv.DictReader(open(f)):
                k = short(r["Kernel_Name"])
                vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                key = (f, r["Dispatch_Id"])
                if key not in seen and r.get("Start_Timestamp"):
                    seen.add(key)
                    durs[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    summary = {}
    for k, cs in vals.items():
        rec = {c: sum(v) / len(v) for c, v in cs.items()}
        rec["dispatches_per_pass"] = max(len(v) for v in cs.values())
        if durs[k]:
            rec["mean_duration_ns"] = sum(durs[k]) / len(durs[k])
        if "GRBM_GUI_ACTIVE" in rec and rec.get("mean_duration_ns"):
            rec["effective_clock_ghz"] = rec["GRBM_GUI_ACTIVE"] / 8 / rec["mean_duration_ns"]
        if "FETCH_SIZE" in rec:
            rec["fetch_bytes_corrected"] = 2 * 1024 * rec["FETCH_SIZE"]
        if "WRITE_SIZE" in rec:
            rec["write_bytes"] = 1024 * rec["WRITE_SIZE"]
        summary[k] = rec
    json.dump({"kernels": summary}, open(out, "w"), indent=1)
    print(json.dumps({"kernels": summary}, indent=1))


if __name__ == "__main__":
    main()
