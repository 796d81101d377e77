"""Summarises rocprofv3 --pmc passes (counter_collection.csv) per kernel and launch shape (kernel name,
grid size): the mean of each counter over the dispatches, the mean dispatch duration, the effective
clock and the HBM bytes, plus these derived figures, each computed WITHIN one dispatch (the counters
of a pass and its timestamps come from the same dispatch, so no clock of another run enters):

* effective_clock_ghz = GRBM_GUI_ACTIVE / 8 XCDs / duration (MI355X_MICROARCH.md "DVFS give-back");
* valu_issue_frac = ((SQ_INSTS_VALU - SQ_ACTIVE_INST_VALU2) x 4 cycles / 1024 SIMDs) / (GRBM_GUI_ACTIVE
  / 8): the SIMD quad-cycles in which the dispatch's VALU instructions issue -- one per instruction (a
  wave64 instruction passes a 16-lane SIMD in 4 cycles; SQ_ACTIVE_INST_VALU, the hardware's own count,
  equals SQ_INSTS_VALU on these kernels) less the quad-cycles that issued two (SQ_ACTIVE_INST_VALU2) --
  over the dispatch's elapsed cycles: clock-free, <= 1;
* valu_issue_frac_4cyc: the same without the dual-issue correction (every instruction its own
  quad-cycle; above 1 where dual issue is frequent);
* valu_dual_issue_share = SQ_ACTIVE_INST_VALU2 / SQ_INSTS_VALU;
* valu_class_share: INT32 / INT64 / CVT / FMA_F64 ... instructions over SQ_INSTS_VALU;
* hbm_bytes = FETCH_SIZE x 2 (gfx950 tallies 128-B read requests at 64 B) + WRITE_SIZE, both KiB.

usage: pmc_summary.py <out.json> <pass_dir> [<pass_dir> ...]
"""
import collections
import csv
import glob
import json
import sys

SIMDS = 1024
ISSUE_CYCLES = 4.0
CLASSES = ("SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64", "SQ_INSTS_VALU_CVT", "SQ_INSTS_VALU_FMA_F64",
           "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_TRANS_F32")


def short(name):
    return name.split("(")[0].replace("void ", "")


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    # per (kernel, grid): counter -> values; per-dispatch derived values
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    durs = collections.defaultdict(list)
    fracs = collections.defaultdict(list)
    fracs4 = collections.defaultdict(list)
    clocks = collections.defaultdict(list)
    for d in dirs:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            disp = collections.defaultdict(dict)
            meta = {}
            for r in csv.DictReader(open(f)):
                key = (short(r["Kernel_Name"]), int(r.get("Grid_Size") or 0))
                did = (f, r["Dispatch_Id"])
                disp[did][r["Counter_Name"]] = disp[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                if r.get("Start_Timestamp"):
                    meta[did] = (key, int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
                else:
                    meta.setdefault(did, (key, 0))
            for did, cs in disp.items():
                key, dur = meta[did]
                for c, v in cs.items():
                    vals[key][c].append(v)
                if dur:
                    durs[key].append(dur)
                g = cs.get("GRBM_GUI_ACTIVE")
                if g and "SQ_INSTS_VALU" in cs:
                    fracs4[key].append(cs["SQ_INSTS_VALU"] * ISSUE_CYCLES / SIMDS / (g / 8))
                    busy = cs["SQ_INSTS_VALU"] - cs.get("SQ_ACTIVE_INST_VALU2", 0.0)
                    fracs[key].append(busy * ISSUE_CYCLES / SIMDS / (g / 8))
                if g and dur:
                    clocks[key].append(g / 8 / dur)
    summary = {}
    for (k, grid), cs in sorted(vals.items(), key=lambda kv: -sum(durs[kv[0]] or [0])):
        key = (k, grid)
        rec = {c: sum(v) / len(v) for c, v in cs.items()}
        rec["kernel"] = k
        rec["grid_size"] = grid
        rec["dispatches_per_pass"] = max(len(v) for v in cs.values())
        if durs[key]:
            rec["mean_duration_ns"] = sum(durs[key]) / len(durs[key])
        if clocks[key]:
            rec["effective_clock_ghz"] = sum(clocks[key]) / len(clocks[key])
        if fracs[key]:
            rec["valu_issue_frac"] = sum(fracs[key]) / len(fracs[key])
            rec["valu_issue_frac_range"] = [min(fracs[key]), max(fracs[key])]
            rec["valu_issue_frac_4cyc"] = sum(fracs4[key]) / len(fracs4[key])
        iv = rec.get("SQ_INSTS_VALU")
        if iv:
            if "SQ_ACTIVE_INST_VALU2" in rec:
                rec["valu_dual_issue_share"] = rec["SQ_ACTIVE_INST_VALU2"] / iv
            rec["valu_class_share"] = {c.replace("SQ_INSTS_VALU_", ""): rec[c] / iv for c in CLASSES if c in rec}
        if "FETCH_SIZE" in rec:
            rec["fetch_bytes_corrected"] = 2 * 1024 * rec["FETCH_SIZE"]
        if "WRITE_SIZE" in rec:
            rec["write_bytes"] = 1024 * rec["WRITE_SIZE"]
        if "fetch_bytes_corrected" in rec and "write_bytes" in rec:
            rec["hbm_bytes"] = rec["fetch_bytes_corrected"] + rec["write_bytes"]
        summary[f"{k} grid={grid}"] = rec
    doc = {"kernels": summary,
           "derived": "per-dispatch: valu_issue_frac = (SQ_INSTS_VALU - SQ_ACTIVE_INST_VALU2)*4/1024/(GRBM_GUI_ACTIVE/8); "
                      "effective_clock_ghz = GRBM_GUI_ACTIVE/8/duration; hbm_bytes = 2*FETCH_SIZE + WRITE_SIZE (KiB)"}
    json.dump(doc, open(out, "w"), indent=1)
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main()
