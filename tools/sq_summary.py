"""Per-launch SQ counter summary of one kernel -> profiles/sq_<kernel>.json (read by bench.py's compute roofline).

Input: the per-kernel counter CSVs tools/pmc_extract.py --out writes for the two SQ passes of
tools/profile_round.sh. SQ_WAVE_CYCLES and SQ_ACTIVE_INST_* count quad-cycles (MI355X_MICROARCH.md:488).

Usage: python tools/sq_summary.py SQ1.csv SQ2.csv --kernel K --envs N --out profiles/sq_K.json
"""
import argparse
import csv
import json
import statistics


def per_dispatch(files, kernel):
    per = {}
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                if row.get("Kernel_Name") != kernel:
                    continue
                d = per.setdefault(row["Counter_Name"], {})
                d[row["Dispatch_Id"]] = d.get(row["Dispatch_Id"], 0.0) + float(row["Counter_Value"])
    return {k: statistics.mean(v.values()) for k, v in per.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--envs", type=int, required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--workload", default=None, help="bench config key when configs share the kernel (C4w)")
    a = ap.parse_args()
    m = per_dispatch(a.csv, a.kernel)
    out = {"kernel": a.kernel, "envs": a.envs, "workload": a.workload, "counters_mean_per_launch": m,
           "valu_insts_per_launch": m.get("SQ_INSTS_VALU"),
           "wave_cycles_per_launch": m.get("SQ_WAVE_CYCLES"),
           "valu_active_frac": (m["SQ_ACTIVE_INST_VALU"] / m["SQ_WAVE_CYCLES"])
           if m.get("SQ_WAVE_CYCLES") and "SQ_ACTIVE_INST_VALU" in m else None,
           "wait_frac": (m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"]) if m.get("SQ_WAVE_CYCLES") and "SQ_WAIT_ANY" in m
           else None,
           "lds_bank_conflict_per_lds_inst": (m["SQ_LDS_BANK_CONFLICT"] / m["SQ_INSTS_LDS"])
           if m.get("SQ_INSTS_LDS") and "SQ_LDS_BANK_CONFLICT" in m else None,
           # rocprofiler-sdk counter_defs.yaml VALUUtilization: active lanes per VALU instruction-cycle / 64 (the
           # third SQ pass holds SQ_THREAD_CYCLES_VALU alone: a counter in two passes would add up per dispatch id here)
           "valu_lane_utilization": (m["SQ_THREAD_CYCLES_VALU"] / (m["SQ_ACTIVE_INST_VALU"] * 64.0))
           if m.get("SQ_THREAD_CYCLES_VALU") and m.get("SQ_ACTIVE_INST_VALU") else None,
           "source": a.csv}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "counters_mean_per_launch"}))


if __name__ == "__main__":
    main()
