"""Shrink a rocprofv3 --pmc output directory to the rows of our kernels (run on the GPU box, so the merged
gpurun_out/ stays small) and print per-kernel means of every counter.

Usage: python tools/pmc_extract.py DIR [--kernel ha_step_kernel] [--out FILE.csv] [--delete]
"""
import argparse
import csv
import glob
import os
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default="ha_step_kernel")
    ap.add_argument("--out", default=None)
    ap.add_argument("--delete", action="store_true")
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True)
    rows, header = [], None
    for fn in files:
        with open(fn) as f:
            r = csv.DictReader(f)
            header = r.fieldnames
            rows += [row for row in r if row.get("Kernel_Name", "") == a.kernel]
    per = {}
    for row in rows:
        per.setdefault(row["Counter_Name"], {}).setdefault(row["Dispatch_Id"], 0.0)
        per[row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
    for name, d in sorted(per.items()):
        vals = list(d.values())
        print(f"{a.kernel} {name:28s} mean {statistics.mean(vals):16.1f} over {len(vals)} dispatches")
    if a.out and header:
        with open(a.out, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=header)
            w.writeheader()
            w.writerows(rows)
    if a.delete:
        for fn in glob.glob(os.path.join(a.dir, "**", "*.csv"), recursive=True):
            os.remove(fn)


if __name__ == "__main__":
    main()
