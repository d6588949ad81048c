"""Per-kernel counter summary of one or more rocprofv3 --pmc pass directories.

    python pmc_kernel.py <kernel regex> <pass dir> [<pass dir> ...]

For every counter found, prints the mean per dispatch of the kernels whose name matches the regex (the first
dispatch of each kernel is dropped: it warms the caches), plus derived ratios when their inputs are present:
  mfma_busy      = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)   (tools/mfma_summary.py)
  wait_any / wait_inst / active_inst   = share of SQ_WAVE_CYCLES (disjoint buckets, MI355X_MICROARCH.md §PMC)
  lds_conflict   = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  per_mfma       = instruction counts per SQ_INSTS_MFMA
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def collect(dirs, pat):
    per = defaultdict(list)               # counter -> values, one per dispatch
    names = set()
    for d in dirs:
        seen = defaultdict(int)
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if not re.search(pat, r["Kernel_Name"]):
                    continue
                names.add(r["Kernel_Name"][:100])
                key = (r["Dispatch_Id"], r["Counter_Name"])
                seen[key] += 1
                per[(r["Counter_Name"], r["Dispatch_Id"])].append(float(r["Counter_Value"]))
    out = defaultdict(list)
    for (c, disp), v in per.items():
        out[c].append((int(disp), sum(v)))
    res = {}
    for c, lst in out.items():
        lst.sort()
        vals = [v for _, v in lst]
        if len(vals) > 1:
            vals = vals[1:]
        res[c] = sum(vals) / len(vals)
    return res, names


def main():
    pat, dirs = sys.argv[1], sys.argv[2:]
    res, names = collect(dirs, pat)
    for n in sorted(names):
        print("kernel:", n)
    for c in sorted(res):
        print(f"{c:32s} {res[c]:16.4g}")
    g = res.get("GRBM_GUI_ACTIVE")
    if g and "SQ_VALU_MFMA_BUSY_CYCLES" in res:
        print(f"{'mfma_busy':32s} {res['SQ_VALU_MFMA_BUSY_CYCLES'] / (g / 8 * 1024):16.4f}")
    w = res.get("SQ_WAVE_CYCLES")
    if w:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_MISC", "SQ_ACTIVE_INST_SCA"):
            if c in res:
                print(f"{c + '/wave_cycles':32s} {res[c] / w:16.4f}")
    if "SQ_LDS_IDX_ACTIVE" in res and "SQ_LDS_BANK_CONFLICT" in res:
        print(f"{'lds_conflict':32s} {res['SQ_LDS_BANK_CONFLICT'] / res['SQ_LDS_IDX_ACTIVE']:16.4f}")
    m = res.get("SQ_INSTS_MFMA")
    if m:
        for c in sorted(res):
            if c.startswith("SQ_INSTS_") and c != "SQ_INSTS_MFMA":
                print(f"{c + '/mfma':32s} {res[c] / m:16.4f}")


if __name__ == "__main__":
    main()
