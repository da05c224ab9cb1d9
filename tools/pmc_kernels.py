#!/usr/bin/env python3
"""Per-kernel PMC summary of a tools/prof_pmc.sh directory: one line per
kernel name (template arguments kept: e.g. each MHRS search round), the
per-dispatch averages of the counters and the derived ratios
(tools/pmc_summary.py's: VALU lane utilisation, FP64 share, wait share,
corrected HBM bytes).  usage: python3 tools/pmc_kernels.py <pmc dir> [substring]"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def main(d, sub=""):
    acc = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True)):
        per = defaultdict(lambda: defaultdict(float))
        for row in csv.DictReader(open(f)):
            k = row.get("Kernel_Name", "")
            if "pht::" not in k or sub not in k:
                continue
            k = re.sub(r"\(.*", "", k).replace("void ", "")
            per[(k, row["Counter_Name"])][row["Dispatch_Id"]] += float(row["Counter_Value"])
        for (k, name), disp in per.items():
            acc[k][name].extend(disp.values())
    out = {}
    for k, cs in sorted(acc.items()):
        avg = {n: sum(v) / len(v) for n, v in cs.items() if v}
        der = {"dispatches": max(len(v) for v in cs.values())}
        if "SQ_THREAD_CYCLES_VALU" in avg and avg.get("SQ_ACTIVE_INST_VALU"):
            der["valu_lane_utilization"] = avg["SQ_THREAD_CYCLES_VALU"] / (64.0 * avg["SQ_ACTIVE_INST_VALU"])
        if avg.get("SQ_INSTS_VALU"):
            f64 = sum(avg.get(c, 0.0) for c in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64",
                                               "SQ_INSTS_VALU_TRANS_F64"))
            der["fp64_share_of_valu"] = f64 / avg["SQ_INSTS_VALU"]
            der["salu_per_valu"] = avg.get("SQ_INSTS_SALU", 0.0) / avg["SQ_INSTS_VALU"]
        if avg.get("SQ_WAVE_CYCLES"):
            der["wait_any_share"] = avg.get("SQ_WAIT_ANY", 0.0) / avg["SQ_WAVE_CYCLES"]
        if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
            der["hbm_bytes_per_launch"] = 2.0 * avg["FETCH_SIZE"] * 1024 + avg["WRITE_SIZE"] * 1024
            der["hbm_write_bytes"] = avg["WRITE_SIZE"] * 1024
        out[k] = {"derived": der, "per_dispatch_avg": avg}
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
