#!/usr/bin/env python3
"""Per-dispatch SQ counter summary of one kernel from rocprofv3 counter_collection CSVs.
usage: python scripts/sq_summary.py <kernel-substr> <units-per-dispatch> file.csv [...]"""
import collections
import csv
import sys

k, units = sys.argv[1], float(sys.argv[2])
d = collections.defaultdict(dict)
for f in sys.argv[3:]:
    for r in csv.DictReader(open(f)):
        if k in r["Kernel_Name"]:
            d[(f, r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
for key, v in d.items():
    w = v.get("SQ_WAVES")
    print(key[1], {a: "%.4g" % b for a, b in sorted(v.items())})
    if w and "SQ_WAVE_CYCLES" in v:
        wc = v["SQ_WAVE_CYCLES"]
        print("  per wave per unit: VALU insts %.0f, wave cycles %.0f; active-any %.2f wait-any %.2f "
              "wait-inst %.2f; VALU active / wave cycles %.2f" % (
                  v["SQ_INSTS_VALU"] / w / units, 4 * wc / w / units,
                  v["SQ_ACTIVE_INST_ANY"] / wc, v["SQ_WAIT_ANY"] / wc, v["SQ_WAIT_INST_ANY"] / wc,
                  v["SQ_ACTIVE_INST_VALU"] / wc))
