#!/usr/bin/env python3
"""Average dispatch duration of one kernel from a rocprofv3 --kernel-trace run (bench.py prints
it beside its own HIP-event figure as roofline.kernel_avg_us_rocprof).

  python scripts/kstats_summary.py --trace gpurun_out/r04x/prof_c5/<pid>_kernel_trace.csv \
      --kernel 'k_block_pk<' --config c5 --skip 0 --out profiles/r04x_kstats_c5.json

--skip drops the kernel's first dispatches (the bench's warm-up launch of a persistent kernel
runs a different number of iterations than the timed ones); --units-per-launch gives the
iterations one timed dispatch runs, so the per-iteration time is reported too.  Falls back to
the --stats kernel_stats.csv average (every dispatch) when no trace is given.
"""
import argparse
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import provenance  # noqa: E402
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace")
    ap.add_argument("--stats")
    ap.add_argument("--kernel", required=True, help="substring of the kernel name")
    ap.add_argument("--config", required=True)
    ap.add_argument("--skip", type=int, default=0)
    ap.add_argument("--units-per-launch", type=int, default=1)
    ap.add_argument("--command", default="")
    ap.add_argument("--out", required=True)
    ap.add_argument("--tree", help="tree.txt of the GPU session (the digest of the tree it ran)")
    a = ap.parse_args()
    out = {"config": a.config, "kernel": a.kernel, "units_per_launch": a.units_per_launch,
           "command": a.command}
    if a.trace:
        d = []
        with open(a.trace, newline="") as f:
            for row in csv.DictReader(f):
                if a.kernel in row["Kernel_Name"]:
                    d.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"])))
        d.sort()
        us = [(e - s) * 1e-3 for s, e in d[a.skip:]]
        if not us:
            raise SystemExit(f"no dispatches of {a.kernel!r} after --skip {a.skip}")
        out.update({"source": a.trace, "dispatches": len(us), "skipped": a.skip,
                    "avg_us": statistics.fmean(us), "median_us": statistics.median(us),
                    "min_us": min(us), "max_us": max(us)})
    elif a.stats:
        with open(a.stats, newline="") as f:
            rows = [r for r in csv.DictReader(f) if a.kernel in r["Name"]]
        if not rows:
            raise SystemExit(f"no row for {a.kernel!r}")
        r = rows[0]
        out.update({"source": a.stats, "dispatches": int(r["Calls"]), "skipped": 0,
                    "avg_us": float(r["AverageNs"]) * 1e-3, "min_us": float(r["MinNs"]) * 1e-3,
                    "max_us": float(r["MaxNs"]) * 1e-3})
    else:
        raise SystemExit("--trace or --stats")
    out["avg_us_per_unit"] = out["avg_us"] / a.units_per_launch
    provenance.stamp(out, digest=provenance.read_digest(a.tree) if a.tree else None)  # the tree measured
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
