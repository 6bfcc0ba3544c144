#!/usr/bin/env python3
"""HBM traffic per launch of the dominant kernel from rocprofv3 PMC passes.

  python scripts/pmc_traffic.py --fetch F.csv --write W.csv --kernel SUBSTR \
      [--calib-fetch CF.csv --calib-write CW.csv] --out profiles/rNN_traffic_<cfg>.json

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (rocprofv3 counter_collection.csv).  Each is
corrected by a factor measured with scripts/calib_stream (a known 1 GiB read + 1 GiB write at
the same access width, fp64 8 B/lane or fp32 4 B/lane), as MI355X_MICROARCH.md prescribes for
widths it does not calibrate.  Output: median corrected bytes per dispatch of the matching kernel,
per launch and per unit (--units-per-launch: the iterations one persistent dispatch runs).
"""
import argparse
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import provenance  # noqa: E402
import statistics


def per_kernel(path, counter, substr, skip=0):
    """The counter's value per dispatch of the kernel, in dispatch order, the first `skip`
    dispatches dropped (a bench's warm-up launches of a different iteration count)."""
    vals = []
    with open(path, newline="") as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] == counter and substr in row["Kernel_Name"]:
                vals.append((int(row["Dispatch_Id"]), float(row["Counter_Value"])))
    return [v for _, v in sorted(vals)[skip:]]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--kernel", required=True, help="substring of the kernel name")
    ap.add_argument("--calib-fetch")
    ap.add_argument("--calib-write")
    ap.add_argument("--calib-kernel", default="k_stream<double>")
    ap.add_argument("--config", default="")
    ap.add_argument("--units-per-launch", type=int, default=1,
                    help="iterations one dispatch runs (k_mcmc_scan: --steps of the bench); "
                         "bytes are reported per iteration, like bench.py's roofline")
    ap.add_argument("--out", required=True)
    ap.add_argument("--skip", type=int, default=0, help="drop the kernel's first N dispatches")
    ap.add_argument("--tree", help="tree.txt of the GPU session (the digest of the tree it ran)")
    a = ap.parse_args()
    fk = per_kernel(a.fetch, "FETCH_SIZE", a.kernel, a.skip)
    wk = per_kernel(a.write, "WRITE_SIZE", a.kernel, a.skip)
    if not fk or not wk:
        raise SystemExit(f"no dispatches of {a.kernel!r} in the PMC files")
    cf = cw = 1.0
    calib = None
    if a.calib_fetch and a.calib_write:
        gib = float(1 << 30)
        cfv = per_kernel(a.calib_fetch, "FETCH_SIZE", a.calib_kernel)
        cwv = per_kernel(a.calib_write, "WRITE_SIZE", a.calib_kernel)
        cf = gib / (statistics.median(cfv) * 1024.0)
        cw = gib / (statistics.median(cwv) * 1024.0)
        calib = {"kernel": a.calib_kernel, "fetch_factor": cf, "write_factor": cw,
                 "fetch_kib_raw": statistics.median(cfv), "write_kib_raw": statistics.median(cwv)}
    f_b = statistics.median(fk) * 1024.0 * cf / a.units_per_launch
    w_b = statistics.median(wk) * 1024.0 * cw / a.units_per_launch
    # per unit (an iteration of a persistent launch; 1 unit per launch otherwise) and per launch
    out = {"config": a.config, "kernel": a.kernel, "dispatches": [len(fk), len(wk)],
           "skipped": a.skip,
           "units_per_launch": a.units_per_launch,
           "fetch_bytes_per_unit": f_b, "write_bytes_per_unit": w_b,
           "traffic_bytes_per_unit": f_b + w_b,
           "traffic_bytes_per_launch": (f_b + w_b) * a.units_per_launch,
           "fetch_kib_raw_median": statistics.median(fk),
           "write_kib_raw_median": statistics.median(wk), "calibration": calib}
    provenance.stamp(out, digest=provenance.read_digest(a.tree) if a.tree else None)  # the tree measured
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
