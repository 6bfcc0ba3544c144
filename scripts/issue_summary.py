#!/usr/bin/env python3
"""Issue-side roofline of one kernel from two rocprofv3 SQ-counter passes (bench.py reads the
output as roofline.issue / roofline.bound).

  python scripts/issue_summary.py --kernel k_mcmc_resident_pc --config c2 --iters 20 \
      --blocks 1024 --steps-per-block 500 --simds 1024 \
      --csv profiles/r02s/c2_sq1_counter_collection.csv profiles/r02s/c2_sq2_counter_collection.csv \
      --out profiles/r02s_issue_c2.json

SQ_WAVE_CYCLES / SQ_ACTIVE_INST_* / SQ_WAIT_* count quad-cycles summed over waves
(MI355X_MICROARCH.md, PMC units); SQ_INSTS_* count wave-instructions.  Per dispatch, then the
median over dispatches:
  valu_active_frac  = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES   (one wave's VALU-issue share)
  simd_valu_busy    = valu_active_frac × waves per SIMD        (share of a SIMD's cycles with a
                                                                VALU instruction issuing)
  wait_any_frac     = SQ_WAIT_ANY / SQ_WAVE_CYCLES
"""
import argparse
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import provenance  # noqa: E402
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--config", required=True)
    ap.add_argument("--iters", type=float, required=True, help="iterations per dispatch")
    ap.add_argument("--blocks", type=int, required=True)
    ap.add_argument("--steps-per-block", type=int, required=True)
    ap.add_argument("--simds", type=int, default=1024)
    ap.add_argument("--command", default="")
    ap.add_argument("--bound", default="valu-latency")
    ap.add_argument("--limiter", default="")
    ap.add_argument("--csv", nargs="+", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--skip", type=int, default=0, help="drop the kernel's first N dispatches")
    ap.add_argument("--tree", help="tree.txt of the GPU session (the digest of the tree it ran)")
    a = ap.parse_args()
    disp = collections.defaultdict(dict)
    for f in a.csv:
        for r in csv.DictReader(open(f)):
            if a.kernel in r["Kernel_Name"]:
                disp[(f, r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    # join the passes dispatch by dispatch (same command, same dispatch order)
    by_id = collections.defaultdict(dict)
    for (f, did), v in disp.items():
        by_id[did].update(v)
    for did in sorted(by_id, key=int)[:a.skip]:  # warm-up dispatches of another shape
        del by_id[did]
    rows = []
    for did, v in by_id.items():
        if "SQ_WAVES" not in v:
            continue
        # the FMA counter of the kernel's own precision, None when that pass did not collect it
        # (an F32 count of an fp64 kernel is not its FMA count)
        fp32 = "float" in a.kernel or "IfE" in a.kernel
        fma = v.get("SQ_INSTS_VALU_FMA_F32" if fp32 else "SQ_INSTS_VALU_FMA_F64")
        w, wc, n = v["SQ_WAVES"], v["SQ_WAVE_CYCLES"], a.iters
        wps = w / a.simds
        rows.append({
            "waves": w,
            "waves_per_simd": wps,
            "valu_insts_per_wave_iteration": v["SQ_INSTS_VALU"] / w / n,
            "valu_insts_per_block_iteration": v["SQ_INSTS_VALU"] / a.blocks / n,
            "valu_insts_per_step": v["SQ_INSTS_VALU"] / a.blocks / n / a.steps_per_block,
            "fma_per_block_iteration": None if fma is None else fma / a.blocks / n,
            "lds_insts_per_block_iteration": v["SQ_INSTS_LDS"] / a.blocks / n if "SQ_INSTS_LDS" in v else None,
            "wave_cycles_per_iteration": 4 * wc / w / n,
            "valu_active_frac": v["SQ_ACTIVE_INST_VALU"] / wc,
            "simd_valu_busy": v["SQ_ACTIVE_INST_VALU"] / wc * wps,
            "wait_any_frac": v["SQ_WAIT_ANY"] / wc,
            "lds_wait_frac": v["SQ_WAIT_INST_LDS"] / wc if "SQ_WAIT_INST_LDS" in v else None,
        })
    if not rows:
        raise SystemExit("no dispatch of that kernel carries both passes")
    out = {"config": a.config, "kernel": a.kernel,
           "source_counters": [os.path.relpath(p) for p in a.csv],
           "command": a.command, "iterations_per_dispatch": a.iters, "dispatches": len(rows)}
    for k in rows[0]:
        vals = [r[k] for r in rows if r[k] is not None]
        out[k] = statistics.median(vals) if vals else None
    out["frac"] = out["simd_valu_busy"]
    out["bound"] = a.bound
    out["limiter"] = a.limiter
    out["note"] = ("issue roofline: frac = share of SIMD cycles in which a VALU instruction "
                   "issues (1.0 = the SIMD's VALU never idle)")
    provenance.stamp(out, digest=provenance.read_digest(a.tree) if a.tree else None)  # the tree measured
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
