"""Latency spread of the caller's separate-call loop (draw, accept, fetch_ll, fetch_ll°) on C2,
per iteration, with the resident service on or off (DMT_SERVICE) — csrc/dmt_callbench.c."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import diffusionmcmctools_amd as dmt  # noqa: E402
from diffusionmcmctools_amd import workloads as W  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
pin = os.environ.get("SVC_PIN")  # "local": run on the GPU's NUMA-local CPUs; "remote": off them
if pin:
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import numa_info
    _, _, cpus = numa_info.gpu_numa()
    local = numa_info.parse_list(cpus) if cpus else set()
    allowed = os.sched_getaffinity(0)
    want = (allowed & local) if pin == "local" else (allowed - local)
    if want:
        os.sched_setaffinity(0, want)
w = W.c2_ou2d()
w.meta["hist_len"] = 2 * n + 8
e = dmt.Ensemble(w.model.kind, w.d, w.m, w.n_points, precision=w.precision, seed=1,
                 grid_shared=w.grid_shared)
lay = W.fill(e, w)
B = w.nblocks
e.loglikhd(lay, 0, 0, B)
# beside the library in use (a DMT_LIB_PATH variant directory holds its own libdmt_callbench.so)
lib_dir = (os.path.dirname(os.environ["DMT_LIB_PATH"]) if os.environ.get("DMT_LIB_PATH")
           else os.path.join(ROOT, "diffusionmcmctools.jl_amd"))
lib = C.CDLL(os.path.join(lib_dir, "libdmt_callbench.so"))
lat = np.zeros(n)
out = {}
for rep in range(2):
    st = lib.dmt_callbench_lat(e.handle, C.c_int32(lay), C.c_int64(0), C.c_int64(B),
                               C.c_int64(1 + rep * n), C.c_int64(n),
                               lat.ctypes.data_as(C.POINTER(C.c_double)))
    assert st == 0, st
    us = lat * 1e6
    out[f"rep{rep}"] = {"median_us": float(np.median(us)), "mean_us": float(us.mean()),
                        "p90_us": float(np.percentile(us, 90)), "max_us": float(us.max()),
                        "n_over_1ms": int((us > 1000).sum()), "first10": [round(x, 1) for x in us[:10]]}
cur = int(open("/proc/self/stat").read().split()[38])
print(json.dumps({"service": os.environ.get("DMT_SERVICE", "1"), "B": B, "pin": pin, "cpu": cur,
                  "affinity_n": len(os.sched_getaffinity(0)), **out}))
e.close()
