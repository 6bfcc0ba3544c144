"""Where the process runs relative to the GPU: allowed CPUs, the current CPU, the GPU's PCI NUMA
node and its local CPU list (the separate-call loop's latency depends on it: host-side spin on
pinned memory and the device's PCIe reads of the posted word)."""
import ctypes as C
import json
import os


def gpu_numa(device=0):
    hip = C.CDLL("libamdhip64.so")
    buf = C.create_string_buffer(64)
    if hip.hipDeviceGetPCIBusId(buf, 64, device) != 0:
        return None, None, None
    bus = buf.value.decode().lower()
    base = f"/sys/bus/pci/devices/{bus}"
    try:
        node = int(open(f"{base}/numa_node").read())
        cpus = open(f"{base}/local_cpulist").read().strip()
    except OSError:
        node, cpus = None, None
    return bus, node, cpus


def parse_list(s):
    out = set()
    for part in s.split(","):
        if "-" in part:
            a, b = part.split("-")
            out.update(range(int(a), int(b) + 1))
        elif part:
            out.add(int(part))
    return out


if __name__ == "__main__":
    bus, node, cpus = gpu_numa()
    allowed = sorted(os.sched_getaffinity(0))
    cur = int(open("/proc/self/stat").read().split()[38])
    local = parse_list(cpus) if cpus else set()
    print(json.dumps({"pci": bus, "gpu_numa_node": node, "gpu_local_cpus": cpus,
                      "allowed": f"{allowed[0]}..{allowed[-1]} ({len(allowed)})",
                      "allowed_local": len(local & set(allowed)), "current_cpu": cur,
                      "current_is_local": cur in local}))
