#!/bin/bash
# Register / scratch / LDS use of the kernels whose names match $1 (regex), gfx950 build.
cd "$(dirname "$0")/../diffusionmcmctools.jl_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-result \
  ${EXTRA_FLAGS} -c dmt_kernels.hip -o /tmp/dmt_kernels_ru.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  python3 -c '
import re, sys
pat = re.compile(sys.argv[1]); cur = None; out = {}
for l in sys.stdin:
    m = re.search(r"Function Name: (\S+)", l)
    if m: cur = m.group(1); out[cur] = {}; continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|LDS Size \[bytes/block\]|Occupancy \[waves/SIMD\]): (\d+)", l)
    if m and cur: out[cur][m.group(1).split()[0]] = int(m.group(2))
for k, v in out.items():
    if pat.search(k): print(k[:90], v)
' "${1:-.}"
