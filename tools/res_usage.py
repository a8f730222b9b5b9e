"""Per-kernel VGPRs / spills of a HIP source (hipcc -Rpass-analysis=kernel-resource-usage).
usage: python tools/res_usage.py protein-structure-tokenizer_amd/csrc/pst_kernels.hip [-DFLAG ...]"""
import re
import subprocess
import sys

cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
       "-fno-fast-math", "-c", sys.argv[1], "-o", "/tmp/res_usage.o", "-Rpass-analysis=kernel-resource-usage"] + sys.argv[2:]
err = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in err.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|VGPRs Spill|SGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1)] = int(m.group(2))
for k, v in rows.items():
    print(f"{k[:60]:60s} vgpr {v.get('VGPRs')} agpr {v.get('AGPRs')} vspill {v.get('VGPRs Spill')} "
          f"sspill {v.get('SGPRs Spill')} occ {v.get('Occupancy [waves/SIMD]')}")
