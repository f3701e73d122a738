#!/usr/bin/env python3
"""Per-kernel VGPRs / spills / LDS / occupancy of one csrc/*.hip file (hipcc resource remarks).
usage: tools/resource_usage.py <csrc stem, e.g. gi_knn_chunk> [extra hipcc flags...]"""
import re, subprocess, sys
stem = sys.argv[1]
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=off",
       "-Iinclude", "-Iglobal-illumination_amd/csrc", *sys.argv[2:], "-c",
       f"global-illumination_amd/csrc/{stem}.hip", "-o", "/tmp/_ru.o", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = {"name": subprocess.run(["c++filt", t.split(":", 1)[1].strip()], capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    print(f'{r.get("VGPRs","?"):>4} vgpr {r.get("AGPRs","0"):>3} agpr  spill v{r.get("VGPRs Spill","?"):>4} s{r.get("SGPRs Spill","?"):>4}  lds {r.get("LDS Size [bytes/block]","?"):>6}  occ {r.get("Occupancy [waves/SIMD]","?"):>2}  {r["name"][:110]}')
