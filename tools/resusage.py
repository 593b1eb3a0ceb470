"""Print VGPR/AGPR/spill/occupancy per kernel of a HIP source (device-only compile).
usage: python tools/resusage.py [file.hip] [extra hipcc flags...]"""
import os
import re
import subprocess
import sys

here = os.path.dirname(os.path.abspath(__file__))
src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(here, "..", "scenedino_amd", "csrc",
                                                          "sdhip_field.hip")
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
       "-DSD_FASTPE=0", "--cuda-device-only", "-c", "-Rpass-analysis=kernel-resource-usage",
       *sys.argv[2:], src, "-o", "/tmp/_ru.o"]
out = subprocess.run(cmd, capture_output=True, text=True, cwd="/tmp").stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?) \[-Rpass", line)
    if not m:
        if "error" in line:
            print(line)
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    g = r.get
    print(f"{r['name'][:58]:58s} v={g('VGPRs')} a={g('AGPRs')} vspill={g('VGPRs Spill')} "
          f"sspill={g('SGPRs Spill')} occ={g('Occupancy [waves/SIMD]')} lds={g('LDS Size [bytes/block]')}")
