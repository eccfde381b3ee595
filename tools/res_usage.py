"""Per-kernel VGPR / spill / occupancy summary of a HIP source (device compile only).

usage: python tools/res_usage.py csrc/lora_demod_fast.hip [name-regex] [extra hipcc flags...]
"""
import re
import subprocess
import sys

src = sys.argv[1]
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-c", src,
       "-o", "/tmp/res_usage.o", "--offload-device-only", "-Rpass-analysis=kernel-resource-usage"] + sys.argv[3:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    if pat.search(r["name"]):
        print("%-72s vgpr=%s spill=%s occ=%s" % (r["name"][:72], r.get("VGPRs"), r.get("VGPRs Spill"),
                                               r.get("Occupancy [waves/SIMD]")))
