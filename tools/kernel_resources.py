"""Per-kernel resources from the code-object metadata of the built library (not the trace):
VGPRs, AGPRs, SGPRs, scratch bytes per lane (private segment), static LDS, and the dynamic
LDS the launch adds where the host code sets one (tools/prof_r04.py joins this with rocprofv3
kernel statistics).  usage: python tools/kernel_resources.py [lib.so] [name-regex] [--json]
"""
import json
import re
import subprocess
import sys
import tempfile

LIB = "lora-sdr-lightweight-standalone-library-_amd/lora_phy_amd/lib/liblora_mi355x.so"
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
CXXFILT = "c++filt"


def code_objects(path):
    """gfx950 ELF images of the clang offload bundles in the library's .hip_fatbin."""
    data = open(path, "rb").read()
    out = []
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    pos = data.find(magic)
    while pos >= 0:
        cnt = int.from_bytes(data[pos + 24:pos + 32], "little")
        p = pos + 32
        # a bundle header (the library also holds the magic as a string literal: skip those)
        if pos % 8 or not 0 < cnt <= 16:
            pos = data.find(magic, pos + 24)
            continue
        for _ in range(cnt):
            off, size, tlen = (int.from_bytes(data[p + 8 * k:p + 8 * k + 8], "little") for k in range(3))
            triple = data[p + 24:p + 24 + tlen].decode(errors="replace")
            p += 24 + tlen
            if tlen > 256 or pos + off + size > len(data):
                break
            if "gfx950" in triple and size:
                out.append(data[pos + off:pos + off + size])
        pos = data.find(magic, pos + 32)
    return out


def kernels(path):
    rows = []
    for img in code_objects(path):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(img)
            f.flush()
            notes = subprocess.run([READELF, "--notes", f.name], capture_output=True, text=True).stdout
        cur = None
        for line in notes.splitlines():
            m = re.match(r"\s*-?\s*\.(\w+):\s+(.*)$", line)
            if not m:
                continue
            k, v = m.group(1), m.group(2).strip()
            if line.lstrip().startswith("- .") and k in ("agpr_count", "args") and cur is None:
                pass
            if k == "name" and not v.endswith(".kd"):
                cur = {"name": v}
                rows.append(cur)
            elif cur is not None and k in ("vgpr_count", "agpr_count", "sgpr_count", "private_segment_fixed_size",
                                           "group_segment_fixed_size", "max_flat_workgroup_size",
                                           "vgpr_spill_count", "sgpr_spill_count", "symbol"):
                cur[k] = int(v) if v.isdigit() else v
    names = [r["name"] for r in rows]
    dem = subprocess.run([CXXFILT], input="\n".join(names), capture_output=True, text=True).stdout.splitlines()
    for r, d in zip(rows, dem):
        r["demangled"] = d.replace("lora::(anonymous namespace)::", "").replace("(lora::KArgs, long, int, long)", "").replace(
            "(lora::KArgs, long, int)", "")
    return rows


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    lib = args[0] if args and args[0].endswith(".so") else LIB
    pat = re.compile(args[-1] if args and not args[-1].endswith(".so") else ".")
    rows = [r for r in kernels(lib) if pat.search(r.get("demangled", r["name"]))]
    if "--json" in sys.argv:
        print(json.dumps(rows, indent=1))
    else:
        for r in rows:
            print("%-60s vgpr=%-3s agpr=%-2s sgpr=%-3s scratch=%-3s lds_static=%-5s spill=%s/%s" % (
                r["demangled"][:60], r.get("vgpr_count"), r.get("agpr_count"), r.get("sgpr_count"),
                r.get("private_segment_fixed_size"), r.get("group_segment_fixed_size"), r.get("vgpr_spill_count"),
                r.get("sgpr_spill_count")))
