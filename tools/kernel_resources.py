"""Per-kernel resources from the code-object metadata of the built library (not the trace):
VGPRs, AGPRs, SGPRs, scratch bytes per lane (private segment), static LDS, and the dynamic
LDS the launch adds where the host code sets one (tools/kernel_stats.py joins this with rocprofv3
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


# ---- the dynamic LDS each launch requests (lora_demod_fast.hip's launch_* functions),
# restated from its constexpr formulas: lds_row<SF>() = N + W3 + sum(LdsMap<SF>::W) + PAD,
# spec_lds_bytes<SF>(), the estimate / certification / fix kernels' row sets
LDS_MAP = {6: (0, (1, 2), 1), 7: (1, (1, 2, 4), 0), 8: (0, (1, 2, 4, 8), 1), 9: (0, (0, 1, 4, 8, 14), 0),
           10: (0, (0, 0, 1, 2, 4, 8), 0), 11: (0, (0, 0, 2, 8, 10, 20, 43), 0),
           12: (0, (0, 0, 0, 0, 1, 2, 4, 8), 0)}


def geo(sf):
    N = 1 << sf
    T = N // 16
    R1 = 8 if sf & 1 else 16
    X = N // R1
    RA = 16 if X >= 16 else X
    npass = 1 + (X > 1) + (X > 16)
    w3, w, pad = LDS_MAP[sf]
    return {"N": N, "T": T, "SPW": 256 // T, "MA_A": R1, "RA": RA, "NPASS": npass, "WL": T <= 64,
            "rowc": N + w3 + sum(w) + pad}


def dynamic_lds(demangled):
    """Dynamic LDS bytes the host requests for a launch of this kernel (SF >= 6), or None."""
    # the modulator, frame-max and compensation kernels use static LDS only
    if re.match(r"void (k_mod_\w+|k_frame_max\w*|k_compensate)\b", demangled):
        return 0
    m = re.match(r"void (k_\w+)<(\d+)(?:, (\w+))?(?:, (\w+))?(?:, (\w+))?(?:, (\w+))?>", demangled)
    if not m or int(m.group(2)) < 6 or int(m.group(2)) > 12:
        return None
    k, sf = m.group(1), int(m.group(2))
    g = geo(sf)
    twl = (15 if g["RA"] == 16 else 3) * g["MA_A"]
    if k == "k_spec_demod":
        dtl_off = ((g["SPW"] * g["rowc"] + twl) * 8 + 15) & ~15
        pf2 = g["WL"] and g["NPASS"] == 2
        if not pf2:
            return 8 * (g["SPW"] * g["rowc"] + twl)
        dtab = 4 * (dtl_off + 16 * g["N"]) <= 160 * 1024
        return dtl_off + (16 * g["N"] if dtab else 128 * g["T"])
    if k in ("k_est_split", "k_cert_split"):
        return 8 * 2 * (64 // (2 * g["T"])) * g["rowc"]
    if k == "k_spec_fix":
        return 8 * g["SPW"] * g["rowc"]
    if k == "k_est_fast":
        mode = int(m.group(3))
        block = 256 if g["T"] >= 64 else 64
        pair = sf >= 7 and g["WL"] and g["NPASS"] == 2 and mode <= 1
        return 8 * (block // g["T"]) * g["rowc"] * (2 if pair else 1)
    if k == "k_demod_fast":
        spec = m.group(5) == "true"
        return 8 * (g["SPW"] * g["rowc"] + (twl if spec else 0))
    return None


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
