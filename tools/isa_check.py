"""Device-ISA audit of lora_demod_fast.hip as the Makefile builds it (scalar fp32 TU):
per kernel matching the regex, out-of-line calls, scratch accesses, vmcnt waits and
vector loads.  usage: python tools/isa_check.py [kernel-regex] [-v]"""
import re
import subprocess
import sys

SRC = "lora-sdr-lightweight-standalone-library-_amd/csrc/lora_demod_fast.hip"
pat = re.compile(sys.argv[1] if len(sys.argv) > 1 else ".")
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
       "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops", "-S", "--offload-device-only",
       SRC, "-o", "/tmp/isa_check.s"]
subprocess.run(cmd, check=True, capture_output=True)
s = open("/tmp/isa_check.s").read()
for name in re.findall(r"^(_Z\w+k_\w+):", s, re.M):
    if not pat.search(name):
        continue
    i = s.index(name + ":")
    body = s[i:s.index(".Lfunc_end", i)]
    waits = re.findall(r"s_waitcnt vmcnt\((\d+)\)", body)
    print("%-64s calls=%d scratch=%d pk=%d vmcnt=%s gload=%d" % (
        name[:64], body.count("s_swappc"), body.count("scratch_"), len(re.findall(r"v_pk_\w+_f32", body)),
        ",".join(waits) if "-v" in sys.argv else len(waits), len(re.findall(r"global_load_dword", body))))
