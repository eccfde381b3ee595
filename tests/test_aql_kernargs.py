"""Kernel-argument layout the C++ drop-in's AQL dispatch relies on (CPU, no GPU).

lora_demodulate dispatches its kernels on a private AQL queue (csrc/lora_aql.hip) and
writes their kernel arguments itself: the explicit arguments packed at their C++ ABI
offsets by lora::record_launch (lora_internal.h), then - only for kernels that use any -
code object v5's implicit block (block counts, group sizes, remainders, global offsets,
grid dims, dynamic LDS size) at the next 8-byte boundary.  This test reads the kernel metadata of the built
library's gfx950 code objects and checks that every kernel lora_demod_batch can launch
has exactly that layout and no other hidden argument (a hostcall buffer, a heap pointer,
... would need the HIP runtime's setup)."""
import os
import shutil
import struct
import subprocess

import pytest
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "lora-sdr-lightweight-standalone-library-_amd", "lora_phy_amd", "lib", "liblora_mi355x.so")
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"

# the kernels lora_demod_batch and lora_mod_batch launch through lora::launch (recorded for the
# AQL queue)
FAMILIES = ("k_spec_demod", "k_est_split", "k_cert_split", "k_spec_fix", "k_est_fast", "k_demod_fast",
            "k_frame_max_wave", "k_frame_max", "k_estimate", "k_mod_phase", "k_mod_samples", "k_mod_frame",
            "k_mod_runs")
V5 = {"hidden_block_count_x": 0, "hidden_block_count_y": 4, "hidden_block_count_z": 8,
      "hidden_group_size_x": 12, "hidden_group_size_y": 14, "hidden_group_size_z": 16,
      "hidden_remainder_x": 18, "hidden_remainder_y": 20, "hidden_remainder_z": 22,
      "hidden_global_offset_x": 40, "hidden_global_offset_y": 48, "hidden_global_offset_z": 56,
      "hidden_grid_dims": 64, "hidden_dynamic_lds_size": 120}


def gfx950_code_objects(fatbin):
    out = []
    pos = fatbin.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", fatbin, pos + 24)[0]
        p = pos + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", fatbin, p)
            triple = fatbin[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if "gfx950" in triple:
                out.append(fatbin[pos + off:pos + off + size])
        pos = fatbin.find(MAGIC, pos + 1)
    return out


def kernels_metadata(tmp_path):
    fb = tmp_path / "fatbin.bin"
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", LIB, str(tmp_path / "x.so")],
                   check=True, capture_output=True)
    kernels = {}
    for i, co in enumerate(gfx950_code_objects(fb.read_bytes())):
        f = tmp_path / f"co{i}.o"
        f.write_bytes(co)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", str(f)], check=True, capture_output=True,
                               text=True).stdout
        doc = notes[notes.index("---"):notes.index("\n...") + 4]
        for k in yaml.safe_load(doc)["amdhsa.kernels"]:
            kernels[k[".name"]] = k
    return kernels


@pytest.mark.skipif(not os.path.exists(LIB) or not shutil.which(f"{LLVM}/llvm-readelf"),
                    reason="library or LLVM tools missing")
def test_dispatched_kernels_have_the_layout_the_aql_path_writes(tmp_path):
    kernels = kernels_metadata(tmp_path)
    checked = 0
    for name, k in kernels.items():
        if not any(f"{len(fam)}{fam}" in name for fam in FAMILIES):  # mangled: <len><name>
            continue
        off = 0
        hidden = []
        for a in k.get(".args", []):
            kind = a[".value_kind"]
            if kind.startswith("hidden"):
                hidden.append(a)
                continue
            size = a[".size"]
            align = 8 if size >= 8 else size
            off = (off + align - 1) // align * align
            assert a[".offset"] == off, (name, a)
            off += size
        if hidden:
            h = (off + 7) // 8 * 8
            for a in hidden:
                assert a[".value_kind"] in V5, (name, a)
                assert a[".offset"] == h + V5[a[".value_kind"]], (name, a)
            assert k[".kernarg_segment_size"] == h + 256, name
        else:
            assert k[".kernarg_segment_size"] == off, name
        assert off <= 384, name  # RecordedLaunch::kArgBytes
        checked += 1
    # every SF 6-12 instantiation of the pipeline kernels and the generic ones
    assert checked >= 50, checked
