#!/usr/bin/env python3
"""Per-kernel resource usage of a built liblbk8s.so, read from its gfx950 code object (no
rebuild): VGPRs, AGPRs, SGPRs, spills, scratch and LDS bytes.

    python tools/kernel_meta.py exp/liblbk8s_x.so [name-substring ...]
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/llvm/bin"


def kernels(lib):
    with tempfile.TemporaryDirectory() as d:
        fb, co = os.path.join(d, "fb.bin"), os.path.join(d, "co.o")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", lib, os.path.join(d, "x")],
                       check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                        f"--input={fb}", f"--output={co}", "--unbundle"], check=True)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True,
                               check=True).stdout
    out, cur = [], None
    for line in notes.splitlines():
        m = re.match(r"\s*-?\s*\.(\w+):\s+(\S+)", line)
        if not m:
            continue
        k, v = m.groups()
        if k == "agpr_count" and line.lstrip().startswith("-"):
            cur = {}
            out.append(cur)
        if cur is None:
            continue
        if k in ("name", "vgpr_count", "agpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count",
                 "private_segment_fixed_size", "group_segment_fixed_size"):
            cur.setdefault(k, v)
    return out


def main():
    lib, pats = sys.argv[1], sys.argv[2:]
    for k in kernels(lib):
        n = k.get("name", "?")
        if pats and not any(p in n for p in pats):
            continue
        print(f"{n[:90]:90s} v={k.get('vgpr_count')} a={k.get('agpr_count')} s={k.get('sgpr_count')} "
              f"vspill={k.get('vgpr_spill_count')} sspill={k.get('sgpr_spill_count')} "
              f"scratch={k.get('private_segment_fixed_size')} lds={k.get('group_segment_fixed_size')}")


if __name__ == "__main__":
    main()
