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


MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def kernels(lib):
    notes = ""
    with tempfile.TemporaryDirectory() as d:
        fb = os.path.join(d, "fb.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", lib, os.path.join(d, "x")],
                       check=True)
        data = open(fb, "rb").read()
        starts = [i for i in range(len(data)) if data.startswith(MAGIC, i)]
        for n, a in enumerate(starts):  # (one bundle per compiled unit)
            b = starts[n + 1] if n + 1 < len(starts) else len(data)
            part, co = os.path.join(d, f"b{n}.bin"), os.path.join(d, f"co{n}.o")
            open(part, "wb").write(data[a:b])
            subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                            f"--input={part}", f"--output={co}", "--unbundle"], check=True)
            notes += subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True,
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
