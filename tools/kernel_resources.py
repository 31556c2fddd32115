#!/usr/bin/env python3
"""Register / LDS / scratch use of every gfx950 kernel in a built library (no GPU needed).

Reads the clang offload bundle embedded in the .so's .hip_fatbin section, writes the gfx950 code object to a
temporary file and prints the AMDGPU metadata notes (llvm-readobj) as one line per kernel:
    vgpr agpr sgpr lds scratch name
Usage: tools/kernel_resources.py [lib/libpolymutt.so] [name-substring ...]
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(path):
    data = open(path, "rb").read()
    out, pos = [], 0
    while True:
        i = data.find(MAGIC, pos)
        if i < 0:
            return out
        n = struct.unpack_from("<Q", data, i + 24)[0]
        p = i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tl].decode()
            p += 24 + tl
            if "gfx950" in triple and size:
                out.append(data[i + off:i + off + size])
        pos = i + len(MAGIC)


def kernels(co):
    with tempfile.NamedTemporaryFile(suffix=".co", delete=False) as f:
        f.write(co)
        name = f.name
    try:
        txt = subprocess.run([os.path.join(LLVM, "llvm-readobj"), "--notes", name], capture_output=True, text=True).stdout
    finally:
        os.unlink(name)
    rows, cur = [], {}
    for line in txt.splitlines():
        m = re.match(r"\s*-?\s*\.(\w+):\s+(.*)", line)
        if not m:
            continue
        k, v = m.group(1), m.group(2).strip()
        if k == "args":
            continue
        if k == "agpr_count" and cur:
            rows.append(cur)
            cur = {}
        cur[k] = v
    if cur:
        rows.append(cur)
    return rows


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1].endswith((".so", ".o")) else \
        os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "polymutt_amd", "lib", "libpolymutt.so")
    pats = [a for a in sys.argv[1:] if not a.endswith((".so", ".o"))]
    demangle = "c++filt"
    for co in code_objects(lib):
        for r in kernels(co):
            nm = r.get("name", "?")
            dn = subprocess.run([demangle, nm], capture_output=True, text=True).stdout.strip() or nm
            if pats and not any(p in dn for p in pats):
                continue
            print(f"{r.get('vgpr_count', '?'):>4} {r.get('agpr_count', '?'):>3} {r.get('sgpr_count', '?'):>4} "
                  f"{r.get('group_segment_fixed_size', '?'):>6} {r.get('private_segment_fixed_size', '?'):>5} {dn}")


if __name__ == "__main__":
    main()
