"""Per-kernel resource usage of the built engine library (VGPRs, SGPRs, spills, scratch, LDS).

Reads the gfx950 code objects out of fluidframework_amd/libmtgpu.so (clang offload bundles in
its .hip_fatbin data) and prints each kernel's AMDGPU metadata from `llvm-readelf --notes`.
usage: python tools/kernel_resources.py [lib.so] [name-substring]   (code = the kernel symbol's bytes)
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
FIELDS = (".name", ".vgpr_count", ".agpr_count", ".sgpr_count", ".vgpr_spill_count", ".sgpr_spill_count",
          ".private_segment_fixed_size", ".group_segment_fixed_size")


def code_objects(data: bytes):
    at = 0
    while True:
        i = data.find(MAGIC, at)
        if i < 0:
            return
        n = struct.unpack_from("<Q", data, i + 24)[0]
        p = i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tl].decode(errors="replace")
            p += 24 + tl
            if "gfx950" in triple:
                yield data[i + off:i + off + size]
        at = i + len(MAGIC)


sizes = {}                    # kernel symbol -> code bytes


def kernels(path: str):
    out = []
    data = open(path, "rb").read()
    with tempfile.TemporaryDirectory() as td:
        for k, co in enumerate(code_objects(data)):
            f = os.path.join(td, f"co{k}.o")
            open(f, "wb").write(co)
            txt = subprocess.run([READELF, "--notes", f], capture_output=True, text=True).stdout
            syms = subprocess.run([READELF, "-sW", f], capture_output=True, text=True).stdout
            for line in syms.splitlines():
                p = line.split()
                if len(p) >= 8 and p[3] == "FUNC":
                    sizes[p[7]] = int(p[2], 0) if p[2].startswith("0x") else int(p[2])
            cur = None
            for line in txt.splitlines():
                m = re.match(r"\s*-?\s*(\.[a-z_]+):\s*(.*)$", line)
                if not m:
                    continue
                key, val = m.group(1), m.group(2).strip()
                if key == ".args":
                    continue
                if key == ".agpr_count" and cur is not None and ".vgpr_count" in cur:   # a kernel's first key
                    out.append(cur)
                    cur = None
                if key in FIELDS:
                    if cur is None:
                        cur = {}
                    if key == ".name" and ".name" in cur:
                        continue
                    cur[key] = val
            if cur and ".vgpr_count" in cur:
                out.append(cur)
    return out


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1].endswith(".so") else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fluidframework_amd", "libmtgpu.so")
    sub = next((a for a in sys.argv[1:] if not a.endswith(".so")), "")
    seen = set()
    for k in kernels(lib):
        name = k.get(".name", "?")
        if sub not in name or name in seen:
            continue
        seen.add(name)
        print(f"{name[:90]:90s} vgpr {k.get('.vgpr_count', '?'):>3} agpr {k.get('.agpr_count', '0'):>3} "
              f"sgpr {k.get('.sgpr_count', '?'):>3} vspill {k.get('.vgpr_spill_count', '?'):>3} "
              f"sspill {k.get('.sgpr_spill_count', '?'):>4} scratch {k.get('.private_segment_fixed_size', '?'):>4} "
              f"lds {k.get('.group_segment_fixed_size', '?'):>6} code {sizes.get(name, 0):>7}")


if __name__ == "__main__":
    main()
