"""Code size of libpyas_hip.so per kernel family.

Reads the gfx950 code objects out of the build's per-part objects
(clang offload bundles in build/pyas/*.o), lists each kernel symbol once
with its size, and sums by kernel template.  CPU only.

    python tools/lib_sizes.py [--top 40] [--json]
"""
import argparse
import collections
import glob
import json
import os
import re
import struct
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def gfx950_objects(path):
    data = open(path, "rb").read()
    i = data.find(MAGIC)
    while i >= 0:
        n = struct.unpack_from("<Q", data, i + 24)[0]
        p = i + 32
        for _ in range(n):
            off, size, idl = struct.unpack_from("<QQQ", data, p)
            tid = data[p + 24:p + 24 + idl].decode()
            p += 24 + idl
            if "gfx950" in tid:
                yield data[i + off:i + off + size]
        i = data.find(MAGIC, i + 32)


def kernels(elf_bytes):
    with tempfile.NamedTemporaryFile(suffix=".elf") as f:
        f.write(elf_bytes)
        f.flush()
        out = subprocess.run([READELF, "-sW", f.name], capture_output=True, text=True, check=True).stdout
    seen = {}
    for line in out.splitlines():
        fld = line.split()
        if len(fld) >= 8 and fld[3] == "FUNC" and fld[7] not in seen:
            seen[fld[7]] = int(fld[2], 0)
    return seen


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args()
    syms = {}
    for obj in sorted(glob.glob(os.path.join(ROOT, "build", "pyas", "*.o"))):
        for co in gfx950_objects(obj):
            syms.update(kernels(co))
    names = list(syms)
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True,
                         check=True).stdout.splitlines()
    size, count = collections.Counter(), collections.Counter()
    for raw, d in zip(names, dem):
        fam = re.sub(r"<.*", "", d).replace("void ", "").split("(")[0]
        size[fam] += syms[raw]
        count[fam] += 1
    lib = os.path.join(ROOT, "pyactivestorage_amd", "lib", "libpyas_hip.so")
    res = {"lib_bytes": os.path.getsize(lib) if os.path.exists(lib) else None,
           "code_bytes": sum(size.values()), "kernels": sum(count.values()),
           "families": [{"kernel": k, "bytes": v, "instances": count[k]} for k, v in size.most_common(a.top)]}
    if a.json:
        print(json.dumps(res, indent=1))
        return
    print(f"lib {res['lib_bytes']} B, gfx950 code {res['code_bytes']} B in {res['kernels']} kernels")
    for f in res["families"]:
        print(f"{f['bytes'] / 1e6:8.2f} MB {f['instances']:5d}  {f['kernel']}")


if __name__ == "__main__":
    main()
