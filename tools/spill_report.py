"""Register spills and scratch of every kernel in the built library, read
from the code objects' metadata notes (no GPU needed): the build-time scan
DESIGN.md section 8 asked for after two kernels lost most of their time to
SGPR spills (uniform values parked in SGPRs and moved through VGPR lanes)
and scratch-resident arrays.

    python tools/spill_report.py [LIB] [--all]   (JSON lines, spilled kernels
                                                  only unless --all)"""
import json
import os
import shutil
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT_LIB = os.path.join(ROOT, "pyabc_amd", "_lib", "libabc_hip.so")
_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
_FIELDS = (".sgpr_spill_count", ".vgpr_spill_count", ".private_segment_fixed_size",
           ".vgpr_count", ".agpr_count", ".sgpr_count")


def readelf():
    for p in ("/opt/rocm/lib/llvm/bin/llvm-readelf", shutil.which("llvm-readelf")):
        if p and os.path.exists(p):
            return p
    return None


def code_objects(lib):
    """gfx950 ELF images of every offload bundle in the library's fat binary"""
    b = open(lib, "rb").read()
    out = []
    i = b.find(_MAGIC)
    while i >= 0:
        n = struct.unpack_from("<Q", b, i + 24)[0]
        q = i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", b, q)
            triple = b[q + 24:q + 24 + tl].decode()
            q += 24 + tl
            if "gfx950" in triple and size:
                out.append(b[i + off:i + off + size])
        i = b.find(_MAGIC, i + 1)
    return out


def kernel_resources(lib=DEFAULT_LIB):
    """{mangled kernel name: {field: int}} over all code objects"""
    tool = readelf()
    if tool is None:
        raise FileNotFoundError("llvm-readelf not found")
    res = {}
    with tempfile.TemporaryDirectory() as d:
        for k, img in enumerate(code_objects(lib)):
            path = os.path.join(d, f"co{k}.elf")
            with open(path, "wb") as f:
                f.write(img)
            txt = subprocess.run([tool, "--notes", path], capture_output=True,
                                 text=True, check=True).stdout
            # metadata keys are sorted: a kernel's .name precedes its counts
            cur = None
            for line in txt.splitlines():
                s = line.strip()
                if s.startswith(".name:"):
                    cur = s.split(None, 1)[1]
                    res[cur] = {}
                elif cur is not None and s.split(":")[0] in _FIELDS:
                    key, val = s.split(":", 1)
                    res[cur][key[1:]] = int(val)
    return res


def demangle(names):
    cf = shutil.which("c++filt")
    if cf is None:
        return {n: n for n in names}
    out = subprocess.run([cf], input="\n".join(names), capture_output=True,
                         text=True).stdout.splitlines()
    return dict(zip(names, out))


def kernel_label(demangled):
    """'void ns::name<args>' without the parameter list"""
    return demangled.replace("(anonymous namespace)::", "").split("(")[0]


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    lib = args[0] if args else DEFAULT_LIB
    res = kernel_resources(lib)
    dm = demangle(list(res))
    for name, r in sorted(res.items(), key=lambda x: dm[x[0]]):
        bad = (r.get("sgpr_spill_count", 0) or r.get("vgpr_spill_count", 0)
               or r.get("private_segment_fixed_size", 0))
        if bad or "--all" in sys.argv:
            print(json.dumps({"kernel": kernel_label(dm[name]), **r}))


if __name__ == "__main__":
    main()
