#!/usr/bin/env python3
"""The shipped library's device code, disassembled: every gfx950 code object embedded in
libmaveric_hip.so's .hip_fatbin section (one clang offload bundle per translation unit) is cut out
and run through llvm-objdump.  Used by tests/test_isa_guard.py to keep instruction forms that are
not safe on this hardware out of the product (packed-FP32 VOP3P instructions whose
low lane reads a source's HIGH half gave wrong bits while other kernels ran concurrently).

    python tools/isa_guard.py [lib.so]     # prints the offending instructions per code object
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def fatbin_section(lib):
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "fatbin")
        # an explicit output file: with the input alone objcopy rewrites the library in place
        # (identical bytes, but under any process that has it mapped)
        subprocess.run(["objcopy", "--dump-section", ".hip_fatbin=" + out, lib, os.path.join(d, "copy.so")],
                       check=True, capture_output=True)
        return open(out, "rb").read()


def code_objects(blob, arch="gfx950"):
    """(bundle index, code object bytes) of every bundle entry for `arch`"""
    out = []
    pos = blob.find(MAGIC)
    k = 0
    while pos >= 0:
        n = struct.unpack_from("<Q", blob, pos + 24)[0]
        p = pos + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", blob, p)
            triple = blob[p + 24:p + 24 + tl].decode()
            p += 24 + tl
            if triple.endswith(arch) and size:
                out.append((k, blob[pos + off:pos + off + size]))
        k += 1
        pos = blob.find(MAGIC, pos + 1)
    return out


def disassemble(co):
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(co)
        f.flush()
        r = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", f.name], check=True,
                           capture_output=True, text=True)
        return r.stdout


# a packed-FP32 VOP3P instruction whose LOW lane reads the HIGH half of a source register pair
# (op_sel bit set): v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32 (tools/diag/pk_probe.py)
PK_HI_TO_LO = re.compile(r"\bv_pk_(fma|mul|add)_f32\b[^\n]*\bop_sel:\[[01],1")


def functions(text):
    """{kernel symbol: its disassembly}"""
    d, cur = {}, None
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <([^>]+)>:", line)
        if m:
            cur = m.group(1)
            d[cur] = []
        elif cur:
            d[cur].append(line)
    return {k: "\n".join(v) for k, v in d.items()}


def scan(lib=None, pattern=PK_HI_TO_LO):
    """[(kernel, instruction)] matching `pattern` over every code object of the library"""
    lib = lib or os.path.join(ROOT, "maveric-slam_amd", "libmaveric_hip.so")
    hits = []
    for _, co in code_objects(fatbin_section(lib)):
        for fn, body in functions(disassemble(co)).items():
            for line in body.splitlines():
                if pattern.search(line):
                    hits.append((fn, line.split("//")[0].strip()))
    return hits


if __name__ == "__main__":
    hits = scan(sys.argv[1] if len(sys.argv) > 1 else None)
    for fn, ins in hits:
        print("%s: %s" % (fn, ins))
    print("%d instruction(s)" % len(hits))
    sys.exit(1 if hits else 0)
