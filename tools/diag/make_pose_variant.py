#!/usr/bin/env python3
"""Diagnosis only: build libmaveric_pose_<name>.so, the shipped library with ONE object
replaced -- k_pose_intended.hip compiled WITH SLP vectorisation and with one region of it kept scalar by
passing every value of that region through an empty asm (the vectoriser cannot pack a value an asm
reads and writes as a 32-bit VGPR).  The product source is not changed: the variant source is a
rewritten copy under build_variants/.

    python tools/diag/make_pose_variant.py qr      # the 8-point Householder QR kept scalar
    python tools/diag/make_pose_variant.py sampson # sampson_inlier / msac_cost kept scalar
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(ROOT, "maveric-slam_amd", "csrc", "hip", "k_pose_intended.hip")
OPQ = '#define PE_OPQ(x) asm volatile("" : "+v"(x))\n'


def opaque_region(text, start, end):
    """every `lhs op= expr;` / `lhs = expr;` float statement between the markers gets PE_OPQ(lhs)"""
    i, j = text.index(start), text.index(end, text.index(start))
    body = text[i:j]
    stmt = re.compile(r"^(\s*)((?:for \([^)]*\)\s*)?)((?:float )?)([A-Za-z_][\w]*(?:\[[^\]]+\])*) (\+|-|\*)?= ([^;{}]+);((?:\s*//.*)?)$", re.M)

    def rep(m):
        ind, loop, decl, lhs, op, rhs, cmt = m.groups()
        name = lhs
        s = "%s%s%s %s= %s; PE_OPQ(%s);" % (decl, lhs, "", op or "", rhs, name)
        s = s.replace(" = ", " = ", 1)
        return ("%s%s{ %s }" % (ind, loop, s) if loop else ind + s) + cmt

    new = stmt.sub(rep, body)
    return text[:i] + new + text[j:], body.count("\n"), sum(1 for _ in stmt.finditer(body))


def main():
    name = sys.argv[1]
    text = open(SRC).read()
    regions = {"qr": ("__device__ __forceinline__ bool eight_point", "__device__ __forceinline__ bool sampson_inlier"),
               "sampson": ("__device__ __forceinline__ bool sampson_inlier", "// msac_cost of two correspondences")}
    start, end = regions[name]
    text, nl, ns = opaque_region(text, start, end)
    text = text.replace('#include "mv_internal.hpp"\n', '#include "mv_internal.hpp"\n' + OPQ, 1)
    vdir = os.path.join(ROOT, "build_variants")
    os.makedirs(vdir, exist_ok=True)
    vsrc = os.path.join(vdir, "k_pose_intended_%s.hip" % name)
    open(vsrc, "w").write(text)
    print("%s: %d statements made opaque over %d lines -> %s" % (name, ns, nl, vsrc))
    obj = os.path.join(vdir, "obj_pose_%s" % name)
    os.makedirs(obj, exist_ok=True)
    base = os.path.join(ROOT, "maveric-slam_amd", "csrc", "build")
    for f in os.listdir(base):
        if f.endswith(".o") and f != "k_pose_intended.o":
            subprocess.check_call(["cp", os.path.join(base, f), obj])
    inc = ["-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "maveric-slam_amd", "csrc", "hip")]
    fl = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-ffp-contract=off",
          "-fhip-fp32-correctly-rounded-divide-sqrt"] + inc
    subprocess.check_call(["/opt/rocm/bin/hipcc"] + fl + ["-c", vsrc, "-o", os.path.join(obj, "k_pose_intended.o")])
    subprocess.check_call(["/opt/rocm/bin/hipcc"] + fl + ["--cuda-device-only", "-S", vsrc, "-o",
                                                          os.path.join(vdir, "k_pose_intended_%s.s" % name)])
    objs = sorted(os.path.join(obj, f) for f in os.listdir(obj) if f.endswith(".o"))
    out = os.path.join(vdir, "libmaveric_pose_%s.so" % name)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out] + objs +
                          ["-Wl,--version-script=" + os.path.join(ROOT, "maveric-slam_amd", "csrc", "exports.map"),
                           "-Wl,-soname,libmaveric_hip.so"])
    s = open(os.path.join(vdir, "k_pose_intended_%s.s" % name)).read()
    print(out, "v_pk_* in the pose ISA:", s.count("v_pk_"))


if __name__ == "__main__":
    main()
