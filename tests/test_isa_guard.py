"""CPU: the shipped library's device code holds no packed-FP32 instruction whose low lane reads the
HIGH half of src1 (v_pk_{fma,mul,add}_f32 ... op_sel:[x,1,...]).  On MI355X that operand read as
zero in ~1.3e-4 of executions while the SuperPoint network ran on another stream
(tools/diag/pk_probe.py) -- what made round 5's SLP-vectorised as-intended pose
nondeterministic.  The scanner is checked on a code object that does contain the form."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
LIB = os.path.join(ROOT, "maveric-slam_amd", "libmaveric_hip.so")

need_tools = pytest.mark.skipif(not (shutil.which("objcopy") and os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump")),
                                reason="objcopy / llvm-objdump not available")


@need_tools
@pytest.mark.skipif(not os.path.exists(LIB), reason="libmaveric_hip.so not built")
def test_no_src1_high_half_packed_fp32_in_library():
    import isa_guard

    cos = isa_guard.code_objects(isa_guard.fatbin_section(LIB))
    assert len(cos) >= 10  # one gfx950 code object per kernel translation unit
    hits = isa_guard.scan(LIB)
    assert hits == [], "packed-FP32 src1 high-half reads in the library:\n" + "\n".join(
        "%s: %s" % h for h in hits[:20])


@need_tools
@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="hipcc not available")
def test_scanner_finds_the_form(tmp_path):
    import isa_guard

    src = tmp_path / "pk.hip"
    src.write_text('''#include <hip/hip_runtime.h>
typedef float f2 __attribute__((ext_vector_type(2)));
__global__ void k_bad(f2 *p) {
    f2 a = p[threadIdx.x], b = p[threadIdx.x + 64], d;
    asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel:[0,1]" : "=v"(d) : "v"(a), "v"(b));
    asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,0,0]" : "+v"(d) : "v"(a), "v"(b));
    p[threadIdx.x] = d;
}
''')
    so = tmp_path / "libpk.so"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-fPIC", "-shared", str(src), "-o", str(so)],
                   check=True, capture_output=True)
    hits = isa_guard.scan(str(so))
    assert len(hits) == 1 and "op_sel:[0,1]" in hits[0][1] and "k_bad" in hits[0][0]
