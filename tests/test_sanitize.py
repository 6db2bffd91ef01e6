"""Host-C sanitizer builds (AddressSanitizer + UndefinedBehaviorSanitizer on the CPU;
GPU sanitizers are not available on the MI355X pool).

1. The product's host C (maveric-slam_amd/csrc/host/*.c: the feature pool, the trajectory file
   I/O, the drop-in shims) built with gcc -fsanitize=address,undefined -fno-sanitize-recover=all
   and driven by tests/c/sanitize_host.c, the HIP entry points answered as on a machine without a
   device (tests/c/no_device_stubs.c).  This build found the feature pool's num_frames underflow
   after a failed delete (feature_pool.c, mv_local_feature_remove_old_frame).
2. The C oracle (oracle/mv_oracle.c + sp_oracle.c) built the same way (oracle/Makefile `san`)
   and the oracle's own CPU tests run against it (MV_ORACLE_SO), the ASan runtime preloaded into
   the Python process (with libstdc++, whose exceptions torch throws)."""
import os
import subprocess
import sys
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "maveric-slam_amd", "csrc", "host")
SANFLAGS = ["-O1", "-g", "-fno-omit-frame-pointer", "-ffp-contract=off", "-fsanitize=address,undefined",
            "-fno-sanitize-recover=all"]


def _gcc_file(name):
    return subprocess.run(["gcc", "-print-file-name=" + name], capture_output=True, text=True,
                          check=True).stdout.strip()


def test_host_c_under_asan_ubsan():
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "sanitize_host")
        srcs = [os.path.join(ROOT, "tests", "c", "sanitize_host.c"), os.path.join(ROOT, "tests", "c", "no_device_stubs.c")]
        srcs += sorted(os.path.join(HOST, f) for f in os.listdir(HOST) if f.endswith(".c"))
        r = subprocess.run(["gcc", "-std=gnu11", "-Wall", "-Werror", "-I" + os.path.join(ROOT, "include")] + SANFLAGS +
                           ["-o", exe] + srcs + ["-lm"], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr[-3000:]
        env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1", UBSAN_OPTIONS="print_stacktrace=1")
        r = subprocess.run([exe, d], capture_output=True, text=True, timeout=300, env=env)
        assert r.returncode == 0 and "runtime error" not in r.stderr, r.stderr[-4000:]
        assert "sanitize_host ok" in r.stdout


ORACLE_TESTS = ["test_oracle_pinning.py", "test_tracking_main_ref.py", "test_image_chain.py", "test_keypoints.py",
                "test_factors.py", "test_lba.py", "test_cellnms.py", "test_two_way.py", "test_trajectory.py",
                "test_superpoint.py"]


@pytest.mark.timeout(900)
def test_oracle_under_asan_ubsan():
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "san"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    so = os.path.join(ROOT, "oracle", "_san", "liboracle_san.so")
    env = dict(os.environ, MV_ORACLE_SO=so, LD_PRELOAD=_gcc_file("libasan.so") + " " + _gcc_file("libstdc++.so.6"),
               ASAN_OPTIONS="detect_leaks=0", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-m", "not gpu", "-p", "no:cacheprovider"] +
                       [os.path.join(ROOT, "tests", t) for t in ORACLE_TESTS],
                       capture_output=True, text=True, timeout=880, env=env, cwd=ROOT)
    tail = (r.stdout[-3000:] + r.stderr[-3000:])
    assert r.returncode == 0, tail
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, tail
    assert " passed" in r.stdout, tail
