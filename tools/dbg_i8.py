import sys, os, numpy as np, torch
sys.path[:0] = ["/root/repo", "/root/repo/maveric-slam_amd", "/root/repo/oracle", "/root/repo/tests"]
os.chdir(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import mvtrack, synth, oracle
from test_gpu_allpairs import run_i8
ctx = mvtrack.Context(0)
for case in range(3):
    if case == 0:
        a, b = synth.synth_pair_i8(0)
    elif case == 1:
        a, b = synth.synth_pair_i8(0, n=512)
    else:
        a, b = synth.synth_pair_i8(0, n=64)
    idx, dot = run_i8(ctx, torch, [(a, b)])
    i2, d2 = oracle.allpairs_i8(a, b)
    bad = np.where((idx[0] != i2) | (dot[0] != d2))[0]
    print("case", case, "n", a.shape[0], "mismatch rows", len(bad), "of", a.shape[0], "matched oracle", (i2 >= 0).sum(), "gpu", (idx[0] >= 0).sum())
    for r in bad[:12]:
        print("  row", r, "gpu", idx[0][r], dot[0][r], "oracle", i2[r], d2[r])
    if len(bad):
        print("  rows mod 32 hist", np.bincount(bad % 32, minlength=32).tolist())
        print("  gpu col mod 64 of mismatches", [int(idx[0][r]) % 64 for r in bad[:20]], "oracle", [int(i2[r]) % 64 for r in bad[:20]])
