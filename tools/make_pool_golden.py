#!/usr/bin/env python3
"""Golden vectors for the local feature pool (tests/test_feature_pool.py), made by the
reference's OWN code: include/local_feature_pool.h driven by src/local_feature_matching.c's
generator (srand(0), 100 frames x 200 word ids), compiled from the reference's sources into
oracle/_ref/libmv_ref_pool.so (oracle/ref_pool_harness.c).  Stores the ids, the pool size
after each frame, a CRC32 of the whole table after each frame and the final table."""
import os
import sys
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402


def main():
    ids, tab, sz = oracle.ref_pool_run(100, 200)
    crc = np.array([zlib.crc32(np.ascontiguousarray(t).tobytes()) for t in tab], np.uint32)
    out = os.path.join(ROOT, "tests", "golden", "feature_pool_ref.npz")
    np.savez_compressed(out, ids=ids.astype(np.int16), sizes=sz, table_crc32=crc, final_table=tab[-1])
    print("wrote", out, "final size", int(sz[-1]))


if __name__ == "__main__":
    main()
