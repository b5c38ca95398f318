"""Diagnostic (GPU box): run the shape-test table (64 x 16 MiB, chunk sizes
512..4096, partial last tiles) in compute mode through LIB_TEST, CRC arrays
pre-filled with a sentinel, and compare with LIB_REF's CRCs; report which
(segment, tile) came back unwritten or wrong.  Usage:
    python tools/exp_lost_tiles.py LIB_REF LIB_TEST [reps]"""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from exp_ab_libs import Seg, chk, open_lib  # noqa: E402

SEG, NSEG = 16 << 20, 64
SENT = 0xA5A5A5A5


def run(lib, order, depth, streams, block, nt, data, crcbufs, segs):
    chk(lib, lib.hdfs_crc32c_set_tile_order(order))
    chk(lib, lib.hdfs_crc32c_set_depth(depth))
    chk(lib, lib.hdfs_crc32c_set_shape(streams, block))
    chk(lib, lib.hdfs_crc32c_set_tuning(nt, None))
    arr = (Seg * NSEG)(*segs)
    plan = ctypes.c_void_p()
    chk(lib, lib.hdfs_crc32c_plan_create(ctypes.byref(plan), 0, arr, NSEG))
    chk(lib, lib.hdfs_crc32c_plan_execute(plan, None))
    chk(lib, lib.hdfs_crc32c_device_sync())
    lib.hdfs_crc32c_plan_destroy(plan)


def main():
    ref, test = open_lib(sys.argv[1]), open_lib(sys.argv[2])
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    out = {}
    for lib in (ref, test):
        lib.hdfs_crc32c_set_tile_order.restype = ctypes.c_int
        lib.hdfs_crc32c_set_depth.restype = ctypes.c_int
        lib.hdfs_crc32c_set_shape.restype = ctypes.c_int
        lib.hdfs_crc32c_set_tuning.restype = ctypes.c_int
        lib.hdfs_crc32c_memset.restype = ctypes.c_int
    sizes = [512 << (i % 4) for i in range(NSEG)]
    lens = [SEG - (i % 5) * cs for i, cs in enumerate(sizes)]
    nch = [n // cs for cs, n in zip(sizes, lens)]
    res = {}
    for name, lib in (("ref", ref), ("test", test)):
        d = ctypes.c_void_p()
        chk(lib, lib.hdfs_crc32c_dev_alloc(ctypes.byref(d), NSEG * SEG))
        chk(lib, lib.hdfs_crc32c_fill_splitmix64(d, NSEG * SEG // 8, ctypes.c_uint64(5), ctypes.c_uint64(0), None))
        bufs = []
        for n in nch:
            b = ctypes.c_void_p()
            chk(lib, lib.hdfs_crc32c_dev_alloc(ctypes.byref(b), n * 4))
            bufs.append(b)
        segs = [Seg(d.value + i * SEG, lens[i], cs, 0, 0, 0, bufs[i].value, None) for i, cs in enumerate(sizes)]
        res[name] = (lib, bufs, segs)
    # reference CRCs
    lib, bufs, segs = res["ref"]
    run(lib, 3, 3, 1, 1024, 2, None, bufs, segs)
    want = []
    for b, n in zip(bufs, nch):
        h = np.empty(n, np.uint32)
        chk(lib, lib.hdfs_crc32c_memcpy(ctypes.c_void_p(h.ctypes.data), b, n * 4, 1))
        want.append(h)
    lib, bufs, segs = res["test"]
    for shape in ((3, 3, 1, 1024, 1), (3, 3, 1, 1024, 2), (2, 3, 1, 1024, 1), (3, 4, 1, 1024, 1)):
        for r in range(reps):
            for b, n in zip(bufs, nch):
                chk(lib, lib.hdfs_crc32c_memset(b, 0xA5, n * 4))
            run(lib, *shape, None, bufs, segs)
            bad = []
            for i, (b, n) in enumerate(zip(bufs, nch)):
                h = np.empty(n, np.uint32)
                chk(lib, lib.hdfs_crc32c_memcpy(ctypes.c_void_p(h.ctypes.data), b, n * 4, 1))
                idx = np.nonzero(h != want[i])[0]
                if len(idx):
                    tiles = sorted(set((idx // 8).tolist()))
                    bad.append({"seg": i, "n": int(len(idx)), "unwritten": int((h[idx] == SENT).sum()),
                                "tiles": tiles[:20], "ntiles": len(tiles), "seg_tiles": (n + 7) // 8})
            out.setdefault(str(shape), []).append(bad)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
