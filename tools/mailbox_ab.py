"""Mailbox latency A/B (GPU box): two builds of libhadoofus_crc32c.so loaded
side by side in ONE process (RTLD_LOCAL, each with its own engine context and
its own resident mailbox), timing the same raw C calls in interleaved rounds.
Per-call wall time (perf_counter_ns around each call), median and mean.

    python tools/mailbox_ab.py LIB_A LIB_B [rounds]
Prints one JSON object and checks that both builds return the same values."""
import ctypes
import json
import os
import statistics
import sys
import time

import numpy as np


def open_lib(path):
    lib = ctypes.CDLL(path, mode=os.RTLD_LOCAL | os.RTLD_NOW)
    for n in ("hdfs_crc32c_mailbox_create", "hdfs_crc32c_mailbox_destroy", "hdfs_crc32c_verify_crcdata",
              "hdfs_crc32c_stream_dev", "hdfs_crc32c_dev_alloc", "hdfs_crc32c_memcpy", "hdfs_crc32c_device_sync",
              "hdfs_crc32c_compose_crcs"):
        getattr(lib, n).restype = ctypes.c_int
    lib._hdfs_crc32c.restype = ctypes.c_uint32
    lib._hdfs_crc32c.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]
    lib.hdfs_crc32c_last_error.restype = ctypes.c_char_p
    return lib


def main():
    paths = sys.argv[1:3]
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    iters = 200
    libs = [open_lib(p) for p in paths]
    rng = np.random.default_rng(3)
    x64k = rng.integers(0, 256, 65536, dtype=np.uint8)
    # wire CRCs of the 64 KiB packet (BE, 512-B chunks) from build A's compose
    crcs = np.zeros(128, np.uint32)
    iov = (ctypes.c_void_p * 1)(x64k.ctypes.data)
    ln = (ctypes.c_size_t * 1)(65536)
    assert libs[0].hdfs_crc32c_compose_crcs(iov, ln, 1, ctypes.c_size_t(65536), 512, 2,
                                            ctypes.c_void_p(crcs.ctypes.data)) == 0
    region = np.concatenate([crcs.view(np.uint8), x64k])
    mbs, dbufs = [], []
    for lib in libs:
        mb = ctypes.c_void_p()
        assert lib.hdfs_crc32c_mailbox_create(ctypes.byref(mb), 0) == 0, lib.hdfs_crc32c_last_error()
        mbs.append(mb)
        d = ctypes.c_void_p()
        assert lib.hdfs_crc32c_dev_alloc(ctypes.byref(d), 65536 + 64) == 0
        assert lib.hdfs_crc32c_memcpy(d, ctypes.c_void_p(x64k.ctypes.data), ctypes.c_uint64(65536), 0) == 0
        dbufs.append(d)
    fb = ctypes.c_int32(-1)
    o = ctypes.c_uint32(0)
    rp = ctypes.c_void_p(region.ctypes.data)

    def cases(lib, d):
        return {
            "dropin_512B": lambda: lib._hdfs_crc32c(0, x64k.ctypes.data, 512),
            "dropin_4KiB": lambda: lib._hdfs_crc32c(0, x64k.ctypes.data, 4096),
            "dropin_64KiB": lambda: lib._hdfs_crc32c(0, x64k.ctypes.data, 65536),
            "verify_crcdata_64KiB": lambda: lib.hdfs_crc32c_verify_crcdata(rp, 512, 512, 65536, 2,
                                                                          ctypes.byref(fb)),
            "stream_dev_64KiB": lambda: (lib.hdfs_crc32c_stream_dev(0, d, ctypes.c_uint64(65536), ctypes.byref(o)),
                                         o.value)[1],
        }

    per = [cases(lib, d) for lib, d in zip(libs, dbufs)]
    for name in per[0]:
        assert per[0][name]() == per[1][name](), name
    samples = [{n: [] for n in per[0]} for _ in libs]
    for _ in range(rounds):
        for k, cs in enumerate(per):
            for n, f in cs.items():
                f()
                for _ in range(iters):
                    t0 = time.perf_counter_ns()
                    f()
                    samples[k][n].append((time.perf_counter_ns() - t0) / 1e3)
    out = {"libs": paths, "rounds": rounds, "iters": iters}
    for n in per[0]:
        for k, tag in enumerate("AB"):
            s = samples[k][n]
            out[f"{tag}_{n}_median_us"] = round(statistics.median(s), 2)
            out[f"{tag}_{n}_mean_us"] = round(statistics.fmean(s), 2)
    for lib, mb in zip(libs, mbs):
        lib.hdfs_crc32c_mailbox_destroy(mb)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
