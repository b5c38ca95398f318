"""Binary A/B (GPU box): two builds of libhadoofus_crc32c.so loaded side by
side in ONE process (RTLD_LOCAL, each with its own engine context, same HIP
runtime and device), timing the same verify / compute plans over the same
128 GiB of device data in interleaved rounds.  For changes that cannot be a
runtime knob (compiler flags, code restructuring).

    python tools/exp_ab_libs.py LIB_A LIB_B [rounds]
Prints one JSON object (GB/s of payload, medians) and checks that both
builds produce identical CRCs and verify verdicts."""
import ctypes
import json
import os
import statistics
import sys

BLOCK = 128 << 20
B = int(os.environ.get("BLOCKS", "1024"))
CS = 512


class Seg(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("len", ctypes.c_uint64), ("chunk_size", ctypes.c_uint32),
                ("flags", ctypes.c_uint32), ("crc_init", ctypes.c_uint32), ("pad", ctypes.c_uint32),
                ("crcs", ctypes.c_void_p), ("bitmap", ctypes.c_void_p)]


def open_lib(path):
    lib = ctypes.CDLL(path, mode=os.RTLD_LOCAL | os.RTLD_NOW)
    for n in ("hdfs_crc32c_dev_alloc", "hdfs_crc32c_fill_splitmix64", "hdfs_crc32c_plan_create",
              "hdfs_crc32c_plan_execute", "hdfs_crc32c_plan_time", "hdfs_crc32c_plan_results",
              "hdfs_crc32c_device_sync", "hdfs_crc32c_stream_dev", "hdfs_crc32c_corrupt", "hdfs_crc32c_init",
              "hdfs_crc32c_memcpy"):
        getattr(lib, n).restype = ctypes.c_int
    lib.hdfs_crc32c_last_error.restype = ctypes.c_char_p
    return lib


def chk(lib, rc):
    if rc:
        raise RuntimeError(lib.hdfs_crc32c_last_error().decode())


def main():
    la, lb = open_lib(sys.argv[1]), open_lib(sys.argv[2])
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    chk(la, la.hdfs_crc32c_init(-1))
    chk(lb, lb.hdfs_crc32c_init(-1))
    ptr = lambda: ctypes.c_void_p()  # noqa: E731
    data, crcs, crcs2, bms = ptr(), ptr(), ptr(), ptr()
    nch = B * BLOCK // CS
    chk(la, la.hdfs_crc32c_dev_alloc(ctypes.byref(data), ctypes.c_uint64(B * BLOCK)))
    chk(la, la.hdfs_crc32c_dev_alloc(ctypes.byref(crcs), ctypes.c_uint64(nch * 4)))
    chk(la, la.hdfs_crc32c_dev_alloc(ctypes.byref(crcs2), ctypes.c_uint64(nch * 4)))
    chk(la, la.hdfs_crc32c_dev_alloc(ctypes.byref(bms), ctypes.c_uint64(nch // 8)))
    chk(la, la.hdfs_crc32c_fill_splitmix64(data, ctypes.c_uint64(B * BLOCK // 8), ctypes.c_uint64(0),
                                           ctypes.c_uint64(0), None))
    chk(la, la.hdfs_crc32c_device_sync())

    def segs(crc_ptr, with_bm):
        arr = (Seg * B)()
        for b in range(B):
            arr[b] = Seg(data.value + b * BLOCK, BLOCK, CS, 1, 0, 0, crc_ptr + b * (BLOCK // CS) * 4,
                         (bms.value + b * (BLOCK // CS) // 8) if with_bm else None)
        return arr

    plans = {}
    for name, lib in (("A", la), ("B", lb)):
        for mode, (cp, bm) in ((0, (crcs2.value, False)), (1, (crcs.value, True))):
            p = ctypes.c_void_p()
            s = segs(cp, bm)
            chk(lib, lib.hdfs_crc32c_plan_create(ctypes.byref(p), mode, s, ctypes.c_size_t(B)))
            plans[(name, mode)] = (lib, p)
    # expected CRCs from A, then the bench's corruption pattern
    lib, p = plans[("A", 0)]
    chk(lib, lib.hdfs_crc32c_plan_execute(p, None))
    chk(la, la.hdfs_crc32c_device_sync())
    chk(la, la.hdfs_crc32c_memcpy(crcs, crcs2, ctypes.c_uint64(nch * 4), 2))
    for b in range(B):
        chk(la, la.hdfs_crc32c_corrupt(ctypes.c_void_p(data.value + b * BLOCK), ctypes.c_uint64(BLOCK),
                                       ctypes.c_uint32(CS), ctypes.c_uint64(b * (BLOCK // CS)),
                                       ctypes.c_uint64(65537), ctypes.c_uint64(7919), None))
    chk(la, la.hdfs_crc32c_device_sync())
    res, digests, mism = {}, {}, {}
    for _ in range(rounds):
        for name in ("A", "B"):
            for mode in (0, 1):
                lib, p = plans[(name, mode)]
                ms = ctypes.c_double(0)
                chk(lib, lib.hdfs_crc32c_plan_time(p, None, 3, ctypes.byref(ms)))
                res.setdefault(f"{'compute' if mode == 0 else 'verify'}_{name}", []).append(
                    B * BLOCK / (ms.value * 1e-3) / 1e9)
                if mode == 0:
                    d = ctypes.c_uint32(0)
                    chk(lib, lib.hdfs_crc32c_stream_dev(0, crcs2, ctypes.c_uint64(nch * 4), ctypes.byref(d)))
                    digests.setdefault(name, set()).add(d.value)
                else:
                    fb = (ctypes.c_uint32 * B)()
                    m = ctypes.c_uint64(0)
                    chk(lib, lib.hdfs_crc32c_plan_results(p, None, fb, ctypes.c_size_t(B), ctypes.byref(m)))
                    mism.setdefault(name, set()).add(m.value)
    out = {"lib_a": sys.argv[1], "lib_b": sys.argv[2], "blocks": B, "rounds": rounds}
    out.update({k + "_GBps_median": round(statistics.median(v), 1) for k, v in res.items()})
    out["same_crcs"] = digests["A"] == digests["B"] and len(digests["A"]) == 1
    out["mismatches"] = {k: sorted(v) for k, v in mism.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
