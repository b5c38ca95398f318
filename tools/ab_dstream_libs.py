"""Same-process A/B of two builds of the engine on device-resident packet runs
(GPU box): a 1 GiB run and one 128 MiB block through hdfs_crc32c_verify_packets
of each library, interleaved, best of N per round, 3 rounds (AB_ROUNDS).  Only the
round-4-stable entry points are bound, so any two builds compare.

    python tools/ab_dstream_libs.py BASE_LIB NEW_LIB [out.json]"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import device_stream_bench as dsb  # noqa: E402
import hadoofus_amd as h  # noqa: E402


def bind(path):
    lib = ctypes.CDLL(path, mode=os.RTLD_LOCAL | os.RTLD_NOW)
    f = lib.hdfs_crc32c_verify_packets
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_uint32, ctypes.c_int,
                  ctypes.POINTER(h.abi.Packet), ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t),
                  ctypes.POINTER(ctypes.c_uint64)]
    return lib


def best(lib, ptr, n, npk, reps):
    arr = (h.abi.Packet * (npk + 8))()
    cnt, used = ctypes.c_size_t(0), ctypes.c_uint64(0)
    t = 1e9
    for i in range(reps + 1):
        t0 = time.perf_counter()
        rc = lib.hdfs_crc32c_verify_packets(ptr, n, h.PROTO_V2, 512, h.CSUM_CRC32C, arr, npk + 8, ctypes.byref(cnt),
                                            ctypes.byref(used))
        if i:
            t = min(t, time.perf_counter() - t0)
        assert rc == 0 and cnt.value == npk, (rc, cnt.value)
    return t * 1e6


def main():
    base, new = bind(sys.argv[1]), bind(sys.argv[2])
    dsb.lib = h.load()
    out = {"base": sys.argv[1], "new": sys.argv[2], "rounds": []}
    imgs = []
    img, npk = dsb.wire_image(1 << 30, 7)
    imgs.append(("run_1GiB", img, npk))
    blk, nblk = dsb.wire_image(128 << 20, 9, empty_last=True)
    imgs.append(("block_128MiB", blk, nblk))
    devs = []
    for name, im, npk in imgs:
        d = h.DeviceBuffer(im.nbytes + 64)
        d.upload(im)
        devs.append((name, d, im.nbytes, npk))
    h.device_sync()
    for _ in range(int(os.environ.get("AB_ROUNDS", "3"))):
        r = {}
        for name, d, n, npk in devs:
            for tag, lib in (("base", base), ("new", new)):
                r[f"{name}_{tag}_us"] = round(best(lib, d.ptr, n, npk, 10), 1)
        out["rounds"].append(r)
    js = json.dumps(out)
    print(js)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(js + "\n")


if __name__ == "__main__":
    main()
