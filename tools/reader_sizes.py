"""Per-call cost of hdfs_crc32c_reader_next by piece size (GPU box): a
128 MiB block of 64 KiB packets in device memory, one reader per pass, the
whole read delivered in pieces of 16 KiB .. 8 MiB into a device buffer, by
launches and with the mailbox (latency mode) open; and the same read in ONE
hdfs_crc32c_read_packets call over 64 buffers.  Prints one JSON line
{"launch"|"mailbox": {piece: {"us_per_call", "GiBps", "calls"}}, "scatter_64"};
run it under
rocprofv3 --kernel-trace --stats to split the call into copy_pieces_kernel
time and the rest.

    python tools/reader_sizes.py [out.json]"""
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


def main():
    lib = h.load()
    dsb.lib = lib
    img, npk = dsb.wire_image(128 << 20, 9, empty_last=True)
    d = h.DeviceBuffer(img.nbytes + 64)
    d.upload(img)
    payload = (npk - 1) * 65536
    dst = h.DeviceBuffer(payload + (8 << 20))
    h.device_sync()
    arr = (h.abi.Packet * (npk + 8))()
    cnt, used, got = ctypes.c_size_t(0), ctypes.c_uint64(0), ctypes.c_uint64(0)
    out = {}
    out["launch"] = sweep(lib, d, img, npk, payload, dst, arr, cnt, used, got)
    with h.Mailbox():  # the latency mode: deliveries <= 1 MiB copied by the resident kernel
        out["mailbox"] = sweep(lib, d, img, npk, payload, dst, arr, cnt, used, got)
    # one call over 64 device buffers (the verify once + one table copy launch)
    sl = payload // 64
    vec = (h.abi.IoVec * 64)(*[h.abi.IoVec(dst.ptr + k * sl, sl) for k in range(64)])
    best = 1e9
    for rep in range(6):
        t0 = time.perf_counter()
        rc = lib.hdfs_crc32c_read_packets(d.ptr, img.nbytes, h.PROTO_V2, 512, h.CSUM_CRC32C, 0, payload, vec, 64, arr,
                                          npk + 8, ctypes.byref(cnt), ctypes.byref(used), ctypes.byref(got))
        t = time.perf_counter() - t0
        assert rc == 0 and got.value == payload, (rc, got.value)
        if rep:
            best = min(best, t)
    out["scatter_64"] = {"us": round(best * 1e6, 1), "GiBps": round(payload / best / 2**30, 2)}
    js = json.dumps(out)
    print(js)
    if len(sys.argv) > 1:
        open(sys.argv[1], "w").write(js + "\n")


def sweep(lib, d, img, npk, payload, dst, arr, cnt, used, got):
    out = {}
    for piece in (16 << 10, 64 << 10, 256 << 10, 1 << 20, 4 << 20, 8 << 20):
        best = 1e9
        for rep in range(4):
            rd = ctypes.c_void_p()
            assert lib.hdfs_crc32c_reader_open(d.ptr, img.nbytes, h.PROTO_V2, 512, h.CSUM_CRC32C, 0, payload,
                                               npk + 8, ctypes.byref(rd)) == 0
            tot, calls = 0, 0
            t0 = time.perf_counter()
            while True:
                vec = (h.abi.IoVec * 1)(h.abi.IoVec(dst.ptr + tot, min(piece, payload - tot)))
                rc = lib.hdfs_crc32c_reader_next(rd, vec, 1, arr, npk + 8, ctypes.byref(cnt), ctypes.byref(used),
                                                 ctypes.byref(got))
                calls += 1
                tot += got.value
                if rc != h.AGAIN:
                    break
            t = time.perf_counter() - t0
            lib.hdfs_crc32c_reader_close(rd)
            assert rc == 0 and tot == payload, (rc, tot)
            if rep:
                best = min(best, t)
        out[piece] = {"us_per_call": round(best * 1e6 / calls, 2), "GiBps": round(payload / best / 2**30, 2),
                      "calls": calls}
    return out


if __name__ == "__main__":
    main()
