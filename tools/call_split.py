"""Where a 1 GiB device-stream verify call spends its host time: 12 calls of
hdfs_crc32c_verify_packets over the composed 1 GiB run (16 384 packets),
each timed from Python; run with HDFS_CRC32C_DSTREAM_TRACE=1 so the library
prints its own split (walk / after the walk) to stderr.  Prints one JSON
list of per-call microseconds (the first call is the warm-up)."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import hadoofus_amd as h  # noqa: E402
import device_stream_bench as dsb  # noqa: E402


def main():
    lib = h.load()
    img, npk = dsb.wire_image(1 << 30, 7)
    d = h.DeviceBuffer(len(img))
    d.upload(img)
    h.device_sync()
    arr = (h.abi.Packet * (npk + 8))()
    cnt, used = ctypes.c_size_t(0), ctypes.c_uint64(0)
    out = []
    for _ in range(12):
        t0 = time.perf_counter()
        rc = lib.hdfs_crc32c_verify_packets(d.ptr, len(img), h.PROTO_V2, 512, h.CSUM_CRC32C, arr, npk + 8,
                                            ctypes.byref(cnt), ctypes.byref(used))
        out.append(round((time.perf_counter() - t0) * 1e6, 1))
        assert rc == 0 and cnt.value == npk and used.value == len(img), (rc, cnt.value, used.value)
    d.free()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
