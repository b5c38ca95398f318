"""One synchronous hdfs_crc32c_verify_packets of a device-resident 128 MiB
block transfer (2 048 v2 packets + the empty last one), and of a one-packet
stream: best and median of `reps` calls (GPU box).  For runtime A/Bs that
are environment variables of the HIP runtime (run once per setting, in fresh
processes).

    python tools/block_latency.py [reps]"""
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import hadoofus_amd as h  # noqa: E402
import device_stream_bench as dsb  # noqa: E402


def times(lib, ptr, n, maxpk, reps):
    arr = (h.abi.Packet * maxpk)()
    cnt, used = ctypes.c_size_t(0), ctypes.c_uint64(0)
    out = []
    for _ in range(reps + 3):
        t0 = time.perf_counter()
        rc = lib.hdfs_crc32c_verify_packets(ptr, n, h.PROTO_V2, 512, h.CSUM_CRC32C, arr, maxpk, ctypes.byref(cnt),
                                            ctypes.byref(used))
        out.append(time.perf_counter() - t0)
        assert rc == 0 and used.value == n, (rc, used.value)
    out = out[3:]
    return {"best_us": round(min(out) * 1e6, 2), "median_us": round(statistics.median(out) * 1e6, 2)}


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    lib = h.load()
    dsb.lib = lib
    res = {"HIP_FORCE_DEV_KERNARG": os.environ.get("HIP_FORCE_DEV_KERNARG")}
    for key, size, empty in (("block_128MiB", 128 << 20, True), ("one_packet_64KiB", 65536, False)):
        img, npk = dsb.wire_image(size, 9, empty_last=empty)
        d = h.DeviceBuffer(img.nbytes + 64)
        d.upload(img)
        h.device_sync()
        res[key] = times(lib, d.ptr, img.nbytes, npk + 8, reps)
        d.free()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
