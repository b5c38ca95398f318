"""Host-resident (H2D + kernel + D2H) rate of the verify path, for DESIGN.md
and bench.py's extra.host_resident.  Data lives in host memory (pinned, and
separately pageable); the engine's pipeline overlaps copies with kernels --
the datanode's socket buffers (src/net.c:241-263, src/datanode.c) are host
memory, so this is the rate of the path as the reference's callers hold
their bytes.  GPU box only."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hadoofus_amd as h  # noqa: E402

GIB = 1 << 30


def measure(n_bytes=8 * GIB, pieces_mib=(64,), reps=3, cs=512):
    """Verify of n_bytes of host memory in pieces of pieces_mib MiB (best of
    reps), pinned and pageable (registered for the call), and compute at 64
    MiB pieces.  -> dict of GiB/s."""
    h.load()
    out = {"bytes": n_bytes, "chunk": cs}
    dev = h.DeviceBuffer(n_bytes)
    h.fill_splitmix64(dev.ptr, n_bytes // 8, 0, 0)
    h.device_sync()
    pin = h.PinnedBuffer(n_bytes)
    dev.copy_to(pin.ptr)
    dev.free()
    try:
        crcs = h.compute_host(pin.array, cs, flags=h.SEG_BE)
        for piece_mib in pieces_mib:
            best = 0.0
            for _ in range(reps):
                t0 = time.perf_counter()
                fb, m, bm = h.verify_host(pin.array, cs, crcs, flags=h.SEG_BE, piece_bytes=piece_mib << 20,
                                          want_bitmap=False)
                dt = time.perf_counter() - t0
                assert m == 0, m
                best = max(best, n_bytes / dt / GIB)
            out[f"pinned_verify_GiBps_piece{piece_mib}MiB"] = round(best, 2)
        t0 = time.perf_counter()
        crcs2 = h.compute_host(pin.array, cs, flags=h.SEG_BE, piece_bytes=64 << 20)
        out["pinned_compute_GiBps_piece64MiB"] = round(n_bytes / (time.perf_counter() - t0) / GIB, 2)
        assert np.array_equal(crcs, crcs2)
        # pageable host memory (registered by the engine for each call)
        pg = np.empty(n_bytes, dtype=np.uint8)
        pg[:] = pin.array
        best = 0.0
        for _ in range(max(1, reps - 1)):
            t0 = time.perf_counter()
            fb, m, bm = h.verify_host(pg, cs, crcs, flags=h.SEG_BE, piece_bytes=64 << 20, want_bitmap=False)
            best = max(best, n_bytes / (time.perf_counter() - t0) / GIB)
            assert m == 0
        out["pageable_verify_GiBps_incl_register_piece64MiB"] = round(best, 2)
        del pg
    finally:
        pin.free()
    return out


def packets_pinned(img, npk, reps=3):
    """hdfs_crc32c_verify_packets over a packet run in pinned host memory
    (framing walk on the host, H2D pieces, de-framing gather and verify on
    the GPU): GiB/s of payload, best of reps.  The C call alone is timed,
    into a preallocated record array (until round 6 the timed region also
    held the Python wrapper's conversion of 16 384 records to dicts, ~14 ms
    of the ~34 ms)."""
    import ctypes
    lib = h.load()
    pin = h.PinnedBuffer(img.nbytes)
    try:
        pin.array[:] = img
        arr = (h.abi.Packet * (npk + 8))()
        cnt, used = ctypes.c_size_t(0), ctypes.c_uint64(0)
        best = 1e9
        for _ in range(reps + 1):  # (the first call is a warm-up)
            t0 = time.perf_counter()
            rc = lib.hdfs_crc32c_verify_packets(pin.ptr, img.nbytes, h.PROTO_V2, 512, h.CSUM_CRC32C, arr, npk + 8,
                                                ctypes.byref(cnt), ctypes.byref(used))
            best = min(best, time.perf_counter() - t0)
            assert rc == 0 and cnt.value == npk and used.value == img.nbytes, (rc, cnt.value, used.value)
        assert all(arr[k].error == 0 and arr[k].data_len == 65536 for k in (0, npk // 2, npk - 1))
        return round(npk * 65536 / best / GIB, 2)
    finally:
        pin.free()


if __name__ == "__main__":
    n = int(float(os.environ.get("H2D_GIB", "8")) * GIB)
    print(json.dumps(measure(n, (16, 64, 256))))
