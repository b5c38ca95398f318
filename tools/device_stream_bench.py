"""Device-resident packet-stream verify (GPU box): hdfs_crc32c_verify_packets
over a 1 GiB v2 packet run already in HBM (16384 packets of 64 KiB, the
wire image of 8 block transfers, composed by hdfs_crc32c_compose_packets),
against the same run in pinned host memory (H2D piece pipeline), and the
latency of short runs.  Prints one JSON object: GiB/s of payload per call,
best of 5, C call with preallocated records."""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hadoofus_amd as h  # noqa: E402

if os.environ.get("DSB_LIB"):  # another build of the library (A/B of a change, same box)
    lib = h.load(os.environ["DSB_LIB"])
elif os.environ.get("DSB_DIAG"):  # the diagnostic build (takes HDFS_CRC32C_* knobs from the environment)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import diaglib  # noqa: E402
    lib = h.load(diaglib.DIAG_LIB_PATH)
else:
    lib = h.load()
# DSB_OLD_COPY: a round-2 build (verify_packets_copy without the read window)
OLD_COPY = bool(os.environ.get("DSB_OLD_COPY"))
if OLD_COPY:
    _P = ctypes.POINTER
    lib.hdfs_crc32c_verify_packets_copy.argtypes = [
        ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_uint32, ctypes.c_int, _P(h.abi.Packet), ctypes.c_size_t,
        _P(ctypes.c_size_t), _P(ctypes.c_uint64), ctypes.c_void_p, ctypes.c_uint64, _P(ctypes.c_uint64)]


def wire_image(nbytes, seed):
    """Composed v2 packets of nbytes of device-filled payload -> host bytes."""
    dev = h.DeviceBuffer(nbytes)
    h.fill_splitmix64(dev.ptr, nbytes // 8, seed, 0)
    h.device_sync()
    hdr, pk = h.compose_packets(None, 0, 0, h.PROTO_V2, h.CSUM_CRC32C, False, dptr=dev.ptr, nbytes=nbytes)
    data = dev.download()
    dev.free()
    hb = np.frombuffer(hdr, np.uint8)
    H = pk[0]["hdr_len"]
    assert all(p["hdr_len"] == H and p["data_len"] == 65536 for p in pk)
    out = np.concatenate([hb.reshape(len(pk), H), data.reshape(len(pk), 65536)], axis=1).reshape(-1)
    return out, len(pk)


def timed(ptr, n, npk, reps=5, fn="hdfs_crc32c_verify_packets", dst=None):
    arr = (h.abi.Packet * (npk + 8))()
    cnt, used, got = ctypes.c_size_t(0), ctypes.c_uint64(0), ctypes.c_uint64(0)
    best, rc = 1e9, None
    for i in range(reps + 1):  # the first call is a warm-up (buffer growth, clocks)
        t0 = time.perf_counter()
        if dst is not None:  # verify + fused copy-out
            win = () if OLD_COPY else (0, h.READ_ALL)
            rc = lib.hdfs_crc32c_verify_packets_copy(ptr, n, h.PROTO_V2, 512, h.CSUM_CRC32C, *win, arr, npk + 8,
                                                     ctypes.byref(cnt), ctypes.byref(used), dst.ptr, dst.nbytes,
                                                     ctypes.byref(got))
        else:
            rc = getattr(lib, fn)(ptr, n, h.PROTO_V2, 512, h.CSUM_CRC32C, arr, npk + 8, ctypes.byref(cnt),
                                  ctypes.byref(used))
        if i:
            best = min(best, time.perf_counter() - t0)
    assert rc >= 0 and cnt.value == npk and used.value == n, (rc, cnt.value, used.value)
    return best, rc, arr


out = {}
N = 1 << 30
img, npk = wire_image(N, 7)
payload = npk * 65536
dev = h.DeviceBuffer(img.nbytes + 64)
dev.upload(img)
pin = h.PinnedBuffer(img.nbytes)
pin.array[:] = img
h.device_sync()
t_dev, rc, _ = timed(dev.ptr, img.nbytes, npk)
assert rc == 0
dst = h.DeviceBuffer(payload)
t_copy, rc, _ = timed(dev.ptr, img.nbytes, npk, dst=dst)
assert rc == 0
# the copied-out payload is the de-framed data, byte for byte
H0 = img.nbytes // npk - 65536
want = img.reshape(npk, H0 + 65536)[:, H0:].reshape(-1)
copy_ok = bool(np.array_equal(dst.download(), want))
if os.environ.get("DSB_POLICIES"):  # diagnostic build: copy-out store policies, interleaved rounds
    pols = [int(x) for x in os.environ["DSB_POLICIES"].split(",")]
    res = {p: [] for p in pols}
    for _ in range(4):
        for p in pols:
            assert lib.hdfs_crc32c_set_store_policy(p) == 0
            t, rc, _ = timed(dev.ptr, img.nbytes, npk, dst=dst)
            res[p].append(round(payload / t / 2**30, 1))
            assert bool(np.array_equal(dst.download(), want)), p
    lib.hdfs_crc32c_set_store_policy(0)
    out["copy_policy_GiBps"] = {str(p): v for p, v in res.items()}
# ceiling for verify + copy-out: a plain device-to-device copy of the same
# payload bytes (hipMemcpy D2D: one read and one write of HBM, no CRC work)
best_cp = 1e9
for _ in range(5):
    h.device_sync()
    t0 = time.perf_counter()
    assert lib.hdfs_crc32c_memcpy(dst.ptr, dev.ptr, payload, 2) == 0
    h.device_sync()
    best_cp = min(best_cp, time.perf_counter() - t0)
out["d2d_copy_GiBps"] = round(payload / best_cp / 2**30, 1)
t_parse, rc, _ = timed(dev.ptr, img.nbytes, npk, fn="hdfs_crc32c_parse_packets")
assert rc == 0
t_hparse, rc, _ = timed(pin.ptr, img.nbytes, npk, fn="hdfs_crc32c_parse_packets")
assert rc == 0
t_pin, rc, _ = timed(pin.ptr, img.nbytes, npk, reps=3)
assert rc == 0
out.update(packets=npk, wire_bytes=int(img.nbytes), device_GiBps=round(payload / t_dev / 2**30, 1),
           device_ms=round(t_dev * 1e3, 3), device_parse_ms=round(t_parse * 1e3, 3),
           host_parse_ms=round(t_hparse * 1e3, 3), pinned_GiBps=round(payload / t_pin / 2**30, 1),
           device_copy_GiBps=round(payload / t_copy / 2**30, 1), device_copy_ms=round(t_copy * 1e3, 3),
           copy_bytes_exact=copy_ok)
# one flipped bit per 1000th packet: verdicts come back for exactly those
flips = list(range(5, npk, 1000))
H = img.nbytes // npk - 65536
for k in flips:
    img[k * (H + 65536) + H + 100] ^= 1
dev.upload(img)
h.device_sync()
t_bad, rc, arr = timed(dev.ptr, img.nbytes, npk)
assert rc == 29 and [i for i in range(npk) if arr[i].error] == flips
assert all(arr[i].first_bad == 0 and arr[i].bad_chunks == 1 for i in flips)
out["device_corrupt_ms"] = round(t_bad * 1e3, 3)
# small runs: one 64 KiB packet, and 64 packets (4 MiB)
for npk_s in (1, 64):
    n = npk_s * (H + 65536)
    t, rc, _ = timed(dev.ptr, n, npk_s, reps=20)
    out[f"device_{npk_s}pkt_us"] = round(t * 1e6, 1)
    t, rc, _ = timed(dev.ptr, n, npk_s, reps=20, dst=dst)
    out[f"device_copy_{npk_s}pkt_us"] = round(t * 1e6, 1)
dst.free()
dev.free()
pin.free()
print(json.dumps(out))
