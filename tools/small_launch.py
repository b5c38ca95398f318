"""Small-launch costs (GPU box): per-execute device time of verify plans over
small inputs and many-segment tables, and the host-side latency of the
drop-in / datanode-mirror calls.  Prints one JSON object."""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hadoofus_amd as h  # noqa: E402

# --diag: the diagnostic build (HDFS_CRC32C_* knobs from the environment,
# e.g. HDFS_CRC32C_MB_STAGE=0 for the pinned mailbox stage); --quick: skip
# the plan timings
DIAG = "--diag" in sys.argv
QUICK = "--quick" in sys.argv
h.load(os.path.join(ROOT, "hadoofus_amd", "lib", "libhadoofus_crc32c_diag.so") if DIAG else h.abi.LIB_PATH)
cs = 512
total = 256 << 20
dbuf = h.DeviceBuffer(total)
h.fill_splitmix64(dbuf.ptr, total // 8, 0, 0)
crcs = h.DeviceBuffer(total // cs * 4)
bms = h.DeviceBuffer(total // cs // 8 + 64)
out = {}


def segs_of(seg_bytes, n):
    return [h.Segment(data=dbuf.ptr + i * seg_bytes, len=seg_bytes, chunk_size=cs, flags=h.SEG_BE, crc_init=0,
                      crcs=crcs.ptr + i * (seg_bytes // cs) * 4, bitmap=bms.ptr + i * (seg_bytes // cs // 8))
            for i in range(n)]


def plan_us(segs, iters):
    h.Plan(h.MODE_COMPUTE, segs).execute()
    vp = h.Plan(h.MODE_VERIFY, segs)
    vp.execute()
    _, m = vp.results()
    assert m == 0
    lib = h.load()
    ms = ctypes.c_double(0)
    assert lib.hdfs_crc32c_plan_time(vp.ptr, None, iters, ctypes.byref(ms)) == 0
    return ms.value * 1e3


for name, seg_bytes, n in [("1x64KiB", 65536, 1), ("1x1MiB", 1 << 20, 1), ("1x16MiB", 16 << 20, 1),
                           ("1x64MiB", 64 << 20, 1), ("1x256MiB", 256 << 20, 1),
                           ("1024x64KiB", 65536, 1024), ("4096x16KiB", 16384, 4096),
                           ("16x16MiB", 16 << 20, 16)][:1 if QUICK else None]:
    us = plan_us(segs_of(seg_bytes, n), 50 if seg_bytes * n <= (64 << 20) else 10)
    out[f"verify_{name}_us"] = round(us, 2)
    out[f"verify_{name}_GBps"] = round(seg_bytes * n * (1 + 4 / cs) / us / 1e3, 1)

# host-side call latency
x512 = np.frombuffer(os.urandom(512), np.uint8)
x64k = np.frombuffer(os.urandom(65536), np.uint8)
x4k = x64k[:4096].copy()
x64k1 = np.frombuffer(os.urandom(65537), np.uint8)
for name, buf in [("512B", x512), ("4KiB", x4k), ("64KiB", x64k), ("64KiB+1", x64k1)]:
    h.crc32c(0, buf)
    t0 = time.perf_counter()
    for _ in range(200):
        h.crc32c(0, buf)
    out[f"dropin_host_{name}_us"] = round((time.perf_counter() - t0) / 200 * 1e6, 1)
t0 = time.perf_counter()
for _ in range(200):
    h.stream_crc_dev(0, dbuf.ptr, 65536)
out["stream_dev_64KiB_us"] = round((time.perf_counter() - t0) / 200 * 1e6, 1)
be = h.compose_crcs([x64k.tobytes()], 512)
region = be + x64k.tobytes()
h.verify_crcdata(region, 512, len(be), 65536)
t0 = time.perf_counter()
for _ in range(200):
    rc, _ = h.verify_crcdata(region, 512, len(be), 65536)
    assert rc == 0
out["verify_crcdata_64KiB_us"] = round((time.perf_counter() - t0) / 200 * 1e6, 1)
# one received v2 packet of 64 KiB (+ the empty last packet) through the packet-run API
hdr = (b"\x09" + (0).to_bytes(8, "little") + b"\x11" + (0).to_bytes(8, "little") + b"\x18\x00\x25" +
       (65536).to_bytes(4, "little"))
last = (b"\x09" + (65536).to_bytes(8, "little") + b"\x11" + (1).to_bytes(8, "little") + b"\x18\x01\x25" +
        (0).to_bytes(4, "little"))
pkt = ((4 + len(be) + 65536).to_bytes(4, "big") + len(hdr).to_bytes(2, "big") + hdr + be + x64k.tobytes() +
       (4).to_bytes(4, "big") + len(last).to_bytes(2, "big") + last)
rc, recs, used = h.verify_packets(pkt)
assert rc == 0 and len(recs) == 2 and used == len(pkt), (rc, recs)
t0 = time.perf_counter()
for _ in range(200):
    h.verify_packets(pkt)
out["verify_packets_1x64KiB_us"] = round((time.perf_counter() - t0) / 200 * 1e6, 1)


def say(*a):
    print(*a, file=sys.stderr, flush=True)


def raw_call_us(prefix, iters=500):
    """Per-call wall time of the C entry points called directly through
    ctypes with prepared pointers (no numpy conversion per call)."""
    lib = h.load()
    reg = np.frombuffer(region, np.uint8).copy()
    fb = ctypes.c_int32(-1)
    for name, buf in [("512B", x512), ("4KiB", x4k), ("64KiB", x64k)]:
        p, n = buf.ctypes.data, buf.nbytes
        say(prefix, name)
        lib._hdfs_crc32c(0, p, n)
        t0 = time.perf_counter()
        for _ in range(iters):
            lib._hdfs_crc32c(0, p, n)
        out[f"{prefix}dropin_{name}_us"] = round((time.perf_counter() - t0) / iters * 1e6, 2)
    rp = reg.ctypes.data
    say(prefix, "verify_crcdata")
    assert lib.hdfs_crc32c_verify_crcdata(rp, 512, len(be), 65536, 2, ctypes.byref(fb)) == 0
    t0 = time.perf_counter()
    for _ in range(iters):
        lib.hdfs_crc32c_verify_crcdata(rp, 512, len(be), 65536, 2, ctypes.byref(fb))
    out[f"{prefix}verify_crcdata_64KiB_us"] = round((time.perf_counter() - t0) / iters * 1e6, 2)
    # the same 64 KiB packet verified as 4 KiB packets (verify_crcdata per packet, 16 calls)
    be4 = h.compose_crcs([x4k.tobytes()], 512)
    r4 = np.frombuffer(be4 + x4k.tobytes(), np.uint8).copy()
    t0 = time.perf_counter()
    for _ in range(iters):
        lib.hdfs_crc32c_verify_crcdata(r4.ctypes.data, 512, len(be4), 4096, 2, ctypes.byref(fb))
    out[f"{prefix}verify_crcdata_4KiB_us"] = round((time.perf_counter() - t0) / iters * 1e6, 2)
    # device-resident source (stream CRC of 64 KiB / 512 B in HBM, unaligned)
    o = ctypes.c_uint32(0)
    for name, n in (("64KiB", 65536), ("512B", 512)):
        lib.hdfs_crc32c_stream_dev(0, dbuf.ptr + 3, n, ctypes.byref(o))
        t0 = time.perf_counter()
        for _ in range(iters):
            lib.hdfs_crc32c_stream_dev(0, dbuf.ptr + 3, n, ctypes.byref(o))
        out[f"{prefix}stream_dev_{name}_unaligned_us"] = round((time.perf_counter() - t0) / iters * 1e6, 2)


# ctypes overhead of a trivial call (subtract by eye)
lib = h.load()
t0 = time.perf_counter()
for _ in range(20000):
    lib.hdfs_crc32c_last_error()
out["ctypes_call_overhead_us"] = round((time.perf_counter() - t0) / 20000 * 1e6, 3)
# what the launch-path calls pay for attributing faults: one hipStreamQuery
# of an idle stream after the completion word (small_call, small_run)
hip = ctypes.CDLL("libamdhip64.so.7")
hip.hipStreamQuery.argtypes = [ctypes.c_void_p]
sq = h.stream_create()
h.stream_sync(sq)
assert hip.hipStreamQuery(sq) == 0
t0 = time.perf_counter()
for _ in range(20000):
    hip.hipStreamQuery(sq)
out["hip_stream_query_us"] = round((time.perf_counter() - t0) / 20000 * 1e6 - out["ctypes_call_overhead_us"], 3)
say("launch path")
raw_call_us("launch_")
say("mailbox")
with h.Mailbox() as mb:
    raw_call_us("mailbox_")
    out["mailbox_calls_launches"] = list(mb.stats())
out["mailbox_stage_env"] = os.environ.get("HDFS_CRC32C_MB_STAGE", "default")
print(json.dumps(out))
