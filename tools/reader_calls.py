"""Per-call cost of a reader's deliveries (GPU box): a 128 MiB block of
64 KiB packets in device memory read through hdfs_crc32c_reader_* into
64 KiB device buffers, three reads each by launches, with the mailbox open
(default idle limit) and with a 1 s idle limit: open time, whole read, the
median / p99 / max of hdfs_crc32c_reader_next, and the mailbox's (calls,
launches) before open, after open and at the end -- one launch per mailbox
means it never idled out or was relaunched between reads.

    python tools/reader_calls.py [out.json]"""
import ctypes
import json
import sys
import time

import numpy as np
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import device_stream_bench as dsb  # noqa: E402
import hadoofus_amd as h  # noqa: E402

lib = h.load(); dsb.lib = lib
blk, npk = dsb.wire_image(128 << 20, 9, empty_last=True)
d = h.DeviceBuffer(blk.nbytes + 64); d.upload(blk); h.device_sync()
payload = 2048 * 65536
dst = h.DeviceBuffer(payload)
arr = (h.abi.Packet * (npk + 8))()
cnt, used, got = ctypes.c_size_t(0), ctypes.c_uint64(0), ctypes.c_uint64(0)
out = []
def run(piece, box):
    rd = ctypes.c_void_p()
    s0 = box.stats() if box else None
    t0 = time.perf_counter()
    assert lib.hdfs_crc32c_reader_open(d.ptr, blk.nbytes, h.PROTO_V2, 512, h.CSUM_CRC32C, 0, payload, npk + 8, ctypes.byref(rd)) == 0
    t_open = time.perf_counter() - t0
    s1 = box.stats() if box else None
    tot, ts = 0, []
    while True:
        vec = (h.abi.IoVec * 1)(h.abi.IoVec(dst.ptr + tot, min(piece, payload - tot)))
        a = time.perf_counter()
        rc = lib.hdfs_crc32c_reader_next(rd, vec, 1, arr, npk + 8, ctypes.byref(cnt), ctypes.byref(used), ctypes.byref(got))
        ts.append(time.perf_counter() - a)
        tot += got.value
        if rc != h.AGAIN: break
    t_all = time.perf_counter() - t0
    lib.hdfs_crc32c_reader_close(rd)
    ts = np.array(ts) * 1e6
    return {"open_us": round(t_open * 1e6, 1), "all_us": round(t_all * 1e6, 1), "next_med": round(float(np.median(ts)), 2),
            "next_p99": round(float(np.percentile(ts, 99)), 2), "next_max": round(float(ts.max()), 1),
            "stats": [s0, s1, box.stats() if box else None]}
for i in range(3): out.append(("launch", run(65536, None)))
with h.Mailbox() as box:
    for i in range(3): out.append(("mb", run(65536, box)))
with h.Mailbox(idle_ms=1000) as box:
    for i in range(3): out.append(("mb1000", run(65536, box)))
js = json.dumps(out)
print(js)
if len(sys.argv) > 1:
    open(sys.argv[1], "w").write(js + "\n")
