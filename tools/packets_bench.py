"""Host-resident packet-stream verify rate (hdfs_crc32c_verify_packets), for
DESIGN.md: a v2 stream of 64 KiB packets (512-B chunks, CRC32C), as the
datanode's recvbuf would hold it, verified end to end (host framing walk,
H2D in 64 MiB pieces, de-framing gather + verify kernels, D2H of results).
Expected CRCs are produced by the engine's own compute path.  GPU box only."""
import json
import os
import struct
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hadoofus_amd as h  # noqa: E402

GIB = 1 << 30
n_pk = int(os.environ.get("PK_PACKETS", "16384"))  # 1 GiB of payload
dlen, cs = 65536, 512
h.load()
payload_bytes = n_pk * dlen
dev = h.DeviceBuffer(payload_bytes)
h.fill_splitmix64(dev.ptr, payload_bytes // 8, 0, 0)
data = np.empty(payload_bytes, np.uint8)
dev.copy_to(data.ctypes.data)
dev.free()
crcs = h.compute_host(data, cs, flags=h.SEG_BE).view(np.uint8)  # BE bytes
ncrc = dlen // cs * 4
hdr_len = 6 + 25
pk_len = hdr_len + ncrc + dlen
total = n_pk * pk_len + 6 + 25
pin = h.PinnedBuffer(total)
s = pin.array
for k in range(n_pk):
    o = k * pk_len
    body = (b"\x09" + struct.pack("<q", k * dlen) + b"\x11" + struct.pack("<q", k) + b"\x18\x00" +
            b"\x25" + struct.pack("<i", dlen))
    s[o:o + hdr_len] = np.frombuffer(struct.pack(">iH", 4 + ncrc + dlen, 25) + body, np.uint8)
    s[o + hdr_len:o + hdr_len + ncrc] = crcs[k * ncrc:(k + 1) * ncrc]
    s[o + hdr_len + ncrc:o + pk_len] = data[k * dlen:(k + 1) * dlen]
body = (b"\x09" + struct.pack("<q", n_pk * dlen) + b"\x11" + struct.pack("<q", n_pk) + b"\x18\x01" +
        b"\x25" + struct.pack("<i", 0))
s[n_pk * pk_len:] = np.frombuffer(struct.pack(">iH", 4, 25) + body, np.uint8)
# one corrupted chunk per 1024 packets
for k in range(0, n_pk, 1024):
    s[k * pk_len + hdr_len + ncrc + 777] ^= 1

out = {"packets": n_pk, "data_len": dlen, "chunk": cs, "stream_bytes": total, "payload_bytes": payload_bytes}
rc, pk, used = h.verify_packets(s, max_pkts=n_pk + 1)  # warm-up (allocations)
assert rc == h.ERR_BAD_CHECKSUM and used == total, (rc, used, total)
assert sum(1 for p in pk if p["error"]) == len(range(0, n_pk, 1024))
import ctypes  # noqa: E402
arr = (h.Packet * (n_pk + 1))()
npk, usd = ctypes.c_size_t(0), ctypes.c_uint64(0)


def raw_call(fn, buf):
    return getattr(h.load(), fn)(buf.ctypes.data, buf.nbytes, h.PROTO_V2, cs, h.CSUM_CRC32C, arr, n_pk + 1,
                                 ctypes.byref(npk), ctypes.byref(usd))


best = 0.0
for _ in range(5):
    t0 = time.perf_counter()
    assert raw_call("hdfs_crc32c_verify_packets", s) == h.ERR_BAD_CHECKSUM
    best = max(best, payload_bytes / (time.perf_counter() - t0) / GIB)
out["pinned_verify_payload_GiBps"] = round(best, 2)
t0 = time.perf_counter()
raw_call("hdfs_crc32c_parse_packets", s)
out["host_framing_walk_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
pg = np.empty(total, np.uint8)
pg[:] = s
t0 = time.perf_counter()
assert raw_call("hdfs_crc32c_verify_packets", pg) == h.ERR_BAD_CHECKSUM
out["pageable_verify_payload_GiBps_incl_register"] = round(payload_bytes / (time.perf_counter() - t0) / GIB, 2)
# streaming session: 8 MiB "socket reads" memmoved into the session's pinned
# slots (the copy stands in for recv() landing in the slot)
sess = h.Session()
arr2 = (h.Packet * 4096)()
n2 = ctypes.c_size_t(0)
lib = h.load()
t0 = time.perf_counter()
got_pk = got_bad = 0
off = 0
while off < total:
    w, room = sess.buffer()
    n = min(room, 8 << 20, total - off)
    ctypes.memmove(w, s.ctypes.data + off, n)
    assert lib.hdfs_crc32c_session_commit(sess.ptr, n) == 0
    off += n
    lib.hdfs_crc32c_session_poll(sess.ptr, arr2, 4096, ctypes.byref(n2), 0)
    got_pk += n2.value
    got_bad += sum(1 for i in range(n2.value) if arr2[i].error)
sess.flush()
while True:
    lib.hdfs_crc32c_session_poll(sess.ptr, arr2, 4096, ctypes.byref(n2), 1)
    if not n2.value:
        break
    got_pk += n2.value
    got_bad += sum(1 for i in range(n2.value) if arr2[i].error)
out["session_payload_GiBps_incl_slot_copy"] = round(payload_bytes / (time.perf_counter() - t0) / GIB, 2)
assert got_pk == n_pk + 1 and got_bad == len(range(0, n_pk, 1024)), (got_pk, got_bad)
sess.close()
t0 = time.perf_counter()
for off in range(0, total, 8 << 20):
    ctypes.memmove(pg.ctypes.data + off, s.ctypes.data + off, min(8 << 20, total - off))
out["host_memmove_GiBps_same_pattern"] = round(total / (time.perf_counter() - t0) / GIB, 2)
pin.free()
print(json.dumps(out))
