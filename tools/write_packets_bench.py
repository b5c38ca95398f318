"""Write-path packet composer rate (GPU box): hdfs_crc32c_compose_packets
over one 128 MiB block (2048 packets of 64 KiB + the finish packet), data
device-resident, in pinned host memory and in pageable host memory.
Prints one JSON object (GiB/s of payload, best of 5)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hadoofus_amd as h  # noqa: E402

BLOCK = 128 << 20
h.load()
dev = h.DeviceBuffer(BLOCK)
h.fill_splitmix64(dev.ptr, BLOCK // 8, 0, 0)
h.device_sync()
pin = h.PinnedBuffer(BLOCK)
dev.copy_to(pin.ptr)
pg = np.array(pin.array, copy=True)
sources = {
    "device": lambda: h.compose_packets(None, 0, 0, h.PROTO_V2, h.CSUM_CRC32C, True, dptr=dev.ptr, nbytes=BLOCK),
    "pinned": lambda: h.compose_packets(pin.array, 0, 0, h.PROTO_V2, h.CSUM_CRC32C, True),
    "pageable": lambda: h.compose_packets(pg, 0, 0, h.PROTO_V2, h.CSUM_CRC32C, True),
}
out = {"block_bytes": BLOCK}
ref = None
for name, fn in sources.items():
    best = 0.0
    for _ in range(5):
        t0 = time.perf_counter()
        hdr, pk = fn()
        best = max(best, BLOCK / (time.perf_counter() - t0) / (1 << 30))
        ref = hdr if ref is None else ref
        assert hdr == ref and len(pk) == 2049
    out[f"{name}_GiBps"] = round(best, 2)
out["header_bytes"] = len(ref)
# the C call alone (preallocated outputs, no Python-side packet dicts)
import ctypes  # noqa: E402
lib = h.load()
hdr_buf = np.zeros(len(ref), dtype=np.uint8)
arr = (h.abi.OutPacket * 2049)()
npk, used = ctypes.c_size_t(0), ctypes.c_uint64(0)
for name, ptr in (("device", dev.ptr), ("pinned", pin.ptr)):
    best = 0.0
    for _ in range(5):
        t0 = time.perf_counter()
        rc = lib.hdfs_crc32c_compose_packets(ptr, BLOCK, 0, 0, h.PROTO_V2, h.CSUM_CRC32C, 1, hdr_buf.ctypes.data,
                                             hdr_buf.nbytes, arr, 2049, ctypes.byref(npk), ctypes.byref(used))
        best = max(best, BLOCK / (time.perf_counter() - t0) / (1 << 30))
        assert rc == 0 and hdr_buf.tobytes() == ref
    out[f"{name}_c_call_GiBps"] = round(best, 2)
print(json.dumps(out))
