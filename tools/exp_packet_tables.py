"""Verify rate of packet-shaped segment tables (GPU box): NPK segments of
64 KiB in one plan, laid out as (a) a de-framed arena (data contiguous and
aligned, CRCs in their own array) or (b) the wire image itself (header of H
bytes, CRCs, data, repeated), for several header lengths (alignments of the
CRCs and the data).  Run once per env setting (HDFS_CRC32C_SMALL_RULE,
HDFS_CRC32C_TILE_ORDER); prints one JSON object."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hadoofus_amd as h  # noqa: E402

h.load()
D, CS = 65536, 512
NCH = D // CS
LAYOUTS = {"arena": None, "arena_crc_odd": -1, "wire_h28": 28, "wire_h25": 25, "wire_h34": 34, "wire_h32": 32}
out = {"env": {k: v for k, v in os.environ.items() if k.startswith("HDFS_CRC32C")}}


def run(NPK, name, H):
    arena = H is None or H < 0  # H = -1: aligned data, CRC array at an odd address
    stride = D if arena else H + 4 * NCH + D
    buf = h.DeviceBuffer(NPK * stride + 4096)
    h.fill_splitmix64(buf.ptr, buf.nbytes // 8, 11, 0)
    crcbuf = h.DeviceBuffer(NPK * NCH * 4 + 64) if arena else None
    bms = h.DeviceBuffer(NPK * NCH // 8)
    segs = []
    for k in range(NPK):
        if arena:
            data, crcs = buf.ptr + k * D, crcbuf.ptr + k * NCH * 4 + (1 if H else 0)
        else:
            crcs = buf.ptr + k * stride + H
            data = crcs + 4 * NCH
        segs.append(h.Segment(data=data, len=D, chunk_size=CS, flags=h.SEG_BE, crc_init=0, crcs=crcs,
                              bitmap=bms.ptr + k * NCH // 8))
    comp = h.Plan(h.MODE_COMPUTE, [h.Segment(data=s.data, len=s.len, chunk_size=CS, flags=h.SEG_BE, crc_init=0,
                                             crcs=s.crcs) for s in segs])
    comp.execute()
    h.device_sync()
    ver = h.Plan(h.MODE_VERIFY, segs)
    ver.execute()
    fb, mism = ver.results()
    ms = ver.time(10)
    for x in (ver, comp):
        x.destroy()
    for b in (buf, crcbuf, bms):
        if b is not None:
            b.free()
    return {"GBps": round(NPK * D / (ms * 1e-3) / 1e9, 1), "ms": round(ms, 4), "mism": int(mism)}


for npk in [int(x) for x in os.environ.get("NPK", "256,1024,4096,16384").split(",")]:
    out[npk] = {name: run(npk, name, H) for name, H in LAYOUTS.items()}
print(json.dumps(out))
