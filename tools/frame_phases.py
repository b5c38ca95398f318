"""Where a device framing pass spends its time (GPU box, diagnostic build):
frame_build_kernel stamps s_memrealtime (100 MHz) per block at the end of
each phase when a stamp buffer is set (Diag.set_tuning(2, ptr)).  Runs the
1 GiB device-resident v2 run of tools/device_stream_bench.py (16 384 packets)
through hdfs_crc32c_verify_packets and prints, per phase, the spread over
the blocks in microseconds from the earliest block start.

Phases: 0 start, 1 framed, 2 aggregate published, 3 look-back done,
4 entries written (inactive blocks: counted), 5 done-counter, 6 last block
published to the host."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import diaglib  # noqa: E402
import hadoofus_amd as h  # noqa: E402

lib = h.load(diaglib.DIAG_LIB_PATH)
D = diaglib.Diag(lib=lib)
NBLK = 1024
OFF = 65536  # kFrameStampOff (crc32c_engine.h): the tiled kernel's per-wave words come first


def wire_image(nbytes, seed):
    """Composed v2 packets of nbytes of device-filled payload -> host bytes
    (as tools/device_stream_bench.py)."""
    d = h.DeviceBuffer(nbytes)
    h.fill_splitmix64(d.ptr, nbytes // 8, seed, 0)
    h.device_sync()
    hdr, pk = h.compose_packets(None, 0, 0, h.PROTO_V2, h.CSUM_CRC32C, False, dptr=d.ptr, nbytes=nbytes)
    data = d.download()
    d.free()
    H = pk[0]["hdr_len"]
    hb = np.frombuffer(hdr, np.uint8)
    return np.concatenate([hb.reshape(len(pk), H), data.reshape(len(pk), 65536)], axis=1).reshape(-1), len(pk)


img, npk = wire_image(1 << 30, 7)
dev = h.DeviceBuffer(img.nbytes + 64)
dev.upload(img)
st = h.DeviceBuffer((OFF + NBLK * 8) * 8)
arr = (h.abi.Packet * (npk + 8))()
cnt, used = ctypes.c_size_t(0), ctypes.c_uint64(0)
out = {"packets": npk, "runs": []}
for rep in range(4):
    st.fill(0)
    h.device_sync()
    D.set_tuning(2, st.ptr if rep else None)
    rc = lib.hdfs_crc32c_verify_packets(dev.ptr, img.nbytes, h.PROTO_V2, 512, h.CSUM_CRC32C, arr, npk + 8,
                                        ctypes.byref(cnt), ctypes.byref(used))
    assert rc >= 0 and cnt.value == npk, (rc, cnt.value)
    h.device_sync()
    if not rep:
        continue
    s = st.download(NBLK * 64, OFF * 8, dtype=np.uint64).reshape(NBLK, 8).astype(np.int64)
    live = s[:, 0] > 0
    t0 = s[live, 0].min()
    run = {"blocks": int(live.sum()), "active": int((s[:, 1] > 0).sum())}
    for ph in range(7):
        v = s[live, ph]
        v = v[v > 0]
        if v.size:
            us = (v - t0) / 100.0
            run[f"p{ph}_us"] = [round(float(us.min()), 2), round(float(np.median(us)), 2), round(float(us.max()), 2)]
    out["runs"].append(run)
D.set_tuning(2, None)
print(json.dumps(out))
