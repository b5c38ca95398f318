"""Where a copy launch of verified read bytes spends its time (GPU box,
diagnostic build): copy_pieces_kernel stamps s_memrealtime (100 MHz) per
workgroup -- 0 entry, 1 first piece-table entries staged (table launches),
2 its stores acknowledged, 3 counted done -- when a stamp buffer is set
(Diag.set_tuning(2, ptr)).  Runs a 128 MiB block of 64 KiB packets in device
memory through a reader (verified at open) delivered by ONE
hdfs_crc32c_reader_next into one device buffer: one table launch of 2 048
pieces (a scatter read copies beside its verify with copy_beside_kernel
instead, which has no stamps).  Prints per phase [min, median, max]
microseconds from the earliest workgroup's entry.

    python tools/copy_phases.py [out.json]"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import diaglib  # noqa: E402
import hadoofus_amd as h  # noqa: E402
from spec_phases import spread, wire_image  # noqa: E402

lib = h.load(diaglib.DIAG_LIB_PATH)
D = diaglib.Diag(lib=lib)
OFF = 110592  # kCopyStampOff (crc32c_internal.h)
NBLK = 4096


def main():
    img, npk = wire_image(128 << 20, 9)
    d = h.DeviceBuffer(img.nbytes + 64)
    d.upload(img)
    payload = npk * 65536
    dst = h.DeviceBuffer(payload + 4096)
    st = h.DeviceBuffer((OFF + NBLK * 4) * 8)
    arr = (h.abi.Packet * (npk + 8))()
    cnt, used, got = ctypes.c_size_t(0), ctypes.c_uint64(0), ctypes.c_uint64(0)
    vec = (h.abi.IoVec * 1)(h.abi.IoVec(dst.ptr, payload))
    runs = []
    for rep in range(5):
        rd = ctypes.c_void_p()
        assert lib.hdfs_crc32c_reader_open(d.ptr, img.nbytes, h.PROTO_V2, 512, h.CSUM_CRC32C, 0, payload, npk + 8,
                                           ctypes.byref(rd)) == 0
        st.fill(0)
        h.device_sync()
        D.set_tuning(2, st.ptr if rep else None)
        t = time.perf_counter()
        rc = lib.hdfs_crc32c_reader_next(rd, vec, 1, arr, npk + 8, ctypes.byref(cnt), ctypes.byref(used),
                                         ctypes.byref(got))
        wall = (time.perf_counter() - t) * 1e6
        lib.hdfs_crc32c_reader_close(rd)
        assert rc >= 0 and got.value == payload, (rc, got.value)
        h.device_sync()
        if not rep:
            continue
        s = st.download(NBLK * 32, OFF * 8, dtype=np.uint64).reshape(NBLK, 4).astype(np.int64)
        live = s[:, 0] > 0
        t0 = s[live, 0].min()
        run = {"wall_us": round(wall, 2), "blocks": int(live.sum())}
        for ph in range(4):
            run[f"p{ph}_us"] = spread(s[live, ph], t0)
        dur = (s[live, 2] - s[live, 0]) / 100.0
        run["block_life_us"] = [round(float(dur.min()), 2), round(float(np.median(dur)), 2), round(float(dur.max()), 2)]
        runs.append(run)
    D.set_tuning(2, None)
    js = json.dumps({"payload_bytes": payload, "runs": runs})
    print(js)
    if len(sys.argv) > 1:
        open(sys.argv[1], "w").write(js + "\n")


if __name__ == "__main__":
    main()
