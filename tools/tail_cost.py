"""What a block's short last packet costs (GPU box): a device-resident v2
block of 2 048 full packets, then a 12 345-B packet and the empty end
packet (a file's last block), against the same block with only the empty
end packet -- hdfs_crc32c_verify_packets, best of 20.  Run once with
HDFS_CRC32C_TAIL_SMALL=0 and once with 1 (diagnostic build: the rest of the
stream after the run framed by a pass, or one short-run launch).

    python tools/tail_cost.py [out.json]"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import device_stream_bench as dsb  # noqa: E402
import diaglib  # noqa: E402
import hadoofus_amd as h  # noqa: E402


def main():
    lib = h.load(diaglib.DIAG_LIB_PATH)
    dsb.lib = lib
    img, npk = dsb.wire_image(128 << 20, 9)
    d = h.DeviceBuffer(12345)
    h.fill_splitmix64(d.ptr, 12345 // 8, 77, 0)
    h.device_sync()
    hdr, pk = h.compose_packets(None, 128 << 20, npk, h.PROTO_V2, h.CSUM_CRC32C, True, dptr=d.ptr, nbytes=12345)
    data = d.download()
    d.free()
    hb = np.frombuffer(hdr, np.uint8)
    H = pk[0]["hdr_len"]
    tail = np.concatenate([hb[:H], data[:12345], hb[H:]])
    blk_e, nblk = dsb.wire_image(128 << 20, 9, empty_last=True)
    out = {"tail_small": os.environ.get("HDFS_CRC32C_TAIL_SMALL", "1"),
           "tail_stream": os.environ.get("HDFS_CRC32C_TAIL_STREAM", "1")}
    for name, im in (("block_empty_end", blk_e), ("block_short_last_packet", np.concatenate([img, tail]))):
        dev = h.DeviceBuffer(im.nbytes + 64)
        dev.upload(im)
        h.device_sync()
        arr = (h.abi.Packet * 4096)()
        cnt, used = ctypes.c_size_t(0), ctypes.c_uint64(0)
        best = 1e9
        for rep in range(21):
            t0 = time.perf_counter()
            rc = lib.hdfs_crc32c_verify_packets(dev.ptr, im.nbytes, h.PROTO_V2, 512, h.CSUM_CRC32C, arr, 4096,
                                                ctypes.byref(cnt), ctypes.byref(used))
            t = time.perf_counter() - t0
            assert rc == 0 and used.value == im.nbytes, (rc, used.value, im.nbytes)
            if rep:
                best = min(best, t)
        out[name] = {"us": round(best * 1e6, 1), "packets": cnt.value}
        dev.free()
    js = json.dumps(out)
    print(js)
    if len(sys.argv) > 1:
        open(sys.argv[1], "w").write(js + "\n")


if __name__ == "__main__":
    main()
