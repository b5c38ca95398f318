"""Diagnosis of a resumed client read (GPU box): the read of
test_gpu_read_resumable_and_scatter[2-512-2-regular], case 2 (client_offset
7 bytes into the block's first packet, the whole block; packet 146 has a bad
chunk), in calls of `piece` bytes, printed call by call beside the oracle's
single read loop -- to tell an engine fault from a property of resuming.

    python tools/diag_resumed_read.py LIB [spec=0|1] [piece]

LIB: a build of libhadoofus_crc32c.so (spec=0 needs the diagnostic build,
whose hdfs_crc32c_set_speculation turns the one-launch path off)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import hadoofus_amd as h  # noqa: E402
from oracle import Oracle  # noqa: E402  (checker)
from packet_stream import build_stream  # noqa: E402


def main():
    lib = h.load(sys.argv[1])
    spec = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    piece = int(sys.argv[3]) if len(sys.argv) > 3 else 65539
    if not spec:
        lib.hdfs_crc32c_set_speculation(0)
    o = Oracle()
    proto, cs, ctype = 2, 512, h.CSUM_CRC32C
    dl = [65536] * 150 + [12345]
    base = 3 * 65536
    s, _ = build_stream(o.crc32c, proto, cs, ctype, dl, seed=len(dl) + 5, corrupt=[(len(dl) - 5, 1)], offset0=base)
    total = sum(dl)
    co, rl = base + 7, total
    want = o.read_packets(s, co, rl, proto, cs, ctype)
    werr = [i for i, r in enumerate(want[1]) if r["error"]]
    buf = h.DeviceBuffer(len(s) + 64)
    buf.upload(np.frombuffer(s, np.uint8))
    h.device_sync()
    dst = h.DeviceBuffer(rl + 4096)
    at, tot, recs, calls = 0, 0, [], []
    while True:
        cap = min(piece, rl - tot)
        rc, pk, used, got = h.read_packets(buf.ptr + at, len(s) - at, dst.ptr + tot, cap, proto, cs, ctype,
                                           client_offset=co + tot, read_len=rl - tot)
        for q in pk:
            q["stream_off"] += at
        calls.append({"at": at, "tot": tot, "rc": rc, "n": len(pk), "used": used, "got": got,
                      "first": pk[0]["stream_off"] if pk else None,
                      "errors": [(q["stream_off"], q["error"], q["first_bad"]) for q in pk if q["error"]]})
        recs += pk
        at += used
        tot += got
        if rc != h.AGAIN or len(calls) > 10000:
            break
    data = dst.download(tot).tobytes()
    same = [i for i in range(min(len(recs), len(want[1]))) if recs[i] != want[1][i]]
    print(json.dumps({
        "lib": sys.argv[1], "spec": spec, "piece": piece,
        "oracle": {"rc": want[0], "n": len(want[1]), "used": want[2], "delivered": len(want[3]), "errors": werr},
        "resumed": {"rc": rc, "n": len(recs), "used": at, "delivered": tot, "calls": len(calls)},
        "records_differ_at": same[:10],
        "records_equal_through_first_error": bool(werr) and len(recs) > werr[0] and not [i for i in same if i <= werr[0]],
        "bytes_equal": data == want[3],
        "last_calls": calls[-3:],
    }))


if __name__ == "__main__":
    main()
