"""Generate tests/golden/write_packets.json: write-path packet fixtures.

Each case is one write (len bytes of splitmix64 payload at a block offset,
a starting seqno, protocol v1/v2, checksum type, finish flag) and the header
buffers the reference's packet loop would send for it: _send_packet's packet
sizing (src/datanode.c:2590: min(remains, PACKET_SIZE = 64 KiB); :2592-2609:
an unaligned offset first completes its 512-B chunk) and
_compose_data_packet_header (src/datanode.c:2781-2868).  Expected bytes are
built here independently of the oracle and the engine: v2 headers with
google.protobuf (PacketHeaderProto declared from
src/proto/datatransfer.proto:228-235, as in gen_golden_packets.py), v1
headers with struct, CRC32C values from the reference built unchanged
(oracle/_ref), CRC32 values from zlib 1.2.11.

    make -C oracle && python oracle/gen_golden_write_packets.py
"""
import json
import os
import struct
import sys
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
from gen_golden_packets import PH  # noqa: E402  (google.protobuf PacketHeaderProto)
from oracle import Reference  # noqa: E402
from packet_stream import CSUM_CRC32, CSUM_CRC32C, CSUM_NULL, payload  # noqa: E402

OUT = os.path.join(HERE, "..", "tests", "golden", "write_packets.json")
PACKET, CHUNK = 64 * 1024, 512

# (name, len, offset, seqno, proto, ctype, finish, seed)
CASES = [
    ("v2_crc32c_aligned_finish", 200000, 0, 0, 2, CSUM_CRC32C, True, 1),
    ("v2_crc32c_unaligned_start", 140000, 1000, 5, 2, CSUM_CRC32C, False, 2),
    ("v1_crc32c_one_full_packet_finish", 65536, 0, 0, 1, CSUM_CRC32C, True, 3),
    ("v2_crc32_finish", 70000, 3 * 512, 17, 2, CSUM_CRC32, True, 4),
    ("v2_null_unaligned_finish", 1000, 7, 2, 2, CSUM_NULL, True, 5),
    ("v2_finish_only", 0, 131072, 9, 2, CSUM_CRC32C, True, 6),
    ("v1_crc32_inside_one_chunk", 100, 100, 3, 1, CSUM_CRC32, False, 7),
    ("v2_crc32c_unaligned_long_tail", 3 * 65536 + 777, 512 * 5 + 300, 40, 2, CSUM_CRC32C, True, 8),
    ("v1_null_two_packets", 65537, 0, 0, 1, CSUM_NULL, False, 9),
]


def main():
    ref = Reference()
    cases = []
    for name, n, off0, seq0, proto, ctype, finish, seed in CASES:
        data = payload(seed, 0, n).tobytes()
        hdr, pkts = b"", []
        off, seq, pos = off0, seq0, 0
        sizes = []
        while pos < n:
            k = min(n - pos, PACKET)
            if off % CHUNK:
                k = min(k, CHUNK - off % CHUNK)
            sizes.append(k)
            off += k
            pos += k
        if finish:
            sizes.append(0)
        off, pos = off0, 0
        for k in sizes:
            chunk_crcs = []
            if ctype != CSUM_NULL:
                for i in range(0, k, CHUNK):
                    piece = data[pos + i:pos + min(i + CHUNK, k)]
                    c = zlib.crc32(piece) if ctype == CSUM_CRC32 else ref.crc32c(0, piece)
                    chunk_crcs.append(struct.pack(">I", c))
            crcs = b"".join(chunk_crcs)
            last = k == 0
            plen = k + len(crcs) + 4
            if proto == 2:
                pb = PH(offsetInBlock=off, seqno=seq, lastPacketInBlock=last, dataLen=k).SerializeToString()
                h = struct.pack(">iH", plen, len(pb)) + pb + crcs
            else:
                h = struct.pack(">iqqBi", plen, off, seq, 1 if last else 0, k) + crcs
            pkts.append({"hdr_off": len(hdr), "data_off": pos, "offset_in_block": off, "seqno": seq,
                         "data_len": k, "hdr_len": len(h), "crc_len": len(crcs), "last": int(last)})
            hdr += h
            off += k
            pos += k
            seq += 1
        cases.append({"name": name, "len": n, "offset": off0, "seqno": seq0, "proto": proto, "ctype": ctype,
                      "finish": finish, "data": {"seed": seed, "g0": 0, "len": n}, "hdr_hex": hdr.hex(),
                      "packets": pkts})
    with open(OUT, "w") as f:
        json.dump({"generator": "oracle/gen_golden_write_packets.py",
                   "source": "src/datanode.c:2583-2609 (_send_packet sizing), :2781-2868 "
                             "(_compose_data_packet_header); headers via google.protobuf / struct, CRC32C from "
                             "the reference build (oracle/_ref), CRC32 from zlib " + zlib.ZLIB_RUNTIME_VERSION,
                   "cases": cases}, f, indent=1)
    print(f"wrote {len(cases)} cases to {OUT}")


if __name__ == "__main__":
    main()
