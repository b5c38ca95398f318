"""Generate tests/golden/packet_cases.json: datanode packet-stream fixtures.

Each case is a wire stream (header / CRC bytes literal, payloads as
splitmix64 recipes) plus the expected per-packet framing and verify verdicts
of _recv_packet -> _process_recv_packet -> _verify_crcdata
(src/datanode.c:2345-2494, 2931-2963).  Expected values come from the
CONSTRUCTION of each case (which packet was malformed or corrupted, and
how), not from the oracle; the oracle and the engine are both checked
against them.  CRC32C values come from the reference built unchanged
(oracle/_ref) and CRC32 values from zlib 1.2.11.

The v2 headers are pinned to the protobuf wire format with google.protobuf:
the PacketHeaderProto descriptor is declared below from
src/proto/datatransfer.proto:228-235, canonical headers must serialize
byte-identically to tests/packet_stream.header_v2, and every hand-made
unusual header is parsed by google.protobuf to check it means what the case
says.  Where protobuf-c (the reference's decoder) and google.protobuf differ
(a known field with the wrong wire type: protobuf-c rejects the message,
google.protobuf keeps it as an unknown field), the case follows protobuf-c
and says so.

    make -C oracle && python oracle/gen_golden_packets.py
"""
import json
import os
import struct
import sys
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
from oracle import Oracle, Reference, have_reference  # noqa: E402
from packet_stream import CSUM_CRC32, CSUM_CRC32C, CSUM_NULL, header_v2, payload  # noqa: E402

OUT = os.path.join(HERE, "..", "tests", "golden", "packet_cases.json")
ERR_PROTO, ERR_SIZE, ERR_CRC_LEN, ERR_UNEXP_CRC, ERR_BAD = 18, 25, 26, 27, 29


def header_class():
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
    fdp = descriptor_pb2.FileDescriptorProto(name="packet_header.proto", package="hadoop.hdfs", syntax="proto2")
    m = fdp.message_type.add(name="PacketHeaderProto")
    F = descriptor_pb2.FieldDescriptorProto
    for name, num, typ, lab in [("offsetInBlock", 1, F.TYPE_SFIXED64, F.LABEL_REQUIRED),
                                ("seqno", 2, F.TYPE_SFIXED64, F.LABEL_REQUIRED),
                                ("lastPacketInBlock", 3, F.TYPE_BOOL, F.LABEL_REQUIRED),
                                ("dataLen", 4, F.TYPE_SFIXED32, F.LABEL_REQUIRED),
                                ("syncBlock", 5, F.TYPE_BOOL, F.LABEL_OPTIONAL)]:
        m.field.add(name=name, number=num, type=typ, label=lab)
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    return message_factory.GetMessageClass(pool.FindMessageTypeByName("hadoop.hdfs.PacketHeaderProto"))


PH = header_class()


def pinned_header(offset, seqno, last, dlen, sync=None):
    kw = dict(offsetInBlock=offset, seqno=seqno, lastPacketInBlock=last, dataLen=dlen)
    if sync is not None:
        kw["syncBlock"] = sync
    want = PH(**kw).SerializeToString()
    got = header_v2(offset, seqno, last, dlen, sync)
    assert got == want, (got.hex(), want.hex())
    return got


def pb_parse(b):
    m = PH()
    m.ParseFromString(b)
    return m


class Case:
    def __init__(self, name, proto, cs, ctype, crcf, note=""):
        self.name, self.proto, self.cs, self.ctype, self.crcf = name, proto, cs, ctype, crcf
        self.parts, self.lit, self.pos, self.pkts = [], b"", 0, []
        self.note = note
        self.max_pkts = None
        self.seed = 11

    def _flush(self):
        if self.lit:
            self.parts.append({"hex": self.lit.hex()})
            self.lit = b""

    def raw(self, b):
        self.lit += b
        self.pos += len(b)

    def crcs(self, d):
        cs = self.cs
        out = []
        for i in range(0, len(d), cs):
            piece = d[i:i + cs].tobytes()
            c = zlib.crc32(piece) if self.ctype == CSUM_CRC32 else self.crcf(0, piece)
            out.append(int(c).to_bytes(4, "big"))
        return b"".join(out)

    def packet(self, dlen, seqno, offset=0, last=False, corrupt=(), hdr=None, plen=None, crc_override=None,
               hdr_dlen=None, sync=None, v1_last_byte=None, expect=None, data=True):
        """Append one packet.  expect: dict of expected fields overriding the
        derived ones (error, header fields) or None."""
        g0 = 10_000 * len(self.pkts)
        d = payload(self.seed, g0, max(dlen, 0))
        crc = b"" if self.ctype == CSUM_NULL and crc_override is None else self.crcs(d)
        if crc_override is not None:
            crc = crc_override
        flips, bad = [], []
        for ch in corrupt:
            clen = min(self.cs, dlen - ch * self.cs)
            off = ch * self.cs + (7919 * (ch + 1)) % clen
            flips.append([off, 1 << (ch % 8)])
            bad.append(ch)
        hd = dlen if hdr_dlen is None else hdr_dlen
        if plen is None:
            plen = 4 + len(crc) + max(dlen, 0)
        start = self.pos
        if self.proto == 1:
            lb = (1 if last else 0) if v1_last_byte is None else v1_last_byte
            h = struct.pack(">iqqBi", plen, offset, seqno, lb, hd)
            hl = 25
        else:
            body = hdr if hdr is not None else pinned_header(offset, seqno, last, hd, sync)
            h = struct.pack(">iH", plen, len(body)) + body
            hl = 6 + len(body)
        self.raw(h + crc)
        if data and dlen > 0:
            self._flush()
            self.parts.append({"data": {"seed": self.seed, "g0": g0, "len": dlen}, "flips": flips})
            self.pos += dlen
        rec = {"stream_off": start, "offset_in_block": offset, "seqno": seqno, "data_len": hd,
               "crc_len": plen - hd - 4, "header_len": hl, "error": ERR_BAD if bad else 0,
               "first_bad": min(bad) if bad else -1, "bad_chunks": len(set(bad)),
               "last": int(bool(last if v1_last_byte is None else v1_last_byte)), "sync": int(bool(sync))}
        if expect:
            rec.update(expect)
        self.pkts.append(rec)
        return rec

    def result(self, n_records, consumed):
        self._flush()
        recs = self.pkts[:n_records]
        rc = next((r["error"] for r in recs if r["error"]), 0)
        return {"name": self.name, "note": self.note, "proto": self.proto, "chunk_size": self.cs,
                "ctype": self.ctype, "max_pkts": self.max_pkts, "parts": self.parts,
                "expect": {"rc": rc, "consumed": consumed, "packets": recs}}


def end_of(c):
    return c.pos


def main():
    crcf = Reference().crc32c if have_reference() else Oracle().crc32c
    cases = []

    def clean_run(c, dlens, corrupt=None, last_empty=True, sync_first=False):
        corrupt = corrupt or {}
        off = 0
        for k, dl in enumerate(dlens):
            last = (k == len(dlens) - 1) and not last_empty
            c.packet(dl, k, off, last=last, corrupt=corrupt.get(k, ()),
                     sync=(True if (sync_first and k == 0) else None))
            off += dl
        if last_empty:
            c.packet(0, len(dlens), off, last=True)
        return off

    # clean and corrupted v2 / v1 streams ---------------------------------
    c = Case("v2_clean", 2, 512, CSUM_CRC32C, crcf, "20 x 64 KiB + 1000 B + empty last packet")
    clean_run(c, [65536] * 20 + [1000], sync_first=True)
    cases.append(c.result(22, end_of(c)))

    c = Case("v2_corrupt", 2, 512, CSUM_CRC32C, crcf, "bit flips in packets 3, 11, 20")
    clean_run(c, [65536] * 20 + [1000], {3: (5, 100), 11: (0,), 20: (1,)})
    cases.append(c.result(22, end_of(c)))

    c = Case("v1_clean", 1, 512, CSUM_CRC32C, crcf, "25-byte headers")
    clean_run(c, [65536] * 10 + [333])
    cases.append(c.result(12, end_of(c)))

    c = Case("v1_corrupt_lastbyte", 1, 512, CSUM_CRC32C, crcf, "last flag byte 0x02 reads as true (s8 != 0)")
    c.packet(65536, 0, 0, corrupt=(127,))
    c.packet(4000, 1, 65536, last=True, v1_last_byte=2)
    cases.append(c.result(2, end_of(c)))

    c = Case("v2_crc32", 2, 512, CSUM_CRC32, crcf, "HDFS_CSUM_CRC32 (zlib)")
    clean_run(c, [65536] * 8, {2: (64,), 7: (127,)})
    cases.append(c.result(9, end_of(c)))

    c = Case("v2_cs4096", 2, 4096, CSUM_CRC32C, crcf, "bytesPerChecksum 4096")
    clean_run(c, [61440] * 5 + [5000], {4: (14,), 5: (1,)})
    cases.append(c.result(7, end_of(c)))

    c = Case("v2_cs100", 2, 100, CSUM_CRC32C, crcf, "bytesPerChecksum 100 (generic kernel)")
    clean_run(c, [6400] * 4 + [77], {1: (63,), 4: (0,)})
    cases.append(c.result(6, end_of(c)))

    # framing errors ------------------------------------------------------
    c = Case("err_crc_len", 2, 512, CSUM_CRC32C, crcf, "packet 4 carries one CRC too few; packet 1 corrupt")
    off = 0
    for k in range(4):
        c.packet(65536, k, off, corrupt=(9,) if k == 1 else ())
        off += 65536
    good = payload(c.seed, 10_000 * 4, 65536)
    short = c.crcs(good)[:-4]
    consumed = c.pos
    c.packet(65536, 4, off, crc_override=short, expect={"error": ERR_CRC_LEN, "first_bad": -1, "bad_chunks": 0})
    cases.append(c.result(5, consumed))

    c = Case("err_negative_dlen", 2, 512, CSUM_CRC32C, crcf, "dataLen -5 -> PACKET_SIZE")
    c.packet(65536, 0, 0)
    c.packet(65536, 1, 65536)
    consumed = c.pos
    c.packet(0, 2, 131072, hdr_dlen=-5, plen=4 + 0 - 5 + 5, data=False, crc_override=b"",
             expect={"error": ERR_SIZE})
    cases.append(c.result(3, consumed))

    c = Case("err_empty_not_last", 2, 512, CSUM_CRC32C, crcf, "dataLen 0 without lastPacketInBlock")
    for k in range(3):
        c.packet(65536, k, 65536 * k)
    consumed = c.pos
    c.packet(0, 3, 3 * 65536, last=False, expect={"error": ERR_SIZE})
    cases.append(c.result(4, consumed))

    c = Case("err_plen_small", 2, 512, CSUM_CRC32C, crcf, "plen < dataLen + 4 -> crcdlen < 0 -> PACKET_SIZE")
    c.packet(65536, 0, 0)
    consumed = c.pos
    c.packet(65536, 1, 65536, plen=65536, data=False, crc_override=b"", expect={"error": ERR_SIZE})
    cases.append(c.result(2, consumed))

    missing = header_v2(65536 * 2, 2, False, 65536)[:-5]  # dataLen dropped
    assert not pb_parse(missing).IsInitialized()
    c = Case("err_proto_missing_field", 2, 512, CSUM_CRC32C, crcf, "PacketHeaderProto without dataLen")
    c.packet(65536, 0, 0)
    c.packet(65536, 1, 65536)
    consumed = c.pos
    c.packet(65536, 2, 0, hdr=missing, data=False, crc_override=b"",
             expect={"error": ERR_PROTO, "offset_in_block": 0, "seqno": 0, "data_len": 0, "crc_len": 0,
                     "last": 0, "sync": 0})
    cases.append(c.result(3, consumed))

    # lastPacketInBlock as fixed32: protobuf-c rejects a known field with the
    # wrong wire type; google.protobuf keeps it as unknown and then lacks the
    # required field -- both refuse it.
    wt = (b"\x09" + struct.pack("<q", 65536) + b"\x11" + struct.pack("<q", 1) + b"\x1d\x01\x00\x00\x00" +
          b"\x25" + struct.pack("<i", 65536))
    assert not pb_parse(wt).IsInitialized()
    c = Case("err_proto_wire_type", 2, 512, CSUM_CRC32C, crcf, "bool field 3 sent as fixed32")
    c.packet(65536, 0, 0)
    consumed = c.pos
    c.packet(65536, 1, 0, hdr=wt, data=False, crc_override=b"",
             expect={"error": ERR_PROTO, "offset_in_block": 0, "seqno": 0, "data_len": 0, "crc_len": 0,
                     "last": 0, "sync": 0})
    cases.append(c.result(2, consumed))

    # unusual but valid encodings: reversed order, unknown fields, 2-byte
    # varint bool, duplicate dataLen (last wins), syncBlock set
    def odd(offset, seqno, last, dlen):
        b = b"\x25" + struct.pack("<i", 12345)  # overwritten below
        b += b"\x38\x96\x01"                     # field 7 varint 150 (unknown)
        b += b"\x18" + (b"\x81\x00" if last else b"\x80\x00")
        b += b"\x4a\x03abc"                      # field 9 bytes "abc" (unknown)
        b += b"\x11" + struct.pack("<q", seqno) + b"\x09" + struct.pack("<q", offset)
        b += b"\x28\x01" + b"\x25" + struct.pack("<i", dlen)
        m = pb_parse(b)
        assert m.IsInitialized() and m.dataLen == dlen and m.lastPacketInBlock == last and m.syncBlock
        assert m.offsetInBlock == offset and m.seqno == seqno
        return b

    c = Case("proto_unusual_ok", 2, 512, CSUM_CRC32C, crcf, "valid but non-canonical PacketHeaderProto")
    off = 0
    for k, dl in enumerate([65536, 65536, 7000]):
        c.packet(dl, k, off, hdr=odd(off, k, False, dl), sync=True, corrupt=(3,) if k == 1 else ())
        off += dl
    c.packet(0, 3, off, hdr=odd(off, 3, True, 0), last=True, sync=True)
    cases.append(c.result(4, end_of(c)))

    c = Case("csum_null_ok", 2, 512, CSUM_NULL, crcf, "checksum type NULL: no CRCs, nothing verified")
    clean_run(c, [65536] * 3 + [100])
    cases.append(c.result(5, end_of(c)))

    c = Case("csum_null_unexpected", 2, 512, CSUM_NULL, crcf, "checksum type NULL but CRC bytes present")
    good = payload(c.seed, 0, 65536)
    crc32c_bytes = Case("crcs", 2, 512, CSUM_CRC32C, crcf).crcs(good)
    c.packet(65536, 0, 0, crc_override=crc32c_bytes, expect={"error": ERR_UNEXP_CRC})
    cases.append(c.result(1, 0))

    # incomplete streams and max_pkts -------------------------------------
    c = Case("truncated_data", 2, 512, CSUM_CRC32C, crcf, "stream ends inside packet 4's data")
    clean_run(c, [65536] * 6, last_empty=False)
    cut = c.pkts[4]["stream_off"] + 1000
    full = c.result(6, end_of(c))
    stream_parts = full["parts"]
    full["name"], full["cut"] = "truncated_data", cut
    full["expect"] = {"rc": 0, "consumed": c.pkts[4]["stream_off"], "packets": c.pkts[:4]}
    full["parts"] = stream_parts
    cases.append(full)

    c = Case("truncated_header", 2, 512, CSUM_CRC32C, crcf, "stream ends inside packet 2's PacketHeaderProto")
    clean_run(c, [65536] * 4, last_empty=False)
    r = c.result(4, end_of(c))
    r["cut"] = c.pkts[2]["stream_off"] + 10
    r["expect"] = {"rc": 0, "consumed": c.pkts[2]["stream_off"], "packets": c.pkts[:2]}
    cases.append(r)

    c = Case("max_pkts", 2, 512, CSUM_CRC32C, crcf, "only 3 packets requested")
    clean_run(c, [65536] * 8, {5: (1,)})
    c.max_pkts = 3
    cases.append(c.result(3, c.pkts[3]["stream_off"]))

    with open(OUT, "w") as f:
        json.dump({"generator": "oracle/gen_golden_packets.py", "zlib": zlib.ZLIB_RUNTIME_VERSION,
                   "cases": cases}, f)
    print("wrote", os.path.abspath(OUT), len(cases), "cases")


if __name__ == "__main__":
    main()
