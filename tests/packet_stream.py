"""Builders for datanode packet streams (test infrastructure).

Wire formats (src/datanode.c:2345-2418, big-endian integers per
src/heapbuf.c:174-215):
  v1: [plen s32][offsetInBlock s64][seqno s64][lastPacketInBlock s8][dataLen s32]
  v2: [plen s32][hlen u16][PacketHeaderProto]
followed by plen - dataLen - 4 bytes of BE chunk CRCs and the data.

header_v2() emits the canonical encoding of PacketHeaderProto
(src/proto/datatransfer.proto:228-235): fields in number order, sfixed64 /
sfixed32 as little-endian fixed-width, bools as one-byte varints, syncBlock
only when set.  oracle/gen_golden_packets.py pins it byte-for-byte to the
google.protobuf encoder.
"""
import struct
import zlib

import numpy as np

from oracle import splitmix64_np

CSUM_NULL, CSUM_CRC32, CSUM_CRC32C = 0, 1, 2


def header_v2(offset, seqno, last, dlen, sync=None):
    b = b"\x09" + struct.pack("<q", offset) + b"\x11" + struct.pack("<q", seqno)
    b += b"\x18" + bytes([1 if last else 0]) + b"\x25" + struct.pack("<i", dlen)
    if sync is not None:
        b += b"\x28" + bytes([1 if sync else 0])
    return b


def frame_v2(hdr, crcs, data, plen=None):
    if plen is None:
        plen = 4 + len(crcs) + len(data)
    return struct.pack(">iH", plen, len(hdr)) + hdr + crcs + data


def frame_v1(offset, seqno, last, crcs, data, plen=None, dlen=None, last_byte=None):
    if plen is None:
        plen = 4 + len(crcs) + len(data)
    if dlen is None:
        dlen = len(data)
    lb = (1 if last else 0) if last_byte is None else last_byte
    return struct.pack(">iqqBi", plen, offset, seqno, lb, dlen) + crcs + data


def chunk_crcs_be(data, cs, ctype, crc32c):
    """BE CRC bytes of data's chunks; crc32c(crc, bytes) is the CRC32C function
    to use (the oracle, in tests and in the fixture generator)."""
    out = []
    for i in range(0, len(data), cs):
        piece = bytes(data[i:i + cs])
        c = zlib.crc32(piece) if ctype == CSUM_CRC32 else crc32c(0, piece)
        out.append(int(c).to_bytes(4, "big"))
    return b"".join(out)


def payload(seed, g0, n):
    return splitmix64_np((n + 7) // 8, seed=seed, g0=g0).view(np.uint8)[:n].copy()


def assemble(parts):
    """Fixture parts -> stream bytes: {"hex": ...} literal wire bytes or
    {"data": {"seed", "g0", "len"}, "flips": [[byte, mask], ...]}."""
    out = []
    for p in parts:
        if "hex" in p:
            out.append(bytes.fromhex(p["hex"]))
        else:
            d = payload(p["data"]["seed"], p["data"]["g0"], p["data"]["len"])
            for off, mask in p.get("flips", []):
                d[off] ^= np.uint8(mask)
            out.append(d.tobytes())
    return b"".join(out)


def build_stream(crc32c, proto, cs, ctype, dlens, seed=0, corrupt=(), last_empty=True, sync_every=0,
                 seqnos=None, offset_skew=None, offset0=0, last_flag=None, sync_at=()):
    """A clean stream of packets with the given data lengths (the last one
    flagged lastPacketInBlock unless last_empty adds the v2-style trailing
    empty packet).  corrupt: iterable of (packet, chunk) -> flip one bit of
    that chunk after its CRC is computed.  seqnos: header seqno per packet
    (default k); offset_skew: {packet: bytes added to its offsetInBlock} --
    header fields off the regular progression, same wire sizes.  offset0:
    offsetInBlock of the first packet (a read from inside a block);
    last_flag: packet index flagged lastPacketInBlock instead; sync_at:
    packets whose v2 header carries syncBlock (27-B headers).  Returns
    (stream bytes, expected per-packet bad chunk lists)."""
    out = []
    bad = {}
    for pk, ch in corrupt:
        bad.setdefault(pk, []).append(ch)
    off = 0
    for k, dl in enumerate(dlens):
        d = payload(seed, off // 8 + 1000 * k, dl)
        crcs = chunk_crcs_be(d, cs, ctype, crc32c) if ctype != CSUM_NULL else b""
        for ch in bad.get(k, []):
            clen = min(cs, dl - ch * cs)
            d[ch * cs + (k * 7919 + ch) % clen] ^= np.uint8(1 << (ch % 8))
        last = (k == len(dlens) - 1) and not last_empty if last_flag is None else k == last_flag
        seq = k if seqnos is None else seqnos[k]
        ho = offset0 + off + (offset_skew or {}).get(k, 0)
        if proto == 1:
            out.append(frame_v1(ho, seq, last, crcs, d.tobytes()))
        else:
            sync = (k % sync_every == 0) if sync_every else (True if k in sync_at else None)
            out.append(frame_v2(header_v2(ho, seq, last, dl, sync), crcs, d.tobytes()))
        off += dl
    if last_empty:
        k = len(dlens)
        if proto == 1:
            out.append(frame_v1(offset0 + off, k, True, b"", b""))
        else:
            out.append(frame_v2(header_v2(offset0 + off, k, True, 0), b"", b""))
    return b"".join(out), {k: sorted(set(v)) for k, v in bad.items()}
