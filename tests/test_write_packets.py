"""Write path: outgoing data packets of one write (_send_packet's sizing,
src/datanode.c:2583-2609, and _compose_data_packet_header, :2781-2868).

CPU: the oracle against the golden fixtures (oracle/gen_golden_write_packets.py:
headers from google.protobuf / struct, CRC32C from the reference build, CRC32
from zlib), and a write -> read round trip through the oracle's packet-stream
verifier.  GPU: the engine (hdfs_crc32c_compose_packets, CRCs on the device)
against the same fixtures with host and device-resident data, against the
oracle on seeded random writes, and the round trip through the engine's own
packet verifier, corruptions included."""
import json
import os

import numpy as np
import pytest

from packet_stream import payload

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "write_packets.json")


def _cases():
    with open(GOLDEN) as f:
        return json.load(f)["cases"]


def _wire(hdr, pkts, data):
    """Header buffer + data of every packet, in send order (the writev of
    _send_packet)."""
    out = []
    for p in pkts:
        out.append(hdr[p["hdr_off"]:p["hdr_off"] + p["hdr_len"]])
        out.append(bytes(data[p["data_off"]:p["data_off"] + p["data_len"]]))
    return b"".join(out)


@pytest.mark.parametrize("case", _cases(), ids=lambda c: c["name"])
def test_oracle_matches_golden(oracle, case):
    d = payload(case["data"]["seed"], case["data"]["g0"], case["data"]["len"])
    hdr, pkts = oracle.compose_packets(d, case["offset"], case["seqno"], case["proto"], case["ctype"], case["finish"])
    assert hdr.hex() == case["hdr_hex"]
    assert pkts == case["packets"]


@pytest.mark.parametrize("case", [c for c in _cases() if c["finish"]], ids=lambda c: c["name"])
def test_oracle_write_read_round_trip(oracle, case):
    d = payload(case["data"]["seed"], case["data"]["g0"], case["data"]["len"])
    hdr, pkts = oracle.compose_packets(d, case["offset"], case["seqno"], case["proto"], case["ctype"], True)
    wire = _wire(hdr, pkts, d)
    rc, got, used = oracle.verify_packets(wire, proto=case["proto"], chunk_size=512, ctype=case["ctype"])
    assert rc == 0 and used == len(wire)
    assert [(p["offset_in_block"], p["seqno"], p["data_len"], p["last"]) for p in got] == \
        [(p["offset_in_block"], p["seqno"], p["data_len"], p["last"]) for p in pkts]


@pytest.mark.gpu
@pytest.mark.parametrize("where", ["host", "device"])
@pytest.mark.parametrize("case", _cases(), ids=lambda c: c["name"])
def test_engine_matches_golden(engine, case, where):
    d = payload(case["data"]["seed"], case["data"]["g0"], case["data"]["len"])
    args = (case["offset"], case["seqno"], case["proto"], case["ctype"], case["finish"])
    if where == "host":
        hdr, pkts = engine.compose_packets(d, *args)
    else:
        dbuf = engine.DeviceBuffer(max(1, d.nbytes))
        if d.nbytes:
            dbuf.upload(d)
        hdr, pkts = engine.compose_packets(None, *args, dptr=dbuf.ptr, nbytes=d.nbytes)
    assert hdr.hex() == case["hdr_hex"]
    assert pkts == case["packets"]


@pytest.mark.gpu
def test_engine_vs_oracle_random_writes(engine, oracle):
    rng = np.random.default_rng(77)
    for i in range(24):
        n = int(rng.choice([0, 1, 511, 512, 513, 65535, 65536, 65537, int(rng.integers(1, 400000))]))
        off = int(rng.choice([0, 512 * int(rng.integers(0, 1000)), int(rng.integers(0, 1 << 30))]))
        args = (off, int(rng.integers(-1, 1 << 40)), int(rng.choice([1, 2])), int(rng.choice([0, 1, 2])),
                bool(rng.integers(0, 2)))
        d = payload(100 + i, 0, n)
        assert engine.compose_packets(d, *args) == oracle.compose_packets(d, *args), (i, n, args)


@pytest.mark.gpu
@pytest.mark.parametrize("proto", [1, 2])
def test_engine_write_read_round_trip(engine, proto):
    """A 2 MiB write at an unaligned block offset, composed on the GPU, read
    back by the GPU packet verifier: clean, then with one data bit flipped and
    one wire CRC flipped."""
    d = payload(9, 0, (2 << 20) + 123)
    hdr, pkts = engine.compose_packets(d, 4321, 1, proto, engine.CSUM_CRC32C, True)
    wire = bytearray(_wire(hdr, pkts, d))
    rc, got, used = engine.verify_packets(bytes(wire), proto=proto)
    assert rc == 0 and used == len(wire) and len(got) == len(pkts)
    assert all(p["error"] == 0 and p["first_bad"] == -1 for p in got)
    # flip a data bit in packet 3, chunk 5, and the wire CRC of packet 7, chunk 0
    p3, p7 = got[3], got[7]
    wire[p3["stream_off"] + p3["header_len"] + p3["crc_len"] + 5 * 512 + 17] ^= 0x04
    wire[p7["stream_off"] + p7["header_len"]] ^= 0x80
    rc, got, _ = engine.verify_packets(bytes(wire), proto=proto)
    assert rc == engine.ERR_BAD_CHECKSUM
    assert [(i, p["first_bad"]) for i, p in enumerate(got) if p["error"]] == [(3, 5), (7, 0)]


@pytest.mark.gpu
@pytest.mark.parametrize("ctype", [0, 1, 2], ids=["null", "crc32", "crc32c"])
def test_datanode_basics_scenario(engine, ctype):
    """The reference's end-to-end test without the cluster
    (tests/t_datanode_basics.c:25-26,85-86,174-274): 70 MiB of '0'+(i%10)
    written as 64 MiB blocks (hdfs_datanode_write + finish_block) with each
    checksum type, the packets of every block read back through the packet
    verifier (v2 stream; the 6 MiB tail block also through a streaming
    session fed in odd-sized reads), payload reassembled and compared."""
    towrite, blocksz = 70 << 20, 64 << 20
    buf = (np.arange(towrite, dtype=np.int64) % 10 + ord("0")).astype(np.uint8)
    rbuf = np.zeros(towrite, dtype=np.uint8)
    wtot = 0
    while wtot < towrite:
        wblk = min(towrite - wtot, blocksz)
        hdr, pkts = engine.compose_packets(buf[wtot:wtot + wblk], 0, 0, engine.PROTO_V2, ctype, True)
        assert sum(p["data_len"] for p in pkts) == wblk and pkts[-1]["last"] == 1
        wire = _wire(hdr, pkts, buf[wtot:wtot + wblk])
        rc, got, used = engine.verify_packets(wire, proto=engine.PROTO_V2, ctype=ctype)
        assert rc == 0 and used == len(wire) and len(got) == len(pkts)
        w = np.frombuffer(wire, dtype=np.uint8)
        for p in got:
            a = p["stream_off"] + p["header_len"] + p["crc_len"]
            rbuf[wtot + p["offset_in_block"]:wtot + p["offset_in_block"] + p["data_len"]] = w[a:a + p["data_len"]]
        if wblk < blocksz:  # the tail block again, through a session
            s = engine.Session(proto=engine.PROTO_V2, ctype=ctype, slot_bytes=1 << 20, nslots=3)
            recs, pos, i = [], 0, 0
            while pos < len(wire):  # odd-sized "socket reads"
                n = min(65537 + 4099 * (i % 7), len(wire) - pos)
                s.write(wire[pos:pos + n])
                pos += n
                i += 1
                recs += s.poll()[1]
            s.flush()
            while True:
                rc, more = s.poll(wait=True)
                assert rc == 0
                if not more:
                    break
                recs += more
            s.close()
            assert [(r["offset_in_block"], r["data_len"], r["error"]) for r in recs] == \
                [(p["offset_in_block"], p["data_len"], 0) for p in got]
        wtot += wblk
    assert np.array_equal(buf, rbuf), "read differed from write"
