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
