"""GPU: streaming sessions (pinned slots fed like socket reads)
against the oracle's packet-stream verdicts on the same bytes."""
import numpy as np
import pytest

from packet_stream import CSUM_CRC32, CSUM_CRC32C, build_stream

pytestmark = pytest.mark.gpu


def _feed(sess, s, rng, max_piece, poll_every=3):
    got, off, i = [], 0, 0
    while off < len(s):
        n = int(rng.integers(1, max_piece))
        sess.write(s[off:off + n])
        off += n
        i += 1
        if i % poll_every == 0:
            got += sess.poll()[1]
    sess.flush()
    while True:
        rc, more = sess.poll(wait=True)
        got += more
        if not more:
            break
    return got


def _shift(pkts, d):
    return [dict(p, stream_off=p["stream_off"] + d) for p in pkts]


@pytest.mark.parametrize("proto,cs,ctype", [(2, 512, CSUM_CRC32C), (1, 512, CSUM_CRC32C), (2, 4096, CSUM_CRC32),
                                            (2, 100, CSUM_CRC32C)])
def test_session_two_blocks_small_slots(engine, oracle, proto, cs, ctype):
    rng = np.random.default_rng(cs + proto + ctype)
    a, _ = build_stream(oracle.crc32c, proto, cs, ctype, [65536] * 40, seed=1, corrupt=[(3, 1), (39, 0)])
    b, _ = build_stream(oracle.crc32c, proto, cs, ctype, [65536] * 30 + [12345], seed=2, corrupt=[(30, 2)])
    want = oracle.verify_packets(a, proto, cs, ctype)[1] + _shift(oracle.verify_packets(b, proto, cs, ctype)[1], len(a))
    sess = engine.Session(proto, cs, ctype, slot_bytes=1 << 20, nslots=3)
    got = _feed(sess, a + b, rng, 300_000)
    sess.close()
    assert got == want


def test_session_large_default_slots(engine, oracle):
    rng = np.random.default_rng(5)
    s, bad = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, [65536] * 3000, seed=3,
                          corrupt=[(int(rng.integers(0, 3000)), int(rng.integers(0, 128))) for _ in range(20)])
    want = oracle.verify_packets(s)[1]
    sess = engine.Session()
    got = _feed(sess, s, rng, 8 << 20, poll_every=5)
    sess.close()
    assert got == want
    assert sum(1 for p in got if p["error"]) == len(bad)


def test_session_stops_at_framing_error(engine, oracle):
    good, _ = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, [65536] * 5, seed=4, last_empty=False)
    broken = bytearray(good)
    # packet 3: plen smaller than dataLen + 4 -> PACKET_SIZE
    off3 = oracle.verify_packets(good)[1][3]["stream_off"]
    broken[off3:off3 + 4] = (100).to_bytes(4, "big")
    sess = engine.Session(slot_bytes=1 << 20, nslots=2)
    sess.write(bytes(broken))
    sess.flush()
    rc, got = sess.poll(wait=True)
    assert rc == engine.ERR_PACKET_SIZE
    assert [p["error"] for p in got] == [0, 0, 0, engine.ERR_PACKET_SIZE]
    with pytest.raises(engine.CRC32CError):
        sess.write(b"\0" * 10)
    sess.close()


def test_session_packet_larger_than_slot(engine, oracle):
    s, _ = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, [200000], seed=6)
    sess = engine.Session(slot_bytes=65536, nslots=2)
    with pytest.raises(engine.CRC32CError):
        sess.write(s)
    sess.close()
