"""Verified reads delivered piece by piece (round 5): hdfs_crc32c_reader_open
verifies the packets of a client read once; hdfs_crc32c_reader_next then
only copies -- the reference's read re-entered with remains_pkt > 0
(src/datanode.c:2356-2361, 2547-2549) without reading any CRC again.  The
pieces, concatenated, equal the oracle's single read loop (oracle_read_packets:
src/datanode.c:1476-1481, 2428-2549): the bytes, the records in order, the
final status and consumed bytes; every call but the last fills its buffer
and returns AGAIN; nothing is written past a buffer.  Call by call, each
return (status, the records it completes, consumed, delivered) equals
_reader_model's, derived from the oracle's read."""
import numpy as np
import pytest

from packet_stream import CSUM_CRC32, CSUM_CRC32C, build_stream

AGAIN = 1000


def _dev(engine, s, shift=0):
    buf = engine.DeviceBuffer(len(s) + shift + 64)
    buf.fill(0)
    buf.upload(np.frombuffer(s, np.uint8), offset=shift)
    engine.device_sync()
    return buf, buf.ptr + shift


ERR_BAD_LASTPACKET = 32


def _reader_model(want, co, rl, piece):
    """What each hdfs_crc32c_reader_next call returns for the oracle's read
    `want` = (rc, records, consumed, bytes) of [co, co + rl) through buffers
    of `piece` bytes: (rc, records completed, consumed, delivered) per call.
    A record is complete once every byte it delivers is out (the read's last
    record -- its error, or the packet that completes it -- with the last
    call); consumed = the end of the last complete packet, the read's own
    at its end; AGAIN until then (src/datanode.c:2547-2549)."""
    rc_f, recs, used_f, data = want
    total = len(data)
    cum, done_at = 0, []
    for r in recs:
        gives = 0
        if not r["error"] or r["error"] == ERR_BAD_LASTPACKET:
            off, dl = r["offset_in_block"], r["data_len"]
            gives = max(0, min(off + dl, co + rl) - max(off, co))
        cum += gives
        done_at.append(cum)
    if done_at:
        done_at[-1] = total
    calls, done, nxt = [], 0, 0
    while True:
        got = min(piece, total - done)
        done += got
        k0 = nxt
        while nxt < len(recs) and done_at[nxt] <= done and (done == total or nxt + 1 < len(recs)):
            nxt += 1
        if done == total:
            calls.append((rc_f, recs[k0:nxt], used_f, got))
            return calls
        r = recs[nxt - 1] if nxt else None
        consumed = r["stream_off"] + r["header_len"] + r["crc_len"] + r["data_len"] if r else 0
        calls.append((AGAIN, recs[k0:nxt], consumed, got))


def _read_through(engine, rd, piece, total_cap, host, model=None):
    """All of a reader's bytes through buffers of `piece` bytes (a fresh
    buffer region each call, a 16-B guard after it); model: each call's
    expected (rc, records, consumed, delivered) (_reader_model)."""
    if host:
        arena = np.full(total_cap + 64 * 1024, 0xA5, np.uint8)
        base = arena.ctypes.data
    else:
        dbuf = engine.DeviceBuffer(total_cap + 64 * 1024)
        dbuf.fill(0xA5)
        base = dbuf.ptr
    at, data, recs, calls = 0, b"", [], 0
    while True:
        rc, pk, used, got = rd.next([(base + at, piece)])
        if model is not None:
            assert calls < len(model) and (rc, pk, used, got) == model[calls], (piece, calls)
        calls += 1
        recs += pk
        if got:
            if host:
                data += arena[at:at + got].tobytes()
                guard = arena[at + piece:at + piece + 16].tobytes()
            else:
                data += dbuf.download(got, offset=at).tobytes()
                guard = dbuf.download(16, offset=at + piece).tobytes()
            assert guard == b"\xa5" * 16
        at += piece + 16
        if rc != AGAIN:
            break
        assert got == piece and calls < 100000
    if not host:
        dbuf.free()
    if model is not None:
        assert calls == len(model), (piece, calls, len(model))
    return rc, recs, used, data, calls


@pytest.mark.gpu
@pytest.mark.parametrize("proto,ctype,sizes", [
    (2, CSUM_CRC32C, "regular"),
    (1, CSUM_CRC32, "regular"),
    (2, CSUM_CRC32C, "mixed"),
])
def test_gpu_reader_vs_oracle(engine, oracle, proto, ctype, sizes):
    rng = np.random.default_rng(len(sizes) + proto)
    if sizes == "regular":
        dl = [65536] * 120 + [12345]
    else:
        dl = [int(x) for x in np.repeat(rng.choice([4096, 61440, 30000, 65536], 25), rng.integers(1, 6, 25))]
    base = 2 * 65536
    s, _ = build_stream(oracle.crc32c, proto, 512, ctype, dl, seed=len(dl) + 3, corrupt=[(len(dl) - 6, 2)],
                        offset0=base)
    total = sum(dl)
    cases = [(base + 1000, total // 3), (base + 7, total), (base + total // 2, total), (base, 1)]
    for ci, (co, rl) in enumerate(cases):
        want = oracle.read_packets(s, co, rl, proto, 512, ctype)
        keep, p = _dev(engine, s, ci % 3)
        # (3 MiB + 5: more pieces than one launch's arguments take -- the table launch)
        # (host 1 MiB + 7: many pieces gathered through the device staging area, one D2H)
        for piece, host in ((4099, False), (65536, False), (100003, True), (1 << 20, False), ((3 << 20) + 5, False),
                            ((1 << 20) + 7, True)):
            rd = engine.Reader(p, len(s), co, rl, proto, 512, ctype)
            try:
                rc, recs, used, data, calls = _read_through(engine, rd, piece, len(want[3]) + piece * 2, host,
                                                            model=_reader_model(want, co, rl, piece))
            finally:
                rd.close()
            assert (rc, recs, used) == want[:3], (co - base, rl, piece)
            assert data == want[3], (co - base, rl, piece)
        keep.free()


@pytest.mark.gpu
def test_gpu_reader_errors_first(engine, oracle):
    """A read whose first packet has bad CRCs delivers nothing and returns
    the error on the first call; a read past the block's end ends with
    BAD_LASTPACKET after its bytes; a read that starts past the stream's
    first packet is UNEXPECTED_READ_OFFSET."""
    dl = [65536] * 10
    s, _ = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, dl, seed=5, corrupt=[(0, 3)])
    s2, _ = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, dl, seed=6)
    for st, co, rl in ((s, 10, 1000), (s2, 100, 11 * 65536), (s2, 3 * 65536, 100)):
        want = oracle.read_packets(st, co, rl)
        keep, p = _dev(engine, st)
        rd = engine.Reader(p, len(st), co, rl)
        rc, recs, used, data, calls = _read_through(engine, rd, 65536, len(want[3]) + 2 * 65536, False,
                                                    model=_reader_model(want, co, rl, 65536))
        rd.close()
        assert (rc, recs, used) == want[:3] and data == want[3]
        assert rc != 0
        keep.free()


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["clean", "seqno_jumps", "offset_skew", "offset_skew_early", "corrupt"])
def test_gpu_scatter_copy_beside_verify(engine, oracle, kind):
    """A scatter read of a run of >= 64 equal packets starts its copy under
    the verify, from the packets predicted at the early block: when the
    verdicts or the actual headers disagree with the prediction (a corrupt
    packet ends the read early; a skewed offsetInBlock moves the window, or
    only a record, as a seqno jump does) the result still equals the oracle's
    read -- bytes, records, consumed, status -- and no guard byte moves."""
    dl = [65536] * 1100 + [9999]  # (a run of >= 1 024 packets is copied beside its verify)
    kw = {}
    if kind == "seqno_jumps":
        kw["seqnos"] = [k + (3 if k >= 900 else 0) for k in range(len(dl))]
    elif kind == "offset_skew":
        kw["offset_skew"] = {700: 4096}
    elif kind == "offset_skew_early":  # packet 1 claims packet 0's offset: a read from 777 takes it from 777 too
        kw["offset_skew"] = {1: -65536}
    elif kind == "corrupt":
        kw["corrupt"] = [(800, 2)]
    s, _ = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, dl, seed=31, **kw)
    keep, p = _dev(engine, s, 3)
    sizes = [8 << 20] * 8 + [123457] * 3
    iov, off = [], 0
    for n in sizes:
        iov.append((off, n))
        off += n + 16
    cap = sum(sizes)
    for co, rl in ((0, cap + 100000), (777, sum(dl) - 777), (5 * 65536 + 3, 1000 * 65536)):
        want = oracle.read_packets(s, co, rl, cap=cap)
        big = engine.DeviceBuffer(off + 64)
        big.fill(0xA5)
        rc, recs, used, got = engine.read_packets(p, len(s), None, 0, client_offset=co, read_len=rl,
                                                  iov=[(big.ptr + a, n) for a, n in iov])
        assert (rc, recs, used) == want[:3], (kind, co)
        flat = big.download(off).tobytes()
        data, left = b"", got
        for a, n in iov:
            take = min(n, left)
            data += flat[a:a + take]
            left -= take
            assert flat[a + n:a + n + 16] == b"\xa5" * 16
        assert data == want[3], (kind, co)
        big.free()
    keep.free()


@pytest.mark.gpu
@pytest.mark.parametrize("nbuf,lo,hi", [(2000, 1, 300), (300, 1000, 40000), (40, 1, 17)])
def test_gpu_scatter_many_buffers(engine, oracle, nbuf, lo, hi):
    """One hdfs_crc32c_read_packets call over many device buffers (the
    reference's iovec array, src/datanode.c:2509-2537): the read is verified
    once and its bytes laid over the buffers by one copy launch -- from a
    table of thousands of pieces (tiny buffers: a workgroup stages several
    rounds of entries), or from the launch's own arguments.  Bytes, records,
    consumed and status equal the oracle's single read; a 16-B guard after
    every buffer is untouched."""
    rng = np.random.default_rng(nbuf + lo)
    dl = [65536] * 40 + [777]
    s, _ = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, dl, seed=nbuf, corrupt=[(30, 2)])
    keep, p = _dev(engine, s, 1)
    sizes = [int(x) for x in rng.integers(lo, hi + 1, nbuf)]
    iov, off = [], 0
    for n in sizes:
        iov.append((off, n))
        off += n + 16 + int(rng.integers(0, 16))
    cap = sum(sizes)
    for co in (0, 5 * 65536 + 333):
        rl = min(cap + 5000, sum(dl) - co)  # more than the buffers hold: AGAIN
        want = oracle.read_packets(s, co, rl, cap=cap)
        big = engine.DeviceBuffer(off + 64)
        big.fill(0xA5)
        rc, recs, used, got = engine.read_packets(p, len(s), None, 0, client_offset=co, read_len=rl,
                                                  iov=[(big.ptr + a, n) for a, n in iov])
        assert (rc, recs, used) == want[:3], (nbuf, co)
        flat = big.download(off).tobytes()
        data, left = b"", got
        for a, n in iov:
            take = min(n, left)
            data += flat[a:a + take]
            left -= take
            assert flat[a + n:a + n + 16] == b"\xa5" * 16
        assert data == want[3], (nbuf, co)
        big.free()
    keep.free()


@pytest.mark.gpu
def test_gpu_reader_through_mailbox(engine, oracle):
    """With the latency mode open (hdfs_crc32c_mailbox_create) a delivery of
    <= 32 pieces and <= 96 KiB is copied by the resident kernel instead of a
    launch: the same bytes, records and status as the oracle's read, guard
    bytes untouched; larger deliveries keep the launch; a small scatter read
    goes the same way; an idled-out mailbox is relaunched by the next call."""
    dl = [65536] * 60 + [4321]
    s, _ = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, dl, seed=44, corrupt=[(50, 3)])
    keep, p = _dev(engine, s, 2)
    co, rl = 1234, sum(dl) - 2000
    want = oracle.read_packets(s, co, rl)
    with engine.Mailbox(idle_ms=50) as mb:
        for piece in (4099, 65536, 98304, (1 << 20) + 17, (3 << 20) + 5):
            c0 = mb.stats()[0]
            rd = engine.Reader(p, len(s), co, rl)
            try:
                rc, recs, used, data, calls = _read_through(engine, rd, piece, len(want[3]) + piece * 2, False,
                                                            model=_reader_model(want, co, rl, piece))
            finally:
                rd.close()
            assert (rc, recs, used) == want[:3], piece
            assert data == want[3], piece
            served = mb.stats()[0] - c0
            if piece <= 98304:
                assert served >= calls - 1, (piece, served, calls)
            else:  # full deliveries launch; only the short last one may be served
                assert served <= 1, (piece, served)
        # a small scatter read: three buffers, one delivery through the mailbox
        c0 = mb.stats()[0]
        big = engine.DeviceBuffer(300000)
        big.fill(0xA5)
        iov = [(0, 40000), (40016, 1000), (41032, 50000)]
        w2 = oracle.read_packets(s, co, rl, cap=91000)
        r2 = engine.read_packets(p, len(s), None, 0, client_offset=co, read_len=rl,
                                 iov=[(big.ptr + a, n) for a, n in iov])
        assert r2[:3] == w2[:3]
        flat = big.download(300000).tobytes()
        assert flat[0:40000] + flat[40016:41016] + flat[41032:91032] == w2[3]
        for a, n in iov:
            assert flat[a + n:a + n + 16] == b"\xa5" * 16
        assert mb.stats()[0] - c0 == 1
        big.free()
        # idle out, then a reader call relaunches the resident kernel
        import time
        time.sleep(0.2)
        l0 = mb.stats()[1]
        rd = engine.Reader(p, len(s), co, rl)
        rc, recs, used, data, calls = _read_through(engine, rd, 65536, len(want[3]) + 2 * 65536, False)
        rd.close()
        assert (rc, recs, used) == want[:3] and data == want[3]
        assert mb.stats()[1] > l0
    keep.free()


@pytest.mark.gpu
def test_gpu_reader_records_or_stream_run_out(engine, oracle):
    """A read the reader cannot complete -- its record array (max_pkts) or
    the stream ends first -- delivers what the oracle's read loop delivers
    (src/datanode.c:1476-1481 stops at the same packet) and ends with the same
    status, records and consumed bytes: the caller resumes at stream +
    consumed with client_offset + delivered."""
    dl = [65536] * 30 + [5000]
    s, _ = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, dl, seed=91)
    whole = oracle.verify_packets(s)[1]
    cut = s[:whole[20]["stream_off"] + 1000]  # ends inside packet 20
    for st, mp in ((s, 7), (cut, None), (cut, 3)):
        co, rl = 777, sum(dl) - 1000
        want = oracle.read_packets(st, co, rl, max_pkts=mp) if mp else oracle.read_packets(st, co, rl)
        keep, p = _dev(engine, st)
        rd = engine.Reader(p, len(st), co, rl, max_pkts=mp)
        try:
            rc, recs, used, data, calls = _read_through(engine, rd, 65536, len(want[3]) + 2 * 65536, False,
                                                        model=_reader_model(want, co, rl, 65536))
        finally:
            rd.close()
        assert (rc, recs, used) == want[:3], mp
        assert data == want[3], mp
        keep.free()


@pytest.mark.gpu
@pytest.mark.parametrize("room", [0, 1, 2])
def test_gpu_reader_small_record_array(engine, oracle, room):
    """next with room for fewer records than the call completes (max_pkts 0,
    1 or 2) loses nothing: the records it has no room for come with the
    following calls (bytes first, then record-only calls that deliver 0
    bytes), in order, and the read's status and consumed come with its last
    record -- the concatenation equals the oracle's single read.  With room
    0, a call completes no record, so consumed never moves past 0 before the
    draining calls."""
    dl = [4096] * 40 + [777]
    s, _ = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, dl, seed=23, corrupt=[(33, 1)])
    co, rl = 100, sum(dl)
    want = oracle.read_packets(s, co, rl)
    keep, p = _dev(engine, s)
    dbuf = engine.DeviceBuffer(len(want[3]) + 65536)
    rd = engine.Reader(p, len(s), co, rl)
    try:
        data, recs, at, calls, last_used = b"", [], 0, 0, 0
        while True:
            piece = 65536
            rc, pk, used, got = rd.next([(dbuf.ptr + at, piece)], room=room if data != want[3] else max(room, 1))
            calls += 1
            assert len(pk) <= max(room, 1 if data == want[3] else room)
            assert used >= last_used
            last_used = used
            recs += pk
            data += dbuf.download(got, offset=at).tobytes() if got else b""
            at += got
            if rc != AGAIN:
                break
            assert calls < 1000
        assert (rc, recs, used) == want[:3]
        assert data == want[3]
        # after the last call: the status again, nothing delivered
        assert rd.next([(dbuf.ptr, 4096)], room=room)[0] == rc
    finally:
        rd.close()
        dbuf.free()
        keep.free()


@pytest.mark.gpu
def test_gpu_reader_host_stream(engine, oracle):
    """A reader over a HOST-resident stream (a host-memory datanode's
    receive buffer): framed on the host, the read's packets verified on the
    GPU once at open, each next a memcpy into the caller's host buffer
    (src/datanode.c:2516) -- equal to the oracle's read; device buffers are
    refused for a host stream, as hdfs_crc32c_read_packets refuses them."""
    dl = [65536] * 50 + [3333]
    s, _ = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, dl, seed=17, corrupt=[(44, 5)])
    hs = np.frombuffer(s, np.uint8).copy()
    for co, rl in ((1000, sum(dl) // 2), (5, sum(dl))):
        want = oracle.read_packets(s, co, rl)
        for piece in (4099, 65536, (1 << 20) + 3):
            rd = engine.Reader(hs.ctypes.data, len(s), co, rl)
            try:
                rc, recs, used, data, calls = _read_through(engine, rd, piece, len(want[3]) + 2 * piece, True,
                                                            model=_reader_model(want, co, rl, piece))
            finally:
                rd.close()
            assert (rc, recs, used) == want[:3], (co, rl, piece)
            assert data == want[3], (co, rl, piece)
    dbuf = engine.DeviceBuffer(65536)
    rd = engine.Reader(hs.ctypes.data, len(s), 0, 100000)
    with pytest.raises(engine.CRC32CError):
        rd.next([(dbuf.ptr, 65536)])
    rd.close()
    dbuf.free()


def test_reader_model_concatenates_to_the_oracle_read(oracle):
    """CPU: the per-call model (_reader_model) adds up to the oracle's single
    read -- every record once and in order, the bytes, consumed at the end --
    for clean, bad-CRC, BAD_LASTPACKET and UNEXPECTED_READ_OFFSET reads and
    buffer sizes around the packet size."""
    dl = [65536] * 12 + [1000]
    s, _ = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, dl, seed=3, corrupt=[(9, 4)])
    s2, _ = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, dl, seed=4)
    for st, co, rl in ((s, 100, 5 * 65536), (s, 70000, 20 * 65536), (s2, 3, sum(dl) + 500), (s2, 0, 1),
                       (s2, 5 * 65536 + 7, 3 * 65536)):
        want = oracle.read_packets(st, co, rl)
        for piece in (1, 4099, 65536, 65537, 1 << 20):
            if len(want[3]) // piece > 5000:
                continue
            m = _reader_model(want, co, rl, piece)
            assert [r for c in m for r in c[1]] == want[1]
            assert sum(c[3] for c in m) == len(want[3])
            assert m[-1][0] == want[0] and m[-1][2] == want[2]
            assert all(c[0] == AGAIN and c[3] == piece for c in m[:-1])


@pytest.mark.gpu
def test_gpu_reader_random(engine, oracle):
    """Seeded random reads: stream shapes (packet sizes mixed and regular, a
    corrupt chunk or none, v1/v2, CRC32/CRC32C), read windows anywhere in the
    block, buffer sizes from 1 B to 2 MiB, device or host buffers, the
    mailbox open or not -- every call equal to _reader_model of the oracle's
    read."""
    rng = np.random.default_rng(2024)
    for case in range(24):
        proto = int(rng.choice([1, 2]))
        ctype = int(rng.choice([CSUM_CRC32, CSUM_CRC32C]))
        npk = int(rng.integers(2, 40))
        if rng.random() < 0.5:
            dl = [65536] * npk + [int(rng.integers(1, 65536))]
        else:
            dl = [int(x) for x in rng.choice([512, 4096, 30000, 61440, 65536], npk)]
        corrupt = [(int(rng.integers(0, len(dl))), 0)] if rng.random() < 0.4 else []
        s, _ = build_stream(oracle.crc32c, proto, 512, ctype, dl, seed=case, corrupt=corrupt,
                            last_empty=proto == 2)
        total = sum(dl)
        co = int(rng.integers(0, total))
        rl = int(rng.integers(1, total - co + 2000))
        want = oracle.read_packets(s, co, rl, proto, 512, ctype)
        piece = int(rng.choice([1, 777, 4096, 65536, 100000, 1 << 21]))
        if len(want[3]) // piece > 2000:
            piece = max(piece, len(want[3]) // 2000 + 1)
        host = bool(rng.random() < 0.3)
        keep, p = _dev(engine, s, case % 4)
        box = engine.Mailbox() if rng.random() < 0.3 else None
        try:
            rd = engine.Reader(p, len(s), co, rl, proto, 512, ctype)
            try:
                rc, recs, used, data, calls = _read_through(engine, rd, piece, len(want[3]) + 2 * piece, host,
                                                            model=_reader_model(want, co, rl, piece))
            finally:
                rd.close()
        finally:
            if box:
                box.close()
            keep.free()
        assert (rc, recs, used) == want[:3], case
        assert data == want[3], case


@pytest.mark.gpu
def test_gpu_readers_threads(engine, oracle):
    """Readers used from several threads at once (ctypes releases the GIL:
    the engine's calls really interleave), beside verify jobs and scatter
    reads on other threads, with the mailbox open: every reader's calls
    still equal the per-call model of the oracle's read."""
    import threading
    dl = [65536] * 24 + [2222]
    streams = [build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, dl, seed=200 + i,
                            corrupt=[(20, 1)] if i % 2 else [])[0] for i in range(4)]
    bufs = [_dev(engine, st, i) for i, st in enumerate(streams)]
    errors = []

    def reader_worker(i):
        try:
            st, (_, p) = streams[i], bufs[i]
            for rep, (co, rl, piece) in enumerate(((100, 20 * 65536, 65536), (7, sum(dl), 30001),
                                                   (65536 * 3, 5 * 65536, 1 << 20))):
                want = oracle.read_packets(st, co, rl)
                rd = engine.Reader(p, len(st), co, rl)
                try:
                    got = _read_through(engine, rd, piece, len(want[3]) + 2 * piece, rep == 1,
                                        model=_reader_model(want, co, rl, piece))
                finally:
                    rd.close()
                assert got[:3] == want[:3] and got[3] == want[3]
        except Exception as e:  # noqa: BLE001 -- reported by the main thread
            errors.append((i, repr(e)))

    def job_worker():
        try:
            for _ in range(3):
                jobs = [engine.VerifyJob(p, len(st)) for st, (_, p) in zip(streams, bufs)]
                for j, st in zip(jobs, streams):
                    assert j.wait() == oracle.verify_packets(st)
        except Exception as e:  # noqa: BLE001
            errors.append(("jobs", repr(e)))

    with engine.Mailbox():
        th = [threading.Thread(target=reader_worker, args=(i,)) for i in range(4)]
        th.append(threading.Thread(target=job_worker))
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=240)
        assert not any(t.is_alive() for t in th)
    assert not errors, errors
    for b, _ in bufs:
        b.free()


@pytest.mark.gpu
def test_gpu_scatter_threads(engine, oracle):
    """Scatter reads of long runs from three threads at once: one copy
    beside a verify is in flight per device (the others copy after their
    verify), and every read equals the oracle's."""
    import threading
    dl = [65536] * 1100 + [4321]
    streams = [build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, dl, seed=300 + i,
                            corrupt=[(900, 1)] if i == 1 else [])[0] for i in range(3)]
    bufs = [_dev(engine, st, i) for i, st in enumerate(streams)]
    sizes = [16 << 20] * 4 + [54321] * 5
    cap = sum(sizes)
    errors = []

    def worker(i):
        try:
            st, (_, p) = streams[i], bufs[i]
            for co in (0, 1234567):
                rl = sum(dl) - co
                want = oracle.read_packets(st, co, rl, cap=cap)
                iov, off = [], 0
                for n in sizes:
                    iov.append((off, n))
                    off += n + 16
                big = engine.DeviceBuffer(off + 64)
                big.fill(0xA5)
                rc, recs, used, got = engine.read_packets(p, len(st), None, 0, client_offset=co, read_len=rl,
                                                          iov=[(big.ptr + a, n) for a, n in iov])
                flat = big.download(off).tobytes()
                big.free()
                data, left = b"", got
                for a, n in iov:
                    take = min(n, left)
                    data += flat[a:a + take]
                    left -= take
                    assert flat[a + n:a + n + 16] == b"\xa5" * 16
                assert (rc, recs, used) == want[:3] and data == want[3], (i, co)
        except Exception as e:  # noqa: BLE001 -- reported by the main thread
            errors.append((i, repr(e)))

    th = [threading.Thread(target=worker, args=(i,)) for i in range(3)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=240)
    assert not any(t.is_alive() for t in th)
    assert not errors, errors
    for b, _ in bufs:
        b.free()
