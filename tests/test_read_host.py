"""Client reads into HOST memory (round 5): hdfs_crc32c_read_packets with
host iovecs, from a device-resident stream (fused verify + copy-out into a
device staging area, then D2H per iovec) and from a host-resident stream
(host framing, GPU verify, the reference's memcpy into the iovecs,
src/datanode.c:2509-2537).  Every read is held to the oracle's read loop
(oracle_read_packets: src/datanode.c:1476-1481, 2428-2549) -- the status,
the records, consumed bytes and the delivered bytes -- with guard bytes
after every buffer."""
import numpy as np
import pytest

from packet_stream import CSUM_CRC32, CSUM_CRC32C, build_stream

AGAIN, BAD = 1000, 29


def _dev(engine, s, shift=0):
    buf = engine.DeviceBuffer(len(s) + shift + 64)
    buf.fill(0)
    buf.upload(np.frombuffer(s, np.uint8), offset=shift)
    engine.device_sync()
    return buf, buf.ptr + shift


class HostIov:
    """Host buffers of the given sizes inside one array, a 16-B guard after each."""

    def __init__(self, sizes, pinned=None):
        self.sizes = list(sizes)
        self.offs, off = [], 0
        for n in self.sizes:
            self.offs.append(off)
            off += n + 16
        self.total = off
        if pinned is not None:
            self.pin = pinned(off)
            self.arr = self.pin.array
        else:
            self.pin = None
            self.arr = np.empty(off, np.uint8)
        self.arr[:] = 0xA5

    def iov(self):
        base = self.arr.ctypes.data
        return [(base + a, n) for a, n in zip(self.offs, self.sizes)]

    def data(self, got):
        out, left = b"", got
        for a, n in zip(self.offs, self.sizes):
            take = min(n, left)
            out += self.arr[a:a + take].tobytes()
            left -= take
        return out

    def guards_ok(self):
        return all(self.arr[a + n:a + n + 16].tobytes() == b"\xa5" * 16 for a, n in zip(self.offs, self.sizes))

    def free(self):
        if self.pin is not None:
            self.pin.free()


def _stream(oracle, proto, cs, ctype, sizes, seed):
    rng = np.random.default_rng(seed)
    if sizes == "regular":
        dl = [65536] * 150 + [12345]
    elif sizes == "mixed":
        dl = [int(x) for x in np.repeat(rng.choice([4096, 61440, 30000, 65536], 30), rng.integers(1, 6, 30))]
    else:
        dl = [int(x) for x in rng.integers(1, 70000, 80)]
    base = 3 * 65536
    s, _ = build_stream(oracle.crc32c, proto, cs, ctype, dl, seed=seed, corrupt=[(len(dl) - 5, 1)], offset0=base)
    return s, dl, base


@pytest.mark.gpu
@pytest.mark.parametrize("where", ["device_stream", "host_stream"])
@pytest.mark.parametrize("proto,cs,ctype,sizes", [
    (2, 512, CSUM_CRC32C, "regular"),
    (1, 512, CSUM_CRC32, "regular"),
    (2, 4096, CSUM_CRC32C, "mixed"),
    (2, 512, CSUM_CRC32C, "random"),
])
def test_gpu_read_into_host_memory(engine, oracle, where, proto, cs, ctype, sizes):
    """Reads ending inside packets, on packet ends, past the block and at the
    bad packet (the read ends there); one host buffer as large as the read,
    a scatter list of uneven buffers, and buffers smaller than the read
    resumed call by call (AGAIN) -- all equal the oracle's read."""
    s, dl, base = _stream(oracle, proto, cs, ctype, sizes, seed=len(sizes) + cs + proto)
    total = sum(dl)
    whole = oracle.verify_packets(s, proto, cs, ctype)[1]
    starts = np.cumsum([0] + dl[:-1])
    rng = np.random.default_rng(total % 1000)
    cases = [(base + 1000, total // 3), (base + 7, total), (base + total // 2 + 11, total // 4), (base, 1)]
    for ci, (co, rl) in enumerate(cases):
        k = int(np.searchsorted(starts, co - base, side="right")) - 1
        sub = s[whole[k]["stream_off"]:]
        want = oracle.read_packets(sub, co, rl, proto, cs, ctype)
        if where == "device_stream":
            keep, p = _dev(engine, sub, ci % 3)
        else:
            keep = np.frombuffer(sub, np.uint8).copy()
            p = keep.ctypes.data
        # one buffer as large as the read, and a scatter list
        for sizes_l in ([rl], [int(x) for x in rng.integers(1000, 200000, 64)]):
            h = HostIov(sizes_l)
            rc, recs, used, got = engine.read_packets(p, len(sub), None, 0, proto, cs, ctype, client_offset=co,
                                                      read_len=rl, iov=h.iov())
            cap = sum(sizes_l)
            w = want if cap >= rl else oracle.read_packets(sub, co, rl, proto, cs, ctype, cap=cap)
            assert (rc, recs, used) == w[:3], (where, co - base, rl, len(sizes_l))
            assert h.data(got) == w[3] and h.guards_ok(), (where, co - base, rl, len(sizes_l))
        # resumed through buffers of 100 003 bytes (every call but the last fills its buffer)
        at, tot, recs_all, calls, data = 0, 0, [], 0, b""
        while True:
            h = HostIov([min(100003, rl - tot)])
            rc, recs, used, got = engine.read_packets(p + at, len(sub) - at, None, 0, proto, cs, ctype,
                                                      client_offset=co + tot, read_len=rl - tot, iov=h.iov())
            assert h.guards_ok()
            for q in recs:
                q["stream_off"] += at
            recs_all += recs
            data += h.data(got)
            at += used
            tot += got
            calls += 1
            if rc != AGAIN:
                break
            assert calls < 500
        assert (rc, recs_all, at) == want[:3], (where, co - base, rl, "resumed")
        assert data == want[3]
        if where == "device_stream":
            keep.free()


@pytest.mark.gpu
@pytest.mark.parametrize("where", ["device_stream", "host_stream"])
def test_gpu_read_all_into_host_memory(engine, oracle, where):
    """Whole payloads (READ_ALL) into one host buffer -- pageable and pinned --
    equal the payloads before the first error, records equal the oracle's
    verify; one byte short is refused with nothing written past the buffer."""
    dl = [65536] * 40 + [777]
    s, _ = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, dl, seed=21, corrupt=[(30, 2)])
    want = oracle.verify_packets(s)
    expect = b""
    for q in want[1]:
        if q["error"]:
            break
        a = q["stream_off"] + q["header_len"] + q["crc_len"]
        expect += s[a:a + q["data_len"]]
    if where == "device_stream":
        keep, p = _dev(engine, s, 1)
    else:
        keep = np.frombuffer(s, np.uint8).copy()
        p = keep.ctypes.data
    for pinned in (None, engine.PinnedBuffer):
        h = HostIov([sum(dl)], pinned=pinned)
        rc, recs, used, got = engine.read_packets(p, len(s), None, 0, iov=h.iov())
        assert (rc, recs, used) == want and got == len(expect) == 30 * 65536
        assert h.data(got) == expect and h.guards_ok()
        h.free()
    h = HostIov([sum(dl) - 1])
    with pytest.raises(engine.CRC32CError):
        engine.read_packets(p, len(s), None, 0, iov=h.iov())
    assert h.guards_ok()
    if where == "device_stream":
        keep.free()


@pytest.mark.gpu
def test_gpu_read_host_refusals(engine, oracle):
    """Refused: host and device buffers in one scatter list, a host stream
    into device buffers."""
    s, _ = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, [65536] * 4, seed=2)
    keep, p = _dev(engine, s)
    dst = engine.DeviceBuffer(4 * 65536)
    host = np.zeros(4 * 65536, np.uint8)
    with pytest.raises(engine.CRC32CError):
        engine.read_packets(p, len(s), None, 0, client_offset=0, read_len=4 * 65536,
                            iov=[(dst.ptr, 65536), (host.ctypes.data, 3 * 65536)])
    src = np.frombuffer(s, np.uint8).copy()
    with pytest.raises(engine.CRC32CError):
        engine.read_packets(src.ctypes.data, len(s), dst.ptr, dst.nbytes)
    keep.free()
    dst.free()
