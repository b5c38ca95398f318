"""Client reads written to a file descriptor (round 6): hdfs_crc32c_read_packets_fd
is the reference's hdfs_datanode_read_file -- _recv_packet_copy_data
pwrite()s each verified packet's bytes at fdoffset and advances it
(src/datanode.c:2531-2541, _hdfs_pwrite_all src/net.c:290-313).  The file's
bytes at [fd_offset, fd_offset + delivered) equal the oracle's read loop
(oracle_read_packets) of the same window; records, status and consumed equal
it too; bytes around them are untouched; a failing write is HDFS_CRC32C_EIO
with the bytes before it written."""
import os
import tempfile

import numpy as np
import pytest

from packet_stream import CSUM_CRC32, CSUM_CRC32C, build_stream

EIO = -5


def _dev(engine, s, shift=0):
    buf = engine.DeviceBuffer(len(s) + shift + 64)
    buf.fill(0)
    buf.upload(np.frombuffer(s, np.uint8), offset=shift)
    engine.device_sync()
    return buf, buf.ptr + shift


def _file(size, fill=0x5A):
    fd, path = tempfile.mkstemp(prefix="hdfs_read_fd_")
    os.write(fd, bytes([fill]) * size)
    return fd, path


@pytest.mark.gpu
@pytest.mark.parametrize("where", ["device", "host"])
def test_gpu_read_fd_vs_oracle(engine, oracle, where):
    dl = [65536] * 90 + [4321]
    s, _ = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, dl, seed=31, corrupt=[(70, 2)], offset0=65536)
    hs = np.frombuffer(s, np.uint8).copy()
    keep = None
    if where == "device":
        keep, p = _dev(engine, s, 1)
    else:
        p = hs.ctypes.data
    total = sum(dl)
    # inside the clean part; across the bad packet (ends at it); one byte; a
    # window larger than the 4 MiB staging buffer; past the block's end
    cases = [(65536 + 1000, 5 * 65536), (65536 + 7, total), (65536 + 3 * 65536 + 5, 1),
             (65536 + 3, 68 * 65536), (65536 + 85 * 65536, 2 * total)]
    s_ok, _ = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, [65536] * 80, seed=32, offset0=65536)
    for ci, (co, rl) in enumerate(cases):
        st, ptr = s, p
        if ci == 3:  # a clean 5 MiB stream for the staging-buffer case
            st = s_ok
            if where == "device":
                k2, ptr = _dev(engine, st)
            else:
                h2 = np.frombuffer(st, np.uint8).copy()
                ptr = h2.ctypes.data
        want = oracle.read_packets(st, co, rl)
        fd, path = _file(len(want[3]) + 3000)
        try:
            got = engine.read_packets_fd(ptr, len(st), fd, 1000, co, rl)
            data = open(path, "rb").read()
        finally:
            os.close(fd)
            os.unlink(path)
        assert got[:3] == want[:3], (where, ci)
        assert got[3] == len(want[3]), (where, ci)
        assert data[1000:1000 + got[3]] == want[3], (where, ci)
        assert data[:1000] == b"\x5a" * 1000 and data[1000 + got[3]:] == b"\x5a" * (len(data) - 1000 - got[3])
        if ci == 3 and where == "device":
            k2.free()
    if keep:
        keep.free()


@pytest.mark.gpu
def test_gpu_read_fd_v1_crc32_and_errors(engine, oracle):
    """CRC32 v1 packets; a bad first packet writes nothing and returns the
    error; a read-only fd is EIO; a negative offset or READ_ALL is EINVAL."""
    dl = [65536] * 20
    s, _ = build_stream(oracle.crc32c, 1, 512, CSUM_CRC32, dl, seed=33, last_empty=False)
    keep, p = _dev(engine, s)
    want = oracle.read_packets(s, 100, 10 * 65536, 1, 512, CSUM_CRC32)
    fd, path = _file(0)
    try:
        got = engine.read_packets_fd(p, len(s), fd, 0, 100, 10 * 65536, proto=1, ctype=CSUM_CRC32)
        assert got[:3] == want[:3] and open(path, "rb").read() == want[3]
    finally:
        os.close(fd)
    bad, _ = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, dl, seed=34, corrupt=[(0, 0)])
    kb, pb = _dev(engine, bad)
    wb = oracle.read_packets(bad, 10, 1000)
    fd = os.open(path, os.O_RDWR | os.O_TRUNC)
    try:
        got = engine.read_packets_fd(pb, len(bad), fd, 0, 10, 1000)
        assert got[:3] == wb[:3] and got[0] == 29 and got[3] == 0
        assert os.path.getsize(path) == 0
    finally:
        os.close(fd)
    s2, _ = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, dl, seed=35)
    k2, p2 = _dev(engine, s2)
    ro = os.open(path, os.O_RDONLY)
    try:
        rc, recs, used, got = engine.read_packets_fd(p2, len(s2), ro, 0, 0, 5 * 65536, check=False)
        assert rc == EIO and got == 0
        with pytest.raises(engine.CRC32CError):
            engine.read_packets_fd(p2, len(s2), ro, -1, 0, 100)
        with pytest.raises(engine.CRC32CError):
            engine.read_packets_fd(p2, len(s2), ro, 0, 0, -1)  # READ_ALL: a window is required
    finally:
        os.close(ro)
        os.unlink(path)
    for b in (keep, kb, k2):
        b.free()
