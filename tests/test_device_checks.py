"""Device checks of the framing kernels (diagnostic build).

libhadoofus_crc32c_diag.so compiles, into frame_build_kernel (framing and
table phases), header_window_kernel, small_run_kernel and
grid_finalize_kernel, a test of the invariant behind each address they touch
(DCHK, hadoofus_amd/csrc/crc32c_kernels.hip): a record slot inside its pass,
a packet's bytes inside the stream, a copy-out window inside the packet's
data and its destination inside the read.  A violation skips the access,
is counted with the kernel and line of the first one, and the device-stream
call that launched the kernel fails with HDFS_CRC32C_EHIP naming them -- so
a broken invariant is attributed to its own kernel and call instead of
surfacing as an illegal address later.  These tests drive every path of the
device-resident packet walk (grid passes, the header-window walk after a size
change, short runs, copy-out, read windows, malformed first headers,
truncation) through the diagnostic build: results equal the oracle's and no
check fires.  The reporting itself is tested by an injected violation."""
import ctypes

import numpy as np
import pytest

from packet_stream import CSUM_CRC32, CSUM_CRC32C, build_stream


@pytest.fixture(scope="module")
def diag(engine):
    from hadoofus_amd import abi, build
    lib = abi.bind_diag(abi.bind_product(ctypes.CDLL(build.DIAG_LIB)))
    yield lib


def _checks(lib, reset=1):
    out = (ctypes.c_uint32 * 3)()
    assert lib.hdfs_crc32c_diag_device_checks(out, reset) == 0
    return tuple(out)


def _dev(engine, s, shift=0):
    buf = engine.DeviceBuffer(len(s) + shift + 64)
    buf.fill(0)
    buf.upload(np.frombuffer(s, np.uint8), offset=shift)
    engine.device_sync()
    return buf, buf.ptr + shift


@pytest.mark.gpu
def test_gpu_device_check_reporting(engine, diag, oracle):
    """An injected violation (kernel id 0) is reported by the next
    device-stream call, with its line, and then cleared."""
    assert _checks(diag) == (0, 0, 0)
    v = _checks(diag, reset=-1)
    assert v[0] == 0 and v[1] > 0 and v[2] == 1
    s, _ = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, [65536] * 8, seed=1)
    keep, p = _dev(engine, s)
    with pytest.raises(engine.CRC32CError) as ei:
        engine.verify_packets(None, dptr=p, nbytes=len(s), lib=diag)
    msg = str(ei.value)
    assert "device check failed in check self-test" in msg and "crc32c_kernels.hip:%d" % v[1] in msg
    assert _checks(diag) == (0, 0, 0)  # cleared by the call that reported it
    assert engine.verify_packets(None, dptr=p, nbytes=len(s), lib=diag) == oracle.verify_packets(s)
    keep.free()


def _payloads(s, pkts):
    out = bytearray()
    for q in pkts:
        if q["error"]:
            break
        a = q["stream_off"] + q["header_len"] + q["crc_len"]
        out += s[a:a + q["data_len"]]
    return bytes(out)


@pytest.mark.gpu
@pytest.mark.parametrize("proto,cs,ctype,sizes,shift", [
    (2, 512, CSUM_CRC32C, "regular", 0),   # grid passes, tiled verify + copy
    (1, 512, CSUM_CRC32C, "regular", 3),
    (2, 512, CSUM_CRC32, "partial", 1),    # generic tiles on every packet
    (2, 4096, CSUM_CRC32C, "mixed", 0),    # grid passes + header-window walk
    (2, 512, CSUM_CRC32C, "random", 2),
    (2, 512, CSUM_CRC32C, "short", 1),     # short runs (small_run_kernel)
])
def test_gpu_device_paths_no_check_fires(engine, diag, oracle, proto, cs, ctype, sizes, shift):
    rng = np.random.default_rng(cs + proto + shift + len(sizes))
    if sizes == "regular":
        dl = [65536] * 400 + [12345]
    elif sizes == "partial":
        dl = [40000] * 150
    elif sizes == "mixed":
        dl = [int(x) for x in np.repeat(rng.choice([4096, 61440, 30000, 65536], 40), rng.integers(1, 8, 40))]
    elif sizes == "short":
        dl = [65536, 65536, 1000]
    else:
        dl = [int(x) for x in rng.integers(1, 70000, 200)]
    corrupt = sorted({(int(k), 0) for k in rng.integers(0, len(dl), 5)})
    s, _ = build_stream(oracle.crc32c, proto, cs, ctype, dl, seed=len(dl) + cs, corrupt=corrupt)
    s_clean, _ = build_stream(oracle.crc32c, proto, cs, ctype, dl, seed=len(dl) + cs)
    total = sum(dl)
    assert _checks(diag) == (0, 0, 0)
    for stream in (s, s_clean):
        keep, p = _dev(engine, stream, shift)
        want = oracle.verify_packets(stream, proto, cs, ctype)
        assert engine.verify_packets(None, proto, cs, ctype, dptr=p, nbytes=len(stream), lib=diag) == want
        assert engine.parse_packets(None, proto, cs, ctype, dptr=p, nbytes=len(stream), lib=diag)[2] == want[2]
        cut = len(stream) - 777
        assert engine.verify_packets(None, proto, cs, ctype, dptr=p, nbytes=cut, lib=diag) == \
            oracle.verify_packets(stream[:cut], proto, cs, ctype)
        dst = engine.DeviceBuffer(total + 4096)
        rc, pkts, used, got = engine.read_packets(p, len(stream), dst.ptr, total, proto, cs, ctype, lib=diag)
        assert (rc, pkts, used) == want
        assert dst.download(got).tobytes() == _payloads(stream, want[1])
        # client reads: windows starting inside a packet, ending inside another
        for co, rl in ((0, 1), (dl[0] - 3, 10), (total // 3 + 5, total // 4), (total - 1, 1)):
            rc2, pk2, used2, got2 = engine.read_packets(p, len(stream), dst.ptr, rl, proto, cs, ctype,
                                                               client_offset=co, read_len=rl, lib=diag)
            wrc, wpk, wused, wdata = oracle.read_packets(stream, co, rl, proto, cs, ctype)
            assert (rc2, pk2, used2, got2) == (wrc, wpk, wused, len(wdata)), (co, rl)
            assert dst.download(got2).tobytes() == wdata
        dst.free()
        keep.free()
        assert _checks(diag) == (0, 0, 0)


@pytest.mark.gpu
@pytest.mark.parametrize("proto", [1, 2])
def test_gpu_malformed_first_headers_no_check_fires(engine, diag, oracle, proto):
    """Wrong first-header strides (negative, huge, short plen) and streams
    shorter than a header: the grid framing reads nothing outside the stream."""
    s, _ = build_stream(oracle.crc32c, proto, 512, CSUM_CRC32C, [65536] * 5 + [777], seed=11)
    cases = [s[:n] for n in range(1, 8)] + [s[:30], s]
    for plen in (-5, 0, 1, 3, 0x7FFFFFF0, 200):
        b = bytearray(s)
        b[0:4] = (plen & 0xFFFFFFFF).to_bytes(4, "big")
        cases.append(bytes(b))
    for c in cases:
        keep, p = _dev(engine, c, 1)
        assert engine.verify_packets(None, proto, 512, CSUM_CRC32C, dptr=p, nbytes=len(c), lib=diag) == \
            oracle.verify_packets(c, proto, 512, CSUM_CRC32C), len(c)
        keep.free()
    assert _checks(diag) == (0, 0, 0)
