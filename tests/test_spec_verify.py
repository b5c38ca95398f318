"""Speculative one-launch verify of device-resident packet runs (round 4).

spec_verify_kernel takes a run's layout from packet 0 and verifies every
packet through a closed-form segment table in ONE launch, checking the other
headers on the side (crc32c_internal.h, SpecCtl).  These tests hold it to the
oracle (oracle_verify_packets / oracle_read_packets: src/datanode.c:2345-2553,
2931-2963) and to the regular device framing path of the same library (the
diagnostic build with hdfs_crc32c_set_speculation(0)), and use the diagnostic
build's counters to show which runs the speculative launch took, which it
handed back (a header off the run: framed the regular way), and which it
never tried (packet 0 does not start a run of equal whole-chunk packets).
"""
import ctypes

import numpy as np
import pytest

from packet_stream import CSUM_CRC32, CSUM_CRC32C, build_stream

BAD, ERR_PACKET_SIZE = 29, 25


@pytest.fixture(scope="module")
def diag(engine):
    from hadoofus_amd import abi, build
    lib = abi.bind_diag(abi.bind_product(ctypes.CDLL(build.DIAG_LIB)))
    assert lib.hdfs_crc32c_set_speculation(1) == 0
    yield lib
    lib.hdfs_crc32c_set_speculation(1)


def _stats(lib):
    out = (ctypes.c_uint64 * 4)()
    assert lib.hdfs_crc32c_diag_spec_stats(out, 1) == 0
    return dict(zip(("launched", "eligible", "taken", "exc"), out))


def _dev(engine, s, shift=0):
    buf = engine.DeviceBuffer(len(s) + shift + 64)
    buf.fill(0)
    buf.upload(np.frombuffer(s, np.uint8), offset=shift)
    engine.device_sync()
    return buf, buf.ptr + shift


def _payloads(s, pkts):
    out = bytearray()
    for p in pkts:
        if p["error"]:
            break
        a = p["stream_off"] + p["header_len"] + p["crc_len"]
        out += s[a:a + p["data_len"]]
    return bytes(out)


def _both(engine, diag, fn):
    """fn(lib) with speculation on (stats returned) and off."""
    _stats(diag)
    on = fn(diag)
    st = _stats(diag)
    assert diag.hdfs_crc32c_set_speculation(0) == 0
    try:
        off = fn(diag)
    finally:
        diag.hdfs_crc32c_set_speculation(1)
    assert _stats(diag)["launched"] == 0
    return on, off, st


# (name, proto, cs, ctype, data lengths, build_stream kwargs, expected speculation outcome)
RUNS = [
    ("v2_block", 2, 512, CSUM_CRC32C, [65536] * 128, {}, "taken"),
    ("v2_block_crc32", 2, 512, CSUM_CRC32, [65536] * 100, {}, "taken"),
    ("v1_block_last_flag", 1, 512, CSUM_CRC32C, [65536] * 100, {"last_empty": False}, "taken"),
    ("v2_cs4096", 2, 4096, CSUM_CRC32C, [65536] * 100, {}, "taken"),
    ("v2_cs1536_partial_tile", 2, 1536, CSUM_CRC32C, [1536 * 20] * 300, {}, "taken"),
    ("v2_short_tail", 2, 512, CSUM_CRC32C, [65536] * 100 + [12345], {}, "taken"),
    ("v2_seq_jumps", 2, 512, CSUM_CRC32C, [65536] * 100, {"seqnos": [k + (7 if k >= 50 else 0) for k in range(100)]},
     "taken"),
    ("v2_offset_skew", 2, 512, CSUM_CRC32C, [65536] * 100, {"offset_skew": {30: 512, 31: -9}}, "taken"),
    ("v2_sync_every", 2, 512, CSUM_CRC32C, [65536] * 100, {"sync_every": 3}, "handed_back"),  # 27-B headers mixed in
    # packet 40 has a 27-B syncBlock header and dataLen cut by 2 --
    # packet 0's stride and CRC length, another layout (later offsets skewed
    # back onto the prediction, so it is the run's only exception)
    ("v2_sync_same_stride", 2, 512, CSUM_CRC32C, [65536] * 40 + [65534] + [65536] * 59,
     {"sync_at": (40,), "offset_skew": {k: 2 for k in range(41, 100)}}, "handed_back"),
    ("v2_size_break", 2, 512, CSUM_CRC32C, [65536] * 60 + [30000] + [65536] * 40, {}, "handed_back"),
    ("v2_many_exceptions", 2, 512, CSUM_CRC32C, [65536] * 100, {"seqnos": [3 * k for k in range(100)]},
     "handed_back"),
    ("v2_partial_chunks", 2, 512, CSUM_CRC32C, [40000] * 200, {}, "not_eligible"),
    ("v2_cs100", 2, 100, CSUM_CRC32C, [6400] * 1000, {}, "not_eligible"),
]


@pytest.mark.gpu
@pytest.mark.parametrize("name,proto,cs,ctype,dl,kw,outcome", RUNS, ids=[r[0] for r in RUNS])
def test_gpu_spec_runs_vs_oracle(engine, diag, oracle, name, proto, cs, ctype, dl, kw, outcome):
    """Records, verdicts, consumed bytes and the copied payload equal the
    oracle's and the regular framing path's; the speculative launch took
    exactly the runs it should."""
    rng = np.random.default_rng(len(dl) + cs + proto)
    corrupt = sorted({(int(k), int(rng.integers(0, dl[k] // cs))) for k in rng.integers(0, len(dl), 6)})
    s, bad = build_stream(oracle.crc32c, proto, cs, ctype, dl, seed=len(dl), corrupt=corrupt, **kw)
    want = oracle.verify_packets(s, proto, cs, ctype)
    for shift in (0, 3):
        keep, p = _dev(engine, s, shift)
        on, off, st = _both(engine, diag, lambda lib: engine.verify_packets(None, proto, cs, ctype, dptr=p,
                                                                            nbytes=len(s), lib=lib))
        assert on == want and off == want, (name, shift)
        assert {k: (q["first_bad"], q["bad_chunks"]) for k, q in enumerate(on[1]) if q["error"] == BAD} == \
            {k: (v[0], len(v)) for k, v in bad.items()}
        if outcome == "taken":
            assert st["taken"] >= 1 and st["exc"] == 0, st
        elif outcome == "handed_back":
            assert st["eligible"] == 1 and st["exc"] == 1 and st["taken"] == 0, st
        else:
            assert st["eligible"] == 0 and st["taken"] == 0, st
        # verify + copy-out: the payload before the first error, byte for byte
        dst = engine.DeviceBuffer(sum(dl) + 64)
        dst.fill(0xA5)
        rc, pkts, used, got = engine.read_packets(p, len(s), dst.ptr, sum(dl), proto, cs, ctype, lib=diag)
        assert (rc, pkts, used) == want
        expect = _payloads(s, want[1])
        assert got == len(expect) and dst.download(got).tobytes() == expect
        assert dst.download(64, offset=sum(dl)).tobytes() == b"\xa5" * 64
        dst.free()
        keep.free()


@pytest.mark.gpu
def test_gpu_spec_tails(engine, diag, oracle):
    """What follows the run: the empty last packet (recorded, the walk ends),
    the stream ending exactly after the run or inside the next packet (not
    recorded), a packet of another size (the next pass frames it), a framing
    error (recorded, the walk ends), max_pkts cutting the run, and the
    speculative launch's own limit of 65 536 packets per pass."""
    cs, dl = 512, [65536] * 80
    s, _ = build_stream(oracle.crc32c, 2, cs, CSUM_CRC32C, dl, seed=5)
    whole = oracle.verify_packets(s)[1]
    end_run = whole[-1]["stream_off"]          # offset of the empty last packet
    stride = whole[1]["stream_off"]
    bad_tail = bytearray(s)
    bad_tail[end_run:end_run + 4] = (0x7FFFFFFF).to_bytes(4, "big")   # plen > 1 GiB: PACKET_SIZE
    cases = {
        "empty_last": s,
        "exact_end": s[:end_run],
        "cut_in_next": s[:end_run - stride // 2],
        "framing_error_tail": bytes(bad_tail),
        "other_size_tail": s[:end_run] + build_stream(oracle.crc32c, 2, cs, CSUM_CRC32C, [1000], seed=6,
                                                      offset0=80 * 65536)[0],
    }
    for name, c in cases.items():
        want = oracle.verify_packets(c)
        keep, p = _dev(engine, c, 1)
        on, off, st = _both(engine, diag, lambda lib: engine.verify_packets(None, dptr=p, nbytes=len(c), lib=lib))
        assert on == want == off, name
        assert st["taken"] == 1, (name, st)
        for mp in (10, 79, 80, 81):
            w = oracle.verify_packets(c, max_pkts=mp)
            assert engine.verify_packets(None, max_pkts=mp, dptr=p, nbytes=len(c), lib=diag) == w, (name, mp)
        keep.free()


@pytest.mark.gpu
def test_gpu_spec_many_passes(engine, diag, oracle):
    """70 000 packets of 2 KiB: the first speculative launch takes 65 536
    (one pass), the second the rest of the run, the 1 000-B tail packet is
    framed by the regular pass; corruption on both sides of the pass edge."""
    n = 70000
    dl = [2048] * n + [1000]
    s, bad = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, dl, seed=77,
                          corrupt=[(5, 0), (65535, 3), (65536, 2), (69999, 1)])
    mp = len(dl) + 2
    want = oracle.verify_packets(s, max_pkts=mp)
    keep, p = _dev(engine, s)
    on, off, st = _both(engine, diag, lambda lib: engine.verify_packets(None, max_pkts=mp, dptr=p, nbytes=len(s),
                                                                        lib=lib))
    assert on == want == off
    assert st["taken"] == 2 and st["exc"] == 0, st
    dst = engine.DeviceBuffer(sum(dl))
    rc, pkts, used, delivered = engine.read_packets(p, len(s), dst.ptr, dst.nbytes, max_pkts=mp, lib=diag)
    assert (rc, pkts, used) == want and delivered == 5 * 2048
    assert dst.download(delivered).tobytes() == _payloads(s, want[1])
    keep.free()
    dst.free()


@pytest.mark.gpu
def test_gpu_spec_read_windows(engine, diag, oracle):
    """Client reads over a run of 300 packets (the speculative launch takes
    only the packets the read needs): starting inside packet 0, on its
    first byte, ending inside a later packet, running past the block's end
    (BAD_LASTPACKET), with bad CRCs inside the read, and with a seqno jump
    (an exception whose offsetInBlock is the predicted one); byte-exact
    against the oracle's read loop and nothing written past the read."""
    base = 5 * 65536
    dl = [65536] * 300
    s, _ = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, dl, seed=3, offset0=base, corrupt=[(200, 4)])
    s2, _ = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, dl, seed=4, offset0=base,
                         seqnos=[k + (9 if k > 100 else 0) for k in range(300)])
    total = sum(dl)
    cases = [(s, base + 1000, 150 * 65536), (s, base, 100 * 65536 + 1), (s, base + 77, total),
             (s, base + 3, 250 * 65536), (s2, base + 5, 200 * 65536), (s, base + 65535, 70000)]
    for i, (st_, co, rl) in enumerate(cases):
        want = oracle.read_packets(st_, co, rl)
        keep, p = _dev(engine, st_, i % 3)
        dst = engine.DeviceBuffer(rl + 64)
        for spec in (1, 0):
            assert diag.hdfs_crc32c_set_speculation(spec) == 0
            dst.fill(0xA5)
            got = engine.read_packets(p, len(st_), dst.ptr, rl, client_offset=co, read_len=rl, lib=diag)
            assert got[:3] == want[:3], (i, spec)
            assert dst.download(got[3]).tobytes() == want[3], (i, spec)
            assert dst.download(64, offset=rl).tobytes() == b"\xa5" * 64, (i, spec)
        diag.hdfs_crc32c_set_speculation(1)
        keep.free()
        dst.free()


@pytest.mark.gpu
def test_gpu_spec_copy_out_too_small(engine, diag, oracle):
    """Whole-payload copy-out into a buffer one byte short of a regular run:
    refused (EINVAL: READ_ALL has no read position to resume from), and
    nothing is written past the buffer.  A client read of the same bytes into
    the same buffer returns AGAIN and resumes (the one rule for a short
    destination in the mode that can resume, include/hadoofus_crc32c.h)."""
    dl = [65536] * 100
    s, _ = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, dl, seed=8)
    keep, p = _dev(engine, s)
    cap = sum(dl) - 1
    dst = engine.DeviceBuffer(cap + 4096)
    dst.fill(0xA5)
    _stats(diag)
    with pytest.raises(engine.CRC32CError):
        engine.read_packets(p, len(s), dst.ptr, cap, lib=diag)
    assert _stats(diag)["taken"] == 1
    assert dst.download(4096, offset=cap).tobytes() == b"\xa5" * 4096
    # the same stream and buffer as a client read of the whole block (the
    # mode with a read position): AGAIN with the buffer full, and the
    # resumed call delivers the last byte -- the oracle's read, split the same way
    want = oracle.read_packets(s, 0, sum(dl), cap=cap)
    assert want[0] == 1000 and len(want[3]) == cap
    dst.fill(0xA5)
    got = engine.read_packets(p, len(s), dst.ptr, cap, client_offset=0, read_len=sum(dl), lib=diag)
    assert got[0] == engine.AGAIN and got[:3] == want[:3] and got[3] == cap
    assert dst.download(cap).tobytes() == want[3]
    assert dst.download(4096, offset=cap).tobytes() == b"\xa5" * 4096
    rest = oracle.read_packets(s[got[2]:], cap, 1, cap=1)
    got2 = engine.read_packets(p + got[2], len(s) - got[2], dst.ptr, 1, client_offset=cap, read_len=1, lib=diag)
    assert got2[:3] == rest[:3] and got2[0] == 0 and dst.download(1).tobytes() == rest[3]
    keep.free()
    dst.free()


@pytest.mark.gpu
def test_gpu_spec_product_library(engine, oracle):
    """The release library takes the same path (no knob: speculation is the
    product behaviour) and gives the oracle's records for a regular block,
    and for one whose header breaks the run half way."""
    for dl in ([65536] * 128, [65536] * 64 + [1000] + [65536] * 63):
        s, _ = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, dl, seed=12, corrupt=[(7, 3), (100, 0)])
        keep, p = _dev(engine, s, 2)
        assert engine.verify_packets(None, dptr=p, nbytes=len(s)) == oracle.verify_packets(s)
        keep.free()
