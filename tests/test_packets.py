"""Packet-stream framing + verify (src/datanode.c:2345-2494, 2931-2963).

CPU: the oracle against the constructed fixtures of
oracle/gen_golden_packets.py, and the engine's host-side framing walk
(hdfs_crc32c_parse_packets, no device work) against the same fixtures.
GPU: hdfs_crc32c_verify_packets against the fixtures and, on large
generated streams, against the oracle."""
import json
import os
import struct

import numpy as np
import pytest

from packet_stream import CSUM_CRC32, CSUM_CRC32C, assemble, build_stream, frame_v2, header_v2

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "packet_cases.json")
BAD = 29


def _cases():
    with open(GOLDEN) as f:
        return json.load(f)["cases"]


CASES = _cases()


def _stream(case):
    s = assemble(case["parts"])
    return s[:case["cut"]] if "cut" in case else s


def _framing_only(pkts):
    """Expected records of a framing-only walk: checksum verdicts cleared."""
    out = []
    for p in pkts:
        p = dict(p)
        if p["error"] == BAD:
            p.update(error=0, first_bad=-1, bad_chunks=0)
        out.append(p)
    return out


def _args(case):
    return case["proto"], case["chunk_size"], case["ctype"], case["max_pkts"]


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_packets_fixture(oracle, case):
    rc, pkts, used = oracle.verify_packets(_stream(case), *_args(case))
    assert (rc, used) == (case["expect"]["rc"], case["expect"]["consumed"])
    assert pkts == case["expect"]["packets"]


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_engine_parse_fixture(case):
    import hadoofus_amd as h
    want = _framing_only(case["expect"]["packets"])
    rc, pkts, used = h.parse_packets(_stream(case), *_args(case))
    assert pkts == want
    assert used == case["expect"]["consumed"]
    assert rc == next((p["error"] for p in want if p["error"]), 0)


def test_engine_parse_rejects_bad_args():
    import hadoofus_amd as h
    for kw in (dict(proto=3), dict(ctype=5), dict(chunk_size=0)):
        with pytest.raises(h.CRC32CError):
            h.parse_packets(b"\0" * 64, **kw)


def test_builder_streams_match_oracle(oracle):
    """The generated streams used at GPU scale are what the oracle expects."""
    s, bad = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, [65536] * 5 + [777], corrupt=[(1, 3), (5, 1)])
    rc, pkts, used = oracle.verify_packets(s)
    assert rc == BAD and used == len(s) and len(pkts) == 7
    assert [p["first_bad"] for p in pkts] == [-1, 3, -1, -1, -1, 1, -1]


# --- GPU ---------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_gpu_verify_packets_fixture(engine, case):
    rc, pkts, used = engine.verify_packets(_stream(case), *_args(case))
    assert pkts == case["expect"]["packets"]
    assert (rc, used) == (case["expect"]["rc"], case["expect"]["consumed"])


@pytest.mark.gpu
@pytest.mark.parametrize("proto,cs,ctype,dlen,npk", [
    (2, 512, CSUM_CRC32C, 65536, 2100),    # ~131 MiB: three 64 MiB pieces, both slots
    (1, 512, CSUM_CRC32C, 65536, 300),
    (2, 512, CSUM_CRC32, 65536, 300),
    (2, 4096, CSUM_CRC32C, 61440, 200),
    (2, 512, CSUM_CRC32C, 40000, 500),     # partial last chunk in every packet
])
def test_gpu_verify_packets_large_vs_oracle(engine, oracle, proto, cs, ctype, dlen, npk):
    rng = np.random.default_rng(npk + cs + proto)
    nch = (dlen + cs - 1) // cs
    corrupt = [(int(rng.integers(0, npk)), int(rng.integers(0, nch))) for _ in range(25)]
    dl = [dlen] * (npk - 1) + [dlen // 3 + 1]
    s, bad = build_stream(oracle.crc32c, proto, cs, ctype, dl, seed=npk, corrupt=corrupt)
    want = oracle.verify_packets(s, proto, cs, ctype)
    got = engine.verify_packets(s, proto, cs, ctype)
    assert got[0] == want[0] == BAD
    assert got[2] == want[2] == len(s)
    assert got[1] == want[1]
    assert {k: (p["first_bad"], p["bad_chunks"]) for k, p in enumerate(got[1]) if p["error"]} == \
        {k: (v[0], len(v)) for k, v in bad.items()}


@pytest.mark.gpu
def test_gpu_verify_packets_huge_packet(engine, oracle):
    """A packet larger than the 64 MiB piece gets a piece of its own."""
    dl = [65536, (80 << 20) + 100, 65536]
    s, bad = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, dl, seed=5, corrupt=[(1, 0), (1, 163840), (2, 7)])
    got = engine.verify_packets(s)
    assert got == oracle.verify_packets(s)
    assert got[1][1]["bad_chunks"] == 2 and got[1][1]["first_bad"] == 0


@pytest.mark.gpu
def test_gpu_verify_packets_pinned_stream(engine, oracle):
    s, _ = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, [65536] * 64, seed=9, corrupt=[(10, 10)])
    pin = engine.PinnedBuffer(len(s))
    pin.array[:] = np.frombuffer(s, np.uint8)
    got = engine.verify_packets(pin.array)
    assert got == oracle.verify_packets(s)
    pin.free()


@pytest.mark.gpu
def test_gpu_packet_consumer_runs(engine, tmp_path):
    """The C consumer (tests/consumer/packet_consumer.c) verifies a packet
    run in one call and through a session fed in odd-sized reads."""
    import subprocess

    from hadoofus_amd import build
    from test_abi import build_c
    exe = build_c(tmp_path, build.LIB, "packet_consumer")
    p = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "0 failures" in p.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("proto,cs,ctype,dlen,last_empty", [
    (2, 512, CSUM_CRC32C, 65536, True),   # one data packet + the empty last one
    (2, 512, CSUM_CRC32C, 65536, False),
    (1, 512, CSUM_CRC32C, 1000, True),
    (2, 100, CSUM_CRC32C, 30000, True),   # chunk 100: still the one-launch path
    (2, 777, CSUM_CRC32C, 30000, True),   # chunk 777 (not a multiple of 4): piece pipeline
    (2, 512, CSUM_CRC32, 65536, True),
    (2, 32, CSUM_CRC32C, 65536, True),    # 2048 chunks: the one-launch path's limit
    (2, 16, CSUM_CRC32C, 65536, True),    # 4096 chunks: piece pipeline
])
def test_gpu_verify_single_packet(engine, oracle, proto, cs, ctype, dlen, last_empty):
    """A run holding one data packet (the per-read case) takes the one-launch
    small-call kernel when it fits; verdicts equal the oracle's, clean and
    with one or two corrupted chunks."""
    nch = (dlen + cs - 1) // cs
    for corrupt in ((), ((0, nch - 1),), ((0, 0), (0, nch // 2))):
        s, bad = build_stream(oracle.crc32c, proto, cs, ctype, [dlen], seed=dlen + cs, corrupt=corrupt,
                              last_empty=last_empty)
        want = oracle.verify_packets(s, proto, cs, ctype)
        got = engine.verify_packets(s, proto, cs, ctype)
        assert got == want
        assert {k: (p["first_bad"], p["bad_chunks"]) for k, p in enumerate(got[1]) if p["error"]} == \
            {k: (v[0], len(v)) for k, v in bad.items()}


# --- GPU: device-resident streams (GPU-direct receive) -----------------------
def _dev(engine, s, shift=0):
    """Stream bytes in device memory at byte offset `shift` of a fresh buffer."""
    buf = engine.DeviceBuffer(len(s) + shift + 64)
    buf.fill(0)
    buf.upload(np.frombuffer(s, np.uint8), offset=shift)
    engine.device_sync()
    return buf, buf.ptr + shift


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_gpu_device_stream_fixture(engine, case):
    """The golden packet runs, uploaded to HBM: framing over header windows
    and verify in place give the fixture's records."""
    s = _stream(case)
    if not s:
        pytest.skip("empty stream")
    proto, cs, ctype, max_pkts = _args(case)
    for shift in (0, 3):
        keep, p = _dev(engine, s, shift)
        got = engine.verify_packets(None, proto, cs, ctype, max_pkts, dptr=p, nbytes=len(s))
        assert got[1] == case["expect"]["packets"]
        assert (got[0], got[2]) == (case["expect"]["rc"], case["expect"]["consumed"])
        rc, pkts, used = engine.parse_packets(None, proto, cs, ctype, max_pkts, dptr=p, nbytes=len(s))
        assert pkts == _framing_only(case["expect"]["packets"]) and used == case["expect"]["consumed"]
        keep.free()


@pytest.mark.gpu
@pytest.mark.parametrize("proto,cs,ctype,sizes,shift", [
    (2, 512, CSUM_CRC32C, "regular", 0),   # one window covers the run
    (1, 512, CSUM_CRC32C, "regular", 1),   # v1: CRCs and data at odd offsets
    (2, 512, CSUM_CRC32, "regular", 0),
    (2, 4096, CSUM_CRC32C, "mixed", 0),    # window misses: sizes change every few packets
    (2, 512, CSUM_CRC32C, "random", 2),    # every packet a different size
])
def test_gpu_device_stream_vs_oracle(engine, oracle, proto, cs, ctype, sizes, shift):
    rng = np.random.default_rng(len(sizes) + cs + proto)
    if sizes == "regular":
        dl = [65536] * 700 + [12345]
    elif sizes == "mixed":
        dl = [int(x) for x in np.repeat(rng.choice([4096, 61440, 30000, 65536], 60), rng.integers(1, 8, 60))]
    else:
        dl = [int(x) for x in rng.integers(1, 70000, 300)]
    corrupt = set()  # distinct chunks (two flips of one chunk would cancel)
    for _ in range(20):
        k = int(rng.integers(0, len(dl)))
        corrupt.add((k, int(rng.integers(0, (dl[k] + cs - 1) // cs))))
    s, bad = build_stream(oracle.crc32c, proto, cs, ctype, dl, seed=len(dl), corrupt=sorted(corrupt))
    want = oracle.verify_packets(s, proto, cs, ctype)
    keep, p = _dev(engine, s, shift)
    got = engine.verify_packets(None, proto, cs, ctype, dptr=p, nbytes=len(s))
    assert got == want
    assert got[0] == BAD and got[2] == len(s)
    assert {k: (q["first_bad"], q["bad_chunks"]) for k, q in enumerate(got[1]) if q["error"]} == \
        {k: (v[0], len(v)) for k, v in bad.items()}
    # the host path over the same bytes agrees, and so does a truncated view
    assert engine.verify_packets(s, proto, cs, ctype) == got
    cut = len(s) - 1000
    assert engine.verify_packets(None, proto, cs, ctype, dptr=p, nbytes=cut) == \
        oracle.verify_packets(s[:cut], proto, cs, ctype)
    # max_pkts stops the walk early exactly like the host path
    assert engine.verify_packets(None, proto, cs, ctype, max_pkts=37, dptr=p, nbytes=len(s)) == \
        engine.verify_packets(s, proto, cs, ctype, max_pkts=37)
    keep.free()


@pytest.mark.gpu
@pytest.mark.parametrize("proto", [1, 2])
def test_gpu_device_stream_first_window_guess(engine, oracle, proto):
    """The first header window takes its stride from the first header on the
    device (header_len + plen - 4).  Wrong guesses -- a first plen that is
    negative, huge or too small, and streams shorter than a header -- must
    give exactly the oracle's records (src/datanode.c:2428-2446)."""
    cs = 512
    s, _ = build_stream(oracle.crc32c, proto, cs, CSUM_CRC32C, [65536] * 5 + [777], seed=11)
    cases = [s[:n] for n in range(0, 8)] + [s[:30], s]
    for plen in (-5, 0, 1, 3, 0x7FFFFFF0, 200):
        b = bytearray(s)
        b[0:4] = (plen & 0xFFFFFFFF).to_bytes(4, "big")
        cases.append(bytes(b))
    for c in cases:
        want = oracle.verify_packets(c, proto, cs, CSUM_CRC32C)
        if not c:
            continue
        keep, p = _dev(engine, c, 1)
        assert engine.verify_packets(None, proto, cs, CSUM_CRC32C, dptr=p, nbytes=len(c)) == want, len(c)
        assert engine.verify_packets(c, proto, cs, CSUM_CRC32C) == want, len(c)
        keep.free()


# --- GPU: device-resident streams, verify + copy-out -------------------------
def _payloads(s, pkts):
    """Data bytes of every packet before the first error (what the reference
    copies out, src/datanode.c:2470-2553), concatenated in stream order."""
    out = bytearray()
    for p in pkts:
        if p["error"]:
            break
        a = p["stream_off"] + p["header_len"] + p["crc_len"]
        out += s[a:a + p["data_len"]]
    return bytes(out)


@pytest.mark.gpu
@pytest.mark.parametrize("proto,cs,ctype,sizes,shift,corrupt_at", [
    (2, 512, CSUM_CRC32C, "regular", 0, None),   # device framing in one pass, tiled kernel copies
    (2, 512, CSUM_CRC32C, "regular", 3, 400),    # odd offsets; copy stops counting at the bad packet
    (1, 512, CSUM_CRC32C, "regular", 1, None),
    (2, 512, CSUM_CRC32, "partial", 0, None),    # 40000-B packets: partial chunks copied by the generic kernel
    (2, 100, CSUM_CRC32C, "partial", 2, 7),      # chunk 100: every chunk on the generic kernel
    (2, 4096, CSUM_CRC32C, "mixed", 0, None),    # sizes change: grid passes + window-walk fallback
    (2, 512, CSUM_CRC32C, "random", 1, 150),
])
def test_gpu_device_stream_copy_out(engine, oracle, proto, cs, ctype, sizes, shift, corrupt_at):
    """Verify + fused copy-out (hdfs_crc32c_read_packets): records equal
    the oracle's, and the destination holds exactly the de-framed payload of
    every packet before the first error, byte for byte."""
    rng = np.random.default_rng(cs + proto + shift)
    if sizes == "regular":
        dl = [65536] * 600 + [12345]
    elif sizes == "partial":
        dl = [40000] * 200
    elif sizes == "mixed":
        dl = [int(x) for x in np.repeat(rng.choice([4096, 61440, 30000, 65536], 40), rng.integers(1, 8, 40))]
    else:
        dl = [int(x) for x in rng.integers(1, 70000, 250)]
    corrupt = [] if corrupt_at is None else [(corrupt_at, 1)]
    s, bad = build_stream(oracle.crc32c, proto, cs, ctype, dl, seed=len(dl) + cs, corrupt=corrupt)
    mp = len(dl) + 2
    want = oracle.verify_packets(s, proto, cs, ctype, max_pkts=mp)
    keep, p = _dev(engine, s, shift)
    total = sum(dl)
    dst = engine.DeviceBuffer(total + 64)
    dst.fill(0xA5)
    rc, pkts, used, delivered = engine.read_packets(p, len(s), dst.ptr, total, proto, cs, ctype, max_pkts=mp)
    assert (rc, pkts, used) == want
    expect = _payloads(s, want[1])
    assert delivered == len(expect)
    assert dst.download(delivered).tobytes() == expect
    if corrupt_at is None:
        assert delivered == total
    # the plain verify of the same bytes agrees
    assert engine.verify_packets(None, proto, cs, ctype, max_pkts=mp, dptr=p, nbytes=len(s)) == want
    keep.free()
    dst.free()


@pytest.mark.gpu
def test_gpu_device_stream_copy_out_errors(engine, oracle):
    """Refused: a destination smaller than the payload, a host stream into
    device buffers and CSUM_NULL (no verify to fuse the copy into).  A host
    destination is accepted (round 5, tests/test_read_host.py)."""
    s, _ = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, [65536] * 8, seed=3)
    keep, p = _dev(engine, s)
    dst = engine.DeviceBuffer(8 * 65536)
    with pytest.raises(engine.CRC32CError):
        engine.read_packets(p, len(s), dst.ptr, 8 * 65536 - 1)
    host = np.zeros(8 * 65536, np.uint8)
    rc, pkts, used, delivered = engine.read_packets(p, len(s), host.ctypes.data, host.nbytes)
    assert rc == 0 and delivered == 8 * 65536 and used == len(s)
    with pytest.raises(engine.CRC32CError):
        engine.read_packets(p, len(s), dst.ptr, dst.nbytes, ctype=0)
    src = np.frombuffer(s, np.uint8).copy()
    with pytest.raises(engine.CRC32CError):
        engine.read_packets(src.ctypes.data, len(s), dst.ptr, dst.nbytes)
    rc, pkts, used, delivered = engine.read_packets(p, len(s), dst.ptr, dst.nbytes)
    assert rc == 0 and delivered == 8 * 65536 and used == len(s)
    keep.free()
    dst.free()


@pytest.mark.gpu
def test_gpu_device_stream_many_passes(engine, oracle):
    """More packets than one device framing pass holds (65 536 grid points):
    2 KiB packets, ~200 MiB of stream, two passes plus the tail; records,
    verdicts and the copied payload are exact."""
    n = 70000
    dl = [2048] * n + [1000]
    s, bad = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, dl, seed=77, corrupt=[(5, 0), (65535, 3), (65536, 2),
                                                                                     (69999, 1)])
    mp = len(dl) + 2
    want = oracle.verify_packets(s, max_pkts=mp)
    keep, p = _dev(engine, s)
    got = engine.verify_packets(None, max_pkts=mp, dptr=p, nbytes=len(s))
    assert got == want
    dst = engine.DeviceBuffer(sum(dl))
    rc, pkts, used, delivered = engine.read_packets(p, len(s), dst.ptr, dst.nbytes, max_pkts=mp)
    assert (rc, pkts, used) == want and delivered == 5 * 2048
    assert dst.download(delivered).tobytes() == _payloads(s, want[1])
    keep.free()
    dst.free()


@pytest.mark.gpu
@pytest.mark.parametrize("dlen,cs", [(4096, 512), (3000, 512), (4096, 100)])
def test_gpu_device_stream_many_bad_packets(engine, oracle, dlen, cs):
    """More bad packets than the verdict area beside the summary holds (1 024):
    the verify launch's bad-packet list spills to HBM and every verdict still
    comes back exact -- tiled chunks only (4 096 B), a partial last chunk per
    packet (3 000 B: one generic tile each, taken by the same launch's waves
    after their tiled rounds), every chunk generic (chunk size 100)."""
    npk = 3000
    rng = np.random.default_rng(dlen + cs)
    ks = sorted(int(k) for k in rng.choice(npk, 1700, replace=False))
    corrupt = [(k, int(rng.integers(0, (dlen + cs - 1) // cs))) for k in ks]
    dl = [dlen] * npk
    s, bad = build_stream(oracle.crc32c, 2, cs, CSUM_CRC32C, dl, seed=npk + dlen, corrupt=corrupt)
    want = oracle.verify_packets(s, 2, cs, CSUM_CRC32C)
    assert sum(1 for q in want[1] if q["error"]) == 1700
    keep, p = _dev(engine, s, 1)
    got = engine.verify_packets(None, 2, cs, CSUM_CRC32C, dptr=p, nbytes=len(s))
    assert got == want
    assert {k: (q["first_bad"], q["bad_chunks"]) for k, q in enumerate(got[1]) if q["error"]} == \
        {k: (v[0], len(v)) for k, v in bad.items()}
    keep.free()


@pytest.mark.gpu
@pytest.mark.parametrize("proto,pattern", [(2, "few"), (1, "few"), (2, "all"), (2, "last")])
def test_gpu_device_stream_irregular_headers(engine, oracle, proto, pattern):
    """Runs of equal-size packets whose headers leave the regular progression
    (seqno + 1, offsetInBlock + dataLen): the device framing reports those
    packets as exceptions to the prediction from packet 0 -- a few (they ride
    with the summary), more than its host area holds (every seqno shuffled:
    the records come back from HBM), or only the final packet."""
    npk = 300
    rng = np.random.default_rng(npk + proto + len(pattern))
    seqnos, skew = list(range(npk)), {}
    if pattern == "few":
        for k in (1, 10, 77, 200, 299):
            seqnos[k] += 5
        skew = {150: 512, 151: -3}
    elif pattern == "all":
        seqnos = [int(x) for x in rng.permutation(npk)]
    else:
        seqnos[-1] = 10 ** 12
    dl = [65536] * npk
    s, bad = build_stream(oracle.crc32c, proto, 512, CSUM_CRC32C, dl, seed=npk, corrupt=[(3, 9), (150, 0)],
                          seqnos=seqnos, offset_skew=skew)
    want = oracle.verify_packets(s, proto, 512, CSUM_CRC32C)
    assert [q["seqno"] for q in want[1][:npk]] == seqnos
    for shift in (0, 1):
        keep, p = _dev(engine, s, shift)
        got = engine.verify_packets(None, proto, 512, CSUM_CRC32C, dptr=p, nbytes=len(s))
        assert got == want
        assert engine.parse_packets(None, proto, 512, CSUM_CRC32C, dptr=p, nbytes=len(s))[1] == \
            _framing_only(want[1])
        dst = engine.DeviceBuffer(sum(dl))
        rc, pkts, used, delivered = engine.read_packets(p, len(s), dst.ptr, dst.nbytes, proto)
        assert (rc, pkts, used) == want and dst.download(delivered).tobytes() == _payloads(s, want[1])
        keep.free()
        dst.free()


@pytest.mark.gpu
@pytest.mark.parametrize("proto,cs,ctype", [(2, 512, CSUM_CRC32C), (1, 512, CSUM_CRC32C), (2, 4096, CSUM_CRC32),
                                            (2, 100, CSUM_CRC32C), (2, 64, CSUM_CRC32C)])
def test_gpu_device_stream_short_runs(engine, oracle, proto, cs, ctype):
    """Short device-resident runs (the per-read case) go through the one-launch
    path (small_run_kernel: framing + verify + optional copy-out per packet
    workgroup) when they fit it and through the regular chain when they do
    not (more than 64 packets, a packet over 64 KiB, several chunks of a size
    that is not a multiple of 64, packets off the grid): every case equals
    the oracle and the host path, and the copied-out payload is exact."""
    rng = np.random.default_rng(cs + proto + ctype)
    cases = [[65536], [65536] * 3, [65536] * 16, [65536] * 64, [65536] * 65, [40000] * 5, [1], [777] * 4,
             [65536, 100, 65536], [70000], [65536] * 15 + [12345], [4096] * 16]
    for dl in cases:
        corrupt = set()
        for _ in range(3):
            k = int(rng.integers(0, len(dl)))
            corrupt.add((k, int(rng.integers(0, (dl[k] + cs - 1) // cs))))
        for last_empty in (True, False):
            s, bad = build_stream(oracle.crc32c, proto, cs, ctype, dl, seed=len(dl), corrupt=sorted(corrupt),
                                  last_empty=last_empty)
            want = oracle.verify_packets(s, proto, cs, ctype)
            for shift in (0, 3):
                keep, p = _dev(engine, s, shift)
                got = engine.verify_packets(None, proto, cs, ctype, dptr=p, nbytes=len(s))
                assert got == want, (dl, last_empty, shift)
                for mp in (1, 2):
                    assert engine.verify_packets(None, proto, cs, ctype, max_pkts=mp, dptr=p, nbytes=len(s)) == \
                        oracle.verify_packets(s, proto, cs, ctype, max_pkts=mp), (dl, mp)
                # verify + copy-out: the payload before the first error, byte for byte
                dstb = engine.DeviceBuffer(sum(dl) + 64)
                dstb.fill(0xA5)
                rc, pkts, used, delivered = engine.read_packets(p, len(s), dstb.ptr, sum(dl), proto, cs, ctype)
                assert (rc, pkts, used) == want, (dl, "copy")
                expect = _payloads(s, want[1])
                assert delivered == len(expect) and dstb.download(delivered).tobytes() == expect, (dl, "copy")
                dstb.free()
                keep.free()
            assert engine.verify_packets(s, proto, cs, ctype) == want


# --- client read windows (hdfs_datanode_read's bloff / len) ------------------
# The reference's read loop over a packet stream (src/datanode.c:1476-1481,
# 2448-2456, 2478-2549).  The reference holds no packet fixtures (its read
# tests need a live cluster): the expectations below follow from the
# construction, the oracle restates the loop (oracle_read_packets), and the
# GPU tests hold the engine to the oracle.
def _payload_of(s, pkts, k):
    p = pkts[k]
    a = p["stream_off"] + p["header_len"] + p["crc_len"]
    return s[a:a + p["data_len"]]


def _read_cases(oracle):
    """(name, stream, client_offset, read_len, expected rc, expected records,
    expected delivered bytes) -- constructed."""
    cs, dl = 512, [65536] * 6 + [12345]
    s, _ = build_stream(oracle.crc32c, 2, cs, CSUM_CRC32C, dl, seed=1, offset0=3 * 65536)
    whole = oracle.verify_packets(s)[1]
    pay = b"".join(_payload_of(s, whole, k) for k in range(len(dl)))
    base = 3 * 65536
    out = []
    # starts inside packet 0, ends inside packet 3
    out.append(("mid_to_mid", s, base + 1000, 3 * 65536 - 500, 0, 4, pay[1000:1000 + 3 * 65536 - 500]))
    # exactly the block's bytes: stops at the last data packet, the empty last packet unread
    total = sum(dl)
    out.append(("whole_block", s, base, total, 0, len(dl), pay))
    # one byte, in the middle of packet 2 (the server starts the stream at packet 2)
    out.append(("one_byte", s[whole[2]["stream_off"]:], base + 2 * 65536 + 7, 1, 0, 1,
                pay[2 * 65536 + 7:2 * 65536 + 8]))
    # more than the block holds: the empty last packet arrives while bytes are wanted
    out.append(("past_block_end", s, base + 5, total, ERR_BAD_LASTPACKET, len(dl) + 1, pay[5:]))
    # the read starts after the first packet's data: UNEXPECTED_READ_OFFSET
    out.append(("read_offset", s, base + 65536 + 3, 100, ERR_UNEXPECTED_READ_OFFSET, 1, b""))
    # a data packet flagged lastPacketInBlock with the read unfinished: its bytes, then the error
    s2, _ = build_stream(oracle.crc32c, 2, cs, CSUM_CRC32C, [65536] * 4, seed=2, last_empty=False, last_flag=1)
    w2 = oracle.verify_packets(s2)[1]
    p2 = _payload_of(s2, w2, 0) + _payload_of(s2, w2, 1)
    out.append(("last_flag_short", s2, 100, 3 * 65536, ERR_BAD_LASTPACKET, 2, p2[100:]))
    # bad CRCs in packet 2 end the read (src/datanode.c:1476-1479, 2470-2475):
    # the bytes before it; the window's own end in packet 4 is never reached
    s3, _ = build_stream(oracle.crc32c, 2, cs, CSUM_CRC32C, [65536] * 6, seed=3, corrupt=[(2, 5)])
    w3 = oracle.verify_packets(s3)[1]
    p3 = b"".join(_payload_of(s3, w3, k) for k in range(2))
    out.append(("bad_crc_mid", s3, 40, 4 * 65536 + 9, BAD, 3, p3[40:]))
    # bad CRCs in the packet the read starts in: nothing delivered
    out.append(("bad_crc_first", s3[w3[2]["stream_off"]:], 2 * 65536 + 5, 1000, BAD, 1, b""))
    # framing errors end the read after the packets before them (src/datanode.c:2439-2456):
    # an empty packet NOT flagged last after packet 2 -- PACKET_SIZE, its header consumed
    # (:2450-2455) -- and packet 2 framed with a plen 4 short -- CRC_LEN, not consumed
    s4, _ = build_stream(oracle.crc32c, 2, cs, CSUM_CRC32C, [65536] * 5, seed=4, last_empty=False)
    w4 = oracle.verify_packets(s4)[1]
    cut = w4[3]["stream_off"]
    empty = frame_v2(header_v2(3 * 65536, 3, False, 0), b"", b"")
    p4 = b"".join(_payload_of(s4, w4, k) for k in range(3))
    out.append(("empty_not_last", s4[:cut] + empty + s4[cut:], 5, 4 * 65536, ERR_PACKET_SIZE, 4, p4[5:]))
    a2 = w4[2]["stream_off"]
    bad2 = struct.pack(">i", struct.unpack(">i", s4[a2:a2 + 4])[0] - 4) + s4[a2 + 4:]
    out.append(("crc_len_mid", s4[:a2] + bad2, 5, 4 * 65536, ERR_CRC_LEN, 3, p4[5:2 * 65536]))
    return out


def _read_consumed(pk):
    """Where a read that ended with record pk stands in the stream: a packet
    whose framing, CRCs or read offset raised the error is not consumed
    (src/datanode.c:2445-2446, 2472-2475, 2483-2486), except the empty packet
    not flagged last, whose header is (PACKET_SIZE, :2450-2455); any other
    packet is consumed whole."""
    if pk["error"] == ERR_PACKET_SIZE and pk["data_len"] == 0 and pk["crc_len"] == 0:
        return pk["stream_off"] + pk["header_len"]
    if pk["error"] and pk["error"] != ERR_BAD_LASTPACKET:
        return pk["stream_off"]
    return pk["stream_off"] + pk["header_len"] + pk["crc_len"] + pk["data_len"]


def test_oracle_read_windows_constructed(oracle):
    for name, s, co, rl, rc, npk, data in _read_cases(oracle):
        got = oracle.read_packets(s, co, rl)
        assert (got[0], len(got[1])) == (rc, npk), name
        assert got[3] == data, name
        assert got[2] == _read_consumed(got[1][-1]), name
        assert all(q["error"] == 0 for q in got[1][:-1]), name  # the read ends at its first error


def test_oracle_read_capacity_resumes(oracle):
    """The oracle's read into a destination smaller than the read (AGAIN,
    src/datanode.c:2547-2549), resumed call by call, gives the single read's
    records, consumed bytes, delivered bytes and final status -- for every
    constructed case and destination sizes that end inside packets, exactly
    on a packet's end, and on one byte."""
    for name, s, co, rl, rc, npk, data in _read_cases(oracle):
        want = oracle.read_packets(s, co, rl)
        for piece in (1, 4096, 65536, 65536 + 3, 100003):
            if piece == 1 and rl > 70000:
                continue
            at, tot, recs, calls = 0, 0, [], 0
            out = b""
            while True:
                r, pk, used, got = oracle.read_packets(s[at:], co + tot, rl - tot, cap=min(piece, rl - tot))
                calls += 1
                for q in pk:
                    q["stream_off"] += at
                recs += pk
                at += used
                tot += len(got)
                out += got
                if r != AGAIN:
                    break
                assert len(got) == min(piece, rl - tot + len(got)), (name, piece)
            assert (r, recs, at) == want[:3], (name, piece)
            assert out == want[3] == data, (name, piece)


AGAIN = 1000


ERR_UNEXPECTED_READ_OFFSET, ERR_BAD_LASTPACKET = 28, 32
ERR_PACKET_SIZE, ERR_CRC_LEN = 25, 26


def _dev_read(engine, s, shift, co, rl, proto=2, cs=512, ctype=CSUM_CRC32C, cap=None, mp=None):
    keep, p = _dev(engine, s, shift)
    cap = rl if cap is None else cap
    dst = engine.DeviceBuffer(cap + 64)
    dst.fill(0xA5)
    try:
        rc, pkts, used, delivered = engine.read_packets(p, len(s), dst.ptr, cap, proto, cs, ctype, max_pkts=mp,
                                                               client_offset=co, read_len=rl)
        guard = dst.download(64, offset=cap).tobytes()
        return rc, pkts, used, dst.download(delivered).tobytes(), guard
    finally:
        keep.free()
        dst.free()


@pytest.mark.gpu
def test_gpu_read_windows_constructed(engine, oracle):
    """Every constructed read window through the fused verify + copy-out
    equals the oracle's read loop: records, verdicts, consumed bytes and the
    delivered bytes themselves; nothing is written past the read."""
    for name, s, co, rl, rc, npk, data in _read_cases(oracle):
        want = oracle.read_packets(s, co, rl)
        for shift in (0, 3):
            got = _dev_read(engine, s, shift, co, rl)
            assert got[:3] == want[:3], (name, shift)
            assert got[3] == want[3] == data, (name, shift)
            assert got[4] == b"\xa5" * 64, (name, shift)


@pytest.mark.gpu
@pytest.mark.parametrize("proto,cs,ctype,sizes", [
    (2, 512, CSUM_CRC32C, "regular"),   # device framing passes (grid), tiled kernel copies
    (1, 512, CSUM_CRC32, "regular"),
    (2, 512, CSUM_CRC32C, "short"),     # <= 64 packets: the one-launch short-run kernel
    (2, 4096, CSUM_CRC32C, "mixed"),    # sizes change: grid passes + the host window walk
    (2, 100, CSUM_CRC32C, "partial"),   # chunk 100: every chunk on the generic kernel
    (2, 512, CSUM_CRC32C, "random"),
])
def test_gpu_read_windows_vs_oracle(engine, oracle, proto, cs, ctype, sizes):
    """Reads starting and ending at many offsets -- inside packets, on packet
    and chunk boundaries, at 16-B piece edges -- on every path of the device
    stream verifier (grid, short run, host walk) and at odd stream
    alignments: byte-exact against the oracle's read loop."""
    rng = np.random.default_rng(cs + proto + len(sizes))
    if sizes == "regular":
        dl = [65536] * 300 + [12345]
    elif sizes == "short":
        dl = [65536] * 40 + [3000]
    elif sizes == "mixed":
        dl = [int(x) for x in np.repeat(rng.choice([4096, 61440, 30000, 65536], 40), rng.integers(1, 8, 40))]
    elif sizes == "partial":
        dl = [40000] * 60
    else:
        dl = [int(x) for x in rng.integers(1, 70000, 120)]
    base = 7 * 65536
    corrupt = [(len(dl) // 2, 1)]
    s, _ = build_stream(oracle.crc32c, proto, cs, ctype, dl, seed=len(dl), corrupt=corrupt, offset0=base)
    total = sum(dl)
    cases = [(base, total), (base + 1, total - 1), (base + 15, 17), (base + 16, 32), (base + 65536 - 3, 10),
             (base + 511, 513), (base + total - 5, 5), (base + total - 5, 50)]
    for _ in range(6):
        a = int(rng.integers(0, total))
        cases.append((base + a, int(rng.integers(1, total - a + 1))))
    cases.append((base + total // 2, 1000))  # the stream below starts at packet 0: UNEXPECTED_READ_OFFSET
    whole = oracle.verify_packets(s, proto, cs, ctype)[1]
    starts = np.cumsum([0] + dl[:-1])
    for i, (co, rl) in enumerate(cases):
        # the server starts the stream at the packet holding client_offset
        k = int(np.searchsorted(starts, co - base, side="right")) - 1 if i + 1 < len(cases) else 0
        sub = s[whole[k]["stream_off"]:]
        want = oracle.read_packets(sub, co, rl, proto, cs, ctype)
        shift = i % 4
        got = _dev_read(engine, sub, shift, co, rl, proto, cs, ctype)
        assert got[:3] == want[:3], (co - base, rl, shift)
        assert got[3] == want[3], (co - base, rl, shift)
        assert got[4] == b"\xa5" * 64, (co - base, rl, shift)
    assert want[0] == ERR_UNEXPECTED_READ_OFFSET


@pytest.mark.gpu
def test_gpu_copy_out_mixed_sizes_never_past_cap(engine, oracle):
    """Whole-payload copy-out into a buffer one byte too small, on a stream
    whose packet sizes vary (the host window walk places the copies): the
    call fails, and the bytes just past the buffer are untouched (ADVICE r2:
    the walk used to place packets without checking the capacity)."""
    rng = np.random.default_rng(9)
    dl = [int(x) for x in np.repeat(rng.choice([4096, 61440, 30000, 65536], 30), rng.integers(1, 5, 30))]
    s, _ = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, dl, seed=9)
    keep, p = _dev(engine, s, 1)
    cap = sum(dl) - 1
    dst = engine.DeviceBuffer(cap + 4096)
    dst.fill(0xA5)
    with pytest.raises(engine.CRC32CError):
        engine.read_packets(p, len(s), dst.ptr, cap)
    assert dst.download(4096, offset=cap).tobytes() == b"\xa5" * 4096
    keep.free()
    dst.free()


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["v1_regular", "v2_seq_jump", "v1_break_group1", "v1_max_pkts", "v2_read_window",
                                  "v1_two_level", "v2_two_level_break"])
def test_gpu_device_stream_many_blocks(engine, oracle, case):
    """Device framing passes of 9 000 small packets (141 framing blocks in 3
    groups of 64) and of 24 000 (376 blocks in 6 groups), so a block's
    prefix comes from both levels of frame_build_kernel's scan (its group's
    block records and earlier groups' totals).  Regular v1 runs with bad chunks spread over the groups; v2
    with a seqno jump and a skewed offsetInBlock in later groups (records
    off the prediction, same wire size: exceptions, no break); a packet of
    another size in group 1 (the pass breaks there, the walk goes on);
    max_pkts inside group 1; a client read window starting and ending in
    later groups.  Records, verdicts, consumed bytes and copied bytes equal
    the oracle's."""
    n, cs = (24000 if "two_level" in case else 9000), 512
    proto = 2 if case.startswith("v2") else 1
    dl = [512] * n
    kw = {}
    if case == "v1_break_group1":
        dl[5000] = 700
    if case == "v2_two_level_break":
        dl[20000] = 700  # group 4 of the two-level scan
    if proto == 2:
        # header varints of one length over the whole run (offsetInBlock in
        # [2^21, 2^28), seqno in [2^14, 2^21)): every packet on one grid
        kw["offset0"] = 1 << 21
        kw["seqnos"] = [20000 + k for k in range(n)]
    if case == "v2_seq_jump":
        kw["seqnos"] = [20000 + k + (100 if k >= 6000 else 0) for k in range(n)]
        kw["offset_skew"] = {8500: 4096}
    corrupt = [(3, 0), (4100, 0), (6000, 0), (8999, 0)] + ([(15000, 0), (23999, 0)] if n > 9000 else [])
    s, bad = build_stream(oracle.crc32c, proto, cs, CSUM_CRC32C, dl, seed=11, corrupt=corrupt, last_empty=False, **kw)
    keep, p = _dev(engine, s, 0)
    try:
        if case == "v2_read_window":
            co, rl = (1 << 21) + 4600 * 512 + 77, 3000 * 512
            want = oracle.read_packets(s, co, rl, proto, cs, CSUM_CRC32C)
            dst = engine.DeviceBuffer(rl + 64)
            dst.fill(0xA5)
            got = engine.read_packets(p, len(s), dst.ptr, rl, proto, cs, CSUM_CRC32C, client_offset=co,
                                             read_len=rl)
            assert got[:3] == want[:3]
            assert dst.download(got[3]).tobytes() == want[3]
            assert dst.download(64, offset=rl).tobytes() == b"\xa5" * 64
            dst.free()
            return
        mp = 8000 if case == "v1_max_pkts" else None
        want = oracle.verify_packets(s, proto, cs, CSUM_CRC32C, max_pkts=mp)
        got = engine.verify_packets(None, proto, cs, CSUM_CRC32C, max_pkts=mp, dptr=p, nbytes=len(s))
        assert got == want
        if mp is None:
            assert {k: (q["first_bad"], q["bad_chunks"]) for k, q in enumerate(got[1]) if q["error"] == BAD} == \
                {k: (v[0], len(v)) for k, v in bad.items()}
    finally:
        keep.free()


# --- resumable reads and scatter lists (round 4) ------------------------------
def _resumed_read(engine, p, n, co, rl, piece, dst, proto, cs, ctype):
    """A client read through hdfs_crc32c_read_packets in calls whose buffer is
    `piece` bytes, each resuming where the previous stopped (AGAIN:
    stream + consumed, client_offset + delivered, read_len - delivered) --
    the reference's re-entry with remains_pkt > 0 (src/datanode.c:2356-2361,
    2547-2549).  -> (rc, records, consumed, bytes, calls)."""
    at, tot, recs, calls = 0, 0, [], 0
    while True:
        cap = min(piece, rl - tot)
        rc, pk, used, got = engine.read_packets(p + at, n - at, dst.ptr + tot, cap, proto, cs, ctype,
                                                client_offset=co + tot, read_len=rl - tot)
        calls += 1
        for q in pk:
            q["stream_off"] += at
        recs += pk
        at += used
        tot += got
        if rc != engine.AGAIN:
            return rc, recs, at, dst.download(tot).tobytes(), calls
        assert got == cap and calls < 10000


@pytest.mark.gpu
@pytest.mark.parametrize("proto,cs,ctype,sizes", [
    (2, 512, CSUM_CRC32C, "regular"),   # speculative launches / device framing passes
    (1, 512, CSUM_CRC32, "regular"),
    (2, 512, CSUM_CRC32C, "short"),     # the one-launch short-run kernel
    (2, 4096, CSUM_CRC32C, "mixed"),    # the host window walk
    (2, 100, CSUM_CRC32C, "partial"),   # generic chunks
])
def test_gpu_read_resumable_and_scatter(engine, oracle, proto, cs, ctype, sizes):
    """A client read into a destination smaller than the read: resumed call
    by call (AGAIN), and in one call over a scatter list of buffers (the
    reference's iovec array, src/datanode.c:2509-2537) -- the bytes, the
    records (each packet once, from the call that completes it), consumed
    and the final status equal the oracle's single read loop, and no byte
    lands past a buffer."""
    rng = np.random.default_rng(cs + proto + len(sizes) + 17)
    if sizes == "regular":
        dl = [65536] * 150 + [12345]
    elif sizes == "short":
        dl = [65536] * 40 + [3000]
    elif sizes == "mixed":
        dl = [int(x) for x in np.repeat(rng.choice([4096, 61440, 30000, 65536], 30), rng.integers(1, 6, 30))]
    else:
        dl = [40000] * 60
    base = 3 * 65536
    s, _ = build_stream(oracle.crc32c, proto, cs, ctype, dl, seed=len(dl) + 5, corrupt=[(len(dl) - 5, 1)],
                        offset0=base)
    total = sum(dl)
    whole = oracle.verify_packets(s, proto, cs, ctype)[1]
    starts = np.cumsum([0] + dl[:-1])
    cases = [(base + 1000, total // 3), (base + 7, total), (base + total // 2 + 11, total // 4)]
    for ci, (co, rl) in enumerate(cases):
        k = int(np.searchsorted(starts, co - base, side="right")) - 1
        sub = s[whole[k]["stream_off"]:]
        want = oracle.read_packets(sub, co, rl, proto, cs, ctype)
        keep, p = _dev(engine, sub, ci % 3)
        dst = engine.DeviceBuffer(rl + 4096)
        # <= 64 KiB: the short-run kernel over the stream's first 4 MiB
        # (grid_walk's small_win); larger: the speculative / framing passes
        for piece in (4099, 65536, 65536 + 3, 100003, 1 << 20):
            dst.fill(0xA5)
            rc, recs, used, data, calls = _resumed_read(engine, p, len(sub), co, rl, piece, dst, proto, cs, ctype)
            assert (rc, recs, used) == want[:3], (co - base, rl, piece)
            assert data == want[3], (co - base, rl, piece)
            assert calls >= min(len(want[3]) // piece, 2) or rc != 0
        # one call over a scatter list: buffers of uneven sizes, a 16-B guard after each
        sizes_l = [int(x) for x in rng.integers(20000, 300000, 64)]
        iov, off = [], 0
        while off < rl + 4096 and len(iov) < 64:
            n = min(sizes_l[len(iov)], rl + 4096 - off)
            iov.append((off, n))
            off += n + 16
        big = engine.DeviceBuffer(off + 64)
        big.fill(0xA5)
        rc, recs, used, got = engine.read_packets(p, len(sub), None, 0, proto, cs, ctype, client_offset=co, read_len=rl,
                                                  iov=[(big.ptr + a, n) for a, n in iov])
        assert (rc, recs, used) == want[:3], (co - base, rl, "iov")
        flat = big.download(off).tobytes()
        data, left = b"", got
        for a, n in iov:
            take = min(n, left)
            data += flat[a:a + take]
            left -= take
            assert flat[a + n:a + n + 16] == b"\xa5" * 16  # guards untouched
        assert data == want[3]
        big.free()
        dst.free()
        keep.free()
