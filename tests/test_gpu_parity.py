"""GPU parity tests: the HIP path (through the C ABI) against the committed
golden fixtures (made by the reference, oracle/gen_golden.py) and against the
CPU oracle on the same seeded inputs.  Bit-exact everywhere (integer work)."""
import numpy as np
import pytest

from oracle import splitmix64_np

pytestmark = pytest.mark.gpu

SWEEP_DATA = splitmix64_np(1024 + 8, seed=7).view(np.uint8)


def _dev(engine, host):
    buf = engine.DeviceBuffer(max(1, host.nbytes))
    buf.upload(host)
    return buf


def _chunk_plan(engine, dbuf, nbytes, cs, mode, crcs_dev, flags=0, bitmap=None, crc_init=0, offset=0):
    seg = engine.Segment(data=dbuf.ptr + offset, len=nbytes, chunk_size=cs, flags=flags,
                         crc_init=crc_init, crcs=crcs_dev.ptr, bitmap=bitmap.ptr if bitmap else None)
    return engine.Plan(mode, [seg])


# --- drop-in symbols (src/crc32c.h) against tests/t_unit.c KATs -------------
def test_kats_dropin(engine, golden):
    for k in golden["kats"]:
        b = bytes.fromhex(k["hex"])
        for entry in ("_hdfs_crc32c", "_hdfs_sse42_crc32c", "_hdfs_armv8_crc32c", "_hdfs_sw_crc32c"):
            assert engine.crc32c(0, b, entry) == k["crc"], (entry, k["len"], k["source"])


def test_chaining_dropin(engine, oracle):
    rng = np.random.default_rng(3)
    a = rng.integers(0, 256, 3001, dtype=np.uint8)
    b = rng.integers(0, 256, 777, dtype=np.uint8)
    whole = oracle.crc32c(0, np.concatenate([a, b]))
    assert engine.crc32c(engine.crc32c(0, a), b) == whole
    assert engine.crc32c(0x12345678, b"") == 0x12345678  # len 0 returns crc


def test_edge_sweep_host_and_device(engine, golden):
    sweep = golden["sweep"]
    dbuf = _dev(engine, SWEEP_DATA)
    lens = list(range(0, 600)) + list(range(600, 4097, 37)) + [4095, 4096]
    for off in range(8):
        for n in lens:
            cin = (0x9E3779B9 * (n + 1) + off) & 0xFFFFFFFF
            if off in (0, 3):  # host-memory drop-in path
                assert engine.crc32c(0, SWEEP_DATA[off:off + n]) == sweep[0, off, n], (off, n)
            # device pointer at every alignment, chained crc_in
            assert engine.stream_crc_dev(cin, dbuf.ptr + off, n) == sweep[1, off, n], (off, n)


# --- batch compute against golden per-chunk arrays --------------------------
@pytest.mark.parametrize("cs", [512, 1024, 2048, 4096])
@pytest.mark.parametrize("kind", ["full", "ragged"])
def test_chunk_crcs_golden(engine, golden, cs, kind):
    host = splitmix64_np(1 << 17, seed=0).view(np.uint8)
    n = host.nbytes if kind == "full" else host.nbytes - 123
    want = golden["chunks"][f"{kind}_{cs}"]
    dbuf = _dev(engine, host[:n])
    out = engine.DeviceBuffer(want.nbytes)
    p = _chunk_plan(engine, dbuf, n, cs, engine.MODE_COMPUTE, out)
    p.execute()
    got = out.download(dtype=np.uint32)
    np.testing.assert_array_equal(got, want)
    # wire order
    pb = _chunk_plan(engine, dbuf, n, cs, engine.MODE_COMPUTE, out, flags=engine.SEG_BE)
    pb.execute()
    np.testing.assert_array_equal(out.download(dtype=">u4").astype(np.uint32), want)


@pytest.mark.parametrize("nchunks", [1, 7, 8, 9, 15, 16, 17, 63, 64, 65, 1000, 4097])
@pytest.mark.parametrize("cs", [512, 1536, 4096])
def test_tiled_shapes_vs_oracle(engine, oracle, nchunks, cs):
    rng = np.random.default_rng(nchunks * 31 + cs)
    host = rng.integers(0, 256, nchunks * cs, dtype=np.uint8)
    dbuf = _dev(engine, host)
    out = engine.DeviceBuffer(nchunks * 4)
    for cin in (0, 0xDEADBEEF):
        p = _chunk_plan(engine, dbuf, host.nbytes, cs, engine.MODE_COMPUTE, out, crc_init=cin)
        assert p.stats()["generic_bytes"] == 0
        p.execute()
        got = out.download(dtype=np.uint32)
        if cin == 0:
            want = oracle.chunk_crcs(host, cs)
        else:
            want = np.array([oracle.crc32c(cin, host[i * cs:(i + 1) * cs]) for i in range(nchunks)], np.uint32)
        np.testing.assert_array_equal(got, want)


def test_generic_path_unaligned_and_odd_sizes(engine, oracle):
    rng = np.random.default_rng(11)
    host = rng.integers(0, 256, 300000, dtype=np.uint8)
    dbuf = _dev(engine, host)
    for off, n, cs in [(1, 100000, 512), (3, 65536, 512), (8, 70001, 4096), (0, 99999, 100),
                       (0, 5000, 1), (5, 12345, 777), (0, 1, 512), (13, 512, 512)]:
        nch = (n + cs - 1) // cs
        out = engine.DeviceBuffer(nch * 4)
        p = _chunk_plan(engine, dbuf, n, cs, engine.MODE_COMPUTE, out, offset=off)
        p.execute()
        want = oracle.chunk_crcs(host[off:off + n], cs)
        np.testing.assert_array_equal(out.download(dtype=np.uint32), want, err_msg=f"{off},{n},{cs}")


def _mixed_segments(engine, rng, nseg=24):
    """A C5-like table: chunk sizes 512<<(i%4), ragged tails, one unaligned
    and one empty segment, all in one plan."""
    specs = []
    for i in range(nseg):
        cs = 512 << (i % 4)
        n = int(rng.integers(0, 40)) * cs + (int(rng.integers(1, cs)) if i % 5 == 2 else 0)
        specs.append((cs, n, 1 if i == 7 else 0))
    specs.append((512, 0, 0))
    total = sum(n + 256 for _, n, _ in specs)
    host = rng.integers(0, 256, total, dtype=np.uint8)
    dbuf = _dev(engine, host)
    offs, o = [], 0
    for cs, n, mis in specs:
        offs.append(o + mis)
        o += n + 256 - (n % 256)
        o = (o + 255) // 256 * 256
    return specs, offs, host, dbuf


def test_mixed_segment_plan_compute_and_verify(engine, oracle):
    rng = np.random.default_rng(21)
    specs, offs, host, dbuf = _mixed_segments(engine, rng)
    nch = [(n + cs - 1) // cs for cs, n, _ in specs]
    crc_bufs = [engine.DeviceBuffer(max(4, c * 4)) for c in nch]
    bm_bufs = [engine.DeviceBuffer(max(4, (c + 7) // 8)) for c in nch]
    segs = [engine.Segment(data=dbuf.ptr + off, len=n, chunk_size=cs, flags=engine.SEG_BE, crc_init=0,
                           crcs=cb.ptr, bitmap=None)
            for (cs, n, _), off, cb in zip(specs, offs, crc_bufs)]
    p = engine.Plan(engine.MODE_COMPUTE, segs)
    p.execute()
    wants = []
    for (cs, n, _), off, cb, c in zip(specs, offs, crc_bufs, nch):
        want = oracle.chunk_crcs(host[off:off + n], cs)
        wants.append(want)
        np.testing.assert_array_equal(cb.download(c * 4, dtype=">u4").astype(np.uint32), want)
    # verify the same table after corrupting chosen chunks
    bad = {}
    for si, ((cs, n, _), off, c) in enumerate(zip(specs, offs, nch)):
        if c and si % 3 == 0:
            picks = sorted(set(int(x) for x in rng.integers(0, c, 3)))
            bad[si] = picks
            for ci in picks:
                clen = min(cs, n - ci * cs)
                bit = int(rng.integers(0, 8 * clen))
                host[off + ci * cs + bit // 8] ^= np.uint8(1 << (bit % 8))
    dbuf.upload(host)
    vsegs = [engine.Segment(data=s.data, len=s.len, chunk_size=s.chunk_size, flags=engine.SEG_BE,
                            crc_init=0, crcs=s.crcs, bitmap=bb.ptr) for s, bb in zip(segs, bm_bufs)]
    vp = engine.Plan(engine.MODE_VERIFY, vsegs)
    vp.execute()
    first_bad, mism = vp.results()
    assert mism == sum(len(v) for v in bad.values())
    for si, c in enumerate(nch):
        exp_bits = np.zeros((c + 7) // 8 * 8, dtype=np.uint8)
        for ci in bad.get(si, []):
            exp_bits[ci] = 1
        got = np.unpackbits(bm_bufs[si].download((c + 7) // 8), bitorder="little")
        np.testing.assert_array_equal(got[: exp_bits.size], exp_bits, err_msg=str(si))
        assert first_bad[si] == (bad[si][0] if si in bad else 0xFFFFFFFF)


# --- datanode mirrors on host memory ----------------------------------------
def test_verify_crcdata_golden(engine, golden):
    for case in golden["verify"]:
        region = bytes.fromhex(case["region_hex"])
        cs, dlen = case["chunk_size"], case["dlen"]
        nch = (dlen + cs - 1) // cs
        err, fb = engine.verify_crcdata(region, cs, nch * 4, dlen)
        assert fb == case["first_bad"], case["mismatch"]
        assert err == (engine.ERR_BAD_CHECKSUM if case["mismatch"] else 0)
        if nch:
            assert engine.verify_crcdata(region, cs, nch * 4 + 4, dlen)[0] == engine.ERR_CRC_LEN
    # CSUM_NULL is not a checksum the reference verifies (src/datanode.c:2938 ASSERT)
    with pytest.raises(engine.CRC32CError):
        engine.verify_crcdata(b"\0" * 8, 512, 4, 512, ctype=engine.CSUM_NULL)


def test_compose_crcs_vs_oracle(engine, oracle):
    rng = np.random.default_rng(8)
    data = rng.integers(0, 256, 65536 + 300, dtype=np.uint8).tobytes()
    for cuts in ([0, 65536 + 300], [0, 1, 100, 513, 40000, 65836], [0, 65536]):
        frags = [data[a:b] for a, b in zip(cuts[:-1], cuts[1:])]
        assert engine.compose_crcs(frags, 512) == oracle.compose_crcs(frags, 512)
        assert engine.compose_crcs(frags, 512, ctype=engine.CSUM_CRC32) == \
            oracle.compose_crcs(frags, 512, ctype=engine.CSUM_CRC32)


# --- large inputs: stream CRC and the pinned full-block digests ---------------
def test_stream_crc_large(engine, oracle):
    host = splitmix64_np(8 << 20, seed=99).view(np.uint8)  # 64 MiB
    dbuf = _dev(engine, host)
    for n in (host.nbytes, host.nbytes - 4095, 12345679):
        assert engine.stream_crc_dev(0, dbuf.ptr, n) == oracle.crc32c(0, host[:n], "hw")
    assert engine.crc32c(7, host[:5000001]) == oracle.crc32c(7, host[:5000001], "hw")


def test_block_digests_on_device(engine, oracle, golden):
    """128 MiB blocks generated on device by formula; digests pinned by the
    reference."""
    hc = engine
    blk_bytes = 128 << 20
    dbuf = engine.DeviceBuffer(blk_bytes)
    for blk in (0, 1):
        hc.fill_splitmix64(dbuf.ptr, blk_bytes // 8, 0, blk << 24)
        for cs in (512, 1024, 2048, 4096):
            out = engine.DeviceBuffer(blk_bytes // cs * 4)
            p = _chunk_plan(engine, dbuf, blk_bytes, cs, engine.MODE_COMPUTE, out)
            p.execute()
            arr = out.download(dtype=np.uint32)
            want = golden["blocks"][f"block{blk}_{cs}"]
            assert int(arr[0]) == want["crc0"], (blk, cs)
            assert oracle.crc32c(0, arr.view(np.uint8), "hw") == want["digest"], (blk, cs)
            # the same digest on device (stream CRC of the device CRC array)
            assert engine.stream_crc_dev(0, out.ptr, out.nbytes) == want["digest"]


def test_all_block_digests_on_device(engine):
    """A spread of the bench's 8192 x 128 MiB blocks (C3 / C5 data of every
    rank of an 8-GPU run) generated on device, per-chunk CRCs at all four
    chunk sizes in ONE mixed compute plan, then each CRC array's digest in one
    launch over the arrays -- the bench's own full-scale parity check --
    against the reference-generated tests/golden/block_digests_all.npz."""
    import os
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "block_digests_all.npz"))
    blocks = [0, 1, 2, 3, 511, 1022, 1023, 1024, 2049, 4095, 6146, 8191]
    blk = 128 << 20
    data = engine.DeviceBuffer(len(blocks) * blk)
    for i, g in enumerate(blocks):
        engine.fill_splitmix64(data.ptr + i * blk, blk // 8, 0, g << 24)
    for shift in range(4):  # every block at every chunk size across the four plans
        sizes = [512 << ((i + shift) % 4) for i in range(len(blocks))]
        offs = np.concatenate([[0], np.cumsum([blk // c for c in sizes])])
        crcs = engine.DeviceBuffer(int(offs[-1]) * 4)
        segs = [engine.Segment(data=data.ptr + i * blk, len=blk, chunk_size=c, flags=engine.SEG_BE, crc_init=0,
                               crcs=crcs.ptr + int(offs[i]) * 4) for i, c in enumerate(sizes)]
        engine.Plan(engine.MODE_COMPUTE, segs).execute()
        digs = engine.DeviceBuffer(4 * len(blocks))
        dsegs = [engine.Segment(data=crcs.ptr + int(offs[i]) * 4, len=blk // c * 4, chunk_size=blk // c * 4,
                                flags=0, crc_init=0, crcs=digs.ptr + 4 * i) for i, c in enumerate(sizes)]
        engine.Plan(engine.MODE_COMPUTE, dsegs).execute()
        got = digs.download(dtype=np.uint32)
        for i, (g, c) in enumerate(zip(blocks, sizes)):
            j = (512, 1024, 2048, 4096).index(c)
            assert got[i] == z["be"][g, j], (g, c)
            first = crcs.download(4, offset=int(offs[i]) * 4, dtype=">u4")[0]
            assert first == z["crc0"][g, j], (g, c)


def test_verify_roundtrip_corruption_pattern(engine):
    """Size-independent property used at full bench scale: compute -> corrupt
    (i % 65537 == 0) -> verify finds exactly the corrupted chunks."""
    hc = engine
    nblk, blk = 4, 128 << 20
    cs = 512
    dbuf = engine.DeviceBuffer(nblk * blk)
    hc.fill_splitmix64(dbuf.ptr, nblk * blk // 8, 0, 0)
    crcs = engine.DeviceBuffer(nblk * blk // cs * 4)
    bms = engine.DeviceBuffer(nblk * blk // cs // 8)
    per = blk // cs
    segs = [engine.Segment(data=dbuf.ptr + b * blk, len=blk, chunk_size=cs, flags=engine.SEG_BE,
                           crc_init=0, crcs=crcs.ptr + b * per * 4, bitmap=bms.ptr + b * per // 8)
            for b in range(nblk)]
    engine.Plan(engine.MODE_COMPUTE, segs).execute()
    for b in range(nblk):
        hc.corrupt(dbuf.ptr + b * blk, blk, cs, b * per, 65537, 7919)
    vp = engine.Plan(engine.MODE_VERIFY, segs)
    vp.execute()
    first_bad, mism = vp.results()
    expected = [i for i in range(nblk * per) if i % 65537 == 0]
    assert mism == len(expected)
    bits = np.unpackbits(bms.download(), bitorder="little")
    assert list(np.nonzero(bits)[0]) == expected
    for b in range(nblk):
        mine = [i - b * per for i in expected if b * per <= i < (b + 1) * per]
        assert first_bad[b] == (mine[0] if mine else 0xFFFFFFFF)


# --- host-resident pipeline (H2D / kernel / D2H overlapped) --------------------
@pytest.mark.parametrize("cs,n,piece", [(512, 3 << 20, 1 << 20), (512, (3 << 20) + 777, 1 << 20),
                                        (4096, 5 << 20, 0), (1000, 2_000_003, 64000), (512, 100, 0)])
def test_host_pipeline_vs_oracle(engine, oracle, cs, n, piece):
    rng = np.random.default_rng(n % 1000 + cs)
    host = rng.integers(0, 256, n, dtype=np.uint8)
    want = oracle.chunk_crcs(host, cs)
    got = engine.compute_host(host, cs, piece_bytes=piece)
    np.testing.assert_array_equal(got, want)
    be = engine.compute_host(host, cs, flags=engine.SEG_BE, piece_bytes=piece)
    np.testing.assert_array_equal(be.byteswap(), want)
    # verify: clean, then with corruptions in several pieces
    fb, m, bm = engine.verify_host(host, cs, be, flags=engine.SEG_BE, piece_bytes=piece)
    assert fb is None and m == 0 and not bm.any()
    nch = want.size
    bad = sorted(set(int(x) for x in rng.integers(0, nch, 4)))
    for ci in bad:
        host[ci * cs + int(rng.integers(0, min(cs, n - ci * cs)))] ^= 0x20
    fb, m, bm = engine.verify_host(host, cs, be, flags=engine.SEG_BE, piece_bytes=piece)
    assert fb == bad[0] and m == len(bad)
    assert list(np.nonzero(np.unpackbits(bm, bitorder="little"))[0]) == bad


def test_host_pipeline_pinned(engine, oracle):
    n, cs = 24 << 20, 512
    pin = engine.PinnedBuffer(n)
    pin.array[:] = np.random.default_rng(2).integers(0, 256, n, dtype=np.uint8)
    want = oracle.chunk_crcs(pin.array, cs)
    np.testing.assert_array_equal(engine.compute_host(pin.array, cs, piece_bytes=4 << 20), want)
    pin.free()


def test_dropin_consumer_runs(engine, tmp_path):
    """A C consumer compiled against include/crc32c.h and linked with the
    engine passes the reference's KATs through all three drop-in symbols."""
    import subprocess

    from hadoofus_amd import build
    from test_abi import build_consumer
    exe, txt = build_consumer(tmp_path, build.LIB)
    p = subprocess.run([str(exe), str(txt)], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "0 failures" in p.stdout


def test_segment_beyond_4gib(engine, oracle):
    """One 5 GiB segment (10.5 M chunks): 64-bit byte offsets everywhere.
    Sampled chunk CRCs against the oracle (data regenerated by formula),
    the C3 corruption pattern across the 4 GiB boundary, and the composite
    of the whole segment against its data-reading stream CRC."""
    n, cs = 5 << 30, 512
    dbuf = engine.DeviceBuffer(n)
    engine.fill_splitmix64(dbuf.ptr, n // 8, 0, 0)
    nch = n // cs
    crcs = engine.DeviceBuffer(nch * 4)
    bm = engine.DeviceBuffer(nch // 8)
    seg = engine.Segment(data=dbuf.ptr, len=n, chunk_size=cs, flags=engine.SEG_BE, crc_init=0,
                         crcs=crcs.ptr, bitmap=bm.ptr)
    engine.Plan(engine.MODE_COMPUTE, [seg]).execute()
    got = crcs.download(dtype=">u4").astype(np.uint32)
    rng = np.random.default_rng(4)
    picks = sorted(set([0, nch - 1, (4 << 30) // cs - 1, (4 << 30) // cs] +
                       [int(x) for x in rng.integers(0, nch, 200)]))
    for i in picks:
        data = splitmix64_np(cs // 8, seed=0, g0=i * (cs // 8)).view(np.uint8)
        assert got[i] == oracle.crc32c(0, data, "hw"), i
    assert engine.composite_crcs([seg])[0] == engine.stream_crc_dev(0, dbuf.ptr, n)
    engine.corrupt(dbuf.ptr, n, cs, 0, 65537, 7919)
    vp = engine.Plan(engine.MODE_VERIFY, [seg])
    vp.execute()
    fb, m = vp.results()
    expected = list(range(0, nch, 65537))
    assert m == len(expected) and fb[0] == 0
    bits = np.unpackbits(bm.download(), bitorder="little")
    assert list(np.nonzero(bits)[0]) == expected


@pytest.mark.parametrize("n", [1, 3, 63, 64, 65, 255, 256, 257, 4095, 4096, 4097, 65535, 65536, 65537, 200001])
def test_dropin_small_launch_sizes(engine, oracle, n):
    """Host buffers up to 64 KiB take the one-launch small kernel (pinned
    stage read over PCIe, zeros-operator combine of 64-B pieces); larger ones
    the staged 4 KiB-piece path.  Both ends of the switch, every piece-count
    remainder, chained from a non-zero CRC, all three drop-in symbols."""
    data = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8)
    for crc0 in (0, 0x9E3779B9):
        want = oracle.crc32c(crc0, data)
        for entry in ("_hdfs_crc32c", "_hdfs_sse42_crc32c", "_hdfs_sw_crc32c"):
            assert engine.crc32c(crc0, data, entry) == want, (entry, crc0)
    # and the CRC32 (zlib) table set through the same kernel
    import zlib
    assert engine.stream_ex(engine.CSUM_CRC32, 0, data) == zlib.crc32(data.tobytes())


@pytest.mark.parametrize("cs", [4, 64, 100, 512, 777, 4096, 65536])
@pytest.mark.parametrize("dlen", [1, 511, 512, 513, 8192, 65535, 65536, 65537])
def test_packet_mirrors_small_and_large(engine, oracle, cs, dlen):
    """_verify_crcdata / the write loop on one packet, through both engine
    paths: the one-launch small kernel (dlen <= 64 KiB, <= 2048 chunks,
    chunk % 4 == 0) and the staged plan path (everything else: cs 4 at 64 KiB
    is 16384 chunks, cs 777, dlen > 64 KiB).  Every chunk CRC, then the
    first-bad answer for a corrupted data byte and for a corrupted CRC word."""
    rng = np.random.default_rng(cs * 100003 + dlen)
    data = rng.integers(0, 256, dlen, dtype=np.uint8)
    nch = (dlen + cs - 1) // cs
    for ctype in (engine.CSUM_CRC32C, engine.CSUM_CRC32):
        want = oracle.compose_crcs([data.tobytes()], cs, ctype=ctype)
        got = engine.compose_crcs([data[: dlen // 3].tobytes(), data[dlen // 3:].tobytes()], cs, ctype=ctype)
        assert got == want
        region = bytearray(want + data.tobytes())
        assert engine.verify_crcdata(bytes(region), cs, nch * 4, dlen, ctype=ctype) == (0, -1)
        bad = int(rng.integers(0, nch))
        pos = nch * 4 + bad * cs + int(rng.integers(0, min(cs, dlen - bad * cs)))
        region[pos] ^= 0x40
        assert engine.verify_crcdata(bytes(region), cs, nch * 4, dlen, ctype=ctype) == (engine.ERR_BAD_CHECKSUM, bad)
        region[pos] ^= 0x40
        region[4 * (nch - 1)] ^= 1  # the last chunk's wire CRC
        assert engine.verify_crcdata(bytes(region), cs, nch * 4, dlen, ctype=ctype) == \
            (engine.ERR_BAD_CHECKSUM, nch - 1)


def test_dropin_concurrent_threads(engine, oracle):
    """The reference's CRC functions are reentrant and thread-safe after load
    (src/crc32c.h): 8 host threads calling the drop-in symbols
    and the per-packet mirror at once (ctypes drops the GIL) all get the
    oracle's answers."""
    import threading
    rng = np.random.default_rng(5)
    bufs = [rng.integers(0, 256, int(n), dtype=np.uint8) for n in rng.integers(1, 200000, 64)]
    want = [oracle.crc32c(0, b) for b in bufs]
    errors = []

    def worker(t):
        try:
            for i in range(t, t + 160):
                k = i % len(bufs)
                got = engine.crc32c(0, bufs[k], ("_hdfs_crc32c", "_hdfs_sse42_crc32c", "_hdfs_sw_crc32c")[i % 3])
                if got != want[k]:
                    errors.append((t, k, got, want[k]))
                if i % 7 == 0:
                    be = oracle.compose_crcs([bufs[k].tobytes()], 512)
                    rc, fb = engine.verify_crcdata(be + bufs[k].tobytes(), 512, len(be), bufs[k].nbytes)
                    if (rc, fb) != (0, -1):
                        errors.append((t, k, "verify", rc, fb))
        except Exception as e:  # surfaced below
            errors.append((t, repr(e)))

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for th in ths:
        th.start()
    for th in ths:
        th.join(timeout=120)
    assert not any(th.is_alive() for th in ths)
    assert not errors, errors[:5]


def test_dropin_max_len(engine, oracle):
    """`unsigned len` at its maximum, 2^32 - 1 bytes (one call
    caps at 4 GiB - 1; src/crc32c.h:13), through the three drop-in symbols on
    device pointers (aligned, and odd with a chained non-zero crc) and on host
    memory, against the oracle's SSE4.2 restatement on the same splitmix64 data."""
    n = (1 << 32) - 1
    host = oracle.splitmix(1 << 29, seed=3).view(np.uint8)
    want0 = oracle.crc32c(0, host[:n], "hw")
    want1 = oracle.crc32c(0xDEADBEEF, host[1:], "hw")
    dbuf = engine.DeviceBuffer(1 << 32)
    engine.fill_splitmix64(dbuf.ptr, 1 << 29, 3, 0)
    lib = engine.load()
    for entry in ("_hdfs_crc32c", "_hdfs_sse42_crc32c", "_hdfs_sw_crc32c"):
        f = getattr(lib, entry)
        assert f(0, dbuf.ptr, n) == want0, entry
        assert f(0xDEADBEEF, dbuf.ptr + 1, n) == want1, entry
    assert engine.crc32c(0, host[:n]) == want0
    assert engine.crc32c(0xDEADBEEF, host[1:]) == want1


def test_verify_crcdata_packet_beyond_staging(engine, oracle):
    """A packet larger than the 64 MiB one-shot staging (the reference's
    framing admits up to 1 GiB, src/datanode.c:2433-2441) is verified through
    the pipelined host path with the reference's result, not refused
    (ADVICE r1): clean -> 0; one corrupted chunk -> BAD_CHECKSUM + its index."""
    cs = 512
    dlen = (80 << 20) + 300  # partial last chunk
    rng = np.random.default_rng(80)
    data = rng.integers(0, 256, dlen, dtype=np.uint8)
    crcs = oracle.chunk_crcs(data, cs).astype(">u4").view(np.uint8)
    region = np.concatenate([crcs, data])
    assert engine.verify_crcdata(region, cs, crcs.nbytes, dlen) == (0, -1)
    k = 150_001
    region[crcs.nbytes + k * cs + 9] ^= 0x40
    assert oracle.verify_crcdata(region, cs, crcs.nbytes, dlen) == (engine.ERR_BAD_CHECKSUM, k)
    assert engine.verify_crcdata(region, cs, crcs.nbytes, dlen) == (engine.ERR_BAD_CHECKSUM, k)


def test_bound_device_explicit(engine):
    """hdfs_crc32c_init(0) binds the engine; bound_device reports it with a
    PCI bus id (what bench.py gathers per rank)."""
    engine.init(0)
    dev, bus = engine.bound_device()
    assert dev == 0 and bus.count(":") == 2 and bus.endswith(".0"), bus


@pytest.mark.parametrize("cs,seg_chunks,nseg,tail,ctype,be", [
    (512, 32768, 40, 0, 2, True),         # 640 MiB: the global pool engaged
    (512, 8 * 8 * 5 - 3, 64, 1, 2, True),  # last main tile of each segment holds 5 chunks; one 64 KiB tail segment
    (4096, 8 * 8 * 3, 20, 0, 2, True),    # 8 rounds per tile: a run is 64 rounds of one wave
    (1024, 8 * 8 * 40, 7, 0, 2, True),
    (512, 8 * 8 * 64, 24, 0, 1, True),    # CRC32 (zlib polynomial) through the gather
    (512, 8 * 8 * 5 - 3, 40, 1, 2, False),  # little-endian CRC arrays through the gather
])
def test_compute_runs_schedule(engine, oracle, cs, seg_chunks, nseg, tail, ctype, be):
    """Compute plans over segments of whole 8-tile groups, on the product
    schedule (the LDS group gather: a group's 64 CRCs collected across the
    workgroup's waves and written with one store; groups holding a partial
    last tile store per tile).  src/datanode.c:2814-2860 computes the same
    chunk CRCs one at a time.  CRC arrays equal the oracle's, nothing outside
    them is written."""
    seg_len = seg_chunks * cs
    lens = [seg_len] * nseg + ([65536 + 100] if tail else [])
    total = sum(lens)
    host = oracle.splitmix((total + 7) // 8, seed=cs + nseg + 17 * ctype).view(np.uint8)[:total]
    flags = (engine.SEG_BE if be else 0) | (engine.SEG_CRC32 if ctype == 1 else 0)
    dbuf = engine.DeviceBuffer(total)
    dbuf.upload(host)
    nchs = [(n + cs - 1) // cs for n in lens]
    crcs = engine.DeviceBuffer(4 * (sum(nchs) + 64))
    crcs.fill(0xA5)
    segs, off, coff = [], 0, 0
    for n, c in zip(lens, nchs):
        segs.append(engine.Segment(data=dbuf.ptr + off, len=n, chunk_size=cs, flags=flags, crc_init=0,
                                   crcs=crcs.ptr + 4 * coff, bitmap=None))
        off += n
        coff += c
    p = engine.Plan(engine.MODE_COMPUTE, segs)
    p.execute()
    got = crcs.download(4 * (coff + 64), dtype=">u4" if be else "<u4").astype(np.uint32)
    off, coff = 0, 0
    for n, c in zip(lens, nchs):
        np.testing.assert_array_equal(got[coff:coff + c], oracle.chunk_crcs(host[off:off + n], cs, ctype=ctype))
        off += n
        coff += c
    assert (got[coff:] == 0xA5A5A5A5).all()
    p.destroy()
    dbuf.free()
    crcs.free()
