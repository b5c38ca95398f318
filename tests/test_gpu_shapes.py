"""Every tiled-kernel schedule and shape (tools/exp_ab.py's A/B variants)
against the oracle on a C5-like table (mixed bytesPerChecksum 512..4096, so
tiles span 1..8 rounds) large enough that schedule 3 and its global pool are
engaged (>= 32 rounds per wave per stream), with segments ending 0..4 chunks
short of a whole tile.  Compute output bit-exact vs the oracle; verify finds
exactly the corrupted chunks (bitmaps, first bad).

The non-product shapes exist only in the diagnostic build
(libhadoofus_crc32c_diag.so, tools/diaglib.py), loaded beside the release
library; the release library's own two shapes are covered through it too."""
import os
import sys

import numpy as np
import pytest

from oracle import CSUM_CRC32, CSUM_CRC32C, splitmix64_np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

pytestmark = pytest.mark.gpu

SEG = 16 << 20
NSEG = 64  # 1 GiB: >= 32 rounds per wave per stream at every shape, so schedule 3 + pool run
# (order, depth, streams, block, loads): the built shapes (crc32c_kernels.hip
# launch_tiles); loads 1 = nontemporal global loads, 2 = nontemporal buffer loads
SHAPES = [(3, 3, 1, 1024, 1), (3, 3, 1, 1024, 2), (3, 4, 1, 1024, 1), (3, 2, 2, 1024, 1), (3, 3, 2, 1024, 1),
          (3, 3, 2, 768, 1), (3, 2, 2, 512, 1), (3, 3, 2, 512, 1), (3, 2, 4, 512, 1), (3, 3, 1, 768, 1),
          (3, 3, 1, 512, 1), (2, 3, 1, 1024, 1), (1, 3, 1, 1024, 1), (0, 3, 1, 1024, 1), (1, 3, 1, 1024, 0)]


@pytest.fixture(scope="module")
def diag(engine):
    import diaglib
    d = diaglib.Diag()
    d.init()
    yield d
    d.reset()


@pytest.fixture(scope="module")
def table(engine, oracle):
    host = splitmix64_np(NSEG * SEG // 8, seed=5).view(np.uint8).copy()
    sizes = [512 << (i % 4) for i in range(NSEG)]
    # segments end 0..4 chunks short of 16 MiB: partial last tiles
    lens = [SEG - (i % 5) * cs for i, cs in enumerate(sizes)]
    want = [oracle.chunk_crcs(host[i * SEG:i * SEG + n], cs) for i, (cs, n) in enumerate(zip(sizes, lens))]
    dbuf = engine.DeviceBuffer(host.nbytes)
    dbuf.upload(host)
    return host, sizes, lens, want, dbuf


def _set(d, order, depth, streams, block, loads):
    d.set_tile_order(order)
    d.set_depth(depth)
    d.set_shape(streams, block)
    d.set_tuning(loads, None)


@pytest.mark.parametrize("order,depth,streams,block,loads", SHAPES)
def test_shape_compute_verify(engine, diag, table, order, depth, streams, block, loads):
    host, sizes, lens, want, dbuf = table
    nch = [n // cs for cs, n in zip(sizes, lens)]
    crcs = [engine.DeviceBuffer(n * 4) for n in nch]
    bms = [engine.DeviceBuffer((n + 7) // 8) for n in nch]
    segs = [engine.Segment(data=dbuf.ptr + i * SEG, len=lens[i], chunk_size=cs, flags=engine.SEG_BE, crc_init=0,
                           crcs=crcs[i].ptr, bitmap=bms[i].ptr) for i, cs in enumerate(sizes)]
    try:
        _set(diag, order, depth, streams, block, loads)
        diag.plan(engine.MODE_COMPUTE, segs).execute()
        for i, n in enumerate(nch):
            np.testing.assert_array_equal(crcs[i].download(n * 4, dtype=">u4").astype(np.uint32), want[i],
                                          err_msg=f"segment {i}")
        # corrupt chunk k*997 + i of every third segment by flipping its expected CRC
        bad = {}
        for i, n in enumerate(nch):
            if i % 3 == 0:
                picks = sorted({(k * 997 + i) % n for k in range(5)})
                bad[i] = picks
                arr = want[i].astype(">u4")
                for c in picks:
                    arr[c] ^= np.uint32(1 << (c % 32))
                crcs[i].upload(arr.view(np.uint8))
        vp = diag.plan(engine.MODE_VERIFY, segs)
        vp.execute()
        first_bad, mism = vp.results()
        assert mism == sum(len(v) for v in bad.values())
        for i, n in enumerate(nch):
            bits = np.unpackbits(bms[i].download((n + 7) // 8), bitorder="little")[:n]
            assert list(np.nonzero(bits)[0]) == bad.get(i, []), i
            assert first_bad[i] == (bad[i][0] if i in bad else 0xFFFFFFFF)
    finally:
        diag.reset()


def test_unaligned_segments_default_schedule(engine, oracle):
    """Segments starting at every byte alignment run on the tiled kernel
    (unaligned buffer loads; schedule 3 + pool engaged at this size) and stay
    bit-exact; partial last chunks go to the generic kernel."""
    nseg, seg = 48, 16 << 20
    host = splitmix64_np((nseg * seg + 64) // 8, seed=11).view(np.uint8).copy()
    dbuf = engine.DeviceBuffer(host.nbytes)
    dbuf.upload(host)
    offs = [i * seg + (i % 16) for i in range(nseg)]
    lens = [seg - 16 - (i % 3) * 100 for i in range(nseg)]  # some partial last chunks
    cs = 512
    want = [oracle.chunk_crcs(host[o:o + n], cs) for o, n in zip(offs, lens)]
    crcs = [engine.DeviceBuffer(w.nbytes) for w in want]
    bms = [engine.DeviceBuffer((w.size + 7) // 8) for w in want]
    segs = [engine.Segment(data=dbuf.ptr + o, len=n, chunk_size=cs, flags=engine.SEG_BE, crc_init=0,
                           crcs=c.ptr, bitmap=b.ptr) for o, n, c, b in zip(offs, lens, crcs, bms)]
    engine.Plan(engine.MODE_COMPUTE, segs).execute()
    for i, w in enumerate(want):
        np.testing.assert_array_equal(crcs[i].download(dtype=">u4").astype(np.uint32), w, err_msg=str(i))
    # flip one expected CRC in every 5th segment; verify finds exactly those
    bad = {}
    for i in range(0, nseg, 5):
        k = (i * 7919) % want[i].size
        arr = want[i].astype(">u4")
        arr[k] ^= np.uint32(0x100)
        crcs[i].upload(arr.view(np.uint8))
        bad[i] = k
    vp = engine.Plan(engine.MODE_VERIFY, segs)
    vp.execute()
    first_bad, mism = vp.results()
    assert mism == len(bad)
    for i in range(nseg):
        assert first_bad[i] == bad.get(i, 0xFFFFFFFF), i


@pytest.mark.parametrize("shift", [1, 2, 3])
@pytest.mark.parametrize("cs,nch", [(512, 8 * 40), (1024, 64), (4096, 8 * 9 + 3), (512, 2_000_000 // 512)])
def test_unaligned_realign_small_and_large(engine, oracle, shift, cs, nch):
    """Byte-unaligned segments take the realigning kernel (aligned loads + one
    dword, v_alignbyte): small launches (schedule 2, global loads) and large
    ones (schedule 3, buffer loads); the data ends exactly at the end of its
    allocation, so the realigning loads must stay inside the data's dwords.
    Compute bit-exact vs the oracle, verify finds exactly the flipped CRCs."""
    n = cs * nch
    rng = np.random.default_rng(shift * 7 + cs)
    host = rng.integers(0, 256, n, dtype=np.uint8)
    buf = engine.DeviceBuffer(n + shift)
    buf.upload(host, offset=shift)  # data = [ptr + shift, ptr + shift + n) == the buffer's end
    want = oracle.chunk_crcs(host, cs)
    crcs = engine.DeviceBuffer(want.nbytes)
    bm = engine.DeviceBuffer((nch + 7) // 8)
    seg = engine.Segment(data=buf.ptr + shift, len=n, chunk_size=cs, flags=engine.SEG_BE, crc_init=0, crcs=crcs.ptr,
                         bitmap=bm.ptr)
    engine.Plan(engine.MODE_COMPUTE, [seg]).execute()
    np.testing.assert_array_equal(crcs.download(dtype=">u4").astype(np.uint32), want)
    picks = sorted({(k * 7919 + shift) % nch for k in range(6)})
    arr = want.astype(">u4")
    for c in picks:
        arr[c] ^= np.uint32(0x80)
    crcs.upload(arr.view(np.uint8))
    vp = engine.Plan(engine.MODE_VERIFY, [seg])
    vp.execute()
    first_bad, mism = vp.results()
    assert mism == len(picks) and first_bad[0] == picks[0]
    bits = np.unpackbits(bm.download(), bitorder="little")[:nch]
    assert list(np.nonzero(bits)[0]) == picks
    # the drop-in stream CRC over the same unaligned device bytes
    assert engine.stream_crc_dev(0x5A5A5A5A, buf.ptr + shift, n) == oracle.crc32c(0x5A5A5A5A, host)


@pytest.mark.parametrize("runs", [0, 1, 2, 3, 4])
def test_compute_store_schedules(engine, diag, oracle, table, runs):
    """Compute mode's store schedules (diagnostic knob set_runs): 0 schedule
    3 (one 32-B store per tile), 1 schedule 4 (a wave per 8-tile group), 2
    schedule 3 with the LDS group gather (a group's CRCs collected across the
    workgroup's waves, one 256-B store by the wave finishing it), 3 the lazy
    gather (the same, with the slot check loaded before the slicing and the
    count read one round later: no LDS round trip waited on per tile), 4
    columns (schedule 7: a wave reads a 32-chunk run 128 B of every chunk per
    round and writes its 32 CRCs as one 128-B line; the gather on tables
    that are not whole 8-tile groups).
    On the C5-like table and on a table of 13-tile segments, where groups
    straddle segments and fall back to per-tile stores."""
    host, sizes, lens, want, dbuf = table
    nch = [n // cs for cs, n in zip(sizes, lens)]
    crcs = engine.DeviceBuffer(4 * (sum(nch) + 64))
    try:
        diag.reset()
        diag.set_runs(runs)
        for case in ("c5", "odd"):
            if case == "c5":
                segs_spec = [(i * SEG, n, cs) for i, (cs, n) in enumerate(zip(sizes, lens))]
                wants = want
            else:
                segs_spec = [(i * 13 * 4096 + 7, 13 * 4096, 512) for i in range(4000)]  # 200 MiB, 13 tiles each
                wants = None
            crcs.fill(0xA5)
            segs, off = [], 0
            for base, n, cs in segs_spec:
                segs.append(engine.Segment(data=dbuf.ptr + base, len=n, chunk_size=cs, flags=engine.SEG_BE,
                                           crc_init=0, crcs=crcs.ptr + 4 * off, bitmap=None))
                off += n // cs
            p = diag.plan(engine.MODE_COMPUTE, segs)
            p.execute()
            got = crcs.download(4 * (off + 64), dtype=">u4").astype(np.uint32)
            o = 0
            for k, (base, n, cs) in enumerate(segs_spec):
                w = wants[k] if wants is not None else oracle.chunk_crcs(host[base:base + n], cs)
                np.testing.assert_array_equal(got[o:o + n // cs], w, err_msg=f"{case} segment {k}")
                o += n // cs
            assert (got[o:] == 0xA5A5A5A5).all()
            p.destroy()
    finally:
        diag.reset()
        crcs.free()


@pytest.mark.parametrize("variant", ["le", "crc32_be", "init", "raw"])
def test_compute_columns_flags(engine, diag, oracle, table, variant):
    """The column schedule (set_runs(4), schedule 7) on 1 GiB of 512-B chunks
    in 64 segments of whole 8-tile groups, the last tile of each segment 0..4
    chunks short: little-endian CRC arrays, the CRC32 (zlib) tables with
    wire-order CRCs, a non-zero crc_init (sampled chunks vs the oracle) and
    raw registers (SEG_RAW: init 0, no final inversion).  Bit-exact; the
    guard words past the array stay untouched."""
    host, _, _, _, dbuf = table
    cs = 512
    lens = [SEG - (i % 5) * cs for i in range(NSEG)]
    nch = [n // cs for n in lens]
    crcs = engine.DeviceBuffer(4 * (sum(nch) + 64))
    flags = {"le": 0, "crc32_be": engine.SEG_BE | engine.SEG_CRC32, "init": engine.SEG_BE,
             "raw": engine.SEG_BE | engine.SEG_RAW}[variant]
    init = 0x1234ABCD if variant == "init" else 0
    try:
        diag.reset()
        diag.set_runs(4)
        crcs.fill(0xA5)
        segs, off = [], 0
        for i, n in enumerate(lens):
            segs.append(engine.Segment(data=dbuf.ptr + i * SEG, len=n, chunk_size=cs, flags=flags, crc_init=init,
                                       crcs=crcs.ptr + 4 * off, bitmap=None))
            off += n // cs
        p = diag.plan(engine.MODE_COMPUTE, segs)
        p.execute()
        got = crcs.download(4 * (off + 64), dtype="<u4" if variant == "le" else ">u4").astype(np.uint32)
        assert (got[off:] == 0xA5A5A5A5).all()
        o = 0
        rng = np.random.default_rng(7)
        for i, n in enumerate(lens):
            seg = host[i * SEG:i * SEG + n]
            if variant in ("le", "crc32_be"):
                ct = CSUM_CRC32 if variant == "crc32_be" else CSUM_CRC32C
                np.testing.assert_array_equal(got[o:o + n // cs], oracle.chunk_crcs(seg, cs, ctype=ct),
                                              err_msg=f"segment {i}")
            else:
                # every chunk of the last run plus a sample
                picks = set(range(max(0, n // cs - 40), n // cs)) | set(rng.integers(0, n // cs, 24).tolist())
                for c in sorted(picks):
                    chunk = seg[c * cs:(c + 1) * cs]
                    if variant == "init":
                        w = oracle.crc32c(init, chunk)
                    else:
                        w = ~oracle.crc32c(0xFFFFFFFF, chunk) & 0xFFFFFFFF
                    assert got[o + c] == w, (i, c)
            o += n // cs
        p.destroy()
    finally:
        diag.reset()
        crcs.free()
