"""GPU: block composite CRC from chunk CRCs (the COMPOSITE_CRC
block checksum of src/proto/datatransfer.proto:316-322).  The composite of a
segment must equal the plain CRC of its whole data: checked against the
oracle (CRC32C) / zlib (CRC32) over the same bytes, and against the engine's
own data-reading stream CRC."""
import zlib

import numpy as np
import pytest

from oracle import splitmix64_np

pytestmark = pytest.mark.gpu


def _plan_crcs(engine, dbuf, specs, flags):
    """Compute plan over (offset, len, cs) specs; returns the segments."""
    segs, keep = [], []
    for off, n, cs in specs:
        out = engine.DeviceBuffer(max(4, (n + cs - 1) // cs * 4))
        keep.append(out)
        segs.append(engine.Segment(data=dbuf.ptr + off, len=n, chunk_size=cs, flags=flags, crc_init=0,
                                   crcs=out.ptr, bitmap=None))
    engine.Plan(engine.MODE_COMPUTE, segs).execute()
    return segs, keep


@pytest.mark.parametrize("flags", [0, 1, 4, 5])  # LE / BE wire order x CRC32C / CRC32
def test_composite_matches_whole_data_crc(engine, oracle, flags):
    rng = np.random.default_rng(flags + 3)
    host = rng.integers(0, 256, 6 << 20, dtype=np.uint8)
    dbuf = engine.DeviceBuffer(host.nbytes)
    dbuf.upload(host)
    specs = [(0, 1 << 20, 512), (1 << 20, (1 << 20) - 333, 512), (2 << 20, 4096 * 100 + 1, 4096),
             (3 << 20, 99999, 100), (4 << 20, 0, 512), (4 << 20, 1, 512), (5 << 20, 512 * 64, 512),
             (5 << 20, 512 * 65 + 7, 1536)]
    segs, keep = _plan_crcs(engine, dbuf, specs, flags)
    got = engine.composite_crcs(segs)
    for (off, n, cs), g in zip(specs, got):
        b = host[off:off + n]
        want = zlib.crc32(b.tobytes()) if flags & 4 else oracle.crc32c(0, b, "hw")
        assert g == want, (off, n, cs, flags)


def test_composite_full_blocks(engine, oracle):
    """1024 x 128 MiB block shape: blocks 0..3 (data generated on device),
    composite == stream CRC of the block read from HBM == oracle."""
    blk = 128 << 20
    dbuf = engine.DeviceBuffer(4 * blk)
    engine.fill_splitmix64(dbuf.ptr, 4 * blk // 8, 0, 0)
    specs = [(b * blk, blk, 512) for b in range(4)]
    segs, keep = _plan_crcs(engine, dbuf, specs, engine.SEG_BE)
    got = engine.composite_crcs(segs)
    for b in range(4):
        assert got[b] == engine.stream_crc_dev(0, dbuf.ptr + b * blk, blk)
    host0 = splitmix64_np(blk // 8, seed=0, g0=0).view(np.uint8)
    assert got[0] == oracle.crc32c(0, host0, "hw")


def test_composite_rejects_nonzero_init(engine):
    dbuf = engine.DeviceBuffer(4096)
    out = engine.DeviceBuffer(64)
    seg = engine.Segment(data=dbuf.ptr, len=4096, chunk_size=512, flags=0, crc_init=5, crcs=out.ptr, bitmap=None)
    with pytest.raises(engine.CRC32CError):
        engine.composite_crcs([seg])
