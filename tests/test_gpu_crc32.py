"""GPU parity for the CRC32 (HDFS_CSUM_CRC32, zlib polynomial) leg.

The reference's CRC32 chunk checksums are zlib crc32() calls
(src/datanode.c:2832-2845 write path, :2940-2952 _verify_crcdata).  The
expected values are the zlib 1.2.11 fixtures of oracle/gen_golden_zlib.py
and the oracle's zlib restatement; the engine runs the same tiled and
generic kernels with the CRC-32 table set.  Bit-exact everywhere."""
import numpy as np
import pytest

from oracle import CSUM_CRC32, splitmix64_np

pytestmark = pytest.mark.gpu

SWEEP_DATA = splitmix64_np(1024 + 8, seed=7).view(np.uint8)


def _dev(engine, host):
    buf = engine.DeviceBuffer(max(1, host.nbytes))
    buf.upload(host)
    return buf


def test_zlib_kats_stream(engine, golden):
    for k in golden["zlib"]["kats"]:
        b = bytes.fromhex(k["hex"])
        assert engine.stream_ex(engine.CSUM_CRC32, 0, b) == k["crc"], k["source"]
    # the CRC32C type through the same entry point is _hdfs_crc32c
    for k in golden["kats"]:
        assert engine.stream_ex(engine.CSUM_CRC32C, 0, bytes.fromhex(k["hex"])) == k["crc"]


def test_zlib_edge_sweep(engine, golden):
    sweep = golden["zlib_sweep"]
    lens = list(range(0, 600)) + list(range(600, 4097, 41)) + [4095, 4096]
    for oi, off in enumerate((0, 3)):
        for n in lens:
            cin = (0x9E3779B9 * (n + 1) + off) & 0xFFFFFFFF
            buf = SWEEP_DATA[off:off + n]
            assert engine.stream_ex(engine.CSUM_CRC32, 0, buf) == sweep[0, oi, n], (off, n)
            assert engine.stream_ex(engine.CSUM_CRC32, cin, buf) == sweep[1, oi, n], (off, n)


@pytest.mark.parametrize("cs", [512, 4096])
@pytest.mark.parametrize("kind", ["full", "ragged"])
def test_zlib_chunk_crcs_golden(engine, golden, cs, kind):
    host = splitmix64_np(1 << 17, seed=0).view(np.uint8)
    n = host.nbytes if kind == "full" else host.nbytes - 123
    want = golden["zlib_chunks"][f"{kind}_{cs}"]
    dbuf = _dev(engine, host[:n])
    out = engine.DeviceBuffer(want.nbytes)
    seg = engine.Segment(data=dbuf.ptr, len=n, chunk_size=cs, flags=engine.SEG_BE | engine.SEG_CRC32,
                         crc_init=0, crcs=out.ptr, bitmap=None)
    engine.Plan(engine.MODE_COMPUTE, [seg]).execute()
    np.testing.assert_array_equal(out.download(dtype=">u4").astype(np.uint32), want)


@pytest.mark.parametrize("nchunks,cs,off", [(1, 512, 0), (9, 512, 0), (65, 1536, 0), (1000, 4096, 0),
                                            (100, 512, 5), (37, 1000, 0)])
def test_zlib_verify_plan(engine, oracle, nchunks, cs, off):
    rng = np.random.default_rng(nchunks + cs + off)
    n = nchunks * cs - (17 if off else 0)
    host = rng.integers(0, 256, n + off, dtype=np.uint8)
    dbuf = _dev(engine, host)
    want = oracle.chunk_crcs(host[off:], cs, ctype=CSUM_CRC32)
    crcs = engine.DeviceBuffer(want.nbytes)
    bm = engine.DeviceBuffer((want.size + 7) // 8)
    seg = engine.Segment(data=dbuf.ptr + off, len=n, chunk_size=cs, flags=engine.SEG_CRC32, crc_init=0,
                         crcs=crcs.ptr, bitmap=bm.ptr)
    engine.Plan(engine.MODE_COMPUTE, [seg]).execute()
    np.testing.assert_array_equal(crcs.download(dtype=np.uint32), want)
    bad = sorted(set(int(x) for x in rng.integers(0, want.size, 3)))
    for ci in bad:
        host[off + ci * cs] ^= 0x01
    dbuf.upload(host)
    vp = engine.Plan(engine.MODE_VERIFY, [seg])
    vp.execute()
    fb, m = vp.results()
    assert m == len(bad) and fb[0] == bad[0]
    assert list(np.nonzero(np.unpackbits(bm.download(), bitorder="little"))[0]) == bad


def test_zlib_plan_rejects_mixed_types(engine):
    dbuf = engine.DeviceBuffer(4096)
    out = engine.DeviceBuffer(64)
    a = engine.Segment(data=dbuf.ptr, len=1024, chunk_size=512, flags=0, crc_init=0, crcs=out.ptr, bitmap=None)
    b = engine.Segment(data=dbuf.ptr, len=1024, chunk_size=512, flags=engine.SEG_CRC32, crc_init=0,
                       crcs=out.ptr, bitmap=None)
    with pytest.raises(engine.CRC32CError):
        engine.Plan(engine.MODE_COMPUTE, [a, b])


def test_zlib_verify_crcdata_golden(engine, golden):
    for case in golden["zlib"]["verify_cases"]:
        region = bytes.fromhex(case["region_hex"])
        cs, dlen = case["chunk_size"], case["dlen"]
        nch = (dlen + cs - 1) // cs
        err, fb = engine.verify_crcdata(region, cs, nch * 4, dlen, ctype=engine.CSUM_CRC32)
        assert fb == case["first_bad"]
        assert err == (engine.ERR_BAD_CHECKSUM if case["mismatch"] else 0)


def test_zlib_host_pipeline(engine, oracle):
    rng = np.random.default_rng(12)
    n, cs = (3 << 20) + 999, 512
    host = rng.integers(0, 256, n, dtype=np.uint8)
    want = oracle.chunk_crcs(host, cs, ctype=CSUM_CRC32)
    be = engine.compute_host(host, cs, flags=engine.SEG_BE | engine.SEG_CRC32, piece_bytes=1 << 20)
    np.testing.assert_array_equal(be.byteswap(), want)
    host[12345] ^= 4
    fb, m, _ = engine.verify_host(host, cs, be, flags=engine.SEG_BE | engine.SEG_CRC32, piece_bytes=1 << 20)
    assert fb == 12345 // cs and m == 1


def test_zlib_block_digests_on_device(engine, golden):
    blk_bytes = 128 << 20
    dbuf = engine.DeviceBuffer(blk_bytes)
    for blk in (0, 1):
        engine.fill_splitmix64(dbuf.ptr, blk_bytes // 8, 0, blk << 24)
        for cs in (512, 4096):
            out = engine.DeviceBuffer(blk_bytes // cs * 4)
            seg = engine.Segment(data=dbuf.ptr, len=blk_bytes, chunk_size=cs, flags=engine.SEG_CRC32,
                                 crc_init=0, crcs=out.ptr, bitmap=None)
            engine.Plan(engine.MODE_COMPUTE, [seg]).execute()
            want = golden["zlib"]["block_digests"][f"block{blk}_{cs}"]
            arr = out.download(dtype=np.uint32)
            assert int(arr[0]) == want["crc0"]
            assert engine.stream_ex(engine.CSUM_CRC32, 0, arr) == want["digest"]
