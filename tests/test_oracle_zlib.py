"""CPU tests: the CRC32 (HDFS_CSUM_CRC32) leg of the oracle, pinned to zlib.

The reference computes CRC32 chunk checksums with zlib's crc32()
(src/datanode.c:2832-2845, :2940-2952); zlib is not vendored in the
reference, so the fixtures come from zlib 1.2.11 itself
(oracle/gen_golden_zlib.py), and zlib is also compared directly here.
"""
import zlib

import numpy as np

from oracle import CSUM_CRC32, splitmix64_np

SWEEP_DATA = splitmix64_np(1024 + 8, seed=7).view(np.uint8)


def test_zlib_pin(golden):
    assert golden["zlib"]["zlib"] == "1.2.11"


def test_zlib_kats(oracle, golden):
    for k in golden["zlib"]["kats"]:
        b = bytes.fromhex(k["hex"])
        assert oracle.crc32c(0, b, "zlib") == k["crc"] == zlib.crc32(b)


def test_zlib_edge_sweep(oracle, golden):
    sweep = golden["zlib_sweep"]
    for oi, off in enumerate((0, 3)):
        for n in range(0, 4097, 1 if off == 0 else 5):
            buf = SWEEP_DATA[off:off + n]
            assert oracle.crc32c(0, buf, "zlib") == sweep[0, oi, n]
            cin = (0x9E3779B9 * (n + 1) + off) & 0xFFFFFFFF
            assert oracle.crc32c(cin, buf, "zlib") == sweep[1, oi, n]


def test_zlib_chunk_crcs(oracle, golden):
    buf = splitmix64_np(1 << 17, seed=0).view(np.uint8)
    for cs in (512, 4096):
        for name, n in (("full", buf.nbytes), ("ragged", buf.nbytes - 123)):
            np.testing.assert_array_equal(oracle.chunk_crcs(buf[:n], cs, ctype=CSUM_CRC32),
                                          golden["zlib_chunks"][f"{name}_{cs}"])


def test_zlib_verify_cases(oracle, golden):
    for case in golden["zlib"]["verify_cases"]:
        region = bytes.fromhex(case["region_hex"])
        cs, dlen = case["chunk_size"], case["dlen"]
        nch = (dlen + cs - 1) // cs
        err, fb = oracle.verify_crcdata(region, cs, nch * 4, dlen, ctype=CSUM_CRC32)
        assert fb == case["first_bad"]
        assert err == (29 if case["mismatch"] else 0)
        if case["mismatch"]:  # the same region is not a valid CRC32C packet either way
            assert oracle.verify_crcdata(region, cs, nch * 4, dlen)[0] == 29


def test_zlib_compose(oracle):
    rng = np.random.default_rng(6)
    data = rng.integers(0, 256, 9000, dtype=np.uint8).tobytes()
    cuts = [0, 3, 512, 513, 2000, 9000]
    frags = [data[a:b] for a, b in zip(cuts[:-1], cuts[1:])]
    want = b"".join(zlib.crc32(data[i:i + 512]).to_bytes(4, "big") for i in range(0, 9000, 512))
    assert oracle.compose_crcs(frags, 512, ctype=CSUM_CRC32) == want
