"""CPU tests: the oracle is pinned to the reference before it is trusted.

The golden fixtures in tests/golden/ were produced by the reference's own
CRC32C compiled unchanged (oracle/_ref, oracle/gen_golden.py).  If the
reference build is present (this container) it is also compared directly.
"""
import os

import numpy as np
import pytest

from oracle import Reference, have_reference, splitmix64_np

SWEEP_DATA = splitmix64_np(1024 + 8, seed=7).view(np.uint8)


def test_kats(oracle, golden):
    # tests/t_unit.c:146-217 plus check value / zero / 0xff blocks
    assert len([k for k in golden["kats"] if k["source"].startswith("tests/t_unit.c")]) == 3
    for k in golden["kats"]:
        b = bytes.fromhex(k["hex"])
        for kind in ("sw", "hw", "bitwise"):
            assert oracle.crc32c(0, b, kind) == k["crc"], (kind, k["len"])


def test_edge_sweep(oracle, golden):
    sweep = golden["sweep"]
    for off in range(8):
        for n in range(0, 4097, 1 if off == 0 else 7):
            buf = SWEEP_DATA[off:off + n]
            assert oracle.crc32c(0, buf, "sw") == sweep[0, off, n]
            cin = (0x9E3779B9 * (n + 1) + off) & 0xFFFFFFFF
            assert oracle.crc32c(cin, buf, "hw") == sweep[1, off, n]


def test_chunk_crcs(oracle, golden):
    buf = splitmix64_np(1 << 17, seed=0).view(np.uint8)
    for cs in (512, 1024, 2048, 4096):
        for name, n in (("full", buf.nbytes), ("ragged", buf.nbytes - 123)):
            np.testing.assert_array_equal(oracle.chunk_crcs(buf[:n], cs), golden["chunks"][f"{name}_{cs}"])


def test_verify_cases(oracle, golden):
    for case in golden["verify"]:
        region = bytes.fromhex(case["region_hex"])
        cs, dlen = case["chunk_size"], case["dlen"]
        nch = (dlen + cs - 1) // cs
        err, fb = oracle.verify_crcdata(region, cs, nch * 4, dlen)
        assert fb == case["first_bad"]
        assert err == (29 if case["mismatch"] else 0)
        # framing: wrong crcdlen -> HDFS_ERR_DATANODE_CRC_LEN (datanode.c:2441-2442)
        if nch:
            assert oracle.verify_crcdata(region, cs, nch * 4 - 4, dlen)[0] == 26


def test_compose_matches_chunking(oracle):
    rng = np.random.default_rng(5)
    data = rng.integers(0, 256, 70000, dtype=np.uint8).tobytes()
    cuts = [0, 1, 511, 512, 513, 4000, 65536, 70000]
    frags = [data[a:b] for a, b in zip(cuts[:-1], cuts[1:])]
    be = oracle.compose_crcs(frags, 512)
    want = oracle.chunk_crcs(np.frombuffer(data, np.uint8), 512, hw=False)
    assert be == want.astype(">u4").tobytes()


def test_combine_identity(oracle):
    rng = np.random.default_rng(9)
    for la, lb in [(0, 0), (1, 0), (0, 1), (17, 33), (512, 512), (1000, 4096), (3, 100000)]:
        a = rng.integers(0, 256, la, dtype=np.uint8)
        b = rng.integers(0, 256, lb, dtype=np.uint8)
        whole = oracle.crc32c(0, np.concatenate([a, b]), "hw")
        assert oracle.combine(oracle.crc32c(0, a), oracle.crc32c(0, b), lb) == whole
        # chaining: f(f(0,A),B) == f(0,A||B) (src/crc32c.h:6-9)
        assert oracle.crc32c(oracle.crc32c(0, a), b) == whole


def test_splitmix_formula(oracle):
    np.testing.assert_array_equal(oracle.splitmix(4096, 0, 12345), splitmix64_np(4096, 0, 12345))
    # block 0 starts af cd 1d 7b 39 a8 20 e2
    assert splitmix64_np(1).view(np.uint8).tobytes().hex() == "afcd1d7b39a820e2"


@pytest.mark.slow
def test_block_digests(oracle, golden):
    """Full 128 MiB blocks 0 and 1 (SURVEY.md 8c pinned digests)."""
    for blk in (0, 1):
        b = oracle.splitmix(1 << 24, 0, blk << 24).view(np.uint8)
        for cs in (512, 4096):
            arr = oracle.chunk_crcs(b, cs)
            want = golden["blocks"][f"block{blk}_{cs}"]
            assert int(arr[0]) == want["crc0"]
            assert oracle.crc32c(0, arr.view(np.uint8), "hw") == want["digest"]


@pytest.mark.skipif(not have_reference(), reason="reference build (oracle/_ref) not present")
def test_oracle_vs_reference_random():
    from oracle import Oracle
    o, r = Oracle(), Reference()
    rng = np.random.default_rng(77)
    for _ in range(300):
        n = int(rng.integers(0, 9000))
        off = int(rng.integers(0, 16))
        buf = rng.integers(0, 256, n + off, dtype=np.uint8)[off:]
        cin = int(rng.integers(0, 1 << 32))
        want = r.crc32c(cin, buf, "sse42")
        assert r.crc32c(cin, buf, "sw") == want
        assert o.crc32c(cin, buf, "sw") == want
        assert o.crc32c(cin, buf, "hw") == want


def test_all_block_digests_sampled(oracle):
    """The oracle restatement against the reference-generated per-block
    digests of the full bench workloads (oracle/gen_block_digests.py,
    tests/golden/block_digests_all.npz): a spread of blocks at every chunk
    size, LE and wire-order digests and crc[0]."""
    import os

    import numpy as np
    from oracle import splitmix64_np  # noqa: F401
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "block_digests_all.npz"))
    assert z["be"].shape == (8192, 4) and list(z["chunk_sizes"]) == [512, 1024, 2048, 4096]
    assert z["le"][0, 0] == 0xF2590C08 and z["le"][1, 0] == 0xEB636035
    buf = np.empty(1 << 24, dtype=np.uint64)
    for b in (2, 1023, 4097, 8191):
        oracle._fill(buf.ctypes.data, 1 << 24, 0, b << 24)
        for j, cs in enumerate((512, 1024, 2048, 4096)):
            crcs = oracle.chunk_crcs(buf.view(np.uint8), cs)
            assert int(crcs[0]) == z["crc0"][b, j]
            assert oracle.crc32c(0, crcs.astype("<u4").view(np.uint8), "hw") == z["le"][b, j], (b, cs)
            assert oracle.crc32c(0, crcs.astype(">u4").view(np.uint8), "hw") == z["be"][b, j], (b, cs)
