"""Generate tests/golden/zlib_* fixtures for the CRC32 (HDFS_CSUM_CRC32) leg.

The reference computes HDFS_CSUM_CRC32 chunk checksums with zlib's crc32()
(src/datanode.c:12 includes <zlib.h>; calls at :2832-2845 and :2940-2952).
zlib is a third-party dependency that /root/reference does not vendor, so the
expected values here come from zlib itself: Python's zlib module, linked to
the image's zlib 1.2.11 (the version is asserted below).  Inputs are the
reference's own KAT bytes (tests/t_unit.c:146-199, parsed as data) and
splitmix64 streams.

    python oracle/gen_golden_zlib.py
"""
import json
import os
import sys
import zlib

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from oracle import splitmix64_np  # noqa: E402
from gen_golden import parse_t_unit_kats  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")
ZLIB_PIN = "1.2.11"


def main():
    assert zlib.ZLIB_RUNTIME_VERSION == ZLIB_PIN, zlib.ZLIB_RUNTIME_VERSION
    os.makedirs(OUT, exist_ok=True)
    fix = {"generator": "oracle/gen_golden_zlib.py", "zlib": zlib.ZLIB_RUNTIME_VERSION}

    # 1. KATs: the reference's t_unit inputs + classic check values, under zlib.
    kats = []
    inputs = [("tests/t_unit.c:146-199 input", b) for b, _ in parse_t_unit_kats()]
    inputs += [("check value", b"123456789"), ("512 zero bytes", bytes(512)),
               ("512 0xff bytes", b"\xff" * 512), ("empty", b"")]
    for name, b in inputs:
        kats.append({"source": name, "len": len(b), "hex": b.hex(), "crc": zlib.crc32(b)})
    assert kats[-4]["crc"] == 0xCBF43926  # the published CRC-32 check value
    fix["kats"] = kats

    # 2. Edge sweep: lengths 0..4096 x start offsets {0, 3} x crc_in {0, chained}.
    data = splitmix64_np(1024 + 8, seed=7).view(np.uint8)
    sweep = np.zeros((2, 2, 4097), dtype=np.uint32)
    for oi, off in enumerate((0, 3)):
        for n in range(4097):
            buf = data[off:off + n].tobytes()
            sweep[0, oi, n] = zlib.crc32(buf)
            cin = (0x9E3779B9 * (n + 1) + off) & 0xFFFFFFFF
            sweep[1, oi, n] = zlib.crc32(buf, cin)
    np.save(os.path.join(OUT, "zlib_edge_sweep.npy"), sweep)

    # 3. Per-chunk CRC-32 arrays of the 1 MiB splitmix64 (seed 0) buffer.
    buf = splitmix64_np(1 << 17, seed=0).view(np.uint8)
    chunks = {}
    for cs in (512, 4096):
        for name, n in (("full", buf.nbytes), ("ragged", buf.nbytes - 123)):
            nch = (n + cs - 1) // cs
            chunks[f"{name}_{cs}"] = np.array(
                [zlib.crc32(buf[i * cs:min(n, (i + 1) * cs)].tobytes()) for i in range(nch)], dtype=np.uint32)
    np.savez(os.path.join(OUT, "zlib_chunk_crcs.npz"), **chunks)

    # 4. Verify packets [BE crc32s | data] with single-bit corruptions.
    rng = np.random.default_rng(4321)
    cases = []
    for case in range(6):
        cs = [512, 512, 4096, 100, 512, 512][case]
        dlen = [16384, 16384 - 77, 20000, 1000, 1, 0][case]
        d = rng.integers(0, 256, size=dlen, dtype=np.uint8)
        nch = (dlen + cs - 1) // cs
        crcs = [zlib.crc32(d[i * cs:min(dlen, (i + 1) * cs)].tobytes()) for i in range(nch)]
        bad = []
        if nch and case % 2 == 1:
            bad = sorted(set(int(x) for x in rng.integers(0, nch, size=2)))
            for i in bad:
                clen = min(cs, dlen - i * cs)
                bit = int(rng.integers(0, 8 * clen))
                d[i * cs + bit // 8] ^= np.uint8(1 << (bit % 8))
        got = [zlib.crc32(d[i * cs:min(dlen, (i + 1) * cs)].tobytes()) for i in range(nch)]
        mism = [i for i in range(nch) if got[i] != crcs[i]]
        assert mism == bad
        be = b"".join(int(c).to_bytes(4, "big") for c in crcs)
        cases.append({"chunk_size": cs, "dlen": dlen, "region_hex": (be + d.tobytes()).hex(),
                      "mismatch": mism, "first_bad": mism[0] if mism else -1})
    fix["verify_cases"] = cases

    # 5. Full-block digests (blocks 0, 1 of SURVEY.md 8c) under CRC-32.
    digests = {}
    for blk in (0, 1):
        b = splitmix64_np(1 << 24, seed=0, g0=blk << 24).view(np.uint8)
        for cs in (512, 4096):
            mv = memoryview(b)
            arr = np.fromiter((zlib.crc32(mv[i:i + cs]) for i in range(0, b.nbytes, cs)),
                              dtype=np.uint32, count=b.nbytes // cs)
            digests[f"block{blk}_{cs}"] = {"digest": zlib.crc32(arr.tobytes()), "crc0": int(arr[0])}
    fix["block_digests"] = digests
    fix["digest"] = "zlib.crc32 of the LE u32 per-chunk CRC-32 array"
    with open(os.path.join(OUT, "zlib_vectors.json"), "w") as f:
        json.dump(fix, f)
    print("zlib fixtures written to", os.path.abspath(OUT))


if __name__ == "__main__":
    main()
