"""Generate tests/golden/ fixtures from the REFERENCE compiled unchanged.

Run in the build container (where /root/reference exists):
    make -C oracle && python oracle/gen_golden.py

Every expected value below is computed by oracle/_ref/libhdfsref.so, i.e. the
reference's src/crc32c.c + crc32c_sw.c + crc32c_sse42.c built by
oracle/Makefile; the dispatcher (_hdfs_crc32c), the software backend and the
SSE4.2 backend are all called and must agree.  Inputs are either the KAT
bytes from the reference's tests/t_unit.c:146-199 (data) or splitmix64
streams defined by formula, so only expected outputs and small
inputs are committed.
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from oracle import Reference, splitmix64_np  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")

T_UNIT = "/root/reference/tests/t_unit.c"


def parse_t_unit_kats(path=T_UNIT):
    """Extract the known-answer vectors of tests/t_unit.c:146-199 as data
    (input bytes, length, expected CRC); the reference file is read as text."""
    import re
    src = open(path).read()
    s0 = src.index("START_TEST(test_crc32c)")
    body = src[s0:src.index("END_TEST", s0)]
    out = []
    for m in re.finditer(r'\{\s*((?:"[^"]*"\s*)+),\s*(\d+),\s*(0x[0-9a-fA-F]+)\s*\}', body):
        lit = "".join(re.findall(r'"([^"]*)"', m.group(1)))
        b = bytes(int(h, 16) for h in re.findall(r"\\x([0-9a-fA-F]{2})", lit))
        assert len(b) == int(m.group(2)), (len(b), m.group(2))
        out.append((b, int(m.group(3), 16)))
    assert len(out) == 3, len(out)
    return out


def crc_all(ref, crc, buf):
    a = ref.crc32c(crc, buf, "dispatch")
    b = ref.crc32c(crc, buf, "sw")
    c = ref.crc32c(crc, buf, "sse42")
    assert a == b == c, (a, b, c)
    return a


def main():
    ref = Reference()
    os.makedirs(OUT, exist_ok=True)

    # 1. KATs --------------------------------------------------------------
    kpath = os.path.join(OUT, "kats.json")
    kats = []
    for b, exp in parse_t_unit_kats():
        got = crc_all(ref, 0, b)
        assert got == exp, (hex(got), hex(exp))
        kats.append({"source": "tests/t_unit.c:146-199", "len": len(b), "hex": b.hex(), "crc": exp})
    extra = [
        ("check value", b"123456789"),
        ("512 zero bytes", bytes(512)),
        ("512 0xff bytes", b"\xff" * 512),
        ("empty", b""),
    ]
    for name, b in extra:
        kats.append({"source": "reference-generated: " + name, "len": len(b), "hex": b.hex(),
                     "crc": crc_all(ref, 0, b)})
    with open(kpath, "w") as f:
        json.dump({"generator": "oracle/gen_golden.py", "kats": kats}, f, indent=1)

    # 2. Edge sweep: lengths 0..4096 x start offsets 0..7 x crc_in {0, chained}
    data = splitmix64_np(1024 + 8, seed=7).view(np.uint8)  # 8256 bytes
    lens = np.arange(0, 4097)
    sweep = np.zeros((2, 8, lens.size), dtype=np.uint32)
    for off in range(8):
        for n in lens:
            buf = data[off:off + n].tobytes()
            sweep[0, off, n] = crc_all(ref, 0, buf)
            cin = (0x9E3779B9 * (n + 1) + off) & 0xFFFFFFFF
            sweep[1, off, n] = crc_all(ref, cin, buf)
    np.save(os.path.join(OUT, "edge_sweep.npy"), sweep)

    # 3. Per-chunk CRC arrays of a 1 MiB splitmix64 (seed 0) buffer and of a
    #    ragged 1 MiB - 123 B prefix (partial last chunk).
    buf = splitmix64_np(1 << 17, seed=0).view(np.uint8)
    chunk_fix = {}
    for cs in (512, 1024, 2048, 4096):
        for name, n in (("full", buf.nbytes), ("ragged", buf.nbytes - 123)):
            nch = (n + cs - 1) // cs
            arr = np.array([crc_all(ref, 0, buf[i * cs:min(n, (i + 1) * cs)].tobytes())
                            for i in range(nch)], dtype=np.uint32)
            chunk_fix[f"{name}_{cs}"] = arr
    np.savez(os.path.join(OUT, "chunk_crcs.npz"), **chunk_fix)

    # 4. Verify fixtures: packet regions [BE crcs | data] with single-bit
    #    corruptions; expected first-bad chunk and mismatch bitmap.
    vfix = []
    rng = np.random.default_rng(1234)
    for case in range(12):
        cs = [512, 512, 512, 1024, 2048, 4096, 512, 100, 512, 512, 4096, 512][case]
        dlen = [65536, 65536 - 77, 512, 65536, 65536, 65536, 1, 1000, 0, 65536, 5000, 33][case]
        d = rng.integers(0, 256, size=dlen, dtype=np.uint8)
        nch = (dlen + cs - 1) // cs
        crcs = [crc_all(ref, 0, d[i * cs:min(dlen, (i + 1) * cs)].tobytes()) for i in range(nch)]
        bad = []
        if nch and case % 3 != 0:
            k = int(rng.integers(1, 4))
            bad = sorted(set(int(x) for x in rng.integers(0, nch, size=k)))
            for i in bad:
                clen = min(cs, dlen - i * cs)
                bit = int(rng.integers(0, 8 * clen))
                d[i * cs + bit // 8] ^= np.uint8(1 << (bit % 8))
        # expected per-chunk result recomputed by the reference on the corrupted data
        got = [crc_all(ref, 0, d[i * cs:min(dlen, (i + 1) * cs)].tobytes()) for i in range(nch)]
        mism = [i for i in range(nch) if got[i] != crcs[i]]
        assert mism == bad, (mism, bad)
        be = b"".join(int(c).to_bytes(4, "big") for c in crcs)
        vfix.append({"chunk_size": cs, "dlen": dlen, "region_hex": (be + d.tobytes()).hex(),
                     "mismatch": mism, "first_bad": mism[0] if mism else -1})
    with open(os.path.join(OUT, "verify_cases.json"), "w") as f:
        json.dump({"generator": "oracle/gen_golden.py", "cases": vfix}, f)

    # 5. Full-block digests (block 0 and 1 of SURVEY.md 8c), re-derived here.
    digests = {}
    for blk in (0, 1):
        words = splitmix64_np(1 << 24, seed=0, g0=blk << 24)
        b = words.view(np.uint8)
        for cs in (512, 1024, 2048, 4096):
            nch = b.nbytes // cs
            arr = np.empty(nch, dtype=np.uint32)
            for i in range(nch):
                arr[i] = ref.crc32c(0, b[i * cs:(i + 1) * cs], "sse42")
            dig = ref.crc32c(0, arr.view(np.uint8), "sse42")
            digests[f"block{blk}_{cs}"] = {"digest": dig, "crc0": int(arr[0])}
    with open(os.path.join(OUT, "block_digests.json"), "w") as f:
        json.dump({"generator": "oracle/gen_golden.py", "data": "splitmix64 seed 0, g = block*2^24 + k",
                   "digest": "_hdfs_crc32c(0, LE u32 crc array)", "blocks": digests}, f, indent=1)
    print("golden fixtures written to", os.path.abspath(OUT))


if __name__ == "__main__":
    main()
