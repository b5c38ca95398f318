"""Per-block digests of the full C2 / C3 / C5 workloads, from the REFERENCE
compiled unchanged (oracle/_ref/libhdfsref.so, recipe oracle/Makefile).

Test infrastructure only.  Run in the build container (where /root/reference
exists):
    make -C oracle && python oracle/gen_block_digests.py

Data: block b is the 2^24 little-endian u64 words
splitmix64(seed 0, g = b*2^24 + k), k < 2^24 (128 MiB), b = 0..1023, i.e.
the bench's 128 GiB.  For every block and chunk size c in 512/1024/2048/4096
the per-chunk CRCs are computed by the reference's _hdfs_crc32c dispatcher
(src/crc32c.c:72-73 -> src/crc32c_sse42.c:214-381), one call per chunk as
_verify_crcdata does (src/datanode.c:2945-2954), on all host cores; the
digests are _hdfs_crc32c(0, crc array as LE u32 bytes) and the same over the
array in wire (big-endian) order (src/util.h:68-92), plus crc[0].  Blocks
0/1 must reproduce SURVEY.md 8c's pinned values.

BLOCKS (default 8192 = 1 TiB: the 1024 blocks of every rank of an 8-GPU
weak-scaling run) blocks are digested.  Writes
tests/golden/block_digests_all.npz: uint32 arrays le / be / crc0 of shape
[BLOCKS, 4] (column j = chunk size 512 << j), ~0.4 MB.
"""
import ctypes
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from oracle import Oracle, Reference  # noqa: E402

OUT = os.path.join(HERE, "..", "tests", "golden", "block_digests_all.npz")
BLOCKS = int(os.environ.get("BLOCKS", "8192"))
WORDS = 1 << 24  # 128 MiB
SIZES = (512, 1024, 2048, 4096)
PINNED = {(0, 512): 0xF2590C08, (1, 512): 0xEB636035, (0, 1024): 0x51D425B4, (0, 2048): 0x02664494,
          (0, 4096): 0xB77BAB49, (1, 1024): 0xCF09BD7D, (1, 2048): 0x21321D29, (1, 4096): 0xEF4F7B33}


def main():
    o, ref = Oracle(), Reference()
    ext = ctypes.cast(ref.crc32c_fn, ctypes.c_void_p).value
    nthreads = len(os.sched_getaffinity(0))
    buf = np.empty(WORDS, dtype=np.uint64)
    parts = 8
    out = {k: np.zeros((BLOCKS, len(SIZES)), dtype=np.uint32) for k in ("le", "be", "crc0")}
    t0 = time.time()
    with ThreadPoolExecutor(parts) as ex:
        for b in range(BLOCKS):
            step = WORDS // parts
            list(ex.map(lambda i: o._fill(buf[i * step:].ctypes.data, step, 0, b * WORDS + i * step), range(parts)))
            data = buf.view(np.uint8)
            for j, c in enumerate(SIZES):
                _, crcs = o.bench_chunks(data, c, nthreads, "ext", ext)
                le = ref.crc32c(0, crcs.astype("<u4").view(np.uint8))
                be = ref.crc32c(0, crcs.astype(">u4").view(np.uint8))
                out["le"][b, j], out["be"][b, j], out["crc0"][b, j] = le, be, crcs[0]
                if (b, c) in PINNED:
                    assert le == PINNED[(b, c)], (b, c, hex(le))
            if b % 64 == 63:
                print(f"block {b + 1}/{BLOCKS} {time.time() - t0:.0f}s", file=sys.stderr, flush=True)
    # spot-check: the slicing-by-8 software backend agrees on a few blocks
    for b in (0, BLOCKS // 2, BLOCKS - 1):
        o._fill(buf.ctypes.data, WORDS, 0, b * WORDS)
        _, crcs = o.bench_chunks(buf.view(np.uint8), 512, nthreads, "ext",
                                 ctypes.cast(ref.sw_fn, ctypes.c_void_p).value)
        assert ref.crc32c(0, crcs.astype("<u4").view(np.uint8)) == out["le"][b, 0], b
    np.savez_compressed(OUT, chunk_sizes=np.array(SIZES, dtype=np.uint32), **out)
    print(f"wrote {OUT} in {time.time() - t0:.0f}s", file=sys.stderr)


if __name__ == "__main__":
    main()
