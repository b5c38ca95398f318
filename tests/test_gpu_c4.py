"""BASELINE config C4 on the HIP path: 8 x MI355X, 64 GiB of 128 MiB blocks
sharded evenly (512 blocks, 64 per GPU), 512-B chunks, independent per-GPU
kernels (the chunks are independent,
src/datanode.c:2945-2954).

The driver has no 8-GPU node to run the sharded bench on, so this test runs
every rank's shard of the C4 workload, one after another, on the one GPU:
each rank's 64 blocks are generated on device at their global block offset
(shard.workload_blocks("C4", r, 8)), computed in one plan, and every block's
CRC array is digest-checked against the reference-generated
tests/golden/block_digests_all.npz.  Then the C3 corruption pattern (global
chunk index i % 65537 == 0) is applied and verified: each shard's mismatch
count must be the one shard.expected_bad predicts, and every bitmap bit and
first-bad index must be exactly the corrupted chunks."""
import os

import numpy as np
import pytest

from hadoofus_amd import shard

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "block_digests_all.npz")
BLK = 128 << 20
CS = 512
PER = BLK // CS  # chunks per block


def test_c4_every_rank_shard(engine):
    z = np.load(GOLDEN)
    world = 8
    _, _, nb = shard.workload_blocks("C4", 0, world)
    assert nb == 64
    data = engine.DeviceBuffer(nb * BLK)          # 8 GiB: one rank's shard
    crcs = engine.DeviceBuffer(nb * PER * 4)
    bms = engine.DeviceBuffer(nb * PER // 8)
    digs = engine.DeviceBuffer(4 * nb)
    total_bad = 0
    covered = []
    try:
        for rank in range(world):
            scaling, b0, nb_r = shard.workload_blocks("C4", rank, world)
            assert scaling == "strong" and nb_r == nb
            covered += list(range(b0, b0 + nb_r))
            for i in range(nb):
                engine.fill_splitmix64(data.ptr + i * BLK, BLK // 8, 0, (b0 + i) << 24)
            segs = [engine.Segment(data=data.ptr + i * BLK, len=BLK, chunk_size=CS, flags=engine.SEG_BE,
                                   crc_init=0, crcs=crcs.ptr + i * PER * 4, bitmap=bms.ptr + i * PER // 8)
                    for i in range(nb)]
            engine.Plan(engine.MODE_COMPUTE, segs).execute()
            # every block's CRC array against the reference's digest (one launch)
            dsegs = [engine.Segment(data=crcs.ptr + i * PER * 4, len=PER * 4, chunk_size=PER * 4, flags=0,
                                    crc_init=0, crcs=digs.ptr + 4 * i) for i in range(nb)]
            engine.Plan(engine.MODE_COMPUTE, dsegs).execute()
            got = digs.download(dtype=np.uint32)
            want = z["be"][b0:b0 + nb, 0]
            assert np.array_equal(got, want), (rank, np.nonzero(got != want)[0][:8])
            # the C3 corruption pattern on global chunk indices, then verify
            for i in range(nb):
                engine.corrupt(data.ptr + i * BLK, BLK, CS, (b0 + i) * PER, 65537, 7919)
            vp = engine.Plan(engine.MODE_VERIFY, segs)
            vp.execute()
            first_bad, mism = vp.results()
            nbad = shard.expected_bad(b0, nb, PER)
            assert mism == nbad, (rank, mism, nbad)
            start = b0 * PER
            expect = np.arange((start + 65536) // 65537 * 65537, start + nb * PER, 65537, dtype=np.int64) - start
            assert expect.size == nbad
            bits = np.unpackbits(bms.download(), bitorder="little")
            assert np.array_equal(np.nonzero(bits)[0], expect), rank
            for i in range(nb):
                mine = expect[(expect >= i * PER) & (expect < (i + 1) * PER)] - i * PER
                assert first_bad[i] == (int(mine[0]) if mine.size else 0xFFFFFFFF), (rank, i)
            total_bad += mism
    finally:
        for b in (data, crcs, bms, digs):
            b.free()
    # the eight shards are the whole 64 GiB workload, each block once
    assert covered == list(range(512))
    assert total_bad == shard.expected_bad(0, 512, PER)
