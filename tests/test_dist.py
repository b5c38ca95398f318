"""CPU multi-process test of the N>1 path: world_size 2 over gloo.

Covers the block sharding (disjoint, complete), the expected-corruption
bookkeeping per rank, and the single aggregation collective bench.py uses
(sum of bytes / mismatches / ok, max of elapsed)."""
import os
import socket

import pytest
import torch.multiprocessing as mp

from hadoofus_amd import shard

BLOCKS_PER_RANK = 5
CHUNKS_PER_BLOCK = 262144


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    col = shard.Collective(backend="gloo")
    b0, nb = shard.rank_blocks(rank, world, BLOCKS_PER_RANK)
    bad = shard.expected_bad(b0, nb, CHUNKS_PER_BLOCK)
    nbytes = nb * (128 << 20)
    elapsed = 1.0 + rank  # rank r "took" 1 + r seconds
    col.barrier()
    tot_bytes, tot_bad, ok, tmax = col.aggregate(nbytes, bad, True, elapsed)
    q.put((rank, b0, nb, bad, tot_bytes, tot_bad, ok, tmax))
    col.close()


@pytest.mark.parametrize("world", [2, 8])
def test_gloo_world2_sharding_and_aggregate(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # disjoint + complete block coverage
    covered = sorted(b for _, b0, nb, *_ in res for b in range(b0, b0 + nb))
    assert covered == list(range(world * BLOCKS_PER_RANK))
    # per-rank expected-bad counts add up to the global count
    total_bad = shard.expected_bad(0, world * BLOCKS_PER_RANK, CHUNKS_PER_BLOCK)
    assert sum(r[3] for r in res) == total_bad
    for r in res:
        assert r[4] == world * BLOCKS_PER_RANK * (128 << 20)
        assert r[5] == total_bad
        assert r[6] == world
        assert r[7] == float(world)  # max elapsed = 1 + (world - 1)


def test_expected_bad_bruteforce():
    for b0, nb, per, mod in [(0, 3, 100, 7), (5, 4, 64, 13), (2, 1, 10, 1000), (0, 0, 10, 3)]:
        want = sum(1 for i in range(b0 * per, (b0 + nb) * per) if i % mod == 0)
        assert shard.expected_bad(b0, nb, per, mod) == want


def test_split_blocks_strong():
    for total in (0, 1, 7, 512):
        for world in (1, 2, 3, 8):
            parts = [shard.split_blocks(total, r, world) for r in range(world)]
            assert sum(n for _, n in parts) == total
            assert all(parts[i][0] + parts[i][1] == parts[i + 1][0] for i in range(world - 1))
