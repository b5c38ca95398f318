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


def _worker(rank, world, port, q, config="C3", dup=False):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    col = shard.Collective(backend="gloo")
    # the device report bench.py gathers (a fake bus id per local rank; dup:
    # every rank claims GPU 0, which rank 0 must refuse)
    infos = col.gather({"rank": rank, "local_rank": rank, "device": 0 if dup else rank,
                        "pci_bus_id": f"0000:{(0 if dup else rank) + 0x11:02x}:00.0", "host": socket.gethostname()})
    try:
        ndev = shard.check_distinct_devices(infos)
    except RuntimeError as e:
        ndev = str(e)
    blocks = BLOCKS_PER_RANK if config == "C3" else None
    scaling, b0, nb = shard.workload_blocks(config, rank, world, blocks)
    bad = shard.expected_bad(b0, nb, CHUNKS_PER_BLOCK)
    nbytes = nb * (128 << 20)
    elapsed = 1.0 + rank  # rank r "took" 1 + r seconds
    col.barrier()
    tot_bytes, tot_bad, ok, tmax = col.aggregate(nbytes, bad, True, elapsed)
    q.put((rank, b0, nb, bad, tot_bytes, tot_bad, ok, tmax, ndev, scaling, [i["rank"] for i in infos]))
    col.close()


def _run(world, **kw):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q), kwargs=kw) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("world", [2, 8])
def test_gloo_world2_sharding_and_aggregate(world):
    res = _run(world)
    for r in res:
        assert r[8] == world  # distinct devices, counted on every rank
        assert r[9] == "weak" and r[10] == list(range(world))
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


@pytest.mark.parametrize("world", [2, 8])
def test_gloo_c4_strong_split(world):
    """C4 (BASELINE.json configs[3]): 512 blocks split evenly over the ranks,
    disjoint and complete, aggregate bytes = the whole 64 GiB."""
    res = _run(world, config="C4")
    covered = sorted(b for _, b0, nb, *_ in res for b in range(b0, b0 + nb))
    assert covered == list(range(512))
    assert max(r[2] for r in res) - min(r[2] for r in res) <= 1
    for r in res:
        assert r[9] == "strong"
        assert r[4] == 512 * (128 << 20)
        assert r[5] == shard.expected_bad(0, 512, CHUNKS_PER_BLOCK)


def test_gloo_duplicate_device_refused():
    """Every rank reporting the same GPU is caught by the gathered check."""
    res = _run(2, dup=True)
    for r in res:
        assert isinstance(r[8], str) and "share GPU" in r[8]


def test_check_distinct_devices_unit():
    assert shard.check_distinct_devices([{"rank": i, "pci_bus_id": f"b{i}"} for i in range(8)]) == 8
    with pytest.raises(RuntimeError):
        shard.check_distinct_devices([{"rank": 0, "pci_bus_id": "x"}, {"rank": 1, "pci_bus_id": "x"}])
    with pytest.raises(RuntimeError):
        shard.check_distinct_devices([{"rank": 0, "pci_bus_id": ""}])
    # multi-node: the same bus id on two hosts is two GPUs, on one host it is one
    two_nodes = [{"rank": r, "host": f"node{r // 8}", "pci_bus_id": f"0000:{r % 8 + 0x11:02x}:00.0"}
                 for r in range(16)]
    assert shard.check_distinct_devices(two_nodes) == 16
    with pytest.raises(RuntimeError):
        shard.check_distinct_devices(two_nodes + [{"rank": 16, "host": "node1", "pci_bus_id": "0000:11:00.0"}])
