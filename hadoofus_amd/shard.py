"""Per-GPU sharding of independent HDFS blocks and the one collective.

Every chunk's CRC depends only on its own bytes (src/datanode.c:2945-2954),
so ranks own disjoint, contiguous block ranges and exchange nothing on the
data path.  The only collective is one small all-reduce per run of
{bytes, mismatches, ok} (sum) and elapsed time (max) -- RCCL over xGMI when
torch.distributed runs the "nccl" backend, gloo in the CPU tests.
"""
import os


def rank_blocks(rank, world, blocks_per_rank):
    """Weak scaling: each rank owns `blocks_per_rank` blocks; global block ids
    [rank * blocks_per_rank, (rank + 1) * blocks_per_rank)."""
    if not 0 <= rank < world:
        raise ValueError((rank, world))
    return rank * blocks_per_rank, blocks_per_rank


def split_blocks(total_blocks, rank, world):
    """Strong scaling: split `total_blocks` as evenly as possible."""
    lo = total_blocks * rank // world
    hi = total_blocks * (rank + 1) // world
    return lo, hi - lo


def expected_bad(first_block, nblocks, chunks_per_block, modulus=65537):
    """Chunks with global index i % modulus == 0 in the rank's block range
    (the deterministic corruption pattern of SURVEY.md 8d, config C3)."""
    start = first_block * chunks_per_block
    end = (first_block + nblocks) * chunks_per_block
    first = (start + modulus - 1) // modulus * modulus
    return 0 if first >= end else (end - 1 - first) // modulus + 1


# BASELINE.json configs: C3 = 1024 x 128 MiB blocks per GPU (weak scaling,
# the headline), C4 = 64 GiB = 512 blocks for the whole node, split evenly
# (strong scaling).
WORKLOADS = {"C3": ("weak", 1024), "C4": ("strong", 512)}


def workload_blocks(config, rank, world, blocks=None):
    """-> (scaling, first global block, blocks of this rank) for a bench
    config; blocks overrides the config's block count (per rank for weak,
    total for strong)."""
    scaling, n = WORKLOADS[config]
    n = n if blocks is None else blocks
    if scaling == "weak":
        b0, nb = rank_blocks(rank, world, n)
    else:
        b0, nb = split_blocks(n, rank, world)
    return scaling, b0, nb


def check_distinct_devices(infos):
    """infos: one dict per rank with 'rank', 'pci_bus_id' (the GPU the rank's
    engine is bound to) and 'host' (socket.gethostname(); ranks on different
    nodes usually report the same bus ids).  Raises if two ranks of one host
    share a GPU -- e.g. every rank silently landing on device 0."""
    seen = {}
    for inf in infos:
        bus = inf["pci_bus_id"]
        if not bus:
            raise RuntimeError(f"rank {inf['rank']} reported no PCI bus id")
        key = (inf.get("host", ""), bus)
        if key in seen:
            raise RuntimeError(f"ranks {seen[key]} and {inf['rank']} share GPU {bus} on host {key[0]!r}")
        seen[key] = inf["rank"]
    return len(seen)


def launched_by_torchrun():
    return "TORCHELASTIC_RUN_ID" in os.environ or int(os.environ.get("WORLD_SIZE", "1")) > 1


class Collective:
    """torch.distributed wrapper: nccl (RCCL) on GPUs, gloo on CPU."""

    def __init__(self, backend=None, device=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.rank = int(os.environ.get("RANK", "0"))
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        self.backend = backend or "nccl"
        if self.backend == "nccl":
            torch.cuda.set_device(self.local)
            self.device = torch.device(f"cuda:{self.local}")
        else:
            self.device = torch.device(device or "cpu")
        if not dist.is_initialized():
            dist.init_process_group(self.backend)

    def barrier(self):
        if self.backend == "nccl":
            self.dist.barrier(device_ids=[self.local])
        else:
            self.dist.barrier()

    def allreduce(self, vals, op):
        t = self.torch.tensor(vals, dtype=self.torch.float64, device=self.device)
        self.dist.all_reduce(t, op=getattr(self.dist.ReduceOp, op))
        return t.tolist()

    def gather(self, obj):
        """All ranks' picklable obj, in rank order (all_gather_object)."""
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def aggregate(self, nbytes, mismatches, ok, elapsed):
        """-> (total bytes, total mismatches, ranks ok, max elapsed)."""
        s = self.allreduce([float(nbytes), float(mismatches), float(bool(ok))], "SUM")
        (t,) = self.allreduce([float(elapsed)], "MAX")
        return s[0], s[1], int(s[2]), t

    def close(self):
        if self.dist.is_initialized():
            self.dist.destroy_process_group()


class Local:
    """Single process, no collective (N = 1 without torchrun)."""

    rank, world, local = 0, 1, 0

    def barrier(self):
        pass

    def gather(self, obj):
        return [obj]

    def aggregate(self, nbytes, mismatches, ok, elapsed):
        return float(nbytes), float(mismatches), int(bool(ok)), float(elapsed)

    def close(self):
        pass
