#!/usr/bin/env python3
"""Benchmark: CRC32C verify GiB/s (device-resident), 512 B chunks over 128 MiB
HDFS blocks (BASELINE.json metric).

One STEP = one verify pass of the hot path over this rank's whole batch of
128 MiB blocks of splitmix64 data generated on device: expected per-chunk
CRCs in wire (big-endian) order, 1 in 65537 chunks corrupted; output = the
mismatch bitmap + first bad chunk per block (_verify_crcdata,
src/datanode.c:2931-2963, over every chunk of every block).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C3|C4]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

`python bench.py --gpus N` (N > 1) outside torchrun starts
torch.distributed.run with N ranks as a child process (before any GPU
call) and exits with its code; under torchrun, --gpus must equal
WORLD_SIZE or the run is refused.  At N > 1 the C3 line is weak scaling
(1024 blocks per GPU) and extra.c4_strong times BASELINE's C4 split.

--config C3 (default, the headline): 1024 blocks (128 GiB) per GPU, weak
scaling.  --config C4: 512 blocks (64 GiB) for the whole node split evenly
over the ranks (BASELINE.json configs[3]), strong scaling.  Ranks shard
independent blocks (hadoofus_amd/shard.py: no data-path collective); each
rank binds its engine to LOCAL_RANK explicitly and the ranks' PCI bus ids
are gathered and checked distinct; one all-reduce aggregates {bytes,
mismatches, ok} (sum) and time (max).

Around the timed C3 loop, outside it: C2 (compute-only) is timed and every
block's CRC array is digest-checked against the reference-generated
tests/golden/block_digests_all.npz; C5 (mixed 512/1024/2048/4096 in one
launch) is computed on clean data, digest-checked per block, then verified
after the corruption with its exact expected bitmap; the C3 bitmap is
compared bit for bit with the corruption pattern; the verify kernel's
load-only twin from the diagnostic build gives the empirical ceiling.
Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import platform
import socket
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "CRC32C verify GiB/s (device-resident), 512B chunks over 128MiB HDFS blocks"
BLOCK = 128 << 20
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
MOD, BITMUL = 65537, 7919  # SURVEY.md 8d corruption pattern
SIZES = (512, 1024, 2048, 4096)
DIGESTS = os.path.join(ROOT, "tests", "golden", "block_digests_all.npz")
# SURVEY.md 8c pinned digests (reference-generated): _hdfs_crc32c(0, LE crc array)
PINNED = {(0, 512): 0xF2590C08}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks, one per GPU (default: WORLD_SIZE under torchrun, else 1); without torchrun, "
                         "N > 1 starts torch.distributed.run as a child process")
    ap.add_argument("--dry-run", action="store_true",
                    help="rank plumbing only: gloo, no device work (the launcher's CPU test)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", choices=("C3", "C4"), default="C3")
    ap.add_argument("--blocks", type=int, default=None,
                    help="override the config's block count (per GPU for C3, total for C4)")
    ap.add_argument("--chunk", type=int, default=512)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-extra", action="store_true", help="skip C2/C5/ceiling side measurements")
    ap.add_argument("--cpu-gib", type=float, default=4.0, help="CPU baseline sample size (GiB)")
    return ap.parse_args(argv)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv):
    """`bench.py --gpus N` without torchrun: run N ranks, one per GPU, as
    `python -m torch.distributed.run --nproc-per-node N bench.py <argv>` in a
    CHILD process (never exec: the caller may be a profiler's process) and
    return its exit code.  Called before anything imports torch or touches a
    GPU; the ranks' stdout (rank 0's JSON line) is this process's stdout."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this driver
    return subprocess.call(cmd, env=env)


def resolve_world(args, torchrun):
    """-> the rank count this process belongs to, validating --gpus against
    torchrun's WORLD_SIZE (a mismatch would print an N-GPU line measured on
    a different number of GPUs)."""
    world = int(os.environ.get("WORLD_SIZE", "1")) if torchrun else 1
    if args.gpus is None:
        return world
    if args.gpus < 1:
        raise SystemExit(f"bench.py: --gpus {args.gpus} must be >= 1")
    if torchrun and args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but torchrun started WORLD_SIZE={world} ranks")
    return args.gpus


def dry_run(args):
    """The launcher's rank plumbing with no device work: gloo collective, one
    gathered record per rank, the same aggregation and line shape as the real
    run (value is meaningless and says so)."""
    from hadoofus_amd import shard
    d = shard.Collective("gloo") if shard.launched_by_torchrun() else shard.Local()
    infos = d.gather({"rank": d.rank, "local_rank": d.local, "pid": os.getpid(), "host": socket.gethostname(),
                      "pci_bus_id": f"dry-run:{d.local}"})
    shard.check_distinct_devices(infos)
    scaling, g0, B = shard.workload_blocks(args.config, d.rank, d.world, args.blocks)
    d.barrier()
    tot_bytes, _, ok, t_max = d.aggregate(B * BLOCK, 0, True, 1.0)
    if d.rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "GiB/s", "n_gpus": d.world, "dry_run": True,
                          "scaling": scaling, "ranks": [i["rank"] for i in infos],
                          "pids": [i["pid"] for i in infos], "all_ranks_ok": ok == d.world,
                          "bytes_per_step": tot_bytes, "config": {"workload": args.config}}), flush=True)
    d.close()


def pmc_traffic(kernel, nbytes, chunk):
    """HBM traffic per launch from the committed rocprofv3 PMC passes
    (tools/pmc_traffic.py -> profiles/<round>/pmc_traffic.json, newest round
    last): the measured bytes-per-payload-byte ratio of the same kernel and
    chunk size, scaled to this launch.  None when no profile is committed."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_traffic.json"))):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        k = d.get("kernels", {}).get(kernel)
        if k and d.get("chunk_size") == chunk:
            best = (f, k)
    if not best:
        return None, None
    f, k = best
    return int(k["traffic_bytes_per_payload_byte"] * nbytes), os.path.relpath(f, ROOT)


def cgroup_cpu_limit():
    """CPUs granted by the cgroup v2 quota (cpu.max), or None."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        return None if q == "max" else round(int(q) / int(p), 2)
    except (OSError, ValueError):
        return None


def cpu_baseline(sample_gib):
    """The reference's CPU path timed on this host (rank 0, N=1): its own
    _hdfs_sse42_crc32c (src/crc32c_sse42.c:214-381) compiled from its sources
    (oracle/_ref) when present, else the oracle's SSE4.2 restatement; one
    call per 512 B chunk as _verify_crcdata makes them, one contiguous chunk
    range per thread, on every core of this process's affinity set; the
    single-core leg pinned to one core with sched_setaffinity.  A reported
    baseline, not the target."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ctypes
    from concurrent.futures import ThreadPoolExecutor

    from oracle import Oracle, Reference, have_reference
    o = Oracle()
    affinity = sorted(os.sched_getaffinity(0))
    # Every CPU this process may use: the affinity set, capped by the cgroup
    # CPU quota when one is set (the GPU box grants 16 CPUs of quota while
    # the affinity set names all 256 hardware threads; more threads than the
    # quota only adds throttling).  The affinity-wide run is reported too.
    quota = cgroup_cpu_limit()
    usable = len(affinity) if quota is None else max(1, min(len(affinity), int(quota)))
    threads = min(usable, 256)
    nbytes = max(1, int(sample_gib * (1 << 30)) // BLOCK) * BLOCK
    words = nbytes // 8
    buf = np.empty(words, dtype=np.uint64)
    t0 = time.time()
    parts = min(threads, 64)
    step = (words + parts - 1) // parts
    with ThreadPoolExecutor(parts) as ex:  # ctypes releases the GIL
        list(ex.map(lambda i: o._fill(buf[i * step:].ctypes.data, max(0, min(step, words - i * step)), 0, i * step),
                    range(parts)))
    gen_s = time.time() - t0
    data = buf.view(np.uint8)
    if have_reference():
        ref = Reference()
        fn, ext, kind = "ext", ref.sse42_addr, "reference"
        label = "_hdfs_sse42_crc32c (src/crc32c_sse42.c built from /root/reference)"
        sw_ext, sw_fn, sw_label = ctypes.cast(ref.sw_fn, ctypes.c_void_p).value, "ext", "_hdfs_sw_crc32c (reference)"
    else:
        fn, ext, kind, label = "hw", None, "port", "oracle SSE4.2 3-way restatement"
        sw_ext, sw_fn, sw_label = None, "sw", "oracle slicing-by-8 restatement"

    def timed(fn_, ext_, view, nthreads, budget_s):
        # whole passes over view until budget_s of timed work (>= 1 pass)
        tot, k, first = 0.0, 0, None
        while k == 0 or tot < budget_s:
            s, crcs = o.bench_chunks(view, 512, nthreads, fn_, ext_)
            first = crcs if first is None else first
            tot += s
            k += 1
        return view.nbytes * k / tot / (1 << 30), k, first

    gib = nbytes / (1 << 30)
    # single core, pinned (the calling thread runs the work when nthreads == 1)
    os.sched_setaffinity(0, {affinity[0]})
    try:
        v1, p1, crc1 = timed(fn, ext, data, 1, 3.0)
        # block 0 through the slicing-by-8 SW backend, one core
        v_sw, p_sw, crc_sw = timed(sw_fn, sw_ext, data[:BLOCK], 1, 1.0)
    finally:
        os.sched_setaffinity(0, set(affinity))
    # all usable cores: three repetitions, the median is the value
    reps = [timed(fn, ext, data, threads, 2.0) for _ in range(3)]
    vals = sorted(r[0] for r in reps)
    wide = timed(fn, ext, data, min(len(affinity), 256), 2.0)[0] if usable < len(affinity) else None
    dig = o.crc32c(0, crc1[: BLOCK // 512].view("uint8"), "hw")
    dig_sw = o.crc32c(0, crc_sw.view("uint8"), "hw")
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {
        "value": round(vals[1], 2),
        "unit": "GiB/s",
        "cores": threads,
        "kind": kind,
        "sample": f"{label}; one call per 512 B chunk over {gib:.0f} GiB of splitmix64 blocks "
                  f"0..{nbytes // BLOCK - 1}, {threads} threads (every usable CPU: affinity {len(affinity)}, cgroup quota "
                  f"{quota}) on contiguous chunk ranges, "
                  f"median of 3 repetitions x {min(r[1] for r in reps)}+ passes; single core pinned "
                  f"(sched_setaffinity) {v1:.2f} GiB/s ({p1} passes)",
        "repetitions": [round(v, 2) for v in vals],
        "single_core_value": round(v1, 3),
        "cpu_model": model or platform.processor(),
        "affinity_cpus": len(affinity),
        "affinity_wide_value": round(wide, 2) if wide else None,
        "nproc": os.cpu_count(),
        "cgroup_cpu_limit": cgroup_cpu_limit(),
        "digest_ok": dig == PINNED[(0, 512)],
        "c1_sw_single_core": {"value": round(v_sw, 3), "unit": "GiB/s", "sample":
                              f"{sw_label}; block 0 (128 MiB), 512 B chunks, 1 pinned core, {p_sw} passes",
                              "digest_ok": dig_sw == PINNED[(0, 512)]},
        "datagen_s": round(gen_s, 2),
    }


class Golden:
    """Reference-generated per-block digests (oracle/gen_block_digests.py)."""

    def __init__(self):
        z = np.load(DIGESTS)
        self.be, self.le, self.n = z["be"], z["le"], z["be"].shape[0]

    def check(self, h, crcs_ptr, offs, blocks, sizes):
        """Digest (CRC of the BE CRC array) of each block's CRC array, all in
        one compute launch over the arrays themselves; -> (ok, pinned)."""
        digs = h.DeviceBuffer(4 * len(blocks))
        segs = [h.Segment(data=crcs_ptr + off, len=BLOCK // cs * 4, chunk_size=BLOCK // cs * 4, flags=0, crc_init=0,
                          crcs=digs.ptr + 4 * i) for i, (off, cs) in enumerate(zip(offs, sizes))]
        p = h.Plan(h.MODE_COMPUTE, segs)
        p.execute()
        got = digs.download(dtype=np.uint32)
        p.destroy()
        digs.free()
        ok = pinned = 0
        for i, (g, cs) in enumerate(zip(blocks, sizes)):
            if g < self.n:
                pinned += 1
                ok += int(got[i] == self.be[g, SIZES.index(cs)])
        return ok, pinned


def corrupted(g0, nblocks, per):
    """Global 512-B chunk indices the corruption pattern flips in blocks
    [g0, g0 + nblocks) (chunk i with i % MOD == 0)."""
    start, end = g0 * per, (g0 + nblocks) * per
    first = (start + MOD - 1) // MOD * MOD
    return np.arange(first, end, MOD, dtype=np.int64)


def bitmap_matches(bm_host, nbits_per_block, bad_local):
    """bm_host: concatenated per-block bitmaps; bad_local: (block, chunk) pairs."""
    bits = np.unpackbits(bm_host, bitorder="little")
    want = np.zeros_like(bits)
    for b, c in bad_local:
        want[b * nbits_per_block + c] = 1
    return bool(np.array_equal(bits, want))


def main():
    args = parse()
    from hadoofus_amd import shard  # no torch, no HIP: safe before the launch decision
    torchrun = shard.launched_by_torchrun()
    n_req = resolve_world(args, torchrun)
    if n_req > 1 and not torchrun:
        sys.exit(launch_ranks(n_req, sys.argv[1:]))
    if args.dry_run:
        return dry_run(args)
    # torch (and with it the HIP runtime it ships) is imported before the
    # engine library only when launched as ranks.
    d = shard.Collective("nccl") if torchrun else shard.Local()
    import hadoofus_amd as h

    h.load()
    h.init(d.local)  # explicit binding: this rank's GPU, whatever torch's current device is
    dev, bus = h.bound_device()
    infos = d.gather({"rank": d.rank, "local_rank": d.local, "device": dev, "pci_bus_id": bus,
                      "host": socket.gethostname()})
    ndev = shard.check_distinct_devices(infos)
    arch, ncu = h.device_info()
    cs = args.chunk
    per = BLOCK // cs
    scaling, g0, B = shard.workload_blocks(args.config, d.rank, d.world, args.blocks)
    stream = h.stream_create()
    gblocks = list(range(g0, g0 + B))

    data = h.DeviceBuffer(B * BLOCK)
    crcs = h.DeviceBuffer(B * per * 4)
    bms = h.DeviceBuffer(B * per // 8)
    h.fill_splitmix64(data.ptr, B * BLOCK // 8, 0, g0 << 24, None)

    def segs(chunk_of, crc_ptr, bm_ptr):
        out, off_c = [], 0
        for b, g in enumerate(gblocks):
            c = chunk_of(g)
            n = BLOCK // c
            out.append(h.Segment(data=data.ptr + b * BLOCK, len=BLOCK, chunk_size=c, flags=h.SEG_BE, crc_init=0,
                                 crcs=crc_ptr + off_c * 4, bitmap=(bm_ptr + off_c // 8) if bm_ptr else None))
            off_c += n
        return out

    extra, parity = {}, {}
    golden = Golden()

    # C2: compute-only, 512 B (also the expected wire CRCs of C3).
    comp = h.Plan(h.MODE_COMPUTE, segs(lambda g: cs, crcs.ptr, None))
    for _ in range(2):
        comp.execute(stream)
    h.stream_sync(stream)
    if not args.no_extra:
        comp.set_timing(max(2, args.steps))
        for _ in range(args.steps):
            comp.execute(stream)
        kms_c, nl_c = comp.kernel_ms()
        t_c = kms_c / nl_c * 1e-3
        alg_c = B * BLOCK * (1 + 4 / cs)
        extra["compute_gibps"] = round(B * BLOCK / t_c / (1 << 30), 1)
        extra["compute_roofline"] = {"achieved": round(alg_c / t_c / 1e9, 1), "frac": round(alg_c / t_c / 1e9 /
                                     HBM_PEAK_GBPS, 4), "kernel_avg_ms": round(t_c * 1e3, 3), "launches": nl_c}
    ok, pinned = golden.check(h, crcs.ptr, [b * per * 4 for b in range(B)], gblocks, [cs] * B)
    parity["c2_block_digests_ok"] = f"{ok}/{pinned}" + ("" if pinned == B else f" ({B - pinned} beyond the golden set)")
    c2_ok = ok == pinned

    # C5: mixed bytesPerChecksum in one launch, computed on CLEAN data.
    c5_of = lambda g: 512 << (g % 4)  # noqa: E731
    c5_sizes = [c5_of(g) for g in gblocks]
    c5_offs = np.concatenate([[0], np.cumsum([BLOCK // c for c in c5_sizes])])  # chunk offsets
    crcs5 = bms5 = None
    c5_ok = True
    if not args.no_extra:
        crcs5 = h.DeviceBuffer(int(c5_offs[-1]) * 4)
        bms5 = h.DeviceBuffer(int(c5_offs[-1]) // 8)
        mixc = h.Plan(h.MODE_COMPUTE, segs(c5_of, crcs5.ptr, None))
        mixc.execute(stream)
        h.stream_sync(stream)
        mixc.destroy()
        ok5, pinned5 = golden.check(h, crcs5.ptr, [int(o) * 4 for o in c5_offs[:-1]], gblocks, c5_sizes)
        parity["c5_block_digests_ok"] = f"{ok5}/{pinned5}"
        c5_ok = ok5 == pinned5

    # Corrupt 1 in 65537 chunks (global 512-B chunk index), then verify.
    for b, g in enumerate(gblocks):
        h.corrupt(data.ptr + b * BLOCK, BLOCK, cs, g * per, MOD, BITMUL, None)
    h.device_sync()
    bad = corrupted(g0, B, per)
    bad_local = [(int(i // per) - g0, int(i % per)) for i in bad]
    expect_bad = len(bad)
    expect_first = {b: c for b, c in reversed(bad_local)}

    ver = h.Plan(h.MODE_VERIFY, segs(lambda g: cs, crcs.ptr, bms.ptr))
    for _ in range(args.warmup):
        ver.execute(stream)
    h.stream_sync(stream)
    _, m = ver.results(stream)
    parity_ok = m == expect_bad

    ver.set_timing(max(2, args.steps))
    d.barrier()
    h.stream_sync(stream)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ver.execute(stream)
    h.stream_sync(stream)
    d.barrier()
    t1 = time.perf_counter()
    kms, nlaunch = ver.kernel_ms()
    first_bad, m = ver.results(stream)
    parity_ok &= m == expect_bad
    parity_ok &= all(first_bad[b] == expect_first.get(b, 0xFFFFFFFF) for b in range(B))
    c3_bitmap_ok = bitmap_matches(bms.download(), per, bad_local)
    parity_ok &= c3_bitmap_ok and c2_ok
    elapsed = t1 - t0

    if not args.no_extra:
        # C5 verify on the corrupted data against the clean mixed CRCs: every
        # corrupted 512-B chunk lies in exactly one C5 chunk (32 MiB apart).
        mixv = h.Plan(h.MODE_VERIFY, segs(c5_of, crcs5.ptr, bms5.ptr))
        mixv.execute(stream)
        mixv.set_timing(max(2, args.steps // 2))
        for _ in range(max(2, args.steps // 2)):
            mixv.execute(stream)
        kms5, nl5 = mixv.kernel_ms()
        fb5, mm = mixv.results(stream)
        bad5 = [(b, c * 512 // c5_sizes[b]) for b, c in bad_local]
        bits5 = np.unpackbits(bms5.download(), bitorder="little")
        want5 = np.zeros_like(bits5)
        for b, c in bad5:
            want5[c5_offs[b] + c] = 1
        first5 = {b: c for b, c in reversed(bad5)}
        c5v_ok = (mm == len(bad5) and bool(np.array_equal(bits5, want5)) and
                  all(fb5[b] == first5.get(b, 0xFFFFFFFF) for b in range(B)))
        extra["mixed_verify_gibps"] = round(B * BLOCK / (kms5 / nl5 * 1e-3) / (1 << 30), 1)
        parity["c5_mismatches"] = int(mm)
        parity["c5_expected"] = len(bad5)
        parity["c5_bitmap_ok"] = c5v_ok
        parity_ok &= c5v_ok and c5_ok
        mixv.destroy()

    # Empirical ceiling: the verify kernel's load-only twin (identical loads
    # and store instructions, no CRC arithmetic) from the diagnostic build,
    # same process, same data and segment table.
    ceiling = None
    if not args.no_extra:
        try:
            sys.path.insert(0, os.path.join(ROOT, "tools"))
            import diaglib
            dg = diaglib.Diag()
            dg.init(d.local)
            dg.set_store_policy(4)
            twin = dg.plan(h.MODE_VERIFY, segs(lambda g: cs, crcs.ptr, bms.ptr))
            twin.execute(stream)
            twin.set_timing(max(2, args.steps // 2))
            for _ in range(max(2, args.steps // 2)):
                twin.execute(stream)
            kt, nt = twin.kernel_ms()
            twin.destroy()
            dg.set_store_policy(0)
            alg_t = B * BLOCK * (1 + 4 / cs + 1 / (8 * cs))
            cands = {"load-only twin of crc32c_tiles_kernel<verify>": alg_t / (kt / nt * 1e-3) / 1e9}
            # streaming-read probes (crc32c_probes.hip): nontemporal buffer
            # loads, grid-interleaved (14) or XCD-major (24), LDS-DMA per-
            # workgroup slices (17, 18: round 1's best, 7230 GB/s at 4 x 256
            # threads per CU) or XCD-major (26), and software-pipelined like
            # the tiled kernel (30-32: 4 or 8 KiB rounds, 3-4 deep), over the
            # same 128 GiB; best of 2 x 2
            for var in (14, 17, 18, 24, 26, 30, 31, 32):
                for gpc, blk in ((1, 1024), (2, 512), (4, 256)):
                    dg.set_probe(var, gpc, blk)
                    g = max(dg.probe_read(data.ptr, B * BLOCK, 2, stream) for _ in range(2))
                    cands[f"read probe {var} ({gpc}x{blk} per CU)"] = g
            dg.set_probe()
            extra["ceiling_candidates_GBps"] = {k: round(v, 1) for k, v in cands.items()}
            # a "ceiling" above the HBM spec means the diagnostic kernel skipped
            # work (e.g. the compiler deleted unused loads): never report it
            bad = {k for k, v in cands.items() if v > HBM_PEAK_GBPS}
            if bad:
                extra["ceiling_rejected_above_spec"] = sorted(bad)
            cands = {k: v for k, v in cands.items() if k not in bad}
            if cands:
                best = max(cands, key=cands.get)
                ceiling = cands[best]
                extra["ceiling_GBps"] = round(ceiling, 1)
                extra["ceiling_source"] = best + " (libhadoofus_crc32c_diag.so, same process)"
        except (ImportError, OSError) as e:
            extra["ceiling_error"] = str(e)[:200]

    # C4 strong scaling predicted on one GPU: the verify
    # kernel time of the whole 64 GiB workload (512 blocks) and of one rank's
    # shard at 2 / 4 / 8 ranks (256 / 128 / 64 blocks), same process; the
    # speed-up bound at N ranks is T(512) / T(512 / N) -- independent chunks,
    # no exchange (src/datanode.c:2945-2954), so launch ramp and tail are
    # what the shard size changes.
    if d.world == 1 and not args.no_extra and B >= 64:
        shard_ms = {}
        for nb in (512, 256, 128, 64):
            if nb > B:
                continue
            sp = h.Plan(h.MODE_VERIFY, segs(lambda g: cs, crcs.ptr, bms.ptr)[:nb])
            sp.execute(stream)
            h.stream_sync(stream)
            sp.set_timing(10)
            for _ in range(10):
                sp.execute(stream)
            k_ms, k_n = sp.kernel_ms()
            sp.destroy()
            shard_ms[nb] = k_ms / k_n
        extra["c4_shard_ms"] = {f"blocks_{k}": round(v, 3) for k, v in shard_ms.items()}
        if 512 in shard_ms:
            extra["c4_speedup_bound"] = {f"{g}gpu": round(shard_ms[512] / shard_ms[512 // g], 3)
                                         for g in (2, 4, 8) if 512 // g in shard_ms}

    # C4 strong scaling beside the weak-scaled headline when N > 1
    # (BASELINE.json configs[3]: 64 GiB for the whole node, split evenly):
    # each rank verifies its 512 / N share, taken from the front of its
    # resident blocks, timed between barriers, max over ranks.
    c4 = None
    if d.world > 1 and args.config == "C3" and not args.no_extra:
        nb4 = min(shard.split_blocks(512, d.rank, d.world)[1], B)
        sp = h.Plan(h.MODE_VERIFY, segs(lambda g: cs, crcs.ptr, bms.ptr)[:nb4])
        sp.execute(stream)
        h.stream_sync(stream)
        k4 = max(2, args.steps)
        d.barrier()
        h.stream_sync(stream)
        t4 = time.perf_counter()
        for _ in range(k4):
            sp.execute(stream)
        h.stream_sync(stream)
        d.barrier()
        t4 = time.perf_counter() - t4
        _, m4 = sp.results(stream)
        sp.destroy()
        want4 = sum(1 for b, _c in bad_local if b < nb4)
        b4, mm4, ok4, tmax4 = d.aggregate(nb4 * BLOCK * k4, m4, m4 == want4, t4)
        c4 = {"workload": "C4 strong: 512 x 128MiB blocks (64 GiB) split evenly over the GPUs, verify, 512B chunks",
              "GiBps": round(b4 / tmax4 / (1 << 30), 1), "total_bytes_per_step": int(b4 / k4),
              "blocks_rank0": nb4, "ms_per_step": round(tmax4 / k4 * 1e3, 3), "steps": k4,
              "mismatches": int(mm4), "all_ranks_ok": ok4 == d.world}

    tot_bytes, tot_mism, ok, t_max = d.aggregate(B * BLOCK * args.steps, m, parity_ok, elapsed)
    n = d.world
    if c4:
        extra["c4_strong"] = c4

    if d.rank == 0:
        gib_s = tot_bytes / t_max / (1 << 30)
        nbytes = B * BLOCK
        alg = nbytes + 4 * nbytes / cs + nbytes / (8 * cs)  # data + expected CRCs + bitmap
        k_avg_s = kms / max(1, nlaunch) * 1e-3
        achieved = alg / k_avg_s / 1e9
        traffic, traffic_src = pmc_traffic("verify", nbytes, cs)
        # an empirical ceiling bounds the kernel only if it is at least the
        # kernel's own rate; a slower "ceiling" (round 2: the load-only twin
        # and every read probe below the verify kernel) is reported as a
        # candidate, never as the peak
        peak_ok = bool(ceiling) and ceiling >= achieved
        if ceiling and not peak_ok:
            extra["measured_peak_note"] = (
                f"no ceiling candidate measured in this process ({round(ceiling, 1)} GB/s at best, "
                f"{extra.get('ceiling_source', '')}) reaches the verify kernel's own {round(achieved, 1)} GB/s, "
                "so no empirical peak is reported; frac is against the 8 TB/s spec only")
        if args.config == "C3":
            workload = (f"C3 verify: {B} x 128MiB HDFS blocks per GPU of splitmix64 data, 512B chunks, BE wire CRCs, "
                        "1/65537 chunks corrupted, bitmap + first-bad out"
                        + (f"; weak scaling over {n} GPUs ({n * B} blocks in all)" if n > 1 else ""))
        else:
            workload = ("C4 verify: 64GiB (512 x 128MiB blocks) split evenly over the GPUs, 512B chunks, BE wire CRCs, "
                        "1/65537 chunks corrupted, bitmap + first-bad out"
                        + (f"; strong scaling over {n} GPUs" if n > 1 else ""))
        line = {
            "metric": METRIC,
            "value": round(gib_s, 1),
            "unit": "GiB/s",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_max / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {
                "workload": workload, "blocks_per_gpu": B, "block_bytes": BLOCK, "chunk_size": cs,
                "bytes_per_gpu_per_step": nbytes, "parallelism": f"shard{n}",
            },
            "roofline": {
                "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                "traffic_unit": "bytes/launch", "traffic_source": traffic_src,
                "frac_of_measured_peak": round(achieved / ceiling, 4) if peak_ok else None,
                "measured_peak": round(ceiling, 1) if peak_ok else None,
                "kernel": "crc32c_tiles_kernel<verify>", "kernel_avg_ms": round(k_avg_s * 1e3, 3),
                "alg_bytes_per_launch": int(alg),
            },
            "parity": dict({"mismatches": int(tot_mism), "expected_per_gpu": int(expect_bad),
                            "all_ranks_ok": ok == n, "c3_bitmap_ok": c3_bitmap_ok}, **parity),
            "device": {"arch": arch, "cus": ncu, "ranks_on_distinct_gpus": ndev,
                       "pci_bus_ids": [i["pci_bus_id"] for i in infos]},
            "extra": extra,
        }
        if n == 1 and not args.no_extra:
            # the packet-stream path on HBM-resident runs (1 GiB, one 128 MiB
            # block) beside a plan over the same packets, and the host-resident
            # rates (the datanode's socket buffers are host memory: PCIe-bound)
            sys.path.insert(0, os.path.join(ROOT, "tools"))
            try:
                import device_stream_bench
                extra["device_stream"] = device_stream_bench.block_and_run(plan_GiBps=gib_s)
            except Exception as e:  # reported, never fatal to the headline line
                extra["device_stream_error"] = repr(e)[:300]
            # the same stream of blocks from a C caller (a datanode's view,
            # no Python between the calls): tools/probes/jobs_bench.c
            exe = os.path.join(ROOT, "tools", "probes", "jobs_bench")
            # (16 blocks, as the Python stream above; and 64, where a stream's
            # first and last lone launches weigh a quarter as much)
            if os.path.exists(exe) and "device_stream" in extra:
                for nb, key in ((16, "stream_of_blocks_c"), (64, "stream_of_64_blocks_c")):
                    try:
                        import subprocess
                        r = subprocess.run([exe, str(nb)], capture_output=True, text=True, timeout=180)
                        c = json.loads(r.stdout.strip().splitlines()[-1])
                        for k, us in c["us_per_block"].items():
                            c.setdefault("frac_of_headline", {})[k] = round((2048 * 65536) / (us * 1e-6) / (1 << 30) / gib_s, 3)
                        extra["device_stream"]["block_128MiB"][key] = c
                    except Exception as e:  # reported, never fatal to the headline line
                        extra["device_stream"][key + "_error"] = repr(e)[:300]
            try:
                import h2d_bench
                hr = h2d_bench.measure(8 << 30, (64,), 3)
                if "device_stream" in extra:
                    hr["packets_1GiB_pinned_GiBps"] = extra["device_stream"]["run_1GiB"].get("host_pinned_GiBps")
                extra["host_resident"] = hr
            except Exception as e:
                extra["host_resident_error"] = repr(e)[:300]
        if n == 1 and not args.no_cpu:
            line["cpu_baseline"] = cpu_baseline(args.cpu_gib)
            if "host_resident" in extra:
                extra["host_resident"]["vs_cpu_baseline"] = round(
                    extra["host_resident"]["pinned_verify_GiBps_piece64MiB"] / line["cpu_baseline"]["value"], 3)
        print(json.dumps(line), flush=True)
    d.close()


if __name__ == "__main__":
    main()
