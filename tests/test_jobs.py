"""Asynchronous verify jobs (round 5): hdfs_crc32c_verify_packets_submit /
hdfs_crc32c_job_wait on device-resident packet streams.  Every job's result
equals the oracle's verify (oracle_verify_packets: src/datanode.c:2345-2494,
2931-2963) -- records, verdicts, consumed bytes, status -- whether the
speculative launch at submit took the run, handed it back (a header off the
run), was never tried (no run of whole-chunk packets, a short stream), or
took only part of it (more packets than one pass, another size after it);
with four jobs in flight at once, waited in any order, and with synchronous
calls in between.  Jobs submitted while a launch runs share one batch
launch (round 6): a stream of 16 blocks, one job each, is verified in a
few launches, every job's result still the oracle's."""
import numpy as np
import pytest

from packet_stream import CSUM_CRC32, CSUM_CRC32C, build_stream

BAD = 29


def _dev(engine, s, shift=0):
    buf = engine.DeviceBuffer(len(s) + shift + 64)
    buf.fill(0)
    buf.upload(np.frombuffer(s, np.uint8), offset=shift)
    engine.device_sync()
    return buf, buf.ptr + shift


def _cases(oracle):
    out = []
    rng = np.random.default_rng(41)

    def add(name, proto, cs, ctype, dl, **kw):
        corrupt = sorted({(int(k), int(rng.integers(0, max(1, dl[k] // cs)))) for k in rng.integers(0, len(dl), 4)})
        s, _ = build_stream(oracle.crc32c, proto, cs, ctype, dl, seed=len(dl) + cs, corrupt=corrupt, **kw)
        out.append((name, proto, cs, ctype, s))

    add("v2_block", 2, 512, CSUM_CRC32C, [65536] * 128)
    add("v1_crc32", 1, 512, CSUM_CRC32, [65536] * 100, last_empty=False)
    add("v2_size_break", 2, 512, CSUM_CRC32C, [65536] * 60 + [30000] + [65536] * 40)
    add("v2_other_size_after_run", 2, 512, CSUM_CRC32C, [65536] * 80 + [4096] * 30)
    add("v2_many_exceptions", 2, 512, CSUM_CRC32C, [65536] * 100, seqnos=[3 * k for k in range(100)])
    add("v2_partial_chunks_not_eligible", 2, 512, CSUM_CRC32C, [40000] * 200)
    add("v2_short_stream", 2, 512, CSUM_CRC32C, [65536] * 20)
    add("v2_cs4096", 2, 4096, CSUM_CRC32C, [65536] * 100)
    s, _ = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, [65536] * 90, seed=9)
    w = oracle.verify_packets(s)[1]
    out.append(("v2_cut_in_next", 2, 512, CSUM_CRC32C, s[:w[-1]["stream_off"] - 1000]))
    bad_tail = bytearray(s)
    e = w[-1]["stream_off"]
    bad_tail[e:e + 4] = (0x7FFFFFFF).to_bytes(4, "big")  # plen > 1 GiB: PACKET_SIZE
    out.append(("v2_framing_error_tail", 2, 512, CSUM_CRC32C, bytes(bad_tail)))
    return out


@pytest.mark.gpu
def test_gpu_jobs_vs_oracle(engine, oracle):
    """Four jobs in flight, waited in reverse order, then the next four: each
    equals the oracle's verify and the synchronous call's."""
    cases = _cases(oracle)
    bufs = [_dev(engine, c[4], i % 3) for i, c in enumerate(cases)]
    want = [oracle.verify_packets(c[4], c[1], c[2], c[3]) for c in cases]
    for i0 in range(0, len(cases), 4):
        idx = list(range(i0, min(i0 + 4, len(cases))))
        jobs = {i: engine.VerifyJob(bufs[i][1], len(cases[i][4]), cases[i][1], cases[i][2], cases[i][3]) for i in idx}
        for i in reversed(idx):
            got = jobs[i].wait()
            assert got == want[i], cases[i][0]
            assert engine.verify_packets(None, cases[i][1], cases[i][2], cases[i][3], dptr=bufs[i][1],
                                         nbytes=len(cases[i][4])) == want[i], cases[i][0]
    for b, _ in bufs:
        b.free()


@pytest.mark.gpu
def test_gpu_jobs_many_passes(engine, oracle):
    """70 000 packets of 2 KiB: the launch at submit takes the first 65 536,
    the wait verifies the rest (a second speculative launch) and the 1 000-B
    tail packet; corruption on both sides of the pass edge."""
    dl = [2048] * 70000 + [1000]
    s, _ = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, dl, seed=77,
                        corrupt=[(5, 0), (65535, 3), (65536, 2), (69999, 1)])
    mp = len(dl) + 2
    want = oracle.verify_packets(s, max_pkts=mp)
    keep, p = _dev(engine, s)
    assert engine.VerifyJob(p, len(s), max_pkts=mp).wait() == want
    # max_pkts inside the first pass: the records stop there, as the synchronous call's
    w2 = oracle.verify_packets(s, max_pkts=1000)
    assert engine.VerifyJob(p, len(s), max_pkts=1000).wait() == w2
    keep.free()


@pytest.mark.gpu
def test_gpu_jobs_limit_and_interleaving(engine, oracle):
    """A 65th job while 64 are outstanding is refused (and the 64 still
    complete correctly); synchronous verifies and reads run between a submit
    and its wait; a waited job makes room for a new one."""
    dl = [65536] * 100
    s, _ = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, dl, seed=3, corrupt=[(50, 7)])
    want = oracle.verify_packets(s)
    bufs = [_dev(engine, s, i) for i in range(5)]
    jobs = [engine.VerifyJob(bufs[i % 4][1], len(s)) for i in range(64)]
    with pytest.raises(engine.CRC32CError):
        engine.VerifyJob(bufs[4][1], len(s))
    for j in jobs[4:]:
        assert j.wait() == want
    jobs = jobs[:4]
    # synchronous calls while the jobs are in flight
    assert engine.verify_packets(None, dptr=bufs[4][1], nbytes=len(s)) == want
    dst = engine.DeviceBuffer(sum(dl))
    rd = engine.read_packets(bufs[4][1], len(s), dst.ptr, sum(dl), client_offset=0, read_len=sum(dl))
    wr = oracle.read_packets(s, 0, sum(dl))
    assert rd[:3] == wr[:3] and dst.download(rd[3]).tobytes() == wr[3]
    assert jobs[1].wait() == want
    j5 = engine.VerifyJob(bufs[4][1], len(s))
    for j in (jobs[0], jobs[2], jobs[3], j5):
        assert j.wait() == want
    dst.free()
    for b, _ in bufs:
        b.free()


# --- batches of blocks in one launch (hdfs_crc32c_verify_blocks_submit) -------
def _block(oracle, k, dl=None, proto=2, ctype=CSUM_CRC32C, corrupt=(), **kw):
    """Block k of a file: 64 KiB packets from offsetInBlock 0, the empty last
    packet, its own data."""
    dl = dl or [65536] * 100
    s, _ = build_stream(oracle.crc32c, proto, 512, ctype, dl, seed=100 + k, corrupt=corrupt, **kw)
    return s


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["equal", "corrupt_and_exceptions", "unequal_counts", "short_last_block",
                                  "one_irregular", "v1_crc32", "single", "sixteen"])
def test_gpu_blocks_vs_oracle(engine, oracle, case):
    """Each block's records, verdicts, consumed bytes and status equal the
    oracle's verify of that block, whether the batch launch took every block
    (equal layouts and counts), or none (a block of another packet count or
    size, an irregular block: each then verified on its own in the wait)."""
    kw = {}
    if case == "equal":
        streams = [_block(oracle, k) for k in range(4)]
    elif case == "corrupt_and_exceptions":
        streams = [_block(oracle, 0, corrupt=[(3, 1), (99, 127)]), _block(oracle, 1),
                   _block(oracle, 2, seqnos=[k + (5 if k > 40 else 0) for k in range(100)], corrupt=[(64, 0)]),
                   _block(oracle, 3, offset_skew={10: 512})]
    elif case == "unequal_counts":  # the launch takes blocks 0 and 2 (one length), block 1 in the wait
        streams = [_block(oracle, 0), _block(oracle, 1, dl=[65536] * 90), _block(oracle, 2)]
    elif case == "short_last_block":
        streams = [_block(oracle, k) for k in range(5)] + [_block(oracle, 5, dl=[65536] * 7 + [1000])]
    elif case == "one_irregular":
        streams = [_block(oracle, 0), _block(oracle, 1, dl=[65536] * 50 + [30000] + [65536] * 49),
                   _block(oracle, 2)]
    elif case == "v1_crc32":
        streams = [_block(oracle, k, proto=1, ctype=CSUM_CRC32, last_empty=False) for k in range(3)]
        kw = {"proto": 1, "ctype": CSUM_CRC32}
    elif case == "single":
        streams = [_block(oracle, 0, corrupt=[(7, 7)])]
    else:
        streams = [_block(oracle, k, corrupt=[(k, k)] if k % 5 == 0 else []) for k in range(16)]
    proto, ctype = kw.get("proto", 2), kw.get("ctype", CSUM_CRC32C)
    bufs = [_dev(engine, st, k % 3) for k, st in enumerate(streams)]
    want = [oracle.verify_packets(st, proto, 512, ctype) for st in streams]
    job = engine.VerifyBlocksJob([(p, len(st)) for (_, p), st in zip(bufs, streams)], proto, 512, ctype)
    rc, got = job.wait()
    for b in range(len(streams)):
        assert got[b] == want[b], (case, b)
    first = next((w[0] for w in want if w[0]), 0)
    assert rc == first
    for bb, _ in bufs:
        bb.free()


@pytest.mark.gpu
def test_gpu_blocks_taken_in_one_launch(engine, oracle):
    """The diagnostic build's counters: a batch of four equal blocks is one
    speculative launch, eligible and taken."""
    import ctypes
    from hadoofus_amd import abi, build
    diag = abi.bind_diag(abi.bind_product(ctypes.CDLL(build.DIAG_LIB)))
    streams = [_block(oracle, k, corrupt=[(k, 0)]) for k in range(4)]
    bufs = [_dev(engine, st) for st in streams]
    out = (ctypes.c_uint64 * 4)()
    diag.hdfs_crc32c_diag_spec_stats(out, 1)
    rc, got = engine.VerifyBlocksJob([(p, len(st)) for (_, p), st in zip(bufs, streams)], lib=diag).wait()
    assert diag.hdfs_crc32c_diag_spec_stats(out, 1) == 0
    assert tuple(out) == (1, 1, 1, 0), tuple(out)
    assert [g for g in got] == [oracle.verify_packets(st) for st in streams]
    # a short last block: the launch still takes the four equal ones
    last = _block(oracle, 9, dl=[65536] * 5 + [777])
    lb = _dev(engine, last)
    diag.hdfs_crc32c_diag_spec_stats(out, 1)
    rc, got = engine.VerifyBlocksJob([(p, len(st)) for (_, p), st in zip(bufs, streams)] + [(lb[1], len(last))],
                                     lib=diag).wait()
    diag.hdfs_crc32c_diag_spec_stats(out, 1)
    assert tuple(out)[:3] == (1, 1, 1), tuple(out)
    assert got == [oracle.verify_packets(st) for st in streams + [last]]
    lb[0].free()
    for bb, _ in bufs:
        bb.free()


def _diag():
    import ctypes
    from hadoofus_amd import abi, build
    return abi.bind_diag(abi.bind_product(ctypes.CDLL(build.DIAG_LIB)))


@pytest.mark.gpu
@pytest.mark.parametrize("order", ["in_order", "reverse", "window4"])
def test_gpu_jobs_coalesce_stream_of_blocks(engine, oracle, order):
    """A datanode's stream of 16 received blocks, one job per block, with a
    bad packet in block 9 (and an irregular header in block 12, which voids
    the batch launch it lands in: those blocks are verified one by one in
    their waits): every job equals the oracle's verify of its block.  Jobs
    submitted while a launch runs go out together, so 16 jobs submitted back
    to back take at most 3 launches (the first alone, the rest as batches)."""
    diag = _diag()
    streams = [_block(oracle, k, corrupt=[(61, 5)] if k == 9 else [],
                      **({"seqnos": [k2 + (3 if k2 > 70 else 0) for k2 in range(100)]} if k == 12 else {}))
               for k in range(16)]
    bufs = [_dev(engine, st, k % 2) for k, st in enumerate(streams)]
    want = [oracle.verify_packets(st) for st in streams]
    assert want[9][0] == BAD and want[12][0] == 0
    out = (__import__("ctypes").c_uint64 * 4)()
    diag.hdfs_crc32c_diag_spec_stats(out, 1)
    got = {}
    if order == "window4":  # at most 4 outstanding: wait for the oldest before the next submit
        q = []
        for k, ((_, p), st) in enumerate(zip(bufs, streams)):
            if len(q) == 4:
                k0, j0 = q.pop(0)
                got[k0] = j0.wait()
            q.append((k, engine.VerifyJob(p, len(st), lib=diag)))
        for k0, j0 in q:
            got[k0] = j0.wait()
    else:
        jobs = [engine.VerifyJob(p, len(st), lib=diag) for (_, p), st in zip(bufs, streams)]
        for k in (range(16) if order == "in_order" else reversed(range(16))):
            got[k] = jobs[k].wait()
    diag.hdfs_crc32c_diag_spec_stats(out, 1)
    for k in range(16):
        assert got[k] == want[k], (order, k)
    launches = out[0]
    if order != "window4":
        # the first job alone, the other 15 in one batch -- plus the single
        # passes of the blocks of a batch that block 12 voided
        assert launches <= 2 + 15, tuple(out)
        assert out[2] >= 1, tuple(out)  # a launch was taken
    for bb, _ in bufs:
        bb.free()


@pytest.mark.gpu
@pytest.mark.parametrize("mode,want_launches", [(2, 1), (0, 16)])
def test_gpu_jobs_coalesce_counts_launches(engine, oracle, mode, want_launches):
    """16 clean equal blocks submitted back to back (diagnostic build).  Hold
    mode (2: queue even on an idle GPU, so the count does not depend on how
    fast the host submits): the 16th submit fills the queue and all 16 go out
    as ONE batch launch, taken.  Mode 0 (the round-5 path): one launch per
    job.  Every result the oracle's either way."""
    diag = _diag()
    streams = [_block(oracle, k) for k in range(16)]
    bufs = [_dev(engine, st) for st in streams]
    want = [oracle.verify_packets(st) for st in streams]
    out = (__import__("ctypes").c_uint64 * 4)()
    assert diag.hdfs_crc32c_set_job_coalesce(mode) == 0
    try:
        diag.hdfs_crc32c_diag_spec_stats(out, 1)
        jobs = [engine.VerifyJob(p, len(st), lib=diag) for (_, p), st in zip(bufs, streams)]
        got = [j.wait() for j in jobs]
        diag.hdfs_crc32c_diag_spec_stats(out, 1)
    finally:
        diag.hdfs_crc32c_set_job_coalesce(1)
    assert got == want
    assert tuple(out)[:3] == (want_launches,) * 3, tuple(out)
    for bb, _ in bufs:
        bb.free()


@pytest.mark.gpu
def test_gpu_jobs_hold_flushes_at_wait(engine, oracle):
    """Hold mode, 5 jobs queued: the first wait sends all 5 out as one launch,
    whichever job it is for; then 3 more jobs of another length (a key
    change sends nothing out by itself while the queue is empty) go out at
    their first wait."""
    diag = _diag()
    a = [_block(oracle, k, corrupt=[(k, 1)]) for k in range(5)]
    b = [_block(oracle, 10 + k, dl=[65536] * 80) for k in range(3)]  # (> 64 packets: not a short run)
    bufs = [_dev(engine, st) for st in a + b]
    want = [oracle.verify_packets(st) for st in a + b]
    out = (__import__("ctypes").c_uint64 * 4)()
    assert diag.hdfs_crc32c_set_job_coalesce(2) == 0
    try:
        diag.hdfs_crc32c_diag_spec_stats(out, 1)
        ja = [engine.VerifyJob(p, len(st), lib=diag) for (_, p), st in zip(bufs[:5], a)]
        assert ja[3].wait() == want[3]
        diag.hdfs_crc32c_diag_spec_stats(out, 0)
        assert out[0] == 1, tuple(out)
        jb = [engine.VerifyJob(p, len(st), lib=diag) for (_, p), st in zip(bufs[5:], b)]
        for k in (0, 1, 2, 4):
            assert ja[k].wait() == want[k], k
        for k in (2, 0, 1):
            assert jb[k].wait() == want[5 + k], k
        diag.hdfs_crc32c_diag_spec_stats(out, 1)
    finally:
        diag.hdfs_crc32c_set_job_coalesce(1)
    assert tuple(out)[:3] == (2, 2, 2), tuple(out)
    for bb, _ in bufs:
        bb.free()


@pytest.mark.gpu
def test_gpu_jobs_coalesce_mixed_keys(engine, oracle):
    """Jobs of alternating lengths and chunk sizes (each key change sends the
    queue out), a short last block and a CRC32 v1 block among them, waited
    out of order: each equals the oracle's verify."""
    specs = []
    for k in range(12):
        if k % 4 == 3:
            specs.append((_block(oracle, k, dl=[65536] * 7 + [1000]), 2, 512, CSUM_CRC32C))
        elif k % 4 == 2:
            specs.append((_block(oracle, k, proto=1, ctype=CSUM_CRC32, last_empty=False, corrupt=[(3, 3)]),
                          1, 512, CSUM_CRC32))
        else:
            specs.append((_block(oracle, k, dl=[65536] * (100 if k % 2 else 80)), 2, 512, CSUM_CRC32C))
    bufs = [_dev(engine, st, k % 3) for k, (st, *_r) in enumerate(specs)]
    want = [oracle.verify_packets(st, pr, cs, ct) for st, pr, cs, ct in specs]
    jobs = [engine.VerifyJob(p, len(st), pr, cs, ct) for (_, p), (st, pr, cs, ct) in zip(bufs, specs)]
    for k in [5, 0, 11, 3, 1, 2, 4, 6, 10, 9, 8, 7]:
        assert jobs[k].wait() == want[k], k
    for bb, _ in bufs:
        bb.free()
