"""Per-run completion of coalesced batches (round 6).  Jobs queued while a
launch runs go out as one batch launch of up to 16 runs; each run's
completion is published on its own (the workgroups count the tiles they own
of each run, and the header groups of the run count too), so a job whose run
is done, verified clean and in the prediction returns while the launch still
verifies the runs after it -- a datanode with 4 blocks outstanding keeps the
GPU fed with batches instead of a batch and a lone run.  The wait on a
launch's last run sends the queue out and collects the launch, as before; a
run with a bad chunk, a header off the prediction or tiles in the launch's
global pool is left to the launch's final block.

Every job's result equals the oracle's verify of its block
(oracle_verify_packets: src/datanode.c:2345-2494, 2931-2963) with per-run
completion on and off, under every dealing of the tiles over the workgroups
the kernel has (XCD-major, plain, XCD-split; groups of 1, 8 and 16 tiles),
with bad chunks at the first and at the last tile of a run, and with the
pool taking part of the batch.  The diagnostic build checks on the device
that each workgroup verified exactly the tiles the kernel said it owns of
each published run (a count too low would publish a run before its last
tiles): no check fires."""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from packet_stream import CSUM_CRC32, CSUM_CRC32C, build_stream

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _diag():
    from hadoofus_amd import abi, build
    return abi.bind_diag(abi.bind_product(ctypes.CDLL(build.DIAG_LIB)))


def _block(oracle, k, n=100, corrupt=()):
    s, _ = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, [65536] * n, seed=300 + k, corrupt=list(corrupt))
    return s


def _dev(engine, s):
    buf = engine.DeviceBuffer(len(s) + 64)
    buf.upload(np.frombuffer(s, np.uint8))
    engine.device_sync()
    return buf


def _checks(diag):
    out = (ctypes.c_uint32 * 3)()
    assert diag.hdfs_crc32c_diag_device_checks(out, 1) == 0
    return tuple(out)


def _early(diag):
    out = (ctypes.c_uint64 * 2)()
    assert diag.hdfs_crc32c_diag_job_early(out, 1) == 0
    return tuple(out)


def _run_held(engine, diag, streams, order):
    """Hold mode: every job queued, the first wait sends them out as one
    batch; the waits in `order`."""
    bufs = [_dev(engine, s) for s in streams]
    assert diag.hdfs_crc32c_set_job_coalesce(2) == 0
    try:
        jobs = [engine.VerifyJob(b.ptr, len(s), lib=diag) for b, s in zip(bufs, streams)]
        got = {k: jobs[k].wait() for k in order}
    finally:
        diag.hdfs_crc32c_set_job_coalesce(1)
    for b in bufs:
        b.free()
    return got


@pytest.mark.gpu
@pytest.mark.parametrize("xcd,gshift", [(1, 3), (0, 3), (2, 3), (1, 0), (1, 4)])
def test_gpu_jobs_per_run_dealings(engine, oracle, xcd, gshift):
    """Six blocks in one batch, bad chunks at the last tile of block 1 and at
    the first tile of block 4, under each tile dealing: every job the
    oracle's, no device check."""
    diag = _diag()
    streams = [_block(oracle, k, corrupt=[(99, 127)] if k == 1 else [(0, 0)] if k == 4 else []) for k in range(6)]
    want = [oracle.verify_packets(s) for s in streams]
    assert want[1][0] != 0 and want[4][0] != 0 and want[0][0] == 0
    assert diag.hdfs_crc32c_set_xcd_major(xcd) == 0 and diag.hdfs_crc32c_set_group_shift(gshift) == 0
    try:
        _checks(diag)
        _early(diag)
        got = _run_held(engine, diag, streams, range(6))
        early = _early(diag)
        checks = _checks(diag)
    finally:
        diag.hdfs_crc32c_set_xcd_major(1)
        diag.hdfs_crc32c_set_group_shift(3)
    for k in range(6):
        assert got[k] == want[k], (xcd, gshift, k)
    assert checks == (0, 0, 0), checks
    assert sum(early) <= 5, early  # (the last run's wait collects the launch)


@pytest.mark.gpu
@pytest.mark.parametrize("proto,cs,ctype,last_empty", [(2, 4096, CSUM_CRC32C, True), (2, 1024, CSUM_CRC32, True),
                                                       (1, 512, CSUM_CRC32, False), (2, 2048, CSUM_CRC32C, True)])
def test_gpu_jobs_per_run_layouts(engine, oracle, proto, cs, ctype, last_empty):
    """Other layouts in one batch (tiles of several rounds at 1-4 KiB chunks,
    CRC32, the v1 protocol): bad chunks at the last tile of block 1 and the
    first of block 3; every job the oracle's, no device check."""
    diag = _diag()
    nch = 65536 // cs
    streams = [build_stream(oracle.crc32c, proto, cs, ctype, [65536] * 100, seed=500 + k, last_empty=last_empty,
                            corrupt=[(99, nch - 1)] if k == 1 else [(0, 0)] if k == 3 else [])[0] for k in range(5)]
    want = [oracle.verify_packets(s, proto=proto, chunk_size=cs, ctype=ctype) for s in streams]
    assert want[1][0] != 0 and want[3][0] != 0 and want[0][0] == 0
    bufs = [_dev(engine, s) for s in streams]
    assert diag.hdfs_crc32c_set_job_coalesce(2) == 0
    try:
        _checks(diag)
        jobs = [engine.VerifyJob(b.ptr, len(s), proto=proto, chunk_size=cs, ctype=ctype, lib=diag)
                for b, s in zip(bufs, streams)]
        got = [j.wait() for j in jobs]
        checks = _checks(diag)
    finally:
        diag.hdfs_crc32c_set_job_coalesce(1)
    for b in bufs:
        b.free()
    assert got == want
    assert checks == (0, 0, 0), checks


@pytest.mark.gpu
@pytest.mark.parametrize("on", [1, 0])
def test_gpu_jobs_per_run_returns_early(engine, oracle, on):
    """Six 32 MiB blocks in one batch, block 3 bad, waited in order: with
    per-run completion the first jobs return before the launch ends (the
    bad block's job never does); without it none does.  Results equal."""
    diag = _diag()
    streams = [_block(oracle, k, n=512, corrupt=[(300, 7)] if k == 3 else []) for k in range(6)]
    want = [oracle.verify_packets(s) for s in streams]
    assert diag.hdfs_crc32c_set_job_early(on) == 0
    try:
        _early(diag)
        got = _run_held(engine, diag, streams, range(6))
        early = _early(diag)
    finally:
        diag.hdfs_crc32c_set_job_early(1)
    assert [got[k] for k in range(6)] == want
    assert _checks(diag) == (0, 0, 0)
    if on:
        assert early[0] >= 1, early
    else:
        assert early == (0, 0), early


@pytest.mark.gpu
@pytest.mark.parametrize("order", ["reverse", "middle_first"])
def test_gpu_jobs_per_run_wait_orders(engine, oracle, order):
    """The batch's jobs waited out of order (the last run first, or a middle
    one): each the oracle's."""
    diag = _diag()
    streams = [_block(oracle, k, corrupt=[(50, 3)] if k == 2 else []) for k in range(5)]
    want = [oracle.verify_packets(s) for s in streams]
    seq = [4, 3, 2, 1, 0] if order == "reverse" else [2, 0, 4, 1, 3]
    got = _run_held(engine, diag, streams, seq)
    assert [got[k] for k in range(5)] == want
    assert _checks(diag) == (0, 0, 0)


@pytest.mark.gpu
@pytest.mark.parametrize("window", [2, 3, 4, 5, 8])
def test_gpu_jobs_per_run_stream_window(engine, oracle, window):
    """The datanode pattern (product coalescing): 16 blocks, at most `window`
    outstanding, the oldest waited before the next submit -- single-run and
    batch launches of different sizes take turns on the job slots, whose
    control words each launch hands on zeroed to the next; bad chunks at the
    last tile of every third block and a block whose headers leave the
    prediction among them."""
    diag = _diag()
    streams = [_block(oracle, k, corrupt=[(99, 127)] if k % 3 == 1 else [(10, 1)] if k == 6 else [])
               for k in range(16)]
    streams[11], _ = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, [65536] * 100, seed=311,
                                  seqnos=[k + (5 if k > 40 else 0) for k in range(100)])
    want = [oracle.verify_packets(s) for s in streams]
    bufs = [_dev(engine, s) for s in streams]
    got, q = {}, []
    for k, (b, s) in enumerate(zip(bufs, streams)):
        if len(q) == window:
            k0, j0 = q.pop(0)
            got[k0] = j0.wait()
        q.append((k, engine.VerifyJob(b.ptr, len(s), lib=diag)))
    for k0, j0 in q:
        got[k0] = j0.wait()
    for b in bufs:
        b.free()
    assert [got[k] for k in range(16)] == want
    assert _checks(diag) == (0, 0, 0)


POOL_CHILD = r"""
import ctypes, json, sys
for p in ({root!r}, {root!r} + "/tools", {root!r} + "/tests", {root!r} + "/oracle"):
    sys.path.insert(0, p)
import numpy as np
import diaglib
import hadoofus_amd as h
lib = h.abi.bind_diag(h.load(diaglib.DIAG_LIB_PATH))
from oracle import Oracle
from packet_stream import CSUM_CRC32, CSUM_CRC32C, build_stream
o = Oracle()
streams = [build_stream(o.crc32c, 2, 512, CSUM_CRC32C, [65536] * 100, seed=400 + k,
                        corrupt=[(99, 127)] if k == 6 else [])[0] for k in range(8)]
bufs = []
for s in streams:
    d = h.DeviceBuffer(len(s) + 64)
    d.upload(np.frombuffer(s, np.uint8))
    bufs.append(d)
h.device_sync()
assert lib.hdfs_crc32c_set_job_coalesce(2) == 0
e = (ctypes.c_uint64 * 2)()
lib.hdfs_crc32c_diag_job_early(e, 1)
jobs = [h.VerifyJob(d.ptr, len(s), lib=lib) for d, s in zip(bufs, streams)]
got = [j.wait() for j in jobs]
lib.hdfs_crc32c_diag_job_early(e, 1)
c = (ctypes.c_uint32 * 3)()
lib.hdfs_crc32c_diag_device_checks(c, 1)
print(json.dumps({{"same": got == [o.verify_packets(s) for s in streams], "early": list(e), "checks": list(c)}}))
"""


@pytest.mark.gpu
def test_gpu_jobs_per_run_with_pool():
    """The launch's global pool in use (HDFS_CRC32C_SPEC_POOL=1: from one
    round per wave): the runs with pool tiles are left to the final block,
    the others may return early; every job the oracle's, no device check."""
    env = dict(os.environ, HDFS_CRC32C_SPEC_POOL="1")
    r = subprocess.run([sys.executable, "-c", POOL_CHILD.format(root=ROOT)], capture_output=True, text=True,
                       timeout=180, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["same"], out
    assert out["checks"] == [0, 0, 0], out
    assert sum(out["early"]) >= 1, out


@pytest.mark.gpu
def test_gpu_jobs_threads(engine, oracle):
    """A datanode's receiver threads: 4 threads, each verifying its own 6
    blocks as jobs with 2 outstanding (their jobs share batch launches and
    per-run completions), while a fifth makes synchronous calls on other
    blocks: every result the oracle's, no device check."""
    import threading
    diag = _diag()
    streams = [_block(oracle, k, corrupt=[(99, 127)] if k % 5 == 2 else []) for k in range(28)]
    want = [oracle.verify_packets(s) for s in streams]
    bufs = [_dev(engine, s) for s in streams]
    got, errs = {}, []

    def receiver(ks):
        try:
            q = []
            for k in ks:
                if len(q) == 2:
                    k0, j0 = q.pop(0)
                    got[k0] = j0.wait()
                q.append((k, engine.VerifyJob(bufs[k].ptr, len(streams[k]), lib=diag)))
            for k0, j0 in q:
                got[k0] = j0.wait()
        except Exception as e:  # reported below
            errs.append(repr(e))

    def sync_caller(ks):
        try:
            for k in ks:
                got[k] = engine.verify_packets(None, dptr=bufs[k].ptr, nbytes=len(streams[k]), lib=diag)
        except Exception as e:
            errs.append(repr(e))

    _checks(diag)
    th = [threading.Thread(target=receiver, args=(range(6 * t, 6 * t + 6),)) for t in range(4)]
    th.append(threading.Thread(target=sync_caller, args=(range(24, 28),)))
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    for b in bufs:
        b.free()
    assert not errs, errs
    assert [got[k] for k in range(28)] == want
    assert _checks(diag) == (0, 0, 0)


@pytest.mark.gpu
def test_gpu_jobs_per_run_wait_room(engine, oracle):
    """A wait whose record array is smaller than the run (less room than at
    the submit) fails with EINVAL whether or not the run completed early --
    as without per-run completion -- and the batch's other jobs are
    unaffected."""
    diag = _diag()
    streams = [_block(oracle, k) for k in range(4)]
    want = [oracle.verify_packets(s) for s in streams]
    bufs = [_dev(engine, s) for s in streams]
    assert diag.hdfs_crc32c_set_job_coalesce(2) == 0
    try:
        jobs = [engine.VerifyJob(b.ptr, len(s), lib=diag) for b, s in zip(bufs, streams)]
        small = (engine.Packet * 50)()
        n, used = ctypes.c_size_t(0), ctypes.c_uint64(0)
        job, jobs[1].job = jobs[1].job, None
        rc = diag.hdfs_crc32c_job_wait(job, small, 50, ctypes.byref(n), ctypes.byref(used))
        got = {k: jobs[k].wait() for k in (0, 2, 3)}
    finally:
        diag.hdfs_crc32c_set_job_coalesce(1)
    for b in bufs:
        b.free()
    assert rc == -1, rc  # HDFS_CRC32C_EINVAL
    assert all(got[k] == want[k] for k in (0, 2, 3))
