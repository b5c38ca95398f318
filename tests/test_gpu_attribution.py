"""Fault attribution without a per-call cost (round 4).

A synchronous call (the drop-in _hdfs_crc32c, verify_crcdata, short device
runs) used to query the engine stream on every call, so that a fault of
EARLIER asynchronous work would be reported by this call rather than the
next: ~2 us per call (profiles/r03/e8_small_launch.json).  The query now runs
only while work no call has seen complete is queued on the stream -- an
asynchronous plan execute -- and a call that sees its own completion word
clears that state (its kernel ran after everything before it).  GPU faults
are not provoked here (they can take the box down); the diagnostic build's
query counter shows when the check runs."""
import ctypes

import numpy as np
import pytest


@pytest.fixture(scope="module")
def diag(engine):
    from hadoofus_amd import abi, build
    return abi.bind_diag(abi.bind_product(ctypes.CDLL(build.DIAG_LIB)))


def _queries(lib):
    q = ctypes.c_uint64(0)
    assert lib.hdfs_crc32c_diag_stream_queries(ctypes.byref(q)) == 0
    return q.value


@pytest.mark.gpu
def test_gpu_stream_query_only_after_async_work(engine, diag, oracle):
    from hadoofus_amd import abi
    data = np.random.default_rng(1).integers(0, 256, 512, dtype=np.uint8).tobytes()
    want = oracle.crc32c(0, data)
    assert diag._hdfs_crc32c(0, data, 512) == want
    q0 = _queries(diag)
    for _ in range(50):  # back-to-back synchronous calls: no query
        assert diag._hdfs_crc32c(0, data, 512) == want
    assert _queries(diag) == q0
    # an asynchronous verify plan on the engine stream: the next synchronous
    # call checks the stream once, the one after it no more
    buf = engine.DeviceBuffer(1 << 20)
    buf.fill(7)
    crcs = engine.DeviceBuffer(8192)
    bm = engine.DeviceBuffer(1024)
    seg = engine.Segment(data=buf.ptr, len=1 << 20, chunk_size=512, flags=engine.SEG_BE, crc_init=0, crcs=crcs.ptr,
                         bitmap=bm.ptr)
    plan = abi.Plan(engine.MODE_VERIFY, [seg], lib=diag)
    assert diag.hdfs_crc32c_plan_execute(plan.ptr, None) == 0
    assert diag._hdfs_crc32c(0, data, 512) == want
    assert _queries(diag) == q0 + 1
    assert diag._hdfs_crc32c(0, data, 512) == want
    assert _queries(diag) == q0 + 1
    plan.results()
    plan.destroy()
    for b in (buf, crcs, bm):
        b.free()
