"""Pinned host memory of the host-memory paths (hadoofus_amd/csrc/crc32c_hostpin.h).

Round 2's one unexplained GPU fault (hipErrorIllegalAddress in the first
H2D copy of a test that followed host-path packet calls on a pageable
buffer) pointed at the engine's host registrations: "pinned already?" was
answered by the runtime for any address, and a failed hipHostUnregister was
dropped.  The engine now keeps its own registry (engine allocations,
refcounted registrations of each call's exact bytes, checked unregistration, streams
drained before unpinning on every return path).

CPU: the registry's bookkeeping against a fake runtime
(tests/consumer/hostpin_selftest.cpp, built with ASan/UBSan): buffers freed
and re-mapped at the same address between calls, shared pages, nesting,
concurrency, refused and failed (un)registrations.
GPU: the same sequences on the real runtime -- host packet runs and host
pipelines on pageable buffers re-mapped at one address, each followed by a
plain H2D copy from the new buffer (the round-2 fault's shape), max_pkts
stops and a framing error mid-run, adjacent arrays sharing pages, memory
pinned by torch, and the engine's own pinned blocks."""
import mmap
import os
import subprocess

import numpy as np
import pytest

from packet_stream import CSUM_CRC32C, build_stream

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_hostpin_registry_selftest(tmp_path):
    exe = tmp_path / "hostpin_selftest"
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-fsanitize=address,undefined", "-pthread",
                           "-I" + os.path.join(ROOT, "hadoofus_amd", "csrc"),
                           os.path.join(ROOT, "tests", "consumer", "hostpin_selftest.cpp"), "-o", str(exe)])
    p = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert p.stdout.strip().endswith("0 failures"), p.stdout


def _mapped(nbytes):
    """A pageable buffer of its own anonymous mapping (freed by close())."""
    m = mmap.mmap(-1, nbytes)
    a = np.frombuffer(m, dtype=np.uint8)
    return m, a


@pytest.mark.gpu
def test_gpu_host_paths_on_remapped_buffers(engine, oracle):
    """The round-2 fault's sequence, several times over: host-path calls pin
    a pageable buffer, the buffer is unmapped, a new buffer is mapped at the
    same address, and a plain H2D copy reads it -- every copy and every
    verdict must be exact."""
    dl = [65536] * 300 + [12345]
    base = None
    reused = 0
    for it in range(6):
        s, bad = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, dl, seed=it, corrupt=[(it * 7 + 3, it + 1)])
        m, a = _mapped(len(s) + 4096)
        a[:len(s)] = np.frombuffer(s, np.uint8)
        view = a[:len(s)]
        addr = a.ctypes.data
        reused += addr == base
        base = addr
        want = oracle.verify_packets(s)
        assert engine.verify_packets(view) == want
        for mp in (1, 37, 299):  # max_pkts stops: only the packets walked are pinned and verified
            assert engine.verify_packets(view, max_pkts=mp) == oracle.verify_packets(s, max_pkts=mp)
        # a framing error in the middle of the run (CRC_LEN on packet 150)
        cut = bytearray(s)
        off = 150 * (6 + 25 + 4 * 128 + 65536)
        cut[off:off + 4] = (65536 + 4 * 127 + 4).to_bytes(4, "big")
        a[:len(s)] = np.frombuffer(bytes(cut), np.uint8)
        assert engine.verify_packets(view) == oracle.verify_packets(bytes(cut))
        # host pipeline on the same mapping: data, then its CRCs right after it
        # (they share a page with each other and with the packet bytes)
        n = 8 << 20
        data = a[:n]
        crcs = np.frombuffer(m, dtype=np.uint32, count=n // 512, offset=n)
        assert engine.load().hdfs_crc32c_compute_host(data.ctypes.data, n, 512, engine.SEG_BE, 0,
                                                      crcs.ctypes.data, 0) == 0
        assert np.array_equal(crcs, oracle.chunk_crcs(data, 512).astype(">u4").view(np.uint32))
        del a, view, data, crcs
        m.close()  # unmapped (no view of it is left)
        # the next mapping usually lands at the same address: a plain H2D copy
        # from it must read the new pages (nothing of the old registration left)
        m2, b = _mapped(len(s) + 4096)
        b[:] = (it * 37 + 11) & 0xFF
        dev = engine.DeviceBuffer(b.nbytes)
        dev.upload(b)
        engine.device_sync()
        assert np.array_equal(dev.download(), b)
        dev.free()
        del b
        m2.close()
    print(f"address reused in {reused} of 5 re-mappings")


@pytest.mark.gpu
def test_gpu_host_pipeline_shared_pages(engine, oracle):
    """Data, expected CRCs and bitmap in one small allocation (they share
    pages): one registration per page, released once, results exact."""
    rng = np.random.default_rng(5)
    cs, nch = 512, 3000
    blob = np.zeros(cs * nch + 4 * nch + (nch + 7) // 8 + 64, np.uint8)
    data = blob[:cs * nch]
    data[:] = rng.integers(0, 256, data.size, dtype=np.uint8)
    crcs = blob[cs * nch + 3: cs * nch + 3 + 4 * nch]  # odd offset, shares a page with data
    crcs[:] = oracle.chunk_crcs(data, cs).astype(">u4").view(np.uint8)
    bm = blob[cs * nch + 3 + 4 * nch:][: (nch + 7) // 8]
    data[cs * 1234 + 5] ^= 1
    import ctypes
    fb, mism = ctypes.c_uint64(0), ctypes.c_uint64(0)
    lib = engine.load()
    rc = lib.hdfs_crc32c_verify_host(data.ctypes.data, data.nbytes, cs, engine.SEG_BE, 0, crcs.ctypes.data,
                                     bm.ctypes.data, 0, ctypes.byref(fb), ctypes.byref(mism))
    assert rc == 0, lib.hdfs_crc32c_last_error()
    assert (fb.value, mism.value) == (1234, 1)
    assert np.nonzero(np.unpackbits(bm, bitorder="little"))[0].tolist() == [1234]
    # compute into the same blob's CRC window, then verify clean
    data[cs * 1234 + 5] ^= 1
    rc = lib.hdfs_crc32c_compute_host(data.ctypes.data, data.nbytes, cs, engine.SEG_BE, 0, crcs.ctypes.data, 0)
    assert rc == 0, lib.hdfs_crc32c_last_error()
    assert np.array_equal(crcs.view(">u4").astype(np.uint32), oracle.chunk_crcs(data, cs))


@pytest.mark.gpu
def test_gpu_host_paths_on_foreign_and_engine_pinned_memory(engine, oracle):
    """Memory pinned by its owner (another hipHostMalloc user, e.g. torch's
    pinned tensors) is used in place and left pinned;
    the engine's own blocks (host_alloc) are used in place; freeing a block
    the engine did not allocate is refused."""
    s, _ = build_stream(oracle.crc32c, 2, 512, CSUM_CRC32C, [65536] * 64, seed=4, corrupt=[(9, 9)])
    want = oracle.verify_packets(s)
    pin = engine.PinnedBuffer(len(s))
    pin.array[:] = np.frombuffer(s, np.uint8)
    assert engine.verify_packets(pin.array) == want
    assert engine.verify_packets(pin.array[100000:], max_pkts=3)[0] in (0, 18, 25, 26, 27, 29)  # odd start: any verdict, no fault
    pin.free()
    # memory pinned by another allocator (the HIP runtime directly, as torch's
    # pinned tensors are): used in place, left pinned
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so.7")  # the runtime the engine library links
    p = ctypes.c_void_p()
    assert hip.hipHostMalloc(ctypes.byref(p), ctypes.c_size_t(len(s) + 4096), 0) == 0
    a = np.ctypeslib.as_array((ctypes.c_uint8 * (len(s) + 4096)).from_address(p.value))
    a[:len(s)] = np.frombuffer(s, np.uint8)
    for _ in range(3):
        assert engine.verify_packets(a[:len(s)]) == want
    a[:] = 0  # still mapped and writable after the engine's calls
    del a
    assert hip.hipHostFree(p) == 0
    junk = np.zeros(4096, np.uint8)
    assert engine.load().hdfs_crc32c_host_free(junk.ctypes.data) == -1  # HDFS_CRC32C_EINVAL
