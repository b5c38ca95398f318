"""Hardware queues of the engine's streams (round 6).  The runtime spreads a
process's streams over at most GPU_MAX_HW_QUEUES queues per priority level,
least used first, so the queue a stream gets depends on what the host
process created before the engine.  The streams that run BESIDE the
speculative kernel (the short rest of a block, a scatter read's copy) must
not share the engine stream's queue, or their work waits behind the kernel:
the engine probes the queue of each (a dispatch that reports the AQL queue
pointer it ran from) and replaces a stream on the engine stream's queue by a
CU-masked one, which the runtime never pools.  Each case runs in a fresh
process that creates `n` streams through HIP before the engine's first call;
the engine's verify of a block ending in a short packet (the short-rest
path) equals the oracle's either way."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import ctypes, json, sys
for p in ({root!r}, {root!r} + "/tools", {root!r} + "/tests", {root!r} + "/oracle"):
    sys.path.insert(0, p)
hip = ctypes.CDLL("libamdhip64.so")
vp = ctypes.c_void_p
hip.hipStreamCreateWithFlags.argtypes = [ctypes.POINTER(vp), ctypes.c_uint]
hip.hipMalloc.argtypes = [ctypes.POINTER(vp), ctypes.c_size_t]
hip.hipMemsetAsync.argtypes = [vp, ctypes.c_int, ctypes.c_size_t, vp]
hip.hipStreamSynchronize.argtypes = [vp]
buf = vp()
assert hip.hipMalloc(ctypes.byref(buf), 64) == 0
streams = []
for _ in range({n}):  # the host process's own streams, each used once
    s = vp()
    assert hip.hipStreamCreateWithFlags(ctypes.byref(s), 1) == 0
    assert hip.hipMemsetAsync(buf, 0, 64, s) == 0 and hip.hipStreamSynchronize(s) == 0
    streams.append(s)
import diaglib
import hadoofus_amd as h
lib = h.load(diaglib.DIAG_LIB_PATH)
import numpy as np
from oracle import Oracle
from packet_stream import CSUM_CRC32C, build_stream
o = Oracle()
s, _ = build_stream(o.crc32c, 2, 512, CSUM_CRC32C, [65536] * 80 + [12345], seed=4, corrupt=[(79, 3)])
d = h.DeviceBuffer(len(s) + 64)
d.upload(np.frombuffer(s, np.uint8))
h.device_sync()
got = h.verify_packets(None, dptr=d.ptr, nbytes=len(s))
q = (ctypes.c_uint64 * 4)()
assert lib.hdfs_crc32c_diag_stream_queues(q) == 0
print(json.dumps({{"queues": list(q), "same_as_oracle": got == o.verify_packets(s)}}))
"""


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 3, 4, 7, 8])
def test_gpu_beside_streams_have_their_own_queue(n):
    r = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT, n=n)], capture_output=True, text=True,
                       timeout=120, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    main, tail, copy, _mb = out["queues"]
    assert main and tail and copy
    assert tail != main and copy != main, (n, out)
    assert out["same_as_oracle"]
