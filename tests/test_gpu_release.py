"""The release library cannot be told to skip work (ADVICE high):
every tuning / diagnostic variable the diagnostic build honours is set in a
FRESH child process -- store policies 2 (drop compute-mode CRC stores) and 4
(verify runs the load-only twin, no CRC arithmetic), other schedules, load
policies, shapes -- and the release library still returns oracle-exact CRCs
(tiled path and the >64 KiB drop-in) and reports every corrupted chunk.
Contract protected: src/datanode.c:2945-2960 (every mismatch is reported)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, sys
import numpy as np
sys.path.insert(0, {root!r}); sys.path.insert(0, {oracle!r})
import hadoofus_amd as h
from oracle import Oracle, splitmix64_np
o = Oracle()
h.load()
cs, nseg, seg = 512, 16, 8 << 20
host = splitmix64_np(nseg * seg // 8, seed=21).view(np.uint8).copy()
want = [o.chunk_crcs(host[i * seg:(i + 1) * seg], cs) for i in range(nseg)]
d = h.DeviceBuffer(host.nbytes); d.upload(host)
crcs = h.DeviceBuffer(nseg * (seg // cs) * 4); bms = h.DeviceBuffer(nseg * (seg // cs) // 8)
segs = [h.Segment(data=d.ptr + i * seg, len=seg, chunk_size=cs, flags=h.SEG_BE, crc_init=0,
                  crcs=crcs.ptr + i * (seg // cs) * 4, bitmap=bms.ptr + i * (seg // cs) // 8) for i in range(nseg)]
h.Plan(h.MODE_COMPUTE, segs).execute()
got = crcs.download(dtype=">u4").astype(np.uint32)
compute_ok = bool(np.array_equal(got, np.concatenate(want)))
# corrupt one byte in each of 37 chunks spread over all segments, then verify
bad = sorted({{(k * 7919) % (nseg * seg // cs) for k in range(37)}})
for c in bad:
    host[c * cs + (c % cs)] ^= 0x5A
d.upload(host)
vp = h.Plan(h.MODE_VERIFY, segs)
vp.execute()
fb, m = vp.results()
bits = np.unpackbits(bms.download(), bitorder="little")
verify_ok = bool(m == len(bad) and list(np.nonzero(bits)[0]) == bad)
first_ok = all(fb[i] == next((c - i * (seg // cs) for c in bad if c // (seg // cs) == i), 0xFFFFFFFF)
               for i in range(nseg))
# drop-in on > 64 KiB host data: the tiled kernel + combine (stream_crc_locked)
big = host[: 3 * 1024 * 1024 + 5]
dropin_ok = h.crc32c(0x1234, big) == o.crc32c(0x1234, big)
print(json.dumps({{"compute_ok": compute_ok, "verify_ok": verify_ok, "first_ok": first_ok,
                  "dropin_ok": bool(dropin_ok), "mism": int(m), "expected": len(bad)}}))
'''

ENVS = [
    {"HDFS_CRC32C_STORE": "4"},
    {"HDFS_CRC32C_STORE": "2"},
    {"HDFS_CRC32C_STORE": "3", "HDFS_CRC32C_TILE_ORDER": "0", "HDFS_CRC32C_NT": "0"},
    {"HDFS_CRC32C_DEPTH": "9", "HDFS_CRC32C_STREAMS": "3", "HDFS_CRC32C_BLOCK": "64",
     "HDFS_CRC32C_GROUP": "15", "HDFS_CRC32C_ALIGN": "4096", "HDFS_CRC32C_SMALL_RULE": "0"},
]


@pytest.mark.parametrize("env", ENVS, ids=lambda e: ",".join(f"{k[12:]}={v}" for k, v in e.items()))
def test_release_ignores_diagnostic_environment(env):
    code = CHILD.format(root=ROOT, oracle=os.path.join(ROOT, "oracle"))
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=180,
                       env=dict(os.environ, **env))
    assert p.returncode == 0, p.stderr[-2000:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["compute_ok"] and r["verify_ok"] and r["first_ok"] and r["dropin_ok"], r
