import os, sys, json, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "oracle"))
import numpy as np
import hadoofus_amd as h
from oracle import Oracle, splitmix64_np
o = Oracle(); h.load()
n = 64 << 20
host = splitmix64_np(n // 8 + 4, seed=3).view(np.uint8)
d = h.DeviceBuffer(host.nbytes); d.upload(host)
out = {"align_env": os.environ.get("HDFS_CRC32C_ALIGN")}
for off in (0, 1, 2, 4, 8, 12):
    seg_len = n - 4096
    want = o.chunk_crcs(host[off:off + seg_len], 512)
    crcs = h.DeviceBuffer(want.nbytes)
    seg = h.Segment(data=d.ptr + off, len=seg_len, chunk_size=512, flags=0, crc_init=0, crcs=crcs.ptr)
    p = h.Plan(h.MODE_COMPUTE, [seg])
    p.execute()
    got = crcs.download(dtype=np.uint32)
    ok = bool(np.array_equal(got, want))
    ms = p.time(5)
    out[f"off{off}"] = {"ok": ok, "GBps": round(seg_len / (ms * 1e-3) / 1e9, 1), "bad": int((got != want).sum())}
print(json.dumps(out))
