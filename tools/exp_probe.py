"""Sweep of streaming-read probe shapes: is the simple probe the HBM ceiling?"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hadoofus_amd as h  # noqa: E402
import diaglib  # noqa: E402

n = 128 << 30
h.load(diaglib.DIAG_LIB_PATH)  # tuning knobs: diagnostic build only
D = diaglib.Diag(lib=h.load())
buf = h.DeviceBuffer(n)
h.fill_splitmix64(buf.ptr, n // 8, 0, 0)
h.device_sync()
out = {}
for variant in (1, 9, 4, 8):
    for gpc, blk in ((2, 1024), (1, 1024), (4, 512), (16, 256)):
        D.set_probe(variant, gpc, blk)
        vals = [D.probe_read(buf.ptr, n, 2) for _ in range(2)]
        out[f"v{variant}_g{gpc}_b{blk}"] = round(max(vals), 1)
D.set_probe()
best = max(out.items(), key=lambda kv: kv[1])
out["best"] = best
print(json.dumps(out))
