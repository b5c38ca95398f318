"""Sweep of streaming-read probe shapes (variants 10..23 of probe2_kernel,
hadoofus_amd/csrc/crc32c_probes.hip) against the classic grid-stride probe
(variants 0..9): which access shape / cache policy / LDS-DMA reads HBM
fastest on this part?  Also times the verify plan itself for reference."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hadoofus_amd as h  # noqa: E402
import diaglib  # noqa: E402

n = int(os.environ.get("PROBE_GIB", "64")) << 30
h.load(diaglib.DIAG_LIB_PATH)  # tuning knobs: diagnostic build only
D = diaglib.Diag(lib=h.load())
buf = h.DeviceBuffer(n)
h.fill_splitmix64(buf.ptr, n // 8, 0, 0)
h.device_sync()
out = {}
shapes = [(1, 1024), (2, 512), (4, 256)]
for variant in [4, 8] + list(range(10, 24)):
    for gpc, blk in shapes:
        if variant < 10 and (gpc, blk) != (1, 1024):
            continue
        D.set_probe(variant, gpc, blk)
        vals = [D.probe_read(buf.ptr, n, 2) for _ in range(2)]
        out[f"v{variant}_g{gpc}_b{blk}"] = round(max(vals), 1)
        print(f"v{variant}_g{gpc}_b{blk}", out[f"v{variant}_g{gpc}_b{blk}"], file=sys.stderr, flush=True)
D.set_probe()
best = sorted(out.items(), key=lambda kv: -kv[1])[:6]
out["best"] = best
print(json.dumps(out))
