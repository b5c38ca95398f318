"""Host-resident (H2D + kernel + D2H) rate of the verify path, for DESIGN.md.
Data lives in host memory (pinned, and separately pageable); the engine's
pipeline overlaps copies with kernels.  GPU box only."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hadoofus_amd as h  # noqa: E402

GIB = 1 << 30
n = int(float(os.environ.get("H2D_GIB", "8")) * GIB)
cs = 512
h.load()
dev = h.DeviceBuffer(n)
h.fill_splitmix64(dev.ptr, n // 8, 0, 0)
h.device_sync()
pin = h.PinnedBuffer(n)
out = {"bytes": n, "chunk": cs}
dev.copy_to(pin.ptr)
dev.free()
crcs = h.compute_host(pin.array, cs, flags=h.SEG_BE)
for piece_mib in (16, 64, 256):
    best = 0.0
    for _ in range(3):
        t0 = time.perf_counter()
        fb, m, bm = h.verify_host(pin.array, cs, crcs, flags=h.SEG_BE, piece_bytes=piece_mib << 20)
        dt = time.perf_counter() - t0
        assert m == 0, m
        best = max(best, n / dt / GIB)
    out[f"pinned_verify_GiBps_piece{piece_mib}MiB"] = round(best, 2)
t0 = time.perf_counter()
crcs2 = h.compute_host(pin.array, cs, flags=h.SEG_BE, piece_bytes=64 << 20)
out["pinned_compute_GiBps_piece64MiB"] = round(n / (time.perf_counter() - t0) / GIB, 2)
assert np.array_equal(crcs, crcs2)
# pageable host memory (registered by the engine for the call)
pg = np.empty(n, dtype=np.uint8)
pg[:] = pin.array
t0 = time.perf_counter()
fb, m, bm = h.verify_host(pg, cs, crcs, flags=h.SEG_BE, piece_bytes=64 << 20)
out["pageable_verify_GiBps_incl_register"] = round(n / (time.perf_counter() - t0) / GIB, 2)
assert m == 0
pin.free()
print(json.dumps(out))
