import json, os, sys, time
import numpy as np
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"])
import hadoofus_amd as h
GIB = 1 << 30
n = 8 * GIB; cs = 512
h.load()
dev = h.DeviceBuffer(n); h.fill_splitmix64(dev.ptr, n // 8, 0, 0); h.device_sync()
pin = h.PinnedBuffer(n); dev.copy_to(pin.ptr); dev.free()
crcs = h.compute_host(pin.array, cs, flags=h.SEG_BE)
pc = h.PinnedBuffer(crcs.nbytes); pc.array[:] = crcs.view(np.uint8)
out = {}
for piece in (64, 16, 64, 256, 64, 32, 128):
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        fb, m, bm = h.verify_host(pin.array, cs, crcs, flags=h.SEG_BE, piece_bytes=piece << 20)
        ts.append(round(n / (time.perf_counter() - t0) / GIB, 1))
    ts2 = []
    for _ in range(2):
        t0 = time.perf_counter()
        fb, m, bm = h.verify_host(pin.array, cs, pc.array.view(np.uint32), flags=h.SEG_BE, piece_bytes=piece << 20)
        ts2.append(round(n / (time.perf_counter() - t0) / GIB, 1))
    out.setdefault(f"p{piece}", []).append({"pageable_crcs": ts, "pinned_crcs": ts2})
    print(piece, ts, ts2, file=sys.stderr, flush=True)
print(json.dumps(out))
