"""Kernel memory ceiling: the verify kernel vs its load-only twin (store
policy 4: same loads and store ops, no CRC arithmetic) vs the streaming-read
probes, interleaved in ONE process on the bench's 128 GiB (GPU box only)."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hadoofus_amd as h  # noqa: E402
import diaglib  # noqa: E402

BLOCK = 128 << 20
B = int(os.environ.get("BLOCKS", "1024"))
cs = 512
h.load(diaglib.DIAG_LIB_PATH)  # tuning knobs: diagnostic build only
D = diaglib.Diag(lib=h.load())
data = h.DeviceBuffer(B * BLOCK)
crcs = h.DeviceBuffer(B * BLOCK // cs * 4)
bms = h.DeviceBuffer(B * BLOCK // cs // 8)
h.fill_splitmix64(data.ptr, B * BLOCK // 8, 0, 0)
segs = [h.Segment(data=data.ptr + b * BLOCK, len=BLOCK, chunk_size=cs, flags=h.SEG_BE, crc_init=0,
                  crcs=crcs.ptr + b * (BLOCK // cs) * 4, bitmap=bms.ptr + b * (BLOCK // cs) // 8) for b in range(B)]
h.Plan(h.MODE_COMPUTE, segs).execute()
ver = h.Plan(h.MODE_VERIFY, segs)
h.device_sync()
alg = B * BLOCK * (1 + 4 / cs + 1 / (8 * cs))
res = {}
PROBES = [int(x) for x in os.environ.get("PROBES", "14,11").split(",")]
for rnd in range(int(os.environ.get("ROUNDS", "4"))):
    for pol in (0, 4):
        D.set_store_policy(pol)
        ms = ver.time(3)
        res.setdefault(f"verify_policy{pol}_alg_GBps", []).append(alg / (ms * 1e-3) / 1e9)
    D.set_store_policy(0)
    for v in PROBES:
        D.set_probe(v, 2, 512)
        res.setdefault(f"probe{v}_g2_b512_GBps", []).append(D.probe_read(data.ptr, B * BLOCK, 3))
    D.set_probe(0, 2, 1024)
D.set_store_policy(0)
ver.execute()
_, m = ver.results()
out = {"blocks": B, "mismatches_policy0": m}
out.update({k: round(statistics.median(v), 1) for k, v in res.items()})
print(json.dumps(out))
