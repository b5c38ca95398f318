"""A/B timing of tiled-kernel variants in ONE process (interleaved rounds),
the streaming-read probe (empirical roofline), and a per-wave timestamp
diagnostic (tail imbalance).  GPU box only."""
import json
import os
import statistics
import sys

import numpy as np

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
crcs = h.DeviceBuffer(B * BLOCK // cs * 4)   # expected CRCs (default shape, clean data)
crcs2 = h.DeviceBuffer(B * BLOCK // cs * 4)  # compute-mode output of the variant under test
bms = h.DeviceBuffer(B * BLOCK // cs // 8)
h.fill_splitmix64(data.ptr, B * BLOCK // 8, 0, 0)
h.device_sync()
out = {"blocks": B}
out["probe_read_GBps"] = [round(D.probe_read(data.ptr, B * BLOCK, 3), 1) for _ in range(3)]
segs = [h.Segment(data=data.ptr + b * BLOCK, len=BLOCK, chunk_size=cs, flags=h.SEG_BE, crc_init=0,
                  crcs=crcs.ptr + b * (BLOCK // cs) * 4, bitmap=bms.ptr + b * (BLOCK // cs) // 8) for b in range(B)]
segs2 = [h.Segment(data=data.ptr + b * BLOCK, len=BLOCK, chunk_size=cs, flags=h.SEG_BE, crc_init=0,
                   crcs=crcs2.ptr + b * (BLOCK // cs) * 4) for b in range(B)]
ref = h.Plan(h.MODE_COMPUTE, segs)
ref.execute()
h.device_sync()
# the bench's corruption pattern: 1 in 65537 chunks
for b in range(B):
    h.corrupt(data.ptr + b * BLOCK, BLOCK, cs, b * (BLOCK // cs), 65537, 7919, None)
h.device_sync()
from hadoofus_amd import shard  # noqa: E402
expect_bad = shard.expected_bad(0, B, BLOCK // cs, 65537)
comp = h.Plan(h.MODE_COMPUTE, segs2)
ver = h.Plan(h.MODE_VERIFY, segs)
comp.execute()
h.device_sync()
digest0 = h.stream_crc_dev(0, crcs2.ptr, B * BLOCK // cs * 4)
out["expect_bad"] = expect_bad
VARIANTS = [tuple(int(x) for x in v.split(",")) for v in
            os.environ.get("AB_VARIANTS", "1,1,3;2,1,3").split(";")]
# (order, nt, depth[, group shift[, streams, block[, store policy]]])
VARIANTS = [(v + (3, 1, 1024, 0)[len(v) - 3:]) if len(v) < 7 else v for v in VARIANTS]


def apply(order, nt, depth, gs, S, blk, pol, diag_ptr=None):
    D.set_tile_order(order)
    D.set_tuning(nt, diag_ptr)
    D.set_depth(depth)
    D.set_group_shift(gs)
    D.set_shape(S, blk)
    D.set_store_policy(pol)


def tag(order, nt, depth, gs, S, blk, pol=0):
    return (f"o{order}_nt{nt}_d{depth}_g{gs}" + ("" if (S, blk) == (1, 1024) else f"_s{S}_b{blk}") +
            ("" if pol == 0 else f"_p{pol}"))
res = {}
for rnd in range(4):
    for v in VARIANTS:
        apply(*v)
        for name, p in (("compute", comp), ("verify", ver)):
            ms = p.time(3)
            res.setdefault(f"{name}_{tag(*v)}", []).append(B * BLOCK / (ms * 1e-3) / 1e9)
        _, m = ver.results()
        ok = m == expect_bad and h.stream_crc_dev(0, crcs2.ptr, B * BLOCK // cs * 4) == digest0
        out.setdefault("parity_ok", {})[tag(*v)] = bool(ok)
for k, v in res.items():
    out[k + "_GBps_median"] = round(statistics.median(v), 1)
# per-wave timestamps for the default variant
nwaves = 256 * 16
diag = h.DeviceBuffer(nwaves * 3 * 8)
for v in list(VARIANTS)[::-1][:2]:
    order, nt, depth, gs, S, blk, pol = v
    apply(*v, diag_ptr=diag.ptr)
    nwaves_v = 256 * (blk // 64)
    diag.fill(0)
    ver.execute()
    h.device_sync()
    d = diag.download(dtype=np.uint64)[: nwaves_v * 3].reshape(nwaves_v, 3).astype(np.float64)
    st, en, nr = d[:, 0], d[:, 1], d[:, 2]
    ok = en > 0
    t0 = st[ok].min()
    span = (en[ok].max() - t0) / 100.0  # 100 MHz ticks -> us
    out[f"diag_{tag(*v)}"] = {
        "span_us": round(span, 1),
        "wave_end_p50_us": round(float(np.percentile(en[ok] - t0, 50)) / 100, 1),
        "wave_end_p05_us": round(float(np.percentile(en[ok] - t0, 5)) / 100, 1),
        "wave_start_max_us": round(float((st[ok] - t0).max()) / 100, 1),
        "rounds_min_max": [int(nr[ok].min()), int(nr[ok].max())],
        "tail_loss_frac": round(float(1 - (en[ok] - t0).mean() / 100 / span), 4),
    }
    e = ((en - t0) / 100.0).reshape(-1, blk // 64)  # [block][wave]
    blk_max, blk_min = e.max(1), e.min(1)
    xcd = np.arange(e.shape[0]) % 8
    out[f"diag_{tag(*v)}"].update({
        "within_block_spread_us_median": round(float(np.median(blk_max - blk_min)), 1),
        "block_end_max_p05_p50_p95_us": [round(float(np.percentile(blk_max, q)), 1) for q in (5, 50, 95)],
        "xcd_mean_block_end_us": [round(float(blk_max[xcd == x].mean()), 1) for x in range(8)],
        "wave_in_block_mean_end_us": [round(float(v), 1) for v in e.mean(0)],
    })
    np.save(os.path.join(ROOT, "gpurun_out", f"diag_{tag(*v)}.npy"), d)
apply(3, 2, 3, 3, 1, 1024, 0)
print(json.dumps(out))
