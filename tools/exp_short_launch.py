"""Short verify launches (GPU box, diagnostic build): the tiled kernel's time
on one 128 MiB block -- the HDFS unit of work -- and on 64 / 256 MiB and
1 GiB, aligned plans, across kernel shapes and schedule knobs, kernel time
from HIP events (hdfs_crc32c_plan_kernel_ms), 2 interleaved passes.  Where
does a short launch lose against the long-launch rate, and does any shape
lose less?

    HDFS_CRC32C_SMALL_RULE=0 python tools/exp_short_launch.py [out.json]
(SMALL_RULE=0 keeps schedule 3 on small launches so its shapes can be
swept; with the default 1 the product's small-launch rule applies.)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import diaglib  # noqa: E402
import hadoofus_amd as h  # noqa: E402

lib = h.load(diaglib.DIAG_LIB_PATH)
D = diaglib.Diag(lib=lib)
MiB = 1 << 20
SMALL_RULE = os.environ.get("HDFS_CRC32C_SMALL_RULE", "1")

# (name, order, nt, depth, streams, group shift, xcd dealing)
CONFIGS = [("s3_d3_product_shape", 3, 2, 3, 1, 3, 1)]
if SMALL_RULE == "0":
    CONFIGS += [
        ("s3_d4", 3, 2, 4, 1, 3, 1),
        ("s3_g2", 3, 2, 3, 1, 2, 1),
        ("s3_g1", 3, 2, 3, 1, 1, 1),
        ("s3_g4", 3, 2, 3, 1, 4, 1),
        ("s3_xcd0", 3, 2, 3, 1, 3, 0),
        ("s3_xcd2", 3, 2, 3, 1, 3, 2),
        ("s3_nt1_d4", 3, 1, 4, 1, 3, 1),
        ("s3_s2_d2", 3, 1, 2, 2, 3, 1),
        ("s2_d3", 2, 1, 3, 1, 3, 1),
    ]


def configure(order, nt, depth, streams, gshift, xcd):
    D.set_tile_order(order)
    D.set_tuning(nt, None)
    D.set_depth(depth)
    D.set_shape(streams, 1024)
    D.set_group_shift(gshift)
    D.set_xcd_major(xcd)


def main():
    big = 1 << 30
    data = h.DeviceBuffer(big)
    crcs = h.DeviceBuffer(big // 512 * 4)
    bm = h.DeviceBuffer(big // 512 // 8 + 4096)
    h.fill_splitmix64(data.ptr, big // 8, 5, 0)
    h.device_sync()
    D.reset()
    comp = h.Plan(h.MODE_COMPUTE, [h.Segment(data=data.ptr, len=big, chunk_size=512, flags=h.SEG_BE, crc_init=0,
                                             crcs=crcs.ptr)], lib=lib)
    comp.execute()
    h.device_sync()
    comp.destroy()
    layouts = {
        "block_128MiB_1seg": [(0, 128 * MiB)],
        "block_128MiB_2048x64KiB": [(k * 65536, 65536) for k in range(2048)],
        "64MiB_1seg": [(0, 64 * MiB)],
        "256MiB_1seg": [(0, 256 * MiB)],
        "1GiB_1seg": [(0, big)],
    }
    res = {}
    for rep in range(2):
        for name, *knobs in CONFIGS:
            try:
                configure(*knobs)
            except h.CRC32CError as e:
                res.setdefault(name, {})["error"] = str(e)[:120]
                continue
            for lay, segs in layouts.items():
                sg = [h.Segment(data=data.ptr + o, len=n, chunk_size=512, flags=h.SEG_BE, crc_init=0,
                                crcs=crcs.ptr + o // 128, bitmap=bm.ptr + o // 4096) for o, n in segs]
                p = D.plan(h.MODE_VERIFY, sg)
                p.execute()
                p.results()
                p.set_timing(20)
                for _ in range(20):
                    p.execute()
                ms, n = p.kernel_ms()
                fb, m = p.results()
                assert m == 0, (name, lay, m)
                p.destroy()
                nbytes = sum(n for _, n in segs)
                us = ms / n * 1e3
                r = res.setdefault(name, {}).setdefault(lay, [])
                r.append({"us": round(us, 2), "GBps_alg": round(nbytes * (1 + 4 / 512 + 1 / 4096) / us / 1e3, 1)})
    D.reset()
    out = {"small_rule": SMALL_RULE, "configs": {c[0]: c[1:] for c in CONFIGS}, "results": res}
    js = json.dumps(out)
    print(js)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as fh:
            fh.write(js + "\n")


if __name__ == "__main__":
    main()
