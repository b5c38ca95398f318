"""Binary A/B of the device-stream path (GPU box): two builds of
libhadoofus_crc32c.so loaded side by side in one process (RTLD_LOCAL, each
with its own engine context), timing hdfs_crc32c_verify_packets on one
128 MiB block (2 048 v2 packets + the empty last one) and a 1 GiB run, and a
stream of 16 blocks as jobs (4 outstanding) and as batches of 8, in
interleaved rounds (A B B A ...).  For kernel changes that cannot be a
runtime knob.

    python tools/spec_ab_libs.py LIB_A LIB_B OUT.json [rounds]"""
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import hadoofus_amd as h  # noqa: E402
import device_stream_bench as dsb  # noqa: E402


def main():
    paths = {"A": sys.argv[1], "B": sys.argv[2]}
    out_path = sys.argv[3]
    rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 6
    h.load()  # the product library: allocation and the wire image
    libs = {k: h.abi.bind_product(ctypes.CDLL(p, mode=os.RTLD_LOCAL | os.RTLD_NOW)) for k, p in paths.items()}
    blk, nblk = dsb.wire_image(128 << 20, 9, empty_last=True)
    run, nrun = dsb.wire_image(1 << 30, 7)
    db = h.DeviceBuffer(blk.nbytes + 64)
    db.upload(blk)
    dr = h.DeviceBuffer(run.nbytes + 64)
    dr.upload(run)
    h.device_sync()
    res = {k: {"block_us": [], "run_1GiB_us": [], "jobs_us_per_block": [], "batch8_us_per_block": []} for k in libs}
    for r in range(rounds):
        for k in (("A", "B") if r % 2 == 0 else ("B", "A")):
            dsb.lib = libs[k]
            res[k]["block_us"].append(round(dsb.timed(db.ptr, blk.nbytes, nblk, 10)[0] * 1e6, 2))
            res[k]["run_1GiB_us"].append(round(dsb.timed(dr.ptr, run.nbytes, nrun, 5)[0] * 1e6, 2))
            sb = dsb.pipelined_blocks(blk, nblk, 2048 * 65536, reps=2)
            res[k]["jobs_us_per_block"].append(sb["jobs"]["us_per_block"])
            res[k]["batch8_us_per_block"].append(sb["batch8"]["us_per_block"])
            print(json.dumps({"round": r, "lib": k, **{m: v[-1] for m, v in res[k].items()}}), flush=True)
    summary = {k: {m: {"median": round(statistics.median(v), 2), "best": round(min(v), 2)} for m, v in d.items()}
               for k, d in res.items()}
    js = {"lib_a": paths["A"], "lib_b": paths["B"], "rounds": rounds, "summary": summary, "raw": res}
    with open(out_path, "w") as f:
        json.dump(js, f, indent=1)
    print(json.dumps(summary))


if __name__ == "__main__":
    main()
