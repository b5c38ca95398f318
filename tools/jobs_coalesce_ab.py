"""A/B of job coalescing in one process (GPU box, diagnostic build): a stream
of 16 device-resident 128 MiB blocks (2 048 v2 packets + the empty last one),
one asynchronous job per block with 4 / 8 / 16 outstanding, the queue-and-
batch product policy (hdfs_crc32c_set_job_coalesce(1)) against launching
every job at its submit (0, round 5), interleaved over 3 rounds; the
synchronous call and explicit batches beside them.  Writes one JSON object.

    python tools/jobs_coalesce_ab.py OUT.json"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
os.environ["DSB_DIAG"] = "1"
import device_stream_bench as dsb  # noqa: E402


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/jobs_coalesce_ab.json"
    dsb.lib = dsb._load()
    blk, nblk = dsb.wire_image(128 << 20, 9, empty_last=True)
    rounds = []
    for r in range(3):
        one = {}
        for mode in ((1, 3, 0) if r % 2 else (0, 3, 1)):
            assert dsb.lib.hdfs_crc32c_set_job_coalesce(mode) == 0
            one[f"coalesce{mode}"] = dsb.pipelined_blocks(blk, nblk, 2048 * 65536)
            print(json.dumps({"round": r, "mode": mode, "jobs": one[f"coalesce{mode}"]["jobs"]}), flush=True)
        rounds.append(one)
    dsb.lib.hdfs_crc32c_set_job_coalesce(1)
    keys = ("sync", "jobs", "jobs_inflight8", "jobs_inflight16", "batch4", "batch8", "batch16")
    best = {f"coalesce{m}": {k: min(rd[f"coalesce{m}"][k]["us_per_block"] for rd in rounds) for k in keys}
            for m in (0, 1, 3)}
    res = {"rounds": rounds, "best_us_per_block": best,
           "note": "diagnostic build; us per 128 MiB block, best of 3 interleaved rounds (each itself best of 3); "
                   "coalesce1 = the product policy, coalesce0 = every job launched at its submit (round 5), "
                   "coalesce3 = as 1 but no lone run sent out behind a running launch"}
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(best))


if __name__ == "__main__":
    main()
