"""Per-run completion of coalesced batches on or off (GPU box, diagnostic
build, HDFS_CRC32C_JOB_EARLY=1 / 0): a stream of 16 device-resident 128 MiB
blocks as jobs (4 / 8 / 16 outstanding) and as batches, each setting in
fresh processes, alternated over `rounds`; the jobs that returned at their
run's completion / at the launch's end reported per process.

    python tools/jobs_early_ab.py OUT.json [rounds] [VAR=a,b]

VAR=a,b: the same stream A/B over another environment knob of the
diagnostic build instead (e.g. HDFS_CRC32C_SPEC_POOL=32,16: the rounds per
wave from which the speculative kernels use the global pool)."""
import ctypes
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def case():
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    os.environ["DSB_DIAG"] = "1"
    import device_stream_bench as dsb
    dsb.lib = dsb._load()
    blk, nblk = dsb.wire_image(128 << 20, 9, empty_last=True)
    sb = dsb.pipelined_blocks(blk, nblk, 2048 * 65536)
    e = (ctypes.c_uint64 * 2)()
    assert dsb.lib.hdfs_crc32c_diag_job_early(e, 1) == 0
    return {"us_per_block": {k: v["us_per_block"] for k, v in sb.items() if isinstance(v, dict)},
            "waits_early_late": list(e)}


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--case":
        print(json.dumps(case()))
        return
    out_path = sys.argv[1]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    var, vals = "HDFS_CRC32C_JOB_EARLY", ("0", "1")
    if len(sys.argv) > 3:
        var, v = sys.argv[3].split("=")
        vals = tuple(v.split(","))
    res = {v: [] for v in vals}
    for r in range(rounds):
        for v in (vals if r % 2 == 0 else vals[::-1]):
            env = dict(os.environ, **{var: v})
            p = subprocess.run([sys.executable, os.path.abspath(__file__), "--case"], env=env, capture_output=True,
                               text=True, timeout=200)
            if p.returncode:
                print(p.stderr[-2000:], file=sys.stderr)
                sys.exit(p.returncode)
            o = json.loads(p.stdout.strip().splitlines()[-1])
            res[v].append(o)
            print(json.dumps({"round": r, var: v, **o}), flush=True)
    keys = res[vals[0]][0]["us_per_block"].keys()
    summary = {v: {k: round(statistics.median(o["us_per_block"][k] for o in res[v]), 1) for k in keys} for v in res}
    with open(out_path, "w") as f:
        json.dump({"summary_median_us_per_block": summary, "runs": res}, f, indent=1)
    print(json.dumps(summary))


if __name__ == "__main__":
    main()
