"""Overlap of asynchronous verify jobs on the GPU (run under rocprofv3
--kernel-trace): 16 device-resident 128 MiB block transfers verified as jobs
with 1..4 in flight (tools/device_stream_bench.pipelined_blocks), one pass per
setting, markers between them; then the trace is read back for the
spec_verify_kernel dispatches' queues, starts and ends.

    rocprofv3 --kernel-trace -d D -o run --output-format csv -- python3 tools/jobs_overlap.py
    python tools/jobs_overlap.py analyse D/run_kernel_trace.csv [out.json]
"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run():
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import device_stream_bench as dsb
    import hadoofus_amd as h
    dsb.lib = h.load()
    blk, nblk = dsb.wire_image(128 << 20, 9, empty_last=True)
    out = {}
    for inflight in (1, 2, 3, 4):
        r = dsb.pipelined_blocks(blk, nblk, 2048 * 65536, nblocks=16, inflight=inflight, reps=2)
        out[inflight] = r
        h.device_sync()
    print(json.dumps(out))


def analyse(path, out_path=None):
    rows = [r for r in csv.DictReader(open(path)) if "spec_verify_kernel" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"]) for r in rows]
    # concurrency: for each dispatch, how long it overlapped any other
    over, tot = 0, 0
    for i, (s, e, q) in enumerate(ev):
        tot += e - s
        lo = s
        for j in range(max(0, i - 8), min(len(ev), i + 9)):
            if j == i:
                continue
            s2, e2, _ = ev[j]
            a, b = max(s, s2), min(e, e2)
            if b > a:
                over += b - a
    res = {"dispatches": len(ev), "queues": sorted(set(q for _, _, q in ev)),
           "avg_us": round(tot / max(1, len(ev)) / 1e3, 2),
           "overlap_frac": round(over / max(1, tot), 3),
           "first_40": [(round((s - ev[0][0]) / 1e3, 1), round((e - s) / 1e3, 1), q) for s, e, q in ev[:40]]}
    js = json.dumps(res)
    print(js)
    if out_path:
        open(out_path, "w").write(js + "\n")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "analyse":
        analyse(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
    else:
        run()
