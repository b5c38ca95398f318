"""Timeline of a stream of 16 device-resident 128 MiB blocks verified as jobs
with W outstanding (GPU box): host CLOCK_MONOTONIC stamps of every submit and
every wait's return, for the last of `reps` passes.  Run under
`rocprofv3 --kernel-trace` to lay the launches beside them
(tools/jobs_timeline.py --merge TRACE.csv EVENTS.json OUT.json).

    python tools/jobs_timeline.py EVENTS.json [W] [reps]"""
import csv
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def now():
    return time.clock_gettime_ns(time.CLOCK_MONOTONIC)


def run(out_path, window, reps):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import device_stream_bench as dsb
    import hadoofus_amd as h
    lib = dsb._load()
    dsb.lib = lib
    blk, nblk = dsb.wire_image(128 << 20, 9, empty_last=True)
    devs = []
    for _ in range(16):
        d = h.DeviceBuffer(blk.nbytes + 64)
        d.upload(blk)
        devs.append(d)
    h.device_sync()
    n = blk.nbytes
    arrs = [(h.abi.Packet * (nblk + 8))() for _ in range(16)]
    cnt, used = ctypes.c_size_t(0), ctypes.c_uint64(0)
    ev = []
    for _ in range(reps):
        ev = []
        q = []
        t0 = now()
        for i, d in enumerate(devs):
            if len(q) == window:
                k, j = q.pop(0)
                rc = lib.hdfs_crc32c_job_wait(j, arrs[k], nblk + 8, ctypes.byref(cnt), ctypes.byref(used))
                assert rc == 0 and cnt.value == nblk, rc
                ev.append(("ret", k, now()))
            j = ctypes.c_void_p()
            ev.append(("sub", i, now()))
            assert lib.hdfs_crc32c_verify_packets_submit(d.ptr, n, h.PROTO_V2, 512, h.CSUM_CRC32C, nblk + 8,
                                                         ctypes.byref(j)) == 0
            q.append((i, j))
        for k, j in q:
            rc = lib.hdfs_crc32c_job_wait(j, arrs[k], nblk + 8, ctypes.byref(cnt), ctypes.byref(used))
            assert rc == 0 and cnt.value == nblk, rc
            ev.append(("ret", k, now()))
        total = now() - t0
    for d in devs:
        d.free()
    with open(out_path, "w") as f:
        json.dump({"window": window, "us_per_block": round(total / 16e3, 1), "events": ev}, f)
    print(json.dumps({"window": window, "us_per_block": round(total / 16e3, 1)}))


def merge(trace_csv, events_json, out_path):
    with open(events_json) as f:
        e = json.load(f)
    ev = e["events"]
    t_first, t_last = ev[0][2], ev[-1][2]
    ks = []
    with open(trace_csv) as f:
        for row in csv.DictReader(f):
            if "spec_verify_kernel" not in row["Kernel_Name"]:
                continue
            s, t = int(row["Start_Timestamp"]), int(row["End_Timestamp"])
            if s >= t_first - 1000 and t <= t_last + 200000:
                ks.append((s, t, "batch" if "ILi0ELi1E" in row["Kernel_Name"] or "<0, 1>" in row["Kernel_Name"]
                           else "single", int(row.get("Grid_Size_X", row.get("Grid_Size", 0)) or 0)))
    items = [(t, "%s %d" % (k, i)) for k, i, t in ev]
    for s, t, kind, g in ks:
        items.append((s, "kernel %s start" % kind))
        items.append((t, "kernel %s end (%.1f us)" % (kind, (t - s) / 1e3)))
    items.sort()
    lines = ["%9.1f  %s" % ((t - t_first) / 1e3, what) for t, what in items]
    with open(out_path, "w") as f:
        json.dump({"us_per_block": e["us_per_block"], "window": e["window"], "timeline_us": lines}, f, indent=0)
    print("\n".join(lines))


if __name__ == "__main__":
    if sys.argv[1] == "--merge":
        merge(sys.argv[2], sys.argv[3], sys.argv[4])
    else:
        run(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 4, int(sys.argv[3]) if len(sys.argv) > 3 else 3)
