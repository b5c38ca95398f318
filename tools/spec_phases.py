"""Where a speculative one-launch verify spends its time (GPU box, diagnostic
build): spec_verify_kernel stamps s_memrealtime (100 MHz) per workgroup at
the end of each phase, and tiles_run stamps each wave's work loop, when a
stamp buffer is set (Diag.set_tuning(2, ptr)).  Runs a device-resident v2
block of 128 MiB of payload (2 048 packets, the HDFS unit of work) and a
1 GiB run (16 384 packets) through hdfs_crc32c_verify_packets and prints,
per phase, [min, median, max] in microseconds from the earliest workgroup's
entry, next to the host wall time of the call.

Phases (per workgroup): 0 entry, 1 LDS tables filled + packet 0 decoded
(first barrier), 2 closed-form table written, work loop entered (second
barrier), 3 header checks done (last barrier), 4 the last workgroup's final
block published.  Per wave: loop start / end and rounds processed.

    python tools/spec_phases.py [out.json]     (SPH_LIB=<diag .so>: another build)"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import diaglib  # noqa: E402
import hadoofus_amd as h  # noqa: E402

# SPH_LIB: another diagnostic build (an A/B of a kernel change on one box)
lib = h.load(os.environ.get("SPH_LIB") or diaglib.DIAG_LIB_PATH)
D = diaglib.Diag(lib=lib)
NBLK = 1024
NWAVES = 4096
OFF = 98304  # kSpecStampOff (crc32c_internal.h)


def wire_image(nbytes, seed):
    """Composed v2 packets of nbytes of device-filled payload -> host bytes."""
    d = h.DeviceBuffer(nbytes)
    h.fill_splitmix64(d.ptr, nbytes // 8, seed, 0)
    h.device_sync()
    hdr, pk = h.compose_packets(None, 0, 0, h.PROTO_V2, h.CSUM_CRC32C, False, dptr=d.ptr, nbytes=nbytes)
    data = d.download()
    d.free()
    H = pk[0]["hdr_len"]
    hb = np.frombuffer(hdr, np.uint8)
    return np.concatenate([hb.reshape(len(pk), H), data.reshape(len(pk), 65536)], axis=1).reshape(-1), len(pk)


def spread(v, t0):
    v = v[v > 0]
    if not v.size:
        return None
    us = (v.astype(np.int64) - t0) / 100.0
    return [round(float(us.min()), 2), round(float(np.median(us)), 2), round(float(us.max()), 2)]


def measure(nbytes, reps=6):
    img, npk = wire_image(nbytes, 7)
    dev = h.DeviceBuffer(img.nbytes + 64)
    dev.upload(img)
    st = h.DeviceBuffer((OFF + NBLK * 8) * 8)
    arr = (h.abi.Packet * (npk + 8))()
    cnt, used = ctypes.c_size_t(0), ctypes.c_uint64(0)
    runs = []
    for rep in range(reps):
        st.fill(0)
        h.device_sync()
        D.set_tuning(2, st.ptr if rep else None)
        t = time.perf_counter()
        rc = lib.hdfs_crc32c_verify_packets(dev.ptr, img.nbytes, h.PROTO_V2, 512, h.CSUM_CRC32C, arr, npk + 8,
                                            ctypes.byref(cnt), ctypes.byref(used))
        wall = (time.perf_counter() - t) * 1e6
        assert rc >= 0 and cnt.value == npk, (rc, cnt.value)
        h.device_sync()
        if not rep:
            continue
        s = st.download(NBLK * 64, OFF * 8, dtype=np.uint64).reshape(NBLK, 8).astype(np.int64)
        w = st.download(NWAVES * 24, 0, dtype=np.uint64).reshape(NWAVES, 3).astype(np.int64)
        live = s[:, 0] > 0
        t0 = s[live, 0].min()
        run = {"wall_us": round(wall, 2), "blocks": int(live.sum())}
        for ph in range(5):
            run[f"p{ph}_us"] = spread(s[live, ph], t0)
        wl = w[:, 0] > 0
        run["waves"] = int(wl.sum())
        run["wave_loop_start_us"] = spread(w[wl, 0], t0)
        run["wave_loop_end_us"] = spread(w[wl, 1], t0)
        r = w[wl, 2]
        run["wave_rounds"] = [int(r.min()), float(np.median(r)), int(r.max())] if r.size else None
        dur = (w[wl, 1] - w[wl, 0]) / 100.0
        run["wave_loop_us"] = [round(float(dur.min()), 2), round(float(np.median(dur)), 2),
                               round(float(dur.max()), 2)] if dur.size else None
        runs.append(run)
    D.set_tuning(2, None)
    dev.free()
    st.free()
    return {"payload_bytes": nbytes, "packets": npk, "wire_bytes": int(img.nbytes), "runs": runs}


if __name__ == "__main__":
    out = {"block_128MiB": measure(128 << 20), "run_1GiB": measure(1 << 30)}
    js = json.dumps(out)
    print(js)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as fh:
            fh.write(js + "\n")
