"""Which streams wait behind the resident mailbox kernel (GPU box, diagnostic
build)?  Each case runs in a fresh process: `nhi` high-priority and `nlo`
normal streams created through HIP before the mailbox opens (a host
process's own streams: torch's, RCCL's), the mailbox opened with its stream
made per HDFS_CRC32C_MB_QUEUE (1 high-priority, the product; 2 CU-masked;
0 normal), then per stream one small hipMemsetAsync timed to completion, a
NULL-stream hipMemcpy, and an engine verify (its plan freed and made again:
a hipFree).  A stream sharing the mailbox's hardware queue showed the
kernel's idle exit (48 ms) before the kernel learned to yield to work queued
behind it (round 6).

    python tools/mb_queue_share.py OUT.json"""
import ctypes
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def case(nhi, nlo):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import diaglib
    import numpy as np
    import hadoofus_amd as h
    lib = h.load(diaglib.DIAG_LIB_PATH)
    hip = ctypes.CDLL("libamdhip64.so")
    vp = ctypes.c_void_p
    hip.hipStreamCreateWithPriority.argtypes = [ctypes.POINTER(vp), ctypes.c_uint, ctypes.c_int]
    hip.hipDeviceGetStreamPriorityRange.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
    hip.hipMemsetAsync.argtypes = [vp, ctypes.c_int, ctypes.c_size_t, vp]
    hip.hipStreamSynchronize.argtypes = [vp]
    hip.hipMemcpy.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_int]
    lo, hi = ctypes.c_int(0), ctypes.c_int(0)
    assert hip.hipDeviceGetStreamPriorityRange(ctypes.byref(lo), ctypes.byref(hi)) == 0
    n = 64 << 20
    data = h.DeviceBuffer(n)
    h.fill_splitmix64(data.ptr, n // 8, 4, 0)
    crcs = h.DeviceBuffer(n // 512 * 4)
    bm = h.DeviceBuffer(n // 512 // 8)
    seg = [h.Segment(data=data.ptr, len=n, chunk_size=512, flags=h.SEG_BE, crc_init=0, crcs=crcs.ptr, bitmap=bm.ptr)]
    h.Plan(h.MODE_COMPUTE, seg).execute()
    scratch = h.DeviceBuffer(4096)
    streams = []
    for k in range(nhi + nlo):
        s = vp()
        assert hip.hipStreamCreateWithPriority(ctypes.byref(s), 1, hi.value if k < nhi else lo.value) == 0
        assert hip.hipMemsetAsync(scratch.ptr, 0, 64, s) == 0  # used once
        assert hip.hipStreamSynchronize(s) == 0
        streams.append(s)
    host = np.zeros(64, np.uint8)
    out = {"nhi": nhi, "nlo": nlo, "stream_ms": [], "memcpy_ms": [], "verify_ms": []}
    with h.Mailbox() as box:
        assert h.crc32c(0, b"123456789") == 0xE3069283  # (through the mailbox)
        time.sleep(0.002)
        for s in streams:
            t0 = time.perf_counter()
            assert hip.hipMemsetAsync(scratch.ptr, 1, 64, s) == 0
            assert hip.hipStreamSynchronize(s) == 0
            out["stream_ms"].append(round((time.perf_counter() - t0) * 1e3, 3))
        for _ in range(2):
            t0 = time.perf_counter()
            assert hip.hipMemcpy(scratch.ptr, host.ctypes.data, 64, 1) == 0
            out["memcpy_ms"].append(round((time.perf_counter() - t0) * 1e3, 3))
            t0 = time.perf_counter()
            p = h.Plan(h.MODE_VERIFY, seg)
            p.execute()
            _, m = p.results()
            assert m == 0
            out["verify_ms"].append(round((time.perf_counter() - t0) * 1e3, 3))
        t0 = time.perf_counter()
        assert h.crc32c(0, b"123456789") == 0xE3069283  # still served (relaunched if it yielded)
        out["call_after_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
        out["mailbox_calls_launches"] = list(box.stats())
    return out


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--case":
        print(json.dumps(case(int(sys.argv[2]), int(sys.argv[3]))))
        return
    res = []
    for q in ("1", "2"):
        for nhi, nlo in ((0, 0), (1, 0), (3, 0), (4, 0), (8, 0), (4, 4)):
            env = dict(os.environ, HDFS_CRC32C_MB_QUEUE=q)
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--case", str(nhi), str(nlo)], env=env,
                               capture_output=True, text=True, timeout=120)
            if r.returncode != 0:
                print(r.stderr[-2000:], file=sys.stderr)
                sys.exit(r.returncode)
            o = json.loads(r.stdout.strip().splitlines()[-1])
            o["mb_queue"] = int(q)
            print(json.dumps(o), flush=True)
            res.append(o)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as fh:
            json.dump({"cases": res}, fh, indent=1)


if __name__ == "__main__":
    main()
