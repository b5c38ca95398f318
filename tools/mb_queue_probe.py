"""Does the resident mailbox kernel hold up other work of the process (GPU
box, diagnostic build)?  The runtime maps a process's normal-priority
streams onto at most GPU_MAX_HW_QUEUES hardware queues; a dispatch queued
behind a persistent kernel on the same queue waits for that kernel to exit
(its 50 ms idle timeout).  Each case runs in a fresh process: the engine's
streams, then `extra` torch streams (each used once), then the mailbox
opened; three readers over one 128 MiB block through 64 KiB buffers and a
verify of the block after each, timed.  HDFS_CRC32C_MB_QUEUE=0 puts the
mailbox on a normal stream (the round-5 build until this probe), 1 on a
high-priority one (the product default).  Prints one JSON object.

    python tools/mb_queue_probe.py [out.json]"""
import ctypes
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def case(extra):
    import torch
    torch.cuda.init()  # (before the engine's library initialises HIP)
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import diaglib
    import hadoofus_amd as h
    lib = h.load(diaglib.DIAG_LIB_PATH)
    import device_stream_bench as dsb
    dsb.lib = lib
    payload = 128 << 20
    img, npk = dsb.wire_image(payload, 7)
    d = h.DeviceBuffer(len(img))
    d.upload(img)
    dst = h.DeviceBuffer(payload)
    arr = (h.abi.Packet * (npk + 8))()
    cnt, used, got = ctypes.c_size_t(0), ctypes.c_uint64(0), ctypes.c_uint64(0)

    def verify():
        t0 = time.perf_counter()
        rc = lib.hdfs_crc32c_verify_packets(d.ptr, len(img), h.PROTO_V2, 512, h.CSUM_CRC32C, arr, npk + 8,
                                            ctypes.byref(cnt), ctypes.byref(used))
        assert rc == 0 and cnt.value == npk, rc
        return round((time.perf_counter() - t0) * 1e6, 1)

    def reader():
        rd = ctypes.c_void_p()
        t0 = time.perf_counter()
        assert lib.hdfs_crc32c_reader_open(d.ptr, len(img), h.PROTO_V2, 512, h.CSUM_CRC32C, 0, payload, npk + 8,
                                           ctypes.byref(rd)) == 0
        tot, calls = 0, 0
        while True:
            vec = (h.abi.IoVec * 1)(h.abi.IoVec(dst.ptr + tot, min(64 << 10, payload - tot)))
            rc = lib.hdfs_crc32c_reader_next(rd, vec, 1, arr, npk + 8, ctypes.byref(cnt), ctypes.byref(used),
                                             ctypes.byref(got))
            calls += 1
            tot += got.value
            if rc != h.AGAIN:
                assert rc == 0 and tot == payload, (rc, tot)
                break
        lib.hdfs_crc32c_reader_close(rd)
        return round((time.perf_counter() - t0) * 1e3, 2), calls

    verify()
    streams = []
    for _ in range(extra):  # more streams of the process, each used once
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            torch.ones(1, device="cuda").add_(1)
        streams.append(s)
    torch.cuda.synchronize()
    out = {"extra_streams": extra, "readers_ms": [], "verify_after_us": []}
    with h.Mailbox() as box:
        for _ in range(3):
            ms, calls = reader()
            out["readers_ms"].append(ms)
            out["verify_after_us"].append(verify())
        out["mailbox_calls_launches"] = list(box.stats())
    out["calls_per_reader"] = calls
    d.free()
    dst.free()
    return out


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--case":
        print(json.dumps(case(int(sys.argv[2]))))
        return
    res = []
    for q in ("0", "1"):
        for extra in (0, 1, 2, 3, 5):
            env = dict(os.environ, HDFS_CRC32C_MB_QUEUE=q)
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--case", str(extra)], env=env,
                               capture_output=True, text=True, timeout=120)
            if r.returncode != 0:
                print(r.stderr[-2000:], file=sys.stderr)
                sys.exit(r.returncode)
            o = json.loads(r.stdout.strip().splitlines()[-1])
            o["mb_queue"] = int(q)
            print(json.dumps(o), file=sys.stderr, flush=True)
            res.append(o)
    js = json.dumps({"cases": res})
    print(js)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as fh:
            fh.write(js + "\n")


if __name__ == "__main__":
    main()
