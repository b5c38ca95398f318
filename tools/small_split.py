"""Where a launched drop-in call (_hdfs_crc32c on 512 B of host memory)
spends its time (GPU box).  Runs itself in a child process with
HDFS_CRC32C_SMALL_TRACE=1 (the engine prints per call: host launch call,
wait for the completion word, and the kernel's own phase stamps -- stage
read, compute, result -- in 10 ns ticks) and prints the medians beside the
median wall time per call.

    python tools/small_split.py [out.json]"""
import ctypes
import json
import os
import re
import statistics as st
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = 2000


def child():
    sys.path.insert(0, ROOT)
    import hadoofus_amd as h
    lib = h.load()
    buf = (ctypes.c_uint8 * 512)(*range(256), *range(256))
    f = lib._hdfs_crc32c
    f(0, buf, 512)
    wall = []
    for _ in range(N):
        t0 = time.perf_counter()
        f(0, buf, 512)
        wall.append((time.perf_counter() - t0) * 1e6)
    print(json.dumps({"wall_us_median": round(st.median(wall), 2), "wall_us_mean": round(st.mean(wall), 2)}))


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child()
        return
    env = dict(os.environ, HDFS_CRC32C_SMALL_TRACE="1")
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child"], env=env, capture_output=True,
                       text=True, timeout=120)
    if r.returncode:
        print(r.stderr[-2000:], file=sys.stderr)
        sys.exit(r.returncode)
    out = json.loads(r.stdout.strip().splitlines()[-1])
    rows = [dict((k, float(v)) for k, v in re.findall(r"(\w+_us)=([\d.]+)", l)) for l in r.stderr.splitlines()
            if l.startswith("small len=512")]
    for k in ("launch_us", "wait_us", "load_us", "comp_us", "out_us"):
        v = [x[k] for x in rows if k in x]
        if v:
            out[k + "_median"] = round(st.median(v), 2)
    out["traced_calls"] = len(rows)
    js = json.dumps(out)
    print(js)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as fh:
            fh.write(js + "\n")


if __name__ == "__main__":
    main()
