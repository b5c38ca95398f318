"""HBM traffic of the tiled kernels from rocprofv3 PMC counters.

Runs two SEPARATE counter passes (FETCH_SIZE, then WRITE_SIZE; each with
kernel-trace only) over the bench, and applies the gfx950 correction from
MI355X_MICROARCH.md: FETCH_SIZE reports half the bytes of a wide coalesced
streaming read, so read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE x 1024 is
taken as is (exact for 16-B stores, uncalibrated for our 1- and 4-B stores:
an upper-bound-ish figure).  Writes profiles/<round>/pmc_traffic.json.

    python tools/pmc_traffic.py r01 [--blocks 512]     (GPU box)
"""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BLOCK = 128 << 20


def run_pass(counter, outdir, blocks):
    cmd = ["rocprofv3", "--pmc", counter, "--kernel-trace", "-d", outdir, "-o", "run", "--output-format", "csv",
           "--", sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1", "--no-cpu",
           "--no-extra", "--blocks", str(blocks)]
    subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, timeout=600)
    rows = list(csv.DictReader(open(os.path.join(outdir, "run_counter_collection.csv"))))
    vals = {}
    for r in rows:
        name = r["Kernel_Name"]
        if "crc32c_tiles_kernel" not in name or r["Counter_Name"] != counter:
            continue
        mode = "verify" if "crc32c_tiles_kernel<1" in name else "compute"
        vals.setdefault(mode, []).append(float(r["Counter_Value"]))
    return vals


def main():
    rnd = sys.argv[1] if len(sys.argv) > 1 else "r01"
    blocks = int(sys.argv[sys.argv.index("--blocks") + 1]) if "--blocks" in sys.argv else 512
    base = os.path.join(ROOT, "gpurun_out", f"pmc_{rnd}")
    fetch = run_pass("FETCH_SIZE", base + "_fetch", blocks)
    write = run_pass("WRITE_SIZE", base + "_write", blocks)
    nbytes = blocks * BLOCK
    out = {"round": rnd, "chunk_size": 512, "blocks": blocks, "payload_bytes_per_launch": nbytes,
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes with --kernel-trace; "
                     "read = 2*FETCH_SIZE*1024 (gfx950), write = WRITE_SIZE*1024",
           "kernels": {}}
    for mode in ("verify", "compute"):
        # the full-size launches are the largest ones of that mode
        f = max(fetch.get(mode, [0])) * 1024 * 2
        w = max(write.get(mode, [0])) * 1024
        alg = nbytes + 4 * nbytes / 512 + (nbytes / 4096 if mode == "verify" else 0)
        out["kernels"][mode] = {"read_bytes": int(f), "write_bytes": int(w), "traffic_bytes": int(f + w),
                                "alg_bytes": int(alg), "traffic_over_alg": round((f + w) / alg, 4),
                                "traffic_bytes_per_payload_byte": (f + w) / nbytes}
    # written under gpurun_out/ too (only that directory comes back from the GPU box)
    for dst in (os.path.join(ROOT, "profiles", rnd), os.path.join(ROOT, "gpurun_out")):
        os.makedirs(dst, exist_ok=True)
        with open(os.path.join(dst, "pmc_traffic.json"), "w") as fh:
            json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
