"""The headline kernel's launch durations from a rocprofv3 --kernel-trace of
bench.py, next to the bench line the same process printed.

bench.py launches the C3 verify plan (crc32c_tiles_kernel<1, 3, ...> over
1024 x 128 MiB) `warmup` times untimed and then `steps` times inside the
timed region, before any other full-size verify launch (C5, the ceiling
twin and the C4 shards come after).  So the timed launches are the first
warmup + steps full-size dispatches of that kernel, minus the first warmup.

    python tools/trace_vs_line.py <kernel_trace.csv> <bench line json/log> [out.json]
"""
import csv
import json
import sys

KERNEL = "crc32c_tiles_kernel<1, 3, 1, 3, 1, 1024, 1, 0, 0, 0>"


def bench_line(path):
    for ln in open(path):
        ln = ln.strip()
        if ln.startswith("{") and '"metric"' in ln:
            return json.loads(ln)
    raise SystemExit(f"no bench line in {path}")


def main():
    trace, log = sys.argv[1], sys.argv[2]
    line = bench_line(log)
    rf = line["roofline"]
    alg = rf["alg_bytes_per_launch"]
    full_ms = alg / (rf["achieved"] * 1e9) * 1e3 * 0.5  # anything above half the line's duration is full size
    durs = []
    for r in csv.DictReader(open(trace)):
        if KERNEL in r["Kernel_Name"]:
            ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            if ms > full_ms:
                durs.append(ms)
    w, k = line["warmup"], line["steps"]
    timed = durs[w:w + k]
    avg = sum(timed) / len(timed)
    frac_trace = alg / (avg * 1e-3) / 1e9 / rf["peak"]
    out = {
        "kernel": KERNEL,
        "trace_file": trace,
        "warmup": w, "steps": k,
        "timed_launch_ms": [round(x, 4) for x in timed],
        "trace_avg_ms": round(avg, 4),
        "line_kernel_avg_ms": rf["kernel_avg_ms"],
        "alg_bytes_per_launch": alg,
        "trace_frac": round(frac_trace, 4),
        "line_frac": rf["frac"],
        "rel_diff": round(frac_trace / rf["frac"] - 1, 4),
        "line_value_GiBps": line["value"],
    }
    js = json.dumps(out)
    print(js)
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as fh:
            fh.write(js + "\n")


if __name__ == "__main__":
    main()
