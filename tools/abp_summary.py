"""Summarise tools/gpu_ab_prof.sh traces: small-run kernel medians per phase
of tools/device_stream_bench.py and the framing kernel median."""
import csv
import statistics
import sys

for tag in sys.argv[1:]:
    rows = sorted(csv.DictReader(open(f"gpurun_out/abp_{tag}/run_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000  # noqa: E731
    sr = [r for r in rows if "small_run" in r["Kernel_Name"]][-84:]
    out = [tag]
    for i, name in enumerate(["1pkt", "copy1", "64pkt", "copy64"]):
        g = sr[i * 21 + 1:(i + 1) * 21]
        sp = [(int(g[j]["Start_Timestamp"]) - int(g[j - 1]["Start_Timestamp"])) / 1000 for j in range(1, len(g))]
        out.append(f"{name} {statistics.median(map(dur, g)):.2f}/{statistics.median(sp):.2f}")
    fb = [dur(r) for r in rows if "frame_build" in r["Kernel_Name"]]
    out.append(f"framing {statistics.median(fb):.2f}" if fb else "")
    print("  ".join(out))
