"""SQ counters of the compute-mode gather kernel with and without its slot
protocol (diagnostic store policies 2 = stores dropped, 20 = protocol skipped
and stores dropped), to see where the protocol's ~5 % goes (GPU box).

    python tools/exp_pmc_gather.py            # driver: one rocprofv3 pass per policy and counter set
    python tools/exp_pmc_gather.py run POLICY # child: 3 compute launches over 512 x 128 MiB blocks

SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles
(MI355X_MICROARCH.md); WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES.
Prints one JSON object: per policy, the largest compute dispatch's counters."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
BLOCK = 128 << 20
B = 512
SETS = [
    "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU "
    "SQ_INSTS_LDS",
    "SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_BUSY_CYCLES SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU "
    "SQ_ACTIVE_INST_LDS",
]


def child(policy):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import diaglib
    import hadoofus_amd as h
    h.load(diaglib.DIAG_LIB_PATH)
    D = diaglib.Diag(lib=h.load())
    D.reset()
    D.set_store_policy(policy)
    per = BLOCK // 512
    data = h.DeviceBuffer(B * BLOCK)
    out = h.DeviceBuffer(B * per * 4)
    h.fill_splitmix64(data.ptr, B * BLOCK // 8, 0, 0)
    segs = [h.Segment(data=data.ptr + b * BLOCK, len=BLOCK, chunk_size=512, flags=h.SEG_BE, crc_init=0,
                      crcs=out.ptr + b * per * 4) for b in range(B)]
    p = D.plan(h.MODE_COMPUTE, segs)
    for _ in range(3):
        p.execute()
    h.device_sync()


def main():
    res = {}
    for pol in (2, 20):
        for i, cs in enumerate(SETS):
            od = os.path.join(ROOT, "gpurun_out", f"pmcg_p{pol}_s{i}")
            cmd = ["timeout", "-s", "KILL", "120", "rocprofv3", "--pmc"] + cs.split() + [
                "--kernel-trace", "-d", od, "-o", "run", "--output-format", "csv", "--", sys.executable,
                os.path.abspath(__file__), "run", str(pol)]
            r = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, timeout=180)
            if r.returncode != 0:
                res.setdefault(f"p{pol}", {})[f"set{i}_error"] = r.stderr.decode()[-300:]
                continue
            rows = list(csv.DictReader(open(os.path.join(od, "run_counter_collection.csv"))))
            best = {}
            for row in rows:
                if "crc32c_tiles_kernel<0" not in row["Kernel_Name"]:
                    continue
                d = int(row["Dispatch_Id"])
                best.setdefault(d, {})[row["Counter_Name"]] = float(row["Counter_Value"])
                best[d]["_ns"] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
            if best:
                big = max(best.values(), key=lambda v: v.get("_ns", 0))  # a full-size launch
                res.setdefault(f"p{pol}", {}).update(big)
    print(json.dumps(res))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "run":
        child(int(sys.argv[2]))
    else:
        main()
