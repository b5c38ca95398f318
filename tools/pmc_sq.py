"""SQ / TA / TD / TCP counters of the product's compute (gather) and verify
kernels in one child process per counter pass (GPU box; rocprofv3 --pmc,
kernel-trace only beside it, one pass per counter group within the per-block
limits of MI355X_MICROARCH.md).  The child runs 3 compute launches then 3
verify launches over 512 x 128 MiB blocks (512 B chunks; the compute output
is the verify's expected CRCs); per kernel the longest dispatch's counters
are kept.

    python tools/pmc_sq.py [out.json]   # driver
    python tools/pmc_sq.py run          # child
    python tools/pmc_sq.py derive f.json  # recompute the derived figures

Derived (per kernel): effective clock, instructions per 4 KiB round, the
average number of vector-memory instructions in flight per wave
(SQ_INST_LEVEL_VMEM / SQ_WAVE_CYCLES... quad-cycle units as
MI355X_MICROARCH.md states), cycles per VMEM read / write instruction, the
L1->L2 write latency (TCP_TCC_WRITE_REQ_LATENCY / TCP_TCC_WRITE_REQ) and
HBM traffic over the algorithmic bytes."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
BLOCK = 128 << 20
B = 512
PASSES = {
    "clk": "GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY "
           "SQ_ACTIVE_INST_ANY",
    "lds": "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS",
    "vmem": "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_INST_LEVEL_VMEM "
            "SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_INSTS_SMEM",
    "fifo": "SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_WAIT_INST_LDS "
            "SQ_INSTS_BRANCH TA_BUFFER_WRITE_WAVEFRONTS TA_BUFFER_COALESCED_WRITE_CYCLES TD_WRITE_ACKT_WAVEFRONT "
            "TD_STORE_WAVEFRONT",
    "tcp": "TCP_TCC_WRITE_REQ TCP_TCC_WRITE_REQ_LATENCY TCP_PENDING_STALL_CYCLES TCP_TCP_TA_DATA_STALL_CYCLES",
    "fetch": "FETCH_SIZE",
    "write": "WRITE_SIZE",
}


def child():
    import hadoofus_amd as h
    h.load()
    per = BLOCK // 512
    data = h.DeviceBuffer(B * BLOCK)
    crcs = h.DeviceBuffer(B * per * 4)
    bms = h.DeviceBuffer(B * per // 8)
    h.fill_splitmix64(data.ptr, B * BLOCK // 8, 0, 0)
    segs = [h.Segment(data=data.ptr + b * BLOCK, len=BLOCK, chunk_size=512, flags=h.SEG_BE, crc_init=0,
                      crcs=crcs.ptr + b * per * 4, bitmap=bms.ptr + b * per // 8) for b in range(B)]
    comp = h.Plan(h.MODE_COMPUTE, segs)
    for _ in range(3):
        comp.execute()
    h.device_sync()
    ver = h.Plan(h.MODE_VERIFY, segs)
    for _ in range(3):
        ver.execute()
    _, m = ver.results()
    assert m == 0, m


def kernel_of(name):
    if "crc32c_tiles_kernel<0" in name:
        return "compute"
    if "crc32c_tiles_kernel<1" in name:
        return "verify"
    return None


def main(out_path):
    res = {"compute": {}, "verify": {}}
    env = dict(os.environ, TMPDIR="/tmp")
    for tag, counters in PASSES.items():
        od = os.path.join(ROOT, "gpurun_out", f"pmcsq_{tag}")
        cmd = ["timeout", "-s", "KILL", "150", "rocprofv3", "--pmc"] + counters.split() + [
            "--kernel-trace", "-d", od, "-o", "run", "--output-format", "csv", "--", sys.executable,
            os.path.abspath(__file__), "run"]
        r = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, env=env, cwd="/tmp", timeout=200)
        if r.returncode != 0:
            res.setdefault("errors", {})[tag] = r.stderr.decode(errors="replace")[-400:]
            if r.returncode in (124, 134, 137, 139, -9):
                break
            continue
        path = None
        for dp, _, files in os.walk(od):
            for f in files:
                if f.endswith("counter_collection.csv"):
                    path = os.path.join(dp, f)
        rows = list(csv.DictReader(open(path)))
        disp = {}
        for row in rows:
            k = kernel_of(row["Kernel_Name"])
            if not k:
                continue
            d = disp.setdefault((k, int(row["Dispatch_Id"])), {})
            d[row["Counter_Name"]] = d.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
            d["_ns"] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
        for k in ("compute", "verify"):
            cand = [v for (kk, _), v in disp.items() if kk == k]
            if cand:
                big = max(cand, key=lambda v: v["_ns"])
                ns = big.pop("_ns")
                res[k].update(big)
                res[k][f"dispatch_ms_{tag}"] = round(ns / 1e6, 4)
    derive(res)
    res["method"] = ("rocprofv3 --pmc, one pass per counter group (tools/pmc_sq.py), kernel-trace only beside it; "
                     "child: 3 compute then 3 verify launches over 512 x 128 MiB blocks, product library; per kernel "
                     "the longest dispatch; SQ cycle counters in quad-cycles, FETCH/WRITE_SIZE in KiB (FETCH_SIZE "
                     "doubled for traffic_over_alg, the gfx950 correction); GRBM counters summed over the 8 XCDs")
    s = json.dumps(res, indent=1)
    if out_path:
        open(out_path, "w").write(s)
    print(s)


XCDS = 8  # MI355X: GRBM_GUI_ACTIVE / GRBM_COUNT come summed over the XCDs


def derive(res):
    """Per-kernel derived figures from the raw counters (in place)."""
    rounds = B * BLOCK // 4096
    for k, c in res.items():
        if k not in ("compute", "verify") or not c:
            continue
        der = {}
        ms = c.get("dispatch_ms_clk")
        if "GRBM_GUI_ACTIVE" in c and ms:
            der["effective_clock_GHz"] = round(c["GRBM_GUI_ACTIVE"] / XCDS / (ms * 1e-3) / 1e9, 3)
        for n in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_RD",
                  "SQ_INSTS_VMEM_WR", "SQ_INSTS_BRANCH"):
            if n in c:
                der[f"{n.lower()}_per_round"] = round(c[n] / rounds, 2)
        if "SQ_INST_LEVEL_VMEM" in c and "SQ_WAVE_CYCLES" in c:
            der["vmem_insts_in_flight_per_wave"] = round(c["SQ_INST_LEVEL_VMEM"] / c["SQ_WAVE_CYCLES"], 3)
        for rw in ("RD", "WR"):
            if f"SQ_INST_CYCLES_VMEM_{rw}" in c and c.get(f"SQ_INSTS_VMEM_{rw}"):
                der[f"cycles_per_vmem_{rw.lower()}"] = round(c[f"SQ_INST_CYCLES_VMEM_{rw}"] / c[f"SQ_INSTS_VMEM_{rw}"], 2)
        if c.get("TCP_TCC_WRITE_REQ"):
            der["tcp_write_latency_cycles"] = round(c.get("TCP_TCC_WRITE_REQ_LATENCY", 0) / c["TCP_TCC_WRITE_REQ"], 1)
        if "SQ_WAIT_ANY" in c and "SQ_WAVE_CYCLES" in c:
            der["wait_frac_of_wave_cycles"] = round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 4)
            der["active_frac_of_wave_cycles"] = round(c.get("SQ_ACTIVE_INST_ANY", 0) / c["SQ_WAVE_CYCLES"], 4)
        alg = B * BLOCK * (1 + 4 / 512 + (1 / 4096 if k == "verify" else 0))
        if "FETCH_SIZE" in c or "WRITE_SIZE" in c:
            # gfx950: FETCH_SIZE counts half the bytes of wide streaming reads
            # (MI355X_MICROARCH.md, HBM/rocprofv3 section): doubled
            der["traffic_over_alg"] = round((2 * c.get("FETCH_SIZE", 0) + c.get("WRITE_SIZE", 0)) * 1024 / alg, 4)
        c["derived"] = der


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "run":
        child()
    elif len(sys.argv) > 2 and sys.argv[1] == "derive":  # re-derive a committed result (no GPU)
        r = json.load(open(sys.argv[2]))
        derive(r)
        open(sys.argv[2], "w").write(json.dumps(r, indent=1))
    else:
        main(sys.argv[1] if len(sys.argv) > 1 else None)
