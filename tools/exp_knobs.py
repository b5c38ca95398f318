"""A/B of diagnostic-build knob settings in ONE process, interleaved rounds,
on the bench's C2/C3 workload (1024 x 128 MiB, 512 B chunks; GPU box only).

    python tools/exp_knobs.py '[{"xcd_major": 0}, {"xcd_major": 1}]' [rounds]

Each variant is a dict of tools/diaglib.Diag setters (value or list of
args).  Per variant and round: compute and verify plans timed with HIP
events over 5 launches (GB/s of payload and of algorithmic bytes); parity:
verify finds exactly the corruption pattern, compute reproduces the
variant-independent CRC array digest.  Prints one JSON object."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import diaglib  # noqa: E402
import hadoofus_amd as h  # noqa: E402
from hadoofus_amd import shard  # noqa: E402

BLOCK = 128 << 20
B = int(os.environ.get("BLOCKS", "1024"))
CS = 512
ITERS = int(os.environ.get("ITERS", "5"))


def apply(D, v):
    D.reset()
    for k, a in v.items():
        getattr(D, "set_" + k)(*(a if isinstance(a, list) else [a]))


def main():
    variants = json.loads(sys.argv[1])
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    h.load(diaglib.DIAG_LIB_PATH)
    D = diaglib.Diag(lib=h.load())
    per = BLOCK // CS
    data = h.DeviceBuffer(B * BLOCK)
    exp = h.DeviceBuffer(B * per * 4)
    out = h.DeviceBuffer(B * per * 4)
    bms = h.DeviceBuffer(B * per // 8)
    h.fill_splitmix64(data.ptr, B * BLOCK // 8, 0, 0)
    mk = lambda crc, bm: [h.Segment(data=data.ptr + b * BLOCK, len=BLOCK, chunk_size=CS, flags=h.SEG_BE,  # noqa
                                    crc_init=0, crcs=crc.ptr + b * per * 4,
                                    bitmap=(bm.ptr + b * per // 8) if bm else None) for b in range(B)]
    D.reset()
    h.Plan(h.MODE_COMPUTE, mk(exp, None)).execute()
    h.device_sync()
    digest = h.stream_crc_dev(0, exp.ptr, exp.nbytes)
    for b in range(B):
        h.corrupt(data.ptr + b * BLOCK, BLOCK, CS, b * per, 65537, 7919, None)
    h.device_sync()
    want_bad = shard.expected_bad(0, B, per, 65537)
    comp, ver = h.Plan(h.MODE_COMPUTE, mk(out, None)), h.Plan(h.MODE_VERIFY, mk(exp, bms))
    alg_c, alg_v = B * BLOCK * (1 + 4 / CS), B * BLOCK * (1 + 4 / CS + 1 / (8 * CS))
    res, par = {}, {}
    for r in range(rounds):
        for i, v in enumerate(variants):
            apply(D, v)
            for name, p, alg in (("compute", comp, alg_c), ("verify", ver, alg_v)):
                p.execute()
                p.set_timing(ITERS)
                for _ in range(ITERS):
                    p.execute()
                ms, n = p.kernel_ms()
                p.set_timing(0)
                res.setdefault(f"v{i}_{name}_alg_GBps", []).append(alg / (ms / n * 1e-3) / 1e9)
            _, m = ver.results()
            # compute ran on the corrupted data: compare a corrupted-data digest across variants
            dg = h.stream_crc_dev(0, out.ptr, out.nbytes)
            par.setdefault(f"v{i}", []).append((m == want_bad, dg))
    D.reset()
    o = {"variants": variants, "blocks": B, "rounds": rounds, "clean_digest": digest}
    for k, v in res.items():
        o[k + "_median"] = round(statistics.median(v), 1)
        o[k + "_all"] = [round(x, 1) for x in v]
    digs = set(d for v in par.values() for _, d in v)
    o["parity_ok"] = all(ok for v in par.values() for ok, _ in v) and len(digs) == 1
    print(json.dumps(o))


if __name__ == "__main__":
    main()
