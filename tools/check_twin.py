import os, sys, json
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tools')
ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tools"))
import hadoofus_amd as h, diaglib
h.load(diaglib.DIAG_LIB_PATH); D = diaglib.Diag(lib=h.load())
B = 64; BLOCK = 128 << 20; per = BLOCK // 512
data = h.DeviceBuffer(B * BLOCK); crcs = h.DeviceBuffer(B * per * 4); bms = h.DeviceBuffer(B * per // 8)
h.fill_splitmix64(data.ptr, B * BLOCK // 8, 0, 0)
segs = [h.Segment(data=data.ptr + b * BLOCK, len=BLOCK, chunk_size=512, flags=h.SEG_BE, crc_init=0,
                  crcs=crcs.ptr + b * per * 4, bitmap=bms.ptr + b * per // 8) for b in range(B)]
h.Plan(h.MODE_COMPUTE, segs).execute(); h.device_sync()
out = {}
for xcd in (0, 1):
    for pol in (0, 4):
        D.reset(); D.set_xcd_major(xcd); D.set_store_policy(pol)
        p = h.Plan(h.MODE_VERIFY, segs)
        p.execute()
        ms = p.time(5)
        out[f"xcd{xcd}_pol{pol}_GBps"] = round(B * BLOCK * (1 + 4/512 + 1/4096) / (ms * 1e-3) / 1e9, 1)
        p.destroy()
print(json.dumps(out))
