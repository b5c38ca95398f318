"""Debug: mailbox call sequence with per-call return codes and times."""
import ctypes, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hadoofus_amd as h
lib = h.load()
def say(*a): print(*a, file=sys.stderr, flush=True)
x64k = np.frombuffer(os.urandom(65536), np.uint8).copy()
be = h.compose_crcs([x64k.tobytes()], 512)
reg = np.frombuffer(be + x64k.tobytes(), np.uint8).copy()
fb = ctypes.c_int32(-1)
def vcall():
    t0 = time.perf_counter()
    rc = lib.hdfs_crc32c_verify_crcdata(reg.ctypes.data, 512, len(be), 65536, 2, ctypes.byref(fb))
    return rc, round((time.perf_counter() - t0) * 1e6, 1), lib.hdfs_crc32c_last_error()
def dcall(n):
    t0 = time.perf_counter()
    v = lib._hdfs_crc32c(0, x64k.ctypes.data, n)
    return v, round((time.perf_counter() - t0) * 1e6, 1)
say("launch path", vcall(), dcall(512))
mb = h.Mailbox()
say("mb stats", mb.stats())
for i in range(3): say("v", i, vcall(), mb.stats())
for i in range(3): say("d", i, dcall(512), mb.stats())
for i in range(200): dcall(65536)
say("after 200 d64k", mb.stats())
for i in range(3): say("v", i, vcall(), mb.stats())
for n in (512, 4096, 65536):
    for i in range(300): dcall(n)
    say("after 300 d", n, mb.stats())
for i in range(3): say("v", i, vcall(), mb.stats())
mb.close()
say("closed")
