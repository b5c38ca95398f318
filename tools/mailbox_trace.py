"""Mailbox phase trace (GPU box, diagnostic build): host staging and wait
time per call plus the kernel's phase stamps, printed by the engine to stderr
under HDFS_CRC32C_SMALL_TRACE=1.  HDFS_CRC32C_MB_STAGE selects the stage
(0 pinned, 1 VRAM on large-BAR devices); HDFS_CRC32C_MB_EXP the mailbox
kernel's timing experiments (wrong results by design)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hadoofus_amd as h  # noqa: E402

lib = h.load(os.path.join(ROOT, "hadoofus_amd", "lib", "libhadoofus_crc32c_diag.so"))
rng = np.random.default_rng(1)
x64k = rng.integers(0, 256, 65536, dtype=np.uint8)
be = h.compose_crcs([x64k.tobytes()], 512)
reg = np.frombuffer(be + x64k.tobytes(), np.uint8).copy()
fb = ctypes.c_int32(-1)
with h.Mailbox():
    for name, n in (("512B", 512), ("4KiB", 4096), ("64KiB", 65536)):
        print(f"-- dropin {name}", file=sys.stderr, flush=True)
        for _ in range(6):
            lib._hdfs_crc32c(0, x64k.ctypes.data, n)
    print("-- verify_crcdata 64KiB", file=sys.stderr, flush=True)
    for _ in range(6):
        rc = lib.hdfs_crc32c_verify_crcdata(reg.ctypes.data, 512, len(be), 65536, 2, ctypes.byref(fb))
        assert rc == 0 or os.environ.get("HDFS_CRC32C_MB_EXP"), rc  # timing experiments give wrong CRCs
