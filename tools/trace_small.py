import os, sys, numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import hadoofus_amd as h
h.load()
for n in (512, 4096, 65536):
    x = np.frombuffer(os.urandom(n), np.uint8)
    for _ in range(5):
        h.crc32c(0, x)
