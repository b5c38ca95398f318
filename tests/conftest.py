import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built HIP library")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def oracle():
    from oracle import Oracle  # test infrastructure only
    return Oracle()


@pytest.fixture(scope="session")
def golden():
    import json

    import numpy as np

    g = {}
    with open(os.path.join(GOLDEN, "kats.json")) as f:
        g["kats"] = json.load(f)["kats"]
    g["sweep"] = np.load(os.path.join(GOLDEN, "edge_sweep.npy"))
    g["chunks"] = dict(np.load(os.path.join(GOLDEN, "chunk_crcs.npz")))
    with open(os.path.join(GOLDEN, "verify_cases.json")) as f:
        g["verify"] = json.load(f)["cases"]
    with open(os.path.join(GOLDEN, "block_digests.json")) as f:
        g["blocks"] = json.load(f)["blocks"]
    # CRC32 (zlib 1.2.11) leg, oracle/gen_golden_zlib.py
    with open(os.path.join(GOLDEN, "zlib_vectors.json")) as f:
        g["zlib"] = json.load(f)
    g["zlib_sweep"] = np.load(os.path.join(GOLDEN, "zlib_edge_sweep.npy"))
    g["zlib_chunks"] = dict(np.load(os.path.join(GOLDEN, "zlib_chunk_crcs.npz")))
    return g


@pytest.fixture(scope="session")
def engine():
    """The product library on a real GPU (gpu tests only)."""
    import hadoofus_amd as h
    h.load()
    arch, ncu = h.device_info()
    assert arch.startswith("gfx950"), arch
    return h
