"""The DIAGNOSTIC engine build (hadoofus_amd/lib/libhadoofus_crc32c_diag.so,
include/hadoofus_crc32c_diag.h) loaded beside the release library.

The release library has no tuning knobs, probes or result-dropping store
policies; experiments (tools/exp_*.py), the shape tests and bench.py's
empirical-ceiling leg use this build instead.  Loaded RTLD_LOCAL, it keeps
its own engine context on the same device and HIP runtime, so device
buffers allocated through either library are valid in both.

    d = Diag()                             # beside the release library, or
    h.load(DIAG_LIB_PATH); d = Diag(lib=h.load())   # as a tool's only library
    d.set_store_policy(4)                  # verify plans -> load-only twin
    p = d.plan(MODE_VERIFY, segments)      # an abi.Plan on the diag build
"""
import ctypes
import os

from hadoofus_amd import abi

DIAG_LIB_PATH = os.path.join(os.path.dirname(abi.LIB_PATH), "libhadoofus_crc32c_diag.so")


class Diag:
    def __init__(self, path=DIAG_LIB_PATH, lib=None):
        """lib: an already loaded diagnostic CDLL (a tool that made the
        diagnostic build its only library: h.load(DIAG_LIB_PATH))."""
        if lib is None:
            if not os.path.exists(path):
                raise ImportError(f"{path} not built; run `python -m hadoofus_amd.build`")
            lib = ctypes.CDLL(path, mode=os.RTLD_LOCAL | os.RTLD_NOW)
        self.lib = abi.bind_diag(abi.bind_product(lib))

    def _c(self, rc):
        abi._check(rc, self.lib)

    def init(self, device=-1):
        self._c(self.lib.hdfs_crc32c_init(device))

    def plan(self, mode, segments):
        return abi.Plan(mode, segments, lib=self.lib)

    def set_tile_order(self, order):
        self._c(self.lib.hdfs_crc32c_set_tile_order(order))

    def set_group_shift(self, shift):
        self._c(self.lib.hdfs_crc32c_set_group_shift(shift))

    def set_xcd_major(self, on):
        self._c(self.lib.hdfs_crc32c_set_xcd_major(int(on)))

    def set_tuning(self, nt_loads=2, diag_ptr=None):
        self._c(self.lib.hdfs_crc32c_set_tuning(nt_loads, diag_ptr))

    def set_depth(self, depth):
        self._c(self.lib.hdfs_crc32c_set_depth(depth))

    def set_shape(self, streams, block):
        self._c(self.lib.hdfs_crc32c_set_shape(streams, block))

    def set_store_policy(self, policy):
        self._c(self.lib.hdfs_crc32c_set_store_policy(policy))

    def set_runs(self, mode):
        self._c(self.lib.hdfs_crc32c_set_runs(int(mode)))

    def set_probe(self, variant=0, grid_per_cu=2, block=1024):
        self._c(self.lib.hdfs_crc32c_set_probe(variant, grid_per_cu, block))

    def probe_read(self, dptr, nbytes, iters=3, stream=None):
        g = ctypes.c_double(0)
        self._c(self.lib.hdfs_crc32c_probe_read(dptr, nbytes, stream, iters, ctypes.byref(g)))
        return g.value

    def reset(self):
        """Back to the product configuration."""
        self.set_tile_order(3)
        self.set_depth(3)
        self.set_shape(1, 1024)
        self.set_tuning(2, None)
        self.set_group_shift(3)
        self.set_store_policy(0)
        self.set_xcd_major(1)
        self.set_runs(2)
