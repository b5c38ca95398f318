"""ctypes loader for the CPU ORACLE (test infrastructure only).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  The product package (hadoofus_amd/) never does.

  liboracle.so        our own C restatement of the reference algorithms
                      (oracle/crc32c_oracle.c, each function cites the
                      reference file:line it follows)
  _ref/libhdfsref.so  the reference's src/crc32c*.c compiled unchanged from
                      /root/reference (recipe: oracle/Makefile); optional.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
REF_LIB = os.path.join(HERE, "_ref", "libhdfsref.so")

_u32 = ctypes.c_uint32
_u64 = ctypes.c_uint64
_sz = ctypes.c_size_t
_vp = ctypes.c_void_p


def build():
    """Compile liboracle.so (and _ref/ when /root/reference is present)."""
    subprocess.check_call(["make", "-s", "-C", HERE, "all"])


def _bind(lib, name, restype, argtypes):
    f = getattr(lib, name)
    f.restype = restype
    f.argtypes = argtypes
    return f


CSUM_NULL, CSUM_CRC32, CSUM_CRC32C = 0, 1, 2  # include/hadoofus/objects.h:172-174


class OraclePacket(ctypes.Structure):
    """struct oracle_packet (same layout as hdfs_crc32c_packet)."""
    _fields_ = [("stream_off", _u64), ("offset_in_block", ctypes.c_int64), ("seqno", ctypes.c_int64),
                ("data_len", ctypes.c_int32), ("crc_len", ctypes.c_int32), ("header_len", _u32),
                ("error", ctypes.c_int32), ("first_bad", ctypes.c_int32), ("bad_chunks", _u32),
                ("last", ctypes.c_uint8), ("sync", ctypes.c_uint8), ("reserved", ctypes.c_uint8 * 6)]


class OracleOutPacket(ctypes.Structure):
    """struct oracle_out_packet (same layout as hdfs_crc32c_out_packet)."""
    _fields_ = [("hdr_off", _u64), ("data_off", _u64), ("offset_in_block", ctypes.c_int64),
                ("seqno", ctypes.c_int64), ("data_len", ctypes.c_int32), ("hdr_len", _u32), ("crc_len", _u32),
                ("last", ctypes.c_uint8), ("reserved", ctypes.c_uint8 * 3)]


class Oracle:
    def __init__(self, path=LIB):
        if not os.path.exists(path):
            build()
        self.lib = lib = ctypes.CDLL(path)
        self._sw = _bind(lib, "oracle_crc32c_sw", _u32, [_u32, _vp, _sz])
        self._hw = _bind(lib, "oracle_crc32c_hw", _u32, [_u32, _vp, _sz])
        self._bit = _bind(lib, "oracle_crc32c_bitwise", _u32, [_u32, _vp, _sz])
        self._zlib = _bind(lib, "oracle_crc32_zlib", _u32, [_u32, _vp, _sz])
        self._comb = _bind(lib, "oracle_crc32c_combine", _u32, [_u32, _u32, _u64])
        self._zap = _bind(lib, "oracle_zeros_apply", _u32, [_u32, _u64])
        self._ver = _bind(lib, "oracle_verify_crcdata", ctypes.c_int,
                          [_vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int,
                           ctypes.POINTER(ctypes.c_int32)])
        self._compose = _bind(lib, "oracle_compose_crcs", None,
                              [ctypes.POINTER(_vp), ctypes.POINTER(_sz), ctypes.c_int,
                               _sz, _u32, ctypes.c_int, _vp])
        self._chunks = _bind(lib, "oracle_chunk_crcs", None, [_vp, _u64, _u32, _vp, ctypes.c_int])
        self._fill = _bind(lib, "oracle_splitmix_fill", None, [_vp, _u64, _u64, _u64])
        self._bench = _bind(lib, "oracle_bench_chunks", ctypes.c_double,
                            [_vp, _u64, _u32, ctypes.c_int, ctypes.c_int, _vp, _vp])
        self._pk = _bind(lib, "oracle_verify_packets", ctypes.c_int,
                         [_vp, _u64, ctypes.c_int, _u32, ctypes.c_int, ctypes.c_int,
                          ctypes.POINTER(OraclePacket), _sz, ctypes.POINTER(_sz), ctypes.POINTER(_u64)])
        self._rd = _bind(lib, "oracle_read_packets", ctypes.c_int,
                         [_vp, _u64, ctypes.c_int, _u32, ctypes.c_int, ctypes.c_int64, ctypes.c_int64, _u64,
                          ctypes.POINTER(OraclePacket), _sz, ctypes.POINTER(_sz), ctypes.POINTER(_u64), _vp,
                          ctypes.POINTER(_u64)])
        self._opk = _bind(lib, "oracle_compose_packets", ctypes.c_int,
                          [_vp, _u64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                           _vp, _u64, ctypes.POINTER(OracleOutPacket), _sz, ctypes.POINTER(_sz),
                           ctypes.POINTER(_u64)])
        self.have_hw = bool(_bind(lib, "oracle_have_hw", ctypes.c_int, [])())

    @staticmethod
    def _buf(b):
        if isinstance(b, np.ndarray):
            return b.ctypes.data, b.nbytes
        mv = memoryview(b).cast("B")
        arr = np.frombuffer(mv, dtype=np.uint8)
        return arr.ctypes.data, arr.nbytes

    def crc32c(self, crc, data, kind="sw"):
        p, n = self._buf(data)
        f = {"sw": self._sw, "hw": self._hw, "bitwise": self._bit, "zlib": self._zlib}[kind]
        return f(crc & 0xFFFFFFFF, p, n)

    def combine(self, crc_a, crc_b, len_b):
        return self._comb(crc_a, crc_b, len_b)

    def zeros_apply(self, reg, nbytes):
        return self._zap(reg, nbytes)

    def verify_crcdata(self, region, chunksize, crcdlen, dlen, ctype=CSUM_CRC32C):
        """-> (err, first_bad) ; err 0 / 26 (CRC_LEN) / 29 (BAD_CHECKSUM)."""
        arr = np.frombuffer(bytes(region), dtype=np.uint8)
        fb = ctypes.c_int32(-1)
        err = self._ver(arr.ctypes.data, chunksize, crcdlen, dlen, ctype, ctypes.byref(fb))
        return err, fb.value

    def compose_crcs(self, iovecs, chunk=512, ctype=CSUM_CRC32C):
        """Write-path BE CRC bytes for a list of byte fragments (datanode.c:2814-2860)."""
        arrs = [np.frombuffer(bytes(v), dtype=np.uint8) for v in iovecs]
        total = sum(a.nbytes for a in arrs)
        n = len(arrs)
        bases = (_vp * max(n, 1))(*[a.ctypes.data for a in arrs])
        lens = (_sz * max(n, 1))(*[a.nbytes for a in arrs])
        out = np.zeros(((total + chunk - 1) // chunk) * 4, dtype=np.uint8)
        self._compose(bases, lens, n, total, chunk, ctype, out.ctypes.data)
        return out.tobytes()

    def chunk_crcs(self, data, chunk, hw=True, ctype=CSUM_CRC32C):
        p, n = self._buf(data)
        out = np.zeros((n + chunk - 1) // chunk, dtype=np.uint32)
        code = 2 if ctype == CSUM_CRC32 else (1 if (hw and self.have_hw) else 0)
        self._chunks(p, n, chunk, out.ctypes.data, code)
        return out

    def compose_packets(self, data, offset_in_block=0, seqno=0, proto=2, ctype=CSUM_CRC32C, finish=False):
        """Write-path packets of one write (src/datanode.c:2583-2609, 2781-2868).
        -> (header bytes, [packet dicts])."""
        p, n = self._buf(data)
        maxp = n // 512 + 3
        hdr = np.zeros(maxp * (31 + 4 * 129), dtype=np.uint8)
        arr = (OracleOutPacket * maxp)()
        npk, used = _sz(0), _u64(0)
        rc = self._opk(p, n, offset_in_block, seqno, proto, ctype, int(finish), hdr.ctypes.data, hdr.nbytes, arr,
                       maxp, ctypes.byref(npk), ctypes.byref(used))
        assert rc == 0
        return hdr[: used.value].tobytes(), [{f: getattr(arr[i], f) for f, _ in OracleOutPacket._fields_
                                              if f != "reserved"} for i in range(npk.value)]

    def verify_packets(self, stream, proto=2, chunk_size=512, ctype=CSUM_CRC32C, max_pkts=None, verify=True):
        """Packet-stream framing + per-chunk verify (src/datanode.c:2345-2494).
        -> (rc, [packet dicts], consumed)."""
        p, n = self._buf(stream)
        if max_pkts is None:
            max_pkts = n // (25 if proto == 1 else 6) + 1
        arr = (OraclePacket * max(1, max_pkts))()
        npk, used = _sz(0), _u64(0)
        rc = self._pk(p, n, proto, chunk_size, ctype, int(verify), arr, max_pkts, ctypes.byref(npk),
                      ctypes.byref(used))
        out = [{f: getattr(arr[i], f) for f, _ in OraclePacket._fields_ if f != "reserved"}
               for i in range(npk.value)]
        return rc, out, used.value

    def read_packets(self, stream, client_offset, read_len, proto=2, chunk_size=512, ctype=CSUM_CRC32C,
                     max_pkts=None, cap=None):
        """A client read of block bytes [client_offset, +read_len) over a packet
        stream into a destination of `cap` bytes (None: the whole read) --
        src/datanode.c:1476-1481, 2428-2549.  The read ends at the first
        error; a destination that fills first returns AGAIN (1000).
        -> (rc, [packet dicts], consumed, delivered bytes)."""
        p, n = self._buf(stream)
        if max_pkts is None:
            max_pkts = n // (25 if proto == 1 else 6) + 1
        arr = (OraclePacket * max(1, max_pkts))()
        npk, used, got = _sz(0), _u64(0), _u64(0)
        cap = (1 << 64) - 1 if cap is None else int(cap)
        dst = np.zeros(max(1, min(read_len, cap)), np.uint8)
        rc = self._rd(p, n, proto, chunk_size, ctype, client_offset, read_len, cap, arr, max_pkts,
                      ctypes.byref(npk), ctypes.byref(used), dst.ctypes.data, ctypes.byref(got))
        out = [{f: getattr(arr[i], f) for f, _ in OraclePacket._fields_ if f != "reserved"}
               for i in range(npk.value)]
        return rc, out, used.value, dst[:got.value].tobytes()

    def splitmix(self, nwords, seed=0, g0=0):
        out = np.empty(nwords, dtype=np.uint64)
        self._fill(out.ctypes.data, nwords, seed, g0)
        return out

    def bench_chunks(self, data, chunk, nthreads, fn="hw", ext_fn=None):
        """Time per-chunk CRCs over data; returns (seconds, crcs)."""
        p, n = self._buf(data)
        out = np.zeros((n + chunk - 1) // chunk, dtype=np.uint32)
        code = {"sw": 0, "hw": 1, "ext": 2}[fn]
        secs = self._bench(p, n, chunk, nthreads, code, ext_fn, out.ctypes.data)
        return secs, out


class Reference:
    """The reference's own CRC32C, compiled from /root/reference (optional)."""

    def __init__(self, path=REF_LIB):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        self.lib = lib = ctypes.CDLL(path)
        ui = ctypes.c_uint
        self.crc32c_fn = _bind(lib, "_hdfs_crc32c", _u32, [_u32, _vp, ui])
        self.sw_fn = _bind(lib, "_hdfs_sw_crc32c", _u32, [_u32, _vp, ui])
        self.sse42_fn = _bind(lib, "_hdfs_sse42_crc32c", _u32, [_u32, _vp, ui])
        self.sse42_addr = ctypes.cast(self.sse42_fn, _vp).value

    def crc32c(self, crc, data, kind="dispatch"):
        p, n = Oracle._buf(data)
        f = {"dispatch": self.crc32c_fn, "sw": self.sw_fn, "sse42": self.sse42_fn}[kind]
        return f(crc & 0xFFFFFFFF, p, n)


def have_reference():
    return os.path.exists(REF_LIB)


def splitmix64_np(nwords, seed=0, g0=0):
    """numpy splitmix64; identical to oracle_splitmix_fill."""
    g = np.arange(g0, g0 + nwords, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (g + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z
