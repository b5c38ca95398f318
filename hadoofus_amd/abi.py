"""ctypes mirror of include/hadoofus_crc32c.h.

Function names follow the reference's interface for this path:
  crc32c(crc, buf)                 <- _hdfs_crc32c (src/crc32c.h:13)
  verify_crcdata(region, ...)      <- _verify_crcdata (src/datanode.c:2931-2963)
  compose_crcs(iovecs, chunk)      <- CRC loop of _compose_data_packet_header
                                      (src/datanode.c:2814-2860)
plus the additive device batch API (Plan / Segment) and device-memory helpers.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libhadoofus_crc32c.so")

# include/objects.h:169-175
CSUM_NULL, CSUM_CRC32, CSUM_CRC32C = 0, 1, 2
# include/objects.h:21-113 (enum hdfs_error_numeric values)
ERR_UNSUPPORTED_CHECKSUM = 8
ERR_INVALID_PACKETHEADERPROTO = 18
ERR_PACKET_SIZE = 25
ERR_CRC_LEN = 26
ERR_UNEXPECTED_CRC_LEN = 27
ERR_UNEXPECTED_READ_OFFSET = 28
ERR_BAD_CHECKSUM = 29
ERR_BAD_LASTPACKET = 32
EIO = -5       # hdfs_crc32c_read_packets_fd: a write to the fd failed
READ_ALL = -1  # read_packets: whole payloads, no client read window
AGAIN = 1000   # read_packets: the destination filled before the read completed (resumable)
ABI_VERSION = 5  # include/hadoofus_crc32c.h HDFS_CRC32C_ABI_VERSION these bindings are written for
MODE_COMPUTE, MODE_VERIFY = 0, 1
PROTO_V1, PROTO_V2 = 1, 2
SEG_BE, SEG_RAW, SEG_CRC32 = 1, 2, 4

_u32, _u64, _vp, _sz, _int = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int


class CRC32CError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"hadoofus_crc32c error {code}: {msg}")
        self.code = code


class Segment(ctypes.Structure):
    """struct hdfs_crc32c_segment."""
    _fields_ = [
        ("data", _vp),
        ("len", _u64),
        ("chunk_size", _u32),
        ("flags", _u32),
        ("crc_init", _u32),
        ("reserved", _u32),
        ("crcs", _vp),
        ("bitmap", _vp),
    ]


class IoVec(ctypes.Structure):
    """hdfs_crc32c_iovec: one device buffer of a read's destination."""
    _fields_ = [("base", ctypes.c_void_p), ("len", ctypes.c_uint64)]


class Packet(ctypes.Structure):
    """struct hdfs_crc32c_packet."""
    _fields_ = [
        ("stream_off", _u64),
        ("offset_in_block", ctypes.c_int64),
        ("seqno", ctypes.c_int64),
        ("data_len", ctypes.c_int32),
        ("crc_len", ctypes.c_int32),
        ("header_len", _u32),
        ("error", ctypes.c_int32),
        ("first_bad", ctypes.c_int32),
        ("bad_chunks", _u32),
        ("last", ctypes.c_uint8),
        ("sync", ctypes.c_uint8),
        ("reserved", ctypes.c_uint8 * 6),
    ]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_ if f != "reserved"}


class OutPacket(ctypes.Structure):
    """struct hdfs_crc32c_out_packet (write path)."""
    _fields_ = [
        ("hdr_off", _u64),
        ("data_off", _u64),
        ("offset_in_block", ctypes.c_int64),
        ("seqno", ctypes.c_int64),
        ("data_len", ctypes.c_int32),
        ("hdr_len", _u32),
        ("crc_len", _u32),
        ("last", ctypes.c_uint8),
        ("reserved", ctypes.c_uint8 * 3),
    ]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_ if f != "reserved"}


_lib = None


def _bind(lib, name, res, args):
    f = getattr(lib, name)
    f.restype = res
    f.argtypes = args
    return f


def bind_product(lib):
    """Bind the C ABI of include/hadoofus_crc32c.h + include/crc32c.h on lib."""
    for n in ("_hdfs_crc32c", "_hdfs_sse42_crc32c", "_hdfs_armv8_crc32c", "_hdfs_sw_crc32c"):
        _bind(lib, n, _u32, [_u32, _vp, ctypes.c_uint])
    _bind(lib, "hdfs_crc32c_last_error", ctypes.c_char_p, [])
    _bind(lib, "hdfs_crc32c_init", _int, [_int])
    _bind(lib, "hdfs_crc32c_device_info", _int, [_int, ctypes.c_char_p, _sz, ctypes.POINTER(_int)])
    _bind(lib, "hdfs_crc32c_bound_device", _int, [ctypes.POINTER(_int), ctypes.c_char_p, _sz])
    _bind(lib, "hdfs_crc32c_plan_create", _int, [ctypes.POINTER(_vp), _int, ctypes.POINTER(Segment), _sz])
    _bind(lib, "hdfs_crc32c_plan_execute", _int, [_vp, _vp])
    _bind(lib, "hdfs_crc32c_plan_results", _int, [_vp, _vp, ctypes.POINTER(_u32), _sz, ctypes.POINTER(_u64)])
    _bind(lib, "hdfs_crc32c_plan_set_timing", _int, [_vp, _int])
    _bind(lib, "hdfs_crc32c_plan_kernel_ms", _int, [_vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_int)])
    _bind(lib, "hdfs_crc32c_plan_stats", _int, [_vp, ctypes.POINTER(_u64), ctypes.POINTER(_u64), ctypes.POINTER(_u64)])
    _bind(lib, "hdfs_crc32c_plan_destroy", None, [_vp])
    _bind(lib, "hdfs_crc32c_plan_time", _int, [_vp, _vp, _int, ctypes.POINTER(ctypes.c_double)])
    _bind(lib, "hdfs_crc32c_stream_dev", _int, [_u32, _vp, _u64, ctypes.POINTER(_u32)])
    _bind(lib, "hdfs_crc32c_stream_ex", _int, [_int, _u32, _vp, _u64, ctypes.POINTER(_u32)])
    _bind(lib, "hdfs_crc32c_verify_crcdata", _int,
          [_vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _int, ctypes.POINTER(ctypes.c_int32)])
    _bind(lib, "hdfs_crc32c_compose_crcs", _int,
          [ctypes.POINTER(_vp), ctypes.POINTER(_sz), _int, _sz, _u32, _int, _vp])
    for name in ("hdfs_crc32c_parse_packets", "hdfs_crc32c_verify_packets"):
        _bind(lib, name, _int, [_vp, _u64, _int, _u32, _int, ctypes.POINTER(Packet), _sz,
                                ctypes.POINTER(_sz), ctypes.POINTER(_u64)])
    _bind(lib, "hdfs_crc32c_read_packets", _int,
          [_vp, _u64, _int, _u32, _int, ctypes.c_int64, ctypes.c_int64, ctypes.POINTER(IoVec), _int,
           ctypes.POINTER(Packet), _sz, ctypes.POINTER(_sz), ctypes.POINTER(_u64), ctypes.POINTER(_u64)])
    _bind(lib, "hdfs_crc32c_verify_packets_submit", _int,
          [_vp, _u64, _int, _u32, _int, _sz, ctypes.POINTER(_vp)])
    _bind(lib, "hdfs_crc32c_job_wait", _int,
          [_vp, ctypes.POINTER(Packet), _sz, ctypes.POINTER(_sz), ctypes.POINTER(_u64)])
    _bind(lib, "hdfs_crc32c_verify_blocks_submit", _int,
          [ctypes.POINTER(_vp), ctypes.POINTER(_u64), _sz, _int, _u32, _int, _sz, ctypes.POINTER(_vp)])
    _bind(lib, "hdfs_crc32c_job_wait_blocks", _int,
          [_vp, ctypes.POINTER(Packet), _sz, ctypes.POINTER(_sz), ctypes.POINTER(_u64), ctypes.POINTER(_int)])
    _bind(lib, "hdfs_crc32c_reader_open", _int,
          [_vp, _u64, _int, _u32, _int, ctypes.c_int64, ctypes.c_int64, _sz, ctypes.POINTER(_vp)])
    _bind(lib, "hdfs_crc32c_reader_next", _int,
          [_vp, ctypes.POINTER(IoVec), _int, ctypes.POINTER(Packet), _sz, ctypes.POINTER(_sz), ctypes.POINTER(_u64),
           ctypes.POINTER(_u64)])
    _bind(lib, "hdfs_crc32c_reader_close", None, [_vp])
    _bind(lib, "hdfs_crc32c_read_packets_fd", _int,
          [_vp, _u64, _int, _u32, _int, ctypes.c_int64, ctypes.c_int64, _int, ctypes.c_int64,
           ctypes.POINTER(Packet), _sz, ctypes.POINTER(_sz), ctypes.POINTER(_u64), ctypes.POINTER(_u64)])
    _bind(lib, "hdfs_crc32c_abi_version", _int, [])
    _bind(lib, "hdfs_crc32c_session_create", _int, [ctypes.POINTER(_vp), _int, _u32, _int, _u64, _sz])
    _bind(lib, "hdfs_crc32c_session_buffer", _int, [_vp, ctypes.POINTER(_vp), ctypes.POINTER(_u64)])
    _bind(lib, "hdfs_crc32c_session_commit", _int, [_vp, _u64])
    _bind(lib, "hdfs_crc32c_session_flush", _int, [_vp])
    _bind(lib, "hdfs_crc32c_session_poll", _int, [_vp, ctypes.POINTER(Packet), _sz, ctypes.POINTER(_sz), _int])
    _bind(lib, "hdfs_crc32c_session_pending", _int, [_vp, ctypes.POINTER(_u64), ctypes.POINTER(_sz)])
    _bind(lib, "hdfs_crc32c_session_destroy", None, [_vp])
    _bind(lib, "hdfs_crc32c_composite_crcs", _int, [ctypes.POINTER(Segment), _sz, ctypes.POINTER(_u32)])
    _bind(lib, "hdfs_crc32c_dev_alloc", _int, [ctypes.POINTER(_vp), _u64])
    _bind(lib, "hdfs_crc32c_dev_free", _int, [_vp])
    _bind(lib, "hdfs_crc32c_memcpy", _int, [_vp, _vp, _u64, _int])
    _bind(lib, "hdfs_crc32c_memset", _int, [_vp, _int, _u64])
    _bind(lib, "hdfs_crc32c_stream_create", _int, [ctypes.POINTER(_vp)])
    _bind(lib, "hdfs_crc32c_stream_destroy", _int, [_vp])
    _bind(lib, "hdfs_crc32c_stream_sync", _int, [_vp])
    _bind(lib, "hdfs_crc32c_fill_splitmix64", _int, [_vp, _u64, _u64, _u64, _vp])
    _bind(lib, "hdfs_crc32c_corrupt", _int, [_vp, _u64, _u32, _u64, _u64, _u64, _vp])
    _bind(lib, "hdfs_crc32c_device_sync", _int, [])
    _bind(lib, "hdfs_crc32c_mailbox_create", _int, [ctypes.POINTER(_vp), _u32])
    _bind(lib, "hdfs_crc32c_mailbox_stats", _int, [_vp, ctypes.POINTER(_u64), ctypes.POINTER(_u64)])
    _bind(lib, "hdfs_crc32c_mailbox_destroy", _int, [_vp])
    _bind(lib, "hdfs_crc32c_compose_packets", _int,
          [_vp, _u64, ctypes.c_int64, ctypes.c_int64, _int, _int, _int, _vp, _u64, ctypes.POINTER(OutPacket), _sz,
           ctypes.POINTER(_sz), ctypes.POINTER(_u64)])
    _bind(lib, "hdfs_crc32c_compute_host", _int, [_vp, _u64, _u32, _u32, _u32, _vp, _u64])
    _bind(lib, "hdfs_crc32c_verify_host", _int,
          [_vp, _u64, _u32, _u32, _u32, _vp, _vp, _u64, ctypes.POINTER(_u64), ctypes.POINTER(_u64)])
    _bind(lib, "hdfs_crc32c_host_alloc", _int, [ctypes.POINTER(_vp), _u64])
    _bind(lib, "hdfs_crc32c_host_free", _int, [_vp])
    return check_abi(lib)


def bind_diag(lib):
    """Bind the extra knobs of the diagnostic build (include/hadoofus_crc32c_diag.h)."""
    _bind(lib, "hdfs_crc32c_set_tile_order", _int, [_int])
    _bind(lib, "hdfs_crc32c_set_group_shift", _int, [_int])
    _bind(lib, "hdfs_crc32c_set_xcd_major", _int, [_int])
    _bind(lib, "hdfs_crc32c_probe_read", _int, [_vp, _u64, _vp, _int, ctypes.POINTER(ctypes.c_double)])
    _bind(lib, "hdfs_crc32c_set_tuning", _int, [_int, _vp])
    _bind(lib, "hdfs_crc32c_set_probe", _int, [_int, _int, _int])
    _bind(lib, "hdfs_crc32c_set_depth", _int, [_int])
    _bind(lib, "hdfs_crc32c_set_shape", _int, [_int, _int])
    _bind(lib, "hdfs_crc32c_set_store_policy", _int, [_int])
    _bind(lib, "hdfs_crc32c_set_runs", _int, [_int])
    _bind(lib, "hdfs_crc32c_diag_device_checks", _int, [ctypes.POINTER(_u32), _int])
    _bind(lib, "hdfs_crc32c_set_speculation", _int, [_int])
    _bind(lib, "hdfs_crc32c_set_job_coalesce", _int, [_int])
    _bind(lib, "hdfs_crc32c_set_job_early", _int, [_int])
    _bind(lib, "hdfs_crc32c_diag_job_early", _int, [ctypes.POINTER(_u64), _int])
    _bind(lib, "hdfs_crc32c_diag_spec_stats", _int, [ctypes.POINTER(_u64), _int])
    _bind(lib, "hdfs_crc32c_diag_stream_queries", _int, [ctypes.POINTER(_u64)])
    _bind(lib, "hdfs_crc32c_diag_stream_queues", _int, [ctypes.POINTER(_u64)])
    _bind(lib, "hdfs_crc32c_diag_job_queues", _int, [ctypes.POINTER(_u64)])
    return lib


def load(path=LIB_PATH):
    """Load the product library (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ImportError(f"{path} not built; run `python -m hadoofus_amd.build` "
                          "(or __graft_entry__.build())")
    _lib = bind_product(ctypes.CDLL(path))
    return _lib


def check_abi(lib):
    """The library's ABI version is the one these bindings were written for
    (a ctypes prototype cannot detect a changed signature by itself)."""
    v = lib.hdfs_crc32c_abi_version()
    if v != ABI_VERSION:
        raise ImportError(f"library ABI version {v}, bindings written for {ABI_VERSION}")
    return lib


def _check(rc, lib=None):
    if rc != 0:
        raise CRC32CError(rc, (lib or load()).hdfs_crc32c_last_error().decode(errors="replace"))


def _host(buf):
    if isinstance(buf, np.ndarray):
        a = np.ascontiguousarray(buf)
        return a, a.ctypes.data, a.nbytes
    a = np.frombuffer(memoryview(buf).cast("B"), dtype=np.uint8)
    return a, (a.ctypes.data if a.nbytes else None), a.nbytes


def device_info(device=-1):
    arch = ctypes.create_string_buffer(64)
    ncu = _int(0)
    _check(load().hdfs_crc32c_device_info(device, arch, 64, ctypes.byref(ncu)))
    return arch.value.decode(), ncu.value


def init(device=-1):
    """hdfs_crc32c_init: device >= 0 binds the engine to that device."""
    _check(load().hdfs_crc32c_init(device))


def bound_device():
    """-> (device ordinal, PCI bus id) the engine runs on."""
    d = _int(-1)
    bus = ctypes.create_string_buffer(64)
    _check(load().hdfs_crc32c_bound_device(ctypes.byref(d), bus, 64))
    return d.value, bus.value.decode()


def crc32c(crc, buf, entry="_hdfs_crc32c"):
    """_hdfs_crc32c(crc, buf, len) on host memory (src/crc32c.h:13)."""
    keep, p, n = _host(buf)
    return getattr(load(), entry)(crc & 0xFFFFFFFF, p, n)


def stream_crc_dev(crc, dptr, nbytes):
    out = _u32(0)
    _check(load().hdfs_crc32c_stream_dev(crc & 0xFFFFFFFF, dptr, nbytes, ctypes.byref(out)))
    return out.value


def verify_crcdata(region, chunksize, crcdlen, dlen, ctype=CSUM_CRC32C):
    """_verify_crcdata on a host packet region [BE crcs | data].

    Returns (err, first_bad): err 0 on success or the reference error number
    (ERR_CRC_LEN / ERR_BAD_CHECKSUM / ...); negative values are engine errors."""
    keep, p, n = _host(region)
    fb = ctypes.c_int32(-1)
    rc = load().hdfs_crc32c_verify_crcdata(p, chunksize, crcdlen, dlen, ctype, ctypes.byref(fb))
    if rc < 0:
        _check(rc)
    return rc, fb.value


def stream_ex(ctype, crc, buf):
    """CRC of a host buffer (bytes / numpy) continuing from crc: ctype
    CSUM_CRC32C is _hdfs_crc32c, CSUM_CRC32 is zlib.crc32."""
    keep, p, n = _host(buf)
    out = _u32(0)
    _check(load().hdfs_crc32c_stream_ex(ctype, crc & 0xFFFFFFFF, p if n else None, n, ctypes.byref(out)))
    return out.value


def _packets(fn, stream, proto, chunk_size, ctype, max_pkts, dptr=None, nbytes=None, lib=None):
    if dptr is not None:  # device-resident stream
        keep, p, n = None, dptr, nbytes
    else:
        keep, p, n = _host(stream)
    if max_pkts is None:
        max_pkts = n // (25 if proto == PROTO_V1 else 6) + 1
    arr = (Packet * max(1, max_pkts))()
    npk, used = _sz(0), _u64(0)
    lib = lib or load()
    rc = getattr(lib, fn)(p, n, proto, chunk_size, ctype, arr, max_pkts, ctypes.byref(npk), ctypes.byref(used))
    if rc < 0:
        _check(rc, lib)
    return rc, [arr[i].as_dict() for i in range(npk.value)], used.value


class Mailbox:
    """Opt-in resident kernel for the synchronous small calls
    (hdfs_crc32c_mailbox_create); a context manager."""

    def __init__(self, idle_ms=0):
        self.ptr = _vp()
        _check(load().hdfs_crc32c_mailbox_create(ctypes.byref(self.ptr), idle_ms))

    def stats(self):
        calls, launches = _u64(0), _u64(0)
        _check(load().hdfs_crc32c_mailbox_stats(self.ptr, ctypes.byref(calls), ctypes.byref(launches)))
        return calls.value, launches.value

    def close(self):
        if self.ptr:
            _check(load().hdfs_crc32c_mailbox_destroy(self.ptr))
            self.ptr = _vp()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class Session:
    """Streaming packet-verify session (hdfs_crc32c_session_*)."""

    def __init__(self, proto=PROTO_V2, chunk_size=512, ctype=CSUM_CRC32C, slot_bytes=0, nslots=0):
        p = _vp()
        _check(load().hdfs_crc32c_session_create(ctypes.byref(p), proto, chunk_size, ctype, slot_bytes, nslots))
        self.ptr = p.value

    def buffer(self):
        w, room = _vp(), _u64(0)
        _check(load().hdfs_crc32c_session_buffer(self.ptr, ctypes.byref(w), ctypes.byref(room)))
        return w.value, room.value

    def write(self, data):
        """Copy bytes in (as a socket read into the slot would), committing
        slot by slot."""
        mv = memoryview(data).cast("B")
        off = 0
        while off < len(mv):
            w, room = self.buffer()
            n = min(room, len(mv) - off)
            ctypes.memmove(w, (ctypes.c_char * n).from_buffer_copy(mv[off:off + n]), n)
            _check(load().hdfs_crc32c_session_commit(self.ptr, n))
            off += n

    def flush(self):
        _check(load().hdfs_crc32c_session_flush(self.ptr))

    def poll(self, max_pkts=4096, wait=False):
        arr = (Packet * max(1, max_pkts))()
        n = _sz(0)
        rc = load().hdfs_crc32c_session_poll(self.ptr, arr, max_pkts, ctypes.byref(n), 1 if wait else 0)
        if rc < 0:
            _check(rc)
        return rc, [arr[i].as_dict() for i in range(n.value)]

    def pending(self):
        b, n = _u64(0), _sz(0)
        _check(load().hdfs_crc32c_session_pending(self.ptr, ctypes.byref(b), ctypes.byref(n)))
        return b.value, n.value

    def close(self):
        if self.ptr:
            load().hdfs_crc32c_session_destroy(self.ptr)
            self.ptr = None


def composite_crcs(segments):
    """Whole-segment CRCs from each segment's device chunk-CRC array."""
    n = len(segments)
    arr = (Segment * max(1, n))(*segments)
    out = (_u32 * max(1, n))()
    _check(load().hdfs_crc32c_composite_crcs(arr, n, out))
    return [out[i] for i in range(n)]


def parse_packets(stream, proto=PROTO_V2, chunk_size=512, ctype=CSUM_CRC32C, max_pkts=None, dptr=None,
                  nbytes=None, lib=None):
    """Framing walk of a packet stream: host bytes `stream` (no device work),
    or device memory (dptr, nbytes).  -> (rc, [packet dicts], consumed).
    lib: the library to run on (default the product; tests pass the
    diagnostic build)."""
    return _packets("hdfs_crc32c_parse_packets", stream, proto, chunk_size, ctype, max_pkts, dptr, nbytes, lib)


def verify_packets(stream, proto=PROTO_V2, chunk_size=512, ctype=CSUM_CRC32C, max_pkts=None, dptr=None,
                   nbytes=None, lib=None):
    """Framing + GPU verification of every packet's chunks, of host bytes
    `stream` or of device memory (dptr, nbytes).
    -> (rc, [packet dicts], consumed); rc = first error in stream order."""
    return _packets("hdfs_crc32c_verify_packets", stream, proto, chunk_size, ctype, max_pkts, dptr, nbytes, lib)


def read_packets(dptr, nbytes, dst, dst_cap, proto=PROTO_V2, chunk_size=512, ctype=CSUM_CRC32C,
                 max_pkts=None, client_offset=0, read_len=READ_ALL, lib=None, iov=None):
    """hdfs_crc32c_read_packets: verify + copy-out of a device-resident stream
    (dptr, nbytes) into the device buffer dst (dst_cap bytes) -- or into the
    scatter list iov = [(ptr, len), ...] -- the payloads de-framed in stream
    order (read_len READ_ALL), or the block bytes [client_offset,
    client_offset + read_len) of a client read (src/datanode.c:2478-2549).
    rc AGAIN: the destination filled first; resume at stream + consumed,
    client_offset + delivered, read_len - delivered.
    -> (rc, [packet dicts], consumed, delivered)."""
    if max_pkts is None:
        max_pkts = nbytes // (25 if proto == PROTO_V1 else 6) + 1
    arr = (Packet * max(1, max_pkts))()
    npk, used, got = _sz(0), _u64(0), _u64(0)
    lib = lib or load()
    if iov is None:
        iov = [(dst, dst_cap)]
    vec = (IoVec * len(iov))(*[IoVec(p, n) for p, n in iov])
    rc = lib.hdfs_crc32c_read_packets(dptr, nbytes, proto, chunk_size, ctype, client_offset, read_len, vec, len(iov),
                                      arr, max_pkts, ctypes.byref(npk), ctypes.byref(used), ctypes.byref(got))
    if rc < 0:
        _check(rc, lib)
    return rc, [arr[i].as_dict() for i in range(npk.value)], used.value, got.value


def read_packets_fd(dptr, nbytes, fd, fd_offset, client_offset, read_len, proto=PROTO_V2, chunk_size=512,
                    ctype=CSUM_CRC32C, max_pkts=None, lib=None, check=True):
    """hdfs_crc32c_read_packets_fd: the client read [client_offset,
    client_offset + read_len) of a stream (device- or host-resident), its
    bytes pwrite()n to fd at fd_offset (hdfs_datanode_read_file,
    src/datanode.c:2531-2541).  -> (rc, [packet dicts], consumed, delivered);
    check=False returns a negative rc instead of raising."""
    if max_pkts is None:
        max_pkts = nbytes // (25 if proto == PROTO_V1 else 6) + 1
    arr = (Packet * max(1, max_pkts))()
    npk, used, got = _sz(0), _u64(0), _u64(0)
    lib = lib or load()
    rc = lib.hdfs_crc32c_read_packets_fd(dptr, nbytes, proto, chunk_size, ctype, client_offset, read_len, fd,
                                         fd_offset, arr, max_pkts, ctypes.byref(npk), ctypes.byref(used),
                                         ctypes.byref(got))
    if rc < 0 and check:
        _check(rc, lib)
    return rc, [arr[i].as_dict() for i in range(npk.value)], used.value, got.value


class Reader:
    """hdfs_crc32c_reader_*: a client read of a device-resident stream
    verified once (open), delivered piece by piece (next)."""

    def __init__(self, dptr, nbytes, client_offset, read_len, proto=PROTO_V2, chunk_size=512, ctype=CSUM_CRC32C,
                 max_pkts=None, lib=None):
        self.lib = lib or load()
        self.max_pkts = nbytes // (25 if proto == PROTO_V1 else 6) + 1 if max_pkts is None else max_pkts
        self.rd = _vp()
        _check(self.lib.hdfs_crc32c_reader_open(dptr, nbytes, proto, chunk_size, ctype, client_offset, read_len,
                                                 self.max_pkts, ctypes.byref(self.rd)), self.lib)
        self.arr = (Packet * max(1, min(self.max_pkts, 1 << 16)))()

    def next(self, iov, room=None):
        """iov = [(ptr, len), ...] -> (rc, [packet dicts], consumed, delivered);
        room: the record array's capacity passed as max_pkts (default: all)."""
        vec = (IoVec * max(1, len(iov)))(*[IoVec(p, n) for p, n in iov])
        npk, used, got = _sz(0), _u64(0), _u64(0)
        room = len(self.arr) if room is None else min(room, len(self.arr))
        rc = self.lib.hdfs_crc32c_reader_next(self.rd, vec, len(iov), self.arr, room, ctypes.byref(npk),
                                              ctypes.byref(used), ctypes.byref(got))
        if rc < 0:
            _check(rc, self.lib)
        return rc, [self.arr[i].as_dict() for i in range(npk.value)], used.value, got.value

    def close(self):
        if self.rd:
            self.lib.hdfs_crc32c_reader_close(self.rd)
            self.rd = None


class VerifyJob:
    """An asynchronous hdfs_crc32c_verify_packets of a device-resident stream
    (hdfs_crc32c_verify_packets_submit); wait() -> (rc, [packet dicts],
    consumed), exactly verify_packets' result."""

    def __init__(self, dptr, nbytes, proto=PROTO_V2, chunk_size=512, ctype=CSUM_CRC32C, max_pkts=None, lib=None):
        self.lib = lib or load()
        self.max_pkts = nbytes // (25 if proto == PROTO_V1 else 6) + 1 if max_pkts is None else max_pkts
        self.job = _vp()
        _check(self.lib.hdfs_crc32c_verify_packets_submit(dptr, nbytes, proto, chunk_size, ctype, self.max_pkts,
                                                           ctypes.byref(self.job)), self.lib)

    def wait(self):
        arr = (Packet * max(1, self.max_pkts))()
        npk, used = _sz(0), _u64(0)
        job, self.job = self.job, None
        rc = self.lib.hdfs_crc32c_job_wait(job, arr, self.max_pkts, ctypes.byref(npk), ctypes.byref(used))
        if rc < 0:
            _check(rc, self.lib)
        return rc, [arr[i].as_dict() for i in range(npk.value)], used.value


class VerifyBlocksJob:
    """Up to 16 device-resident block streams verified in one launch
    (hdfs_crc32c_verify_blocks_submit); wait() -> (rc, [(rc_b, [packet
    dicts], consumed_b) per block]), each block's entry exactly
    verify_packets' result for it."""

    def __init__(self, blocks, proto=PROTO_V2, chunk_size=512, ctype=CSUM_CRC32C, max_pkts=None, lib=None):
        """blocks: [(dptr, nbytes), ...]"""
        self.lib = lib or load()
        self.n = len(blocks)
        big = max(n for _, n in blocks)
        self.max_pkts = big // (25 if proto == PROTO_V1 else 6) + 1 if max_pkts is None else max_pkts
        ptrs = (_vp * self.n)(*[p for p, _ in blocks])
        lens = (_u64 * self.n)(*[n for _, n in blocks])
        self.job = _vp()
        _check(self.lib.hdfs_crc32c_verify_blocks_submit(ptrs, lens, self.n, proto, chunk_size, ctype, self.max_pkts,
                                                          ctypes.byref(self.job)), self.lib)

    def wait(self):
        arr = (Packet * max(1, self.max_pkts * self.n))()
        npk, used, rcs = (_sz * self.n)(), (_u64 * self.n)(), (_int * self.n)()
        job, self.job = self.job, None
        rc = self.lib.hdfs_crc32c_job_wait_blocks(job, arr, self.max_pkts, npk, used, rcs)
        if rc < 0:
            _check(rc, self.lib)
        out = [(rcs[b], [arr[b * self.max_pkts + i].as_dict() for i in range(npk[b])], used[b]) for b in range(self.n)]
        return rc, out


def compose_packets(data, offset_in_block=0, seqno=0, proto=PROTO_V2, ctype=CSUM_CRC32C, finish=False,
                    dptr=None, nbytes=None):
    """Outgoing packets of one write (_send_packet + _compose_data_packet_header,
    src/datanode.c:2583-2609, 2781-2868) of host bytes `data`, or of device
    memory (dptr, nbytes).  -> (header bytes, [packet dicts])."""
    lib = load()
    if dptr is not None:
        p, n, keep = dptr, nbytes, None
    else:
        keep, p, n = _host(data)
    npk, used = _sz(0), _u64(0)
    _check(lib.hdfs_crc32c_compose_packets(p if n else None, n, offset_in_block, seqno, proto, ctype, int(finish),
                                           None, 0, None, 0, ctypes.byref(npk), ctypes.byref(used)))
    hdr = np.zeros(max(1, used.value), dtype=np.uint8)
    arr = (OutPacket * max(1, npk.value))()
    _check(lib.hdfs_crc32c_compose_packets(p if n else None, n, offset_in_block, seqno, proto, ctype, int(finish),
                                           hdr.ctypes.data, used.value, arr, npk.value, ctypes.byref(npk),
                                           ctypes.byref(used)))
    return hdr[: used.value].tobytes(), [arr[i].as_dict() for i in range(npk.value)]


def compose_crcs(iovecs, chunk=512, ctype=CSUM_CRC32C):
    """BE CRC bytes for the concatenation of host fragments (write path)."""
    arrs = [_host(v) for v in iovecs]
    total = sum(a[2] for a in arrs)
    n = len(arrs)
    bases = (_vp * max(n, 1))(*[a[1] for a in arrs])
    lens = (_sz * max(n, 1))(*[a[2] for a in arrs])
    out = np.zeros(((total + chunk - 1) // chunk) * 4, dtype=np.uint8)
    if total:
        _check(load().hdfs_crc32c_compose_crcs(bases, lens, n, total, chunk, ctype, out.ctypes.data))
    return out.tobytes()


class DeviceBuffer:
    """hipMalloc'd memory owned by the engine's device."""

    def __init__(self, nbytes):
        self.nbytes = int(nbytes)
        p = _vp()
        _check(load().hdfs_crc32c_dev_alloc(ctypes.byref(p), self.nbytes))
        self.ptr = p.value

    def upload(self, host, offset=0):
        keep, p, n = _host(host)
        assert offset + n <= self.nbytes
        if n:
            _check(load().hdfs_crc32c_memcpy(self.ptr + offset, p, n, 0))

    def download(self, nbytes=None, offset=0, dtype=np.uint8):
        nbytes = self.nbytes - offset if nbytes is None else nbytes
        out = np.empty(nbytes, dtype=np.uint8)
        if nbytes:
            _check(load().hdfs_crc32c_memcpy(out.ctypes.data, self.ptr + offset, nbytes, 1))
        return out.view(dtype)

    def copy_to(self, host_ptr, nbytes=None, offset=0):
        """D2H into caller-owned host memory (e.g. a PinnedBuffer)."""
        nbytes = self.nbytes - offset if nbytes is None else nbytes
        _check(load().hdfs_crc32c_memcpy(host_ptr, self.ptr + offset, nbytes, 1))

    def fill(self, value=0):
        _check(load().hdfs_crc32c_memset(self.ptr, value, self.nbytes))

    def free(self):
        if self.ptr:
            load().hdfs_crc32c_dev_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Plan:
    """Batch compute/verify plan over a list of Segment descriptors.  lib:
    the library to run it on (default: the product library; tools pass the
    diagnostic build loaded side by side)."""

    def __init__(self, mode, segments, lib=None):
        self.lib = lib or load()
        self.mode = mode
        self.nseg = len(segments)
        arr = (Segment * max(1, self.nseg))(*segments)
        self._segs = arr
        p = _vp()
        self._check(self.lib.hdfs_crc32c_plan_create(ctypes.byref(p), mode, arr, self.nseg))
        self.ptr = p.value

    def _check(self, rc):
        _check(rc, self.lib)

    def execute(self, stream=None):
        self._check(self.lib.hdfs_crc32c_plan_execute(self.ptr, stream))

    def results(self, stream=None):
        fb = (_u32 * max(1, self.nseg))()
        m = _u64(0)
        self._check(self.lib.hdfs_crc32c_plan_results(self.ptr, stream, fb, self.nseg, ctypes.byref(m)))
        return list(fb)[: self.nseg], m.value

    def set_timing(self, on=True):
        """on: False/True, or an int > 1 = event pairs to pre-create."""
        self._check(self.lib.hdfs_crc32c_plan_set_timing(self.ptr, int(on)))

    def kernel_ms(self):
        t = ctypes.c_double(0)
        n = _int(0)
        self._check(self.lib.hdfs_crc32c_plan_kernel_ms(self.ptr, ctypes.byref(t), ctypes.byref(n)))
        return t.value, n.value

    def stats(self):
        a, b, c = _u64(), _u64(), _u64()
        self._check(self.lib.hdfs_crc32c_plan_stats(self.ptr, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        return {"main_bytes": a.value, "generic_bytes": b.value, "nchunks": c.value}

    def time(self, iters, stream=None):
        ms = ctypes.c_double(0)
        self._check(self.lib.hdfs_crc32c_plan_time(self.ptr, stream, iters, ctypes.byref(ms)))
        return ms.value

    def destroy(self):
        if self.ptr:
            self.lib.hdfs_crc32c_plan_destroy(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


def stream_create():
    s = _vp()
    _check(load().hdfs_crc32c_stream_create(ctypes.byref(s)))
    return s.value


def stream_sync(s):
    _check(load().hdfs_crc32c_stream_sync(s))


def fill_splitmix64(dptr, nwords, seed=0, g0=0, stream=None):
    _check(load().hdfs_crc32c_fill_splitmix64(dptr, nwords, seed, g0, stream))


def corrupt(dptr, nbytes, chunk, chunk0, modulus=65537, bitmul=7919, stream=None):
    _check(load().hdfs_crc32c_corrupt(dptr, nbytes, chunk, chunk0, modulus, bitmul, stream))


def device_sync():
    _check(load().hdfs_crc32c_device_sync())


def compute_host(data, chunk_size, flags=0, crc_init=0, piece_bytes=0):
    """Per-chunk CRCs of a host buffer via the pipelined H2D path."""
    keep, p, n = _host(data)
    nch = (n + chunk_size - 1) // chunk_size
    out = np.zeros(max(1, nch), dtype=np.uint32)
    _check(load().hdfs_crc32c_compute_host(p, n, chunk_size, flags, crc_init, out.ctypes.data, piece_bytes))
    return out[:nch]


def verify_host(data, chunk_size, crcs, flags=0, crc_init=0, piece_bytes=0, want_bitmap=True):
    """-> (first_bad or None, mismatches, bitmap bytes or None)."""
    keep, p, n = _host(data)
    ck, cp, cn = _host(crcs)
    nch = (n + chunk_size - 1) // chunk_size
    assert cn >= nch * 4
    bm = np.zeros(max(1, (nch + 7) // 8), dtype=np.uint8) if want_bitmap else None
    fb, m = _u64(0), _u64(0)
    _check(load().hdfs_crc32c_verify_host(p, n, chunk_size, flags, crc_init, cp,
                                          bm.ctypes.data if bm is not None else None, piece_bytes,
                                          ctypes.byref(fb), ctypes.byref(m)))
    return (None if fb.value == 2**64 - 1 else fb.value), m.value, (bm[:(nch + 7) // 8] if bm is not None else None)


class PinnedBuffer:
    """Page-locked host memory (hipHostMalloc) viewed as a numpy array."""

    def __init__(self, nbytes):
        p = _vp()
        _check(load().hdfs_crc32c_host_alloc(ctypes.byref(p), int(nbytes)))
        self.ptr, self.nbytes = p.value, int(nbytes)
        self.array = np.ctypeslib.as_array((ctypes.c_uint8 * self.nbytes).from_address(self.ptr))

    def free(self):
        if self.ptr:
            load().hdfs_crc32c_host_free(self.ptr)
            self.ptr = None
