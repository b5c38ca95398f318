"""hadoofus_amd -- MI355X-native CRC32C chunk engine for hadoofus's datanode path.

The product is the C-ABI shared library ``hadoofus_amd/lib/libhadoofus_crc32c.so``
(include/hadoofus_crc32c.h, include/crc32c.h).  This package is a thin ctypes
mirror of that ABI used by the tests and bench; it has no compute of its own
and no fallback: if the library or a gfx950 device is missing, calls fail.
Tuning knobs live only in the separate diagnostic build (tools/diaglib.py).
"""
from .abi import (  # noqa: F401
    LIB_PATH, bind_product, bind_diag, CSUM_NULL, CSUM_CRC32, CSUM_CRC32C, ERR_BAD_CHECKSUM, ERR_CRC_LEN,
    ERR_PACKET_SIZE, ERR_INVALID_PACKETHEADERPROTO, ERR_UNEXPECTED_CRC_LEN, ERR_UNEXPECTED_READ_OFFSET,
    ERR_BAD_LASTPACKET, READ_ALL, PROTO_V1, PROTO_V2, Packet, parse_packets, verify_packets, read_packets,
    AGAIN, IoVec, ERR_UNSUPPORTED_CHECKSUM, MODE_COMPUTE, MODE_VERIFY, SEG_BE, SEG_RAW, SEG_CRC32,
    CRC32CError, DeviceBuffer, Mailbox, Plan, Segment, Session, crc32c, compose_crcs, compose_packets,
    composite_crcs, compute_host, verify_host, PinnedBuffer, corrupt, fill_splitmix64, stream_create,
    stream_sync, device_info, init, bound_device, device_sync, load, stream_crc_dev, stream_ex,
    verify_crcdata, VerifyJob, VerifyBlocksJob, Reader, read_packets_fd, EIO,
)

__all__ = [n for n in dir() if not n.startswith("_")]
