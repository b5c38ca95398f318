// Packet framing shared by the host walk (crc32c_packets.cpp) and the
// device framing kernel (crc32c_kernels.hip, frame_build_kernel): ONE source
// for the sequential part of _recv_packet / _process_recv_packet
// (src/datanode.c:2345-2446), so a packet framed on the GPU gets exactly the
// record the host walk would give it.
//
// Wire formats (big-endian integers, src/heapbuf.c:174-215):
//   v1 (proto < HDFS_DATANODE_AP_2_0, include/hadoofus/lowlevel.h:429-433):
//     [plen s32][offsetInBlock s64][seqno s64][lastPacketInBlock s8][dataLen s32]
//     = 25 header bytes                                  (src/datanode.c:2363-2384)
//   v2: [plen s32][hlen u16][PacketHeaderProto, hlen bytes] (src/datanode.c:2387-2418)
//     message PacketHeaderProto { required sfixed64 offsetInBlock = 1;
//       required sfixed64 seqno = 2; required bool lastPacketInBlock = 3;
//       required sfixed32 dataLen = 4; optional bool syncBlock = 5; }
//                                                   (src/proto/datatransfer.proto:228-235)
//   then crcdlen = plen - dataLen - 4 bytes of BE CRCs and dataLen data bytes.
//
// The reference unpacks the header with protobuf-c; decode_header() restates
// the parts of protobuf-c's unpack that decide success for this message:
// tag/wire-type scan, wire type must match each known field's type, unknown
// fields skipped, groups and wire types 6/7 rejected, truncation rejected,
// every required field present, last occurrence wins, bool = any nonzero
// varint payload bit.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "hadoofus_crc32c.h"

#define HDFS_HD __host__ __device__ inline

namespace hdfs_crc32c {
namespace frame {

constexpr int64_t kOneGB = 1024 * 1024 * 1024;  // src/datanode.c:2430

// One step of the walk (see frame_step).
enum { kStepNext = 0, kStepStop = 1, kStepMore = 2 };

HDFS_HD uint32_t be32(const uint8_t *p) {
  return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | p[3];
}
HDFS_HD uint64_t be64(const uint8_t *p) { return (uint64_t(be32(p)) << 32) | be32(p + 4); }
HDFS_HD uint32_t le32(const uint8_t *p) {
  return uint32_t(p[0]) | (uint32_t(p[1]) << 8) | (uint32_t(p[2]) << 16) | (uint32_t(p[3]) << 24);
}
HDFS_HD uint64_t le64(const uint8_t *p) { return uint64_t(le32(p)) | (uint64_t(le32(p + 4)) << 32); }

struct Header {
  int64_t offset = 0, seqno = 0;
  int32_t dlen = 0;
  bool last = false, sync = false;
};

// Varint of at most maxb bytes; returns its length or 0 if unterminated.
HDFS_HD size_t varint_len(const uint8_t *p, size_t rem, size_t maxb) {
  const size_t n = rem < maxb ? rem : maxb;
  for (size_t i = 0; i < n; i++)
    if (!(p[i] & 0x80)) return i + 1;
  return 0;
}

HDFS_HD uint64_t varint_val(const uint8_t *p, size_t n) {
  uint64_t v = 0;
  for (size_t i = 0; i < n; i++) v |= uint64_t(p[i] & 0x7f) << (7 * i);
  return v;
}

HDFS_HD bool decode_header(const uint8_t *p, size_t n, Header &h) {
  // Canonical encoding (what HDFS and protobuf-c emit: fields 1..4 in order,
  // one-byte bools, syncBlock only when present): read at fixed offsets.
  // Gives exactly what the general scan below gives for these bytes.
  if ((n == 25 || n == 27) && p[0] == 0x09 && p[9] == 0x11 && p[18] == 0x18 && p[19] < 0x80 && p[20] == 0x25 &&
      (n == 25 || (p[25] == 0x28 && p[26] < 0x80))) {
    h.offset = int64_t(le64(p + 1));
    h.seqno = int64_t(le64(p + 10));
    h.last = p[19] != 0;
    h.dlen = int32_t(le32(p + 21));
    h.sync = n == 27 && p[26] != 0;
    return true;
  }
  unsigned seen = 0;
  size_t pos = 0;
  while (pos < n) {
    const uint8_t *q = p + pos;
    const size_t rem = n - pos;
    if ((q[0] & 0xf8) == 0) return false;  // field number 0
    const size_t tl = varint_len(q, rem, 5);
    if (!tl) return false;
    const uint64_t tag = varint_val(q, tl);
    const unsigned wt = unsigned(tag & 7);
    const uint64_t field = tag >> 3;
    const uint8_t *v = q + tl;
    const size_t vrem = rem - tl;
    size_t vl = 0;
    switch (wt) {
      case 0:
        vl = varint_len(v, vrem, 10);
        if (!vl) return false;
        break;
      case 1:
        if (vrem < 8) return false;
        vl = 8;
        break;
      case 2: {
        const size_t ll = varint_len(v, vrem, 5);
        if (!ll) return false;
        const uint64_t l = varint_val(v, ll);
        if (l > vrem - ll) return false;
        vl = ll + size_t(l);
        break;
      }
      case 5:
        if (vrem < 4) return false;
        vl = 4;
        break;
      default:
        return false;  // groups (3, 4) and 6, 7
    }
    switch (field) {
      case 1:
        if (wt != 1) return false;
        h.offset = int64_t(le64(v));
        seen |= 1;
        break;
      case 2:
        if (wt != 1) return false;
        h.seqno = int64_t(le64(v));
        seen |= 2;
        break;
      case 3:
      case 5: {
        if (wt != 0) return false;
        bool b = false;
        for (size_t i = 0; i < vl; i++) b |= (v[i] & 0x7f) != 0;
        if (field == 3) {
          h.last = b;
          seen |= 4;
        } else {
          h.sync = b;
        }
        break;
      }
      case 4:
        if (wt != 5) return false;
        h.dlen = int32_t(le32(v));
        seen |= 8;
        break;
      default:
        break;  // unknown field: skipped
    }
    pos += tl + vl;
  }
  return seen == 15;
}

// The packet at stream offset `pos`, whose first bytes are at p (rem = bytes
// of the stream from pos on).  Returns kStepNext (k is a complete packet of
// `total` wire bytes; the walk goes on at pos + total), kStepStop (k is
// recorded and the walk ends: framing error or the empty last packet) or
// kStepMore (the packet is incomplete; nothing recorded).  Reads at most
// min(rem, 25) bytes (v1) or min(rem, 6 + hlen) bytes (v2) at p.
HDFS_HD int frame_step(const uint8_t *p, uint64_t rem, uint64_t pos, int proto, uint32_t chunk_size, int ctype,
                       hdfs_crc32c_packet &k, uint64_t &total) {
  k = hdfs_crc32c_packet{};
  k.stream_off = pos;
  k.first_bad = -1;
  int64_t plen = 0, dlen = 0;
  if (proto == HDFS_CRC32C_PROTO_V1) {  // src/datanode.c:2363-2384
    if (rem < 25) return kStepMore;
    plen = int32_t(be32(p));
    k.offset_in_block = int64_t(be64(p + 4));
    k.seqno = int64_t(be64(p + 12));
    k.last = p[20] != 0;
    dlen = int32_t(be32(p + 21));
    k.header_len = 25;
  } else {  // src/datanode.c:2387-2418
    if (rem < 6) return kStepMore;
    plen = int32_t(be32(p));
    const uint32_t hlen = (uint32_t(p[4]) << 8) | p[5];
    if (rem < 6 + uint64_t(hlen)) return kStepMore;
    k.header_len = 6 + hlen;
    Header h;
    if (!decode_header(p + 6, hlen, h)) {
      k.error = HDFS_CRC32C_ERR_INVALID_PACKETHEADERPROTO;
      return kStepStop;
    }
    k.offset_in_block = h.offset;
    k.seqno = h.seqno;
    k.last = h.last;
    k.sync = h.sync;
    dlen = h.dlen;
  }
  // _process_recv_packet framing checks (src/datanode.c:2428-2446)
  const int64_t crcdlen = plen - dlen - 4;
  k.data_len = int32_t(dlen);
  k.crc_len = int32_t(crcdlen);
  if (plen < 0 || dlen < 0 || dlen > kOneGB || plen > kOneGB || crcdlen < 0)
    k.error = HDFS_CRC32C_ERR_DATANODE_PACKET_SIZE;
  else if (ctype != HDFS_CRC32C_CSUM_NULL && crcdlen != ((dlen + chunk_size - 1) / chunk_size) * 4)
    k.error = HDFS_CRC32C_ERR_DATANODE_CRC_LEN;
  else if (ctype == HDFS_CRC32C_CSUM_NULL && crcdlen > 0)
    k.error = HDFS_CRC32C_ERR_DATANODE_UNEXPECTED_CRC_LEN;
  if (k.error) return kStepStop;
  if (dlen == 0) {  // src/datanode.c:2448-2456: v2's trailing empty packet
    if (!k.last) k.error = HDFS_CRC32C_ERR_DATANODE_PACKET_SIZE;
    total = k.header_len;
    return kStepStop;
  }
  total = uint64_t(k.header_len) + uint64_t(crcdlen) + uint64_t(dlen);
  if (rem < total) return kStepMore;  // incomplete: the reference reads more (src/datanode.c:2463-2467)
  return kStepNext;
}

// Client read window of the read path (_process_recv_packet /
// _recv_packet_copy_data, src/datanode.c:2478-2549): a read of the block's
// bytes [client_offset, client_offset + remains_tot) takes from a verified
// packet its data from c_begin = client_offset - offsetInBlock on (0 when
// the packet starts at or after client_offset); c_begin >= dataLen is
// UNEXPECTED_READ_OFFSET (:2483-2486).  Returns avail = dataLen - c_begin,
// the bytes the packet can deliver (0 for that error, for a packet with a
// framing error and for an empty one).  win = false: whole payloads
// (c_begin 0).  In 64 bits: the reference keeps c_begin in an int32_t, which
// differs only for client_offset - offsetInBlock >= 2^31 (beyond any block;
// dataLen <= 1 GiB, so such a packet is UNEXPECTED_READ_OFFSET here).
HDFS_HD uint32_t read_avail(const hdfs_crc32c_packet &r, bool win, int64_t client_offset, uint32_t &c_begin) {
  c_begin = 0;
  if (r.error || r.data_len <= 0) return 0u;
  if (win && r.offset_in_block < client_offset) {
    const uint64_t cb = uint64_t(client_offset) - uint64_t(r.offset_in_block);
    if (cb >= uint64_t(r.data_len)) return 0u;
    c_begin = uint32_t(cb);
  }
  return uint32_t(r.data_len) - c_begin;
}

// Where packet k's delivered bytes go: `before` = the avail of every earlier
// packet of the walk (their sum), `want` = bytes of the destination (the
// read's remains_tot, or the buffer for whole payloads).  Bytes [c_begin,
// c_begin + *len) of its data land at dst + *at; *len = 0 past the window.
HDFS_HD void read_place(uint64_t before, uint32_t avail, uint64_t want, uint64_t &at, uint32_t &len) {
  at = before < want ? before : want;
  const uint64_t room = want - at;
  len = uint32_t(avail < room ? avail : room);
}

}  // namespace frame
}  // namespace hdfs_crc32c
