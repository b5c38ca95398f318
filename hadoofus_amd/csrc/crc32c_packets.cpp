// Host-side framing of datanode packet streams: the sequential part of
// _recv_packet / _process_recv_packet (src/datanode.c:2345-2446), so that the
// CRC work of a whole run of packets can go to the GPU in one launch.
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
// The reference unpacks the header with protobuf-c; decode_header() below
// restates the parts of protobuf-c's unpack that decide success for this
// message: tag/wire-type scan, wire type must match each known field's type,
// unknown fields skipped, groups and wire types 6/7 rejected, truncation
// rejected, every required field present, last occurrence wins, bool = any
// nonzero varint payload bit.
#include "crc32c_packets.h"

#include <cstdio>
#include <cstring>

namespace hdfs_crc32c {
namespace {

constexpr int64_t kOneGB = 1024 * 1024 * 1024;  // src/datanode.c:2430

inline uint32_t be32(const uint8_t *p) {
  return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | p[3];
}
inline uint64_t be64(const uint8_t *p) { return (uint64_t(be32(p)) << 32) | be32(p + 4); }
inline uint32_t le32(const uint8_t *p) { uint32_t v; std::memcpy(&v, p, 4); return v; }
inline uint64_t le64(const uint8_t *p) { uint64_t v; std::memcpy(&v, p, 8); return v; }

struct Header {
  int64_t offset = 0, seqno = 0;
  int32_t dlen = 0;
  bool last = false, sync = false;
};

// Varint of at most maxb bytes; returns its length or 0 if unterminated.
size_t varint_len(const uint8_t *p, size_t rem, size_t maxb) {
  const size_t n = rem < maxb ? rem : maxb;
  for (size_t i = 0; i < n; i++)
    if (!(p[i] & 0x80)) return i + 1;
  return 0;
}

uint64_t varint_val(const uint8_t *p, size_t n) {
  uint64_t v = 0;
  for (size_t i = 0; i < n; i++) v |= uint64_t(p[i] & 0x7f) << (7 * i);
  return v;
}

bool decode_header(const uint8_t *p, size_t n, Header &h) {
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
        (field == 3 ? h.last : h.sync) = b;
        if (field == 3) seen |= 4;
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

}  // namespace

int parse_packet_stream(const uint8_t *s, uint64_t len, int proto, uint32_t chunk_size, int ctype,
                        size_t max_pkts, std::vector<hdfs_crc32c_packet> &out, uint64_t *consumed,
                        char *errbuf, size_t errlen) {
  out.clear();
  *consumed = 0;
  if (proto != HDFS_CRC32C_PROTO_V1 && proto != HDFS_CRC32C_PROTO_V2) {
    std::snprintf(errbuf, errlen, "bad packet protocol %d", proto);
    return HDFS_CRC32C_EINVAL;
  }
  if (ctype != HDFS_CRC32C_CSUM_NULL && ctype != HDFS_CRC32C_CSUM_CRC32 && ctype != HDFS_CRC32C_CSUM_CRC32C) {
    std::snprintf(errbuf, errlen, "bad checksum type %d", ctype);
    return HDFS_CRC32C_EINVAL;
  }
  if (ctype != HDFS_CRC32C_CSUM_NULL && chunk_size == 0) {
    std::snprintf(errbuf, errlen, "chunk_size 0");
    return HDFS_CRC32C_EINVAL;
  }
  if (len && !s) {
    std::snprintf(errbuf, errlen, "null stream");
    return HDFS_CRC32C_EINVAL;
  }
  uint64_t pos = 0;
  while (out.size() < max_pkts) {
    const uint8_t *p = s + pos;
    const uint64_t rem = len - pos;
    hdfs_crc32c_packet k;
    std::memset(&k, 0, sizeof(k));
    k.stream_off = pos;
    k.first_bad = -1;
    int64_t plen = 0, dlen = 0;
    if (proto == HDFS_CRC32C_PROTO_V1) {  // src/datanode.c:2363-2384
      if (rem < 25) break;
      plen = int32_t(be32(p));
      k.offset_in_block = int64_t(be64(p + 4));
      k.seqno = int64_t(be64(p + 12));
      k.last = p[20] != 0;
      dlen = int32_t(be32(p + 21));
      k.header_len = 25;
    } else {  // src/datanode.c:2387-2418
      if (rem < 6) break;
      plen = int32_t(be32(p));
      const uint32_t hlen = (uint32_t(p[4]) << 8) | p[5];
      if (rem < 6 + uint64_t(hlen)) break;
      k.header_len = 6 + hlen;
      Header h;
      if (!decode_header(p + 6, hlen, h)) {
        k.error = HDFS_CRC32C_ERR_INVALID_PACKETHEADERPROTO;
        out.push_back(k);
        break;
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
    if (k.error) {
      out.push_back(k);
      break;
    }
    if (dlen == 0) {  // src/datanode.c:2448-2456: v2's trailing empty packet
      if (!k.last) k.error = HDFS_CRC32C_ERR_DATANODE_PACKET_SIZE;
      out.push_back(k);
      if (!k.error) *consumed = pos + k.header_len;
      break;
    }
    const uint64_t total = uint64_t(k.header_len) + uint64_t(crcdlen) + uint64_t(dlen);
    if (rem < total) break;  // incomplete: the reference reads more (src/datanode.c:2463-2467)
    out.push_back(k);
    pos += total;
    *consumed = pos;
  }
  return HDFS_CRC32C_OK;
}

}  // namespace hdfs_crc32c
