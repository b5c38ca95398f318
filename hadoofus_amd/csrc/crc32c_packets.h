// Host-side framing of datanode packet streams (internal, not public ABI).
//
// The framing walk is inherently sequential (packet k+1 starts where packet
// k's plen says), touches ~30 header bytes per 64 KiB packet and runs on the
// host; the CRC work it feeds runs on the GPU (crc32c_engine.cpp).
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

#include "hadoofus_crc32c.h"

namespace hdfs_crc32c {

// Parse up to max_pkts packets of a v1/v2 stream (src/datanode.c:2345-2446).
// Every parsed packet is appended to `out` with its framing verdict in
// .error; the walk stops after a framing error (the reference returns it and
// abandons the stream), after an empty last packet (end of block,
// src/datanode.c:2448-2456), or at an incomplete packet (the reference would
// read more from the socket).  *consumed = bytes of complete, framing-clean
// packets.  Returns HDFS_CRC32C_OK or HDFS_CRC32C_EINVAL (bad arguments;
// message in errbuf).
int parse_packet_stream(const uint8_t *s, uint64_t len, int proto, uint32_t chunk_size, int ctype,
                        size_t max_pkts, std::vector<hdfs_crc32c_packet> &out, uint64_t *consumed,
                        char *errbuf, size_t errlen);

// Argument checks shared by every framing entry (EINVAL + message).
int check_framing_args(int proto, uint32_t chunk_size, int ctype, char *errbuf, size_t errlen);

// One step of the walk: the packet at stream offset `pos`, whose first bytes
// are at p (rem = bytes of the stream from pos on; p must hold
// min(rem, kHdrWin) bytes, enough for any v1 header and any v2 header of
// up to kHdrWin - 6 bytes -- a longer v2 header needs 6 + hlen).
enum { kStepNext = 0, kStepStop = 1, kStepMore = 2 };
int frame_step(const uint8_t *p, uint64_t rem, uint64_t pos, int proto, uint32_t chunk_size, int ctype,
               hdfs_crc32c_packet &k, uint64_t &total);

}  // namespace hdfs_crc32c
