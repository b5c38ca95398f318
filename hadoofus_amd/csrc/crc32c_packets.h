// Host-side framing of datanode packet streams (internal, not public ABI).
//
// The framing walk is inherently sequential (packet k+1 starts where packet
// k's plen says), touches ~30 header bytes per 64 KiB packet and runs on the
// host; the CRC work it feeds runs on the GPU (crc32c_engine.cpp).
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

#include "crc32c_frame.h"
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

// One step of the walk (crc32c_frame.h, shared with the device framing
// kernel): the packet at stream offset `pos`, whose first bytes are at p.
using frame::frame_step;
using frame::kStepMore;
using frame::kStepNext;
using frame::kStepStop;

}  // namespace hdfs_crc32c
