/*
 * Drop-in replacement for the reference's private header src/crc32c.h
 * (alexsmith1612/hadoofus).  Same include guard and the same three
 * declarations (src/crc32c.h:13, :17, :24), so src/datanode.c:16
 * (`#include "crc32c.h"`) and tests/t_unit.c compile unchanged against
 * libhadoofus_crc32c.so.  Semantics are those of the reference: the CRC is
 * pre- and post-inverted inside the call; pass 0 to start and the previous
 * return value to continue.  Every backend symbol is served by the MI355X
 * engine (include/hadoofus_crc32c.h), with the reference's per-architecture
 * declarations (src/crc32c.h:15-22); the library defines all four, so
 * either declaration set links.
 */
#ifndef _HADOOFUS_CRC32C_H
#define _HADOOFUS_CRC32C_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

uint32_t _hdfs_crc32c(uint32_t crc, const void *buf, unsigned len);

#if defined(__amd64__) || defined(__i386__)
uint32_t _hdfs_sse42_crc32c(uint32_t crc, const void *buf, unsigned len);
#elif defined(__aarch64__)
uint32_t _hdfs_armv8_crc32c(uint32_t crc, const void *buf, unsigned len);
#endif

uint32_t _hdfs_sw_crc32c(uint32_t crc, const void *buf, unsigned len);

#ifdef __cplusplus
}
#endif
#endif /* _HADOOFUS_CRC32C_H */
