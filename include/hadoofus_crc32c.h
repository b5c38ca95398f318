/*
 * hadoofus_crc32c.h -- C ABI of the MI355X-native CRC32C engine
 * (libhadoofus_crc32c.so, built from hadoofus_amd/csrc/).
 *
 * Two layers:
 *
 * 1. DROP-IN: the three symbols of the reference's private header
 *    src/crc32c.h:13-24 (also declared, with the reference's include guard,
 *    in include/crc32c.h so src/datanode.c:16 compiles unchanged).  Same
 *    semantics: pre/post inversion inside, crc=0 starts, chaining by passing
 *    the previous return value, len==0 returns crc, any alignment, total
 *    function.  All three run on the GPU engine; with no usable GPU they
 *    abort() with a message (there is no CPU fallback).
 *
 * The release library has no tuning or diagnostic knobs: it reads nothing
 * from the environment that changes what it computes.  Those live in the
 * separate diagnostic build, include/hadoofus_crc32c_diag.h.
 *
 * 2. BATCH (additive): per-chunk compute / verify over a table of chunk
 *    streams in device memory, the shape of the two datanode loops
 *    (src/datanode.c:2814-2860 write compute, src/datanode.c:2931-2963 read
 *    verify), plus host-memory mirrors of those two loops.
 *
 * No HIP or torch types appear in the signatures: streams are passed as
 * `void *` (a hipStream_t, NULL = the engine's own stream).
 */
#ifndef HADOOFUS_CRC32C_H
#define HADOOFUS_CRC32C_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- 1. drop-in (replaces src/crc32c.h:13, :17, :24) -------------------- */
uint32_t _hdfs_crc32c(uint32_t crc, const void *buf, unsigned len);
uint32_t _hdfs_sse42_crc32c(uint32_t crc, const void *buf, unsigned len);
uint32_t _hdfs_armv8_crc32c(uint32_t crc, const void *buf, unsigned len);  /* aarch64 name, same engine */
uint32_t _hdfs_sw_crc32c(uint32_t crc, const void *buf, unsigned len);

/* ---- status codes ------------------------------------------------------- */
#define HDFS_CRC32C_OK 0
#define HDFS_CRC32C_EINVAL (-1)   /* bad argument / descriptor */
#define HDFS_CRC32C_ENODEV (-2)   /* no usable gfx950 device / HIP runtime */
#define HDFS_CRC32C_ENOMEM (-3)   /* device or pinned allocation failed */
#define HDFS_CRC32C_EHIP (-4)     /* HIP runtime error (see last_error) */
#define HDFS_CRC32C_EIO (-5)      /* writing a read's bytes to a file descriptor failed (errno in last_error) */
/* Datanode-level results reuse the reference's enum hdfs_error_numeric
 * values (include/objects.h:21-113; checked by compiling that header). */
#define HDFS_CRC32C_ERR_DATANODE_UNSUPPORTED_CHECKSUM 8
#define HDFS_CRC32C_ERR_INVALID_PACKETHEADERPROTO 18
#define HDFS_CRC32C_ERR_DATANODE_PACKET_SIZE 25
#define HDFS_CRC32C_ERR_DATANODE_CRC_LEN 26
#define HDFS_CRC32C_ERR_DATANODE_UNEXPECTED_CRC_LEN 27
#define HDFS_CRC32C_ERR_DATANODE_UNEXPECTED_READ_OFFSET 28
#define HDFS_CRC32C_ERR_DATANODE_BAD_CHECKSUM 29
#define HDFS_CRC32C_ERR_DATANODE_BAD_LASTPACKET 32

/* enum hdfs_checksum_type (include/objects.h:169-175) */
#define HDFS_CRC32C_CSUM_NULL 0
#define HDFS_CRC32C_CSUM_CRC32 1
#define HDFS_CRC32C_CSUM_CRC32C 2

/* ABI version of this header.  Every exported symbol carries the version
 * node HADOOFUS_CRC32C_<n> (hadoofus_amd/csrc/exports.map), and a function
 * whose signature changes gets a new name: a caller built against another
 * version fails to bind instead of passing shifted arguments.  Bindings that
 * load the library at run time (ctypes, dlsym) compare
 * hdfs_crc32c_abi_version() with the version they were written for.
 *   3: round 3 (unversioned exports)
 *   4: hdfs_crc32c_verify_packets_copy -> hdfs_crc32c_read_packets (iovecs,
 *      resumable reads); versioned exports
 *   5: hdfs_crc32c_read_packets: a client read ends at its first error (bad
 *      CRCs included), host-memory iovecs and streams; asynchronous verify
 *      jobs (hdfs_crc32c_verify_packets_submit / hdfs_crc32c_job_wait),
 *      batches of blocks (hdfs_crc32c_verify_blocks_submit /
 *      hdfs_crc32c_job_wait_blocks), verified reads delivered piece by
 *      piece (hdfs_crc32c_reader_*) */
#define HDFS_CRC32C_ABI_VERSION 5
int hdfs_crc32c_abi_version(void);

const char *hdfs_crc32c_last_error(void);
/* Initialise the engine on `device`.  device >= 0 also BINDS the engine to
 * it: every later call that names no device (all of them) runs there, with
 * no reliance on the caller's current-device state (one process per GPU:
 * a rank calls hdfs_crc32c_init(LOCAL_RANK) first).  -1: the bound device,
 * else the calling thread's current HIP device.  Called implicitly (with -1)
 * by every entry point. */
int hdfs_crc32c_init(int device);
/* The device the engine runs on (ordinal in this process) and its PCI bus
 * id ("0000:xx:00.0", hipDeviceGetPCIBusId), so launchers can check that
 * ranks landed on distinct GPUs. */
int hdfs_crc32c_bound_device(int *device, char *pci_bus_id, size_t len);
/* gfx arch string of the engine's device, e.g. "gfx950". */
int hdfs_crc32c_device_info(int device, char *arch, size_t arch_len, int *num_cu);

/* ---- 2. batch API -------------------------------------------------------- */
#define HDFS_CRC32C_MODE_COMPUTE 0
#define HDFS_CRC32C_MODE_VERIFY 1

#define HDFS_CRC32C_SEG_BE 1u   /* crcs[] in wire (big-endian) order, src/util.h:68-92 */
#define HDFS_CRC32C_SEG_RAW 2u  /* compute: raw register (init 0, no final inversion) */
/* Chunks use zlib's CRC-32 polynomial 0xEDB88320 (HDFS_CSUM_CRC32, the
 * crc32() calls of src/datanode.c:2832-2845,2940-2952) instead of CRC-32C.
 * All segments of one plan must agree. */
#define HDFS_CRC32C_SEG_CRC32 4u

/* One chunk stream: chunk i = bytes [i*chunk_size, min((i+1)*chunk_size, len))
 * of `data`; the last chunk may be partial (src/datanode.c:2946). */
typedef struct hdfs_crc32c_segment {
	const void *data;      /* device pointer */
	uint64_t len;          /* bytes */
	uint32_t chunk_size;   /* bytesPerChecksum, > 0 */
	uint32_t flags;        /* HDFS_CRC32C_SEG_* */
	uint32_t crc_init;     /* value each chunk's CRC starts from (reference: 0) */
	uint32_t reserved;
	void *crcs;            /* device u32[nchunks]: compute out / verify expected in */
	uint8_t *bitmap;       /* verify: device out, ceil(nchunks/8) bytes, bit i = chunk i bad */
} hdfs_crc32c_segment;

typedef struct hdfs_crc32c_plan hdfs_crc32c_plan;

/* Validate the segment table and upload it to the device (done once). */
int hdfs_crc32c_plan_create(hdfs_crc32c_plan **plan, int mode,
    const hdfs_crc32c_segment *segs, size_t nseg);
/* Enqueue one pass over every chunk of every segment on `stream`
 * (graph-capturable: no allocation or synchronisation inside). */
int hdfs_crc32c_plan_execute(hdfs_crc32c_plan *plan, void *stream);
/* Verify plans: wait for the stream and return the first bad chunk of each
 * segment (UINT32_MAX if none) and the total number of bad chunks. */
int hdfs_crc32c_plan_results(hdfs_crc32c_plan *plan, void *stream,
    uint32_t *first_bad, size_t nseg, uint64_t *mismatches);
/* Optional device-side timing of the tiled kernel (HIP events recorded on
 * the execute stream around each launch).  on > 1 pre-creates that many
 * event pairs; kernel_ms sums and resets the recorded launches. */
int hdfs_crc32c_plan_set_timing(hdfs_crc32c_plan *plan, int on);
int hdfs_crc32c_plan_kernel_ms(hdfs_crc32c_plan *plan, double *total_ms, int *launches);
/* Bytes per pass the tiled and generic kernels cover (for roofline maths). */
int hdfs_crc32c_plan_stats(const hdfs_crc32c_plan *plan, uint64_t *main_bytes,
    uint64_t *generic_bytes, uint64_t *nchunks);
void hdfs_crc32c_plan_destroy(hdfs_crc32c_plan *plan);

/* CRC of one arbitrary device buffer continuing from `crc` (the
 * _hdfs_crc32c contract on device memory); synchronous. */
int hdfs_crc32c_stream_dev(uint32_t crc, const void *dbuf, uint64_t len, uint32_t *out);
/* Same for host or device memory and either checksum type: ctype
 * HDFS_CRC32C_CSUM_CRC32C is _hdfs_crc32c, HDFS_CRC32C_CSUM_CRC32 is zlib's
 * crc32(crc, buf, len) (the CRC32 branch of src/datanode.c:2845,2952). */
int hdfs_crc32c_stream_ex(int ctype, uint32_t crc, const void *buf, uint64_t len, uint32_t *out);

/* Block composite CRC (the COMPOSITE_CRC block checksum of
 * src/proto/datatransfer.proto:316-322, src/proto/hdfs.proto:483-497, which
 * the reference declares but does not compute): for each segment, the CRC of
 * its whole data, derived from the per-chunk CRCs in segs[i].crcs (device
 * memory, as a compute plan wrote them: wire order if HDFS_CRC32C_SEG_BE,
 * CRC32 tables if HDFS_CRC32C_SEG_CRC32) with the combine identity
 * c(A||B) = Z_|B|(c(A)) ^ c(B) -- the data is not re-read.  crc_init must be
 * 0 (or SEG_RAW: raw registers combine the same way).  out: host or device
 * u32[nseg]; synchronous. */
int hdfs_crc32c_composite_crcs(const hdfs_crc32c_segment *segs, size_t nseg, uint32_t *out);

/* ---- datanode mirrors on host memory (synchronous) ---------------------- */
/* _verify_crcdata (src/datanode.c:2931-2963) plus the CRC-length framing
 * check of _process_recv_packet (src/datanode.c:2441-2442) on a packet region
 * [crcdlen bytes of BE CRCs | dlen bytes of data].  Returns 0, or
 * HDFS_CRC32C_ERR_DATANODE_{PACKET_SIZE,CRC_LEN,BAD_CHECKSUM}, or a negative
 * HDFS_CRC32C_E* status (EINVAL for a ctype other than CRC32 / CRC32C, which
 * the reference ASSERTs); *first_bad = first mismatching chunk or -1. */
int hdfs_crc32c_verify_crcdata(const void *crcdata, int32_t chunksize, int32_t crcdlen,
    int32_t dlen, int ctype, int32_t *first_bad);
/* CRC loop of _compose_data_packet_header (src/datanode.c:2814-2860):
 * ceil(total/chunk) big-endian CRCs of the concatenation of iovcnt
 * fragments (CRCs chain across fragment boundaries); ctype is the packet's
 * sendcsum_type (HDFS_CRC32C_CSUM_CRC32 or _CRC32C). */
int hdfs_crc32c_compose_crcs(const void *const *iov_base, const size_t *iov_len, int iovcnt,
    size_t total, uint32_t chunk, int ctype, void *crc_be_out);

/* ---- datanode packet streams (src/datanode.c:2345-2494) ----------------- */
/* Framing of a run of received packets, the sequential part of _recv_packet /
 * _process_recv_packet:
 *   PROTO_V1 (proto < HDFS_DATANODE_AP_2_0, include/hadoofus/lowlevel.h:429-433):
 *     [plen s32][offsetInBlock s64][seqno s64][last s8][dataLen s32], 25 bytes
 *   PROTO_V2: [plen s32][hlen u16][PacketHeaderProto (hlen bytes)]
 *   followed by crcdlen = plen - dataLen - 4 bytes of BE CRCs and the data. */
#define HDFS_CRC32C_PROTO_V1 1
#define HDFS_CRC32C_PROTO_V2 2

typedef struct hdfs_crc32c_packet {
	uint64_t stream_off;      /* offset of the packet (its plen) in the stream */
	int64_t offset_in_block;  /* header offsetInBlock */
	int64_t seqno;            /* header seqno */
	int32_t data_len;         /* dataLen */
	int32_t crc_len;          /* crcdlen = plen - dataLen - 4; CRCs at stream_off + header_len */
	uint32_t header_len;      /* 25 (v1) or 6 + hlen (v2) */
	int32_t error;            /* 0 or the HDFS_CRC32C_ERR_* this packet raises */
	int32_t first_bad;        /* first bad chunk of the packet, -1 if none */
	uint32_t bad_chunks;      /* number of bad chunks in the packet */
	uint8_t last;             /* lastPacketInBlock */
	uint8_t sync;             /* syncBlock (v2) */
	uint8_t reserved[6];
} hdfs_crc32c_packet;

/* Framing only: walks up to max_pkts packets of the stream (host memory:
 * no device work; device memory: the headers are read through
 * device framing kernels, with a host walk over header windows for streams
 * of mixed packet sizes), applying the checks of src/datanode.c:2428-2456
 * (PACKET_SIZE, CRC_LEN, UNEXPECTED_CRC_LEN, empty non-last packet) and the
 * header decode (INVALID_PACKETHEADERPROTO).  The walk stops after a framing
 * error (recorded in that packet's .error), after an empty last packet (end
 * of block), or at an incomplete packet (not recorded).  *consumed = bytes of
 * complete, framing-clean packets.  Returns the first packet error, 0, or a
 * negative HDFS_CRC32C_E* status.  ctype: HDFS_CRC32C_CSUM_*. */
int hdfs_crc32c_parse_packets(const void *stream, uint64_t len, int proto, uint32_t chunk_size,
    int ctype, hdfs_crc32c_packet *pkts, size_t max_pkts, size_t *npkts, uint64_t *consumed);
/* Framing as above, then every chunk of every framing-clean packet verified
 * on the GPU (_verify_crcdata, src/datanode.c:2931-2963): a host stream goes
 * H2D once in pieces overlapped with a de-framing gather kernel and the
 * verify kernels; a device-resident stream is verified in place (its bytes
 * must be complete: the caller synchronises whatever wrote them).  Per packet: .error = BAD_CHECKSUM, .first_bad,
 * .bad_chunks.  Returns the first error in stream order (what the reference
 * returns from its packet loop), 0, or a negative status. */
int hdfs_crc32c_verify_packets(const void *stream, uint64_t len, int proto, uint32_t chunk_size,
    int ctype, hdfs_crc32c_packet *pkts, size_t max_pkts, size_t *npkts, uint64_t *consumed);

/* Read of a packet stream: hdfs_crc32c_verify_packets, and the packets'
 * data delivered, de-framed and in stream order, to the caller's buffers --
 * the read path's _process_recv_packet / _recv_packet_copy_data
 * (src/datanode.c:2470-2553).  (Round 4: replaces round 3's
 * hdfs_crc32c_verify_packets_copy, whose signature had changed under the
 * same name; see HDFS_CRC32C_ABI_VERSION.)  Where the bytes live:
 *   - device stream, device buffers (GPU-direct receive): the copy is fused
 *     into the verify kernel, each payload byte read once and written once;
 *   - device stream, host buffers: the same fused pass into an engine-owned
 *     device staging area (grown to the read's size on demand), then one
 *     D2H copy per iovec;
 *   - host stream, host buffers (a datanode receiving into host memory):
 *     framed on the host, the packets the read takes verified on the GPU
 *     (the host pipeline of hdfs_crc32c_verify_packets), then their bytes
 *     memcpy()ed into the iovecs as the reference does (:2516);
 *   - host stream, device buffers: EINVAL.
 * (Host buffers since ABI 5; the signature is unchanged, a version-4
 * library refuses them with EINVAL.)
 *
 * iov / iovcnt: the destination, buffers filled in order (the reference's
 * iovec array, :2509-2537), all device memory of the stream's device or all
 * host memory (pageable or pinned); total capacity cap = sum of
 * iov[i].len.
 * read_len = HDFS_CRC32C_READ_ALL: every framing-clean packet's whole
 *   payload (iovcnt must be 1): hdfs_crc32c_verify_packets with the payload
 *   copied -- records for every packet of the run, verdicts past an error
 *   included; *delivered = payload bytes of the packets before the first
 *   packet with an error.  This mode has no read position (no client
 *   offset) to resume from, so a buffer too small for the framed payload is
 *   a sizing error: EINVAL, nothing written past the buffer (size it from
 *   hdfs_crc32c_parse_packets, or use a read window, which resumes).
 * read_len > 0: a client read of the block's bytes [client_offset,
 *   client_offset + read_len) (hdfs_datanode_read's bloff / len,
 *   src/datanode.c:1363-1377), the reference's read loop
 *   (src/datanode.c:1476-1481).  Packets are taken while the read wants
 *   bytes.  The read ENDS AT ITS FIRST ERROR, which is the call's return
 *   value and its last record:
 *     - a framing error, or bad CRCs (HDFS_CRC32C_ERR_DATANODE_BAD_CHECKSUM:
 *       the reference stops its loop there, :1476-1479, :2470-2475): the
 *       packet delivers nothing and *consumed ends before it;
 *     - c_begin = client_offset - offsetInBlock >= dataLen:
 *       HDFS_CRC32C_ERR_DATANODE_UNEXPECTED_READ_OFFSET (:2478-2486), *consumed
 *       ends before the packet;
 *     - a lastPacketInBlock packet that leaves the read short (after its
 *       bytes are delivered), or an empty last packet before the read is
 *       complete: HDFS_CRC32C_ERR_DATANODE_BAD_LASTPACKET (:2452-2454,
 *       :2545-2546), *consumed ends after it.
 *   A packet that starts before client_offset delivers from c_begin on; a
 *   packet delivers at most what is left of the read.  Without an error the
 *   walk ends with the packet that completes the read; later packets are
 *   not returned.  *delivered = the bytes the reference copies to the
 *   caller before its loop returns (a BAD_LASTPACKET packet's own bytes
 *   included).  Records, *consumed, *delivered and the status do not depend
 *   on how the destination is split.  (Several device buffers: the read is
 *   verified once and its bytes laid over them by one copy launch.)
 *   A destination smaller than the rest of the read is RESUMABLE, as the
 *   reference's read is (`rlen == 0 && remains_tot > 0` -> HDFS_AGAIN,
 *   :2547-2549, re-entered with remains_pkt > 0, :2356-2361): once the
 *   buffers are full the call returns HDFS_CRC32C_AGAIN with *delivered =
 *   cap, and *consumed = where the stream must resume -- the start of the
 *   packet whose bytes were only partly delivered (its record is returned
 *   by the call that completes it), or the end of the last packet if the
 *   buffers filled exactly there.  The caller continues with stream +
 *   consumed, client_offset + delivered and read_len - delivered: the
 *   re-passed packet then delivers from its new c_begin on.  (Bad CRCs in a
 *   packet that would overflow the buffers end the read: the reference
 *   verifies a packet before it copies any of it.)
 * Bytes of the buffers past *delivered are unspecified, bytes past them (or
 * past the read) are never written.  ctype must be CRC32 or CRC32C.
 * Returns the error that ended the read (READ_ALL: the first error in stream
 * order), 0, HDFS_CRC32C_AGAIN, or a negative status. */
#define HDFS_CRC32C_READ_ALL (-1)
/* Not an error: the destination filled before the read completed (the
 * reference's HDFS_AGAIN); outside the range of the datanode errors. */
#define HDFS_CRC32C_AGAIN 1000
typedef struct hdfs_crc32c_iovec {
	void *base;     /* device memory of the stream's device, or host memory */
	uint64_t len;
} hdfs_crc32c_iovec;
int hdfs_crc32c_read_packets(const void *stream, uint64_t len, int proto, uint32_t chunk_size, int ctype,
    int64_t client_offset, int64_t read_len, const hdfs_crc32c_iovec *iov, int iovcnt,
    hdfs_crc32c_packet *pkts, size_t max_pkts, size_t *npkts, uint64_t *consumed, uint64_t *delivered);

/* Asynchronous hdfs_crc32c_verify_packets of a DEVICE-resident stream (a
 * datanode verifying a stream of received blocks): submit launches the
 * verify and returns; hdfs_crc32c_job_wait returns exactly what
 * hdfs_crc32c_verify_packets would (records, consumed, first error) and
 * releases the job.  Up to 64 jobs per device may be outstanding (submitted,
 * not yet waited for; one more is EINVAL).  Jobs submitted while an earlier
 * launch is still running queue and go out together as ONE batch launch
 * (as hdfs_crc32c_verify_blocks_submit's) -- when a submit finds the GPU
 * idle, when a wait needs a queued job or would block on a running launch,
 * or at 16 queued runs or a run of another length or layout -- so a stream
 * of blocks pays the launch's fixed cost once per batch; up to 4 launches
 * run at once (a submit or wait may first collect the oldest).  The wait
 * on a job of such a batch returns as soon as its own block is verified --
 * clean, its headers the predicted ones -- while the launch verifies the
 * blocks after it (the wait on the batch's last block, or on a block with a
 * bad chunk or an irregular header, returns with the launch).  A run of
 * equal packets is verified by the speculative launch; whatever it does not take
 * (another packet size, more than 65 536 packets, no run at all) is framed
 * and verified inside the wait.  The stream's bytes must stay unchanged, and
 * written before the submit (synchronise whatever wrote them), until the
 * wait returns; every submitted job must be waited for.  max_pkts at the
 * wait must be at least the submit's. */
typedef struct hdfs_crc32c_job hdfs_crc32c_job;
int hdfs_crc32c_verify_packets_submit(const void *stream, uint64_t len, int proto, uint32_t chunk_size, int ctype,
    size_t max_pkts, hdfs_crc32c_job **job);
int hdfs_crc32c_job_wait(hdfs_crc32c_job *job, hdfs_crc32c_packet *pkts, size_t max_pkts, size_t *npkts,
    uint64_t *consumed);
/* A job of up to 16 BLOCKS (separate device-resident streams, one block
 * transfer each) verified in ONE launch when their packets share one layout
 * (packet size and header length; each block's own offsets and seqnos): the
 * launch's fixed cost is paid once per batch.  The launch covers the largest
 * group of blocks of one length (blocks of one layout and length hold the
 * same number of packets); the other blocks -- a file's short last block --
 * and any the launch cannot take are verified one by one inside the wait.  hdfs_crc32c_job_wait_blocks:
 * block b's records at pkts + b * max_pkts, npkts[b], consumed[b], and
 * rcs[b] = what hdfs_crc32c_verify_packets returns for block b; returns the
 * first negative status, else the first nonzero rcs[b], else 0. */
int hdfs_crc32c_verify_blocks_submit(const void *const *streams, const uint64_t *lens, size_t nblocks, int proto,
    uint32_t chunk_size, int ctype, size_t max_pkts, hdfs_crc32c_job **job);
int hdfs_crc32c_job_wait_blocks(hdfs_crc32c_job *job, hdfs_crc32c_packet *pkts, size_t max_pkts, size_t *npkts,
    uint64_t *consumed, int *rcs);

/* A client read VERIFIED ONCE and then delivered piece by piece -- the
 * reference's read re-entered with remains_pkt > 0 (src/datanode.c:2356-2361,
 * 2547-2549) for a caller whose buffer is smaller than the read, without
 * framing or verifying any packet again.  open frames and verifies the
 * packets of the read [client_offset, client_offset + read_len) under
 * hdfs_crc32c_read_packets' rules (the read ends at its first error;
 * max_pkts: room for its records) and keeps their records; each next
 * delivers the following bytes into iov -- from a DEVICE-resident stream
 * into device memory of its device (one copy launch, or a request to the
 * open mailbox for <= 96 KiB) or host memory (D2H); from a HOST-resident
 * stream (framed on the host, its read's packets verified on the GPU at
 * open) into host memory only (memcpy, src/datanode.c:2516) --
 * *delivered = bytes this call, *consumed = the end of the last packet
 * delivered whole so far (the read's own consumed at its end), into pkts
 * the records of the packets whose last byte this call delivered (the
 * read's last record with the last call) -- at most max_pkts of them; the
 * rest come with the following calls, which may deliver no bytes -- and
 * returns HDFS_CRC32C_AGAIN while bytes or records remain, then the read's
 * status: 0, or the error that ended
 * it, whose record comes last.  A read the stream or max_pkts cannot
 * complete ends with 0 and fewer bytes than read_len, as
 * hdfs_crc32c_read_packets' does: resume at stream + consumed.  The stream
 * must stay unchanged until close; calls after the last return the status
 * again and deliver nothing. */
typedef struct hdfs_crc32c_reader hdfs_crc32c_reader;
int hdfs_crc32c_reader_open(const void *stream, uint64_t len, int proto, uint32_t chunk_size, int ctype,
    int64_t client_offset, int64_t read_len, size_t max_pkts, hdfs_crc32c_reader **rd);
int hdfs_crc32c_reader_next(hdfs_crc32c_reader *rd, const hdfs_crc32c_iovec *iov, int iovcnt,
    hdfs_crc32c_packet *pkts, size_t max_pkts, size_t *npkts, uint64_t *consumed, uint64_t *delivered);
void hdfs_crc32c_reader_close(hdfs_crc32c_reader *rd);

/* A client read whose bytes go to a FILE DESCRIPTOR (the reference's
 * hdfs_datanode_read_file: _recv_packet_copy_data pwrite()s each verified
 * packet's bytes at fdoffset and advances it, src/datanode.c:2531-2541,
 * src/net.c:290-313): the read [client_offset, client_offset + read_len) of
 * the stream under hdfs_crc32c_read_packets' rules -- records, status,
 * consumed as that call returns them with a destination of read_len bytes --
 * with the delivered bytes written to fd at fd_offset, fd_offset +
 * *delivered ... (pwrite, retried until complete; the fd may be a regular
 * file, a pipe is not seekable and fails).  The stream is verified once; the
 * bytes leave through a bounded host staging buffer (device streams: D2H)
 * in stream order, so a failing write leaves exactly the bytes before it
 * written: HDFS_CRC32C_EIO, *delivered = the bytes written, errno's text in
 * hdfs_crc32c_last_error().  read_len > 0 (a window; no READ_ALL). */
int hdfs_crc32c_read_packets_fd(const void *stream, uint64_t len, int proto, uint32_t chunk_size, int ctype,
    int64_t client_offset, int64_t read_len, int fd, int64_t fd_offset, hdfs_crc32c_packet *pkts, size_t max_pkts,
    size_t *npkts, uint64_t *consumed, uint64_t *delivered);

/* ---- write path: outgoing data packets ---------------------------------- */
/* One outgoing data packet, as _send_packet sizes it and
 * _compose_data_packet_header builds its header buffer
 * (src/datanode.c:2583-2609, 2781-2868): hdr_out[hdr_off, +hdr_len) is the
 * header buffer the reference would writev() before the packet's data
 * ([plen s32][hlen u16][PacketHeaderProto] (v2) or the 25-byte v1 header,
 * then 4 BE CRC bytes per 512-B chunk), data[data_off, +data_len) the data. */
typedef struct hdfs_crc32c_out_packet {
	uint64_t hdr_off;         /* header + CRC bytes in hdr_out */
	uint64_t data_off;        /* data bytes in the caller's buffer */
	int64_t offset_in_block;  /* header offsetInBlock */
	int64_t seqno;            /* header seqno */
	int32_t data_len;         /* dataLen */
	uint32_t hdr_len;         /* header bytes incl. plen, hlen and CRCs */
	uint32_t crc_len;         /* CRC bytes (4 per chunk; 0 for CSUM_NULL) */
	uint8_t last;             /* lastPacketInBlock */
	uint8_t reserved[3];
} hdfs_crc32c_out_packet;

/* Compose the outgoing packets of one write of len bytes (host or device
 * memory) starting at block offset offset_in_block with sequence number
 * seqno: packets of at most 64 KiB (PACKET_SIZE, src/datanode.c:38), the
 * first one cut at the next 512-B chunk boundary when offset_in_block is
 * unaligned (src/datanode.c:2590-2609); finish != 0 appends the empty
 * lastPacketInBlock packet of hdfs_datanode_finish_block.  Every chunk CRC
 * (CRC32C or zlib CRC32 by ctype; none for CSUM_NULL) is computed on the GPU
 * in one pass over the data.  With hdr_out or pkts NULL (or too small) only
 * the sizes are returned: *npkts packets, *hdr_used header bytes (an
 * undersized call returns HDFS_CRC32C_EINVAL). */
int hdfs_crc32c_compose_packets(const void *data, uint64_t len, int64_t offset_in_block, int64_t seqno,
    int proto, int ctype, int finish, void *hdr_out, uint64_t hdr_cap, hdfs_crc32c_out_packet *pkts,
    size_t max_pkts, size_t *npkts, uint64_t *hdr_used);

/* Streaming sessions for socket-fed packets (pinned ring
 * buffers fed by socket reads, src/net.c:241-263 -> src/datanode.c:2345-2494):
 * the session owns nslots pinned host slots of slot_bytes (defaults 4 x
 * 64 MiB); the caller receives straight into the current slot
 * (session_buffer -> recv() -> session_commit).  A full slot (or a flush) is
 * framed on the host and its packets verified asynchronously on the GPU
 * while the caller keeps receiving into the next slot; the incomplete tail
 * packet moves to the next slot.  session_poll returns finished packet
 * records in stream order (stream_off counts from the session start; an
 * empty last packet ends a block and the next block may follow).  A framing
 * error stops the session (its record is still returned).  A packet larger
 * than slot_bytes is an error.  One thread per session. */
typedef struct hdfs_crc32c_session hdfs_crc32c_session;
int hdfs_crc32c_session_create(hdfs_crc32c_session **s, int proto, uint32_t chunk_size, int ctype,
    uint64_t slot_bytes, size_t nslots);
/* Write pointer and free bytes of the current slot. */
int hdfs_crc32c_session_buffer(hdfs_crc32c_session *s, void **wptr, uint64_t *room);
/* nbytes were written at the write pointer; a full slot is submitted. */
int hdfs_crc32c_session_commit(hdfs_crc32c_session *s, uint64_t nbytes);
/* Submit the current slot's complete packets now (end of input, or latency). */
int hdfs_crc32c_session_flush(hdfs_crc32c_session *s);
/* Up to max_pkts finished records; wait != 0 blocks until every submitted
 * slot is done.  Returns the first packet error among the returned records,
 * 0, or a negative status. */
int hdfs_crc32c_session_poll(hdfs_crc32c_session *s, hdfs_crc32c_packet *pkts, size_t max_pkts,
    size_t *npkts, int wait);
/* Bytes waiting in the current slot; submitted-but-unreturned packet count. */
int hdfs_crc32c_session_pending(const hdfs_crc32c_session *s, uint64_t *buffered, size_t *inflight);
void hdfs_crc32c_session_destroy(hdfs_crc32c_session *s);

/* ---- host-resident streaming (pipelined H2D / kernel / D2H) -------------- */
/* Per-chunk CRCs of a HOST buffer: pieces of piece_bytes (0 = 64 MiB, rounded
 * to whole 8-chunk tiles) are copied H2D on a copy stream into one of two
 * device slots while the other slot runs on a compute stream; CRCs come back
 * D2H behind each kernel.  Pageable buffers are host-registered for the call.
 * crcs_out: host u32[ceil(len/chunk_size)], wire order if HDFS_CRC32C_SEG_BE. */
int hdfs_crc32c_compute_host(const void *data, uint64_t len, uint32_t chunk_size, uint32_t flags,
    uint32_t crc_init, void *crcs_out, uint64_t piece_bytes);
/* Verify a HOST buffer against host expected CRCs; optional host bitmap out;
 * *first_bad = first bad chunk (UINT64_MAX if none), *mismatches = count. */
int hdfs_crc32c_verify_host(const void *data, uint64_t len, uint32_t chunk_size, uint32_t flags,
    uint32_t crc_init, const void *crcs, uint8_t *bitmap_out, uint64_t piece_bytes,
    uint64_t *first_bad, uint64_t *mismatches);
/* Pinned (page-locked) host memory for zero-copy-staging pipelines. */
int hdfs_crc32c_host_alloc(void **p, uint64_t bytes);
/* Only for blocks from hdfs_crc32c_host_alloc OF THE SAME LIBRARY (EINVAL
 * otherwise, and the block stays allocated): each loaded copy of the engine
 * (the release and the diagnostic build loaded side by side, say) keeps its
 * own registry of pinned memory (DMA-ed in place). */
int hdfs_crc32c_host_free(void *p);

/* ---- resident mailbox for the synchronous small calls ------------------- */
/* Opt-in latency mode for the reference's per-packet call pattern
 * (_verify_crcdata per received packet, src/datanode.c:2470-2476; the
 * drop-in _hdfs_crc32c family; compose_crcs): while a mailbox is open on the
 * engine's device, ONE workgroup of the engine stays resident on one CU with
 * its tables in LDS and serves the synchronous calls on <= 64 KiB of host
 * memory (chunk size a multiple of 64, or a single chunk) from a request
 * line in pinned memory -- no kernel launch per call.  Other calls keep
 * their one-launch path.  The resident kernel exits on its own after idle_ms
 * without a request (0: 50 ms; the next call relaunches it) and on destroy.
 * While a mailbox is open the engine's bulk kernels leave one CU per XCD to
 * it.  The resident kernel runs on a high-priority stream, usually a
 * hardware queue of its own; a process with GPU_MAX_HW_QUEUES or more
 * high-priority streams shares one with it.  Anything queued behind the
 * kernel on its queue -- another stream's work there, the marker a NULL-
 * stream copy, a free or a device-wide synchronisation puts on it -- makes it
 * leave at once (it watches its AQL queue's write index), and the next call
 * relaunches it: such work waits microseconds, not idle_ms (round 5's
 * 50 ms stalls, profiles/r06/r6c_mb_share.json vs r6e_mb_share.json).
 * One mailbox per device (EBUSY-style HDFS_CRC32C_EINVAL for a second). */
typedef struct hdfs_crc32c_mailbox hdfs_crc32c_mailbox;
int hdfs_crc32c_mailbox_create(hdfs_crc32c_mailbox **mb, uint32_t idle_ms);
/* Calls served by the resident kernel and kernel launches (first + relaunches after idle exits and yields). */
int hdfs_crc32c_mailbox_stats(const hdfs_crc32c_mailbox *mb, uint64_t *calls, uint64_t *launches);
int hdfs_crc32c_mailbox_destroy(hdfs_crc32c_mailbox *mb);

/* ---- device memory + synthetic data helpers (bench / tests) ------------- */
int hdfs_crc32c_dev_alloc(void **dptr, uint64_t bytes);
int hdfs_crc32c_dev_free(void *dptr);
int hdfs_crc32c_memcpy(void *dst, const void *src, uint64_t bytes, int kind /* 0 h2d, 1 d2h, 2 d2d */);
int hdfs_crc32c_memset(void *dptr, int value, uint64_t bytes);
int hdfs_crc32c_stream_create(void **stream);
int hdfs_crc32c_stream_destroy(void *stream);
int hdfs_crc32c_stream_sync(void *stream);
/* w[k] = splitmix64(seed, g0 + k), k < nwords (SURVEY.md 8c data). */
int hdfs_crc32c_fill_splitmix64(void *dptr, uint64_t nwords, uint64_t seed, uint64_t g0, void *stream);
/* Flip bit (i*bitmul) mod (8*chunk_len) of every chunk whose global index
 * i = chunk0 + local satisfies i % modulus == 0. */
int hdfs_crc32c_corrupt(void *dptr, uint64_t len, uint32_t chunk, uint64_t chunk0,
    uint64_t modulus, uint64_t bitmul, void *stream);
/* Elapsed device time of `iters` back-to-back plan executions on `stream`
 * measured with HIP events (ms per execution). */
int hdfs_crc32c_plan_time(hdfs_crc32c_plan *plan, void *stream, int iters, double *ms_per_iter);
/* hipDeviceSynchronize on the engine's device (with a mailbox open: the
 * engine's streams, the NULL stream and every stream hdfs_crc32c_stream_create
 * handed out, not the resident kernel). */
int hdfs_crc32c_device_sync(void);

#ifdef __cplusplus
}
#endif
#endif /* HADOOFUS_CRC32C_H */
