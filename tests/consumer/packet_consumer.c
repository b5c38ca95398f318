/*
 * C consumer of the packet-stream API (include/hadoofus_crc32c.h), written
 * the way a datanode receive loop would use it (src/datanode.c:2345-2494):
 * builds a v2 packet stream in memory (PacketHeaderProto encoded by hand,
 * CRCs from the engine's own write-path mirror hdfs_crc32c_compose_crcs),
 * corrupts one chunk, then verifies it (1) in one hdfs_crc32c_verify_packets
 * call and (2) through a streaming session fed in odd-sized "socket reads";
 * then (3) composes the packets of one write (hdfs_crc32c_compose_packets)
 * and reads them back through the verifier; (4) uploads the stream to the
 * GPU and reads two client windows out of it with the fused verify +
 * copy-out (hdfs_crc32c_read_packets: c_begin, remains_tot,
 * src/datanode.c:2478-2549), once into one buffer and once resumed over a
 * scatter list of small buffers (HDFS_CRC32C_AGAIN); (5) maps an engine failure the way a datanode
 * must -- an I/O error, never a checksum error;
 * (6) reads into host memory from the host and the device stream; (7)
 * verifies three device-resident blocks as asynchronous jobs and as one
 * batch (ABI 5); (8) reads through a reader; (9) writes a read to a file
 * descriptor (hdfs_crc32c_read_packets_fd).
 * Prints "0 failures" on success.  Test infrastructure (tests/test_abi.py
 * links it on CPU, tests/test_packets.py runs it on the GPU).
 */
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "hadoofus_crc32c.h"

#define NPK 40
#define DLEN 65536
#define CS 512

static int failures;

static void check(int cond, const char *what)
{
	if (!cond) {
		printf("FAIL: %s (%s)\n", what, hdfs_crc32c_last_error());
		failures++;
	}
}

static size_t put_be32(uint8_t *p, uint32_t v)
{
	p[0] = v >> 24; p[1] = v >> 16; p[2] = v >> 8; p[3] = v;
	return 4;
}

/* [plen s32][hlen u16][PacketHeaderProto]: fields 1,2 sfixed64, 3 bool, 4 sfixed32 */
static size_t put_header(uint8_t *p, int64_t off, int64_t seq, int last, int32_t dlen, int32_t crclen)
{
	size_t n = put_be32(p, (uint32_t)(4 + crclen + dlen));
	p[n++] = 0;
	p[n++] = 25;
	p[n++] = 0x09; memcpy(p + n, &off, 8); n += 8;
	p[n++] = 0x11; memcpy(p + n, &seq, 8); n += 8;
	p[n++] = 0x18; p[n++] = (uint8_t)(last != 0);
	p[n++] = 0x25; memcpy(p + n, &dlen, 4); n += 4;
	return n;
}

/* The datanode's mapping of an engine return code:
 * > 0 is the reference's own hdfs_error_numeric (error_from_hdfs), < 0 an
 * engine failure, which becomes an errno-kind error (error_from_errno(EIO))
 * -- never HDFS_ERR_DATANODE_BAD_CHECKSUM, which would make
 * _compose_client_read_status report ERROR_CHECKSUM for a healthy block
 * (src/datanode.c:1012-1013).  Returned here as {kind, value}. */
struct dn_error {
	int kind; /* 0 success, 1 hdfs error number, 2 errno */
	int num;
};
static struct dn_error map_engine_rc(int rc)
{
	struct dn_error e = { 0, 0 };
	if (rc > 0) {
		e.kind = 1;
		e.num = rc;
	} else if (rc < 0) {
		e.kind = 2;
		e.num = EIO;
	}
	return e;
}

int main(void)
{
	const size_t crclen = DLEN / CS * 4, pk = 31 + crclen + DLEN;
	const size_t total = NPK * pk + 31;
	uint8_t *s = malloc(total), *data = malloc(DLEN);
	hdfs_crc32c_packet rec[NPK + 1];
	size_t n = 0;
	uint64_t used = 0;
	uint32_t x = 12345;

	for (int k = 0; k < NPK; k++) {
		uint8_t *p = s + k * pk;
		for (int i = 0; i < DLEN; i++) {
			x = x * 1103515245u + 12345u;
			data[i] = (uint8_t)(x >> 16);
		}
		size_t h = put_header(p, (int64_t)k * DLEN, k, 0, DLEN, (int32_t)crclen);
		const void *base = data;
		size_t len = DLEN;
		check(hdfs_crc32c_compose_crcs(&base, &len, 1, DLEN, CS, HDFS_CRC32C_CSUM_CRC32C, p + h) == 0,
		    "compose_crcs");
		memcpy(p + h + crclen, data, DLEN);
	}
	put_header(s + NPK * pk, (int64_t)NPK * DLEN, NPK, 1, 0, 0);
	s[7 * pk + 31 + crclen + 3 * CS + 17] ^= 0x40; /* packet 7, chunk 3 */

	int rc = hdfs_crc32c_verify_packets(s, total, HDFS_CRC32C_PROTO_V2, CS, HDFS_CRC32C_CSUM_CRC32C,
	    rec, NPK + 1, &n, &used);
	check(rc == HDFS_CRC32C_ERR_DATANODE_BAD_CHECKSUM, "verify_packets rc");
	check(n == NPK + 1 && used == total, "verify_packets count");
	for (size_t i = 0; i < n; i++)
		check(rec[i].error == (i == 7 ? HDFS_CRC32C_ERR_DATANODE_BAD_CHECKSUM : 0) &&
		    rec[i].first_bad == (i == 7 ? 3 : -1), "per-packet verdict");

	hdfs_crc32c_session *sess = NULL;
	check(hdfs_crc32c_session_create(&sess, HDFS_CRC32C_PROTO_V2, CS, HDFS_CRC32C_CSUM_CRC32C,
	    1 << 20, 3) == 0, "session_create");
	size_t off = 0, got = 0, bad = 0;
	while (off < total && !failures) {
		void *w;
		uint64_t room;
		check(hdfs_crc32c_session_buffer(sess, &w, &room) == 0, "session_buffer");
		size_t chunk = 70001 < room ? 70001 : (size_t)room;
		if (chunk > total - off)
			chunk = total - off;
		memcpy(w, s + off, chunk); /* recv() would write here */
		check(hdfs_crc32c_session_commit(sess, chunk) == 0, "session_commit");
		off += chunk;
	}
	check(hdfs_crc32c_session_flush(sess) == 0, "session_flush");
	for (;;) {
		size_t k = 0;
		rc = hdfs_crc32c_session_poll(sess, rec, NPK + 1, &k, 1);
		check(rc >= 0, "session_poll");
		if (!k)
			break;
		for (size_t i = 0; i < k; i++)
			bad += rec[i].error != 0;
		got += k;
	}
	hdfs_crc32c_session_destroy(sess);
	check(got == NPK + 1 && bad == 1, "session records");

	/* write path: one 1 MiB + 100 B write at an unaligned block offset,
	 * composed by the engine (sizes first), sent as header buffer + data per
	 * packet, read back by the packet verifier */
	{
		const size_t wlen = (1 << 20) + 100;
		uint8_t *w = malloc(wlen), *hdr, *wire;
		hdfs_crc32c_out_packet *opk;
		size_t nopk = 0, wpos = 0;
		uint64_t hlen = 0;
		for (size_t i = 0; i < wlen; i++) {
			x = x * 1103515245u + 12345u;
			w[i] = (uint8_t)(x >> 16);
		}
		check(hdfs_crc32c_compose_packets(w, wlen, 1000, 5, HDFS_CRC32C_PROTO_V2, HDFS_CRC32C_CSUM_CRC32C, 1,
		    NULL, 0, NULL, 0, &nopk, &hlen) == 0, "compose_packets sizes");
		hdr = malloc(hlen);
		opk = calloc(nopk, sizeof(*opk));
		wire = malloc(hlen + wlen);
		check(hdfs_crc32c_compose_packets(w, wlen, 1000, 5, HDFS_CRC32C_PROTO_V2, HDFS_CRC32C_CSUM_CRC32C, 1,
		    hdr, hlen, opk, nopk, &nopk, &hlen) == 0, "compose_packets");
		check(nopk == 19 && opk[0].data_len == 24 && opk[nopk - 1].last, "compose_packets layout");
		for (size_t i = 0; i < nopk; i++) { /* writev(hdr part, data part) */
			memcpy(wire + wpos, hdr + opk[i].hdr_off, opk[i].hdr_len);
			wpos += opk[i].hdr_len;
			memcpy(wire + wpos, w + opk[i].data_off, (size_t)opk[i].data_len);
			wpos += (size_t)opk[i].data_len;
		}
		hdfs_crc32c_packet *rrec = calloc(nopk, sizeof(*rrec));
		rc = hdfs_crc32c_verify_packets(wire, wpos, HDFS_CRC32C_PROTO_V2, CS, HDFS_CRC32C_CSUM_CRC32C, rrec,
		    nopk, &n, &used);
		check(rc == 0 && n == nopk && used == wpos, "write -> read round trip");
		for (size_t i = 0; i < n; i++)
			check(rrec[i].seqno == opk[i].seqno && rrec[i].offset_in_block == opk[i].offset_in_block &&
			    rrec[i].data_len == opk[i].data_len && rrec[i].last == opk[i].last, "round-trip fields");
		free(rrec);
		free(wire);
		free(opk);
		free(hdr);
		free(w);
	}
	/* (4) the stream in device memory (GPU-direct receive), two client reads
	 * through the fused verify + copy-out */
	{
		void *dstream = NULL, *duser = NULL;
		const uint64_t ucap = 8 * DLEN;
		uint8_t *back = malloc(ucap);
		check(hdfs_crc32c_dev_alloc(&dstream, total) == 0 && hdfs_crc32c_dev_alloc(&duser, ucap) == 0, "dev_alloc");
		check(hdfs_crc32c_memcpy(dstream, s, total, 0) == 0, "upload");
		uint64_t delivered = 0;
		/* bloff = 8 * DLEN + 5, len = 2 * DLEN: the server starts at packet 8;
		 * its first 5 bytes are skipped, packet 10 gives 5 bytes, the read ends */
		hdfs_crc32c_iovec iov1 = {duser, ucap};
		rc = hdfs_crc32c_read_packets((uint8_t *)dstream + 8 * pk, total - 8 * pk, HDFS_CRC32C_PROTO_V2, CS,
		    HDFS_CRC32C_CSUM_CRC32C, 8 * (int64_t)DLEN + 5, 2 * (int64_t)DLEN, &iov1, 1, rec, NPK + 1, &n, &used,
		    &delivered);
		check(rc == 0 && n == 3 && delivered == 2 * DLEN && used == 3 * pk, "read window: clean read");
		check(hdfs_crc32c_memcpy(back, duser, delivered, 1) == 0, "download");
		for (size_t k = 0, at = 0; k < 3; k++) {
			const size_t skip = k == 0 ? 5 : 0, take = k == 2 ? 5 : DLEN - skip;
			check(memcmp(back + at, s + (8 + k) * pk + 31 + crclen + skip, take) == 0, "read window bytes");
			at += take;
		}
		/* bloff = 3 * DLEN + 1000 over packets 3.. with packet 7 corrupt: the
		 * read gets packets 3..6 (the first from byte 1000 on) and ends at
		 * packet 7 with BAD_CHECKSUM (src/datanode.c:1476-1479, 2470-2475):
		 * its record is the last, and the stream is consumed up to it */
		rc = hdfs_crc32c_read_packets((uint8_t *)dstream + 3 * pk, total - 3 * pk, HDFS_CRC32C_PROTO_V2, CS,
		    HDFS_CRC32C_CSUM_CRC32C, 3 * (int64_t)DLEN + 1000, 5 * (int64_t)DLEN + 777, &iov1, 1, rec, NPK + 1, &n,
		    &used, &delivered);
		check(rc == HDFS_CRC32C_ERR_DATANODE_BAD_CHECKSUM && n == 5 && rec[4].first_bad == 3 &&
		    rec[4].error == HDFS_CRC32C_ERR_DATANODE_BAD_CHECKSUM && used == 4 * pk &&
		    delivered == 4 * DLEN - 1000, "read window: bad packet");
		check(map_engine_rc(rc).kind == 1 && map_engine_rc(rc).num == HDFS_CRC32C_ERR_DATANODE_BAD_CHECKSUM,
		    "checksum error maps to the reference's error");
		/* the clean read again, into a user buffer of 3 pieces smaller than
		 * the read, in calls of one piece each: AGAIN until the last, each
		 * resuming where the previous stopped (stream + consumed, bloff +
		 * delivered, len - delivered), the bytes identical */
		{
			const uint64_t piece = DLEN / 2 + 3;  /* every piece ends inside a packet */
			uint64_t at_stream = 8 * pk, got_tot = 0;
			int64_t bloff = 8 * (int64_t)DLEN + 5, left = 2 * (int64_t)DLEN;
			int calls = 0;
			do {
				hdfs_crc32c_iovec iv = {(uint8_t *)duser + got_tot, piece};
				rc = hdfs_crc32c_read_packets((uint8_t *)dstream + at_stream, total - at_stream, HDFS_CRC32C_PROTO_V2,
				    CS, HDFS_CRC32C_CSUM_CRC32C, bloff, left, &iv, 1, rec, NPK + 1, &n, &used, &delivered);
				at_stream += used;
				got_tot += delivered;
				bloff += (int64_t)delivered;
				left -= (int64_t)delivered;
				calls++;
			} while (rc == HDFS_CRC32C_AGAIN && calls < 16);
			check(rc == 0 && got_tot == 2 * DLEN && calls == 4, "resumed read: AGAIN until complete");
			check(hdfs_crc32c_memcpy(back, duser, got_tot, 1) == 0, "download");
			for (size_t k = 0, at = 0; k < 3; k++) {
				const size_t skip = k == 0 ? 5 : 0, take = k == 2 ? 5 : DLEN - skip;
				check(memcmp(back + at, s + (8 + k) * pk + 31 + crclen + skip, take) == 0, "resumed read bytes");
				at += take;
			}
			/* the same read as one call over a scatter list of the pieces */
			hdfs_crc32c_iovec iv4[4];
			for (int j = 0; j < 4; j++) {
				iv4[j].base = (uint8_t *)duser + (uint64_t)j * piece;
				iv4[j].len = piece;
			}
			rc = hdfs_crc32c_read_packets((uint8_t *)dstream + 8 * pk, total - 8 * pk, HDFS_CRC32C_PROTO_V2, CS,
			    HDFS_CRC32C_CSUM_CRC32C, 8 * (int64_t)DLEN + 5, 2 * (int64_t)DLEN, iv4, 4, rec, NPK + 1, &n, &used,
			    &delivered);
			check(rc == 0 && delivered == 2 * DLEN && n == 3 && used == 3 * pk, "scatter read");
		}
		hdfs_crc32c_dev_free(duser);
		hdfs_crc32c_dev_free(dstream);
		free(back);
	}

	/* (5) an engine failure (here: a host-resident stream into a device
	 * buffer, which the engine refuses) is an I/O error for the datanode,
	 * not a checksum error */
	{
		uint64_t delivered = 0;
		void *dbuf = NULL;
		check(hdfs_crc32c_dev_alloc(&dbuf, DLEN) == 0, "dev_alloc");
		hdfs_crc32c_iovec dv = {dbuf, DLEN};
		rc = hdfs_crc32c_read_packets(s, total, HDFS_CRC32C_PROTO_V2, CS, HDFS_CRC32C_CSUM_CRC32C, 0, DLEN, &dv, 1,
		    rec, NPK + 1, &n, &used, &delivered);
		const struct dn_error e = map_engine_rc(rc);
		check(rc == HDFS_CRC32C_EINVAL && e.kind == 2 && e.num == EIO, "engine failure -> EIO");
		hdfs_crc32c_dev_free(dbuf);
	}
	/* (6) a host-memory datanode (ABI 5): the same client read from the
	 * host stream into the user's host iovecs in one call -- framed on the
	 * host, verified on the GPU, copied as src/datanode.c:2516 does -- and
	 * from the device stream into host memory */
	{
		uint64_t delivered = 0;
		uint8_t *u0 = malloc(DLEN), *u1 = malloc(2 * DLEN);
		hdfs_crc32c_iovec hv[2] = {{u0, DLEN}, {u1, 2 * DLEN}};
		rc = hdfs_crc32c_read_packets(s + 8 * pk, total - 8 * pk, HDFS_CRC32C_PROTO_V2, CS, HDFS_CRC32C_CSUM_CRC32C,
		    8 * (int64_t)DLEN + 5, 2 * (int64_t)DLEN, hv, 2, rec, NPK + 1, &n, &used, &delivered);
		check(rc == 0 && n == 3 && delivered == 2 * DLEN && used == 3 * pk, "host read: records");
		check(memcmp(u0, s + 8 * pk + 31 + crclen + 5, DLEN - 5) == 0 &&
		    memcmp(u0 + DLEN - 5, s + 9 * pk + 31 + crclen, 5) == 0 &&
		    memcmp(u1, s + 9 * pk + 31 + crclen + 5, DLEN - 5) == 0 &&
		    memcmp(u1 + DLEN - 5, s + 10 * pk + 31 + crclen, 5) == 0, "host read: bytes");
		/* the bad packet ends the read there, as on the device */
		rc = hdfs_crc32c_read_packets(s + 3 * pk, total - 3 * pk, HDFS_CRC32C_PROTO_V2, CS, HDFS_CRC32C_CSUM_CRC32C,
		    3 * (int64_t)DLEN + 1000, 5 * (int64_t)DLEN + 777, hv, 2, rec, NPK + 1, &n, &used, &delivered);
		check(rc == HDFS_CRC32C_AGAIN && n == 3 && delivered == 3 * DLEN, "host read: buffers fill before the bad packet");
		void *dstream = NULL;
		check(hdfs_crc32c_dev_alloc(&dstream, total) == 0 && hdfs_crc32c_memcpy(dstream, s, total, 0) == 0, "upload");
		memset(u0, 0, DLEN);
		memset(u1, 0, 2 * DLEN);
		rc = hdfs_crc32c_read_packets((uint8_t *)dstream + 8 * pk, total - 8 * pk, HDFS_CRC32C_PROTO_V2, CS,
		    HDFS_CRC32C_CSUM_CRC32C, 8 * (int64_t)DLEN + 5, 2 * (int64_t)DLEN, hv, 2, rec, NPK + 1, &n, &used,
		    &delivered);
		check(rc == 0 && delivered == 2 * DLEN && memcmp(u1 + DLEN - 5, s + 10 * pk + 31 + crclen, 5) == 0,
		    "device stream into host memory");
		/* (7) three received blocks in HBM: asynchronous jobs, and one batch */
		void *blk[3] = {dstream, NULL, NULL};
		uint64_t blen[3] = {total, total, total};
		for (int b = 1; b < 3; b++)
			check(hdfs_crc32c_dev_alloc(&blk[b], total) == 0 && hdfs_crc32c_memcpy(blk[b], s, total, 0) == 0,
			    "upload block");
		hdfs_crc32c_job *job[3];
		for (int b = 0; b < 3; b++)
			check(hdfs_crc32c_verify_packets_submit(blk[b], total, HDFS_CRC32C_PROTO_V2, CS, HDFS_CRC32C_CSUM_CRC32C,
			    NPK + 1, &job[b]) == 0, "submit");
		for (int b = 2; b >= 0; b--) {
			rc = hdfs_crc32c_job_wait(job[b], rec, NPK + 1, &n, &used);
			check(rc == HDFS_CRC32C_ERR_DATANODE_BAD_CHECKSUM && n == NPK + 1 && used == total &&
			    rec[7].first_bad == 3, "job wait");
		}
		hdfs_crc32c_packet *brec = calloc(3 * (NPK + 1), sizeof(*brec));
		size_t bn[3];
		uint64_t bused[3];
		int brc[3];
		check(hdfs_crc32c_verify_blocks_submit((const void *const *)blk, blen, 3, HDFS_CRC32C_PROTO_V2, CS,
		    HDFS_CRC32C_CSUM_CRC32C, NPK + 1, &job[0]) == 0, "blocks submit");
		rc = hdfs_crc32c_job_wait_blocks(job[0], brec, NPK + 1, bn, bused, brc);
		check(rc == HDFS_CRC32C_ERR_DATANODE_BAD_CHECKSUM, "blocks wait rc");
		for (int b = 0; b < 3; b++)
			check(brc[b] == HDFS_CRC32C_ERR_DATANODE_BAD_CHECKSUM && bn[b] == NPK + 1 && bused[b] == total &&
			    brec[b * (NPK + 1) + 7].first_bad == 3 && brec[b * (NPK + 1) + NPK].last, "blocks wait records");
		free(brec);
		/* (8) the clean client read once more through a reader (ABI 5):
		 * verified once at open, then delivered piece by piece into host
		 * memory, each piece ending inside a packet (src/datanode.c:2547-2549) */
		{
			hdfs_crc32c_reader *rdr = NULL;
			check(hdfs_crc32c_reader_open((uint8_t *)blk[0] + 8 * pk, total - 8 * pk, HDFS_CRC32C_PROTO_V2, CS,
			    HDFS_CRC32C_CSUM_CRC32C, 8 * (int64_t)DLEN + 5, 2 * (int64_t)DLEN, NPK + 1, &rdr) == 0, "reader open");
			const uint64_t piece = DLEN / 2 + 3;
			uint64_t got_tot = 0;
			size_t nrec = 0;
			int calls = 0;
			memset(u1, 0, 2 * DLEN);
			do {
				const uint64_t left = 2 * DLEN - got_tot;
				hdfs_crc32c_iovec iv = {u1 + got_tot, left < piece ? left : piece};
				rc = hdfs_crc32c_reader_next(rdr, &iv, 1, rec + nrec, NPK + 1 - nrec, &n, &used, &delivered);
				nrec += n;
				got_tot += delivered;
				calls++;
			} while (rc == HDFS_CRC32C_AGAIN && calls < 16);
			hdfs_crc32c_reader_close(rdr);
			check(rc == 0 && got_tot == 2 * DLEN && nrec == 3 && used == 3 * pk && calls == 4, "reader: pieces");
			check(memcmp(u1, s + 8 * pk + 31 + crclen + 5, DLEN - 5) == 0 &&
			    memcmp(u1 + DLEN - 5, s + 9 * pk + 31 + crclen, DLEN) == 0 &&
			    memcmp(u1 + 2 * DLEN - 5, s + 10 * pk + 31 + crclen, 5) == 0, "reader: bytes");
		}
		/* (9) the same client read written to a file descriptor, as
		 * hdfs_datanode_read_file does (pwrite at fdoffset,
		 * src/datanode.c:2531-2541), at file offset 100 */
		{
			char path[] = "/tmp/hdfs_crc32c_fd_XXXXXX";
			const int fd = mkstemp(path);
			check(fd >= 0, "mkstemp");
			rc = hdfs_crc32c_read_packets_fd((uint8_t *)blk[0] + 8 * pk, total - 8 * pk, HDFS_CRC32C_PROTO_V2, CS,
			    HDFS_CRC32C_CSUM_CRC32C, 8 * (int64_t)DLEN + 5, 2 * (int64_t)DLEN, fd, 100, rec, NPK + 1, &n, &used,
			    &delivered);
			check(rc == 0 && n == 3 && used == 3 * pk && delivered == 2 * DLEN, "fd read: records");
			memset(u1, 0, 2 * DLEN);
			check(pread(fd, u1, 2 * DLEN, 100) == (ssize_t)(2 * DLEN), "fd read: pread");
			check(memcmp(u1, s + 8 * pk + 31 + crclen + 5, DLEN - 5) == 0 &&
			    memcmp(u1 + 2 * DLEN - 5, s + 10 * pk + 31 + crclen, 5) == 0, "fd read: bytes");
			/* the read across the bad packet: the bytes before it, then its error */
			rc = hdfs_crc32c_read_packets_fd((uint8_t *)blk[0] + 3 * pk, total - 3 * pk, HDFS_CRC32C_PROTO_V2, CS,
			    HDFS_CRC32C_CSUM_CRC32C, 3 * (int64_t)DLEN + 1000, 5 * (int64_t)DLEN, fd, 0, rec, NPK + 1, &n, &used,
			    &delivered);
			check(rc == HDFS_CRC32C_ERR_DATANODE_BAD_CHECKSUM && n == 5 && delivered == 4 * DLEN - 1000,
			    "fd read: ends at the bad packet");
			close(fd);
			unlink(path);
		}
		for (int b = 0; b < 3; b++)
			hdfs_crc32c_dev_free(blk[b]);
		free(u0);
		free(u1);
	}
	printf("%d failures\n", failures);
	free(s);
	free(data);
	return failures != 0;
}
