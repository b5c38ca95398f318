/*
 * A datanode's stream of received blocks in C (GPU box): NB (argv[1], 16 by
 * default, at most 64) device-resident
 * 128 MiB block transfers (2 048 v2 packets of 64 KiB + the empty last one,
 * composed by hdfs_crc32c_compose_packets from device-filled data), verified
 *   - synchronously, one hdfs_crc32c_verify_packets per block;
 *   - as asynchronous jobs with W = 4 / 8 / 16 outstanding (wait for the
 *     oldest before the next submit);
 *   - as batches of 8 blocks (hdfs_crc32c_verify_blocks_submit, two in flight).
 * The same patterns as tools/device_stream_bench.py's stream_of_blocks,
 * without the Python caller: what a C datanode sees.  Best of 5; prints one
 * JSON line (us per block).
 *   cc -O2 -I include tools/probes/jobs_bench.c -L hadoofus_amd/lib -lhadoofus_crc32c -o tools/probes/jobs_bench
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "hadoofus_crc32c.h"

#define NBMAX 64
#define BLOCK (128ull << 20)

static double now_us(void)
{
	struct timespec t;
	clock_gettime(CLOCK_MONOTONIC, &t);
	return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

#define CHK(x) do { int rc_ = (x); if (rc_ < 0) { fprintf(stderr, "%s: %d %s\n", #x, rc_, hdfs_crc32c_last_error()); exit(1); } } while (0)

int main(int argc, char **argv)
{
	const int NB = argc > 1 ? atoi(argv[1]) : 16;
	if (NB < 8 || NB > NBMAX || NB % 8) { fprintf(stderr, "blocks: a multiple of 8 in [8, %d]\n", NBMAX); return 1; }
	/* one block's wire image, built on the host from composed headers */
	void *ddata = NULL;
	CHK(hdfs_crc32c_dev_alloc(&ddata, BLOCK));
	CHK(hdfs_crc32c_fill_splitmix64(ddata, BLOCK / 8, 9, 0, NULL));
	CHK(hdfs_crc32c_device_sync());
	size_t npk = 0;
	uint64_t hlen = 0;
	CHK(hdfs_crc32c_compose_packets(ddata, BLOCK, 0, 0, HDFS_CRC32C_PROTO_V2, HDFS_CRC32C_CSUM_CRC32C, 1, NULL, 0,
	    NULL, 0, &npk, &hlen));
	uint8_t *hdr = malloc(hlen);
	hdfs_crc32c_out_packet *op = calloc(npk, sizeof(*op));
	CHK(hdfs_crc32c_compose_packets(ddata, BLOCK, 0, 0, HDFS_CRC32C_PROTO_V2, HDFS_CRC32C_CSUM_CRC32C, 1, hdr, hlen,
	    op, npk, &npk, &hlen));
	uint8_t *data = malloc(BLOCK);
	CHK(hdfs_crc32c_memcpy(data, ddata, BLOCK, 1));
	const uint64_t wlen = hlen + BLOCK;
	uint8_t *wire = malloc(wlen);
	uint64_t w = 0;
	for (size_t i = 0; i < npk; i++) {
		memcpy(wire + w, hdr + op[i].hdr_off, op[i].hdr_len);
		w += op[i].hdr_len;
		memcpy(wire + w, data + op[i].data_off, (size_t)op[i].data_len);
		w += (uint64_t)op[i].data_len;
	}
	void *blk[NBMAX];
	uint64_t blen[NBMAX];
	for (int b = 0; b < NB; b++) {
		CHK(hdfs_crc32c_dev_alloc(&blk[b], wlen));
		CHK(hdfs_crc32c_memcpy(blk[b], wire, wlen, 0));
		blen[b] = wlen;
	}
	CHK(hdfs_crc32c_device_sync());
	const size_t maxpk = npk + 8;
	hdfs_crc32c_packet *rec = calloc(NB * maxpk, sizeof(*rec));
	size_t n = 0, bn[NBMAX];
	uint64_t used = 0, bused[NBMAX];
	int brc[NBMAX];
	double best[6] = {1e18, 1e18, 1e18, 1e18, 1e18, 1e18};
	for (int rep = 0; rep < 6; rep++) {
		double t0 = now_us();
		for (int b = 0; b < NB; b++) {
			int rc = hdfs_crc32c_verify_packets(blk[b], wlen, HDFS_CRC32C_PROTO_V2, 512, HDFS_CRC32C_CSUM_CRC32C, rec,
			    maxpk, &n, &used);
			if (rc != 0 || n != npk || used != wlen) { fprintf(stderr, "sync %d %zu\n", rc, n); return 1; }
		}
		double t = now_us() - t0;
		if (rep && t < best[0]) best[0] = t;
		const int wins[3] = {4, 8, 16};
		for (int k = 0; k < 3; k++) {
			const int W = wins[k];
			hdfs_crc32c_job *job[NB];
			int head = 0;
			t0 = now_us();
			for (int b = 0; b < NB; b++) {
				if (b - head == W) {
					int rc = hdfs_crc32c_job_wait(job[head], rec + (size_t)(head % W) * maxpk, maxpk, &n, &used);
					if (rc != 0 || n != npk) { fprintf(stderr, "wait %d\n", rc); return 1; }
					head++;
				}
				CHK(hdfs_crc32c_verify_packets_submit(blk[b], wlen, HDFS_CRC32C_PROTO_V2, 512, HDFS_CRC32C_CSUM_CRC32C,
				    maxpk, &job[b]));
			}
			for (; head < NB; head++) {
				int rc = hdfs_crc32c_job_wait(job[head], rec + (size_t)(head % W) * maxpk, maxpk, &n, &used);
				if (rc != 0 || n != npk) { fprintf(stderr, "wait %d\n", rc); return 1; }
			}
			t = now_us() - t0;
			if (rep && t < best[1 + k]) best[1 + k] = t;
		}
		t0 = now_us();
		{  /* batches of 8 blocks, two in flight */
			hdfs_crc32c_job *bj[NBMAX / 8];
			for (int g = 0; g < NB / 8; g++) {
				if (g >= 2) {
					int rc = hdfs_crc32c_job_wait_blocks(bj[g - 2], rec, maxpk, bn, bused, brc);
					if (rc != 0 || bn[0] != npk) { fprintf(stderr, "blocks %d\n", rc); return 1; }
				}
				CHK(hdfs_crc32c_verify_blocks_submit((const void *const *)(blk + 8 * g), blen + 8 * g, 8,
				    HDFS_CRC32C_PROTO_V2, 512, HDFS_CRC32C_CSUM_CRC32C, maxpk, &bj[g]));
			}
			for (int g = NB / 8 - 2; g < NB / 8; g++) {
				int rc = hdfs_crc32c_job_wait_blocks(bj[g], rec, maxpk, bn, bused, brc);
				if (rc != 0 || bn[0] != npk) { fprintf(stderr, "blocks %d\n", rc); return 1; }
			}
		}
		t = now_us() - t0;
		if (rep && t < best[4]) best[4] = t;
	}
	printf("{\"blocks\": %d, \"block_bytes\": %llu, \"packets\": %zu, \"us_per_block\": {\"sync\": %.1f, "
	    "\"jobs\": %.1f, \"jobs_inflight8\": %.1f, \"jobs_inflight16\": %.1f, \"batch8_two_in_flight\": %.1f}, "
	    "\"note\": \"C caller, best of 5 after one warm-up pass\"}\n",
	    NB, (unsigned long long)BLOCK, npk, best[0] / NB, best[1] / NB, best[2] / NB, best[3] / NB, best[4] / NB);
	return 0;
}
