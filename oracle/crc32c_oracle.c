/*
 * crc32c_oracle.c -- CPU ORACLE for the hadoofus CRC32C hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in hadoofus_amd/ links, loads or calls
 * this file; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg do, and only as the checker (or the timed CPU baseline), never as the
 * thing that is measured or shipped.
 *
 * This is our own restatement of the reference's algorithms (nothing copied);
 * every function cites the reference file:line it follows
 * (paths relative to alexsmith1612/hadoofus, mounted at /root/reference):
 *
 *   oracle_crc32c_sw      <- src/crc32c_sw.c:63 (poly), :72-94 (tables),
 *                            :97-127 (slicing-by-8 little-endian loop),
 *                            :207-213 (_hdfs_sw_crc32c entry)
 *   oracle_crc32c_hw      <- src/crc32c_sse42.c:80-81 (LONG/SHORT),
 *                            :99-200 (GF(2) zeros operator + shift tables),
 *                            :214-381 (3-way interleaved crc32q loop)
 *   oracle_verify_crcdata <- src/datanode.c:2931-2963 (_verify_crcdata) and
 *                            the framing check of src/datanode.c:2438-2446
 *   oracle_read_packets   <- src/datanode.c:1476-1481 (read loop), :2428-2549
 *                            (_process_recv_packet read window +
 *                            _recv_packet_copy_data)
 *   oracle_compose_crcs   <- src/datanode.c:2814-2860 (write-path CRC loop,
 *                            chained across iovec fragments)
 *   oracle_compose_packets <- src/datanode.c:2583-2609 (_send_packet packet
 *                            sizing) + :2781-2868 (_compose_data_packet_header)
 *   oracle_zeros/combine  <- src/crc32c_sse42.c:99-200 generalised to any n
 *   oracle_crc32_zlib     <- zlib crc32() (third-party dependency of
 *                            src/datanode.c:12,2832-2845,2940-2952, not in
 *                            /root/reference; pinned version: the image's
 *                            zlib 1.2.11).  Restates zlib's published
 *                            algorithm: reflected CRC-32, poly 0xEDB88320,
 *                            register pre/post inverted, crc32(0,..) start.
 *
 * Parity is PINNED: tests/test_oracle.py checks every function here against
 * the reference's own KATs (tests/t_unit.c:146-217) and against golden
 * vectors produced by the reference compiled unchanged from /root/reference
 * (oracle/_ref, recipe in oracle/Makefile, generator oracle/gen_golden.py).
 * The CRC32 (zlib) leg is pinned against zlib 1.2.11 itself (Python's zlib
 * module in this container; fixtures tests/golden/zlib_*.json).
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>
#include <pthread.h>
#include <time.h>

#define ORACLE_POLY 0x82f63b78u /* src/crc32c_sw.c:63 */
#define ORACLE_POLY_ZLIB 0xedb88320u /* zlib crc32(), HDFS_CSUM_CRC32 */
#define ORACLE_CSUM_NULL 0   /* include/hadoofus/objects.h:172 */
#define ORACLE_CSUM_CRC32 1  /* include/hadoofus/objects.h:173 */
#define ORACLE_CSUM_CRC32C 2

/* ------------------------------------------------------------------ */
/* Software slicing-by-8 (src/crc32c_sw.c:72-127)                      */
/* ------------------------------------------------------------------ */
static uint32_t sw_tab[8][256];
static int sw_ready;

static void sw_init(void)
{
	for (uint32_t n = 0; n < 256; n++) {
		uint32_t c = n;
		for (int k = 0; k < 8; k++)
			c = (c >> 1) ^ (ORACLE_POLY & (0u - (c & 1u)));
		sw_tab[0][n] = c;
	}
	for (uint32_t n = 0; n < 256; n++) {
		uint32_t c = sw_tab[0][n];
		for (int t = 1; t < 8; t++) {
			c = sw_tab[0][c & 0xff] ^ (c >> 8);
			sw_tab[t][n] = c;
		}
	}
	sw_ready = 1;
}

static uint32_t zlib_tab[256];

static void zlib_init(void)
{
	for (uint32_t n = 0; n < 256; n++) {
		uint32_t c = n;
		for (int k = 0; k < 8; k++)
			c = (c >> 1) ^ (ORACLE_POLY_ZLIB & (0u - (c & 1u)));
		zlib_tab[n] = c;
	}
}

__attribute__((constructor)) static void oracle_ctor(void)
{
	sw_init();
	zlib_init();
}

/* zlib crc32(crc, buf, len): byte-at-a-time table form of the reflected
 * CRC-32 (see header for the pinning). */
uint32_t oracle_crc32_zlib(uint32_t crc, const void *buf, size_t len)
{
	const uint8_t *p = buf;
	uint32_t c = ~crc;
	while (len--)
		c = zlib_tab[(c ^ *p++) & 0xff] ^ (c >> 8);
	return ~c;
}


uint32_t oracle_crc32c_sw(uint32_t crc, const void *buf, size_t len)
{
	const uint8_t *p = buf;
	uint32_t c = ~crc;

	while (len && ((uintptr_t)p & 7)) {
		c = sw_tab[0][(c ^ *p++) & 0xff] ^ (c >> 8);
		len--;
	}
	while (len >= 8) {
		uint64_t w;
		memcpy(&w, p, 8);
		w ^= c;
		c = sw_tab[7][w & 0xff] ^ sw_tab[6][(w >> 8) & 0xff] ^
		    sw_tab[5][(w >> 16) & 0xff] ^ sw_tab[4][(w >> 24) & 0xff] ^
		    sw_tab[3][(w >> 32) & 0xff] ^ sw_tab[2][(w >> 40) & 0xff] ^
		    sw_tab[1][(w >> 48) & 0xff] ^ sw_tab[0][w >> 56];
		p += 8;
		len -= 8;
	}
	while (len--)
		c = sw_tab[0][(c ^ *p++) & 0xff] ^ (c >> 8);
	return ~c;
}

/* Bitwise definition; the slowest and most obviously-correct form. */
uint32_t oracle_crc32c_bitwise(uint32_t crc, const void *buf, size_t len)
{
	const uint8_t *p = buf;
	uint32_t c = ~crc;
	while (len--) {
		c ^= *p++;
		for (int k = 0; k < 8; k++)
			c = (c >> 1) ^ (ORACLE_POLY & (0u - (c & 1u)));
	}
	return ~c;
}

/* ------------------------------------------------------------------ */
/* GF(2) "append n zero bytes" operator (src/crc32c_sse42.c:99-200)   */
/* Works on the raw (pre-inverted) register.                           */
/* ------------------------------------------------------------------ */
static uint32_t gf2_times(const uint32_t *mat, uint32_t vec)
{
	uint32_t sum = 0;
	while (vec) {
		if (vec & 1)
			sum ^= *mat;
		vec >>= 1;
		mat++;
	}
	return sum;
}

static void gf2_square(uint32_t *sq, const uint32_t *mat)
{
	for (int n = 0; n < 32; n++)
		sq[n] = gf2_times(mat, mat[n]);
}

/* Operator for n zero BYTES, any n (the reference builds powers of two only;
 * this is the same squaring ladder applied per set bit of n). */
void oracle_zeros_op(uint32_t op[32], uint64_t nbytes)
{
	uint32_t pow[32], tmp[32], acc[32];
	/* identity */
	for (int i = 0; i < 32; i++)
		acc[i] = 1u << i;
	/* operator for one zero bit */
	pow[0] = ORACLE_POLY;
	for (int i = 1; i < 32; i++)
		pow[i] = 1u << (i - 1);
	/* square 3 times: one zero byte */
	gf2_square(tmp, pow);
	gf2_square(pow, tmp);
	gf2_square(tmp, pow);
	memcpy(pow, tmp, sizeof(pow));
	while (nbytes) {
		if (nbytes & 1) {
			for (int i = 0; i < 32; i++)
				tmp[i] = gf2_times(pow, acc[i]);
			memcpy(acc, tmp, sizeof(acc));
		}
		nbytes >>= 1;
		if (nbytes) {
			gf2_square(tmp, pow);
			memcpy(pow, tmp, sizeof(pow));
		}
	}
	memcpy(op, acc, sizeof(acc));
}

uint32_t oracle_zeros_apply(uint32_t reg, uint64_t nbytes)
{
	uint32_t op[32];
	oracle_zeros_op(op, nbytes);
	return gf2_times(op, reg);
}

/* c(A||B) from c(A), c(B), |B| -- public (conditioned) CRC values. */
uint32_t oracle_crc32c_combine(uint32_t crcA, uint32_t crcB, uint64_t lenB)
{
	/* raw registers: regA = ~crcA ; CRC(~0, A||B) = Z_lenB(~crcA) ^ raw(B)
	 * and c(B) = ~(Z_lenB(~0) ^ raw(B)). */
	uint32_t zA = oracle_zeros_apply(~crcA, lenB);
	uint32_t zI = oracle_zeros_apply(~0u, lenB);
	return ~(zA ^ zI ^ ~crcB);
}

/* Byte tables for an operator: zt[m][e] = op(e << 8m). */
static void zeros_tables(uint32_t zt[4][256], uint64_t nbytes)
{
	uint32_t op[32];
	oracle_zeros_op(op, nbytes);
	for (uint32_t e = 0; e < 256; e++)
		for (int m = 0; m < 4; m++)
			zt[m][e] = gf2_times(op, e << (8 * m));
}

static inline uint32_t zshift(uint32_t zt[4][256], uint32_t c)
{
	return zt[0][c & 0xff] ^ zt[1][(c >> 8) & 0xff] ^ zt[2][(c >> 16) & 0xff] ^
	    zt[3][c >> 24];
}

/* ------------------------------------------------------------------ */
/* SSE4.2 3-way interleaved restatement (src/crc32c_sse42.c:214-381)   */
/* ------------------------------------------------------------------ */
#if defined(__x86_64__)
#define HW_LONG 128  /* src/crc32c_sse42.c:80 */
#define HW_SHORT 64  /* src/crc32c_sse42.c:81 */
static uint32_t hw_long[4][256], hw_2long[4][256], hw_short[4][256], hw_2short[4][256];
static int hw_ready;

__attribute__((constructor)) static void oracle_hw_ctor(void)
{
	zeros_tables(hw_long, HW_LONG);
	zeros_tables(hw_2long, 2 * HW_LONG);
	zeros_tables(hw_short, HW_SHORT);
	zeros_tables(hw_2short, 2 * HW_SHORT);
	hw_ready = 1;
}

__attribute__((target("sse4.2")))
static inline uint64_t c8(uint64_t c, uint8_t b) { return __builtin_ia32_crc32qi((uint32_t)c, b); }
__attribute__((target("sse4.2")))
static inline uint64_t c64(uint64_t c, uint64_t w) { return __builtin_ia32_crc32di(c, w); }

__attribute__((target("sse4.2")))
uint32_t oracle_crc32c_hw(uint32_t crc, const void *buf, size_t len)
{
	const uint8_t *p = buf;
	uint64_t s0 = (uint32_t)~crc, s1, s2, acc;

	while (len && ((uintptr_t)p & 7)) {
		s0 = c8(s0, *p++);
		len--;
	}
	/* three streams of LONG bytes, merged with the zeros operator */
	acc = 0;
	while (len >= 3 * HW_LONG) {
		const uint8_t *end = p + HW_LONG;
		s1 = 0;
		s2 = 0;
		do {
			uint64_t a, b, c;
			memcpy(&a, p, 8);
			memcpy(&b, p + HW_LONG, 8);
			memcpy(&c, p + 2 * HW_LONG, 8);
			s0 = c64(s0, a);
			s1 = c64(s1, b);
			s2 = c64(s2, c);
			p += 8;
		} while (p < end);
		acc = zshift(hw_long, (uint32_t)acc) ^ (uint32_t)s0;
		s1 = zshift(hw_long, (uint32_t)s1);
		acc = zshift(hw_2long, (uint32_t)acc) ^ (uint32_t)s1;
		s0 = s2;
		p += 2 * HW_LONG;
		len -= 3 * HW_LONG;
	}
	s0 ^= acc;
	acc = 0;
	while (len >= 3 * HW_SHORT) {
		const uint8_t *end = p + HW_SHORT;
		s1 = 0;
		s2 = 0;
		do {
			uint64_t a, b, c;
			memcpy(&a, p, 8);
			memcpy(&b, p + HW_SHORT, 8);
			memcpy(&c, p + 2 * HW_SHORT, 8);
			s0 = c64(s0, a);
			s1 = c64(s1, b);
			s2 = c64(s2, c);
			p += 8;
		} while (p < end);
		acc = zshift(hw_short, (uint32_t)acc) ^ (uint32_t)s0;
		s1 = zshift(hw_short, (uint32_t)s1);
		acc = zshift(hw_2short, (uint32_t)acc) ^ (uint32_t)s1;
		s0 = s2;
		p += 2 * HW_SHORT;
		len -= 3 * HW_SHORT;
	}
	s0 ^= acc;
	while (len >= 8) {
		uint64_t a;
		memcpy(&a, p, 8);
		s0 = c64(s0, a);
		p += 8;
		len -= 8;
	}
	while (len--)
		s0 = c8(s0, *p++);
	return ~(uint32_t)s0;
}

int oracle_have_hw(void)
{
	unsigned a, b, c, d;
	__asm__("cpuid" : "=a"(a), "=b"(b), "=c"(c), "=d"(d) : "a"(1), "c"(0));
	return (c >> 20) & 1; /* src/crc32c.c:20-28 */
}
#else
uint32_t oracle_crc32c_hw(uint32_t crc, const void *buf, size_t len)
{
	return oracle_crc32c_sw(crc, buf, len);
}
int oracle_have_hw(void) { return 0; }
#endif

/* ------------------------------------------------------------------ */
/* Datanode call sites                                                 */
/* ------------------------------------------------------------------ */
static inline uint32_t be32dec(const uint8_t *p) /* src/util.h:68-80 */
{
	return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

static inline void be32enc(uint8_t *p, uint32_t v) /* src/util.h:82-92 */
{
	p[0] = v >> 24;
	p[1] = v >> 16;
	p[2] = v >> 8;
	p[3] = v;
}

static uint32_t crc_of(int ctype, uint32_t crc, const void *buf, size_t len)
{
	return ctype == ORACLE_CSUM_CRC32 ? oracle_crc32_zlib(crc, buf, len)
					  : oracle_crc32c_sw(crc, buf, len);
}

/* Reference error numbers (include/objects.h:21-113, values checked by
 * compiling the reference header in this container). */
#define ORACLE_ERR_CRC_LEN 26
#define ORACLE_ERR_BAD_CHECKSUM 29

/*
 * _verify_crcdata (src/datanode.c:2931-2963) on [BE crcs (crcdlen) | data
 * (dlen)] for CRC32C, preceded by the CRC-length framing check of
 * _process_recv_packet (src/datanode.c:2441-2442).  Returns 0, or the
 * reference error number; *first_bad receives the first mismatching chunk
 * (-1 if none), which is where the reference's loop returns.
 */
int oracle_verify_crcdata(const void *crcdata, int32_t chunksize, int32_t crcdlen,
    int32_t dlen, int ctype, int32_t *first_bad)
{
	const uint8_t *crcs = crcdata;
	const uint8_t *data = crcs + crcdlen;
	*first_bad = -1;
	if (crcdlen != ((dlen + chunksize - 1) / chunksize) * 4)
		return ORACLE_ERR_CRC_LEN;
	for (int32_t i = 0; i < (dlen + chunksize - 1) / chunksize; i++) {
		int32_t clen = dlen - i * chunksize;
		if (clen > chunksize)
			clen = chunksize;
		/* crcinit: crc32(0L, Z_NULL, 0) == 0 for CRC32, 0 for CRC32C
		 * (src/datanode.c:2940-2943) */
		uint32_t crc = crc_of(ctype, 0, data + (size_t)i * chunksize, clen);
		if (crc != be32dec(crcs + 4 * (size_t)i)) {
			*first_bad = i;
			return ORACLE_ERR_BAD_CHECKSUM;
		}
	}
	return 0;
}

/*
 * Write-path loop of _compose_data_packet_header (src/datanode.c:2814-2860):
 * one BE CRC per CHUNK of the packet, chained across the iovec fragments
 * (iov_base[k], iov_len[k]).  Writes ceil(total/chunk) * 4 bytes.
 */
void oracle_compose_crcs(const void *const *iov_base, const size_t *iov_len, int iovcnt,
    size_t total, uint32_t chunk, int ctype, void *crc_be_out)
{
	uint8_t *out = crc_be_out;
	size_t nch = (total + chunk - 1) / chunk;
	int k = 0;
	size_t off = 0;
	for (size_t i = 0; i < nch; i++) {
		uint32_t crc = 0;
		size_t clen = total - i * chunk;
		if (clen > chunk)
			clen = chunk;
		while (clen > 0 && k < iovcnt) {
			size_t t = iov_len[k] - off;
			if (t > clen)
				t = clen;
			crc = crc_of(ctype, crc, (const uint8_t *)iov_base[k] + off, t);
			clen -= t;
			off += t;
			if (off == iov_len[k]) {
				k++;
				off = 0;
			}
		}
		be32enc(out + 4 * i, crc);
	}
}

/* Per-chunk CRCs (LE u32 out) of a buffer; the last chunk may be partial.
 * use_hw: 0 sw slicing, 1 SSE4.2, 2 zlib CRC32. */
void oracle_chunk_crcs(const void *data, uint64_t len, uint32_t chunk, uint32_t *out, int use_hw)
{
	const uint8_t *p = data;
	uint64_t nch = (len + chunk - 1) / chunk;
	for (uint64_t i = 0; i < nch; i++) {
		uint64_t clen = len - i * chunk;
		if (clen > chunk)
			clen = chunk;
		out[i] = use_hw == 2 ? oracle_crc32_zlib(0, p + i * chunk, clen)
			 : use_hw ? oracle_crc32c_hw(0, p + i * chunk, clen)
				  : oracle_crc32c_sw(0, p + i * chunk, clen);
	}
}

/* ------------------------------------------------------------------ */
/* Packet streams: _recv_packet -> _process_recv_packet -> _verify_crcdata */
/* (src/datanode.c:2345-2494, 2931-2963)                                */
/* ------------------------------------------------------------------ */
#define ORACLE_ERR_INVALID_PACKETHEADERPROTO 18 /* include/hadoofus/objects.h:68 */
#define ORACLE_ERR_PACKET_SIZE 25
#define ORACLE_ERR_UNEXPECTED_CRC_LEN 27

struct oracle_packet { /* same layout as hdfs_crc32c_packet */
	uint64_t stream_off;
	int64_t offset_in_block, seqno;
	int32_t data_len, crc_len;
	uint32_t header_len;
	int32_t error, first_bad;
	uint32_t bad_chunks;
	uint8_t last, sync, reserved[6];
};

static int64_t rd_be(const uint8_t *p, int n) /* _hdfs_bslurp_s*, src/heapbuf.c:174-215 */
{
	uint64_t v = 0;
	for (int i = 0; i < n; i++)
		v = (v << 8) | p[i];
	if (n == 4)
		return (int32_t)(uint32_t)v;
	if (n == 1)
		return (int8_t)v;
	return (int64_t)v;
}

/* protobuf-c unpack of PacketHeaderProto (src/proto/datatransfer.proto:228-235):
 * field table {number, wire type}; returns 0 on success. */
static int pb_header(const uint8_t *p, size_t n, int64_t *off, int64_t *seq,
    uint8_t *last, int32_t *dlen, uint8_t *sync)
{
	static const int want_wt[6] = { -1, 1, 1, 0, 5, 0 };
	int have = 0;
	size_t i = 0;
	while (i < n) {
		uint64_t tag = 0;
		int k;
		if (!(p[i] & 0xf8))
			return -1;
		for (k = 0; k < 5 && i + k < n; k++) {
			tag |= (uint64_t)(p[i + k] & 0x7f) << (7 * k);
			if (!(p[i + k] & 0x80))
				break;
		}
		if (k == 5 || i + k >= n)
			return -1;
		i += k + 1;
		int wt = tag & 7;
		uint64_t fn = tag >> 3;
		const uint8_t *v = p + i;
		size_t vlen;
		if (wt == 0) {
			for (k = 0; k < 10 && i + k < n; k++)
				if (!(p[i + k] & 0x80))
					break;
			if (k == 10 || i + k >= n)
				return -1;
			vlen = k + 1;
		} else if (wt == 1) {
			vlen = 8;
		} else if (wt == 5) {
			vlen = 4;
		} else if (wt == 2) {
			uint64_t l = 0;
			for (k = 0; k < 5 && i + k < n; k++) {
				l |= (uint64_t)(p[i + k] & 0x7f) << (7 * k);
				if (!(p[i + k] & 0x80))
					break;
			}
			if (k == 5 || i + k >= n)
				return -1;
			vlen = k + 1 + l;
		} else {
			return -1;
		}
		if (vlen > n - i)
			return -1;
		if (fn >= 1 && fn <= 5) {
			if (wt != want_wt[fn])
				return -1;
			uint64_t le = 0;
			int any = 0;
			for (size_t b = 0; b < vlen; b++) {
				if (wt != 0)
					le |= (uint64_t)v[b] << (8 * b);
				else if (v[b] & 0x7f)
					any = 1;
			}
			switch (fn) {
			case 1: *off = (int64_t)le; break;
			case 2: *seq = (int64_t)le; break;
			case 3: *last = (uint8_t)any; break;
			case 4: *dlen = (int32_t)(uint32_t)le; break;
			case 5: *sync = (uint8_t)any; break;
			}
			if (fn <= 4)
				have |= 1 << fn;
		}
		i += vlen;
	}
	return have == 0x1e ? 0 : -1;
}

/* Per-chunk verify of one packet: every chunk, not only up to the first
 * mismatch (the build's per-packet report); the reference's verdict is the
 * first mismatch (src/datanode.c:2945-2960). */
static void verify_one(const uint8_t *crcs, const uint8_t *data, int32_t dlen, uint32_t cs,
    int ctype, struct oracle_packet *k)
{
	for (int64_t i = 0; i < ((int64_t)dlen + cs - 1) / cs; i++) {
		int64_t clen = dlen - i * (int64_t)cs;
		if (clen > cs)
			clen = cs;
		if (crc_of(ctype, 0, data + i * cs, (size_t)clen) != be32dec(crcs + 4 * i)) {
			if (k->first_bad < 0)
				k->first_bad = (int32_t)i;
			k->bad_chunks++;
			k->error = ORACLE_ERR_BAD_CHECKSUM;
		}
	}
}

/* One packet of the walk at stream offset pos (src/datanode.c:2345-2456):
 * header decode (v1 / v2) and the framing checks of _process_recv_packet.
 * Returns 2 (incomplete: nothing recorded), 1 (recorded and the walk ends:
 * framing error, or the empty last packet -- *total = its header bytes) or
 * 0 (a complete packet of *total wire bytes). */
static int frame_one(const uint8_t *s, uint64_t len, uint64_t pos, int proto, uint32_t cs, int ctype,
    struct oracle_packet *k, uint64_t *total)
{
	memset(k, 0, sizeof(*k));
	k->stream_off = pos;
	k->first_bad = -1;
	const uint8_t *p = s + pos;
	uint64_t rem = len - pos;
	int64_t plen, dlen;
	if (proto == 1) { /* v1: src/datanode.c:2363-2384 */
		if (rem < 25)
			return 2;
		plen = rd_be(p, 4);
		k->offset_in_block = rd_be(p + 4, 8);
		k->seqno = rd_be(p + 12, 8);
		k->last = rd_be(p + 20, 1) != 0;
		dlen = rd_be(p + 21, 4);
		k->header_len = 25;
	} else { /* v2: src/datanode.c:2387-2418 */
		if (rem < 6)
			return 2;
		plen = rd_be(p, 4);
		uint16_t hlen = (uint16_t)rd_be(p + 4, 2);
		if (rem < 6u + hlen)
			return 2;
		k->header_len = 6u + hlen;
		int32_t d32 = 0;
		if (pb_header(p + 6, hlen, &k->offset_in_block, &k->seqno, &k->last, &d32, &k->sync)) {
			k->offset_in_block = k->seqno = 0;
			k->last = k->sync = 0;
			k->error = ORACLE_ERR_INVALID_PACKETHEADERPROTO;
			return 1;
		}
		dlen = d32;
	}
	/* _process_recv_packet: src/datanode.c:2428-2446 */
	int64_t crcdlen = plen - dlen - 4;
	const int64_t onegb = 1024 * 1024 * 1024;
	k->data_len = (int32_t)dlen;
	k->crc_len = (int32_t)crcdlen;
	if (plen < 0 || dlen < 0 || dlen > onegb || plen > onegb || crcdlen < 0)
		k->error = ORACLE_ERR_PACKET_SIZE;
	else if (ctype != 0 && crcdlen != ((dlen + cs - 1) / cs) * 4)
		k->error = ORACLE_ERR_CRC_LEN;
	else if (ctype == 0 && crcdlen > 0)
		k->error = ORACLE_ERR_UNEXPECTED_CRC_LEN;
	if (k->error)
		return 1;
	if (dlen == 0) { /* src/datanode.c:2448-2456 */
		if (!k->last)
			k->error = ORACLE_ERR_PACKET_SIZE;
		*total = k->header_len;
		return 1;
	}
	*total = k->header_len + (uint64_t)crcdlen + (uint64_t)dlen;
	return rem < *total ? 2 : 0;
}

/* Returns the first packet error in stream order (0 if none); *npkts
 * records and *consumed bytes as documented for hdfs_crc32c_verify_packets. */
int oracle_verify_packets(const uint8_t *s, uint64_t len, int proto, uint32_t cs, int ctype,
    int do_verify, struct oracle_packet *out, size_t max_pkts, size_t *npkts, uint64_t *consumed)
{
	size_t n = 0;
	uint64_t pos = 0;
	*consumed = 0;
	while (n < max_pkts) {
		struct oracle_packet k;
		uint64_t total = 0;
		const int st = frame_one(s, len, pos, proto, cs, ctype, &k, &total);
		if (st == 2)
			break;
		if (st == 1) {
			if (!k.error)
				*consumed = pos + total;
			out[n++] = k;
			break;
		}
		if (do_verify && k.crc_len > 0)
			verify_one(s + pos + k.header_len, s + pos + k.header_len + k.crc_len, k.data_len, cs, ctype, &k);
		out[n++] = k;
		pos += total;
		*consumed = pos;
	}
	*npkts = n;
	for (size_t i = 0; i < n; i++)
		if (out[i].error)
			return out[i].error;
	return 0;
}

/* A client read over a packet stream: _datanode_read's loop
 * `while (remains_tot > 0) _recv_packet(...)` (src/datanode.c:1476-1481)
 * through _process_recv_packet and _recv_packet_copy_data
 * (src/datanode.c:2428-2549) for the block bytes [client_offset,
 * client_offset + read_len), into a destination of cap bytes
 * (UINT64_MAX: as large as the read).  Per packet, in the reference's order:
 *   - a framing error ends the read (:2439-2446), not consumed -- except an
 *     empty packet not flagged last (PACKET_SIZE), whose header is consumed
 *     (:2450-2455);
 *   - an empty last packet while bytes are still wanted is BAD_LASTPACKET
 *     (:2450-2456; its header is consumed, :2455);
 *   - bad CRCs end the read (:2470-2475 set bad_crcs, the loop breaks on it
 *     at :1478, the call returns BAD_CHECKSUM at :1500-1505): the packet is
 *     recorded, none of its bytes are delivered and it is not consumed;
 *   - c_begin = client_offset - offsetInBlock (0 when the packet starts
 *     later) >= dataLen is UNEXPECTED_READ_OFFSET (:2478-2486), not consumed;
 *   - the packet gives min(dataLen - c_begin, remains) bytes from c_begin on
 *     (:2488, :2507-2542); a lastPacketInBlock packet that leaves the read
 *     short is BAD_LASTPACKET after its bytes are copied (:2545-2546);
 *   - a destination that fills before the read is complete returns AGAIN
 *     (`rlen == 0 && remains_tot > 0`, :2547-2549).  A packet only partly
 *     delivered is not recorded and *consumed stays at its start: the caller
 *     re-enters with stream + consumed, client_offset + delivered and
 *     read_len - delivered (the reference re-enters with remains_pkt > 0,
 *     :2356-2361; here the packet is framed and verified again and delivers
 *     from its new c_begin).  Filled exactly at a packet's end: that packet
 *     is recorded and consumed.
 * c_begin is computed in 64 bits (the reference's int32_t differs only for
 * client_offset - offsetInBlock >= 2^31).  dst receives the delivered bytes;
 * returns the error that ended the read, ORACLE_AGAIN, or 0. */
#define ORACLE_ERR_UNEXPECTED_READ_OFFSET 28 /* include/hadoofus/objects.h:91 */
#define ORACLE_ERR_BAD_LASTPACKET 32        /* include/hadoofus/objects.h:98 */
#define ORACLE_AGAIN 1000                   /* HDFS_CRC32C_AGAIN (the reference's HDFS_AGAIN) */
int oracle_read_packets(const uint8_t *s, uint64_t len, int proto, uint32_t cs, int ctype,
    int64_t client_offset, int64_t read_len, uint64_t cap, struct oracle_packet *out, size_t max_pkts,
    size_t *npkts, uint64_t *consumed, uint8_t *dst, uint64_t *delivered)
{
	size_t n = 0;
	uint64_t pos = 0, got = 0;
	int64_t remains = read_len;
	int rc = 0;
	*consumed = 0;
	while (n < max_pkts && remains > 0) {
		struct oracle_packet k;
		uint64_t total = 0;
		const int st = frame_one(s, len, pos, proto, cs, ctype, &k, &total);
		if (st == 2)
			break;
		if (st == 1) {
			if (!k.error) { /* the empty last packet: the read wanted more */
				k.error = ORACLE_ERR_BAD_LASTPACKET;
				*consumed = pos + total;
			} else if (total) { /* an empty packet not flagged last: PACKET_SIZE with its
			                       header consumed (src/datanode.c:2451-2455) */
				*consumed = pos + total;
			}
			out[n++] = k;
			rc = k.error;
			break;
		}
		const uint8_t *crcs = s + pos + k.header_len, *data = crcs + k.crc_len;
		if (k.crc_len > 0)
			verify_one(crcs, data, k.data_len, cs, ctype, &k);
		if (k.error) { /* bad CRCs: recorded, not consumed, nothing delivered */
			out[n++] = k;
			rc = k.error;
			break;
		}
		int64_t c_begin = 0;
		if (k.offset_in_block < client_offset) {
			const uint64_t d = (uint64_t)client_offset - (uint64_t)k.offset_in_block;
			c_begin = d >= (uint64_t)k.data_len ? k.data_len : (int64_t)d;
		}
		if (c_begin >= k.data_len) {
			k.error = ORACLE_ERR_UNEXPECTED_READ_OFFSET;
			out[n++] = k;
			rc = k.error;
			break;
		}
		const int64_t c_len = k.data_len - c_begin < remains ? k.data_len - c_begin : remains;
		const uint64_t room = cap - got;
		if ((uint64_t)c_len > room) { /* the destination fills inside this packet */
			memcpy(dst + got, data + c_begin, (size_t)room);
			got += room;
			rc = ORACLE_AGAIN;
			break;
		}
		memcpy(dst + got, data + c_begin, (size_t)c_len);
		got += (uint64_t)c_len;
		remains -= c_len;
		pos += total;
		*consumed = pos;
		if (k.last && remains > 0)
			k.error = ORACLE_ERR_BAD_LASTPACKET;
		out[n++] = k;
		if (k.error) {
			rc = k.error;
			break;
		}
		if (remains > 0 && got == cap) { /* full exactly at this packet's end */
			rc = ORACLE_AGAIN;
			break;
		}
	}
	*npkts = n;
	*delivered = got;
	return rc;
}

/* ------------------------------------------------------------------ */
/* Write path: outgoing data packets                                    */
/* ------------------------------------------------------------------ */
/* Same layout as hdfs_crc32c_out_packet. */
struct oracle_out_packet {
	uint64_t hdr_off, data_off;
	int64_t offset_in_block, seqno;
	int32_t data_len;
	uint32_t hdr_len, crc_len;
	uint8_t last, reserved[3];
};

static uint8_t *bput(uint8_t *p, uint64_t v, int n) /* _hdfs_bappend_s*, src/heapbuf.c */
{
	for (int i = n - 1; i >= 0; i--)
		*p++ = (uint8_t)(v >> (8 * i));
	return p;
}

/*
 * One write of len bytes through the reference's packet loop: _send_packet
 * sizes each new packet (src/datanode.c:2590: min(remains_tot, PACKET_SIZE =
 * 64 KiB, :38); :2592-2609: an offset that is not a multiple of CHUNK_SIZE =
 * 512 first completes its chunk) and _compose_data_packet_header
 * (src/datanode.c:2781-2868) builds its header buffer: plen = dataLen +
 * 4*crclen + 4, then the v2 [hlen s16][PacketHeaderProto] or the v1 25-byte
 * header, then one BE CRC per 512-B chunk of the packet (crcinit 0 for
 * CRC32C, crc32(0, NULL, 0) = 0 for CRC32).  finish appends
 * hdfs_datanode_finish_block's empty packet (lastPacketInBlock =
 * (remains_pkt == 0)).  The PacketHeaderProto bytes restate protobuf-c's
 * packing of the fields the reference sets (:2799-2806): field 1 sfixed64,
 * 2 sfixed64, 3 bool varint, 4 sfixed32, in field order.
 * Returns 0, or -1 when hdr_cap / max_pkts are too small.
 */
int oracle_compose_packets(const uint8_t *data, uint64_t len, int64_t offset, int64_t seqno, int proto,
    int ctype, int finish, uint8_t *hdr, uint64_t hdr_cap, struct oracle_out_packet *pk, size_t max_pkts,
    size_t *npkts, uint64_t *hdr_used)
{
	const int64_t PACKET = 64 * 1024, CHUNK = 512;
	uint64_t remains_tot = len, fed = 0, used = 0;
	size_t n = 0;
	int last_done = 0;
	while (remains_tot > 0 || (finish && !last_done)) {
		int64_t remains_pkt = remains_tot < (uint64_t)PACKET ? (int64_t)remains_tot : PACKET;
		if (offset % CHUNK && remains_pkt > CHUNK - offset % CHUNK)
			remains_pkt = CHUNK - offset % CHUNK;
		int64_t crclen = ctype != ORACLE_CSUM_NULL ? (remains_pkt + CHUNK - 1) / CHUNK : 0;
		uint64_t hlen = (proto == 1 ? 25 : 4 + 2 + 25) + 4 * (uint64_t)crclen;
		if (n >= max_pkts || used + hlen > hdr_cap)
			return -1;
		uint8_t *h = hdr + used, *q = h;
		q = bput(q, (uint64_t)(uint32_t)(remains_pkt + 4 * crclen + 4), 4);
		if (proto == 1) {
			q = bput(q, (uint64_t)offset, 8);
			q = bput(q, (uint64_t)seqno, 8);
			*q++ = remains_pkt == 0;
			q = bput(q, (uint64_t)(uint32_t)remains_pkt, 4);
		} else {
			uint8_t pb[25];
			pb[0] = (1 << 3) | 1;
			for (int i = 0; i < 8; i++)
				pb[1 + i] = (uint8_t)((uint64_t)offset >> (8 * i));
			pb[9] = (2 << 3) | 1;
			for (int i = 0; i < 8; i++)
				pb[10 + i] = (uint8_t)((uint64_t)seqno >> (8 * i));
			pb[18] = (3 << 3) | 0;
			pb[19] = remains_pkt == 0;
			pb[20] = (4 << 3) | 5;
			for (int i = 0; i < 4; i++)
				pb[21 + i] = (uint8_t)((uint32_t)remains_pkt >> (8 * i));
			q = bput(q, sizeof(pb), 2);
			memcpy(q, pb, sizeof(pb));
			q += sizeof(pb);
		}
		for (int64_t i = 0; i < crclen; i++) {
			int64_t clen = remains_pkt - i * CHUNK < CHUNK ? remains_pkt - i * CHUNK : CHUNK;
			be32enc(q, crc_of(ctype, 0, data + fed + (uint64_t)(i * CHUNK), (size_t)clen));
			q += 4;
		}
		memset(&pk[n], 0, sizeof(pk[n]));
		pk[n].hdr_off = used;
		pk[n].data_off = fed;
		pk[n].offset_in_block = offset;
		pk[n].seqno = seqno;
		pk[n].data_len = (int32_t)remains_pkt;
		pk[n].hdr_len = (uint32_t)(q - h);
		pk[n].crc_len = (uint32_t)(4 * crclen);
		pk[n].last = remains_pkt == 0;
		if (remains_pkt == 0)
			last_done = 1;
		n++;
		used += (uint64_t)(q - h);
		fed += (uint64_t)remains_pkt;
		remains_tot -= (uint64_t)remains_pkt;
		offset += remains_pkt;
		seqno++;
	}
	*npkts = n;
	*hdr_used = used;
	return 0;
}

/* ------------------------------------------------------------------ */
/* Synthetic data: LE u64 words w[g] = splitmix64(seed,g) */
/* ------------------------------------------------------------------ */
static inline uint64_t splitmix64(uint64_t seed, uint64_t g)
{
	uint64_t z = seed + (g + 1) * 0x9E3779B97F4A7C15ull;
	z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
	z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
	return z ^ (z >> 31);
}

void oracle_splitmix_fill(uint64_t *out, uint64_t nwords, uint64_t seed, uint64_t g0)
{
	for (uint64_t k = 0; k < nwords; k++)
		out[k] = splitmix64(seed, g0 + k);
}

/* ------------------------------------------------------------------ */
/* CPU baseline timing (bench.py cpu_baseline leg): per-chunk CRCs over  */
/* [data, data+len) split into contiguous chunk ranges, one per thread.  */
/* fn: 0 = oracle sw, 1 = oracle hw (sse4.2 restatement), 2 = external  */
/* function pointer (the reference's own _hdfs_sse42_crc32c from _ref).  */
/* ------------------------------------------------------------------ */
typedef uint32_t (*crc_fn_t)(uint32_t, const void *, unsigned);

struct bench_arg {
	const uint8_t *data;
	uint64_t c0, c1;
	uint32_t chunk;
	int fn;
	crc_fn_t ext;
	uint32_t *out;
	uint64_t len;
};

static void *bench_worker(void *vp)
{
	struct bench_arg *a = vp;
	for (uint64_t i = a->c0; i < a->c1; i++) {
		uint64_t clen = a->len - i * a->chunk;
		if (clen > a->chunk)
			clen = a->chunk;
		const uint8_t *p = a->data + i * a->chunk;
		uint32_t c;
		if (a->fn == 2)
			c = a->ext(0, p, (unsigned)clen);
		else if (a->fn == 1)
			c = oracle_crc32c_hw(0, p, clen);
		else
			c = oracle_crc32c_sw(0, p, clen);
		a->out[i] = c;
	}
	return NULL;
}

/* Returns wall seconds. */
double oracle_bench_chunks(const void *data, uint64_t len, uint32_t chunk, int nthreads,
    int fn, void *ext_fn, uint32_t *out)
{
	uint64_t nch = (len + chunk - 1) / chunk;
	pthread_t th[256];
	struct bench_arg args[256];
	struct timespec t0, t1;
	if (nthreads < 1)
		nthreads = 1;
	if (nthreads > 256)
		nthreads = 256;
	clock_gettime(CLOCK_MONOTONIC, &t0);
	for (int t = 0; t < nthreads; t++) {
		args[t].data = data;
		args[t].c0 = nch * t / nthreads;
		args[t].c1 = nch * (t + 1) / nthreads;
		args[t].chunk = chunk;
		args[t].fn = fn;
		args[t].ext = (crc_fn_t)ext_fn;
		args[t].out = out;
		args[t].len = len;
		if (nthreads == 1)
			bench_worker(&args[t]);
		else
			pthread_create(&th[t], NULL, bench_worker, &args[t]);
	}
	if (nthreads > 1)
		for (int t = 0; t < nthreads; t++)
			pthread_join(th[t], NULL);
	clock_gettime(CLOCK_MONOTONIC, &t1);
	return (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
}
