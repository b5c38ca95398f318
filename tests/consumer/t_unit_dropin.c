/*
 * Stand-alone consumer of the drop-in header: the shape of the reference's
 * CRC32C unit test (tests/t_unit.c:146-217), linked against
 * libhadoofus_crc32c.so instead of the reference's crc32c*.o.
 *
 * Reads known-answer vectors "len crc hex" (one per line) from argv[1] and
 * checks every drop-in symbol, plus chaining across a split point.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "crc32c.h"

static int hexval(int c)
{
	return c <= '9' ? c - '0' : (c | 0x20) - 'a' + 10;
}

int main(int argc, char **argv)
{
	FILE *f;
	char line[8192];
	int failures = 0, cases = 0;

	if (argc != 2 || !(f = fopen(argv[1], "r"))) {
		fprintf(stderr, "usage: %s kats.txt\n", argv[0]);
		return 2;
	}
	while (fgets(line, sizeof(line), f)) {
		unsigned len, i;
		unsigned long exp;
		char *hex = NULL;
		unsigned char buf[4096];

		if (sscanf(line, "%u %lx", &len, &exp) != 2 || len > sizeof(buf))
			continue;
		hex = strrchr(line, ' ') + 1;
		for (i = 0; i < len; i++)
			buf[i] = (unsigned char)(hexval(hex[2 * i]) << 4 | hexval(hex[2 * i + 1]));
		uint32_t a = _hdfs_crc32c(0, buf, len);
		uint32_t b = _hdfs_sse42_crc32c(0, buf, len);
		uint32_t c = _hdfs_sw_crc32c(0, buf, len);
		uint32_t d = _hdfs_crc32c(_hdfs_crc32c(0, buf, len / 3), buf + len / 3, len - len / 3);
		if (a != exp || b != exp || c != exp || d != exp) {
			fprintf(stderr, "len %u: want %08lx got %08x %08x %08x chained %08x\n",
			    len, exp, a, b, c, d);
			failures++;
		}
		cases++;
	}
	fclose(f);
	printf("%d cases, %d failures\n", cases, failures);
	return failures || !cases;
}
