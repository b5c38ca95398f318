// Host-side CRC32C table construction for the MI355X engine.
//
// The arithmetic follows the reference's definitions:
//   - reflected Castagnoli polynomial 0x82f63b78   (src/crc32c_sw.c:63)
//   - byte table / slicing tables                  (src/crc32c_sw.c:72-94)
//   - GF(2) "append n zero bytes" operator         (src/crc32c_sse42.c:99-200)
// but the table SHAPES are the ones the gfx950 kernels need (see DESIGN.md
// "LDS layout"): slicing-by-4 tables t0..t3 and per-distance byte tables
// Z_n[m][e] = Z_n(e << 8m) for the lane-combine and the stream combine.
#pragma once
#include <cstdint>
#include <cstring>

namespace hdfs_crc32c {

constexpr uint32_t kPoly = 0x82f63b78u;      // CRC-32C (Castagnoli), src/crc32c_sw.c:63
constexpr uint32_t kPolyZlib = 0xedb88320u;  // CRC-32 (IEEE, zlib crc32()), HDFS_CSUM_CRC32

// t[k][e]: register contribution of byte e followed by k zero bytes,
// i.e. the classic slicing table t_k.
inline void make_slicing4(uint32_t t[4][256], uint32_t poly = kPoly) {
  for (uint32_t e = 0; e < 256; e++) {
    uint32_t c = e;
    for (int b = 0; b < 8; b++) c = (c >> 1) ^ (poly & (0u - (c & 1u)));
    t[0][e] = c;
  }
  for (uint32_t e = 0; e < 256; e++) {
    uint32_t c = t[0][e];
    for (int k = 1; k < 4; k++) {
      c = t[0][c & 0xff] ^ (c >> 8);
      t[k][e] = c;
    }
  }
}

// 32x32 GF(2) matrices stored as column images: m[i] = M(e_i).
struct Gf2 {
  uint32_t col[32];
  uint32_t apply(uint32_t v) const {
    uint32_t s = 0;
    for (int i = 0; v; i++, v >>= 1)
      if (v & 1) s ^= col[i];
    return s;
  }
  Gf2 compose(const Gf2 &inner) const {  // this o inner
    Gf2 r;
    for (int i = 0; i < 32; i++) r.col[i] = apply(inner.col[i]);
    return r;
  }
  static Gf2 identity() {
    Gf2 r;
    for (int i = 0; i < 32; i++) r.col[i] = 1u << i;
    return r;
  }
  static Gf2 one_zero_byte(uint32_t poly = kPoly) {
    Gf2 bit;  // one zero bit: c -> (c >> 1) ^ (c & 1 ? poly : 0)
    bit.col[0] = poly;
    for (int i = 1; i < 32; i++) bit.col[i] = 1u << (i - 1);
    Gf2 r = bit;
    for (int k = 0; k < 3; k++) r = r.compose(r);
    return r;
  }
};

// Operator for n zero bytes (square-and-multiply).
inline Gf2 zeros_op(uint64_t n, uint32_t poly = kPoly) {
  Gf2 acc = Gf2::identity(), p = Gf2::one_zero_byte(poly);
  while (n) {
    if (n & 1) acc = p.compose(acc);
    n >>= 1;
    if (n) p = p.compose(p);
  }
  return acc;
}

// Mailbox multipliers (kTabKxWords per type): x^(8n) mod P is the image of
// the polynomial 1 (bit 31) under the n-zero-byte operator.
inline void make_kx(uint32_t *out, uint32_t poly = kPoly) {
  const Gf2 z64 = zeros_op(64, poly), z1 = zeros_op(1, poly);
  out[0] = out[1024] = 0x80000000u;
  for (int m = 1; m < 1024; m++) out[m] = z64.apply(out[m - 1]);
  for (int r = 1; r < 64; r++) out[1024 + r] = z1.apply(out[1024 + r - 1]);
}

// Byte tables for an operator: out[m*256 + e] = op(e << 8m).
inline void zeros_byte_tables(const Gf2 &op, uint32_t *out) {
  for (int m = 0; m < 4; m++)
    for (uint32_t e = 0; e < 256; e++) out[m * 256 + e] = op.apply(e << (8 * m));
}

}  // namespace hdfs_crc32c
