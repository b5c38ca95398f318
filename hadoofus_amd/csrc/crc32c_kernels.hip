// gfx950 (MI355X / CDNA4) kernels for the hadoofus CRC32C chunk path.
//
// Replaces the per-chunk _hdfs_crc32c loops of src/datanode.c:2931-2963
// (read verify) and src/datanode.c:2814-2860 (write compute); arithmetic as
// in src/crc32c_sw.c / src/crc32c_sse42.c (reflected poly 0x82f63b78, pre-
// and post-inversion inside, src/crc32c.h:6-9).  Design notes: DESIGN.md.
//
// Tiled kernel, per wave and per ROUND (4 KiB = 512 B of each of 8 chunks):
//   1. four fully coalesced global_load_dwordx4 (1 KiB each); lane L of
//      load k holds 16-B piece p = 64k + L of the round;
//   2. a 4x4 in-register transpose (two DPP quad_perm exchanges) leaves each
//      lane with 64 CONTIGUOUS bytes (quad q = 16*(L&3) + (L>>2));
//   3. 16 serial slicing-by-4 steps; every table read is one v_perm_b32 (the
//      byte goes straight into the LDS address) + one conflict-free ds_read:
//      the tables are replicated 32x so lane l always hits bank l;
//   4. between rounds of a chunk > 512 B, the lane state jumps over the other
//      lanes' 448 bytes with Z_448; after a chunk's last round each lane
//      shifts its state by Z_{64(7-i)} and the 8 lanes of the chunk XOR-reduce
//      (CRC linearity, src/crc32c_sse42.c:270-319 uses the same algebra).
#include <hip/hip_runtime.h>

#include "crc32c_internal.h"

namespace hdfs_crc32c {

#define DEV __device__ __forceinline__

// Global-address-space views: segment pointers come through a struct, so
// without these casts hipcc emits flat_* accesses, which count against
// lgkmcnt too and would make every LDS-table wait also wait for the data
// prefetch.  (A cast on a templated HIP_vector_type pointer is dropped by
// the front end, hence explicit ext_vector types.)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define GAS __attribute__((address_space(1)))
DEV u32x4 gload16(const void *p) { return *(const GAS u32x4 *)(const GAS uint8_t *)p; }
DEV uint32_t gload32(const void *p) { return *(const GAS uint32_t *)(const GAS uint8_t *)p; }
DEV uint8_t gload8(const void *p) { return *(const GAS uint8_t *)p; }
DEV void gstore32(void *p, uint32_t v) { *(GAS uint32_t *)(GAS uint8_t *)p = v; }
DEV void gstore8(void *p, uint8_t v) { *(GAS uint8_t *)p = v; }

DEV uint32_t lds_at(const uint32_t *lds, uint32_t byteaddr) {
  return *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(lds) + byteaddr);
}

template <int CTRL>
DEV uint32_t dpp(uint32_t v) {
  return static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v), CTRL, 0xF, 0xF, true));
}

template <int PATTERN>
DEV uint32_t swizzle(uint32_t v) {
  return static_cast<uint32_t>(__builtin_amdgcn_ds_swizzle(static_cast<int>(v), PATTERN));
}

// One slicing-by-4 step on x = state ^ word.  Byte j of x indexes table
// t_{3-j}; v_perm_b32 drops byte j into bits [15:8] of the lane's base
// address (entry stride 256 B, lane stride 4 B, byte 2 selects the 64 KiB
// table pair), so each lookup costs one VALU op and one ds_read_b32.
DEV uint32_t slice4(const uint32_t *lds, uint32_t x, uint32_t lb0, uint32_t lb1) {
  const uint32_t a0 = __builtin_amdgcn_perm(x, lb0, 0x0C020400u);
  const uint32_t a1 = __builtin_amdgcn_perm(x, lb0, 0x0C020500u);
  const uint32_t a2 = __builtin_amdgcn_perm(x, lb1, 0x0C020600u);
  const uint32_t a3 = __builtin_amdgcn_perm(x, lb1, 0x0C020700u);
  return lds_at(lds, a0) ^ lds_at(lds, a1 + 128u) ^ lds_at(lds, a2) ^ lds_at(lds, a3 + 128u);
}

// Apply a zero-byte operator stored as 4 x 256 byte tables at word `base`.
DEV uint32_t zshift(const uint32_t *lds, uint32_t base, uint32_t x) {
  const uint32_t *t = lds + base;
  return t[x & 0xffu] ^ t[256u + ((x >> 8) & 0xffu)] ^ t[512u + ((x >> 16) & 0xffu)] ^
         t[768u + (x >> 24)];
}

// Exchange register-index bit with lane bit (0: partner = lane^1, 1: lane^2).
template <int CTRL, int STRIDE>
DEV void exchange(uint32_t (&d)[16], bool hi) {
#pragma unroll
  for (int k = 0; k < 4; k++) {
    if (k & STRIDE) continue;
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const uint32_t a = d[k * 4 + c], b = d[(k + STRIDE) * 4 + c];
      const uint32_t pa = dpp<CTRL>(a), pb = dpp<CTRL>(b);
      d[k * 4 + c] = hi ? pb : a;
      d[(k + STRIDE) * 4 + c] = hi ? b : pa;
    }
  }
}

struct TileCtx {
  const uint8_t *base;  // data of chunk 8*tile
  uint32_t *crcs;
  uint8_t *bitmap;
  uint64_t round_start;
  uint32_t seg, tile, cs, S, nch, flags, reg_init, main_tiles, nchunks;
};

DEV void load_tile(TileCtx &c, const SegDev *segs, uint32_t s, uint32_t t) {
  const SegDev &g = segs[s];
  c.seg = s;
  c.tile = t;
  c.cs = g.chunk_size;
  c.S = g.chunk_size / kRoundBytes;
  c.base = g.data + static_cast<uint64_t>(t) * kTileChunks * g.chunk_size;
  c.nchunks = g.nchunks;
  c.nch = min(kTileChunks, g.nchunks - t * kTileChunks);
  c.crcs = g.crcs;
  c.bitmap = g.bitmap;
  c.flags = g.flags;
  c.reg_init = g.reg_init;
  c.main_tiles = g.main_tiles;
  c.round_start = g.round_start;
}

DEV void load_round(uint32_t (&d)[16], const TileCtx &c, uint32_t r, uint32_t half, uint32_t l31) {
  const uint8_t *p = c.base + static_cast<uint64_t>(r) * kRoundBytes + 16u * l31;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t g = 2u * k + half;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (g < c.nch) v = gload16(p + static_cast<uint64_t>(g) * c.cs);
    d[4 * k + 0] = v.x;
    d[4 * k + 1] = v.y;
    d[4 * k + 2] = v.z;
    d[4 * k + 3] = v.w;
  }
}

template <int MODE>
__global__ __launch_bounds__(1024) void crc32c_tiles_kernel(
    const SegDev *__restrict__ segs, uint32_t nseg, uint64_t total_rounds,
    const uint32_t *__restrict__ gtab, uint32_t *__restrict__ first_bad,
    unsigned long long *__restrict__ mism) {
  __shared__ uint32_t lds[kLdsWords];

  // LDS image: word (P*16384 + e*64 + h*32 + l) = t_{3-(2P+h)}[e] for all 32 l.
  for (uint32_t idx = threadIdx.x; idx < kLdsSliceBytes / 4; idx += blockDim.x) {
    const uint32_t P = idx >> 14, e = (idx >> 6) & 255u, h = (idx >> 5) & 1u;
    lds[idx] = gtab[(3u - (2u * P + h)) * 256u + e];
  }
  for (uint32_t w = threadIdx.x; w < kTabZposWords; w += blockDim.x)
    lds[kLdsSliceBytes / 4 + w] = gtab[kTabSliceWords + w];
  __syncthreads();

  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wpb = blockDim.x >> 6;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * wpb + (threadIdx.x >> 6));
  const uint32_t nwaves = gridDim.x * wpb;
  const uint64_t r0 = total_rounds * wave / nwaves;
  const uint64_t r1 = total_rounds * (wave + 1) / nwaves;
  if (r0 >= r1) return;

  // First tile whose first round lies in [r0, r1).
  uint32_t lo = 0, hi = nseg;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (segs[mid].round_start <= r0) lo = mid; else hi = mid;
  }
  uint32_t s = lo;
  uint32_t t;
  {
    const uint32_t S = segs[s].chunk_size / kRoundBytes;
    t = static_cast<uint32_t>((r0 - segs[s].round_start + S - 1) / S);
  }
  while (s < nseg && t >= segs[s].main_tiles) { s++; t = 0; }
  if (s >= nseg) return;

  TileCtx cur;
  load_tile(cur, segs, s, t);
  if (cur.round_start + static_cast<uint64_t>(t) * cur.S >= r1) return;

  const uint32_t half = lane >> 5, l31 = lane & 31u;
  const uint32_t lb0 = l31 * 4u, lb1 = 65536u + l31 * 4u;
  const uint32_t qi = (lane >> 2) & 7u;        // 64-B position within the chunk's 512-B round
  const uint32_t qg = 2u * (lane & 3u) + half;  // chunk within the tile after the transpose
  const uint32_t zk = 7u - qi;
  const uint32_t zbase = kLdsSliceBytes / 4 + (zk ? zk - 1u : 0u) * 1024u;
  const uint32_t z448 = kLdsSliceBytes / 4 + 6u * 1024u;
  const bool b0 = lane & 1u, b1 = lane & 2u;

  uint32_t A[16], B[16];
  uint32_t r = 0;
  uint32_t expA = 0, expB = 0;
  load_round(A, cur, 0, half, l31);
  if (MODE == kModeVerify && cur.S == 1 && qi == 0 && qg < cur.nch)
    expA = gload32(cur.crcs + cur.tile * kTileChunks + qg);
  uint32_t st = 0;

  for (;;) {
    // ---- next cursor + prefetch -------------------------------------
    TileCtx nxt = cur;
    uint32_t nr;
    bool have_next;
    if (r + 1 < cur.S) {
      nr = r + 1;
      have_next = true;
    } else {
      uint32_t ns = cur.seg, nt = cur.tile + 1;
      while (ns < nseg && nt >= segs[ns].main_tiles) { ns++; nt = 0; }
      have_next = false;
      nr = 0;
      if (ns < nseg) {
        load_tile(nxt, segs, ns, nt);
        have_next = nxt.round_start + static_cast<uint64_t>(nt) * nxt.S < r1;
      }
    }
    if (have_next) {
      load_round(B, nxt, nr, half, l31);
      if (MODE == kModeVerify && nr + 1 == nxt.S && qi == 0 && qg < nxt.nch)
        expB = gload32(nxt.crcs + nxt.tile * kTileChunks + qg);
    }

    // ---- process round r of the current tile ------------------------
    exchange<0xB1, 1>(A, b0);  // quad_perm [1,0,3,2]: register bit 0 <-> lane bit 0
    exchange<0x4E, 2>(A, b1);  // quad_perm [2,3,0,1]: register bit 1 <-> lane bit 1
    if (r == 0) st = (qi == 0) ? cur.reg_init : 0u;
    else st = zshift(lds, z448, st);
#pragma unroll
    for (int w = 0; w < 16; w++) st = slice4(lds, st ^ A[w], lb0, lb1);

    if (r + 1 == cur.S) {
      uint32_t v = zk ? zshift(lds, zbase, st) : st;
      v ^= swizzle<0x101F>(v);  // xor lane 4
      v ^= swizzle<0x201F>(v);  // xor lane 8
      v ^= swizzle<0x401F>(v);  // xor lane 16
      const uint32_t out = (cur.flags & kSegRaw) ? v : ~v;
      const bool leader = (qi == 0) && (qg < cur.nch);
      const uint32_t chunk = cur.tile * kTileChunks + qg;
      if (MODE == kModeCompute) {
        if (leader) gstore32(cur.crcs + chunk, (cur.flags & kSegBigEndian) ? __builtin_bswap32(out) : out);
      } else {
        const uint32_t e = (cur.flags & kSegBigEndian) ? __builtin_bswap32(expA) : expA;
        const uint64_t m = __ballot(leader && e != out);
        if (lane == 0) {
          uint32_t byte = 0;
#pragma unroll
          for (int g = 0; g < 8; g++) byte |= static_cast<uint32_t>((m >> ((g >> 1) | ((g & 1) << 5))) & 1u) << g;
          gstore8(cur.bitmap + cur.tile, static_cast<uint8_t>(byte));
          if (byte) {
            atomicMin(&first_bad[cur.seg], cur.tile * kTileChunks + __builtin_ctz(byte));
            atomicAdd(mism, static_cast<unsigned long long>(__builtin_popcount(byte)));
          }
        }
      }
    }

    if (!have_next) break;
    cur = nxt;
    r = nr;
#pragma unroll
    for (int w = 0; w < 16; w++) A[w] = B[w];
    expA = expB;
  }
}

// Generic path: one lane per chunk, 8 lanes per tile.  Serves chunks the
// tiled kernel cannot: partial last chunks, chunk sizes that are not a
// multiple of 512, and segments whose data pointer is not 16-B aligned.
template <int MODE>
__global__ __launch_bounds__(256) void crc32c_generic_kernel(
    const SegDev *__restrict__ segs, uint32_t nseg, uint64_t total_gtiles,
    const uint32_t *__restrict__ gtab, uint32_t *__restrict__ first_bad,
    unsigned long long *__restrict__ mism) {
  __shared__ uint32_t tt[1024];
  for (uint32_t i = threadIdx.x; i < 1024u; i += blockDim.x) tt[i] = gtab[i];
  __syncthreads();
  const uint32_t *t0 = tt, *t1 = tt + 256, *t2 = tt + 512, *t3 = tt + 768;

  const uint64_t gid = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint64_t gt = gid >> 3;
  const uint32_t g = gid & 7u;
  const uint32_t lane = threadIdx.x & 63u;
  const bool active = gt < total_gtiles;

  uint32_t s = 0, tile = 0, chunk = 0, out = 0, flags = 0;
  bool valid = false;
  if (active) {
    uint32_t lo = 0, hi = nseg;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (segs[mid].gtile_start <= gt) lo = mid; else hi = mid;
    }
    s = lo;
    const SegDev &sg = segs[s];
    tile = sg.main_tiles + static_cast<uint32_t>(gt - sg.gtile_start);
    chunk = tile * kTileChunks + g;
    flags = sg.flags;
    valid = chunk < sg.nchunks;
    if (valid) {
      const uint64_t off = static_cast<uint64_t>(chunk) * sg.chunk_size;
      const uint8_t *p = sg.data + off;
      uint64_t n = min(static_cast<uint64_t>(sg.chunk_size), sg.len - off);
      uint32_t c = sg.reg_init;
      while (n && (reinterpret_cast<uintptr_t>(p) & 3u)) {
        c = t0[(c ^ gload8(p++)) & 0xffu] ^ (c >> 8);
        n--;
      }
      while (n >= 4) {
        const uint32_t x = c ^ gload32(p);
        c = t3[x & 0xffu] ^ t2[(x >> 8) & 0xffu] ^ t1[(x >> 16) & 0xffu] ^ t0[x >> 24];
        p += 4;
        n -= 4;
      }
      while (n) {
        c = t0[(c ^ gload8(p++)) & 0xffu] ^ (c >> 8);
        n--;
      }
      out = (flags & kSegRaw) ? c : ~c;
      if (MODE == kModeCompute)
        gstore32(sg.crcs + chunk, (flags & kSegBigEndian) ? __builtin_bswap32(out) : out);
    }
  }
  if (MODE == kModeVerify) {
    bool bad = false;
    if (valid) {
      uint32_t e = gload32(segs[s].crcs + chunk);
      if (flags & kSegBigEndian) e = __builtin_bswap32(e);
      bad = e != out;
    }
    const uint64_t m = __ballot(bad);
    if (active && g == 0) {
      const uint32_t byte = static_cast<uint32_t>((m >> (lane & 56u)) & 0xffu);
      gstore8(segs[s].bitmap + tile, static_cast<uint8_t>(byte));
      if (byte) {
        atomicMin(&first_bad[s], tile * kTileChunks + __builtin_ctz(byte));
        atomicAdd(mism, static_cast<unsigned long long>(__builtin_popcount(byte)));
      }
    }
  }
}

// Stream combine: acc ^= Z_{len-end_i}(raw_i) for all i, plus Z_len(reg0).
// raws are raw registers of consecutive cs-byte pieces of one stream.
DEV uint32_t zapply(const uint32_t *__restrict__ pow2, uint32_t x, uint64_t d) {
  for (uint32_t b = 0; d; b++, d >>= 1) {
    if (d & 1u) {
      const uint32_t *t = pow2 + b * 1024u;
      x = t[x & 0xffu] ^ t[256u + ((x >> 8) & 0xffu)] ^ t[512u + ((x >> 16) & 0xffu)] ^
          t[768u + (x >> 24)];
    }
  }
  return x;
}

__global__ __launch_bounds__(256) void crc32c_combine_kernel(
    const uint32_t *__restrict__ raws, uint64_t nraw, uint32_t cs, uint64_t len,
    const uint32_t *__restrict__ pow2, uint32_t reg0, uint32_t *__restrict__ acc) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  uint32_t v = 0;
  if (i < nraw) {
    const uint64_t end = min((i + 1) * static_cast<uint64_t>(cs), len);
    v = zapply(pow2, raws[i], len - end);
  }
  if (i == 0) v ^= zapply(pow2, reg0, len);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v ^= __shfl_xor(v, off);
  if ((threadIdx.x & 63u) == 0 && v) atomicXor(acc, v);
}

// splitmix64 synthetic blocks: w[k] = splitmix64(seed, g0 + k).
DEV uint64_t splitmix64(uint64_t seed, uint64_t g) {
  uint64_t z = seed + (g + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void splitmix_fill_kernel(uint64_t *__restrict__ out,
                                                             uint64_t nwords, uint64_t seed,
                                                             uint64_t g0) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x * 2;
  for (uint64_t k = (static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x) * 2; k < nwords;
       k += stride) {
    if (k + 1 < nwords) {
      ulonglong2 v;
      v.x = splitmix64(seed, g0 + k);
      v.y = splitmix64(seed, g0 + k + 1);
      *reinterpret_cast<ulonglong2 *>(out + k) = v;
    } else {
      out[k] = splitmix64(seed, g0 + k);
    }
  }
}

// Deterministic corruption: for global chunk index
// i with i % modulus == 0, flip bit (i * bitmul) mod (8 * chunk_len).
__global__ __launch_bounds__(256) void corrupt_kernel(uint8_t *__restrict__ data, uint64_t len,
                                                       uint32_t cs, uint64_t chunk0,
                                                       uint64_t modulus, uint64_t bitmul) {
  const uint64_t nch = (len + cs - 1) / cs;
  const uint64_t first = (chunk0 + modulus - 1) / modulus * modulus;
  const uint64_t i = first + (static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x) * modulus;
  if (i >= chunk0 + nch) return;
  const uint64_t local = i - chunk0;
  const uint64_t clen = min(static_cast<uint64_t>(cs), len - local * cs);
  const uint64_t bit = (i * bitmul) % (8 * clen);
  data[local * cs + bit / 8] ^= static_cast<uint8_t>(1u << (bit % 8));
}

// ---------------------------------------------------------------------------
// Host-side launchers (used by crc32c_engine.cpp).
// ---------------------------------------------------------------------------
hipError_t launch_tiles(int mode, int grid, const SegDev *segs, uint32_t nseg, uint64_t total_rounds,
                        const uint32_t *gtab, uint32_t *first_bad, unsigned long long *mism,
                        hipStream_t stream) {
  if (mode == kModeVerify)
    hipLaunchKernelGGL(crc32c_tiles_kernel<kModeVerify>, dim3(grid), dim3(1024), 0, stream, segs,
                       nseg, total_rounds, gtab, first_bad, mism);
  else
    hipLaunchKernelGGL(crc32c_tiles_kernel<kModeCompute>, dim3(grid), dim3(1024), 0, stream, segs,
                       nseg, total_rounds, gtab, first_bad, mism);
  return hipGetLastError();
}

hipError_t launch_generic(int mode, const SegDev *segs, uint32_t nseg, uint64_t total_gtiles,
                          const uint32_t *gtab, uint32_t *first_bad, unsigned long long *mism,
                          hipStream_t stream) {
  const uint64_t threads = total_gtiles * kTileChunks;
  const uint32_t blocks = static_cast<uint32_t>((threads + 255) / 256);
  if (mode == kModeVerify)
    hipLaunchKernelGGL(crc32c_generic_kernel<kModeVerify>, dim3(blocks), dim3(256), 0, stream, segs,
                       nseg, total_gtiles, gtab, first_bad, mism);
  else
    hipLaunchKernelGGL(crc32c_generic_kernel<kModeCompute>, dim3(blocks), dim3(256), 0, stream,
                       segs, nseg, total_gtiles, gtab, first_bad, mism);
  return hipGetLastError();
}

hipError_t launch_combine(const uint32_t *raws, uint64_t nraw, uint32_t cs, uint64_t len,
                          const uint32_t *pow2, uint32_t reg0, uint32_t *acc, hipStream_t stream) {
  const uint64_t n = nraw ? nraw : 1;
  const uint32_t blocks = static_cast<uint32_t>((n + 255) / 256);
  hipLaunchKernelGGL(crc32c_combine_kernel, dim3(blocks), dim3(256), 0, stream, raws, nraw, cs, len,
                     pow2, reg0, acc);
  return hipGetLastError();
}

hipError_t launch_fill(uint64_t *out, uint64_t nwords, uint64_t seed, uint64_t g0, hipStream_t stream) {
  uint64_t want = (nwords / 2 + 255) / 256;
  const uint32_t blocks = static_cast<uint32_t>(want < 1 ? 1 : (want > 65536 ? 65536 : want));
  hipLaunchKernelGGL(splitmix_fill_kernel, dim3(blocks), dim3(256), 0, stream, out, nwords, seed, g0);
  return hipGetLastError();
}

hipError_t launch_corrupt(uint8_t *data, uint64_t len, uint32_t cs, uint64_t chunk0, uint64_t modulus,
                          uint64_t bitmul, hipStream_t stream) {
  const uint64_t nch = (len + cs - 1) / cs;
  const uint64_t cand = nch / modulus + 2;
  const uint32_t blocks = static_cast<uint32_t>((cand + 255) / 256);
  hipLaunchKernelGGL(corrupt_kernel, dim3(blocks), dim3(256), 0, stream, data, len, cs, chunk0,
                     modulus, bitmul);
  return hipGetLastError();
}

}  // namespace hdfs_crc32c
