// Diagnostic build only (-DHDFS_CRC32C_DIAG, libhadoofus_crc32c_diag.so):
// the tiled kernel's epilogue hooks (ReleaseEP in crc32c_kernels.hip) with
// the store-policy experiments of tools/exp_knobs.py and the load-only twin
// of the verify kernel.  The policy comes from the launch's tune word
// (hdfs_crc32c_set_store_policy); 0 is the product's behaviour at every site.
// Included by crc32c_kernels.hip after ReleaseEP; never part of the release
// library.
#pragma once
#ifndef HDFS_CRC32C_DIAG
#error "crc32c_diag_ep.h is part of the diagnostic build only"
#endif

namespace hdfs_crc32c {

struct DiagEP : ReleaseEP {
  DEV static uint32_t policy(uint32_t tune) { return rfl(tune); }
  // 21 / 23: the expected CRCs loaded nontemporal
  DEV static uint32_t exp_load(uint32_t pol, __amdgpu_buffer_rsrc_t re, uint32_t off) {
    if (pol == 21u || pol == 23u) return __builtin_amdgcn_raw_buffer_load_b32(re, off, 0, 2);
    return ReleaseEP::exp_load(pol, re, off);
  }
  // 2: result records dropped (compute CRCs, verify bitmap bytes)
  DEV static bool drop(uint32_t pol) { return pol == 2u; }
  // 20: the gather kernel with its slot protocol skipped and every CRC store
  // dropped (what the protocol itself costs)
  // 26 / 27 / 28: as 20, plus a workgroup barrier every 1 / 2 / 4 iterations
  // of the round loop (3 / 6 / 12 rounds) -- what a barrier-flushed gather (no
  // slot protocol; CRCs staged in LDS and written behind a barrier) would pay
  // for its barriers alone.  Never combined with the slot protocol: a wave
  // waiting for a slot while the slot's finisher waits at the barrier is a
  // deadlock (the protocol's spin limit traps it, as a first probe found).
  // A wave that has left the loop no longer counts for s_barrier.
  DEV static bool gather_off(uint32_t pol) { return pol == 20u || (pol >= 26u && pol <= 28u); }
  DEV static void loop_hook(uint32_t pol, uint32_t it) {
    if (pol >= 26u && pol <= 28u && (it & ((1u << (pol - 26u)) - 1u)) == 0u) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    }
  }
  DEV static const uint32_t *group_base(uint32_t pol, const uint32_t *b, const SegHot &sh, uint32_t gt) {
    if (pol == 14u) {
      // the group's 256 B land at a scattered group position of the segment
      // (q -> 37 q mod 2^k): same bytes and lines, written in no spatial
      // order (the CRCs end up permuted)
      const uint32_t ng = sh.main_tiles >> 3, q = ((gt & ~7u) - static_cast<uint32_t>(sh.mtile_start)) >> 3;
      if (ng && (ng & (ng - 1u)) == 0u) return sh.crcs + ((q * 37u) & (ng - 1u)) * 64u;
    }
    // 15: every group store lands in the segment's first 256 KiB (an
    // L2-resident window: the stores' CU / L2 cost without the HBM write-back)
    if (pol == 15u) return sh.crcs + ((((gt & ~7u) - static_cast<uint32_t>(sh.mtile_start)) * kTileChunks) & 65535u);
    return b;
  }
  // columns: 15 as for the gather (every run's 128 B inside the segment's
  // first 256 KiB of CRCs: an L2-resident window)
  DEV static const uint32_t *col_base(uint32_t pol, const uint32_t *b, const SegHot &sh, uint32_t tile) {
    return pol == 15u ? sh.crcs + ((tile * kTileChunks) & 65535u) : b;
  }
  DEV static void group_store(uint32_t pol, uint32_t v, __amdgpu_buffer_rsrc_t r, uint32_t off) {
    if (pol == 5u) __builtin_amdgcn_raw_buffer_store_b32(v, r, off, 0, 16);        // sc1
    else if (pol == 6u) __builtin_amdgcn_raw_buffer_store_b32(v, r, off, 0, 17);   // sc0 sc1
    else if (pol == 7u) __builtin_amdgcn_raw_buffer_store_b32(v, r, off, 0, 18);   // nt sc1
    else if (pol == 8u) __builtin_amdgcn_raw_buffer_store_b32(v, r, off, 0, 1);    // sc0
    else if (pol == 11u) __builtin_amdgcn_raw_buffer_store_b32(v, r, off, 0, 0);   // default
    else ReleaseEP::group_store(pol, v, r, off);
  }
  // compute, one store per tile: true if a policy wrote the tile another way
  static constexpr bool kAltTileStores = true;
  template <class Tab>
  DEV static bool tile_store_alt(uint32_t pol, const SegHot &sh, Tab segs, const Cursor &c, bool keep, uint32_t nch,
                                 bool leader, const LaneConst &L, uint32_t val) {
    if (pol == 3u) {
      // 128-B full-line write per tile (crcs must hold 16 B per chunk)
      const __amdgpu_buffer_rsrc_t r4 = __builtin_amdgcn_make_buffer_rsrc(
          segs[c.seg].crcs + c.tile * kTileChunks * 4, 0, keep ? static_cast<int>(nch * 16u) : 0, 0x00020000);
      u32x4 v4 = {val, val, val, val};
      __builtin_amdgcn_raw_buffer_store_b128(v4, r4, leader ? L.qg * 16u : 0x80000000u, 0, 0);
      return true;
    }
    if (pol == 12u || pol == 13u) {
      // only the last tile of each 8-tile group stores -- 12: one 256-B store
      // over the whole group's CRCs (64 lanes x 4 B, sc1; the values are not
      // the group's CRCs), 13: its own 32 B as usual
      const bool grp = keep && (c.tile & 7u) == 7u;
      const bool full = pol == 12u;
      const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc(
          reinterpret_cast<uint32_t *>(
              rfl64(reinterpret_cast<uint64_t>(sh.crcs + (full ? (c.tile & ~7u) : c.tile) * kTileChunks))),
          0, static_cast<int>(rfl(grp ? (full ? 256u : nch * 4u) : 0u)), 0x00020000);
      __builtin_amdgcn_raw_buffer_store_b32(val, rg, full ? L.lane * 4u : (leader ? L.qg * 4u : 0x80000000u), 0, 16);
      return true;
    }
    if (pol == 9u) {
      // every tile's 32 B lands in a 256 KiB window (L2-resident writes)
      const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
          reinterpret_cast<uint32_t *>(rfl64(reinterpret_cast<uint64_t>(sh.crcs))), 0,
          static_cast<int>(rfl(keep ? 262144u : 0u)), 0x00020000);
      const uint32_t wo = ((c.tile * 32u) & 262143u) + L.qg * 4u;
      __builtin_amdgcn_raw_buffer_store_b32(val, rw, leader ? wo : 0x80000000u, 0, 0);
      return true;
    }
    return false;
  }
  DEV static void tile_store(uint32_t pol, uint32_t v, __amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t qg) {
    if (pol == 10u && qg != 0) off = 0x80000000u;  // 4 B per tile
    if (pol == 1u) __builtin_amdgcn_raw_buffer_store_b32(v, r, off, 0, 2);         // nt
    else if (pol == 5u) __builtin_amdgcn_raw_buffer_store_b32(v, r, off, 0, 16);   // sc1
    else if (pol == 6u) __builtin_amdgcn_raw_buffer_store_b32(v, r, off, 0, 17);   // sc0 sc1
    else if (pol == 7u) __builtin_amdgcn_raw_buffer_store_b32(v, r, off, 0, 18);   // nt sc1
    else if (pol == 8u) __builtin_amdgcn_raw_buffer_store_b32(v, r, off, 0, 1);    // sc0
    else if (pol == 11u) __builtin_amdgcn_raw_buffer_store_b32(v, r, off, 0, 0);   // default
    else ReleaseEP::tile_store(pol, v, r, off, qg);
  }
  DEV static void bitmap_store(uint32_t pol, uint8_t b, __amdgpu_buffer_rsrc_t r, uint32_t off) {
    if (pol == 22u || pol == 23u) __builtin_amdgcn_raw_buffer_store_b8(b, r, off, 0, 2);   // nt
    else if (pol == 24u) __builtin_amdgcn_raw_buffer_store_b8(b, r, off, 0, 16);          // sc1
    else if (pol == 25u) __builtin_amdgcn_raw_buffer_store_b8(b, r, off, 0, 17);          // sc0 sc1
    else ReleaseEP::bitmap_store(pol, b, r, off);
  }
  DEV static void copy_store(uint32_t pol, u32x4 v, __amdgpu_buffer_rsrc_t r, uint32_t off) {
    if (pol == 16u) __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 2);         // nt
    else if (pol == 17u) __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 16);   // sc1
    else if (pol == 19u) __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 0);    // default
    else ReleaseEP::copy_store(pol, v, r, off);
  }
  // Load-only twin of verify (store policy 4): the same loads and the same
  // bitmap store op with its record dropped, no CRC arithmetic.  The loaded
  // words fold into st, and an impossible condition on st keeps them live
  // (without it the compiler deletes the unused loads).
  template <int S, class Tab>
  DEV static void load_only_round(const uint32_t (&d)[S][16], const uint32_t (&exp)[S], const Cursor (&c)[S], Tab segs,
                                  uint32_t (&st)[S], unsigned long long *__restrict__ mism) {
#pragma unroll
    for (int s = 0; s < S; s++) {
      uint32_t v = exp[s];
#pragma unroll
      for (int w = 0; w < 16; w++) v ^= d[s][w];
      st[s] ^= v;
      const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
          reinterpret_cast<uint8_t *>(rfl64(reinterpret_cast<uint64_t>(segs[c[s].seg].bitmap + c[s].tile))), 0, 0,
          0x00020000);
      __builtin_amdgcn_raw_buffer_store_b8(static_cast<uint8_t>(st[s]), rb, 0u, 0, 0);
      if (st[s] == 0x9E3779B9u && c[s].r == 0xFFFFFFFFu) atomicAdd(mism, 1ull);
    }
  }
};

}  // namespace hdfs_crc32c
