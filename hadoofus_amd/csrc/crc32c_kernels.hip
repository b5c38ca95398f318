// gfx950 (MI355X / CDNA4) kernels for the hadoofus CRC32C chunk path.
//
// Replaces the per-chunk _hdfs_crc32c loops of src/datanode.c:2931-2963
// (read verify) and src/datanode.c:2814-2860 (write compute); arithmetic as
// in src/crc32c_sw.c / src/crc32c_sse42.c (reflected poly 0x82f63b78, pre-
// and post-inversion inside, src/crc32c.h:6-9).  Design notes: DESIGN.md.
//
// Tiled kernel, per wave and per ROUND (4 KiB = 512 B of each of 8 chunks):
//   1. four fully coalesced global_load_dwordx4 (1 KiB each); lane L of
//      load k holds 16-B piece p = 64k + 4*(L&15) + (L>>4) of the round
//      (a lane permutation inside each contiguous 1 KiB);
//   2. an in-register transpose of two v_permlane16_swap / v_permlane32_swap
//      stages (register bit <-> lane bit 4, then 5) leaves lane L with the
//      64 CONTIGUOUS bytes of quad L (chunk L>>3, position L&7);
//   3. 16 serial slicing-by-4 steps; every table read is one v_perm_b32 (the
//      byte goes straight into the LDS address) + one conflict-free ds_read:
//      the tables are replicated 32x so lane l always hits bank l;
//   4. between rounds of a chunk > 512 B, the lane state jumps over the other
//      lanes' 448 bytes with Z_448; after a chunk's last round each lane
//      shifts its state by Z_{64(7-i)} and the 8 lanes of the chunk XOR-reduce
//      (CRC linearity, src/crc32c_sse42.c:270-319 uses the same algebra).
#include <hip/hip_runtime.h>

#include "crc32c_frame.h"
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
DEV u32x4 gload16_nt(const void *p) {
  return __builtin_nontemporal_load((const GAS u32x4 *)(const GAS uint8_t *)p);
}
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
DEV uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }

// The step also folds in the NEXT data word: returns t0^t1^t2^t3^next with
// two v_bitop3_b32 (3-input XOR), so a step is 4 v_perm + 2 VALU + 4 ds_read.
DEV uint32_t slice4(const uint32_t *lds, uint32_t x, uint32_t next, uint32_t lb0, uint32_t lb1) {
  const uint32_t a0 = __builtin_amdgcn_perm(x, lb0, 0x0C020400u);
  const uint32_t a1 = __builtin_amdgcn_perm(x, lb0, 0x0C020500u);
  const uint32_t a2 = __builtin_amdgcn_perm(x, lb1, 0x0C020600u);
  const uint32_t a3 = __builtin_amdgcn_perm(x, lb1, 0x0C020700u);
  return xor3(xor3(lds_at(lds, a0), lds_at(lds, a1 + 128u), lds_at(lds, a2)), lds_at(lds, a3 + 128u), next);
}

// Apply a zero-byte operator stored as 4 x 256 byte tables at word `base`.
DEV uint32_t zshift(const uint32_t *lds, uint32_t base, uint32_t x) {
  const uint32_t *t = lds + base;
  return t[x & 0xffu] ^ t[256u + ((x >> 8) & 0xffu)] ^ t[512u + ((x >> 16) & 0xffu)] ^
         t[768u + (x >> 24)];
}

// In-register 4x4 transpose of a round: register bit 0 <-> lane bit 4
// (v_permlane16_swap: odd 16-lane rows of one register trade places with
// even rows of the other), then register bit 1 <-> lane bit 5
// (v_permlane32_swap: upper 32 lanes of one with lower 32 of the other).
// One instruction moves two registers: 16 per round for 16 dwords.
DEV void transpose(uint32_t (&d)[16]) {
#pragma unroll
  for (int c = 0; c < 4; c++) {
#pragma unroll
    for (int k = 0; k < 4; k += 2) {
      const auto r = __builtin_amdgcn_permlane16_swap(d[k * 4 + c], d[(k + 1) * 4 + c], false, false);
      d[k * 4 + c] = r[0];
      d[(k + 1) * 4 + c] = r[1];
    }
  }
#pragma unroll
  for (int c = 0; c < 4; c++) {
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const auto r = __builtin_amdgcn_permlane32_swap(d[k * 4 + c], d[(k + 2) * 4 + c], false, false);
      d[k * 4 + c] = r[0];
      d[(k + 2) * 4 + c] = r[1];
    }
  }
}

DEV uint32_t rfl(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
DEV uint64_t rfl64(uint64_t x) {
  return (static_cast<uint64_t>(rfl(static_cast<uint32_t>(x >> 32))) << 32) | rfl(static_cast<uint32_t>(x));
}

// Device checks (diagnostic build only): an invariant a kernel relies on
// for an address it is about to touch -- a record slot inside the pass, a
// packet's bytes inside the stream, a copy-out inside the destination.  A
// violation is counted in g_dchk with the kernel and source line of the
// first one, and the access it guards is skipped, so a broken invariant is
// reported by the call that broke it (diag_device_checks(), read by the
// engine after each device-stream call) instead of surfacing as an illegal
// address in whatever runs next.  Release build: DCHK(c, k) is `true` and c
// is never evaluated.
#ifdef HDFS_CRC32C_DIAG
__device__ uint32_t g_dchk[4];  // kernel of the first violation, its line, violations
DEV bool dchk(bool ok, uint32_t kid, uint32_t line) {
  if (!ok && atomicAdd(&g_dchk[2], 1u) == 0u) {
    g_dchk[0] = kid;
    g_dchk[1] = line;
  }
  return ok;
}
#define DCHK(c, kid) dchk((c), (kid), __LINE__)
#else
#define DCHK(c, kid) true
#endif

// The segment table is read through the constant address space: loads with
// a wave-uniform index then always lower to s_load (scalar cache, lgkmcnt),
// never to vector loads that would enter the vmcnt ordering the prefetch.
#define CAS __attribute__((address_space(4)))
typedef const CAS SegDev *SegP;

// The first 48 bytes of a SegDev (the fields read every round), fetched as
// one aggregate so it lowers to two wide scalar loads instead of one load
// per field.
struct SegHot {
  const uint8_t *data;
  uint32_t *crcs;
  uint8_t *bitmap;
  uint64_t mtile_start;
  uint32_t chunk_size, flags, nchunks, main_tiles;
};
static_assert(sizeof(SegHot) == 48, "SegHot is the head of SegDev");
DEV SegHot seg_hot(SegP segs, uint32_t s) {
  const CAS SegHot *p = reinterpret_cast<const CAS SegHot *>(&segs[s]);
  return SegHot{p->data, p->crcs, p->bitmap, p->mtile_start, p->chunk_size, p->flags, p->nchunks, p->main_tiles};
}

// A closed-form segment table (spec_verify_kernel): segment k is packet k of
// a run of equal packets at crc0 + k * stride -- its CRCs there, its data
// 4 * nch bytes later, its bitmap at bm0 + k * T -- with every field a
// function of k and packet 0's header, so no table is built or read.  The
// tiled kernel's helpers take either this or a SegP (`segs[s].field`).
// Copy-out: packet k delivers dataLen bytes (packet 0: dataLen - cb0, the
// client read window's c_begin), placed after the avail of the packets
// before it, never past copy_cap (frame::read_avail / read_place in closed
// form).  The parameters sit in HBM (each workgroup writes its own copy
// after decoding packet 0) and are read, like a SegDev, with scalar loads
// through the constant address space: carried in SGPRs across the work
// loop they pushed the kernel past the SGPR budget and into spills.
// BATCH: the table of a batch of equal runs (spec_verify_kernel<0, 1>); the
// single-run kernels keep the plain closed form in their hot loop.
// Per-run completion of a coalesced batch (SpecArgs::early): one more of
// run r's count -- a workgroup done with its tiles of r, or a header group of
// r checked.  What it depends on (the run's mismatch count, its header mark)
// are agent-scope atomics the contributor has waited for (vmcnt) before it
// counts: relaxed atomics and no fences here -- an agent-scope release /
// acquire is an L2 write-back and invalidate, once per workgroup and run.
// The contribution that reaches the run's target publishes the run's
// verdict to the host as ONE 16-B store {seq, mism, bad} (no fence).
DEV void spec_run_contribute(SpecCtl *ctl, uint8_t *hdone, uint32_t seq, uint32_t target, uint32_t r) {
  const uint32_t n = __hip_atomic_fetch_add(&ctl->run_done[r], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (n + 1u != target) return;
  const uint32_t mism = __hip_atomic_load(&ctl->run_mism[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t bad = (__hip_atomic_load(&ctl->run_bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> r) & 1u;
  *(volatile GAS u32x4 *)(GAS uint8_t *)(hdone + sizeof(SpecRunDone) * r) = u32x4{seq, mism, bad, 0u};
}

// LDS words of the per-run completion (BATCH): [0, 16) tiles of run r this
// workgroup has verified, [16, 32) tiles of run r it owns (kEarlyOff: r has
// pool tiles, not published), [32, 48) run r's target (workgroups + header
// groups), [48] the owned tiles' sum, [49] per-run completion on
constexpr uint32_t kEarlyWords = 50, kEarlyOff = 0xFFFFFFFFu;

template <bool BATCH>
struct SpecTabT {
  const CAS SpecTabData *p;
  uint32_t *e;  // BATCH: the per-run completion words (LDS, kEarlyWords)
  // per-run completion on for this wave: the owned tiles the prologue
  // restated from the schedule add up to the wave's own static tickets
  DEV uint32_t early_ok(uint32_t nk) const {
    if constexpr (BATCH) return rfl(e[49] != 0u && e[48] == nk ? 1u : 0u);
    return 0u;
  }
  // the tile of packet k verified (its last round; byte = its mismatch bits):
  // counted for its run, and the workgroup's last tile of the run contributes
  DEV void tile_done(uint32_t k, uint32_t byte, uint32_t lane) const {
    if constexpr (BATCH) {
      const uint32_t r = rfl(static_cast<uint32_t>(__umul64hi(static_cast<uint64_t>(k), p->um)));
      SpecCtl *const ctl = p->ctl;
      if (byte) {  // rare: the run's mismatches, acknowledged before the tile counts
        if (lane == 0)
          __hip_atomic_fetch_add(&ctl->run_mism[r], static_cast<uint32_t>(__builtin_popcount(byte)), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
      }
      uint32_t old = 0;
      if (lane == 0) old = __hip_atomic_fetch_add(&e[r], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      old = __builtin_amdgcn_readlane(old, 0);
      if (old + 1u == rfl(e[16u + r]) && lane == 0) spec_run_contribute(ctl, p->hdone, p->seq, e[32u + r], r);
    }
  }
  DEV SegDev operator[](uint32_t k) const {
    SegDev d;
    SpecTabData q;
    q.crc0 = p->crc0;
    q.bm0 = p->bm0;
    q.copy_base = p->copy_base;
    q.stride = p->stride;
    q.copy_cap = p->copy_cap;
    q.nch = p->nch;
    q.cs = p->cs;
    q.cb0 = p->cb0;
    const uint32_t T = (q.nch + kTileChunks - 1u) / kTileChunks, dlen = q.nch * q.cs;
    const uint8_t *c;
    if constexpr (BATCH) {  // a batch of equal runs: packet k is packet k - r * per of run r = k / per (uniform)
      const uint32_t r = static_cast<uint32_t>(__umul64hi(static_cast<uint64_t>(k), p->um));
      c = p->crc0r[r] + static_cast<uint64_t>(k - r * p->per) * q.stride;
    } else {
      c = q.crc0 + static_cast<uint64_t>(k) * q.stride;
    }
    d.data = c + 4u * q.nch;
    d.crcs = reinterpret_cast<uint32_t *>(const_cast<uint8_t *>(c));
    d.bitmap = q.bm0 + static_cast<uint64_t>(k) * T;
    d.mtile_start = static_cast<uint64_t>(k) * T;
    d.chunk_size = q.cs;
    d.flags = kSegBigEndian;  // wire CRCs; the table set is the launch's
    d.nchunks = q.nch;
    d.main_tiles = T;
    d.reg_init = 0xFFFFFFFFu;
    d.gen_tiles = 0u;
    d.len = dlen;
    d.round_start = static_cast<uint64_t>(k) * T * (q.cs / kRoundBytes);
    d.gtile_start = 0u;
    const uint32_t w0 = k ? 0u : q.cb0;
    const uint64_t before = k ? static_cast<uint64_t>(k) * dlen - q.cb0 : 0u;
    uint64_t at = 0;
    uint32_t clen = 0;
    frame::read_place(before, dlen - w0, q.copy_cap, at, clen);
    d.copy_dst = q.copy_base && clen ? q.copy_base + at : nullptr;
    d.copy_w0 = w0;
    d.copy_w1 = w0 + clen;
    return d;
  }
};
using SpecTab = SpecTabT<false>;
template <class Tab>
struct TabEarly {
  static constexpr bool value = false;
};
template <>
struct TabEarly<SpecTabT<true>> {
  static constexpr bool value = true;
};
template <bool BATCH>
DEV SegHot seg_hot(const SpecTabT<BATCH> &t, uint32_t k) {
  const SegDev d = t[k];
  return SegHot{d.data, d.crcs, d.bitmap, d.mtile_start, d.chunk_size, d.flags, d.nchunks, d.main_tiles};
}

// Per-stream copy of the current segment's hot fields (and reg_init), kept
// in SGPRs across rounds: issue / process / finish / advance of a round
// re-read the table only when the cursor's segment changed (a wave-uniform
// compare), instead of s_load + s_waitcnt lgkmcnt(0) several times a round.
struct SegCache {
  uint32_t seg;
  uint32_t reg_init;
  SegHot h;
};
template <class Tab>
DEV const SegCache &hot(SegCache &k, Tab segs, uint32_t s) {
  if (s != k.seg) {
    k.h = seg_hot(segs, s);
    k.reg_init = segs[s].reg_init;
    k.seg = s;
  }
  return k;
}

// Wave-uniform position of one round: (segment, tile, round).
struct Cursor {
  uint32_t seg, tile, r;
  bool valid;
  uint32_t grp = 0;  // compute gather (RUN 2): workgroup-local group ordinal = ticket >> 3
};

// Work schedule of one wave.
//  ORDER 0 (static): the wave owns the tiles whose first round lies in its
//    slice [r0, r1) of the global round sequence.
//  ORDER 1 (workgroup-dynamic): the workgroup owns the tiles whose first
//    round lies in its slice; its 16 waves take them one at a time from an
//    LDS counter (ds_add_rtn_u32).  Waves of one SIMD run at different speeds
//    (age-ordered issue arbitration: measured 18.9 / 20.4 / 22.5 / 24.6 ms for
//    wave slots 0-3 / 4-7 / 8-11 / 12-15 under a static split), so a static
//    split leaves the oldest waves idle for the last ~15 % of the kernel.
//    The LDS atomic counts in lgkmcnt, never in the vmcnt that orders the
//    data prefetch.
//  ORDER 2 (two-phase): as ORDER 1 over the first kPhase1Num/kPhase1Den of
//    the rounds; the remaining tiles form a global pool of kUnit-tile units
//    that workgroups claim with one global atomic each once their own slice
//    is done (published to the workgroup's other waves through an LDS slot).
//    The pool absorbs the cross-workgroup / cross-XCD speed spread; its
//    atomics only happen at the end, off the hot loop.
//  ORDER 3 (interleaved two-phase): as ORDER 2, but the static phase deals
//    groups of 2^gshift consecutive tiles round-robin over the workgroups
//    (workgroup b takes groups b, b+G, b+2G, ...), so at any moment the
//    whole grid reads one contiguous window of memory instead of G separate
//    streams; the read probes of crc32c_probes.hip measured this shape
//    faster on MI355X HBM.  Groups of >= 4 tiles own whole 128-B lines of
//    expected / computed CRCs (8 chunks x 4 B per tile), so no two XCDs'
//    L2s fetch or write the same CRC line (default 8 tiles per group).
//  ORDER 4 (runs, compute mode): as ORDER 3 with 8-tile groups, but a ticket
//    is a whole group and ONE wave processes its 8 tiles in a row, collecting
//    the 64 CRCs in one register (lane 8j + q = tile j, chunk q) and writing
//    them as one 256-B store (two whole lines) instead of eight 32-B stores
//    from eight waves: each store that leaves the CU costs, per instruction
//    as well as per byte (tools/exp_knobs.py, profiles/r02/).  Needs every
//    segment's main tiles to be a multiple of 8 (the host checks).  Unit size (runtime,
//    a power of two in [16, 256]) targets >= 4 units per workgroup; launches
//    with < 32 rounds per wave skip the pool (one unit per workgroup would
//    make the tail, not shorten it).
//  ORDER 7 (columns, compute mode): ORDER 4's dealing with 4-tile tickets
//    (32 chunks, one 128-B line of CRCs), but a round is a COLUMN of the
//    run: 128 B of each of its 32 chunks instead of 512 B of each of 8.
//    Each 1 KiB load instruction still reads 8 whole 128-B lines; after the
//    transpose lane L holds 64 B of chunk L>>1 (half L&1), the lane pair
//    combines every round (Z_64 on the even lane, one DPP XOR) and carries
//    the chunk's register into the next column, so after the last column the
//    even lanes hold the run's 32 CRCs and write them as ONE 128-B store.  No
//    cross-wave LDS protocol (the gather's cost) and no per-tile stores.
//    Diagnostic build only: measured 1-2 % below the gather in one process
//    (the column reads cost ~1.6 % with stores dropped, the 128-B stores
//    5-6.5 % even inside an L2-sized window; profiles/r03/exp_columns*.json).
constexpr uint32_t kUnitMaxShift = 8, kUnitMinShift = 4;
constexpr uint32_t kColBytes = 128;  // ORDER 7: bytes of each chunk per round
constexpr uint32_t kColShift = 2;    // ORDER 7: log2 tiles per ticket (32 chunks)
constexpr uint32_t kSlots = 8;  // LDS slots for published units
// Compute gather (schedule 3, RUN 2): the CRCs of an 8-tile group, finished
// by up to eight waves of the workgroup, collect in one of kGatherSlots LDS
// slots (the 4 KiB the tables leave free) and the wave finishing the group
// writes them as one 256-B store.  Slot s serves groups s, s + kGatherSlots,
// ... in order; its owner word holds (group << 4) | tiles counted.
#ifndef HDFS_GATHER_SLOTS  // a power of two; fewer only in A/B builds (-DHDFS_GATHER_SLOTS=n)
#define HDFS_GATHER_SLOTS 8
#endif
static_assert((HDFS_GATHER_SLOTS & (HDFS_GATHER_SLOTS - 1)) == 0, "gather slots: a power of two");
constexpr uint32_t kGatherSlots = HDFS_GATHER_SLOTS, kGatherWords = kGatherSlots * 65;
#ifndef HDFS_PHASE1_NUM  // A/B builds only (-DHDFS_PHASE1_NUM=n)
#define HDFS_PHASE1_NUM 23
#endif
constexpr uint64_t kPhase1Num = HDFS_PHASE1_NUM, kPhase1Den = 25;  // 92 % static

struct Sched {
  uint64_t r1;       // ORDER 0: end of the wave's round slice
  uint64_t gfirst;   // ORDER 1/2: first global tile of the workgroup's slice (3: blockIdx)
  uint32_t nk;       // ORDER 1/2: tiles of the workgroup's slice
  uint32_t *ctr;     // ORDER 1/2: LDS ticket counter
  uint32_t lane;
  uint64_t p2first;  // ORDER 2: first global tile of the pool
  uint64_t ntiles;   // ORDER 2: total tiles
  uint32_t *gctr;    // ORDER 2: global unit counter (zeroed per launch)
  uint64_t *slots;   // ORDER 2: LDS [kSlots] of (unit + 1) << 32 | global unit
  uint32_t ushift;   // ORDER 2/3: log2 tiles per pool unit
  uint32_t gstride;  // ORDER 3: group stride of the static phase (gridDim)
  uint32_t gshift;   // ORDER 3: log2 tiles per group
  // Uniform tables (ut != 0): segment s holds global main tiles [s*ut, s*ut +
  // main_tiles_s) with main_tiles_s == ut for every segment but the last (the
  // packets of a block transfer).  A tile's segment is then g / ut -- a shift
  // (ush) or a multiply-high by um = floor(2^64 / ut) + 1, exact for g < 2^32
  // -- instead of a binary search of the table.
  uint32_t ut, ush;
  uint64_t um;
};

DEV Cursor ulocate(const Sched &w, uint64_t g) {
  const uint32_t s = w.ush != 0xFFFFFFFFu ? static_cast<uint32_t>(g >> w.ush) : static_cast<uint32_t>(__umul64hi(g, w.um));
  return Cursor{rfl(s), rfl(static_cast<uint32_t>(g - uint64_t(s) * w.ut)), 0u, true};
}

DEV uint32_t grab(const Sched &w) {
  uint32_t k = 0;
  if (w.lane == 0) k = atomicAdd(w.ctr, 1u);
  return rfl(k);
}

// Ticket -> global tile.  Tickets below nk are the workgroup's own slice;
// later tickets walk the pool unit by unit.
template <int ORDER>
DEV bool ticket_tile(const Sched &w, uint32_t t, uint64_t &g) {
  if (t < w.nk) {
    if (ORDER == 4 || ORDER == 7)
      g = (w.gfirst + uint64_t(t) * w.gstride) << w.gshift;
    else if (ORDER == 3)
      g = ((w.gfirst + uint64_t(t >> w.gshift) * w.gstride) << w.gshift) + (t & ((1u << w.gshift) - 1u));
    else
      g = w.gfirst + t;
    return true;
  }
  if (ORDER < 2) return false;
  // ORDER 4 / 7: a ticket is 2^gshift tiles, a pool unit 2^(ushift - gshift) tickets
  const uint32_t tsh = (ORDER == 4 || ORDER == 7) ? w.gshift : 0u;
  const uint32_t j = t - w.nk, u = j >> (w.ushift - tsh), o = (j & ((1u << (w.ushift - tsh)) - 1u)) << tsh,
                 s = u % kSlots;
  if (o == 0) {  // first ticket of local unit u: claim a pool unit and publish it
    uint32_t gu = 0;
    if (w.lane == 0) gu = atomicAdd(w.gctr, 1u);
    gu = rfl(gu);
    if (w.lane == 0)
      __hip_atomic_store(&w.slots[s], (uint64_t(u + 1) << 32) | gu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  uint64_t v;
  for (;;) {  // the publisher is a running wave that already holds ticket u << ushift
    v = __hip_atomic_load(&w.slots[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (rfl(static_cast<uint32_t>(v >> 32)) == u + 1) break;
    __builtin_amdgcn_s_sleep(2);
  }
  g = w.p2first + (uint64_t(rfl(static_cast<uint32_t>(v))) << w.ushift) + o;
  return g < w.ntiles;
}

constexpr uint64_t kWalkTiles = 64;  // forward hops of up to this many tiles walk the table

// Global tile g -> (segment, tile), walking forward from segment s.
template <class Tab>
DEV Cursor locate(Tab segs, uint32_t s, uint64_t g) {
  while (g >= segs[s].mtile_start + segs[s].main_tiles) s++;
  return Cursor{rfl(s), rfl(static_cast<uint32_t>(g - segs[s].mtile_start)), 0u, true};
}

// Global tile g -> cursor, from the current cursor c (whose segment's hot
// fields are sh).  Pool tiles may lie behind the slice or far ahead of it (a
// table of thousands of packet-sized segments: a forward walk from the slice
// to the pool cost 8x the whole kernel, tools/exp_packet_tables.py);
// interleaved tiles jump G ahead.  Short hops walk, long ones search.
template <int ORDER, class Tab>
DEV Cursor find_tile(const Cursor c, const SegHot &sh, Tab segs, uint32_t nseg, const Sched &w, uint64_t g) {
  const uint64_t end = sh.mtile_start + sh.main_tiles;
  if (w.ut && (g < sh.mtile_start || g >= end)) return ulocate(w, g);
  if (g < sh.mtile_start || g >= end + (ORDER >= 3 ? 0u : kWalkTiles)) {
    uint32_t lo = 0, hi = nseg;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (segs[mid].mtile_start <= g) lo = mid; else hi = mid;
    }
    return locate(segs, lo, g);
  }
  if (g < end)  // same segment (the common case): from the cached fields, no table read
    return Cursor{c.seg, rfl(static_cast<uint32_t>(g - sh.mtile_start)), 0u, true};
  return locate(segs, c.seg, g);
}

// Next round owned by this wave.  An exhausted cursor keeps its last
// position (so speculative loads stay in bounds) with valid = false.
template <int ORDER, class Tab>
DEV Cursor advance(Cursor c, Tab segs, uint32_t nseg, const Sched &w, SegCache &kc) {
  if (!c.valid) return c;
  const SegHot &sh = hot(kc, segs, c.seg).h;
  // ORDER 7: a cursor is a whole 4-tile run, one round per 128-B column
  if (c.r + 1 < (ORDER == 7 ? sh.chunk_size / kColBytes : sh.chunk_size / kRoundBytes)) {
    c.r++;
    return c;
  }
  if (ORDER == 4 && ((c.tile + 1u) & ((1u << w.gshift) - 1u)) != 0u) {  // the run's next tile (whole groups)
    c.tile++;
    c.r = 0;
    return c;
  }
  if (ORDER != 0) {
    uint64_t g;
    const uint32_t tk = grab(w);
    if (!ticket_tile<ORDER>(w, tk, g)) {
      c.valid = false;
      return c;
    }
    Cursor n = find_tile<ORDER>(c, sh, segs, nseg, w, g);
    n.grp = tk >> 3;
    return n;
  }
  uint32_t s = c.seg, t = c.tile + 1;
  while (s < nseg && t >= segs[s].main_tiles) {
    t = 0;
    s++;
  }
  if (s >= nseg || segs[s].round_start + uint64_t(t) * (segs[s].chunk_size / kRoundBytes) >= w.r1) {
    c.valid = false;
    return c;
  }
  return Cursor{rfl(s), rfl(t), 0u, true};
}

// Global index of the first tile whose first round is >= r.
template <class Tab>
DEV uint64_t tile_at_round(Tab segs, uint32_t nseg, uint64_t r, uint64_t total_tiles) {
  uint32_t lo = 0, hi = nseg;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (segs[mid].round_start <= r) lo = mid; else hi = mid;
  }
  const uint32_t S = segs[lo].chunk_size / kRoundBytes;
  const uint64_t g = segs[lo].mtile_start + (r - segs[lo].round_start + S - 1) / S;
  return g < total_tiles ? g : total_tiles;
}

struct LaneConst {
  uint32_t lane, hsel, loff, lb0, lb1, qi, qg, zk, zbase, z448, z64;
  uint64_t ntiles;   // RUN 2: main tiles of the launch
  uint32_t rmask;    // RUN 1: tiles per run - 1
  uint32_t *gslot;   // RUN 2: LDS [kGatherSlots] owner words, then [kGatherSlots][64] CRC words
  // the diagnostic build's store-policy experiment (EP::policy); 0 in the
  // release build, where no hook reads it
  uint32_t store_policy;
  uint32_t early;    // a coalesced batch's per-run completion (TabEarly tables)
};

// Store / load sites of the tiled kernel's epilogue.  The product kernels
// use ReleaseEP: one instruction per site with the cache bits the
// measurements chose, nothing else.  The diagnostic build
// (-DHDFS_CRC32C_DIAG) instantiates the same kernels with DiagEP
// (crc32c_diag_ep.h), which puts the store-policy experiments of
// tools/exp_knobs.py behind these hooks -- the product functions below carry
// no diagnostic branch of their own.
struct ReleaseEP {
  DEV static uint32_t policy(uint32_t) { return 0u; }
  // verify: the expected CRC of the lane's chunk (default policy)
  DEV static uint32_t exp_load(uint32_t, __amdgpu_buffer_rsrc_t re, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b32(re, off, 0, 0);
  }
  // result records dropped (compute CRCs, verify bitmap bytes)
  DEV static bool drop(uint32_t) { return false; }
  // compute gather: the slot protocol skipped, its stores dropped
  DEV static bool gather_off(uint32_t) { return false; }
  // once per iteration of the round loop (diagnostic barrier probes)
  DEV static void loop_hook(uint32_t, uint32_t) {}
  // compute gather: where a whole group's 256 B go
  DEV static const uint32_t *group_base(uint32_t, const uint32_t *b, const SegHot &, uint32_t) { return b; }
  // columns (ORDER 7): where a run's 128 B go
  DEV static const uint32_t *col_base(uint32_t, const uint32_t *b, const SegHot &, uint32_t) { return b; }
  // compute gather: nt (pipelined gather kernel, one process: sc1 6 797,
  // nt 6 835, nt sc1 6 827, sc0 sc1 6 771 GB/s alg,
  // profiles/r02/s6/exp_gather_store_policy.json)
  DEV static void group_store(uint32_t, uint32_t v, __amdgpu_buffer_rsrc_t r, uint32_t off) {
    __builtin_amdgcn_raw_buffer_store_b32(v, r, off, 0, 2);
  }
  // compute, one store per tile: no other way of writing a tile
  static constexpr bool kAltTileStores = false;
  // compute, one store per tile: sc1.  Compute mode loses ~13 % to its CRC
  // stores, per written-back line rather than per byte (4 B per tile costs
  // as much as 32 B; an L2-resident window recovers half); sc1 stores
  // measured +1.7 % compute, verify unchanged (tools/exp_knobs.py,
  // profiles/r02/).
  DEV static void tile_store(uint32_t, uint32_t v, __amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t) {
    __builtin_amdgcn_raw_buffer_store_b32(v, r, off, 0, 16);
  }
  // verify: the tile's bitmap byte (default policy; nt / sc1 cost 6 %,
  // profiles/r02/s8/exp_verify_cache_policies.json)
  DEV static void bitmap_store(uint32_t, uint8_t b, __amdgpu_buffer_rsrc_t r, uint32_t off) {
    __builtin_amdgcn_raw_buffer_store_b8(b, r, off, 0, 0);
  }
  // verify + copy-out: nt sc1 (streaming; 1 GiB device run, one process:
  // default 2 083, sc1 2 172, nt 2 220, nt sc1 2 250 GiB/s,
  // profiles/r02/s6/exp_copy_store_policy.json)
  DEV static void copy_store(uint32_t, u32x4 v, __amdgpu_buffer_rsrc_t r, uint32_t off) {
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 18);
  }
};
#ifdef HDFS_CRC32C_DIAG
}  // namespace hdfs_crc32c
#include "crc32c_diag_ep.h"
namespace hdfs_crc32c {
using EP = DiagEP;
#else
using EP = ReleaseEP;
#endif

// Issue the loads of one round: four fully coalesced 1 KiB dwordx4 loads
// (lanes with bit 3 clear / set cover sub-chunks 2k / 2k+1, in the permuted
// lane order the permlane transpose expects) plus, in verify mode, the
// expected CRC of the lane's chunk.  Unconditional (addresses clamped into
// the tile) so the vector-memory count is static and the compiler's
// s_waitcnt vmcnt(N) for the round being processed stays counted.
// Per-lane load offsets for the buffer-load form of issue(): chunk g's
// 16-B piece of the lane sits at (2k + hsel) * cs + loff from the round's
// base; cached per chunk size (wave-uniform compare, no VALU in the common
// case of one chunk size).
struct LaneOff {
  uint32_t cs;
  uint32_t v[4];
  uint32_t t;  // UNA: lanes 0..7 -> offset of the dword after chunk lane's 512-B round part
};

// UNA (byte-unaligned segment data, e.g. packet payloads inside a wire
// image): with a = data & 3 the four 1 KiB loads start a bytes early (4-B
// aligned: the fast path of the memory pipeline).  After the transpose lane
// L holds the 64 bytes of its quad starting a bytes early; the a bytes it
// lacks at the end are the first dword of the next quad's window (lane L+1,
// one DPP row shift) -- or, for the last quad of a chunk's round, the dword
// just after the round part, which ONE extra load per round fetches for
// all 8 chunks (lanes 0..7; ds_bpermute hands it to lanes 8j+7); 16
// v_alignbyte_b32 then shift the lane's 17 dwords into place.  Every extra
// byte read lies in a dword that also holds data of the segment, so no read
// leaves the data's pages.  The shift rides with the round (rounds in
// flight may belong to different segments).
template <int MODE, int NT, int BUF, int UNA, int COL = 0, class P = EP, class Tab = SegP>
DEV void issue(uint32_t (&d)[16], uint32_t &exp, uint32_t &tl, uint32_t &sh_a, const Cursor c, Tab segs,
               uint32_t hsel, uint32_t loff, uint32_t qg, uint32_t lane, LaneOff &lo, SegCache &kc,
               uint32_t pol = 0u) {
  static_assert(!COL || (BUF && !UNA && MODE == kModeCompute), "columns: compute, buffer loads, aligned data");
  const SegHot &sh = hot(kc, segs, c.seg).h;
  const uint32_t cs = sh.chunk_size;
  const uint32_t a = UNA ? static_cast<uint32_t>(reinterpret_cast<uintptr_t>(sh.data)) & 3u : 0u;
  if (UNA) sh_a = a;
  if constexpr (BUF) {
    // Buffer loads: the round's base in SGPRs, per-lane offsets from the
    // cache, and the descriptor's range (the valid bytes of this round's
    // chunks) returns zeros for chunks past a partial tile's end instead of
    // clamping addresses.
    // COL (ORDER 7): the round is column r of a 32-chunk run -- bytes
    // [128 r, 128 r + 128) of each chunk; quad Q = 16k + (L & 15) of load k
    // is half Q & 1 of chunk Q >> 1, so load k reads chunks 8k .. 8k + 7,
    // one whole 128-B line each
    constexpr uint32_t kRb = COL ? kColBytes : kRoundBytes;
    const uint32_t nch = min(COL ? kTileChunks << kColShift : kTileChunks, sh.nchunks - c.tile * kTileChunks);
    const uint8_t *base = sh.data + static_cast<uint64_t>(c.tile) * kTileChunks * cs +
                          static_cast<uint64_t>(c.r) * kRb - a;
    if (lo.cs != cs) {
      lo.cs = cs;
#pragma unroll
      for (int k = 0; k < 4; k++)
        lo.v[k] = COL ? (8u * k + ((lane >> 1) & 7u)) * cs + (lane & 1u) * 64u + 16u * (lane >> 4)
                      : (2u * k + hsel) * cs + loff;
      if (UNA) lo.t = lane < kTileChunks ? lane * cs + kRoundBytes : 0x80000000u;
    }
    // UNA: the range ends with the dword holding the last data byte
    const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t *>(base), 0, static_cast<int>((nch - 1u) * cs + kRb + (a ? 4u : 0u)), 0x00020000);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const u32x4 v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rd, lo.v[k], 0, NT ? 2 : 0));
      d[4 * k + 0] = v.x;
      d[4 * k + 1] = v.y;
      d[4 * k + 2] = v.z;
      d[4 * k + 3] = v.w;
    }
    if (UNA) tl = __builtin_amdgcn_raw_buffer_load_b32(rd, lo.t, 0, NT ? 2 : 0);
    if (MODE != kModeCompute) {
      const __amdgpu_buffer_rsrc_t re = __builtin_amdgcn_make_buffer_rsrc(
          sh.crcs + c.tile * kTileChunks, 0, static_cast<int>(nch * 4u), 0x00020000);
      exp = P::exp_load(pol, re, qg * 4u);
    }
  } else {
    const uint32_t last = min(kTileChunks, segs[c.seg].nchunks - c.tile * kTileChunks) - 1u;
    const uint8_t *rb = segs[c.seg].data + static_cast<uint64_t>(c.tile) * kTileChunks * cs +
                        static_cast<uint64_t>(c.r) * kRoundBytes - a;
    const uint8_t *p = rb + loff;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t g = min(2u * k + hsel, last);
      const u32x4 v = NT ? gload16_nt(p + static_cast<uint64_t>(g) * cs) : gload16(p + static_cast<uint64_t>(g) * cs);
      d[4 * k + 0] = v.x;
      d[4 * k + 1] = v.y;
      d[4 * k + 2] = v.z;
      d[4 * k + 3] = v.w;
    }
    // a == 0: an in-bounds dummy (the dword after the data end may lie past its page)
    if (UNA) tl = gload32(rb + static_cast<uint64_t>(min(lane, last)) * cs + (a ? kRoundBytes : kRoundBytes - 4u));
    if (MODE != kModeCompute) {
      // buffer load: expected CRCs of a packet sit at any byte offset of the wire image
      const __amdgpu_buffer_rsrc_t re = __builtin_amdgcn_make_buffer_rsrc(
          segs[c.seg].crcs + c.tile * kTileChunks, 0, static_cast<int>((last + 1u) * 4u), 0x00020000);
      exp = __builtin_amdgcn_raw_buffer_load_b32(re, qg * 4u, 0, 0);
    }
  }
}


// Finish one round of one stream after its 16 slicing steps: on a tile's
// last round, combine the 8 lanes of each chunk and write / compare.  The
// finalize issues no vector-memory op (LDS and swizzles only).  The result
// store runs every round, by every lane, through a bounds-checked buffer
// descriptor: its size is 0 unless this is a valid last round, and lanes
// that must not write get an out-of-range offset, so the hardware drops
// them.  Every round therefore issues exactly the same vector-memory ops
// (4 loads, [1 expected-CRC load], 1 store) and the compiler's vmcnt waits
// stay exact.
// Per-stream epilogue state carried across rounds: RUN 1's run CRCs, and
// RUN 3's pending tile (the lazy gather, below).
struct Gst {
  uint32_t acc;                              // RUN 1: lane 8j + q = tile j, chunk q
  uint32_t chk, old, dat;                    // RUN 3 (VGPRs): slot check, returned count, finisher's word
  uint32_t pslot, pgrp, pexpect, pelig, fin;  // RUN 3 (uniform): the pending tile (pslot ~0: none)
  const uint32_t *pbase;                     // RUN 3: the pending eligible group's CRC destination
};
constexpr uint32_t kNoSlot = 0xFFFFFFFFu;

// RUN 3, before a round's slicing steps: the count the stream's previous
// tile added to its group's slot (its add was issued a round ago) says
// whether this wave finished that group -- then its word of the group's CRCs
// is read now -- and, on a tile's last round, the owner word of the tile's
// slot is loaded.  Both LDS reads complete under the 64 table reads of the
// slicing: nothing is waited on.
template <class Tab>
DEV void lazy_pre(Gst &g, const Cursor &c, Tab segs, SegCache &kc, const LaneConst &L) {
  g.fin = 0u;
  if (g.pslot != kNoSlot && (rfl(g.old) & 15u) + 1u == g.pexpect) {
    g.fin = 1u;
    if (g.pelig) g.dat = L.gslot[kGatherSlots + g.pslot * 64u + L.lane];
  }
  const SegHot &sh = hot(kc, segs, c.seg).h;
  if (c.valid && c.r + 1 == sh.chunk_size / kRoundBytes)
    g.chk = __hip_atomic_load(L.gslot + (c.grp & (kGatherSlots - 1u)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// RUN 3: the pending group's finisher stores the group's CRCs (256 B) and
// hands the slot on to group + kGatherSlots.  Its word of the group was read
// before the release is written, and a wave's LDS operations execute in
// order, so the next group's writers cannot overwrite it first.
template <class P>
DEV void lazy_flush(Gst &g, const SegHot &sh, const LaneConst &L) {
  uint32_t range = 0u;
  const uint32_t *base = sh.crcs;
  if (g.pslot != kNoSlot && g.fin) {
    if (g.pelig) {
      range = P::drop(L.store_policy) ? 0u : 256u;
      base = g.pbase;
    }
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    if (L.lane == 0)
      __hip_atomic_store(L.gslot + g.pslot, (g.pgrp + kGatherSlots) << 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  g.pslot = kNoSlot;
  const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<uint32_t *>(rfl64(reinterpret_cast<uint64_t>(base))), 0, static_cast<int>(rfl(range)),
      0x00020000);
  P::group_store(L.store_policy, g.dat, rg, L.lane * 4u);
}

template <int MODE, int RUN, class P = EP, class Tab = SegP>
DEV void finish(const uint32_t *lds, uint32_t exp, const Cursor c, Tab segs, uint32_t st, const LaneConst &L,
                uint32_t *__restrict__ first_bad, unsigned long long *__restrict__ mism, SegCache &kc,
                Gst &gs) {
  const SegHot &sh = hot(kc, segs, c.seg).h;
  if constexpr (RUN == 4) {
    // ORDER 7 (columns): st is each chunk's register through this column
    // (process() combined the lane pair); after the last column the even
    // lanes hold the run's 32 CRCs -> one 128-B store (dropped otherwise)
    static_assert(MODE == kModeCompute, "columns: compute mode");
    const bool lastc = c.valid && (c.r + 1 == sh.chunk_size / kColBytes);
    const uint32_t nch = min(kTileChunks << kColShift, sh.nchunks - c.tile * kTileChunks);
    const uint32_t out = (sh.flags & kSegRaw) ? st : ~st;
    const uint32_t val = (sh.flags & kSegBigEndian) ? __builtin_bswap32(out) : out;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<uint32_t *>(
            rfl64(reinterpret_cast<uint64_t>(P::col_base(L.store_policy, sh.crcs + c.tile * kTileChunks, sh, c.tile)))),
        0, static_cast<int>(rfl(lastc && !P::drop(L.store_policy) ? nch * 4u : 0u)), 0x00020000);
    P::group_store(L.store_policy, val, rs, (L.lane & 1u) ? 0x80000000u : (L.lane >> 1) * 4u);
    return;
  }
  const bool last = c.valid && (c.r + 1 == sh.chunk_size / kRoundBytes);
  const uint32_t flags = sh.flags;
  const uint32_t nch = min(kTileChunks, sh.nchunks - c.tile * kTileChunks);
  const bool leader = last && (L.qi == 0) && (L.qg < nch);
  const uint32_t pol = L.store_policy;
  uint32_t out = 0, byte = 0;
  if (last) {
    uint32_t v = L.zk ? zshift(lds, L.zbase, st) : st;
    // XOR of the chunk's 8 lanes with DPP (VALU, which has headroom) rather
    // than ds_swizzle (LDS instruction slots, which the table reads fill):
    // quad_perm [1,0,3,2] and [2,3,0,1] give every lane its quad's XOR,
    // row_half_mirror (lane i <-> 7 - i within 8) swaps the two quads' XORs
    v ^= dpp<0xB1>(v);
    v ^= dpp<0x4E>(v);
    v ^= dpp<0x141>(v);
    out = (flags & kSegRaw) ? v : ~v;
    if (MODE == kModeVerify) {
      const uint32_t e = (flags & kSegBigEndian) ? __builtin_bswap32(exp) : exp;
      // leaders are lanes 8g, so the ballot has bits only at multiples of 8;
      // one multiply gathers bit 8g into bit 56+g (no carries: each byte of
      // the product collects at most one term per bit)
      const uint64_t m = __ballot(leader && e != out);
      byte = static_cast<uint32_t>((m * 0x0102040810204080ull) >> 56);
    }
  }
  byte = rfl(byte);
  if (MODE == kModeCompute) {
    const bool keep = last && !P::drop(pol);
    const uint32_t val = (flags & kSegBigEndian) ? __builtin_bswap32(out) : out;
    if constexpr (RUN == 2) {
      // schedule 3 gather: an eligible group's tiles (8 full tiles of one
      // segment) park their CRCs in the group's LDS slot and the wave that
      // finishes the group stores all 64; other groups' tiles store their own
      // 32 B but still count in the slot, so it passes on to the next group
      uint32_t sval = val, soff = leader ? L.qg * 4u : 0x80000000u, range = keep ? nch * 4u : 0u;
      const uint32_t *sbase = sh.crcs + c.tile * kTileChunks;
      const bool off = P::gather_off(pol);
      if (off) range = 0u;
      if (last && !off) {
        // eligible: the group's 8 tiles are whole tiles of this segment.  A
        // segment whose main tiles start and end on group boundaries (every
        // block of a transfer) has only such groups, bar a partial last
        // tile: decided in 32-bit scalar ops, the 64-bit tile arithmetic only
        // for the other groups (they count their tiles up to the launch end)
        const bool whole = ((static_cast<uint32_t>(sh.mtile_start) | sh.main_tiles) & 7u) == 0u;
        bool elig = whole && (uint64_t(c.tile | 7u) + 1u) * kTileChunks <= sh.nchunks;
        uint32_t expect = 8u;
        if (!elig) {
          const uint64_t gs = (sh.mtile_start + c.tile) & ~7ull;
          expect = static_cast<uint32_t>(min<uint64_t>(8u, L.ntiles - gs));
          elig = expect == 8u && gs >= sh.mtile_start && gs + 8u <= sh.mtile_start + sh.main_tiles &&
                 (gs + 8u - sh.mtile_start) * kTileChunks <= sh.nchunks;
        }
        const uint32_t gt = static_cast<uint32_t>(sh.mtile_start) + c.tile;  // low bits of the global tile
        const uint32_t s = c.grp & (kGatherSlots - 1u);
        uint32_t *own = L.gslot + s;
        uint32_t *dat = L.gslot + kGatherSlots + s * 64u;
        // the slot's previous group (grp - kGatherSlots) holds only older
        // tickets, which never wait on newer ones: the wait ends.
        // Ordering: the slot's words and owner live in LDS, so the fences are
        // LDS-only ("local": s_waitcnt lgkmcnt(0)).  Plain acquire / release
        // atomics also order global memory, i.e. wait vmcnt(0) -- that drained
        // the wave's whole round pipeline (2 rounds of loads in flight) once
        // per tile.
        for (uint32_t spin = 0;; spin++) {
          const uint32_t o = rfl(__hip_atomic_load(own, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
          if ((o >> 4) == c.grp) break;
          // never expected: fail loudly rather than hang.  s_trap as an
          // ordinary instruction: __builtin_trap() is noreturn, and the
          // unreachable edge it adds made the CFG structurizer route a path
          // back to the loop head on which the waitcnt pass saw the next
          // round's loads as the newest -- s_waitcnt vmcnt(0) at every loop
          // head, i.e. no loads in flight across the round boundary.
          if (spin > (1u << 24)) {
            asm volatile("s_trap 2");
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
        if (elig && leader) dat[(gt & 7u) * kTileChunks + L.qg] = val;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        uint32_t old = 0;
        if (L.lane == 0) old = __hip_atomic_fetch_add(own, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        old = rfl(old);
        const bool fin = (old & 15u) + 1u == expect;
        if (elig) range = 0u;
        if (fin) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
          if (elig) {
            sval = dat[L.lane];
            soff = L.lane * 4u;
            // eligible: the group starts at segment tile (gt & ~7) - mtile_start
            sbase = P::group_base(
                pol, sh.crcs + static_cast<uint64_t>((gt & ~7u) - static_cast<uint32_t>(sh.mtile_start)) * kTileChunks,
                sh, gt);
            range = P::drop(pol) ? 0u : 256u;
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
          if (L.lane == 0)
            __hip_atomic_store(own, (c.grp + kGatherSlots) << 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
      const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc(
          reinterpret_cast<uint32_t *>(rfl64(reinterpret_cast<uint64_t>(sbase))), 0, static_cast<int>(rfl(range)),
          0x00020000);
      P::group_store(pol, sval, rg, soff);
      return;
    }
    if constexpr (RUN == 1) {
      // ORDER 4: lane 8j + q collects chunk q of the run's tile j from that
      // chunk's leader lane 8q; the run's last tile writes the CRCs of its
      // R = rmask + 1 tiles (32 R bytes: whole lines for R >= 4) with one store
      const uint32_t j = c.tile & L.rmask;
      const uint32_t v =
          static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(static_cast<int>((L.lane & 7u) * 32u), static_cast<int>(val)));
      gs.acc = (last && (L.lane >> 3) == j) ? v : gs.acc;
      const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
          reinterpret_cast<uint32_t *>(rfl64(reinterpret_cast<uint64_t>(sh.crcs + (c.tile & ~L.rmask) * kTileChunks))), 0,
          static_cast<int>(rfl(last && j == L.rmask ? (8u * L.rmask + nch) * 4u : 0u)), 0x00020000);
      __builtin_amdgcn_raw_buffer_store_b32(gs.acc, rr, L.lane * 4u, 0, 16);
      return;
    }
    if constexpr (RUN == 3) {
      // Lazy gather (schedule 3): as RUN 2, but no LDS round trip is waited
      // on per tile -- the slot check was loaded before the slicing
      // (lazy_pre), the count this tile adds is read one round later, and the
      // group's finisher stores it then (lazy_flush).  A wave hands on the
      // slot of its pending group before it ever waits for a slot itself, so
      // the oldest unfinished group never waits: the wait ends.
      lazy_flush<P>(gs, sh, L);
      uint32_t range = keep ? nch * 4u : 0u;
      if (last) {
        const bool whole = ((static_cast<uint32_t>(sh.mtile_start) | sh.main_tiles) & 7u) == 0u;
        bool elig = whole && (uint64_t(c.tile | 7u) + 1u) * kTileChunks <= sh.nchunks;
        uint32_t expect = 8u;
        if (!elig) {
          const uint64_t gs0 = (sh.mtile_start + c.tile) & ~7ull;
          expect = static_cast<uint32_t>(min<uint64_t>(8u, L.ntiles - gs0));
          elig = expect == 8u && gs0 >= sh.mtile_start && gs0 + 8u <= sh.mtile_start + sh.main_tiles &&
                 (gs0 + 8u - sh.mtile_start) * kTileChunks <= sh.nchunks;
        }
        const uint32_t gt = static_cast<uint32_t>(sh.mtile_start) + c.tile;
        const uint32_t sl = c.grp & (kGatherSlots - 1u);
        uint32_t *own = L.gslot + sl;
        uint32_t o = rfl(gs.chk);
        for (uint32_t spin = 0; (o >> 4) != c.grp; spin++) {  // rare: the slot's previous group is still open
          if (spin > (1u << 24)) {  // never expected: fail loudly (s_trap, see RUN 2)
            asm volatile("s_trap 2");
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          o = rfl(__hip_atomic_load(own, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        }
        if (elig && leader) L.gslot[kGatherSlots + sl * 64u + (gt & 7u) * kTileChunks + L.qg] = val;
        __atomic_signal_fence(__ATOMIC_SEQ_CST);  // the CRC words before the count (in-order LDS)
        uint32_t old = 0;
        if (L.lane == 0) old = __hip_atomic_fetch_add(own, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        gs.old = old;  // read one round later (lazy_pre)
        gs.pslot = sl;
        gs.pgrp = c.grp;
        gs.pexpect = expect;
        gs.pelig = elig ? 1u : 0u;
        gs.pbase = sh.crcs + static_cast<uint64_t>((gt & ~7u) - static_cast<uint32_t>(sh.mtile_start)) * kTileChunks;
        if (elig) range = 0u;
      }
      // tiles of groups that are not 8 whole tiles of one segment: their own 32 B
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          reinterpret_cast<uint32_t *>(rfl64(reinterpret_cast<uint64_t>(sh.crcs + c.tile * kTileChunks))), 0,
          static_cast<int>(rfl(range)), 0x00020000);
      P::group_store(pol, val, rs, leader ? L.qg * 4u : 0x80000000u);
      return;
    }
    if constexpr (P::kAltTileStores)
      if (P::tile_store_alt(pol, sh, segs, c, keep, nch, leader, L, val)) return;
    // descriptor fields forced uniform (readfirstlane): otherwise the
    // compiler may treat them as divergent and wrap the store in a
    // waterfall loop
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<uint32_t *>(rfl64(reinterpret_cast<uint64_t>(sh.crcs + c.tile * kTileChunks))), 0,
        static_cast<int>(rfl(keep ? nch * 4u : 0u)), 0x00020000);
    P::tile_store(pol, val, rs, leader ? L.qg * 4u : 0x80000000u, L.qg);
  } else {
    const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<uint8_t *>(rfl64(reinterpret_cast<uint64_t>(sh.bitmap + c.tile))), 0,
        static_cast<int>(rfl((last && !P::drop(pol)) ? 1u : 0u)), 0x00020000);
    P::bitmap_store(pol, static_cast<uint8_t>(byte), rb, L.lane == 0 ? 0u : 0x80000000u);
    if (byte && L.lane == 0) {  // rare: only tiles with a mismatch
      atomicMin(&first_bad[c.seg], c.tile * kTileChunks + __builtin_ctz(byte));
      atomicAdd(mism, static_cast<unsigned long long>(__builtin_popcount(byte)));
    }
    if constexpr (TabEarly<Tab>::value)
      if (last && L.early) segs.tile_done(c.seg, byte, L.lane);
  }
}

// Verify + copy-out (COPY kernels): the round's data, still in the loaded
// lane order, goes to the segment's copy_dst at the offsets it was loaded
// from (fully coalesced 1 KiB per instruction, the mirror of issue()),
// restricted to the segment's copy window [copy_w0, copy_w1) -- the whole
// payload, or the part of the packet a client read takes
// (src/datanode.c:2478-2488, 2527-2540): data byte j lands at copy_dst +
// (j - copy_w0).  A 16-B piece inside the window is one lane of the vector
// store; a piece outside it (and every piece of a parked cursor or of a
// segment without copy_dst) gets an out-of-range offset and is dropped; a
// piece that straddles an edge of the window -- only where a read starts or
// ends inside a packet, at most two pieces per read -- is stored byte by
// byte.  (Tiled rounds cover whole chunks, so a window edge at the payload's
// end never falls inside a piece.)
template <class P = EP, class Tab = SegP>
DEV void copy_round(const uint32_t (&d)[16], const Cursor c, Tab segs, const LaneConst &L, SegCache &kc) {
  const SegHot &sh = hot(kc, segs, c.seg).h;
  const uint32_t cs = sh.chunk_size;
  uint8_t *dst = segs[c.seg].copy_dst;
  const uint32_t w0 = segs[c.seg].copy_w0, w1 = segs[c.seg].copy_w1;
  const uint32_t nch = min(kTileChunks, sh.nchunks - c.tile * kTileChunks);
  const bool ok = c.valid && dst != nullptr;
  // data offset of the round, and the window relative to it (payloads are
  // < 2^31 bytes: int32 arithmetic)
  const int32_t rp = static_cast<int32_t>(c.tile * kTileChunks * cs + c.r * kRoundBytes);
  const int32_t lo = static_cast<int32_t>(w0) - rp, hi = static_cast<int32_t>(w1) - rp;
  // descriptor base: where the round's first byte would land (may precede
  // copy_dst when the window starts later; nothing below it is written)
  uint8_t *base = ok ? dst - w0 + rp : dst;
  const uint32_t valid = (nch - 1u) * cs + kRoundBytes;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<uint8_t *>(rfl64(reinterpret_cast<uint64_t>(base))), 0,
      static_cast<int>(rfl(ok && hi > 0 ? min(valid, static_cast<uint32_t>(hi)) : 0u)), 0x00020000);
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const u32x4 v = {d[4 * k + 0], d[4 * k + 1], d[4 * k + 2], d[4 * k + 3]};
    const int32_t o = static_cast<int32_t>((2u * k + L.hsel) * cs + L.loff);
    const bool inside = o >= lo && o + 16 <= hi;
    P::copy_store(L.store_policy, v, rs, inside ? static_cast<uint32_t>(o) : 0x80000000u);
    if (ok && !inside && o < hi && o + 16 > lo) {  // rare: the read starts or ends inside this piece
      for (int b = 0; b < 16; b++)
        if (o + b >= lo && o + b < hi)
          __builtin_amdgcn_raw_buffer_store_b8(static_cast<uint8_t>(v[b >> 2] >> (8 * (b & 3))), rs,
                                               static_cast<uint32_t>(o + b), 0, 0);
    }
  }
}

// Vector-memory stores process() issues per stream and round, on every path
// (dropped ones included): the bitmap byte (verify) or the CRC store
// (compute; the lazy gather also flushes its pending group; the load-only
// twin's byte), plus four copy stores (COPY).
template <int MODE, int COPY, int RUN>
constexpr int round_stores() {
  return (RUN == 3 ? 2 : 1) + (COPY ? 4 : 0);
}

// A vector store that writes nothing (a zero-size buffer range): it counts in
// vmcnt exactly as a dropped store of process() does.
DEV void pad_store(const void *base) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<uint32_t *>(rfl64(reinterpret_cast<uint64_t>(base))), 0, 0, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b32(0u, r, 0x80000000u, 0, 0);
}

// Process one round of each of the wave's S streams (d[s] for cursor c[s]);
// st[s] is stream s's running lane register across the rounds of a tile.
// The S slicing chains are independent and interleaved step by step, so one
// lane keeps S table lookups in flight (latency hiding by ILP, not waves).

template <int MODE, int S, int COPY, int UNA, int RUN, class P = EP, class Tab = SegP>
DEV void process(const uint32_t *lds, uint32_t (&d)[S][16], const uint32_t (&exp)[S], const uint32_t (&tl)[S],
                 const uint32_t (&sh_a)[S], const Cursor (&c)[S], Tab segs, uint32_t (&st)[S], const LaneConst &L,
                 uint32_t *__restrict__ first_bad, unsigned long long *__restrict__ mism, SegCache (&kc)[S],
                 Gst (&gs)[S]) {
  if constexpr (MODE == kModeLoadOnly) {  // diagnostic build only (the launcher refuses it otherwise)
    P::template load_only_round<S>(d, exp, c, segs, st, mism);
    return;
  }
  if constexpr (COPY && !UNA) {
#pragma unroll
    for (int s = 0; s < S; s++) copy_round<P>(d[s], c[s], segs, L, kc[s]);
  }
  if constexpr (RUN == 3) {
#pragma unroll
    for (int s = 0; s < S; s++) lazy_pre(gs[s], c[s], segs, kc[s], L);
  }
  uint32_t x[S];
#pragma unroll
  for (int s = 0; s < S; s++) {
    transpose(d[s]);
    if constexpr (UNA) {
      const uint32_t a = sh_a[s];
      const uint32_t nxt = dpp<0x101>(d[s][0]);  // row_shl:1 -- lane L + 1's first dword
      const uint32_t tv = static_cast<uint32_t>(
          __builtin_amdgcn_ds_bpermute(static_cast<int>((L.lane >> 3) * 4u), static_cast<int>(tl[s])));
      const uint32_t w16 = (L.lane & 7u) == 7u ? tv : nxt;
#pragma unroll
      for (int j = 0; j < 15; j++) d[s][j] = __builtin_amdgcn_alignbyte(d[s][j + 1], d[s][j], a);
      d[s][15] = __builtin_amdgcn_alignbyte(w16, d[s][15], a);
      if constexpr (COPY) {
        // the transpose is an involution: applied to the realigned quads it
        // gives back the loaded lane order, so the copy goes out as four fully
        // coalesced 1 KiB stores (quad-order stores touch 4x the lines each)
        uint32_t e[16];
#pragma unroll
        for (int j = 0; j < 16; j++) e[j] = d[s][j];
        transpose(e);
        copy_round<P>(e, c[s], segs, L, kc[s]);
      }
    }
    const uint32_t ri = hot(kc[s], segs, c[s].seg).reg_init;  // uniform control flow: kc stays in SGPRs
    if constexpr (RUN == 4) {
      // columns: the even lane of a chunk's pair continues the chunk's
      // register (reg_init in column 0), the odd lane starts from zero
      if (c[s].r == 0) st[s] = (L.lane & 1u) ? 0u : ri;
      else st[s] = (L.lane & 1u) ? 0u : st[s];
    } else {
      if (c[s].r == 0) st[s] = (L.qi == 0) ? ri : 0u;
      else st[s] = zshift(lds, L.z448, st[s]);
    }
    x[s] = st[s] ^ d[s][0];
  }
#pragma unroll
  for (int w = 0; w < 15; w++) {
#pragma unroll
    for (int s = 0; s < S; s++) x[s] = slice4(lds, x[s], d[s][w + 1], L.lb0, L.lb1);
  }
#pragma unroll
  for (int s = 0; s < S; s++) st[s] = slice4(lds, x[s], 0u, L.lb0, L.lb1);
  if constexpr (RUN == 4) {
    // columns: register of the chunk through this column = Z_64(even) ^ odd
    // (CRC linearity); quad_perm [1,0,3,2] hands it to both lanes of the pair
#pragma unroll
    for (int s = 0; s < S; s++) {
      const uint32_t z = zshift(lds, L.z64, st[s]);
      const uint32_t v = (L.lane & 1u) ? st[s] : z;
      st[s] = v ^ dpp<0xB1>(v);
    }
  }
#pragma unroll
  for (int s = 0; s < S; s++) finish<MODE, RUN, P>(lds, exp[s], c[s], segs, st[s], L, first_bad, mism, kc[s], gs[s]);
}

// Generic tiles inside a device-framed verify launch.  One lane per
// chunk of a generic tile, as crc32c_generic_kernel, but on the tiled
// kernel's replicated LDS tables (lane l reads its own copy: lb0 / lb1).
// gt: the lane's generic tile of the run (8 lanes per tile).
DEV void fused_generic_chunk(const uint32_t *lds, const SegDev *__restrict__ segs, uint32_t nseg, uint64_t gt,
                             bool active, const LaneConst &L, uint32_t *__restrict__ first_bad,
                             unsigned long long *__restrict__ mism) {
  const uint32_t g = L.lane & 7u;
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
      if (sg.copy_dst) {  // verify + copy-out: the chunk's bytes inside the window
        const uint64_t a = max<uint64_t>(off, sg.copy_w0), e = min<uint64_t>(off + n, sg.copy_w1);
        for (uint64_t j = a; j < e; j++) gstore8(sg.copy_dst + (j - sg.copy_w0), gload8(sg.data + j));
      }
      uint32_t c = sg.reg_init;
      // byte steps on t0 (pair 1, half 1 of the image), word steps by slice4
      while (n && (reinterpret_cast<uintptr_t>(p) & 3u)) {
        c = lds_at(lds, L.lb1 + 128u + (((c ^ gload8(p++)) & 0xffu) << 8)) ^ (c >> 8);
        n--;
      }
      while (n >= 4) {
        c = slice4(lds, c ^ gload32(p), 0u, L.lb0, L.lb1);
        p += 4;
        n -= 4;
      }
      while (n) {
        c = lds_at(lds, L.lb1 + 128u + (((c ^ gload8(p++)) & 0xffu) << 8)) ^ (c >> 8);
        n--;
      }
      out = (flags & kSegRaw) ? c : ~c;
    }
  }
  bool bad = false;
  if (valid) {
    uint32_t e = gload32(segs[s].crcs + chunk);
    if (flags & kSegBigEndian) e = __builtin_bswap32(e);
    bad = e != out;
  }
  const uint64_t m = __ballot(bad);
  if (active && g == 0) {
    const uint32_t byte = static_cast<uint32_t>((m >> (L.lane & 56u)) & 0xffu);
    gstore8(segs[s].bitmap + tile, static_cast<uint8_t>(byte));
    if (byte) {
      atomicMin(&first_bad[s], tile * kTileChunks + __builtin_ctz(byte));
      atomicAdd(mism, static_cast<unsigned long long>(__builtin_popcount(byte)));
    }
  }
}

// The bad-packet list of a verified run (one workgroup of BLOCK threads):
// every segment with a bad chunk -> one GridBad (packet, first bad chunk,
// bad chunks from its bitmap), to the device list and the first host_cap to
// pinned host memory, the count, then (one system fence later) the sequence
// number the host polls.  nb: an LDS word.
template <int BLOCK>
DEV void bad_list(const SegDev *__restrict__ segs, uint32_t nseg, const uint32_t *__restrict__ seg2pkt,
                  const uint32_t *__restrict__ fb, GridBad *__restrict__ bad, uint32_t bad_cap,
                  GridSummary *__restrict__ sum, uint8_t *__restrict__ hsum2, uint32_t host_cap, uint32_t seq,
                  uint32_t *nb) {
  if (threadIdx.x == 0) *nb = 0u;
  __syncthreads();
  auto *hbad = reinterpret_cast<GridBad *>(hsum2 + 256);
  // first-bad words in batches of 16 per thread, every load of a batch issued
  // before the first is tested (16 K segments: one round trip, not 16)
  for (uint32_t i0 = threadIdx.x; i0 < nseg; i0 += 16u * BLOCK) {
    uint32_t f[16];
#pragma unroll
    for (uint32_t u = 0; u < 16; u++) f[u] = i0 + u * BLOCK < nseg ? fb[i0 + u * BLOCK] : 0xFFFFFFFFu;
#pragma unroll
    for (uint32_t u = 0; u < 16; u++) {
      if (f[u] == 0xFFFFFFFFu) continue;  // rare: a segment with a bad chunk
      const uint32_t i = i0 + u * BLOCK;
      const SegDev d = segs[i];
      const uint32_t nbyte = (d.nchunks + 7u) / 8u;
      uint32_t n = 0;
      // the segment's bitmap bytes 16 at a time, every load of a batch issued
      // before the first is counted (a 64 KiB packet: one round trip, not 16
      // dependent ones -- a run with bad packets paid ~8 us for them)
      for (uint32_t j0 = 0; j0 < nbyte; j0 += 16u) {
        uint32_t by[16];
#pragma unroll
        for (uint32_t u = 0; u < 16; u++) by[u] = j0 + u < nbyte ? uint32_t(d.bitmap[j0 + u]) : 0u;
#pragma unroll
        for (uint32_t u = 0; u < 16; u++) {
          uint32_t byte = by[u];
          if (j0 + u == d.nchunks / 8u) byte &= (1u << (d.nchunks % 8u)) - 1u;  // bits past the last chunk
          n += __builtin_popcount(byte);
        }
      }
      const uint32_t slot = atomicAdd(nb, 1u);
      const GridBad g{seg2pkt[i], int32_t(f[u]), n, 0u};
      if (slot < bad_cap) bad[slot] = g;
      if (slot < host_cap) hbad[slot] = g;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    sum->nbad = *nb;
    reinterpret_cast<GridSummary *>(hsum2)->nbad = *nb;
  }
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_store(&reinterpret_cast<GridSummary *>(hsum2)->seq, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The generic tiles of a device-framed run, taken by the verify launch's
// own waves once they have no tiled round left: 8 tiles per wave and step,
// dealt statically over the launch's waves (one atomic per wave on one
// counter would serialise: 16 K waves cost ~50 us even with no generic tile
// to take).  No completion protocol: the bad-packet list is the next launch
// (grid_finalize_kernel), after the kernel boundary has made every bitmap
// store visible -- a last-workgroup-done protocol here needed an agent-scope
// fence (L2 write-back) per workgroup and cost more (+14 us per GiB) than
// the launch it saved.
template <int BLOCK>
DEV void fused_generic(const uint32_t *lds, const SegDev *__restrict__ segs, const GridSummary *__restrict__ dyn,
                       const LaneConst &L, uint32_t *__restrict__ first_bad, unsigned long long *__restrict__ mism) {
  const uint32_t nseg = dyn->nseg;
  const uint64_t ngt = dyn->gtiles;
  const uint64_t nw = uint64_t(gridDim.x) * (BLOCK / 64);
  const uint64_t wid = uint64_t(blockIdx.x) * (BLOCK / 64) + (threadIdx.x >> 6);
  for (uint64_t g0 = wid * 8u; g0 < ngt; g0 += nw * 8u) {
    const uint64_t gt = g0 + (L.lane >> 3);
    fused_generic_chunk(lds, segs, nseg, gt, gt < ngt, L, first_bad, mism);
  }
}

// LDS image of the tiled kernels (+ ticket counter, pad, kSlots 64-bit pool
// slots, + GATHER: the group slots), filled by every thread of the
// workgroup; no barrier (the caller's __syncthreads follows).
// LDS image: word (P*16384 + e*64 + h*32 + l) = t_{3-(2P+h)}[e] for all 32 l.
// Filled with 16-B stores, consecutive lanes on consecutive 16 B (no bank
// conflicts); the source words a lane needs are loaded up front so the
// fill costs about one L2 round trip, not one per store.
template <int BLOCK, int GATHER>
DEV void fill_tables(uint32_t *lds, const uint32_t *__restrict__ gtab) {
  if (threadIdx.x < 2 + 2 * kSlots) lds[kLdsWords + threadIdx.x] = 0u;
  // group slot s starts owned by group s, no tile counted
  if (GATHER && threadIdx.x < kGatherSlots) lds[kLdsWords + 2 + 2 * kSlots + threadIdx.x] = threadIdx.x << 4;
  constexpr uint32_t kStores = kLdsSliceBytes / 16;
  constexpr uint32_t kQ = (kStores + BLOCK - 1) / BLOCK;  // 16-B stores per thread
  constexpr uint32_t kZ = (kTabZposWords / 4 + BLOCK - 1) / BLOCK;
  uint32_t v[kQ];
#pragma unroll
  for (uint32_t k = 0; k < kQ; k++) {
    const uint32_t idx = 4u * min(k * BLOCK + threadIdx.x, kStores - 1u);
    const uint32_t P = idx >> 14, e = (idx >> 6) & 255u, h = (idx >> 5) & 1u;
    v[k] = gtab[(3u - (2u * P + h)) * 256u + e];
  }
  u32x4 z[kZ];
#pragma unroll
  for (uint32_t k = 0; k < kZ; k++) {
    const uint32_t q = k * BLOCK + threadIdx.x;
    z[k] = q < kTabZposWords / 4 ? gload16(gtab + kTabSliceWords + 4u * q) : u32x4{0u, 0u, 0u, 0u};
  }
#pragma unroll
  for (uint32_t k = 0; k < kQ; k++) {
    const uint32_t q = k * BLOCK + threadIdx.x;
    if (kStores % BLOCK == 0 || q < kStores)
      *reinterpret_cast<u32x4 *>(&lds[4u * q]) = u32x4{v[k], v[k], v[k], v[k]};
  }
#pragma unroll
  for (uint32_t k = 0; k < kZ; k++) {
    const uint32_t q = k * BLOCK + threadIdx.x;
    if (q < kTabZposWords / 4) *reinterpret_cast<u32x4 *>(&lds[kLdsSliceBytes / 4 + 4u * q]) = z[k];
  }
}

// The tiled kernels' work loop after the LDS tables are in place: schedule,
// round pipeline, epilogue.  MODE compute / verify; ORDER schedule (above);
// NT nontemporal data loads; DEPTH register round buffers per stream (DEPTH-1
// rounds stay in flight while one is processed); S independent tile streams
// per wave (S x 4 KiB per round, S chains of ILP); BLOCK threads per
// workgroup (one workgroup per CU: the LDS image takes 156 KiB).  Tab: the
// segment table -- a SegP in HBM (crc32c_tiles_kernel) or the closed form of
// a run of equal packets (SpecTab, spec_verify_kernel).  segs: the table in
// HBM for the fused generic tiles (fused only).
template <int MODE, int ORDER, int NT, int DEPTH, int S, int BLOCK, int BUF, int COPY, int UNA, int GATHER,
          class Tab>
DEV void tiles_run(uint32_t *lds, const Tab sg, const SegDev *__restrict__ segs, uint32_t nseg, uint64_t total_rounds,
                   uint64_t total_tiles, uint32_t *__restrict__ first_bad, unsigned long long *__restrict__ mism,
                   unsigned long long *__restrict__ diag, uint32_t tune, uint32_t *__restrict__ gctr,
                   const GridSummary *__restrict__ dyn, uint32_t utiles, bool fused) {
  static_assert(ORDER != 0 || S == 1, "static per-wave slices serve one stream");
  static_assert(ORDER != 7 || (MODE == kModeCompute && S == 1 && BUF && !COPY && !UNA && !GATHER), "columns shape");
  static_assert(DEPTH >= 2 && DEPTH <= 4 && S >= 1 && S <= 4, "shape");
  // GATHER 1: the compute gather (RUN 2); 2: the lazy gather (RUN 3)
  static_assert(GATHER == 0 || (MODE == kModeCompute && ORDER == 3 && S == 1), "gather: compute, schedule 3");
  LaneConst L;
  // tune: [7:0] store policy (diagnostic build), [11:8] ORDER-3 group shift,
  // [13:12] ORDER-3 dealing: 0 plain, 1 XCD-major, 2 XCD-split, [23:16] pool
  // threshold in rounds per wave (uniform: SGPR)
  L.store_policy = EP::policy(tune & 0xffu);
  L.lane = threadIdx.x & 63u;
  L.hsel = (L.lane >> 3) & 1u;                              // load: odd sub-chunk of each 1 KiB
  L.loff = 16u * (4u * (L.lane & 7u) + (L.lane >> 4));      // load: byte offset in the sub-chunk
  L.lb0 = (L.lane & 31u) * 4u;
  L.lb1 = 65536u + (L.lane & 31u) * 4u;
  L.qi = L.lane & 7u;                    // 64-B position within the chunk's 512-B round
  L.qg = L.lane >> 3;                    // chunk within the tile after the transpose
  L.zk = 7u - L.qi;
  L.zbase = kLdsSliceBytes / 4 + (L.zk ? L.zk - 1u : 0u) * 1024u;
  L.z448 = kLdsSliceBytes / 4 + 6u * 1024u;
  L.z64 = kLdsSliceBytes / 4;  // ORDER 7: Z_64
  L.ntiles = total_tiles;
  L.gslot = &lds[kLdsWords + 2 + 2 * kSlots];
  L.rmask = 7u;
  L.early = 0u;

  constexpr uint32_t wpb = BLOCK / 64;
  const uint32_t wave = rfl(blockIdx.x * wpb + (threadIdx.x >> 6));
  const uint32_t nwaves = gridDim.x * wpb;
  // Diagnostic build path (diag != nullptr): per-wave start / end wall clock
  // (s_memrealtime, 100 MHz) and rounds processed; nothing is computed from it.
  if (kDiag && diag && L.lane == 0) diag[3 * wave] = __builtin_amdgcn_s_memrealtime();
  uint64_t nrounds = 0;
  Sched w{0, 0, 0, &lds[kLdsWords], L.lane};
  w.ut = utiles;
  w.ush = (utiles & (utiles - 1u)) == 0u ? static_cast<uint32_t>(__builtin_ctz(utiles | (utiles == 0u ? 1u : 0u)))
                                         : 0xFFFFFFFFu;
  w.um = (utiles && w.ush == 0xFFFFFFFFu) ? ~0ull / utiles + 1ull : 0ull;
  Cursor cur[DEPTH][S];
#pragma unroll
  for (int s = 0; s < S; s++) cur[0][s] = Cursor{0u, 0u, 0u, false};
  if (ORDER == 0) {
    Cursor &c0 = cur[0][0];
    const uint64_t r0 = rfl64(total_rounds * wave / nwaves);
    w.r1 = rfl64(total_rounds * (wave + 1) / nwaves);
    if (r0 < w.r1) {
      const uint64_t g = tile_at_round(sg, nseg, r0, total_tiles);
      if (g < total_tiles) {
        uint32_t lo = 0, hi = nseg;
        while (hi - lo > 1) {
          const uint32_t mid = (lo + hi) >> 1;
          if (sg[mid].mtile_start <= g) lo = mid; else hi = mid;
        }
        c0 = locate(sg, lo, g);
        c0.valid = sg[c0.seg].round_start + uint64_t(c0.tile) * (sg[c0.seg].chunk_size / kRoundBytes) < w.r1;
      }
    }
  } else {
    // tune bits 23:16: rounds per wave from which the pool is used (0: 32)
    const uint32_t pmin = (tune >> 16) & 0xffu;
    const bool pool = ORDER >= 2 && total_rounds >= uint64_t(pmin ? pmin : 32u) * nwaves * S;
    if (ORDER >= 3) {
      // static phase: whole groups only; the pool takes the rest
      // ORDER 4: 2^gshift tiles per run (8 in the diagnostic default; 4 = one
      // 128-B CRC line per run), at most 8 (one register of CRCs)
      w.gshift = ORDER == 7 ? kColShift : ORDER == 4 ? min((tune >> 8) & 15u, 3u) : (tune >> 8) & 15u;
      if (ORDER == 4) L.rmask = (1u << w.gshift) - 1u;
      const uint64_t ngroups = (pool ? total_tiles * kPhase1Num / kPhase1Den : total_tiles) >> w.gshift;
      // tune bit 12: XCD-major dealing.  Workgroups are dispatched to the 8
      // XCDs round-robin (XCD = blockIdx % 8), so with the plain dealing the
      // groups an XCD works on at one time are 8 apart; dealing by the
      // virtual id (blockIdx % 8) * (G / 8) + blockIdx / 8 gives each XCD
      // (and its L2) a contiguous run of G / 8 groups per sweep step.
      // tune bits 13:12 = 2: XCD-split dealing.  XCD x owns the contiguous
      // eighth [x * ngx, (x + 1) * ngx) of the static groups and deals it over
      // its G/8 workgroups, so the 8 XCDs sweep 8 separate windows (their
      // compute-mode CRC writes land in 8 separate regions at any moment);
      // the < 8 leftover groups go to the pool.
      const uint32_t b = blockIdx.x, G = gridDim.x, xm = (tune >> 12) & 3u;
      if (xm == 2u && (G % 8u) == 0 && ngroups >= 8ull * (G / 8u)) {
        const uint64_t ngx = ngroups / 8u;
        const uint32_t G8 = G / 8u, l = b / 8u;
        w.gfirst = (b % 8u) * ngx + l;
        w.gstride = G8;
        w.nk = static_cast<uint32_t>(((ngx - 1 - l) / G8 + 1) << (ORDER == 4 || ORDER == 7 ? 0u : w.gshift));
        w.p2first = (ngx * 8u) << w.gshift;
      } else {
        w.gfirst = xm != 0u && (G % 8u) == 0 ? (b % 8u) * (G / 8u) + b / 8u : b;
        w.gstride = gridDim.x;
        // tickets of the static phase: tiles (ORDER 3) or whole groups (ORDER 4)
        w.nk = ngroups > w.gfirst
                   ? static_cast<uint32_t>(((ngroups - 1 - w.gfirst) / gridDim.x + 1) << (ORDER == 4 || ORDER == 7 ? 0u : w.gshift))
                   : 0u;
        w.p2first = ngroups << w.gshift;
      }
    } else {
      const uint64_t r_static = pool ? total_rounds * kPhase1Num / kPhase1Den : total_rounds;
      const uint64_t b0 = rfl64(r_static * blockIdx.x / gridDim.x);
      const uint64_t b1 = rfl64(r_static * (blockIdx.x + 1) / gridDim.x);
      w.gfirst = tile_at_round(sg, nseg, b0, total_tiles);
      w.nk = static_cast<uint32_t>(tile_at_round(sg, nseg, b1, total_tiles) - w.gfirst);
      w.p2first = tile_at_round(sg, nseg, r_static, total_tiles);
    }
    w.ntiles = total_tiles;
    if constexpr (TabEarly<Tab>::value) L.early = sg.early_ok(w.nk);
    {
      const uint64_t per = (total_tiles - w.p2first) / (4ull * gridDim.x);
      w.ushift = per >= (1ull << kUnitMaxShift) ? kUnitMaxShift
               : per < (1ull << kUnitMinShift) ? kUnitMinShift
                                               : 63u - static_cast<uint32_t>(__builtin_clzll(per));
    }
    w.gctr = gctr;
    w.slots = reinterpret_cast<uint64_t *>(&lds[kLdsWords + 2]);
#pragma unroll
    for (int s = 0; s < S; s++) {
      uint64_t g;
      const uint32_t tk = grab(w);
      if (ticket_tile<ORDER>(w, tk, g)) {
        if (w.ut) {
          cur[0][s] = ulocate(w, g);
        } else {
          uint32_t lo = 0, hi = nseg;
          while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (sg[mid].mtile_start <= g) lo = mid; else hi = mid;
          }
          cur[0][s] = locate(sg, lo, g);
        }
        cur[0][s].grp = tk >> 3;
      }
    }
  }
  bool any = false;
#pragma unroll
  for (int s = 0; s < S; s++) any |= cur[0][s].valid;
  if (!any) {
    if constexpr (MODE == kModeVerify)
      if (fused) fused_generic<BLOCK>(lds, segs, dyn, L, first_bad, mism);
    if (kDiag && diag && L.lane == 0) diag[3 * wave + 1] = __builtin_amdgcn_s_memrealtime();
    return;
  }
  // A stream that got no tile parks on stream 0's position (valid = false):
  // its loads stay in bounds and its stores are dropped.
#pragma unroll
  for (int s = 1; s < S; s++)
    if (!cur[0][s].valid) cur[0][s] = Cursor{cur[0][0].seg, cur[0][0].tile, cur[0][0].r, false};

  // DEPTH round buffers per stream in rotation: slot k is processed, then
  // refilled with the round after the newest cursor (slot k-1).  Fully
  // unrolled, so every buffer stays in fixed registers.  One exit test per
  // iteration (after all issues) and no memory op under a condition: every
  // path issues the same vector-memory ops in the same order, so the vmcnt
  // bookkeeping stays exact.  Rounds of an exhausted cursor are processed
  // with their stores dropped.
  uint32_t buf[DEPTH][S][16];
  uint32_t ex[DEPTH][S];
  uint32_t tl[DEPTH][S];   // UNA: lanes 0..7, the dword after chunk lane's round part
  uint32_t sha[DEPTH][S];  // UNA: byte shift of the round's segment
  uint32_t st[S];
  Gst gs[S];  // epilogue state: ORDER 4 compute's run CRCs, the lazy gather's pending tile
  LaneOff lo{0u, {0u, 0u, 0u, 0u}, 0u};
  SegCache kc[S];
#pragma unroll
  for (int s = 0; s < S; s++) {
    st[s] = 0u;
    gs[s] = Gst{0u, 0u, 0u, 0u, kNoSlot, 0u, 0u, 0u, 0u, nullptr};
    kc[s].seg = 0xFFFFFFFFu;
  }
#pragma unroll
  for (int k = 1; k < DEPTH; k++) {
#pragma unroll
    for (int s = 0; s < S; s++) cur[k][s] = advance<ORDER>(cur[k - 1][s], sg, nseg, w, kc[s]);
  }
#pragma unroll
  for (int k = 0; k < DEPTH; k++) {
#pragma unroll
    for (int s = 0; s < S; s++) {
      ex[k][s] = 0u;
      tl[k][s] = 0u;
      sha[k][s] = 0u;
      issue<MODE, NT, BUF, UNA, ORDER == 7>(buf[k][s], ex[k][s], tl[k][s], sha[k][s], cur[k][s], sg, L.hsel, L.loff, L.qg, L.lane,
                                lo, kc[s], L.store_policy);
    }
    // In the loop every round's loads are separated from the next round's by
    // that round's stores; the prologue issues as many empty stores between
    // its rounds, so the loop head -- where the compiler's vmcnt count merges
    // the prologue with the back edge -- sees the same number of younger
    // operations.  Without them the count assumed no stores in flight and the
    // first two of the three unrolled rounds waited for 2 and 1 operations
    // more than their own loads (vmcnt(13)/(11)/(10) instead of (15)/(13)/(12)
    // in verify): the oldest store and the next round's first load, a load
    // issued one round later than the data being waited for.
    if (k + 1 < DEPTH) {
      constexpr int RUN = ORDER == 7 ? 4 : (ORDER == 4 && MODE == kModeCompute) ? 1 : GATHER == 2 ? 3 : GATHER ? 2 : 0;
#pragma unroll
      for (int j = 0; j < S * round_stores<MODE, COPY, RUN>(); j++) pad_store(first_bad);
    }
  }
  for (uint32_t it = 0;; it++) {
    EP::loop_hook(L.store_policy, it);
#pragma unroll
    for (int k = 0; k < DEPTH; k++) {
      process<MODE, S, COPY, UNA,
              ORDER == 7 ? 4 : (ORDER == 4 && MODE == kModeCompute) ? 1 : GATHER == 2 ? 3 : GATHER ? 2 : 0>(
          lds, buf[k], ex[k], tl[k], sha[k], cur[k], sg, st, L, first_bad, mism, kc, gs);
#pragma unroll
      for (int s = 0; s < S; s++) nrounds += cur[k][s].valid ? 1u : 0u;
      const int prev = (k + DEPTH - 1) % DEPTH;
#pragma unroll
      for (int s = 0; s < S; s++) {
        cur[k][s] = advance<ORDER>(cur[prev][s], sg, nseg, w, kc[s]);
        issue<MODE, NT, BUF, UNA, ORDER == 7>(buf[k][s], ex[k][s], tl[k][s], sha[k][s], cur[k][s], sg, L.hsel, L.loff, L.qg,
                                  L.lane, lo, kc[s], L.store_policy);
      }
    }
    bool more = false;
#pragma unroll
    for (int s = 0; s < S; s++) more |= cur[0][s].valid;
    if (!more) break;
  }
  if constexpr (GATHER == 2) {  // the lazy gather's last pending tile: its group may still be this wave's to store
#pragma unroll
    for (int s = 0; s < S; s++) {
      lazy_pre(gs[s], cur[0][s], sg, kc[s], L);
      lazy_flush<EP>(gs[s], hot(kc[s], sg, cur[0][s].seg).h, L);
    }
  }
  if constexpr (MODE == kModeVerify)
    if (fused) fused_generic<BLOCK>(lds, segs, dyn, L, first_bad, mism);
  if (kDiag && diag && L.lane == 0) {
    diag[3 * wave + 1] = __builtin_amdgcn_s_memrealtime();
    diag[3 * wave + 2] = nrounds;
  }
}

// Tiled kernel over a segment table in HBM (plans, packet pieces, device-
// framed runs).  dyn: sizes of a segment table built on the device
// (frame_build_kernel), read here instead of passed by the host -- no host
// round trip between framing and verify.
template <int MODE, int ORDER, int NT, int DEPTH, int S, int BLOCK, int BUF = 0, int COPY = 0, int UNA = 0,
          int GATHER = 0>
__global__ __launch_bounds__(BLOCK) void crc32c_tiles_kernel(
    const SegDev *__restrict__ segs, uint32_t nseg, uint64_t total_rounds, uint64_t total_tiles,
    const uint32_t *__restrict__ gtab, uint32_t *__restrict__ first_bad,
    unsigned long long *__restrict__ mism, unsigned long long *__restrict__ diag, uint32_t tune,
    uint32_t *__restrict__ gctr, const GridSummary *__restrict__ dyn, uint32_t utiles, uint32_t fuse) {
  // fused epilogue (verify with a device-built table only; uniform)
  const bool fused = MODE == kModeVerify && dyn && fuse;
  if (dyn) {
    nseg = dyn->nseg;
    total_rounds = dyn->rounds;
    total_tiles = dyn->mtiles;
    utiles = dyn->utiles;
  }
  __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsWords + 2 + 2 * kSlots + (GATHER ? kGatherWords : 0)];
  fill_tables<BLOCK, GATHER>(lds, gtab);
  __syncthreads();
  tiles_run<MODE, ORDER, NT, DEPTH, S, BLOCK, BUF, COPY, UNA, GATHER>(lds, (SegP)(segs), segs, nseg, total_rounds,
                                                                       total_tiles, first_bad, mism, diag, tune, gctr,
                                                                       dyn, utiles, fused);
}


// Generic path: one lane per chunk, 8 lanes per tile.  Serves chunks the
// tiled kernel cannot: partial last chunks, chunk sizes that are not a
// multiple of 512 (and, with HDFS_CRC32C_ALIGN > 1, data below that alignment).
template <int MODE>
__global__ __launch_bounds__(256) void crc32c_generic_kernel(
    const SegDev *__restrict__ segs, uint32_t nseg, uint64_t total_gtiles,
    const uint32_t *__restrict__ gtab, uint32_t *__restrict__ first_bad,
    unsigned long long *__restrict__ mism, const GridSummary *__restrict__ dyn) {
  if (dyn) {  // sizes from a device-built table (the launch's grid is an upper bound)
    nseg = dyn->nseg;
    total_gtiles = dyn->gtiles;
  }
  // blocks past the work leave before the table load (a device-built run
  // usually has no generic tiles at all: the whole grid exits here)
  if (static_cast<uint64_t>(blockIdx.x) * blockDim.x / kTileChunks >= total_gtiles) return;
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
      if (sg.copy_dst) {  // verify + copy-out: this lane's chunk (tails and odd chunk sizes) inside the window
        const uint64_t a = max<uint64_t>(off, sg.copy_w0), e = min<uint64_t>(off + n, sg.copy_w1);
        for (uint64_t j = a; j < e; j++) gstore8(sg.copy_dst + (j - sg.copy_w0), gload8(sg.data + j));
      }
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

// GF(2) product a * b mod P of two reflected polynomials (x^0 at bit 31),
// branch-free: bit 31 - i of a is the x^i coefficient; b steps through
// b * x^i.  About 5 VALU ops per bit and no table (the LDS stays free for
// the replicated slicing tables).
DEV uint32_t gf2_mulmod(uint32_t a, uint32_t b, uint32_t poly) {
  uint32_t p = 0u;
#pragma unroll
  for (int i = 31; i >= 0; i--) {
    p ^= b & (0u - ((a >> i) & 1u));
    b = (b >> 1) ^ (poly & (0u - (b & 1u)));
  }
  return p;
}

// One-launch kernel for the synchronous host-memory calls on <= kSmallMax
// bytes: the drop-in _hdfs_crc32c family (src/crc32c.h:13-24, one chunk of
// `len` bytes continuing from the caller's register), the write loop mirror
// (src/datanode.c:2814-2860, compute) and _verify_crcdata
// (src/datanode.c:2931-2963, verify).  The caller's bytes are staged in
// fine-grained VRAM written through the BAR (large-BAR devices) or pinned
// host memory read over PCIe (coalesced 1 KiB per wave instruction, no DMA
// copy, no second launch); results and a completion sequence number go
// straight back to pinned host memory, which the host polls.
//
// Each chunk is split in 16/32/64-B pieces, one per thread: piece k of chunk
// j yields the raw register r (the chunk's first piece starts from `reg0`),
// moved past the rest of its chunk (dd = 64 m + r bytes) by GF(2) multiplies
// with x^(512 m) and x^(8 r) mod P (kx; the combine algebra of
// src/crc32c_sse42.c:99-200) and XOR-ed into the chunk's accumulator in LDS.
// Needs chunk_size % 4 == 0 and at most kSmallMaxChunks chunks.
// meta: [0] first bad chunk (verify, 0xFFFFFFFF none) [1] mismatches
//       [2] completion sequence number; crcs: compute output (u32, BE if be)
template <int MODE>
__global__ __launch_bounds__(1024) void small_chunks_kernel(const uint8_t *__restrict__ p, uint32_t len,
                                                             uint32_t exact, uint32_t cs, uint32_t reg0, uint32_t be,
                                                             const uint32_t *__restrict__ expect,
                                                             const uint32_t *__restrict__ tab,
                                                             const uint32_t *__restrict__ kx, uint32_t poly,
                                                             uint32_t *__restrict__ meta,
                                                             uint32_t *__restrict__ crcs, uint32_t seq) {
  __shared__ uint32_t tt[1024];                             // t0..t3
  __shared__ uint32_t dat[kSmallMax / 4 + kSmallMax / 64];  // one pad word per 16
  __shared__ __attribute__((aligned(16))) uint32_t acc[kSmallMaxChunks];  // (a copy request: its staged pieces)
  __shared__ uint32_t res[2];
  const uint32_t tid = threadIdx.x;
  // piece size: 16, 32 or 64 B, the smallest that keeps the pieces within
  // one pass of the block (short chains for short inputs)
  const uint32_t nch = (len + cs - 1) / cs;
  uint32_t psz = 16u;
  while (psz < 64u && nch * ((cs + psz - 1) / psz) > 1024u) psz *= 2u;
  const uint32_t ppc = (cs + psz - 1) / psz;
  // Every global / host load of the prologue is issued before any LDS
  // store (one round trip for the data, one HBM/L2 trip for the table and
  // this thread's first two multipliers).
  static_assert(kSmallMax / 16 == 4 * 1024 && kSmallMaxChunks == 2 * 1024, "prologue shape");
  const uint64_t ts0 = __builtin_amdgcn_s_memrealtime();  // phase stamps (100 MHz) -> meta[4..11]
  const uint32_t nvec = (len + 15u) / 16u;
  const uint32_t tv = tab[tid];
  // shift distance of this thread's first piece (the loop below starts there)
  uint32_t km0 = 0x80000000u, kr0 = 0x80000000u;
  if (tid < nch * ppc) {
    const uint32_t j = tid / ppc, cend = min((j + 1u) * cs, len), b0 = j * cs + psz * (tid - j * ppc);
    if (b0 < cend) {
      const uint32_t dd = cend - min(b0 + psz, cend);
      km0 = kx[dd >> 6];
      kr0 = kx[1024u + (dd & 63u)];
    }
  }
  u32x4 dv[4];
  uint32_t ev[2] = {0u, 0u};
  // buffer loads, sc0 sc1 (system-coherent: the stage is VRAM the host
  // wrote through the BAR, or pinned memory): a device source (exact) at any
  // byte address (a global dwordx4 load returns the aligned-down bytes), the
  // stage in whole 16 B
  const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t *>(p), 0, static_cast<int>(exact ? len : 16u * nvec), 0x00020000);
#pragma unroll
  for (uint32_t k = 0; k < 4; k++) {
    const uint32_t q = k * 1024u + tid;
    dv[k] = u32x4{0u, 0u, 0u, 0u};
    if (q < nvec) {
      if (exact && 16u * q + 16u > len) {  // device source: never read past len
        uint32_t wds[4] = {0u, 0u, 0u, 0u};
        for (uint32_t b = 16u * q; b < len; b++) wds[(b >> 2) & 3u] |= uint32_t(gload8(p + b)) << (8u * (b & 3u));
        dv[k] = u32x4{wds[0], wds[1], wds[2], wds[3]};
      } else {
        dv[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rp, 16u * q, 0, 17));
      }
    }
  }
  if (MODE == kModeVerify) {
    const __amdgpu_buffer_rsrc_t re = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t *>(expect), 0,
                                                                        static_cast<int>(4u * nch), 0x00020000);
#pragma unroll
    for (uint32_t k = 0; k < 2; k++)
      if (k * 1024u + tid < nch) ev[k] = __builtin_amdgcn_raw_buffer_load_b32(re, 4u * (k * 1024u + tid), 0, 17);
  }
  tt[tid] = tv;
  for (uint32_t j = tid; j < nch; j += 1024u) acc[j] = 0u;
  if (tid < 2) res[tid] = tid == 0 ? 0xFFFFFFFFu : 0u;
#pragma unroll
  for (uint32_t k = 0; k < 4; k++) {
    const uint32_t q = k * 1024u + tid;
    if (q < nvec) {
      const uint32_t w = 4u * q + (q >> 2);
      dat[w] = dv[k].x;
      dat[w + 1] = dv[k].y;
      dat[w + 2] = dv[k].z;
      dat[w + 3] = dv[k].w;
    }
  }
  __syncthreads();
  const uint64_t ts1 = __builtin_amdgcn_s_memrealtime();
  // aligned groups of g pieces lie in one chunk (g = lowest set bit of the
  // pieces per chunk, 64 for a single chunk): XOR-reduced across lanes
  // before one LDS atomic per group
  const uint32_t g = nch == 1u ? 64u : min(64u, ppc & (0u - ppc));
  for (uint32_t t0 = 0; t0 < nch * ppc; t0 += 1024u) {  // uniform
    const uint32_t t = t0 + tid;
    const uint32_t j = t / ppc, k = t - j * ppc;
    const uint32_t cend = min((j + 1u) * cs, len);
    const uint32_t b0 = j * cs + psz * k;
    uint32_t c = 0u;
    if (t < nch * ppc && b0 < cend) {  // (the last chunk may be short)
      const uint32_t e = min(b0 + psz, cend);
      c = k == 0 ? reg0 : 0u;
      uint32_t b = b0;
      for (; b + 4u <= e; b += 4u) {
        const uint32_t w = b >> 2;
        const uint32_t x = c ^ dat[w + (w >> 4)];
        c = tt[768u + (x & 0xffu)] ^ tt[512u + ((x >> 8) & 0xffu)] ^ tt[256u + ((x >> 16) & 0xffu)] ^ tt[x >> 24];
      }
      for (; b < e; b++) {
        const uint32_t w = b >> 2;
        const uint32_t byte = (dat[w + (w >> 4)] >> (8u * (b & 3u))) & 0xffu;
        c = tt[(c ^ byte) & 0xffu] ^ (c >> 8);
      }
      const uint32_t dd = cend - e;
      if (dd) {
        const bool first = t0 == 0u;  // multipliers prefetched in the prologue
        const uint32_t km = first ? km0 : kx[dd >> 6], kr = first ? kr0 : kx[1024u + (dd & 63u)];
        if (dd & 63u) c = gf2_mulmod(kr, c, poly);
        if (dd >> 6) c = gf2_mulmod(km, c, poly);
      }
    }
#pragma unroll
    for (uint32_t sh = 1; sh < 64u; sh <<= 1)
      if (sh < g) c ^= __shfl_xor(c, sh);
    if ((tid & (g - 1u)) == 0u && c) atomicXor(&acc[j], c);
  }
  __syncthreads();
  const uint64_t ts2 = __builtin_amdgcn_s_memrealtime();
  if (MODE == kModeVerify) {
#pragma unroll
    for (uint32_t k = 0; k < 2; k++) {
      const uint32_t j = k * 1024u + tid;
      if (j < nch && (be ? __builtin_bswap32(ev[k]) : ev[k]) != ~acc[j]) {
        atomicMin(&res[0], j);
        atomicAdd(&res[1], 1u);
      }
    }
    __syncthreads();
  }
  // Wave 0 alone writes every result to host memory, so one system-scope
  // fence (one PCIe write round trip) orders them all before the sequence
  // number the host polls.
  if (tid < 64u) {
    if (MODE == kModeCompute) {
      for (uint32_t j = tid; j < nch; j += 64u) {
        const uint32_t v = ~acc[j];
        crcs[j] = be ? __builtin_bswap32(v) : v;
      }
    }
    if (tid == 0) {
      const uint64_t ts3 = __builtin_amdgcn_s_memrealtime();
      meta[0] = res[0];
      meta[1] = res[1];
      meta[4] = uint32_t(ts0);
      meta[5] = uint32_t(ts1);
      meta[6] = uint32_t(ts2);
      meta[7] = uint32_t(ts3);
    }
    __threadfence_system();
    if (tid == 0) __hip_atomic_store(&meta[2], seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Funnel shift: bytes [sh, sh + 4) of the 8-B value hi:lo.
DEV uint32_t align_word(uint32_t hi, uint32_t lo, uint32_t sh) {
  return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

// Copy of a verified read's next bytes.  Thread u of the grid (strided when
// the call has more units than threads) takes unit u: the 16-B aligned
// destination block D of piece i = the first with uend[i] > u (the piece
// table is staged in LDS).  A whole unit reads the dword-aligned window
// around its 16 source bytes and funnel-shifts it into place (packet payloads
// sit at any byte offset of the wire stream), one dwordx4 store; the piece's
// first and last unit go byte by byte.  Consecutive lanes take consecutive
// units: loads and stores coalesce.  Stores are sc1 (written through the
// XCD's L2 to memory, so no L2 write-back is needed for another XCD or a
// later kernel to read them); every wave waits for its stores, and after the
// workgroup barrier one lane counts the workgroup done (agent atomic); the
// last one resets the counter and publishes the sequence number to the host
// (one pinned word: no stream synchronisation).
DEV void store16_sc1(uint8_t *p, u32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
DEV void store8_sc1(uint8_t *p, uint32_t v) {
  asm volatile("global_store_byte %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}

// One unit: the 16-B destination block at D of a piece [d, e) whose byte d
// comes from src.
DEV void copy_unit(const uint8_t *src, uintptr_t d, uintptr_t e, uintptr_t D) {
  if (D >= d && D + 16u <= e) {
    const uintptr_t sa = reinterpret_cast<uintptr_t>(src) + (D - d);
    const uint32_t sh = uint32_t(sa & 3u);
    const uint8_t *a0 = reinterpret_cast<const uint8_t *>(sa - sh);
    uint32_t w[5];
#pragma unroll
    for (int k = 0; k < 4; k++) w[k] = gload32(a0 + 4 * k);
    w[4] = sh ? gload32(a0 + 16) : 0u;  // only when it holds one of the bytes
    u32x4 v;
    v.x = align_word(w[1], w[0], sh);
    v.y = align_word(w[2], w[1], sh);
    v.z = align_word(w[3], w[2], sh);
    v.w = align_word(w[4], w[3], sh);
    store16_sc1(reinterpret_cast<uint8_t *>(D), v);
  } else {
    const uintptr_t x0 = D > d ? D : d, x1 = D + 16u < e ? D + 16u : e;
    for (uintptr_t x = x0; x < x1; x++) store8_sc1(reinterpret_cast<uint8_t *>(x), gload8(src + (x - d)));
  }
}

// The staged piece (0 .. cnt - 1) that holds unit u: luend[k] = the first
// unit of staged piece k, luend[cnt] the end of the last.
DEV uint32_t staged_piece(const uint32_t *luend, uint32_t cnt, uint32_t u) {
  uint32_t lo = 0, hi = cnt - 1u;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (luend[mid + 1u] > u) hi = mid; else lo = mid + 1u;
  }
  return lo;
}

// A unit's loads (the issue half) and its store (the other half).
struct CopyLd {
  uint32_t w[5], sh, pk, mode;  // mode 0: none, 1: whole 16 B, 2: byte by byte at the store
  uintptr_t D;
};

DEV void copy_issue(CopyLd &x, const uint8_t *const *lsrc, const uintptr_t *ldst, const uintptr_t *lend,
                    const uint32_t *luend, uint32_t cnt, uint32_t u, uint32_t uend) {
  x.mode = 0u;
  if (u >= uend) return;
  const uint32_t p = staged_piece(luend, cnt, u);
  const uintptr_t d = ldst[p], e = lend[p];
  x.pk = p;
  x.D = (d & ~uintptr_t(15)) + 16u * uintptr_t(u - luend[p]);
  x.mode = (x.D >= d && x.D + 16u <= e) ? 1u : 2u;
  if (x.mode == 1u) {
    const uintptr_t sa = reinterpret_cast<uintptr_t>(lsrc[p]) + (x.D - d);
    x.sh = uint32_t(sa & 3u);
    const uint8_t *a0 = reinterpret_cast<const uint8_t *>(sa - x.sh);
#pragma unroll
    for (int q = 0; q < 4; q++) x.w[q] = gload32(a0 + 4 * q);
    x.w[4] = x.sh ? gload32(a0 + 16) : 0u;  // only when it holds one of the bytes
  }
}

DEV void copy_finish(const CopyLd &x, const uint8_t *const *lsrc, const uintptr_t *ldst, const uintptr_t *lend) {
  if (x.mode == 1u) {
    u32x4 v;
    v.x = align_word(x.w[1], x.w[0], x.sh);
    v.y = align_word(x.w[2], x.w[1], x.sh);
    v.z = align_word(x.w[3], x.w[2], x.sh);
    v.w = align_word(x.w[4], x.w[3], x.sh);
    store16_sc1(reinterpret_cast<uint8_t *>(x.D), v);
  } else if (x.mode == 2u) {
    copy_unit(lsrc[x.pk], ldst[x.pk], lend[x.pk], x.D);
  }
}

// Units ucur, ucur + step, ... < uend of the staged pieces, U per thread at
// a time and software-pipelined: the next U units' loads are issued before
// this U's stores, so a lane has up to 2U x 16 B in flight and the loads
// never wait behind the write-through stores' acknowledgements (one in-order
// counter covers both on gfx950).
template <int U = 4>
DEV void copy_staged(const uint8_t *const *lsrc, const uintptr_t *ldst, const uintptr_t *lend, const uint32_t *luend,
                     uint32_t cnt, uint32_t ucur, uint32_t uend, uint32_t step) {
  CopyLd cur[U], nxt[U];
#pragma unroll
  for (int k = 0; k < U; k++) copy_issue(cur[k], lsrc, ldst, lend, luend, cnt, ucur + uint32_t(k) * step, uend);
  for (uint32_t ub = ucur; ub < uend; ub += uint32_t(U) * step) {
#pragma unroll
    for (int k = 0; k < U; k++)
      copy_issue(nxt[k], lsrc, ldst, lend, luend, cnt, ub + uint32_t(U + k) * step, uend);
#pragma unroll
    for (int k = 0; k < U; k++) copy_finish(cur[k], lsrc, ldst, lend);
#pragma unroll
    for (int k = 0; k < U; k++) cur[k] = nxt[k];
  }
}

// Resident "mailbox" variant of small_chunks_kernel (opt-in,
// hdfs_crc32c_mailbox_create): ONE workgroup stays on one CU and serves the
// synchronous small calls (_hdfs_crc32c and aliases, verify_crcdata,
// compose_crcs on <= 64 KiB, src/datanode.c:2470-2476 is the per-packet call
// pattern) without a kernel launch per call.  The host writes the caller's
// bytes to the input stage and then a 16-B request {seq, len, cs | flags,
// reg0}; the stage is fine-grained VRAM the host writes through the BAR
// (large-BAR devices) or pinned host memory.  Wave 0 polls the request line
// (system-coherent loads), the block reads the data with coalesced
// system-coherent 1 KiB loads, and lane L of wave w ends up with bytes
// [4096 w + 64 L, +64) (the tiled kernel's load order + permlane transpose).
// Each lane runs 16 conflict-free slicing steps on the 32x replicated tables
// and moves its state to the end of its chunk with ONE GF(2) multiply by
// x^(8 dd) mod P (VALU, no table levels).  Results go to the same pinned
// output block as small_chunks_kernel, its completion sequence number last.
// Requests must have chunk_size % 64 == 0 or a single chunk (else the host
// launches small_chunks_kernel).  Exit: a quit request, idle_ticks (100 MHz
// s_memrealtime) without a request, or another packet written to the
// kernel's own hardware queue (below) -- every wave leaves through the same
// barrier-synchronised test; status[0] = (epoch << 1) | alive.
// Yield: a persistent kernel holds up every packet queued behind it on its
// hardware queue, and the runtime shares a process's queues among its
// streams (at most GPU_MAX_HW_QUEUES per priority level: a host process with
// that many high-priority streams of its own shares one with the mailbox's;
// tools/mb_queue_share.py measured such a stream's work waiting the whole
// 50 ms idle exit).  While idle, wave 0 also polls the write index of the
// AQL queue it was dispatched from (amd_queue_t.write_dispatch_id, through
// the queue pointer the CP passes in SGPRs): once anything is written behind
// it, the kernel leaves as on an idle exit, and the next call relaunches it
// behind that work.
constexpr unsigned kAqlWriteIdOff = 56;  // offsetof(amd_queue_t, write_dispatch_id) (hsa/amd_hsa_queue.h)
DEV uint64_t aql_write_index() {
  const char *q = (const char *)(unsigned long long)(__builtin_amdgcn_queue_ptr());
  return *(const volatile uint64_t *)(q + kAqlWriteIdOff);  // system-coherent (sc0 sc1)
}

DEV u32x4 sysload16(const __amdgpu_buffer_rsrc_t r, uint32_t off) {
  // sc0 sc1: system-coherent, never served from a stale cache line
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 17));
}

// Replicated slicing-by-4 image of one table set (the tiled kernel's layout:
// word P*16384 + e*64 + h*32 + l = t_{3-(2P+h)}[e] for every lane slot l),
// filled by all 1024 threads with 16-B stores.
DEV void fill_slices(uint32_t *lt, const uint32_t *__restrict__ gtab, uint32_t tid) {
  constexpr uint32_t kPer = kLdsSliceBytes / 16 / 1024;
  uint32_t v[kPer];
#pragma unroll
  for (uint32_t k = 0; k < kPer; k++) {
    const uint32_t idx = 4u * (k * 1024u + tid);
    const uint32_t P = idx >> 14, e = (idx >> 6) & 255u, h = (idx >> 5) & 1u;
    v[k] = gtab[(3u - (2u * P + h)) * 256u + e];
  }
#pragma unroll
  for (uint32_t k = 0; k < kPer; k++)
    *reinterpret_cast<u32x4 *>(&lt[4u * (k * 1024u + tid)]) = u32x4{v[k], v[k], v[k], v[k]};
}

// Z_64, Z_128, Z_256 byte tables (the main blob's Z_{64k}, k = 1, 2, 4) for
// the mailbox's in-wave combine tree.
DEV void fill_ztree(uint32_t *zt, const uint32_t *__restrict__ gtab, uint32_t tid) {
#pragma unroll
  for (uint32_t s = 0; s < 3; s++) zt[s * 1024u + tid] = gtab[kTabSliceWords + ((1u << s) - 1u) * 1024u + tid];
}

// A copy request served by the mailbox: n CopyEntry records at the start of
// the input stage (read system-coherent: the host wrote them just before the
// request line) staged in LDS, then every unit by the block's 1 024 threads,
// write-through stores as copy_pieces_kernel's; returns once every wave's
// stores are acknowledged.
DEV void mb_copy(const __amdgpu_buffer_rsrc_t rin, uint32_t n, uint32_t *lds, uint32_t tid) {
  auto *lsrc = reinterpret_cast<const uint8_t **>(lds);
  auto *ldst = reinterpret_cast<uintptr_t *>(lds + 2u * kCopyPiecesMax);
  auto *lend = reinterpret_cast<uintptr_t *>(lds + 4u * kCopyPiecesMax);
  uint32_t *luend = lds + 6u * kCopyPiecesMax;
  if (tid < n) {
    uint32_t w[6];
#pragma unroll
    for (uint32_t q = 0; q < 6; q++) w[q] = __builtin_amdgcn_raw_buffer_load_b32(rin, 24u * tid + 4u * q, 0, 17);
    const uintptr_t src = (uintptr_t(w[1]) << 32) | w[0], dst = (uintptr_t(w[3]) << 32) | w[2];
    lsrc[tid] = reinterpret_cast<const uint8_t *>(src);
    ldst[tid] = dst;
    lend[tid] = dst + w[4];
    luend[tid + 1u] = w[5];
  }
  if (tid == 0) luend[0] = 0u;
  __syncthreads();
  copy_staged<2>(lsrc, ldst, lend, luend, n, tid, luend[n], 1024u);  // (the CRC path's registers: no spills)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

__global__ __launch_bounds__(1024) void mailbox_kernel(const uint32_t *__restrict__ req, const uint8_t *__restrict__ in,
                                                       uint32_t *__restrict__ meta, uint32_t *__restrict__ crcs,
                                                       const uint32_t *__restrict__ tab0, const uint32_t *__restrict__ tab1,
                                                       const uint32_t *__restrict__ kxg, uint32_t *__restrict__ status,
                                                       uint32_t epoch, uint32_t seq0, uint32_t idle_ticks,
                                                       uint32_t exp) {
  // exp (diagnostic build, timing experiments only -- wrong results): bit 0
  // skips the GF(2) multiplies, bit 1 the slicing steps, bit 2 the lane XOR
  if (!kDiag) exp = 0u;
  // slicing tables of the current checksum type, replicated 32x (lane l reads
  // bank l, as in the tiled kernel); a request of the other type refills them
  __shared__ __attribute__((aligned(16))) uint32_t lt[kLdsSliceBytes / 4];
  __shared__ uint32_t kx[2 * kTabKxWords];
  __shared__ uint32_t zt[3 * 1024];                 // Z_64, Z_128, Z_256 of the current type
  __shared__ uint32_t slot[2 * (kSmallMax / 512)];  // tree mode: 512-B group partials {crc, j | m << 16}
  __shared__ __attribute__((aligned(16))) uint32_t acc[kSmallMaxChunks];  // (a copy request: its staged pieces)
  __shared__ uint32_t res[2];
  __shared__ uint32_t ctl[6];
  __shared__ uint32_t tailacc;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
  const uint32_t lb0 = (lane & 31u) * 4u, lb1 = 65536u + (lane & 31u) * 4u;
  fill_slices(lt, tab0, tid);
  fill_ztree(zt, tab0, tid);
  for (uint32_t k = tid; k < 2u * kTabKxWords; k += 1024u) kx[k] = kxg[k];
  uint32_t cur = 0u;
  const __amdgpu_buffer_rsrc_t rin =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(in), 0, static_cast<int>(kSmallMax + 4u * kSmallMaxChunks),
                                        0x00020000);
  // tiled-kernel load order for one 4 KiB round of 8 x 512 B (see issue())
  const uint32_t hsel = (lane >> 3) & 1u, loff = 16u * (4u * (lane & 7u) + (lane >> 4));
  uint32_t last = seq0;
  uint64_t t_idle = __builtin_amdgcn_s_memrealtime();
  const uint64_t qw0 = tid == 0 ? aql_write_index() : 0u;  // the queue's write index at our start
  for (;;) {
    if (tid == 0) {
      u32x4 v;
      for (uint32_t spin = 0;; spin++) {
        // volatile: a plain (or buffer-intrinsic) load is hoisted out of the
        // loop by the compiler, which then spins on a stale value; volatile
        // global loads are also system-coherent (sc0 sc1) on gfx950
        v = *(const volatile GAS u32x4 *)(const GAS uint8_t *)req;
        if (v.x != last) break;
        if (__builtin_amdgcn_s_memrealtime() - t_idle > idle_ticks || ((spin & 15u) == 15u && aql_write_index() != qw0)) {
          v = u32x4{last, 0u, kMbQuitFlag, 0u};  // idle, or work queued behind us: leave
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      ctl[0] = v.x;
      ctl[1] = v.y;
      ctl[2] = v.z;
      ctl[3] = v.w;
      if (v.z & kMbDevFlag) {  // device-memory source: its address follows the request line
        const uint64_t p = *(const volatile GAS uint64_t *)(const GAS uint8_t *)(req + 4);
        ctl[4] = uint32_t(p);
        ctl[5] = uint32_t(p >> 32);
      }
      res[0] = 0xFFFFFFFFu;
      res[1] = 0u;
      tailacc = 0u;
    }
#ifdef HDFS_CRC32C_DIAG
    const uint64_t ts0 = __builtin_amdgcn_s_memrealtime();  // request seen
#endif
    __syncthreads();
    // the request words are the same in every lane (LDS): readfirstlane lets
    // the compiler see them uniform -- scalar branches, and descriptors in
    // SGPRs instead of waterfall loops
    const uint32_t seq = rfl(ctl[0]), len = rfl(ctl[1]), csf = rfl(ctl[2]), reg0 = rfl(ctl[3]);
    const bool dev = (csf & kMbDevFlag) != 0u;
    if (csf & kMbQuitFlag) break;  // uniform: every wave leaves here
    if (csf & kMbCopyFlag) {       // uniform: a reader's delivery, len = pieces
      mb_copy(rin, len, acc, tid);
      if (tid == 0) *(volatile GAS u32x4 *)(GAS uint8_t *)meta = u32x4{0xFFFFFFFFu, 0u, seq, 0u};
      last = seq;
      t_idle = __builtin_amdgcn_s_memrealtime();
      __syncthreads();  // the stage in acc is rewritten by the next request
      continue;
    }
    const uint32_t cs = csf & 0x1FFFFu, ct = (csf & kMbCrc32Flag) ? 1u : 0u;
    const bool verify = (csf & kMbVerifyFlag) != 0u, be = (csf & kMbBeFlag) != 0u;
    const uint32_t nch = (len + cs - 1u) / cs;
    if (ct != cur) {  // uniform
      fill_slices(lt, ct ? tab1 : tab0, tid);
      fill_ztree(zt, ct ? tab1 : tab0, tid);
      cur = ct;
    }
    for (uint32_t j = tid; j < nch; j += 1024u) acc[j] = 0u;
    // every load before any compute: one round trip
    uint32_t d[16] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
    const uint32_t base = 4096u * w;
    // device source: exactly len bytes in range (a 16-B load that crosses
    // the end returns zeros, so that piece is read byte by byte); host
    // stage: the whole stage (bytes past len never enter a CRC)
    const __amdgpu_buffer_rsrc_t rd =
        dev ? __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<uint8_t *>((uint64_t(rfl(ctl[5])) << 32) | rfl(ctl[4])),
                                                0, static_cast<int>(len), 0x00020000)
            : rin;
    if (base < len) {
#pragma unroll
      for (uint32_t k = 0; k < 4; k++) {
        const uint32_t p = base + (2u * k + hsel) * 512u + loff;
        u32x4 x = sysload16(rd, p);
        if (dev && p < len && p + 16u > len) {
          uint32_t wd[4] = {0u, 0u, 0u, 0u};
          for (uint32_t b = p; b < len; b++)
            wd[(b - p) >> 2] |= uint32_t(__builtin_amdgcn_raw_buffer_load_b8(rd, b, 0, 17)) << (8u * (b & 3u));
          x = u32x4{wd[0], wd[1], wd[2], wd[3]};
        }
        d[4 * k + 0] = x.x;
        d[4 * k + 1] = x.y;
        d[4 * k + 2] = x.z;
        d[4 * k + 3] = x.w;
      }
    }
    uint32_t ev[2] = {0u, 0u};
    if (verify) {
#pragma unroll
      for (uint32_t k = 0; k < 2; k++)
        if (k * 1024u + tid < nch)
          ev[k] = __builtin_amdgcn_raw_buffer_load_b32(rin, kSmallMax + 4u * (k * 1024u + tid), 0, 17);
    }
    __syncthreads();  // acc cleared, tables of this type in place
#ifdef HDFS_CRC32C_DIAG
    // wave 0's loads landed (the barrier above does not wait for them)
    if (w == 0) __builtin_amdgcn_s_waitcnt(0);
    const uint64_t ts1 = __builtin_amdgcn_s_memrealtime();
#endif
    // Tree mode (uniform): len a multiple of 512 and 8 | lanes per chunk, so
    // every aligned 8-lane group holds 512 whole bytes of one chunk.  Three
    // in-wave levels (shuffle + one Z_{64 2^s} table step) leave each group's
    // CRC at the group end; a group not at its chunk's end is moved there by
    // one GF(2) multiply in a second phase (at most 128 groups, two waves),
    // instead of one multiply per lane.  Otherwise every lane multiplies.
    const uint32_t lpc = cs >> 6, np = len >> 6;
    const uint32_t poly = ct ? 0xedb88320u : 0x82f63b78u;
    const bool tree = (len & 511u) == 0u && (nch == 1u || (lpc & 7u) == 0u);
    const bool tree2 = tree && (nch == 1u ? np > 8u : lpc > 8u);
    if (base < len) {  // uniform per wave
      transpose(d);
      const uint32_t b0 = 64u * (64u * w + lane);  // this lane's piece
      const uint32_t j = b0 / cs;
      uint32_t c = 0u, ctl_ = 0u;  // contribution to acc[j] / to tailacc
      if (b0 < len) {
        const uint32_t ce = min((j + 1u) * cs, len), n = min(64u, ce - b0);
        c = (b0 == j * cs) ? reg0 : 0u;
        if (kDiag && (exp & 2u)) {
          c ^= d[0] ^ d[15];
        } else if (n == 64u) {
          uint32_t x = c ^ d[0];
#pragma unroll
          for (uint32_t q = 0; q < 15; q++) x = slice4(lt, x, d[q + 1], lb0, lb1);
          c = slice4(lt, x, 0u, lb0, lb1);
        } else {  // the last piece of a chunk
#pragma unroll
          for (uint32_t q = 0; q < 16; q++)
            if (4u * q + 4u <= n) c = slice4(lt, c ^ d[q], 0u, lb0, lb1);
          if (n & 3u) {
            uint32_t tw = 0u;
#pragma unroll
            for (uint32_t q = 0; q < 16; q++) tw = (q == (n >> 2)) ? d[q] : tw;
            for (uint32_t b = 0; b < (n & 3u); b++)  // byte table t0: pair 1, half 1
              c = lds_at(lt, lb1 + 128u + (((c ^ (tw >> (8u * b))) & 0xffu) << 8)) ^ (c >> 8);
          }
        }
        if (!tree) {
          // Bytes of the chunk after this piece: dd = 64 m + r.  r = ce mod 64
          // is the same for every full piece of a chunk and non-zero only in
          // the final chunk of a length that is not a multiple of 64: those
          // pieces gather in tailacc, shifted by x^(8r) once below.
          const uint32_t dd = ce - b0 - n, m = dd >> 6;
          if (m && !(kDiag && (exp & 1u))) c = gf2_mulmod(kx[ct * kTabKxWords + m], c, poly);
          if (dd & 63u) {
            ctl_ = c;
            c = 0u;
          }
        }
      }
      if (tree) {
#pragma unroll
        for (uint32_t sl = 0; sl < 3; sl++) {  // the left block moves past its right neighbour
          const uint32_t r = __shfl_xor(c, 1u << sl);
          const uint32_t z = zshift(zt, sl * 1024u, c) ^ r;
          c = (lane & (1u << sl)) ? c : z;
        }
        if ((lane & 7u) == 0u && b0 < len) {
          if (tree2) {
            const uint32_t ce = min((j + 1u) * cs, len), gid = b0 >> 9;
            slot[2u * gid] = c;
            slot[2u * gid + 1u] = j | (((ce - b0 - 512u) >> 6) << 16);
          } else if (c) {
            atomicXor(&acc[j], c);  // the group is its whole chunk
          }
        }
      } else {
        // XOR the lanes of one chunk together before the LDS atomic: groups
        // of g aligned lanes lie in one chunk (g = the lanes per chunk's
        // lowest set bit, 64 for a single chunk)
        const uint32_t g = (kDiag && (exp & 4u)) ? 1u : nch == 1u ? 64u : min(64u, lpc & (0u - lpc));
        const bool tail = (len & 63u) != 0u;  // uniform
#pragma unroll
        for (uint32_t sh = 1; sh < 64u; sh <<= 1) {
          if (sh < g) {
            c ^= __shfl_xor(c, sh);
            if (tail) ctl_ ^= __shfl_xor(ctl_, sh);
          }
        }
        if ((lane & (g - 1u)) == 0u && b0 < len) {
          if (c) atomicXor(&acc[j], c);
          if (ctl_) atomicXor(&tailacc, ctl_);
        }
      }
    }
    __syncthreads();
    if (tree2) {  // uniform: group partials to their chunk ends
      if (tid < (np >> 3)) {
        uint32_t v = slot[2u * tid];
        const uint32_t jm = slot[2u * tid + 1u], mg = jm >> 16;
        if (mg && !(kDiag && (exp & 1u))) v = gf2_mulmod(kx[ct * kTabKxWords + mg], v, poly);
        if (v) atomicXor(&acc[jm & 0xFFFFu], v);
      }
      __syncthreads();
    }
    if (len & 63u) {  // uniform
      if (tid == 0 && tailacc)
        acc[nch - 1u] ^= gf2_mulmod(kx[ct * kTabKxWords + 1024u + (len & 63u)], tailacc, poly);
      __syncthreads();
    }
    if (verify) {
#pragma unroll
      for (uint32_t k = 0; k < 2; k++) {
        const uint32_t j = k * 1024u + tid;
        if (j < nch && (be ? __builtin_bswap32(ev[k]) : ev[k]) != ~acc[j]) {
          atomicMin(&res[0], j);
          atomicAdd(&res[1], 1u);
        }
      }
      __syncthreads();
    }
    // Completion: {first bad, mismatches, seq, CRC of a single chunk} as ONE
    // 16-B system-scope store, so verify and single-chunk calls need no
    // fence round trip; multi-chunk CRC arrays go first, then one fence.
    if (w == 0) {
      const bool one = verify || nch == 1u;
      if (!one) {
        for (uint32_t j = lane; j < nch; j += 64u) {
          const uint32_t v = ~acc[j];
          crcs[j] = be ? __builtin_bswap32(v) : v;
        }
        __threadfence_system();
      }
      if (lane == 0) {
        const uint32_t v0 = ~acc[0];
#ifdef HDFS_CRC32C_DIAG
        // diagnostic phase stamps (10 ns ticks): request seen, wave 0's data
        // loaded, results ready; posted ahead of the completion store
        const uint64_t ts2 = __builtin_amdgcn_s_memrealtime();
        *(volatile GAS u32x4 *)(GAS uint8_t *)(meta + 4) =
            u32x4{uint32_t(ts0), uint32_t(ts1), uint32_t(ts2), uint32_t(ts2 - ts0)};
#endif
        *(volatile GAS u32x4 *)(GAS uint8_t *)meta = u32x4{res[0], res[1], seq, be ? __builtin_bswap32(v0) : v0};
      }
    }
    last = seq;
    t_idle = __builtin_amdgcn_s_memrealtime();
    __syncthreads();  // ctl / res / acc are rewritten by the next request
  }
  if (tid == 0) {
    __threadfence_system();
    __hip_atomic_store(&status[0], epoch << 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

hipError_t launch_mailbox(const uint32_t *req, const uint8_t *in, uint32_t *meta, uint32_t *crcs, const uint32_t *tab0,
                          const uint32_t *tab1, const uint32_t *kx, uint32_t *status, uint32_t epoch, uint32_t seq0,
                          uint32_t idle_ticks, uint32_t exp, hipStream_t stream) {
  hipLaunchKernelGGL(mailbox_kernel, dim3(1), dim3(1024), 0, stream, req, in, meta, crcs, tab0, tab1, kx, status, epoch,
                     seq0, idle_ticks, exp);
  return hipGetLastError();
}

// Composite CRC of whole segments from their chunk CRCs (no data re-read):
// c(A||B) = Z_|B|(c(A)) ^ c(B), so c(seg) = XOR_i Z_{bytes after chunk i}(c_i).
// One thread folds a run of kCompRun chunks sequentially
// (acc = Z_{len_i}(acc) ^ c_i, one table application per chunk for
// power-of-two chunk sizes), then shifts its partial past the rest of the
// segment; partials XOR-reduce per wave (or per lane when a wave straddles
// two segments) into out[seg].
constexpr uint32_t kCompRun = 64;

__global__ __launch_bounds__(256) void composite_kernel(const SegDev *__restrict__ segs, uint32_t nseg,
                                                         const uint64_t *__restrict__ run_prefix,
                                                         uint64_t total_runs, const uint32_t *__restrict__ pow2,
                                                         uint32_t *__restrict__ out) {
  const uint64_t r = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  uint32_t s = 0, v = 0;
  if (r < total_runs) {
    uint32_t lo = 0, hi = nseg - 1;  // last segment with run_prefix <= r
    while (lo < hi) {
      const uint32_t mid = (lo + hi + 1) >> 1;
      if (run_prefix[mid] <= r) lo = mid; else hi = mid - 1;
    }
    s = lo;
    const SegDev sg = segs[s];
    const uint64_t j = r - run_prefix[s];
    const uint64_t c0 = j * kCompRun, c1 = min(c0 + kCompRun, static_cast<uint64_t>(sg.nchunks));
    uint32_t acc = 0;
    for (uint64_t i = c0; i < c1; i++) {
      const uint64_t l = min(static_cast<uint64_t>(sg.chunk_size), sg.len - i * sg.chunk_size);
      uint32_t c = sg.crcs[i];
      if (sg.flags & kSegBigEndian) c = __builtin_bswap32(c);
      acc = zapply(pow2, acc, l) ^ c;
    }
    const uint64_t end = min(c1 * sg.chunk_size, sg.len);
    v = zapply(pow2, acc, sg.len - end);
  }
  const uint32_t s0 = __builtin_amdgcn_readfirstlane(s);
  if (__all(s == s0)) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v ^= __shfl_xor(v, off);
    if ((threadIdx.x & 63u) == 0 && v) atomicXor(out + s0, v);
  } else if (v) {
    atomicXor(out + s, v);
  }
}

// Per-launch reset of the verify results and the pool counter in one launch
// (instead of up to three hipMemsetAsync fills).
__global__ __launch_bounds__(256) void prep_kernel(uint32_t *__restrict__ fb, uint32_t nfb,
                                                    unsigned long long *__restrict__ mism,
                                                    uint32_t *__restrict__ gctr) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (fb && i < nfb) fb[i] = 0xFFFFFFFFu;
  if (i == 0) {
    if (mism) *mism = 0ull;
    if (gctr) *gctr = 0u;
  }
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

// De-framing gather for the packet-stream verifier: one workgroup per
// 64 KiB slice of one packet's data.  Packet payloads sit at arbitrary byte
// offsets of the wire stream (header 25 or 6+hlen bytes, then 4 B per chunk),
// so each lane reads the dword-aligned window around its 16 output bytes and
// funnel-shifts it into place (v_alignbyte_b32); stores are 16-B aligned.
// The slice also moves its share of the packet's BE CRC words.

__global__ __launch_bounds__(256) void packet_gather_kernel(const uint8_t *__restrict__ raw,
                                                             const PktDesc *__restrict__ descs, uint32_t npk,
                                                             uint8_t *__restrict__ arena,
                                                             uint8_t *__restrict__ crc_arena) {
  const uint32_t u = blockIdx.x;
  uint32_t lo = 0, hi = npk - 1;  // last packet with unit0 <= u
  while (lo < hi) {
    const uint32_t mid = (lo + hi + 1) >> 1;
    if (descs[mid].unit0 <= u) lo = mid; else hi = mid - 1;
  }
  const PktDesc d = descs[lo];
  const uint32_t s = u - d.unit0;
  const uint8_t *src = raw + d.src_crc + 4ull * d.ncrc;
  uint8_t *dst = arena + d.dst_data;
  const uint64_t b0 = uint64_t(s) * kGatherSlice;
  const uint64_t b1 = min(uint64_t(d.dlen), b0 + kGatherSlice);
  for (uint64_t o = b0 + 16ull * threadIdx.x; o < b1; o += 16ull * blockDim.x) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(src + o);
    const uint32_t sh = uint32_t(a & 3);
    const uint8_t *a0 = reinterpret_cast<const uint8_t *>(a - sh);
    uint32_t w[5];
#pragma unroll
    for (int i = 0; i < 5; i++) w[i] = gload32(a0 + 4 * i);
    u32x4 v;
    v.x = align_word(w[1], w[0], sh);
    v.y = align_word(w[2], w[1], sh);
    v.z = align_word(w[3], w[2], sh);
    v.w = align_word(w[4], w[3], sh);
    *(GAS u32x4 *)(GAS uint8_t *)(dst + o) = v;
  }
  // CRC words [s*q, (s+1)*q) of this packet, q = ceil(ncrc / nunits)
  const uint32_t q = (d.ncrc + d.nunits - 1) / d.nunits;
  const uint32_t w1 = min(d.ncrc, (s + 1) * q);
  const uint8_t *csrc = raw + d.src_crc;
  uint8_t *cdst = crc_arena + d.dst_crc;
  for (uint32_t w = s * q + threadIdx.x; w < w1; w += blockDim.x) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(csrc + 4ull * w);
    const uint32_t sh = uint32_t(a & 3);
    const uint8_t *a0 = reinterpret_cast<const uint8_t *>(a - sh);
    gstore32(cdst + 4ull * w, align_word(gload32(a0 + 4), gload32(a0), sh));
  }
}

// ---------------------------------------------------------------------------
// Device framing of device-resident packet streams.  The reference's walk is
// sequential (packet k+1 starts where packet k's plen puts it,
// src/datanode.c:2345-2446), but the packets of a block transfer all have
// the same wire size, so thread k frames the packet at base + k * stride
// (stride = the wire size of the packet at base) with the host walk's own
// frame_step (crc32c_frame.h) and the first grid point that is not a
// complete, framing-clean packet of exactly that size ends the run.  The
// scan kernel turns the run into a verify segment table in HBM (the host
// never sees the headers), and the host continues from where the run left
// the grid.
// Per-packet share of the run's segment table (classify() rules of
// crc32c_engine.cpp: tiled kernel for chunk sizes that are multiples of 512,
// a partial last chunk moves the last tile to the generic kernel).
struct GridContrib {
  uint32_t nseg, rounds, mtiles, gtiles, bm, payload;
};

DEV GridContrib grid_contrib(const hdfs_crc32c_packet &r, uint32_t cs, int verify, int rwin, int64_t client_offset) {
  GridContrib a{0u, 0u, 0u, 0u, 0u, 0u};
  if (r.error) return a;
  uint32_t cb = 0;
  a.payload = frame::read_avail(r, rwin != 0, client_offset, cb);  // bytes the packet can deliver
  if (!verify || r.crc_len <= 0) return a;
  const uint32_t nch = uint32_t(r.crc_len) / 4u, ntiles = (nch + 7u) / 8u;
  const bool eligible = cs % kRoundBytes == 0;
  const bool partial = uint32_t(r.data_len) % cs != 0;
  const uint32_t main = eligible ? (partial ? ntiles - 1u : ntiles) : 0u;
  a.nseg = 1u;
  a.rounds = main * (cs / kRoundBytes);
  a.mtiles = main;
  a.gtiles = ntiles - main;
  a.bm = ntiles;
  return a;
}

// Wire size of the packet at base from its first six bytes (header_len +
// plen - 4, 0 if not positive; src/datanode.c:2428 with the v1 / v2 header
// length): the grid of a device framing pass.  The six byte loads go out
// together through a buffer descriptor whose range ends with the stream
// (bytes past it read 0) -- no per-byte bounds test, so no load waits for
// the one before it.
DEV uint64_t grid_stride(const uint8_t *s, uint64_t len, uint64_t base, int proto) {
  const uint64_t rem = base < len ? len - base : 0;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t *>(s + (base < len ? base : 0)), 0, static_cast<int>(rem < 8 ? rem : 8), 0x00020000);
  uint32_t b[6];
#pragma unroll
  for (int i = 0; i < 6; i++) b[i] = __builtin_amdgcn_raw_buffer_load_b8(r, i, 0, 0);
  const int32_t plen = int32_t((b[0] << 24) | (b[1] << 16) | (b[2] << 8) | b[3]);
  const int64_t hl = proto == HDFS_CRC32C_PROTO_V2 ? 6 + int64_t((b[4] << 8) | b[5]) : 25;
  const int64_t tot = hl + int64_t(plen) - 4;
  return tot > 0 ? uint64_t(tot) : 0;
}

// A packet's first kHdrWin bytes, staged in LDS with four 16-B loads, so
// frame_step's byte reads hit LDS instead of making ~30 dependent trips to
// memory.  Only when the whole window lies inside the stream (a packet
// within kHdrWin bytes of the stream end is framed from memory directly).
// (Buffer loads: they serve any byte address; a global_load_dwordx4 at an
// address that is not 4-B aligned returns the aligned-down bytes.)
// The packet sits at ub + voff: ub wave-uniform (the descriptor's base, in
// SGPRs), voff per lane.  A descriptor built from a per-lane address is a
// waterfall loop -- one pass per distinct lane address, and the compiler
// waited for each of the four loads before issuing the next: four
// dependent HBM round trips, 12.8 of a 1 GiB framing pass's 31 us
// (tools/frame_phases.py); now the four loads of every lane go out together.
DEV void stage_header(const uint8_t *s, uint64_t len, uint64_t ub, uint32_t voff, uint8_t *win) {
  const uint64_t pos = ub + voff;
  const uint64_t span = len > ub ? len - ub : 0;
  const uint32_t nrec = span > 0xFFFFFFFFull ? 0xFFFFFFFFu : static_cast<uint32_t>(span);
  // readfirstlane: the fields are uniform, and the compiler must see it (a
  // descriptor it takes for divergent is a waterfall loop again)
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<uint8_t *>(rfl64(reinterpret_cast<uint64_t>(s + ub))), 0, static_cast<int>(rfl(nrec)), 0x00020000);
  if (pos > len || len - pos < kHdrWin) return;
  u32x4 v[kHdrWin / 16];
#pragma unroll
  for (int k = 0; k < int(kHdrWin / 16); k++)
    v[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff + 16u * k, 0, 0));
#pragma unroll
  for (int k = 0; k < int(kHdrWin / 16); k++) *reinterpret_cast<u32x4 *>(win + 16 * k) = v[k];
}

// frame_step on the staged header when it holds the whole header, on the
// stream itself near the stream end or when a v2 header is longer than the
// window.
DEV int grid_frame(const uint8_t *s, uint64_t len, uint64_t pos, const uint8_t *win, int proto, uint32_t cs,
                   int ctype, hdfs_crc32c_packet &r, uint64_t &total) {
  const uint64_t rem = len - pos;
  const bool fits = rem >= kHdrWin && (proto == HDFS_CRC32C_PROTO_V1 ||
                                       6u + ((uint32_t(win[4]) << 8) | win[5]) <= kHdrWin);
  // two calls, not one on a selected pointer: each inlined copy then knows
  // its address space (ds_read_u8 from the staged window instead of flat
  // loads, which wait on both the LDS and the vector-memory counters)
  if (fits) return frame::frame_step(win, rem, pos, proto, cs, ctype, r, total);
  return frame::frame_step(s + pos, rem, pos, proto, cs, ctype, r, total);
}

// 64 threads (one wave) per block: a pass of 16 K packets spreads over all
// 256 CUs (the per-thread decode is a latency chain, so occupancy per CU
// matters less than CUs engaged)
constexpr uint32_t kGridBlock = 64;

// One device framing pass in one launch: frame the grid points, then a
// single-pass scan of their shares of the segment table over the blocks
// (each block publishes its own sums at once; the sums before it are the
// records of its group of 64 blocks before it plus the totals of the
// earlier groups, which each group's last block publishes: two levels, no
// chain), then
// the verify segment entries of the run's packets, the run's summary and,
// from the last block to finish, the host copy.  Block b only waits for
// blocks < b, which the dispatcher started before it, so the wait ends.
// (A decoupled look-back -- windows of 64 predecessors back to the nearest
// published inclusive prefix -- chained 4 windows deep for a 1 GiB run:
// look-back done at 22 us median, tools/frame_phases.py.)
// Aggregate record of one block; flag = (pass seq << 2) | 1 once agg / mins
// are out.  Tagging with the pass's sequence number means no reset between
// passes (the area is zeroed once when it is allocated; seqs start at 1).
// Every field is written and read with agent-scope relaxed atomics
// (write-through stores, loads past this XCD's L2) and a record's flag is
// stored only after its fields' stores are acknowledged (s_waitcnt
// vmcnt(0)): no L2 write-back or invalidate per publish -- with an
// agent-scope fence per publish and per look-back window the pass took
// 62 us instead of ~35.
struct GridLook {
  uint64_t agg[6];   // the block's shares of the recorded packets' table
  uint64_t mins;     // first grid point of the block that is not On (~0: none)
  uint64_t flag;
  uint64_t rec0[7];  // block 0 only: packet 0's record (the prediction of the others)
  uint64_t T;        // block 0 only: main tiles of packet 0's segment (the uniform layout's tiles per segment)
  uint64_t pad[16];
};
static_assert(sizeof(GridLook) == kGridLookBytes, "look-back record");
static_assert(sizeof(hdfs_crc32c_packet) == 7 * 8, "packet 0's record in the look-back area");

DEV uint64_t at_ld(const uint64_t *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
DEV void at_st(uint64_t *p, uint64_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
DEV void at_st32(uint32_t *p, uint32_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
// every store of this wave acknowledged (write-through stores: at the point
// of coherence) before the next one
DEV void stores_done() { __builtin_amdgcn_s_waitcnt(0x0F70); }  // s_waitcnt vmcnt(0)

__global__ __launch_bounds__(kGridBlock) void frame_build_kernel(
    const uint8_t *__restrict__ s, uint64_t len, uint64_t base, uint32_t count, int proto, uint32_t cs, int ctype,
    int verify, uint32_t sflags, uint8_t *__restrict__ bm_base, uint8_t *__restrict__ copy_base, uint64_t copy_cap,
    int rwin, int64_t client_offset, hdfs_crc32c_packet *__restrict__ recs, GridLook *__restrict__ look,
    SegDev *__restrict__ segs, uint32_t *__restrict__ seg2pkt, uint32_t *__restrict__ fb, uint32_t *__restrict__ gctr,
    uint32_t *__restrict__ done, uint32_t *__restrict__ exc, GridSummary *__restrict__ sum, uint8_t *__restrict__ hsum,
    uint32_t seq, unsigned long long *__restrict__ stamps) {
  static_assert(kGridBlock == 64, "one wave per block: the scans are wave-wide");
  // diagnostic build: s_memrealtime (100 MHz) per block at the end of each
  // phase -> stamps[8 b + phase] (tools/frame_phases.py)
  auto stamp = [&](uint32_t ph) {
    if (kDiag && stamps && threadIdx.x == 0) stamps[8u * blockIdx.x + ph] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  static_assert(sizeof(hdfs_crc32c_packet) == kGridRecBytes, "host record layout");
  __shared__ __attribute__((aligned(16))) uint8_t win[kGridBlock][kHdrWin];
  __shared__ uint32_t islast;
  const uint32_t t = threadIdx.x, b = blockIdx.x, k = b * kGridBlock + t, lane = t;
  const uint32_t nblk = gridDim.x;
  const uint64_t tag = uint64_t(seq) << 2;
  // 1. frame this thread's grid point.  The stride comes from the first 6
  // bytes of the packet at base: header_len + plen - 4 is exactly the wire
  // size frame_step gives a complete, clean packet, so no thread decodes
  // packet 0's PacketHeaderProto just to find the grid.  If packet 0 is not
  // such a packet its status ends the run (first_break = 0).
  const uint64_t stride = rfl64(grid_stride(s, len, base, proto));  // one value in every lane
  // Grid points past the stream's end are kGridMore, so the run ends at the
  // latest at k0 = ceil((len - base) / stride), the first point at or past
  // the end: the pass acts on points [0, ceff), ceff = k0 + 1 (1 without a
  // grid), which decides exactly what the whole count would.  Blocks past
  // ceff only count themselves done -- a pass is sized before the host knows
  // the stride (up to kGridMaxCount points: 1 024 blocks for a 1 GiB run of
  // 16 384 packets), and without this the look-back chain ran through every
  // block (16 windows deep instead of 4).
  const uint32_t ceff =
      stride ? static_cast<uint32_t>(min<uint64_t>(count, (len - base + stride - 1) / stride + 1)) : 1u;
  if (b * kGridBlock >= ceff) {
    // block 0 resets the counters before its flag: wait for it before counting
    if (lane == 0)
      for (uint32_t spins = 0; (at_ld(&look[0].flag) >> 2) != uint64_t(seq);) {
        if (++spins > (1u << 24)) {  // never expected: fail loudly, see the gather
          asm volatile("s_trap 2");
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
  } else {
  hdfs_crc32c_packet r{};
  uint64_t total = 0;
  uint32_t code = kGridMore;
  GridContrib a{0u, 0u, 0u, 0u, 0u, 0u};
  if (k < ceff && (k == 0 || stride)) {
    const uint64_t pos = base + uint64_t(k) * stride;
    if (pos < len) {
      // the block's headers through one descriptor at its first point when
      // the block's points lie within 2^32 bytes of it (strides < 64 MiB)
      if (stride < (1ull << 26)) stage_header(s, len, base + uint64_t(b) * kGridBlock * stride, t * uint32_t(stride), win[t]);
      else stage_header(s, len, pos, 0u, win[t]);
      const int st = grid_frame(s, len, pos, win[t], proto, cs, ctype, r, total);
      code = st == frame::kStepMore ? kGridMore
           : st == frame::kStepStop ? kGridStop
           : total == stride        ? kGridOn
                                    : kGridOff;
      // a recorded clean packet's bytes lie inside the stream (the verify
      // segments built from its record read them), the pass inside its buffers
      if (code != kGridMore &&
          DCHK(r.error || r.stream_off + r.header_len + uint64_t(r.crc_len) + uint64_t(r.data_len) <= len,
               kDkFrameGrid) &&
          DCHK(count <= kGridMaxCount, kDkFrameGrid)) {
        recs[k] = r;
        a = grid_contrib(r, cs, verify, rwin, client_offset);
      }
    }
  }
  stamp(1);
  const uint32_t mk = (k < ceff && code != kGridOn) ? k : 0xFFFFFFFFu;
  // 2. the block's aggregate: shares of its grid points (a point past the
  // run's end is excluded later, where the end is known) and its first point
  // that is not On
  uint64_t v[6] = {a.nseg, a.rounds, a.mtiles, a.gtiles, a.bm, a.payload};
  uint32_t m = mk;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
#pragma unroll
    for (int q = 0; q < 6; q++) v[q] += __shfl_xor(v[q], off);
    m = min(m, static_cast<uint32_t>(__shfl_xor(static_cast<int>(m), off)));
  }
  // Block 0 also publishes packet 0's record and resets the pass's counters
  // before its flag: every other block waits for block 0's flag before it
  // touches them.
  if (lane == 0) {
    GridLook &L = look[b];
#pragma unroll
    for (int q = 0; q < 6; q++) at_st(&L.agg[q], v[q]);
    at_st(&L.mins, uint64_t(m) | 0xFFFFFFFF00000000ull);
    if (b == 0) {
      const uint64_t *x = reinterpret_cast<const uint64_t *>(&r);
#pragma unroll
      for (int q = 0; q < 7; q++) at_st(&L.rec0[q], x[q]);
      at_st(&L.T, a.nseg ? a.mtiles : 0u);
      at_st32(&sum->unaligned, 0u);
      at_st32(&sum->nonuni, 0u);
      at_st32(&done[0], 0u);  // blocks finished
      at_st32(&done[1], 0u);  // exceptions found
      sum->stride = stride;
    }
    stores_done();
    at_st(&L.flag, tag | 1u);
  }
  stamp(2);
  // 3. the shares and first break of blocks 0..b-1, in two levels with no
  // chain between them: (a) lane l < i reads block 64 g + l of this block's
  // group of 64 (g = b / 64, i = b % 64); (c) the group's last block then
  // publishes the group's total (its 64 aggregates) at once; (b) lane h < g
  // reads the total of group h.  A block waits for at most 63 block records
  // and 15 group records, each lane's flag loads issued together, then its
  // field loads: O(64 + B / 64) records per block for B blocks.  Block 0's
  // flag is seen through (a) or through group 0's total (published after
  // its last block saw block 0's flag; every record is acknowledged at the
  // point of coherence before its flag): its record and counter resets are
  // out before this block uses them.
  uint64_t pre[6] = {0, 0, 0, 0, 0, 0};
  uint32_t pmin = 0xFFFFFFFFu;
  // packet 0's record and T (the prediction step 4 checks against): block
  // 0's own lane 0, or loaded by lane 0 once block 0 is known to be out (one
  // request per block on block 0's record, not one per use)
  uint64_t r0w[7];
  uint64_t T64 = a.nseg ? a.mtiles : 0u;
  {
    const uint64_t *x = reinterpret_cast<const uint64_t *>(&r);
#pragma unroll
    for (int q = 0; q < 7; q++) r0w[q] = x[q];
  }
  const uint32_t gi = b / 64u, ii = b % 64u;
  GridLook *const grp = look + kGridMaxCount / kGridBlock;  // kGridGroups group records
  auto wait_flag = [&](const GridLook *rec, bool want) {
    for (uint32_t spins = 0;;) {
      const bool out = !want || at_ld(&rec->flag) == (tag | 1u);
      if (__ballot(!out) == 0ull) break;
      if (++spins > (1u << 24)) {  // never expected (blocks < b run to their publish): fail loudly, see the gather
        asm volatile("s_trap 2");
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  };
  if (ii > 0) {  // (a)
    const GridLook *rec = &look[gi * 64u + lane];
    wait_flag(rec, lane < ii);
    if (lane < ii) {
#pragma unroll
      for (int f = 0; f < 6; f++) pre[f] = at_ld(&rec->agg[f]);
      pmin = static_cast<uint32_t>(at_ld(&rec->mins));
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
#pragma unroll
      for (int f = 0; f < 6; f++) pre[f] += __shfl_xor(pre[f], off);
      pmin = min(pmin, static_cast<uint32_t>(__shfl_xor(static_cast<int>(pmin), off)));
    }
  }
  if (ii == 63u && (uint64_t(b) + 1u) * kGridBlock < ceff && lane == 0) {  // (c) a later block needs it
    GridLook &G = grp[gi];
#pragma unroll
    for (int f = 0; f < 6; f++) at_st(&G.agg[f], pre[f] + v[f]);
    at_st(&G.mins, uint64_t(min(pmin, m)) | 0xFFFFFFFF00000000ull);
    stores_done();
    at_st(&G.flag, tag | 1u);
  }
  if (gi > 0) {  // (b)
    const GridLook *rec = &grp[lane];
    wait_flag(rec, lane < gi);
    uint64_t x[6] = {0, 0, 0, 0, 0, 0};
    uint32_t xm = 0xFFFFFFFFu;
    if (lane < gi) {
#pragma unroll
      for (int f = 0; f < 6; f++) x[f] = at_ld(&rec->agg[f]);
      xm = static_cast<uint32_t>(at_ld(&rec->mins));
    }
    if (lane == 0) {  // (group 0's total is out: so is block 0)
#pragma unroll
      for (int q = 0; q < 7; q++) r0w[q] = at_ld(&look[0].rec0[q]);
      T64 = at_ld(&look[0].T);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
#pragma unroll
      for (int f = 0; f < 6; f++) x[f] += __shfl_xor(x[f], off);
      xm = min(xm, static_cast<uint32_t>(__shfl_xor(static_cast<int>(xm), off)));
    }
#pragma unroll
    for (int f = 0; f < 6; f++) pre[f] += x[f];
    pmin = min(pmin, xm);
  } else if (b > 0 && lane == 0) {  // group 0: block 0 was seen in (a)
#pragma unroll
    for (int q = 0; q < 7; q++) r0w[q] = at_ld(&look[0].rec0[q]);
    T64 = at_ld(&look[0].T);
  }
  stamp(3);
  // 4. the run's end as this block sees it: the first point that is not On
  // (before this block: the block is past the run; in it; or none up to
  // here).  A point is recorded if it lies before the end, or is the end and
  // was framed (Off / Stop).
  const uint32_t fbk = min(min(pmin, m), ceff);
  const bool past = pmin != 0xFFFFFFFFu;
  const bool inrun = !past && (k < fbk || (k == fbk && k < ceff && code != kGridMore));
#pragma unroll
  for (int q = 0; q < 7; q++) r0w[q] = static_cast<uint64_t>(__shfl(static_cast<long long>(r0w[q]), 0));
  const uint32_t T = static_cast<uint32_t>(__shfl(static_cast<long long>(T64), 0));
  if (!past) {
    // in-block exclusive scan of the recorded points' shares
    const uint64_t own[6] = {inrun ? a.nseg : 0u, inrun ? a.rounds : 0u, inrun ? a.mtiles : 0u,
                             inrun ? a.gtiles : 0u, inrun ? a.bm : 0u, inrun ? uint64_t(a.payload) : 0u};
    uint64_t incl[6] = {own[0], own[1], own[2], own[3], own[4], own[5]};
#pragma unroll
    for (int q = 0; q < 6; q++) {
#pragma unroll
      for (uint32_t off = 1; off < 64; off <<= 1) {
        const uint64_t o = __shfl_up(incl[q], off);
        if (lane >= off) incl[q] += o;
      }
    }
    uint64_t ex[6];
#pragma unroll
    for (int q = 0; q < 6; q++) ex[q] = pre[q] + incl[q] - own[q];
    // the segment entry of a recorded packet with CRCs
    if (inrun && a.nseg) {
      const uint32_t nch = uint32_t(r.crc_len) / 4u, ntiles = (nch + 7u) / 8u;
      const uint32_t sg = static_cast<uint32_t>(ex[0]);
      const uint8_t *crcp = s + r.stream_off + r.header_len;
      SegDev d;
      d.data = crcp + r.crc_len;
      d.crcs = reinterpret_cast<uint32_t *>(const_cast<uint8_t *>(crcp));
      d.bitmap = bm_base + ex[4];
      d.mtile_start = ex[2];
      d.chunk_size = cs;
      d.flags = sflags;
      d.nchunks = nch;
      d.main_tiles = a.mtiles;
      d.reg_init = 0xFFFFFFFFu;
      d.gen_tiles = ntiles - a.mtiles;
      d.len = uint64_t(r.data_len);
      d.round_start = ex[1];
      d.gtile_start = ex[3];
      // copy-out: the packet's delivered bytes [c_begin, c_begin + len) at
      // their place in the destination, never past it (copy_cap: what is
      // left of the read, or of the buffer, at this pass)
      uint32_t cb = 0, clen = 0;
      uint64_t at = 0;
      (void)frame::read_avail(r, rwin != 0, client_offset, cb);
      frame::read_place(ex[5], static_cast<uint32_t>(own[5]), copy_cap, at, clen);
      d.copy_dst = copy_base && clen ? copy_base + at : nullptr;
      d.copy_w0 = cb;
      d.copy_w1 = cb + clen;
      // one entry per recorded packet at most; a copy window inside the
      // packet's data and its destination inside the read's
      if (DCHK(sg <= k, kDkGridBuild) &&
          DCHK(!clen || (uint64_t(cb) + clen <= uint64_t(r.data_len) && at + clen <= copy_cap), kDkGridBuild)) {
        segs[sg] = d;
        seg2pkt[sg] = k;
        fb[sg] = 0xFFFFFFFFu;
      }
    }
    // one atomic per wave that has a byte-unaligned tiled segment / a segment
    // off the uniform layout (per-thread atomics on one word serialise)
    {
      const bool una = inrun && a.nseg && a.mtiles &&
                       ((reinterpret_cast<uintptr_t>(s) + r.stream_off + r.header_len + uint32_t(r.crc_len)) & 3u);
      if (__ballot(una) && lane == 0) atomicOr(&sum->unaligned, 1u);
      const bool off_layout = inrun && a.nseg && (ex[2] != ex[0] * T || a.mtiles > T);
      if (__ballot(off_layout) && lane == 0) atomicOr(&sum->nonuni, 1u);
    }
    // records that differ from the prediction from packet 0 (wave-aggregated slots)
    {
      bool diff = false;
      if (k >= 1 && inrun) {
        hdfs_crc32c_packet p;
        uint64_t *px = reinterpret_cast<uint64_t *>(&p);
#pragma unroll
        for (int q = 0; q < 7; q++) px[q] = r0w[q];
        p.stream_off = base + uint64_t(k) * stride;
        p.offset_in_block += int64_t(k) * p.data_len;
        p.seqno += int64_t(k);
        const uint64_t *x = reinterpret_cast<const uint64_t *>(&p), *y = reinterpret_cast<const uint64_t *>(&r);
#pragma unroll
        for (int q = 0; q < int(kGridRecBytes / 8); q++) diff |= x[q] != y[q];
      }
      const uint64_t bal = __ballot(diff);
      uint32_t at = 0;
      if (lane == 0 && bal) at = atomicAdd(&done[1], static_cast<uint32_t>(__builtin_popcountll(bal)));
      at = static_cast<uint32_t>(__shfl(static_cast<int>(at), 0));
      const uint32_t ix = at + static_cast<uint32_t>(__builtin_popcountll(bal & ((1ull << lane) - 1ull)));
      if (diff && DCHK(ix < count, kDkGridBuild)) exc[ix] = k;
    }
    // the summary, from the thread at the run's end (the break point, or the
    // pass's last point when every point is On): the table's totals are this
    // block's prefix plus its recorded points
    uint64_t tot[6];
#pragma unroll
    for (int q = 0; q < 6; q++) tot[q] = pre[q] + static_cast<uint64_t>(__shfl(static_cast<long long>(incl[q]), 63));
    if (fbk < ceff ? k == fbk : k == ceff - 1u) {
      uint64_t consumed, next;
      uint32_t recorded, st_fb;
      if (fbk == ceff) {  // only when ceff == count (else point ceff - 1 is past the stream: a break)
        consumed = next = base + uint64_t(ceff) * stride;
        recorded = ceff;
        st_fb = kGridOn;
      } else if (code == kGridMore) {
        consumed = next = base + uint64_t(fbk) * stride;
        recorded = fbk;
        st_fb = code;
      } else {
        next = r.stream_off + r.header_len + uint64_t(r.crc_len) + uint64_t(r.data_len);
        consumed = r.error ? base + uint64_t(fbk) * stride : next;
        recorded = fbk + 1u;
        st_fb = code;
      }
      sum->first_break = fbk;
      sum->recorded = recorded;
      sum->last_status = st_fb;
      sum->nseg = static_cast<uint32_t>(tot[0]);
      sum->rounds = tot[1];
      sum->mtiles = tot[2];
      sum->gtiles = tot[3];
      sum->bm_bytes = tot[4];
      sum->payload = tot[5];
      sum->consumed = consumed;
      sum->next_pos = next;
      sum->nbad = 0;
      *gctr = 0u;    // the verify launch's pool counter (no separate reset launch)
    }
  }
  }  // active block
  stamp(4);
  // 5. the last block to finish publishes the summary, packet 0's record and
  // the exceptions to pinned host memory, then (one system-scope fence later)
  // the sequence number the host polls.  The barrier makes every wave's
  // stores complete (workgroup release: they are in this XCD's L2); ONE
  // agent-scope fence then writes the L2 back for the other XCDs before the
  // block counts itself done (not one fence per thread).
  __syncthreads();
  if (t == 0) {
    __threadfence();
    islast = atomicAdd(&done[0], 1u) == nblk - 1u ? 1u : 0u;
  }
  __syncthreads();
  stamp(5);
  if (!islast) return;
  __threadfence();  // acquire: the other blocks' summary fields, flags and exception slots
  const uint32_t nexc = done[1];
  if (t == 0) {
    sum->nexc = nexc;
    const uint32_t T = static_cast<uint32_t>(at_ld(&look[0].T));
    sum->utiles = (sum->nonuni || (sum->mtiles >> 32)) ? 0u : T;  // read by the verify kernel
    GridSummary h = *sum;
    h.seq = 0u;
    *reinterpret_cast<GridSummary *>(hsum) = h;
    const uint64_t *x = reinterpret_cast<const uint64_t *>(&recs[0]);
    uint64_t *y = reinterpret_cast<uint64_t *>(hsum + kGridHostRec0);
    for (int q = 0; q < int(kGridRecBytes / 8); q++) y[q] = x[q];
  }
  for (uint32_t j = t; j < min(nexc, kExcMax); j += kGridBlock) {
    const uint32_t i = exc[j];
    reinterpret_cast<uint32_t *>(hsum + kGridHostIdx)[j] = i;
    const uint64_t *x = reinterpret_cast<const uint64_t *>(&recs[i]);
    uint64_t *y = reinterpret_cast<uint64_t *>(hsum + kGridHostExc + size_t(j) * kGridRecBytes);
    for (int q = 0; q < int(kGridRecBytes / 8); q++) y[q] = x[q];
  }
  __threadfence_system();
  __syncthreads();
  if (t == 0)
    __hip_atomic_store(&reinterpret_cast<GridSummary *>(hsum)->seq, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  stamp(6);
}

// After verify: every segment with a bad chunk -> one compact GridBad entry
// (packet index, first bad chunk, number of bad chunks from its bitmap).
// One workgroup, so it can publish without a cross-block protocol: the
// first host_cap entries and the count go straight to pinned host memory
// (hsum2: a GridSummary whose nbad / seq fields are written, then the list),
// every entry to the device list; one system fence, then the sequence
// number the host polls -- no copy launch behind the verify kernel.
__global__ __launch_bounds__(1024) void grid_finalize_kernel(const SegDev *__restrict__ segs, uint32_t nseg,
                                                             const uint32_t *__restrict__ seg2pkt,
                                                             const uint32_t *__restrict__ fb,
                                                             GridBad *__restrict__ bad, uint32_t bad_cap,
                                                             GridSummary *__restrict__ sum, uint8_t *__restrict__ hsum2,
                                                             uint32_t host_cap, uint32_t seq) {
  __shared__ uint32_t nb;
  if (nseg == 0xFFFFFFFFu) nseg = sum->nseg;  // launched before the host knows the run's size
  if (!DCHK(nseg <= bad_cap, kDkFinalize)) nseg = bad_cap;  // one segment per packet of the pass
  bad_list<1024>(segs, nseg, seg2pkt, fb, bad, bad_cap, sum, hsum2, host_cap, seq, &nb);
}

// ---------------------------------------------------------------------------
// Speculative one-launch verify of a device-resident packet run (round 4).
// The device framing chain (frame_build_kernel -> verify -> finalize) pays
// ~21 + 7 us of dependent global round trips per pass before and after the
// verify; a block transfer is a run of equal packets, so this kernel takes
// the run's layout from packet 0 alone (every workgroup decodes it in its
// prologue, beside the LDS table fill), verifies it through the closed-form
// table (SpecTab), and checks the headers on the side: packet k must carry
// packet 0's header bytes but for offsetInBlock = off0 + k * dataLen and
// seqno = seq0 + k -- then frame_step gives it exactly the record predicted
// from packet 0, as frame_build_kernel would.  One differing header raises
// SpecCtl::exc and the host frames the run the regular way (the launch's
// results are discarded; its copy-out stayed inside the destination).
// crc32c_internal.h (SpecCtl) has the control-word ring.
// Positions of offsetInBlock / seqno in a canonical header: v1 big-endian at
// 4 / 12 (src/datanode.c:2363-2384); v2 little-endian sfixed64 at 7 / 16 of
// [plen][hlen][PacketHeaderProto] in protobuf-c's field order (decode_header's
// fast path).
DEV bool spec_canonical(const uint8_t *w, int proto, uint32_t hl) {
  if (proto == HDFS_CRC32C_PROTO_V1) return hl == 25u;
  const uint32_t n = hl - 6u;
  const uint8_t *p = w + 6;
  return (n == 25u || n == 27u) && p[0] == 0x09 && p[9] == 0x11 && p[18] == 0x18 && p[19] < 0x80 && p[20] == 0x25 &&
         (n == 25u || (p[25] == 0x28 && p[26] < 0x80));
}

// Header byte j (a compile-time constant after unrolling) of packet k of the
// run: packet 0's byte b0 but inside the offsetInBlock / seqno fields.
template <uint32_t J>
DEV uint32_t spec_hdr_byte(uint32_t b0, bool v1, uint64_t off, uint64_t sq) {
  uint32_t e1 = b0, e2 = b0;
  if constexpr (J >= 4 && J < 12) e1 = static_cast<uint32_t>(off >> (8 * (11 - J))) & 0xffu;
  if constexpr (J >= 12 && J < 20) e1 = static_cast<uint32_t>(sq >> (8 * (19 - J))) & 0xffu;
  if constexpr (J >= 7 && J < 15) e2 = static_cast<uint32_t>(off >> (8 * (J - 7))) & 0xffu;
  if constexpr (J >= 16 && J < 24) e2 = static_cast<uint32_t>(sq >> (8 * (J - 16))) & 0xffu;
  return v1 ? e1 : e2;
}

template <uint32_t D>
DEV uint32_t spec_hdr_word(const uint8_t *w0, bool v1, uint64_t off, uint64_t sq) {
  return spec_hdr_byte<4 * D>(w0[4 * D], v1, off, sq) | (spec_hdr_byte<4 * D + 1>(w0[4 * D + 1], v1, off, sq) << 8) |
         (spec_hdr_byte<4 * D + 2>(w0[4 * D + 2], v1, off, sq) << 16) |
         (spec_hdr_byte<4 * D + 3>(w0[4 * D + 3], v1, off, sq) << 24);
}

// The run a speculative launch takes, decoded from packet 0 (LDS, shared by
// the workgroup's waves).
struct SpecRun {
  uint32_t eligible, count, hl, crc_len, dlen, nch, T, cb0, v1;
  uint64_t stride, off0, seq0;
};

constexpr uint32_t kSpecHdrBytes = 48;  // header bytes compared per packet (canonical headers: <= 33)

template <int COPY, int BATCH>
__global__ __launch_bounds__(1024) void spec_verify_kernel(SpecArgs a) {
  static_assert(!(COPY && BATCH), "a batch is verify only");
  __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsWords + 2 + 2 * kSlots];
  // packet 0 of run r in win[r]; after the decode win[r + 1] takes the point
  // after run r (the tails: win[0] stays the header template)
  __shared__ __attribute__((aligned(16))) uint8_t win[kSpecRunsMax + 1][kHdrWin];
  __shared__ SpecRun run;
  __shared__ uint64_t run_r0[kSpecRunsMax][7];  // each run's packet 0 record, for the early blocks
  __shared__ uint64_t run_total;
  // run r: packets at rS[r] + rP[r] + k * stride, k < rcount[r], records'
  // stream_off relative to rS[r] (run 0: the call's stream and base)
  __shared__ const uint8_t *rS[kSpecRunsMax];
  __shared__ uint64_t rN[kSpecRunsMax], rP[kSpecRunsMax], roff0[kSpecRunsMax], rseq0[kSpecRunsMax];
  __shared__ uint32_t rcount[kSpecRunsMax], rprefix[kSpecRunsMax + 1], gprefix[kSpecRunsMax + 1];
  // what the epilogue needs, parked in LDS: kept in SGPRs across the work
  // loop they pushed it past the SGPR budget (spills)
  __shared__ SpecCtl *ep_ctl;
  __shared__ SpecExc *ep_exc;
  __shared__ uint8_t *ep_hout;
  __shared__ SpecRunTail *ep_xtail;
  __shared__ uint32_t ep_seq, ep_nruns;
  __shared__ uint32_t ecnt[kEarlyWords];  // BATCH: per-run completion (SpecTabT::e)
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  // diagnostic build: phase stamps of this workgroup (0 entry, 1 tables +
  // packet 0 decoded + closed-form table written, 2 work loop entered, 3
  // header checks done, 4 the last workgroup's final block published)
  unsigned long long *const ps = kDiag && a.stamps ? a.stamps + kSpecStampOff + 8u * blockIdx.x : nullptr;
  auto stamp = [&](int ph) {
    if (kDiag && ps && t == 0) ps[ph] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  const uint32_t nruns = !BATCH || a.nruns < 1u ? 1u : (a.nruns > kSpecRunsMax ? kSpecRunsMax : a.nruns);
  if (t == 0) {
    ep_ctl = a.ctl + a.parity;
    ep_exc = a.exc + a.parity * kSpecExcMax;
    ep_hout = a.hout;
    ep_xtail = a.xtail ? a.xtail + a.parity * kSpecRunsMax : nullptr;
    ep_seq = a.seq;
    ep_nruns = nruns;
  }
  SpecCtl *const ctl = a.ctl + a.parity;
  const uint64_t rem = a.len > a.base ? a.len - a.base : 0u;
  // run r's stream, length and packet 0 position (per lane: a select over
  // the argument slots, no dynamic index into the kernel arguments)
  auto run_of = [&](uint32_t r, const uint8_t *&S, uint64_t &N, uint64_t &P) {
    S = a.s;
    N = a.len;
    P = rem ? a.base : 0u;
#pragma unroll
    for (uint32_t i = 1; i < kSpecRunsMax; i++)
      if (r == i) {
        S = a.xs[i];
        N = a.xlen[i];
        P = 0u;
      }
  };
  if (wv == 0) {
    // packet 0's first kHdrWin bytes of each run (zeros past its stream) ->
    // win[r]: lane 4 r + q loads bytes [16 q, 16 q + 16) of run r
    const uint32_t r = lane >> 2, q = lane & 3u;
    if (r < nruns) {
      const uint8_t *S;
      uint64_t N, P;
      run_of(r, S, N, P);
      const uint64_t left = N > P ? N - P : 0u;
      if (r == 0) {  // one uniform descriptor: buffer loads clamp at the stream's end
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t *>(a.s + (rem ? a.base : 0u)), 0, static_cast<int>(rem < kHdrWin ? rem : kHdrWin),
            0x00020000);
        *reinterpret_cast<u32x4 *>(&win[0][16 * q]) =
            __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, 16u * q, 0, 0));
      } else {
        uint32_t wd[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (uint32_t i = 0; i < 16; i++)
          if (16u * q + i < left) wd[i / 4] |= uint32_t(S[P + 16u * q + i]) << (8u * (i % 4));
        *reinterpret_cast<u32x4 *>(&win[r][16 * q]) = u32x4{wd[0], wd[1], wd[2], wd[3]};
      }
    }
  }
  fill_tables<1024, 0>(lds, a.gtab);
  if (wv == 0) {
    // The critical path of every workgroup: each run's packet 0 decoded
    // (lane r: run r), the batch's layout checked, and this workgroup's copy
    // of the closed-form table (written with vector stores, acknowledged
    // before the barrier; read back with scalar loads in the work loop).
    // What only the host or the epilogue needs -- the points after the runs,
    // the early blocks, the next launch's control slot -- is left to one
    // wave of workgroup 0 after the barrier.
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");  // the windows' LDS stores, this wave's own
    const uint32_t r = lane;
    SpecRun d{};
    hdfs_crc32c_packet rr{};
    uint64_t total = 0;
    bool ok = false;
    uint32_t count = 0;
    const uint8_t *S = a.s;
    uint64_t N = 0, P = 0;
    if (r < nruns) {
      run_of(r, S, N, P);
      const uint64_t left = N > P ? N - P : 0u;
      const uint32_t hl = a.proto == HDFS_CRC32C_PROTO_V2 ? 6u + ((uint32_t(win[r][4]) << 8) | win[r][5]) : 25u;
      const bool fits = left >= 6u && hl <= kHdrWin;
      const int st = fits ? frame::frame_step(win[r], left, P, a.proto, a.cs, a.ctype, rr, total) : frame::kStepMore;
      uint32_t cb0 = 0;
      const bool rwin = a.rwin != 0 && nruns == 1u;
      const uint32_t avail0 = st == frame::kStepNext ? frame::read_avail(rr, rwin, a.client_offset, cb0) : 0u;
      ok = st == frame::kStepNext && !rr.error && !rr.last && rr.crc_len > 0 && rr.data_len > 0 &&
           a.cs % kRoundBytes == 0 && uint32_t(rr.data_len) % a.cs == 0 && total < kSpecMaxStride &&
           spec_canonical(win[r], a.proto, hl) && avail0 > 0u;
      if (ok) {
        const uint64_t by_len = left / total;
        uint64_t cnt = min<uint64_t>(by_len, a.max_count);
        // a client read takes the packets up to the one that completes it
        if (rwin && a.copy_cap > avail0)
          cnt = min<uint64_t>(cnt, 1u + (a.copy_cap - avail0 + uint64_t(rr.data_len) - 1u) / uint64_t(rr.data_len));
        else if (rwin)
          cnt = 1u;
        count = static_cast<uint32_t>(cnt);
        ok = count >= 2u;
        d.stride = total;
        d.hl = rr.header_len;
        d.crc_len = uint32_t(rr.crc_len);
        d.dlen = uint32_t(rr.data_len);
        d.nch = uint32_t(rr.crc_len) / 4u;
        d.T = (d.nch + kTileChunks - 1u) / kTileChunks;
        d.cb0 = cb0;
        d.v1 = a.proto == HDFS_CRC32C_PROTO_V1 ? 1u : 0u;
        d.off0 = uint64_t(rr.offset_in_block);
        d.seq0 = uint64_t(rr.seqno);
      }
    }
    // the batch takes its layout from run 0; every run must share it
    const uint32_t hl0 = __builtin_amdgcn_readlane(d.hl, 0), cl0 = __builtin_amdgcn_readlane(d.crc_len, 0),
                   dl0 = __builtin_amdgcn_readlane(d.dlen, 0);
    const uint64_t st0 = (uint64_t(__builtin_amdgcn_readlane(static_cast<uint32_t>(total >> 32), 0)) << 32) |
                         __builtin_amdgcn_readlane(static_cast<uint32_t>(total), 0);
    // (and, for a batch, its packet count: the table maps packet k to run k / count)
    const uint32_t cnt0 = __builtin_amdgcn_readlane(count, 0);
    const bool bad = r < nruns && !(ok && d.hl == hl0 && d.crc_len == cl0 && d.dlen == dl0 && total == st0 &&
                                    (nruns == 1u || count == cnt0));
    const bool all_ok = __builtin_amdgcn_ballot_w64(bad) == 0ull;
    // prefixes of the runs' packets and of their 64-packet header groups
    uint32_t pre = 0, tot = 0, gpre = 0, gtot = 0;
#pragma unroll
    for (uint32_t i = 0; i < kSpecRunsMax; i++) {
      const uint32_t ci = __builtin_amdgcn_readlane(count, i);
      if (i < nruns) {
        if (i < r) {
          pre += ci;
          gpre += (ci + 63u) / 64u;
        }
        tot += ci;
        gtot += (ci + 63u) / 64u;
      }
    }
    if (r < nruns) {
      rS[r] = S;
      rN[r] = N;
      rP[r] = P;
      roff0[r] = d.off0;
      rseq0[r] = d.seq0;
      rcount[r] = count;
      rprefix[r] = pre;
      gprefix[r] = gpre;
      const uint64_t *x = reinterpret_cast<const uint64_t *>(&rr);
#pragma unroll
      for (int q = 0; q < 7; q++) run_r0[r][q] = x[q];
    }
    if (r == 0) {
      rprefix[nruns] = tot;
      gprefix[nruns] = gtot;
      d.eligible = all_ok ? 1u : 0u;
      d.count = tot;
      run = d;
      run_total = total;
    }
    if (all_ok) {
      SpecTabData *q = a.tabs + blockIdx.x;
      if (r < nruns) q->crc0r[r] = S + P + d.hl;
      if (r == 0) {
        q->crc0 = S + P + d.hl;
        q->bm0 = a.bm;
        q->copy_base = COPY ? a.copy_base : nullptr;
        q->stride = d.stride;
        q->copy_cap = COPY ? a.copy_cap : 0u;
        q->nch = d.nch;
        q->cs = a.cs;
        q->cb0 = COPY ? d.cb0 : 0u;
        q->nruns = nruns;
        q->per = count;
        q->um = count ? ~0ull / count + 1ull : 0ull;
        q->pad = 0u;
        q->ctl = ctl;
        q->hdone = a.hout + kSpecRunDoneOff;
        q->seq = a.seq;
      }
      stores_done();
    }
    if (BATCH && r < kSpecRunsMax) ecnt[r] = 0u;  // per-run completion: tiles counted per run
    if (BATCH && r == 0) ecnt[49] = 0u;           // (off until every wave has restated the dealing)
  }
  __syncthreads();
  stamp(1);
  // uniform: readfirstlane'd into SGPRs (read from LDS, the compiler would
  // keep them in VGPRs and build every descriptor of the loop from them)
  SpecRun d;
  d.eligible = rfl(run.eligible);
  d.count = rfl(run.count);
  d.hl = rfl(run.hl);
  d.crc_len = rfl(run.crc_len);
  d.dlen = rfl(run.dlen);
  d.nch = rfl(run.nch);
  d.T = rfl(run.T);
  d.cb0 = rfl(run.cb0);
  d.v1 = rfl(run.v1);
  d.stride = rfl64(run.stride);
  d.off0 = rfl64(run.off0);
  d.seq0 = rfl64(run.seq0);
  if (BATCH && d.eligible) {
    // Per-run completion (a coalesced batch, a.early): the tiles this
    // workgroup owns of each run -- tiles_run's schedule 3 dealing restated
    // (static groups of 2^gshift tiles, gfirst + i * gstride; the pool takes
    // tiles from p2first on) -- each run's target, and the runs with pool
    // tiles, which are not published.  Every wave writes the same words
    // (lane r: run r) before its own tiles; tiles_run checks the
    // restatement against the wave's own static tickets (early_ok) before
    // any tile counts.  32-bit: a batch has < 2^31 tiles.
    const uint32_t cnt0 = rfl(rcount[0]);
    const uint32_t per_t = cnt0 * d.T, ntl = per_t * nruns;
    const uint32_t G = gridDim.x, b = blockIdx.x, pmin = (a.tune >> 16) & 0xffu;
    const bool pool = uint64_t(ntl) * (a.cs / kRoundBytes) >= uint64_t(pmin ? pmin : 32u) * G * 16u;
    const uint32_t gsh = (a.tune >> 8) & 15u, xm = (a.tune >> 12) & 3u;
    const uint32_t ng = static_cast<uint32_t>((pool ? uint64_t(ntl) * kPhase1Num / kPhase1Den : ntl) >> gsh);
    uint32_t gf, gst, nkg, p2;
    if (xm == 2u && (G % 8u) == 0 && ng >= 8u * (G / 8u)) {
      const uint32_t ngx = ng / 8u, G8 = G / 8u, l = b / 8u;
      gf = (b % 8u) * ngx + l;
      gst = G8;
      nkg = (ngx - 1u - l) / G8 + 1u;
      p2 = (ngx * 8u) << gsh;
    } else {
      gf = xm != 0u && (G % 8u) == 0 ? (b % 8u) * (G / 8u) + b / 8u : b;
      gst = G;
      nkg = ng > gf ? (ng - 1u - gf) / G + 1u : 0u;
      p2 = ng << gsh;
    }
    auto below = [&](uint32_t x) -> uint32_t {  // this workgroup's static groups under group x
      return x > gf ? min(nkg, (x - gf + gst - 1u) / gst) : 0u;
    };
    const bool on = a.early != 0u && nruns > 1u && (per_t & ((1u << gsh) - 1u)) == 0u &&
                    uint64_t(cnt0) * d.T * nruns < (1ull << 31);
    const uint32_t r = lane;
    uint32_t owned = 0, dis = 1;
    if (r < nruns) {
      owned = (below(((r + 1u) * per_t) >> gsh) - below((r * per_t) >> gsh)) << gsh;
      dis = (r + 1u) * per_t > p2 ? 1u : 0u;
      ecnt[16u + r] = dis ? kEarlyOff : owned;
      ecnt[32u + r] = G + (rcount[r] + 63u) / 64u;
    }
    uint32_t sum = 0;
#pragma unroll
    for (uint32_t i = 0; i < kSpecRunsMax; i++) sum += __builtin_amdgcn_readlane(owned, i);
    if (r == 0) {
      ecnt[48] = sum;
      ecnt[49] = on ? 1u : 0u;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");  // (this wave's reads of them follow)
    // a workgroup that owns none of a run's tiles is done with it now
    if (wv == 0 && on && r < nruns && !dis && owned == 0u)
      spec_run_contribute(ctl, a.hout + kSpecRunDoneOff, a.seq, G + (rcount[r] + 63u) / 64u, r);
  }
  // Workgroup 0, last wave: the next launch's control slot zeroed and the
  // early block to the host (which fills the runs' records while the kernel
  // verifies them); then lane 0 the point after each run (where its walk
  // goes on, or what ends it) into its control slot, one run at a time
  // (stage_header's descriptor is uniform).  This wave joins the work loop
  // after it; the other waves take the workgroup's tiles meanwhile.
  if (blockIdx.x == 0 && wv == 15u) {
    if (lane < nruns && nruns > 1u) {  // the batch's per-run early records
      auto *er = reinterpret_cast<SpecRunEarly *>(a.hout + kSpecRunEarlyOff) + lane;
#pragma unroll
      for (int q = 0; q < 7; q++) er->r0[q] = run_r0[lane][q];
      er->count = rcount[lane];
      er->early = BATCH && ecnt[49] != 0u &&
                          ecnt[16u + lane] != kEarlyOff ? 1u : 0u;
    }
    if (lane < kSpecRunsMax) {
      // the next launch's per-run words start at zero too -- from every
      // kernel of the ring, batch or not: the next launch may be a batch
      SpecCtl *nx = a.ctl + (a.parity ^ 1u);
      nx->run_done[lane] = 0u;
      nx->run_mism[lane] = 0u;
      if (lane == 0) nx->run_bad = 0u;
    }
    if (lane == 0) {
      // the next launch's control slot starts at zero (this launch's was
      // zeroed by the one before)
      SpecCtl *nx = a.ctl + (a.parity ^ 1u);
      nx->mism = 0ull;
      nx->gctr = 0u;
      nx->done = 0u;
      nx->exc = 0u;
      nx->nexc = 0u;
      auto *e = reinterpret_cast<SpecEarly *>(a.hout);
#pragma unroll
      for (int q = 0; q < 7; q++) e->r0[q] = run_r0[0][q];
      e->stride = run_total;
      e->eligible = d.eligible;
      e->count = d.count;
    }
    stores_done();
    __threadfence_system();
    if (lane == 0) __hip_atomic_store(&reinterpret_cast<SpecEarly *>(a.hout)->seq, a.seq, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_SYSTEM);
    for (uint32_t r = 0; lane == 0 && d.eligible && r < nruns; r++) {
      const uint8_t *S = rS[r];
      const uint64_t N = rN[r], P = rP[r], cnt = rcount[r];
      uint32_t ts = kGridOn;
      uint64_t ttot = 0;
      hdfs_crc32c_packet tr{};
      const uint64_t by_len = (N - P) / d.stride;
      // (the caller's record array holds count + 1 records only when the
      // run was not cut at max_count)
      if (cnt == by_len && cnt < a.max_count) {  // the run ends with the stream's whole strides
        const uint64_t pt = P + cnt * d.stride;
        if (pt >= N) {
          ts = kGridMore;
        } else {
          stage_header(S, N, pt, 0u, win[r + 1]);
          const int tst = grid_frame(S, N, pt, win[r + 1], a.proto, a.cs, a.ctype, tr, ttot);
          ts = tst == frame::kStepMore ? kGridMore : tst == frame::kStepStop ? kGridStop : kGridOff;
        }
      }
      const uint64_t *x = reinterpret_cast<const uint64_t *>(&tr);
      if (r == 0) {
#pragma unroll
        for (int q = 0; q < 7; q++) at_st(&ctl->tail[q], x[q]);
        at_st(&ctl->tail_total, ttot);
        at_st32(&ctl->tail_status, ts);
      } else if (a.xtail) {
        SpecRunTail *y = a.xtail + a.parity * kSpecRunsMax + r;
#pragma unroll
        for (int q = 0; q < 7; q++) at_st(&y->rec[q], x[q]);
        at_st(&y->total, ttot);
        at_st32(&y->status, ts);
        at_st32(&y->seq, a.seq);  // (the final block's copy of the entry keeps the host's sequence number)
      }
      if (BATCH && ecnt[49]) {
        // per-run completion: what follows run r in the host area now, for
        // a job that returns before the launch ends
        auto *ht = reinterpret_cast<SpecRunTail *>(a.hout + kSpecRunTailOff) + r;
#pragma unroll
        for (int q = 0; q < 7; q++) ht->rec[q] = x[q];
        ht->total = ttot;
        ht->status = ts;
        __threadfence_system();
        __hip_atomic_store(&ht->seq, a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
  if (!d.eligible) return;
  const bool v1 = d.v1 != 0u;
  // header checks: groups of 64 packets of a run, group g (over the runs in
  // order) on wave (g / G) % 16 of workgroup g % G; lane l compares packet
  // 64 j + l of the group's run (packet 0 of a run is its prediction
  // itself).  A wave's first group is loaded here and compared after the
  // verify loop: its loads ride ahead of the loop's first rounds instead of
  // holding every wave of the workgroup at the barrier for a round trip (a
  // 1 GiB run has one group per workgroup; longer runs load the rest later)
  const uint32_t G = gridDim.x;
  const uint32_t j0 = wv * G + blockIdx.x;
  const uint32_t ngroups = rfl(gprefix[nruns]);
  auto group_run = [&](uint32_t g) {
    uint32_t r = 0;
#pragma unroll
    for (uint32_t i = 1; i < kSpecRunsMax; i++) r += (i < nruns && g >= gprefix[i]) ? 1u : 0u;
    return rfl(r);
  };
  // group g: its run, the group's first packet position in the run's stream
  auto hdr_rsrc = [&](uint32_t r, uint32_t jr) {
    const uint64_t p0 = rfl64(rP[r]) + uint64_t(64u * jr) * d.stride;
    const uint64_t n = rfl64(rN[r]);
    const uint64_t span = n > p0 ? n - p0 : 0u;
    return __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<uint8_t *>(rfl64(reinterpret_cast<uint64_t>(rS[r] + p0))), 0,
        static_cast<int>(rfl(span > 0xFFFFFFFFull ? 0xFFFFFFFFu : static_cast<uint32_t>(span))), 0x00020000);
  };
  const uint32_t vo = lane * static_cast<uint32_t>(d.stride);
  u32x4 h0[kSpecHdrBytes / 16];
  if (j0 < ngroups) {
    const uint32_t r = group_run(j0);
    const __amdgpu_buffer_rsrc_t rs = hdr_rsrc(r, j0 - rfl(gprefix[r]));
#pragma unroll
    for (int q = 0; q < int(kSpecHdrBytes / 16); q++)
      h0[q] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, vo + 16u * q, 0, 0));
  }
  stamp(2);
  // a coalesced batch with per-run completion checks a wave's first header
  // group before its tiles: a run is published only once its headers are
  const bool hdr_first = BATCH && rfl(ecnt[49]) != 0u;
  auto check = [&](uint32_t j, const u32x4 (&h)[kSpecHdrBytes / 16]) {
    const uint32_t r = group_run(j), jr = j - rfl(gprefix[r]);
    const uint64_t p0 = rfl64(rP[r]) + uint64_t(64u * jr) * d.stride;
    const uint32_t kr = 64u * jr + lane;
    const uint32_t cnt_r = rfl(rcount[r]);
    const uint64_t off = rfl64(roff0[r]) + uint64_t(kr) * d.dlen, sq = rfl64(rseq0[r]) + kr;
    uint32_t e[kSpecHdrBytes / 4];
    e[0] = spec_hdr_word<0>(win[0], v1, off, sq);
    e[1] = spec_hdr_word<1>(win[0], v1, off, sq);
    e[2] = spec_hdr_word<2>(win[0], v1, off, sq);
    e[3] = spec_hdr_word<3>(win[0], v1, off, sq);
    e[4] = spec_hdr_word<4>(win[0], v1, off, sq);
    e[5] = spec_hdr_word<5>(win[0], v1, off, sq);
    e[6] = spec_hdr_word<6>(win[0], v1, off, sq);
    e[7] = spec_hdr_word<7>(win[0], v1, off, sq);
    e[8] = spec_hdr_word<8>(win[0], v1, off, sq);
    e[9] = spec_hdr_word<9>(win[0], v1, off, sq);
    e[10] = spec_hdr_word<10>(win[0], v1, off, sq);
    e[11] = spec_hdr_word<11>(win[0], v1, off, sq);
    uint32_t diff = 0;
#pragma unroll
    for (uint32_t w = 0; w < kSpecHdrBytes / 4; w++) {
      // bytes of the header only (hl <= 33)
      const uint32_t m = 4u * w >= d.hl ? 0u : 4u * w + 4u <= d.hl ? 0xFFFFFFFFu : (1u << (8u * (d.hl - 4u * w))) - 1u;
      diff |= (h[w / 4][w % 4] ^ e[w]) & m;
    }
    if (kr < cnt_r && diff != 0u) {
      // rare: frame the packet as frame_build_kernel would.  Clean and in
      // the run's layout -- same header length, dataLen and CRC length, so
      // its CRCs and data sit where the closed-form table puts them (the
      // same wire size alone is not enough: a 27-B syncBlock header with
      // dataLen cut by 2 has packet 0's stride) -- an exception with its own
      // record; anything else voids the launch
      hdfs_crc32c_packet rec{};
      uint64_t tot = 0;
      const uint64_t pos = p0 + vo;
      const uint8_t *S = rS[r];
      const uint64_t N = rfl64(rN[r]);
      const int st = frame::frame_step(S + pos, N - pos, pos, a.proto, a.cs, a.ctype, rec, tot);
      bool keep = st == frame::kStepNext && !rec.error && tot == d.stride && rec.header_len == d.hl &&
                  static_cast<uint32_t>(rec.data_len) == d.dlen && static_cast<uint32_t>(rec.crc_len) == d.crc_len &&
                  (!a.rwin || static_cast<uint64_t>(rec.offset_in_block) == off);
      if (keep) {
        const uint32_t slot = __hip_atomic_fetch_add(&ctl->nexc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (slot < kSpecExcMax) {
          SpecExc *x = a.exc + a.parity * kSpecExcMax + slot;
          const uint64_t *w = reinterpret_cast<const uint64_t *>(&rec);
#pragma unroll
          for (int q = 0; q < 7; q++) at_st(&x->rec[q], w[q]);
          at_st32(&x->k, rfl(rprefix[r]) + kr);  // global packet index over the runs
        } else {
          keep = false;
        }
      }
      if (!keep) __hip_atomic_fetch_or(&ctl->exc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (hdr_first) {
      // the group's part of its run: a header off the prediction marks the
      // run (never published), then the group counts (after the mark)
      if (__ballot(kr < cnt_r && diff != 0u) != 0ull) {  // rare
        if (lane == 0) __hip_atomic_fetch_or(&ctl->run_bad, 1u << r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        stores_done();
      }
      if (lane == 0) spec_run_contribute(ctl, a.hout + kSpecRunDoneOff, a.seq, ecnt[32u + r], r);
    }
  };
  if (hdr_first && j0 < ngroups) check(j0, h0);
  const SpecTabT<BATCH != 0> tab{(const CAS SpecTabData *)(a.tabs + blockIdx.x), ecnt};
  const uint64_t tiles = uint64_t(d.count) * d.T;
  tiles_run<kModeVerify, 3, 1, 3, 1, 1024, 1, COPY, 1, 0>(lds, tab, nullptr, d.count, tiles * (a.cs / kRoundBytes),
                                                          tiles, a.fb, &ctl->mism, kDiag ? a.stamps : nullptr, a.tune,
                                                          &ctl->gctr, nullptr, d.T, false);
  for (uint32_t j = hdr_first ? j0 + 16u * G : j0; j < ngroups; j += 16u * G) {
    u32x4 h[kSpecHdrBytes / 16];
    if (j == j0) {
#pragma unroll
      for (int q = 0; q < int(kSpecHdrBytes / 16); q++) h[q] = h0[q];
    } else {
      const uint32_t r = group_run(j), jr = j - rfl(gprefix[r]);
      const __amdgpu_buffer_rsrc_t rs = hdr_rsrc(r, jr);
#pragma unroll
      for (int q = 0; q < int(kSpecHdrBytes / 16); q++)
        h[q] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, vo + 16u * q, 0, 0));
    }
    check(j, h);
  }
  // every wave's stores and atomics (mismatch count, exception flag) are
  // acknowledged before its workgroup counts itself done; the last
  // workgroup then reads the counters and publishes the final block
  stores_done();
  __syncthreads();
  stamp(3);
  // diagnostic build: every tile this workgroup verified of a published run
  // counted, and the count is the prologue's restatement of what it owns
  // (an owned count too low would publish a run before its last tiles)
  if (kDiag && BATCH && wv == 0 && lane < nruns && ecnt[49] && ecnt[16u + lane] != kEarlyOff)
    (void)DCHK(ecnt[lane] == ecnt[16u + lane], kDkSpecEarly);
  if (t < 64u) {
    // wave 0: lane 0 counts the workgroup done; in the last workgroup the
    // wave copies the counters, exceptions and run tails to the host area one
    // dword per lane -- every load in flight at once instead of a chain of
    // dependent agent-scope round trips (~2.6 us of the block's end) -- and
    // lane 0 publishes the sequence number after the wave's stores
    SpecCtl *const c = ep_ctl;
    uint32_t n = 0;
    if (lane == 0) n = __hip_atomic_fetch_add(&c->done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    n = static_cast<uint32_t>(__shfl(static_cast<int>(n), 0));
    if (n == gridDim.x - 1u) {
      // SpecFinal dword j <- SpecCtl dword: mism 0-1, exc 4, tail_status 5,
      // tail_total 6-7, tail 8-21, nexc 22 (dword 20 is the sequence number)
      static_assert(offsetof(SpecCtl, exc) == 16 && offsetof(SpecCtl, tail_total) == 24 &&
                        offsetof(SpecCtl, tail) == 32 && offsetof(SpecCtl, nexc) == 88 &&
                        offsetof(SpecFinal, exc) == 8 && offsetof(SpecFinal, tail_total) == 16 &&
                        offsetof(SpecFinal, tail) == 24 && offsetof(SpecFinal, seq) == 80 &&
                        offsetof(SpecFinal, nexc) == 84,
                    "the final block's dword map");
      const uint32_t src = lane < 2u ? lane : lane < 20u ? lane + 2u : 22u;
      uint32_t v = 0;
      if (lane < 22u && lane != 20u)
        v = __hip_atomic_load(reinterpret_cast<const uint32_t *>(c) + src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      auto *f = reinterpret_cast<uint32_t *>(ep_hout + sizeof(SpecEarly));
      if (lane < 22u && lane != 20u) f[lane] = v;
      const uint32_t nexc = static_cast<uint32_t>(__shfl(static_cast<int>(v), 21));
      const uint32_t nxd = min(nexc, kSpecExcMax) * uint32_t(sizeof(SpecExc) / 4u);
      const auto *xs = reinterpret_cast<const uint32_t *>(ep_exc);
      auto *xd = reinterpret_cast<uint32_t *>(ep_hout + 256);
      for (uint32_t q = lane; q < nxd; q += 64u)
        xd[q] = __hip_atomic_load(xs + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (ep_xtail) {  // run r >= 1's tail (SpecRunTail r)
        constexpr uint32_t kW = uint32_t(sizeof(SpecRunTail) / 4u);
        const auto *ts = reinterpret_cast<const uint32_t *>(ep_xtail);
        auto *td = reinterpret_cast<uint32_t *>(ep_hout + kSpecRunTailOff);
        for (uint32_t q = kW + lane; q < kW * ep_nruns; q += 64u)
          td[q] = __hip_atomic_load(ts + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __threadfence_system();
      if (lane == 0) __hip_atomic_store(&f[20], ep_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      stamp(4);
    }
  }
}

hipError_t launch_spec_verify(const SpecArgs &a, int grid, int copy, hipStream_t stream) {
  if (grid < 1 || !a.seq || !a.ctl || !a.exc || !a.hout || !a.tabs || a.parity > 1u) return hipErrorInvalidValue;
  if (a.nruns > 1u && (copy || a.rwin || a.nruns > kSpecRunsMax || !a.xtail)) return hipErrorInvalidValue;
  if (a.nruns > 1u) hipLaunchKernelGGL((spec_verify_kernel<0, 1>), dim3(grid), dim3(1024), 0, stream, a);
  else if (copy) hipLaunchKernelGGL((spec_verify_kernel<1, 0>), dim3(grid), dim3(1024), 0, stream, a);
  else hipLaunchKernelGGL((spec_verify_kernel<0, 0>), dim3(grid), dim3(1024), 0, stream, a);
  return hipGetLastError();
}

// Short device-resident runs in one launch (the per-read case of a
// GPU-direct receive: one or a few packets per call).  Workgroup k frames the
// packet at k * stride (stride from packet 0's first bytes, the device
// framing's grid) with the shared frame_step, and -- when it is a clean
// packet with CRCs of <= 64 KiB -- verifies its chunks itself: one 64-B
// piece per thread from HBM, slicing tables and the zeros operators it can
// need in LDS, pieces shifted to their chunk's end and XOR-ed per chunk
// (small_chunks_kernel's algebra).  The last workgroup to finish works out
// the run (first grid point that is not On, as frame_build_kernel) and
// publishes summary, records and verdicts to pinned memory, its sequence
// number last.  A packet it cannot take (more data, too many chunks, a chunk
// size that is not a multiple of 64 with several chunks) is flagged and the
// host takes the regular path.
__global__ __launch_bounds__(1024) void small_run_kernel(const uint8_t *__restrict__ s, uint64_t len, uint32_t count,
                                                         int proto, uint32_t cs, int ctype, int verify,
                                                         const uint32_t *__restrict__ tab,
                                                         const uint32_t *__restrict__ pow2,
                                                         uint8_t *__restrict__ copy_dst, uint64_t copy_cap,
                                                         int rwin, int64_t client_offset,
                                                         uint8_t *__restrict__ hout, uint32_t seq) {
  __shared__ uint32_t tt[1024];
  __shared__ __attribute__((aligned(16))) uint32_t zt[16 * 1024];  // Z_{2^b}, b < 16 (the levels a shift can use)
  __shared__ uint32_t acc[kSmallMaxChunks];
  __shared__ __attribute__((aligned(16))) uint8_t win[kSmallRunMax][kHdrWin];
  __shared__ hdfs_crc32c_packet rec;
  // code, verify this packet, unsupported, first bad, bad chunks, levels,
  // copy-out: destination offset (lo, hi), copy it (every earlier packet On
  // and clean, something to deliver), window [c_begin, c_begin + len)
  __shared__ uint32_t ctl[11];
  __shared__ uint32_t sdl[kSmallRunMax], son[kSmallRunMax];
  const uint32_t tid = threadIdx.x, k = blockIdx.x;
  tt[tid] = tab[tid];
  // Copy-out needs this packet's place in the de-framed payload: thread t
  // frames packet t of the run for t <= k (k + 1 headers in parallel, one
  // round trip) -- every earlier packet must be On and framing-clean, and
  // their data lengths sum to the destination offset.  Without copy-out
  // only thread 0 frames, packet k.
  const uint32_t nfr = copy_dst ? k + 1u : 1u;
  if (tid < nfr && DCHK(nfr <= kSmallRunMax && k < count, kDkSmallRun)) {
    const uint32_t pk = copy_dst ? tid : k;
    const uint64_t stride = grid_stride(s, len, 0, proto);  // the grid, as frame_build_kernel
    hdfs_crc32c_packet r{};
    uint32_t code = kGridMore;
    uint64_t total = 0;
    const uint64_t pos = uint64_t(pk) * stride;
    if ((pk == 0 || stride) && pos < len) {
      stage_header(s, len, 0u, static_cast<uint32_t>(pos), win[tid]);  // pos < len <= kSmallRunBytes
      const int st = grid_frame(s, len, pos, win[tid], proto, cs, ctype, r, total);
      code = st == frame::kStepMore ? kGridMore : st == frame::kStepStop ? kGridStop : total == stride ? kGridOn : kGridOff;
    }
    uint32_t cb = 0;
    sdl[tid] = code != kGridMore ? frame::read_avail(r, rwin != 0, client_offset, cb) : 0u;  // bytes it delivers
    son[tid] = code == kGridOn && !r.error ? 1u : 0u;
    if (pk == k) {
      const bool want = verify && code != kGridMore && !r.error && r.crc_len > 0 && ctype != HDFS_CRC32C_CSUM_NULL;
      const uint32_t nch = want ? uint32_t(r.crc_len) / 4u : 0u;
      const bool fits = uint32_t(r.data_len) <= kSmallMax && nch <= kSmallMaxChunks && (cs % 64u == 0 || nch == 1u);
      // the bytes this workgroup will load: inside the stream
      const bool inside =
          !(want && fits) ||
          DCHK(r.stream_off + r.header_len + uint64_t(r.crc_len) + uint64_t(r.data_len) <= len, kDkSmallRun);
      rec = r;
      ctl[0] = code;
      ctl[1] = want && fits && inside ? 1u : 0u;
      ctl[2] = want && !fits ? 1u : 0u;
      ctl[3] = 0xFFFFFFFFu;
      ctl[4] = 0u;
      const uint32_t span = min(cs, uint32_t(r.data_len));  // longest shift: < one chunk
      ctl[5] = span > 1u ? 32u - __builtin_clz(span - 1u) : 1u;
    }
  }
  __syncthreads();
  if (tid == 0 && copy_dst) {
    uint64_t before = 0, at = 0;
    uint32_t ok = 1, cb = 0, clen = 0;
    for (uint32_t t = 0; t < k; t++) {
      before += sdl[t];
      ok &= son[t];
    }
    (void)frame::read_avail(rec, rwin != 0, client_offset, cb);
    frame::read_place(before, sdl[k], copy_cap, at, clen);
    ctl[6] = uint32_t(at);
    ctl[7] = uint32_t(at >> 32);
    // the window inside the packet's data, its place inside the destination
    ctl[8] = ok && clen &&
                     DCHK(uint64_t(cb) + clen <= uint64_t(uint32_t(rec.data_len)) && at + clen <= copy_cap, kDkSmallRun)
                 ? 1u
                 : 0u;
    ctl[9] = cb;
    ctl[10] = cb + clen;
  }
  __syncthreads();
  if (ctl[1] && DCHK(ctl[5] <= 16u, kDkSmallRun)) {  // zt holds 16 levels
    const uint32_t nlev = ctl[5];
    for (uint32_t q = tid; q < nlev * 256u; q += 1024u)
      *reinterpret_cast<u32x4 *>(&zt[4u * q]) = gload16(pow2 + 4u * q);
    const uint32_t dlen = uint32_t(rec.data_len), nch = uint32_t(rec.crc_len) / 4u;
    const uint8_t *crcp = s + rec.stream_off + rec.header_len;
    const uint8_t *dp = crcp + rec.crc_len;
    for (uint32_t j = tid; j < nch; j += 1024u) acc[j] = 0u;
    // the piece's 64 bytes (any byte alignment: buffer loads; past dlen: zeros).
    // rec is in LDS, so the compiler takes its fields for divergent:
    // readfirstlane keeps the descriptors in SGPRs (no waterfall loops)
    const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<uint8_t *>(rfl64(reinterpret_cast<uint64_t>(dp))), 0, static_cast<int>(rfl(dlen)), 0x00020000);
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<uint8_t *>(rfl64(reinterpret_cast<uint64_t>(crcp))), 0, static_cast<int>(rfl(nch * 4u)),
        0x00020000);
    const uint32_t b0 = 64u * tid;
    uint32_t d[16];
#pragma unroll
    for (uint32_t m = 0; m < 4; m++) {
      const u32x4 x = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rd, b0 + 16u * m, 0, 0));
      d[4 * m + 0] = x.x;
      d[4 * m + 1] = x.y;
      d[4 * m + 2] = x.z;
      d[4 * m + 3] = x.w;
    }
    if (b0 < dlen && b0 + 64u > dlen && (dlen & 15u)) {
      // the piece holding the packet's last bytes: a 16-B load that crosses
      // the descriptor's range returns zeros, so the last partial 16 B are
      // read byte by byte (one lane)
      const uint32_t q0 = (dlen - b0) & ~15u;
#pragma unroll
      for (uint32_t q = 0; q < 16; q++) {
        if (4u * q >= q0 && 4u * q < dlen - b0) {
          uint32_t wv = 0;
          for (uint32_t b = 0; b < 4u && b0 + 4u * q + b < dlen; b++)
            wv |= uint32_t(__builtin_amdgcn_raw_buffer_load_b8(rd, b0 + 4u * q + b, 0, 0)) << (8u * b);
          d[q] = wv;
        }
      }
    }
    uint32_t ev[2];
#pragma unroll
    for (uint32_t q = 0; q < 2; q++) ev[q] = __builtin_amdgcn_raw_buffer_load_b32(rc, 4u * (q * 1024u + tid), 0, 0);
    __syncthreads();  // tables and acc ready
    if (b0 < dlen) {
      const uint32_t j = b0 / cs, ce = min((j + 1u) * cs, dlen), n = min(64u, ce - b0);
      uint32_t c = (b0 == j * cs) ? 0xFFFFFFFFu : 0u;
#pragma unroll
      for (uint32_t q = 0; q < 16; q++) {
        if (4u * q + 4u <= n) {
          const uint32_t x = c ^ d[q];
          c = tt[768u + (x & 0xffu)] ^ tt[512u + ((x >> 8) & 0xffu)] ^ tt[256u + ((x >> 16) & 0xffu)] ^ tt[x >> 24];
        }
      }
      if (n & 3u) {
        uint32_t tw = 0u;
#pragma unroll
        for (uint32_t q = 0; q < 16; q++) tw = (q == (n >> 2)) ? d[q] : tw;
        for (uint32_t b = 0; b < (n & 3u); b++) c = tt[(c ^ (tw >> (8u * b))) & 0xffu] ^ (c >> 8);
      }
      for (uint32_t dd = ce - b0 - n, lvl = 0; dd; lvl++, dd >>= 1) {
        if (dd & 1u) {
          const uint32_t *z = zt + lvl * 1024u;
          c = z[c & 0xffu] ^ z[256u + ((c >> 8) & 0xffu)] ^ z[512u + ((c >> 16) & 0xffu)] ^ z[768u + (c >> 24)];
        }
      }
      atomicXor(&acc[j], c);
    }
    __syncthreads();
#pragma unroll
    for (uint32_t q = 0; q < 2; q++) {
      const uint32_t j = q * 1024u + tid;
      if (j < nch && __builtin_bswap32(ev[q]) != ~acc[j]) {
        atomicMin(&ctl[3], j);
        atomicAdd(&ctl[4], 1u);
      }
    }
    if (copy_dst && ctl[8] && b0 < dlen) {
      // verify + copy-out: the piece, still in registers, to its place in the
      // de-framed payload -- data bytes [w0, w1) of the packet (the whole
      // payload, or the part a client read takes) at copy_dst + at + (j - w0).
      // 16-B pieces inside the window go out whole; a piece at an edge of it
      // (a read starting or ending inside the packet, the packet's last
      // partial 16 B) byte by byte
      const uint32_t w0 = rfl(ctl[9]), w1 = rfl(ctl[10]);  // LDS words: uniform, in SGPRs
      uint8_t *dst = copy_dst + ((uint64_t(rfl(ctl[7])) << 32) | rfl(ctl[6])) - w0;
      const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(dst, 0, static_cast<int>(w1), 0x00020000);
#pragma unroll
      for (uint32_t m = 0; m < 4; m++) {
        const uint32_t o = b0 + 16u * m;
        if (o >= w0 && o + 16u <= w1) {
          const u32x4 v = {d[4 * m], d[4 * m + 1], d[4 * m + 2], d[4 * m + 3]};
          __builtin_amdgcn_raw_buffer_store_b128(v, rw, o, 0, 0);
        } else if (o < w1 && o + 16u > w0) {
          for (uint32_t b = max(o, w0); b < min(o + 16u, w1); b++)
            __builtin_amdgcn_raw_buffer_store_b8(static_cast<uint8_t>(d[(b - b0) >> 2] >> (8u * (b & 3u))), rw, b, 0, 0);
        }
      }
    }
  }
  __syncthreads();
  // this packet's slot in pinned host memory: record, status, verdict, then
  // (one system fence later) the call's sequence number.  No cross-workgroup
  // step: the host reads the count slots and works out the run itself.
  if (tid == 0) {
    uint8_t *slot = hout + size_t(k) * kSrSlot;
    const uint64_t *x = reinterpret_cast<const uint64_t *>(&rec);
    uint64_t *y = reinterpret_cast<uint64_t *>(slot);
    for (int q = 0; q < int(kGridRecBytes / 8); q++) y[q] = x[q];
    uint32_t *w = reinterpret_cast<uint32_t *>(slot + kGridRecBytes);
    w[0] = ctl[0] | (ctl[2] << 8);
    w[1] = ctl[3];
    w[2] = ctl[4];
    __threadfence_system();
    __hip_atomic_store(&w[3], seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// The delivery of verified bytes (the unit, store and completion protocol:
// "Copy of a verified read's next bytes" above the mailbox kernel, which
// serves small deliveries with the same unit code).  !TAB: the pieces in the
// kernel arguments, staged in LDS, units strided over the grid.  TAB: the
// device table, each workgroup a contiguous unit range from its first entry.
template <bool TAB>
__global__ __launch_bounds__(256) void copy_pieces_kernel(CopyPieces a) {
  constexpr uint32_t kStage = TAB ? kCopyTabStage : kCopyPiecesMax;
  __shared__ const uint8_t *lsrc[kStage];
  __shared__ uintptr_t ldst[kStage], lend[kStage];
  __shared__ uint32_t luend[kStage + 1];
  const uint32_t n = a.n, tid = threadIdx.x;
  // diagnostic phase stamps (100 MHz): 0 entry, 1 first entries staged, 2
  // stores acknowledged, 3 counted done
  unsigned long long *const ps = kDiag && a.stamps ? a.stamps + kCopyStampOff + 4u * blockIdx.x : nullptr;
  auto stamp = [&](uint32_t ph) {
    if (kDiag && ps && tid == 0) ps[ph] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  if (!TAB) {
    if (tid < n) {
      lsrc[tid] = a.src[tid];
      ldst[tid] = reinterpret_cast<uintptr_t>(a.dst[tid]);
      lend[tid] = reinterpret_cast<uintptr_t>(a.dst[tid]) + a.len[tid];
      luend[tid + 1u] = a.uend[tid];
    }
    if (tid == 0) luend[0] = 0u;
    __syncthreads();
    const uint32_t total = luend[n];
    copy_staged(lsrc, ldst, lend, luend, n, blockIdx.x * 256u + tid, total, gridDim.x * 256u);
  } else {
    // this workgroup's units [u0, u1), from entry e on: staged kStage entries
    // at a time (each entry is read by the workgroups it spans)
    const uint32_t u0 = blockIdx.x * a.per, u1 = min(a.total, u0 + a.per);
    uint32_t e = __builtin_amdgcn_readfirstlane(a.wg0[blockIdx.x]);
    uint32_t ucur = u0;
    while (ucur < u1) {
      const uint32_t cnt = min(kStage, n - e);
      if (tid < cnt) {
        const CopyEntry x = a.tab[e + tid];
        lsrc[tid] = x.src;
        ldst[tid] = reinterpret_cast<uintptr_t>(x.dst);
        lend[tid] = reinterpret_cast<uintptr_t>(x.dst) + x.len;
        luend[tid + 1u] = x.uend;
      }
      if (tid == 0) luend[0] = e ? a.tab[e - 1u].uend : 0u;
      __syncthreads();
      if (ucur == u0) stamp(1);
      const uint32_t cend = min(u1, luend[cnt]);
      copy_staged(lsrc, ldst, lend, luend, cnt, ucur + tid, cend, 256u);
      ucur = cend;
      e += cnt;
      __syncthreads();  // the stage is rewritten
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  stamp(2);
  if (tid == 0) {
    const uint32_t prev = __hip_atomic_fetch_add(a.count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev + 1u == gridDim.x) {
      __hip_atomic_store(a.count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.done, a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  stamp(3);
}

// The same delivery BESIDE a running verify (read_dev_scatter starts it
// from the packets predicted at the speculative launch's early block): no
// LDS -- the verify's workgroups hold each CU's -- and few enough VGPRs that
// one workgroup fits next to a verify workgroup on every CU, so the copy
// streams while the verify does.  Table launches only; a thread walks its
// units (strided by 256) with its own entry cursor; a
// piece's edge blocks go byte by byte on the spot.  Four units in flight
// per lane; more workgroups than fit beside the verify, so the rest start as
// its workgroups retire.
struct CopyLdG {
  uint32_t w[5], sh, ok;
  uintptr_t D;
};

DEV void copyg_issue(CopyLdG &x, const CopyEntry *__restrict__ tab, uint32_t &ec, uint32_t &us, uint32_t &ue,
                     uint32_t u, uint32_t u1) {
  x.ok = 0u;
  if (u >= u1) return;
  while (u >= ue) {
    ec++;
    us = ue;
    ue = tab[ec].uend;
  }
  const CopyEntry xe = tab[ec];
  const uintptr_t d = reinterpret_cast<uintptr_t>(xe.dst), e = d + xe.len;
  const uintptr_t D = (d & ~uintptr_t(15)) + 16u * uintptr_t(u - us);
  if (D >= d && D + 16u <= e) {
    const uintptr_t sa = reinterpret_cast<uintptr_t>(xe.src) + (D - d);
    x.sh = uint32_t(sa & 3u);
    const uint8_t *a0 = reinterpret_cast<const uint8_t *>(sa - x.sh);
#pragma unroll
    for (int q = 0; q < 4; q++) x.w[q] = gload32(a0 + 4 * q);
    x.w[4] = x.sh ? gload32(a0 + 16) : 0u;
    x.D = D;
    x.ok = 1u;
  } else {
    copy_unit(xe.src, d, e, D);
  }
}

DEV void copyg_finish(const CopyLdG &x) {
  if (!x.ok) return;
  u32x4 v;
  v.x = align_word(x.w[1], x.w[0], x.sh);
  v.y = align_word(x.w[2], x.w[1], x.sh);
  v.z = align_word(x.w[3], x.w[2], x.sh);
  v.w = align_word(x.w[4], x.w[3], x.sh);
  store16_sc1(reinterpret_cast<uint8_t *>(x.D), v);
}

__global__ __launch_bounds__(256) void copy_beside_kernel(CopyPieces a) {
  const uint32_t tid = threadIdx.x;
  const uint32_t u0 = blockIdx.x * a.per, u1 = min(a.total, u0 + a.per);
  const CopyEntry *__restrict__ tab = a.tab;
  uint32_t ec = __builtin_amdgcn_readfirstlane(a.wg0[blockIdx.x]);
  uint32_t us = ec ? tab[ec - 1u].uend : 0u, ue = tab[ec].uend;
  constexpr int U = 4;
  CopyLdG cur[U], nxt[U];
#pragma unroll
  for (int k = 0; k < U; k++) copyg_issue(cur[k], tab, ec, us, ue, u0 + tid + 256u * uint32_t(k), u1);
  for (uint32_t ub = u0 + tid; ub < u1; ub += 256u * U) {
#pragma unroll
    for (int k = 0; k < U; k++) copyg_issue(nxt[k], tab, ec, us, ue, ub + 256u * uint32_t(U + k), u1);
#pragma unroll
    for (int k = 0; k < U; k++) copyg_finish(cur[k]);
#pragma unroll
    for (int k = 0; k < U; k++) cur[k] = nxt[k];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const uint32_t prev = __hip_atomic_fetch_add(a.count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev + 1u == gridDim.x) {
      __hip_atomic_store(a.count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.done, a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

hipError_t launch_copy_beside(const CopyPieces &a, int grid, hipStream_t stream) {
  if (!a.n || grid < 1 || grid > int(kCopyTabBlocks) || !a.done || !a.count || !a.tab || !a.wg0 || !a.per ||
      uint64_t(a.per) * uint32_t(grid) < a.total)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(copy_beside_kernel, dim3(grid), dim3(256), 0, stream, a);
  return hipGetLastError();
}

hipError_t launch_copy_pieces(const CopyPieces &a, int grid, hipStream_t stream) {
  if (!a.n || grid < 1 || !a.done || !a.count) return hipErrorInvalidValue;
  if (a.tab) {
    if (grid > int(kCopyTabBlocks) || !a.wg0 || !a.per || uint64_t(a.per) * uint32_t(grid) < a.total)
      return hipErrorInvalidValue;
    hipLaunchKernelGGL(copy_pieces_kernel<true>, dim3(grid), dim3(256), 0, stream, a);
  } else {
    if (a.n > kCopyPiecesMax || grid > int(kCopyBlocksMax)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(copy_pieces_kernel<false>, dim3(grid), dim3(256), 0, stream, a);
  }
  return hipGetLastError();
}

hipError_t launch_small_run(const uint8_t *s, uint64_t len, uint32_t count, int proto, uint32_t cs, int ctype,
                            int verify, const uint32_t *tab, const uint32_t *pow2, uint8_t *copy_dst,
                            uint64_t copy_cap, int win, int64_t client_offset, uint8_t *hout, uint32_t seq,
                            hipStream_t stream) {
  if (!count || count > kSmallRunMax) return hipErrorInvalidValue;
  hipLaunchKernelGGL(small_run_kernel, dim3(count), dim3(1024), 0, stream, s, len, count, proto, cs, ctype, verify, tab,
                     pow2, copy_dst, copy_cap, win, client_offset, hout, seq);
  return hipGetLastError();
}

hipError_t launch_grid_finalize(const SegDev *segs, uint32_t nseg, const uint32_t *seg2pkt, const uint32_t *fb,
                                GridBad *bad, uint32_t bad_cap, GridSummary *sum, uint8_t *hsum2, uint32_t host_cap,
                                uint32_t seq, hipStream_t stream) {
  // nseg 0xFFFFFFFF: the run's size is read from *sum
  hipLaunchKernelGGL(grid_finalize_kernel, dim3(1), dim3(1024), 0, stream, segs, nseg, seg2pkt, fb, bad, bad_cap, sum,
                     hsum2, host_cap, seq);
  return hipGetLastError();
}

hipError_t launch_frame_grid(const uint8_t *s, uint64_t len, uint64_t base, uint32_t count, int proto, uint32_t cs,
                             int ctype, int verify, uint32_t sflags, uint8_t *bm_base, uint8_t *copy_base,
                             uint64_t copy_cap, int win, int64_t client_offset, GridBufs g, hipStream_t stream,
                             unsigned long long *stamps) {
  if (!count || count > kGridMaxCount || base >= len || !g.seq) return hipErrorInvalidValue;
  const uint32_t nblk = (count + kGridBlock - 1) / kGridBlock;
  hipLaunchKernelGGL(frame_build_kernel, dim3(nblk), dim3(kGridBlock), 0, stream, s, len, base, count, proto, cs,
                     ctype, verify, sflags, bm_base, copy_base, copy_cap, win, client_offset, g.recs,
                     reinterpret_cast<GridLook *>(g.look), g.segs, g.seg2pkt, g.fb, g.gctr, g.done, g.exc, g.sum,
                     g.hsum, g.seq, kDiag ? stamps : nullptr);
  return hipGetLastError();
}


// ---------------------------------------------------------------------------
// Host-side launchers (used by crc32c_engine.cpp).
// ---------------------------------------------------------------------------
hipError_t launch_gather(const uint8_t *raw, const PktDesc *descs, uint32_t npk, uint32_t units, uint8_t *arena,
                         uint8_t *crc_arena, hipStream_t stream) {
  if (!npk || !units) return hipSuccess;
  hipLaunchKernelGGL(packet_gather_kernel, dim3(units), dim3(256), 0, stream, raw, descs, npk, arena, crc_arena);
  return hipGetLastError();
}

// Header windows of a device-resident packet stream: row k of out is the
// kHdrWin bytes at base + k * stride (zero past len).  The host framing walk
// (crc32c_packets.cpp) reads them after one D2H copy instead of fetching
// each header with its own copy; for the fixed-size packets of a block
// transfer one window covers the whole stream.  One thread per dword of a
// row; byte loads because the rows sit at any byte offset.
// proto != 0 (first window of a walk, stride unknown to the host): the
// stride is the wire size of the packet at base, header_len + plen - 4 as
// frame_step computes it (v1 header 25 B, v2 6 + hlen), and thread 0 writes
// it to *stride_out.  A wrong guess (a malformed first packet) costs nothing
// but the window: every row holds the real bytes at its address, and the
// host only reads a row whose address the walk reaches.
__global__ __launch_bounds__(256) void header_window_kernel(const uint8_t *__restrict__ s, uint64_t len,
                                                            uint64_t base, uint64_t stride, uint32_t count,
                                                            int proto, uint32_t *__restrict__ out,
                                                            uint64_t *__restrict__ stride_out) {
  const uint32_t t = blockIdx.x * 256u + threadIdx.x;
  constexpr uint32_t kWords = kHdrWin / 4;
  if (proto) {
    stride = grid_stride(s, len, base, proto);
    // the stride slot follows the rows (one D2H copy takes both)
    if (t == 0 && DCHK(reinterpret_cast<uintptr_t>(stride_out) >= reinterpret_cast<uintptr_t>(out + count * kWords),
                       kDkHeaderWindow))
      *stride_out = stride;
  }
  if (t >= count * kWords || !DCHK(uint64_t(count) * kWords <= 0xFFFFFFFFull, kDkHeaderWindow)) return;
  const uint64_t at = base + uint64_t(t / kWords) * stride + 4ull * (t % kWords);
  uint32_t w = 0;
#pragma unroll
  for (int b = 0; b < 4; b++)
    if (at + b < len) w |= uint32_t(s[at + b]) << (8 * b);
  out[t] = w;
}

// Device checks of the diagnostic build (DCHK above): {kernel id of the
// first violation, its line, violations}; reset clears them.  The release
// build has none and reports zeros.
#ifdef HDFS_CRC32C_DIAG
// reset < 0: record one violation from kernel id 0 (the plumbing's own test)
__global__ void dchk_inject_kernel() { (void)DCHK(threadIdx.x != 0u, 0u); }
#endif

hipError_t read_device_checks(uint32_t out[3], int reset) {
#ifdef HDFS_CRC32C_DIAG
  if (reset < 0) {
    hipLaunchKernelGGL(dchk_inject_kernel, dim3(1), dim3(64), 0, nullptr);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) return e;
    reset = 0;
  }
  uint32_t v[4] = {0u, 0u, 0u, 0u};
  hipError_t e = hipMemcpyFromSymbol(v, HIP_SYMBOL(g_dchk), sizeof(v), 0, hipMemcpyDeviceToHost);
  if (e == hipSuccess && reset && v[2]) {
    const uint32_t z[4] = {0u, 0u, 0u, 0u};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_dchk), z, sizeof(z), 0, hipMemcpyHostToDevice);
  }
  out[0] = v[0];
  out[1] = v[1];
  out[2] = v[2];
  return e;
#else
  (void)reset;
  out[0] = out[1] = out[2] = 0u;
  return hipSuccess;
#endif
}

__global__ void queue_probe_kernel(uint64_t *out) {
  if (threadIdx.x == 0) *out = (uint64_t)(unsigned long long)(__builtin_amdgcn_queue_ptr());
}

hipError_t launch_queue_probe(uint64_t *out, hipStream_t stream) {
  hipLaunchKernelGGL(queue_probe_kernel, dim3(1), dim3(64), 0, stream, out);
  return hipGetLastError();
}

hipError_t launch_header_window(const uint8_t *s, uint64_t len, uint64_t base, uint64_t stride, uint32_t count,
                                int proto, uint8_t *out, uint64_t *stride_out, hipStream_t stream) {
  if (!count) return hipSuccess;
  if (proto && !stride_out) return hipErrorInvalidValue;
  const uint32_t threads = count * (kHdrWin / 4);
  hipLaunchKernelGGL(header_window_kernel, dim3((threads + 255) / 256), dim3(256), 0, stream, s, len, base, stride,
                     count, proto, reinterpret_cast<uint32_t *>(out), stride_out);
  return hipGetLastError();
}

hipError_t launch_tiles(int mode, int order, int nt, int depth, int streams, int block, int grid,
                        const SegDev *segs, uint32_t nseg, uint64_t total_rounds, uint64_t total_tiles,
                        const uint32_t *gtab, uint32_t *first_bad, unsigned long long *mism,
                        unsigned long long *diag, uint32_t tune, uint32_t *gctr, hipStream_t stream, int copy,
                        int una, const GridSummary *dyn, uint32_t utiles, int fuse_generic) {
  const uint32_t fn = dyn && fuse_generic ? 1u : 0u;
  // uniform-table look-up: tile indices must fit 32 bits (multiply-high form)
  if (utiles && !dyn && (total_tiles >> 32)) utiles = 0;
#define HDFS_LAUNCH_CUG(M, O, N, D, S, B, BUF, C, U, G)                                                          \
  hipLaunchKernelGGL((crc32c_tiles_kernel<M, O, N, D, S, B, BUF, C, U, G>), dim3(grid), dim3(B), 0, stream,      \
                     segs, nseg, total_rounds, total_tiles, gtab, first_bad, mism, diag, tune, gctr, dyn, utiles, fn)
#define HDFS_LAUNCH_CU(M, O, N, D, S, B, BUF, C, U) HDFS_LAUNCH_CUG(M, O, N, D, S, B, BUF, C, U, 0)
#define HDFS_LAUNCH_C(M, O, N, D, S, B, BUF, C) HDFS_LAUNCH_CU(M, O, N, D, S, B, BUF, C, 0)
#define HDFS_LAUNCH(M, O, N, D, S, B, BUF) HDFS_LAUNCH_C(M, O, N, D, S, B, BUF, 0)
#define HDFS_SHAPE(O, N, D, S, B) (order == (O) && nt == (N) && depth == (D) && streams == (S) && block == (B))
  if (mode != kModeCompute && mode != kModeVerify && !(kDiag && mode == kModeLoadOnly)) return hipErrorInvalidValue;
  if (copy || una) {
    // verify + copy-out (device packet streams) and byte-unaligned data: the
    // two product shapes only
    if (copy && mode != kModeVerify) return hipErrorInvalidValue;
#define HDFS_LAUNCH_PRODUCT_CU(M, C, U)                                                           \
    if (HDFS_SHAPE(3, 2, 3, 1, 1024)) HDFS_LAUNCH_CU(M, 3, 1, 3, 1, 1024, 1, C, U);               \
    else if (HDFS_SHAPE(2, 1, 3, 1, 1024)) HDFS_LAUNCH_CU(M, 2, 1, 3, 1, 1024, 0, C, U);          \
    else return hipErrorInvalidValue;
    if (mode == kModeCompute) {
      HDFS_LAUNCH_PRODUCT_CU(kModeCompute, 0, 1)
    } else if (copy && una) {
      HDFS_LAUNCH_PRODUCT_CU(kModeVerify, 1, 1)
    } else if (copy) {
      HDFS_LAUNCH_PRODUCT_CU(kModeVerify, 1, 0)
    } else {
      HDFS_LAUNCH_PRODUCT_CU(kModeVerify, 0, 1)
    }
#undef HDFS_LAUNCH_PRODUCT_CU
    return hipGetLastError();
  }
  // Release build: the two product shapes only -- schedule 3 with nontemporal
  // buffer loads (nt 2), and schedule 2 (small launches / tables of small
  // segments) with nontemporal global loads; depth 3, one tile stream, 1024
  // threads.  Anything else is refused, never silently replaced.
#define HDFS_LAUNCH_PRODUCT(M)                                                                  \
  if (HDFS_SHAPE(3, 2, 3, 1, 1024)) HDFS_LAUNCH(M, 3, 1, 3, 1, 1024, 1);                        \
  else if (HDFS_SHAPE(2, 1, 3, 1, 1024)) HDFS_LAUNCH(M, 2, 1, 3, 1, 1024, 0);
#ifndef HDFS_CRC32C_DIAG
  if (mode == kModeVerify) {
    HDFS_LAUNCH_PRODUCT(kModeVerify)
    else return hipErrorInvalidValue;
  } else {
    HDFS_LAUNCH_PRODUCT(kModeCompute)
    else if (HDFS_SHAPE(5, 2, 3, 1, 1024)) HDFS_LAUNCH_CUG(kModeCompute, 3, 1, 3, 1, 1024, 1, 0, 0, 1);
    else return hipErrorInvalidValue;
  }
#else
  // Diagnostic build: the tuning shapes of tools/exp_ab.py and
  // tests/test_gpu_shapes.py, each launched only when requested exactly.
#define HDFS_LAUNCH_ALL(M)                                                                      \
  HDFS_LAUNCH_PRODUCT(M)                                                                        \
  else if (HDFS_SHAPE(3, 2, 4, 1, 1024)) HDFS_LAUNCH(M, 3, 1, 4, 1, 1024, 1);                   \
  else if (HDFS_SHAPE(3, 1, 3, 1, 1024)) HDFS_LAUNCH(M, 3, 1, 3, 1, 1024, 0);                   \
  else if (HDFS_SHAPE(3, 1, 4, 1, 1024)) HDFS_LAUNCH(M, 3, 1, 4, 1, 1024, 0);                   \
  else if (HDFS_SHAPE(3, 1, 2, 2, 1024)) HDFS_LAUNCH(M, 3, 1, 2, 2, 1024, 0);                   \
  else if (HDFS_SHAPE(3, 1, 3, 2, 1024)) HDFS_LAUNCH(M, 3, 1, 3, 2, 1024, 0);                   \
  else if (HDFS_SHAPE(3, 1, 3, 2, 768)) HDFS_LAUNCH(M, 3, 1, 3, 2, 768, 0);                     \
  else if (HDFS_SHAPE(3, 1, 2, 2, 512)) HDFS_LAUNCH(M, 3, 1, 2, 2, 512, 0);                     \
  else if (HDFS_SHAPE(3, 1, 3, 2, 512)) HDFS_LAUNCH(M, 3, 1, 3, 2, 512, 0);                     \
  else if (HDFS_SHAPE(3, 1, 2, 4, 512)) HDFS_LAUNCH(M, 3, 1, 2, 4, 512, 0);                     \
  else if (HDFS_SHAPE(3, 1, 3, 1, 768)) HDFS_LAUNCH(M, 3, 1, 3, 1, 768, 0);                     \
  else if (HDFS_SHAPE(3, 1, 3, 1, 512)) HDFS_LAUNCH(M, 3, 1, 3, 1, 512, 0);                     \
  else if (HDFS_SHAPE(2, 1, 4, 1, 1024)) HDFS_LAUNCH(M, 2, 1, 4, 1, 1024, 0);                   \
  else if (HDFS_SHAPE(1, 1, 3, 1, 1024)) HDFS_LAUNCH(M, 1, 1, 3, 1, 1024, 0);                   \
  else if (HDFS_SHAPE(1, 1, 4, 1, 1024)) HDFS_LAUNCH(M, 1, 1, 4, 1, 1024, 0);                   \
  else if (HDFS_SHAPE(1, 0, 3, 1, 1024)) HDFS_LAUNCH(M, 1, 0, 3, 1, 1024, 0);                   \
  else if (HDFS_SHAPE(0, 1, 3, 1, 1024)) HDFS_LAUNCH(M, 0, 1, 3, 1, 1024, 0);                   \
  else if (HDFS_SHAPE(0, 0, 3, 1, 1024)) HDFS_LAUNCH(M, 0, 0, 3, 1, 1024, 0);
  if (mode == kModeLoadOnly) {
    if (HDFS_SHAPE(3, 2, 3, 1, 1024)) HDFS_LAUNCH(kModeLoadOnly, 3, 1, 3, 1, 1024, 1);
    else return hipErrorInvalidValue;
  } else if (mode == kModeVerify) {
    HDFS_LAUNCH_ALL(kModeVerify)
    else return hipErrorInvalidValue;
  } else {
    HDFS_LAUNCH_ALL(kModeCompute)
    else if (HDFS_SHAPE(4, 2, 3, 1, 1024)) HDFS_LAUNCH(kModeCompute, 4, 1, 3, 1, 1024, 1);
    else if (HDFS_SHAPE(5, 2, 3, 1, 1024)) HDFS_LAUNCH_CUG(kModeCompute, 3, 1, 3, 1, 1024, 1, 0, 0, 1);
    else if (HDFS_SHAPE(6, 2, 3, 1, 1024)) HDFS_LAUNCH_CUG(kModeCompute, 3, 1, 3, 1, 1024, 1, 0, 0, 2);
    else if (HDFS_SHAPE(7, 2, 3, 1, 1024)) HDFS_LAUNCH(kModeCompute, 7, 1, 3, 1, 1024, 1);
    else if (HDFS_SHAPE(7, 2, 4, 1, 1024)) HDFS_LAUNCH(kModeCompute, 7, 1, 4, 1, 1024, 1);
    else if (HDFS_SHAPE(5, 2, 4, 1, 1024)) HDFS_LAUNCH_CUG(kModeCompute, 3, 1, 4, 1, 1024, 1, 0, 0, 1);
    else return hipErrorInvalidValue;
  }
#undef HDFS_LAUNCH_ALL
#endif
#undef HDFS_LAUNCH_PRODUCT
#undef HDFS_SHAPE
#undef HDFS_LAUNCH
#undef HDFS_LAUNCH_C
#undef HDFS_LAUNCH_CU
#undef HDFS_LAUNCH_CUG
  return hipGetLastError();
}

#ifdef HDFS_CRC32C_DIAG
// Streaming-read probe: the empirical HBM read roofline for 16-B-per-lane
// fully coalesced loads, no compute.  NLOAD loads in flight per lane, NT =
// nontemporal policy.
template <int NLOAD, int NT, int PERM = 0>
__global__ __launch_bounds__(1024) void probe_read_kernel(const uint8_t *__restrict__ p, uint64_t nbytes,
                                                          uint32_t *__restrict__ out) {
  const uint64_t n16 = nbytes / 16;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  // PERM: lanes of a wave read the wave's 1 KiB in the permuted order
  // 4*(lane&15) + (lane>>4) (still one contiguous 1 KiB per instruction).
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t l2 = PERM ? (4u * (lane & 15u) + (lane >> 4)) : lane;
  uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + (threadIdx.x & ~63u) + l2;
  u32x4 acc = {0u, 0u, 0u, 0u};
  for (; i + (NLOAD - 1) * stride < n16; i += NLOAD * stride) {
    u32x4 v[NLOAD];
#pragma unroll
    for (int k = 0; k < NLOAD; k++) v[k] = NT ? gload16_nt(p + 16 * (i + k * stride)) : gload16(p + 16 * (i + k * stride));
#pragma unroll
    for (int k = 0; k < NLOAD; k++) acc ^= v[k];
  }
  for (; i < n16; i += stride) acc ^= gload16(p + 16 * i);
  const uint32_t v = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (v == 0x9E3779B9u) out[0] = v;  // keeps the loads live; practically never stores
}

// Same, but each lane reads 64 CONTIGUOUS bytes per quad (4 loads at +0/16/
// 32/48): per instruction the wave touches a 4 KiB span with a 64-B lane
// stride.  NQUAD quads in flight per lane.
template <int NQUAD>
__global__ __launch_bounds__(1024) void probe_quad_kernel(const uint8_t *__restrict__ p, uint64_t nbytes,
                                                          uint32_t *__restrict__ out) {
  const uint64_t n64 = nbytes / 64;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  u32x4 acc = {0u, 0u, 0u, 0u};
  for (; i + (NQUAD - 1) * stride < n64; i += NQUAD * stride) {
    u32x4 v[NQUAD][4];
#pragma unroll
    for (int m = 0; m < NQUAD; m++)
#pragma unroll
      for (int k = 0; k < 4; k++) v[m][k] = gload16_nt(p + 64 * (i + m * stride) + 16 * k);
#pragma unroll
    for (int m = 0; m < NQUAD; m++)
#pragma unroll
      for (int k = 0; k < 4; k++) acc ^= v[m][k];
  }
  const uint32_t v = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (v == 0x9E3779B9u) out[0] = v;
}

hipError_t launch_probe2(const uint8_t *p, uint64_t nbytes, uint32_t *out, int grid, int block, int variant,
                         hipStream_t stream);

hipError_t launch_probe_read(const uint8_t *p, uint64_t nbytes, uint32_t *out, int grid, int block, int variant,
                             hipStream_t stream) {
  if (variant >= 10) return launch_probe2(p, nbytes, out, grid, block, variant, stream);
  switch (variant) {
    case 1: hipLaunchKernelGGL((probe_read_kernel<4, 1>), dim3(grid), dim3(block), 0, stream, p, nbytes, out); break;
    case 2: hipLaunchKernelGGL((probe_read_kernel<8, 0>), dim3(grid), dim3(block), 0, stream, p, nbytes, out); break;
    case 3: hipLaunchKernelGGL((probe_read_kernel<8, 1>), dim3(grid), dim3(block), 0, stream, p, nbytes, out); break;
    case 4: hipLaunchKernelGGL((probe_read_kernel<16, 1>), dim3(grid), dim3(block), 0, stream, p, nbytes, out); break;
    case 5: hipLaunchKernelGGL((probe_quad_kernel<1>), dim3(grid), dim3(block), 0, stream, p, nbytes, out); break;
    case 6: hipLaunchKernelGGL((probe_quad_kernel<2>), dim3(grid), dim3(block), 0, stream, p, nbytes, out); break;
    case 7: hipLaunchKernelGGL((probe_quad_kernel<4>), dim3(grid), dim3(block), 0, stream, p, nbytes, out); break;
    case 8: hipLaunchKernelGGL((probe_read_kernel<16, 1, 1>), dim3(grid), dim3(block), 0, stream, p, nbytes, out); break;
    case 9: hipLaunchKernelGGL((probe_read_kernel<4, 1, 1>), dim3(grid), dim3(block), 0, stream, p, nbytes, out); break;
    default: hipLaunchKernelGGL((probe_read_kernel<4, 0>), dim3(grid), dim3(block), 0, stream, p, nbytes, out);
  }
  return hipGetLastError();
}

#endif  // HDFS_CRC32C_DIAG

hipError_t launch_generic(int mode, const SegDev *segs, uint32_t nseg, uint64_t total_gtiles,
                          const uint32_t *gtab, uint32_t *first_bad, unsigned long long *mism,
                          hipStream_t stream, const GridSummary *dyn) {
  const uint64_t threads = total_gtiles * kTileChunks;
  const uint32_t blocks = static_cast<uint32_t>((threads + 255) / 256);
  if (!blocks) return hipSuccess;
  if (mode == kModeVerify)
    hipLaunchKernelGGL(crc32c_generic_kernel<kModeVerify>, dim3(blocks), dim3(256), 0, stream, segs,
                       nseg, total_gtiles, gtab, first_bad, mism, dyn);
  else
    hipLaunchKernelGGL(crc32c_generic_kernel<kModeCompute>, dim3(blocks), dim3(256), 0, stream,
                       segs, nseg, total_gtiles, gtab, first_bad, mism, dyn);
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

hipError_t launch_composite(const SegDev *segs, uint32_t nseg, const uint64_t *run_prefix, uint64_t total_runs,
                            const uint32_t *pow2, uint32_t *out, hipStream_t stream) {
  if (!total_runs) return hipSuccess;
  const uint32_t blocks = static_cast<uint32_t>((total_runs + 255) / 256);
  hipLaunchKernelGGL(composite_kernel, dim3(blocks), dim3(256), 0, stream, segs, nseg, run_prefix, total_runs, pow2,
                     out);
  return hipGetLastError();
}

hipError_t launch_small_chunks(int mode, const uint8_t *p, uint32_t len, uint32_t exact, uint32_t cs, uint32_t reg0,
                               uint32_t be, const uint32_t *expect, const uint32_t *tab, const uint32_t *kx,
                               uint32_t poly, uint32_t *meta, uint32_t *crcs, uint32_t seq, hipStream_t stream) {
  const uint32_t nch = cs ? (len + cs - 1) / cs : 0u;
  if (!len || len > kSmallMax || !cs || (cs % 4u && nch > 1) || nch > kSmallMaxChunks ||
      (!exact && (reinterpret_cast<uintptr_t>(p) & 15u)))
    return hipErrorInvalidValue;
  if (mode == kModeVerify)
    hipLaunchKernelGGL(small_chunks_kernel<kModeVerify>, dim3(1), dim3(1024), 0, stream, p, len, exact, cs, reg0, be,
                       expect, tab, kx, poly, meta, crcs, seq);
  else
    hipLaunchKernelGGL(small_chunks_kernel<kModeCompute>, dim3(1), dim3(1024), 0, stream, p, len, exact, cs, reg0,
                       be, expect, tab, kx, poly, meta, crcs, seq);
  return hipGetLastError();
}

hipError_t launch_prep(uint32_t *fb, uint32_t nfb, unsigned long long *mism, uint32_t *gctr, hipStream_t stream) {
  const uint32_t n = nfb ? nfb : 1u;
  hipLaunchKernelGGL(prep_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, fb, nfb, mism, gctr);
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
