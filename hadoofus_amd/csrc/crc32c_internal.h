// Internal structures shared by the gfx950 kernels and the host engine.
// Not part of the public C ABI (include/hadoofus_crc32c.h).
#pragma once
#include <cstdint>

struct hdfs_crc32c_packet;  // include/hadoofus_crc32c.h

namespace hdfs_crc32c {

// Diagnostic build (libhadoofus_crc32c_diag.so, -DHDFS_CRC32C_DIAG, for
// tools/ and the bench's ceiling measurement): tuning shapes, the load-only
// twin, store-policy experiments, per-wave clock stamps and read probes.
// The release library compiles none of them and reads no tuning knob from
// the environment: nothing outside the code can change what it computes.
#ifdef HDFS_CRC32C_DIAG
constexpr bool kDiag = true;
#else
constexpr bool kDiag = false;
#endif

// Kernels that carry device checks in the diagnostic build (DCHK,
// crc32c_kernels.hip): the id recorded with a violation.
enum DevCheckKernel : uint32_t {
  kDkFrameGrid = 1,
  kDkGridBuild = 2,
  kDkHeaderWindow = 3,
  kDkSmallRun = 4,
  kDkFinalize = 5,
  kDkSpecEarly = 6,  // spec_verify_kernel<0, 1>: a workgroup's tiles of a run != what it was said to own
};

// Segment flags (also mirrored as HDFS_CRC32C_SEG_* in the public header).
enum : uint32_t {
  kSegBigEndian = 1u,  // crcs[] are in wire byte order (src/util.h:68-92)
  kSegRaw = 2u,        // write the raw register (init 0, no final inversion)
};

// kModeLoadOnly: diagnostic twin of verify (same loads, same store ops with
// their records dropped, no CRC arithmetic) -- the kernel's own memory
// ceiling, for DESIGN.md; instantiated only in the diagnostic build.
enum Mode : int { kModeCompute = 0, kModeVerify = 1, kModeLoadOnly = 2 };

// One entry of the device-resident segment table.  A segment is one chunk
// stream with one bytesPerChecksum (src/datanode.c:2186); chunk i covers
// bytes [i*cs, min((i+1)*cs, len)).  Chunks are grouped in TILES of 8
// (tile t = chunks 8t..8t+7), which is also the bitmap byte they own.
// The fields the tiled kernel reads every round come first (bytes 0..51),
// so the compiler can fetch them with few wide scalar loads.
struct SegDev {
  const uint8_t *data;   // device pointer
  uint32_t *crcs;        // compute: out; verify: expected in
  uint8_t *bitmap;       // verify: out, one bit per chunk, byte t per tile t
  uint64_t mtile_start;  // global index of this segment's first main-path tile
  uint32_t chunk_size;   // bytes per checksum
  uint32_t flags;        // kSeg*
  uint32_t nchunks;      // ceil(len / chunk_size)
  uint32_t main_tiles;   // tiles [0, main_tiles) run on the tiled kernel
  uint32_t reg_init;     // register value each chunk starts from (~crc_init, or 0 if raw)
  uint32_t gen_tiles;    // tiles [main_tiles, main_tiles+gen_tiles) run generic
  uint64_t len;          // bytes
  uint64_t round_start;  // global index of this segment's first main-path round
  uint64_t gtile_start;  // global index of this segment's first generic tile
  // verify + copy-out: data bytes [copy_w0, copy_w1) of the segment are also
  // written to copy_dst + (j - copy_w0) (copy_dst null: no copy-out) -- the
  // whole payload, or the part of it a client read window takes
  uint8_t *copy_dst;
  uint32_t copy_w0, copy_w1;
};
static_assert(sizeof(SegDev) == 96, "SegDev layout");

// Device framing of a device-resident packet stream (frame_build_kernel):
// packets at base + k * stride, stride = the wire size of
// the packet at base.  Status per grid point k:
enum : uint32_t {
  kGridOn = 0,    // complete, framing-clean, wire size == stride: the walk goes on at k + 1
  kGridOff = 1,   // complete, framing-clean, other size: recorded, the walk goes on off the grid
  kGridStop = 2,  // recorded and the walk ends (framing error, empty last packet)
  kGridMore = 3,  // incomplete / past the stream: not recorded, the walk ends
};
struct GridSummary {
  uint32_t first_break;  // first grid point whose status is not kGridOn (count if none)
  uint32_t recorded;     // packets of the walk framed by this pass
  uint32_t last_status;  // status of first_break (kGridOn if none)
  uint32_t nseg;         // verify segments built
  uint64_t stride;
  uint64_t rounds, mtiles, gtiles;  // tiled / generic work of the segment table
  uint64_t payload;      // data bytes of the recorded framing-clean packets
  uint64_t consumed;     // stream offset after the last complete framing-clean packet
  uint64_t next_pos;     // where the walk continues (kGridOn / kGridOff)
  uint64_t bm_bytes;     // bitmap bytes of the segment table
  uint32_t nbad;         // verify: packets with bad chunks (grid_finalize_kernel)
  uint32_t unaligned;    // some tiled segment's data is not 4-B aligned (realigning kernel)
  uint32_t seq;          // host copy only: written last (after a system fence) by frame_build_kernel
  uint32_t nonuni;       // some segment breaks the uniform layout (OR-ed by frame_build_kernel)
  uint32_t utiles;       // main tiles per segment of a uniform table (0: not uniform), for the verify kernel
  uint32_t nexc;         // recorded packets whose record differs from the prediction from packet 0
};
// Records of a device-framed run reach the host as packet 0's record plus
// the packets that differ from the prediction from it (stream_off + k *
// stride, offsetInBlock + k * dataLen, seqno + k, every other field equal):
// up to kExcMax of them land in pinned memory with the summary, the host
// synthesises the rest.  Host area after the 256-B summary:
//   [kGridHostRec0]  packet 0's record
//   [kGridHostIdx]   kExcMax u32 grid indices of the exceptions
//   [kGridHostExc]   kExcMax records of the exceptions
constexpr uint32_t kExcMax = 64;
constexpr uint32_t kGridRecBytes = 56;  // sizeof(hdfs_crc32c_packet), checked where it is complete
constexpr uint32_t kGridHostRec0 = 256;
constexpr uint32_t kGridHostIdx = kGridHostRec0 + 64;
constexpr uint32_t kGridHostExc = kGridHostIdx + kExcMax * 4;
constexpr uint32_t kGridHostBytes = kGridHostExc + kExcMax * kGridRecBytes;
// Device tables of one framing pass (count grid points).
struct GridBufs {
  ::hdfs_crc32c_packet *recs;  // [count] records
  void *look;                  // [blocks] look-back records of the scan (kGridLookBytes each; zeroed when allocated)
  SegDev *segs;                // [count] verify segments
  uint32_t *seg2pkt;           // [count] segment -> grid point
  uint32_t *fb;                // [count] first bad chunk per segment
  uint32_t *gctr;              // tiled-kernel pool counter (zeroed by frame_build_kernel)
  uint32_t *done;              // [2]: blocks finished, exceptions found (reset by block 0 of the pass)
  uint32_t *exc;               // [count] grid indices of the exceptions
  GridSummary *sum;
  // pinned host memory mapped into the device: the summary, packet 0's
  // record and the exceptions (kGridHost*) are written there by the pass's
  // last block (no copy launch, which would queue behind the verify kernel
  // for CUs)
  uint8_t *hsum;
  uint32_t seq;                // written to the host summary's seq once the area is complete (> 0)
};
constexpr uint32_t kGridLookBytes = 256;

// Speculative one-launch verify of a device-resident run of equal packets
// (spec_verify_kernel, round 4).  Every workgroup decodes packet 0 itself;
// if it is a canonical, framing-clean packet of whole 512-B-multiple chunks,
// the run is the `count` packets at base + k * stride and every segment of
// the verify is a closed-form function of k (SpecTab) -- no framing pass,
// no segment table.  The workgroups check the headers of the run against
// the prediction from packet 0 (byte-equal but for offsetInBlock and seqno,
// which must continue packet 0's).  A header that differs is framed on the
// spot: a clean packet of the same wire size (a seqno jump, a skewed
// offset, lastPacketInBlock on the last data packet of a v1 block) is an
// EXCEPTION -- its layout is the run's, only its record differs, and it
// goes to the host with the results (up to kSpecExcMax; with a client read
// window only if its offsetInBlock is the predicted one, which places its
// copy); anything else raises `exc`, and the host discards the launch's
// results and frames the run the regular way.  Control words live in a
// ring of two SpecCtl slots: launch n uses slot n & 1 (zero when it starts)
// and zeroes slot (n + 1) & 1 for the next launch, so no reset command runs
// between launches.
constexpr uint32_t kSpecExcMax = 64;
struct SpecExc {
  uint64_t rec[7];  // the packet's record (hdfs_crc32c_packet)
  uint32_t k, pad;  // its index in the run
};
static_assert(sizeof(SpecExc) == 64, "SpecExc");
struct SpecCtl {
  unsigned long long mism;  // mismatching chunks of the run
  uint32_t gctr;            // tiled-kernel pool counter
  uint32_t done;            // workgroups finished
  uint32_t exc;             // a header off the run: the launch's results are void
  uint32_t tail_status;     // kGrid* of the point after the run (kGridOn: the run was cut, not ended)
  uint64_t tail_total;      // its wire size when kGridStop
  uint64_t tail[7];         // its record (hdfs_crc32c_packet) when kGridStop
  uint32_t nexc, pad0;      // exceptions found (entries past kSpecExcMax are not kept: exc is raised)
  // a coalesced batch's per-run completion (SpecArgs::early): run r is done
  // once every workgroup has verified its tiles of r and every header group
  // of r is checked -- run_done[r] counts both; bit r of run_bad: a header of
  // run r left the prediction
  uint32_t run_done[16];
  uint32_t run_mism[16];    // mismatching chunks of run r
  uint32_t run_bad, pad1[7];
};
static_assert(sizeof(SpecCtl) == 256, "SpecCtl");
// Pinned host area of one speculative launch: [0, 128) early block, written
// by workgroup 0 right after its decode of packet 0 (the host fills the
// run's records while the kernel verifies); [128, 256) final block and then
// the exceptions (kSpecExcMax SpecExc), written by the last workgroup to
// finish.  Sequence numbers last.
struct SpecEarly {
  uint64_t r0[7];           // packet 0's record (hdfs_crc32c_packet)
  uint64_t stride;
  uint32_t eligible;        // 0: not a run this launch takes (every workgroup returned)
  uint32_t count;           // packets of the run
  uint32_t seq;
  uint32_t pad[13];
};
struct SpecFinal {
  unsigned long long mism;
  uint32_t exc, tail_status;
  uint64_t tail_total;
  uint64_t tail[7];
  uint32_t seq, nexc;
  uint32_t pad[10];
};
static_assert(sizeof(SpecEarly) == 128 && sizeof(SpecFinal) == 128, "spec host blocks");
// A BATCH launch verifies up to kSpecRunsMax runs (one block transfer each,
// separate streams) of one packet layout in one grid: one launch's fixed cost
// for the batch.  Run r's packet 0 record and packet count (early, written
// by workgroup 0 with the early block) and what follows the run (final,
// copied by the last workgroup) land in the host area after the exceptions.
constexpr uint32_t kSpecRunsMax = 16;
struct SpecRunEarly {
  uint64_t r0[7];           // the run's packet 0 record (stream_off relative to the run's stream)
  uint32_t count;           // packets of the run this launch verifies
  uint32_t early;           // 1: the run's completion is published (SpecRunDone; no pool tiles in it)
};
static_assert(kSpecRunsMax == 16, "SpecCtl's per-run words");
struct SpecRunTail {        // what follows run r (the host area's entry 0 only for per-run completion)
  uint64_t rec[7];
  uint64_t total;
  uint32_t status, seq;     // seq: the launch's, once the entry is in the host area (per-run completion)
};
// Per-run completion of a coalesced batch (SpecArgs::early): the workgroup
// that completes run r (SpecCtl::run_done) publishes its verdict, sequence
// number last.  The host returns a job whose run is done, clean (no
// mismatch) and in the prediction (no header off it) without waiting for
// the rest of the launch.
struct SpecRunDone {
  uint32_t seq, mism, bad, pad;
};
static_assert(sizeof(SpecRunEarly) == 64 && sizeof(SpecRunTail) == 72 && sizeof(SpecRunDone) == 16, "spec run blocks");
constexpr size_t kSpecRunEarlyOff = 256 + size_t(kSpecExcMax) * sizeof(SpecExc);
constexpr size_t kSpecRunTailOff = kSpecRunEarlyOff + size_t(kSpecRunsMax) * sizeof(SpecRunEarly);
constexpr size_t kSpecRunDoneOff = kSpecRunTailOff + size_t(kSpecRunsMax) * sizeof(SpecRunTail);
constexpr size_t kSpecHostBytes = kSpecRunDoneOff + size_t(kSpecRunsMax) * sizeof(SpecRunDone);
// Parameters of the closed-form segment table (SpecTab, crc32c_kernels.hip).
// A batch of runs of `per` packets each: packet k (global) is packet k - r *
// per of run r = k / per (a multiply-high by um = floor(2^64 / per) + 1,
// exact for k < 2^32), whose CRCs start at crc0r[r] + (k - r * per) *
// stride; one run: nruns 1.
struct SpecTabData {
  const uint8_t *crc0;          // packet 0's CRCs
  uint8_t *bm0, *copy_base;
  uint64_t stride, copy_cap;
  uint32_t nch, cs, cb0, nruns; // dataLen = nch * cs (whole chunks), crc_len = 4 * nch
  uint64_t um;
  uint32_t per, pad;
  const uint8_t *crc0r[kSpecRunsMax];
  // per-run completion (a BATCH launch with SpecArgs::early)
  SpecCtl *ctl;
  uint8_t *hdone;               // host area: SpecRunDone[kSpecRunsMax]
  uint32_t seq, pad1;
};
static_assert(sizeof(SpecTabData) == 56 + 16 + 128 + 24, "SpecTabData");
struct SpecArgs {
  const uint8_t *s;
  uint64_t len, base;
  uint32_t max_count;       // grid points the pass may take (max_pkts, kGridMaxCount)
  int proto, ctype;
  uint32_t cs, sflags;
  int rwin;                 // copy-out: client read window from client_offset
  int64_t client_offset;
  uint8_t *bm;              // bitmap area (>= count * T bytes)
  uint8_t *copy_base;       // copy-out destination (null: none)
  uint64_t copy_cap;        // bytes left in it for this pass
  const uint32_t *gtab;     // slicing / zeros tables of the checksum type
  uint32_t *fb;             // first-bad scratch (>= count words; results unused)
  SpecCtl *ctl;             // [2] ring
  SpecExc *exc;             // [2][kSpecExcMax] exception records, by ring slot
  uint32_t parity, seq, tune;
  uint8_t *hout;            // pinned host area (device address): SpecEarly, SpecFinal
  SpecTabData *tabs;        // [gridDim.x] per-workgroup copies of the closed-form table
  // diagnostic build only (null in the release build): per-wave start / end
  // stamps of the work loop at [3 * wave], and per-workgroup phase stamps at
  // [kSpecStampOff + 8 * block + phase] (s_memrealtime, 100 MHz)
  unsigned long long *stamps;
  // batch: runs 1 .. nruns - 1 (run 0 is s + base, len - base), verify only
  // (no read window, no copy-out); max_count caps each run
  uint32_t nruns;
  uint32_t early;           // batch: publish each run's completion (SpecRunDone)
  const uint8_t *xs[kSpecRunsMax];
  uint64_t xlen[kSpecRunsMax];
  SpecRunTail *xtail;       // [2][kSpecRunsMax] by ring slot (device)
};
constexpr size_t kSpecStampOff = 98304;
constexpr uint64_t kSpecMaxStride = uint64_t(1) << 26;  // per-lane header offsets within a wave fit 32 bits

// Compact verify verdict of one packet (grid_finalize_kernel).
struct GridBad {
  uint32_t pkt;
  int32_t first_bad;
  uint32_t bad_chunks;
  uint32_t pad;
};


// LDS image of the tiled kernel (bytes).
//  [0, 128 KiB)          slicing-by-4 tables, each replicated 32x so that
//                        lane l always reads bank l (conflict-free)
//  [128 KiB, +28 KiB)    Z_{64k} byte tables, k = 1..7 (lane combine; k = 7
//                        doubles as the 448-byte jump between rounds)
constexpr uint32_t kLdsSliceBytes = 131072;
constexpr uint32_t kLdsZposBytes = 7 * 4096;
constexpr uint32_t kLdsBytes = kLdsSliceBytes + kLdsZposBytes;  // 159744
constexpr uint32_t kLdsWords = kLdsBytes / 4;

// Global table blob consumed by the kernels (u32 words).
//  [0, 1024)       t0..t3 (t_k at k*256)
//  [1024, 8192)    Z_{64k}[m][e] for k = 1..7 (k-1)*1024 + m*256 + e
constexpr uint32_t kTabSliceWords = 1024;
constexpr uint32_t kTabZposWords = 7 * 1024;
constexpr uint32_t kTabMainWords = kTabSliceWords + kTabZposWords;
// Power-of-two zero operators for the stream combine: Z_{2^b}, b < 48.
constexpr uint32_t kPow2Levels = 48;
constexpr uint32_t kTabPow2Words = kPow2Levels * 1024;

// Multiply-mod constants of the mailbox kernel, per checksum type:
//  [0, 1024)     x^(512 m) mod P, m < 1024 (append 64 m zero bytes)
//  [1024, 1088)  x^(8 r) mod P, r < 64
// reflected polynomials, x^0 at bit 31; both types back to back.
constexpr uint32_t kTabKxWords = 1088;

// One received packet inside a de-framing piece (packet-stream verifier).
// The piece's raw bytes are the wire bytes; the gather kernel copies each
// packet's CRCs to a 4-B aligned CRC arena and its data to a 16-B aligned
// data arena so the verify kernels see ordinary segments.
struct PktDesc {
  uint64_t src_crc;   // piece-relative offset of the packet's CRC bytes (data follows)
  uint64_t dst_data;  // data arena offset (16-B aligned)
  uint64_t dst_crc;   // CRC arena offset (4-B aligned)
  uint32_t dlen;      // data bytes
  uint32_t ncrc;      // CRC words
  uint32_t unit0;     // first gather unit of the packet (piece-relative)
  uint32_t nunits;    // gather units: ceil(dlen / kGatherSlice)
};
constexpr uint32_t kGatherSlice = 65536;  // data bytes per gather workgroup
constexpr uint32_t kHdrWin = 64;          // header-window row bytes (device packet streams)

constexpr uint32_t kGridMaxCount = 65536;  // grid points per device framing pass
constexpr uint32_t kGridGroups = kGridMaxCount / 64 / 64;  // frame_build_kernel: group totals after the block records

// Short device-resident runs (the per-read case): small_run_kernel frames
// and verifies up to kSmallRunMax packets of <= kSmallMax data bytes in ONE
// launch, one workgroup per grid point.  Host area: one kSrSlot-byte slot
// per grid point: the record (56 B), then u32 {status | unsupported << 8,
// first bad chunk, bad chunks, seq} -- seq written last.
constexpr uint32_t kSmallRunMax = 64;
// Delivery of an already verified client read (hdfs_crc32c_reader_next):
// pieces (packet payload bytes at any alignment -> the caller's device
// buffers) in one launch of copy_pieces_kernel.  A piece is cut into units,
// the 16-B aligned blocks of its destination it touches (whole ones stored as
// one dwordx4, its first and last byte by byte); the last workgroup to
// finish (a device counter) publishes the call's sequence number to one
// pinned word.  Up to kCopyPiecesMax pieces travel in the kernel arguments;
// more go in a table of CopyEntry, written in pinned memory and copied to
// device memory ahead of the launch on the same stream, each workgroup
// taking `per` consecutive units from the entry wg0[blockIdx.x] on.
constexpr uint32_t kCopyPiecesMax = 32;
constexpr uint32_t kCopyBlocksMax = 512;    // kernel-argument launches
constexpr uint32_t kCopyTabBlocks = 4096;   // table launches: the kernel's limit
constexpr uint32_t kCopyTabGrid = 1024;     //   and the host's choice
constexpr uint32_t kCopyTabStage = 64;      // table entries a workgroup stages in LDS at a time
struct CopyEntry {
  const uint8_t *src;
  uint8_t *dst;
  uint32_t len, uend;  // uend: cumulative units, as CopyPieces::uend
};
static_assert(sizeof(CopyEntry) == 24, "CopyEntry layout (the mailbox reads it as 6 words)");
struct CopyPieces {
  const uint8_t *src[kCopyPiecesMax];
  uint8_t *dst[kCopyPiecesMax];
  uint32_t len[kCopyPiecesMax];
  uint32_t uend[kCopyPiecesMax];  // cumulative units: piece i covers units [uend[i - 1], uend[i])
  uint32_t n, seq;
  uint32_t *done;                 // pinned, device address: the completion word
  uint32_t *count;                // device: workgroups finished (the last one resets it)
  const CopyEntry *tab;           // table launches: n entries (pinned, device address), then
  const uint32_t *wg0;            //   the first entry of each workgroup
  uint32_t per, total;            //   units per workgroup, all units
  unsigned long long *stamps;     // diagnostic build: [kCopyStampOff + 4 * block + phase]
};
constexpr size_t kCopyStampOff = 110592;
// Units of a piece whose destination starts at d and holds len bytes.
inline uint32_t copy_units(uintptr_t d, uint64_t len) {
  return len ? uint32_t(((d + len + 15u) & ~uintptr_t(15)) - (d & ~uintptr_t(15))) / 16u : 0u;
}
constexpr uint32_t kSrSlot = 128;
constexpr uint32_t kSrHostBytes = kSmallRunMax * kSrSlot;
constexpr uint64_t kSmallRunBytes = uint64_t(kSmallRunMax) * (65536 + 4096);  // streams up to this try it

// Synchronous host-memory calls up to this size (and chunk count) run as one
// small kernel reading pinned host memory (small_chunks_kernel).
constexpr uint32_t kSmallMax = 65536;
constexpr uint32_t kSmallMaxChunks = 2048;

// Mailbox request line (resident small-call kernel): word 2 = chunk_size | flags.
constexpr uint32_t kMbVerifyFlag = 1u << 24, kMbBeFlag = 1u << 25, kMbCrc32Flag = 1u << 26, kMbQuitFlag = 1u << 27;
// device-memory source: its 64-bit address is the word pair after the line
constexpr uint32_t kMbDevFlag = 1u << 28;
// a reader's delivery (hdfs_crc32c_reader_next): word 1 = n <= kCopyPiecesMax
// CopyEntry records staged at the start of the input stage
constexpr uint32_t kMbCopyFlag = 1u << 29;


constexpr uint32_t kRoundBytes = 512;  // sub-chunk handled by 8 lanes per round
constexpr uint32_t kTileChunks = 8;

}  // namespace hdfs_crc32c
