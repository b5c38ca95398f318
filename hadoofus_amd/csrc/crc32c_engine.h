// Engine internals shared by the host translation units of
// libhadoofus_crc32c.so (not part of the public C ABI).
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdarg>
#include <cstddef>
#include <cstdint>
#include <initializer_list>
#include <mutex>
#include <vector>

#include "crc32c_hostpin.h"
#include "crc32c_internal.h"
#include "hadoofus_crc32c.h"

namespace hdfs_crc32c {

// ---- kernel launchers (crc32c_kernels.hip) ----
hipError_t launch_tiles(int mode, int order, int nt, int depth, int streams, int block, int grid,
                        const SegDev *segs, uint32_t nseg, uint64_t total_rounds, uint64_t total_tiles,
                        const uint32_t *gtab, uint32_t *first_bad, unsigned long long *mism,
                        unsigned long long *diag, uint32_t tune, uint32_t *gctr, hipStream_t stream,
                        int copy = 0, int una = 0, const GridSummary *dyn = nullptr, uint32_t utiles = 0,
                        int fuse_generic = 0);
hipError_t launch_probe_read(const uint8_t *p, uint64_t nbytes, uint32_t *out, int grid, int block, int variant,
                             hipStream_t stream);
hipError_t launch_generic(int mode, const SegDev *segs, uint32_t nseg, uint64_t total_gtiles,
                          const uint32_t *gtab, uint32_t *first_bad, unsigned long long *mism,
                          hipStream_t stream, const GridSummary *dyn = nullptr);
hipError_t launch_combine(const uint32_t *raws, uint64_t nraw, uint32_t cs, uint64_t len,
                          const uint32_t *pow2, uint32_t reg0, uint32_t *acc, hipStream_t stream);
hipError_t launch_fill(uint64_t *out, uint64_t nwords, uint64_t seed, uint64_t g0, hipStream_t stream);
hipError_t launch_corrupt(uint8_t *data, uint64_t len, uint32_t cs, uint64_t chunk0, uint64_t modulus,
                          uint64_t bitmul, hipStream_t stream);
hipError_t launch_composite(const SegDev *segs, uint32_t nseg, const uint64_t *run_prefix, uint64_t total_runs,
                            const uint32_t *pow2, uint32_t *out, hipStream_t stream);
hipError_t launch_small_chunks(int mode, const uint8_t *p, uint32_t len, uint32_t exact, uint32_t cs, uint32_t reg0,
                               uint32_t be, const uint32_t *expect, const uint32_t *tab, const uint32_t *kx,
                               uint32_t poly, uint32_t *meta, uint32_t *crcs, uint32_t seq, hipStream_t stream);
hipError_t launch_prep(uint32_t *fb, uint32_t nfb, unsigned long long *mism, uint32_t *gctr, hipStream_t stream);
// The hardware queue a stream's dispatches land on: the AQL queue pointer the
// CP passes the kernel, written to *out (device memory).
hipError_t launch_queue_probe(uint64_t *out, hipStream_t stream);
int stream_queue(hipStream_t s, uint64_t *dq, uint64_t *q);
// Resident mailbox kernel (one workgroup; exits on a quit request or after
// idle_ticks of 10 ns without one; status[0] = (epoch << 1) | alive).
hipError_t launch_mailbox(const uint32_t *req, const uint8_t *in, uint32_t *meta, uint32_t *crcs, const uint32_t *tab0,
                          const uint32_t *tab1, const uint32_t *kx, uint32_t *status, uint32_t epoch, uint32_t seq0,
                          uint32_t idle_ticks, uint32_t exp, hipStream_t stream);
hipError_t launch_gather(const uint8_t *raw, const PktDesc *descs, uint32_t npk, uint32_t units, uint8_t *arena,
                         uint8_t *crc_arena, hipStream_t stream);
// proto 1 / 2: derive the stride from the packet at base (v1 / v2 header)
// and store it in *stride_out; proto 0: rows at the given stride.
hipError_t launch_header_window(const uint8_t *s, uint64_t len, uint64_t base, uint64_t stride, uint32_t count,
                                int proto, uint8_t *out, uint64_t *stride_out, hipStream_t stream);

// device framing of device-resident packet streams (crc32c_kernels.hip)
// frame_build_kernel: one device framing pass (framing, scan, segment table).
// Short device-resident run in one launch (count <= kSmallRunMax grid
// points, one workgroup each); hout: pinned host slots (device address),
// kSrHostBytes.
// Copy-out (copy_dst non-null): each packet delivers frame::read_avail bytes
// (win: the client read window from client_offset; else whole payloads),
// placed by frame::read_place within copy_cap bytes of copy_dst.
// A verified read's next bytes to device buffers (copy_pieces_kernel), grid
// workgroups of 256 threads, <= kCopyBlocksMax.
hipError_t launch_copy_pieces(const CopyPieces &a, int grid, hipStream_t stream);
// The same from a device table, beside a running verify (no LDS, one
// workgroup per CU next to a verify workgroup).
hipError_t launch_copy_beside(const CopyPieces &a, int grid, hipStream_t stream);
hipError_t launch_small_run(const uint8_t *s, uint64_t len, uint32_t count, int proto, uint32_t cs, int ctype,
                            int verify, const uint32_t *tab, const uint32_t *pow2, uint8_t *copy_dst,
                            uint64_t copy_cap, int win, int64_t client_offset, uint8_t *hout, uint32_t seq,
                            hipStream_t stream);
hipError_t launch_frame_grid(const uint8_t *s, uint64_t len, uint64_t base, uint32_t count, int proto, uint32_t cs,
                             int ctype, int verify, uint32_t sflags, uint8_t *bm_base, uint8_t *copy_base,
                             uint64_t copy_cap, int win, int64_t client_offset, GridBufs g, hipStream_t stream,
                             unsigned long long *stamps = nullptr);
// Speculative one-launch verify of a run of equal packets (spec_verify_kernel;
// crc32c_internal.h, SpecArgs): grid workgroups of 1024 threads.
hipError_t launch_spec_verify(const SpecArgs &a, int grid, int copy, hipStream_t stream);
// device-resident packet runs: try spec_verify_kernel first (diagnostic
// build: hdfs_crc32c_set_speculation)
extern int g_spec;
// asynchronous jobs: queue and batch (1), launch at submit (0), hold (2)
extern int g_job_coalesce;
extern int g_job_early;
extern std::atomic<uint64_t> g_job_early_stats[2];
// job slot streams on hardware queues of their own (1) or as placed (0)
extern int g_job_queues;
// diagnostic build: per-wave / per-block s_memrealtime stamps (set_tuning)
extern unsigned long long *g_diag;
// frame_build_kernel's stamps sit after the tiled kernel's per-wave words
// (3 per wave, at most 4 096 waves): 8 per block from this word on
constexpr size_t kFrameStampOff = 65536;
// One workgroup: the bad-packet list to *bad (device) and, with its count and
// then seq, to the pinned host area hsum2 (device address; first host_cap
// entries after 256 bytes).
hipError_t launch_grid_finalize(const SegDev *segs, uint32_t nseg, const uint32_t *seg2pkt, const uint32_t *fb,
                                GridBad *bad, uint32_t bad_cap, GridSummary *sum, uint8_t *hsum2, uint32_t host_cap,
                                uint32_t seq, hipStream_t stream);

// ---- errors ----
extern thread_local char g_err[512];
int fail(int code, const char *fmt, ...);
hipError_t read_device_checks(uint32_t out[3], int reset);
// Diagnostic build: EHIP naming the kernel and line of a device-check
// violation since the last call (then cleared); release build: 0, no work.
int device_checks(const char *call);

#define HIPCHK(expr)                                                                   \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess)                                                              \
      return ::hdfs_crc32c::fail(HDFS_CRC32C_EHIP, "%s: %s (%s:%d)", #expr,            \
                                 hipGetErrorString(e_), __FILE__, __LINE__);           \
  } while (0)

// ---- per-device engine context ----
constexpr int kMaxDev = 64;
constexpr uint32_t kStreamPiece = 4096;          // stream CRC: raw CRC per 4 KiB piece
constexpr size_t kStageCap = size_t(64) << 20;   // host->device staging for one-shots
// small synchronous calls: input = data [0, kSmallMax) + wire CRCs; output =
// kSmallMeta meta words + CRCs
constexpr size_t kSmallIn = kSmallMax + size_t(kSmallMaxChunks) * 4 + 64;
constexpr uint32_t kSmallMeta = 16;
constexpr size_t kSmallOut = (kSmallMeta + size_t(kSmallMaxChunks)) * 4;

// Device buffers of one in-flight packet piece (packet-stream verifier):
// wire bytes, de-framed data / CRC arenas, and the piece's tables
// (descs | segs | first-bad | bitmaps).
struct PieceSlot {
  uint8_t *raw = nullptr, *arena = nullptr, *crc = nullptr, *meta = nullptr;
  size_t raw_cap = 0, arena_cap = 0, crc_cap = 0, meta_cap = 0;
  uint32_t *gctr = nullptr;            // tiled-kernel pool counter
  unsigned long long *mism = nullptr;  // mismatch count
  hipEvent_t copied = nullptr;         // copy stream: wire bytes and tables landed
  hipEvent_t done = nullptr;           // compute stream: slot free again
};

// State of one speculative launch at a time (spec_verify_kernel): the
// control-word ring [2] (zeroed when allocated), per-workgroup table copies,
// the pinned landing area (SpecEarly | SpecFinal | exceptions) and the number
// of launches so far (its parity picks the ring slot).  Asynchronous job
// slots also own a stream and the run's bitmap / first-bad scratch.
// Launches of copy_pieces_kernel (a reader's own, or a device context's):
// the pinned completion word and its sequence number, the device workgroup
// counter, and the pinned entry table of table launches (grown on demand;
// only rewritten once the previous launch has completed).
struct CopyCtl {
  uint32_t *hdone = nullptr, *ddone = nullptr, *count = nullptr;
  uint32_t seq = 0;
  uint8_t *htab = nullptr, *dtab = nullptr;
  size_t tab_cap = 0;
  uint8_t *vtab = nullptr;  // device-memory copy of the table (g_copy_dev_tab)
  size_t vtab_cap = 0;
};

struct SpecSlot {
  SpecCtl *ctl = nullptr;
  SpecExc *exc = nullptr;
  SpecRunTail *xtail = nullptr;  // [2][kSpecRunsMax]: what follows runs 1.. of a batch
  SpecTabData *tabs = nullptr;
  uint8_t *h = nullptr, *hd = nullptr;
  uint64_t n = 0;
  hipStream_t stream = nullptr;
  uint64_t q = 0;  // the hardware queue `stream` landed on (job slots: probed when made)
  uint8_t *scratch = nullptr;
  uint64_t scratch_cap = 0;
};
// asynchronous verify jobs: launches in flight per device (job slots), and
// jobs submitted and not yet waited for per device
constexpr int kMaxJobs = 4;
constexpr size_t kMaxJobsOut = 64;
struct JobQueue;

struct DevCtx {
  // published with release after every field below is set up; the unlocked
  // fast path of ctx_init reads it with acquire
  std::atomic<bool> ready{false};
  int dev = -1;
  int num_cu = 0;
  int num_xcd = 8;  // gfx950 (MI355X): 8 XCDs of 32 CUs; workgroups dealt round-robin
  char arch[64] = "";
  // table sets per checksum type: [0] CRC32C, [1] CRC32 (zlib polynomial)
  uint32_t *d_tab_main_t[2] = {nullptr, nullptr};
  uint32_t *d_tab_pow2_t[2] = {nullptr, nullptr};
  uint32_t *d_tab_kx = nullptr;  // mailbox multipliers, kTabKxWords per type
  hipStream_t stream = nullptr;
  // one-shot scratch (guarded by mu)
  uint8_t *h_stage = nullptr;
  uint8_t *d_stage = nullptr;
  uint32_t *d_raw = nullptr;
  size_t raw_cap = 0;
  SegDev *d_seg = nullptr;
  uint32_t *d_small = nullptr;  // [0] acc, [1] first_bad, [2..3] mismatches
  // small synchronous calls: fine-grained pinned input stage (data, then
  // expected CRCs) and output block (meta words, then CRCs), read / written
  // by small_chunks_kernel directly (no DMA copies); seq = completion number
  uint8_t *h_small_in = nullptr, *dv_small_in = nullptr;
  // large-BAR devices: the input stage is fine-grained VRAM the host writes
  // through the BAR ([0, 256) the mailbox request line, then the stage at
  // h_small_in == dv_small_in), so the kernels read HBM instead of PCIe;
  // null: pinned host memory
  uint8_t *stage_vram = nullptr;
  uint32_t *h_small_out = nullptr, *dv_small_out = nullptr;
  uint32_t small_seq = 0;
  // Work enqueued on `stream` whose completion no call has observed (an
  // asynchronous plan execute): the next synchronous call queries the
  // stream for a fault of it.  Epochs, not a flag (a plan
  // enqueued by another thread after a synchronous call's launch must stay
  // unconfirmed when that call completes): plan_execute bumps queued_epoch
  // AFTER its enqueue; a synchronous call reads queued_epoch BEFORE its
  // launch and, once it sees its own completion word, raises confirmed_epoch
  // to that value -- its kernel ran after everything enqueued before the
  // read, which therefore completed (a fault stops the stream).
  // Back-to-back synchronous calls skip the query (~2 us per launch-path
  // call, profiles/r03/e8).
  std::atomic<uint64_t> queued_epoch{0}, confirmed_epoch{0};
  bool unconfirmed() const {
    return queued_epoch.load(std::memory_order_acquire) != confirmed_epoch.load(std::memory_order_acquire);
  }
  void confirm(uint64_t e) {
    uint64_t cur = confirmed_epoch.load(std::memory_order_acquire);
    while (cur < e && !confirmed_epoch.compare_exchange_weak(cur, e, std::memory_order_acq_rel)) {
    }
  }
  uint64_t stream_queries = 0;  // diagnostic build: queries made (hdfs_crc32c_diag_stream_queries)
  // device CRC scratch of chunk_crcs_to_host (guarded by mu)
  void *d_crc_scratch = nullptr;
  uint64_t crc_scratch_cap = 0;
  // host pipeline (guarded by mu): two staging slots on two streams
  hipStream_t copy_stream = nullptr, comp_stream = nullptr;
  hipEvent_t ev_copy[2] = {nullptr, nullptr}, ev_comp[2] = {nullptr, nullptr};
  uint8_t *p_data[2] = {nullptr, nullptr};
  uint32_t *p_crc[2] = {nullptr, nullptr};
  uint8_t *p_bm[2] = {nullptr, nullptr};
  size_t p_cap = 0;        // bytes per data slot
  size_t p_chunk_cap = 0;  // chunks per CRC slot
  SegDev *p_segs = nullptr;
  uint32_t *p_fb = nullptr;
  uint32_t *p_gctr = nullptr;  // [2], one per slot
  unsigned long long *p_mism = nullptr;
  size_t p_npieces_cap = 0;
  // packet-stream verifier (guarded by mu): two device piece slots and the
  // pinned host tables of one call
  PieceSlot kslot[2];
  uint8_t *k_hmeta = nullptr;
  size_t k_hmeta_cap = 0;
  // device-resident packet streams (guarded by mu): header windows (device
  // rows + pinned host copy) and the verify tables (segs | first-bad | bitmaps)
  uint8_t *w_dev = nullptr, *w_host = nullptr;
  uint32_t w_cap = 0;  // rows
  struct VBatch {
    uint8_t *h = nullptr, *d = nullptr;  // pinned / device tables of one verify batch
    size_t hcap = 0, dcap = 0;
  };
  std::vector<VBatch> v_batch;
  hipStream_t v_stream = nullptr;
  // device framing passes (guarded by mu): device tables of one pass
  // (records | status | segments | seg2pkt | first-bad | summary | bad list |
  // counters | exceptions | bitmaps) and its pinned host landing area
  // (summary + packet 0 + exceptions after framing | summary after verify |
  // bad list)
  struct GridSlot {
    uint8_t *d = nullptr, *h = nullptr;
    size_t dcap = 0, hcap = 0;
    uint8_t *hd = nullptr;  // device address of h (coherent, mapped)
  };
  uint32_t grid_seq = 0;
  // short device runs (small_run_kernel): device scratch + pinned host area
  uint8_t *sr_h = nullptr, *sr_hd = nullptr;
  uint8_t *sr2_h = nullptr, *sr2_hd = nullptr;  // the rest of a stream, launched under a speculative verify
  // its stream: beside the speculative kernel, so it starts on the first CU
  // that kernel frees instead of after its last workgroup
  hipStream_t t_stream = nullptr;
  // AQL queues (amd_queue_t addresses) of stream, t_stream and cp_stream as
  // probed at init: the streams beside the speculative kernel must not share
  // its queue (queue_probe_streams)
  uint64_t q_main = 0, q_tail = 0, q_copy = 0, q_mb = 0;  // (q_mb: the mailbox stream's, once created)
  hipStream_t r_stream = nullptr;  // device framing: record copies of runs with many exceptions
  std::vector<GridSlot> grid;
  // speculative one-launch verify (spec_verify_kernel; guarded by mu): the
  // synchronous calls' slot, and the slots of asynchronous jobs
  // (hdfs_crc32c_verify_packets_submit), each with its own stream and
  // bitmap / first-bad scratch
  SpecSlot spec;
  SpecSlot job_slot[kMaxJobs];
  bool job_busy[kMaxJobs] = {};  // the slot holds a launch not yet collected
  // asynchronous jobs: submitted runs waiting to share one launch, launches
  // in flight (crc32c_packets.cpp; guarded by mu, created on first use)
  JobQueue *jobq = nullptr;
  // client reads into host memory (hdfs_crc32c_read_packets with host
  // iovecs): the device staging the fused copy-out fills before the D2H
  // scatter; rd_mu is held across the verify and the scatter (taken before mu)
  std::mutex rd_mu;
  uint8_t *rd_stage = nullptr;
  uint64_t rd_stage_cap = 0;
  // client reads over several device iovecs: the copy kernel's completion
  // word and table (guarded by mu)
  CopyCtl cp;
  // the copy a scatter read starts beside its verify (copy_beside_kernel)
  // and its stream (guarded by mu)
  CopyCtl cp_beside;
  hipStream_t cp_stream = nullptr;
  // held by a scatter read from before its verify until its copy beside the
  // verify has completed (one such copy in flight per device: its table and
  // completion word are rewritten by the next); taken before mu, try-locked
  // (a concurrent scatter read copies after its verify instead)
  std::mutex beside_mu;
  // readers' copy state, kept for the next reader (a free would synchronise
  // the device, which waits for an open mailbox to idle out)
  std::vector<CopyCtl> cp_pool;
  // opt-in resident mailbox (guarded by mu): pinned request line ([0..3]
  // seq, len, chunk_size | flags, register) and status word ([16])
  bool mb_on = false, mb_alive = false;
  uint32_t *h_mb = nullptr, *dv_mb = nullptr;
  // request line the mailbox polls: in stage_vram when there is one, else
  // h_mb (host-writable view mb_req, device view mb_req_d).  The host never
  // reads VRAM back (uncached BAR reads), so mb_posted shadows the last
  // sequence number written.
  uint32_t *mb_req = nullptr, *mb_req_d = nullptr;
  uint32_t mb_posted = 0;
  hipStream_t mb_stream = nullptr;
  uint32_t mb_epoch = 0, mb_idle_ticks = 0;
  uint64_t mb_calls = 0, mb_launches = 0;
  // streams handed out by hdfs_crc32c_stream_create (non-blocking: they do
  // not serialise with the NULL stream, so device_sync with a mailbox open
  // synchronises each of them)
  std::vector<hipStream_t> user_streams;
  // Workgroups of the bulk (one-workgroup-per-CU) kernels.  With the mailbox
  // resident, one CU per XCD is left out, not one in all: workgroups are dealt
  // to the XCDs round-robin, so a grid of num_cu - 1 still gives the
  // mailbox's XCD one workgroup per CU, and the one that lands after the
  // others waits for the mailbox to idle out (round 5: a reader's open
  // stalled by the idle limit on every read).  num_xcd is the gfx950 part's
  // XCD count (ctx_init admits gfx950 only), not derived from num_cu.
  int bulk_cus() const { return num_cu - (mb_on ? num_xcd : 0); }
  std::mutex mu;
};

extern DevCtx g_ctx[kMaxDev];
// A non-blocking stream whose hardware queue is none of avoid[0..n): a plain
// one if the runtime placed it so, else (g_job_queues) a CU-masked one,
// which the runtime never pools; *q its queue.
int stream_on_own_queue(DevCtx &c, hipStream_t *s, uint64_t *q, const uint64_t *avoid, int n);

struct DeviceGuard {
  int prev = -1;
  bool changed = false;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) == hipSuccess && prev != dev) {
      changed = hipSetDevice(dev) == hipSuccess;
    }
  }
  ~DeviceGuard() {
    if (changed) (void)hipSetDevice(prev);
  }
};

int ctx_init(int device, DevCtx **out);
// Split a segment between the tiled and the generic kernel (prefix indices).
void classify(SegDev &s, uint64_t &rounds, uint64_t &gtiles, uint64_t &mtiles);
int fill_seg(const hdfs_crc32c_segment &in, int mode, SegDev &s, size_t idx);
// Table set of a segment: 0 = CRC32C, 1 = CRC32 (zlib polynomial).
inline int seg_ctype(uint32_t flags) { return (flags & HDFS_CRC32C_SEG_CRC32) ? 1 : 0; }
bool device_accessible(const void *p);
// Enqueue one compute / verify pass (prep + tiled + generic kernels) on st.
int launch_all(DevCtx &c, int mode, const SegDev *d_segs, uint32_t nseg, uint64_t rounds, uint64_t mtiles,
               uint64_t gtiles, uint32_t *d_fb, unsigned long long *d_mism, uint32_t *d_gctr, hipStream_t st,
               hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr, bool reset = true, int ctype = 0,
               bool copy = false, bool gctr_zeroed = false, bool una = false, uint32_t utiles = 0,
               bool runs = false);
// Every segment's main tiles come in whole 8-tile groups (compute mode can
// then run schedule 4: one wave per group, one 256-B CRC store per group).
bool whole_groups(const SegDev *segs, size_t n);
// Main tiles per segment when the table is uniform (every segment but the
// last has the same main_tiles T, the last at most T), else 0.
uint32_t uniform_tiles(const SegDev *segs, size_t n);
// Verify pass over a segment table built on the device (frame_build_kernel):
// sizes read by the kernel from *dyn; grid sized for rounds_ub / gtiles_ub
// (upper bounds).  Schedule 3 with the uniform-table look-up the summary
// enables for runs of equal packets, realigning kernel; the run's generic
// tiles in the same launch.
int launch_verify_dyn(DevCtx &c, const SegDev *d_segs, const GridSummary *dyn, uint64_t rounds_ub, uint64_t gtiles_ub,
                      uint32_t *d_fb, unsigned long long *d_mism, uint32_t *d_gctr, hipStream_t st, int ctype,
                      bool copy);
// The tiled kernel's tune word (schedule-3 group shift, XCD dealing; the
// diagnostic build's store policy).
uint32_t tile_tune();
// spec_verify_kernel: rounds per wave from which the global pool is used
// (tune bits 23:16 of the tiled kernel; 0 there means 32)
extern uint32_t g_spec_pool_min;
// copy_pieces_kernel table launches: fewest units per workgroup; piece table
// in device memory (1) or read from pinned memory (0)
extern uint32_t g_copy_wg_units;
extern int g_copy_dev_tab;
// Any segment whose data is not 4-B aligned (selects the realigning kernel).
bool any_unaligned(const SegDev *segs, size_t n);
// Copy / compute streams, events and the small pipeline buffers.
int pipe_reserve(DevCtx &c, size_t piece, uint32_t cs, size_t npieces);
// A reader's delivery of n <= kCopyPiecesMax pieces through the open mailbox
// (caller holds c.mu, c.mb_on).
int mailbox_copy(DevCtx &c, const CopyEntry *e, uint32_t n);
// Deliveries up to this many bytes go to the open mailbox (one CU copies;
// larger ones launch copy_pieces_kernel).
extern uint64_t g_mb_copy_max;
// the short rest of a stream after a taken run: one short-run launch
extern int g_tail_small;
extern int g_tail_stream;

// One-launch path for synchronous calls on <= kSmallMax bytes
// (small_chunks_kernel or the open mailbox; caller holds c.mu and has staged
// the data in c.h_small_in[0, len), wire CRCs at + kSmallMax for verify,
// unless dsrc names a device source or hsrc / hcrc are given).  ctype: table set (0
// CRC32C, 1 CRC32).  Results: c.h_small_out[0] first bad, [1] mismatches,
// CRCs from c.h_small_out + kSmallMeta.
bool small_ok(uint64_t len, uint64_t cs);
// hsrc (host bytes, len) / hcrc (wire CRCs, crc_bytes): staged by the call.
int small_call(DevCtx &c, int mode, uint32_t len, uint32_t cs, uint32_t reg0, bool be, int ctype,
               const uint8_t *dsrc = nullptr, const uint8_t *hsrc = nullptr, const uint8_t *hcrc = nullptr,
               uint32_t crc_bytes = 0);
// BE per-chunk CRCs (chunk cs; ctype HDFS_CRC32C_CSUM_*) of a host or
// device buffer into host memory.
int chunk_crcs_to_host(const void *data, uint64_t len, uint32_t cs, int ctype, uint32_t *out_be);
int host_pipeline(int mode, const uint8_t *data, uint64_t len, uint32_t cs, uint32_t flags, uint32_t crc_init,
                  void *crcs, uint8_t *bitmap, uint64_t piece_req, uint64_t *first_bad, uint64_t *mismatches);

// Pinned host memory of the host-memory paths (crc32c_hostpin.h): the
// engine's registry, and the pins of one call.  HostPins::pin() pins the
// caller buffers of the call (or finds it pinned: an engine allocation, a
// range another call holds, memory its owner pinned); done(rc) drains the
// streams that may still touch the buffers, then unpins, reporting a failed
// unregistration.  An early return (rc already set, or HIPCHK) drains and
// unpins in the destructor, so no GPU work queued by the call outlives the
// registration of the memory it reads or writes.
PinRegistry &pins();
struct HostPins {
  PinRegistry::Scope s;
  std::vector<hipStream_t> drain;
  bool finished = false;
  explicit HostPins(std::initializer_list<hipStream_t> st) : s(pins()), drain(st) {}
  HostPins(const HostPins &) = delete;
  HostPins &operator=(const HostPins &) = delete;
  ~HostPins() {
    if (!finished)
      for (hipStream_t st : drain)
        if (st) (void)hipStreamSynchronize(st);
  }
  // every host buffer of the call at once (buffers sharing a page become one
  // registration: a DMA never straddles two)
  int pin(std::initializer_list<std::pair<const void *, size_t>> bufs);
  int done(int rc);
};

inline uint64_t align_up(uint64_t v, uint64_t a) { return (v + a - 1) / a * a; }

}  // namespace hdfs_crc32c
