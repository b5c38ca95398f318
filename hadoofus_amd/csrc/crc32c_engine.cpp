// Host engine + C ABI of libhadoofus_crc32c.so (declared in
// include/hadoofus_crc32c.h and include/crc32c.h).
//
// Replaces the reference's CRC32C dispatcher src/crc32c.c:55-110 (ifunc /
// constructor backend selection) with a per-device engine: tables are built
// once per device (the analogue of the constructors src/crc32c_sw.c:73 and
// src/crc32c_sse42.c:204), segment tables are uploaded once per plan, and
// every CRC is computed by the gfx950 kernels in crc32c_kernels.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <chrono>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include <unistd.h>

#include "crc32c_engine.h"
#include "crc32c_tables.h"
#ifdef HDFS_CRC32C_DIAG
#include "hadoofus_crc32c_diag.h"
#endif

namespace hdfs_crc32c {

thread_local char g_err[512] = "";

int fail(int code, const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

DevCtx g_ctx[kMaxDev];
std::mutex g_init_mu;
// Device the engine is bound to by hdfs_crc32c_init(device >= 0) (one
// process per GPU: torchrun ranks bind LOCAL_RANK explicitly); -1 = the
// calling thread's current HIP device.  Explicit, so the engine never
// depends on sharing a HIP runtime (and its current-device state) with torch.
std::atomic<int> g_bound_dev{-1};

// Tiled-kernel launch configuration.  The release build runs the product
// shapes only (schedule 3, nontemporal buffer loads, 3-deep pipeline, one
// tile stream, 1024 threads, 8-tile groups; schedule 2 for small launches)
// and reads nothing from the environment.  The diagnostic build
// (-DHDFS_CRC32C_DIAG) starts from the same values, takes overrides from
// HDFS_CRC32C_* variables and the setters of include/hadoofus_crc32c_diag.h.
#ifdef HDFS_CRC32C_DIAG
int env_int(const char *name, int dflt) {
  const char *e = std::getenv(name);
  return e ? std::atoi(e) : dflt;
}
#define HDFS_KNOB(name, dflt) env_int(name, dflt)
#else
#define HDFS_KNOB(name, dflt) (dflt)
#endif
// Wave -> tile assignment of the tiled kernel (0 static, 1 workgroup-dynamic,
// 2 two-phase contiguous, 3 two-phase interleaved).
int g_tile_order = HDFS_KNOB("HDFS_CRC32C_TILE_ORDER", 3);
// Data-stream loads of the tiled kernel: 0 default policy, 1 nontemporal,
// 2 nontemporal buffer loads (SGPR base + cached per-lane offsets).
int g_nt_loads = HDFS_KNOB("HDFS_CRC32C_NT", 2);
// Rounds in flight per wave + 1 (register buffers of the tiled kernel): 2..4.
int g_depth = HDFS_KNOB("HDFS_CRC32C_DEPTH", 3);
// Tile streams per wave (1, 2, 4) and threads per workgroup (512, 768, 1024).
int g_streams = HDFS_KNOB("HDFS_CRC32C_STREAMS", 1);
int g_block = HDFS_KNOB("HDFS_CRC32C_BLOCK", 1024);
// Result-store policy (diagnostic build only; the release kernel ignores it):
// 0 default, 1 nontemporal, 2 drop compute-mode CRC stores, 3 full-line
// writes, 4 verify plans run the load-only twin.
uint32_t g_store_policy = uint32_t(HDFS_KNOB("HDFS_CRC32C_STORE", 0));
// Schedule 3: log2 tiles per round-robin group (0..6).
uint32_t g_group_shift = uint32_t(HDFS_KNOB("HDFS_CRC32C_GROUP", 3)) & 15u;
// Schedule 3: deal groups XCD-major (1: each XCD sweeps a contiguous window
// of G/8 groups per step), by plain workgroup id (0), or XCD-split (2: each
// XCD sweeps its own contiguous eighth of the launch).
uint32_t g_xcd_major = uint32_t(HDFS_KNOB("HDFS_CRC32C_XCD", 1)) & 3u;
// Speculative verify (spec_verify_kernel): rounds per wave from which the
// launch keeps the last 8 % of its tiles in the global pool (schedule 3's
// two-phase split; the plan kernels use 32).
uint32_t g_spec_pool_min = uint32_t(HDFS_KNOB("HDFS_CRC32C_SPEC_POOL", 32)) & 255u;
// Table launches of copy_pieces_kernel: fewest units per workgroup, and
// whether the piece table is copied to device memory first (1) or read
// over the bus from pinned memory (0).
uint32_t g_copy_wg_units = uint32_t(HDFS_KNOB("HDFS_CRC32C_COPY_WG_UNITS", 1024));
int g_copy_dev_tab = HDFS_KNOB("HDFS_CRC32C_COPY_DEV_TAB", 1);
// (r05 reader_sizes: the resident block copies ~16 GB/s; 64 KiB 7.4 us per
// delivery against 10.5 launched, 256 KiB 19 against 10.6)
// What follows a taken run, when short, in one short-run launch (1) or a
// framing pass (0, diagnostic A/B).
int g_tail_small = HDFS_KNOB("HDFS_CRC32C_TAIL_SMALL", 1);
// the rest queued under a speculative verify: on its own stream (1) or
// behind the kernel on the call's stream (0)
int g_tail_stream = HDFS_KNOB("HDFS_CRC32C_TAIL_STREAM", 1);
uint64_t g_mb_copy_max = uint64_t(HDFS_KNOB("HDFS_CRC32C_MB_COPY_MAX", 96 << 10));
// Compute-mode CRC stores: 2 (product) schedule 3 with the LDS group gather
// (one 256-B store per 8-tile group); diagnostic build only: 1 schedule 4
// on tables of whole groups, 0 one 32-B store per tile
// (profiles/r02/exp_compute_store_schedules.json: 0 / 1 / 2 = 6377 / 6595 /
// 6626 GB/s of algorithmic bytes in one process).
int g_runs = HDFS_KNOB("HDFS_CRC32C_RUNS", 2);
// Device-resident packet runs: try the speculative one-launch verify first
// (spec_verify_kernel; 1, the product) or always frame the run (0,
// diagnostic build only: the A/B of round 4).
int g_spec = HDFS_KNOB("HDFS_CRC32C_SPEC", 1);
// Asynchronous jobs (hdfs_crc32c_verify_packets_submit): 1 (the product)
// queue a job submitted while a launch runs and send the queue out as one
// batch launch; 0 (diagnostic A/B) launch every job at its submit, as round
// 5 did; 2 (diagnostic, deterministic tests) queue even on an idle GPU --
// the queue goes out only when a wait needs it, when full, or on a key change;
// 3 (diagnostic A/B) as 1, but a wait that blocks on a running launch sends
// the queue out behind it only if it holds two runs or more.
int g_job_coalesce = HDFS_KNOB("HDFS_CRC32C_JOB_COALESCE", 1);
// Coalesced batches: 1 (the product) publish each run's completion and
// return a job once its own run is done (a clean run in the prediction); 0
// (diagnostic A/B) jobs return when the whole launch has.
int g_job_early = HDFS_KNOB("HDFS_CRC32C_JOB_EARLY", 1);
// jobs of coalesced batches returned {at their run's completion, at the launch's end}
std::atomic<uint64_t> g_job_early_stats[2];
// Job slot streams: 1 (the product) each on a hardware queue of its own
// (none of the engine stream's or another slot's: two launches on one queue
// run back to back, never side by side); 0 (diagnostic A/B) as the runtime
// places them.
int g_job_queues = HDFS_KNOB("HDFS_CRC32C_JOB_QUEUES", 1);
// Small-call input stage: 1 fine-grained VRAM written through the BAR when
// the device is large-BAR, else (and 0) pinned host memory.
int g_stage_vram = HDFS_KNOB("HDFS_CRC32C_MB_STAGE", 1);
// Mailbox timing experiments (diagnostic build only; see mailbox_kernel).
int g_mb_exp = HDFS_KNOB("HDFS_CRC32C_MB_EXP", 0);
// The resident kernel's stream: 1 a high-priority stream (a hardware queue
// of its own), 0 a normal one (diagnostic: it then shares one of the
// process's GPU_MAX_HW_QUEUES queues with other streams, and every dispatch
// queued behind it there waits for its idle exit)
int g_mb_queue = HDFS_KNOB("HDFS_CRC32C_MB_QUEUE", 1);
// Diagnostic per-wave timestamps (device buffer, 3 x u64 per wave) or null.
unsigned long long *g_diag = nullptr;


// The AQL queue a stream's dispatches land on (one tiny dispatch, waited for).
int stream_queue(hipStream_t s, uint64_t *dq, uint64_t *q) {
  HIPCHK(launch_queue_probe(dq, s));
  HIPCHK(hipMemcpyAsync(q, dq, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  return HDFS_CRC32C_OK;
}

// The streams beside the speculative kernel (t_stream: the short rest of a
// block; cp_stream: a scatter read's copy) must not share c.stream's
// hardware queue, or their work waits behind the kernel it was meant to run
// beside.  The runtime spreads a process's streams over at most
// GPU_MAX_HW_QUEUES queues per priority level (least used first), so which
// queue a stream gets depends on what the host process created before: it
// is probed here (queue_probe_kernel reports the queue a dispatch ran from)
// and a stream on c.stream's queue is replaced by a CU-masked one over every
// CU, which the runtime never pools -- a queue of its own (measured:
// tools/mb_queue_share.py, mailbox stream variant 2).
int stream_on_own_queue(DevCtx &c, hipStream_t *s, uint64_t *q, const uint64_t *avoid, int n) {
  *s = nullptr;
  *q = 0;
  uint64_t *dq = nullptr;
  HIPCHK(hipMalloc(&dq, sizeof(uint64_t)));
  auto shared = [&](uint64_t x) {
    for (int i = 0; i < n; i++)
      if (avoid[i] && avoid[i] == x) return true;
    return false;
  };
  int rc = HDFS_CRC32C_OK;
  if (hipStreamCreateWithFlags(s, hipStreamNonBlocking) != hipSuccess) {
    (void)hipGetLastError();
    *s = nullptr;
    rc = fail(HDFS_CRC32C_EHIP, "stream");
  } else if (!(rc = stream_queue(*s, dq, q)) && g_job_queues && shared(*q)) {
    std::vector<uint32_t> mask(size_t((c.num_cu + 31) / 32), 0u);
    for (int cu = 0; cu < c.num_cu; cu++) mask[size_t(cu / 32)] |= 1u << (cu % 32);
    hipStream_t own = nullptr;
    uint64_t q2 = 0;
    if (hipExtStreamCreateWithCUMask(&own, uint32_t(mask.size()), mask.data()) != hipSuccess) {
      (void)hipGetLastError();
    } else if (!stream_queue(own, dq, &q2) && !shared(q2)) {
      (void)hipStreamDestroy(*s);
      *s = own;
      *q = q2;
    } else {
      (void)hipStreamDestroy(own);
    }
  }
  (void)hipFree(dq);
  return rc;
}

// A replacement that cannot be made leaves the stream as it was (slower
// beside-work, never a failed init).
int queue_probe_streams(DevCtx &c) {
  uint64_t *dq = nullptr;
  HIPCHK(hipMalloc(&dq, sizeof(uint64_t)));
  int rc = stream_queue(c.stream, dq, &c.q_main);
  for (int k = 0; k < 2 && !rc; k++) {
    hipStream_t &s = k == 0 ? c.t_stream : c.cp_stream;
    uint64_t &q = k == 0 ? c.q_tail : c.q_copy;
    if ((rc = stream_queue(s, dq, &q))) break;
    if (q != c.q_main) continue;
    std::vector<uint32_t> mask(size_t((c.num_cu + 31) / 32), 0u);
    for (int cu = 0; cu < c.num_cu; cu++) mask[size_t(cu / 32)] |= 1u << (cu % 32);
    hipStream_t own = nullptr;
    uint64_t q2 = 0;
    if (hipExtStreamCreateWithCUMask(&own, uint32_t(mask.size()), mask.data()) != hipSuccess) {
      (void)hipGetLastError();
      continue;
    }
    if ((rc = stream_queue(own, dq, &q2))) break;
    if (q2 == c.q_main) {
      (void)hipStreamDestroy(own);
      continue;
    }
    (void)hipStreamDestroy(s);
    s = own;
    q = q2;
  }
  (void)hipFree(dq);
  return rc;
}

int ctx_init(int device, DevCtx **out) {
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev <= 0)
    return fail(HDFS_CRC32C_ENODEV, "no HIP device visible (%s)",
                e != hipSuccess ? hipGetErrorString(e) : "count 0");
  if (device < 0) device = g_bound_dev.load(std::memory_order_acquire);
  if (device < 0) {
    if (hipGetDevice(&device) != hipSuccess) device = 0;
  }
  if (device >= ndev || device >= kMaxDev)
    return fail(HDFS_CRC32C_ENODEV, "device %d out of range (%d visible)", device, ndev);
  DevCtx &c = g_ctx[device];
  if (c.ready.load(std::memory_order_acquire)) {
    *out = &c;
    return HDFS_CRC32C_OK;
  }
  std::lock_guard<std::mutex> lk(g_init_mu);
  if (c.ready.load(std::memory_order_relaxed)) {
    *out = &c;
    return HDFS_CRC32C_OK;
  }
  hipDeviceProp_t prop;
  HIPCHK(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(HDFS_CRC32C_ENODEV, "device %d is %s; this engine is built for gfx950 (MI355X) only",
                device, prop.gcnArchName);
  DeviceGuard g(device);
  c.dev = device;
  c.num_cu = prop.multiProcessorCount;
  std::snprintf(c.arch, sizeof(c.arch), "%s", prop.gcnArchName);

  // Tables (cf. the reference's load-time constructors), one set per
  // checksum polynomial: CRC32C and zlib's CRC32 (src/datanode.c:2940-2952).
  for (int ct = 0; ct < 2; ct++) {
    const uint32_t poly = ct == 0 ? kPoly : kPolyZlib;
    std::vector<uint32_t> main(kTabMainWords), pow2(kTabPow2Words);
    uint32_t t[4][256];
    make_slicing4(t, poly);
    std::memcpy(main.data(), t, sizeof(t));
    for (int k = 1; k <= 7; k++)
      zeros_byte_tables(zeros_op(64ull * k, poly), main.data() + kTabSliceWords + (k - 1) * 1024);
    Gf2 op = zeros_op(1, poly);
    for (uint32_t b = 0; b < kPow2Levels; b++) {
      zeros_byte_tables(op, pow2.data() + b * 1024);
      op = op.compose(op);
    }
    HIPCHK(hipMalloc(&c.d_tab_main_t[ct], main.size() * 4));
    HIPCHK(hipMalloc(&c.d_tab_pow2_t[ct], pow2.size() * 4));
    HIPCHK(hipMemcpy(c.d_tab_main_t[ct], main.data(), main.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c.d_tab_pow2_t[ct], pow2.data(), pow2.size() * 4, hipMemcpyHostToDevice));
  }
  {
    std::vector<uint32_t> kx(2 * kTabKxWords);
    make_kx(kx.data(), kPoly);
    make_kx(kx.data() + kTabKxWords, kPolyZlib);
    HIPCHK(hipMalloc(&c.d_tab_kx, kx.size() * 4));
    HIPCHK(hipMemcpy(c.d_tab_kx, kx.data(), kx.size() * 4, hipMemcpyHostToDevice));
  }
  // Blocking stream: it serialises with the legacy NULL stream, so the
  // synchronous helpers (hipMemcpy/hipMemset) see prior plan work.
  HIPCHK(hipStreamCreate(&c.stream));
  // the short rest of a verified stream runs beside the speculative kernel
  // on t_stream, which must not share c.stream's hardware queue (created
  // later, it shared it in a process with more streams and waited behind
  // the kernel again): its queue is probed below (queue_probe_streams)
  HIPCHK(hipStreamCreateWithFlags(&c.t_stream, hipStreamNonBlocking));
  // (and a scatter read's copy beside the same kernel, for the same reason)
  HIPCHK(hipStreamCreateWithFlags(&c.cp_stream, hipStreamNonBlocking));
  HIPCHK(hipHostMalloc(&c.h_stage, kStageCap, hipHostMallocDefault));
  HIPCHK(hipMalloc(&c.d_stage, kStageCap));
  HIPCHK(hipMalloc(&c.d_seg, sizeof(SegDev)));
  HIPCHK(hipMalloc(&c.d_small, 64));  // [0] acc [1] first_bad [2..3] mism [8] pool counter
  if (const int rq = queue_probe_streams(c)) return rq;
  // Small-call input stage.  Large-BAR devices: fine-grained VRAM the host
  // writes through the BAR (64 KiB in ~1.3 us), which the kernels then read
  // from HBM instead of across PCIe; otherwise pinned host memory.
  int large_bar = 0;
  if (g_stage_vram == 1 && hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, device) == hipSuccess &&
      large_bar) {
    void *v = nullptr;
    if (hipExtMallocWithFlags(&v, 256 + kSmallIn, hipDeviceMallocFinegrained) == hipSuccess) {
      c.stage_vram = static_cast<uint8_t *>(v);
      std::memset(c.stage_vram, 0, 256);
      __builtin_ia32_sfence();
      c.h_small_in = c.dv_small_in = c.stage_vram + 256;
    }
  }
  (void)hipGetLastError();
  if (!c.stage_vram) {
    HIPCHK(hipHostMalloc(&c.h_small_in, kSmallIn, hipHostMallocCoherent | hipHostMallocMapped));
    HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void **>(&c.dv_small_in), c.h_small_in, 0));
  }
  HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&c.h_small_out), kSmallOut, hipHostMallocCoherent | hipHostMallocMapped));
  std::memset(c.h_small_out, 0, kSmallOut);
  HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void **>(&c.dv_small_out), c.h_small_out, 0));
  c.ready.store(true, std::memory_order_release);
  *out = &c;
  return HDFS_CRC32C_OK;
}

// Split a segment between the tiled kernel and the generic kernel.
// Tiled: chunk_size a multiple of 512, full chunks only (any data alignment).
// Data alignment the tiled kernel requires.  gfx950 under ROCm serves
// dwordx4 buffer / global loads at any byte address (unaligned access mode),
// so any segment start works: 4-B aligned data runs at the aligned rate,
// byte-unaligned data at ~0.6 of it -- both ~2-3x the one-lane-per-chunk
// generic kernel they used to take (tools/exp_unaligned.py,
// profiles/r01/exp_unaligned.json).  HDFS_CRC32C_ALIGN=16 restores the old
// rule.
static const uintptr_t g_tile_align = uintptr_t(std::max(1, HDFS_KNOB("HDFS_CRC32C_ALIGN", 1)));

void classify(SegDev &s, uint64_t &rounds, uint64_t &gtiles, uint64_t &mtiles) {
  const uint64_t ntiles = (uint64_t(s.nchunks) + kTileChunks - 1) / kTileChunks;
  const bool eligible = s.nchunks > 0 && (reinterpret_cast<uintptr_t>(s.data) % g_tile_align) == 0 &&
                        s.chunk_size % kRoundBytes == 0;
  const bool partial = s.len % s.chunk_size != 0;
  if (eligible) {
    s.main_tiles = static_cast<uint32_t>(partial ? ntiles - 1 : ntiles);
    s.gen_tiles = partial ? 1u : 0u;
  } else {
    s.main_tiles = 0;
    s.gen_tiles = static_cast<uint32_t>(ntiles);
  }
  s.round_start = rounds;
  s.gtile_start = gtiles;
  s.mtile_start = mtiles;
  mtiles += s.main_tiles;
  rounds += uint64_t(s.main_tiles) * (s.chunk_size / kRoundBytes);
  gtiles += s.gen_tiles;
}

int fill_seg(const hdfs_crc32c_segment &in, int mode, SegDev &s, size_t idx) {
  if (in.chunk_size == 0) return fail(HDFS_CRC32C_EINVAL, "segment %zu: chunk_size 0", idx);
  const uint64_t nch = (in.len + in.chunk_size - 1) / in.chunk_size;
  if (nch > 0xFFFFFFF0ull) return fail(HDFS_CRC32C_EINVAL, "segment %zu: too many chunks", idx);
  if (in.len && !in.data) return fail(HDFS_CRC32C_EINVAL, "segment %zu: null data", idx);
  if (nch && !in.crcs) return fail(HDFS_CRC32C_EINVAL, "segment %zu: null crcs", idx);
  if (mode == HDFS_CRC32C_MODE_VERIFY && nch && !in.bitmap)
    return fail(HDFS_CRC32C_EINVAL, "segment %zu: verify needs a bitmap", idx);
  if (mode == HDFS_CRC32C_MODE_VERIFY && (in.flags & HDFS_CRC32C_SEG_RAW))
    return fail(HDFS_CRC32C_EINVAL, "segment %zu: RAW flag is compute-only", idx);
  if (in.flags & ~(HDFS_CRC32C_SEG_BE | HDFS_CRC32C_SEG_RAW | HDFS_CRC32C_SEG_CRC32))
    return fail(HDFS_CRC32C_EINVAL, "segment %zu: unknown flags 0x%x", idx, in.flags);
  std::memset(&s, 0, sizeof(s));
  s.data = static_cast<const uint8_t *>(in.data);
  s.len = in.len;
  s.crcs = static_cast<uint32_t *>(in.crcs);
  s.bitmap = in.bitmap;
  s.chunk_size = in.chunk_size;
  s.flags = in.flags;
  s.nchunks = static_cast<uint32_t>(nch);
  s.reg_init = (in.flags & HDFS_CRC32C_SEG_RAW) ? 0u : ~in.crc_init;
  return HDFS_CRC32C_OK;
}

bool device_accessible(const void *p) {
  if (!p) return true;
  hipPointerAttribute_t a;
  hipError_t e = hipPointerGetAttributes(&a, p);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.devicePointer != nullptr;
}

uint32_t tile_tune() { return (kDiag ? g_store_policy : 0u) | (g_group_shift << 8) | (g_xcd_major << 12); }

int launch_verify_dyn(DevCtx &c, const SegDev *d_segs, const GridSummary *dyn, uint64_t rounds_ub, uint64_t gtiles_ub,
                      uint32_t *d_fb, unsigned long long *d_mism, uint32_t *d_gctr, hipStream_t st, int ctype,
                      bool copy) {
  // grid from the upper bounds of the run's rounds (>= 4 rounds per wave
  // before adding workgroups, as launch_all) and generic tiles (>= 4 claims
  // of 8 per wave): a short run must not make 256 workgroups fill their
  // 156 KiB LDS tables for a handful of tiles
  const uint64_t want = std::max((rounds_ub + 63) / 64, (gtiles_ub + 511) / 512);
  const int grid = int(want < 1 ? 1 : (want > uint64_t(c.bulk_cus()) ? c.bulk_cus() : want));
  (void)d_gctr;  // zeroed by frame_build_kernel
  // schedule 3: a device-framed run is packets of one wire size, so its table
  // is uniform (dyn->utiles, no segment search per tile); the kernel falls
  // back to searching the table when it is not
  const hipError_t le = launch_tiles(kModeVerify, 3, g_nt_loads, 3, 1, 1024, grid, d_segs, 0, 0, 0,
                                     c.d_tab_main_t[ctype], d_fb, d_mism, nullptr,
                                     (kDiag ? g_store_policy : 0u) | (g_group_shift << 8) | (g_xcd_major << 12), d_gctr,
                                     st, copy ? 1 : 0, 1, dyn, 0u, 1);
  if (le == hipErrorInvalidValue) return fail(HDFS_CRC32C_EINVAL, "verify kernel shape not built");
  HIPCHK(le);
  return HDFS_CRC32C_OK;
}

uint32_t uniform_tiles(const SegDev *segs, size_t n) {
  if (!n || !segs[0].main_tiles) return 0;
  const uint32_t T = segs[0].main_tiles;
  for (size_t i = 1; i < n; i++)
    if (i + 1 < n ? segs[i].main_tiles != T : segs[i].main_tiles > T) return 0;
  return T;
}

bool whole_groups(const SegDev *segs, size_t n) {
  uint64_t m = 0;
  for (size_t i = 0; i < n; i++) {
    if (segs[i].main_tiles % kTileChunks) return false;
    m += segs[i].main_tiles;
  }
  return m > 0;
}

bool any_unaligned(const SegDev *segs, size_t n) {
  for (size_t i = 0; i < n; i++)
    if (segs[i].main_tiles && (reinterpret_cast<uintptr_t>(segs[i].data) & 3u)) return true;
  return false;
}

// HDFS_CRC32C_SMALL_RULE=0 (experiments): keep schedule 3 for small launches
// and tables of small segments.
static const int g_small_rule = HDFS_KNOB("HDFS_CRC32C_SMALL_RULE", 1);

// ctype: 0 = CRC32C, 1 = CRC32 (zlib polynomial) -- selects the table set.
int launch_all(DevCtx &c, int mode, const SegDev *d_segs, uint32_t nseg, uint64_t rounds,
               uint64_t mtiles, uint64_t gtiles, uint32_t *d_fb, unsigned long long *d_mism,
               uint32_t *d_gctr, hipStream_t st, hipEvent_t ev0, hipEvent_t ev1, bool reset, int ctype, bool copy,
               bool gctr_zeroed, bool una, uint32_t utiles, bool runs) {
  const bool vreset = mode == kModeVerify && reset;
  uint32_t *gz = (rounds && g_tile_order >= 2 && !gctr_zeroed) ? d_gctr : nullptr;
  if (vreset || gz)
    HIPCHK(launch_prep(vreset ? d_fb : nullptr, vreset ? (nseg ? nseg : 1u) : 0u, vreset ? d_mism : nullptr, gz, st));
  if (rounds) {
    // >= 4 rounds per wave (16 waves per block) before adding blocks: each
    // block pays a ~156 KiB LDS table fill.
    uint64_t want = (rounds + 63) / 64;
    int grid = static_cast<int>(want < 1 ? 1 : (want > uint64_t(c.bulk_cus()) ? c.bulk_cus() : want));
    if (ev0) HIPCHK(hipEventRecord(ev0, st));
    // The interleaved schedule (3) pays a segment look-up whenever a strided
    // tile leaves the current segment: small launches (which also skip the
    // pool) and tables of small segments keep the contiguous slices (2) --
    // unless the table is uniform, where the look-up is a division.
    const bool small = rounds < 32ull * 16u * uint64_t(grid) || (!utiles && mtiles < 2ull * uint64_t(grid) * nseg);
    const bool to_small = g_tile_order == 3 && small && g_small_rule;
    int order = to_small ? 2 : g_tile_order;
    // buffer loads (nt 2) exist for schedules 3 / 4 only; the others use nontemporal global loads
    const int nt = order >= 3 ? g_nt_loads : std::min(g_nt_loads, 1);
    // the small-launch fallback always runs the product's schedule-2 shape
    const int depth = to_small ? 3 : g_depth, streams = to_small ? 1 : g_streams, block = to_small ? 1024 : g_block;
    // compute mode, product shape: schedule 4 (runs, tables of whole 8-tile
    // groups) or schedule 3 with the LDS group gather ("order 5")
    if (order == 3 && mode == kModeCompute && !una && !copy && nt == 2 && (depth == 3 || (kDiag && depth == 4)) &&
        streams == 1 &&
        block == 1024) {
      if (g_runs == 1 && runs) order = 4;
      else if (g_runs == 2) order = 5;
      else if (g_runs == 3) order = 6;  // diagnostic build: the lazy gather
      else if (g_runs == 4) order = runs ? 7 : 5;  // diagnostic build: columns on whole 8-tile groups
    }
    // store policy 4 (diagnostic build): verify plans run the load-only twin
    const int kmode = (kDiag && mode == kModeVerify && g_store_policy == 4) ? int(kModeLoadOnly) : mode;
    const hipError_t le = launch_tiles(kmode, order, nt, depth, streams, block, grid, d_segs, nseg, rounds,
                                       mtiles, c.d_tab_main_t[ctype], d_fb, d_mism, kDiag ? g_diag : nullptr,
                                       (kDiag ? g_store_policy : 0u) | (g_group_shift << 8) | (g_xcd_major << 12),
                                       d_gctr, st, copy ? 1 : 0, una ? 1 : 0, nullptr, order >= 3 ? utiles : 0u);
    if (le == hipErrorInvalidValue)
      return fail(HDFS_CRC32C_EINVAL, "tiled kernel shape (order %d, nt %d, depth %d, streams %d, block %d) is not built",
                  order, nt, depth, streams, block);
    HIPCHK(le);
    if (ev1) HIPCHK(hipEventRecord(ev1, st));
  }
  if (gtiles) HIPCHK(launch_generic(mode, d_segs, nseg, gtiles, c.d_tab_main_t[ctype], d_fb, d_mism, st));
  return HDFS_CRC32C_OK;
}

// CRC of one device buffer continuing from crc (caller holds c.mu).
int stream_crc_locked(DevCtx &c, uint32_t crc, const void *dbuf, uint64_t len, uint32_t *out, int ctype = 0) {
  if (len == 0) {
    *out = crc;
    return HDFS_CRC32C_OK;
  }
  const uint64_t nraw = (len + kStreamPiece - 1) / kStreamPiece;
  if (nraw > c.raw_cap) {
    if (c.d_raw) HIPCHK(hipFree(c.d_raw));
    c.d_raw = nullptr;
    size_t cap = 1024;
    while (cap < nraw) cap *= 2;
    HIPCHK(hipMalloc(&c.d_raw, cap * 4));
    c.raw_cap = cap;
  }
  hdfs_crc32c_segment in = {dbuf, len, kStreamPiece,
                            HDFS_CRC32C_SEG_RAW | (ctype ? HDFS_CRC32C_SEG_CRC32 : 0u), 0, 0, c.d_raw, nullptr};
  SegDev s;
  int rc = fill_seg(in, HDFS_CRC32C_MODE_COMPUTE, s, 0);
  if (rc) return rc;
  uint64_t rounds = 0, gtiles = 0, mtiles = 0;
  classify(s, rounds, gtiles, mtiles);
  HIPCHK(hipMemcpyAsync(c.d_seg, &s, sizeof(s), hipMemcpyHostToDevice, c.stream));
  rc = launch_all(c, kModeCompute, c.d_seg, 1, rounds, mtiles, gtiles, nullptr, nullptr, c.d_small + 8, c.stream,
                  nullptr, nullptr, true, ctype, false, false, any_unaligned(&s, 1));
  if (rc) return rc;
  HIPCHK(hipMemsetAsync(c.d_small, 0, 4, c.stream));
  HIPCHK(launch_combine(c.d_raw, nraw, kStreamPiece, len, c.d_tab_pow2_t[ctype], ~crc, c.d_small, c.stream));
  uint32_t acc = 0;
  HIPCHK(hipMemcpyAsync(&acc, c.d_small, 4, hipMemcpyDeviceToHost, c.stream));
  HIPCHK(hipStreamSynchronize(c.stream));
  *out = ~acc;
  return HDFS_CRC32C_OK;
}

// Small synchronous call (small_chunks_kernel): the caller has written the
// data to h_small_in[0, len) (and for verify the wire CRCs to
// h_small_in[kSmallMax, +4*nch)).  One launch; the host polls the completion
// sequence number the kernel stores to pinned memory after its results
// (a fault is caught by the stream synchronisation the poll falls back to).
bool small_ok(uint64_t len, uint64_t cs) {
  if (!len || len > kSmallMax || !cs) return false;
  const uint64_t nch = (len + cs - 1) / cs;
  return nch <= kSmallMaxChunks && (cs % 4 == 0 || nch == 1);
}

static const bool g_small_trace = std::getenv("HDFS_CRC32C_SMALL_TRACE") != nullptr;

// Mailbox path of small_call: the resident kernel (re)launched if it is not
// running, then one request line; same pinned result block and sequence
// number as the launch path.
int mb_launch(DevCtx &c, uint32_t seq0) {
  c.mb_epoch++;
  __atomic_store_n(&c.h_mb[16], (c.mb_epoch << 1) | 1u, __ATOMIC_RELEASE);
  HIPCHK(launch_mailbox(c.mb_req_d, c.dv_small_in, c.dv_small_out, c.dv_small_out + kSmallMeta, c.d_tab_main_t[0],
                        c.d_tab_main_t[1], c.d_tab_kx, c.dv_mb + 16, c.mb_epoch, seq0, c.mb_idle_ticks,
                        uint32_t(g_mb_exp), c.mb_stream));
  c.mb_alive = true;
  c.mb_launches++;
  return HDFS_CRC32C_OK;
}

// Writes one request line: the fields, then the sequence number the kernel
// polls.  Pinned stage: x86-TSO store order is the order the device sees.
// VRAM stage: the BAR mapping is write-combining, so a store fence drains
// the staged bytes and fields before the sequence number, and a second one
// pushes the sequence number out instead of leaving it in a WC buffer.
void mb_post(DevCtx &c, uint32_t seq, uint32_t len, uint32_t csf, uint32_t reg0, const uint8_t *dsrc) {
  volatile uint32_t *r = c.mb_req;
  r[1] = len;
  r[2] = csf;
  r[3] = reg0;
  if (dsrc) {  // device data is read in place (HBM), any alignment
    r[4] = uint32_t(reinterpret_cast<uintptr_t>(dsrc));
    r[5] = uint32_t(reinterpret_cast<uintptr_t>(dsrc) >> 32);
  }
  if (c.stage_vram) {
    __builtin_ia32_sfence();
    r[0] = seq;
    __builtin_ia32_sfence();
  } else {
    __atomic_store_n(&c.mb_req[0], seq, __ATOMIC_RELEASE);  // staged data and fields first (x86-TSO / release)
  }
  c.mb_posted = seq;
}

bool mb_exited(const DevCtx &c) { return __atomic_load_n(&c.h_mb[16], __ATOMIC_ACQUIRE) == (c.mb_epoch << 1); }

int mb_wait(DevCtx &c, uint32_t seq, std::chrono::steady_clock::time_point t0);

int mailbox_call(DevCtx &c, int mode, uint32_t len, uint32_t cs, uint32_t reg0, bool be, int ctype,
                 const uint8_t *dsrc, const uint8_t *hsrc, const uint8_t *hcrc, uint32_t crc_bytes) {
  const uint32_t seq = ++c.small_seq;
  const auto ta = std::chrono::steady_clock::now();
  if (c.mb_alive && mb_exited(c)) c.mb_alive = false;  // idled out since the last call
  if (!c.mb_alive) {
    const int rc = mb_launch(c, c.mb_posted);
    if (rc) return rc;
  }
  // Staged before the request line.  (Staging 16 KiB pieces behind it with
  // a progress word the waves poll measured slower: 512 B 6.5 -> 7.9 us,
  // 64 KiB verify 9.6 -> 10.4 us -- the extra PCIe poll costs more than the
  // overlap saves.)
  if (hsrc) {
    std::memcpy(c.h_small_in, hsrc, len);
    if (crc_bytes) std::memcpy(c.h_small_in + kSmallMax, hcrc, crc_bytes);
  }
  const uint32_t csf = cs | (mode == kModeVerify ? kMbVerifyFlag : 0u) | (be ? kMbBeFlag : 0u) |
                       (ctype ? kMbCrc32Flag : 0u) | (dsrc ? kMbDevFlag : 0u);
  mb_post(c, seq, len, csf, reg0, dsrc);
  const auto t0 = std::chrono::steady_clock::now();
  const int rc = mb_wait(c, seq, t0);
  if (rc) return rc;
  if (g_small_trace) {  // diagnostic: host staging / wait, kernel phases (diag build, 10 ns ticks)
    const auto t1 = std::chrono::steady_clock::now();
    const uint32_t *m = c.h_small_out;
    std::fprintf(stderr, "mailbox len=%u cs=%u stage_us=%.2f wait_us=%.2f load_us=%.2f comp_us=%.2f\n", len, cs,
                 std::chrono::duration<double, std::micro>(t0 - ta).count(),
                 std::chrono::duration<double, std::micro>(t1 - t0).count(), (m[5] - m[4]) / 100.0,
                 (m[6] - m[5]) / 100.0);
  }
  // a single chunk's CRC came with the completion word (one store)
  if (mode != kModeVerify && len <= cs) c.h_small_out[kSmallMeta] = c.h_small_out[3];
  return HDFS_CRC32C_OK;
}

// A reader's delivery through the open mailbox: n <= kCopyPiecesMax pieces
// staged at the start of the input stage, one request line, the completion
// line awaited as for a small call.  Caller holds c.mu and has checked
// c.mb_on.
int mailbox_copy(DevCtx &c, const CopyEntry *e, uint32_t n) {
  if (!n || n > kCopyPiecesMax) return fail(HDFS_CRC32C_EINVAL, "mailbox copy of %u pieces", n);
  const uint32_t seq = ++c.small_seq;
  if (c.mb_alive && mb_exited(c)) c.mb_alive = false;
  if (!c.mb_alive) {
    const int rc = mb_launch(c, c.mb_posted);
    if (rc) return rc;
  }
  std::memcpy(c.h_small_in, e, size_t(n) * sizeof(CopyEntry));
  mb_post(c, seq, n, kMbCopyFlag, 0u, nullptr);
  return mb_wait(c, seq, std::chrono::steady_clock::now());
}

// Waits for request seq's completion line; relaunches a mailbox that idled
// out before it saw the request.
int mb_wait(DevCtx &c, uint32_t seq, std::chrono::steady_clock::time_point t0) {
  for (uint32_t spin = 1;; spin++) {
    if (__atomic_load_n(&c.h_small_out[2], __ATOMIC_ACQUIRE) == seq) {
      // the completion line is the resident kernel's last memory operation
      // for a request; a fault while serving it ends the kernel before it
      // (caught by the stream query below after 200 ms)
      c.mb_calls++;
      return HDFS_CRC32C_OK;
    }
    if ((spin & 255u) == 0 && mb_exited(c)) {
      // it idled out before it saw the request: a new one serves it
      if (__atomic_load_n(&c.h_small_out[2], __ATOMIC_ACQUIRE) == seq) continue;
      const int rc = mb_launch(c, seq - 1u);
      if (rc) return rc;
    }
    if ((spin & 4095u) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(200)) {
      const hipError_t e = hipStreamQuery(c.mb_stream);
      if (e != hipSuccess && e != hipErrorNotReady) {
        c.mb_alive = false;
        return fail(HDFS_CRC32C_EHIP, "mailbox kernel: %s", hipGetErrorString(e));
      }
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2))
        return fail(HDFS_CRC32C_EHIP, "mailbox kernel did not answer request %u", seq);
    }
#if defined(__x86_64__) || defined(__i386__)
    __builtin_ia32_pause();
#endif
  }
}

// Calls the open mailbox serves (chunk size a multiple of 64, or one chunk:
// chunk size = len, which fits the request line).
bool mb_serves(const DevCtx &c, uint32_t len, uint32_t cs) { return c.mb_on && (cs % 64u == 0 || len <= cs); }

int small_call(DevCtx &c, int mode, uint32_t len, uint32_t cs, uint32_t reg0, bool be, int ctype,
               const uint8_t *dsrc, const uint8_t *hsrc, const uint8_t *hcrc, uint32_t crc_bytes) {
  if (mb_serves(c, len, cs))
    return mailbox_call(c, mode, len, len <= cs ? len : cs, reg0, be, ctype, dsrc, hsrc, hcrc, crc_bytes);
  if (hsrc) {
    std::memcpy(c.h_small_in, hsrc, len);
    if (crc_bytes) std::memcpy(c.h_small_in + kSmallMax, hcrc, crc_bytes);
  }
  // a VRAM stage is write-combining: drain it before the launch
  if (c.stage_vram) __builtin_ia32_sfence();
  const uint32_t seq = ++c.small_seq;
  const uint64_t epoch = c.queued_epoch.load(std::memory_order_acquire);  // before the launch
  const auto tl = std::chrono::steady_clock::now();
  HIPCHK(launch_small_chunks(mode, dsrc ? dsrc : c.dv_small_in, len, dsrc ? 1u : 0u, cs, reg0, be ? 1u : 0u,
                             reinterpret_cast<const uint32_t *>(c.dv_small_in + kSmallMax), c.d_tab_main_t[ctype],
                             c.d_tab_kx + ctype * kTabKxWords, ctype ? kPolyZlib : kPoly, c.dv_small_out,
                             c.dv_small_out + kSmallMeta, seq, c.stream));
  // a fault of EARLIER work on the stream is this call's error, not the next
  // caller's: while work nobody has seen complete is queued before this
  // call's kernel (c.unconfirmed()), one query while the kernel is in flight,
  // so the runtime's bookkeeping of the previous dispatch overlaps the wait
  // (a query after the completion word cost every call ~5 us, one before
  // the launch ~3 us: profiles/r03/e2, e4 small_launch.json)
  if (c.unconfirmed()) {
    if (kDiag) c.stream_queries++;
    if (const hipError_t q = hipStreamQuery(c.stream); q != hipSuccess && q != hipErrorNotReady)
      return fail(HDFS_CRC32C_EHIP, "earlier work on the stream: %s", hipGetErrorString(q));
  }
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t spin = 1;; spin++) {
    if (__atomic_load_n(&c.h_small_out[2], __ATOMIC_ACQUIRE) == seq) {
      // the sequence number is the kernel's last memory operation: a fault of
      // this launch cannot be followed by it, and everything queued before
      // it has completed
      c.confirm(epoch);
      if (g_small_trace) {  // diagnostic: host launch / wait time, kernel phase stamps (10 ns ticks)
        const auto t1 = std::chrono::steady_clock::now();
        const uint32_t *m = c.h_small_out;
        std::fprintf(stderr, "small len=%u cs=%u launch_us=%.2f wait_us=%.2f load_us=%.2f comp_us=%.2f out_us=%.2f\n",
                     len, cs, std::chrono::duration<double, std::micro>(t0 - tl).count(),
                     std::chrono::duration<double, std::micro>(t1 - t0).count(), (m[5] - m[4]) / 100.0,
                     (m[6] - m[5]) / 100.0, (m[7] - m[6]) / 100.0);
      }
      return HDFS_CRC32C_OK;
    }
    if ((spin & 4095u) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(200)) {
      HIPCHK(hipStreamSynchronize(c.stream));
      if (__atomic_load_n(&c.h_small_out[2], __ATOMIC_ACQUIRE) == seq) return HDFS_CRC32C_OK;
      return fail(HDFS_CRC32C_EHIP, "small kernel finished without publishing its result");
    }
#if defined(__x86_64__) || defined(__i386__)
    __builtin_ia32_pause();
#endif
  }
}

int stream_crc_any(uint32_t crc, const void *buf, uint64_t len, uint32_t *out, int ctype = 0) {
  DevCtx *c = nullptr;
  int rc = ctx_init(-1, &c);
  if (rc) return rc;
  DeviceGuard g(c->dev);
  std::lock_guard<std::mutex> lk(c->mu);
  if (len == 0) {
    *out = crc;
    return HDFS_CRC32C_OK;
  }
  if (device_accessible(buf)) {
    // one launch (or the resident mailbox), any source alignment
    if (small_ok(len, len)) {
      rc = small_call(*c, kModeCompute, uint32_t(len), uint32_t(len), ~crc, false, ctype,
                      static_cast<const uint8_t *>(buf));
      if (rc) return rc;
      *out = c->h_small_out[kSmallMeta];
      return HDFS_CRC32C_OK;
    }
    return stream_crc_locked(*c, crc, buf, len, out, ctype);
  }
  if (small_ok(len, len)) {
    // one chunk of len bytes continuing from the caller's register
    rc = small_call(*c, kModeCompute, uint32_t(len), uint32_t(len), ~crc, false, ctype, nullptr,
                    static_cast<const uint8_t *>(buf));
    if (rc) return rc;
    *out = c->h_small_out[kSmallMeta];
    return HDFS_CRC32C_OK;
  }
  const uint8_t *p = static_cast<const uint8_t *>(buf);
  while (len) {
    const size_t n = len < kStageCap ? size_t(len) : kStageCap;
    std::memcpy(c->h_stage, p, n);
    HIPCHK(hipMemcpyAsync(c->d_stage, c->h_stage, n, hipMemcpyHostToDevice, c->stream));
    rc = stream_crc_locked(*c, crc, c->d_stage, n, &crc, ctype);
    if (rc) return rc;
    p += n;
    len -= n;
  }
  *out = crc;
  return HDFS_CRC32C_OK;
}

// HIP side of the pinned-memory registry (crc32c_hostpin.h).
namespace {
struct HipPinBackend final : PinBackend {
  int reg(uintptr_t p, size_t n) override {
    const hipError_t e = hipHostRegister(reinterpret_cast<void *>(p), n, hipHostRegisterDefault);
    if (e == hipSuccess) return kOk;
    (void)hipGetLastError();
    // refused: "already pinned" only if the runtime knows the start as
    // page-locked host memory (the registry then checks both ends of the
    // caller's bytes); anything else is a failure
    return pinned_elsewhere(p) ? kAlready : kFail;
  }
  int unreg(uintptr_t p) override {
    const hipError_t e = hipHostUnregister(reinterpret_cast<void *>(p));
    if (e == hipSuccess) return kOk;
    (void)hipGetLastError();
    return kFail;
  }
  bool pinned_elsewhere(uintptr_t p) override {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, reinterpret_cast<void *>(p)) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    return a.type == hipMemoryTypeHost;
  }
};
HipPinBackend g_pin_backend;
}  // namespace

PinRegistry &pins() {
  static PinRegistry r(&g_pin_backend, size_t(sysconf(_SC_PAGESIZE)));
  return r;
}

int HostPins::pin(std::initializer_list<std::pair<const void *, size_t>> bufs) {
  if (s.acquire(bufs)) return fail(HDFS_CRC32C_EHIP, "%s", pins().last_error());
  return HDFS_CRC32C_OK;
}

int HostPins::done(int rc) {
  for (hipStream_t st : drain) {
    const hipError_t e = st ? hipStreamSynchronize(st) : hipSuccess;
    if (e != hipSuccess && !rc) rc = fail(HDFS_CRC32C_EHIP, "stream: %s", hipGetErrorString(e));
  }
  finished = true;
  if (s.release() && !rc) rc = fail(HDFS_CRC32C_EHIP, "%s", pins().last_error());
  return rc;
}


int pipe_reserve(DevCtx &c, size_t piece, uint32_t cs, size_t npieces) {
  if (!c.copy_stream) {
    HIPCHK(hipStreamCreateWithFlags(&c.copy_stream, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&c.comp_stream, hipStreamNonBlocking));
    for (int b = 0; b < 2; b++) {
      HIPCHK(hipEventCreateWithFlags(&c.ev_copy[b], hipEventDisableTiming));
      HIPCHK(hipEventCreateWithFlags(&c.ev_comp[b], hipEventDisableTiming));
    }
  }
  if (piece > c.p_cap) {
    for (int b = 0; b < 2; b++) {
      if (c.p_data[b]) HIPCHK(hipFree(c.p_data[b]));
      c.p_data[b] = nullptr;
    }
    c.p_cap = 0;
    for (int b = 0; b < 2; b++) HIPCHK(hipMalloc(&c.p_data[b], piece));
    c.p_cap = piece;
  }
  const size_t chunks = (piece + cs - 1) / cs;
  if (chunks > c.p_chunk_cap) {
    for (int b = 0; b < 2; b++) {
      if (c.p_crc[b]) HIPCHK(hipFree(c.p_crc[b]));
      if (c.p_bm[b]) HIPCHK(hipFree(c.p_bm[b]));
      c.p_crc[b] = nullptr;
      c.p_bm[b] = nullptr;
    }
    c.p_chunk_cap = 0;
    for (int b = 0; b < 2; b++) {
      HIPCHK(hipMalloc(&c.p_crc[b], chunks * 4));
      HIPCHK(hipMalloc(&c.p_bm[b], chunks / 8 + 8));
    }
    c.p_chunk_cap = chunks;
  }
  if (npieces > c.p_npieces_cap) {
    if (c.p_segs) HIPCHK(hipFree(c.p_segs));
    if (c.p_fb) HIPCHK(hipFree(c.p_fb));
    c.p_segs = nullptr;
    c.p_fb = nullptr;
    HIPCHK(hipMalloc(&c.p_segs, npieces * sizeof(SegDev)));
    HIPCHK(hipMalloc(&c.p_fb, npieces * sizeof(uint32_t)));
    if (!c.p_mism) HIPCHK(hipMalloc(&c.p_mism, sizeof(unsigned long long)));
    if (!c.p_gctr) HIPCHK(hipMalloc(&c.p_gctr, 64));
    c.p_npieces_cap = npieces;
  }
  return HDFS_CRC32C_OK;
}

// Host-resident pass: pieces of `piece` bytes go H2D on the copy stream into
// one of two device slots while the other slot is verified/computed on the
// compute stream; results go D2H behind each kernel.
int host_pipeline(int mode, const uint8_t *data, uint64_t len, uint32_t cs, uint32_t flags,
                  uint32_t crc_init, void *crcs, uint8_t *bitmap, uint64_t piece_req,
                  uint64_t *first_bad, uint64_t *mismatches) {
  if (first_bad) *first_bad = UINT64_MAX;
  if (mismatches) *mismatches = 0;
  if (!cs) return fail(HDFS_CRC32C_EINVAL, "chunk_size 0");
  if (!len) return HDFS_CRC32C_OK;
  if (!data || !crcs) return fail(HDFS_CRC32C_EINVAL, "null host buffer");
  if (flags & ~(HDFS_CRC32C_SEG_BE | HDFS_CRC32C_SEG_RAW | HDFS_CRC32C_SEG_CRC32))
    return fail(HDFS_CRC32C_EINVAL, "bad flags");
  if (mode == kModeVerify && (flags & HDFS_CRC32C_SEG_RAW)) return fail(HDFS_CRC32C_EINVAL, "RAW is compute-only");
  const uint64_t unit = uint64_t(cs) * 8;  // pieces hold whole tiles: bitmap bytes never straddle
  uint64_t piece = piece_req ? piece_req : (uint64_t(64) << 20);
  piece = piece < unit ? unit : piece / unit * unit;
  const uint64_t nch = (len + cs - 1) / cs;
  if (nch > 0xFFFFFFF0ull) return fail(HDFS_CRC32C_EINVAL, "too many chunks");
  const uint64_t npieces = (len + piece - 1) / piece;
  DevCtx *cp = nullptr;
  int rc = ctx_init(-1, &cp);
  if (rc) return rc;
  DevCtx &c = *cp;
  DeviceGuard g(c.dev);
  std::lock_guard<std::mutex> lk(c.mu);
  rc = pipe_reserve(c, piece, cs, npieces);
  if (rc) return rc;
  // Per-piece descriptors, uploaded once -- BEFORE the caller's buffers are
  // registered: buffers of one call that share a page are one registration
  // spanning the bytes between them (crc32c_hostpin.h), and a heap block of
  // the engine that landed in such a gap would look pinned to the runtime
  // and be DMA-ed as if it were; no engine heap object is copied
  // while the call's pins exist.
  std::vector<SegDev> segs(npieces);
  std::vector<uint64_t> rounds(npieces), mt(npieces), gt(npieces);
  for (uint64_t i = 0; i < npieces; i++) {
    const uint64_t off = i * piece, n = std::min(piece, len - off);
    const int b = int(i & 1);
    hdfs_crc32c_segment in = {c.p_data[b], n, cs, flags, crc_init, 0, c.p_crc[b], c.p_bm[b]};
    rc = fill_seg(in, mode, segs[i], size_t(i));
    if (rc) return rc;
    uint64_t r = 0, m = 0, gg = 0;
    classify(segs[i], r, gg, m);
    rounds[i] = r;
    mt[i] = m;
    gt[i] = gg;
  }
  HIPCHK(hipMemcpyAsync(c.p_segs, segs.data(), npieces * sizeof(SegDev), hipMemcpyHostToDevice, c.comp_stream));
  HIPCHK(hipStreamSynchronize(c.comp_stream));  // the pageable source consumed before any pin exists
  // the caller's buffers stay pinned until both streams are drained, on
  // every return path (an early return drains in the destructor)
  HostPins hp({c.copy_stream, c.comp_stream});
  if ((rc = hp.pin({{data, len}, {crcs, nch * 4}, {mode == kModeVerify ? bitmap : nullptr, (nch + 7) / 8}})))
    return rc;
  if (mode == kModeVerify) {
    HIPCHK(hipMemsetAsync(c.p_fb, 0xFF, npieces * 4, c.comp_stream));
    HIPCHK(hipMemsetAsync(c.p_mism, 0, 8, c.comp_stream));
  }
  HIPCHK(hipEventRecord(c.ev_comp[0], c.comp_stream));
  HIPCHK(hipEventRecord(c.ev_comp[1], c.comp_stream));
  uint8_t *hc = static_cast<uint8_t *>(crcs);
  for (uint64_t i = 0; i < npieces; i++) {
    const int b = int(i & 1);
    const uint64_t off = i * piece, n = std::min(piece, len - off);
    const uint64_t c0 = off / cs, nc = (n + cs - 1) / cs;
    HIPCHK(hipStreamWaitEvent(c.copy_stream, c.ev_comp[b], 0));  // slot free
    HIPCHK(hipMemcpyAsync(c.p_data[b], data + off, n, hipMemcpyHostToDevice, c.copy_stream));
    if (mode == kModeVerify)
      HIPCHK(hipMemcpyAsync(c.p_crc[b], hc + c0 * 4, nc * 4, hipMemcpyHostToDevice, c.copy_stream));
    HIPCHK(hipEventRecord(c.ev_copy[b], c.copy_stream));
    HIPCHK(hipStreamWaitEvent(c.comp_stream, c.ev_copy[b], 0));
    rc = launch_all(c, mode, c.p_segs + i, 1, rounds[i], mt[i], gt[i], c.p_fb + i, c.p_mism, c.p_gctr + b,
                    c.comp_stream, nullptr, nullptr, false, seg_ctype(flags));
    if (rc) return rc;
    if (mode == kModeCompute)
      HIPCHK(hipMemcpyAsync(hc + c0 * 4, c.p_crc[b], nc * 4, hipMemcpyDeviceToHost, c.comp_stream));
    else if (bitmap)
      HIPCHK(hipMemcpyAsync(bitmap + c0 / 8, c.p_bm[b], (nc + 7) / 8, hipMemcpyDeviceToHost, c.comp_stream));
    HIPCHK(hipEventRecord(c.ev_comp[b], c.comp_stream));
  }
  if ((rc = hp.done(HDFS_CRC32C_OK))) return rc;  // both streams drained, buffers unpinned
  if (mode == kModeVerify) {
    std::vector<uint32_t> fb(npieces);
    unsigned long long m = 0;
    HIPCHK(hipMemcpy(fb.data(), c.p_fb, npieces * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(&m, c.p_mism, 8, hipMemcpyDeviceToHost));
    if (mismatches) *mismatches = m;
    for (uint64_t i = 0; i < npieces; i++)
      if (fb[i] != 0xFFFFFFFFu) {
        if (first_bad) *first_bad = i * (piece / cs) + fb[i];
        break;
      }
  }
  return HDFS_CRC32C_OK;
}

// BE per-chunk CRCs of a host or device buffer into HOST memory (the write
// path's packet composer): small host / aligned device buffers in one launch
// of small_chunks_kernel, larger host buffers through the H2D pipeline,
// larger device buffers as one compute pass.
int chunk_crcs_to_host(const void *data, uint64_t len, uint32_t cs, int ctype, uint32_t *out_be) {
  if (!len) return HDFS_CRC32C_OK;
  if (!data || !out_be || !cs) return fail(HDFS_CRC32C_EINVAL, "bad chunk CRC request");
  const uint32_t flags = HDFS_CRC32C_SEG_BE | (ctype == HDFS_CRC32C_CSUM_CRC32 ? HDFS_CRC32C_SEG_CRC32 : 0u);
  const int tset = seg_ctype(flags);
  const uint64_t nch = (len + cs - 1) / cs;
  const bool dev = device_accessible(data);
  if (!dev && !small_ok(len, cs)) {
    // >= 8 pieces per call (4..64 MiB) so the H2D copies overlap the kernels
    const uint64_t piece = std::min<uint64_t>(uint64_t(64) << 20, std::max<uint64_t>(uint64_t(4) << 20, len / 8));
    return host_pipeline(kModeCompute, static_cast<const uint8_t *>(data), len, cs, flags, 0, out_be, nullptr, piece,
                         nullptr, nullptr);
  }
  DevCtx *c = nullptr;
  int rc = ctx_init(-1, &c);
  if (rc) return rc;
  DeviceGuard g(c->dev);
  std::lock_guard<std::mutex> lk(c->mu);
  if (small_ok(len, cs)) {  // device sources at any alignment
    if (!dev) std::memcpy(c->h_small_in, data, size_t(len));
    rc = small_call(*c, kModeCompute, uint32_t(len), cs, 0xFFFFFFFFu, true, tset,
                    dev ? static_cast<const uint8_t *>(data) : nullptr);
    if (rc) return rc;
    std::memcpy(out_be, c->h_small_out + kSmallMeta, size_t(nch) * 4);
    return HDFS_CRC32C_OK;
  }
  if (nch > c->crc_scratch_cap) {  // grown, never shrunk (guarded by mu)
    if (c->d_crc_scratch) HIPCHK(hipFree(c->d_crc_scratch));
    c->d_crc_scratch = nullptr;
    c->crc_scratch_cap = 0;
    HIPCHK(hipMalloc(&c->d_crc_scratch, size_t(nch) * 4));
    c->crc_scratch_cap = nch;
  }
  void *d_out = c->d_crc_scratch;
  hdfs_crc32c_segment in = {data, len, cs, flags, 0, 0, d_out, nullptr};
  SegDev sd;
  rc = fill_seg(in, HDFS_CRC32C_MODE_COMPUTE, sd, 0);
  uint64_t rounds = 0, gtiles = 0, mtiles = 0;
  if (!rc) {
    classify(sd, rounds, gtiles, mtiles);
    hipError_t e = hipMemcpyAsync(c->d_seg, &sd, sizeof(sd), hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) rc = fail(HDFS_CRC32C_EHIP, "segment upload: %s", hipGetErrorString(e));
  }
  if (!rc)
    rc = launch_all(*c, kModeCompute, c->d_seg, 1, rounds, mtiles, gtiles, nullptr, nullptr, c->d_small + 8,
                    c->stream, nullptr, nullptr, true, tset, false, false, any_unaligned(&sd, 1));
  if (!rc) {
    hipError_t e = hipMemcpyAsync(out_be, d_out, size_t(nch) * 4, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) rc = fail(HDFS_CRC32C_EHIP, "chunk CRCs: %s", hipGetErrorString(e));
  }
  return rc;
}

[[noreturn]] void die(const char *who) {
  std::fprintf(stderr, "%s: MI355X CRC32C engine unavailable: %s\n", who, g_err);
  std::abort();
}

int device_checks(const char *call) {
  if (!kDiag) return HDFS_CRC32C_OK;
  static const char *const kName[] = {"check self-test", "frame_build_kernel (framing)", "frame_build_kernel (table)", "header_window_kernel",
                                      "small_run_kernel", "grid_finalize_kernel", "spec_verify_kernel (per-run completion)"};
  uint32_t v[3];
  const hipError_t e = read_device_checks(v, 1);
  if (e != hipSuccess) return fail(HDFS_CRC32C_EHIP, "%s: reading the device checks: %s", call, hipGetErrorString(e));
  if (!v[2]) return HDFS_CRC32C_OK;
  return fail(HDFS_CRC32C_EHIP, "%s: device check failed in %s at crc32c_kernels.hip:%u (%u violations)", call,
              kName[v[0] < 7 ? v[0] : 0], v[1], v[2]);
}

}  // namespace hdfs_crc32c

using namespace hdfs_crc32c;

struct hdfs_crc32c_plan {
  int dev = -1;
  int mode = 0;
  int ctype = 0;  // table set: 0 CRC32C, 1 CRC32 (zlib)
  uint32_t nseg = 0;
  SegDev *d_segs = nullptr;
  uint32_t *d_first_bad = nullptr;
  unsigned long long *d_mism = nullptr;
  uint32_t *d_gctr = nullptr;  // tiled-kernel pool counter (schedule 2)
  uint64_t rounds = 0, mtiles = 0, gtiles = 0, main_bytes = 0, gen_bytes = 0, nchunks = 0;
  bool timing = false;
  bool una = false;  // some tiled segment's data is not 4-B aligned
  uint32_t utiles = 0;  // uniform table: main tiles per segment
  bool runs = false;    // compute plan over whole 8-tile groups (schedule 4)
  std::vector<std::pair<hipEvent_t, hipEvent_t>> events;  // pre-created pool
  size_t next_event = 0;
};

extern "C" {

int hdfs_crc32c_abi_version(void) { return HDFS_CRC32C_ABI_VERSION; }

const char *hdfs_crc32c_last_error(void) { return g_err; }

int hdfs_crc32c_init(int device) {
  DevCtx *c = nullptr;
  const int rc = ctx_init(device, &c);
  if (rc == HDFS_CRC32C_OK && device >= 0) g_bound_dev.store(device, std::memory_order_release);
  return rc;
}

int hdfs_crc32c_bound_device(int *device, char *pci_bus_id, size_t len) {
  DevCtx *c = nullptr;
  int rc = ctx_init(-1, &c);
  if (rc) return rc;
  if (device) *device = c->dev;
  if (pci_bus_id && len) {
    char buf[64] = "";
    HIPCHK(hipDeviceGetPCIBusId(buf, int(sizeof(buf)), c->dev));
    std::snprintf(pci_bus_id, len, "%s", buf);
  }
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_device_info(int device, char *arch, size_t arch_len, int *num_cu) {
  DevCtx *c = nullptr;
  int rc = ctx_init(device, &c);
  if (rc) return rc;
  if (arch && arch_len) std::snprintf(arch, arch_len, "%s", c->arch);
  if (num_cu) *num_cu = c->num_cu;
  return HDFS_CRC32C_OK;
}

uint32_t _hdfs_crc32c(uint32_t crc, const void *buf, unsigned len) {
  uint32_t out = 0;
  if (len == 0) return crc;
  if (stream_crc_any(crc, buf, len, &out)) die("_hdfs_crc32c");
  return out;
}

uint32_t _hdfs_sse42_crc32c(uint32_t crc, const void *buf, unsigned len) {
  uint32_t out = 0;
  if (len == 0) return crc;
  if (stream_crc_any(crc, buf, len, &out)) die("_hdfs_sse42_crc32c");
  return out;
}

uint32_t _hdfs_armv8_crc32c(uint32_t crc, const void *buf, unsigned len) {
  uint32_t out = 0;
  if (len == 0) return crc;
  if (stream_crc_any(crc, buf, len, &out)) die("_hdfs_armv8_crc32c");
  return out;
}

uint32_t _hdfs_sw_crc32c(uint32_t crc, const void *buf, unsigned len) {
  uint32_t out = 0;
  if (len == 0) return crc;
  if (stream_crc_any(crc, buf, len, &out)) die("_hdfs_sw_crc32c");
  return out;
}

int hdfs_crc32c_stream_dev(uint32_t crc, const void *dbuf, uint64_t len, uint32_t *out) {
  if (!out) return fail(HDFS_CRC32C_EINVAL, "null out");
  if (len && !dbuf) return fail(HDFS_CRC32C_EINVAL, "null buffer");
  return stream_crc_any(crc, dbuf, len, out);
}

int hdfs_crc32c_stream_ex(int ctype, uint32_t crc, const void *buf, uint64_t len, uint32_t *out) {
  if (!out) return fail(HDFS_CRC32C_EINVAL, "null out");
  if (len && !buf) return fail(HDFS_CRC32C_EINVAL, "null buffer");
  if (ctype != HDFS_CRC32C_CSUM_CRC32C && ctype != HDFS_CRC32C_CSUM_CRC32)
    return fail(HDFS_CRC32C_EINVAL, "bad checksum type %d", ctype);
  return stream_crc_any(crc, buf, len, out, ctype == HDFS_CRC32C_CSUM_CRC32 ? 1 : 0);
}

int hdfs_crc32c_plan_create(hdfs_crc32c_plan **plan, int mode, const hdfs_crc32c_segment *segs,
                            size_t nseg) {
  if (!plan) return fail(HDFS_CRC32C_EINVAL, "null plan pointer");
  *plan = nullptr;
  if (mode != HDFS_CRC32C_MODE_COMPUTE && mode != HDFS_CRC32C_MODE_VERIFY)
    return fail(HDFS_CRC32C_EINVAL, "bad mode %d", mode);
  if (nseg && !segs) return fail(HDFS_CRC32C_EINVAL, "null segment table");
  if (nseg > 0xFFFFFFF0u) return fail(HDFS_CRC32C_EINVAL, "too many segments");
  DevCtx *c = nullptr;
  int rc = ctx_init(-1, &c);
  if (rc) return rc;
  DeviceGuard g(c->dev);
  std::vector<SegDev> host(nseg ? nseg : 1);
  uint64_t rounds = 0, gtiles = 0, mtiles = 0, main_bytes = 0, gen_bytes = 0, nch = 0;
  const int ctype = nseg ? seg_ctype(segs[0].flags) : 0;
  for (size_t i = 0; i < nseg; i++) {
    rc = fill_seg(segs[i], mode, host[i], i);
    if (rc) return rc;
    if (seg_ctype(segs[i].flags) != ctype)
      return fail(HDFS_CRC32C_EINVAL, "segment %zu: CRC32/CRC32C mixed within one plan", i);
    if (!device_accessible(segs[i].data) || !device_accessible(segs[i].crcs) ||
        !device_accessible(segs[i].bitmap))
      return fail(HDFS_CRC32C_EINVAL, "segment %zu: pointer is not device-accessible memory", i);
    classify(host[i], rounds, gtiles, mtiles);
    const uint64_t mb = std::min<uint64_t>(segs[i].len, uint64_t(host[i].main_tiles) * kTileChunks *
                                                            segs[i].chunk_size);
    main_bytes += mb;
    gen_bytes += segs[i].len - mb;
    nch += host[i].nchunks;
  }
  auto *p = new hdfs_crc32c_plan;
  p->dev = c->dev;
  p->mode = mode;
  p->ctype = ctype;
  p->nseg = static_cast<uint32_t>(nseg);
  p->rounds = rounds;
  p->mtiles = mtiles;
  p->gtiles = gtiles;
  p->main_bytes = main_bytes;
  p->gen_bytes = gen_bytes;
  p->nchunks = nch;
  p->una = any_unaligned(host.data(), nseg);
  p->utiles = uniform_tiles(host.data(), nseg);
  p->runs = mode == HDFS_CRC32C_MODE_COMPUTE && whole_groups(host.data(), nseg);
  hipError_t e = hipMalloc(&p->d_segs, sizeof(SegDev) * host.size());
  if (e == hipSuccess) e = hipMemcpy(p->d_segs, host.data(), sizeof(SegDev) * host.size(), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMalloc(&p->d_first_bad, sizeof(uint32_t) * host.size());
  if (e == hipSuccess) e = hipMalloc(&p->d_mism, sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMalloc(&p->d_gctr, 64);
  if (e != hipSuccess) {
    hdfs_crc32c_plan_destroy(p);
    return fail(HDFS_CRC32C_ENOMEM, "plan allocation: %s", hipGetErrorString(e));
  }
  *plan = p;
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_plan_execute(hdfs_crc32c_plan *p, void *stream) {
  if (!p) return fail(HDFS_CRC32C_EINVAL, "null plan");
  DevCtx &c = g_ctx[p->dev];
  DeviceGuard g(p->dev);
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : c.stream;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (p->timing && p->rounds) {
    if (p->next_event == p->events.size()) {  // pool exhausted: grow (outside any timed loop
      hipEvent_t a, b;                         // when set_timing pre-sized it)
      HIPCHK(hipEventCreate(&a));
      HIPCHK(hipEventCreate(&b));
      p->events.emplace_back(a, b);
    }
    e0 = p->events[p->next_event].first;
    e1 = p->events[p->next_event].second;
    p->next_event++;
  }
  const int rc = launch_all(c, p->mode, p->d_segs, p->nseg, p->rounds, p->mtiles, p->gtiles, p->d_first_bad,
                            p->d_mism, p->d_gctr, st, e0, e1, true, p->ctype, false, false, p->una, p->utiles, p->runs);
  // after the enqueue (failed or not: part of it may be queued), so a
  // synchronous call that read the old epoch cannot confirm this work
  if (st == c.stream) c.queued_epoch.fetch_add(1, std::memory_order_acq_rel);
  return rc;
}

int hdfs_crc32c_plan_results(hdfs_crc32c_plan *p, void *stream, uint32_t *first_bad, size_t nseg,
                             uint64_t *mismatches) {
  if (!p) return fail(HDFS_CRC32C_EINVAL, "null plan");
  if (p->mode != HDFS_CRC32C_MODE_VERIFY) return fail(HDFS_CRC32C_EINVAL, "not a verify plan");
  DevCtx &c = g_ctx[p->dev];
  DeviceGuard g(p->dev);
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : c.stream;
  HIPCHK(hipStreamSynchronize(st));
  if (first_bad && nseg) {
    const size_t n = nseg < p->nseg ? nseg : p->nseg;
    HIPCHK(hipMemcpy(first_bad, p->d_first_bad, n * 4, hipMemcpyDeviceToHost));
  }
  if (mismatches) {
    unsigned long long m = 0;
    HIPCHK(hipMemcpy(&m, p->d_mism, 8, hipMemcpyDeviceToHost));
    *mismatches = m;
  }
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_plan_set_timing(hdfs_crc32c_plan *p, int on) {
  if (!p) return fail(HDFS_CRC32C_EINVAL, "null plan");
  DeviceGuard g(p->dev);
  p->timing = on > 0;
  // on > 1: pre-create that many event pairs so no hipEventCreate runs
  // inside the caller's timed loop.
  while (on > 1 && p->events.size() < size_t(on)) {
    hipEvent_t a, b;
    HIPCHK(hipEventCreate(&a));
    HIPCHK(hipEventCreate(&b));
    p->events.emplace_back(a, b);
  }
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_plan_kernel_ms(hdfs_crc32c_plan *p, double *total_ms, int *launches) {
  if (!p) return fail(HDFS_CRC32C_EINVAL, "null plan");
  DeviceGuard g(p->dev);
  double tot = 0;
  int n = 0;
  for (size_t i = 0; i < p->next_event; i++) {
    auto &ev = p->events[i];
    HIPCHK(hipEventSynchronize(ev.second));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, ev.first, ev.second));
    tot += ms;
    n++;
  }
  p->next_event = 0;
  if (total_ms) *total_ms = tot;
  if (launches) *launches = n;
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_plan_stats(const hdfs_crc32c_plan *p, uint64_t *main_bytes, uint64_t *generic_bytes,
                           uint64_t *nchunks) {
  if (!p) return fail(HDFS_CRC32C_EINVAL, "null plan");
  if (main_bytes) *main_bytes = p->main_bytes;
  if (generic_bytes) *generic_bytes = p->gen_bytes;
  if (nchunks) *nchunks = p->nchunks;
  return HDFS_CRC32C_OK;
}

void hdfs_crc32c_plan_destroy(hdfs_crc32c_plan *p) {
  if (!p) return;
  DeviceGuard g(p->dev);
  for (auto &ev : p->events) {
    (void)hipEventDestroy(ev.first);
    (void)hipEventDestroy(ev.second);
  }
  if (p->d_segs) (void)hipFree(p->d_segs);
  if (p->d_first_bad) (void)hipFree(p->d_first_bad);
  if (p->d_mism) (void)hipFree(p->d_mism);
  if (p->d_gctr) (void)hipFree(p->d_gctr);
  delete p;
}

int hdfs_crc32c_plan_time(hdfs_crc32c_plan *p, void *stream, int iters, double *ms_per_iter) {
  if (!p || iters <= 0) return fail(HDFS_CRC32C_EINVAL, "bad plan/iters");
  DevCtx &c = g_ctx[p->dev];
  DeviceGuard g(p->dev);
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : c.stream;
  hipEvent_t a, b;
  HIPCHK(hipEventCreate(&a));
  HIPCHK(hipEventCreate(&b));
  HIPCHK(hipEventRecord(a, st));
  for (int i = 0; i < iters; i++) {
    int rc = hdfs_crc32c_plan_execute(p, st);
    if (rc) return rc;
  }
  HIPCHK(hipEventRecord(b, st));
  HIPCHK(hipEventSynchronize(b));
  float ms = 0;
  HIPCHK(hipEventElapsedTime(&ms, a, b));
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  if (ms_per_iter) *ms_per_iter = ms / iters;
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_verify_crcdata(const void *crcdata, int32_t chunksize, int32_t crcdlen, int32_t dlen,
                               int ctype, int32_t *first_bad) {
  if (first_bad) *first_bad = -1;
  // The reference ASSERTs ctype is CRC32 or CRC32C (src/datanode.c:2938);
  // CSUM_NULL and unknown types are refused here.
  if (ctype != HDFS_CRC32C_CSUM_CRC32C && ctype != HDFS_CRC32C_CSUM_CRC32)
    return fail(HDFS_CRC32C_EINVAL, "bad checksum type %d", ctype);
  const uint32_t pflag = ctype == HDFS_CRC32C_CSUM_CRC32 ? HDFS_CRC32C_SEG_CRC32 : 0u;
  if (chunksize <= 0 || dlen < 0 || crcdlen < 0)
    return fail(HDFS_CRC32C_ERR_DATANODE_PACKET_SIZE, "bad packet sizes");
  const int64_t nch = (int64_t(dlen) + chunksize - 1) / chunksize;
  if (int64_t(crcdlen) != nch * 4)
    return fail(HDFS_CRC32C_ERR_DATANODE_CRC_LEN, "crcdlen %d != %lld", crcdlen, (long long)(nch * 4));
  if (dlen == 0) return HDFS_CRC32C_OK;
  if (!crcdata) return fail(HDFS_CRC32C_EINVAL, "null packet region");
  const uint8_t *reg = static_cast<const uint8_t *>(crcdata);
  {
    // A packet beyond the one-shot staging (the reference's framing accepts
    // up to 1 GiB, src/datanode.c:2433-2441) goes through the pipelined
    // host path; the region is registered once so its CRC and data parts,
    // which may share a page, are never registered separately.
    const size_t off_crc = (size_t(dlen) + 255) & ~size_t(255);
    const size_t off_bm = off_crc + ((size_t(crcdlen) + 255) & ~size_t(255));
    if (off_bm + size_t((nch + 7) / 8) > kStageCap) {
      HostPins whole({});  // host_pipeline drains its streams before it returns
      int rc = whole.pin({{reg, size_t(crcdlen) + size_t(dlen)}});
      if (rc) return rc;
      uint64_t fb64 = UINT64_MAX, m = 0;
      rc = host_pipeline(kModeVerify, reg + crcdlen, uint64_t(dlen), uint32_t(chunksize), HDFS_CRC32C_SEG_BE | pflag, 0,
                         const_cast<uint8_t *>(reg), nullptr, 0, &fb64, &m);
      if ((rc = whole.done(rc))) return rc;
      if (fb64 != UINT64_MAX) {
        if (first_bad) *first_bad = int32_t(fb64);
        return fail(HDFS_CRC32C_ERR_DATANODE_BAD_CHECKSUM, "chunk %llu: bad checksum", (unsigned long long)fb64);
      }
      return HDFS_CRC32C_OK;
    }
  }
  DevCtx *c = nullptr;
  int rc = ctx_init(-1, &c);
  if (rc) return rc;
  DeviceGuard g(c->dev);
  std::lock_guard<std::mutex> lk(c->mu);
  if (small_ok(uint64_t(dlen), uint64_t(chunksize))) {
    rc = small_call(*c, kModeVerify, uint32_t(dlen), uint32_t(chunksize), 0xFFFFFFFFu, true, seg_ctype(pflag), nullptr,
                    reg + crcdlen, reg, uint32_t(crcdlen));
    if (rc) return rc;
    const uint32_t fb = c->h_small_out[0];
    if (fb != 0xFFFFFFFFu) {
      if (first_bad) *first_bad = int32_t(fb);
      return fail(HDFS_CRC32C_ERR_DATANODE_BAD_CHECKSUM, "chunk %u: bad checksum", fb);
    }
    return HDFS_CRC32C_OK;
  }
  const size_t off_crc = (size_t(dlen) + 255) & ~size_t(255);
  const size_t off_bm = off_crc + ((size_t(crcdlen) + 255) & ~size_t(255));
  const uint8_t *region = static_cast<const uint8_t *>(crcdata);
  std::memcpy(c->h_stage, region + crcdlen, size_t(dlen));  // data (16-B aligned on device)
  std::memcpy(c->h_stage + off_crc, region, size_t(crcdlen));
  HIPCHK(hipMemcpyAsync(c->d_stage, c->h_stage, off_bm, hipMemcpyHostToDevice, c->stream));
  hdfs_crc32c_segment in = {c->d_stage, uint64_t(dlen), uint32_t(chunksize), HDFS_CRC32C_SEG_BE | pflag, 0, 0,
                            c->d_stage + off_crc, c->d_stage + off_bm};
  SegDev s;
  rc = fill_seg(in, HDFS_CRC32C_MODE_VERIFY, s, 0);
  if (rc) return rc;
  uint64_t rounds = 0, gtiles = 0, mtiles = 0;
  classify(s, rounds, gtiles, mtiles);
  HIPCHK(hipMemcpyAsync(c->d_seg, &s, sizeof(s), hipMemcpyHostToDevice, c->stream));
  uint32_t *d_fb = c->d_small + 1;
  auto *d_m = reinterpret_cast<unsigned long long *>(c->d_small + 2);
  rc = launch_all(*c, kModeVerify, c->d_seg, 1, rounds, mtiles, gtiles, d_fb, d_m, c->d_small + 8, c->stream,
                  nullptr, nullptr, true, seg_ctype(pflag));
  if (rc) return rc;
  uint32_t fb = 0;
  HIPCHK(hipMemcpyAsync(&fb, d_fb, 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (fb != 0xFFFFFFFFu) {
    if (first_bad) *first_bad = int32_t(fb);
    return fail(HDFS_CRC32C_ERR_DATANODE_BAD_CHECKSUM, "chunk %u: bad checksum", fb);
  }
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_compose_crcs(const void *const *iov_base, const size_t *iov_len, int iovcnt, size_t total,
                             uint32_t chunk, int ctype, void *crc_be_out) {
  if (chunk == 0) return fail(HDFS_CRC32C_EINVAL, "chunk 0");
  // src/datanode.c:2826 ASSERTs the send checksum is CRC32 or CRC32C.
  if (ctype != HDFS_CRC32C_CSUM_CRC32C && ctype != HDFS_CRC32C_CSUM_CRC32)
    return fail(HDFS_CRC32C_EINVAL, "bad checksum type %d", ctype);
  const uint32_t pflag = ctype == HDFS_CRC32C_CSUM_CRC32 ? HDFS_CRC32C_SEG_CRC32 : 0u;
  if (total == 0) return HDFS_CRC32C_OK;
  if (!iov_base || !iov_len || iovcnt <= 0 || !crc_be_out) return fail(HDFS_CRC32C_EINVAL, "bad iovecs");
  const size_t nch = (total + chunk - 1) / chunk;
  const size_t off_crc = (total + 255) & ~size_t(255);
  DevCtx *c = nullptr;
  int rc = ctx_init(-1, &c);
  if (rc) return rc;
  if (off_crc + nch * 4 > kStageCap) return fail(HDFS_CRC32C_EINVAL, "packet larger than staging");
  DeviceGuard g(c->dev);
  std::lock_guard<std::mutex> lk(c->mu);
  const bool small = small_ok(total, chunk);
  uint8_t *dst = small ? c->h_small_in : c->h_stage;
  size_t have = 0;
  for (int k = 0; k < iovcnt && have < total; k++) {
    const size_t n = iov_len[k] < total - have ? iov_len[k] : total - have;
    if (n && !iov_base[k]) return fail(HDFS_CRC32C_EINVAL, "null iovec %d", k);
    std::memcpy(dst + have, iov_base[k], n);
    have += n;
  }
  if (have != total) return fail(HDFS_CRC32C_EINVAL, "iovecs hold %zu of %zu bytes", have, total);
  if (small) {
    rc = small_call(*c, kModeCompute, uint32_t(total), chunk, 0xFFFFFFFFu, true, seg_ctype(pflag));
    if (rc) return rc;
    std::memcpy(crc_be_out, c->h_small_out + kSmallMeta, nch * 4);
    return HDFS_CRC32C_OK;
  }
  HIPCHK(hipMemcpyAsync(c->d_stage, c->h_stage, total, hipMemcpyHostToDevice, c->stream));
  hdfs_crc32c_segment in = {c->d_stage, total, chunk, HDFS_CRC32C_SEG_BE | pflag, 0, 0, c->d_stage + off_crc,
                            nullptr};
  SegDev s;
  rc = fill_seg(in, HDFS_CRC32C_MODE_COMPUTE, s, 0);
  if (rc) return rc;
  uint64_t rounds = 0, gtiles = 0, mtiles = 0;
  classify(s, rounds, gtiles, mtiles);
  HIPCHK(hipMemcpyAsync(c->d_seg, &s, sizeof(s), hipMemcpyHostToDevice, c->stream));
  rc = launch_all(*c, kModeCompute, c->d_seg, 1, rounds, mtiles, gtiles, nullptr, nullptr, c->d_small + 8, c->stream,
                  nullptr, nullptr, true, seg_ctype(pflag));
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(crc_be_out, c->d_stage + off_crc, nch * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_dev_alloc(void **dptr, uint64_t bytes) {
  DevCtx *c = nullptr;
  int rc = ctx_init(-1, &c);
  if (rc) return rc;
  DeviceGuard g(c->dev);
  hipError_t e = hipMalloc(dptr, bytes ? bytes : 1);
  if (e != hipSuccess) return fail(HDFS_CRC32C_ENOMEM, "hipMalloc(%llu): %s", (unsigned long long)bytes,
                                   hipGetErrorString(e));
  return HDFS_CRC32C_OK;
}

// Helpers below run on the engine's device (DeviceGuard), not on whatever
// device the calling thread's HIP runtime has current.
#define HDFS_ON_ENGINE_DEVICE()         \
  DevCtx *ec_ = nullptr;                \
  if (int rc_ = ctx_init(-1, &ec_)) return rc_; \
  DeviceGuard eg_(ec_->dev)

int hdfs_crc32c_dev_free(void *dptr) {
  HDFS_ON_ENGINE_DEVICE();
  HIPCHK(hipFree(dptr));
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_memcpy(void *dst, const void *src, uint64_t bytes, int kind) {
  hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice : kind == 1 ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
  HDFS_ON_ENGINE_DEVICE();
  HIPCHK(hipMemcpy(dst, src, bytes, k));
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_memset(void *dptr, int value, uint64_t bytes) {
  HDFS_ON_ENGINE_DEVICE();
  HIPCHK(hipMemset(dptr, value, bytes));
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_stream_create(void **stream) {
  DevCtx *c = nullptr;
  int rc = ctx_init(-1, &c);
  if (rc) return rc;
  DeviceGuard g(c->dev);
  hipStream_t s;
  HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  {
    std::lock_guard<std::mutex> lk(c->mu);
    c->user_streams.push_back(s);
  }
  *stream = s;
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_stream_destroy(void *stream) {
  HDFS_ON_ENGINE_DEVICE();
  {
    std::lock_guard<std::mutex> lk(ec_->mu);
    auto &v = ec_->user_streams;
    v.erase(std::remove(v.begin(), v.end(), static_cast<hipStream_t>(stream)), v.end());
  }
  HIPCHK(hipStreamDestroy(static_cast<hipStream_t>(stream)));
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_stream_sync(void *stream) {
  HDFS_ON_ENGINE_DEVICE();
  HIPCHK(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_fill_splitmix64(void *dptr, uint64_t nwords, uint64_t seed, uint64_t g0, void *stream) {
  HDFS_ON_ENGINE_DEVICE();
  HIPCHK(launch_fill(static_cast<uint64_t *>(dptr), nwords, seed, g0, static_cast<hipStream_t>(stream)));
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_corrupt(void *dptr, uint64_t len, uint32_t chunk, uint64_t chunk0, uint64_t modulus,
                        uint64_t bitmul, void *stream) {
  if (!chunk || !modulus) return fail(HDFS_CRC32C_EINVAL, "chunk/modulus 0");
  if (!len) return HDFS_CRC32C_OK;
  HDFS_ON_ENGINE_DEVICE();
  HIPCHK(launch_corrupt(static_cast<uint8_t *>(dptr), len, chunk, chunk0, modulus, bitmul,
                        static_cast<hipStream_t>(stream)));
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_compute_host(const void *data, uint64_t len, uint32_t chunk_size, uint32_t flags,
                              uint32_t crc_init, void *crcs_out, uint64_t piece_bytes) {
  return host_pipeline(kModeCompute, static_cast<const uint8_t *>(data), len, chunk_size, flags, crc_init,
                       crcs_out, nullptr, piece_bytes, nullptr, nullptr);
}

int hdfs_crc32c_verify_host(const void *data, uint64_t len, uint32_t chunk_size, uint32_t flags,
                             uint32_t crc_init, const void *crcs, uint8_t *bitmap_out, uint64_t piece_bytes,
                             uint64_t *first_bad, uint64_t *mismatches) {
  return host_pipeline(kModeVerify, static_cast<const uint8_t *>(data), len, chunk_size, flags, crc_init,
                       const_cast<void *>(crcs), bitmap_out, piece_bytes, first_bad, mismatches);
}

int hdfs_crc32c_host_alloc(void **p, uint64_t bytes) {
  DevCtx *c = nullptr;
  int rc = ctx_init(-1, &c);
  if (rc) return rc;
  DeviceGuard g(c->dev);
  hipError_t e = hipHostMalloc(p, bytes ? bytes : 1, hipHostMallocDefault);
  if (e != hipSuccess) return fail(HDFS_CRC32C_ENOMEM, "hipHostMalloc(%llu): %s", (unsigned long long)bytes,
                                   hipGetErrorString(e));
  pins().add_owned(*p, bytes ? bytes : 1);  // the host paths DMA it in place
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_host_free(void *p) {
  HDFS_ON_ENGINE_DEVICE();
  if (p && !pins().remove_owned(p)) return fail(HDFS_CRC32C_EINVAL, "%p is not a hdfs_crc32c_host_alloc block", p);
  HIPCHK(hipHostFree(p));
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_device_sync(void) {
  HDFS_ON_ENGINE_DEVICE();
  if (!ec_->mb_on) {
    HIPCHK(hipDeviceSynchronize());
    return HDFS_CRC32C_OK;
  }
  // a resident mailbox kernel never finishes while it is in use: every
  // stream but its own -- the engine's, the NULL stream and the caller's
  // streams from hdfs_crc32c_stream_create (non-blocking, so the NULL
  // stream does not order them)
  std::lock_guard<std::mutex> lk(ec_->mu);
  HIPCHK(hipStreamSynchronize(nullptr));
  for (hipStream_t s : {ec_->stream, ec_->v_stream, ec_->r_stream, ec_->copy_stream, ec_->comp_stream})
    if (s) HIPCHK(hipStreamSynchronize(s));
  for (hipStream_t s : ec_->user_streams) HIPCHK(hipStreamSynchronize(s));
  return HDFS_CRC32C_OK;
}

struct hdfs_crc32c_mailbox {
  int dev;
};

int hdfs_crc32c_mailbox_create(hdfs_crc32c_mailbox **mb, uint32_t idle_ms) {
  if (!mb) return fail(HDFS_CRC32C_EINVAL, "null mailbox pointer");
  *mb = nullptr;
  DevCtx *c = nullptr;
  int rc = ctx_init(-1, &c);
  if (rc) return rc;
  DeviceGuard g(c->dev);
  std::lock_guard<std::mutex> lk(c->mu);
  if (c->mb_on) return fail(HDFS_CRC32C_EINVAL, "a mailbox is already open on device %d", c->dev);
  if (!c->h_mb) {
    HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&c->h_mb), 256, hipHostMallocCoherent | hipHostMallocMapped));
    std::memset(c->h_mb, 0, 256);
    HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void **>(&c->dv_mb), c->h_mb, 0));
  }
  if (!c->mb_req) {
    if (c->stage_vram) {
      c->mb_req = c->mb_req_d = reinterpret_cast<uint32_t *>(c->stage_vram);
    } else {
      c->mb_req = c->h_mb;
      c->mb_req_d = c->dv_mb;
    }
    c->mb_posted = 0;
  }
  if (!c->mb_stream) {
    // A persistent kernel must not share a hardware queue: the runtime maps
    // a process's normal-priority streams onto at most GPU_MAX_HW_QUEUES
    // (4) queues, and a dispatch queued behind the resident kernel on its
    // queue -- a verify on c.stream, say -- waits for its idle exit (50 ms:
    // measured as a 50 ms stall per reader in some processes).  High-priority
    // streams come from a queue pool of their own, where the mailbox is the
    // only one.
    int lo = 0, hi = 0;
    if (g_mb_queue == 2) {  // diagnostic: a CU-masked stream (all CUs), which the runtime never pools
      std::vector<uint32_t> mask(size_t((c->num_cu + 31) / 32), 0u);
      for (int cu = 0; cu < c->num_cu; cu++) mask[size_t(cu / 32)] |= 1u << (cu % 32);
      HIPCHK(hipExtStreamCreateWithCUMask(&c->mb_stream, uint32_t(mask.size()), mask.data()));
    } else if (g_mb_queue && hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess && hi != lo) {
      HIPCHK(hipStreamCreateWithPriority(&c->mb_stream, hipStreamNonBlocking, hi));
    } else {
      HIPCHK(hipStreamCreateWithFlags(&c->mb_stream, hipStreamNonBlocking));
    }
  }
  if (!c->q_mb) {  // (diagnostics: the queue the resident kernel lands on)
    uint64_t *dq = nullptr;
    HIPCHK(hipMalloc(&dq, sizeof(uint64_t)));
    rc = stream_queue(c->mb_stream, dq, &c->q_mb);
    (void)hipFree(dq);
    if (rc) return rc;
  }
  const uint64_t ms = idle_ms ? idle_ms : 50u;
  c->mb_idle_ticks = uint32_t(std::min<uint64_t>(ms * 100000u, 0xFFFFFFFFu));  // s_memrealtime: 100 MHz
  c->mb_calls = c->mb_launches = 0;
  // the bulk kernels' next launches leave the mailbox its CU
  HIPCHK(hipStreamSynchronize(c->stream));
  c->mb_on = true;
  rc = mb_launch(*c, c->mb_posted);
  if (rc) {
    c->mb_on = false;
    return rc;
  }
  *mb = new hdfs_crc32c_mailbox{c->dev};
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_mailbox_stats(const hdfs_crc32c_mailbox *mb, uint64_t *calls, uint64_t *launches) {
  if (!mb) return fail(HDFS_CRC32C_EINVAL, "null mailbox");
  DevCtx &c = g_ctx[mb->dev];
  std::lock_guard<std::mutex> lk(c.mu);
  if (calls) *calls = c.mb_calls;
  if (launches) *launches = c.mb_launches;
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_mailbox_destroy(hdfs_crc32c_mailbox *mb) {
  if (!mb) return HDFS_CRC32C_OK;
  DevCtx &c = g_ctx[mb->dev];
  DeviceGuard g(mb->dev);
  delete mb;
  std::lock_guard<std::mutex> lk(c.mu);
  if (!c.mb_on) return HDFS_CRC32C_OK;
  c.mb_on = false;
  if (c.mb_alive && !mb_exited(c)) {  // a quit request; the kernel acknowledges through its status word
    mb_post(c, ++c.small_seq, 0u, kMbQuitFlag, 0u, nullptr);
  }
  c.mb_alive = false;
  HIPCHK(hipStreamSynchronize(c.mb_stream));
  return HDFS_CRC32C_OK;
}

#ifdef HDFS_CRC32C_DIAG
// ---- diagnostic build only (include/hadoofus_crc32c_diag.h) ----
int hdfs_crc32c_diag_device_checks(uint32_t *out3, int reset) {
  if (!out3) return fail(HDFS_CRC32C_EINVAL, "null output");
  const hipError_t e = read_device_checks(out3, reset);
  if (e != hipSuccess) return fail(HDFS_CRC32C_EHIP, "reading the device checks: %s", hipGetErrorString(e));
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_set_store_policy(int policy) {
  if (policy < 0 || policy > 28) return fail(HDFS_CRC32C_EINVAL, "store policy 0..28");
  g_store_policy = uint32_t(policy);
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_diag_stream_queries(uint64_t *out) {
  DevCtx *c = nullptr;
  int rc = ctx_init(-1, &c);
  if (rc) return rc;
  if (!out) return fail(HDFS_CRC32C_EINVAL, "null out");
  *out = c->stream_queries;
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_diag_stream_queues(uint64_t *out4) {
  DevCtx *c = nullptr;
  int rc = ctx_init(-1, &c);
  if (rc) return rc;
  if (!out4) return fail(HDFS_CRC32C_EINVAL, "null out");
  out4[0] = c->q_main;
  out4[1] = c->q_tail;
  out4[2] = c->q_copy;
  out4[3] = c->q_mb;
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_set_speculation(int on) {
  if (on != 0 && on != 1) return fail(HDFS_CRC32C_EINVAL, "speculation 0 or 1");
  g_spec = on;
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_diag_job_queues(uint64_t *out4) {
  DevCtx *c = nullptr;
  int rc = ctx_init(-1, &c);
  if (rc) return rc;
  if (!out4) return fail(HDFS_CRC32C_EINVAL, "null out");
  std::lock_guard<std::mutex> lk(c->mu);
  for (int i = 0; i < kMaxJobs; i++) out4[i] = c->job_slot[i].q;
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_set_job_coalesce(int mode) {
  if (mode < 0 || mode > 3)
    return fail(HDFS_CRC32C_EINVAL, "job coalescing 0 (off), 1 (product), 2 (hold) or 3 (no lone run behind a launch)");
  g_job_coalesce = mode;
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_set_job_early(int on) {
  if (on < 0 || on > 1) return fail(HDFS_CRC32C_EINVAL, "per-run completion 0 (off) or 1 (product)");
  g_job_early = on;
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_diag_job_early(uint64_t *out2, int reset) {
  if (!out2) return fail(HDFS_CRC32C_EINVAL, "null out");
  for (int i = 0; i < 2; i++) out2[i] = reset ? g_job_early_stats[i].exchange(0) : g_job_early_stats[i].load();
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_set_runs(int on) {
  if (on < 0 || on > 4)
    return fail(HDFS_CRC32C_EINVAL, "runs 0 (schedule 3), 1 (schedule 4), 2 (gather), 3 (lazy gather) or 4 (columns)");
  g_runs = on;
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_set_depth(int depth) {
  if (depth < 2 || depth > 4) return fail(HDFS_CRC32C_EINVAL, "depth must be 2..4");
  g_depth = depth;
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_set_shape(int streams, int block) {
  if (streams != 1 && streams != 2 && streams != 4) return fail(HDFS_CRC32C_EINVAL, "streams must be 1, 2 or 4");
  if (block != 512 && block != 768 && block != 1024) return fail(HDFS_CRC32C_EINVAL, "block must be 512, 768 or 1024");
  g_streams = streams;
  g_block = block;
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_set_tuning(int nt_loads, void *diag) {
  if (nt_loads < 0 || nt_loads > 2) return fail(HDFS_CRC32C_EINVAL, "nt_loads 0..2");
  g_nt_loads = nt_loads;
  g_diag = static_cast<unsigned long long *>(diag);
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_set_group_shift(int shift) {
  if (shift < 0 || shift > 6) return fail(HDFS_CRC32C_EINVAL, "group shift must be 0..6");
  g_group_shift = uint32_t(shift);
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_set_xcd_major(int on) {
  if (on < 0 || on > 2) return fail(HDFS_CRC32C_EINVAL, "xcd_major must be 0, 1 or 2");
  g_xcd_major = uint32_t(on);
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_set_tile_order(int order) {
  if (order < 0 || order > 3) return fail(HDFS_CRC32C_EINVAL, "tile order must be 0..3");
  g_tile_order = order;
  return HDFS_CRC32C_OK;
}

int g_probe_variant = 0, g_probe_grid_per_cu = 2, g_probe_block = 1024;

int hdfs_crc32c_set_probe(int variant, int grid_per_cu, int block) {
  g_probe_variant = variant;
  g_probe_grid_per_cu = grid_per_cu > 0 ? grid_per_cu : 2;
  g_probe_block = block > 0 ? block : 1024;
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_probe_read(const void *dptr, uint64_t bytes, void *stream, int iters, double *gbps) {
  if (!dptr || !bytes || iters <= 0 || !gbps) return fail(HDFS_CRC32C_EINVAL, "bad probe args");
  DevCtx *c = nullptr;
  int rc = ctx_init(-1, &c);
  if (rc) return rc;
  DeviceGuard g(c->dev);
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : c->stream;
  hipEvent_t a, b;
  HIPCHK(hipEventCreate(&a));
  HIPCHK(hipEventCreate(&b));
  HIPCHK(launch_probe_read(static_cast<const uint8_t *>(dptr), bytes, c->d_small, c->num_cu * g_probe_grid_per_cu,
                           g_probe_block, g_probe_variant, st));
  HIPCHK(hipEventRecord(a, st));
  for (int i = 0; i < iters; i++)
    HIPCHK(launch_probe_read(static_cast<const uint8_t *>(dptr), bytes, c->d_small, c->num_cu * g_probe_grid_per_cu,
                           g_probe_block, g_probe_variant, st));
  HIPCHK(hipEventRecord(b, st));
  HIPCHK(hipEventSynchronize(b));
  float ms = 0;
  HIPCHK(hipEventElapsedTime(&ms, a, b));
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  *gbps = double(bytes) * iters / (ms * 1e-3) / 1e9;
  return HDFS_CRC32C_OK;
}
#endif  // HDFS_CRC32C_DIAG

int hdfs_crc32c_composite_crcs(const hdfs_crc32c_segment *segs, size_t nseg, uint32_t *out) {
  if (nseg && (!segs || !out)) return fail(HDFS_CRC32C_EINVAL, "null segments / out");
  if (nseg > 0xFFFFFFF0u) return fail(HDFS_CRC32C_EINVAL, "too many segments");
  if (!nseg) return HDFS_CRC32C_OK;
  DevCtx *cp = nullptr;
  int rc = ctx_init(-1, &cp);
  if (rc) return rc;
  DevCtx &c = *cp;
  DeviceGuard g(c.dev);
  const int ctype = seg_ctype(segs[0].flags);
  std::vector<SegDev> host(nseg);
  std::vector<uint64_t> prefix(nseg);
  uint64_t runs = 0;
  for (size_t i = 0; i < nseg; i++) {
    rc = fill_seg(segs[i], HDFS_CRC32C_MODE_COMPUTE, host[i], i);
    if (rc) return rc;
    if (seg_ctype(segs[i].flags) != ctype)
      return fail(HDFS_CRC32C_EINVAL, "segment %zu: CRC32/CRC32C mixed in one call", i);
    if (segs[i].crc_init && !(segs[i].flags & HDFS_CRC32C_SEG_RAW))
      return fail(HDFS_CRC32C_EINVAL, "segment %zu: composite needs chunk CRCs started from 0", i);
    if (segs[i].len && !device_accessible(segs[i].crcs))
      return fail(HDFS_CRC32C_EINVAL, "segment %zu: crcs is not device-accessible memory", i);
    prefix[i] = runs;
    runs += (uint64_t(host[i].nchunks) + 63) / 64;
  }
  std::lock_guard<std::mutex> lk(c.mu);
  SegDev *d_segs = nullptr;
  uint64_t *d_prefix = nullptr;
  uint32_t *d_out = nullptr;
  hipError_t e = hipMalloc(&d_segs, nseg * sizeof(SegDev));
  if (e == hipSuccess) e = hipMalloc(&d_prefix, nseg * 8);
  if (e == hipSuccess) e = hipMalloc(&d_out, nseg * 4);
  if (e == hipSuccess) e = hipMemcpyAsync(d_segs, host.data(), nseg * sizeof(SegDev), hipMemcpyHostToDevice, c.stream);
  if (e == hipSuccess) e = hipMemcpyAsync(d_prefix, prefix.data(), nseg * 8, hipMemcpyHostToDevice, c.stream);
  if (e == hipSuccess) e = hipMemsetAsync(d_out, 0, nseg * 4, c.stream);
  if (e == hipSuccess)
    e = launch_composite(d_segs, uint32_t(nseg), d_prefix, runs, c.d_tab_pow2_t[ctype], d_out, c.stream);
  if (e == hipSuccess) e = hipMemcpyAsync(out, d_out, nseg * 4, hipMemcpyDefault, c.stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c.stream);
  if (d_segs) (void)hipFree(d_segs);
  if (d_prefix) (void)hipFree(d_prefix);
  if (d_out) (void)hipFree(d_out);
  if (e != hipSuccess) return fail(HDFS_CRC32C_EHIP, "composite: %s", hipGetErrorString(e));
  return HDFS_CRC32C_OK;
}

}  // extern "C"
