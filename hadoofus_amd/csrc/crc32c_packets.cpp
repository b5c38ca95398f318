// Host-side framing of datanode packet streams: the sequential part of
// _recv_packet / _process_recv_packet (src/datanode.c:2345-2446), so that the
// CRC work of a whole run of packets can go to the GPU in one launch.
//
// Framing rules and the PacketHeaderProto decode live in crc32c_frame.h,
// shared with the device framing kernel.
#include "crc32c_packets.h"

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <thread>
#include <vector>

#include <unistd.h>

#include "crc32c_engine.h"

namespace hdfs_crc32c {

int check_framing_args(int proto, uint32_t chunk_size, int ctype, char *errbuf, size_t errlen) {
  if (proto != HDFS_CRC32C_PROTO_V1 && proto != HDFS_CRC32C_PROTO_V2) {
    std::snprintf(errbuf, errlen, "bad packet protocol %d", proto);
    return HDFS_CRC32C_EINVAL;
  }
  if (ctype != HDFS_CRC32C_CSUM_NULL && ctype != HDFS_CRC32C_CSUM_CRC32 && ctype != HDFS_CRC32C_CSUM_CRC32C) {
    std::snprintf(errbuf, errlen, "bad checksum type %d", ctype);
    return HDFS_CRC32C_EINVAL;
  }
  if (ctype != HDFS_CRC32C_CSUM_NULL && chunk_size == 0) {
    std::snprintf(errbuf, errlen, "chunk_size 0");
    return HDFS_CRC32C_EINVAL;
  }
  return HDFS_CRC32C_OK;
}

int parse_packet_stream(const uint8_t *s, uint64_t len, int proto, uint32_t chunk_size, int ctype,
                        size_t max_pkts, std::vector<hdfs_crc32c_packet> &out, uint64_t *consumed,
                        char *errbuf, size_t errlen) {
  out.clear();
  *consumed = 0;
  int rc = check_framing_args(proto, chunk_size, ctype, errbuf, errlen);
  if (rc) return rc;
  if (len && !s) {
    std::snprintf(errbuf, errlen, "null stream");
    return HDFS_CRC32C_EINVAL;
  }
  uint64_t pos = 0;
  while (out.size() < max_pkts) {
    hdfs_crc32c_packet k;
    uint64_t total = 0;
    const int st = frame_step(s + pos, len - pos, pos, proto, chunk_size, ctype, k, total);
    if (st == kStepMore) break;
    out.push_back(k);
    if (st == kStepStop) {
      if (!k.error) *consumed = pos + total;
      break;
    }
    pos += total;
    *consumed = pos;
  }
  return HDFS_CRC32C_OK;
}

}  // namespace hdfs_crc32c

// ===========================================================================
// GPU side: pieces of framing-clean packets -> H2D, de-framing gather, verify
// ===========================================================================
namespace hdfs_crc32c {
namespace {

constexpr uint64_t kPieceCap = uint64_t(64) << 20;  // wire bytes per piece (sync verify)

struct PieceLayout {
  size_t n = 0;                 // packets in the piece
  uint64_t src0 = 0, span = 0;  // wire bytes [src0, src0 + span) of the host buffer
  uint64_t arena = 0, crcb = 0, bm = 0;
  uint32_t units = 0;
  uint64_t rounds = 0, mtiles = 0, gtiles = 0;
  uint32_t utiles = 0;          // uniform table: main tiles per segment (0: not uniform)
  size_t off_segs = 0, off_fb = 0, off_bm = 0, meta = 0;  // table layout (device and pinned host)
};

uint64_t wire_begin(const hdfs_crc32c_packet &k) { return k.stream_off + k.header_len; }
uint64_t wire_end(const hdfs_crc32c_packet &k) {
  return k.stream_off + k.header_len + uint64_t(k.crc_len) + uint64_t(k.data_len);
}

void layout_piece(const hdfs_crc32c_packet *recs, const size_t *idx, size_t n, PieceLayout &L) {
  L = PieceLayout{};
  L.n = n;
  L.src0 = wire_begin(recs[idx[0]]);
  L.span = wire_end(recs[idx[n - 1]]) - L.src0;
  for (size_t v = 0; v < n; v++) {
    const hdfs_crc32c_packet &k = recs[idx[v]];
    L.arena += align_up(uint64_t(k.data_len), 16);
    L.crcb += uint64_t(k.crc_len);
    L.bm += (uint64_t(k.crc_len) / 4 + 7) / 8;
    L.units += uint32_t((uint64_t(k.data_len) + kGatherSlice - 1) / kGatherSlice);
  }
  L.off_segs = align_up(n * sizeof(PktDesc), 256);
  L.off_fb = L.off_segs + align_up(n * sizeof(SegDev), 256);
  L.off_bm = L.off_fb + align_up(n * 4, 256);
  L.meta = L.off_bm + align_up(L.bm, 256);
}

int grow(uint8_t *&buf, size_t &cap, size_t need) {
  if (need <= cap) return HDFS_CRC32C_OK;
  if (buf) HIPCHK(hipFree(buf));
  buf = nullptr;
  cap = 0;
  HIPCHK(hipMalloc(&buf, need));
  cap = need;
  return HDFS_CRC32C_OK;
}

// Make slot s large enough for L (waits for the slot's previous piece first
// if a buffer has to be replaced).
int reserve_slot(PieceSlot &s, const PieceLayout &L) {
  if (!s.done) {
    HIPCHK(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&s.copied, hipEventDisableTiming));
    HIPCHK(hipMalloc(&s.gctr, 64));
    HIPCHK(hipMalloc(&s.mism, 64));
  }
  if (L.span + 64 > s.raw_cap || L.arena + 64 > s.arena_cap || L.crcb + 64 > s.crc_cap || L.meta > s.meta_cap) {
    HIPCHK(hipEventSynchronize(s.done));
    int rc;
    if ((rc = grow(s.raw, s.raw_cap, L.span + 64)) || (rc = grow(s.arena, s.arena_cap, L.arena + 64)) ||
        (rc = grow(s.crc, s.crc_cap, L.crcb + 64)) || (rc = grow(s.meta, s.meta_cap, L.meta)))
      return rc;
  }
  return HDFS_CRC32C_OK;
}

void release_slot(PieceSlot &s) {
  if (s.done) (void)hipEventSynchronize(s.done);
  for (uint8_t *p : {s.raw, s.arena, s.crc, s.meta})
    if (p) (void)hipFree(p);
  if (s.gctr) (void)hipFree(s.gctr);
  if (s.mism) (void)hipFree(s.mism);
  if (s.done) (void)hipEventDestroy(s.done);
  if (s.copied) (void)hipEventDestroy(s.copied);
  s = PieceSlot{};
}

// Build the piece's gather descriptors and verify segments in hmeta
// (pinned; device addresses of slot s) and finish L's tile counts.
int build_piece(const hdfs_crc32c_packet *recs, const size_t *idx, PieceLayout &L, uint32_t cs, int ctype,
                const PieceSlot &s, uint8_t *hmeta) {
  auto *hd = reinterpret_cast<PktDesc *>(hmeta);
  auto *hs = reinterpret_cast<SegDev *>(hmeta + L.off_segs);
  const uint32_t sflags = HDFS_CRC32C_SEG_BE | (ctype == HDFS_CRC32C_CSUM_CRC32 ? HDFS_CRC32C_SEG_CRC32 : 0u);
  uint64_t aoff = 0, coff = 0, boff = 0;
  uint32_t unit = 0;
  L.rounds = L.mtiles = L.gtiles = 0;
  for (size_t v = 0; v < L.n; v++) {
    const hdfs_crc32c_packet &k = recs[idx[v]];
    PktDesc &d = hd[v];
    d.src_crc = wire_begin(k) - L.src0;
    d.dst_data = aoff;
    d.dst_crc = coff;
    d.dlen = uint32_t(k.data_len);
    d.ncrc = uint32_t(k.crc_len / 4);
    d.unit0 = unit;
    d.nunits = uint32_t((uint64_t(d.dlen) + kGatherSlice - 1) / kGatherSlice);
    hdfs_crc32c_segment in = {s.arena + aoff, uint64_t(d.dlen), cs, sflags, 0, 0, s.crc + coff,
                              s.meta + L.off_bm + boff};
    int rc = fill_seg(in, HDFS_CRC32C_MODE_VERIFY, hs[v], v);
    if (rc) return rc;
    classify(hs[v], L.rounds, L.gtiles, L.mtiles);
    aoff += align_up(d.dlen, 16);
    coff += 4ull * d.ncrc;
    boff += (uint64_t(d.ncrc) + 7) / 8;
    unit += d.nunits;
  }
  L.utiles = uniform_tiles(hs, L.n);
  return HDFS_CRC32C_OK;
}

// Copy stream: tables + wire bytes H2D once slot s is free; compute stream:
// gather, verify, results D2H into hmeta.  s.done marks completion.
int enqueue_piece(DevCtx &c, const uint8_t *host, const PieceLayout &L, PieceSlot &s, uint8_t *hmeta, int ctype,
                  hipStream_t copy, hipStream_t comp) {
  HIPCHK(hipStreamWaitEvent(copy, s.done, 0));
  HIPCHK(hipMemcpyAsync(s.meta, hmeta, L.off_fb, hipMemcpyHostToDevice, copy));
  HIPCHK(hipMemcpyAsync(s.raw, host + L.src0, L.span, hipMemcpyHostToDevice, copy));
  HIPCHK(hipEventRecord(s.copied, copy));
  HIPCHK(hipStreamWaitEvent(comp, s.copied, 0));
  HIPCHK(launch_gather(s.raw, reinterpret_cast<const PktDesc *>(s.meta), uint32_t(L.n), L.units, s.arena, s.crc,
                       comp));
  int rc = launch_all(c, kModeVerify, reinterpret_cast<const SegDev *>(s.meta + L.off_segs), uint32_t(L.n),
                      L.rounds, L.mtiles, L.gtiles, reinterpret_cast<uint32_t *>(s.meta + L.off_fb), s.mism,
                      s.gctr, comp, nullptr, nullptr, true, ctype == HDFS_CRC32C_CSUM_CRC32 ? 1 : 0, false, false,
                      false, L.utiles);
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(hmeta + L.off_fb, s.meta + L.off_fb, L.meta - L.off_fb, hipMemcpyDeviceToHost, comp));
  HIPCHK(hipEventRecord(s.done, comp));
  return HDFS_CRC32C_OK;
}

// After the piece completed: per-packet verdicts from first-bad + bitmaps.
void finish_piece(hdfs_crc32c_packet *recs, const size_t *idx, const PieceLayout &L, const uint8_t *hmeta) {
  const auto *fb = reinterpret_cast<const uint32_t *>(hmeta + L.off_fb);
  const uint8_t *bm = hmeta + L.off_bm;
  for (size_t v = 0; v < L.n; v++) {
    hdfs_crc32c_packet &k = recs[idx[v]];
    const uint32_t nch = uint32_t(k.crc_len / 4), nb = (nch + 7) / 8;
    if (fb[v] != 0xFFFFFFFFu) {
      uint32_t bad = 0;
      for (uint32_t j = 0; j < nb; j++) {
        uint32_t byte = bm[j];
        if (j == nch / 8) byte &= (1u << (nch % 8)) - 1u;  // bits past the last chunk
        bad += uint32_t(__builtin_popcount(byte));
      }
      k.error = HDFS_CRC32C_ERR_DATANODE_BAD_CHECKSUM;
      k.first_bad = int32_t(fb[v]);
      k.bad_chunks = bad;
    }
    bm += nb;
  }
}

int first_error(const hdfs_crc32c_packet *p, size_t n) {
  for (size_t i = 0; i < n; i++)
    if (p[i].error) return p[i].error;
  return HDFS_CRC32C_OK;
}

// ---- device-resident packet streams ----
// The framing walk needs ~30 header bytes per packet from a stream the host
// cannot read.  It asks header_window_kernel for rows of kHdrWin bytes at
// base + k * stride, where stride is the size of the packet just framed
// (for a walk's first window the kernel reads it from the first header):
// the fixed-size packets of a block transfer all land on that grid, so a
// regular stream of up to 8 192 packets costs one small D2H round trip.  A packet off the grid (a short tail, a trailing
// empty packet, a stream of mixed sizes) starts a new window at its offset;
// the window length grows while windows keep hitting and drops back after a
// miss, so an irregular stream does not pay for rows it never reads.
static const bool g_dstream_trace = std::getenv("HDFS_CRC32C_DSTREAM_TRACE") != nullptr;

struct HeaderWindows {
  DevCtx &c;
  const uint8_t *d;
  uint64_t len;
  int proto;
  uint64_t base = 0, stride = 0;
  uint32_t count = 0, used = 0, budget = 8192, nfetch = 0;

  const uint8_t *lookup(uint64_t pos) {
    if (!count || pos < base) return nullptr;
    const uint64_t off = pos - base;
    const uint64_t k = stride ? off / stride : 0;
    if ((stride ? off % stride : off) != 0 || k >= count) return nullptr;
    used = std::max(used, uint32_t(k) + 1);
    return c.w_host + k * kHdrWin;
  }

  int fetch(uint64_t pos, uint64_t stride_guess, size_t rows_left) {
    constexpr uint32_t kMaxRows = 1u << 16;  // 4 MiB of rows per window
    if (count) budget = (used * 2 >= count) ? std::min(kMaxRows, budget * 8) : 64;
    // no stride yet: the kernel takes it from the header at pos; size the
    // window for packets of >= 4 KiB (block transfers send 64 KiB ones)
    const int sproto = stride_guess ? 0 : proto;
    uint64_t n = (len - pos) / (stride_guess ? stride_guess : 4096) + 1;
    n = std::min<uint64_t>({n, rows_left, budget});
    if (n == 0) n = 1;
    if (n + 1 > c.w_cap) {  // + 1 row: the derived stride
      uint32_t cap = 1024;
      while (cap < n + 1) cap *= 2;
      if (c.w_dev) HIPCHK(hipFree(c.w_dev));
      if (c.w_host) HIPCHK(hipHostFree(c.w_host));
      c.w_dev = c.w_host = nullptr;
      c.w_cap = 0;
      HIPCHK(hipMalloc(&c.w_dev, size_t(cap) * kHdrWin));
      HIPCHK(hipHostMalloc(&c.w_host, size_t(cap) * kHdrWin, hipHostMallocDefault));
      c.w_cap = cap;
    }
    auto *sdev = reinterpret_cast<uint64_t *>(c.w_dev + size_t(n) * kHdrWin);
    HIPCHK(launch_header_window(d, len, pos, stride_guess, uint32_t(n), sproto, c.w_dev, sdev, c.stream));
    HIPCHK(hipMemcpyAsync(c.w_host, c.w_dev, size_t(n) * kHdrWin + (sproto ? 8 : 0), hipMemcpyDeviceToHost,
                          c.stream));
    HIPCHK(hipStreamSynchronize(c.stream));
    base = pos;
    stride = stride_guess;
    if (sproto) std::memcpy(&stride, c.w_host + size_t(n) * kHdrWin, 8);
    count = uint32_t(n);
    nfetch++;
    used = 0;
    return HDFS_CRC32C_OK;
  }
};

// One verify launch over packets vidx[v0, v1) of a device-resident stream:
// no copies and no de-framing gather -- every packet is one verify segment
// pointing into the stream itself (CRCs at stream_off + header_len, data
// right after them; the tiled kernel takes both at any byte offset).  Tables
// go H2D, results D2H, all on c.v_stream, asynchronously: the framing walk
// keeps reading header windows (on c.stream) while earlier batches verify.
struct DevBatch {
  size_t v0 = 0, v1 = 0;
  PieceLayout L;
};

// Copy-out of a device-resident verify (hdfs_crc32c_read_packets):
// every framing-clean packet delivers frame::read_avail bytes (its whole
// payload, or the part of it a client read window takes) to its place in
// dst (frame::read_place), never past `cap` bytes -- the read's length, or
// the buffer for whole payloads.
struct CopyOut {
  uint8_t *dst = nullptr;  // null: no copy-out
  uint64_t cap = 0;        // bytes of dst the copies may fill (placement: never past it)
  bool win = false;
  int64_t client_offset = 0;
  uint64_t want = 0;       // win: bytes the read still wants (remains_tot; >= cap)
};
// Where one packet's copy goes (host-built segment tables).
struct CopyPlace {
  uint64_t at;
  uint32_t w0, w1;
};

int submit_device_batch(DevCtx &c, const uint8_t *d, const std::vector<hdfs_crc32c_packet> &recs,
                        const std::vector<size_t> &vidx, size_t bi, DevBatch &b, uint32_t cs, int ctype,
                        uint8_t *copy_dst, const std::vector<CopyPlace> &vpay) {
  PieceLayout &L = b.L;
  L = PieceLayout{};
  L.n = b.v1 - b.v0;
  for (size_t v = b.v0; v < b.v1; v++) L.bm += (uint64_t(recs[vidx[v]].crc_len) / 4 + 7) / 8;
  L.off_segs = 0;
  L.off_fb = align_up(L.n * sizeof(SegDev), 256);
  L.off_bm = L.off_fb + align_up(L.n * 4, 256);
  L.meta = L.off_bm + align_up(L.bm, 256);
  if (bi >= c.v_batch.size()) c.v_batch.resize(bi + 1);
  DevCtx::VBatch &vb = c.v_batch[bi];  // previous user: an earlier call, synchronised at its end
  if (L.meta > vb.hcap) {
    if (vb.h) HIPCHK(hipHostFree(vb.h));
    vb.h = nullptr;
    vb.hcap = 0;
    HIPCHK(hipHostMalloc(&vb.h, L.meta, hipHostMallocDefault));
    vb.hcap = L.meta;
  }
  if (L.meta + 64 > vb.dcap) {
    if (vb.d) HIPCHK(hipFree(vb.d));
    vb.d = nullptr;
    vb.dcap = 0;
    HIPCHK(hipMalloc(&vb.d, L.meta + 64));
    vb.dcap = L.meta + 64;
  }
  uint8_t *hm = vb.h, *dm = vb.d;
  auto *hs = reinterpret_cast<SegDev *>(hm);
  const uint32_t sflags = HDFS_CRC32C_SEG_BE | (ctype == HDFS_CRC32C_CSUM_CRC32 ? HDFS_CRC32C_SEG_CRC32 : 0u);
  uint64_t boff = 0;
  for (size_t v = 0; v < L.n; v++) {
    const hdfs_crc32c_packet &k = recs[vidx[b.v0 + v]];
    const uint8_t *crcp = d + wire_begin(k);
    hdfs_crc32c_segment in = {crcp + k.crc_len, uint64_t(k.data_len), cs, sflags, 0, 0,
                              const_cast<uint8_t *>(crcp), dm + L.off_bm + boff};
    int rc = fill_seg(in, HDFS_CRC32C_MODE_VERIFY, hs[v], v);
    if (rc) return rc;
    if (copy_dst) {  // placed within the destination by the walk (never past it)
      const CopyPlace &cp = vpay[b.v0 + v];
      hs[v].copy_dst = cp.w1 > cp.w0 ? copy_dst + cp.at : nullptr;
      hs[v].copy_w0 = cp.w0;
      hs[v].copy_w1 = cp.w1;
    }
    classify(hs[v], L.rounds, L.gtiles, L.mtiles);
    boff += (uint64_t(k.crc_len) / 4 + 7) / 8;
  }
  // the pool counter and mismatch word live past the tables
  auto *gctr = reinterpret_cast<uint32_t *>(dm + L.meta);
  auto *mism = reinterpret_cast<unsigned long long *>(dm + L.meta + 8);
  HIPCHK(hipMemcpyAsync(dm, hm, L.off_fb, hipMemcpyHostToDevice, c.v_stream));
  int rc = launch_all(c, kModeVerify, reinterpret_cast<const SegDev *>(dm), uint32_t(L.n), L.rounds, L.mtiles,
                      L.gtiles, reinterpret_cast<uint32_t *>(dm + L.off_fb), mism, gctr, c.v_stream, nullptr,
                      nullptr, true, ctype == HDFS_CRC32C_CSUM_CRC32 ? 1 : 0, copy_dst != nullptr, false,
                      any_unaligned(hs, L.n), uniform_tiles(hs, L.n));
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(hm + L.off_fb, dm + L.off_fb, L.meta - L.off_fb, hipMemcpyDeviceToHost, c.v_stream));
  return HDFS_CRC32C_OK;
}

// Host framing walk over device memory through header windows (same
// records and stopping rules as parse_packet_stream), from stream offset
// `pos`, appending to `out`: the fallback of grid_walk for the part of a
// stream whose packets are not all one size.  Verifies as it goes when
// `verify`: framing-clean packets with CRCs are submitted in batches of
// 1 024 growing to 4 096 packets (the first launch starts early; later ones
// amortise the launch), overlapped with the rest of the walk.  co: verify +
// copy-out, each packet's delivered bytes placed by frame::read_place after
// *payload bytes of earlier packets (advanced by every framing-clean
// packet) -- inside co.cap, so a stream whose payload exceeds the buffer is
// never written past it (the call then fails).  A client read window ends
// the walk once no packet can deliver more.  Caller holds c.mu.
int walk_device_stream(DevCtx &c, const uint8_t *d, uint64_t len, int proto, uint32_t cs, int ctype,
                       size_t max_pkts, bool verify, std::vector<hdfs_crc32c_packet> &out, uint64_t *consumed,
                       uint64_t pos, const CopyOut &co, uint64_t *payload) {
  verify = verify && ctype != HDFS_CRC32C_CSUM_NULL;
  if (verify && !c.v_stream) HIPCHK(hipStreamCreateWithFlags(&c.v_stream, hipStreamNonBlocking));
  HeaderWindows w{c, d, len, proto};
  std::vector<uint8_t> big;  // v2 headers longer than a window row
  std::vector<size_t> vidx;     // packets to verify
  std::vector<CopyPlace> vpay;  // their copy-out placement
  std::vector<DevBatch> batches;
  size_t batch_cap = 1024, v_sub = 0;
  auto submit = [&]() -> int {
    DevBatch b;
    b.v0 = v_sub;
    b.v1 = vidx.size();
    v_sub = b.v1;
    batches.push_back(b);
    return submit_device_batch(c, d, out, vidx, batches.size() - 1, batches.back(), cs, ctype, co.dst, vpay);
  };
  uint64_t stride = 0;
  int rc = HDFS_CRC32C_OK;
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  double t_submit = 0;
  while (out.size() < max_pkts && pos < len) {
    const uint8_t *p = w.lookup(pos);
    if (!p) {
      if ((rc = w.fetch(pos, stride, max_pkts - out.size()))) break;
      p = w.lookup(pos);
    }
    if (proto == HDFS_CRC32C_PROTO_V2 && len - pos >= 6) {
      const uint64_t need = 6 + ((uint64_t(p[4]) << 8) | p[5]);
      if (need > kHdrWin && len - pos >= need) {
        big.resize(need);
        hipError_t e = hipMemcpy(big.data(), d + pos, need, hipMemcpyDeviceToHost);
        if (e != hipSuccess) {
          rc = fail(HDFS_CRC32C_EHIP, "header copy: %s", hipGetErrorString(e));
          break;
        }
        p = big.data();
      }
    }
    hdfs_crc32c_packet k;
    uint64_t total = 0;
    const int st = frame_step(p, len - pos, pos, proto, cs, ctype, k, total);
    if (st == kStepMore) break;
    out.push_back(k);
    uint32_t cb = 0, clen = 0;
    const uint32_t avail = frame::read_avail(k, co.win, co.client_offset, cb);
    if (verify && !k.error && k.crc_len > 0) {
      uint64_t at = 0;
      frame::read_place(*payload, avail, co.cap, at, clen);
      vidx.push_back(out.size() - 1);
      vpay.push_back(CopyPlace{at, cb, cb + clen});
      if (vidx.size() - v_sub >= batch_cap) {
        const auto ts = clk::now();
        rc = submit();
        t_submit += std::chrono::duration<double, std::micro>(clk::now() - ts).count();
        if (rc) break;
        batch_cap = std::min<size_t>(batch_cap * 2, 4096);
      }
    }
    *payload += avail;
    if (st == kStepStop) {
      if (!k.error) *consumed = pos + total;
      break;
    }
    pos += total;
    stride = total;
    *consumed = pos;
    // a read window is over: the read is complete, or this packet ends it
    // (UNEXPECTED_READ_OFFSET, the last packet of the block) -- later
    // packets are never taken (src/datanode.c:1476, 2483-2486, 2545-2546)
    if (co.win && !k.error && (*payload >= co.cap || avail == 0 || k.last)) break;
  }
  const auto t1 = clk::now();
  if (!rc && vidx.size() > v_sub) rc = submit();
  const auto t2 = clk::now();
  if (!batches.empty()) {
    // drain the batches already queued even after an error (their tables
    // and results live in this context's buffers)
    hipError_t e = hipStreamSynchronize(c.v_stream);
    if (!rc && e != hipSuccess) rc = fail(HDFS_CRC32C_EHIP, "verify: %s", hipGetErrorString(e));
  }
  if (g_dstream_trace) {  // diagnostic: where a device-stream call spends its time (us)
    const auto t3 = clk::now();
    auto us = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    std::fprintf(stderr, "dstream pkts=%zu batches=%zu windows=%u walk_us=%.1f (submit %.1f) last_submit_us=%.1f drain_us=%.1f\n",
                 out.size(), batches.size(), w.nfetch, us(t0, t1), t_submit, us(t1, t2), us(t2, t3));
  }
  if (rc) return rc;
  for (size_t bi = 0; bi < batches.size(); bi++)
    finish_piece(out.data(), vidx.data() + batches[bi].v0, batches[bi].L, c.v_batch[bi].h);
  return HDFS_CRC32C_OK;
}

// Device memory of which device (-1: host / unknown memory).
int stream_device(const void *stream) {
  hipPointerAttribute_t pa;
  if (hipPointerGetAttributes(&pa, stream) == hipSuccess && pa.type == hipMemoryTypeDevice) return pa.device;
  (void)hipGetLastError();
  return -1;
}

// ---- device framing (frame_build_kernel) ----
// Sequence number of a device framing pass or short run: what the host
// polls for in pinned memory and what tags the pass's look-back records --
// never 0 (the value of zeroed memory)
static uint32_t next_grid_seq(DevCtx &c) {
  if (++c.grid_seq == 0u) ++c.grid_seq;
  return c.grid_seq;
}

// Layout of one pass's device tables and pinned landing area.
constexpr uint32_t kBadFirst = 1024;  // bad-packet entries copied back with the verify summary
struct GridLayout {
  size_t look, recs, segs, seg2pkt, fb, sum, bad, ctr, done, exc, bm, dtotal;  // device
  size_t h_sum, h_sum2, htotal;  // pinned offsets (h_sum: summary + packet 0 + exceptions, kGridHost*;
                                 // h_sum2: summary after verify, then the bad list)
  GridLayout(uint32_t count, uint64_t bm_cap) {
    size_t o = 0;
    auto take = [&](size_t n) { const size_t at = o; o += align_up(n, 256); return at; };
    // the look-back records first, sized for the largest pass: always the
    // same bytes of the slot, zeroed when the slot is allocated and written
    // by nothing else, so a record's flag is either 0 or tagged with the
    // sequence number of the pass that wrote it
    look = take(size_t(kGridMaxCount / 64 + kGridGroups) * kGridLookBytes);
    recs = take(size_t(count) * sizeof(hdfs_crc32c_packet));
    segs = take(size_t(count) * sizeof(SegDev));
    seg2pkt = take(size_t(count) * 4);
    fb = take(size_t(count) * 4);
    sum = take(256);  // the bad list follows the summary: one copy back
    bad = take(size_t(count) * sizeof(GridBad));
    ctr = take(128);  // pool counter, mismatch count
    done = take(64);  // frame_build_kernel: blocks finished, exceptions found
    exc = take(size_t(count) * 4);
    bm = take(size_t(bm_cap));
    dtotal = o;
    o = 0;
    h_sum = take(kGridHostBytes);
    h_sum2 = take(256 + size_t(kBadFirst) * sizeof(GridBad));
    htotal = o;
  }
};
static_assert(sizeof(hdfs_crc32c_packet) == kGridRecBytes, "host record layout");
static_assert(sizeof(GridSummary) <= kGridHostRec0, "summary area");

int reserve_grid(DevCtx &c, size_t si, const GridLayout &L) {
  if (si >= c.grid.size()) c.grid.resize(si + 1);
  DevCtx::GridSlot &g = c.grid[si];  // previous user: an earlier call, complete (its last command published) or synchronised
  if (L.dtotal > g.dcap) {
    if (g.d) HIPCHK(hipFree(g.d));
    g.d = nullptr;
    g.dcap = 0;
    HIPCHK(hipMalloc(&g.d, L.dtotal));
    HIPCHK(hipMemset(g.d, 0, L.recs));  // the look-back records: no flag of any pass
    g.dcap = L.dtotal;
  }
  if (L.htotal > g.hcap) {
    if (g.h) HIPCHK(hipHostFree(g.h));
    g.h = g.hd = nullptr;
    g.hcap = 0;
    // fine-grained (coherent) and mapped: frame_build_kernel writes the
    // summary, packet 0's record and the exceptions here directly
    HIPCHK(hipHostMalloc(&g.h, L.htotal, hipHostMallocCoherent | hipHostMallocMapped));
    HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void **>(&g.hd), g.h, 0));
    g.hcap = L.htotal;
  }
  return HDFS_CRC32C_OK;
}

// Framing + verify of a device-resident stream, run by run on the device:
// each pass frames up to kGridMaxCount packets on the grid of the first
// packet's size, builds their verify segment table in HBM (one launch of
// frame_build_kernel) and returns only a summary, packet 0's record and
// the records that differ from the prediction from it; the verify launch
// (plus the optional fused copy-out) is queued behind them straight from the
// device-built summary.  The host writes the pass's records into the
// caller's array while the verify kernel runs.  A pass that leaves the grid
// after at most two packets (a stream of mixed sizes) hands the rest to the
// host window walk (walk_device_stream).  Same records, stopping rules and
// consumed offset as parse_packet_stream.
// Short runs (<= kSmallRunMax packets of <= 64 KiB, the per-read case; verify
// or framing only):
// framing and verify in ONE launch (small_run_kernel) instead of the framing
// pass + verify chain.  Returns 1 when the run is fully resolved
// there (records in dst), 0 when the regular path must run (a packet the
// kernel cannot take, a packet off the grid, more packets than it covers),
// < 0 on an engine error.
// truncated: len is the first kSmallRunBytes of a longer stream, for a
// client read that wants little of it (a read resumed into a small buffer):
// resolved only when the read is decided inside what was framed -- the
// destination fills there, or a packet ends the read (read_stopper).
bool read_window_over(const hdfs_crc32c_packet *p, size_t n, const CopyOut &co, const uint32_t *idx, size_t nidx);
// One short-run launch in flight: its pinned slot set (the synchronous
// calls' c.sr_h, or c.sr2_h for the rest of a stream launched under a
// speculative verify), sequence number, grid points and the epoch read
// before the launch.
struct SrLaunch {
  uint8_t *h = nullptr;
  uint32_t seq = 0, count = 0;
  uint64_t epoch = 0;
  hipStream_t st = nullptr;  // the stream it was queued on
};

int sr_launch(DevCtx &c, bool second, const uint8_t *d, uint64_t len, int proto, uint32_t cs, int ctype, bool verify,
              const CopyOut &co, size_t max_pkts, SrLaunch &L, hipStream_t st = nullptr) {
  uint8_t *&h = second ? c.sr2_h : c.sr_h;
  uint8_t *&hd = second ? c.sr2_hd : c.sr_hd;
  if (!h) {
    HIPCHK(hipHostMalloc(&h, kSrHostBytes, hipHostMallocCoherent | hipHostMallocMapped));
    std::memset(h, 0, kSrHostBytes);
    HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void **>(&hd), h, 0));
  }
  L.h = h;
  L.count = uint32_t(std::min<uint64_t>({uint64_t(kSmallRunMax), uint64_t(max_pkts), len / 6 + 1}));
  L.seq = next_grid_seq(c);
  const int tset = ctype == HDFS_CRC32C_CSUM_CRC32 ? 1 : 0;
  L.epoch = c.queued_epoch.load(std::memory_order_acquire);  // before the launch
  L.st = st ? st : c.stream;
  HIPCHK(launch_small_run(d, len, L.count, proto, cs, ctype, verify ? 1 : 0, c.d_tab_main_t[tset], c.d_tab_pow2_t[tset],
                          co.dst, co.cap, co.win ? 1 : 0, co.client_offset, hd, L.seq, L.st));
  return HDFS_CRC32C_OK;
}

// Waits for a short-run launch and turns its slots into records; 0 when the
// walk does not end inside it (the caller frames the stream instead).
int sr_collect(DevCtx &c, const SrLaunch &L, uint64_t len, const CopyOut &co, size_t max_pkts,
               hdfs_crc32c_packet *dst, size_t *nout, uint64_t *consumed, uint64_t *payload, bool truncated = false);

int small_run(DevCtx &c, const uint8_t *d, uint64_t len, int proto, uint32_t cs, int ctype, bool verify,
              const CopyOut &co, size_t max_pkts, hdfs_crc32c_packet *dst, size_t *nout, uint64_t *consumed,
              uint64_t *payload, bool truncated = false) {
  SrLaunch L;
  const int rc = sr_launch(c, false, d, len, proto, cs, ctype, verify, co, max_pkts, L);
  if (rc) return rc;
  return sr_collect(c, L, len, co, max_pkts, dst, nout, consumed, payload, truncated);
}

int sr_collect(DevCtx &c, const SrLaunch &L, uint64_t len, const CopyOut &co, size_t max_pkts,
               hdfs_crc32c_packet *dst, size_t *nout, uint64_t *consumed, uint64_t *payload, bool truncated) {
  const uint32_t count = L.count, seq = L.seq;
  const uint64_t epoch = L.epoch;
  // a fault of earlier work on the stream is this call's error, not the next
  // caller's: queried while the kernel is in flight when unconfirmed work
  // is queued before it (as small_call)
  if (c.unconfirmed()) {
    if (kDiag) c.stream_queries++;
    if (const hipError_t q = hipStreamQuery(c.stream); q != hipSuccess && q != hipErrorNotReady)
      return fail(HDFS_CRC32C_EHIP, "earlier work on the stream: %s", hipGetErrorString(q));
  }
  auto word = [&](uint32_t k, int i) -> const uint32_t * {
    return reinterpret_cast<const uint32_t *>(L.h + size_t(k) * kSrSlot + kGridRecBytes) + i;
  };
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  for (uint32_t k = 0; k < count; k++) {
    for (uint32_t spin = 1; __atomic_load_n(word(k, 3), __ATOMIC_ACQUIRE) != seq; spin++) {
      if ((spin & 4095u) == 0 && clk::now() - t0 > std::chrono::milliseconds(200)) {
        HIPCHK(hipStreamSynchronize(L.st));
        if (__atomic_load_n(word(k, 3), __ATOMIC_ACQUIRE) != seq) return fail(HDFS_CRC32C_EHIP, "short-run kernel");
        break;
      }
#if defined(__x86_64__) || defined(__i386__)
      __builtin_ia32_pause();
#endif
    }
  }
  // every slot is published (each workgroup's sequence word is its last
  // memory operation, so a fault of this launch cannot be followed by it;
  // and, on c.stream, everything queued before the launch has completed)
  if (L.st == c.stream) c.confirm(epoch);
  // the run: grid points up to the first that is not On (grid_build_kernel's rule)
  auto rec = [&](uint32_t k) {
    hdfs_crc32c_packet r;
    std::memcpy(&r, L.h + size_t(k) * kSrSlot, sizeof(r));
    return r;
  };
  uint32_t fbk = count, unsup = 0;
  for (uint32_t k = 0; k < count; k++)
    if ((*word(k, 0) & 0xffu) != kGridOn) {
      fbk = k;
      break;
    }
  const uint32_t st_fb = fbk < count ? (*word(fbk, 0) & 0xffu) : uint32_t(kGridOn);
  const uint32_t recorded = fbk + (fbk < count && st_fb != kGridMore ? 1u : 0u);
  const hdfs_crc32c_packet r0 = rec(0);
  const uint64_t stride = recorded && (*word(0, 0) & 0xffu) == kGridOn
                              ? uint64_t(r0.header_len) + uint64_t(r0.crc_len) + uint64_t(r0.data_len)
                              : 0u;
  uint64_t next = 0, used = 0, pay = 0;
  if (fbk == count) {
    used = next = uint64_t(count) * stride;
  } else if (st_fb == kGridMore) {
    used = next = uint64_t(fbk) * stride;
  } else {
    const hdfs_crc32c_packet rf = rec(fbk);
    next = rf.stream_off + rf.header_len + uint64_t(rf.crc_len) + uint64_t(rf.data_len);
    used = rf.error ? uint64_t(fbk) * stride : next;
  }
  for (uint32_t k = 0; k < recorded; k++) unsup |= *word(k, 0) >> 8;
  const bool ended = st_fb == kGridStop || st_fb == kGridMore || (fbk == count && (count == max_pkts || next >= len));
  if (unsup || !(ended || truncated)) return 0;
  for (uint32_t k = 0; k < recorded; k++) {
    dst[k] = rec(k);
    uint32_t cb = 0;
    pay += frame::read_avail(dst[k], co.win, co.client_offset, cb);  // before the verdict is set
    if (*word(k, 2)) {
      dst[k].error = HDFS_CRC32C_ERR_DATANODE_BAD_CHECKSUM;
      dst[k].first_bad = int32_t(*word(k, 1));
      dst[k].bad_chunks = *word(k, 2);
    }
  }
  // a truncated stream: the records must decide the read (a framing error
  // among them does too: the read ends there)
  if (truncated) {
    bool decided = co.win && pay >= co.cap;
    for (uint32_t k = 0; k < recorded && !decided; k++) decided = dst[k].error && dst[k].error != HDFS_CRC32C_ERR_DATANODE_BAD_CHECKSUM;
    if (!decided) decided = co.win && read_window_over(dst, recorded, co, nullptr, 0);
    if (!decided) return 0;
  }
  *nout = recorded;
  *consumed = used;
  *payload = pay;
  return 1;
}

// ---- speculative one-launch verify (spec_verify_kernel) ----
// A run of equal packets (a block transfer) verified in ONE launch that
// takes the run's layout from packet 0 and checks the other headers on the
// side (crc32c_internal.h, SpecCtl); the host fills the records from packet
// 0 while the kernel runs.  Not taken (the caller frames the run the regular
// way from the same offset) when packet 0 does not start such a run or a
// header differs from the prediction.
struct SpecResult {
  std::vector<uint32_t> exc_idx;  // records that are not the prediction from packet 0 (exceptions, the tail)
  bool taken = false;     // verified by the speculative launch
  bool end = false;       // the walk ends with this pass
  uint32_t recorded = 0;  // records written to dst
  uint64_t payload = 0;   // bytes the recorded packets deliver (frame::read_avail)
  uint64_t consumed = 0, next = 0;
  uint32_t first_err = UINT32_MAX;  // the first record with an error (bad chunks, the tail's), if any
};

// diagnostic build: {launches, eligible, taken, header exceptions}
// (hdfs_crc32c_diag_spec_stats)
uint64_t g_spec_stats[4] = {0, 0, 0, 0};

int spec_alloc(DevCtx &c, SpecSlot &S) {
  if (S.ctl) return HDFS_CRC32C_OK;
  SpecCtl *ctl = nullptr;
  SpecExc *exc = nullptr;
  SpecRunTail *xtail = nullptr;
  SpecTabData *tabs = nullptr;
  uint8_t *h = nullptr, *hd = nullptr;
  hipError_t e = hipMalloc(&ctl, 2 * sizeof(SpecCtl));
  if (e == hipSuccess) e = hipMemset(ctl, 0, 2 * sizeof(SpecCtl));  // the ring starts at zero
  if (e == hipSuccess) e = hipMalloc(&exc, 2 * kSpecExcMax * sizeof(SpecExc));
  if (e == hipSuccess) e = hipMalloc(&xtail, 2 * kSpecRunsMax * sizeof(SpecRunTail));
  if (e == hipSuccess) e = hipMalloc(&tabs, size_t(std::max(c.num_cu, 1)) * sizeof(SpecTabData));
  if (e == hipSuccess) e = hipHostMalloc(&h, kSpecHostBytes, hipHostMallocCoherent | hipHostMallocMapped);
  if (e == hipSuccess) {
    std::memset(h, 0, kSpecHostBytes);
    e = hipHostGetDevicePointer(reinterpret_cast<void **>(&hd), h, 0);
  }
  if (e != hipSuccess) {
    if (ctl) (void)hipFree(ctl);
    if (exc) (void)hipFree(exc);
    if (xtail) (void)hipFree(xtail);
    if (tabs) (void)hipFree(tabs);
    if (h) (void)hipHostFree(h);
    return fail(HDFS_CRC32C_EHIP, "speculative verify buffers: %s", hipGetErrorString(e));
  }
  S.exc = exc;
  S.xtail = xtail;
  S.tabs = tabs;
  S.h = h;
  S.hd = hd;
  S.n = 0;
  S.ctl = ctl;
  return HDFS_CRC32C_OK;
}

// Wait for a sequence number a kernel publishes to pinned memory as its last
// memory operation; after 200 ms the stream synchronisation reports a fault.
int poll_seq(const uint32_t *word, uint32_t seq, const char *what, hipStream_t st) {
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  for (uint32_t spin = 1; __atomic_load_n(word, __ATOMIC_ACQUIRE) != seq; spin++) {
    if ((spin & 4095u) == 0 && clk::now() - t0 > std::chrono::milliseconds(200)) {
      HIPCHK(hipStreamSynchronize(st));
      if (__atomic_load_n(word, __ATOMIC_ACQUIRE) != seq) return fail(HDFS_CRC32C_EHIP, "%s: no completion word", what);
      break;
    }
#if defined(__x86_64__) || defined(__i386__)
    __builtin_ia32_pause();
#endif
  }
  return HDFS_CRC32C_OK;
}

// One speculative launch in flight on slot S: what collecting it needs.
struct SpecLaunch {
  uint32_t seq = 0;
  int grid = 0;
  uint64_t pos = 0;
  uint8_t *bm = nullptr;
  hipStream_t st = nullptr;
  std::chrono::steady_clock::time_point t0, t1;  // launch call (diagnostic trace)
};

// nruns > 1: a batch -- runs 1 .. nruns - 1 at xs[r] (xlen[r] bytes) beside
// run 0 at d + pos, all verified in this launch (no read window, no copy)
int spec_launch(DevCtx &c, SpecSlot &S, hipStream_t st, const uint8_t *d, uint64_t len, uint64_t pos,
                uint32_t max_count, int proto, uint32_t cs, int ctype, const CopyOut &co, uint64_t done_b, uint8_t *bm,
                uint32_t *fb, SpecLaunch &L, uint32_t nruns = 1, const uint8_t *const *xs = nullptr,
                const uint64_t *xlen = nullptr, bool per_run = false) {
  int rc = spec_alloc(c, S);
  if (rc) return rc;
  uint64_t left = len - pos;
  for (uint32_t r = 1; r < nruns; r++) left += xlen[r];
  const uint64_t want = (left / kRoundBytes + 63) / 64;  // >= 4 rounds per wave (launch_verify_dyn)
  L.grid = int(std::max<uint64_t>(1, std::min<uint64_t>(want, uint64_t(c.bulk_cus()))));
  L.seq = next_grid_seq(c);
  L.pos = pos;
  L.bm = bm;
  L.st = st;
  auto *early = reinterpret_cast<SpecEarly *>(S.h);
  auto *fin = reinterpret_cast<SpecFinal *>(S.h + sizeof(SpecEarly));
  __atomic_store_n(&early->seq, 0u, __ATOMIC_RELEASE);
  __atomic_store_n(&fin->seq, 0u, __ATOMIC_RELEASE);
  SpecArgs a{};
  a.s = d;
  a.len = len;
  a.base = pos;
  a.max_count = max_count;
  a.proto = proto;
  a.ctype = ctype;
  a.cs = cs;
  a.sflags = HDFS_CRC32C_SEG_BE | (ctype == HDFS_CRC32C_CSUM_CRC32 ? HDFS_CRC32C_SEG_CRC32 : 0u);
  a.rwin = co.win ? 1 : 0;
  a.client_offset = co.client_offset;
  a.bm = bm;
  a.copy_base = co.dst ? co.dst + done_b : nullptr;
  // (a client read with no copy in the pass -- a reader, a scatter read --
  // still sizes the run by what is left of its capacity)
  a.copy_cap = (co.dst || co.win) ? co.cap - done_b : 0u;
  a.gtab = c.d_tab_main_t[ctype == HDFS_CRC32C_CSUM_CRC32 ? 1 : 0];
  a.fb = fb;
  a.ctl = S.ctl;
  a.exc = S.exc;
  a.parity = uint32_t(S.n & 1u);
  a.seq = L.seq;
  a.tune = tile_tune() | (g_spec_pool_min << 16);
  a.hout = S.hd;
  a.tabs = S.tabs;
  a.stamps = kDiag ? g_diag : nullptr;
  a.nruns = nruns;
  a.early = per_run && nruns > 1 ? 1u : 0u;
  for (uint32_t r = 1; r < nruns; r++) {
    a.xs[r] = xs[r];
    a.xlen[r] = xlen[r];
  }
  a.xtail = S.xtail;
  L.t0 = std::chrono::steady_clock::now();
  HIPCHK(launch_spec_verify(a, L.grid, co.dst ? 1 : 0, st));
  S.n++;
  if (kDiag) g_spec_stats[0]++;
  L.t1 = std::chrono::steady_clock::now();
  return HDFS_CRC32C_OK;
}

// The host side of a speculative launch: packet 0's record and the run's
// records predicted from it (filled while the kernel verifies), then the
// final block: exceptions, verdicts, what follows the run.  Not taken
// (res.taken false) when packet 0 starts no run or a header left the
// prediction -- the caller frames the run the regular way.
// Called by the first speculative pass of a call (stream offset 0) once the
// run's records are predicted from the early block, while the kernel still
// verifies: a scatter read starts its copy there (read_dev_scatter).  Set
// for the duration of one call on the calling thread.
struct EarlyHook {
  std::function<void(const hdfs_crc32c_packet *recs, uint32_t count)> fn;
};
thread_local const EarlyHook *t_early_hook = nullptr;
// grid_walk's own: the short rest of a verified stream launched at the early
// block (E.count, E.stride), queued behind the speculative kernel
thread_local const std::function<void(uint32_t count, uint64_t stride)> *t_tail_hook = nullptr;

int spec_collect(DevCtx &c, SpecSlot &S, const SpecLaunch &L, const CopyOut &co, hdfs_crc32c_packet *dst,
                 SpecResult &res) {
  (void)c;
  res = SpecResult{};
  using clk = std::chrono::steady_clock;
  auto *early = reinterpret_cast<SpecEarly *>(S.h);
  auto *fin = reinterpret_cast<SpecFinal *>(S.h + sizeof(SpecEarly));
  const uint64_t pos = L.pos;
  int rc;
  if ((rc = poll_seq(&early->seq, L.seq, "speculative verify", L.st))) return rc;
  const auto t2 = clk::now();
  SpecEarly E;
  std::memcpy(&E, early, sizeof(E));
  if (!E.eligible) return HDFS_CRC32C_OK;  // every workgroup returns at once; work queued behind it runs next
  if (kDiag) g_spec_stats[1]++;
  hdfs_crc32c_packet r0;
  std::memcpy(&r0, E.r0, sizeof(r0));
  // the run's records while the kernel verifies it
  for (uint32_t k = 0; k < E.count; k++) {
    hdfs_crc32c_packet &r = dst[k];
    r = r0;
    r.stream_off = pos + uint64_t(k) * E.stride;
    r.offset_in_block = r0.offset_in_block + int64_t(k) * r0.data_len;
    r.seqno = r0.seqno + int64_t(k);
  }
  if (t_early_hook && pos == 0) t_early_hook->fn(dst, E.count);
  if (t_tail_hook) (*t_tail_hook)(E.count, E.stride);
  const auto t3 = clk::now();
  if ((rc = poll_seq(&fin->seq, L.seq, "speculative verify", L.st))) return rc;
  if (g_dstream_trace) {  // diagnostic: where a speculative launch spends its time (us)
    auto us = [](clk::time_point x, clk::time_point y) { return std::chrono::duration<double, std::micro>(y - x).count(); };
    std::fprintf(stderr, "dstream spec grid=%d count=%u launch_us=%.1f early_us=%.1f fill_us=%.1f final_us=%.1f\n", L.grid,
                 E.count, us(L.t0, L.t1), us(L.t1, t2), us(t2, t3), us(t3, clk::now()));
  }
  SpecFinal F;
  std::memcpy(&F, fin, sizeof(F));
  if (F.exc) {  // a header off the prediction: frame the run instead
    if (kDiag) g_spec_stats[3]++;
    return HDFS_CRC32C_OK;
  }
  res.taken = true;
  if (kDiag) g_spec_stats[2]++;
  // same-size packets whose headers left the prediction: their own records
  const auto *hx = reinterpret_cast<const SpecExc *>(S.h + 256);
  for (uint32_t j = 0; j < F.nexc; j++) {  // (more than kSpecExcMax raised exc)
    SpecExc x;
    std::memcpy(&x, hx + j, sizeof(x));
    if (x.k >= E.count) return fail(HDFS_CRC32C_EHIP, "speculative verify: exception record %u of %u", x.k, E.count);
    std::memcpy(&dst[x.k], x.rec, sizeof(hdfs_crc32c_packet));
    res.exc_idx.push_back(x.k);
    if (dst[x.k].error) res.first_err = std::min(res.first_err, x.k);
  }
  if (r0.error) res.first_err = 0;
  if (F.mism) {
    // packets with bad chunks: first bad chunk and count from the bitmap
    // (rare; the kernel's results are complete once the copy, queued
    // behind it, has run)
    const uint32_t nch = uint32_t(r0.crc_len) / 4u, nb = (nch + 7u) / 8u;
    std::vector<uint8_t> bmh(size_t(E.count) * nb);
    HIPCHK(hipMemcpyAsync(bmh.data(), L.bm, bmh.size(), hipMemcpyDeviceToHost, L.st));
    HIPCHK(hipStreamSynchronize(L.st));
    for (uint32_t k = 0; k < E.count; k++) {
      const uint8_t *b = bmh.data() + size_t(k) * nb;
      uint32_t bad = 0;
      int32_t first = -1;
      for (uint32_t j = 0; j < nb; j++) {
        uint32_t byte = b[j];
        if (j == nch / 8u) byte &= (1u << (nch % 8u)) - 1u;  // bits past the last chunk
        if (!byte) continue;
        if (first < 0) first = int32_t(8u * j + uint32_t(__builtin_ctz(byte)));
        bad += uint32_t(__builtin_popcount(byte));
      }
      if (bad) {
        dst[k].error = HDFS_CRC32C_ERR_DATANODE_BAD_CHECKSUM;
        dst[k].first_bad = first;
        dst[k].bad_chunks = bad;
        if (res.first_err == UINT32_MAX) res.first_err = k;
      }
    }
  }
  uint32_t cb0 = 0;
  const uint64_t avail0 = frame::read_avail(r0, co.win, co.client_offset, cb0);
  res.payload = uint64_t(E.count - 1u) * uint64_t(r0.data_len) + avail0;
  const uint64_t run_end = pos + uint64_t(E.count) * E.stride;
  res.recorded = E.count;
  res.consumed = res.next = run_end;
  if (F.tail_status == kGridStop) {  // the empty last packet or a framing error ends the walk
    hdfs_crc32c_packet &t = dst[E.count];
    std::memcpy(&t, F.tail, sizeof(t));
    if (!t.error) res.consumed = run_end + F.tail_total;
    else res.first_err = std::min(res.first_err, E.count);
    res.exc_idx.push_back(E.count);
    res.recorded++;
    res.end = true;
  } else if (F.tail_status == kGridMore) {  // the stream ends inside the next packet
    res.end = true;
  }  // kGridOff (another size) / kGridOn (the pass was cut): the walk goes on at run_end
  return HDFS_CRC32C_OK;
}

// The host side of a BATCH launch (nruns runs, run r's packet 0 at pos0[r]
// of its stream): each run's records predicted from its own packet 0 into
// dst[r], then exceptions (global packet index -> run), verdicts and what
// follows each run.  All runs taken or none (a header off the prediction in
// any run voids the launch).
struct SpecRunResult {
  bool taken = false, end = false;
  uint32_t recorded = 0;
  uint64_t consumed = 0, next = 0;
};
// A run's records predicted from its packet 0 (stream offsets from pos0).
void predict_run(const hdfs_crc32c_packet &r0, uint32_t count, uint64_t stride, uint64_t pos0, hdfs_crc32c_packet *dst) {
  for (uint32_t k = 0; k < count; k++) {
    hdfs_crc32c_packet &q = dst[k];
    q = r0;
    q.stream_off = pos0 + uint64_t(k) * stride;
    q.offset_in_block = r0.offset_in_block + int64_t(k) * r0.data_len;
    q.seqno = r0.seqno + int64_t(k);
  }
}
// What follows a run of `count` packets (the point after it: status, wire
// size, record) -> its result, and the record that ends the walk at
// dst[count] when there is one.
void run_tail(uint32_t count, uint64_t stride, uint64_t pos0, uint32_t status, uint64_t total, const uint64_t *rec,
              hdfs_crc32c_packet *dst, SpecRunResult &o) {
  o.taken = true;
  o.recorded = count;
  const uint64_t run_end = pos0 + uint64_t(count) * stride;
  o.consumed = o.next = run_end;
  if (status == kGridStop) {  // the empty last packet or a framing error ends the walk
    hdfs_crc32c_packet &t = dst[count];
    std::memcpy(&t, rec, sizeof(t));
    if (!t.error) o.consumed = run_end + total;
    o.recorded++;
    o.end = true;
  } else if (status == kGridMore) {  // the stream ends inside the next packet
    o.end = true;
  }  // kGridOff (another size) / kGridOn (the pass was cut): the walk goes on at run_end
}

int spec_collect_batch(SpecSlot &S, const SpecLaunch &L, uint32_t nruns, const uint64_t *pos0,
                       hdfs_crc32c_packet *const *dst, std::vector<SpecRunResult> &res) {
  res.assign(nruns, SpecRunResult{});
  auto *early = reinterpret_cast<SpecEarly *>(S.h);
  auto *fin = reinterpret_cast<SpecFinal *>(S.h + sizeof(SpecEarly));
  int rc;
  if ((rc = poll_seq(&early->seq, L.seq, "speculative batch verify", L.st))) return rc;
  SpecEarly E;
  std::memcpy(&E, early, sizeof(E));
  if (!E.eligible) return HDFS_CRC32C_OK;
  if (kDiag) g_spec_stats[1]++;
  std::vector<SpecRunEarly> er(nruns);
  std::memcpy(er.data(), S.h + kSpecRunEarlyOff, nruns * sizeof(SpecRunEarly));
  std::vector<uint32_t> prefix(nruns + 1, 0);
  std::vector<hdfs_crc32c_packet> r0(nruns);
  for (uint32_t r = 0; r < nruns; r++) {
    std::memcpy(&r0[r], er[r].r0, sizeof(hdfs_crc32c_packet));
    prefix[r + 1] = prefix[r] + er[r].count;
    predict_run(r0[r], er[r].count, E.stride, pos0[r], dst[r]);
  }
  if (prefix[nruns] != E.count) return fail(HDFS_CRC32C_EHIP, "speculative batch: %u packets, runs hold %u", E.count,
                                            prefix[nruns]);
  if ((rc = poll_seq(&fin->seq, L.seq, "speculative batch verify", L.st))) return rc;
  SpecFinal F;
  std::memcpy(&F, fin, sizeof(F));
  if (F.exc) {
    if (kDiag) g_spec_stats[3]++;
    return HDFS_CRC32C_OK;
  }
  if (kDiag) g_spec_stats[2]++;
  auto run_of = [&](uint32_t k) {
    return uint32_t(std::upper_bound(prefix.begin(), prefix.end(), k) - prefix.begin()) - 1u;
  };
  const auto *hx = reinterpret_cast<const SpecExc *>(S.h + 256);
  for (uint32_t j = 0; j < F.nexc; j++) {
    SpecExc x;
    std::memcpy(&x, hx + j, sizeof(x));
    if (x.k >= E.count) return fail(HDFS_CRC32C_EHIP, "speculative batch: exception record %u of %u", x.k, E.count);
    const uint32_t r = run_of(x.k);
    std::memcpy(&dst[r][x.k - prefix[r]], x.rec, sizeof(hdfs_crc32c_packet));
  }
  if (F.mism) {  // first bad chunk and count from the bitmap (global packet index)
    const uint32_t nch = uint32_t(r0[0].crc_len) / 4u, nb = (nch + 7u) / 8u;
    std::vector<uint8_t> bmh(size_t(E.count) * nb);
    HIPCHK(hipMemcpyAsync(bmh.data(), L.bm, bmh.size(), hipMemcpyDeviceToHost, L.st));
    HIPCHK(hipStreamSynchronize(L.st));
    for (uint32_t k = 0; k < E.count; k++) {
      const uint8_t *b = bmh.data() + size_t(k) * nb;
      uint32_t bad = 0;
      int32_t first = -1;
      for (uint32_t j = 0; j < nb; j++) {
        uint32_t byte = b[j];
        if (j == nch / 8u) byte &= (1u << (nch % 8u)) - 1u;
        if (!byte) continue;
        if (first < 0) first = int32_t(8u * j + uint32_t(__builtin_ctz(byte)));
        bad += uint32_t(__builtin_popcount(byte));
      }
      if (bad) {
        const uint32_t r = run_of(k);
        hdfs_crc32c_packet &q = dst[r][k - prefix[r]];
        q.error = HDFS_CRC32C_ERR_DATANODE_BAD_CHECKSUM;
        q.first_bad = first;
        q.bad_chunks = bad;
      }
    }
  }
  std::vector<SpecRunTail> tails(nruns);
  std::memcpy(tails.data(), S.h + kSpecRunTailOff, nruns * sizeof(SpecRunTail));
  for (uint32_t r = 0; r < nruns; r++) {
    uint32_t status;
    uint64_t total;
    const uint64_t *rec;
    if (r == 0) {
      status = F.tail_status;
      total = F.tail_total;
      rec = F.tail;
    } else {
      status = tails[r].status;
      total = tails[r].total;
      rec = tails[r].rec;
    }
    run_tail(er[r].count, E.stride, pos0[r], status, total, rec, dst[r], res[r]);
  }
  return HDFS_CRC32C_OK;
}

// Per-run completion of a coalesced batch (SpecArgs::early): run i's
// results before the launch ends, when its completion is published, clean
// (no mismatch) and in the prediction (no header off it), and what follows
// it is in the host area.  1: results in dst / o; 0: not yet; -1: not for
// this run (mismatches, exceptions, pool tiles, more records than `cap`, or
// the launch took no run) -- the launch's final block decides it.
int spec_run_early(const SpecSlot &S, const SpecLaunch &L, uint32_t i, size_t cap, hdfs_crc32c_packet *dst,
                   SpecRunResult &o) {
  const auto *early = reinterpret_cast<const SpecEarly *>(S.h);
  if (__atomic_load_n(&early->seq, __ATOMIC_ACQUIRE) != L.seq) return 0;
  if (!early->eligible) return -1;
  const auto *er = reinterpret_cast<const SpecRunEarly *>(S.h + kSpecRunEarlyOff) + i;
  if (!er->early) return -1;
  const auto *f = reinterpret_cast<const SpecRunDone *>(S.h + kSpecRunDoneOff) + i;
  if (__atomic_load_n(&f->seq, __ATOMIC_ACQUIRE) != L.seq) return 0;
  if (f->mism || f->bad) return -1;
  const auto *tl = reinterpret_cast<const SpecRunTail *>(S.h + kSpecRunTailOff) + i;
  if (__atomic_load_n(&tl->seq, __ATOMIC_ACQUIRE) != L.seq) return 0;
  SpecRunEarly e;
  SpecRunTail t;
  std::memcpy(&e, er, sizeof(e));
  std::memcpy(&t, tl, sizeof(t));
  if (size_t(e.count) + (t.status == kGridStop ? 1u : 0u) > cap) return -1;
  hdfs_crc32c_packet r0;
  std::memcpy(&r0, e.r0, sizeof(r0));
  predict_run(r0, e.count, early->stride, 0, dst);
  o = SpecRunResult{};
  run_tail(e.count, early->stride, 0, t.status, t.total, t.rec, dst, o);
  return 1;
}

// A synchronous speculative pass on the engine stream.
int spec_pass(DevCtx &c, const uint8_t *d, uint64_t len, uint64_t pos, uint32_t max_count, int proto, uint32_t cs,
              int ctype, const CopyOut &co, uint64_t done_b, uint8_t *bm, uint32_t *fb, hdfs_crc32c_packet *dst,
              SpecResult &res) {
  res = SpecResult{};
  SpecLaunch L;
  int rc = spec_launch(c, c.spec, c.stream, d, len, pos, max_count, proto, cs, ctype, co, done_b, bm, fb, L);
  if (rc) return rc;
  return spec_collect(c, c.spec, L, co, dst, res);
}

// A client read is decided by a packet that ends apply_read_window's walk
// -- an empty packet, a lastPacketInBlock packet, or one that starts past
// the read (UNEXPECTED_READ_OFFSET) -- so once a pass holds one, no later
// pass is framed or verified (a read that ended early kept
// framing and verifying the rest of the stream, possibly GiBs, only to drop
// it).
bool read_stopper(const hdfs_crc32c_packet &r, const CopyOut &co) {
  if (r.data_len <= 0 || r.last) return true;
  hdfs_crc32c_packet h = r;
  h.error = 0;
  uint32_t cb = 0;
  return frame::read_avail(h, true, co.client_offset, cb) == 0;
}
// Records of a pass predicted from its first packet (offsetInBlock rising by
// dataLen: avail never falls) but for the exceptions at idx[0, nidx) (all
// n records when idx is null): only those can hold a stopper.
bool read_window_over(const hdfs_crc32c_packet *p, size_t n, const CopyOut &co, const uint32_t *idx, size_t nidx) {
  if (!n) return false;
  if (!idx) {
    for (size_t k = 0; k < n; k++)
      if (read_stopper(p[k], co)) return true;
    return false;
  }
  if (read_stopper(p[0], co) || read_stopper(p[n - 1], co)) return true;
  for (size_t j = 0; j < nidx; j++)
    if (idx[j] < n && read_stopper(p[idx[j]], co)) return true;
  return false;
}

int grid_walk(DevCtx &c, const uint8_t *d, uint64_t len, int proto, uint32_t cs, int ctype, size_t max_pkts,
              bool verify, const CopyOut &co, hdfs_crc32c_packet *dst, size_t *nout, uint64_t *consumed,
              uint64_t *payload_out, bool allow_spec = true, size_t *first_err_out = nullptr) {
  *nout = 0;
  *consumed = 0;
  // the first record with an error, when the walk knows it without a scan
  // (speculative passes and short runs: SIZE_MAX otherwise)
  bool ferr_known = true;
  size_t ferr = SIZE_MAX;
  auto scan_err = [&](size_t from, size_t cnt) {
    for (size_t k = from; k < from + cnt && ferr == SIZE_MAX; k++)
      if (dst[k].error) ferr = k;
  };
  if (first_err_out) *first_err_out = SIZE_MAX;
  verify = verify && ctype != HDFS_CRC32C_CSUM_NULL;
  // a stream of at most kSmallRunBytes, or a client read whose destination
  // is at most 64 KiB of a longer one (a read resumed into a small buffer:
  // the packets it needs lie in the stream's first kSmallRunBytes unless
  // they are not all 64 KiB ones -- then the regular path runs)
  const bool small_win = co.win && co.dst && co.cap <= kSmallMax && len > kSmallRunBytes;
  if (max_pkts && (len <= kSmallRunBytes || small_win)) {  // verify (+ copy-out) or framing only
    uint64_t pay = 0;
    const int r = small_run(c, d, std::min<uint64_t>(len, kSmallRunBytes), proto, cs, ctype, verify, co, max_pkts, dst,
                            nout, consumed, &pay, small_win);
    if (r < 0) return r;
    if (r == 1) {
      if (co.dst && !co.win && pay > co.cap)
        return fail(HDFS_CRC32C_EINVAL, "copy-out buffer of %llu bytes is too small (%llu needed)",
                    (unsigned long long)co.cap, (unsigned long long)pay);
      if (payload_out) *payload_out = pay;
      scan_err(0, *nout);
      if (first_err_out) *first_err_out = ferr == SIZE_MAX ? *nout : ferr;
      return HDFS_CRC32C_OK;
    }
    *nout = 0;
    *consumed = 0;
  }
  if (!c.v_stream) HIPCHK(hipStreamCreateWithFlags(&c.v_stream, hipStreamNonBlocking));
  const uint32_t sflags = HDFS_CRC32C_SEG_BE | (ctype == HDFS_CRC32C_CSUM_CRC32 ? HDFS_CRC32C_SEG_CRC32 : 0u);
  const int tset = ctype == HDFS_CRC32C_CSUM_CRC32 ? 1 : 0;
  struct Pass {
    size_t slot, off, n;
    uint32_t nseg, count;
    uint64_t bm_cap;
    uint32_t seq;
  };
  std::vector<Pass> passes;
  uint64_t pos = 0, payload = 0;
  size_t n = 0;  // records in dst
  int rc = HDFS_CRC32C_OK;
  bool fallback = false;
  // speculation: tried at each pass of a large enough stream until a launch
  // meets a header off its prediction (an irregular stream: later passes
  // frame); last_spec = the call's last command was a taken speculative
  // launch, whose completion word the host has seen
  bool try_spec = verify && g_spec && allow_spec, last_spec = false;
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  double t_enq = 0, t_sync = 0, t_fill = 0;
  auto us_since = [](clk::time_point a, clk::time_point b) {
    return std::chrono::duration<double, std::micro>(b - a).count();
  };
  // (a read window that is full takes no further packets)
  while (n < max_pkts && pos < len && !(co.win && payload >= co.cap)) {
    const uint64_t left = len - pos;
    const uint32_t count = uint32_t(std::min<uint64_t>({uint64_t(max_pkts - n), kGridMaxCount, left / 6 + 1}));
    const uint64_t bm_cap = left / 32 + count + 64;  // >= sum of ceil(chunks / 8) over the run
    const auto tq0 = clk::now();
    const GridLayout L(count, bm_cap);
    const size_t si = passes.size();
    if ((rc = reserve_grid(c, si, L))) break;
    uint8_t *dg = c.grid[si].d, *hg = c.grid[si].h;
    auto *recs = reinterpret_cast<hdfs_crc32c_packet *>(dg + L.recs);
    auto *sum = reinterpret_cast<GridSummary *>(dg + L.sum);
    auto *ctr = reinterpret_cast<uint32_t *>(dg + L.ctr);
    const GridBufs gb{recs,
                      dg + L.look,
                      reinterpret_cast<SegDev *>(dg + L.segs),
                      reinterpret_cast<uint32_t *>(dg + L.seg2pkt),
                      reinterpret_cast<uint32_t *>(dg + L.fb),
                      ctr,
                      reinterpret_cast<uint32_t *>(dg + L.done),
                      reinterpret_cast<uint32_t *>(dg + L.exc),
                      sum,
                      c.grid[si].hd + L.h_sum,
                      next_grid_seq(c)};
    auto *hsum = reinterpret_cast<GridSummary *>(hg + L.h_sum);
    __atomic_store_n(&hsum->seq, 0u, __ATOMIC_RELEASE);
    // framing and the segment table on c.stream; the verify of the run is
    // queued behind it right away, sized by the device-built summary (no host
    // round trip before the GPU starts verifying)
    // copy-out: this pass fills the destination from what earlier passes
    // delivered on, within what is left of it
    const uint64_t done_b = std::min(payload, co.cap);
    if (pos > 0 && left <= kSmallRunBytes && g_tail_small) {
      // what follows a taken run -- a block's short last packet, the empty
      // end packet -- in ONE short-run launch instead of a framing pass and
      // its verify (three launches); it hands back (0) unless the walk ends
      // inside it, and the regular pass takes over
      CopyOut co2 = co;
      if (co.dst) {
        co2.dst = co.dst + done_b;
        co2.cap = co.cap - done_b;
      }
      size_t nr = 0;
      uint64_t used_r = 0, pay_r = 0;
      const int r = small_run(c, d + pos, left, proto, cs, ctype, verify, co2, max_pkts - n, dst + n, &nr, &used_r,
                              &pay_r);
      if (r < 0) {
        rc = r;
        break;
      }
      if (r == 1) {
        for (size_t k = 0; k < nr; k++) dst[n + k].stream_off += pos;
        scan_err(n, nr);
        if (co.dst && !co.win && payload + pay_r > co.cap) {
          rc = fail(HDFS_CRC32C_EINVAL, "copy-out buffer of %llu bytes is too small (%llu needed so far)",
                    (unsigned long long)co.cap, (unsigned long long)(payload + pay_r));
          break;
        }
        n += nr;
        payload += pay_r;
        *consumed = pos + used_r;
        last_spec = true;  // (its completion words were seen: the call's last command has run)
        break;
      }
    }
    if (try_spec && left > kSmallRunBytes) {
      SpecResult sr;
      // a verify (no copy-out; a read window is applied to the records
      // afterwards): when the stream's rest after the run is short -- a
      // block's short last packet and the empty end packet -- its short-run
      // launch is queued behind the speculative kernel as soon as the early
      // block sizes the run, so it runs without a host round trip in between
      SrLaunch tl;
      uint64_t tail_at = 0;
      const std::function<void(uint32_t, uint64_t)> tail_fn = [&](uint32_t cnt, uint64_t stride) {
        const uint64_t at = pos + uint64_t(cnt) * stride;
        const size_t room = max_pkts - n > cnt ? max_pkts - n - cnt : 0;
        // (a rest within one header window is one packet the kernel frames
        // itself -- the empty end packet of a block -- and needs no launch)
        if (at >= len || len - at <= kHdrWin || len - at > kSmallRunBytes || !room || !g_tail_small) return;
        // (on its own stream: the kernel's early block means every command
        // queued before it has run, so the rest's bytes are as ready as the
        // run's; it starts on the first CU the speculative kernel frees)
        hipStream_t ts = g_tail_stream ? c.t_stream : nullptr;
        if (sr_launch(c, true, d + at, len - at, proto, cs, ctype, verify, CopyOut{}, room, tl, ts) == 0) tail_at = at;
      };
      if (!co.dst) t_tail_hook = &tail_fn;  // (a window without copy-out: the host applies it to the records after)
      rc = spec_pass(c, d, len, pos, count, proto, cs, ctype, co, done_b, dg + L.bm,
                     reinterpret_cast<uint32_t *>(dg + L.fb), dst + n, sr);
      t_tail_hook = nullptr;
      // the queued rest: taken when the walk goes on exactly there, else
      // waited for and dropped
      size_t nt = 0;
      uint64_t used_t = 0, pay_t = 0;
      int got_tail = 0;
      if (tail_at) {
        const bool usable = !rc && sr.taken && !sr.end && sr.next == tail_at;
        std::vector<hdfs_crc32c_packet> scratch;
        hdfs_crc32c_packet *to = dst + n + sr.recorded;
        if (!usable) {
          scratch.resize(tl.count);
          to = scratch.data();
        }
        const size_t room = usable ? max_pkts - n - sr.recorded : tl.count;
        const int r2 = sr_collect(c, tl, len - tail_at, CopyOut{}, room, to, &nt, &used_t, &pay_t);
        if (r2 < 0 && !rc) rc = r2;
        got_tail = usable && r2 == 1 ? 1 : 0;
      }
      if (rc) break;
      if (sr.taken) {
        if (co.dst && !co.win && payload + sr.payload > co.cap) {
          rc = fail(HDFS_CRC32C_EINVAL, "copy-out buffer of %llu bytes is too small (%llu needed so far)",
                    (unsigned long long)co.cap, (unsigned long long)(payload + sr.payload));
          break;
        }
        const bool read_over = co.win && read_window_over(dst + n, sr.recorded, co, sr.exc_idx.data(),
                                                          sr.exc_idx.size());
        if (sr.first_err != UINT32_MAX && ferr == SIZE_MAX) ferr = n + sr.first_err;
        n += sr.recorded;
        payload += sr.payload;
        *consumed = sr.consumed;
        last_spec = true;
        if (sr.end || read_over) break;
        if (got_tail) {  // the rest, verified behind the run
          for (size_t k = 0; k < nt; k++) dst[n + k].stream_off += tail_at;
          scan_err(n, nt);
          n += nt;
          payload += pay_t;
          *consumed = tail_at + used_t;
          break;
        }
        pos = sr.next;
        continue;
      }
      // not taken: the regular pass from the same offset (an irregular run
      // gets no further speculative launches in this call)
      try_spec = false;
    }
    last_spec = false;
    ferr_known = false;  // (a framing pass: its verdicts arrive with the records)
    hipError_t e = launch_frame_grid(d, len, pos, count, proto, cs, ctype, verify ? 1 : 0, sflags, dg + L.bm,
                                     co.dst ? co.dst + done_b : nullptr, co.dst ? co.cap - done_b : 0, co.win ? 1 : 0,
                                     co.client_offset, gb, c.stream,
                                     (kDiag && g_diag) ? g_diag + kFrameStampOff : nullptr);
    if (e != hipSuccess) {
      rc = fail(HDFS_CRC32C_EHIP, "device framing: %s", hipGetErrorString(e));
      break;
    }
    if (verify) {
      // generic tiles: at most one per packet for chunk sizes the tiled
      // kernel takes, else every tile of every packet
      const uint64_t gtiles_ub = cs % kRoundBytes == 0 ? count : left / (uint64_t(cs) * kTileChunks) + 2ull * count;
      // rounds: at most one per 512 B of the rest of the stream
      // (the generic tiles ride in the verify launch)
      rc = launch_verify_dyn(c, reinterpret_cast<const SegDev *>(dg + L.segs), sum, left / kRoundBytes, gtiles_ub,
                             reinterpret_cast<uint32_t *>(dg + L.fb), reinterpret_cast<unsigned long long *>(ctr + 16),
                             ctr, c.stream, tset, co.dst != nullptr);
      if (rc) break;
      auto *bad = reinterpret_cast<GridBad *>(dg + L.bad);
      __atomic_store_n(&reinterpret_cast<GridSummary *>(hg + L.h_sum2)->seq, 0u, __ATOMIC_RELEASE);
      HIPCHK(launch_grid_finalize(reinterpret_cast<const SegDev *>(dg + L.segs), 0xFFFFFFFFu,
                                  reinterpret_cast<const uint32_t *>(dg + L.seg2pkt),
                                  reinterpret_cast<const uint32_t *>(dg + L.fb), bad, count, sum,
                                  c.grid[si].hd + L.h_sum2, kBadFirst, gb.seq, c.stream));
    }
    // the summary lands in pinned memory with its sequence number last: poll
    // it (a fault is caught by the stream synchronisation after 200 ms)
    const auto tq = clk::now();
    for (uint32_t spin = 1;; spin++) {
      if (__atomic_load_n(&hsum->seq, __ATOMIC_ACQUIRE) == gb.seq) break;
      if ((spin & 4095u) == 0 && clk::now() - tq > std::chrono::milliseconds(200)) {
        e = hipStreamSynchronize(c.stream);
        if (e == hipSuccess && __atomic_load_n(&hsum->seq, __ATOMIC_ACQUIRE) != gb.seq) e = hipErrorUnknown;
        break;
      }
#if defined(__x86_64__) || defined(__i386__)
      __builtin_ia32_pause();
#endif
    }
    t_enq += us_since(tq0, tq);
    const auto tf = clk::now();
    t_sync += us_since(tq, tf);
    if (e != hipSuccess) {
      rc = fail(HDFS_CRC32C_EHIP, "device framing: %s", hipGetErrorString(e));
      break;
    }
    GridSummary S;
    std::memcpy(&S, hsum, sizeof(S));
    if (co.dst && !co.win && payload + S.payload > co.cap) {
      rc = fail(HDFS_CRC32C_EINVAL, "copy-out buffer of %llu bytes is too small (%llu needed so far)",
                (unsigned long long)co.cap, (unsigned long long)(payload + S.payload));
      break;
    }
    // the pass's records, written while the verify kernel runs: predicted
    // from packet 0, then the exceptions (all of them from HBM if the host
    // area could not hold them)
    if (S.recorded) {
      hdfs_crc32c_packet r0;
      std::memcpy(&r0, hg + L.h_sum + kGridHostRec0, sizeof(r0));
      hdfs_crc32c_packet *out = dst + n;
      for (uint32_t k = 0; k < S.recorded; k++) {
        hdfs_crc32c_packet &r = out[k];
        r = r0;
        r.stream_off = pos + uint64_t(k) * S.stride;
        r.offset_in_block = r0.offset_in_block + int64_t(k) * r0.data_len;
        r.seqno = r0.seqno + int64_t(k);
      }
      if (S.nexc <= kExcMax) {
        const auto *idx = reinterpret_cast<const uint32_t *>(hg + L.h_sum + kGridHostIdx);
        const uint8_t *er = hg + L.h_sum + kGridHostExc;
        for (uint32_t j = 0; j < S.nexc; j++) std::memcpy(&out[idx[j]], er + size_t(j) * kGridRecBytes, kGridRecBytes);
      } else {
        if (!c.r_stream) HIPCHK(hipStreamCreateWithFlags(&c.r_stream, hipStreamNonBlocking));
        HIPCHK(hipMemcpyAsync(out, recs, size_t(S.recorded) * sizeof(hdfs_crc32c_packet), hipMemcpyDeviceToHost,
                              c.r_stream));
        HIPCHK(hipStreamSynchronize(c.r_stream));
      }
    }
    t_fill += us_since(tf, clk::now());
    passes.push_back({si, n, S.recorded, verify ? S.nseg : 0u, count, bm_cap, gb.seq});
    const bool read_over =
        co.win && read_window_over(dst + n, S.recorded, co,
                                   S.nexc <= kExcMax ? reinterpret_cast<const uint32_t *>(hg + L.h_sum + kGridHostIdx)
                                                     : nullptr,
                                   S.nexc);
    n += S.recorded;
    payload += S.payload;
    *consumed = S.consumed;
    if (S.last_status == kGridStop || S.last_status == kGridMore || read_over) break;
    pos = S.next_pos;
    if (S.last_status == kGridOff && S.recorded <= 2) {
      fallback = true;
      break;
    }
  }
  const auto t1 = clk::now();
  if (!rc && fallback && n < max_pkts) {
    std::vector<hdfs_crc32c_packet> more;
    rc = walk_device_stream(c, d, len, proto, cs, ctype, max_pkts - n, verify, more, consumed, pos, co, &payload);
    if (!rc && !more.empty()) {
      std::memcpy(dst + n, more.data(), more.size() * sizeof(hdfs_crc32c_packet));
      n += more.size();
    }
  }
  const auto t1d = clk::now();
  // The last command this call queued on c.stream publishes a sequence
  // number to pinned memory as its last memory operation: the last pass's
  // finalize (verify; launched for every verify pass, with or without
  // segments) or its framing pass (parse only, polled above).  Once it is
  // seen, every command of the call has run to completion without a fault
  // (a faulting kernel stops the stream: nothing after it runs), so the
  // stream synchronisation -- ~15 us right after the dispatch, the
  // runtime's completion bookkeeping (HDFS_CRC32C_DSTREAM_TRACE) -- is
  // skipped; otherwise (an error, a poll timeout) it drains the stream and
  // reports the fault.
  bool all_done = !rc && !fallback && last_spec;
  if (!rc && !fallback && !last_spec && !passes.empty()) {
    if (!verify) {
      all_done = true;
    } else {
      const Pass &pl = passes.back();
      const auto *s2 = reinterpret_cast<const GridSummary *>(c.grid[pl.slot].h + GridLayout(pl.count, pl.bm_cap).h_sum2);
      const auto tq = clk::now();
      for (uint32_t spin = 1;; spin++) {
        if (__atomic_load_n(&s2->seq, __ATOMIC_ACQUIRE) == pl.seq) {
          all_done = true;
          break;
        }
        if ((spin & 4095u) == 0 && clk::now() - tq > std::chrono::milliseconds(200)) break;  // the sync below reports
#if defined(__x86_64__) || defined(__i386__)
        __builtin_ia32_pause();
#endif
      }
    }
  }
  // drained even after an error: the tables of queued work live in this context
  hipError_t e = all_done ? hipSuccess : hipStreamSynchronize(c.stream);
  const hipError_t e2 = fallback ? hipStreamSynchronize(c.v_stream) : hipSuccess;
  const auto t1e = clk::now();
  if (!rc && e != hipSuccess) rc = fail(HDFS_CRC32C_EHIP, "verify: %s", hipGetErrorString(e));
  if (!rc && e2 != hipSuccess) rc = fail(HDFS_CRC32C_EHIP, "verify: %s", hipGetErrorString(e2));
  if (!rc && co.dst && !co.win && payload > co.cap)
    rc = fail(HDFS_CRC32C_EINVAL, "copy-out buffer of %llu bytes is too small (%llu needed)",
              (unsigned long long)co.cap, (unsigned long long)payload);
  if (rc) return rc;
  // verify verdicts: the compact list of packets with bad chunks
  for (const Pass &p : passes) {
    if (!p.nseg) continue;
    const GridLayout L(p.count, p.bm_cap);
    const uint8_t *hg = c.grid[p.slot].h;
    const uint32_t nbad = reinterpret_cast<const GridSummary *>(hg + L.h_sum2)->nbad;
    std::vector<GridBad> more;
    const GridBad *bad = reinterpret_cast<const GridBad *>(hg + L.h_sum2 + 256);
    if (nbad > kBadFirst) {
      more.resize(nbad);
      HIPCHK(hipMemcpy(more.data(), c.grid[p.slot].d + L.bad, nbad * sizeof(GridBad), hipMemcpyDeviceToHost));
      bad = more.data();
    }
    for (uint32_t i = 0; i < nbad; i++) {
      hdfs_crc32c_packet &k = dst[p.off + bad[i].pkt];
      k.error = HDFS_CRC32C_ERR_DATANODE_BAD_CHECKSUM;
      k.first_bad = bad[i].first_bad;
      k.bad_chunks = bad[i].bad_chunks;
    }
  }
  if (g_dstream_trace) {  // diagnostic: where a device-stream call spends its time (us)
    const auto t2 = clk::now();
    auto us = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    std::fprintf(stderr,
                 "dstream grid pkts=%zu passes=%zu fallback=%d enq_us=%.1f sum_sync_us=%.1f fill_us=%.1f "
                 "loop_us=%.1f fallback_us=%.1f verify_sync_us=%.1f total_us=%.1f\n",
                 n, passes.size(), int(fallback), t_enq, t_sync, t_fill, us(t0, t1), us(t1, t1d), us(t1d, t1e),
                 us(t0, t2));
  }
  *nout = n;
  if (payload_out) *payload_out = payload;
  if (first_err_out && ferr_known && !fallback) *first_err_out = ferr == SIZE_MAX ? n : ferr;
  return HDFS_CRC32C_OK;
}

// The read loop over a walked run, for a client read window
// (_datanode_read's `while (remains_tot > 0) _recv_packet(...)`,
// src/datanode.c:1476-1481, through _process_recv_packet and
// _recv_packet_copy_data, :2439-2456, :2470-2549).  The read ends at its
// first error, as the reference's does:
//   - a framing error (:2439-2446) or bad CRCs (:2470-2475: bad_crcs, the
//     loop breaks at :1478 and the call returns BAD_CHECKSUM, :1500-1505):
//     the packet is recorded, delivers nothing and is not consumed;
//   - a framing error is not consumed, except an empty packet not flagged
//     last (PACKET_SIZE, :2450-2455: its header is);
//   - an empty last packet while the read wants bytes is BAD_LASTPACKET
//     (:2450-2456; its header is consumed);
//   - a packet that starts past the read (c_begin >= dataLen) is
//     UNEXPECTED_READ_OFFSET (:2483-2486), not consumed;
//   - a packet delivers min(dataLen - c_begin, remains) bytes, and one
//     flagged lastPacketInBlock that leaves the read short is BAD_LASTPACKET
//     after its bytes are copied (:2545-2546).
// Records past the packet that ends the read are dropped (the device may have
// verified them: the window is a function of the headers only, which lets it
// place every copy before any verdict is known; the reference never reads
// them), so the result does not depend on how the destination is split.  The
// destination (co.cap bytes) may be smaller than the read (co.want): once it
// is full the walk stops with AGAIN (`rlen == 0 && remains_tot > 0`,
// :2547-2549) -- a packet whose bytes were only partly delivered is dropped
// from the records and `consumed` ends before it (the caller re-passes it
// with client_offset advanced, so its new c_begin skips what it delivered:
// the reference's remains_pkt, :2356-2361).  *delivered = the bytes the
// reference copies before its loop returns.  Returns 1 for AGAIN, else 0.
// pieces (optional): the delivered bytes as (stream offset, length) in
// delivery order -- what a host-memory copy-out copies.
using Pieces = std::vector<std::pair<uint64_t, uint64_t>>;
// examined (optional): records the walk looked at (the one it stopped at
// included, a partly delivered packet too).
int apply_read_window(hdfs_crc32c_packet *p, size_t &n, uint64_t &consumed, const CopyOut &co,
                      uint64_t *delivered, Pieces *pieces = nullptr, size_t *examined = nullptr) {
  uint64_t remains = co.want, room = co.cap, got = 0;
  int again = 0;
  if (pieces) pieces->clear();
  if (examined) *examined = n;
  auto piece = [&](const hdfs_crc32c_packet &r, uint32_t cb, uint64_t bytes) {
    if (pieces && bytes) pieces->push_back({r.stream_off + r.header_len + uint64_t(r.crc_len) + cb, bytes});
  };
  for (size_t k = 0; k < n; k++) {
    hdfs_crc32c_packet &r = p[k];
    const uint64_t end = r.stream_off + r.header_len + uint64_t(r.crc_len > 0 ? r.crc_len : 0) +
                         uint64_t(r.data_len > 0 ? r.data_len : 0);
    if (examined) *examined = k + 1;
    if (r.error) {  // framing error or bad CRCs
      n = k + 1;
      // an empty packet not flagged last fails with its header consumed
      // (src/datanode.c:2450-2455); no other framing error consumes anything
      const bool empty_not_last = r.error == HDFS_CRC32C_ERR_DATANODE_PACKET_SIZE && r.data_len == 0 && r.crc_len == 0;
      consumed = r.stream_off + (empty_not_last ? r.header_len : 0);
      break;
    }
    if (r.data_len == 0) {  // the empty last packet (a non-last one is a framing error)
      r.error = HDFS_CRC32C_ERR_DATANODE_BAD_LASTPACKET;
      n = k + 1;
      consumed = end;
      break;
    }
    uint32_t cb = 0;
    const uint32_t avail = frame::read_avail(r, true, co.client_offset, cb);
    if (avail == 0) {
      r.error = HDFS_CRC32C_ERR_DATANODE_UNEXPECTED_READ_OFFSET;
      n = k + 1;
      consumed = r.stream_off;
      break;
    }
    const uint64_t want = std::min<uint64_t>(avail, remains);  // remains_pkt
    if (want > room) {
      // the destination fills inside this packet: its rest is the next
      // call's (the reference returns AGAIN here with remains_pkt > 0)
      got += room;
      piece(r, cb, room);
      n = k;
      consumed = r.stream_off;
      again = 1;
      break;
    }
    remains -= want;
    room -= want;
    got += want;
    piece(r, cb, want);
    if (r.last && remains > 0) r.error = HDFS_CRC32C_ERR_DATANODE_BAD_LASTPACKET;
    if (r.error || remains == 0 || room == 0) {
      n = k + 1;
      consumed = end;
      again = !r.error && remains > 0;  // full exactly at this packet's end
      break;
    }
  }
  if (delivered) *delivered = got;
  return again;
}

int verify_packets_dev_impl(int dev, const uint8_t *stream, uint64_t len, int proto, uint32_t cs, int ctype,
                            hdfs_crc32c_packet *pkts, size_t max_pkts, size_t *npkts, uint64_t *consumed,
                            bool verify, const CopyOut &co = CopyOut{}, uint64_t *delivered = nullptr,
                            Pieces *pieces = nullptr) {
  DevCtx *cp = nullptr;
  int rc;
  if ((rc = ctx_init(dev, &cp))) return rc;
  DevCtx &c = *cp;
  DeviceGuard g(c.dev);
  std::lock_guard<std::mutex> lk(c.mu);
  uint64_t used = 0;
  size_t n = 0, fe = SIZE_MAX;
  const auto tw0 = std::chrono::steady_clock::now();
  rc = grid_walk(c, stream, len, proto, cs, ctype, max_pkts, verify, co, pkts, &n, &used, nullptr, true, &fe);
  const auto tw1 = std::chrono::steady_clock::now();
  if (kDiag) {  // a broken kernel invariant outranks whatever it led to
    const int r2 = device_checks("device packet run");
    if (r2) return r2;
  }
  if (rc) return rc;
  int again = 0;
  if (co.win) {
    again = apply_read_window(pkts, n, used, co, delivered, pieces);
  } else if (delivered) {  // what the reference copies out before its loop returns an error (src/datanode.c:2470-2486)
    uint64_t b = 0;
    for (size_t i = 0; i < n; i++) {
      if (pkts[i].error) break;
      b += uint64_t(pkts[i].data_len);
    }
    *delivered = b;
  }
  if (npkts) *npkts = n;
  if (consumed) *consumed = used;
  // the call's status: the first record's error, known to the walk without
  // a scan when its passes were speculative or short runs (a scan of 16384
  // records after a 1 GiB walk costs ~5 us)
  if (co.win || fe == SIZE_MAX) {
    rc = first_error(pkts, n);
  } else {
    rc = fe < n ? pkts[fe].error : HDFS_CRC32C_OK;
    if (kDiag && rc != first_error(pkts, n))
      return fail(HDFS_CRC32C_EHIP, "first-error hint %zu of %zu disagrees with the records", fe, n);
  }
  if (g_dstream_trace) {  // diagnostic: the call around its walk (us)
    auto us = [](std::chrono::steady_clock::time_point x, std::chrono::steady_clock::time_point y) {
      return std::chrono::duration<double, std::micro>(y - x).count();
    };
    std::fprintf(stderr, "dstream call pkts=%zu walk_us=%.1f after_walk_us=%.1f\n", n, us(tw0, tw1),
                 us(tw1, std::chrono::steady_clock::now()));
  }
  return rc ? rc : again ? HDFS_CRC32C_AGAIN : HDFS_CRC32C_OK;
}

// Synchronous packet-run verify: framing, then pieces of <= 64 MiB of wire
// bytes alternate between the context's two device slots (H2D of piece k+1
// overlaps the kernels of piece k).
int verify_packets_impl(const uint8_t *stream, uint64_t len, int proto, uint32_t cs, int ctype,
                        hdfs_crc32c_packet *pkts, size_t max_pkts, size_t *npkts, uint64_t *consumed, bool verify) {
  if (npkts) *npkts = 0;
  if (consumed) *consumed = 0;
  if (max_pkts && !pkts) return fail(HDFS_CRC32C_EINVAL, "null packet array");
  int rc = check_framing_args(proto, cs, ctype, g_err, sizeof(g_err));
  if (rc) return rc;
  if (len && stream) {
    const int dev = stream_device(stream);
    if (dev >= 0) return verify_packets_dev_impl(dev, stream, len, proto, cs, ctype, pkts, max_pkts, npkts, consumed,
                                                 verify);
  }
  std::vector<hdfs_crc32c_packet> recs;
  uint64_t used = 0;
  rc = parse_packet_stream(stream, len, proto, cs, ctype, max_pkts, recs, &used, g_err, sizeof(g_err));
  if (rc) return rc;
  std::vector<size_t> vidx;  // packets whose chunks go to the GPU
  if (verify && ctype != HDFS_CRC32C_CSUM_NULL)
    for (size_t i = 0; i < recs.size(); i++)
      if (!recs[i].error && recs[i].crc_len > 0) vidx.push_back(i);
  if (!vidx.empty()) {
    DevCtx *cp = nullptr;
    if ((rc = ctx_init(-1, &cp))) return rc;
    DevCtx &c = *cp;
    DeviceGuard g(c.dev);
    std::lock_guard<std::mutex> lk(c.mu);
    // One packet of <= 64 KiB (the common per-read case): one launch of the
    // small-call kernel instead of the H2D / gather / verify piece pipeline.
    if (vidx.size() == 1 && small_ok(uint64_t(recs[vidx[0]].data_len), cs)) {
      hdfs_crc32c_packet &k = recs[vidx[0]];
      const uint8_t *crcp = stream + k.stream_off + k.header_len;
      rc = small_call(c, kModeVerify, uint32_t(k.data_len), cs, 0xFFFFFFFFu, true,
                      ctype == HDFS_CRC32C_CSUM_CRC32 ? 1 : 0, nullptr, crcp + k.crc_len, crcp, uint32_t(k.crc_len));
      if (rc) return rc;
      if (c.h_small_out[0] != 0xFFFFFFFFu) {
        k.error = HDFS_CRC32C_ERR_DATANODE_BAD_CHECKSUM;
        k.first_bad = int32_t(c.h_small_out[0]);
        k.bad_chunks = c.h_small_out[1];
      }
      vidx.clear();
    }
  }
  if (!vidx.empty()) {
    DevCtx *cp = nullptr;
    if ((rc = ctx_init(-1, &cp))) return rc;
    DevCtx &c = *cp;
    DeviceGuard g(c.dev);
    std::lock_guard<std::mutex> lk(c.mu);
    std::vector<std::pair<size_t, size_t>> pieces;  // [v0, v1) into vidx
    for (size_t v = 0; v < vidx.size(); v++) {
      if (pieces.empty() || wire_end(recs[vidx[v]]) - wire_begin(recs[vidx[pieces.back().first]]) > kPieceCap)
        pieces.push_back({v, v});
      pieces.back().second = v + 1;
    }
    std::vector<PieceLayout> lay(pieces.size());
    std::vector<size_t> hoff(pieces.size());
    size_t htotal = 0;
    for (size_t i = 0; i < pieces.size(); i++) {
      layout_piece(recs.data(), vidx.data() + pieces[i].first, pieces[i].second - pieces[i].first, lay[i]);
      hoff[i] = htotal;
      htotal += align_up(lay[i].meta, 256);
    }
    if (htotal > c.k_hmeta_cap) {
      if (c.k_hmeta) HIPCHK(hipHostFree(c.k_hmeta));
      c.k_hmeta = nullptr;
      c.k_hmeta_cap = 0;
      HIPCHK(hipHostMalloc(&c.k_hmeta, htotal, hipHostMallocDefault));
      c.k_hmeta_cap = htotal;
    }
    if ((rc = pipe_reserve(c, kGatherSlice, 512, 1))) return rc;  // copy / compute streams
    // the wire bytes of the verified packets stay pinned until both streams
    // are drained, on every return path (crc32c_hostpin.h)
    HostPins hp({c.copy_stream, c.comp_stream});
    const uint64_t w0 = wire_begin(recs[vidx.front()]), w1 = wire_end(recs[vidx.back()]);
    if ((rc = hp.pin({{stream + w0, w1 - w0}}))) return rc;
    for (size_t i = 0; i < pieces.size(); i++) {
      PieceSlot &s = c.kslot[i & 1];
      if ((rc = reserve_slot(s, lay[i])) ||
          (rc = build_piece(recs.data(), vidx.data() + pieces[i].first, lay[i], cs, ctype, s, c.k_hmeta + hoff[i])) ||
          (rc = enqueue_piece(c, stream, lay[i], s, c.k_hmeta + hoff[i], ctype, c.copy_stream, c.comp_stream)))
        return rc;
    }
    if ((rc = hp.done(HDFS_CRC32C_OK))) return rc;
    for (size_t i = 0; i < pieces.size(); i++)
      finish_piece(recs.data(), vidx.data() + pieces[i].first, lay[i], c.k_hmeta + hoff[i]);
  }
  if (!recs.empty()) std::memcpy(pkts, recs.data(), recs.size() * sizeof(hdfs_crc32c_packet));
  if (npkts) *npkts = recs.size();
  if (consumed) *consumed = used;
  return first_error(recs.data(), recs.size());
}

// ---- asynchronous verify jobs (hdfs_crc32c_verify_packets_submit / _wait) ----
// A device-resident run is verified by a speculative launch on a job slot's
// own stream; the wait collects it and, when the launch did not take the
// whole stream (another packet size follows, more packets than one pass, or
// no run at all), frames and verifies the rest synchronously -- so the result
// is hdfs_crc32c_verify_packets' in every case.
// Coalescing (a datanode verifying a stream of received blocks, one job per
// block): a launch carries a fixed cost of ~13 us whatever its size, so runs
// submitted while an earlier launch is still running are not launched one by
// one: they queue (runs of one layout key: protocol, chunk size, checksum
// type, length, record room) and go out together as ONE batch launch of up to
// kSpecRunsMax runs (spec_verify_kernel<..., 1>, the path of
// hdfs_crc32c_verify_blocks_submit) when
//   - a submit finds no launch running (the GPU would idle),
//   - a wait needs a queued job, or would block on a running launch (the
//     queue goes out first, so the GPU has it behind the running one),
//   - the queue holds kSpecRunsMax runs, or a run of another key arrives.
// The results are per job exactly as before.  A launch's results are copied
// out of its slot when it is collected (by the first wait of one of its
// jobs, or to free the slot for a new launch), so its jobs may be waited in
// any order.
struct JobGroup {
  int slot = -1;
  SpecLaunch L;
  uint32_t m = 0;                          // runs in the launch
  size_t per = 0;                          // records per run in recs
  bool collected = false, single_not_taken = false;
  int rc = 0;                              // the collection's status
  // [m][per], not zero-filled: per is max_pkts-sized (up to 65 537) and
  // only the records a run produces are written and read
  std::unique_ptr<hdfs_crc32c_packet[]> recs;
  std::vector<SpecRunResult> rr;           // [m]
  int refs = 0;                            // jobs not yet waited for
};
}  // namespace
struct JobQueue {
  std::vector<hdfs_crc32c_job *> pending;  // queued runs, in submit order
  struct Key {
    int proto, ctype;
    uint32_t cs;
    uint64_t len;
    size_t max_pkts;
    bool operator==(const Key &o) const {
      return proto == o.proto && ctype == o.ctype && cs == o.cs && len == o.len && max_pkts == o.max_pkts;
    }
  } key{};
  std::vector<JobGroup *> running;         // launched, not collected (oldest first)
  size_t outstanding = 0;                  // jobs submitted and not yet waited for
};
}  // namespace hdfs_crc32c

struct hdfs_crc32c_job {
  int dev = -1;
  std::vector<const uint8_t *> runs;  // the block streams (one for hdfs_crc32c_verify_packets_submit)
  std::vector<uint64_t> lens;
  bool batch = false;                 // hdfs_crc32c_verify_blocks_submit
  std::vector<size_t> sel;            // the blocks the launch covers (its runs, in order)
  int proto = 0, ctype = 0;
  uint32_t cs = 0;
  size_t max_pkts = 0;
  bool queued = false;                // waiting in the device's queue for a launch
  hdfs_crc32c::JobGroup *grp = nullptr;  // its launch (runs grp_run .. grp_run + sel.size() - 1)
  uint32_t grp_run = 0;
};

namespace hdfs_crc32c {
namespace {

JobQueue &jobq(DevCtx &c) {
  if (!c.jobq) c.jobq = new JobQueue;
  return *c.jobq;
}

// A launch is done once its early block says the run was not taken (every
// workgroup returns at once) or its final block is published.
bool group_done(DevCtx &c, const JobGroup &g) {
  const SpecSlot &S = c.job_slot[g.slot];
  const auto *early = reinterpret_cast<const SpecEarly *>(S.h);
  const auto *fin = reinterpret_cast<const SpecFinal *>(S.h + sizeof(SpecEarly));
  if (__atomic_load_n(&early->seq, __ATOMIC_ACQUIRE) != g.L.seq) return false;
  if (!__atomic_load_n(&early->eligible, __ATOMIC_RELAXED)) return true;
  return __atomic_load_n(&fin->seq, __ATOMIC_ACQUIRE) == g.L.seq;
}

// Copy a launch's results out of its slot and free the slot.
int group_collect(DevCtx &c, JobQueue &q, JobGroup *g) {
  if (g->collected) return g->rc;
  SpecSlot &S = c.job_slot[g->slot];
  g->recs.reset(new (std::nothrow) hdfs_crc32c_packet[g->per * g->m]);
  g->rr.assign(g->m, SpecRunResult{});
  if (!g->recs) {
    g->collected = true;
    g->rc = fail(HDFS_CRC32C_ENOMEM, "records of %u runs", g->m);
    // the launch still owns its slot until it has run: wait for it first
    (void)hipStreamSynchronize(S.stream);
    c.job_busy[g->slot] = false;
    q.running.erase(std::remove(q.running.begin(), q.running.end(), g), q.running.end());
    return g->rc;
  }
  int rc;
  if (g->m == 1) {
    SpecResult sr;
    rc = spec_collect(c, S, g->L, CopyOut{}, g->recs.get(), sr);
    g->rr[0].taken = sr.taken;
    g->rr[0].end = sr.end;
    g->rr[0].recorded = sr.recorded;
    g->rr[0].consumed = sr.consumed;
    g->rr[0].next = sr.next;
    g->single_not_taken = !sr.taken;
  } else {
    std::vector<hdfs_crc32c_packet *> dst(g->m);
    std::vector<uint64_t> pos0(g->m, 0);
    for (uint32_t r = 0; r < g->m; r++) dst[r] = g->recs.get() + r * g->per;
    rc = spec_collect_batch(S, g->L, g->m, pos0.data(), dst.data(), g->rr);
  }
  g->collected = true;
  g->rc = rc;
  c.job_busy[g->slot] = false;
  q.running.erase(std::remove(q.running.begin(), q.running.end(), g), q.running.end());
  return rc;
}

// Launch runs (streams[r], lens[r]) of one layout key as one speculative
// launch on a free job slot -- collecting the oldest running launch first
// when all slots are busy.  -> the group (refs 0), or null with rc set.
JobGroup *group_launch(DevCtx &c, JobQueue &q, const uint8_t *const *streams, const uint64_t *lens, uint32_t m,
                       int proto, uint32_t cs, int ctype, size_t max_pkts, int *rcp, bool early) {
  int slot = -1;
  for (;;) {
    for (int i = 0; i < kMaxJobs && slot < 0; i++)
      if (!c.job_busy[i]) slot = i;
    if (slot >= 0 || q.running.empty()) break;
    JobGroup *old = q.running.front();
    (void)group_collect(c, q, old);  // (its status stays with its jobs)
    if (old->refs == 0) delete old;  // every job of it returned before the launch ended
  }
  if (slot < 0) {
    *rcp = fail(HDFS_CRC32C_EHIP, "no free job slot");
    return nullptr;
  }
  SpecSlot &S = c.job_slot[slot];
  if (!S.stream) {  // on a hardware queue of its own: launches of different slots overlap
    uint64_t avoid[kMaxJobs + 1] = {c.q_main};
    for (int i = 0; i < kMaxJobs; i++) avoid[i + 1] = c.job_slot[i].q;
    int rq;
    if ((rq = stream_on_own_queue(c, &S.stream, &S.q, avoid, kMaxJobs + 1))) {
      *rcp = rq;
      return nullptr;
    }
  }
  // per run at most `count` packets; the bitmap takes ceil(chunks / 8) bytes
  // per packet (<= len / 32 + 1), first-bad one word per packet
  const uint32_t count = uint32_t(std::min<uint64_t>(uint64_t(max_pkts), kGridMaxCount));
  uint64_t bm_cap = 64, fbw = 0;
  for (uint32_t r = 0; r < m; r++) {
    const uint64_t cr = std::min<uint64_t>(count, lens[r] / 6 + 1);
    bm_cap += lens[r] / 32 + cr;
    fbw += cr;
  }
  bm_cap = align_up(bm_cap, 256);
  const uint64_t need = bm_cap + fbw * 4u + 256u;
  if (need > S.scratch_cap) {
    if (S.scratch) (void)hipFree(S.scratch);
    S.scratch = nullptr;
    S.scratch_cap = 0;
    if (hipMalloc(&S.scratch, need) != hipSuccess) {
      (void)hipGetLastError();
      *rcp = fail(HDFS_CRC32C_ENOMEM, "job scratch of %llu bytes", (unsigned long long)need);
      return nullptr;
    }
    S.scratch_cap = need;
  }
  auto *g = new (std::nothrow) JobGroup;
  if (!g) {
    *rcp = fail(HDFS_CRC32C_ENOMEM, "job launch");
    return nullptr;
  }
  g->slot = slot;
  g->m = m;
  g->per = size_t(count) + 1;
  int rc = spec_launch(c, S, S.stream, streams[0], lens[0], 0, count, proto, cs, ctype, CopyOut{}, 0, S.scratch,
                       reinterpret_cast<uint32_t *>(S.scratch + bm_cap), g->L, m, streams, lens, early);
  if (rc) {
    delete g;
    *rcp = rc;
    return nullptr;
  }
  c.job_busy[slot] = true;
  q.running.push_back(g);
  *rcp = HDFS_CRC32C_OK;
  return g;
}

// The queue goes out as one launch.  If the launch fails, its jobs are
// verified synchronously in their waits instead (the wait reports an error
// that persists).
void queue_flush(DevCtx &c, JobQueue &q) {
  if (q.pending.empty()) return;
  std::vector<const uint8_t *> s;
  std::vector<uint64_t> l;
  for (hdfs_crc32c_job *j : q.pending) {
    s.push_back(j->runs[0]);
    l.push_back(j->lens[0]);
  }
  int rc = 0;
  JobGroup *g = group_launch(c, q, s.data(), l.data(), uint32_t(s.size()), q.key.proto, q.key.cs, q.key.ctype,
                             q.key.max_pkts, &rc, g_job_early != 0);
  for (size_t r = 0; r < q.pending.size(); r++) {
    hdfs_crc32c_job *j = q.pending[r];
    j->queued = false;
    if (g) {
      j->grp = g;
      j->grp_run = uint32_t(r);
      g->refs++;
    }
  }
  q.pending.clear();
}

bool any_running(DevCtx &c, JobQueue &q) {
  for (JobGroup *g : q.running)
    if (!group_done(c, *g)) return true;
  return false;
}

int job_submit(const uint8_t *const *runs, const uint64_t *lens, size_t n, bool batch, int proto, uint32_t cs,
               int ctype, size_t max_pkts, hdfs_crc32c_job **out) {
  const int dev = stream_device(runs[0]);
  if (dev < 0) return fail(HDFS_CRC32C_EINVAL, "asynchronous verify takes device-resident streams");
  for (size_t r = 1; r < n; r++)
    if (stream_device(runs[r]) != dev) return fail(HDFS_CRC32C_EINVAL, "block %zu: not on device %d", r, dev);
  DevCtx *cp = nullptr;
  int rc;
  if ((rc = ctx_init(dev, &cp))) return rc;
  DevCtx &c = *cp;
  DeviceGuard g(c.dev);
  std::lock_guard<std::mutex> lk(c.mu);
  JobQueue &q = jobq(c);
  if (q.outstanding >= kMaxJobsOut)
    return fail(HDFS_CRC32C_EINVAL, "%zu verify jobs already outstanding on device %d", kMaxJobsOut, dev);
  auto *j = new (std::nothrow) hdfs_crc32c_job;
  if (!j) return fail(HDFS_CRC32C_ENOMEM, "job");
  j->dev = dev;
  j->runs.assign(runs, runs + n);
  j->lens.assign(lens, lens + n);
  j->batch = batch;
  j->proto = proto;
  j->ctype = ctype;
  j->cs = cs;
  j->max_pkts = max_pkts;
  // The launch covers the largest group of blocks of one length (the first
  // such group on a tie): blocks of one layout and length hold the same
  // number of packets, which a batch launch needs (its table maps packet k
  // to run k / count); the others -- a file's short last block, say -- are
  // verified one by one in the wait.  A stream too short for a run the
  // launch would take is left to the wait too.
  for (size_t b = 0; b < n; b++) {
    if (lens[b] <= kSmallRunBytes) continue;
    size_t same = 0;
    for (size_t q2 = 0; q2 < n; q2++) same += lens[q2] == lens[b] ? 1u : 0u;
    if (j->sel.empty() || same > j->sel.size()) {
      j->sel.clear();
      for (size_t q2 = 0; q2 < n; q2++)
        if (lens[q2] == lens[b]) j->sel.push_back(q2);
    }
  }
  q.outstanding++;
  *out = j;
  const bool spec = ctype != HDFS_CRC32C_CSUM_NULL && g_spec && max_pkts >= 2 && !j->sel.empty();
  if (!spec) return HDFS_CRC32C_OK;  // all of it in the wait
  if (batch) {  // a job of blocks: its own launch now
    std::vector<const uint8_t *> s;
    std::vector<uint64_t> l;
    for (size_t b : j->sel) {
      s.push_back(runs[b]);
      l.push_back(lens[b]);
    }
    JobGroup *grp = group_launch(c, q, s.data(), l.data(), uint32_t(s.size()), proto, cs, ctype, max_pkts, &rc, false);
    if (grp) {
      j->grp = grp;
      grp->refs = 1;
    }
    return HDFS_CRC32C_OK;  // (a failed launch: the blocks are verified in the wait)
  }
  const JobQueue::Key key{proto, ctype, cs, lens[0], max_pkts};
  if (!q.pending.empty() && !(q.key == key)) queue_flush(c, q);
  q.key = key;
  j->queued = true;
  q.pending.push_back(j);
  if (q.pending.size() >= kSpecRunsMax || g_job_coalesce == 0 || (g_job_coalesce != 2 && !any_running(c, q)))
    queue_flush(c, q);
  return HDFS_CRC32C_OK;
}

// Block b of a job: its records at pkts + b * max_pkts.  rcs[b] = what
// hdfs_crc32c_verify_packets returns for it; the call returns the first
// negative status, else the first nonzero rcs[b] in block order, else 0.
int job_wait(hdfs_crc32c_job *j, hdfs_crc32c_packet *pkts, size_t max_pkts, size_t *npkts, uint64_t *consumed,
             int *rcs) {
  DevCtx *cp = nullptr;
  int rc;
  if ((rc = ctx_init(j->dev, &cp))) return rc;
  DevCtx &c = *cp;
  DeviceGuard g(c.dev);
  std::lock_guard<std::mutex> lk(c.mu);
  JobQueue &q = jobq(c);
  struct Release {  // the job (and its launch's results, after its last job) on every return path
    JobQueue &q;
    hdfs_crc32c_job *j;
    ~Release() {
      q.outstanding--;
      // (a launch still running when its last job returns early is deleted
      // once collected: group_launch)
      if (j->grp && --j->grp->refs == 0 && j->grp->collected) delete j->grp;
      delete j;
    }
  } rel{q, j};
  if (j->queued) queue_flush(c, q);  // this job's run goes out now, with every queued one
  JobGroup *grp = j->grp;
  const size_t n = j->runs.size();
  const size_t cap = std::min(max_pkts, j->max_pkts);
  std::vector<SpecRunResult> res(n);
  bool early_done = false;
  if (grp && !grp->collected) {
    // the queue goes out behind the running launch (diagnostic mode 3: only
    // two runs or more; a single one waits for the next submit or wait)
    auto flush = [&] {
      if (!q.pending.empty() && (g_job_coalesce != 3 || q.pending.size() >= 2) && !grp->collected && !group_done(c, *grp))
        queue_flush(c, q);
    };
    if (g_job_early && j->grp_run + 1 < grp->m && !j->batch && j->sel.size() == 1) {
      // Per-run completion: the job of a run before the launch's last
      // returns once its own run is published, while the launch verifies
      // the runs after it.  The queue goes out when the wait is on the
      // launch's last run (the caller submits the jobs the earlier returns
      // make room for meanwhile: they go out together), which also collects
      // the launch, or on a run that will not be published.
      const uint32_t i = j->grp_run;
      hdfs_crc32c_packet *dst = pkts + j->sel[0] * max_pkts;
      const auto t0 = std::chrono::steady_clock::now();
      for (uint32_t spin = 0; !grp->collected && !group_done(c, *grp); spin++) {
        const int e = spec_run_early(c.job_slot[grp->slot], grp->L, i, cap, dst, res[j->sel[0]]);
        if (e > 0) {
          early_done = true;
          break;
        }
        if (e < 0) break;
        if ((spin & 255u) == 255u && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) break;
#if defined(__x86_64__) || defined(__i386__)
        __builtin_ia32_pause();
#endif
      }
      g_job_early_stats[early_done ? 0 : 1]++;
    }
    if (!early_done) {
      flush();
      if (!grp->collected) group_collect(c, q, grp);
    }
  }
  if (grp && grp->rc && !early_done) return grp->rc;
  bool allow_spec = true;
  if (grp && !early_done) {
    // the launch's records (count + 1 per run), into the caller's array at
    // the run's block
    for (size_t r = 0; r < j->sel.size(); r++) {
      const size_t b = j->sel[r];
      const SpecRunResult &rr = grp->rr[j->grp_run + r];
      res[b] = rr;
      if (!rr.taken) continue;
      if (rr.recorded > cap) return fail(HDFS_CRC32C_EINVAL, "wait: %u records, room for %zu", rr.recorded, cap);
      std::memcpy(pkts + b * max_pkts, grp->recs.get() + (j->grp_run + r) * grp->per,
                  size_t(rr.recorded) * sizeof(hdfs_crc32c_packet));
    }
    if (grp->single_not_taken && n == 1) allow_spec = false;  // this stream has no run the launch takes: frame it
  }
  int first = HDFS_CRC32C_OK;
  for (size_t r = 0; r < n; r++) {
    hdfs_crc32c_packet *out = pkts + r * max_pkts;
    size_t k = res[r].taken ? res[r].recorded : 0;
    uint64_t used = res[r].taken ? res[r].consumed : 0, from = res[r].taken ? res[r].next : 0;
    const bool done = res[r].taken && (res[r].end || k >= cap);
    if (!done && from < j->lens[r]) {
      // the rest (or all) of the block, synchronously on the engine stream
      size_t n2 = 0;
      uint64_t used2 = 0;
      rc = grid_walk(c, j->runs[r] + from, j->lens[r] - from, j->proto, j->cs, j->ctype, cap - k, true, CopyOut{},
                     out + k, &n2, &used2, nullptr, allow_spec);
      if (kDiag) {
        const int r2 = device_checks("verify job");
        if (r2) return r2;
      }
      if (rc) return rc;
      for (size_t q2 = 0; q2 < n2; q2++) out[k + q2].stream_off += from;
      k += n2;
      if (n2 || used2) used = from + used2;
    }
    npkts[r] = k;
    consumed[r] = used;
    rcs[r] = first_error(out, k);
    if (!first) first = rcs[r];
  }
  return first;
}

// ---- client reads into host memory (hdfs_crc32c_read_packets, host iovecs) ----
// The read path of a datanode whose user buffers are host memory: the
// reference verifies a packet and then memcpy()s its payload into the
// caller's iovecs (src/datanode.c:2470-2476, 2509-2537).
struct CopyJob {
  const uint8_t *src;
  uint8_t *dst;
  uint64_t len;
};
// Lay `pieces` (offsets into src) end to end over the iovecs, in order.
void scatter_jobs(const uint8_t *src, const Pieces &pieces, const hdfs_crc32c_iovec *iov, int iovcnt,
                  std::vector<CopyJob> &jobs) {
  jobs.clear();
  int i = 0;
  uint64_t io = 0;
  for (const auto &pc : pieces) {
    uint64_t off = pc.first, left = pc.second;
    while (left) {
      while (i < iovcnt && io == iov[i].len) {
        i++;
        io = 0;
      }
      if (i == iovcnt) return;  // (the pieces never exceed the iovecs' capacity)
      const uint64_t take = std::min(left, iov[i].len - io);
      jobs.push_back({src + off, static_cast<uint8_t *>(iov[i].base) + io, take});
      off += take;
      left -= take;
      io += take;
    }
  }
}
// Host-to-host copies (the reference's memcpy), split over a few threads for
// large reads.
void run_host_jobs(const std::vector<CopyJob> &jobs) {
  uint64_t total = 0;
  for (const auto &j : jobs) total += j.len;
  const unsigned nt = total >= (64ull << 20) ? std::min(8u, std::max(1u, std::thread::hardware_concurrency())) : 1u;
  auto work = [&](unsigned t) {
    const uint64_t a = total * t / nt, b = total * (t + 1) / nt;
    uint64_t pos = 0;
    for (const auto &j : jobs) {
      const uint64_t s0 = std::max(a, pos), e0 = std::min(b, pos + j.len);
      if (s0 < e0) std::memcpy(j.dst + (s0 - pos), j.src + (s0 - pos), e0 - s0);
      pos += j.len;
      if (pos >= b) break;
    }
  };
  std::vector<std::thread> th;
  for (unsigned t = 1; t < nt; t++) th.emplace_back(work, t);
  work(0);
  for (auto &x : th) x.join();
}

// The device staging area of reads into host memory, at least cap bytes
// (caller holds c.rd_mu).
int rd_stage_reserve(DevCtx &c, uint64_t cap) {
  if (cap <= c.rd_stage_cap) return HDFS_CRC32C_OK;
  if (c.rd_stage) HIPCHK(hipFree(c.rd_stage));
  c.rd_stage = nullptr;
  c.rd_stage_cap = 0;
  const uint64_t want = align_up(cap, uint64_t(1) << 20);
  if (hipMalloc(&c.rd_stage, want) != hipSuccess) {
    (void)hipGetLastError();
    return fail(HDFS_CRC32C_ENOMEM, "read staging of %llu bytes", (unsigned long long)want);
  }
  c.rd_stage_cap = want;
  return HDFS_CRC32C_OK;
}

// Device-resident stream, host destination: the fused verify + copy-out into
// a device staging area (one pass, the whole capacity), then D2H per iovec.
int read_dev_to_host(int dev, const uint8_t *s, uint64_t len, int proto, uint32_t cs, int ctype, int64_t client_offset,
                     int64_t read_len, const hdfs_crc32c_iovec *iov, int iovcnt, uint64_t total,
                     hdfs_crc32c_packet *pkts, size_t max_pkts, size_t *npkts, uint64_t *consumed,
                     uint64_t *delivered) {
  DevCtx *cp = nullptr;
  int rc;
  if ((rc = ctx_init(dev, &cp))) return rc;
  DevCtx &c = *cp;
  DeviceGuard g(c.dev);
  std::lock_guard<std::mutex> lk(c.rd_mu);
  const bool win = read_len != HDFS_CRC32C_READ_ALL;
  // the delivered payload never exceeds the stream's own bytes: a host buffer
  // larger than the stream does not size (and pin) a larger staging area
  const uint64_t cap = std::min<uint64_t>(win ? std::min<uint64_t>(total, uint64_t(read_len)) : total, len);
  if ((rc = rd_stage_reserve(c, cap))) return rc;
  CopyOut co;
  co.dst = c.rd_stage;
  co.cap = cap;
  if (win) {
    co.win = true;
    co.client_offset = client_offset;
    co.want = uint64_t(read_len);
  }
  size_t n = 0;
  uint64_t used = 0, got = 0;
  rc = verify_packets_dev_impl(dev, s, len, proto, cs, ctype, pkts, max_pkts, &n, &used, true, co, &got);
  if (rc < 0) return rc;
  std::vector<CopyJob> jobs;
  scatter_jobs(c.rd_stage, Pieces{{0, got}}, iov, iovcnt, jobs);
  {
    std::lock_guard<std::mutex> lk2(c.mu);
    for (const auto &j : jobs) HIPCHK(hipMemcpyAsync(j.dst, j.src, j.len, hipMemcpyDeviceToHost, c.stream));
    HIPCHK(hipStreamSynchronize(c.stream));
  }
  *npkts = n;
  *consumed = used;
  *delivered = got;
  return rc;
}

// A client read of a host-resident stream, planned: the window is a function
// of the headers (which packets the read takes), so the stream is framed on
// the host, only the packets the window walk looked at are verified on the
// GPU (hdfs_crc32c_verify_packets' host pipeline), and the window applied
// to their verdicts -> records, delivered byte ranges, consumed, delivered,
// again.  Returns a negative status or 0.
int host_window_plan(const uint8_t *s, uint64_t len, int proto, uint32_t cs, int ctype, const CopyOut &co,
                     size_t max_pkts, std::vector<hdfs_crc32c_packet> &recs, Pieces &pieces, uint64_t *used,
                     uint64_t *got, int *again) {
  int rc;
  *used = 0;
  if ((rc = parse_packet_stream(s, len, proto, cs, ctype, max_pkts, recs, used, g_err, sizeof(g_err)))) return rc;
  size_t nh = recs.size(), seen = 0;
  uint64_t ch = *used;
  (void)apply_read_window(recs.data(), nh, ch, co, nullptr, nullptr, &seen);
  // verified: up to the start of the first packet the walk did not look at
  const uint64_t vlen = seen < recs.size() ? recs[seen].stream_off : len;
  recs.assign(seen, hdfs_crc32c_packet{});
  size_t nv = 0;
  rc = verify_packets_impl(s, vlen, proto, cs, ctype, recs.data(), recs.size(), &nv, used, true);
  if (rc < 0) return rc;
  recs.resize(nv);
  *again = apply_read_window(recs.data(), nv, *used, co, got, &pieces);
  recs.resize(nv);
  return HDFS_CRC32C_OK;
}

// Host-resident stream, host destination: framed on the host, the packets
// the read takes verified on the GPU (hdfs_crc32c_verify_packets' host
// pipeline), then their delivered bytes copied.
int read_host_to_host(const uint8_t *s, uint64_t len, int proto, uint32_t cs, int ctype, int64_t client_offset,
                      int64_t read_len, const hdfs_crc32c_iovec *iov, int iovcnt, uint64_t total,
                      hdfs_crc32c_packet *pkts, size_t max_pkts, size_t *npkts, uint64_t *consumed,
                      uint64_t *delivered) {
  const bool win = read_len != HDFS_CRC32C_READ_ALL;
  std::vector<hdfs_crc32c_packet> recs;
  uint64_t used = 0;
  int rc;
  Pieces pieces;
  uint64_t got = 0;
  int again = 0;
  size_t n = 0;
  if (win) {
    CopyOut co;
    co.win = true;
    co.client_offset = client_offset;
    co.want = uint64_t(read_len);
    co.cap = std::min<uint64_t>(total, uint64_t(read_len));
    if ((rc = host_window_plan(s, len, proto, cs, ctype, co, max_pkts, recs, pieces, &used, &got, &again)) < 0)
      return rc;
    n = recs.size();
  } else {
    // straight into the caller's records (max_pkts of them)
    size_t nv = 0;
    rc = verify_packets_impl(s, len, proto, cs, ctype, pkts, max_pkts, &nv, &used, true);
    if (rc < 0) return rc;
    n = nv;
    recs.assign(pkts, pkts + n);
    // every framing-clean packet's payload must fit (as on the device path);
    // the packets before the first error are delivered
    uint64_t payload = 0;
    bool err = false;
    for (size_t k = 0; k < n; k++) {
      const hdfs_crc32c_packet &r = recs[k];
      const bool clean = !r.error || r.error == HDFS_CRC32C_ERR_DATANODE_BAD_CHECKSUM;
      if (clean && r.data_len > 0) payload += uint64_t(r.data_len);
      if (r.error) err = true;
      if (!err && r.data_len > 0) {
        pieces.push_back({wire_begin(r) + uint64_t(r.crc_len), uint64_t(r.data_len)});
        got += uint64_t(r.data_len);
      }
    }
    if (payload > total)
      return fail(HDFS_CRC32C_EINVAL, "copy-out buffer of %llu bytes is too small (%llu needed)",
                  (unsigned long long)total, (unsigned long long)payload);
  }
  std::vector<CopyJob> jobs;
  scatter_jobs(s, pieces, iov, iovcnt, jobs);
  run_host_jobs(jobs);
  if (n) std::memcpy(pkts, recs.data(), n * sizeof(hdfs_crc32c_packet));
  *npkts = n;
  *consumed = used;
  *delivered = got;
  rc = first_error(recs.data(), n);
  return rc ? rc : again ? HDFS_CRC32C_AGAIN : HDFS_CRC32C_OK;
}

// ---- device-to-device delivery of verified bytes (copy_pieces_kernel) ----
int copyctl_init(CopyCtl &k) {
  if (k.hdone) return HDFS_CRC32C_OK;
  if (hipHostMalloc(&k.hdone, sizeof(uint32_t), hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
    (void)hipGetLastError();
    k.hdone = nullptr;
    return fail(HDFS_CRC32C_ENOMEM, "copy completion word");
  }
  *k.hdone = 0;
  HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void **>(&k.ddone), k.hdone, 0));
  if (hipMalloc(&k.count, sizeof(uint32_t)) != hipSuccess) {
    (void)hipGetLastError();
    k.count = nullptr;
    (void)hipHostFree(k.hdone);
    k.hdone = nullptr;
    return fail(HDFS_CRC32C_ENOMEM, "copy counter");
  }
  HIPCHK(hipMemset(k.count, 0, sizeof(uint32_t)));
  return HDFS_CRC32C_OK;
}

// A reader's copy state from the device's pool (caller holds c.mu), and back.
CopyCtl copyctl_take(DevCtx &c) {
  if (c.cp_pool.empty()) return CopyCtl{};
  CopyCtl k = c.cp_pool.back();
  c.cp_pool.pop_back();
  return k;
}

void copyctl_give(int dev, CopyCtl &k) {
  DevCtx *cp = nullptr;
  if (!k.hdone || ctx_init(dev, &cp)) return;
  std::lock_guard<std::mutex> lk(cp->mu);
  cp->cp_pool.push_back(k);
  k = CopyCtl{};
}

void copyctl_free(CopyCtl &k) {
  if (k.hdone) (void)hipHostFree(k.hdone);
  if (k.count) (void)hipFree(k.count);
  if (k.htab) (void)hipHostFree(k.htab);
  if (k.vtab) (void)hipFree(k.vtab);
  k = CopyCtl{};
}

// The device table of a table launch: entries n jobs (< 2^31 units in all),
// each workgroup's first entry, written in pinned memory and (g_copy_dev_tab)
// copied to device memory on st; fills a's table fields.
int copy_table(CopyCtl &k, hipStream_t st, const CopyJob *jobs, uint32_t n, uint64_t units, uint32_t grid,
               CopyPieces &a) {
  const uint32_t per = uint32_t((units + grid - 1u) / grid);
  const size_t wg_off = align_up(size_t(n) * sizeof(CopyEntry), size_t(256));
  const size_t need = wg_off + size_t(grid) * sizeof(uint32_t);
  if (need > k.tab_cap) {
    if (k.htab) HIPCHK(hipHostFree(k.htab));
    k.htab = k.dtab = nullptr;
    k.tab_cap = 0;
    const size_t want = align_up(need, size_t(1) << 16);
    if (hipHostMalloc(&k.htab, want, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
      (void)hipGetLastError();
      k.htab = nullptr;
      return fail(HDFS_CRC32C_ENOMEM, "copy table of %zu bytes", want);
    }
    HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void **>(&k.dtab), k.htab, 0));
    k.tab_cap = want;
  }
  auto *ent = reinterpret_cast<CopyEntry *>(k.htab);
  auto *wg0 = reinterpret_cast<uint32_t *>(k.htab + wg_off);
  uint32_t cum = 0, b = 0;
  for (uint32_t i = 0; i < n; i++) {
    const CopyJob &x = jobs[i];
    cum += copy_units(reinterpret_cast<uintptr_t>(x.dst), x.len);
    ent[i] = CopyEntry{x.src, x.dst, uint32_t(x.len), cum};
    // workgroups whose first unit lies in entry i
    for (; b < grid && uint64_t(b) * per < cum; b++) wg0[b] = i;
  }
  for (; b < grid; b++) wg0[b] = n - 1u;  // (past the end: no units)
  a.n = n;
  const uint8_t *tab = k.dtab;
  if (g_copy_dev_tab) {
    if (need > k.vtab_cap) {
      if (k.vtab) HIPCHK(hipFree(k.vtab));
      k.vtab = nullptr;
      k.vtab_cap = 0;
      if (hipMalloc(&k.vtab, k.tab_cap) != hipSuccess) {
        (void)hipGetLastError();
        k.vtab = nullptr;
        return fail(HDFS_CRC32C_ENOMEM, "copy table");
      }
      k.vtab_cap = k.tab_cap;
    }
    HIPCHK(hipMemcpyAsync(k.vtab, k.htab, need, hipMemcpyHostToDevice, st));
    tab = k.vtab;
  }
  a.tab = reinterpret_cast<const CopyEntry *>(tab);
  a.wg0 = reinterpret_cast<const uint32_t *>(tab + wg_off);
  a.per = per;
  a.total = uint32_t(units);
  return HDFS_CRC32C_OK;
}

// The jobs (device source -> device destination) in launches of
// copy_pieces_kernel on st, each waited for on the completion word: up to
// kCopyPiecesMax pieces in the kernel arguments, more through the pinned
// table (one launch for up to 2^31 units, 32 GiB).  Caller holds the lock
// that serialises st and k.
int copy_jobs_dev(CopyCtl &k, hipStream_t st, const std::vector<CopyJob> &jobs_in, DevCtx *mb = nullptr) {
  int rc;
  if (mb && mb->mb_on && !jobs_in.empty() && jobs_in.size() <= kCopyPiecesMax) {
    // a small delivery with the latency mode open: the resident kernel copies
    uint64_t bytes = 0;
    for (const auto &j : jobs_in) bytes += j.len;
    if (bytes <= g_mb_copy_max) {
      CopyEntry e[kCopyPiecesMax];
      uint32_t units = 0, n = 0;
      for (const auto &j : jobs_in) {
        units += copy_units(reinterpret_cast<uintptr_t>(j.dst), j.len);
        e[n++] = CopyEntry{j.src, j.dst, uint32_t(j.len), units};
      }
      return mailbox_copy(*mb, e, n);
    }
  }
  if ((rc = copyctl_init(k))) return rc;
  std::vector<CopyJob> jobs;  // pieces of < 1 GiB (32-bit lengths)
  jobs.reserve(jobs_in.size());
  for (const auto &j : jobs_in)
    for (uint64_t o = 0; o < j.len; o += 1ull << 30) jobs.push_back({j.src + o, j.dst + o, std::min<uint64_t>(j.len - o, 1ull << 30)});
  auto next_seq = [&]() {
    if (++k.seq == 0) ++k.seq;
    return k.seq;
  };
  size_t j = 0;
  while (j < jobs.size()) {
    CopyPieces a{};
    a.stamps = kDiag ? g_diag : nullptr;
    a.done = k.ddone;
    a.count = k.count;
    if (jobs.size() - j <= kCopyPiecesMax) {
      uint32_t units = 0;
      for (; j < jobs.size(); j++) {
        a.src[a.n] = jobs[j].src;
        a.dst[a.n] = jobs[j].dst;
        a.len[a.n] = uint32_t(jobs[j].len);
        units += copy_units(reinterpret_cast<uintptr_t>(jobs[j].dst), jobs[j].len);
        a.uend[a.n++] = units;
      }
      a.seq = next_seq();
      // one unit per thread up to kCopyBlocksMax workgroups (2 MiB), strided beyond
      const int grid = int(std::min<uint64_t>(kCopyBlocksMax, std::max<uint64_t>(1, (uint64_t(units) + 255u) / 256u)));
      HIPCHK(launch_copy_pieces(a, grid, st));
    } else {
      // as many jobs as fit 2^31 units
      const auto tb = std::chrono::steady_clock::now();
      size_t j1 = j;
      uint64_t units = 0;
      while (j1 < jobs.size()) {
        const uint32_t u = copy_units(reinterpret_cast<uintptr_t>(jobs[j1].dst), jobs[j1].len);
        if (units + u > (1ull << 31)) break;
        units += u;
        j1++;
      }
      const uint32_t n = uint32_t(j1 - j);
      // workgroups of >= g_copy_wg_units units (1024), at most 1024 of them
      // (about what is resident at once: a workgroup stages its first
      // entries once, then streams; r05 copy_sweep: 1 024 workgroups of 8 192
      // units 53 us for 128 MiB, 4 096 of 2 048 units 67 us)
      const uint64_t wgu = std::max<uint32_t>(256u, g_copy_wg_units);
      const uint32_t grid = uint32_t(std::min<uint64_t>(kCopyTabGrid, std::max<uint64_t>(1, (units + wgu - 1u) / wgu)));
      if ((rc = copy_table(k, st, jobs.data() + j, n, units, grid, a))) return rc;
      a.seq = next_seq();
      const auto tl = std::chrono::steady_clock::now();
      HIPCHK(launch_copy_pieces(a, int(grid), st));
      if (g_dstream_trace) {
        const auto tw = std::chrono::steady_clock::now();
        if ((rc = poll_seq(k.hdone, a.seq, "read delivery", st))) return rc;
        auto us = [](std::chrono::steady_clock::time_point x, std::chrono::steady_clock::time_point y) {
          return std::chrono::duration<double, std::micro>(y - x).count();
        };
        std::fprintf(stderr, "dstream copy table n=%u grid=%u build_us=%.1f launch_us=%.1f wait_us=%.1f\n", n, grid,
                     us(tb, tl), us(tl, tw), us(tw, std::chrono::steady_clock::now()));
      }
      j = j1;
    }
    if ((rc = poll_seq(k.hdone, a.seq, "read delivery", st))) return rc;
  }
  return HDFS_CRC32C_OK;
}

// Runs shorter than this (packets) are not copied beside their verify: the
// copy could only start when a short verify has ended (the host prepares it
// from the early block in 10-30 us), and alone the LDS-staged copy kernel is
// the faster one.
constexpr uint32_t kBesideMinPackets = 1024;

// The jobs launched beside a running verify on the context's copy stream
// (copy_beside_kernel, one workgroup per CU next to the verify's); *seq: the
// completion word's value to wait for.  Returns 1 when the jobs do not fit
// one launch (nothing launched).  Caller holds c.mu.
int copy_launch_beside(DevCtx &c, const std::vector<CopyJob> &jobs_in, uint32_t *seq) {
  int rc;
  if ((rc = copyctl_init(c.cp_beside))) return rc;
  if (!c.cp_stream) HIPCHK(hipStreamCreateWithFlags(&c.cp_stream, hipStreamNonBlocking));
  std::vector<CopyJob> jobs;
  uint64_t units = 0;
  for (const auto &j : jobs_in)
    for (uint64_t o = 0; o < j.len; o += 1ull << 30) {
      jobs.push_back({j.src + o, j.dst + o, std::min<uint64_t>(j.len - o, 1ull << 30)});
      units += copy_units(reinterpret_cast<uintptr_t>(j.dst + o), jobs.back().len);
    }
  if (jobs.empty() || units > (1ull << 31)) return 1;
  // (one workgroup per CU fits beside the verify; the others start as its
  // workgroups retire)
  const uint32_t grid = uint32_t(std::min<uint64_t>(kCopyTabGrid, std::max<uint64_t>(1, (units + 2047u) / 2048u)));
  CopyPieces a{};
  a.done = c.cp_beside.ddone;
  a.count = c.cp_beside.count;
  if ((rc = copy_table(c.cp_beside, c.cp_stream, jobs.data(), uint32_t(jobs.size()), units, grid, a))) return rc;
  if (++c.cp_beside.seq == 0) ++c.cp_beside.seq;
  a.seq = c.cp_beside.seq;
  HIPCHK(launch_copy_beside(a, int(grid), c.cp_stream));
  *seq = a.seq;
  return HDFS_CRC32C_OK;
}

// iov with its first `skip` bytes dropped.
std::vector<hdfs_crc32c_iovec> iov_after(const hdfs_crc32c_iovec *iov, int iovcnt, uint64_t skip) {
  std::vector<hdfs_crc32c_iovec> out;
  for (int i = 0; i < iovcnt; i++) {
    if (skip >= iov[i].len) {
      skip -= iov[i].len;
      continue;
    }
    out.push_back({static_cast<uint8_t *>(iov[i].base) + skip, iov[i].len - skip});
    skip = 0;
  }
  return out;
}

// Device-resident stream, several device iovecs: the read verified ONCE with
// the whole capacity (no copy-out in the pass; its delivered byte ranges
// kept), then all its bytes laid over the iovecs by one copy launch -- the
// same result as one pass per buffer, each resuming where the last stopped.
int read_dev_scatter(int dev, const uint8_t *s, uint64_t len, int proto, uint32_t cs, int ctype, int64_t client_offset,
                     int64_t read_len, const hdfs_crc32c_iovec *iov, int iovcnt, uint64_t total,
                     hdfs_crc32c_packet *pkts, size_t max_pkts, size_t *npkts, uint64_t *consumed,
                     uint64_t *delivered) {
  DevCtx *cp = nullptr;
  int rc;
  if ((rc = ctx_init(dev, &cp))) return rc;
  DevCtx &c = *cp;
  DeviceGuard g(c.dev);
  CopyOut co;  // the window only: no copy in the pass
  co.win = true;
  co.client_offset = client_offset;
  co.want = uint64_t(read_len);
  co.cap = std::min<uint64_t>(total, uint64_t(read_len));
  size_t n = 0;
  uint64_t used = 0, got = 0;
  Pieces pieces;
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  // The copy starts under the verify: when the speculative launch's early
  // block predicts the run's records, their window pieces are copied by
  // copy_beside_kernel while the kernel verifies (bytes past what the read
  // delivers are unspecified, as in the fused copy).  The verdicts then
  // decide what was delivered; pieces the prediction missed (the packets
  // after the run) are copied after, and a run whose headers left the
  // prediction is copied again from the actual pieces.
  Pieces pred;
  uint32_t pred_seq = 0;
  int pred_rc = 0;
  std::unique_lock<std::mutex> beside(c.beside_mu, std::try_to_lock);
  EarlyHook hook{[&](const hdfs_crc32c_packet *recs, uint32_t count) {
    if (count < kBesideMinPackets || pred_seq || !beside.owns_lock()) return;
    std::vector<hdfs_crc32c_packet> tmp(recs, recs + count);
    size_t nn = count;
    uint64_t u = 0, gp = 0;
    (void)apply_read_window(tmp.data(), nn, u, co, &gp, &pred);
    std::vector<CopyJob> pj;
    scatter_jobs(s, pred, iov, iovcnt, pj);
    if (pj.empty()) return;
    const int r = copy_launch_beside(c, pj, &pred_seq);  // (c.mu is held by the verify)
    if (r < 0) pred_rc = r;
    if (r) pred_seq = 0;
  }};
  t_early_hook = &hook;
  rc = verify_packets_dev_impl(dev, s, len, proto, cs, ctype, pkts, max_pkts, &n, &used, true, co, &got, &pieces);
  t_early_hook = nullptr;
  const auto t1 = clk::now();
  // the copy started under the verify is waited for on every path
  if (pred_seq) {
    const int r = poll_seq(c.cp_beside.hdone, pred_seq, "read delivery beside the verify", c.cp_stream);
    if (r) return r;
  }
  if (beside.owns_lock()) beside.unlock();
  if (rc < 0) return rc;
  if (pred_rc < 0) return pred_rc;
  // what the prediction copied: the pieces both agree on, in order
  size_t same = 0;
  uint64_t off = 0;
  if (pred_seq) {
    while (same < pieces.size() && same < pred.size() && pieces[same] == pred[same]) off += pieces[same++].second;
    if (same < pieces.size() && same < pred.size()) same = 0, off = 0;  // left the prediction: copy it all again
  }
  std::vector<CopyJob> jobs;
  if (same < pieces.size()) {
    const Pieces rest(pieces.begin() + long(same), pieces.end());
    const std::vector<hdfs_crc32c_iovec> iv = iov_after(iov, iovcnt, off);
    scatter_jobs(s, rest, iv.data(), int(iv.size()), jobs);
  }
  const auto t2 = clk::now();
  if (!jobs.empty()) {
    std::lock_guard<std::mutex> lk(c.mu);
    int r2 = copy_jobs_dev(c.cp, c.stream, jobs, &c);
    if (r2) return r2;
  }
  if (g_dstream_trace) {  // diagnostic: where a scatter read spends its time (us)
    auto us = [](clk::time_point x, clk::time_point y) { return std::chrono::duration<double, std::micro>(y - x).count(); };
    std::fprintf(stderr,
                 "dstream scatter pieces=%zu predicted=%zu kept=%zu jobs_after=%zu verify_us=%.1f jobs_us=%.1f "
                 "copy_after_us=%.1f\n",
                 pieces.size(), pred.size(), same, jobs.size(), us(t0, t1), us(t1, t2), us(t2, clk::now()));
  }
  *npkts = n;
  *consumed = used;
  *delivered = got;
  return rc;
}

// ---- verified reads delivered piece by piece (hdfs_crc32c_reader_*) ----
}  // namespace
}  // namespace hdfs_crc32c

struct hdfs_crc32c_reader {
  int dev = -1;
  const uint8_t *s = nullptr;
  std::vector<hdfs_crc32c_packet> recs;  // the read's records (the one that ended it last)
  hdfs_crc32c::Pieces pieces;            // its bytes: (stream offset, length) in delivery order
  std::vector<uint64_t> rec_done;        // records[k] is complete once this many bytes are delivered
  int status = 0;                        // what the read returns once delivered (0 or the error)
  uint64_t total = 0, done = 0, consumed = 0;
  size_t piece = 0, rec_next = 0;
  uint64_t piece_off = 0;
  hdfs_crc32c::CopyCtl cc;               // its copy launches
};

namespace hdfs_crc32c {
namespace {

int reader_open(const uint8_t *s, uint64_t len, int proto, uint32_t cs, int ctype, int64_t client_offset,
                int64_t read_len, size_t max_pkts, hdfs_crc32c_reader **out) {
  const int dev = stream_device(s);
  auto *rd = new (std::nothrow) hdfs_crc32c_reader;
  if (!rd) return fail(HDFS_CRC32C_ENOMEM, "reader");
  std::unique_ptr<hdfs_crc32c_reader, void (*)(hdfs_crc32c_reader *)> guard(rd, [](hdfs_crc32c_reader *r) {
    copyctl_give(r->dev, r->cc);
    delete r;
  });
  rd->dev = dev;
  rd->s = s;
  rd->recs.resize(std::max<size_t>(1, max_pkts));
  CopyOut co;  // the window only: no copy now, the bytes go out with each next
  co.win = true;
  co.client_offset = client_offset;
  co.want = co.cap = uint64_t(read_len);
  size_t n = 0;
  uint64_t used = 0, got = 0;
  int rc;
  if (dev >= 0) {
    rc = verify_packets_dev_impl(dev, s, len, proto, cs, ctype, rd->recs.data(), max_pkts, &n, &used, true, co, &got,
                                 &rd->pieces);
    if (rc < 0) return rc;
    rd->recs.resize(n);
  } else {  // a host-resident stream: framed on the host, the read's packets verified on the GPU
    int again = 0;
    if ((rc = host_window_plan(s, len, proto, cs, ctype, co, max_pkts, rd->recs, rd->pieces, &used, &got, &again)) < 0)
      return rc;
    n = rd->recs.size();
    rc = first_error(rd->recs.data(), n);
    if (!rc && again) rc = HDFS_CRC32C_AGAIN;
  }
  rd->status = rc == HDFS_CRC32C_AGAIN ? HDFS_CRC32C_OK : rc;  // (the window is the whole read: no AGAIN)
  rd->total = got;
  rd->consumed = used;
  // a record is complete once every byte before the end of its data is out
  rd->rec_done.resize(n);
  {
    size_t pi = 0;
    uint64_t cum = 0;
    for (size_t k = 0; k < n; k++) {
      const hdfs_crc32c_packet &r = rd->recs[k];
      const uint64_t d0 = wire_begin(r) + uint64_t(r.crc_len > 0 ? r.crc_len : 0);
      const uint64_t d1 = d0 + uint64_t(r.data_len > 0 ? r.data_len : 0);
      while (pi < rd->pieces.size() && rd->pieces[pi].first >= d0 && rd->pieces[pi].first < d1) {
        cum += rd->pieces[pi].second;
        pi++;
      }
      rd->rec_done[k] = k + 1 == n ? got : cum;  // the last record (an error, or the read's end) goes with the end
    }
  }
  if (dev >= 0) {
    DeviceGuard g(dev);
    {
      DevCtx *cp = nullptr;
      if ((rc = ctx_init(dev, &cp))) return rc;
      std::lock_guard<std::mutex> lk(cp->mu);
      rd->cc = copyctl_take(*cp);
    }
    if ((rc = copyctl_init(rd->cc))) return rc;
  }
  *out = guard.release();
  return HDFS_CRC32C_OK;
}

int reader_next(hdfs_crc32c_reader *rd, const hdfs_crc32c_iovec *iov, int iovcnt, hdfs_crc32c_packet *pkts,
                size_t max_pkts, size_t *npkts, uint64_t *consumed, uint64_t *delivered) {
  int rc;
  bool any_host = false, any_dev = false;
  uint64_t cap = 0;
  for (int i = 0; i < iovcnt; i++) {
    if (!iov[i].len) continue;
    if (!iov[i].base) return fail(HDFS_CRC32C_EINVAL, "iovec %d: null base", i);
    const int d = stream_device(iov[i].base);
    if (d < 0) any_host = true;
    else if (d == rd->dev) any_dev = true;
    else if (rd->dev < 0) return fail(HDFS_CRC32C_EINVAL, "iovec %d: a host-resident stream copies out to host memory", i);
    else return fail(HDFS_CRC32C_EINVAL, "iovec %d: memory of device %d, the stream is on %d", i, d, rd->dev);
    cap += iov[i].len;
  }
  if (any_host && any_dev) return fail(HDFS_CRC32C_EINVAL, "iovecs mix host and device memory");
  DevCtx *cp = nullptr;
  if ((rc = ctx_init(rd->dev, &cp))) return rc;  // (a host stream: the default device's, unused)
  DevCtx &c = *cp;
  DeviceGuard g(c.dev);
  const uint64_t want = std::min(cap, rd->total - rd->done);
  // the call's copy jobs: the next `want` bytes of the pieces, laid over the iovecs
  Pieces mine;
  {
    uint64_t left = want;
    size_t pi = rd->piece;
    uint64_t po = rd->piece_off;
    while (left) {
      const uint64_t take = std::min(left, rd->pieces[pi].second - po);
      mine.push_back({rd->pieces[pi].first + po, take});
      left -= take;
      po += take;
      if (po == rd->pieces[pi].second) {
        pi++;
        po = 0;
      }
    }
    rd->piece = pi;
    rd->piece_off = po;
  }
  std::vector<CopyJob> jobs;
  scatter_jobs(rd->s, mine, iov, iovcnt, jobs);
  if (rd->dev < 0) {
    run_host_jobs(jobs);  // host stream to host memory: the reference's memcpy (src/datanode.c:2516)
  } else if (!jobs.empty() && any_host && mine.size() > 2) {
    // many pieces into host memory: gathered contiguous in the device
    // staging area by one copy, then one D2H per iovec (not one per piece)
    std::lock_guard<std::mutex> lk0(c.rd_mu);
    if ((rc = rd_stage_reserve(c, want))) return rc;
    std::lock_guard<std::mutex> lk(c.mu);
    std::vector<CopyJob> gather;
    const hdfs_crc32c_iovec sv{c.rd_stage, want};
    scatter_jobs(rd->s, mine, &sv, 1, gather);
    if ((rc = copy_jobs_dev(rd->cc, c.stream, gather, &c))) return rc;
    scatter_jobs(c.rd_stage, Pieces{{0, want}}, iov, iovcnt, jobs);
    for (const auto &j : jobs) HIPCHK(hipMemcpyAsync(j.dst, j.src, j.len, hipMemcpyDeviceToHost, c.stream));
    HIPCHK(hipStreamSynchronize(c.stream));
  } else if (!jobs.empty()) {
    std::lock_guard<std::mutex> lk(c.mu);
    if (any_host) {
      for (const auto &j : jobs) HIPCHK(hipMemcpyAsync(j.dst, j.src, j.len, hipMemcpyDeviceToHost, c.stream));
      HIPCHK(hipStreamSynchronize(c.stream));
    } else {
      if ((rc = copy_jobs_dev(rd->cc, c.stream, jobs, &c))) return rc;
    }
  }
  rd->done += want;
  // records completed so far, at most max_pkts of them; the rest wait for the
  // next call (which may deliver no bytes); the read's last record (and its
  // status) once all bytes are out
  size_t k = 0;
  while (k < max_pkts && rd->rec_next < rd->recs.size() && rd->rec_done[rd->rec_next] <= rd->done &&
         (rd->done == rd->total || rd->rec_next + 1 < rd->recs.size()))
    pkts[k++] = rd->recs[rd->rec_next++];
  *npkts = k;
  *delivered = want;
  // consumed: the end of the last complete packet so far, the read's own at its end
  if (rd->done == rd->total && rd->rec_next == rd->recs.size()) {
    *consumed = rd->consumed;
    return rd->status;
  }
  uint64_t at = 0;
  for (size_t q = rd->rec_next; q-- > 0;) {
    const hdfs_crc32c_packet &r = rd->recs[q];
    at = wire_begin(r) + uint64_t(r.crc_len > 0 ? r.crc_len : 0) + uint64_t(r.data_len > 0 ? r.data_len : 0);
    break;
  }
  *consumed = at;
  return HDFS_CRC32C_AGAIN;
}

}  // namespace
}  // namespace hdfs_crc32c

using namespace hdfs_crc32c;

// ===========================================================================
// Streaming sessions: a pinned ring of host slots that socket reads land in
// directly; full slots are framed and verified asynchronously while the
// caller keeps receiving into the next slot.
// ===========================================================================
struct hdfs_crc32c_session {
  int dev = -1, proto = 0, ctype = 0;
  uint32_t cs = 0;
  uint64_t slot_bytes = 0;
  std::vector<uint8_t *> hslot;      // pinned wire-byte slots
  std::vector<uint64_t> hfill;
  std::vector<uint8_t *> hmeta;      // pinned tables per host slot
  std::vector<size_t> hmeta_cap;
  std::vector<hipEvent_t> hdone;     // last GPU work reading / writing host slot i
  std::vector<bool> hbusy;
  PieceSlot dslot[2];
  hipStream_t copy = nullptr, comp = nullptr;
  size_t cur = 0;
  uint64_t base_off = 0;             // session stream offset of hslot[cur][0]
  uint64_t nsub = 0;
  int sticky = 0;                    // framing error / oversized packet: no more input
  struct Sub {
    size_t hs;
    bool gpu;
    std::vector<hdfs_crc32c_packet> recs;
    std::vector<size_t> vidx;
    PieceLayout L;
  };
  std::deque<Sub> inflight;
  std::deque<hdfs_crc32c_packet> ready;
};

namespace {

int session_finish_front(hdfs_crc32c_session *s, bool wait, bool *progressed) {
  *progressed = false;
  if (s->inflight.empty()) return HDFS_CRC32C_OK;
  hdfs_crc32c_session::Sub &f = s->inflight.front();
  if (f.gpu) {
    if (wait) {
      HIPCHK(hipEventSynchronize(s->hdone[f.hs]));
    } else {
      const hipError_t q = hipEventQuery(s->hdone[f.hs]);
      if (q == hipErrorNotReady) return HDFS_CRC32C_OK;
      HIPCHK(q);
    }
    finish_piece(f.recs.data(), f.vidx.data(), f.L, s->hmeta[f.hs]);
  }
  s->hbusy[f.hs] = false;
  for (auto &k : f.recs) s->ready.push_back(k);
  s->inflight.pop_front();
  *progressed = true;
  return HDFS_CRC32C_OK;
}

// Host slot i must be free (its submission finished) before reuse.
int session_wait_slot(hdfs_crc32c_session *s, size_t i) {
  while (s->hbusy[i]) {
    bool p = false;
    int rc = session_finish_front(s, true, &p);
    if (rc) return rc;
  }
  return HDFS_CRC32C_OK;
}

int session_submit(hdfs_crc32c_session *s) {
  const size_t hs = s->cur;
  const uint64_t fill = s->hfill[hs];
  if (!fill) return HDFS_CRC32C_OK;
  const uint8_t *base = s->hslot[hs];
  hdfs_crc32c_session::Sub sub;
  sub.hs = hs;
  sub.gpu = false;
  uint64_t off = 0;
  for (;;) {  // one parse per block: an empty last packet ends a block, the next may follow
    std::vector<hdfs_crc32c_packet> part;
    uint64_t used = 0;
    int rc = parse_packet_stream(base + off, fill - off, s->proto, s->cs, s->ctype, SIZE_MAX, part, &used, g_err,
                                 sizeof(g_err));
    if (rc) return rc;
    for (auto &k : part) {
      k.stream_off += off;  // slot-relative here; made absolute below
      sub.recs.push_back(k);
    }
    off += used;
    if (!part.empty() && part.back().error) {
      s->sticky = part.back().error;
      break;
    }
    const bool end_of_block = !part.empty() && part.back().data_len == 0 && part.back().last;
    if (!end_of_block || off >= fill) break;
  }
  if (!s->sticky && off == 0 && fill == s->slot_bytes) {
    s->sticky = HDFS_CRC32C_EINVAL;
    return fail(HDFS_CRC32C_EINVAL, "a packet is larger than the session slot (%llu bytes)",
                (unsigned long long)s->slot_bytes);
  }
  if (s->ctype != HDFS_CRC32C_CSUM_NULL)
    for (size_t i = 0; i < sub.recs.size(); i++)
      if (!sub.recs[i].error && sub.recs[i].crc_len > 0) sub.vidx.push_back(i);
  // the next slot receives the incomplete tail of this one
  const size_t nx = (hs + 1) % s->hslot.size();
  int rc = session_wait_slot(s, nx);
  if (rc) return rc;
  const uint64_t tail = s->sticky ? 0 : fill - off;
  if (tail) std::memcpy(s->hslot[nx], base + off, tail);
  s->hfill[nx] = tail;
  if (!sub.vidx.empty()) {
    DevCtx &c = g_ctx[s->dev];
    layout_piece(sub.recs.data(), sub.vidx.data(), sub.vidx.size(), sub.L);
    if (sub.L.meta > s->hmeta_cap[hs]) {
      if (s->hmeta[hs]) HIPCHK(hipHostFree(s->hmeta[hs]));
      s->hmeta[hs] = nullptr;
      s->hmeta_cap[hs] = 0;
      HIPCHK(hipHostMalloc(&s->hmeta[hs], sub.L.meta, hipHostMallocDefault));
      s->hmeta_cap[hs] = sub.L.meta;
    }
    PieceSlot &d = s->dslot[s->nsub & 1];
    if ((rc = reserve_slot(d, sub.L)) ||
        (rc = build_piece(sub.recs.data(), sub.vidx.data(), sub.L, s->cs, s->ctype, d, s->hmeta[hs])) ||
        (rc = enqueue_piece(c, base, sub.L, d, s->hmeta[hs], s->ctype, s->copy, s->comp)))
      return rc;
    HIPCHK(hipEventRecord(s->hdone[hs], s->comp));
    sub.gpu = true;
    s->nsub++;
  }
  for (auto &k : sub.recs) k.stream_off += s->base_off;
  s->hbusy[hs] = true;
  s->inflight.push_back(std::move(sub));
  s->base_off += off;
  s->cur = nx;
  return HDFS_CRC32C_OK;
}

void session_free(hdfs_crc32c_session *s) {
  if (s->comp) (void)hipStreamSynchronize(s->comp);
  if (s->copy) (void)hipStreamSynchronize(s->copy);
  for (auto &d : s->dslot) release_slot(d);
  for (auto p : s->hslot)
    if (p) {
      pins().remove_owned(p);
      (void)hipHostFree(p);
    }
  for (auto p : s->hmeta)
    if (p) (void)hipHostFree(p);
  for (auto e : s->hdone)
    if (e) (void)hipEventDestroy(e);
  if (s->copy) (void)hipStreamDestroy(s->copy);
  if (s->comp) (void)hipStreamDestroy(s->comp);
  delete s;
}

// ---- write path (_send_packet / _compose_data_packet_header) -------------
constexpr int64_t kPacketSize = 64 * 1024;  // PACKET_SIZE, src/datanode.c:38
constexpr uint32_t kWriteChunk = 512;       // CHUNK_SIZE, src/datanode.c:37

struct OutPlan {
  int64_t offset;
  int64_t seqno;
  uint64_t data_off;
  int32_t dlen;
  bool last;
};

// Packet sizing of one write: src/datanode.c:2590 (min(remains_tot,
// PACKET_SIZE)) and :2592-2609 (an unaligned offset first completes its chunk).
void plan_out_packets(uint64_t len, int64_t off, int64_t seq, bool finish, std::vector<OutPlan> &v) {
  uint64_t pos = 0;
  while (pos < len) {
    int64_t n = int64_t(std::min<uint64_t>(len - pos, uint64_t(kPacketSize)));
    if (off % kWriteChunk) n = std::min<int64_t>(n, kWriteChunk - off % kWriteChunk);
    v.push_back(OutPlan{off, seq, pos, int32_t(n), false});
    off += n;
    pos += uint64_t(n);
    seq++;
  }
  // hdfs_datanode_finish_block: an empty packet, lastPacketInBlock = (remains_pkt == 0)
  if (finish) v.push_back(OutPlan{off, seq, pos, 0, true});
}

inline uint8_t *put_be(uint8_t *p, uint64_t v, int n) {
  for (int i = n - 1; i >= 0; i--) *p++ = uint8_t(v >> (8 * i));
  return p;
}
inline uint8_t *put_le(uint8_t *p, uint64_t v, int n) {
  for (int i = 0; i < n; i++) *p++ = uint8_t(v >> (8 * i));
  return p;
}

// protobuf-c packing of PacketHeaderProto as the reference fills it
// (src/datanode.c:2795-2806): required fields in number order, sfixed64 /
// sfixed32 little-endian, the bool as a one-byte varint, syncBlock unset.
constexpr uint32_t kHdrProtoBytes = 25;
uint8_t *put_header_proto(uint8_t *p, int64_t off, int64_t seq, bool last, int32_t dlen) {
  *p++ = 0x09;  // field 1, wire type 1 (64-bit)
  p = put_le(p, uint64_t(off), 8);
  *p++ = 0x11;  // field 2, wire type 1
  p = put_le(p, uint64_t(seq), 8);
  *p++ = 0x18;  // field 3, wire type 0 (varint)
  *p++ = last ? 1 : 0;
  *p++ = 0x25;  // field 4, wire type 5 (32-bit)
  return put_le(p, uint32_t(dlen), 4);
}

uint32_t out_header_bytes(int proto) { return proto == HDFS_CRC32C_PROTO_V1 ? 25u : 4u + 2u + kHdrProtoBytes; }

}  // namespace

extern "C" {

int hdfs_crc32c_parse_packets(const void *stream, uint64_t len, int proto, uint32_t chunk_size, int ctype,
                              hdfs_crc32c_packet *pkts, size_t max_pkts, size_t *npkts, uint64_t *consumed) {
  return verify_packets_impl(static_cast<const uint8_t *>(stream), len, proto, chunk_size, ctype, pkts, max_pkts,
                             npkts, consumed, false);
}

int hdfs_crc32c_verify_packets(const void *stream, uint64_t len, int proto, uint32_t chunk_size, int ctype,
                               hdfs_crc32c_packet *pkts, size_t max_pkts, size_t *npkts, uint64_t *consumed) {
  return verify_packets_impl(static_cast<const uint8_t *>(stream), len, proto, chunk_size, ctype, pkts, max_pkts,
                             npkts, consumed, true);
}

int hdfs_crc32c_read_packets(const void *stream, uint64_t len, int proto, uint32_t chunk_size, int ctype,
                             int64_t client_offset, int64_t read_len, const hdfs_crc32c_iovec *iov, int iovcnt,
                             hdfs_crc32c_packet *pkts, size_t max_pkts, size_t *npkts, uint64_t *consumed,
                             uint64_t *delivered) {
  if (npkts) *npkts = 0;
  if (consumed) *consumed = 0;
  if (delivered) *delivered = 0;
  if (max_pkts && !pkts) return fail(HDFS_CRC32C_EINVAL, "null packet array");
  int rc = check_framing_args(proto, chunk_size, ctype, g_err, sizeof(g_err));
  if (rc) return rc;
  if (ctype == HDFS_CRC32C_CSUM_NULL)
    return fail(HDFS_CRC32C_EINVAL, "verify + copy-out needs CRC32 or CRC32C (src/datanode.c:2470-2486)");
  if (iovcnt < 1 || !iov) return fail(HDFS_CRC32C_EINVAL, "no destination (iovcnt %d)", iovcnt);
  const bool win = read_len != HDFS_CRC32C_READ_ALL;
  if (win && (read_len <= 0 || client_offset < 0))  // a client read (src/datanode.c:1363-1377: bloff >= 0, len > 0)
    return fail(HDFS_CRC32C_EINVAL, "read window: offset %lld, length %lld", (long long)client_offset,
                (long long)read_len);
  if (!win && iovcnt != 1) return fail(HDFS_CRC32C_EINVAL, "whole payloads (READ_ALL) go to one buffer");
  if (!len) return HDFS_CRC32C_OK;
  if (!stream) return fail(HDFS_CRC32C_EINVAL, "null stream");
  const int dev = stream_device(stream);
  // destinations: all device memory of the stream's device (the fused
  // de-framing copy), or all host memory
  bool any_host = false, any_dev = false;
  uint64_t total = 0;
  int nbuf = 0;
  for (int i = 0; i < iovcnt; i++) {
    if (!iov[i].len) continue;
    if (!iov[i].base) return fail(HDFS_CRC32C_EINVAL, "iovec %d: null base", i);
    const int d = stream_device(iov[i].base);
    if (d < 0) any_host = true;
    else if (d == dev) any_dev = true;
    else return fail(HDFS_CRC32C_EINVAL, "iovec %d: memory of device %d, the stream is on %d", i, d, dev);
    total += iov[i].len;
    nbuf++;
  }
  if (any_host && any_dev) return fail(HDFS_CRC32C_EINVAL, "iovecs mix host and device memory");
  if (!total) return HDFS_CRC32C_OK;
  if (dev < 0 && any_dev) return fail(HDFS_CRC32C_EINVAL, "a host-resident stream copies out to host memory");
  if (dev < 0 || any_host) {
    size_t n = 0;
    uint64_t used = 0, got = 0;
    rc = dev < 0 ? read_host_to_host(static_cast<const uint8_t *>(stream), len, proto, chunk_size, ctype,
                                     client_offset, read_len, iov, iovcnt, total, pkts, max_pkts, &n, &used, &got)
                 : read_dev_to_host(dev, static_cast<const uint8_t *>(stream), len, proto, chunk_size, ctype,
                                    client_offset, read_len, iov, iovcnt, total, pkts, max_pkts, &n, &used, &got);
    if (rc < 0) return rc;
    if (npkts) *npkts = n;
    if (consumed) *consumed = used;
    if (delivered) *delivered = got;
    return rc;
  }
  if (nbuf > 1) {  // (a client read: READ_ALL takes one buffer)
    size_t n = 0;
    uint64_t used = 0, got = 0;
    rc = read_dev_scatter(dev, static_cast<const uint8_t *>(stream), len, proto, chunk_size, ctype, client_offset,
                          read_len, iov, iovcnt, total, pkts, max_pkts, &n, &used, &got);
    if (rc < 0) return rc;
    if (npkts) *npkts = n;
    if (consumed) *consumed = used;
    if (delivered) *delivered = got;
    return rc;
  }
  // One buffer: the fused verify + copy-out.  (Kept general: one pass per
  // buffer, each delivers into its buffer and stops with AGAIN
  // when the buffer is full, and the next resumes where the read stands
  // (the stream from the packet it stopped in, the client offset advanced
  // by what was delivered) -- the reference's re-entry with remains_pkt > 0.
  const auto *s = static_cast<const uint8_t *>(stream);
  uint64_t off = 0, got_all = 0;
  size_t n_all = 0;
  int64_t co_off = client_offset, rl = read_len;
  rc = HDFS_CRC32C_OK;
  for (int i = 0; i < iovcnt; i++) {
    if (!iov[i].len) continue;
    CopyOut co;
    co.dst = static_cast<uint8_t *>(iov[i].base);
    co.cap = iov[i].len;
    if (win) {
      co.win = true;
      co.client_offset = co_off;
      co.want = uint64_t(rl);
      co.cap = std::min<uint64_t>(co.cap, co.want);
    }
    size_t n = 0;
    uint64_t used = 0, got = 0;
    rc = verify_packets_dev_impl(dev, s + off, len - off, proto, chunk_size, ctype, pkts ? pkts + n_all : nullptr,
                                 max_pkts - n_all, &n, &used, true, co, &got);
    if (rc < 0) return rc;
    for (size_t k = 0; k < n; k++) pkts[n_all + k].stream_off += off;
    n_all += n;
    got_all += got;
    off += used;
    if (npkts) *npkts = n_all;
    if (consumed) *consumed = off;
    if (delivered) *delivered = got_all;
    if (rc != HDFS_CRC32C_AGAIN) return rc;  // the read completed or ended with an error
    co_off += int64_t(got);
    rl -= int64_t(got);
    if (n_all >= max_pkts && i + 1 < iovcnt) return rc;  // no room for more records: the caller resumes
  }
  return rc;
}

int hdfs_crc32c_reader_open(const void *stream, uint64_t len, int proto, uint32_t chunk_size, int ctype,
                            int64_t client_offset, int64_t read_len, size_t max_pkts, hdfs_crc32c_reader **rd) {
  if (!rd) return fail(HDFS_CRC32C_EINVAL, "null reader");
  *rd = nullptr;
  int rc = check_framing_args(proto, chunk_size, ctype, g_err, sizeof(g_err));
  if (rc) return rc;
  if (ctype == HDFS_CRC32C_CSUM_NULL) return fail(HDFS_CRC32C_EINVAL, "a verified read needs CRC32 or CRC32C");
  if (!stream || !len) return fail(HDFS_CRC32C_EINVAL, "empty stream");
  if (read_len <= 0 || client_offset < 0)
    return fail(HDFS_CRC32C_EINVAL, "read window: offset %lld, length %lld", (long long)client_offset,
                (long long)read_len);
  if (!max_pkts) return fail(HDFS_CRC32C_EINVAL, "no room for records");
  return reader_open(static_cast<const uint8_t *>(stream), len, proto, chunk_size, ctype, client_offset, read_len,
                     max_pkts, rd);
}

int hdfs_crc32c_reader_next(hdfs_crc32c_reader *rd, const hdfs_crc32c_iovec *iov, int iovcnt, hdfs_crc32c_packet *pkts,
                            size_t max_pkts, size_t *npkts, uint64_t *consumed, uint64_t *delivered) {
  if (npkts) *npkts = 0;
  if (delivered) *delivered = 0;
  if (!rd) return fail(HDFS_CRC32C_EINVAL, "null reader");
  if (iovcnt < 0 || (iovcnt && !iov)) return fail(HDFS_CRC32C_EINVAL, "iovecs");
  if (max_pkts && !pkts) return fail(HDFS_CRC32C_EINVAL, "null packet array");
  size_t n = 0;
  uint64_t used = 0, got = 0;
  const int rc = reader_next(rd, iov, iovcnt, pkts, max_pkts, &n, &used, &got);
  if (rc < 0) return rc;
  if (npkts) *npkts = n;
  if (consumed) *consumed = used;
  if (delivered) *delivered = got;
  return rc;
}

void hdfs_crc32c_reader_close(hdfs_crc32c_reader *rd) {
  if (!rd) return;
  copyctl_give(rd->dev, rd->cc);  // (kept for the next reader: no device synchronisation here)
  delete rd;
}

// hdfs_datanode_read_file's copy-out (src/datanode.c:2531-2541): a reader
// verifies the read once, each next delivers the following bytes into a
// host staging buffer, and they are pwrite()n at the fd offset -- retried
// until complete, as _hdfs_pwrite_all does (src/net.c:290-313).
int hdfs_crc32c_read_packets_fd(const void *stream, uint64_t len, int proto, uint32_t chunk_size, int ctype,
                                int64_t client_offset, int64_t read_len, int fd, int64_t fd_offset,
                                hdfs_crc32c_packet *pkts, size_t max_pkts, size_t *npkts, uint64_t *consumed,
                                uint64_t *delivered) {
  if (npkts) *npkts = 0;
  if (consumed) *consumed = 0;
  if (delivered) *delivered = 0;
  if (fd < 0 || fd_offset < 0) return fail(HDFS_CRC32C_EINVAL, "fd %d at offset %lld", fd, (long long)fd_offset);
  if (read_len <= 0 || client_offset < 0)  // a client read (src/datanode.c:870-878: bloff, len)
    return fail(HDFS_CRC32C_EINVAL, "read window: offset %lld, length %lld", (long long)client_offset,
                (long long)read_len);
  if (max_pkts && !pkts) return fail(HDFS_CRC32C_EINVAL, "null packet array");
  if (!len) return HDFS_CRC32C_OK;
  hdfs_crc32c_reader *rd = nullptr;
  int rc = hdfs_crc32c_reader_open(stream, len, proto, chunk_size, ctype, client_offset, read_len, max_pkts, &rd);
  if (rc < 0) return rc;
  constexpr uint64_t kStage = uint64_t(4) << 20;
  std::vector<uint8_t> buf(size_t(std::min<uint64_t>(uint64_t(read_len), kStage)));
  size_t n_all = 0;
  uint64_t got_all = 0, used = 0;
  for (;;) {
    const hdfs_crc32c_iovec iov{buf.data(), buf.size()};
    size_t n = 0;
    uint64_t u = 0, got = 0;
    rc = hdfs_crc32c_reader_next(rd, &iov, 1, pkts ? pkts + n_all : nullptr, max_pkts - n_all, &n, &u, &got);
    if (rc < 0) break;
    n_all += n;
    used = u;
    for (uint64_t w = 0; w < got;) {
      const ssize_t k = pwrite(fd, buf.data() + w, size_t(got - w), off_t(fd_offset + int64_t(got_all + w)));
      if (k < 0 && errno == EINTR) continue;
      if (k <= 0) {
        const int e = k < 0 ? errno : 0;
        got_all += w;
        hdfs_crc32c_reader_close(rd);
        if (npkts) *npkts = n_all;
        if (consumed) *consumed = used;
        if (delivered) *delivered = got_all;
        return fail(HDFS_CRC32C_EIO, "pwrite to fd %d at %lld: %s", fd, (long long)(fd_offset + int64_t(got_all)),
                    e ? std::strerror(e) : "wrote nothing (end of file)");
      }
      w += uint64_t(k);
    }
    got_all += got;
    if (rc != HDFS_CRC32C_AGAIN) break;
  }
  hdfs_crc32c_reader_close(rd);
  if (rc < 0) return rc;
  if (npkts) *npkts = n_all;
  if (consumed) *consumed = used;
  if (delivered) *delivered = got_all;
  return rc;
}

int hdfs_crc32c_verify_packets_submit(const void *stream, uint64_t len, int proto, uint32_t chunk_size, int ctype,
                                      size_t max_pkts, hdfs_crc32c_job **job) {
  if (!job) return fail(HDFS_CRC32C_EINVAL, "null job");
  *job = nullptr;
  int rc = check_framing_args(proto, chunk_size, ctype, g_err, sizeof(g_err));
  if (rc) return rc;
  if (!stream || !len) return fail(HDFS_CRC32C_EINVAL, "empty stream");
  const uint8_t *s = static_cast<const uint8_t *>(stream);
  return job_submit(&s, &len, 1, false, proto, chunk_size, ctype, max_pkts, job);
}

int hdfs_crc32c_verify_blocks_submit(const void *const *streams, const uint64_t *lens, size_t nblocks, int proto,
                                     uint32_t chunk_size, int ctype, size_t max_pkts, hdfs_crc32c_job **job) {
  if (!job) return fail(HDFS_CRC32C_EINVAL, "null job");
  *job = nullptr;
  int rc = check_framing_args(proto, chunk_size, ctype, g_err, sizeof(g_err));
  if (rc) return rc;
  if (!streams || !lens || nblocks < 1 || nblocks > kSpecRunsMax)
    return fail(HDFS_CRC32C_EINVAL, "blocks: 1 to %u streams (%zu given)", kSpecRunsMax, nblocks);
  for (size_t b = 0; b < nblocks; b++)
    if (!streams[b] || !lens[b]) return fail(HDFS_CRC32C_EINVAL, "block %zu: empty stream", b);
  return job_submit(reinterpret_cast<const uint8_t *const *>(streams), lens, nblocks, true, proto, chunk_size, ctype,
                    max_pkts, job);
}

int hdfs_crc32c_job_wait(hdfs_crc32c_job *job, hdfs_crc32c_packet *pkts, size_t max_pkts, size_t *npkts,
                         uint64_t *consumed) {
  if (npkts) *npkts = 0;
  if (consumed) *consumed = 0;
  if (!job) return fail(HDFS_CRC32C_EINVAL, "null job");
  if (job->batch) return fail(HDFS_CRC32C_EINVAL, "a job of blocks: hdfs_crc32c_job_wait_blocks");
  if (max_pkts && !pkts) return fail(HDFS_CRC32C_EINVAL, "null packet array");
  size_t n = 0;
  uint64_t used = 0;
  int rcb = 0;
  const int rc = job_wait(job, pkts, max_pkts, &n, &used, &rcb);
  if (rc < 0) return rc;
  if (npkts) *npkts = n;
  if (consumed) *consumed = used;
  return rc;
}

int hdfs_crc32c_job_wait_blocks(hdfs_crc32c_job *job, hdfs_crc32c_packet *pkts, size_t max_pkts, size_t *npkts,
                                uint64_t *consumed, int *rcs) {
  if (!job) return fail(HDFS_CRC32C_EINVAL, "null job");
  const size_t n = job->runs.size();
  if (!npkts || !consumed || !rcs || (max_pkts && !pkts))
    return fail(HDFS_CRC32C_EINVAL, "null output arrays (%zu blocks)", n);
  for (size_t b = 0; b < n; b++) {
    npkts[b] = 0;
    consumed[b] = 0;
    rcs[b] = 0;
  }
  return job_wait(job, pkts, max_pkts, npkts, consumed, rcs);
}

#ifdef HDFS_CRC32C_DIAG
int hdfs_crc32c_diag_spec_stats(uint64_t *out4, int reset) {
  if (!out4) return fail(HDFS_CRC32C_EINVAL, "null out4");
  for (int i = 0; i < 4; i++) {
    out4[i] = g_spec_stats[i];
    if (reset) g_spec_stats[i] = 0;
  }
  return HDFS_CRC32C_OK;
}
#endif

int hdfs_crc32c_compose_packets(const void *data, uint64_t len, int64_t offset_in_block, int64_t seqno, int proto,
                                int ctype, int finish, void *hdr_out, uint64_t hdr_cap, hdfs_crc32c_out_packet *pkts,
                                size_t max_pkts, size_t *npkts, uint64_t *hdr_used) {
  if (npkts) *npkts = 0;
  if (hdr_used) *hdr_used = 0;
  if (proto != HDFS_CRC32C_PROTO_V1 && proto != HDFS_CRC32C_PROTO_V2)
    return fail(HDFS_CRC32C_EINVAL, "proto must be 1 or 2");
  if (ctype != HDFS_CRC32C_CSUM_NULL && ctype != HDFS_CRC32C_CSUM_CRC32 && ctype != HDFS_CRC32C_CSUM_CRC32C)
    return fail(HDFS_CRC32C_EINVAL, "bad checksum type %d", ctype);
  if (offset_in_block < 0) return fail(HDFS_CRC32C_EINVAL, "negative block offset");
  if (len && !data) return fail(HDFS_CRC32C_EINVAL, "null data");
  std::vector<OutPlan> plan;
  plan_out_packets(len, offset_in_block, seqno, finish != 0, plan);
  const bool csum = ctype != HDFS_CRC32C_CSUM_NULL;
  const uint32_t hb = out_header_bytes(proto);
  uint64_t need = 0;
  for (const OutPlan &k : plan)
    need += hb + (csum ? 4ull * ((uint64_t(k.dlen) + kWriteChunk - 1) / kWriteChunk) : 0ull);
  if (npkts) *npkts = plan.size();
  if (hdr_used) *hdr_used = need;
  if (!hdr_out || !pkts) return HDFS_CRC32C_OK;  // size query
  if (max_pkts < plan.size() || hdr_cap < need)
    return fail(HDFS_CRC32C_EINVAL, "need %zu packets / %llu header bytes", plan.size(), (unsigned long long)need);
  // Chunk CRCs of the whole write on the GPU: the chunk grid is uniform
  // (512 B from the first chunk-aligned byte) except for the first packet of
  // an unaligned write, which is a single short chunk of its own.
  std::vector<uint32_t> head, body;
  uint64_t n0 = 0;
  if (csum && len) {
    n0 = (offset_in_block % kWriteChunk) ? uint64_t(plan[0].dlen) : 0;
    if (n0) {
      head.resize(1);
      int rc = chunk_crcs_to_host(data, n0, uint32_t(n0), ctype, head.data());
      if (rc) return rc;
    }
    if (len > n0) {
      body.resize((len - n0 + kWriteChunk - 1) / kWriteChunk);
      int rc = chunk_crcs_to_host(static_cast<const uint8_t *>(data) + n0, len - n0, kWriteChunk, ctype,
                                  body.data());
      if (rc) return rc;
    }
  }
  uint8_t *out = static_cast<uint8_t *>(hdr_out);
  uint64_t pos = 0;
  for (size_t i = 0; i < plan.size(); i++) {
    const OutPlan &k = plan[i];
    const uint64_t ncrc = csum ? (uint64_t(k.dlen) + kWriteChunk - 1) / kWriteChunk : 0;
    uint8_t *p = out + pos;
    p = put_be(p, uint64_t(uint32_t(int32_t(k.dlen + 4 * ncrc + 4))), 4);  // plen (src/datanode.c:2792)
    if (proto == HDFS_CRC32C_PROTO_V2) {
      p = put_be(p, kHdrProtoBytes, 2);  // hlen (s16)
      p = put_header_proto(p, k.offset, k.seqno, k.last, k.dlen);
    } else {  // src/datanode.c:2808-2812
      p = put_be(p, uint64_t(k.offset), 8);
      p = put_be(p, uint64_t(k.seqno), 8);
      *p++ = k.last ? 1 : 0;
      p = put_be(p, uint32_t(k.dlen), 4);
    }
    if (ncrc) {  // CRCs are already in wire (BE) byte order
      const uint32_t *src = (n0 && i == 0) ? head.data() : body.data() + (k.data_off - n0) / kWriteChunk;
      std::memcpy(p, src, size_t(ncrc) * 4);
      p += ncrc * 4;
    }
    hdfs_crc32c_out_packet &o = pkts[i];
    std::memset(&o, 0, sizeof(o));
    o.hdr_off = pos;
    o.data_off = k.data_off;
    o.offset_in_block = k.offset;
    o.seqno = k.seqno;
    o.data_len = k.dlen;
    o.hdr_len = uint32_t(p - (out + pos));
    o.crc_len = uint32_t(ncrc * 4);
    o.last = k.last ? 1 : 0;
    pos += o.hdr_len;
  }
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_session_create(hdfs_crc32c_session **out, int proto, uint32_t chunk_size, int ctype,
                               uint64_t slot_bytes, size_t nslots) {
  if (!out) return fail(HDFS_CRC32C_EINVAL, "null session pointer");
  *out = nullptr;
  if (proto != HDFS_CRC32C_PROTO_V1 && proto != HDFS_CRC32C_PROTO_V2)
    return fail(HDFS_CRC32C_EINVAL, "bad packet protocol %d", proto);
  if (ctype != HDFS_CRC32C_CSUM_NULL && ctype != HDFS_CRC32C_CSUM_CRC32 && ctype != HDFS_CRC32C_CSUM_CRC32C)
    return fail(HDFS_CRC32C_EINVAL, "bad checksum type %d", ctype);
  if (ctype != HDFS_CRC32C_CSUM_NULL && chunk_size == 0) return fail(HDFS_CRC32C_EINVAL, "chunk_size 0");
  if (!slot_bytes) slot_bytes = uint64_t(64) << 20;
  if (slot_bytes < 4096) return fail(HDFS_CRC32C_EINVAL, "slot_bytes < 4096");
  if (!nslots) nslots = 4;
  if (nslots < 2) return fail(HDFS_CRC32C_EINVAL, "need at least 2 slots");
  DevCtx *c = nullptr;
  int rc = ctx_init(-1, &c);
  if (rc) return rc;
  DeviceGuard g(c->dev);
  auto *s = new hdfs_crc32c_session;
  s->dev = c->dev;
  s->proto = proto;
  s->cs = chunk_size;
  s->ctype = ctype;
  s->slot_bytes = slot_bytes;
  s->hslot.assign(nslots, nullptr);
  s->hfill.assign(nslots, 0);
  s->hmeta.assign(nslots, nullptr);
  s->hmeta_cap.assign(nslots, 0);
  s->hdone.assign(nslots, nullptr);
  s->hbusy.assign(nslots, false);
  hipError_t e = hipStreamCreateWithFlags(&s->copy, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&s->comp, hipStreamNonBlocking);
  for (size_t i = 0; i < nslots && e == hipSuccess; i++) {
    e = hipHostMalloc(&s->hslot[i], slot_bytes, hipHostMallocDefault);
    if (e == hipSuccess) pins().add_owned(s->hslot[i], slot_bytes);  // the caller receives into it
    if (e == hipSuccess) e = hipEventCreateWithFlags(&s->hdone[i], hipEventDisableTiming);
  }
  if (e != hipSuccess) {
    session_free(s);
    return fail(HDFS_CRC32C_ENOMEM, "session allocation: %s", hipGetErrorString(e));
  }
  *out = s;
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_session_buffer(hdfs_crc32c_session *s, void **wptr, uint64_t *room) {
  if (!s || !wptr || !room) return fail(HDFS_CRC32C_EINVAL, "null argument");
  if (s->sticky) return fail(HDFS_CRC32C_EINVAL, "session stopped after error %d", s->sticky);
  *wptr = s->hslot[s->cur] + s->hfill[s->cur];
  *room = s->slot_bytes - s->hfill[s->cur];
  return HDFS_CRC32C_OK;
}

int hdfs_crc32c_session_commit(hdfs_crc32c_session *s, uint64_t nbytes) {
  if (!s) return fail(HDFS_CRC32C_EINVAL, "null session");
  if (s->sticky) return fail(HDFS_CRC32C_EINVAL, "session stopped after error %d", s->sticky);
  if (nbytes > s->slot_bytes - s->hfill[s->cur]) return fail(HDFS_CRC32C_EINVAL, "commit past the slot");
  DeviceGuard g(s->dev);
  s->hfill[s->cur] += nbytes;
  return s->hfill[s->cur] == s->slot_bytes ? session_submit(s) : HDFS_CRC32C_OK;
}

int hdfs_crc32c_session_flush(hdfs_crc32c_session *s) {
  if (!s) return fail(HDFS_CRC32C_EINVAL, "null session");
  if (s->sticky) return HDFS_CRC32C_OK;
  DeviceGuard g(s->dev);
  return session_submit(s);
}

int hdfs_crc32c_session_poll(hdfs_crc32c_session *s, hdfs_crc32c_packet *pkts, size_t max_pkts, size_t *npkts,
                             int wait) {
  if (!s || !npkts || (max_pkts && !pkts)) return fail(HDFS_CRC32C_EINVAL, "null argument");
  *npkts = 0;
  DeviceGuard g(s->dev);
  bool p = true;
  while (p && s->ready.size() < max_pkts) {
    int rc = session_finish_front(s, wait != 0, &p);
    if (rc) return rc;
  }
  size_t n = 0;
  while (n < max_pkts && !s->ready.empty()) {
    pkts[n++] = s->ready.front();
    s->ready.pop_front();
  }
  *npkts = n;
  return first_error(pkts, n);
}

int hdfs_crc32c_session_pending(const hdfs_crc32c_session *s, uint64_t *buffered, size_t *inflight) {
  if (!s) return fail(HDFS_CRC32C_EINVAL, "null session");
  if (buffered) *buffered = s->hfill[s->cur];
  if (inflight) *inflight = s->inflight.size() + s->ready.size();
  return HDFS_CRC32C_OK;
}

void hdfs_crc32c_session_destroy(hdfs_crc32c_session *s) {
  if (!s) return;
  DeviceGuard g(s->dev);
  session_free(s);
}

}  // extern "C"
