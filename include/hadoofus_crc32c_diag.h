/*
 * hadoofus_crc32c_diag.h -- DIAGNOSTIC build of the CRC32C engine
 * (libhadoofus_crc32c_diag.so, compiled with -DHDFS_CRC32C_DIAG).
 *
 * The diagnostic library exports everything in hadoofus_crc32c.h plus the
 * tuning and measurement knobs below, which the release library
 * (libhadoofus_crc32c.so) does not contain: alternative tiled-kernel
 * schedules and shapes, per-wave clock stamps, streaming-read probes, and
 * store policies that DROP results (a load-only twin of the verify kernel
 * that does no CRC arithmetic).  Used by tools/ experiments and by
 * bench.py's empirical-ceiling measurement; never by a datanode.
 * Environment overrides (HDFS_CRC32C_TILE_ORDER, _NT, _DEPTH, _STREAMS,
 * _BLOCK, _STORE, _GROUP, _ALIGN, _SMALL_RULE, _SPEC_POOL) are read by this build only.
 */
#ifndef HADOOFUS_CRC32C_DIAG_H
#define HADOOFUS_CRC32C_DIAG_H

#include "hadoofus_crc32c.h"

#ifdef __cplusplus
extern "C" {
#endif
/* Tiled-kernel schedule: 0 static per-wave slices, 1 workgroup-dynamic,
 * 2 workgroup-dynamic over contiguous slices of 92 % of the tiles + a global
 * pool of 16-256-tile units, 3 (default) as 2 but the static 92 % dealt
 * round-robin over the workgroups (the grid sweeps one contiguous window;
 * launches that are small or made of small segments fall back to 2).
 * Waves of a workgroup take tiles from an LDS counter.  Env
 * HDFS_CRC32C_TILE_ORDER. */
int hdfs_crc32c_set_tile_order(int order);
/* Schedule 3: 2^shift consecutive tiles per round-robin group (default 3:
 * 32 KiB of 512-B chunks, two whole 128-B lines of CRCs per group).  Env
 * HDFS_CRC32C_GROUP. */
int hdfs_crc32c_set_group_shift(int shift);
/* Schedule 3: deal the static groups XCD-major (workgroup b takes virtual
 * slot (b % 8) * (G / 8) + b / 8, so each XCD sweeps a contiguous run of
 * groups) instead of by workgroup id.  Env HDFS_CRC32C_XCD. */
int hdfs_crc32c_set_xcd_major(int on);
/* Tuning / diagnostics: nt_loads=1 streams chunk data with nontemporal global loads,
 * 2 (default) with nontemporal buffer loads (schedule 3 default shape; other
 * schedules and shapes use 1), 0 default-policy loads (env HDFS_CRC32C_NT); diag = device u64[3 * waves] receiving per-wave
 * start/end s_memrealtime stamps and rounds processed (NULL = off). */
int hdfs_crc32c_set_tuning(int nt_loads, void *diag);
/* Register round buffers per tile stream of the tiled kernel (2..4; depth-1
 * rounds stay in flight while one is processed).  Env HDFS_CRC32C_DEPTH. */
int hdfs_crc32c_set_depth(int depth);
/* Tiled-kernel shape: independent tile streams per wave (1, 2, 4) and
 * threads per workgroup (512, 768, 1024).  Only the shapes built into
 * launch_tiles run; any other combination fails (EINVAL) at launch.
 * Env HDFS_CRC32C_STREAMS / HDFS_CRC32C_BLOCK. */
int hdfs_crc32c_set_shape(int streams, int block);
/* Compute-mode result store policy: 0 default (the product's sc1 store), 1 nontemporal, 2 diagnostic
 * (stores dropped; output undefined -- timing experiments only), 4
 * diagnostic: verify plans run a load-only twin of the kernel (same loads and
 * store ops, no CRC arithmetic, results undefined) -- the memory ceiling of
 * the kernel's access pattern; 5 / 6 / 7 / 8: compute-mode CRC stores with
 * cache policy sc1 / sc0 sc1 / nt sc1 / sc0; 9: every tile's CRCs written into
 * one 256 KiB window (L2-resident writes); 10: only chunk 0 of each tile
 * stored (4 B per tile) -- timing experiments only, output undefined; 11:
 * default-policy (no cache bits) CRC stores; 12: only the last tile of each
 * 8-tile group stores, one 256-B store over the group's CRC area; 13: only
 * that tile stores its own 32 B -- 12 / 13 timing experiments only, output
 * undefined; 14..25 further store / load-policy experiments
 * (hadoofus_amd/csrc/crc32c_diag_ep.h); 20 the compute gather with its slot
 * protocol skipped and its stores dropped; 26 / 27 / 28 as 20 plus a
 * workgroup barrier every 3 / 6 / 12 rounds (the barriers' own cost).
 * Env HDFS_CRC32C_STORE. */
int hdfs_crc32c_set_store_policy(int policy);
/* Compute plans: 2 (default, the product) schedule 3 with the LDS group
 * gather (a group's CRCs collected across the workgroup's waves, one 256-B
 * store per 8-tile group); 1 schedule 4 on tables of whole 8-tile groups
 * (one wave per group, one 256-B CRC store per group); 0 schedule 3 with a
 * 32-B store per tile; 3 the lazy gather (schedule 3, the gather's slot
 * check and count read off the critical path, the group stored one round
 * after its last tile).
 * Env HDFS_CRC32C_RUNS. */
int hdfs_crc32c_set_runs(int on);
/* Device-resident packet runs (hdfs_crc32c_verify_packets and the copy-out
 * entry): 1 (default, the product) tries the speculative one-launch verify
 * of a run of equal packets first, 0 always frames the run on the device
 * first (the round-3 path) -- for same-process A/Bs.  Env HDFS_CRC32C_SPEC. */
int hdfs_crc32c_set_speculation(int on);
/* Asynchronous jobs (hdfs_crc32c_verify_packets_submit): 1 (default, the
 * product) queues a job submitted while a launch runs and sends the queue
 * out as one batch launch; 0 launches every job at its submit (the round-5
 * path, for same-process A/Bs); 2 queues even on an idle GPU (the queue goes
 * out only when a wait needs it, at 16 runs or on a key change: launch
 * counts a test can predict); 3 as 1, but a wait blocking on a running
 * launch sends the queue out behind it only if it holds two runs or more.
 * Env HDFS_CRC32C_JOB_COALESCE. */
int hdfs_crc32c_set_job_coalesce(int mode);
/* Per-run completion of coalesced batches: 1 (default, the product) a job
 * whose run is done -- verified clean, its headers in the prediction --
 * returns while the batch launch verifies the runs after it; 0 every job
 * waits for its whole launch (for same-process A/Bs).  Env
 * HDFS_CRC32C_JOB_EARLY. */
int hdfs_crc32c_set_job_early(int on);
/* Waits on jobs of coalesced batches (with per-run completion on): out2 =
 * {returned at their run's completion, returned at the launch's end};
 * reset != 0 clears them. */
int hdfs_crc32c_diag_job_early(uint64_t *out2, int reset);
/* Speculative one-launch verifies since the last reset: out4 = {launches,
 * eligible (packet 0 starts a run of equal packets), taken (no header off
 * the prediction), header exceptions}; reset != 0 clears them. */
int hdfs_crc32c_diag_spec_stats(uint64_t *out4, int reset);
/* Stream queries the synchronous calls made so far (a fault check of
 * earlier work on the engine stream, made only while work no call has seen
 * complete -- an asynchronous plan execute -- is queued before them). */
int hdfs_crc32c_diag_stream_queries(uint64_t *out);
/* The hardware (AQL) queues the engine's streams landed on, as probed: out4 =
 * {engine stream, short-rest stream, copy-beside stream, mailbox stream (0
 * until a mailbox was created)}.  The two beside streams never share the
 * engine stream's queue (replaced by a CU-masked stream at init if they did). */
int hdfs_crc32c_diag_stream_queues(uint64_t *out4);
/* The hardware queues of the 4 asynchronous-job slot streams (0: not made
 * yet).  With HDFS_CRC32C_JOB_QUEUES=1 (default) each is none of the engine
 * stream's or another slot's: two job launches run side by side, never
 * back to back on one queue.  Env HDFS_CRC32C_JOB_QUEUES=0: as placed. */
int hdfs_crc32c_diag_job_queues(uint64_t *out4);
/* Device checks: the framing kernels (frame_build, header_window, small_run,
 * grid_finalize) test, in this build, the invariants
 * behind each address they touch (a record slot inside its pass, a packet's bytes inside
 * the stream, a copy-out inside its window and destination) and skip an
 * access whose invariant fails, counting it.  Every device-stream call reads
 * the count at its end and fails with HDFS_CRC32C_EHIP naming the kernel and
 * source line of the first violation.  out3 = {kernel id (1 frame_build framing,
 * 2 frame_build table, 3 header_window, 4 small_run, 5 grid_finalize), line,
 * violations}; reset > 0 clears them; reset < 0 first records one violation
 * of kernel id 0 (a test of the reporting itself). */
int hdfs_crc32c_diag_device_checks(uint32_t *out3, int reset);
/* Empirical streaming-read bandwidth of `bytes` at dptr (GB/s, 1e9 B/s):
 * fully coalesced 16-B-per-lane loads, no compute; the measured roofline. */
int hdfs_crc32c_probe_read(const void *dptr, uint64_t bytes, void *stream, int iters, double *gbps);
/* Probe shape (diagnostics): variant 0..4 = {4 loads, 4 nt, 8, 8 nt, 16 nt}
 * in flight per lane; grid = grid_per_cu x CUs blocks of `block` threads. */
int hdfs_crc32c_set_probe(int variant, int grid_per_cu, int block);


#ifdef __cplusplus
}
#endif
#endif /* HADOOFUS_CRC32C_DIAG_H */
