// npr_capi.hip — the C-ABI (include/npr.h) over the gfx950 kernels in npr_kernels.hip.
//
// Host-side single-object parsers (GlobalHeader::parse, PcapRecord::parse: 24 / 16 bytes) run
// on the CPU by design; every multi-record path runs on the device.  There is no CPU fallback:
// without a HIP device npr_ctx_create fails.
#include <hip/hip_runtime.h>
#include <sched.h>
#include <stdarg.h>
#include <stdio.h>
#include <time.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/npr.h"
#include "npr_internal.hpp"

#define NPR_VERSION_STRING "net-parser-rs_amd 0.1.0 (gfx950)"

struct DevBuf {
  void *p = nullptr;
  size_t cap = 0;
};

struct npr_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  DevBuf slots;            // npr::TileSlot[]
  uint32_t epoch = 0;      // last granule tag used (1..65535)
  uint32_t *abort_word = nullptr;
  npr_summary *summary = nullptr;   // device
  npr_summary *summary_h = nullptr; // pinned host
  uint32_t *stats = nullptr;        // device diagnostic counters (npr_ctx_set_stats)
  int stats_mode = 0;               // 2 = also per-tile phase stamps
  DevBuf stamps;
  uint64_t stamp_tiles = 0;
  DevBuf srec;             // pass-1 record offsets: kMaxRec u16 per tile
  int resident = 1;        // NPR_OPT_RESIDENT
  uint32_t res_waves = 0;  // persistent waves of the resident single pass (0: not queried yet)
  int cus = 0;             // compute units of the device (0: not queried yet)
  bool res_pack = false;   // chained(): its links pack sparse tiles into kept rounds
  int last_pass = 0;       // npr_ctx_last_pass
  DevBuf chain;            // npr_dev_parse_extract_chunked: two alternating intermediate summaries
  // which launch (epoch) wrote which summary, newest last: npr_dev_check checks a summary against
  // the launch that wrote it, a chained launch the epoch of the one that wrote its `prev`
  std::vector<std::pair<const npr_summary *, uint32_t>> sum_log;
  // staging for the host-memory entry points
  DevBuf in, recs, status, flows, flows_v6, flows2, flows2_v6, agg;
  // host flows-only parses: the capture's H2D copy in chunks on copy_stream, each chunk's chained
  // launch as soon as its bytes (and the next chunk's, for records that straddle) have landed
  uint64_t stream_chunk = 0;  // NPR_OPT_STREAM_CHUNK (KiB in the option; 0 = one copy, the default)
  hipStream_t copy_stream = nullptr;
  std::vector<hipEvent_t> copied;       // one per chunk in flight
  // npr_parse_extract_pipelined: D2H of each link's flow rows, the per-link summaries on the host
  hipStream_t d2h_stream = nullptr;
  std::vector<hipEvent_t> linked;
  npr_summary *sum_host = nullptr;
  uint8_t *head_h = nullptr;  // pinned: the first bytes of a large capture (link sizing)
  uint8_t *small_h = nullptr;  // pinned arena of the small-call path (small_call)
  uint64_t small_cap = 0;
  uint64_t sum_host_cap = 0;
  // ... through a bounded device window (NPR_OPT_DEVICE_WINDOW): chunk ring + flow-row ring
  int window = 0;                        // chunks (0 = auto: only when the staged capture would not fit)
  std::vector<hipEvent_t> row_copied;    // D2H of a flow-ring slot done (the slot may be rewritten)
  // the sparse record walk (npr_sparse.hip): NPR_OPT_SPARSE / NPR_OPT_SPARSE_CAP, the lane-range bytes
  // this call's flows-only launches use (0 = the resident pass), its workspace
  int sparse_mode = 0;
  uint32_t sparse_cap = 0;
  uint64_t sparse_span = 0;
  DevBuf sparse;
  // record density of recently probed captures (device pointer, range, byte order -> bytes per
  // record): the choice of pass never changes a result, so a stale entry only costs time.  An entry
  // goes when the host stages new bytes at that address (stage_input), when the caller says the
  // bytes changed (npr_ctx_forget_density), and it is corrected from the parse's own summary when
  // npr_dev_check reads one whose density disagrees (the next call then chooses by the new bytes)
  struct Probe {
    const void *input = nullptr;
    uint64_t start = 0, stop = 0, mean = 0;
    int e = -1;
    const npr_summary *sum = nullptr;  // the summary of the last parse that chose by this entry
  };
  Probe probes[8];
  uint32_t probe_next = 0;
  std::string err;
};

namespace {

// control words: abort word [0, 64), the resident pass's pacing counter [64, 128)
constexpr size_t kCtlCounters = 64, kCtlBytes = kCtlCounters + 64;
constexpr uint32_t kTimeoutTicks = 100u * 1000u * 1000u;  // 1 s of s_memrealtime (100 MHz)

npr_status fail(npr_ctx *c, npr_status st, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (c) c->err = buf;
  return st;
}

#define HIP_CHECK(c, expr)                                                                 \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess)                                                                  \
      return fail((c), NPR_ERR_DEVICE, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_),     \
                  __FILE__, __LINE__);                                                     \
  } while (0)

npr_status ensure(npr_ctx *c, DevBuf &b, size_t bytes, bool zero = false) {
  if (bytes == 0) bytes = 16;
  if (b.cap >= bytes) return NPR_OK;
  if (b.p) {
    HIP_CHECK(c, hipStreamSynchronize(c->stream));
    HIP_CHECK(c, hipFree(b.p));
    b.p = nullptr;
    b.cap = 0;
  }
  size_t want = std::max(bytes, b.cap + b.cap / 2);
  want = (want + 4095) & ~(size_t)4095;
  HIP_CHECK(c, hipMalloc(&b.p, want));
  if (zero) {  // visible to launches on any stream: finish it here (allocation is rare)
    HIP_CHECK(c, hipMemsetAsync(b.p, 0, want, c->stream));
    HIP_CHECK(c, hipStreamSynchronize(c->stream));
  }
  b.cap = want;
  return NPR_OK;
}

// The next granule tag (1..65535) for a launch on stream s; on wrap every slot is cleared once.
static npr_status next_epoch(npr_ctx *c, hipStream_t s) {
  if (++c->epoch > 0xffffu) {
    c->epoch = 1;
    if (c->slots.p) HIP_CHECK(c, hipMemsetAsync(c->slots.p, 0, c->slots.cap, s));
    HIP_CHECK(c, hipMemsetAsync(c->abort_word, 0, kCtlBytes, s));
  }
  return NPR_OK;
}


inline uint32_t rd_u32(const uint8_t *p, bool big) {
  uint32_t v;
  memcpy(&v, p, 4);
  return big ? __builtin_bswap32(v) : v;
}
inline uint16_t rd_u16(const uint8_t *p, bool big) {
  uint16_t v;
  memcpy(&v, p, 2);
  return big ? (uint16_t)__builtin_bswap16(v) : v;
}

// persistent waves of the resident single pass: CUs x resident waves per CU, at most kResMaxWaves
npr_status res_geometry(npr_ctx *c) {
  if (c->res_waves) return NPR_OK;
  int cus = 0;
  HIP_CHECK(c, hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device));
  const int per = npr::resident_waves_per_cu();
  c->res_waves = (uint32_t)std::max(1, std::min<int>((int)npr::kResMaxWaves, cus * per));
  return NPR_OK;
}

uint64_t tiles_for(uint64_t len, uint64_t start, uint64_t *org_out) {
  const uint64_t org = start - start % npr::kTile;
  if (org_out) *org_out = org;
  const uint64_t span = len > org ? len - org : 0;
  const uint64_t nt = (span + npr::kTile - 1) / npr::kTile;
  return nt ? nt : 1;
}

hipStream_t pick(npr_ctx *c, void *stream) { return stream ? (hipStream_t)stream : c->stream; }

// ---- which flows-only pass: the record density of a device capture ----------------------------
constexpr uint64_t kProbeBytes = 256u << 10;        // walked from the known first record
// auto: the sparse walk for ranges from this size on.  The choice costs one pinned copy and a sync
// per capture not seen recently (~20 us): from 256 MiB on that is small against any parse of the
// range (a 16-MiB floor made single launches of 21-MB C2-shaped captures from many buffers 52 us
// instead of 13: scripts/bench_batch_small.py, round 4)
constexpr uint64_t kSparseMinBytes = 256ull << 20;
constexpr uint64_t kSparseMinMean = 384;            // ... of at least this many bytes per record (16 + incl)
constexpr uint64_t kSparseSpanDefault = 16u << 10;  // lane range when the density is unknown
constexpr uint64_t kSparseSpanRecords = 48;         // lane range of a small range: this many mean records (24 -> 48: C3 walk 573 -> 508 us)
constexpr uint64_t kSparseLaneRecords = 64;         // most mean records per lane when the range fills the chip (slots: 96;
                                                    // C3 at 61 per lane: 0.635 ms, 2.47 GB; at 41: 0.637 ms, 2.59 GB)
constexpr uint64_t kSparseCuLanes = 256;            // lanes of one k_sparse_walk workgroup (kSpBlock)
// Records from the exact record start `start` in the capture's first kProbeBytes: *n and their
// bytes per record (header included), 0 when fewer than 16 fit.  One pinned D2H copy and a sync,
// remembered per capture (the choice of pass never changes a result: a stale entry costs time only).
npr_status probe_density(npr_ctx *c, const void *input, uint64_t start, uint64_t stop, npr_endianness e,
                         void *stream, uint64_t &mean, uint64_t &n) {
  for (const auto &pr : c->probes)
    if (pr.input == input && pr.start == start && pr.stop == stop && pr.e == (int)e) {
      mean = pr.mean;
      n = pr.mean ? 16 : 0;
      return NPR_OK;
    }
  const uint64_t nb = std::min<uint64_t>(stop - start, kProbeBytes);
  if (!c->head_h) HIP_CHECK(c, hipHostMalloc((void **)&c->head_h, kProbeBytes, 0));
  hipStream_t s = pick(c, stream);
  HIP_CHECK(c, hipMemcpyAsync(c->head_h, (const uint8_t *)input + start, nb, hipMemcpyDeviceToHost, s));
  HIP_CHECK(c, hipStreamSynchronize(s));
  uint64_t off = 0;
  n = 0;
  while (off + 16 <= nb) {
    const uint32_t incl = rd_u32(c->head_h + off + 8, e == NPR_BIG);
    if (off + 16 + incl > nb) break;
    off += 16 + (uint64_t)incl;
    ++n;
  }
  mean = n >= 16 ? off / n : 0;
  npr_ctx::Probe &pr = c->probes[c->probe_next++ % 8];
  pr.input = input;
  pr.start = start;
  pr.stop = stop;
  pr.e = (int)e;
  pr.mean = mean;
  pr.sum = nullptr;
  return NPR_OK;
}
// The parse whose summary is `sum` chose its pass by the entry for (input, start, stop, e): that
// entry alone is corrected by what the summary reports.  A summary buffer is reused (one Workspace
// alternating between two captures): the other entries that held it let it go, so a check of one
// capture's parse never rewrites another capture's density.
void probe_note(npr_ctx *c, const void *input, uint64_t start, uint64_t stop, npr_endianness e, const npr_summary *sum) {
  for (auto &pr : c->probes) {
    if (pr.input && pr.input == input && pr.start == start && pr.stop == stop && pr.e == (int)e) pr.sum = sum;
    else if (pr.sum == sum) pr.sum = nullptr;
  }
}
// A parse that chose by no entry (a shard, a speculative start, a record-table launch, a caller's
// own range or chain link) writes `sum`: no entry is corrected by it.
void probe_unbind(npr_ctx *c, const npr_summary *sum) {
  for (auto &pr : c->probes)
    if (pr.sum == sum) pr.sum = nullptr;
}
// Forget the density of the capture at `input` (nullptr: of every capture).
void probe_forget(npr_ctx *c, const void *input) {
  for (auto &pr : c->probes)
    if (!input || pr.input == input) pr = npr_ctx::Probe{};
}
// npr_dev_check read summary `h` (written to `sum`): an entry that chose by a density more than 2x
// off the parse's own (records and bytes consumed) takes the parse's.
void probe_correct(npr_ctx *c, const npr_summary *sum, const npr_summary &h) {
  for (auto &pr : c->probes) {
    if (!pr.input || pr.sum != sum || h.n_records < 16 || h.consumed <= pr.start) continue;
    const uint64_t got = (h.consumed - pr.start) / h.n_records;
    if (got > 2 * pr.mean || 2 * got < pr.mean) pr.mean = got;
  }
}
bool sparse_forced(const npr_ctx *c) { return c->sparse_mode == 2 || c->sparse_mode >= 64; }
// Lane-range bytes of the sparse record walk for a flows-only parse of records starting in
// [start, stop), 0 = the resident pass.  known: `start` is an exact record start of a capture that
// `input` holds from byte 0 (not a shard, not a speculative start), so its density can be probed.
npr_status sparse_choice(npr_ctx *c, const void *input, uint64_t start, uint64_t stop, npr_endianness e, bool known,
                         void *stream, uint64_t &span) {
  span = 0;
  const int m = c->sparse_mode;
  if (m == 1) return NPR_OK;
  if (m >= 64) {
    span = (uint64_t)m;
    return NPR_OK;
  }
  if (m == 0 && (!known || stop <= start || stop - start < kSparseMinBytes)) return NPR_OK;
  uint64_t mean = 0, n = 0;
  if (known && stop > start) {
    const npr_status st = probe_density(c, input, start, stop, e, stream, mean, n);
    if (st) return st;
  }
  uint64_t sized = std::min<uint64_t>(std::max<uint64_t>(kSparseSpanRecords * mean, 4u << 10), npr::kSparseSpanMax);
  // A range of more records than one 256-lane workgroup per CU holds at ~24 each: k workgroups per CU
  // exactly (k = the fewest that keep lanes at <= 64 mean records: fewer lanes speculate less).  The walk is bound per CU (its
  // random 16-B loads), so its time follows the most lane-records any CU holds: C3 at 36.9 … 61 KB
  // lanes took 0.636–0.716 ms in step with that maximum (3 workgroups on some CUs and 2 on others:
  // 0.716; 2 or 3 on every CU: 0.636), profiles/r04_c3_span_sweep.json.
  if (mean && stop > start) {
    if (!c->cus) (void)hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, c->device);
    const int cus = c->cus;
    if (cus > 0) {
      const uint64_t range = stop - start, est = range / mean, slots = (uint64_t)cus * kSparseCuLanes;
      if (est >= 24 * slots) {
        const uint64_t k = (est + slots * kSparseLaneRecords - 1) / (slots * kSparseLaneRecords);
        sized = std::min<uint64_t>(std::max<uint64_t>((range + k * slots - 1) / (k * slots), 4u << 10), npr::kSparseSpanMax);
      }
    }
  }
  if (m == 2) span = mean ? sized : kSparseSpanDefault;
  else if (mean >= kSparseMinMean) span = sized;
  return NPR_OK;
}
struct SpanScope {  // this call's flows-only launches run the sparse walk; later calls choose again
  npr_ctx *c;
  ~SpanScope() { c->sparse_span = 0; }
};

// ---- launch order across contexts ------------------------------------------------------------
// The look-back kernels (k_parse_resident, the two-pass folds, k_convert_records) have workgroups
// that wait for lower workgroups of the SAME launch, which is safe only while no other such launch
// interleaves with it on the device: workgroups are dealt round-robin to the XCDs and each XCD
// dispatches its share in order, so two launches in flight can each hold the CUs the other's lower
// workgroups need (two contexts on two streams deadlocked until the bounded waits
// aborted).  So these launches are serialised per device, process-wide: each waits for an event
// recorded behind the previous one (whatever context or stream issued it) and records its own.
// The reference's functions are pure and reentrant (src/errors.rs:13-14: its errors are Send +
// Sync); with this, any number of host threads with their own contexts may call the C-ABI at once.
constexpr int kOrderEvents = 8;   // a ring: a wait captures the event's last record when enqueued
constexpr int kMaxDevices = 64;
struct DeviceOrder {
  std::mutex m;
  hipEvent_t ev[kOrderEvents] = {};
  int cur = -1;                     // the event behind the last ordered launch (-1: none yet)
  hipStream_t last = nullptr;       // the stream of the last ordered launch
  bool pending = false;             // mode 3: that launch has no event yet
};
DeviceOrder &device_order(int dev) {
  static DeviceOrder orders[kMaxDevices];
  return orders[dev & (kMaxDevices - 1)];
}
// How the order is kept (NPR_LAUNCH_ORDER, for A/B timing only; measured on C2, µs per launch):
//   3 (default): a launch records no event; the next launch from ANOTHER stream first records one
//     on the previous launch's stream, then waits for it (30.0, as with no ordering at all);
//   1: every launch waits for the previous launch's event and records its own (33.0: an event
//     record between two launches costs ~2.7 us of GPU time); 2: the wait only across streams
//     (33.0); 0: no ordering (30.0; two contexts' launches may deadlock).
int launch_order_mode() {
  static const int mode = [] {
    const char *e = getenv("NPR_LAUNCH_ORDER");
    return e && e[0] >= '0' && e[0] <= '3' ? e[0] - '0' : 3;
  }();
  return mode;
}
npr_status order_record(npr_ctx *c, DeviceOrder &o, hipStream_t s) {
  const int k = (o.cur + 1) % kOrderEvents;
  if (!o.ev[k]) HIP_CHECK(c, hipEventCreateWithFlags(&o.ev[k], hipEventDisableTiming));
  HIP_CHECK(c, hipEventRecord(o.ev[k], s));
  o.cur = k;
  return NPR_OK;
}
// Run `launch` (enqueues one look-back kernel on s) after every earlier look-back launch on this
// device; the device's order lock is held from the wait to the record.
template <class F>
npr_status ordered_launch(npr_ctx *c, hipStream_t s, F &&launch) {
  const int mode = launch_order_mode();
  if (mode == 0) {
    HIP_CHECK(c, launch());
    return NPR_OK;
  }
  DeviceOrder &o = device_order(c->device);
  std::lock_guard<std::mutex> g(o.m);
  npr_status st;
  if (mode == 3 && o.pending && o.last != s) {  // the previous launch's event, recorded only now
    if ((st = order_record(c, o, o.last))) return st;
    o.pending = false;
  }
  if (o.cur >= 0 && (mode == 1 || o.last != s)) HIP_CHECK(c, hipStreamWaitEvent(s, o.ev[o.cur], 0));
  HIP_CHECK(c, launch());
  o.last = s;
  if (mode == 3) {
    o.pending = true;
  } else if ((st = order_record(c, o, s))) {
    return st;
  }
  return NPR_OK;
}

}  // namespace

extern "C" {

const char *npr_version(void) { return NPR_VERSION_STRING; }
int npr_ctx_last_pass(const npr_ctx *c) { return c ? c->last_pass : 0; }
npr_status npr_ctx_forget_density(npr_ctx *c, const void *input) {
  if (!c) return NPR_ERR_ARG;
  probe_forget(c, input);
  return NPR_OK;
}
int npr_abi_version(void) { return NPR_ABI_VERSION; }

// elements per level: [0] tiles, [l] = ceil([l-1] / 64)
static void level_sizes(uint64_t nt, uint64_t n[npr::kLevels + 1]) {
  n[0] = nt;
  for (int l = 1; l <= npr::kLevels; ++l) n[l] = (n[l - 1] + 63) / 64;
}
// group slots after the tile slots: the two-pass kernels' level-1..3 folds, or the resident pass's
// one aggregate per workgroup (rgroups = groups[1], up to ceil(min(nt, kResMaxWaves) / kResWgMin)
// slots, which can exceed the fold levels' ceil(nt/64) + ceil(nt/4096) + ...)
static uint64_t group_slots(uint64_t nt) {
  uint64_t n[npr::kLevels + 1];
  level_sizes(nt, n);
  uint64_t folds = 0;
  for (int l = 1; l <= npr::kLevels; ++l) folds += n[l];
  const uint64_t res = (std::min<uint64_t>(nt, npr::kResMaxWaves) + npr::kResWgMin - 1) / npr::kResWgMin;
  return std::max(folds, res);
}
// tile slots, then the group slots: one allocation (granules are epoch-tagged, so the layout may
// shift between launches)
static uint64_t slot_bytes(uint64_t nt) { return nt * sizeof(npr::TileSlot) + group_slots(nt) * sizeof(npr::GroupSlot); }

uint64_t npr_workspace_bytes(uint64_t len) {
  const uint64_t nt = tiles_for(len, 0, nullptr);
  return slot_bytes(nt) + nt * npr::kMaxRec * sizeof(uint16_t);  // + pass 1's record-offset scratch
}

npr_status npr_ctx_create(int device, npr_ctx **out) {
  if (!out) return NPR_ERR_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= device || device < 0) return NPR_ERR_DEVICE;
  npr_ctx *c = new npr_ctx();
  c->device = device;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc((void **)&c->abort_word, kCtlBytes) != hipSuccess || hipMalloc((void **)&c->summary, sizeof(npr_summary)) != hipSuccess ||
      hipHostMalloc((void **)&c->summary_h, sizeof(npr_summary), 0) != hipSuccess ||
      hipMemset(c->abort_word, 0, kCtlBytes) != hipSuccess) {
    npr_ctx_destroy(c);
    return NPR_ERR_DEVICE;
  }
  const char *env = getenv("NPR_RESIDENT");
  if (env && env[0] == '0') c->resident = 0;
  *out = c;
  return NPR_OK;
}

// A caller stream is about to be destroyed: if the device's last ordered launch ran on it and its
// order event is still pending (mode 3 records it lazily, from the next launch on another stream),
// record it now, while the stream exists.
npr_status npr_stream_release(npr_ctx *c, void *stream) {
  if (!c) return NPR_ERR_ARG;
  HIP_CHECK(c, hipSetDevice(c->device));
  hipStream_t s = pick(c, stream);
  DeviceOrder &o = device_order(c->device);
  std::lock_guard<std::mutex> g(o.m);
  if (o.pending && o.last == s) {
    if (npr_status st = order_record(c, o, s)) return st;
    o.pending = false;
  }
  return NPR_OK;
}

void npr_ctx_destroy(npr_ctx *c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  {  // the launch order must not record on this context's stream after it is gone (its work is done)
    DeviceOrder &o = device_order(c->device);
    std::lock_guard<std::mutex> g(o.m);
    if (o.last == c->stream) {
      o.last = nullptr;
      o.pending = false;
    }
  }
  for (DevBuf *b : {&c->slots, &c->srec, &c->stamps, &c->chain, &c->in, &c->recs, &c->status, &c->flows, &c->flows_v6, &c->flows2,
                    &c->flows2_v6, &c->agg, &c->sparse})
    if (b->p) (void)hipFree(b->p);
  if (c->abort_word) (void)hipFree(c->abort_word);
  if (c->summary) (void)hipFree(c->summary);
  if (c->summary_h) (void)hipHostFree(c->summary_h);
  if (c->stats) (void)hipFree(c->stats);
  if (c->copy_stream) (void)hipStreamSynchronize(c->copy_stream);
  if (c->d2h_stream) (void)hipStreamSynchronize(c->d2h_stream);
  for (hipEvent_t ev : c->copied) (void)hipEventDestroy(ev);
  for (hipEvent_t ev : c->linked) (void)hipEventDestroy(ev);
  for (hipEvent_t ev : c->row_copied) (void)hipEventDestroy(ev);
  if (c->sum_host) (void)hipHostFree(c->sum_host);
  if (c->head_h) (void)hipHostFree(c->head_h);
  if (c->small_h) (void)hipHostFree(c->small_h);
  if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
  if (c->d2h_stream) (void)hipStreamDestroy(c->d2h_stream);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

const char *npr_ctx_last_error(const npr_ctx *c) { return c ? c->err.c_str() : "null context"; }

npr_status npr_ctx_set_option(npr_ctx *c, int option, int value) {
  if (!c) return NPR_ERR_ARG;
  switch (option) {
    case NPR_OPT_PARK_FLOWS:  // accepted for ABI 2 callers; one decode path since ABI 3
      (void)value;
      return NPR_OK;
    case NPR_OPT_RESIDENT:  // 0 off, 1 auto, N > 1: at most N waves (tests: long ranges, deferral)
      if (value < 0) return fail(c, NPR_ERR_ARG, "NPR_OPT_RESIDENT must be >= 0");
      c->resident = value;
      return NPR_OK;
    case NPR_OPT_PIPE:  // the pipelined pass was an experiment: not in this library
      if (value == 0) return NPR_OK;
      return fail(c, NPR_ERR_ARG, "NPR_OPT_PIPE: the pipelined resident pass is not built into this library");
    case NPR_OPT_DEVICE_WINDOW:  // chunks of the capture on the device at once (0 = auto)
      if (value < 0 || value == 1 || value == 2) return fail(c, NPR_ERR_ARG, "NPR_OPT_DEVICE_WINDOW: 0 (auto) or >= 3 chunks");
      c->window = value;
      return NPR_OK;
    case NPR_OPT_SPARSE:  // 0 auto (record density), 1 never, 2 always, N >= 64: always, lane ranges of N bytes
      if (value < 0 || (value > 2 && value < 64)) return fail(c, NPR_ERR_ARG, "NPR_OPT_SPARSE: 0, 1, 2 or >= 64 bytes");
      c->sparse_mode = value;
      return NPR_OK;
    case NPR_OPT_SPARSE_CAP:  // Ok-flow slots per lane (0 = the default)
      if (value < 0 || value > (int)npr::kSparseCapMax) return fail(c, NPR_ERR_ARG, "NPR_OPT_SPARSE_CAP: 0 .. 128");
      c->sparse_cap = (uint32_t)value;
      return NPR_OK;
    case NPR_OPT_STREAM_CHUNK:  // KiB; 0 = stage the whole capture first
      if (value < 0 || (value > 0 && value < 64)) return fail(c, NPR_ERR_ARG, "NPR_OPT_STREAM_CHUNK: 0 or >= 64 KiB");
      c->stream_chunk = (uint64_t)value << 10;
      return NPR_OK;
    default:
      return fail(c, NPR_ERR_ARG, "unknown option");
  }
}

npr_status npr_ctx_set_stats(npr_ctx *c, int enable) {
  if (!c) return NPR_ERR_ARG;
  HIP_CHECK(c, hipSetDevice(c->device));
  c->stats_mode = enable;
  if (enable && !c->stats) {
    HIP_CHECK(c, hipMalloc((void **)&c->stats, npr::kStatCount * sizeof(uint32_t)));
    HIP_CHECK(c, hipMemset(c->stats, 0, npr::kStatCount * sizeof(uint32_t)));
  } else if (!enable && c->stats) {
    HIP_CHECK(c, hipStreamSynchronize(c->stream));
    HIP_CHECK(c, hipFree(c->stats));
    c->stats = nullptr;
  }
  return NPR_OK;
}

npr_status npr_ctx_read_stamps(npr_ctx *c, uint64_t *out, uint64_t cap, uint64_t *n_tiles) {
  if (!c || (!out && cap)) return NPR_ERR_ARG;
  if (!c->stamps.p) return fail(c, NPR_ERR_ARG, "stamps not enabled (npr_ctx_set_stats(ctx, 2))");
  HIP_CHECK(c, hipSetDevice(c->device));
  HIP_CHECK(c, hipDeviceSynchronize());
  const uint64_t n = std::min<uint64_t>(cap, c->stamp_tiles * npr::kStampWords);
  if (n) HIP_CHECK(c, hipMemcpy(out, c->stamps.p, n * 8, hipMemcpyDeviceToHost));
  if (n_tiles) *n_tiles = c->stamp_tiles;
  return NPR_OK;
}

npr_status npr_ctx_read_stats(npr_ctx *c, uint32_t *out, int n, int reset) {
  if (!c || !out || n <= 0) return NPR_ERR_ARG;
  if (!c->stats) return fail(c, NPR_ERR_ARG, "stats not enabled");
  HIP_CHECK(c, hipSetDevice(c->device));
  HIP_CHECK(c, hipDeviceSynchronize());
  uint32_t tmp[npr::kStatCount];
  HIP_CHECK(c, hipMemcpy(tmp, c->stats, sizeof tmp, hipMemcpyDeviceToHost));
  for (int i = 0; i < n && i < (int)npr::kStatCount; ++i) out[i] = tmp[i];
  if (reset) HIP_CHECK(c, hipMemset(c->stats, 0, sizeof tmp));
  return NPR_OK;
}

// ---- GlobalHeader::parse (src/global_header.rs:40-70) ----------------------------------------
npr_status npr_global_header_parse(const uint8_t *in, size_t len, npr_global_header *out, size_t *consumed) {
  if (!out || (!in && len)) return NPR_ERR_ARG;
  if (len < 24) return NPR_INCOMPLETE;  // every field is a fixed-width nom primitive
  uint32_t magic;
  memcpy(&magic, in, 4);  // u32!(NATIVE_ENDIAN), little-endian host
  const bool big = magic != 0xA1B2C3D4u;  // == MAGIC => native (Little), else Big (:43-53)
  out->endianness = big ? NPR_BIG : NPR_LITTLE;
  out->version_major = rd_u16(in + 4, big);
  out->version_minor = rd_u16(in + 6, big);
  out->zone = (int32_t)rd_u32(in + 8, big);
  out->sig_figs = (int32_t)rd_u32(in + 12, big);
  out->snap_length = rd_u32(in + 16, big);
  out->network = rd_u32(in + 20, big);
  if (consumed) *consumed = 24;
  return NPR_OK;
}

// ---- PcapRecord::parse (src/record.rs:102-121) ------------------------------------------------
npr_status npr_record_parse(const uint8_t *in, size_t len, npr_endianness e, npr_record *out, size_t *consumed) {
  if (!out || (!in && len)) return NPR_ERR_ARG;
  if (len < 16) return NPR_INCOMPLETE;
  const bool big = e == NPR_BIG;
  const uint32_t incl = rd_u32(in + 8, big);
  if (len - 16 < incl) return NPR_INCOMPLETE;  // take!(actual_length)
  out->offset = 0;
  out->ts_sec = rd_u32(in, big);
  out->ts_usec = rd_u32(in + 4, big);
  out->actual_length = incl;
  out->original_length = rd_u32(in + 12, big);
  if (consumed) *consumed = 16 + (size_t)incl;
  return NPR_OK;
}

// ---- device-resident hot path -----------------------------------------------------------------
// A shard's buffer holds file bytes [base, len) only: byte offsets stay file offsets, and the
// speculation context (the magic's ts_usec bound, a reference ts_sec) comes from the host.
struct ShardSpec {
  uint64_t base = 0;
  uint32_t frac_max = 1000000000u;
  bool has_ref = false;
  uint32_t ts_ref = 0;
};

static npr_status launch_range(npr_ctx *c, const void *input, uint64_t len, uint64_t start, uint64_t stop,
                               npr_endianness e, int speculative_start, uint64_t ref_record,
                               const npr_summary *prev, const npr_dev_outputs *o, void *stream,
                               const ShardSpec *sh = nullptr);

npr_status npr_dev_parse_extract(npr_ctx *c, const void *input, uint64_t len, uint64_t start,
                                 npr_endianness e, const npr_dev_outputs *o, void *stream) {
  // flows-only captures larger than one launch keeps in registers: chained chunks of that size
  if (c && o && c->resident && !o->record_offsets && !o->records && !o->record_status && len > start && input &&
      ((uintptr_t)input & 15u) == 0) {
    npr_status st = res_geometry(c);
    if (st) return st;
    uint64_t span = 0;  // long records: the sparse walk, one launch set for any size
    if ((st = sparse_choice(c, input, start, len, e, true, stream, span))) return st;
    probe_note(c, input, start, len, e, o->summary);
    if (span) {
      SpanScope scope{c};
      c->sparse_span = span;
      return launch_range(c, input, len, start, len, e, 0, start, nullptr, o, stream);
    }
    if (len - start > (uint64_t)c->res_waves * npr::kResSlots * npr::kTile)
      return npr_dev_parse_extract_chunked(c, input, len, start, e, o, 0, stream);
    return launch_range(c, input, len, start, len, e, 0, start, nullptr, o, stream);
  }
  return npr_dev_parse_extract_range(c, input, len, start, len, e, 0, start, o, stream);
}

// the epoch of the last launch that wrote summary s (0: none of ours)
static uint32_t summary_epoch(const npr_ctx *c, const npr_summary *s) {
  for (auto it = c->sum_log.rbegin(); it != c->sum_log.rend(); ++it)
    if (it->first == s) return it->second;
  return 0;
}
static void log_summary(npr_ctx *c, const npr_summary *s) {
  if (c->sum_log.size() >= 256) c->sum_log.erase(c->sum_log.begin(), c->sum_log.begin() + 128);
  c->sum_log.emplace_back(s, c->epoch);
}
static npr_status chained(npr_ctx *c, const void *input, uint64_t len, uint64_t start, uint64_t stop,
                          npr_endianness e, int speculative_start, uint64_t ref_record, const npr_dev_outputs *o,
                          uint64_t chunk_bytes, void *stream, const ShardSpec *sh);
static npr_status range_params(npr_ctx *c, const void *input, uint64_t len, uint64_t start, uint64_t stop,
                               npr_endianness e, int speculative_start, uint64_t ref_record, const ShardSpec *sh,
                               npr::ParseParams &p, uint64_t &nt);

npr_status npr_dev_parse_extract_range(npr_ctx *c, const void *input, uint64_t len, uint64_t start,
                                       uint64_t stop, npr_endianness e, int speculative_start,
                                       uint64_t ref_record, const npr_dev_outputs *o, void *stream) {
  if (c && o) probe_unbind(c, o->summary);
  return launch_range(c, input, len, start, stop, e, speculative_start, ref_record, nullptr, o, stream);
}

npr_status npr_dev_parse_extract_chain(npr_ctx *c, const void *input, uint64_t len, uint64_t start,
                                       uint64_t stop, npr_endianness e, const npr_summary *prev,
                                       uint64_t ref_record, const npr_dev_outputs *o, void *stream) {
  if (c && o) probe_unbind(c, o->summary);
  return launch_range(c, input, len, start, stop, e, 0, ref_record, prev, o, stream);
}

npr_status npr_dev_parse_extract_chunked(npr_ctx *c, const void *input, uint64_t len, uint64_t start,
                                         npr_endianness e, const npr_dev_outputs *o, uint64_t chunk_bytes,
                                         void *stream) {
  if (!c || !o || !o->summary || (!input && len)) return fail(c, NPR_ERR_ARG, "null argument");
  if (start > len) return fail(c, NPR_ERR_ARG, "need start <= len");
  return chained(c, input, len, start, len, e, 0, start, o, chunk_bytes, stream, nullptr);
}

// Records starting in [start, stop) as chained resident launches of about chunk_bytes each (the
// first one may speculate its start); launches that need a record table / offsets / status run
// the two-pass kernels in one launch instead.
static npr_status chained(npr_ctx *c, const void *input, uint64_t len, uint64_t start, uint64_t stop,
                          npr_endianness e, int speculative_start, uint64_t ref_record, const npr_dev_outputs *o,
                          uint64_t chunk_bytes, void *stream, const ShardSpec *sh) {
  const bool flows_only = !o->record_offsets && !o->records && !o->record_status;
  probe_unbind(c, o->summary);  // (noted below when this parse chooses by the capture's density)
  if (!c->resident || !flows_only || stop <= start)
    return launch_range(c, input, len, start, stop, e, speculative_start, ref_record, nullptr, o, stream, sh);
  npr_status st = res_geometry(c);
  if (st) return st;
  uint64_t span = 0;  // long records: sparse links (chunk_bytes 0: one sparse launch set for the range)
  if ((st = sparse_choice(c, input, start, stop, e, !speculative_start && !sh, stream, span))) return st;
  if (!speculative_start && !sh) probe_note(c, input, start, stop, e, o->summary);
  SpanScope span_scope{c};
  if (span) {
    c->sparse_span = span;
    if (!chunk_bytes) return launch_range(c, input, len, start, stop, e, speculative_start, ref_record, nullptr, o, stream, sh);
  }
  uint64_t chunk = chunk_bytes;
  // the waves one link runs (NPR_OPT_RESIDENT N > 1 caps them, as launch_range does)
  const uint64_t waves = c->resident > 1 ? std::min<uint64_t>(c->res_waves, (uint64_t)c->resident) : c->res_waves;
  bool pack = chunk_bytes > waves * npr::kResSlots * npr::kTile;
  if (!chunk) {  // one launch keeps kResSlots rounds of 64 records per wave in registers
    const uint64_t dense = waves * npr::kResSlots * npr::kTile;  // >= 64 records per tile
    chunk = dense;
    if (stop - start >= 8 * dense && !speculative_start && !sh) {
      // large: size the links by the record density of the capture's first 256 KiB, walked here from
      // the known first record (one small D2H copy and a sync; results never depend on it)
      uint64_t mean = 0, n = 0;
      if ((st = probe_density(c, input, start, stop, e, stream, mean, n))) return st;
      if (mean) {  // 7/8 of the kept capacity at that many bytes per record
        const uint64_t fit = waves * npr::kResSlots * 64 * 7 / 8 * mean;
        chunk = std::max(dense, fit);
      }
      pack = chunk > dense;  // links past one kept round per tile: sparse tiles must share rounds
    }
  }
  if ((st = ensure(c, c->chain, 2 * sizeof(npr_summary), true))) return st;
  struct PackScope {  // this call's links run the packing resident pass; later launches do not
    npr_ctx *c;
    ~PackScope() { c->res_pack = false; }
  } pack_scope{c};
  c->res_pack = pack;
  npr_dev_outputs oc = *o;
  const npr_summary *prev = nullptr;
  uint64_t lo = start;
  for (uint64_t k = 0;; ++k) {
    const uint64_t hi = stop - lo <= chunk ? stop : lo + chunk;
    oc.summary = hi == stop ? o->summary : (npr_summary *)c->chain.p + (k & 1u);
    if ((st = launch_range(c, input, len, lo, hi, e, k == 0 ? speculative_start : 0, ref_record, prev, &oc, stream,
                           sh)))
      return st;
    if (hi == stop) return NPR_OK;
    prev = oc.summary;
    lo = hi;
  }
}

npr_status npr_dev_parse_extract_shard(npr_ctx *c, const void *input, uint64_t input_len, npr_endianness e,
                                       const npr_shard *shard, const npr_dev_outputs *o, void *stream) {
  if (!c || !o || !o->summary || !shard || (!input && input_len)) return fail(c, NPR_ERR_ARG, "null argument");
  const uint64_t len = shard->base + input_len;
  if (shard->start < shard->base || shard->start > shard->stop || shard->stop > len)
    return fail(c, NPR_ERR_ARG, "need base <= start <= stop <= base + input_len");
  ShardSpec sh;
  sh.base = shard->base;
  sh.frac_max = shard->usec_magic ? 1000000u : 1000000000u;
  sh.has_ref = shard->ts_ref != NPR_NO_ENTRY;
  sh.ts_ref = (uint32_t)shard->ts_ref;
  return chained(c, input, len, shard->start, shard->stop, e, shard->speculative_start, NPR_NO_ENTRY, o,
                 shard->chunk_bytes, stream, &sh);
}

// The range-dependent launch parameters of records starting in [start, stop) (no workspace).
static npr_status range_params(npr_ctx *c, const void *input, uint64_t len, uint64_t start, uint64_t stop,
                               npr_endianness e, int speculative_start, uint64_t ref_record, const ShardSpec *sh,
                               npr::ParseParams &p, uint64_t &nt) {
  const uint64_t base = sh ? sh->base : 0;
  if (start < base) return fail(c, NPR_ERR_ARG, "need start >= base");
  uint64_t org = 0;
  nt = tiles_for(stop - base, start - base, &org);  // tiles cover [org, stop)
  org += base;
  if (nt > 0x7fffffffull) return fail(c, NPR_ERR_ARG, "input too large");
  p.buf = (const uint8_t *)input - base;  // buf + o = file byte o (only o >= base is ever read)
  p.base = base;
  p.len = len;
  p.start = start;
  p.org = org;
  p.big = e == NPR_BIG;
  p.ntiles = (uint32_t)nt;
  p.frac_max = 1000000000u;
  p.stop = stop;
  p.ref = ref_record < len ? ref_record : ~0ull;
  // a capture file: bytes 0..3 hold the pcap magic (the kernel checks its value)
  p.flags = (start >= 24 || (ref_record != NPR_NO_ENTRY && ref_record >= 24)) ? npr::kFlagMagicAtZero : 0u;
  if (speculative_start) p.flags |= npr::kFlagSpecStart;
  if (sh) {  // a shard: bytes 0..3 (the magic) and the first record are not in its buffer
    p.flags = (p.flags & ~npr::kFlagMagicAtZero) | npr::kFlagHostSpec | (sh->has_ref ? npr::kFlagHostRef : 0u);
    p.frac_max = sh->frac_max;
    p.ts_ref = sh->ts_ref;
    p.ref = ~0ull;
  }
  return NPR_OK;
}

// The sparse record walk (npr_sparse.hip) over records starting in [p.start, p.stop): lane ranges
// of `span` bytes, 64 per group; its workspace: lanes | group aggregates | first entries | group
// prefixes | control word | Ok-flow slots (flows requested only).
static npr_status sparse_launch(npr_ctx *c, npr::ParseParams &p, const npr_summary *prev, const npr_dev_outputs *o,
                                hipStream_t s, uint64_t span) {
  npr::SparseParams sp{};
  const uint64_t range = p.stop > p.start ? p.stop - p.start : 0;
  sp.span = std::min<uint64_t>(span, npr::kSparseSpanMax);  // (a slot keeps 18 bits of record offset)
  sp.nlanes = (range + sp.span - 1) / sp.span;  // (lanes of the clamped span cover the range)
  const uint64_t ng = (sp.nlanes + 63) / 64;
  if (ng > 0x7fffffffull) return fail(c, NPR_ERR_ARG, "input too large for the sparse walk");
  sp.ngroups = (uint32_t)ng;
  sp.cap = c->sparse_cap ? c->sparse_cap : npr::kSparseCapDefault;
  auto a256 = [](uint64_t x) { return (x + 255) & ~255ull; };
  const uint64_t o_agg = a256(sp.nlanes * sizeof(npr::SparseLane)), o_first = o_agg + a256(ng * npr::kSparseAggWords * 8),
                 o_lite = o_first + a256(ng * 8), o_pre = o_lite + a256(3 * ng * 8),
                 o_scan = o_pre + a256(ng * sizeof(npr::SparsePre)),
                 o_ctl = o_scan + a256(npr::sparse_scan_words(ng) * 8), o_area = o_ctl + 256,
                 o_area_b = o_area + a256(ng * sp.cap * 64 * 16),
                 total = o->flows ? o_area_b + ng * sp.cap * 64 * 12 : o_area;
  npr_status st = ensure(c, c->sparse, total);
  if (st) return st;
  char *b = (char *)c->sparse.p;
  sp.lanes = (npr::SparseLane *)b;
  sp.aggs = (uint64_t *)(b + o_agg);
  sp.first_entry = (uint64_t *)(b + o_first);
  sp.pre = (npr::SparsePre *)(b + o_pre);
  sp.scan = (uint64_t *)(b + o_scan);
  sp.lite = (uint64_t *)(b + o_lite);
  sp.ctl = (uint64_t *)(b + o_ctl);
  sp.area = o->flows ? (uint32_t *)(b + o_area) : nullptr;
  sp.area_b = o->flows ? (uint32_t *)(b + o_area_b) : nullptr;
  if ((st = next_epoch(c, s))) return st;
  p.epoch = c->epoch;
  p.timeout_ticks = kTimeoutTicks;
  p.abort_word = c->abort_word;
  p.flows = (uint32_t *)o->flows;
  p.flows_v6 = (uint32_t *)o->flows_v6;
  p.flow_cap = o->flow_cap;
  p.summary = o->summary;
  p.stats = c->stats;
  if (prev) {
    p.prev = prev;
    p.prev_epoch = summary_epoch(c, prev);
  }
  sp.kp = p;
  log_summary(c, o->summary);  // before launching: a failed launch leaves the summary stale, and unclaimed
  if ((st = ordered_launch(c, s, [&] { return npr::launch_sparse(sp, s); }))) return st;
  c->last_pass = 8;
  return NPR_OK;
}

static npr_status launch_range(npr_ctx *c, const void *input, uint64_t len, uint64_t start, uint64_t stop,
                               npr_endianness e, int speculative_start, uint64_t ref_record,
                               const npr_summary *prev, const npr_dev_outputs *o, void *stream,
                               const ShardSpec *sh) {
  if (!c || !o || !o->summary || (!input && len)) return fail(c, NPR_ERR_ARG, "null argument");
  if (stop > len || start > stop) return fail(c, NPR_ERR_ARG, "need start <= stop <= len");
  if (((uintptr_t)input & 15u) != 0) return fail(c, NPR_ERR_ARG, "input must be 16-byte aligned");
  if (o->flows && (((uintptr_t)o->flows & 15u) != 0 || (o->flows_v6 && ((uintptr_t)o->flows_v6 & 15u))))
    return fail(c, NPR_ERR_ARG, "flow arrays must be 16-byte aligned");
  if (len >= (1ull << 40)) return fail(c, NPR_ERR_ARG, "input larger than 1 TiB (40-bit record offsets)");
  HIP_CHECK(c, hipSetDevice(c->device));
  npr::ParseParams p{};
  uint64_t nt = 0;
  npr_status st = range_params(c, input, len, start, stop, e, speculative_start, ref_record, sh, p, nt);
  if (st) return st;
  const bool flows_only = !o->record_offsets && !o->records && !o->record_status;
  if (c->resident && flows_only && (c->sparse_span || sparse_forced(c))) {
    const uint64_t span = c->sparse_span ? c->sparse_span : (c->sparse_mode >= 64 ? (uint64_t)c->sparse_mode : kSparseSpanDefault);
    if (prev && speculative_start) return fail(c, NPR_ERR_ARG, "a chained launch continues an exact chain");
    return sparse_launch(c, p, prev, o, pick(c, stream), span);
  }
  if ((st = ensure(c, c->slots, slot_bytes(nt), true))) return st;
  if ((st = ensure(c, c->srec, nt * npr::kMaxRec * sizeof(uint16_t), false))) return st;
  hipStream_t s = pick(c, stream);
  if ((st = next_epoch(c, s))) return st;
  p.epoch = c->epoch;
  p.timeout_ticks = kTimeoutTicks;
  p.slots = (npr::TileSlot *)c->slots.p;
  uint64_t nl[npr::kLevels + 1];
  level_sizes(nt, nl);
  npr::GroupSlot *gs = (npr::GroupSlot *)((char *)c->slots.p + nt * sizeof(npr::TileSlot));
  p.ngroups[0] = (uint32_t)nt;
  p.groups[0] = nullptr;
  for (int l = 1; l <= npr::kLevels; ++l) {
    p.groups[l] = gs;
    p.ngroups[l] = (uint32_t)nl[l];
    gs += nl[l];
  }
  p.srec_g = (uint16_t *)c->srec.p;
  p.abort_word = c->abort_word;
  p.rec_off = o->record_offsets;
  p.recs = o->records;
  p.rec_status = o->record_status;
  p.rec_cap = o->record_cap;
  p.flows = (uint32_t *)o->flows;
  p.flows_v6 = (uint32_t *)o->flows_v6;
  p.flow_cap = o->flow_cap;
  p.summary = o->summary;
  p.stats = c->stats;
  p.stamps = nullptr;
  if (c->stats_mode >= 2) {
    if ((st = ensure(c, c->stamps, nt * npr::kStampWords * 8, true))) return st;
    p.stamps = (uint64_t *)c->stamps.p;
    c->stamp_tiles = nt;
  }
  // flows-only launches: the resident single pass, one wave per (CU x resident waves), at most
  // kResMaxWaves and at most one per tile
  const bool resident = c->resident && !p.rec_off && !p.recs && !p.rec_status;
  if (prev) {
    if (!resident) return fail(c, NPR_ERR_ARG, "a chained launch produces flows only (resident pass)");
    if (speculative_start) return fail(c, NPR_ERR_ARG, "a chained launch continues an exact chain");
    p.prev = prev;
    p.prev_epoch = 0;  // the epoch of the launch that wrote *prev, when it was one of ours: the
    // most recent of the last two launches that wrote that address (an older launch may have
    // used the same summary slot)
    p.prev_epoch = summary_epoch(c, prev);
  }
  if (resident) {
    if ((st = res_geometry(c))) return st;
    uint64_t wv = std::min<uint64_t>(nt, c->res_waves);
    if (c->resident > 1) wv = std::min<uint64_t>(wv, (uint64_t)c->resident);
    p.nwaves = (uint32_t)wv;
    if (wv % npr::kResWgMin == 0) {  // per workgroup, then per wave (res_range)
      const uint64_t nwg = wv / npr::kResWgMin;
      p.wg_q = (uint32_t)(nt / nwg);
      p.wg_r = (uint32_t)(nt % nwg);
    }
    p.rslots = (npr::RangeSlot *)c->slots.p;
    p.rgroups = p.groups[1];
    p.pack = c->res_pack ? 1u : 0u;
    // every workgroup aggregate the launch writes must lie inside the slot allocation
    const uint64_t nb = (wv + npr::kResWgMin - 1) / npr::kResWgMin;
    if ((const char *)(p.rgroups + nb) > (const char *)c->slots.p + c->slots.cap)
      return fail(c, NPR_ERR_ARG, "internal: resident workgroup slots exceed the workspace (%llu groups)",
                  (unsigned long long)nb);
    p.rcnt = (uint32_t *)((char *)c->abort_word + kCtlCounters);
  }
  // who writes which summary (npr_dev_check and chained launches check it), logged before the launch:
  // if the launch fails, the summary keeps an older epoch than its log entry and npr_dev_check
  // reports it instead of returning the previous parse's results
  log_summary(c, o->summary);
  if ((st = ordered_launch(c, s, [&] { return npr::launch_parse_extract(p, s); }))) return st;
  c->last_pass = resident ? 2 : 1;
  return NPR_OK;
}

npr_status npr_dev_check(npr_ctx *c, const npr_dev_outputs *o, void *stream, npr_summary *hs) {
  if (!c || !o || !o->summary) return NPR_ERR_ARG;
  hipStream_t s = pick(c, stream);
  HIP_CHECK(c, hipMemcpyAsync(c->summary_h, o->summary, sizeof(npr_summary), hipMemcpyDeviceToHost, s));
  HIP_CHECK(c, hipStreamSynchronize(s));
  if (hs) *hs = *c->summary_h;
  const uint32_t want = summary_epoch(c, o->summary);  // the launch that wrote this summary
  if (c->summary_h->epoch == (want ? want : c->epoch)) probe_correct(c, o->summary, *c->summary_h);
  if (c->summary_h->epoch != (want ? want : c->epoch)) {
    return fail(c, NPR_ERR_TIMEOUT, "parse did not complete (tile hand-off timed out)");
  }
  if (c->summary_h->flags) return fail(c, NPR_ERR_CAPACITY, "output capacity exceeded (flags=%u)", c->summary_h->flags);
  return NPR_OK;
}

// ---- K independent captures, one call ------------------------------------------------------------
// Each item is the ordinary npr_dev_parse_extract launch, in order on the stream.  Round 3 ran up to
// 8 flows-only items in one resident launch (k_parse_batch); measured on 8 captures of 16 K / 64 K /
// 262 K / 1 M records it gained 1.06x / 1.09x / 1.01x / 0.96x (profiles/r04_batch_small.jsonl), not
// the 1.3x that would pay for a second kernel instantiation, so the entry point stays and the
// kernel went.
npr_status npr_dev_parse_extract_batch(npr_ctx *c, const npr_batch_item *items, uint32_t n, void *stream) {
  if (!c || (!items && n)) return fail(c, NPR_ERR_ARG, "null argument");
  for (uint32_t i = 0; i < n; ++i) {
    const npr_batch_item &it = items[i];
    if (npr_status st = npr_dev_parse_extract(c, it.input, it.len, it.start, (npr_endianness)it.endianness, &it.out, stream))
      return st;
  }
  return NPR_OK;
}

// convert_records over device records: one pass, look-back words in the slot allocation
static npr_status convert_launch(npr_ctx *c, const void *input, uint64_t len, const npr_record *recs, uint64_t n,
                                 npr_flow *out, npr_flow_v6 *out_v6, uint64_t cap, uint64_t *total, hipStream_t s) {
  if (!c->cus) (void)hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, c->device);
  npr_status st = ensure(c, c->slots, std::max<uint64_t>(npr::convert_look_words(n, c->cus), 1) * 8, true);
  if (st) return st;
  if ((st = next_epoch(c, s))) return st;
  return ordered_launch(c, s, [&] {
    return npr::launch_convert_records((const uint8_t *)input, len, recs, n, (uint32_t *)out, (uint32_t *)out_v6, cap,
                                       (uint64_t *)c->slots.p, c->epoch, total, kTimeoutTicks, c->cus, s);
  });
}

npr_status npr_dev_flow_aggregate(npr_ctx *c, const npr_flow *flows, const npr_flow_v6 *flows_v6,
                                  const uint64_t *weights, uint64_t n, npr_flow *out, npr_flow_v6 *out_v6,
                                  uint64_t *counts, uint64_t cap, uint64_t *n_out, void *stream) {
  if (!c || (!flows && n) || !n_out || (!out && cap)) return fail(c, NPR_ERR_ARG, "null argument");
  if (n > npr::kMaxAggRows) return fail(c, NPR_ERR_ARG, "at most 2^30 flow rows per call");
  HIP_CHECK(c, hipSetDevice(c->device));
  npr_status st = ensure(c, c->agg, npr::flow_table_bytes(n));
  if (st) return st;
  HIP_CHECK(c, npr::launch_flow_aggregate((const uint32_t *)flows, (const uint32_t *)flows_v6, weights, n, c->agg.p,
                                          (uint32_t *)out, (uint32_t *)out_v6, counts, cap, n_out, pick(c, stream)));
  return NPR_OK;
}

npr_status npr_dev_vxlan_flows(npr_ctx *c, const void *input, uint64_t len, const npr_record *recs, uint64_t n,
                               uint32_t dst_port, npr_endianness e, npr_flow *flows, npr_flow_v6 *flows_v6,
                               uint8_t *status, uint32_t *vni, void *stream) {
  if (!c || (!input && len) || (!recs && n)) return fail(c, NPR_ERR_ARG, "null argument");
  if (dst_port > 0xffffu) return fail(c, NPR_ERR_ARG, "dst_port must be 0..65535");
  HIP_CHECK(c, hipSetDevice(c->device));
  HIP_CHECK(c, npr::launch_vxlan_flows((const uint8_t *)input, len, recs, n, dst_port, e == NPR_BIG, (uint32_t *)flows,
                                       (uint32_t *)flows_v6, status, vni, pick(c, stream)));
  return NPR_OK;
}

npr_status npr_dev_flow_details(npr_ctx *c, const void *input, uint64_t len, const npr_record *recs, uint64_t n,
                                uint8_t *status, uint64_t *detail, void *stream) {
  if (!c || (!input && len) || (!recs && n)) return fail(c, NPR_ERR_ARG, "null argument");
  HIP_CHECK(c, hipSetDevice(c->device));
  HIP_CHECK(c, npr::launch_flow_detail((const uint8_t *)input, len, recs, n, status, detail, pick(c, stream)));
  return NPR_OK;
}

npr_status npr_dev_convert_records(npr_ctx *c, const void *input, uint64_t len, const npr_record *recs, uint64_t n,
                                   npr_flow *out, npr_flow_v6 *out_v6, uint64_t cap, uint64_t *n_out, void *stream) {
  if (!c || (!input && len) || (!recs && n) || !n_out || (!out && cap)) return fail(c, NPR_ERR_ARG, "null argument");
  HIP_CHECK(c, hipSetDevice(c->device));
  return convert_launch(c, input, len, recs, n, out, out_v6, cap, n_out, pick(c, stream));
}

npr_status npr_dev_extract_flows(npr_ctx *c, const void *input, uint64_t len, const npr_record *recs,
                                 uint64_t n, npr_flow *flows, npr_flow_v6 *flows_v6, uint8_t *status,
                                 void *stream) {
  if (!c || (!input && len) || (!recs && n)) return fail(c, NPR_ERR_ARG, "null argument");
  HIP_CHECK(c, hipSetDevice(c->device));
  HIP_CHECK(c, npr::launch_extract_dense((const uint8_t *)input, len, recs, n, (uint32_t *)flows,
                                         (uint32_t *)flows_v6, status, pick(c, stream)));
  return NPR_OK;
}

// ---- host-memory entry points ---------------------------------------------------------------
// Small host calls (a handful of records: the Rust crate's per-record FlowExtraction::extract_flow
// and its error-payload query) skip the device staging buffers: input and records are packed into
// one page-locked arena that the kernel reads over PCIe, and it writes its outputs there too, so a
// call is one launch and one synchronisation instead of five pageable copies (65 us -> see
// scripts/bench_records_api.py host_extract_flow_one_record).  Arena layout: input | records |
// then the outputs at the offsets the caller asks for (16-B aligned).
constexpr uint64_t kSmallBytes = 256u << 10;  // input + records at most this many bytes
static uint64_t a16(uint64_t x) { return (x + 15) & ~15ull; }
static npr_status small_arena(npr_ctx *c, const uint8_t *in, size_t len, const npr_record *records, size_t n,
                              uint64_t out_bytes, uint8_t *&arena, uint64_t &rec_off, uint64_t &out_off) {
  rec_off = a16(len);
  out_off = a16(rec_off + n * sizeof(npr_record));
  const uint64_t need = out_off + out_bytes;
  if (need > c->small_cap) {
    if (c->small_h) HIP_CHECK(c, hipHostFree(c->small_h));
    c->small_h = nullptr;
    c->small_cap = 0;
    const uint64_t cap = std::max<uint64_t>(need, 64u << 10);
    HIP_CHECK(c, hipHostMalloc((void **)&c->small_h, cap, 0));
    c->small_cap = cap;
  }
  arena = c->small_h;
  if (len) memcpy(arena, in, len);
  if (n) memcpy(arena + rec_off, records, n * sizeof(npr_record));
  return NPR_OK;
}
static bool small_call(size_t len, size_t n) { return len + n * sizeof(npr_record) <= kSmallBytes; }

static npr_status stage_input(npr_ctx *c, const uint8_t *in, size_t len) {
  npr_status st = ensure(c, c->in, len + 16);
  if (st) return st;
  probe_forget(c, c->in.p);  // new bytes at the staging address: its density is probed afresh
  if (len) HIP_CHECK(c, hipMemcpyAsync(c->in.p, in, len, hipMemcpyHostToDevice, c->stream));
  return NPR_OK;
}

// Flows-only host parse, overlapped: chunk j = bytes [a_j, a_j+1) of the capture (a_j = j x chunk)
// goes H2D on copy_stream; link j of the chain (records starting in [max(start, a_j), a_j+1))
// launches on the compute stream once chunks j and j+1 have landed, reading at most up to a_j+2.
// A record longer than a chunk therefore ends that link's chain early; the caller checks for
// that on the host and parses again without streaming (npr_dev_parse_extract_chain semantics
// otherwise: same rows, counts and summary as one launch).
static npr_status stream_parse(npr_ctx *c, const uint8_t *in, size_t len, uint64_t start, npr_endianness e,
                               const npr_dev_outputs *o) {
  const uint64_t chunk = c->stream_chunk;
  const uint64_t nchunks = (len + chunk - 1) / chunk;
  npr_status st = ensure(c, c->in, len + 16);
  if (st) return st;
  probe_forget(c, c->in.p);
  if ((st = ensure(c, c->chain, 2 * sizeof(npr_summary), true))) return st;
  if (!c->copy_stream) HIP_CHECK(c, hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
  while (c->copied.size() < nchunks) {
    hipEvent_t ev;
    HIP_CHECK(c, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    c->copied.push_back(ev);
  }
  uint8_t *dev = (uint8_t *)c->in.p;
  // the compute stream's earlier work (a previous parse reading the staging buffer) comes first
  HIP_CHECK(c, hipEventRecord(c->copied[0], c->stream));
  HIP_CHECK(c, hipStreamWaitEvent(c->copy_stream, c->copied[0], 0));
  for (uint64_t j = 0; j < nchunks; ++j) {
    const uint64_t a = j * chunk, b = std::min<uint64_t>(len, a + chunk);
    HIP_CHECK(c, hipMemcpyAsync(dev + a, in + a, b - a, hipMemcpyHostToDevice, c->copy_stream));
    HIP_CHECK(c, hipEventRecord(c->copied[j], c->copy_stream));
  }
  npr_dev_outputs oc = *o;
  const npr_summary *prev = nullptr;
  uint64_t k = 0;
  for (uint64_t j = 0; j < nchunks; ++j) {
    const uint64_t lo = std::max<uint64_t>(start, j * chunk), hi = std::min<uint64_t>(len, (j + 1) * chunk);
    if (hi <= lo && hi < len) continue;  // (start past this chunk)
    const uint64_t jn = std::min<uint64_t>(j + 1, nchunks - 1);
    HIP_CHECK(c, hipStreamWaitEvent(c->stream, c->copied[jn], 0));
    const uint64_t readable = std::min<uint64_t>(len, (jn + 1) * chunk);
    oc.summary = hi == len ? o->summary : (npr_summary *)c->chain.p + (k++ & 1u);
    if ((st = launch_range(c, dev, readable, lo, hi, e, 0, start, prev, &oc, c->stream))) return st;
    if (hi == len) break;
    prev = oc.summary;
  }
  return NPR_OK;
}

// ---- pinned, overlapped host path (row f1): H2D chunks | chained launches | D2H of each link's rows
static npr_status grow_events(npr_ctx *c, std::vector<hipEvent_t> &v, uint64_t n) {
  while (v.size() < n) {
    hipEvent_t ev;
    HIP_CHECK(c, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    v.push_back(ev);
  }
  return NPR_OK;
}

constexpr size_t kRegisterMin = 1u << 20;  // caller buffers registered for a pipelined call: at least this size

// Is [p, p + n) page-locked host memory (hipHostMalloc'ed or registered)?
static bool host_pinned(const void *p, size_t n) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  (void)n;
  return a.type == hipMemoryTypeHost && a.hostPointer != nullptr;
}

// ---- row f1 past device memory: the capture streams through a bounded device window --------------
// Chunk j (file bytes [j*chunk, (j+1)*chunk)) is uploaded into ring slot j % W; kWinHalo bytes past
// the ring's end mirror slot 0's head, so link j reads [j*chunk, (j+1)*chunk + kWinHalo) contiguously
// from its slot (the records that straddle its chunk end).  Link j (records starting in chunk j)
// launches once chunk j+1 has landed and writes its convert_records rows into flow-ring slot
// j % kWinRowSlots: the kernel writes the k-th Ok flow of the capture to row flow_cap - 1 - k, so the
// slot passed with flow_cap = S + K (K = the Ok flows before link j, read back after link j-1) gets
// link j's rows right-aligned at its end.  The host reads each link's summary as it completes, copies
// its rows to the caller's table on the D2H stream and launches the next link; the upload of chunk
// j+W waits for link j.  PCIe, not the parse, sets the pace: the copy stream always holds W chunks.
constexpr uint64_t kWinHalo = 260u << 10;  // >= 16 + 262144 B, the largest pcap snaplen's record
constexpr uint64_t kWinRowSlots = 3;
constexpr uint64_t kWinMinChunk = 512u << 10;

static npr_status windowed_parse(npr_ctx *c, const uint8_t *in, size_t len, npr_endianness e, uint64_t chunk,
                                 uint64_t W, npr_flow *hout, npr_flow_v6 *hout6, uint64_t fcap, npr_summary &fin) {
  const uint64_t start = 24;
  const uint64_t nlinks = (len + chunk - 1) / chunk;
  const uint64_t S = chunk / 16 + 1;  // rows one link can produce: every record is >= 16 B
  npr_status st;
  if ((st = ensure(c, c->in, W * chunk + kWinHalo + 4096))) return st;
  if ((st = ensure(c, c->flows, kWinRowSlots * S * sizeof(npr_flow)))) return st;
  if (hout6 && (st = ensure(c, c->flows_v6, kWinRowSlots * S * sizeof(npr_flow_v6)))) return st;
  if ((st = ensure(c, c->chain, 2 * sizeof(npr_summary), true))) return st;
  if (c->sum_host_cap < 2) {
    if (c->sum_host) HIP_CHECK(c, hipHostFree(c->sum_host));
    c->sum_host = nullptr;
    c->sum_host_cap = 0;
    HIP_CHECK(c, hipHostMalloc((void **)&c->sum_host, 2 * sizeof(npr_summary), 0));
    c->sum_host_cap = 2;
  }
  if (!c->copy_stream) HIP_CHECK(c, hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
  if (!c->d2h_stream) HIP_CHECK(c, hipStreamCreateWithFlags(&c->d2h_stream, hipStreamNonBlocking));
  if ((st = grow_events(c, c->copied, W))) return st;
  if ((st = grow_events(c, c->linked, W))) return st;
  if ((st = grow_events(c, c->row_copied, kWinRowSlots))) return st;
  uint8_t *ring = (uint8_t *)c->in.p;
  npr_flow *rows = (npr_flow *)c->flows.p;
  npr_flow_v6 *rows6 = hout6 ? (npr_flow_v6 *)c->flows_v6.p : nullptr;
  npr_summary *dsum = (npr_summary *)c->chain.p;
  // links past the first do not hold the magic or the first record: their speculation context
  // (the magic's ts_usec bound, the first record's ts_sec) comes from the host, as for a shard
  ShardSpec sh;
  uint32_t magic;
  memcpy(&magic, in, 4);
  sh.frac_max = (magic == 0xA1B2C3D4u || magic == 0xD4C3B2A1u) ? 1000000u : 1000000000u;
  sh.has_ref = len >= start + 16;
  sh.ts_ref = sh.has_ref ? rd_u32(in + start, e == NPR_BIG) : 0u;
  // the compute stream's earlier work (a previous call reading the ring) comes first
  HIP_CHECK(c, hipEventRecord(c->copied[0], c->stream));
  HIP_CHECK(c, hipStreamWaitEvent(c->copy_stream, c->copied[0], 0));
  HIP_CHECK(c, hipStreamWaitEvent(c->d2h_stream, c->copied[0], 0));
  auto upload = [&](uint64_t m) -> npr_status {
    const uint64_t a = m * chunk, b = std::min<uint64_t>(len, a + chunk);
    HIP_CHECK(c, hipMemcpyAsync(ring + (m % W) * chunk, in + a, b - a, hipMemcpyHostToDevice, c->copy_stream));
    if (m % W == 0)  // slot 0's head, mirrored past the ring's end for link m-1
      HIP_CHECK(c, hipMemcpyAsync(ring + W * chunk, in + a, std::min<uint64_t>(kWinHalo, b - a), hipMemcpyHostToDevice,
                                  c->copy_stream));
    HIP_CHECK(c, hipEventRecord(c->copied[m % W], c->copy_stream));
    return NPR_OK;
  };
  for (uint64_t m = 0; m < std::min<uint64_t>(W, nlinks); ++m)
    if ((st = upload(m))) return st;
  uint64_t K = 0;  // Ok flows of the links done so far
  fin = npr_summary{};
  for (uint64_t j = 0; j < nlinks; ++j) {
    const uint64_t a = j * chunk, lo = std::max<uint64_t>(start, a), hi = std::min<uint64_t>(len, a + chunk);
    const uint64_t flen = std::min<uint64_t>(len, hi + kWinHalo);  // file bytes this link may read
    HIP_CHECK(c, hipStreamWaitEvent(c->stream, c->copied[std::min<uint64_t>(j + 1, nlinks - 1) % W], 0));
    if (j >= kWinRowSlots) HIP_CHECK(c, hipStreamWaitEvent(c->stream, c->row_copied[j % kWinRowSlots], 0));
    npr_dev_outputs o{};
    o.flows = rows + (j % kWinRowSlots) * S;
    o.flows_v6 = rows6 ? rows6 + (j % kWinRowSlots) * S : nullptr;
    o.flow_cap = S + K;
    o.summary = dsum + (j & 1u);
    if (j == 0) {
      st = launch_range(c, ring, flen, std::min(lo, hi), hi, e, 0, start, nullptr, &o, c->stream);
    } else {
      ShardSpec shj = sh;
      shj.base = a;
      st = launch_range(c, ring + (j % W) * chunk, flen, lo, hi, e, 0, NPR_NO_ENTRY, dsum + ((j - 1) & 1u), &o,
                        c->stream, &shj);
    }
    if (st) return st;
    HIP_CHECK(c, hipMemcpyAsync(c->sum_host, o.summary, sizeof(npr_summary), hipMemcpyDeviceToHost, c->stream));
    HIP_CHECK(c, hipEventRecord(c->linked[j % W], c->stream));
    if (j + W < nlinks) {  // chunk j+W reuses link j's slot
      HIP_CHECK(c, hipStreamWaitEvent(c->copy_stream, c->linked[j % W], 0));
      if ((st = upload(j + W))) return st;
    }
    HIP_CHECK(c, hipEventSynchronize(c->linked[j % W]));
    const npr_summary sj = *c->sum_host;
    if (sj.epoch != c->epoch) {
      uint32_t ab = 0;
      HIP_CHECK(c, hipMemcpy(&ab, c->abort_word, 4, hipMemcpyDeviceToHost));
      return fail(c, NPR_ERR_TIMEOUT, "windowed parse did not complete: link %llu of %llu (epoch %u, abort word %u)",
                  (unsigned long long)j, (unsigned long long)nlinks, c->epoch, ab);
    }
    // flows k in [K, min(Kj, fcap)) sit at slot rows S-1-(k-K) and belong at caller rows fcap-1-k
    const uint64_t hk = std::min<uint64_t>(sj.n_flows, fcap);
    if (hk > K) {
      const uint64_t n = hk - K;
      HIP_CHECK(c, hipStreamWaitEvent(c->d2h_stream, c->linked[j % W], 0));
      HIP_CHECK(c, hipMemcpyAsync(hout + (fcap - hk), o.flows + (S - n), n * sizeof(npr_flow), hipMemcpyDeviceToHost,
                                  c->d2h_stream));
      if (hout6)
        HIP_CHECK(c, hipMemcpyAsync(hout6 + (fcap - hk), o.flows_v6 + (S - n), n * sizeof(npr_flow_v6),
                                    hipMemcpyDeviceToHost, c->d2h_stream));
    }
    HIP_CHECK(c, hipEventRecord(c->row_copied[j % kWinRowSlots], c->d2h_stream));
    K = sj.n_flows;
    fin = sj;
  }
  HIP_CHECK(c, hipStreamSynchronize(c->d2h_stream));
  return NPR_OK;
}

// Chunks of the capture the device window holds (0 = stage the whole capture): NPR_OPT_DEVICE_WINDOW,
// or (auto) 8 when staging the capture and its flow table would not fit in free device memory.
static uint64_t window_chunks(npr_ctx *c, size_t len, uint64_t chunk, uint64_t fcap, bool v6) {
  const uint64_t nlinks = (len + chunk - 1) / chunk;
  if (c->window >= 3) return nlinks > (uint64_t)c->window ? (uint64_t)c->window : 0;
  auto grow = [](const DevBuf &b, uint64_t want) { return want > b.cap ? want - b.cap : 0; };
  const uint64_t need = grow(c->in, len + 16) + grow(c->flows, fcap * sizeof(npr_flow)) +
                        (v6 ? grow(c->flows_v6, fcap * sizeof(npr_flow_v6)) : 0);
  size_t free_b = 0, total_b = 0;
  if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return need > free_b / 10 * 9 && nlinks > 8 ? 8 : 0;
}

npr_status npr_parse_extract_pipelined(npr_ctx *c, const uint8_t *in, size_t len, npr_global_header *hdr,
                                       npr_flow *out, npr_flow_v6 *out_v6, size_t flow_cap, size_t *n_flows,
                                       size_t *consumed, uint64_t chunk_bytes) {
  if (!c || !hdr || !out || (!in && len)) return fail(c, NPR_ERR_ARG, "null argument");
  npr_status st = npr_global_header_parse(in, len, hdr, nullptr);  // file.rs:18
  if (st) return st;
  HIP_CHECK(c, hipSetDevice(c->device));
  const uint64_t start = 24;
  const npr_endianness e = (npr_endianness)hdr->endianness;
  const uint64_t chunk = std::max<uint64_t>(chunk_bytes ? chunk_bytes : (32ull << 20), 1ull << 16);
  const uint64_t nlinks = (len + chunk - 1) / chunk;
  const uint64_t max_rec = (len - start) / 16 + 1;
  const uint64_t fcap = std::min<uint64_t>(flow_cap, max_rec);
  // device row r is the caller's row r + shift: the flows end at out[flow_cap - 1]
  const uint64_t shift = flow_cap - fcap;
  npr_flow *hout = out + shift;
  npr_flow_v6 *hout6 = out_v6 ? out_v6 + shift : nullptr;
  // the caller's buffers: page-locked for the DMA engines (registered for this call unless they
  // are).  Buffers under 1 MiB stay pageable (HIP stages them): a small heap buffer shares its pages
  // with other objects and with the call's other small buffers, and registering such page-sharing
  // ranges is where a later pageable D2H copy in the same process once failed with
  // hipErrorIllegalAddress (round 6); small copies gain nothing from pinning anyway
  struct Unreg {  // unregister on every exit path, and let the runtime finish releasing them before
                  // the caller may free (and the allocator reuse) the memory
    void *p[3] = {nullptr, nullptr, nullptr};
    ~Unreg() {
      bool any = false;
      for (void *q : p)
        if (q) {
          (void)hipHostUnregister(q);
          any = true;
        }
      if (any) (void)hipDeviceSynchronize();
    }
  } unreg;
  const void *bufs[3] = {in, hout, hout6};
  const size_t sizes[3] = {len, fcap * sizeof(npr_flow), hout6 ? fcap * sizeof(npr_flow_v6) : 0};
  for (int i = 0; i < 3; ++i) {
    if (sizes[i] < kRegisterMin || host_pinned(bufs[i], sizes[i])) continue;
    const hipError_t r = hipHostRegister((void *)bufs[i], sizes[i], hipHostRegisterDefault);
    if (r == hipErrorHostMemoryAlreadyRegistered) {
      (void)hipGetLastError();
      continue;
    }
    HIP_CHECK(c, r);
    unreg.p[i] = (void *)bufs[i];
  }
  const uint64_t wchunk = (std::max<uint64_t>(chunk, kWinMinChunk) + 4095) & ~4095ull;
  if (const uint64_t W = window_chunks(c, len, wchunk, fcap, out_v6 != nullptr)) {
    npr_summary fin{};
    if ((st = windowed_parse(c, in, len, e, wchunk, W, hout, hout6, fcap, fin))) return st;
    if (fin.consumed + 16 <= len) {  // the chain stopped at a record: complete, yet longer than the halo?
      const uint64_t incl = rd_u32(in + fin.consumed + 8, e == NPR_BIG);
      if (incl <= len - fin.consumed - 16)
        return fail(c, NPR_ERR_CAPACITY, "the record at offset %llu (%llu B) crosses a chunk end and is longer than "
                    "the device window's %llu-B halo", (unsigned long long)fin.consumed, (unsigned long long)incl,
                    (unsigned long long)kWinHalo);
    }
    if (n_flows) *n_flows = fin.n_flows;
    if (consumed) *consumed = fin.consumed;
    if (fin.n_flows > flow_cap || fin.flags) return fail(c, NPR_ERR_CAPACITY, "output capacity exceeded");
    return NPR_OK;
  }
  if ((st = ensure(c, c->in, len + 16))) return st;
  if ((st = ensure(c, c->flows, std::max<uint64_t>(fcap, 1) * sizeof(npr_flow)))) return st;
  if (out_v6 && (st = ensure(c, c->flows_v6, std::max<uint64_t>(fcap, 1) * sizeof(npr_flow_v6)))) return st;
  if ((st = ensure(c, c->chain, std::max<uint64_t>(nlinks, 2) * sizeof(npr_summary), true))) return st;
  if (c->sum_host_cap < nlinks) {
    if (c->sum_host) HIP_CHECK(c, hipHostFree(c->sum_host));
    c->sum_host = nullptr;
    c->sum_host_cap = 0;
    HIP_CHECK(c, hipHostMalloc((void **)&c->sum_host, nlinks * sizeof(npr_summary), 0));
    c->sum_host_cap = nlinks;
  }
  if (!c->copy_stream) HIP_CHECK(c, hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
  if (!c->d2h_stream) HIP_CHECK(c, hipStreamCreateWithFlags(&c->d2h_stream, hipStreamNonBlocking));
  if ((st = grow_events(c, c->copied, nlinks))) return st;
  if ((st = grow_events(c, c->linked, nlinks))) return st;
  uint8_t *dev = (uint8_t *)c->in.p;
  npr_summary *dsum = (npr_summary *)c->chain.p;
  // the compute stream's earlier work (a previous parse reading the staging buffer) comes first
  HIP_CHECK(c, hipEventRecord(c->copied[0], c->stream));
  HIP_CHECK(c, hipStreamWaitEvent(c->copy_stream, c->copied[0], 0));
  HIP_CHECK(c, hipStreamWaitEvent(c->d2h_stream, c->copied[0], 0));
  HIP_CHECK(c, hipMemsetAsync(dsum, 0, nlinks * sizeof(npr_summary), c->stream));  // no stale summaries
  for (uint64_t j = 0; j < nlinks; ++j) {  // every H2D chunk queued up front
    const uint64_t a = j * chunk, b = std::min<uint64_t>(len, a + chunk);
    HIP_CHECK(c, hipMemcpyAsync(dev + a, in + a, b - a, hipMemcpyHostToDevice, c->copy_stream));
    HIP_CHECK(c, hipEventRecord(c->copied[j], c->copy_stream));
  }
  npr_dev_outputs o{};
  o.flows = fcap ? (npr_flow *)c->flows.p : nullptr;
  o.flows_v6 = (fcap && out_v6) ? (npr_flow_v6 *)c->flows_v6.p : nullptr;
  o.flow_cap = fcap;
  const npr_summary *prev = nullptr;
  uint64_t last = 0;
  for (uint64_t j = 0; j < nlinks; ++j) {  // link j: records starting in chunk j, once j and j+1 landed
    const uint64_t lo = std::max<uint64_t>(start, j * chunk), hi = std::min<uint64_t>(len, (j + 1) * chunk);
    const uint64_t jn = std::min<uint64_t>(j + 1, nlinks - 1);
    HIP_CHECK(c, hipStreamWaitEvent(c->stream, c->copied[jn], 0));
    const uint64_t readable = std::min<uint64_t>(len, (jn + 1) * chunk);
    o.summary = dsum + j;
    if (hi > lo || hi == len) {
      if ((st = launch_range(c, dev, readable, std::min(lo, hi), hi, e, 0, start, prev, &o, c->stream))) return st;
      prev = o.summary;
    } else {  // the header alone spans this chunk: carry the previous summary (nothing starts here)
      HIP_CHECK(c, hipMemsetAsync(o.summary, 0, sizeof(npr_summary), c->stream));
    }
    HIP_CHECK(c, hipMemcpyAsync(c->sum_host + j, prev ? prev : o.summary, sizeof(npr_summary), hipMemcpyDeviceToHost,
                                c->stream));
    HIP_CHECK(c, hipEventRecord(c->linked[j], c->stream));
    last = j;
  }
  // the flow rows of each link go back as soon as it is done, while later chunks still upload:
  // link j's rows are [fcap - cum_j, fcap - cum_{j-1}) of the right-aligned table (cum = running
  // n_flows), the same rows of the caller's table
  uint64_t cum = 0;
  npr_summary fin{};
  for (uint64_t j = 0; j <= last; ++j) {
    HIP_CHECK(c, hipEventSynchronize(c->linked[j]));
    const npr_summary sj = c->sum_host[j];
    if (sj.epoch == 0) continue;  // nothing launched yet (a header spanning the first chunk)
    fin = sj;
    const uint64_t nc = std::min<uint64_t>(sj.n_flows, fcap);
    if (nc > cum) {
      HIP_CHECK(c, hipStreamWaitEvent(c->d2h_stream, c->linked[j], 0));
      HIP_CHECK(c, hipMemcpyAsync(hout + (fcap - nc), (npr_flow *)c->flows.p + (fcap - nc), (nc - cum) * sizeof(npr_flow),
                                  hipMemcpyDeviceToHost, c->d2h_stream));
      if (hout6)
        HIP_CHECK(c, hipMemcpyAsync(hout6 + (fcap - nc), (npr_flow_v6 *)c->flows_v6.p + (fcap - nc),
                                    (nc - cum) * sizeof(npr_flow_v6), hipMemcpyDeviceToHost, c->d2h_stream));
      cum = nc;
    }
  }
  HIP_CHECK(c, hipStreamSynchronize(c->d2h_stream));
  if (fin.epoch != c->epoch) {  // which link stopped, and did a bounded wait abort it?
    uint32_t ab = 0;
    HIP_CHECK(c, hipMemcpy(&ab, c->abort_word, 4, hipMemcpyDeviceToHost));
    uint64_t bad = 0;
    while (bad <= last && c->sum_host[bad].epoch != 0) ++bad;
    return fail(c, NPR_ERR_TIMEOUT,
                "pipelined parse did not complete: link %llu of %llu wrote no summary (last epoch %u, context epoch %u, "
                "abort word %u)",
                (unsigned long long)bad, (unsigned long long)(last + 1), fin.epoch, c->epoch, ab);
  }
  if (fin.consumed + 16 <= len) {  // the chain stopped at a complete record longer than a chunk:
    const uint64_t incl = rd_u32(in + fin.consumed + 8, e == NPR_BIG);  // parse the staged capture whole
    if (incl <= len - fin.consumed - 16) {
      o.summary = c->summary;
      if ((st = npr_dev_parse_extract(c, dev, len, start, e, &o, c->stream))) return st;
      if ((st = npr_dev_check(c, &o, c->stream, &fin)) && st != NPR_ERR_CAPACITY) return st;
      const uint64_t nc = std::min<uint64_t>(fin.n_flows, fcap);
      if (nc) {
        HIP_CHECK(c, hipMemcpyAsync(hout + (fcap - nc), (npr_flow *)c->flows.p + (fcap - nc), nc * sizeof(npr_flow),
                                    hipMemcpyDeviceToHost, c->stream));
        if (hout6)
          HIP_CHECK(c, hipMemcpyAsync(hout6 + (fcap - nc), (npr_flow_v6 *)c->flows_v6.p + (fcap - nc),
                                      nc * sizeof(npr_flow_v6), hipMemcpyDeviceToHost, c->stream));
        HIP_CHECK(c, hipStreamSynchronize(c->stream));
      }
    }
  }
  if (n_flows) *n_flows = fin.n_flows;
  if (consumed) *consumed = fin.consumed;
  if (fin.n_flows > flow_cap || fin.flags) return fail(c, NPR_ERR_CAPACITY, "output capacity exceeded");
  return NPR_OK;
}

// ---- the multi-GPU step's node-local summary exchange (parallel.ShmExchange) -------------------
npr_status npr_shm_all_gather(void *seg, int world, int rank, int depth, uint64_t rec, uint64_t seq,
                              const void *mine, uint64_t n, void *out, int timeout_ms) {
  if (!seg || world <= 0 || rank < 0 || rank >= world || depth < 2 || rec < 64 + n || !seq || (n && (!mine || !out)))
    return NPR_ERR_ARG;
  uint8_t *base = (uint8_t *)seg;
  const uint64_t d = seq % (uint64_t)depth;
  uint8_t *my = base + ((uint64_t)rank * depth + d) * rec;
  memcpy(my + 64, mine, n);
  __atomic_store_n((uint64_t *)my, seq, __ATOMIC_RELEASE);  // the payload before the sequence word
  timespec t0{};
  bool timed = false;
  for (int r = 0; r < world; ++r) {
    const uint8_t *sl = base + ((uint64_t)r * depth + d) * rec;
    for (uint32_t spins = 0; __atomic_load_n((const uint64_t *)sl, __ATOMIC_ACQUIRE) != seq; ++spins) {
      if (spins < 512) {
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
        continue;
      }
      sched_yield();  // ranks may share host cores
      if ((spins & 255u) == 0) {
        timespec t;
        clock_gettime(CLOCK_MONOTONIC, &t);
        if (!timed) {
          t0 = t;
          timed = true;
        } else if ((t.tv_sec - t0.tv_sec) * 1000 + (t.tv_nsec - t0.tv_nsec) / 1000000 > timeout_ms) {
          return NPR_ERR_TIMEOUT;
        }
      }
    }
    memcpy((uint8_t *)out + (uint64_t)r * n, sl + 64, n);
  }
  return NPR_OK;
}

npr_status npr_host_alloc(npr_ctx *c, size_t bytes, void **out) {
  if (!c || !out) return fail(c, NPR_ERR_ARG, "null argument");
  HIP_CHECK(c, hipSetDevice(c->device));
  *out = nullptr;
  HIP_CHECK(c, hipHostMalloc(out, bytes ? bytes : 1, 0));
  return NPR_OK;
}

npr_status npr_host_free(npr_ctx *c, void *p) {
  if (!c) return NPR_ERR_ARG;
  if (p) HIP_CHECK(c, hipHostFree(p));
  return NPR_OK;
}

// Shared body of records_parse / capture_file_parse / parse_extract.
static npr_status host_parse(npr_ctx *c, const uint8_t *in, size_t len, uint64_t start, npr_endianness e,
                             npr_record *out_recs, size_t rec_cap, size_t *n_records, npr_flow *out_flows,
                             npr_flow_v6 *out_v6, size_t flow_cap, size_t *n_flows, size_t *consumed) {
  HIP_CHECK(c, hipSetDevice(c->device));
  // flows only, a capture of several chunks: copies overlapped with the parse
  const bool streamed = !out_recs && c->resident && c->stream_chunk && len > start &&
                        len - start > 2 * c->stream_chunk && len > start + 16;
  npr_status st = streamed ? NPR_OK : stage_input(c, in, len);
  if (st) return st;
  const uint64_t max_rec = len > start ? (len - start) / 16 + 1 : 1;
  const uint64_t rcap = std::min<uint64_t>(rec_cap, max_rec);
  const uint64_t fcap = std::min<uint64_t>(flow_cap, max_rec);
  npr_dev_outputs o{};
  if (out_recs && rcap) {
    if ((st = ensure(c, c->recs, rcap * sizeof(npr_record)))) return st;
    o.records = (npr_record *)c->recs.p;
    o.record_cap = rcap;
  }
  if (out_flows && fcap) {
    if ((st = ensure(c, c->flows, fcap * sizeof(npr_flow)))) return st;
    o.flows = (npr_flow *)c->flows.p;
    o.flow_cap = fcap;
    if (out_v6) {
      if ((st = ensure(c, c->flows_v6, fcap * sizeof(npr_flow_v6)))) return st;
      o.flows_v6 = (npr_flow_v6 *)c->flows_v6.p;
    }
  }
  o.summary = c->summary;
  if ((st = streamed ? stream_parse(c, in, len, start, e, &o) : npr_dev_parse_extract(c, c->in.p, len, start, e, &o, c->stream)))
    return st;
  npr_summary sm;
  st = npr_dev_check(c, &o, c->stream, &sm);
  if (st && st != NPR_ERR_CAPACITY) return st;
  if (streamed && sm.consumed + 16 <= len) {  // the chain stopped at a complete record: one longer
    const uint64_t incl = rd_u32(in + sm.consumed + 8, e == NPR_BIG);  // than a chunk; parse again whole
    if (incl <= len - sm.consumed - 16) {
      if ((st = npr_dev_parse_extract(c, c->in.p, len, start, e, &o, c->stream))) return st;
      st = npr_dev_check(c, &o, c->stream, &sm);
      if (st && st != NPR_ERR_CAPACITY) return st;
    }
  }
  const uint64_t nr = std::min<uint64_t>(sm.n_records, rcap);
  const uint64_t nf = std::min<uint64_t>(sm.n_flows, fcap);
  if (o.records && nr)
    HIP_CHECK(c, hipMemcpyAsync(out_recs, o.records, nr * sizeof(npr_record), hipMemcpyDeviceToHost, c->stream));
  if (o.flows && nf) {  // device flows are right-aligned; the host API returns them left-aligned
    HIP_CHECK(c, hipMemcpyAsync(out_flows, o.flows + (fcap - nf), nf * sizeof(npr_flow), hipMemcpyDeviceToHost,
                                c->stream));
    if (o.flows_v6)
      HIP_CHECK(c, hipMemcpyAsync(out_v6, o.flows_v6 + (fcap - nf), nf * sizeof(npr_flow_v6),
                                  hipMemcpyDeviceToHost, c->stream));
  }
  HIP_CHECK(c, hipStreamSynchronize(c->stream));
  if (n_records) *n_records = sm.n_records;
  if (n_flows) *n_flows = sm.n_flows;
  if (consumed) *consumed = sm.consumed;
  if ((out_recs && sm.n_records > rec_cap) || (out_flows && sm.n_flows > flow_cap))
    return fail(c, NPR_ERR_CAPACITY, "output capacity exceeded");
  return NPR_OK;
}

npr_status npr_records_parse(npr_ctx *c, const uint8_t *in, size_t len, npr_endianness e, npr_record *out,
                             size_t cap, size_t *n_out, size_t *consumed) {
  if (!c || (!in && len)) return fail(c, NPR_ERR_ARG, "null argument");
  return host_parse(c, in, len, 0, e, out, out ? cap : 0, n_out, nullptr, nullptr, 0, nullptr, consumed);
}

npr_status npr_capture_file_parse(npr_ctx *c, const uint8_t *in, size_t len, npr_global_header *hdr,
                                  npr_record *out, size_t cap, size_t *n_out, size_t *consumed) {
  if (!c || !hdr || (!in && len)) return fail(c, NPR_ERR_ARG, "null argument");
  npr_status st = npr_global_header_parse(in, len, hdr, nullptr);  // file.rs:18
  if (st) return st;
  return host_parse(c, in, len, 24, (npr_endianness)hdr->endianness, out, out ? cap : 0, n_out, nullptr,
                    nullptr, 0, nullptr, consumed);
}

npr_status npr_parse_extract(npr_ctx *c, const uint8_t *in, size_t len, npr_global_header *hdr, npr_record *recs,
                             size_t rec_cap, size_t *n_records, npr_flow *out, npr_flow_v6 *out_v6, size_t flow_cap,
                             size_t *n_flows, size_t *consumed) {
  if (!c || !hdr || (!in && len)) return fail(c, NPR_ERR_ARG, "null argument");
  npr_status st = npr_global_header_parse(in, len, hdr, nullptr);
  if (st) return st;
  return host_parse(c, in, len, 24, (npr_endianness)hdr->endianness, recs, recs ? rec_cap : 0, n_records, out,
                    out_v6, out ? flow_cap : 0, n_flows, consumed);
}

npr_status npr_extract_flows(npr_ctx *c, const uint8_t *in, size_t len, const npr_record *records, size_t n,
                             npr_flow *flows, npr_flow_v6 *flows_v6, uint8_t *status) {
  if (!c || (!in && len) || (!records && n)) return fail(c, NPR_ERR_ARG, "null argument");
  HIP_CHECK(c, hipSetDevice(c->device));
  npr_status st;
  if (n && small_call(len, n)) {  // one launch over the page-locked arena
    uint8_t *ar = nullptr;
    uint64_t ro = 0, oo = 0;
    const uint64_t fo = 0, vo = a16(n * sizeof(npr_flow)), so = vo + a16(n * sizeof(npr_flow_v6));
    if ((st = small_arena(c, in, len, records, n, so + n, ar, ro, oo))) return st;
    if (flows_v6) memset(ar + oo + vo, 0, n * sizeof(npr_flow_v6));  // the kernel writes IPv6 flows' side rows only
    HIP_CHECK(c, npr::launch_extract_dense(ar, len, (const npr_record *)(ar + ro), n, (uint32_t *)(ar + oo + fo),
                                           (uint32_t *)(ar + oo + vo), ar + oo + so, c->stream));
    HIP_CHECK(c, hipStreamSynchronize(c->stream));
    if (flows) memcpy(flows, ar + oo + fo, n * sizeof(npr_flow));
    if (flows_v6) memcpy(flows_v6, ar + oo + vo, n * sizeof(npr_flow_v6));
    if (status) memcpy(status, ar + oo + so, n);
    return NPR_OK;
  }
  st = stage_input(c, in, len);
  if (st) return st;
  if (n == 0) return NPR_OK;
  if ((st = ensure(c, c->recs, n * sizeof(npr_record)))) return st;
  if ((st = ensure(c, c->flows, n * sizeof(npr_flow)))) return st;
  if ((st = ensure(c, c->flows_v6, n * sizeof(npr_flow_v6)))) return st;
  if ((st = ensure(c, c->status, n))) return st;
  HIP_CHECK(c, hipMemcpyAsync(c->recs.p, records, n * sizeof(npr_record), hipMemcpyHostToDevice, c->stream));
  // the host call's side table is dense (zero rows for non-IPv6 records): the kernel writes IPv6 flows' rows only
  if (flows_v6) HIP_CHECK(c, hipMemsetAsync(c->flows_v6.p, 0, n * sizeof(npr_flow_v6), c->stream));
  HIP_CHECK(c, npr::launch_extract_dense((const uint8_t *)c->in.p, len, (const npr_record *)c->recs.p, n,
                                         (uint32_t *)c->flows.p, flows_v6 ? (uint32_t *)c->flows_v6.p : nullptr,
                                         (uint8_t *)c->status.p, c->stream));
  if (flows) HIP_CHECK(c, hipMemcpyAsync(flows, c->flows.p, n * sizeof(npr_flow), hipMemcpyDeviceToHost, c->stream));
  if (flows_v6)
    HIP_CHECK(c, hipMemcpyAsync(flows_v6, c->flows_v6.p, n * sizeof(npr_flow_v6), hipMemcpyDeviceToHost, c->stream));
  if (status) HIP_CHECK(c, hipMemcpyAsync(status, c->status.p, n, hipMemcpyDeviceToHost, c->stream));
  HIP_CHECK(c, hipStreamSynchronize(c->stream));
  return NPR_OK;
}

npr_status npr_flow_details(npr_ctx *c, const uint8_t *in, size_t len, const npr_record *records, size_t n,
                            uint8_t *status, uint64_t *detail) {
  if (!c || (!in && len) || (!records && n)) return fail(c, NPR_ERR_ARG, "null argument");
  HIP_CHECK(c, hipSetDevice(c->device));
  npr_status st;
  if (n && small_call(len, n)) {  // one launch over the page-locked arena
    uint8_t *ar = nullptr;
    uint64_t ro = 0, oo = 0;
    const uint64_t so = a16(n * sizeof(uint64_t));  // details first (8-B aligned), then status
    if ((st = small_arena(c, in, len, records, n, so + n, ar, ro, oo))) return st;
    HIP_CHECK(c, npr::launch_flow_detail(ar, len, (const npr_record *)(ar + ro), n, ar + oo + so,
                                         (uint64_t *)(ar + oo), c->stream));
    HIP_CHECK(c, hipStreamSynchronize(c->stream));
    if (status) memcpy(status, ar + oo + so, n);
    if (detail) memcpy(detail, ar + oo, n * sizeof(uint64_t));
    return NPR_OK;
  }
  st = stage_input(c, in, len);
  if (st) return st;
  if (n == 0) return NPR_OK;
  if ((st = ensure(c, c->recs, n * sizeof(npr_record)))) return st;
  if ((st = ensure(c, c->status, n))) return st;
  if ((st = ensure(c, c->flows2, n * sizeof(uint64_t)))) return st;  // the details
  HIP_CHECK(c, hipMemcpyAsync(c->recs.p, records, n * sizeof(npr_record), hipMemcpyHostToDevice, c->stream));
  HIP_CHECK(c, npr::launch_flow_detail((const uint8_t *)c->in.p, len, (const npr_record *)c->recs.p, n,
                                       (uint8_t *)c->status.p, (uint64_t *)c->flows2.p, c->stream));
  if (status) HIP_CHECK(c, hipMemcpyAsync(status, c->status.p, n, hipMemcpyDeviceToHost, c->stream));
  if (detail) HIP_CHECK(c, hipMemcpyAsync(detail, c->flows2.p, n * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
  HIP_CHECK(c, hipStreamSynchronize(c->stream));
  return NPR_OK;
}

npr_status npr_vxlan_flows(npr_ctx *c, const uint8_t *in, size_t len, const npr_record *records, size_t n,
                           uint32_t dst_port, npr_endianness e, npr_flow *flows, npr_flow_v6 *flows_v6, uint8_t *status,
                           uint32_t *vni) {
  if (!c || (!in && len) || (!records && n)) return fail(c, NPR_ERR_ARG, "null argument");
  if (dst_port > 0xffffu) return fail(c, NPR_ERR_ARG, "dst_port must be 0..65535");
  HIP_CHECK(c, hipSetDevice(c->device));
  npr_status st = stage_input(c, in, len);
  if (st) return st;
  if (n == 0) return NPR_OK;
  if ((st = ensure(c, c->recs, n * sizeof(npr_record)))) return st;
  if ((st = ensure(c, c->flows, n * sizeof(npr_flow)))) return st;
  if ((st = ensure(c, c->flows_v6, n * sizeof(npr_flow_v6)))) return st;
  if ((st = ensure(c, c->status, n))) return st;
  if ((st = ensure(c, c->flows2, n * sizeof(uint32_t)))) return st;  // the VNIs
  HIP_CHECK(c, hipMemcpyAsync(c->recs.p, records, n * sizeof(npr_record), hipMemcpyHostToDevice, c->stream));
  HIP_CHECK(c, npr::launch_vxlan_flows((const uint8_t *)c->in.p, len, (const npr_record *)c->recs.p, n, dst_port,
                                       e == NPR_BIG, (uint32_t *)c->flows.p, (uint32_t *)c->flows_v6.p,
                                       (uint8_t *)c->status.p, (uint32_t *)c->flows2.p, c->stream));
  if (flows) HIP_CHECK(c, hipMemcpyAsync(flows, c->flows.p, n * sizeof(npr_flow), hipMemcpyDeviceToHost, c->stream));
  if (flows_v6)
    HIP_CHECK(c, hipMemcpyAsync(flows_v6, c->flows_v6.p, n * sizeof(npr_flow_v6), hipMemcpyDeviceToHost, c->stream));
  if (status) HIP_CHECK(c, hipMemcpyAsync(status, c->status.p, n, hipMemcpyDeviceToHost, c->stream));
  if (vni) HIP_CHECK(c, hipMemcpyAsync(vni, c->flows2.p, n * sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
  HIP_CHECK(c, hipStreamSynchronize(c->stream));
  return NPR_OK;
}

npr_status npr_convert_records(npr_ctx *c, const uint8_t *in, size_t len, const npr_record *records, size_t n,
                               npr_flow *out, npr_flow_v6 *out_v6, size_t cap, size_t *n_out) {
  if (!c || (!in && len) || (!records && n)) return fail(c, NPR_ERR_ARG, "null argument");
  HIP_CHECK(c, hipSetDevice(c->device));
  npr_status st;
  if (n == 0) {
    if (n_out) *n_out = 0;
    return NPR_OK;
  }
  if (!small_call(len, n) && (st = stage_input(c, in, len))) return st;
  const uint64_t ocap = std::min<uint64_t>(cap, n);
  if (small_call(len, n)) {  // one launch over the page-locked arena (rows, side rows, total)
    uint8_t *ar = nullptr;
    uint64_t ro = 0, oo = 0;
    const uint64_t vo = a16(std::max<uint64_t>(ocap, 1) * sizeof(npr_flow));
    const uint64_t to = vo + a16(std::max<uint64_t>(ocap, 1) * sizeof(npr_flow_v6));
    if ((st = small_arena(c, in, len, records, n, to + 8, ar, ro, oo))) return st;
    uint64_t *total = (uint64_t *)(ar + oo + to);
    if ((st = convert_launch(c, ar, len, (const npr_record *)(ar + ro), n, (npr_flow *)(ar + oo),
                             out_v6 ? (npr_flow_v6 *)(ar + oo + vo) : nullptr, ocap, total, c->stream)))
      return st;
    HIP_CHECK(c, hipStreamSynchronize(c->stream));
    const uint64_t tot = *(volatile uint64_t *)total;
    if (tot == ~0ull) return fail(c, NPR_ERR_TIMEOUT, "convert_records did not complete (look-back timed out)");
    const uint64_t k = std::min<uint64_t>(tot, ocap);
    if (k && out) memcpy(out, ar + oo, k * sizeof(npr_flow));
    if (k && out_v6) memcpy(out_v6, ar + oo + vo, k * sizeof(npr_flow_v6));
    if (n_out) *n_out = tot;
    if (tot > cap) return fail(c, NPR_ERR_CAPACITY, "output capacity exceeded");
    return NPR_OK;
  }
  if ((st = ensure(c, c->recs, n * sizeof(npr_record)))) return st;
  if ((st = ensure(c, c->flows2, std::max<uint64_t>(ocap, 1) * sizeof(npr_flow)))) return st;
  if ((st = ensure(c, c->flows2_v6, std::max<uint64_t>(ocap, 1) * sizeof(npr_flow_v6)))) return st;
  HIP_CHECK(c, hipMemcpyAsync(c->recs.p, records, n * sizeof(npr_record), hipMemcpyHostToDevice, c->stream));
  uint64_t *total = (uint64_t *)c->summary;  // scratch word
  if ((st = convert_launch(c, c->in.p, len, (const npr_record *)c->recs.p, n, (npr_flow *)c->flows2.p,
                           out_v6 ? (npr_flow_v6 *)c->flows2_v6.p : nullptr, ocap, total, c->stream)))
    return st;
  uint64_t tot = 0;
  HIP_CHECK(c, hipMemcpyAsync(&tot, total, 8, hipMemcpyDeviceToHost, c->stream));
  HIP_CHECK(c, hipStreamSynchronize(c->stream));
  if (tot == ~0ull) return fail(c, NPR_ERR_TIMEOUT, "convert_records did not complete (look-back timed out)");
  const uint64_t k = std::min<uint64_t>(tot, ocap);
  if (k) {
    if (out) HIP_CHECK(c, hipMemcpyAsync(out, c->flows2.p, k * sizeof(npr_flow), hipMemcpyDeviceToHost, c->stream));
    if (out_v6)
      HIP_CHECK(c, hipMemcpyAsync(out_v6, c->flows2_v6.p, k * sizeof(npr_flow_v6), hipMemcpyDeviceToHost, c->stream));
    HIP_CHECK(c, hipStreamSynchronize(c->stream));
  }
  if (n_out) *n_out = tot;
  if (tot > cap) return fail(c, NPR_ERR_CAPACITY, "output capacity exceeded");
  return NPR_OK;
}

}  // extern "C"
