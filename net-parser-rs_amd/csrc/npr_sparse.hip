// npr_sparse.hip — the SPARSE record walk: flows-only parses of captures whose
// records are long (SURVEY.md §8 d, C3: 16 + min(incl, 64) bytes of a ~800-B record are all the
// path needs).  It replaces, on the device, the same reference paths as the resident pass:
//   PcapRecords::parse loop        src/record.rs:21-54   (offset_{k+1} = offset_k + 16 + incl_len_k)
//   PcapRecord::parse              src/record.rs:102-121
//   FlowExtraction::extract_flow   src/flow/mod.rs:20-48 (decode_fast / decode<>)
//   flow::convert_records          src/flow/mod.rs:101-123 (reverse-order rows of the Ok flows)
// without streaming the payloads through the chip:
//   k_sparse_walk  [start, stop) is cut into lane ranges of `span` bytes, one per LANE.  A lane
//     speculates its first record (a zero-byte mask over 112-B windows screens every byte offset
//     for the high bytes of incl_len / orig_len, survivors are checked on their header and two
//     chained headers), then hops header to header: each record is ONE 112-B window (the header
//     and the decoder's bytes) loaded straight into registers, the next record's window in flight
//     while this one decodes.  Ok flows go to the lane's slots; each 64-lane group (one wave)
//     publishes its aggregate under the chain-consistency monoid.
//   k_sparse_scan  one workgroup scans the group aggregates from the anchor (start, or the previous
//     link's summary).  Groups whose speculation is contradicted are resolved from their incoming
//     chain position (lanes a record spans are marked passed over, mis-speculated lanes re-walked
//     exactly, all such lanes of all flagged groups at once, to a fixed point) and the scan repeats
//     until every link is exact; then it writes each group's exact prefix and the summary.
//   k_sparse_rows  one workgroup per group moves its lanes' slots to their convert_records rows
//     (destination order: whole-line stores); a lane with more Ok flows than slots walks the rest
//     again from its first slotless record.
// A wrong speculation costs a re-walk, never a result: the summary and rows are the serial chain's.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "npr_decode.hpp"
#include "npr_device.hpp"
#include "npr_internal.hpp"

namespace npr {
namespace {

constexpr int kSpBlock = 256;                // walk / rows kernels: four 64-lane groups per workgroup
constexpr int kSpWin = 112;                  // a record's full window: [header & ~15, +112) (80 B in the fast path)
constexpr int kSpRow = kSpWin / 4 + 1;       // a lane's LDS row (odd dword stride: conflict-free)
constexpr int kScanThreads = 256;            // k_sparse_scan: one workgroup (at 1024 threads its serial
                                             // paths spilled to scratch: 37 us for the fast path alone)
constexpr int kResolvers = 256;              // groups resolved per scan round
constexpr uint32_t kScanWin = 2048;          // groups staged in LDS at a time by the scan's fast path
constexpr uint32_t kTasks = 2048;            // lane re-walks queued per resolve pass (more wait for the next pass)
static_assert(15 + 16 + 17 * 4 + 4 <= kSpWin, "header + decode_fast's 68-B window fit the row at any misalignment");

typedef const __attribute__((address_space(1))) u32x4 *gv4_t;  // global (not flat) loads: vmcnt only
constexpr int kSpWords = kSpWin / 4;  // a record's window in registers: words [4 k, 4 k + 4) = chunk k

__device__ __forceinline__ const uint8_t *align16(const uint8_t *p) {
  return (const uint8_t *)((uintptr_t)p & ~(uintptr_t)15);
}
__device__ __noinline__ uint32_t tail_dword(const uint8_t *p, const uint8_t *end) {
  uint32_t x = 0;
  for (int b = 0; b < 4; ++b)
    if (p + b < end) x |= (uint32_t)p[b] << (8 * b);
  return x;
}
// a 4-aligned dword of the input, bytes at or past `end` read as 0
__device__ __forceinline__ uint32_t dword_at(const uint8_t *p, const uint8_t *end) {
  return p + 4 <= end ? *reinterpret_cast<const uint32_t *>(p) : (p < end ? tail_dword(p, end) : 0u);
}
// chunks [K0, K1) of the window at a16 (16 B each) into w[4 K0 .. 4 K1): dwordx4 loads issued back
// to back, or dword by dword for the buffer's last bytes
template <int K0, int K1>
__device__ __forceinline__ void load_chunks(const uint8_t *a16, const uint8_t *end, uint32_t (&w)[kSpWords]) {
  if (a16 + 16 * K1 <= end) {
    const gv4_t s = (gv4_t)(uintptr_t)a16;
#pragma unroll
    for (int k = K0; k < K1; ++k) {
      const u32x4 v = s[k];
#pragma unroll
      for (int e = 0; e < 4; ++e) w[4 * k + e] = v[e];
    }
  } else {
#pragma unroll
    for (int k = K0; k < K1; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e) w[4 * k + e] = dword_at(a16 + 16 * k + 4 * e, end);
  }
}
// lanes whose bit of m is set: a, the others: b
__device__ __forceinline__ uint32_t vsel(uint64_t m, uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(b), "v"(a), "s"(m));
  return r;
}
// Window words at a per-lane byte offset, with no register indexing: word (off >> 2) + j is chosen
// by two selects (off & 8, off & 4) and shifted by off & 3 (v_alignbyte).
// a[k] = window bytes [base + off + 4k, +4) for k < K (base a multiple of 4, off < 16)
template <int BASE, int K, int N>
__device__ __forceinline__ void words_at(const uint32_t (&w)[kSpWords], uint32_t off, uint32_t (&a)[N]) {
  static_assert(BASE / 4 + K + 4 <= kSpWords, "window words");
  // (v_cndmask by hand: a C select between two elements of one array is folded into an indexed
  // access, which puts the array in scratch memory)
  const uint64_t b1 = __ballot((off & 8u) != 0), b0 = __ballot((off & 4u) != 0);
  const uint32_t sh = off & 3u;
  uint32_t S[K + 2], T[K + 1];
#pragma unroll
  for (int m = 0; m < K + 2; ++m) S[m] = vsel(b1, w[BASE / 4 + 2 + m], w[BASE / 4 + m]);
#pragma unroll
  for (int m = 0; m < K + 1; ++m) T[m] = vsel(b0, S[m + 1], S[m]);
#pragma unroll
  for (int k = 0; k < K; ++k) a[k] = __builtin_amdgcn_alignbyte(T[k + 1], T[k], sh);
}

// payload reader over a lane's staged window, global bytes (bounds-checked) past it
struct SpRowReader {
  const uint32_t *w;  // the lane's LDS row
  uint32_t rel;       // payload start inside the row
  const uint8_t *g;   // payload start in global memory
  uint64_t gavail;    // bytes of the input from the payload start
  __device__ __forceinline__ uint32_t le32(uint32_t q) const {
    const uint64_t a = (uint64_t)rel + q;
    if (a + 4 <= (uint64_t)kSpWin) return lds_le32(w, (uint32_t)a);
    return u8g(q) | (u8g(q + 1) << 8) | (u8g(q + 2) << 16) | (u8g(q + 3) << 24);
  }
  __device__ __forceinline__ uint32_t u8(uint32_t q) const {
    const uint64_t a = (uint64_t)rel + q;
    if (a < (uint64_t)kSpWin) return ((const uint8_t *)w)[a];
    return u8g(q);
  }
  __device__ __forceinline__ uint32_t u8g(uint32_t q) const { return (uint64_t)q < gavail ? g[q] : 0u; }
};

// ---- lane geometry and the monoid over lanes --------------------------------------------------
__device__ __forceinline__ uint64_t lane_lo(const SparseParams &sp, uint64_t i) { return sp.kp.start + i * sp.span; }
__device__ __forceinline__ uint64_t sp_end(const SparseParams &sp, int64_t i) {  // end of lane i (i = -1: start)
  const uint64_t e = sp.kp.start + (uint64_t)(i + 1) * sp.span;
  return e < sp.kp.stop ? e : sp.kp.stop;
}

// X then Y (Y's lanes follow X's), the chain-consistency monoid of the resident pass (combine())
// over lane ranges.  A contradicted link records the lowest mis-speculated lane and then carries
// Y's speculated exit on (the scan resolves contradictions group by group, each from the chain
// position the groups before it deliver, so the propagation must not stop at the first one).
__device__ __forceinline__ Seg sp_cat(const SparseParams &sp, const Seg &X, const Seg &Y) {
  Seg r = X;
  r.last = Y.last;
  if (X.exit < sp_end(sp, X.last)) return r;   // the chain ended inside X (Q3): Y is moot
  if (X.exit >= sp_end(sp, Y.last)) return r;  // one record spans all of Y: no record starts there
  const bool bad = X.exit != Y.entry;
  r.exit = Y.exit;
  r.cnt = X.cnt + Y.cnt;
  r.ok = X.ok + Y.ok;
  if (X.valid && (bad || !Y.valid)) {
    r.valid = 0;
    r.mism = bad ? Y.first : Y.mism;
  }
  return r;
}
// lane li's segment (a lane without a speculated start: its range end as the exit guess)
__device__ __forceinline__ Seg lane_seg(const SparseParams &sp, uint64_t li, const SparseLane &L) {
  Seg s;
  s.entry = L.entry;
  s.exit = L.entry == kNone ? sp_end(sp, (int64_t)li) : L.exit;
  s.cnt = L.cnt;
  s.ok = L.ok;
  s.first = s.last = (int64_t)li;
  s.mism = -1;
  s.valid = 1;
  s.spare = 0;
  return s;
}
__device__ __forceinline__ void put_seg(uint64_t *d, const Seg &s) {
  d[0] = s.entry;
  d[1] = s.exit;
  d[2] = s.cnt;
  d[3] = s.ok;
  d[4] = (uint64_t)s.first;
  d[5] = (uint64_t)s.last;
  d[6] = (uint64_t)s.mism;
  d[7] = s.valid;
}
// a group aggregate's link fields into the scan's arrays (group g of ng)
__device__ __forceinline__ void put_lite(const SparseParams &sp, uint32_t g, const Seg &s) {
  sp.lite[g] = s.entry;
  sp.lite[sp.ngroups + g] = s.exit;
  sp.lite[2 * (uint64_t)sp.ngroups + g] = (s.cnt & 0xffffffffull) | ((s.ok & 0x7fffffffull) << 32) | ((uint64_t)(s.valid != 0) << 63);
}
__device__ __forceinline__ Seg get_seg(const uint64_t *d) {
  Seg s;
  s.entry = d[0];
  s.exit = d[1];
  s.cnt = d[2];
  s.ok = d[3];
  s.first = (int64_t)d[4];
  s.last = (int64_t)d[5];
  s.mism = (int64_t)d[6];
  s.valid = (uint32_t)d[7];
  s.spare = 0;
  return s;
}

// ---- speculation ------------------------------------------------------------------------------
// bit i: byte i of d is zero
__device__ __forceinline__ uint32_t zmask4(uint32_t d) {
  const uint32_t z = ~(((d & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | d | 0x7F7F7F7Fu);
  return ((z >> 7) * 0x01020408u) >> 24;
}
// the 16-B record header at file offset q (any alignment) in the capture's byte order
__device__ __forceinline__ void hdr_at(const ParseParams &kp, uint64_t q, uint32_t (&h)[4]) {
  const uint8_t *end = kp.buf + kp.len, *p = kp.buf + q;
  const uint8_t *a4 = (const uint8_t *)((uintptr_t)p & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)((uintptr_t)p & 3u);
  uint32_t x[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) x[k] = dword_at(a4 + 4 * k, end);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t v = __builtin_amdgcn_alignbyte(x[k + 1], x[k], sh);
    h[k] = kp.big ? __builtin_bswap32(v) : v;
  }
}
// Does the chain from a candidate (its header: ts, incl at q0) go on plausibly for two more
// headers?  Headers past the input (an exact end, a truncated tail) cannot be checked and pass
// (chain_grade()'s "weak" starts).  A heuristic only: the scan verifies every start exactly.
__device__ bool chain_ok(const ParseParams &kp, const SpecCtx &sc, uint64_t q0, uint32_t ts, uint32_t incl) {
  uint64_t q = q0 + 16 + incl;
  for (int hop = 0; hop < 2; ++hop) {
    if (q >= kp.len || kp.len - q < 16) return true;
    uint32_t h[4];
    hdr_at(kp, q, h);
    if (!plaus(sc, h[0], h[1], h[2], h[3]) || h[0] - ts + kTsWindow > 2u * kTsWindow) return false;
    if (kp.len - q - 16 < h[2]) return true;
    ts = h[0];
    q += 16 + (uint64_t)h[2];
  }
  return true;
}
// The first plausible record start in [lo, hi), kNone if none.  Windows of 64 candidate offsets
// (80 B loaded): every candidate needs the high bytes of incl_len and orig_len zero (both <= 2^18),
// which one zero-byte mask over the window screens at once; the survivors are checked on their
// own header (plaus(), the payload fits) and their chain (chain_ok()), in offset order.
__device__ __forceinline__ uint64_t lane_speculate(const ParseParams &kp, const SpecCtx &sc, uint64_t lo, uint64_t hi,
                                                   uint32_t *row) {
  const uint8_t *end = kp.buf + kp.len;
  const uint32_t za = kp.big ? 8u : 11u, zb = kp.big ? 12u : 15u;  // the zero high bytes of incl / orig
  uint64_t c = lo;
  const uint8_t *a16 = align16(kp.buf + c);
  uint32_t w[kSpWords], wn[kSpWords];
  load_chunks<0, 5>(a16, end, w);
  while (c < hi) {
    const uint32_t r0 = (uint32_t)((uintptr_t)(kp.buf + c) & 15u);  // candidates r0 .. 63 of the window
    const uint64_t cn = c + (64u - r0);
    const bool more = cn < hi;
    if (more) load_chunks<0, 5>(a16 + 64, end, wn);  // in flight while this window is screened
    uint64_t z0 = 0, z1 = 0;  // bit b: window byte b is zero (b < 80)
#pragma unroll
    for (int i = 0; i < 16; ++i) z0 |= (uint64_t)zmask4(w[i]) << (4 * i);
#pragma unroll
    for (int i = 0; i < 4; ++i) z1 |= (uint64_t)zmask4(w[16 + i]) << (4 * i);
    uint64_t m = ((z0 >> za) | (z1 << (64u - za))) & ((z0 >> zb) | (z1 << (64u - zb))) & ~((1ull << r0) - 1ull);
    if (__ballot(m != 0ull)) {
      if (m) {
#pragma unroll
        for (int j = 0; j < 20; ++j) row[j] = w[j];
      }
      while (m) {
        const uint32_t p = (uint32_t)__builtin_ctzll(m);
        m &= m - 1;
        const uint64_t q = c + (p - r0);
        if (q >= hi) return kNone;
        uint32_t h[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t v = lds_le32(row, p + 4u * (uint32_t)k);
          h[k] = kp.big ? __builtin_bswap32(v) : v;
        }
        const uint64_t avail = kp.len - q;
        if (avail >= 16 && plaus(sc, h[0], h[1], h[2], h[3]) && avail - 16 >= h[2] && chain_ok(kp, sc, q, h[0], h[2]))
          return q;
      }
    }
    if (!more) break;
    c = cn;
    a16 += 64;
#pragma unroll
    for (int j = 0; j < 20; ++j) w[j] = wn[j];
  }
  return kNone;
}

// ---- the walk -----------------------------------------------------------------------------------
// One record's status + flow from its window (w[0..19] = 80 B from the header's 16-B aligned
// start: the header and payload bytes [0, 48) at any alignment).  The IPv4 shapes decode from
// registers; IPv6 frames take two more chunks (payload bytes up to 68); any other shape stages
// the window in the lane's LDS row and runs the general decode<> (bytes past it from global).
__device__ __forceinline__ uint32_t rec_decode(const ParseParams &kp, uint32_t *row, const uint8_t *pp, uint64_t avail,
                                               uint32_t rel, uint32_t incl, uint32_t (&w)[kSpWords], FlowWords &f) {
  const uint8_t *end = kp.buf + kp.len, *a16 = align16(pp);
  uint32_t a[17];
  words_at<16, 12>(w, rel, a);
#pragma unroll
  for (int k = 12; k < 17; ++k) a[k] = 0u;
  const uint32_t etype = ((a[3] & 0xffu) << 8) | ((a[3] >> 8) & 0xffu);
  const bool six = etype == 0x86ddu;
  bool full = false;
  if (__ballot(six)) {
    if (six) {
      load_chunks<5, 7>(a16, end, w);
      words_at<16, 17>(w, rel, a);
      full = true;
    }
  }
  uint32_t st = decode_fast_core<true, true>(a, incl, f, true);
  if (__ballot(st == 0xffu)) {
    if (st == 0xffu) {
      if (!full) load_chunks<5, 7>(a16, end, w);
#pragma unroll
      for (int j = 0; j < kSpWords; ++j) row[j] = w[j];
      const SpRowReader r{row, rel + 16u, pp + 16, avail - 16};
      st = decode<true>(r, incl, f);
    }
  }
  return st;
}

// The serial chain (src/record.rs:30-49) from `pos` while records start before hi: one 80-B
// window per record (the next record's in flight while this one decodes); every record's status
// and flow go to sink(record offset, ok, flow words).  Returns the exit: the first chain offset
// >= hi, or (chain END, Q3) the offset of the first incomplete record.
template <class Sink>
__device__ __forceinline__ uint64_t lane_walk(const ParseParams &kp, uint32_t *row, uint64_t pos, uint64_t hi,
                                              uint32_t &cnt, Sink &sink) {
  if (pos >= hi) return pos;
  const uint8_t *end = kp.buf + kp.len;
  uint32_t w[kSpWords];
  load_chunks<0, 5>(align16(kp.buf + pos), end, w);
  for (;;) {
    const uint8_t *pp = kp.buf + pos;
    const uint32_t rel = (uint32_t)((uintptr_t)pp & 15u);
    uint32_t h[1];
    words_at<8, 1>(w, rel, h);  // incl_len
    const uint32_t incl = kp.big ? __builtin_bswap32(h[0]) : h[0];
    const uint64_t avail = kp.len - pos;
    if (avail < 16 || avail - 16 < incl) break;  // Err(Incomplete): the chain stops here (:37-45)
    const uint64_t next = pos + 16 + incl;
    const bool more = next < hi;
    uint32_t wn[kSpWords];
    if (more) load_chunks<0, 5>(align16(kp.buf + next), end, wn);
    FlowWords f{};
    const uint32_t st = rec_decode(kp, row, pp, avail, rel, incl, w, f);
    sink(pos, st == NPR_FLOW_OK, f);
    ++cnt;
    pos = next;
    if (!more) break;
#pragma unroll
    for (int j = 0; j < 20; ++j) w[j] = wn[j];
  }
  return pos;
}

// a flow row as k_sparse_rows writes it (IPv6: word 0 holds the address block's payload offset)
__device__ __forceinline__ void row_image(const FlowWords &f, uint64_t p, u32x4 &r0, u32x4 &r1) {
  // a mask, not `v6 ? f.v6off : f.d[0]`: that select became a select of the two field addresses,
  // which kept the whole FlowWords in scratch memory (80-B private segment)
  const uint32_t m = 0u - ((f.d[6] >> 16) & NPR_FLOW_KIND_IPV6);
  r0 = u32x4{(f.v6off & m) | (f.d[0] & ~m), f.d[1], f.d[2], f.d[3]};
  r1 = u32x4{f.d[4], f.d[5], f.d[6] | ((uint32_t)(p & 0xffu) << 24), (uint32_t)(p >> 8)};
}
// every record of the lane into its slot (record k: slot k, while k < cap), Ok or not, so that a
// wave's store instructions write 64 consecutive slots whatever its lanes decoded (Ok flows only,
// densely, measured slower: lanes' slot indices drift apart at the first failed record, and C3's
// walk went 479 -> 505 us); two mask words of the Ok ones, 96 slots (64: C3's 61-record lanes
// overflowed into re-walks, rows 125 -> 111 us, walk 479 -> 489 us).
// A slot is 28 B in two arrays (npr_internal.hpp SparseParams::area / area_b): the 32-B row image
// less what the rows kernel rebuilds -- the record offset from the lane's start (18 bits; lane
// ranges are at most 256 KiB) and the flow kind's spare bits -- so each record's slot is one 16-B
// and one 12-B store, and a wave's pair of store instructions writes 1 KiB + 768 B contiguously.
// Slots and rows are plain (write-back) stores: non-temporal and write-through (sc1, sc0 sc1)
// stores measured slower for both the scattered slot rows and the whole-line row blocks (DESIGN.md
// §3.8)
__device__ __forceinline__ void row_store(u32x4 *d, u32x4 v) { *d = v; }
// the 28-B slot image of a record at offset p of a lane starting at lo (p - lo < 2^18)
__device__ __forceinline__ void slot_image(const FlowWords &f, uint64_t p, uint64_t lo, u32x4 &a, uint32_t (&b)[3]) {
  const uint32_t m = 0u - ((f.d[6] >> 16) & NPR_FLOW_KIND_IPV6);  // (a mask: see row_image)
  a = u32x4{(f.v6off & m) | (f.d[0] & ~m), f.d[1], f.d[2], (f.d[3] >> 16) | (f.d[6] << 16)};
  b[0] = f.d[4];
  b[1] = f.d[5];
  b[2] = (f.d[3] & 0xfffu) | (((f.d[6] >> 16) & 3u) << 12) | ((uint32_t)(p - lo) << 14);
}
// the 32-B row of a slot (row_image's words) at file offset p
__device__ __forceinline__ void slot_row(u32x4 a, uint32_t b0, uint32_t b1, uint32_t b2, uint64_t p, u32x4 &r0,
                                         u32x4 &r1) {
  r0 = u32x4{a[0], a[1], a[2], (b2 & 0xfffu) | (a[3] << 16)};
  r1 = u32x4{b0, b1, (a[3] >> 16) | (((b2 >> 12) & 3u) << 16) | ((uint32_t)(p & 0xffu) << 24), (uint32_t)(p >> 8)};
}
struct AreaSink {
  u32x4 *slot_a;     // the lane's slot 0 in area (16-B units); NULL: count only
  uint32_t *slot_b;  // ... in area_b (dwords)
  uint64_t lo;       // the lane's start (slots keep offsets relative to it)
  uint32_t cap, n, okn;
  uint64_t okmask, okmask2, ovf;
  __device__ __forceinline__ void operator()(uint64_t p, bool ok, const FlowWords &f) {
    if (n < cap) {
      if (slot_a) {
        u32x4 a;
        uint32_t b[3];
        slot_image(f, p, lo, a, b);
        slot_a[(uint64_t)n * 64u] = a;
        uint32_t *d = slot_b + (uint64_t)n * 192u;
        d[0] = b[0];
        d[1] = b[1];
        d[2] = b[2];
      }
      if (n < 64) okmask |= (uint64_t)ok << n;
      else okmask2 |= (uint64_t)ok << (n - 64u);
    } else if (n == cap) {
      ovf = p;
    }
    ++n;
    okn += ok ? 1u : 0u;
  }
};
// the sink of lane l in group g: slot k at r = (g cap + k) 64 + l
__device__ __forceinline__ AreaSink area_sink(const SparseParams &sp, uint64_t g, uint32_t lane) {
  const uint64_t r0 = (uint64_t)g * sp.cap * 64u + lane;
  const bool fl = sp.kp.flows != nullptr;
  return AreaSink{fl ? reinterpret_cast<u32x4 *>(sp.area) + r0 : nullptr, fl ? sp.area_b + r0 * 3u : nullptr,
                  lane_lo(sp, g * 64u + lane), sp.cap, 0u, 0u, 0ull, 0ull, kNone};
}

// one output row (+ the IPv6 side row: its 32 address bytes re-read from the capture)
__device__ __forceinline__ void put_row(const ParseParams &kp, uint64_t o, u32x4 s0, u32x4 s1) {
  const bool v6 = (s1[2] & (NPR_FLOW_KIND_IPV6 << 16)) != 0;
  u32x4 *d = reinterpret_cast<u32x4 *>(kp.flows + o * 8);
  row_store(d, u32x4{v6 ? 0u : s0[0], s0[1], s0[2], s0[3]});
  row_store(d + 1, s1);
  if (v6 && kp.flows_v6) {
    const uint64_t p = (uint64_t)(s1[2] >> 24) | ((uint64_t)s1[3] << 8);
    const uint8_t *end = kp.buf + kp.len, *a = kp.buf + p + 16 + s0[0];
    const uint8_t *a4 = (const uint8_t *)((uintptr_t)a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)((uintptr_t)a & 3u);
    uint32_t x[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) x[k] = dword_at(a4 + 4 * k, end);
    u32x4 *d6 = reinterpret_cast<u32x4 *>(kp.flows_v6 + o * 8);
    d6[0] = u32x4{__builtin_amdgcn_alignbyte(x[1], x[0], sh), __builtin_amdgcn_alignbyte(x[2], x[1], sh),
                  __builtin_amdgcn_alignbyte(x[3], x[2], sh), __builtin_amdgcn_alignbyte(x[4], x[3], sh)};
    d6[1] = u32x4{__builtin_amdgcn_alignbyte(x[5], x[4], sh), __builtin_amdgcn_alignbyte(x[6], x[5], sh),
                  __builtin_amdgcn_alignbyte(x[7], x[6], sh), __builtin_amdgcn_alignbyte(x[8], x[7], sh)};
  }
}
// Ok flows of an overflowing lane from rank `rank` on, straight to their rows
struct RowSink {
  const ParseParams *kp;
  uint64_t base;  // the lane's first Ok flow's convert_records index
  uint32_t rank;
  __device__ __forceinline__ void operator()(uint64_t p, bool ok, const FlowWords &f) {
    if (!ok) return;
    const uint64_t g = base + rank++;
    if (g < kp->flow_cap) {
      u32x4 r0, r1;
      row_image(f, p, r0, r1);
      put_row(*kp, kp->flow_cap - 1 - g, r0, r1);
    }
  }
};

// =============================================================================================
// k_sparse_walk: one lane range per lane, one 64-lane group per wave
// =============================================================================================
__global__ __launch_bounds__(kSpBlock) __attribute__((amdgpu_waves_per_eu(4))) void k_sparse_walk(SparseParams sp) {
  __shared__ uint32_t rows[kSpBlock * kSpRow];
  const ParseParams &kp = sp.kp;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t g = blockIdx.x * (kSpBlock / 64) + (threadIdx.x >> 6);
  if (blockIdx.x == 0 && threadIdx.x == 0) *sp.ctl = 0;  // the rows kernel runs only after a new exact scan
  if (g >= sp.ngroups) return;  // (wave-uniform)
  const uint64_t li = (uint64_t)g * 64 + lane;
  const bool act = li < sp.nlanes;
  const SpecCtx sc = spec_ctx(kp, spec_ctx_load(kp));
  uint32_t *row = rows + threadIdx.x * kSpRow;
  const uint64_t lo = lane_lo(sp, li);
  const uint64_t hi = act ? sp_end(sp, (int64_t)li) : lo;
  uint64_t entry = kNone;
  if (act) {
    if (li == 0 && !(kp.flags & kFlagSpecStart) && !kp.prev) {
      entry = kp.start;
    } else {
      if (li == 0 && kp.prev) {  // a chained launch: where the previous one left the chain (checked by the scan)
        const uint64_t pc = kp.prev->consumed;
        if (pc >= lo && pc < hi) entry = pc;
      }
      if (entry == kNone) entry = lane_speculate(kp, sc, lo, hi, row);
    }
  }
  uint32_t cnt = 0;
  AreaSink sink = area_sink(sp, g, lane);
  uint64_t exit = 0;
  if (entry != kNone) exit = lane_walk(kp, row, entry, hi, cnt, sink);
  SparseLane L{entry, exit, cnt, sink.okn, sink.ovf, sink.okmask, sink.okmask2};
  if (act) sp.lanes[li] = L;
  // the group's aggregate: every link consistent (no END before the last lane, no lane a record
  // spans) -> two wave sums; otherwise the serial monoid
  const uint32_t size = sp.nlanes - (uint64_t)g * 64 < 64 ? (uint32_t)(sp.nlanes - (uint64_t)g * 64) : 64u;
  const Seg me = lane_seg(sp, li, L);
  const uint64_t prev_exit = shfl_up64(me.exit);
  const bool link_bad = act && (me.entry == kNone || (lane > 0 && me.entry != prev_exit));
  const bool end_mid = act && lane + 1 < size && me.exit < hi;
  Seg agg;
  if (__ballot(link_bad || end_mid) == 0ull) {
    uint64_t c = act ? me.cnt : 0, o = act ? me.ok : 0;
    for (int k = 32; k > 0; k >>= 1) {
      c += __shfl_xor(c, k);
      o += __shfl_xor(o, k);
    }
    agg.entry = rl64(me.entry, 0);
    agg.exit = rl64(me.exit, (int)size - 1);
    agg.cnt = c;
    agg.ok = o;
    agg.first = (int64_t)g * 64;
    agg.last = (int64_t)g * 64 + size - 1;
    agg.mism = -1;
    agg.valid = 1;
  } else {
    const uint64_t bnone = __ballot(me.entry == kNone);
    agg = lane_seg(sp, (uint64_t)g * 64, SparseLane{rl64(L.entry, 0), rl64(L.exit, 0), (uint32_t)__builtin_amdgcn_readlane((int)cnt, 0),
                                                     (uint32_t)__builtin_amdgcn_readlane((int)sink.okn, 0), 0, 0});
    for (uint32_t j = 1; j < size; ++j) {
      const SparseLane Lj{(bnone >> j) & 1ull ? kNone : rl64(L.entry, (int)j), rl64(L.exit, (int)j),
                          (uint32_t)__builtin_amdgcn_readlane((int)cnt, (int)j),
                          (uint32_t)__builtin_amdgcn_readlane((int)sink.okn, (int)j), 0, 0};
      agg = sp_cat(sp, agg, lane_seg(sp, (uint64_t)g * 64 + j, Lj));
    }
  }
  const uint64_t has = __ballot(act && entry != kNone);
  if (lane == 0) {
    put_seg(sp.aggs + (uint64_t)g * kSparseAggWords, agg);
    put_lite(sp, g, agg);
    sp.first_entry[g] = has ? rl64(entry, __builtin_ctzll(has)) : kNone;
  }
}

// =============================================================================================
// k_sparse_scan: one workgroup.  Rounds of: cut the groups into runs of plainly linked groups (each
// continues its predecessor's speculated chain exactly: those compose by sums), walk the runs from
// the anchor (one step per run: the group the incoming position lands in must start there); if
// nothing is contradicted, write every group's incoming chain state + the summary and stop; else
// resolve the contradicted groups (up to kResolvers at once, one thread each) and go again.  Each
// round settles the lowest contradiction exactly (its incoming position is exact), so rounds end.
// (A tree of composite aggregates is not exact here: a record that spans a composite's first group
// enters it past its entry, which only the lanes can settle.)
// =============================================================================================
__device__ __forceinline__ void fence_agent() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent"); }

// a group's plain link: it continues its predecessor's chain exactly (the predecessor did not end
// the chain, its exit lands in this group and is this group's first lane's entry, no contradiction
// inside): runs of plainly linked groups compose by sums
__device__ __forceinline__ bool plain_link(const SparseParams &sp, const Seg &p, const Seg &a) {
  return a.valid && p.exit >= sp_end(sp, p.last) && p.exit < sp_end(sp, a.last) && p.exit == a.entry;
}
// the fields of a group aggregate the fast path reads
struct Lite {
  uint64_t entry, exit, cnt, ok;
  int64_t last;
  uint32_t valid;
};
__device__ __forceinline__ bool plain_lite(const SparseParams &sp, const Lite &p, const Lite &a) {
  const bool v = a.valid != 0, live = p.exit >= sp_end(sp, p.last), in = p.exit < sp_end(sp, a.last);
  return v && live && in && p.exit == a.entry;
}
__device__ __forceinline__ int64_t group_last_lane(const SparseParams &sp, uint64_t w) {
  const uint64_t l = (w + 1) * 64;
  return (int64_t)(l < sp.nlanes ? l : sp.nlanes) - 1;
}
// exclusive block-wide scan of (c, o, n) over kScanThreads threads
__device__ void block_scan3(uint64_t &c, uint64_t &o, uint32_t &n, uint64_t &tc, uint64_t &to, uint32_t &tn,
                            uint64_t *sc, uint64_t *so, uint32_t *sn) {
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
  uint64_t ic = c, io = o;
  uint32_t in = n;
  for (int d = 1; d < 64; d <<= 1) {  // inclusive scan inside the wave
    const uint64_t yc = __shfl_up(ic, d, 64), yo = __shfl_up(io, d, 64);
    const uint32_t yn = __shfl_up(in, d, 64);
    if ((int)lane >= d) {
      ic += yc;
      io += yo;
      in += yn;
    }
  }
  if (lane == 63) {
    sc[wv] = ic;
    so[wv] = io;
    sn[wv] = in;
  }
  __syncthreads();
  if (tid == 0) {
    uint64_t ac = 0, ao = 0;
    uint32_t an = 0;
    for (uint32_t k = 0; k < kScanThreads / 64; ++k) {
      const uint64_t xc = sc[k], xo = so[k];
      const uint32_t xn = sn[k];
      sc[k] = ac;
      so[k] = ao;
      sn[k] = an;
      ac += xc;
      ao += xo;
      an += xn;
    }
    sc[kScanThreads / 64] = ac;
    so[kScanThreads / 64] = ao;
    sn[kScanThreads / 64] = an;
  }
  __syncthreads();
  c = sc[wv] + ic - c;
  o = so[wv] + io - o;
  n = sn[wv] + in - n;
  tc = sc[kScanThreads / 64];
  to = so[kScanThreads / 64];
  tn = sn[kScanThreads / 64];
  __syncthreads();
}

struct RunInfo {       // a run of plainly linked groups [s, e): the chain state it is entered with and
  uint64_t exit, cnt, ok, g;  // the group it enters at (g = e: none, the chain ended or passes over it)
};

__global__ __launch_bounds__(kScanThreads) void k_sparse_scan(SparseParams sp) {
  __shared__ uint64_t wsc[kScanThreads / 64 + 1], wso[kScanThreads / 64 + 1];
  __shared__ uint64_t s_en[kScanWin], s_ex[kScanWin + 1], s_co[kScanWin];  // the fast path's staged link fields
  __shared__ uint32_t wsn[kScanThreads / 64 + 1];
  __shared__ Seg badx[kResolvers];
  __shared__ uint32_t bad[kResolvers];
  __shared__ uint32_t nbad, first_w, fail, rewalks, qfull;
  __shared__ uint64_t entry0;
  __shared__ Seg E0, TOT;
  __shared__ uint32_t rows[kResolvers * kSpRow];
  __shared__ uint32_t task[kTasks], ntask, npass;  // the resolve's re-walk tasks: flagged index << 6 | lane
                                                   // (slots 0..63: the lowest flagged group's, reserved)
  __shared__ uint64_t tpos[kTasks];                // ... and each task's exact entry
  const ParseParams &kp = sp.kp;
  const uint32_t tid = threadIdx.x, W = sp.ngroups;
  const uint32_t q = W ? (W + kScanThreads - 1) / kScanThreads : 1u;  // groups per thread
  const uint32_t w0 = tid * q < W ? tid * q : W, w1 = w0 + q < W ? w0 + q : W;
  // scan scratch: exclusive sums of the groups' records / Ok flows (W + 1 each), each group's run,
  // the runs' first groups, the runs' entry states
  uint64_t *scnt = sp.scan, *sok = scnt + (W + 1);
  uint32_t *run_of = reinterpret_cast<uint32_t *>(sok + (W + 1)), *runs = run_of + W;
  RunInfo *rinfo = reinterpret_cast<RunInfo *>(sok + (W + 1) + W);
  auto agg = [&](uint32_t w) { return get_seg(sp.aggs + (uint64_t)w * kSparseAggWords); };
  if (tid == 0) {
    first_w = ~0u;
    fail = 0;
    rewalks = 0;
    qfull = 0;
  }
  __syncthreads();
  if ((kp.flags & kFlagSpecStart) && !kp.prev)  // the anchor: the first lane entry found
    for (uint32_t w = w0; w < w1; ++w)
      if (sp.first_entry[w] != kNone) {
        atomicMin(&first_w, w);
        break;
      }
  __syncthreads();
  if (tid == 0) {
    Seg E{};
    E.entry = E.exit = kp.start;
    E.first = E.last = -1;
    E.mism = -1;
    E.valid = 1;
    uint64_t e0 = kp.start;
    if (kp.prev) {  // a chained launch: the chain continues where the previous one left it
      if (kp.prev_epoch != 0 && kp.prev->epoch != kp.prev_epoch) fail = 1;  // it did not complete
      E.entry = E.exit = kp.prev->consumed;
      E.cnt = kp.prev->n_records;
      E.ok = kp.prev->n_flows;
      e0 = kp.prev->entry;
    } else if (kp.flags & kFlagSpecStart) {
      e0 = first_w == ~0u ? kNone : sp.first_entry[first_w];
      E.entry = E.exit = e0 == kNone ? kp.stop : e0;
    }
    E0 = E;
    entry0 = e0;
  }
  __syncthreads();
  if (fail) return;  // no summary: npr_dev_check reports the previous link's failure as a timeout
  // Fast path (C3: the anchor and every group link plainly, one run): each group's incoming state
  // is its predecessor's exit and two sums.  The link fields are staged in LDS kScanWin groups at a
  // time by coalesced loads; each thread then takes kScanWin / kScanThreads consecutive groups.
  {
    const Seg E = E0;
    uint64_t carry_c = E.cnt, carry_o = E.ok;
    bool linked = true;
    for (uint32_t v0 = 0; v0 < W; v0 += kScanWin) {
      const uint32_t nw = W - v0 < kScanWin ? W - v0 : kScanWin;
      {  // every load in flight before the first LDS store (a loop would wait for each in turn)
        constexpr uint32_t kPer = kScanWin / kScanThreads;
        uint64_t en[kPer], ex[kPer], co[kPer];
#pragma unroll
        for (uint32_t u = 0; u < kPer; ++u) {
          const uint32_t i = tid + u * kScanThreads, ii = i < nw ? i : 0u;
          en[u] = sp.lite[v0 + ii];
          ex[u] = sp.lite[W + v0 + ii];
          co[u] = sp.lite[2 * (uint64_t)W + v0 + ii];
        }
#pragma unroll
        for (uint32_t u = 0; u < kPer; ++u) {
          const uint32_t i = tid + u * kScanThreads;
          if (i < nw) {
            s_en[i] = en[u];
            s_ex[i + 1] = ex[u];
            s_co[i] = co[u];
          }
        }
      }
      if (tid == 0) s_ex[0] = v0 ? sp.lite[W + v0 - 1] : E.exit;
      __syncthreads();
      constexpr uint32_t kPer = kScanWin / kScanThreads;
      const uint32_t i0 = tid * kPer, i1 = i0 + kPer < nw ? i0 + kPer : nw;
      uint64_t c = 0, o = 0;
      for (uint32_t i = i0; i < i1; ++i) {
        const uint32_t w = v0 + i;
        const uint64_t co = s_co[i];
        const Lite pr{0, s_ex[i], 0, 0, w ? group_last_lane(sp, w - 1) : E.last, 1};
        const Lite a{s_en[i], s_ex[i + 1], co & 0xffffffffull, (co >> 32) & 0x7fffffffull, group_last_lane(sp, w),
                     (uint32_t)(co >> 63)};
        linked = linked && plain_lite(sp, pr, a);
        c += a.cnt;
        o += a.ok;
      }
      uint64_t tc, to;
      uint32_t n = 0, tn;
      block_scan3(c, o, n, tc, to, tn, wsc, wso, wsn);
      for (uint32_t i = i0; i < i1; ++i) {
        const uint64_t co = s_co[i];
        sp.pre[v0 + i] = SparsePre{s_ex[i], carry_c + c, carry_o + o, 0};
        c += co & 0xffffffffull;
        o += (co >> 32) & 0x7fffffffull;
      }
      carry_c += tc;
      carry_o += to;
      __syncthreads();
    }
    if (__syncthreads_and(linked ? 1 : 0)) {
      if (tid == 0) {
        npr_summary *sm = kp.summary;
        sm->n_records = carry_c;
        sm->n_flows = carry_o;
        sm->consumed = W ? sp.lite[W + W - 1] : E.exit;
        sm->flags = (kp.flows && carry_o > kp.flow_cap) ? NPR_SUMMARY_FLOW_OVERFLOW : 0u;
        sm->epoch = kp.epoch;
        sm->entry = entry0;
        __hip_atomic_store(sp.ctl, gran(kp.epoch, 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      return;
    }
  }
  for (uint32_t round = 0;; ++round) {
    // every round settles the lowest contradicted group for good: more rounds than groups is a bug,
    // and the launch then ends without a summary (npr_dev_check reports it) instead of spinning
    if (round > W + 1) return;
    // (1) runs of plainly linked groups; exclusive sums of records / Ok flows over the groups
    uint64_t c = 0, o = 0;
    uint32_t ns = 0;
    {
      Seg p = w0 > 0 && w0 < W ? agg(w0 - 1) : Seg{};
      for (uint32_t w = w0; w < w1; ++w) {
        const Seg a = agg(w);
        ns += (w == 0 || !plain_link(sp, p, a)) ? 1u : 0u;
        c += a.cnt;
        o += a.ok;
        p = a;
      }
    }
    uint64_t tc, to;
    uint32_t tn;
    block_scan3(c, o, ns, tc, to, tn, wsc, wso, wsn);
    {
      Seg p = w0 > 0 && w0 < W ? agg(w0 - 1) : Seg{};
      for (uint32_t w = w0; w < w1; ++w) {
        const Seg a = agg(w);
        if (w == 0 || !plain_link(sp, p, a)) runs[ns++] = w;
        run_of[w] = ns - 1;
        scnt[w] = c;
        sok[w] = o;
        c += a.cnt;
        o += a.ok;
        p = a;
      }
    }
    if (tid == 0) {
      scnt[W] = tc;
      sok[W] = to;
    }
    fence_agent();
    __syncthreads();
    fence_agent();
    // (2) the runs in order from the anchor (one thread; C3 has one run): each is entered at the
    //     group its incoming position lands in, and a contradiction there flags the group
    if (tid == 0) {
      uint64_t ex = E0.exit, cn = E0.cnt, ok = E0.ok;
      int64_t last = E0.last;
      uint32_t nb = 0;
      for (uint32_t r = 0; r < tn; ++r) {
        const uint32_t e = r + 1 < tn ? runs[r + 1] : W;  // this run: groups [runs[r], e)
        RunInfo ri{ex, cn, ok, e};
        const int64_t run_last = group_last_lane(sp, e - 1);
        if (ex >= sp_end(sp, last) && ex < sp_end(sp, run_last)) {  // not ended, lands in this run
          const uint64_t g = (ex - kp.start) / (64 * sp.span);
          ri.g = g;
          const Seg a = agg((uint32_t)g);
          if (!(a.valid && a.entry == ex)) {  // contradicted: resolve g from this state
            if (nb < (uint32_t)kResolvers) {
              Seg x{};
              x.entry = x.exit = ex;
              x.cnt = cn;
              x.ok = ok;
              x.first = x.last = (int64_t)g * 64 - 1;
              x.mism = -1;
              x.valid = 1;
              bad[nb] = (uint32_t)g;
              badx[nb] = x;
            }
            ++nb;
          }
          ex = agg(e - 1).exit;  // (contradicted: as if its resolution rejoins the speculated chain)
          cn += scnt[e] - scnt[g];
          ok += sok[e] - sok[g];
          last = run_last;
        } else if (ex >= sp_end(sp, last)) {  // one record spans the whole run
          last = run_last;
        }
        rinfo[r] = ri;
      }
      nbad = nb;
      Seg t{};
      t.exit = ex;
      t.cnt = cn;
      t.ok = ok;
      TOT = t;
    }
    fence_agent();
    __syncthreads();
    fence_agent();
    if (nbad == 0) {  // every link exact: each group's incoming chain state, and the summary
      for (uint32_t w = w0; w < w1; ++w) {
        const RunInfo ri = rinfo[run_of[w]];
        SparsePre pr{ri.exit, ri.cnt, ri.ok, 0};
        if (w > ri.g) {
          pr.exit = agg(w - 1).exit;
          pr.cnt = ri.cnt + scnt[w] - scnt[ri.g];
          pr.ok = ri.ok + sok[w] - sok[ri.g];
        }
        sp.pre[w] = pr;
      }
      if (tid == 0) {
        npr_summary *sm = kp.summary;
        sm->n_records = TOT.cnt;
        sm->n_flows = TOT.ok;
        sm->consumed = TOT.exit;
        sm->flags = (kp.flows && TOT.ok > kp.flow_cap) ? NPR_SUMMARY_FLOW_OVERFLOW : 0u;
        sm->epoch = kp.epoch;
        sm->entry = entry0;
        __hip_atomic_store(sp.ctl, gran(kp.epoch, 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (kp.stats && rewalks) atomicAdd(kp.stats + kStatRewalk, rewalks);
        if (kp.stats && qfull) atomicAdd(kp.stats + kStatQueueFull, qfull);
        if (kp.stats) atomicAdd(kp.stats + kStatScanRounds, round + 1);
      }
      return;
    }
    // (3) resolve the flagged groups (the lowest from its exact incoming state), then scan again:
    // the serial rule per group is "walk its lanes in order from the incoming position; a lane a
    // record spans is passed over (entry = exit = the position), a lane whose speculated entry is
    // not the position walks again from it".  Here lane-parallel, to a fixed point: each wave takes flagged groups and works out, from a group's
    // incoming state and its lanes' CURRENT exits, the position entering each lane; lanes a record
    // spans are set passed over, every lane whose entry differs becomes a re-walk task, and all 256
    // threads take the tasks.  Repeat until no lane changes: each pass makes at least the first
    // inconsistent lane of the LOWEST flagged group exact (its tasks have 64 reserved queue slots;
    // the other groups share the rest, and what does not fit waits for the next pass), so the lowest
    // group settles within 65 passes, and the fixed point is the serial rule's.  Each scan round
    // therefore settles its lowest flagged group for good (the outer `round` bound relies on that).
    // Round 4's one thread per group walked a group's lanes in turn: 15.3 ms of
    // the 300-MB adversarial capture's 16.3 (901 re-walks).
    const uint32_t nr = nbad < (uint32_t)kResolvers ? nbad : (uint32_t)kResolvers;
    {
      const uint32_t lane = tid & 63u, wv = tid >> 6;
      uint32_t rw = 0;
      for (uint32_t it = 0; it <= 65u; ++it) {
        if (tid == 0) {
          ntask = 0;
          npass = 0;
        }
        if (tid < 64) task[tid] = ~0u;  // the lowest group's reserved slots: empty unless claimed
        __syncthreads();
        for (uint32_t b = wv; b < nr; b += kScanThreads / 64) {  // (a) the tasks of group bad[b]
          const uint32_t w = bad[b];
          const Seg sx = badx[b];
          const uint64_t l0 = (uint64_t)w * 64;
          const uint32_t size = sp.nlanes - l0 < 64 ? (uint32_t)(sp.nlanes - l0) : 64u;
          const uint64_t li = l0 + lane;
          const bool in = lane < size;
          const SparseLane L = in ? sp.lanes[li] : SparseLane{};
          const uint64_t hi = in ? sp_end(sp, (int64_t)li) : 0ull;
          uint64_t pos = sx.exit, pred = kNone;
          int64_t last = sx.last;
          for (uint32_t j = 0; j < size; ++j) {  // (wave-uniform: readlanes of the lanes' current state)
            if (pos < sp_end(sp, last)) break;   // the chain ended before lane j
            if (lane == j) pred = pos;
            last = (int64_t)(l0 + j);
            if (pos >= rl64(hi, (int)j)) continue;  // a record spans lane j: the position passes on
            pos = rl64(L.exit, (int)j);
          }
          if (in && pred != kNone) {
            if (pred >= hi) {  // passed over
              if (L.entry != pred || L.exit != pred || L.cnt || L.ok) {
                sp.lanes[li] = SparseLane{pred, pred, 0u, 0u, kNone, 0ull, 0ull};
                atomicAdd(&npass, 1u);
              }
            } else if (L.entry != pred) {  // mis-speculated (or its predecessor moved): walk again
              const uint32_t k = b == 0 ? lane : 64u + atomicAdd(&ntask, 1u);
              if (k < kTasks) {
                task[k] = (b << 6) | lane;
                tpos[k] = pred;
              }
              if (b == 0) atomicAdd(&npass, 1u);  // (a pass with only reserved tasks still runs)
            }
          }
        }
        fence_agent();
        __syncthreads();
        fence_agent();
        const uint32_t nt = ntask < kTasks - 64u ? 64u + ntask : kTasks;
        if (ntask == 0 && npass == 0) break;
        if (tid == 0 && ntask > kTasks - 64u) ++qfull;
        for (uint32_t k = tid; k < nt; k += kScanThreads) {  // (b) every thread re-walks tasks
          if (task[k] == ~0u) continue;  // an unclaimed reserved slot
          const uint32_t b = task[k] >> 6, j = task[k] & 63u, w = bad[b];
          const uint64_t li = (uint64_t)w * 64 + j, p = tpos[k];
          uint32_t cnt = 0;
          AreaSink sink = area_sink(sp, w, j);
          const uint64_t ex = lane_walk(kp, rows + tid * kSpRow, p, sp_end(sp, (int64_t)li), cnt, sink);
          sp.lanes[li] = SparseLane{p, ex, cnt, sink.okn, sink.ovf, sink.okmask, sink.okmask2};
          ++rw;
        }
        fence_agent();
        __syncthreads();
        fence_agent();
      }
      if (rw) atomicAdd(&rewalks, rw);
      if (tid < nr) {  // (c) the resolved groups' aggregates
        const uint32_t w = bad[tid];
        const uint64_t l0 = (uint64_t)w * 64;
        const uint32_t size = sp.nlanes - l0 < 64 ? (uint32_t)(sp.nlanes - l0) : 64u;
        Seg a = lane_seg(sp, l0, sp.lanes[l0]);
        for (uint32_t j = 1; j < size; ++j) a = sp_cat(sp, a, lane_seg(sp, l0 + j, sp.lanes[l0 + j]));
        put_seg(sp.aggs + (uint64_t)w * kSparseAggWords, a);
        put_lite(sp, w, a);
      }
    }
    fence_agent();
    __syncthreads();
    fence_agent();
  }
}

// =============================================================================================
// k_sparse_rows: group w's Ok flows (file order i = 0 .. okw-1, global index O + i) to rows
// flow_cap - 1 - (O + i).  The group's slots go through LDS kRowChunk slot rows at a time: a slot row
// is 1 KiB of 16-B slot heads (area) + 768 B of 12-B slot tails (area_b), read as 112 contiguous
// 16-B chunks, a chunk only when a slot in it holds an Ok flow; written back as each lane's run of
// consecutive rows (thread 4j + s takes lane j's slots k0 + s + 4m: the four threads of a lane
// store neighbouring rows), each row's record offset rebuilt from the lane's start.  The next
// chunk's loads are in flight (registers) while the current one is written; the first chunk's are
// issued before the lanes' chain walk-through, which wave 0 runs from registers.
// =============================================================================================
constexpr uint32_t kRowChunk = 16;                       // slot rows (of 64 lanes) per LDS stage: 28 KiB
constexpr uint32_t kSlotChunks = 64u + 48u;              // 16-B chunks per slot row: heads, then tails
constexpr uint32_t kHeadPer = kRowChunk * 64u / kSpBlock;  // head chunks per thread per stage (lane tid & 63)
constexpr uint32_t kTailPer = kRowChunk * 48u / kSpBlock;  // tail chunks per thread per stage
static_assert(kRowChunk * 64u % kSpBlock == 0 && kRowChunk * 48u % kSpBlock == 0, "whole chunks per thread");
__device__ __forceinline__ bool bit_k(uint64_t m, uint64_t m2, uint32_t k) {
  return ((k < 64u ? m >> k : m2 >> (k - 64u)) & 1ull) != 0;
}
__global__ __launch_bounds__(kSpBlock) void k_sparse_rows(SparseParams sp) {
  __shared__ uint32_t opre[65];
  __shared__ uint32_t okl[64], sl[64];  // Ok flows of the lane, in its slots
  __shared__ uint64_t ovf[64], hil[64], msk[64], msk2[64];
  __shared__ uint32_t kmax_sh;
  __shared__ __attribute__((aligned(16))) u32x4 stage[kRowChunk * kSlotChunks];
  const ParseParams &kp = sp.kp;
  const uint32_t w = blockIdx.x, tid = threadIdx.x;
  if (__hip_atomic_load(sp.ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != gran(kp.epoch, 1)) return;
  // the first chunk (slot rows 0 .. 15 of every lane): lanes hold ~40-60 records, so these are
  // nearly always needed; loaded while wave 0 works out which lanes the chain runs through.
  // Thread t stages heads of lane t & 63 (slot rows (t >> 6) + 4 u) and tail chunks t + 256 u.
  const u32x4 *heads = reinterpret_cast<const u32x4 *>(sp.area) + (uint64_t)w * sp.cap * 64u;
  const u32x4 *tails = reinterpret_cast<const u32x4 *>(sp.area_b + (uint64_t)w * sp.cap * 192u);  // 48 chunks per slot row
  const uint32_t rows0 = sp.cap < kRowChunk ? sp.cap : kRowChunk;
  u32x4 vh[kHeadPer], vt[kTailPer];
#pragma unroll
  for (uint32_t u = 0; u < kHeadPer; ++u) {
    const uint32_t k = (tid >> 6) + 4u * u;
    vh[u] = k < rows0 ? heads[k * 64u + (tid & 63u)] : u32x4{0u, 0u, 0u, 0u};
  }
#pragma unroll
  for (uint32_t u = 0; u < kTailPer; ++u) {
    const uint32_t q = tid + u * kSpBlock;
    vt[u] = q < rows0 * 48u ? tails[q] : u32x4{0u, 0u, 0u, 0u};
  }
  const uint64_t l0 = (uint64_t)w * 64;
  const uint32_t size = sp.nlanes - l0 < 64 ? (uint32_t)(sp.nlanes - l0) : 64u;
  if (tid < 64) {  // wave 0: lane tid's walk; which lanes the exact chain runs through (every link is consistent now)
    const SparsePre P = sp.pre[w];
    const bool in = tid < size;
    SparseLane L{};
    if (in) L = sp.lanes[l0 + tid];
    const uint64_t hi = in ? sp_end(sp, (int64_t)(l0 + tid)) : 0ull;
    // the serial rule, on wave-uniform values: a lane whose end the chain position has passed is
    // spanned by a record (skipped); a lane whose exit is short of its end ends the chain
    uint64_t pos = P.exit, part = 0;
    bool ended = pos < sp_end(sp, (int64_t)l0 - 1);
    for (uint32_t j = 0; j < size && !ended; ++j) {
      const uint64_t hj = rl64(hi, (int)j);
      if (pos >= hj) continue;
      part |= 1ull << j;
      pos = rl64(L.exit, (int)j);
      ended = pos < hj;
    }
    const bool me = (part >> tid) & 1ull;
    const uint32_t ok = me ? L.ok : 0u;
    const uint64_t m = me ? L.okmask : 0ull, m2 = me ? L.okmask2 : 0ull;
    const uint32_t ex = excl_scan_u32(ok);
    opre[tid] = ex;
    okl[tid] = ok;
    msk[tid] = m;
    msk2[tid] = m2;
    sl[tid] = (uint32_t)__builtin_popcountll(m) + (uint32_t)__builtin_popcountll(m2);
    ovf[tid] = L.ovf;
    hil[tid] = hi;
    uint32_t km = m2 ? 128u - (uint32_t)__builtin_clzll(m2) : m ? 64u - (uint32_t)__builtin_clzll(m) : 0u;
    for (int o = 32; o > 0; o >>= 1) km = max(km, (uint32_t)__shfl_xor((int)km, o));
    if (tid == 63) opre[64] = ex + ok;
    if (tid == 0) kmax_sh = km;
  }
  __syncthreads();
  const uint32_t kmax = kmax_sh;
  const uint64_t O = sp.pre[w].ok;
  const uint32_t j = tid >> 2, sub = tid & 3u;
  const uint64_t mj = msk[j], mj2 = msk2[j];
  const uint32_t pj = opre[j];
  const uint32_t c0j = (uint32_t)__builtin_popcountll(mj);  // Ok flows of lane j in slots 0 .. 63
  const uint64_t loj = lane_lo(sp, l0 + j);
  const uint32_t *stw = reinterpret_cast<const uint32_t *>(stage);
  const uint64_t mh = msk[tid & 63u], mh2 = msk2[tid & 63u];  // the Ok slots of this thread's head lane
  for (uint32_t k0 = 0; k0 < kmax; k0 += kRowChunk) {
    const uint32_t nk = kmax - k0 < kRowChunk ? kmax - k0 : kRowChunk;
#pragma unroll
    for (uint32_t u = 0; u < kHeadPer; ++u) {
      const uint32_t k = (tid >> 6) + 4u * u;
      if (k < nk) stage[k * kSlotChunks + (tid & 63u)] = vh[u];
    }
#pragma unroll
    for (uint32_t u = 0; u < kTailPer; ++u) {
      const uint32_t q = tid + u * kSpBlock, k = q / 48u;
      if (k < nk) stage[k * kSlotChunks + 64u + q % 48u] = vt[u];
    }
    __syncthreads();
    const uint32_t k1 = k0 + kRowChunk;
    if (k1 < kmax) {  // the next chunk's loads (a chunk only when a slot in it holds an Ok flow),
                      // in flight while this one is written
      const uint32_t nk1 = kmax - k1 < kRowChunk ? kmax - k1 : kRowChunk;
#pragma unroll
      for (uint32_t u = 0; u < kHeadPer; ++u) {
        const uint32_t k = (tid >> 6) + 4u * u;
        vh[u] = k < nk1 && bit_k(mh, mh2, k1 + k) ? heads[(k1 + k) * 64u + (tid & 63u)] : u32x4{0u, 0u, 0u, 0u};
      }
#pragma unroll
      for (uint32_t u = 0; u < kTailPer; ++u) {
        const uint32_t q = tid + u * kSpBlock, k = q / 48u, c = q % 48u;
        const uint32_t l1 = (16u * c) / 12u, l2 = (16u * c + 15u) / 12u;  // the lanes whose tails it holds
        const bool need = bit_k(msk[l1] | msk[l2], msk2[l1] | msk2[l2], k1 + k);
        vt[u] = k < nk1 && need ? tails[(k1 + k) * 48u + c] : u32x4{0u, 0u, 0u, 0u};
      }
    }
#pragma unroll
    for (uint32_t m = 0; m < kRowChunk / 4; ++m) {
      const uint32_t k = k0 + sub + 4 * m;
      const bool okk = k < 64u ? ((mj >> k) & 1ull) : ((mj2 >> (k - 64u)) & 1ull);
      if (k < k0 + nk && okk) {
        const uint32_t below = k < 64u ? (uint32_t)__builtin_popcountll(mj & ((1ull << k) - 1ull))
                                       : c0j + (uint32_t)__builtin_popcountll(mj2 & ((1ull << (k - 64u)) - 1ull));
        const uint64_t gi = O + pj + below;
        if (gi < kp.flow_cap) {
          const uint32_t rk = k - k0;
          const uint32_t tb = (rk * kSlotChunks + 64u) * 4u + 3u * j;  // the tail's first dword
          const uint32_t b2 = stw[tb + 2];
          u32x4 r0, r1;
          slot_row(stage[rk * kSlotChunks + j], stw[tb], stw[tb + 1], b2, loj + (b2 >> 14), r0, r1);
          put_row(kp, kp.flow_cap - 1 - gi, r0, r1);
        }
      }
    }
    __syncthreads();
  }
  if (tid < 64 && okl[tid] > sl[tid]) {  // Ok flows past the lane's slots: walked again from its first slotless record
    RowSink sink{&kp, O + opre[tid], sl[tid]};
    uint32_t cnt = 0;
    (void)lane_walk(kp, reinterpret_cast<uint32_t *>(stage) + tid * kSpRow, ovf[tid], hil[tid], cnt, sink);
  }
}

}  // namespace

hipError_t launch_sparse(const SparseParams &sp, hipStream_t s) {
  if (sp.ngroups) {
    hipLaunchKernelGGL(k_sparse_walk, dim3((sp.ngroups + kSpBlock / 64 - 1) / (kSpBlock / 64)), dim3(kSpBlock), 0, s, sp);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k_sparse_scan, dim3(1), dim3(kScanThreads), 0, s, sp);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !sp.ngroups || !sp.kp.flows) return e;
  hipLaunchKernelGGL(k_sparse_rows, dim3(sp.ngroups), dim3(kSpBlock), 0, s, sp);
  return hipGetLastError();
}

}  // namespace npr
