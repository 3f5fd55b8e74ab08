// rowblk_decode.hip — gfx950 decoder for Pebble row-oriented data blocks.
//
// One 256-thread workgroup per block (block id = an atomic ticket, so the
// decoupled look-back always waits on resident predecessors).
//
//   stage   the block HBM -> LDS once, 16-byte coalesced loads
//   P1      one lane per restart run walks its entries (restart points cut the
//           prefix chain, rowblk_writer.go:147-155), parking each entry offset
//           and its in-run key/value output prefix in a slot; a block scan of
//           the per-run sums gives the block's totals
//   look-back  wave 0 publishes the totals and resolves the batch-wide output
//           bases (decoupled look-back: single pass, no size pass) WHILE waves
//           1-3 expand the slots into per-KV arrays (P2)
//   write   per-KV arrays; key and value bytes as 16-byte granules, each the
//           merge of a few LDS segment gathers (a key's bytes are the segments
//           of its prefix chain), one dwordx4 store per full granule
//
// Semantics follow cockroachdb/pebble sstable/rowblk/rowblk_iter.go:
//   Init :241-276 (numRestarts, restarts offset), readFirstKey :418-485,
//   readEntry :333-416 (3 uint32 varints, fullKey = fullKey[:shared]+unshared),
//   decodeInternalKey :487-504 (LE64 trailer & TrailerObsoleteMask, <8 B =>
//   InternalKeyKindInvalid), value prefix :1192-1199 (block/kv.go:14-41),
//   decodeRestart :1092-1096, RawIter.readEntry :1784-1794 (PBL_ROW_RAW_KEYS).
// Blocks whose restart table is inconsistent with a per-run walk, or that do
// not fit the LDS limits, take the general path (rowblk_general.hip.h): a
// wave-serial restatement of Iter.First/Next, bit-identical by construction.
#include <algorithm>
#include <atomic>

#include "common.hip.h"
#include "colblk_block.hip.h"

namespace pbl {
namespace row {

constexpr int kPad = 16;                  // LDS front pad: segment gathers may start up to 15 B early
constexpr int kLdsBlkBytes = kPad + 32768 + 32;  // block staging (any 16-B phase of a <=32 KiB block)
constexpr uint32_t kMaxFastLen = 32768;   // blocks up to this length take the LDS path
constexpr int kKvCap = 512;               // KVs per block on the LDS path
constexpr int kRunCap = kKvCap;           // restart runs per block on the LDS path
constexpr uint32_t kMaxFastKeyBytes = 65535;  // user-key bytes per block on the LDS path (u16 offsets)
constexpr int kBkt = 256;                 // bytes per output bucket of the granule -> KV index
constexpr uint32_t kRestartMask = 0x7fffffffu;
constexpr uint64_t kTrailerObsoleteMask = ((((uint64_t)1 << 56) - 1) << 8) | 191u;
constexpr uint64_t kKindInvalid = kKindInvalidTrailer;

// aux (u16) area: run-walk slots, per-run prefixes, output buckets
constexpr int kSlotPos = 0;                          // [kKvCap] entry offset of slot q
constexpr int kSlotCk = kSlotPos + kKvCap;           // [kKvCap] in-run user-key prefix of slot q
constexpr int kSlotCv = kSlotCk + kKvCap;            // [kKvCap] in-run value prefix of slot q
constexpr int kSlotSh = kSlotCv + kKvCap;            // [kKvCap] shared length of slot q
constexpr int kSlotPar = kSlotSh + kKvCap;           // [kKvCap] in-run index of slot q's prefix parent
constexpr int kRunKv0 = kSlotPar + kKvCap;           // [kRunCap+1] first KV of run r
constexpr int kRunKb0 = kRunKv0 + kRunCap + 1;       // [kRunCap+1] key-byte offset of run r
constexpr int kRunVb0 = kRunKb0 + kRunCap + 1;       // [kRunCap+1] value-byte offset of run r
constexpr int kAuxWords = (kRunVb0 + kRunCap + 1 + 7) & ~7;

struct Lds {
  uint4 blk4[kLdsBlkBytes / 16];  // block byte i at byte kPad+shift+i
  uint16_t eoff[kKvCap];          // entry offset
  uint16_t ksrc[kKvCap];          // offset of the unshared key bytes
  uint16_t sh[kKvCap];            // shared length
  uint16_t klen[kKvCap];          // internal key length
  uint16_t vsrc[kKvCap];          // value offset (after prefix stripping)
  uint16_t vlen[kKvCap];          // value length (after prefix stripping)
  uint32_t kout[kKvCap + 1];      // user-key output offsets (block relative)
  uint32_t vout[kKvCap + 1];      // value output offsets (block relative)
  uint8_t kvf[kKvCap];            // PBL_KV_* flags
  uint16_t par[kKvCap];           // prefix parent: max{i < j in run : shared_i < shared_j}
  uint16_t aux[kAuxWords];
  uint32_t scratch[16];
  uint64_t bases[kNumComp];
  uint32_t status, slow, nkv, nres, S, shift, tot_kb, tot_vb;
  int32_t roff;
  // persistent kernel: tickets / descriptors of the next blocks
  uint32_t nxt, n2, n2_len, nxt_len;
  uint64_t n2_off, nxt_off;
};

// Unaligned LDS access.  gfx950 runs in unaligned access mode (the HSA
// runtime's default), where one ds_read_b128 / b64 / b32 serves any byte
// address: a 16-byte gather is one instruction instead of five dword reads
// and four alignbytes.  Measured on config 2 (same box, A/B): unaligned 16-byte
// gathers +2.7 % (992 vs 965 GiB/s), unaligned 8-byte header reads in the
// parse walk -1.5 %; so gathers are unaligned and ld8/le32 stay dword reads
// (PBL_LDS_UA8 / PBL_LDS_UA16 switch each form for A/B builds).
typedef u32x4 u32x4_u __attribute__((aligned(1)));
typedef u32x2 u32x2_u __attribute__((aligned(1)));
typedef uint32_t u32_u __attribute__((aligned(1)));
#ifndef PBL_LDS_UA8
#define PBL_LDS_UA8 0
#endif
#ifndef PBL_LDS_UA16
#define PBL_LDS_UA16 1
#endif

// 16 bytes at LDS byte address a (any alignment)
__device__ inline uint4 lds_gather16(lptr<const uint32_t> W, uint32_t a) {
#if !PBL_LDS_UA16
  uint32_t q = a >> 2, r = a & 3;
  uint32_t x0 = W[q], x1 = W[q + 1], x2 = W[q + 2], x3 = W[q + 3], x4 = W[q + 4];
  return make_uint4(__builtin_amdgcn_alignbyte(x1, x0, r), __builtin_amdgcn_alignbyte(x2, x1, r),
                    __builtin_amdgcn_alignbyte(x3, x2, r), __builtin_amdgcn_alignbyte(x4, x3, r));
#else
  const u32x4 v = *(lptr<const u32x4_u>)(reinterpret_cast<lptr<const uint8_t>>(W) + a);
  return make_uint4(v.x, v.y, v.z, v.w);
#endif
}

// Read-only view of the staged block: its base offset lives in a register.
struct View;
__device__ __forceinline__ View lds_view(const void* lds, uint32_t base);
struct View {
  lptr<const uint8_t> B;   // LDS bytes (array start)
  lptr<const uint32_t> W;  // LDS words (array start)
  uint32_t base;      // byte index of block byte 0 (kPad + shift)
  __device__ inline uint32_t byte(uint32_t i) const { return B[base + i]; }
  // 8 block bytes [i, i+8) as a little-endian u64
  __device__ inline uint64_t ld8(uint32_t i) const {
#if !PBL_LDS_UA8
    uint32_t a = base + i, q = a >> 2, r = a & 3;
    uint32_t x0 = W[q], x1 = W[q + 1], x2 = W[q + 2];
    uint32_t lo = __builtin_amdgcn_alignbyte(x1, x0, r);
    uint32_t hi = __builtin_amdgcn_alignbyte(x2, x1, r);
    return uint64_t(hi) << 32 | lo;
#else
    const u32x2 v = *(lptr<const u32x2_u>)(B + base + i);
    return uint64_t(v.y) << 32 | v.x;
#endif
  }
  __device__ inline uint32_t le32(uint32_t i) const {
#if !PBL_LDS_UA8
    uint32_t a = base + i, q = a >> 2, r = a & 3;
    return __builtin_amdgcn_alignbyte(W[q + 1], W[q], r);
#else
    return *(lptr<const u32_u>)(B + base + i);
#endif
  }
  // 16 block bytes starting at block offset i (i may be up to 15 below 0)
  __device__ inline uint4 ld16(int32_t i) const { return lds_gather16(W, uint32_t(int32_t(base) + i)); }
};

__device__ __forceinline__ View lds_view(const void* lds, uint32_t base) {
  return View{to_lds_ptr(reinterpret_cast<const uint8_t*>(lds)), to_lds_ptr(reinterpret_cast<const uint32_t*>(lds)),
              base};
}

// mask of the low n bytes of a word, n clamped to [0, 4]
__device__ inline uint32_t low_bytes(int n) {
  n = n < 0 ? 0 : n;
  return n >= 4 ? 0xffffffffu : (1u << (8 * n)) - 1u;
}
// byte mask of bytes [a, b) within the 4-byte word k of a 16-byte granule
__device__ inline uint32_t word_mask(int k, uint32_t a, uint32_t b) {
  return low_bytes(int(b) - 4 * k) & ~low_bytes(int(a) - 4 * k);
}
__device__ inline void merge16(uint4& w, const uint4& v, uint32_t a, uint32_t b) {
  uint32_t m;
  m = word_mask(0, a, b); w.x = (w.x & ~m) | (v.x & m);
  m = word_mask(1, a, b); w.y = (w.y & ~m) | (v.y & m);
  m = word_mask(2, a, b); w.z = (w.z & ~m) | (v.z & m);
  m = word_mask(3, a, b); w.w = (w.w & ~m) | (v.w & m);
}

// varint from LDS (rowblk_iter.go:2020-2038); returns bytes used, 0 if it runs past `end`
__device__ inline uint32_t lds_varint(const View& V, uint32_t p, uint32_t end, uint32_t* v) {
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 5; i++) {
    if (p + i >= end) return 0;
    uint32_t b = V.byte(p + i);
    if (i == 4) { *v = r | (b << 28); return 5; }
    if (b < 128) { *v = r | (b << (7 * i)); return i + 1; }
    r |= (b & 0x7f) << (7 * i);
  }
  return 0;
}

// Decode the 3 varints of the entry at `pos` (fast path: all three 1 byte).
__device__ inline uint32_t entry_header(const View& V, uint32_t pos, uint32_t end, uint32_t* sh,
                                        uint32_t* un, uint32_t* vl) {
  uint64_t w = V.ld8(pos);
  if (pos + 3 <= end && (w & 0x808080ull) == 0) {
    *sh = uint32_t(w) & 0xff;
    *un = uint32_t(w >> 8) & 0xff;
    *vl = uint32_t(w >> 16) & 0xff;
    return 3;
  }
  uint32_t x = lds_varint(V, pos, end, sh);
  uint32_t y = x ? lds_varint(V, pos + x, end, un) : 0;
  uint32_t z = y ? lds_varint(V, pos + x + y, end, vl) : 0;
  return z ? x + y + z : 0;
}

// byte p of the internal key of entry j: source entry = max{i <= j : shared_i <= p}
// (a run's first entry has shared == 0 so the walk stays inside the run)
__device__ inline uint32_t key_byte(const Lds& s, const View& V, int j, uint32_t p) {
  while (p < uint32_t(s.sh[j])) j--;
  return V.byte(s.ksrc[j] + p - s.sh[j]);
}

// trailer + flags of entry j (LDS path)
__device__ inline uint64_t entry_trailer(const Lds& s, const View& V, int j, uint8_t* fl, uint32_t flags) {
  if (flags & PBL_ROW_RAW_KEYS) return 0;
  uint32_t kl = s.klen[j];
  if (kl < 8) { *fl |= PBL_KV_INVALID_KEY; return kKindInvalid; }
  uint32_t sh = s.sh[j];
  uint64_t raw;
  if (kl - 8 >= sh) {  // all 8 trailer bytes are in this entry's unshared part
    raw = V.ld8(s.ksrc[j] + (kl - 8 - sh));
  } else {
    raw = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) raw |= uint64_t(key_byte(s, V, j, kl - 8 + i)) << (8 * i);
  }
  if (raw & 64u) *fl |= PBL_KV_OBSOLETE;
  return raw & kTrailerObsoleteMask;
}

// Block-wide exclusive scan of three u32 sequences (one value each per thread).
__device__ inline void block_excl_scan3(uint32_t a, uint32_t b, uint32_t c, uint32_t* e, uint32_t* tot,
                                        uint32_t* scratch) {
  uint32_t ia = wave_incl_scan(a), ib = wave_incl_scan(b), ic = wave_incl_scan(c);
  const int w = wave_id(), l = lane_id();
  if (l == kWave - 1) { scratch[w] = ia; scratch[4 + w] = ib; scratch[8 + w] = ic; }
  __syncthreads();
  uint32_t p[3] = {0, 0, 0}, tt[3] = {0, 0, 0};
#pragma unroll
  for (int i = 0; i < kTPB / kWave; i++) {
#pragma unroll
    for (int k = 0; k < 3; k++) {
      uint32_t v = scratch[4 * k + i];
      if (i < w) p[k] += v;
      tt[k] += v;
    }
  }
  e[0] = p[0] + ia - a;
  e[1] = p[1] + ib - b;
  e[2] = p[2] + ic - c;
  tot[0] = tt[0];
  tot[1] = tt[1];
  tot[2] = tt[2];
}


#ifdef PBL_STAMPS
// diagnostic build only: per-block phase timestamps (s_memtime) written past
// the look-back state in the workspace; never part of an output
#define STAMPT(i, tid)                                                                    \
  do {                                                                                    \
    if (threadIdx.x == (tid))                                                             \
      reinterpret_cast<uint64_t*>(ws + ws_bytes(nb))[uint64_t(b) * 16 + (i)] =           \
          __builtin_amdgcn_s_memtime();                                                   \
  } while (0)
#define STAMP(i) STAMPT(i, 0)
#else
#define STAMPT(i, tid) do {} while (0)
#define STAMP(i) do {} while (0)
#endif

#include "rowblk_general.hip.h"

// Store bytes [lo, hi) of the 16-byte granule w to p[lo..hi) (p 16-B aligned)
// with the fewest naturally aligned byte/short/dword/qword stores.  The granule
// is handled as two u64 halves and shifts: indexing its dwords with a runtime
// index would place it in scratch (a scratch round trip per granule, whose
// vmcnt wait drains every outstanding store).
template <class P>
__device__ __forceinline__ void store_partial16(P p, const uint4& w, uint32_t lo, uint32_t hi) {
  const uint64_t qa = uint64_t(w.x) | (uint64_t(w.y) << 32);
  const uint64_t qb = uint64_t(w.z) | (uint64_t(w.w) << 32);
  uint32_t x = lo;
  while (x < hi) {
    const uint64_t v = (x < 8 ? qa : qb) >> (8 * (x & 7));
    if ((x & 1) || hi - x < 2) {
      *(gptr<uint8_t>)(p + x) = uint8_t(v);
      x += 1;
    } else if ((x & 3) || hi - x < 4) {
      *(gptr<uint16_t>)(p + x) = uint16_t(v);
      x += 2;
    } else if ((x & 7) || hi - x < 8) {
      *(gptr<uint32_t>)(p + x) = uint32_t(v);
      x += 4;
    } else {
      *(gptr<uint64_t>)(p + x) = v;
      x += 8;
    }
  }
}

// P1 for run r: walk entries, park offsets and in-run output prefixes in the
// slots of run r, return (count, user-key bytes, value bytes).  `ok` clears when
// the run does not end exactly at the next restart (general path).
__device__ inline void walk_run(Lds& s, const View& V, uint32_t r, uint32_t nres, uint32_t roff, uint32_t S,
                                uint32_t flags, uint32_t* cnt_o, uint32_t* kb_o, uint32_t* vb_o) {
  uint32_t st = roff + 4 * r;
  uint32_t s0 = V.le32(st) & kRestartMask;
  uint32_t e0 = (r + 1 < nres) ? (V.le32(st + 4) & kRestartMask) : roff;
  uint32_t cnt = 0, kb = 0, vb = 0, prev_kl = 0, prev_sh = 0, pp = 0, ppsh = 0;
  bool ok = (r != 0 || s0 == 0) && s0 < e0 && e0 <= roff;
  uint32_t pos = s0;
  while (ok && pos < e0) {
    uint32_t sh, un, vl;
    uint32_t h = entry_header(V, pos, e0, &sh, &un, &vl);
    if (!h || (cnt == 0 && sh != 0) || cnt >= S) { ok = false; break; }
    uint64_t np = uint64_t(pos) + h + un + vl;
    if (np > e0) { ok = false; break; }
    // fullKey[:shared] needs shared <= len(previous key) (rowblk_iter.go:403)
    if (sh > prev_kl && cnt > 0) atomicMax(&s.status, uint32_t(PBL_CORRUPT_BOUNDS));
    uint32_t q = r * S + cnt;
    s.aux[kSlotPos + q] = uint16_t(pos);
    s.aux[kSlotCk + q] = uint16_t(kb);
    s.aux[kSlotCv + q] = uint16_t(vb);
    s.aux[kSlotSh + q] = uint16_t(sh);
    // prefix parent = nearest earlier entry of the run with a smaller shared
    // length (all-nearest-smaller-values walk over the parents: amortised O(1))
    // The previous entry and its parent are kept in registers; deeper steps
    // read the parked slots.
    uint32_t par = cnt, parsh = 0;
    if (sh != 0) {
      uint32_t c = cnt - 1, csh = prev_sh;
      if (csh >= sh) { c = pp; csh = ppsh; }
      while (csh >= sh) {
        c = s.aux[kSlotPar + r * S + c];
        csh = s.aux[kSlotSh + r * S + c];
      }
      par = c;
      parsh = csh;
    }
    s.aux[kSlotPar + q] = uint16_t(par);
    prev_sh = sh;
    pp = par;
    ppsh = parsh;
    uint32_t kl = sh + un;
    kb += (flags & PBL_ROW_RAW_KEYS) ? kl : (kl >= 8 ? kl - 8 : 0);
    vb += vl;
    prev_kl = kl;
    pos = uint32_t(np);
    cnt++;
  }
  if (!ok) atomicOr(&s.slow, 1u);
  *cnt_o = cnt;
  *kb_o = kb;
  *vb_o = vb;
}

// P2 for slot q: expand into KV arrays at its final index; mark output buckets.
__device__ inline void expand_slot(Lds& s, const View& V, uint32_t q, uint32_t S, uint32_t roff,
                                   uint32_t flags) {
  uint32_t r = q / S, k = q - r * S;
  uint32_t kv0 = s.aux[kRunKv0 + r], kv1 = s.aux[kRunKv0 + r + 1];
  if (kv0 + k >= kv1) return;
  uint32_t j = kv0 + k;
  uint32_t pos = s.aux[kSlotPos + q], sh, un, vl;
  uint32_t h = entry_header(V, pos, roff, &sh, &un, &vl);
  uint32_t kl = sh + un;
  uint32_t ko = uint32_t(s.aux[kRunKb0 + r]) + s.aux[kSlotCk + q];
  uint32_t vo = uint32_t(s.aux[kRunVb0 + r]) + s.aux[kSlotCv + q];
  s.eoff[j] = uint16_t(pos);
  s.ksrc[j] = uint16_t(pos + h);
  s.sh[j] = uint16_t(sh);
  s.klen[j] = uint16_t(kl);
  s.vsrc[j] = uint16_t(pos + h + un);
  s.vlen[j] = uint16_t(vl);
  s.kout[j] = ko;
  s.vout[j] = vo;
  uint8_t fl = (!(flags & PBL_ROW_RAW_KEYS) && kl < 8) ? uint8_t(PBL_KV_INVALID_KEY) : uint8_t(0);
  if (k == 0) fl |= uint8_t(PBL_KV_RESTART | ((V.le32(roff + 4 * r) >> 31) ? PBL_KV_RESTART_SAMEPFX : 0));
  s.kvf[j] = fl;
  // prefix parent (computed in P1): the nearest earlier entry of the run whose
  // own bytes start below shared_j; entries in between contribute nothing.
  s.par[j] = uint16_t(sh != 0 ? kv0 + s.aux[kSlotPar + q] : j);
  // bucket b (bytes [b*kBkt, ...)) belongs to the KV that holds its first byte
}

// Bytes [p_lo, p_hi) of the user key of KV j (length klen), placed at bytes
// [q, ...) of a 16-byte granule.  The key is the concatenation of its prefix-
// chain segments: [shared_i, cur) of entry i, walking i = j, par[j], ...
// (rowblk_iter.go:403 unrolled backwards); each segment is one LDS gather
// merged under a byte mask.
__device__ __forceinline__ uint4 key_part(const Lds& s, const View& V, int j, uint32_t klen, uint32_t p_lo,
                                          uint32_t p_hi, uint32_t q) {
  uint4 w = make_uint4(0, 0, 0, 0);
  uint32_t cur = klen;
  int i = j;
  while (cur > p_lo) {
    const uint32_t shi = s.sh[i];
    const uint32_t lo_i = shi < cur ? shi : cur;
    const uint32_t a = lo_i > p_lo ? lo_i : p_lo, z = cur < p_hi ? cur : p_hi;
    if (a < z) {
      const uint32_t gq = q + (a - p_lo);
      const int32_t src = int32_t(s.ksrc[i]) - int32_t(shi) + int32_t(a);  // block offset of key byte a
      const uint4 v = V.ld16(src - int32_t(gq));
      if (gq == 0 && z - a == 16) w = v;
      else merge16(w, v, gq, gq + (z - a));
    }
    cur = lo_i;
    i = s.par[i];
  }
  return w;
}

// ---------------------------------------------------------------------------
// The decode kernel.
// ---------------------------------------------------------------------------
// Init checks of one row block (Init :248-256, readFirstKey :418-485) read
// through `rd` (LDS when staged, else global).  Thread 0 only.
template <class Rd>
__device__ __forceinline__ void row_init(Lds& s, const Rd& rd, uint32_t blen, uint32_t flags, bool fits) {
  uint32_t st = PBL_OK;
  int64_t roff = 0;
  int32_t nr = 0;
  if (blen < 4) st = PBL_CORRUPT_BOUNDS;
  else {
    nr = int32_t(rd.le32(blen - 4));
    if (nr == 0) st = PBL_CORRUPT_NO_RESTARTS;
    else if (nr < 0) st = PBL_CORRUPT_BOUNDS;
    else {
      roff = int64_t(blen) - 4 * (1 + int64_t(nr));
      if (roff < 0) st = PBL_CORRUPT_BOUNDS;
      else if (roff > 0 && !(flags & PBL_ROW_RAW_KEYS)) {
        if (rd.byte(0) != 0) st = PBL_CORRUPT_FIRST_KEY;
        else {
          uint32_t un, vl;
          uint32_t n1 = rd.varint(1, blen, &un);
          uint32_t n2 = n1 ? rd.varint(1 + n1, blen, &vl) : 0;
          if (!n2) st = PBL_CORRUPT_BOUNDS;
          else if (un < 8) st = PBL_CORRUPT_FIRST_KEY;
        }
      }
    }
  }
  s.status = st;
  s.roff = int32_t(roff);
  s.nres = (st == PBL_OK) ? uint32_t(nr) : 0;
  s.S = (st == PBL_OK && nr > 0) ? uint32_t(kKvCap) / uint32_t(nr) : 1;
  s.slow = (st == PBL_OK && (!fits || uint32_t(nr) > uint32_t(kRunCap))) ? 1u : 0u;
  s.nkv = 0;
  s.tot_kb = s.tot_vb = 0;
  s.kout[0] = s.vout[0] = 0;
}

struct LdsRd {  // staged block through the View
  View V;
  __device__ uint32_t byte(uint32_t i) const { return V.byte(i); }
  __device__ uint32_t le32(uint32_t i) const { return V.le32(i); }
  __device__ uint32_t varint(uint32_t p, uint32_t end, uint32_t* v) const { return lds_varint(V, p, end, v); }
};
struct GlbRd {  // unstaged block in global memory
  const uint8_t* g;
  __device__ uint32_t byte(uint32_t i) const { return g[i]; }
  __device__ uint32_t le32(uint32_t i) const { return g_le32(g + i); }
  __device__ uint32_t varint(uint32_t p, uint32_t end, uint32_t* v) const { return g_varint(g + p, g + end, v); }
};

// Stage block bytes from global memory into LDS (granule g of the 16-B aligned
// source lands at blk4[1 + g]).
__device__ __forceinline__ void row_stage(Lds& s, const uint8_t* blocks, uint64_t boff, uint32_t blen) {
  const uint64_t a0 = boff & ~uint64_t(15);
  const uint64_t a1 = (boff + blen + 15) & ~uint64_t(15);
  const uint4* src = reinterpret_cast<const uint4*>(blocks + a0);
  const uint32_t n16 = uint32_t((a1 - a0) >> 4);
  for (uint32_t g = threadIdx.x; g < n16; g += kTPB) s.blk4[1 + g] = src[g];
}

constexpr int kPfWaves = kTPB / kWave - 1;                  // waves 1-3 prefetch
constexpr int kPfThreads = kPfWaves * kWave;                // 192
constexpr int kPfRegs = (kLdsBlkBytes / 16 + kPfThreads - 1) / kPfThreads;  // 11 granules / lane
static_assert(kPfRegs == 11, "PBL_PF_LIST");
// 11 named granule registers per prefetching lane (an array ends up in scratch:
// it is live across the whole decode of the current block).
#define PBL_PF_LIST(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10)

// The next block, held in registers by waves 1-3 while the current one decodes.
struct PfRegs {
#define PBL_PF_DECL(i) u32x4 r##i;
  PBL_PF_LIST(PBL_PF_DECL)
#undef PBL_PF_DECL
  // load the block at [off, off+len) (clamped: lanes past the end re-read the
  // last granule instead of running off the block)
  __device__ __forceinline__ void load(const uint8_t* blocks, uint64_t off, uint32_t len) {
    const uint64_t a0 = off & ~uint64_t(15);
    const uint32_t n16 = uint32_t((((off + len + 15) & ~uint64_t(15)) - a0) >> 4);
    if (n16 == 0) return;
    gptr<const u32x4> src = to_glb(reinterpret_cast<const u32x4*>(blocks + a0));
    const uint32_t l = threadIdx.x - kWave;
#define PBL_PF_LOAD(i)                                               \
    {                                                                \
      const uint32_t g = l + uint32_t(i) * kPfThreads;               \
      r##i = src[g < n16 ? g : n16 - 1];                             \
    }
    PBL_PF_LIST(PBL_PF_LOAD)
#undef PBL_PF_LOAD
  }
  __device__ __forceinline__ void store(Lds& s, uint64_t off, uint32_t len) const {
    const uint64_t a0 = off & ~uint64_t(15);
    const uint32_t n16 = uint32_t((((off + len + 15) & ~uint64_t(15)) - a0) >> 4);
    const uint32_t l = threadIdx.x - kWave;
#define PBL_PF_STORE(i)                                              \
    {                                                                \
      const uint32_t g = l + uint32_t(i) * kPfThreads;               \
      if (g < n16) reinterpret_cast<u32x4*>(s.blk4)[1 + g] = r##i;   \
    }
    PBL_PF_LIST(PBL_PF_STORE)
#undef PBL_PF_STORE
  }
};

// Persistent kernel hooks (wave 0 lane 0): take the next ticket right after
// this block publishes its aggregate, and publish the next block's descriptor
// once the look-back has resolved, so the next block starts decoding right
// after this one's outputs: ticket order stays ~= processing order.
__device__ __forceinline__ void next_descriptor(Lds& s, const Args& A, uint32_t tk) {
  s.nxt = tk;
  if (tk < A.in.n_blocks) {
    s.nxt_off = A.in.block_off[tk];
    s.nxt_len = A.in.block_len[tk];
  }
}
// waves 1-3: start loading the next block into registers
__device__ __forceinline__ void next_prefetch(Lds& s, const Args& A, bool persist, PfRegs& pf) {
  if (persist && threadIdx.x >= kWave) {
    const uint32_t n = s.nxt;
    if (n < A.in.n_blocks && s.nxt_len <= kMaxFastLen) pf.load(A.in.blocks, s.nxt_off, s.nxt_len);
  }
}

// Decode row block b whose bytes are staged in LDS (when blen <= kMaxFastLen).
// `persist`: persistent mode (ticket for the next block + its prefetch into pf).
__device__ __forceinline__ void row_process(Lds& s, const Args& A, const uint32_t b, const uint64_t boff,
                                            const uint32_t blen, const bool persist, PfRegs& pf) {
  const int t = threadIdx.x;
  const pbl_decode_out& O = A.out;
  const uint32_t nb = A.in.n_blocks;
  const uint32_t flags = A.in.flags;
  const bool vprefix = (flags & PBL_ROW_VALUE_PREFIX) && !(flags & PBL_ROW_RAW_KEYS);
  uint8_t* ws = reinterpret_cast<uint8_t*>(O.workspace);
  uint64_t* lb_state = reinterpret_cast<uint64_t*>(ws + kWsHeader);
  const uint8_t* gblk = A.in.blocks + boff;
  const bool fits = blen <= kMaxFastLen;
  STAMP(0);
  const View V = lds_view(s.blk4, uint32_t(kPad + (boff & 15)));
  if (t == 0) {
    s.shift = uint32_t(boff & 15);
    if (fits) row_init(s, LdsRd{V}, blen, flags, true);
    else row_init(s, GlbRd{gblk}, blen, flags, false);
  }
  __syncthreads();
  STAMP(1);

  // ---- P1: run walks + block scan of the per-run sums -----------------------------
  const uint32_t nres = s.nres;
  const uint32_t roff = uint32_t(s.roff);
  const uint32_t S = s.S;
  if (s.status == PBL_OK && !s.slow && roff > 0) {
    // thread t owns run t (nres <= 256) or runs 2t, 2t+1
    const bool two = nres > uint32_t(kTPB);
    uint32_t rA = two ? 2 * t : t, rB = 2 * t + 1;
    uint32_t cA = 0, kA = 0, vA = 0, cB = 0, kB = 0, vB = 0;
    if (rA < nres) walk_run(s, V, rA, nres, roff, S, flags, &cA, &kA, &vA);
    if (two && rB < nres) walk_run(s, V, rB, nres, roff, S, flags, &cB, &kB, &vB);
    STAMP(2);
    uint32_t e[3], tot[3];
    block_excl_scan3(cA + cB, kA + kB, vA + vB, e, tot, s.scratch);
    if (rA < nres) { s.aux[kRunKv0 + rA] = e[0]; s.aux[kRunKb0 + rA] = e[1]; s.aux[kRunVb0 + rA] = e[2]; }
    if (two && rB < nres) {
      s.aux[kRunKv0 + rB] = e[0] + cA; s.aux[kRunKb0 + rB] = e[1] + kA; s.aux[kRunVb0 + rB] = e[2] + vA;
    }
    if (t == 0) {
      s.aux[kRunKv0 + nres] = tot[0];
      s.nkv = tot[0];
      s.tot_kb = tot[1];
      s.tot_vb = tot[2];
      s.kout[tot[0] <= uint32_t(kKvCap) ? tot[0] : 0] = tot[1];
      s.vout[tot[0] <= uint32_t(kKvCap) ? tot[0] : 0] = tot[2];
      if (tot[0] > uint32_t(kKvCap) || tot[1] > kMaxFastKeyBytes) s.slow = 1;
    }
  }
  __syncthreads();
  STAMP(3);

  // ---- general path (wave 0 only) -------------------------------------------------
  if (s.slow && s.status == PBL_OK) {
    // keybuf: the block staging area when the block is read from global memory,
    // else the per-KV arrays (unused on this path)
    uint8_t* keybuf = fits ? reinterpret_cast<uint8_t*>(s.eoff) : reinterpret_cast<uint8_t*>(s.blk4);
    uint32_t keycap = fits ? uint32_t(reinterpret_cast<uint8_t*>(s.scratch) - reinterpret_cast<uint8_t*>(s.eoff))
                           : uint32_t(kLdsBlkBytes);
    const uint8_t* src = fits ? reinterpret_cast<const uint8_t*>(s.blk4) + kPad + s.shift : gblk;
    SlowState ss;
    uint64_t agg[kNumComp], excl[kNumComp];
    uint32_t status = PBL_OK;
    if (wave_id() == 0) {
      uint64_t dummy[kNumComp] = {0, 0, 0, 0};
      slow_walk(src, fits, blen, flags, A.in.synthetic_seq_num, keybuf, keycap, 0, A.out, b, dummy, &ss);
      bool ok = ss.status == PBL_OK;
      agg[0] = ok ? ss.nkv : 0;
      agg[1] = ok ? ss.kb : 0;
      agg[2] = ok ? ss.vb : 0;
      agg[3] = ok ? ss.nr : 0;
      lookback(lb_state, nb, b, agg, excl, &O.totals->status_mask);
      status = ss.status;
      if (ok && overflows(O, excl, agg)) status = PBL_OVERFLOW;
    }
    if (persist) {
      __syncthreads();
      if (t == kWave) next_descriptor(s, A, atomicAdd(reinterpret_cast<uint32_t*>(ws), 1u));
      __syncthreads();
      next_prefetch(s, A, persist, pf);
    }
    if (wave_id() != 0) return;
    if (status == PBL_OK) {
      slow_walk(src, fits, blen, flags, A.in.synthetic_seq_num, keybuf, keycap, 1, A.out, b, excl, &ss);
    } else if (lane_id() == 0 && O.key_off && excl[0] + b < O.kv_cap + nb) {
      O.key_off[excl[0] + b] = 0;
      O.val_off[excl[0] + b] = 0;
    }
    if (lane_id() == 0) write_block_meta(O, b, nb, status, excl, agg, true);
    return;
  }

  // ---- P2 (+ look-back) ------------------------------------------------------------
  const bool ok = s.status == PBL_OK;
  const uint32_t nkv = ok ? s.nkv : 0;
  if (ok && roff > 0 && vprefix) {
    // value-prefix classification needs every trailer kind before the value
    // totals are final: expand with all threads, classify, re-scan values
    for (uint32_t q = t; q < nres * S; q += kTPB) expand_slot(s, V, q, S, roff, flags);
    __syncthreads();
    uint32_t vl2[2];
#pragma unroll
    for (int qq = 0; qq < 2; qq++) {
      uint32_t j = 2 * t + qq;
      vl2[qq] = 0;
      if (j < nkv) {
        uint8_t fl = s.kvf[j];
        uint64_t tr = entry_trailer(s, V, j, &fl, flags);
        uint32_t vs = s.vsrc[j], vl = s.vlen[j];
        if ((tr & 0xff) == 1) {
          if (vl == 0) {
            atomicMax(&s.status, uint32_t(PBL_CORRUPT_BOUNDS));  // Go: i.val[0] panics
          } else {
            uint32_t pre = V.byte(vs);
            if ((pre & 0xC0) == 0 || (flags & PBL_ROW_NO_VALUER)) { vs++; vl--; }
            else if ((pre & 0xC0) == 0x80) fl |= PBL_KV_VALBLK_HANDLE;
            else fl |= PBL_KV_BLOB_HANDLE;
          }
          s.vsrc[j] = uint16_t(vs);
          s.vlen[j] = uint16_t(vl);
        }
        s.kvf[j] = fl;
        vl2[qq] = vl;
      }
    }
    uint32_t ev, ed, tv, td;
    block_excl_scan2(vl2[0] + vl2[1], 0, &ev, &ed, s.scratch, &tv, &td);
    {
      uint32_t j = 2 * t;
      if (j < nkv) s.vout[j] = ev;
      if (j + 1 < nkv) s.vout[j + 1] = ev + vl2[0];
      if (t == 0) { s.vout[nkv] = tv; s.tot_vb = tv; }
    }
    __syncthreads();
  }
  STAMP(4);
  if (wave_id() == 0) {
    uint64_t agg[kNumComp], excl[kNumComp];
    bool okk = s.status == PBL_OK;  // (vprefix classification may have flagged it)
    agg[0] = okk ? nkv : 0;
    agg[1] = okk ? s.tot_kb : 0;
    agg[2] = okk ? s.tot_vb : 0;
    agg[3] = okk ? nres : 0;
    lookback(lb_state, nb, b, agg, excl, &O.totals->status_mask);
    STAMP(9);
    if (lane_id() == 0) {
      uint32_t status = s.status;
      if (okk && overflows(O, excl, agg)) status = PBL_OVERFLOW;
      s.status = status;
#pragma unroll
      for (int c = 0; c < kNumComp; c++) s.bases[c] = excl[c];
      if (status != PBL_OK && O.key_off && excl[0] + b < O.kv_cap + nb) {
        O.key_off[excl[0] + b] = 0;
        O.val_off[excl[0] + b] = 0;
      }
      write_block_meta(O, b, nb, status, excl, agg, false);
    }
  } else if (ok && roff > 0 && !vprefix) {
    // waves 1-3 expand the slots while wave 0 waits on the look-back
    for (uint32_t q = t - kWave; q < nres * S; q += kTPB - kWave) expand_slot(s, V, q, S, roff, flags);
    STAMPT(10, kWave);
  }
  __syncthreads();
  STAMP(5);
  // persistent mode: the next ticket is taken only now, after this block's prefix
  // has resolved (a workgroup never holds a ticket while it waits), and is
  // prefetched during the value copy below
  if (s.status != PBL_OK) {
    if (persist) {
      if (t == kWave) next_descriptor(s, A, atomicAdd(reinterpret_cast<uint32_t*>(ws), 1u));
      __syncthreads();
      next_prefetch(s, A, persist, pf);
    }
    return;
  }

  const uint64_t kvb = s.bases[0], kbb = s.bases[1], vbb = s.bases[2], rbb = s.bases[3];
  // per-KV arrays (coalesced, thread per KV)
  for (uint32_t j = t; j <= nkv; j += kTPB) {
    uint64_t o = kvb + b + j;
    O.key_off[o] = s.kout[j];
    O.val_off[o] = s.vout[j];
    if (j < nkv) {
      uint8_t fl = s.kvf[j];
      O.trailer[kvb + j] = with_seq(entry_trailer(s, V, j, &fl, flags), A.in.synthetic_seq_num, flags);
      if (O.kv_flags) O.kv_flags[kvb + j] = fl;
      if (O.entry_off) O.entry_off[kvb + j] = s.eoff[j];
    }
  }
  if (O.restarts)
    for (uint32_t r = t; r < nres; r += kTPB) O.restarts[rbb + r] = V.le32(roff + 4 * r);
  STAMP(6);
  // the ticket for the next block is taken here (its latency overlaps the key
  // copy); waves 1-3 start its prefetch before the value copy
  if (persist && t == kWave) next_descriptor(s, A, atomicAdd(reinterpret_cast<uint32_t*>(ws), 1u));

  // key bytes: one thread per KV writes its user key (16-B aligned destination
  // granules; the edge granules shared with neighbours as byte-exact partial
  // stores)
  for (uint32_t j = t; j < nkv; j += kTPB) {
    const uint32_t k0 = s.kout[j], k1 = s.kout[j + 1];
    const uint64_t d0 = kbb + k0, d1 = kbb + k1;
    for (uint64_t a = d0 & ~uint64_t(15); a < d1; a += 16) {
      const uint32_t lo = a < d0 ? uint32_t(d0 - a) : 0u, hi = a + 16 <= d1 ? 16u : uint32_t(d1 - a);
      const uint32_t p_lo = uint32_t(a + lo - d0), p_hi = uint32_t(a + hi - d0);
      const uint4 w = key_part(s, V, int(j), k1 - k0, p_lo, p_hi, lo);
      if (lo == 0 && hi == 16) *reinterpret_cast<uint4*>(O.key_bytes + a) = w;
      else store_partial16(O.key_bytes + a, w, lo, hi);
    }
  }
  STAMP(7);
  if (persist) {
    __syncthreads();
    next_prefetch(s, A, persist, pf);
  }
  // value bytes: one thread per KV copies its value (16-B aligned destination
  // granules: whole ones as dwordx4 stores, the two edge granules it shares with
  // its neighbours as byte-exact partial stores) -- no output-to-KV search
  for (uint32_t j = t; j < nkv; j += kTPB) {
    const uint32_t v0 = s.vout[j], n = s.vout[j + 1] - v0;
    const int32_t src = int32_t(s.vsrc[j]);
    const uint64_t d0 = vbb + v0, d1 = d0 + n;
    for (uint64_t a = d0 & ~uint64_t(15); a < d1; a += 16) {
      const uint4 w = V.ld16(src + int32_t(int64_t(a) - int64_t(d0)));
      const uint32_t lo = a < d0 ? uint32_t(d0 - a) : 0u, hi = a + 16 <= d1 ? 16u : uint32_t(d1 - a);
      if (lo == 0 && hi == 16) *reinterpret_cast<uint4*>(O.val_bytes + a) = w;
      else store_partial16(O.val_bytes + a, w, lo, hi);
    }
  }
#ifdef PBL_STAMPS
  __syncthreads();
  STAMP(8);
#endif
}

// Non-persistent form: stage from global memory, then decode (mixed batches).
__device__ __forceinline__ void row_block(Lds& s, const Args& A, const uint32_t b) {
  const uint64_t boff = A.in.block_off[b];
  const uint32_t blen = A.in.block_len[b];
  if (blen <= kMaxFastLen) row_stage(s, A.in.blocks, boff, blen);
  __syncthreads();
  PfRegs unused;
  row_process(s, A, b, boff, blen, false, unused);
}

// Persistent row kernel: each workgroup loops over tickets.  While block `cur`
// writes its outputs, waves 1-3 load the NEXT block into registers (PfRegs), so
// the HBM latency of staging overlaps the previous block's output phase.  The
// next ticket is taken when the current block publishes its aggregate, keeping
// ticket order ~= processing order; the smallest unfinished block always has
// its predecessors published, so the look-back is deadlock-free for any residency.
__global__ void __launch_bounds__(kTPB, 3) rowblk_decode_kernel(Args A) {
  __shared__ Lds s;
  const int t = threadIdx.x;
  const uint32_t nb = A.in.n_blocks;
  PfRegs pf;
  if (t == 0) next_descriptor(s, A, atomicAdd(reinterpret_cast<uint32_t*>(A.out.workspace), 1u));
  __syncthreads();
  next_prefetch(s, A, true, pf);
  while (true) {
    __syncthreads();  // s.nxt is published; the previous block's LDS reads are done
    const uint32_t cur = s.nxt;
    if (cur >= nb) break;
    const uint64_t cur_off = s.nxt_off;
    const uint32_t cur_len = s.nxt_len;
    if (t >= kWave && cur_len <= kMaxFastLen) pf.store(s, cur_off, cur_len);
    __syncthreads();
    row_process(s, A, cur, cur_off, cur_len, true, pf);
  }
}

#include "rowblk_pipe.hip.h"
#include "rowblk_pool.hip.h"
#include "rowblk_res.hip.h"

// Mixed row + colblk batch (config 4): per-block format from block_format[];
// both paths share the ticket order and the look-back state.
union MixedLds {
  Lds row;
  col::Lds col;
};

__global__ void __launch_bounds__(kTPB) mixed_decode_kernel(Args A) {
  __shared__ MixedLds s;
  __shared__ uint32_t ticket;
  if (threadIdx.x == 0) ticket = atomicAdd(reinterpret_cast<uint32_t*>(A.out.workspace), 1u);
  __syncthreads();
  const uint32_t b = ticket;
  const uint32_t fmt = A.in.block_format[b];
  if (fmt == PBL_FMT_ROW) row_block(s.row, A, b);
  else col::col_block(s.col, A, b, fmt);
}

}  // namespace row
}  // namespace pbl

#define PBL_COL_PIPE_BODY_ONLY
#include "colblk_pipe.hip.h"

namespace pbl {
namespace row {

// ---- mixed row + colblk batches, pipelined (config 4) -------------------------------
// The batch's block ids are split by format into two ascending lists
// (mixed_split_*); one persistent launch then runs the row pipeline body
// (rowblk_pipe.hip.h) in its first workgroups and the colblk pipeline body
// (colblk_pipe.hip.h) in the rest, each taking tickets from its own list.
// Both publish into ONE look-back state indexed by the block id, so every
// block's exclusive prefix is over the batch order, as in the single-format
// kernels.  Deadlock-free because every workgroup of the launch is resident
// (persistent grid) and each list is ticketed in ascending id order: the
// smallest unfinished block has been ticketed and all its predecessors have
// published.  The workgroup split follows the lists' lengths weighted by the
// per-block cost of each pipeline (kMixColCost, colblk relative to row, x1000).
#ifndef PBL_MIX_COL_COST
#define PBL_MIX_COL_COST 1300
#endif
#ifndef PBL_MIX_ROW_LB_WIN
#define PBL_MIX_ROW_LB_WIN 2  // measured 2 / 4 / 8 windows: 965 / 954 / 946 GiB/s on config 4
#endif

__global__ void __launch_bounds__(kTPB) mixed_split_count_kernel(Args A, uint32_t* counts) {
  const uint32_t nb = A.in.n_blocks;
  const uint32_t c0 = blockIdx.x * kSplitChunk;
  uint32_t k = 0;
  for (uint32_t i = c0 + threadIdx.x; i < nb && i < c0 + kSplitChunk; i += kTPB)
    k += to_glb(A.in.block_format)[i] == PBL_FMT_ROW;
  __shared__ uint32_t red[kTPB / kWave];
  k = wave_sum(k);
  if (lane_id() == 0) red[wave_id()] = k;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t s = 0;
    for (int w = 0; w < kTPB / kWave; w++) s += red[w];
    counts[blockIdx.x] = s;
  }
}

__global__ void __launch_bounds__(kTPB) mixed_split_scatter_kernel(Args A, const uint32_t* counts, uint32_t n_chunks,
                                                                   uint32_t* ids) {
  const uint32_t nb = A.in.n_blocks;
  const uint32_t c = blockIdx.x;
  __shared__ uint32_t sc[kTPB];
  __shared__ uint32_t base_row, base_col;
  if (threadIdx.x == 0) {
    uint32_t before = 0, total = 0;
    for (uint32_t i = 0; i < n_chunks; i++) {
      const uint32_t x = to_glb(counts)[i];
      if (i < c) before += x;
      total += x;
    }
    base_row = before;
    base_col = total + (c * kSplitChunk - before);  // col ids follow all row ids
    if (c == 0) to_glb(reinterpret_cast<uint32_t*>(A.out.workspace))[kWsRowCount] = total;
  }
  __syncthreads();
  // in-order compaction of the chunk, kTPB ids at a time
  for (uint32_t i0 = c * kSplitChunk; i0 < nb && i0 < (c + 1) * kSplitChunk; i0 += kTPB) {
    const uint32_t i = i0 + threadIdx.x;
    const bool live = i < nb && i < (c + 1) * kSplitChunk;
    const uint32_t isrow = live && to_glb(A.in.block_format)[i] == PBL_FMT_ROW;
    sc[threadIdx.x] = isrow;
    __syncthreads();
    // inclusive scan (Hillis-Steele over kTPB entries)
    for (uint32_t d = 1; d < kTPB; d <<= 1) {
      const uint32_t v = threadIdx.x >= d ? sc[threadIdx.x - d] : 0u;
      __syncthreads();
      sc[threadIdx.x] += v;
      __syncthreads();
    }
    const uint32_t incl = sc[threadIdx.x], nrow = sc[kTPB - 1];
    const uint32_t nlive = (nb - i0 < kTPB ? nb - i0 : kTPB);
    if (live) {
      if (isrow) to_glb(ids)[base_row + incl - 1] = i;
      else to_glb(ids)[base_col + (threadIdx.x - (incl - isrow))] = i;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      base_row += nrow;
      base_col += nlive - nrow;
    }
    __syncthreads();
  }
}

// Mixed batches: three persistent launches over the split id lists.  (A single
// launch running both pipeline bodies, the first form, measured 892 against
// 976 GiB/s on config 4.)  (1) mixed_col_size_kernel parses every
// colblk block and publishes its aggregate; (2) mixed_row_kernel runs the row
// pipeline over the row list, its look-back walking through the colblk
// aggregates; (3) mixed_col_kernel runs the colblk pipeline over the colblk
// list (its predecessors' prefixes are all published: its look-back ends at
// the row block before it).  Each launch gets its own occupancy (row 2, colblk
// 3 workgroups per CU) and its own code: the single mixed launch holds both
// bodies under the union LDS layout (2 workgroups per CU for both roles) and
// its roles advance at the pace of the slower one.  Deadlock-free: (2) waits
// only on aggregates published by (1) or by its own resident workgroups in
// ticket order, (3) on aggregates published by (1) and its own workgroups.
constexpr int kWsColTick2 = 4;  // header u32 [4]: the colblk queue of launch (3)

// (1): one wave per colblk block, straight from global memory (no staging: a
// size needs the header, the key columns' offsets and the value bounds only),
// many waves per CU to hide the latency (measured: a 256-thread workgroup per
// block 0.73 ms, a wave per block 0.47 ms on config 4's 64 Ki colblk blocks).
// Same parse_block_wave / row_parts / value_ok as the pipeline, so the
// aggregate is the one the pipeline publishes again in (3).
#ifndef PBL_COL_SIZE_WAVES
#define PBL_COL_SIZE_WAVES 8  // waves per SIMD (64 VGPRs): config 4 951 at 4 (101 VGPRs), 975 at 8
#endif
// kHide (PBL_ROW_HIDE_OBSOLETE): the aggregate counts the visible rows, as
// col_rows_hide publishes it again in (3).
template <bool kHide>
__global__ void __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(PBL_COL_SIZE_WAVES)))
mixed_col_size_kernel(Args A, const uint32_t* ids) {
  __shared__ col::Desc d;
  const uint32_t nb = A.in.n_blocks;
  uint32_t* hdr = reinterpret_cast<uint32_t*>(A.out.workspace);
  uint64_t* lb_state = reinterpret_cast<uint64_t*>(reinterpret_cast<uint8_t*>(A.out.workspace) + kWsHeader);
  const uint32_t n_row = __hip_atomic_load(to_glb(hdr) + kWsRowCount, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t n_col = nb - n_row;
  for (uint32_t i = blockIdx.x; i < n_col; i += gridDim.x) {
    const uint32_t b = to_glb(ids)[n_row + i];
    const uint32_t blen = to_glb(A.in.block_len)[b];
    const uint32_t schema = to_glb(A.in.block_format)[b];
    const col::Src S{nullptr, nullptr, (col::glb_cu8)(A.in.blocks + to_glb(A.in.block_off)[b]), 0u, 0xffffffffu, blen};
    uint32_t st = col::parse_block_wave(S, schema, &d);
    const uint32_t rows = st == PBL_OK ? d.rows : 0;
    uint64_t kb = 0, nv = 0, vb = 0;
    bool bad = false;
    // (not unrolled: 4 rows per lane in flight measured 0.89 against 0.47 ms)
    for (uint32_t r = lane_id(); r < rows; r += kWave) {
      const col::RowParts p = col::row_parts<false>(S, d, schema, r);
      bad |= !p.ok || !col::value_ok(S, d, r);
      if (!kHide || !col::row_obsolete(S, d, r)) {
        kb += p.klen;
        if (kHide) {
          nv++;
          vb += col::row_voff(S, d, r + 1) - col::row_voff(S, d, r);
        }
      }
    }
    kb = wave_sum(kb);
    if (kHide) {
      nv = wave_sum(nv);
      vb = wave_sum(vb);
    } else {
      nv = rows;
      vb = uint64_t(d.v_hi - d.v_lo);
    }
    if (st == PBL_OK) {
      if (__ballot(bad)) st = PBL_CORRUPT_BOUNDS;
      else if (kb > 0xffffffffull || vb > 0xffffffffull) st = PBL_UNSUPPORTED;
    }
    const bool ok = st == PBL_OK;
    const uint64_t agg[kNumComp] = {ok ? nv : 0u, ok ? kb : 0ull, ok ? vb : 0ull, 0ull};
    lb_publish(lb_state, nb, b, agg);
    wave_sync();  // (d is rewritten by the next block's parse)
  }
}

__global__ void __launch_bounds__(pipe::kPTPB) __attribute__((amdgpu_waves_per_eu(PBL_PIPE_WAVES / 2, PBL_PIPE_WAVES / 2)))
mixed_row_kernel(Args A, const uint32_t* ids) {
  __shared__ pipe::PLds S;
  const uint32_t nb = A.in.n_blocks;
  uint32_t* hdr = reinterpret_cast<uint32_t*>(A.out.workspace);
  const uint32_t n_row = __hip_atomic_load(to_glb(hdr) + kWsRowCount, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // (its look-back walks over the interleaved colblk aggregates as well)
  pipe::row_pipe_body<true, ListQueue, PBL_MIX_ROW_LB_WIN>(S, A, ListQueue{hdr, ids, n_row, nb});
}

__global__ void __launch_bounds__(kTPB, PBL_COL_PIPE_WG) mixed_col_kernel(Args A, const uint32_t* ids) {
  __shared__ col::cpipe::CLds L;
  const uint32_t nb = A.in.n_blocks;
  uint32_t* hdr = reinterpret_cast<uint32_t*>(A.out.workspace);
  const uint32_t n_row = __hip_atomic_load(to_glb(hdr) + kWsRowCount, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  col::cpipe::col_pipe_body(L, A, ListQueue{hdr + kWsColTick2, ids + n_row, nb - n_row, nb});
}

// (3) with HideObsoletePoints fused: the one-block-per-workgroup colblk form
// (col_rows_hide) over the colblk list, in ticket order; every row block has
// its inclusive prefix by now.
__global__ void __launch_bounds__(kTPB) mixed_col_hide_kernel(Args A, const uint32_t* ids) {
  __shared__ col::Lds s;
  __shared__ uint32_t tk;
  const uint32_t nb = A.in.n_blocks;
  uint32_t* hdr = reinterpret_cast<uint32_t*>(A.out.workspace);
  const uint32_t n_row = __hip_atomic_load(to_glb(hdr) + kWsRowCount, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (;;) {
    if (threadIdx.x == 0) tk = g_atomic_add(hdr + kWsColTick2, 1u);
    __syncthreads();
    const uint32_t t = tk;
    if (t >= nb - n_row) break;
    const uint32_t b = to_glb(ids)[n_row + t];
    col::col_block<true>(s, A, b, to_glb(A.in.block_format)[b]);
    __syncthreads();  // (the LDS and tk are the next block's)
  }
}

// Size pass epilogue: a block that decoded reports PBL_OK, not the forced
// overflow of the pass.
__global__ void size_fixup_kernel(uint32_t* blk_status, pbl_totals* totals, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) __hip_atomic_fetch_and(&totals->status_mask, ~(1u << PBL_OVERFLOW), __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
  if (i < n && blk_status[i] == PBL_OVERFLOW) {
    blk_status[i] = PBL_OK;
    g_atomic_add(&totals->n_bad_blocks, ~0u);  // (-1)
  }
}

__global__ void rebase_kernel(uint64_t* kvb, uint64_t* kb, uint64_t* vb, uint64_t* rb, uint32_t n,
                              uint64_t dkv, uint64_t dk, uint64_t dv, uint64_t dr) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > n) return;
  kvb[i] += dkv;
  kb[i] += dk;
  vb[i] += dv;
  if (rb) rb[i] += dr;
}

__global__ void offset_concat_kernel(uint64_t* kvb, uint64_t* kb, uint64_t* vb, uint64_t* rb, uint32_t n,
                                     const uint64_t* rank_totals, uint32_t rank) {
  uint64_t d[4] = {0, 0, 0, 0};
  for (uint32_t r = 0; r < rank; r++)
    for (int c = 0; c < 4; c++) d[c] += rank_totals[4 * r + c];
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += gridDim.x * blockDim.x) {
    kvb[i] += d[0];
    kb[i] += d[1];
    vb[i] += d[2];
    if (rb) rb[i] += d[3];
  }
}

}  // namespace row
}  // namespace pbl

namespace pbl {

namespace {
constexpr int kMaxDevices = 64;
std::atomic<int> g_cus[kMaxDevices];
std::atomic<int> g_per_cu[kMaxDevices][kKNum];
}  // namespace

uint64_t persistent_grid(hipStream_t st, PersistentKernel k, const void* fn, uint64_t n_units, int* cus_out,
                         int block_threads) {
  int dev = -1;
  if (st ? hipStreamGetDevice(st, &dev) != hipSuccess : hipGetDevice(&dev) != hipSuccess) return 0;
  if (dev < 0 || dev >= kMaxDevices) return 0;
  int cus = g_cus[dev].load(std::memory_order_relaxed);
  int per_cu = g_per_cu[dev][k].load(std::memory_order_relaxed);
  if (cus <= 0 || per_cu <= 0) {
    // the occupancy query answers for the current device: switch to the
    // stream's device for it and back
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess) return 0;
    if (cur != dev && hipSetDevice(dev) != hipSuccess) return 0;
    const bool ok = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
                    hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, block_threads, 0) == hipSuccess;
    if (cur != dev) (void)hipSetDevice(cur);
    if (!ok) return 0;
    cus = cus > 0 ? cus : 1;
    per_cu = per_cu > 0 ? per_cu : 1;
    g_cus[dev].store(cus, std::memory_order_relaxed);
    g_per_cu[dev][k].store(per_cu, std::memory_order_relaxed);
  }
  if (cus_out) *cus_out = cus;
  uint64_t grid = uint64_t(cus) * uint64_t(per_cu);
  if (grid > n_units) grid = n_units;
  return grid ? grid : 1;
}

}  // namespace pbl

namespace {
// Row batches on the staging-pool kernel (rowblk_pool.hip.h), with the same
// big-block passes around it.
int launch_row_pool(const pbl::Args& a, hipStream_t st, bool values) {
  const uint32_t nb = a.in.n_blocks;
  const bool hide = (a.in.flags & PBL_ROW_HIDE_OBSOLETE) && !(a.in.flags & PBL_ROW_RAW_KEYS);
  const void* fn = hide ? reinterpret_cast<const void*>(pbl::row::pool::rowblk_pool_kernel<true>)
                        : reinterpret_cast<const void*>(pbl::row::pool::rowblk_pool_kernel<false>);
  int cus = 0;
  const uint64_t grid = pbl::persistent_grid(st, pbl::kKRowPool, fn,
                                             (uint64_t(nb) + pbl::row::pool::kNW - 1) / pbl::row::pool::kNW, &cus,
                                             pbl::row::pool::kTPBP);
  if (!grid) return PBL_DEVICE_ERROR;
  const uint32_t small = uint32_t(std::min<uint64_t>(nb, uint64_t(cus > 0 ? cus : 1) * 4));
  hipLaunchKernelGGL(pbl::row::pipe::big_block_sizes_kernel, dim3(small), dim3(pbl::kWave), 0, st, a);
  if (hide)
    hipLaunchKernelGGL(pbl::row::pool::rowblk_pool_kernel<true>, dim3(uint32_t(grid)), dim3(pbl::row::pool::kTPBP), 0,
                       st, a, static_cast<const uint32_t*>(nullptr));
  else
    hipLaunchKernelGGL(pbl::row::pool::rowblk_pool_kernel<false>, dim3(uint32_t(grid)), dim3(pbl::row::pool::kTPBP),
                       0, st, a, static_cast<const uint32_t*>(nullptr));
  if (values) hipLaunchKernelGGL(pbl::row::pipe::big_block_values_kernel, dim3(small), dim3(pbl::kWave), 0, st, a);
  return hipGetLastError() == hipSuccess ? PBL_OK : PBL_DEVICE_ERROR;
}

// Row batches on the block-resident kernel (rowblk_res.hip.h), with the same
// big-block passes around it.
int launch_row_res(const pbl::Args& a, hipStream_t st, bool values) {
  const uint32_t nb = a.in.n_blocks;
  const bool hide = (a.in.flags & PBL_ROW_HIDE_OBSOLETE) && !(a.in.flags & PBL_ROW_RAW_KEYS);
  const void* fn = hide ? reinterpret_cast<const void*>(pbl::row::res::rowblk_res_kernel<true>)
                        : reinterpret_cast<const void*>(pbl::row::res::rowblk_res_kernel<false>);
  int cus = 0;
  const uint64_t grid = pbl::persistent_grid(st, pbl::kKRowRes, fn,
                                             (uint64_t(nb) + pbl::row::res::kNW - 1) / pbl::row::res::kNW, &cus,
                                             pbl::row::res::kTPBR);
  if (!grid) return PBL_DEVICE_ERROR;
  const uint32_t small = uint32_t(std::min<uint64_t>(nb, uint64_t(cus > 0 ? cus : 1) * 4));
  hipLaunchKernelGGL(pbl::row::pipe::big_block_sizes_kernel, dim3(small), dim3(pbl::kWave), 0, st, a);
  if (hide)
    hipLaunchKernelGGL(pbl::row::res::rowblk_res_kernel<true>, dim3(uint32_t(grid)), dim3(pbl::row::res::kTPBR), 0,
                       st, a, static_cast<const uint32_t*>(nullptr));
  else
    hipLaunchKernelGGL(pbl::row::res::rowblk_res_kernel<false>, dim3(uint32_t(grid)), dim3(pbl::row::res::kTPBR), 0,
                       st, a, static_cast<const uint32_t*>(nullptr));
  if (values) hipLaunchKernelGGL(pbl::row::pipe::big_block_values_kernel, dim3(small), dim3(pbl::kWave), 0, st, a);
  return hipGetLastError() == hipSuccess ? PBL_OK : PBL_DEVICE_ERROR;
}

// HideObsoletePoints fused into the decode: the row staging-pool kernel (and
// the general walk it hands blocks to) and the colblk kernels implement it;
// other row kernels are A/B forms only, so such batches always take the pool.
bool hide_row(const pbl_block_batch* b) {
  return (b->flags & PBL_ROW_HIDE_OBSOLETE) && !(b->flags & PBL_ROW_RAW_KEYS) && !b->block_format &&
         b->format == PBL_FMT_ROW;
}

#ifndef PBL_MIXED_POOL
#define PBL_MIXED_POOL 1  // mixed batches' row blocks on the staging-pool kernel (0: the row pipeline)
#endif
// Mixed batches: PBL_KERNEL_SINGLE keeps the one-block-per-workgroup kernel
// (A/B); the default splits the ids by format and runs the mixed pipeline,
// with the big row blocks' size / value passes around it.
int launch_mixed(const pbl_block_batch* batch, const pbl::Args& a, hipStream_t st, bool single, bool values) {
  // HideObsoletePoints: colblk rows by their isObsolete bit, row entries by
  // their trailer's obsolete bit unless the keys are raw
  const bool hide = (batch->flags & PBL_ROW_HIDE_OBSOLETE) != 0;
  const bool hide_rows = hide && !(batch->flags & PBL_ROW_RAW_KEYS);
  if (single && !hide) {
    hipLaunchKernelGGL(pbl::row::mixed_decode_kernel, dim3(batch->n_blocks), dim3(pbl::kTPB), 0, st, a);
    return hipGetLastError() == hipSuccess ? PBL_OK : PBL_DEVICE_ERROR;
  }
  const uint32_t nb = batch->n_blocks;
  uint8_t* ws = reinterpret_cast<uint8_t*>(a.out.workspace);
  uint32_t* ids = reinterpret_cast<uint32_t*>(ws + pbl::ws_ids_offset(nb));
  uint32_t* counts = ids + nb;
  const uint32_t nch = (nb + pbl::kSplitChunk - 1) / pbl::kSplitChunk;
  hipLaunchKernelGGL(pbl::row::mixed_split_count_kernel, dim3(nch), dim3(pbl::kTPB), 0, st, a, counts);
  hipLaunchKernelGGL(pbl::row::mixed_split_scatter_kernel, dim3(nch), dim3(pbl::kTPB), 0, st, a,
                     static_cast<const uint32_t*>(counts), nch, ids);
  int cus = 0;
  const uint64_t g_r = pbl::persistent_grid(st, pbl::kKMixedRow, reinterpret_cast<const void*>(pbl::row::mixed_row_kernel),
                                            nb, &cus, pbl::row::pipe::kPTPB);
  const uint64_t g_c = pbl::persistent_grid(st, pbl::kKMixedCol, reinterpret_cast<const void*>(pbl::row::mixed_col_kernel),
                                            nb, &cus);
  if (!g_r || !g_c) return PBL_DEVICE_ERROR;
  const uint32_t g_cs = uint32_t(std::min<uint64_t>(nb, uint64_t(cus > 0 ? cus : 1) * 32));
  const uint32_t small = uint32_t(std::min<uint64_t>(nb, uint64_t(cus > 0 ? cus : 1) * 4));
  const uint32_t* cids = static_cast<const uint32_t*>(ids);
  hipLaunchKernelGGL(pbl::row::pipe::big_block_sizes_kernel, dim3(small), dim3(pbl::kWave), 0, st, a);
  if (hide)
    hipLaunchKernelGGL(pbl::row::mixed_col_size_kernel<true>, dim3(g_cs), dim3(pbl::kWave), 0, st, a, cids);
  else
    hipLaunchKernelGGL(pbl::row::mixed_col_size_kernel<false>, dim3(g_cs), dim3(pbl::kWave), 0, st, a, cids);
#if PBL_MIXED_POOL
  // the row blocks on the staging-pool kernel, over the row id list
  const void* pfn = hide_rows ? reinterpret_cast<const void*>(pbl::row::pool::rowblk_pool_kernel<true>)
                              : reinterpret_cast<const void*>(pbl::row::pool::rowblk_pool_kernel<false>);
  const uint64_t g_p = pbl::persistent_grid(st, pbl::kKRowPool, pfn,
                                            (uint64_t(nb) + pbl::row::pool::kNW - 1) / pbl::row::pool::kNW, &cus,
                                            pbl::row::pool::kTPBP);
  if (!g_p) return PBL_DEVICE_ERROR;
  (void)g_r;
  if (hide_rows)
    hipLaunchKernelGGL(pbl::row::pool::rowblk_pool_kernel<true>, dim3(uint32_t(g_p)), dim3(pbl::row::pool::kTPBP), 0,
                       st, a, cids);
  else
    hipLaunchKernelGGL(pbl::row::pool::rowblk_pool_kernel<false>, dim3(uint32_t(g_p)), dim3(pbl::row::pool::kTPBP), 0,
                       st, a, cids);
#else
  hipLaunchKernelGGL(pbl::row::mixed_row_kernel, dim3(uint32_t(g_r)), dim3(pbl::row::pipe::kPTPB), 0, st, a, cids);
#endif
  if (hide)  // (workgroups loop over the colblk list's tickets; 21 KB of LDS each)
    hipLaunchKernelGGL(pbl::row::mixed_col_hide_kernel, dim3(uint32_t(std::min<uint64_t>(nb, uint64_t(cus) * 7))),
                       dim3(pbl::kTPB), 0, st, a, cids);
  else
    hipLaunchKernelGGL(pbl::row::mixed_col_kernel, dim3(uint32_t(g_c)), dim3(pbl::kTPB), 0, st, a, cids);
  if (values)
    hipLaunchKernelGGL(pbl::row::pipe::big_block_values_kernel, dim3(small), dim3(pbl::kWave), 0, st, a);
  return hipGetLastError() == hipSuccess ? PBL_OK : PBL_DEVICE_ERROR;
}
}  // namespace

extern "C" {

int pbl_abi_version(void) { return PBL_ABI_VERSION; }

uint64_t pbl_workspace_bytes(uint32_t n_blocks) { return pbl::ws_alloc_bytes(n_blocks); }

int pbl_decode_batch_colblk(const pbl_block_batch* batch, pbl_decode_out* out, void* stream);

int pbl_decode_batch(const pbl_block_batch* batch, pbl_decode_out* out, void* stream) {
  if (!batch || !out || (batch->synthetic_seq_num >> 56)) return PBL_INVALID_ARG;  // (base.SeqNumMax)
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (!out->totals || !out->blk_kv_base || !out->blk_key_base || !out->blk_val_base || !out->blk_status)
    return PBL_INVALID_ARG;
  if (hipMemsetAsync(out->totals, 0, sizeof(pbl_totals), st) != hipSuccess) return PBL_DEVICE_ERROR;
  if (batch->n_blocks == 0) return PBL_OK;
  if (!batch->blocks || !batch->block_off || !batch->block_len || !out->trailer || !out->key_off ||
      !out->val_off || !out->key_bytes || !out->val_bytes || !out->workspace ||
      out->workspace_bytes < pbl::ws_alloc_bytes(batch->n_blocks))
    return PBL_INVALID_ARG;
  if (!batch->block_format && batch->format != PBL_FMT_ROW) return pbl_decode_batch_colblk(batch, out, stream);
  if (hipMemsetAsync(out->workspace, 0, pbl::ws_bytes(batch->n_blocks), st) != hipSuccess)
    return PBL_DEVICE_ERROR;
  pbl::Args a;
  a.in = *batch;
  a.out = *out;
  if (batch->block_format) {
    const int rc = launch_mixed(batch, a, st, batch->flags & PBL_KERNEL_SINGLE, true);
    if (rc != PBL_OK) return rc;
  } else {
    // Row batches take the staging-pool kernel (every block shape: the fast
    // path, the general walk, the big-block passes around it; HideObsoletePoints
    // fused).  PBL_KERNEL_SINGLE / PBL_KERNEL_PIPE keep the one-block-per-
    // workgroup kernel and the two-stage pipeline for A/B measurement.
    const bool single = (batch->flags & PBL_KERNEL_SINGLE) != 0;
    if (batch->flags & PBL_KERNEL_RES) return launch_row_res(a, st, true);
    if (hide_row(batch) || !(batch->flags & (PBL_KERNEL_SINGLE | PBL_KERNEL_PIPE))) return launch_row_pool(a, st, true);
    const void* fn = single ? reinterpret_cast<const void*>(pbl::row::rowblk_decode_kernel)
                            : reinterpret_cast<const void*>(pbl::row::pipe::rowblk_pipe_kernel);
    int cus = 0;
    const uint64_t grid = pbl::persistent_grid(st, single ? pbl::kKRowSingle : pbl::kKRowPipe, fn,
                                         batch->n_blocks, &cus,
                                         single ? pbl::kTPB : pbl::row::pipe::kPTPB);
    if (!grid) return PBL_DEVICE_ERROR;
    if (single)
      hipLaunchKernelGGL(pbl::row::rowblk_decode_kernel, dim3(uint32_t(grid)), dim3(pbl::kTPB), 0, st, a);
    else {
      // sizes of the blocks past the LDS stage first (one wave each, all at once)
      hipLaunchKernelGGL(pbl::row::pipe::big_block_sizes_kernel, dim3(uint32_t(std::min<uint64_t>(
                             batch->n_blocks, uint64_t(cus > 0 ? cus : 1) * 4))), dim3(pbl::kWave), 0, st, a);
      hipLaunchKernelGGL(pbl::row::pipe::rowblk_pipe_kernel, dim3(uint32_t(grid)), dim3(pbl::row::pipe::kPTPB), 0,
                         st, a);
      // then their value bytes (all big blocks at once, bandwidth-bound)
      hipLaunchKernelGGL(pbl::row::pipe::big_block_values_kernel, dim3(uint32_t(std::min<uint64_t>(
                             batch->n_blocks, uint64_t(cus > 0 ? cus : 1) * 4))), dim3(pbl::kWave), 0, st, a);
    }
  }
  return hipGetLastError() == hipSuccess ? PBL_OK : PBL_DEVICE_ERROR;
}

int pbl_size_batch(const pbl_block_batch* batch, pbl_decode_out* out, void* stream) {
  if (!batch || !out || (batch->synthetic_seq_num >> 56)) return PBL_INVALID_ARG;
  if (!out->totals || !out->blk_kv_base || !out->blk_key_base || !out->blk_val_base || !out->blk_status)
    return PBL_INVALID_ARG;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (batch->n_blocks == 0) return pbl_decode_batch(batch, out, stream);
  if (!batch->blocks || !batch->block_off || !batch->block_len || !out->workspace ||
      out->workspace_bytes < pbl::ws_alloc_bytes(batch->n_blocks))
    return PBL_INVALID_ARG;
  // the decode with every per-KV pointer NULL and zero capacities: each block
  // takes its overflow branch (sizes computed and published, nothing written);
  // the fixup then reports the statuses the decode would have had
  pbl_decode_out o = *out;
  o.trailer = nullptr;
  o.kv_flags = nullptr;
  o.entry_off = nullptr;
  o.key_off = nullptr;
  o.val_off = nullptr;
  o.key_bytes = nullptr;
  o.val_bytes = nullptr;
  o.restarts = nullptr;
  o.kv_cap = o.key_cap = o.val_cap = o.rst_cap = 0;
  if (hipMemsetAsync(o.totals, 0, sizeof(pbl_totals), st) != hipSuccess) return PBL_DEVICE_ERROR;
  if (hipMemsetAsync(o.workspace, 0, pbl::ws_bytes(batch->n_blocks), st) != hipSuccess) return PBL_DEVICE_ERROR;
  pbl::Args a;
  a.in = *batch;
  a.out = o;
  int rc = PBL_OK;
  if (!batch->block_format && batch->format != PBL_FMT_ROW) {
    rc = pbl_decode_batch_colblk(batch, &o, stream);
  } else {
    // the launch sequence of pbl_decode_batch (whose checks require output
    // pointers), minus the big-block value pass
    if (batch->block_format) {
      rc = launch_mixed(batch, a, st, batch->flags & PBL_KERNEL_SINGLE, false);
      if (rc != PBL_OK) return rc;
    } else if (batch->flags & PBL_KERNEL_RES) {
      rc = launch_row_res(a, st, false);
      if (rc != PBL_OK) return rc;
    } else if (hide_row(batch) || !(batch->flags & PBL_KERNEL_PIPE)) {
      rc = launch_row_pool(a, st, false);
      if (rc != PBL_OK) return rc;
    } else {
      int cus = 0;
      const uint64_t grid = pbl::persistent_grid(
          st, pbl::kKRowPipe, reinterpret_cast<const void*>(pbl::row::pipe::rowblk_pipe_kernel), batch->n_blocks,
          &cus, pbl::row::pipe::kPTPB);
      if (!grid) return PBL_DEVICE_ERROR;
      const uint32_t small = uint32_t(std::min<uint64_t>(batch->n_blocks, uint64_t(cus) * 4));
      hipLaunchKernelGGL(pbl::row::pipe::big_block_sizes_kernel, dim3(small), dim3(pbl::kWave), 0, st, a);
      hipLaunchKernelGGL(pbl::row::pipe::rowblk_pipe_kernel, dim3(uint32_t(grid)), dim3(pbl::row::pipe::kPTPB), 0,
                         st, a);
    }
    if (hipGetLastError() != hipSuccess) rc = PBL_DEVICE_ERROR;
  }
  if (rc != PBL_OK) return rc;
  hipLaunchKernelGGL(pbl::row::size_fixup_kernel, dim3((batch->n_blocks + 255) / 256), dim3(256), 0, st,
                     o.blk_status, o.totals, batch->n_blocks);
  return hipGetLastError() == hipSuccess ? PBL_OK : PBL_DEVICE_ERROR;
}

size_t pbl_struct_layout(uint64_t* out, size_t cap) {
#define PBL_OFF(T, f) uint64_t(offsetof(T, f))
  const uint64_t v[] = {
      sizeof(pbl_block_batch), PBL_OFF(pbl_block_batch, blocks), PBL_OFF(pbl_block_batch, block_off),
      PBL_OFF(pbl_block_batch, block_len), PBL_OFF(pbl_block_batch, n_blocks), PBL_OFF(pbl_block_batch, format),
      PBL_OFF(pbl_block_batch, flags), PBL_OFF(pbl_block_batch, reserved), PBL_OFF(pbl_block_batch, block_format),
      PBL_OFF(pbl_block_batch, synthetic_seq_num),
      sizeof(pbl_totals), PBL_OFF(pbl_totals, n_kv), PBL_OFF(pbl_totals, key_bytes), PBL_OFF(pbl_totals, val_bytes),
      PBL_OFF(pbl_totals, n_restarts), PBL_OFF(pbl_totals, status_mask), PBL_OFF(pbl_totals, n_bad_blocks),
      PBL_OFF(pbl_totals, n_slow_blocks), PBL_OFF(pbl_totals, pad),
      sizeof(pbl_decode_out), PBL_OFF(pbl_decode_out, trailer), PBL_OFF(pbl_decode_out, kv_flags),
      PBL_OFF(pbl_decode_out, entry_off), PBL_OFF(pbl_decode_out, key_off), PBL_OFF(pbl_decode_out, val_off),
      PBL_OFF(pbl_decode_out, key_bytes), PBL_OFF(pbl_decode_out, val_bytes), PBL_OFF(pbl_decode_out, restarts),
      PBL_OFF(pbl_decode_out, blk_kv_base), PBL_OFF(pbl_decode_out, blk_key_base),
      PBL_OFF(pbl_decode_out, blk_val_base), PBL_OFF(pbl_decode_out, blk_rst_base),
      PBL_OFF(pbl_decode_out, blk_status), PBL_OFF(pbl_decode_out, totals), PBL_OFF(pbl_decode_out, kv_cap),
      PBL_OFF(pbl_decode_out, key_cap), PBL_OFF(pbl_decode_out, val_cap), PBL_OFF(pbl_decode_out, rst_cap),
      PBL_OFF(pbl_decode_out, workspace), PBL_OFF(pbl_decode_out, workspace_bytes),
      sizeof(pbl_transforms), PBL_OFF(pbl_transforms, synthetic_seq_num),
      PBL_OFF(pbl_transforms, hide_obsolete_points), PBL_OFF(pbl_transforms, split), PBL_OFF(pbl_transforms, prefix),
      PBL_OFF(pbl_transforms, suffix), PBL_OFF(pbl_transforms, prefix_len), PBL_OFF(pbl_transforms, suffix_len),
      PBL_OFF(pbl_transforms, blocks),
      sizeof(pbl_footer), PBL_OFF(pbl_footer, table_format), PBL_OFF(pbl_footer, checksum_type),
      PBL_OFF(pbl_footer, metaindex_off), PBL_OFF(pbl_footer, metaindex_len), PBL_OFF(pbl_footer, index_off),
      PBL_OFF(pbl_footer, index_len), PBL_OFF(pbl_footer, footer_off), PBL_OFF(pbl_footer, footer_len),
      PBL_OFF(pbl_footer, attributes), PBL_OFF(pbl_footer, reserved),
      sizeof(pbl_index_out), PBL_OFF(pbl_index_out, handle_off), PBL_OFF(pbl_index_out, handle_len),
      PBL_OFF(pbl_index_out, props_off), PBL_OFF(pbl_index_out, props_len), PBL_OFF(pbl_index_out, blk_base),
      PBL_OFF(pbl_index_out, blk_status), PBL_OFF(pbl_index_out, cap),
      sizeof(pbl_kv_out), PBL_OFF(pbl_kv_out, key_off), PBL_OFF(pbl_kv_out, key_len), PBL_OFF(pbl_kv_out, val_off),
      PBL_OFF(pbl_kv_out, val_len), PBL_OFF(pbl_kv_out, blk_base), PBL_OFF(pbl_kv_out, blk_status),
      PBL_OFF(pbl_kv_out, cap),
      sizeof(pbl_value_out), PBL_OFF(pbl_value_out, val_off), PBL_OFF(pbl_value_out, val_bytes),
      PBL_OFF(pbl_value_out, blk_val_base), PBL_OFF(pbl_value_out, blk_status), PBL_OFF(pbl_value_out, val_cap),
      sizeof(pbl_kv), PBL_OFF(pbl_kv, user_key), PBL_OFF(pbl_kv, user_key_len), PBL_OFF(pbl_kv, trailer),
      PBL_OFF(pbl_kv, value), PBL_OFF(pbl_kv, value_len), PBL_OFF(pbl_kv, kv_flags), PBL_OFF(pbl_kv, reserved)};
#undef PBL_OFF
  const size_t n = sizeof(v) / sizeof(v[0]);
  for (size_t i = 0; i < n && i < cap && out; i++) out[i] = v[i];
  return n;
}

int pbl_rebase_blocks(pbl_decode_out* out, uint32_t n_blocks, uint64_t kv_base, uint64_t key_base,
                      uint64_t val_base, uint64_t rst_base, void* stream) {
  if (!out || !out->blk_kv_base || !out->blk_key_base || !out->blk_val_base) return PBL_INVALID_ARG;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  uint32_t n = n_blocks + 1;
  hipLaunchKernelGGL(pbl::row::rebase_kernel, dim3((n + 255) / 256), dim3(256), 0, st, out->blk_kv_base,
                     out->blk_key_base, out->blk_val_base, out->blk_rst_base, n_blocks, kv_base, key_base,
                     val_base, rst_base);
  return hipGetLastError() == hipSuccess ? PBL_OK : PBL_DEVICE_ERROR;
}

int pbl_offset_concat(pbl_decode_out* out, uint32_t n_blocks, const uint64_t* rank_totals, uint32_t rank,
                      void* stream) {
  if (!out || !rank_totals || !out->blk_kv_base || !out->blk_key_base || !out->blk_val_base)
    return PBL_INVALID_ARG;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  uint32_t n = n_blocks + 1;
  uint32_t grid = (n + 255) / 256;
  if (grid > 1024) grid = 1024;
  hipLaunchKernelGGL(pbl::row::offset_concat_kernel, dim3(grid), dim3(256), 0, st, out->blk_kv_base,
                     out->blk_key_base, out->blk_val_base, out->blk_rst_base, n_blocks, rank_totals, rank);
  return hipGetLastError() == hipSuccess ? PBL_OK : PBL_DEVICE_ERROR;
}

}  // extern "C"
