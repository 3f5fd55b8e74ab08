// rowblk_pipe.hip.h — the row-format decode as a two-stage, wave-specialised
// pipeline inside a persistent 256-thread workgroup (two workgroups per CU).
//
//   wave 0 ("parse")     block a_i, staged in LDS buffer X[i&1]: Init checks,
//                        the restart-run walks (lane per run, two passes: count,
//                        then write per-KV metadata at final indices), prefix
//                        parents, output-bucket tables; publishes a_i's
//                        aggregate to the look-back state.  Never waits.
//   waves 1-3 ("emit")   block a_{i-1}, parsed one iteration earlier (X[(i-1)&1],
//                        meta slot M[(i-1)&1]): resolves its exclusive prefix
//                        (its predecessors published at least an iteration ago,
//                        so the look-back almost never waits), then writes the
//                        per-KV arrays, restart words, and key / value bytes as
//                        coalesced 16-B granules gathered from LDS; meanwhile the
//                        same waves load block a_{i+1} into registers, stored to
//                        the free LDS buffer after the iteration's barrier.
//
// The look-back is therefore off the critical path: a block's outputs are
// placed one iteration after its sizes are published.  Deadlock freedom: only
// resident workgroups take tickets; the parse stage never waits (except the
// general path below, which waits only on smaller tickets), so the smallest
// unpublished ticket always makes progress.
//
// Blocks outside the LDS limits (> 32 KiB, > kKv KVs or runs, > kKeyCap user-key
// bytes, or a restart table inconsistent with per-run walks) take the general
// path on wave 0 inside the parse stage (rowblk_general.hip.h: a wave-serial
// restatement of Iter.First/Next), which resolves its own look-back.
//
// Semantics: cockroachdb/pebble sstable/rowblk/rowblk_iter.go — Init :241-276,
// readFirstKey :418-485, readEntry :333-416, decodeInternalKey :487-504, value
// prefix :1192-1199 (sstable/block/kv.go:14-41), decodeRestart :1092-1096.
#pragma once

namespace pipe {

#ifdef PBL_STAMPS
// diagnostic build only: per-block phase timestamps (s_memtime) written past the
// look-back state in the workspace; never part of an output
#define PSTAMP(A_, b_, i_, lane0_)                                                             \
  do {                                                                                          \
    if (lane0_)                                                                                 \
      reinterpret_cast<uint64_t*>(reinterpret_cast<uint8_t*>((A_).out.workspace) +             \
                                  ws_bytes((A_).in.n_blocks))[uint64_t(b_) * 16 + (i_)] =       \
          __builtin_amdgcn_s_memtime();                                                         \
  } while (0)
// slot i_ = the wave's HW_ID (SIMD / CU / SE) and XCC_ID: where the roles run
#define PHWID(A_, b_, i_, lane0_)                                                              \
  do {                                                                                          \
    if (lane0_)                                                                                 \
      reinterpret_cast<uint64_t*>(reinterpret_cast<uint8_t*>((A_).out.workspace) +             \
                                  ws_bytes((A_).in.n_blocks))[uint64_t(b_) * 16 + (i_)] =       \
          uint64_t(__builtin_amdgcn_s_getreg(4 | (31 << 11))) |                                 \
          uint64_t(__builtin_amdgcn_s_getreg(20 | (15 << 11))) << 32;                           \
  } while (0)
#else
#define PSTAMP(A_, b_, i_, lane0_) do {} while (0)
#define PHWID(A_, b_, i_, lane0_) do {} while (0)
#endif

constexpr int kKv = 400;                       // KVs (and runs) per block on the pipelined path
constexpr uint32_t kKeyCap = 32768;            // user-key bytes per block on the pipelined path
constexpr int kBs = 7;                         // output bucket = 128 bytes
constexpr int kKBkt = kKeyCap >> kBs;          // key buckets
constexpr int kVBkt = kMaxFastLen >> kBs;      // value buckets (values <= block length)
#ifndef PBL_EMIT_PF_EARLY
#define PBL_EMIT_PF_EARLY 2
#endif
#ifndef PBL_VU
#define PBL_VU 2
#endif
constexpr int kVU = PBL_VU;  // value granules per emit-loop step (their LDS round trips interleaved)
#ifndef PBL_PIPE_WAVES
#define PBL_PIPE_WAVES 4
#endif
constexpr int kPTPB = PBL_PIPE_WAVES * kWave;  // threads per pipelined workgroup
constexpr int kEmit = kPTPB - kWave;           // emitter threads (waves 1..)

enum { kModeNone = 0, kModeFast = 1, kModeErr = 2, kModeDone = 3 };

// One parsed block.  Offsets are block-relative (u16: the block is <= 32 KiB,
// user-key bytes <= kKeyCap).
struct Meta {
  uint16_t eoff[kKv];      // entry offset (KVEncoding.Offset)
  uint16_t ksrc[kKv];      // offset of the unshared key bytes
  uint16_t sh[kKv];        // shared length
  uint16_t klen[kKv];      // internal key length
  uint16_t par[kKv];       // prefix parent: max{i < j in run : shared_i < shared_j} (j itself if shared_j == 0)
  uint16_t kout[kKv + 1];  // user-key output offsets
  uint32_t vp[kKv + 5];    // value output offset | value source offset (after prefix stripping) << 16;
                           // entries nkv..nkv+4 hold the block's value total (window reads)
  uint16_t kbkt[kKBkt];    // KV holding key output byte q*128
  uint16_t vbkt[kVBkt];    // KV holding value output byte q*128
  uint8_t kvf[kKv];        // PBL_KV_* flags (OBSOLETE is added at emit time)
  uint64_t boff;
  uint64_t excl[kNumComp];  // exclusive prefix (resolved by the parse wave)
  uint32_t b, blen, status, mode, nkv, nres, roff, tot_kb, tot_vb;
};

__device__ __forceinline__ uint32_t vout_of(const Meta& M, uint32_t j) { return M.vp[j] & 0xffffu; }
__device__ __forceinline__ uint32_t vsrc_of(const Meta& M, uint32_t j) { return M.vp[j] >> 16; }

struct PLds {
  uint4 x[2][kLdsBlkBytes / 16];  // block staging, double-buffered
  Meta m[2];
  uint32_t nxt;                   // ticket of the block after the current one
};
static_assert(sizeof(PLds) <= 163840 / 2, "two pipelined workgroups per CU");

// ---- parse-stage helpers (wave 0) --------------------------------------------

// Entry header (rowblk_iter.go:345-398: three uint32 varints) decoded without
// branches from the 8 bytes at the entry: each varint 1 or 2 bytes.  Returns
// false if any needs 3+ bytes (value >= 16384: the block takes the general path).
// Entry header: three uint32 varints decoded from one 8-byte window.  The
// common 1-2 byte form is decoded inline; a 3-byte varint (values of 16 KiB and
// more, config 5) takes hdr3 on the lanes that need it.  Anything longer takes
// the general path.
__device__ __forceinline__ bool hdr3(uint64_t w, uint32_t* sh, uint32_t* un, uint32_t* vl, uint32_t* h) {
  uint32_t p = 0, v[3];
  bool ok = true;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const uint32_t x = uint32_t(w >> (8 * p));  // p <= 6 here
    const uint32_t b0 = x & 0xff, b1 = (x >> 8) & 0xff, b2 = (x >> 16) & 0xff;
    const bool c0 = (b0 & 0x80) != 0, c1 = c0 && (b1 & 0x80) != 0;
    v[k] = c1 ? ((b0 & 0x7f) | ((b1 & 0x7f) << 7) | (b2 << 14)) : c0 ? ((b0 & 0x7f) | (b1 << 7)) : b0;
    ok = ok && !(c1 && (b2 & 0x80));
    p += c1 ? 3 : c0 ? 2 : 1;
  }
  *sh = v[0];
  *un = v[1];
  *vl = v[2];
  *h = p;
  // RunBuf packs unshared in 14 bits and the header length in 3
  return ok && p <= 7 && v[1] < 16384u;
}

__device__ __forceinline__ bool hdr2(uint64_t w, uint32_t* sh, uint32_t* un, uint32_t* vl, uint32_t* h) {
  if (__builtin_expect((uint32_t(w) & 0x808080u) == 0, 1)) {  // three 1-byte varints (values < 128)
    *sh = uint32_t(w) & 0xffu;
    *un = uint32_t(w >> 8) & 0xffu;
    *vl = uint32_t(w >> 16) & 0xffu;
    *h = 3;
    return true;
  }
  uint32_t p = 0, v[3];
  bool ok = true;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const uint32_t x = uint32_t(w >> (8 * p));
    const uint32_t b0 = x & 0xff, b1 = (x >> 8) & 0xff;
    const bool two = (b0 & 0x80) != 0;
    v[k] = two ? ((b0 & 0x7f) | (b1 << 7)) : b0;
    ok = ok && !(two && (b1 & 0x80));
    p += two ? 2 : 1;
  }
  *sh = v[0];
  *un = v[1];
  *vl = v[2];
  *h = p;
  if (__builtin_expect(!ok, 0)) ok = hdr3(w, sh, un, vl, h);
  return ok;
}

struct RunAcc {
  uint32_t cnt, kb, vb;
};

// Pass 1 over run r: count entries and output bytes; `ok` clears if the run is
// not walkable per run (general path), `bad` sets on shared > len(previous key)
// (rowblk_iter.go:403), `vbad` on a SET value without its prefix byte.
// Count entries [pos, e0) of a run whose first `cnt` entries were already
// counted (prev_kl = the length of the last one).
__device__ __forceinline__ void run_count_span(const View& V, uint32_t pos, uint32_t e0, uint32_t cnt,
                                               uint32_t prev_kl, uint32_t flags, bool vprefix, RunAcc& acc,
                                               bool& ok, bool& bad, bool& vbad) {
  const uint32_t cnt0 = cnt;
  while (pos < e0) {
    uint32_t sh, un, vl, h;
    const bool hok = hdr2(V.ld8(pos), &sh, &un, &vl, &h);
    const uint32_t np = pos + h + un + vl;  // < 2^23: no overflow
    if (!hok || (cnt == 0 && sh != 0) || np > e0) { ok = false; return; }
    bad = bad || (cnt > 0 && sh > prev_kl);
    const uint32_t kl = sh + un;
    uint32_t vlen = vl;
    if (vprefix && kl >= 8) {
      if (kl - 8 < sh) { ok = false; return; }  // kind byte inside the shared prefix
      if ((V.byte(pos + h + (kl - 8 - sh)) & 0xBF) == 1) {
        if (vl == 0) vbad = true;
        else if ((V.byte(pos + h + un) & 0xC0) == 0 || (flags & PBL_ROW_NO_VALUER)) vlen--;
      }
    }
    acc.kb += (flags & PBL_ROW_RAW_KEYS) ? kl : (kl >= 8 ? kl - 8 : 0);
    acc.vb += vlen;
    cnt++;
    prev_kl = kl;
    pos = np;
  }
  acc.cnt += cnt - cnt0;
}

__device__ __forceinline__ void run_count(const View& V, uint32_t r, uint32_t nres, uint32_t roff, uint32_t flags,
                                          bool vprefix, RunAcc& acc, bool& ok, bool& bad, bool& vbad) {
  const uint32_t st = roff + 4 * r;
  const uint32_t s0 = V.le32(st) & kRestartMask;
  const uint32_t e0 = (r + 1 < nres) ? (V.le32(st + 4) & kRestartMask) : roff;
  if (!((r != 0 || s0 == 0) && s0 < e0 && e0 <= roff)) { ok = false; return; }
  run_count_span(V, s0, e0, 0, 0, flags, vprefix, acc, ok, bad, vbad);
}

// Pass 2 over run r (validated by pass 1): per-KV metadata at final indices.
// Prefix-parent chain state carried from one entry of a run to the next.
struct ParState {
  uint32_t prev_sh, pp, ppsh;
};

// Write entries [pos, e0) of a run at final indices acc.cnt.. (P = the chain
// state after the entries before pos; `first` = pos is the restart point).
__device__ __forceinline__ void run_write_span(Meta& M, const View& V, uint32_t pos, uint32_t e0, uint32_t rw,
                                               bool first, ParState P, uint32_t flags, bool vprefix, RunAcc& acc) {
  uint32_t j = acc.cnt, kb = acc.kb, vb = acc.vb;
  uint32_t prev_sh = P.prev_sh, pp = P.pp, ppsh = P.ppsh;
  while (pos < e0) {
    uint32_t sh, un, vl, h;
    hdr2(V.ld8(pos), &sh, &un, &vl, &h);
    const uint32_t kl = sh + un;
    uint32_t vs = pos + h + un, vlen = vl;
    uint8_t fl = 0;
    if (first) fl = uint8_t(PBL_KV_RESTART | ((rw >> 31) ? PBL_KV_RESTART_SAMEPFX : 0));
    if (!(flags & PBL_ROW_RAW_KEYS) && kl < 8) fl |= PBL_KV_INVALID_KEY;
    if (vprefix && kl >= 8 && (V.byte(pos + h + (kl - 8 - sh)) & 0xBF) == 1) {
      const uint32_t pre = V.byte(vs);
      if ((pre & 0xC0) == 0 || (flags & PBL_ROW_NO_VALUER)) { vs++; vlen--; }
      else if ((pre & 0xC0) == 0x80) fl |= PBL_KV_VALBLK_HANDLE;
      else fl |= PBL_KV_BLOB_HANDLE;
    }
    // prefix parent: all-nearest-smaller-values over the run (amortised O(1));
    // the previous entry and its parent are kept in registers
    uint32_t par = j, parsh = 0;
    if (sh != 0) {
      uint32_t c = j - 1, csh = prev_sh;
      if (csh >= sh) { c = pp; csh = ppsh; }
      while (csh >= sh) {
        c = M.par[c];
        csh = M.sh[c];
      }
      par = c;
      parsh = csh;
    }
    M.eoff[j] = uint16_t(pos);
    M.ksrc[j] = uint16_t(pos + h);
    M.sh[j] = uint16_t(sh);
    M.klen[j] = uint16_t(kl);
    M.par[j] = uint16_t(par);
    M.kout[j] = uint16_t(kb);
    M.vp[j] = vb | (vs << 16);
    M.kvf[j] = fl;
    prev_sh = sh;
    pp = par;
    ppsh = parsh;
    kb += (flags & PBL_ROW_RAW_KEYS) ? kl : (kl >= 8 ? kl - 8 : 0);
    vb += vlen;
    j++;
    first = false;
    pos = pos + h + un + vl;
  }
  acc.cnt = j;
  acc.kb = kb;
  acc.vb = vb;
}

// Pass 2 over run r (validated by pass 1): per-KV metadata at final indices.
__device__ __forceinline__ void run_write(Meta& M, const View& V, uint32_t r, uint32_t nres, uint32_t roff,
                                          uint32_t flags, bool vprefix, RunAcc& acc) {
  const uint32_t st = roff + 4 * r;
  const uint32_t rw = V.le32(st);
  const uint32_t e0 = (r + 1 < nres) ? (V.le32(st + 4) & kRestartMask) : roff;
  run_write_span(M, V, rw & kRestartMask, e0, rw, true, ParState{0, 0, 0}, flags, vprefix, acc);
}

// Single-walk form of passes 1+2 for runs of at most kRunBuf entries (every
// run of a block written with restart interval <= 16): the run is walked once,
// each entry's header parked in two packed registers (static indices: no
// scratch), and the per-KV metadata is written from registers once the block
// scan has placed the run.
constexpr int kRunBuf = 16;

struct RunBuf {
  uint32_t ea[kRunBuf];  // pos | shared << 16
  uint32_t eb[kRunBuf];  // unshared | header length << 14 | value length << 17
  uint32_t cnt, s0, rw;
  uint32_t pos, e0, prev_kl;  // continuation of a run longer than kRunBuf (over)
};

// Walk run r once.  `ok` clears as in run_count; `over` sets if the run has more
// than kRunBuf entries.
__device__ __forceinline__ void run_walk(const View& V, uint32_t r, uint32_t nres, uint32_t roff, uint32_t flags,
                                         bool vprefix, RunBuf& B, RunAcc& acc, bool& ok, bool& bad, bool& vbad,
                                         bool& over) {
  const uint32_t st = roff + 4 * r;
  B.rw = V.le32(st);
  const uint32_t s0 = B.rw & kRestartMask;
  const uint32_t e0 = (r + 1 < nres) ? (V.le32(st + 4) & kRestartMask) : roff;
  B.s0 = s0;
  B.cnt = 0;
  if (!((r != 0 || s0 == 0) && s0 < e0 && e0 <= roff)) { ok = false; return; }
  uint32_t pos = s0, cnt = 0, prev_kl = 0;
  bool go = true;
#pragma unroll
  for (int k = 0; k < kRunBuf; k++) {
    if (go && pos < e0) {
      uint32_t sh, un, vl, h;
      const bool hok = hdr2(V.ld8(pos), &sh, &un, &vl, &h);
      const uint32_t np = pos + h + un + vl;
      if (!hok || (k == 0 && sh != 0) || np > e0) {
        ok = false;
        go = false;
      } else {
        bad = bad || (k > 0 && sh > prev_kl);
        const uint32_t kl = sh + un;
        uint32_t vlen = vl;
        if (vprefix && kl >= 8) {
          if (kl - 8 < sh) { ok = false; go = false; }
          else if ((V.byte(pos + h + (kl - 8 - sh)) & 0xBF) == 1) {
            if (vl == 0) vbad = true;
            else if ((V.byte(pos + h + un) & 0xC0) == 0 || (flags & PBL_ROW_NO_VALUER)) vlen--;
          }
        }
        B.ea[k] = pos | (sh << 16);
        B.eb[k] = un | (h << 14) | (vl << 17);
        acc.kb += (flags & PBL_ROW_RAW_KEYS) ? kl : (kl >= 8 ? kl - 8 : 0);
        acc.vb += vlen;
        cnt++;
        prev_kl = kl;
        pos = np;
      }
    }
  }
  if (go && pos < e0) over = true;
  B.pos = pos;
  B.e0 = e0;
  B.prev_kl = prev_kl;
  B.cnt = cnt;
  acc.cnt += cnt;
}

// Write the parked entries of one run at final indices (acc = the run's bases).
__device__ __forceinline__ void run_emit_meta(Meta& M, const View& V, const RunBuf& B, uint32_t flags, bool vprefix,
                                              RunAcc& acc, ParState& P) {
  uint32_t j = acc.cnt, kb = acc.kb, vb = acc.vb;
  uint32_t prev_sh = 0, pp = 0, ppsh = 0;
#pragma unroll
  for (int k = 0; k < kRunBuf; k++) {
    if (uint32_t(k) < B.cnt) {
      const uint32_t pos = B.ea[k] & 0xffffu, sh = B.ea[k] >> 16;
      const uint32_t un = B.eb[k] & 0x3fffu, h = (B.eb[k] >> 14) & 7u, vl = B.eb[k] >> 17;
      const uint32_t kl = sh + un;
      uint32_t vs = pos + h + un, vlen = vl;
      uint8_t fl = 0;
      if (k == 0) fl = uint8_t(PBL_KV_RESTART | ((B.rw >> 31) ? PBL_KV_RESTART_SAMEPFX : 0));
      if (!(flags & PBL_ROW_RAW_KEYS) && kl < 8) fl |= PBL_KV_INVALID_KEY;
      if (vprefix && kl >= 8 && (V.byte(pos + h + (kl - 8 - sh)) & 0xBF) == 1) {
        const uint32_t pre = V.byte(vs);
        if ((pre & 0xC0) == 0 || (flags & PBL_ROW_NO_VALUER)) { vs++; vlen--; }
        else if ((pre & 0xC0) == 0x80) fl |= PBL_KV_VALBLK_HANDLE;
        else fl |= PBL_KV_BLOB_HANDLE;
      }
      uint32_t par = j, parsh = 0;
      if (sh != 0) {
        uint32_t c = j - 1, csh = prev_sh;
        if (csh >= sh) { c = pp; csh = ppsh; }
        while (csh >= sh) {
          c = M.par[c];
          csh = M.sh[c];
        }
        par = c;
        parsh = csh;
      }
      M.eoff[j] = uint16_t(pos);
      M.ksrc[j] = uint16_t(pos + h);
      M.sh[j] = uint16_t(sh);
      M.klen[j] = uint16_t(kl);
      M.par[j] = uint16_t(par);
      M.kout[j] = uint16_t(kb);
      M.vp[j] = vb | (vs << 16);
      M.kvf[j] = fl;
      prev_sh = sh;
      pp = par;
      ppsh = parsh;
      kb += (flags & PBL_ROW_RAW_KEYS) ? kl : (kl >= 8 ? kl - 8 : 0);
      vb += vlen;
      j++;
    }
  }
  acc = RunAcc{j, kb, vb};
  P = ParState{prev_sh, pp, ppsh};
}

// Init checks (Init :248-256, readFirstKey :418-485) evaluated by every lane.
// Returns the status; *roff_o / *nres_o are set when it is PBL_OK.
template <class Rd>
__device__ __forceinline__ uint32_t init_checks(const Rd& rd, uint32_t blen, uint32_t flags, uint32_t* roff_o,
                                                uint32_t* nres_o) {
  *roff_o = 0;
  *nres_o = 0;
  if (blen < 4) return PBL_CORRUPT_BOUNDS;
  const uint32_t nw = rd.le32(blen - 4);
  if (nw == 0) return PBL_CORRUPT_NO_RESTARTS;
  if (nw >> 31) return PBL_CORRUPT_BOUNDS;
  const uint64_t need = 4ull * (1ull + nw);
  if (need > blen) return PBL_CORRUPT_BOUNDS;
  const uint32_t roff = blen - uint32_t(need);
  if (roff > 0 && !(flags & PBL_ROW_RAW_KEYS)) {
    if (rd.byte(0) != 0) return PBL_CORRUPT_FIRST_KEY;
    uint32_t un, vl;
    const uint32_t n1 = rd.varint(1, blen, &un);
    const uint32_t n2 = n1 ? rd.varint(1 + n1, blen, &vl) : 0;
    if (!n2) return PBL_CORRUPT_BOUNDS;
    if (un < 8) return PBL_CORRUPT_FIRST_KEY;
  }
  *roff_o = roff;
  *nres_o = nw;
  return PBL_OK;
}

template <typename T>
__device__ __forceinline__ T wave_bcast_last(T v) {
  return __shfl(v, kWave - 1, kWave);
}

// General path for one block (wave 0, inside the parse stage): a wave-serial
// Iter.First/Next (rowblk_general.hip.h) that resolves its own look-back and
// writes every output.  Kept out of line: it is rare and large.
__device__ __noinline__ void parse_slow(Meta& M, uint4* X, const Args A) {
  const int l = lane_id();
  const uint32_t b = M.b, blen = M.blen;
  const uint64_t boff = M.boff;
  const uint32_t nb = A.in.n_blocks, flags = A.in.flags;
  const bool fits = blen <= kMaxFastLen;
  const uint8_t* gblk = A.in.blocks + boff;
  uint8_t* ws = reinterpret_cast<uint8_t*>(A.out.workspace);
  uint64_t* lb_state = reinterpret_cast<uint64_t*>(ws + kWsHeader);
    // ---- general path (wave-serial Iter.Next), resolving its own look-back --------
    SlowState ss;
    uint64_t excl[kNumComp];
    if (!fits) {
      // a block past the LDS stage: big_block_sizes_kernel walked it, published
      // its aggregate and left {status, counts} in its block-metadata slots;
      // big_block_values_kernel writes its outputs after this launch
      ss.status = to_glb(A.out.blk_status)[b];
      ss.nkv = to_glb(A.out.blk_kv_base)[b];
      ss.kb = to_glb(A.out.blk_key_base)[b];
      ss.vb = to_glb(A.out.blk_val_base)[b];
      ss.nr = ss.status == PBL_OK ? SlowGlb{to_glb(gblk), blen}.le32(blen - 4) : 0;
    } else {
      // key buffer: the meta slot's per-KV arrays; if a key outgrows it, re-run
      // from global memory with the whole staging buffer as the key buffer
      const uint8_t* src = reinterpret_cast<const uint8_t*>(X) + kPad + (boff & 15);
      uint64_t dummy[kNumComp] = {0, 0, 0, 0};
      bool from_lds = true;
      uint8_t* keybuf = reinterpret_cast<uint8_t*>(&M);
      uint32_t keycap = uint32_t(offsetof(Meta, boff));
      slow_walk(src, true, blen, flags, A.in.synthetic_seq_num, keybuf, keycap, kPassCount, A.out, b, dummy, &ss);
      if (ss.status == PBL_UNSUPPORTED) {
        from_lds = false;
        src = gblk;
        keybuf = reinterpret_cast<uint8_t*>(X);
        keycap = uint32_t(kLdsBlkBytes);
        slow_walk(src, false, blen, flags, A.in.synthetic_seq_num, keybuf, keycap, kPassCount, A.out, b, dummy, &ss);
      }
      const bool okk = ss.status == PBL_OK;
      const uint64_t agg[kNumComp] = {okk ? ss.nkv : 0, okk ? ss.kb : 0, okk ? ss.vb : 0, okk ? ss.nr : 0};
      lookback(lb_state, nb, b, agg, excl, &A.out.totals->status_mask);
      uint32_t st2 = ss.status;
      if (okk && overflows(A.out, excl, agg)) st2 = PBL_OVERFLOW;
      if (st2 == PBL_OK) slow_walk(src, from_lds, blen, flags, A.in.synthetic_seq_num, keybuf, keycap, kPassAll, A.out, b, excl, &ss);
      else if (l == 0 && A.out.key_off && excl[0] + b < A.out.kv_cap + nb) {
        A.out.key_off[excl[0] + b] = 0;
        A.out.val_off[excl[0] + b] = 0;
      }
      if (l == 0) {
        write_block_meta(A.out, b, nb, st2, excl, agg, true);
        M.mode = kModeDone;
      }
      return;
    }
    const bool okk = ss.status == PBL_OK;
    const uint64_t agg[kNumComp] = {okk ? ss.nkv : 0, okk ? ss.kb : 0, okk ? ss.vb : 0, okk ? ss.nr : 0};
    lb_resolve(lb_state, nb, b, agg, excl, &A.out.totals->status_mask);
    uint32_t st2 = ss.status;
    if (okk && overflows(A.out, excl, agg)) st2 = PBL_OVERFLOW;
    if (st2 != PBL_OK && l == 0 && A.out.key_off && excl[0] + b < A.out.kv_cap + nb) {
      A.out.key_off[excl[0] + b] = 0;
      A.out.val_off[excl[0] + b] = 0;
    }
    if (l == 0) {
      write_block_meta(A.out, b, nb, st2, excl, agg, true);
      M.mode = kModeDone;
    }
}

// Size pass for the blocks past the LDS stage (blen > kMaxFastLen), one wave
// per block, launched ahead of rowblk_pipe_kernel on the same stream.  Their
// count walk reads global memory entry by entry; inside the pipeline it would
// hold back the look-back of every later ticket.  Here all of them walk at
// once and publish their aggregates, so the pipeline's parse_slow only
// resolves.  Same init checks and the same slow_walk as parse_slow, so the
// aggregate is the one parse_slow computes.
__global__ void __launch_bounds__(kWave) big_block_sizes_kernel(Args A) {
  __shared__ uint4 keybuf4[kLdsBlkBytes / 16];
  const uint32_t nb = A.in.n_blocks, flags = A.in.flags;
  uint8_t* ws = reinterpret_cast<uint8_t*>(A.out.workspace);
  uint64_t* lb_state = reinterpret_cast<uint64_t*>(ws + kWsHeader);
  // 64 lengths per wave per round; the big blocks among them one after another
  for (uint64_t base = uint64_t(blockIdx.x) * kWave; base < nb; base += uint64_t(gridDim.x) * kWave) {
   const uint64_t bl = base + lane_id();
   // (row blocks only: a mixed batch's colblk blocks are the colblk pipeline's)
   uint64_t big = __ballot(bl < nb && to_glb(A.in.block_len)[bl] > kMaxFastLen &&
                           (!A.in.block_format || to_glb(A.in.block_format)[bl] == PBL_FMT_ROW));
   while (big) {
    const uint32_t b = uint32_t(base) + uint32_t(__builtin_ctzll(big));
    big &= big - 1;
    const uint32_t blen = A.in.block_len[b];
    const uint8_t* gblk = A.in.blocks + A.in.block_off[b];
    uint32_t roff, nres;
    if (init_checks(GlbRd{gblk}, blen, flags, &roff, &nres) != PBL_OK) continue;  // (parse_block's error path publishes)
    SlowState ss;
    uint64_t dummy[kNumComp] = {0, 0, 0, 0};
    slow_walk(gblk, false, blen, flags, A.in.synthetic_seq_num, reinterpret_cast<uint8_t*>(keybuf4), uint32_t(kLdsBlkBytes), 0, A.out, b, dummy,
              &ss);
    const bool okk = ss.status == PBL_OK;
    const uint64_t agg[kNumComp] = {okk ? ss.nkv : 0, okk ? ss.kb : 0, okk ? ss.vb : 0, okk ? ss.nr : 0};
    lb_publish(lb_state, nb, b, agg);
    if (lane_id() == 0) {  // for parse_slow (write_block_meta replaces them)
      g_atomic_add(reinterpret_cast<uint32_t*>(ws) + kWsBigCount, 1u);
      to_glb(A.out.blk_status)[b] = ss.status;
      to_glb(A.out.blk_kv_base)[b] = agg[0];
      to_glb(A.out.blk_key_base)[b] = agg[1];
      to_glb(A.out.blk_val_base)[b] = agg[2];
    }
   }
  }
}

// Outputs of the blocks past the LDS stage, launched after rowblk_pipe_kernel
// on the same stream (which resolved their bases into blk_*_base).  One wave
// per block, all big blocks at once, 8 value granules per lane in flight: a big
// value is HBM-bandwidth work, which a single wave inside the pipeline (each
// granule behind the previous store's vmcnt) turned into latency-bound work,
// and its serial walk would hold the workgroup's pipeline.
__global__ void __launch_bounds__(kWave) big_block_values_kernel(Args A) {
  __shared__ uint4 keybuf4[kLdsBlkBytes / 16];
  const uint32_t nb = A.in.n_blocks, flags = A.in.flags;
  // (the size pass counted the big blocks; usually there are none)
  if (__hip_atomic_load(to_glb(reinterpret_cast<uint32_t*>(A.out.workspace) + kWsBigCount), __ATOMIC_RELAXED,
                        __HIP_MEMORY_SCOPE_AGENT) == 0)
    return;
  for (uint64_t base = uint64_t(blockIdx.x) * kWave; base < nb; base += uint64_t(gridDim.x) * kWave) {
    const uint64_t bl = base + lane_id();
    uint64_t big = __ballot(bl < nb && to_glb(A.in.block_len)[bl] > kMaxFastLen &&
                            (!A.in.block_format || to_glb(A.in.block_format)[bl] == PBL_FMT_ROW) &&
                            to_glb(A.out.blk_status)[bl] == PBL_OK);
    while (big) {
      const uint32_t b = uint32_t(base) + uint32_t(__builtin_ctzll(big));
      big &= big - 1;
      const uint32_t blen = A.in.block_len[b];
      const uint64_t bases[kNumComp] = {A.out.blk_kv_base[b], A.out.blk_key_base[b], A.out.blk_val_base[b],
                                        A.out.blk_rst_base ? A.out.blk_rst_base[b] : 0};
      SlowState ss;
      slow_walk_t<SlowGlb, 8>(SlowGlb{to_glb(A.in.blocks + A.in.block_off[b]), blen}, blen, flags, A.in.synthetic_seq_num,
                              to_lds_ptr(reinterpret_cast<uint8_t*>(keybuf4)), uint32_t(kLdsBlkBytes), kPassAll,
                              A.out, b, bases, &ss);
    }
  }
}

// Parse stage: wave 0, block M.b staged in X (if it fits).
template <int W = kLbWin>
__device__ __forceinline__ void parse_block(Meta& M, uint4* X, const Args& A) {
  const int l = lane_id();
  const uint32_t b = M.b, blen = M.blen;
  const uint64_t boff = M.boff;
  const uint32_t nb = A.in.n_blocks, flags = A.in.flags;
  const bool vprefix = (flags & PBL_ROW_VALUE_PREFIX) && !(flags & PBL_ROW_RAW_KEYS);
  const bool fits = blen <= kMaxFastLen;
  const uint8_t* gblk = A.in.blocks + boff;
  uint8_t* ws = reinterpret_cast<uint8_t*>(A.out.workspace);
  uint64_t* lb_state = reinterpret_cast<uint64_t*>(ws + kWsHeader);
  const View V = lds_view(X, uint32_t(kPad + (boff & 15)));
  PSTAMP(A, b, 0, l == 0);
  PHWID(A, b, 14, l == 0);

  uint32_t roff, nres;
  uint32_t status = fits ? init_checks(LdsRd{V}, blen, flags, &roff, &nres)
                         : init_checks(GlbRd{gblk}, blen, flags, &roff, &nres);
  bool slow = status == PBL_OK && (!fits || nres > uint32_t(kKv));
  uint32_t nkv = 0, tkb = 0, tvb = 0;
  bool published = false;
  if (status == PBL_OK && !slow && roff > 0) {
    // lane l owns runs [r0, r1): contiguous, so a lane scan orders them
    const uint32_t R = (nres + kWave - 1) / kWave;
    const uint32_t r0 = min(uint32_t(l) * R, nres), r1 = min(r0 + R, nres);
    RunAcc acc{0, 0, 0};
    bool ok = true, bad = false, vbad = false, over = false;
    RunBuf RB;
    const bool single = R == 1;
    if (single) {
      if (r0 < nres) run_walk(V, r0, nres, roff, flags, vprefix, RB, acc, ok, bad, vbad, over);
      else RB.cnt = 0;
    }
    // a run longer than kRunBuf keeps its parked head and counts only its tail
    if (single && over && ok) run_count_span(V, RB.pos, RB.e0, RB.cnt, RB.prev_kl, flags, vprefix, acc, ok, bad, vbad);
    const bool walked = single;
    if (!walked) {
      acc = RunAcc{0, 0, 0};
      ok = true; bad = false; vbad = false;
      for (uint32_t r = r0; r < r1 && ok; r++) run_count(V, r, nres, roff, flags, vprefix, acc, ok, bad, vbad);
    }
    PSTAMP(A, b, 1, l == 0);
    const uint32_t ic = wave_incl_scan(acc.cnt), ik = wave_incl_scan(acc.kb), iv = wave_incl_scan(acc.vb);
    nkv = wave_bcast_last(ic);
    tkb = wave_bcast_last(ik);
    tvb = wave_bcast_last(iv);
    if (__ballot(bad)) status = PBL_CORRUPT_BOUNDS;
    else if (__ballot(!ok) || nkv > uint32_t(kKv) || tkb > kKeyCap) slow = true;
    else if (__ballot(vbad)) status = PBL_CORRUPT_BOUNDS;  // Go: i.val[0] on an empty SET value
    if (status == PBL_OK && !slow) {
      // the sizes are final: publish before the write pass
      const uint64_t agg[kNumComp] = {nkv, tkb, tvb, nres};
      lb_publish(lb_state, nb, b, agg);
      published = true;
      RunAcc w{ic - acc.cnt, ik - acc.kb, iv - acc.vb};
      if (walked) {
        ParState P;
        run_emit_meta(M, V, RB, flags, vprefix, w, P);
        if (over) run_write_span(M, V, RB.pos, RB.e0, RB.rw, false, P, flags, vprefix, w);
      }
      else
        for (uint32_t r = r0; r < r1; r++) run_write(M, V, r, nres, roff, flags, vprefix, w);
      PSTAMP(A, b, 2, l == 0);
      if (l < 5) M.vp[nkv + l] = tvb;
      if (l == 0) M.kout[nkv] = uint16_t(tkb);
      wave_sync();
      // output buckets: the KV holding byte q*128 of the block's keys / values
      for (uint32_t j = l; j < nkv; j += kWave) {
        const uint32_t k0 = M.kout[j], k1 = M.kout[j + 1];
        for (uint32_t q = (k0 + 127) >> kBs; (q << kBs) < k1; q++) M.kbkt[q] = uint16_t(j);
        const uint32_t v0 = vout_of(M, j), v1 = vout_of(M, j + 1);
        for (uint32_t q = (v0 + 127) >> kBs; (q << kBs) < v1; q++) M.vbkt[q] = uint16_t(j);
      }
    }
  }

  if (status == PBL_OK && slow) {
    parse_slow(M, X, A);
    return;
  }
  const bool okb = status == PBL_OK;
  const uint64_t agg[kNumComp] = {okb ? nkv : 0, okb ? tkb : 0, okb ? tvb : 0, okb ? nres : 0};
  if (!published) lb_publish(lb_state, nb, b, agg);
  PSTAMP(A, b, 3, l == 0);
  // resolve this block's exclusive prefix now: the parse wave has slack, the
  // emit waves then start on their stores at once next iteration
  uint64_t excl[kNumComp];
  lb_resolve<W>(lb_state, nb, b, agg, excl, &A.out.totals->status_mask);
  PSTAMP(A, b, 4, l == 0);
  if (okb && overflows(A.out, excl, agg)) status = PBL_OVERFLOW;
  if (l == 0) {
    if (status != PBL_OK && A.out.key_off && excl[0] + b < A.out.kv_cap + nb) {
      to_glb(A.out.key_off)[excl[0] + b] = 0;
      to_glb(A.out.val_off)[excl[0] + b] = 0;
    }
    write_block_meta(A.out, b, nb, status, excl, agg, false);
#pragma unroll
    for (int c = 0; c < kNumComp; c++) M.excl[c] = excl[c];
    M.kout[nkv] = uint16_t(tkb);  // (also the lone N+1 offset of a block with no entries)
    M.vp[nkv] = tvb;
    M.status = status;
    M.mode = status == PBL_OK ? kModeFast : kModeDone;
    M.nkv = nkv;
    M.nres = okb ? nres : 0;
    M.roff = roff;
    M.tot_kb = tkb;
    M.tot_vb = tvb;
  }
}

// ---- emit-stage helpers (waves 1-3) --------------------------------------------

// byte p of the internal key of KV j (source = max{i <= j : shared_i <= p})
__device__ __forceinline__ uint32_t mkey_byte(const Meta& M, const View& V, int j, uint32_t p) {
  while (p < uint32_t(M.sh[j])) j--;
  return V.byte(M.ksrc[j] + p - M.sh[j]);
}

__device__ __forceinline__ uint64_t mtrailer(const Meta& M, const View& V, int j, uint8_t* fl, uint32_t flags) {
  if (flags & PBL_ROW_RAW_KEYS) return 0;
  const uint32_t kl = M.klen[j];
  if (kl < 8) return kKindInvalid;
  const uint32_t sh = M.sh[j];
  uint64_t raw;
  if (kl - 8 >= sh) {
    raw = V.ld8(M.ksrc[j] + (kl - 8 - sh));
  } else {
    raw = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) raw |= uint64_t(mkey_byte(M, V, j, kl - 8 + i)) << (8 * i);
  }
  if (raw & 64u) *fl |= PBL_KV_OBSOLETE;
  return raw & kTrailerObsoleteMask;
}

// Merge user-key bytes [p_lo, p_hi) of KV j (user-key length ukl) into granule
// bytes [q, ...) of w: walk the prefix-parent chain, one LDS gather per segment.
__device__ __forceinline__ void mkey_part(uint4& w, const Meta& M, const View& V, int j, uint32_t ukl,
                                          uint32_t p_lo, uint32_t p_hi, uint32_t q) {
  uint32_t cur = ukl;
  int i = j;
  while (cur > p_lo) {
    const uint32_t shi = M.sh[i];
    const uint32_t lo_i = shi < cur ? shi : cur;
    const uint32_t a = lo_i > p_lo ? lo_i : p_lo, z = cur < p_hi ? cur : p_hi;
    if (a < z) {
      const uint32_t gq = q + (a - p_lo);
      const int32_t src = int32_t(M.ksrc[i]) - int32_t(shi) + int32_t(a);
      const uint4 v = V.ld16(src - int32_t(gq));
      if (gq == 0 && z - a == 16) w = v;
      else merge16(w, v, gq, gq + (z - a));
    }
    cur = lo_i;
    i = M.par[i];
  }
}

__device__ __forceinline__ void put16(gptr<uint8_t> base, uint64_t a, const uint4& w, uint32_t lo, uint32_t hi) {
  if (lo == 0 && hi == 16) *(gptr<u32x4>)(base + a) = u32x4{w.x, w.y, w.z, w.w};
  else store_partial16(base + a, w, lo, hi);
}

// Emit stage, part 1 (waves 1-3): resolve the exclusive prefix of block M.b
// (parsed in the previous iteration) and write its block metadata.  Every
// emitter wave resolves the (normally ready) prefix itself: no cross-wave
// hand-off inside the stage.  Returns whether the block's outputs are written.
__device__ __forceinline__ bool emit_resolve(const Meta& M, const Args& A, uint64_t excl[kNumComp]) {
  (void)A;
  if (M.mode != kModeFast) return false;
#pragma unroll
  for (int c = 0; c < kNumComp; c++) excl[c] = M.excl[c];
  return true;
}

// Emit stage, part 2 (waves 1-3): per-KV arrays, restart words, key and value
// bytes of block M.b at the resolved bases.
template <class F>
__device__ __forceinline__ void emit_write(const Meta& M, const uint4* X, const Args& A, const uint64_t* excl,
                                           const F& mid) {
  const int tb = int(threadIdx.x) - kWave;
  const uint32_t b = M.b, flags = A.in.flags;
  const pbl_decode_out& O = A.out;
  const uint32_t nkv = M.nkv, nres = M.nres, roff = M.roff, tkb = M.tot_kb, tvb = M.tot_vb;
  const View V = lds_view(X, uint32_t(kPad + (M.boff & 15)));
  const uint64_t kvb = excl[0], kbb = excl[1], vbb = excl[2], rbb = excl[3];
  PSTAMP(A, b, 5, tb == 0);
  PHWID(A, b, 15, tb == 0);

  const gptr<uint32_t> key_off = to_glb(O.key_off), val_off = to_glb(O.val_off);
  const gptr<uint64_t> trailer = to_glb(O.trailer);
  const gptr<uint8_t> kv_flags = to_glb(O.kv_flags);
  const gptr<uint32_t> entry_off = to_glb(O.entry_off), restarts = to_glb(O.restarts);

  auto per_kv = [&]() {
  // per-KV arrays (coalesced, thread per KV)
  for (uint32_t j = tb; j <= nkv; j += kEmit) {
    const uint64_t o = kvb + b + j;
    key_off[o] = M.kout[j];
    val_off[o] = vout_of(M, j);
    if (j < nkv) {
      uint8_t fl = M.kvf[j];
      trailer[kvb + j] = with_seq(mtrailer(M, V, int(j), &fl, flags), A.in.synthetic_seq_num, flags);
      if (O.kv_flags) kv_flags[kvb + j] = fl;
      if (O.entry_off) entry_off[kvb + j] = M.eoff[j];
    }
  }
  if (O.restarts)
    for (uint32_t r = tb; r < nres; r += kEmit) restarts[rbb + r] = V.le32(roff + 4 * r);
  PSTAMP(A, b, 6, tb == 0);

  };
  auto key_bytes = [&]() {
  // key bytes: one 16-B aligned output granule per thread; each the merge of
  // the segments of the 1-2 keys it overlaps (each key its prefix chain)
  if (tkb) {
    const uint64_t d0 = kbb, d1 = kbb + tkb;
    for (uint64_t a = (d0 & ~uint64_t(15)) + 16 * uint64_t(tb); a < d1; a += 16 * kEmit) {
      const uint32_t lo = a < d0 ? uint32_t(d0 - a) : 0u, hi = a + 16 <= d1 ? 16u : uint32_t(d1 - a);
      const uint32_t o = uint32_t(a + lo - d0), oe = uint32_t(a + hi - d0);
      uint32_t j = M.kbkt[o >> kBs];
      while (M.kout[j + 1] <= o) j++;
      uint4 w = make_uint4(0, 0, 0, 0);
      for (;;) {
        const uint32_t k0 = M.kout[j], k1 = M.kout[j + 1];
        const uint32_t s = o > k0 ? o : k0, e = oe < k1 ? oe : k1;
        if (s < e) mkey_part(w, M, V, int(j), k1 - k0, s - k0, e - k0, uint32_t(d0 + s - a));
        if (k1 >= oe) break;
        j++;
      }
      put16(to_glb(O.key_bytes), a, w, lo, hi);
    }
  }
  PSTAMP(A, b, 7, tb == 0);
  };
  auto value_bytes = [&]() {
  // value bytes: one 16-B aligned output granule per thread, two granules per
  // step with their LDS round trips interleaved: (1) bucket -> first KV,
  // (2) a 5-word window of packed (vout | vsrc) words -> the KV holding the
  // granule's first byte and the next one, (3) both segments gathered at once,
  // merged when the granule straddles two values.  Granules touching 3+ values
  // (values < 16 B) or more than 3 bucket steps take the general loop.
  if (tvb) {
    const uint64_t d0 = vbb, d1 = vbb + tvb;
    const gptr<uint8_t> vbytes = to_glb(O.val_bytes);
    uint64_t a = (d0 & ~uint64_t(15)) + 16 * uint64_t(tb);
    for (; a < d1; a += 16 * kVU * kEmit) {
      uint4 w[kVU];
      uint32_t lo[kVU], hi[kVU], o[kVU], oe[kVU], j0[kVU];
      bool live[kVU];
#pragma unroll
      for (int u = 0; u < kVU; u++) {
        const uint64_t g = a + uint64_t(u) * 16 * kEmit;
        live[u] = g < d1;
        lo[u] = g < d0 ? uint32_t(d0 - g) : 0u;
        hi[u] = !live[u] ? 0u : (g + 16 <= d1 ? 16u : uint32_t(d1 - g));
        o[u] = live[u] ? uint32_t(g + lo[u] - d0) : 0u;
        oe[u] = live[u] ? uint32_t(g + hi[u] - d0) : 0u;
        j0[u] = M.vbkt[o[u] >> kBs];
      }
      uint32_t vw[kVU][5];
#pragma unroll
      for (int u = 0; u < kVU; u++)
#pragma unroll
        for (int k = 0; k < 5; k++) vw[u][k] = M.vp[j0[u] + k];
      uint4 ga[kVU], gb[kVU];
      uint32_t sa[kVU], ea[kVU], sb[kVU], eb[kVU];
      bool gen[kVU];
#pragma unroll
      for (int u = 0; u < kVU; u++) {
        const uint32_t q = o[u];
        const bool s1 = (vw[u][1] & 0xffff) <= q;
        const bool s2 = s1 && (vw[u][2] & 0xffff) <= q;
        const bool s3 = s2 && (vw[u][3] & 0xffff) <= q;
        const uint32_t k = uint32_t(s1) + uint32_t(s2) + uint32_t(s3);
        const uint32_t A0 = k == 0 ? vw[u][0] : k == 1 ? vw[u][1] : k == 2 ? vw[u][2] : vw[u][3];
        const uint32_t A1 = k == 0 ? vw[u][1] : k == 1 ? vw[u][2] : k == 2 ? vw[u][3] : vw[u][4];
        const uint32_t A2 = k == 0 ? vw[u][2] : k == 1 ? vw[u][3] : k == 2 ? vw[u][4] : vw[u][4];
        const uint32_t v0 = A0 & 0xffff, v1 = A1 & 0xffff, v2 = A2 & 0xffff;
        // general loop if the window ran out, or the granule reaches a third value
        gen[u] = live[u] && ((s3 && (vw[u][4] & 0xffff) <= q) || (oe[u] > v1 && oe[u] > v2) || k == 3);
        sa[u] = q;
        ea[u] = oe[u] < v1 ? oe[u] : v1;
        sb[u] = v1;
        eb[u] = oe[u] < v2 ? oe[u] : v2;
        const uint32_t gqa = uint32_t(d0 + sa[u] - (a + uint64_t(u) * 16 * kEmit));
        ga[u] = V.ld16(int32_t(A0 >> 16) + int32_t(sa[u] - v0) - int32_t(gqa));
        const uint32_t gqb = gqa + (sb[u] - sa[u]);
        // (only read when the granule straddles into the next value: keep the
        // address inside the block otherwise)
        gb[u] = V.ld16(oe[u] > v1 && !gen[u] ? int32_t(A1 >> 16) - int32_t(gqb) : 0);
      }
#pragma unroll
      for (int u = 0; u < kVU; u++) {
        if (!live[u]) continue;
        const uint64_t g = a + uint64_t(u) * 16 * kEmit;
        if (!gen[u]) {
          const uint32_t gqa = uint32_t(d0 + sa[u] - g);
          if (gqa == 0 && ea[u] - sa[u] == 16) {
            w[u] = ga[u];
          } else {
            w[u] = make_uint4(0, 0, 0, 0);
            merge16(w[u], ga[u], gqa, gqa + (ea[u] - sa[u]));
            if (oe[u] > sb[u]) {
              const uint32_t gqb = gqa + (sb[u] - sa[u]);
              merge16(w[u], gb[u], gqb, gqb + (eb[u] - sb[u]));
            }
          }
        } else {
          uint32_t j = j0[u];
          while (vout_of(M, j + 1) <= o[u]) j++;
          w[u] = make_uint4(0, 0, 0, 0);
          for (;;) {
            const uint32_t v0 = vout_of(M, j), v1 = vout_of(M, j + 1);
            const uint32_t s_ = o[u] > v0 ? o[u] : v0, e_ = oe[u] < v1 ? oe[u] : v1;
            const uint32_t gq = uint32_t(d0 + s_ - g);
            merge16(w[u], V.ld16(int32_t(vsrc_of(M, j)) + int32_t(s_ - v0) - int32_t(gq)), gq, gq + (e_ - s_));
            if (v1 >= oe[u]) break;
            j++;
          }
        }
        put16(vbytes, g, w[u], lo[u], hi[u]);
      }
    }
  }
  };
#if PBL_EMIT_PF_EARLY == 2
  mid();
  value_bytes();
  per_kv();
  key_bytes();
#elif PBL_EMIT_PF_EARLY
  // values first: the next block's loads (mid) then land during the key and
  // per-KV phases instead of between the iteration's barriers
  value_bytes();
  mid();
  per_kv();
  key_bytes();
#else
  per_kv();
  key_bytes();
  value_bytes();
  mid();
#endif
  PSTAMP(A, b, 8, tb == 0);
#ifdef PBL_STAMPS
  // the last emitter wave to finish: per-wave end stamps
  PSTAMP(A, b, 9 + (tb >> 6), (tb & 63) == 0);
#endif
}

// The next block, held in registers by the emit waves between their loads
// (after the emit stores) and the store to LDS after the iteration's first
// barrier: kPfE granules per emit lane.
constexpr int kPfE = (kLdsBlkBytes / 16 + kEmit - 1) / kEmit;
struct PfEmit {
  u32x4 r[kPfE];
  __device__ __forceinline__ void load(const uint8_t* blocks, uint64_t off, uint32_t len) {
    const uint64_t a0 = off & ~uint64_t(15);
    const uint32_t n16 = uint32_t((((off + len + 15) & ~uint64_t(15)) - a0) >> 4);
    if (n16 == 0) return;
    gptr<const u32x4> src = to_glb(reinterpret_cast<const u32x4*>(blocks + a0));
    const uint32_t l = threadIdx.x - kWave;
#pragma unroll
    for (int i = 0; i < kPfE; i++) {
      const uint32_t g = l + uint32_t(i) * kEmit;
      r[i] = src[g < n16 ? g : n16 - 1];
    }
  }
  __device__ __forceinline__ void store(uint4* X, uint64_t off, uint32_t len) const {
    const uint64_t a0 = off & ~uint64_t(15);
    const uint32_t n16 = uint32_t((((off + len + 15) & ~uint64_t(15)) - a0) >> 4);
    const uint32_t l = threadIdx.x - kWave;
    lptr<u32x4> dst = to_lds_ptr(reinterpret_cast<u32x4*>(X)) + 1;
#pragma unroll
    for (int i = 0; i < kPfE; i++) {
      const uint32_t g = l + uint32_t(i) * kEmit;
      if (g < n16) dst[g] = r[i];
    }
  }
};

// The next block, held in registers by the parse wave (64 lanes x 33 granules
// >= the 2051 granules of the largest staged block) between its load at the
// start of an iteration and its store to LDS after the iteration's first
// barrier.  The registers are live only inside the parse wave's branch, so the
// emit waves' register budget (and their vmcnt drains) never see these loads.
constexpr int kPfRegs0 = (kLdsBlkBytes / 16 + kWave - 1) / kWave;
static_assert(kPfRegs0 == 33, "PBL_PF0_LIST");
#define PBL_PF0_LIST(X)                                                                                    \
  X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16) X(17) X(18) \
  X(19) X(20) X(21) X(22) X(23) X(24) X(25) X(26) X(27) X(28) X(29) X(30) X(31) X(32)

struct PfWave {
#define PBL_PF0_DECL(i) u32x4 r##i;
  PBL_PF0_LIST(PBL_PF0_DECL)
#undef PBL_PF0_DECL
  __device__ __forceinline__ static uint32_t granules(uint64_t off, uint32_t len) {
    return uint32_t((((off + len + 15) & ~uint64_t(15)) - (off & ~uint64_t(15))) >> 4);
  }
  // lanes past the end re-read the last granule instead of running off the block
  __device__ __forceinline__ void load(const uint8_t* blocks, uint64_t off, uint32_t len) {
    const uint32_t n16 = granules(off, len);
    gptr<const u32x4> src = to_glb(reinterpret_cast<const u32x4*>(blocks + (off & ~uint64_t(15))));
    const uint32_t l = lane_id();
#define PBL_PF0_LOAD(i)                                  \
    {                                                    \
      const uint32_t g = l + uint32_t(i) * kWave;        \
      r##i = src[g < n16 ? g : n16 - 1];                 \
    }
    PBL_PF0_LIST(PBL_PF0_LOAD)
#undef PBL_PF0_LOAD
  }
  __device__ __forceinline__ void store(uint4* X, uint64_t off, uint32_t len) const {
    const uint32_t n16 = granules(off, len);
    lptr<u32x4> dst = to_lds_ptr(reinterpret_cast<u32x4*>(X)) + 1;
    const uint32_t l = lane_id();
#define PBL_PF0_STORE(i)                                 \
    {                                                    \
      const uint32_t g = l + uint32_t(i) * kWave;        \
      if (g < n16) dst[g] = r##i;                        \
    }
    PBL_PF0_LIST(PBL_PF0_STORE)
#undef PBL_PF0_STORE
  }
};

// The pipelined persistent kernel.  Iteration i: wave 0 loads a_{i+1} into
// registers and parses a_i from X[i&1] into M[i&1]; waves 1-3 emit a_{i-1}
// from X/M[(i-1)&1].  After the first barrier wave 0 stores a_{i+1} into
// X[(i+1)&1] (free again) and rotates the descriptors; the second barrier
// publishes them.  Each role executes its own copies of the two barriers, so
// the prefetch registers stay confined to the parse wave's code.
template <bool kPrio, class Q, int W = kLbWin>  // W: the parse wave's look-back windows per round trip
__device__ __forceinline__ void row_pipe_body(PLds& S, const Args& A, const Q& Q_) {
  const Q& q = Q_;
  const int t = threadIdx.x;
  const uint32_t nb = A.in.n_blocks;
  if (t == 0) {
    const uint32_t t0 = q.take();
    S.m[0].b = t0;
    S.m[0].mode = kModeNone;
    S.m[1].mode = kModeNone;
    S.m[1].b = nb;
    if (t0 < nb) {
      S.m[0].boff = to_glb(A.in.block_off)[t0];
      S.m[0].blen = to_glb(A.in.block_len)[t0];
      S.nxt = q.take();
    } else {
      S.nxt = nb;
    }
  }
  __syncthreads();
  if (S.m[0].b < nb && S.m[0].blen <= kMaxFastLen) {
    // prologue: the first block straight into LDS by every thread
    const uint64_t off = S.m[0].boff;
    const uint32_t n16 = PfWave::granules(off, S.m[0].blen);
    gptr<const u32x4> src = to_glb(reinterpret_cast<const u32x4*>(A.in.blocks + (off & ~uint64_t(15))));
    lptr<u32x4> dst = to_lds_ptr(reinterpret_cast<u32x4*>(S.x[0])) + 1;
    for (uint32_t g = t; g < n16; g += kPTPB) dst[g] = src[g];
  }
  __syncthreads();
  // the parse wave is the pipeline's critical path: it wins VALU arbitration
  // against the emit wave of the other workgroup on its SIMD
#ifndef PBL_PARSE_PRIO
#define PBL_PARSE_PRIO 2
#endif
  if (kPrio && t < kWave) __builtin_amdgcn_s_setprio(PBL_PARSE_PRIO);
  for (uint32_t i = 0;; i++) {
    Meta& cur = S.m[i & 1];
    Meta& prv = S.m[(i + 1) & 1];
    const uint32_t cb = cur.b, nx = S.nxt;
    if (cb >= nb && prv.mode == kModeNone) break;
    uint64_t nx_off = 0;
    uint32_t nx_len = 0;
    if (nx < nb) {
      nx_off = to_glb(A.in.block_off)[nx];
      nx_len = to_glb(A.in.block_len)[nx];
    }
    const bool pf_on = nx < nb && nx_len <= kMaxFastLen;
    PfEmit pf;
    if (t < kWave) {
      if (cb < nb) parse_block<W>(cur, S.x[i & 1], A);
    } else {
      uint64_t excl[kNumComp];
#ifdef PBL_EXP_NO_EMIT
      emit_resolve(prv, A, excl);  // diagnostic build: parse timing without the emit stage
      if (pf_on) pf.load(A.in.blocks, nx_off, nx_len);
#else
      // the next block's loads go out once this wave's value stores are issued
      auto pf_issue = [&]() {
        if (pf_on) pf.load(A.in.blocks, nx_off, nx_len);
      };
      if (emit_resolve(prv, A, excl)) emit_write(prv, S.x[(i + 1) & 1], A, excl, pf_issue);
      else pf_issue();
#endif
    }
    __syncthreads();
    PSTAMP(A, cb, 13, t == 0 && cb < nb);
    PSTAMP(A, prv.b, 12, t == kWave && prv.mode != kModeNone);
    if (t >= kWave && pf_on) pf.store(S.x[(i + 1) & 1], nx_off, nx_len);
    if (t == 0) {
      prv.b = nx < nb ? nx : nb;
      prv.boff = nx_off;
      prv.blen = nx_len;
      prv.mode = kModeNone;
      S.nxt = nx < nb ? q.take() : nb;
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(kPTPB) __attribute__((amdgpu_waves_per_eu(PBL_PIPE_WAVES / 2, PBL_PIPE_WAVES / 2))) rowblk_pipe_kernel(Args A) {
  __shared__ PLds S;
  row_pipe_body<true>(S, A, TicketQueue{reinterpret_cast<uint32_t*>(A.out.workspace), A.in.n_blocks});
}

}  // namespace pipe
