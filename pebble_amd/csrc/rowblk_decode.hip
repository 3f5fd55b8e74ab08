// rowblk_decode.hip — gfx950 decoder for Pebble row-oriented data blocks.
//
// One 256-thread workgroup per block (block id = an atomic ticket, so the
// decoupled look-back always waits on resident predecessors).  The block is
// staged HBM -> LDS once with 16-byte coalesced loads; the varint headers are
// parsed out of LDS one lane per restart run (restart points cut the prefix
// chain, rowblk_writer.go:147-155); per-KV sizes are block-scanned; a
// decoupled look-back over the batch turns the per-block totals into output
// bases (single pass, no size pass); then every thread writes 16-byte granules
// of the key and value regions, gathering bytes out of LDS.
//
// Semantics follow cockroachdb/pebble sstable/rowblk/rowblk_iter.go:
//   Init :241-276 (numRestarts, restarts offset), readFirstKey :418-485,
//   readEntry :333-416 (3 uint32 varints, fullKey = fullKey[:shared]+unshared),
//   decodeInternalKey :487-504 (LE64 trailer & TrailerObsoleteMask, <8 B =>
//   InternalKeyKindInvalid), value prefix :1192-1199 (block/kv.go:14-41),
//   decodeRestart :1092-1096.
// Blocks whose restart table is inconsistent with a per-run walk, or that do
// not fit the LDS limits, take the general path: a wave-serial restatement of
// Iter.First/Next (bit-identical by construction, slower).
#include "common.hip.h"

namespace pbl {
namespace row {

constexpr int kLdsBlkBytes = 32768 + 32;  // block staging (any 16-B phase of a <=32 KiB block)
constexpr int kKvCap = 512;               // KVs per block on the LDS path
constexpr int kRunCap = kKvCap;           // restart runs per block on the LDS path
constexpr uint32_t kRestartMask = 0x7fffffffu;
constexpr uint64_t kTrailerObsoleteMask = ((((uint64_t)1 << 56) - 1) << 8) | 191u;
constexpr uint64_t kKindInvalid = 191u;
constexpr uint16_t kRunStart = 0x8000u;   // top bit of sh[] marks the first entry of a run

struct Lds {
  uint4 blk4[kLdsBlkBytes / 16];          // block bytes, block byte i at blk[shift+i]
  uint16_t eoff[kKvCap];                  // entry offset
  uint16_t ksrc[kKvCap];                  // offset of the unshared key bytes
  uint16_t sh[kKvCap];                    // shared length (| kRunStart)
  uint16_t klen[kKvCap];                  // internal key length
  uint16_t vsrc[kKvCap];                  // value offset (after prefix stripping)
  uint16_t vlen[kKvCap];                  // value length (after prefix stripping)
  uint32_t kout[kKvCap + 1];              // user-key output offsets (block relative)
  uint32_t vout[kKvCap + 1];              // value output offsets; first reused as run kv0
  uint8_t kvf[kKvCap];                    // PBL_KV_* flags
  uint32_t scratch[16];
  uint64_t bases[kNumComp];
  uint32_t ticket, status, slow, nkv, nrun, nres, shift;
  int32_t restarts_off;
  uint32_t tot_kb, tot_vb;
};

__device__ inline uint8_t lb(const Lds& s, uint32_t i) {
  return reinterpret_cast<const uint8_t*>(s.blk4)[s.shift + i];
}
__device__ inline uint32_t lds_le32(const Lds& s, uint32_t i) {
  return uint32_t(lb(s, i)) | uint32_t(lb(s, i + 1)) << 8 | uint32_t(lb(s, i + 2)) << 16 |
         uint32_t(lb(s, i + 3)) << 24;
}

// varint from LDS (rowblk_iter.go:2020-2038); returns bytes used, 0 if it runs past `end`
__device__ inline int lds_varint(const Lds& s, uint32_t p, uint32_t end, uint32_t* v) {
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 5; i++) {
    if (p + i >= end) return 0;
    uint32_t b = lb(s, p + i);
    if (i == 4) { *v = r | (b << 28); return 5; }
    if (b < 128) { *v = r | (b << (7 * i)); return i + 1; }
    r |= (b & 0x7f) << (7 * i);
  }
  return 0;
}

// byte p of the internal key of entry j (resolve the prefix chain backwards;
// a run's first entry has shared == 0 so the walk stays inside the run)
__device__ inline uint8_t key_byte(const Lds& s, int j, uint32_t p) {
  while (p < uint32_t(s.sh[j] & 0x7fff)) j--;
  return lb(s, s.ksrc[j] + p - (s.sh[j] & 0x7fff));
}

// 16-byte gather of block bytes [src, src+16) out of LDS (any alignment)
__device__ inline uint4 lds_gather16(const Lds& s, uint32_t src) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(s.blk4);
  uint32_t a = s.shift + src, q = a >> 2, sh = (a & 3) * 8;
  uint32_t x0 = w[q], x1 = w[q + 1], x2 = w[q + 2], x3 = w[q + 3], x4 = w[q + 4];
  uint4 r;
  if (sh == 0) { r.x = x0; r.y = x1; r.z = x2; r.w = x3; return r; }
  r.x = (x0 >> sh) | (x1 << (32 - sh));
  r.y = (x1 >> sh) | (x2 << (32 - sh));
  r.z = (x2 >> sh) | (x3 << (32 - sh));
  r.w = (x3 >> sh) | (x4 << (32 - sh));
  return r;
}

__device__ inline void put_byte(uint4& g, int i, uint32_t b) {
  uint32_t* w = reinterpret_cast<uint32_t*>(&g);
  // i is small and the loop is unrolled by callers
  w[i >> 2] |= b << ((i & 3) * 8);
}

// Store granule g covering global bytes [gaddr, gaddr+16) of which only
// [lo, hi) (absolute byte addresses) belong to this block.
__device__ inline void store_granule(uint8_t* base, uint64_t gaddr, uint64_t lo, uint64_t hi,
                                     const uint4& g) {
  if (gaddr >= lo && gaddr + 16 <= hi) {
    *reinterpret_cast<uint4*>(base + gaddr) = g;
  } else {
    const uint8_t* gb = reinterpret_cast<const uint8_t*>(&g);
#pragma unroll
    for (int i = 0; i < 16; i++) {
      uint64_t a = gaddr + i;
      if (a >= lo && a < hi) base[a] = gb[i];
    }
  }
}

// trailer + flags of entry j (LDS path)
__device__ inline uint64_t entry_trailer(const Lds& s, int j, uint8_t* fl, uint32_t flags) {
  uint32_t kl = s.klen[j];
  if (flags & PBL_ROW_RAW_KEYS) return 0;
  if (kl < 8) { *fl |= PBL_KV_INVALID_KEY; return kKindInvalid; }
  uint64_t raw = 0;
  uint32_t sh = s.sh[j] & 0x7fff;
  if (kl - 8 >= sh) {  // all 8 trailer bytes are in this entry's unshared part
    uint32_t src = s.ksrc[j] + (kl - 8 - sh);
#pragma unroll
    for (int i = 0; i < 8; i++) raw |= uint64_t(lb(s, src + i)) << (8 * i);
  } else {
#pragma unroll
    for (int i = 0; i < 8; i++) raw |= uint64_t(key_byte(s, j, kl - 8 + i)) << (8 * i);
  }
  if (raw & 64u) *fl |= PBL_KV_OBSOLETE;
  return raw & kTrailerObsoleteMask;
}

struct Args {
  pbl_block_batch in;
  pbl_decode_out out;
};

// ---------------------------------------------------------------------------
// General path: a wave-serial restatement of Iter.First/Next, block bytes read
// from global memory, current key in LDS.  Executed by wave 0 only.
// ---------------------------------------------------------------------------
struct SlowState {
  uint64_t nkv, kb, vb, nr;
  uint32_t status;
};

__device__ inline uint32_t g_varint(const uint8_t* p, const uint8_t* end, uint32_t* v) {
  uint32_t r = 0;
  for (int i = 0; i < 5; i++) {
    if (p + i >= end) return 0;
    uint32_t b = p[i];
    if (i == 4) { *v = r | (b << 28); return 5; }
    if (b < 128) { *v = r | (b << (7 * i)); return i + 1; }
    r |= (b & 0x7f) << (7 * i);
  }
  return 0;
}

__device__ inline uint32_t g_le32(const uint8_t* p) {
  return uint32_t(p[0]) | uint32_t(p[1]) << 8 | uint32_t(p[2]) << 16 | uint32_t(p[3]) << 24;
}

// pass 0 counts; pass 1 writes outputs at the given bases.
__device__ void slow_walk(const uint8_t* blk, uint64_t len, uint32_t flags, uint8_t* keybuf,
                          uint32_t keycap, int pass, const Args& A, uint32_t b,
                          const uint64_t* bases, SlowState* st) {
  const int l = lane_id();
  const uint8_t* end = blk + len;
  int32_t nr = int32_t(g_le32(blk + len - 4));
  int64_t restarts = int64_t(len) - 4 * (1 + int64_t(nr));
  const uint8_t* rtab = blk + restarts;
  uint64_t nkv = 0, kb = 0, vb = 0, full_len = 0;
  int64_t offset = 0;
  uint32_t ri = 0;
  uint32_t status = PBL_OK;
  const pbl_decode_out& O = A.out;
  while (offset >= 0 && offset < restarts) {
    const uint8_t* p = blk + offset;
    uint32_t shared, unshared, vlen;
    uint32_t a = g_varint(p, end, &shared);
    uint32_t bb = a ? g_varint(p + a, end, &unshared) : 0;
    uint32_t c = bb ? g_varint(p + a + bb, end, &vlen) : 0;
    if (!c) { status = PBL_CORRUPT_BOUNDS; break; }
    const uint8_t* kp = p + a + bb + c;
    if (uint64_t(end - kp) < unshared) { status = PBL_CORRUPT_BOUNDS; break; }
    const uint8_t* vp = kp + unshared;
    if (uint64_t(end - vp) < vlen) { status = PBL_CORRUPT_BOUNDS; break; }
    if (shared > full_len) { status = PBL_CORRUPT_BOUNDS; break; }
    uint64_t klen = uint64_t(shared) + unshared;
    if (klen > keycap) { status = PBL_UNSUPPORTED; break; }
    wave_sync();
    for (uint32_t i = l; i < unshared; i += kWave) keybuf[shared + i] = kp[i];
    wave_sync();
    full_len = klen;
    uint64_t trailer, ukl;
    uint8_t fl = 0;
    if (flags & PBL_ROW_RAW_KEYS) {
      trailer = 0;
      ukl = klen;
    } else if (klen >= 8) {
      uint64_t raw = 0;
      for (int i = 0; i < 8; i++) raw |= uint64_t(keybuf[klen - 8 + i]) << (8 * i);
      if (raw & 64u) fl |= PBL_KV_OBSOLETE;
      trailer = raw & kTrailerObsoleteMask;
      ukl = klen - 8;
    } else {
      trailer = kKindInvalid;
      ukl = 0;
      fl |= PBL_KV_INVALID_KEY;
    }
    const uint8_t* v = vp;
    uint64_t vl = vlen;
    if ((flags & PBL_ROW_VALUE_PREFIX) && !(flags & PBL_ROW_RAW_KEYS) && (trailer & 0xff) == 1) {
      if (vl == 0) { status = PBL_CORRUPT_BOUNDS; break; }
      uint8_t pre = v[0];
      if ((pre & 0xC0) == 0 || (flags & PBL_ROW_NO_VALUER)) { v++; vl--; }
      else if ((pre & 0xC0) == 0x80) fl |= PBL_KV_VALBLK_HANDLE;
      else fl |= PBL_KV_BLOB_HANDLE;
    }
    while (ri < uint32_t(nr) && int64_t(g_le32(rtab + 4 * ri) & kRestartMask) < offset) ri++;
    if (ri < uint32_t(nr) && int64_t(g_le32(rtab + 4 * ri) & kRestartMask) == offset) {
      fl |= PBL_KV_RESTART;
      if (g_le32(rtab + 4 * ri) & 0x80000000u) fl |= PBL_KV_RESTART_SAMEPFX;
    }
    if (pass == 1) {
      uint64_t kv = bases[0] + nkv, o = bases[0] + b + nkv;
      if (l == 0) {
        O.trailer[kv] = trailer;
        if (O.kv_flags) O.kv_flags[kv] = fl;
        if (O.entry_off) O.entry_off[kv] = uint32_t(offset);
        O.key_off[o] = uint32_t(kb);
        O.val_off[o] = uint32_t(vb);
      }
      uint8_t* kd = O.key_bytes + bases[1] + kb;
      for (uint64_t i = l; i < ukl; i += kWave) kd[i] = keybuf[i];
      uint8_t* vd = O.val_bytes + bases[2] + vb;
      for (uint64_t i = l; i < vl; i += kWave) vd[i] = v[i];
    }
    nkv++;
    kb += ukl;
    vb += vl;
    offset = int64_t(vp - blk) + vlen;
  }
  if (status == PBL_OK && (kb >> 32 || vb >> 32)) status = PBL_UNSUPPORTED;
  if (pass == 1 && status == PBL_OK) {
    uint64_t o = bases[0] + b + nkv;
    if (l == 0) { O.key_off[o] = uint32_t(kb); O.val_off[o] = uint32_t(vb); }
    if (O.restarts)
      for (int32_t r = l; r < nr; r += kWave) O.restarts[bases[3] + r] = g_le32(rtab + 4 * r);
  }
  st->status = status;
  st->nkv = nkv;
  st->kb = kb;
  st->vb = vb;
  st->nr = uint64_t(nr);
}

// ---------------------------------------------------------------------------
// The decode kernel.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kTPB) rowblk_decode_kernel(Args A) {
  __shared__ Lds s;
  const int t = threadIdx.x;
  const pbl_decode_out& O = A.out;
  const uint32_t nb = A.in.n_blocks;
  const uint32_t flags = A.in.flags;
  uint8_t* ws = reinterpret_cast<uint8_t*>(O.workspace);
  uint32_t* ticket_ctr = reinterpret_cast<uint32_t*>(ws);
  uint64_t* lb_state = reinterpret_cast<uint64_t*>(ws + kWsHeader);

  if (t == 0) {
    s.ticket = atomicAdd(ticket_ctr, 1u);
    s.status = PBL_OK;
    s.slow = 0;
  }
  __syncthreads();
  const uint32_t b = s.ticket;
  const uint64_t boff = A.in.block_off[b];
  const uint32_t blen = A.in.block_len[b];
  const uint8_t* gblk = A.in.blocks + boff;

  // ---- stage the block into LDS (16-byte coalesced loads) --------------------
  const uint64_t a0 = boff & ~uint64_t(15);
  const uint64_t a1 = (boff + blen + 15) & ~uint64_t(15);
  const bool fits = (a1 - a0) <= uint64_t(kLdsBlkBytes);
  if (fits) {
    const uint4* src = reinterpret_cast<const uint4*>(A.in.blocks + a0);
    const uint32_t n16 = uint32_t((a1 - a0) >> 4);
    for (uint32_t g = t; g < n16; g += kTPB) s.blk4[g] = src[g];
  }
  if (t == 0) {
    s.shift = uint32_t(boff & 15);
    // Init :248-256, readFirstKey :418-485 (cheap scalar checks from global)
    uint32_t st = PBL_OK;
    int64_t roff = 0;
    int32_t nr = 0;
    if (blen < 4) st = PBL_CORRUPT_BOUNDS;
    else {
      nr = int32_t(g_le32(gblk + blen - 4));
      if (nr == 0) st = PBL_CORRUPT_NO_RESTARTS;
      else if (nr < 0) st = PBL_CORRUPT_BOUNDS;
      else {
        roff = int64_t(blen) - 4 * (1 + int64_t(nr));
        if (roff < 0) st = PBL_CORRUPT_BOUNDS;
        else if (roff > 0 && !(flags & PBL_ROW_RAW_KEYS)) {
          if (gblk[0] != 0) st = PBL_CORRUPT_FIRST_KEY;
          else {
            uint32_t un, vl;
            uint32_t n1 = g_varint(gblk + 1, gblk + blen, &un);
            uint32_t n2 = n1 ? g_varint(gblk + 1 + n1, gblk + blen, &vl) : 0;
            if (!n2) st = PBL_CORRUPT_BOUNDS;
            else if (un < 8) st = PBL_CORRUPT_FIRST_KEY;
          }
        }
      }
    }
    s.status = st;
    s.restarts_off = int32_t(roff);
    s.nres = (st == PBL_OK) ? uint32_t(nr) : 0;
    s.slow = (st == PBL_OK && (!fits || uint32_t(nr) > uint32_t(kRunCap))) ? 1u : 0u;
  }
  __syncthreads();

  // ---- LDS path: run walks ------------------------------------------------------
  const uint32_t nres = s.nres;
  const int32_t roff = s.restarts_off;
  if (s.status == PBL_OK && !s.slow && roff > 0) {
    // A1: one lane per restart run counts its entries and checks that the walk
    // lands exactly on the next restart (else: general path).
    for (uint32_t r = t; r < nres; r += kTPB) {
      uint32_t st = uint32_t(roff) + 4 * r;
      uint32_t s0 = lds_le32(s, st) & kRestartMask;
      uint32_t e0 = (r + 1 < nres) ? (lds_le32(s, st + 4) & kRestartMask) : uint32_t(roff);
      uint32_t cnt = 0;
      bool ok = (r != 0 || s0 == 0) && s0 < e0 && e0 <= uint32_t(roff);
      uint32_t pos = s0;
      while (ok && pos < e0) {
        uint32_t sh, un, vl;
        int x = lds_varint(s, pos, e0, &sh);
        int y = x ? lds_varint(s, pos + x, e0, &un) : 0;
        int z = y ? lds_varint(s, pos + x + y, e0, &vl) : 0;
        if (!z || (cnt == 0 && sh != 0)) { ok = false; break; }
        uint64_t np = uint64_t(pos) + x + y + z + un + vl;
        if (np > e0) { ok = false; break; }
        pos = uint32_t(np);
        cnt++;
      }
      if (!ok || pos != e0) atomicOr(&s.slow, 1u);
      s.vout[r] = cnt;  // run counts (vout reused as scratch)
    }
    __syncthreads();
    if (!s.slow) {
      // exclusive scan of run counts -> run kv0 (2 runs per thread)
      uint32_t r0 = 2 * t, r1 = 2 * t + 1;
      uint32_t c0 = r0 < nres ? s.vout[r0] : 0, c1 = r1 < nres ? s.vout[r1] : 0;
      uint32_t e0, ed, tot, totd;
      block_excl_scan2(c0 + c1, 0, &e0, &ed, s.scratch, &tot, &totd);
      __syncthreads();
      if (r0 < nres) s.vout[r0] = e0;
      if (r1 < nres) s.vout[r1] = e0 + c0;
      if (t == 0) { s.nkv = tot; if (tot > uint32_t(kKvCap)) s.slow = 1; }
      __syncthreads();
    }
    if (!s.slow) {
      // A2: re-walk each run, recording per-entry geometry
      for (uint32_t r = t; r < nres; r += kTPB) {
        uint32_t st = uint32_t(roff) + 4 * r;
        uint32_t w0 = lds_le32(s, st);
        uint32_t s0 = w0 & kRestartMask;
        uint32_t e0 = (r + 1 < nres) ? (lds_le32(s, st + 4) & kRestartMask) : uint32_t(roff);
        uint32_t j = s.vout[r];
        uint32_t pos = s0, prev_kl = 0;
        bool first = true;
        while (pos < e0) {
          uint32_t sh, un, vl;
          int x = lds_varint(s, pos, e0, &sh);
          int y = lds_varint(s, pos + x, e0, &un);
          int z = lds_varint(s, pos + x + y, e0, &vl);
          if (sh > prev_kl) atomicMax(&s.status, uint32_t(PBL_CORRUPT_BOUNDS));
          s.eoff[j] = uint16_t(pos);
          s.ksrc[j] = uint16_t(pos + x + y + z);
          s.sh[j] = uint16_t(sh) | (first ? kRunStart : 0);
          s.klen[j] = uint16_t(sh + un);
          s.vsrc[j] = uint16_t(pos + x + y + z + un);
          s.vlen[j] = uint16_t(vl);
          s.kvf[j] = first ? uint8_t(PBL_KV_RESTART | ((w0 >> 31) ? PBL_KV_RESTART_SAMEPFX : 0)) : 0;
          prev_kl = sh + un;
          pos += x + y + z + un + vl;
          first = false;
          j++;
        }
      }
      __syncthreads();
      // per-KV sizes (value-prefix classification needs the trailer kind)
      const uint32_t nkv = s.nkv;
      uint32_t kl2[2], vl2[2];
#pragma unroll
      for (int q = 0; q < 2; q++) {
        uint32_t j = 2 * t + q;
        kl2[q] = vl2[q] = 0;
        if (j < nkv) {
          uint8_t fl = s.kvf[j];
          uint64_t tr = entry_trailer(s, j, &fl, flags);
          uint32_t kl = s.klen[j];
          kl2[q] = (flags & PBL_ROW_RAW_KEYS) ? kl : kl >= 8 ? kl - 8 : 0;
          uint32_t vs = s.vsrc[j], vl = s.vlen[j];
          if ((flags & PBL_ROW_VALUE_PREFIX) && !(flags & PBL_ROW_RAW_KEYS) && (tr & 0xff) == 1) {
            if (vl == 0) {
              atomicMax(&s.status, uint32_t(PBL_CORRUPT_BOUNDS));
            } else {
              uint8_t pre = lb(s, vs);
              if ((pre & 0xC0) == 0 || (flags & PBL_ROW_NO_VALUER)) { vs++; vl--; }
              else if ((pre & 0xC0) == 0x80) fl |= PBL_KV_VALBLK_HANDLE;
              else fl |= PBL_KV_BLOB_HANDLE;
            }
          }
          s.vsrc[j] = uint16_t(vs);
          s.vlen[j] = uint16_t(vl);
          s.kvf[j] = fl;
          vl2[q] = vl;
        }
      }
      uint32_t ek, ev, tk, tv;
      block_excl_scan2(kl2[0] + kl2[1], vl2[0] + vl2[1], &ek, &ev, s.scratch, &tk, &tv);
      {
        uint32_t j = 2 * t;
        if (j < nkv) { s.kout[j] = ek; s.vout[j] = ev; }
        if (j + 1 < nkv) { s.kout[j + 1] = ek + kl2[0]; s.vout[j + 1] = ev + vl2[0]; }
        if (t == 0) { s.kout[nkv] = tk; s.vout[nkv] = tv; s.tot_kb = tk; s.tot_vb = tv; }
      }
      __syncthreads();
    }
  } else if (t == 0) {
    s.nkv = 0;
    s.tot_kb = s.tot_vb = 0;
    if (s.status == PBL_OK && !s.slow) {  // empty block (restarts offset 0)
      s.kout[0] = s.vout[0] = 0;
    }
  }
  __syncthreads();

  // ---- general path (wave 0 only) -------------------------------------------------
  if (s.slow && s.status == PBL_OK) {
    if (wave_id() != 0) return;
    // keybuf: the block staging area when the block is read from global memory,
    // else the per-KV arrays (unused on this path)
    uint8_t* keybuf = fits ? reinterpret_cast<uint8_t*>(s.eoff)
                           : reinterpret_cast<uint8_t*>(s.blk4);
    uint32_t keycap = fits ? uint32_t(reinterpret_cast<uint8_t*>(s.scratch) -
                                      reinterpret_cast<uint8_t*>(s.eoff))
                           : uint32_t(kLdsBlkBytes);
    const uint8_t* src = fits ? reinterpret_cast<const uint8_t*>(s.blk4) + s.shift : gblk;
    SlowState ss;
    uint64_t dummy[kNumComp] = {0, 0, 0, 0};
    slow_walk(src, blen, flags, keybuf, keycap, 0, A, b, dummy, &ss);
    uint64_t agg[kNumComp], excl[kNumComp];
    bool ok = ss.status == PBL_OK;
    agg[0] = ok ? ss.nkv : 0;
    agg[1] = ok ? ss.kb : 0;
    agg[2] = ok ? ss.vb : 0;
    agg[3] = ok ? ss.nr : 0;
    lookback(lb_state, nb, b, agg, excl, &O.totals->status_mask);
    uint32_t status = ss.status;
    if (ok && (excl[0] + agg[0] > O.kv_cap || excl[1] + agg[1] > O.key_cap ||
               excl[2] + agg[2] > O.val_cap || (O.restarts && excl[3] + agg[3] > O.rst_cap)))
      status = PBL_OVERFLOW;
    if (status == PBL_OK) {
      slow_walk(src, blen, flags, keybuf, keycap, 1, A, b, excl, &ss);
    } else if (lane_id() == 0 && excl[0] + b < O.kv_cap + nb) {
      O.key_off[excl[0] + b] = 0;
      O.val_off[excl[0] + b] = 0;
    }
    if (lane_id() == 0) {
      O.blk_kv_base[b] = excl[0];
      O.blk_key_base[b] = excl[1];
      O.blk_val_base[b] = excl[2];
      if (O.blk_rst_base) O.blk_rst_base[b] = excl[3];
      O.blk_status[b] = status;
      atomicAdd(&O.totals->n_slow_blocks, 1u);
      if (status != PBL_OK) {
        atomicOr(&O.totals->status_mask, 1u << status);
        atomicAdd(&O.totals->n_bad_blocks, 1u);
      }
      if (b == nb - 1) {
        O.blk_kv_base[nb] = excl[0] + agg[0];
        O.blk_key_base[nb] = excl[1] + agg[1];
        O.blk_val_base[nb] = excl[2] + agg[2];
        if (O.blk_rst_base) O.blk_rst_base[nb] = excl[3] + agg[3];
        O.totals->n_kv = excl[0] + agg[0];
        O.totals->key_bytes = excl[1] + agg[1];
        O.totals->val_bytes = excl[2] + agg[2];
        O.totals->n_restarts = excl[3] + agg[3];
      }
    }
    return;
  }

  // ---- LDS path: look-back, then writes -------------------------------------------
  const bool ok = s.status == PBL_OK;
  const uint32_t nkv = ok ? s.nkv : 0;
  if (wave_id() == 0) {
    uint64_t agg[kNumComp], excl[kNumComp];
    agg[0] = nkv;
    agg[1] = ok ? s.tot_kb : 0;
    agg[2] = ok ? s.tot_vb : 0;
    agg[3] = ok ? nres : 0;
    lookback(lb_state, nb, b, agg, excl, &O.totals->status_mask);
    if (lane_id() == 0) {
      uint32_t status = s.status;
      if (ok && (excl[0] + agg[0] > O.kv_cap || excl[1] + agg[1] > O.key_cap ||
                 excl[2] + agg[2] > O.val_cap || (O.restarts && excl[3] + agg[3] > O.rst_cap)))
        status = PBL_OVERFLOW;
      s.status = status;
#pragma unroll
      for (int c = 0; c < kNumComp; c++) s.bases[c] = excl[c];
      O.blk_kv_base[b] = excl[0];
      O.blk_key_base[b] = excl[1];
      O.blk_val_base[b] = excl[2];
      if (O.blk_rst_base) O.blk_rst_base[b] = excl[3];
      O.blk_status[b] = status;
      if (status != PBL_OK) {
        atomicOr(&O.totals->status_mask, 1u << status);
        atomicAdd(&O.totals->n_bad_blocks, 1u);
        if (excl[0] + b < O.kv_cap + nb) { O.key_off[excl[0] + b] = 0; O.val_off[excl[0] + b] = 0; }
      }
      if (b == nb - 1) {
        O.blk_kv_base[nb] = excl[0] + agg[0];
        O.blk_key_base[nb] = excl[1] + agg[1];
        O.blk_val_base[nb] = excl[2] + agg[2];
        if (O.blk_rst_base) O.blk_rst_base[nb] = excl[3] + agg[3];
        O.totals->n_kv = excl[0] + agg[0];
        O.totals->key_bytes = excl[1] + agg[1];
        O.totals->val_bytes = excl[2] + agg[2];
        O.totals->n_restarts = excl[3] + agg[3];
      }
    }
  }
  __syncthreads();
  if (s.status != PBL_OK) return;

  const uint64_t kvb = s.bases[0], kbb = s.bases[1], vbb = s.bases[2], rbb = s.bases[3];
  // per-KV arrays (coalesced, thread per KV)
  for (uint32_t j = t; j <= nkv; j += kTPB) {
    uint64_t o = kvb + b + j;
    O.key_off[o] = s.kout[j];
    O.val_off[o] = s.vout[j];
    if (j < nkv) {
      uint8_t fl = s.kvf[j];
      uint64_t tr = entry_trailer(s, j, &fl, flags);
      O.trailer[kvb + j] = tr;
      if (O.kv_flags) O.kv_flags[kvb + j] = fl;
      if (O.entry_off) O.entry_off[kvb + j] = s.eoff[j];
    }
  }
  if (O.restarts)
    for (uint32_t r = t; r < nres; r += kTPB) O.restarts[rbb + r] = lds_le32(s, uint32_t(roff) + 4 * r);

  // key bytes: 16-byte granules over [kbb, kbb + KB)
  {
    const uint64_t lo = kbb, hi = kbb + s.tot_kb;
    const uint64_t g0 = lo & ~uint64_t(15);
    for (uint64_t ga = g0 + 16ull * t; ga < hi; ga += 16ull * kTPB) {
      uint4 g = make_uint4(0, 0, 0, 0);
      uint64_t first = ga < lo ? lo : ga;
      uint32_t o = uint32_t(first - lo);
      // largest j with kout[j] <= o (skipping empty keys)
      int lo_j = 0, hi_j = int(nkv) - 1;
      while (lo_j < hi_j) {
        int mid = (lo_j + hi_j + 1) >> 1;
        if (s.kout[mid] <= o) lo_j = mid; else hi_j = mid - 1;
      }
      int j = lo_j;
      int src = -1;  // resolved source entry for the current key/position
#pragma unroll
      for (int i = 0; i < 16; i++) {
        uint64_t a = ga + i;
        if (a < lo || a >= hi) continue;
        uint32_t oo = uint32_t(a - lo);
        while (s.kout[j + 1] <= oo) { j++; src = -1; }
        uint32_t p = oo - s.kout[j];
        if (src < 0) {
          src = j;
          while (p < uint32_t(s.sh[src] & 0x7fff)) src--;
        } else {
          while (src < j && uint32_t(s.sh[src + 1] & 0x7fff) <= p) src++;
        }
        put_byte(g, i, lb(s, s.ksrc[src] + p - (s.sh[src] & 0x7fff)));
      }
      store_granule(O.key_bytes, ga, lo, hi, g);
    }
  }
  // value bytes: 16-byte granules over [vbb, vbb + VB)
  {
    const uint64_t lo = vbb, hi = vbb + s.tot_vb;
    const uint64_t g0 = lo & ~uint64_t(15);
    for (uint64_t ga = g0 + 16ull * t; ga < hi; ga += 16ull * kTPB) {
      uint64_t first = ga < lo ? lo : ga;
      uint32_t o = uint32_t(first - lo);
      int lo_j = 0, hi_j = int(nkv) - 1;
      while (lo_j < hi_j) {
        int mid = (lo_j + hi_j + 1) >> 1;
        if (s.vout[mid] <= o) lo_j = mid; else hi_j = mid - 1;
      }
      int j = lo_j;
      uint4 g;
      if (ga >= lo && ga + 16 <= hi && ga + 16 - lo <= s.vout[j + 1]) {
        g = lds_gather16(s, s.vsrc[j] + (o - s.vout[j]));
      } else {
        g = make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 16; i++) {
          uint64_t a = ga + i;
          if (a < lo || a >= hi) continue;
          uint32_t oo = uint32_t(a - lo);
          while (s.vout[j + 1] <= oo) j++;
          put_byte(g, i, lb(s, s.vsrc[j] + (oo - s.vout[j])));
        }
      }
      store_granule(O.val_bytes, ga, lo, hi, g);
    }
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

extern "C" {

int pbl_abi_version(void) { return PBL_ABI_VERSION; }

uint64_t pbl_workspace_bytes(uint32_t n_blocks) { return pbl::ws_bytes(n_blocks); }

int pbl_decode_batch_colblk(const pbl_block_batch* batch, pbl_decode_out* out, void* stream);

int pbl_decode_batch(const pbl_block_batch* batch, pbl_decode_out* out, void* stream) {
  if (!batch || !out) return PBL_INVALID_ARG;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (!out->totals || !out->blk_kv_base || !out->blk_key_base || !out->blk_val_base ||
      !out->blk_status)
    return PBL_INVALID_ARG;
  if (hipMemsetAsync(out->totals, 0, sizeof(pbl_totals), st) != hipSuccess) return PBL_DEVICE_ERROR;
  if (batch->n_blocks == 0) return PBL_OK;
  if (!batch->blocks || !batch->block_off || !batch->block_len || !out->trailer ||
      !out->key_off || !out->val_off || !out->key_bytes || !out->val_bytes || !out->workspace ||
      out->workspace_bytes < pbl::ws_bytes(batch->n_blocks))
    return PBL_INVALID_ARG;
  if (batch->format != PBL_FMT_ROW) return pbl_decode_batch_colblk(batch, out, stream);
  if (hipMemsetAsync(out->workspace, 0, pbl::ws_bytes(batch->n_blocks), st) != hipSuccess)
    return PBL_DEVICE_ERROR;
  pbl::row::Args a;
  a.in = *batch;
  a.out = *out;
  hipLaunchKernelGGL(pbl::row::rowblk_decode_kernel, dim3(batch->n_blocks), dim3(pbl::kTPB), 0, st, a);
  return hipGetLastError() == hipSuccess ? PBL_OK : PBL_DEVICE_ERROR;
}

int pbl_rebase_blocks(pbl_decode_out* out, uint32_t n_blocks, uint64_t kv_base, uint64_t key_base,
                      uint64_t val_base, uint64_t rst_base, void* stream) {
  if (!out || !out->blk_kv_base || !out->blk_key_base || !out->blk_val_base) return PBL_INVALID_ARG;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  uint32_t n = n_blocks + 1;
  hipLaunchKernelGGL(pbl::row::rebase_kernel, dim3((n + 255) / 256), dim3(256), 0, st,
                     out->blk_kv_base, out->blk_key_base, out->blk_val_base, out->blk_rst_base,
                     n_blocks, kv_base, key_base, val_base, rst_base);
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
