// zstd_fast.hip.h — the batch path of the zstd decoder (zstd.hip): the
// sequential parts of every block run one lane per chain, so their latency
// chains overlap across the whole batch instead of stalling one wave per block.
//
// A Pebble zstd block is one frame holding one compressed zstd block for every
// block Pebble writes (32 KiB of data, zstd_cgo.go:45-66; the zstd block limit
// is 128 KiB).  Such blocks take four launches; everything else (raw / RLE zstd
// blocks, several frames or blocks, skippable frames, a treeless or repeat
// table in the first block, any inconsistency found while planning, decoded
// blocks past the window) is left to zstd_kernel, which decodes every block
// the plan did not take and reports its status.
//
//   zstd_prep_kernel  a wave per block: frame, block and literals headers, the
//                     Huffman table and the three sequence tables (RFC 8878
//                     §4.1, §4.2) built in LDS from two staged 1 KiB header
//                     windows and written to the block's table slot; raw / RLE
//                     literals copied to the end of the block's output; a
//                     descriptor per block (fast or not, streams, counts)
//   zstd_lit_kernel   a lane per Huffman stream (four per block): the stream's
//                     literals to [D - regen + s * seg, ...) of the output,
//                     table lookups from the slot, aligned 4-B stores
//   zstd_seq_kernel   a lane per block: the FSE states and the repeat offsets
//                     (§3.1.1.5, §4.1.2) to one packed 8-B word per sequence
//   zstd_exec_kernel  a wave per block, the decoded block in an LDS window:
//                     64 sequences at a time, their literal runs and output
//                     places from two wave scans, literals copied lane per
//                     sequence from the output's literal region, then the
//                     matches in groups of sequences whose sources lie below
//                     the group's first output (lane per match; a match past
//                     64 bytes takes the whole wave); the window written out
//                     as 16-B granules, overwriting the literal region last.
//
// Corruption found by the lanes (a stream that does not end exactly on its
// first bit, a sequence out of bounds) gives PBL_CORRUPT_COMPRESSION, as
// zstd_kernel would; corruption found while planning leaves the block to
// zstd_kernel, so every status is zstd_kernel's.
#pragma once

namespace pbl {
namespace zstd {

constexpr uint32_t kFastWin = kOut;   // decoded bytes per block on this path (LDS window)
constexpr uint32_t kHdrWin = 1024;    // staged header bytes per window
constexpr uint32_t kTblBytes = 6656;  // per-block table slot: Huffman 2048 x u16, LL 512 / OF 256 / ML 512 x u16
// sequence words of workspace per block, shared through a bump counter (text
// at level 3 runs ~4.7 K sequences per 32 KiB block; a block that finds the
// area full is left to zstd_kernel)
// Sequence words reserved per block ON AVERAGE: the area is one bump
// allocation (seq_ctr) over the whole batch, so a long block borrows from short
// ones; a batch that runs out sends the rest of its blocks to zstd_kernel.  A
// 32 KiB text block at ratio 2.66 holds ~3-4 K sequences.
constexpr uint32_t kSeqPerBlock = 4096;

struct FDesc {
  uint32_t fast, D, regen, ltype;
  uint32_t streams, huf_log, nseq, seq_base;
  uint32_t s_off[4];  // Huffman streams: byte offsets from the Pebble block start
  uint32_t s_len[4];
  uint32_t cnt[4];    // literals per stream
  uint32_t q_off, q_len, al, cksum;  // sequence bitstream; al_ll | al_of << 8 | al_ml << 16; checksum flag
  uint32_t ck, flags, rsv0, rsv1;    // expected checksum (low 32 bits of XXH64); bad-stream bits (set by lanes)
  uint32_t rsv2[4];
};
static_assert(sizeof(FDesc) == 128, "descriptor slot");

struct WsHdr {
  uint32_t seq_ctr;  // bump counter of the sequence area
  uint32_t pad[63];
};

struct FastWs {
  WsHdr* hdr;
  FDesc* desc;
  uint8_t* tbl;
  uint64_t* seq;
  uint32_t seq_cap;
  __device__ __host__ static uint64_t bytes(uint32_t n) {
    return sizeof(WsHdr) + uint64_t(n) * sizeof(FDesc) + uint64_t(n) * kTblBytes + uint64_t(n) * kSeqPerBlock * 8;
  }
  __device__ __host__ static FastWs at(void* ws, uint32_t n) {
    FastWs W;
    uint8_t* p = static_cast<uint8_t*>(ws);
    W.hdr = reinterpret_cast<WsHdr*>(p);
    W.desc = reinterpret_cast<FDesc*>(p + sizeof(WsHdr));
    W.tbl = p + sizeof(WsHdr) + uint64_t(n) * sizeof(FDesc);
    W.seq = reinterpret_cast<uint64_t*>(W.tbl + uint64_t(n) * kTblBytes);
    W.seq_cap = uint32_t(std::min<uint64_t>(uint64_t(n) * kSeqPerBlock, 0xffffffffull));
    return W;
  }
  __device__ uint16_t* huf(uint32_t b) const { return reinterpret_cast<uint16_t*>(tbl + uint64_t(b) * kTblBytes); }
  __device__ uint16_t* ll(uint32_t b) const { return reinterpret_cast<uint16_t*>(tbl + uint64_t(b) * kTblBytes + 4096); }
  __device__ uint16_t* of(uint32_t b) const { return ll(b) + 512; }
  __device__ uint16_t* ml(uint32_t b) const { return ll(b) + 768; }
};

// Sequence-table entry (u16): the state's occurrence counter x (10 bits: the
// FSE build's next[s]++, in [count, 2 count)) | symbol << 10.  A decoder gets
// nb = al - highbit(x) and the next-state base (x << nb) - 2^al from it
// (RFC 8878 §4.1.1), and the symbol's baseline and extra bits from the
// symbol; 2.5 KB of tables per block keeps a batch's tables inside the
// Infinity Cache.  From the LDS build's entries (sym | nb << 8 | base << 16).
__device__ __forceinline__ uint16_t seq_entry(uint32_t e, uint32_t al) {
  const uint32_t nb = (e >> 8) & 0xff, x = ((e >> 16) + (1u << al)) >> nb;
  return uint16_t(x | (e & 0xff) << 10);
}

// Bytes [lo, lo + len) of the block staged in LDS; reads outside read 0 (the
// parsers are handed lengths that end inside the window).
struct WinIn {
  lptr<const uint8_t> p;
  uint32_t lo;
  __device__ uint32_t operator[](uint32_t i) const { return p[i - lo]; }
};

struct PrepLds {
  alignas(16) uint8_t win[2][kHdrWin + 32];
  uint32_t fse[3][512];
  uint32_t wt[64];
  uint16_t huf[2048];
  uint8_t w[256];
  int16_t norm[256];
  uint16_t aux[256];
};

// Stage block bytes [a, a + kHdrWin) (clipped to the block's readable end) into
// win at offset (a & 15); returns the WinIn for it.
__device__ inline WinIn stage_win(uint8_t* win, const uint8_t* blk, uint32_t a, uint32_t n_read) {
  const uint64_t sa = reinterpret_cast<uint64_t>(blk + a);
  const uint32_t ssh = uint32_t(sa & 15);
  const uint32_t want = n_read > a ? min(n_read - a, kHdrWin) : 0u;
  const uint32_t ng = (ssh + want + 15) / 16;
  const gptr<const u32x4> sg = to_glb(reinterpret_cast<const u32x4*>(sa - ssh));
  lds_stage16(to_lds_ptr(reinterpret_cast<u32x4*>(win)), sg, ng);
  WinIn W;
  W.p = to_lds_ptr(static_cast<const uint8_t*>(win)) + ssh;
  W.lo = a;
  return W;
}

// The last step of an FSE table build (fse_build after its spread) by the
// whole wave: entry u of symbol s gets x = next[s]++ in u order, i.e. next[s]
// plus the number of entries of s before u.  Lanes take 64 entries at a time;
// a lane's rank among the chunk's lanes with its symbol comes from one ballot
// per distinct symbol in the chunk.
__device__ inline void fse_finish_wave(lptr<uint32_t> T, lptr<uint16_t> next, uint32_t al) {
  const uint32_t lane = lane_id(), size = 1u << al;
  for (uint32_t c = 0; c < size; c += kWave) {
    const uint32_t u = c + lane;
    const bool valid = u < size;
    const uint32_t s = valid ? (T[u] & 0xff) : 0xffffu;
    uint32_t rank = 0, cnt = 0;
    for (uint64_t rem = __ballot(valid); rem;) {
      const uint32_t sl = __builtin_amdgcn_readlane(s, __builtin_ctzll(rem));
      const uint64_t m = __ballot(valid && s == sl);
      if (valid && s == sl) {
        rank = uint32_t(__builtin_popcountll(m & ((1ull << lane) - 1)));
        cnt = uint32_t(__builtin_popcountll(m));
      }
      rem &= ~m;
    }
    const uint32_t x = (valid ? uint32_t(next[s]) : 0u) + rank;
    wave_sync();  // (every lane has read next[] before any lane bumps it)
    if (valid && rank + 1 == cnt) next[s] = uint16_t(x + 1);
    if (valid) {
      const uint32_t nb = al - uint32_t(highbit(x));
      T[u] = s | nb << 8 | ((x << nb) - size) << 16;
    }
    wave_sync();
  }
}

// ---- plan --------------------------------------------------------------------
__global__ void __launch_bounds__(kWave) zstd_prep_kernel(const pbl_phys_batch B, uint8_t* out, const uint64_t* out_off,
                                                          const uint32_t* out_cap, void* ws) {
  __shared__ PrepLds L;
  const uint32_t lane = lane_id();
  const FastWs W = FastWs::at(ws, B.n_blocks);
  for (uint32_t b = blockIdx.x; b < B.n_blocks; b += gridDim.x) {
    FDesc d;
    d.fast = 0;
    const uint32_t n = to_glb(B.block_len)[b];
    const uint8_t* blk = B.bytes + to_glb(B.block_off)[b];
    const gptr<const uint8_t> src = to_glb(blk);
    bool fast = src[n] == PBL_COMPRESSION_ZSTD;
    uint32_t D = 0, used = 0;
    if (fast) fast = uvarint32(src, n, &D, &used) && D > 0 && used < n && D <= kFastWin && D <= to_glb(out_cap)[b];
    // ---- frame header, block header, literals section (window 0) ----------
    uint32_t q = used, end = n;
    WinIn w0{};
    if (fast) w0 = stage_win(L.win[0], blk, used, n + 4);
    const uint32_t e0 = min(n, used + kHdrWin);  // parse limit inside window 0
    uint32_t fl = 0, cks = 0, bs = 0;
    if (fast) {
      fast = e0 - q >= 6 && le_n(w0, q, 4) == 0xFD2FB528u;
      if (fast) {
        q += 4;
        const uint32_t fhd = w0[q++];
        const uint32_t fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, did = fhd & 3;
        cks = (fhd >> 2) & 1;
        const uint32_t dl = did == 0 ? 0 : did == 1 ? 1 : did == 2 ? 2 : 4;
        fl = fcs_flag == 0 ? (single ? 1 : 0) : fcs_flag == 1 ? 2 : fcs_flag == 2 ? 4 : 8;
        fast = !(fhd & 8) && did == 0 && q + (single ? 0 : 1) + dl + fl + 3 <= e0;
        if (fast) {
          q += single ? 0 : 1;
          uint64_t fcs = 0;
          for (uint32_t i = 0; i < fl; i++) fcs |= uint64_t(w0[q + i]) << (8 * i);
          if (fl == 2) fcs += 256;
          q += fl;
          if (fl && fcs != D) fast = false;
          const uint32_t bh = w0[q] | w0[q + 1] << 8 | w0[q + 2] << 16;
          q += 3;
          bs = bh >> 3;
          // one compressed, last block; the frame (and its checksum) ends the Pebble block
          fast = fast && (bh & 1) && ((bh >> 1) & 3) == 2 && bs <= (1u << 17) && q + bs + 4 * cks == n && bs >= 1;
          end = q + bs;
          if (fast && cks) d.ck = le_n(GIn{src}, end, 4);
        }
      }
    }
    // literals header
    uint32_t ltype = 0, regen = 0, csize = 0, streams = 1, h = 0;
    if (fast) {
      const uint32_t b0 = w0[q], sf = (b0 >> 2) & 3;
      ltype = b0 & 3;
      if (ltype < 2) {
        h = (sf == 0 || sf == 2) ? 1 : sf == 1 ? 2 : 3;
        if (q + h > e0) fast = false;
        else regen = h == 1 ? b0 >> 3 : h == 2 ? (b0 >> 4) + (w0[q + 1] << 4) : (b0 >> 4) + (w0[q + 1] << 4) + (w0[q + 2] << 12);
      } else {
        h = sf < 2 ? 3 : sf == 2 ? 4 : 5;
        if (q + h > e0) {
          fast = false;
        } else if (sf < 2) {
          regen = (b0 >> 4) + ((w0[q + 1] & 0x3f) << 4);
          csize = (w0[q + 1] >> 6) + (w0[q + 2] << 2);
          streams = sf == 0 ? 1 : 4;
        } else if (sf == 2) {
          regen = (b0 >> 4) + (w0[q + 1] << 4) + ((w0[q + 2] & 3) << 12);
          csize = (w0[q + 2] >> 2) + (w0[q + 3] << 6);
          streams = 4;
        } else {
          regen = (b0 >> 4) + (w0[q + 1] << 4) + ((w0[q + 2] & 0x3f) << 12);
          csize = (w0[q + 2] >> 6) + (w0[q + 3] << 2) + (w0[q + 4] << 10);
          streams = 4;
        }
      }
      fast = fast && ltype != 3 && regen <= D;
    }
    const uint32_t lit0 = D - regen;
    uint8_t* dst = out + to_glb(out_off)[b];
    uint32_t huf_log = 0;
    if (fast) {
      const uint32_t lq = q + h;
      if (ltype == 0) {
        fast = lq + regen <= end;
        if (fast)
          for (uint32_t i = lane; i < regen; i += kWave) to_glb(dst)[lit0 + i] = src[lq + i];
        q = lq + regen;
      } else if (ltype == 1) {
        fast = lq + 1 <= end;
        if (fast) {
          const uint8_t v = src[lq];
          for (uint32_t i = lane; i < regen; i += kWave) to_glb(dst)[lit0 + i] = v;
        }
        q = lq + 1;
      } else {
        fast = lq + csize <= end;
        if (fast) {
          // the tree description must end inside window 0
          const int32_t t = huf_read(L, w0, lq, min(csize, e0 > lq ? e0 - lq : 0u), &huf_log);
          fast = t >= 0;
          uint32_t c = lq + uint32_t(t > 0 ? t : 0), cn = csize - uint32_t(t > 0 ? t : 0);
          if (fast && streams == 4) {
            fast = cn >= 6 && c + 6 <= e0;
            if (fast) {
              const uint32_t l1 = w0[c] | w0[c + 1] << 8, l2 = w0[c + 2] | w0[c + 3] << 8, l3 = w0[c + 4] | w0[c + 5] << 8;
              const uint32_t seg = (regen + 3) / 4;
              fast = 6 + l1 + l2 + l3 <= cn && 3 * seg <= regen;
              d.s_off[0] = c + 6;
              d.s_len[0] = l1;
              d.s_off[1] = c + 6 + l1;
              d.s_len[1] = l2;
              d.s_off[2] = c + 6 + l1 + l2;
              d.s_len[2] = l3;
              d.s_off[3] = c + 6 + l1 + l2 + l3;
              d.s_len[3] = cn - 6 - l1 - l2 - l3;
              d.cnt[0] = d.cnt[1] = d.cnt[2] = seg;
              d.cnt[3] = regen - 3 * seg;
            }
          } else if (fast) {
            d.s_off[0] = c;
            d.s_len[0] = cn;
            d.cnt[0] = regen;
          }
        }
        q = lq + csize;
      }
    }
    // ---- sequences section header and tables (window 1) ----------------------
    uint32_t nseq = 0, al_ll = 0, al_of = 0, al_ml = 0;
    if (fast) fast = q < end;
    if (fast) {
      WinIn w1 = stage_win(L.win[1], blk, q, n + 4);
      const uint32_t e1 = min(end, q + kHdrWin);
      {
        nseq = w1[q];
        if (nseq < 128) {
          q += 1;
        } else if (nseq < 255) {
          fast = q + 2 <= e1;
          if (fast) nseq = ((nseq - 128) << 8) + w1[q + 1];
          q += 2;
        } else {
          fast = q + 3 <= e1;
          if (fast) nseq = w1[q + 1] + (w1[q + 2] << 8) + 0x7F00;
          q += 3;
        }
      }
      if (fast && nseq > 0) {
        fast = q < e1;
        const uint32_t modes = fast ? w1[q] : 0u;
        q++;
        // no repeat mode in a frame's first block (zstd_kernel reports it)
        fast = fast && !(modes & 3) && (modes >> 6) != 3 && ((modes >> 4) & 3) != 3 && ((modes >> 2) & 3) != 3;
        // each table: lane 0 reads its description and spreads its symbols,
        // the wave finishes it (modes 0 and 2; an RLE table is one entry)
        const uint32_t lim = e1 > q ? e1 - q : 0u;
        const uint32_t mode[3] = {modes >> 6, (modes >> 4) & 3, (modes >> 2) & 3};
        int32_t u = 0;
        uint32_t al3[3] = {0, 0, 0};
        for (int t = 0; t < 3 && fast; t++) {
          int32_t ut = 0;
          uint32_t alt = 0;
          if (lane == 0) {
            bool have = false;
            const uint32_t at = q + uint32_t(u), lt = lim - uint32_t(u);
            ut = t == 0 ? seq_table<true>(to_lds_ptr(L.fse[0]), L, mode[0], kLLDef, 36, 6, 9, 35, w1, at, lt, &alt, &have)
                 : t == 1 ? seq_table<true>(to_lds_ptr(L.fse[1]), L, mode[1], kOFDef, 29, 5, 8, 31, w1, at, lt, &alt, &have)
                          : seq_table<true>(to_lds_ptr(L.fse[2]), L, mode[2], kMLDef, 53, 6, 9, 52, w1, at, lt, &alt, &have);
          }
          ut = __shfl(ut, 0, kWave);
          alt = __shfl(alt, 0, kWave);
          wave_sync();
          if (ut < 0) {
            u = -1;
            break;
          }
          if (mode[t] != 1) fse_finish_wave(to_lds_ptr(L.fse[t]), to_lds_ptr(static_cast<uint16_t*>(L.aux)), alt);
          al3[t] = alt;
          u += ut;
        }
        al_ll = al3[0];
        al_of = al3[1];
        al_ml = al3[2];
        fast = fast && u >= 0 && q + uint32_t(u) < end;
        if (fast) {
          q += uint32_t(u);
          // the tables, baselines folded in (RFC 8878 §3.1.1.3.2.1.1)
          for (uint32_t i = lane; i < (1u << al_ll); i += kWave) to_glb(W.ll(b))[i] = seq_entry(L.fse[0][i], al_ll);
          for (uint32_t i = lane; i < (1u << al_of); i += kWave) to_glb(W.of(b))[i] = seq_entry(L.fse[1][i], al_of);
          for (uint32_t i = lane; i < (1u << al_ml); i += kWave) to_glb(W.ml(b))[i] = seq_entry(L.fse[2][i], al_ml);
        }
      } else if (fast && q != end) {
        fast = false;
      }
    }
    if (fast && ltype == 2) {
      const lptr<const uint16_t> H = to_lds_ptr(static_cast<const uint16_t*>(L.huf));
      for (uint32_t i = lane; i < (1u << huf_log); i += kWave) to_glb(W.huf(b))[i] = H[i];
    }
    // the sequence words
    uint32_t sb = 0;
    if (fast && lane == 0 && nseq) sb = g_atomic_add(&W.hdr->seq_ctr, nseq);
    sb = __shfl(sb, 0, kWave);
    if (fast && nseq && (sb > W.seq_cap || nseq > W.seq_cap - sb)) fast = false;
    wave_sync();
    if (lane == 0) {
      FDesc* g = W.desc + b;
      g->D = D;
      g->regen = regen;
      g->ltype = ltype;
      g->streams = streams;
      g->huf_log = huf_log;
      g->nseq = nseq;
      g->seq_base = sb;
      for (int s = 0; s < 4; s++) {
        g->s_off[s] = ltype == 2 && s < int(streams) ? d.s_off[s] : 0u;
        g->s_len[s] = ltype == 2 && s < int(streams) ? d.s_len[s] : 0u;
        g->cnt[s] = ltype == 2 && s < int(streams) ? d.cnt[s] : 0u;
      }
      g->q_off = q;
      g->q_len = end > q ? end - q : 0u;
      g->al = al_ll | al_of << 8 | al_ml << 16;
      g->cksum = cks;
      g->ck = cks ? d.ck : 0u;
      g->flags = 0;
      g->fast = fast ? 1u : 0u;
    }
  }
}

// ---- lane-per-stream / lane-per-block bit reader ------------------------------
// Backward bitstream over global bytes [0, n) of p (RFC 8878 §4.1): unread bits
// [0, pos); the container c holds bits [cb, cb + 64), refilled from a register
// window: stream bytes [wb, wb + 64) of p in eight u64 (wb a 16-B aligned
// address), slid 16 bytes down whenever a refill reaches the window's lowest 16
// bytes, so the granule a slide loads is first needed ~16 bytes of stream later
// (a few symbols or sequences): refills read registers, not memory.  Granules
// below p's own granule or past its last byte read as 0.
struct GBitsW {
  uint64_t pa, lo_a, hi_a;  // p; lowest and highest loadable granule addresses
  uint32_t n;
  int32_t pos, cb;
  uint64_t c, wb;
  uint64_t w0, w1, w2, w3, w4, w5, w6, w7;
  __device__ __forceinline__ void ld(uint64_t a, uint64_t& x, uint64_t& y) const {
    if (a >= lo_a && a <= hi_a) {
      const u32x4 v = *(gptr<const u32x4>)(reinterpret_cast<const u32x4*>(a));
      x = uint64_t(v[0]) | uint64_t(v[1]) << 32;
      y = uint64_t(v[2]) | uint64_t(v[3]) << 32;
    } else {
      x = y = 0;
    }
  }
  __device__ __forceinline__ uint64_t sel(uint32_t k) const {
    const uint64_t a = (k & 1) ? w1 : w0, b = (k & 1) ? w3 : w2, cc = (k & 1) ? w5 : w4, d = (k & 1) ? w7 : w6;
    const uint64_t e = (k & 2) ? b : a, f = (k & 2) ? d : cc;
    return (k & 4) ? f : e;
  }
  __device__ __forceinline__ void refill() {
    int32_t b = (pos - 57) >> 3;
    if (b < 0) b = 0;
    cb = 8 * b;
    const uint64_t a = pa + uint32_t(b);
    if (a < wb || a - wb > 56) {  // (only after a corrupt jump)
      wb = (a & ~uint64_t(15)) - 32;
      ld(wb, w0, w1);
      ld(wb + 16, w2, w3);
      ld(wb + 32, w4, w5);
      ld(wb + 48, w6, w7);
    } else {
      while (a < wb + 16 && wb > lo_a) {
        w7 = w5; w6 = w4; w5 = w3; w4 = w2; w3 = w1; w2 = w0;
        wb -= 16;
        ld(wb, w0, w1);
      }
    }
    const uint32_t o = uint32_t(a - wb), k = o >> 3, sh = 8 * (o & 7);
    const uint64_t lo = sel(k);
    c = sh ? (lo >> sh) | (sel(k + 1) << (64 - sh)) : lo;
    if (uint32_t(b) + 8 > n) c &= (~0ull >> (8 * (uint32_t(b) + 8 - n)));  // (bytes past the stream)
  }
  __device__ __forceinline__ bool init(gptr<const uint8_t> src, uint32_t len) {
    pa = reinterpret_cast<uint64_t>(src);
    n = len;
    if (len == 0) return false;
    lo_a = pa & ~uint64_t(15);
    hi_a = (pa + len - 1) & ~uint64_t(15);
    const uint32_t last = src[len - 1];
    if (last == 0) return false;
    pos = int32_t(8 * len) - 8 + highbit(last);
    wb = hi_a - 48;
    ld(wb, w0, w1);
    ld(wb + 16, w2, w3);
    ld(wb + 32, w4, w5);
    ld(wb + 48, w6, w7);
    refill();
    return true;
  }
  __device__ __forceinline__ uint32_t read(uint32_t k) {
    if (k == 0) return 0;
    const int32_t lo = pos - int32_t(k);
    if (lo < cb && cb > 0) refill();
    uint64_t v;
    if (lo >= cb) v = c >> (lo - cb);
    else if (pos <= 0) v = 0;
    else v = c << (-lo);
    pos = lo;
    return uint32_t(v & ((1ull << k) - 1));
  }
  __device__ __forceinline__ uint32_t peek(uint32_t k) {
    const int32_t p0 = pos;
    const uint32_t v = read(k);
    pos = p0;
    return v;
  }
};

// ---- literals: a lane per Huffman stream ---------------------------------------
__global__ void __launch_bounds__(256) zstd_lit_kernel(const pbl_phys_batch B, uint8_t* out, const uint64_t* out_off,
                                                       void* ws) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t b = t >> 2, s = t & 3;
  if (b >= B.n_blocks) return;
  const FastWs W = FastWs::at(ws, B.n_blocks);
  const gptr<const FDesc> g = to_glb(static_cast<const FDesc*>(W.desc + b));
  if (!g->fast || g->ltype != 2 || s >= g->streams) return;
  const uint32_t D = g->D, regen = g->regen, lg = g->huf_log, cnt = g->cnt[s];
  const uint32_t seg = g->streams == 4 ? (regen + 3) / 4 : 0u;
  const gptr<const uint8_t> src = to_glb(B.bytes + to_glb(B.block_off)[b]);
  const gptr<uint8_t> o = to_glb(out + to_glb(out_off)[b] + (D - regen) + s * seg);
  const gptr<const uint16_t> H = to_glb(static_cast<const uint16_t*>(W.huf(b)));
  GBitsW br;
  bool bad = !br.init(src + g->s_off[s], g->s_len[s]);
  if (!bad) {
    // bytes until o is 4-B aligned, then whole words, then the tail
    const uint32_t head = min(cnt, uint32_t((4 - (reinterpret_cast<uint64_t>(o) & 3)) & 3));
    uint32_t i = 0;
    for (; i < head; i++) {
      const uint32_t e = H[br.peek(lg)];
      o[i] = uint8_t(e);
      br.pos -= int32_t(e >> 8);
    }
    for (; i + 4 <= cnt; i += 4) {
      uint32_t wv = 0;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t e = H[br.peek(lg)];
        wv |= (e & 0xffu) << (8 * k);
        br.pos -= int32_t(e >> 8);
      }
      *(gptr<uint32_t>)(o + i) = wv;
    }
    for (; i < cnt; i++) {
      const uint32_t e = H[br.peek(lg)];
      o[i] = uint8_t(e);
      br.pos -= int32_t(e >> 8);
    }
    bad = br.pos != 0;
  }
  if (bad) g_atomic_or(&W.desc[b].flags, 1u << s);
}

// ---- sequences: a lane per block ------------------------------------------------
// Packed sequence word: literal length (21 bits) | match length (21) | offset
// (22), each saturated (a saturated value exceeds every window: corrupt).
__device__ __forceinline__ uint64_t seq_pack(uint32_t ll, uint32_t ml, uint32_t off) {
  return uint64_t(min(ll, 0x1FFFFFu)) | uint64_t(min(ml, 0x1FFFFFu)) << 21 | uint64_t(min(off, 0x3FFFFFu)) << 42;
}

// A sequence-table entry's symbol and next-state fields.
struct SeqSym {
  uint32_t sym, nb, base;
};
__device__ __forceinline__ SeqSym seq_sym(uint32_t e, uint32_t al) {
  const uint32_t x = e & 0x3ff;
  SeqSym r;
  r.sym = e >> 10;
  r.nb = al - uint32_t(highbit(x));
  r.base = (x << r.nb) - (1u << al);
  return r;
}

// One block's sequences (a lane's chain).
__device__ __forceinline__ void seq_block(const pbl_phys_batch& B, const FastWs& W, uint32_t b,
                                          lptr<const uint32_t> XL, lptr<const uint32_t> XM) {
  const gptr<const FDesc> g = to_glb(static_cast<const FDesc*>(W.desc + b));
  if (!g->fast) return;
  const uint32_t nseq = g->nseq;
  if (nseq == 0) return;
  const uint32_t al = g->al, all = al & 0xff, alo = (al >> 8) & 0xff, alm = (al >> 16) & 0xff;
  const gptr<const uint8_t> src = to_glb(B.bytes + to_glb(B.block_off)[b]);
  const gptr<const uint16_t> TL = to_glb(static_cast<const uint16_t*>(W.ll(b)));
  const gptr<const uint16_t> TO = to_glb(static_cast<const uint16_t*>(W.of(b)));
  const gptr<const uint16_t> TM = to_glb(static_cast<const uint16_t*>(W.ml(b)));
  const gptr<uint64_t> S = to_glb(W.seq + g->seq_base);
  GBitsW br;
  bool bad = !br.init(src + g->q_off, g->q_len);
  if (!bad) {
    uint32_t stl = br.read(all), sto = br.read(alo), stm = br.read(alm);
    uint32_t rep0 = 1, rep1 = 4, rep2 = 8;
    for (uint32_t i = 0; i < nseq; i++) {
      const SeqSym el = seq_sym(TL[stl], all), eo = seq_sym(TO[sto], alo), em = seq_sym(TM[stm], alm);
      const uint32_t xlv = el.sym < 16 ? el.sym : XL[el.sym], xmv = em.sym < 32 ? em.sym + 3 : XM[em.sym];
      const uint32_t ofv = (1u << eo.sym) + br.read(eo.sym);
      const uint32_t ml = (xmv & 0xffffff) + br.read(xmv >> 24);
      const uint32_t ll = (xlv & 0xffffff) + br.read(xlv >> 24);
      if (i + 1 < nseq) {
        stl = el.base + br.read(el.nb);
        stm = em.base + br.read(em.nb);
        sto = eo.base + br.read(eo.nb);
      }
      uint32_t off;
      if (ofv > 3) {
        off = ofv - 3;
        rep2 = rep1;
        rep1 = rep0;
        rep0 = off;
      } else {
        const uint32_t k = ofv - 1 + (ll == 0);
        if (k == 0) {
          off = rep0;
        } else {
          off = k == 3 ? rep0 - 1u : (k == 1 ? rep1 : rep2);
          if (k != 1) rep2 = rep1;
          rep1 = rep0;
          rep0 = off;
        }
      }
      S[i] = seq_pack(ll, ml, off);
    }
    bad = br.pos != 0;
  }
  if (bad) g_atomic_or(&W.desc[b].flags, 16u);
}

// A lane per block, every block's chain live at once: capping the live lanes
// so the tables stay in L2 (12 K / 24 K / 48 K lanes) measured 71.8 / 37.2 /
// 26.1 ms against 15.7 per 64 Ki text blocks: the chains are latency-bound.
__global__ void __launch_bounds__(256) zstd_seq_kernel(const pbl_phys_batch B, void* ws) {
  // baselines and extra bits of the literal-length codes past 15 and the
  // match-length codes past 31 (below them: the code itself, and code + 3)
  __shared__ uint32_t xl[36], xm[53];
  if (threadIdx.x < 36) xl[threadIdx.x] = kLLBase[threadIdx.x] | uint32_t(kLLBits[threadIdx.x]) << 24;
  if (threadIdx.x < 53) xm[threadIdx.x] = kMLBase[threadIdx.x] | uint32_t(kMLBits[threadIdx.x]) << 24;
  __syncthreads();
  const FastWs W = FastWs::at(ws, B.n_blocks);
  const lptr<const uint32_t> XL = to_lds_ptr(static_cast<const uint32_t*>(xl));
  const lptr<const uint32_t> XM = to_lds_ptr(static_cast<const uint32_t*>(xm));
  for (uint32_t b = blockIdx.x * blockDim.x + threadIdx.x; b < B.n_blocks; b += gridDim.x * blockDim.x)
    seq_block(B, W, b, XL, XM);
}

// ---- execution: a wave per block ---------------------------------------------
struct ExecLds {
  alignas(16) uint8_t win[kFastWin + 64];
};

// 16 bytes at o[i] of a global region readable up to `lim` (i < lim): one
// unaligned load when it fits, else byte loads.
__device__ __forceinline__ u32x4 ld16_lim(gptr<const uint8_t> o, uint32_t i, uint32_t lim) {
  if (i + 16 <= lim) return *(gptr<const u32x4 __attribute__((aligned(1)))>)(o + i);
  uint32_t w[4] = {0, 0, 0, 0};
  for (uint32_t k = 0; k < 16 && i + k < lim; k++) w[k >> 2] |= uint32_t(o[i + k]) << (8 * (k & 3));
  return u32x4{w[0], w[1], w[2], w[3]};
}

__device__ __forceinline__ void lds_put(lptr<uint8_t> wv, uint32_t at, const u32x4& v, uint32_t n) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (uint32_t k = 0; k < 16; k++)
    if (k < n) wv[at + k] = uint8_t(w[k >> 2] >> (8 * (k & 3)));
}

// Exclusive wave scan by DPP row shifts and row broadcasts (no LDS round trip).
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t* total) {
  uint32_t x = v;
  x += __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false);  // row_bcast:15
  x += __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xc, 0xf, false);  // row_bcast:31
  *total = __builtin_amdgcn_readlane(x, kWave - 1);
  return x - v;
}

// One batch of up to 64 sequences (lane = sequence): lengths, offset, literal
// source / literal destination / match destination from two wave scans (lp,
// pos: literals consumed and bytes written before the batch), the batch's
// totals, whether the lane's sequence is out of bounds, and the first 16
// literal bytes (the load issued here, consumed a batch later).
struct XBatch {
  uint32_t ll, ml, off, lsrc, ldst, mdst, tll, tout;
  bool bad;
  u32x4 lit;
};
__device__ __forceinline__ void x_plan(XBatch& X, uint64_t sw, bool live, uint32_t lp, uint32_t pos,
                                       gptr<const uint8_t> lits, uint32_t regen, uint32_t D) {
  X.ll = uint32_t(sw & 0x1FFFFF);
  X.ml = uint32_t((sw >> 21) & 0x1FFFFF);
  X.off = uint32_t(sw >> 42);
  const uint32_t lpx = wave_excl_scan(X.ll, &X.tll);
  const uint32_t opx = wave_excl_scan(X.ll + X.ml, &X.tout);
  X.lsrc = lp + lpx;
  X.ldst = pos + opx;
  X.mdst = X.ldst + X.ll;
  X.bad = live && (X.lsrc + X.ll > regen || X.mdst + X.ml > D || X.off == 0 || X.off > X.mdst);
  X.lit = (X.ll && !X.bad && X.lsrc < regen) ? ld16_lim(lits, X.lsrc, regen) : u32x4{0, 0, 0, 0};
}

__global__ void __launch_bounds__(kWave) zstd_exec_kernel(const pbl_phys_batch B, uint8_t* out, const uint64_t* out_off,
                                                          uint32_t* out_len, uint32_t* status, void* ws) {
  __shared__ ExecLds X;
  const uint32_t lane = lane_id();
  const FastWs W = FastWs::at(ws, B.n_blocks);
  const lptr<uint8_t> win = to_lds_ptr(static_cast<uint8_t*>(X.win));
  for (uint32_t b = blockIdx.x; b < B.n_blocks; b += gridDim.x) {
    const gptr<const FDesc> g = to_glb(static_cast<const FDesc*>(W.desc + b));
    if (!g->fast) continue;
    const uint32_t D = g->D, regen = g->regen, nseq = g->nseq, lit0 = D - regen;
    uint8_t* dptr = out + to_glb(out_off)[b];
    const gptr<const uint8_t> lits = to_glb(static_cast<const uint8_t*>(dptr)) + lit0;
    const gptr<const uint64_t> S = to_glb(static_cast<const uint64_t*>(W.seq + g->seq_base));
    bool ok = g->flags == 0;
    uint32_t pos = 0, lp = 0;
    // Batch k + 1 is planned (scans, checks, its first literal chunk's load)
    // before batch k's matches run, and its sequence words are loaded a batch
    // earlier still: the loads run under the previous batch's LDS work.
    uint64_t sw_n = kWave + lane < nseq ? S[kWave + lane] : 0ull;
    XBatch X;
    if (nseq) x_plan(X, lane < nseq ? S[lane] : 0ull, lane < nseq, 0, 0, lits, regen, D);
    for (uint32_t r0 = 0; ok && r0 < nseq; r0 += kWave) {
      const uint32_t i = r0 + lane;
      const XBatch C = X;
      if (__ballot(C.bad) || lp + C.tll > regen || pos + C.tout > D) { ok = false; break; }
      // literal runs, lane per sequence (the literal region is never written here)
      if (C.ll) lds_put(win, C.ldst, C.lit, min(16u, C.ll));
      for (uint32_t c = 16; c < C.ll; c += 16) lds_put(win, C.ldst + c, ld16_lim(lits, C.lsrc + c, regen), min(16u, C.ll - c));
      wave_sync();
      lp += C.tll;
      pos += C.tout;
      if (r0 + kWave < nseq) {
        const uint64_t sw = sw_n;
        sw_n = i + 2 * kWave < nseq ? S[i + 2 * kWave] : 0ull;
        x_plan(X, sw, i + kWave < nseq, lp, pos, lits, regen, D);
      }
      const uint32_t ml = C.ml, off = C.off, mdst = C.mdst;
      // matches: groups whose sources lie below the group's first output
      uint64_t pend = __ballot(i < nseq && ml > 0);
      while (pend) {
        const int gl = __builtin_ctzll(pend);
        const uint32_t gstart = __builtin_amdgcn_readlane(mdst, gl), gml = __builtin_amdgcn_readlane(ml, gl),
                       goff = __builtin_amdgcn_readlane(off, gl);
        if (gml > kWave) {
          // a long match: the whole wave, 64-byte rounds (period goff when it overlaps)
          for (uint32_t j0 = 0; j0 < gml; j0 += kWave) {
            const uint32_t j = j0 + lane;
            if (goff >= kWave) {
              const uint32_t v = j < gml ? uint32_t(win[gstart - goff + j]) : 0u;
              if (j < gml) win[gstart + j] = uint8_t(v);
            } else if (j < gml) {
              win[gstart + j] = win[gstart - goff + (j % goff)];
            }
            wave_sync();
          }
          pend &= pend - 1;
          continue;
        }
        const bool mine = ((pend >> lane) & 1) && ml <= kWave && (int(lane) == gl || mdst - off + ml <= gstart);
        if (mine) {
          // chunks of min(off, 16) bytes: a chunk's reads never see its own writes,
          // so its byte reads are independent (one LDS latency per chunk)
          const uint32_t ck = off < 16 ? off : 16u;
          for (uint32_t j = 0; j < ml; j += ck) {
            uint8_t t[16];
#pragma unroll
            for (uint32_t k = 0; k < 16; k++)
              if (k < ck && j + k < ml) t[k] = win[mdst - off + j + k];
#pragma unroll
            for (uint32_t k = 0; k < 16; k++)
              if (k < ck && j + k < ml) win[mdst + j + k] = t[k];
          }
        }
        wave_sync();
        pend &= ~__ballot(mine);
      }
    }
    if (ok) {
      const uint32_t rest = regen - lp;
      ok = pos + rest == D;
      if (ok) {
        for (uint32_t c = 16 * lane; c < rest; c += 16 * kWave)
          lds_put(win, pos + c, ld16_lim(lits, lp + c, regen), min(16u, rest - c));
        wave_sync();
      }
    }
    if (ok && g->cksum) {
      uint32_t h = 0;
      if (lane == 0) h = xxh64_lo(LOut{win}, 0, D);
      ok = __shfl(h, 0, kWave) == g->ck;
    }
    if (ok) {
      // every literal read has returned (its bytes are in the window): overwrite
      const uint64_t da = reinterpret_cast<uint64_t>(dptr);
      const uint32_t dsh = uint32_t(da & 15);
      const uint32_t nd = (dsh + D + 15) / 16;
      const gptr<u32x4> dg = to_glb(reinterpret_cast<u32x4*>(da - dsh));
      for (uint32_t gi = lane; gi < nd; gi += kWave) {
        const uint32_t lo = gi == 0 ? dsh : 0u, hi = gi + 1 == nd ? dsh + D - 16 * gi : 16u;
        uint32_t w[4] = {0, 0, 0, 0};
        for (uint32_t k = lo; k < hi; k++) w[k >> 2] |= uint32_t(win[16 * gi + k - dsh]) << (8 * (k & 3));
        if (lo == 0 && hi == 16) {
          dg[gi] = u32x4{w[0], w[1], w[2], w[3]};
        } else {
          gptr<uint8_t> db = reinterpret_cast<gptr<uint8_t>>(dg + gi);
          for (uint32_t k = lo; k < hi; k++) db[k] = uint8_t(w[k >> 2] >> (8 * (k & 3)));
        }
      }
    }
    if (lane == 0) {
      to_glb(out_len)[b] = ok ? D : 0u;
      to_glb(status)[b] = ok ? uint32_t(PBL_OK) : uint32_t(PBL_CORRUPT_COMPRESSION);
    }
    wave_sync();
  }
}

}  // namespace zstd
}  // namespace pbl
