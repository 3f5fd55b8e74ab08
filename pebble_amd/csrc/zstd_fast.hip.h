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
constexpr uint32_t kTblBytes = 14336; // per-block table slot: Huffman 2048 x u16, LL 512 / OF 256 / ML 512 x u64
constexpr uint32_t kSeqPerBlock = 3072;  // sequence words of workspace per block (shared by a bump counter)

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
    W.seq_cap = n * kSeqPerBlock;
    return W;
  }
  __device__ uint16_t* huf(uint32_t b) const { return reinterpret_cast<uint16_t*>(tbl + uint64_t(b) * kTblBytes); }
  __device__ uint64_t* ll(uint32_t b) const { return reinterpret_cast<uint64_t*>(tbl + uint64_t(b) * kTblBytes + 4096); }
  __device__ uint64_t* of(uint32_t b) const { return ll(b) + 512; }
  __device__ uint64_t* ml(uint32_t b) const { return ll(b) + 768; }
};

// Sequence-table entry (u64): next-state base (16) | state bits (8) | extra
// bits (8) | baseline value (32).
__device__ __forceinline__ uint64_t seq_entry(uint32_t e, uint32_t extra, uint32_t value) {
  return uint64_t(e >> 16) | uint64_t((e >> 8) & 0xff) << 16 | uint64_t(extra) << 24 | uint64_t(value) << 32;
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
        int32_t u = 0;
        if (fast && lane == 0) {
          bool hl = false, ho = false, hm = false;
          const uint32_t lim = e1 > q ? e1 - q : 0u;
          u = seq_table(to_lds_ptr(L.fse[0]), L, modes >> 6, kLLDef, 36, 6, 9, 35, w1, q, lim, &al_ll, &hl);
          const int32_t u2 = u < 0 ? -1
                                   : seq_table(to_lds_ptr(L.fse[1]), L, (modes >> 4) & 3, kOFDef, 29, 5, 8, 31, w1, q + u,
                                               lim - u, &al_of, &ho);
          const int32_t u3 = u2 < 0 ? -1
                                    : seq_table(to_lds_ptr(L.fse[2]), L, (modes >> 2) & 3, kMLDef, 53, 6, 9, 52, w1,
                                                q + u + u2, lim - u - u2, &al_ml, &hm);
          u = u3 < 0 ? -1 : u + u2 + u3;
        }
        u = __shfl(u, 0, kWave);
        al_ll = __shfl(al_ll, 0, kWave);
        al_of = __shfl(al_of, 0, kWave);
        al_ml = __shfl(al_ml, 0, kWave);
        wave_sync();
        fast = fast && u >= 0 && q + uint32_t(u) < end;
        if (fast) {
          q += uint32_t(u);
          // the tables, baselines folded in (RFC 8878 §3.1.1.3.2.1.1)
          for (uint32_t i = lane; i < (1u << al_ll); i += kWave) {
            const uint32_t e = L.fse[0][i], s = e & 0xff;
            to_glb(W.ll(b))[i] = seq_entry(e, kLLBits[s], kLLBase[s]);
          }
          for (uint32_t i = lane; i < (1u << al_of); i += kWave) {
            const uint32_t e = L.fse[1][i], s = e & 0xff;
            to_glb(W.of(b))[i] = seq_entry(e, s, 1u << (s & 31));
          }
          for (uint32_t i = lane; i < (1u << al_ml); i += kWave) {
            const uint32_t e = L.fse[2][i], s = e & 0xff;
            to_glb(W.ml(b))[i] = seq_entry(e, kMLBits[s], kMLBase[s]);
          }
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

// ---- lane-per-stream / lane-per-block bit readers ------------------------------
// Backward bitstream over global bytes [0, n) of p (RFC 8878 §4.1): unread bits
// [0, pos); the container holds bits [cb, cb + 64), refilled by one unaligned
// 8-B load that never ends past byte n (byte loads for streams under 8 bytes).
struct GBits {
  gptr<const uint8_t> p;
  uint32_t n;
  int32_t pos, cb;
  uint64_t c;
  __device__ __forceinline__ void refill() {
    int32_t b = (pos - 57) >> 3;
    if (b < 0) b = 0;
    cb = 8 * b;
    if (uint32_t(b) + 8 <= n) {
      c = *(gptr<const uint64_t __attribute__((aligned(1)))>)(p + b);
    } else {
      c = 0;
      for (uint32_t i = uint32_t(b); i < n; i++) c |= uint64_t(p[i]) << (8 * (i - b));
    }
  }
  __device__ __forceinline__ bool init(gptr<const uint8_t> src, uint32_t len) {
    p = src;
    n = len;
    if (len == 0) return false;
    const uint32_t last = p[len - 1];
    if (last == 0) return false;
    pos = int32_t(8 * len) - 8 + highbit(last);
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
  GBits br;
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

__global__ void __launch_bounds__(256) zstd_seq_kernel(const pbl_phys_batch B, void* ws) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B.n_blocks) return;
  const FastWs W = FastWs::at(ws, B.n_blocks);
  const gptr<const FDesc> g = to_glb(static_cast<const FDesc*>(W.desc + b));
  if (!g->fast) return;
  const uint32_t nseq = g->nseq;
  if (nseq == 0) return;
  const uint32_t al = g->al;
  const gptr<const uint8_t> src = to_glb(B.bytes + to_glb(B.block_off)[b]);
  const gptr<const uint64_t> TL = to_glb(static_cast<const uint64_t*>(W.ll(b)));
  const gptr<const uint64_t> TO = to_glb(static_cast<const uint64_t*>(W.of(b)));
  const gptr<const uint64_t> TM = to_glb(static_cast<const uint64_t*>(W.ml(b)));
  const gptr<uint64_t> S = to_glb(W.seq + g->seq_base);
  GBits br;
  bool bad = !br.init(src + g->q_off, g->q_len);
  if (!bad) {
    uint32_t stl = br.read(al & 0xff), sto = br.read((al >> 8) & 0xff), stm = br.read((al >> 16) & 0xff);
    uint32_t rep0 = 1, rep1 = 4, rep2 = 8;
    for (uint32_t i = 0; i < nseq; i++) {
      const uint64_t el = TL[stl], eo = TO[sto], em = TM[stm];
      const uint32_t ofv = uint32_t(eo >> 32) + br.read(uint32_t(eo >> 24) & 0xff);
      const uint32_t ml = uint32_t(em >> 32) + br.read(uint32_t(em >> 24) & 0xff);
      const uint32_t ll = uint32_t(el >> 32) + br.read(uint32_t(el >> 24) & 0xff);
      if (i + 1 < nseq) {
        stl = uint32_t(el & 0xffff) + br.read(uint32_t(el >> 16) & 0xff);
        stm = uint32_t(em & 0xffff) + br.read(uint32_t(em >> 16) & 0xff);
        sto = uint32_t(eo & 0xffff) + br.read(uint32_t(eo >> 16) & 0xff);
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

__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t* total) {
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, kWave);
    if (lane_id() >= d) x += y;
  }
  *total = __shfl(x, kWave - 1, kWave);
  return x - v;
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
    for (uint32_t r0 = 0; ok && r0 < nseq; r0 += kWave) {
      const uint32_t i = r0 + lane;
      const uint64_t sw = i < nseq ? S[i] : 0ull;
      const uint32_t ll = uint32_t(sw & 0x1FFFFF), ml = uint32_t((sw >> 21) & 0x1FFFFF), off = uint32_t(sw >> 42);
      uint32_t tll, tout;
      const uint32_t lpx = wave_excl_scan(ll, &tll);
      const uint32_t opx = wave_excl_scan(ll + ml, &tout);
      const uint32_t lsrc = lp + lpx, ldst = pos + opx, mdst = ldst + ll;
      const bool bad = i < nseq && (lsrc + ll > regen || mdst + ml > D || off == 0 || off > mdst);
      if (__ballot(bad) || lp + tll > regen || pos + tout > D) { ok = false; break; }
      // literal runs, lane per sequence (the literal region is never written here)
      for (uint32_t c = 0; c < ll; c += 16) {
        const uint32_t k = min(16u, ll - c);
        lds_put(win, ldst + c, ld16_lim(lits, lsrc + c, regen), k);
      }
      wave_sync();
      // matches: groups whose sources lie below the group's first output
      uint64_t pend = __ballot(i < nseq && ml > 0);
      while (pend) {
        const int gl = __builtin_ctzll(pend);
        const uint32_t gstart = __shfl(mdst, gl, kWave), gml = __shfl(ml, gl, kWave), goff = __shfl(off, gl, kWave);
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
        if (mine)
          for (uint32_t j = 0; j < ml; j++) win[mdst + j] = win[mdst - off + j];
        wave_sync();
        pend &= ~__ballot(mine);
      }
      pos += tout;
      lp += tll;
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
