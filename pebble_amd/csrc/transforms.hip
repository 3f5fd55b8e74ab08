// transforms.hip — blockiter.Transforms on the device.
//
// Pebble applies its iteration-time transforms inside the block iterators
// (sstable/blockiter/transforms.go:20-56,170-248): SyntheticSeqNum rewrites
// every trailer's sequence number (rowblk_iter.go:487-503; data_block.go
// 1680-1697), HideObsoletePoints skips obsolete points (rowblk_iter.go
// 1168-1179; data_block.go:1299-1303,1479-1543), SyntheticPrefix is prepended
// to every user key (rowblk_iter.go:400; data_block.go:1311-1312) and
// SyntheticSuffix replaces the suffix that the comparer's Split finds
// (rowblk_iter.go:505-517,1181-1187; data_block.go:444-460).
//
// Here they are a second, HBM-bound pass over a decoded batch (the
// no-transform decode, the baseline, is untouched): `in` is the output of
// pbl_decode_batch, `out` receives the transformed batch in the same layout
// contract (include/pebble_amd.h).  Three stream-ordered launches:
//   tf_count_kernel    one wave per block: visible KVs and their new key and
//                      value bytes
//   tf_scan_kernel     one workgroup: exclusive scan of the per-block counts ->
//                      out.blk_*_base, totals, capacity check
//   tf_scatter_kernel  one wave per block: compacted per-KV arrays, keys
//                      (prefix ++ key[:Split] ++ suffix), values, restarts
#include <algorithm>

#include "common.hip.h"

namespace pbl {
namespace tf {

// Workspace: [0, 64) header (u32 overflow flag, u32 tile ticket), then the
// tile look-back state (tf_scan_kernel, 80 B per tile), then 4 u32 counts per
// block (tf_count_kernel).  The header and the look-back state are zeroed per launch.
constexpr int kTfWs = 64;
constexpr uint32_t kTfTile = 1024;  // blocks per scan tile (256 threads x 4)
__host__ __device__ inline uint64_t tf_tiles(uint32_t nb) { return (uint64_t(nb) + kTfTile - 1) / kTfTile; }
__host__ __device__ inline uint64_t tf_lb_bytes(uint32_t nb) { return 80ull * tf_tiles(nb); }
__host__ __device__ inline uint64_t tf_cnt_offset(uint32_t nb) { return kTfWs + tf_lb_bytes(nb); }
constexpr uint64_t kTfMask = ((1ull << 56) - 1) << 8 | 191u;  // TrailerObsoleteMask (rowblk_writer.go:30-42)
constexpr uint64_t kTfInvalid = 191u;                          // InternalKeyKindInvalid

struct TfArgs {
  pbl_decode_out in, out;
  pbl_transforms t;
  pbl_block_batch src;  // the batch `in` was decoded from (row blocks: raw short keys)
  uint32_t n_blocks;
};

// Comparer.Split over F = pfx[0:fp] ++ key[0:kn] (transforms.go:105-118 needs it
// for the suffix; a row key's Split sees the synthetic prefix too,
// rowblk_iter.go:400,1183).
struct FKey {
  gptr<const uint8_t> pfx, key;
  uint32_t fp, kn;
  __device__ uint8_t at(uint32_t i) const { return i < fp ? pfx[i] : key[i - fp]; }
  __device__ uint32_t len() const { return fp + kn; }
};
__device__ inline uint32_t split_len(const FKey& k, uint32_t split) {
  const uint32_t n = k.len();
  if (split == PBL_SPLIT_TESTKEYS) {  // testkeys.Comparer: before the last '@' (internal/testkeys/testkeys.go:144-150)
    for (uint32_t i = n; i > 0; i--)
      if (k.at(i - 1) == '@') return i - 1;
    return n;
  }
  if (split == PBL_SPLIT_CRDB) {  // cockroachkvs.Split: the last byte is the version length (+1), 0 if none
    if (n == 0) return 0;
    const uint32_t v = k.at(n - 1);
    return v <= n ? n - v : 0;
  }
  return n;  // base.DefaultSplit: the whole key
}

// uint32 varint of rowblk_iter.go:2020-2038 (5th byte << 28); returns bytes read
__device__ inline uint32_t tf_varint(gptr<const uint8_t> p, uint32_t* v) {
  uint32_t r = 0;
  for (uint32_t i = 0; i < 5; i++) {
    const uint32_t b = p[i];
    if (i == 4) { *v = r | (b << 28); return 5; }
    r |= (b & 0x7fu) << (7 * i);
    if (b < 128) { *v = r; return i + 1; }
  }
  return 5;
}

// The raw internal key (< 8 bytes, byte i at bits 8i) of row entry j, an entry
// the decode left PBL_KV_INVALID_KEY: its bytes past `shared` from the block,
// the shared ones from the previous entry -- an invalid one again (its header
// re-read), or a decoded one, whose raw key is user key ++ LE64(trailer | the
// obsolete bit).  Entries are in block order and a block's first entry has
// shared 0, so the walk ends inside the block.
__device__ inline uint64_t raw_short_key(const TfArgs& A, gptr<const uint8_t> blk, uint64_t kv0, uint64_t kb_in,
                                         uint32_t b, uint32_t j, uint32_t* kl_out) {
  const pbl_decode_out& I = A.in;
  uint32_t s, u, vl;
  uint32_t e = to_glb(I.entry_off)[kv0 + j];
  uint32_t h = tf_varint(blk + e, &s);
  h += tf_varint(blk + e + h, &u);
  h += tf_varint(blk + e + h, &vl);
  const uint32_t kl = s + u;
  *kl_out = kl;
  uint64_t raw = 0;
  uint32_t need = kl, k = j, ks = s, kkl = kl;
  for (;;) {
    for (uint32_t i = ks; i < need && i < kkl; i++) raw |= uint64_t(blk[e + h + (i - ks)]) << (8 * i);
    need = need < ks ? need : ks;
    if (need == 0 || k == 0) break;
    k--;
    const uint8_t fk = to_glb(I.kv_flags)[kv0 + k];
    if (!(fk & PBL_KV_INVALID_KEY)) {
      const uint64_t o = kv0 + b + k;
      const uint32_t ko = to_glb(I.key_off)[o], ukl = to_glb(I.key_off)[o + 1] - ko;
      const uint64_t tk = to_glb(I.trailer)[kv0 + k] | ((fk & PBL_KV_OBSOLETE) ? 64u : 0u);
      for (uint32_t i = 0; i < need; i++) {
        const uint64_t x = i < ukl ? uint64_t(to_glb(I.key_bytes)[kb_in + ko + i]) : (tk >> (8 * (i - ukl))) & 0xffu;
        raw |= x << (8 * i);
      }
      break;
    }
    e = to_glb(I.entry_off)[kv0 + k];
    h = tf_varint(blk + e, &ks);
    h += tf_varint(blk + e + h, &u);
    h += tf_varint(blk + e + h, &vl);
    kkl = ks + u;
  }
  return raw;
}

struct KvView {
  bool vis, valid, corrupt;
  uint8_t fl;
  uint64_t tr;
  FKey F;        // the user key before the suffix step
  uint32_t p;    // Split point in F (= F.len() without a suffix)
  uint32_t vo, vlen, nk;
};

__device__ inline uint32_t block_format(const TfArgs& A, uint32_t b) {
  return A.src.block_format ? to_glb(A.src.block_format)[b] : A.src.format;
}

__device__ inline KvView kv_view(const TfArgs& A, uint32_t b, uint64_t kv0, uint64_t kb_in, uint64_t vb_in,
                                 uint32_t j) {
  const pbl_decode_out& I = A.in;
  const pbl_transforms& T = A.t;
  KvView v;
  const bool row = block_format(A, b) == PBL_FMT_ROW && !(A.src.flags & PBL_ROW_RAW_KEYS);
  v.fl = I.kv_flags ? to_glb(I.kv_flags)[kv0 + j] : uint8_t(0);
  v.tr = to_glb(I.trailer)[kv0 + j];
  v.corrupt = false;
  v.vis = !(T.hide_obsolete_points && (v.fl & PBL_KV_OBSOLETE));
  v.valid = !(v.fl & PBL_KV_INVALID_KEY);
  const uint64_t o = kv0 + b + j;
  const uint32_t ko = to_glb(I.key_off)[o];
  v.vo = to_glb(I.val_off)[o];
  v.vlen = to_glb(I.val_off)[o + 1] - v.vo;
  v.F = FKey{to_glb(T.prefix), to_glb(I.key_bytes) + kb_in + ko, T.prefix_len, to_glb(I.key_off)[o + 1] - ko};
  if (row && !v.valid && T.prefix_len) {
    // rowblk_iter.go:400,1168-1199: the prefix is part of the key the trailer
    // is decoded from, so a raw key shorter than 8 B can become a valid one
    const gptr<const uint8_t> blk = to_glb(A.src.blocks) + to_glb(A.src.block_off)[b];
    uint32_t kl;
    const uint64_t rk = raw_short_key(A, blk, kv0, kb_in, b, j, &kl);
    if (T.prefix_len + kl >= 8) {
      const uint32_t ukl = T.prefix_len + kl - 8;  // the user key lies inside the prefix
      uint64_t raw = rk << (8 * (8 - kl));
      for (uint32_t i = 0; i < 8 - kl; i++) raw |= uint64_t(to_glb(T.prefix)[ukl + i]) << (8 * i);
      v.valid = true;
      v.fl = uint8_t((v.fl & ~PBL_KV_INVALID_KEY) | ((raw & 64u) ? PBL_KV_OBSOLETE : 0u));
      v.vis = !(T.hide_obsolete_points && (raw & 64u));
      v.tr = raw & kTfMask;
      v.F.fp = ukl;
      v.F.kn = 0;
      if ((A.src.flags & PBL_ROW_VALUE_PREFIX) && (v.tr & 0xffu) == 1u) {  // kind SET: the value prefix
        if (v.vlen == 0) {
          v.corrupt = v.vis;  // Go: i.val[0] panics (only reached for a visible point)
        } else {
          const uint32_t pre = to_glb(I.val_bytes)[vb_in + v.vo];
          if ((pre & 0xC0u) == 0 || (A.src.flags & PBL_ROW_NO_VALUER)) { v.vo++; v.vlen--; }
          else v.fl |= (pre & 0xC0u) == 0x80u ? PBL_KV_VALBLK_HANDLE : PBL_KV_BLOB_HANDLE;
        }
      }
    }
  }
  if (!v.valid) {
    v.nk = 0;
    v.p = 0;
    return v;  // trailer stays InternalKeyKindInvalid (no SetSeqNum: rowblk_iter.go:1189-1191)
  }
  if (T.synthetic_seq_num) v.tr = (T.synthetic_seq_num << 8) | (v.tr & 0xffu);  // InternalKey.SetSeqNum
  const uint32_t flen = v.F.len();
  if (T.suffix_len) {
    if (row) {
      v.p = split_len(v.F, T.split);  // Split(prefix ++ key)
    } else {
      // colblk: the KeySeeker keeps the schema's prefix (data_block.go:444-460,
      // cockroachkvs.go:1073-1089) = Split of the stored key, after the prefix
      const FKey K{v.F.pfx, v.F.key, 0, v.F.kn};
      v.p = T.prefix_len + split_len(K, T.split);
    }
    v.nk = v.p + T.suffix_len;
  } else {
    v.p = flen;
    v.nk = flen;
  }
  return v;
}

__global__ void __launch_bounds__(kTPB) tf_count_kernel(TfArgs A) {
  uint32_t* cnt = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(A.out.workspace) + tf_cnt_offset(A.n_blocks));
  const uint32_t lane = lane_id();
  const uint32_t wpb = kTPB / kWave;
  for (uint32_t b = blockIdx.x * wpb + wave_id(); b < A.n_blocks; b += gridDim.x * wpb) {
    uint32_t c = 0, kb = 0, vb = 0;
    bool bad = false;
    if (to_glb(A.in.blk_status)[b] == PBL_OK) {
      const uint64_t kv0 = to_glb(A.in.blk_kv_base)[b], n = to_glb(A.in.blk_kv_base)[b + 1] - kv0;
      const uint64_t kb_in = to_glb(A.in.blk_key_base)[b], vb_in = to_glb(A.in.blk_val_base)[b];
      for (uint32_t j = lane; j < n; j += kWave) {
        const KvView v = kv_view(A, b, kv0, kb_in, vb_in, j);
        bad = bad || v.corrupt;
        if (v.vis) {
          c++;
          kb += v.nk;
          vb += v.vlen;
        }
      }
      c = wave_sum(c);
      kb = wave_sum(kb);
      vb = wave_sum(vb);
      bad = __ballot(bad) != 0;
    }
    if (lane == 0) {
      cnt[4 * uint64_t(b)] = bad ? 0u : c;
      cnt[4 * uint64_t(b) + 1] = bad ? 0u : kb;
      cnt[4 * uint64_t(b) + 2] = bad ? 0u : vb;
      cnt[4 * uint64_t(b) + 3] = bad ? 1u : 0u;
    }
  }
}

// Tiles of kTfTile blocks, one workgroup each, in ticket order: the tile's
// counts are loaded (4 blocks per thread), scanned in the workgroup, the tile's
// aggregate {KVs, key bytes, value bytes, newly corrupt blocks} published and
// its exclusive prefix resolved by decoupled look-back; then every block's
// bases and status.  The last tile writes the batch totals and the overflow
// flag (the scatter turns OK blocks into PBL_OVERFLOW when it is set).
__global__ void __launch_bounds__(kTPB) tf_scan_kernel(TfArgs A) {
  __shared__ uint32_t s_tile;
  __shared__ uint64_t s_wsum[kTPB / kWave][4];
  __shared__ uint64_t s_excl[4];
  uint8_t* ws = reinterpret_cast<uint8_t*>(A.out.workspace);
  uint32_t* hdr = reinterpret_cast<uint32_t*>(ws);
  uint64_t* lb_state = reinterpret_cast<uint64_t*>(ws + kTfWs);
  const uint4* cnt4 = reinterpret_cast<const uint4*>(ws + tf_cnt_offset(A.n_blocks));
  const uint32_t nb = A.n_blocks, nt = uint32_t(tf_tiles(nb)), t = threadIdx.x;
  const pbl_decode_out& I = A.in;
  const pbl_decode_out& O = A.out;
  for (;;) {
    if (t == 0) s_tile = g_atomic_add(hdr + 1, 1u);
    __syncthreads();
    const uint32_t tile = s_tile;
    __syncthreads();  // (s_tile is rewritten next iteration)
    if (tile >= nt) return;
    const uint32_t b0 = tile * kTfTile + 4 * t;
    uint4 c[4];
    uint64_t s4[4] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 4; k++) {
      c[k] = make_uint4(0, 0, 0, 0);
      if (b0 + k < nb) c[k] = cnt4[b0 + k];
      s4[0] += c[k].x;
      s4[1] += c[k].y;
      s4[2] += c[k].z;
      s4[3] += c[k].w;
    }
    // workgroup exclusive scan of the per-thread sums
    uint64_t in4[4];
#pragma unroll
    for (int q = 0; q < 4; q++) in4[q] = wave_incl_scan(s4[q]);
    if (lane_id() == kWave - 1)
      for (int q = 0; q < 4; q++) s_wsum[wave_id()][q] = in4[q];
    __syncthreads();
    uint64_t before[4] = {0, 0, 0, 0}, agg[4] = {0, 0, 0, 0};
    for (int w = 0; w < kTPB / kWave; w++)
#pragma unroll
      for (int q = 0; q < 4; q++) {
        if (w < wave_id()) before[q] += s_wsum[w][q];
        agg[q] += s_wsum[w][q];
      }
    if (wave_id() == 0) {
      uint64_t excl[4];
      lb_publish(lb_state, nt, tile, agg);
      lb_resolve(lb_state, nt, tile, agg, excl, &O.totals->status_mask);
      if (lane_id() == 0)
        for (int q = 0; q < 4; q++) s_excl[q] = excl[q];
    }
    __syncthreads();
    uint64_t e[3];
#pragma unroll
    for (int q = 0; q < 3; q++) e[q] = s_excl[q] + before[q] + in4[q] - s4[q];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t b = b0 + k;
      if (b < nb) {
        to_glb(O.blk_kv_base)[b] = e[0];
        to_glb(O.blk_key_base)[b] = e[1];
        to_glb(O.blk_val_base)[b] = e[2];
        if (O.blk_rst_base) to_glb(O.blk_rst_base)[b] = to_glb(I.blk_rst_base)[b];
        uint32_t st = to_glb(I.blk_status)[b];
        if (st == PBL_OK && c[k].w) st = PBL_CORRUPT_BOUNDS;
        to_glb(O.blk_status)[b] = st;
        e[0] += c[k].x;
        e[1] += c[k].y;
        e[2] += c[k].z;
      }
    }
    if (tile == nt - 1 && t == 0) {
      uint64_t tot[4];
      for (int q = 0; q < 4; q++) tot[q] = s_excl[q] + agg[q];
      const uint64_t nr = to_glb(I.blk_rst_base)[nb];
      to_glb(O.blk_kv_base)[nb] = tot[0];
      to_glb(O.blk_key_base)[nb] = tot[1];
      to_glb(O.blk_val_base)[nb] = tot[2];
      if (O.blk_rst_base) to_glb(O.blk_rst_base)[nb] = nr;
      const bool over = tot[0] > O.kv_cap || tot[1] > O.key_cap || tot[2] > O.val_cap || (O.restarts && nr > O.rst_cap);
      pbl_totals to = *I.totals;  // (one thread: a generic access is fine here)
      to.n_kv = tot[0];
      to.key_bytes = tot[1];
      to.val_bytes = tot[2];
      to.n_restarts = nr;
      if (over) to.status_mask |= 1u << PBL_OVERFLOW;
      if (tot[3]) {  // row blocks whose transformed iteration would panic
        to.status_mask |= 1u << PBL_CORRUPT_BOUNDS;
        to.n_bad_blocks += uint32_t(tot[3]);
      }
      if (over) to.n_bad_blocks = nb;  // (every block is now OVERFLOW or bad)
      to.status_mask |= __hip_atomic_load(&O.totals->status_mask, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *O.totals = to;
      __hip_atomic_store(hdr, over ? 1u : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// dst[0, n) = src[0, n) by 16-B chunks (unaligned global loads / stores; the
// sources are readable 15 bytes past their end), exact at the tail.
typedef u32x4 u32x4_u __attribute__((aligned(1)));
typedef uint64_t u64_u __attribute__((aligned(1)));
typedef uint32_t u32_u __attribute__((aligned(1)));
typedef uint16_t u16_u __attribute__((aligned(1)));
__device__ __forceinline__ void copy_chunks(gptr<uint8_t> dst, gptr<const uint8_t> src, uint32_t n) {
  uint32_t c = 0;
  for (; c + 64 <= n; c += 64) {
    u32x4 x[4];
#pragma unroll
    for (int u = 0; u < 4; u++) x[u] = *(gptr<const u32x4_u>)(src + c + 16 * u);
#pragma unroll
    for (int u = 0; u < 4; u++) *(gptr<u32x4_u>)(dst + c + 16 * u) = x[u];
  }
  for (; c + 16 <= n; c += 16) *(gptr<u32x4_u>)(dst + c) = *(gptr<const u32x4_u>)(src + c);
  if (c < n) {
    const u32x4 w = *(gptr<const u32x4_u>)(src + c);
    const uint32_t r = n - c;
    uint64_t lo = uint64_t(w.x) | uint64_t(w.y) << 32, hi = uint64_t(w.z) | uint64_t(w.w) << 32;
    uint32_t o = c;
    if (r & 8) {
      *(gptr<u64_u>)(dst + o) = lo;
      lo = hi;
      o += 8;
    }
    if (r & 4) {
      *(gptr<u32_u>)(dst + o) = uint32_t(lo);
      lo >>= 32;
      o += 4;
    }
    if (r & 2) {
      *(gptr<u16_u>)(dst + o) = uint16_t(lo);
      lo >>= 16;
      o += 2;
    }
    if (r & 1) dst[o] = uint8_t(lo);
  }
}

#ifndef PBL_TF_SCATTER_WAVES
#define PBL_TF_SCATTER_WAVES 5  // 96 VGPRs, no scratch: 1167 -> 1260 GiB/s on the transform bench (6: 84 B/lane of scratch, 1190)
#endif
__global__ void __launch_bounds__(kTPB) __attribute__((amdgpu_waves_per_eu(PBL_TF_SCATTER_WAVES)))
tf_scatter_kernel(TfArgs A) {
  if (*to_glb(reinterpret_cast<const uint32_t*>(A.out.workspace)) != 0) {  // overflow: sizes and statuses only
    for (uint32_t b = blockIdx.x * kTPB + threadIdx.x; b < A.n_blocks; b += gridDim.x * kTPB)
      if (to_glb(A.out.blk_status)[b] == PBL_OK) to_glb(A.out.blk_status)[b] = PBL_OVERFLOW;
    return;
  }
  const pbl_decode_out& I = A.in;
  const pbl_decode_out& O = A.out;
  const uint32_t lane = lane_id();
  const uint32_t wpb = kTPB / kWave;
  const gptr<const uint8_t> sfx = to_glb(A.t.suffix);
  for (uint32_t b = blockIdx.x * wpb + wave_id(); b < A.n_blocks; b += gridDim.x * wpb) {
    const uint64_t okv = to_glb(O.blk_kv_base)[b], okb = to_glb(O.blk_key_base)[b], ovb = to_glb(O.blk_val_base)[b];
    // restart words are the block's own (entry offsets never move); kept even
    // when the transformed iteration turns the block corrupt
    if (O.restarts && I.restarts) {
      const uint64_t r0 = to_glb(I.blk_rst_base)[b], r1 = to_glb(I.blk_rst_base)[b + 1];
      for (uint64_t r = r0 + lane; r < r1; r += kWave) to_glb(O.restarts)[r] = to_glb(I.restarts)[r];
    }
    if (to_glb(O.blk_status)[b] != PBL_OK) {
      if (lane == 0) {
        to_glb(O.key_off)[okv + b] = 0;
        to_glb(O.val_off)[okv + b] = 0;
      }
      continue;
    }
    const uint64_t kv0 = to_glb(I.blk_kv_base)[b], n = to_glb(I.blk_kv_base)[b + 1] - kv0;
    const uint64_t kb_in = to_glb(I.blk_key_base)[b], vb_in = to_glb(I.blk_val_base)[b];
    uint32_t jo = 0, kcur = 0, vcur = 0;  // output index and offsets (wave-uniform)
    for (uint64_t j0 = 0; j0 < n; j0 += kWave) {
      const uint32_t j = uint32_t(j0) + lane;
      const bool act = j < n;
      KvView v{};
      if (act) v = kv_view(A, b, kv0, kb_in, vb_in, j);
      const bool vis = act && v.vis;
      const uint64_t vm = __ballot(vis);
      const uint32_t rank = __builtin_popcountll(vm & ((1ull << lane) - 1));
      const uint32_t kx = wave_incl_scan(vis ? v.nk : 0u), vx = wave_incl_scan(vis ? v.vlen : 0u);
      const uint32_t ko = kcur + kx - (vis ? v.nk : 0u), vo = vcur + vx - (vis ? v.vlen : 0u);
      if (vis) {
        const uint64_t k = okv + jo + rank;
        to_glb(O.trailer)[k] = v.tr;
        if (O.kv_flags) to_glb(O.kv_flags)[k] = v.fl;
        if (O.entry_off && I.entry_off) to_glb(O.entry_off)[k] = to_glb(I.entry_off)[kv0 + j];
        if (O.tiering_span_id && I.tiering_span_id) {  // KVMeta travels with its KV
          to_glb(O.tiering_span_id)[k] = to_glb(I.tiering_span_id)[kv0 + j];
          to_glb(O.tiering_attr)[k] = to_glb(I.tiering_attr)[kv0 + j];
        }
        to_glb(O.key_off)[okv + b + jo + rank] = ko;
        to_glb(O.val_off)[okv + b + jo + rank] = vo;
        // key: F[:p] ++ (suffix | F[p:]),  F = prefix ++ key
        if (v.valid) {
          // F[:p] ++ (suffix | F[p:]), F = prefix[:fp] ++ key[:kn]: up to four
          // contiguous copies by 16-B chunks
          gptr<uint8_t> dst = to_glb(O.key_bytes) + okb + ko;
          const uint32_t fp = v.F.fp, kn = v.F.kn, p = v.p;
          const uint32_t a1 = p < fp ? p : fp;  // prefix bytes before the split
          copy_chunks(dst, v.F.pfx, a1);
          copy_chunks(dst + a1, v.F.key, p - a1);
          if (A.t.suffix_len) {
            copy_chunks(dst + p, sfx, A.t.suffix_len);
          } else {
            copy_chunks(dst + p, v.F.pfx + a1, fp - a1);
            const uint32_t k0 = p > fp ? p - fp : 0u;
            copy_chunks(dst + p + (fp - a1), v.F.key + k0, kn - k0);
          }
        }
      }
      // values of at most 512 B: 8 lanes per KV (lane c of a group copies the
      // value's 16-B chunks c, c + 8, ...), so one store instruction covers
      // eight contiguous 128-B runs instead of 64 scattered 16-B pieces
      // (lane per KV: 999 GiB/s at 1.92x traffic on the transform bench)
#ifndef PBL_TF_VAL_GROUP
#define PBL_TF_VAL_GROUP 1
#endif
      if (PBL_TF_VAL_GROUP) {
#pragma unroll 1
        for (uint32_t u = 0; u < kWave / 8; u++) {
          const int sl = int(8 * u + (lane >> 3));
          const bool sv = __shfl(int(vis && v.vlen <= 512), sl, kWave) != 0;
          const uint32_t so = uint32_t(__shfl(int(v.vo), sl, kWave)), sn = uint32_t(__shfl(int(v.vlen), sl, kWave));
          const uint32_t dofs = uint32_t(__shfl(int(vo), sl, kWave));
          if (!sv) continue;
          const gptr<const uint8_t> s = to_glb(I.val_bytes) + vb_in + so;
          gptr<uint8_t> d = to_glb(O.val_bytes) + ovb + dofs;
          for (uint32_t i = 16 * (lane & 7u); i < sn; i += 128) copy_chunks(d + i, s + i, sn - i < 16 ? sn - i : 16u);
        }
      } else if (vis && v.vlen <= 512) {
        copy_chunks(to_glb(O.val_bytes) + ovb + vo, to_glb(I.val_bytes) + vb_in + v.vo, v.vlen);
      }
      for (uint64_t m = __ballot(vis && v.vlen > 512); m; m &= m - 1) {
        const int src_lane = __builtin_ctzll(m);
        const uint32_t so = uint32_t(__shfl(int(v.vo), src_lane, kWave));
        const uint32_t sl = uint32_t(__shfl(int(v.vlen), src_lane, kWave));
        const uint32_t dofs = uint32_t(__shfl(int(vo), src_lane, kWave));
        const gptr<const uint8_t> s = to_glb(I.val_bytes) + vb_in + so;
        gptr<uint8_t> d = to_glb(O.val_bytes) + ovb + dofs;
        for (uint32_t i = 16 * lane; i < sl; i += 16 * kWave) copy_chunks(d + i, s + i, sl - i < 16 ? sl - i : 16u);
      }
      jo += __builtin_popcountll(vm);
      kcur += uint32_t(__shfl(int(kx), kWave - 1, kWave));
      vcur += uint32_t(__shfl(int(vx), kWave - 1, kWave));
    }
    if (lane == 0) {
      to_glb(O.key_off)[okv + b + jo] = kcur;
      to_glb(O.val_off)[okv + b + jo] = vcur;
    }
  }
}

}  // namespace tf
}  // namespace pbl

extern "C" {

uint64_t pbl_transform_workspace_bytes(uint32_t n_blocks) {
  return pbl::tf::tf_cnt_offset(n_blocks) + 16ull * n_blocks;
}

int pbl_transform_batch(const pbl_decode_out* in, uint32_t n_blocks, const pbl_transforms* t, pbl_decode_out* out,
                        void* stream) {
  if (!in || !out || !t) return PBL_INVALID_ARG;
  if (!in->totals || !in->blk_kv_base || !in->blk_key_base || !in->blk_val_base || !in->blk_rst_base ||
      !in->blk_status || !in->key_off || !in->val_off || !in->key_bytes || !in->val_bytes || !in->trailer)
    return PBL_INVALID_ARG;
  if (!out->totals || !out->blk_kv_base || !out->blk_key_base || !out->blk_val_base || !out->blk_status ||
      !out->key_off || !out->val_off || !out->key_bytes || !out->val_bytes || !out->trailer || !out->workspace ||
      out->workspace_bytes < pbl_transform_workspace_bytes(n_blocks))
    return PBL_INVALID_ARG;
  if (t->hide_obsolete_points && !in->kv_flags) return PBL_INVALID_ARG;
  if (!in->tiering_span_id != !in->tiering_attr || !out->tiering_span_id != !out->tiering_attr) return PBL_INVALID_ARG;
  if ((t->prefix_len && !t->prefix) || (t->suffix_len && !t->suffix) || t->split > PBL_SPLIT_CRDB)
    return PBL_INVALID_ARG;
  if (t->synthetic_seq_num >> 56) return PBL_INVALID_ARG;  // base.SeqNumMax
  const pbl_block_batch* src = t->blocks;
  if (!src || src->n_blocks != n_blocks) return PBL_INVALID_ARG;
  // row blocks: invalid keys are re-read from the block (entry offsets, flags)
  const bool rows = src->format == PBL_FMT_ROW || src->block_format;
  if (rows && !(src->flags & PBL_ROW_RAW_KEYS) && (!in->kv_flags || (t->prefix_len && (!in->entry_off || !src->blocks))))
    return PBL_INVALID_ARG;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  pbl::tf::TfArgs a;
  a.in = *in;
  a.out = *out;
  a.t = *t;
  a.src = *src;
  a.n_blocks = n_blocks;
  if (n_blocks == 0) {
    if (hipMemcpyAsync(out->totals, in->totals, sizeof(pbl_totals), hipMemcpyDeviceToDevice, st) != hipSuccess)
      return PBL_DEVICE_ERROR;
    return PBL_OK;
  }
  const uint32_t wpb = pbl::kTPB / pbl::kWave;
  const uint32_t grid = uint32_t(std::min<uint64_t>((n_blocks + wpb - 1) / wpb, 8192));
  if (hipMemsetAsync(out->workspace, 0, pbl::tf::tf_cnt_offset(n_blocks), st) != hipSuccess) return PBL_DEVICE_ERROR;
  hipLaunchKernelGGL(pbl::tf::tf_count_kernel, dim3(grid), dim3(pbl::kTPB), 0, st, a);
  const uint32_t nt = uint32_t(pbl::tf::tf_tiles(n_blocks));
  hipLaunchKernelGGL(pbl::tf::tf_scan_kernel, dim3(std::min<uint32_t>(nt, 1024)), dim3(pbl::kTPB), 0, st, a);
  hipLaunchKernelGGL(pbl::tf::tf_scatter_kernel, dim3(grid), dim3(pbl::kTPB), 0, st, a);
  return hipGetLastError() == hipSuccess ? PBL_OK : PBL_DEVICE_ERROR;
}

}  // extern "C"
