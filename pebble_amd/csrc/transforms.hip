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

constexpr int kTfWs = 64;  // workspace header: overflow flag

struct TfArgs {
  pbl_decode_out in, out;
  pbl_transforms t;
  uint32_t n_blocks;
};

// Comparer.Split of a user key (transforms.go:105-118 needs it for the suffix).
__device__ inline uint32_t split_len(gptr<const uint8_t> k, uint32_t n, uint32_t split) {
  if (split == PBL_SPLIT_TESTKEYS) {  // testkeys.Comparer: before the last '@' (internal/testkeys/testkeys.go:144-150)
    for (uint32_t i = n; i > 0; i--)
      if (k[i - 1] == '@') return i - 1;
    return n;
  }
  if (split == PBL_SPLIT_CRDB) {  // cockroachkvs.Split: the last byte is the version length (+1), 0 if none
    if (n == 0) return 0;
    const uint32_t v = k[n - 1];
    return v <= n ? n - v : 0;
  }
  return n;  // base.DefaultSplit: the whole key
}

struct KvView {
  bool vis, valid;
  uint32_t ko, klen, vo, vlen, p, nk;
};

__device__ inline KvView kv_view(const TfArgs& A, uint32_t b, uint64_t kv0, uint64_t kb_in, uint32_t j) {
  const pbl_decode_out& I = A.in;
  KvView v;
  const uint8_t fl = I.kv_flags ? to_glb(I.kv_flags)[kv0 + j] : uint8_t(0);
  v.vis = !(A.t.hide_obsolete_points && (fl & PBL_KV_OBSOLETE));
  v.valid = !(fl & PBL_KV_INVALID_KEY);
  const uint64_t o = kv0 + b + j;
  v.ko = to_glb(I.key_off)[o];
  v.klen = to_glb(I.key_off)[o + 1] - v.ko;
  v.vo = to_glb(I.val_off)[o];
  v.vlen = to_glb(I.val_off)[o + 1] - v.vo;
  v.p = v.klen;
  if (v.valid && A.t.suffix_len) v.p = split_len(to_glb(I.key_bytes) + kb_in + v.ko, v.klen, A.t.split);
  v.nk = v.valid ? A.t.prefix_len + v.p + (A.t.suffix_len ? A.t.suffix_len : v.klen - v.p) : 0u;
  return v;
}

__global__ void __launch_bounds__(kTPB) tf_count_kernel(TfArgs A) {
  uint32_t* cnt = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(A.out.workspace) + kTfWs);
  const uint32_t lane = lane_id();
  const uint32_t wpb = kTPB / kWave;
  for (uint32_t b = blockIdx.x * wpb + wave_id(); b < A.n_blocks; b += gridDim.x * wpb) {
    uint32_t c = 0, kb = 0, vb = 0;
    if (to_glb(A.in.blk_status)[b] == PBL_OK) {
      const uint64_t kv0 = to_glb(A.in.blk_kv_base)[b], n = to_glb(A.in.blk_kv_base)[b + 1] - kv0;
      const uint64_t kb_in = to_glb(A.in.blk_key_base)[b];
      for (uint32_t j = lane; j < n; j += kWave) {
        const KvView v = kv_view(A, b, kv0, kb_in, j);
        if (v.vis) {
          c++;
          kb += v.nk;
          vb += v.vlen;
        }
      }
      c = wave_sum(c);
      kb = wave_sum(kb);
      vb = wave_sum(vb);
    }
    if (lane == 0) {
      cnt[3 * uint64_t(b)] = c;
      cnt[3 * uint64_t(b) + 1] = kb;
      cnt[3 * uint64_t(b) + 2] = vb;
    }
  }
}

// One workgroup of kTPB threads; thread t scans a contiguous chunk of blocks.
__global__ void __launch_bounds__(kTPB) tf_scan_kernel(TfArgs A) {
  __shared__ uint64_t part[3][kTPB];
  const uint32_t* cnt = reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(A.out.workspace) + kTfWs);
  uint32_t* flag = reinterpret_cast<uint32_t*>(A.out.workspace);
  const uint32_t nb = A.n_blocks, t = threadIdx.x;
  const uint32_t chunk = (nb + kTPB - 1) / kTPB, b0 = min(nb, t * chunk), b1 = min(nb, b0 + chunk);
  uint64_t s[3] = {0, 0, 0};
  for (uint32_t b = b0; b < b1; b++)
    for (int q = 0; q < 3; q++) s[q] += cnt[3 * uint64_t(b) + q];
  for (int q = 0; q < 3; q++) part[q][t] = s[q];
  __syncthreads();
  if (t < 3) {  // serial scan of the kTPB chunk sums (one lane per component)
    uint64_t acc = 0;
    for (uint32_t i = 0; i < kTPB; i++) {
      const uint64_t x = part[t][i];
      part[t][i] = acc;
      acc += x;
    }
  }
  __syncthreads();
  const pbl_decode_out& I = A.in;
  const pbl_decode_out& O = A.out;
  uint64_t e[3] = {part[0][t], part[1][t], part[2][t]};
  for (uint32_t b = b0; b < b1; b++) {
    to_glb(O.blk_kv_base)[b] = e[0];
    to_glb(O.blk_key_base)[b] = e[1];
    to_glb(O.blk_val_base)[b] = e[2];
    if (O.blk_rst_base) to_glb(O.blk_rst_base)[b] = to_glb(I.blk_rst_base)[b];
    for (int q = 0; q < 3; q++) e[q] += cnt[3 * uint64_t(b) + q];
  }
  if (t == kTPB - 1) {
    const uint64_t nr = to_glb(I.blk_rst_base)[nb];
    to_glb(O.blk_kv_base)[nb] = e[0];
    to_glb(O.blk_key_base)[nb] = e[1];
    to_glb(O.blk_val_base)[nb] = e[2];
    if (O.blk_rst_base) to_glb(O.blk_rst_base)[nb] = nr;
    const bool over = e[0] > O.kv_cap || e[1] > O.key_cap || e[2] > O.val_cap || (O.restarts && nr > O.rst_cap);
    pbl_totals to = *I.totals;  // (one thread: a generic access is fine here)
    to.n_kv = e[0];
    to.key_bytes = e[1];
    to.val_bytes = e[2];
    to.n_restarts = nr;
    if (over) to.status_mask |= 1u << PBL_OVERFLOW;
    *O.totals = to;
    *to_glb(flag) = over ? 1u : 0u;
  }
  __syncthreads();
  // statuses: the decode's, PBL_OVERFLOW for the blocks that would have been written
  const bool over = *to_glb(flag) != 0;
  for (uint32_t b = b0; b < b1; b++) {
    uint32_t st = to_glb(I.blk_status)[b];
    if (over && st == PBL_OK) st = PBL_OVERFLOW;
    to_glb(O.blk_status)[b] = st;
  }
  if (over && t == 0) to_glb(O.totals)->n_bad_blocks = nb;  // (every block is now OVERFLOW or bad)
}

__global__ void __launch_bounds__(kTPB) tf_scatter_kernel(TfArgs A) {
  if (*to_glb(reinterpret_cast<const uint32_t*>(A.out.workspace)) != 0) return;  // overflow: sizes only
  const pbl_decode_out& I = A.in;
  const pbl_decode_out& O = A.out;
  const uint32_t lane = lane_id();
  const uint32_t wpb = kTPB / kWave;
  const gptr<const uint8_t> pfx = to_glb(A.t.prefix), sfx = to_glb(A.t.suffix);
  for (uint32_t b = blockIdx.x * wpb + wave_id(); b < A.n_blocks; b += gridDim.x * wpb) {
    const uint64_t okv = to_glb(O.blk_kv_base)[b], okb = to_glb(O.blk_key_base)[b], ovb = to_glb(O.blk_val_base)[b];
    if (to_glb(I.blk_status)[b] != PBL_OK) {
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
      if (act) v = kv_view(A, b, kv0, kb_in, j);
      const bool vis = act && v.vis;
      const uint64_t vm = __ballot(vis);
      const uint32_t rank = __builtin_popcountll(vm & ((1ull << lane) - 1));
      const uint32_t kx = wave_incl_scan(vis ? v.nk : 0u), vx = wave_incl_scan(vis ? v.vlen : 0u);
      const uint32_t ko = kcur + kx - (vis ? v.nk : 0u), vo = vcur + vx - (vis ? v.vlen : 0u);
      if (vis) {
        const uint64_t k = okv + jo + rank;
        uint64_t tr = to_glb(I.trailer)[kv0 + j];
        if (A.t.synthetic_seq_num) tr = (A.t.synthetic_seq_num << 8) | (tr & 0xffu);  // InternalKey.SetSeqNum
        to_glb(O.trailer)[k] = tr;
        if (O.kv_flags) to_glb(O.kv_flags)[k] = I.kv_flags ? to_glb(I.kv_flags)[kv0 + j] : uint8_t(0);
        if (O.entry_off && I.entry_off) to_glb(O.entry_off)[k] = to_glb(I.entry_off)[kv0 + j];
        to_glb(O.key_off)[okv + b + jo + rank] = ko;
        to_glb(O.val_off)[okv + b + jo + rank] = vo;
        // key: prefix ++ key[:p] ++ (suffix | key[p:])
        if (v.valid) {
          const gptr<const uint8_t> src = to_glb(I.key_bytes) + kb_in + v.ko;
          gptr<uint8_t> dst = to_glb(O.key_bytes) + okb + ko;
          uint32_t w = 0;
          for (uint32_t i = 0; i < A.t.prefix_len; i++) dst[w++] = pfx[i];
          for (uint32_t i = 0; i < v.p; i++) dst[w++] = src[i];
          if (A.t.suffix_len)
            for (uint32_t i = 0; i < A.t.suffix_len; i++) dst[w++] = sfx[i];
          else
            for (uint32_t i = v.p; i < v.klen; i++) dst[w++] = src[i];
        }
      }
      // values: each visible KV's bytes by the whole wave
      for (uint64_t m = vm; m; m &= m - 1) {
        const int src_lane = __builtin_ctzll(m);
        const uint32_t so = uint32_t(__shfl(int(v.vo), src_lane, kWave));
        const uint32_t sl = uint32_t(__shfl(int(v.vlen), src_lane, kWave));
        const uint32_t dofs = uint32_t(__shfl(int(vo), src_lane, kWave));
        const gptr<const uint8_t> s = to_glb(I.val_bytes) + vb_in + so;
        gptr<uint8_t> d = to_glb(O.val_bytes) + ovb + dofs;
        for (uint32_t i = lane; i < sl; i += kWave) d[i] = s[i];
      }
      jo += __builtin_popcountll(vm);
      kcur += uint32_t(__shfl(int(kx), kWave - 1, kWave));
      vcur += uint32_t(__shfl(int(vx), kWave - 1, kWave));
    }
    if (lane == 0) {
      to_glb(O.key_off)[okv + b + jo] = kcur;
      to_glb(O.val_off)[okv + b + jo] = vcur;
    }
    // restart words are the block's own (entry offsets never move)
    if (O.restarts && I.restarts) {
      const uint64_t r0 = to_glb(I.blk_rst_base)[b], r1 = to_glb(I.blk_rst_base)[b + 1];
      for (uint64_t r = r0 + lane; r < r1; r += kWave) to_glb(O.restarts)[r] = to_glb(I.restarts)[r];
    }
  }
}

}  // namespace tf
}  // namespace pbl

extern "C" {

uint64_t pbl_transform_workspace_bytes(uint32_t n_blocks) {
  return uint64_t(pbl::tf::kTfWs) + 12ull * n_blocks;
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
  if ((t->prefix_len && !t->prefix) || (t->suffix_len && !t->suffix) || t->split > PBL_SPLIT_CRDB)
    return PBL_INVALID_ARG;
  if (t->synthetic_seq_num >> 56) return PBL_INVALID_ARG;  // base.SeqNumMax
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  pbl::tf::TfArgs a;
  a.in = *in;
  a.out = *out;
  a.t = *t;
  a.n_blocks = n_blocks;
  if (n_blocks == 0) {
    if (hipMemcpyAsync(out->totals, in->totals, sizeof(pbl_totals), hipMemcpyDeviceToDevice, st) != hipSuccess)
      return PBL_DEVICE_ERROR;
    return PBL_OK;
  }
  const uint32_t wpb = pbl::kTPB / pbl::kWave;
  const uint32_t grid = uint32_t(std::min<uint64_t>((n_blocks + wpb - 1) / wpb, 8192));
  hipLaunchKernelGGL(pbl::tf::tf_count_kernel, dim3(grid), dim3(pbl::kTPB), 0, st, a);
  hipLaunchKernelGGL(pbl::tf::tf_scan_kernel, dim3(1), dim3(pbl::kTPB), 0, st, a);
  hipLaunchKernelGGL(pbl::tf::tf_scatter_kernel, dim3(grid), dim3(pbl::kTPB), 0, st, a);
  return hipGetLastError() == hipSuccess ? PBL_OK : PBL_DEVICE_ERROR;
}

}  // extern "C"
