// data_iter.cpp — SURVEY.md §8 f2, host side: a blockiter.Data iterator over
// one decoded block of a batch (the flat arrays of pbl_decode_out, copied to
// host memory).  This is the adapter the Go shim exposes behind
// sstable/blockiter (block_iter.go:19-108): rowblk.Iter / colblk.DataBlockIter
// semantics for positioning, with the KVs already materialized by the device.
//
// Positions follow rowblk.Iter (rowblk_iter.go): SeekGE / SeekLT compare user
// keys with the block's comparer (:606-781, :782-1054), stepping past either
// end leaves the iterator exhausted there and the opposite step re-enters at
// the last / first KV (Next :1145-1201 after SeekLT past the front, Prev
// :1504-1635 after a forward walk off the end); SeekPrefixGE / NextWithSamePrefix
// / NextPrefix / IsLowerBound as :542-598, :1204-1218; HideObsoletePoints
// (blockiter.Transforms) skips KVs whose trailer carried the obsolete bit
// (PBL_KV_OBSOLETE), as :1168-1179.  *_with_meta: colblk.DataBlockIter's
// FirstWithMeta / NextWithMeta / SeekGEWithMeta (sstable/colblk/data_block.go:
// 1574-1600, decodeMeta :1633-1641) over the decoded KVMeta arrays.  Comparers: base.DefaultComparer
// (internal/base/comparer.go: bytes.Compare, Split = len), testkeys.Comparer
// (internal/testkeys/testkeys.go:136-171) and cockroachkvs.Comparer
// (cockroachkvs/cockroachkvs.go:298-339, :479-...).
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <new>

#include "../../include/pebble_amd.h"

struct pbl_data_iter {
  const uint64_t* trailer = nullptr;
  const uint8_t* kv_flags = nullptr;
  const uint32_t* key_off = nullptr;  // n + 1, block relative
  const uint32_t* val_off = nullptr;
  const uint8_t* key_bytes = nullptr;  // this block's bytes
  const uint8_t* val_bytes = nullptr;
  const uint64_t* span = nullptr;  // KVMeta arrays (NULL: not decoded, KVMeta{})
  const uint64_t* attr = nullptr;
  int64_t n = 0;
  int64_t i = -1;  // -1: before the first KV; n: past the last
  uint32_t cmp = PBL_CMP_DEFAULT;
  bool hide_obsolete = false;
  bool invalidated = true;
  // NextWithSamePrefix's saved prefix (rowblk_iter.go:571-598)
  const uint8_t* pfx = nullptr;
  uint64_t pfx_len = 0;
  bool has_pfx = false;
  pbl_kv kv{};
};

namespace {

int bytes_cmp(const uint8_t* a, uint64_t al, const uint8_t* b, uint64_t bl) {
  const int c = memcmp(a, b, std::min(al, bl));
  if (c) return c < 0 ? -1 : 1;
  return al < bl ? -1 : al > bl ? 1 : 0;
}

// ---- testkeys.Comparer -------------------------------------------------------
uint64_t tk_split(const uint8_t* a, uint64_t n) {
  for (uint64_t i = n; i > 0; i--)
    if (a[i - 1] == '@') return i - 1;
  return n;
}
// "@N" -> N (parseUintBytes base 10); malformed suffixes (Go panics) sort by bytes
bool tk_ts(const uint8_t* s, uint64_t n, uint64_t* v) {
  static const char kIgn[] = "_synthetic";
  const uint64_t il = sizeof(kIgn) - 1;
  if (n >= il && memcmp(s + n - il, kIgn, il) == 0) n -= il;
  if (n < 2 || s[0] != '@') return false;
  uint64_t x = 0;
  for (uint64_t k = 1; k < n; k++) {
    if (s[k] < '0' || s[k] > '9') return false;
    x = x * 10 + (s[k] - '0');
  }
  *v = x;
  return true;
}
uint64_t tk_trim(const uint8_t* s, uint64_t n) {
  static const char kIgn[] = "_synthetic";
  const uint64_t il = sizeof(kIgn) - 1;
  return (n >= il && memcmp(s + n - il, kIgn, il) == 0) ? n - il : n;
}
int tk_cmp(const uint8_t* a, uint64_t al, const uint8_t* b, uint64_t bl) {
  const uint64_t ai = tk_split(a, al), bi = tk_split(b, bl);
  const int c = bytes_cmp(a, ai, b, bi);
  if (c) return c;
  const uint64_t as = tk_trim(a + ai, al - ai), bs = tk_trim(b + bi, bl - bi);
  if (as == 0 || bs == 0) return as < bs ? -1 : as > bs ? 1 : 0;  // the empty suffix sorts first
  uint64_t x, y;
  if (!tk_ts(a + ai, al - ai, &x) || !tk_ts(b + bi, bl - bi, &y)) return bytes_cmp(a + ai, as, b + bi, bs);
  return y < x ? -1 : y > x ? 1 : 0;  // cmp.Compare(bi, ai): newer first
}

// ---- cockroachkvs.Comparer ---------------------------------------------------
uint64_t crdb_split(const uint8_t* a, uint64_t n) {  // cockroachkvs.go:298-311
  if (n == 0) return 0;
  const uint64_t s = uint64_t(a[n - 1]);
  return s <= n ? n - s : 0;
}
// normalizeEngineSuffixForCompare (cockroachkvs.go): the suffix without its
// length byte, with a zero logical component and a synthetic bit dropped so that
// equal timestamps compare equal
uint64_t crdb_norm(const uint8_t* s, uint64_t n) {
  if (n == 0) return 0;
  uint64_t v = n - 1;  // the version, without the length byte
  // engineKeyVersionWallLogicalAndSyntheticTimeLen = 13, WallAndLogical = 12,
  // WallTime = 8: drop the synthetic byte, then a zero logical
  if (v == 13) v = 12;
  if (v == 12) {
    const uint8_t* lg = s + 8;
    if (lg[0] == 0 && lg[1] == 0 && lg[2] == 0 && lg[3] == 0) v = 8;
  }
  return v;
}
int crdb_cmp(const uint8_t* a, uint64_t al, const uint8_t* b, uint64_t bl) {  // cockroachkvs.go:313-339
  if (al == 0 || bl == 0) return al < bl ? -1 : al > bl ? 1 : 0;
  const uint64_t asl = a[al - 1], bsl = b[bl - 1];
  const uint64_t ass = asl <= al ? al - asl : 0, bss = bsl <= bl ? bl - bsl : 0;
  const int c = bytes_cmp(a, ass, b, bss);
  if (c) return c;
  if (asl == 0 || bsl == 0) return asl < bsl ? -1 : asl > bsl ? 1 : 0;
  const uint64_t an = crdb_norm(a + ass, al - ass), bn = crdb_norm(b + bss, bl - bss);
  return bytes_cmp(b + bss, bn, a + ass, an);  // descending versions
}

int key_cmp(uint32_t cmp, const uint8_t* a, uint64_t al, const uint8_t* b, uint64_t bl) {
  switch (cmp) {
    case PBL_CMP_TESTKEYS: return tk_cmp(a, al, b, bl);
    case PBL_CMP_CRDB: return crdb_cmp(a, al, b, bl);
    default: return bytes_cmp(a, al, b, bl);
  }
}
uint64_t key_split(uint32_t cmp, const uint8_t* a, uint64_t n) {
  switch (cmp) {
    case PBL_CMP_TESTKEYS: return tk_split(a, n);
    case PBL_CMP_CRDB: return crdb_split(a, n);
    default: return n;
  }
}

inline const uint8_t* ukey(const pbl_data_iter* it, int64_t j, uint64_t* len) {
  *len = uint64_t(it->key_off[j + 1]) - it->key_off[j];
  return it->key_bytes + it->key_off[j];
}
inline bool hidden(const pbl_data_iter* it, int64_t j) {
  return it->hide_obsolete && it->kv_flags && (it->kv_flags[j] & PBL_KV_OBSOLETE);
}

const pbl_kv* at(pbl_data_iter* it) {
  if (it->i < 0 || it->i >= it->n) return nullptr;
  const int64_t j = it->i;
  it->kv.user_key = ukey(it, j, &it->kv.user_key_len);
  it->kv.trailer = it->trailer[j];
  it->kv.value = it->val_bytes + it->val_off[j];
  it->kv.value_len = uint64_t(it->val_off[j + 1]) - it->val_off[j];
  it->kv.kv_flags = it->kv_flags ? it->kv_flags[j] : 0u;
  return &it->kv;
}
const pbl_kv* fwd(pbl_data_iter* it, int64_t j) {  // first visible KV at or after j
  while (j < it->n && hidden(it, j)) j++;
  it->i = j < it->n ? j : it->n;
  return at(it);
}
const pbl_kv* bwd(pbl_data_iter* it, int64_t j) {  // last visible KV at or before j
  while (j >= 0 && hidden(it, j)) j--;
  it->i = j >= 0 ? j : -1;
  return at(it);
}
// first KV whose user key is >= key (strict: >)
int64_t lower(const pbl_data_iter* it, const uint8_t* k, uint64_t kl, bool strict) {
  int64_t lo = 0, hi = it->n;
  while (lo < hi) {
    const int64_t m = lo + (hi - lo) / 2;
    uint64_t ml;
    const uint8_t* mk = ukey(it, m, &ml);
    const int c = key_cmp(it->cmp, mk, ml, k, kl);
    if (c < 0 || (strict && c == 0)) lo = m + 1;
    else hi = m;
  }
  return lo;
}

}  // namespace

extern "C" {

pbl_data_iter* pbl_data_iter_new(void) { return new (std::nothrow) pbl_data_iter(); }

void pbl_data_iter_free(pbl_data_iter* it) { delete it; }

int pbl_data_iter_init(pbl_data_iter* it, const pbl_decode_out* host, uint32_t n_blocks, uint32_t block,
                       uint32_t comparer, uint32_t hide_obsolete_points) {
  if (!it || !host || block >= n_blocks || comparer > PBL_CMP_CRDB || !host->trailer || !host->key_off ||
      !host->val_off || !host->key_bytes || !host->val_bytes || !host->blk_kv_base || !host->blk_key_base ||
      !host->blk_val_base || !host->blk_status)
    return PBL_INVALID_ARG;
  *it = pbl_data_iter();
  if (host->blk_status[block] != PBL_OK) return int(host->blk_status[block]);  // (InitHandle's error)
  const uint64_t kv0 = host->blk_kv_base[block];
  it->n = int64_t(host->blk_kv_base[block + 1] - kv0);
  it->trailer = host->trailer + kv0;
  it->kv_flags = host->kv_flags ? host->kv_flags + kv0 : nullptr;
  it->key_off = host->key_off + kv0 + block;
  it->val_off = host->val_off + kv0 + block;
  it->key_bytes = host->key_bytes + host->blk_key_base[block];
  it->val_bytes = host->val_bytes + host->blk_val_base[block];
  if (host->tiering_span_id && host->tiering_attr) {
    it->span = host->tiering_span_id + kv0;
    it->attr = host->tiering_attr + kv0;
  }
  it->cmp = comparer;
  it->hide_obsolete = hide_obsolete_points != 0;
  it->invalidated = false;
  it->i = -1;
  return PBL_OK;
}

const pbl_kv* pbl_data_iter_first(pbl_data_iter* it) {
  it->has_pfx = false;
  return it->invalidated ? nullptr : fwd(it, 0);
}
const pbl_kv* pbl_data_iter_last(pbl_data_iter* it) {
  it->has_pfx = false;
  return it->invalidated ? nullptr : bwd(it, it->n - 1);
}
const pbl_kv* pbl_data_iter_next(pbl_data_iter* it) {
  it->has_pfx = false;
  if (it->invalidated) return nullptr;
  return it->i >= it->n ? nullptr : fwd(it, it->i + 1);
}
const pbl_kv* pbl_data_iter_prev(pbl_data_iter* it) {
  it->has_pfx = false;
  if (it->invalidated) return nullptr;
  return it->i < 0 ? nullptr : bwd(it, it->i - 1);
}
const pbl_kv* pbl_data_iter_seek_ge(pbl_data_iter* it, const uint8_t* key, uint64_t key_len, uint32_t flags) {
  (void)flags;  // (TrySeekUsingNext is an optimisation: same result)
  it->has_pfx = false;
  return it->invalidated ? nullptr : fwd(it, lower(it, key, key_len, false));
}
const pbl_kv* pbl_data_iter_seek_lt(pbl_data_iter* it, const uint8_t* key, uint64_t key_len, uint32_t flags) {
  (void)flags;
  it->has_pfx = false;
  return it->invalidated ? nullptr : bwd(it, lower(it, key, key_len, false) - 1);
}
}  // extern "C"

namespace {
// decodeMeta (data_block.go:1633-1641): the KV's meta, KVMeta{} when there is none
const pbl_kv* with_meta(const pbl_data_iter* it, const pbl_kv* kv, pbl_kv_meta* meta) {
  meta->tiering_span_id = meta->tiering_attribute = 0;
  if (kv && it->span) {
    meta->tiering_span_id = it->span[it->i];
    meta->tiering_attribute = it->attr[it->i];
  }
  return kv;
}
}  // namespace

extern "C" {

const pbl_kv* pbl_data_iter_first_with_meta(pbl_data_iter* it, pbl_kv_meta* meta) {
  return with_meta(it, pbl_data_iter_first(it), meta);
}
const pbl_kv* pbl_data_iter_next_with_meta(pbl_data_iter* it, pbl_kv_meta* meta) {
  return with_meta(it, pbl_data_iter_next(it), meta);
}
const pbl_kv* pbl_data_iter_seek_ge_with_meta(pbl_data_iter* it, const uint8_t* key, uint64_t key_len,
                                              uint32_t flags, pbl_kv_meta* meta) {
  return with_meta(it, pbl_data_iter_seek_ge(it, key, key_len, flags), meta);
}
const pbl_kv* pbl_data_iter_seek_prefix_ge(pbl_data_iter* it, const uint8_t* key, uint64_t key_len, uint32_t flags,
                                           int* prefix_did_not_match) {
  *prefix_did_not_match = 0;
  const pbl_kv* kv = pbl_data_iter_seek_ge(it, key, key_len, flags);
  if (!kv) return nullptr;
  const uint64_t sp = key_split(it->cmp, key, key_len), kp = key_split(it->cmp, kv->user_key, kv->user_key_len);
  if (sp != kp || memcmp(key, kv->user_key, sp) != 0) {
    *prefix_did_not_match = 1;
    return nullptr;
  }
  return kv;
}
const pbl_kv* pbl_data_iter_next_with_same_prefix(pbl_data_iter* it, int* prefix_exhausted) {
  *prefix_exhausted = 0;
  if (!it->has_pfx) {
    const pbl_kv* cur = at(it);
    if (it->invalidated || !cur) return nullptr;
    it->pfx = cur->user_key;
    it->pfx_len = key_split(it->cmp, cur->user_key, cur->user_key_len);
  }
  const uint8_t* p = it->pfx;
  const uint64_t pl = it->pfx_len;
  const pbl_kv* kv = pbl_data_iter_next(it);
  if (!kv) return nullptr;
  const uint64_t n = key_split(it->cmp, kv->user_key, kv->user_key_len);
  if (n != pl || memcmp(kv->user_key, p, n) != 0) {
    *prefix_exhausted = 1;  // positioned at the new-prefix KV
    return nullptr;
  }
  it->pfx = p;
  it->pfx_len = pl;
  it->has_pfx = true;
  return kv;
}
const pbl_kv* pbl_data_iter_next_prefix(pbl_data_iter* it, const uint8_t* succ_key, uint64_t succ_len) {
  it->has_pfx = false;
  if (it->invalidated) return nullptr;
  // the first visible KV after the current one whose user key is >= succKey
  const int64_t from = it->i + 1 > 0 ? it->i + 1 : 0;
  const int64_t lb = std::max(from, lower(it, succ_key, succ_len, false));
  return fwd(it, std::min<int64_t>(lb, it->n));
}
int pbl_data_iter_is_lower_bound(const pbl_data_iter* it, const uint8_t* key, uint64_t key_len) {
  // Compare(firstUserKey, k) >= 0; an empty block bounds any key
  if (it->invalidated || it->n == 0) return 1;
  uint64_t fl;
  const uint8_t* f = ukey(it, 0, &fl);
  return key_cmp(it->cmp, f, fl, key, key_len) >= 0;
}
int pbl_data_iter_valid(const pbl_data_iter* it) { return !it->invalidated && it->i >= 0 && it->i < it->n; }
const pbl_kv* pbl_data_iter_kv(pbl_data_iter* it) { return it->invalidated ? nullptr : at(it); }
void pbl_data_iter_invalidate(pbl_data_iter* it) {
  *it = pbl_data_iter();
  it->invalidated = true;
}
int pbl_data_iter_is_data_invalidated(const pbl_data_iter* it) { return it->invalidated ? 1 : 0; }
int pbl_key_compare(uint32_t comparer, const uint8_t* a, uint64_t a_len, const uint8_t* b, uint64_t b_len) {
  return key_cmp(comparer, a, a_len, b, b_len);
}
uint64_t pbl_key_split(uint32_t comparer, const uint8_t* key, uint64_t key_len) {
  return key_split(comparer, key, key_len);
}

}  // extern "C"
