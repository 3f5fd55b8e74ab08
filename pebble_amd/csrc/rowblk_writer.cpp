// rowblk_writer.cpp — native restatement of Pebble's row-oriented block writer
// (the format PRODUCER; host code), plus the seeded synthetic batch generator
// used by tests and bench.py.
//
// Follows sstable/rowblk/rowblk_writer.go (cockroachdb/pebble):
//   Writer fields / restart flag          :48-99
//   storeWithOptionalValuePrefix          :128-243
//   Add / AddWithOptionalValuePrefix      :246-286
//   Finish / EstimatedSize                :289-320
//   AddRaw                                :323-334
// InternalKey encoding (user key || LE64 trailer): internal/base/internal.go:441-444.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/pebble_amd.h"

namespace {

constexpr uint32_t kSetHasSameKeyPrefixRestartMask = 1u << 31;  // :99
constexpr uint64_t kMaximumRestartOffset = (1ull << 31) - 1;      // :24
constexpr uint64_t kTrailerObsoleteBit = 64;                      // :38

inline size_t varint_len(uint32_t x) {
  size_t n = 1;
  while (x >= 0x80) { x >>= 7; n++; }
  return n;
}
inline void put_varint(std::vector<uint8_t>& b, uint32_t x) {
  while (x >= 0x80) { b.push_back(uint8_t(x) | 0x80); x >>= 7; }
  b.push_back(uint8_t(x));
}

}  // namespace

struct pbl_rowblk_writer {
  int restart_interval = 16;
  int n_entries = 0;
  int next_restart = 0;
  std::vector<uint8_t> buf;
  std::vector<uint32_t> restarts;
  std::vector<uint8_t> cur_key, prev_key;
  bool same_prefix_since_restart = false;

  void reset(int ri) {
    restart_interval = ri;
    n_entries = next_restart = 0;
    buf.clear();
    restarts.clear();
    cur_key.clear();
    prev_key.clear();
    same_prefix_since_restart = false;
  }

  size_t shared_len(size_t max_shared) const {
    size_t n = std::min(max_shared, prev_key.size());
    n = std::min(n, cur_key.size());
    size_t s = 0;
    while (s < n && cur_key[s] == prev_key[s]) s++;
    return s;
  }

  // storeWithOptionalValuePrefix :128-243
  int store(size_t key_size, const uint8_t* value, size_t value_len, int64_t max_shared,
            bool add_prefix, uint8_t prefix, bool set_same) {
    if (buf.size() >= kMaximumRestartOffset) return PBL_UNSUPPORTED;  // ErrBlockTooBig
    size_t shared = 0;
    if (!set_same) same_prefix_since_restart = false;
    if (n_entries == next_restart) {
      next_restart = n_entries + restart_interval;
      uint32_t r = uint32_t(buf.size());
      if (same_prefix_since_restart) r |= kSetHasSameKeyPrefixRestartMask;
      same_prefix_since_restart = true;
      restarts.push_back(r);
    } else {
      shared = shared_len(max_shared < 0 ? 0 : size_t(max_shared));
    }
    size_t vlen = value_len + (add_prefix ? 1 : 0);
    put_varint(buf, uint32_t(shared));
    put_varint(buf, uint32_t(key_size - shared));
    put_varint(buf, uint32_t(vlen));
    buf.insert(buf.end(), cur_key.begin() + shared, cur_key.begin() + key_size);
    if (add_prefix) buf.push_back(prefix);
    if (value_len) buf.insert(buf.end(), value, value + value_len);
    n_entries++;
    return PBL_OK;
  }

  // Exact encoded growth (entry + restart word) of the next Add, used to fill
  // blocks to a byte budget without overshooting.
  size_t next_entry_growth(const uint8_t* ikey, size_t klen, size_t value_len, int64_t max_shared,
                           bool add_prefix) const {
    size_t shared = 0, grow = 0;
    if (n_entries == next_restart) {
      grow += 4;
    } else {
      size_t n = std::min<size_t>(max_shared < 0 ? 0 : size_t(max_shared), cur_key.size());
      n = std::min(n, klen);
      while (shared < n && ikey[shared] == cur_key[shared]) shared++;
    }
    size_t vlen = value_len + (add_prefix ? 1 : 0);
    grow += varint_len(uint32_t(shared)) + varint_len(uint32_t(klen - shared)) +
            varint_len(uint32_t(vlen)) + (klen - shared) + vlen;
    return grow;
  }

  size_t estimated_size() const { return buf.size() + 4 * restarts.size() + 4; }

  size_t finish(uint8_t* dst, size_t cap) {  // :289-315
    if (n_entries == 0) restarts.assign(1, 0u);
    for (uint32_t x : restarts)
      for (int i = 0; i < 4; i++) buf.push_back(uint8_t(x >> (8 * i)));
    uint32_t n = uint32_t(restarts.size());
    for (int i = 0; i < 4; i++) buf.push_back(uint8_t(n >> (8 * i)));
    size_t sz = buf.size();
    if (dst && cap >= sz) std::memcpy(dst, buf.data(), sz);
    n_entries = next_restart = 0;
    buf.clear();
    restarts.clear();
    return sz;
  }
};

extern "C" {

pbl_rowblk_writer* pbl_rowblk_writer_new(int restart_interval) {
  auto* w = new pbl_rowblk_writer();
  w->reset(restart_interval);
  return w;
}
void pbl_rowblk_writer_free(pbl_rowblk_writer* w) { delete w; }
void pbl_rowblk_writer_reset(pbl_rowblk_writer* w, int ri) { w->reset(ri); }

int pbl_rowblk_writer_add(pbl_rowblk_writer* w, const uint8_t* user_key, size_t ukl,
                          uint64_t trailer, int is_obsolete, const uint8_t* value,
                          size_t value_len, int64_t max_shared_key_len, int add_value_prefix,
                          uint8_t value_prefix, int set_has_same_key_prefix) {
  std::swap(w->cur_key, w->prev_key);  // :272
  if (is_obsolete) trailer |= kTrailerObsoleteBit;
  w->cur_key.resize(ukl + 8);
  if (ukl) std::memcpy(w->cur_key.data(), user_key, ukl);
  for (int i = 0; i < 8; i++) w->cur_key[ukl + i] = uint8_t(trailer >> (8 * i));
  return w->store(ukl + 8, value, value_len, max_shared_key_len, add_value_prefix != 0,
                  value_prefix, set_has_same_key_prefix != 0);
}

int pbl_rowblk_writer_add_raw(pbl_rowblk_writer* w, const uint8_t* key, size_t key_len,
                              const uint8_t* value, size_t value_len) {
  std::swap(w->cur_key, w->prev_key);
  w->cur_key.assign(key, key + key_len);
  return w->store(key_len, value, value_len, int64_t(key_len), false, 0, false);
}

size_t pbl_rowblk_writer_estimated_size(const pbl_rowblk_writer* w) { return w->estimated_size(); }
size_t pbl_rowblk_writer_entry_count(const pbl_rowblk_writer* w) { return size_t(w->n_entries); }
size_t pbl_rowblk_writer_finish(pbl_rowblk_writer* w, uint8_t* dst, size_t cap) {
  return w->finish(dst, cap);
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Synthetic batch generator.
// ---------------------------------------------------------------------------
namespace {

inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

void fill_bytes(uint8_t* p, size_t n, uint64_t s) {
  for (size_t i = 0; i < n; i += 8) {
    uint64_t r = splitmix64(s + i);
    size_t k = std::min<size_t>(8, n - i);
    std::memcpy(p + i, &r, k);
  }
}

uint64_t gen_one_block(uint64_t seed, uint32_t b, uint32_t block_size, int ri, uint32_t key_len,
                       uint32_t val_len, bool vprefix, uint32_t obsolete_every, uint8_t* dst, uint32_t* out_len) {
  pbl_rowblk_writer w;
  w.reset(ri);
  std::vector<uint8_t> ukey(key_len), ikey(key_len + 8), val(val_len);
  uint64_t k = 0;
  for (;; k++) {
    uint64_t r = (uint64_t(b) << 20) + k;
    for (int i = 0; i < 8 && i < int(key_len); i++) ukey[i] = uint8_t(r >> (56 - 8 * i));
    if (key_len > 8) {
      uint64_t h = splitmix64(seed ^ r);
      for (uint32_t i = 8; i < key_len; i++) {
        if (i > 8 && (i % 8) == 0) h = splitmix64(h);
        ukey[i] = uint8_t(h >> (56 - 8 * (i % 8)));
      }
    }
    uint64_t trailer = (r << 8) | 1u;  // MakeTrailer(seq = r, SET)
    std::memcpy(ikey.data(), ukey.data(), key_len);
    for (int i = 0; i < 8; i++) ikey[key_len + i] = uint8_t(trailer >> (8 * i));
    size_t grow = w.next_entry_growth(ikey.data(), key_len + 8, val_len, int64_t(key_len), vprefix);
    if (w.estimated_size() + grow > block_size) break;
    fill_bytes(val.data(), val_len, seed + r * 0x9E3779B97F4A7C15ull);
    const int obs = obsolete_every && (k % obsolete_every) == obsolete_every - 1;
    pbl_rowblk_writer_add(&w, ukey.data(), key_len, trailer, obs, val.data(), val_len,
                          int64_t(key_len), vprefix ? 1 : 0, 0x00, 0);
  }
  size_t sz = w.finish(dst, block_size);
  *out_len = uint32_t(sz);
  std::memset(dst + sz, 0, block_size - sz);
  return k;
}

}  // namespace

extern "C" uint64_t pbl_gen_row_blocks_obs(uint64_t seed, uint32_t first_block, uint32_t n_blocks,
                                           uint32_t block_size, int restart_interval, uint32_t key_len,
                                           uint32_t val_len, int value_prefix, uint32_t obsolete_every,
                                           uint8_t* dst, uint64_t* block_off, uint32_t* block_len, int n_threads) {
  if (n_threads <= 0) n_threads = int(std::max(1u, std::thread::hardware_concurrency()));
  n_threads = std::min<int>(n_threads, 64);
  if (key_len < 8) key_len = 8;
  std::vector<uint64_t> counts(size_t(n_threads), 0);
  auto work = [&](int t) {
    uint64_t c = 0;
    for (uint32_t b = uint32_t(t); b < n_blocks; b += uint32_t(n_threads)) {
      block_off[b] = uint64_t(b) * block_size;
      c += gen_one_block(seed, first_block + b, block_size, restart_interval, key_len, val_len,
                         value_prefix != 0, obsolete_every, dst + uint64_t(b) * block_size, &block_len[b]);
    }
    counts[size_t(t)] = c;
  };
  std::vector<std::thread> th;
  for (int t = 1; t < n_threads; t++) th.emplace_back(work, t);
  work(0);
  for (auto& x : th) x.join();
  uint64_t total = 0;
  for (auto c : counts) total += c;
  return total;
}

extern "C" uint64_t pbl_gen_row_blocks(uint64_t seed, uint32_t n_blocks, uint32_t block_size,
                                       int restart_interval, uint32_t key_len, uint32_t val_len,
                                       int value_prefix, uint8_t* dst, uint64_t* block_off,
                                       uint32_t* block_len, int n_threads) {
  return pbl_gen_row_blocks_obs(seed, 0, n_blocks, block_size, restart_interval, key_len, val_len, value_prefix, 0,
                                dst, block_off, block_len, n_threads);
}
