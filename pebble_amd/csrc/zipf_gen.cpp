// Synthetic config-5 batches (BASELINE.json configs[4]):
// Zipf-skewed key lengths (8-1024 B) and value lengths (0-64 KiB), row format
// at a chosen restart interval or colblk with colblk.DefaultKeySchema.  Blocks
// target `block_size` but a block always takes its first KV, so one large KV
// makes a block larger than the target; blocks are variable-length and packed
// back to back at 8-B alignment (colblk requires it, data_block.go:1097), so
// the batch is described by (offset, len) pairs instead of a fixed stride.
//
// Host-side test/bench data producer built on the format writers
// (rowblk_writer.cpp, colblk_writer.cpp); not on the decode path.

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/pebble_amd.h"

namespace {

inline uint64_t sm64(uint64_t& s) {
  uint64_t x = (s += 0x9E3779B97F4A7C15ull);
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// P(x) ~ 1 / (x - lo + 1)^s on [lo, hi], sampled by inverse CDF.
struct Zipf {
  uint32_t lo = 0;
  std::vector<double> cdf;
  Zipf(uint32_t lo_, uint32_t hi, double s) : lo(lo_) {
    cdf.resize(size_t(hi - lo_) + 1);
    double acc = 0;
    for (size_t i = 0; i < cdf.size(); i++) cdf[i] = (acc += std::pow(double(i + 1), -s));
    for (auto& c : cdf) c /= acc;
  }
  uint32_t operator()(uint64_t& st) const {
    const double u = double(sm64(st) >> 11) * (1.0 / 9007199254740992.0);
    size_t i = size_t(std::upper_bound(cdf.begin(), cdf.end(), u) - cdf.begin());
    return lo + uint32_t(std::min(i, cdf.size() - 1));
  }
};

// Key of row r: 8 base-26 letters of r (big-endian, so keys ascend with r and
// never contain the default schema's '@' separator), then random letters.
void make_key(uint64_t r, uint32_t len, uint64_t& st, std::vector<uint8_t>& k) {
  k.resize(len);
  uint64_t x = r;
  for (int i = 7; i >= 0; i--) {
    const uint8_t c = uint8_t('a' + x % 26);
    x /= 26;
    if (uint32_t(i) < len) k[size_t(i)] = c;
  }
  for (uint32_t i = 8; i < len; i++) k[i] = uint8_t('a' + sm64(st) % 26);
}

void fill_value(std::vector<uint8_t>& v, uint32_t len, uint64_t& st) {
  v.resize(len);
  for (uint32_t i = 0; i < len; i += 8) {
    const uint64_t w = sm64(st);
    std::memcpy(v.data() + i, &w, std::min<uint32_t>(8, len - i));
  }
}

uint64_t gen_row(const pbl_zipf_config& c, const Zipf& zk, const Zipf& zv, uint32_t b, std::vector<uint8_t>& out) {
  pbl_rowblk_writer* w = pbl_rowblk_writer_new(c.restart_interval);
  uint64_t st = c.seed ^ (0x5A1Full * (uint64_t(b) + 1));
  std::vector<uint8_t> key, val;
  uint64_t k = 0;
  for (;; k++) {
    const uint32_t kl = zk(st), vl = zv(st);
    // upper bound of the entry's growth: 3 varints, key, trailer, value, restart word
    const size_t grow = 15 + kl + 8 + vl + 4;
    if (k > 0 && pbl_rowblk_writer_estimated_size(w) + grow > c.block_size) break;
    const uint64_t r = (uint64_t(b) << 20) + k;
    make_key(r, kl, st, key);
    fill_value(val, vl, st);
    pbl_rowblk_writer_add(w, key.data(), kl, (r << 8) | 1u, 0, val.data(), vl, int64_t(kl), 0, 0, 0);
  }
  out.resize(pbl_rowblk_writer_estimated_size(w) + 8);
  out.resize(pbl_rowblk_writer_finish(w, out.data(), out.size()));
  pbl_rowblk_writer_free(w);
  return k;
}

uint64_t gen_col(const pbl_zipf_config& c, const Zipf& zk, const Zipf& zv, uint32_t b, std::vector<uint8_t>& out) {
  pbl_colblk_writer* w = pbl_colblk_writer_new(PBL_FMT_COL_DEFAULT, 16);
  uint64_t st = c.seed ^ (0xC01Dull * (uint64_t(b) + 1));
  std::vector<uint8_t> key, val;
  uint32_t rows = 0;
  for (uint64_t k = 0;; k++) {
    const uint32_t kl = zk(st), vl = zv(st);
    const uint64_t r = (uint64_t(b) << 20) + k;
    make_key(r, kl, st, key);
    fill_value(val, vl, st);
    pbl_colblk_writer_add(w, key.data(), kl, -1, (r << 8) | 1u, val.data(), vl, 0, 0);
    rows = pbl_colblk_writer_rows(w);
    if (rows > 1 && pbl_colblk_writer_size(w, rows) > c.block_size) {
      rows--;  // Finish(rows-1): the overflowing KV is dropped
      break;
    }
  }
  const size_t n = pbl_colblk_writer_size(w, rows);
  out.resize(n);
  out.resize(pbl_colblk_writer_finish(w, rows, out.data(), n));
  pbl_colblk_writer_free(w);
  return rows;
}

}  // namespace

extern "C" uint64_t pbl_gen_zipf_blocks(const pbl_zipf_config* cfgp, uint32_t format, uint32_t n_blocks,
                                        uint8_t* dst, uint64_t dst_cap, uint64_t* block_off, uint32_t* block_len,
                                        uint64_t* bytes_used, int n_threads) {
  const pbl_zipf_config c = *cfgp;
  if ((format != PBL_FMT_ROW && format != PBL_FMT_COL_DEFAULT) || c.key_min < 8 || c.key_max < c.key_min ||
      c.val_max < c.val_min || (format == PBL_FMT_ROW && c.restart_interval < 1))
    return UINT64_MAX;
  if (n_threads < 1) n_threads = 1;
  const Zipf zk(c.key_min, c.key_max, c.s), zv(c.val_min, c.val_max, c.s);
  std::vector<std::vector<uint8_t>> blocks(n_blocks);
  std::vector<uint64_t> counts(size_t(n_threads), 0);
  auto gen = [&](int t) {
    for (uint32_t b = uint32_t(t); b < n_blocks; b += uint32_t(n_threads))
      counts[size_t(t)] += format == PBL_FMT_ROW ? gen_row(c, zk, zv, c.first_block + b, blocks[b])
                                                 : gen_col(c, zk, zv, c.first_block + b, blocks[b]);
  };
  std::vector<std::thread> th;
  for (int t = 1; t < n_threads; t++) th.emplace_back(gen, t);
  gen(0);
  for (auto& x : th) x.join();
  uint64_t pos = 0;
  for (uint32_t b = 0; b < n_blocks; b++) {
    block_off[b] = pos;
    block_len[b] = uint32_t(blocks[b].size());
    pos = (pos + blocks[b].size() + 7) & ~uint64_t(7);
  }
  *bytes_used = pos;
  if (pos > dst_cap) return UINT64_MAX;
  auto copy = [&](int t) {
    for (uint32_t b = uint32_t(t); b < n_blocks; b += uint32_t(n_threads)) {
      std::memcpy(dst + block_off[b], blocks[b].data(), blocks[b].size());
      const uint64_t end = b + 1 < n_blocks ? block_off[b + 1] : pos;
      std::memset(dst + block_off[b] + blocks[b].size(), 0, end - block_off[b] - blocks[b].size());
      std::vector<uint8_t>().swap(blocks[b]);
    }
  };
  th.clear();
  for (int t = 1; t < n_threads; t++) th.emplace_back(copy, t);
  copy(0);
  for (auto& x : th) x.join();
  uint64_t total = 0;
  for (auto n : counts) total += n;
  return total;
}
