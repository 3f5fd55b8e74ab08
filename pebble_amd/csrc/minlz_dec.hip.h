// minlz_dec.hip.h — MinLZ block decompression on the device (compression
// indicator 8: sstable/block/compression.go:192,229-230; internal/compression/
// minlz.go:52-72 calls minlz.Decode / minlz.DecodedLen).  Included by
// physical.hip inside namespace pbl::phys, after the snappy decoders.
//
// A block whose first byte is not 0 is a Snappy block (what the minlz
// compressor's Snappy fallback writes, minlz.go:21-27; the MinLZ decoder must
// decode it, minlz_test.go:31-36): the snappy kernels take those.  The rest,
// the MinLZ form, is decoded here: 0x00, a uvarint decoded length (0 = the
// remaining bytes are stored as is), then literal / repeat / copy1 / copy2 /
// fused-literal copy2 and copy3 ops (the format is restated op by op in
// oracle/minlz_oracle.c's header; the oracle decodes the same bytes).
//
//   minlz_kernel   one wave per block.  The compressed bytes are staged in LDS
//                  and the block is decoded LDS -> LDS by the wave (op headers
//                  read with uniform control flow, every lane parsing the same
//                  bytes; literals and long-offset copies 16 B per lane, short-
//                  offset copies byte per lane over the period), then written
//                  out as aligned 16-B granules.  Blocks past the stage decode
//                  on one lane from global memory.  Stored blocks are copied.
#pragma once

// (minlz_header and snappy_form sit in physical.hip, before the length kernel.)

// Decode the ops of one MinLZ block from input byte s0 (after the header) into
// dlen output bytes.  (lane, step): the wave's lanes (lane_id(), 64) or one
// lane alone (0, 1).  Returns whether the ops decode to exactly dlen bytes.
template <class Src, class Dst>
__device__ inline bool minlz_wave(Src src, uint32_t n, uint32_t s0, Dst dst, uint32_t dlen, uint32_t lane,
                                  uint32_t step) {
  uint32_t s = s0, d = 0, last = 1;
  bool ok = true;
  while (ok && s < n) {
    const uint32_t t = src[s];
    uint32_t lits = 0, lit = 0, len = 0, off = 0;
    const uint32_t kind = t & 3;
    if (kind == 0) {
      const uint32_t x = t >> 3;
      uint32_t l;
      if (x < 29) {
        l = x + 1;
        s += 1;
      } else {
        const uint32_t nb = x - 28;  // 1..3 length bytes
        if (s + 1 + nb > n) { ok = false; break; }
        l = 0;
        for (uint32_t i = 0; i < nb; i++) l |= uint32_t(src[s + 1 + i]) << (8 * i);
        l += 30;
        s += 1 + nb;
      }
      if (t & 4) {  // repeat: the last offset
        len = l;
        off = last;
      } else {
        lits = l;
      }
    } else if (kind == 1) {
      if (s + 2 > n) { ok = false; break; }
      off = ((t | uint32_t(src[s + 1]) << 8) >> 6) + 1;
      len = (t >> 2) & 15;
      s += 2;
      if (len == 15) {
        if (s + 1 > n) { ok = false; break; }
        len = 18 + src[s];
        s += 1;
      } else {
        len += 4;
      }
    } else if (kind == 2) {
      if (s + 3 > n) { ok = false; break; }
      const uint32_t l = t >> 2;
      off = (uint32_t(src[s + 1]) | uint32_t(src[s + 2]) << 8) + 64;
      s += 3;
      if (l <= 60) {
        len = l + 4;
      } else {
        const uint32_t nb = l - 60;
        if (s + nb > n) { ok = false; break; }
        len = 0;
        for (uint32_t i = 0; i < nb; i++) len |= uint32_t(src[s + i]) << (8 * i);
        len += 64;
        s += nb;
      }
    } else if (t & 4) {  // copy3, 0..3 literals first
      if (s + 4 > n) { ok = false; break; }
      const uint32_t v = t | uint32_t(src[s + 1]) << 8 | uint32_t(src[s + 2]) << 16 | uint32_t(src[s + 3]) << 24;
      lits = (v >> 3) & 3;
      const uint32_t l = (v >> 5) & 63;
      off = (v >> 11) + 65536;
      s += 4;
      if (l <= 60) {
        len = l + 4;
      } else {
        const uint32_t nb = l - 60;
        if (s + nb > n) { ok = false; break; }
        len = 0;
        for (uint32_t i = 0; i < nb; i++) len |= uint32_t(src[s + i]) << (8 * i);
        len += 64;
        s += nb;
      }
    } else {  // copy2 with 1..4 literals first
      if (s + 3 > n) { ok = false; break; }
      const uint32_t v = t | uint32_t(src[s + 1]) << 8 | uint32_t(src[s + 2]) << 16;
      lits = ((v >> 3) & 3) + 1;
      len = ((v >> 5) & 7) + 4;
      off = ((v >> 8) & 0xffff) + 64;
      s += 3;
    }
    if (lits) {
      if (lits > n - s || lits > dlen - d) { ok = false; break; }
      lit = s;
      s += lits;
      if constexpr (Src::kVec) {
        for (uint32_t i = 16 * lane; i < lits; i += 16 * step) dst.set16(d + i, src.get16(lit + i));
      } else {
        for (uint32_t i = lane; i < lits; i += step) dst.set(d + i, src[lit + i]);
      }
      wave_sync();
      d += lits;
    }
    if (len) {
      if (off == 0 || off > d || len > dlen - d) { ok = false; break; }
      if constexpr (Src::kVec) {
        // a chunk may write up to 15 bytes past the copy's end (rewritten by
        // later ops); a copy whose offset spans a whole step never reads what
        // the same step writes
        if (off >= 16 * kWave) {
          for (uint32_t i = 16 * lane; i < len; i += 16 * step) dst.set16(d + i, dst.get16(d - off + i));
        } else {
          for (uint32_t i = lane; i < len; i += step) dst.set(d + i, dst.get(d - off + (i % off)));
        }
      } else {
        for (uint32_t i = lane; i < len; i += step) dst.set(d + i, dst.get(d - off + (i % off)));
      }
      wave_sync();
      d += len;
      last = off;
    }
  }
  return ok && d == dlen;
}

__global__ void __launch_bounds__(kWave) minlz_kernel(const pbl_phys_batch B, uint8_t* out, const uint64_t* out_off,
                                                      const uint32_t* out_cap, uint32_t* out_len, uint32_t* status) {
  __shared__ SnapLds S;
  const uint32_t lane = lane_id();
  for (uint32_t b = blockIdx.x; b < B.n_blocks; b += gridDim.x) {
    const uint32_t n = to_glb(B.block_len)[b];
    const uint64_t boff = to_glb(B.block_off)[b];
    const gptr<const uint8_t> src = to_glb(B.bytes + boff);
    if (src[n] != PBL_COMPRESSION_MINLZ || snappy_form(PBL_COMPRESSION_MINLZ, src, n)) continue;
    if (!(B.flags & PBL_PHYS_MINLZ_NATIVE)) {  // the MinLZ form is opt-in (parity unpinned)
      if (lane == 0) {
        to_glb(out_len)[b] = 0;
        to_glb(status)[b] = PBL_UNSUPPORTED;
      }
      continue;
    }
    gptr<uint8_t> dst = to_glb(out + to_glb(out_off)[b]);
    const uint32_t cap = to_glb(out_cap)[b];
    uint32_t st = PBL_OK, dl = 0, hdr = 0;
    bool stored = false;
    if (n == 0 || !minlz_header(src, n, &dl, &hdr, &stored)) {
      st = PBL_CORRUPT_COMPRESSION;
    } else if (dl > cap) {
      st = PBL_OVERFLOW;
    } else if (stored) {
      for (uint32_t i = lane; i < dl; i += kWave) dst[i] = src[hdr + i];
    } else if (n <= kSnapCap && dl <= kSnapCap) {
      // stage the compressed bytes at their global 16-B phase, decode LDS ->
      // LDS, write the output as aligned 16-B granules
      const uint64_t sa = reinterpret_cast<uint64_t>(B.bytes + boff);
      const uint32_t ssh = uint32_t(sa & 15), ng = (ssh + n + 15) / 16;
      const gptr<const u32x4> sg = to_glb(reinterpret_cast<const u32x4*>(sa - ssh));
      lptr<u32x4> sl = to_lds_ptr(reinterpret_cast<u32x4*>(S.src4));
      for (uint32_t g = lane; g < ng; g += kWave) sl[g] = sg[g];
      const uint64_t da = reinterpret_cast<uint64_t>(out + to_glb(out_off)[b]);
      const uint32_t dsh = uint32_t(da & 15);
      lptr<uint8_t> sdst = to_lds_ptr(reinterpret_cast<uint8_t*>(S.dst4)) + dsh;
      wave_sync();
      const bool ok = minlz_wave(LdsBytes{to_lds_ptr(reinterpret_cast<uint8_t*>(S.src4)) + ssh}, n, hdr,
                                 LdsBytesW{sdst}, dl, lane, kWave);
      wave_sync();
      if (!ok) {
        st = PBL_CORRUPT_COMPRESSION;
      } else {
        const uint32_t nd = (dsh + dl + 15) / 16;
        const gptr<u32x4> dg = to_glb(reinterpret_cast<u32x4*>(da - dsh));
        const lptr<const u32x4> dl4 = to_lds_ptr(reinterpret_cast<const u32x4*>(S.dst4));
        for (uint32_t g = lane; g < nd; g += kWave) {
          const u32x4 v = dl4[g];
          const uint32_t lo = g == 0 ? dsh : 0u, hi = g + 1 == nd ? dsh + dl - 16 * g : 16u;
          if (lo == 0 && hi == 16) {
            dg[g] = v;
          } else {
            gptr<uint8_t> db = reinterpret_cast<gptr<uint8_t>>(dg + g);
            for (uint32_t k = lo; k < hi; k++) {
              const uint32_t w = k < 4 ? v.x : k < 8 ? v.y : k < 12 ? v.z : v.w;
              db[k] = uint8_t(w >> (8 * (k & 3)));
            }
          }
        }
      }
    } else {
      // large blocks: global -> global on one lane (program order makes every
      // earlier output byte visible to its own loads)
      uint32_t okl = 0;
      if (lane == 0) okl = minlz_wave(GlbBytes{src}, n, hdr, GlbBytesW{dst}, dl, 0, 1) ? 1u : 0u;
      if (!__shfl(okl, 0, kWave)) st = PBL_CORRUPT_COMPRESSION;
    }
    if (lane == 0) {
      to_glb(out_len)[b] = st == PBL_OK ? dl : 0u;
      to_glb(status)[b] = st;
    }
    wave_sync();
  }
}
