// rowblk_general.hip.h — the general (non-LDS-fast-path) row-block decoder and
// the per-block metadata helpers shared by both paths.  Included by
// rowblk_decode.hip inside namespace pbl::row (needs Args, kTrailerObsoleteMask,
// kKindInvalid, kRestartMask).
#pragma once


// ---------------------------------------------------------------------------
// General path: a wave-serial restatement of Iter.First/Next (block bytes read
// through a generic pointer: LDS when staged, else global), current key in LDS.
// Executed by wave 0 only.
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
__device__ __noinline__ void slow_walk(const uint8_t* blk, uint64_t len, uint32_t flags, uint8_t* keybuf,
                          uint32_t keycap, int pass, const pbl_decode_out O, uint32_t b,
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


