// zstd.hip — Zstandard block decompression on the device.
//
// Pebble's zstd blocks (indicator 7) are a uvarint decoded length followed by
// Zstandard frames (internal/compression/zstd_cgo.go:45-66 Compress, :86-108
// DecompressInto via DataDog/zstd v1.5.7 = facebook/zstd 1.5.7): the frames
// must decode to exactly that length.  This decodes the published format (RFC
// 8878), restated on the CPU in oracle/zstd_oracle.c and checked against it:
// frame headers, skippable frames, raw / RLE / compressed blocks, literals
// (raw, RLE, Huffman with 1 or 4 streams, treeless), sequences (predefined /
// RLE / FSE / repeat tables), repeat offsets, the XXH64 content checksum.
//
// One wave per Pebble block (persistent grid over the batch):
//   * the compressed bytes are staged in LDS at their 16-B phase;
//   * the decoded block lives in an LDS window of the decoded length D.  Each
//     compressed zstd block's literals are decoded to the END of that window
//     ([D - regen, D)): sequence execution writes the output front-to-back and
//     never overtakes the literals it has not consumed yet (output so far =
//     literals consumed + match bytes, and the match bytes of a valid block
//     fit before D - regen), so literals and output share one buffer;
//   * headers and table descriptions are parsed with uniform control flow
//     (every lane reads the same bytes); FSE / Huffman tables are built by lane
//     0 (spread) and the wave (Huffman fill) into LDS;
//   * Huffman streams: lane s decodes stream s (1 or 4 lanes);
//   * sequences: lane 0 decodes up to kSeq sequences into LDS (a 64-bit bit
//     container refilled from LDS), then the wave executes them in order, each
//     literal run and match copied by all lanes (an overlapping match repeats
//     its period: byte i reads out[d - off + i % off]);
//   * the window is written out as aligned 16-B granules.
// Blocks whose compressed or decoded size exceeds the LDS buffers run the same
// code on global memory (inputs read in place, output written in place with
// workgroup fences between dependent copies).
#include <algorithm>

#include "common.hip.h"

#include "zstd_dec.hip.h"

namespace pbl {
namespace zstd {

__device__ inline bool uvarint32(gptr<const uint8_t> p, uint32_t n, uint32_t* v, uint32_t* used) {
  uint64_t x = 0;
  for (uint32_t i = 0; i < n && i < 10; i++) {
    x |= uint64_t(p[i] & 0x7f) << (7 * i);
    if (p[i] < 0x80) {
      if (x > 0xffffffffull) return false;
      *v = uint32_t(x);
      *used = i + 1;
      return true;
    }
  }
  return false;
}

}  // namespace zstd
}  // namespace pbl
#include "zstd_fast.hip.h"
namespace pbl {
namespace zstd {

// Every zstd block the batch path (zstd_fast.hip.h) did not take; `ws` is that
// path's workspace (null: every zstd block).
__global__ void __launch_bounds__(kWave) zstd_kernel(const pbl_phys_batch B, uint8_t* out, const uint64_t* out_off,
                                                     const uint32_t* out_cap, uint32_t* out_len, uint32_t* status,
                                                     const void* ws) {
  __shared__ Lds L;
  const uint32_t lane = lane_id();
  for (uint32_t b = blockIdx.x; b < B.n_blocks; b += gridDim.x) {
    const uint32_t n = to_glb(B.block_len)[b];
    const uint64_t boff = to_glb(B.block_off)[b];
    const gptr<const uint8_t> src = to_glb(B.bytes + boff);
    if (src[n] != PBL_COMPRESSION_ZSTD) continue;
    if (ws && to_glb(FastWs::at(const_cast<void*>(ws), B.n_blocks).desc)[b].fast) continue;  // zstd_exec_kernel's
    uint32_t st = PBL_OK, D = 0, used = 0;
    const uint32_t cap = to_glb(out_cap)[b];
    if (!uvarint32(src, n, &D, &used)) st = PBL_CORRUPT_COMPRESSION;
    else if (D > cap) st = PBL_OVERFLOW;
    else if (used == n || D == 0) st = PBL_CORRUPT_COMPRESSION;  // "empty src / dst buffer" (zstd_cgo.go:91-96)
    if (st == PBL_OK) {
      const uint32_t cn = n - used;
      uint8_t* dptr = out + to_glb(out_off)[b];
      uint32_t r;
      if (cn <= kIn && D <= kOut) {
        const uint64_t sa = reinterpret_cast<uint64_t>(B.bytes + boff + used);
        const uint32_t ssh = uint32_t(sa & 15), ng = (ssh + cn + 15) / 16;
        const gptr<const u32x4> sg = to_glb(reinterpret_cast<const u32x4*>(sa - ssh));
        lds_stage16(to_lds_ptr(reinterpret_cast<u32x4*>(L.in)), sg, ng);
        const uint64_t da = reinterpret_cast<uint64_t>(dptr);
        const uint32_t dsh = uint32_t(da & 15);
        r = decode_frames(L, LIn{to_lds_ptr(static_cast<const uint8_t*>(L.in))}, ssh, cn,
                          LOut{to_lds_ptr(static_cast<uint8_t*>(L.out)) + dsh}, D);
        if (r == kOk) {
          const uint32_t nd = (dsh + D + 15) / 16;
          const gptr<u32x4> dg = to_glb(reinterpret_cast<u32x4*>(da - dsh));
          const lptr<const u32x4> dl4 = to_lds_ptr(reinterpret_cast<const u32x4*>(L.out));
          for (uint32_t g = lane; g < nd; g += kWave) {
            const u32x4 v = dl4[g];
            const uint32_t lo = g == 0 ? dsh : 0u, hi = g + 1 == nd ? dsh + D - 16 * g : 16u;
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
        r = decode_frames(L, GIn{src}, used, cn, GOut{to_glb(dptr)}, D);
      }
      st = r == kOk ? PBL_OK : r == kUnsupported ? PBL_UNSUPPORTED : PBL_CORRUPT_COMPRESSION;
    }
    if (lane == 0) {
      to_glb(out_len)[b] = st == PBL_OK ? D : 0u;
      to_glb(status)[b] = st;
    }
    wave_sync();
  }
}

}  // namespace zstd

// Launched by pbl_decompress_blocks (physical.hip) after the snappy kernel: it
// handles exactly the blocks whose indicator is zstd.
// The batch path runs in a stream-ordered workspace (hipMallocAsync, freed on
// the stream after the last launch); without one (PBL_ZSTD_FAST=0 builds, or
// the allocation failing) zstd_kernel decodes every zstd block.
#ifndef PBL_ZSTD_FAST
#define PBL_ZSTD_FAST 1
#endif

hipError_t launch_zstd(const pbl_phys_batch& batch, uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                       uint32_t* out_len, uint32_t* status, hipStream_t st) {
  const uint32_t n = batch.n_blocks;
  void* ws = nullptr;
  if (PBL_ZSTD_FAST && hipMallocAsync(&ws, zstd::FastWs::bytes(n), st) != hipSuccess) {
    (void)hipGetLastError();
    ws = nullptr;
  }
  if (ws) {
    if (hipMemsetAsync(ws, 0, sizeof(zstd::WsHdr), st) != hipSuccess) {
      const hipError_t e = hipGetLastError();
      (void)hipFreeAsync(ws, st);
      return e;
    }
    hipLaunchKernelGGL(zstd::zstd_prep_kernel, dim3(std::min<uint32_t>(n, 8192)), dim3(kWave), 0, st, batch, out, out_off,
                       out_cap, ws);
    hipLaunchKernelGGL(zstd::zstd_lit_kernel, dim3((4ull * n + 255) / 256), dim3(256), 0, st, batch, out, out_off, ws);
    hipLaunchKernelGGL(zstd::zstd_seq_kernel, dim3((n + 255) / 256), dim3(256), 0, st, batch, ws);
    hipLaunchKernelGGL(zstd::zstd_exec_kernel, dim3(std::min<uint32_t>(n, 4096)), dim3(kWave), 0, st, batch, out,
                       out_off, out_len, status, ws);
  }
  const uint32_t grid = std::min<uint32_t>(n, 2048);
  hipLaunchKernelGGL(zstd::zstd_kernel, dim3(grid), dim3(kWave), 0, st, batch, out, out_off, out_cap, out_len, status,
                     static_cast<const void*>(ws));
  const hipError_t e = hipGetLastError();
  if (ws) (void)hipFreeAsync(ws, st);
  return e;
}

}  // namespace pbl

