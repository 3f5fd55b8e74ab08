// colblk_decode.hip — gfx950 decoder for batches of Pebble columnar (colblk)
// data blocks (colblk.DefaultKeySchema / cockroachkvs "crdb1").  One 256-thread
// workgroup per block in ticket order; per-block work in colblk_block.hip.h.
#include <algorithm>

#include "common.hip.h"
#include "colblk_block.hip.h"
#include "colblk_pipe.hip.h"
#include "colblk_wave.hip.h"

namespace pbl {
namespace col {

#ifndef PBL_COL_SINGLE_WAVES
#define PBL_COL_SINGLE_WAVES 7  // waves per SIMD (= workgroups per CU: 7 x 21.4 KB LDS); config 5 colblk 4: 433, 5: 524, 6: 643, 7: 690, 8: 466 GiB/s (64 VGPRs spill)
#endif
__global__ void __launch_bounds__(kTPB) __attribute__((amdgpu_waves_per_eu(PBL_COL_SINGLE_WAVES)))
colblk_decode_kernel(Args A) {
  __shared__ Lds s;
  __shared__ uint32_t ticket;
  uint32_t* ticket_ctr = reinterpret_cast<uint32_t*>(A.out.workspace);
  if (threadIdx.x == 0) ticket = atomicAdd(ticket_ctr, 1u);
  __syncthreads();
  col_block(s, A, ticket, A.in.format);
}

}  // namespace col
}  // namespace pbl

// Called by pbl_decode_batch (rowblk_decode.hip) once the arguments are checked
// and the totals are cleared, for a batch whose blocks are all colblk.
extern "C" int pbl_decode_batch_colblk(const pbl_block_batch* batch, pbl_decode_out* out, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (hipMemsetAsync(out->workspace, 0, pbl::ws_bytes(batch->n_blocks), st) != hipSuccess)
    return PBL_DEVICE_ERROR;
  pbl::Args a;
  a.in = *batch;
  a.out = *out;
  // default: the two-pass wave form (colblk_wave.hip.h): sizes, the bases
  // scan, then every block's outputs with no look-back.  HideObsoletePoints
  // (PBL_ROW_HIDE_OBSOLETE) is fused into the pipeline (colblk_pipe_kernel
  // <true>); PBL_KERNEL_PIPE / PBL_KERNEL_SINGLE force the pipeline / the
  // one-block-per-workgroup kernel (A/B).
  const uint32_t f = batch->flags;
  const bool hide = (f & PBL_ROW_HIDE_OBSOLETE) != 0;
  if (!hide && (f & PBL_KERNEL_SINGLE)) {
    hipLaunchKernelGGL(pbl::col::colblk_decode_kernel, dim3(batch->n_blocks), dim3(pbl::kTPB), 0, st, a);
  } else if (!hide && !(f & PBL_KERNEL_PIPE)) {
    int dev = 0, cus = 256;
    if (hipStreamGetDevice(st, &dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return PBL_DEVICE_ERROR;
    namespace cw = pbl::col::cwave;
    const uint32_t g_s = uint32_t(std::min<uint64_t>(batch->n_blocks, uint64_t(cus) * 4 * PBL_CW_SWAVES));
    const uint32_t nt = (batch->n_blocks + cw::kScanTile - 1) / cw::kScanTile;
    const uint32_t* no_ids = nullptr;
    hipLaunchKernelGGL((cw::colblk_wave_size_kernel<false, false>), dim3(g_s), dim3(pbl::kWave), 0, st, a, no_ids);
    hipLaunchKernelGGL(cw::bases_scan_kernel<false>, dim3(std::min<uint32_t>(nt, uint32_t(cus) * 2)), dim3(pbl::kTPB),
                       0, st, a);
    // variable-length blocks (config 5: one long values range each) read more
    // of their values from a larger stage
    if (f & PBL_BATCH_VARLEN)
      hipLaunchKernelGGL((cw::colblk_wave_emit_kernel<PBL_CW_STAGE_VARLEN, false>), dim3(batch->n_blocks),
                         dim3(pbl::kWave), 0, st, a, no_ids);
    else
      hipLaunchKernelGGL((cw::colblk_wave_emit_kernel<PBL_CW_STAGE, false>), dim3(batch->n_blocks), dim3(pbl::kWave),
                         0, st, a, no_ids);
  } else {
    const void* fn = hide ? reinterpret_cast<const void*>(pbl::col::cpipe::colblk_pipe_kernel<true>)
                          : reinterpret_cast<const void*>(pbl::col::cpipe::colblk_pipe_kernel<false>);
    const uint64_t grid = pbl::persistent_grid(st, hide ? pbl::kKColPipeHide : pbl::kKColPipe, fn, batch->n_blocks,
                                               nullptr);
    if (!grid) return PBL_DEVICE_ERROR;
    if (hide)
      hipLaunchKernelGGL(pbl::col::cpipe::colblk_pipe_kernel<true>, dim3(uint32_t(grid)), dim3(pbl::kTPB), 0, st, a);
    else
      hipLaunchKernelGGL(pbl::col::cpipe::colblk_pipe_kernel<false>, dim3(uint32_t(grid)), dim3(pbl::kTPB), 0, st, a);
  }
  return hipGetLastError() == hipSuccess ? PBL_OK : PBL_DEVICE_ERROR;
}
