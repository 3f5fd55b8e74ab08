// colblk_decode.hip — gfx950 decoder for batches of Pebble columnar (colblk)
// data blocks (colblk.DefaultKeySchema / cockroachkvs "crdb1").  One 256-thread
// workgroup per block in ticket order; per-block work in colblk_block.hip.h.
#include "common.hip.h"
#include "colblk_block.hip.h"

namespace pbl {
namespace col {

__global__ void __launch_bounds__(kTPB) colblk_decode_kernel(Args A) {
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
  hipLaunchKernelGGL(pbl::col::colblk_decode_kernel, dim3(batch->n_blocks), dim3(pbl::kTPB), 0, st, a);
  return hipGetLastError() == hipSuccess ? PBL_OK : PBL_DEVICE_ERROR;
}
