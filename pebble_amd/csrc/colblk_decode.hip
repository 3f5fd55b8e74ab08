// colblk_decode.hip — gfx950 decoder for Pebble columnar (colblk) data blocks.
// (filled in below the row decoder)
#include "common.hip.h"

extern "C" int pbl_decode_batch_colblk(const pbl_block_batch* batch, pbl_decode_out* out,
                                       void* stream) {
  (void)batch; (void)out; (void)stream;
  return PBL_UNSUPPORTED;
}
