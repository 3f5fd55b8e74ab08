/*
 * pebble_amd.h — C-ABI of the MI355X-native Pebble SSTable data-block decoder.
 *
 * This is the drop-in boundary described in SURVEY.md §8(b).  A thin cgo shim
 * behind Pebble's `sstable/blockiter.Data` interface (or the Python host layer
 * in pebble_amd/) calls these entry points once per BATCH of data blocks; the
 * per-KV work runs in hand-written gfx950 HIP kernels.
 *
 * Reference interfaces replaced (paths relative to cockroachdb/pebble):
 *   pbl_decode_batch      rowblk.Iter.Init/First/Next  sstable/rowblk/rowblk_iter.go:241-276,1061-1087,1145-1201
 *                         colblk.DataBlockDecoder.Init sstable/colblk/data_block.go:1096-1109
 *                         colblk.DataBlockIter.Next    sstable/colblk/data_block.go:1662-1708
 *                         (driven by singleLevelIterator.loadDataBlock, sstable/reader_iter_single_lvl.go:485-547)
 *   pbl_rowblk_writer_*   rowblk.Writer                sstable/rowblk/rowblk_writer.go:48-320 (format producer)
 *   PBL_STATUS_*          base.CorruptionErrorf sites  sstable/rowblk/rowblk_iter.go:249-251,471-476;
 *                                                      sstable/colblk/data_block.go:1005-1009
 *
 * Conventions
 *   - Every pointer in pbl_block_batch / pbl_decode_out is a DEVICE pointer unless
 *     the field says otherwise.  The caller owns every buffer; the library never
 *     allocates or frees caller memory (mirrors block.BufferHandle ownership,
 *     sstable/blockiter/block_iter.go:76-81).
 *   - `stream` is a hipStream_t passed as void* (0 = legacy default stream).  All
 *     device entry points are stream-ordered and asynchronous; they never
 *     synchronise and are safe to capture into a hipGraph.
 *   - A launch runs on the device of its `stream` (hipStreamGetDevice), whatever
 *     the calling thread's current device.  The library is reentrant across
 *     streams and devices; its only process-wide state is a per-device cache of
 *     hardware properties (CU count, resident workgroups per kernel), written
 *     once.  Kernel choice depends only on the batch (format, flags), never on
 *     the environment.
 */
#ifndef PEBBLE_AMD_H
#define PEBBLE_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PBL_ABI_VERSION 8

/* ---- status codes (per block, and OR-ed as bit masks into totals) ---------- */
enum {
  PBL_OK = 0,
  PBL_CORRUPT_NO_RESTARTS = 1,   /* rowblk_iter.go:249-251 */
  PBL_CORRUPT_FIRST_KEY = 2,     /* rowblk_iter.go:429-434,471-476 */
  PBL_CORRUPT_BOUNDS = 3,        /* entry/column extends past the block */
  PBL_CORRUPT_COLBLK_HEADER = 4, /* data_block.go:1005-1009 (panic -> corruption) */
  PBL_UNSUPPORTED = 5,           /* legal but outside this build's limits */
  PBL_OVERFLOW = 6,              /* an output capacity was too small: nothing written */
  PBL_INVALID_ARG = 7,
  PBL_DEVICE_ERROR = 8,
  PBL_TIMEOUT = 9,               /* in-kernel look-back spin bound hit (never expected) */
  PBL_CORRUPT_CHECKSUM = 10,     /* block.go:177-195 "checksum mismatch"        */
  PBL_CORRUPT_COMPRESSION = 11,  /* snappy.ErrCorrupt -> base.MarkCorruptionError (block.go:550-565) */
  PBL_CORRUPT_FOOTER = 12,       /* parseFooter's CorruptionErrorf sites (sstable/table.go:328-404) */
  PBL_CORRUPT_INDEX = 13,        /* DecodeHandleWithProperties "invalid block.Handle" (block/block.go:94-104) */
  PBL_CORRUPT_VALUE_HANDLE = 14  /* valblk handle/index entry out of bounds (valblk/valblk.go:370-393,
                                    valblk/reader.go:280-302) */
};

/* ---- block formats ---------------------------------------------------------- */
enum {
  PBL_FMT_ROW = 0,          /* sstable/rowblk data block                          */
  PBL_FMT_COL_DEFAULT = 1,  /* colblk data block, colblk.DefaultKeySchema          */
  PBL_FMT_COL_CRDB1 = 2     /* colblk data block, cockroachkvs.KeySchema ("crdb1") */
};

/* batch flags */
#define PBL_ROW_VALUE_PREFIX 0x1u /* TableFormat >= Pebblev3: SET values carry a
                                     1-byte block.ValuePrefix (rowblk_iter.go:298-300) */
#define PBL_ROW_NO_VALUER 0x2u    /* iterator has no lazy valuer: strip the prefix
                                     byte even for handles (rowblk_iter.go:1195)   */
#define PBL_ROW_RAW_KEYS 0x4u     /* rowblk.RawIter semantics (rowblk_iter.go:1743-1794):
                                     keys are emitted whole, no trailer split, no
                                     first-key check; trailer[] = 0              */
#define PBL_ROW_HIDE_OBSOLETE 0x8u /* blockiter.Transforms.HideObsoletePoints fused into
                                     the decode (rowblk_iter.go:1168-1179; colblk
                                     data_block.go:1680-1697): KVs whose trailer has
                                     the obsolete bit (row) or whose isObsolete bit
                                     is set (colblk) are not emitted; every count and
                                     offset covers the visible KVs only, restart
                                     words are kept.  Row blocks ignore it with
                                     PBL_ROW_RAW_KEYS (a raw key has no trailer);
                                     colblk blocks always honour it.  Single-format
                                     and mixed (block_format) batches alike.  (The
                                     name is historical: it applies to colblk
                                     blocks too.)                                   */
#define PBL_COL_TIERING 0x10u     /* colblk blocks carry the Pebblev8 tiering columns
                                     (TableFormat.TieringColumnConfig, sstable/format.go:
                                     305-316: WithTieringColumns, data_block.go:594-601):
                                     the data columns tieringSpanID (Uint), tieringAttribute
                                     (Uint) and secondaryBlobHandle (RawBytes) follow
                                     isObsolete (data_block.go:514-525).  With it, every
                                     colblk KV's KVMeta -- what DataBlockIter.FirstWithMeta
                                     / NextWithMeta / SeekGEWithMeta return
                                     (data_block.go:1574-1641) -- is written to
                                     pbl_decode_out.tiering_span_id / tiering_attr when
                                     those are non-NULL, and the two Uint columns are
                                     decoded with DecodeColumn's checks (a block missing
                                     them, or failing them, is PBL_CORRUPT_COLBLK_HEADER:
                                     the reference panics in initTieringMetadata).
                                     Without it the meta arrays, when given, receive
                                     zeros (KVMeta{}: !SupportsTiering).  Row blocks
                                     always give zeros (rowblk.Iter has no meta columns;
                                     NextWithMeta on the row iterator returns KVMeta{}).
                                     Keys and values decode identically either way.   */
#define PBL_BATCH_VARLEN 0x100u   /* scheduling hint, no effect on results: block
                                     lengths vary widely (e.g. Zipf value sizes).
                                     colblk batches read more of each block's
                                     values from LDS; row batches take the
                                     two-pass form (lane-per-block size walk, bases
                                     scan, wave-per-block emit from LDS, no
                                     look-back) unless HideObsoletePoints or value
                                     prefixes need key bytes to size a block.  Set
                                     it for row batches of value-dominated blocks
                                     (few entries per block); blocks of many small
                                     KVs decode faster without it.  The caller
                                     knows the lengths on the host (block handles
                                     carry them); the Python layer also samples
                                     entry counts (batch.varlen_hint).             */
#define PBL_KERNEL_SINGLE 0x200u  /* A/B measurement, no effect on results: colblk
                                     batches on the one-block-per-workgroup kernel
                                     instead of the two-pass wave form (row
                                     batches ignore it)                            */
#define PBL_KERNEL_PIPE 0x400u    /* A/B measurement, no effect on results: colblk
                                     batches on the persistent pipeline instead of
                                     the two-pass wave form (row batches ignore
                                     it)                                           */
/* 0x800u, 0x1000u, 0x2000u, 0x8000u: retired A/B kernels (one-wave-per-block
   flat, run-major, HBM-walking and block-resident row kernels; removed, the
   bits are ignored)                                                            */
#define PBL_KERNEL_POOL 0x4000u   /* A/B measurement, no effect on results: row
                                     batches on the staging-pool kernel
                                     (rowblk_pool.hip.h, the default without
                                     PBL_BATCH_VARLEN) even with PBL_BATCH_VARLEN  */

/* per-KV flag byte (kv_flags[]) */
#define PBL_KV_RESTART 0x01u       /* entry offset is a restart point            */
#define PBL_KV_RESTART_SAMEPFX 0x02u /* restart word bit 31 (setHasSameKeyPrefix) */
#define PBL_KV_OBSOLETE 0x04u      /* trailer had InternalKeyKindSSTableInternalObsoleteBit */
#define PBL_KV_INVALID_KEY 0x08u   /* key < 8 bytes: kind Invalid, nil user key   */
#define PBL_KV_VALBLK_HANDLE 0x10u /* value bytes are prefix+valblk.Handle        */
#define PBL_KV_BLOB_HANDLE 0x20u   /* value bytes are prefix+blob handle / colblk external */
#define PBL_KV_PREFIX_CHANGED 0x40u /* colblk prefixChanged bit                   */
/* colblk rows: OBSOLETE = isObsolete bit (data_block.go:519); an isValueExternal
   row (data_block.go:1700-1704) is VALBLK_HANDLE or BLOB_HANDLE by its first
   (value-prefix) byte, and its value bytes are the raw column slice; the
   trailer is trailers.At(row) unmasked; entry_off[] is the row index. */

/* ---- batch descriptor ------------------------------------------------------- */
typedef struct pbl_block_batch {
  const uint8_t* blocks;     /* concatenated, already-decompressed block bytes (no 5 B
                                physical trailer).  Must be readable up to the next
                                16-byte boundary after every block.                 */
  const uint64_t* block_off; /* [n_blocks] byte offset of each block in `blocks`    */
  const uint32_t* block_len; /* [n_blocks] byte length of each block (< 4 GiB: the
                                rowblk 64-bit offsets of rowblk_64bit_test.go:28-183
                                are out of scope; blocks are <= 32 KiB in practice
                                and the general path handles any u32 length)      */
  uint32_t n_blocks;
  uint32_t format;           /* PBL_FMT_* for every block of the batch              */
  uint32_t flags;            /* PBL_ROW_* flags                                     */
  uint32_t reserved;
  const uint8_t* block_format; /* optional [n_blocks] PBL_FMT_* per block (mixed
                                row + colblk batches); NULL = `format` for all   */
  uint64_t synthetic_seq_num;  /* blockiter.SyntheticSeqNum fused into the decode
                                (transforms.go:90-99; 0 = unset, < 2^56): every
                                decodable key's trailer becomes seq << 8 | kind
                                (rowblk_iter.go:1168-1191, data_block.go:1693-
                                1695); invalid row keys keep the Invalid trailer;
                                ignored with PBL_ROW_RAW_KEYS                    */
} pbl_block_batch;

/* ---- batch totals (device struct, written by the decode kernel) -------------- */
typedef struct pbl_totals {
  uint64_t n_kv;        /* KVs decoded over all blocks                         */
  uint64_t key_bytes;   /* user-key bytes                                      */
  uint64_t val_bytes;   /* value bytes                                         */
  uint64_t n_restarts;  /* restart words (row format)                          */
  uint32_t status_mask; /* OR of (1u << status) over blocks with status != OK  */
  uint32_t n_bad_blocks;/* blocks whose status != PBL_OK                       */
  uint32_t n_slow_blocks;/* blocks decoded by the general (non-LDS) path      */
  uint32_t pad;
} pbl_totals;

/*
 * Output arrays (all caller-allocated, device).  Indexing for block b, KV j:
 *   kv  = blk_kv_base[b] + j                (per-KV arrays)
 *   o   = blk_kv_base[b] + b + j, j<=nkv_b  (per-block N+1 offset arrays)
 * key j of block b  = key_bytes[blk_key_base[b] + key_off[o] .. + key_off[o+1])
 * value j of block b= val_bytes[blk_val_base[b] + val_off[o] .. + val_off[o+1])
 * restart r of b    = restarts[blk_rst_base[b] + r]  (raw LE32 word, bit 31 kept)
 * Optional arrays may be NULL.  The blk_*_base arrays have n_blocks+1 entries; the
 * last entry holds the batch total.  When a capacity is exceeded the kernel still
 * computes every size (totals, blk_*_base) but writes no bytes, and reports
 * PBL_OVERFLOW: re-run with larger buffers.
 */
typedef struct pbl_decode_out {
  uint64_t* trailer;      /* [kv_cap] base.InternalKeyTrailer (obsolete bit cleared) */
  uint8_t* kv_flags;      /* [kv_cap] PBL_KV_* (optional)                        */
  uint32_t* entry_off;    /* [kv_cap] KVEncoding.Offset of each row entry (optional) */
  uint32_t* key_off;      /* [kv_cap + n_blocks] block-relative key offsets       */
  uint32_t* val_off;      /* [kv_cap + n_blocks] block-relative value offsets     */
  uint8_t* key_bytes;     /* [key_cap]                                            */
  uint8_t* val_bytes;     /* [val_cap]                                            */
  uint32_t* restarts;     /* [rst_cap] raw restart words (optional, row format)   */
  uint64_t* blk_kv_base;  /* [n_blocks+1]                                         */
  uint64_t* blk_key_base; /* [n_blocks+1]                                         */
  uint64_t* blk_val_base; /* [n_blocks+1]                                         */
  uint64_t* blk_rst_base; /* [n_blocks+1] (optional)                              */
  uint32_t* blk_status;   /* [n_blocks] PBL_* status per block                    */
  pbl_totals* totals;     /* [1]                                                  */
  uint64_t kv_cap, key_cap, val_cap, rst_cap;
  void* workspace;        /* device scratch of pbl_workspace_bytes(n_blocks) bytes */
  uint64_t workspace_bytes;
  uint64_t* tiering_span_id; /* [kv_cap] (optional) base.KVMeta.TieringSpanID per KV   */
  uint64_t* tiering_attr;    /* [kv_cap] (optional) base.KVMeta.TieringAttribute per KV;
                                both or neither; see PBL_COL_TIERING                  */
} pbl_decode_out;

/* ABI version of the loaded library (== PBL_ABI_VERSION). */
int pbl_abi_version(void);

/* Device scratch the decode needs for a batch of n_blocks (look-back state). */
uint64_t pbl_workspace_bytes(uint32_t n_blocks);

/*
 * Decode every block of `batch` into `out` on `stream`: one stream-ordered
 * single-pass launch (plus a memset of the workspace).  Returns PBL_OK or
 * PBL_INVALID_ARG / PBL_DEVICE_ERROR for launch problems; per-block corruption is
 * reported in out->blk_status and out->totals (read them after the stream syncs).
 */
int pbl_decode_batch(const pbl_block_batch* batch, pbl_decode_out* out, void* stream);

/*
 * Size pass: the same parse as pbl_decode_batch, writing only
 * the per-block results: blk_{kv,key,val,rst}_base (n_blocks+1 entries, the last
 * = batch totals), blk_status and totals.  Only those arrays, `totals` and the
 * workspace are required in `out`; every other pointer and capacity is ignored
 * and nothing else is written.  A caller without exact sizes runs this, then
 * pbl_decode_batch into exactly sized buffers (instead of guessing capacities
 * and re-running on PBL_OVERFLOW).  Statuses are those pbl_decode_batch reports,
 * PBL_OVERFLOW excepted.
 */
int pbl_size_batch(const pbl_block_batch* batch, pbl_decode_out* out, void* stream);

/*
 * Layout of the ABI structs as this library was compiled, for binding checks
 * (ctypes, cgo): writes up to `cap` u64 values and returns how many it has:
 *   sizeof(pbl_block_batch), the offsets of its 9 fields in declaration order,
 *   sizeof(pbl_totals), the offsets of its 8 fields,
 *   sizeof(pbl_decode_out), the offsets of its 22 fields,
 *   then likewise pbl_transforms, pbl_footer, pbl_index_out, pbl_kv_out,
 *   pbl_value_out, pbl_kv and pbl_kv_meta (sizeof, then every field's offset in
 *   declaration order).
 */
size_t pbl_struct_layout(uint64_t* out, size_t cap);

/*
 * Offset concat for a sharded batch: add this rank's global
 * bases (exclusive prefix over lower ranks of n_kv / key_bytes / val_bytes /
 * n_restarts, all-gathered over RCCL) to the n_blocks+1 entries of each
 * blk_*_base array.  Per-KV offsets are block-relative and never need rebasing.
 */
int pbl_rebase_blocks(pbl_decode_out* out, uint32_t n_blocks, uint64_t kv_base,
                      uint64_t key_base, uint64_t val_base, uint64_t rst_base,
                      void* stream);


/*
 * Same offset concat, fully stream-ordered: `rank_totals` is the DEVICE array of
 * world*4 u64 {n_kv, key_bytes, val_bytes, n_restarts} per rank exactly as an
 * RCCL all-gather of each rank's pbl_totals prefix leaves it; the kernel forms
 * this rank's exclusive prefix itself (no host round trip).
 */
int pbl_offset_concat(pbl_decode_out* out, uint32_t n_blocks, const uint64_t* rank_totals,
                      uint32_t rank, void* stream);

/* ---- physical blocks: checksums and decompression --------- */
/* Blocks as they sit in an SST: [block bytes][compression indicator u8][checksum
 * LE32] (sstable/block/block.go:539-571); block_len is the block.Handle length
 * (the 5-byte trailer follows it).  The kernels read in aligned 16-B granules:
 * `bytes` must stay readable for 16 bytes past every block's trailer (an SST
 * file's own following bytes, or 16 bytes of padding after the buffer). */
typedef struct pbl_phys_batch {
  const uint8_t* bytes;      /* DEVICE bytes                                           */
  const uint64_t* block_off; /* [n_blocks] DEVICE offset of each block in `bytes`        */
  const uint32_t* block_len; /* [n_blocks] DEVICE block.Handle.Length (trailer excluded) */
  uint32_t n_blocks;
  uint32_t flags;            /* PBL_PHYS_* (0: the defaults)                           */
} pbl_phys_batch;
/* MinLZ blocks in the MinLZ form (first byte 0, internal/compression/minlz.go:
   52-72) are decoded on the device only with this flag: the format is restated
   without bytes from the real encoder to pin it (github.com/minio/minlz is an
   absent dependency), so by default such blocks report
   PBL_UNSUPPORTED and the caller decodes them on the host.  MinLZ blocks in
   the Snappy form (minlz_test.go:31-36) are always decoded.                    */
#define PBL_PHYS_MINLZ_NATIVE 0x1u
enum { /* block.ChecksumType (block.go:106-114) */
  PBL_CHECKSUM_NONE = 0, PBL_CHECKSUM_CRC32C = 1, PBL_CHECKSUM_XXHASH = 2, PBL_CHECKSUM_XXHASH64 = 3
};
enum { /* block.CompressionIndicator (compression.go:170-193) */
  PBL_COMPRESSION_NONE = 0, PBL_COMPRESSION_SNAPPY = 1, PBL_COMPRESSION_ZSTD = 7, PBL_COMPRESSION_MINLZ = 8
};

/*
 * ValidateChecksum (block.go:164-197) for every block: status[b] = PBL_OK or
 * PBL_CORRUPT_CHECKSUM; computed[b] (optional) = the checksum computed over the
 * block bytes and the indicator byte.  CRC32C (internal/crc: Castagnoli, then
 * Value()'s rotation and delta) or XXH64 truncated to 32 bits; other types return
 * PBL_UNSUPPORTED.
 */
int pbl_verify_checksums(const pbl_phys_batch* batch, uint32_t checksum_type, uint32_t* status, uint32_t* computed,
                         void* stream);
/*
 * Decompressor.DecompressedLen (block.go:549-556) of every block: out_len[b];
 * status[b] = PBL_OK, PBL_CORRUPT_COMPRESSION or PBL_UNSUPPORTED (the legacy
 * codecs are not decoded on the device).  Snappy: its uvarint header; zstd: the
 * uvarint Pebble prefixes (zstd_cgo.go:111-119); MinLZ: minlz.DecodedLen
 * (internal/compression/minlz.go:70-73; a block in the Snappy form, first byte
 * not 0, by its Snappy header).
 */
int pbl_decompressed_lengths(const pbl_phys_batch* batch, uint32_t* out_len, uint32_t* status, void* stream);
/*
 * DecompressInto (block.go:557-565): block b's decoded bytes at out + out_off[b]
 * (out_cap[b] bytes available; DEVICE arrays), its length in out_len[b] and
 * status[b] = PBL_OK / PBL_CORRUPT_COMPRESSION / PBL_OVERFLOW / PBL_UNSUPPORTED.
 * Uncompressed blocks are copied; snappy (golang/snappy block format) and zstd
 * (RFC 8878 frames after Pebble's uvarint length, zstd_cgo.go:86-108: the frames
 * must decode to exactly that length; a frame naming a dictionary is
 * PBL_UNSUPPORTED) are decoded on the device.  The outputs form a pbl_block_batch {out,
 * out_off, out_len} for pbl_decode_batch (keep out_off 8-B aligned for colblk).
 * zstd's batch path takes a stream-ordered workspace (hipMallocAsync on `stream`,
 * ~40 KB per block, freed on the stream after its last launch); when that
 * allocation fails every zstd block takes the one-wave-per-block decoder instead.
 */
int pbl_decompress_blocks(const pbl_phys_batch* batch, uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                          uint32_t* out_len, uint32_t* status, void* stream);

/* ---- table footer and index blocks ------------------------ */
enum { /* TableFormat (sstable/format.go:20-60); the footer's (magic, version) */
  PBL_TABLE_LEVELDB = 1, PBL_TABLE_ROCKSDBV2 = 2,
  PBL_TABLE_PEBBLEV1 = 3, PBL_TABLE_PEBBLEV2 = 4, PBL_TABLE_PEBBLEV3 = 5, PBL_TABLE_PEBBLEV4 = 6,
  PBL_TABLE_PEBBLEV5 = 7, PBL_TABLE_PEBBLEV6 = 8, PBL_TABLE_PEBBLEV7 = 9, PBL_TABLE_PEBBLEV8 = 10
};
typedef struct pbl_footer {
  uint32_t table_format;   /* PBL_TABLE_*                                               */
  uint32_t checksum_type;  /* PBL_CHECKSUM_* of every block of the table                */
  uint64_t metaindex_off, metaindex_len;
  uint64_t index_off, index_len;  /* the (top-level) index block's handle             */
  uint64_t footer_off, footer_len;
  uint32_t attributes;     /* Pebblev7+ attribute bitset, else 0                        */
  uint32_t reserved;
} pbl_footer;
/*
 * parseFooter (sstable/table.go:328-404) on HOST memory: `buf` holds the last
 * buf_len bytes of a file of file_size bytes (readFooter reads the last
 * maxFooterLen = 61 bytes).  LevelDB, RocksDBv2 and Pebblev1-v8 footers; the
 * Pebblev6+ footer checksum (CRC32C Value) is verified.  Returns PBL_OK or
 * PBL_CORRUPT_FOOTER (bad magic, unsupported version or checksum type, short
 * footer, checksum mismatch, handles past the end of the file).
 */
int pbl_parse_footer(const uint8_t* buf, uint64_t buf_len, uint64_t file_size, pbl_footer* out);

typedef struct pbl_index_out {
  uint64_t* handle_off;  /* [cap] block.Handle.Offset of each entry, in block order              */
  uint64_t* handle_len;  /* [cap] block.Handle.Length                                             */
  uint64_t* props_off;   /* [cap] (nullable) where the entry's block-property bytes start: in the
                            decoded val_bytes (row) or in the batch's block bytes (colblk)         */
  uint32_t* props_len;   /* [cap] (nullable)                                                      */
  uint64_t* blk_base;    /* [n_blocks + 1] first entry of each index block; [n_blocks] = total    */
  uint32_t* blk_status;  /* [n_blocks] PBL_OK / PBL_CORRUPT_INDEX / PBL_CORRUPT_COLBLK_HEADER /
                            PBL_OVERFLOW (or the row decode's status)                             */
  uint64_t cap;          /* entries the handle arrays hold                                         */
} pbl_index_out;
/*
 * rowblk.IndexIter.BlockHandleWithProperties (rowblk/rowblk_index_iter.go:82-84)
 * for every entry of a batch of row-format index blocks that pbl_decode_batch
 * (flags 0) has decoded into `decoded`: entry k's value at
 * val_bytes[blk_val_base[b] + val_off[..]] through block.DecodeHandleWithProperties
 * (block/block.go:80-104: uvarint offset, uvarint length, the rest = properties).
 * Entry k of the handle arrays is KV k of `decoded` (blk_base = blk_kv_base).  A
 * value that is not a handle makes its block PBL_CORRUPT_INDEX.
 */
int pbl_index_handles_row(const pbl_decode_out* decoded, uint32_t n_blocks, pbl_index_out* out, void* stream);
/*
 * colblk.IndexIter over a batch of columnar index blocks (colblk/index_block.go:
 * IndexBlockDecoder.Init :150-156, BlockHandleWithProperties :310-321):
 * separators RawBytes, offsets and lengths Uint, block properties RawBytes;
 * column layout checks as for data blocks (PBL_CORRUPT_COLBLK_HEADER).  Blocks
 * are sized first (blk_base), then written; a total past cap reports
 * PBL_OVERFLOW for the blocks that do not fit and writes none of their entries.
 */
int pbl_index_handles_col(const pbl_block_batch* batch, pbl_index_out* out, void* stream);

typedef struct pbl_kv_out {
  uint64_t* key_off;     /* [cap] where KeyAt(i) starts in the batch's block bytes      */
  uint32_t* key_len;     /* [cap]                                                        */
  uint64_t* val_off;     /* [cap] where ValueAt(i) starts in the batch's block bytes    */
  uint32_t* val_len;     /* [cap]                                                        */
  uint64_t* blk_base;    /* [n_blocks + 1] first entry of each block; [n_blocks] = total */
  uint32_t* blk_status;  /* [n_blocks] PBL_OK / PBL_CORRUPT_COLBLK_HEADER /
                            PBL_CORRUPT_BOUNDS / PBL_OVERFLOW                            */
  uint64_t cap;          /* entries the arrays hold                                       */
} pbl_kv_out;
/*
 * colblk.KeyValueBlockDecoder (colblk/key_value_block.go:76-89) over a batch of
 * key-value blocks -- the metaindex of Pebblev6+ tables and the properties
 * block of Pebblev7+ tables (sstable/reader.go:536-545,601-617;
 * layout.go:789-824): no custom header, column 0 the keys and column 1 the
 * values (RawBytes).  Every row's key and value are reported as slices of the
 * batch's bytes (zero-copy, as KeyAt / ValueAt).  Column layout checks as for
 * data blocks; a slice past its block is PBL_CORRUPT_BOUNDS.  Sized, scanned,
 * then written; a total past cap reports PBL_OVERFLOW for the blocks that do
 * not fit.
 */
int pbl_kv_blocks(const pbl_block_batch* batch, pbl_kv_out* out, void* stream);

/*
 * The value-block index (valblk/valblk.go:338-393) on the device: `vbi` holds
 * the decompressed index block (vbi_len bytes, DEVICE memory), rows of
 * num_w + off_w + len_w little-endian bytes (valblk.IndexHandle widths, each
 * 1..8).  Writes the handle of value block i to handle_off[i] / handle_len[i]
 * for i < min(rows, cap) and *n_blocks = rows (DEVICE u32; rows = vbi_len / row
 * width).  *status (DEVICE u32) = PBL_OK, or PBL_CORRUPT_VALUE_HANDLE when a
 * row's block number is not its index, the block has a partial row, or a
 * width is 0 or > 8 (DecodeIndex's errors).
 */
int pbl_valblk_index(const uint8_t* vbi, uint64_t vbi_len, uint32_t num_w, uint32_t off_w, uint32_t len_w,
                     uint64_t* handle_off, uint64_t* handle_len, uint32_t cap, uint32_t* n_blocks,
                     uint32_t* status, void* stream);

typedef struct pbl_value_out {
  uint32_t* val_off;     /* [kv_cap + n_blocks] block-relative value offsets (as pbl_decode_out) */
  uint8_t* val_bytes;    /* [val_cap]                                                            */
  uint64_t* blk_val_base;/* [n_blocks + 1]; [n_blocks] = total                                   */
  uint32_t* blk_status;  /* [n_blocks] the decode's status, else PBL_OK /
                            PBL_CORRUPT_VALUE_HANDLE / PBL_OVERFLOW                              */
  uint64_t val_cap;
} pbl_value_out;
/*
 * Resolve value-block handles (valueBlockFetcher.Fetch, valblk/reader.go:251-302)
 * for every KV of a decoded batch: a KV whose kv_flags has PBL_KV_VALBLK_HANDLE
 * holds the value prefix byte + valblk.Handle (uvarint ValueLen, BlockNum,
 * OffsetInBlock; valblk.go:218-279); its value becomes
 * value_blocks[BlockNum][OffsetInBlock : OffsetInBlock + ValueLen] of the
 * batch of (decompressed) value blocks.  Every other value is copied as is
 * (blob handles stay handles, as a reader without blob files reports them).
 * `decoded` needs kv_flags, val_off, val_bytes, blk_kv_base, blk_val_base and
 * blk_status.  A handle past its value block, or naming a block past the
 * batch, makes its block PBL_CORRUPT_VALUE_HANDLE.  Sized, scanned, then
 * written; a total past val_cap reports PBL_OVERFLOW for the blocks that do
 * not fit.
 */
int pbl_resolve_values(const pbl_decode_out* decoded, uint32_t n_blocks, const pbl_block_batch* value_blocks,
                       pbl_value_out* out, void* stream);

/* ---- blockiter.Transforms on the device ------------------ */
/* Comparer.Split used to find the suffix a SyntheticSuffix replaces. */
enum {
  PBL_SPLIT_WHOLE = 0,    /* base.DefaultSplit: no suffix (internal/base/comparer.go:206-208) */
  PBL_SPLIT_TESTKEYS = 1, /* testkeys.Comparer: before the last '@' (internal/testkeys/testkeys.go:144-150) */
  PBL_SPLIT_CRDB = 2      /* cockroachkvs.Split: last byte = version length (cockroachkvs/cockroachkvs.go:298-309) */
};
typedef struct pbl_transforms {
  uint64_t synthetic_seq_num;    /* blockiter.SyntheticSeqNum; 0 = unset (transforms.go:90-99) */
  uint32_t hide_obsolete_points; /* drop PBL_KV_OBSOLETE KVs (transforms.go:24-27)            */
  uint32_t split;                /* PBL_SPLIT_* (only used with a suffix)                     */
  const uint8_t* prefix;         /* DEVICE bytes of the SyntheticPrefix (transforms.go:120-162) */
  const uint8_t* suffix;         /* DEVICE bytes of the SyntheticSuffix (transforms.go:101-118) */
  uint32_t prefix_len, suffix_len;
  const pbl_block_batch* blocks; /* REQUIRED: the batch `in` was decoded from (host struct,
                                    device arrays).  Row blocks are read by rowblk.Iter
                                    with the prefix inside fullKey (rowblk_iter.go:259-263,
                                    400): a key shorter than 8 B is re-read from its block
                                    and decodes as a valid key when prefix ++ key is 8 B or
                                    longer (:1168-1199), and Split runs on prefix ++ key
                                    (:1183).  Colblk blocks follow their KeySeeker
                                    (data_block.go:444-460; cockroachkvs.go:1073-1089).     */
} pbl_transforms;

/* Device scratch pbl_transform_batch needs in out->workspace. */
uint64_t pbl_transform_workspace_bytes(uint32_t n_blocks);

/*
 * Apply `t` to a decoded batch (`in`, as pbl_decode_batch left it, n_blocks
 * blocks) into `out` (same layout contract; caller-allocated; out->workspace of
 * pbl_transform_workspace_bytes): every visible KV (HideObsoletePoints drops the
 * obsolete ones) keeps its order, flags, entry offset, KVMeta (tiering_span_id /
 * tiering_attr, copied when both `in` and `out` carry them) and value; its trailer
 * takes the synthetic sequence number (InternalKey.SetSeqNum); its user key
 * becomes F[:Split(F)] ++ suffix (suffix set) or F, F = prefix ++ key (row
 * blocks; colblk: prefix ++ key[:Split(key)] ++ suffix); keys of entries that
 * stay PBL_KV_INVALID_KEY are empty and keep the Invalid trailer.  Restart words
 * are the input's; statuses too, except a row block whose transformed iteration
 * would panic (a key made valid by the prefix, kind SET, empty value, value
 * prefix on): PBL_CORRUPT_BOUNDS.  A block whose decode failed stays failed.
 * Keys and values are copied in 16-byte chunks: in->key_bytes, in->val_bytes,
 * t->prefix and t->suffix must be readable 16 bytes past their capacity /
 * length (pebble_amd's allocations pad them).  A workspace memset and three
 * stream-ordered launches (count; scan: tiles of 1024 blocks with decoupled
 * look-back; scatter); on a capacity overflow every decodable block reports
 * PBL_OVERFLOW and only sizes are written.  Replaces the iteration-time transforms of rowblk.Iter
 * (rowblk_iter.go:400,487-517,1168-1187) and colblk.DataBlockIter
 * (data_block.go:1299-1303,1437-1462,1680-1697) for a whole batch.
 */
int pbl_transform_batch(const pbl_decode_out* in, uint32_t n_blocks, const pbl_transforms* t, pbl_decode_out* out,
                        void* stream);

/* ---- rowblk.Writer (format producer; host memory) ---------------------------- */
typedef struct pbl_rowblk_writer pbl_rowblk_writer;
pbl_rowblk_writer* pbl_rowblk_writer_new(int restart_interval);
void pbl_rowblk_writer_free(pbl_rowblk_writer* w);
void pbl_rowblk_writer_reset(pbl_rowblk_writer* w, int restart_interval);
/* rowblk_writer.go:263-286.  `trailer` is base.InternalKeyTrailer. */
int pbl_rowblk_writer_add(pbl_rowblk_writer* w, const uint8_t* user_key, size_t user_key_len,
                          uint64_t trailer, int is_obsolete, const uint8_t* value,
                          size_t value_len, int64_t max_shared_key_len, int add_value_prefix,
                          uint8_t value_prefix, int set_has_same_key_prefix);
/* rowblk_writer.go:323-334 (raw key, no trailer). */
int pbl_rowblk_writer_add_raw(pbl_rowblk_writer* w, const uint8_t* key, size_t key_len,
                              const uint8_t* value, size_t value_len);
size_t pbl_rowblk_writer_estimated_size(const pbl_rowblk_writer* w);
size_t pbl_rowblk_writer_entry_count(const pbl_rowblk_writer* w);
/* Finish; copies the block into `dst` if dst_cap suffices; returns the block size. */
size_t pbl_rowblk_writer_finish(pbl_rowblk_writer* w, uint8_t* dst, size_t dst_cap);

/*
 * Synthetic batch generator (host memory, multithreaded), SURVEY.md §8(d):
 * key of row r = BE64(r) || BE64(splitmix64(seed ^ r)) (key_len 16; longer keys
 * append splitmix bytes), row r = (block << 20) + k, trailer MakeTrailer(r, SET),
 * value bytes from splitmix64(seed + r).  Each block is filled while
 * EstimatedSize()+entry <= block_size and is placed at a fixed `block_size`
 * stride in `dst` (dst must hold n_blocks*block_size bytes).  Fills
 * block_off/block_len (host arrays) and returns total KVs.  Block content
 * depends only on (seed, global block index).
 */
uint64_t pbl_gen_row_blocks(uint64_t seed, uint32_t n_blocks, uint32_t block_size,
                            int restart_interval, uint32_t key_len, uint32_t val_len,
                            int value_prefix, uint8_t* dst, uint64_t* block_off,
                            uint32_t* block_len, int n_threads);
/* The same from global block `first_block` on (output block i = global block
 * first_block + i: a rank's shard of one global batch), with obsolete points
 * (HideObsoletePoints measurements): key k of a block carries the trailer's
 * obsolete bit when obsolete_every > 0 and k % obsolete_every ==
 * obsolete_every - 1 (rowblk_writer.go:30-42).                              */
uint64_t pbl_gen_row_blocks_obs(uint64_t seed, uint32_t first_block, uint32_t n_blocks, uint32_t block_size,
                                int restart_interval, uint32_t key_len, uint32_t val_len,
                                int value_prefix, uint32_t obsolete_every, uint8_t* dst,
                                uint64_t* block_off, uint32_t* block_len, int n_threads);

/* ---- colblk.DataBlockEncoder (format producer; host memory) ------------------ */
/*
 * sstable/colblk/data_block.go:600-790 with colblk.DefaultKeySchema
 * (schema PBL_FMT_COL_DEFAULT, key prefix = bytes before the first '@', the
 * testkeys comparer; data_block.go:207-345) or cockroachkvs.KeySchema
 * (PBL_FMT_COL_CRDB1, cockroachkvs/cockroachkvs.go:505-766).
 */
typedef struct pbl_colblk_writer pbl_colblk_writer;
pbl_colblk_writer* pbl_colblk_writer_new(uint32_t schema, int bundle_size);
void pbl_colblk_writer_free(pbl_colblk_writer* w);
void pbl_colblk_writer_reset(pbl_colblk_writer* w);
/* Add one KV (DataBlockEncoder.Add after KeyWriter.ComparePrev).  prefix_len < 0
 * = the schema's Split.  value_kind: 0 in place, 1 valblk handle, 2 blob handle
 * (stored as prefix byte || value, isValueExternal set).  Returns 1 when the key's
 * prefix equals the previous key's, 0 otherwise, PBL_INVALID_ARG (7) on a bad key. */
int pbl_colblk_writer_add(pbl_colblk_writer* w, const uint8_t* key, size_t key_len, int64_t prefix_len,
                          uint64_t trailer, const uint8_t* value, size_t value_len, int value_kind,
                          int is_obsolete);
/* Pebblev8 data blocks (sstable/format.go:305-316): DataBlockEncoder.Init with
 * WithTieringColumns() (data_block.go:610-627).  Call on a fresh or reset writer,
 * before the first add; the setting survives pbl_colblk_writer_reset. */
void pbl_colblk_writer_set_tiering(pbl_colblk_writer* w, int tiering);
/* DataBlockEncoder.AddWithSecondaryBlobHandle (data_block.go:712-765) with a
 * base.KVMeta: the meta is stored only when its attribute is non-zero
 * (KVMeta.IsSet, internal/base/internal.go:698-702), and meta and handle are
 * ignored unless the writer has the tiering columns.  Same returns as
 * pbl_colblk_writer_add. */
int pbl_colblk_writer_add_meta(pbl_colblk_writer* w, const uint8_t* key, size_t key_len, int64_t prefix_len,
                               uint64_t trailer, const uint8_t* value, size_t value_len, int value_kind,
                               int is_obsolete, uint64_t tiering_span_id, uint64_t tiering_attr,
                               const uint8_t* secondary_handle, size_t secondary_handle_len);
uint32_t pbl_colblk_writer_rows(const pbl_colblk_writer* w);
/* DataBlockEncoder.Size() as it was at `rows` rows (rows() or rows()-1). */
size_t pbl_colblk_writer_size(const pbl_colblk_writer* w, uint32_t rows);
/* Finish(rows, Size(rows)) with rows == rows() or rows()-1; copies the block to
 * dst when dst_cap suffices; returns the block size (0 on a bad row count).  The
 * writer must be reset before reuse. */
size_t pbl_colblk_writer_finish(pbl_colblk_writer* w, uint32_t rows, uint8_t* dst, size_t dst_cap);

/* cockroachkvs.KeyGenConfig (cockroachkvs/test_utils.go) + value length. */
typedef struct pbl_colgen_config {
  uint64_t seed;
  uint32_t alphabet_len;       /* PrefixAlphabetLen                        */
  uint32_t prefix_len_shared;  /* PrefixLenShared                          */
  uint32_t roach_key_len;      /* RoachKeyLen                              */
  uint32_t avg_keys_per_prefix;/* AvgKeysPerPrefix                         */
  uint64_t base_wall_time;     /* BaseWallTime                             */
  uint32_t pct_logical;        /* PercentLogical                           */
  uint32_t value_len;
  uint32_t obsolete_every;     /* 0, or: row k of a block has isObsolete set
                                  when k % obsolete_every == obsolete_every-1
                                  (HideObsoletePoints measurements)         */
  uint32_t tiering;            /* 0, or: Pebblev8 blocks with the tiering
                                  columns; row k's KVMeta is span 1 + r % tiering,
                                  attribute (base_wall_time / 1e9) + r % 3600,
                                  unset (KVMeta{}) for one row in ten, r drawn
                                  per row from the block's seed             */
  uint32_t first_block;        /* global index of the first block generated:
                                  block i of the output is global block
                                  first_block + i (a rank's shard of one
                                  global batch)                              */
  uint32_t reserved;
} pbl_colgen_config;

/*
 * Synthetic colblk batch (config 3): per block, sorted KVs drawn per
 * cockroachkvs.RandomKVs with a per-block seed, trailer MakeTrailer((block<<20)+k,
 * SET), random value bytes; rows are added while the finished block stays
 * <= block_size (Finish(rows-1) on overflow, as the sstable writer does) and
 * blocks are placed at a fixed `block_size` stride.  Returns total rows.
 */
uint64_t pbl_gen_col_blocks(const pbl_colgen_config* cfg, uint32_t schema, uint32_t n_blocks,
                            uint32_t block_size, uint8_t* dst, uint64_t* block_off,
                            uint32_t* block_len, int n_threads);

/* Config 5 (BASELINE.json configs[4]): Zipf(s)-skewed key and value lengths. */
typedef struct pbl_zipf_config {
  uint64_t seed;
  uint32_t key_min, key_max;   /* user-key length range, key_min >= 8 (8, 1024)  */
  uint32_t val_min, val_max;   /* value length range (0, 65536)                   */
  double s;                    /* Zipf exponent (1.1)                             */
  uint32_t block_size;         /* target block size; a block always takes its
                                  first KV, so one large KV may exceed it         */
  int32_t restart_interval;    /* row format only (1, 16, 32)                     */
  uint32_t first_block;        /* output block i = global block first_block + i   */
  uint32_t reserved;
} pbl_zipf_config;

/*
 * Synthetic config-5 batch in host memory: format PBL_FMT_ROW (rowblk.Writer)
 * or PBL_FMT_COL_DEFAULT (DataBlockEncoder + DefaultKeySchema).  Key of row k of
 * block b: 8 base-26 letters of (b << 20) + k, then random letters to its Zipf
 * length; trailer MakeTrailer((b << 20) + k, SET); random value bytes.  Blocks
 * are variable-length, packed at 8-B alignment into dst; *bytes_used is the
 * packed size.  Returns total KVs, or UINT64_MAX on a bad config or when
 * dst_cap < *bytes_used (nothing copied).
 */
uint64_t pbl_gen_zipf_blocks(const pbl_zipf_config* cfg, uint32_t format, uint32_t n_blocks,
                             uint8_t* dst, uint64_t dst_cap, uint64_t* block_off, uint32_t* block_len,
                             uint64_t* bytes_used, int n_threads);

/* ---- blockiter.Data over one decoded block (host side) ----
 * The adapter a Go shim exposes behind sstable/blockiter
 * (sstable/blockiter/block_iter.go:19-108): rowblk.Iter / colblk.DataBlockIter
 * positioning over the arrays of a decoded batch COPIED TO HOST MEMORY (every
 * pointer of `host` is a host pointer; nothing here touches the device).  A
 * positioning call returns the KV it lands on or NULL (exhausted); the pbl_kv
 * it points to lives in the iterator and is valid until the next call. */
#define PBL_CMP_DEFAULT 0u  /* base.DefaultComparer: bytes.Compare, Split = len   */
#define PBL_CMP_TESTKEYS 1u /* testkeys.Comparer (internal/testkeys/testkeys.go)  */
#define PBL_CMP_CRDB 2u     /* cockroachkvs.Comparer (cockroachkvs/cockroachkvs.go) */

typedef struct pbl_kv {   /* base.InternalKV over the decoded arrays (block/kv.go) */
  const uint8_t* user_key;
  uint64_t user_key_len;
  uint64_t trailer;       /* InternalKeyTrailer, as decoded (transforms applied) */
  const uint8_t* value;   /* in-place value bytes, or the handle bytes          */
  uint64_t value_len;
  uint32_t kv_flags;      /* PBL_KV_*                                          */
  uint32_t reserved;
} pbl_kv;

typedef struct pbl_kv_meta { /* base.KVMeta (internal/base/internal.go:686-689)    */
  uint64_t tiering_span_id;
  uint64_t tiering_attribute;
} pbl_kv_meta;

typedef struct pbl_data_iter pbl_data_iter;
pbl_data_iter* pbl_data_iter_new(void);
void pbl_data_iter_free(pbl_data_iter* it);
/* InitHandle (block_iter.go:84-90) for block `block` of a decoded batch of
 * n_blocks: PBL_OK, or the block's decode status (the iterator is then
 * invalidated), or PBL_INVALID_ARG.  hide_obsolete_points: the
 * HideObsoletePoints transform (KVs with PBL_KV_OBSOLETE are skipped). */
int pbl_data_iter_init(pbl_data_iter* it, const pbl_decode_out* host, uint32_t n_blocks, uint32_t block,
                       uint32_t comparer, uint32_t hide_obsolete_points);
const pbl_kv* pbl_data_iter_first(pbl_data_iter* it);
const pbl_kv* pbl_data_iter_last(pbl_data_iter* it);
const pbl_kv* pbl_data_iter_next(pbl_data_iter* it);
const pbl_kv* pbl_data_iter_prev(pbl_data_iter* it);
const pbl_kv* pbl_data_iter_seek_ge(pbl_data_iter* it, const uint8_t* key, uint64_t key_len, uint32_t flags);
const pbl_kv* pbl_data_iter_seek_lt(pbl_data_iter* it, const uint8_t* key, uint64_t key_len, uint32_t flags);
/* FirstWithMeta / NextWithMeta / SeekGEWithMeta (colblk data_block.go:1574-1600;
 * the MetaIterator of sstable/reader_iter.go:26-33): the same positioning, and
 * *meta = the KV's KVMeta from the decoded tiering_span_id / tiering_attr
 * arrays, or KVMeta{} when the iterator lands on no KV or the arrays were not
 * decoded (NULL in `host`, as for row blocks and non-tiering formats). */
const pbl_kv* pbl_data_iter_first_with_meta(pbl_data_iter* it, pbl_kv_meta* meta);
const pbl_kv* pbl_data_iter_next_with_meta(pbl_data_iter* it, pbl_kv_meta* meta);
const pbl_kv* pbl_data_iter_seek_ge_with_meta(pbl_data_iter* it, const uint8_t* key, uint64_t key_len,
                                              uint32_t flags, pbl_kv_meta* meta);
/* (kv, 0) same prefix; (NULL, 1) positioned at a KV of another prefix; (NULL, 0) none */
const pbl_kv* pbl_data_iter_seek_prefix_ge(pbl_data_iter* it, const uint8_t* key, uint64_t key_len, uint32_t flags,
                                           int* prefix_did_not_match);
const pbl_kv* pbl_data_iter_next_with_same_prefix(pbl_data_iter* it, int* prefix_exhausted);
const pbl_kv* pbl_data_iter_next_prefix(pbl_data_iter* it, const uint8_t* succ_key, uint64_t succ_len);
int pbl_data_iter_is_lower_bound(const pbl_data_iter* it, const uint8_t* key, uint64_t key_len);
int pbl_data_iter_valid(const pbl_data_iter* it);
const pbl_kv* pbl_data_iter_kv(pbl_data_iter* it);
void pbl_data_iter_invalidate(pbl_data_iter* it);
int pbl_data_iter_is_data_invalidated(const pbl_data_iter* it);
/* the comparers themselves (Compare < 0 / 0 / > 0, Split) */
int pbl_key_compare(uint32_t comparer, const uint8_t* a, uint64_t a_len, const uint8_t* b, uint64_t b_len);
uint64_t pbl_key_split(uint32_t comparer, const uint8_t* key, uint64_t key_len);

#ifdef __cplusplus
}
#endif
#endif /* PEBBLE_AMD_H */
