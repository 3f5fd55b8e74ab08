/*
 * oracle/oracle.h — TEST INFRASTRUCTURE ONLY: shared definitions of the CPU
 * restatements (rowblk_oracle.c, colblk_oracle.c).  Status codes, flags and the
 * batch layout mirror include/pebble_amd.h.
 */
#ifndef PBL_ORACLE_H
#define PBL_ORACLE_H
#include <stdint.h>

enum { OK = 0, CORRUPT_NO_RESTARTS = 1, CORRUPT_FIRST_KEY = 2, CORRUPT_BOUNDS = 3,
       CORRUPT_COLBLK_HEADER = 4, UNSUPPORTED = 5 };
enum { FMT_ROW = 0, FMT_COL_DEFAULT = 1, FMT_COL_CRDB1 = 2 };

#define FLAG_VALUE_PREFIX 0x1u
#define FLAG_NO_VALUER 0x2u
#define FLAG_RAW_KEYS 0x4u /* rowblk.RawIter (rowblk_iter.go:1743-1794) */
#define FLAG_HIDE_OBSOLETE 0x8u /* blockiter.Transforms.HideObsoletePoints during the decode */
#define FLAG_TIERING 0x10u /* colblk blocks carry the Pebblev8 tiering columns (decodeMeta) */

#define KV_RESTART 0x01u
#define KV_RESTART_SAMEPFX 0x02u
#define KV_OBSOLETE 0x04u
#define KV_INVALID_KEY 0x08u
#define KV_VALBLK 0x10u
#define KV_BLOB 0x20u
#define KV_PREFIX_CHANGED 0x40u

typedef struct orc_block_out {
  /* counts (always written) */
  uint64_t n_kv, key_bytes, val_bytes, n_restarts;
  /* outputs; NULL = count only.  key_off/val_off hold n_kv+1 entries. */
  uint64_t* trailer;
  uint8_t* kv_flags;
  uint32_t* entry_off;
  uint32_t* key_off;
  uint32_t* val_off;
  uint8_t* keys;
  uint8_t* vals;
  uint32_t* restarts;
  /* base.KVMeta per KV (NULL = not requested; zeros unless FLAG_TIERING) */
  uint64_t* span;
  uint64_t* attr;
} orc_block_out;

/* Batch form in exactly the device layout of include/pebble_amd.h
 * (pbl_decode_out).  blk_*_base have n_blocks+1 entries. */
typedef struct orc_batch_out {
  uint64_t* trailer;
  uint8_t* kv_flags;
  uint32_t* entry_off;
  uint32_t* key_off;
  uint32_t* val_off;
  uint8_t* key_bytes;
  uint8_t* val_bytes;
  uint32_t* restarts;
  uint64_t* blk_kv_base;
  uint64_t* blk_key_base;
  uint64_t* blk_val_base;
  uint64_t* blk_rst_base;
  uint32_t* blk_status;
  uint64_t n_kv, key_bytes_total, val_bytes_total, n_restarts;
  uint32_t status_mask, n_bad_blocks;
  uint64_t* tiering_span_id; /* optional, as pbl_decode_out */
  uint64_t* tiering_attr;
} orc_batch_out;

/* blockiter.Transforms (sstable/blockiter/transforms.go:20-56) for the row
 * restatement; split is PBL_SPLIT_* (0 default, 1 testkeys, 2 cockroachkvs). */
typedef struct orc_transforms {
  uint64_t seq;
  int hide;
  int split;
  const uint8_t* prefix;
  uint64_t prefix_len;
  const uint8_t* suffix;
  uint64_t suffix_len;
} orc_transforms;

uint64_t orc_split(const uint8_t* k, uint64_t n, int split);
int orc_rowblk_decode_tf(const uint8_t* blk, uint64_t len, uint32_t flags, const orc_transforms* t,
                         orc_block_out* o);
int orc_decode_varint(const uint8_t* p, const uint8_t* end, uint32_t* v);
int orc_rowblk_decode(const uint8_t* blk, uint64_t len, uint32_t flags, orc_block_out* o);
uint64_t orc_rowblk_scan_checksum(const uint8_t* blk, uint64_t len, uint32_t flags, uint64_t* n_kv);
int orc_colblk_decode(const uint8_t* blk, uint64_t len, uint32_t schema, orc_block_out* o);
int orc_colblk_decode_flags(const uint8_t* blk, uint64_t len, uint32_t schema, uint32_t flags, orc_block_out* o);
uint64_t orc_colblk_scan_checksum(const uint8_t* blk, uint64_t len, uint32_t schema, uint64_t* n_kv);
#endif
