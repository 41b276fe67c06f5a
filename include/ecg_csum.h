/*
 * ecg_csum.h -- chunked checksums of device-resident extents, DAOS csummer
 * semantics (checksums on regenerated parity and
 * recovered cells).
 *
 * Replaces, for data already in HBM, the checksum step DAOS runs right after
 * the codec on the rebuild path:
 *   daos_csummer_calc_iods(csummer, &sgl, iod, ...)
 *       ref:src/object/srv_obj_migrate.c:1156 (regenerated parity cells)
 *   -> calc_csum_recx -> calc_csum_recx_with_no_map
 *       ref:src/common/checksum.c:631-664, 467-497
 * with the hash functions DAOS registers (ref:src/common/multihash_isal.c):
 *   ECG_HASH_CRC16   crc16_t10dif      (:27-82)
 *   ECG_HASH_CRC32   crc32_iscsi       (:84-139)
 *   ECG_HASH_CRC64   crc64_ecma_refl   (:195-257)
 *   ECG_HASH_ADLER32 isal_adler32      (:140-193)
 * each reset to 0 before every chunk.  The cryptographic types (SHA1/256/512,
 * ref:src/include/daos/multihash.h:27-29) are not provided: -DER_NOTSUPPORTED.
 *
 * Checksums are written little-endian, csum_len bytes each, extent-major
 * ([n_ext][nchunks]) -- the layout of dcs_csum_info.cs_csum for one recx
 * (ci_idx2csum, ref:src/common/checksum.c:1203-1220).
 */
#ifndef ECG_CSUM_H
#define ECG_CSUM_H

#include <stdint.h>

#include "ecg.h"

#ifdef __cplusplus
extern "C" {
#endif

/* enum DAOS_HASH_TYPE values, ref:src/include/daos/multihash.h:22-33 */
#define ECG_HASH_CRC16		1
#define ECG_HASH_CRC32		2
#define ECG_HASH_CRC64		3
#define ECG_HASH_ADLER32	7

#define ECG_DER_NOTSUPPORTED	2037

/* Checksum length in bytes (daos_csummer_get_csum_len): 2, 4, 8 or 4;
 * -ECG_DER_NOTSUPPORTED for other types. */
int ecg_csum_len(int type);

/* Chunk bytes for a record size (csum_record_chunksize,
 * ref:src/common/checksum.c:1475-1482). */
uint64_t ecg_csum_record_chunksize(uint64_t chunksize, uint64_t rec_size);

/* Number of checksums of one extent (daos_recx_calc_chunks,
 * ref:src/common/checksum.c:1444-1454). */
uint32_t ecg_csum_chunk_count(uint64_t chunksize, uint64_t rec_size, uint64_t rx_idx,
			      uint64_t rx_nr);

/* Checksum n_ext extents on the device.  Extent e holds rx_nr records of
 * rec_size bytes at buf + e * ext_stride and starts at record index rx_idx
 * (the same index for every extent: chunk boundaries fall on multiples of the
 * record chunk size in index space).  csums: device memory for
 * n_ext * ecg_csum_chunk_count(...) * ecg_csum_len(type) bytes.  Asynchronous
 * on `stream` (NULL = the context stream).  Returns 0 or a negative errno. */
int ecg_csum_extents(ecg_ctx_t *ctx, int type, uint64_t chunksize, uint64_t rec_size,
		     uint64_t rx_idx, uint64_t rx_nr, const void *buf, int64_t ext_stride,
		     uint32_t n_ext, void *csums, void *stream);

/* Encode with checksums of the parity cells it writes, in one pass: the same
 * operands as ecg_encode (include/ecg.h), plus the hash type, the csummer's
 * chunk size and record size (cell_bytes must be a multiple of rec_size;
 * every parity cell is checksummed as an extent that starts on a chunk
 * boundary, as DAOS cells do when the cell's record count is a multiple of
 * the chunk's).  csums: device memory, [p][nstripes][nch] checksums of
 * ecg_csum_len(type) bytes, nch = ecg_csum_chunk_count(chunksize, rec_size, 0,
 * cell_bytes / rec_size).  Replaces obj_ec_encode_buf + daos_csummer_calc_iods
 * on the rebuild path (ref:src/object/srv_obj_migrate.c:1122-1160).
 * CRC types with a 4 KiB-multiple record chunk and 16-byte aligned cells run
 * as one fused kernel that never re-reads the parity; other shapes run the
 * product and ecg_csum_extents back to back on the stream. */
int ecg_encode_csum(ecg_ctx_t *ctx, int k, int p, uint64_t cell_bytes, uint32_t nstripes,
		    const void *data, int64_t data_stripe_stride, void *parity,
		    int64_t parity_cell_stride, int64_t parity_stripe_stride, int type,
		    uint64_t chunksize, uint64_t rec_size, void *csums, void *stream);

/* Recover erased cells in place (as ecg_recover) and checksum them:
 * csums[nerrs][nstripes][nch] in err_list order (degraded-read / rebuild of
 * data cells, ref:src/object/cli_ec.c:2626-2643 then the csummer). */
int ecg_recover_csum(ecg_ctx_t *ctx, int k, int p, uint64_t cell_bytes, uint32_t nstripes,
		     void *stripes, int64_t stripe_stride, const uint32_t *err_list, int nerrs,
		     int type, uint64_t chunksize, uint64_t rec_size, void *csums, void *stream);

/* Launch tuning: cap on checksum workgroups (4 chunks in flight each, grid-
 * stride beyond); 0 restores the default. */
int ecg_set_csum_launch(ecg_ctx_t *ctx, uint32_t max_blocks);

/* Launch tuning: 4 KiB columns per work item of the fused product +
 * checksum kernels (ecg_encode_csum / ecg_recover_csum); 0 restores the
 * default (env ECG_FUSED_COLS, else by hash type, k and output rows: 2 for
 * crc32 with k = 8 and two rows, 4 for one row or k >= 8, else 8).  Same
 * results either way. */
int ecg_set_fused_cols(ecg_ctx_t *ctx, uint32_t ncols);

#ifdef __cplusplus
}
#endif

#endif
