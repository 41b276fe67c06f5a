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

#ifdef __cplusplus
}
#endif

#endif
