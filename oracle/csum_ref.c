/*
 * csum_ref.c -- CPU ORACLE for DAOS chunked checksums of EC cells (SURVEY
 * §8f rank 4: checksums on regenerated parity / recovered cells).
 *
 * TEST INFRASTRUCTURE ONLY (see ec_ref.h): used by tests/ and smoke() as the
 * checker; nothing under daos_amd/ or include/ links it.
 *
 * What it restates:
 *   - the four non-cryptographic DAOS hash types, as DAOS drives them
 *     (ref:src/common/multihash_isal.c:27-256; type numbers
 *     ref:src/include/daos/multihash.h:22-33), each reset to 0 before every
 *     chunk (ref:src/common/checksum.c:481-483):
 *       HASH_TYPE_CRC16   crc16_t10dif(seed, buf, len)      (ISA-L crc)
 *       HASH_TYPE_CRC32   crc32_iscsi(buf, len, seed)       (ISA-L crc)
 *       HASH_TYPE_CRC64   crc64_ecma_refl(seed, buf, len)   (ISA-L crc64)
 *       HASH_TYPE_ADLER32 isal_adler32(seed, buf, len)      (ISA-L igzip)
 *     ISA-L v2.31.1 is not in /root/reference or this image; its published
 *     base semantics are restated bit by bit here (no lookup tables, so this
 *     file shares no table math with the device kernels):
 *       crc16_t10dif  : poly 0x8BB7, MSB first, state = seed, no xorout
 *       crc32_iscsi   : poly 0x1EDC6F41 reflected (0x82F63B78), state = seed,
 *                       no pre/post inversion
 *       crc64_ecma_refl: poly 0x42F0E1EBA9EA3693 reflected
 *                       (0xC96C5795D7870F42), state = ~seed, result ~state
 *       adler32       : A = seed & 0xffff, B = seed >> 16, mod 65521
 *   - the csummer's chunking of one array extent (recx):
 *       chunk bytes per record size   csum_record_chunksize
 *                                     ref:src/common/checksum.c:1475-1482
 *       number of chunks              daos_recx_calc_chunks / csum_chunk_count
 *                                     ref:src/common/checksum.c:1444-1454,1568-1581
 *       chunk i's record range        csum_recx_chunkidx2range ->
 *                                     csum_chunkidx2range -> csum_recidx2range
 *                                     ref:src/common/checksum.c:1489-1565
 *       per-chunk hash                calc_csum_recx_with_no_map
 *                                     ref:src/common/checksum.c:467-497
 *
 * PINNING: the reference's checksum unit tests use a fake algorithm
 * (ref:src/common/tests/checksum_tests.c) and hold no real CRC values, so the
 * hash bytes are pinned by the published check values of the CRC catalogue
 * ("123456789": CRC-16/T10-DIF 0xD0DB, CRC-32/ISCSI 0xE3069283, CRC-64/XZ
 * 0x995DC9BBDF1939FA, Adler-32 0x091E01DE; tests/golden/kat.json), by
 * Python's zlib.adler32 for adler32, and by an independent table-driven
 * Python restatement (tests/test_csum_oracle.py).  The chunking is pinned by
 * the reference's own chunk-count and range cases, restated in the tests.
 */
#include <stdint.h>
#include <string.h>

#include "ec_ref.h"

uint16_t ref_crc16_t10dif(uint16_t seed, const unsigned char *buf, uint64_t len)
{
	uint16_t crc = seed;

	for (uint64_t i = 0; i < len; i++) {
		crc ^= (uint16_t)(buf[i] << 8);
		for (int b = 0; b < 8; b++)
			crc = (crc & 0x8000) ? (uint16_t)((crc << 1) ^ 0x8BB7) : (uint16_t)(crc << 1);
	}
	return crc;
}

uint32_t ref_crc32_iscsi(const unsigned char *buf, uint64_t len, uint32_t seed)
{
	uint32_t crc = seed;

	for (uint64_t i = 0; i < len; i++) {
		crc ^= buf[i];
		for (int b = 0; b < 8; b++)
			crc = (crc & 1) ? (crc >> 1) ^ 0x82F63B78u : crc >> 1;
	}
	return crc;
}

uint64_t ref_crc64_ecma_refl(uint64_t seed, const unsigned char *buf, uint64_t len)
{
	uint64_t crc = ~seed;

	for (uint64_t i = 0; i < len; i++) {
		crc ^= buf[i];
		for (int b = 0; b < 8; b++)
			crc = (crc & 1) ? (crc >> 1) ^ 0xC96C5795D7870F42ull : crc >> 1;
	}
	return ~crc;
}

uint32_t ref_adler32(uint32_t seed, const unsigned char *buf, uint64_t len)
{
	uint64_t a = seed & 0xffff, b = seed >> 16;

	for (uint64_t i = 0; i < len; i++) {
		a = (a + buf[i]) % 65521;
		b = (b + a) % 65521;
	}
	return (uint32_t)((b << 16) | a);
}

int ref_csum_len(int type)
{
	switch (type) {
	case REF_HASH_CRC16:
		return 2;
	case REF_HASH_CRC32:
	case REF_HASH_ADLER32:
		return 4;
	case REF_HASH_CRC64:
		return 8;
	default:
		return -1;
	}
}

/* one chunk, hash reset to 0 first (ref:src/common/checksum.c:481-496) */
static void hash_chunk(int type, const unsigned char *buf, uint64_t len, unsigned char *out)
{
	uint16_t h16;
	uint32_t h32;
	uint64_t h64;

	switch (type) {
	case REF_HASH_CRC16:
		h16 = ref_crc16_t10dif(0, buf, len);
		memcpy(out, &h16, 2);
		break;
	case REF_HASH_CRC32:
		h32 = ref_crc32_iscsi(buf, len, 0);
		memcpy(out, &h32, 4);
		break;
	case REF_HASH_CRC64:
		h64 = ref_crc64_ecma_refl(0, buf, len);
		memcpy(out, &h64, 8);
		break;
	case REF_HASH_ADLER32:
		h32 = ref_adler32(0, buf, len);
		memcpy(out, &h32, 4);
		break;
	}
}

/* csum_record_chunksize, ref:src/common/checksum.c:1475-1482 */
uint64_t ref_csum_record_chunksize(uint64_t chunksize, uint64_t rec_size)
{
	if (rec_size > chunksize)
		return rec_size;
	return (chunksize / rec_size) * rec_size;
}

/* daos_recx_calc_chunks / csum_chunk_count, ref:src/common/checksum.c:1444-1454,
 * 1568-1581; csum_align_boundaries widens [lo, hi] to whole chunks. */
uint32_t ref_csum_chunk_count(uint64_t rec_chunksize, uint64_t rec_size, uint64_t rx_idx,
			      uint64_t rx_nr)
{
	uint64_t per, lo, hi;

	if (rx_nr == 0 || rec_size == 0)
		return 0;
	if (rx_nr == 1)
		return 1;
	per = rec_chunksize / rec_size;
	lo = rx_idx / per;		/* aligned chunk numbers: no overflow near UINT64_MAX */
	hi = (rx_idx + (rx_nr - 1)) / per;
	return (uint32_t)(hi - lo + 1);
}

/* calc_csum_recx_with_no_map over one extent whose records are contiguous in
 * buf (ref:src/common/checksum.c:467-497, ranges :1489-1565).  Returns the
 * number of checksums written to out (csum_len bytes each, little-endian). */
uint32_t ref_csum_extent(int type, uint64_t chunksize, uint64_t rec_size, uint64_t rx_idx,
			 uint64_t rx_nr, const unsigned char *buf, unsigned char *out)
{
	const int cl = ref_csum_len(type);
	uint64_t rcs, per, lo, hi;
	uint32_t n;

	if (cl < 0 || rec_size == 0 || rx_nr == 0)
		return 0;
	rcs = ref_csum_record_chunksize(chunksize, rec_size);
	per = rcs / rec_size;
	n = ref_csum_chunk_count(rcs, rec_size, rx_idx, rx_nr);
	lo = rx_idx;
	hi = rx_idx + (rx_nr - 1);
	for (uint32_t i = 0; i < n; i++) {
		/* csum_chunkidx2range: record index of chunk i's aligned start */
		uint64_t r = (lo - lo % per) + (uint64_t)i * per;
		uint64_t clo = r - r % per, chi = clo + (per - 1);

		if (chi < clo)		/* csum_chunk_align_ceiling overflow guard */
			chi = UINT64_MAX;
		if (clo < lo)
			clo = lo;
		if (chi > hi)
			chi = hi;
		hash_chunk(type, buf + (clo - rx_idx) * rec_size, (chi - clo + 1) * rec_size,
			   out + (uint64_t)i * cl);
	}
	return n;
}

/* n_ext extents at buf + e * ext_stride, all with the same (rx_idx, rx_nr):
 * csums out[e][chunk]; OpenMP over extents. */
void ref_csum_extents(int type, uint64_t chunksize, uint64_t rec_size, uint64_t rx_idx,
		      uint64_t rx_nr, const unsigned char *buf, int64_t ext_stride, uint32_t n_ext,
		      unsigned char *out, int nthreads)
{
	const uint64_t rcs = ref_csum_record_chunksize(chunksize, rec_size);
	const uint32_t n = ref_csum_chunk_count(rcs, rec_size, rx_idx, rx_nr);
	const int cl = ref_csum_len(type);

	if (cl < 0)
		return;
#pragma omp parallel for num_threads(nthreads > 0 ? nthreads : 1) schedule(dynamic)
	for (int64_t e = 0; e < (int64_t)n_ext; e++)
		ref_csum_extent(type, chunksize, rec_size, rx_idx, rx_nr, buf + e * ext_stride,
				out + (uint64_t)e * n * cl);
}
