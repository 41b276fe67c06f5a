/*
 * ecg_migrate.c -- the rebuild of one EC parity shard, batched on the device
 * (include/ecg_daos.h ecg_migrate_update_parity).
 *
 * migrate_update_parity (ref:src/object/srv_obj_migrate.c:1096-1181) walks a
 * fetched record range piece by piece: a full stripe is encoded with
 * obj_ec_encode_buf and only the rebuilt shard's parity cell is written (with
 * its VOS parity index, :1122-1142); anything else is written as replicated
 * records (:1145-1151); each piece is checksummed (daos_csummer_calc_iods,
 * :1156) and handed to vos_obj_update.  Here the same walk yields a plan of
 * pieces, every kept parity cell of the range comes out of ONE product launch
 * with a single output row (the (k+1)*C of traffic per stripe the cell needs,
 * not the (k+p)*C of a full encode), and every piece's checksums out of
 * checksum launches grouped by chunk geometry -- fused into the product when
 * the parity cells start on chunk boundaries.
 */
#include <string.h>

#include "ecg_internal.h"
#include "../../../include/ecg_daos.h"
#include "../../../include/ecg_csum.h"

struct mplan {
	uint32_t n, nparity;
	uint64_t first_parity_off;	/* buffer byte offset of the first full stripe */
	uint64_t csum_bytes;
};

/* The reference walk (:1114-1177).  pieces may be NULL (sizing only). */
static void migrate_walk(uint32_t k, uint64_t e_len, uint64_t iod_size, uint64_t offset, uint64_t size,
			 int encode, int csum_type, uint64_t chunksize, ecg_migrate_piece_t *pieces,
			 struct mplan *pl)
{
	const uint64_t stride_nr = (uint64_t)k * e_len, cell_nr = e_len;
	const uint64_t split = encode ? stride_nr : cell_nr;
	const int cl = csum_type ? ecg_csum_len(csum_type) : 0;
	uint64_t boff = 0;

	memset(pl, 0, sizeof(*pl));
	while (size > 0) {
		uint64_t write_nr, nch;
		ecg_migrate_piece_t pc;

		if (offset % split != 0) {
			write_nr = (offset / split + 1) * split - offset;
			if (write_nr > size)
				write_nr = size;
		} else {
			write_nr = split < size ? split : size;
		}
		memset(&pc, 0, sizeof(pc));
		if (write_nr == stride_nr && encode) {
			pc.recx.rx_idx = ecg_obj_ec_idx_daos2vos(offset, stride_nr, cell_nr) | ECG_EC_PARITY_BIT;
			pc.recx.rx_nr = cell_nr;
			pc.parity = 1;
			pc.buf_off = (uint64_t)pl->nparity * cell_nr * iod_size;	/* in parity_out */
			if (pl->nparity++ == 0)
				pl->first_parity_off = boff;
		} else {
			pc.recx.rx_idx = offset;
			pc.recx.rx_nr = write_nr;
			pc.buf_off = boff;					/* in buffer */
		}
		pc.buf_len = pc.recx.rx_nr * iod_size;
		nch = cl > 0 ? ecg_csum_chunk_count(chunksize, iod_size, pc.recx.rx_idx, pc.recx.rx_nr) : 0;
		pc.nr_csums = (uint32_t)nch;
		pc.csum_off = pl->csum_bytes;
		pl->csum_bytes += nch * (uint64_t)(cl > 0 ? cl : 0);
		if (pieces)
			pieces[pl->n] = pc;
		pl->n++;
		size -= write_nr;
		offset += write_nr;
		boff += write_nr * iod_size;
	}
}

static int check_args(uint32_t oc_id, uint64_t e_len, uint64_t iod_size, int csum_type, uint64_t chunksize,
		      int *k, int *p)
{
	int rc = ecg_obj_ec_class_kp(oc_id, k, p);

	if (rc)
		return rc;
	if (e_len == 0 || iod_size == 0)
		return ecg_fail(-ECG_DER_INVAL, "migrate: e_len=%lu iod_size=%lu", (unsigned long)e_len,
				(unsigned long)iod_size);
	if (csum_type && (ecg_csum_len(csum_type) < 0 || chunksize == 0))
		return ecg_fail(-ECG_DER_NOTSUPPORTED, "migrate: checksum type %d / chunk %lu", csum_type,
				(unsigned long)chunksize);
	return 0;
}

int ecg_migrate_plan_size(uint32_t oc_id, uint64_t e_len, uint64_t iod_size, uint64_t offset, uint64_t size,
			  int encode, int csum_type, uint64_t chunksize, uint32_t *npieces, uint32_t *nparity,
			  uint64_t *csum_bytes)
{
	struct mplan pl;
	int k, p, rc;

	rc = check_args(oc_id, e_len, iod_size, csum_type, chunksize, &k, &p);
	if (rc)
		return rc;
	migrate_walk((uint32_t)k, e_len, iod_size, offset, size, encode, csum_type, chunksize, NULL, &pl);
	if (npieces)
		*npieces = pl.n;
	if (nparity)
		*nparity = pl.nparity;
	if (csum_bytes)
		*csum_bytes = pl.csum_bytes;
	return 0;
}

/* Checksums of pieces [i0, i1): consecutive pieces of one chunk geometry
 * (record count and index modulo the record chunk) whose bytes lie a fixed
 * stride apart share one ecg_csum_extents launch; their checksums are
 * consecutive in csums_out by construction. */
static int csum_pieces(ecg_ctx_t *ctx, const ecg_migrate_piece_t *pc, uint32_t i0, uint32_t i1,
		       const unsigned char *buffer, const unsigned char *parity_out, int type, uint64_t chunksize,
		       uint64_t iod_size, unsigned char *csums_out, hipStream_t st)
{
	const uint64_t per = ecg_csum_record_chunksize(chunksize, iod_size) / iod_size;
	uint32_t i = i0;

	while (i < i1) {
		const unsigned char *b0 = (pc[i].parity ? parity_out : buffer) + pc[i].buf_off;
		uint32_t j = i + 1;
		int64_t stride = 0;
		int rc;

		while (j < i1 && pc[j].parity == pc[i].parity && pc[j].recx.rx_nr == pc[i].recx.rx_nr &&
		       pc[j].recx.rx_idx % per == pc[i].recx.rx_idx % per) {
			const int64_t d = (int64_t)(pc[j].buf_off - pc[j - 1].buf_off);

			if (j == i + 1)
				stride = d;
			else if (d != stride)
				break;
			j++;
		}
		rc = ecg_csum_extents(ctx, type, chunksize, iod_size, pc[i].recx.rx_idx, pc[i].recx.rx_nr, b0,
				      stride, j - i, csums_out + pc[i].csum_off, (void *)st);
		if (rc)
			return rc;
		i = j;
	}
	return 0;
}

int ecg_migrate_update_parity(ecg_ctx_t *ctx, uint32_t oc_id, uint64_t e_len, uint64_t iod_size,
			      uint32_t shard, const void *buffer, uint64_t offset, uint64_t size, int encode,
			      int csum_type, uint64_t chunksize, void *parity_out, void *csums_out,
			      ecg_migrate_piece_t *pieces, uint32_t pieces_cap, uint32_t *npieces, void *stream)
{
	unsigned char en[(ECG_MAX_K + ECG_MAX_P) * ECG_MAX_K];
	const unsigned char *buf = buffer;
	struct mplan pl;
	uint32_t first = 0, last = 0;
	hipStream_t st;
	int k, p, rc;

	rc = check_args(oc_id, e_len, iod_size, csum_type, chunksize, &k, &p);
	if (rc)
		return rc;
	if (ctx == NULL || pieces == NULL || npieces == NULL || (size && buffer == NULL))
		return ecg_fail(-ECG_DER_INVAL, "migrate: NULL argument");
	if (encode && (shard < (uint32_t)k || shard >= (uint32_t)(k + p)))	/* :1129-1131 */
		return ecg_fail(-ECG_DER_INVAL, "migrate: shard %u is not a parity shard of %d+%d", shard, k, p);
	migrate_walk((uint32_t)k, e_len, iod_size, offset, size, encode, csum_type, chunksize, NULL, &pl);
	if (pl.n > pieces_cap)
		return ecg_fail(-ECG_DER_REC2BIG, "migrate: %u pieces > capacity %u", pl.n, pieces_cap);
	if ((pl.nparity && parity_out == NULL) || (pl.csum_bytes && csums_out == NULL))
		return ecg_fail(-ECG_DER_INVAL, "migrate: NULL output buffer");
	migrate_walk((uint32_t)k, e_len, iod_size, offset, size, encode, csum_type, chunksize, pieces, &pl);
	*npieces = pl.n;
	if (pl.n == 0)
		return 0;
	rc = ecg_ctx_enter(ctx);
	if (rc)
		return rc;
	st = ecg_pick_stream(ctx, stream);

	if (pl.nparity) {
		const uint64_t C = e_len * iod_size;
		const uint64_t per = csum_type ? ecg_csum_record_chunksize(chunksize, iod_size) / iod_size : 1;
		const unsigned char *coef;
		int64_t soff[ECG_MAX_K], doff[1] = {0};
		uint32_t slot[1] = {0};

		while (!pieces[first].parity)
			first++;
		last = first + pl.nparity;
		for (int j = 0; j < k; j++)
			soff[j] = (int64_t)j * (int64_t)C;
		ecg_gen_cauchy1(k, p, en);
		coef = &en[(size_t)shard * k];		/* matrix row `shard`: this shard's parity */
		if (csum_type && pieces[first].recx.rx_idx % per == 0 && e_len % per == 0) {
			/* every kept cell starts on a chunk boundary: checksums as
			 * extents from index 0, fused into the product where the
			 * shape allows */
			rc = ecg_matmul_csum(ctx, k, 1, coef, C, pl.nparity, buf + pl.first_parity_off, soff,
					     (int64_t)k * (int64_t)C, parity_out, doff, (int64_t)C, csum_type,
					     chunksize, iod_size, (unsigned char *)csums_out + pieces[first].csum_off,
					     slot, (void *)st);
		} else {
			rc = ecg_matmul(ctx, k, 1, coef, C, pl.nparity, buf + pl.first_parity_off, soff,
					(int64_t)k * (int64_t)C, parity_out, doff, (int64_t)C, 0, (void *)st);
			if (rc == 0 && csum_type)
				rc = csum_pieces(ctx, pieces, first, last, buf, parity_out, csum_type, chunksize,
						 iod_size, csums_out, st);
		}
		if (rc)
			return rc;
	}
	if (csum_type) {			/* replicated pieces before and after the stripes */
		rc = csum_pieces(ctx, pieces, 0, first, buf, parity_out, csum_type, chunksize, iod_size, csums_out,
				 st);
		if (rc == 0)
			rc = csum_pieces(ctx, pieces, last, pl.n, buf, parity_out, csum_type, chunksize, iod_size,
					 csums_out, st);
	}
	return rc;
}
