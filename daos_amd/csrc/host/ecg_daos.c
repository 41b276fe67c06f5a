/*
 * ecg_daos.c -- DAOS EC codec surface over the MI355X engine
 * (see include/ecg_daos.h for the reference function each one mirrors).
 */
#include <stdlib.h>
#include <string.h>

#include "../../../include/ecg_daos.h"
#include "../../../include/ecg_isal.h"
#include "ecg_internal.h"

/* OR_RS_* order of ref:src/include/daos_obj_class.h:70-80 */
static const int g_rs_kp[ECG_OR_RS_LAST - ECG_OR_RS_FIRST + 1][2] = {
	{2, 1}, {2, 2}, {4, 1}, {4, 2}, {8, 1}, {8, 2}, {16, 1}, {16, 2}, {4, 3}, {8, 3}, {16, 3},
};
#define N_RS ((int)(sizeof(g_rs_kp) / sizeof(g_rs_kp[0])))

static struct ecg_obj_ec_codec g_codecs[N_RS];
static int g_codecs_ready;
static pthread_mutex_t g_codec_lock = PTHREAD_MUTEX_INITIALIZER;

/* The batched host entry points with ctx == NULL: the calling thread's
 * default device (ecg_dropin.c), or the CPU path when the process has none. */
static ecg_ctx_t *default_ctx(ecg_ctx_t *ctx)
{
	return ctx ? ctx : ecg_dropin_ctx();
}

int ecg_obj_ec_class_kp(uint32_t oc_id, int *k, int *p)
{
	uint32_t redun = oc_id >> ECG_OC_REDUN_SHIFT;

	if (redun < ECG_OR_RS_FIRST || redun > ECG_OR_RS_LAST)
		return ecg_fail(-ECG_DER_INVAL, "oc_id 0x%x is not an EC class", oc_id);
	*k = g_rs_kp[redun - ECG_OR_RS_FIRST][0];
	*p = g_rs_kp[redun - ECG_OR_RS_FIRST][1];
	return 0;
}

void ecg_obj_ec_codec_fini(void)
{
	int i;

	pthread_mutex_lock(&g_codec_lock);
	for (i = 0; i < N_RS; i++) {
		free(g_codecs[i].ec_en_matrix);
		free(g_codecs[i].ec_gftbls);
		memset(&g_codecs[i], 0, sizeof(g_codecs[i]));
	}
	g_codecs_ready = 0;
	pthread_mutex_unlock(&g_codec_lock);
}

/* obj_ec_codec_init (ref:src/object/obj_class.c:548-631): one Cauchy1
 * matrix + ISA-L tables per EC redundancy (every group count of a (k, p)
 * shares it; the reference builds one per class id with identical bytes). */
int ecg_obj_ec_codec_init(void)
{
	int i, rc = 0;

	pthread_mutex_lock(&g_codec_lock);
	if (g_codecs_ready) {
		pthread_mutex_unlock(&g_codec_lock);
		return 0;
	}
	for (i = 0; i < N_RS; i++) {
		struct ecg_obj_ec_codec *c = &g_codecs[i];
		int k = g_rs_kp[i][0], p = g_rs_kp[i][1];

		c->k = k;
		c->p = p;
		c->ec_en_matrix = malloc((size_t)(k + p) * k);
		c->ec_gftbls = malloc((size_t)k * p * 32);
		if (c->ec_en_matrix == NULL || c->ec_gftbls == NULL) {
			rc = ecg_fail(-ECG_DER_NOMEM, "codec_init: malloc");
			break;
		}
		ecg_gen_cauchy1(k, p, c->ec_en_matrix);
		ec_init_tables(k, p, &c->ec_en_matrix[k * k], c->ec_gftbls);
	}
	g_codecs_ready = rc == 0;
	pthread_mutex_unlock(&g_codec_lock);
	if (rc)
		ecg_obj_ec_codec_fini();
	return rc;
}

struct ecg_obj_ec_codec *ecg_obj_ec_codec_get(uint32_t oc_id)
{
	uint32_t redun = oc_id >> ECG_OC_REDUN_SHIFT;

	if (!g_codecs_ready || redun < ECG_OR_RS_FIRST || redun > ECG_OR_RS_LAST)
		return NULL;
	return &g_codecs[redun - ECG_OR_RS_FIRST];
}

int ecg_obj_ec_encode_buf(uint32_t oc_id, uint64_t cell_bytes, unsigned char *buffer,
			  unsigned char *p_bufs[])
{
	unsigned char en[(ECG_MAX_K + ECG_MAX_P) * ECG_MAX_K];
	unsigned char *data[ECG_MAX_K];
	int k, p, i, rc;

	rc = ecg_obj_ec_class_kp(oc_id, &k, &p);
	if (rc)
		return rc;
	if (cell_bytes > 0x7fffffffULL)
		return ecg_fail(-ECG_DER_INVAL, "encode_buf: cell %llu too large",
				(unsigned long long)cell_bytes);
	/* same allocation rule as the reference: leading NULL p_bufs only */
	for (i = 0; i < p && p_bufs[i] == NULL; i++) {
		p_bufs[i] = malloc(cell_bytes ? cell_bytes : 1);
		if (p_bufs[i] == NULL)
			return ecg_fail(-ECG_DER_NOMEM, "encode_buf: malloc");
	}
	for (i = 0; i < k; i++)
		data[i] = buffer + (size_t)i * cell_bytes;
	ecg_gen_cauchy1(k, p, en);
	return ecg_dropin_product("obj_ec_encode_buf", NULL, (int)cell_bytes, k, p, &en[k * k], data, p_bufs, 0);
}

struct ecg_obj_ec_recov_codec *ecg_obj_ec_recov_codec_alloc(void)
{
	return calloc(1, sizeof(struct ecg_obj_ec_recov_codec));
}

void ecg_obj_ec_recov_codec_free(struct ecg_obj_ec_recov_codec *recov)
{
	free(recov);
}

int ecg_obj_ec_recov_codec_init(uint32_t oc_id, const uint32_t *err_list, uint32_t nerrs,
				struct ecg_obj_ec_recov_codec *rv)
{
	unsigned char en[(ECG_MAX_K + ECG_MAX_P) * ECG_MAX_K];
	int k, p, rc, reused = 0;
	uint32_t i;

	if (rv == NULL || err_list == NULL || nerrs == 0)
		return ecg_fail(-ECG_DER_INVAL, "recov_codec_init: bad arguments");
	rc = ecg_obj_ec_class_kp(oc_id, &k, &p);
	if (rc)
		return rc;
	if (nerrs > (uint32_t)p)
		return ecg_fail(-ECG_DER_DATA_LOSS, "recov_codec_init: nerrs %u > p %d", nerrs, p);
	/* the codec already holds these erasures' rows: nothing to build
	 * (obj_ec_err_match, ref:src/object/cli_ec.c:2176-2185; the class is
	 * compared too, the reference's codec belongs to one object) */
	if (rv->er_builds && rv->k == k && rv->p == p && rv->er_nerrs == nerrs) {
		for (i = 0; i < nerrs && rv->er_err_list[i] == err_list[i]; i++)
			;
		if (i == nerrs)
			return 0;
	}
	{
		const uint32_t builds = rv->er_builds;

		memset(rv, 0, sizeof(*rv));
		rv->er_builds = builds;
	}
	rv->k = k;
	rv->p = p;
	for (i = 0; i < nerrs; i++) {
		if (err_list[i] >= (uint32_t)(k + p))
			return ecg_fail(-ECG_DER_INVAL, "recov_codec_init: cell %u of a %d+%d stripe", err_list[i], k, p);
		rv->er_err_list[i] = err_list[i];
		if (err_list[i] < (uint32_t)k)
			rv->er_data_nerrs++;
	}
	ecg_gen_cauchy1(k, p, en);
	rc = ecg_recov_matrix(k, p, en, err_list, (int)nerrs, rv->er_de_matrix, rv->er_dec_idx,
			      &reused);
	if (rc)
		return rc;
	rv->reused_encode = reused;
	ec_init_tables(k, (int)nerrs, rv->er_de_matrix, rv->er_gftbls);
	/* published last: a failed build leaves er_nerrs 0, which never matches */
	rv->er_nerrs = nerrs;
	rv->er_builds++;
	return 0;
}

int ecg_obj_ec_recov_data(ecg_ctx_t *ctx, const struct ecg_obj_ec_recov_codec *rv,
			  uint64_t cell_sz, unsigned char *buf_stripes, uint32_t nstripes)
{
	unsigned char en[(ECG_MAX_K + ECG_MAX_P) * ECG_MAX_K], rows[ECG_MAX_P * ECG_MAX_K];
	uint32_t out_idx[ECG_MAX_P], dec_idx[ECG_MAX_K];
	unsigned char *src[ECG_MAX_K], *dst[ECG_MAX_P];
	int rc, reused, i;
	uint32_t s;

	if (rv == NULL || buf_stripes == NULL)
		return ecg_fail(-ECG_DER_INVAL, "recov_data: NULL argument");
	ctx = default_ctx(ctx);
	if (ctx)
		return ecg_recover_host(ctx, rv->k, rv->p, cell_sz, nstripes, buf_stripes,
					rv->er_err_list, (int)rv->er_nerrs, 0);
	/* no usable device: obj_ec_recov_stripe's loop on the CPU path */
	if (cell_sz > 0x7fffffffULL)
		return ecg_fail(-ECG_DER_INVAL, "recov_data: cell %llu too large", (unsigned long long)cell_sz);
	ecg_gen_cauchy1(rv->k, rv->p, en);
	rc = ecg_recov_rows(rv->k, rv->p, en, rv->er_err_list, (int)rv->er_nerrs, rows, out_idx, dec_idx,
			    &reused);
	for (s = 0; rc == 0 && s < nstripes; s++) {
		unsigned char *st = buf_stripes + (size_t)s * (size_t)(rv->k + rv->p) * cell_sz;

		for (i = 0; i < rv->k; i++)
			src[i] = st + (size_t)dec_idx[i] * cell_sz;
		for (i = 0; i < (int)rv->er_nerrs; i++)
			dst[i] = st + (size_t)out_idx[i] * cell_sz;
		rc = ecg_cpu_matmul((int)cell_sz, rv->k, (int)rv->er_nerrs, rows, src, dst, 0);
	}
	return rc;
}

int ecg_obj_ec_encode_stripes(ecg_ctx_t *ctx, uint32_t oc_id, uint64_t cell_bytes,
			      uint32_t nstripes, const unsigned char *data, unsigned char *parity)
{
	int k, p, rc;

	unsigned char en[(ECG_MAX_K + ECG_MAX_P) * ECG_MAX_K];
	unsigned char *src[ECG_MAX_K], *dst[ECG_MAX_P];
	uint32_t s;
	int i;

	rc = ecg_obj_ec_class_kp(oc_id, &k, &p);
	if (rc)
		return rc;
	ctx = default_ctx(ctx);
	if (ctx)
		return ecg_encode_host(ctx, k, p, cell_bytes, nstripes, data, parity, 0);
	/* no usable device: obj_ec_recx_encode's stripe loop on the CPU path */
	if (cell_bytes > 0x7fffffffULL)
		return ecg_fail(-ECG_DER_INVAL, "encode_stripes: cell %llu too large",
				(unsigned long long)cell_bytes);
	ecg_gen_cauchy1(k, p, en);
	for (s = 0; rc == 0 && s < nstripes; s++) {
		for (i = 0; i < k; i++)
			src[i] = (unsigned char *)data + ((size_t)s * k + i) * cell_bytes;
		for (i = 0; i < p; i++)
			dst[i] = parity + ((size_t)i * nstripes + s) * cell_bytes;
		rc = ecg_cpu_matmul((int)cell_bytes, k, p, &en[k * k], src, dst, 0);
	}
	return rc;
}

static int bit_isset(const uint8_t *bm, uint32_t j)
{
	return (bm[j / 8] >> (j % 8)) & 1u;
}

/* The byte ranges of cell `cell_idx` that agg_diff_preprocess zeroes in the
 * diff (ref:src/object/srv_ec_aggregate.c:1006-1058) -- between and after the
 * new extents, the tail only once some extent has touched the cell
 * (hole_off > 0) -- get `old` copied over `dst`, so old ^ dst is zero there. */
static void for_each_hole(uint64_t len, uint64_t rsize, uint32_t cell_idx, const uint64_t *es,
			  const uint64_t *en, uint32_t n, unsigned char *dst, const unsigned char *old)
{
	const uint64_t cs = (uint64_t)cell_idx * len, ce = cs + len;
	uint64_t hole_off = 0;
	uint32_t i;

	for (i = 0; i < n; i++) {
		const uint64_t estart = es[i], eend = es[i] + en[i];
		uint64_t hole_end;

		if (estart >= ce)
			break;
		if (eend <= cs)
			continue;
		hole_end = cs + hole_off;
		if (estart > hole_end)
			memcpy(dst + hole_off * rsize, old + hole_off * rsize, (estart - hole_end) * rsize);
		hole_off = eend - cs;
	}
	if (hole_off > 0 && hole_off < len)
		memcpy(dst + hole_off * rsize, old + hole_off * rsize, (len - hole_off) * rsize);
}

/* agg_update_parity: parity[r] ^= coef[r][j] * (old_i ^ new_i'), where new_i'
 * is new_i with holes replaced by old_i (so the diff is zero there, exactly
 * the reference's memset of the diff).  (old ^ new') * c == old*c ^ new'*c,
 * so both feed the same device product as two sources with equal
 * coefficients, accumulated into parity. */
int ecg_agg_update_parity(ecg_ctx_t *ctx, uint32_t oc_id, uint64_t cell_recs, uint64_t rsize,
			  const uint8_t *bit_map, uint32_t cell_cnt,
			  const unsigned char *old_cells, const unsigned char *new_cells,
			  const uint64_t *ext_start, const uint64_t *ext_nr, uint32_t n_ext,
			  unsigned char *parity)
{
	unsigned char en[(ECG_MAX_K + ECG_MAX_P) * ECG_MAX_K];
	unsigned char coef[ECG_MAX_P * 2 * ECG_MAX_K];
	unsigned char *src[2 * ECG_MAX_K], *dst[ECG_MAX_P];
	unsigned char *masked = NULL;
	const uint64_t cb = cell_recs * rsize;
	uint32_t i, j;
	int k, p, r, rc;

	rc = ecg_obj_ec_class_kp(oc_id, &k, &p);
	if (rc)
		return rc;
	if (cell_cnt == 0)
		return 0;
	if (cell_cnt > (uint32_t)k || cb == 0 || cb > 0x7fffffffULL || bit_map == NULL ||
	    (n_ext && (ext_start == NULL || ext_nr == NULL)))
		return ecg_fail(-ECG_DER_INVAL, "agg_update_parity: bad arguments");
	if (n_ext) {
		masked = malloc((size_t)cb * cell_cnt);
		if (masked == NULL)
			return ecg_fail(-ECG_DER_NOMEM, "agg_update_parity: malloc");
	}
	ecg_gen_cauchy1(k, p, en);
	for (i = 0, j = 0; i < cell_cnt; i++, j++) {
		const unsigned char *o = old_cells + (size_t)i * cb;
		const unsigned char *nw = new_cells + (size_t)i * cb;

		while (j < (uint32_t)k && !bit_isset(bit_map, j))
			j++;
		if (j >= (uint32_t)k) {
			free(masked);
			return ecg_fail(-ECG_DER_INVAL, "agg_update_parity: bitmap has < %u cells", cell_cnt);
		}
		if (masked) {
			unsigned char *m = masked + (size_t)i * cb;

			memcpy(m, nw, cb);
			for_each_hole(cell_recs, rsize, j, ext_start, ext_nr, n_ext, m, o);
			nw = m;
		}
		src[2 * i] = (unsigned char *)o;
		src[2 * i + 1] = (unsigned char *)nw;
		for (r = 0; r < p; r++) {
			coef[r * 2 * cell_cnt + 2 * i] = en[(k + r) * k + j];
			coef[r * 2 * cell_cnt + 2 * i + 1] = en[(k + r) * k + j];
		}
	}
	for (r = 0; r < p; r++)
		dst[r] = parity + (size_t)r * cb;
	rc = ecg_dropin_product("agg_update_parity", ctx, (int)cb, (int)(2 * cell_cnt), p, coef, src, dst,
				ECG_F_ACCUMULATE);
	free(masked);
	return rc;
}

int ecg_agg_recalc_parity(ecg_ctx_t *ctx, uint32_t oc_id, uint64_t cb, const uint8_t *bit_map,
			  uint32_t cell_cnt, const unsigned char *rbuf, const unsigned char *lbuf,
			  unsigned char *parity)
{
	unsigned char en[(ECG_MAX_K + ECG_MAX_P) * ECG_MAX_K];
	unsigned char *data[ECG_MAX_K], *dst[ECG_MAX_P];
	uint32_t rr = 0, ll = 0;
	int k, p, i, rc;

	rc = ecg_obj_ec_class_kp(oc_id, &k, &p);
	if (rc)
		return rc;
	if (cb == 0 || cb > 0x7fffffffULL || bit_map == NULL || cell_cnt > (uint32_t)k)
		return ecg_fail(-ECG_DER_INVAL, "agg_recalc_parity: bad arguments");
	for (i = 0; i < k; i++) {
		if (bit_isset(bit_map, (uint32_t)i))
			data[i] = (unsigned char *)rbuf + (size_t)rr++ * cb;
		else
			data[i] = (unsigned char *)lbuf + (size_t)ll++ * cb;
	}
	if (rr != cell_cnt)	/* D_ASSERT(r == cell_cnt) in the reference */
		return ecg_fail(-ECG_DER_INVAL, "agg_recalc_parity: bitmap has %u cells, not %u", rr,
				cell_cnt);
	for (i = 0; i < p; i++)
		dst[i] = parity + (size_t)i * cb;
	ecg_gen_cauchy1(k, p, en);
	return ecg_dropin_product("agg_recalc_parity", ctx, (int)cb, k, p, &en[k * k], data, dst, 0);
}

uint64_t ecg_obj_ec_singv_cell_bytes(uint32_t oc_id, uint64_t iod_size)
{
	uint64_t c;
	int k, p;

	if (ecg_obj_ec_class_kp(oc_id, &k, &p))
		return 0;
	c = iod_size / (uint64_t)k + (iod_size % (uint64_t)k != 0);
	return (c + 7) & ~7ull;		/* OBJ_EC_SINGV_CELL_ALIGN */
}

int ecg_obj_ec_singv_encode(uint32_t oc_id, uint64_t iod_size, const unsigned char *value,
			    unsigned char *p_bufs[])
{
	unsigned char en[(ECG_MAX_K + ECG_MAX_P) * ECG_MAX_K];
	unsigned char *data[ECG_MAX_K];
	unsigned char *cells;
	uint64_t cb;
	int k, p, i, rc;

	rc = ecg_obj_ec_class_kp(oc_id, &k, &p);
	if (rc)
		return rc;
	cb = ecg_obj_ec_singv_cell_bytes(oc_id, iod_size);
	if (iod_size == 0 || value == NULL || cb > 0x7fffffffULL)
		return ecg_fail(-ECG_DER_INVAL, "singv_encode: bad arguments");
	for (i = 0; i < p && p_bufs[i] == NULL; i++) {
		p_bufs[i] = malloc(cb);
		if (p_bufs[i] == NULL)
			return ecg_fail(-ECG_DER_NOMEM, "singv_encode: malloc");
	}
	/* the last data cell is zero padded (ref:src/object/cli_ec.c:494-503) */
	cells = calloc((size_t)k, cb);
	if (cells == NULL)
		return ecg_fail(-ECG_DER_NOMEM, "singv_encode: calloc");
	memcpy(cells, value, iod_size);
	for (i = 0; i < k; i++)
		data[i] = cells + (size_t)i * cb;
	ecg_gen_cauchy1(k, p, en);
	rc = ecg_dropin_product("obj_ec_singv_encode", NULL, (int)cb, k, p, &en[k * k], data, p_bufs, 0);
	free(cells);
	return rc;
}

/* ---- stripe / index math, ref:src/object/obj_ec.h:271-350 ---- */
uint64_t ecg_obj_ec_stripe_rec_nr(uint32_t k, uint64_t e_len)
{
	return (uint64_t)k * e_len;
}

uint64_t ecg_obj_ec_cell_bytes(uint64_t e_len, uint64_t iod_size)
{
	return e_len * iod_size;
}

uint32_t ecg_obj_ec_tgt_of_recx_idx(uint64_t idx, uint64_t stripe_rec_nr, uint64_t e_len)
{
	return (uint32_t)((idx % stripe_rec_nr) / e_len);
}

uint64_t ecg_obj_ec_idx_daos2vos(uint64_t idx, uint64_t stripe_rec_nr, uint64_t e_len)
{
	return (idx / stripe_rec_nr) * e_len + idx % e_len;
}

uint64_t ecg_obj_ec_idx_vos2daos(uint64_t vos_idx, uint64_t stripe_rec_nr, uint64_t e_len,
				 uint32_t tgt_idx)
{
	return (vos_idx / e_len) * stripe_rec_nr + (uint64_t)tgt_idx * e_len + vos_idx % e_len;
}

uint64_t ecg_obj_ec_idx_parity2daos(uint64_t vos_off, uint64_t e_len, uint64_t stripe_rec_nr)
{
	return (vos_off / e_len) * stripe_rec_nr;
}

uint32_t ecg_obj_ec_shard_off_by_start(uint32_t tgt_idx, uint32_t tgt_nr, uint32_t start_tgt)
{
	return (tgt_idx + tgt_nr - start_tgt) % tgt_nr;
}
