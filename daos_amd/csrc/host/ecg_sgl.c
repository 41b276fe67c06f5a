/*
 * ecg_sgl.c -- the byte movement around the EC codec on device memory:
 *   - the degraded fetch's stripe list (obj_ec_stripe_list_init and
 *     obj_ec_stripe_list_add, ref:src/object/cli_ec.c:2252-2381);
 *   - the fill-back of recovered records into the user's scatter-gather
 *     list (obj_ec_recov_fill_back + obj_ec_sgl_copy / oes_copy,
 *     ref:src/object/cli_ec.c:2645-2812, over daos_sgl_processor,
 *     ref:src/common/misc.c:313-385);
 *   - the segment list + launcher of ecg_copy_segs_kernel, shared with the
 *     client encode's gather of cells that span iovs (ecg_ptrs.c).
 *
 * The walks over recxs, stripes and iovs touch a few descriptors on the
 * host; they emit (dst, src, len) segments and every byte moves in one
 * launch.
 */
#include <stdlib.h>
#include <string.h>

#include "ecg_internal.h"
#include "../../../include/ecg_daos.h"

int ecg_segs_add(struct ecg_segs *v, uint64_t dst, uint64_t src, uint64_t len)
{
	ecg_copy_seg_t *s;

	if (len == 0)
		return 0;
	if (v->n == v->cap) {
		size_t cap = v->cap ? 2 * v->cap : 64;

		if (v->fixed)
			return ecg_fail(-ECG_DER_INVAL, "copy segments: more than the %zu counted", v->cap);
		s = realloc(v->seg, cap * sizeof(*s));
		if (s == NULL)
			return ecg_fail(-ECG_DER_NOMEM, "copy segments: realloc");
		v->seg = s;
		v->cap = cap;
	}
	s = &v->seg[v->n++];
	s->dst = dst;
	s->src = src;
	s->len = len;
	s->tile0 = v->tiles;
	v->tiles += ecg_k_copy_tiles(dst, len);
	return 0;
}

void ecg_segs_fini(struct ecg_segs *v)
{
	if (!v->fixed)
		free(v->seg);
	memset(v, 0, sizeof(*v));
}

int ecg_segs_launch(const struct ecg_segs *v, const void *segs_dev, hipStream_t st)
{
	uint32_t kid = 0;
	int ke;

	if (v->n == 0)
		return 0;
	if (v->n > UINT32_MAX)
		return ecg_fail(-ECG_DER_INVAL, "copy segments: %zu segments", v->n);
	ke = ecg_k_launch_copy_segs((const ecg_copy_seg_t *)segs_dev, (uint32_t)v->n, v->tiles, (void *)st,
				    &kid);
	if (ke != 0)
		return ecg_hip_fail((hipError_t)ke, "segment copy launch");
	ecg_set_last_kernel(ecg_k_kernel_name(kid));
	return 0;
}

/* Stage v's table through a scratch slot and launch (ctx->lock held). */
static int segs_submit(ecg_ctx_t *ctx, const struct ecg_segs *v, hipStream_t st)
{
	const size_t b = v->n * sizeof(ecg_copy_seg_t);
	struct ecg_scratch_slot *sc = NULL;
	int rc;

	if (v->n == 0)
		return 0;
	rc = ecg_scratch_reserve(ctx, b, b, &sc);
	if (rc)
		return rc;
	memcpy(sc->pin, v->seg, b);
	rc = ecg_table_upload(sc, b, st, "segment table");
	if (rc == 0)
		rc = ecg_segs_launch(v, sc->dev, st);
	if (hipEventRecord(sc->done, st) == hipSuccess)	/* the H2D may still read pin */
		sc->pending = 1;
	return rc;
}

/* ---- sgl bookkeeping (daos_sgl_get_bytes with check_buf = true) -------- */

struct sgl_idx {
	uint32_t iov_idx;
	uint64_t iov_offset;
};

/* The next piece of at most `req` bytes at idx, idx advanced past it.
 * Returns 0 with *have = 0 when the sgl is already exhausted; *end = 1 once
 * idx has reached the end (ref:src/common/misc.c:313-356).  A zero-capacity
 * iov yields an empty piece and is stepped over. */
static uint64_t sgl_get_bytes(const ecg_sgl_t *sgl, struct sgl_idx *idx, uint64_t req, uint64_t *addr,
			      int *have, int *end)
{
	uint64_t len, n;

	if (idx->iov_idx >= sgl->sg_nr) {
		*have = 0;
		*end = 1;
		return 0;
	}
	len = sgl->sg_iovs[idx->iov_idx].iov_buf_len;
	*addr = (uint64_t)(uintptr_t)sgl->sg_iovs[idx->iov_idx].iov_buf + idx->iov_offset;
	n = len - idx->iov_offset;
	if (req < n)
		n = req;
	idx->iov_offset += n;
	if (idx->iov_offset == len) {
		idx->iov_idx++;
		idx->iov_offset = 0;
	}
	*have = 1;
	*end = idx->iov_idx == sgl->sg_nr;
	return n;
}

/* Where daos_sgl_processor leaves idx after skipping `off` > 0 bytes
 * (ref:src/common/misc.c:359-385), found by binary search over the prefix
 * sums of the iov capacities (cap[i] = pre[i+1] - pre[i]) instead of the
 * reference's walk from iov 0 on every copy: the first iov whose end
 * reaches `off`, or the one after it when `off` is exactly that end. */
static struct sgl_idx sgl_skip(const ecg_sgl_t *sgl, const uint64_t *pre, uint64_t off)
{
	struct sgl_idx idx = {sgl->sg_nr, 0};
	uint32_t lo = 0, hi = sgl->sg_nr;

	if (off == 0)
		return (struct sgl_idx){0, 0};
	if (sgl->sg_nr == 0 || pre[sgl->sg_nr] < off)
		return idx;				/* sgl exhausted */
	while (lo < hi) {				/* smallest i: pre[i+1] >= off */
		const uint32_t mid = lo + (hi - lo) / 2;

		if (pre[mid + 1] >= off)
			hi = mid;
		else
			lo = mid + 1;
	}
	if (pre[lo + 1] == off)
		return (struct sgl_idx){lo + 1, 0};
	return (struct sgl_idx){lo, off - pre[lo]};
}

/* obj_ec_sgl_copy (ref:src/object/cli_ec.c:2681-2707): skip `off` bytes of
 * the sgl, then copy `size` bytes from src into it; oes_copy's iov_len
 * updates (:2653-2679) and the final sg_nr_out.  Copies what fits when the
 * sgl is short, as the reference does. */
static int sgl_copy(ecg_sgl_t *sgl, const uint64_t *pre, uint64_t off, uint64_t src, uint64_t size,
		    struct ecg_segs *v)
{
	struct sgl_idx idx = sgl_skip(sgl, pre, off);
	uint64_t req, copied = 0, addr = 0, n;
	int have, end = 0, rc;

	req = size;
	end = 0;
	while (req > 0 && !end) {
		n = sgl_get_bytes(sgl, &idx, req, &addr, &have, &end);
		req -= n;
		if (!have)
			continue;
		rc = ecg_segs_add(v, addr, src + copied, n);
		if (rc)
			return rc;
		copied += n;
		if (idx.iov_offset == 0) {
			ecg_iov_t *iov = &sgl->sg_iovs[idx.iov_idx - 1];

			iov->iov_len = iov->iov_buf_len;
		} else {
			ecg_iov_t *iov = &sgl->sg_iovs[idx.iov_idx];

			if (iov->iov_len < idx.iov_offset)
				iov->iov_len = idx.iov_offset;
		}
	}
	sgl->sg_nr_out = idx.iov_offset == 0 ? idx.iov_idx : idx.iov_idx + 1;
	return 0;
}

static int recx_overlap(const ecg_recx_t *a, const ecg_recx_t *b)
{
	return a->rx_idx < b->rx_idx + b->rx_nr && b->rx_idx < a->rx_idx + a->rx_nr;
}

static uint64_t min64(uint64_t a, uint64_t b)
{
	return a < b ? a : b;
}

/* The reference's fill-back walk (ref:src/object/cli_ec.c:2731-2811). */
static int fill_back_walk(uint64_t iod_size, const ecg_recx_t *iod_recxs, uint32_t iod_nr, ecg_sgl_t *sgl,
			  const uint64_t *pre, const ecg_recx_ep_t *recov, uint32_t recov_nr, const ecg_recx_ep_t *stripes,
			  uint32_t stripe_nr, uint64_t sbuf, uint64_t stripe_total_sz, uint64_t stripe_rec_nr,
			  struct ecg_segs *v)
{
	for (uint32_t i = 0; i < recov_nr; i++) {
		ecg_recx_t rr = recov[i].re_recx, ovl = {0, 0};

		for (;;) {	/* "again:" -- the rest of rr after one iod recx */
			uint64_t rec_nr = 0, iod_off, stripe_total_nr = 0;
			int overlapped = 0, done = 0;

			for (uint32_t j = 0; j < iod_nr; j++) {
				const ecg_recx_t *ir = &iod_recxs[j];

				if (!recx_overlap(&rr, ir)) {
					rec_nr += ir->rx_nr;
					continue;
				}
				overlapped = 1;
				if (rr.rx_idx < ir->rx_idx)
					return ecg_fail(-ECG_DER_INVAL,
							"fill_back: recov recx %lu starts before iod recx %lu",
							(unsigned long)rr.rx_idx, (unsigned long)ir->rx_idx);
				ovl.rx_idx = rr.rx_idx;
				ovl.rx_nr = min64(rr.rx_idx + rr.rx_nr, ir->rx_idx + ir->rx_nr) - ovl.rx_idx;
				rec_nr += rr.rx_idx - ir->rx_idx;
				break;
			}
			if (!overlapped)
				break;
			iod_off = rec_nr * iod_size;

			/* the recx per stripe: copy from the recovered full stripe */
			for (uint32_t j = 0; j < stripe_nr && !done; j++) {
				ecg_recx_t sr = stripes[j].re_recx;
				const uint64_t ns = sr.rx_nr / stripe_rec_nr;

				sr.rx_nr = stripe_rec_nr;
				for (uint64_t s = 0; s < ns; s++) {
					const uint64_t soff = stripe_total_nr * stripe_total_sz;

					if (recx_overlap(&ovl, &sr)) {
						uint64_t cnt;
						int rc;

						if (ovl.rx_idx < sr.rx_idx)
							return ecg_fail(-ECG_DER_INVAL,
									"fill_back: record %lu not in the stripe list",
									(unsigned long)ovl.rx_idx);
						cnt = min64(ovl.rx_idx + ovl.rx_nr, sr.rx_idx + sr.rx_nr) - ovl.rx_idx;
						rc = sgl_copy(sgl, pre, iod_off,
							      sbuf + soff + iod_size * (ovl.rx_idx - sr.rx_idx),
							      cnt * iod_size, v);
						if (rc)
							return rc;
						iod_off += cnt * iod_size;
						ovl.rx_idx += cnt;
						ovl.rx_nr -= cnt;
						if (ovl.rx_nr == 0) {
							done = 1;
							break;
						}
					}
					sr.rx_idx += stripe_rec_nr;
					stripe_total_nr++;
				}
			}
			if (ovl.rx_nr != 0)
				return ecg_fail(-ECG_DER_INVAL, "fill_back: records %lu+%lu not in the stripe list",
						(unsigned long)ovl.rx_idx, (unsigned long)ovl.rx_nr);
			if (ovl.rx_idx >= rr.rx_idx + rr.rx_nr)
				break;
			rr.rx_nr = rr.rx_idx + rr.rx_nr - ovl.rx_idx;
			rr.rx_idx = ovl.rx_idx;
		}
	}
	return 0;
}

int ecg_obj_ec_recov_fill_back(ecg_ctx_t *ctx, uint64_t iod_size, int singv, const ecg_recx_t *iod_recxs,
			       uint32_t iod_nr, ecg_sgl_t *sgl, const ecg_recx_ep_t *recov, uint32_t recov_nr,
			       const ecg_recx_ep_t *stripes, uint32_t stripe_nr, const void *stripe_buf,
			       uint64_t stripe_total_sz, uint64_t stripe_rec_nr, void *stream)
{
	const uint64_t sbuf = (uint64_t)(uintptr_t)stripe_buf;
	struct ecg_segs v = {0};
	uint64_t *pre;
	hipStream_t st;
	int rc;

	if (ctx == NULL || sgl == NULL || stripe_buf == NULL || (sgl->sg_nr && sgl->sg_iovs == NULL))
		return ecg_fail(-ECG_DER_INVAL, "fill_back: NULL argument");
	pre = malloc(((size_t)sgl->sg_nr + 1) * sizeof(*pre));	/* iov capacity prefix sums */
	if (pre == NULL)
		return ecg_fail(-ECG_DER_NOMEM, "fill_back: malloc");
	pre[0] = 0;
	for (uint32_t i = 0; i < sgl->sg_nr; i++)
		pre[i + 1] = pre[i] + sgl->sg_iovs[i].iov_buf_len;
	if (singv) {
		rc = sgl_copy(sgl, pre, 0, sbuf, iod_size, &v);		/* :2725-2729 */
	} else {
		rc = 0;
		if ((iod_nr && iod_recxs == NULL) || (recov_nr && recov == NULL) ||
		    (stripe_nr && stripes == NULL) || stripe_rec_nr == 0)
			rc = ecg_fail(-ECG_DER_INVAL, "fill_back: bad recx lists");
		for (uint32_t j = 0; rc == 0 && j < stripe_nr; j++)
			if (stripes[j].re_recx.rx_nr % stripe_rec_nr)		/* :2767 */
				rc = ecg_fail(-ECG_DER_INVAL, "fill_back: stripe recx %u is not whole stripes", j);
		if (rc == 0)
			rc = fill_back_walk(iod_size, iod_recxs, iod_nr, sgl, pre, recov, recov_nr, stripes,
					    stripe_nr, sbuf, stripe_total_sz, stripe_rec_nr, &v);
	}
	free(pre);
	if (rc == 0 && v.n) {
		rc = ecg_ctx_enter(ctx);
		if (rc == 0) {
			st = ecg_pick_stream(ctx, stream);
			pthread_mutex_lock(&ctx->lock);
			rc = segs_submit(ctx, &v, st);
			pthread_mutex_unlock(&ctx->lock);
		}
	}
	ecg_segs_fini(&v);
	return rc;
}

/* obj_ec_singv_one_tgt (ref:src/object/obj_ec.h:409-419): a single value of at
 * most OBJ_EC_SINGV_EVENDIST_SZ bytes lives on one target, unencoded. */
static int singv_one_tgt(uint64_t iod_size, const ecg_sgl_t *sgl, int k)
{
	const uint64_t evendist = ((uint64_t)k / 8 + 1) * 4096;	/* OBJ_EC_SINGV_EVENDIST_SZ */
	uint64_t buf = 0;

	if (iod_size != 0 && iod_size <= evendist)
		return 1;
	if (sgl == NULL)
		return 0;
	for (uint32_t i = 0; i < sgl->sg_nr; i++)
		buf += sgl->sg_iovs[i].iov_buf_len;
	return buf <= evendist;
}

int ecg_obj_ec_recov_data_dev(ecg_ctx_t *ctx, uint32_t oc_id, uint64_t e_len,
			      const struct ecg_obj_ec_recov_codec *recov, ecg_recov_iod_t *iods, uint32_t iod_nr,
			      void *stream)
{
	int k, p, rc;

	if (ctx == NULL || recov == NULL || (iod_nr && iods == NULL))
		return ecg_fail(-ECG_DER_INVAL, "recov_data_dev: NULL argument");
	rc = ecg_obj_ec_class_kp(oc_id, &k, &p);
	if (rc)
		return rc;
	if (recov->k != k || recov->p != p || e_len == 0)
		return ecg_fail(-ECG_DER_INVAL, "recov_data_dev: codec %d+%d for class %d+%d, e_len %lu",
				recov->k, recov->p, k, p, (unsigned long)e_len);
	for (uint32_t i = 0; i < iod_nr; i++) {		/* ref:src/object/cli_ec.c:2839-2884 */
		ecg_recov_iod_t *io = &iods[i];
		const uint64_t srn = (uint64_t)k * e_len;
		uint64_t cell, nst = 0;

		if (!io->singv && (io->recov_nr == 0 || io->stripe_nr == 0))
			continue;
		cell = io->singv ? ecg_obj_ec_singv_cell_bytes(oc_id, io->iod_size) : e_len * io->iod_size;
		if (io->singv) {
			nst = singv_one_tgt(io->iod_size, io->sgl, k) ? 0 : 1;
		} else {
			for (uint32_t j = 0; j < io->stripe_nr; j++) {
				if (io->stripes[j].re_recx.rx_nr % srn)
					return ecg_fail(-ECG_DER_INVAL, "recov_data_dev: stripe recx %u of iod %u", j,
							i);
				nst += io->stripes[j].re_recx.rx_nr / srn;
			}
		}
		if (nst > UINT32_MAX)
			return ecg_fail(-ECG_DER_INVAL, "recov_data_dev: %lu stripes", (unsigned long)nst);
		if (nst) {
			rc = ecg_recover(ctx, k, p, cell, (uint32_t)nst, io->stripe_buf, (int64_t)(cell * (k + p)),
					 recov->er_err_list, (int)recov->er_nerrs, stream);
			if (rc)
				return rc;
		}
		rc = ecg_obj_ec_recov_fill_back(ctx, io->iod_size, (int)io->singv, io->iod_recxs, io->iod_nr, io->sgl,
						io->recov, io->recov_nr, io->stripes, io->stripe_nr, io->stripe_buf,
						cell * (uint64_t)(k + p), srn, stream);
		if (rc)
			return rc;
	}
	return 0;
}

/* ---- stripe list (obj_ec_stripe_list_init / _add) ----------------------- */

/* obj_ec_stripe_list_add (ref:src/object/cli_ec.c:2252-2310) */
static int stripe_list_add(ecg_recx_ep_t *list, uint32_t *n, uint32_t cap, const ecg_recx_ep_t *sr)
{
	for (uint32_t i = 0; i < *n; i++) {
		ecg_recx_ep_t *e = &list[i];
		uint64_t start, end;

		if (!recx_overlap(&e->re_recx, &sr->re_recx)) {
			if (e->re_ep != sr->re_ep)
				continue;
			/* merge adjacent stripe for same shadow ep */
			if (e->re_recx.rx_idx + e->re_recx.rx_nr == sr->re_recx.rx_idx) {
				e->re_recx.rx_nr += sr->re_recx.rx_nr;
				return 0;
			} else if (sr->re_recx.rx_idx + sr->re_recx.rx_nr == e->re_recx.rx_idx) {
				e->re_recx.rx_idx = sr->re_recx.rx_idx;
				e->re_recx.rx_nr += sr->re_recx.rx_nr;
				return 0;
			}
			continue;
		}
		if (e->re_ep < sr->re_ep)	/* overlapped: keep the higher epoch */
			e->re_ep = sr->re_ep;
		start = min64(e->re_recx.rx_idx, sr->re_recx.rx_idx);
		end = e->re_recx.rx_idx + e->re_recx.rx_nr;
		if (end < sr->re_recx.rx_idx + sr->re_recx.rx_nr)
			end = sr->re_recx.rx_idx + sr->re_recx.rx_nr;
		e->re_recx.rx_nr = end - start;
		e->re_recx.rx_idx = start;
		return 0;
	}
	if (*n >= cap)
		return ecg_fail(-ECG_DER_INVAL, "stripe_list: capacity %u exceeded", cap);
	list[(*n)++] = *sr;
	return 0;
}

int ecg_obj_ec_stripe_list_init(uint64_t stripe_rec_nr, const ecg_recx_ep_t *recx, uint32_t recx_nr,
				ecg_recx_ep_t *stripes, uint32_t cap, uint32_t *stripe_nr)
{
	uint32_t n = 0;
	int rc;

	if (stripe_rec_nr == 0 || stripe_nr == NULL || (recx_nr && recx == NULL) || (cap && stripes == NULL))
		return ecg_fail(-ECG_DER_INVAL, "stripe_list: bad arguments");
	for (uint32_t i = 0; i < recx_nr; i++) {		/* :2355-2372 */
		ecg_recx_ep_t sr = recx[i];
		uint64_t start, end;

		if (sr.re_type != ECG_DRT_SHADOW)
			continue;
		start = sr.re_recx.rx_idx / stripe_rec_nr * stripe_rec_nr;
		end = (sr.re_recx.rx_idx + sr.re_recx.rx_nr + stripe_rec_nr - 1) / stripe_rec_nr * stripe_rec_nr;
		sr.re_recx.rx_idx = start;
		sr.re_recx.rx_nr = end - start;
		rc = stripe_list_add(stripes, &n, cap, &sr);
		if (rc)
			return rc;
	}
	*stripe_nr = n;
	return 0;
}
