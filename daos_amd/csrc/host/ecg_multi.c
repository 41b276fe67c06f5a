/*
 * ecg_multi.c -- stripe sharding over several devices in one process
 * (include/ecg_multi.h).
 *
 * One worker thread per shard, each owning an ecg_ctx_t on its device.  A
 * call publishes one job (function + arguments) to every worker, each runs
 * it on its stripe range, and the caller waits for all of them: the
 * reference's per-stripe loops (ref:src/object/cli_ec.c:627-659,
 * ref:src/object/srv_obj_migrate.c:1116-1177) have no cross-stripe data, so
 * the shards never talk to each other.
 */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../../include/ecg_multi.h"
#include "../../../include/ecg_csum.h"
#include "ecg_internal.h"

struct mjob {
	int op;
	int k, p, nerrs;
	uint64_t C;
	uint32_t S;			/* host ops: the whole batch */
	const uint32_t *nstripes;	/* device ops: per shard */
	const void *const *src;
	const void *const *src2;	/* updates: new cells (src = old cells) */
	void *const *dst;
	void *const *aux;		/* checksum outputs per shard */
	const void *hsrc;
	void *hdst;
	int64_t s1, s2, s3, s4;
	const uint32_t *err;		/* erasures; updates: updated cell indices */
	uint32_t chunk;
	unsigned flags;
	/* checksums */
	int csum_type;
	uint64_t chunksize, rec_size;
	/* parity-shard rebuild */
	uint32_t oc_id, shard;
	uint64_t e_len, offset, size;
	int encode;
	ecg_migrate_piece_t *pieces;
	const uint32_t *first;		/* per shard: first piece index, [n + 1] */
};

enum { MOP_NOP, MOP_ENCODE, MOP_RECOVER, MOP_SYNC, MOP_ENCODE_HOST, MOP_RECOVER_HOST, MOP_ENCODE_CSUM,
       MOP_RECOVER_CSUM, MOP_UPDATE, MOP_MIGRATE };

struct mworker {
	struct ecg_multi *m;
	int idx;
	ecg_ctx_t *ctx;
	pthread_t th;
	int started;
	int numa_node;		/* node the worker runs on, -1 = not pinned */
	int rc;
	char err[256];		/* the shard's ecg_strerror() when rc != 0 */
};

struct ecg_multi {
	int n;
	struct mworker w[ECG_MULTI_MAX];
	pthread_mutex_t call;		/* one call at a time */
	pthread_mutex_t lock;
	pthread_cond_t cv_go, cv_done;
	uint64_t gen;
	int pending, stop;
	struct mjob job;
};

int ecg_parse_devices(const char *spec, int *dev, int max)
{
	int n = 0;

	if (spec == NULL || *spec == '\0' || strcmp(spec, "all") == 0) {
		int nd = ecg_device_count();

		for (n = 0; n < nd && n < max; n++)
			dev[n] = n;
		return n;
	}
	while (*spec && n < max) {
		char *end;
		long v = strtol(spec, &end, 10);

		if (end == spec || v < 0)
			return -ECG_DER_INVAL;
		dev[n++] = (int)v;
		spec = end;
		while (*spec == ',' || *spec == ' ')
			spec++;
	}
	return n;
}

int ecg_multi_range(const ecg_multi_t *m, uint32_t S, int i, uint32_t *first, uint32_t *count)
{
	uint32_t base, extra, f, c;

	if (m == NULL || i < 0 || i >= m->n || first == NULL || count == NULL)
		return ecg_fail(-ECG_DER_INVAL, "multi_range: bad argument");
	base = S / (uint32_t)m->n;
	extra = S % (uint32_t)m->n;
	c = base + ((uint32_t)i < extra ? 1u : 0u);
	f = base * (uint32_t)i + ((uint32_t)i < extra ? (uint32_t)i : extra);
	*first = f;
	*count = c;
	return 0;
}

static int run_one(struct ecg_multi *m, struct mworker *w)
{
	const struct mjob *j = &m->job;
	ecg_ctx_t *ctx = w->ctx;
	uint32_t s0 = 0, ns = 0;
	int rc = 0;

	switch (j->op) {
	case MOP_NOP:
		return 0;
	case MOP_ENCODE:
		if (j->nstripes[w->idx] == 0)
			return 0;
		rc = ecg_encode(ctx, j->k, j->p, j->C, j->nstripes[w->idx], j->src[w->idx], j->s1,
				j->dst[w->idx], j->s2, j->s3, NULL);
		break;
	case MOP_RECOVER:
		if (j->nstripes[w->idx] == 0)
			return 0;
		rc = ecg_recover(ctx, j->k, j->p, j->C, j->nstripes[w->idx], j->dst[w->idx], j->s1,
				 j->err, j->nerrs, NULL);
		break;
	case MOP_ENCODE_CSUM:
		if (j->nstripes[w->idx] == 0)
			return 0;
		rc = ecg_encode_csum(ctx, j->k, j->p, j->C, j->nstripes[w->idx], j->src[w->idx], j->s1,
				     j->dst[w->idx], j->s2, j->s3, j->csum_type, j->chunksize, j->rec_size,
				     j->aux[w->idx], NULL);
		break;
	case MOP_RECOVER_CSUM:
		if (j->nstripes[w->idx] == 0)
			return 0;
		rc = ecg_recover_csum(ctx, j->k, j->p, j->C, j->nstripes[w->idx], j->dst[w->idx], j->s1, j->err,
				      j->nerrs, j->csum_type, j->chunksize, j->rec_size, j->aux[w->idx], NULL);
		break;
	case MOP_UPDATE:
		if (j->nstripes[w->idx] == 0)
			return 0;
		rc = ecg_update(ctx, j->k, j->p, j->C, j->nstripes[w->idx], j->nerrs, j->err, j->src[w->idx],
				j->src2[w->idx], j->s4, j->dst[w->idx], j->s2,
				j->s3, NULL);
		break;
	case MOP_MIGRATE: {
		uint64_t off = 0, sz = 0;
		uint32_t got = 0, cap = j->first[w->idx + 1] - j->first[w->idx];

		(void)ecg_multi_migrate_range(m, j->oc_id, j->e_len, j->rec_size, j->offset, j->size, j->encode,
					      w->idx, &off, &sz);
		if (sz == 0)
			return 0;
		rc = ecg_migrate_update_parity(ctx, j->oc_id, j->e_len, j->rec_size, j->shard, j->src[w->idx], off,
					       sz, j->encode, j->csum_type, j->chunksize, j->dst[w->idx],
					       j->aux ? j->aux[w->idx] : NULL, j->pieces + j->first[w->idx], cap,
					       &got, NULL);
		if (rc == 0 && got != cap)
			rc = ecg_fail(-ECG_DER_INVAL, "multi_migrate: shard %d cut %u pieces, planned %u", w->idx,
				      got, cap);
		break;
	}
	case MOP_SYNC:
		return ecg_stream_sync(ctx, NULL);
	case MOP_ENCODE_HOST:
		(void)ecg_multi_range(m, j->S, w->idx, &s0, &ns);
		if (ns == 0)
			return 0;
		return ecg_encode_host_rows(ctx, j->k, j->p, j->C, ns,
					    (const unsigned char *)j->hsrc + (size_t)s0 * j->k * j->C,
					    (unsigned char *)j->hdst + (size_t)s0 * j->C,
					    (size_t)j->S * j->C, j->chunk);
	case MOP_RECOVER_HOST:
		(void)ecg_multi_range(m, j->S, w->idx, &s0, &ns);
		if (ns == 0)
			return 0;
		return ecg_recover_host(ctx, j->k, j->p, j->C, ns,
					(unsigned char *)j->hdst + (size_t)s0 * (j->k + j->p) * j->C, j->err,
					j->nerrs, j->chunk);
	default:
		return ecg_fail(-ECG_DER_INVAL, "multi: bad op %d", j->op);
	}
	if (rc == 0 && !(j->flags & ECG_MULTI_ASYNC))
		rc = ecg_stream_sync(ctx, NULL);
	return rc;
}

static void *worker_main(void *arg)
{
	struct mworker *w = arg;
	struct ecg_multi *m = w->m;
	uint64_t seen = 0;

	/* on the CPUs of the device's NUMA node: the shard's host-side copies
	 * and staging then use the memory and PCIe root of its own socket */
	w->numa_node = ecg_numa_bind_thread(ecg_ctx_device(w->ctx), NULL);
	pthread_mutex_lock(&m->lock);
	for (;;) {
		while (!m->stop && m->gen == seen)
			pthread_cond_wait(&m->cv_go, &m->lock);
		if (m->stop)
			break;
		seen = m->gen;
		pthread_mutex_unlock(&m->lock);
		ecg_trace_push("ecg:multi_shard");
		w->rc = run_one(m, w);
		ecg_trace_pop();
		if (w->rc)
			snprintf(w->err, sizeof(w->err), "%s", ecg_strerror());
		pthread_mutex_lock(&m->lock);
		if (--m->pending == 0)
			pthread_cond_broadcast(&m->cv_done);
	}
	pthread_mutex_unlock(&m->lock);
	return NULL;
}

/* Publish m->job (filled by the caller under m->call) to every worker and
 * wait for all; the first failing shard's code wins. */
static int run_all(struct ecg_multi *m)
{
	int i, rc = 0;

	pthread_mutex_lock(&m->lock);
	m->pending = m->n;
	m->gen++;
	pthread_cond_broadcast(&m->cv_go);
	while (m->pending > 0)
		pthread_cond_wait(&m->cv_done, &m->lock);
	pthread_mutex_unlock(&m->lock);
	for (i = 0; i < m->n && rc == 0; i++)
		if (m->w[i].rc)
			rc = ecg_fail(m->w[i].rc, "shard %d (device %d): %s", i,
				      ecg_ctx_device(m->w[i].ctx), m->w[i].err);
	return rc;
}

void ecg_multi_destroy(ecg_multi_t *m)
{
	int i;

	if (m == NULL)
		return;
	pthread_mutex_lock(&m->lock);
	m->stop = 1;
	pthread_cond_broadcast(&m->cv_go);
	pthread_mutex_unlock(&m->lock);
	for (i = 0; i < m->n; i++) {
		if (m->w[i].started)
			pthread_join(m->w[i].th, NULL);
		ecg_ctx_destroy(m->w[i].ctx);
	}
	pthread_mutex_destroy(&m->call);
	pthread_mutex_destroy(&m->lock);
	pthread_cond_destroy(&m->cv_go);
	pthread_cond_destroy(&m->cv_done);
	free(m);
}

int ecg_multi_create(const int *devices, int n, ecg_multi_t **out)
{
	int dev[ECG_MULTI_MAX];
	struct ecg_multi *m;
	int i, rc = 0;

	if (out == NULL)
		return ecg_fail(-ECG_DER_INVAL, "multi_create: NULL out");
	*out = NULL;
	if (devices == NULL || n <= 0) {
		n = ecg_parse_devices(getenv("ECG_DEVICES"), dev, ECG_MULTI_MAX);
		if (n < 0)
			return ecg_fail(-ECG_DER_INVAL, "multi_create: bad ECG_DEVICES '%s'",
					getenv("ECG_DEVICES"));
		if (n == 0)
			return ecg_fail(-ECG_DER_NOSYS, "multi_create: no gfx950 device");
	} else {
		if (n > ECG_MULTI_MAX)
			return ecg_fail(-ECG_DER_INVAL, "multi_create: %d shards > %d", n, ECG_MULTI_MAX);
		memcpy(dev, devices, sizeof(int) * (size_t)n);
	}
	m = calloc(1, sizeof(*m));
	if (m == NULL)
		return ecg_fail(-ECG_DER_NOMEM, "multi_create: calloc");
	pthread_mutex_init(&m->call, NULL);
	pthread_mutex_init(&m->lock, NULL);
	pthread_cond_init(&m->cv_go, NULL);
	pthread_cond_init(&m->cv_done, NULL);
	for (i = 0; i < n && rc == 0; i++) {
		m->w[i].m = m;
		m->w[i].idx = i;
		rc = ecg_ctx_create(dev[i], &m->w[i].ctx);
		if (rc == 0)
			m->n = i + 1;
	}
	for (i = 0; i < m->n && rc == 0; i++) {
		if (pthread_create(&m->w[i].th, NULL, worker_main, &m->w[i]) != 0)
			rc = ecg_fail(-ECG_DER_NOMEM, "multi_create: pthread_create");
		else
			m->w[i].started = 1;
	}
	if (rc == 0) {		/* every worker has started (and bound itself to its node) */
		m->job = (struct mjob){.op = MOP_NOP};
		rc = run_all(m);
	}
	if (rc) {
		ecg_multi_destroy(m);
		return rc;
	}
	*out = m;
	return 0;
}

int ecg_multi_count(const ecg_multi_t *m)
{
	return m ? m->n : 0;
}

int ecg_multi_numa_node(const ecg_multi_t *m, int i)
{
	return m && i >= 0 && i < m->n ? m->w[i].numa_node : -1;
}

ecg_ctx_t *ecg_multi_ctx(ecg_multi_t *m, int i)
{
	return m && i >= 0 && i < m->n ? m->w[i].ctx : NULL;
}

static int check_common(ecg_multi_t *m, int k, int p)
{
	if (m == NULL)
		return ecg_fail(-ECG_DER_INVAL, "multi: NULL handle");
	if (k < 1 || k > ECG_MAX_K || p < 1 || p > ECG_MAX_P)
		return ecg_fail(-ECG_DER_INVAL, "multi: bad k=%d p=%d", k, p);
	return 0;
}

int ecg_multi_encode(ecg_multi_t *m, int k, int p, uint64_t C, const uint32_t *nstripes,
		     const void *const *data, int64_t dstride, void *const *parity, int64_t pcell,
		     int64_t pstripe, unsigned flags)
{
	int rc = check_common(m, k, p);

	if (rc)
		return rc;
	if (nstripes == NULL || data == NULL || parity == NULL)
		return ecg_fail(-ECG_DER_INVAL, "multi_encode: NULL array");
	pthread_mutex_lock(&m->call);
	m->job = (struct mjob){.op = MOP_ENCODE, .k = k, .p = p, .C = C, .nstripes = nstripes,
			       .src = data, .dst = parity, .s1 = dstride, .s2 = pcell, .s3 = pstripe,
			       .flags = flags};
	rc = run_all(m);
	pthread_mutex_unlock(&m->call);
	return rc;
}

int ecg_multi_recover(ecg_multi_t *m, int k, int p, uint64_t C, const uint32_t *nstripes,
		      void *const *stripes, int64_t stride, const uint32_t *err_list, int nerrs,
		      unsigned flags)
{
	int rc = check_common(m, k, p);

	if (rc)
		return rc;
	if (nstripes == NULL || stripes == NULL || err_list == NULL)
		return ecg_fail(-ECG_DER_INVAL, "multi_recover: NULL array");
	if (nerrs > p)
		return ecg_fail(-ECG_DER_DATA_LOSS, "multi_recover: %d erasures > p=%d", nerrs, p);
	pthread_mutex_lock(&m->call);
	m->job = (struct mjob){.op = MOP_RECOVER, .k = k, .p = p, .C = C, .nstripes = nstripes,
			       .dst = stripes, .s1 = stride, .err = err_list, .nerrs = nerrs,
			       .flags = flags};
	rc = run_all(m);
	pthread_mutex_unlock(&m->call);
	return rc;
}

int ecg_multi_sync(ecg_multi_t *m)
{
	int rc;

	if (m == NULL)
		return ecg_fail(-ECG_DER_INVAL, "multi_sync: NULL handle");
	pthread_mutex_lock(&m->call);
	m->job = (struct mjob){.op = MOP_SYNC};
	rc = run_all(m);
	pthread_mutex_unlock(&m->call);
	return rc;
}

int ecg_multi_encode_host(ecg_multi_t *m, int k, int p, uint64_t C, uint32_t S, const void *data,
			  void *parity, uint32_t chunk)
{
	int rc = check_common(m, k, p);

	if (rc)
		return rc;
	if (data == NULL || parity == NULL)
		return ecg_fail(-ECG_DER_INVAL, "multi_encode_host: NULL buffer");
	pthread_mutex_lock(&m->call);
	m->job = (struct mjob){.op = MOP_ENCODE_HOST, .k = k, .p = p, .C = C, .S = S, .hsrc = data,
			       .hdst = parity, .chunk = chunk};
	rc = run_all(m);
	pthread_mutex_unlock(&m->call);
	return rc;
}

int ecg_multi_recover_host(ecg_multi_t *m, int k, int p, uint64_t C, uint32_t S, void *stripes,
			   const uint32_t *err_list, int nerrs, uint32_t chunk)
{
	int rc = check_common(m, k, p);

	if (rc)
		return rc;
	if (stripes == NULL || err_list == NULL)
		return ecg_fail(-ECG_DER_INVAL, "multi_recover_host: NULL argument");
	if (nerrs > p)
		return ecg_fail(-ECG_DER_DATA_LOSS, "multi_recover_host: %d erasures > p=%d", nerrs, p);
	pthread_mutex_lock(&m->call);
	m->job = (struct mjob){.op = MOP_RECOVER_HOST, .k = k, .p = p, .C = C, .S = S, .hdst = stripes,
			       .err = err_list, .nerrs = nerrs, .chunk = chunk};
	rc = run_all(m);
	pthread_mutex_unlock(&m->call);
	return rc;
}

/* ---- rebuild / aggregation ops ------------------------------------------- */
int ecg_multi_encode_csum(ecg_multi_t *m, int k, int p, uint64_t C, const uint32_t *nstripes,
			  const void *const *data, int64_t dstride, void *const *parity, int64_t pcell,
			  int64_t pstripe, int type, uint64_t chunksize, uint64_t rec_size, void *const *csums,
			  unsigned flags)
{
	int rc = check_common(m, k, p);

	if (rc)
		return rc;
	if (nstripes == NULL || data == NULL || parity == NULL || csums == NULL)
		return ecg_fail(-ECG_DER_INVAL, "multi_encode_csum: NULL array");
	pthread_mutex_lock(&m->call);
	m->job = (struct mjob){.op = MOP_ENCODE_CSUM, .k = k, .p = p, .C = C, .nstripes = nstripes,
			       .src = data, .dst = parity, .aux = csums, .s1 = dstride, .s2 = pcell,
			       .s3 = pstripe, .csum_type = type, .chunksize = chunksize, .rec_size = rec_size,
			       .flags = flags};
	rc = run_all(m);
	pthread_mutex_unlock(&m->call);
	return rc;
}

int ecg_multi_recover_csum(ecg_multi_t *m, int k, int p, uint64_t C, const uint32_t *nstripes,
			   void *const *stripes, int64_t stride, const uint32_t *err_list, int nerrs, int type,
			   uint64_t chunksize, uint64_t rec_size, void *const *csums, unsigned flags)
{
	int rc = check_common(m, k, p);

	if (rc)
		return rc;
	if (nstripes == NULL || stripes == NULL || err_list == NULL || csums == NULL)
		return ecg_fail(-ECG_DER_INVAL, "multi_recover_csum: NULL array");
	if (nerrs > p)
		return ecg_fail(-ECG_DER_DATA_LOSS, "multi_recover_csum: %d erasures > p=%d", nerrs, p);
	pthread_mutex_lock(&m->call);
	m->job = (struct mjob){.op = MOP_RECOVER_CSUM, .k = k, .p = p, .C = C, .nstripes = nstripes,
			       .dst = stripes, .aux = csums, .s1 = stride, .err = err_list, .nerrs = nerrs,
			       .csum_type = type, .chunksize = chunksize, .rec_size = rec_size, .flags = flags};
	rc = run_all(m);
	pthread_mutex_unlock(&m->call);
	return rc;
}

int ecg_multi_update(ecg_multi_t *m, int k, int p, uint64_t C, const uint32_t *nstripes, int nupd,
		     const uint32_t *cell_idx, const void *const *old_cells, const void *const *new_cells,
		     int64_t upd_stripe_stride, void *const *parity, int64_t pcell, int64_t pstripe,
		     unsigned flags)
{
	int rc = check_common(m, k, p);

	if (rc)
		return rc;
	if (nstripes == NULL || cell_idx == NULL || old_cells == NULL || new_cells == NULL || parity == NULL ||
	    nupd < 1 || nupd > k)
		return ecg_fail(-ECG_DER_INVAL, "multi_update: bad argument");
	pthread_mutex_lock(&m->call);
	m->job = (struct mjob){.op = MOP_UPDATE, .k = k, .p = p, .C = C, .nstripes = nstripes,
			       .src = old_cells, .src2 = new_cells, .dst = parity, .err = cell_idx,
			       .nerrs = nupd, .s4 = upd_stripe_stride, .s2 = pcell,
			       .s3 = pstripe, .flags = flags};
	rc = run_all(m);
	pthread_mutex_unlock(&m->call);
	return rc;
}

/* Shard i's records of a fetched range: whole split units (stripes when
 * encoding, else cells -- the walk's own cut points, so every shard's pieces
 * are exactly the pieces the single walk cuts there) in contiguous runs;
 * shard 0 also takes the partial head, the last shard the partial tail. */
int ecg_multi_migrate_range(const ecg_multi_t *m, uint32_t oc_id, uint64_t e_len, uint64_t iod_size,
			    uint64_t offset, uint64_t size, int encode, int i, uint64_t *off, uint64_t *sz)
{
	uint64_t unit, b0, bl, end = offset + size, units, base, extra, f, c, lo, hi;
	int k, p, rc;

	if (m == NULL || i < 0 || i >= m->n || off == NULL || sz == NULL || e_len == 0 || iod_size == 0)
		return ecg_fail(-ECG_DER_INVAL, "multi_migrate_range: bad argument");
	rc = ecg_obj_ec_class_kp(oc_id, &k, &p);
	if (rc)
		return rc;
	unit = encode ? (uint64_t)k * e_len : e_len;
	b0 = (offset + unit - 1) / unit * unit;
	bl = end / unit * unit;
	if (b0 >= bl) {				/* no whole unit: shard 0 walks it all */
		*off = offset;
		*sz = i == 0 ? size : 0;
		return 0;
	}
	units = (bl - b0) / unit;
	base = units / (uint64_t)m->n;
	extra = units % (uint64_t)m->n;
	c = base + ((uint64_t)i < extra ? 1 : 0);
	f = base * (uint64_t)i + ((uint64_t)i < extra ? (uint64_t)i : extra);
	lo = i == 0 ? offset : b0 + f * unit;
	hi = i == m->n - 1 ? end : b0 + (f + c) * unit;
	*off = lo;
	*sz = hi - lo;
	return 0;
}

int ecg_multi_migrate_update_parity(ecg_multi_t *m, uint32_t oc_id, uint64_t e_len, uint64_t iod_size,
				    uint32_t shard, const void *const *buffers, uint64_t offset, uint64_t size,
				    int encode, int csum_type, uint64_t chunksize, void *const *parity_out,
				    void *const *csums_out, ecg_migrate_piece_t *pieces, uint32_t pieces_cap,
				    uint32_t *npieces, uint32_t *shard_first, unsigned flags)
{
	uint32_t first[ECG_MULTI_MAX + 1];
	int i, rc;

	if (m == NULL || buffers == NULL || parity_out == NULL || pieces == NULL || npieces == NULL ||
	    (csum_type && csums_out == NULL))
		return ecg_fail(-ECG_DER_INVAL, "multi_migrate: NULL argument");
	first[0] = 0;
	for (i = 0; i < m->n; i++) {		/* plan: where each shard's pieces go */
		uint64_t off, sz;
		uint32_t n = 0;

		rc = ecg_multi_migrate_range(m, oc_id, e_len, iod_size, offset, size, encode, i, &off, &sz);
		if (rc == 0 && sz)
			rc = ecg_migrate_plan_size(oc_id, e_len, iod_size, off, sz, encode, csum_type, chunksize, &n,
						   NULL, NULL);
		if (rc)
			return rc;
		first[i + 1] = first[i] + n;
	}
	if (first[m->n] > pieces_cap)
		return ecg_fail(-ECG_DER_REC2BIG, "multi_migrate: %u pieces > capacity %u", first[m->n], pieces_cap);
	pthread_mutex_lock(&m->call);
	m->job = (struct mjob){.op = MOP_MIGRATE, .oc_id = oc_id, .e_len = e_len, .rec_size = iod_size,
			       .shard = shard, .src = buffers, .offset = offset, .size = size, .encode = encode,
			       .csum_type = csum_type, .chunksize = chunksize, .dst = parity_out,
			       .aux = csums_out, .pieces = pieces, .first = first, .flags = flags};
	rc = run_all(m);
	pthread_mutex_unlock(&m->call);
	if (rc == 0) {
		*npieces = first[m->n];
		if (shard_first)
			memcpy(shard_first, first, sizeof(uint32_t) * (size_t)(m->n + 1));
	}
	return rc;
}
