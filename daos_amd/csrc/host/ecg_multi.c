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
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../../include/ecg_multi.h"
#include "ecg_internal.h"

struct mjob {
	int op;
	int k, p, nerrs;
	uint64_t C;
	uint32_t S;			/* host ops: the whole batch */
	const uint32_t *nstripes;	/* device ops: per shard */
	const void *const *src;
	void *const *dst;
	const void *hsrc;
	void *hdst;
	int64_t s1, s2, s3;
	const uint32_t *err;
	uint32_t chunk;
	unsigned flags;
};

enum { MOP_ENCODE, MOP_RECOVER, MOP_SYNC, MOP_ENCODE_HOST, MOP_RECOVER_HOST };

struct mworker {
	struct ecg_multi *m;
	int idx;
	ecg_ctx_t *ctx;
	pthread_t th;
	int started;
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
