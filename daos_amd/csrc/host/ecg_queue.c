/*
 * ecg_queue.c -- batching facade: one-stripe requests from many threads ->
 * batched device launches (see include/ecg.h, "batching facade").
 *
 * Why: every DAOS caller hands the codec one stripe at a time (SURVEY §0.6;
 * ref:src/object/cli_ec.c:627-659, ref:src/object/srv_obj_migrate.c:1116-1177,
 * ref:src/object/srv_ec_aggregate.c:701-734), and a single-stripe GPU call is
 * launch- and PCIe-latency bound.  The queue turns N concurrent
 * one-stripe calls into one device product over N stripes.
 *
 * Structure: a FIFO guarded by a mutex, one worker thread.  The worker takes
 * the oldest request's "class" (op, k, p, cell size, erasure set), waits up to
 * max_wait_us for more of the same class unless max_batch are already queued,
 * gathers the batch into pinned staging with a 64-byte-aligned cell pitch (so
 * the vector kernels apply for any cell size), runs one ecg_matmul on the
 * device, scatters the results back and fires each request's callback.
 */
#include <errno.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "ecg_internal.h"

#define OP_ENCODE 0
#define OP_RECOVER 1

struct qreq {
	struct qreq *next;
	int op, k, p, nerrs;
	uint64_t C;
	unsigned char *src[ECG_MAX_K];
	unsigned char *dst[ECG_MAX_P];
	unsigned char *stripe;
	uint32_t err[ECG_MAX_P];
	ecg_done_cb_t cb;
	void *arg;
	uint64_t t_ns;
};

struct ecg_queue {
	ecg_ctx_t *ctx;
	ecg_queue_attr_t attr;
	uint64_t staging_bytes;
	pthread_mutex_t lock;
	pthread_cond_t cv_work;
	pthread_cond_t cv_done;
	struct qreq *head, *tail;
	uint64_t submitted, completed, batches;
	uint64_t flush_target;	/* a flush waits for this many completions */
	int stop;
	pthread_t worker;
	unsigned char *host;
	size_t host_bytes;
	unsigned char *dev;
	size_t dev_bytes;
	hipStream_t st;
};

static uint64_t now_ns(void)
{
	struct timespec ts;

	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

static int same_class(const struct qreq *a, const struct qreq *b)
{
	return a->op == b->op && a->k == b->k && a->p == b->p && a->C == b->C &&
	       a->nerrs == b->nerrs &&
	       (a->op != OP_RECOVER || memcmp(a->err, b->err, sizeof(uint32_t) * a->nerrs) == 0);
}

static uint64_t pitch_of(uint64_t C)
{
	return (C + 63) & ~63ull;
}

/* Stripes of this class that fit one batch. */
static uint32_t batch_limit(const struct ecg_queue *q, const struct qreq *r)
{
	uint64_t per = pitch_of(r->C) * (uint64_t)(r->k + r->p);
	uint64_t n = per ? q->staging_bytes / per : q->attr.max_batch;

	if (n < 1)
		n = 1;
	if (n > q->attr.max_batch)
		n = q->attr.max_batch;
	return (uint32_t)n;
}

static int staging_reserve(struct ecg_queue *q, size_t bytes)
{
	hipError_t e;

	if (q->host_bytes < bytes) {
		if (q->host)
			(void)hipHostFree(q->host);
		q->host = NULL;
		q->host_bytes = 0;
		e = hipHostMalloc((void **)&q->host, bytes, hipHostMallocDefault);
		if (e != hipSuccess)
			return ecg_hip_fail(e, "queue pinned staging");
		q->host_bytes = bytes;
	}
	if (q->dev_bytes < bytes) {
		if (q->dev)
			(void)hipFree(q->dev);
		q->dev = NULL;
		q->dev_bytes = 0;
		e = hipMalloc((void **)&q->dev, bytes);
		if (e != hipSuccess)
			return ecg_hip_fail(e, "queue device staging");
		q->dev_bytes = bytes;
	}
	return 0;
}

/* Run one batch of same-class requests.  Staging layout: stripe i at
 * i*(k+p)*pitch, cell c at c*pitch inside it (logical order, as the
 * reference's recovery buffer). */
static int run_batch(struct ecg_queue *q, struct qreq **b, uint32_t n)
{
	const struct qreq *r0 = b[0];
	const int k = r0->k, p = r0->p;
	const uint64_t C = r0->C, pitch = pitch_of(C);
	const uint64_t sstride = pitch * (uint64_t)(k + p);
	unsigned char coef[ECG_MAX_P * ECG_MAX_K];
	uint32_t out_idx[ECG_MAX_P], dec_idx[ECG_MAX_K];
	int64_t soff[ECG_MAX_K], doff[ECG_MAX_P];
	int rows, rc, reused, j;
	uint32_t i;
	hipError_t e;

	rc = ecg_ctx_enter(q->ctx);
	if (rc)
		return rc;
	rc = staging_reserve(q, (size_t)(sstride * n));
	if (rc)
		return rc;
	if (r0->op == OP_ENCODE) {
		unsigned char en[(ECG_MAX_K + ECG_MAX_P) * ECG_MAX_K];

		ecg_gen_cauchy1(k, p, en);
		memcpy(coef, &en[k * k], (size_t)p * k);
		rows = p;
		for (j = 0; j < k; j++)
			dec_idx[j] = (uint32_t)j;
		for (j = 0; j < p; j++)
			out_idx[j] = (uint32_t)(k + j);
	} else {
		unsigned char en[(ECG_MAX_K + ECG_MAX_P) * ECG_MAX_K];

		ecg_gen_cauchy1(k, p, en);
		rc = ecg_recov_rows(k, p, en, r0->err, r0->nerrs, coef, out_idx, dec_idx, &reused);
		if (rc)
			return rc;
		rows = r0->nerrs;
	}
	/* gather the cells the product reads */
	for (i = 0; i < n; i++) {
		unsigned char *s = q->host + i * sstride;

		for (j = 0; j < k; j++) {
			const unsigned char *from = b[i]->op == OP_ENCODE ? b[i]->src[j]
					: b[i]->stripe + (uint64_t)dec_idx[j] * C;

			memcpy(s + (uint64_t)dec_idx[j] * pitch, from, C);
		}
	}
	e = hipMemcpyAsync(q->dev, q->host, (size_t)(sstride * n), hipMemcpyHostToDevice, q->st);
	if (e != hipSuccess)
		return ecg_hip_fail(e, "queue H2D");
	for (j = 0; j < k; j++)
		soff[j] = (int64_t)(dec_idx[j] * pitch);
	for (j = 0; j < rows; j++)
		doff[j] = (int64_t)(out_idx[j] * pitch);
	rc = ecg_matmul(q->ctx, k, rows, coef, C, n, q->dev, soff, (int64_t)sstride, q->dev, doff,
			(int64_t)sstride, 0, q->st);
	if (rc)
		return rc;
	e = hipMemcpyAsync(q->host, q->dev, (size_t)(sstride * n), hipMemcpyDeviceToHost, q->st);
	if (e == hipSuccess)
		e = hipStreamSynchronize(q->st);
	if (e != hipSuccess)
		return ecg_hip_fail(e, "queue D2H");
	/* scatter the cells the product wrote */
	for (i = 0; i < n; i++) {
		const unsigned char *s = q->host + i * sstride;

		for (j = 0; j < rows; j++) {
			unsigned char *to = b[i]->op == OP_ENCODE ? b[i]->dst[j]
					: b[i]->stripe + (uint64_t)out_idx[j] * C;

			memcpy(to, s + (uint64_t)out_idx[j] * pitch, C);
		}
	}
	return 0;
}

static void *worker_main(void *argp)
{
	struct ecg_queue *q = argp;
	struct qreq **batch = calloc(q->attr.max_batch, sizeof(*batch));

	if (batch == NULL)
		abort();
	(void)hipSetDevice(q->ctx->device);
	pthread_mutex_lock(&q->lock);
	for (;;) {
		struct qreq *r, *prev, *next;
		uint32_t n = 0, limit, avail = 0;
		int rc;

		if (q->head == NULL) {
			if (q->stop)
				break;
			pthread_cond_wait(&q->cv_work, &q->lock);
			continue;
		}
		limit = batch_limit(q, q->head);
		for (r = q->head; r && avail < limit; r = r->next)
			avail += same_class(r, q->head);
		if (avail < limit && !q->stop && q->completed >= q->flush_target) {
			uint64_t deadline = q->head->t_ns + (uint64_t)q->attr.max_wait_us * 1000ull;
			uint64_t t = now_ns();

			if (t < deadline) {
				struct timespec ts;

				clock_gettime(CLOCK_REALTIME, &ts);
				t = deadline - t;
				ts.tv_sec += (time_t)(t / 1000000000ull);
				ts.tv_nsec += (long)(t % 1000000000ull);
				if (ts.tv_nsec >= 1000000000L) {
					ts.tv_sec++;
					ts.tv_nsec -= 1000000000L;
				}
				pthread_cond_timedwait(&q->cv_work, &q->lock, &ts);
				continue;
			}
		}
		/* unlink up to `limit` requests of the head's class, FIFO order */
		{
			struct qreq *key = q->head;

			prev = NULL;
			for (r = q->head; r && n < limit; r = next) {
				next = r->next;
				if (same_class(r, key)) {
					if (prev)
						prev->next = next;
					else
						q->head = next;
					if (q->tail == r)
						q->tail = prev;
					r->next = NULL;
					batch[n++] = r;
				} else {
					prev = r;
				}
			}
		}
		pthread_mutex_unlock(&q->lock);
		rc = run_batch(q, batch, n);
		for (uint32_t i = 0; i < n; i++) {
			if (batch[i]->cb)
				batch[i]->cb(batch[i]->arg, rc);
			free(batch[i]);
		}
		pthread_mutex_lock(&q->lock);
		q->completed += n;
		q->batches++;
		pthread_cond_broadcast(&q->cv_done);
	}
	pthread_mutex_unlock(&q->lock);
	free(batch);
	return NULL;
}

int ecg_queue_create(ecg_ctx_t *ctx, const ecg_queue_attr_t *attr, ecg_queue_t **out)
{
	struct ecg_queue *q;
	pthread_condattr_t ca;
	hipError_t e;
	int rc;

	if (ctx == NULL || out == NULL)
		return ecg_fail(-ECG_DER_INVAL, "queue_create: NULL argument");
	rc = ecg_ctx_enter(ctx);
	if (rc)
		return rc;
	q = calloc(1, sizeof(*q));
	if (q == NULL)
		return ecg_fail(-ECG_DER_NOMEM, "queue_create: calloc");
	q->ctx = ctx;
	if (attr)
		q->attr = *attr;
	if (q->attr.max_batch == 0)
		q->attr.max_batch = 256;
	if (q->attr.max_wait_us == 0)
		q->attr.max_wait_us = 50;
	if (q->attr.max_cell_bytes == 0)
		q->attr.max_cell_bytes = 1 << 20;
	/* staging for a full batch of 8+2 stripes at max_cell_bytes, capped at
	 * 512 MiB (larger classes just get proportionally fewer stripes) */
	q->staging_bytes = pitch_of(q->attr.max_cell_bytes) * 10ull * q->attr.max_batch;
	if (q->staging_bytes > (512ull << 20))
		q->staging_bytes = 512ull << 20;
	pthread_mutex_init(&q->lock, NULL);
	pthread_condattr_init(&ca);
	pthread_cond_init(&q->cv_work, &ca);
	pthread_cond_init(&q->cv_done, &ca);
	pthread_condattr_destroy(&ca);
	e = hipStreamCreateWithFlags(&q->st, hipStreamNonBlocking);
	if (e != hipSuccess) {
		free(q);
		return ecg_hip_fail(e, "queue stream");
	}
	if (pthread_create(&q->worker, NULL, worker_main, q) != 0) {
		(void)hipStreamDestroy(q->st);
		free(q);
		return ecg_fail(-ECG_DER_NOMEM, "queue_create: pthread_create");
	}
	*out = q;
	return 0;
}

void ecg_queue_destroy(ecg_queue_t *q)
{
	if (q == NULL)
		return;
	pthread_mutex_lock(&q->lock);
	q->stop = 1;
	pthread_cond_broadcast(&q->cv_work);
	pthread_mutex_unlock(&q->lock);
	pthread_join(q->worker, NULL);
	(void)hipSetDevice(q->ctx->device);
	if (q->host)
		(void)hipHostFree(q->host);
	if (q->dev)
		(void)hipFree(q->dev);
	(void)hipStreamDestroy(q->st);
	pthread_cond_destroy(&q->cv_work);
	pthread_cond_destroy(&q->cv_done);
	pthread_mutex_destroy(&q->lock);
	free(q);
}

static int enqueue(struct ecg_queue *q, struct qreq *r)
{
	r->t_ns = now_ns();
	pthread_mutex_lock(&q->lock);
	if (q->stop) {
		pthread_mutex_unlock(&q->lock);
		free(r);
		return ecg_fail(-ECG_DER_INVAL, "queue is being destroyed");
	}
	if (q->tail)
		q->tail->next = r;
	else
		q->head = r;
	q->tail = r;
	q->submitted++;
	pthread_cond_signal(&q->cv_work);
	pthread_mutex_unlock(&q->lock);
	return 0;
}

int ecg_queue_encode(ecg_queue_t *q, int k, int p, uint64_t C, unsigned char *const *data,
		     unsigned char *const *parity, ecg_done_cb_t cb, void *arg)
{
	struct qreq *r;
	int j;

	if (q == NULL || data == NULL || parity == NULL || k < 1 || k > ECG_MAX_K || p < 1 ||
	    p > ECG_MAX_P || C == 0)
		return ecg_fail(-ECG_DER_INVAL, "queue_encode: bad arguments");
	r = calloc(1, sizeof(*r));
	if (r == NULL)
		return ecg_fail(-ECG_DER_NOMEM, "queue_encode: calloc");
	r->op = OP_ENCODE;
	r->k = k;
	r->p = p;
	r->C = C;
	for (j = 0; j < k; j++)
		r->src[j] = data[j];
	for (j = 0; j < p; j++)
		r->dst[j] = parity[j];
	r->cb = cb;
	r->arg = arg;
	return enqueue(q, r);
}

int ecg_queue_recover(ecg_queue_t *q, int k, int p, uint64_t C, unsigned char *stripe,
		      const uint32_t *err_list, int nerrs, ecg_done_cb_t cb, void *arg)
{
	struct qreq *r;
	int i;

	if (q == NULL || stripe == NULL || err_list == NULL || k < 1 || k > ECG_MAX_K || p < 1 ||
	    p > ECG_MAX_P || C == 0 || nerrs < 1)
		return ecg_fail(-ECG_DER_INVAL, "queue_recover: bad arguments");
	if (nerrs > p)
		return ecg_fail(-ECG_DER_DATA_LOSS, "queue_recover: %d erasures > p=%d", nerrs, p);
	for (i = 0; i < nerrs; i++)
		if (err_list[i] >= (uint32_t)(k + p))
			return ecg_fail(-ECG_DER_INVAL, "queue_recover: cell %u", err_list[i]);
	r = calloc(1, sizeof(*r));
	if (r == NULL)
		return ecg_fail(-ECG_DER_NOMEM, "queue_recover: calloc");
	r->op = OP_RECOVER;
	r->k = k;
	r->p = p;
	r->C = C;
	r->stripe = stripe;
	r->nerrs = nerrs;
	memcpy(r->err, err_list, sizeof(uint32_t) * nerrs);
	r->cb = cb;
	r->arg = arg;
	return enqueue(q, r);
}

int ecg_queue_flush(ecg_queue_t *q)
{
	uint64_t target;

	if (q == NULL)
		return ecg_fail(-ECG_DER_INVAL, "queue_flush: NULL queue");
	pthread_mutex_lock(&q->lock);
	target = q->submitted;
	if (q->flush_target < target)
		q->flush_target = target;
	pthread_cond_broadcast(&q->cv_work);
	while (q->completed < target)
		pthread_cond_wait(&q->cv_done, &q->lock);
	pthread_mutex_unlock(&q->lock);
	return 0;
}

int ecg_queue_stats(ecg_queue_t *q, uint64_t *requests, uint64_t *batches)
{
	if (q == NULL)
		return ecg_fail(-ECG_DER_INVAL, "queue_stats: NULL queue");
	pthread_mutex_lock(&q->lock);
	if (requests)
		*requests = q->completed;
	if (batches)
		*batches = q->batches;
	pthread_mutex_unlock(&q->lock);
	return 0;
}
