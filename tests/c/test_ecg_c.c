/*
 * test_ecg_c.c -- native C driver for the libecg C-ABI, checked against the
 * CPU oracle (oracle/ec_ref.c, test infrastructure).
 *
 * Host-only checks always run.  With a gfx950 device present it also runs
 * the device paths, including ISA-L-convention calls from many pthreads at
 * once (the reference calls ec_encode_data concurrently from client threads
 * and engine xstreams) and the batching queue.
 * Built plain and with -fsanitize=address,undefined on the host code
 * (tests/c/Makefile).  Exit status 0 = pass.
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ec_ref.h"
#include "ecg.h"
#include "ecg_daos.h"
#include "ecg_isal.h"

static int g_fail;

#define CHECK(cond, ...)                                               \
	do {                                                           \
		if (!(cond)) {                                         \
			fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
			fprintf(stderr, __VA_ARGS__);                  \
			fprintf(stderr, "\n");                         \
			g_fail++;                                      \
		}                                                      \
	} while (0)

static uint64_t g_rng = 0xDA05EC00ull;

static unsigned char rnd(void)
{
	g_rng ^= g_rng << 13;
	g_rng ^= g_rng >> 7;
	g_rng ^= g_rng << 17;
	return (unsigned char)(g_rng >> 24);
}

static void fill(unsigned char *p, size_t n)
{
	for (size_t i = 0; i < n; i++)
		p[i] = rnd();
}

/* Host-side C-ABI from several threads at once, starting together so the
 * library's one-time initialisations (GF tables, codec table lookups) race:
 * the ThreadSanitizer build (tests/c/Makefile) checks this part without a
 * GPU.  Each thread compares against the oracle. */
struct host_job {
	int id, bad;
	pthread_barrier_t *go;
};

static void *host_thread(void *arg)
{
	struct host_job *j = arg;
	static const int kp[][2] = {{2, 1}, {4, 2}, {8, 2}, {8, 3}, {16, 2}};
	unsigned char a[(16 + 3) * 16], b[(16 + 3) * 16], inv[16 * 16], tmp[16 * 16];
	unsigned char tb[16 * 3 * 32], rtb[16 * 3 * 32];

	pthread_barrier_wait(j->go);
	for (int x = j->id; x < 256; x += 7)
		for (int y = 0; y < 256; y += 5)
			j->bad += gf_mul(x, y) != ref_gf_mul(x, y);
	for (size_t t = 0; t < sizeof(kp) / sizeof(kp[0]); t++) {
		const int k = kp[t][0], p = kp[t][1];

		gf_gen_cauchy1_matrix(a, k + p, k);
		ref_gf_gen_cauchy1_matrix(b, k + p, k);
		j->bad += memcmp(a, b, (size_t)(k + p) * k) != 0;
		ec_init_tables(k, p, &a[k * k], tb);
		ref_ec_init_tables(k, p, &b[k * k], rtb);
		j->bad += memcmp(tb, rtb, (size_t)k * p * 32) != 0;
		for (int e = 0; e < k + p; e++) {
			uint32_t err[1] = {(uint32_t)((e + j->id) % (k + p))};
			unsigned char rows[8 * 16];
			uint32_t dec[16];
			int reused = 0;

			j->bad += ecg_recov_matrix(k, p, a, err, 1, rows, dec, &reused) != 0;
		}
		memcpy(tmp, a + (size_t)p * k, (size_t)k * k);	/* rows p..p+k-1: invertible */
		j->bad += gf_invert_matrix(tmp, inv, k) != 0;
	}
	j->bad += ecg_obj_ec_codec_get((37u << 24) | 1) == NULL;
	return NULL;
}

static void host_threads(void)
{
	enum { NT = 8 };
	pthread_t th[NT];
	struct host_job jobs[NT];
	pthread_barrier_t go;

	pthread_barrier_init(&go, NULL, NT);
	for (int t = 0; t < NT; t++) {
		jobs[t] = (struct host_job){.id = t, .bad = 0, .go = &go};
		pthread_create(&th[t], NULL, host_thread, &jobs[t]);
	}
	for (int t = 0; t < NT; t++) {
		pthread_join(th[t], NULL);
		CHECK(jobs[t].bad == 0, "host thread %d: %d mismatches", t, jobs[t].bad);
	}
	pthread_barrier_destroy(&go);
}

static void host_checks(void)
{
	static const int kp[][2] = {{2, 1}, {2, 2}, {4, 1}, {4, 2}, {4, 3}, {8, 1}, {8, 2},
				    {8, 3}, {16, 1}, {16, 2}, {16, 3}};
	unsigned char a[(64 + 8) * 64], b[(64 + 8) * 64];
	size_t t;

	for (int x = 0; x < 256; x++)
		for (int y = 0; y < 256; y += 3)
			CHECK(gf_mul(x, y) == ref_gf_mul(x, y), "gf_mul %d %d", x, y);
	for (t = 0; t < sizeof(kp) / sizeof(kp[0]); t++) {
		int k = kp[t][0], p = kp[t][1];

		gf_gen_cauchy1_matrix(a, k + p, k);
		ref_gf_gen_cauchy1_matrix(b, k + p, k);
		CHECK(memcmp(a, b, (size_t)(k + p) * k) == 0, "cauchy %d+%d", k, p);
		/* every single and double erasure: data-first decode rows equal
		 * the reference's obj_ec_recov_codec_init rows */
		for (int e0 = 0; e0 < k + p; e0++) {
			for (int e1 = e0; e1 < k + p; e1++) {
				uint32_t err[2] = {(uint32_t)e0, (uint32_t)e1};
				int nerrs = e1 == e0 ? 1 : 2, reused = 0, rreused = 0;
				unsigned char rows[8 * 64], rrows[8 * 64], tb[64 * 8 * 32];
				uint32_t dec[64], rdec[64], rel[8];

				if (nerrs > p)
					continue;
				CHECK(ecg_recov_matrix(k, p, a, err, nerrs, rows, dec, &reused) == 0,
				      "recov %d+%d", k, p);
				CHECK(ref_obj_ec_recov_codec_init(k, p, b, err, nerrs, rrows, rdec, rel, tb,
								  &rreused) == 0, "ref recov");
				CHECK(reused == rreused, "reused %d+%d", k, p);
				if (!reused)
					CHECK(memcmp(rows, rrows, (size_t)nerrs * k) == 0 &&
					      memcmp(dec, rdec, sizeof(uint32_t) * k) == 0,
					      "rows %d+%d {%d,%d}", k, p, e0, e1);
			}
		}
	}
	{
		uint32_t err[3] = {0, 1, 2};
		unsigned char rows[8 * 64];
		uint32_t dec[64];
		int reused;

		CHECK(ecg_recov_matrix(4, 2, a, err, 3, rows, dec, &reused) == -ECG_DER_DATA_LOSS,
		      "data loss");
	}
	CHECK(ecg_obj_ec_codec_init() == 0, "codec_init");
	host_threads();
	CHECK(ecg_obj_ec_codec_get((37u << 24) | 1) != NULL, "codec_get 8P2");
	CHECK(ecg_obj_ec_codec_get((1u << 24) | 1) == NULL, "codec_get RP");
	ecg_obj_ec_codec_fini();
}

/* ---- the queue's CPU executor under many submitters ------------------------
 * ecg_queue_create(NULL): no device, the same lock-free reservations (CAS on
 * the slot's generation|open|count word), slot close / reopen and completion
 * threads as the device queue.  Small slots (max_batch 4) make every slot
 * close and reopen hundreds of times; threads mix encodes, in-place
 * recoveries and parity updates of their own stripes, wait for their own
 * callbacks, and some call ecg_queue_flush while others submit.  Run under
 * ThreadSanitizer in the host-only half (tests/c/Makefile test_ecg_c_tsan). */
struct qcpu_job {
	ecg_queue_t *q;
	int id, rounds, bad;
	pthread_mutex_t lock;
	pthread_cond_t cv;
	int pending, rcs;
};

static void qcpu_cb(void *arg, int rc)
{
	struct qcpu_job *j = arg;

	pthread_mutex_lock(&j->lock);
	j->pending--;
	j->rcs += rc != 0;
	pthread_cond_signal(&j->cv);
	pthread_mutex_unlock(&j->lock);
}

static void *qcpu_thread(void *arg)
{
	enum { K = 4, P = 2, NR = 6, CMAX = 1536 };
	struct qcpu_job *j = arg;
	unsigned char en[(K + P) * K], tb[K * P * 32], rtb[K * P * 32];
	static unsigned char bufs[48][NR][(K + P) * CMAX], want[48][NR][(K + P) * CMAX];
	unsigned char (*b)[(K + P) * CMAX] = bufs[j->id], (*w)[(K + P) * CMAX] = want[j->id];
	uint64_t st = 0x9E3779B97F4A7C15ull * (uint64_t)(j->id + 3);

	ref_gf_gen_cauchy1_matrix(en, K + P, K);
	ref_ec_init_tables(K, P, &en[K * K], tb);
	memcpy(rtb, tb, sizeof(tb));
	for (int it = 0; it < j->rounds; it++) {
		/* every other round one cell size for all threads: their requests
		 * share classes, so submitters race on one slot's reservation word;
		 * the other rounds spread over many classes (slot opens) */
		const int C = it % 2 ? 256 + (int)((uint64_t)(j->id * 131 + it * 17) % (CMAX - 256)) : 1024;
		unsigned char *data[K], *par[P], *wd[K], *wp[P];

		for (int n = 0; n < NR; n++)
			for (int i = 0; i < (K + P) * C; i++) {
				st ^= st << 13;
				st ^= st >> 7;
				st ^= st << 17;
				b[n][i] = (unsigned char)st;
			}
		/* expected results first (the oracle), then the requests */
		for (int n = 0; n < NR; n++) {
			memcpy(w[n], b[n], (size_t)(K + P) * C);
			for (int c = 0; c < K; c++)
				wd[c] = w[n] + c * C;
			for (int r = 0; r < P; r++)
				wp[r] = w[n] + (K + r) * C;
			if (n % 3 == 2) {		/* update: cell 1 changes to cell 3's bytes */
				unsigned char delta[CMAX];

				for (int i = 0; i < C; i++)
					delta[i] = w[n][1 * C + i] ^ w[n][3 * C + i];
				ref_ec_encode_data_update(C, K, P, 1, rtb, delta, wp);
			} else {			/* encode; recovery regenerates the same */
				ref_ec_encode_data(C, K, P, rtb, wd, wp);
			}
		}
		pthread_mutex_lock(&j->lock);
		j->pending = NR;
		pthread_mutex_unlock(&j->lock);
		for (int n = 0; n < NR; n++) {
			int rc;

			for (int c = 0; c < K; c++)
				data[c] = b[n] + c * C;
			for (int r = 0; r < P; r++)
				par[r] = b[n] + (K + r) * C;
			if (n % 3 == 0) {
				rc = ecg_queue_encode(j->q, K, P, (uint64_t)C, data, par, qcpu_cb, j);
			} else if (n % 3 == 1) {
				/* true parity in, then d2 and p1 erased and recovered */
				static const uint32_t err[2] = {2, 5};

				memcpy(b[n] + K * C, w[n] + K * C, (size_t)P * C);
				memset(b[n] + 2 * C, 0, (size_t)C);
				memset(b[n] + 5 * C, 0, (size_t)C);
				rc = ecg_queue_recover(j->q, K, P, (uint64_t)C, b[n], err, 2, qcpu_cb, j);
			} else {
				rc = ecg_queue_update(j->q, K, P, (uint64_t)C, 1, b[n] + 1 * C, b[n] + 3 * C, par,
						      qcpu_cb, j);
			}
			if (rc) {
				j->bad++;
				qcpu_cb(j, rc);
			}
		}
		if (j->id % 4 == 0 && it % 5 == 0)
			j->bad += ecg_queue_flush(j->q) != 0;
		pthread_mutex_lock(&j->lock);
		while (j->pending)
			pthread_cond_wait(&j->cv, &j->lock);
		pthread_mutex_unlock(&j->lock);
		for (int n = 0; n < NR; n++) {
			/* an update leaves the data cells as they were; w has cell 1
			 * unchanged too (only its delta went into the parity) */
			j->bad += memcmp(b[n], w[n], (size_t)(K + P) * C) != 0;
		}
	}
	return NULL;
}

static void queue_cpu_stress(void)
{
	static const int nthreads[] = {2, 12, 48};
	struct qcpu_job jobs[48];
	pthread_t th[48];

	for (size_t x = 0; x < sizeof(nthreads) / sizeof(nthreads[0]); x++) {
		const int T = nthreads[x];
		ecg_queue_attr_t attr = {.max_batch = 4, .max_wait_us = 20, .max_cell_bytes = 2048};
		ecg_queue_t *q = NULL;
		uint64_t nreq = 0, nb = 0;
		int bad = 0, rcs = 0;

		CHECK(ecg_queue_create(NULL, &attr, &q) == 0, "cpu queue_create: %s", ecg_strerror());
		if (q == NULL)
			return;
		for (int t = 0; t < T; t++) {
			jobs[t] = (struct qcpu_job){.q = q, .id = t, .rounds = T > 12 ? 12 : 30};
			pthread_mutex_init(&jobs[t].lock, NULL);
			pthread_cond_init(&jobs[t].cv, NULL);
			pthread_create(&th[t], NULL, qcpu_thread, &jobs[t]);
		}
		for (int t = 0; t < T; t++) {
			pthread_join(th[t], NULL);
			bad += jobs[t].bad;
			rcs += jobs[t].rcs;
			pthread_mutex_destroy(&jobs[t].lock);
			pthread_cond_destroy(&jobs[t].cv);
		}
		CHECK(ecg_queue_flush(q) == 0, "cpu queue flush");
		CHECK(ecg_queue_stats(q, &nreq, &nb) == 0, "cpu queue stats");
		ecg_queue_destroy(q);
		CHECK(bad == 0 && rcs == 0, "cpu queue, %d threads: %d mismatches, %d failed requests", T, bad, rcs);
		/* 4-request slots: many closes and reopens */
		CHECK(nb >= nreq / 4 && nb > 50, "cpu queue, %d threads: %llu requests in %llu batches", T,
		      (unsigned long long)nreq, (unsigned long long)nb);
		printf("cpu queue: %d threads, %llu requests, %llu batches\n", T, (unsigned long long)nreq,
		       (unsigned long long)nb);
	}
}

/* ---- device checks -------------------------------------------------------- */
struct tjob {
	int k, p, len, iters, id;
	int fails;
};

static void *isal_thread(void *arg)
{
	struct tjob *j = arg;
	unsigned char en[(16 + 4) * 16], tb[16 * 4 * 32], rtb[16 * 4 * 32];
	unsigned char *data[16], *par[4], *want[4];
	uint64_t st = 0x9E3779B97F4A7C15ull * (uint64_t)(j->id + 1);

	gf_gen_cauchy1_matrix(en, j->k + j->p, j->k);
	ec_init_tables(j->k, j->p, &en[j->k * j->k], tb);
	ref_ec_init_tables(j->k, j->p, &en[j->k * j->k], rtb);
	for (int c = 0; c < j->k; c++)
		data[c] = malloc(j->len);
	for (int r = 0; r < j->p; r++) {
		par[r] = malloc(j->len);
		want[r] = malloc(j->len);
	}
	for (int it = 0; it < j->iters; it++) {
		for (int c = 0; c < j->k; c++)
			for (int i = 0; i < j->len; i++) {
				st ^= st << 13;
				st ^= st >> 7;
				st ^= st << 17;
				data[c][i] = (unsigned char)st;
			}
		ec_encode_data(j->len, j->k, j->p, tb, data, par);
		ref_ec_encode_data(j->len, j->k, j->p, rtb, data, want);
		for (int r = 0; r < j->p; r++)
			j->fails += memcmp(par[r], want[r], j->len) != 0;
	}
	for (int c = 0; c < j->k; c++)
		free(data[c]);
	for (int r = 0; r < j->p; r++) {
		free(par[r]);
		free(want[r]);
	}
	return NULL;
}

/* ec_encode_data on DEVICE cells (an engine whose buffers live in HBM keeps
 * its ISA-L call sites): the drop-in launches on them in place */
struct djob {
	ecg_ctx_t *ctx;
	int k, p, len, iters, id;
	int fails;
};

static void *isal_device_thread(void *arg)
{
	struct djob *j = arg;
	unsigned char en[(16 + 4) * 16], tb[16 * 4 * 32], rtb[16 * 4 * 32];
	unsigned char *hdata[16], *want[4], *got, *data[16], *par[4];
	void *dbuf = NULL;
	const size_t slot = ((size_t)j->len + 64) & ~(size_t)15;
	uint64_t st = 0xC2B2AE3D27D4EB4Full * (uint64_t)(j->id + 1);

	gf_gen_cauchy1_matrix(en, j->k + j->p, j->k);
	ec_init_tables(j->k, j->p, &en[j->k * j->k], tb);
	ref_ec_init_tables(j->k, j->p, &en[j->k * j->k], rtb);
	if (ecg_dev_alloc(j->ctx, slot * (size_t)(j->k + j->p) + 64, &dbuf) != 0) {
		j->fails++;
		return NULL;
	}
	got = malloc(j->len);
	for (int c = 0; c < j->k; c++) {
		hdata[c] = malloc(j->len);
		data[c] = (unsigned char *)dbuf + c * slot + (c & 3);	/* odd offsets */
	}
	for (int r = 0; r < j->p; r++) {
		want[r] = malloc(j->len);
		par[r] = (unsigned char *)dbuf + (j->k + r) * slot + 1;
	}
	for (int it = 0; it < j->iters; it++) {
		for (int c = 0; c < j->k; c++) {
			for (int i = 0; i < j->len; i++) {
				st ^= st << 13;
				st ^= st >> 7;
				st ^= st << 17;
				hdata[c][i] = (unsigned char)st;
			}
			j->fails += ecg_memcpy(j->ctx, data[c], hdata[c], j->len, 0, NULL) != 0;
		}
		j->fails += ecg_stream_sync(j->ctx, NULL) != 0;
		ec_encode_data(j->len, j->k, j->p, tb, data, par);
		ref_ec_encode_data(j->len, j->k, j->p, rtb, hdata, want);
		for (int r = 0; r < j->p; r++) {
			j->fails += ecg_memcpy(j->ctx, got, par[r], j->len, 1, NULL) != 0 ||
				    ecg_stream_sync(j->ctx, NULL) != 0;
			j->fails += memcmp(got, want[r], j->len) != 0;
		}
	}
	for (int c = 0; c < j->k; c++)
		free(hdata[c]);
	for (int r = 0; r < j->p; r++)
		free(want[r]);
	free(got);
	ecg_dev_free(j->ctx, dbuf);
	return NULL;
}

struct qdone {
	pthread_mutex_t lock;
	int done, bad;
};

static void qcb(void *arg, int rc)
{
	struct qdone *d = arg;

	pthread_mutex_lock(&d->lock);
	d->done++;
	d->bad += rc != 0;
	pthread_mutex_unlock(&d->lock);
}

/* concurrent ISA-L-convention calls on host cells, mixed shapes and odd
 * lengths: the CPU path (ecg_cpu.c) with or without a device -- under
 * ThreadSanitizer in the host-only run -- and, with a device, once more with
 * the crossover at 0 so the same calls take the GPU staging path */
static void isal_threads(const char *what)
{
	enum { NT = 12 };
	pthread_t th[NT];
	struct tjob jobs[NT];
	int t;

	for (t = 0; t < NT; t++) {
		static const int shapes[][3] = {{4, 2, 4096}, {8, 2, 933}, {16, 3, 8569}, {2, 1, 37}};

		jobs[t] = (struct tjob){shapes[t % 4][0], shapes[t % 4][1], shapes[t % 4][2], 20, t, 0};
		pthread_create(&th[t], NULL, isal_thread, &jobs[t]);
	}
	for (t = 0; t < NT; t++) {
		pthread_join(th[t], NULL);
		CHECK(jobs[t].fails == 0, "%s thread %d: %d mismatches", what, t, jobs[t].fails);
	}
}

/* device-cell requests to one queue from several pthreads: thread t posts
 * stripes t, t + NQT, ... -- encodes of even stripes, {d1, p0} recoveries of
 * odd ones -- with device pointers (the queue batches them into pointer-
 * table launches in place) */
enum { NQT = 4 };
struct qdev_job {
	ecg_queue_t *q;
	unsigned char *d;		/* device image: stripe s at s * sst + off(s) */
	int k, p, S, t;
	uint64_t C;
	size_t sst;
	struct qdone *qd;
	int fails;
};

static size_t qdev_off(int s)
{
	return (size_t)(s * 5) % 16;
}

static void *qdev_thread(void *arg)
{
	struct qdev_job *j = arg;
	static const uint32_t err[2] = {1, 8};

	for (int s = j->t; s < j->S; s += NQT) {
		unsigned char *base = j->d + (size_t)s * j->sst + qdev_off(s), *data[16], *par[8];

		for (int c = 0; c < j->k; c++)
			data[c] = base + c * j->C;
		for (int r = 0; r < j->p; r++)
			par[r] = base + (j->k + r) * j->C;
		if ((s & 1) == 0)
			j->fails += ecg_queue_encode(j->q, j->k, j->p, j->C, data, par, qcb, j->qd) != 0;
		else
			j->fails += ecg_queue_recover(j->q, j->k, j->p, j->C, base, err, 2, qcb, j->qd) != 0;
	}
	return NULL;
}

static void device_checks(void)
{
	const uint64_t crossover = ecg_dropin_crossover();
	ecg_ctx_t *ctx = NULL;
	int t;

	CHECK(ecg_set_dropin_crossover(0) == 0, "crossover");
	isal_threads("gpu-staged");
	ecg_set_dropin_crossover(crossover);

	/* batched device encode + recovery through ecg.h */
	CHECK(ecg_ctx_create(0, &ctx) == 0, "ctx_create: %s", ecg_strerror());
	if (ctx == NULL)
		return;
	/* concurrent ISA-L-convention calls on device cells */
	{
		enum { ND = 8 };
		pthread_t dth[ND];
		struct djob djobs[ND];

		for (t = 0; t < ND; t++) {
			static const int shapes[][3] = {{4, 2, 4096}, {8, 2, 933}, {16, 3, 8569}, {2, 1, 37}};

			djobs[t] = (struct djob){ctx, shapes[t % 4][0], shapes[t % 4][1], shapes[t % 4][2], 10, t, 0};
			pthread_create(&dth[t], NULL, isal_device_thread, &djobs[t]);
		}
		for (t = 0; t < ND; t++) {
			pthread_join(dth[t], NULL);
			CHECK(djobs[t].fails == 0, "device-cell thread %d: %d failures", t, djobs[t].fails);
		}
	}
	{
		const int k = 8, p = 2, S = 6;
		const uint64_t C = 65536 + 16;
		const size_t sst = (size_t)(k + p) * C;
		unsigned char *h = malloc(S * sst), *g = malloc(S * sst);
		unsigned char en[10 * 8], tb[8 * 2 * 32], *src[8], *dst[2];
		void *d = NULL;
		uint32_t err[2] = {1, 8};

		fill(h, S * sst);
		CHECK(ecg_dev_alloc(ctx, S * sst, &d) == 0, "dev_alloc");
		CHECK(ecg_memcpy(ctx, d, h, S * sst, 0, NULL) == 0, "h2d");
		CHECK(ecg_encode(ctx, k, p, C, S, d, (int64_t)sst, (char *)d + k * C, (int64_t)C,
				 (int64_t)sst, NULL) == 0, "encode: %s", ecg_strerror());
		CHECK(ecg_memcpy(ctx, g, d, S * sst, 1, NULL) == 0 && ecg_stream_sync(ctx, NULL) == 0,
		      "d2h");
		ref_gf_gen_cauchy1_matrix(en, k + p, k);
		ref_ec_init_tables(k, p, &en[k * k], tb);
		for (int s = 0; s < S; s++) {
			unsigned char want0[65536 + 16], want1[65536 + 16];

			for (int c = 0; c < k; c++)
				src[c] = g + s * sst + c * C;
			dst[0] = want0;
			dst[1] = want1;
			ref_ec_encode_data((int)C, k, p, tb, src, dst);
			CHECK(memcmp(want0, g + s * sst + k * C, C) == 0 &&
			      memcmp(want1, g + s * sst + (k + 1) * C, C) == 0, "parity stripe %d", s);
		}
		/* wipe d1 and p0, recover on device */
		memcpy(h, g, S * sst);
		for (int s = 0; s < S; s++) {
			memset(h + s * sst + 1 * C, 0, C);
			memset(h + s * sst + 8 * C, 0, C);
		}
		CHECK(ecg_memcpy(ctx, d, h, S * sst, 0, NULL) == 0, "h2d 2");
		CHECK(ecg_recover(ctx, k, p, C, S, d, (int64_t)sst, err, 2, NULL) == 0, "recover");
		CHECK(ecg_memcpy(ctx, h, d, S * sst, 1, NULL) == 0 && ecg_stream_sync(ctx, NULL) == 0,
		      "d2h 2");
		CHECK(memcmp(h, g, S * sst) == 0, "recovered stripes");
		ecg_dev_free(ctx, d);
		free(h);
		free(g);
	}
	/* batching queue from several threads' worth of submissions, host cells
	 * on both routes: computed on the completion threads (below the
	 * drop-in crossover) and staged through the device (crossover 0) */
	for (int route = 0; route < 2; route++) {
		ecg_queue_t *q = NULL;
		struct qdone qd = {PTHREAD_MUTEX_INITIALIZER, 0, 0};
		enum { N = 64 };
		const int k = 4, p = 2, C = 4096 + 8;
		unsigned char *cells = malloc((size_t)N * (k + p) * C);
		unsigned char en[6 * 4], tb[4 * 2 * 32];
		const uint64_t cross = ecg_dropin_crossover();

		ecg_set_dropin_crossover(route == 0 ? UINT64_MAX : 0);
		fill(cells, (size_t)N * (k + p) * C);
		CHECK(ecg_queue_create(ctx, NULL, &q) == 0, "queue_create");
		for (int i = 0; i < N; i++) {
			unsigned char *data[4], *par[2];

			for (int c = 0; c < k; c++)
				data[c] = cells + ((size_t)i * (k + p) + c) * C;
			for (int r = 0; r < p; r++)
				par[r] = cells + ((size_t)i * (k + p) + k + r) * C;
			CHECK(ecg_queue_encode(q, k, p, C, data, par, qcb, &qd) == 0, "queue_encode");
		}
		CHECK(ecg_queue_flush(q) == 0 && qd.done == N && qd.bad == 0, "queue done %d bad %d",
		      qd.done, qd.bad);
		ref_gf_gen_cauchy1_matrix(en, k + p, k);
		ref_ec_init_tables(k, p, &en[k * k], tb);
		for (int i = 0; i < N; i++) {
			unsigned char *src[4], *dst[2], w0[4096 + 8], w1[4096 + 8];

			for (int c = 0; c < k; c++)
				src[c] = cells + ((size_t)i * (k + p) + c) * C;
			dst[0] = w0;
			dst[1] = w1;
			ref_ec_encode_data(C, k, p, tb, src, dst);
			CHECK(memcmp(w0, cells + ((size_t)i * (k + p) + k) * C, C) == 0 &&
			      memcmp(w1, cells + ((size_t)i * (k + p) + k + 1) * C, C) == 0, "queue stripe %d (%s)",
			      i, route == 0 ? "cpu" : "staged");
		}
		ecg_queue_destroy(q);
		ecg_set_dropin_crossover(cross);
		free(cells);
	}
	/* the same queue API on device cells, from NQT pthreads */
	{
		ecg_queue_t *q = NULL;
		struct qdone qd = {PTHREAD_MUTEX_INITIALIZER, 0, 0};
		const int k = 8, p = 2, S = 48;
		const uint64_t C = 8192 + 4;
		const size_t sst = (size_t)(k + p) * C + 16;
		unsigned char *h = malloc(S * sst), *g = malloc(S * sst), en[10 * 8], tb[8 * 2 * 32];
		pthread_t qth[NQT];
		struct qdev_job jobs[NQT];
		void *d = NULL;

		fill(h, S * sst);
		ref_gf_gen_cauchy1_matrix(en, k + p, k);
		ref_ec_init_tables(k, p, &en[k * k], tb);
		for (int s = 0; s < S; s++) {		/* odd stripes: true parity, then d1 / p0 erased */
			unsigned char *b = h + (size_t)s * sst + qdev_off(s), *src[8], *dst[2];

			if ((s & 1) == 0)
				continue;
			for (int c = 0; c < k; c++)
				src[c] = b + c * C;
			dst[0] = b + k * C;
			dst[1] = b + (k + 1) * C;
			ref_ec_encode_data((int)C, k, p, tb, src, dst);
		}
		memcpy(g, h, S * sst);			/* g: the expected image */
		for (int s = 0; s < S; s++) {
			unsigned char *b = h + (size_t)s * sst + qdev_off(s), *src[8], *dst[2];

			if (s & 1) {
				memset(b + 1 * C, 0, C);
				memset(b + 8 * C, 0, C);
				continue;
			}
			b = g + (size_t)s * sst + qdev_off(s);
			for (int c = 0; c < k; c++)
				src[c] = b + c * C;
			dst[0] = b + k * C;
			dst[1] = b + (k + 1) * C;
			ref_ec_encode_data((int)C, k, p, tb, src, dst);
		}
		CHECK(ecg_dev_alloc(ctx, S * sst, &d) == 0 && ecg_memcpy(ctx, d, h, S * sst, 0, NULL) == 0 &&
		      ecg_stream_sync(ctx, NULL) == 0, "device image");
		CHECK(ecg_queue_create(ctx, NULL, &q) == 0, "queue_create (device cells)");
		for (int t = 0; t < NQT && q && d; t++) {
			jobs[t] = (struct qdev_job){q, d, k, p, S, t, C, sst, &qd, 0};
			pthread_create(&qth[t], NULL, qdev_thread, &jobs[t]);
		}
		for (int t = 0; t < NQT && q && d; t++) {
			pthread_join(qth[t], NULL);
			CHECK(jobs[t].fails == 0, "device-cell queue thread %d: %d refused", t, jobs[t].fails);
		}
		if (q) {
			CHECK(ecg_queue_flush(q) == 0 && qd.done == S && qd.bad == 0, "device-cell queue done %d bad %d",
			      qd.done, qd.bad);
			ecg_queue_destroy(q);
		}
		CHECK(ecg_memcpy(ctx, h, d, S * sst, 1, NULL) == 0 && ecg_stream_sync(ctx, NULL) == 0, "d2h 3");
		for (int s = 0; s < S; s++)
			CHECK(memcmp(h + (size_t)s * sst + qdev_off(s), g + (size_t)s * sst + qdev_off(s),
				     (size_t)(k + p) * C) == 0, "device-cell queue stripe %d", s);
		ecg_dev_free(ctx, d);
		free(h);
		free(g);
	}
	ecg_ctx_destroy(ctx);
}

int main(void)
{
	host_checks();
	isal_threads("cpu-path");
	queue_cpu_stress();
	if (ecg_device_count() > 0)
		device_checks();
	else
		printf("no gfx950 device: host-only checks\n");
	printf("%s (%d failures)\n", g_fail ? "FAIL" : "PASS", g_fail);
	return g_fail ? 1 : 0;
}
