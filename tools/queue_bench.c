/*
 * queue_bench.c -- one-stripe callers, the reference's calling pattern
 * (SURVEY §0.6): T pthreads each encode N stripes of EC_k+p with C-byte
 * cells, one stripe per call, via
 *   isal : ec_encode_data()        (synchronous ISA-L drop-in: host cells run the
 *                                   product CPU path at the default crossover,
 *                                   the GPU with ECG_DROPIN_CROSSOVER=0)
 *   queue: ecg_queue_encode()      (batching facade, async completion)
 *   cpu  : ref_simd_encode_data()  (ISA-L-equivalent CPU restatement, the
 *                                   baseline DAOS runs today)
 * and prints one JSON line of GiB/s (user data).  With a third argument
 * "update" the calls are aggregation delta updates of one data cell per call
 * (agg_update_parity, ref:src/object/srv_ec_aggregate.c:1086-1102):
 *   isal : xor_gen(old, new -> diff) + ec_encode_data_update(vec_i)  (drop-in)
 *   queue: ecg_queue_update()
 *   cpu  : diff loop + ref_simd_encode_data(k = 1, the vec_i column) XORed
 *          into the parity (ISA-L-equivalent CPU restatement)
 * and GiB/s counts the updated cell bytes.  With "device" the cells live in
 * device memory: the drop-in (ec_encode_data on device cells, in place, the
 * calling threads spread over the context's drop-in stream pool, each call
 * waiting for its own launch) and the queue (device-cell requests batched
 * into pointer-table launches in place; QB_VERIFY=1: one queue run over a
 * patterned image, every stripe's parity checked against the CPU
 * restatement -- in host mode likewise, parity zeroed first).
 * With "devupdate" the update calls run on DEVICE cells: the drop-in
 * (xor_gen + ec_encode_data_update on device cells, one synchronous launch
 * pair per call) against the queue (ecg_queue_update on device cells, batched
 * into ecg_update_ptrs launches in place); QB_VERIFY=1 checks every stripe's
 * parity after one queue run against the CPU restatement.  QB_CPU_QUEUE=1
 * creates the queue with no context (the CPU executor; host cells).
 * QB_LATENCY=1: one request at a time, each waited for (queue latency), and
 * the same call through the synchronous drop-in.
 * usage: queue_bench C T [update|device|devupdate] [stripes per thread, default 64].
 * Bench infrastructure.
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "ec_ref.h"
#include "ecg.h"
#include "ecg_isal.h"

static int K = 8, P = 2, T = 8, N = 64;
static uint64_t CB = 128 << 10;
static unsigned char *g_cells;		/* T * N stripes of (K + P) cells */
static unsigned char *g_dcells;		/* the same in device memory ("device") */
static unsigned char g_tbls[64 * 8 * 32];
static ecg_queue_t *g_q;
static int g_mode;			/* 0 isal, 1 queue, 2 cpu */
static int g_update;			/* calls are one-cell delta updates */
static unsigned char *g_new;		/* T * N new cells (update) */
static unsigned char *g_dnew;		/* the same in device memory ("devupdate") */
static unsigned char *g_ddiff;		/* T device diff cells (drop-in devupdate) */
static unsigned char g_col[64][8 * 32];	/* vec_i -> the P tables of column vec_i */

struct cnt {
	pthread_mutex_t lock;
	pthread_cond_t cv;
	long done;
};
static struct cnt g_cnt = {PTHREAD_MUTEX_INITIALIZER, PTHREAD_COND_INITIALIZER, 0};

static double now(void)
{
	struct timespec ts;

	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void done_cb(void *arg, int rc)
{
	(void)arg;
	if (rc)
		fprintf(stderr, "request failed rc=%d\n", rc);
	pthread_mutex_lock(&g_cnt.lock);
	g_cnt.done++;
	pthread_cond_broadcast(&g_cnt.cv);
	pthread_mutex_unlock(&g_cnt.lock);
}

static void update_one(long t, int i)
{
	unsigned char *s = (g_dcells ? g_dcells : g_cells) + ((size_t)t * N + i) * (K + P) * CB;
	unsigned char *nw = (g_dnew ? g_dnew : g_new) + ((size_t)t * N + i) * CB;
	const int vec_i = (int)((t * N + i) % K);
	unsigned char *old = s + vec_i * CB, *par[8];

	for (int r = 0; r < P; r++)
		par[r] = s + (K + r) * CB;
	if (g_mode == 1) {
		ecg_queue_update(g_q, K, P, CB, vec_i, old, nw, par, done_cb, NULL);
		return;
	}
	unsigned char *diff = g_ddiff ? g_ddiff + (size_t)t * CB : malloc(CB), *tmp[8];

	if (g_mode == 0) {
		void *arr[3] = {old, nw, diff};

		xor_gen(3, (int)CB, arr);
		ec_encode_data_update((int)CB, K, P, vec_i, g_tbls, diff, par);
	} else {
		for (uint64_t b = 0; b < CB; b += 8) {
			uint64_t x, y;

			memcpy(&x, old + b, 8);
			memcpy(&y, nw + b, 8);
			x ^= y;
			memcpy(diff + b, &x, 8);
		}
		for (int r = 0; r < P; r++)
			tmp[r] = malloc(CB);
		ref_simd_encode_data((int)CB, 1, P, g_col[vec_i], &diff, tmp);
		for (int r = 0; r < P; r++) {
			for (uint64_t b = 0; b < CB; b += 8) {
				uint64_t x, y;

				memcpy(&x, par[r] + b, 8);
				memcpy(&y, tmp[r] + b, 8);
				x ^= y;
				memcpy(par[r] + b, &x, 8);
			}
			free(tmp[r]);
		}
	}
	if (!g_ddiff)
		free(diff);
}

/* thread t's i-th call in the current mode */
static void request(long t, int i)
{
	if (g_update) {
		update_one(t, i);
		return;
	}
	unsigned char *s = (g_dcells ? g_dcells : g_cells) + ((size_t)t * N + i) * (K + P) * CB;
	unsigned char *data[64], *par[8];

	for (int c = 0; c < K; c++)
		data[c] = s + c * CB;
	for (int r = 0; r < P; r++)
		par[r] = s + (K + r) * CB;
	if (g_mode == 0)
		ec_encode_data((int)CB, K, P, g_tbls, data, par);
	else if (g_mode == 1)
		ecg_queue_encode(g_q, K, P, CB, data, par, done_cb, NULL);
	else
		ref_simd_encode_data((int)CB, K, P, g_tbls, data, par);
}

static void *worker(void *arg)
{
	long t = (long)arg;

	for (int i = 0; i < N; i++)
		request(t, i);
	return NULL;
}

static int cmp_d(const void *a, const void *b)
{
	const double x = *(const double *)a, y = *(const double *)b;

	return x < y ? -1 : x > y;
}

/* QB_LATENCY=1: one request at a time from one thread, each waited for
 * (submit -> callback), median and 90th percentile in us; the synchronous
 * drop-in call of the same request beside it. */
static void latency(const char *cells)
{
	enum { R = 200, WARM = 20 };
	static double q_us[R], d_us[R];

	for (int i = 0; i < R + WARM; i++) {
		long before;
		double t0;

		g_mode = 1;
		pthread_mutex_lock(&g_cnt.lock);
		before = g_cnt.done;
		pthread_mutex_unlock(&g_cnt.lock);
		t0 = now();
		request(0, i % N);
		pthread_mutex_lock(&g_cnt.lock);
		while (g_cnt.done == before)
			pthread_cond_wait(&g_cnt.cv, &g_cnt.lock);
		pthread_mutex_unlock(&g_cnt.lock);
		if (i >= WARM)
			q_us[i - WARM] = (now() - t0) * 1e6;
		g_mode = 0;
		t0 = now();
		request(0, i % N);
		if (i >= WARM)
			d_us[i - WARM] = (now() - t0) * 1e6;
	}
	qsort(q_us, R, sizeof(double), cmp_d);
	qsort(d_us, R, sizeof(double), cmp_d);
	printf("{\"op\": \"%s\", \"cells\": \"%s\", \"k\": %d, \"p\": %d, \"cell_bytes\": %llu, "
	       "\"queue_latency_us\": {\"p50\": %.1f, \"p90\": %.1f}, \"dropin_call_us\": {\"p50\": %.1f, \"p90\": %.1f}}\n",
	       g_update ? "update" : "encode", cells, K, P, (unsigned long long)CB, q_us[R / 2], q_us[R * 9 / 10],
	       d_us[R / 2], d_us[R * 9 / 10]);
}

static double run(int mode)
{
	pthread_t th[64];
	double t0, t1;

	g_mode = mode;
	g_cnt.done = 0;
	t0 = now();
	for (long t = 0; t < T; t++)
		pthread_create(&th[t], NULL, worker, (void *)t);
	for (int t = 0; t < T; t++)
		pthread_join(th[t], NULL);
	if (mode == 1) {
		pthread_mutex_lock(&g_cnt.lock);
		while (g_cnt.done < (long)T * N)
			pthread_cond_wait(&g_cnt.cv, &g_cnt.lock);
		pthread_mutex_unlock(&g_cnt.lock);
	}
	t1 = now();
	return (double)T * N * (g_update ? 1 : K) * CB / (t1 - t0) / (1 << 30);
}

int main(int argc, char **argv)
{
	unsigned char en[(64 + 8) * 64];
	ecg_ctx_t *ctx = NULL;
	ecg_queue_attr_t qa = {256, 100, 0};
	double isal, queue, cpu;
	uint64_t reqs = 0, batches = 0;

	if (argc > 1)
		CB = strtoull(argv[1], NULL, 0);
	if (argc > 2)
		T = atoi(argv[2]);
	const int devupdate = argc > 3 && strcmp(argv[3], "devupdate") == 0;
	g_update = argc > 3 && (strcmp(argv[3], "update") == 0 || devupdate);
	const int device = argc > 3 && (strcmp(argv[3], "device") == 0 || devupdate);
	if (argc > 4)
		N = atoi(argv[4]);	/* stripes per thread (device cells: HBM holds many) */
	if (N < 1 || T < 1 || T > 64)
		return 2;
	g_cells = malloc(device ? 1 : (size_t)T * N * (K + P) * CB);
	g_new = malloc(device ? 1 : (size_t)T * N * CB);
	for (size_t i = 0; !device && i < (size_t)T * N * (K + P) * CB; i++)
		g_cells[i] = (unsigned char)(i * 2654435761u >> 13);
	for (size_t i = 0; !device && i < (size_t)T * N * CB; i++)
		g_new[i] = (unsigned char)(i * 40503u >> 7);
	gf_gen_cauchy1_matrix(en, K + P, K);
	ec_init_tables(K, P, &en[K * K], g_tbls);
	for (int j = 0; j < K; j++)	/* ISA-L layout: row r, source j at (r * K + j) * 32 */
		for (int r = 0; r < P; r++)
			memcpy(&g_col[j][r * 32], &g_tbls[(r * K + j) * 32], 32);
	/* the CPU executor needs no device (host modes then skip nothing: the
	 * drop-in rows run the CPU path) */
	if ((!getenv("QB_CPU_QUEUE") && ecg_ctx_create(0, &ctx)) ||
	    ecg_queue_create(getenv("QB_CPU_QUEUE") ? NULL : ctx, &qa, &g_q)) {
		fprintf(stderr, "no device: %s\n", ecg_strerror());
		return 1;
	}
	if (device) {
		void *d = NULL;
		const size_t nb = (size_t)T * N * (K + P) * CB;
		/* QB_ONE_ALLOC=1: the new cells share the stripes' allocation (one
		 * placement lookup per request instead of two) */
		const int one = devupdate && getenv("QB_ONE_ALLOC") != NULL;

		if (ecg_dev_alloc(ctx, nb + (one ? (size_t)T * N * CB : 0), &d) || ecg_memset(ctx, d, 0x5A, nb, NULL) ||
		    ecg_stream_sync(ctx, NULL)) {
			fprintf(stderr, "device cells: %s\n", ecg_strerror());
			return 1;
		}
		g_dcells = d;
		if (devupdate) {
			void *dn = one ? (unsigned char *)d + nb : NULL, *dd = NULL;

			if ((!one && ecg_dev_alloc(ctx, (size_t)T * N * CB, &dn)) || ecg_dev_alloc(ctx, (size_t)T * CB, &dd) ||
			    ecg_memset(ctx, dn, 0xA7, (size_t)T * N * CB, NULL) || ecg_stream_sync(ctx, NULL)) {
				fprintf(stderr, "device new cells: %s\n", ecg_strerror());
				return 1;
			}
			g_dnew = dn;
			g_ddiff = dd;
		}
		if (getenv("QB_VERIFY") && devupdate) {
			/* patterned image and new cells, one queue run, every stripe's
			 * parity against parity ^= coef[vec_i] * (old ^ new) on the CPU */
			const size_t nn = (size_t)T * N * CB;
			unsigned char *h = malloc(nb), *g = malloc(nb), *hn = malloc(nn), *delta = malloc(CB);
			long bad = 0;

			for (size_t i = 0; i < nb / 8; i++) {
				const uint64_t v = (i + 1) * 0x9E3779B97F4A7C15ull;

				memcpy(h + i * 8, &v, 8);
			}
			for (size_t i = 0; i < nn / 8; i++) {
				const uint64_t v = (i + 7) * 0xC2B2AE3D27D4EB4Full;

				memcpy(hn + i * 8, &v, 8);
			}
			if (ecg_memcpy(ctx, d, h, nb, 0, NULL) || ecg_memcpy(ctx, g_dnew, hn, nn, 0, NULL) ||
			    ecg_stream_sync(ctx, NULL))
				return 1;
			run(1);
			if (ecg_memcpy(ctx, g, d, nb, 1, NULL) || ecg_stream_sync(ctx, NULL))
				return 1;
			for (size_t st = 0; st < (size_t)T * N; st++) {
				unsigned char *s = h + st * (K + P) * CB, *par[8];
				const int vec_i = (int)(st % K);

				for (uint64_t b = 0; b < CB; b++)
					delta[b] = s[vec_i * CB + b] ^ hn[st * CB + b];
				for (int r = 0; r < P; r++)
					par[r] = s + (K + r) * CB;
				ref_ec_encode_data_update((int)CB, K, P, vec_i, g_tbls, delta, par);
				bad += memcmp(s, g + st * (K + P) * CB, (size_t)(K + P) * CB) != 0;
			}
			printf("{\"op\": \"update\", \"cells\": \"device\", \"verify\": true, \"k\": %d, \"p\": %d, "
			       "\"cell_bytes\": %llu, \"threads\": %d, \"stripes\": %d, \"bad_stripes\": %ld}\n", K, P,
			       (unsigned long long)CB, T, T * N, bad);
			return bad ? 1 : 0;
		}
		if (getenv("QB_VERIFY")) {
			/* every stripe distinct: one queue run over a patterned image,
			 * then every stripe's parity against the CPU restatement */
			unsigned char *h = malloc(nb), *want = malloc(P * CB);
			long bad = 0;

			for (size_t i = 0; i < nb / 8; i++) {
				const uint64_t v = (i + 1) * 0x9E3779B97F4A7C15ull;

				memcpy(h + i * 8, &v, 8);
			}
			if (ecg_memcpy(ctx, d, h, nb, 0, NULL) || ecg_stream_sync(ctx, NULL))
				return 1;
			run(1);
			if (ecg_memcpy(ctx, h, d, nb, 1, NULL) || ecg_stream_sync(ctx, NULL))
				return 1;
			for (size_t st = 0; st < (size_t)T * N; st++) {
				unsigned char *s = h + st * (K + P) * CB, *src[64], *dst[8];

				for (int c = 0; c < K; c++)
					src[c] = s + c * CB;
				for (int r = 0; r < P; r++)
					dst[r] = want + r * CB;
				ref_simd_encode_data((int)CB, K, P, g_tbls, src, dst);
				bad += memcmp(want, s + (size_t)K * CB, (size_t)P * CB) != 0;
			}
			printf("{\"op\": \"encode\", \"cells\": \"device\", \"verify\": true, \"k\": %d, \"p\": %d, "
			       "\"cell_bytes\": %llu, \"threads\": %d, \"stripes\": %d, \"bad_stripes\": %ld}\n", K, P,
			       (unsigned long long)CB, T, T * N, bad);
			free(h);
			free(want);
			return bad ? 1 : 0;
		}
		if (getenv("QB_LATENCY")) {
			latency("device");
			return 0;
		}
		run(0);
		isal = run(0);
		run(1);
		queue = run(1);
		ecg_queue_stats(g_q, &reqs, &batches);
		if (getenv("QB_REPS")) {	/* spread of repeated queue runs */
			for (int r = atoi(getenv("QB_REPS")); r > 0; r--) {
				uint64_t r0 = reqs, b0 = batches;
				const double v = run(1);

				ecg_queue_stats(g_q, &reqs, &batches);
				fprintf(stderr, "queue run: %.2f GiB/s, %llu requests in %llu batches\n", v,
					(unsigned long long)(reqs - r0), (unsigned long long)(batches - b0));
			}
		}
		printf("{\"op\": \"%s\", \"cells\": \"device\", \"k\": %d, \"p\": %d, \"cell_bytes\": %llu, "
		       "\"threads\": %d, \"stripes_per_thread\": %d, \"isal_one_stripe_GiBps\": %.2f, "
		       "\"queue_GiBps\": %.2f, \"queue_requests\": %llu, \"queue_batches\": %llu}\n",
		       g_update ? "update" : "encode", K, P, (unsigned long long)CB, T, N, isal, queue, (unsigned long long)reqs,
		       (unsigned long long)batches);
		ecg_dev_free(ctx, d);
		if (g_dnew) {
			if (!one)
				ecg_dev_free(ctx, g_dnew);
			ecg_dev_free(ctx, g_ddiff);
		}
		ecg_queue_destroy(g_q);
		ecg_ctx_destroy(ctx);
		free(g_cells);
		free(g_new);
		return 0;
	}
	if (getenv("QB_LATENCY")) {
		latency(getenv("QB_CPU_QUEUE") ? "host, CPU executor" : "host");
		return 0;
	}
	if (getenv("QB_VERIFY") && !g_update) {
		/* host cells: parity zeroed, one queue run, every stripe checked */
		unsigned char *want = malloc(P * CB);
		long bad = 0;

		for (size_t st = 0; st < (size_t)T * N; st++)
			memset(g_cells + (st * (K + P) + K) * CB, 0, (size_t)P * CB);
		run(1);
		for (size_t st = 0; st < (size_t)T * N; st++) {
			unsigned char *s = g_cells + st * (K + P) * CB, *src[64], *dst[8];

			for (int c = 0; c < K; c++)
				src[c] = s + c * CB;
			for (int r = 0; r < P; r++)
				dst[r] = want + r * CB;
			ref_simd_encode_data((int)CB, K, P, g_tbls, src, dst);
			bad += memcmp(want, s + (size_t)K * CB, (size_t)P * CB) != 0;
		}
		printf("{\"op\": \"encode\", \"cells\": \"host\", \"verify\": true, \"k\": %d, \"p\": %d, "
		       "\"cell_bytes\": %llu, \"threads\": %d, \"stripes\": %d, \"bad_stripes\": %ld}\n", K, P,
		       (unsigned long long)CB, T, T * N, bad);
		free(want);
		return bad ? 1 : 0;
	}
	run(0);			/* warm up staging / code objects */
	isal = run(0);
	run(1);
	queue = run(1);
	ecg_queue_stats(g_q, &reqs, &batches);
	cpu = run(2);
	printf("{\"op\": \"%s\", \"queue\": \"%s\", \"k\": %d, \"p\": %d, \"cell_bytes\": %llu, \"threads\": %d, \"stripes_per_thread\": %d, "
	       "\"isal_one_stripe_GiBps\": %.2f, \"queue_GiBps\": %.2f, \"queue_requests\": %llu, "
	       "\"queue_batches\": %llu, \"cpu_gfni_same_threads_GiBps\": %.2f}\n",
	       g_update ? "update" : "encode", getenv("QB_CPU_QUEUE") ? "cpu-executor" : "gpu", K, P,
	       (unsigned long long)CB, T, N, isal, queue, (unsigned long long)reqs,
	       (unsigned long long)batches, cpu);
	ecg_queue_destroy(g_q);
	if (ctx)
		ecg_ctx_destroy(ctx);
	free(g_cells);
	free(g_new);
	return 0;
}
