/*
 * upd_latency.c -- host-side cost of one batched call, the queue's per-batch
 * launch: ecg_update_ptrs (n one-cell EC_8P2 updates on distinct device
 * stripes) against ecg_matmul_ptrs (n EC_8P2 stripe encodes), n = 1 .. 256.
 * Per call: the time inside the call (host work + enqueue) and the time to
 * completion (call + stream sync), median of 200 calls; and the time inside
 * the call when calls are issued back to back behind running work ("busy").
 * One JSON line per n.
 * usage: upd_latency [cell bytes, default 131072].  Bench infrastructure.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "ecg.h"

static double now_us(void)
{
	struct timespec t;

	clock_gettime(CLOCK_MONOTONIC, &t);
	return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

static int cmp(const void *a, const void *b)
{
	const double x = *(const double *)a, y = *(const double *)b;

	return x < y ? -1 : x > y;
}

static double median(double *v, int n)
{
	qsort(v, n, sizeof(*v), cmp);
	return v[n / 2];
}

int main(int argc, char **argv)
{
	enum { K = 8, P = 2, REPS = 200, NMAX = 256 };
	const uint64_t C = argc > 1 ? strtoull(argv[1], NULL, 0) : 131072;
	static const int ns[] = {1, 4, 17, 64, 256};
	unsigned char en[(K + P) * K];
	ecg_ctx_t *ctx = NULL;
	void *d = NULL, *st = NULL;
	static void *ucells[NMAX * (2 + P)], *ecells[NMAX * (K + P)];
	static uint8_t vec[NMAX];
	static double call_u[REPS], done_u[REPS], call_e[REPS], done_e[REPS], async_u[REPS], async_e[REPS];

	if (ecg_ctx_create(0, &ctx) || ecg_stream_create(ctx, &st) ||
	    ecg_dev_alloc(ctx, (size_t)NMAX * (K + P + 1) * C, &d)) {
		fprintf(stderr, "setup: %s\n", ecg_strerror());
		return 1;
	}
	ecg_gen_cauchy1(K, P, en);
	for (int s = 0; s < NMAX; s++) {
		unsigned char *b = (unsigned char *)d + (size_t)s * (K + P + 1) * C;

		for (int j = 0; j < K + P; j++)
			ecells[s * (K + P) + j] = b + (size_t)j * C;
		ucells[s * (2 + P)] = b + (size_t)(s % K) * C;	/* old: the stripe's data cell */
		ucells[s * (2 + P) + 1] = b + (size_t)(K + P) * C;	/* new: the stripe's spare cell */
		for (int r = 0; r < P; r++)
			ucells[s * (2 + P) + 2 + r] = b + (size_t)(K + r) * C;
		vec[s] = (uint8_t)(s % K);
	}
	/* shuffle the encode table's stripes so it stays a pointer table (not affine) */
	for (int s = NMAX - 1; s > 0; s--) {
		const int o = (s * 7919) % (s + 1);
		void *tmp[K + P];

		memcpy(tmp, &ecells[s * (K + P)], sizeof(tmp));
		memcpy(&ecells[s * (K + P)], &ecells[o * (K + P)], sizeof(tmp));
		memcpy(&ecells[o * (K + P)], tmp, sizeof(tmp));
	}
	for (size_t x = 0; x < sizeof(ns) / sizeof(ns[0]); x++) {
		const int n = ns[x];

		for (int i = 0; i < 20; i++) {		/* warm-up */
			ecg_update_ptrs(ctx, K, P, C, (uint32_t)n, ucells, vec, st);
			ecg_matmul_ptrs(ctx, K, P, &en[K * K], C, (uint32_t)n, ecells, st);
		}
		ecg_stream_sync(ctx, st);
		for (int i = 0; i < REPS; i++) {
			double t0 = now_us(), t1, t2;

			if (ecg_update_ptrs(ctx, K, P, C, (uint32_t)n, ucells, vec, st))
				return fprintf(stderr, "update_ptrs: %s\n", ecg_strerror()), 1;
			t1 = now_us();
			ecg_stream_sync(ctx, st);
			t2 = now_us();
			call_u[i] = t1 - t0;
			done_u[i] = t2 - t0;
			t0 = now_us();
			if (ecg_matmul_ptrs(ctx, K, P, &en[K * K], C, (uint32_t)n, ecells, st))
				return fprintf(stderr, "matmul_ptrs: %s\n", ecg_strerror()), 1;
			t1 = now_us();
			ecg_stream_sync(ctx, st);
			t2 = now_us();
			call_e[i] = t1 - t0;
			done_e[i] = t2 - t0;
		}
		/* back to back, the stream kept busy (synchronised every 8 calls):
		 * what a queue's worker sees, launching behind its last batch */
		for (int i = 0; i < REPS; i++) {
			double t0 = now_us();

			if (ecg_update_ptrs(ctx, K, P, C, (uint32_t)n, ucells, vec, st))
				return fprintf(stderr, "update_ptrs: %s\n", ecg_strerror()), 1;
			async_u[i] = now_us() - t0;
			if (i % 8 == 7)
				ecg_stream_sync(ctx, st);
		}
		ecg_stream_sync(ctx, st);
		for (int i = 0; i < REPS; i++) {
			double t0 = now_us();

			if (ecg_matmul_ptrs(ctx, K, P, &en[K * K], C, (uint32_t)n, ecells, st))
				return fprintf(stderr, "matmul_ptrs: %s\n", ecg_strerror()), 1;
			async_e[i] = now_us() - t0;
			if (i % 8 == 7)
				ecg_stream_sync(ctx, st);
		}
		ecg_stream_sync(ctx, st);
		printf("{\"n\": %d, \"cell_bytes\": %llu, \"update_ptrs_call_us\": %.1f, \"update_ptrs_done_us\": %.1f, "
		       "\"matmul_ptrs_call_us\": %.1f, \"matmul_ptrs_done_us\": %.1f, \"update_ptrs_busy_call_us\": %.1f, "
		       "\"matmul_ptrs_busy_call_us\": %.1f}\n", n, (unsigned long long)C,
		       median(call_u, REPS), median(done_u, REPS), median(call_e, REPS), median(done_e, REPS),
		       median(async_u, REPS), median(async_e, REPS));
		fflush(stdout);
	}
	ecg_dev_free(ctx, d);
	ecg_stream_destroy(ctx, st);
	ecg_ctx_destroy(ctx);
	return 0;
}
