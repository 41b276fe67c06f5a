/*
 * dropin_bench.c -- where the ISA-L drop-in's crossover lies.  One thread
 * calls ec_encode_data (one stripe per call, the reference's pattern:
 * ref:src/object/cli_ec.c:540, srv_ec_aggregate.c:693) on HOST cells
 * (malloc'd, as DAOS's bio/sgl buffers are) through
 *   cpu : the product CPU path          (ecg_set_dropin_crossover(UINT64_MAX))
 *   gpu : the GPU with pinned staging   (ecg_set_dropin_crossover(0))
 * and on DEVICE cells (dev: the HIP kernel in place), for EC_4P2 / EC_8P2 /
 * EC_16P2 and cells of 4 KiB .. 16 MiB; plus ec_encode_data_update and
 * xor_gen(3) (agg_update_parity's pair) at each cell size.  One JSON line per
 * row on stdout, then a summary line with the measured crossover: the
 * smallest len * (k + p) from which the GPU path beats the CPU path at every
 * larger measured size (none if the CPU wins throughout).
 * Bench infrastructure; no oracle (parity is the tests' job).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "ecg.h"
#include "ecg_isal.h"

static double now(void)
{
	struct timespec t;

	clock_gettime(CLOCK_MONOTONIC, &t);
	return t.tv_sec + t.tv_nsec * 1e-9;
}

/* median-of-3 of the mean time per call over >= 30 ms, microseconds */
static double time_us(void (*fn)(void *), void *arg)
{
	double best[3];
	int r, it, n;

	fn(arg);
	fn(arg);
	for (n = 1;; n *= 2) {
		double t = now();

		for (it = 0; it < n; it++)
			fn(arg);
		if (now() - t > 0.03)
			break;
	}
	for (r = 0; r < 3; r++) {
		double t = now();

		for (it = 0; it < n; it++)
			fn(arg);
		best[r] = (now() - t) / n * 1e6;
	}
	/* median */
	if (best[0] > best[1]) { double x = best[0]; best[0] = best[1]; best[1] = x; }
	if (best[1] > best[2]) { double x = best[1]; best[1] = best[2]; best[2] = x; }
	if (best[0] > best[1]) { double x = best[0]; best[0] = best[1]; best[1] = x; }
	return best[1];
}

struct call {
	int len, k, p;
	unsigned char *tbls;
	unsigned char *data[16], *coding[3];
	unsigned char *old, *diff;
};

static void enc(void *a)
{
	struct call *c = a;

	ec_encode_data(c->len, c->k, c->p, c->tbls, c->data, c->coding);
}

/* agg_update_parity's per-cell pair: diff = old ^ new, parity ^= coef * diff */
static void upd(void *a)
{
	struct call *c = a;
	void *v[3] = {c->old, c->data[0], c->diff};

	xor_gen(3, c->len, v);
	ec_encode_data_update(c->len, c->k, c->p, 1, c->tbls, c->diff, c->coding);
}

int main(int argc, char **argv)
{
	static const int kp[][2] = {{4, 2}, {8, 2}, {16, 2}};
	const int maxlen = argc > 1 ? atoi(argv[1]) : 16 << 20;
	const int gpu = ecg_device_count() > 0;
	uint64_t cross = UINT64_MAX;	/* smallest len*(k+p) with the GPU ahead from there on */
	ecg_ctx_t *ctx = NULL;
	size_t t;

	if (gpu && ecg_ctx_create(0, &ctx) != 0) {
		fprintf(stderr, "ctx: %s\n", ecg_strerror());
		return 1;
	}
	for (t = 0; t < sizeof(kp) / sizeof(kp[0]); t++) {
		const int k = kp[t][0], p = kp[t][1];
		unsigned char en[(16 + 2) * 16], tbls[16 * 2 * 32];
		uint64_t row_cross = UINT64_MAX;
		int len;

		gf_gen_cauchy1_matrix(en, k + p, k);
		ec_init_tables(k, p, &en[k * k], tbls);
		for (len = 4096; len <= maxlen; len *= 4) {
			struct call c = {.len = len, .k = k, .p = p, .tbls = tbls};
			double cpu_us, gpu_us = -1, dev_us = -1, ucpu = -1, ugpu = -1;
			void *dbuf = NULL;
			int j;

			for (j = 0; j < k; j++) {
				c.data[j] = malloc(len);
				for (int i = 0; i < len; i++)
					c.data[j][i] = (unsigned char)(i * 7 + j * 13 + (i >> 9));
			}
			for (j = 0; j < p; j++)
				c.coding[j] = calloc(1, len);
			c.old = calloc(1, len);
			c.diff = malloc(len);
			ecg_set_dropin_crossover(UINT64_MAX);
			cpu_us = time_us(enc, &c);
			ucpu = time_us(upd, &c);
			if (gpu) {
				struct call d = c;

				ecg_set_dropin_crossover(0);
				gpu_us = time_us(enc, &c);
				ugpu = time_us(upd, &c);
				if (ecg_dev_alloc(ctx, (size_t)(k + p) * len, &dbuf) == 0) {
					for (j = 0; j < k; j++)
						d.data[j] = (unsigned char *)dbuf + (size_t)j * len;
					for (j = 0; j < p; j++)
						d.coding[j] = (unsigned char *)dbuf + (size_t)(k + j) * len;
					dev_us = time_us(enc, &d);
					ecg_dev_free(ctx, dbuf);
				}
				if (gpu_us < cpu_us) {
					if (row_cross == UINT64_MAX)
						row_cross = (uint64_t)len * (k + p);
				} else {
					row_cross = UINT64_MAX;
				}
			}
			printf("{\"k\": %d, \"p\": %d, \"len\": %d, \"cpu_us\": %.2f, \"gpu_staged_us\": %.2f, "
			       "\"device_cells_us\": %.2f, \"cpu_GiBps\": %.2f, \"gpu_staged_GiBps\": %.2f, "
			       "\"update_cpu_us\": %.2f, \"update_gpu_us\": %.2f, \"cpu_isa\": \"%s\"}\n",
			       k, p, len, cpu_us, gpu_us, dev_us, (double)k * len / cpu_us * 1e6 / (1 << 30),
			       gpu_us > 0 ? (double)k * len / gpu_us * 1e6 / (1 << 30) : -1.0, ucpu, ugpu,
			       ecg_cpu_isa());
			fflush(stdout);
			for (j = 0; j < k; j++)
				free(c.data[j]);
			for (j = 0; j < p; j++)
				free(c.coding[j]);
			free(c.old);
			free(c.diff);
		}
		if (row_cross < cross)
			cross = row_cross;
	}
	if (cross == UINT64_MAX)
		printf("{\"crossover_bytes\": null, \"note\": \"CPU path ahead at every measured size\"}\n");
	else
		printf("{\"crossover_bytes\": %llu}\n", (unsigned long long)cross);
	if (ctx)
		ecg_ctx_destroy(ctx);
	return 0;
}
