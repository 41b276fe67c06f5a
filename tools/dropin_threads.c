/*
 * dropin_threads.c -- T pthreads calling the ISA-L drop-in's ec_encode_data
 * on their own host cells (EC_k+p, C-byte cells, N calls each): aggregate
 * GiB/s of data.  Run with and without a visible GPU to see what the
 * per-call placement query costs under contention (without a device the
 * drop-in never asks the HIP runtime where a pointer lives).  With "tiny"
 * as 5th argument every call has len = 1: the per-call overhead alone.
 * usage: dropin_threads C T [N] [k] [tiny] -> one JSON line.  Bench
 * infrastructure.
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "ecg.h"
#include "ecg_isal.h"

static int K = 8, P = 2, T = 16, N = 2000, CB = 32768, TINY;
static unsigned char g_tbls[64 * 8 * 32];
static pthread_barrier_t g_go;

static double now(void)
{
	struct timespec t;

	clock_gettime(CLOCK_MONOTONIC, &t);
	return t.tv_sec + t.tv_nsec * 1e-9;
}

static void *worker(void *arg)
{
	unsigned char *data[64], *par[8];
	int i;

	(void)arg;
	for (i = 0; i < K; i++) {
		data[i] = malloc(CB);
		memset(data[i], i * 7 + 1, CB);
	}
	for (i = 0; i < P; i++)
		par[i] = malloc(CB);
	ec_encode_data(CB, K, P, g_tbls, data, par);
	pthread_barrier_wait(&g_go);
	for (i = 0; i < N; i++)
		ec_encode_data(TINY ? 1 : CB, K, P, g_tbls, data, par);
	pthread_barrier_wait(&g_go);
	for (i = 0; i < K; i++)
		free(data[i]);
	for (i = 0; i < P; i++)
		free(par[i]);
	return NULL;
}

int main(int argc, char **argv)
{
	unsigned char en[(64 + 8) * 64];
	pthread_t th[256];
	double t0, t1;
	int t;

	if (argc > 1)
		CB = atoi(argv[1]);
	if (argc > 2)
		T = atoi(argv[2]);
	if (argc > 3)
		N = atoi(argv[3]);
	if (argc > 4)
		K = atoi(argv[4]);
	TINY = argc > 5 && strcmp(argv[5], "tiny") == 0;
	if (T < 1 || T > 256 || K < 1 || K > 64)
		return 2;
	gf_gen_cauchy1_matrix(en, K + P, K);
	ec_init_tables(K, P, &en[K * K], g_tbls);
	pthread_barrier_init(&g_go, NULL, (unsigned)T + 1);
	for (t = 0; t < T; t++)
		pthread_create(&th[t], NULL, worker, NULL);
	pthread_barrier_wait(&g_go);
	t0 = now();
	pthread_barrier_wait(&g_go);
	t1 = now();
	for (t = 0; t < T; t++)
		pthread_join(th[t], NULL);
	printf("{\"k\": %d, \"p\": %d, \"cell_bytes\": %d, \"threads\": %d, \"calls_per_thread\": %d, \"tiny\": %d, "
	       "\"us_per_call\": %.3f, \"GiBps\": %.2f, \"devices\": %d, \"kernel\": \"%s\"}\n",
	       K, P, CB, T, N, TINY, (t1 - t0) / N * 1e6,
	       TINY ? 0.0 : (double)T * N * K * CB / (t1 - t0) / (1 << 30), ecg_device_count(), ecg_cpu_isa());
	return 0;
}
