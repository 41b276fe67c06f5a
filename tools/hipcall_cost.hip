/*
 * hipcall_cost.c -- what the runtime calls around one synchronous device-cell
 * drop-in call cost on this box (us per call, median of 5 x 2000): pointer
 * attribute and address-range queries, event record / stream wait / event
 * synchronize, stream query and synchronize, an empty-kernel launch.  Sizes
 * the per-call overheads of ecg_stage.c's matmul_device.  Bench
 * infrastructure; the placement queries are also timed from 1 / 4 / 16
 * threads at once.  Build: hipcc -O2 --offload-arch=gfx950 -lhsa-runtime64
 * -o build/tools/hipcall_cost tools/hipcall_cost.hip
 */
#include <hip/hip_runtime.h>
#include <hsa/hsa_ext_amd.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

__global__ void nop_kernel(int *p)
{
	if (p && threadIdx.x == 1000)
		p[0] = 1;
}

static double now(void)
{
	struct timespec t;

	clock_gettime(CLOCK_MONOTONIC, &t);
	return t.tv_sec + t.tv_nsec * 1e-9;
}

#define N 2000
#define TIME(name, body)                                                          \
	do {                                                                      \
		double best[5];                                                   \
		for (int r = 0; r < 5; r++) {                                     \
			double t0 = now();                                        \
			for (int i = 0; i < N; i++) {                             \
				body;                                             \
			}                                                         \
			best[r] = (now() - t0) / N * 1e6;                         \
		}                                                                 \
		for (int a = 0; a < 5; a++)                                       \
			for (int b = a + 1; b < 5; b++)                           \
				if (best[b] < best[a]) {                          \
					double x = best[a];                       \
					best[a] = best[b];                        \
					best[b] = x;                              \
				}                                                 \
		printf("{\"call\": \"%s\", \"us\": %.3f}\n", name, best[2]);     \
	} while (0)

/* a placement query from T threads at once, each on its own host buffer */
static int g_which;
static pthread_barrier_t g_bar;

static void *qthread(void *arg)
{
	char *h = (char *)malloc(65536);
	hipPointerAttribute_t a;
	hsa_amd_pointer_info_t info;
	unsigned int mt;

	(void)arg;
	pthread_barrier_wait(&g_bar);
	for (int i = 0; i < 20000; i++) {
		if (g_which == 0) {
			(void)hipPointerGetAttributes(&a, h + 64);
			(void)hipGetLastError();
		} else if (g_which == 1) {
			(void)hipPointerGetAttribute(&mt, HIP_POINTER_ATTRIBUTE_MEMORY_TYPE, (hipDeviceptr_t)(h + 64));
			(void)hipGetLastError();
		} else {
			info.size = sizeof(info);
			(void)hsa_amd_pointer_info(h + 64, &info, NULL, NULL, NULL);
		}
	}
	pthread_barrier_wait(&g_bar);
	free(h);
	return NULL;
}

static void threaded(void)
{
	static const char *names[] = {"hipPointerGetAttributes", "hipPointerGetAttribute(MEMORY_TYPE)",
				      "hsa_amd_pointer_info"};
	for (int w = 0; w < 3; w++)
		for (int T = 1; T <= 16; T *= 4) {
			pthread_t th[16];
			double t0, t1;

			g_which = w;
			pthread_barrier_init(&g_bar, NULL, T + 1);
			for (int t = 0; t < T; t++)
				pthread_create(&th[t], NULL, qthread, NULL);
			pthread_barrier_wait(&g_bar);
			t0 = now();
			pthread_barrier_wait(&g_bar);
			t1 = now();
			for (int t = 0; t < T; t++)
				pthread_join(th[t], NULL);
			pthread_barrier_destroy(&g_bar);
			printf("{\"call\": \"%s (host ptr)\", \"threads\": %d, \"us\": %.3f}\n", names[w], T,
			       (t1 - t0) / 20000 * 1e6);
		}
}

int main(void)
{
	hipStream_t st, st2;
	hipEvent_t ev, ev2;
	hipPointerAttribute_t a;
	hipDeviceptr_t base;
	size_t size;
	void *d;
	char *h = (char *)malloc(1 << 20);

	if (hipSetDevice(0) != hipSuccess || hipMalloc(&d, 64 << 20) != hipSuccess)
		return 1;
	hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
	hipStreamCreateWithFlags(&st2, hipStreamNonBlocking);
	hipEventCreateWithFlags(&ev, hipEventDisableTiming);
	hipEventCreateWithFlags(&ev2, hipEventDisableTiming);
	TIME("hipPointerGetAttributes(device)", hipPointerGetAttributes(&a, (char *)d + 4096));
	TIME("hipPointerGetAttributes(host malloc)", (void)hipPointerGetAttributes(&a, h + 64); (void)hipGetLastError());
	TIME("hipMemGetAddressRange(device)", hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)((char *)d + 4096)));
	TIME("hipStreamQuery(idle)", hipStreamQuery(st2));
	TIME("hipEventRecord+hipStreamWaitEvent", hipEventRecord(ev2, st2); hipStreamWaitEvent(st, ev2, 0));
	TIME("launch+hipStreamSynchronize", hipLaunchKernelGGL(nop_kernel, dim3(1), dim3(64), 0, st, (int *)0);
	     hipStreamSynchronize(st));
	TIME("launch+hipEventRecord+hipEventSynchronize", hipLaunchKernelGGL(nop_kernel, dim3(1), dim3(64), 0, st,
									      (int *)0);
	     hipEventRecord(ev, st); hipEventSynchronize(ev));
	TIME("launch+hipEventRecord+poll hipEventQuery", hipLaunchKernelGGL(nop_kernel, dim3(1), dim3(64), 0, st,
									     (int *)0);
	     hipEventRecord(ev, st); while (hipEventQuery(ev) == hipErrorNotReady););
	TIME("launch+poll hipStreamQuery", hipLaunchKernelGGL(nop_kernel, dim3(1), dim3(64), 0, st, (int *)0);
	     while (hipStreamQuery(st) == hipErrorNotReady););
	TIME("hipSetDevice", hipSetDevice(0));
	threaded();
	hipFree(d);
	return 0;
}
