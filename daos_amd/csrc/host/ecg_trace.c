/*
 * ecg_trace.c -- roctx ranges around launches, staging and queue batches
 * (the reference's EC trace hook is compile-time EC_DEBUG /
 * EC_REASB_TRACE logging, ref:src/object/cli_ec.c:20-31; here the ranges
 * land in rocprofv3 --marker-trace timelines next to the kernels).
 *
 * The roctx library is dlopen'ed on first use, so libecg has no link-time
 * dependency on the profiler SDK and costs one predictable branch per range
 * when it is absent.  ECG_ROCTX=0 turns the ranges off.
 */
#include <dlfcn.h>
#include <pthread.h>
#include <stdlib.h>

#include "ecg_internal.h"

typedef int (*push_fn_t)(const char *);
typedef int (*pop_fn_t)(void);

static push_fn_t g_push;
static pop_fn_t g_pop;
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void trace_init(void)
{
	static const char *const libs[] = {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so",
					   "libroctx64.so.4", "libroctx64.so"};
	const char *env = getenv("ECG_ROCTX");
	void *h = NULL;

	if (env && env[0] == '0')
		return;
	for (unsigned i = 0; i < sizeof(libs) / sizeof(libs[0]) && h == NULL; i++)
		h = dlopen(libs[i], RTLD_NOW | RTLD_LOCAL);
	if (h == NULL)
		return;
	g_push = (push_fn_t)dlsym(h, "roctxRangePushA");
	g_pop = (pop_fn_t)dlsym(h, "roctxRangePop");
	if (g_push == NULL || g_pop == NULL)
		g_push = NULL, g_pop = NULL;
}

void ecg_trace_push(const char *name)
{
	pthread_once(&g_once, trace_init);
	if (g_push)
		g_push(name);
}

void ecg_trace_pop(void)
{
	if (g_pop)
		g_pop();
}

int ecg_trace_active(void)
{
	pthread_once(&g_once, trace_init);
	return g_push != NULL;
}
