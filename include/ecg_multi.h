/*
 * ecg_multi.h -- stripe sharding over several MI355X devices inside one
 * process.
 *
 * A DAOS engine is one process with many xstreams; the rebuild loop over
 * full stripes (migrate_update_parity, ref:src/object/srv_obj_migrate.c:
 * 1116-1177) and the aggregation ULTs on the offload xstream
 * (ref:src/object/srv_ec_aggregate.c:701-734) hand the codec independent
 * stripes.  An ecg_multi splits a batch of S stripes into contiguous ranges,
 * one per shard, and runs each range on its own device from its own host
 * thread, with its own context (streams, staging, decode-matrix cache).  No
 * collective and no device-to-device traffic: stripes are independent.
 *
 * Shards are listed by device index; a device may appear several times (each
 * entry still gets its own context and thread), which is how the API is
 * exercised on a one-GPU box.  devices == NULL / n == 0 takes the list from
 * $ECG_DEVICES ("0,1,2,3", or "all"), else every visible gfx950 device.
 *
 * All calls return 0 or a negative DAOS errno (ecg.h).  Calls on one
 * ecg_multi_t are serialised; different ecg_multi_t are independent.
 */
#ifndef ECG_MULTI_H
#define ECG_MULTI_H

#include <stddef.h>
#include <stdint.h>

#include "ecg.h"

#ifdef __cplusplus
extern "C" {
#endif

#define ECG_MULTI_MAX 64	/* shards per ecg_multi_t */
/* Device-resident calls only: return once every shard's launches are
 * enqueued; ecg_multi_sync waits for them.  Every buffer the call names must
 * stay allocated and untouched by the caller until ecg_multi_sync returns
 * (ecg_multi_destroy also waits).  The _host calls ignore it: they always
 * return with their outputs in host memory. */
#define ECG_MULTI_ASYNC 0x1u

typedef struct ecg_multi ecg_multi_t;

int ecg_multi_create(const int *devices, int n, ecg_multi_t **m);
/* Waits for outstanding work, stops the threads, destroys the contexts. */
void ecg_multi_destroy(ecg_multi_t *m);
int ecg_multi_count(const ecg_multi_t *m);
/* Shard i's context: allocate shard i's device buffers through it.  Owned by
 * the ecg_multi_t (do not destroy). NULL when i is out of range. */
ecg_ctx_t *ecg_multi_ctx(ecg_multi_t *m, int i);
/* Shard i's contiguous range [*first, *first + *count) of a batch of S
 * stripes (the first S % n shards get one extra stripe). */
int ecg_multi_range(const ecg_multi_t *m, uint32_t S, int i, uint32_t *first, uint32_t *count);

/* ---- device-resident batches: shard i's stripes live on shard i's device --
 * Arrays are indexed by shard: nstripes[i] stripes at data[i] / parity[i] /
 * stripes[i], in the layouts of ecg_encode / ecg_recover (same strides for
 * every shard).  Each shard's thread launches on its context's stream; the
 * call returns when every shard has finished (or, with ECG_MULTI_ASYNC, when
 * every launch is enqueued).  The first failing shard's code is returned. */
int ecg_multi_encode(ecg_multi_t *m, int k, int p, uint64_t cell_bytes, const uint32_t *nstripes,
		     const void *const *data, int64_t data_stripe_stride, void *const *parity,
		     int64_t parity_cell_stride, int64_t parity_stripe_stride, unsigned flags);
int ecg_multi_recover(ecg_multi_t *m, int k, int p, uint64_t cell_bytes, const uint32_t *nstripes,
		      void *const *stripes, int64_t stripe_stride, const uint32_t *err_list, int nerrs,
		      unsigned flags);
/* Waits for every shard's context stream. */
int ecg_multi_sync(ecg_multi_t *m);

/* ---- host-resident batches (PCIe-inclusive): ONE batch in host memory ----
 * data [S][k][C] -> parity [p][S][C] (ecg_encode_host), or in place over
 * [S][k+p][C] (ecg_recover_host); shard i streams its stripe range through
 * its device's staging.  Synchronous. */
int ecg_multi_encode_host(ecg_multi_t *m, int k, int p, uint64_t cell_bytes, uint32_t nstripes,
			  const void *data, void *parity, uint32_t chunk_stripes);
int ecg_multi_recover_host(ecg_multi_t *m, int k, int p, uint64_t cell_bytes, uint32_t nstripes,
			   void *stripes, const uint32_t *err_list, int nerrs, uint32_t chunk_stripes);

/* Batching facade spread over the shards' devices: the queue's staging slots
 * are assigned to the shards round-robin (ecg.h, ecg_queue_*).  The queue
 * must be destroyed before the ecg_multi_t. */
int ecg_queue_create_multi(ecg_multi_t *m, const ecg_queue_attr_t *attr, ecg_queue_t **q);

#ifdef __cplusplus
}
#endif
#endif
