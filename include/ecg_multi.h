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
#include "ecg_daos.h"

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
/* NUMA node shard i's worker thread runs on (its device's node, from sysfs),
 * -1 when it is not pinned (unknown node, $ECG_NUMA=0). */
int ecg_multi_numa_node(const ecg_multi_t *m, int i);
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

/* ---- device-resident rebuild / aggregation ops ---------------------------
 * The ops DAOS's rebuild and aggregation paths run, sharded like
 * ecg_multi_encode: per-shard arrays (nstripes[i], buffers and checksum
 * outputs on shard i's device), the operands of the single-device call
 * otherwise, same strides for every shard; each shard's checksums go to its
 * own csums[i] in that call's layout.  ECG_MULTI_ASYNC as above.
 *   ecg_multi_encode_csum   ecg_encode_csum (parity + chunk checksums of the
 *                           parity: obj_ec_encode_buf + daos_csummer_calc_iods,
 *                           ref:src/object/srv_obj_migrate.c:1122-1160)
 *   ecg_multi_recover_csum  ecg_recover_csum (regenerated cells + their
 *                           checksums)
 *   ecg_multi_update        ecg_update (agg_update_parity's xor_gen +
 *                           ec_encode_data_update, ref:src/object/
 *                           srv_ec_aggregate.c:1086-1102) */
int ecg_multi_encode_csum(ecg_multi_t *m, int k, int p, uint64_t cell_bytes, const uint32_t *nstripes,
			  const void *const *data, int64_t data_stripe_stride, void *const *parity,
			  int64_t parity_cell_stride, int64_t parity_stripe_stride, int type, uint64_t chunksize,
			  uint64_t rec_size, void *const *csums, unsigned flags);
int ecg_multi_recover_csum(ecg_multi_t *m, int k, int p, uint64_t cell_bytes, const uint32_t *nstripes,
			   void *const *stripes, int64_t stripe_stride, const uint32_t *err_list, int nerrs,
			   int type, uint64_t chunksize, uint64_t rec_size, void *const *csums, unsigned flags);
int ecg_multi_update(ecg_multi_t *m, int k, int p, uint64_t cell_bytes, const uint32_t *nstripes, int nupd,
		     const uint32_t *cell_idx, const void *const *old_cells, const void *const *new_cells,
		     int64_t upd_stripe_stride, void *const *parity, int64_t parity_cell_stride,
		     int64_t parity_stripe_stride, unsigned flags);

/* Rebuild of a parity shard over a fetched record range, sharded
 * (migrate_update_parity, ref:src/object/srv_obj_migrate.c:1096-1181;
 * ecg_migrate_update_parity in ecg_daos.h).  ecg_multi_migrate_range gives
 * shard i's records [*off, *off + *sz): contiguous runs of whole stripes
 * (whole cells when !encode), the partial head on shard 0 and the partial
 * tail on the last shard -- the walk's own cut points, so the shards cut
 * exactly the pieces one walk of the whole range cuts.  buffers[i] holds
 * shard i's records on its device; its parity cells go to parity_out[i] and
 * its checksums to csums_out[i].  pieces receives every piece in range
 * order, shard i's at [shard_first[i], shard_first[i+1]) (shard_first:
 * n + 1 entries, may be NULL) with buf_off / csum_off relative to that
 * shard's buffers.  Synchronous unless ECG_MULTI_ASYNC. */
int ecg_multi_migrate_range(const ecg_multi_t *m, uint32_t oc_id, uint64_t e_len, uint64_t iod_size,
			    uint64_t offset, uint64_t size, int encode, int i, uint64_t *off, uint64_t *sz);
int ecg_multi_migrate_update_parity(ecg_multi_t *m, uint32_t oc_id, uint64_t e_len, uint64_t iod_size,
				    uint32_t shard, const void *const *buffers, uint64_t offset, uint64_t size,
				    int encode, int csum_type, uint64_t chunksize, void *const *parity_out,
				    void *const *csums_out, ecg_migrate_piece_t *pieces, uint32_t pieces_cap,
				    uint32_t *npieces, uint32_t *shard_first, unsigned flags);

/* Batching facade spread over the shards' devices: the queue's staging slots
 * are assigned to the shards round-robin (ecg.h, ecg_queue_*).  The queue
 * must be destroyed before the ecg_multi_t. */
int ecg_queue_create_multi(ecg_multi_t *m, const ecg_queue_attr_t *attr, ecg_queue_t **q);

#ifdef __cplusplus
}
#endif
#endif
