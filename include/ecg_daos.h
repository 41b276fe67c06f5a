/*
 * ecg_daos.h -- the DAOS EC codec surface (src/object/obj_ec.h) backed by
 * the MI355X engine.
 *
 * Mirrors, with the same argument meaning, return codes and buffer
 * ownership, the codec functions of ref:src/object/obj_ec.h:731-845 and
 * ref:src/object/cli_ec.c.  DAOS-private aggregates (dc_object,
 * obj_reasb_req, daos_oclass_attr) are replaced by the scalars the codec
 * actually consumes (class id, k, p, cell bytes, LOGICAL cell indices --
 * the obj_ec_shard_off physical->logical mapping stays in the caller).
 * Names carry an ecg_ prefix so the library links next to libdaos; the
 * maintainer's glue forwards the reference functions here.
 *
 *   ecg_obj_ec_codec_init/fini/get  <- obj_ec_codec_init/fini/get
 *                                      ref:src/object/obj_class.c:511-649
 *   ecg_obj_ec_encode_buf           <- obj_ec_encode_buf
 *                                      ref:src/object/cli_ec.c:548-573
 *   ecg_obj_ec_recov_codec_init     <- obj_ec_recov_codec_alloc + _init
 *                                      ref:src/object/cli_ec.c:1953-1993, 2152-2250
 *   ecg_obj_ec_recov_data           <- obj_ec_recov_data's stripe loop over
 *                                      obj_ec_recov_stripe
 *                                      ref:src/object/cli_ec.c:2626-2643, 2814-2885
 *   ecg_obj_ec_encode_stripes       <- obj_ec_recx_encode's stripe loop
 *                                      ref:src/object/cli_ec.c:593-663
 *   ecg_agg_update_parity           <- agg_update_parity + agg_diff_preprocess
 *                                      ref:src/object/srv_ec_aggregate.c:1006-1105
 *   ecg_agg_recalc_parity           <- agg_recalc_parity
 *                                      ref:src/object/srv_ec_aggregate.c:1110-1138
 *   ecg_obj_ec_singv_cell_bytes /   <- obj_ec_singv_cell_bytes, obj_ec_singv_encode
 *   ecg_obj_ec_singv_encode            ref:src/object/obj_ec.h:421-434, cli_ec.c:1447-1465
 *   ecg_obj_ec_recx_encode          <- obj_ec_recx_encode + obj_ec_stripe_encode over an sgl
 *                                      ref:src/object/cli_ec.c:476-546, 593-663
 *   ecg_obj_ec_stripe_list_init     <- obj_ec_stripe_list_init / _add
 *                                      ref:src/object/cli_ec.c:2252-2381
 *   ecg_obj_ec_recov_fill_back      <- obj_ec_recov_fill_back + obj_ec_sgl_copy
 *                                      ref:src/object/cli_ec.c:2645-2812
 */
#ifndef ECG_DAOS_H
#define ECG_DAOS_H

#include <stdint.h>

#include "ecg.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Object class id = (redundancy << 24) | group count
 * (ref:src/include/daos_obj_class.h:22-23); EC redundancy OR_RS_2P1 = 32 ..
 * OR_RS_16P3 = 42 (ref:src/include/daos_obj_class.h:70-80). */
#define ECG_OC_REDUN_SHIFT	24
#define ECG_OR_RS_FIRST		32
#define ECG_OR_RS_LAST		42

/* struct obj_ec_codec (ref:src/object/obj_ec.h:33-41) + its k, p. */
struct ecg_obj_ec_codec {
	unsigned char *ec_en_matrix;	/* (k+p) x k Cauchy1 */
	unsigned char *ec_gftbls;	/* k*p*32 ISA-L-layout tables */
	int k;
	int p;
};

/* struct obj_ec_recov_codec (ref:src/object/obj_ec.h:213-224). */
struct ecg_obj_ec_recov_codec {
	unsigned char er_gftbls[ECG_MAX_K * ECG_MAX_P * 32];
	unsigned char er_de_matrix[ECG_MAX_P * ECG_MAX_K];	/* err_list order */
	uint32_t er_dec_idx[ECG_MAX_K];
	uint32_t er_err_list[ECG_MAX_P];			/* logical cells */
	uint32_t er_nerrs;
	uint32_t er_data_nerrs;
	int k;
	int p;
	int reused_encode;	/* all-parity-lost shortcut (cli_ec.c:2205-2210) */
	uint32_t er_builds;	/* times ecg_obj_ec_recov_codec_init built the rows into this
				 * codec (a repeat init with the same erasures builds nothing) */
};

/* 0, or -ECG_DER_NOMEM. Idempotent. */
int ecg_obj_ec_codec_init(void);
void ecg_obj_ec_codec_fini(void);
/* NULL when oc_id is not an EC class (or init has not run). */
struct ecg_obj_ec_codec *ecg_obj_ec_codec_get(uint32_t oc_id);
/* The k, p of an EC class id; -ECG_DER_INVAL if not EC. */
int ecg_obj_ec_class_kp(uint32_t oc_id, int *k, int *p);

/* Encode one contiguous stripe buffer[k*cell_bytes] into p_bufs[p].  As in
 * the reference, leading NULL entries of p_bufs are allocated here
 * (cell_bytes each, caller frees with free()).  0 / -ECG_DER_NOMEM /
 * -ECG_DER_INVAL (not an EC class).  Synchronous; placed like an ISA-L
 * drop-in call (ecg.h ecg_set_dropin_crossover: host cells on the CPU path
 * below the crossover or without a usable device, else the GPU; device cells
 * on their GPU).  The same holds for ecg_agg_update_parity,
 * ecg_agg_recalc_parity and ecg_obj_ec_singv_encode below, whose ctx (may be
 * NULL) only picks the GPU when the GPU is used. */
int ecg_obj_ec_encode_buf(uint32_t oc_id, uint64_t cell_bytes, unsigned char *buffer,
			  unsigned char *p_bufs[]);

/* obj_ec_recov_codec_alloc (ref:src/object/cli_ec.c:1953-1993): heap
 * allocation of a recovery codec (the struct is ~17 KiB -- too large for an
 * Argobots ULT stack).  NULL on allocation failure. */
struct ecg_obj_ec_recov_codec *ecg_obj_ec_recov_codec_alloc(void);
void ecg_obj_ec_recov_codec_free(struct ecg_obj_ec_recov_codec *recov);

/* Build the recovery codec for LOGICAL erased cells err_list[nerrs].
 * 0 / -ECG_DER_DATA_LOSS (nerrs > p) / -ECG_DER_INVAL.  As the reference's
 * obj_ec_recov_codec_init with its per-object codec (efi_recov_codec,
 * ref:src/object/cli_ec.c:2176-2185, obj_ec_err_match :2141-2150): when
 * `recov` already holds the rows of this class and the same nerrs and
 * err_list (same order), it returns 0 at once and rebuilds nothing
 * (er_builds unchanged).  `recov` must therefore come from
 * ecg_obj_ec_recov_codec_alloc (zeroed, like the reference's D_ALLOC) or be
 * zeroed by the caller before its first init. */
int ecg_obj_ec_recov_codec_init(uint32_t oc_id, const uint32_t *err_list, uint32_t nerrs,
				struct ecg_obj_ec_recov_codec *recov);

/* Regenerate the erased cells of `nstripes` host stripes laid out
 * [nstripes][k+p][cell_sz] (the recovery buffer of ref:src/object/cli_ec.c:
 * 2449-2464), in place, through device ctx's staging pipeline (NULL = the
 * calling thread's default device; in a process without a usable device, or
 * with ECG_FORCE_CPU=1, the product CPU path, stripe by stripe).
 *
 * One deliberate byte difference from the reference: when err_list names a
 * PARITY cell before a data cell (DAOS keeps failures in insertion order,
 * ref:src/object/cli_ec.c:1388-1391), the reference indexes its inverse with
 * the first er_data_nerrs entries (:2226-2231) and reads an all-zero row
 * of its zeroed (k+p) x k buffer (:1963-1984), so it writes that parity cell
 * as ZEROS.  This codec builds its rows data-first and writes the TRUE parity
 * there.  Every data cell is byte-identical to the reference's, and a
 * degraded read never returns a parity cell; only that parity cell differs
 * (tests/test_gpu_parity.py::test_recover_parity_first_order asserts the true
 * parity; oracle/ec_ref.c reproduces the reference's zeros,
 * tests/test_oracle.py::test_reference_quirk_parity_first). */
int ecg_obj_ec_recov_data(ecg_ctx_t *ctx, const struct ecg_obj_ec_recov_codec *recov,
			  uint64_t cell_sz, unsigned char *buf_stripes, uint32_t nstripes);

/* Full-stripe encode of host stripes: data [S][k][C] (user sgl order),
 * parity [p][S][C] (oer_pbufs layout, ref:src/object/cli_ec.c:75-97); ctx as
 * for ecg_obj_ec_recov_data (NULL without a device: the CPU path). */
int ecg_obj_ec_encode_stripes(ecg_ctx_t *ctx, uint32_t oc_id, uint64_t cell_bytes,
			      uint32_t nstripes, const unsigned char *data,
			      unsigned char *parity);

/* agg_update_parity + agg_diff_preprocess for one stripe
 * (ref:src/object/srv_ec_aggregate.c:1006-1105), host buffers as in the
 * reference: old/new replica cells [cell_cnt][C] (AGG_IOV_ODATA /
 * AGG_IOV_DATA), parity [p][C] updated in place, C = cell_recs * rsize.  The
 * i-th updated cell is the i-th set bit of bit_map.  ext_start/ext_nr are the
 * stripe's new-data extents in records relative to the stripe start, sorted
 * (the reference's as_dextents with holes and old epochs already skipped);
 * bytes of an updated cell outside them count as unchanged, with the
 * reference's exact rules (no extent touching the cell -> whole cell counts;
 * n_ext = 0 -> no hole processing).  old ^ new is fused on the device: no
 * AGG_IOV_DIFF buffer. */
int ecg_agg_update_parity(ecg_ctx_t *ctx, uint32_t oc_id, uint64_t cell_recs, uint64_t rsize,
			  const uint8_t *bit_map, uint32_t cell_cnt,
			  const unsigned char *old_cells, const unsigned char *new_cells,
			  const uint64_t *ext_start, const uint64_t *ext_nr, uint32_t n_ext,
			  unsigned char *parity);

/* agg_recalc_parity (ref:src/object/srv_ec_aggregate.c:1110-1138): re-encode
 * a stripe whose data cells come from two buffers -- cell j from rbuf (fetched
 * from peers) when bit j of bit_map is set, else from lbuf (local replicas),
 * each consumed in order.  parity [p][cell_bytes]. */
int ecg_agg_recalc_parity(ecg_ctx_t *ctx, uint32_t oc_id, uint64_t cell_bytes,
			  const uint8_t *bit_map, uint32_t cell_cnt, const unsigned char *rbuf,
			  const unsigned char *lbuf, unsigned char *parity);

/* obj_ec_singv_cell_bytes (ref:src/object/obj_ec.h:421-434): cell size of an
 * evenly distributed single value of iod_size bytes. 0 if not an EC class. */
uint64_t ecg_obj_ec_singv_cell_bytes(uint32_t oc_id, uint64_t iod_size);

/* Single-value encode (obj_ec_singv_encode / obj_ec_stripe_encode's singv
 * branch, ref:src/object/cli_ec.c:476-546, 1447-1465): the value is split into
 * k cells of ecg_obj_ec_singv_cell_bytes, the last one zero padded, and the p
 * parity cells are written to p_bufs (leading NULL entries allocated here, as
 * obj_ec_encode_buf; caller frees). */
int ecg_obj_ec_singv_encode(uint32_t oc_id, uint64_t iod_size, const unsigned char *value,
			    unsigned char *p_bufs[]);

/* ---- client full-stripe encode over a scatter-gather list --------------
 * obj_ec_recx_encode + obj_ec_stripe_encode (ref:src/object/cli_ec.c:476-546,
 * 593-663) for an array iod whose sgl and parity buffers are in device
 * memory.  The sgl is walked exactly as the reference does (daos_sgl_move
 * semantics, iov_buf_len): for recx i the cursor moves to byte_off, then
 * stripe_nr full stripes of k cells are consumed; a cell wholly inside one
 * iov is encoded in place, a cell spanning iovs is gathered on the device
 * first.  Parity of the n-th stripe overall goes to pbufs[m] + n*cell_bytes
 * (oer_pbufs).  One launch for all stripes.  -DER_REC2BIG when the sgl runs
 * out (as the reference), -DER_INVAL for recxs out of order. */
typedef struct ecg_iov {	/* d_iov_t (ref:src/include/gurt/types.h:93-100), device buffer */
	void *iov_buf;
	uint64_t iov_buf_len;
	uint64_t iov_len;
} ecg_iov_t;

typedef struct ecg_ec_recx {	/* struct obj_ec_recx: oer_byte_off, oer_stripe_nr */
	uint64_t byte_off;
	uint32_t stripe_nr;
	uint32_t pad;
} ecg_ec_recx_t;

int ecg_obj_ec_recx_encode(ecg_ctx_t *ctx, uint32_t oc_id, uint64_t cell_bytes,
			   const ecg_iov_t *iovs, uint32_t iov_nr, const ecg_ec_recx_t *recxs,
			   uint32_t recx_nr, unsigned char *const *pbufs, void *stream);

/* ---- degraded read: stripe list and fill-back ---------------------------
 * After a degraded fetch the client reads whole stripes of the records it
 * could not get (the "stripe list", obj_ec_stripe_list_init/_add,
 * ref:src/object/cli_ec.c:2252-2381) into one [stripes][k+p][C] buffer,
 * regenerates the lost cells (ecg_recover / obj_ec_recov_stripe), then
 * copies the records it was missing back into the user's sgl
 * (obj_ec_recov_fill_back + obj_ec_sgl_copy, :2645-2812).  Types mirror
 * daos_recx_t, struct daos_recx_ep (ref:src/include/daos/object.h:714-719)
 * and d_sg_list_t (ref:src/include/gurt/types.h:127-132). */
typedef struct ecg_recx {	/* daos_recx_t */
	uint64_t rx_idx;
	uint64_t rx_nr;
} ecg_recx_t;

#define ECG_DRT_SHADOW		2	/* DRT_SHADOW: a to-be-recovered recx */

typedef struct ecg_recx_ep {	/* struct daos_recx_ep */
	ecg_recx_t re_recx;
	uint64_t re_ep;
	uint32_t re_rec_size;
	uint8_t re_type;
} ecg_recx_ep_t;

typedef struct ecg_sgl {	/* d_sg_list_t, iov buffers in device memory */
	uint32_t sg_nr;
	uint32_t sg_nr_out;
	ecg_iov_t *sg_iovs;
} ecg_sgl_t;

/* obj_ec_stripe_list_init for one array iod: every DRT_SHADOW recx rounded
 * out to whole stripes of stripe_rec_nr records, merged into stripes[] in
 * the reference's order (overlapping entries merge whatever their epochs,
 * keeping the higher; adjacent ones only with equal epochs).  *stripe_nr =
 * entries written.  cap >= recx_nr always suffices; -ECG_DER_INVAL if cap
 * is exceeded or stripe_rec_nr == 0. */
int ecg_obj_ec_stripe_list_init(uint64_t stripe_rec_nr, const ecg_recx_ep_t *recx, uint32_t recx_nr,
				ecg_recx_ep_t *stripes, uint32_t cap, uint32_t *stripe_nr);

/* obj_ec_recov_fill_back for one iod: copy the recovered records of each
 * recov recx from the stripe buffer (device, stripe n of the stripe list at
 * stripe_buf + n * stripe_total_sz, its records from byte 0 in index order)
 * to their place in the user sgl (offset = records of the iod recxs before
 * it times iod_size), with the reference's sgl bookkeeping: iov_len grows
 * over copied bytes, sg_nr_out is set by the last copy.  singv != 0: single
 * value, iod_size bytes from stripe_buf[0] (recxs ignored).  All copies go
 * to `stream` as one launch; the host structs are updated on return.
 * -ECG_DER_INVAL where the reference asserts (a recov recx starting before
 * the iod recx it overlaps, stripe recxs not whole stripes, a recov recx not
 * covered by the stripe list).  Iovs of zero capacity are skipped (the
 * reference asserts). */
int ecg_obj_ec_recov_fill_back(ecg_ctx_t *ctx, uint64_t iod_size, int singv,
			       const ecg_recx_t *iod_recxs, uint32_t iod_nr, ecg_sgl_t *sgl,
			       const ecg_recx_ep_t *recov, uint32_t recov_nr,
			       const ecg_recx_ep_t *stripes, uint32_t stripe_nr,
			       const void *stripe_buf, uint64_t stripe_total_sz, uint64_t stripe_rec_nr,
			       void *stream);

/* obj_ec_recov_data (ref:src/object/cli_ec.c:2814-2885) on device buffers:
 * for every iod, regenerate the erased cells (recov->er_err_list) of all
 * stripes of its stripe list in one launch -- the cell size is e_len *
 * iod_size, or obj_ec_singv_cell_bytes for a single value (one stripe,
 * skipped when the value lives on one target, obj_ec_singv_one_tgt) -- then
 * fill the recovered records back into its sgl (ecg_obj_ec_recov_fill_back).
 * Array iods with an empty recov or stripe list are skipped, as in the
 * reference.  Asynchronous on `stream`; sgl bookkeeping done on return. */
typedef struct ecg_recov_iod {
	uint64_t iod_size;
	uint32_t singv;			/* DAOS_IOD_SINGLE */
	uint32_t iod_nr;		/* iod recxs */
	const ecg_recx_t *iod_recxs;
	ecg_sgl_t *sgl;			/* the user's sgl (device buffers) */
	const ecg_recx_ep_t *recov;	/* efi_recx_lists[i] */
	uint32_t recov_nr;
	uint32_t stripe_nr;
	const ecg_recx_ep_t *stripes;	/* efi_stripe_lists[i] */
	void *stripe_buf;		/* efi_stripe_sgls[i]: [n][k+p][cell] (device) */
} ecg_recov_iod_t;

int ecg_obj_ec_recov_data_dev(ecg_ctx_t *ctx, uint32_t oc_id, uint64_t e_len,
			      const struct ecg_obj_ec_recov_codec *recov, ecg_recov_iod_t *iods, uint32_t iod_nr,
			      void *stream);

/* ---- rebuild of a parity shard ------------------------------------------
 * migrate_update_parity (ref:src/object/srv_obj_migrate.c:1096-1181) over a
 * fetched range of records [offset, offset + size) of iod_size bytes, held in
 * `buffer` (device) in record order.  The range is cut exactly as the
 * reference cuts it (at stripe boundaries when `encode`, else at cell
 * boundaries); every full stripe becomes a parity piece -- this shard's
 * parity cell, VOS index obj_ec_idx_daos2vos(offset) | ECG_EC_PARITY_BIT,
 * e_len records -- and every other piece is written as replicated records.
 * All parity cells come from one product launch with a single output row
 * into parity_out ([nparity][e_len * iod_size], device); with csum_type (an
 * ECG_HASH_* of ecg_csum.h, 0 = none) every piece's chunk checksums
 * (daos_csummer_calc_iods, :1156) go to csums_out (device) at the piece's
 * csum_off.  `shard` is the logical cell index of the shard being rebuilt
 * (k .. k+p-1, obj_ec_shard_off_by_layout_ver in the caller).  The caller
 * then hands each piece to vos_obj_update as the reference does.
 * -ECG_DER_REC2BIG when pieces_cap is too small (ecg_migrate_plan_size gives
 * the counts), -ECG_DER_INVAL for a shard that is not a parity shard. */
typedef struct ecg_migrate_piece {
	ecg_recx_t recx;	/* the recx for vos_obj_update */
	uint64_t buf_off;	/* bytes into parity_out (parity pieces) or buffer */
	uint64_t buf_len;
	uint64_t csum_off;	/* bytes into csums_out: nr_csums checksums */
	uint32_t nr_csums;
	uint32_t parity;	/* 1: this shard's parity cell of a full stripe */
} ecg_migrate_piece_t;

/* Sizing for ecg_migrate_update_parity: pieces, parity cells, checksum bytes. */
int ecg_migrate_plan_size(uint32_t oc_id, uint64_t e_len, uint64_t iod_size, uint64_t offset, uint64_t size,
			  int encode, int csum_type, uint64_t chunksize, uint32_t *npieces, uint32_t *nparity,
			  uint64_t *csum_bytes);

int ecg_migrate_update_parity(ecg_ctx_t *ctx, uint32_t oc_id, uint64_t e_len, uint64_t iod_size,
			      uint32_t shard, const void *buffer, uint64_t offset, uint64_t size, int encode,
			      int csum_type, uint64_t chunksize, void *parity_out, void *csums_out,
			      ecg_migrate_piece_t *pieces, uint32_t pieces_cap, uint32_t *npieces, void *stream);

/* ---- stripe / index math (ref:src/object/obj_ec.h:271-350) -------------
 * e_len = records per cell (oca->u.ec.e_len), stripe_rec_nr = k * e_len.
 * Parity extents carry ECG_EC_PARITY_BIT in their VOS index
 * (DAOS_EC_PARITY_BIT, ref:src/include/daos/object.h:19). */
#define ECG_EC_PARITY_BIT	(1ULL << 63)

uint64_t ecg_obj_ec_stripe_rec_nr(uint32_t k, uint64_t e_len);	/* obj_ec_stripe_rec_nr */
uint64_t ecg_obj_ec_cell_bytes(uint64_t e_len, uint64_t iod_size);	/* obj_ec_cell_bytes */
/* data target (0..k-1) holding daos record idx: obj_ec_tgt_of_recx_idx */
uint32_t ecg_obj_ec_tgt_of_recx_idx(uint64_t idx, uint64_t stripe_rec_nr, uint64_t e_len);
/* daos record idx -> VOS idx on its data target: obj_ec_idx_daos2vos */
uint64_t ecg_obj_ec_idx_daos2vos(uint64_t idx, uint64_t stripe_rec_nr, uint64_t e_len);
/* VOS idx on data target tgt_idx -> daos record idx: obj_ec_idx_vos2daos */
uint64_t ecg_obj_ec_idx_vos2daos(uint64_t vos_idx, uint64_t stripe_rec_nr, uint64_t e_len,
				 uint32_t tgt_idx);
/* parity VOS offset -> daos idx of the stripe start: obj_ec_idx_parity2daos */
uint64_t ecg_obj_ec_idx_parity2daos(uint64_t vos_off, uint64_t e_len, uint64_t stripe_rec_nr);
/* physical target -> logical cell index given the group's start target:
 * obj_ec_shard_off_by_start */
uint32_t ecg_obj_ec_shard_off_by_start(uint32_t tgt_idx, uint32_t tgt_nr, uint32_t start_tgt);

#ifdef __cplusplus
}
#endif
#endif
