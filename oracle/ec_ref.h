/*
 * ec_ref.h -- CPU ORACLE for the DAOS EC stripe-cell codec.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (daos_amd/, include/) may
 * include, link or call this.  Only tests/, __graft_entry__.smoke() and the
 * bench.py `cpu_baseline` leg use it, and only as the checker / CPU baseline.
 *
 * What it restates:
 *   - ISA-L v2.31.1 erasure_code base semantics (the library DAOS links for
 *     this path, pinned at ref:utils/build.config:8; NOT vendored in
 *     /root/reference and absent from this image, so it is restated from its
 *     published algorithm -- see SURVEY.md Appendix A):
 *       gf_mul / gf_inv (GF(2^8), poly 0x11d, generator 2),
 *       gf_gen_cauchy1_matrix, ec_init_tables (32-B nibble-table layout),
 *       ec_encode_data_base, ec_encode_data_update_base, gf_invert_matrix,
 *       xor_gen.
 *   - DAOS's own logic around those calls:
 *       codec matrix choice            ref:src/object/obj_class.c:602-617
 *       recovery (decode) codec build  ref:src/object/cli_ec.c:2152-2250
 *       per-stripe recovery pointers   ref:src/object/cli_ec.c:2626-2643
 *       obj_ec_encode_buf              ref:src/object/cli_ec.c:548-573
 *
 * PARITY PINNING: the reference holds no golden parity bytes for this path
 * (its only byte-level check, ref:src/tests/suite/daos_aggregate_ec.c:394-440,
 * computes expected parity with ISA-L at run time on a live cluster).  This
 * oracle is therefore "parity unpinned" by any reference fixture; it is pinned
 * instead by (a) the field/matrix definitions, (b) an independent numpy
 * log/exp restatement (oracle/gf_np.py) that must agree byte for byte, and
 * (c) the known-answer values of SURVEY.md App. A.5 (tests/golden/kat.json).
 *
 * All symbols are prefixed ref_ so the oracle can never be confused with (or
 * interpose on) the product's ISA-L-compatible exports.
 */
#ifndef ECG_ORACLE_EC_REF_H
#define ECG_ORACLE_EC_REF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define REF_DER_INVAL     1003
#define REF_DER_NOMEM     1009
#define REF_DER_DATA_LOSS 2026

/* ---- GF(2^8) field (ISA-L ec_base.c gf_mul / gf_inv) ---- */
unsigned char ref_gf_mul(unsigned char a, unsigned char b);
unsigned char ref_gf_inv(unsigned char a);

/* ---- matrices ---- */
void ref_gf_gen_cauchy1_matrix(unsigned char *a, int m, int k);
int  ref_gf_invert_matrix(unsigned char *in, unsigned char *out, int n);

/* ---- ISA-L data-plane semantics (base/scalar path) ---- */
void ref_ec_init_tables(int k, int rows, const unsigned char *a, unsigned char *gftbls);
void ref_ec_encode_data(int len, int k, int rows, const unsigned char *gftbls,
                        unsigned char **data, unsigned char **coding);
void ref_ec_encode_data_update(int len, int k, int rows, int vec_i,
                               const unsigned char *gftbls, const unsigned char *data,
                               unsigned char **coding);
int  ref_xor_gen(int vects, int len, void **array);

/* ---- DAOS recovery codec (ref:src/object/cli_ec.c:2152-2250) ----
 * err_list: LOGICAL cell indices (already mapped through obj_ec_shard_off),
 * in the caller's order.  Outputs:
 *   de_matrix[nerrs*k], dec_idx[k], out_err_list[nerrs] (the order rows of
 *   de_matrix / gftbls correspond to), gftbls[k*p*32].
 * Returns 0, or -REF_DER_DATA_LOSS when nerrs > p.
 * *reused_encode is set when the "all parity lost" shortcut
 * (ref:src/object/cli_ec.c:2205-2210) applied: gftbls are then the encode
 * tables and de_matrix is left untouched (as in the reference). */
int ref_obj_ec_recov_codec_init(int k, int p, const unsigned char *en_matrix,
                                const uint32_t *err_list, int nerrs,
                                unsigned char *de_matrix, uint32_t *dec_idx,
                                uint32_t *out_err_list, unsigned char *gftbls,
                                int *reused_encode);

/* obj_ec_recov_stripe (ref:src/object/cli_ec.c:2626-2643): in place on one
 * [(k+p) x cell_sz] logical-order stripe buffer. */
void ref_obj_ec_recov_stripe(int k, int nerrs, const unsigned char *gftbls,
                             const uint32_t *dec_idx, const uint32_t *err_list,
                             unsigned char *stripe, uint64_t cell_sz);

/* obj_ec_encode_buf (ref:src/object/cli_ec.c:548-573) with caller buffers. */
void ref_obj_ec_encode_buf(int k, int p, const unsigned char *en_matrix,
                           uint64_t cell_bytes, const unsigned char *buffer,
                           unsigned char **p_bufs);

/* ---- aggregation / single-value helpers ---- */
/* agg_diff_preprocess (ref:src/object/srv_ec_aggregate.c:1006-1058): zero the
 * parts of `diff` (one cell, len records of rsize bytes, cell index cell_idx)
 * not covered by the new-data extents.  Extents are (start, nr) in records
 * relative to the stripe start, sorted, as the reference's as_dextents list
 * (holes / old-epoch extents already filtered out by the caller). */
void ref_agg_diff_preprocess(unsigned char *diff, uint64_t len, uint64_t rsize,
                             unsigned int cell_idx, const uint64_t *ext_start,
                             const uint64_t *ext_nr, unsigned int n_ext);
/* agg_update_parity (ref:src/object/srv_ec_aggregate.c:1062-1105): for the
 * i-th updated cell (cell index = i-th set bit of bit_map): diff = old ^ new,
 * preprocess, ec_encode_data_update into parity[p][cell_bytes]. */
int ref_agg_update_parity(int k, int p, uint64_t len, uint64_t rsize, const uint8_t *bit_map,
                          unsigned int cell_cnt, const unsigned char *obuf,
                          const unsigned char *nbuf, const uint64_t *ext_start,
                          const uint64_t *ext_nr, unsigned int n_ext, unsigned char *parity);
/* obj_ec_singv_cell_bytes (ref:src/object/obj_ec.h:421-434). */
uint64_t ref_singv_cell_bytes(uint64_t rec_gsize, int k);
/* Single-value encode (ref:src/object/cli_ec.c:476-546 singv branch,
 * 1447-1465): value split into k cells of cell_bytes, last one zero padded. */
void ref_singv_encode(int k, int p, uint64_t iod_size, const unsigned char *value,
                      unsigned char **p_bufs);

/* ---- batch helpers used by tests / cpu_baseline (layouts of SURVEY §8a) ---- */
/* Encode S stripes: data [S][k][C] -> parity [p][S][C] (obj_ec_pbufs_init
 * layout, ref:src/object/cli_ec.c:75-97, 638-640). nthreads<=1: serial. */
void ref_encode_batch(int k, int p, uint64_t C, uint32_t S,
                      const unsigned char *data, unsigned char *parity, int nthreads);
/* In-place recovery over [S][k+p][C] with a prepared recovery codec. */
void ref_recov_batch(int k, int nerrs, const unsigned char *gftbls,
                     const uint32_t *dec_idx, const uint32_t *err_list,
                     uint64_t C, uint64_t stripe_stride, uint32_t S,
                     unsigned char *stripes, int nthreads);

/* ---- SIMD CPU baseline ("ISA-L-equivalent restatement", ec_simd.c) ----
 * Same contract as ref_ec_encode_data; uses AVX2 vpshufb nibble tables (the
 * algorithm of ISA-L gf_vect_dot_prod_avx2) or GFNI when available.
 * Returns the variant used: 0 scalar, 1 avx2, 2 gfni-avx512. */
int  ref_simd_variant(void);
void ref_simd_encode_data(int len, int k, int rows, const unsigned char *gftbls,
                          unsigned char **data, unsigned char **coding);
void ref_simd_encode_batch(int k, int p, uint64_t C, uint32_t S,
                           const unsigned char *data, unsigned char *parity,
                           int nthreads);
void ref_simd_recov_batch(int k, int nerrs, const unsigned char *gftbls,
                          const uint32_t *dec_idx, const uint32_t *err_list,
                          uint64_t C, uint64_t stripe_stride, uint32_t S,
                          unsigned char *stripes, int nthreads);

/* ---- chunked checksums (oracle/csum_ref.c) ---- */
#define REF_HASH_CRC16   1
#define REF_HASH_CRC32   2
#define REF_HASH_CRC64   3
#define REF_HASH_ADLER32 7
uint16_t ref_crc16_t10dif(uint16_t seed, const unsigned char *buf, uint64_t len);
uint32_t ref_crc32_iscsi(const unsigned char *buf, uint64_t len, uint32_t seed);
uint64_t ref_crc64_ecma_refl(uint64_t seed, const unsigned char *buf, uint64_t len);
uint32_t ref_adler32(uint32_t seed, const unsigned char *buf, uint64_t len);
int ref_csum_len(int type);
uint64_t ref_csum_record_chunksize(uint64_t chunksize, uint64_t rec_size);
uint32_t ref_csum_chunk_count(uint64_t rec_chunksize, uint64_t rec_size, uint64_t rx_idx,
			      uint64_t rx_nr);
uint32_t ref_csum_extent(int type, uint64_t chunksize, uint64_t rec_size, uint64_t rx_idx,
			 uint64_t rx_nr, const unsigned char *buf, unsigned char *out);
void ref_csum_extents(int type, uint64_t chunksize, uint64_t rec_size, uint64_t rx_idx,
		      uint64_t rx_nr, const unsigned char *buf, int64_t ext_stride, uint32_t n_ext,
		      unsigned char *out, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
