/*
 * ecg_kabi.h -- the private ABI between the C host layer (daos_amd/csrc/host)
 * and the HIP kernels (daos_amd/csrc/kernels).  Plain C, no HIP types.
 *
 * One launch = one batched GF(2^8) "matrix x cells" product over S stripes:
 *
 *     dst[s][r][i] (^)= XOR_{j<k} coef[r][j] * src[s][j][i]      i in [0, C)
 *
 * which is ISA-L ec_encode_data (ref:src/object/cli_ec.c:540) when coef are
 * the Cauchy parity rows, DAOS recovery (ref:src/object/cli_ec.c:2641) when
 * coef are the decode rows, and ec_encode_data_update / agg_update_parity
 * (ref:src/object/srv_ec_aggregate.c:1089-1101) with `accumulate` and
 * `diff` set (src = old ^ new).
 *
 * Cell j of stripe s lives at  src + s*src_stripe_stride + src_cell_off[j];
 * that covers the DAOS layouts: client data [S][k][C], parity [p][S][C]
 * (ref:src/object/cli_ec.c:75-97,638-640), recovery [S][k+p][C]
 * (ref:src/object/cli_ec.c:2449-2464, 2626-2643), aggregation [k][C]/[p][C]
 * (ref:src/object/srv_ec_aggregate.c:686-691).
 *
 * GF multiply tables ("perm tables"): a byte x splits into bit groups
 * x = (x & 0x07) ^ (x & 0x38) ^ (x & 0xC0) and, GF multiplication being
 * linear over GF(2),  c*x = T0[x & 7] ^ T1[(x >> 3) & 7] ^ T2[x >> 6]  with
 * T0[i] = c*i, T1[i] = c*(i<<3), T2[i] = c*(i<<6).  Each table has <= 8 byte
 * entries, i.e. exactly what one v_perm_b32 can index.  Packed little-endian:
 * t0lo = T0[0..3], t0hi = T0[4..7], t1lo/t1hi likewise, t2 = T2[0..3].
 */
#ifndef ECG_KABI_H
#define ECG_KABI_H

#include <stdint.h>

#define ECG_KMAX_K 16	/* data cells per launch; host splits larger k */
#define ECG_KMAX_R 8	/* output rows per launch */

typedef struct ecg_ptbl {
	uint32_t t0lo, t0hi, t1lo, t1hi, t2;
} ecg_ptbl_t;

typedef struct ecg_mm_params {
	const uint8_t *src;		/* cell bases (stripe 0) */
	const uint8_t *src2;		/* diff mode: second source, same layout */
	uint8_t *dst;
	int64_t src_stripe_stride;
	int64_t src2_stripe_stride;
	int64_t dst_stripe_stride;
	int64_t src_cell_off[ECG_KMAX_K];
	int64_t src2_cell_off[ECG_KMAX_K];
	int64_t dst_cell_off[ECG_KMAX_R];
	uint64_t cell_bytes;
	uint32_t nstripes;
	uint32_t k;
	uint32_t rows;
	uint32_t accumulate;		/* dst ^= product instead of dst = product */
	uint32_t diff;			/* source cell j = src[j] ^ src2[j] */
	uint32_t order;			/* block -> (stripe, column) map, 0 = 2D grid (ecg_kernels.hip) */
	ecg_ptbl_t tbl[ECG_KMAX_R][ECG_KMAX_K];
} ecg_mm_params_t;

/* launch tuning (host fills; 0 = kernel default) */
typedef struct ecg_launch_cfg {
	uint32_t grid_x;	/* chunks per stripe handled in parallel */
	uint32_t grid_y;	/* stripes handled in parallel */
	uint32_t variant;	/* 0 auto, 1 force generic, 2 force byte kernel, 3 dword
				 * lanes at any alignment (hardware unaligned access) */
	uint32_t order;		/* 0 = 2D grid x columns / y stripes; 1-3 1D orders (ecg_kernels.hip) */
	uint32_t wg_per_cu;	/* product kernel blocks per CU: 0 = per-shape default, 1..16 = cap,
				 * ECG_WG_UNCAPPED = none (ecg_kernels.hip mm_wg_cap) */
	uint32_t no_unaligned;	/* the device did not serve misaligned dword accesses at context
				 * creation (ecg_k_unaligned_check): operands that need them take
				 * the byte kernels */
} ecg_launch_cfg_t;
#define ECG_WG_UNCAPPED 255u


/*
 * Chunked checksums (DAOS csummer semantics, ref:src/common/checksum.c:467-497):
 * n_ext extents at src + e*ext_stride, each ext_bytes long and cut into
 * nchunks chunks: chunk 0 = [0, first_bytes), chunk c >= 1 =
 * [first_bytes + (c-1)*chunk_bytes, ... + chunk_bytes) clipped to ext_bytes.
 * out[e*nchunks + c] = hash of that chunk (2, 4 or 8 bytes, little-endian).
 * CRC tables (host-built, ecg_csum.c) at tbl: W-bit words T
 *   sl[NB][256]  slice tables: sl[j][v] = CRC state after byte v then j zero bytes
 *   sh[NB][256]  "shift by ECG_CSUM_STRIDE zero bytes" as a byte-wise linear map
 *   k[64]        x^(8*16*(63-lane)) mod P, for the final per-lane shift
 *   sh4k[NB][256] shift by ECG_MMCS_STRIDE zero bytes (fused kernels)
 *   k256[256]    x^(8*16*(255-thread)) mod P (host builds the fused kh rows from it)
 *   p2[48]       x^(8*2^j) mod P (shift by any byte count: product over its bits)
 *   sh256[NB][256] shift by ECG_CSUM_GSTRIDE zero bytes (lane-group kernel)
 * with NB = W/8, T = uint32_t (W <= 32) or uint64_t (W = 64).
 */
#define ECG_CSUM_STRIDE 1024	/* bytes a wave consumes per step (64 lanes x 16 B) */
#define ECG_KID_CSUM 1000	/* kernel ids of the checksum kernels start here */

#define ECG_MMCS_STRIDE 4096	/* fused kernels: 256 threads x 16 B per step */
#define ECG_CSUM_NP2 48
/*
 * 5-bit tables (conflict-free LDS lookups: a 32-entry table of 4-byte words
 * covers the 32 banks ds_read_b32 sees, one of 8-byte words the 64 banks of
 * ds_read_b64, so lanes never collide -- the byte tables above run ~3x
 * conflicted on random data).  A 16-byte piece is 4 dwords x 7 fields (bits
 * 5i..5i+4, the 7th field bits 30-31):
 *   p5[28][32]   p5[7j + i][v] = raw CRC of the piece whose dword j is v << 5i
 *   a5*[NA][32]  a register shifted by 1 KiB / 256 B / 4 KiB of zero bytes,
 *                fields of each 32-bit half of the register (NA = 7 per half;
 *                4 for crc16: bits 0-19)
 */
#define ECG_CSUM_NF5 28
#define ECG_CSUM_NA5(NB) ((NB) == 2 ? 4 : 7 * (NB) / 4)
#define ECG_CSUM_OFF_P5(NB) (4 * (NB) * 256 + 64 + 256 + ECG_CSUM_NP2)
#define ECG_CSUM_OFF_A5_1K(NB) (ECG_CSUM_OFF_P5(NB) + ECG_CSUM_NF5 * 32)
#define ECG_CSUM_OFF_A5_256(NB) (ECG_CSUM_OFF_A5_1K(NB) + ECG_CSUM_NA5(NB) * 32)
#define ECG_CSUM_OFF_A5_4K(NB) (ECG_CSUM_OFF_A5_256(NB) + ECG_CSUM_NA5(NB) * 32)
/* s16[16][256]: register after byte v and then j zero bytes, j < 16 (the
 * raw CRC of a 16-byte piece is 16 independent lookups, no serial fold) */
#define ECG_CSUM_OFF_S16(NB) (ECG_CSUM_OFF_A5_4K(NB) + ECG_CSUM_NA5(NB) * 32)
/* positional p5 tables: p5x*[u-1] = p5 followed by u strides (1 KiB / 256 B)
 * of zero bytes, u = 1 .. ECG_CSUM_P5U-1 (the standalone CRC kernels shift the
 * register once per ECG_CSUM_P5U pieces: a5 of 4 KiB / 1 KiB) */
#define ECG_CSUM_P5U 4
#define ECG_CSUM_OFF_P5X_1K(NB) (ECG_CSUM_OFF_S16(NB) + 16 * 256)
#define ECG_CSUM_OFF_P5X_256(NB) (ECG_CSUM_OFF_P5X_1K(NB) + (ECG_CSUM_P5U - 1) * ECG_CSUM_NF5 * 32)
/* the fused workgroup kernel's 4 KiB columns: positional tables of 1 ..
 * ECG_MMCS_P5U-1 columns and the a5 of ECG_MMCS_P5U columns (an item of at
 * most ECG_MMCS_P5U columns needs no register shift at all, so its columns can
 * be walked in any order) */
#define ECG_MMCS_P5U 8
#define ECG_CSUM_OFF_P5X_4K(NB) (ECG_CSUM_OFF_P5X_256(NB) + (ECG_CSUM_P5U - 1) * ECG_CSUM_NF5 * 32)
#define ECG_CSUM_OFF_A5_32K(NB) (ECG_CSUM_OFF_P5X_4K(NB) + (ECG_MMCS_P5U - 1) * ECG_CSUM_NF5 * 32)
/* reflected CRCs (crc32, crc64): the fused workgroup kernel multiplies a
 * lane's value by x^(8*16*(63-lane)) nibble by nibble --
 *   nibl[n][lane] = (n at the register's 4 lowest powers) * x^(8*16*(63-lane))
 *   r4[m]         = m (register bits 0-3) * x^4, the reduction of a 4-bit shift
 * (n-major, so lane l's entries sit in bank l: conflict-free) */
#define ECG_CSUM_OFF_NIBL(NB) (ECG_CSUM_OFF_A5_32K(NB) + ECG_CSUM_NA5(NB) * 32)
#define ECG_CSUM_OFF_R4(NB) (ECG_CSUM_OFF_NIBL(NB) + 16 * 64)
/* nibble tables (4-bit fields, addressed by one SDWA byte select each;
 * ecg_crc_dev.h horner4u): a 16-byte piece is 32 nibbles (nibble t = bits
 * 4t..4t+3 of the piece, little-endian), the register W/4 nibbles.
 *   q4*[u][32][16]  q4[u][t][v] = raw CRC of the piece whose nibble t is v,
 *                   followed by u strides of zero bytes (u = 0 .. U-1)
 *   a4*[16][16]     a4[t][v] = register nibble t = v shifted by the U-stride
 *                   (rows >= W/4 unused)
 * 1 KiB stride (wave kernels, U = ECG_CSUM_P5U; a4 of 4 KiB), 256 B stride
 * (lane-group kernel, U = ECG_CSUM_P5U; a4 of 1 KiB), 4 KiB stride (fused
 * workgroup kernel, U = ECG_MMCS_P5U; a4 of 32 KiB). */
#define ECG_CSUM_NQ4 (32 * 16)
#define ECG_CSUM_OFF_Q4_1K(NB) (ECG_CSUM_OFF_R4(NB) + 16)
#define ECG_CSUM_OFF_A4_4K(NB) (ECG_CSUM_OFF_Q4_1K(NB) + ECG_CSUM_P5U * ECG_CSUM_NQ4)
#define ECG_CSUM_OFF_Q4_256(NB) (ECG_CSUM_OFF_A4_4K(NB) + 256)
#define ECG_CSUM_OFF_A4_1K(NB) (ECG_CSUM_OFF_Q4_256(NB) + ECG_CSUM_P5U * ECG_CSUM_NQ4)
#define ECG_CSUM_OFF_Q4_4K(NB) (ECG_CSUM_OFF_A4_1K(NB) + 256)
#define ECG_CSUM_OFF_A4_32K(NB) (ECG_CSUM_OFF_Q4_4K(NB) + ECG_MMCS_P5U * ECG_CSUM_NQ4)
#define ECG_CSUM_TBL_ENTRIES(NB) (ECG_CSUM_OFF_A4_32K(NB) + 256)
#define ECG_CSUM_OFF_P2(NB) (3 * (NB) * 256 + 64 + 256)
#define ECG_CSUM_OFF_SH256(NB) (3 * (NB) * 256 + 64 + 256 + ECG_CSUM_NP2)
#define ECG_CSUM_GLANES 16	/* lanes per chunk in the lane-group CRC kernel */
#define ECG_CSUM_GSTRIDE (16 * ECG_CSUM_GLANES)	/* bytes a lane group consumes per step */
#define ECG_CSUM_OFF_SH(NB) ((NB) * 256)
#define ECG_CSUM_OFF_K64(NB) (2 * (NB) * 256)
#define ECG_CSUM_OFF_SH4K(NB) (2 * (NB) * 256 + 64)
#define ECG_CSUM_OFF_K256(NB) (3 * (NB) * 256 + 64)

typedef struct ecg_csum_params {
	const uint8_t *src;
	uint8_t *out;
	const void *tbl;
	int64_t ext_stride;
	uint64_t ext_bytes;
	uint64_t first_bytes;
	uint64_t chunk_bytes;
	uint64_t init;			/* CRC register before the first byte */
	uint64_t xorout;		/* XORed into the final register */
	uint64_t poly;			/* reflected (or MSB-first for crc16) polynomial */
	uint32_t n_ext;
	uint32_t nchunks;
	uint32_t type;			/* DAOS hash type: 1 crc16, 2 crc32, 3 crc64, 7 adler32 */
	uint32_t variant;		/* CRC: 0 auto, 1 wave per chunk, 2 workgroup per chunk,
					 * 3 a 16-lane group per chunk */
	uint32_t pad1, pad2;
	/* workgroup-per-chunk CRC: a chunk of m 1 KiB steps is cut into
	 * ECG_CSUM_SPLIT_NW slices; split_sh[c][w] = x^(8 * bytes after slice w)
	 * mod P for the chunk lengths' step counts split_m[c] (first, middle and
	 * last chunk of an extent), filled by the host */
	uint64_t split_m[3];
	uint64_t split_sh[3][8];
} ecg_csum_params_t;

#define ECG_CSUM_SPLIT_NW 8
/* 1 KiB steps of a wave over len bytes (lanes take 16-byte pieces; a zero
 * prefix pads to a whole number of ECG_CSUM_P5U-piece Horner steps), and the
 * steps of each of the split kernel's ECG_CSUM_SPLIT_NW slices */
#define ECG_CSUM_STEPS(len) \
	((((len) / 16 + 63) / 64 + ECG_CSUM_P5U - 1) / ECG_CSUM_P5U * ECG_CSUM_P5U)
#define ECG_CSUM_SPLIT_MS(m) \
	((((m) + ECG_CSUM_SPLIT_NW - 1) / ECG_CSUM_SPLIT_NW + ECG_CSUM_P5U - 1) / ECG_CSUM_P5U * ECG_CSUM_P5U)

/*
 * Fused product + checksum: a launch of the GF product (ecg_mm_params_t)
 * that also checksums every output cell it writes, chunk by chunk, while the
 * bytes are still in registers.  Each output cell starts on a chunk boundary;
 * chunk_bytes is a multiple of ECG_MMCS_STRIDE; cell_bytes a multiple of 16.
 * out[(row_slot[r] * nstripes + s) * nch + c] = checksum of chunk c of output
 * row r of stripe s (zeroed by the host: workgroups XOR their partials in).
 *
 * Work items: chunk c (m 4 KiB columns; m_last for the last chunk of a cell)
 * is cut into sub-chunks of ncols columns, item = (c, h) with h < nh (nh_last
 * for the last chunk), numbered c * nh + h; nitems = (nch - 1) * nh + nh_last.
 * A workgroup Horner-accumulates its sub-chunk's columns per thread and then
 * moves thread t's value to the end of the chunk: a factor x^(8 * (16 * (255 -
 * t) + 4096 * (columns after the sub-chunk))) mod P, times x^(-8Z) in the last
 * chunk's rows, Z being the zero bytes that pad the cell to whole columns.
 * crc16: kh[(row0 + h) * 256 + t] holds that factor (row0 = 0, or nh for the
 * last chunk).  Reflected CRCs: the lane part x^(8*16*(63-lane)) comes from the
 * nibl tables (staged in LDS), each wave XOR-reduces, and the rest f =
 * x^(8 * (1024 * (3 - wave) + 4096 * (columns after))) (* x^(-8Z)) is applied
 * once per wave, bit-parallel: kh[((row0 + h) * 4 + wave) * 64 + b] = e_b * f
 * (e_b = the register with only bit b set, zero for b >= W).  CRC is linear,
 * so the values XOR to the chunk's CRC.
 */
typedef struct ecg_mmcs_params {
	const void *tbl;
	uint8_t *out;
	const void *kh;			/* (nh + nh_last) x 256 (crc16) or x 4 x 64 (reflected:
					 * per-wave bit-products, ecg_csum.c fused_kh), T as tbl */
	uint64_t chunk_bytes;
	uint64_t init, xorout, poly;
	uint32_t nch;
	uint32_t type;
	uint32_t m, m_last;		/* 4 KiB columns per chunk / in the last chunk */
	uint32_t ncols;			/* columns per item */
	uint32_t nh, nh_last;		/* items per chunk / in the last chunk */
	uint32_t nitems;
	uint32_t pad3;
	uint32_t row_slot[ECG_KMAX_R];
} ecg_mmcs_params_t;

/*
 * Batched byte-range copies (kernels/ecg_copy_kernels.hip): segment s copies
 * len bytes from src to dst (device addresses, any alignment, no overlap)
 * and owns the launch's 16 KiB destination tiles [tile0, tile0 +
 * ecg_k_copy_tiles(dst, len)); segments are listed in tile0 order from 0.
 */
typedef struct ecg_copy_seg {
	uint64_t dst;
	uint64_t src;
	uint64_t len;
	uint64_t tile0;
} ecg_copy_seg_t;

#define ECG_KID_COPY_SEGS 900

#ifdef __cplusplus
extern "C" {
#endif
/* Whether the device serves misaligned dword loads and stores (the unaligned
 * access mode the ROCm driver enables on gfx9+), which the product kernels
 * use for destinations off a dword boundary and for partial columns of
 * unaligned sources: 4 lanes copy dwords from src+1+4i to dst+3+4i of small
 * scratch buffers and the bytes are compared.  *ok = 1 when they arrived
 * intact.  Synchronous on `stream`. */
int ecg_k_unaligned_check(void *stream, int *ok);
/* Tiles one segment occupies (0 when len == 0). */
uint64_t ecg_k_copy_tiles(uint64_t dst, uint64_t len);
/* A launch's table (pointer table, update records, copy segments) from the
 * pinned host buffer it was written into to device memory: a kernel reading
 * the host words over PCIe at system scope, queued on `stream` like any
 * launch -- where a small hipMemcpyAsync behind running work keeps the
 * calling thread busy in the runtime until that work drains. */
int ecg_k_launch_fetch(const uint64_t *host_src, uint64_t *dst, uint32_t nwords, void *stream);
/* One launch of ntiles workgroups over nseg segments (segs_dev in device memory). */
int ecg_k_launch_copy_segs(const ecg_copy_seg_t *segs_dev, uint32_t nseg, uint64_t ntiles,
			   void *stream, uint32_t *kernel_id);
/* Implemented in kernels/ecg_kernels.hip.  Returns a hipError_t value. */
int ecg_k_launch_matmul(const ecg_mm_params_t *p, const ecg_launch_cfg_t *cfg,
			void *stream, uint32_t *kernel_id);
/* One-cell product with a per-stripe coefficient column (p->k == 1):
 * dst[s][r] = tbl[r][sel_dev[s]] * src[s]; tables for columns < ncols <= 16.
 * 16-byte aligned operands only (hipErrorInvalidValue otherwise). */
int ecg_k_launch_matmul_sel(const ecg_mm_params_t *p, const uint8_t *sel_dev, uint32_t ncols,
			    void *stream, uint32_t *kernel_id);
/* Streaming kernels used only to measure the box's achievable HBM rates:
 * mode 0 copy, 1 read-only, 2 write-only. */
int ecg_k_launch_copy(const void *src, void *dst, uint64_t bytes, int mode, void *stream,
		      uint32_t max_blocks, uint32_t *kernel_id);
/* Fused product + checksum (kernels/ecg_fused_kernels.hip).  Returns 1 (and
 * launches nothing) when the operands are not 16-byte aligned. */
int ecg_k_launch_matmul_csum(const ecg_mm_params_t *p, const ecg_mmcs_params_t *q,
			     const ecg_launch_cfg_t *cfg, void *stream, uint32_t *kernel_id);
#define ECG_KID_FUSED 500u	/* fused kernel ids start here (below ECG_KID_COPY_SEGS) */
const char *ecg_k_fused_kernel_name(uint32_t kernel_id);
/* The common alignment (16, 8, 4 or 1 bytes) of every cell address of a
 * product launch: the lane access granule the product kernels use. */
uint32_t ecg_k_align_granule(const ecg_mm_params_t *p);
/* Pointer-table product (kernels/ecg_ptr_kernels.hip): cells_dev[s*(k+rows)+j]
 * = device address of input cell j / output cell j-k of stripe s.  granule:
 * 16 = every address 16-byte aligned; 4 = inputs dword-aligned; 2 = k = 8
 * with an input off a 16-byte boundary (16-byte lanes, funnel-shifted); 1 =
 * an input at any byte -- with outputs at any byte in the last three (stored
 * misaligned, so they need the device's unaligned access mode); 0 = the
 * byte-granular kernel (ecg_ptrs.c ptr_granule). */
int ecg_k_launch_matmul_ptrs(const ecg_mm_params_t *p, const uint64_t *cells_dev, int granule,
			     const ecg_launch_cfg_t *cfg, void *stream, uint32_t *kernel_id);
#define ECG_KID_PTR 600u	/* pointer-table kernel ids start here */
const char *ecg_k_ptr_kernel_name(uint32_t kernel_id);
/* Per-request delta updates through a pointer table (the batching queue's
 * device-cell aggregation updates, ecg_update_ptrs):  item s of the launch,
 * a record of ECG_UPD_REC(rows) uint64_t at items_dev + s * ECG_UPD_REC(rows):
 *   [0, rows)            parity cell r (device address; updated in place)
 *   rows + 2m, + 2m + 1  old / new cell of pair m (m < ECG_UPD_MU)
 *   rows + 2 MU          byte m = coefficient column of pair m (< ncols)
 *   rows + 2 MU + 1      n, the pairs in use (1 .. ECG_UPD_MU)
 *   parity[r] ^= XOR_{m<n} tbl[r][col_m] * (old_m ^ new_m)
 * p->nstripes = items, p->rows, p->cell_bytes and p->tbl[r][0 .. ncols) are
 * used.  No two items of one launch may share a parity byte (the host splits
 * such requests into ordered launches).  granule: 16 (every address and C
 * 16-byte aligned), 4 (C % 4 == 0; addresses dword-aligned, or any address on
 * a device that serves misaligned dwords), 0 = one byte per lane. */
#define ECG_UPD_MU 8
#define ECG_UPD_REC(rows) ((rows) + 2 * ECG_UPD_MU + 2)
int ecg_k_launch_update_ptrs(const ecg_mm_params_t *p, const uint64_t *items_dev, uint32_t ncols, int granule,
			     void *stream, uint32_t *kernel_id);
/* Chunked checksums (kernels/ecg_csum_kernels.hip). max_blocks 0 = default. */
int ecg_k_launch_csum(const ecg_csum_params_t *p, void *stream, uint32_t max_blocks,
		      uint32_t *kernel_id);
const char *ecg_k_csum_kernel_name(uint32_t kernel_id);
const char *ecg_k_kernel_name(uint32_t kernel_id);
#ifdef __cplusplus
}
#endif

#endif
