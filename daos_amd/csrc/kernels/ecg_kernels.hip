// ecg_kernels.hip -- CDNA4 (gfx950) kernels for the DAOS EC stripe-cell codec.
//
// One kernel family computes every hot-path product of SURVEY.md §8a:
//   encode   (ISA-L ec_encode_data,          ref:src/object/cli_ec.c:540,571)
//   recovery (DAOS obj_ec_recov_stripe,      ref:src/object/cli_ec.c:2626-2643)
//   update   (xor_gen + ec_encode_data_update, ref:src/object/srv_ec_aggregate.c:1089-1101)
// as  dst[s][r] (^)= XOR_j coef[r][j] * src[s][j]  over GF(2^8)/0x11d.
//
// Design (MI355X-first, not a port of ISA-L's SIMD):
//  * Byte-field arithmetic on the VALU; no MFMA.  c*x is linear over
//    GF(2), so with x = (x&0x07)^(x&0x38)^(x&0xC0) a multiply by a constant is
//    three 8-entry byte lookups, and one v_perm_b32 does an 8-entry lookup for
//    4 bytes at once.  Per 4 source bytes per coefficient: 3 v_perm_b32 + 1.5
//    v_bitop3 (3-way XOR).  The selectors (3 per source dword) are shared by
//    all output rows.  Tables travel in the kernel arguments (no device-side
//    table copy, so launches are graph-capturable) and are staged per block
//    into a few hundred bytes of LDS, read back as broadcasts.
//  * Memory: each lane owns 16 B of every cell (global_load_dwordx4), a
//    256-thread block owns a 4 KiB column of one stripe: every wave issues
//    k x 1 KiB fully coalesced loads before any arithmetic, then p x 1 KiB
//    dwordx4 stores.  Stripes are independent: no inter-workgroup traffic,
//    so XCD placement only affects speed, never results.
//  * Loads/stores are non-temporal: every cell byte is touched exactly once.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "../ecg_kabi.h"
#include "ecg_mm_dev.h"

// K, R: compile-time data cells / output rows (0 = runtime, bounded by the
// ECG_KMAX_* maxima).  ACC: XOR into dst.  DIFF: source = src ^ src2.
//
// Perm tables are staged once per block from the kernel arguments into LDS,
// cell-major: for cell j, RM x {t0lo,t0hi,t1lo,t1hi} then the rows' t2 words
// packed 4 per 16 B.  They are re-read (wave-uniform address -> broadcast,
// conflict-free ds_read_b128) right before cell j is consumed.  Holding them
// in registers instead costs 5 x k x rows dwords: that overflows the SGPR
// file at EC_8P2 (the compiler then spills through v_writelane/v_readlane)
// and caps VGPR occupancy at 1-2 waves/SIMD for k = 16.  An empty asm on the
// LDS index each item keeps LICM from hoisting the reads back out.
// G: lane access granule (lane_off / ld_g), 16 unless an operand is only 4-
// or 8-byte aligned.
template <int K, int R, bool ACC, bool DIFF, int G = 16>
__global__ void __launch_bounds__(BLOCK, ECG_MM_WPE(K, R, G) ? ECG_MM_WPE(K, R, G) : 1)
ecg_mm_kernel(const ecg_mm_params_t P)
{
	constexpr int KM = K ? K : ECG_KMAX_K;
	constexpr int RM = R ? R : ECG_KMAX_R;
	constexpr int T2V = (RM + 3) / 4;		// u32x4 holding t2 of all rows
	constexpr int PER_J = RM + T2V;			// u32x4 per cell
	__shared__ u32x4 s_tbl[KM * PER_J];
	const int k = K ? K : (int)P.k;
	const int rows = R ? R : (int)P.rows;
	const uint64_t C = P.cell_bytes;
	const uint32_t nchunk = (uint32_t)((C + CHUNK_BYTES - 1) / CHUNK_BYTES);
	const uint32_t lo = lane_off<G>();

	for (int i = threadIdx.x; i < KM * RM; i += BLOCK) {
		const int j = i / RM, r = i % RM;
		if (j < k && r < rows) {
			const ecg_ptbl_t &t = P.tbl[r][j];
			s_tbl[j * PER_J + r] = (u32x4){t.t0lo, t.t0hi, t.t1lo, t.t1hi};
			reinterpret_cast<uint32_t *>(&s_tbl[j * PER_J + RM])[r] = t.t2;
		}
	}
	__syncthreads();

	if (P.order) {
		// 1D grid over the S x nchunk (stripe, column) items in the order
		// item_map picks (tuning of the block -> address mapping).
		const uint32_t total = P.nstripes * nchunk;

		for (uint32_t it = blockIdx.x; it < total; it += gridDim.x) {
			uint32_t s, ch, z = 0;

			item_map(P.order, it, total, nchunk, P.nstripes, s, ch);
			const uint64_t cbase = (uint64_t)ch * CHUNK_BYTES;

			asm volatile("" : "+v"(z));
			const u32x4 *tb = s_tbl + z;
			if (cbase + CHUNK_BYTES <= C)
				mm_item<KM, RM, ACC, DIFF, false, G>(P, tb, k, rows, s, cbase, lo);
			else
				mm_partial<KM, RM, ACC, DIFF, G>(P, tb, k, rows, s, cbase, lo);
		}
		return;
	}
	// Normally one item per block (grid = columns x stripes); the loops only
	// stride when a grid dimension would exceed 65535.
	for (uint32_t s = blockIdx.y; s < P.nstripes; s += gridDim.y) {
		for (uint32_t ch = blockIdx.x; ch < nchunk; ch += gridDim.x) {
			const uint64_t cbase = (uint64_t)ch * CHUNK_BYTES;
			uint32_t z = 0;

			asm volatile("" : "+v"(z));
			const u32x4 *tb = s_tbl + z;

			// wave-uniform test first: every full 4 KiB column (all of them
			// when C % 4096 == 0) takes the vector path with no lane mask
			if (cbase + CHUNK_BYTES <= C)
				mm_item<KM, RM, ACC, DIFF, false, G>(P, tb, k, rows, s, cbase, lo);
			else
				mm_partial<KM, RM, ACC, DIFF, G>(P, tb, k, rows, s, cbase, lo);
		}
	}
}

// One-cell product with a per-stripe coefficient column (the batching
// facade's aggregation updates: ec_encode_data_update with vec_i differing
// from stripe to stripe, ref:src/object/srv_ec_aggregate.c:1099-1101):
//   dst[s][r] = coef[r][sel[s]] * src[s]        r < rows, sel[s] < ncols
// The tables of every (row, column) pair are staged in LDS once per block;
// the stripe's column picks the table base (a wave-uniform scalar load), so
// the arithmetic and memory shape are exactly ecg_mm_kernel's with k = 1.
template <int R>
__global__ void __launch_bounds__(BLOCK)
ecg_mm_sel_kernel(const ecg_mm_params_t P, const uint8_t *__restrict__ sel, uint32_t ncols)
{
	constexpr int RM = R ? R : ECG_KMAX_R;
	constexpr int T2V = (RM + 3) / 4;
	constexpr int PER_J = RM + T2V;
	__shared__ u32x4 s_tbl[ECG_KMAX_K * PER_J];
	const int rows = R ? R : (int)P.rows;
	const uint64_t C = P.cell_bytes;
	const uint32_t nchunk = (uint32_t)((C + CHUNK_BYTES - 1) / CHUNK_BYTES);
	const uint32_t lo = threadIdx.x * 16u;

	for (int i = threadIdx.x; i < ECG_KMAX_K * RM; i += BLOCK) {
		const int j = i / RM, r = i % RM;
		if (j < (int)ncols && r < rows) {
			const ecg_ptbl_t &t = P.tbl[r][j];
			s_tbl[j * PER_J + r] = (u32x4){t.t0lo, t.t0hi, t.t1lo, t.t1hi};
			reinterpret_cast<uint32_t *>(&s_tbl[j * PER_J + RM])[r] = t.t2;
		}
	}
	__syncthreads();

	for (uint32_t s = blockIdx.y; s < P.nstripes; s += gridDim.y) {
		const uint32_t j = sel[s];

		if (j >= ncols)		// host-validated; never index past the tables
			continue;
		for (uint32_t ch = blockIdx.x; ch < nchunk; ch += gridDim.x) {
			const uint64_t cbase = (uint64_t)ch * CHUNK_BYTES;
			uint32_t z = 0;

			asm volatile("" : "+v"(z));
			const u32x4 *tb = s_tbl + j * PER_J + z;

			if (cbase + CHUNK_BYTES <= C)
				mm_item<1, RM, false, false>(P, tb, 1, rows, s, cbase, lo);
			else if (cbase + lo + 16 <= C)
				mm_item<1, RM, false, false>(P, tb, 1, rows, s, cbase, lo);
			else if (cbase + lo < C)
				mm_tail<RM, false, false>(P, tb, 1, rows, s, cbase + lo, (int)(C - cbase - lo));
		}
	}
}

// Any alignment, any length: one byte per lane-iteration.  Not chosen by the
// launcher (the lane kernels take every alignment); forced by launch variant
// 2 as a second, independent implementation for tests and A/B runs.
__global__ void __launch_bounds__(BLOCK)
ecg_mm_byte_kernel(const ecg_mm_params_t P)
{
	const uint64_t C = P.cell_bytes;
	const uint64_t total = C * P.nstripes;
	const int k = (int)P.k, rows = (int)P.rows;

	for (uint64_t e = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; e < total;
	     e += (uint64_t)gridDim.x * BLOCK) {
		const uint64_t s = e / C, i = e % C;
		const uint8_t *sb = P.src + (int64_t)s * P.src_stripe_stride;
		const uint8_t *sb2 = P.diff ? P.src2 + (int64_t)s * P.src2_stripe_stride : nullptr;
		uint8_t *db = P.dst + (int64_t)s * P.dst_stripe_stride;
		uint8_t o[ECG_KMAX_R];

		for (int r = 0; r < ECG_KMAX_R; r++)
			o[r] = 0;
		for (int j = 0; j < k; j++) {
			uint32_t v = sb[P.src_cell_off[j] + i];
			if (P.diff)
				v ^= sb2[P.src2_cell_off[j] + i];
			for (int r = 0; r < rows; r++)
				o[r] ^= gf_mul1(P.tbl[r][j], v);
		}
		for (int r = 0; r < rows; r++) {
			uint8_t *d = db + P.dst_cell_off[r] + i;
			*d = P.accumulate ? (uint8_t)(*d ^ o[r]) : o[r];
		}
	}
}

// Streaming kernels used by bench.py to measure this box's achievable HBM
// rates next to the spec peak: mode 0 copy, 1 read-only (XOR-reduce, one
// 16 B word per thread written), 2 write-only.  16 B per lane, 4 accesses in
// flight per lane per iteration.
template <int MODE>
__global__ void __launch_bounds__(BLOCK)
ecg_stream_kernel(const uint8_t *src, uint8_t *dst, uint64_t n16)
{
	const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
	uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
	u32x4 acc = (u32x4){0u, 0u, 0u, 0u};

	for (; i + 3 * stride < n16; i += 4 * stride) {
		if (MODE == 2) {
			const u32x4 v = (u32x4){(uint32_t)i, 1u, 2u, 3u};
#pragma unroll
			for (int q = 0; q < 4; q++)
				st_nt(dst + (i + q * stride) * 16, v);
		} else {
			u32x4 v[4];
#pragma unroll
			for (int q = 0; q < 4; q++)
				v[q] = ld_nt(src + (i + q * stride) * 16);
#pragma unroll
			for (int q = 0; q < 4; q++) {
				if (MODE == 0)
					st_nt(dst + (i + q * stride) * 16, v[q]);
				else
					acc ^= v[q];
			}
		}
	}
	for (; i < n16; i += stride) {
		if (MODE == 0)
			st_nt(dst + i * 16, ld_nt(src + i * 16));
		else if (MODE == 1)
			acc ^= ld_nt(src + i * 16);
		else
			st_nt(dst + i * 16, (u32x4){(uint32_t)i, 1u, 2u, 3u});
	}
	if (MODE == 1)
		st_nt(dst + ((uint64_t)blockIdx.x * BLOCK + threadIdx.x) * 16, acc);
}

// ---------------------------------------------------------------------------
// Dispatch
// ---------------------------------------------------------------------------
typedef void (*mm_fn_t)(const ecg_mm_params_t);

struct kentry {
	int k, r, acc, diff, g;
	mm_fn_t fn;
	const char *name;
};

#define KE(K_, R_, A_, D_) \
	{K_, R_, A_, D_, 16, ecg_mm_kernel<K_, R_, (bool)A_, (bool)D_>, \
	 "ecg_mm_kernel<" #K_ "," #R_ "," #A_ "," #D_ ">"}
#define KEG(K_, R_, A_, D_, G_) \
	{K_, R_, A_, D_, G_, ecg_mm_kernel<K_, R_, (bool)A_, (bool)D_, G_>, \
	 "ecg_mm_kernel<" #K_ "," #R_ "," #A_ "," #D_ ",g" #G_ ">"}
#define KEG_SET(G_) \
	KEG(2, 1, 0, 0, G_), KEG(2, 2, 0, 0, G_), KEG(2, 3, 0, 0, G_), \
	KEG(4, 1, 0, 0, G_), KEG(4, 2, 0, 0, G_), KEG(4, 3, 0, 0, G_), \
	KEG(8, 1, 0, 0, G_), KEG(8, 2, 0, 0, G_), KEG(8, 3, 0, 0, G_), \
	KEG(16, 1, 0, 0, G_), KEG(16, 2, 0, 0, G_), KEG(16, 3, 0, 0, G_), \
	KEG(0, 0, 0, 0, G_), KEG(0, 0, 1, 0, G_), KEG(0, 0, 0, 1, G_), KEG(0, 0, 1, 1, G_)

// Specialised shapes: every (k, p) of the DAOS EC classes
// (ref:src/include/daos_obj_class.h:70-80): k in {2,4,8,16}, rows in 1..3
// (encode rows = p; recovery rows = nerrs <= p).  Everything else runs the
// runtime-shaped instantiation (K = R = 0).  The same set again for operands
// that are only 8- or 4-byte aligned (DAOS rounds parity rows to 8 bytes,
// ref:src/object/cli_ec.c:86; user sgl cells carry no alignment,
// ref:src/object/cli_ec.c:510-536).
static const kentry g_kernels[] = {
	KE(2, 1, 0, 0), KE(2, 2, 0, 0), KE(2, 3, 0, 0),
	KE(4, 1, 0, 0), KE(4, 2, 0, 0), KE(4, 3, 0, 0),
	KE(8, 1, 0, 0), KE(8, 2, 0, 0), KE(8, 3, 0, 0),
	KE(16, 1, 0, 0), KE(16, 2, 0, 0), KE(16, 3, 0, 0),
	// aggregation's delta update of 1-4 cells per stripe (ACC + DIFF, rows =
	// p), ref:src/object/srv_ec_aggregate.c:1099-1101 -- DAOS re-encodes the
	// stripe instead when more of it changed (agg_recalc_parity): the runtime-
	// shaped ACC + DIFF kernel holds 189 VGPRs (2 waves per SIMD) and ran these
	// at half the rate (profiles/r04/ec_ab/ec_ab_update*.json)
	KE(1, 1, 1, 1), KE(1, 2, 1, 1), KE(1, 3, 1, 1),
	KE(2, 1, 1, 1), KE(2, 2, 1, 1), KE(2, 3, 1, 1),
	KE(3, 1, 1, 1), KE(3, 2, 1, 1), KE(3, 3, 1, 1),
	KE(4, 1, 1, 1), KE(4, 2, 1, 1), KE(4, 3, 1, 1),
	KE(0, 0, 0, 0), KE(0, 0, 1, 0), KE(0, 0, 0, 1), KE(0, 0, 1, 1),
	KEG_SET(4), KEG_SET(1),
	// k = 8 sources off a 16-byte boundary: 16-byte lanes, funnel-shifted
	// (ld_src16); measured neutral at k = 2 / 4 and slower at k = 16
	// (tools/unaligned_ab.py, profiles/r05/unaligned_ab/), so only k = 8 has them
	KEG(8, 1, 0, 0, 2), KEG(8, 2, 0, 0, 2), KEG(8, 3, 0, 0, 2),
};
#define N_KERNELS ((uint32_t)(sizeof(g_kernels) / sizeof(g_kernels[0])))




#define KID_SEL 700u		/* per-stripe column kernels: <1>, <2>, <0> */

#define KID_BYTE N_KERNELS
#define KID_COPY (N_KERNELS + 1)
#define KID_READ (N_KERNELS + 2)
#define KID_WRITE (N_KERNELS + 3)

// All output cells equally far (md bytes) past a dword boundary: *head = the
// 4 - md bytes before their first aligned dword (1).  0 if they differ.
// 4 lanes copy a dword from in + 1 + 4i to out + 3 + 4i: misaligned vector
// loads and stores exactly as the product's lanes issue them (per-lane
// addresses, so never scalar-memory accesses)
__global__ void ecg_unaligned_probe_kernel(const uint8_t *in, uint8_t *out)
{
	const uint32_t i = threadIdx.x;

	if (i < 4) {
		const uint32_t v = *reinterpret_cast<const uint32_t *>(in + 1 + 4 * i);
		*reinterpret_cast<uint32_t *>(out + 3 + 4 * i) = v;
	}
}

extern "C" int ecg_k_unaligned_check(void *stream, int *ok)
{
	hipStream_t st = (hipStream_t)stream;
	uint8_t h[64], *d = nullptr;
	hipError_t e;

	*ok = 0;
	for (int i = 0; i < 32; i++)
		h[i] = (uint8_t)(0x40 + i);
	memset(h + 32, 0xEE, 32);
	e = hipMalloc(&d, 64);
	if (e != hipSuccess)
		return (int)e;
	e = hipMemcpyAsync(d, h, 64, hipMemcpyHostToDevice, st);
	if (e == hipSuccess) {
		hipLaunchKernelGGL(ecg_unaligned_probe_kernel, dim3(1), dim3(64), 0, st, d, d + 32);
		e = hipGetLastError();
	}
	if (e == hipSuccess)
		e = hipMemcpyAsync(h, d, 64, hipMemcpyDeviceToHost, st);
	if (e == hipSuccess)
		e = hipStreamSynchronize(st);
	(void)hipFree(d);
	if (e != hipSuccess)
		return (int)e;
	*ok = 1;
	for (int i = 0; i < 32; i++) {
		const uint8_t want = i >= 3 && i < 19 ? (uint8_t)(0x40 + i - 2) : 0xEE;

		if (h[32 + i] != want)
			*ok = 0;
	}
	return 0;
}

// destinations off a dword boundary (their stores, and ACC loads, are
// misaligned dword accesses)
static bool dst_misaligned(const ecg_mm_params_t *p)
{
	uint64_t db = (uint64_t)(uintptr_t)p->dst | (uint64_t)p->dst_stripe_stride;

	for (uint32_t r = 0; r < p->rows; r++)
		db |= (uint64_t)p->dst_cell_off[r];
	return (db & 3u) != 0;
}

// Sources (not only destinations) off a 16-byte boundary.
static bool src_off16(const ecg_mm_params_t *p)
{
	uint64_t sb = (uint64_t)(uintptr_t)p->src | (uint64_t)p->src_stripe_stride;

	for (uint32_t j = 0; j < p->k; j++)
		sb |= (uint64_t)p->src_cell_off[j];
	if (p->diff) {
		sb |= (uint64_t)(uintptr_t)p->src2 | (uint64_t)p->src2_stripe_stride;
		for (uint32_t j = 0; j < p->k; j++)
			sb |= (uint64_t)p->src2_cell_off[j];
	}
	return (sb & 15u) != 0;
}

// A G = 2 instantiation exists for this shape.
static bool has_g2(const ecg_mm_params_t *p)
{
	for (uint32_t i = 0; i < N_KERNELS; i++)
		if (g_kernels[i].g == 2 && g_kernels[i].k == (int)p->k && g_kernels[i].r == (int)p->rows &&
		    g_kernels[i].acc == (int)(p->accumulate != 0) && g_kernels[i].diff == (int)(p->diff != 0))
			return true;
	return false;
}

extern "C" uint32_t ecg_k_align_granule(const ecg_mm_params_t *p)
{
	return align_granule(p);
}

extern "C" const char *ecg_k_kernel_name(uint32_t id)
{
	if (id < N_KERNELS)
		return g_kernels[id].name;
	if (id == KID_BYTE)
		return "ecg_mm_byte_kernel";
	if (id == KID_COPY)
		return "ecg_stream_kernel<copy>";
	if (id == KID_READ)
		return "ecg_stream_kernel<read>";
	if (id == KID_WRITE)
		return "ecg_stream_kernel<write>";
	if (id >= ECG_KID_CSUM)
		return ecg_k_csum_kernel_name(id);
	if (id >= ECG_KID_FUSED && id < ECG_KID_FUSED + 100u)	/* below KID_PTR */
		return ecg_k_fused_kernel_name(id);
	if (id >= ECG_KID_PTR && id < ECG_KID_PTR + 100u)
		return ecg_k_ptr_kernel_name(id);
	if (id == ECG_KID_COPY_SEGS)
		return "ecg_copy_segs_kernel";
	if (id == KID_SEL)
		return "ecg_mm_sel_kernel<1>";
	if (id == KID_SEL + 1)
		return "ecg_mm_sel_kernel<2>";
	if (id == KID_SEL + 2)
		return "ecg_mm_sel_kernel<0>";

	return "?";
}

extern "C" int ecg_k_launch_matmul(const ecg_mm_params_t *p, const ecg_launch_cfg_t *cfg,
				   void *stream, uint32_t *kernel_id)
{
	hipStream_t st = (hipStream_t)stream;
	const uint32_t variant = cfg ? cfg->variant : 0;
	const uint64_t nchunk = (p->cell_bytes + CHUNK_BYTES - 1) / CHUNK_BYTES;

	if (p->nstripes == 0 || p->cell_bytes == 0 || p->rows == 0)
		return (int)hipSuccess;

	// the widest lane access every operand's alignment allows (16 / 4 B;
	// 1: a source at any byte -- funnel-shifted loads); destinations at any
	// byte take the dword lanes' (misaligned) stores
	int g = (int)align_granule(p);
	if (cfg && cfg->no_unaligned && (g == 1 || dst_misaligned(p)))
		g = 0;		// the device serves no misaligned dwords: bytewise
	else if (variant == 3 && g < 4)
		g = 4;		// A/B: misaligned source dwords loaded as they are
	else if (variant == 0 && g < 16 && !(cfg && cfg->no_unaligned) && src_off16(p) && has_g2(p))
		g = 2;		// k = 8, sources off a 16-byte boundary: funnel-shifted 16-byte lanes
	if (variant == 2 || g == 0) {
		uint64_t total = p->cell_bytes * p->nstripes;
		uint64_t blocks = (total + BLOCK - 1) / BLOCK;
		if (blocks > 8192)
			blocks = 8192;
		hipLaunchKernelGGL(ecg_mm_byte_kernel, dim3((uint32_t)blocks), dim3(BLOCK), 0, st, *p);
		if (kernel_id)
			*kernel_id = KID_BYTE;
		return (int)hipGetLastError();
	}

	uint32_t id = N_KERNELS;
	if (variant != 1) {
		for (uint32_t i = 0; i < N_KERNELS; i++)
			if (g_kernels[i].g == g && g_kernels[i].k == (int)p->k && g_kernels[i].r == (int)p->rows &&
			    g_kernels[i].acc == (int)(p->accumulate != 0) && g_kernels[i].diff == (int)(p->diff != 0)) {
				id = i;
				break;
			}
	}
	if (id == N_KERNELS) {
		for (uint32_t i = 0; i < N_KERNELS; i++)
			if (g_kernels[i].g == g && g_kernels[i].k == 0 && g_kernels[i].acc == (int)(p->accumulate != 0) &&
			    g_kernels[i].diff == (int)(p->diff != 0)) {
				id = i;
				break;
			}
	}
	if (id == N_KERNELS)
		return (int)hipErrorInvalidDeviceFunction;

	// Grid: x over the 4 KiB columns of a stripe, y over stripes, one
	// (stripe, column) item per block.  Measured on MI355X (tools/tune2.py,
	// profiles/r01/tune2.json): one-shot blocks beat a ~8 blocks/CU
	// grid-stride grid by 15-30 % on every shape (EC_4P2 encode 4.7 ->
	// 6.2 TB/s) -- the dispatcher refills CUs faster than a resident block
	// re-issues its next item's loads.  Both loops still stride for
	// grids beyond 65535.
	const uint64_t total = nchunk * p->nstripes;
	const uint32_t order = cfg ? cfg->order : 0;
	if (order >= 1 && order <= 3 && total < (1ull << 31) && (order == 1 || total % 8 == 0)) {
		ecg_mm_params_t q = *p;
		uint32_t gx = cfg->grid_x ? cfg->grid_x : (uint32_t)total;

		q.order = order;
		hipLaunchKernelGGL(g_kernels[id].fn, dim3(gx), dim3(BLOCK), 0, st, q);
		if (kernel_id)
			*kernel_id = id;
		return (int)hipGetLastError();
	}
	uint32_t gx = cfg && cfg->grid_x ? cfg->grid_x : (uint32_t)(nchunk < 65535 ? nchunk : 65535);
	uint32_t gy = cfg && cfg->grid_y ? cfg->grid_y : (p->nstripes < 65535 ? p->nstripes : 65535);
	const size_t lds = mm_dyn_lds(mm_wg_cap(p, cfg, (uint64_t)gx * gy), g_kernels[id].k, g_kernels[id].r);
	if (p->order) {
		ecg_mm_params_t q = *p;

		q.order = 0;
		hipLaunchKernelGGL(g_kernels[id].fn, dim3(gx, gy), dim3(BLOCK), lds, st, q);
	} else {
		hipLaunchKernelGGL(g_kernels[id].fn, dim3(gx, gy), dim3(BLOCK), lds, st, *p);
	}
	if (kernel_id)
		*kernel_id = id;
	return (int)hipGetLastError();
}

extern "C" int ecg_k_launch_copy(const void *src, void *dst, uint64_t bytes, int mode, void *stream,
				 uint32_t max_blocks, uint32_t *kernel_id)
{
	const uint64_t n16 = bytes / 16;
	uint64_t blocks = (n16 + 4 * BLOCK - 1) / (4 * BLOCK);
	hipStream_t st = (hipStream_t)stream;

	if (max_blocks == 0)
		max_blocks = 1u << 20;
	if (blocks > max_blocks)
		blocks = max_blocks;
	if (blocks == 0)
		return (int)hipSuccess;
	if (mode == 1)
		hipLaunchKernelGGL(ecg_stream_kernel<1>, dim3((uint32_t)blocks), dim3(BLOCK), 0, st,
				   (const uint8_t *)src, (uint8_t *)dst, n16);
	else if (mode == 2)
		hipLaunchKernelGGL(ecg_stream_kernel<2>, dim3((uint32_t)blocks), dim3(BLOCK), 0, st,
				   (const uint8_t *)src, (uint8_t *)dst, n16);
	else
		hipLaunchKernelGGL(ecg_stream_kernel<0>, dim3((uint32_t)blocks), dim3(BLOCK), 0, st,
				   (const uint8_t *)src, (uint8_t *)dst, n16);
	if (kernel_id)
		*kernel_id = mode == 1 ? KID_READ : mode == 2 ? KID_WRITE : KID_COPY;
	return (int)hipGetLastError();
}

extern "C" int ecg_k_launch_matmul_sel(const ecg_mm_params_t *p, const uint8_t *sel_dev, uint32_t ncols,
				      void *stream, uint32_t *kernel_id)
{
	const uint64_t nchunk = (p->cell_bytes + CHUNK_BYTES - 1) / CHUNK_BYTES;

	if (p->nstripes == 0 || p->cell_bytes == 0 || p->rows == 0)
		return (int)hipSuccess;
	if (!aligned16(p) || p->k != 1 || p->accumulate || p->diff || ncols == 0 || ncols > ECG_KMAX_K ||
	    p->rows > ECG_KMAX_R)
		return (int)hipErrorInvalidValue;
	uint32_t gx = (uint32_t)(nchunk < 65535 ? nchunk : 65535);
	uint32_t gy = p->nstripes < 65535 ? p->nstripes : 65535;
	// the DAOS classes' p = 1, 2 specialised; 3..8 parity rows runtime-shaped
	const uint32_t v = p->rows == 1 ? 0 : p->rows == 2 ? 1 : 2;
	if (v == 0)
		hipLaunchKernelGGL(ecg_mm_sel_kernel<1>, dim3(gx, gy), dim3(BLOCK), 0, (hipStream_t)stream, *p,
				   sel_dev, ncols);
	else if (v == 1)
		hipLaunchKernelGGL(ecg_mm_sel_kernel<2>, dim3(gx, gy), dim3(BLOCK), 0, (hipStream_t)stream, *p,
				   sel_dev, ncols);
	else
		hipLaunchKernelGGL(ecg_mm_sel_kernel<0>, dim3(gx, gy), dim3(BLOCK), 0, (hipStream_t)stream, *p,
				   sel_dev, ncols);
	if (kernel_id)
		*kernel_id = KID_SEL + v;
	return (int)hipGetLastError();
}
