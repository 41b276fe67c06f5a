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

#include "../ecg_kabi.h"
#include "ecg_crc_dev.h"

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CHUNK_BYTES 4096u	// 256 lanes x 16 B
#define BLOCK 256
#ifndef ECG_FUSED_PF64
#define ECG_FUSED_PF64 1	// prefetch in the crc64 fused kernels too
#endif
#ifndef ECG_MM_WG_DEFAULT
// per-shape default blocks per CU (mm_wg_cap) by the cell streams a block
// keeps in flight (k + rows): none -- see mm_wg_cap
#define ECG_MM_WG_DEFAULT(streams) 0u
#endif
#ifndef ECG_EXP_DYN_LDS
#define ECG_EXP_DYN_LDS 0	// experimental builds: unused dynamic LDS per block caps blocks per CU
#endif
#ifndef ECG_FUSED_PF_MAXK
#define ECG_FUSED_PF_MAXK 8	// fused kernels: next column's loads in flight for k <= this
#endif
// fused kernels: the waves per SIMD their register budget targets.  crc16 /
// crc32 get the 3-wave budget (<= 168 VGPRs): at a 4-wave budget the register
// allocator spilled EC_8P2's pipelined loop to scratch, at 3 it settles at
// 104 VGPRs -- 4 waves anyway, no spills.  crc64 fits 4 waves without spills.
#ifndef ECG_FUSED_WPE
#define ECG_FUSED_WPE(W) ((W) == 64 ? 4 : 3)
#endif
// fused workgroup kernel: fold each column's outputs into the CRC one column
// later, while the next column's product is computed (independent work the
// scheduler can interleave with the lookup chains).  Bit 0: crc16/crc32,
// bit 1: crc64.  Measured (tools/fused_libs.py, 3 interleaved rounds,
// profiles/r03/defer/): EC_8P2 x 512 crc64 0.906 -> 0.886 ms (encode 0.838),
// crc32 and EC_4P2 unchanged within +-0.5 %.
#ifndef ECG_FUSED_DEFER
#define ECG_FUSED_DEFER 3
#endif

template <bool B>
struct ecg_bool {
	static constexpr bool value = B;
};

__device__ __forceinline__ u32x4 ld_nt(const uint8_t *p)
{
	return __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
}

__device__ __forceinline__ void st_nt(uint8_t *p, u32x4 v)
{
	__builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(p));
}

// c*x for the 4 bytes of one dword, given that dword's 3 selector words.
__device__ __forceinline__ uint32_t gf_mul4(const ecg_ptbl_t &t, uint32_t s0, uint32_t s1, uint32_t s2)
{
	return __builtin_amdgcn_perm(t.t0hi, t.t0lo, s0) ^
	       __builtin_amdgcn_perm(t.t1hi, t.t1lo, s1) ^
	       __builtin_amdgcn_perm(t.t2, t.t2, s2);
}

// Byte-granular product for the < 16-byte tail of a cell (and the
// misaligned fallback): same tables, one byte in the low lane of a dword.
__device__ __forceinline__ uint8_t gf_mul1(const ecg_ptbl_t &t, uint32_t x)
{
	return (uint8_t)gf_mul4(t, x & 7u, (x >> 3) & 7u, x >> 6);
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c)
{
	return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// One (stripe, 4 KiB column) item of the product.  Addresses are a
// wave-uniform 64-bit base per cell (SGPRs) plus the lane's 32-bit offset.
// The uniform cell offsets are passed through an empty asm per item so LICM
// cannot hoist k+rows 64-bit pointers out of the stripe loop (they land in
// VGPRs and spill at EC_8P2/EC_16P2).
template <int KM, bool DIFF>
__device__ __forceinline__ void mm_load(const ecg_mm_params_t &P, int k, uint32_t s, uint64_t cbase,
					uint32_t lo, u32x4 *x)
{
	const int64_t s_src = (int64_t)s * P.src_stripe_stride + (int64_t)cbase;
	const int64_t s_src2 = DIFF ? (int64_t)s * P.src2_stripe_stride + (int64_t)cbase : 0;

#pragma unroll
	for (int j = 0; j < KM; j++) {
		if (j < k) {
			int64_t o = P.src_cell_off[j] + s_src;
			asm volatile("" : "+s"(o));
			x[j] = ld_nt(P.src + o + lo);
			if (DIFF) {
				int64_t o2 = P.src2_cell_off[j] + s_src2;
				asm volatile("" : "+s"(o2));
				x[j] ^= ld_nt(P.src2 + o2 + lo);
			}
		}
	}
}

// mm_load with no branch: lanes whose 16 bytes would pass the cell end read
// the column's first 16 bytes instead (C % 16 == 0; callers never use those
// lanes' values)
template <int KM>
__device__ __forceinline__ void mm_load_any(const ecg_mm_params_t &P, int k, uint32_t s, uint64_t cbase,
					    uint32_t lo, u32x4 *x)
{
	mm_load<KM, false>(P, k, s, cbase, cbase + lo + 16 <= P.cell_bytes ? lo : 0u, x);
}

template <int KM, int RM, bool ACC, bool KEEP, bool STORE = true>
__device__ __forceinline__ void mm_compute(const ecg_mm_params_t &P, const u32x4 *tb, int k, int rows,
					   uint32_t s, uint64_t cbase, uint32_t lo, const u32x4 *x,
					   u32x4 *keep);

template <int KM, int RM, bool ACC, bool DIFF, bool KEEP = false>
__device__ __forceinline__ void mm_item(const ecg_mm_params_t &P, const u32x4 *tb, int k, int rows,
					uint32_t s, uint64_t cbase, uint32_t lo, u32x4 *keep = nullptr)
{
	u32x4 x[KM];

	mm_load<KM, DIFF>(P, k, s, cbase, lo, x);
	mm_compute<KM, RM, ACC, KEEP>(P, tb, k, rows, s, cbase, lo, x, keep);
}

// The product of one loaded column: x[j] = the lane's 16 bytes of cell j.
// STORE = false leaves the stores to the caller (outputs returned in keep).
template <int KM, int RM, bool ACC, bool KEEP, bool STORE>
__device__ __forceinline__ void mm_compute(const ecg_mm_params_t &P, const u32x4 *tb, int k, int rows,
					   uint32_t s, uint64_t cbase, uint32_t lo, const u32x4 *x,
					   u32x4 *keep)
{
	constexpr int T2V = (RM + 3) / 4;
	constexpr int PER_J = RM + T2V;
	const int64_t s_dst = (int64_t)s * P.dst_stripe_stride + (int64_t)cbase;

	u32x4 acc[RM];
#pragma unroll
	for (int r = 0; r < RM; r++) {
		if (r < rows) {
			if (ACC) {
				int64_t o = P.dst_cell_off[r] + s_dst;
				asm volatile("" : "+s"(o));
				acc[r] = ld_nt(P.dst + o + lo);
			} else {
				acc[r] = (u32x4){0u, 0u, 0u, 0u};
			}
		}
	}
#pragma unroll
	for (int j = 0; j < KM; j++) {
#ifdef ECG_EXP_XOR_ONLY
		// experimental build (tools/ec_libs.py): XOR instead of the GF
		// multiply -- same memory traffic, grid and address registers
		if (j < k) {
#pragma unroll
			for (int r = 0; r < RM; r++)
				if (r < rows)
					acc[r] ^= x[j];
		}
		continue;
#endif
		if (j < k) {
			u32x4 sel0, sel1, sel2;
#pragma unroll
			for (int w = 0; w < 4; w++) {
				const uint32_t v = x[j][w];
				sel0[w] = v & 0x07070707u;
				sel1[w] = (v >> 3) & 0x07070707u;
				sel2[w] = (v >> 6) & 0x03030303u;
			}
			u32x4 t2v[T2V];
#pragma unroll
			for (int q = 0; q < T2V; q++)
				t2v[q] = tb[j * PER_J + RM + q];
#pragma unroll
			for (int r = 0; r < RM; r++) {
				if (r < rows) {
					const u32x4 t = tb[j * PER_J + r];
					const uint32_t t2 = t2v[r / 4][r % 4];
#pragma unroll
					for (int w = 0; w < 4; w++) {
						const uint32_t p0 = __builtin_amdgcn_perm(t[1], t[0], sel0[w]);
						const uint32_t p1 = __builtin_amdgcn_perm(t[3], t[2], sel1[w]);
						const uint32_t p2 = __builtin_amdgcn_perm(t2, t2, sel2[w]);
						acc[r][w] = xor3(acc[r][w], p0, xor3(p1, p2, 0u));
					}
				}
			}
		}
	}
#pragma unroll
	for (int r = 0; r < RM; r++) {
		if (r < rows) {
			if (STORE) {
				int64_t o = P.dst_cell_off[r] + s_dst;
				asm volatile("" : "+s"(o));
				st_nt(P.dst + o + lo, acc[r]);
			}
			if (KEEP)
				keep[r] = acc[r];
		}
	}
}

// Ragged tail: fewer than 16 bytes of this lane's slot are inside the cell.
template <int RM, bool ACC, bool DIFF>
__device__ __forceinline__ void mm_tail(const ecg_mm_params_t &P, const u32x4 *tb, int k, int rows,
				     uint32_t s, uint64_t off, int nb)
{
	constexpr int T2V = (RM + 3) / 4;
	constexpr int PER_J = RM + T2V;
	const uint8_t *sb = P.src + (int64_t)s * P.src_stripe_stride;
	const uint8_t *sb2 = DIFF ? P.src2 + (int64_t)s * P.src2_stripe_stride : nullptr;
	uint8_t *db = P.dst + (int64_t)s * P.dst_stripe_stride;

	for (int b = 0; b < nb; b++) {
		uint32_t o[RM];
#pragma unroll
		for (int r = 0; r < RM; r++)
			o[r] = 0;
		for (int j = 0; j < k; j++) {
			uint32_t v = sb[P.src_cell_off[j] + off + b];
			if (DIFF)
				v ^= sb2[P.src2_cell_off[j] + off + b];
			const uint32_t s0 = v & 7u, s1 = (v >> 3) & 7u, s2 = v >> 6;
#pragma unroll
			for (int r = 0; r < RM; r++) {
				if (r < rows) {
					const u32x4 t = tb[j * PER_J + r];
					const uint32_t t2 = reinterpret_cast<const uint32_t *>(&tb[j * PER_J + RM])[r];
					o[r] ^= __builtin_amdgcn_perm(t[1], t[0], s0) ^
						__builtin_amdgcn_perm(t[3], t[2], s1) ^
						__builtin_amdgcn_perm(t2, t2, s2);
				}
			}
		}
#pragma unroll
		for (int r = 0; r < RM; r++) {
			if (r < rows) {
				uint8_t *d = db + P.dst_cell_off[r] + off + b;
				*d = ACC ? (uint8_t)(*d ^ o[r]) : (uint8_t)o[r];
			}
		}
	}
}

// 1D item orders (P.order): which (stripe, 4 KiB column) block `it` of a
// 1D grid works on.  The hardware dispatcher hands consecutive block ids to
// the 8 XCDs round-robin, so `it & 7` is (nearly) the block's XCD.
//   1  stripe-fastest: consecutive blocks touch the same column of
//      consecutive stripes
//   2  XCD-blocked, column-fastest: XCD x walks the x-th eighth of the
//      column-fastest item list (each XCD streams its own stripe range)
//   3  XCD-blocked, stripe-fastest
__device__ __forceinline__ void item_map(uint32_t order, uint32_t it, uint32_t total, uint32_t nchunk,
					 uint32_t S, uint32_t &s, uint32_t &ch)
{
	uint32_t g = it;

	if (order >= 2) {
		const uint32_t per = (total + 7) / 8;	// items per XCD slice
		const uint32_t x = it & 7, j = it >> 3;

		g = x * per + j;
		if (g >= total)			// uneven tail: fall back to the plain id
			g = it;
	}
	if (order == 1 || order == 3) {
		s = g % S;
		ch = g / S;
	} else {
		s = g / nchunk;
		ch = g - s * nchunk;
	}
}

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
template <int K, int R, bool ACC, bool DIFF>
__global__ void __launch_bounds__(BLOCK)
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
	const uint32_t lo = threadIdx.x * 16u;

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
				mm_item<KM, RM, ACC, DIFF>(P, tb, k, rows, s, cbase, lo);
			else if (cbase + lo + 16 <= C)
				mm_item<KM, RM, ACC, DIFF>(P, tb, k, rows, s, cbase, lo);
			else if (cbase + lo < C)
				mm_tail<RM, ACC, DIFF>(P, tb, k, rows, s, cbase + lo, (int)(C - cbase - lo));
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
			if (cbase + CHUNK_BYTES <= C) {
				mm_item<KM, RM, ACC, DIFF>(P, tb, k, rows, s, cbase, lo);
			} else if (cbase + lo + 16 <= C) {
				mm_item<KM, RM, ACC, DIFF>(P, tb, k, rows, s, cbase, lo);
			} else if (cbase + lo < C) {
				mm_tail<RM, ACC, DIFF>(P, tb, k, rows, s, cbase + lo, (int)(C - cbase - lo));
			}
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

// Work item `it` of the fused kernel -> chunk c, sub-chunk h, its columns
// [col0, col1) and the row of Q.kh its threads multiply by (ecg_kabi.h).
__device__ __forceinline__ void mmcs_item(const ecg_mmcs_params_t &Q, uint32_t it, uint32_t &c, uint32_t &col0,
					  uint32_t &col1, uint32_t &khrow)
{
	c = it / Q.nh;
	const uint32_t h = it - c * Q.nh;
	const bool lastc = c + 1 == Q.nch;
	const uint32_t m = lastc ? Q.m_last : Q.m;

	col0 = h * Q.ncols;
	col1 = col0 + Q.ncols < m ? col0 + Q.ncols : m;
	khrow = (lastc ? Q.nh : 0) + h;
}

// One column of a fused product + checksum item (the workgroup kernel's 4 KiB
// columns, the wave kernel's 1 KiB rows; STRIDE bytes): with PF, first the
// next column's loads into nxt (when `more`), then the product of cur -- the
// sources already in registers -- and its stores, then each output row's
// 16-byte piece folded into the row's CRC.  TB 0: pos = columns to the item
// end mod U selects the positional table; the register is shifted by U
// columns at each group start (pos == U - 1).  `first`: this piece starts
// the chunk, the initial register is folded into it.  `next`: the column the
// prefetch reads (the walk need not be in address order); gshift = false for
// a walk whose positions all fit the U tables (no register shift at all).
// The kernel arguments re-read (scalar loads, K$ hits) where they are used:
// an empty asm on their constant-space address stops the compiler from
// keeping every cell offset of the launch live in SGPRs across a column loop
// (the fused kernels spilled SGPRs into VGPR lanes).
typedef __attribute__((address_space(4))) const ecg_mm_params_t kparams_t;

__device__ __forceinline__ const ecg_mm_params_t &kernarg_fresh()
{
	// the kernel's first argument sits at the start of the kernarg segment
	kparams_t *p = (kparams_t *)__builtin_amdgcn_kernarg_segment_ptr();

	asm volatile("" : "+s"(p));
	return *(const ecg_mm_params_t *)p;
}

// A column's outputs waiting to be folded (ECG_FUSED_DEFER): the fold of
// column i runs after column i+1's product.  The zero state (have = false,
// gshift = false) folds to nothing on a zero register.
template <int RM>
struct mmcs_pend {
	u32x4 v[RM];
	bool have, first, gshift;
	uint32_t pos;
};

// Fold one column's output pieces into the rows' CRC registers: the register
// shift of the table kind, then the piece's lookups (see mmcs_col).
template <int RM, int W, bool REFL, int TB, int U, int FP, typename T>
__device__ __forceinline__ void mmcs_fold(const T *s_sl, const T *s_sh, int rows, const u32x4 *outv, bool have,
					  bool first, uint64_t init, uint32_t pos, bool gshift, T *crc)
{
	using F5 = ecg_crc::f5u<W, U>;
#pragma unroll
	for (int r = 0; r < RM; r++) {
		if (r < rows) {
#ifndef ECG_EXP_NO_CRC
			if constexpr (TB == 3 || (TB == 4 && FP < 0))
				crc[r] = ecg_crc::lin_map4<W>(crc[r], s_sh);	// a4 of one column
			else if constexpr (TB == 4)
				;	// fixed position FP: no register shift
			else if constexpr (TB != 0)
				crc[r] = ecg_crc::lin_map5<W>(crc[r], s_sh);	// a5 of one column
			else if (gshift && pos == F5::U - 1)
				crc[r] = ecg_crc::lin_map5<W>(crc[r], s_sl + F5::U * F5::NF * 32);
#endif
			if (have) {
				uint32_t d[4] = {outv[r][0], outv[r][1], outv[r][2], outv[r][3]};
				if (first) {	// initial register
					d[0] ^= (uint32_t)init;
					if constexpr (W == 64)
						d[1] ^= (uint32_t)(init >> 32);
				}
#ifndef ECG_EXP_NO_CRC
				if constexpr (TB == 1)
					crc[r] ^= ecg_crc::piece_crc<W, REFL>(d, s_sl);
				else if constexpr (TB == 2)
					crc[r] ^= ecg_crc::piece_crc16<W>(d, s_sl);
				else if constexpr (TB == 3)
					crc[r] ^= ecg_crc::piece_crc16s<W>(d, s_sl);
				else if constexpr (TB == 4)	// nibble tables of position FP (0: Horner with the shift)
					crc[r] ^= ecg_crc::piece_crc4(d, s_sl + (FP < 0 ? 0 : FP) * ECG_CSUM_NQ4);
				else
					crc[r] ^= ecg_crc::piece_crc5p<W>(d, s_sl, pos * (uint32_t)(F5::NF * 32 * sizeof(T)));
#else
				crc[r] ^= (T)(d[0] ^ d[1] ^ d[2] ^ d[3]);
#endif
			}
		}
	}
}

// DF: 0 fold this column now; 1 fold the pending column (fixed position FPP)
// and leave this one pending; 2 leave this one pending (nothing pending yet).
template <int KM, int RM, int W, bool REFL, int TB, bool PF, uint32_t STRIDE, bool FULL, int U, int FP = -1,
	  int DF = 0, int FPP = -1, typename T>
__device__ __forceinline__ void mmcs_col(const ecg_mm_params_t &P0, const u32x4 *s_tbl, const T *s_sl,
					 const T *s_sh, int k, int rows, uint32_t s, uint64_t cbase, uint64_t next,
					 uint32_t lo, bool more, bool first, uint64_t init, uint32_t pos, bool gshift,
					 u32x4 *cur, u32x4 *nxt, T *crc, mmcs_pend<RM> *pd = nullptr)
{
#ifdef ECG_EXP_KARG_CACHED
	const ecg_mm_params_t &P = P0;			// experimental: arguments held by the compiler
#else
	const ecg_mm_params_t &P = kernarg_fresh();	// == P0 (first kernel argument)
	(void)P0;
#endif
	const uint64_t C = P.cell_bytes;
	const bool have = FULL || cbase + lo + 16 <= C;	// C % 16 == 0
	u32x4 outv[RM];
	uint32_t z = 0;

	if constexpr (PF) {
		// no branch around the prefetch: a load that may or may not be
		// issued makes the compiler's waitcnt merge wait for everything
		// (vmcnt(0)) before the product.  Past the item's last column the
		// wave re-reads stripe 0's first column (cache-resident, unused).
		mm_load_any<KM>(P, k, more ? s : 0, more ? next : 0, lo, nxt);
	} else {
		// unconditional (clamped) loads: a load skipped by some lanes would
		// keep cur live across columns and items (zero-filled and spilled)
		mm_load_any<KM>(P, k, s, cbase, lo, cur);
	}
	asm volatile("" : "+v"(z));
	const u32x4 *tb = s_tbl + z;
	// FULL (the column lies inside the cell): no branch, so the pipelined
	// loop of the callers has one path -- a partial-column path that may skip
	// the loads or use other registers for its stores makes the compiler wait
	// for everything (vmcnt(0)) at the loop head
	if constexpr (!FULL && DF != 0) {
#pragma unroll
		for (int r = 0; r < RM; r++)
			outv[r] = (u32x4){0, 0, 0, 0};
	}
	if (FULL || cbase + STRIDE <= C)
		mm_compute<KM, RM, false, true>(P, tb, k, rows, s, cbase, lo, cur, outv);
	else if (have)
		mm_compute<KM, RM, false, true>(P, tb, k, rows, s, cbase, lo, cur, outv);
	if constexpr (DF == 0) {
		mmcs_fold<RM, W, REFL, TB, U, FP>(s_sl, s_sh, rows, outv, have, first, init, pos, gshift, crc);
	} else {
		if constexpr (DF == 1)
			mmcs_fold<RM, W, REFL, TB, U, FPP>(s_sl, s_sh, rows, pd->v, pd->have, pd->first, init, pd->pos,
							   pd->gshift, crc);
#pragma unroll
		for (int r = 0; r < RM; r++)
			pd->v[r] = outv[r];
		pd->have = have;
		pd->first = first;
		pd->pos = pos;
		pd->gshift = gshift;
	}
}

// Fused product + checksum of every output cell (ecg_kabi.h, ecg_mmcs_params).
// Block = a stream of (stripe, sub-chunk) items of a few 4 KiB columns each;
// it walks the columns, computing and storing the outputs exactly as
// ecg_mm_kernel does, and folds each thread's 16-byte output piece into a
// per-row Horner CRC (acc = shift_4KiB(acc) ^ crc(piece)).  At the end of an
// item every thread multiplies by its kh entry (moves its pieces to the end
// of the chunk, undoes a ragged last chunk's zero padding), the waves
// XOR-reduce and XOR their values into the zeroed checksum.  Cutting a
// chunk into several items keeps one workgroup from walking a whole 32 KiB+
// chunk serially (tools/tune8.py: ~4 columns per workgroup is best).
// The outputs are never re-read from HBM: the checksum costs LDS lookups on
// p/(k+p) of the traffic instead of a second pass over the regenerated
// cells (ref:src/object/srv_obj_migrate.c:1156 checksums them after encode).
template <int K, int R, int W, bool REFL, int TB = 0>
__global__ void __launch_bounds__(BLOCK, ECG_FUSED_WPE(W))
ecg_mm_csum_kernel(const ecg_mm_params_t P, const ecg_mmcs_params_t Q)
{
	using T = typename ecg_crc::reg<W>::T;
	constexpr int UF = ECG_MMCS_P5U;
	using F5 = ecg_crc::f5u<W, UF>;
	constexpr int NB = W / 8;
	constexpr int KM = K ? K : ECG_KMAX_K;
	constexpr int RM = R ? R : ECG_KMAX_R;
	constexpr bool PF = K != 0 && K <= ECG_FUSED_PF_MAXK && (ECG_FUSED_PF64 || W != 64);	// prefetch: 4*KM more VGPRs
	constexpr bool DEFER = (ECG_FUSED_DEFER & (W == 64 ? 2 : 1)) != 0;	// fold one column late
	constexpr int T2V = (RM + 3) / 4;
	constexpr int PER_J = RM + T2V;
	__shared__ u32x4 s_tbl[KM * PER_J];
	// CRC tables (TB): 0 5-bit (conflict-free, ecg_kabi.h: positional p5 of
	// 0..U-1 columns + a5 shift by U columns, U = ECG_CSUM_P5U); 1 byte
	// tables sl (slice-by-NB, register folded) + the a5 4 KiB shift; 2 byte tables s16 (16
	// independent lookups per piece) + the a5 shift
	// 4 nibble tables q4 of the first FQ4 positions (4 KiB stride): a piece is
	// 32 conflict-free lookups, and an item of exactly FQ4 full columns takes
	// each column's position from the unrolled walk (no register shift)
	constexpr int FQ4 = 4;
	constexpr int NSL = TB == 0 ? F5::N : TB == 1 ? NB * 256 : TB == 4 ? FQ4 * ECG_CSUM_NQ4 : 16 * 256;
	__shared__ T s_sl[NSL];
	// TB 1/2: the column shift as 5-bit a5 tables; TB 3/4: as nibble a4 tables
	__shared__ T s_sh[TB >= 3 ? 16 * 16 : TB ? ECG_CSUM_NA5(NB) * 32 : 1];
	__shared__ T s_r4[REFL ? 16 : 1];		// reflected: 4-bit reduction of the lane multiply
	__shared__ T s_nibl[REFL ? 16 * 64 : 1];	// reflected: the lane factors' nibble tables
	const int k = K ? K : (int)P.k;
	const int rows = R ? R : (int)P.rows;
	const uint64_t C = P.cell_bytes;
	const uint32_t lo = threadIdx.x * 16u;
	const T *gt = (const T *)Q.tbl;
	const T *kh = (const T *)Q.kh;
	const T poly = (T)Q.poly;

	// Prologue.  The tables are staged in two phases around the first
	// column's HBM loads: every entry this thread stages is loaded into
	// registers (L2 hits), then the workgroup's first item's first column is
	// requested, then the entries are written to LDS -- vmcnt counts in issue
	// order, so the writes wait only for the table loads and the staging and
	// barrier run in the shadow of the first HBM round trip (a workgroup
	// normally owns exactly one item).
	constexpr int P5 = ECG_CSUM_NF5 * 32;
	constexpr int NSH = TB >= 3 ? 16 * 16 : TB ? ECG_CSUM_NA5(NB) * 32 : 0;
	constexpr int NNB = REFL ? 16 * 64 + 16 : 0;		// nibl, then r4
	constexpr int NST = NSL + NSH + NNB;
	constexpr int QST = (NST + BLOCK - 1) / BLOCK;
	static_assert(KM * RM <= BLOCK, "one product-table entry per thread");
	auto st_src = [&](int i) -> int {		// entry i of the staged image -> index in gt
		if (i < NSL) {
			if constexpr (TB == 0)
				return i < P5 ? ECG_CSUM_OFF_P5(NB) + i
				     : i < UF * P5 ? ECG_CSUM_OFF_P5X_4K(NB) + i - P5 : ECG_CSUM_OFF_A5_32K(NB) + i - UF * P5;
			else
				return (TB == 1 ? 0 : TB == 4 ? ECG_CSUM_OFF_Q4_4K(NB) : ECG_CSUM_OFF_S16(NB)) + i;
		}
		i -= NSL;
		if (i < NSH)
			return (TB >= 3 ? ECG_CSUM_OFF_A4_4K(NB) : ECG_CSUM_OFF_A5_4K(NB)) + i;
		i -= NSH;
		return i < 16 * 64 ? ECG_CSUM_OFF_NIBL(NB) + i : ECG_CSUM_OFF_R4(NB) + i - 16 * 64;
	};
	auto st_dst = [&](int i) -> T * {
		if (i < NSL)
			return &s_sl[i];
		i -= NSL;
		if (i < NSH)
			return &s_sh[i];
		i -= NSH;
		return i < 16 * 64 ? &s_nibl[i] : &s_r4[i - 16 * 64];
	};
	T sv[QST];
#pragma unroll
	for (int q = 0; q < QST; q++)
		if (q * BLOCK + (int)threadIdx.x < NST)
			sv[q] = gt[st_src(q * BLOCK + (int)threadIdx.x)];
	const int tj = (int)threadIdx.x / RM, tr = (int)threadIdx.x % RM;
	const bool tst = (int)threadIdx.x < KM * RM && tj < k && tr < rows;
	ecg_ptbl_t tv;
	if (tst)
		tv = P.tbl[tr][tj];

	// the first item's first column (unconditional, clamped: a load only
	// some paths issue makes the compiler wait for everything)
	u32x4 xa[KM];
	if constexpr (PF) {
		uint32_t c, i, col1, khrow;

		mmcs_item(Q, blockIdx.x, c, i, col1, khrow);
		const uint64_t c0 = (uint64_t)c * Q.chunk_bytes + (uint64_t)i * CHUNK_BYTES;
		mm_load_any<KM>(P, k, c0 < C ? blockIdx.y : 0u, c0 < C ? c0 : 0u, lo, xa);
	}
#pragma unroll
	for (int q = 0; q < QST; q++)
		if (q * BLOCK + (int)threadIdx.x < NST)
			*st_dst(q * BLOCK + (int)threadIdx.x) = sv[q];
	if (tst) {
		s_tbl[tj * PER_J + tr] = (u32x4){tv.t0lo, tv.t0hi, tv.t1lo, tv.t1hi};
		reinterpret_cast<uint32_t *>(&s_tbl[tj * PER_J + RM])[tr] = tv.t2;
	}
	__syncthreads();

	// One item: its 4 KiB columns in order.  With PF the next column's loads
	// are issued before this column's product, so HBM requests stay in
	// flight across it.  Live state is kept small on purpose: the crc64
	// instantiations ran out of SGPRs.
	// PRE: this is the workgroup's first item, its first column already
	// requested into xa by the prologue
	auto walk = [&](uint32_t s, uint32_t it, auto pre) {
			constexpr bool PRE = decltype(pre)::value;
			uint32_t c, i, col1, khrow;
			T crc[RM];

			mmcs_item(Q, it, c, i, col1, khrow);
			const uint64_t c0 = (uint64_t)c * Q.chunk_bytes;
			// reflected: this wave's item factor as W bit-products, lane b
			// holding e_b * f(item row, wave) (ecg_csum.c fused_kh); loaded
			// now, used after the walk -- its latency hides behind the walk
			T kbv = 0;
			if constexpr (REFL) {
				const uint32_t lane = threadIdx.x & 63u;
				const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

				if (lane < (uint32_t)W)
					kbv = kh[((size_t)khrow * 4u + wv) * 64u + lane];
			}
#pragma unroll
			for (int r = 0; r < RM; r++)
				crc[r] = 0;
			// Pipelined pairs of full columns, the prefetch buffers swapping
			// roles (a register copy xa = xb would wait for the prefetched loads
			// and serialise the walk); then the rest -- an odd full column, the
			// partial column of a cell that is not a multiple of 4 KiB -- one at
			// a time without prefetch, outside the pipelined loop so that loop
			// has a single path (a path that skips loads or stores makes the
			// compiler wait for everything at the loop head).  (Walking an
			// item's columns rotated, so concurrently running items stream
			// different address residues, measured no better:
			// profiles/r02/fused_libs/rotation.json.)
			const uint64_t nfull = (C - c0) / CHUNK_BYTES;
			const uint32_t ifull = nfull < col1 ? (uint32_t)nfull : col1;
			// DEFER: each column's fold runs one column late (mmcs_pend);
			// the zero state folds to nothing on the zero register
			mmcs_pend<RM> pd;
			constexpr int D1 = DEFER ? 1 : 0;	// steady state
			constexpr int D2 = DEFER ? 2 : 0;	// a walk's first column
			bool tb4done = false;
#pragma unroll
			for (int r = 0; r < RM; r++)
				pd.v[r] = (u32x4){0, 0, 0, 0};
			pd.have = pd.first = pd.gshift = false;
			pd.pos = 0;
			if constexpr (TB == 4 && PF) {
				// an item of exactly FQ4 full columns: positions FQ4-1 .. 0
				// as constants, the prefetch buffers alternating
				if (col1 - i == FQ4 && ifull == col1) {
					u32x4 xb[KM];
					const uint64_t cb = c0 + (uint64_t)i * CHUNK_BYTES;

					if constexpr (!PRE)
						mm_load_any<KM>(P, k, s, cb, lo, xa);
					mmcs_col<KM, RM, W, REFL, TB, true, CHUNK_BYTES, true, UF, 3, D2>(
						P, s_tbl, s_sl, s_sh, k, rows, s, cb, cb + CHUNK_BYTES, lo, true,
						i == 0 && threadIdx.x == 0, Q.init, 0, false, xa, xb, crc, &pd);
					mmcs_col<KM, RM, W, REFL, TB, true, CHUNK_BYTES, true, UF, 2, D1, 3>(
						P, s_tbl, s_sl, s_sh, k, rows, s, cb + CHUNK_BYTES, cb + 2 * CHUNK_BYTES, lo, true,
						false, Q.init, 0, false, xb, xa, crc, &pd);
					mmcs_col<KM, RM, W, REFL, TB, true, CHUNK_BYTES, true, UF, 1, D1, 2>(
						P, s_tbl, s_sl, s_sh, k, rows, s, cb + 2 * CHUNK_BYTES, cb + 3 * CHUNK_BYTES, lo, true,
						false, Q.init, 0, false, xa, xb, crc, &pd);
					mmcs_col<KM, RM, W, REFL, TB, true, CHUNK_BYTES, true, UF, 0, D1, 1>(
						P, s_tbl, s_sl, s_sh, k, rows, s, cb + 3 * CHUNK_BYTES, 0, lo, false,
						false, Q.init, 0, false, xb, xa, crc, &pd);
					if constexpr (DEFER)
						mmcs_fold<RM, W, REFL, TB, UF, 0>(s_sl, s_sh, rows, pd.v, pd.have, pd.first,
										  Q.init, pd.pos, pd.gshift, crc);
					tb4done = true;
					i = col1;
				}
			}
			const uint32_t iend = ifull > i ? i + ((ifull - i) & ~1u) : i;
			if (PF && i < iend) {
				u32x4 xb[PF ? KM : 1];
				u32x4 *xc = PF ? xb : xa;

				if constexpr (!PRE)
					mm_load_any<KM>(P, k, s, c0 + (uint64_t)i * CHUNK_BYTES, lo, xa);
				if constexpr (DEFER) {
					// the first trip peeled: nothing pending at its first column
					const uint64_t cb = c0 + (uint64_t)i * CHUNK_BYTES;
					mmcs_col<KM, RM, W, REFL, TB, true, CHUNK_BYTES, true, UF, -1, D2>(
						P, s_tbl, s_sl, s_sh, k, rows, s, cb, cb + CHUNK_BYTES, lo, true,
						i == 0 && threadIdx.x == 0, Q.init, (col1 - 1 - i) % UF, true, xa, xc, crc, &pd);
					mmcs_col<KM, RM, W, REFL, TB, true, CHUNK_BYTES, true, UF, -1, D1>(
						P, s_tbl, s_sl, s_sh, k, rows, s, cb + CHUNK_BYTES, cb + 2 * CHUNK_BYTES, lo,
						i + 2 < iend, false, Q.init, (col1 - 2 - i) % UF, true, xc, xa, crc, &pd);
					i += 2;
				}
				for (; i < iend; i += 2) {
					const uint64_t cb = c0 + (uint64_t)i * CHUNK_BYTES;
					mmcs_col<KM, RM, W, REFL, TB, true, CHUNK_BYTES, true, UF, -1, D1>(
						P, s_tbl, s_sl, s_sh, k, rows, s, cb, cb + CHUNK_BYTES, lo, true,
						i == 0 && threadIdx.x == 0, Q.init, (col1 - 1 - i) % UF, true, xa, xc, crc, &pd);
					mmcs_col<KM, RM, W, REFL, TB, true, CHUNK_BYTES, true, UF, -1, D1>(
						P, s_tbl, s_sl, s_sh, k, rows, s, cb + CHUNK_BYTES, cb + 2 * CHUNK_BYTES, lo,
						i + 2 < iend, false, Q.init, (col1 - 2 - i) % UF, true, xc, xa, crc, &pd);
				}
			}
			for (; i < col1; i++)
				mmcs_col<KM, RM, W, REFL, TB, false, CHUNK_BYTES, false, UF, -1, D1>(
					P, s_tbl, s_sl, s_sh, k, rows, s, c0 + (uint64_t)i * CHUNK_BYTES, 0, lo, false,
					i == 0 && threadIdx.x == 0, Q.init, (col1 - 1 - i) % UF, true, xa, xa, crc, &pd);
			if constexpr (DEFER) {
				if (!tb4done)
					mmcs_fold<RM, W, REFL, TB, UF, -1>(s_sl, s_sh, rows, pd.v, pd.have, pd.first, Q.init,
									   pd.pos, pd.gshift, crc);
			}
			// each wave XORs its partial into the (zeroed) output: no
			// workgroup barrier, other waves keep streaming.  Reflected CRCs:
			// every lane's value is multiplied by its lane factor
			// x^(8*16*(63-l)) from the LDS nibble tables (W/4 steps), the wave
			// XOR-reduces, and the wave's sum is multiplied by the item factor
			// bit-parallel -- lane b keeps e_b * f if bit b of the sum is set,
			// one more XOR reduction.  No table read in the tail depends on
			// HBM: the r03 per-(row, wave) nibble tables in HBM cost crc64 up
			// to 30 % at 4-column items (serialised L2 round trips under the
			// streaming load, tools/fused_libs.py -DECG_EXP_NO_TAIL,
			// profiles/r03/fused_tail/).  crc16: a W-step multiply per thread.
			// The rows are finished side by side (one basic block: their
			// lookup chains and reductions interleave), reduced with DPP into
			// wave-uniform values, then lane 0 XORs them into the output.
			T v[RM];
			const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
			for (int r = 0; r < RM; r++) {
				if constexpr (REFL) {
#ifdef ECG_EXP_NO_TAIL
					v[r] = crc[r];	// experimental: no lane / item factor (wrong checksums)
#else
					v[r] = ecg_crc::lane_mul_nib<W>(crc[r], s_nibl, s_r4, lane);
#endif
				} else {
					v[r] = ecg_crc::mulmod<W, REFL>(kh[khrow * 256 + threadIdx.x], crc[r], poly);
				}
			}
#pragma unroll
			for (int r = 0; r < RM; r++)
				v[r] = ecg_crc::wave_xor_uniform(v[r]);
#if !defined(ECG_EXP_NO_TAIL)
			if constexpr (REFL) {
#pragma unroll
				for (int r = 0; r < RM; r++)
					v[r] = ecg_crc::wave_xor_uniform(((v[r] >> (lane & (uint32_t)(W - 1))) & 1u) ? kbv : (T)0);
			}
#else
			(void)kbv;
#endif
			if (lane == 0) {
#pragma unroll
				for (int r = 0; r < RM; r++) {
					if (r < rows) {
						T x = v[r];
						if (threadIdx.x == 0 && khrow == (c + 1 == Q.nch ? Q.nh : 0))
							x ^= (T)Q.xorout;	// once per chunk
						const uint64_t slot = ((uint64_t)Q.row_slot[r] * P.nstripes + s) * Q.nch + c;
						if constexpr (W == 16)
							atomicXor((uint32_t *)Q.out + slot / 2, (uint32_t)x << (16 * (slot & 1)));
						else
							atomicXor((T *)Q.out + slot, x);
					}
				}
			}
	};
	// The workgroup's work: items blockIdx.x, blockIdx.x + gridDim.x, ... of
	// stripe blockIdx.y (+ gridDim.y ...) -- the grid never exceeds the item
	// and stripe counts, so the first is always there
	walk(blockIdx.y, blockIdx.x, ecg_bool<true>{});
	for (uint32_t s = blockIdx.y; s < P.nstripes; s += gridDim.y)
		for (uint32_t it = s == blockIdx.y ? blockIdx.x + gridDim.x : blockIdx.x; it < Q.nitems; it += gridDim.x)
			walk(s, it, ecg_bool<false>{});
}

// Fused product + checksum, one WAVE per (stripe, chunk): the wave walks the
// chunk's 1 KiB rows in order (lane l: bytes 16l..16l+15 of each row, every
// load and store a coalesced 1 KiB), computes and stores the product exactly
// as ecg_mm_kernel does, and Horner-accumulates each output row's pieces
// with the 1 KiB shift.  At the chunk end each lane multiplies by
// Q.kh[last][lane] = x^(8*16*(63-lane)) (x^(-8Z) for a last chunk padded by Z
// zero bytes), the wave XOR-reduces and lane 0 stores the checksum: no
// atomics, no memset, and one W-step multiply per lane per CHUNK (32 KiB:
// 32 rows) instead of one per thread per work item of the workgroup kernel
// -- the multiply dominates crc64's cost there (tools/fused_sweep.py).
// Tables (TB as ecg_mm_csum_kernel) with the 1 KiB shift.
template <int K, int R, int W, bool REFL, int TB>
__global__ void __launch_bounds__(BLOCK, ECG_FUSED_WPE(W))
ecg_mm_csum_wave_kernel(const ecg_mm_params_t P, const ecg_mmcs_params_t Q)
{
	using T = typename ecg_crc::reg<W>::T;
	using F5 = ecg_crc::f5u<W>;
	constexpr int NB = W / 8;
	constexpr int KM = K ? K : ECG_KMAX_K;
	constexpr int RM = R ? R : ECG_KMAX_R;
	constexpr bool PF = K != 0 && K <= ECG_FUSED_PF_MAXK && (ECG_FUSED_PF64 || W != 64);	// next row's loads in flight
	constexpr int T2V = (RM + 3) / 4;
	constexpr int PER_J = RM + T2V;
	constexpr int NSL = TB == 0 ? F5::N : TB == 1 ? NB * 256 : 16 * 256;
	__shared__ u32x4 s_tbl[KM * PER_J];
	__shared__ T s_sl[NSL];
	// TB 1/2: the row shift as 5-bit a5 tables; TB 3: as nibble a4 tables
	__shared__ T s_sh[TB == 3 ? 16 * 16 : TB ? ECG_CSUM_NA5(NB) * 32 : 1];
	__shared__ T s_r4[REFL ? 16 : 1];		// reflected: 4-bit reduction of the lane multiply
	const int k = K ? K : (int)P.k;
	const int rows = R ? R : (int)P.rows;
	const uint64_t C = P.cell_bytes;
	const int lane = threadIdx.x & 63;
	const uint32_t lo = (uint32_t)lane * 16u;
	const T *gt = (const T *)Q.tbl;

	for (int i = threadIdx.x; i < KM * RM; i += BLOCK) {
		const int j = i / RM, r = i % RM;
		if (j < k && r < rows) {
			const ecg_ptbl_t &t = P.tbl[r][j];
			s_tbl[j * PER_J + r] = (u32x4){t.t0lo, t.t0hi, t.t1lo, t.t1hi};
			reinterpret_cast<uint32_t *>(&s_tbl[j * PER_J + RM])[r] = t.t2;
		}
	}
	if constexpr (TB != 0) {
		for (int i = threadIdx.x; i < NSL; i += BLOCK)
			s_sl[i] = gt[(TB == 1 ? 0 : ECG_CSUM_OFF_S16(NB)) + i];
		if constexpr (TB == 3)
			for (int i = threadIdx.x; i < 16 * 16; i += BLOCK)
				s_sh[i] = gt[ECG_CSUM_OFF_A4_1K(NB) + i];
		else
			for (int i = threadIdx.x; i < ECG_CSUM_NA5(NB) * 32; i += BLOCK)
				s_sh[i] = gt[ECG_CSUM_OFF_A5_1K(NB) + i];
	} else {
		ecg_crc::stage5u<W>(s_sl, gt, ECG_CSUM_OFF_P5X_1K(NB), ECG_CSUM_OFF_A5_4K(NB), BLOCK);
	}
	__shared__ T s_nibl[REFL ? 16 * 64 : 1];	// reflected: the lane factors' nibble tables
	const T *kw = (const T *)Q.kh;
	if constexpr (REFL) {
		if (threadIdx.x < 16)
			s_r4[threadIdx.x] = gt[ECG_CSUM_OFF_R4(NB) + threadIdx.x];
		for (int i = threadIdx.x; i < 16 * 64; i += BLOCK)
			s_nibl[i] = gt[ECG_CSUM_OFF_NIBL(NB) + i];
	}
	const T poly = (T)Q.poly;
	__syncthreads();

	const uint64_t total = (uint64_t)P.nstripes * Q.nch;
	// the wave index is wave-uniform: readfirstlane keeps the item's offsets
	// in SGPRs (mm_load / mm_compute require it)
	const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	for (uint64_t g = (uint64_t)blockIdx.x * (BLOCK / 64) + wv; g < total;
	     g += (uint64_t)gridDim.x * (BLOCK / 64)) {
		const uint32_t s = (uint32_t)(g / Q.nch), c = (uint32_t)(g - (uint64_t)s * Q.nch);
		const bool lastc = c + 1 == Q.nch;
		const uint64_t c0 = (uint64_t)c * Q.chunk_bytes;
		const uint64_t len = lastc ? C - c0 : Q.chunk_bytes;
		const uint32_t m = (uint32_t)((len + ECG_CSUM_STRIDE - 1) / ECG_CSUM_STRIDE);
		T crc[RM];
		u32x4 xa[KM];
		// reflected, last chunk of a cell: the zero padding's inverse shift
		// x^(-8Z) as W bit-products (lane b: e_b * x^(-8Z)), loaded now and
		// used after the walk; crc16: the lane's multiplier
		const T kcur = REFL ? (lastc && lane < W ? kw[lane] : (T)0) : kw[(lastc ? 64 : 0) + lane];

#pragma unroll
		for (int r = 0; r < RM; r++)
			crc[r] = 0;
		// pipelined pairs of full rows, then the rest one at a time (as
		// ecg_mm_csum_kernel)
		const uint32_t mfull = (uint32_t)(len / ECG_CSUM_STRIDE);
		const uint32_t iend = mfull & ~1u;
		uint32_t i = 0;
		if (PF && iend) {
			u32x4 xb[PF ? KM : 1];
			u32x4 *xc = PF ? xb : xa;

			mm_load_any<KM>(P, k, s, c0, lo, xa);
			for (; i < iend; i += 2) {
				const uint64_t cb = c0 + (uint64_t)i * ECG_CSUM_STRIDE;
				mmcs_col<KM, RM, W, REFL, TB, true, ECG_CSUM_STRIDE, true, F5::U>(
					P, s_tbl, s_sl, s_sh, k, rows, s, cb, cb + ECG_CSUM_STRIDE, lo, true,
					i == 0 && lane == 0, Q.init, (m - 1 - i) % F5::U, true, xa, xc, crc);
				mmcs_col<KM, RM, W, REFL, TB, true, ECG_CSUM_STRIDE, true, F5::U>(
					P, s_tbl, s_sl, s_sh, k, rows, s, cb + ECG_CSUM_STRIDE, cb + 2 * ECG_CSUM_STRIDE, lo,
					i + 2 < iend, false, Q.init, (m - 2 - i) % F5::U, true, xc, xa, crc);
			}
		}
		for (; i < m; i++)
			mmcs_col<KM, RM, W, REFL, TB, false, ECG_CSUM_STRIDE, false, F5::U>(
				P, s_tbl, s_sl, s_sh, k, rows, s, c0 + (uint64_t)i * ECG_CSUM_STRIDE, 0, lo, false,
				i == 0 && lane == 0, Q.init, (m - 1 - i) % F5::U, true, xa, xa, crc);
		// reflected: the lane factor x^(8*16*(63-l)) from the LDS nibble
		// tables (W/4 steps), the wave XOR-reduces, a last chunk's sum is
		// multiplied by x^(-8Z) bit-parallel (ecg_csum.c fused_kw); crc16: a
		// W-step multiply per lane by Q.kh[2][64]
		T v[RM];
#pragma unroll
		for (int r = 0; r < RM; r++)
			v[r] = REFL ? ecg_crc::lane_mul_nib<W>(crc[r], s_nibl, s_r4, (uint32_t)lane)
				    : ecg_crc::mulmod<W, REFL>(kcur, crc[r], poly);
#pragma unroll
		for (int r = 0; r < RM; r++)
			v[r] = ecg_crc::wave_xor_uniform(v[r]);
		if (REFL && lastc) {
#pragma unroll
			for (int r = 0; r < RM; r++)
				v[r] = ecg_crc::wave_xor_uniform(((v[r] >> ((uint32_t)lane & (uint32_t)(W - 1))) & 1u) ? kcur
													  : (T)0);
		}
#pragma unroll
		for (int r = 0; r < RM; r++) {
			if (r < rows) {
				if (lane == 0) {
					const uint64_t slot = ((uint64_t)Q.row_slot[r] * P.nstripes + s) * Q.nch + c;
					const T x = v[r] ^ (T)Q.xorout;
					if constexpr (W == 16)
						((uint16_t *)Q.out)[slot] = (uint16_t)x;
					else
						((T *)Q.out)[slot] = x;
				}
			}
		}
	}
}

template <int KM, int RM>
__device__ __forceinline__ void mm_ptr_item(const ecg_mm_params_t &P, const u32x4 *tb, int k, int rows,
					    uint32_t s, uint64_t cbase, uint32_t lo, const uint64_t *a)
{
	u32x4 x[KM], outv[RM];

#pragma unroll
	for (int j = 0; j < KM; j++)
		if (j < k)
			x[j] = ld_nt(reinterpret_cast<const uint8_t *>(a[j]) + lo);
	mm_compute<KM, RM, false, true, false>(P, tb, k, rows, s, cbase, lo, x, outv);
#pragma unroll
	for (int r = 0; r < RM; r++)
		if (r < rows)
			st_nt(reinterpret_cast<uint8_t *>(a[KM + r]) + lo, outv[r]);
}

// Pointer-table product (ISA-L's data[]/coding[] convention batched over
// stripes): cells[s*(k+rows) + j] is the device address of input cell j (j < k)
// or output cell j-k of stripe s.  Same columns, tables and arithmetic as
// ecg_mm_kernel; a stripe's k+rows addresses are wave-uniform (scalar loads).
template <int K, int R>
__global__ void __launch_bounds__(BLOCK)
ecg_mm_ptr_kernel(const ecg_mm_params_t P, const uint64_t *__restrict__ cells)
{
	constexpr int KM = K ? K : ECG_KMAX_K;
	constexpr int RM = R ? R : ECG_KMAX_R;
	constexpr int T2V = (RM + 3) / 4;
	constexpr int PER_J = RM + T2V;
	__shared__ u32x4 s_tbl[KM * PER_J];
	const int k = K ? K : (int)P.k;
	const int rows = R ? R : (int)P.rows;
	const uint64_t C = P.cell_bytes;
	const uint32_t nchunk = (uint32_t)((C + CHUNK_BYTES - 1) / CHUNK_BYTES);
	const uint32_t lo = threadIdx.x * 16u;

	for (int i = threadIdx.x; i < KM * RM; i += BLOCK) {
		const int j = i / RM, r = i % RM;
		if (j < k && r < rows) {
			const ecg_ptbl_t &t = P.tbl[r][j];
			s_tbl[j * PER_J + r] = (u32x4){t.t0lo, t.t0hi, t.t1lo, t.t1hi};
			reinterpret_cast<uint32_t *>(&s_tbl[j * PER_J + RM])[r] = t.t2;
		}
	}
	__syncthreads();

	for (uint32_t s = blockIdx.y; s < P.nstripes; s += gridDim.y) {
		const uint64_t *pt = cells + (uint64_t)s * (uint32_t)(k + rows);
		uint64_t base[KM + RM];

		// the stripe's addresses: one dependent (scalar) load per stripe, not
		// per column -- the workgroup then walks several columns
#pragma unroll
		for (int j = 0; j < KM + RM; j++)
			if (j < k || (j >= KM && j - KM < rows))
				base[j] = pt[j < KM ? j : k + (j - KM)];
		for (uint32_t ch = blockIdx.x; ch < nchunk; ch += gridDim.x) {
			const uint64_t cbase = (uint64_t)ch * CHUNK_BYTES;
			uint64_t a[KM + RM];
			uint32_t z = 0;

#pragma unroll
			for (int j = 0; j < KM + RM; j++) {
				if (j < k || (j >= KM && j - KM < rows)) {
					a[j] = base[j] + cbase;
					asm volatile("" : "+s"(a[j]));
				}
			}
			asm volatile("" : "+v"(z));
			const u32x4 *tb = s_tbl + z;
			if (cbase + CHUNK_BYTES <= C)
				mm_ptr_item<KM, RM>(P, tb, k, rows, s, cbase, lo, a);
			else if (cbase + lo + 16 <= C)	// C % 16 == 0 on this path
				mm_ptr_item<KM, RM>(P, tb, k, rows, s, cbase, lo, a);
		}
	}
}

// Pointer-table product, any alignment and length: one byte per lane.
__global__ void __launch_bounds__(BLOCK)
ecg_mm_ptr_byte_kernel(const ecg_mm_params_t P, const uint64_t *cells)
{
	const uint64_t C = P.cell_bytes;
	const uint64_t total = C * P.nstripes;
	const int k = (int)P.k, rows = (int)P.rows;

	for (uint64_t e = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; e < total;
	     e += (uint64_t)gridDim.x * BLOCK) {
		const uint64_t s = e / C, i = e % C;
		const uint64_t *pt = cells + s * (uint64_t)(k + rows);
		uint8_t o[ECG_KMAX_R];

		for (int r = 0; r < ECG_KMAX_R; r++)
			o[r] = 0;
		for (int j = 0; j < k; j++) {
			const uint32_t v = reinterpret_cast<const uint8_t *>(pt[j])[i];
			for (int r = 0; r < rows; r++)
				o[r] ^= gf_mul1(P.tbl[r][j], v);
		}
		for (int r = 0; r < rows; r++)
			reinterpret_cast<uint8_t *>(pt[k + r])[i] = o[r];
	}
}

// Any alignment, any length: one byte per lane-iteration.  Used only when a
// caller hands cell bases/strides that are not 16-byte aligned.
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
	int k, r, acc, diff;
	mm_fn_t fn;
	const char *name;
};

#define KE(K_, R_, A_, D_) \
	{K_, R_, A_, D_, ecg_mm_kernel<K_, R_, (bool)A_, (bool)D_>, \
	 "ecg_mm_kernel<" #K_ "," #R_ "," #A_ "," #D_ ">"}


// Specialised shapes: every (k, p) of the DAOS EC classes
// (ref:src/include/daos_obj_class.h:70-80): k in {2,4,8,16}, rows in 1..3
// (encode rows = p; recovery rows = nerrs <= p).  Everything else runs the
// runtime-shaped instantiation (K = R = 0).
static const kentry g_kernels[] = {
	KE(2, 1, 0, 0), KE(2, 2, 0, 0), KE(2, 3, 0, 0),
	KE(4, 1, 0, 0), KE(4, 2, 0, 0), KE(4, 3, 0, 0),
	KE(8, 1, 0, 0), KE(8, 2, 0, 0), KE(8, 3, 0, 0),
	KE(16, 1, 0, 0), KE(16, 2, 0, 0), KE(16, 3, 0, 0),
	KE(0, 0, 0, 0), KE(0, 0, 1, 0), KE(0, 0, 0, 1), KE(0, 0, 1, 1),
};
#define N_KERNELS ((uint32_t)(sizeof(g_kernels) / sizeof(g_kernels[0])))




typedef void (*mmcs_fn_t)(const ecg_mm_params_t, const ecg_mmcs_params_t);

struct csentry {
	int k, r, type;
	mmcs_fn_t fn;
	const char *name;
	int b8;		/* CRC table kind TB of the instantiation */
};

#define CSE(K_, R_, T_, W_, RF_, N_) \
	{K_, R_, T_, ecg_mm_csum_kernel<K_, R_, W_, RF_, W_ == 64 ? 1 : 0>, "ecg_mm_csum_kernel<" #K_ "," #R_ "," N_ ">", \
	 W_ == 64 ? 1 : 0}
#define CSE3(K_, R_) CSE(K_, R_, 1, 16, false, "crc16"), CSE(K_, R_, 2, 32, true, "crc32"), \
		     CSE(K_, R_, 3, 64, true, "crc64")

/* the other table kind than the default (crc16/crc32 5-bit, crc64 byte tables) */
#define CSB(K_, R_, T_, W_, RF_, N_, TB_) \
	{K_, R_, T_, ecg_mm_csum_kernel<K_, R_, W_, RF_, TB_>, \
	 "ecg_mm_csum_kernel<" #K_ "," #R_ "," N_ ",tb" #TB_ ">", TB_}

static const csentry g_cskernels[] = {
	CSE3(2, 1), CSE3(2, 2), CSE3(2, 3), CSE3(4, 1), CSE3(4, 2), CSE3(4, 3),
	CSE3(8, 1), CSE3(8, 2), CSE3(8, 3), CSE3(16, 1), CSE3(16, 2), CSE3(16, 3),
	CSE3(0, 0),
	/* the other table kind, A/B measurements only (ecg_set_csum_variant bits 4/5) */
	CSB(8, 2, 2, 32, true, "crc32", 1), CSB(8, 2, 2, 32, true, "crc32", 2), CSB(8, 2, 3, 64, true, "crc64", 0),
	CSB(8, 2, 3, 64, true, "crc64", 2), CSB(4, 2, 2, 32, true, "crc32", 2), CSB(4, 2, 3, 64, true, "crc64", 2),
	CSB(8, 1, 2, 32, true, "crc32", 2),
	/* TB 4: positional nibble tables (4 KiB stride, 4 positions) + nibble a4 column shift */
	CSB(8, 2, 2, 32, true, "crc32", 4), CSB(8, 2, 3, 64, true, "crc64", 4), CSB(4, 2, 2, 32, true, "crc32", 4),
	CSB(4, 2, 3, 64, true, "crc64", 4), CSB(8, 1, 2, 32, true, "crc32", 4), CSB(8, 1, 3, 64, true, "crc64", 4),
	CSB(16, 2, 2, 32, true, "crc32", 4), CSB(16, 2, 3, 64, true, "crc64", 4),
	CSB(8, 3, 2, 32, true, "crc32", 4), CSB(8, 3, 3, 64, true, "crc64", 4),
	/* TB 3: s16 byte tables with SDWA addresses + nibble a4 column shift */
	CSB(8, 2, 2, 32, true, "crc32", 3), CSB(8, 2, 3, 64, true, "crc64", 3), CSB(4, 2, 2, 32, true, "crc32", 3),
	CSB(4, 2, 3, 64, true, "crc64", 3), CSB(8, 1, 2, 32, true, "crc32", 3), CSB(16, 2, 2, 32, true, "crc32", 3),
	CSB(8, 3, 2, 32, true, "crc32", 3), CSB(4, 1, 2, 32, true, "crc32", 3), CSB(16, 1, 2, 32, true, "crc32", 3),
};
#define N_CSKERNELS ((uint32_t)(sizeof(g_cskernels) / sizeof(g_cskernels[0])))

#define CSW(K_, R_, T_, W_, RF_, N_) \
	{K_, R_, T_, ecg_mm_csum_wave_kernel<K_, R_, W_, RF_, W_ == 64 ? 1 : 0>, \
	 "ecg_mm_csum_wave_kernel<" #K_ "," #R_ "," N_ ">", W_ == 64 ? 1 : 0}
#define CSW3(K_, R_) CSW(K_, R_, 1, 16, false, "crc16"), CSW(K_, R_, 2, 32, true, "crc32"), \
		     CSW(K_, R_, 3, 64, true, "crc64")

static const csentry g_cswkernels[] = {
	CSW3(2, 1), CSW3(4, 2), CSW3(8, 1), CSW3(8, 2), CSW3(16, 2), CSW3(0, 0),
	/* the default path for crc64 with k <= 4 (ecg_csum.c) */
	CSW(2, 2, 3, 64, true, "crc64"), CSW(2, 3, 3, 64, true, "crc64"), CSW(4, 1, 3, 64, true, "crc64"),
	CSW(4, 3, 3, 64, true, "crc64"),
};
#define N_CSWKERNELS ((uint32_t)(sizeof(g_cswkernels) / sizeof(g_cswkernels[0])))
#define KID_FUSED_WAVE 800u
#define KID_FUSED 500u		/* fused kernel ids: KID_FUSED + index */

typedef void (*mmptr_fn_t)(const ecg_mm_params_t, const uint64_t *);

struct pentry {
	int k, r;
	mmptr_fn_t fn;
	const char *name;
};

#define PE(K_, R_) {K_, R_, ecg_mm_ptr_kernel<K_, R_>, "ecg_mm_ptr_kernel<" #K_ "," #R_ ">"}

static const pentry g_pkernels[] = {
	PE(2, 1), PE(2, 2), PE(2, 3), PE(4, 1), PE(4, 2), PE(4, 3),
	PE(8, 1), PE(8, 2), PE(8, 3), PE(16, 1), PE(16, 2), PE(16, 3), PE(0, 0),
};
#define N_PKERNELS ((uint32_t)(sizeof(g_pkernels) / sizeof(g_pkernels[0])))
#define KID_PTR 600u		/* pointer-table kernel ids: KID_PTR + index */
#define KID_PTR_BYTE (KID_PTR + N_PKERNELS)

#define KID_SEL 700u		/* per-stripe column kernels: <1>, <2>, <0> */

#define KID_BYTE N_KERNELS
#define KID_COPY (N_KERNELS + 1)
#define KID_READ (N_KERNELS + 2)
#define KID_WRITE (N_KERNELS + 3)

static bool aligned16(const ecg_mm_params_t *p)
{
	uint64_t bits = (uint64_t)(uintptr_t)p->src | (uint64_t)(uintptr_t)p->dst |
			(uint64_t)p->src_stripe_stride | (uint64_t)p->dst_stripe_stride;
	for (uint32_t j = 0; j < p->k; j++) {
		bits |= (uint64_t)p->src_cell_off[j];
		if (p->diff)
			bits |= (uint64_t)p->src2_cell_off[j];
	}
	if (p->diff)
		bits |= (uint64_t)(uintptr_t)p->src2 | (uint64_t)p->src2_stripe_stride;
	for (uint32_t r = 0; r < p->rows; r++)
		bits |= (uint64_t)p->dst_cell_off[r];
	return (bits & 15u) == 0;
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
	if (id >= KID_FUSED && id < KID_FUSED + N_CSKERNELS)
		return g_cskernels[id - KID_FUSED].name;
	if (id >= KID_FUSED_WAVE && id < KID_FUSED_WAVE + N_CSWKERNELS)
		return g_cswkernels[id - KID_FUSED_WAVE].name;
	if (id >= KID_PTR && id < KID_PTR + N_PKERNELS)
		return g_pkernels[id - KID_PTR].name;
	if (id == KID_PTR_BYTE)
		return "ecg_mm_ptr_byte_kernel";
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

// Blocks per CU of the product kernel's 2D grid (ecg_set_wg_per_cu; 0 =
// none).  A block streams k + rows cells at once (one 4 KiB column of each);
// with every block the registers allow resident, wide stripes keep so many
// cell streams in flight that HBM efficiency drops.  Swept over the EC
// classes (tools/wg_cap_sweep.py, profiles/r02/wg_cap/, caps interleaved
// launch by launch): k = 16 best at 2 blocks per CU (encode +3-10 %, decode
// +2-7 % over the register limit of 4), k = 8 at 3 (+1-5 %), k <= 4 uncapped
// (any cap <= 4 loses).  Timed back to back as bench.py does, the gain does
// not hold: k = 16 at 2 blocks per CU +2 % on one box and -4..-6 % on
// another, k = 8 at 3 -2..-4 % (bench_wg*.log), so no shape is capped by
// default; the knob stays for A/B runs.  A default cap would apply only to
// launches of more than 2048 blocks (a smaller grid is latency-bound).
__host__ static uint32_t mm_wg_cap(const ecg_mm_params_t *p, const ecg_launch_cfg_t *cfg, uint64_t blocks)
{
	const uint32_t c = cfg ? cfg->wg_per_cu : 0;

	if (c == ECG_WG_UNCAPPED)
		return 0;
	if (c)
		return c < 2 ? 2 : c;
	return blocks > 2048 ? ECG_MM_WG_DEFAULT(p->k + p->rows) : 0u;
}

// Unused dynamic LDS that leaves room for exactly `cap` blocks per CU (160 KiB
// of LDS; a block may take at most 64 KiB, so cap >= 2).
__host__ static size_t mm_dyn_lds(uint32_t cap, int k, int r)
{
	const int km = k ? k : ECG_KMAX_K, rm = r ? r : ECG_KMAX_R;
	const size_t stat = (size_t)km * (rm + (rm + 3) / 4) * 16;	// ecg_mm_kernel's s_tbl
	size_t d;

	if (cap == 0)
		return ECG_EXP_DYN_LDS;
	d = (size_t)(163840.0 / (cap + 0.5));
	if (d > 65536)
		d = 65536;
	return d > stat ? (d - stat) & ~(size_t)255 : 0;
}

extern "C" int ecg_k_launch_matmul(const ecg_mm_params_t *p, const ecg_launch_cfg_t *cfg,
				   void *stream, uint32_t *kernel_id)
{
	hipStream_t st = (hipStream_t)stream;
	const uint32_t variant = cfg ? cfg->variant : 0;
	const uint64_t nchunk = (p->cell_bytes + CHUNK_BYTES - 1) / CHUNK_BYTES;

	if (p->nstripes == 0 || p->cell_bytes == 0 || p->rows == 0)
		return (int)hipSuccess;

	if (variant == 2 || !aligned16(p)) {
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
	if (variant != 1 && !p->accumulate && !p->diff) {
		for (uint32_t i = 0; i < N_KERNELS; i++)
			if (g_kernels[i].k == (int)p->k && g_kernels[i].r == (int)p->rows &&
			    !g_kernels[i].acc && !g_kernels[i].diff) {
				id = i;
				break;
			}
	}
	if (id == N_KERNELS) {
		for (uint32_t i = 0; i < N_KERNELS; i++)
			if (g_kernels[i].k == 0 && g_kernels[i].acc == (int)(p->accumulate != 0) &&
			    g_kernels[i].diff == (int)(p->diff != 0)) {
				id = i;
				break;
			}
	}

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

extern "C" int ecg_k_launch_matmul_csum(const ecg_mm_params_t *p, const ecg_mmcs_params_t *q,
				       const ecg_launch_cfg_t *cfg, void *stream, uint32_t *kernel_id)
{
	uint32_t id = N_CSKERNELS;

	if (p->nstripes == 0 || p->cell_bytes == 0 || p->rows == 0)
		return (int)hipSuccess;
	if (!aligned16(p) || p->accumulate || p->diff || (p->cell_bytes & 15u) ||
	    (q->chunk_bytes % CHUNK_BYTES) || q->chunk_bytes == 0)
		return 1;
	if (q->wave) {
		const csentry *tab = g_cswkernels;
		uint32_t n = N_CSWKERNELS, w = n;

		for (uint32_t i = 0; i < n && w == n; i++)
			if (tab[i].type == (int)q->type && tab[i].k == (int)p->k && tab[i].r == (int)p->rows &&
			    tab[i].b8 == (int)q->byte_tables)
				w = i;
		for (uint32_t i = 0; i < n && w == n; i++)
			if (tab[i].type == (int)q->type && tab[i].k == 0 && tab[i].b8 == (int)q->byte_tables)
				w = i;
		if (w == n || q->kh == nullptr)	// no instantiation (not 1: that means "two-pass")
			return (int)hipErrorInvalidDeviceFunction;
		const uint64_t items = (uint64_t)p->nstripes * q->nch;
		uint64_t gx = (items + BLOCK / 64 - 1) / (BLOCK / 64);
		if (cfg && cfg->grid_x)
			gx = cfg->grid_x;
		if (gx > 0x7fffffffu)
			gx = 0x7fffffffu;
		hipLaunchKernelGGL(tab[w].fn, dim3((uint32_t)gx), dim3(BLOCK), 0, (hipStream_t)stream, *p, *q);
		if (kernel_id)
			*kernel_id = KID_FUSED_WAVE + w;
		return (int)hipGetLastError();
	}
	for (uint32_t i = 0; i < N_CSKERNELS; i++)
		if (g_cskernels[i].type == (int)q->type && g_cskernels[i].k == (int)p->k &&
		    g_cskernels[i].r == (int)p->rows && g_cskernels[i].b8 == (int)q->byte_tables) {
			id = i;
			break;
		}
	if (id == N_CSKERNELS)
		for (uint32_t i = 0; i < N_CSKERNELS; i++)
			if (g_cskernels[i].type == (int)q->type && g_cskernels[i].k == 0 &&
			    g_cskernels[i].b8 == (int)q->byte_tables) {
				id = i;
				break;
			}
	if (id == N_CSKERNELS)			// no instantiation (not 1: that means "two-pass")
		return (int)hipErrorInvalidDeviceFunction;
	if (q->nitems == 0 || q->ncols == 0 || q->kh == nullptr)
		return (int)hipErrorInvalidDeviceFunction;
	// default: ~16 KiB of columns per workgroup (tools/tune8.py,
	// profiles/r01/tune8_fused_chunks.json: walking more columns per
	// workgroup loses HBM parallelism, fewer pays a reduction per column);
	// one-column items (4 KiB chunks) 8 per workgroup, two-column items 2,
	// longer items one per workgroup
	const uint64_t ipb = q->ncols == 1 ? 8 : q->ncols == 2 ? 2 : 1;
	uint32_t gx = cfg && cfg->grid_x ? cfg->grid_x : (uint32_t)((q->nitems + ipb - 1) / ipb);
	uint32_t gy = cfg && cfg->grid_y ? cfg->grid_y : (p->nstripes < 65535 ? p->nstripes : 65535);
	if (gx > 65535)
		gx = 65535;
	hipLaunchKernelGGL(g_cskernels[id].fn, dim3(gx, gy), dim3(BLOCK), 0, (hipStream_t)stream, *p, *q);
	if (kernel_id)
		*kernel_id = KID_FUSED + id;
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

extern "C" int ecg_k_launch_matmul_ptrs(const ecg_mm_params_t *p, const uint64_t *cells_dev,
				       int aligned, const ecg_launch_cfg_t *cfg, void *stream,
				       uint32_t *kernel_id)
{
	hipStream_t st = (hipStream_t)stream;
	const uint64_t nchunk = (p->cell_bytes + CHUNK_BYTES - 1) / CHUNK_BYTES;
	uint32_t id = N_PKERNELS;

	if (p->nstripes == 0 || p->cell_bytes == 0 || p->rows == 0)
		return (int)hipSuccess;
	if (!aligned || (p->cell_bytes & 15u) || (cfg && cfg->variant == 2)) {
		uint64_t blocks = (p->cell_bytes * p->nstripes + BLOCK - 1) / BLOCK;
		if (blocks > 8192)
			blocks = 8192;
		hipLaunchKernelGGL(ecg_mm_ptr_byte_kernel, dim3((uint32_t)blocks), dim3(BLOCK), 0, st, *p,
				   cells_dev);
		if (kernel_id)
			*kernel_id = KID_PTR_BYTE;
		return (int)hipGetLastError();
	}
	for (uint32_t i = 0; i < N_PKERNELS && (!cfg || cfg->variant != 1); i++)
		if (g_pkernels[i].k == (int)p->k && g_pkernels[i].r == (int)p->rows) {
			id = i;
			break;
		}
	if (id == N_PKERNELS)
		id = N_PKERNELS - 1;	/* runtime-shaped */
	uint32_t gx = cfg && cfg->grid_x ? cfg->grid_x : (uint32_t)(nchunk < 65535 ? nchunk : 65535);
	uint32_t gy = cfg && cfg->grid_y ? cfg->grid_y : (p->nstripes < 65535 ? p->nstripes : 65535);
	hipLaunchKernelGGL(g_pkernels[id].fn, dim3(gx, gy), dim3(BLOCK), 0, st, *p, cells_dev);
	if (kernel_id)
		*kernel_id = KID_PTR + id;
	return (int)hipGetLastError();
}
