// ecg_mm_dev.h -- device building blocks of the GF(2^8) product shared by
// the product kernels (ecg_kernels.hip) and the fused product + checksum
// kernels (ecg_fused_kernels.hip): lane layouts, cell loads and stores, the
// v_perm_b32 multiply, ragged tails.  Design notes: ecg_kernels.hip header.
#ifndef ECG_MM_DEV_H
#define ECG_MM_DEV_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../ecg_kabi.h"


typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CHUNK_BYTES 4096u	// 256 lanes x 16 B
#define BLOCK 256

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

// Lane access granule G (16, 4, 2 or 1; align_granule below picks it per
// launch).  A wave always covers 1 KiB of each cell per column and a lane
// always owns 4 dwords of it; only how the dwords are fetched changes:
//   G = 16: one dwordx4 at wave*1024 + lane*16
//   G = 4 : four dwords at wave*1024 + {0, 256, 512, 768} + lane*4
//   G = 2 : the G = 16 layout, source pieces funnel-shifted out of
//           dword-aligned dwordx4 loads (ld_src16 below); destinations as
//           dwordx4 at their own (possibly misaligned) addresses
//   G = 1 : the G = 4 layout, source dwords funnel-shifted (ld_src below)
// so every wave-wide access is one contiguous 1024- or 256-byte run.  GF
// arithmetic is per byte, so which bytes a lane owns does not matter, only
// that loads and stores agree.

template <int G>
__device__ __forceinline__ uint32_t lane_off()
{
	constexpr uint32_t GL = G == 1 ? 4u : G == 2 ? 16u : (uint32_t)G;
	return (threadIdx.x >> 6) * 1024u + (threadIdx.x & 63u) * GL;
}

// byte offset of dword i of the lane's piece from lane_off<G>()
template <int G>
__device__ __forceinline__ uint32_t elem_off(int i)
{
	return G == 16 || G == 2 ? 4u * i : (uint32_t)i * 256u;
}

// G = 1 (sources at any byte alignment): the dword layout of G = 4 for the
// lanes and every store (and ACC read) of the destinations; a source dword at
// byte address a is funnel-shifted out of the aligned dwords around it,
// v_alignbyte_b32(hi, lo, a & 3).  hi holds byte a + 3, so it never leaves
// the cell's pages; when a is aligned hi is read from lo's own address
// (no branch: the shift is then 0).  m = a & 3 is wave-uniform per cell.

template <int G>
__device__ __forceinline__ u32x4 ld_g(const uint8_t *p)
{
	if constexpr (G == 1) {
		return ld_g<4>(p);	// destinations (ACC reads)
	} else if constexpr (G == 16 || G == 2) {
		return ld_nt(p);
	} else {
		static_assert(G == 4, "granule");
		const uint32_t *q = reinterpret_cast<const uint32_t *>(p);
		return (u32x4){__builtin_nontemporal_load(q), __builtin_nontemporal_load(q + 64),
			       __builtin_nontemporal_load(q + 128), __builtin_nontemporal_load(q + 192)};
	}
}

template <int G>
__device__ __forceinline__ void st_g(uint8_t *p, u32x4 v)
{
	if constexpr (G == 1) {
		st_g<4>(p, v);
	} else if constexpr (G == 16 || G == 2) {
		st_nt(p, v);
	} else {
		uint32_t *q = reinterpret_cast<uint32_t *>(p);
		__builtin_nontemporal_store(v[0], q);
		__builtin_nontemporal_store(v[1], q + 64);
		__builtin_nontemporal_store(v[2], q + 128);
		__builtin_nontemporal_store(v[3], q + 192);
	}
}

// G = 2: the lane's 16 bytes at cell + lo (the G = 16 layout) for a cell at
// any byte.  With m = cell & 3 (wave-uniform) they are bytes [m, m + 16) of
// the 20 bytes {a, b}: a = the lane's dwordx4 at cell - m + lo (dword-aligned,
// served by the hardware's unaligned access mode), b = the dword after it,
// which is lane l+1's a0 (a DPP wave rotate, no second load) except for lane
// 63, whose b is the dword right after the wave's 1 KiB (one wave-uniform
// load; when m = 0 it reads the wave's own last dword instead, so nothing
// past the column is read).  Dword w = v_alignbyte_b32(next, a_w, m).  No
// branch: with m = 0 the shift is 0, so the k loads of a column still issue
// back to back.
__device__ __forceinline__ u32x4 ld_src16(const uint8_t *cell, uint32_t lo)
{
	const uint32_t m = (uint32_t)(uintptr_t)cell & 3u;
	const uint8_t *base = cell - m;
	const u32x4 a = ld_nt(base + lo);
	const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	const uint32_t e = __builtin_nontemporal_load(
		reinterpret_cast<const uint32_t *>(base + wv * 1024u + (m ? 1024u : 1020u)));
	// lane 63's b is written into the rotate with v_writelane, not chosen by
	// a per-lane select: the compiler turns such a select of a load into a
	// branch, sinks the rotate under it, and lane 62 then reads a disabled
	// lane
	const uint32_t es = __builtin_amdgcn_readfirstlane(e);
	uint32_t b = (uint32_t)__builtin_amdgcn_mov_dpp((int)a[0], 0x134, 0xf, 0xf, false);

	asm("v_writelane_b32 %0, %1, 63" : "+v"(b) : "s"(es));

	return (u32x4){__builtin_amdgcn_alignbyte(a[1], a[0], m), __builtin_amdgcn_alignbyte(a[2], a[1], m),
		       __builtin_amdgcn_alignbyte(a[3], a[2], m), __builtin_amdgcn_alignbyte(b, a[3], m)};
}

// The lane's 4 dwords of a source cell at (wave-uniform) address `cell`.
// G = 1: the cell's dwords at lane offsets lo + 256 i, funnel-shifted out of
// the aligned dwords a_i (one load each, as G = 4) and the next aligned dword
// b_i, which is lane l+1's a_i -- a DPP wave rotate, no second load -- except
// for lane 63, whose b_i is lane 0's a_(i+1), and for b_3 of lane 63, the
// aligned dword after the wave's 1 KiB (one wave-uniform load).  When the
// cell is aligned (m = 0) the shift is 0 and b is never used; the uniform
// load then reads the wave's own last dword, so nothing past the column is
// ever read.
template <int G>
__device__ __forceinline__ u32x4 ld_src(const uint8_t *cell, uint32_t lo)
{
	if constexpr (G == 1) {
		const uint32_t m = (uint32_t)(uintptr_t)cell & 3u;
		const uint8_t *base = cell - m;
		const u32x4 a = ld_g<4>(base + lo);
		const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
		const uint32_t e = __builtin_nontemporal_load(
			reinterpret_cast<const uint32_t *>(base + wv * 1024u + (m ? 1024u : 1020u)));
		const bool last = (threadIdx.x & 63u) == 63u;
		uint32_t r[4];
		u32x4 x;

#pragma unroll
		for (int w = 0; w < 4; w++)	// lane l <- lane l+1 (wave_rol:1)
			r[w] = (uint32_t)__builtin_amdgcn_mov_dpp((int)a[w], 0x134, 0xf, 0xf, false);
#pragma unroll
		for (int w = 0; w < 4; w++) {
			const uint32_t b = last ? (w < 3 ? r[w + 1] : e) : r[w];
			x[w] = __builtin_amdgcn_alignbyte(b, a[w], m);
		}
		return x;
	} else if constexpr (G == 2) {
		return ld_src16(cell, lo);
	} else {
		return ld_g<G>(cell + lo);
	}
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
// JN, j0: load only cells [j0, j0 + JN) (phased loads of wide stripes; j0
// is a constant once the caller's loop is unrolled).
template <int KM, bool DIFF, int G = 16, int JN = KM>
__device__ __forceinline__ void mm_load(const ecg_mm_params_t &P, int k, uint32_t s, uint64_t cbase,
					uint32_t lo, u32x4 *x, int j0 = 0)
{
	const int64_t s_src = (int64_t)s * P.src_stripe_stride + (int64_t)cbase;
	const int64_t s_src2 = DIFF ? (int64_t)s * P.src2_stripe_stride + (int64_t)cbase : 0;

#pragma unroll
	for (int j = j0; j < j0 + JN; j++) {
		if (j < k) {
			int64_t o = P.src_cell_off[j] + s_src;
			asm volatile("" : "+s"(o));
			x[j] = ld_src<G>(P.src + o, lo);
			if (DIFF) {
				int64_t o2 = P.src2_cell_off[j] + s_src2;
				asm volatile("" : "+s"(o2));
				x[j] ^= ld_src<G>(P.src2 + o2, lo);
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

// Cells loaded per phase of the product kernel for k = K and lane granule G
// (0 = all k cells of a column before any arithmetic).  With PH > 0 a block
// keeps PH x 4 KiB of loads in flight per column instead of k x 4 KiB, and
// one phase's arithmetic overlaps the next phase's loads.  ECG_MM_WPE(K, R, G):
// the waves per SIMD the register budget of those instantiations targets (0 =
// the compiler's choice; a phased kernel needs a budget -- unconstrained, the
// scheduler computes the selectors of a whole phase at once and spills to
// AGPRs at 1 wave per SIMD).  With three output rows the 4-wave budget
// spills 84 bytes per lane to scratch; a 3-wave budget (141 VGPRs, no
// spill) measured the same (EC_8P3 1 MiB x 512 encode 0.982-0.988 vs
// 0.971-0.985 ms, decode 0.984-0.986 vs 0.981-0.984, profiles/r04/ec_ab/
// ec_ab_8p3_budget.json), so every R keeps 4.  Measured (tools/ec_ab.py, profiles/r04/ec_ab/,
// ms, back-to-back launches): k = 8 in 2 phases of 4 at 4 waves --
// EC_8P2 1 MiB x 512 decode 0.873 -> 0.836 (the best capped geometry before:
// 0.859), encode 0.844 -> 0.831, the dword-lane (G = 4) variant 0.895 ->
// 0.887.  The funnel-shift kernels (G = 1) spill when phased.  k = 16 in
// phases of 4 lost 5-20 % at 4 or 5 waves (phases of 8 spill).
// (The g2 lanes run one phase: two phases of 4 measured the same,
// profiles/r05/unaligned_ab/g2_phased.log.)
#ifndef ECG_MM_PHASE
#define ECG_MM_PHASE(K, G) ((K) == 8 && ((G) == 16 || (G) == 4) ? 4 : 0)
#endif
#ifndef ECG_MM_WPE
#define ECG_MM_WPE(K, R, G) ((K) == 8 && ((G) == 16 || (G) == 4) ? 4 : 0)
#endif

// The product of one column: x[j] = the lane's 16 bytes of cell j.  STORE =
// false leaves the stores to the caller (outputs returned in keep).  PH > 0:
// only cells [0, PH) are loaded on entry, and cells [j, j + PH) are loaded
// when the fold reaches j (DIFF: their src2 too).  (One function on purpose: the same loops split
// into init / fold / store helpers made the register allocator keep EC_16P2
// at 256 VGPRs + AGPRs, 1 wave per SIMD, instead of 114 / 4 waves.)
// PA (the pointer-table kernel): the phase loads read cell j at the
// wave-uniform address pa[j] (+ lo) instead of P's offsets.
template <int KM, int RM, bool ACC, bool KEEP, bool STORE = true, int G = 16, int PH = 0, bool DIFF = false,
	  bool PA = false>
__device__ __forceinline__ void mm_compute(const ecg_mm_params_t &P, const u32x4 *tb, int k, int rows,
					   uint32_t s, uint64_t cbase, uint32_t lo, u32x4 *x, u32x4 *keep,
					   const uint64_t *pa = nullptr)
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
				acc[r] = ld_g<G>(P.dst + o + lo);
			} else {
				acc[r] = (u32x4){0u, 0u, 0u, 0u};
			}
		}
	}
#pragma unroll
	for (int j = 0; j < KM; j++) {
		if constexpr (PH > 0) {
			if (j > 0 && j % PH == 0) {
				// the next phase's loads and table reads depend (falsely)
				// on every accumulator: none of them can be issued before
				// this phase's arithmetic is done
				uint32_t lo2 = lo, z2 = 0, dep = 0;
#pragma unroll
				for (int r = 0; r < RM; r++)
					if (r < rows)
						dep ^= acc[r][0] ^ acc[r][1] ^ acc[r][2] ^ acc[r][3];
				asm volatile("" : "+v"(lo2), "+v"(z2) : "v"(dep));
				tb += z2;
				if constexpr (PA) {
#pragma unroll
					for (int i = j; i < j + PH && i < KM; i++)
						if (i < k)
							x[i] = ld_src<G>(reinterpret_cast<const uint8_t *>(pa[i]), lo2);
				} else {
					mm_load<KM, DIFF, G, PH>(P, k, s, cbase, lo2, x, j);
				}
			}
		}
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
				st_g<G>(P.dst + o + lo, acc[r]);
			}
			if (KEEP)
				keep[r] = acc[r];
		}
	}
}

template <int KM, int RM, bool ACC, bool DIFF, bool KEEP = false, int G = 16>
__device__ __forceinline__ void mm_item(const ecg_mm_params_t &P, const u32x4 *tb, int k, int rows,
					uint32_t s, uint64_t cbase, uint32_t lo, u32x4 *keep = nullptr)
{
	constexpr int PH = (ECG_MM_PHASE(KM, G) > 0 && ECG_MM_PHASE(KM, G) < KM && KM % ECG_MM_PHASE(KM, G) == 0)
				   ? ECG_MM_PHASE(KM, G) : 0;
	u32x4 x[KM];

	mm_load<KM, DIFF, G, PH ? PH : KM>(P, k, s, cbase, lo, x);
	mm_compute<KM, RM, ACC, KEEP, true, G, PH, DIFF>(P, tb, k, rows, s, cbase, lo, x, keep);
}

// One dword of every output row at byte offset `off` of the cells (the
// partial last column of a G = 4 / 1 launch: the dword lies inside the cell).
// The k loads are issued together.  Cells off a dword boundary (G = 1, and
// destinations at any byte) are read and written with misaligned dword
// accesses, which the hardware's unaligned access mode serves (the ROCm
// default on gfx9+; the compiler itself emits such accesses for byte-aligned
// data).
template <int KM, int RM, bool ACC, bool DIFF>
__device__ __forceinline__ void mm_dword(const ecg_mm_params_t &P, const u32x4 *tb, int k, int rows,
					 uint32_t s, uint64_t off)
{
	constexpr int T2V = (RM + 3) / 4;
	constexpr int PER_J = RM + T2V;
	constexpr int JB = KM < 4 ? KM : 4;	// loads in flight (more cost k = 16 a wave per SIMD)
	const uint8_t *sb = P.src + (int64_t)s * P.src_stripe_stride + off;
	const uint8_t *sb2 = DIFF ? P.src2 + (int64_t)s * P.src2_stripe_stride + off : nullptr;
	uint8_t *db = P.dst + (int64_t)s * P.dst_stripe_stride + off;
	uint32_t o[RM];

#pragma unroll
	for (int r = 0; r < RM; r++)
		o[r] = 0;
#pragma nounroll
	for (int j0 = 0; j0 < k; j0 += JB) {
		uint32_t x[JB];

#pragma unroll
		for (int i = 0; i < JB; i++) {
			if (j0 + i < k) {
				// laundered like mm_load's: LICM would hoist the unrolled
				// cell offsets out of the stripe loop into VGPRs
				int64_t o1 = P.src_cell_off[j0 + i];
				asm volatile("" : "+s"(o1));
				x[i] = *reinterpret_cast<const uint32_t *>(sb + o1);
				if (DIFF) {
					int64_t o2 = P.src2_cell_off[j0 + i];
					asm volatile("" : "+s"(o2));
					x[i] ^= *reinterpret_cast<const uint32_t *>(sb2 + o2);
				}
			}
		}
#pragma unroll
		for (int i = 0; i < JB; i++) {
			const int j = j0 + i;

			if (j >= k)
				continue;
			const uint32_t v = x[i];
			const uint32_t s0 = v & 0x07070707u, s1 = (v >> 3) & 0x07070707u, s2 = (v >> 6) & 0x03030303u;
#pragma unroll
			for (int r = 0; r < RM; r++) {
				if (r < rows) {
					const u32x4 t = tb[j * PER_J + r];
					const uint32_t t2 = reinterpret_cast<const uint32_t *>(&tb[j * PER_J + RM])[r];
					o[r] ^= __builtin_amdgcn_perm(t[1], t[0], s0) ^ __builtin_amdgcn_perm(t[3], t[2], s1) ^
						__builtin_amdgcn_perm(t2, t2, s2);
				}
			}
		}
	}
#pragma unroll
	for (int r = 0; r < RM; r++) {
		if (r < rows) {
			uint32_t *d = reinterpret_cast<uint32_t *>(db + P.dst_cell_off[r]);
			*d = ACC ? *d ^ o[r] : o[r];
		}
	}
}

// The same dword, the k loads one after another: the G = 4 partial column
// (the batched form above changed the G = 4 main path's register
// allocation, and 8-byte-aligned parity rows ran 1-2 % slower,
// profiles/r04/ec_ab/).
template <int RM, bool ACC, bool DIFF>
__device__ __forceinline__ void mm_dword_plain(const ecg_mm_params_t &P, const u32x4 *tb, int k, int rows,
					 uint32_t s, uint64_t off)
{
	constexpr int T2V = (RM + 3) / 4;
	constexpr int PER_J = RM + T2V;
	const uint8_t *sb = P.src + (int64_t)s * P.src_stripe_stride + off;
	const uint8_t *sb2 = DIFF ? P.src2 + (int64_t)s * P.src2_stripe_stride + off : nullptr;
	uint8_t *db = P.dst + (int64_t)s * P.dst_stripe_stride + off;
	uint32_t o[RM];

#pragma unroll
	for (int r = 0; r < RM; r++)
		o[r] = 0;
	for (int j = 0; j < k; j++) {
		uint32_t v = *reinterpret_cast<const uint32_t *>(sb + P.src_cell_off[j]);
		if (DIFF)
			v ^= *reinterpret_cast<const uint32_t *>(sb2 + P.src2_cell_off[j]);
		const uint32_t s0 = v & 0x07070707u, s1 = (v >> 3) & 0x07070707u, s2 = (v >> 6) & 0x03030303u;
#pragma unroll
		for (int r = 0; r < RM; r++) {
			if (r < rows) {
				const u32x4 t = tb[j * PER_J + r];
				const uint32_t t2 = reinterpret_cast<const uint32_t *>(&tb[j * PER_J + RM])[r];
				o[r] ^= __builtin_amdgcn_perm(t[1], t[0], s0) ^ __builtin_amdgcn_perm(t[3], t[2], s1) ^
					__builtin_amdgcn_perm(t2, t2, s2);
			}
		}
	}
#pragma unroll
	for (int r = 0; r < RM; r++) {
		if (r < rows) {
			uint32_t *d = reinterpret_cast<uint32_t *>(db + P.dst_cell_off[r]);
			*d = ACC ? *d ^ o[r] : o[r];
		}
	}
}

// Ragged tail: fewer than 16 bytes of this lane's slot are inside the cell
// (G = 16: the lane straddling the cell's end).  A plain loop: inlined into
// every kernel, a batched version changed the register allocation of the
// main path (EC_4P2 76 -> 61 VGPRs and 2 % slower, profiles/r04/unaligned_ab/).
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

// The < 4 bytes after a cell's last whole dword (G = 4 / 1 partial
// columns): bytewise, up to 4 of a byte's k loads issued together.
template <int KM, int RM, bool ACC, bool DIFF>
__device__ __forceinline__ void mm_tail_b(const ecg_mm_params_t &P, const u32x4 *tb, int k, int rows,
				     uint32_t s, uint64_t off, int nb)
{
	constexpr int T2V = (RM + 3) / 4;
	constexpr int PER_J = RM + T2V;
	constexpr int JB = KM < 4 ? KM : 4;
	const uint8_t *sb = P.src + (int64_t)s * P.src_stripe_stride;
	const uint8_t *sb2 = DIFF ? P.src2 + (int64_t)s * P.src2_stripe_stride : nullptr;
	uint8_t *db = P.dst + (int64_t)s * P.dst_stripe_stride;

	for (int b = 0; b < nb; b++) {
		uint32_t o[RM];
#pragma unroll
		for (int r = 0; r < RM; r++)
			o[r] = 0;
#pragma nounroll
		for (int j0 = 0; j0 < k; j0 += JB) {
			uint32_t x[JB];

#pragma unroll
			for (int i = 0; i < JB; i++) {
				if (j0 + i < k) {
					int64_t o1 = P.src_cell_off[j0 + i];
					asm volatile("" : "+s"(o1));
					x[i] = sb[o1 + off + b];
					if (DIFF) {
						int64_t o2 = P.src2_cell_off[j0 + i];
						asm volatile("" : "+s"(o2));
						x[i] ^= sb2[o2 + off + b];
					}
				}
			}
#pragma unroll
			for (int i = 0; i < JB; i++) {
				const int j = j0 + i;

				if (j >= k)
					continue;
				const uint32_t v = x[i];
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

// The last, partial column of a cell (C % 4096 != 0): G = 16 as a full
// lane piece where the lane's 16 bytes are inside the cell, else bytewise;
// G = 4 / 1 dword by dword (G = 1: misaligned source dwords), the bytes
// after the cell's last whole dword bytewise.
template <int KM, int RM, bool ACC, bool DIFF, int G>
__device__ __forceinline__ void mm_partial(const ecg_mm_params_t &P, const u32x4 *tb, int k, int rows,
					   uint32_t s, uint64_t cbase, uint32_t lo)
{
	const uint64_t C = P.cell_bytes;

	if constexpr (G == 2) {
		// the funnel needs every lane of the wave: the partial column runs
		// the G = 1 dword layout instead (misaligned dword loads)
		mm_partial<KM, RM, ACC, DIFF, 1>(P, tb, k, rows, s, cbase, lane_off<1>());
	} else if constexpr (G == 16) {
		if (cbase + lo + 16 <= C)
			mm_item<KM, RM, ACC, DIFF>(P, tb, k, rows, s, cbase, lo);
		else if (cbase + lo < C)
			mm_tail<RM, ACC, DIFF>(P, tb, k, rows, s, cbase + lo, (int)(C - cbase - lo));
	} else {
		// not unrolled: four inlined copies of the byte loop cost ~70 VGPRs
		// in every instantiation (this path runs once per cell at most)
#pragma nounroll
		for (int i = 0; i < 4; i++) {
			const uint64_t off = cbase + lo + elem_off<G>(i);

			if constexpr (G == 1) {
				if (off + 4 <= C)
					mm_dword<KM, RM, ACC, DIFF>(P, tb, k, rows, s, off);
				else if (off < C)
					mm_tail_b<KM, RM, ACC, DIFF>(P, tb, k, rows, s, off, (int)(C - off));
			} else {
				if (off + 4 <= C)
					mm_dword_plain<RM, ACC, DIFF>(P, tb, k, rows, s, off);
				else if (off < C)
					mm_tail<RM, ACC, DIFF>(P, tb, k, rows, s, off, (int)(C - off));
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
// default: without a cap from the context (ecg_set_wg_per_cu) or the launch
// tuner (ecg_tune.c, which measures one per shape) a launch is uncapped.
__host__ static inline uint32_t mm_wg_cap(const ecg_mm_params_t *p, const ecg_launch_cfg_t *cfg, uint64_t blocks)
{
	const uint32_t c = cfg ? cfg->wg_per_cu : 0;

	(void)p;
	(void)blocks;
	if (c == ECG_WG_UNCAPPED || c == 0)
		return 0;
	return c < 2 ? 2 : c;
}

// Unused dynamic LDS that leaves room for exactly `cap` blocks per CU (160 KiB
// of LDS; a block may take at most 64 KiB, so cap >= 2); k, r: the
// instantiation's (0 = runtime-shaped), whose static table takes the rest.
__host__ static inline size_t mm_dyn_lds(uint32_t cap, int k, int r)
{
	const int km = k ? k : ECG_KMAX_K, rm = r ? r : ECG_KMAX_R;
	const size_t stat = (size_t)km * (rm + (rm + 3) / 4) * 16;	// ecg_mm_kernel's s_tbl
	size_t d;

	if (cap == 0)
		return 0;
	d = (size_t)(163840.0 / (cap + 0.5));
	if (d > 65536)
		d = 65536;
	return d > stat ? (d - stat) & ~(size_t)255 : 0;
}

static inline uint32_t granule_of(uint64_t bits)
{
	return (bits & 15u) == 0 ? 16u : (bits & 7u) == 0 ? 8u : (bits & 3u) == 0 ? 4u : 1u;
}

// The lane access a launch uses: 16 when every cell address is 16-byte
// aligned, 4 when every source is dword-aligned; 1 when a source is off a
// dword boundary (the funnel-shifted loads of ld_src<1>).  Destinations off a
// dword boundary take the dword lanes' stores as they are: misaligned dword
// stores (and ACC loads), served by the hardware's unaligned access mode,
// ran 0.93-0.96 of the aligned kernel where the byte kernel ran 0.10 of the
// HBM spec (tools/unaligned_ab.py, profiles/r04/unaligned_ab/).  The launcher
// (ecg_k_launch_matmul) then runs k = 8 launches whose sources are off a
// 16-byte boundary on G = 2 (profiles/r05/unaligned_ab/).
static inline uint32_t align_granule(const ecg_mm_params_t *p)
{
	uint64_t sb = (uint64_t)(uintptr_t)p->src | (uint64_t)p->src_stripe_stride;
	uint64_t db = (uint64_t)(uintptr_t)p->dst | (uint64_t)p->dst_stripe_stride;
	for (uint32_t j = 0; j < p->k; j++) {
		sb |= (uint64_t)p->src_cell_off[j];
		if (p->diff)
			sb |= (uint64_t)p->src2_cell_off[j];
	}
	if (p->diff)
		sb |= (uint64_t)(uintptr_t)p->src2 | (uint64_t)p->src2_stripe_stride;
	for (uint32_t r = 0; r < p->rows; r++)
		db |= (uint64_t)p->dst_cell_off[r];
	const uint32_t gs = granule_of(sb), gd = granule_of(db);

	if (gs < 4)
		return 1;
	/* 8-byte alignment takes the dword lanes too: the dwordx2-lane variant
	 * ran 0.84-0.94 of the aligned kernel on different boxes, the dword one
	 * (two-phase at k = 8) 0.94-0.98 (profiles/r04/run2/) */
	return gs == 16 && gd == 16 ? 16 : 4;
}

static inline bool aligned16(const ecg_mm_params_t *p)
{
	return align_granule(p) == 16u;
}

#endif
