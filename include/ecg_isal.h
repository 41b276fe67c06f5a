/*
 * ecg_isal.h -- ISA-L-signature drop-in for the erasure-code entry points
 * DAOS links (`#include <isa-l.h>`, ref:src/object/obj_ec.h:14; library
 * pinned at ref:utils/build.config:8 = ISA-L v2.31.1).
 *
 * libecg.so exports these symbols under their ISA-L names, so relinking the
 * DAOS object module against libecg instead of libisal swaps the CPU codec
 * for the MI355X one with no source change.  Every function keeps ISA-L's
 * signature, argument meaning, return convention and output bytes:
 *
 *   symbol                  DAOS call site(s) it serves
 *   gf_gen_cauchy1_matrix   ref:src/object/obj_class.c:614
 *   ec_init_tables          ref:src/object/obj_class.c:616, ref:src/object/cli_ec.c:2246
 *   ec_encode_data          ref:src/object/cli_ec.c:540,571,2641,
 *                           ref:src/object/srv_ec_aggregate.c:693,1136,
 *                           ref:src/tests/suite/daos_aggregate_ec.c:395,531
 *   ec_encode_data_update   ref:src/object/srv_ec_aggregate.c:1099
 *   gf_invert_matrix        ref:src/object/cli_ec.c:2223
 *   gf_mul                  ref:src/object/cli_ec.c:2239
 *   xor_gen                 ref:src/object/srv_ec_aggregate.c:1092
 * plus gf_inv, gf_vect_mul_init, gf_gen_rs_matrix to complete the surface.
 *
 * gftbls layout: ec_init_tables writes ISA-L's 32-byte-per-coefficient
 * nibble tables (c*{0..15}, c*{0x00,0x10..0xf0}); DAOS treats them as opaque
 * (it only allocates k*p*32 bytes and memcpy's them, ref:src/object/cli_ec.c:
 * 2205-2210).  ec_encode_data recovers each coefficient as byte 1 (= c*1).
 *
 * Data-plane calls (ec_encode_data, ec_encode_data_update, xor_gen) run
 * where their cells are (ecg.h ecg_set_dropin_crossover):
 *   - cells in device memory (every pointer of the call inside a hipMalloc'd
 *     allocation -- an engine whose buffers live in HBM): the gfx950 kernels
 *     in place, on the cells' device (listed in $ECG_DEVICES), synchronous;
 *   - host cells: the product CPU path (GFNI / AVX2 / scalar by cpuid) below
 *     the measured crossover (by default: always -- one core beats a staged
 *     PCIe round trip at every size measured), in any process without a usable
 *     gfx950 device (a libdaos client node), and with $ECG_FORCE_CPU=1; above
 *     the crossover, the GPU through per-thread pinned staging ($ECG_DEVICES /
 *     $ECG_DEVICE pick the devices), with the CPU as fallback.
 * Like ISA-L's, these calls succeed on any CPU.  A call on device cells that
 * cannot run (device not listed, a cell past its allocation, a HIP failure)
 * prints the cause and aborts: the ABI is `void`, and skipping the parity
 * silently would corrupt stored objects.
 */
#ifndef ECG_ISAL_H
#define ECG_ISAL_H

#ifdef __cplusplus
extern "C" {
#endif

void ec_init_tables(int k, int rows, unsigned char *a, unsigned char *gftbls);
void ec_encode_data(int len, int k, int rows, unsigned char *gftbls,
		    unsigned char **data, unsigned char **coding);
void ec_encode_data_update(int len, int k, int rows, int vec_i, unsigned char *gftbls,
			   unsigned char *data, unsigned char **coding);
void gf_vect_mul_init(unsigned char c, unsigned char *gftbl);
unsigned char gf_mul(unsigned char a, unsigned char b);
unsigned char gf_inv(unsigned char a);
void gf_gen_rs_matrix(unsigned char *a, int m, int k);
void gf_gen_cauchy1_matrix(unsigned char *a, int m, int k);
int gf_invert_matrix(unsigned char *in, unsigned char *out, const int n);
/* raid.h: array[vects-1] = XOR of array[0..vects-2]; 0 pass, non-zero fail
 * (fewer than two sources). */
int xor_gen(int vects, int len, void **array);

#ifdef __cplusplus
}
#endif
#endif
