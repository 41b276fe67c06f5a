/*
 * ecg_buildinfo.c -- identity of this build (include/ecg.h ecg_build_info):
 * the hash of the sources it was compiled from, the hipcc that compiled the
 * kernels and the offload target, all fixed by the Makefile at build time.
 */
#include "../../../include/ecg.h"

/* daos_amd/csrc/Makefile sets all three; the sanitizer test builds
 * (tests/c/Makefile) compile the host sources directly and say so */
#ifndef ECG_SRC_HASH
#define ECG_SRC_HASH "none(test-build)"
#endif
#ifndef ECG_HIPCC
#define ECG_HIPCC "unknown"
#endif
#ifndef ECG_ARCH
#define ECG_ARCH "gfx950"
#endif

const char *ecg_build_info(void)
{
	return "src_sha256=" ECG_SRC_HASH ";hipcc=" ECG_HIPCC ";arch=" ECG_ARCH;
}
