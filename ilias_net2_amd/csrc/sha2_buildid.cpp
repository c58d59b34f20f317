/*
 * sha2_buildid.cpp -- identity of the kernel build linked into
 * libnet2_sha2.so (net2_sha2_build_id, include/net2/sha2_batch.h): the first
 * 16 hex digits of the SHA-256 of sha2_kernels.o's device code (its
 * .hip_fatbin section), so two builds with the same machine code share an
 * id whatever changed in the sources around it, and an A/B build (other -D
 * flags) gets its own.  The Makefile (and tools/build_ab.sh) compile this
 * file after the kernels with -DNET2_KERNEL_BUILD_ID.  Profiles record the
 * id next to the counters they measured (tools/pmc_summary.py), and
 * bench.py uses counters only of the build it loaded.
 */
#ifndef NET2_KERNEL_BUILD_ID
#define NET2_KERNEL_BUILD_ID "unstamped"
#endif

extern "C" __attribute__((visibility("default"))) const char *
net2_sha2_build_id(void)
{
	return NET2_KERNEL_BUILD_ID;
}
