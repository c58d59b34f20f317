/*
 * net2/sha2_batch.h -- C ABI of the MI355X batched SHA-2 digest path.
 *
 * Drop-in boundary for the reference's SHA-2 integrity hash:
 *   - replaces the per-payload SHA{256,384,512}Init/Update/Final sequence of
 *     src/sha2.c:280-563 / :566-919 (declared in the absent
 *     include/ilias/net2/bsd_compat/sha2.h, included from src/sha2.c:38,
 *     src/sign.c:36, types/packet.n2t:80) with one call over many
 *     independent packets;
 *   - is what net2_hashctx_hashbuf (called at types/signature.n2t:92,147)
 *     and net2_signctx_fingerprint (src/sign.c:298-307) bottom out in; see
 *     net2/hash.h for that registry layer.
 *
 * Conventions:
 *   - plain pointers and sizes only; no HIP, torch or C++ types;
 *   - return 0 on success, or an errno value: EINVAL (bad alg / argument),
 *     ENOMEM (allocation), ENODEV (no usable MI355X), EIO (HIP runtime
 *     error; net2_sha2_last_hip_error() has the HIP code).  Nothing aborts;
 *   - thread-safe: calls may come from any number of host threads (the
 *     reference runs signature work on threadpool workers,
 *     include/ilias/net2/threadpool.h:33-34);
 *   - there is no CPU fallback: without a usable gfx950 device every
 *     compute entry point fails with ENODEV.
 *
 * Digest byte order and values are those of src/sha2.c's *Final
 * (big-endian state words, 32 / 48 / 64 bytes).
 */
#ifndef NET2_SHA2_BATCH_H
#define NET2_SHA2_BATCH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NET2_SHA2_ABI_VERSION 1

/* Algorithm indices = rows of the hash registry in net2/hash.h. */
#define NET2_HASH_NIL		0
#define NET2_HASH_SHA256	1
#define NET2_HASH_SHA384	2
#define NET2_HASH_SHA512	3
#define NET2_HASH_HMAC_SHA256	4
#define NET2_HASH_HMAC_SHA384	5
#define NET2_HASH_HMAC_SHA512	6

/* ABI version of the loaded library (NET2_SHA2_ABI_VERSION). */
int net2_sha2_abi_version(void);

/*
 * Identity of the kernel build: the first 16 hex digits of the SHA-256 of
 * the kernels' device code (identical machine code, identical id; an A/B
 * build with other -D flags gets its own).  Profiles record it next to the
 * counters they measured (profiles/pmc_*.json), so measurements of another
 * build are recognisable as such.  A static string.
 */
const char *net2_sha2_build_id(void);

/* Number of usable gfx950 devices, via *count.  0 / ENODEV. */
int net2_sha2_device_count(int *count);

/*
 * The calling thread's device for the single-message calls (net2/hash.h
 * net2_hashctx_hashiov, the SHA2_CTX calls of net2/sha2.h) and the first
 * device of its batches: index < the device count (the device list; under
 * the test knob NET2_SHA2_VIRTUAL_DEVICES=k every GPU is listed k times), or
 * -1 to follow the thread's current HIP device (the default; a thread whose
 * current device is not a gfx950 uses the first).  A selection also makes
 * that GPU the thread's current HIP device.  *prev (may be NULL) receives
 * the previous selection (-1: none), so a helper thread can run one task on
 * its submitter's device and restore its own.  0, EINVAL or ENODEV.
 *
 * The reference runs signature work on workq threads of a shared
 * threadpool (include/ilias/net2/threadpool.h:33-34), which have no device
 * of their own: a caller that drives GPU k hands its selection
 * (net2_sha2_get_device) to the tasks it submits, as the signed carver's
 * helper pool does (csrc/host/signed_carver.c pool_run).
 */
int net2_sha2_set_device(int index, int *prev);

/* The device index the calling thread's single-message calls go to now
 * (its selection, else the one its current HIP device maps to).  0, EINVAL
 * or ENODEV. */
int net2_sha2_get_device(int *index);

/*
 * NUMA placement of net2_sha2_batch's host-side work (diagnostics): for
 * device index `device` of its device list, the NUMA node the GPU hangs
 * off (-1 when the host does not say), the slices it has run, and how many
 * of them ended on a CPU of that node (each slice's thread and its pack
 * threads are bound to the node's CPUs while the slice runs;
 * NET2_SHA2_NUMA=0 turns that off).  Any pointer may be NULL.  0, EINVAL or
 * ENODEV.
 */
int net2_sha2_numa_stats(int device, int *numa_node, uint64_t *slices,
    uint64_t *slices_on_node);

/* HIP error code behind the calling thread's last EIO (0 if none). */
int net2_sha2_last_hip_error(void);

/* Human-readable text for a return code of this API. */
const char *net2_sha2_strerror(int err);

/*
 * Device-resident batch, fixed stride (config "1M x 1 KiB").
 * Packet i is d_base[i * stride .. i * stride + len); its digest is written
 * to d_digests + i * hashlen (32 / 48 / 64).  All pointers are device
 * memory of the calling thread's current HIP device.  Asynchronous on
 * `stream` (a hipStream_t; NULL = the null stream); the call returns once
 * the work is enqueued.  Requires len <= stride when n > 1.
 */
int net2_sha2_dev_fixed(int alg, const void *d_base, uint64_t stride,
    uint32_t len, uint64_t n, void *d_digests, void *stream);

/*
 * Device-resident batch, packed variable-length packets (config "1M x
 * mixed {64, 512, 1500} B"): packet i is d_base[d_offsets[i] ..
 * d_offsets[i] + d_lens[i]).  Lengths are binned on the device so lanes of
 * a wave share a block count (one binning launch); d_ws must hold
 * net2_sha2_dev_var_workspace(n) bytes of device memory (4-byte aligned,
 * see net2_sha2_workspace_init) or be NULL to hash in submission order
 * (slower on mixed lengths).
 * Asynchronous on `stream`; d_ws must stay allocated until it completes.
 */
int net2_sha2_dev_var(int alg, const void *d_base, const uint64_t *d_offsets,
    const uint32_t *d_lens, uint64_t n, void *d_digests, void *d_ws,
    size_t ws_bytes, void *stream);

/* Bytes of scratch net2_sha2_dev_var needs for n packets. */
size_t net2_sha2_dev_var_workspace(uint64_t n);

/*
 * Prepare a variable-layout workspace (net2_sha2_dev_var, the variable
 * layouts of net2_hmac_dev / _sign_dev / _verify_dev, and a packet-burst
 * workspace, net2/packet.h, whose binning area comes first), asynchronously
 * on `stream`; zeroes its counters (net2_sha2_workspace_stats).  Optional:
 * the binning keeps its state in the workspace and cleans up after itself,
 * so a workspace reused call after call needs this at most once; an
 * unprepared one (fresh memory) hashes its first batch in submission order
 * -- same digests, only without the length binning -- while it prepares
 * itself.  A workspace used for other data in between should be prepared
 * again: the binning detects a histogram that is not its own (the batch is
 * then hashed in submission order and counted as a mismatch), but only
 * preparation restores binning from the next call on.  A workspace must not
 * serve two launches that may run at once.  0, EINVAL (NULL, misaligned or
 * smaller than net2_sha2_dev_var_workspace(0)), ENODEV or EIO.
 */
int net2_sha2_workspace_init(void *d_ws, size_t ws_bytes, void *stream);

/*
 * What the length binning of a workspace has done since
 * net2_sha2_workspace_init, or since the first use of a fresh one
 * (diagnostics; the binning falls back to submission order -- same digests,
 * slower -- and counts why):
 *   prepared    the header is valid (the next launch bins);
 *   binned      launches whose grid barrier completed (binned, unless
 *               counted as a mismatch too);
 *   aborts      grid barriers that timed out (the binning grid was not
 *               co-resident, e.g. beside long kernels on other streams);
 *   mismatches  launches whose global histogram did not add up to the
 *               batch (the workspace was overwritten between calls);
 *   unprepared  launches that found the header unprepared (fresh memory, or
 *               the launch after an abort or a mismatch).
 */
struct net2_bin_stats {
	uint32_t prepared;
	uint32_t binned;
	uint32_t aborts;
	uint32_t mismatches;
	uint32_t unprepared;
};

/*
 * Reads a workspace's counters (synchronous device-to-host copy of its
 * header; synchronise the streams that use it first).  0, EINVAL, ENODEV
 * or EIO.
 */
int net2_sha2_workspace_stats(const void *d_ws, size_t ws_bytes,
    struct net2_bin_stats *stats);

/*
 * Limits of the one-launch binning, process-wide (diagnostics and tests):
 * grid_cap caps its persistent grid (0: the device's co-resident capacity
 * of the binning kernel, at most 256 workgroups -- the default); timeout_us
 * is how long its grid barrier waits for every workgroup before deciding
 * ABORT (< 0: the default 50 ms; 0 makes every launch whose workgroups are
 * not all there at once abort).  Always 0.
 */
int net2_sha2_bin_limits(uint32_t grid_cap, int64_t timeout_us);

/*
 * Host-memory batch, end to end: packets are read from host memory (DMA'd
 * directly when the buffer is page-locked and the layout fixed, else staged
 * through pinned buffers), hashed on every usable device (contiguous packet
 * slices -- by bytes for the variable layout -- one host thread and stream
 * pair per device, 64 MiB chunks double-buffered), and the digests stored
 * by the kernels into page-locked host memory (the caller's buffer when it
 * is page-locked).  Synchronous.  offsets == NULL selects the fixed layout
 * base[i * stride .. + fixed_len); otherwise packet i is
 * base[offsets[i] .. + lens[i]) and stride / fixed_len are ignored.
 * max_devices <= 0 uses every device, but no slice smaller than 16 MiB of
 * payload (NET2_SHA2_SLICE_MIN_BYTES): a small batch stays on one device.
 * The device list starts at the calling thread's current HIP device (so
 * max_devices == 1 means "this device" for a one-process-per-GPU caller).
 * NUMA: each slice's thread is bound to the CPUs of its GPU's node (within
 * the process's cpuset) while the slice runs; the first slice runs on the
 * calling thread, so that thread's affinity is the node's for the duration
 * of the call and is restored before it returns (NET2_SHA2_NUMA=0: off).
 */
int net2_sha2_batch(int alg, const void *base, const uint64_t *offsets,
    const uint32_t *lens, uint64_t stride, uint32_t fixed_len, uint64_t n,
    void *digests, int max_devices);

#ifdef __cplusplus
}
#endif
#endif /* NET2_SHA2_BATCH_H */
