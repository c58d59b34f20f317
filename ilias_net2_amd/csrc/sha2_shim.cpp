/*
 * sha2_shim.cpp -- the C-ABI front of the MI355X SHA-2 path
 * (include/net2/sha2_batch.h, include/net2/hash.h).
 *
 * Host orchestration only: argument checks with errno-style returns (the
 * reference maps hash failures to ENOMEM / NET2_P{EN,DE}CODE_RESOURCE,
 * types/signature.n2t:93-95, types/packet.n2t:246-249), device discovery,
 * pinned staging and stream management.  Every digest is computed by the
 * HIP kernels in sha2_kernels.hip; there is deliberately no CPU hashing
 * path here, so a missing or unusable GPU is an ENODEV, never a silent
 * fallback.
 */
#include "sha2_launch.h"
#include "sha2_coalesce.h"

#include <hip/hip_runtime.h>

#include <errno.h>
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <string.h>
#include <sys/uio.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#define NET2_EXPORT extern "C" __attribute__((visibility("default")))

#include "../../include/net2/hash.h"
#include "../../include/net2/packet.h"
#include "../../include/net2/sha2.h"

namespace {

thread_local int tl_last_hip_error = 0;

int hip_fail(hipError_t e)
{
	tl_last_hip_error = (int)e;
	return e == hipErrorOutOfMemory ? ENOMEM : EIO;
}

#define HIP_TRY(expr)                                                        \
	do {                                                                 \
		hipError_t _e = (expr);                                      \
		if (_e != hipSuccess)                                        \
			return hip_fail(_e);                                 \
	} while (0)

/*
 * Test-only fault injection (a -DNET2_FAULT_INJECT=1 build, libnet2_sha2_fi.so;
 * the shipped library compiles it out).  net2_fault_inject(site, k) makes the
 * k-th pass through `site` of a host-pipeline chunk fail as if its HIP call
 * had: FI_H2D once the chunk's input copy is queued, FI_KERNEL once its first
 * kernel is launched, FI_RECORD in place of the chunk's event record.
 * tests/test_gpu_failures.py drives it.
 */
#ifndef NET2_FAULT_INJECT
#define NET2_FAULT_INJECT 0
#endif
enum { FI_H2D = 1, FI_KERNEL = 2, FI_RECORD = 3 };
#if NET2_FAULT_INJECT
std::atomic<int> g_fi_site{0}, g_fi_left{0};
bool fi_hit(int site)
{
	if (g_fi_site.load(std::memory_order_relaxed) != site)
		return false;
	if (g_fi_left.fetch_sub(1, std::memory_order_relaxed) != 1)
		return false;
	g_fi_site.store(0, std::memory_order_relaxed);
	return true;
}
#else
constexpr bool fi_hit(int) { return false; }
#endif
#define FI_POINT(site)                                                       \
	do {                                                                 \
		if (fi_hit(site))                                            \
			return hip_fail(hipErrorLaunchFailure);              \
	} while (0)

/*
 * After a chunk failed part-way: wait for whatever it already queued on its
 * stream (a copy still reading the caller's input or the slot's staging, a
 * kernel still storing into the caller's mapped output), so nothing of the
 * failed call runs after it returns and the slot can be reused.  The first
 * error's HIP code is kept for net2_sha2_last_hip_error.
 */
void quiesce(hipStream_t st)
{
	if (st == nullptr)
		return;
	const int keep = tl_last_hip_error;
	(void)hipStreamSynchronize(st);
	(void)hipGetLastError();
	tl_last_hip_error = keep;
}

/* ---- registry (include/net2/hash.h) ------------------------------------ */

struct HashRow {
	const char *name;
	int hashlen;
	int keylen;
};

const HashRow kRows[] = {
	{ "nil", 0, 0 },
	{ "SHA256", 32, 0 },
	{ "SHA384", 48, 0 },
	{ "SHA512", 64, 0 },
	{ "HMAC-SHA256", 32, 32 },
	{ "HMAC-SHA384", 48, 48 },
	{ "HMAC-SHA512", 64, 64 },
};
constexpr int kNumRows = sizeof(kRows) / sizeof(kRows[0]);

bool unkeyed_sha2(int alg)
{
	return alg == NET2_HASH_SHA256 || alg == NET2_HASH_SHA384 ||
	    alg == NET2_HASH_SHA512;
}

int digest_len(int alg)
{
	return alg >= 0 && alg < kNumRows ? kRows[alg].hashlen : -1;
}

/* ---- device discovery --------------------------------------------------- */

std::once_flag g_disc_once;
std::vector<int> g_devices;	/* HIP ordinals of usable gfx950 devices */

void discover()
{
	int n = 0;
	if (hipGetDeviceCount(&n) != hipSuccess)
		return;
	for (int d = 0; d < n; d++) {
		hipDeviceProp_t p;
		if (hipGetDeviceProperties(&p, d) != hipSuccess)
			continue;
		if (strncmp(p.gcnArchName, "gfx950", 6) == 0)
			g_devices.push_back(d);
	}
}

const std::vector<int> &devices()
{
	std::call_once(g_disc_once, discover);
	return g_devices;
}

/*
 * Devices a host-memory batch (net2_sha2_batch) is sharded over.  Test
 * knob NET2_SHA2_VIRTUAL_DEVICES=k (read per call): every real device is
 * listed k times, so each entry gets its own DeviceCtx, stream pair and
 * host thread and the multi-device slicing runs on a one-GPU machine.
 */
std::vector<int> batch_devices()
{
	std::vector<int> dv = devices();
	const char *v = getenv("NET2_SHA2_VIRTUAL_DEVICES");
	const int k = v != nullptr ? atoi(v) : 1;
	if (k > 1 && k <= 64 && !dv.empty()) {
		const std::vector<int> real = dv;
		for (int r = 1; r < k; r++)
			dv.insert(dv.end(), real.begin(), real.end());
	}
	return dv;
}

/*
 * Least payload per device slice of net2_sha2_batch (NET2_SHA2_SLICE_MIN_BYTES,
 * read per call; default 16 MiB, 0 = no limit).  A small batch's latency is
 * one lane's serial chain of compressions, which more devices do not
 * shorten, while each extra device costs a host thread, its own copies and
 * a synchronisation: a 4096 x 1 KiB signing tick stays on one GPU, a 1 GiB
 * batch spreads over eight.
 */
uint64_t slice_min_bytes()
{
	const char *v = getenv("NET2_SHA2_SLICE_MIN_BYTES");
	if (v == nullptr || *v == '\0')
		return 16ull << 20;
	return strtoull(v, nullptr, 10);
}

/* Is the calling thread's current device one we built code for? */
int check_current_device()
{
	int cur = -1;
	const std::vector<int> &dv = devices();
	if (dv.empty())
		return ENODEV;
	if (hipGetDevice(&cur) != hipSuccess)
		return ENODEV;
	return std::find(dv.begin(), dv.end(), cur) != dv.end() ? 0 : ENODEV;
}

/* ---- per-device staging for the host-memory paths -------------------- */

/*
 * One pipeline slot: pinned input and digest staging, device input,
 * offsets/lengths and digests, binning workspace, and a stream.  Two slots
 * per device double-buffer host gather / H2D / kernel / D2H.
 */
struct Slot {
	hipStream_t stream = nullptr;
	hipEvent_t done = nullptr;
	bool busy = false;
	uint8_t *h_in = nullptr, *h_dig = nullptr;
	/* a chunk's offsets (8 n bytes) then lengths (4 n): one copy */
	uint64_t *h_off = nullptr;
	uint8_t *d_in = nullptr, *d_dig = nullptr;
	uint64_t *d_off = nullptr;
	uint32_t *d_ws = nullptr;
	size_t cap_in = 0, cap_n = 0;
	/* digests of the chunk in flight go back to the caller here */
	uint8_t *user_dig = nullptr;
	size_t user_bytes = 0;

	void release()
	{
		if (h_in) (void)hipHostFree(h_in);
		if (h_dig) (void)hipHostFree(h_dig);
		if (h_off) (void)hipHostFree(h_off);
		if (d_in) (void)hipFree(d_in);
		if (d_dig) (void)hipFree(d_dig);
		if (d_off) (void)hipFree(d_off);
		if (d_ws) (void)hipFree(d_ws);
		h_in = h_dig = nullptr;
		h_off = nullptr;
		d_in = d_dig = nullptr;
		d_off = nullptr;
		d_ws = nullptr;
		cap_in = cap_n = 0;
	}

	/*
	 * Grow to hold `in` payload bytes and `n` packets.  host_in == false:
	 * the payload is DMA'd straight from the caller's pinned memory, so
	 * no pinned input staging is allocated (or kept) for it.
	 */
	int reserve(size_t in, size_t n, bool host_in = true)
	{
		if (stream == nullptr) {
			HIP_TRY(hipStreamCreateWithFlags(&stream,
			    hipStreamNonBlocking));
			HIP_TRY(hipEventCreateWithFlags(&done,
			    hipEventDisableTiming));
		}
		if (in <= cap_in && n <= cap_n && (!host_in || h_in != nullptr))
			return 0;
		/* grow both dimensions monotonically, with headroom: chunks of a
		 * variable-length batch differ slightly in bytes and packet count,
		 * and re-sizing to each one exactly re-allocated the pinned
		 * buffers (~10 ms) on every other chunk */
		in = std::max<size_t>({in + in / 8, cap_in, 4096});
		n = std::max<size_t>({n + n / 4, cap_n, 64});
		release();
		if (host_in)
			HIP_TRY(hipHostMalloc((void **)&h_in, in,
			    hipHostMallocDefault));
		HIP_TRY(hipHostMalloc((void **)&h_dig, n * 64,
		    hipHostMallocDefault));
		HIP_TRY(hipHostMalloc((void **)&h_off, n * 12,
		    hipHostMallocDefault));
		HIP_TRY(hipMalloc((void **)&d_in, in));
		HIP_TRY(hipMalloc((void **)&d_dig, n * 64));
		HIP_TRY(hipMalloc((void **)&d_off, n * 12));
		HIP_TRY(hipMalloc((void **)&d_ws,
		    (NET2_BIN_WS_WORDS + n) * sizeof(uint32_t)));
		/* prepared once, so the first variable-layout chunk bins too */
		HIP_TRY(net2_bin_ws_init((uint32_t *)d_ws, nullptr));
		HIP_TRY(hipStreamSynchronize(nullptr));
		cap_in = in;
		cap_n = n;
		return 0;
	}
};

/*
 * Host worker threads for packing staged chunks, kept alive between chunks
 * and calls: spawning and joining 16 threads twice per 64 MiB chunk cost
 * about a third of the pack itself.  run(nt, f) calls f(0) on the caller and
 * f(1..nt-1) on workers and returns when all are done.  Workers that took
 * part in a job spin for about half a millisecond after it, the others for
 * 50 us after seeing one (a chunk runs a small job and then a full-width
 * one back to back), then sleep on a condition variable: every worker
 * spinning half a millisecond after every job burnt ~6 CPUs during a 1
 * M-datagram host burst (tools/burst_debug_timing.py), none spinning after
 * a job it sat out cost the pageable host bursts 8-40 % (the full-width
 * pack waited for sleeping workers).  This way: ~34 ms of CPU per 1 M
 * datagrams against ~105, call times the same or better
 * (profiles/round6/spin_ab/).  The job word packs the
 * generation with nt, so a worker that wakes late never runs a job it is
 * not counted in.  Pools are never destroyed (their threads are detached
 * and may be parked at process exit).  One job at a time: job_, pending_
 * and word_ describe a single job, so run() is serialised by run_mu_ -- a
 * device's pool is shared by net2_sha2_batch and the host packet bursts,
 * which hold different locks and may run at once on one device.
 */
#ifndef NET2_POOL_SPIN_US
#define NET2_POOL_SPIN_US 500
#endif
/* keyed host bursts of at most this many datagrams read their datagrams and
 * metadata through the host mapping (enqueue_burst_steps) */
#ifndef NET2_BURST_ZC_MAX
#define NET2_BURST_ZC_MAX 16384
#endif
#ifndef NET2_POOL_SPIN_IDLE_US
#define NET2_POOL_SPIN_IDLE_US 50
#endif

class WorkPool {
public:
	template <class F>
	void run(size_t nt, const F &f)
	{
		if (nt <= 1) {
			f((size_t)0);
			return;
		}
		std::lock_guard<std::mutex> one(run_mu_);
		grow(nt - 1);
		const std::function<void(size_t)> job = f;
		job_ = &job;
		pending_.store(nt - 1, std::memory_order_relaxed);
		{
			std::lock_guard<std::mutex> g(m_);
			word_.store(((word_.load(std::memory_order_relaxed) >> 8) + 1)
			    << 8 | nt, std::memory_order_release);
		}
		cv_.notify_all();
		f((size_t)0);
		while (pending_.load(std::memory_order_acquire) != 0)
			__builtin_ia32_pause();
	}

private:
	void grow(size_t want)
	{
		/* a new worker starts from the word before this job's bump */
		const uint64_t now = word_.load(std::memory_order_relaxed);
		while (nworkers_ < want) {
			const size_t idx = ++nworkers_;
			std::thread([this, idx, now]() { worker(idx, now); })
			    .detach();
		}
	}

	void worker(size_t idx, uint64_t seen)
	{
		/* named, so per-thread CPU time can be told apart
		 * (/proc/<pid>/task/<tid>/comm, tools/burst_debug_timing.py) */
		pthread_setname_np(pthread_self(), "net2-pack");
		bool ran = false;	/* took part in the last job */
		for (;;) {
			uint64_t w = seen;
			const double t0 = dbg_clock();
			const double spin_ms = (ran ? NET2_POOL_SPIN_US :
			    NET2_POOL_SPIN_IDLE_US) * 1e-3;
			for (unsigned i = 1; w == seen; i++) {
				__builtin_ia32_pause();
				w = word_.load(std::memory_order_acquire);
				if ((i & 255) == 0 && dbg_clock() - t0 > spin_ms)
					break;
			}
			if (w == seen) {
				std::unique_lock<std::mutex> lk(m_);
				cv_.wait(lk, [&]() {
					return word_.load(std::memory_order_acquire)
					    != seen;
				});
				w = word_.load(std::memory_order_acquire);
			}
			seen = w;
			ran = idx < (w & 0xff);
			if (ran) {
				(*job_)(idx);
				pending_.fetch_sub(1, std::memory_order_release);
			}
		}
	}

	static double dbg_clock()
	{
		struct timespec ts;
		clock_gettime(CLOCK_MONOTONIC, &ts);
		return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
	}

	std::atomic<uint64_t> word_{0};	/* generation << 8 | nt */
	std::atomic<size_t> pending_{0};
	const std::function<void(size_t)> *job_ = nullptr;
	size_t nworkers_ = 0;
	std::mutex run_mu_;	/* one run() at a time */
	std::mutex m_;
	std::condition_variable cv_;
};

struct DeviceCtx {
	WorkPool *pool = new WorkPool();	/* never freed, see WorkPool */
	std::mutex mu;		/* one host-memory batch per device at a time */
	Slot slot[2];
	/* net2_sha2_numa_stats: slices run, and those whose thread was on
	 * the device's NUMA node when it finished */
	std::atomic<uint64_t> slices{0}, slices_on_node{0};
};

std::mutex g_ctx_mu;
std::vector<std::unique_ptr<DeviceCtx>> g_ctx;

DeviceCtx *ctx_for(size_t idx)
{
	std::lock_guard<std::mutex> g(g_ctx_mu);
	if (g_ctx.size() <= idx)
		g_ctx.resize(idx + 1);
	if (!g_ctx[idx])
		g_ctx[idx].reset(new DeviceCtx());
	return g_ctx[idx].get();
}

/*
 * NUMA placement of a device's host-side work.  A host-memory batch is
 * sharded over every GPU, one host thread per device (net2_sha2_batch); the
 * thread packs pageable input into pinned staging, and the staging is
 * allocated (and first touched) by it.  On a two-socket host half of the
 * GPUs hang off the other socket, so an unplaced thread pulls its slice's
 * ~55 GB/s of H2D traffic across the socket link.  The slice thread -- and
 * the pack pool threads it starts, which inherit its mask -- is bound to the
 * CPUs of the device's node (sysfs numa_node of its PCI function, within the
 * process's CPUs) for the slice, and restored after.  NET2_SHA2_NUMA=0
 * turns it off.  Slice 0 runs on the calling thread, so for the duration of
 * a net2_sha2_batch call that thread's affinity is the node's CPUs (its own
 * mask is restored before the call returns; include/net2/sha2_batch.h).
 */
struct NumaPlace {
	int node = -1;
	bool have = false;	/* cpus holds at least one usable CPU */
	cpu_set_t cpus;
};

bool parse_cpulist(const char *s, cpu_set_t *set)
{
	CPU_ZERO(set);
	while (*s && *s != '\n') {
		char *e;
		long a = strtol(s, &e, 10), b = a;
		if (e == s)
			return false;
		if (*e == '-') {
			s = e + 1;
			b = strtol(s, &e, 10);
			if (e == s)
				return false;
		}
		for (long c = a; c <= b && c < CPU_SETSIZE; c++)
			if (c >= 0)
				CPU_SET((int)c, set);
		s = *e == ',' ? e + 1 : e;
	}
	return true;
}

/*
 * The CPUs this process may run on, whoever asks: the cgroup's effective
 * cpuset when it is readable, else the affinity of the thread that loaded
 * the library.  Not the calling thread's own mask: a caller pinned to one
 * CPU must not narrow the placement every later slice of the device gets
 * (the result is cached per device).
 */
cpu_set_t g_load_mask;
bool g_load_mask_ok = false;

__attribute__((constructor)) void capture_load_mask()
{
	g_load_mask_ok = sched_getaffinity(0, sizeof(g_load_mask),
	    &g_load_mask) == 0;
}

bool process_cpus(cpu_set_t *out)
{
	char buf[4096];
	FILE *f = fopen("/sys/fs/cgroup/cpuset.cpus.effective", "r");
	if (f != nullptr) {
		const bool ok = fgets(buf, sizeof(buf), f) != nullptr &&
		    parse_cpulist(buf, out) && CPU_COUNT(out) > 0;
		fclose(f);
		if (ok)
			return true;
	}
	if (g_load_mask_ok) {
		*out = g_load_mask;
		return true;
	}
	return sched_getaffinity(0, sizeof(*out), out) == 0;
}

const NumaPlace &numa_place(int ordinal)
{
	static std::mutex mu;
	static std::vector<std::unique_ptr<NumaPlace>> cache;
	std::lock_guard<std::mutex> g(mu);
	if (cache.size() <= (size_t)ordinal)
		cache.resize((size_t)ordinal + 1);
	if (cache[ordinal])
		return *cache[ordinal];
	std::unique_ptr<NumaPlace> p(new NumaPlace());
	CPU_ZERO(&p->cpus);
	char bus[64] = { 0 }, path[160], buf[4096];
	if (hipDeviceGetPCIBusId(bus, sizeof(bus) - 1, ordinal) == hipSuccess) {
		for (char *c = bus; *c; c++)
			if (*c >= 'A' && *c <= 'F')
				*c = (char)(*c - 'A' + 'a');
		snprintf(path, sizeof(path), "/sys/bus/pci/devices/%s/numa_node",
		    bus);
		FILE *f = fopen(path, "r");
		if (f != nullptr) {
			if (fscanf(f, "%d", &p->node) != 1)
				p->node = -1;
			fclose(f);
		}
	} else {
		(void)hipGetLastError();
	}
	if (p->node >= 0) {
		snprintf(path, sizeof(path),
		    "/sys/devices/system/node/node%d/cpulist", p->node);
		FILE *f = fopen(path, "r");
		cpu_set_t node_cpus, mine;
		if (f != nullptr && fgets(buf, sizeof(buf), f) != nullptr &&
		    parse_cpulist(buf, &node_cpus) && process_cpus(&mine)) {
			CPU_AND(&p->cpus, &node_cpus, &mine);
			p->have = CPU_COUNT(&p->cpus) > 0;
		}
		if (f != nullptr)
			fclose(f);
	}
	cache[ordinal] = std::move(p);
	return *cache[ordinal];
}

bool numa_enabled()
{
	const char *e = getenv("NET2_SHA2_NUMA");
	return e == nullptr || strcmp(e, "0") != 0;
}

/* Binds the calling thread to a device's node for its lifetime. */
class NumaBind {
public:
	explicit NumaBind(const NumaPlace &np)
	{
		if (!np.have || !numa_enabled())
			return;
		if (pthread_getaffinity_np(pthread_self(), sizeof(saved_),
		    &saved_) == 0 && pthread_setaffinity_np(pthread_self(),
		    sizeof(np.cpus), &np.cpus) == 0)
			bound_ = true;
	}
	~NumaBind()
	{
		if (bound_)
			(void)pthread_setaffinity_np(pthread_self(),
			    sizeof(saved_), &saved_);
	}
private:
	cpu_set_t saved_;
	bool bound_ = false;
};

/* Chunk payload target for the host pipeline. */
constexpr size_t kChunkBytes = 64u << 20;

/* Page-locked (pinned or registered) host memory can be DMA'd directly. */
bool is_pinned(const void *p)
{
	hipPointerAttribute_t a;
	if (p == nullptr || hipPointerGetAttributes(&a, p) != hipSuccess) {
		(void)hipGetLastError();	/* clear the sticky lookup error */
		return false;
	}
	return a.type == hipMemoryTypeHost;
}

/*
 * [p, p + bytes) lies in one page-locked allocation, so the GPU may DMA from
 * it or store into it through its device mapping: both ends are page-locked,
 * map to the device at the same distance as on the host, and belong to the
 * same allocation (the same HIP buffer id).
 * A range that only starts in a registered region -- or spans two adjacent
 * page-locked allocations -- fails, and the caller stages it instead.
 */
bool pinned_span(const void *p, size_t bytes)
{
	if (p == nullptr || bytes == 0)
		return false;
	const uint8_t *a = (const uint8_t *)p, *b = a + bytes - 1;
	hipPointerAttribute_t pa, pb;
	if (hipPointerGetAttributes(&pa, a) != hipSuccess ||
	    hipPointerGetAttributes(&pb, b) != hipSuccess) {
		(void)hipGetLastError();
		return false;
	}
	if (pa.type != hipMemoryTypeHost || pb.type != hipMemoryTypeHost ||
	    pa.devicePointer == nullptr ||
	    (const uint8_t *)pb.devicePointer - (const uint8_t *)pa.devicePointer !=
	    (ptrdiff_t)(bytes - 1))
		return false;
	/* hipMemGetAddressRange reports no base for hipHostRegister'ed memory
	 * on this runtime; the buffer id names the allocation for both kinds
	 * (tools/ptr_probe.py, profiles/round6/ptr_probe.txt) */
	unsigned long long ida = 0, idb = 0;
	if (hipPointerGetAttribute(&ida, HIP_POINTER_ATTRIBUTE_BUFFER_ID,
	    (hipDeviceptr_t)a) != hipSuccess ||
	    hipPointerGetAttribute(&idb, HIP_POINTER_ATTRIBUTE_BUFFER_ID,
	    (hipDeviceptr_t)b) != hipSuccess) {
		(void)hipGetLastError();
		return false;
	}
	return ida == idb && ida != 0;
}

/* memcpy of a large range split over the pool's threads (staging copies). */
void par_memcpy(WorkPool &pool, uint8_t *dst, const uint8_t *src,
    size_t bytes)
{
	const size_t piece = 8u << 20;
	if (bytes == 0)		/* n empty packets at stride 0 */
		return;
	const size_t nt = std::min<size_t>(8, (bytes + piece - 1) / piece);
	pool.run(nt, [=](size_t t) {
		const size_t a = bytes * t / nt, b = bytes * (t + 1) / nt;
		memcpy(dst + a, src + a, b - a);
	});
}

/* NET2_SHA2_DEBUG_TIMING=1: per-chunk host timings on stderr. */
bool dbg_timing()
{
	static const bool on = getenv("NET2_SHA2_DEBUG_TIMING") != nullptr;
	return on;
}
double dbg_now()
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

/*
 * Pack n packets into pinned staging with 16-byte aligned starts and write
 * their staged offsets and lengths, split over up to kPackThreads threads
 * (the CPU share of one GPU on an MI355X node): pack_sizes sums each
 * thread's range of padded lengths (the chunk's byte count, and each
 * range's start), pack_fill then writes offsets and copies packets.  A
 * serial scan and gather over MTU-sized datagrams held the host path well
 * below the PCIe rate.
 */
#ifndef NET2_PACK_THREADS
#define NET2_PACK_THREADS 16
#endif
constexpr size_t kPackThreads = NET2_PACK_THREADS;

struct PackPlan {
	size_t nt = 1;
	size_t start[kPackThreads + 1] = {};	/* start[nt] = total bytes */
};

PackPlan pack_sizes(WorkPool &pool, const uint32_t *lens, uint64_t n,
    int per_shift = 12)
{
	PackPlan pl;
	/* one thread per 2^per_shift packets: ~4 K by default (the fill copies
	 * ~MiBs each) */
	pl.nt = std::min<size_t>(kPackThreads, std::max<size_t>(1,
	    n >> per_shift));
	size_t *st = pl.start;
	const size_t nt = pl.nt;
	pool.run(nt, [=](size_t t) {
		size_t sum = 0;
		for (uint64_t i = n * t / nt; i < n * (t + 1) / nt; i++)
			sum += ((size_t)lens[i] + 15) & ~(size_t)15;
		st[t + 1] = sum;
	});
	for (size_t t = 1; t <= nt; t++)
		st[t] += st[t - 1];
	return pl;
}

void pack_fill(WorkPool &pool, const PackPlan &pl, uint8_t *dst, uint64_t *dst_off,
    uint32_t *dst_len, const uint8_t *base, const uint64_t *offsets,
    const uint32_t *lens, uint64_t n)
{
	const size_t nt = pl.nt;
	const size_t *st = pl.start;
	pool.run(nt, [=](size_t t) {
		size_t at = st[t];
		for (uint64_t i = n * t / nt; i < n * (t + 1) / nt; i++) {
			const uint32_t l = lens[i];
			dst_off[i] = at;
			dst_len[i] = l;
			memcpy(dst + at, base + offsets[i], l);
			at += ((size_t)l + 15) & ~(size_t)15;
		}
	});
}

/*
 * Digests of the host path: the kernel stores them straight into pinned
 * host memory (the caller's buffer when it is pinned, else the slot's
 * staging) through its device mapping, so a chunk costs one H2D copy and no
 * D2H copy.  With a D2H copy per chunk the copies of every slot shared one
 * DMA queue in submission order: chunk k's D2H, waiting for its kernel,
 * held chunk k+1's H2D back, and the path ran at 91 % of the link's copy
 * rate.  NET2_SHA2_D2H_COPY=1 restores the copy (A/B).
 */
bool d2h_copy()
{
	static const bool on = getenv("NET2_SHA2_D2H_COPY") != nullptr &&
	    atoi(getenv("NET2_SHA2_D2H_COPY")) != 0;
	return on;
}

/*
 * The byte range [*rs, *re) (offsets from base) of packets off / ln [0, n)
 * when it can be DMA'd as it lies: within one page-locked allocation
 * (pinned_span) and dense -- at most a
 * quarter more bytes than the packets themselves, as when a receive loop
 * fills one pinned arena back to back.
 */
bool dense_pinned(WorkPool &pool, const uint8_t *base, const uint64_t *off,
    const uint32_t *ln, uint64_t n, uint64_t *rs, uint64_t *re)
{
	const size_t nt = std::min<size_t>(kPackThreads,
	    std::max<size_t>(1, n >> 14));
	uint64_t lo_t[kPackThreads], hi_t[kPackThreads], sum_t[kPackThreads];
	pool.run(nt, [&](size_t t) {
		uint64_t a = UINT64_MAX, b = 0, m = 0;
		for (uint64_t j = n * t / nt; j < n * (t + 1) / nt; j++) {
			a = std::min<uint64_t>(a, off[j]);
			b = std::max<uint64_t>(b, off[j] + ln[j]);
			m += ln[j];
		}
		lo_t[t] = a;
		hi_t[t] = b;
		sum_t[t] = m;
	});
	uint64_t a = UINT64_MAX, b = 0, m = 0;
	for (size_t t = 0; t < nt; t++) {
		a = std::min(a, lo_t[t]);
		b = std::max(b, hi_t[t]);
		m += sum_t[t];
	}
	if (n == 0 || b <= a || b - a > m + m / 4 || !pinned_span(base + a, b - a))
		return false;
	*rs = a;
	*re = b;
	return true;
}

/*
 * One chunk [lo, hi) of the caller's packets into slot s: H2D (straight from
 * the caller's buffer when it is pinned -- for the variable layout when the
 * chunk's packets also lie densely, dense_pinned -- else through the slot's
 * pinned staging, packed with 16-byte aligned packet starts), kernel
 * writing the digests to pinned host memory (the caller's buffer when that
 * is pinned).
 */
int enqueue_chunk_steps(WorkPool &pool, Slot &s, int alg, const uint8_t *base,
    const uint64_t *offsets, const uint32_t *lens, uint64_t stride,
    uint32_t fixed_len, uint64_t lo, uint64_t hi, uint8_t *user_dig,
    bool src_pinned, bool dst_pinned)
{
	const uint64_t n = hi - lo;
	const int dl = digest_len(alg);
	size_t bytes;
	int rc;
	PackPlan plan;

	uint64_t rs = 0, re = 0;
	const bool var_direct = offsets != nullptr && src_pinned &&
	    dense_pinned(pool, base, offsets + lo, lens + lo, n, &rs, &re);
	if (offsets == nullptr) {
		bytes = src_pinned ? (size_t)(n - 1) * stride + fixed_len
		    : (size_t)n * ((fixed_len + 15) & ~15u);
	} else if (var_direct) {
		bytes = re - rs;
	} else {
		plan = pack_sizes(pool, lens + lo, n);
		bytes = plan.start[plan.nt];
	}
	const double tr0 = dbg_now();
	if ((rc = s.reserve(bytes, n, !((offsets == nullptr && src_pinned) ||
	    var_direct))) != 0)
		return rc;
	if (dbg_timing())
		fprintf(stderr, "net2: reserve %.3f ms\n", dbg_now() - tr0);
	/* where the kernel stores the digests (see d2h_copy) */
	uint8_t *const host_dig = dst_pinned ? user_dig : s.h_dig;
	uint8_t *kout = s.d_dig;
	bool direct = false;
	if (!d2h_copy()) {
		void *dp = nullptr;
		if (hipHostGetDevicePointer(&dp, host_dig, 0) == hipSuccess &&
		    dp != nullptr) {
			kout = static_cast<uint8_t *>(dp);
			direct = true;
		} else {
			(void)hipGetLastError();
		}
	}

	if (offsets == nullptr && src_pinned) {
		if (bytes != 0)
			HIP_TRY(hipMemcpyAsync(s.d_in, base + lo * stride,
			    bytes, hipMemcpyHostToDevice, s.stream));
		FI_POINT(FI_H2D);
		HIP_TRY(net2_launch_fixed(alg, s.d_in, stride, fixed_len, n,
		    kout, s.stream));
		FI_POINT(FI_KERNEL);
	} else if (offsets == nullptr) {
		const size_t st = (fixed_len + 15) & ~15u;
		if (st == stride) {
			/* contiguous; the caller's buffer ends at the last
			 * packet's last byte, not at a stride boundary */
			par_memcpy(pool, s.h_in, base + lo * stride,
			    (size_t)(n - 1) * stride + fixed_len);
		} else {
			const size_t nt = std::min<size_t>(kPackThreads,
			    std::max<size_t>(1, bytes >> 22));
			uint8_t *dst = s.h_in;
			const uint8_t *src = base + lo * stride;
			pool.run(nt, [=](size_t t) {
				for (uint64_t i = n * t / nt; i < n * (t + 1) / nt; i++)
					memcpy(dst + i * st, src + i * stride,
					    fixed_len);
			});
		}
		if (bytes != 0)
			HIP_TRY(hipMemcpyAsync(s.d_in, s.h_in, bytes,
			    hipMemcpyHostToDevice, s.stream));
		FI_POINT(FI_H2D);
		HIP_TRY(net2_launch_fixed(alg, s.d_in, st, fixed_len, n,
		    kout, s.stream));
		FI_POINT(FI_KERNEL);
	} else {
		const double tg0 = dbg_now();
		if (var_direct) {
			/* offsets from the range's start; the bytes as they lie
			 * (the kernel picks its address mode per wave) */
			const uint64_t *off = offsets + lo;
			const uint32_t *ln = lens + lo;
			uint64_t *ho = s.h_off;
			uint32_t *hl = (uint32_t *)(s.h_off + n);
			const size_t nt = std::min<size_t>(kPackThreads,
			    std::max<size_t>(1, n >> 14));
			pool.run(nt, [=](size_t t) {
				for (uint64_t j = n * t / nt; j < n * (t + 1) / nt;
				    j++) {
					ho[j] = off[j] - rs;
					hl[j] = ln[j];
				}
			});
		} else {
			pack_fill(pool, plan, s.h_in, s.h_off,
			    (uint32_t *)(s.h_off + n), base, offsets + lo,
			    lens + lo, n);
		}
		if (dbg_timing())
			fprintf(stderr, "net2: %s %zu B, %llu packets: %.3f ms\n",
			    var_direct ? "direct" : "pack", bytes,
			    (unsigned long long)n, dbg_now() - tg0);
		if (bytes != 0)
			HIP_TRY(hipMemcpyAsync(s.d_in, var_direct ? base + rs :
			    s.h_in, bytes, hipMemcpyHostToDevice, s.stream));
		HIP_TRY(hipMemcpyAsync(s.d_off, s.h_off, n * 12,
		    hipMemcpyHostToDevice, s.stream));
		FI_POINT(FI_H2D);
		HIP_TRY(net2_launch_var(alg, s.d_in, s.d_off,
		    (const uint32_t *)(s.d_off + n), n, kout,
		    n >= 4096 ? s.d_ws : nullptr, s.stream));
		FI_POINT(FI_KERNEL);
	}
	if (!direct)
		HIP_TRY(hipMemcpyAsync(host_dig, s.d_dig, (size_t)n * dl,
		    hipMemcpyDeviceToHost, s.stream));
	FI_POINT(FI_RECORD);
	HIP_TRY(hipEventRecord(s.done, s.stream));
	s.busy = true;
	s.user_dig = dst_pinned ? nullptr : user_dig;
	s.user_bytes = (size_t)n * dl;
	return 0;
}

/* enqueue_chunk_steps; a chunk that fails part-way is waited for (quiesce)
 * before the error goes back, and its slot stays free. */
int enqueue_chunk(WorkPool &pool, Slot &s, int alg, const uint8_t *base,
    const uint64_t *offsets, const uint32_t *lens, uint64_t stride,
    uint32_t fixed_len, uint64_t lo, uint64_t hi, uint8_t *user_dig,
    bool src_pinned, bool dst_pinned)
{
	const int rc = enqueue_chunk_steps(pool, s, alg, base, offsets, lens,
	    stride, fixed_len, lo, hi, user_dig, src_pinned, dst_pinned);
	if (rc != 0)
		quiesce(s.stream);
	return rc;
}

int drain(Slot &s)
{
	if (!s.busy)
		return 0;
	s.busy = false;
	HIP_TRY(hipEventSynchronize(s.done));
	if (s.user_dig != nullptr)
		memcpy(s.user_dig, s.h_dig, s.user_bytes);
	return 0;
}

/* One device's share of a host-memory batch. */
int run_device_slice(size_t didx, int ordinal, int alg, const uint8_t *base,
    const uint64_t *offsets, const uint32_t *lens, uint64_t stride,
    uint32_t fixed_len, uint64_t lo, uint64_t hi, uint8_t *digests)
{
	/* on the device's node before anything is allocated or touched */
	const NumaPlace &np = numa_place(ordinal);
	NumaBind bind(np);
	DeviceCtx *c = ctx_for(didx);
	std::lock_guard<std::mutex> g(c->mu);
	struct Count {
		DeviceCtx *c;
		const NumaPlace &np;
		~Count()
		{
			const int cpu = sched_getcpu();
			c->slices.fetch_add(1, std::memory_order_relaxed);
			if (np.node >= 0 && cpu >= 0 && CPU_ISSET(cpu, &np.cpus))
				c->slices_on_node.fetch_add(1,
				    std::memory_order_relaxed);
		}
	} count = { c, np };
	const int dl = digest_len(alg);
	int rc = 0, cur = 0;

	HIP_TRY(hipSetDevice(ordinal));
	/* fixed layout: DMA'd as it lies when the slice's whole span is in one
	 * page-locked allocation; variable: when its chunk's packets also lie
	 * densely in one (enqueue_chunk, dense_pinned).  Digests are stored
	 * through the output's mapping only when the slice's whole output range
	 * is in one page-locked allocation (pinned_span). */
	const bool src_pinned = offsets == nullptr ?
	    pinned_span(base + lo * stride, (size_t)(hi - 1 - lo) * stride +
	    fixed_len) : is_pinned(base);
	const bool dst_pinned = pinned_span(digests + lo * dl,
	    (size_t)(hi - lo) * dl);
	/*
	 * Packets per chunk: kChunkBytes of (padded) payload at the slice's
	 * mean packet size.  A chunk of unusually large packets just grows the
	 * staging (Slot::reserve); the exact byte count comes from pack_sizes.
	 */
	uint64_t per_chunk;
	if (offsets == nullptr) {
		/* the direct-DMA path copies whole strides (a chunk spans
		 * (n - 1) * stride + fixed_len bytes), the staged one packs
		 * packets at 16-byte granularity */
		const size_t per = std::max<size_t>(src_pinned ? stride :
		    (fixed_len + 15) & ~15u, 16);
		per_chunk = std::max<size_t>(kChunkBytes / per, 1);
	} else {
		const PackPlan all = pack_sizes(*c->pool, lens + lo, hi - lo);
		const size_t mean = std::max<size_t>(
		    all.start[all.nt] / std::max<uint64_t>(hi - lo, 1), 16);
		per_chunk = std::max<size_t>(kChunkBytes / mean, 1);
	}
	for (uint64_t at = lo; at < hi && rc == 0;) {
		const double tc0 = dbg_now();
		const uint64_t end = std::min<uint64_t>(hi, at + per_chunk);
		Slot &s = c->slot[cur];
		const double td0 = dbg_now();
		if ((rc = drain(s)) != 0)
			break;
		if (dbg_timing())
			fprintf(stderr, "net2: drain wait %.3f ms\n", dbg_now() - td0);
		const double te0 = dbg_now();
		rc = enqueue_chunk(*c->pool, s, alg, base, offsets, lens, stride,
		    fixed_len, at, end, digests + at * dl, src_pinned,
		    dst_pinned);
		if (dbg_timing())
			fprintf(stderr, "net2: enqueue %.3f ms (+%.3f ms before it)\n",
			    dbg_now() - te0, te0 - tc0);
		at = end;
		cur ^= 1;
	}
	int rc2 = drain(c->slot[0]);
	int rc3 = drain(c->slot[1]);
	return rc ? rc : rc2 ? rc2 : rc3;
}

/*
 * The calling thread's device selection (net2_sha2_set_device): an index
 * into the device list (batch_devices()), or -1 to follow the thread's
 * current HIP device.  Helper threads that run work submitted by another
 * thread (the signed carver's pool) take the submitter's selection.
 */
thread_local int tl_dev_sel = -1;

/* The device (index into dv = batch_devices()) a single-message call runs
 * on: the thread's selection; else its current HIP device when that is a
 * usable one (one process per GPU stays on its GPU); else the first. */
size_t small_device(const std::vector<int> &dv)
{
	if (tl_dev_sel >= 0 && (size_t)tl_dev_sel < dv.size())
		return (size_t)tl_dev_sel;
	int cur = -1;
	(void)hipGetDevice(&cur);
	for (size_t d = 0; d < dv.size(); d++)
		if (dv[d] == cur)
			return d;
	return 0;
}

/*
 * One persistent host thread per device index for the slices of a sharded
 * call (shard_batch): a thread created and joined per call cost ~30-60 us
 * per extra device on every net2_sha2_batch / host burst.  Jobs of
 * concurrent callers queue in order; a slice takes its device's lock anyway.
 * Workers are detached and live as long as the process.
 */
class SliceWorker {
public:
	void post(std::function<void()> f)
	{
		std::lock_guard<std::mutex> g(m_);
		if (!started_) {
			std::thread([this]() { loop(); }).detach();
			started_ = true;
		}
		q_.push_back(std::move(f));
		cv_.notify_one();
	}

private:
	void loop()
	{
		pthread_setname_np(pthread_self(), "net2-slice");
		for (;;) {
			std::function<void()> f;
			{
				std::unique_lock<std::mutex> lk(m_);
				cv_.wait(lk, [&]() { return !q_.empty(); });
				f = std::move(q_.front());
				q_.pop_front();
			}
			f();
		}
	}

	std::mutex m_;
	std::condition_variable cv_;
	std::deque<std::function<void()>> q_;
	bool started_ = false;
};

SliceWorker *slice_worker(size_t idx)
{
	static std::mutex mu;
	static std::vector<SliceWorker *> w;	/* never freed, see above */
	std::lock_guard<std::mutex> g(mu);
	if (w.size() <= idx)
		w.resize(idx + 1, nullptr);
	if (w[idx] == nullptr)
		w[idx] = new SliceWorker();
	return w[idx];
}

/*
 * Shards a host-memory batch of n packets over the devices (net2_sha2_batch,
 * the host packet bursts): contiguous slices -- by packet count for the
 * fixed layout (lens == NULL), by bytes otherwise -- no slice under
 * slice_min_bytes() of payload, each extra device's slice on that device's
 * persistent worker (SliceWorker).  The device list starts at the caller's
 * device (small_device), so one process per GPU with max_devices == 1 stays
 * on its own device.  fn(didx, ordinal, lo, hi)
 * runs one slice; the first error is returned.
 */
template <class F>
int shard_batch(uint64_t n, const uint32_t *lens, uint32_t fixed_len,
    int max_devices, const F &fn)
{
	const std::vector<int> dv = batch_devices();
	if (dv.empty())
		return ENODEV;
	size_t nd = dv.size();
	if (max_devices > 0 && (size_t)max_devices < nd)
		nd = (size_t)max_devices;
	if ((uint64_t)nd > n)
		nd = (size_t)n;
	uint64_t total = 0;
	if (lens == nullptr) {
		total = n * (uint64_t)fixed_len;
	} else {
		for (uint64_t i = 0; i < n; i++)
			total += lens[i];
	}
	const uint64_t min_slice = slice_min_bytes();
	if (min_slice > 0 && nd > 1)
		nd = (size_t)std::max<uint64_t>(1, std::min<uint64_t>(nd,
		    total / min_slice));

	/* Contiguous slices: by packet count, or by bytes for var layout. */
	std::vector<uint64_t> cut(nd + 1, 0);
	cut[nd] = n;
	if (lens == nullptr) {
		for (size_t d = 1; d < nd; d++)
			cut[d] = n * d / nd;
	} else {
		uint64_t acc = 0;
		size_t d = 1;
		for (uint64_t i = 0; i < n && d < nd; i++) {
			acc += lens[i];
			while (d < nd && acc * nd >= total * d)
				cut[d++] = i + 1;
		}
		for (; d < nd; d++)
			cut[d] = n;
	}

	int prev = -1;
	(void)hipGetDevice(&prev);
	const size_t first = small_device(dv);
	std::vector<int> rcs(nd, 0);
	struct {
		std::mutex m;
		std::condition_variable cv;
		size_t left;
	} done;
	done.left = nd - 1;
	for (size_t d = 1; d < nd; d++) {
		const size_t e = (first + d) % dv.size();
		slice_worker(e)->post([&, d, e]() {
			rcs[d] = fn(e, dv[e], cut[d], cut[d + 1]);
			std::lock_guard<std::mutex> g(done.m);
			if (--done.left == 0)
				done.cv.notify_all();
		});
	}
	rcs[0] = fn(first, dv[first], cut[0], cut[1]);
	{
		std::unique_lock<std::mutex> lk(done.m);
		done.cv.wait(lk, [&]() { return done.left == 0; });
	}
	if (prev >= 0)
		(void)hipSetDevice(prev);
	for (int r : rcs)
		if (r != 0)
			return r;
	return 0;
}

} /* namespace */

int net2_co_run(const net2co::Request &r)
{
	const std::vector<int> dv = batch_devices();
	if (dv.empty())
		return ENODEV;
	const size_t d = small_device(dv);
	int herr = 0;
	const int rc = net2co::submit(d, dv[d], r, &herr);
	if (rc == EIO)
		tl_last_hip_error = herr;
	return rc;
}

/* ---- exported C ABI ---------------------------------------------------- */

NET2_EXPORT int net2_coalesce_stats(int device, uint64_t *calls,
    uint64_t *launches)
{
	const std::vector<int> dv = batch_devices();
	if (dv.empty())
		return ENODEV;
	if (device < -1 || device >= (int)dv.size())
		return EINVAL;
	net2co::stats(device < 0 ? small_device(dv) : (size_t)device, calls,
	    launches);
	return 0;
}

NET2_EXPORT const int net2_hashmax = kNumRows;

NET2_EXPORT int net2_sha2_abi_version(void)
{
	return NET2_SHA2_ABI_VERSION;
}

NET2_EXPORT int net2_sha2_device_count(int *count)
{
	if (count == nullptr)
		return EINVAL;
	*count = (int)devices().size();
	return *count > 0 ? 0 : ENODEV;
}

NET2_EXPORT int net2_sha2_set_device(int index, int *prev)
{
	if (prev != nullptr)
		*prev = tl_dev_sel;
	if (index == -1) {
		tl_dev_sel = -1;
		return 0;
	}
	const std::vector<int> dv = batch_devices();
	if (dv.empty())
		return ENODEV;
	if (index < -1 || index >= (int)dv.size())
		return EINVAL;
	HIP_TRY(hipSetDevice(dv[index]));
	tl_dev_sel = index;
	return 0;
}

NET2_EXPORT int net2_sha2_get_device(int *index)
{
	if (index == nullptr)
		return EINVAL;
	const std::vector<int> dv = batch_devices();
	if (dv.empty())
		return ENODEV;
	*index = (int)small_device(dv);
	return 0;
}

#if NET2_FAULT_INJECT
NET2_EXPORT int net2_fault_inject(int site, int k)
{
	if (site < 0 || site > FI_RECORD || k < 0)
		return EINVAL;
	g_fi_site.store(0);
	g_fi_left.store(k);
	g_fi_site.store(k > 0 ? site : 0);
	return 0;
}
#endif

NET2_EXPORT int net2_sha2_last_hip_error(void)
{
	return tl_last_hip_error;
}

NET2_EXPORT const char *net2_sha2_strerror(int err)
{
	switch (err) {
	case 0: return "success";
	case EINVAL: return "invalid argument";
	case ENOMEM: return "out of memory";
	case ENODEV: return "no usable gfx950 (MI355X) device";
	case EIO: return "HIP runtime error";
	case ENOSYS: return "not implemented";
	default: return "unknown error";
	}
}

NET2_EXPORT int net2_sha2_dev_fixed(int alg, const void *d_base,
    uint64_t stride, uint32_t len, uint64_t n, void *d_digests, void *stream)
{
	if (!unkeyed_sha2(alg))
		return EINVAL;
	if (n == 0)
		return 0;
	if (d_digests == nullptr || (d_base == nullptr && len > 0))
		return EINVAL;
	if (n > 1 && stride < len)
		return EINVAL;
	int rc = check_current_device();
	if (rc != 0)
		return rc;
	HIP_TRY(net2_launch_fixed(alg, (const uint8_t *)d_base, stride, len, n,
	    (uint8_t *)d_digests, (hipStream_t)stream));
	return 0;
}

NET2_EXPORT size_t net2_sha2_dev_var_workspace(uint64_t n)
{
	return ((size_t)NET2_BIN_WS_WORDS + (size_t)n) * sizeof(uint32_t);
}

NET2_EXPORT int net2_sha2_workspace_init(void *d_ws, size_t ws_bytes,
    void *stream)
{
	if (d_ws == nullptr || ws_bytes < net2_sha2_dev_var_workspace(0) ||
	    ((uintptr_t)d_ws & 3) != 0)
		return EINVAL;
	int rc = check_current_device();
	if (rc != 0)
		return rc;
	HIP_TRY(net2_bin_ws_init((uint32_t *)d_ws, (hipStream_t)stream));
	return 0;
}

NET2_EXPORT int net2_sha2_bin_limits(uint32_t grid_cap, int64_t timeout_us)
{
	net2_bin_set_limits(grid_cap, timeout_us);
	return 0;
}

NET2_EXPORT int net2_sha2_workspace_stats(const void *d_ws, size_t ws_bytes,
    struct net2_bin_stats *st)
{
	if (d_ws == nullptr || st == nullptr ||
	    ws_bytes < net2_sha2_dev_var_workspace(0) ||
	    ((uintptr_t)d_ws & 7) != 0)
		return EINVAL;
	int rc = check_current_device();
	if (rc != 0)
		return rc;
	uint32_t h[NET2_BIN_HDR];
	HIP_TRY(hipMemcpy(h, d_ws, sizeof(h), hipMemcpyDeviceToHost));
	const uint64_t tag = (uint64_t)h[NET2_BIN_W_TAG + 1] << 32 |
	    h[NET2_BIN_W_TAG];
	st->prepared = (uint32_t)(tag >> 32) == 0x4e324253u;	/* "N2BS" */
	st->binned = h[NET2_BIN_W_BINNED];
	st->aborts = h[NET2_BIN_W_ABORTS];
	st->mismatches = h[NET2_BIN_W_MISMATCH];
	st->unprepared = h[NET2_BIN_W_UNPREP];
	return 0;
}

NET2_EXPORT int net2_sha2_dev_var(int alg, const void *d_base,
    const uint64_t *d_offsets, const uint32_t *d_lens, uint64_t n,
    void *d_digests, void *d_ws, size_t ws_bytes, void *stream)
{
	if (!unkeyed_sha2(alg))
		return EINVAL;
	if (n == 0)
		return 0;
	if (d_offsets == nullptr || d_lens == nullptr || d_digests == nullptr)
		return EINVAL;
	if (d_ws != nullptr && (ws_bytes < net2_sha2_dev_var_workspace(n) ||
	    ((uintptr_t)d_ws & 3) != 0 || n > UINT32_MAX))
		return EINVAL;
	int rc = check_current_device();
	if (rc != 0)
		return rc;
	HIP_TRY(net2_launch_var(alg, (const uint8_t *)d_base, d_offsets, d_lens,
	    n, (uint8_t *)d_digests, (uint32_t *)d_ws, (hipStream_t)stream));
	return 0;
}

NET2_EXPORT int net2_sha2_batch(int alg, const void *base,
    const uint64_t *offsets, const uint32_t *lens, uint64_t stride,
    uint32_t fixed_len, uint64_t n, void *digests, int max_devices)
{
	if (!unkeyed_sha2(alg))
		return EINVAL;
	if (n == 0)
		return 0;
	if (digests == nullptr || (offsets != nullptr && lens == nullptr))
		return EINVAL;
	if (offsets == nullptr && (base == nullptr && fixed_len > 0))
		return EINVAL;
	if (offsets == nullptr && n > 1 && stride < fixed_len)
		return EINVAL;
	return shard_batch(n, offsets != nullptr ? lens : nullptr, fixed_len,
	    max_devices, [&](size_t didx, int ordinal, uint64_t lo,
	    uint64_t hi) {
		return run_device_slice(didx, ordinal, alg,
		    (const uint8_t *)base, offsets, lens, stride, fixed_len,
		    lo, hi, (uint8_t *)digests);
	});
}

NET2_EXPORT int net2_sha2_numa_stats(int device, int *numa_node,
    uint64_t *slices, uint64_t *slices_on_node)
{
	const std::vector<int> dv = batch_devices();
	if (dv.empty())
		return ENODEV;
	if (device < 0 || (size_t)device >= dv.size())
		return EINVAL;
	const NumaPlace &np = numa_place(dv[device]);
	DeviceCtx *c = ctx_for((size_t)device);
	if (numa_node)
		*numa_node = np.node;
	if (slices)
		*slices = c->slices.load(std::memory_order_relaxed);
	if (slices_on_node)
		*slices_on_node = c->slices_on_node.load(std::memory_order_relaxed);
	return 0;
}

NET2_EXPORT const char *net2_hash_getname(int alg)
{
	return alg >= 0 && alg < kNumRows ? kRows[alg].name : nullptr;
}

NET2_EXPORT int net2_hash_findname(const char *name)
{
	if (name == nullptr)
		return -1;
	for (int i = 0; i < kNumRows; i++)
		if (strcmp(kRows[i].name, name) == 0)
			return i;
	return -1;
}

NET2_EXPORT int net2_hash_gethashlen(int alg)
{
	return alg >= 0 && alg < kNumRows ? kRows[alg].hashlen : -1;
}

NET2_EXPORT int net2_hash_getkeylen(int alg)
{
	return alg >= 0 && alg < kNumRows ? kRows[alg].keylen : -1;
}

/*
 * A message longer than this (NET2_SHA2_STREAM_CHUNK, default 64 MiB) is
 * hashed through the streaming context, whose Update sends it in requests
 * of at most that size: one request would stage the whole message in
 * page-locked memory.
 */
static size_t long_message_bytes()
{
	const char *e = getenv("NET2_SHA2_STREAM_CHUNK");
	return e != nullptr && *e != '\0' ? strtoull(e, nullptr, 10) :
	    (size_t)64 << 20;
}

/* net2_hashctx_hashiov of a long message: SHA*Init / Update per segment /
 * Final, and for HMAC the same over K' ^ ipad || m, then K' ^ opad || inner
 * (RFC 2104, as hash-openssl.cc's HMAC_* calls). */
static int hashiov_streamed(int alg, const void *key, size_t keylen,
    const struct iovec *iov, size_t iovcnt, uint8_t *out)
{
	const bool keyed = !unkeyed_sha2(alg);
	const int halg = keyed ? alg - 3 : alg;
	const size_t B = halg == NET2_HASH_SHA256 ? 64 : 128;
	uint8_t kp[128] = { 0 }, blk[128], inner[64];
	SHA2_CTX c;
	int rc;
	if (keyed) {
		if (keylen > B)
			return EINVAL;
		memcpy(kp, key, keylen);
	}
	if ((rc = net2_sha2_ctx_init(halg, &c)) != 0)
		return rc;
	if (keyed) {
		for (size_t i = 0; i < B; i++)
			blk[i] = kp[i] ^ 0x36;
		if ((rc = net2_sha2_ctx_update(halg, &c, blk, B)) != 0)
			return rc;
	}
	{
		/* many small segments are gathered into requests of up to one
		 * stream chunk (one GPU round trip each, not one per segment);
		 * a segment of a chunk or more with nothing gathered goes as is */
		const size_t chunk = std::max(long_message_bytes(), B);
		std::vector<uint8_t> gbuf;
		size_t have = 0;
		for (size_t i = 0; i < iovcnt; i++) {
			const uint8_t *q = (const uint8_t *)iov[i].iov_base;
			size_t left = iov[i].iov_len;
			if (have == 0 && left >= chunk) {
				if ((rc = net2_sha2_ctx_update(halg, &c, q, left)) != 0)
					return rc;
				continue;
			}
			while (left > 0) {
				if (gbuf.empty())
					gbuf.resize(chunk);
				const size_t take = std::min(left, chunk - have);
				memcpy(gbuf.data() + have, q, take);
				have += take;
				q += take;
				left -= take;
				if (have == chunk) {
					if ((rc = net2_sha2_ctx_update(halg, &c,
					    gbuf.data(), have)) != 0)
						return rc;
					have = 0;
				}
			}
		}
		if (have > 0 && (rc = net2_sha2_ctx_update(halg, &c, gbuf.data(),
		    have)) != 0)
			return rc;
	}
	if ((rc = net2_sha2_ctx_final(halg, keyed ? inner : out, &c)) != 0 ||
	    !keyed)
		return rc;
	for (size_t i = 0; i < B; i++)
		blk[i] = kp[i] ^ 0x5c;
	if ((rc = net2_sha2_ctx_init(halg, &c)) != 0 ||
	    (rc = net2_sha2_ctx_update(halg, &c, blk, B)) != 0 ||
	    (rc = net2_sha2_ctx_update(halg, &c, inner,
	    (size_t)kRows[alg].hashlen)) != 0)
		return rc;
	return net2_sha2_ctx_final(halg, out, &c);
}

NET2_EXPORT int net2_hashctx_hashiov(int alg, const void *key, size_t keylen,
    const struct iovec *iov, size_t iovcnt, void *out, size_t outlen)
{
	if (alg < 0 || alg >= kNumRows)
		return EINVAL;
	if ((size_t)kRows[alg].keylen != keylen ||
	    (keylen > 0 && key == nullptr))
		return EINVAL;
	if (iovcnt > 0 && iov == nullptr)
		return EINVAL;
	if (alg == NET2_HASH_NIL)
		return 0;
	if (out == nullptr || outlen < (size_t)kRows[alg].hashlen)
		return EINVAL;
	size_t total = 0;
	for (size_t i = 0; i < iovcnt; i++)
		total += iov[i].iov_len;
	if (total > long_message_bytes())
		return hashiov_streamed(alg, key, keylen, iov, iovcnt,
		    (uint8_t *)out);
	/* one coalesced request: concurrent callers share a launch */
	net2co::Request r = {};
	r.kind = unkeyed_sha2(alg) ? net2co::DIGEST : net2co::HMAC;
	r.alg = unkeyed_sha2(alg) ? alg : alg - 3;
	r.iov = iov;
	r.iovcnt = iovcnt;
	r.key = (const uint8_t *)key;
	r.keylen = keylen;
	r.out = (uint8_t *)out;
	return net2_co_run(r);
}

/* Argument checks shared by the datagram sign / verify entry points. */
static int check_dgram_args(int alg, const void *key, size_t keylen,
    const void *d_base, const uint64_t *d_offsets, const uint32_t *d_lens,
    uint64_t n, const void *d_ws, size_t ws_bytes)
{
	if (alg < NET2_HASH_HMAC_SHA256 || alg > NET2_HASH_HMAC_SHA512)
		return EINVAL;
	if ((size_t)kRows[alg].keylen != keylen || key == nullptr)
		return EINVAL;
	if (n == 0)
		return 0;
	if (d_base == nullptr || d_offsets == nullptr || d_lens == nullptr)
		return EINVAL;
	if (d_ws != nullptr && (ws_bytes < net2_sha2_dev_var_workspace(n) ||
	    ((uintptr_t)d_ws & 3) != 0 || n > UINT32_MAX))
		return EINVAL;
	return check_current_device();
}

NET2_EXPORT int net2_hmac_sign_dev(int alg, const void *key, size_t keylen,
    void *d_base, const uint64_t *d_offsets, const uint32_t *d_lens,
    uint64_t n, void *d_ws, size_t ws_bytes, void *stream)
{
	int rc = check_dgram_args(alg, key, keylen, d_base, d_offsets, d_lens,
	    n, d_ws, ws_bytes);
	if (rc != 0 || n == 0)
		return rc;
	HIP_TRY(net2_launch_hmac(alg, (const uint8_t *)key, keylen,
	    (const uint8_t *)d_base, d_offsets, d_lens, 0, 0, n,
	    (uint8_t *)d_base, (uint32_t *)d_ws, (hipStream_t)stream,
	    NET2_HMAC_MODE_SIGN));
	return 0;
}

NET2_EXPORT int net2_hmac_verify_dev(int alg, const void *key,
    size_t keylen, const void *d_base, const uint64_t *d_offsets,
    const uint32_t *d_lens, uint64_t n, uint8_t *d_result, void *d_ws,
    size_t ws_bytes, void *stream)
{
	int rc = check_dgram_args(alg, key, keylen, d_base, d_offsets, d_lens,
	    n, d_ws, ws_bytes);
	if (rc != 0 || n == 0)
		return rc;
	if (d_result == nullptr)
		return EINVAL;
	HIP_TRY(net2_launch_hmac(alg, (const uint8_t *)key, keylen,
	    (const uint8_t *)d_base, d_offsets, d_lens, 0, 0, n, d_result,
	    (uint32_t *)d_ws, (hipStream_t)stream, NET2_HMAC_MODE_VERIFY));
	return 0;
}

NET2_EXPORT int net2_hmac_dev(int alg, const void *key, size_t keylen,
    const void *d_base, const uint64_t *d_offsets, const uint32_t *d_lens,
    uint64_t stride, uint32_t fixed_len, uint64_t n, void *d_digests,
    void *d_ws, size_t ws_bytes, void *stream)
{
	if (alg < NET2_HASH_HMAC_SHA256 || alg > NET2_HASH_HMAC_SHA512)
		return EINVAL;
	if ((size_t)kRows[alg].keylen != keylen || key == nullptr)
		return EINVAL;
	if (n == 0)
		return 0;
	if (d_digests == nullptr)
		return EINVAL;
	if (d_offsets != nullptr) {
		if (d_lens == nullptr)
			return EINVAL;
		if (d_ws != nullptr && (ws_bytes < net2_sha2_dev_var_workspace(n) ||
		    ((uintptr_t)d_ws & 3) != 0 || n > UINT32_MAX))
			return EINVAL;
	} else {
		if (d_base == nullptr && fixed_len > 0)
			return EINVAL;
		if (n > 1 && stride < fixed_len)
			return EINVAL;
	}
	int rc = check_current_device();
	if (rc != 0)
		return rc;
	HIP_TRY(net2_launch_hmac(alg, (const uint8_t *)key, keylen,
	    (const uint8_t *)d_base, d_offsets, d_lens, stride, fixed_len, n,
	    (uint8_t *)d_digests, d_offsets ? (uint32_t *)d_ws : nullptr,
	    (hipStream_t)stream));
	return 0;
}

NET2_EXPORT int net2_ph_to_iv_buf(const struct net2_packet_header *ph,
    size_t ivlen, void *iv)
{
	uint8_t hdr[8];
	uint8_t *out = (uint8_t *)iv;
	uint8_t d[32];
	size_t have = 0;

	if (ph == nullptr || (iv == nullptr && ivlen > 0))
		return EINVAL;
	for (int i = 0; i < 4; i++) {
		hdr[i] = (uint8_t)(ph->seq >> (24 - 8 * i));
		hdr[4 + i] = (uint8_t)(ph->flags >> (24 - 8 * i));
	}
	while (have < ivlen) {		/* packet.n2t:127-144 */
		struct iovec v[2] = { { hdr, sizeof(hdr) }, { out, have } };
		int rc = net2_hashctx_hashiov(NET2_HASH_SHA256, nullptr, 0, v, 2,
		    d, sizeof(d));
		if (rc != 0)
			return rc;
		size_t take = std::min<size_t>(32, ivlen - have);
		memcpy(out + have, d, take);
		have += take;
	}
	return 0;
}

NET2_EXPORT int net2_ph_to_iv_dev(const uint32_t *d_seq,
    const uint32_t *d_flags, uint64_t n, uint32_t ivlen, void *d_iv,
    void *stream)
{
	if (n == 0 || ivlen == 0)
		return 0;
	if (ivlen > 64 || d_seq == nullptr || d_flags == nullptr ||
	    d_iv == nullptr)
		return EINVAL;
	int rc = check_current_device();
	if (rc != 0)
		return rc;
	HIP_TRY(net2_launch_ph_iv(d_seq, d_flags, n, ivlen, (uint8_t *)d_iv,
	    (hipStream_t)stream));
	return 0;
}

/* ---- packet bursts (include/net2/packet.h) --------------------------------- */

namespace {

/* Workspace of a burst, carved in this order, every piece 16-byte aligned:
 * the binning scratch first -- its header and histograms at offset 0 for
 * every n, so one workspace serves bursts of any size up to its own and
 * net2_sha2_workspace_init / _stats apply to it -- then region offsets and
 * lengths for the prep kernel, status and verdict bytes, decoded headers. */
struct BurstWs {
	uint64_t *sub_off;
	uint32_t *sub_len;
	uint8_t *status, *verdict;
	uint32_t *seq, *flags;
	uint32_t *bin;
};

size_t a16(size_t x)
{
	return (x + 15) & ~(size_t)15;
}

size_t burst_layout(uint64_t n, uint8_t *base, BurstWs *w)
{
	size_t at = 0;
	auto take = [&](size_t bytes) {
		uint8_t *p = base ? base + at : nullptr;
		at += a16(bytes);
		return p;
	};
	uint32_t *bn = (uint32_t *)take(((size_t)NET2_BIN_WS_WORDS + n) * 4);
	uint64_t *so = (uint64_t *)take(8 * n);
	uint32_t *sl = (uint32_t *)take(4 * n);
	uint8_t *st = take(n);
	uint8_t *vd = take(n);
	uint32_t *sq = (uint32_t *)take(4 * n);
	uint32_t *fl = (uint32_t *)take(4 * n);
	if (w != nullptr)
		*w = { so, sl, st, vd, sq, fl, bn };
	return at;
}

/* hash_alg 0 (none) or an HMAC row with its key; ivlen <= 64 */
int check_burst_args(int hash_alg, const void *key, size_t keylen,
    uint32_t ivlen, const void *d_base, const uint64_t *d_offsets,
    const uint32_t *d_lens, uint64_t n, const uint8_t *d_result,
    const void *d_ws, size_t ws_bytes)
{
	if (hash_alg != NET2_HASH_NIL && (hash_alg < NET2_HASH_HMAC_SHA256 ||
	    hash_alg > NET2_HASH_HMAC_SHA512))
		return EINVAL;
	if (hash_alg != NET2_HASH_NIL && ((size_t)kRows[hash_alg].keylen !=
	    keylen || key == nullptr))
		return EINVAL;
	if (ivlen > 64)
		return EINVAL;
	if (n == 0)
		return 0;
	if (d_base == nullptr || d_offsets == nullptr || d_lens == nullptr ||
	    d_result == nullptr || d_ws == nullptr || n > UINT32_MAX)
		return EINVAL;
	if (ws_bytes < burst_layout(n, nullptr, nullptr) ||
	    ((uintptr_t)d_ws & 15) != 0)
		return EINVAL;
	return check_current_device();
}

/* net2_sha2_burst_limits' binning threshold (-1: none) */
std::atomic<int64_t> g_burst_bin_min{-1};

/*
 * The binning workspace a burst's HMAC kernel is given: below the binning
 * threshold (default 65,536 datagrams: one lane per datagram, one wave per
 * SIMD) none -- every wave then has a SIMD of its own, the burst takes its
 * longest wave's time whatever the order, and the binning launch is pure
 * fixed cost (tools/burst_sizes.py).  The threshold is
 * net2_sha2_burst_limits' setting, else NET2_BURST_BIN_MIN from the
 * environment at first use (A/B runs), else the default.
 */
uint32_t *burst_bins(uint64_t n, uint32_t *bin)
{
	int64_t min_n = g_burst_bin_min.load(std::memory_order_relaxed);
	if (min_n < 0) {
		static const int64_t env = [] {
			const char *e = getenv("NET2_BURST_BIN_MIN");
			return e != nullptr && *e != '\0' ?
			    (int64_t)(strtoull(e, nullptr, 10) & INT64_MAX) :
			    (int64_t)65536;
		}();
		min_n = env;
	}
	return n >= (uint64_t)min_n ? bin : nullptr;
}

/*
 * The hash steps of net2_packet_decode for a device-resident burst.
 * hdr_out: d_seq / d_flags are copies the final kernel makes (the host
 * path: mapped host memory) -- the HMAC kernel keeps the decoded headers in
 * the workspace; otherwise they are where the HMAC kernel decodes to.
 */
int decode_burst(const struct net2_burst_rx_keys *k, uint32_t ivlen,
    const void *d_base, const uint64_t *d_offsets, const uint32_t *d_lens,
    uint64_t n, uint8_t *d_result, void *d_iv, uint32_t *d_seq,
    uint32_t *d_flags, void *d_ws, hipStream_t s, bool hdr_out)
{
	const int hash_alg = k->hash_alg;
	const int hash_set = hash_alg != NET2_HASH_NIL;
	const bool alt = hash_set && k->alt_hash_key != nullptr;
	BurstWs w;
	burst_layout(n, (uint8_t *)d_ws, &w);
	uint32_t *seq = d_seq && !hdr_out ? d_seq : w.seq;
	uint32_t *flags = d_flags && !hdr_out ? d_flags : w.flags;
	const int enc_set = k->enc_alg != 0;
	if (hash_set) {
		/* header decode, key choice, flag checks and HMAC verify in one
		 * kernel over the wire datagrams (binned by datagram length) */
		BurstArgs rx = {};
		rx.seq = seq;
		rx.flags = flags;
		rx.status = w.status;
		rx.enc_set = enc_set;
		if (alt) {
			const uint8_t *ak = (const uint8_t *)k->alt_hash_key;
			rx.alt = 1;
			rx.alt_enc_set = enc_set;
			rx.no_cutoff = k->alt_no_cutoff != 0;
			rx.cutoff = k->alt_cutoff;
			rx.rx_start = k->rx_start;
			for (size_t i = 0; i < k->alt_hash_keylen; i++)
				rx.altkey[i / 4] |= (uint32_t)ak[i] << (24 - 8 * (i % 4));
		}
		if (n <= net2_burst_wave_max()) {
			/* a small burst: 1 to 16 datagrams per workgroup,
			 * codes, headers and IVs stored by that one launch */
			rx.seq = d_seq;
			rx.flags = d_flags;
			rx.status = nullptr;
			HIP_TRY(net2_launch_burst_wave(hash_alg,
			    (const uint8_t *)k->hash_key, k->hash_keylen,
			    (const uint8_t *)d_base, d_offsets, d_lens, n, &rx,
			    d_result, enc_set ? (uint8_t *)d_iv : nullptr,
			    enc_set ? ivlen : 0, nullptr, NET2_HMAC_MODE_BURST_RX,
			    s));
			FI_POINT(FI_KERNEL);
			return 0;
		}
		HIP_TRY(net2_launch_hmac(hash_alg, (const uint8_t *)k->hash_key,
		    k->hash_keylen, (const uint8_t *)d_base, d_offsets, d_lens, 0,
		    0, n, w.verdict, burst_bins(n, w.bin), s,
		    NET2_HMAC_MODE_BURST_RX, &rx));
	} else {
		HIP_TRY(net2_launch_burst_prep((uint8_t *)d_base, d_offsets,
		    d_lens, n, 0, 0, enc_set, 0, nullptr, nullptr, seq,
		    flags, w.sub_off, w.sub_len, w.status, s));
	}
	FI_POINT(FI_KERNEL);
	HIP_TRY(net2_launch_burst_final(n, w.status, w.verdict, seq, flags,
	    enc_set ? ivlen : 0, (uint8_t *)d_iv, d_result, s,
	    hdr_out ? d_seq : nullptr, hdr_out ? d_flags : nullptr));
	return 0;
}

/*
 * The hash steps of net2_packet_encode for a device-resident burst.  rec
 * (keyed hash only): header and hash field of every datagram to a record of
 * their own (BurstArgs::rec) instead of into d_base.  bin: length-bin the
 * burst at or above the threshold (burst_bins); the host path passes false
 * where the order of the records matters more than the kernel's time.
 */
int encode_burst(int hash_alg, const void *hash_key, size_t hash_keylen,
    int enc_alg, const uint32_t *d_seq, const uint32_t *d_flags,
    void *d_base, const uint64_t *d_offsets, const uint32_t *d_lens,
    uint64_t n, uint8_t *d_result, void *d_ws, hipStream_t s, uint8_t *rec,
    bool bin = true, uint8_t *seal_to = nullptr)
{
	/* seal_to (keyed, no rec): headers and hash fields go there, at the
	 * datagrams' offsets, instead of into d_base (the host path: the
	 * caller's page-locked buffer through its device mapping) */
	uint8_t *const out = seal_to != nullptr ? seal_to : (uint8_t *)d_base;
	BurstWs w;
	burst_layout(n, (uint8_t *)d_ws, &w);
	if (hash_alg != NET2_HASH_NIL) {
		/* flag and room checks, header write and HMAC sign in one
		 * kernel over the wire datagrams; the TX code is final (no
		 * verdict to fold in), so the kernel writes it to d_result */
		BurstArgs tx = {};
		tx.seq = const_cast<uint32_t *>(d_seq);
		tx.flags = const_cast<uint32_t *>(d_flags);
		tx.status = d_result;
		tx.enc_set = enc_alg != 0;
		tx.rec = rec;
		if (n <= net2_burst_wave_max()) {
			/* a small burst: 1 to 16 datagrams per workgroup */
			HIP_TRY(net2_launch_burst_wave(hash_alg,
			    (const uint8_t *)hash_key, hash_keylen,
			    (const uint8_t *)d_base, d_offsets, d_lens, n, &tx,
			    d_result, nullptr, 0, out, NET2_HMAC_MODE_BURST_TX, s));
			FI_POINT(FI_KERNEL);
			return 0;
		}
		HIP_TRY(net2_launch_hmac(hash_alg, (const uint8_t *)hash_key,
		    hash_keylen, (const uint8_t *)d_base, d_offsets, d_lens, 0,
		    0, n, out, bin ? burst_bins(n, w.bin) : nullptr, s,
		    NET2_HMAC_MODE_BURST_TX, &tx));
		FI_POINT(FI_KERNEL);
		return 0;
	}
	HIP_TRY(net2_launch_burst_prep((uint8_t *)d_base, d_offsets,
	    d_lens, n, 1, 0, enc_alg != 0, 0, d_seq, d_flags, nullptr,
	    nullptr, w.sub_off, w.sub_len, w.status, s));
	FI_POINT(FI_KERNEL);
	HIP_TRY(net2_launch_burst_final(n, w.status, nullptr, d_seq, d_flags, 0,
	    nullptr, d_result, s));
	return 0;
}

}	/* namespace */

NET2_EXPORT size_t net2_packet_burst_workspace(uint64_t n)
{
	return burst_layout(n, nullptr, nullptr);
}

NET2_EXPORT int net2_sha2_burst_limits(int64_t wave_max, int64_t bin_min)
{
	net2_set_burst_wave_max(wave_max);
	g_burst_bin_min.store(bin_min < 0 ? -1 : bin_min, std::memory_order_relaxed);
	return 0;
}

NET2_EXPORT int net2_packet_decode_burst_ck(const struct net2_burst_rx_keys *k,
    uint32_t ivlen, const void *d_base, const uint64_t *d_offsets,
    const uint32_t *d_lens, uint64_t n, uint8_t *d_result, void *d_iv,
    uint32_t *d_seq, uint32_t *d_flags, void *d_ws, size_t ws_bytes,
    void *stream)
{
	if (k == nullptr)
		return EINVAL;
	int rc = check_burst_args(k->hash_alg, k->hash_key, k->hash_keylen,
	    ivlen, d_base, d_offsets, d_lens, n, d_result, d_ws, ws_bytes);
	if (rc != 0)
		return rc;
	/* an alternate key is new key material under the same algorithms */
	const bool alt = k->hash_alg != NET2_HASH_NIL &&
	    k->alt_hash_key != nullptr;
	if (alt && k->alt_hash_keylen != k->hash_keylen)
		return EINVAL;
	if (n == 0)
		return 0;
	if ((d_seq == nullptr) != (d_flags == nullptr))
		return EINVAL;
	return decode_burst(k, ivlen, d_base, d_offsets, d_lens, n, d_result,
	    d_iv, d_seq, d_flags, d_ws, (hipStream_t)stream, false);
}

NET2_EXPORT int net2_packet_decode_burst(int hash_alg, const void *hash_key,
    size_t hash_keylen, int enc_alg, uint32_t ivlen, const void *d_base,
    const uint64_t *d_offsets, const uint32_t *d_lens, uint64_t n,
    uint8_t *d_result, void *d_iv, uint32_t *d_seq, uint32_t *d_flags,
    void *d_ws, size_t ws_bytes, void *stream)
{
	struct net2_burst_rx_keys k = {};
	k.hash_alg = hash_alg;
	k.hash_key = hash_key;
	k.hash_keylen = hash_keylen;
	k.enc_alg = enc_alg;
	return net2_packet_decode_burst_ck(&k, ivlen, d_base, d_offsets, d_lens,
	    n, d_result, d_iv, d_seq, d_flags, d_ws, ws_bytes, stream);
}

NET2_EXPORT int net2_packet_encode_burst(int hash_alg, const void *hash_key,
    size_t hash_keylen, int enc_alg, const uint32_t *d_seq,
    const uint32_t *d_flags, void *d_base, const uint64_t *d_offsets,
    const uint32_t *d_lens, uint64_t n, uint8_t *d_result, void *d_ws,
    size_t ws_bytes, void *stream)
{
	int rc = check_burst_args(hash_alg, hash_key, hash_keylen, 0, d_base,
	    d_offsets, d_lens, n, d_result, d_ws, ws_bytes);
	if (rc != 0 || n == 0)
		return rc;
	if (d_seq == nullptr || d_flags == nullptr)
		return EINVAL;
	return encode_burst(hash_alg, hash_key, hash_keylen, enc_alg, d_seq,
	    d_flags, d_base, d_offsets, d_lens, n, d_result, d_ws,
	    (hipStream_t)stream, nullptr);
}

/* ---- packet bursts from host memory ----------------------------------------- */

namespace {

/*
 * One pipeline slot of the host burst path: pinned staging for the packed
 * datagrams, their offsets / lengths and (TX) headers, pinned staging for
 * results bound for pageable memory, the device copies and the burst
 * workspace, a stream.  Two slots per device double-buffer pack / H2D /
 * kernels / copy-back, as Slot does for digests.
 */
struct BurstSlot {
	hipStream_t stream = nullptr;
	hipEvent_t done = nullptr;
	bool busy = false;
	uint8_t *h_in = nullptr, *h_out = nullptr;
	/* a chunk's per-datagram metadata, one block so it is one copy:
	 * offsets (8 n), lengths (4 n), TX headers (8 n) -- see Meta */
	uint8_t *h_meta = nullptr;
	uint8_t *d_in = nullptr, *d_ws = nullptr, *d_meta = nullptr;
	size_t cap_in = 0, cap_n = 0;

	/* The metadata arrays of an n-datagram chunk inside a meta block. */
	struct Meta {
		uint64_t *off;
		uint32_t *len, *hdr;
		Meta(uint8_t *m, size_t n) : off((uint64_t *)m),
		    len((uint32_t *)(m + 8 * n)), hdr((uint32_t *)(m + 12 * n)) {}
	};
	static size_t meta_bytes(size_t n, bool tx)
	{
		return n * (tx ? 20 : 12);
	}
	/* run once the chunk's kernels are done: results to the caller */
	std::function<int()> finish;

	/* results staged per datagram: RX code + IV (<= 64) + header; TX code
	 * + record (hash field + header, <= 80) */
	static size_t out_bytes(size_t n)
	{
		return n * 81 + 256;
	}

	void release()
	{
		if (h_in) (void)hipHostFree(h_in);
		if (h_out) (void)hipHostFree(h_out);
		if (h_meta) (void)hipHostFree(h_meta);
		if (d_in) (void)hipFree(d_in);
		if (d_ws) (void)hipFree(d_ws);
		if (d_meta) (void)hipFree(d_meta);
		h_in = h_out = h_meta = nullptr;
		d_in = d_ws = d_meta = nullptr;
		cap_in = cap_n = 0;
	}

	int reserve(size_t in, size_t n)
	{
		if (stream == nullptr) {
			HIP_TRY(hipStreamCreateWithFlags(&stream,
			    hipStreamNonBlocking));
			HIP_TRY(hipEventCreateWithFlags(&done,
			    hipEventDisableTiming));
		}
		if (in <= cap_in && n <= cap_n)
			return 0;
		in = std::max<size_t>({in + in / 8, cap_in, 4096});
		n = std::max<size_t>({n + n / 4, cap_n, 64});
		release();
		HIP_TRY(hipHostMalloc((void **)&h_in, in, hipHostMallocDefault));
		HIP_TRY(hipHostMalloc((void **)&h_out, out_bytes(n),
		    hipHostMallocDefault));
		HIP_TRY(hipHostMalloc((void **)&h_meta, meta_bytes(n, true),
		    hipHostMallocDefault));
		HIP_TRY(hipMalloc((void **)&d_in, in));
		HIP_TRY(hipMalloc((void **)&d_meta, meta_bytes(n, true)));
		HIP_TRY(hipMalloc((void **)&d_ws, burst_layout(n, nullptr,
		    nullptr)));
		/* its binning area prepared once, so the first chunk bins */
		HIP_TRY(net2_bin_ws_init((uint32_t *)d_ws, nullptr));
		HIP_TRY(hipStreamSynchronize(nullptr));
		cap_in = in;
		cap_n = n;
		return 0;
	}

	int drain()
	{
		if (!busy)
			return 0;
		busy = false;
		const double t0 = dbg_now();
		HIP_TRY(hipEventSynchronize(done));
		const double t1 = dbg_now();
		std::function<int()> f;
		f.swap(finish);
		const int rc = f ? f() : 0;
		if (dbg_timing())
			fprintf(stderr, "net2 burst: wait %.3f ms, finish %.3f ms\n",
			    t1 - t0, dbg_now() - t1);
		return rc;
	}
};

struct BurstCtx {
	std::mutex mu;		/* one host burst per device at a time */
	BurstSlot slot[2];
};

std::mutex g_bctx_mu;
std::vector<std::unique_ptr<BurstCtx>> g_bctx;

BurstCtx *bctx_for(size_t idx)
{
	std::lock_guard<std::mutex> g(g_bctx_mu);
	if (g_bctx.size() <= idx)
		g_bctx.resize(idx + 1);
	if (!g_bctx[idx])
		g_bctx[idx].reset(new BurstCtx());
	return g_bctx[idx].get();
}

/*
 * Where the kernels store a chunk's output of `bytes` bytes bound for the
 * caller's `user` (its chunk slice): straight into it through its device
 * mapping when it is page-locked, else into `stage` (the slot's pinned
 * results, mapped) -- then *copy is set and the caller copies it over once
 * the chunk is done.
 */
uint8_t *out_ptr(void *user, bool user_pinned, uint8_t *stage, bool *copy)
{
	void *dp = nullptr;
	*copy = false;
	if (user_pinned && hipHostGetDevicePointer(&dp, user, 0) == hipSuccess &&
	    dp != nullptr)
		return (uint8_t *)dp;
	(void)hipGetLastError();
	if (hipHostGetDevicePointer(&dp, stage, 0) == hipSuccess && dp != nullptr) {
		*copy = true;
		return (uint8_t *)dp;
	}
	(void)hipGetLastError();
	return nullptr;
}

/* The pinned state of each caller buffer of a host burst (looked up once). */
struct BurstPins {
	bool result = false, iv = false, seq = false, flags = false;
	bool base = false;	/* the datagram buffer's start is page-locked */
};

/* What a host burst is asked to do; pointers are the caller's. */
struct HostBurst {
	bool tx;
	/* RX */
	const struct net2_burst_rx_keys *keys;
	uint32_t ivlen;
	void *iv;
	uint32_t *seq_out, *flags_out;
	/* TX */
	int hash_alg;
	const void *hash_key;
	size_t hash_keylen;
	int enc_alg;
	const uint32_t *seq_in, *flags_in;
	/* both */
	uint8_t *base;
	const uint64_t *offsets;
	const uint32_t *lens;
	uint8_t *result;
};

/* dense_pinned (above) for datagrams [lo, lo + n) of a host burst */
bool dense_pinned_range(WorkPool &pool, const HostBurst &hb, uint64_t lo,
    uint64_t n, uint64_t *rs, uint64_t *re)
{
	return dense_pinned(pool, hb.base, hb.offsets + lo, hb.lens + lo, n, rs,
	    re);
}

/* Chunk [lo, hi) of a host burst into slot s. */
int enqueue_burst_steps(WorkPool &pool, BurstSlot &s, const HostBurst &hb,
    const BurstPins &pins, uint64_t lo, uint64_t hi)
{
	const uint64_t n = hi - lo;
	int rc;
	const double tp0 = dbg_now();
	uint64_t rs = 0, re = 0;
	const bool direct = pins.base && dense_pinned_range(pool, hb, lo, n, &rs,
	    &re);
	PackPlan plan;
	if (!direct)
		/* RX packs with a thread per ~512 datagrams: 10-12 % faster
		 * decode calls from 4,096 datagrams up than per ~4 K, 1-4 %
		 * faster again than per ~1 K from 1,024 to 4,096; TX measured
		 * 15-18 % slower per ~1 K and keeps ~4 K
		 * (profiles/round6/pack_ab/) */
		plan = pack_sizes(pool, hb.lens + lo, n, hb.tx ? 12 : 9);
	const size_t bytes = direct ? re - rs : plan.start[plan.nt];
	if ((rc = s.reserve(bytes, n)) != 0)
		return rc;
	/*
	 * A small keyed burst (the one-launch form): its kernel reads the
	 * datagrams and their metadata through their host mapping -- the
	 * caller's page-locked buffer or the slot's staging -- instead of
	 * waiting for two copies: 5-13 % faster from 64 to 16,384 datagrams,
	 * RX and TX, pinned and pageable (profiles/round6/zc_ab/, three
	 * alternations in flipped order).
	 */
	const bool keyed = hb.tx ? hb.hash_alg != NET2_HASH_NIL :
	    hb.keys->hash_alg != NET2_HASH_NIL;
	uint8_t *z_in = nullptr, *z_meta = nullptr;
	if (keyed && n <= NET2_BURST_ZC_MAX && n <= net2_burst_wave_max()) {
		void *a = nullptr, *m = nullptr;
		if (hipHostGetDevicePointer(&a, direct ? (void *)(hb.base + rs) :
		    (void *)s.h_in, 0) == hipSuccess && a != nullptr &&
		    hipHostGetDevicePointer(&m, s.h_meta, 0) == hipSuccess &&
		    m != nullptr) {
			z_in = (uint8_t *)a;
			z_meta = (uint8_t *)m;
		} else {
			(void)hipGetLastError();
		}
	}
	uint8_t *const d_in = z_in != nullptr ? z_in : s.d_in;
	const BurstSlot::Meta hm(s.h_meta, n),
	    dm(z_meta != nullptr ? z_meta : s.d_meta, n);
	if (direct) {
		/* the chunk's datagrams lie densely in one page-locked
		 * allocation: copied as they lie, no host pack */
		const uint64_t *off = hb.offsets + lo;
		const uint32_t *ln = hb.lens + lo;
		uint64_t *ho = hm.off;
		uint32_t *hl = hm.len;
		const size_t nt = std::min<size_t>(kPackThreads,
		    std::max<size_t>(1, n >> 14));
		pool.run(nt, [=](size_t t) {
			for (uint64_t j = n * t / nt; j < n * (t + 1) / nt; j++) {
				ho[j] = off[j] - rs;
				hl[j] = ln[j];
			}
		});
		if (bytes != 0 && z_in == nullptr)
			HIP_TRY(hipMemcpyAsync(s.d_in, hb.base + rs, bytes,
			    hipMemcpyHostToDevice, s.stream));
		if (dbg_timing())
			fprintf(stderr, "net2 burst: direct %zu B: %.3f ms\n", bytes,
			    dbg_now() - tp0);
	} else {
		pack_fill(pool, plan, s.h_in, hm.off, hm.len, hb.base,
		    hb.offsets + lo, hb.lens + lo, n);
		if (dbg_timing())
			fprintf(stderr, "net2 burst: pack %zu B: %.3f ms (%zu "
			    "threads)\n", bytes, dbg_now() - tp0, plan.nt);
		if (bytes != 0 && z_in == nullptr)
			HIP_TRY(hipMemcpyAsync(s.d_in, s.h_in, bytes,
			    hipMemcpyHostToDevice, s.stream));
	}
	if (hb.tx) {
		memcpy(hm.hdr, hb.seq_in + lo, (size_t)n * 4);
		memcpy(hm.hdr + n, hb.flags_in + lo, (size_t)n * 4);
	}
	/* offsets, lengths (and TX headers): one copy */
	if (z_meta == nullptr)
		HIP_TRY(hipMemcpyAsync(s.d_meta, s.h_meta,
		    BurstSlot::meta_bytes(n, hb.tx), hipMemcpyHostToDevice,
		    s.stream));
	FI_POINT(FI_H2D);

	/* staged results: [code n][IV n x ivlen | records][seq n][flags n] */
	uint8_t *st_res = s.h_out;
	uint8_t *st_b = st_res + a16(n);
	bool c_res, c_iv = false, c_seq = false, c_fl = false;
	uint8_t *k_res = out_ptr(hb.result + lo, pins.result, st_res, &c_res);
	if (k_res == nullptr)
		return EIO;
	std::vector<std::function<void()>> copies;
	bool sealed = false;	/* TX sealed in place by the kernel */
	if (!hb.tx) {
		const uint32_t ivlen = hb.keys->enc_alg != 0 ? hb.ivlen : 0;
		uint8_t *st_iv = st_b;
		uint8_t *st_sq = st_iv + a16((size_t)n * ivlen);
		uint8_t *st_fl = st_sq + a16((size_t)n * 4);
		uint8_t *k_iv = nullptr, *k_sq = nullptr, *k_fl = nullptr;
		if (hb.iv != nullptr && ivlen > 0 &&
		    (k_iv = out_ptr((uint8_t *)hb.iv + lo * ivlen, pins.iv, st_iv,
		    &c_iv)) == nullptr)
			return EIO;
		if (hb.seq_out != nullptr &&
		    ((k_sq = out_ptr(hb.seq_out + lo, pins.seq, st_sq, &c_seq)) ==
		    nullptr || (k_fl = out_ptr(hb.flags_out + lo, pins.flags,
		    st_fl, &c_fl)) == nullptr))
			return EIO;
		if ((rc = decode_burst(hb.keys, hb.ivlen, d_in, dm.off, dm.len,
		    n, k_res, k_iv, (uint32_t *)k_sq, (uint32_t *)k_fl, s.d_ws,
		    s.stream, true)) != 0)
			return rc;
		if (c_iv)
			copies.push_back([=]() { memcpy((uint8_t *)hb.iv +
			    lo * ivlen, st_iv, (size_t)n * ivlen); });
		if (c_seq)
			copies.push_back([=]() { memcpy(hb.seq_out + lo, st_sq,
			    (size_t)n * 4); });
		if (c_fl)
			copies.push_back([=]() { memcpy(hb.flags_out + lo, st_fl,
			    (size_t)n * 4); });
	} else {
		/*
		 * Datagrams copied as they lie from one page-locked allocation:
		 * the kernel seals headers and hash fields straight into the
		 * caller's buffer through its mapping (no records, no host
		 * scatter).  Otherwise it fills one record per datagram in the
		 * slot's mapped staging, scattered by the host when the chunk is
		 * done.
		 */
		void *recd = nullptr, *seal = nullptr;
		if (keyed && direct && (hipHostGetDevicePointer(&seal, hb.base + rs,
		    0) != hipSuccess || seal == nullptr)) {
			(void)hipGetLastError();
			seal = nullptr;
		}
		if (keyed && seal == nullptr &&
		    (hipHostGetDevicePointer(&recd, st_b, 0) != hipSuccess ||
		    recd == nullptr)) {
			(void)hipGetLastError();
			return EIO;
		}
		/*
		 * Datagrams copied as they lie (page-locked input) are hashed in
		 * arrival order and sealed in place by the kernel: TX from
		 * pinned memory 2-7 % faster from 1,024 to 16,384 datagrams
		 * than records scattered by the host, the same at 1 M
		 * (profiles/round6/seal_*.jsonl).  Before the kernel sealed
		 * them, arrival order already won over the binned order by
		 * letting the host scatter walk the buffer front to back
		 * (txbin*_*.jsonl); the unbinned kernel stays hidden under the
		 * next chunk's copy.  Packed (pageable) input keeps the binning
		 * and the records: there the pack of the next chunk shares the
		 * host threads with the scatter, and with no binning at all it
		 * measured 1.5 % slower (binoff_*.jsonl).
		 */
		if ((rc = encode_burst(hb.hash_alg, hb.hash_key, hb.hash_keylen,
		    hb.enc_alg, dm.hdr, dm.hdr + n, d_in, dm.off, dm.len, n,
		    k_res, s.d_ws, s.stream, (uint8_t *)recd, !direct,
		    (uint8_t *)seal)) != 0)
			return rc;
		sealed = seal != nullptr;
	}
	FI_POINT(FI_RECORD);
	HIP_TRY(hipEventRecord(s.done, s.stream));
	s.busy = true;
	const bool tx = hb.tx;
	/* dl != 0: records to scatter (keyed TX, not sealed by the kernel) */
	const int dl = tx && hb.hash_alg != NET2_HASH_NIL && !sealed ?
	    digest_len(hb.hash_alg) : 0;
	WorkPool *pp = &pool;
	s.finish = [=]() {
		if (c_res && !(tx && dl != 0))
			memcpy(hb.result + lo, st_res, (size_t)n);
		for (const std::function<void()> &c : copies)
			c();
		if (!tx || sealed)
			return 0;
		/* TX: the code of every datagram, and the sealed header (and
		 * hash field) of every OK one into the caller's slot
		 * (packet.n2t:384-392, :417-427) */
		const size_t nt = std::min<size_t>(kPackThreads,
		    std::max<size_t>(1, n >> 12));
		pp->run(nt, [=](size_t t) {
			for (uint64_t j = n * t / nt; j < n * (t + 1) / nt; j++) {
				if (dl != 0) {
					/* record of binned position j */
					const uint8_t *r = st_b + j * (dl + 16);
					uint32_t w[4];
					memcpy(w, r + dl, 16);
					const uint64_t i = lo + w[2];
					hb.result[i] = (uint8_t)w[3];
					if (w[3] != NET2_PENCODE_OK)
						continue;
					uint8_t *dg = hb.base + hb.offsets[i];
					memcpy(dg, w, 8);
					memcpy(dg + 8, r, dl);
					continue;
				}
				if (hb.result[lo + j] != NET2_PENCODE_OK)
					continue;
				uint8_t *dg = hb.base + hb.offsets[lo + j];
				const uint32_t sq = hb.seq_in[lo + j];
				const uint32_t fl = hb.flags_in[lo + j];
				for (int b = 0; b < 4; b++) {
					dg[b] = (uint8_t)(sq >> (24 - 8 * b));
					dg[4 + b] = (uint8_t)(fl >> (24 - 8 * b));
				}
			}
		});
		return 0;
	};
	return 0;
}

/* enqueue_burst_steps; a chunk that fails part-way is waited for (quiesce)
 * before the error goes back, and its slot stays free. */
int enqueue_burst_chunk(WorkPool &pool, BurstSlot &s, const HostBurst &hb,
    const BurstPins &pins, uint64_t lo, uint64_t hi)
{
	const int rc = enqueue_burst_steps(pool, s, hb, pins, lo, hi);
	if (rc != 0)
		quiesce(s.stream);
	return rc;
}

/* One device's share [lo, hi) of a host burst, chunked and double-buffered. */
int run_burst_slice(size_t didx, int ordinal, const HostBurst &hb,
    uint64_t lo, uint64_t hi)
{
	const NumaPlace &np = numa_place(ordinal);
	NumaBind bind(np);
	DeviceCtx *c = ctx_for(didx);
	BurstCtx *b = bctx_for(didx);
	std::lock_guard<std::mutex> g(b->mu);
	HIP_TRY(hipSetDevice(ordinal));
	/* outputs are stored through their mapping only when the slice's
	 * whole range of each is in one page-locked allocation */
	const uint64_t m = hi - lo;
	const double tq0 = dbg_now();
	BurstPins pins;
	pins.base = is_pinned(hb.base);
	pins.result = pinned_span(hb.result + lo, m);
	if (!hb.tx) {
		const uint32_t ivl = hb.keys->enc_alg != 0 ? hb.ivlen : 0;
		pins.iv = hb.iv != nullptr && ivl > 0 && pinned_span((uint8_t *)hb.iv +
		    lo * ivl, m * ivl);
		pins.seq = hb.seq_out != nullptr && pinned_span(hb.seq_out + lo,
		    m * 4);
		pins.flags = hb.flags_out != nullptr && pinned_span(hb.flags_out +
		    lo, m * 4);
	}
	if (dbg_timing())
		fprintf(stderr, "net2 burst: page-lock lookups %.3f ms\n",
		    dbg_now() - tq0);
	const PackPlan all = pack_sizes(*c->pool, hb.lens + lo, hi - lo);
	const size_t mean = std::max<size_t>(all.start[all.nt] /
	    std::max<uint64_t>(hi - lo, 1), 16);
	const uint64_t per_chunk = std::max<size_t>(kChunkBytes / mean, 1);
	/*
	 * Chunk k is enqueued into its slot first, then chunk k - 1 (the other
	 * slot) is waited for and its results handed over -- the TX scatter
	 * of sealed headers runs while chunk k copies and hashes, and by the
	 * next iteration that slot is free again.  (Draining a slot right
	 * before reusing it put the scatter between two copies: TX 17.6 ms per
	 * 1 M datagrams against RX's 15.2 ms.)
	 */
	int rc = 0, cur = 0;
	for (uint64_t at = lo; at < hi && rc == 0;) {
		const uint64_t end = std::min<uint64_t>(hi, at + per_chunk);
		const double t0 = dbg_now();
		rc = enqueue_burst_chunk(*c->pool, b->slot[cur], hb, pins, at, end);
		const double t1 = dbg_now();
		if (rc == 0)
			rc = b->slot[cur ^ 1].drain();
		if (dbg_timing())
			fprintf(stderr, "net2 burst: enqueue %.3f ms, drain+finish "
			    "%.3f ms (%llu datagrams)\n", t1 - t0, dbg_now() - t1,
			    (unsigned long long)(end - at));
		at = end;
		cur ^= 1;
	}
	/* both slots drained whatever happened: no kernel may still write
	 * into the caller's memory when the call returns */
	const int rc2 = b->slot[0].drain();
	const int rc3 = b->slot[1].drain();
	return rc ? rc : rc2 ? rc2 : rc3;
}

/* Host-memory arguments: no device, workspace or size requirement. */
int check_host_burst(int hash_alg, const void *key, size_t keylen,
    uint32_t ivlen, const void *base, const uint64_t *offsets,
    const uint32_t *lens, uint64_t n, const uint8_t *result)
{
	if (hash_alg != NET2_HASH_NIL && (hash_alg < NET2_HASH_HMAC_SHA256 ||
	    hash_alg > NET2_HASH_HMAC_SHA512))
		return EINVAL;
	if (hash_alg != NET2_HASH_NIL && ((size_t)kRows[hash_alg].keylen !=
	    keylen || key == nullptr))
		return EINVAL;
	if (ivlen > 64)
		return EINVAL;
	if (n == 0)
		return 0;
	if (base == nullptr || offsets == nullptr || lens == nullptr ||
	    result == nullptr || n > UINT32_MAX)
		return EINVAL;
	return 0;
}

}	/* namespace */

NET2_EXPORT int net2_packet_decode_burst_host(
    const struct net2_burst_rx_keys *k, uint32_t ivlen, const void *base,
    const uint64_t *offsets, const uint32_t *lens, uint64_t n,
    uint8_t *result, void *iv, uint32_t *seq, uint32_t *flags,
    int max_devices)
{
	if (k == nullptr)
		return EINVAL;
	int rc = check_host_burst(k->hash_alg, k->hash_key, k->hash_keylen,
	    ivlen, base, offsets, lens, n, result);
	if (rc != 0 || n == 0)
		return rc;
	if (k->hash_alg != NET2_HASH_NIL && k->alt_hash_key != nullptr &&
	    k->alt_hash_keylen != k->hash_keylen)
		return EINVAL;
	if ((seq == nullptr) != (flags == nullptr))
		return EINVAL;
	HostBurst hb = {};
	hb.tx = false;
	hb.keys = k;
	hb.ivlen = ivlen;
	hb.iv = iv;
	hb.seq_out = seq;
	hb.flags_out = flags;
	hb.base = (uint8_t *)const_cast<void *>(base);
	hb.offsets = offsets;
	hb.lens = lens;
	hb.result = result;
	return shard_batch(n, lens, 0, max_devices, [&](size_t didx,
	    int ordinal, uint64_t lo, uint64_t hi) {
		return run_burst_slice(didx, ordinal, hb, lo, hi);
	});
}

NET2_EXPORT int net2_packet_encode_burst_host(int hash_alg,
    const void *hash_key, size_t hash_keylen, int enc_alg,
    const uint32_t *seq, const uint32_t *flags, void *base,
    const uint64_t *offsets, const uint32_t *lens, uint64_t n,
    uint8_t *result, int max_devices)
{
	int rc = check_host_burst(hash_alg, hash_key, hash_keylen, 0, base,
	    offsets, lens, n, result);
	if (rc != 0 || n == 0)
		return rc;
	if (seq == nullptr || flags == nullptr)
		return EINVAL;
	HostBurst hb = {};
	hb.tx = true;
	hb.hash_alg = hash_alg;
	hb.hash_key = hash_key;
	hb.hash_keylen = hash_keylen;
	hb.enc_alg = enc_alg;
	hb.seq_in = seq;
	hb.flags_in = flags;
	hb.base = (uint8_t *)base;
	hb.offsets = offsets;
	hb.lens = lens;
	hb.result = result;
	return shard_batch(n, lens, 0, max_devices, [&](size_t didx,
	    int ordinal, uint64_t lo, uint64_t hi) {
		return run_burst_slice(didx, ordinal, hb, lo, hi);
	});
}
